"""McClendon difficulty / complexity restated in plain Python (TEST INFRASTRUCTURE: the oracle for
csrc/mz_difficulty.hip and csrc/mz_mcclendon.hip; only tests/ may import it).

Follows ComplexityEvaluation (reference lib/maze_difficulty_evaluation/maze_complexity_evaluation
.py:38-329) without networkx, keeping every order its float64 result depends on:
  * the graph: nodes in first-insertion order, per-node neighbours in first-insertion order
    (create_graph_branch :115-123 over the solution and then every dead end's path, :62-80);
  * hallway sums (complexity_of_hallway :286-296) iterate the hallway's edges the way networkx
    3.4's subgraph view does (G.subgraph(all_nodes), :217-218): the view's nodes are
    show_nodes(nbunch_iter(all_nodes)).nodes, a set built from all_nodes' iteration order; when
    2 * |that set| < |G| FilterAdjacency iterates that set (CPython set-table order, oracle/
    pyset.py), otherwise G's node order; each node's neighbours in G's adjacency order, an edge
    reported from the end iterated first (EdgeDataView);
  * all_nodes = set(component).union(adjacent_split_points) (:205-217), the component being the
    set _plain_bfs built (nx.connected_components on temp_graph = G.copy() minus the split and
    solution points, :194-201): BFS from the component's first node in node order, neighbours in
    the COPY's adjacency order — G.copy() re-adds edges (u, v) for u in node order, v in adj[u],
    so a node's copied adjacency lists its earlier neighbours (in node order) first, then its
    later ones in its own order; adjacent_split_points is filled in component-set order, each
    node's neighbours in G's order, with the reference's break after a solution junction
    (:208-214);
  * branches (:223-259): components of G minus the non-junction solution points, in first-node
    order; a branch sums its hallways in hallway-id order; the product runs over branches 1..m,
    then branch 0 (:319-329).
Paths: the reference's depth-unlimited heapq A* (lib/a_star_algos/a_star.py:9-80), restated.
"""
import heapq
import math

from pyset import PySet


def cantor(p):
    """cantor_pairing (maze_complexity_evaluation.py:7-20)."""
    x, y = p
    return (x + y) * (x + y + 1) // 2 + y


def astar(maze, start, goal):
    """astar_limited_partial with max_depth 1e6 (a_star.py:9-80): the path as a list of cells."""
    rows, cols = len(maze), len(maze[0])
    h = lambda a: abs(a[0] - goal[0]) + abs(a[1] - goal[1])  # noqa: E731
    heap = [(h(start), start)]
    came, g = {}, {start: 0}
    best, best_g = start, 0
    while heap:
        _, cur = heapq.heappop(heap)
        if g[cur] > best_g:
            best, best_g = cur, g[cur]
        if cur == goal:
            best = cur
            break
        for dr, dc in ((-1, 0), (1, 0), (0, -1), (0, 1)):
            nb = (cur[0] + dr, cur[1] + dc)
            if 0 <= nb[0] < rows and 0 <= nb[1] < cols and maze[nb[0]][nb[1]] != 0:
                t = g[cur] + 1
                if nb not in g or t < g[nb]:
                    came[nb] = cur
                    g[nb] = t
                    heapq.heappush(heap, (t + h(nb), nb))
    path = [best]
    while path[-1] in came:
        path.append(came[path[-1]])
    return path[::-1]


class Graph:
    """Insertion-ordered undirected graph (what networkx.Graph's dicts keep)."""

    def __init__(self):
        self.adj = {}  # node -> {neighbour: None} in insertion order

    def add_node(self, v):
        self.adj.setdefault(v, {})

    def add_edge(self, u, v):
        self.add_node(u)
        self.add_node(v)
        self.adj[u].setdefault(v, None)
        self.adj[v].setdefault(u, None)

    def copy_adjacency(self, removed):
        """The adjacency of G.copy() with `removed` nodes taken out (G.copy() then
        remove_nodes_from): earlier neighbours first (node order), then later ones in own order."""
        pos = {v: i for i, v in enumerate(self.adj)}
        out = {}
        for v in self.adj:
            if v in removed:
                continue
            nb = [u for u in self.adj[v] if u not in removed]
            early = sorted((u for u in nb if pos[u] < pos[v]), key=pos.__getitem__)
            out[v] = early + [u for u in nb if pos[u] > pos[v]]
        return out


def _nbrs(maze, p):
    return sum(1 for dr, dc in ((-1, 0), (1, 0), (0, -1), (0, 1)) if maze[p[0] + dr][p[1] + dc] != 0)


def _decompose(maze, path):
    """decompose_in_turns (:125-136)."""
    out = [path[0]]
    for i in range(1, len(path) - 1):
        a, b = path[i - 1], path[i + 1]
        if (a[0] != b[0] and a[1] != b[1]) or _nbrs(maze, path[i]) > 2:
            out.append(path[i])
    out.append(path[-1])
    return out


def _components(adj):
    """nx.connected_components over an adjacency dict: (first-node order) the list of BFS
    insertion sequences (_plain_bfs: level by level, neighbours in adjacency order)."""
    seen = set()
    comps = []
    for v in adj:
        if v in seen:
            continue
        order, level = [v], [v]
        seen.add(v)
        while level:
            nxt = []
            for x in level:
                for w in adj[x]:
                    if w not in seen:
                        seen.add(w)
                        order.append(w)
                        nxt.append(w)
            level = nxt
        comps.append(order)
    return comps


def _edge_terms(G, dmap, view_order, members):
    """get_edge_attributes(view, "d") in the view's edge order: [(d), ...]."""
    seen = set()
    ds = []
    for n in view_order:
        for u in G.adj[n]:
            if u in members and u not in seen:
                ds.append(dmap[(n, u)] if (n, u) in dmap else dmap[(u, n)])
        seen.add(n)
    return ds


def _hallway_complexity(ds):
    """complexity_of_hallway (:286-296): D_h * sum(1 / (2 d)), sum() from int 0."""
    s = 0
    for d in ds:
        s = s + 1 / (2 * d)
    return sum(ds) * s


def hallway_orders(maze, start, goal):
    """The graph and the per-hallway node iteration orders (for tests); see evaluate()."""
    return _build(maze, start, goal)[1]


def _build(maze, start, goal):
    maze = [list(map(int, r)) for r in maze]
    start, goal = tuple(start), tuple(goal)
    G = Graph()
    dmap = {}

    def branch(ns, path):  # create_graph_branch (:115-123) + calculate_lenght_arcs (:176-184)
        ids = [cantor(p) for p in ns]
        G.add_node(ids[0])
        for i in range(1, len(ids)):
            G.add_node(ids[i])
            G.add_edge(ids[i - 1], ids[i])
        where = {}
        for i, p in enumerate(path):
            where.setdefault(p, i)
        for i in range(len(ns) - 1):
            dmap[(ids[i], ids[i + 1])] = len(path[where[ns[i]]:where[ns[i + 1]] - 1])

    sol = astar(maze, start, goal)
    s_nodes = _decompose(maze, sol)
    branch(s_nodes, sol)
    sol_ids = [cantor(p) for p in s_nodes]
    sol_graph_order = list(dict.fromkeys(sol_ids))
    sol_d = dict(dmap)
    junctions = [p for p in s_nodes if _nbrs(maze, p) == 3]
    sol_cells = set(sol)
    H, W = len(maze), len(maze[0])
    for i in range(1, H - 1):  # get_dead_ends (:152-166)
        for j in range(1, W - 1):
            if maze[i][j] == 1 and _nbrs(maze, (i, j)) == 1 and (i, j) not in sol_cells:
                path = astar(maze, (i, j), start)  # calculate_path (:168-174)
                pn = _decompose(maze, path)
                junctions += [p for p in pn if _nbrs(maze, p) == 3]
                branch(pn, path)
    p_ids = [cantor(x) for x in set(junctions)]
    p_set = set(p_ids)
    s_set = set(sol_ids)
    nG = len(G.adj)
    # extract_hallways (:186-221)
    halls = []
    for comp in _components(G.copy_adjacency(p_set | s_set)):
        cset = PySet.from_iter(comp).copy()  # _plain_bfs's `seen`, then set(component_nodes)
        asp = PySet()
        for node in cset:
            for nb in G.adj[node]:
                if nb in p_set:
                    asp.add(nb)
                    if nb in s_set:
                        break
        all_nodes = cset.union(asp)
        shown = PySet.from_iter(n for n in all_nodes if n in G.adj)  # show_nodes(nbunch_iter(.))
        members = set(shown)
        if 2 * len(shown) < nG:
            order = list(shown)
        else:
            order = [v for v in G.adj if v in members]
        halls.append((order, members))
    return (G, dmap, sol_graph_order, sol_d, halls, p_set, s_nodes, s_set), halls


def evaluate(maze, start, goal):
    """(difficulty_of_maze(), complexity_of_maze()) (:310-329) of a euclidean grid."""
    (G, dmap, sol_order, sol_d, halls, p_set, s_nodes, s_set), _ = _build(maze, start, goal)
    # hallway 0: solution_branch = G.copy() right after the solution (:65-71) — a path graph
    sol_members = set(sol_order)
    sol_adj = Graph()
    for a, b in zip(sol_order, sol_order[1:]):
        sol_adj.add_edge(a, b)
    c0 = _hallway_complexity(_edge_terms(sol_adj, sol_d, sol_order, sol_members))
    ch = [c0] + [_hallway_complexity(_edge_terms(G, dmap, order, members)) for order, members in halls]
    hall_nodes = [sol_members] + [members for _, members in halls]
    # get_branches (:223-259)
    rm = {cantor(x) for x in s_nodes} - p_set
    keep_adj = {v: [u for u in G.adj[v] if u not in rm] for v in G.adj if v not in rm}
    taken = set()
    branch_c = []
    for comp in _components(keep_adj):
        bset = set(comp)
        s = 0
        for i, hn in enumerate(hall_nodes):
            if i not in taken and hn <= bset:
                taken.add(i)
                s = s + ch[i]
        branch_c.append(s)
    branch_c.append(ch[0])  # self.branches[0] = [0], inserted last (:91)
    p, s = 1, 0
    for b, cx in enumerate(branch_c):
        last = b == len(branch_c) - 1
        p = p * cx if last else p * (cx + 1)
        s = s + cx
    return math.log(p), math.log(s)
