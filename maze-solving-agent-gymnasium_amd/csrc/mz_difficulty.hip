// mz_difficulty.hip — McClendon maze difficulty (host C++ in libmazerl.so).
//
// Restates ComplexityEvaluation (lib/maze_difficulty_evaluation/maze_complexity_evaluation.py:38-329)
// without networkx. The value is a float64 built from sums and products whose order the reference
// fixes through networkx's insertion-ordered dicts, so the graph here keeps exactly that order:
//   - node order = first insertion by create_graph_branch (:115-123) / add_edge (u before v);
//   - per-node adjacency order = first insertion of each edge (re-adding keeps the position);
//   - connected components are listed by their first node in node order (nx.connected_components);
//   - a hallway's edges iterate (view node order, adjacency order, each edge once), the view's
//     node order being CPython 3.10 set-table order of show_nodes' set when it holds fewer than
//     half of G's nodes (networkx 3.4 FilterAdjacency), else node order — the sets rebuilt as the
//     reference builds them (PySetEm, extract_hallways :194-218);
//   - branch products run over branch ids 1..m, then branch 0 (:323-329).
// Used by BaseMazeEnv.get_maze_difficulty (base_maze_env.py:99-105) and best-of-6 generation
// (base_maze_env.py:78-97). Paths come from a depth-unlimited A* with Python heapq order
// (a_star.py:9-100), so mazes with cycles get the same (shortest) path choice as the reference.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/mazerl.h"

namespace {

struct HeapNode {
  int f, r, c;
};
inline bool heap_less(const HeapNode& a, const HeapNode& b) {  // Python tuple order (f, (r, c))
  if (a.f != b.f) return a.f < b.f;
  if (a.r != b.r) return a.r < b.r;
  return a.c < b.c;
}
struct HeapGreater {
  bool operator()(const HeapNode& a, const HeapNode& b) const { return heap_less(b, a); }
};

// astar_limited_partial(maze, src, goal) with max_depth 1e6 (euclidean): the path as cell ids.
std::vector<int> astar_path(const uint8_t* g, int H, int W, int sr, int sc, int gr, int gc) {
  const int n = H * W;
  std::vector<int> gs(n, -1), from(n, -1);
  std::vector<HeapNode> heap;
  auto h = [&](int r, int c) { return std::abs(r - gr) + std::abs(c - gc); };
  const int s = sr * W + sc, goal = gr * W + gc;
  gs[s] = 0;
  heap.push_back({h(sr, sc), sr, sc});
  int best = s, best_g = 0, end = -1;
  static const int AR[4] = {-1, 1, 0, 0}, AC[4] = {0, 0, -1, 1};  // a_star.py:60
  while (!heap.empty()) {
    std::pop_heap(heap.begin(), heap.end(), HeapGreater());
    const HeapNode cur = heap.back();
    heap.pop_back();
    const int ci = cur.r * W + cur.c;
    if (gs[ci] > best_g) { best_g = gs[ci]; best = ci; }
    if (ci == goal) { end = ci; break; }
    for (int k = 0; k < 4; ++k) {
      const int nr = cur.r + AR[k], nc = cur.c + AC[k];
      if (nr < 0 || nr >= H || nc < 0 || nc >= W) continue;
      const int ni = nr * W + nc;
      if (g[ni] == 0) continue;
      const int tg = gs[ci] + 1;
      if (gs[ni] < 0 || tg < gs[ni]) {
        from[ni] = ci;
        gs[ni] = tg;
        heap.push_back({tg + h(nr, nc), nr, nc});
        std::push_heap(heap.begin(), heap.end(), HeapGreater());
      }
    }
  }
  if (end < 0) end = best;
  std::vector<int> path;
  for (int v = end; v >= 0; v = from[v]) path.push_back(v);
  std::reverse(path.begin(), path.end());
  return path;
}

struct Graph {  // insertion-ordered undirected graph (what networkx.Graph keeps)
  std::vector<int> order;                   // node ids in insertion order
  std::unordered_map<int, int> idx;         // node id -> position in `order`
  std::vector<std::vector<int>> adj;        // per node (by position): neighbours in insertion order
  std::unordered_map<int64_t, int> d;       // edge (min,max) -> "d"

  int add_node(int v) {
    auto it = idx.find(v);
    if (it != idx.end()) return it->second;
    const int p = (int)order.size();
    idx.emplace(v, p);
    order.push_back(v);
    adj.emplace_back();
    return p;
  }
  static int64_t key(int u, int v) {
    const int a = std::min(u, v), b = std::max(u, v);
    return ((int64_t)a << 32) | (uint32_t)b;
  }
  void add_edge(int u, int v) {
    const int pu = add_node(u), pv = add_node(v);
    auto& au = adj[pu];
    if (std::find(au.begin(), au.end(), v) == au.end()) au.push_back(v);
    auto& av = adj[pv];
    if (std::find(av.begin(), av.end(), u) == av.end()) av.push_back(u);
  }
};

// CPython 3.10 set table for int keys (hash(n) == n), Objects/setobject.c: the order networkx's
// subgraph views iterate their node set in (oracle/pyset.py restates it and checks it against the
// interpreter). No deletions occur, so no dummy entries.
struct PySetEm {
  static constexpr int32_t EMPTY = -1;
  std::vector<int32_t> t = std::vector<int32_t>(8, EMPTY);
  size_t mask = 7, fill = 0, used = 0;
  bool small = true;  // still the 8-slot smalltable

  static void insert_clean(std::vector<int32_t>& tab, size_t m, int32_t key) {
    size_t perturb = (size_t)key, i = (size_t)key & m;
    for (;;) {
      if (tab[i] == EMPTY) { tab[i] = key; return; }
      if (i + 9 <= m)
        for (size_t j = 1; j <= 9; ++j)
          if (tab[i + j] == EMPTY) { tab[i + j] = key; return; }
      perturb >>= 5;
      i = (i * 5 + 1 + perturb) & m;
    }
  }
  void resize(size_t minused) {  // set_table_resize
    size_t ns = 8;
    while (ns <= minused) ns <<= 1;
    if (ns == 8 && small) return;
    std::vector<int32_t> old;
    old.swap(t);
    t.assign(ns, EMPTY);
    mask = ns - 1;
    small = ns == 8;
    for (int32_t k : old)
      if (k != EMPTY) insert_clean(t, mask, k);
    fill = used;
  }
  void add(int32_t key) {  // set_add_entry
    size_t perturb = (size_t)key, i = (size_t)key & mask;
    for (;;) {
      size_t e = i, probes = i + 9 <= mask ? 9 : 0;
      for (;;) {
        if (t[e] == EMPTY) {
          t[e] = key;
          ++fill;
          ++used;
          if (fill * 5 >= mask * 3) resize(used > 50000 ? used * 2 : used * 4);
          return;
        }
        if (t[e] == key) return;
        if (probes-- == 0) break;
        ++e;
      }
      perturb >>= 5;
      i = (i * 5 + 1 + perturb) & mask;
    }
  }
  void merge(const PySetEm& o) {  // set_merge with a set argument
    if (&o == this || o.used == 0) return;
    if ((fill + o.used) * 5 >= mask * 3) resize((used + o.used) * 2);
    if (fill == 0 && mask == o.mask) { t = o.t; fill = o.fill; used = o.used; return; }
    if (fill == 0) {
      for (int32_t k : o.t)
        if (k != EMPTY) insert_clean(t, mask, k);
      fill = used = o.used;
      return;
    }
    for (int32_t k : o.t)
      if (k != EMPTY) add(k);
  }
  PySetEm copy() const { PySetEm s; s.merge(*this); return s; }
  template <class F> void each(F f) const {
    for (int32_t k : t)
      if (k != EMPTY) f(k);
  }
};

// A node-induced view's edges (EdgeDataView): nodes in `order`, each node's neighbours in G's
// adjacency order restricted to the view, every edge reported once from the end met first.
// complexity_of_hallway (:286-296): D_h * sum(1 / (2 d_e)), D_h = sum(d_e)
double hallway_complexity(const Graph& G, const std::unordered_map<int64_t, int>& dmap,
                          const std::unordered_set<int>& nodes, const std::vector<int>& order) {
  long D = 0;
  double s = 0.0;
  bool first = true;
  std::unordered_set<int> seen;
  for (int v : order) {
    const int pv = G.idx.at(v);
    for (int u : G.adj[pv]) {
      if (!nodes.count(u) || seen.count(u)) continue;
      auto it = dmap.find(Graph::key(v, u));
      if (it == dmap.end()) continue;  // get_edge_attributes skips edges without "d"
      D += it->second;
      const double t = 1.0 / (2.0 * (double)it->second);
      s = first ? (0 + t) : s + t;  // sum() starts from int 0
      first = false;
    }
    seen.insert(v);
  }
  return (double)D * s;
}

// nx.connected_components(G.copy() minus `removed`): components by first node in G's node order,
// each as _plain_bfs's insertion sequence (level by level, neighbours in the COPY's adjacency
// order: G.copy() re-adds edges (u, v) for u in node order, v in adj[u], so a node lists its
// earlier neighbours by node position first, then its later ones in its own order)
std::vector<std::vector<int>> components(const Graph& G, const std::unordered_set<int>& removed) {
  std::vector<std::vector<int>> out;
  std::unordered_set<int> seen;
  std::vector<int> nb;
  for (int v : G.order) {
    if (removed.count(v) || seen.count(v)) continue;
    std::vector<int> comp{v};
    seen.insert(v);
    for (size_t h = 0; h < comp.size(); ++h) {
      const int x = comp[h], px = G.idx.at(x);
      nb.clear();
      for (int u : G.adj[px])
        if (G.idx.at(u) < px) nb.push_back(u);
      std::sort(nb.begin(), nb.end(), [&](int a, int b) { return G.idx.at(a) < G.idx.at(b); });
      for (int u : G.adj[px])
        if (G.idx.at(u) > px) nb.push_back(u);
      for (int u : nb) {
        if (removed.count(u) || seen.count(u)) continue;
        seen.insert(u);
        comp.push_back(u);
      }
    }
    out.push_back(std::move(comp));
  }
  return out;
}

// difficulty_of_maze (:319-329) and complexity_of_maze (:311-317) of one euclidean grid
int mcclendon(const uint8_t* g, int32_t H, int32_t W, int32_t sr, int32_t sc, int32_t gr,
              int32_t gc, double* difficulty, double* complexity, double* prod_out = nullptr) {
  if (!g || H < 3 || W < 3) return MZ_EINVAL;
  auto open = [&](int r, int c) { return g[r * W + c] != 0; };
  auto nbrs = [&](int v) {
    const int r = v / W, c = v % W;
    return (int)open(r - 1, c) + (int)open(r + 1, c) + (int)open(r, c - 1) + (int)open(r, c + 1);
  };
  // decompose_in_turns (:125-136)
  auto decompose = [&](const std::vector<int>& path) {
    std::vector<int> ris{path[0]};
    for (size_t i = 1; i + 1 < path.size(); ++i) {
      const int a = path[i - 1], b = path[i + 1];
      const bool turn = (a / W != b / W) && (a % W != b % W);
      if (turn || nbrs(path[i]) > 2) ris.push_back(path[i]);
    }
    ris.push_back(path.back());
    return ris;
  };
  Graph G;
  std::unordered_map<int64_t, int> dmap;
  // create_graph_branch (:115-123)
  auto add_branch = [&](const std::vector<int>& ns) {
    G.add_node(ns[0]);
    for (size_t i = 1; i + 1 < ns.size(); ++i) {
      G.add_node(ns[i]);
      G.add_edge(ns[i - 1], ns[i]);
    }
    G.add_node(ns.back());
    G.add_edge(ns[ns.size() - 2], ns.back());
  };
  // calculate_lenght_arcs (:176-184): d = index(ns[i+1]) - 1 - index(ns[i]) (>= 0)
  auto arcs = [&](const std::vector<int>& ns, const std::vector<int>& path) {
    std::unordered_map<int, int> pos;
    for (size_t i = 0; i < path.size(); ++i) pos.emplace(path[i], (int)i);
    for (size_t i = 0; i + 1 < ns.size(); ++i) {
      const int d = std::max(0, pos.at(ns[i + 1]) - 1 - pos.at(ns[i]));
      dmap[Graph::key(ns[i], ns[i + 1])] = d;
    }
  };
  auto junctions_of = [&](const std::vector<int>& ns, std::vector<int>& js) {
    for (int v : ns)
      if (nbrs(v) == 3) js.push_back(v);  // get_junctions (:138-150): exactly 3
  };

  // Perfect mazes (open squares form a tree, all generators here and in the reference) have one
  // simple path between two cells, which is the path A* returns: take it from BFS parents rooted
  // at the start. Mazes with cycles fall back to the heapq-ordered A* (tie-breaking matters).
  std::vector<int> parent(H * W, -2);
  bool tree = true;
  {
    long n_open = 0, n_edges = 0;
    for (int r = 0; r < H; ++r)
      for (int c = 0; c < W; ++c) {
        if (!open(r, c)) continue;
        ++n_open;
        if (r + 1 < H && open(r + 1, c)) ++n_edges;
        if (c + 1 < W && open(r, c + 1)) ++n_edges;
      }
    tree = n_edges == n_open - 1;
    if (tree) {
      std::vector<int> q{sr * W + sc};
      parent[sr * W + sc] = -1;
      for (size_t h = 0; h < q.size(); ++h) {
        const int v = q[h], r = v / W, c = v % W;
        const int nb[4] = {v - W, v + W, v - 1, v + 1};
        const bool ok[4] = {r > 0, r + 1 < H, c > 0, c + 1 < W};
        for (int k = 0; k < 4; ++k)
          if (ok[k] && g[nb[k]] != 0 && parent[nb[k]] == -2) { parent[nb[k]] = v; q.push_back(nb[k]); }
      }
      tree = parent[gr * W + gc] != -2;
    }
  }
  auto path_to_start = [&](int x) {  // x -> ... -> start
    std::vector<int> p;
    for (int v = x; v >= 0; v = parent[v]) p.push_back(v);
    return p;
  };
  std::vector<int> sol;
  if (tree) {
    sol = path_to_start(gr * W + gc);
    std::reverse(sol.begin(), sol.end());
  } else {
    sol = astar_path(g, H, W, sr, sc, gr, gc);
  }
  if (sol.size() < 2 || sol.back() != gr * W + gc) return MZ_EINVAL;
  const std::vector<int> s_nodes = decompose(sol);
  add_branch(s_nodes);
  Graph H0 = G;  // solution_branch = G.copy() (:66)
  arcs(s_nodes, sol);
  const std::unordered_map<int64_t, int> d_sol = dmap;
  std::vector<int> junc;
  junctions_of(s_nodes, junc);
  // get_dead_ends (:152-166): value 1, one open neighbour, not on the solution, row-major
  std::unordered_set<int> sol_set(sol.begin(), sol.end());
  for (int r = 1; r < H - 1; ++r)
    for (int c = 1; c < W - 1; ++c) {
      const int v = r * W + c;
      if (g[v] != 1 || nbrs(v) != 1 || sol_set.count(v)) continue;
      // calculate_path (:168-174): dead end -> start
      const std::vector<int> path = tree ? path_to_start(v) : astar_path(g, H, W, r, c, sr, sc);
      if (path.size() < 2) continue;
      const std::vector<int> pn = decompose(path);
      junctions_of(pn, junc);
      add_branch(pn);
      arcs(pn, path);
    }
  const std::unordered_set<int> p(junc.begin(), junc.end());        // split points
  const std::unordered_set<int> s_p(s_nodes.begin(), s_nodes.end()); // solution points

  // extract_hallways (:186-221)
  std::unordered_set<int> rm_h(p);
  rm_h.insert(s_p.begin(), s_p.end());
  std::vector<std::unordered_set<int>> hallways;  // index i+1
  std::vector<std::vector<int>> hall_order;        // the view's node iteration order
  const size_t nG = G.order.size();
  for (const auto& comp : components(G, rm_h)) {
    // the sets hold the reference's node ids, cantor_pairing((r, c)) (:7-20), which are also
    // their hashes; cell ids here are r * W + c
    auto cid = [&](int v) { const int r = v / W, c = v % W; return (r + c) * (r + c + 1) / 2 + c; };
    std::unordered_map<int, int> cell_of;
    PySetEm seen;  // _plain_bfs's `seen`, then set(component_nodes) (:205)
    for (int v : comp) { seen.add(cid(v)); cell_of[cid(v)] = v; }
    const PySetEm cset = seen.copy();
    PySetEm asp;   // adjacent_split_points, filled in cset's order (:208-214)
    cset.each([&](int k) {
      for (int u : G.adj[G.idx.at(cell_of.at(k))]) {
        if (!p.count(u)) continue;
        asp.add(cid(u));
        cell_of[cid(u)] = u;
        if (s_p.count(u)) break;  // the reference's break (:213-214)
      }
    });
    PySetEm all = cset.copy();  // component_nodes.union(adjacent_split_points) (:217)
    all.merge(asp);
    PySetEm shown;              // show_nodes(nbunch_iter(all_nodes)).nodes (G.subgraph, :218)
    all.each([&](int k) { shown.add(k); });
    std::unordered_set<int> members;
    std::vector<int> order;
    shown.each([&](int k) { members.insert(cell_of.at(k)); order.push_back(cell_of.at(k)); });
    if (2 * shown.used >= nG) {  // FilterAdjacency iterates G's node order then
      std::sort(order.begin(), order.end(),
                [&](int a, int b) { return G.idx.at(a) < G.idx.at(b); });
    }
    hallways.push_back(std::move(members));
    hall_order.push_back(std::move(order));
  }
  // get_branches (:223-259): components of G minus non-junction solution points
  std::unordered_set<int> rm_b;
  for (int v : s_nodes)
    if (!p.count(v)) rm_b.insert(v);
  const std::unordered_set<int> h0_nodes(s_nodes.begin(), s_nodes.end());
  const std::vector<int> h0_order(H0.order);  // solution_branch is a Graph: its node order
  std::vector<char> taken(hallways.size() + 1, 0);
  double prod = 1.0, sum = 0.0;  // p = 1 / s = 0, over branches 1..m then branch 0
  for (const auto& comp : components(G, rm_b)) {
    const std::unordered_set<int> bset(comp.begin(), comp.end());
    double cx = 0.0;
    bool any = false;
    for (size_t i = 0; i <= hallways.size(); ++i) {
      if (taken[i]) continue;
      const std::unordered_set<int>& hs = i == 0 ? h0_nodes : hallways[i - 1];
      bool sub = true;
      for (int v : hs)
        if (!bset.count(v)) { sub = false; break; }
      if (!sub) continue;
      taken[i] = 1;
      const double c = i == 0 ? hallway_complexity(H0, d_sol, h0_nodes, h0_order)
                              : hallway_complexity(G, dmap, hallways[i - 1], hall_order[i - 1]);
      cx = any ? cx + c : 0 + c;  // s = 0; s += ...
      any = true;
    }
    prod *= (any ? cx : 0.0) + 1;  // p *= complexity_of_branch(h) + 1
    sum += any ? cx : 0.0;         // s += complexity_of_branch(b)
  }
  const double c0 = hallway_complexity(H0, d_sol, h0_nodes, h0_order);  // branch 0 = [0], last
  prod *= c0;
  sum += c0;
  if (prod_out) *prod_out = prod;
  if (difficulty) {
    if (!(prod > 0.0)) return MZ_EINVAL;  // math.log domain error in the reference
    *difficulty = std::log(prod);
  }
  if (complexity) {
    if (!(sum > 0.0)) return MZ_EINVAL;
    *complexity = std::log(sum);
  }
  return MZ_OK;
}

}  // namespace

extern "C" int mz_difficulty(const uint8_t* g, int32_t H, int32_t W, int32_t sr, int32_t sc,
                             int32_t gr, int32_t gc, double* out) {
  if (!out) return MZ_EINVAL;
  return mcclendon(g, H, W, sr, sc, gr, gc, out, nullptr);
}

extern "C" int mz_maze_complexity(const uint8_t* g, int32_t H, int32_t W, int32_t sr, int32_t sc,
                                  int32_t gr, int32_t gc, double* difficulty, double* complexity) {
  if (!difficulty && !complexity) return MZ_EINVAL;
  return mcclendon(g, H, W, sr, sc, gr, gc, difficulty, complexity);
}

// The product difficulty_of_maze takes the log of (the quantity k_mcclendon outputs): the
// best-of-C selection's host fallback for candidates the GPU kernel declines (mz_api.hip).
int mz_mcclendon_host_prod(const uint8_t* g, int32_t H, int32_t W, int32_t sr, int32_t sc,
                           int32_t gr, int32_t gc, double* prod) {
  if (!prod) return MZ_EINVAL;
  return mcclendon(g, H, W, sr, sc, gr, gc, nullptr, nullptr, prod);
}
