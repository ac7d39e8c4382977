"""CPU restatements of the maze-build algorithms of mz_build.inc.h, checked against the oracle's
BFS (oracle/mzoracle.c) on oracle-generated mazes. CPU-only: this pins the algorithms the HIP
build uses; the kernels themselves are compared with the oracle on the GPU
(tests/test_gpu_env.py::test_generated_distance_field_matches_bfs and the generation tests).

  * mz_tree_dist / mz_cs_dist: on a perfect maze, the distance to the goal from the carve depths
    (distance from the start): parents at depth - 1, the goal's root path marked, in-place
    pointer jumping to each square's first path ancestor a(x), D = dep(x) + dep(goal) - 2 dep(a(x)).
  * mz_build_cells' passage rule: an open passage square is one step from the nearer of its two
    cells.
  * the toroidal build's BFS over row masks (one N-bit row per lane, a level = rotate / shift / or /
    and-not of the frontier rows).
"""
import numpy as np
import pytest

import pyoracle as O


def _tree_dist(g, start, goal):
    N = g.shape[0]
    dep = O.bfs(g, start).ravel()  # the carve depth: distance from the start in the tree
    gf = g.ravel()
    C = N * N
    s, t = start[0] * N + start[1], goal[0] * N + goal[1]
    A = np.full(C, -1)
    for p in np.flatnonzero(gf):
        if p == s:
            A[p] = p
            continue
        r, c = divmod(p, N)
        for q, ok in ((p - N, r > 0), (p + N, r + 1 < N), (p - 1, c > 0), (p + 1, c + 1 < N)):
            if ok and gf[q] and dep[q] == dep[p] - 1:
                A[p] = q
        assert A[p] >= 0, "a square without a parent: not a tree"
    mark = np.zeros(C, bool)
    x = t
    while True:
        mark[x] = True
        if x == s:
            break
        x = A[x]
    for _ in range(32):  # in place, as the lanes interleave
        changed = False
        for p in np.flatnonzero(A >= 0):
            a = A[p]
            if not mark[a]:
                A[p] = A[a]
                changed = True
        if not changed:
            break
    else:
        raise AssertionError("pointer jumping did not converge")
    D = np.full(C, -1)
    for p in np.flatnonzero(A >= 0):
        a = p if mark[p] else A[p]
        D[p] = dep[p] + dep[t] - 2 * dep[a]
    return D.reshape(N, N)


@pytest.mark.parametrize("dim", [9, 15, 41, 81])
@pytest.mark.parametrize("algo", [0, 1, 2])
def test_tree_distance_equals_bfs(dim, algo):
    for k in range(3):
        (sr, sc), (gr, gc), g = O.generate(dim, algo, 0x7EE0 + 97 * dim + k)
        want = O.bfs(g, (gr, gc))
        got = _tree_dist(g, (sr, sc), (gr, gc))
        op = g != 0
        np.testing.assert_array_equal(got[op], want[op])


@pytest.mark.parametrize("dim", [15, 41, 81])
def test_passage_distance_from_its_cells(dim):
    for algo in range(3):
        _, (gr, gc), g = O.generate(dim, algo, 0x9A55 + dim + algo)
        D = O.bfs(g, (gr, gc))
        for r in range(dim):
            for c in range(dim):
                if not g[r, c] or (r & 1 and c & 1):
                    continue  # walls and cells
                a, b = ((r, c - 1), (r, c + 1)) if r & 1 else ((r - 1, c), (r + 1, c))
                assert D[r, c] == min(D[a], D[b]) + 1


def _torus_bfs_rows(g, goal):
    N = g.shape[0]
    mask = (1 << N) - 1
    O_ = [sum(1 << x for x in range(N) if g[y, x]) for y in range(N)]
    V = [0] * N
    F = [0] * N
    V[goal[0]] = F[goal[0]] = 1 << goal[1]
    D = np.full((N, N), -1)
    D[goal] = 0
    level = 0
    while True:
        level += 1
        nxt = []
        for y in range(N):
            f = F[y]
            reach = (f | ((f << 1) & mask) | (f >> (N - 1)) | (f >> 1) | ((f & 1) << (N - 1)) |
                     F[(y - 1) % N] | F[(y + 1) % N])
            nw = reach & O_[y] & ~V[y]
            V[y] |= nw
            nxt.append(nw)
            x = 0
            while nw:
                if nw & 1:
                    D[y, x] = level
                nw >>= 1
                x += 1
        F = nxt
        if not any(F):
            return D


@pytest.mark.parametrize("dim", [9, 17, 29, 41])
def test_torus_row_mask_bfs_equals_bfs(dim):
    for algo in range(3):
        _, (gr, gc), g = O.generate(dim, algo, 0x70E0 + dim + algo, True)
        want = O.bfs(g, (gr, gc), True)
        got = _torus_bfs_rows(g, (gr, gc))
        op = g != 0
        np.testing.assert_array_equal(got[op], want[op])
