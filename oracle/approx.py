"""TEST INFRASTRUCTURE ONLY — restatement of the randomized estimators.

Plain-Python restatement of the reference's estimators as this engine runs
them (superman_amd/csrc/approx_core.hpp), used by tests to pin the C++/HIP
code sample by sample:
  * Rasmussen — kernel_rasmussen, gpu_approximation_dense.cu:155-229 (row with
    the fewest remaining nonzeros, first on ties; X *= its degree; a uniformly
    drawn remaining column is removed; X = 0 when a row runs out);
  * scaling-guided sampling — kernel_approximation,
    gpu_approximation_dense.cu:231-371 (Sinkhorn passes every `intervals`
    steps, `times` passes each, fp32 factors and fp64 sums; column j drawn with
    probability d_r[row]·d_c[j] / S; X /= p_j).
The reference draws from curand (XORWOW, seeded rand()*tid); the engine uses
Philox4x32-10 (Salmon et al., SC'11) with counter (sample, step), restated
here and checked against the published known-answer vectors.  Statistical
parity with the permanent itself is tested separately (unbiasedness).
"""
from __future__ import annotations

import numpy as np

M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = (int(x) & MASK for x in ctr)
    k0, k1 = (int(x) & MASK for x in key)
    for _ in range(10):
        p0, p1 = M0 * c0, M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & MASK, p1 & MASK, ((p0 >> 32) ^ c3 ^ k1) & MASK, p0 & MASK
        k0, k1 = (k0 + W0) & MASK, (k1 + W1) & MASK
    return c0, c1, c2, c3


def draw(seed: int, sample: int, step: int):
    return philox4x32_10((sample & MASK, sample >> 32, step, 0x5AB1E), (seed & MASK, (seed >> 32) & MASK))


def _f32(x: float) -> float:
    return float(np.float32(x))


def _pick_row(rowsets, rows_left, cols_left):
    best, brow, live = len(rowsets) + 1, 0, []
    for r, cs in enumerate(rowsets):
        m = [c for c in cs if c in cols_left]
        if r in rows_left and len(m) < best:
            best, brow, live = len(m), r, m
    return best, brow, live


def rasmussen_sample(a, seed: int, sample: int) -> tuple[float, bool]:
    n = a.shape[0]
    rowsets = [sorted(np.nonzero(a[r])[0].tolist()) for r in range(n)]
    rows_left, cols_left = set(range(n)), set(range(n))
    est = 1.0
    for it in range(n):
        best, row, live = _pick_row(rowsets, rows_left, cols_left)
        if best == 0:
            return 0.0, True
        est *= float(best)
        u = draw(seed, sample, it)[0]
        k = (u * best) >> 32
        col = live[k]
        cols_left.discard(col)
        rows_left.discard(row)
    return est, False


def scaling_sample(a, intervals: int, times: int, seed: int, sample: int) -> tuple[float, bool]:
    n = a.shape[0]
    rowsets = [sorted(np.nonzero(a[r])[0].tolist()) for r in range(n)]
    colsets = [sorted(np.nonzero(a[:, c])[0].tolist()) for c in range(n)]
    rows_left, cols_left = set(range(n)), set(range(n))
    dr, dc = [1.0] * n, [1.0] * n
    est = 1.0
    for it in range(n):
        _, row, live = _pick_row(rowsets, rows_left, cols_left)
        if intervals > 0 and it % intervals == 0:
            for _ in range(times):
                for j in sorted(cols_left):
                    s = 0.0
                    for i in colsets[j]:
                        if i in rows_left:
                            s += dr[i]
                    if s == 0.0:
                        return 0.0, True
                    dc[j] = _f32(1.0 / s)
                for i in sorted(rows_left):
                    s = 0.0
                    for j in rowsets[i]:
                        if j in cols_left:
                            s += dc[j]
                    if s == 0.0:
                        return 0.0, True
                    dr[i] = _f32(1.0 / s)
        rr = dr[row]
        S = 0.0
        for j in live:
            S += rr * dc[j]
        if S == 0.0:
            return 0.0, True
        d = draw(seed, sample, it)
        bits = ((d[0] << 21) ^ (d[1] >> 11)) & ((1 << 53) - 1)
        target = float(bits + 1) * (1.0 / 9007199254740992.0) * S
        acc, pj, col = 0.0, 0.0, 0
        for j in live:
            s = rr * dc[j]
            acc += s
            col, pj = j, s / S
            if target <= acc:
                break
        est /= pj
        cols_left.discard(col)
        rows_left.discard(row)
    return est, False


def pairwise64(v):
    v = list(v) + [0.0] * (64 - len(v))
    w = 64
    while w > 1:
        v = [v[2 * i] + v[2 * i + 1] for i in range(w // 2)]
        w //= 2
    return v[0]


def block_sums(a, method: str, seed: int, block: int, intervals: int = 4, times: int = 5):
    """(sum, sum of squares, zero count) of samples 64*block .. 64*block+63, in
    the engine's pairwise order."""
    e = []
    for lane in range(64):
        s = 64 * block + lane
        e.append(rasmussen_sample(a, seed, s) if method == "rasmussen" else
                 scaling_sample(a, intervals, times, seed, s))
    vals = [x for x, _ in e]
    return pairwise64(vals), pairwise64([x * x for x in vals]), pairwise64([1.0 if z else 0.0 for _, z in e])


def domino_tilings(m: int, n: int) -> int:
    """Number of domino tilings of an m x n board, exact (column transfer
    matrix over the profile of dominoes sticking into the next column)."""
    if m > n:
        m, n = n, m
    if (m * n) % 2:
        return 0
    from functools import lru_cache

    @lru_cache(maxsize=None)
    def fill(col: int, mask: int) -> int:
        if col == n:
            return 1 if mask == 0 else 0
        total = 0

        def rec(row: int, cur: int, nxt: int):
            nonlocal total
            if row == m:
                total += fill(col + 1, nxt)
                return
            if cur >> row & 1:
                rec(row + 1, cur, nxt)
                return
            rec(row + 1, cur, nxt | (1 << row))  # horizontal domino into the next column
            if row + 1 < m and not (cur >> (row + 1) & 1):
                rec(row + 2, cur, nxt)  # vertical domino
        rec(0, mask, 0)
        return total

    return fill(0, 0)
