"""oracle — TEST INFRASTRUCTURE ONLY (the parity checker).

ctypes access to ``oracle/liboracle.so`` (C restatement of the reference CPU
algorithms + engine-schedule mirror, see oracle.c) and an exact big-integer
Ryser for small n.  Only tests/, ``__graft_entry__.smoke()`` and bench.py's
``cpu_baseline`` leg may import this package; the product never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE, "all"], check=True, capture_output=True)
        lib = C.CDLL(LIB)
        P, I, D, LL, U = C.c_void_p, C.c_int, C.c_double, C.c_longlong, C.c_ulonglong
        lib.orc_ref_dense.argtypes = [P, I, I]
        lib.orc_ref_dense_partial.argtypes = [P, I, LL, LL, I]
        lib.orc_ref_sparse.argtypes = [P, I, I]
        lib.orc_ref_sparse_partial.argtypes = [P, I, LL, LL, I]
        lib.orc_ref_skip.argtypes = [P, I, I, C.POINTER(U)]
        lib.orc_ref_skip_partial.argtypes = [P, I, LL, LL, I]
        lib.orc_engine_range.argtypes = [P, I, I, P, I, I, I, I, U, U, I, C.POINTER(U)]
        lib.orc_engine_perman.argtypes = [P, I, I, P, I, I, I]
        lib.orc_nw_start.argtypes = [P, I, P, P]
        lib.orc_exact_mod.argtypes = [P, I, U, I]
        lib.orc_exact_mod.restype = U
        lib.orc_engine_layout.argtypes = [I, C.POINTER(I), C.POINTER(I), C.POINTER(I)]
        for f in ("orc_ref_dense", "orc_ref_dense_partial", "orc_ref_sparse", "orc_ref_sparse_partial",
                  "orc_ref_skip", "orc_ref_skip_partial", "orc_engine_range", "orc_engine_perman"):
            getattr(lib, f).restype = D
        lib.orc_nw_start.restype = None
        lib.orc_engine_layout.restype = None
        _lib = lib
    return _lib


def _d(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def ref_dense(a, threads: int = 8) -> float:
    """cpu_algos.hpp:761 parallel_perman64<double,double>."""
    a = _d(a)
    return load().orc_ref_dense(a.ctypes.data, a.shape[0], threads)


def ref_dense_partial(a, start: int, end: int, threads: int = 8) -> float:
    """gpu_exact_dense.cu:6 cpu_perman64 over [start, end)."""
    a = _d(a)
    return load().orc_ref_dense_partial(a.ctypes.data, a.shape[0], start, end, threads)


def ref_sparse(a, threads: int = 8) -> float:
    """cpu_algos.hpp:635 parallel_perman64_sparse<double,double>."""
    a = _d(a)
    return load().orc_ref_sparse(a.ctypes.data, a.shape[0], threads)


def ref_sparse_partial(a, start: int, end: int, threads: int = 8) -> float:
    a = _d(a)
    return load().orc_ref_sparse_partial(a.ctypes.data, a.shape[0], start, end, threads)


def ref_skip(a, threads: int = 8) -> tuple[float, int]:
    """cpu_algos.hpp:1035 parallel_skip_perman64_w_balanced<double,double>; (perm, visited)."""
    a = _d(a)
    v = C.c_ulonglong(0)
    r = load().orc_ref_skip(a.ctypes.data, a.shape[0], threads, C.byref(v))
    return r, v.value


def ref_skip_partial(a, start: int, end: int, threads: int = 8) -> float:
    a = _d(a)
    return load().orc_ref_skip_partial(a.ctypes.data, a.shape[0], start, end, threads)


def nw_start(a) -> tuple[np.ndarray, float]:
    a = _d(a)
    n = a.shape[0]
    x0 = np.zeros(n)
    p0 = C.c_double(0.0)
    load().orc_nw_start(a.ctypes.data, n, x0.ctypes.data, C.addressof(p0))
    return x0, p0.value


def engine_layout(n: int) -> tuple[int, int, int]:
    L, m, h = C.c_int(), C.c_int(), C.c_int()
    load().orc_engine_layout(n, C.byref(L), C.byref(m), C.byref(h))
    return L.value, m.value, h.value


KINDS = {"dense": 0, "sparse": 1, "skip": 2, "seg": 3, "lds": 0, 0: 0, 1: 1, 2: 2, 3: 3}  # lds: dense, X in LDS


def _colmap(colmap):
    if colmap is None:
        return None, None
    cm = np.ascontiguousarray(np.asarray(colmap, dtype=np.int32))
    return cm, cm.ctypes.data


def engine_range(a, kind, c0: int, c1: int, L: int, m: int, colmap=None, threads: int = 8,
                 cached: int = 0, pair_bits: int = 0) -> tuple[float, int]:
    """Engine-schedule mirror over wave-chunks [c0, c1): (partial, visited).
    colmap: engine bit -> matrix column (None = identity); cached, pair_bits:
    the segmented walk's cached walk bits and specialised pair bits
    (plan_info()["cached"], ["pair_bits"]; pair_bits 0 = the default 5)."""
    a = _d(a)
    v = C.c_ulonglong(0)
    keep, ptr = _colmap(colmap)
    r = load().orc_engine_range(a.ctypes.data, a.shape[0], KINDS[kind], ptr, int(cached), int(pair_bits), L, m, c0,
                                c1, threads, C.byref(v))
    return r, v.value


def engine_perman(a, kind="dense", colmap=None, threads: int = 8, cached: int = 0, pair_bits: int = 0) -> float:
    """Full permanent enumerated exactly as the gfx950 kernels do (bit-exact
    mirror), for walk `kind`, engine column map `colmap` and (segmented walk)
    `cached` walk bits and `pair_bits` specialised pair bits."""
    a = _d(a)
    keep, ptr = _colmap(colmap)
    return load().orc_engine_perman(a.ctypes.data, a.shape[0], KINDS[kind], ptr, int(cached), int(pair_bits),
                                    threads)


def engine_perman_as(sup_module, a, kernel="dense", threads: int = 8, jit: int = 0) -> float:
    """Mirror of exactly the plan the product runs for `kernel` (walk kind,
    column map and cached walk bits queried through the C ABI's sup_plan_info)."""
    info = sup_module.plan_info(a, kernel, jit=jit)
    n = _d(a).shape[0]
    L, m, _ = engine_layout(n)
    if (info["L"], info["m"]) == (L, m):
        return engine_perman(a, info["kind"], info["colmap"], threads, info.get("cached", 0),
                             info.get("pair_bits", 0))
    # the plan's own layout (the segmented walk lengthens its wave-chunks)
    h = n - 1 - info["L"] - info["m"]
    s, _ = engine_range(a, info["kind"], 0, 1 << h, info["L"], info["m"], info["colmap"], threads,
                        info.get("cached", 0), info.get("pair_bits", 0))
    return (4 * (n & 1) - 2) * s


def exact_perman(a) -> Fraction:
    """Exact permanent by Ryser's formula over rationals (any n <= ~22)."""
    # Independent of the reference: plain Ryser, perm = sum_{S != {}} (-1)^{n-|S|}
    # prod_i sum_{j in S} a_ij, walked in Gray order with exact rationals.
    rows = [[Fraction(v) for v in r] for r in np.asarray(a).tolist()]
    n = len(rows)
    if n == 0:
        return Fraction(1)
    s = [Fraction(0)] * n
    total = Fraction(0)
    size = 0
    prev = 0
    for i in range(1, 1 << n):
        g = i ^ (i >> 1)
        k = (g ^ prev).bit_length() - 1
        prev = g
        if (g >> k) & 1:
            size += 1
            for r in range(n):
                s[r] += rows[r][k]
        else:
            size -= 1
            for r in range(n):
                s[r] -= rows[r][k]
        p = Fraction(1)
        for r in range(n):
            if s[r] == 0:
                p = Fraction(0)
                break
            p *= s[r]
        total += p if (n - size) % 2 == 0 else -p
    return total


def _is_prime(n: int) -> bool:
    if n < 2:
        return False
    for q in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % q == 0:
            return n == q
    d, s = n - 1, 0
    while d % 2 == 0:
        d, s = d // 2, s + 1
    for b in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        x = pow(b, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def exact_perman_crt(a, threads: int = 8) -> int:
    """Exact permanent of an integer matrix, independent of the engine's exact
    path: plain Ryser over all 2^n column subsets modulo primes just below
    2^55 (oracle.c orc_exact_mod), joined here by CRT with Python integers.
    |perm| <= prod_i sum_j |a_ij| fixes how many primes are needed."""
    a = np.ascontiguousarray(np.asarray(a), dtype=np.int64)
    n = a.shape[0]
    bound = 1
    for r in np.abs(a).sum(axis=1).tolist():
        bound *= int(r)
    if bound == 0:
        return 0
    primes, M, c = [], 1, (1 << 55) - 1
    while M <= 2 * bound:
        if _is_prime(c):
            primes.append(c)
            M *= c
        c -= 2
    x, mod = 0, 1
    for p in primes:
        r = int(load().orc_exact_mod(a.ctypes.data, n, p, threads))
        # x' = x + mod * ((r - x) / mod mod p)
        t = (r - x) * pow(mod, -1, p) % p
        x, mod = x + mod * t, mod * p
    return x - M if x > M // 2 else x


def exact_perman_brute(a) -> Fraction:
    """Permanent by definition (sum over permutations) — tiny n only (n <= 8)."""
    from itertools import permutations
    rows = [[Fraction(v) for v in r] for r in np.asarray(a).tolist()]
    n = len(rows)
    total = Fraction(0)
    for perm in permutations(range(n)):
        p = Fraction(1)
        for i in range(n):
            p *= rows[i][perm[i]]
        total += p
    return total
