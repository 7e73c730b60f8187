#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/golden.json (run in the build
container, where /root/reference exists; never on the GPU box).

Every value here is produced by the REFERENCE's own CPU code
(revised_perman/cpu_algos.hpp, compiled unmodified by `make -C oracle ref`
into oracle/_ref/ref_v2):
  dense    parallel_perman64<double,double>        cpu_algos.hpp:761
  dense_q  parallel_perman64<__float128,double>    (reference -q mode; the accuracy golden)
  sparse   parallel_perman64_sparse<double,double> cpu_algos.hpp:635
  skip     parallel_skip_perman64_w_balanced       cpu_algos.hpp:1035
  order    the reference's SortOrder / SkipOrder rewrite of the matrix (util.h:813, 964)

  read     the reference's MatrixMarket reader (mmio.c + read_matrix.hpp) — stored
           as sha256 of the fp64 matrix bytes
  reduce   the -o / -u driver (main.cpp:993-1259, restated in the harness) over the
           reference's own d1compress / d2compress / d34compress / scalesk
           (util.h), leaves by parallel_perman64<double,double>
  leaves   the same reductions' leaf matrices — stored as count + sha256

Inputs: (a) copies of reference corpus files (tests/fixtures/*, data only,
including the MatrixMarket files under tests/fixtures/mtx/) and (b) small
synthetic matrices in the same v1 format, generated here with a fixed seed
(tests/fixtures/synth/*).

usage: python tests/golden/make_golden.py [--quick]
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
FIX = os.path.join(ROOT, "tests", "fixtures")
SYN = os.path.join(FIX, "synth")
OUT = os.path.join(ROOT, "tests", "golden", "golden.json")
REF_V2 = os.path.join(ROOT, "oracle", "_ref", "ref_v2")

CORPUS = ["int/30_0.50_0", "double/30_0.50_0", "double/30_0.20_0", "int/30_0.20_0", "float/30_0.50_0",
          "double/32_0.50_0", "double/36_0.20_0", "double/40_0.50_0", "int/36_0.20_0",
          "real/ibm32.mtxzero"]


def write_v1(path: str, a: np.ndarray, typ: str) -> None:
    n = a.shape[0]
    nz = [(i, j, a[i, j]) for i in range(n) for j in range(n) if a[i, j] != 0]
    with open(path, "w") as f:
        f.write(f"{n} {len(nz)} {typ}\n")
        for i, j, v in nz:
            f.write(f"{i} {j} {int(v) if typ == 'int' else repr(float(v))}\n")


def synth() -> list[str]:
    """Small seeded matrices in the reference corpus' style (Bernoulli(d)
    pattern; int values U{1..5}, double values U(0,5)), plus edge cases."""
    os.makedirs(SYN, exist_ok=True)
    names = []
    rng = np.random.default_rng(20261015)
    for n in (1, 2, 3, 4, 5, 7, 8, 9, 12, 16, 17, 20, 22):
        for typ in ("int", "double"):
            for d in (0.5, 0.2):
                pat = rng.random((n, n)) < d
                pat[np.arange(n), rng.permutation(n)] = True  # no empty row/column
                vals = rng.integers(1, 6, (n, n)) if typ == "int" else rng.random((n, n)) * 5
                a = np.where(pat, vals, 0)
                name = f"{n}_{d:.2f}_{typ}"
                write_v1(os.path.join(SYN, name), a, typ)
                names.append("synth/" + name)
    # edge cases: all-ones J_n (perm = n!), identity, a zero row, negative entries
    for n in (6, 10, 12):
        write_v1(os.path.join(SYN, f"ones_{n}"), np.ones((n, n), dtype=int), "int")
        names.append(f"synth/ones_{n}")
    write_v1(os.path.join(SYN, "ident_9"), np.eye(9, dtype=int), "int")
    names.append("synth/ident_9")
    z = rng.integers(0, 4, (10, 10))
    z[3, :] = 0
    z[0, 0] = 1  # header nnz irrelevant; row 3 empty -> perm 0
    write_v1(os.path.join(SYN, "zero_row_10"), z, "int")
    names.append("synth/zero_row_10")
    neg = np.round(rng.standard_normal((14, 14)) * 2, 3)
    neg[rng.random((14, 14)) < 0.4] = 0
    write_v1(os.path.join(SYN, "neg_14"), neg, "double")
    names.append("synth/neg_14")
    return names


def ref(path: str, algo: str, threads: int = 8, binary: int = 0, prep: int = 0) -> str:
    r = subprocess.run([REF_V2, path, algo, str(threads), str(binary), str(prep)], capture_output=True,
                       text=True, check=True)
    return r.stdout.strip()


MTX_DIRS = ["revised_perman/matrices", "revised_perman/elektrik_matrices/known_perman"]
# (file, min_n, scale threshold or -1): reductions whose leaves / result are pinned
MTX_REDUCE = [("Tina_DisCog_p.mtx", 30, -1), ("Trefethen_20_s.mtx", 30, -1), ("can_24_ps.mtx", 20, -1),
              ("can_24_ps.mtx", 20, 4), ("ibm32_p.mtx", 30, -1), ("ibm32_p.mtx", 20, -1), ("ibm32_p.mtx", 20, 4),
              ("mycielskian5_ps.mtx", 20, -1), ("mycielskian5_ps.mtx", 20, 4), ("chesapeake.mtx", 20, -1),
              ("chesapeake.mtx", 30, -1), ("will57.mtx", 30, -1), ("dwt_59.mtx", 30, -1)]
MTX_PERM_REDUCE = [("Tina_DisCog_p.mtx", 30, -1), ("Trefethen_20_s.mtx", 30, -1), ("can_24_ps.mtx", 20, -1),
                   ("can_24_ps.mtx", 20, 4), ("ibm32_p.mtx", 20, -1), ("ibm32_p.mtx", 20, 4),
                   ("mycielskian5_ps.mtx", 20, -1), ("mycielskian5_ps.mtx", 20, 4), ("chesapeake.mtx", 20, -1)]


def leaves_digest(text: str) -> dict:
    """count + sha256 of the fp64 bytes of every leaf (harness 'leaves' output)."""
    import hashlib
    lines = text.strip().splitlines()
    h, sizes, i = hashlib.sha256(), [], 0
    while i < len(lines) and lines[i].startswith("leaf"):
        k = int(lines[i].split()[1])
        m = np.array([[float(x) for x in ln.split()] for ln in lines[i + 1:i + 1 + k]], dtype=np.float64)
        h.update(np.ascontiguousarray(m.reshape(k, k)).tobytes())
        sizes.append(k)
        i += 1 + k
    return {"count": len(sizes), "sha256": h.hexdigest(), "max_n": max(sizes) if sizes else 0}


def mtx_goldens(gold: dict, put) -> None:
    import glob
    import hashlib
    dst = os.path.join(FIX, "mtx")
    os.makedirs(dst, exist_ok=True)
    for d in MTX_DIRS:
        for f in sorted(glob.glob(os.path.join(REF, d, "*.mtx"))):
            if not os.path.exists(os.path.join(dst, os.path.basename(f))):
                shutil.copy(f, dst)
    for f in sorted(glob.glob(os.path.join(dst, "*.mtx"))):
        name = "mtx/" + os.path.basename(f)
        for b in (0, 1):
            key = f"{name}|read|b{b}|sha256"
            if key not in gold:
                txt = ref(f, "read", 1, b)
                m = np.array([[float(x) for x in ln.split()] for ln in txt.splitlines()], dtype=np.float64)
                put(key, hashlib.sha256(np.ascontiguousarray(m).tobytes()).hexdigest())
                put(f"{name}|read|b{b}|n", int(m.shape[0]))
        n = int([ln for ln in open(f) if not ln.startswith("%")][0].split()[0])
        key = f"{name}|dense|r0|b0|t8"
        if n <= 30 and key not in gold:
            put(key, float(ref(f, "dense", 8).split()[0]))
    for fn, min_n, thr in MTX_REDUCE:
        key = f"mtx/{fn}|leaves|n{min_n}|u{thr}"
        if key not in gold:
            r = subprocess.run([REF_V2, os.path.join(dst, fn), "leaves", "1", "0", "0", str(min_n), str(thr)],
                               capture_output=True, text=True, check=True)
            put(key, leaves_digest(r.stdout))
    for fn, min_n, thr in MTX_PERM_REDUCE:
        key = f"mtx/{fn}|reduce|n{min_n}|u{thr}|t8"
        if key not in gold:
            r = subprocess.run([REF_V2, os.path.join(dst, fn), "reduce", "8", "0", "0", str(min_n), str(thr)],
                               capture_output=True, text=True, check=True)
            put(key, float(r.stdout.split()[0]))
            print(key, r.stdout.strip(), flush=True)


def main() -> None:
    quick = "--quick" in sys.argv
    if not os.path.exists(REF_V2):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    os.makedirs(FIX, exist_ok=True)
    for c in CORPUS:
        dst = os.path.join(FIX, c.replace("/", "__"))
        if not os.path.exists(dst):
            shutil.copy(os.path.join(REF, c), dst)
    gold = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            gold = json.load(f)

    def put(key: str, val) -> None:
        gold[key] = val
        with open(OUT, "w") as f:
            json.dump(gold, f, indent=1, sort_keys=True)

    mtx_goldens(gold, put)
    names = synth()
    for name in names:
        p = os.path.join(FIX, name)
        n = int(open(p).readline().split()[0])
        for algo in ("dense", "sparse", "skip") + (("dense_q",) if n <= 22 else ()):
            for prep in ((0, 1, 2) if algo in ("sparse", "skip") else (0,)):
                key = f"{name}|{algo}|r{prep}|b0|t4"
                if key not in gold:
                    put(key, float(ref(p, algo, 4, 0, prep).split()[0]))
        for prep in (1, 2):
            key = f"{name}|order|r{prep}"
            if key not in gold:
                put(key, ref(p, "order", 1, 0, prep))
        key = f"{name}|dense|r0|b1|t4"
        if key not in gold:
            put(key, float(ref(p, "dense", 4, 1, 0).split()[0]))
    # corpus: fp64 at 8 threads, then (slow) quad accuracy goldens
    plan = [("int__30_0.50_0", "dense", 0, 0), ("double__30_0.50_0", "dense", 0, 0),
            ("double__30_0.20_0", "dense", 0, 0), ("int__30_0.20_0", "dense", 0, 0),
            ("float__30_0.50_0", "dense", 0, 0), ("int__30_0.50_0", "dense", 0, 1),
            ("double__30_0.20_0", "sparse", 1, 0), ("double__30_0.20_0", "skip", 2, 0),
            ("int__30_0.20_0", "sparse", 1, 0), ("int__30_0.20_0", "skip", 2, 0),
            ("double__32_0.50_0", "dense", 0, 0), ("real__ibm32.mtxzero", "skip", 2, 0)]
    if not quick:
        plan += [("double__30_0.50_0", "dense_q", 0, 0), ("int__30_0.50_0", "dense_q", 0, 0),
                 ("double__30_0.20_0", "dense_q", 0, 0), ("int__30_0.20_0", "dense_q", 0, 0),
                 # round 6: BASELINE config 2's matrix through the reference's -q mode
                 # (parallel_perman64<__float128,double>, ~15 min on 8 cores): the exact path's
                 # value at n = 32 against the reference's own quad result
                 ("double__32_0.50_0", "dense_q", 0, 0),
                 ("double__36_0.20_0", "sparse", 1, 0), ("int__36_0.20_0", "skip", 2, 0),
                 # the metric config (n = 40) and its d = 0.2 companion through the reference's own
                 # parallel_perman64<double,double> (cpu_algos.hpp:761-873): ~55 min each on 8 cores
                 ("double__40_0.50_0", "dense", 0, 0), ("double__40_0.20_0", "dense", 0, 0)]
    for name, algo, prep, binary in plan:
        key = f"{name}|{algo}|r{prep}|b{binary}|t8"
        if key not in gold:
            out = ref(os.path.join(FIX, name), algo, 8, binary, prep).split()
            put(key, float(out[0]))
            put(key + "|seconds", float(out[1]))
            print(key, out, flush=True)
    for name in ("int__30_0.20_0", "double__36_0.20_0", "int__36_0.20_0"):
        for prep in (1, 2):
            key = f"{name}|order|r{prep}"
            if key not in gold:
                put(key, ref(os.path.join(FIX, name), "order", 1, 0, prep))


if __name__ == "__main__":
    main()
