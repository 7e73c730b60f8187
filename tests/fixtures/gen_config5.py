"""Synthetic inputs for BASELINE config 5 (n = 44, d = 0.15), which the
reference corpora lack.

Same semantics as the corpora: Bernoulli(d) pattern per entry, `int` values
U{1..5}, `double` values U(0,5); v1 file format (`n nnz type`, then 0-based
`i j v`).  Seed = 1000·n + round(100·d)·10 + rep, fed to
numpy's MT19937; matrices with an empty row or column (perm = 0) are
rejected and the next rep is drawn.

    python tests/fixtures/gen_config5.py   # writes tests/fixtures/synth44_0.15_{int,double}
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def generate(n: int, d: float, typ: str, rep: int = 0) -> tuple[np.ndarray, int]:
    while True:
        rng = np.random.Generator(np.random.MT19937(1000 * n + round(100 * d) * 10 + rep))
        pat = rng.random((n, n)) < d
        vals = rng.integers(1, 6, (n, n)) if typ == "int" else rng.random((n, n)) * 5.0
        if pat.any(0).all() and pat.any(1).all():
            return np.where(pat, vals, 0), rep
        rep += 1


def write_v1(path: str, a: np.ndarray, typ: str) -> None:
    n = a.shape[0]
    nz = [(i, j, a[i, j]) for i in range(n) for j in range(n) if a[i, j] != 0]
    with open(path, "w") as f:
        f.write(f"{n} {len(nz)} {typ}\n")
        for i, j, v in nz:
            f.write(f"{i} {j} {int(v) if typ == 'int' else repr(float(v))}\n")


if __name__ == "__main__":
    for typ in ("int", "double"):
        a, rep = generate(44, 0.15, typ)
        path = os.path.join(HERE, f"synth44_0.15_{typ}")
        write_v1(path, a, typ)
        print(path, "rep", rep, "nnz", int((a != 0).sum()))
