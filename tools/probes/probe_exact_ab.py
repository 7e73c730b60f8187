"""-o -E (exact leaves) with and without the chunk-end check (SUP_NO_CHUNK_ENDS),
beside -o -q (double-double leaves): the exact results must not move.

    python3 tools/probes/probe_exact_ab.py [matrix.mtx ...]
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
names = sys.argv[1:] or ["will57.mtx"]
CODE = """
import os, sys, time
sys.path.insert(0, {root!r})
import numpy as np
import superman_amd as S
m = S.read_mtx(os.path.join({root!r}, "tests", "fixtures", "mtx", {name!r}))[0]
t = time.perf_counter()
v, st = S.perman_reduced_exact(m.astype(np.int32), return_stats=True)
print("exact", v, "%.2f s" % (time.perf_counter() - t), st["leaves"], "leaves", flush=True)
"""
for name in names:
    for off in ("0", "1"):
        env = dict(os.environ, SUP_NO_CHUNK_ENDS=off)
        r = subprocess.run([sys.executable, "-c", CODE.format(root=ROOT, name=name)], env=env,
                           capture_output=True, text=True)
        print(name, "SUP_NO_CHUNK_ENDS=" + off, r.stdout.strip(), r.stderr.strip()[-300:], flush=True)
