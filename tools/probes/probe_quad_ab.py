"""-o -q (double-double leaves) with and without the chunk-end check
(SUP_NO_CHUNK_ENDS), wall times; prints as it goes.

    python3 tools/probes/probe_quad_ab.py [matrix.mtx[:both|:on] ...]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CODE = """
import os, sys, time
sys.path.insert(0, {root!r})
import superman_amd as S
m = S.read_mtx(os.path.join({root!r}, "tests", "fixtures", "mtx", {name!r}))[0]
t = time.perf_counter()
(hi, lo), st = S.perman_reduced_quad(m, return_stats=True)
print("quad", repr(hi), repr(lo), "%.2f s" % (time.perf_counter() - t), st["leaves"], "leaves", flush=True)
"""
for arg in sys.argv[1:] or ["will57.mtx"]:
    name, _, mode = arg.partition(":")
    for off in (("0", "1") if mode in ("", "both") else ("0",)):
        env = dict(os.environ, SUP_NO_CHUNK_ENDS=off)
        r = subprocess.run([sys.executable, "-c", CODE.format(root=ROOT, name=name)], env=env,
                           capture_output=True, text=True)
        print(name, "SUP_NO_CHUNK_ENDS=" + off, r.stdout.strip(), r.stderr.strip()[-300:], flush=True)
