"""Config 5 through the ahead-of-time SkipPer kernel (`-p8 -s -r2 --jit -1`,
walk_skip<44>): kernel time per call, visited states, and the permanent
against the segmented walk's (<= 1.8 s per step)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import superman_amd._lib as _L  # noqa: E402
if len(sys.argv) > 2:  # experiments: another build of the library
    _L.LIB_PATH = os.path.abspath(sys.argv[2])
import superman_amd as S  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
a = S.skip_order(S.read_matrix(os.path.join(ROOT, "tests", "fixtures", "synth44_0.15_int"))[0])[0]
seg = S.perman(a, 8, sparse=True, jit=1)
for i in range(reps):
    r, st = S.perman(a, 8, sparse=True, jit=-1, return_stats=True)
    print(f"skip kernel: {st['kernel_ms']:.1f} ms, walk_kind {st['walk_kind']}, visited "
          f"{st['visited_steps'] / st['gray_steps']:.4f}, permanent {r!r} (segmented {seg!r}, rel "
          f"{abs(r - seg) / abs(seg):.2e})", flush=True)
