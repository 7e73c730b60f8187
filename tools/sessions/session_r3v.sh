# round-3 session V: bit-set walk-order planning — per-call overhead with a new matrix per call, the reduction
# tests, dwt_59 at 1 and 8 leaf workers
bash tools/gpu_session.sh r3v \
 "overhead=python3 -u tools/probe_overhead.py" \
 "reduce_tests=python3 -u -m pytest -q --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_reduce_workers.py -m gpu" \
 "dwt59=python3 -u -c \"
import os, sys, time
sys.path.insert(0, '.')
import superman_amd as S
a = S.read_mtx('tests/fixtures/mtx/dwt_59.mtx')[0]
for w in ('8', '1'):
    os.environ['SUP_LEAF_WORKERS'] = w
    t = time.perf_counter(); v, st = S.perman_reduced(a, algo=4, return_stats=True); wall = time.perf_counter() - t
    print('dwt_59 workers', w, st['leaves'], 'leaves wall %.2f s kernels %.2f s perm %r' % (wall, st['kernel_ms'] / 1e3, v), flush=True)
\""
