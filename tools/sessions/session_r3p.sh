# round-3 session P: -o reductions on the GPU, one leaf at a time (SUP_LEAF_WORKERS=1) against 4 and 8
# concurrent leaves on their own context lanes; the GPU reduction tests; dwt_59 (145,798 leaves) at 1 and 4
bash tools/gpu_session.sh r3p \
 "probe_reduce=python3 -u tools/probe_reduce.py" \
 "reduce_tests=python3 -u -m pytest -q --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_reduce_workers.py -m gpu -k 'reduce or workers'" \
 "dwt59=python3 -u -c \"
import os, sys, time
sys.path.insert(0, '.')
import superman_amd as S
a = S.read_mtx('tests/fixtures/mtx/dwt_59.mtx')[0]
for w in ('4', '1'):
    os.environ['SUP_LEAF_WORKERS'] = w
    t = time.perf_counter(); v, st = S.perman_reduced(a, algo=4, return_stats=True); wall = time.perf_counter() - t
    print('dwt_59 workers', w, st['leaves'], 'leaves wall %.2f s kernels %.2f s perm %r' % (wall, st['kernel_ms'] / 1e3, v), flush=True)
\""
