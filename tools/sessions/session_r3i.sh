# round-3 session I: lane id re-read + static queue head; suite, A/B, HBM
P="rocprofv3 --kernel-trace -o run --output-format csv"
B1="python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0 --pmc 0 --cold 0"
bash tools/gpu_session.sh r3i \
 "pytest_gpu=python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 "ab_static=python3 -u tools/probe_ab.py SUP_WALK_NOSTATIC=1" \
 "pmc_fetch_d050=$P --pmc FETCH_SIZE -d gpurun_out/r3i/pmc_fetch_d050 -- $B1" \
 "pmc_write_d050=$P --pmc WRITE_SIZE -d gpurun_out/r3i/pmc_write_d050 -- $B1" \
 "pmc_tcc_d050=$P --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum -d gpurun_out/r3i/pmc_tcc_d050 -- $B1" \
 "shards=python3 -u tools/probe_shards.py" \
 "bench=python3 bench.py"
