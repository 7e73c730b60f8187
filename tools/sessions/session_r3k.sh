# round-3 session K: the tree with up to 4 cached walk bits and 16 polish starts — suite,
# shard probe, bench line, rocprofv3 stats, the profiles the bench reads
P="rocprofv3 --kernel-trace -o run --output-format csv"
B1="python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0 --pmc 0 --cold 0"
F64="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
bash tools/gpu_session.sh r3k \
 "pytest_gpu=python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 "shards=python3 -u tools/probe_shards.py" \
 "bench=python3 bench.py" \
 "prof=rocprofv3 --kernel-trace --stats -d gpurun_out/r3k/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --configs 0 --also= --pmc 0 --cold 0" \
 "pmc_f64_d050=$P --pmc $F64 -d gpurun_out/r3k/pmc_f64_d050 -- $B1" \
 "pmc_fetch_d050=$P --pmc FETCH_SIZE -d gpurun_out/r3k/pmc_fetch_d050 -- $B1" \
 "pmc_write_d050=$P --pmc WRITE_SIZE -d gpurun_out/r3k/pmc_write_d050 -- $B1" \
 "pmc_tcc_d050=$P --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum -d gpurun_out/r3k/pmc_tcc_d050 -- $B1" \
 "pmc_f64_d020=$P --pmc $F64 -d gpurun_out/r3k/pmc_f64_d020 -- $B1 --matrix tests/fixtures/double__40_0.20_0" \
 "pmc_f64_d090=$P --pmc $F64 -d gpurun_out/r3k/pmc_f64_d090 -- $B1 --matrix tests/fixtures/double__40_0.90_0"
