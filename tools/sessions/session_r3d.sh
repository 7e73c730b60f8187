# round-3 session D: walk length of the segmented walk (current code), and the
# d = 0.9 kernel's stall counters (scalar cache, instruction cache, waits)
P="rocprofv3 --kernel-trace -o run --output-format csv"
B9="python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0 --pmc 0 --cold 0 --matrix tests/fixtures/double__40_0.90_0"
bash tools/gpu_session.sh r3d \
 "walklen=PROBE_CASES=double__40_0.50_0,double__40_0.90_0,double__40_0.20_0,double__32_0.50_0 python3 -u tools/probe_walklen.py 0 14 15 16" \
 "pmc_sqc_d090=$P --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_WAVE_CYCLES -d gpurun_out/r3d/pmc_sqc_d090 -- $B9" \
 "pmc_wait_d090=$P --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/r3d/pmc_wait_d090 -- $B9" \
 "pmc_wait_d050=$P --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/r3d/pmc_wait_d050 -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0 --pmc 0 --cold 0"
