# round-3 session E: opaque_c A/B (config 3 slower than round 2?), chunk-group
# tail probe, and what the walk's WRITE_SIZE is made of
P="rocprofv3 --kernel-trace -o run --output-format csv"
B5="python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0 --pmc 0 --cold 0"
bash tools/gpu_session.sh r3e \
 "ab_opaque=python3 -u tools/probe_ab.py SUP_JIT_OPAQUE_R2=1" \
 "group=python3 -u tools/probe_group.py double__40_0.50_0 16 8 4 32" \
 "pmc_tcc_d050=$P --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum -d gpurun_out/r3e/pmc_tcc_d050 -- $B5"
