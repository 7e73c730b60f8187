# round-4 session T: LLVM machine-scheduler strategies for the generated walk (SUP_JIT_SCHED), interleaved on one box
bash tools/gpu_session.sh r4t \
 "ab_sched=env PROBE_TORCH=1 PROBE_CASES=double__40_0.50_0,double__40_0.90_0,double__40_0.20_0 python3 tools/probe_ab.py SUP_JIT_SCHED=max-ilp SUP_JIT_SCHED=max-memory-clause SUP_JIT_SCHED=iterative-maxocc - SUP_JIT_SCHED=max-ilp"
