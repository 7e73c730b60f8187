# round-4 session L: pieces per region without the prefetch's double SGPR set (SUP_JIT_KP 5-8 with SUP_JIT_PF=0)
# against the default (4, prefetch), near-dense and bench matrices, interleaved on one box
bash tools/gpu_session.sh r4l \
 "ab_kp=env PROBE_TORCH=1 PROBE_CASES=double__40_0.90_0,double__40_0.50_0 python3 tools/probe_ab.py SUP_JIT_KP=5 SUP_JIT_KP=5,SUP_JIT_PF=0 SUP_JIT_KP=6,SUP_JIT_PF=0 SUP_JIT_KP=8,SUP_JIT_PF=0 -"
