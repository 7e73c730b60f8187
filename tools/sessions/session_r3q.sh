# round-3 session Q: A/B of static wave priority (SUP_JIT_PRIO) on one box, interleaved three times
PROBE_TORCH=1 PROBE_CASES=double__40_0.50_0,double__40_0.90_0,double__40_0.20_0,double__36_0.20_0 bash tools/gpu_session.sh r3q2 \
 "prio=python3 -u tools/probe_ab.py SUP_JIT_PRIO=1 - SUP_JIT_PRIO=1 - SUP_JIT_PRIO=1"
