# round-3 session Q: A/B of static wave priority (SUP_JIT_PRIO) on the bench matrix and d = 0.9, one box,
# interleaved: default, prio, default, prio
PROBE_TORCH=1 PROBE_CASES=double__40_0.50_0,double__40_0.90_0 bash tools/gpu_session.sh r3q \
 "prio=python3 -u tools/probe_ab.py SUP_JIT_PRIO=1 - SUP_JIT_PRIO=1"
