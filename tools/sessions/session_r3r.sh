# round-3 session R (final tree): GPU suite, smoke, A/B of static wave priority (SUP_JIT_PRIO, one box,
# interleaved three times), -o probe with concurrent leaves (double-double and exact reductions included in the suite)
PROBE_TORCH=1 PROBE_CASES=double__40_0.50_0,double__40_0.90_0,double__40_0.20_0,double__36_0.20_0 bash tools/gpu_session.sh r3r \
 "pytest_gpu=python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 smoke \
 "prio=python3 -u tools/probe_ab.py SUP_JIT_PRIO=1 - SUP_JIT_PRIO=1 - SUP_JIT_PRIO=1" \
 "probe_reduce=python3 -u tools/probe_reduce.py chesapeake.mtx will57.mtx"
