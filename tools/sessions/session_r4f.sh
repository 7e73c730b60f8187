# round-4 session F: code-generation knobs on the near-dense d = 0.9 walk (interleaved A/B on one box) and its
# stall counters on the final kernel; the 8-rank bench path from plain python (--gpus 8 --rehearse: 8 processes,
# gloo, all on GPU 0)
P="rocprofv3 --kernel-trace -o run --output-format csv"
CHILD="python3 bench.py --pmc-child --kernel dense --jit 1 --prep 0 --matrix tests/fixtures/double__40_0.90_0"
O=gpurun_out/r4f
bash tools/gpu_session.sh r4f \
 "ab_d090=env PROBE_TORCH=1 PROBE_CASES=double__40_0.90_0 python3 tools/probe_ab.py SUP_JIT_KP=3 SUP_JIT_KP=6 SUP_JIT_CC=2 SUP_JIT_B=4 SUP_JIT_PF=0 SUP_JIT_XSTEP=0 SUP_JIT_PRIO=1 -" \
 "pmc_wait_d090=$P --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc_wait_d090 -- $CHILD" \
 "rehearse8=python3 bench.py --gpus 8 --rehearse --steps 2 --warmup 1 --configs 0 --cpu-seconds 0 --pmc 0 --cold 0"
