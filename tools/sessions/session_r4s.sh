# round-4 session S: counters of the ahead-of-time SkipPer kernel on config 5 (the kernel itself, --jit -1), for
# where its time goes (VALU / SALU / scalar loads per visited state, waits)
P="rocprofv3 --kernel-trace -o run --output-format csv"
O=gpurun_out/r4s
RUN="python3 tools/run_one.py synth44_0.15_int 2 skip 1 -1"
bash tools/gpu_session.sh r4s \
 "sq_skip=$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $O/sq_skip -- $RUN" \
 "f64_skip=$P --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_BRANCH -d $O/f64_skip -- $RUN" \
 "wait_skip=$P --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES -d $O/wait_skip -- $RUN"
