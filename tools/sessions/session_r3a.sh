# round-3 session A: new GPU tests (multi-rank shards, reference wrappers,
# RCCL slots), the budget probe, F64 / HBM PMC passes, exact ground truth
bash tools/gpu_session.sh r3a \
 "python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_multi.py tests/test_gpu_capi_runalgo.py tests/test_gpu_parity.py::test_rccl_combine_single_device" \
 "python3 -u tools/probe_budgets.py double__40_0.50_0 186 190 198 206 214" \
 "rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d gpurun_out/r3a/pmc_f64_d050 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0" \
 "rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r3a/pmc_fetch_d050 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0" \
 "rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r3a/pmc_write_d050 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0" \
 "rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d gpurun_out/r3a/pmc_f64_d090 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0 --matrix tests/fixtures/double__40_0.90_0" \
 "python3 -u tools/probe_exact_truth.py"
