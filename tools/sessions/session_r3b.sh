# round-3 session B: the whole GPU suite on the current tree (walk_common.hpp's
# opaque_c changed every kernel's address code), budget probe, bench line, PMC
P="rocprofv3 --kernel-trace -o run --output-format csv"
B1="python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0"
bash tools/gpu_session.sh r3b \
 "pytest_gpu=python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 "budgets=python3 -u tools/probe_budgets.py double__40_0.50_0 190 206 214 222" \
 "bench=python3 bench.py --steps 5 --warmup 1" \
 "pmc_f64_d050=$P --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/r3b/pmc_f64_d050 -- $B1" \
 "pmc_fetch_d050=$P --pmc FETCH_SIZE -d gpurun_out/r3b/pmc_fetch_d050 -- $B1" \
 "pmc_write_d050=$P --pmc WRITE_SIZE -d gpurun_out/r3b/pmc_write_d050 -- $B1" \
 "pmc_f64_d090=$P --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/r3b/pmc_f64_d090 -- $B1 --matrix tests/fixtures/double__40_0.90_0" \
 "pmc_f64_d020=$P --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/r3b/pmc_f64_d020 -- $B1 --matrix tests/fixtures/double__40_0.20_0"
