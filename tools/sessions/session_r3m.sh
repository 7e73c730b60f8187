# round-3 session M: logical-device map (SUP_DEVICE_MAP) tests + the whole GPU suite; hiprtc key by content
# (plan keys printed on the box to compare with the build container); HBM/F64 PMC passes summarised ON THE
# BOX (tools/pmc_r3.py computes the plan key there), then the bench line, which reads them
P="rocprofv3 --kernel-trace -o run --output-format csv"
B1="python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0 --pmc 0 --cold 0"
F64="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
O=gpurun_out/r3m
M20=tests/fixtures/double__40_0.20_0
M90=tests/fixtures/double__40_0.90_0
M50=tests/fixtures/double__40_0.50_0
bash tools/gpu_session.sh r3m \
 "stat=stat -c '%n %s %Y' /usr/local/lib/python3.10/dist-packages/torch/lib/libhiprtc.so /opt/rocm/lib/libhiprtc.so.7.2.70200" \
 "multidev=python3 -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_multidev.py -m gpu" \
 "pytest_gpu=python3 -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu" \
 "keys=python3 -c \"import torch, superman_amd as S; [print(f, hex(S.plan_key(S.read_matrix(f)[0], 'dense', jit=1))) for f in ('$M50', '$M20', '$M90')]\"" \
 "pmc_fetch_d050=$P --pmc FETCH_SIZE -d $O/pmc_fetch_d050 -- $B1" \
 "pmc_write_d050=$P --pmc WRITE_SIZE -d $O/pmc_write_d050 -- $B1" \
 "pmc_f64_d050=$P --pmc $F64 -d $O/pmc_f64_d050 -- $B1" \
 "pmc_fetch_d020=$P --pmc FETCH_SIZE -d $O/pmc_fetch_d020 -- $B1 --matrix $M20" \
 "pmc_write_d020=$P --pmc WRITE_SIZE -d $O/pmc_write_d020 -- $B1 --matrix $M20" \
 "pmc_f64_d020=$P --pmc $F64 -d $O/pmc_f64_d020 -- $B1 --matrix $M20" \
 "pmc_f64_d090=$P --pmc $F64 -d $O/pmc_f64_d090 -- $B1 --matrix $M90" \
 "sum=python3 tools/pmc_r3.py hbm $O/pmc_fetch_d050 $O/pmc_write_d050 profiles/r3/pmc_hbm_d050.json $M50 && python3 tools/pmc_r3.py hbm $O/pmc_fetch_d020 $O/pmc_write_d020 profiles/r3/pmc_hbm_d020.json $M20 && python3 tools/pmc_r3.py f64 $O/pmc_f64_d050 profiles/r3/pmc_f64_d050.json $M50 && python3 tools/pmc_r3.py f64 $O/pmc_f64_d020 profiles/r3/pmc_f64_d020.json $M20 && python3 tools/pmc_r3.py f64 $O/pmc_f64_d090 profiles/r3/pmc_f64_d090.json $M90 && cp profiles/r3/pmc_hbm_d0*.json profiles/r3/pmc_f64_d0*.json $O/" \
 "bench=python3 bench.py" \
 "prof=rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --configs 0 --also= --pmc 0 --cold 0"
