# round-3 session O: final tree — smoke, bench line (reads the committed HBM/F64 profiles of the same plan keys),
# rocprofv3 stats of the headline, and the CLI with a checkpoint end to end on the bench matrix (-p6)
bash tools/gpu_session.sh r3o \
 smoke \
 "bench=python3 bench.py" \
 "prof=rocprofv3 --kernel-trace --stats -d gpurun_out/r3o/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --configs 0 --also= --pmc 0 --cold 0" \
 "ckpt_cli=rm -f /tmp/b40.ckpt && superman_amd/bin/perman -f tests/fixtures/double__40_0.50_0 -g -p6 -d1 --jit 1 --checkpoint /tmp/b40.ckpt && superman_amd/bin/perman -f tests/fixtures/double__40_0.50_0 -g -p6 -d1 --jit 1 --checkpoint /tmp/b40.ckpt -v | grep -E 'Checkpoint|Permanent' && superman_amd/bin/perman -f tests/fixtures/double__40_0.50_0 -g -p4 --jit 1 | grep Permanent"
