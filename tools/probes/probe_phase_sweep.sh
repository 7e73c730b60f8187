# Phase offset between the two waves of a SIMD (SUP_JIT_PHASE: odd workgroups sleep 64 k cycles at entry).
mkdir -p gpurun_out/phase
for ph in 0 2 4 8; do
  SUP_JIT_PHASE=$ph timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --also= --configs 0 > gpurun_out/phase/ph$ph.log 2>&1 || exit $?
  echo "phase $ph: $(grep '^{' gpurun_out/phase/ph$ph.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_avg"])')"
done
