mkdir -p gpurun_out/s4h
for r in 210 220 230 240; do
  SUP_JIT_REGMAX=$r SUP_JIT_VERBOSE=1 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --also= --configs 0 > gpurun_out/s4h/r$r.log 2>&1 || exit $?
  echo "regmax $r: $(grep -o 'seg plan.*' gpurun_out/s4h/r$r.log | head -1 | cut -c1-80) $(grep '^{' gpurun_out/s4h/r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_avg"])')"
done
