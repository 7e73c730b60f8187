# round-4 session C: leaf batches (GPU bit-exactness + dwt_59 / will57 / chesapeake wall time by batch size and
# workers), the per-call cost breakdown after the fused reduction pass and the prepared shard call, the d = 0.5
# WRITE_SIZE re-measured (session B read 150 MB against round 3's 10.7 MB on the same plan key) in both the
# --pmc-child and the bench flow, and the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4c
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -eq 124 ] || [ $rc -ge 128 ]; then echo "STOP: $name exit $rc"; exit $rc; fi
}
CHILD="python3 bench.py --pmc-child --kernel dense --jit 1 --prep 0 --matrix tests/fixtures/double__40_0.50_0"
B1="python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0 --pmc 0 --cold 0"
step batch_tests 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_reduce_workers.py tests/test_gpu_parity.py -m gpu
step overhead 300 python3 tools/probe_overhead.py
step write_child_a 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write_child_a" -o run --output-format csv -- $CHILD
step write_child_b 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write_child_b" -o run --output-format csv -- $CHILD
step write_bench 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write_bench" -o run --output-format csv -- $B1
step write_tcc 120 rocprofv3 --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_ATOMIC --kernel-trace -d "$OUT/write_tcc" -o run --output-format csv -- $CHILD
step reduce_probe 900 env PROBE_SPARSE=0 PROBE_BATCHES=1,16 PROBE_WORKERS=1,8 python3 tools/probe_reduce.py chesapeake.mtx will57.mtx dwt_59.mtx
step bench 600 python3 bench.py --steps 3 --warmup 1
echo "== done"
