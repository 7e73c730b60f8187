#!/bin/bash
# Round-6 GPU sessions: each step under its own time limit, stop at the first
# crash / timeout (exit >= 124), keep going after ordinary test failures.
# usage: tools/session_r6.sh <tag> <step>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "$O/$name.log"
  if [ $rc -eq 124 ] || [ $rc -ge 128 ]; then echo "STOP: $name exit $rc"; exit $rc; fi
}
PYT="python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider"
for step in "$@"; do
  case $step in
    rccl) run pytest_rccl 900 $PYT tests/test_gpu_rccl_branch.py;;
    rccl_parity) run pytest_rccl_parity 600 $PYT tests/test_gpu_parity.py -k "rccl or schedulers";;
    skip_tests) run pytest_skip 900 $PYT tests/test_gpu_parity.py tests/test_gpu_pinned.py tests/test_gpu_checkpoint.py \
                  tests/test_gpu_multidev.py -k "skip or config5 or p8 or sparse_and_skipper";;
    skip_forms) run pytest_skip_forms 600 $PYT tests/test_gpu_skip_forms.py tests/test_gpu_fuzz.py tests/test_gpu_maxsize.py;;
    skip_time) run probe_skip 300 python3 -u tools/probes/probe_skip.py 3;;
    skip_pmc) run pmc_skip 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_ADD_F64 \
                SQ_INSTS_VALU_MUL_F64 SQ_WAVES SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_skip -o run \
                --output-format csv -- python3 tools/probes/probe_skip.py 1;;
    cold) run cold_start 400 python3 -c "import sys, json; sys.path.insert(0, '.'); import bench; print(json.dumps(bench.cold_start('tests/fixtures/double__40_0.50_0'), indent=1))";;
    trace) run probe_trace 400 python3 -u tools/probes/probe_trace.py;;
    trace_cfg2) run probe_trace_cfg2 400 python3 -u tools/probes/probe_trace.py double__32_0.50_0 --walk-log2 0 9 11;;
    pmc_cfg2) run pmc_cfg2 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU \
                SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc_cfg2 -o run --output-format csv -- \
                python3 bench.py --pmc-child --matrix tests/fixtures/double__32_0.50_0 --kernel dense --jit 1;;
    multidev) SUP_CHECK_DEVICE=1 run pytest_multidev 800 $PYT tests/test_gpu_multidev.py;;
    bench_cold) run bench_cold 400 python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0 --pmc 0;;
    gpu_all) run pytest_gpu 1200 $PYT tests -m gpu;;
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()";;
    bench) run bench 900 python3 bench.py;;
    stats) run stats 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
             python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --configs 0 --also= --pmc 0 --cold 0;;
    rehearse)
      for g in 2 4 8; do
        run rehearse_$g 400 python3 bench.py --gpus $g --rehearse --steps 3 --warmup 1 --cpu-seconds 0 --pmc 0 --cold 0
      done;;
    hbm)  # FETCH_SIZE / WRITE_SIZE passes (separate: TCC counter limits) of every bench walk
      P="rocprofv3 --kernel-trace -o run --output-format csv"
      while read -r tag m k j pr w vis; do
        [ -n "${HBM_ONLY:-}" ] && [ "$tag" != "$HBM_ONLY" ] && continue
        C="python3 bench.py --pmc-child --matrix tests/fixtures/$m --kernel $k --jit $j --prep $pr"
        run fetch_$tag 240 $P --pmc FETCH_SIZE -d $O/fetch_$tag -- $C
        run write_$tag 240 $P --pmc WRITE_SIZE -d $O/write_$tag -- $C
        run sum_$tag 300 python3 tools/pmc_r4.py $O/pmc_hbm_$tag.json tests/fixtures/$m $O/fetch_$tag $O/write_$tag \
          --kernel $k --jit $j --prep $pr --walk "$w" $vis
      done <<'LIST'
d050 double__40_0.50_0 dense 1 0 sup_walk_seg
d020 double__40_0.20_0 dense 1 0 sup_walk_seg
d090 double__40_0.90_0 dense 1 0 sup_walk_seg
cfg2 double__32_0.50_0 dense 1 0 sup_walk_seg
cfg3 double__36_0.20_0 sparse 1 1 sup_walk_seg
cfg5skip synth44_0.15_int skip -1 2 walk_skip<44> --visited
cfg5 synth44_0.15_int skip 0 2 sup_walk_seg --visited
LIST
      ;;
    *) echo "unknown step $step"; exit 2;;
  esac
done
echo "== done"
