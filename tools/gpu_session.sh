#!/bin/bash
# One GPU session on the MI355X box: each step under its own time limit; stop
# at the first crash/timeout (exit codes 124/134/137/139 or >128), keep going
# after ordinary failures (test failures, a rejected counter name).
# usage: tools/gpu_session.sh <tag> [steps...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=${1//[^A-Za-z0-9_.-]/_} secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -4 "$OUT/$name.log"
  if [ $rc -eq 124 ] || [ $rc -ge 128 ]; then echo "STOP: $name exit $rc"; exit $rc; fi
  return 0
}
BENCH1="python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also= --configs 0 ${BENCH_EXTRA:-}"
prof_pmc() {  # name counters...
  local name=$1; shift
  run "$name" 600 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv -- $BENCH1
}
rocm-smi --showproductname --showclocks > "$OUT/rocm_smi.log" 2>&1 || true
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()";;
    test)  run pytest_gpu 1200 python3 -m pytest tests -m gpu -q -x -p no:cacheprovider;;
    testall) run pytest_gpu 1200 python3 -m pytest tests -m gpu -q -p no:cacheprovider;;
    bench) run bench 600 python3 bench.py --steps 3 --warmup 1;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --also= --configs 0 ${BENCH_EXTRA:-};;
    list)  run counters 120 rocprofv3 -L;;
    pmc)   prof_pmc pmc_fetch FETCH_SIZE
           prof_pmc pmc_write WRITE_SIZE
           prof_pmc pmc_sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
           prof_pmc pmc_lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY;;
    pmcsqc) run pmc_sqc 120 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_WAVE_CYCLES --kernel-trace -d "$OUT/pmc_sqc" -o run --output-format csv -- $BENCH1;;
    probe) run probe 300 python3 tools/probe.py;;
    pmc44) for k in sparse skip; do
             run "pmc44_sq_$k" 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d "$OUT/pmc44_sq_$k" -o run --output-format csv -- python3 tools/run_one.py synth44_0.15_int 2 $k
             run "pmc44_wait_$k" 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_ANY --kernel-trace -d "$OUT/pmc44_wait_$k" -o run --output-format csv -- python3 tools/run_one.py synth44_0.15_int 2 $k
           done;;
    *=*) run "${step%%=*}" 900 bash -c "${step#*=}";;   # name=command
    *) run "$step" 900 bash -c "$step";;
  esac
done
echo "== done"
