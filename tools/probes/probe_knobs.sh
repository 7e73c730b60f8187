#!/bin/bash
# A/B of segmented-walk code-generation knobs on one matrix: one process per
# setting ("NAME=VAL ..." strings), 3 launches each.
# usage: tools/probes/probe_knobs.sh <fixture> <prep> <kernel> "<env settings>"...
set -u
fx=$1 prep=$2 kern=$3; shift 3
for spec in "$@"; do
  echo -n "[$spec] "
  env $spec SUP_JIT_VERBOSE=1 timeout -k 10 120 python3 tools/probes/run_one.py "$fx" "$prep" "$kern" 3 2>&1 | grep -v amdgpu.ids | tr '\n' ' '
  rc=${PIPESTATUS[0]}
  echo
  if [ "$rc" -ne 0 ]; then echo "STOP rc=$rc"; exit "$rc"; fi
done
