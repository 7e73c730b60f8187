#!/bin/bash
# The segmented walk on the bench matrix, its d = 0.2 companion and BASELINE
# configs 2, 3, 5 (one process each, 3 launches): kernel time and op model.
set -u
for spec in "double__40_0.50_0 0 seg" "double__40_0.20_0 0 seg" "double__32_0.50_0 0 seg" \
            "double__36_0.20_0 1 seg" "synth44_0.15_int 2 seg"; do
  set -- $spec
  SUP_JIT_VERBOSE=1 timeout -k 10 120 python3 tools/probes/run_one.py "$1" "$2" "$3" 3 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}
  if [ "$rc" -ne 0 ]; then echo "STOP rc=$rc"; exit "$rc"; fi
done
