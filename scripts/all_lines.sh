#!/bin/bash
# Every bench line at HEAD without the CPU-baseline legs, one after another on one box,
# each under its own time limit; stops at the first failure.  Output: gpurun_out/all_lines/<model>.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out=gpurun_out/${ROUND:-r06}/all_lines
mkdir -p $out
for m in ${MODELS:-segnn ponita egnn_mc eqv2 eqv2_l6 gravity segnn_train ponita_train eqv2_train egnn_mc_train}; do
  timeout -k 10 300 python bench.py --model $m --no-cpu-baseline > $out/$m.log 2>&1 || { echo "$m failed"; tail -8 $out/$m.log; exit 1; }
  echo "$m: $(grep '^{' $out/$m.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d.get("cpu_baseline") or {}; print(d["value"], d["unit"], d["ms_per_step"], "cpu", c.get("value"), c.get("unit"))')"
done
