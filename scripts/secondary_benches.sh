#!/bin/bash
# Secondary bench lines (C3 PONITA, C1 EGNN-MC, C5 integrator) -> gpurun_out/sec/*.json, each
# step under its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/sec
for m in ponita egnn_mc gravity; do
  timeout -k 10 300 python bench.py --model $m > gpurun_out/sec/$m.json 2> gpurun_out/sec/$m.err
  rc=$?; echo "$m rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/sec/$m.err; exit $rc; }
  tail -c 300 gpurun_out/sec/$m.json
done
