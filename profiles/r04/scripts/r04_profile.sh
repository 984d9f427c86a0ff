#!/bin/bash
# Round-4 measurement session: C2 bench repeats (driver shape 20/5 and 100/10), a per-dispatch
# kernel trace of the driver-shape run, then kernel summaries + HBM PMC passes of the HEAD binaries
# (scripts/profile_models.sh).  Every GPU step under its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
run() {
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -n 2 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run bench20a 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run bench20b 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run bench100 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline
run trace 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
bash scripts/profile_models.sh ${PROFILE_MODELS:-segnn segnn_train ponita_train eqv2_train} || exit $?
echo done
