#!/bin/bash
# Round-4 measurement session 2: the composed lmax 6 EquiformerV2 bench, the deterministic-BN A/B on
# C2, then kernel summaries + HBM PMC passes of the HEAD binaries for every bench line
# (scripts/profile_models.sh).  Every GPU step under its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
run() {
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -n 1 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "$O/$name.log"; exit $rc; fi
}
run eqv2_l6 300 python bench.py --model eqv2_l6
run segnn_atomic 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline
run segnn_det 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --deterministic-bn
run segnn_atomic2 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline
run segnn_det2 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --deterministic-bn
bash scripts/profile_models.sh ${PROFILE_MODELS:-segnn ponita eqv2 eqv2_l6 eqv2_train egnn_mc egnn_mc_train gravity} || exit $?
echo done
