#!/bin/bash
# EquiformerV2 GPU session: parity tests -> timing -> kernel profile (logs in gpurun_out/).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-tests time prof}"
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -n 20 "gpurun_out/$name.log"; echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for s in $STEPS; do
  case $s in
    tests) run eqv2_tests 500 python -u -m pytest tests/test_gpu_eqv2.py -v -p no:cacheprovider --timeout 240 --timeout-method thread
           grep -E "PASS|FAIL|^E +Assert|passed|failed" gpurun_out/eqv2_tests.log | tail -12 ;;
    time)  run eqv2_time 300 python -u tools/eqv2_time.py; cat gpurun_out/eqv2_time.log | grep -v amdgpu ;;
    prof)  rm -rf gpurun_out/prof_eqv2
           run prof_eqv2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_eqv2 -o eqv2 \
               -- python tools/eqv2_time.py --iters 5 --frames 3
           python tools/kstats.py gpurun_out/prof_eqv2/eqv2_kernel_stats.csv ;;
  esac
done
