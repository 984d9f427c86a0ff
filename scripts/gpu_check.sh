#!/bin/bash
# One GPU session: smoke -> GPU tests -> bench -> rocprofv3 kernel trace.
# Stops at the first step that exits with anything other than 0 / 1 (fault,
# abort, timeout), per the pool rules.  Logs land in gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-smoke tests bench prof}"
run() {
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for s in $STEPS; do
  case $s in
    smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run gpu_tests 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} ;;
    bench) run bench 600 python bench.py --steps 100 --warmup 10 ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o segnn \
               -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline ;;
    pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o segnn \
               -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline &&
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o segnn \
               -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline &&
           python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_tp_kernels.json ;;
  esac
done
echo done
