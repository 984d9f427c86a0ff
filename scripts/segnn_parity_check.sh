#!/bin/bash
# r06: parity items on the GPU -- rollout ensemble placement per path, then the SEGNN parity, path,
# range-guard and hand-off invariant tests
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/r06/${1:-c}
mkdir -p $O
[ -n "${PATHS:-}" ] && { timeout -k 10 400 python -u scripts/rollout_paths.py "" NBX_UPD_DV=0 NBX_SPLIT=x3 NBX_X3=0 > $O/paths.log 2>&1 || exit $?; }
[ -n "${PATHS:-}" ] && grep "==" $O/paths.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_segnn.py tests/test_gpu_segnn_paths.py tests/test_gpu_segnn_range.py \
    -x -v --timeout 600 --timeout-method thread -s -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
