#!/bin/bash
# Round-4 GPU session: the SEGNN / training GPU tests touched by this round's changes, then the
# measurement session (scripts/r04_profile.sh).  Stops at the first GPU failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
echo "[$(date +%T)] tests"
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
    ${TESTS:-tests/test_gpu_segnn.py tests/test_gpu_segnn_train.py tests/test_gpu_ponita_train.py tests/test_gpu_eqv2_train.py} > gpurun_out/r04/tests.log 2>&1
rc=$?
echo "[$(date +%T)] tests rc=$rc"; grep -E "passed|failed" gpurun_out/r04/tests.log | tail -2
grep "C2 long rollout" gpurun_out/r04/tests.log | tail -4 | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
[ -n "${NO_PROFILE:-}" ] && exit 0
bash scripts/r04_profile.sh
