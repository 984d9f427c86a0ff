#!/bin/bash
# Round-4 GPU session: the whole -m gpu suite (as the driver runs it), then the PONITA fibre A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
echo "[$(date +%T)] gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 240 --timeout-method thread \
    > gpurun_out/r04/gpu_suite.log 2>&1
rc=$?
echo "[$(date +%T)] gpu suite rc=$rc"; grep -E "passed|failed" gpurun_out/r04/gpu_suite.log | tail -2
if [ $rc -ne 0 ]; then exit $rc; fi
[ -n "${NO_AB:-}" ] && exit 0
bash scripts/r04_ponita_ab.sh ${AB_VALS:-1024 512 256}
