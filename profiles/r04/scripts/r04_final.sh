#!/bin/bash
# Round-4 closing GPU session at HEAD: the whole -m gpu suite (as the driver runs it), smoke(), the default
# bench line (as the driver runs it, CPU baseline included), then refreshed kernel summaries + PMC traffic
# for the lines this round's last changes touched.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
out=gpurun_out/final
mkdir -p $out
echo "[$(date +%T)] gpu suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $out/gpu_suite.log 2>&1
rc=$?
echo "[$(date +%T)] gpu suite rc=$rc"; grep -E "passed|failed|error" $out/gpu_suite.log | tail -2
[ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] smoke"
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -3 $out/smoke.log
echo "[$(date +%T)] bench (default)"
timeout -k 10 600 python bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
grep '^{' $out/bench.log | tail -1 | cut -c1-400
if [ -n "${AB_ENV:-}" ]; then
  echo "[$(date +%T)] training A/B ($AB_ENV)"
  ROUNDS=${ROUNDS:-1} MODELS="${AB_MODELS:-segnn_train ponita_train}" bash scripts/ab_train_env.sh || exit 1
fi
[ -n "${NO_PROFILE:-}" ] && exit 0
bash scripts/profile_models.sh ${PROFILE_MODELS:-ponita gravity}
