#!/bin/bash
# Round-5 GPU session: the whole -m gpu suite (as the driver runs it), smoke(), then the default
# bench line (N = 1, the driver's BENCH command).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
out=gpurun_out/r05/${1:-full}
mkdir -p "$out"
echo "[$(date +%T)] gpu suite"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 240 --timeout-method thread \
    > "$out/gpu_suite.log" 2>&1
rc=$?
echo "[$(date +%T)] gpu suite rc=$rc"; grep -E "passed|failed|error" "$out/gpu_suite.log" | tail -3
[ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
echo "[$(date +%T)] bench"
timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
tail -n 1 "$out/bench.json"
