#!/bin/bash
# A/B of SEGNN kernel variants: GPU SEGNN tests once, then one short bench per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/ab
VAR="${VAR:-NBX_MSG_VARIANT}"
timeout -k 10 300 python -m pytest tests/test_gpu_segnn.py -q -x -p no:cacheprovider > gpurun_out/ab/tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab/tests.log; [ $rc -ne 0 ] && exit $rc
for v in "$@"; do
  env $VAR=$v timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err
  rc=$?; [ $rc -ne 0 ] && { echo "variant $v rc=$rc"; tail -3 gpurun_out/ab/$v.err; exit $rc; }
  python - "$v" <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/ab/{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], "steps/s", {k.split("(")[0][-40:]: v["avg_launch_us"] for k, v in d["roofline"]["per_kind"].items()})
PY
done
