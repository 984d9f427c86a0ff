#!/bin/bash
# A/B of PONITA variants selected by an env var ($VAR): the PONITA GPU tests under each value,
# then one short C3 bench per value (interleaved twice).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/abp
VAR="${VAR:-NBX_PO_FK_LDS}"
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python -u -m pytest tests -m gpu -k ponita -q -x -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/abp/tests_$v.log 2>&1
  rc=$?; echo "tests $v: $(tail -1 gpurun_out/abp/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 200 python bench.py --model ponita --steps 10 --warmup 2 --no-cpu-baseline \
        > gpurun_out/abp/$v.json 2> gpurun_out/abp/$v.err
    rc=$?; [ $rc -ne 0 ] && { echo "variant $v rc=$rc"; tail -3 gpurun_out/abp/$v.err; exit $rc; }
    python - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/abp/{sys.argv[1]}.json").read().strip().splitlines()[-1])
pk = {v["role"] if "role" in v else k[:30]: v["avg_launch_us"] for k, v in d["roofline"]["per_kind"].items()}
print(sys.argv[1], d["value"], "steps/s", pk)
PY
  done
done
