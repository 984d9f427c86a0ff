#!/bin/bash
# PONITA fibre-kernel grid A/B (NBX_PO_FIB_BLOCKS): the PONITA GPU tests and two interleaved C3 bench
# runs per value (scripts/ab_ponita.sh), then FETCH_SIZE / WRITE_SIZE passes per value for the
# po_fiber_ln_kernel HBM bytes (gpurun_out/abp/pmc_<value>.json).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
VALS="${*:-1024 512 256}"
VAR=NBX_PO_FIB_BLOCKS bash scripts/ab_ponita.sh $VALS || exit $?
for v in $VALS; do
  for p in FETCH_SIZE WRITE_SIZE; do
    env NBX_PO_FIB_BLOCKS=$v timeout -s KILL 200 rocprofv3 --pmc $p --output-format csv -d gpurun_out/abp/pmc_$v/$p \
        -o run -- python bench.py --model ponita --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abp/pmc_${v}_${p}.log 2>&1 \
        || { echo "pmc $v $p failed"; exit 1; }
  done
  python tools/pmc_report.py gpurun_out/abp/pmc_$v gpurun_out/abp/pmc_$v.json > /dev/null
  python - "$v" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/abp/pmc_{sys.argv[1]}.json"))["kernels"]
for k, x in d.items():
    if "po_fiber_ln" in k or "lin_kernel<4, 0, 3" in k:
        print(sys.argv[1], k[:60], "MB/launch", round(x.get("hbm_bytes_per_launch", 0) / 1e6, 1))
PY
done
