#!/bin/bash
# PMC passes over a short bench run, one rocprofv3 run per counter group (the
# per-pass slot limits of MI355X_MICROARCH.md: <= 8 SQ, <= 4 TCC).  Usage:
#   bash scripts/pmc_passes.sh [bench args...]    (default: the C2 SEGNN line)
# Output: gpurun_out/pmc/<pass>/ + gpurun_out/pmc/summary.json
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS="${*:---steps 3 --warmup 1 --no-cpu-baseline}"
declare -A PASSES=(
  [sq]="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
  [lds]="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS"
  [fetch]="FETCH_SIZE"
  [write]="WRITE_SIZE"
  [l2]="TCC_HIT_sum TCC_MISS_sum"
)
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
for p in sq fetch write l2 lds; do
  echo "[$(date +%T)] pass $p: ${PASSES[$p]}"
  timeout -s KILL 120 rocprofv3 --pmc ${PASSES[$p]} --output-format csv -d gpurun_out/pmc/$p -o run \
      -- python bench.py $ARGS > gpurun_out/pmc/$p.log 2>&1
  rc=$?
  echo "pass $p rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/$p.log; exit $rc; fi
done
python tools/pmc_report.py gpurun_out/pmc gpurun_out/pmc/summary.json
