#!/bin/bash
# rocprofv3 kernel summaries + HBM PMC passes for the bench lines (one rocprofv3 run per pass,
# each under its own time limit; stops at the first failure).  Usage:
#   bash scripts/profile_models.sh [models...]     (default: segnn ponita egnn_mc egnn_mc_train segnn_train ponita_train eqv2_train eqv2 gravity)
# Output: gpurun_out/prof/<model>/{stats,fetch,write}/ and gpurun_out/prof/<model>_summary.md,
#         gpurun_out/prof/pmc_<model>.json (per-kernel HBM bytes per launch)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
MODELS="${*:-segnn ponita egnn_mc egnn_mc_train segnn_train ponita_train eqv2_train eqv2 gravity}"
declare -A ARGS=(
  [segnn]="--model segnn --steps 20 --warmup 2 --no-cpu-baseline"
  [ponita]="--model ponita --steps 4 --warmup 1 --no-cpu-baseline"
  [egnn_mc]="--model egnn_mc --steps 50 --warmup 5 --no-cpu-baseline"
  [egnn_mc_train]="--model egnn_mc_train --steps 20 --warmup 3 --no-cpu-baseline"
  [segnn_train]="--model segnn_train --steps 10 --warmup 2 --no-cpu-baseline"
  [ponita_train]="--model ponita_train --steps 10 --warmup 2 --no-cpu-baseline"
  [eqv2_train]="--model eqv2_train --steps 10 --warmup 2 --no-cpu-baseline --eager"
  [eqv2]="--model eqv2 --steps 5 --warmup 1 --no-cpu-baseline"
  [eqv2_l6]="--model eqv2_l6 --steps 3 --warmup 1 --no-cpu-baseline"
  [gravity]="--model gravity --steps 200 --warmup 10 --no-cpu-baseline"
)
mkdir -p gpurun_out/prof
for m in $MODELS; do
  a="${ARGS[$m]}"
  d=gpurun_out/prof/$m
  mkdir -p $d
  echo "[$(date +%T)] $m: kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/stats -o run -- python bench.py $a \
      > $d/stats.log 2>&1 || { echo "$m stats failed"; tail -5 $d/stats.log; exit 1; }
  for p in FETCH_SIZE WRITE_SIZE; do
    echo "[$(date +%T)] $m: pmc $p"
    timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d $d/$p -o run -- python bench.py $a \
        > $d/$p.log 2>&1 || { echo "$m $p failed"; tail -5 $d/$p.log; exit 1; }
  done
  python tools/pmc_report.py $d gpurun_out/prof/pmc_$m.json > /dev/null
  stats=$(ls $d/stats/*kernel_stats.csv 2>/dev/null | head -1)
  [ -z "$stats" ] && stats=$(find $d/stats -name "*kernel_stats.csv" | head -1)
  python tools/kernel_summary.py "$stats" gpurun_out/prof/pmc_$m.json gpurun_out/prof/${m}_summary.md \
      "python bench.py $a"
  cp "$stats" gpurun_out/prof/${m}_kernel_stats.csv
  grep "^{\"metric\"" $d/stats.log | tail -n 1 > gpurun_out/prof/bench_${m}.json || true
  echo "$m done"
done
