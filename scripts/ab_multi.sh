#!/bin/bash
# A/B/C... of several environment settings on the C2 bench, interleaved, in one box session:
#   bash scripts/ab_multi.sh ROUNDS "" "NBX_UPD2_PF=16" "NBX_UPD1_PF=5 NBX_UPD2_PF=16" ...
# prints steps/s and the per-kind kernel averages (us) of every run
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/ab
R="$1"; shift
for i in $(seq 1 $R); do
  j=0
  for e in "$@"; do
    j=$((j+1))
    timeout -k 10 120 env $e python bench.py --steps 200 --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab/v$j.$i.json 2>gpurun_out/ab/v$j.$i.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab/v$j.$i.json'));k=d['roofline']['per_kind'];print('[$e]', d['value'], [round(x['avg_launch_us'],2) for x in k.values()])"
  done
done
