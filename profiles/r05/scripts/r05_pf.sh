#!/bin/bash
# Round-5 A/B (temporary switches): A-ring depth of the fp16x2 node TPs (NBX_PF) and message kernel (NBX_MSG_D).
set -o pipefail
O=gpurun_out/r05/pf
mkdir -p $O
for r in 1 2; do
  for v in "" "NBX_PF=5" "NBX_PF=7" "NBX_MSG_D=4" "NBX_MSG_D=5"; do
    tag=${v:-base}; tag=${tag//=/_}
    env $v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_${tag}_$r.json 2> $O/bench_${tag}_$r.err || exit 1
  done
done
for f in $O/bench_*.json; do echo "$f $(python -c "
import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], [round(v['avg_launch_us'],2) for v in d['roofline']['per_kind'].values()])")"; done
