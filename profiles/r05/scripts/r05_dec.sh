#!/bin/bash
# Round-5 check of the msg_pre hand-off fix: corruption stress (scripts/r05_pairs.py) of the default
# build, then the C2 bench against the block-barrier hand-off build (libnbx_dec0.so), interleaved.
set -o pipefail
O=gpurun_out/r05/${1:-dec}
mkdir -p $O
P=extending-the-n-body-benchmark-a-cross-model-study-of-geometric-deep-learning-architectures_amd/lib
timeout -k 10 600 python -u scripts/r05_pairs.py 1000 '' > $O/pairs.log 2>&1 || exit 1
cat $O/pairs.log
for r in 1 2; do
  for v in "" "NBX_LIB=$P/libnbx_dec0.so"; do
    tag=${v:-base}; tag=$(echo "$tag" | sed "s#[^ ]*/lib/libnbx_##; s#\.so##" | tr -c "A-Za-z0-9_\n" "_")
    env $v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_${tag}_$r.json 2> $O/bench_${tag}_$r.err || exit 1
  done
done
for f in $O/bench_*.json; do echo "$f $(python -c "
import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], [round(v['avg_launch_us'],2) for v in d['roofline']['per_kind'].values()])")"; done
