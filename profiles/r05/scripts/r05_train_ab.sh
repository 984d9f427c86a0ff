#!/bin/bash
# Same-box A/B of the training steps: the current library vs a tagged side build (NBX_LIB), interleaved,
# two rounds.  usage: bash scripts/r05_train_ab.sh <out tag> <lib path> <model> [<model> ...]
set -o pipefail
O=gpurun_out/r05/${1:-train_ab}
LIBB=$2
shift 2
mkdir -p $O
for r in 1 2; do
  for m in "$@"; do
    timeout -k 10 200 python bench.py --model $m --steps 50 --warmup 5 --no-cpu-baseline > $O/${m}_cur_$r.json 2> $O/${m}_cur_$r.err || exit 1
    NBX_LIB=$LIBB timeout -k 10 200 python bench.py --model $m --steps 50 --warmup 5 --no-cpu-baseline > $O/${m}_alt_$r.json 2> $O/${m}_alt_$r.err || exit 1
  done
done
for f in $O/*.json; do echo "$f $(python -c "import json; print(json.load(open('$f'))['value'])")"; done
