#!/bin/bash
# Round-5 A/B: fp16x2 split path (default) vs bf16x3 (NBX_SPLIT=x3) on the C2 headline.
set -o pipefail
O=gpurun_out/r05/h2_ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_segnn.py \
    > $O/gpu_segnn.log 2>&1 || { echo "segnn gpu tests failed"; tail -30 $O/gpu_segnn.log; exit 1; }
for i in 1 2; do
    timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_h2_$i.json 2> $O/bench_h2_$i.err || exit 1
    NBX_SPLIT=x3 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_x3_$i.json 2> $O/bench_x3_$i.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
for f in $O/bench_*.json; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])")"; done
