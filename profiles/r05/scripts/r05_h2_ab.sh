#!/bin/bash
# Round-5 A/B: fp16x2 split path (default) vs bf16x3 (NBX_SPLIT=x3) on the C2 headline.
set -o pipefail
O=gpurun_out/r05/h2_ab
mkdir -p $O
timeout -k 10 60 ./tools/ubench/mfma_f16_denorm > $O/mfma_f16_denorm.txt 2>&1; cat $O/mfma_f16_denorm.txt
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_segnn.py -k "forward_matches_oracle or c2_full_batch or rollout_c2" \
    > $O/gpu_segnn.log 2>&1; tail -15 $O/gpu_segnn.log
for i in 1 2; do
    timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_h2_$i.json 2> $O/bench_h2_$i.err || exit 1
    NBX_SPLIT=x3 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_x3_$i.json 2> $O/bench_x3_$i.err || exit 1
done
# per-wave phase clocks of every TP kernel (stage / loop / epilogue), both paths
NBX_TP_DEBUG=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/dbg_h2.json 2> $O/dbg_h2.err || exit 1
NBX_SPLIT=x3 NBX_TP_DEBUG=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/dbg_x3.json 2> $O/dbg_x3.err || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
for f in $O/bench_*.json; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])")"; done
