#!/bin/bash
# Round-5: XCD-grouped TP block order + fp16x2; accuracy of the three split paths on the small configs.
set -o pipefail
O=gpurun_out/r05/xcd
mkdir -p $O
for v in h2 x3 fp32; do
    case $v in h2) E="";; x3) E="NBX_SPLIT=x3";; fp32) E="NBX_X3=0";; esac
    env $E timeout -k 10 300 python -u -m pytest -s -v --timeout 120 --timeout-method thread tests/test_gpu_segnn.py \
        -k "forward_matches_oracle or c2_full_batch" > $O/acc_$v.log 2>&1
    echo "$v: $(grep -c PASSED $O/acc_$v.log) passed, $(grep -c FAILED $O/acc_$v.log) failed"
    grep "\[cols\]" $O/acc_$v.log | tr '\n' ' '; echo
done
for i in 1 2; do
    timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_h2_$i.json 2> $O/bench_h2_$i.err || exit 1
done
NBX_SPLIT=x3 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_x3.json 2> $O/bench_x3.err || exit 1
NBX_TP_DEBUG=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/dbg_h2.json 2> $O/dbg_h2.err || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
for f in $O/bench_*.json; do echo "$f $(python -c "
import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], [round(v['avg_launch_us'],2) for v in d['roofline']['per_kind'].values()])")"; done
