#!/bin/bash
# Round-5 A/B: loader-wave image staging (NBX_LW=1) for the fp16x2 node TPs, on top of the XCD order.
set -o pipefail
O=gpurun_out/r05/lw
mkdir -p $O
NBX_LW=1 timeout -k 10 300 python -u -m pytest -s -v --timeout 120 --timeout-method thread tests/test_gpu_segnn.py \
    -k "forward_matches_oracle or c2_full_batch or rollout_c2_matches or deterministic" > $O/acc_lw.log 2>&1
echo "LW tests: $(grep -c PASSED $O/acc_lw.log) passed, $(grep -c FAILED $O/acc_lw.log) failed"; grep FAILED $O/acc_lw.log | head
grep -q "Fatal\|core dumped\|Segmentation\|HSA_STATUS" $O/acc_lw.log && { echo "GPU fault in LW tests"; exit 1; }
for i in 1 2; do
    NBX_LW=1 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_lw_$i.json 2> $O/bench_lw_$i.err || exit 1
    NBX_LW=0 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_nolw_$i.json 2> $O/bench_nolw_$i.err || exit 1
done
NBX_LW=1 NBX_TP_DEBUG=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/dbg_lw.json 2> $O/dbg_lw.err || exit 1
for f in $O/bench_*.json; do echo "$f $(python -c "
import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], [round(v['avg_launch_us'],2) for v in d['roofline']['per_kind'].values()])")"; done
grep "tp16" $O/dbg_lw.err | head -4
