#!/bin/bash
# Round-5 check of the current HEAD build: SEGNN GPU tests, two bench runs, phase clocks.
# usage: bash scripts/r05_step.sh <tag>
set -o pipefail
O=gpurun_out/r05/${1:-step}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_segnn.py tests/test_gpu_rollout.py \
    > $O/tests.log 2>&1
echo "tests: $(grep -c PASSED $O/tests.log) passed, $(grep -c FAILED $O/tests.log) failed"; grep FAILED $O/tests.log | head
grep -q "core dumped\|Segmentation fault\|HSA_STATUS_ERROR\|Memory access fault" $O/tests.log && { echo "GPU fault"; exit 1; }
for i in 1 2; do
    timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
done
NBX_TP_DEBUG=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/dbg.json 2> $O/dbg.err || exit 1
for f in $O/bench_*.json; do echo "$f $(python -c "
import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], [round(v['avg_launch_us'],2) for v in d['roofline']['per_kind'].values()])")"; done
grep "tp_debug" $O/dbg.err | head -5
