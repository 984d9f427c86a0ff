#!/bin/bash
# scratch GPU step: staging probe + SEGNN bench + SEGNN GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
NBX_STAGE_PROBE=1 NBX_TP_DEBUG=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/dbg1.json 2> gpurun_out/dbg1.err || exit 1
grep "tp_debug" gpurun_out/dbg1.err | sed -n '60,63p'
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b1.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/b1.json'));print('segnn', d['value'], d['ms_per_step'], {k[:30]:v['avg_launch_us'] for k,v in d['roofline']['per_kind'].items()})"
timeout -k 10 300 python -m pytest tests/test_gpu_segnn.py tests/test_gpu_rollout.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; tail -3 gpurun_out/t.log
