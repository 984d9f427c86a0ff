#!/bin/bash
# Round-5 A/B of the current build: SEGNN + rollout GPU tests, then the C2 bench with the default
# settings and with each listed environment setting, interleaved, two rounds.
# usage: bash scripts/r05_ab.sh <tag> "NBX_X=0" ["NBX_Y=1 NBX_LIB=<pkg>/lib/libnbx_<build tag>.so" ...]
set -o pipefail
O=gpurun_out/r05/${1:-ab}
shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_segnn.py tests/test_gpu_rollout.py \
    > $O/tests.log 2>&1
echo "tests: $(grep -c PASSED $O/tests.log) passed, $(grep -c FAILED $O/tests.log) failed"; grep FAILED $O/tests.log | head
grep -q "core dumped\|Segmentation fault\|HSA_STATUS_ERROR\|Memory access fault" $O/tests.log && { echo "GPU fault"; exit 1; }
for r in 1 2; do
  for v in "" "$@"; do
    tag=${v:-base}; tag=$(echo "$tag" | sed "s#[^ ]*/lib/libnbx_##; s#\.so##" | tr -c "A-Za-z0-9_\n" "_")
    env $v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_${tag}_$r.json 2> $O/bench_${tag}_$r.err || exit 1
  done
done
NBX_TP_DEBUG=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/dbg.json 2> $O/dbg.err || exit 1
for f in $O/bench_*.json; do echo "$f $(python -c "
import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], [round(v['avg_launch_us'],2) for v in d['roofline']['per_kind'].values()])")"; done
grep "tp_debug" $O/dbg.err | head -5
