#!/bin/bash
# r06: PONITA (C3) and EquiformerV2 (C4) on fp16x2: the reference-fixture tests, the split switches, C3 / C4
# bench A/B against bf16x3; then the SEGNN parity / path / range / hand-off tests
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/r06/${1:-s3}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_ponita.py tests/test_gpu_eqv2.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -s -p no:cacheprovider > $O/family_tests.log 2>&1
rc=$?; grep -E "passed|failed|cols|Error" $O/family_tests.log | tail -25; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for m in ponita eqv2; do
    for e in "" "NBX_PO_SPLIT=x3 NBX_EQ_SPLIT=x3"; do
      t=${m}_$([ -z "$e" ] && echo h2 || echo x3)_$i
      timeout -k 10 300 env $e python bench.py --model $m --no-cpu-baseline > $O/$t.json 2> $O/$t.err || { tail -5 $O/$t.err; exit 1; }
      python -c "import json;d=json.loads(open('$O/$t.json').read().strip().splitlines()[-1]);print('$t', d['value'], d['ms_per_step'])"
    done
  done
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_switches.py -k "PO_ or EQ_" -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/switch_tests.log 2>&1
rc=$?; tail -3 $O/switch_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/segnn_parity_check.sh ${1:-s3}
