#!/bin/bash
# A/B of the EquiformerV2 node-block kernel's weight-row batching (NBX_EQ_NB = 4 default, 1, 8) on the C4
# line, after the EquiformerV2 GPU tests; then its kernel summary.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/eqnode_ab
mkdir -p $out
timeout -k 10 420 python -u -m pytest tests/test_gpu_eqv2.py tests/test_gpu_eqv2_general.py tests/test_gpu_eqv2_train.py -q -x \
    --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for r in 1 2; do
  for nb in 4 1 8; do
    NBX_EQ_NB=$nb timeout -k 10 200 python bench.py --model eqv2 --no-cpu-baseline > $out/eqv2_nb${nb}_$r.log 2>&1 \
        || { tail -20 $out/eqv2_nb${nb}_$r.log; exit 1; }
    echo "eqv2 nb=$nb r$r: $(grep '^{' $out/eqv2_nb${nb}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"])')"
  done
done
bash scripts/profile_models.sh eqv2
