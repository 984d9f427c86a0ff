#!/bin/bash
# A/B of an environment switch on the training benches (same box, alternating):
#   AB_ENV="NBX_BIAS_COLSUM=1" [MODELS="segnn_train ponita_train"] [TESTS="tests/..."] [ROUNDS=2] bash scripts/ab_train_env.sh
# B runs with AB_ENV set, A without.  Optional GPU tests first.
set -o pipefail
out=gpurun_out/ab_train
mkdir -p $out
if [ -n "$TESTS" ]; then
  timeout -k 10 420 python -u -m pytest $TESTS -q -x --timeout 120 --timeout-method thread > $out/tests.log 2>&1 \
      || { tail -30 $out/tests.log; exit 1; }
  tail -2 $out/tests.log
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for m in ${MODELS:-segnn_train ponita_train eqv2_train egnn_mc_train}; do
    for v in A B; do
      if [ $v = A ]; then e=""; else e="$AB_ENV"; fi
      timeout -k 10 200 env $e python bench.py --model $m --no-cpu-baseline > $out/${m}_${v}$r.log 2>&1 \
          || { tail -20 $out/${m}_${v}$r.log; exit 1; }
      echo "$m $v$r: $(grep '^{' $out/${m}_${v}$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"])')"
    done
  done
done
