#!/bin/bash
# Round-4 A/B of the 32 x 32-tile training GEMM (NBX_GEMM_TILE32=0 keeps 64 x 64 everywhere):
# GEMM / training parity tests first, then each training bench with both settings.
set -o pipefail
out=gpurun_out/gemm32
mkdir -p $out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 420 python -u -m pytest tests/test_gpu_segnn_train.py tests/test_gpu_ponita_train.py \
      tests/test_gpu_eqv2_train.py tests/test_gpu_eqv2_general.py tests/test_gpu_eqv2.py \
      -q -x --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
  tail -3 $out/tests.log
fi
for m in ${MODELS:-segnn_train ponita_train eqv2_train egnn_mc_train}; do
  for t in 0 1; do
    NBX_GEMM_TILE32=$t timeout -k 10 200 python bench.py --model $m --no-cpu-baseline > $out/${m}_t$t.log 2>&1 \
        || { tail -20 $out/${m}_t$t.log; exit 1; }
    echo "$m tile32=$t: $(grep '^{' $out/${m}_t$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"])')"
  done
done
