#!/bin/bash
# A/B of the XCD-grouped block order of the gathering lin_kernel epilogues (NBX_LIN_XCD=0 = plain order):
# PONITA / EquiformerV2 GPU tests, C3 and C4 bench lines alternating, then FETCH_SIZE / WRITE_SIZE
# passes of the C3 line with each order.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/lin_xcd
mkdir -p $out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 420 python -u -m pytest tests/test_ponita.py tests/test_gpu_eqv2.py -m gpu -q -x --timeout 120 \
      --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
  tail -2 $out/tests.log
fi
for r in 1 2; do
  for m in ponita eqv2; do
    for v in A B; do
      if [ $v = A ]; then e=""; else e="NBX_LIN_XCD=0"; fi
      timeout -k 10 200 env $e python bench.py --model $m --no-cpu-baseline > $out/${m}_${v}$r.log 2>&1 \
          || { tail -20 $out/${m}_${v}$r.log; exit 1; }
      echo "$m $v$r: $(grep '^{' $out/${m}_${v}$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"])')"
    done
  done
done
for v in A B; do
  if [ $v = A ]; then e=""; else e="NBX_LIN_XCD=0"; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 env $e rocprofv3 --pmc $c --output-format csv -d $out/pmc_${v}_$c -o run \
        -- python bench.py --model ponita --steps 2 --warmup 1 --no-cpu-baseline > $out/pmc_${v}_$c.log 2>&1 \
        || { tail -5 $out/pmc_${v}_$c.log; exit 1; }
  done
done
echo done
