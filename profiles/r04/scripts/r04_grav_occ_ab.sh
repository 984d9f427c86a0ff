#!/bin/bash
# A/B of the gravity integrator's register budget (default: <= 64 VGPRs, two 1024-thread workgroups per
# CU; NBX_GRAV_OCC=1: the compiler's allocation, one per CU): gravity GPU tests, then the C5 line alternating.
set -o pipefail
out=gpurun_out/grav_occ
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -q -x --timeout 120 --timeout-method thread \
    > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then e=""; else e="NBX_GRAV_OCC=1"; fi
    timeout -k 10 200 env $e python bench.py --model gravity --no-cpu-baseline > $out/gravity_${v}$r.log 2>&1 \
        || { tail -20 $out/gravity_${v}$r.log; exit 1; }
    echo "gravity $v$r: $(grep '^{' $out/gravity_${v}$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], d["roofline"]["frac"])')"
  done
done
