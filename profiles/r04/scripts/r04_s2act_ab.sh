#!/bin/bash
# A/B of the compile-time alpha count in EquiformerV2's S2 activation kernel (NBX_EQV2_S2_NA0=1 = run-time
# count): EquiformerV2 GPU tests, then the C4 line alternating, then its kernel summary.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s2act_ab
mkdir -p $out
timeout -k 10 420 python -u -m pytest tests/test_gpu_eqv2.py tests/test_gpu_eqv2_general.py -q -x --timeout 120 \
    --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then e=""; else e="NBX_EQV2_S2_NA0=1"; fi
    timeout -k 10 200 env $e python bench.py --model eqv2 --no-cpu-baseline > $out/eqv2_${v}$r.log 2>&1 \
        || { tail -20 $out/eqv2_${v}$r.log; exit 1; }
    echo "eqv2 $v$r: $(grep '^{' $out/eqv2_${v}$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"])')"
  done
done
bash scripts/profile_models.sh eqv2
