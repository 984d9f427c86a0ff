#!/bin/bash
# A/B of an environment switch on the C2 bench, alternating runs in one box session:
#   bash scripts/ab_env.sh "NBX_MP_XCD=0" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/ab
ENVB="$1"; R="${2:-3}"
for i in $(seq 1 $R); do
  for v in A B; do
    if [ $v = A ]; then e=""; else e="$ENVB"; fi
    timeout -k 10 120 env $e python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/ab/$v$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab/$v$i.json'));k=d['roofline']['per_kind'];print('$v', d['value'], [round(x['avg_launch_us'],2) for x in k.values()])"
  done
done
