#!/bin/bash
# Round-4 close at HEAD: the whole -m gpu suite, smoke, the default bench line (scripts/r04_final.sh without
# profiles), then the EquiformerV2 node-block batching A/B on the C4 line and its kernel summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
NO_PROFILE=1 bash scripts/r04_final.sh || exit 1
out=gpurun_out/eqnode_ab
mkdir -p $out
for r in 1 2; do
  for nb in 4 1 8; do
    NBX_EQ_NB=$nb timeout -k 10 200 python bench.py --model eqv2 --no-cpu-baseline > $out/eqv2_nb${nb}_$r.log 2>&1 \
        || { tail -20 $out/eqv2_nb${nb}_$r.log; exit 1; }
    echo "eqv2 nb=$nb r$r: $(grep '^{' $out/eqv2_nb${nb}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"])')"
  done
done
bash scripts/profile_models.sh eqv2
