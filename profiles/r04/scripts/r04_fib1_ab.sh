#!/bin/bash
# PONITA fibre kernel A/B: one-pass (NBX_PO_FIB_ONEPASS=1, X1 read once, FK slices double-buffered
# through LDS-DMA) against the range-split kernel: the PONITA parity tests, C3 bench and HBM PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
O=gpurun_out/fib1
mkdir -p $O
step() { local name=$1 to=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 "$to" "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -20 $O/$name.log; exit 1; }; tail -n 1 $O/$name.log | cut -c1-200; }
export NBX_PO_FIB_ONEPASS=1
[ -n "${SKIP_TESTS:-}" ] || step tests 300 python -u -m pytest tests -m gpu -k ponita -x -q --timeout 120 --timeout-method thread
VARS=${FIB1_VARIANTS:-32768,512,4,512;32768,512,2,512;32768,1024,4,512;20480,512,4,512}
IFS=';' read -ra VLIST <<< "$VARS"
for v in "${VLIST[@]}"; do
  IFS=',' read -r a1 a2 a3 a4 <<< "$v"
  set -- $a1 $a2 $a3 $a4
  export NBX_PO_FK1_LDS=$1 NBX_PO_FIB1_BLOCKS=$2 NBX_PO_FIB1_W=$3 NBX_PO_FIB1_NT=${4:-512}
  step bench_${1}_${2}_${3}_$4 200 python bench.py --model ponita --steps 10 --warmup 2 --no-cpu-baseline
  python -c "
import json; l=[x for x in open('$O/bench_${1}_${2}_${3}_$4.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$1 $2 $3 $4', d['value'], {k[:30]: v.get('avg_launch_us', v.get('avg_group_us')) for k, v in d['roofline'].get('per_kind', {}).items()})"
done
if [ -z "${NO_BASELINE:-}" ]; then
  unset NBX_PO_FIB_ONEPASS
  step bench_rangesplit 200 python bench.py --model ponita --steps 10 --warmup 2 --no-cpu-baseline
  python -c "
import json; l=[x for x in open('$O/bench_rangesplit.log') if x.startswith('{')][-1]; d=json.loads(l)
print('range-split', d['value'], {k[:30]: v.get('avg_launch_us', v.get('avg_group_us')) for k, v in d['roofline'].get('per_kind', {}).items()})"
  export NBX_PO_FIB_ONEPASS=1
fi
export NBX_PO_FK1_LDS=${BEST_LDS:-32768} NBX_PO_FIB1_BLOCKS=${BEST_BLOCKS:-512} NBX_PO_FIB1_W=${BEST_W:-4}
for p in FETCH_SIZE WRITE_SIZE; do
  step pmc_$p 200 rocprofv3 --pmc $p --output-format csv -d $O/$p -o run -- python bench.py --model ponita --steps 4 --warmup 1 --no-cpu-baseline
done
step stats 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --model ponita --steps 4 --warmup 1 --no-cpu-baseline
python tools/pmc_report.py $O $O/pmc.json > /dev/null
python -c "
import json; d=json.load(open('$O/pmc.json'))['kernels']
for k, v in d.items():
    if 'fiber' in k: print(k[:60], v['hbm_bytes_per_launch'] / 1e6, 'MB')"
grep -h "fiber_ln" $O/stats/*kernel_stats.csv | cut -c1-200
