cd $GRAFT_REPO_ROOT
for v in 0 6 12 0 20; do
NBX_STAGGER=$v timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/b.json 2>gpurun_out/b.err || exit 1
python -c "
import json;d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]);print('$v', d['value'], [v['avg_launch_us'] for k,v in d['roofline']['per_kind'].items()])"; done
