cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; tail -1 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/b.json 2>gpurun_out/b.err || exit 1
python -c "
import json;d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]);print(d['value'], [v['avg_launch_us'] for k,v in d['roofline']['per_kind'].items()], d['roofline']['traffic'])"
