cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; tail -1 gpurun_out/t.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/t.log | head -5; exit $rc; }
NBX_TP_DEBUG=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dbg.json 2> gpurun_out/dbg.err || exit 1
grep "tp_debug msg_pre" gpurun_out/dbg.err | head -1
for k in 1 2; do timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/b.json 2>gpurun_out/b.err || exit 1
python -c "
import json;d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]);print(d['value'], [v['avg_launch_us'] for k,v in d['roofline']['per_kind'].items()])"; done
