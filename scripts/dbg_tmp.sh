cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; tail -1 gpurun_out/t.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/t.log | head -5; exit $rc; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o s -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/p2.log 2>&1 || exit 1
python - <<'PY'
import csv,glob
f=(glob.glob('gpurun_out/prof2/**/s_kernel_stats.csv',recursive=True)+glob.glob('gpurun_out/prof2/s_kernel_stats.csv'))[0]
for r in csv.DictReader(open(f)):
    if 'featurize' in r['Name'] or 'nbx::' in r['Name'] or 'pp' in r['Name'][:40] or 'bn_' in r['Name']: print(f"{float(r['AverageNs'])/1e3:7.2f} {r['Calls']:>5} {r['Name'][:80]}")
PY
