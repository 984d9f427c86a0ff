cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_segnn.py -q -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; grep -E "passed|failed|FAILED|max err" gpurun_out/t.log | head -30; [ $rc -ne 0 ] && exit $rc
for m in ponita egnn_mc gravity; do
  timeout -k 10 300 python bench.py --model $m --no-cpu-baseline > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err; rc=$?
  echo "$m rc=$rc"; tail -c 600 gpurun_out/bench_$m.json; echo
  [ $rc -ne 0 ] && exit $rc
done
