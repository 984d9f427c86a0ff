cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_segnn.py tests/test_gpu_native.py tests/test_boundary.py -q -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; grep -E "passed|failed|FAILED|max err" gpurun_out/t.log | head -30; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_msg.sh 8x3
