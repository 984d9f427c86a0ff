cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_segnn.py -q -x -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
VAR=NBX_STATIC bash scripts/ab_msg.sh 0 1
