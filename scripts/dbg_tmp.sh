cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_segnn.py -q -x -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
NBX_TP_DEBUG=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dbg.json 2> gpurun_out/dbg0.err || exit 1
grep tp_debug gpurun_out/dbg0.err | sed 's/span=[0-9]* //' | awk '{print $2,$3,$4,$5,$6,$7,$8, $9}' | sort | awk '{k=$1" "$2; if(!(k in seen)){seen[k]=1; print}}'
bash scripts/ab_msg.sh 8x2 8x3
