timeout -k 5 60 ./tools/hazard/mfma_war > gpurun_out/mfma_war.txt 2>&1
cat gpurun_out/mfma_war.txt
timeout -k 10 400 python -u -m pytest tests/test_ponita.py tests/test_gpu_segnn.py::test_rollout_c2_matches_oracle_fixture -m gpu -v -s -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/t4.log 2>&1
grep -E "C2 |passed|failed|Error|PASS|FAIL" gpurun_out/t4.log | tail -30
for v in "" "NBX_PO_X3=0"; do timeout -k 10 200 env $v python bench.py --model ponita --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/po_$v.json 2>gpurun_out/po_err.txt || { tail -5 gpurun_out/po_err.txt; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/po_$v.json'));print('$v', d['value'], {k[:20]:v['avg_launch_us'] for k,v in d['roofline']['per_kind'].items()})"; done
