#!/bin/bash
# A/B of library builds (lib/libnbx_<tag>.so side builds, "main" = lib/libnbx.so): SEGNN GPU tests
# with the main build, then interleaved C2 benches per build, then a kernel trace of the main build.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/ab
LIBDIR=$(ls -d extending-*/lib)
timeout -k 10 300 python -u -m pytest tests/test_gpu_segnn.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
rc=$?; tail -1 gpurun_out/ab/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for t in "$@"; do
    if [ "$t" = main ]; then L=$PWD/$LIBDIR/libnbx.so; else L=$PWD/$LIBDIR/libnbx_$t.so; fi
    NBX_LIB=$L timeout -k 10 120 python bench.py --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/ab/$t.json 2> gpurun_out/ab/$t.err
    rc=$?; [ $rc -ne 0 ] && { echo "$t rc=$rc"; tail -3 gpurun_out/ab/$t.err; exit $rc; }
    python -c "
import json;d=json.loads(open('gpurun_out/ab/$t.json').read().strip().splitlines()[-1]);print('$t', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/prof -o segnn -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/ab/prof.log 2>&1 || exit $?
f=$(find gpurun_out/ab/prof -name '*kernel_stats.csv' | head -1); python -c "
import csv
for r in csv.DictReader(open('$f')):
    print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,2))" | head -12
