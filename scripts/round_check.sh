#!/bin/bash
# Full measurement session: PMC passes (-> profiles/pmc_tp_kernels.json), then smoke, GPU
# tests, bench and the rocprofv3 kernel trace (scripts/gpu_check.sh); the files to commit
# under profiles/ are collected in gpurun_out/profiles_new/.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash scripts/pmc_passes.sh || exit $?
cp gpurun_out/pmc/summary.json profiles/pmc_tp_kernels.json
mkdir -p gpurun_out/profiles_new && cp gpurun_out/pmc/summary.json gpurun_out/profiles_new/pmc_tp_kernels.json
bash scripts/gpu_check.sh || exit $?
cp gpurun_out/prof/segnn_kernel_stats.csv gpurun_out/profiles_new/segnn_bench_kernel_stats.csv
tail -n 1 gpurun_out/bench.log > gpurun_out/profiles_new/bench_segnn_c2.json
python tools/kernel_summary.py gpurun_out/prof/segnn_kernel_stats.csv gpurun_out/pmc/summary.json \
    gpurun_out/profiles_new/segnn_kernel_summary.md "python bench.py --steps 20 --warmup 2 --no-cpu-baseline"
