#!/bin/bash
# Full measurement session: PMC passes (-> profiles/pmc_tp_kernels.json), then smoke, GPU
# tests, bench and the rocprofv3 kernel trace (scripts/gpu_check.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash scripts/pmc_passes.sh || exit $?
cp gpurun_out/pmc/summary.json profiles/pmc_tp_kernels.json
mkdir -p gpurun_out/profiles_new && cp gpurun_out/pmc/summary.json gpurun_out/profiles_new/pmc_tp_kernels.json
bash scripts/gpu_check.sh
