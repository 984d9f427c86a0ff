#!/bin/bash
# r06 session: phase clocks of the C2 kernels, interleaved A/B of the update-layer variants, then the
# SEGNN parity / path / range / hand-off tests
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/r06/${1:-s2}
mkdir -p $O
NBX_TP_DEBUG=1 timeout -k 10 120 python -u scripts/tp_phase_clocks.py > $O/phase.log 2>&1 || { tail -5 $O/phase.log; exit 1; }
grep -A40 "forward 1" $O/phase.log | grep tp_debug | head -30
timeout -k 10 700 bash scripts/ab_multi.sh 2 "" "NBX_UPD1_V=1" "NBX_UPD1_V=2" "NBX_UPD2_V=1" "NBX_UPD2_V=2" "NBX_UPD2_V=3" "NBX_UPD2_V=4" > $O/ab.log 2>&1
rc=$?; cat $O/ab.log; [ $rc -ne 0 ] && exit $rc
bash scripts/segnn_parity_check.sh ${1:-s2}
