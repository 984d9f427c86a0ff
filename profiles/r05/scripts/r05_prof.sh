#!/bin/bash
# Round-5 profiles of the C2 line at HEAD: rocprofv3 stats + FETCH/WRITE (profile_models.sh), then the
# SQ / L2 / LDS counter passes (pmc_passes.sh).
set -o pipefail
bash scripts/profile_models.sh segnn || exit 1
bash scripts/pmc_passes.sh --steps 3 --warmup 1 --no-cpu-baseline || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/pmc/summary.json"))["kernels"]
for k, v in sorted(d.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:8]:
    hit = v.get("TCC_HIT_sum", 0); miss = v.get("TCC_MISS_sum", 0)
    print(k[:70], "L2 hit %.3f" % (hit / max(hit + miss, 1)), "wait_any %.2f wait_inst %.2f active %.2f" %
          (v.get("frac_wait_any", 0), v.get("frac_wait_inst", 0), v.get("frac_active", 0)),
          "mfma_busy", v.get("SQ_VALU_MFMA_BUSY_CYCLES"), "busy", v.get("SQ_BUSY_CYCLES"))
PY
