#!/usr/bin/env python
"""Per-kernel averages of every PMC counter collected by scripts/pmc_passes.sh.

    python tools/pmc_report.py gpurun_out/pmc out.json

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads (MI355X_MICROARCH.md,
HBM section); WRITE_SIZE is exact for 16-B/lane stores, approximate otherwise.
"""
import collections
import csv
import glob
import json
import os
import sys


def main(root, out):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in vals.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = int(2 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024)
        if d.get("SQ_WAVE_CYCLES"):
            w = d["SQ_WAVE_CYCLES"]
            d["frac_wait_any"] = d.get("SQ_WAIT_ANY", 0) / w
            d["frac_wait_inst"] = d.get("SQ_WAIT_INST_ANY", 0) / w
            d["frac_active"] = d.get("SQ_ACTIVE_INST_ANY", 0) / w
        res[k] = d
    json.dump({"note": "per-dispatch averages; hbm_bytes_per_launch = 2*FETCH_SIZE + WRITE_SIZE (KiB->B)",
               "kernels": res}, open(out, "w"), indent=1)
    for k, d in sorted(res.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        short = {c: (round(v, 3) if isinstance(v, float) else v) for c, v in d.items()}
        print(k[:90])
        print("   ", short)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
