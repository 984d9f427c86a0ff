#!/usr/bin/env python
"""Summarise rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE: separate passes, as
MI355X_MICROARCH.md prescribes) into per-launch HBM bytes per kernel.

    python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/pmc_tp_kernels.json

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  On gfx950 FETCH_SIZE reports half
the bytes of a wide (16 B/lane) coalesced streaming read, which is how the fused
kernels read A and B, so the read side is doubled; WRITE_SIZE is taken as is
(4-B-per-lane stores are uncalibrated: treat the write side as approximate).
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def main(fetch_dir, write_dir, out):
    fe, wr = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fe) | set(wr)):
        if "tp16_kernel" not in k and "tp_fused_kernel" not in k and "msg1" not in k:
            continue
        f = sum(fe.get(k, [0])) / max(len(fe.get(k, [])), 1)
        w = sum(wr.get(k, [0])) / max(len(wr.get(k, [])), 1)
        res[k] = {"dispatches": len(fe.get(k, [])), "fetch_kib": round(f, 1), "write_kib": round(w, 1),
                  "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024)}
    json.dump({"note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, per dispatch",
               "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(k[:70], v)


if __name__ == "__main__":
    main(*sys.argv[1:4])
