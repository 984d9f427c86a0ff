#!/usr/bin/env python
"""Markdown table of a rocprofv3 --stats kernel summary, joined with the PMC HBM bytes per launch.

    python tools/kernel_summary.py <kernel_stats.csv> <pmc summary.json> <out.md> "<command line>"
"""
import csv
import json
import sys


def main(stats, pmc, out, cmd):
    rows = list(csv.DictReader(open(stats)))
    kern = json.load(open(pmc)).get("kernels", {}) if pmc else {}
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# rocprofv3 --kernel-trace --stats --output-format csv -- {cmd}",
             "# MI355X gfx950, ROCm 7.2; HBM bytes per launch from separate FETCH_SIZE / WRITE_SIZE passes",
             "# (scripts/pmc_passes.sh): 2 x FETCH_SIZE + WRITE_SIZE", "",
             "| kernel | calls | avg us | total % | HBM MB/launch |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:20]:
        name = r["Name"]
        hbm = kern.get(name, {}).get("hbm_bytes_per_launch")
        hbm_s = f"{hbm / 1e6:.1f}" if hbm else "-"
        lines.append(f"| `{name[:110]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                     f"{100 * float(r['TotalDurationNs']) / total:.2f} | {hbm_s} |")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:5])
