"""Timeline of a rocprofv3 --kernel-trace CSV: per-kernel busy time, inter-kernel gaps, and the
split of a window of dispatches into busy / idle.

    python tools/trace_gaps.py <kernel_trace.csv> [--last N] [--top K]

``--last N``: analyse the last N dispatches (e.g. the timed rollout at the end of a bench run).
Prints: wall span, Σ kernel time, Σ gaps, the gap distribution, the largest gaps with the kernels
on either side, and per-kernel-name totals inside the window."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = ("Start_Timestamp", "End_Timestamp")
    ev = sorted(((int(r[ks[0]]), int(r[ks[1]]), r["Kernel_Name"]) for r in rows), key=lambda e: e[0])
    if a.last:
        ev = ev[-a.last:]
    span = ev[-1][1] - ev[0][0]
    busy = sum(e[1] - e[0] for e in ev)
    gaps = [(ev[i + 1][0] - ev[i][1], i) for i in range(len(ev) - 1)]
    g = sorted(x for x, _ in gaps)
    print(f"dispatches {len(ev)}  span {span / 1e3:.1f} us  kernel {busy / 1e3:.1f} us  "
          f"gaps {sum(g) / 1e3:.1f} us ({100 * sum(g) / span:.1f} %)")
    if g:
        q = lambda p: g[min(len(g) - 1, int(p * len(g)))] / 1e3
        print(f"gap us: min {g[0] / 1e3:.2f} p10 {q(.1):.2f} median {q(.5):.2f} p90 {q(.9):.2f} max {g[-1] / 1e3:.2f}")
    print("largest gaps:")
    for x, i in sorted(gaps, reverse=True)[:a.top]:
        print(f"  {x / 1e3:8.2f} us after #{i} {ev[i][2][:70]}  ->  {ev[i + 1][2][:70]}")
    tot = collections.defaultdict(lambda: [0, 0])
    for s, e, n in ev:
        tot[n][0] += e - s
        tot[n][1] += 1
    print("per kernel in the window:")
    for n, (t, c) in sorted(tot.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"  {t / 1e3:9.1f} us {c:5d} x {t / c / 1e3:7.2f} us  {n[:100]}")


if __name__ == "__main__":
    main()
