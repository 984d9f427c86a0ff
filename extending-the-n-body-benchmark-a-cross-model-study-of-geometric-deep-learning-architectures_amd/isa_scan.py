"""Scan gfx950 assembly for MFMA operand write-after-read pairs (tools/hazard/mfma_war.hip):
a VMEM / LDS load (ds_read*, buffer_load*, global_load*) whose destination VGPRs overlap the
SrcA / SrcB of an MFMA issued fewer than `gap` wait states earlier (each instruction in
between = 1 state, s_nop N = N + 1).

Measured on MI355X (profiles/r02/mfma_war.txt): only SrcA of v_mfma_f32_16x16x32_bf16 is
unsafe, and only at 0 wait states (a load in the very next slot, when the MFMA queues behind
others); one state suffices, and SrcB of that shape as well as SrcA / SrcB of 32x32x16 bf16,
32x32x2 f32 and 16x16x4 f32 are safe at 0 states.  ROCm 7.2's hazard recognizer does not pad
it.  `rule=True` restricts the scan to that measured hazard (build.py runs it on every build
and fails on a hit); otherwise every pair within `gap` states is listed.

    python tools/hazard/scan_isa.py [--rule] <package>/lib/isa/*.s [--gap 4]

The scan is linear within each function (branch targets are not followed), which is exact
for the straight-line MFMA blocks of the TP kernels.
"""
from __future__ import annotations

import argparse
import re
import sys

REG = re.compile(r"^(v|a)(?:\[(\d+):(\d+)\]|(\d+))$")
LOAD = re.compile(r"^(ds_read\w*|ds_load\w*|buffer_load_(?!.*lds)\w*|global_load_(?!lds)\w*|flat_load\w*)$")
# the measured shape, and its fp16 twin (same pipeline; assumed to share the hazard, never measured safe)
HAZARD_MFMA = ("v_mfma_f32_16x16x32_bf16", "v_mfma_f32_16x16x32_f16")


def regs(tok):
    """'v[4:7]' -> ('v', 4, 7); 'v5' -> ('v', 5, 5); else None."""
    m = REG.match(tok.strip())
    if not m:
        return None
    if m.group(2) is not None:
        return m.group(1), int(m.group(2)), int(m.group(3))
    return m.group(1), int(m.group(4)), int(m.group(4))


def overlap(a, b):
    return bool(a and b and a[0] == b[0] and a[1] <= b[2] and b[1] <= a[2])


def scan(path, gap, rule=False):
    """-> [(path, function, line, load text, mfma line, mfma text, 'SrcA'|'SrcB', wait states)]"""
    found = []
    func = None
    hist = []     # recent instructions: (line no, mnemonic, operands)
    for no, line in enumerate(open(path), 1):
        s = line.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":") and not s.startswith("."):
            if not s.startswith(".LBB"):
                func, hist = s[:-1], []
            continue
        if s.startswith("."):
            continue
        parts = s.split(None, 1)
        mn = parts[0]
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        if LOAD.match(mn) and ops:
            dst = regs(ops[0])
            states = 0
            for pno, pmn, pops in reversed(hist):
                if states >= gap:
                    break
                if pmn.startswith("v_mfma") and len(pops) >= 3:
                    for which, tok in (("SrcA", pops[1]), ("SrcB", pops[2])):
                        if rule and (pmn not in HAZARD_MFMA or which != "SrcA"):
                            continue
                        if overlap(dst, regs(tok)):
                            found.append((path, func, no, s, pno, f"{pmn} {', '.join(pops)}", which, states))
                if pmn == "s_nop":
                    states += int(pops[0], 0) + 1 if pops else 1
                else:
                    states += 1
        hist.append((no, mn, ops))
        if len(hist) > 64:
            hist.pop(0)
    return found


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--gap", type=int, default=4, help="wait states to scan back")
    ap.add_argument("--rule", action="store_true", help="only the measured hazard: SrcA of 16x16x32 bf16, 0 states")
    a = ap.parse_args(argv)
    if a.rule:
        a.gap = 1
    total = 0
    for f in a.files:
        hits = scan(f, a.gap, a.rule)
        for path, func, no, load, pno, mfma, which, states in hits:
            print(f"{path}:{no} [{func}] {load}  <- overwrites {which} of line {pno}: {mfma}  ({states} wait states)")
        total += len(hits)
        mf = sum(1 for ln in open(f) if ln.strip().startswith("v_mfma"))
        print(f"{f}: {mf} MFMAs, {len(hits)} load(s) into a pending MFMA's SrcA/SrcB within {a.gap} wait states")
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
