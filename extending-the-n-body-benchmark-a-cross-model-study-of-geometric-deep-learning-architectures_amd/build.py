"""Build libnbx.so for gfx950 with hipcc (in-tree: <package>/lib/libnbx.so).

    python <package>/build.py [--jobs 8] [--verbose]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ISA_DIR = os.path.join(HERE, "lib", "isa")   # device assembly of every object (hazard check, inspection)
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "lib")
# NBX_BUILD_TAG: a side build (lib/libnbx_<tag>.so, loaded with NBX_LIB=...) for A/B timing only
_TAG = os.environ.get("NBX_BUILD_TAG", "")
OBJ_DIR = os.path.join(HERE, "lib", "obj" + (f"_{_TAG}" if _TAG else ""))
LIB = os.path.join(OUT_DIR, f"libnbx_{_TAG}.so" if _TAG else "libnbx.so")
ARCH = os.environ.get("NBX_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result",
         "-munsafe-fp-atomics", "-save-temps=obj"]
# per-file extra flags: the split-precision MFMA kernels' VALU work (operand splits, the message
# kernel's edge combination) runs beside MFMAs, where packed fp32 VALU costs extra cycles; with
# SLP vectorisation off these files run 1.8 % more steps/s (measured, C2).
# NBX_FILE_FLAGS="file.hip:-flag,-flag;..." adds more (A/B builds).
FILE_FLAGS = {"segnn.hip": ["-fno-slp-vectorize"], "msg_pre.hip": ["-fno-slp-vectorize"]}
for _item in filter(None, os.environ.get("NBX_FILE_FLAGS", "").split(";")):
    _f, _fl = _item.split(":", 1)
    FILE_FLAGS.setdefault(_f, []).extend(_fl.split(","))


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _needs(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(jobs: int = 8, verbose: bool = False, force: bool = False) -> str:
    os.makedirs(OBJ_DIR, exist_ok=True)
    hipcc = _hipcc()
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(HERE, "..", "include", "*.h"))
    objs, cmds = [], []
    for s in srcs:
        o = os.path.join(OBJ_DIR, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or _needs(o, [s] + headers):
            cmds.append([hipcc, *FLAGS, *FILE_FLAGS.get(os.path.basename(s), []), "-c", s, "-o", o])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r.stderr

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for err in ex.map(run, cmds):
            if verbose and err:
                print(err, file=sys.stderr)
    _keep_device_asm()
    if cmds or not os.path.exists(LIB) or _needs(LIB, objs):
        # librccl.so.1: csrc/comm.hip (under PyTorch the loader reuses torch's copy, same soname)
        run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs, "-L/opt/rocm/lib", "-lrccl"])
    check_isa()
    return LIB


def _keep_device_asm():
    """-save-temps=obj leaves every compilation stage next to the objects: keep the device
    assembly (lib/isa/*.s) and drop the rest."""
    os.makedirs(ISA_DIR, exist_ok=True)
    for f in os.listdir(OBJ_DIR):
        p = os.path.join(OBJ_DIR, f)
        if f.endswith(f"-{ARCH}.s") and "-hip-amdgcn-" in f:
            os.replace(p, os.path.join(ISA_DIR, f))
        elif not f.endswith(".o") or "-hip-amdgcn-" in f or "-host-" in f:
            os.remove(p)


def check_isa():
    """The gfx950 hazard ROCm 7.2 does not pad (DESIGN.md "gfx950 MFMA SrcA hazard"): a load
    issued right after a v_mfma_f32_16x16x32_bf16 (or its fp16 twin) into that MFMA's SrcA
    registers.  Any occurrence in the built kernels fails the build."""
    import glob as _g
    from importlib import import_module
    scan = import_module(__package__ + ".isa_scan" if __package__ else "isa_scan").scan
    hits = [h for f in sorted(_g.glob(os.path.join(ISA_DIR, "*.s"))) for h in scan(f, 1, rule=True)]
    if hits:
        msg = "\n".join(f"{os.path.basename(p)}:{no} [{fn}] {ld} <- SrcA of line {pno}: {mf}"
                        for p, fn, no, ld, pno, mf, _, _ in hits)
        raise RuntimeError("gfx950 MFMA SrcA hazard in the built kernels (a load into the SrcA registers of the "
                           "v_mfma_f32_16x16x32_bf16 / _f16 issued just before it):\n" + msg)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    print(build(a.jobs, a.verbose, a.force))
