"""Microbenchmark of nbx_gemm_f32_grouped on the training steps' launch shapes (scripts/gemm_shapes.py
census): each group of problems launched REPS times back to back on one stream, event-timed; prints
us per launch (GEMM kernel + split-K reduce).  NBX_LIB selects a side build for A/B.

    python scripts/gemm_micro.py [--reps 200]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (flags, M, N, K) per problem; flags as in the census (1 TRANS_A, 2 TRANS_B, 4 B_ONES, 8 ONES_TAIL)
GROUPS = {
    "eqv2_bwd_ffn": [(13, 288, 385, 1280), (0, 1280, 384, 288), (1, 256, 512, 1280), (0, 1280, 512, 256)],
    "eqv2_fwd_so2": [(2, 1280, 96, 384), (2, 1280, 192, 384), (2, 1280, 256, 512)],
    "eqv2_bwd_rad": [(13, 640, 65, 1280), (0, 1280, 64, 640)],
    "eqv2_bwd_1152": [(13, 64, 1153, 1280), (0, 1280, 1152, 64)],
    "eqv2_fwd_1152": [(2, 1280, 64, 1152)],
    "eqv2_so3lin": [(0, 320, 64, 64), (0, 960, 64, 64), (0, 1600, 64, 64), (1, 64, 64, 320), (1, 64, 64, 960),
                    (1, 64, 64, 1600), (5, 64, 1, 320)],
    "segnn_bwd": [(13, 288, 387, 1280), (1, 96, 192, 3840), (0, 1280, 386, 288), (0, 3840, 192, 96)],
    "segnn_fwd": [(2, 1280, 288, 386), (2, 3840, 96, 192)],
    # EquiformerV2 lmax 6 forward (N = 20, B = 64: 24 320 edges): SO(2) conv 1 / conv 2, radial output
    "l6_conv1": [(2, 24320, 96, 896), (2, 24320, 448, 896), (2, 24320, 768, 1536), (2, 24320, 640, 1280)],
    "l6_conv2": [(2, 24320, 112, 448), (2, 24320, 192, 768), (2, 24320, 160, 640)],
    "l6_rad1152": [(2, 24320, 64, 1152)],
    "l6_rad2304": [(2, 24320, 2304, 64)],
    "l6_rad448": [(2, 24320, 448, 64)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--only", help="comma-separated group names")
    ap.add_argument("--check", action="store_true", help="compare each problem with torch fp64")
    ap.add_argument("--dump", help="save every C to this .npz (bit-identity checks between builds / modes)")
    a = ap.parse_args()
    import ctypes
    import nbody_amd._lib as L
    from nbody_amd.segnn_train import gemm_grouped, _at
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    dump = {}
    for name, probs in GROUPS.items():
        if a.only and name not in a.only.split(","):
            continue
        ps, ref = [], []
        for fl, M, N, K in probs:
            ta, tb, ones, tail = fl & 1, fl & 2, fl & 4, fl & 8
            Nb = N - (1 if ones else 0)
            A = torch.randn((K, M) if ta else (M, K), generator=g).to(dev)
            B = torch.randn((Nb, K) if tb else (K, Nb), generator=g).to(dev) if Nb else torch.zeros(1, device=dev)
            C = torch.empty(M * N, device=dev)
            ldc = N - (1 if tail else 0)
            ps.append((fl, M, N, K, _at(A, 0), M if ta else K, _at(B, 0), K if tb else Nb, _at(C, 0), ldc, 0.0,
                       1, 0, 0, 0))
            ref.append((A, B, C, fl, M, N))
        for _ in range(3):
            gemm_grouped(ps, dev)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            gemm_grouped(ps, dev)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        fl = sum(2.0 * M * N * K for _, M, N, K in probs)
        err = ""
        if a.check:
            worst = 0.0
            for A, B, C, f, M, N in ref:
                opA = A.double().t() if f & 1 else A.double()
                opB = B.double().t() if f & 2 else B.double()
                if f & 4 and N == 1:
                    opB = torch.ones(opA.shape[1], 1, dtype=torch.float64, device=dev)
                elif f & 4:
                    opB = torch.cat([opB, torch.ones(opB.shape[0], 1, dtype=torch.float64, device=dev)], 1)
                want = opA @ opB
                if f & 8:
                    got = torch.cat([C[:M * (N - 1)].view(M, N - 1), C[M * (N - 1):].view(M, 1)], 1)
                else:
                    got = C.view(M, N)
                worst = max(worst, ((got.double() - want).abs().max() / want.abs().max()).item())
            err = f"  max rel err {worst:.2e}"
        print(f"{name:16s} {us:8.2f} us/launch  {fl / us / 1e6:7.2f} TFLOP/s{err}", flush=True)
        for j, (_, _, C, _, _, _) in enumerate(ref):
            dump[f"{name}_{j}"] = C.cpu().numpy()
    if a.dump:
        import numpy as np
        np.savez(a.dump, **dump)
    del ctypes, L


if __name__ == "__main__":
    main()
