"""Per-launch shape / time table of the nbx_gemm_f32* launches of one eager training step (diagnostic for
DESIGN.md §6.6 / §10: where the EquiformerV2 training step's GEMM time goes).

    python scripts/gemm_shapes.py [--model eqv2_train|segnn_train|ponita_train] [--top 40]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="eqv2_train")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import bench
    import nbody_amd.segnn_train as ST
    log = []
    orig = {n: getattr(ST, n) for n in ("gemm", "gemm_batched", "gemm_grouped")}

    def wrap(name):
        f = orig[name]

        def g(*args, **kw):
            n0 = len(ST.gemm_timer) if ST.gemm_timer is not None else None
            out = f(*args, **kw)
            if n0 is not None and len(ST.gemm_timer) > n0:
                if name == "gemm":
                    dims = [(args[1], args[2], args[3], args[0])]
                else:
                    dims = [(p[1], p[2], p[3], p[0]) for p in args[0] if p[1] > 0 and p[2] > 0]
                log.append((name, dims, ST.gemm_timer[-1]))
            return out
        return g
    for n in orig:
        setattr(ST, n, wrap(n))
    # the training modules import the functions by name: patch their bindings too
    import nbody_amd.eqv2_train  # noqa: F401
    import nbody_amd.ponita_train  # noqa: F401
    for mod in list(sys.modules.values()):
        if mod is not ST and any(getattr(mod, n, None) is orig[n] for n in orig):
            for n in orig:
                if getattr(mod, n, None) is orig[n]:
                    setattr(mod, n, getattr(ST, n))
    sys.argv = ["bench.py", "--model", a.model, "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--eager"]
    bench.main()
    torch.cuda.synchronize()
    rows = []
    for name, dims, (e0, e1, fl) in log:
        rows.append((e0.elapsed_time(e1) * 1e3, name, dims, fl))
    tot = sum(r[0] for r in rows)
    print(f"# {len(rows)} GEMM launches, {tot:.1f} us total (first eager step; includes the one-time calibration "
          f"of the first step)")
    rows.sort(key=lambda r: -r[0])
    for us, name, dims, fl in rows[:a.top]:
        print(f"{us:8.1f} us  {fl / us / 1e6 if us else 0:7.2f} TF  {name:12s} " +
              " ".join(f"{m}x{n}x{k}/f{f}" for m, n, k, f in dims))


if __name__ == "__main__":
    main()
