"""Diagnosis: PONITA's calibrating first forward on the fp16x2 and bf16x3 paths (one spawned child per
setting): the calibration factors and the conv output moments against the reference fixture."""
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def child(env, q):
    os.environ.update(env)
    try:
        import torch
        import test_ponita as TP
        g = np.load(os.path.join(ROOT, "tests", "golden", "ponita.npz"))
        dev = torch.device("cuda:0")
        m = TP.make().to(dev)
        raw = {k: v.detach().clone().cpu().numpy() for k, v in m.state_dict().items() if "kernel.weight" in k}
        mom = {}
        orig = m._callibrate
        def spy(moments, n):
            mom["m"] = moments.double().cpu().numpy().copy()
            mom["n"] = n
            return orig(moments, n)
        m._callibrate = spy
        with torch.no_grad():
            m(TP.gpu_graph(g["loc"], g["vel"], g["mass"], 4, 5, dev))
        sd = m.state_dict()
        fac = {k: float(np.median(sd[k].cpu().numpy() / raw[k])) for k in raw}
        ref = TP.ref_params(g, "f32")
        rfac = {k: float(np.median(ref[k] / raw[k])) for k in raw}
        q.put((fac, rfac, mom["m"].tolist(), mom["n"]))
    except Exception as e:
        import traceback
        q.put(repr(e) + traceback.format_exc())


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    envs = [dict(kv.split("=", 1) for kv in a.split(",")) if a else {} for a in sys.argv[1:]] or [{}, {"NBX_PO_SPLIT": "x3"}]
    for env in envs:
        q = ctx.Queue()
        p = ctx.Process(target=child, args=(env, q))
        p.start()
        r = q.get(timeout=300)
        p.join(timeout=60)
        print(env or "default", r if isinstance(r, str) else "", flush=True)
        if not isinstance(r, str):
            fac, rfac, mom, n = r
            for k in fac:
                print(f"  {k}: factor {fac[k]:.6f} reference {rfac[k]:.6f}")
            print("  moments (sum, sum sq) per layer [in, x1, x2]:", np.array(mom).reshape(-1, 3, 2).tolist(), "n", n)
