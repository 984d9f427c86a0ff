"""Diagnosis: accuracy of the register-formed dot operands (NBX_UPD_DV) against the materialised ones.

1. C2 rollouts (tests/golden/segnn_c2_rollout.npz, 10 steps) per path, REPS times, with the atomic
   BatchNorm sums (default) and with SEGNN(deterministic=True): per-step pos MSE vs the fp64 oracle.
2. One train-mode C2 forward (B = 1024) on two seeded batches per path vs the fp64 numpy oracle:
   rms and max error over each output column, relative to the column's rms.
usage: python scripts/dv_accuracy.py REPS "ENV=V" ...    ('' = defaults)"""
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def child(env, reps, q):
    os.environ.update(env)
    try:
        import torch
        import nbody_amd.segnn as S
        import test_gpu_segnn as T
        fx = np.load(os.path.join(ROOT, "tests", "golden", "segnn_c2_rollout.npz"))
        dev = torch.device("cuda:0")
        res = {}
        for det in (False, True):
            torch.manual_seed(0)
            model = S.SEGNN(hidden_features=192, num_layers=6, deterministic=det).to(dev).train()
            sd0 = {k: v.clone() for k, v in model.state_dict().items()}
            t = lambda a: torch.tensor(a, dtype=torch.float32, device=dev)
            Tn = fx["traj_loc"].shape[1]
            runs = []
            for _ in range(reps):
                model.load_state_dict(sd0)
                tp, _ = model.rollout(t(fx["loc0"]), t(fx["vel0"]), t(np.ones(fx["loc0"].shape[:2] + (1,))), Tn)
                runs.append(tp.double().cpu().numpy())
            res["roll_det" if det else "roll_atomic"] = runs
        model = T.make_model(192, 6, dev, perturb_bn=False).train()
        sd0 = {k: v.clone() for k, v in model.state_dict().items()}
        fw = []
        for seed in (3, 21):
            model.load_state_dict(sd0)
            pos, vel, mass = T.states(1024, 5, seed=seed)
            fw.append(T.gpu_forward(model, pos, vel, mass, 1024, 5, dev))
        res["fwd"] = fw
        q.put(res)
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put(repr(e) + traceback.format_exc())


if __name__ == "__main__":
    import torch
    import test_gpu_segnn as T
    reps = int(sys.argv[1])
    envs = [dict(kv.split("=", 1) for kv in a.split(",")) if a else {} for a in sys.argv[2:]] or [{}]
    fx = T.c2_fixture()
    rl = fx["traj_loc"].astype(np.float64)
    model = T.make_model(192, 6, torch.device("cpu"), perturb_bn=False).train()
    refs = []
    for seed in (3, 21):
        pos, vel, mass = T.states(1024, 5, seed=seed)
        refs.append(T.oracle_forward(model, T.params_of(model), pos, vel, mass, 1024, 5, True)[0])
    print("oracle forwards done", flush=True)
    ctx = mp.get_context("spawn")
    for env in envs:
        q = ctx.Queue()
        p = ctx.Process(target=child, args=(env, reps, q))
        p.start()
        r = q.get(timeout=900)
        p.join(timeout=60)
        tag = ",".join(f"{k}={v}" for k, v in env.items()) or "default"
        if isinstance(r, str):
            print(f"{tag}: FAILED {r}", flush=True)
            continue
        for kind in ("roll_atomic", "roll_det"):
            for i, tp in enumerate(r[kind]):
                mse = [((tp[:, k] - rl[:, k]) ** 2).mean() for k in range(1, tp.shape[1])]
                print(f"{tag} {kind} run {i}: pos MSE per step " + " ".join(f"{m:.1e}" for m in mse), flush=True)
        for i, (got, ref) in enumerate(zip(r["fwd"], refs)):
            e = got - ref
            rms = np.sqrt((ref ** 2).mean(0))
            print(f"{tag} forward {i}: rms err / col rms " + " ".join(f"{x:.2e}" for x in np.sqrt((e ** 2).mean(0)) / rms)
                  + " | max err / col rms " + " ".join(f"{x:.2e}" for x in np.abs(e).max(0) / rms), flush=True)
