"""Where each SEGNN kernel path's C2 rollout falls in the ensemble of equally valid fp32 computations
(tests/golden/make_segnn_c2_ensemble.py), one spawned child per path setting (the library reads its
switches once per process).  Prints, per path and step, the envelope checks of
tests/test_gpu_segnn.py::test_rollout_c2_matches_oracle_fixture and a one-line verdict.

usage: python scripts/rollout_paths.py ["ENV=V,ENV2=V" ...]    ('' = defaults)"""
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
        import nbody_amd.segnn as S
        import test_gpu_segnn as TG
        torch.manual_seed(0)
        dev = torch.device("cuda:0")
        model = S.SEGNN(hidden_features=192, num_layers=6).to(dev).train()
        samples, _ = TG.c2_device_samples(model, TG.c2_fixture(), TG.c2_ensemble(), dev)
        q.put(samples)
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put(repr(e) + traceback.format_exc())


if __name__ == "__main__":
    import test_gpu_segnn as TG
    envs = [dict(kv.split("=", 1) for kv in a.split(",")) if a else {} for a in sys.argv[1:]] or [{}]
    ens = TG.c2_ensemble()
    ctx = mp.get_context("spawn")
    for env in envs:
        q = ctx.Queue()
        p = ctx.Process(target=child, args=(env, q))
        p.start()
        r = q.get(timeout=600)
        p.join(timeout=60)
        tag = ",".join(f"{k}={v}" for k, v in env.items()) or "default"
        if isinstance(r, str):
            print(f"{tag}: FAILED {r}", flush=True)
            continue
        for i, smp in enumerate(r):   # each sample alone: where single draws land
            single = TG.c2_rollout_envelope_check(smp[None], ens, label=f"{tag} sample {i}", q=1.0)
            print(f"-- {tag} sample {i}: {'inside' if not single else f'{len(single)} checks outside'}", flush=True)
        bad = TG.c2_rollout_envelope_check(r, ens, label=tag)
        print(f"== {tag}: {'inside the ensemble at every step' if not bad else bad}", flush=True)
