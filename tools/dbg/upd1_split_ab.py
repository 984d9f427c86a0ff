"""A/B of the split update_layer_1 (NBX_UPD1_SPLIT=1, default) against the combined kernel (=0):
one C2 forward (train mode) and the C2 fixture rollout (tests/golden/segnn_c2_rollout.npz) per
variant, each in its own process (the switch is read once per process); prints the forward
difference between the variants and each variant's per-step rollout MSE against the fp64 oracle."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "gpurun_out")


def child(tag):
    sys.path.insert(0, ROOT)
    import torch
    import nbody_amd.segnn as S
    dev = torch.device("cuda:0")
    fx = np.load(os.path.join(ROOT, "tests", "golden", "segnn_c2_rollout.npz"))
    torch.manual_seed(0)
    model = S.SEGNN(hidden_features=192, num_layers=6).to(dev).train()
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=dev)
    loc0, vel0 = fx["loc0"], fx["vel0"]
    B, N = loc0.shape[:2]
    mass = np.ones((B, N, 1))
    from nbody_amd.graph import fc_edge_index

    class G:
        pass
    g = G()
    g.pos, g.vel, g.mass = t(loc0.reshape(-1, 3)), t(vel0.reshape(-1, 3)), t(mass.reshape(-1, 1))
    g.edge_index = fc_edge_index(B, N, dev)
    with torch.no_grad():
        out = model(g).cpu().numpy()
    model.load_state_dict(sd)
    T = fx["traj_loc"].shape[1]
    tp, tv = model.rollout(t(loc0), t(vel0), t(mass), T)
    np.savez(os.path.join(OUT, f"upd1_ab_{tag}.npz"), out=out, tp=tp.cpu().numpy(), tv=tv.cpu().numpy())


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child(sys.argv[1])
        sys.exit(0)
    os.makedirs(OUT, exist_ok=True)
    for v in ("1", "0"):
        env = dict(os.environ, NBX_UPD1_SPLIT=v)
        subprocess.run([sys.executable, __file__, v], env=env, check=True, timeout=300)
    a, b = (np.load(os.path.join(OUT, f"upd1_ab_{v}.npz")) for v in ("1", "0"))
    fx = np.load(os.path.join(ROOT, "tests", "golden", "segnn_c2_rollout.npz"))
    d = np.abs(a["out"] - b["out"]).max(0) / np.abs(b["out"]).max(0)
    print("C2 forward split vs combined: max |diff| / max |out| per column", d)
    rl = fx["traj_loc"].astype(np.float64)
    for k in range(1, rl.shape[1]):
        m = [float(((x["tp"][:, k] - rl[:, k]) ** 2).mean()) for x in (a, b)]
        ab = float(((a["tp"][:, k] - b["tp"][:, k]) ** 2).mean())
        print(f"step {k}: MSE vs fp64 oracle split {m[0]:.3e} combined {m[1]:.3e}; split vs combined {ab:.3e}")
