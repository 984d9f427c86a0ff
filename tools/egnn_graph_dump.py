"""Diagnosis of the EGNN-MC training-step graph-replay race: capture the
training step of bench.py --model egnn_mc_train (small widths) into a torch.cuda.CUDAGraph with
debug mode on, dump the HIP graph (hipGraphDebugDotPrint through CUDAGraph.debug_dump) and report
the zeroing node's dependencies; then replay K steps and compare the loss sequence with K eager
steps.  Run once with NBX_ET_MEMSET=1 (hipMemsetAsync zeroing) and once without (kernel zeroing):

    NBX_ET_MEMSET=1 python tools/egnn_graph_dump.py gpurun_out/egnn_memset.dot
    python tools/egnn_graph_dump.py gpurun_out/egnn_kernel.dot
"""
import os
import re
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nbody_amd  # noqa: E402,F401
import nbody_amd.graph as G  # noqa: E402
from nbody_amd.egnn_mc import EGNNMultiChannel  # noqa: E402


def dump_graph(cg, path):
    """hipGraphDebugDotPrint of the captured hipGraph_t (CUDAGraph(keep_graph=True).raw_cuda_graph())."""
    import ctypes
    try:
        g = cg.raw_cuda_graph()
        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipGraphDebugDotPrint(ctypes.c_void_p(g), path.encode(), ctypes.c_uint(1 << 0 | 1 << 2 | 1 << 3))
        print(f"hipGraphDebugDotPrint -> {rc}")
    except Exception as e:   # diagnosis only
        print(f"graph dump unavailable: {e!r}")


def main(path):
    dev = torch.device("cuda:0")
    B, N, K, W = 64, 5, 12, 3
    rng = np.random.default_rng(5)

    class Gr:
        pass
    gr = Gr()
    gr.pos = torch.tensor(rng.standard_normal((B * N, 3)), dtype=torch.float32, device=dev)
    gr.vel = torch.tensor(rng.standard_normal((B * N, 3)) * 0.5, dtype=torch.float32, device=dev)
    gr.mass = torch.ones(B * N, 1, device=dev)
    gr.edge_index = G.fc_edge_index(B, N, dev)
    gr.nbx_system_size = N
    tgt = torch.tensor(rng.standard_normal((B * N, 6)) * 0.1, dtype=torch.float32, device=dev)

    def run(graph):
        torch.manual_seed(0)
        model = EGNNMultiChannel(node_input_dim=2, edge_attr_dim=4, hidden_node_dim=128, hidden_edge_dim=128,
                                 hidden_coord_dim=128, num_layers=6, target_names=("pos_dt", "vel"), norm_diff=True,
                                 tanh=True, device=dev)
        params = list(model.parameters())
        opt = torch.optim.AdamW(params, lr=1e-3, fused=True, capturable=graph)
        if graph:
            for grp in opt.param_groups:
                grp["lr"] = torch.tensor(1e-3, dtype=torch.float32, device=dev)

        def body():
            opt.zero_grad(set_to_none=True)
            loss = torch.nn.functional.mse_loss(model(gr), tgt)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(params, 1.0, foreach=True)
            opt.step()
            return loss
        losses = []
        if not graph:
            for _ in range(K):
                losses.append(float(body().detach()))
            return losses
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(W):
                losses.append(float(body().detach()))
        torch.cuda.current_stream().wait_stream(side)
        try:
            cg = torch.cuda.CUDAGraph(keep_graph=True)
        except TypeError:
            cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg):
            sl = body()
        dump_graph(cg, path)
        # back-to-back replays, no host synchronisation in between (the r02 symptom's setting): each
        # replay's loss is copied on the stream into its own slot
        hist = torch.empty(K - W, device=dev)
        for i in range(K - W):
            cg.replay()
            hist[i].copy_(sl.detach())
        torch.cuda.synchronize()
        return losses + hist.tolist(), cg

    eager = run(False)
    graphed, cg = run(True)
    print("eager  ", " ".join(f"{x:.9g}" for x in eager))
    print("graphed", " ".join(f"{x:.9g}" for x in graphed))
    print("max |diff| over the replays:", max(abs(a - b) for a, b in zip(eager, graphed)))
    if not os.path.exists(path):
        print("no graph dump written")
        return
    txt = open(path).read()
    nodes = dict(re.findall(r'"?(\w+)"?\s*\[[^\]]*label="([^"]*)', txt))
    print(f"graph dump: {path}, {len(nodes)} nodes")
    for name, lab in nodes.items():
        if "emset" in lab or "MEMSET" in lab or "egnn_zero" in lab or "egnn_train_bwd" in lab or "grad_reduce" in lab:
            preds = re.findall(r'"?(\w+)"?\s*->\s*"?%s"?' % name, txt)
            succ = re.findall(r'"?%s"?\s*->\s*"?(\w+)"?' % name, txt)
            print(f"node {name}: {lab[:120]!r}\n   preds {[nodes.get(p, p)[:60] for p in preds]}\n"
                  f"   succs {[nodes.get(q, q)[:60] for q in succ]}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/egnn_graph.dot")
