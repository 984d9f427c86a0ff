"""Every non-SEGNN environment switch of the library against the default path.

The library reads each switch once per process, so every setting runs in a spawned child of its
own, which computes the outputs of the model families the switch touches on seeded inputs; the
parent compares them with a child run on the defaults.  The default path itself is pinned to the
reference fixtures and oracles by the family tests (test_ponita.py, test_egnn_mc.py,
test_gpu_eqv2*.py, test_gpu_native.py), so agreement here puts each alternative on that footing.
Tolerances: the families' own fp32 tolerances (PONITA / EGNN-MC per column 3e-5 / 1e-5 of the
column scale, EquiformerV2 2e-5 abs + 2e-5 rel, gradients per tensor 2e-4 of the tensor scale);
switches that only change scheduling, block shapes or diagnostics must agree to the same bounds,
the gravity integrator's register allocation bit for bit."""
import multiprocessing as mp
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)

# setting -> families it touches
SWITCHES = [
    ({"NBX_PO_X3": "0"}, ["ponita"]),
    ({"NBX_PO_SPLIT": "x3"}, ["ponita"]),
    ({"NBX_PO_BASIS1": "0"}, ["ponita"]),
    ({"NBX_PO_BASIS_FUSED": "0"}, ["ponita"]),
    ({"NBX_PO_FIB_ONEPASS": "0"}, ["ponita"]),
    ({"NBX_PO_FIB_ONEPASS": "0", "NBX_PO_FIB1_NT": "256", "NBX_PO_FIB1_W": "2", "NBX_PO_FIB1_BLOCKS": "256",
      "NBX_PO_FK1_LDS": "16384"}, ["ponita"]),
    ({"NBX_PO_FIB_BLOCKS": "256", "NBX_PO_FK_LDS": "32768"}, ["ponita"]),
    ({"NBX_LIN_XCD": "0"}, ["ponita"]),
    ({"NBX_PO_FFN_DEBUG": "1"}, ["ponita"]),
    ({"NBX_EGNN_PERSIST": "0"}, ["egnn"]),
    ({"NBX_ET_MEMSET": "1"}, ["egnn_grad"]),
    ({"NBX_ET_DEBUG": "1"}, ["egnn_grad"]),
    ({"NBX_EQ_NPW": "1"}, ["eqv2"]),
    ({"NBX_EQ_SPLIT": "x3"}, ["eqv2"]),
    ({"NBX_EQ_RAD2": "1"}, ["eqv2"]),
    ({"NBX_EQ_NB": "4"}, ["eqv2"]),
    ({"NBX_EQV2_S2_NA0": "1"}, ["eqv2"]),
    ({"NBX_EQV2_SPECIALISED": "1"}, ["eqv2_grad"]),
    ({"NBX_GEMM_X3": "0"}, ["eqv2_l6"]),
    ({"NBX_GRAV_OCC": "1"}, ["gravity"]),
    ({"NBX_TP_DEBUG": "1"}, ["segnn"]),
]
FAMILIES = ["ponita", "egnn", "egnn_grad", "eqv2", "eqv2_l6", "eqv2_grad", "gravity", "segnn"]


class _Graph:
    pass


def _ponita(torch, dev):
    import test_ponita as TP
    m = TP.make(128, 2, num_ori=20).to(dev).eval()
    rng = np.random.default_rng(1)
    B, N = 32, 5
    pos, vel = rng.standard_normal((B * N, 3)), rng.standard_normal((B * N, 3))
    mass = rng.uniform(0.5, 1.5, (B * N, 1))
    with torch.no_grad():
        return {"out": m(TP.gpu_graph(pos, vel, mass, B, N, dev)).double().cpu().numpy()}


def _egnn_graph(torch, dev, B, N, seed):
    import nbody_amd.graph as G
    rng = np.random.default_rng(seed)
    gr = _Graph()
    gr.pos = torch.tensor(rng.standard_normal((B * N, 3)), dtype=torch.float32, device=dev)
    gr.vel = torch.tensor(rng.standard_normal((B * N, 3)), dtype=torch.float32, device=dev)
    gr.mass = torch.ones(B * N, 1, device=dev)
    gr.edge_index = G.fc_edge_index(B, N, dev)
    return gr


def _egnn(torch, dev):
    import test_egnn_mc as TE
    m = TE.make(128, 6, torch.float32).to(dev)
    with torch.no_grad():
        return {"out": m(_egnn_graph(torch, dev, 64, 5, 1)).double().cpu().numpy()}


def _egnn_grad(torch, dev):
    import test_egnn_mc as TE
    m = TE.make(64, 2, torch.float32).to(dev)
    gr = _egnn_graph(torch, dev, 8, 5, 2)
    pred = m(gr)
    G = torch.tensor(np.random.default_rng(3).standard_normal(tuple(pred.shape)), dtype=torch.float32, device=dev)
    (pred * G).sum().backward()
    res = {"pred": pred.detach().double().cpu().numpy()}
    res.update({"g/" + k: p.grad.double().cpu().numpy() for k, p in m.named_parameters()})
    return res


def _eqv2(torch, dev):
    import test_gpu_eqv2 as TQ
    rng = np.random.default_rng(7)
    B, N = 8, 20
    loc = rng.standard_normal((B, N, 3)) * 1.5
    vel = rng.standard_normal((B, N, 3)) * 0.3
    mass = np.ones((B, N, 1))
    gauge = rng.uniform(0, 1, (B * N * (N - 1), 3)).astype(np.float32)
    return {"out": TQ.run(TQ.make_model("c4", dev), loc, vel, mass, gauge, dev)}


def _eqv2_l6(torch, dev):
    """The lmax 6 / mmax 2 bench model (bench.py eqv2_l6) at B = 64, N = 20: its SO(2) convolution
    GEMMs (24 320 edge rows) run on the bf16x3 kernel by default, on fp32 MFMA under NBX_GEMM_X3=0."""
    import bench
    from nbody_amd.equiformer_v2 import EquiformerV2_nbody
    torch.manual_seed(0)
    m = EquiformerV2_nbody(**dict(bench.EQV2_C4, lmax_list=[6], mmax_list=[2])).to(dev).eval()
    t = lambda x: torch.tensor(x, dtype=torch.float32, device=dev)
    loc, vel, mass = bench.initial_states(64, 20, 0)
    tp, tv = m.rollout(t(loc), t(vel), t(mass), 3, seed=1)
    return {"pos": tp.double().cpu().numpy(), "vel": tv.double().cpu().numpy()}


def _eqv2_grad(torch, dev):
    import test_gpu_eqv2_train as TT
    m = TT._model(TT.SMALL, dev)
    loc, vel, mass, gauge, tgt = TT._inputs(3, 5, seed=35)
    loss, pred, grads = TT._train_step(m, loc, vel, mass, gauge, tgt, dev)
    res = {"pred": pred}
    res.update({"g/" + k: v for k, v in grads.items()})
    return res


def _gravity(torch, dev):
    from nbody_amd.gravity import GravitySim
    sim = GravitySim(n_balls=100, interaction_strength=2, dt=0.01, softening=0.2, device=dev)
    ics = [sim.initial_conditions(200 + s) for s in range(12)]
    pos = np.stack([c[0] for c in ics]); vel = np.stack([c[1] for c in ics]); mass = np.stack([c[2] for c in ics])
    ps, vs, fs = (t.cpu().numpy() for t in sim.sample_trajectories(pos, vel, mass, T=40, sample_freq=10))
    return {"pos": ps, "vel": vs, "force": fs}


def _segnn(torch, dev):
    import test_gpu_segnn as TS
    m = TS.make_model(192, 6, dev, perturb_bn=False).eval()
    pos, vel, mass = TS.states(64, 5, seed=12)
    return {"out": TS.gpu_forward(m, pos, vel, mass, 64, 5, dev)}


def _child(env, fams, q):
    os.environ.update(env)
    sys.path.insert(0, ROOT)
    try:
        import torch
        dev = torch.device("cuda:0")
        fn = {"ponita": _ponita, "egnn": _egnn, "egnn_grad": _egnn_grad, "eqv2": _eqv2, "eqv2_l6": _eqv2_l6,
              "eqv2_grad": _eqv2_grad, "gravity": _gravity, "segnn": _segnn}
        q.put({f: fn[f](torch, dev) for f in fams})
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put(repr(e) + traceback.format_exc())


def _run(env, fams):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(env, fams, q))
    p.start()
    r = q.get(timeout=400)
    p.join(timeout=60)
    assert not isinstance(r, str), r
    return r


@pytest.fixture(scope="module")
def defaults():
    return _run({}, FAMILIES)


def _compare(fam, got, ref, exact):
    for k, r in ref.items():
        g = got[k]
        assert g.shape == r.shape, (fam, k)
        if exact:
            np.testing.assert_array_equal(g, r, err_msg=f"{fam} {k}")
        elif fam in ("eqv2", "eqv2_l6"):
            err = np.abs(g - r)
            assert (err <= 2e-5 + 2e-5 * np.abs(r)).all(), (fam, k, err.max())
        elif k.startswith("g/"):
            e, sc = np.abs(g - r).max(), np.abs(r).max()
            assert e <= 2e-4 * sc + 1e-7, (fam, k, e, sc)
        else:
            rel = 3e-5 if fam == "ponita" else 1e-5
            g2, r2 = g.reshape(-1, g.shape[-1]), r.reshape(-1, r.shape[-1])
            err, sc = np.abs(g2 - r2).max(0), np.abs(r2).max(0)
            assert (err <= rel * sc + 1e-7).all(), (fam, k, (err / np.maximum(sc, 1e-30)).max())


@pytest.mark.parametrize("env,fams", SWITCHES, ids=lambda x: ",".join(f"{k}={v}" for k, v in x.items())
                         if isinstance(x, dict) else None)
def test_switch_matches_default_path(env, fams, defaults):
    got = _run(env, fams)
    for f in fams:
        _compare(f, got[f], defaults[f], exact=f == "gravity")
