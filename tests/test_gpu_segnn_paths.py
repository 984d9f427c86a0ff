"""Every SEGNN kernel-path switch against the fp64 oracle (DESIGN.md appendix "environment switches").

The library reads each switch once per process, so every setting runs in a spawned child process of
its own (sequentially: one GPU process at a time besides this one).  Each child computes two forwards
on the same seeded inputs -- the C2 widths (hidden 192, 6 layers; mul 96) at B = 64 and a mul-32
model (hidden 64, 2 layers), train-mode BatchNorm -- and the parent checks them against the numpy
oracle with the per-column tolerance of tests/test_gpu_segnn.py (SMALL_REL: the batch statistics
come from 320 / 20 nodes).  The default path is in the list too, so a switch that silently falls
back to it still has to be right."""
import multiprocessing as mp
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

SWITCHES = [
    {},                              # defaults: fp16x2 images, register-formed dot operands, atomic BN sums
    {"NBX_MSG_DV": "0"},             # message_layer_2 reads the m_v . rhat half of M1S
    {"NBX_UPD_DV": "0"},             # update_layer_1 / pre_pool1 read XD / AD
    {"NBX_SPLIT": "x3"},             # bf16x3 images
    {"NBX_X3": "0"},                 # fp32 MFMA
    {"NBX_STATIC": "0"},             # run-time-shaped K loops
    {"NBX_MP_XCD": "0"},             # msg_pre chunk-major block order
    {"NBX_BN_ATOMIC": "0"},          # BatchNorm through finalize launches
]
CONFIGS = [(192, 6, 64, 5), (64, 2, 4, 5)]   # hidden, layers, B, N


def _child(env, q):
    os.environ.update(env)
    sys.path.insert(0, ROOT)
    try:
        import torch
        import test_gpu_segnn as T
        dev = torch.device("cuda:0")
        outs = []
        for hidden, layers, B, N in CONFIGS:
            model = T.make_model(hidden, layers, dev).train()
            pos, vel, mass = T.states(B, N, seed=11)
            outs.append(T.gpu_forward(model, pos, vel, mass, B, N, dev))
        q.put(outs)
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put(repr(e) + traceback.format_exc())


@pytest.fixture(scope="module")
def oracle_outputs():
    import torch
    import test_gpu_segnn as T
    refs = []
    for hidden, layers, B, N in CONFIGS:
        model = T.make_model(hidden, layers, torch.device("cpu")).train()
        pos, vel, mass = T.states(B, N, seed=11)
        ref, _ = T.oracle_forward(model, T.params_of(model), pos, vel, mass, B, N, True)
        refs.append(ref)
    return refs


@pytest.mark.parametrize("env", SWITCHES, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()) or "default")
def test_segnn_path_switch_matches_oracle(env, oracle_outputs):
    import test_gpu_segnn as T
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(env, q))
    p.start()
    outs = q.get(timeout=240)
    p.join(timeout=60)
    assert not isinstance(outs, str), outs
    for (hidden, layers, B, N), got, ref in zip(CONFIGS, outs, oracle_outputs):
        print(f"[{env or 'default'}] hidden {hidden} layers {layers} B {B}")
        T.assert_close_cols(got, ref, rel=T.SMALL_REL)
