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
        T.assert_close_cols(got, ref, rel=T.small_rel(env))


def _child_c2(env, q):
    """C2 widths at B = 1024, deterministic train-mode BatchNorm (fixed-order sums): one forward and a
    4-frame rollout."""
    os.environ.update(env)
    sys.path.insert(0, ROOT)
    try:
        import numpy as np
        import torch
        import nbody_amd.segnn as S
        import test_gpu_segnn as T
        dev = torch.device("cuda:0")
        torch.manual_seed(0)
        model = S.SEGNN(hidden_features=192, num_layers=6, deterministic=True).to(dev).train()
        pos, vel, mass = T.states(1024, 5, seed=17)
        fwd = T.gpu_forward(model, pos, vel, mass, 1024, 5, dev)
        t = lambda a: torch.tensor(a.reshape(1024, 5, -1), dtype=torch.float32, device=dev)
        tp, tv = model.rollout(t(pos), t(vel), t(mass), 4)
        q.put([fwd, tp.cpu().numpy(), tv.cpu().numpy()])
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put(repr(e) + traceback.format_exc())


def test_register_dot_operands_bit_identical():
    """The register-formed dot operands (default: message_layer_2's m_v . rhat, update_layer_1's
    x_v . na / a_v . na, update_layer_2's h_v . na, pre_pool1's x_v . na; tp_fused.h TpStream) are
    the materialised operands bit for bit: the consumer forms the dot of the stored values in the
    producers' fmaf order and then applies the segment's BatchNorm scale, as the materialised path
    does.  C2 forward + 4-frame rollout, deterministic BatchNorm, default vs
    NBX_UPD_DV=0 + NBX_MSG_DV=0."""
    import numpy as np
    ctx = mp.get_context("spawn")
    outs = []
    for env in ({}, {"NBX_UPD_DV": "0", "NBX_MSG_DV": "0"}):
        q = ctx.Queue()
        p = ctx.Process(target=_child_c2, args=(env, q))
        p.start()
        outs.append(q.get(timeout=240))
        p.join(timeout=60)
        assert not isinstance(outs[-1], str), outs[-1]
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


def _child_mp_check(env, q):
    """NBX_MP_CHECK builds of msg_pre's hand-off: C2 widths at B = 1024, 8 eval-mode and 8 train-mode
    forwards on different batches and a 6-frame train-mode rollout; returns the eval outputs and the
    number of hand-off invariant violations counted."""
    os.environ.update(env)
    sys.path.insert(0, ROOT)
    try:
        import ctypes
        import torch
        import nbody_amd._lib as L
        import test_gpu_segnn as T
        dev = torch.device("cuda:0")
        model = T.make_model(192, 6, dev, perturb_bn=False)
        model.range_check = os.environ.get("NBX_MP_CHECK") != "2"   # injected faults may give non-finite values
        sd0 = {k: v.clone() for k, v in model.state_dict().items()}
        evals = []
        for mode in ("eval", "train"):
            model.train(mode == "train")
            for k in range(8):
                model.load_state_dict(sd0)
                pos, vel, mass = T.states(1024, 5, seed=300 + k)
                o = T.gpu_forward(model, pos, vel, mass, 1024, 5, dev)
                if mode == "eval":
                    evals.append(o)
        model.load_state_dict(sd0)
        pos, vel, mass = T.states(1024, 5, seed=400)
        t = lambda a: torch.tensor(a.reshape(1024, 5, -1), dtype=torch.float32, device=dev)
        model.rollout(t(pos), t(vel), t(mass), 6)
        n = ctypes.c_uint32(0)
        L.check(L.lib().nbx_debug_msg_pre_check(ctypes.byref(n), 1), "nbx_debug_msg_pre_check")
        q.put((evals, int(n.value)))
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put(repr(e) + traceback.format_exc())


def test_msg_pre_handoff_invariant():
    """DESIGN.md §3.5b (the r05 hand-off race): with NBX_MP_CHECK=1 every wave of message_layer_1 checks the
    stage tag of each exchange buffer it consumes against the group its per-wave counters promised.  No
    mismatch over 16 C2 forwards (eval and train mode) and a rollout, and the checked kernel computes the
    default kernel's eval-mode outputs bit for bit.  NBX_MP_CHECK=2 drops the edge waves' wait (fault
    injection): the check must then fire, so a clean count means something."""
    import numpy as np
    ctx = mp.get_context("spawn")
    res = {}
    for tag, env in (("default", {}), ("check", {"NBX_MP_CHECK": "1"}), ("inject", {"NBX_MP_CHECK": "2"})):
        q = ctx.Queue()
        p = ctx.Process(target=_child_mp_check, args=(env, q))
        p.start()
        res[tag] = q.get(timeout=300)
        p.join(timeout=60)
        assert not isinstance(res[tag], str), res[tag]
        print(f"[{tag}] hand-off mismatches counted: {res[tag][1]}")
    assert res["default"][1] == 0            # check off: nothing counted
    assert res["check"][1] == 0, res["check"][1]
    for a, b in zip(res["default"][0], res["check"][0]):
        np.testing.assert_array_equal(a, b)
    assert res["inject"][1] > 0
