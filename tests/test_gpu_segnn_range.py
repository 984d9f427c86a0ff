"""fp16x2 range guard and the configured C2 horizon (include/nbx.h nbx_segnn_range_check).

The default SEGNN path splits every fp32 tensor-product operand into two fp16 parts: fp32-accurate for
|a| < 65504, while an operand at |a| >= 65520 becomes an fp16 infinity.  Every split kernel raises the
call's range flag when one of its output tiles is not finite, and SEGNN.forward / rollout report it as
NbxError (the reference would return non-finite values or, for an operand the fp32 path handles,
finite ones: the bf16x3 path, NBX_SPLIT=x3, has the fp32 exponent range).

The library reads its path switches once per process: paths other than the default run in spawned
children (one at a time)."""
import multiprocessing as mp
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import test_gpu_segnn as T  # noqa: E402


def _spawn(fn, env, *args, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=fn, args=(env, q) + args)
    p.start()
    r = q.get(timeout=timeout)
    p.join(timeout=60)
    assert not isinstance(r, str), r
    return r


def test_large_magnitude_inputs_in_range_match_oracle(hip_device):
    """Eval-mode BatchNorm (running statistics: nothing renormalises the first layer's inputs) with
    positions ~30x the C2 spread and speeds ~10x: every operand stays inside the fp16 range, the call
    returns finite outputs that match the fp64 oracle per column (1e-5)."""
    model = T.make_model(192, 6, hip_device, perturb_bn=True).eval()
    B, N = 64, 5
    pos, vel, mass = T.states(B, N, seed=31)
    pos, vel = pos * 30.0, vel * 10.0
    got = T.gpu_forward(model, pos, vel, mass, B, N, hip_device)
    ref, _ = T.oracle_forward(model, T.params_of(model), pos, vel, mass, B, N, False)
    assert np.isfinite(got).all()
    T.assert_close_cols(got, ref)


def test_out_of_range_operand_raises(hip_device):
    """Positions ~1e6 (eval mode): the first layer's operands exceed the fp16 range.  The default path
    raises NbxError instead of returning non-finite values; a non-finite input raises too."""
    import nbody_amd._lib as L
    model = T.make_model(64, 2, hip_device, perturb_bn=False).eval()
    B, N = 8, 5
    pos, vel, mass = T.states(B, N, seed=32)
    with pytest.raises(L.NbxError, match="fp16"):
        T.gpu_forward(model, pos * 1e6, vel, mass, B, N, hip_device)
    bad = pos.copy()
    bad[3, 1] = np.nan
    with pytest.raises(L.NbxError, match="fp16"):
        T.gpu_forward(model, bad, vel, mass, B, N, hip_device)
    # the flag belongs to the call: an in-range call on the same workspace afterwards is clean
    out = T.gpu_forward(model, pos, vel, mass, B, N, hip_device)
    assert np.isfinite(out).all()
    # and a rollout whose later frame leaves the range is reported too (the flag spans every frame)
    t = lambda a: torch.tensor(a.reshape(B, N, -1), dtype=torch.float32, device=hip_device)
    with pytest.raises(L.NbxError, match="fp16"):
        model.rollout(t(pos * 1e6), t(vel), t(mass), 3)


def _child_bf16x3_large(env, q):
    os.environ.update(env)
    sys.path.insert(0, ROOT)
    try:
        import torch as th
        import test_gpu_segnn as TT
        dev = th.device("cuda:0")
        model = TT.make_model(64, 2, dev, perturb_bn=False).eval()
        pos, vel, mass = TT.states(8, 5, seed=32)
        q.put(TT.gpu_forward(model, pos * 1e6, vel, mass, 8, 5, dev))
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put(repr(e) + traceback.format_exc())


def test_out_of_range_input_on_bf16x3_path_is_finite():
    """The same out-of-range call on the bf16x3 path (NBX_SPLIT=x3: bf16 parts carry the fp32 exponent
    range) returns finite outputs, which match the fp64 oracle per column at 1e-4 (operands ~1e6:
    cancellation in the relative positions costs fp32 digits on every path)."""
    got = _spawn(_child_bf16x3_large, {"NBX_SPLIT": "x3"})
    assert np.isfinite(got).all()
    model = T.make_model(64, 2, torch.device("cpu"), perturb_bn=False).eval()
    pos, vel, mass = T.states(8, 5, seed=32)
    ref, _ = T.oracle_forward(model, T.params_of(model), pos * 1e6, vel, mass, 8, 5, False)
    T.assert_close_cols(got, ref, rel=1e-4)


QS = (0.5, 0.9, 0.99)
FRAMES = (100, 500, 999)


def _child_c2_1000(env, q):
    """The configured C2 rollout (BASELINE.json configs[1]: 1000 frames = 999 model steps, B = 1024,
    train-mode BatchNorm with the bench's atomic sums), GravitySim frame-0 states: percentiles of
    |pos| and |vel| per body at FRAMES."""
    os.environ.update(env)
    sys.path.insert(0, ROOT)
    try:
        import torch as th
        import nbody_amd.segnn as S
        fx = np.load(os.path.join(ROOT, "tests", "golden", "segnn_c2_rollout.npz"))
        dev = th.device("cuda:0")
        th.manual_seed(0)
        model = S.SEGNN(hidden_features=192, num_layers=6).to(dev).train()
        t = lambda a: th.tensor(a, dtype=th.float32, device=dev)
        tp, tv = model.rollout(t(fx["loc0"]), t(fx["vel0"]), t(np.ones(fx["loc0"].shape[:2] + (1,))), 1000)
        finite = bool(th.isfinite(tp).all().item() and th.isfinite(tv).all().item())
        res = {"finite": finite}
        for f in FRAMES:
            for name, x in (("pos", tp[:, f]), ("vel", tv[:, f])):
                n = x.norm(dim=-1).reshape(-1).double()
                res[(name, f)] = [float(th.quantile(n, qq).item()) for qq in QS]
        q.put(res)
    except Exception as e:  # surfaced by the parent
        import traceback
        q.put(repr(e) + traceback.format_exc())


def test_c2_1000_frame_rollout_in_range_and_matches_fp32_statistics():
    """The configured C2 horizon (infer_self_feed.py:70-82: T_save - 1 = 999 model steps) on the default
    fp16x2 path: no operand leaves the fp16 range (no NbxError), every frame is finite, and the |pos| /
    |vel| distributions over the 5 120 bodies at frames 100, 500 and 999 (p50, p90, p99) agree with the
    fp32-MFMA path's (NBX_X3=0) within a factor of 2.  The rollout is chaotic past ~5 steps (docstring
    of test_rollout_c2_matches_oracle_fixture), so trajectories are compared as distributions."""
    d = _spawn(_child_c2_1000, {}, timeout=600)
    f = _spawn(_child_c2_1000, {"NBX_X3": "0"}, timeout=600)
    assert d["finite"] and f["finite"]
    bad = []
    for fr in FRAMES:
        for name in ("pos", "vel"):
            a, b = np.array(d[(name, fr)]), np.array(f[(name, fr)])
            print(f"frame {fr} |{name}| p50/p90/p99: default {a.round(3).tolist()} fp32-MFMA {b.round(3).tolist()}")
            ratio = np.maximum(a, 1e-12) / np.maximum(b, 1e-12)
            if (ratio > 2.0).any() or (ratio < 0.5).any():
                bad.append((fr, name, a.tolist(), b.tolist()))
    assert not bad, bad
