"""fp16x2 range guard of the PONITA and EquiformerV2 calls (include/nbx.h nbx_ponita_range_check /
nbx_eqv2_range_check, ABI 17).

Both families run their GEMMs on the fp16x2 split by default: fp32-accurate for operands |a| < 65504,
while a larger operand becomes an fp16 infinity in its hi part.  Every split GEMM raises the call's flag
when a live output tile is not finite, and the modules report it as NbxError after the forward or the
rollout instead of returning non-finite values.  The checks here: an out-of-range input and a NaN input
raise (PONITA: positions 1e6x the unit spread reach the kernel-basis MLP's GEMM unnormalised; every
EquiformerV2 GEMM input is normalised, so there large inputs stay in range); inputs inside the range do
not raise (no false positive) and stay finite; the flag belongs to one call, so a good call after a bad
one succeeds and reproduces the earlier result bit for bit."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _states(B, N, seed):
    rng = np.random.default_rng(seed)
    loc = rng.standard_normal((B, N, 3))
    vel = rng.standard_normal((B, N, 3)) * 0.3
    return loc, vel, np.ones((B, N, 1))


def test_ponita_out_of_range_raises_and_in_range_is_finite(hip_device):
    import nbody_amd._lib as L
    import test_ponita as TP
    m = TP.make(32, 2).to(hip_device)
    m.eval()
    B, N = 8, 5
    loc, vel, mass = _states(B, N, 41)
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=hip_device)
    # in range: positions 3x the unit spread (pair distances up to ~20, Poly(3) invariant features up to
    # ~1e4 before the basis MLP's first layer): no false positive
    tp, tv = m.rollout(t(loc * 3.0), t(vel), t(mass), 3)
    assert torch.isfinite(tp).all() and torch.isfinite(tv).all()
    with pytest.raises(L.NbxError, match="fp16"):
        m.rollout(t(loc * 1e6), t(vel), t(mass), 3)
    bad = loc.copy()
    bad[0, 0, 0] = np.nan
    with pytest.raises(L.NbxError, match="fp16"):
        m.rollout(t(bad), t(vel), t(mass), 2)
    # the flag is per call
    tp2, _ = m.rollout(t(loc * 3.0), t(vel), t(mass), 3)
    assert torch.equal(tp2, tp)


def test_eqv2_nonfinite_input_raises_and_large_inputs_stay_in_range(hip_device):
    import nbody_amd._lib as L
    import test_gpu_eqv2 as TE
    m = TE.make_model("c4", hip_device)
    B, N = 2, 20
    loc, vel, mass = _states(B, N, 42)
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=hip_device)
    # large inputs: EquiformerV2 normalises every GEMM input (RMS / LayerNorm, the radial LayerNorms), so
    # positions and speeds 1e3x the unit spread keep every split operand in range: finite, no error
    tp, tv = m.rollout(t(loc * 1e3), t(vel * 1e3), t(mass), 3, seed=5)
    assert torch.isfinite(tp).all() and torch.isfinite(tv).all()
    bad = vel.copy()
    bad[1, 3, 2] = np.nan
    with pytest.raises(L.NbxError, match="fp16"):
        m.rollout(t(loc), t(bad), t(mass), 2, seed=5)
    tp2, _ = m.rollout(t(loc * 1e3), t(vel * 1e3), t(mass), 3, seed=5)
    assert torch.equal(tp2, tp)
