"""EquiformerV2 product module on the CPU: reference-compatible state dict, seeded initialisation,
constant buffers and the weight packing the C-ABI reads (no device call)."""
import math
import json
import os
import sys

import numpy as np
import pytest
import torch

from nbody_amd import so3
from nbody_amd.equiformer_v2 import EquiformerV2_nbody

HERE = os.path.dirname(os.path.abspath(__file__))
Z = np.load(os.path.join(HERE, "golden", "eqv2.npz"))
STATE = json.load(open(os.path.join(HERE, "golden", "eqv2_state.json")))
sys.path.insert(0, os.path.join(HERE, "golden"))


def model(tag, seed=0):
    torch.manual_seed(seed)
    return EquiformerV2_nbody(device=None, **STATE[tag]["config"])


@pytest.mark.parametrize("tag", ["c4", "inf"])
def test_state_dict_matches_reference_keys_and_shapes(tag):
    sd = model(tag).state_dict()
    ref = STATE[tag]["keys"]
    assert sorted(sd) == sorted(ref)
    for k, shape in ref.items():
        assert list(sd[k].shape) == shape, k
    assert sorted(k for k, _ in model(tag).named_parameters()) == sorted(STATE[tag]["params"])


def test_seeded_init_matches_reference():
    """torch.manual_seed(0) -> the reference's parameters (RNG draws in the reference's order)."""
    m = model("c4", 0)
    names = [str(n) for n in Z["seed0/names"]]
    params = dict(m.named_parameters())
    assert names == [k for k, _ in m.named_parameters()]
    for i, k in enumerate(names):
        p = params[k].detach().reshape(-1).double()
        n = min(4, p.numel())
        np.testing.assert_array_equal(p[:n].numpy(), Z["seed0/head"][i, :n], err_msg=k)
        assert p.sum().item() == pytest.approx(Z["seed0/sum"][i], rel=1e-6, abs=1e-6), k


def test_grid_and_mapping_buffers_match_reference():
    for l in range(3):
        for m in range(l + 1):
            to, fr = so3.so3_grid(l, m)
            np.testing.assert_allclose(to.numpy(), Z[f"grid/{l}{m}/to"], rtol=2e-7, atol=1e-7)
            np.testing.assert_allclose(fr.numpy(), Z[f"grid/{l}{m}/from"], rtol=2e-7, atol=1e-7)
    mp = so3.coefficient_mapping([2], [1])
    assert mp["m_size"].tolist() == [3.0, 2.0]
    perm = mp["to_m"].argmax(1).tolist()
    assert perm == [0, 2, 5, 3, 6, 1, 4]          # m-primary order of the 7 kept coefficients


def test_reference_checkpoint_round_trip(tmp_path):
    """A reference-format checkpoint ({"model_state_dict": ...}) loads strictly."""
    m = model("c4", 3)
    torch.save({"model_state_dict": m.state_dict()}, tmp_path / "ck.pt")
    m2 = model("c4", 4)
    m2.load_state_dict(torch.load(tmp_path / "ck.pt", weights_only=True)["model_state_dict"])
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k


def test_packing_folds_the_first_radial_layer():
    """h1 = W0 [dexp(d) | E_s[z_s] | E_t[z_t]] + b0 == d a + c + us[z_s] + ut[z_t]."""
    m = model("c4", 1)
    P = m.packed_tensors("cpu")
    rad = m.blocks[0].ga.so2_conv_1.rad_func.net
    d, zs, zt = 1.7, 1, 3
    dexp = m.distance_expansion(torch.tensor([[d]]))
    x = torch.cat([dexp, m.blocks[0].ga.source_embedding.weight[zs:zs + 1],
                   m.blocks[0].ga.target_embedding.weight[zt:zt + 1]], 1)
    ref = rad[0](x).detach().double()[0]
    p = "blocks.0.ga.rad."
    got = d * P[p + "a"].double() + P[p + "c"].double() + P[p + "us"][zs].double() + P[p + "ut"][zt].double()
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    # permuted last radial layer: row 160 cb + 32 g + i <- original g * 2C + 32 cb + i
    C = m.sphere_channels
    b2 = rad[6].bias.detach()
    for cb in range(2 * C // 32):
        for g in range(5):
            assert torch.equal(P[p + "b2"][160 * cb + 32 * g:160 * cb + 32 * g + 32],
                               b2[g * 2 * C + 32 * cb:g * 2 * C + 32 * cb + 32])


def test_pack_weights_fills_every_pointer():
    import nbody_amd._lib as lib
    m = model("c4", 2)
    W = m.pack_weights("cpu")
    assert W.num_layers == 4 and W.sphere_channels == 64

    def walk(s, path=""):
        for name, _ in s._fields_:
            v = getattr(s, name)
            if isinstance(v, lib.ctypes.Structure):
                yield from walk(v, path + name + ".")
            elif isinstance(v, lib.ctypes.Array):
                continue
            elif name not in ("sphere_channels", "attn_hidden", "num_heads", "alpha_channels", "value_channels",
                              "ffn_hidden", "edge_channels", "num_layers", "num_elements", "h2_pad"):
                yield path + name, v
    nulls = [k for k, v in walk(W) if not v]
    # the attention radials use the bf16x3 / fp16x2 images of nbx_eqv2_attn, the edge-degree radial the fp32
    # matrix and its own fp16x2 image (ABI 18)
    assert sorted(nulls) == ["edge_degree.w2_x3", "force.rad.w2", "force.rad.w2_h2"], nulls
    for i in range(4):
        assert [k for k, v in walk(W.blocks[i]) if not v] == ["ga.rad.w2", "ga.rad.w2_h2"]
    # the fp16x2 descale factors are powers of two
    for s in (W.edge_degree.w1_sinv, W.edge_degree.w2_sinv, W.force.rad.w1_sinv, W.blocks[0].ga.rad.w1_sinv):
        assert s > 0 and math.frexp(s)[0] == 0.5, s


def test_unsupported_configuration_fails_loudly():
    torch.manual_seed(0)
    m = EquiformerV2_nbody(num_layers=1, sphere_channels=48, attn_hidden_channels=32, ffn_hidden_channels=32,
                           edge_channels=32, num_heads=2, attn_alpha_channels=8, attn_value_channels=4,
                           lmax_list=[2], mmax_list=[1])
    with pytest.raises(NotImplementedError):
        m._weights(torch.device("cpu"))
