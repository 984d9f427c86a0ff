"""The SEGNN weight images (include/nbx.h "TP operand images") hold exactly the
elements the HIP kernels read: the kernels' LDS addressing (tp16.h / tp_fused.h
B-fragment reads) is restated here in numpy and checked against the packed
matrices.  CPU only."""
import numpy as np
import pytest
import torch

from nbody_amd.segnn import SEGNN


def read_cw16(img, off, c, kc, lane, half):
    base = off + kc * 512 + half * 256 + lane * 4
    return img[c, base:base + 4]


def read_cw32(img, off, c, kc, lane, q):
    base = off + kc * 1024 + q * 256 + lane * 4
    return img[c, base:base + 4]


@pytest.mark.parametrize("cw", [16, 32])
@pytest.mark.parametrize("Ks", [(96, 96, 48), (40, 24)])
def test_frag_image_addressing(cw, Ks):
    g = torch.Generator().manual_seed(0)
    rows = 70
    subs = [(torch.randn(rows, max(Ks), generator=g), K) for K in Ks]
    vec = (torch.randn(rows, 64, generator=g), 64)
    chunks = -(-rows // cw)
    img = SEGNN.frag_image(subs, vec, cw, chunks).numpy()
    kcs = [-(-K // 32) for K in Ks] + [2]
    assert img.shape == (chunks, sum(kcs) * 32 * cw)
    offs = np.concatenate([[0], np.cumsum(kcs)[:-1]]) * 32 * cw
    mats = [(W.numpy(), K) for W, K in subs] + [(vec[0].numpy(), vec[1])]
    for (W, K), off, kc_n in zip(mats, offs, kcs):
        for c in range(chunks):
            for kc in range(kc_n):
                for lane in range(64):
                    for part in range(2 if cw == 16 else 4):
                        if cw == 16:
                            got = read_cw16(img, off, c, kc, lane, part)
                            ch, k0 = c * 16 + lane % 16, 32 * kc + 8 * (lane // 16) + 4 * part
                        else:
                            got = read_cw32(img, off, c, kc, lane, part)
                            ch, k0 = c * 32 + lane % 32, 32 * kc + 16 * (lane // 32) + 4 * part
                        want = np.array([W[ch, k] if (ch < W.shape[0] and k < K) else 0.0
                                         for k in range(k0, k0 + 4)], dtype=np.float32)
                        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("hidden", [192, 32])
def test_tp_images_shapes(hidden):
    torch.manual_seed(0)
    m = SEGNN(hidden_features=hidden, num_layers=2)
    M = m.mul
    P = SEGNN.tp_images(m.packed_matrices(), M)
    kc = lambda K: -(-K // 32)  # noqa: E731
    c16 = -(-(-(-M // 16)) // 4) * 4
    assert P["layers.0.node_pre_s_img"].shape == (c16, 6 * kc(M) * 512)
    assert P["layers.0.node_pre_v_img"].shape == (c16, 6 * kc(M) * 512)
    assert P["layers.0.msg2_img"].shape == (-(-M // 32), (2 * kc(2 * M) + 2 * kc(M)) * 1024)
    assert P["layers.1.upd1_img"].shape == (c16, (2 * kc(4 * M) + 2 * kc(2 * M)) * 512)
    assert P["layers.1.upd2_img"].shape == (c16, (kc(2 * M) + 2 * kc(M)) * 512)
    assert P["pp1_img"].shape == (c16, (2 * kc(2 * M) + 2 * kc(M)) * 512)
    assert not any(k.endswith("_s_t") or k.endswith("_v_t") for k in P)
