"""The SEGNN weight images (include/nbx.h "TP operand images") hold exactly the
elements the HIP kernels read: the kernels' LDS addressing (tp16.h / tp_fused.h
B-fragment reads) is restated here in numpy and checked against the packed
matrices.  CPU only."""
import math

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
    assert P["layers.0.msg2_img_x3"].shape == (-(-M // 32), (2 * kc(2 * M) + 2 * kc(M)) * 3072)
    assert P["layers.0.msg2_img_x3"].dtype == torch.int16
    assert P["layers.1.upd1_img"].shape == (c16, (2 * kc(4 * M) + 2 * kc(2 * M)) * 512)
    assert P["layers.1.upd1_img_x3"].shape == (c16, (2 * kc(4 * M) + 2 * kc(2 * M)) * 1536)
    assert P["layers.1.upd2_img"].shape == (c16, (kc(2 * M) + 2 * kc(M)) * 512)
    assert P["pp1_img"].shape == (c16, (2 * kc(2 * M) + 2 * kc(M)) * 512)
    assert not any(k.endswith("_s_t") or k.endswith("_v_t") for k in P)


def test_frag_image_x3_addressing_and_split():
    """bf16x3 image (tp_fused.h StatSKX3 path): lane l, MFMA m, element j of part p holds part p of
    W[32 c + (l & 31)][32 kc + 16 (l >> 5) + 8 m + j]; hi + mid + lo reconstructs W to 2^-27."""
    g = torch.Generator().manual_seed(1)
    rows, Ks = 40, (64, 40)
    subs = [(torch.randn(rows, max(Ks), generator=g) * 10.0 ** torch.randint(-3, 3, (rows, 1), generator=g), K)
            for K in Ks]
    vec = (torch.randn(rows, 32, generator=g), 32)
    chunks = -(-rows // 32)
    img = SEGNN.frag_image_x3(subs, vec, chunks).view(torch.bfloat16).float().numpy()
    kcs = [-(-K // 32) for K in Ks] + [1]
    assert img.shape == (chunks, sum(kcs) * 3072)
    offs = np.concatenate([[0], np.cumsum(kcs)[:-1]]) * 3072
    mats = [(W.double().numpy(), K) for W, K in subs] + [(vec[0].double().numpy(), vec[1])]
    lane = np.arange(64)
    for (W, K), off, kc_n in zip(mats, offs, kcs):
        for c in range(chunks):
            for kc in range(kc_n):
                for m in range(2):
                    blk = img[c, off + kc * 3072:off + (kc + 1) * 3072].reshape(3, 2, 64, 8)[:, m]
                    ch = c * 32 + lane % 32
                    k = 32 * kc + 16 * (lane // 32)[:, None] + 8 * m + np.arange(8)[None, :]
                    want = np.zeros((64, 8))
                    ok = (ch[:, None] < W.shape[0]) & (k < K)
                    want[ok] = W[np.broadcast_to(ch[:, None], k.shape)[ok], k[ok]]
                    got = blk.astype(np.float64).sum(0)
                    np.testing.assert_allclose(got, want, rtol=2.0 ** -26, atol=0)
                    # the parts are ordered and non-overlapping: |mid| <= ulp_bf16(hi)/2, |lo| <= ulp(mid)/2
                    assert np.all(np.abs(blk[1]) <= np.abs(blk[0]) * 2.0 ** -8 + 1e-38)
                    assert np.all(np.abs(blk[2]) <= np.abs(blk[1]) * 2.0 ** -8 + 1e-38)


def test_frag_image_x3_cw16_addressing():
    """CW = 16 bf16x3 image (msg_pre.hip X3 node GEMM, v_mfma_f32_16x16x32_bf16): lane l, element j
    of part p holds part p of W[16 c + (l & 15)][32 kc + 8 (l >> 4) + j]."""
    g = torch.Generator().manual_seed(2)
    rows, Ks = 40, (96, 96)
    subs = [(torch.randn(rows, 96, generator=g), K) for K in Ks]
    chunks = -(-rows // 16)
    img = SEGNN.frag_image_x3(subs, None, chunks, 16).view(torch.bfloat16).float().numpy()
    assert img.shape == (chunks, 2 * 3 * 3 * 64 * 8)
    lane = np.arange(64)
    for j, (W, K) in enumerate(subs):
        W = W.double().numpy()
        for c in range(chunks):
            for kc in range(3):
                off = (j * 3 + kc) * 1536
                blk = img[c, off:off + 1536].reshape(3, 64, 8)
                ch = c * 16 + lane % 16
                k = 32 * kc + 8 * (lane // 16)[:, None] + np.arange(8)[None, :]
                want = np.where(ch[:, None] < rows, W[np.minimum(ch, rows - 1)[:, None], k], 0.0)
                np.testing.assert_allclose(blk.astype(np.float64).sum(0), want, rtol=2.0 ** -26, atol=0)


@pytest.mark.parametrize("cw", [32, 16])
def test_frag_image_h2_addressing_and_split(cw):
    """fp16x2 image (include/nbx.h "fp16x2 images"; tp_fused.h / tp16.h StatSKH2, msg_pre PREC 2):
    the bf16x3 addressing with two fp16 parts of W s, s = SEGNN.h2_scale; hi + lo reconstructs W s to
    2^-22 relative (max |W s| in [2^9, 2^10)), and hi is W s rounded to fp16 (RNE)."""
    g = torch.Generator().manual_seed(3)
    rows, Ks = 40, (64, 40)
    subs = [(torch.randn(rows, max(Ks), generator=g) * 10.0 ** torch.randint(-3, 1, (rows, 1), generator=g), K)
            for K in Ks]
    vec = (torch.randn(rows, 32, generator=g), 32)
    s = SEGNN.h2_scale(*[W[:, :K] for W, K in subs], vec[0])
    mx = max(float(W[:, :K].abs().max()) for W, K in subs + [vec])
    assert 2.0 ** 9 <= mx * s < 2.0 ** 10 and math.log2(s) == int(math.log2(s))
    chunks = -(-rows // cw)
    img = SEGNN.frag_image_h2(subs, vec, chunks, cw, s).view(torch.float16).float().numpy()
    kcs = [-(-K // 32) for K in Ks] + [1]
    blk_n = 2 * 32 * cw
    assert img.shape == (chunks, sum(kcs) * blk_n)
    offs = np.concatenate([[0], np.cumsum(kcs)[:-1]]) * blk_n
    mats = [(W.double().numpy() * s, K) for W, K in subs] + [(vec[0].double().numpy() * s, vec[1])]
    lane = np.arange(64)
    for (W, K), off, kc_n in zip(mats, offs, kcs):
        for c in range(chunks):
            for kc in range(kc_n):
                blk = img[c, off + kc * blk_n:off + (kc + 1) * blk_n]
                ms = [blk.reshape(2, 2, 64, 8)[:, m] for m in range(2)] if cw == 32 else [blk.reshape(2, 64, 8)]
                for m, b in enumerate(ms):
                    ch = c * cw + lane % cw
                    k = (32 * kc + 16 * (lane // 32)[:, None] + 8 * m if cw == 32
                         else 32 * kc + 8 * (lane // 16)[:, None]) + np.arange(8)[None, :]
                    want = np.zeros((64, 8))
                    ok = (ch[:, None] < W.shape[0]) & (k < K)
                    want[ok] = W[np.broadcast_to(ch[:, None], k.shape)[ok], k[ok]]
                    np.testing.assert_allclose(b.astype(np.float64).sum(0), want, rtol=2.0 ** -21,
                                               atol=2.0 ** -24)
                    np.testing.assert_array_equal(b[0], want.astype(np.float32).astype(np.float16).astype(np.float32))


def test_tp_images_h2_entries():
    """tp_images emits an fp16x2 image + descale for every TP the fp16x2 kernels run (node_pre pair,
    msg2 CW 32, upd1 / upd2 / pp1 CW 16), each image the same bytes as the fp32 one."""
    M = 96
    m = SEGNN(hidden_features=2 * M, num_layers=2)
    P = SEGNN.tp_images(m.packed_matrices(), M)
    for k in ("layers.0.node_pre_s_img", "layers.0.node_pre_v_img", "layers.1.msg2_img", "layers.0.upd1_img",
              "layers.1.upd2_img", "pp1_img"):
        h2 = P[k + "_h2"]
        assert h2.dtype == torch.int16 and h2.numel() * 2 == P[k].numel() * 4
    for k in ("layers.0.node_pre_h2_descale", "layers.1.msg2_h2_descale", "layers.0.upd1_h2_descale",
              "layers.1.upd2_h2_descale", "pp1_h2_descale"):
        d = P[k]
        assert isinstance(d, float) and d > 0 and math.log2(d) == int(math.log2(d))
