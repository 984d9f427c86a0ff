// Fine-grained variant of the fused tensor-product kernel: v_mfma_f32_16x16x4_f32,
// 16-row tiles, CG chunks of 16 output channels per wave.
//
// Same contract as tp_fused.h (TpProb, epilogues), but the weight chunks are
// 16 channels wide (B rows stored [chunks16][NS][16][K]) so node-row problems
// (V = B*N rows) spread over ~4x more waves, and accumulators are 4 registers
// per tile, which keeps 4 waves per SIMD resident.
//   16x16x4 f32 fragments: A lane l -> A[row = l & 15][k = l >> 4], B -> B[k = l >> 4][col = l & 15],
//   C register j -> row 4 (l >> 4) + j, col l & 15.  Dependent-issue latency is 40 cycles, so
//   the MFMAs of a k-step are issued round-robin over the (NS + 3 NV) x CG accumulators.
// Inside a 32-deep K chunk lane quarter qd supplies k = 8 qd + s at step s (permuted, same sum).
#pragma once
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "tp_fused.h"

namespace nbx {

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ inline float f4get(const float4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }

constexpr int T16_WAVES = 8, T16_THREADS = 64 * T16_WAVES;

// Two independent problems of the same shape class can share one launch (P0 for blocks below
// `split`, P1 above): node_pre's scalar-row and vector-row GEMMs fill the chip together.
template <int NS, int NV, int EPI, int CG, int WAVES = T16_WAVES, int PF = 3, int KS = 1, bool DUAL = false,
          class SK = DynSK>
__global__ __launch_bounds__(64 * WAVES, (SK::PREC || PF > 4) ? 1 : 2) void tp16_kernel(const TpProb P0, const TpProb P1, int split) {
    const bool second = DUAL && (int)blockIdx.x >= split;
    const TpProb& P = second ? P1 : P0;
    const int bidx = second ? (int)blockIdx.x - split : (int)blockIdx.x;
    constexpr int THREADS = 64 * WAVES;
    constexpr int TW = WAVES / KS;            // row-tile slots per block; KS waves split each tile's K
    static_assert(WAVES % KS == 0, "KS must divide WAVES");
    constexpr int NACC = CG * (NS + 3 * NV);
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int NT = NS + NV;  // B sub-tiles per chunk
    int cgroup, blk;   // group of CG 16-channel chunks, row-range block
    tp_block_map(P, bidx, cgroup, blk);
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, c16 = lane & 15, qd = lane >> 4;
    const int slice = wave % KS, tslot = wave / KS;
    const int nchunks16 = P.chunks;                        // total 16-channel chunks

    int sub_off[NS + 1];
    tp_img_offsets<NS>(P, 16, sub_off);
    const int stride_g = P.img_floats;                    // one 16-channel chunk image
    const int ks_chunks = (P.K[0] + 31) >> 5;
    const int kv_chunks = NV ? (P.Kv + 31) >> 5 : 0;
    const float kv_inv = 1.0f / (float)(kv_chunks > 0 ? kv_chunks : 1);
    const int n_chunks = ks_chunks + 3 * kv_chunks;
    const int c_lo = slice * n_chunks / KS, c_hi = (slice + 1) * n_chunks / KS;   // this wave's K chunks
    const int row_tiles = (P.rows + 15) >> 4;
    const int wstride = P.blocks_per_chunk * TW;
    const int wid = blk * TW + tslot;
    // iterations are uniform across the block (split-K waves meet at barriers)
    const int iters = (row_tiles - blk * TW + wstride - 1) / wstride;

    double st0[CG], st1[CG], st2[CG];
#pragma unroll
    for (int g = 0; g < CG; ++g) st0[g] = st1[g] = st2[g] = 0.0;

    // A loads are bounds-checked buffer loads: an invalid lane gets an out-of-range offset and
    // reads zeros, so every load issues unconditionally and the waitcnt pass can count them
    // (conditional loads would force vmcnt(0) at each use).  Buffers are < 2 GiB (launch check).
    const __amdgpu_buffer_rsrc_t rsS = __builtin_amdgcn_make_buffer_rsrc((void*)P.As, (short)0, 0x7FFFFFF0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsV =
        __builtin_amdgcn_make_buffer_rsrc((void*)(NV ? P.Av : P.As), (short)0, 0x7FFFFFF0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsSeg = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(SK::SEG > 0 ? P.seg_base : P.As), (short)0, 0x7FFFFFF0, 0x00020000);
    auto load_a = [&](int rt, int i, float4 (&a)[2]) {
        // branch-free: both the scalar- and the vector-chunk offsets are computed and selected,
        // so one pair of loads is issued from one code path; chunks outside [c_lo, c_hi) (ring
        // padding) and rows past the end read zeros
        const int row = rt * 16 + c16;
        const bool rok = row < P.rows && i < c_hi;
        const bool sc = !NV || i < ks_chunks;                      // wave-uniform
        const int v = sc ? 0 : i - ks_chunks;
        const int plane = NV ? tp_udiv_small(v, kv_inv) : 0;
        const int k = (sc ? i * 32 : (v - plane * kv_chunks) * 32) + 8 * qd;
        const bool ok = rok && k < (sc ? P.K[0] : P.Kv);
        const size_t eo = sc ? (size_t)row * P.lda_s + k
                             : (size_t)plane * P.plane_stride + (size_t)row * P.lda_v + k;
        const uint32_t off = ok ? (uint32_t)(eo * 4) : 0x7FFFFFF0u;
        const __amdgpu_buffer_rsrc_t rs = sc ? rsS : rsV;
        a[0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        a[1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? off + 16 : off, 0, 0));
    };

    // A streams through a ring of PF chunk buffers with fixed roles: chunk c_lo + u of a tile
    // lives in ring[u % PF] (the chunk stream is padded to a multiple of PF), and the load of
    // chunk u + PF - 1 (wrapping into the next tile) is issued before the MFMAs of chunk u, so
    // PF - 1 chunks are in flight behind the current one.  The first PF - 1 loads are issued
    // before the weight staging so both latencies overlap.
    const unsigned long long c_start = P.dbg ? clock64() : 0ull;
    const unsigned long long w_start = P.dbg ? wall_clock64() : 0ull;   // 100 MHz, chip-wide
    unsigned long long c_loop = 0ull, c_epi = 0ull, c_mark = 0ull;   // per-phase sums over tiles
    int rt = wid;
    const int nck = c_hi - c_lo;
    const int nc_pad = (nck + PF - 1) / PF * PF;
    float4 ring[PF][2];

    // ---- static schedule (SK::on): items of a tile = K0 scalar chunks (the first NA(i) sub-tiles
    // live) then KV chunks of each vector plane; split-K slice s owns items [s N / KS, (s+1) N / KS)
    constexpr int SNIT = SK::K0 + 3 * SK::KV;
    auto load_item = [&](auto ic, int rt_, float4 (&a)[2]) {
        constexpr int item = decltype(ic)::value;
        constexpr bool sc = item < SK::K0;
        constexpr int v = sc ? 0 : item - SK::K0;
        constexpr int plane = sc ? 0 : v / (SK::KV > 0 ? SK::KV : 1);
        constexpr int kc = sc ? item : v - plane * SK::KV;
        const int row = rt_ * 16 + c16;
        if constexpr (SK::SEG > 0) {
            // segment q of width M = (K0 / SEG) chunks (scalar) or (KV / (SEG / 2)) chunks (vector);
            // one resource over all segments (seg_base), the segment / plane as the scalar offset
            constexpr int cps = sc ? SK::K0 / SK::SEG : SK::KV / (SK::SEG / 2);
            constexpr int q = kc / cps, kk = (kc - q * cps) * 32;
            const int k = kk + 8 * qd;
            const bool ok = row < P.rows;
            const uint32_t soff = sc ? P.seg_boff[q] : P.seg_boff[4 + q] + (uint32_t)(plane * P.seg_vplane * 4);
            const uint32_t off = ok ? (uint32_t)(((size_t)row * P.M + k) * 4) : 0x7FFFFFF0u;
            a[0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsSeg, off, soff, 0));
            a[1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsSeg, ok ? off + 16 : off, soff, 0));
        } else {
            const int k = kc * 32 + 8 * qd;
            const bool ok = row < P.rows && k < (sc ? P.K[0] : P.Kv);
            const size_t eo =
                sc ? (size_t)row * P.lda_s + k : (size_t)plane * P.plane_stride + (size_t)row * P.lda_v + k;
            const uint32_t off = ok ? (uint32_t)(eo * 4) : 0x7FFFFFF0u;
            const __amdgpu_buffer_rsrc_t rs = sc ? rsS : rsV;
            a[0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
            a[1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? off + 16 : off, 0, 0));
        }
    };
    auto slice_call = [&](auto&& fn) {
        static_for<0, KS>([&](auto sc_) {
            if (slice == decltype(sc_)::value) fn(sc_);
        });
    };
    // DV (TpStream): the scalar operand's trailing dot chunks are formed from the vector chunks, not
    // loaded; loads run in TpStream load order (the item order unless DV)
    using TS = TpStream<SK>;
    static_assert(!SK::DV || (KS == 1 && NV == 1 && SK::PREC >= 1 && SK::K0 > SK::KV),
                  "DV: a split-precision scalar operand ending in KV dot chunks");
    constexpr int NLD = TS::NLOAD;   // DV loads (KS = 1)
    if constexpr (SK::on) {
        slice_call([&](auto sc_) {
            constexpr int lo = decltype(sc_)::value * SNIT / KS, hi = (decltype(sc_)::value + 1) * SNIT / KS;
            static_for<0, PF - 1>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                if constexpr (SK::DV) {
                    if constexpr (u < NLD) load_item(std::integral_constant<int, TS::item(TS::lpos(u))>{}, rt, ring[u % PF]);
                } else if constexpr (lo + u < hi) {
                    load_item(std::integral_constant<int, lo + u>{}, rt, ring[u % PF]);
                }
            });
        });
    } else {
#pragma unroll
        for (int u = 0; u < PF - 1; ++u) load_a(rt, c_lo + u, ring[u]);
    }

    // ---- segmented input: the BatchNorm coefficient inputs, loaded before the image DMA (one
    // evaluation per thread: message BN at t < 2M, feature BN at 2M <= t < 4M; kind = which half)
    // (evaluation index i = t + e THREADS over the 4M evaluations: NEV per thread for blocks smaller
    // than 4M threads; the segmented paths have M <= 96)
    const int bn_M = P.M;
    const bool bn_m = SK::SEG == 4 && P.mbn.sums != nullptr;   // message BN finalised here
    const bool bn_x = SK::SEG > 0 && P.xbn.sums != nullptr;    // pending feature BN finalised here
    constexpr int NEV = SK::SEG > 0 ? (4 * 96 + THREADS - 1) / THREADS : 1;
    BnPre bn_pre[NEV];
#pragma unroll
    for (int e = 0; e < NEV; ++e) {
        const int i = t + e * THREADS;
        const int which = i < 2 * bn_M ? 0 : 1, kind = (i % (2 * bn_M)) / bn_M, k = i < 4 * bn_M ? i % bn_M : 0;
        const bool on = SK::SEG > 0 && i < 4 * bn_M && (which == 0 ? bn_m : bn_x);
        bn_pre[e] = bn_pre_load(bn_src_sel(P.mbn, P.xbn, which == 1), bn_M, kind, k, on,
                                SK::SEG > 0 ? (const void*)P.seg_base : (const void*)P.As);
    }

    // ---- segmented input: the per-(segment, k) coefficients the table takes from an earlier kernel
    // (xcoef: the pending feature BN finalised by message_layer_1's block 0; mcoef: a finalised message
    // BN), loaded here, before the image DMA, into registers (branch-free, a dummy address for table
    // entries that need none): loaded after the DMA they cost one more memory round trip behind it
    constexpr int NSEG_IT = SK::SEG > 0 ? (10 * 96 + THREADS - 1) / THREADS : 1;
    float seg_raw[NSEG_IT];
#pragma unroll
    for (int j = 0; j < NSEG_IT; ++j) {
        const int i = t + j * THREADS;
        const int part = i / bn_M, k = i - part * bn_M;
        const bool isx = part == 0 || part == 2 || part == 4 || part == 8;
        const bool ism = SK::SEG == 4 && (part == 1 || part == 3 || part == 5 || part == 9);
        const bool need = SK::SEG > 0 && i < 10 * bn_M &&
                          ((isx && !bn_x && P.xcoef != nullptr) || (ism && !bn_m && P.mcoef != nullptr));
        const int idx = (part == 0 || part == 1) ? k : (part == 4 || part == 5) ? 2 * bn_M + k : bn_M + k;
        const float* src = need ? (isx ? P.xcoef : P.mcoef)
                                : static_cast<const float*>(SK::SEG > 0 ? (const void*)P.seg_base : (const void*)P.As);
        const float raw = src[need ? idx : 0];
        seg_raw[j] = need ? raw : 0.f;
    }

    // ---- stage the CG chunk images of this group in LDS (LDS-DMA, verbatim copy; the image
    // array holds a multiple of 4 chunks, so a group never runs past it)
    {
        const int stride = P.img_stride > 0 ? P.img_stride : P.img_floats;
        if (stride == P.img_floats) {
            tp_dma_image<WAVES>(P.B + (size_t)cgroup * CG * P.img_floats, lds, CG * P.img_floats);
        } else {
#pragma unroll
            for (int g = 0; g < CG; ++g)
                tp_dma_image<WAVES>(P.B + (size_t)(cgroup * CG + g) * stride, lds + g * P.img_floats, P.img_floats);
        }
    }
    // segmented update input: per-(segment, k) scale / shift table, after the images
    float* segtab = lds + CG * P.img_floats;
    if constexpr (SK::SEG > 0) {
        const int M = P.M;
        const bool mfin = bn_m, xfin = bn_x;
        // the BatchNorm parts from the preloaded inputs: message BN -> parts 1 (0e scale), 5 (shift x
        // deg), 3 and 9 (1o scale); feature BN -> parts 0, 4, 2 and 8
#pragma unroll
        for (int e = 0; e < NEV; ++e) {
            const int i = t + e * THREADS;
            const int bn_which = i < 2 * M ? 0 : 1, bn_kind = (i % (2 * M)) / M, bn_k = i % M;
            if (!(i < 4 * M && (bn_which == 0 ? bn_m : bn_x))) continue;
            const float2 c = bn_pre_coef(bn_which == 0 ? P.mbn : P.xbn, bn_pre[e], M, bn_kind, bn_k, blockIdx.x == 0);
            if (bn_which == 0) {
                if (bn_kind == 0) { segtab[1 * M + bn_k] = c.x; segtab[5 * M + bn_k] = P.deg * c.y; }
                else { segtab[3 * M + bn_k] = c.x; segtab[9 * M + bn_k] = c.x; }
            } else {
                if (bn_kind == 0) { segtab[0 * M + bn_k] = c.x; segtab[4 * M + bn_k] = c.y; }
                else { segtab[2 * M + bn_k] = c.x; segtab[8 * M + bn_k] = c.x; }
            }
        }
#pragma unroll
        for (int j = 0; j < NSEG_IT; ++j) {
            const int i = t + j * THREADS;
            if (i >= 10 * M) continue;
            const int part = i / M;   // part 0-3 scales, 4-7 shifts, 8-9 vector scales
            if (mfin && (part == 1 || part == 3 || part == 5 || part == 9)) continue;
            if (xfin && (part == 0 || part == 2 || part == 4 || part == 8)) continue;
            const float raw = seg_raw[j];   // xcoef / mcoef entry of this part (preloaded)
            float v;
            switch (part) {
                case 0: case 2: case 8: v = P.xcoef ? raw : 1.f; break;
                case 4: v = P.xcoef ? raw : 0.f; break;
                case 1: case 3: case 9: v = SK::SEG == 4 ? raw : 0.f; break;
                case 5: v = SK::SEG == 4 ? P.deg * raw : 0.f; break;
                default: v = 0.f;
            }
            segtab[i] = v;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long c_staged = P.dbg ? clock64() : 0ull;
    c_mark = c_staged;

    float* kred = lds + P.lds_floats - (KS > 1 ? TW * (KS - 1) * NACC * 4 * 64 : 0);  // split-K partials
    for (int it = 0; it < iters; ++it) {
        {
            // RESID: the epilogue's residual X rows and node attributes, loaded before the K loop so
            // their latency hides under the MFMAs (not after the last chunk)
            float rres[EPI == TP_RESID ? CG : 1][4][4];
            float rna[4][3];
            if constexpr (EPI == TP_RESID) {
                const int row0p = rt * 16 + 4 * qd;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int row = row0p + jj;
                    const bool rok = rt < row_tiles && row < P.rows;
#pragma unroll
                    for (int k = 0; k < 3; ++k) rna[jj][k] = rok ? P.geom[(size_t)row * 4 + 1 + k] : 0.f;
#pragma unroll
                    for (int g = 0; g < CG; ++g) {
                        const int ch = (cgroup * CG + g) * 16 + c16;
                        const bool ok = rok && ch < P.M;
                        const size_t o = (size_t)row * P.M + ch;
                        rres[g][jj][0] = ok ? P.out_s[o] : 0.f;
                        rres[g][jj][1] = ok ? P.out_v[o] : 0.f;
                        rres[g][jj][2] = ok ? P.out_v[P.out_plane + o] : 0.f;
                        rres[g][jj][3] = ok ? P.out_v[2 * P.out_plane + o] : 0.f;
                    }
                }
            }
            floatx4 acc[CG][NS + 3 * NV];
#pragma unroll
            for (int g = 0; g < CG; ++g)
#pragma unroll
                for (int j = 0; j < NS + 3 * NV; ++j) acc[g][j] = floatx4{0.f, 0.f, 0.f, 0.f};
            const int next_rt = rt + wstride;
            auto chunk = [&](const float4 (&cb)[2], int i) {
                const float av[8] = {cb[0].x, cb[0].y, cb[0].z, cb[0].w, cb[1].x, cb[1].y, cb[1].z, cb[1].w};
                if (i < ks_chunks) {
                    const int k0 = i * 32;
                    // sub-tiles are ordered by K descending (checked at launch): the first `na`
                    // are live at this k0.  Dispatch to a compile-time count so the B fragments
                    // are read in one batch and the MFMAs interleave over independent accumulators.
                    auto step = [&](auto na_c) {
                        constexpr int NA = decltype(na_c)::value;
                        float4 b[CG][NA][2];
#pragma unroll
                        for (int g = 0; g < CG; ++g)
#pragma unroll
                            for (int j = 0; j < NA; ++j) {
                                const float* bp = &lds[g * stride_g + sub_off[j] + i * 512 + 4 * lane];
                                b[g][j][0] = *reinterpret_cast<const float4*>(bp);
                                b[g][j][1] = *reinterpret_cast<const float4*>(bp + 256);
                            }
#pragma unroll
                        for (int s = 0; s < 8; ++s)
#pragma unroll
                            for (int g = 0; g < CG; ++g)
#pragma unroll
                                for (int j = 0; j < NA; ++j)
                                    acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                                        av[s], f4get(b[g][j][s >> 2], s & 3), acc[g][j], 0, 0, 0);
                    };
                    int na = 0;
#pragma unroll
                    for (int j = 0; j < NS; ++j) na += k0 < P.K[j] ? 1 : 0;
                    if (na >= NS) step(std::integral_constant<int, NS>{});
                    else if constexpr (NS >= 2) {
                        if (na == NS - 1) step(std::integral_constant<int, NS - 1>{});
                        else if constexpr (NS >= 3) {
                            if (na == NS - 2) step(std::integral_constant<int, NS - 2>{});
                        }
                    }
                } else if (NV) {
                    const int v = i - ks_chunks, plane = tp_udiv_small(v, kv_inv);
                    const int kc = v - plane * kv_chunks;
                    float4 b[CG][2];
#pragma unroll
                    for (int g = 0; g < CG; ++g) {
                        const float* bp = &lds[g * stride_g + sub_off[NS] + kc * 512 + 4 * lane];
                        b[g][0] = *reinterpret_cast<const float4*>(bp);
                        b[g][1] = *reinterpret_cast<const float4*>(bp + 256);
                    }
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl) {
                        if (pl != plane) continue;
#pragma unroll
                        for (int s = 0; s < 8; ++s)
#pragma unroll
                            for (int g = 0; g < CG; ++g) {
                                const float bv = f4get(b[g][s >> 2], s & 3);
                                acc[g][NS + pl] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv, acc[g][NS + pl], 0, 0, 0);
                            }
                    }
                }
            };
            // CG == 1: the vector chunks' 8 steps alternate between two accumulators per plane so
            // consecutive MFMAs are independent (16x16x4 f32: 32-cycle issue, 40-cycle latency)
            floatx4 accv2[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) accv2[pl] = floatx4{0.f, 0.f, 0.f, 0.f};
            // item's A chunk (lane quarter qd: k = 8 qd + e), with the segmented input's per-(segment, k)
            // BatchNorm scale / shift applied
            auto item_a = [&](auto ic, const float4 (&cb)[2], float (&av)[8]) {
                constexpr int item = decltype(ic)::value;
                constexpr bool sc = item < SK::K0;
                av[0] = cb[0].x; av[1] = cb[0].y; av[2] = cb[0].z; av[3] = cb[0].w;
                av[4] = cb[1].x; av[5] = cb[1].y; av[6] = cb[1].z; av[7] = cb[1].w;
                if constexpr (SK::SEG > 0) {
                    // table parts (segtab): scalar segment q -> part q (SEG 4) / 2 q (SEG 2: x_s, x_v.na),
                    // shifts for the 0e segments x_s (and a_s), vector segment q -> part 8 + q
                    constexpr int kc = sc ? item : (item - SK::K0) % SK::KV;
                    constexpr int cps = sc ? SK::K0 / SK::SEG : SK::KV / (SK::SEG / 2);
                    constexpr int q = kc / cps, kk = (kc - q * cps) * 32;
                    constexpr int part = sc ? (SK::SEG == 4 ? q : 2 * q) : 8 + q;
                    constexpr bool shifted = sc && (SK::SEG == 4 ? q < 2 : q == 0);
                    const int M = P.M;
                    const float* tsc = segtab + part * M + kk + 8 * qd;
                    const float4 s0 = *reinterpret_cast<const float4*>(tsc);
                    const float4 s1 = *reinterpret_cast<const float4*>(tsc + 4);
                    const float scv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
                    if constexpr (shifted) {
                        const float* tsh = segtab + 4 * M + q * M + kk + 8 * qd;
                        const float4 h0 = *reinterpret_cast<const float4*>(tsh);
                        const float4 h1 = *reinterpret_cast<const float4*>(tsh + 4);
                        const float shv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
                        for (int e = 0; e < 8; ++e) av[e] = fmaf(scv[e], av[e], shv[e]);
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) av[e] *= scv[e];
                    }
                }
            };
            auto compute_item = [&](auto ic, const float4 (&cb)[2]) {
                constexpr int item = decltype(ic)::value;
                constexpr bool sc = item < SK::K0;
                float av[8];
                item_a(ic, cb, av);
                if constexpr (sc) {
                    constexpr int NA = (item < SK::K0 ? 1 : 0) + (NS > 1 && item < SK::K1 ? 1 : 0) +
                                       (NS > 2 && item < SK::K2 ? 1 : 0);
                    float4 b[CG][NA][2];
#pragma unroll
                    for (int g = 0; g < CG; ++g)
#pragma unroll
                        for (int j = 0; j < NA; ++j) {
                            const float* bp = &lds[g * stride_g + sub_off[j] + item * 512 + 4 * lane];
                            b[g][j][0] = *reinterpret_cast<const float4*>(bp);
                            b[g][j][1] = *reinterpret_cast<const float4*>(bp + 256);
                        }
#pragma unroll
                    for (int s = 0; s < 8; ++s)
#pragma unroll
                        for (int g = 0; g < CG; ++g)
#pragma unroll
                            for (int j = 0; j < NA; ++j)
                                acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], f4get(b[g][j][s >> 2], s & 3),
                                                                                 acc[g][j], 0, 0, 0);
                } else {
                    constexpr int v = item - SK::K0, plane = v / SK::KV, kc = v - plane * SK::KV;
                    float4 b[CG][2];
#pragma unroll
                    for (int g = 0; g < CG; ++g) {
                        const float* bp = &lds[g * stride_g + sub_off[NS] + kc * 512 + 4 * lane];
                        b[g][0] = *reinterpret_cast<const float4*>(bp);
                        b[g][1] = *reinterpret_cast<const float4*>(bp + 256);
                    }
#pragma unroll
                    for (int s = 0; s < 8; ++s) {
                        if constexpr (CG == 1) {
                            if (s & 1)
                                accv2[plane] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], f4get(b[0][s >> 2], s & 3),
                                                                                    accv2[plane], 0, 0, 0);
                            else
                                acc[0][NS + plane] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                                    av[s], f4get(b[0][s >> 2], s & 3), acc[0][NS + plane], 0, 0, 0);
                        } else {
#pragma unroll
                            for (int g = 0; g < CG; ++g)
                                acc[g][NS + plane] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                                    av[s], f4get(b[g][s >> 2], s & 3), acc[g][NS + plane], 0, 0, 0);
                        }
                    }
                }
            };
            if (SK::PREC >= 1 && rt < row_tiles) {
                if constexpr (SK::PREC >= 1) {
                    // Split-precision path (tp_fused.h StatSKX3): v_mfma_f32_16x16x32_bf16, whose A
                    // fragment (lane quarter qd: k = 8 qd + j) is exactly the chunk a lane loads.
                    // Item u's B fragments are read from LDS while item u-1's MFMAs run, into a
                    // register set that stays allocated (empty asm uses) until item u+1's MFMAs have
                    // issued, so no load lands on the operands of an MFMA issued just before it
                    // (the measured gfx950 hazard is a load into the SrcA of the preceding
                    // v_mfma_f32_16x16x32_bf16 at 0 wait states; build.py checks the ISA for it).
                    // (PREC 2: the fp16x2 path, 2 parts and 3 terms on v_mfma_f32_16x16x32_f16, same structure)
                    using SP = SplitP<SK::PREC>;
                    using SPT = typename SP::T;
                    constexpr int NP = SP::NP;
                    constexpr int OB[4] = {0, SK::K0, SK::K0 + SK::K1, SK::K0 + SK::K1 + SK::K2};
                    auto read_b = [&](auto ic, SPT (&bx)[CG][NS > 1 ? NS : 1][NP]) {
                        constexpr int item = decltype(ic)::value;
                        if constexpr (item < SK::K0) {
                            static_for<0, NS>([&](auto jc) {
                                constexpr int j = decltype(jc)::value;
                                constexpr int KCj = j == 0 ? SK::K0 : j == 1 ? SK::K1 : SK::K2;
                                if constexpr (item < KCj)
#pragma unroll
                                    for (int g = 0; g < CG; ++g)
#pragma unroll
                                        for (int p3 = 0; p3 < NP; ++p3)
                                            bx[g][j][p3] = reinterpret_cast<const SPT*>(lds + g * stride_g)
                                                [(OB[j] + item) * (NP * 64) + p3 * 64 + lane];
                            });
                        } else {
                            constexpr int kc = (item - SK::K0) % SK::KV;
#pragma unroll
                            for (int g = 0; g < CG; ++g)
#pragma unroll
                                for (int p3 = 0; p3 < NP; ++p3)
                                    bx[g][0][p3] = reinterpret_cast<const SPT*>(lds + g * stride_g)
                                        [(OB[NS] + kc) * (NP * 64) + p3 * 64 + lane];
                        }
                    };
                    auto keep = [&](const SPT& v) { asm volatile("" ::"v"(v)); };
                    // B (SrcB) fragment sets: three (item u in set u % 3, each kept live until item u+1's
                    // MFMAs issued) or, with a deep A ring (PF > 3), two: the measured gfx950 hazard is on
                    // SrcA only (a load over an MFMA's SrcB at 0 wait states is safe, tools/hazard), and
                    // the 36 VGPRs saved hold the deeper A ring
                    constexpr int NBS = PF > 3 ? 2 : 3;
                    // DV: the node attributes of this lane's row (the dot weights) and the dot chunk being formed
                    float yv[3] = {0.f, 0.f, 0.f};
                    float dacc[8];
                    if constexpr (SK::DV) {
                        const int row = rt * 16 + c16;
                        if (row < P.rows) {
                            yv[0] = P.geom[(size_t)row * 4 + 1]; yv[1] = P.geom[(size_t)row * 4 + 2];
                            yv[2] = P.geom[(size_t)row * 4 + 3];
                        }
                    }
                    slice_call([&](auto sc_) {
                        // positions lo .. lo + n - 1 of the slice (TpStream; = items unless DV, where KS = 1)
                        constexpr int lo = decltype(sc_)::value * SNIT / KS;
                        constexpr int n = (decltype(sc_)::value + 1) * SNIT / KS - lo;
                        constexpr int nld = SK::DV ? TS::NLOAD : n;   // loads of the slice
                        SPT bx[NBS][CG][NS > 1 ? NS : 1][NP];   // position u in set u % NBS
                        SPT ax[3][NP];
                        read_b(std::integral_constant<int, TS::item(lo)>{}, bx[0]);
                        static_for<0, n>([&](auto uc) {
                            constexpr int u = decltype(uc)::value, pos = lo + u, item = TS::item(pos);
                            constexpr bool der = TS::derived(pos);
                            constexpr int l = der ? 0 : TS::lidx(pos) - TS::lidx(lo);   // load index in the slice
                            if constexpr (!der && l + PF - 1 < nld)
                                load_item(std::integral_constant<int, TS::item(TS::lpos(TS::lidx(lo) + l + PF - 1))>{}, rt,
                                          ring[(l + PF - 1) % PF]);
                            __builtin_amdgcn_sched_barrier(0);
                            if constexpr (u + 1 < n) read_b(std::integral_constant<int, TS::item(pos + 1)>{}, bx[(u + 1) % NBS]);
                            float av[8];
                            if constexpr (der) {
                                // the dot chunk, then its segment's BatchNorm scale: the same arithmetic as
                                // the materialised operand (producer dot of the stored values, scale applied
                                // by item_a as the chunk is consumed), so both paths give identical bits
                                const float4 dc[2] = {float4{dacc[0], dacc[1], dacc[2], dacc[3]},
                                                      float4{dacc[4], dacc[5], dacc[6], dacc[7]}};
                                item_a(std::integral_constant<int, item>{}, dc, av);
                            } else {
                                item_a(std::integral_constant<int, item>{}, ring[l % PF], av);
                                if constexpr (SK::DV && TS::plane(pos) >= 0) {
                                    // dot of the stored (unscaled) values, in the producers' fmaf order
                                    constexpr int pl = TS::plane(pos);
                                    const float4 (&cb)[2] = ring[l % PF];
                                    const float raw[8] = {cb[0].x, cb[0].y, cb[0].z, cb[0].w,
                                                          cb[1].x, cb[1].y, cb[1].z, cb[1].w};
#pragma unroll
                                    for (int e = 0; e < 8; ++e)
                                        dacc[e] = pl == 0 ? raw[e] * yv[0] : __builtin_fmaf(raw[e], yv[pl], dacc[e]);
                                }
                            }
                            SP::split(float4{av[0], av[1], av[2], av[3]}, float4{av[4], av[5], av[6], av[7]}, ax[u % 3]);
                            const SPT (&b)[CG][NS > 1 ? NS : 1][NP] = bx[u % NBS];
                            const SPT (&a)[NP] = ax[u % 3];
                            if constexpr (item < SK::K0) {
                                constexpr int NA = 1 + (NS > 1 && item < SK::K1 ? 1 : 0) + (NS > 2 && item < SK::K2 ? 1 : 0);
#pragma unroll
                                for (int tt = 0; tt < SP::NT; ++tt)
#pragma unroll
                                    for (int g = 0; g < CG; ++g)
#pragma unroll
                                        for (int j = 0; j < NA; ++j)
                                            acc[g][j] = mfma16x16(a[SP::TA[tt]], b[g][j][SP::TB[tt]], acc[g][j]);
                            } else {
                                constexpr int plane = (item - SK::K0) / SK::KV;
#pragma unroll
                                for (int tt = 0; tt < SP::NT; ++tt) {
                                    if constexpr (CG == 1) {
                                        if (tt & 1)
                                            accv2[plane] = mfma16x16(a[SP::TA[tt]], b[0][0][SP::TB[tt]], accv2[plane]);
                                        else
                                            acc[0][NS + plane] =
                                                mfma16x16(a[SP::TA[tt]], b[0][0][SP::TB[tt]], acc[0][NS + plane]);
                                    } else {
#pragma unroll
                                        for (int g = 0; g < CG; ++g)
                                            acc[g][NS + plane] =
                                                mfma16x16(a[SP::TA[tt]], b[g][0][SP::TB[tt]], acc[g][NS + plane]);
                                    }
                                }
                            }
                            // position u-1's operands may be reused from here on
                            if constexpr (u > 0) {
                                constexpr int pu = (u + 2) % 3, pitem = TS::item(pos - 1);   // position u-1's set
                                constexpr int PNA = pitem < SK::K0 ? 1 + (NS > 1 && pitem < SK::K1 ? 1 : 0) +
                                                                         (NS > 2 && pitem < SK::K2 ? 1 : 0)
                                                                   : 1;
#pragma unroll
                                for (int p3 = 0; p3 < NP; ++p3) keep(ax[pu][p3]);
                                if constexpr (NBS == 3) {
#pragma unroll
                                    for (int g = 0; g < CG; ++g)
#pragma unroll
                                        for (int j = 0; j < PNA; ++j)
#pragma unroll
                                            for (int p3 = 0; p3 < NP; ++p3) keep(bx[pu][g][j][p3]);
                                }
                            }
                            __builtin_amdgcn_sched_barrier(0);
                        });
                        // the last item's operands are free after one wait state: the gfx950 hazard
                        // (DESIGN.md "gfx950 MFMA SrcA hazard", tools/hazard/mfma_war.hip) is a load
                        // into the SrcA of the v_mfma_f32_16x16x32_bf16 issued in the slot before it
                        asm volatile("s_nop 0" ::: "memory");
                        static_for<0, PF - 1>([&](auto uc) {
                            constexpr int u = decltype(uc)::value;
                            if constexpr (u < nld)
                                load_item(std::integral_constant<int, TS::item(TS::lpos(TS::lidx(lo) + u))>{}, next_rt,
                                          ring[u % PF]);
                        });
                    });
                    if constexpr (CG == 1 && NV)
#pragma unroll
                        for (int pl = 0; pl < 3; ++pl) acc[0][NS + pl] += accv2[pl];
                }
            } else if (SK::on && rt < row_tiles) {
                if constexpr (SK::on) {
                    slice_call([&](auto sc_) {
                        constexpr int lo = decltype(sc_)::value * SNIT / KS;
                        constexpr int n = (decltype(sc_)::value + 1) * SNIT / KS - lo;
                        static_for<0, n>([&](auto uc) {
                            constexpr int u = decltype(uc)::value;
                            if constexpr (u + PF - 1 < n)
                                load_item(std::integral_constant<int, lo + u + PF - 1>{}, rt, ring[(u + PF - 1) % PF]);
                            __builtin_amdgcn_sched_barrier(0);
                            compute_item(std::integral_constant<int, lo + u>{}, ring[u % PF]);
                            __builtin_amdgcn_sched_barrier(0);
                        });
                        // the next tile's first chunks, behind this tile's epilogue
                        static_for<0, PF - 1>([&](auto uc) {
                            constexpr int u = decltype(uc)::value;
                            if constexpr (u < n) load_item(std::integral_constant<int, lo + u>{}, next_rt, ring[u % PF]);
                        });
                    });
                    if constexpr (CG == 1 && NV)
#pragma unroll
                        for (int pl = 0; pl < 3; ++pl) acc[0][NS + pl] += accv2[pl];
                }
            } else if (!SK::on && rt < row_tiles) {
                // sched_barrier keeps each prefetch issued ahead of the MFMAs that follow it
                for (int u0 = 0; u0 < nc_pad; u0 += PF) {
#pragma unroll
                    for (int u = 0; u < PF; ++u) {
                        int pu = u0 + u + PF - 1, prt = rt;
                        if (pu >= nc_pad) { pu -= nc_pad; prt = next_rt; }
                        load_a(prt, c_lo + pu, ring[(u + PF - 1) % PF]);
                        __builtin_amdgcn_sched_barrier(0);
                        if (u0 + u < nck) chunk(ring[u], c_lo + u0 + u);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }

            if constexpr (KS > 1) {   // fold the K slices into slice 0 through LDS
                __syncthreads();
                if (slice > 0) {
                    float* dst = kred + ((tslot * (KS - 1) + slice - 1) * NACC) * 256;
#pragma unroll
                    for (int g = 0; g < CG; ++g)
#pragma unroll
                        for (int j = 0; j < NS + 3 * NV; ++j)
                            *reinterpret_cast<floatx4*>(dst + (g * (NS + 3 * NV) + j) * 256 + 4 * lane) = acc[g][j];
                }
                __syncthreads();
                if (slice == 0) {
#pragma unroll
                    for (int s2 = 1; s2 < KS; ++s2) {
                        const float* src = kred + ((tslot * (KS - 1) + s2 - 1) * NACC) * 256;
#pragma unroll
                        for (int g = 0; g < CG; ++g)
#pragma unroll
                            for (int j = 0; j < NS + 3 * NV; ++j)
                                acc[g][j] += *reinterpret_cast<const floatx4*>(src + (g * (NS + 3 * NV) + j) * 256 +
                                                                              4 * lane);
                    }
                }
            }

            if constexpr (SK::PREC == 2) {   // undo the fp16x2 image's weight scale; range guard
                float z = 0.f;
#pragma unroll
                for (int g = 0; g < CG; ++g)
#pragma unroll
                    for (int j = 0; j < NS + 3 * NV; ++j) {
                        acc[g][j] *= P.bscale;
#pragma unroll
                        for (int e = 0; e < 4; ++e) z = tp_nonfinite_fold(z, acc[g][j][e]);
                    }
                tp_range_flag(P.range_flag, z);
            }
            if (P.dbg) { const unsigned long long c = clock64(); c_loop += c - c_mark; c_mark = c; }
            // ------------------------------------------------------------ epilogue
            const int row0 = rt * 16 + 4 * qd;   // rows of registers 0..3: row0 + jj
#pragma unroll
            for (int g = 0; g < CG; ++g) {
                if (slice != 0 || rt >= row_tiles) break;
                const int ch = (cgroup * CG + g) * 16 + c16;
                const int M = P.M;
                if constexpr (EPI == TP_PLAIN) {
#pragma unroll
                    for (int j = 0; j < NS; ++j) {
                        const bool pm = P.col_part_stride > 0;
                        const int col = pm ? (P.col_part0 + j) * P.col_part_stride + ch
                                           : ((cgroup * CG + g) * NS + j) * 16 + c16;
                        if (pm ? ch < M : col < P.ncols)
#pragma unroll
                            for (int jj = 0; jj < 4; ++jj)
                                if (row0 + jj < P.rows) st_out<false>(&P.C[(size_t)(row0 + jj) * P.ldc + col], acc[g][j][jj]);
                    }
                } else if constexpr (EPI == TP_MSG) {
                    const bool live = ch < M;
                    const float ba = live ? P.bias[ch] : 0.f, bg = live ? P.bias[M + ch] : 0.f;
                    float ms[4], m0[4], m1[4], m2[4];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) {
                        const int row = row0 + jj;
                        const float* gm = P.geom + (size_t)(row < P.rows ? row : 0) * 8;
                        const bool ok = live && row < P.rows && (row & (P.group - 1)) < P.valid_per_group &&
                                        gm[3] >= 0.f;   // |rel| < 0: a general graph's padding slot
                        const float s = kC_SILU * tp_silu(acc[g][0][jj] + ba);
                        const float gg = kC_SIGMOID * tp_sigmoid(acc[g][1][jj] + bg);
                        const float tt = acc[g][2][jj];
                        ms[jj] = ok ? s : 0.f;
                        m0[jj] = ok ? gg * (gm[0] * tt + acc[g][NS + 0][jj]) : 0.f;
                        m1[jj] = ok ? gg * (gm[1] * tt + acc[g][NS + 1][jj]) : 0.f;
                        m2[jj] = ok ? gg * (gm[2] * tt + acc[g][NS + 2][jj]) : 0.f;
                        st0[g] += (double)ms[jj];
                        st1[g] += (double)ms[jj] * ms[jj];
                        st2[g] += (double)m0[jj] * m0[jj] + (double)m1[jj] * m1[jj] + (double)m2[jj] * m2[jj];
                    }
                    const int G = P.group;
                    const int lg = __builtin_ctz((unsigned)G);
                    auto put = [&](int row, float a0, float a1, float a2, float a3) {
                        if (live && row < P.rows) {
                            const size_t o = (size_t)(row >> lg) * M + ch;
                            st_out<false>(&P.out_s[o], a0);
                            st_out<false>(&P.out_v[o], a1);
                            st_out<false>(&P.out_v[P.out_plane + o], a2);
                            st_out<false>(&P.out_v[2 * P.out_plane + o], a3);
                        }
                    };
                    if (G <= 4) {
#pragma unroll
                        for (int s0 = 0; s0 < 4; ++s0) {
                            if (s0 % G) continue;
                            float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                if (s0 + u >= 4 || u >= G) continue;
                                a0 += ms[s0 + u]; a1 += m0[s0 + u]; a2 += m1[s0 + u]; a3 += m2[s0 + u];
                            }
                            put(row0 + s0, a0, a1, a2, a3);
                        }
                    } else {  // G = 8 or 16: lanes qd and qd^1 (^2) hold the other rows of the group
                        float a0 = ms[0] + ms[1] + ms[2] + ms[3], a1 = m0[0] + m0[1] + m0[2] + m0[3];
                        float a2 = m1[0] + m1[1] + m1[2] + m1[3], a3 = m2[0] + m2[1] + m2[2] + m2[3];
                        a0 += __shfl_xor(a0, 16); a1 += __shfl_xor(a1, 16);
                        a2 += __shfl_xor(a2, 16); a3 += __shfl_xor(a3, 16);
                        if (G == 16) {
                            a0 += __shfl_xor(a0, 32); a1 += __shfl_xor(a1, 32);
                            a2 += __shfl_xor(a2, 32); a3 += __shfl_xor(a3, 32);
                        }
                        if ((qd & (G / 4 - 1)) == 0) put(row0, a0, a1, a2, a3);
                    }
                } else if constexpr (EPI == TP_GATE_NODE) {
                    const bool live = ch < M;
                    const float ba = live ? P.bias[ch] : 0.f, bg = live ? P.bias[M + ch] : 0.f;
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) {
                        const int row = row0 + jj;
                        if (!live || row >= P.rows) continue;
                        const float* na = P.geom + (size_t)row * 4;
                        const float hs = kC_SILU * tp_silu(acc[g][0][jj] + ba);
                        const float gg = kC_SIGMOID * tp_sigmoid(acc[g][1][jj] + bg);
                        const float tt = acc[g][2][jj];
                        const float h0 = gg * (na[1] * tt + acc[g][NS + 0][jj]);
                        const float h1 = gg * (na[2] * tt + acc[g][NS + 1][jj]);
                        const float h2 = gg * (na[3] * tt + acc[g][NS + 2][jj]);
                        st_out<false>(&P.out_s[(size_t)row * 2 * M + ch], hs);
                        if (!P.skip_gate_dot)
                            st_out<false>(&P.out_s[(size_t)row * 2 * M + M + ch], fmaf(h2, na[3], fmaf(h1, na[2], h0 * na[1])));
                        st_out<false>(&P.out_v[(size_t)row * M + ch], h0);
                        st_out<false>(&P.out_v[P.out_plane + (size_t)row * M + ch], h1);
                        st_out<false>(&P.out_v[2 * P.out_plane + (size_t)row * M + ch], h2);
                    }
                } else if constexpr (EPI == TP_RESID) {
                    const bool live = ch < M;
                    const float b = live ? P.bias[ch] : 0.f;
                    // the residual X still carries the previous layer's pending BatchNorm
                    const float xs_sc = live && P.xcoef ? P.xcoef[ch] : 1.f;
                    const float xv_sc = live && P.xcoef ? P.xcoef[M + ch] : 1.f;
                    const float xs_sh = live && P.xcoef ? P.xcoef[2 * M + ch] : 0.f;
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) {
                        const int row = row0 + jj;
                        if (!live || row >= P.rows) continue;
                        const float* na = rna[jj] - 1;   // na[1..3]
                        const float tt = acc[g][1][jj];
                        float* xs = P.out_s + (size_t)row * M + ch;
                        const float s = fmaf(xs_sc, rres[g][jj][0], xs_sh) + (acc[g][0][jj] + b);
                        st_out<true>(xs, s);
                        float* x0 = P.out_v + (size_t)row * M + ch;
                        float* x1 = x0 + P.out_plane;
                        float* x2 = x1 + P.out_plane;
                        const float v0 = xv_sc * rres[g][jj][1] + (na[1] * tt + acc[g][NS + 0][jj]);
                        const float v1 = xv_sc * rres[g][jj][2] + (na[2] * tt + acc[g][NS + 1][jj]);
                        const float v2 = xv_sc * rres[g][jj][3] + (na[3] * tt + acc[g][NS + 2][jj]);
                        if (P.out_dot) st_out<true>(&P.out_dot[(size_t)row * M + ch], fmaf(v2, na[3], fmaf(v1, na[2], v0 * na[1])));
                        st_out<true>(x0, v0); st_out<true>(x1, v1); st_out<true>(x2, v2);
                        st0[g] += (double)s;
                        st1[g] += (double)s * s;
                        st2[g] += (double)v0 * v0 + (double)v1 * v1 + (double)v2 * v2;
                    }
                }
            }
            if (P.dbg) { const unsigned long long c = clock64(); c_epi += c - c_mark; c_mark = c; }
            rt = next_rt;
        }
    }
    if (P.dbg && lane == 0) {
        unsigned long long* d = P.dbg + ((size_t)bidx * WAVES + wave) * 6;
        // [start, staged, sum over tiles of the K loop, sum over tiles of the epilogue, wall start]
        d[0] = c_start; d[1] = c_staged; d[2] = c_loop; d[3] = c_epi; d[4] = w_start;
    }
    if constexpr (EPI == TP_MSG || EPI == TP_RESID) {
        // reduce the 8 waves of the block in LDS (the weights are no longer needed), one
        // partial row per block: layout [chunk16][block][3][16]
        __syncthreads();
        double* red = reinterpret_cast<double*>(lds);   // [CG][3][8 waves][16]
#pragma unroll
        for (int g = 0; g < CG; ++g) {
            double a = st0[g], b = st1[g], c = st2[g];
            a += __shfl_xor(a, 16); b += __shfl_xor(b, 16); c += __shfl_xor(c, 16);
            a += __shfl_xor(a, 32); b += __shfl_xor(b, 32); c += __shfl_xor(c, 32);
            if (qd == 0) {
                red[((g * 3 + 0) * WAVES + wave) * 16 + c16] = a;
                red[((g * 3 + 1) * WAVES + wave) * 16 + c16] = b;
                red[((g * 3 + 2) * WAVES + wave) * 16 + c16] = c;
            }
        }
        __syncthreads();
        if (t < CG * 3 * 16) {
            const int g = t / 48, st = (t / 16) % 3, c = t % 16;
            double acc = 0.0;
            for (int w = 0; w < WAVES; ++w) acc += red[((g * 3 + st) * WAVES + w) * 16 + c];
            const int ch16 = cgroup * CG + g;
            if (P.bn_sums) {
                const int ch = ch16 * 16 + c;
                if (ch16 < nchunks16 && ch < P.M) bn_atomic_add(P.bn_sums + st * P.M + ch, acc);
            } else if (ch16 < nchunks16) {
                P.partial[((size_t)ch16 * P.blocks_per_chunk + blk) * 48 + st * 16 + c] = acc;
            }
        }
    }
    if (P.dbg && lane == 0) P.dbg[((size_t)bidx * WAVES + wave) * 6 + 5] = wall_clock64();   // wall end
}

template <int CG>
inline int tp16_lds_floats(const TpProb& p) { return tp_img_floats(p, 16) * CG; }

// geometry of one problem: fills p.lds_floats / blocks_per_chunk, returns the block count
// prec 1: bf16x3 images (1.5x the floats of the fp32 ones)
template <int NS, int NV, int EPI, int CG, int WAVES, int KS>
int tp16_geom(TpProb& p, int num_cus, int* blocks, int prec = 0) {
    p.NS = NS;
    p.NV = NV;
    p.epi = EPI;
    *blocks = 0;
    if (p.rows <= 0 || p.chunks <= 0) return NBX_OK;
    if ((double)p.rows * p.lda_s * 4.0 >= 2147483632.0 ||
        (p.NV && ((double)p.plane_stride * 3 + (double)p.rows * p.lda_v) * 4.0 >= 2147483632.0)) {
        set_error("tp: A operand spans >= 2 GiB (32-bit buffer offsets)");
        return NBX_E_UNSUPPORTED;
    }
    for (int j = 1; j < NS; ++j)
        if (p.K[j] > p.K[j - 1]) {
            set_error("tp16: scalar sub-tile K must be non-increasing");
            return NBX_E_INVAL;
        }
    p.img_floats = tp_img_floats(p, 16) * (prec == 1 ? 3 : 2) / 2;   // bf16x3: 1.5x the fp32 floats; fp16x2: the same
    p.lds_floats = p.img_floats * CG + (p.seg_s[0] ? ((10 * p.M + 3) & ~3) : 0);
    if (KS > 1) p.lds_floats += (WAVES / KS) * (KS - 1) * CG * (NS + 3 * NV) * 4 * 64;
    const size_t lds = (size_t)p.lds_floats * 4;
    if (lds > 160 * 1024) {
        set_error("tp16: weight chunk group needs %zu bytes of LDS (> 160 KiB)", lds);
        return NBX_E_UNSUPPORTED;
    }
    const int groups = (p.chunks + CG - 1) / CG;
    int per_cu = (int)((160 * 1024) / lds);
    if (per_cu > 16 / WAVES) per_cu = 16 / WAVES;
    if (per_cu < 1) per_cu = 1;
    const int row_tiles = (p.rows + 15) / 16;
    int bpc = (num_cus * per_cu + groups - 1) / groups;
    const int max_bpc = (row_tiles + WAVES / KS - 1) / (WAVES / KS);
    if (bpc > max_bpc) bpc = max_bpc;
    if (bpc < 1) bpc = 1;
    p.blocks_per_chunk = bpc;
    p.waves_per_chunk = bpc;  // partial rows per chunk (one per block)
    p.xcd_groups = (groups > 1 && bpc % 8 == 0) ? groups : 0;
    *blocks = groups * bpc;
    return NBX_OK;
}

template <class SK>
int tp16_check_static(const TpProb& p) {
    if constexpr (SK::on) {
        auto kc = [](int K) { return (K + 31) / 32; };
        const bool ok = kc(p.K[0]) == SK::K0 && (p.NS < 2 || kc(p.K[1]) == SK::K1) &&
                        (p.NS < 3 || kc(p.K[2]) == SK::K2) && (p.NV ? kc(p.Kv) : 0) == SK::KV;
        if (!ok) {
            set_error("tp16: static chunk schedule does not match the problem's K");
            return NBX_E_INVAL;
        }
        if (SK::SEG == 2 && (p.M * 2 != SK::K0 * 32 || p.M != SK::KV * 32 || !p.seg_s[0] || !p.seg_s[1] ||
                             !p.seg_v[0])) {
            set_error("tp16: segmented pre_pool input needs mul %% 32 == 0 and the segment pointers");
            return NBX_E_INVAL;
        }
        if (SK::SEG == 4 && (p.M * 4 != SK::K0 * 32 || (SK::KV && p.M * 2 != SK::KV * 32) || !p.seg_s[0] ||
                             !p.seg_s[1] || !p.seg_s[2] || !p.seg_s[3] || (SK::KV && (!p.seg_v[0] || !p.seg_v[1])) ||
                             (!p.mcoef && !p.mbn.sums))) {
            set_error("tp16: segmented update input needs mul %% 32 == 0 and all segment pointers");
            return NBX_E_INVAL;
        }
    }
    return NBX_OK;
}

// segmented input (StatSK SEG > 0): one buffer resource over every segment -- the lowest segment
// pointer and each segment's byte offset from it (all segments live in one workspace)
inline int tp16_seg_prepare(TpProb& p) {
    if (!p.seg_s[0]) return NBX_OK;
    const float* ptrs[6] = {p.seg_s[0], p.seg_s[1], p.seg_s[2], p.seg_s[3], p.seg_v[0], p.seg_v[1]};
    const float* base = nullptr;
    for (const float* q : ptrs)
        if (q && (!base || q < base)) base = q;
    p.seg_base = base;
    for (int i = 0; i < 6; ++i) {
        const long long off = ptrs[i] ? (long long)((const char*)ptrs[i] - (const char*)base) : 0;
        const long long end = off + (long long)(i >= 4 ? 3 : 1) * p.seg_vplane * 4;
        if (end >= 0x7FFFFFF0LL) {
            set_error("tp16: segmented input spans >= 2 GiB (32-bit buffer offsets)");
            return NBX_E_UNSUPPORTED;
        }
        p.seg_boff[i] = (unsigned)off;
    }
    return NBX_OK;
}

template <int NS, int NV, int EPI, int CG, int WAVES, int PF, int KS, bool DUAL, class SK = DynSK>
int tp16_go(TpProb& p0, TpProb& p1, int b0, int b1, hipStream_t st) {
    if (b0 + b1 == 0) return NBX_OK;
    if constexpr (SK::SEG > 0) {
        if (int rc = tp16_seg_prepare(p0)) return rc;
        if (DUAL)
            if (int rc = tp16_seg_prepare(p1)) return rc;
    }
    if (int rc = tp16_check_static<SK>(p0)) return rc;
    if (DUAL)
        if (int rc = tp16_check_static<SK>(p1)) return rc;
    NBX_LDS_160K((tp16_kernel<NS, NV, EPI, CG, WAVES, PF, KS, DUAL, SK>));
    const size_t lds = (size_t)std::max(b0 ? p0.lds_floats : 0, b1 ? p1.lds_floats : 0) * 4;
    NBX_TIMED_LAUNCH((tp16_kernel<NS, NV, EPI, CG, WAVES, PF, KS, DUAL, SK>), dim3(b0 + b1), dim3(64 * WAVES), lds,
                     st, p0, p1, b0);
    NBX_HIP(hipGetLastError());
    return NBX_OK;
}

// p.chunks = number of 16-channel chunks; grid = ceil(chunks / CG) groups x blocks_per_chunk
template <int NS, int NV, int EPI, int CG, int WAVES = T16_WAVES, int PF = 3, int KS = 1, class SK = DynSK>
int tp16_launch(TpProb& p, hipStream_t st, int num_cus = 256) {
    int b = 0;
    if (int rc = tp16_geom<NS, NV, EPI, CG, WAVES, KS>(p, num_cus, &b, SK::PREC)) return rc;
    return tp16_go<NS, NV, EPI, CG, WAVES, PF, KS, false, SK>(p, p, b, 0, st);
}

// two independent problems in one launch (same template shape)
template <int NS, int NV, int EPI, int CG, int WAVES = T16_WAVES, int PF = 3, int KS = 1>
int tp16_launch2(TpProb& p0, TpProb& p1, hipStream_t st, int num_cus = 256) {
    int b0 = 0, b1 = 0;
    if (int rc = tp16_geom<NS, NV, EPI, CG, WAVES, KS>(p0, num_cus, &b0)) return rc;
    if (int rc = tp16_geom<NS, NV, EPI, CG, WAVES, KS>(p1, num_cus, &b1)) return rc;
    p0.xcd_groups = p1.xcd_groups = 0;   // the second problem's blocks start at an arbitrary id
    return tp16_go<NS, NV, EPI, CG, WAVES, PF, KS, true>(p0, p1, b0, b1, st);
}

}  // namespace nbx
