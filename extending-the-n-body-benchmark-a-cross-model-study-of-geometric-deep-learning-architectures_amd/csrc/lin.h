// Generic weight-stationary fp32 linear layer on CDNA4 matrix cores:
//   Y[row, n] = epilogue( sum_k A[row, k] * Wt[n, k] )
// where A is the concatenation along K of up to 3 segments, each optionally
// gathered through a per-row index (EGNN edge inputs [h_row | h_col | radial, attrs]).
//
// A block owns NT x 32 output columns: that slice of Wt is staged in LDS once
// (zero-padded, pitch = 32k + 4 floats) and its 8 waves stream 32-row tiles of A
// from global memory (3-deep register prefetch, no barrier in the main loop)
// through v_mfma_f32_32x32x2_f32.  Epilogues: bias, activation (SiLU / exact
// GELU / tanh), optional residual "Y = R + s (.) act(...)" and optional
// accumulate of a per-row dot product with a vector (EGNN's 128 -> 1 heads).
// LIN_CONV instead multiplies each output by a gathered source feature and sums
// groups of G consecutive rows in registers (PONITA's message aggregation).
// Fragment maps and the in-chunk K permutation are those of tp_fused.h.
#pragma once
#include "nbx_internal.h"
#include "tp_fused.h"   // bf16x3 split helpers, LDS-DMA image staging

namespace nbx {

enum LinAct : int { ACT_NONE = 0, ACT_SILU = 1, ACT_GELU = 2, ACT_TANH = 3 };
enum LinEpi : int { LIN_STORE = 0, LIN_CONV = 1, LIN_EQMSG = 2, LIN_LNSILU = 3 };

struct LinSeg {
    const float* ptr;   // segment base
    const int64_t* idx; // optional row gather index (row -> source row), else identity
    int ld;             // row stride (floats)
    int K;              // padded width (multiple of 32) occupied in the concatenated K
    int Kvalid;         // real columns (multiple of 4); the rest reads as zero
};

struct LinProb {
    LinSeg seg[3];
    int nseg;
    int rows, N, Ktot;  // Ktot = sum of seg[].K
    const float* Wt;    // [N][ldw]  (columns of the concatenated K)
    int ldw;
    // optional split-precision (bf16x3) image of Wt (include/nbx.h "bf16x3 images", CW = 32, one
    // sub-tile): [N/32 column tiles][Ktot/32 chunks][part 3][m 2][lane 64][8] bf16; when set (and N %
    // 32 == 0) lin_auto runs the PREC = 1 kernel: fp32-accurate products on v_mfma_f32_32x32x16_bf16
    const void* Wx3;
    // optional fp16x2 image of Wt (include/nbx.h "fp16x2 images", the Wx3 layout with two fp16 parts,
    // W s = hi + lo) with h2_sinv = 1 / s: lin_auto runs the PREC = 2 kernel (three fp16 products per fp32
    // product); range_flag: the call's fp16x2 range flag (tp_fused.h tp_range_flag), or null
    const void* Wh2;
    float h2_sinv;
    int* range_flag;
    const float* bias;  // [N] or null
    float* Y;           // [rows][ldy] (may be null when only the row dot is wanted)
    int ldy;
    const float* resid; // optional residual R [rows][ldr] (may alias Y)
    int ldr;
    const float* scale; // optional per-column scale s (layer_scale)
    const float* dotw;  // optional: rowdot[row] += sum_n act(...)[n] * dotw[n]
    float* rowdot;      // [rows] accumulated with atomics across column blocks (zero it first)
    // LIN_CONV (PONITA FiberBundleConv spatial part on a fully-connected graph): rows are
    // (d, o, q) with G >= N-1 edge slots q per (node d, orientation o), slot q < N-1 holding the
    // message from src(d, q) = system base + (q < d ? q : q + 1);
    // Y[(d*O + o), n] = sum_q acc[(d, o, q), n] * X[(src(d, q)*O + o), n]
    int conv_G, conv_O, conv_nodes;  // slots per (d,o) (power of two <= 32), orientations, N
    const int* conv_slot;            // general graphs: [V][G] source (local index) per slot, -1 padding; null = FC
    const float* conv_x;             // [V*O][ldx]
    int conv_ldx;
    int blocks_per_chunk;
    int chunks;         // ceil(N / (NT*32))
    // LIN_EQMSG (EquiformerV2 SO(2)-conv input, eqv2.hip): rows are edges of fully-connected systems of
    // eq_nodes nodes; the block's 5 column tiles are the radial-function outputs of one 32-channel block
    // of the message [x_src | x_dst] for the 5 groups (m=0: l=0,1,2; m=1: l=1,2).  The epilogue rotates
    // the gathered node irreps into the edge frame (eq_rot: R rows, D^2 rows m=-1,0,1) and writes
    // rad * message to eq_a0 [rows][3 * 2C] (m = 0) and eq_a1 [2 rows][2 * 2C] (m = +1 row, m = -1 row).
    const float* eq_x;  // [V][9][C]
    const float* eq_rot;
    float* eq_a0;
    float* eq_a1;
    int eq_C, eq_nodes;
    // LIN_LNSILU: Y = SiLU(LayerNorm(acc + bias) * ln_w + ln_b) over the row's N = NT * 32 columns
    // (one column chunk), eps 1e-5 (EquiformerV2 RadialFunction hidden layers)
    const float* ln_w;
    const float* ln_b;
    // set by lin_launch: block b runs logical block (b % 8) * (nblocks / 8) + b / 8, so the blocks of a
    // contiguous row range share one XCD (b % 8) and its L2 -- the gathering LIN_CONV epilogue then
    // fetches a system's source rows into one L2 instead of one per neighbouring block
    int xcd_remap;
};

constexpr int LIN_WAVES = 8, LIN_THREADS = 64 * LIN_WAVES;

__device__ inline float lin_act(float x, int act) {
    switch (act) {
        case ACT_SILU: return x / (1.0f + __expf(-x));
        case ACT_GELU: return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
        case ACT_TANH: return tanhf(x);
        default: return x;
    }
}

// PREC 0: fp32 v_mfma_f32_32x32x2_f32 with the Wt slice staged row-major (pitch 32k + 4).
// PREC 1: the split-precision path (tp_fused.h StatSKX3): the block's NT column tiles of the bf16x3
// image are copied verbatim into LDS by LDS-DMA; every A chunk is split into hi + mid + lo bf16 as
// it is consumed (once per chunk, shared by the NT column tiles) and each 32 x 32 x 32 block is
// the fp32 sum of the six leading cross products on v_mfma_f32_32x32x16_bf16 (12 x 32 cycles
// instead of 16 x 64).
constexpr int LIN_X3_BLK = 1536;   // floats of one (column tile, 32-deep chunk) bf16x3 block
constexpr int LIN_H2_BLK = 1024;   // the same block of an fp16x2 image (two fp16 parts)

template <int NT, int ACT, int EPI = LIN_STORE, int PREC = 0>
__global__ __launch_bounds__(LIN_THREADS, 2) void lin_kernel(const LinProb P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int bid = P.xcd_remap ? ((int)blockIdx.x & 7) * ((int)gridDim.x >> 3) + ((int)blockIdx.x >> 3) : (int)blockIdx.x;
    const int chunk = bid / P.blocks_per_chunk;
    const int blk = bid - chunk * P.blocks_per_chunk;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, r = lane & 31, h = lane >> 5;
    const int pitch = ((P.Ktot + 31) & ~31) + 4;
    const int n0 = chunk * NT * 32;
    const int n_chunks = P.Ktot >> 5;

    constexpr int BLK = PREC == 2 ? LIN_H2_BLK : LIN_X3_BLK;
    if constexpr (PREC >= 1) {
        // ---- stage the block's column tiles of the bf16x3 / fp16x2 image (contiguous) in LDS
        const int tiles = min(NT, (P.N >> 5) - chunk * NT);
        tp_dma_image<LIN_WAVES>(reinterpret_cast<const float*>(PREC == 2 ? P.Wh2 : P.Wx3) + (size_t)chunk * NT * n_chunks * BLK,
                                lds, tiles * n_chunks * BLK);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        // ---- stage Wt[n0 : n0 + NT*32, :] in LDS
        const int q4 = pitch / 4;
        for (int i = t; i < NT * 32 * q4; i += LIN_THREADS) {
            const int row = i / q4, kq = (i - row * q4) * 4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (n0 + row < P.N && kq < P.Ktot)
                v = *reinterpret_cast<const float4*>(P.Wt + (size_t)(n0 + row) * P.ldw + kq);
            *reinterpret_cast<float4*>(&lds[row * pitch + kq]) = v;
        }
    }
    __syncthreads();

    const int row_tiles = (P.rows + 31) >> 5;
    const int wstride = P.blocks_per_chunk * LIN_WAVES;

    // Segment table hoisted into (scalar) registers: the hot loop never indexes the kernel
    // argument array (a dynamic P.seg[s] is an s_load, and its lgkmcnt wait would also drain
    // the LDS reads in flight).
    const int nseg = P.nseg;
    const float* sp0 = P.seg[0].ptr;
    const float* sp1 = nseg > 1 ? P.seg[1].ptr : sp0;
    const float* sp2 = nseg > 2 ? P.seg[2].ptr : sp1;
    const int64_t* si0 = P.seg[0].idx;
    const int64_t* si1 = nseg > 1 ? P.seg[1].idx : nullptr;
    const int64_t* si2 = nseg > 2 ? P.seg[2].idx : nullptr;
    const int sl0 = P.seg[0].ld, sl1 = nseg > 1 ? P.seg[1].ld : 0, sl2 = nseg > 2 ? P.seg[2].ld : 0;
    const int kv0 = P.seg[0].Kvalid, kv1 = nseg > 1 ? P.seg[1].Kvalid : 0, kv2 = nseg > 2 ? P.seg[2].Kvalid : 0;
    const int ce0 = P.seg[0].K >> 5;                               // chunk ends of segments 0 and 1
    const int ce1 = ce0 + (nseg > 1 ? P.seg[1].K >> 5 : 0);

    // per-tile source rows of the (up to 3) segments; gathered segments read their index once
    // per tile.  Plain scalars (no struct / reference captures) keep them in registers.
    auto tile_rows = [&](int rt, int64_t& s0, int64_t& s1, int64_t& s2, bool& ok) {
        const int row = rt * 32 + r;
        ok = row < P.rows;
        const int64_t rr = ok ? row : 0;
        s0 = si0 ? si0[rr] : rr;
        s1 = si1 ? si1[rr] : rr;
        s2 = si2 ? si2[rr] : rr;
    };
    // A chunk loader: 32-deep K chunk i of a tile -> 16 floats per lane
    auto load_a = [&](int64_t s0, int64_t s1, int64_t s2, bool ok, int i, float4 (&a)[4]) {
        // segment select by arithmetic (a ternary chain gets turned into a scratch lookup table)
        const int g1 = i >= ce0 ? 1 : 0, g2 = i >= ce1 ? 1 : 0;
        const int k0 = (i - g1 * ce0 - g2 * (ce1 - ce0)) * 32;
        const float* base = sp0 + g1 * (sp1 - sp0) + g2 * (sp2 - sp1);
        const int64_t src = s0 + g1 * (s1 - s0) + g2 * (s2 - s1);
        const int ld = sl0 + g1 * (sl1 - sl0) + g2 * (sl2 - sl1);
        const int kvalid = kv0 + g1 * (kv1 - kv0) + g2 * (kv2 - kv1);
        const int kk = k0 + 16 * h;
        // Buffer loads with hardware bounds checking: invalid lanes get an out-of-range offset and
        // read zeros, so every load is issued unconditionally (exec-masked branches around the
        // loads would make the in-flight count unknown to the waitcnt pass and force vmcnt(0)
        // at every use).  Segments are < 2 GiB (checked by lin_launch).
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7FFFFFF0, 0x00020000);
        const uint32_t off = (uint32_t)(((size_t)src * ld + kk) * 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool v = ok && kk + 4 * q < kvalid;
            a[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, v ? off + 16 * q : 0x7FFFFFF0u, 0, 0));
        }
    };

    // A streams in steps of SUP 32-deep chunks: two chunks for the fp16x2 gathering convolution (8 KB per
    // wave in flight behind the step being consumed instead of 4 KB: C3's spatial conv 500 -> 478 us,
    // profiles/r06/lin_sup), otherwise one (EquiformerV2's so2_conv_2 GEMMs measured 64 -> 70 us with
    // two).  A step past the last chunk loads zeros (out-of-range offsets) and is not consumed.
    constexpr int SUP = (PREC == 2 && EPI == LIN_CONV) ? 2 : 1;
    const int n_steps = (n_chunks + SUP - 1) / SUP;
    auto load_s = [&](int64_t s0, int64_t s1, int64_t s2, bool ok, int st, float4 (&a)[4 * SUP]) {
#pragma unroll
        for (int u = 0; u < SUP; ++u)
            load_a(s0, s1, s2, ok, SUP * st + u, *reinterpret_cast<float4(*)[4]>(&a[4 * u]));
    };

    int rt = blk * LIN_WAVES + wave;
    if (rt >= row_tiles) return;
    // A is double-buffered with the two buffers' roles fixed by an unroll-by-2 of the step
    // loop (bA <- even steps, bB <- odd steps), the next tile's step 0 always landing in bA
    // during the current tile's last step.  No register move ever reads a load still in
    // flight, so the waitcnt pass waits only for the step about to be consumed (a
    // cur <- nxt <- nx2 shuffle would force vmcnt(0) on every step).
    float4 bA[4 * SUP], bB[4 * SUP];
    int64_t r0, r1, r2;
    bool rok;
    tile_rows(rt, r0, r1, r2, rok);
    load_s(r0, r1, r2, rok, 0, bA);
    while (true) {
        floatx16 acc[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
        auto consume = [&](const float4 (&cur)[4], int k0) {
            if constexpr (PREC >= 1) {
                // lane (r, h) holds k = 16 h + 4 q + e of the chunk; MFMA m takes k = 16 h + 8 m + j
                using SP = SplitP<PREC>;
                using SPT = typename SP::T;
                SPT a[SP::NP][2];
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    SPT t3[SP::NP];
                    SP::split(cur[2 * m], cur[2 * m + 1], t3);
#pragma unroll
                    for (int p3 = 0; p3 < SP::NP; ++p3) a[p3][m] = t3[p3];
                }
                const SPT* ldsx = reinterpret_cast<const SPT*>(lds);
                const int kc = k0 >> 5;
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    const SPT* bp = ldsx + (j * n_chunks + kc) * (BLK / 4) + lane;
#pragma unroll
                    for (int m = 0; m < 2; ++m) {   // block [part p][m][lane][8]: smallest terms first
                        SPT b[SP::NP];
#pragma unroll
                        for (int p3 = 0; p3 < SP::NP; ++p3) b[p3] = bp[(2 * p3 + m) * 64];
#pragma unroll
                        for (int tt = 0; tt < SP::NT; ++tt) acc[j] = mfma32x32(a[SP::TA[tt]][m], b[SP::TB[tt]], acc[j]);
                    }
                }
                return;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float4 b4[NT];
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    b4[j] = *reinterpret_cast<const float4*>(&lds[(32 * j + r) * pitch + k0 + 16 * h + 4 * q]);
#pragma unroll
                for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].x, b4[j].x, acc[j], 0, 0, 0);
#pragma unroll
                for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].y, b4[j].y, acc[j], 0, 0, 0);
#pragma unroll
                for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].z, b4[j].z, acc[j], 0, 0, 0);
#pragma unroll
                for (int j = 0; j < NT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].w, b4[j].w, acc[j], 0, 0, 0);
            }
        };
        // the chunks of step st (a step's second chunk past the last is skipped, wave-uniform)
        auto consume_s = [&](const float4 (&cur)[4 * SUP], int st) {
#pragma unroll
            for (int u = 0; u < SUP; ++u)
                if (u == 0 || SUP * st + u < n_chunks)
                    consume(*reinterpret_cast<const float4(*)[4]>(&cur[4 * u]), (SUP * st + u) * 32);
        };
        const int nrt = rt + wstride;       // next tile of this wave
        int i = 0;
        int64_t n0r, n1r, n2r;              // next tile's source rows
        bool nok = false;
        // sched_barrier keeps each prefetch issued ahead of the MFMAs that follow it
        for (; i + 1 < n_steps; i += 2) {
            load_s(r0, r1, r2, rok, i + 1, bB);
            __builtin_amdgcn_sched_barrier(0);
            consume_s(bA, i);
            if (i + 2 < n_steps) {
                load_s(r0, r1, r2, rok, i + 2, bA);
            } else if (nrt < row_tiles) {
                tile_rows(nrt, n0r, n1r, n2r, nok);
                load_s(n0r, n1r, n2r, nok, 0, bA);
            }
            __builtin_amdgcn_sched_barrier(0);
            consume_s(bB, i + 1);
        }
        if (i < n_steps) {                  // odd step count: the last step sits in bA
            consume_s(bA, i);
            if (nrt < row_tiles) {
                tile_rows(nrt, n0r, n1r, n2r, nok);
                load_s(n0r, n1r, n2r, nok, 0, bA);
            }
        }
        if constexpr (PREC == 2) {   // undo the image's weight scale; fp16x2 range guard
            float z = 0.f;
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                // (a column tile past N was not staged: its accumulators hold whatever the LDS held and
                // are never stored, so they stay out of the guard)
                const bool live_tile = n0 + 32 * j < P.N;
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    acc[j][e] *= P.h2_sinv;
                    if (live_tile) z = tp_nonfinite_fold(z, acc[j][e]);
                }
            }
            tp_range_flag(P.range_flag, z);
        }
        // ---- epilogue: col = n0 + 32 j + r; row = rt*32 + (e&3) + 8(e>>2) + 4h
        if constexpr (EPI == LIN_EQMSG) {
            static_assert(NT == 5, "LIN_EQMSG: one block = the 5 groups of one 32-channel block");
            const int C = P.eq_C, C2 = 2 * C, NN = P.eq_nodes, deg = NN - 1, per = NN * deg;
            const int ch = chunk * 32 + r;                  // message channel (< C: source node, else target)
            const bool tgt = ch >= C;
            const int cc = tgt ? ch - C : ch;
            float bb[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) bb[j] = P.bias[n0 + 32 * j + r];
            // fully unrolled: every row's gathers (9 x values, 24 rotation entries) can be in flight together
            // (unroll 2 / 4 / 16: 154 / 148 / 137 us per launch at C4, profiles/r06/eqmsg_unroll)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = rt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                if (row >= P.rows) continue;
                const int b = row / per, rr = row - b * per, i = rr / deg, jj = rr - i * deg;
                const int node = b * NN + (tgt ? (jj < i ? jj : jj + 1) : i);
                const float* xp = P.eq_x + (size_t)node * 9 * C + cc;
                float x[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) x[k] = xp[k * C];
                const float* D = P.eq_rot + (size_t)row * 32;
                const float m0 = x[0];
                const float m1 = D[3] * x[1] + D[4] * x[2] + D[5] * x[3];
                const float re1 = D[6] * x[1] + D[7] * x[2] + D[8] * x[3];
                const float im1 = D[0] * x[1] + D[1] * x[2] + D[2] * x[3];
                float im2 = 0.f, m2 = 0.f, re2 = 0.f;
#pragma unroll
                for (int k = 0; k < 5; ++k) {
                    im2 += D[9 + k] * x[4 + k];
                    m2 += D[14 + k] * x[4 + k];
                    re2 += D[19 + k] * x[4 + k];
                }
                float* a0 = P.eq_a0 + (size_t)row * 3 * C2 + ch;
                a0[0] = (acc[0][e] + bb[0]) * m0;
                a0[C2] = (acc[1][e] + bb[1]) * m1;
                a0[2 * C2] = (acc[2][e] + bb[2]) * m2;
                const float r3 = acc[3][e] + bb[3], r4 = acc[4][e] + bb[4];
                float* a1 = P.eq_a1 + (size_t)row * 4 * C2 + ch;
                a1[0] = r3 * re1;
                a1[C2] = r4 * re2;
                a1[2 * C2] = r3 * im1;
                a1[3 * C2] = r4 * im2;
            }
        } else if constexpr (EPI == LIN_LNSILU) {
            float bb[NT], gw[NT], gb[NT];
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                bb[j] = P.bias[32 * j + r];
                gw[j] = P.ln_w[32 * j + r];
                gb[j] = P.ln_b[32 * j + r];
            }
            const float invn = 1.0f / (NT * 32);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = rt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                float y[NT], s = 0.f;
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    y[j] = acc[j][e] + bb[j];
                    s += y[j];
                }
                for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o);   // the 32 lanes of this row
                const float mu = s * invn;
                float q = 0.f;
#pragma unroll
                for (int j = 0; j < NT; ++j) q += (y[j] - mu) * (y[j] - mu);
                for (int o = 16; o > 0; o >>= 1) q += __shfl_xor(q, o);
                const float rs = 1.0f / sqrtf(q * invn + 1e-5f);
                if (row < P.rows)
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        const float z = (y[j] - mu) * rs * gw[j] + gb[j];
                        P.Y[(size_t)row * P.ldy + 32 * j + r] = z * __builtin_amdgcn_rcpf(1.0f + __expf(-z));
                    }
            }
        } else if constexpr (EPI == LIN_CONV) {
            const int G = P.conv_G, O = P.conv_O, NN = P.conv_nodes;
            // gathered source row offset of each accumulator row (-1: padded slot / past the end),
            // shared by all NT column sub-tiles
            int xoff[16];  // host guarantees V*O*ldx < 2^31
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = rt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                const int q = row & (G - 1), dq = row / G, d = dq / O, o = dq - d * O;
                const int dl = d % NN;
                const int sq = row >= P.rows ? -1
                               : P.conv_slot ? P.conv_slot[d * G + q] : (q < NN - 1 ? (q < dl ? q : q + 1) : -1);
                xoff[e] = sq >= 0 ? ((d - dl + sq) * O + o) * P.conv_ldx : -1;
            }
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int col = n0 + 32 * j + r;
                const bool live = col < P.N;
                float xv[16];
#pragma unroll
                for (int e = 0; e < 16; ++e) xv[e] = (live && xoff[e] >= 0) ? P.conv_x[xoff[e] + col] : 0.f;
                float m[16];
#pragma unroll
                for (int e = 0; e < 16; ++e) m[e] = acc[j][e] * xv[e];
                auto put = [&](int row, float a) {
                    if (live && row < P.rows) P.Y[(size_t)(row / G) * P.ldy + col] = a;
                };
                if (G <= 4) {
#pragma unroll
                    for (int e0 = 0; e0 < 16; e0 += 4)
#pragma unroll
                        for (int s0 = 0; s0 < 4; ++s0) {
                            if (s0 % G) continue;
                            float a = 0.f;
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                                if (s0 + u < 4 && u < G) a += m[e0 + s0 + u];
                            put(rt * 32 + s0 + 8 * (e0 >> 2) + 4 * h, a);
                        }
                } else {
                    float b8[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        b8[k] = m[4 * k] + m[4 * k + 1] + m[4 * k + 2] + m[4 * k + 3];
                        b8[k] += __shfl_xor(b8[k], 32);
                    }
                    const int nb = G / 8;
#pragma unroll
                    for (int gb = 0; gb < 4; ++gb) {
                        if (gb % nb) continue;
                        float a = 0.f;
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            if (k >= gb && k < gb + nb) a += b8[k];
                        if (h == 0) put(rt * 32 + 8 * gb, a);
                    }
                }
            }
        } else {
            float dot[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) dot[e] = 0.f;
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int col = n0 + 32 * j + r;
                const bool live = col < P.N;
                const float b = (live && P.bias) ? P.bias[col] : 0.f;
                const float sc = (live && P.scale) ? P.scale[col] : 1.f;
                const float dw = (live && P.dotw) ? P.dotw[col] : 0.f;
                float res[16];   // residual loads batched ahead of their uses
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int row = rt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                    res[e] = (P.resid && live && row < P.rows) ? P.resid[(size_t)row * P.ldr + col] : 0.f;
                }
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int row = rt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                    float y = lin_act(acc[j][e] + b, ACT);
                    dot[e] += y * dw;
                    if (live && row < P.rows && P.Y) {
                        if (P.resid) y = res[e] + sc * y;
                        P.Y[(size_t)row * P.ldy + col] = y;
                    }
                }
            }
            if (P.dotw) {
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    float v = dot[e];
                    for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off);  // sum over the 32 columns
                    const int row = rt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
                    if (r == 0 && row < P.rows) atomicAdd(&P.rowdot[row], v);
                }
            }
        }
        rt += wstride;
        if (rt >= row_tiles) break;
        r0 = n0r; r1 = n1r; r2 = n2r; rok = nok;
    }
}

// LDS bytes of a block's weight slice: fp32 rows with pitch, or NT bf16x3 / fp16x2 column tiles
inline size_t lin_lds_bytes(int nt, int Ktot, int prec) {
    return prec ? (size_t)nt * (Ktot >> 5) * (prec == 2 ? LIN_H2_BLK : LIN_X3_BLK) * 4
                : (size_t)nt * 32 * (((Ktot + 31) & ~31) + 4) * 4;
}

template <int NT, int ACT, int EPI = LIN_STORE, int PREC = 0>
int lin_launch(LinProb& p, hipStream_t st, int num_cus = 256) {
    if (p.rows <= 0 || p.N <= 0) return NBX_OK;
    if (p.Ktot % 32) {
        set_error("lin: Ktot must be a multiple of 32 (got %d)", p.Ktot);
        return NBX_E_INVAL;
    }
    if ((PREC == 1 && !p.Wx3) || (PREC == 2 && !p.Wh2) || (PREC && p.N % 32)) {
        set_error("lin: the split-precision path needs its image and N %% 32 == 0");
        return NBX_E_INVAL;
    }
    for (int s = 0; s < p.nseg; ++s)   // buffer-load offsets are 32-bit, OOB sentinel at 2 GiB
        if (!p.seg[s].idx && (double)p.rows * p.seg[s].ld * 4.0 >= 2147483632.0) {
            set_error("lin: segment %d spans >= 2 GiB", s);
            return NBX_E_UNSUPPORTED;
        }
    const size_t lds = lin_lds_bytes(NT, p.Ktot, PREC);
    if (lds > 160 * 1024) {
        set_error("lin: weight slice needs %zu bytes of LDS", lds);
        return NBX_E_UNSUPPORTED;
    }
    p.chunks = (p.N + NT * 32 - 1) / (NT * 32);
    int per_cu = (int)((160 * 1024) / lds);
    if (per_cu > 2) per_cu = 2;
    if (per_cu < 1) per_cu = 1;
    const int row_tiles = (p.rows + 31) / 32;
    int bpc = (num_cus * per_cu + p.chunks - 1) / p.chunks;
    const int max_bpc = (row_tiles + LIN_WAVES - 1) / LIN_WAVES;
    if (bpc > max_bpc) bpc = max_bpc;
    if (bpc < 1) bpc = 1;
    p.blocks_per_chunk = bpc;
    // XCD-grouped block order for the gathering epilogues (a bijection only when the grid is a
    // multiple of 8 blocks; NBX_LIN_XCD=0 keeps the plain order, A/B)
    static const bool xcd = !(getenv("NBX_LIN_XCD") && getenv("NBX_LIN_XCD")[0] == '0');
    // (LIN_CONV only: C3's spatial conv 1.64 -> 1.39 GB per launch at the same time; EquiformerV2's
    // LIN_EQMSG measured 1 % slower with it, profiles/r04/lin_xcd_ab)
    p.xcd_remap = (xcd && EPI == LIN_CONV && (p.chunks * bpc) % 8 == 0) ? 1 : 0;
    NBX_LDS_160K((lin_kernel<NT, ACT, EPI, PREC>));
    hipLaunchKernelGGL((lin_kernel<NT, ACT, EPI, PREC>), dim3(p.chunks * bpc), dim3(LIN_THREADS), lds, st, p);
    NBX_HIP(hipGetLastError());
    return NBX_OK;
}

// ---------------------------------------------------------------------------------------------------
// Row-panel split-precision GEMM: Y[row, n] = act(sum_k A[row, k] W[n, k] + bias[n]) for ALL
// NTILES * 32 output columns in one workgroup, so A is read from HBM exactly once (the weight-
// stationary lin_kernel re-reads A once per column chunk).  The weights stream through LDS by 32-deep
// K chunk: a chunk-major bf16x3 image [K/32][NTILES][3][2][64][8] bf16 (the "bf16x3 images" blocks
// reordered so one chunk of every column tile is contiguous), double-buffered by LDS-DMA while the
// MFMAs consume the other buffer.  8 waves, one 32-row tile each (a 256-row panel per workgroup).
struct LinRpProb {
    const float* A;
    int lda, rows, K;   // K % 32 == 0
    const void* Wx3;    // chunk-major image
    const float* bias;  // [NTILES * 32] or null
    float* Y;
    int ldy, N;         // N: columns stored (<= NTILES * 32)
    const float* resid; // optional: Y = R + scale (.) act(...)  (R may alias Y)
    int ldr;
    const float* scale; // optional per-column scale (layer_scale)
    // PREC 2 (an fp16x2 image in Wx3's place, W s = hi + lo): h2_sinv = 1 / s; the call's range flag
    float h2_sinv;
    int* range_flag;
};

constexpr int RP_WAVES = 8;

// PREC 1: bf16x3 image blocks (six products per fp32 product); PREC 2: fp16x2 blocks (three)
template <int NTILES, int ACT, int PREC = 1>
__global__ __launch_bounds__(64 * RP_WAVES, 1) void lin_rp_kernel(const LinRpProb P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    using SP = SplitP<PREC>;
    using SPT = typename SP::T;
    constexpr int BLK = PREC == 2 ? LIN_H2_BLK : LIN_X3_BLK;
    constexpr int SLAB = NTILES * BLK;                 // floats of one K chunk of every column tile
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, r = lane & 31, h = lane >> 5;
    const int nk = P.K >> 5;
    const int rt = blockIdx.x * RP_WAVES + wave;
    const int row = rt * 32 + r;
    const bool ok = row < P.rows;
    const float* W = reinterpret_cast<const float*>(P.Wx3);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)P.A, (short)0, 0x7FFFFFF0, 0x00020000);
    const uint32_t base = (uint32_t)(((size_t)(ok ? row : 0) * P.lda + 16 * h) * 4);
    auto load_a = [&](int kc, float4 (&a)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            a[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rs, ok ? base + (uint32_t)(kc * 128 + 16 * q) : 0x7FFFFFF0u, 0, 0));
    };
    floatx16 acc[NTILES];
#pragma unroll
    for (int j = 0; j < NTILES; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
    // one A register buffer: a chunk is split into its parts first, then the next chunk's A load is
    // issued into the same registers and lands while this chunk's MFMAs run
    auto split_a = [&](const float4 (&cur)[4], SPT (&a)[SP::NP][2]) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            SPT t3[SP::NP];
            SP::split(cur[2 * m], cur[2 * m + 1], t3);
#pragma unroll
            for (int p3 = 0; p3 < SP::NP; ++p3) a[p3][m] = t3[p3];
        }
    };
    auto mfmas = [&](const SPT (&a)[SP::NP][2], const float* buf) {
        const SPT* ldsx = reinterpret_cast<const SPT*>(buf);
#pragma unroll
        for (int j = 0; j < NTILES; ++j) {
            const SPT* bp = ldsx + j * (BLK / 4) + lane;
#pragma unroll
            for (int m = 0; m < 2; ++m) {   // smallest terms first (as lin_kernel)
                SPT b[SP::NP];
#pragma unroll
                for (int p3 = 0; p3 < SP::NP; ++p3) b[p3] = bp[(2 * p3 + m) * 64];
#pragma unroll
                for (int tt = 0; tt < SP::NT; ++tt) acc[j] = mfma32x32(a[SP::TA[tt]][m], b[SP::TB[tt]], acc[j]);
            }
        }
    };
    if constexpr (NTILES <= 5 || PREC == 2) {
        // small panels (N <= 160), and any panel on fp16x2 images (2/3 of the bf16x3 slab): three LDS
        // slabs and two A register buffers, both streams issued two chunks ahead.  At the end of chunk kc only chunk kc + 2's slab pieces and A loads may still be
        // in flight: vmcnt(this wave's slab pieces + 4) (the slab pieces per wave are counted so the
        // immediate is exact; a slab is BLK / 256 pieces per column tile).
        const int ndma = ((BLK / 256) * NTILES - wave + RP_WAVES - 1) / RP_WAVES;
        auto wait_all_but_one_chunk = [&]() {
            switch (ndma) {
                case 1: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
                case 2: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
                case 3: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
                case 4: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
                case 5: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
                default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
            }
        };
        float4 bA[4], bB[4];
        tp_dma_image<RP_WAVES>(W, lds, SLAB);
        load_a(0, bA);
        if (nk > 1) {
            tp_dma_image<RP_WAVES>(W + SLAB, lds + SLAB, SLAB);
            load_a(1, bB);
            wait_all_but_one_chunk();
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        auto step = [&](int kc, float4 (&cur)[4]) {
            SPT a[SP::NP][2];
            split_a(cur, a);
            const bool ahead = kc + 2 < nk;
            if (ahead) {
                tp_dma_image<RP_WAVES>(W + (size_t)(kc + 2) * SLAB, lds + ((kc + 2) % 3) * SLAB, SLAB);
                load_a(kc + 2, cur);
            }
            __builtin_amdgcn_sched_barrier(0);
            mfmas(a, lds + (kc % 3) * SLAB);
            if (ahead)
                wait_all_but_one_chunk();
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        };
        for (int kc = 0; kc < nk; kc += 2) {
            step(kc, bA);
            if (kc + 1 < nk) step(kc + 1, bB);
        }
    } else {
        float4 cur[4];
        tp_dma_image<RP_WAVES>(W, lds, SLAB);
        load_a(0, cur);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        for (int kc = 0; kc < nk; ++kc) {
            SPT a[SP::NP][2];
            split_a(cur, a);
            if (kc + 1 < nk) {
                load_a(kc + 1, cur);
                tp_dma_image<RP_WAVES>(W + (size_t)(kc + 1) * SLAB, lds + ((kc + 1) & 1) * SLAB, SLAB);
            }
            __builtin_amdgcn_sched_barrier(0);
            mfmas(a, lds + (kc & 1) * SLAB);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
    }
    if constexpr (PREC == 2) {   // undo the image's weight scale; fp16x2 range guard
        float z = 0.f;
#pragma unroll
        for (int j = 0; j < NTILES; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                acc[j][e] *= P.h2_sinv;
                z = tp_nonfinite_fold(z, acc[j][e]);
            }
        tp_range_flag(P.range_flag, z);
    }
#pragma unroll
    for (int j = 0; j < NTILES; ++j) {
        const int col = 32 * j + r;
        const bool live = col < P.N;
        const float b = (live && P.bias) ? P.bias[col] : 0.f;
        const float sc = (live && P.scale) ? P.scale[col] : 1.f;
        // residual: all 16 loads of the tile issued before any use (one latency, not 16)
        float res[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int rr = rt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
            res[e] = (P.resid && live && rr < P.rows) ? P.resid[(size_t)rr * P.ldr + col] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int rr = rt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
            if (live && rr < P.rows) {
                float y = lin_act(acc[j][e] + b, ACT);
                if (P.resid) y = res[e] + sc * y;
                P.Y[(size_t)rr * P.ldy + col] = y;
            }
        }
    }
}

template <int NTILES, int ACT, int PREC = 1>
int lin_rp_launch(const LinRpProb& p, hipStream_t st) {
    if (p.rows <= 0) return NBX_OK;
    if (p.K % 32 || !p.Wx3 || p.N > NTILES * 32) {
        set_error("lin_rp: K %% 32 == 0, an image and N <= %d required", NTILES * 32);
        return NBX_E_INVAL;
    }
    if ((double)p.rows * p.lda * 4.0 >= 2147483632.0) {
        set_error("lin_rp: A spans >= 2 GiB");
        return NBX_E_UNSUPPORTED;
    }
    const size_t lds = ((NTILES <= 5 || PREC == 2) ? 3 : 2) * (size_t)NTILES * (PREC == 2 ? LIN_H2_BLK : LIN_X3_BLK) * 4;
    NBX_LDS_160K((lin_rp_kernel<NTILES, ACT, PREC>));
    const unsigned blocks = (unsigned)((p.rows + 32 * RP_WAVES - 1) / (32 * RP_WAVES));
    hipLaunchKernelGGL((lin_rp_kernel<NTILES, ACT, PREC>), dim3(blocks), dim3(64 * RP_WAVES), lds, st, p);
    NBX_HIP(hipGetLastError());
    return NBX_OK;
}

inline LinProb lin_dense(const float* A, int lda, int K, int rows, const float* Wt, int ldw, int N, const float* bias,
                         float* Y, int ldy) {
    LinProb p;
    memset(&p, 0, sizeof(p));
    p.seg[0] = LinSeg{A, nullptr, lda, (K + 31) & ~31, K};
    p.nseg = 1;
    p.rows = rows;
    p.N = N;
    p.Ktot = (K + 31) & ~31;
    p.Wt = Wt;
    p.ldw = ldw;
    p.bias = bias;
    p.Y = Y;
    p.ldy = ldy;
    return p;
}

}  // namespace nbx
