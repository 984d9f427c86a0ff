// Fused message path of one SEGNN layer (msg_pre.h "MsgFusedProb"): message_layer_1 and
// message_layer_2 with aggregation and the message-BatchNorm sums in one kernel
// (segnn.py:264-284 message(), o3_building_blocks.py:170-203 / :96-128 for the two TPs).
//
// Block = one node group (NG = 15 nodes = 3 systems at N = 5, G = 4 edge slots each, 60 edge
// rows padded to 4 row tiles of 16).  The M = 96 input channels of message_layer_2 are walked
// in three 32-channel slices; per slice:
//   1. node GEMM of the slice's two 16-channel chunks (X rows pre-split into bf16x3 A fragments
//      in LDS once per block; B fragments straight from the L2-resident node_pre x3 images):
//        waves 0-5: chunk w / 3, vector planes 1-3 x parts {2 (w % 3), 2 (w % 3) + 1} (one B
//                   fragment feeds three planes),
//        waves 6-7: chunk w - 6, scalar plane 0 x parts 0-5;
//      -> NP [2 chunks][4 planes][6 parts][16 rows][16 ch] in LDS (quad-swizzled rows);
//   2. edge combination (thread = (edge row, 4 channels)): the msg_pre edge arithmetic + gate,
//      written as the slice of M1 = [m_s | m_v . rhat | m_v (3 planes)], split into bf16x3 and
//      stored in v_mfma_f32_16x16x32_bf16 A-fragment order (5 K-steps x 4 row tiles);
//   3. message_layer_2 K-slice: waves 0-5 own output chunk cc = w (16 channels of s, gate, t and
//      the three v planes) for all 4 row tiles: 24 accumulator tiles that live in registers
//      across the slices; B fragments from the CW = 16 msg2 x3 image.
// Epilogue (waves 0-5): gate, edge mask, aggregation of the G rows of each destination (one
// lane's 4 accumulator rows), AGG / AD stores and the fp64 message-BN sums (one atomic per
// channel and statistic per block).  M1 (39 MB per layer at C2) never reaches HBM.
#include "msg_pre.h"
#include "tp16.h"

namespace nbx {

namespace {

constexpr int MF_THREADS = 512;
constexpr int MF_M = 96;          // channels (mul)
constexpr int MF_KCT = 3;         // 32-deep K chunks of the node GEMM (M / 32)
constexpr int MF_SLICES = 3;      // 32-channel K slices of message_layer_2
constexpr int MF_IMG1 = 6 * MF_KCT * 3 * 64;   // bf16x8 per 16-channel chunk of a node_pre x3 image
constexpr int MF_IMG2 = 18 * 3 * 64;           // bf16x8 per 16-channel chunk of the msg2 x3 image
// LDS (floats): NP 12288 | M1A 15360 | XA 9216 | XC 288 | EGL 512 | NAL 64
constexpr int MF_NP = 0, MF_M1A = 12288, MF_XA = MF_M1A + 15360, MF_XC = MF_XA + 9216, MF_EGL = MF_XC + 288,
              MF_NAL = MF_EGL + 512, MF_LDS_FLOATS = MF_NAL + 64;

// six cross terms of the bf16x3 product, smallest first: (A part, B part)
constexpr int TA[6] = {2, 1, 0, 1, 0, 0}, TB[6] = {0, 1, 2, 0, 1, 0};

__device__ inline floatx4 mma(const bf16x8& a, const bf16x8& b, const floatx4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 4 floats -> three bf16 parts, 4 bf16 (8 bytes) each
__device__ inline void split4(const float v[4], uint2& hi, uint2& mid, uint2& lo) {
    unsigned H[2], Mi[2], L[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const tp_f2 f{v[2 * i], v[2 * i + 1]};
        const unsigned h = tp_pk_bf16(f);
        const tp_f2 r = tp_sub2(f, tp_unpk_bf16(h));
        const unsigned m = tp_pk_bf16(r);
        H[i] = h;
        Mi[i] = m;
        L[i] = tp_pk_bf16(tp_sub2(r, tp_unpk_bf16(m)));
    }
    hi = uint2{H[0], H[1]};
    mid = uint2{Mi[0], Mi[1]};
    lo = uint2{L[0], L[1]};
}

template <int G>
__global__ __launch_bounds__(MF_THREADS, 1) void msg_fused_kernel(const MsgFusedProb P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* NP = lds + MF_NP;
    bf16x8* M1A = reinterpret_cast<bf16x8*>(lds + MF_M1A);   // [5 K-steps][4 row tiles][3 parts][64]
    bf16x8* XA = reinterpret_cast<bf16x8*>(lds + MF_XA);     // [4 planes][3 kc][3 parts][64]
    float* XC = lds + MF_XC;                                 // [sc_s | sc_v | sh] x 96
    float4* EGL = reinterpret_cast<float4*>(lds + MF_EGL);   // [64 rows][2]: (rhat, |rel|), (m_i m_j, ...)
    float4* NAL = reinterpret_cast<float4*>(lds + MF_NAL);   // [16 nodes] (1, na)
    constexpr int M = MF_M;
    constexpr int LG = G == 4 ? 2 : (G == 2 ? 1 : 0);
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, c16 = lane & 15, qd = lane >> 4;
    const int N = P.N, NG = P.NG, rows = NG * G;
    const long node0 = (long)blockIdx.x * NG;
    const unsigned long long c_start = P.dbg ? clock64() : 0ull;
    unsigned long long c_mark = c_start, c_node = 0, c_comb = 0, c_mma = 0, c_bar = 0;
    auto tick = [&](unsigned long long& acc) {
        if (P.dbg) { const unsigned long long c = clock64(); acc += c - c_mark; c_mark = c; }
    };

    // ---------------------------------------------------------------- prologue
    // pending feature BatchNorm of X (finalised from the atomic sums: block 0 owns the running
    // statistics and the coefficient copy for the layer's later consumers)
    for (int i = t; i < 3 * M; i += MF_THREADS) {
        const int part = i / M, k = i - part * M;
        XC[i] = P.xbn.sums ? bn_coef(P.xbn, M, part, k, blockIdx.x == 0)
                           : (P.xcoef ? P.xcoef[part * M + k] : (part < 2 ? 1.f : 0.f));
    }
    if (t < 64) {
        const int e = t;
        float4 a{0.f, 0.f, 0.f, 0.f}, b{0.f, 0.f, 0.f, 0.f};
        if (e < rows && node0 + (e >> LG) < P.V) {
            const float4* src = reinterpret_cast<const float4*>(P.EG + (node0 * G + e) * 8);
            a = src[0];
            b = src[1];
        }
        EGL[2 * e] = a;
        EGL[2 * e + 1] = b;
    } else if (t < 80) {
        const int r = t - 64;
        NAL[r] = (r < NG && node0 + r < P.V) ? *reinterpret_cast<const float4*>(P.NA + (node0 + r) * 4)
                                              : float4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
    // X rows of the group -> bf16x3 A fragments (lane (row c16, quarter qd) holds k = 32 kc + 8 qd + j)
    for (int pk = wave; pk < 4 * MF_KCT; pk += 8) {
        const int plane = pk / MF_KCT, kc = pk - plane * MF_KCT;
        const long node = node0 + c16;
        const int k = kc * 32 + 8 * qd;
        float4 x0{0.f, 0.f, 0.f, 0.f}, x1{0.f, 0.f, 0.f, 0.f};
        if (c16 < NG && node < P.V) {
            const float4* src = reinterpret_cast<const float4*>(P.X + ((long)plane * P.V + node) * M + k);
            x0 = src[0];
            x1 = src[1];
        }
        const float* sc = XC + (plane ? M : 0) + k;
        const float* sh = XC + 2 * M + k;
        const float ps = plane ? 0.f : 1.f;   // the shift applies to the 0e plane only
        const float4 v0{fmaf(sc[0], x0.x, ps * sh[0]), fmaf(sc[1], x0.y, ps * sh[1]), fmaf(sc[2], x0.z, ps * sh[2]),
                        fmaf(sc[3], x0.w, ps * sh[3])};
        const float4 v1{fmaf(sc[4], x1.x, ps * sh[4]), fmaf(sc[5], x1.y, ps * sh[5]), fmaf(sc[6], x1.z, ps * sh[6]),
                        fmaf(sc[7], x1.w, ps * sh[7])};
        bf16x8 a0, a1, a2;
        tp_split3(v0, v1, a0, a1, a2);
        bf16x8* dst = XA + (pk * 3) * 64 + lane;
        dst[0] = a0;
        dst[64] = a1;
        dst[128] = a2;
    }
    __syncthreads();
    tick(c_bar);

    // ---------------------------------------------------------------- per-wave roles
    const bool vwave = wave < 6;                  // node GEMM on the vector planes + message_layer_2
    const int nh = vwave ? wave / 3 : wave - 6;   // which 16-channel chunk of the slice
    const int jp = vwave ? 2 * (wave % 3) : 0;    // first part (vector waves: 2 parts)
    floatx4 acc2[4][6];                           // message_layer_2 tiles [row tile][s, gate, t, v0, v1, v2]
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 6; ++j) acc2[r][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    auto np_at = [&](int h, int pl, int part, int row, int cq) -> float* {
        return NP + (((h * 4 + pl) * 6 + part) * 16 + row) * 16 + 4 * (cq ^ ((row >> 2) & 3));
    };

    for (int sl = 0; sl < MF_SLICES; ++sl) {
        const int chunk = 2 * sl + nh;
        // ------------------------------------------------ 1. node GEMM of the slice -> NP
        if (vwave) {
            // planes 1-3 x parts jp, jp+1: 6 accumulators, each B fragment feeds three planes
            const bf16x8* bimg = reinterpret_cast<const bf16x8*>(P.Vimg) + (size_t)chunk * MF_IMG1 + lane;
            floatx4 acc[3][2];
#pragma unroll
            for (int p = 0; p < 3; ++p) acc[p][0] = acc[p][1] = floatx4{0.f, 0.f, 0.f, 0.f};
            bf16x8 bb[2][2][3];
            auto load_b = [&](int kc, bf16x8 (&b)[2][3]) {
#pragma unroll
                for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                    for (int p3 = 0; p3 < 3; ++p3) b[jj][p3] = bimg[((jp + jj) * MF_KCT + kc) * 192 + p3 * 64];
            };
            load_b(0, bb[0]);
            static_for<0, MF_KCT>([&](auto kcc) {
                constexpr int kc = decltype(kcc)::value;
                if constexpr (kc + 1 < MF_KCT) load_b(kc + 1, bb[(kc + 1) & 1]);
                bf16x8 a[3][3];
#pragma unroll
                for (int p = 0; p < 3; ++p)
#pragma unroll
                    for (int p3 = 0; p3 < 3; ++p3) a[p][p3] = XA[(((1 + p) * MF_KCT + kc) * 3 + p3) * 64 + lane];
                const bf16x8 (&b)[2][3] = bb[kc & 1];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int tt = 0; tt < 6; ++tt)
#pragma unroll
                    for (int p = 0; p < 3; ++p)
#pragma unroll
                        for (int jj = 0; jj < 2; ++jj) acc[p][jj] = mma(a[p][TA[tt]], b[jj][TB[tt]], acc[p][jj]);
                __builtin_amdgcn_sched_barrier(0);
            });
            const int col = (c16 & 3) | (((c16 >> 2) ^ qd) << 2);
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        NP[(((nh * 4 + 1 + p) * 6 + jp + jj) * 16 + 4 * qd + r) * 16 + col] = acc[p][jj][r];
        } else {
            // scalar plane 0 x parts 0-5
            const bf16x8* bimg = reinterpret_cast<const bf16x8*>(P.Simg) + (size_t)chunk * MF_IMG1 + lane;
            floatx4 acc[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
            // (single-buffered B: acc2 is live in every wave, so a second 72-VGPR buffer would spill)
            static_for<0, MF_KCT>([&](auto kcc) {
                constexpr int kc = decltype(kcc)::value;
                bf16x8 b[6][3];
#pragma unroll
                for (int j = 0; j < 6; ++j)
#pragma unroll
                    for (int p3 = 0; p3 < 3; ++p3) b[j][p3] = bimg[(j * MF_KCT + kc) * 192 + p3 * 64];
                bf16x8 a[3];
#pragma unroll
                for (int p3 = 0; p3 < 3; ++p3) a[p3] = XA[(kc * 3 + p3) * 64 + lane];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int tt = 0; tt < 6; ++tt)
#pragma unroll
                    for (int j = 0; j < 6; ++j) acc[j] = mma(a[TA[tt]], b[j][TB[tt]], acc[j]);
                __builtin_amdgcn_sched_barrier(0);
            });
            const int col = (c16 & 3) | (((c16 >> 2) ^ qd) << 2);
#pragma unroll
            for (int j = 0; j < 6; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) NP[(((nh * 4 + 0) * 6 + j) * 16 + 4 * qd + r) * 16 + col] = acc[j][r];
        }
        tick(c_node);
        __syncthreads();
        tick(c_bar);

        // ------------------------------------------------ 2. edge combination -> M1 slice (A fragments)
        {
            const int e = t >> 3, quad = t & 7, hh = quad >> 2, cq = quad & 3;
            const int chl = 16 * hh + 4 * cq;          // channel within the slice
            const int ch = 32 * sl + chl;              // input channel of message_layer_2
            const int ld = e >> LG, q = e & (G - 1);
            const bool ok = e < rows && q < N - 1 && node0 + ld < P.V;
            float o[5][4];
            if (ok) {
                const int d = ld % N;                  // position in the system
                const int sq = q < d ? q : q + 1;      // source slot (fully connected, ascending)
                const int sr = ld - d + sq;            // source row in the group
                const float4 g0 = EGL[2 * e];
                const float pm = EGL[2 * e + 1].x;
                const float hk[3] = {g0.x, g0.y, g0.z};
                const float dist = g0.w;
                auto ld4 = [&](const float* p) { return *reinterpret_cast<const float4*>(p + ch); };
                const float4 ea0 = ld4(P.amf), eg0 = ld4(P.amf + M), et0 = ld4(P.amf + 2 * M);
                const float4 ea1 = ld4(P.amf + 3 * M), eg1 = ld4(P.amf + 4 * M), et1 = ld4(P.amf + 5 * M);
                const float4 ba = ld4(P.bias1), bg = ld4(P.bias1 + M);
                float sa[4], sg[4], tt[4], vv[3][4];
                {
                    const float4 d0 = *reinterpret_cast<const float4*>(np_at(hh, 0, 0, ld, cq));
                    const float4 d1 = *reinterpret_cast<const float4*>(np_at(hh, 0, 1, ld, cq));
                    const float4 d2 = *reinterpret_cast<const float4*>(np_at(hh, 0, 2, ld, cq));
                    const float4 s0 = *reinterpret_cast<const float4*>(np_at(hh, 0, 3, sr, cq));
                    const float4 s1 = *reinterpret_cast<const float4*>(np_at(hh, 0, 4, sr, cq));
                    const float4 s2 = *reinterpret_cast<const float4*>(np_at(hh, 0, 5, sr, cq));
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        sa[c] = fmaf(f4get(ea1, c), pm, fmaf(f4get(ea0, c), dist, f4get(d0, c) + f4get(s0, c))) +
                                f4get(ba, c);
                        sg[c] = fmaf(f4get(eg1, c), pm, fmaf(f4get(eg0, c), dist, f4get(d1, c) + f4get(s1, c))) +
                                f4get(bg, c);
                        tt[c] = fmaf(f4get(et1, c), pm, fmaf(f4get(et0, c), dist, f4get(d2, c) + f4get(s2, c)));
                    }
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    // one plane's operands at a time (acc2 holds 96 VGPRs in the vector waves)
                    __builtin_amdgcn_sched_barrier(0);
                    const float4 d0 = *reinterpret_cast<const float4*>(np_at(hh, 1 + k, 0, ld, cq));
                    const float4 d1 = *reinterpret_cast<const float4*>(np_at(hh, 1 + k, 1, ld, cq));
                    const float4 d2 = *reinterpret_cast<const float4*>(np_at(hh, 1 + k, 2, ld, cq));
                    const float4 s0 = *reinterpret_cast<const float4*>(np_at(hh, 1 + k, 3, sr, cq));
                    const float4 s1 = *reinterpret_cast<const float4*>(np_at(hh, 1 + k, 4, sr, cq));
                    const float4 s2 = *reinterpret_cast<const float4*>(np_at(hh, 1 + k, 5, sr, cq));
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        sa[c] = fmaf(hk[k], f4get(d0, c) + f4get(s0, c), sa[c]);
                        sg[c] = fmaf(hk[k], f4get(d1, c) + f4get(s1, c), sg[c]);
                        vv[k][c] = fmaf(hk[k], tt[c], f4get(d2, c)) + f4get(s2, c);
                    }
                }
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float gg = kC_SIGMOID * tp_sigmoid(sg[c]);
                    o[0][c] = kC_SILU * tp_silu(sa[c]);
                    o[2][c] = gg * vv[0][c];
                    o[3][c] = gg * vv[1][c];
                    o[4][c] = gg * vv[2][c];
                    o[1][c] = fmaf(o[4][c], hk[2], fmaf(o[3][c], hk[1], o[2][c] * hk[0]));
                }
            } else {
#pragma unroll
                for (int T = 0; T < 5; ++T)
#pragma unroll
                    for (int c = 0; c < 4; ++c) o[T][c] = 0.f;
            }
            // A fragment of row tile e >> 4: lane (e & 15) + 16 (chl >> 3), elements chl & 7 .. +3
            uint2* m1 = reinterpret_cast<uint2*>(M1A) + (size_t)((e >> 4) * 3) * 128 +
                        ((e & 15) + 16 * (chl >> 3)) * 2 + ((chl >> 2) & 1);
#pragma unroll
            for (int T = 0; T < 5; ++T) {
                uint2 hi, mid, lo;
                split4(o[T], hi, mid, lo);
                m1[(T * 4 * 3 + 0) * 128] = hi;
                m1[(T * 4 * 3 + 1) * 128] = mid;
                m1[(T * 4 * 3 + 2) * 128] = lo;
            }
        }
        tick(c_comb);
        __syncthreads();
        tick(c_bar);

        // ------------------------------------------------ 3. message_layer_2 K-slice
        if (vwave) {
            // B fragments of this slice for output chunk cc = wave: s and gate at K-steps sl (m_s)
            // and 3 + sl (m_v . rhat), t at sl (its m_v . rhat half is zero), v at sl
            bf16x8 b2[6][3];
            const bf16x8* w2 = reinterpret_cast<const bf16x8*>(P.W2) + (size_t)wave * MF_IMG2 + lane;
            const int off[6] = {sl, 3 + sl, 6 + sl, 9 + sl, 12 + sl, 15 + sl};
#pragma unroll
            for (int f = 0; f < 6; ++f)
#pragma unroll
                for (int p3 = 0; p3 < 3; ++p3) b2[f][p3] = w2[off[f] * 192 + p3 * 64];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                // scalar part: K-steps m_s and m_v . rhat
                {
                    bf16x8 a[2][3];
#pragma unroll
                    for (int T = 0; T < 2; ++T)
#pragma unroll
                        for (int p3 = 0; p3 < 3; ++p3) a[T][p3] = M1A[((T * 4 + r) * 3 + p3) * 64 + lane];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int tt = 0; tt < 6; ++tt) {
                        const int ia = TA[tt], ib = TB[tt];
                        acc2[r][0] = mma(a[0][ia], b2[0][ib], acc2[r][0]);
                        acc2[r][1] = mma(a[0][ia], b2[2][ib], acc2[r][1]);
                        acc2[r][2] = mma(a[0][ia], b2[4][ib], acc2[r][2]);
                        acc2[r][0] = mma(a[1][ia], b2[1][ib], acc2[r][0]);
                        acc2[r][1] = mma(a[1][ia], b2[3][ib], acc2[r][1]);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                // vector part: one K-step per plane
                {
                    bf16x8 a[3][3];
#pragma unroll
                    for (int T = 0; T < 3; ++T)
#pragma unroll
                        for (int p3 = 0; p3 < 3; ++p3) a[T][p3] = M1A[(((2 + T) * 4 + r) * 3 + p3) * 64 + lane];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int tt = 0; tt < 6; ++tt)
#pragma unroll
                        for (int T = 0; T < 3; ++T)
                            acc2[r][3 + T] = mma(a[T][TA[tt]], b2[5][TB[tt]], acc2[r][3 + T]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            tick(c_mma);
        }
    }

    // ---------------------------------------------------------------- epilogue (waves 0-5)
    if (vwave) {
        const int ch = 16 * wave + c16;
        const float ba = P.bias2[ch], bg = P.bias2[M + ch];
        double st0 = 0.0, st1 = 0.0, st2 = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float ms[4], mv[3][4];
            float f0 = 0.f, f1 = 0.f, f2 = 0.f;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int e = 16 * r + 4 * qd + jj;
                const int ld = e >> LG;
                const bool ok = e < rows && (e & (G - 1)) < N - 1 && node0 + ld < P.V;
                const float4 g = EGL[2 * e];
                const float s = kC_SILU * tp_silu(acc2[r][0][jj] + ba);
                const float gg = kC_SIGMOID * tp_sigmoid(acc2[r][1][jj] + bg);
                const float tt = acc2[r][2][jj];
                ms[jj] = ok ? s : 0.f;
                mv[0][jj] = ok ? gg * (g.x * tt + acc2[r][3][jj]) : 0.f;
                mv[1][jj] = ok ? gg * (g.y * tt + acc2[r][4][jj]) : 0.f;
                mv[2][jj] = ok ? gg * (g.z * tt + acc2[r][5][jj]) : 0.f;
                f0 += ms[jj];
                f1 += ms[jj] * ms[jj];
                f2 += mv[0][jj] * mv[0][jj] + mv[1][jj] * mv[1][jj] + mv[2][jj] * mv[2][jj];
            }
            st0 += (double)f0;
            st1 += (double)f1;
            st2 += (double)f2;
            // aggregate the G rows of each destination (registers of this lane)
#pragma unroll
            for (int j0 = 0; j0 < 4; j0 += G) {
                float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
                for (int u = 0; u < G; ++u) {
                    a0 += ms[j0 + u];
                    a1 += mv[0][j0 + u];
                    a2 += mv[1][j0 + u];
                    a3 += mv[2][j0 + u];
                }
                const int ld = (16 * r + 4 * qd + j0) >> LG;
                const long node = node0 + ld;
                if (ld < NG && node < P.V) {
                    const size_t o = (size_t)node * M + ch;
                    const size_t pl = (size_t)P.V * M;
                    P.AGG[o] = a0;
                    P.AGG[pl + o] = a1;
                    P.AGG[2 * pl + o] = a2;
                    P.AGG[3 * pl + o] = a3;
                    const float4 na = NAL[ld];
                    P.AD[o] = a1 * na.y + a2 * na.z + a3 * na.w;
                }
            }
        }
        st0 += __shfl_xor(st0, 16);
        st1 += __shfl_xor(st1, 16);
        st2 += __shfl_xor(st2, 16);
        st0 += __shfl_xor(st0, 32);
        st1 += __shfl_xor(st1, 32);
        st2 += __shfl_xor(st2, 32);
        if (qd == 0) {
            bn_atomic_add(P.bn_sums + ch, st0);
            bn_atomic_add(P.bn_sums + M + ch, st1);
            bn_atomic_add(P.bn_sums + 2 * M + ch, st2);
        }
    }
    tick(c_bar);
    if (P.dbg && lane == 0) {
        unsigned long long* d = P.dbg + ((size_t)blockIdx.x * 8 + wave) * 4;
        d[0] = c_node; d[1] = c_comb; d[2] = c_mma; d[3] = c_bar;
    }
}

}  // namespace

bool msg_fused_supported(int M, int N) { return M == MF_M && N >= 2 && N <= 5; }

int msg_fused_launch(MsgFusedProb& p, hipStream_t st) {
    if (p.V <= 0) return NBX_OK;
    if (!msg_fused_supported(p.M, p.N) || p.NG != msg_pre_group(p.N) || p.NG * p.G > 64 || !p.bn_sums ||
        !p.Simg || !p.Vimg || !p.W2) {
        set_error("msg_fused: needs mul 96, 2 <= N <= 5, bf16x3 images and atomic BatchNorm sums");
        return NBX_E_UNSUPPORTED;
    }
    const size_t lds = (size_t)MF_LDS_FLOATS * 4;
    static bool attr_set = false;
    if (!attr_set) {
        for (const void* k : {(const void*)msg_fused_kernel<1>, (const void*)msg_fused_kernel<2>,
                              (const void*)msg_fused_kernel<4>})
            NBX_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        attr_set = true;
    }
    const dim3 grid((unsigned)((p.V + p.NG - 1) / p.NG));
    switch (p.G) {
        case 4: NBX_TIMED_LAUNCH(msg_fused_kernel<4>, grid, dim3(MF_THREADS), lds, st, p); break;
        case 2: NBX_TIMED_LAUNCH(msg_fused_kernel<2>, grid, dim3(MF_THREADS), lds, st, p); break;
        case 1: NBX_TIMED_LAUNCH(msg_fused_kernel<1>, grid, dim3(MF_THREADS), lds, st, p); break;
        default: set_error("msg_fused: G = %d", p.G); return NBX_E_UNSUPPORTED;
    }
    NBX_HIP(hipGetLastError());
    return NBX_OK;
}

}  // namespace nbx
