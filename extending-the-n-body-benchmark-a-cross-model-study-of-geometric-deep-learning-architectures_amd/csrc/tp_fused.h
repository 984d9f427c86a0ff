// Weight-stationary fused O(3) tensor-product kernel (fp32 MFMA) for SEGNN.
//
// Every l <= 1 tensor product of the path is a pair of GEMMs on the same rows:
//   scalar part  A_S[row, K_S] x B_S -> NS sub-tiles of 32 output columns (e.g. s, gate, t)
//   vector part  A_V[k][row, K_V] x B_V -> 1 sub-tile per component plane k = 0..2
// for one 32-channel "chunk" of the output.  A block owns one chunk: its slices
// of B_S / B_V are loaded into LDS once and stay there while the block's waves
// stream 32-row tiles of A straight from global memory (register double
// buffering, no barrier in the main loop).  A wave keeps the whole chunk of its
// 32 rows in accumulators (NS + 3 tiles of v_mfma_f32_32x32x2_f32), so the
// epilogue - SiLU/sigmoid gate, aggregation over a node's incoming edges,
// BatchNorm partial sums, residual update - runs in registers.
//
// MFMA 32x32x2 f32 fragment maps (cdna_hip_programming.md §3):
//   A: lane l holds A[row = l & 31][k = l >> 5];  B: B[k = l >> 5][col = l & 31]
//   C: col = l & 31, row = (j & 3) + 8 (j >> 2) + 4 (l >> 5), j = register 0..15
// Inside every 32-deep K chunk the K order is permuted so that a lane reads 16
// consecutive k (lane half h supplies k = 16h + s at MFMA step s for both
// operands: the sum is unchanged).
#pragma once
#include <cstdlib>
#include <type_traits>

#include "nbx_internal.h"

namespace nbx {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

enum TpEpi : int { TP_PLAIN = 0, TP_MSG = 1, TP_GATE_NODE = 2, TP_RESID = 3 };

// BatchNorm statistics accumulated by the producing kernel with device-scope fp64 atomics
// ([3][M]: sum s and sum s^2 over the 0e channels, sum |v|^2 over the 1o channels) and
// finalised by the consuming kernel in its prologue (bn_coef), in place of a separate
// finalize launch.  Sums arrive in any order: results can differ run to run in the last bits.
struct BnSrc {
    const double* sums;   // null: not in use
    const float* weight;
    const float* bias;
    float* rmean;
    float* rvar;
    float* coef_out;      // block 0 stores [sc_s | sc_v | sh] here for later consumers, or null
    double count;
    float eps, momentum;
    int training;
    int update;           // block 0 applies the running-stat update
};

// Coefficient `part` (0: 0e scale, 1: 1o scale, 2: 0e shift) of channel k, the same arithmetic
// as segnn.hip bn_finalize_kernel; the owner (one thread of block 0 per (part, k)) also writes
// the running statistics (parts 0 and 1) and coef_out.
__device__ inline float bn_coef(const BnSrc& b, int M, int part, int k, bool owner) {
    if (part == 1) {
        const double n = b.training ? b.sums[2 * M + k] / (3.0 * b.count) : (double)b.rvar[M + k];
        const float sc = (float)(1.0 / sqrt(n + (double)b.eps)) * b.weight[M + k];
        if (owner) {
            if (b.training && b.update) b.rvar[M + k] = (1.0f - b.momentum) * b.rvar[M + k] + b.momentum * (float)n;
            if (b.coef_out) b.coef_out[M + k] = sc;
        }
        return sc;
    }
    double mu, var;
    if (b.training) {
        mu = b.sums[k] / b.count;
        var = b.sums[M + k] / b.count - mu * mu;
        if (var < 0.0) var = 0.0;
    } else {
        mu = b.rmean[k];
        var = b.rvar[k];
    }
    const float sc = (float)(1.0 / sqrt(var + (double)b.eps)) * b.weight[k];
    const float sh = b.bias[k] - sc * (float)mu;
    if (owner) {
        if (part == 0) {
            if (b.training && b.update) {
                b.rmean[k] = (1.0f - b.momentum) * b.rmean[k] + b.momentum * (float)mu;
                b.rvar[k] = (1.0f - b.momentum) * b.rvar[k] + b.momentum * (float)var;
            }
            if (b.coef_out) b.coef_out[k] = sc;
        } else if (b.coef_out) {
            b.coef_out[2 * M + k] = sh;
        }
    }
    return part == 0 ? sc : sh;
}

// The same arithmetic with the inputs loaded up front: a consumer prologue issues these loads before its
// weight-image DMA (vmcnt retires in issue order, so loads issued after the DMA would wait for all of
// it), one evaluation per thread.  kind 0 = channel k's (0e scale, 0e shift) [bn_coef parts 0, 2],
// kind 1 = its 1o scale [part 1]; the owner (block 0) applies the running-stat update and coef_out.
struct BnPre {
    double s0, s1;
    float w, b, rm, rv;
};
// The inputs of one coefficient evaluation (kind 0: 0e mean / variance, kind 1: 1o norm; `on`: this
// thread evaluates one).  Branch-free: every thread issues the same six loads -- an unused slot reads
// `dummy`, any readable address with 3 M doubles behind it -- into registers of their own and selects
// afterwards.  Loads under a divergent branch made the waitcnt pass drain every load in flight, the A
// ring's first chunks included, before the weight-image DMA was issued: one memory latency added to
// the staging of update_layer_1, pre_pool1 and msg_pre.
__device__ inline BnPre bn_pre_load(const BnSrc& b, int M, int kind, int k, bool on, const void* dummy) {
    const double* dd = static_cast<const double*>(dummy);
    const float* df = static_cast<const float*>(dummy);
    const bool tr = on && b.training && b.sums;
    const bool k0 = kind == 0;
    const double* sums = tr ? b.sums : dd;
    const float* rmean = on && b.rmean ? b.rmean : df;
    const float* rvar = on && b.rvar ? b.rvar : df;
    const float* weight = on && b.weight ? b.weight : df;
    const float* bias = on && b.bias ? b.bias : df;
    const int iv = k0 ? k : M + k;
    const double s0 = sums[k0 ? k : 2 * M + k], s1 = sums[M + k];
    const float rm = rmean[k], rv = rvar[iv], w = weight[iv], bb = bias[k];
    BnPre p;
    p.s0 = tr ? s0 : 0.0;
    p.s1 = tr && k0 ? s1 : 0.0;
    p.rm = on && k0 ? rm : 0.f;
    p.rv = on ? rv : 0.f;
    p.w = on ? w : 0.f;
    p.b = on && k0 ? bb : 0.f;
    return p;
}
// one of two sources, selected per lane field by field (no pointer to either struct is formed)
__device__ inline BnSrc bn_src_sel(const BnSrc& a, const BnSrc& b, bool use_b) {
    BnSrc s;
    s.sums = use_b ? b.sums : a.sums;
    s.weight = use_b ? b.weight : a.weight;
    s.bias = use_b ? b.bias : a.bias;
    s.rmean = use_b ? b.rmean : a.rmean;
    s.rvar = use_b ? b.rvar : a.rvar;
    s.coef_out = use_b ? b.coef_out : a.coef_out;
    s.count = use_b ? b.count : a.count;
    s.eps = use_b ? b.eps : a.eps;
    s.momentum = use_b ? b.momentum : a.momentum;
    s.training = use_b ? b.training : a.training;
    s.update = use_b ? b.update : a.update;
    return s;
}
__device__ inline float2 bn_pre_coef(const BnSrc& b, const BnPre& p, int M, int kind, int k, bool owner) {
    if (kind == 1) {
        const double n = b.training ? p.s0 / (3.0 * b.count) : (double)p.rv;
        const float sc = (float)(1.0 / sqrt(n + (double)b.eps)) * p.w;
        if (owner) {
            if (b.training && b.update) b.rvar[M + k] = (1.0f - b.momentum) * p.rv + b.momentum * (float)n;
            if (b.coef_out) b.coef_out[M + k] = sc;
        }
        return float2{sc, 0.f};
    }
    double mu, var;
    if (b.training) {
        mu = p.s0 / b.count;
        var = p.s1 / b.count - mu * mu;
        if (var < 0.0) var = 0.0;
    } else {
        mu = p.rm;
        var = p.rv;
    }
    const float sc = (float)(1.0 / sqrt(var + (double)b.eps)) * p.w;
    const float sh = p.b - sc * (float)mu;
    if (owner) {
        if (b.training && b.update) {
            b.rmean[k] = (1.0f - b.momentum) * p.rm + b.momentum * (float)mu;
            b.rvar[k] = (1.0f - b.momentum) * p.rv + b.momentum * (float)var;
        }
        if (b.coef_out) { b.coef_out[k] = sc; b.coef_out[2 * M + k] = sh; }
    }
    return float2{sc, sh};
}

// no-return device-scope fp64 add (executes at the memory side, so adders on every XCD agree)
__device__ inline void bn_atomic_add(double* p, double v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Epilogue output stores.  WT: write-through (an agent-scope relaxed store = global_store ... sc1),
// so the line leaves the XCD's L2 as the epilogue writes it and the kernel ends without dirty lines
// for the end-of-kernel L2 write-back (MI355X_MICROARCH.md price list, row 'boundary': + B / 6 TB/s
// for B dirty bytes).  Used where a wave instruction stores whole 128-B rows (message_layer_2's
// aggregated messages: 32 lanes x 4 B) and for update_layer_2's residual update; tp16's gate
// epilogue (16 lanes x 4 B = 64-B pieces) keeps plain stores: sc1 made it slower (one fabric write
// per piece).  r05 A/B on one box: msg2 21.3 -> 20.0 us, upd2 12.3 -> 12.0, upd1 19.1 -> 19.7
// (profiles/r05/wtdv).
template <bool WT>
__device__ inline void st_out(float* p, float v) {
    if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

struct TpProb {
    // scalar part: NS sub-tiles, sub-tile j contracts the first K_j columns of A
    const float* As;   // [rows][lda_s]
    int lda_s, NS;
    int K[3];
    // vector part (NV = 1: three planes, NV = 0: none)
    const float* Av;   // plane k, row r at Av + k * plane_stride + r * lda_v
    long plane_stride;
    int lda_v, Kv, NV;
    // weights: MFMA-fragment-ordered LDS image, [chunks][img_floats] (include/nbx.h
    // "TP operand images"); a block copies its chunk's image into LDS verbatim
    const float* B;
    int img_floats;
    int img_stride;      // tp16: floats between consecutive chunk images (0: img_floats)
    // tp16 PLAIN: 0 -> column ((chunk * NS + j) * 16 + c); > 0 -> part-major output
    // columns (col_part0 + j) * col_part_stride + chunk * 16 + c, valid below M
    int col_part_stride, col_part0;
    int rows, chunks, M;  // M = real channels (epilogue mask)
    int epi;
    // PLAIN: C[row][chunk*NS*32 + 32 j + col]
    float* C;
    int ldc, ncols;
    // epilogue operands
    const float* bias;   // gate: [2M] (s, gate); resid: [M]
    const float* geom;   // MSG: per-edge [rows][8] (rhat xyz ...); GATE_NODE/RESID: node attrs [rows][4]
    const float* xcoef;  // RESID: pending feature BN of the residual X [sc_s | sc_v | sh] (M each), or null
    int group;           // MSG: edges per destination (power of two <= 32)
    int valid_per_group; // MSG: real edges per destination (<= group)
    float* out_s;        // MSG: AGG plane 0 [nodes][M]; GATE_NODE: U2S [rows][2M]; RESID: X plane 0
    float* out_v;        // MSG: AGG planes 1..3; GATE_NODE: U2V planes; RESID: X planes 1..3
    long out_plane;      // stride between output planes (elements)
    double* partial;     // MSG / RESID: [chunks][waves_per_chunk][3][32] fp64 BN partial sums
    double* bn_sums;     // MSG / RESID atomic mode (non-null): [3][M] fp64 sums instead of partial rows
    int waves_per_chunk;
    // grid geometry (set by the launcher)
    int blocks_per_chunk;
    int lds_floats;
    unsigned long long* dbg;  // optional per-wave phase clocks [waves][4] (tuning only)
    // tp16 static path with StatSK<..., SEG = 4> (update_layer_1 without a materialised input):
    // scalar A = 4 segments of M columns read from seg_s[q] ([rows][M]: x_s, a_s, x_v.na, a_v.na),
    // vector A = 2 segments from seg_v[q] (planes seg_vplane apart: x_v, a_v); each element is
    // scaled / shifted per (segment, k): x segments by the pending feature BN (xcoef, or identity),
    // a segments by the message BN (mcoef, shift x deg)
    const float* seg_s[4];
    const float* seg_v[2];
    long seg_vplane;
    // (set by the tp16 launcher) one buffer resource for all segments: the lowest segment pointer,
    // and each segment's byte offset from it (seg_s 0-3, seg_v 4-5) passed as the load's soffset,
    // so the kernel holds one 4-SGPR resource instead of one per (segment, plane)
    const float* seg_base;
    unsigned seg_boff[6];
    const float* mcoef;
    BnSrc mbn;           // SEG = 4 with mbn.sums: message BN finalised here from atomic sums (mcoef unused)
    BnSrc xbn;           // SEG > 0 with xbn.sums: pending feature BN finalised here (the segment table's
                         // x parts; xcoef unused there)
    float deg;
    // dot outputs (null: none): MSG: out_dot[dst][ch] = sum_k a_v,k na_k[dst] (na: node attrs
    // [V][4]); RESID: out_dot[row][ch] = sum_k x_v,k na_k[row] of the new x
    const float* na;
    float* out_dot;
    // fp16x2 images (StatSKH2): the factor that undoes the image's power-of-two weight scale
    float bscale;
    // XCD-grouped block order (set by the launchers when blocks_per_chunk % 8 == 0): the number of
    // chunk groups G; blocks b, b + 8, ... run on one XCD, so the G chunk groups of one row range are
    // given ids with equal b % 8 and that XCD's L2 fetches the range's A rows once for all G of them
    // (0: chunk-major order)
    int xcd_groups;
    // GATE_NODE: 1 = the [h_v . na] half of out_s is not written (its consumer forms it: TpStream DV)
    int skip_gate_dot;
    // fp16x2 range guard (tp_range_flag): set to 1 when a tile's accumulators are not finite; null: off
    int* range_flag;
};

// fp16x2 operand range guard.  An A operand with |a| >= 65520 rounds to an fp16 infinity (the split
// keeps fp32 accuracy everywhere below that), and every product it enters is then inf
// or NaN.  z = the sum over a tile's accumulators of acc * 0 is NaN exactly when one of them is not
// finite; the lane raises the call's flag (a vector store of a constant: racing lanes agree), which
// the host reads after the call and reports as NBX_E_RANGE instead of returning non-finite values.
__device__ inline float tp_nonfinite_fold(float z, float a) { return __builtin_fmaf(a, 0.f, z); }
__device__ inline void tp_range_flag(int* flag, float z) {
    if (flag != nullptr && !(z == 0.f)) *flag = 1;
}

// block id -> (chunk group, row-range block): chunk-major, or XCD-grouped (TpProb::xcd_groups)
__device__ inline void tp_block_map(const TpProb& P, int bidx, int& group, int& blk) {
    if (P.xcd_groups > 0) {
        const int xcd = bidx & 7, s = bidx >> 3;
        group = s % P.xcd_groups;
        blk = (s / P.xcd_groups) * 8 + xcd;
    } else {
        group = bidx / P.blocks_per_chunk;
        blk = bidx - group * P.blocks_per_chunk;
    }
}

constexpr int TP_WAVES = 8, TP_THREADS = 64 * TP_WAVES;

// Chunk schedule of a TP's K loop.  DynSK: chunk counts read from TpProb at run time (any
// shape).  StatSK<K0, K1, K2, KV>: the counts of 32-deep chunks of the scalar sub-tiles and of
// the vector sub-tile are compile-time, so the whole per-tile stream of A chunks is unrolled with
// static ring slots and static accumulator selection -- no branches around the MFMAs and no
// accumulator copies at control-flow merges (the dynamic loop pays ~50 v_mov per chunk for them).
struct DynSK {
    static constexpr bool on = false;
    static constexpr int K0 = 0, K1 = 0, K2 = 0, KV = 0, SEG = 0, PREC = 0, DV = 0;
};
template <int A, int B, int C, int V, int S = 0>
struct StatSK {
    static constexpr bool on = true;
    static constexpr int K0 = A, K1 = B, K2 = C, KV = V, SEG = S, PREC = 0, DV = 0;
};

// StatSK with the split-precision MFMA path (include/nbx.h "bf16x3 images"): A and B are split
// into three bf16 parts each and every product is the fp32 sum of the six leading cross terms on
// v_mfma_f32_32x32x16_bf16 -- fp32-level accuracy at 2.7x the fp32 MFMA rate (12 x 32 cycles per
// 32 x 32 x 32 block instead of 16 x 64).  The weight image is the bf16x3 one (1.5x the fp32 bytes).
template <int A, int B, int C, int V, int S = 0>
struct StatSKX3 {
    static constexpr bool on = true;
    static constexpr int K0 = A, K1 = B, K2 = C, KV = V, SEG = S, PREC = 1, DV = 0;
};

// x = hi + mid + lo (+ <= 2^-27 |x|), each part bf16: RNE conversions (v_cvt_pk_bf16_f32, two
// elements per instruction), the residuals are exact (v_pk_add_f32); 4.5 VALU per element
typedef __bf16 tp_bf16x2 __attribute__((ext_vector_type(2)));
typedef float tp_f2 __attribute__((ext_vector_type(2)));
typedef unsigned tp_u4 __attribute__((ext_vector_type(4)));
__device__ inline unsigned tp_pk_bf16(tp_f2 v) { return __builtin_bit_cast(unsigned, __builtin_convertvector(v, tp_bf16x2)); }
__device__ inline tp_f2 tp_unpk_bf16(unsigned u) {
    return tp_f2{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
}
// plain v_sub_f32: the files holding split-precision kernels are built with -fno-slp-vectorize
// (build.py), so these are not packed into v_pk_add_f32, which costs extra cycles beside MFMAs
// (MI355X_MICROARCH "price of one filler beside MFMAs"; measured +1.8 % steps/s)
__device__ inline float tp_sub(float a, float b) { return a - b; }
__device__ inline tp_f2 tp_sub2(tp_f2 a, tp_f2 b) { return tp_f2{tp_sub(a.x, b.x), tp_sub(a.y, b.y)}; }
__device__ inline void tp_split3(const float4& a, const float4& b, bf16x8& hi, bf16x8& mid, bf16x8& lo) {
    const tp_f2 f[4] = {{a.x, a.y}, {a.z, a.w}, {b.x, b.y}, {b.z, b.w}};
    tp_u4 H, Mi, L;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const unsigned h = tp_pk_bf16(f[i]);
        const tp_f2 r = tp_sub2(f[i], tp_unpk_bf16(h));
        const unsigned m = tp_pk_bf16(r);
        H[i] = h;
        Mi[i] = m;
        L[i] = tp_pk_bf16(tp_sub2(r, tp_unpk_bf16(m)));
    }
    hi = __builtin_bit_cast(bf16x8, H);
    mid = __builtin_bit_cast(bf16x8, Mi);
    lo = __builtin_bit_cast(bf16x8, L);
}

// StatSK with the fp16x2 split path (include/nbx.h "fp16x2 images"): x = hi + lo, both fp16 (RNE,
// v_cvt_pk_f16_f32), the residual unscaled; the weights are pre-scaled by a power of two per TP
// (max |w s| in [2^9, 2^10), so their residuals stay normal fp16) and the accumulator is descaled
// by TpProb::bscale = 1/s in the epilogue.  A product is the fp32 sum of hi.lo + lo.hi + hi.hi on
// v_mfma_f32_{16x16x32,32x32x16}_f16: half the MFMAs, two thirds of the operand bytes and of the
// split VALU of bf16x3.  Representation error <= ~2^-22 |a||b| per product (rms 7.6e-8 relative
// on a K = 192..384 GEMM), below the fp32 accumulation error of the same GEMM.
// D = 1 (TpStream): the scalar A's trailing dot chunks are formed in registers from the vector
// planes instead of being read.
template <int A, int B, int C, int V, int S = 0, int D = 0>
struct StatSKH2 {
    static constexpr bool on = true;
    static constexpr int K0 = A, K1 = B, K2 = C, KV = V, SEG = S, PREC = 2, DV = D;
};

// Position stream of the static split-precision K loop.  Without DV: position u = item u (scalar
// chunk u < K0, then vector chunk K0 + plane * KV + kc), every item loaded, in order.  With DV the
// scalar operand ends in KV dot chunks (chunk ND + kc = sum_p y_p v_p of vector chunk kc, ND = K0 - KV):
//   message_layer_2: [m_s | m_v . rhat] (ND = KV), update_layer_1: [x_s | a_s | x_v . na | a_v . na]
//   (ND = KV = 6), pre_pool1: [x_s | x_v . na] (ND = KV = 3);
//   update_layer_2: [h_s | h_v . na] (ND = KV = 3);
// the dot chunks are not loaded but formed in registers from the three vector chunks of the same
// channels (fmaf(v2, y2, fmaf(v1, y1, v0 * y0)), the chain their producers evaluate), so positions run
// the ND scalar chunks, then per kc: vec(0, kc), vec(1, kc), vec(2, kc), dot(kc) -- 20 % fewer A bytes.
template <class SK>
struct TpStream {
    static constexpr int KV = SK::KV, ND = SK::K0 - SK::KV;
    static constexpr int NPOS = SK::K0 + 3 * SK::KV;
    static constexpr int NLOAD = SK::DV ? NPOS - SK::KV : NPOS;
    static constexpr bool derived(int u) { return SK::DV && u >= ND && (u - ND) % 4 == 3; }
    // logical item of position u (a dot position: its scalar chunk ND + kc)
    static constexpr int item(int u) {
        if (!SK::DV || u < ND) return u;
        const int w = u - ND, kc = w / 4, s = w % 4;
        return s < 3 ? SK::K0 + s * KV + kc : ND + kc;
    }
    // load index of a loaded position, and the position of load index l
    static constexpr int lidx(int u) { return (!SK::DV || u < ND) ? u : ND + (u - ND) / 4 * 3 + (u - ND) % 4; }
    static constexpr int lpos(int l) { return (!SK::DV || l < ND) ? l : ND + (l - ND) / 3 * 4 + (l - ND) % 3; }
    // vector plane of position u (-1: not a vector chunk)
    static constexpr int plane(int u) {
        const int it = item(u);
        return (derived(u) || it < SK::K0) ? -1 : (it - SK::K0) / KV;
    }
};

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 tp_h2 __attribute__((ext_vector_type(2)));

// x = hi + lo (fp16 each, residual |x - hi - lo| <= 2^-22 |x| for |x| >= 2^-3; below that an
// absolute 2^-25): v_cvt_pk_f16_f32, two v_cvt_f32_f16, two v_sub_f32, v_cvt_pk_f16_f32 per pair
__device__ inline void tp_split_h2(const float4& a, const float4& b, h16x8& hi, h16x8& lo) {
    const tp_f2 f[4] = {{a.x, a.y}, {a.z, a.w}, {b.x, b.y}, {b.z, b.w}};
    tp_u4 H, L;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const tp_h2 h = __builtin_convertvector(f[i], tp_h2);
        const tp_f2 r = tp_sub2(f[i], __builtin_convertvector(h, tp_f2));
        H[i] = __builtin_bit_cast(unsigned, h);
        L[i] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, tp_h2));
    }
    hi = __builtin_bit_cast(h16x8, H);
    lo = __builtin_bit_cast(h16x8, L);
}

// Split-precision traits: PREC 1 = bf16x3 (3 parts, 6 terms), PREC 2 = fp16x2 (2 parts, 3 terms).
// Term t multiplies A part TA[t] by B part TB[t]; terms run smallest first.
template <int PREC> struct SplitP;
template <> struct SplitP<1> {
    using T = bf16x8;
    static constexpr int NP = 3, NT = 6;
    static constexpr int TA[6] = {2, 1, 0, 1, 0, 0}, TB[6] = {0, 1, 2, 0, 1, 0};
    __device__ static void split(const float4& a, const float4& b, T (&p)[3]) { tp_split3(a, b, p[0], p[1], p[2]); }
};
template <> struct SplitP<2> {
    using T = h16x8;
    static constexpr int NP = 2, NT = 3;
    static constexpr int TA[3] = {0, 1, 0}, TB[3] = {1, 0, 0};
    __device__ static void split(const float4& a, const float4& b, T (&p)[2]) { tp_split_h2(a, b, p[0], p[1]); }
};
// (PREC 0 never instantiates the split code; this keeps the templates well-formed)
template <> struct SplitP<0> : SplitP<1> {};

__device__ inline floatx4 mfma16x16(const bf16x8& a, const bf16x8& b, const floatx4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ inline floatx4 mfma16x16(const h16x8& a, const h16x8& b, const floatx4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ inline floatx16 mfma32x32(const bf16x8& a, const bf16x8& b, const floatx16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ inline floatx16 mfma32x32(const h16x8& a, const h16x8& b, const floatx16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// v_exp_f32 + v_rcp_f32 (1 ulp) instead of the IEEE division sequence
__device__ inline float tp_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ inline float tp_silu(float x) { return x * tp_sigmoid(x); }

// exact floor(a / b) for 0 <= a, b < 2^10 given inv = 1/b: one multiply instead of
// the ~20-instruction integer division sequence
__device__ inline int tp_udiv_small(int a, float inv) { return (int)(((float)a + 0.5f) * inv); }

// LDS-DMA copy of a weight image (nfloats a multiple of 256): one 1 KiB global_load_lds_dwordx4
// per wave-instruction, no VGPRs, all pieces in flight at once.  The caller drains with
// s_waitcnt vmcnt(0) + a barrier before reading the LDS.
template <int WAVES>
__device__ inline void tp_dma_image(const float* src, float* lds, int nfloats) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int pieces = nfloats >> 8;
    for (int p = wave; p < pieces; p += WAVES)
        __builtin_amdgcn_global_load_lds((const void*)(src + p * 256 + lane * 4),
                                         (__attribute__((address_space(3))) void*)(lds + p * 256), 16, 0, 0);
}

// offset (floats) of each sub-tile block inside one chunk image: KC = ceil(K/32) blocks of
// 32 x cw floats per sub-tile, scalar sub-tiles first, then the vector sub-tile
template <int NS>
__device__ inline void tp_img_offsets(const TpProb& P, int cw, int (&off)[NS + 1]) {
    int o = 0;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        off[j] = o;
        o += ((P.K[j] + 31) >> 5) * 32 * cw;
    }
    off[NS] = o;
}

template <int NS, int NV, int EPI, int WAVES = TP_WAVES, int D = 2, class SK = DynSK>
__global__ __launch_bounds__(64 * WAVES, (WAVES + 3) / 4) void tp_fused_kernel(const TpProb P) {
    constexpr int THREADS = 64 * WAVES;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    int chunk, blk;
    tp_block_map(P, (int)blockIdx.x, chunk, blk);
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, r = lane & 31, h = lane >> 5;

    int off[NS + 1];
    tp_img_offsets<NS>(P, 32, off);
    static_assert(SK::PREC == 0 || SK::on, "split-precision path needs a static schedule");
    static_assert(!SK::DV || (SK::PREC >= 1 && EPI == TP_MSG && NS == 3 && NV == 1 && SK::K0 == 2 * SK::KV &&
                              SK::K1 == 2 * SK::KV && SK::K2 == SK::KV),
                  "DV: message_layer_2's [m_s | m_v . rhat] scalar operand only");
    using SP = SplitP<SK::PREC>;
    using SPT = typename SP::T;
    constexpr int XBLK = SP::NP * 128;   // split parts x (m 2) x 64 lanes per 32-deep block (PREC 1: 384)
    const SPT* ldsx = reinterpret_cast<const SPT*>(lds);

    const int ks_chunks = (P.K[0] + 31) >> 5;            // K_S = K[0] (sub-tile 0 uses all of it)
    const int kv_chunks = NV ? (P.Kv + 31) >> 5 : 0;
    const float kv_inv = 1.0f / (float)(kv_chunks > 0 ? kv_chunks : 1);
    const int n_chunks = ks_chunks + 3 * kv_chunks;      // A chunks per row tile
    const int nc_pad = (n_chunks + D - 1) / D * D;       // chunk stream padded to the ring depth
    const int row_tiles = (P.rows + 31) >> 5;
    const int wstride = P.blocks_per_chunk * WAVES;
    const int wid = blk * WAVES + wave;                  // wave index within this chunk

    double st0 = 0.0, st1 = 0.0, st2 = 0.0;              // BN partial sums for column r
    // MSG epilogue operands that do not depend on the tile, loaded before the first K loop
    float ba = 0.f, bg = 0.f;
    const int lg = EPI == TP_MSG ? __builtin_ctz((unsigned)P.group) : 0;
    if constexpr (EPI == TP_MSG) {
        const int ch = chunk * 32 + r;
        if (ch < P.M) { ba = P.bias[ch]; bg = P.bias[P.M + ch]; }
    }

    // A-chunk loader: chunk i of a row tile -> 16 floats per lane (4 x dwordx4).  Bounds-checked
    // buffer loads, branch-free (invalid lanes, padding chunks and tiles past the end read zeros
    // through an out-of-range offset), so every load issues unconditionally and the waitcnt pass
    // can count the loads in flight.  Buffers are < 2 GiB (launch check).
    const __amdgpu_buffer_rsrc_t rsS = __builtin_amdgcn_make_buffer_rsrc((void*)P.As, (short)0, 0x7FFFFFF0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsV =
        __builtin_amdgcn_make_buffer_rsrc((void*)(NV ? P.Av : P.As), (short)0, 0x7FFFFFF0, 0x00020000);
    auto load_a = [&](int rt, int i, float4 (&a)[4]) {
        const int row = rt * 32 + r;
        const bool rok = row < P.rows && i < n_chunks;
        const bool sc = !NV || i < ks_chunks;                      // wave-uniform
        const int v = sc ? 0 : i - ks_chunks;
        const int plane = NV ? tp_udiv_small(v, kv_inv) : 0;
        const int k = (sc ? i * 32 : (v - plane * kv_chunks) * 32) + 16 * h;
        const bool ok = rok && k < (sc ? P.K[0] : P.Kv);
        const size_t eo = sc ? (size_t)row * P.lda_s + k
                             : (size_t)plane * P.plane_stride + (size_t)row * P.lda_v + k;
        const uint32_t off = ok ? (uint32_t)(eo * 4) : 0x7FFFFFF0u;
        const __amdgpu_buffer_rsrc_t rs = sc ? rsS : rsV;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            a[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? off + 16 * q : off, 0, 0));
    };

    // A ring of D chunk buffers with fixed roles: chunk i of a tile always lives in buf[i % D]
    // (the stream is padded to a multiple of D), and the load for chunk i + D - 1 is issued
    // before the MFMAs of chunk i.  The first D - 1 loads go out before the weight staging.
    const unsigned long long c_start = P.dbg ? clock64() : 0ull;
    const unsigned long long w_start = P.dbg ? wall_clock64() : 0ull;   // 100 MHz, chip-wide
    int rt = wid;
    float4 buf[D][4];
    // static schedule (SK::on): items = K0 scalar chunks, then KV chunks per vector plane
    constexpr int SNIT = SK::K0 + 3 * SK::KV;
    auto load_item = [&](auto ic, int rt_, float4 (&a)[4]) {
        constexpr int item = decltype(ic)::value;
        constexpr bool sc = item < SK::K0;
        constexpr int v = sc ? 0 : item - SK::K0;
        constexpr int plane = sc ? 0 : v / (SK::KV > 0 ? SK::KV : 1);
        constexpr int kc = sc ? item : v - plane * SK::KV;
        const int row = rt_ * 32 + r;
        const int k = kc * 32 + 16 * h;
        const bool ok = row < P.rows && k < (sc ? P.K[0] : P.Kv);
        const size_t eo = sc ? (size_t)row * P.lda_s + k : (size_t)plane * P.plane_stride + (size_t)row * P.lda_v + k;
        const uint32_t off = ok ? (uint32_t)(eo * 4) : 0x7FFFFFF0u;
        const __amdgpu_buffer_rsrc_t rs = sc ? rsS : rsV;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            a[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? off + 16 * q : off, 0, 0));
    };
    if constexpr (SK::on) {
        static_for<0, D - 1>([&](auto uc) {
            constexpr int u = decltype(uc)::value;   // load index (TpStream; = the item unless DV)
            if constexpr (u < TpStream<SK>::NLOAD)
                load_item(std::integral_constant<int, TpStream<SK>::item(TpStream<SK>::lpos(u))>{}, rt, buf[u % D]);
        });
    } else {
#pragma unroll
        for (int u = 0; u < D - 1; ++u) load_a(rt, u, buf[u]);
    }

    // ---- stage this chunk's weight image in LDS (LDS-DMA, verbatim copy)
    tp_dma_image<WAVES>(P.B + (size_t)chunk * P.img_floats, lds, P.img_floats);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long c_staged = P.dbg ? clock64() : 0ull;
    unsigned long long c_loop = 0ull;

    if (rt >= row_tiles) goto done;
    {
        while (true) {
            floatx16 acc[NS + 3 * NV];
#pragma unroll
            for (int j = 0; j < NS + 3 * NV; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
            const int next_rt = rt + wstride;
            // MSG: this tile's edge geometry (rhat) is fetched now and parked in LDS before the
            // epilogue, so the epilogue reads it without global-memory latency
            // (and, for the dot output, the node attributes of its 32 / group destinations)
            float4 gq = make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (EPI == TP_MSG) {
                const int grow = rt * 32 + r;
                if (h == 0 && grow < P.rows) gq = *reinterpret_cast<const float4*>(P.geom + (size_t)grow * 8);
                const int dst = ((rt * 32) >> lg) + r;
                if (h == 1 && P.out_dot && r < (32 >> lg) && dst < (P.rows >> lg))
                    gq = *reinterpret_cast<const float4*>(P.na + (size_t)dst * 4);
            }
            auto chunk_mma = [&](const float4 (&cur)[4], int i) {
                if (i < ks_chunks) {
                    const int k0 = i * 32;
#pragma unroll
                    for (int j = 0; j < NS; ++j) {
                        if (k0 >= P.K[j]) continue;
                        const float* bp = &lds[off[j] + i * 1024 + 4 * lane];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const float4 b4 = *reinterpret_cast<const float4*>(bp + 256 * q);
                            acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].x, b4.x, acc[j], 0, 0, 0);
                            acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].y, b4.y, acc[j], 0, 0, 0);
                            acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].z, b4.z, acc[j], 0, 0, 0);
                            acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].w, b4.w, acc[j], 0, 0, 0);
                        }
                    }
                } else if (NV && i < n_chunks) {
                    const int v = i - ks_chunks, plane = tp_udiv_small(v, kv_inv);
                    const int kc = v - plane * kv_chunks;
                    const float* bp = &lds[off[NS] + kc * 1024 + 4 * lane];
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl) {
                        if (pl != plane) continue;
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const float4 b4 = *reinterpret_cast<const float4*>(bp + 256 * q);
                            acc[NS + pl] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].x, b4.x, acc[NS + pl], 0, 0, 0);
                            acc[NS + pl] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].y, b4.y, acc[NS + pl], 0, 0, 0);
                            acc[NS + pl] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].z, b4.z, acc[NS + pl], 0, 0, 0);
                            acc[NS + pl] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].w, b4.w, acc[NS + pl], 0, 0, 0);
                        }
                    }
                }
            };
            // PREC 1 / 2: item u's A chunk, split into [part][m] (lane (r, h) holds k = 16 h + 4 q + e
            // of the chunk; MFMA m takes k = 16 h + 8 m + j)
            auto split_item = [&](const float4 (&cur)[4], SPT (&a)[SP::NP][2]) {
                SPT p0[SP::NP], p1[SP::NP];
                SP::split(cur[0], cur[1], p0);
                SP::split(cur[2], cur[3], p1);
#pragma unroll
                for (int p = 0; p < SP::NP; ++p) { a[p][0] = p0[p]; a[p][1] = p1[p]; }
            };
            auto mma_item_x3 = [&](auto ic, const SPT (&a)[SP::NP][2]) {
                constexpr int item = decltype(ic)::value;
                {
                    // block [p][m][lane][j]: smallest terms first
                    auto mma6 = [&](floatx16& c, int blk) {
                        const SPT* bp = ldsx + blk * XBLK + lane;
#pragma unroll
                        for (int m = 0; m < 2; ++m) {
                            SPT b[SP::NP];
#pragma unroll
                            for (int p = 0; p < SP::NP; ++p) b[p] = bp[(2 * p + m) * 64];
#pragma unroll
                            for (int tt = 0; tt < SP::NT; ++tt) c = mfma32x32(a[SP::TA[tt]][m], b[SP::TB[tt]], c);
                        }
                    };
                    // first block of each sub-tile (compile-time image offsets)
                    constexpr int OB[4] = {0, SK::K0, SK::K0 + SK::K1, SK::K0 + SK::K1 + SK::K2};
                    if constexpr (item < SK::K0) {
                        static_for<0, NS>([&](auto jc) {
                            constexpr int j = decltype(jc)::value;
                            constexpr int KCj = j == 0 ? SK::K0 : j == 1 ? SK::K1 : SK::K2;
                            if constexpr (item < KCj) mma6(acc[j], OB[j] + item);
                        });
                    } else {
                        constexpr int v = item - SK::K0, plane = v / SK::KV, kc = v - plane * SK::KV;
                        mma6(acc[NS + plane], OB[NS] + kc);
                    }
                }
            };
            auto compute_item = [&](auto ic, const float4 (&cur)[4]) {
                constexpr int item = decltype(ic)::value;
                if constexpr (item < SK::K0) {
                    static_for<0, NS>([&](auto jc) {
                        constexpr int j = decltype(jc)::value;
                        constexpr int KCj = j == 0 ? SK::K0 : j == 1 ? SK::K1 : SK::K2;
                        if constexpr (item < KCj) {
                            const float* bp = &lds[off[j] + item * 1024 + 4 * lane];
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const float4 b4 = *reinterpret_cast<const float4*>(bp + 256 * q);
                                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].x, b4.x, acc[j], 0, 0, 0);
                                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].y, b4.y, acc[j], 0, 0, 0);
                                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].z, b4.z, acc[j], 0, 0, 0);
                                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].w, b4.w, acc[j], 0, 0, 0);
                            }
                        }
                    });
                } else {
                    constexpr int v = item - SK::K0, plane = v / SK::KV, kc = v - plane * SK::KV;
                    const float* bp = &lds[off[NS] + kc * 1024 + 4 * lane];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float4 b4 = *reinterpret_cast<const float4*>(bp + 256 * q);
                        acc[NS + plane] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].x, b4.x, acc[NS + plane], 0, 0, 0);
                        acc[NS + plane] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].y, b4.y, acc[NS + plane], 0, 0, 0);
                        acc[NS + plane] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].z, b4.z, acc[NS + plane], 0, 0, 0);
                        acc[NS + plane] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[q].w, b4.w, acc[NS + plane], 0, 0, 0);
                    }
                }
            };
            if constexpr (SK::PREC >= 1) {
                // positions of the A stream (TpStream: with DV the dot chunks are formed, not loaded);
                // the split of position u + 1 runs in the shadow of position u's MFMAs (no barrier
                // between them)
                using TS = TpStream<SK>;
                float4 rh = make_float4(0.f, 0.f, 0.f, 0.f);   // DV: rhat of this lane's row
                float4 dacc[4];                                 // DV: the dot chunk being formed
                if constexpr (SK::DV) {
                    const int grow = rt * 32 + r;
                    if (grow < P.rows) rh = *reinterpret_cast<const float4*>(P.geom + (size_t)grow * 8);
                }
                auto dot_acc = [&](auto pc, const float4 (&cur)[4]) {
                    constexpr int pl = decltype(pc)::value;
                    const float rk = pl == 0 ? rh.x : pl == 1 ? rh.y : rh.z;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if constexpr (pl == 0) {
                            dacc[q] = make_float4(cur[q].x * rk, cur[q].y * rk, cur[q].z * rk, cur[q].w * rk);
                        } else {
                            dacc[q] = make_float4(__builtin_fmaf(cur[q].x, rk, dacc[q].x), __builtin_fmaf(cur[q].y, rk, dacc[q].y),
                                                  __builtin_fmaf(cur[q].z, rk, dacc[q].z), __builtin_fmaf(cur[q].w, rk, dacc[q].w));
                        }
                    }
                };
                auto pin4 = [&](float4 (&x)[4]) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        floatx4 v = __builtin_bit_cast(floatx4, x[q]);
                        asm volatile("" : "+v"(v));
                        x[q] = __builtin_bit_cast(float4, v);
                    }
                };
                SPT ax[2][SP::NP][2];
                split_item(buf[0], ax[0]);   // position 0 = load 0 (a scalar chunk)
                static_for<0, TS::NPOS>([&](auto uc) {
                    constexpr int u = decltype(uc)::value;
                    if constexpr (!TS::derived(u)) {
                        constexpr int l = TS::lidx(u);
                        if constexpr (l + D - 1 < TS::NLOAD)
                            load_item(std::integral_constant<int, TS::item(TS::lpos(l + D - 1))>{}, rt, buf[(l + D - 1) % D]);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    mma_item_x3(std::integral_constant<int, TS::item(u)>{}, ax[u % 2]);
                    if constexpr (u + 1 < TS::NPOS) {
                        // pin the split below the barrier (its pure arithmetic would otherwise be
                        // hoisted into the previous region by instruction selection)
                        if constexpr (TS::derived(u + 1)) {
                            pin4(dacc);
                            split_item(dacc, ax[(u + 1) % 2]);
                        } else {
                            constexpr int l1 = TS::lidx(u + 1);
                            pin4(buf[l1 % D]);
                            if constexpr (SK::DV && TS::plane(u + 1) >= 0)
                                dot_acc(std::integral_constant<int, TS::plane(u + 1)>{}, buf[l1 % D]);
                            split_item(buf[l1 % D], ax[(u + 1) % 2]);
                        }
                        // ... and its results above the next barrier (else they sink into the next block)
#pragma unroll
                        for (int p3 = 0; p3 < SP::NP; ++p3)
#pragma unroll
                            for (int m = 0; m < 2; ++m) asm volatile("" : "+v"(ax[(u + 1) % 2][p3][m]));
                        // spread the split's VALU over the MFMA gaps (<= ~5 per gap hide, MI355X_MICROARCH)
                        constexpr int it = TS::item(u);
                        constexpr int nsub = it < SK::K0 ? (it < SK::K2) + (it < SK::K1) + 1 : 1;
                        constexpr int nm = 2 * SP::NT * nsub;
                        constexpr int per = ((SK::PREC == 1 ? 120 : 64) + nm - 1) / nm;
                        static_for<0, nm>([&](auto) {
                            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                            __builtin_amdgcn_sched_group_barrier(0x002, per, 0);
                        });
                    }
                    __builtin_amdgcn_sched_barrier(0);
                });
                static_for<0, D - 1>([&](auto uc) {
                    constexpr int l = decltype(uc)::value;
                    if constexpr (l < TS::NLOAD)
                        load_item(std::integral_constant<int, TS::item(TS::lpos(l))>{}, next_rt, buf[l % D]);
                });
            } else if constexpr (SK::on) {
                static_for<0, SNIT>([&](auto uc) {
                    constexpr int u = decltype(uc)::value;
                    if constexpr (u + D - 1 < SNIT)
                        load_item(std::integral_constant<int, u + D - 1>{}, rt, buf[(u + D - 1) % D]);
                    __builtin_amdgcn_sched_barrier(0);
                    compute_item(std::integral_constant<int, u>{}, buf[u % D]);
                    __builtin_amdgcn_sched_barrier(0);
                });
                // the next tile's first chunks, behind this tile's epilogue
                static_for<0, D - 1>([&](auto uc) {
                    constexpr int u = decltype(uc)::value;
                    if constexpr (u < SNIT) load_item(std::integral_constant<int, u>{}, next_rt, buf[u % D]);
                });
            }
            for (int i0 = 0; !SK::on && i0 < nc_pad; i0 += D) {
#pragma unroll
                for (int u = 0; u < D; ++u) {
                    // prefetch chunk i0 + u + D - 1 (wrapping into the next tile) into the buffer
                    // the previous step consumed
                    int pi = i0 + u + D - 1, prt = rt;
                    if (pi >= nc_pad) { pi -= nc_pad; prt = next_rt; }
                    load_a(prt, pi, buf[(u + D - 1) % D]);
                    __builtin_amdgcn_sched_barrier(0);
                    chunk_mma(buf[u], i0 + u);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }

            if constexpr (SK::PREC == 2) {   // undo the fp16x2 image's weight scale
                float z = 0.f;
#pragma unroll
                for (int j = 0; j < NS + 3 * NV; ++j) {
                    acc[j] *= P.bscale;
#pragma unroll
                    for (int e = 0; e < 16; ++e) z = tp_nonfinite_fold(z, acc[j][e]);
                }
                tp_range_flag(P.range_flag, z);
            }
            if (P.dbg) c_loop = clock64();
            // ------------------------------------------------------------ epilogue
            const int ch = chunk * 32 + r;          // output channel of this lane's column
            const int row0 = rt * 32;
            if constexpr (EPI == TP_PLAIN) {
#pragma unroll
                for (int j = 0; j < NS; ++j) {
                    const int col = (chunk * NS + j) * 32 + r;
                    if (col < P.ncols) {
#pragma unroll
                        for (int e = 0; e < 16; ++e) {
                            const int row = row0 + (e & 3) + 8 * (e >> 2) + 4 * h;
                            if (row < P.rows) st_out<false>(&P.C[(size_t)row * P.ldc + col], acc[j][e]);
                        }
                    }
                }
            } else if constexpr (EPI == TP_MSG) {
                // rows are edges, dst-major, `group` (power of two) slots per destination
                const int M = P.M;
                const bool live = ch < M;
                float4* gl = reinterpret_cast<float4*>(lds + P.lds_floats) + wave * 64;   // [32 rows] rhat
                float4* gn = gl + 32;                                                     // [32 / group] na
                if (h == 0) gl[r] = gq; else gn[r] = gq;
                __builtin_amdgcn_wave_barrier();
                float ms[16], mv0[16], mv1[16], mv2[16];
                float f0 = 0.f, f1 = 0.f, f2 = 0.f;   // per-tile BN partials (16 rows), fp64 across tiles
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int rr = (e & 3) + 8 * (e >> 2) + 4 * h;
                    const int row = row0 + rr;
                    const float4 g = gl[rr];   // .w = |rel|, < 0 on a general graph's padding slots
                    const bool ok = live && row < P.rows && (row & (P.group - 1)) < P.valid_per_group && g.w >= 0.f;
                    const float s = kC_SILU * tp_silu(acc[0][e] + ba);
                    const float gg = kC_SIGMOID * tp_sigmoid(acc[1][e] + bg);
                    const float tt = acc[2][e];
                    ms[e] = ok ? s : 0.f;
                    mv0[e] = ok ? gg * (g.x * tt + acc[NS + 0][e]) : 0.f;
                    mv1[e] = ok ? gg * (g.y * tt + acc[NS + 1][e]) : 0.f;
                    mv2[e] = ok ? gg * (g.z * tt + acc[NS + 2][e]) : 0.f;
                    f0 += ms[e];
                    f1 += ms[e] * ms[e];
                    f2 += mv0[e] * mv0[e] + mv1[e] * mv1[e] + mv2[e] * mv2[e];
                }
                st0 += (double)f0;
                st1 += (double)f1;
                st2 += (double)f2;
                // aggregate the `group` consecutive rows of each destination (all indices
                // compile-time so the per-row arrays stay in registers)
                const int G = P.group;
                auto put = [&](int row, float a0, float a1, float a2, float a3) {
                    if (live && row < P.rows) {
                        const size_t o = (size_t)(row >> lg) * M + ch;
                        st_out<true>(&P.out_s[o], a0);
                        st_out<true>(&P.out_v[o], a1);
                        st_out<true>(&P.out_v[P.out_plane + o], a2);
                        st_out<true>(&P.out_v[2 * P.out_plane + o], a3);
                        if (P.out_dot) {
                            const float4 na4 = gn[(row - row0) >> lg];
                            st_out<true>(&P.out_dot[o], fmaf(a3, na4.w, fmaf(a2, na4.z, a1 * na4.y)));
                        }
                    }
                };
                if (G <= 4) {
#pragma unroll
                    for (int e0 = 0; e0 < 16; e0 += 4) {
#pragma unroll
                        for (int s0 = 0; s0 < 4; ++s0) {
                            if (s0 % G) continue;
                            float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                if (s0 + u >= 4 || u >= G) continue;
                                a0 += ms[e0 + s0 + u]; a1 += mv0[e0 + s0 + u];
                                a2 += mv1[e0 + s0 + u]; a3 += mv2[e0 + s0 + u];
                            }
                            put(row0 + s0 + 8 * (e0 >> 2) + 4 * h, a0, a1, a2, a3);
                        }
                    }
                } else {
                    // 8/16/32-row groups: (h, e&3) covers 8 rows, e>>2 selects the 8-row block
                    float b0[4], b1[4], b2[4], b3[4];
#pragma unroll
                    for (int b8 = 0; b8 < 4; ++b8) {
                        b0[b8] = ms[4 * b8] + ms[4 * b8 + 1] + ms[4 * b8 + 2] + ms[4 * b8 + 3];
                        b1[b8] = mv0[4 * b8] + mv0[4 * b8 + 1] + mv0[4 * b8 + 2] + mv0[4 * b8 + 3];
                        b2[b8] = mv1[4 * b8] + mv1[4 * b8 + 1] + mv1[4 * b8 + 2] + mv1[4 * b8 + 3];
                        b3[b8] = mv2[4 * b8] + mv2[4 * b8 + 1] + mv2[4 * b8 + 2] + mv2[4 * b8 + 3];
                        b0[b8] += __shfl_xor(b0[b8], 32); b1[b8] += __shfl_xor(b1[b8], 32);
                        b2[b8] += __shfl_xor(b2[b8], 32); b3[b8] += __shfl_xor(b3[b8], 32);
                    }
                    const int nb = G / 8;
#pragma unroll
                    for (int gb = 0; gb < 4; ++gb) {
                        if (gb % nb) continue;
                        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
                        for (int b8 = 0; b8 < 4; ++b8) {
                            if (b8 < gb || b8 >= gb + nb) continue;
                            a0 += b0[b8]; a1 += b1[b8]; a2 += b2[b8]; a3 += b3[b8];
                        }
                        if (h == 0) put(row0 + 8 * gb, a0, a1, a2, a3);
                    }
                }
            } else if constexpr (EPI == TP_GATE_NODE) {
                // rows are nodes; writes the next TP's inputs [h_s | h_v . na] and h_v planes
                const int M = P.M;
                const bool live = ch < M;
                const float ba = live ? P.bias[ch] : 0.f, bg = live ? P.bias[M + ch] : 0.f;
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int row = row0 + (e & 3) + 8 * (e >> 2) + 4 * h;
                    if (!live || row >= P.rows) continue;
                    const float* na = P.geom + (size_t)row * 4;
                    const float hs = kC_SILU * tp_silu(acc[0][e] + ba);
                    const float gg = kC_SIGMOID * tp_sigmoid(acc[1][e] + bg);
                    const float tt = acc[2][e];
                    const float h0 = gg * (na[1] * tt + acc[NS + 0][e]);
                    const float h1 = gg * (na[2] * tt + acc[NS + 1][e]);
                    const float h2 = gg * (na[3] * tt + acc[NS + 2][e]);
                    st_out<false>(&P.out_s[(size_t)row * 2 * M + ch], hs);
                    st_out<false>(&P.out_s[(size_t)row * 2 * M + M + ch], h0 * na[1] + h1 * na[2] + h2 * na[3]);
                    st_out<false>(&P.out_v[(size_t)row * M + ch], h0);
                    st_out<false>(&P.out_v[P.out_plane + (size_t)row * M + ch], h1);
                    st_out<false>(&P.out_v[2 * P.out_plane + (size_t)row * M + ch], h2);
                }
            } else if constexpr (EPI == TP_RESID) {
                // rows are nodes: x += update (update_layer_2 output), BN partial sums of the new x
                const int M = P.M;
                const bool live = ch < M;
                const float b = live ? P.bias[ch] : 0.f;
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int row = row0 + (e & 3) + 8 * (e >> 2) + 4 * h;
                    if (!live || row >= P.rows) continue;
                    const float* na = P.geom + (size_t)row * 4;
                    const float tt = acc[1][e];
                    float* xs = P.out_s + (size_t)row * M + ch;
                    const float s = *xs + (acc[0][e] + b);
                    st_out<false>(xs, s);
                    float* x0 = P.out_v + (size_t)row * M + ch;
                    float* x1 = x0 + P.out_plane;
                    float* x2 = x1 + P.out_plane;
                    const float v0 = *x0 + (na[1] * tt + acc[NS + 0][e]);
                    const float v1 = *x1 + (na[2] * tt + acc[NS + 1][e]);
                    const float v2 = *x2 + (na[3] * tt + acc[NS + 2][e]);
                    st_out<false>(x0, v0); st_out<false>(x1, v1); st_out<false>(x2, v2);
                    st0 += (double)s;
                    st1 += (double)s * s;
                    st2 += (double)v0 * v0 + (double)v1 * v1 + (double)v2 * v2;
                }
            }
            rt = next_rt;
            if (rt >= row_tiles) break;
        }
    }
done:
    if (P.dbg && lane == 0) {
        unsigned long long* d = P.dbg + ((size_t)blockIdx.x * WAVES + wave) * 6;
        d[0] = c_start; d[1] = c_staged; d[2] = c_loop; d[3] = clock64();
        d[4] = w_start; d[5] = wall_clock64();
    }
    if constexpr (EPI == TP_MSG || EPI == TP_RESID) {
        // reduce the block's waves in LDS: one partial row per block, layout [chunk][block][3][32]
        __syncthreads();
        double* red = reinterpret_cast<double*>(lds);   // [3][WAVES][32]
        st0 += __shfl_xor(st0, 32);
        st1 += __shfl_xor(st1, 32);
        st2 += __shfl_xor(st2, 32);
        if (h == 0) {
            red[(0 * WAVES + wave) * 32 + r] = st0;
            red[(1 * WAVES + wave) * 32 + r] = st1;
            red[(2 * WAVES + wave) * 32 + r] = st2;
        }
        __syncthreads();
        if (t < 96) {
            const int st = t / 32, c = t % 32;
            double acc = 0.0;
            for (int w = 0; w < WAVES; ++w) acc += red[(st * WAVES + w) * 32 + c];
            if (P.bn_sums) {
                const int ch = chunk * 32 + c;
                if (ch < P.M) bn_atomic_add(P.bn_sums + st * P.M + ch, acc);
            } else {
                P.partial[((size_t)chunk * P.blocks_per_chunk + blk) * 96 + st * 32 + c] = acc;
            }
        }
    }
}

// floats of one chunk image (cw = channels per chunk: 32 here, 16 for tp16)
inline int tp_img_floats(const TpProb& p, int cw) {
    int n = 0;
    for (int j = 0; j < p.NS; ++j) n += ((p.K[j] + 31) / 32) * 32 * cw;
    if (p.NV) n += ((p.Kv + 31) / 32) * 32 * cw;
    return n;
}

inline int tp_lds_floats(const TpProb& p) { return tp_img_floats(p, 32); }

// Grid: `blocks_per_chunk` blocks per 32-channel chunk, chosen to fill the CUs
// (as many blocks per CU as the LDS footprint allows) without idle waves.
// prec 1: bf16x3 image, 1.5x the floats of the fp32 one.
inline void tp_geometry(TpProb& p, int waves = TP_WAVES, int num_cus = 256, int prec = 0) {
    p.img_floats = tp_img_floats(p, 32) * (prec == 1 ? 3 : 2) / 2;   // bf16x3: 1.5x the fp32 floats; fp16x2: the same
    p.lds_floats = p.img_floats;
    const int lds_bytes = p.lds_floats * 4;
    int per_cu = (160 * 1024) / (lds_bytes > 0 ? lds_bytes : 1);
    if (per_cu < 1) per_cu = 1;
    if (per_cu > 16 / waves) per_cu = 16 / waves > 0 ? 16 / waves : 1;  // at most 16 waves / CU
    const int row_tiles = (p.rows + 31) / 32;
    int bpc = (num_cus * per_cu + p.chunks - 1) / p.chunks;
    const int max_bpc = (row_tiles + waves - 1) / waves;
    if (bpc > max_bpc) bpc = max_bpc;
    if (bpc < 1) bpc = 1;
    p.blocks_per_chunk = bpc;
    p.waves_per_chunk = bpc;  // partial rows per chunk (one per block)
    p.xcd_groups = (p.chunks > 1 && bpc % 8 == 0) ? p.chunks : 0;
}

template <int NS, int NV, int EPI, int WAVES = TP_WAVES, int D = 2, class SK = DynSK>
int tp_launch(const TpProb& p, hipStream_t st) {
    if (p.rows <= 0 || p.chunks <= 0) return NBX_OK;
    if ((double)p.rows * p.lda_s * 4.0 >= 2147483632.0 ||
        (p.NV && ((double)p.plane_stride * 3 + (double)p.rows * p.lda_v) * 4.0 >= 2147483632.0)) {
        set_error("tp: A operand spans >= 2 GiB (32-bit buffer offsets)");
        return NBX_E_UNSUPPORTED;
    }
    const size_t lds = (size_t)p.lds_floats * 4 + (EPI == TP_MSG ? (size_t)WAVES * 64 * 16 : 0);
    if (lds > 160 * 1024) {
        set_error("tp_fused: weight chunk needs %zu bytes of LDS (> 160 KiB)", lds);
        return NBX_E_UNSUPPORTED;
    }
    NBX_LDS_160K((tp_fused_kernel<NS, NV, EPI, WAVES, D, SK>));
    if constexpr (SK::on) {
        auto kc = [](int K) { return (K + 31) / 32; };
        if (!(kc(p.K[0]) == SK::K0 && (NS < 2 || kc(p.K[1]) == SK::K1) && (NS < 3 || kc(p.K[2]) == SK::K2) &&
              (NV ? kc(p.Kv) : 0) == SK::KV)) {
            set_error("tp_fused: static chunk schedule does not match the problem's K");
            return NBX_E_INVAL;
        }
    }
    NBX_TIMED_LAUNCH((tp_fused_kernel<NS, NV, EPI, WAVES, D, SK>), dim3(p.chunks * p.blocks_per_chunk), dim3(64 * WAVES),
                     lds, st, p);
    NBX_HIP(hipGetLastError());
    return NBX_OK;
}

}  // namespace nbx
