// PONITA fibre-bundle forward + device-resident self-feed rollout (fp32).
//
// Reference: models/ponita/ponita_nbody.py:82-95, models/ponita/models/ponita_pg.py:134-192,
// transforms/position_orientation_graph.py:58-87, geometry/invariants.py:9-51,
// nn/embedding.py:4-15, nn/conv.py:65-140, nn/convnext.py:4-32, utils/to_from_sphere.py:4-14,
// helper_scripts/infer_self_feed.py:131-147 (graph prep), 182-194 (rollout update).
//
// Layout.  Node-orientation rows (v, o) -> v*O + o, features C contiguous.  Edge rows are
// destination-major with G = next_pow2(N-1) slots per node and the orientation in between:
// row (d, o, q) -> (d*O + o)*G + q, so the G messages a (d, o) fibre point receives are
// consecutive rows of one MFMA tile and the aggregation is an in-register sum (lin.h
// LIN_CONV).  General graphs (kNN, any simple within-system edge_index): SLOT [V][G] names the
// source of each slot (csrc/graph.hip), -1 padding.  Per forward:
//   attr    : P16[(d,o,q)] = poly3(rel . ori_o, |rel - (rel . ori_o) ori_o|)       (14 of 16)
//   basis   : KB = GELU(GELU(P16 Wb1' + b) Wb2' + b)        cached for all layers (E*O x Bk)
//   fibre   : FK_l = GELU(GELU(poly3(ori_o . ori_p) Wf1' + b) Wf2' + b) Wfk_l'  (O*O x L*C)
//   lift    : X = [mass, vel . ori_o] Wemb'
//   layer l : X1 = sum_q (KB Wk_l')[(d,o,q)] * X[(src,o)]            (MFMA + fused gather/sum)
//             XN = LayerNorm(sum_o X1[d,o] * FK_l[o,p] / O + bias)     (fibre conv, VALU)
//             X  = X + s * (GELU(XN W1' + b1) W2' + b2)                (MFMA, residual epilogue)
//             RO += X Wro_l' + bro_l                                   (readout, 2 channels)
//   out     : sum_o (RO / #readouts)[v,o,c] * ori_o / O  -> [V, 6]
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <cstdio>
#include <vector>

#include "launch_timer.h"
#include "lin.h"
#include "nbx_internal.h"
#include "rollout_state.h"

namespace {

constexpr int PO_OMAX = 24;

unsigned g1(int64_t n) { return (unsigned)nbx::ceil_div(n > 0 ? n : 1, 256); }

// invariant_attr_r3s2_fiber_bundle (separable) + PolynomialFeatures(3) per edge slot.
__global__ void po_attr_kernel(const float* __restrict__ pos, const float* __restrict__ ori, int64_t R, int N, int O,
                               int G, float* __restrict__ P16, const int* __restrict__ slot) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= R) return;
    const int q = (int)(r % G);
    const int64_t t = r / G;
    const int o = (int)(t % O);
    const int64_t d = t / O;
    float f[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) f[i] = 0.f;
    const int dl = (int)(d % N);
    const int sq = slot ? slot[d * G + q] : (q < N - 1 ? (q < dl ? q : q + 1) : -1);
    if (sq >= 0) {
        const int64_t s = d - dl + sq;
        const float rx = pos[3 * s] - pos[3 * d], ry = pos[3 * s + 1] - pos[3 * d + 1],
                    rz = pos[3 * s + 2] - pos[3 * d + 2];
        const float ox = ori[3 * o], oy = ori[3 * o + 1], oz = ori[3 * o + 2];
        const float a = rx * ox + ry * oy + rz * oz;
        const float ux = rx - a * ox, uy = ry - a * oy, uz = rz - a * oz;
        const float b = sqrtf(ux * ux + uy * uy + uz * uz);
        const float x[2] = {a, b};
        f[0] = a;
        f[1] = b;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) f[2 + 2 * i + j] = f[i] * x[j];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) f[6 + 2 * i + j] = f[2 + i] * x[j];
    }
    float4* dst = reinterpret_cast<float4*>(P16 + r * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[i] = make_float4(f[4 * i], f[4 * i + 1], f[4 * i + 2], f[4 * i + 3]);
}

// fibre invariant ori_o . ori_p -> PolynomialFeatures(3) = [s, s^2, s^3, 0]
__global__ void po_fattr_kernel(const float* __restrict__ ori, int O, float* __restrict__ FP) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= O * O) return;
    const int i = r / O, j = r - i * O;
    const float s = ori[3 * j] * ori[3 * i] + ori[3 * j + 1] * ori[3 * i + 1] + ori[3 * j + 2] * ori[3 * i + 2];
    const float s2 = s * s;
    FP[4 * r] = s;
    FP[4 * r + 1] = s2;
    FP[4 * r + 2] = s2 * s;
    FP[4 * r + 3] = 0.f;
}

// scalar_to_sphere / vec_to_sphere lift + x_embedder (no bias): X[(v,o), c]
__global__ void po_lift_kernel(const float* __restrict__ mass, const float* __restrict__ vel,
                               const float* __restrict__ ori, const float* __restrict__ We, int64_t V, int O, int C,
                               float* __restrict__ X) {
    // thread = (fibre point row = v O + o, 4 channels): one 32-bit division per thread and a float4
    // store (the per-element 64-bit index arithmetic ran this pure write at 1.5 TB/s)
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int CQ = C >> 2;
    if (i >= V * O * CQ) return;
    const int64_t row = i / CQ;   // C / 4 is a power of two: a shift
    const int c = 4 * (int)(i - row * CQ);
    const int v = (int)(row / O), o = (int)(row - (int64_t)v * O);
    const float f1 = vel[3 * v] * ori[3 * o] + vel[3 * v + 1] * ori[3 * o + 1] + vel[3 * v + 2] * ori[3 * o + 2];
    const float m = mass[v];
    const float4 w01 = *reinterpret_cast<const float4*>(We + 2 * c), w23 = *reinterpret_cast<const float4*>(We + 2 * c + 4);
    *reinterpret_cast<float4*>(X + row * C + c) =
        float4{m * w01.x + f1 * w01.y, m * w01.z + f1 * w01.w, m * w23.x + f1 * w23.y, m * w23.z + f1 * w23.w};
}

__device__ inline double block_sum_double(double v, double* red) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) red[wv] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0)
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
    __syncthreads();
    return s;
}

// (sum, sum of squares) in fp64 for FiberBundleConv.callibrate's std()s
__global__ void po_moments_kernel(const float* __restrict__ x, int64_t n, double* __restrict__ m) {
    __shared__ double red[16];
    double s1 = 0.0, s2 = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double v = x[i];
        s1 += v;
        s2 += v * v;
    }
    s1 = block_sum_double(s1, red);
    s2 = block_sum_double(s2, red);
    if (threadIdx.x == 0) {
        atomicAdd(&m[0], s1);
        atomicAdd(&m[1], s2);
    }
}

// Depthwise fibre convolution + conv bias + LayerNorm (conv.py:121-124, convnext.py:18):
//   y[d,p,c] = sum_o X1[d,o,c] * FK[o,p,c] / O + bias[c];  XN[d,p] = LN_c(y[d,p])
// Block (x: node groups, y: orientation range [p0, p0+PR)) keeps FK[:, p0:p0+PR, :] in LDS.
// A thread owns (node, 4 channels): it loads X1[d, :, c..c+3] once (coalesced rows) and
// produces its channels of every p in the range; the C/4 lanes of a node reduce the
// LayerNorm moments with shuffles.  X1 is re-read once per orientation range (O/PR times,
// from L2 / MALL), FK never leaves LDS.
constexpr int PO_FIB_THREADS = 512;

template <int OMAX, int MINW>
__global__ __launch_bounds__(PO_FIB_THREADS, MINW) void po_fiber_ln_kernel(
    const float* __restrict__ X1, const float* __restrict__ FK, int ldfk, const float* __restrict__ cbias,
    const float* __restrict__ nw, const float* __restrict__ nb, int64_t V, int O, int C, int PR,
    float* __restrict__ XN, double* __restrict__ mom) {
    extern __shared__ __attribute__((aligned(16))) float fks[];
    __shared__ double red[16];
    const int CG = C >> 2, npi = PO_FIB_THREADS / CG;
    const int t = threadIdx.x, ns = t / CG, cg = t - ns * CG, c = 4 * cg;
    const int p0 = blockIdx.y * PR, pn = min(PR, O - p0);
    // FK slice -> LDS [o][pl][C], addressed as float4 so every access is one 16-byte LDS op
    // (float indices with a run-time C let the compiler split them into ds_read2_b32 pairs,
    // which bank-conflict 4-way: 70 % of the kernel's LDS cycles were conflicts)
    float4* fk4 = reinterpret_cast<float4*>(fks);
    for (int i = t; i < O * pn * CG; i += PO_FIB_THREADS) {
        const int o = i / (pn * CG), r = i - o * pn * CG, pl = r / CG, q = r - pl * CG;
        fk4[(o * PR + pl) * CG + q] = *reinterpret_cast<const float4*>(FK + (size_t)(o * O + p0 + pl) * ldfk + 4 * q);
    }
    __syncthreads();
    const float4 cb = *reinterpret_cast<const float4*>(cbias + c);
    const float4 w4 = *reinterpret_cast<const float4*>(nw + c);
    const float4 b4 = *reinterpret_cast<const float4*>(nb + c);
    const float invO = 1.0f / (float)O, invC = 1.0f / (float)C;
    double s1 = 0.0, s2 = 0.0;
    for (int64_t d0 = (int64_t)blockIdx.x * npi; d0 < V; d0 += (int64_t)gridDim.x * npi) {
        const int64_t d = d0 + ns;
        const bool active = d < V;
        float4 x[OMAX];
        const float* x1 = X1 + (size_t)(active ? d : 0) * O * C + c;
#pragma unroll
        for (int o = 0; o < OMAX; ++o)
            x[o] = (o < O) ? *reinterpret_cast<const float4*>(x1 + (size_t)o * C) : make_float4(0.f, 0.f, 0.f, 0.f);
        for (int pl = 0; pl < pn; ++pl) {
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int o = 0; o < OMAX; ++o) {
                if (o < O) {
                    const float4 f = fk4[(o * PR + pl) * CG + cg];
                    a.x += x[o].x * f.x;
                    a.y += x[o].y * f.y;
                    a.z += x[o].z * f.z;
                    a.w += x[o].w * f.w;
                }
            }
            a.x *= invO; a.y *= invO; a.z *= invO; a.w *= invO;
            if (mom && active) {
                s1 += (double)a.x + (double)a.y + (double)a.z + (double)a.w;
                s2 += (double)a.x * a.x + (double)a.y * a.y + (double)a.z * a.z + (double)a.w * a.w;
            }
            const float y0 = a.x + cb.x, y1 = a.y + cb.y, y2 = a.z + cb.z, y3 = a.w + cb.w;
            float s = y0 + y1 + y2 + y3;
            for (int off = CG >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off);
            const float mu = s * invC;
            const float e0 = y0 - mu, e1 = y1 - mu, e2 = y2 - mu, e3 = y3 - mu;
            float v = e0 * e0 + e1 * e1 + e2 * e2 + e3 * e3;
            for (int off = CG >> 1; off > 0; off >>= 1) v += __shfl_xor(v, off);
            const float rs = 1.0f / sqrtf(v * invC + 1e-5f);
            if (active)
                *reinterpret_cast<float4*>(XN + ((size_t)d * O + p0 + pl) * C + c) =
                    make_float4(e0 * rs * w4.x + b4.x, e1 * rs * w4.y + b4.y, e2 * rs * w4.z + b4.z,
                                e3 * rs * w4.w + b4.w);
        }
    }
    if (mom) {
        s1 = block_sum_double(s1, red);
        s2 = block_sum_double(s2, red);
        if (threadIdx.x == 0) {
            atomicAdd(&mom[0], s1);
            atomicAdd(&mom[1], s2);
        }
    }
}

// One-pass variant: X1 is read from HBM exactly once.  A block walks node tiles (npi nodes of C/4
// lanes each); for every tile it keeps X1[d, :, c..c+3] in registers and runs through ALL the
// orientation ranges, the FK slices streaming through two LDS buffers: range k+1's slice is DMA-ed
// (global_load_lds, 16 B per lane, no registers) into the other buffer while range k is computed,
// one barrier per range.  The slices are re-fetched per tile from L2 (FK is 200 KB, L2-resident),
// so HBM sees X1 once and XN once: the algorithmic traffic.  LDS slice layout [o][pl][C/4] float4
// with the range's own width pn (so the DMA destination is linear).
template <int OMAX, int MINW, int NT = PO_FIB_THREADS>
__global__ __launch_bounds__(NT, MINW) void po_fiber_ln1_kernel(
    const float* __restrict__ X1, const float* __restrict__ FK, int ldfk, const float* __restrict__ cbias,
    const float* __restrict__ nw, const float* __restrict__ nb, int64_t V, int O, int C, int PR, int slice4,
    float* __restrict__ XN, double* __restrict__ mom) {
    extern __shared__ __attribute__((aligned(16))) float fks[];
    __shared__ double red[16];
    const int CG = C >> 2, npi = NT / CG;
    const int t = threadIdx.x, ns = t / CG, cg = t - ns * CG, c = 4 * cg;
    const int wave = t >> 6, lane = t & 63;
    const int R = (O + PR - 1) / PR;
    float4* fk4 = reinterpret_cast<float4*>(fks);
    // DMA range r's slice into buffer b: element i = (o pn + pl) CG + q <- FK row (o O + p0 + pl), float4 q
    auto dma = [&](int r, int b) {
        const int p0 = r * PR, pn = min(PR, O - p0), n = O * pn * CG, per_o = pn * CG;
        for (int piece = wave; piece * 64 < n; piece += NT / 64) {
            int i = piece * 64 + lane;
            i = i < n ? i : n - 1;                        // tail lanes re-read a valid element
            const int o = i / per_o, rr = i - o * per_o, pl = rr / CG, q = rr - pl * CG;
            __builtin_amdgcn_global_load_lds((const void*)(FK + (size_t)(o * O + p0 + pl) * ldfk + 4 * q),
                                             (__attribute__((address_space(3))) void*)(fk4 + b * slice4 + piece * 64),
                                             16, 0, 0);
        }
    };
    const float4 cb = *reinterpret_cast<const float4*>(cbias + c);
    const float4 w4 = *reinterpret_cast<const float4*>(nw + c);
    const float4 b4 = *reinterpret_cast<const float4*>(nb + c);
    const float invO = 1.0f / (float)O, invC = 1.0f / (float)C;
    double s1 = 0.0, s2 = 0.0;
    const int64_t first = (int64_t)blockIdx.x * npi, step_d = (int64_t)gridDim.x * npi;
    if (first < V) dma(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int bsel = 0;                         // LDS buffer holding the current range
    for (int64_t d0 = first; d0 < V; d0 += step_d) {
        const int64_t d = d0 + ns;
        const bool active = d < V;
        float4 x[OMAX];
        const float* x1 = X1 + (size_t)(active ? d : 0) * O * C + c;
#pragma unroll
        for (int o = 0; o < OMAX; ++o)
            x[o] = (o < O) ? *reinterpret_cast<const float4*>(x1 + (size_t)o * C) : make_float4(0.f, 0.f, 0.f, 0.f);
        const bool more_tiles = d0 + step_d < V;
        for (int r = 0; r < R; ++r) {
            if (r + 1 < R || more_tiles) dma(r + 1 < R ? r + 1 : 0, bsel ^ 1);   // the next step's slice
            const int p0 = r * PR, pn = min(PR, O - p0);
            const float4* sl = fk4 + bsel * slice4;
            for (int pl = 0; pl < pn; ++pl) {
                float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int o = 0; o < OMAX; ++o) {
                    if (o < O) {
                        const float4 f = sl[(o * pn + pl) * CG + cg];
                        a.x += x[o].x * f.x;
                        a.y += x[o].y * f.y;
                        a.z += x[o].z * f.z;
                        a.w += x[o].w * f.w;
                    }
                }
                a.x *= invO; a.y *= invO; a.z *= invO; a.w *= invO;
                if (mom && active) {
                    s1 += (double)a.x + (double)a.y + (double)a.z + (double)a.w;
                    s2 += (double)a.x * a.x + (double)a.y * a.y + (double)a.z * a.z + (double)a.w * a.w;
                }
                const float y0 = a.x + cb.x, y1 = a.y + cb.y, y2 = a.z + cb.z, y3 = a.w + cb.w;
                float s = y0 + y1 + y2 + y3;
                for (int off = CG >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off);
                const float mu = s * invC;
                const float e0 = y0 - mu, e1 = y1 - mu, e2 = y2 - mu, e3 = y3 - mu;
                float v = e0 * e0 + e1 * e1 + e2 * e2 + e3 * e3;
                for (int off = CG >> 1; off > 0; off >>= 1) v += __shfl_xor(v, off);
                const float rs = 1.0f / sqrtf(v * invC + 1e-5f);
                if (active)
                    *reinterpret_cast<float4*>(XN + ((size_t)d * O + p0 + pl) * C + c) =
                        make_float4(e0 * rs * w4.x + b4.x, e1 * rs * w4.y + b4.y, e2 * rs * w4.z + b4.z,
                                    e3 * rs * w4.w + b4.w);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            bsel ^= 1;
        }
    }
    if (mom) {
        s1 = block_sum_double(s1, red);
        s2 = block_sum_double(s2, red);
        if (threadIdx.x == 0) {
            atomicAdd(&mom[0], s1);
            atomicAdd(&mom[1], s2);
        }
    }
}

// read_out_layers[l]: RO[row, k] (+)= X[row] . Wro[k] + bro[k], k < 2; C/4 lanes per row
__global__ void po_readout_kernel(const float* __restrict__ X, const float* __restrict__ Wro,
                                  const float* __restrict__ bro, int64_t rows, int C, int first,
                                  float* __restrict__ RO) {
    // thread = (row, 16 channels): four float4 loads in flight per thread and a log2(C / 16)-level
    // reduction over the row's lanes (one float4 per thread and log2(C / 4) levels ran at 3.4 TB/s)
    const int LPR = C >> 4;   // lanes per row (C = 32, 64, 128 -> 2, 4, 8)
    const int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t row = g / LPR;
    const int j = (int)(g - row * LPR);
    float d0 = 0.f, d1 = 0.f;
    if (row < rows) {
        const float4* x = reinterpret_cast<const float4*>(X + row * C + 16 * j);
        const float4* w0 = reinterpret_cast<const float4*>(Wro + 16 * j);
        const float4* w1 = reinterpret_cast<const float4*>(Wro + C + 16 * j);
        float4 xv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) xv[q] = x[q];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 a = w0[q], b = w1[q];
            d0 += xv[q].x * a.x + xv[q].y * a.y + xv[q].z * a.z + xv[q].w * a.w;
            d1 += xv[q].x * b.x + xv[q].y * b.y + xv[q].z * b.z + xv[q].w * b.w;
        }
    }
    for (int off = LPR >> 1; off > 0; off >>= 1) {
        d0 += __shfl_xor(d0, off);
        d1 += __shfl_xor(d1, off);
    }
    if (row < rows && j == 0) {
        const float r0 = d0 + bro[0], r1 = d1 + bro[1];
        RO[2 * row] = first ? r0 : RO[2 * row] + r0;
        RO[2 * row + 1] = first ? r1 : RO[2 * row + 1] + r1;
    }
}

// mean of readouts -> sphere_to_vec: out[v, 3c + k] = sum_o (RO[v,o,c] / nro) ori[o,k] / O
__global__ void po_out_kernel(const float* __restrict__ RO, const float* __restrict__ ori, int64_t V, int O, int nro,
                              float* __restrict__ out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= V * 6) return;
    const int64_t v = i / 6;
    const int j = (int)(i - v * 6), c = j / 3, k = j - 3 * c;
    const float inv = 1.0f / (float)nro;
    float s = 0.f;
    for (int o = 0; o < O; ++o) s += (RO[(v * O + o) * 2 + c] * inv) * ori[3 * o + k];
    out[i] = s / (float)O;
}

struct PoDims {
    int64_t B, N, V, G, R;  // R = V*O*G edge-orientation rows
    int O, C, Bk, mlp, L;
};

struct PoWs {
    float *P16, *B1H1, *KB, *FP, *FB1, *FKB, *FK, *X, *X1, *XN, *RO, *out;
    int* SLOT;                 // general graphs: [V*G] source per slot
    float* DEG;                // [V] in-degree (unused by the model: FiberBundleConv sums)
    unsigned long long* ADJ;   // [V]
    int* ERR;                  // [64]
    int* RANGE;                // [64]: the call's fp16x2 range flag (tp_fused.h tp_range_flag)
};

int next_pow2(int x) {
    int g = 1;
    while (g < x) g <<= 1;
    return g;
}

PoDims po_dims(const nbx_ponita_weights* w, int64_t B, int64_t N) {
    PoDims d;
    d.B = B; d.N = N; d.V = B * N;
    d.G = next_pow2((int)(N > 1 ? N - 1 : 1));
    d.O = w->num_ori; d.C = w->hidden; d.Bk = w->basis_dim; d.mlp = w->widening * w->hidden; d.L = w->num_layers;
    d.R = d.V * d.O * d.G;
    return d;
}

size_t po_carve(PoWs* ws, void* base, const PoDims& d) {
    size_t off = 0;
    auto take = [&](size_t n) -> float* {
        off = (off + 255) & ~size_t(255);
        float* p = base ? (float*)((char*)base + off) : nullptr;
        off += n * 4;
        return p;
    };
    const size_t VO = (size_t)d.V * d.O, OO = (size_t)d.O * d.O;
    PoWs w;
    w.P16 = take((size_t)d.R * 16);
    w.B1H1 = take(std::max((size_t)d.R * d.C, VO * d.mlp));
    w.KB = take((size_t)d.R * d.Bk);
    w.FP = take(OO * 4);
    w.FB1 = take(OO * d.C);
    w.FKB = take(OO * d.Bk);
    w.FK = take(OO * (size_t)d.L * d.C);
    w.X = take(VO * d.C);
    w.X1 = take(VO * d.C);
    w.XN = take(VO * d.C);
    w.RO = take(VO * 2);
    w.out = take((size_t)d.V * 6);
    w.SLOT = (int*)take((size_t)d.V * d.G);
    w.DEG = take((size_t)d.V);
    w.ADJ = (unsigned long long*)take((size_t)d.V * 2);
    w.ERR = (int*)take(64);
    w.RANGE = (int*)take(64);
    if (ws) *ws = w;
    return (off + 255) & ~size_t(255);
}

inline int kp(int k) { return (k + 31) & ~31; }

// ---- fused ConvNext MLP (nn/convnext.py:19-27): X = X + s * (GELU(XN W1' + b1) W2' + b2), with the
// [rows][4C] hidden activation kept in registers.  A workgroup owns FFN_WAVES x 32 fibre-point rows;
// each wave holds its 32 x C input rows pre-split into bf16x3 MFMA operands and walks the hidden
// dimension in 32-wide chunks j:
//   GEMM 1  D1 = W1[32j..32j+31, :] x XN^T (32 hidden x 32 rows, v_mfma_f32_32x32x16_bf16 with the
//           weights as the A operand), so lane (row = lane & 31, h = lane >> 5) ends up holding
//           hidden units (e & 3) + 8 (e >> 2) + 4 h of its own row in register e;
//   GELU    + b1 (branch-free erfc form), split into bf16x3 in place: registers 8m..8m+7 are the A
//           operand of MFMA step m;
//   GEMM 2  acc[t] += H_j x W2'[.., 32t..32t+31] for the C/32 output tiles; the weight image's K
//           order is permuted on the host to match the registers (ponita.py _ffn_image), so the
//           hidden activations never leave the lane that computed them.
// Software pipeline: iteration j issues GEMM 1 of chunk j + 1 beside chunk j's GELU and GEMM 2.
// The weights stream through two LDS rings of three buffers (W1 chunks, W2 chunks; C/32 blocks of
// 6 KiB each) by LDS-DMA, W1 three chunks and W2 two chunks ahead of use, with an exact vmcnt (the
// DMA pieces per wave are counted; nothing else is in flight inside the loop).  HBM traffic: XN and
// X read once, X written once; the 4C-wide hidden activation (839 MB per layer at C3) is never stored.
constexpr int FFN_WAVES = 4;

// exact-GELU 0.5 x (1 + erf(x / sqrt2)) = 0.5 x erfc(-x / sqrt2) without branches (OCML's erff
// branches on |x|, which splits the MFMA loop into basic blocks the scheduler cannot interleave):
// erfc(z) = t exp(-z^2 + P(t)), t = 1 / (1 + z / 2), z >= 0, with the Chebyshev-fitted P of
// Numerical Recipes (erfcc, fractional error < 1.2e-7 everywhere), and erfc(-z) = 2 - erfc(z).
// Max |error| over [-12, 12] in fp32: 3.8e-7 (the erff form: 4.5e-7).
__device__ inline float gelu_nb(float x) {
    const float u = x * 0.70710678118654752f, z = fabsf(u);
    const float t = __builtin_amdgcn_rcpf(1.0f + 0.5f * z);
    float p = 0.17087277f;
    p = fmaf(p, t, -0.82215223f);
    p = fmaf(p, t, 1.48851587f);
    p = fmaf(p, t, -1.13520398f);
    p = fmaf(p, t, 0.27886807f);
    p = fmaf(p, t, -0.18628806f);
    p = fmaf(p, t, 0.09678418f);
    p = fmaf(p, t, 0.37409196f);
    p = fmaf(p, t, 1.00002368f);
    p = fmaf(p, t, -1.26551223f);
    const float ec = t * __expf(fmaf(-z, z, p));
    return 0.5f * x * (u >= 0.f ? 2.0f - ec : ec);
}

// kernel-basis MLP layer 1 (ponita_pg.py:92-98 basis_fn[1] + GELU, K = 16 polynomial features):
// Y[r, c] = GELU(sum_k P16[r, k] W[c, k] + b[c]).  K is tiny, so this is a streaming write of the
// [E O][C] hidden activation (839 MB at C3), not a GEMM: thread = (row, 4 channels) with its 64
// weights and 4 biases in registers for every row it visits (persistent grid), the row's 16
// features read as four float4 (shared by the row's C / 4 lanes through L1), one float4 store.
// (The generic lin_kernel ran it at 2.1 TB/s; OCML's branchy erff made this kernel VALU-bound.)  W: [C][32] (basis1_t), features 14-31 zero-padded.
__global__ __launch_bounds__(256) void po_basis1_kernel(const float* __restrict__ P16, const float* __restrict__ W,
                                                        const float* __restrict__ b, int64_t rows, int C,
                                                        float* __restrict__ Y) {
    const int CQ = C >> 2;
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int q = (int)(t % CQ);
    const int64_t r0 = t / CQ, rstride = (int64_t)gridDim.x * blockDim.x / CQ;
    float w[4][16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
            const float4 v = *reinterpret_cast<const float4*>(W + (size_t)(4 * q + j) * 32 + 4 * k4);
            w[j][4 * k4] = v.x; w[j][4 * k4 + 1] = v.y; w[j][4 * k4 + 2] = v.z; w[j][4 * k4 + 3] = v.w;
        }
    const float4 bb = *reinterpret_cast<const float4*>(b + 4 * q);
    for (int64_t r = r0; r < rows; r += rstride) {
        float x[16];
        const float4* pr = reinterpret_cast<const float4*>(P16 + r * 16);
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
            const float4 v = pr[k4];
            x[4 * k4] = v.x; x[4 * k4 + 1] = v.y; x[4 * k4 + 2] = v.z; x[4 * k4 + 3] = v.w;
        }
        float y[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < 16; ++k) y[j] = fmaf(x[k], w[j][k], y[j]);
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = gelu_nb(y[j]);   // branch-free exact-erf GELU (3.8e-7 max error)
        *reinterpret_cast<float4*>(Y + r * C + 4 * q) = float4{y[0], y[1], y[2], y[3]};
    }
}

struct FfnProb {
    const float* XN;      // [rows][ldi] GEMM 1 input: the LayerNorm output (ConvNext), P16 (kernel basis)
    float* X;             // [rows][C] residual in, layer output (in place); the kernel basis KB (FFN_BASIS)
    const void* img;      // [F/32] slabs [W1 chunk | W2 chunk] (include/nbx.h ffn_img_x3 / ffn_img_h2)
    const float* b1;      // [F]
    const float* b2;      // [C]
    const float* scale;   // [C] layer_scale or null
    int64_t rows;
    int F;                // hidden width (multiple of 32, <= FFN_FMAX)
    int ldi;              // GEMM 1 input row stride (floats); input columns >= ldi read as zeros
    unsigned long long* dbg;   // tuning only (NBX_PO_FFN_DEBUG): per-wave phase clocks [4]
    // fp16x2 images (PREC 2): the factors undoing the images' power-of-two weight scales (W1, W2), and the
    // call's range flag (tp_fused.h tp_range_flag; null: off)
    float s1inv, s2inv;
    int* range_flag;
};
constexpr int FFN_FMAX = 1024;

// MODE FFN_CONVNEXT: the ConvNext MLP, X = X + scale (W2 GELU(W1 XN + b1) + b2), input width NTI 32 =
// output width NTO 32 = C.  MODE FFN_BASIS (r03): the kernel-basis MLP of ponita_pg.py:92-98,140-142,
// KB = GELU(W2 GELU(W1 P16 + b1) + b2), input the 16 polynomial features (NTI = 1: one 32-deep K chunk,
// columns 16-31 read as zeros against zero weights), output Bk = NTO 32 columns stored, so the [E O][C]
// hidden activation (839 MB at C3) never reaches HBM.
constexpr int FFN_CONVNEXT = 0, FFN_BASIS = 1;
// PREC 1: bf16x3 images (six bf16 products per fp32 product); PREC 2: fp16x2 images (three fp16 products,
// tp_fused.h StatSKH2; the accumulators are descaled by s1inv / s2inv).  Block of one (column tile, chunk):
// [part][m 2][lane 64][8] with 3 (bf16x3) or 2 (fp16x2) parts.
template <int NTI, int NTO, int MODE, int PREC = 1>
__global__ __launch_bounds__(64 * FFN_WAVES, 1) void po_ffn_kernel(const FfnProb P) {
    using nbx::floatx16;
    using SP = nbx::SplitP<PREC>;
    using SPT = typename SP::T;
    constexpr int NP = SP::NP, NTRM = SP::NT;
    constexpr int BLK = PREC == 2 ? nbx::LIN_H2_BLK : nbx::LIN_X3_BLK;
    constexpr int NT = NTO;               // output column tiles (the scheduling groups' unit)
    constexpr int C = NTO * 32;           // output width
    constexpr int PART1 = NTI * BLK;      // floats of one chunk's W1 blocks
    constexpr int PART = NTO * BLK;       // floats of one chunk's W2 blocks
    constexpr int NP1 = PART1 / 256;               // W1 DMA pieces (1 KiB each) per chunk
    constexpr int PW1 = (NP1 + FFN_WAVES - 1) / FFN_WAVES;
    constexpr int PW = PART / 256 / FFN_WAVES;    // W2 DMA pieces per wave per part
    static_assert(PART % (256 * FFN_WAVES) == 0, "po_ffn: a W2 part must split evenly over the waves");
    static_assert(PART1 % 256 == 0, "po_ffn: a W1 part is whole DMA pieces");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* ring1 = lds;                 // 3 x PART1: W1 chunks (chunk c in slot c % 3)
    float* ring2 = lds + 3 * PART1;     // 3 x PART: W2 chunks
    float* b1s = ring2 + 3 * PART;      // [F]
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, r = lane & 31, h = lane >> 5;
    const int nj = P.F >> 5;
    const int64_t row0 = ((int64_t)blockIdx.x * FFN_WAVES + wave) * 32;
    const int64_t row = row0 + r;
    const bool ok = row < P.rows;
    const float* img = reinterpret_cast<const float*>(P.img);
    const unsigned long long c0t = P.dbg ? clock64() : 0ull;
    auto w1src = [&](int j) { return img + (size_t)j * (PART1 + PART); };
    auto w2src = [&](int j) { return img + (size_t)j * (PART1 + PART) + PART1; };

    // prologue: input rows (lane (row, h) holds k = 32 kc + 16 h + 8 m + i, the image K order), b1,
    // W1 chunks 0-2 and W2 chunk 0; W2 chunk 1 then goes in flight
    SPT ax[NTI][NP][2];
    {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)P.XN, (short)0, 0x7FFFFFF0, 0x00020000);
        const uint32_t base = (uint32_t)(((ok ? row : 0) * P.ldi + 16 * h) * 4);
        float4 a[NTI][4];
#pragma unroll
        for (int kc = 0; kc < NTI; ++kc)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool in = ok && 32 * kc + 16 * h + 4 * q < P.ldi;   // (ldi % 4 == 0)
                a[kc][q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                          rs, in ? base + (uint32_t)(kc * 128 + 16 * q) : 0x7FFFFFF0u, 0, 0));
            }
        float bv[FFN_FMAX / (64 * FFN_WAVES)];
#pragma unroll
        for (int u = 0; u < FFN_FMAX / (64 * FFN_WAVES); ++u) {
            const int i = t + u * 64 * FFN_WAVES;
            bv[u] = i < P.F ? P.b1[i] : 0.f;
        }
        for (int c = 0; c < 3 && c < nj; ++c) nbx::tp_dma_image<FFN_WAVES>(w1src(c), ring1 + c * PART1, PART1);
        nbx::tp_dma_image<FFN_WAVES>(w2src(0), ring2, PART);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < FFN_FMAX / (64 * FFN_WAVES); ++u) {
            const int i = t + u * 64 * FFN_WAVES;
            if (i < P.F) b1s[i] = bv[u];
        }
#pragma unroll
        for (int kc = 0; kc < NTI; ++kc)
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                SPT t3[NP];
                SP::split(a[kc][2 * m], a[kc][2 * m + 1], t3);
#pragma unroll
                for (int p3 = 0; p3 < NP; ++p3) ax[kc][p3][m] = t3[p3];
            }
        // the input operands live in AGPRs for the whole loop (MFMA reads A/B from either file), which
        // leaves the architectural VGPRs to the weight fragments and the GELU arithmetic
#pragma unroll
        for (int kc = 0; kc < NTI; ++kc)
#pragma unroll
            for (int p3 = 0; p3 < NP; ++p3)
#pragma unroll
                for (int m = 0; m < 2; ++m) asm volatile("" : "+a"(ax[kc][p3][m]));
    }
    __syncthreads();
    if (nj > 1) nbx::tp_dma_image<FFN_WAVES>(w2src(1), ring2 + PART, PART);

    floatx16 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
    // GEMM 1 of one hidden chunk into one accumulator (a dependent chain of v_mfma_f32_32x32x16_bf16
    // issues at full rate; the first MFMA takes an inline 0 accumulator)
    auto gemm1 = [&](const float* buf) {
        // all of the chunk's fragments are read first (one LDS latency per chunk, not per 6 MFMAs)
        const SPT* w1 = reinterpret_cast<const SPT*>(buf) + lane;
        SPT b[NTI][2][NP];
#pragma unroll
        for (int kc = 0; kc < NTI; ++kc)
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int p3 = 0; p3 < NP; ++p3) b[kc][m][p3] = w1[kc * (BLK / 4) + m * 64 + p3 * 128];
        floatx16 g;
#pragma unroll
        for (int kc = 0; kc < NTI; ++kc)
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const SPT(&a)[NP][2] = ax[kc];
                const SPT(&w)[NP] = b[kc][m];
#pragma unroll
                for (int tt = 0; tt < NTRM; ++tt)   // smallest terms first; the weights are the MFMA's A
                    g = nbx::mfma32x32(w[SP::TB[tt]], a[SP::TA[tt]][m], (kc == 0 && m == 0 && tt == 0) ? floatx16{} : g);
            }
        if constexpr (PREC == 2) g *= P.s1inv;
        return g;
    };
    // b1 + GELU of chunk j's GEMM 1 result, split into the GEMM 2 A operand (registers 8m..8m+7 ->
    // MFMA step m)
    auto gelu_split = [&](int j, const floatx16& g, SPT (&hx)[NP][2]) {
        float hv[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) hv[e] = gelu_nb(g[e] + b1s[32 * j + (e & 3) + 8 * (e >> 2) + 4 * h]);
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            SPT t3[NP];
            SP::split(float4{hv[8 * m], hv[8 * m + 1], hv[8 * m + 2], hv[8 * m + 3]},
                      float4{hv[8 * m + 4], hv[8 * m + 5], hv[8 * m + 6], hv[8 * m + 7]}, t3);
#pragma unroll
            for (int p3 = 0; p3 < NP; ++p3) hx[p3][m] = t3[p3];
        }
    };
    auto gemm2 = [&](const float* buf, const SPT (&hx)[NP][2]) {
        const SPT* w2 = reinterpret_cast<const SPT*>(buf) + lane;
        SPT b[NT][2][NP];
#pragma unroll
        for (int tt = 0; tt < NT; ++tt)
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int p3 = 0; p3 < NP; ++p3) b[tt][m][p3] = w2[tt * (BLK / 4) + m * 64 + p3 * 128];
#pragma unroll
        for (int tt = 0; tt < NT; ++tt)
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const SPT(&w)[NP] = b[tt][m];
#pragma unroll
                for (int t3 = 0; t3 < NTRM; ++t3) acc[tt] = nbx::mfma32x32(hx[SP::TA[t3]][m], w[SP::TB[t3]], acc[tt]);
            }
    };
    // Two-deep software pipeline: iteration j issues GEMM 1 of chunk j + 2 and GEMM 2 of chunk j
    // (96 MFMAs, none waiting on VALU work) and, between them, GELU + split of chunk j + 1 (whose
    // GEMM 1 ran in iteration j - 1); scheduling groups interleave ~4 vector instructions per MFMA.
    // Rings: iteration j reads W1 chunk j + 2 and W2 chunk j; it refills W1 slot j % 3 with chunk
    // j + 3 (needed next iteration) and W2 slot (j + 2) % 3 with chunk j + 2.
    floatx16 gq[2];
    SPT hq[2][NP][2];
    gq[0] = gemm1(ring1);                               // chunk 0
    if (nj > 1) gq[1] = gemm1(ring1 + PART1);          // chunk 1
    gelu_split(0, gq[0], hq[0]);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                      // ring1 slot 0 is refilled in iteration 0
    const unsigned long long c1t = P.dbg ? clock64() : 0ull;
    // DMA of one part with a compile-time piece count per wave (no loop in the scheduling region)
    auto dma_part = [&](const float* src, float* dst) {
#pragma unroll
        for (int i = 0; i < PW; ++i) {
            const int p = wave + i * FFN_WAVES;
            __builtin_amdgcn_global_load_lds((const void*)(src + p * 256 + lane * 4),
                                             (__attribute__((address_space(3))) void*)(dst + p * 256), 16, 0, 0);
        }
    };
    // a W1 part (NP1 pieces, possibly fewer than one per wave per round): issued before the same
    // iteration's W2 part, so the wait for all but W2's PW pieces covers it
    auto dma_part1 = [&](const float* src, float* dst) {
#pragma unroll
        for (int i = 0; i < PW1; ++i) {
            const int p = wave + i * FFN_WAVES;
            if (p < NP1)
                __builtin_amdgcn_global_load_lds((const void*)(src + p * 256 + lane * 4),
                                                 (__attribute__((address_space(3))) void*)(dst + p * 256), 16, 0, 0);
        }
    };
    // iteration j; FULL: every step of the steady state (W1 chunk j + 3 and W2 chunk j + 2 exist), so
    // the body is one basic block the scheduling groups can interleave
    // SLOT: j % 3 when known at compile time (the steady state is unrolled by 6), else -1
    auto iteration = [&](int j, auto par, auto full, auto slotc) {
        constexpr int cur = decltype(par)::value, nxt = 1 - cur;
        constexpr bool FULL = decltype(full)::value;
        constexpr int SLOT = decltype(slotc)::value;
        const int s0 = SLOT >= 0 ? SLOT : j % 3, s2 = SLOT >= 0 ? (SLOT + 2) % 3 : (j + 2) % 3;
        const bool d1 = FULL || j + 3 < nj, d2 = FULL || j + 2 < nj;
        if (d1) dma_part1(w1src(j + 3), ring1 + s0 * PART1);
        if (d2) dma_part(w2src(j + 2), ring2 + s2 * PART);
        // gq[nxt] holds chunk j + 1's GEMM 1 result; gq[cur] receives chunk j + 2's
        if (FULL || j + 1 < nj) gelu_split(j + 1, gq[nxt], hq[nxt]);
        if (FULL || j + 2 < nj) gq[cur] = gemm1(ring1 + s2 * PART1);
        gemm2(ring2 + s0 * PART, hq[cur]);
        if constexpr (FULL) {
            // GEMM 1's fragment reads first; its 2 NTRM NT MFMAs each followed by ~5 (bf16x3) / ~10
            // (fp16x2: half the MFMAs for the same GELU) vector instructions (the GELU of chunk j + 1)
            // with GEMM 2's fragment reads spread among them, so every read lands long before its MFMA;
            // then GEMM 2's MFMAs with the remaining vector work
            constexpr int VA = PREC == 2 ? 10 : 5, VB = PREC == 2 ? 8 : 4;
            __builtin_amdgcn_sched_group_barrier(0x100, 2 * NP * NT, 0);
#pragma unroll
            for (int i = 0; i < 2 * NTRM * NT; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, VA, 0);
                if (PREC == 2 || (i & 1)) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
#pragma unroll
            for (int i = 0; i < 2 * NTRM * NT; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, VB, 0);
            }
        }
        // the next iteration reads W1 chunk j + 3 (issued above) and W2 chunk j + 1 (issued in j - 1):
        // only W2 chunk j + 2's pieces may stay in flight
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (d2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using IN = std::integral_constant<int, -1>;
    int j = 0;
    for (; j + 8 < nj; j += 6) {   // j % 6 == 0: parities and ring slots are compile-time
        iteration(j, I0{}, std::true_type{}, I0{});
        iteration(j + 1, I1{}, std::true_type{}, I1{});
        iteration(j + 2, I0{}, std::true_type{}, I2{});
        iteration(j + 3, I1{}, std::true_type{}, I0{});
        iteration(j + 4, I0{}, std::true_type{}, I1{});
        iteration(j + 5, I1{}, std::true_type{}, I2{});
    }
    for (; j < nj; j += 2) {
        iteration(j, I0{}, std::false_type{}, IN{});
        if (j + 1 < nj) iteration(j + 1, I1{}, std::false_type{}, IN{});
    }
    const unsigned long long c2t = P.dbg ? clock64() : 0ull;

    // epilogue: X = X + s * (acc + b2).  The accumulators (lane -> column, register e -> row
    // (e & 3) + 8 (e >> 2) + 4 h) are transposed through this wave's slice of the now idle rings,
    // so the residual loads and the stores are row-contiguous float4 (16 each per lane, not 64)
    {
        constexpr int LDR = C + 8;                        // padded row stride (floats)
        float* tile = lds + wave * 32 * LDR;
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            const int col = 32 * tt + r;
            const float b = P.b2[col];
            const float sc = P.scale ? P.scale[col] : 1.f;
            if constexpr (PREC == 2) {   // undo W2's image scale; fp16x2 range guard
                float z = 0.f;
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    acc[tt][e] *= P.s2inv;
                    z = nbx::tp_nonfinite_fold(z, acc[tt][e]);
                }
                nbx::tp_range_flag(P.range_flag, z);
            }
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const float v = MODE == FFN_BASIS ? gelu_nb(acc[tt][e] + b) : sc * (acc[tt][e] + b);
                tile[((e & 3) + 8 * (e >> 2) + 4 * h) * LDR + col] = v;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's own tile: no cross-wave hand-off
        constexpr int F4 = 32 * C / 4 / 64;   // float4 per lane
        float4 res[F4];
#pragma unroll
        for (int i = 0; i < F4; ++i) {
            const int f = lane + 64 * i, rr = f / (C / 4), c4 = f % (C / 4);
            res[i] = MODE == FFN_CONVNEXT && row0 + rr < P.rows
                         ? *reinterpret_cast<const float4*>(P.X + (row0 + rr) * C + 4 * c4)
                         : float4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int i = 0; i < F4; ++i) {
            const int f = lane + 64 * i, rr = f / (C / 4), c4 = f % (C / 4);
            const float4 v = *reinterpret_cast<const float4*>(tile + rr * LDR + 4 * c4);
            if (row0 + rr < P.rows)
                *reinterpret_cast<float4*>(P.X + (row0 + rr) * C + 4 * c4) =
                    float4{res[i].x + v.x, res[i].y + v.y, res[i].z + v.z, res[i].w + v.w};
        }
    }
    if (P.dbg && lane == 0) {
        unsigned long long* d = P.dbg + ((size_t)blockIdx.x * FFN_WAVES + wave) * 4;
        d[0] = c1t - c0t; d[1] = c2t - c1t; d[2] = 0; d[3] = clock64() - c2t;
    }
}

template <int NTI, int NTO, int MODE, int PREC = 1>
int po_ffn_launch(const FfnProb& p, hipStream_t st) {
    if (p.rows <= 0) return NBX_OK;
    NBX_CHECK_ARG(p.F % 32 == 0 && p.F >= 32 && p.F <= FFN_FMAX && p.img && p.b1 && p.b2,
                  "po_ffn: 32 <= F <= %d, F %% 32 == 0, an image, b1 and b2 required", FFN_FMAX);
    NBX_CHECK_ARG((double)p.rows * p.ldi * 4.0 < 2147483632.0, "po_ffn: XN spans >= 2 GiB");
    NBX_CHECK_ARG(p.ldi % 4 == 0 && p.ldi <= NTI * 32, "po_ffn: input stride must be a multiple of 4, <= %d", NTI * 32);
    // the rings + b1, and at least the epilogue's transpose tiles (FFN_WAVES x 32 rows x (C + 8) floats), which
    // reuse the ring space: with the smaller fp16x2 blocks and one input chunk (FFN_BASIS) the tiles are the
    // larger of the two
    const size_t lds = std::max<size_t>((3 * (size_t)(NTI + NTO) * (PREC == 2 ? nbx::LIN_H2_BLK : nbx::LIN_X3_BLK) + p.F) * 4,
                                        (size_t)FFN_WAVES * 32 * (NTO * 32 + 8) * 4);
    NBX_CHECK_ARG(lds <= 160 * 1024, "po_ffn: %zu bytes of LDS", lds);
    NBX_LDS_160K((po_ffn_kernel<NTI, NTO, MODE, PREC>));
    const unsigned blocks = (unsigned)((p.rows + 32 * FFN_WAVES - 1) / (32 * FFN_WAVES));
    static const bool debug = getenv("NBX_PO_FFN_DEBUG") != nullptr;
    static unsigned long long* dbg = nullptr;
    FfnProb q = p;
    const size_t nw = (size_t)blocks * FFN_WAVES;
    if (debug && !dbg) NBX_HIP(hipMalloc(&dbg, nw * 4 * sizeof(unsigned long long)));
    q.dbg = debug ? dbg : nullptr;
    hipLaunchKernelGGL((po_ffn_kernel<NTI, NTO, MODE, PREC>), dim3(blocks), dim3(64 * FFN_WAVES), lds, st, q);
    NBX_HIP(hipGetLastError());
    if (debug) {   // tuning only: average clocks per wave of prologue / loop / loop-end waits / epilogue
        std::vector<unsigned long long> hb(nw * 4);
        NBX_HIP(hipStreamSynchronize(st));
        NBX_HIP(hipMemcpy(hb.data(), dbg, hb.size() * 8, hipMemcpyDeviceToHost));
        double a[4] = {0, 0, 0, 0};
        for (size_t i = 0; i < nw; ++i)
            for (int k = 0; k < 4; ++k) a[k] += (double)hb[i * 4 + k];
        fprintf(stderr, "po_ffn_debug waves=%zu prologue=%.0f loop=%.0f epilogue=%.0f clocks/wave\n", nw, a[0] / nw,
                a[1] / nw, a[3] / nw);
    }
    return NBX_OK;
}

// widest column tile whose weight slice fits the LDS; the split-precision (bf16x3) kernel when the
// layer carries an image (NBX_PO_X3=0: fp32 MFMA path, A/B only)
bool po_x3_enabled() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("NBX_PO_X3");
        v = (e && e[0] == '0') ? 0 : 1;
    }
    return v == 1;
}

// the fp16x2 images when the weights carry them (NBX_PO_SPLIT=x3: the bf16x3 images, A/B only)
bool po_h2_enabled() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("NBX_PO_SPLIT");
        v = (po_x3_enabled() && !(e && (e[0] == 'x' || e[0] == '1'))) ? 1 : 0;
    }
    return v == 1;
}

template <int ACT, int EPI = nbx::LIN_STORE>
int lin_auto(nbx::LinProb& p, hipStream_t st) {
    const int need = (p.N + 31) / 32;
    if (p.Wh2 && po_h2_enabled() && p.N % 32 == 0) {
        auto lds = [&](int nt) { return nbx::lin_lds_bytes(nt, p.Ktot, 2); };
        if (need >= 3 && lds(4) <= 160 * 1024) return nbx::lin_launch<4, ACT, EPI, 2>(p, st);
        if (need >= 2 && lds(2) <= 160 * 1024) return nbx::lin_launch<2, ACT, EPI, 2>(p, st);
        if (lds(1) <= 160 * 1024) return nbx::lin_launch<1, ACT, EPI, 2>(p, st);
    }
    if (p.Wx3 && po_x3_enabled() && p.N % 32 == 0) {
        auto lds = [&](int nt) { return nbx::lin_lds_bytes(nt, p.Ktot, 1); };
        if (need >= 3 && lds(4) <= 160 * 1024) return nbx::lin_launch<4, ACT, EPI, 1>(p, st);
        if (need >= 2 && lds(2) <= 160 * 1024) return nbx::lin_launch<2, ACT, EPI, 1>(p, st);
        if (lds(1) <= 160 * 1024) return nbx::lin_launch<1, ACT, EPI, 1>(p, st);
    }
    auto lds = [&](int nt) { return nbx::lin_lds_bytes(nt, p.Ktot, 0); };
    if (need >= 3 && lds(4) <= 160 * 1024) return nbx::lin_launch<4, ACT, EPI>(p, st);
    if (need >= 2 && lds(2) <= 160 * 1024) return nbx::lin_launch<2, ACT, EPI>(p, st);
    return nbx::lin_launch<1, ACT, EPI>(p, st);
}

// launch kinds of nbx_ponita_forward_timed
enum PoKind : int { PK_CONV = 0, PK_LIN1 = 1, PK_LIN2 = 2, PK_BASIS = 3, PK_FIBER = 4 };

int po_forward_impl(const nbx_ponita_weights* w, const float* pos, const float* vel, const float* mass,
                    const PoDims& d, float* out, double* mom, const PoWs& ws, hipStream_t st,
                    nbx::LaunchTimer* tm = nullptr, const int* slot = nullptr) {
    using nbx::LinProb;
    const int O = d.O, C = d.C, Bk = d.Bk, L = d.L;
    const int64_t VO = d.V * O;
    const int OO = O * O;
    const double Ev = (double)VO * (double)(d.N - 1);  // real (edge, orientation) rows
    const double f4 = 4.0;
    // ---- invariants, kernel bases (shared by all layers), lift
    hipLaunchKernelGGL(po_attr_kernel, dim3(g1(d.R)), dim3(256), 0, st, pos, w->ori_grid, d.R, (int)d.N, O, (int)d.G,
                       ws.P16, slot);
    hipLaunchKernelGGL(po_fattr_kernel, dim3(g1(OO)), dim3(256), 0, st, w->ori_grid, O, ws.FP);
    hipLaunchKernelGGL(po_lift_kernel, dim3(g1(VO * (C / 4))), dim3(256), 0, st, mass, vel, w->ori_grid, w->embed_w, d.V, O,
                       C, ws.X);
    NBX_LAUNCH_CHECK("ponita prep");
    // both kernel-basis layers in one kernel when the weights carry the fused image (NBX_PO_BASIS_FUSED=0:
    // the two-kernel path, A/B only)
    static const bool basis_fused = !(getenv("NBX_PO_BASIS_FUSED") && getenv("NBX_PO_BASIS_FUSED")[0] == '0');
    const bool basis_h2 = w->basis_ffn_img_h2 && po_h2_enabled();
    if ((basis_h2 || w->basis_ffn_img_x3) && basis_fused && (Bk == 128 || Bk == 64) && C % 32 == 0 && C <= FFN_FMAX) {
        const FfnProb fb{ws.P16, ws.KB, basis_h2 ? w->basis_ffn_img_h2 : w->basis_ffn_img_x3, w->basis1_b,
                         w->basis2_b, nullptr, d.R, C, 16, nullptr, w->basis_ffn_h2_s1inv, w->basis_ffn_h2_s2inv,
                         ws.RANGE};
        if (int rc = nbx::timed(tm, st, PK_BASIS, 2.0 * Ev * (14 * C + C * Bk), Ev * f4 * (16 + Bk), [&] {
                if (basis_h2)
                    return Bk == 128 ? po_ffn_launch<1, 4, FFN_BASIS, 2>(fb, st) : po_ffn_launch<1, 2, FFN_BASIS, 2>(fb, st);
                return Bk == 128 ? po_ffn_launch<1, 4, FFN_BASIS>(fb, st) : po_ffn_launch<1, 2, FFN_BASIS>(fb, st);
            }))
            return rc;
    } else {
        LinProb p = nbx::lin_dense(ws.P16, 16, 16, (int)d.R, w->basis1_t, 32, C, w->basis1_b, ws.B1H1, C);
        // layer 1 as a streaming kernel (NBX_PO_BASIS1=0: the generic GEMM, A/B only)
        static const bool b1s = !(getenv("NBX_PO_BASIS1") && getenv("NBX_PO_BASIS1")[0] == '0');
        if (int rc = nbx::timed(tm, st, PK_BASIS, 2.0 * Ev * 14 * C, Ev * f4 * (16 + C), [&] {
                if (!b1s) return lin_auto<nbx::ACT_GELU>(p, st);
                const int64_t threads = std::min<int64_t>(d.R * (C / 4), (int64_t)256 * 8 * 256);
                hipLaunchKernelGGL(po_basis1_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st,
                                   ws.P16, w->basis1_t, w->basis1_b, d.R, C, ws.B1H1);
                return (int)NBX_OK;
            }))
            return rc;
        LinProb q = nbx::lin_dense(ws.B1H1, C, C, (int)d.R, w->basis2_t, kp(C), Bk, w->basis2_b, ws.KB, Bk);
        q.Wx3 = w->basis2_img_x3;
        if (int rc = nbx::timed(tm, st, PK_BASIS, 2.0 * Ev * C * Bk, Ev * f4 * (C + Bk),
                                [&] { return lin_auto<nbx::ACT_GELU>(q, st); }))
            return rc;
    }
    {
        LinProb f1 = nbx::lin_dense(ws.FP, 4, 4, OO, w->fbasis1_t, 32, C, w->fbasis1_b, ws.FB1, C);
        if (int rc = lin_auto<nbx::ACT_GELU>(f1, st)) return rc;
        LinProb f2 = nbx::lin_dense(ws.FB1, C, C, OO, w->fbasis2_t, kp(C), Bk, w->fbasis2_b, ws.FKB, Bk);
        if (int rc = lin_auto<nbx::ACT_GELU>(f2, st)) return rc;
        LinProb f3 = nbx::lin_dense(ws.FKB, Bk, Bk, OO, w->fiber_t, kp(Bk), L * C, nullptr, ws.FK, L * C);
        if (int rc = lin_auto<nbx::ACT_NONE>(f3, st)) return rc;
    }
    if (mom) NBX_HIP(hipMemsetAsync(mom, 0, sizeof(double) * 6 * L, st));
    int nro = 0;
    for (int l = 0; l < L; ++l) {
        const nbx_ponita_layer& Ly = w->layers[l];
        if (mom)
            hipLaunchKernelGGL(po_moments_kernel, dim3(512), dim3(256), 0, st, ws.X, VO * C, mom + 6 * l);
        {   // spatial conv: X1[(d,o)] = sum_q (KB Wk')[(d,o,q)] * X[(src,o)]
            LinProb p = nbx::lin_dense(ws.KB, Bk, Bk, (int)d.R, Ly.kernel_t, kp(Bk), C, nullptr, ws.X1, C);
            p.Wx3 = Ly.kernel_img_x3;
            p.Wh2 = Ly.kernel_img_h2;
            p.h2_sinv = Ly.kernel_h2_sinv;
            p.range_flag = ws.RANGE;
            p.conv_G = (int)d.G;
            p.conv_O = O;
            p.conv_nodes = (int)d.N;
            p.conv_slot = slot;
            p.conv_x = ws.X;
            p.conv_ldx = C;
            if (int rc = nbx::timed(tm, st, PK_CONV, 2.0 * Ev * Bk * C + 2.0 * Ev * C,
                                    Ev * f4 * Bk + (double)VO * C * f4 * 2,
                                    [&] { return lin_auto<nbx::ACT_NONE, nbx::LIN_CONV>(p, st); }))
                return rc;
        }
        if (mom)
            hipLaunchKernelGGL(po_moments_kernel, dim3(512), dim3(256), 0, st, ws.X1, VO * C, mom + 6 * l + 2);
        {
            // orientation range per block (X1 is re-read once per range): a 64 KiB FK slice, C3: 6 of
            // 20 orientations, 4 ranges -- with conflict-free LDS reads 176 us against 196 us for
            // 72 KiB / 3 ranges (occupancy beats the re-read).  NBX_PO_FK_LDS: the budget in bytes (tuning)
            static const size_t fk_lds = getenv("NBX_PO_FK_LDS") ? (size_t)atol(getenv("NBX_PO_FK_LDS")) : 64 * 1024;
            const int PR = std::max(1, std::min(O, (int)(fk_lds / ((size_t)O * C * 4))));
            const int R = (O + PR - 1) / PR;
            const int npi = PO_FIB_THREADS / (C / 4);
            // NBX_PO_FIB_BLOCKS: total workgroups over all ranges (the ranges of one node group sit on the
            // same XCD since gx % 8 == 0, so co-resident ranges share X1 through that XCD's L2).  Measured
            // (profiles/r04/ponita_fib_ab): 1024 -> 181 us / 989 MB, 512 -> 169 us / 762 MB, 256 -> 261 us /
            // 610 MB per launch; fewer groups re-read less but 256 no longer fills the chip
            static const int fib_blocks = getenv("NBX_PO_FIB_BLOCKS") ? atoi(getenv("NBX_PO_FIB_BLOCKS")) : 512;
            // po_fiber_ln1_kernel (default; NBX_PO_FIB_ONEPASS=0 selects the range-split kernel below): X1
            // read once, FK slices double-buffered through LDS-DMA.  Measured (profiles/r04/ponita_fib_onepass):
            // 450 MB per launch (1.07x algorithmic) in 184 us against the range-split kernel's 762 MB in
            // 167 us; C3 steps/s equal within run-to-run noise (103.55 vs 103.51).  256-thread blocks,
            // 16-20 KiB slices and 1024-2048 blocks measured slower (219-287 us)
            static const bool onepass = !getenv("NBX_PO_FIB_ONEPASS") || atoi(getenv("NBX_PO_FIB_ONEPASS")) != 0;
            static const size_t fk1_lds = getenv("NBX_PO_FK1_LDS") ? (size_t)atol(getenv("NBX_PO_FK1_LDS")) : 32 * 1024;
            const int PR1 = std::max(1, std::min(O, (int)(fk1_lds / ((size_t)O * C * 4))));
            if (onepass && O <= 20 && C % 4 == 0 && PO_FIB_THREADS % (C / 4) == 0) {
                static const int fib1_blocks =
                    getenv("NBX_PO_FIB1_BLOCKS") ? atoi(getenv("NBX_PO_FIB1_BLOCKS")) : 512;
                int gx1;
                const int slice4 = (O * PR1 * (C / 4) + 63) / 64 * 64;     // whole DMA pieces
                const size_t lds1 = 2 * (size_t)slice4 * 16;
                // NBX_PO_FIB1_W: waves per EU the register budget targets (4: <= 128 VGPRs, two blocks per CU)
                static const int fib1_w = getenv("NBX_PO_FIB1_W") ? atoi(getenv("NBX_PO_FIB1_W")) : 4;
                // NBX_PO_FIB1_NT: threads per block (256: more, smaller blocks interleave the per-range barriers)
                static const int fib1_nt = getenv("NBX_PO_FIB1_NT") ? atoi(getenv("NBX_PO_FIB1_NT")) : 512;
                const int nt1 = (fib1_nt == 256 && 256 % (C / 4) == 0) ? 256 : 512;
                const int npi1 = nt1 / (C / 4);
                gx1 = (int)std::min<int64_t>((d.V + npi1 - 1) / npi1, std::max(1, fib1_blocks));
                auto k1 = nt1 == 256 ? (fib1_w >= 4 ? po_fiber_ln1_kernel<20, 4, 256> : po_fiber_ln1_kernel<20, 2, 256>)
                                     : (fib1_w >= 4 ? po_fiber_ln1_kernel<20, 4> : po_fiber_ln1_kernel<20, 2>);
                NBX_CHECK_ARG(lds1 <= 160 * 1024, "ponita: one-pass fibre kernel needs %zu bytes of LDS", lds1);
                if (lds1 > 64 * 1024)
                    NBX_HIP(hipFuncSetAttribute((const void*)k1, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                (int)lds1));
                if (int rc = nbx::timed(tm, st, PK_FIBER, 2.0 * VO * O * C, (double)VO * C * f4 * 2, [&] {
                        hipLaunchKernelGGL(k1, dim3(gx1), dim3(nt1), lds1, st, ws.X1,
                                           ws.FK + (size_t)l * C, L * C, Ly.conv_bias, Ly.norm_w, Ly.norm_b, d.V,
                                           O, C, PR1, slice4, ws.XN, mom ? mom + 6 * l + 4 : nullptr);
                        return (int)NBX_OK;
                    }))
                    return rc;
                goto fiber_done;
            }
            {
            const int gx = (int)std::min<int64_t>((d.V + npi - 1) / npi, std::max(1, fib_blocks / R));
            const size_t lds = (size_t)O * PR * C * 4;
            auto kern = O <= 20 ? po_fiber_ln_kernel<20, 4> : po_fiber_ln_kernel<PO_OMAX, 2>;
            if (lds > 64 * 1024) {
                NBX_CHECK_ARG(lds <= 160 * 1024, "ponita: fibre kernel slice needs %zu bytes of LDS", lds);
                NBX_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)lds));
            }
            if (int rc = nbx::timed(tm, st, PK_FIBER, 2.0 * VO * O * C, (double)VO * C * f4 * 2, [&] {
                    hipLaunchKernelGGL(kern, dim3(gx, R), dim3(PO_FIB_THREADS), lds, st, ws.X1,
                                       ws.FK + (size_t)l * C, L * C, Ly.conv_bias, Ly.norm_w, Ly.norm_b, d.V, O, C,
                                       PR, ws.XN, mom ? mom + 6 * l + 4 : nullptr);
                    return (int)NBX_OK;
                }))
                return rc;
            }
        fiber_done:;
        }
        const bool ffn_h2 = Ly.ffn_img_h2 && po_h2_enabled();
        if ((ffn_h2 || Ly.ffn_img_x3) && po_x3_enabled() && (C == 64 || C == 128) && d.mlp % 32 == 0 &&
            d.mlp <= FFN_FMAX) {
            // ConvNext MLP fused (linear_1 + GELU + linear_2 + layer_scale + residual): the hidden
            // activation stays in registers (po_ffn_kernel), on the fp16x2 image when present
            const FfnProb fp{ws.XN, ws.X, ffn_h2 ? Ly.ffn_img_h2 : Ly.ffn_img_x3, Ly.lin1_b, Ly.lin2_b, Ly.layer_scale, VO,
                             d.mlp, C, nullptr, Ly.ffn_h2_s1inv, Ly.ffn_h2_s2inv, ws.RANGE};
            if (int rc = nbx::timed(tm, st, PK_LIN1, 2.0 * 2.0 * VO * C * d.mlp, (double)VO * f4 * 3 * C, [&] {
                    if (ffn_h2)
                        return C == 128 ? po_ffn_launch<4, 4, FFN_CONVNEXT, 2>(fp, st)
                                        : po_ffn_launch<2, 2, FFN_CONVNEXT, 2>(fp, st);
                    return C == 128 ? po_ffn_launch<4, 4, FFN_CONVNEXT>(fp, st) : po_ffn_launch<2, 2, FFN_CONVNEXT>(fp, st);
                }))
                return rc;
        } else {   // ConvNext MLP with the residual in the epilogue
            LinProb p = nbx::lin_dense(ws.XN, C, C, (int)VO, Ly.lin1_t, kp(C), d.mlp, Ly.lin1_b, ws.B1H1, d.mlp);
            p.Wx3 = Ly.lin1_img_x3;
            if (int rc = nbx::timed(tm, st, PK_LIN1, 2.0 * VO * C * d.mlp, (double)VO * f4 * (C + d.mlp),
                                    [&] { return lin_auto<nbx::ACT_GELU>(p, st); }))
                return rc;
            // linear_2 (K = 4C -> C): the row-panel kernel reads the [V O][4C] hidden activations once
            // (the column-chunked kernel re-read them C / 32 times); the image is chunk-major
            auto lin2 = [&]() -> int {
                if (Ly.lin2_img_x3 && po_x3_enabled() && d.mlp % 32 == 0) {
                    nbx::LinRpProb r{ws.B1H1, d.mlp, (int)VO, d.mlp, Ly.lin2_img_x3, Ly.lin2_b, ws.X, C, C,
                                     ws.X, C, Ly.layer_scale};
                    switch (C) {
                        case 32: return nbx::lin_rp_launch<1, nbx::ACT_NONE>(r, st);
                        case 64: return nbx::lin_rp_launch<2, nbx::ACT_NONE>(r, st);
                        case 128: return nbx::lin_rp_launch<4, nbx::ACT_NONE>(r, st);
                        default: break;
                    }
                }
                LinProb q = nbx::lin_dense(ws.B1H1, d.mlp, d.mlp, (int)VO, Ly.lin2_t, kp(d.mlp), C, Ly.lin2_b, ws.X, C);
                q.resid = ws.X;
                q.ldr = C;
                q.scale = Ly.layer_scale;
                return lin_auto<nbx::ACT_NONE>(q, st);
            };
            if (int rc = nbx::timed(tm, st, PK_LIN2, 2.0 * VO * C * d.mlp, (double)VO * f4 * (d.mlp + 2 * C), lin2))
                return rc;
        }
        if (Ly.readout_w) {
            const int64_t thr = VO * (C / 16);
            hipLaunchKernelGGL(po_readout_kernel, dim3(g1(thr)), dim3(256), 0, st, ws.X, Ly.readout_w, Ly.readout_b,
                               VO, C, nro == 0 ? 1 : 0, ws.RO);
            ++nro;
        }
        NBX_LAUNCH_CHECK("ponita layer");
    }
    if (nro == 0) {
        nbx::set_error("ponita: no read-out layer");
        return NBX_E_INVAL;
    }
    hipLaunchKernelGGL(po_out_kernel, dim3(g1(d.V * 6)), dim3(256), 0, st, ws.RO, w->ori_grid, d.V, O, nro, out);
    NBX_LAUNCH_CHECK("ponita out");
    return NBX_OK;
}

int po_prepare(const nbx_ponita_weights* w, int64_t B, int64_t N, void* ws_ptr, size_t bytes, PoDims* dims,
               PoWs* ws) {
    NBX_CHECK_ARG(w, "ponita: null weights");
    NBX_CHECK_ARG(w->hidden == 32 || w->hidden == 64 || w->hidden == 128, "ponita: hidden must be 32, 64 or 128");
    NBX_CHECK_ARG(w->basis_dim > 0 && w->basis_dim % 4 == 0 && w->basis_dim <= 1024, "ponita: basis_dim %% 4 != 0");
    NBX_CHECK_ARG(w->widening >= 1 && w->widening * w->hidden <= 1024, "ponita: widening * hidden must be <= 1024");
    NBX_CHECK_ARG(w->num_layers >= 1 && w->num_layers <= NBX_PONITA_MAX_LAYERS, "ponita: bad num_layers");
    NBX_CHECK_ARG(w->num_ori >= 1 && w->num_ori <= PO_OMAX, "ponita: num_ori must be 1..24");
    NBX_CHECK_ARG(B >= 1 && N >= 2 && N <= 33, "ponita: need B >= 1 and 2 <= N <= 33");
    *dims = po_dims(w, B, N);
    NBX_CHECK_ARG(dims->R < ((int64_t)1 << 31) && dims->V * dims->O * std::max(dims->C, dims->mlp) < ((int64_t)1 << 31),
                  "ponita: B*N*num_ori*max(G, 4*hidden) exceeds 2^31");
    const size_t need = po_carve(ws, ws_ptr, *dims);
    if (!ws_ptr || bytes < need) {
        nbx::set_error("ponita: workspace too small (%zu < %zu bytes)", bytes, need);
        return NBX_E_WORKSPACE;
    }
    return NBX_OK;
}

}  // namespace

extern "C" int nbx_ponita_workspace_bytes(const nbx_ponita_weights* w, int64_t B, int64_t N, size_t* bytes) {
    NBX_CHECK_ARG(w && bytes && B >= 1 && N >= 2, "nbx_ponita_workspace_bytes: bad arguments");
    *bytes = po_carve(nullptr, nullptr, po_dims(w, B, N));
    return NBX_OK;
}

extern "C" int nbx_ponita_forward(const nbx_ponita_weights* w, const float* pos, const float* vel, const float* mass,
                                  int64_t B, int64_t N, float* out, double* calib_moments, void* workspace,
                                  size_t workspace_bytes, void* stream) {
    PoDims d;
    PoWs ws;
    if (int rc = po_prepare(w, B, N, workspace, workspace_bytes, &d, &ws)) return rc;
    NBX_HIP(hipMemsetAsync(ws.RANGE, 0, sizeof(int), (hipStream_t)stream));
    return po_forward_impl(w, pos, vel, mass, d, out, calib_moments, ws, (hipStream_t)stream);
}

extern "C" int nbx_ponita_forward_timed(const nbx_ponita_weights* w, const float* pos, const float* vel,
                                        const float* mass, int64_t B, int64_t N, float* out, void* workspace,
                                        size_t workspace_bytes, void* stream, float kind_ms[8],
                                        int32_t kind_launches[8], double kind_flops[8], double kind_bytes[8],
                                        float* total_ms) {
    PoDims d;
    PoWs ws;
    if (int rc = po_prepare(w, B, N, workspace, workspace_bytes, &d, &ws)) return rc;
    hipStream_t st = (hipStream_t)stream;
    NBX_HIP(hipMemsetAsync(ws.RANGE, 0, sizeof(int), st));
    nbx::LaunchTimer tm;
    hipEvent_t a, b;
    NBX_HIP(hipEventCreate(&a));
    NBX_HIP(hipEventCreate(&b));
    NBX_HIP(hipEventRecord(a, st));
    int rc = po_forward_impl(w, pos, vel, mass, d, out, nullptr, ws, st, &tm);
    NBX_HIP(hipEventRecord(b, st));
    if (!rc) rc = tm.collect(kind_ms);
    NBX_HIP(hipEventSynchronize(b));
    NBX_HIP(hipEventElapsedTime(total_ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    for (int k = 0; k < 8; ++k) {
        kind_launches[k] = tm.launches[k];
        kind_flops[k] = tm.flops[k];
        kind_bytes[k] = tm.bytes[k];
    }
    return rc;
}

extern "C" int nbx_ponita_rollout(const nbx_ponita_weights* w, float* pos, float* vel, const float* mass, int64_t B,
                                  int64_t N, int64_t num_frames, int32_t flags, float* traj_pos, float* traj_vel, void* workspace,
                                  size_t workspace_bytes, void* stream) {
    PoDims d;
    PoWs ws;
    if (int rc = po_prepare(w, B, N, workspace, workspace_bytes, &d, &ws)) return rc;
    NBX_CHECK_ARG(num_frames >= 1, "nbx_ponita_rollout: num_frames >= 1");
    hipStream_t st = (hipStream_t)stream;
    NBX_HIP(hipMemsetAsync(ws.RANGE, 0, sizeof(int), st));
    const int64_t V = d.V;
    hipLaunchKernelGGL(nbx::rollout_state_kernel, dim3(g1(3 * V)), dim3(256), 0, st, pos, vel, ws.out, V, (int)N,
                       (int64_t)0, num_frames, traj_pos, traj_vel, flags & NBX_ROLLOUT_ABSOLUTE);
    for (int64_t f = 1; f < num_frames; ++f) {
        if (int rc = po_forward_impl(w, pos, vel, mass, d, ws.out, nullptr, ws, st)) return rc;
        hipLaunchKernelGGL(nbx::rollout_state_kernel, dim3(g1(3 * V)), dim3(256), 0, st, pos, vel, ws.out, V, (int)N,
                           f, num_frames, traj_pos, traj_vel, flags & NBX_ROLLOUT_ABSOLUTE);
    }
    NBX_LAUNCH_CHECK("ponita rollout");
    return NBX_OK;
}

extern "C" int nbx_ponita_forward_graph(const nbx_ponita_weights* w, const float* pos, const float* vel,
                                        const float* mass, int64_t B, int64_t N, const int64_t* edge_index,
                                        int64_t num_edges, float* out, double* calib_moments, void* workspace,
                                        size_t workspace_bytes, void* stream) {
    PoDims d;
    PoWs ws;
    if (int rc = po_prepare(w, B, N, workspace, workspace_bytes, &d, &ws)) return rc;
    NBX_CHECK_ARG(num_edges >= 0 && (num_edges == 0 || edge_index), "nbx_ponita_forward_graph: bad edge_index");
    hipStream_t st = (hipStream_t)stream;
    NBX_HIP(hipMemsetAsync(ws.RANGE, 0, sizeof(int), st));
    if (int rc = nbx::graph_slots_from_edges(edge_index, num_edges, d.V, (int)N, (int)d.G, ws.ADJ, ws.SLOT, ws.DEG,
                                             ws.ERR, st))
        return rc;
    return po_forward_impl(w, pos, vel, mass, d, out, calib_moments, ws, st, nullptr, ws.SLOT);
}

extern "C" int nbx_ponita_rollout_knn(const nbx_ponita_weights* w, float* pos, float* vel, const float* mass,
                                      int64_t B, int64_t N, int64_t num_frames, int32_t flags, int64_t num_neighbors,
                                      float* traj_pos, float* traj_vel, void* workspace, size_t workspace_bytes,
                                      void* stream) {
    if (num_neighbors < 0) num_neighbors = N - 1;   // the reference's None
    NBX_CHECK_ARG(num_neighbors < N, "Graph cannot have more neighbors than there are nodes in simulation - 1");
    if (num_neighbors == N - 1)   // build_graph_with_knn returns the fully-connected pattern
        return nbx_ponita_rollout(w, pos, vel, mass, B, N, num_frames, flags, traj_pos, traj_vel, workspace,
                                  workspace_bytes, stream);
    NBX_CHECK_ARG(num_neighbors >= 1, "nbx_ponita_rollout_knn: num_neighbors must be >= 1");
    PoDims d;
    PoWs ws;
    if (int rc = po_prepare(w, B, N, workspace, workspace_bytes, &d, &ws)) return rc;
    NBX_CHECK_ARG(num_frames >= 1, "nbx_ponita_rollout_knn: num_frames >= 1");
    hipStream_t st = (hipStream_t)stream;
    NBX_HIP(hipMemsetAsync(ws.RANGE, 0, sizeof(int), st));
    const int64_t V = d.V;
    hipLaunchKernelGGL(nbx::rollout_state_kernel, dim3(g1(3 * V)), dim3(256), 0, st, pos, vel, ws.out, V, (int)N,
                       (int64_t)0, num_frames, traj_pos, traj_vel, flags & NBX_ROLLOUT_ABSOLUTE);
    for (int64_t f = 1; f < num_frames; ++f) {
        // each frame's kNN graph from its positions (infer_self_feed.py:137-142)
        if (int rc = nbx::graph_slots_from_knn(pos, V, (int)N, (int)d.G, (int)num_neighbors, ws.ADJ, ws.SLOT, ws.DEG,
                                               ws.ERR, st))
            return rc;
        if (int rc = po_forward_impl(w, pos, vel, mass, d, ws.out, nullptr, ws, st, nullptr, ws.SLOT)) return rc;
        hipLaunchKernelGGL(nbx::rollout_state_kernel, dim3(g1(3 * V)), dim3(256), 0, st, pos, vel, ws.out, V, (int)N,
                           f, num_frames, traj_pos, traj_vel, flags & NBX_ROLLOUT_ABSOLUTE);
    }
    NBX_LAUNCH_CHECK("ponita rollout");
    return NBX_OK;
}

extern "C" int nbx_ponita_range_check(const nbx_ponita_weights* w, const void* workspace, size_t workspace_bytes,
                                      int64_t B, int64_t N, void* stream) {
    PoDims d;
    PoWs ws;
    if (int rc = po_prepare(w, B, N, const_cast<void*>(workspace), workspace_bytes, &d, &ws)) return rc;
    int flag = 0;
    NBX_HIP(hipMemcpyAsync(&flag, ws.RANGE, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
    NBX_HIP(hipStreamSynchronize((hipStream_t)stream));
    if (flag) {
        nbx::set_error("ponita: a GEMM operand left the fp16 range of the fp16x2 split path (|a| >= 65520) or the "
                       "input is not finite; the bf16x3 path (NBX_PO_SPLIT=x3) keeps the fp32 exponent range");
        return NBX_E_RANGE;
    }
    return NBX_OK;
}
