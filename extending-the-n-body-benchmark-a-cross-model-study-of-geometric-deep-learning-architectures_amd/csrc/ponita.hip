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
// LIN_CONV).  Per forward:
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

#include "launch_timer.h"
#include "lin.h"
#include "nbx_internal.h"
#include "rollout_state.h"

namespace {

constexpr int PO_OMAX = 24;

unsigned g1(int64_t n) { return (unsigned)nbx::ceil_div(n > 0 ? n : 1, 256); }

// invariant_attr_r3s2_fiber_bundle (separable) + PolynomialFeatures(3) per edge slot.
__global__ void po_attr_kernel(const float* __restrict__ pos, const float* __restrict__ ori, int64_t R, int N, int O,
                               int G, float* __restrict__ P16) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= R) return;
    const int q = (int)(r % G);
    const int64_t t = r / G;
    const int o = (int)(t % O);
    const int64_t d = t / O;
    float f[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) f[i] = 0.f;
    if (q < N - 1) {
        const int dl = (int)(d % N);
        const int64_t s = d - dl + (q < dl ? q : q + 1);
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
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= V * O * C) return;
    const int c = (int)(i % C);
    const int64_t t = i / C;
    const int o = (int)(t % O);
    const int64_t v = t / O;
    const float f1 = vel[3 * v] * ori[3 * o] + vel[3 * v + 1] * ori[3 * o + 1] + vel[3 * v + 2] * ori[3 * o + 2];
    X[i] = mass[v] * We[2 * c] + f1 * We[2 * c + 1];
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

// read_out_layers[l]: RO[row, k] (+)= X[row] . Wro[k] + bro[k], k < 2; C/4 lanes per row
__global__ void po_readout_kernel(const float* __restrict__ X, const float* __restrict__ Wro,
                                  const float* __restrict__ bro, int64_t rows, int C, int first,
                                  float* __restrict__ RO) {
    const int CG = C >> 2;
    const int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t row = g / CG;
    const int j = (int)(g - row * CG);
    float d0 = 0.f, d1 = 0.f;
    if (row < rows) {
        const float4 x = *reinterpret_cast<const float4*>(X + row * C + 4 * j);
        const float4 w0 = *reinterpret_cast<const float4*>(Wro + 4 * j);
        const float4 w1 = *reinterpret_cast<const float4*>(Wro + C + 4 * j);
        d0 = x.x * w0.x + x.y * w0.y + x.z * w0.z + x.w * w0.w;
        d1 = x.x * w1.x + x.y * w1.y + x.z * w1.z + x.w * w1.w;
    }
    for (int off = CG >> 1; off > 0; off >>= 1) {
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
    if (ws) *ws = w;
    return (off + 255) & ~size_t(255);
}

inline int kp(int k) { return (k + 31) & ~31; }

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

template <int ACT, int EPI = nbx::LIN_STORE>
int lin_auto(nbx::LinProb& p, hipStream_t st) {
    const int need = (p.N + 31) / 32;
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
                    nbx::LaunchTimer* tm = nullptr) {
    using nbx::LinProb;
    const int O = d.O, C = d.C, Bk = d.Bk, L = d.L;
    const int64_t VO = d.V * O;
    const int OO = O * O;
    const double Ev = (double)VO * (double)(d.N - 1);  // real (edge, orientation) rows
    const double f4 = 4.0;
    // ---- invariants, kernel bases (shared by all layers), lift
    hipLaunchKernelGGL(po_attr_kernel, dim3(g1(d.R)), dim3(256), 0, st, pos, w->ori_grid, d.R, (int)d.N, O, (int)d.G,
                       ws.P16);
    hipLaunchKernelGGL(po_fattr_kernel, dim3(g1(OO)), dim3(256), 0, st, w->ori_grid, O, ws.FP);
    hipLaunchKernelGGL(po_lift_kernel, dim3(g1(VO * C)), dim3(256), 0, st, mass, vel, w->ori_grid, w->embed_w, d.V, O,
                       C, ws.X);
    NBX_LAUNCH_CHECK("ponita prep");
    {
        LinProb p = nbx::lin_dense(ws.P16, 16, 16, (int)d.R, w->basis1_t, 32, C, w->basis1_b, ws.B1H1, C);
        if (int rc = nbx::timed(tm, st, PK_BASIS, 2.0 * Ev * 14 * C, Ev * f4 * (16 + C),
                                [&] { return lin_auto<nbx::ACT_GELU>(p, st); }))
            return rc;
        LinProb q = nbx::lin_dense(ws.B1H1, C, C, (int)d.R, w->basis2_t, kp(C), Bk, w->basis2_b, ws.KB, Bk);
        q.Wx3 = w->basis2_img_x3;
        if (int rc = nbx::timed(tm, st, PK_BASIS, 2.0 * Ev * C * Bk, Ev * f4 * (C + Bk),
                                [&] { return lin_auto<nbx::ACT_GELU>(q, st); }))
            return rc;
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
            p.conv_G = (int)d.G;
            p.conv_O = O;
            p.conv_nodes = (int)d.N;
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
            const int gx = (int)std::min<int64_t>((d.V + npi - 1) / npi, std::max(1, 1024 / R));
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
        {   // ConvNext MLP with the residual in the epilogue
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
            const int64_t thr = VO * (C / 4);
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
