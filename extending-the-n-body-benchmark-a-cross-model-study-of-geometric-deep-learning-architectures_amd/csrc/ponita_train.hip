// PONITA training step (trainer.py:233-358: pred = model(graph); loss.backward()) —
// the PONITA-specific operators of the training forward and backward (fp32).  The dense layers
// (basis MLPs, kernel / fiber-kernel projections, ConvNext MLP, embedding, read-outs) run on the
// fp32 MFMA GEMM of csrc/segnn_train.hip (nbx_gemm_f32) and the column sums (bias / LayerNorm
// parameter gradients) on nbx_colsum; this file adds, on the fibre-bundle layout of DESIGN.md §4.4
// (node rows [V][O][C], edge rows [E][O][*], fibre rows [O][O][*]):
//   * featurisation: invariants + polynomial features of the edges and fibres, the lifted input
//     (transforms/position_orientation_graph.py:58-87, geometry/invariants.py:9-51,
//     nn/embedding.py:4-15) — no gradient (positions and velocities are data);
//   * bias + activation (nn.GELU, exact erf form) and its backward;
//   * the spatial message x1[v,o,c] = sum_{e: dst=v} k[e,o,c] h[src_e,o,c] (nn/conv.py:103-107,
//     131-133, aggr "add" at edge_index[1]) over the destination CSR, and its backward: dk per edge,
//     dh over the source CSR (no atomics);
//   * the depth-wise fibre convolution x2[v,p,c] = (1/O) sum_o x1[v,o,c] fk[o,p,c] + bias[c]
//     (conv.py:108-111) and its backward (dfk reduced over nodes in fixed-size chunks, fixed order);
//   * LayerNorm over the channels (convnext.py:18-25, eps 1e-5, biased variance) and its backward.
// Every reduction runs in a fixed order: the training step is bit-reproducible.
#include <algorithm>

#include "nbx_internal.h"

namespace {

unsigned nblk(int64_t n, int t = 256) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

// ---------------------------------------------------------------- featurisation (no gradient)
// attr [E*O][16]: the 14 degree-3 polynomial features of (inv1, inv2) = (r.o, |r - (r.o) o|),
// r = pos[src] - pos[dst] (dataloaders/ponita_n_body_dataloader.py:31-33), zero-padded to 16;
// fiber [O*O][4]: (s, s^2, s^3, 0), s = o_p . o_o; lift [V*O][2] = (mass, vel . o).
__global__ void po_train_featurize_kernel(int64_t V, int64_t E, int O, const float* __restrict__ pos,
                                          const float* __restrict__ vel, const float* __restrict__ mass,
                                          const float* __restrict__ ori, const int* __restrict__ src,
                                          const int* __restrict__ dst, float* __restrict__ attr,
                                          float* __restrict__ fiber, float* __restrict__ lift) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < E * O) {
        const int64_t e = i / O;
        const int o = (int)(i - e * O);
        const int64_t s = src[e], d = dst[e];
        const float ox = ori[3 * o], oy = ori[3 * o + 1], oz = ori[3 * o + 2];
        const float rx = pos[3 * s] - pos[3 * d], ry = pos[3 * s + 1] - pos[3 * d + 1];
        const float rz = pos[3 * s + 2] - pos[3 * d + 2];
        const float a = rx * ox + ry * oy + rz * oz;
        const float qx = rx - a * ox, qy = ry - a * oy, qz = rz - a * oz;
        const float b = sqrtf(qx * qx + qy * qy + qz * qz);
        const float x[2] = {a, b};
        float f[16];
        f[0] = a;
        f[1] = b;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int w = 0; w < 2; ++w) f[2 + 2 * u + w] = x[u] * x[w];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int w = 0; w < 2; ++w) f[6 + 2 * u + w] = f[2 + u] * x[w];
        f[14] = f[15] = 0.f;
        float4* out = reinterpret_cast<float4*>(attr + i * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q) out[q] = make_float4(f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]);
    }
    if (i < V * O) {
        const int64_t v = i / O;
        const int o = (int)(i - v * O);
        lift[2 * i] = mass[v];
        lift[2 * i + 1] = vel[3 * v] * ori[3 * o] + vel[3 * v + 1] * ori[3 * o + 1] + vel[3 * v + 2] * ori[3 * o + 2];
    }
    if (i < (int64_t)O * O) {
        const int o = (int)(i / O), p = (int)(i % O);
        const float s = ori[3 * p] * ori[3 * o] + ori[3 * p + 1] * ori[3 * o + 1] + ori[3 * p + 2] * ori[3 * o + 2];
        fiber[4 * i] = s;
        fiber[4 * i + 1] = s * s;
        fiber[4 * i + 2] = s * s * s;
        fiber[4 * i + 3] = 0.f;
    }
}

// ---------------------------------------------------------------- bias + activation
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float x) {
    return 0.5f * (1.0f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}

// nn.SiLU (EquiformerV2 radial function / gates) and SmoothLeakyReLU(0.2) = 0.6 x + 0.4 x (2 sigmoid(x) - 1)
// (equiformer_v2 activation.py; the attention logits)
__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }
__device__ __forceinline__ float act_f(int act, float x) {
    if (act == NBX_ACT_GELU) return gelu_f(x);
    if (act == NBX_ACT_SILU) return x * sigm(x);
    if (act == NBX_ACT_SLRELU) return 0.2f * x + 0.8f * x * sigm(x);
    return x;
}
__device__ __forceinline__ float act_grad(int act, float x) {
    if (act == NBX_ACT_GELU) return gelu_grad(x);
    const float s = sigm(x);
    if (act == NBX_ACT_SILU) return s + x * s * (1.0f - s);
    if (act == NBX_ACT_SLRELU) return 0.2f + 0.8f * (s + x * s * (1.0f - s));
    return 1.0f;
}

// Y[r][c] = act(Z[r][c] + bias[c])
__global__ void bias_act_kernel(int64_t rows, int cols, const float* __restrict__ Z, int64_t ldz,
                                const float* __restrict__ bias, int act, float* __restrict__ Y, int64_t ldy) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= rows * cols) return;
    const int64_t r = i / cols;
    const int c = (int)(i - r * cols);
    Y[r * ldy + c] = act_f(act, Z[r * ldz + c] + (bias ? bias[c] : 0.f));
}

// dZ[r][c] = dY[r][c] act'(Z[r][c] + bias[c])   (dY, dZ contiguous [rows][cols])
__global__ void bias_act_bwd_kernel(int64_t rows, int cols, const float* __restrict__ Z, int64_t ldz,
                                    const float* __restrict__ bias, int act, const float* __restrict__ dY,
                                    float* __restrict__ dZ) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= rows * cols) return;
    const int64_t r = i / cols;
    const int c = (int)(i - r * cols);
    dZ[i] = act == NBX_ACT_NONE ? dY[i] : dY[i] * act_grad(act, Z[r * ldz + c] + (bias ? bias[c] : 0.f));
}

// ---------------------------------------------------------------- spatial message (separable conv)
// X1[v][o][c] = sum_{j in [dptr[v], dptr[v+1])} K[e_j][o][c] H[src[e_j]][o][c],  e_j = deid[j]
__global__ void po_message_kernel(int64_t V, int O, int C, const int* __restrict__ dptr, const int* __restrict__ deid,
                                  const int* __restrict__ src, const float* __restrict__ K,
                                  const float* __restrict__ H, float* __restrict__ X1) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t OC = (int64_t)O * C;
    if (i >= V * OC) return;
    const int64_t v = i / OC;
    const int64_t oc = i - v * OC;
    float acc = 0.f;
    const int j0 = dptr[v], j1 = dptr[v + 1];
    for (int j = j0; j < j1; ++j) {
        const int64_t e = deid[j];
        acc += K[e * OC + oc] * H[(int64_t)src[e] * OC + oc];
    }
    X1[i] = acc;
}

// dK[e][o][c] = dX1[dst_e][o][c] H[src_e][o][c]
__global__ void po_message_bwd_k_kernel(int64_t E, int O, int C, const int* __restrict__ src,
                                        const int* __restrict__ dst, const float* __restrict__ H,
                                        const float* __restrict__ dX1, float* __restrict__ dK) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t OC = (int64_t)O * C;
    if (i >= E * OC) return;
    const int64_t e = i / OC;
    const int64_t oc = i - e * OC;
    dK[i] = dX1[(int64_t)dst[e] * OC + oc] * H[(int64_t)src[e] * OC + oc];
}

// dH[u][o][c] = sum_{j in [sptr[u], sptr[u+1])} dX1[dst[e_j]][o][c] K[e_j][o][c],  e_j = seid[j]
__global__ void po_message_bwd_h_kernel(int64_t V, int O, int C, const int* __restrict__ sptr,
                                        const int* __restrict__ seid, const int* __restrict__ dst,
                                        const float* __restrict__ K, const float* __restrict__ dX1,
                                        float* __restrict__ dH) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t OC = (int64_t)O * C;
    if (i >= V * OC) return;
    const int64_t u = i / OC;
    const int64_t oc = i - u * OC;
    float acc = 0.f;
    const int j0 = sptr[u], j1 = sptr[u + 1];
    for (int j = j0; j < j1; ++j) {
        const int64_t e = seid[j];
        acc += dX1[(int64_t)dst[e] * OC + oc] * K[e * OC + oc];
    }
    dH[i] = acc;
}

// ---------------------------------------------------------------- depth-wise fibre convolution
// X2[v][p][c] = (sum_o X1[v][o][c] FK[o][p][c]) / O + bias[c]
__global__ void po_fiber_kernel(int64_t V, int O, int C, const float* __restrict__ X1, const float* __restrict__ FK,
                                const float* __restrict__ bias, float* __restrict__ X2) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t OC = (int64_t)O * C;
    if (i >= V * OC) return;
    const int64_t v = i / OC;
    const int pc = (int)(i - v * OC);
    const int p = pc / C, c = pc - p * C;
    const float* x = X1 + v * OC + c;
    const float* f = FK + (int64_t)p * C + c;
    float acc = 0.f;
    for (int o = 0; o < O; ++o) acc += x[(int64_t)o * C] * f[(int64_t)o * OC];
    X2[i] = acc / (float)O + (bias ? bias[c] : 0.f);
}

// dX1[v][o][c] = (sum_p dX2[v][p][c] FK[o][p][c]) / O
__global__ void po_fiber_bwd_x_kernel(int64_t V, int O, int C, const float* __restrict__ FK,
                                      const float* __restrict__ dX2, float* __restrict__ dX1) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t OC = (int64_t)O * C;
    if (i >= V * OC) return;
    const int64_t v = i / OC;
    const int oc = (int)(i - v * OC);
    const int o = oc / C, c = oc - o * C;
    const float* g = dX2 + v * OC + c;
    const float* f = FK + (int64_t)o * OC + c;
    float acc = 0.f;
    for (int p = 0; p < O; ++p) acc += g[(int64_t)p * C] * f[(int64_t)p * C];
    dX1[i] = acc / (float)O;
}

// part[chunk][o][p][c] = sum_{v in chunk} X1[v][o][c] dX2[v][p][c]  (fp64, nodes in order)
__global__ void po_fiber_bwd_fk_partial_kernel(int64_t V, int O, int C, int64_t chunk, const float* __restrict__ X1,
                                               const float* __restrict__ dX2, double* __restrict__ part) {
    const int64_t OOC = (int64_t)O * O * C;
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= OOC) return;
    const int64_t OC = (int64_t)O * C;
    const int op = (int)(i / C), c = (int)(i - (int64_t)op * C);
    const int o = op / O, p = op - o * O;
    const int64_t v0 = (int64_t)blockIdx.y * chunk, v1 = std::min<int64_t>(V, v0 + chunk);
    double acc = 0.0;
    for (int64_t v = v0; v < v1; ++v) acc += (double)(X1[v * OC + (int64_t)o * C + c] * dX2[v * OC + (int64_t)p * C + c]);
    part[(int64_t)blockIdx.y * OOC + i] = acc;
}

__global__ void po_fiber_bwd_fk_final_kernel(int64_t n, int nchunks, int O, const double* __restrict__ part,
                                             float* __restrict__ dFK) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    double s = 0.0;
    for (int k = 0; k < nchunks; ++k) s += part[(int64_t)k * n + i];
    dFK[i] = (float)(s / O);
}

int64_t fiber_chunk(int64_t V) { return std::max<int64_t>(64, (V + 63) / 64); }

// ---------------------------------------------------------------- LayerNorm over the channels
// one 64-lane wave per row, C <= 1024 (16 values per lane); save[r] = mean, save[rows + r] = rstd
constexpr int LN_MAXJ = 16;

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    return x;
}

__global__ __launch_bounds__(256) void layernorm_fwd_kernel(int64_t rows, int C, const float* __restrict__ X,
                                                            const float* __restrict__ w, const float* __restrict__ b,
                                                            float eps, float* __restrict__ Y, float* __restrict__ save) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const float* x = X + r * C;
    float v[LN_MAXJ];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < LN_MAXJ; ++j) {
        const int c = lane + 64 * j;
        v[j] = c < C ? x[c] : 0.f;
        s += v[j];
    }
    const float mu = wave_sum(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < LN_MAXJ; ++j) {
        const int c = lane + 64 * j;
        const float d = c < C ? v[j] - mu : 0.f;
        q += d * d;
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)C + eps);
#pragma unroll
    for (int j = 0; j < LN_MAXJ; ++j) {
        const int c = lane + 64 * j;
        if (c < C) Y[r * C + c] = (v[j] - mu) * rstd * w[c] + b[c];
    }
    if (lane == 0) {
        save[r] = mu;
        save[rows + r] = rstd;
    }
}

// dX = rstd (g - mean(g) - xhat mean(g xhat)), g = dY w;  G[r] = [dY xhat | dY] for the parameter sums
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(int64_t rows, int C, const float* __restrict__ X,
                                                            const float* __restrict__ w, const float* __restrict__ save,
                                                            const float* __restrict__ dY, float* __restrict__ dX,
                                                            float* __restrict__ G) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const float mu = save[r], rstd = save[rows + r];
    float xh[LN_MAXJ], g[LN_MAXJ];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int j = 0; j < LN_MAXJ; ++j) {
        const int c = lane + 64 * j;
        if (c < C) {
            const float dy = dY[r * C + c];
            xh[j] = (X[r * C + c] - mu) * rstd;
            g[j] = dy * w[c];
            G[r * 2 * C + c] = dy * xh[j];
            G[r * 2 * C + C + c] = dy;
        } else {
            xh[j] = g[j] = 0.f;
        }
        sg += g[j];
        sgx += g[j] * xh[j];
    }
    const float mg = wave_sum(sg) / (float)C, mgx = wave_sum(sgx) / (float)C;
#pragma unroll
    for (int j = 0; j < LN_MAXJ; ++j) {
        const int c = lane + 64 * j;
        if (c < C) dX[r * C + c] = rstd * (g[j] - mg - xh[j] * mgx);
    }
}

}  // namespace

// ======================================================================== C ABI (include/nbx.h)
extern "C" int nbx_ponita_train_featurize(int64_t V, int64_t E, int32_t O, const float* pos, const float* vel,
                                          const float* mass, const float* ori_grid, const int32_t* src,
                                          const int32_t* dst, float* attr, float* fiber, float* lift, void* stream) {
    NBX_CHECK_ARG(V >= 1 && E >= 0 && O >= 1, "nbx_ponita_train_featurize: bad sizes");
    NBX_CHECK_ARG(pos && vel && mass && ori_grid && fiber && lift && (E == 0 || (src && dst && attr)),
                  "nbx_ponita_train_featurize: null operand");
    NBX_CHECK_ARG((uintptr_t)attr % 16 == 0, "nbx_ponita_train_featurize: attr must be 16-byte aligned");
    const int64_t n = std::max(std::max(E * O, V * O), (int64_t)O * O);
    hipLaunchKernelGGL(po_train_featurize_kernel, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, V, E, O, pos, vel,
                       mass, ori_grid, src, dst, attr, fiber, lift);
    NBX_LAUNCH_CHECK("ponita_train_featurize");
    return NBX_OK;
}

extern "C" int nbx_bias_act(int64_t rows, int32_t cols, const float* Z, int64_t ldz, const float* bias, int32_t act,
                            float* Y, int64_t ldy, void* stream) {
    NBX_CHECK_ARG(rows >= 0 && cols >= 0 && ldz >= cols && ldy >= cols, "nbx_bias_act: bad sizes");
    NBX_CHECK_ARG(act >= NBX_ACT_NONE && act <= NBX_ACT_SLRELU, "nbx_bias_act: unknown activation %d", act);
    if (rows == 0 || cols == 0) return NBX_OK;
    hipLaunchKernelGGL(bias_act_kernel, dim3(nblk(rows * cols)), dim3(256), 0, (hipStream_t)stream, rows, cols, Z, ldz,
                       bias, act, Y, ldy);
    NBX_LAUNCH_CHECK("bias_act");
    return NBX_OK;
}

extern "C" int nbx_bias_act_backward(int64_t rows, int32_t cols, const float* Z, int64_t ldz, const float* bias,
                                     int32_t act, const float* dY, float* dZ, void* stream) {
    NBX_CHECK_ARG(rows >= 0 && cols >= 0 && ldz >= cols, "nbx_bias_act_backward: bad sizes");
    NBX_CHECK_ARG(act >= NBX_ACT_NONE && act <= NBX_ACT_SLRELU, "nbx_bias_act_backward: unknown activation %d",
                  act);
    if (rows == 0 || cols == 0) return NBX_OK;
    hipLaunchKernelGGL(bias_act_bwd_kernel, dim3(nblk(rows * cols)), dim3(256), 0, (hipStream_t)stream, rows, cols, Z,
                       ldz, bias, act, dY, dZ);
    NBX_LAUNCH_CHECK("bias_act_backward");
    return NBX_OK;
}

extern "C" int nbx_po_message(int64_t V, int32_t O, int32_t C, const int32_t* dst_ptr, const int32_t* dst_eid,
                              const int32_t* src, const float* K, const float* H, float* X1, void* stream) {
    NBX_CHECK_ARG(V >= 0 && O >= 1 && C >= 1, "nbx_po_message: bad sizes");
    if (V == 0) return NBX_OK;
    hipLaunchKernelGGL(po_message_kernel, dim3(nblk(V * O * C)), dim3(256), 0, (hipStream_t)stream, V, O, C, dst_ptr,
                       dst_eid, src, K, H, X1);
    NBX_LAUNCH_CHECK("po_message");
    return NBX_OK;
}

extern "C" int nbx_po_message_backward(int64_t V, int64_t E, int32_t O, int32_t C, const int32_t* src,
                                       const int32_t* dst, const int32_t* src_ptr, const int32_t* src_eid,
                                       const float* K, const float* H, const float* dX1, float* dK, float* dH,
                                       void* stream) {
    NBX_CHECK_ARG(V >= 0 && E >= 0 && O >= 1 && C >= 1, "nbx_po_message_backward: bad sizes");
    hipStream_t st = (hipStream_t)stream;
    if (E > 0 && dK) {
        hipLaunchKernelGGL(po_message_bwd_k_kernel, dim3(nblk(E * O * C)), dim3(256), 0, st, E, O, C, src, dst, H, dX1,
                           dK);
        NBX_LAUNCH_CHECK("po_message_bwd_k");
    }
    if (V > 0 && dH) {
        hipLaunchKernelGGL(po_message_bwd_h_kernel, dim3(nblk(V * O * C)), dim3(256), 0, st, V, O, C, src_ptr, src_eid,
                           dst, K, dX1, dH);
        NBX_LAUNCH_CHECK("po_message_bwd_h");
    }
    return NBX_OK;
}

extern "C" int nbx_po_fiber_conv(int64_t V, int32_t O, int32_t C, const float* X1, const float* FK, const float* bias,
                                 float* X2, void* stream) {
    NBX_CHECK_ARG(V >= 0 && O >= 1 && C >= 1, "nbx_po_fiber_conv: bad sizes");
    if (V == 0) return NBX_OK;
    hipLaunchKernelGGL(po_fiber_kernel, dim3(nblk(V * O * C)), dim3(256), 0, (hipStream_t)stream, V, O, C, X1, FK, bias,
                       X2);
    NBX_LAUNCH_CHECK("po_fiber_conv");
    return NBX_OK;
}

extern "C" int nbx_po_fiber_conv_workspace_bytes(int64_t V, int32_t O, int32_t C, size_t* bytes) {
    NBX_CHECK_ARG(bytes && V >= 0 && O >= 1 && C >= 1, "nbx_po_fiber_conv_workspace_bytes: bad arguments");
    const int64_t nch = std::max<int64_t>(1, (V + fiber_chunk(V) - 1) / fiber_chunk(V));
    *bytes = (size_t)nch * O * O * C * sizeof(double);
    return NBX_OK;
}

extern "C" int nbx_po_fiber_conv_backward(int64_t V, int32_t O, int32_t C, const float* X1, const float* FK,
                                          const float* dX2, float* dX1, float* dFK, void* workspace,
                                          size_t workspace_bytes, void* stream) {
    NBX_CHECK_ARG(V >= 1 && O >= 1 && C >= 1, "nbx_po_fiber_conv_backward: bad sizes");
    hipStream_t st = (hipStream_t)stream;
    if (dX1) {
        hipLaunchKernelGGL(po_fiber_bwd_x_kernel, dim3(nblk(V * O * C)), dim3(256), 0, st, V, O, C, FK, dX2, dX1);
        NBX_LAUNCH_CHECK("po_fiber_bwd_x");
    }
    if (dFK) {
        const int64_t chunk = fiber_chunk(V);
        const int nch = (int)((V + chunk - 1) / chunk);
        const int64_t n = (int64_t)O * O * C;
        NBX_CHECK_ARG(workspace && workspace_bytes >= (size_t)nch * n * sizeof(double),
                      "nbx_po_fiber_conv_backward: workspace too small");
        double* part = (double*)workspace;
        hipLaunchKernelGGL(po_fiber_bwd_fk_partial_kernel, dim3(nblk(n), (unsigned)nch), dim3(256), 0, st, V, O, C,
                           chunk, X1, dX2, part);
        NBX_LAUNCH_CHECK("po_fiber_bwd_fk_partial");
        hipLaunchKernelGGL(po_fiber_bwd_fk_final_kernel, dim3(nblk(n)), dim3(256), 0, st, n, nch, O, part, dFK);
        NBX_LAUNCH_CHECK("po_fiber_bwd_fk_final");
    }
    return NBX_OK;
}

extern "C" int nbx_layernorm_forward(int64_t rows, int32_t C, const float* X, const float* weight, const float* bias,
                                     float eps, float* Y, float* save, void* stream) {
    NBX_CHECK_ARG(rows >= 0 && C >= 1 && C <= 64 * LN_MAXJ, "nbx_layernorm_forward: need 1 <= C <= %d", 64 * LN_MAXJ);
    if (rows == 0) return NBX_OK;
    hipLaunchKernelGGL(layernorm_fwd_kernel, dim3(nblk(rows, 4)), dim3(256), 0, (hipStream_t)stream, rows, C, X, weight,
                       bias, eps, Y, save);
    NBX_LAUNCH_CHECK("layernorm_fwd");
    return NBX_OK;
}

extern "C" int nbx_layernorm_backward(int64_t rows, int32_t C, const float* X, const float* weight, const float* save,
                                      const float* dY, float* dX, float* G, void* stream) {
    NBX_CHECK_ARG(rows >= 0 && C >= 1 && C <= 64 * LN_MAXJ, "nbx_layernorm_backward: need 1 <= C <= %d", 64 * LN_MAXJ);
    if (rows == 0) return NBX_OK;
    hipLaunchKernelGGL(layernorm_bwd_kernel, dim3(nblk(rows, 4)), dim3(256), 0, (hipStream_t)stream, rows, C, X, weight,
                       save, dY, dX, G);
    NBX_LAUNCH_CHECK("layernorm_bwd");
    return NBX_OK;
}
