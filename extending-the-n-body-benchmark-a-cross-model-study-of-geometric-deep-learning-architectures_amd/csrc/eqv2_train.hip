// EquiformerV2 training step (trainer.py:233-358: pred = model(data); loss.backward())
// — the EquiformerV2-specific operators of the training forward and backward (fp32).  The dense
// layers (distance expansion, radial MLPs, SO(2) convolutions' fc layers, SO3_LinearV2 per degree,
// gating and embedding layers) run on nbx_gemm_f32 with nbx_bias_act (SiLU / SmoothLeakyReLU) and
// nbx_layernorm_*; the edge frames on nbx_eqv2_train_edges (csrc/eqv2.hip); this file adds, on the
// layout of DESIGN.md §6.5 (node irreps [V][9][C], edge irreps [E][7 or 9][C], coefficients
// l-primary, channels contiguous):
//   * the edge-frame rotation of irreps (SO3_Rotation.rotate / rotate_inv, so3.py:485-531) with
//     the reduced Wigner rows Dsel [E][7][9] and the l = 2 rescale of get_rotate_inv_rescale
//     (so3.py:160-185), and their adjoints;
//   * the separable S2 activation's grid round trip out = F^T SiLU(T x) (activation.py:155-202,
//     SO3_Grid to / from grid matrices) and its backward;
//   * the segment softmax of the attention logits over edge_index[1] (torch_geometric softmax,
//     transformer_block.py:331-339, + 1e-16) and its backward;
//   * EquivariantRMSNormArraySphericalHarmonicsV2 (layer_norm.py:327-441: l = 0 centering, degree-
//     balanced RMS over (coefficient, channel), per-degree affine weight, l = 0 bias) and its backward.
// Every reduction runs in a fixed order: the training step is bit-reproducible.
#include <algorithm>

#include "nbx_internal.h"

namespace {

unsigned nblk(int64_t n, int t = 256) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

constexpr float kRescale2 = 1.2909944487358056f;   // sqrt(5 / 3): l = 2 > mmax = 1

// ---------------------------------------------------------------- edge-frame rotation
// MODE 0: out [E][7][C] = Dsel in [E][9][C]       (rotate; rescale: rows l = 2 times sqrt(5/3))
// MODE 1: out [E][9][C] = Dsel^T in [E][7][C]     (rotate_inv; rescale: outputs l = 2 times sqrt(5/3))
// in may carry a row stride (ld_in floats between consecutive edges' blocks) and a channel offset.
template <int MODE>
__global__ void eqv2_rotate_kernel(int64_t E, int C, const float* __restrict__ D, const float* __restrict__ in,
                                   int64_t ld_in, float* __restrict__ out, int rescale) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= E * C) return;
    const int64_t e = i / C;
    const int c = (int)(i - e * C);
    const float* d = D + e * 63;
    const float* x = in + e * ld_in + c;
    if (MODE == 0) {
        float v[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) v[k] = x[(int64_t)k * C];
        float* o = out + e * 7 * C + c;
        o[0] = v[0];
#pragma unroll
        for (int r = 1; r < 4; ++r) o[(int64_t)r * C] = d[r * 9 + 1] * v[1] + d[r * 9 + 2] * v[2] + d[r * 9 + 3] * v[3];
        const float s = rescale ? kRescale2 : 1.0f;
#pragma unroll
        for (int r = 4; r < 7; ++r) {
            float a = 0.f;
#pragma unroll
            for (int k = 4; k < 9; ++k) a += d[r * 9 + k] * v[k];
            o[(int64_t)r * C] = s * a;
        }
    } else {
        float v[7];
#pragma unroll
        for (int r = 0; r < 7; ++r) v[r] = x[(int64_t)r * C];
        float* o = out + e * 9 * C + c;
        o[0] = v[0];
#pragma unroll
        for (int k = 1; k < 4; ++k) o[(int64_t)k * C] = d[9 + k] * v[1] + d[18 + k] * v[2] + d[27 + k] * v[3];
        const float s = rescale ? kRescale2 : 1.0f;
#pragma unroll
        for (int k = 4; k < 9; ++k) o[(int64_t)k * C] = s * (d[36 + k] * v[4] + d[45 + k] * v[5] + d[54 + k] * v[6]);
    }
}

// ---------------------------------------------------------------- separable S2 activation (grid part)
// out[r][i][h] = sum_p F[p][i] SiLU(sum_j T[p][j] x[r][j][h]) for the I coefficients of a row and P
// grid points; backward dx[r][j][h] = sum_p T[p][j] SiLU'(t_p) sum_i F[p][i] dout[r][i][h].  T and F
// sit in LDS (2 P I4 floats, I padded to 4: 87 KB at lmax 6, SO3_Grid(6, 6) = 14 x 15 points); a thread keeps one
// (row, channel)'s coefficients in registers (MAXI = 9 up to lmax 2, 49 up to lmax 6).
constexpr int S2_MAXI = 49, S2_MAXP = 240;   // LDS: 2 x 240 x 52 floats = 99.8 KB

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }

template <int MAXI, bool BWD, int NT>
__global__ __launch_bounds__(NT) void eqv2_s2_kernel(int64_t rows, int I, int P, int H, const float* __restrict__ T,
                                                      const float* __restrict__ F, const float* __restrict__ X,
                                                      const float* __restrict__ dOut, float* __restrict__ out) {
    // T / F rows padded to a multiple of 4 coefficients with zeros and read as float4: the lanes of a
    // wave share one row, so each ds_read_b128 is a broadcast feeding four FMAs (one b32 read per FMA
    // left the kernel LDS-issue bound)
    constexpr int M4 = (MAXI + 3) / 4;
    extern __shared__ __attribute__((aligned(16))) float s2_lds[];
    const int I4 = (I + 3) >> 2;
    float4* sT = reinterpret_cast<float4*>(s2_lds);
    float4* sF = sT + P * I4;
    for (int k = threadIdx.x; k < P * I4 * 4; k += blockDim.x) {
        const int p = k / (I4 * 4), i = k - p * I4 * 4;
        s2_lds[k] = i < I ? T[p * I + i] : 0.f;
        s2_lds[P * I4 * 4 + k] = i < I ? F[p * I + i] : 0.f;
    }
    __syncthreads();
    const int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (g >= rows * H) return;
    const int64_t r = g / H;
    const int h = (int)(g - r * H);
    const int64_t base = r * I * H + h;
    float x[4 * M4], d[4 * M4], o[4 * M4];
#pragma unroll
    for (int i = 0; i < 4 * M4; ++i) {
        x[i] = i < I ? X[base + (int64_t)i * H] : 0.f;
        d[i] = (BWD && i < I) ? dOut[base + (int64_t)i * H] : 0.f;
        o[i] = 0.f;
    }
    for (int p = 0; p < P; ++p) {
        const float4* tp = sT + p * I4;
        const float4* fp = sF + p * I4;
        // four independent chains (one per float4 component): a single chain of I dependent FMAs per
        // grid point was latency bound at the one or two waves per SIMD the LDS footprint allows
        float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
#pragma unroll
        for (int q = 0; q < M4; ++q)
            if (q < I4) {
                const float4 v = tp[q];
                t0 = fmaf(v.x, x[4 * q], t0); t1 = fmaf(v.y, x[4 * q + 1], t1);
                t2 = fmaf(v.z, x[4 * q + 2], t2); t3 = fmaf(v.w, x[4 * q + 3], t3);
            }
        const float t = (t0 + t1) + (t2 + t3);
        const float s = sigm(t);
        if (!BWD) {
            const float a = t * s;
#pragma unroll
            for (int q = 0; q < M4; ++q)
                if (q < I4) {
                    const float4 v = fp[q];
                    o[4 * q] += v.x * a; o[4 * q + 1] += v.y * a; o[4 * q + 2] += v.z * a; o[4 * q + 3] += v.w * a;
                }
        } else {
            float g0 = 0.f, g1 = 0.f, g2 = 0.f, g3 = 0.f;
#pragma unroll
            for (int q = 0; q < M4; ++q)
                if (q < I4) {
                    const float4 v = fp[q];
                    g0 = fmaf(v.x, d[4 * q], g0); g1 = fmaf(v.y, d[4 * q + 1], g1);
                    g2 = fmaf(v.z, d[4 * q + 2], g2); g3 = fmaf(v.w, d[4 * q + 3], g3);
                }
            const float gsum = (g0 + g1) + (g2 + g3);
            const float dt = gsum * (s + t * s * (1.0f - s));
#pragma unroll
            for (int q = 0; q < M4; ++q)
                if (q < I4) {
                    const float4 v = tp[q];
                    o[4 * q] += v.x * dt; o[4 * q + 1] += v.y * dt; o[4 * q + 2] += v.z * dt; o[4 * q + 3] += v.w * dt;
                }
        }
    }
#pragma unroll
    for (int i = 0; i < 4 * M4; ++i)
        if (i < I) out[base + (int64_t)i * H] = o[i];
}

#ifndef NBX_S2_NT32
#define NBX_S2_NT32 512
#endif
// block threads of the I <= 32 form (-DNBX_S2_NT32 A/B builds): eqv2_l6 63.3 steps/s at 512 against 63.1 at
// 256 and 62.0 at 1 024, same box (profiles/r06/s2_l6/nt_*)
constexpr int S2_NT32 = NBX_S2_NT32;

template <bool BWD>
int s2_launch(int64_t rows, int I, int P, int H, const float* T, const float* F, const float* X, const float* dOut,
              float* out, hipStream_t st) {
    const size_t lds = 2 * (size_t)P * ((I + 3) / 4 * 4) * sizeof(float);
    const int which = I <= 9 ? 0 : I <= 32 ? 1 : 2;
    // one copy of the grid matrices per block: the large-I forms take 512 threads, so the LDS that
    // limits a CU to one or two blocks still holds 2+ waves per SIMD; the lmax 2 form keeps 256
    const int nt = which == 0 ? 256 : which == 1 ? S2_NT32 : 512;
    auto kern = which == 0 ? eqv2_s2_kernel<9, BWD, 256>
              : which == 1 ? eqv2_s2_kernel<32, BWD, S2_NT32> : eqv2_s2_kernel<S2_MAXI, BWD, 512>;
    if (lds > 64 * 1024) NBX_LDS_160K(kern);
    hipLaunchKernelGGL(kern, dim3(nblk(rows * H, nt)), dim3(nt), lds, st, rows, I, P, H, T, F, X, dOut, out);
    return NBX_OK;
}

// ---------------------------------------------------------------- segment softmax over edge_index[1]
// alpha[e][h] = exp(l[e][h] - max) / (sum over the edges into dst_e of exp(l - max) + 1e-16)
__global__ void eqv2_softmax_kernel(int64_t V, int nh, const int* __restrict__ dptr, const int* __restrict__ deid,
                                    const float* __restrict__ L, float* __restrict__ A) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= V * nh) return;
    const int64_t v = i / nh;
    const int h = (int)(i - v * nh);
    const int j0 = dptr[v], j1 = dptr[v + 1];
    float mx = -INFINITY;
    for (int j = j0; j < j1; ++j) mx = fmaxf(mx, L[(int64_t)deid[j] * nh + h]);
    float s = 0.f;
    for (int j = j0; j < j1; ++j) s += __expf(L[(int64_t)deid[j] * nh + h] - mx);
    const float inv = 1.0f / (s + 1e-16f);
    for (int j = j0; j < j1; ++j) {
        const int64_t e = deid[j];
        A[e * nh + h] = __expf(L[e * nh + h] - mx) * inv;
    }
}

// dl[e][h] = alpha[e][h] (dalpha[e][h] - sum over the edges e' into dst_e of alpha[e'][h] dalpha[e'][h])
__global__ void eqv2_softmax_bwd_kernel(int64_t V, int nh, const int* __restrict__ dptr, const int* __restrict__ deid,
                                        const float* __restrict__ A, const float* __restrict__ dA,
                                        float* __restrict__ dL) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= V * nh) return;
    const int64_t v = i / nh;
    const int h = (int)(i - v * nh);
    const int j0 = dptr[v], j1 = dptr[v + 1];
    float s = 0.f;
    for (int j = j0; j < j1; ++j) {
        const int64_t e = deid[j];
        s += A[e * nh + h] * dA[e * nh + h];
    }
    for (int j = j0; j < j1; ++j) {
        const int64_t e = deid[j];
        dL[e * nh + h] = A[e * nh + h] * (dA[e * nh + h] - s);
    }
}

// ---------------------------------------------------------------- RMS norm over the spherical harmonics
// one 64-lane wave per node, lane = channel c (+ 64 k), C <= 128; coefficient i of degree l(i):
//   xc = x (l = 0 row centred over channels), n = (1/C) sum_{i,c} bal(i) xc[i][c]^2, bal = 1/((2l+1)(L+1))
//   out[i][c] = xc[i][c] (n + eps)^-1/2 w[l(i)][c] (+ b[c] for i = 0)
constexpr int RMS_MAXK = 2;

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    return x;
}

__device__ __forceinline__ int deg_of(int i) { return i == 0 ? 0 : (i < 4 ? 1 : 2); }

__global__ __launch_bounds__(256) void eqv2_rmsnorm_kernel(int64_t V, int C, const float* __restrict__ X,
                                                          const float* __restrict__ w, const float* __restrict__ b,
                                                          float eps, float* __restrict__ Y, float* __restrict__ save) {
    const int lane = threadIdx.x & 63;
    const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= V) return;
    const float* x = X + v * 9 * C;
    float xc[RMS_MAXK][9];
    float m0 = 0.f;
#pragma unroll
    for (int k = 0; k < RMS_MAXK; ++k) {
        const int c = lane + 64 * k;
#pragma unroll
        for (int i = 0; i < 9; ++i) xc[k][i] = c < C ? x[i * C + c] : 0.f;
        m0 += xc[k][0];
    }
    m0 = wave_sum(m0) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < RMS_MAXK; ++k) {
        const int c = lane + 64 * k;
        if (c < C) xc[k][0] -= m0;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const float bal = 1.0f / ((2 * deg_of(i) + 1) * 3.0f);
            q += bal * xc[k][i] * xc[k][i];
        }
    }
    const float n = wave_sum(q) / (float)C;
    const float s = 1.0f / sqrtf(n + eps);
#pragma unroll
    for (int k = 0; k < RMS_MAXK; ++k) {
        const int c = lane + 64 * k;
        if (c >= C) continue;
#pragma unroll
        for (int i = 0; i < 9; ++i) Y[v * 9 * C + i * C + c] = xc[k][i] * s * w[deg_of(i) * C + c] + (i == 0 ? b[c] : 0.f);
    }
    if (lane == 0) {
        save[v] = m0;
        save[V + v] = s;
    }
}

// dX, and G [V][4C] = (sum over the degree-l coefficients of dY xc s for l = 0, 1, 2 | dY[0]): the
// column sums of G are dweight [3][C] | dbias [C]
__global__ __launch_bounds__(256) void eqv2_rmsnorm_bwd_kernel(int64_t V, int C, const float* __restrict__ X,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ save,
                                                              const float* __restrict__ dY, float* __restrict__ dX,
                                                              float* __restrict__ G) {
    const int lane = threadIdx.x & 63;
    const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= V) return;
    const float m0 = save[v], s = save[V + v];
    const float* x = X + v * 9 * C;
    const float* dy = dY + v * 9 * C;
    float xc[RMS_MAXK][9], g[RMS_MAXK][9];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < RMS_MAXK; ++k) {
        const int c = lane + 64 * k;
        const bool on = c < C;
        float gw[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            xc[k][i] = on ? x[i * C + c] - (i == 0 ? m0 : 0.f) : 0.f;
            const float d = on ? dy[i * C + c] : 0.f;
            g[k][i] = on ? d * w[deg_of(i) * C + c] : 0.f;
            gw[deg_of(i)] += d * xc[k][i] * s;
            dot += g[k][i] * xc[k][i];
        }
        if (on) {
            float* gr = G + v * 4 * C;
            gr[c] = gw[0];
            gr[C + c] = gw[1];
            gr[2 * C + c] = gw[2];
            gr[3 * C + c] = dy[c];
        }
    }
    dot = wave_sum(dot);
    const float coef = s * s * s / (float)C * dot;
    // d xc[i][c] = s g[i][c] - coef bal(i) xc[i][c];  l = 0 row: minus its channel mean (centering)
    float dm = 0.f;
#pragma unroll
    for (int k = 0; k < RMS_MAXK; ++k) {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const float bal = 1.0f / ((2 * deg_of(i) + 1) * 3.0f);
            g[k][i] = s * g[k][i] - coef * bal * xc[k][i];
        }
        if (lane + 64 * k < C) dm += g[k][0];
    }
    dm = wave_sum(dm) / (float)C;
#pragma unroll
    for (int k = 0; k < RMS_MAXK; ++k) {
        const int c = lane + 64 * k;
        if (c >= C) continue;
#pragma unroll
        for (int i = 0; i < 9; ++i) dX[v * 9 * C + i * C + c] = g[k][i] - (i == 0 ? dm : 0.f);
    }
}

}  // namespace

// ======================================================================== C ABI (include/nbx.h)
extern "C" int nbx_eqv2_rotate(int64_t E, int32_t C, const float* dsel, const float* in, int64_t ld_in, float* out,
                               int32_t inverse, int32_t rescale, void* stream) {
    NBX_CHECK_ARG(E >= 0 && C >= 1 && ld_in >= (inverse ? 7 : 9) * (int64_t)C, "nbx_eqv2_rotate: bad sizes");
    if (E == 0) return NBX_OK;
    hipStream_t st = (hipStream_t)stream;
    if (inverse)
        hipLaunchKernelGGL(eqv2_rotate_kernel<1>, dim3(nblk(E * C)), dim3(256), 0, st, E, C, dsel, in, ld_in, out,
                           rescale);
    else
        hipLaunchKernelGGL(eqv2_rotate_kernel<0>, dim3(nblk(E * C)), dim3(256), 0, st, E, C, dsel, in, ld_in, out,
                           rescale);
    NBX_LAUNCH_CHECK("eqv2_rotate");
    return NBX_OK;
}

extern "C" int nbx_eqv2_s2_act(int64_t rows, int32_t I, int32_t P, int32_t H, const float* to_grid,
                               const float* from_grid, const float* X, float* out, void* stream) {
    NBX_CHECK_ARG(rows >= 0 && I >= 1 && I <= S2_MAXI && P >= 1 && P <= S2_MAXP && H >= 1,
                  "nbx_eqv2_s2_act: need I <= %d coefficients, P <= %d grid points", S2_MAXI, S2_MAXP);
    if (rows == 0) return NBX_OK;
    if (int rc = s2_launch<false>(rows, I, P, H, to_grid, from_grid, X, nullptr, out, (hipStream_t)stream)) return rc;
    NBX_LAUNCH_CHECK("eqv2_s2_act");
    return NBX_OK;
}

extern "C" int nbx_eqv2_s2_act_backward(int64_t rows, int32_t I, int32_t P, int32_t H, const float* to_grid,
                                        const float* from_grid, const float* X, const float* dOut, float* dX,
                                        void* stream) {
    NBX_CHECK_ARG(rows >= 0 && I >= 1 && I <= S2_MAXI && P >= 1 && P <= S2_MAXP && H >= 1,
                  "nbx_eqv2_s2_act_backward: need I <= %d coefficients, P <= %d grid points", S2_MAXI, S2_MAXP);
    if (rows == 0) return NBX_OK;
    if (int rc = s2_launch<true>(rows, I, P, H, to_grid, from_grid, X, dOut, dX, (hipStream_t)stream)) return rc;
    NBX_LAUNCH_CHECK("eqv2_s2_act_backward");
    return NBX_OK;
}

extern "C" int nbx_segment_softmax(int64_t V, int32_t nh, const int32_t* dst_ptr, const int32_t* dst_eid,
                                   const float* logits, float* alpha, void* stream) {
    NBX_CHECK_ARG(V >= 0 && nh >= 1, "nbx_segment_softmax: bad sizes");
    if (V == 0) return NBX_OK;
    hipLaunchKernelGGL(eqv2_softmax_kernel, dim3(nblk(V * nh)), dim3(256), 0, (hipStream_t)stream, V, nh, dst_ptr,
                       dst_eid, logits, alpha);
    NBX_LAUNCH_CHECK("segment_softmax");
    return NBX_OK;
}

extern "C" int nbx_segment_softmax_backward(int64_t V, int32_t nh, const int32_t* dst_ptr, const int32_t* dst_eid,
                                            const float* alpha, const float* dalpha, float* dlogits, void* stream) {
    NBX_CHECK_ARG(V >= 0 && nh >= 1, "nbx_segment_softmax_backward: bad sizes");
    if (V == 0) return NBX_OK;
    hipLaunchKernelGGL(eqv2_softmax_bwd_kernel, dim3(nblk(V * nh)), dim3(256), 0, (hipStream_t)stream, V, nh, dst_ptr,
                       dst_eid, alpha, dalpha, dlogits);
    NBX_LAUNCH_CHECK("segment_softmax_backward");
    return NBX_OK;
}

extern "C" int nbx_eqv2_rms_norm(int64_t V, int32_t C, const float* X, const float* weight, const float* bias,
                                 float eps, float* Y, float* save, void* stream) {
    NBX_CHECK_ARG(V >= 0 && C >= 1 && C <= 64 * RMS_MAXK, "nbx_eqv2_rms_norm: need 1 <= C <= %d", 64 * RMS_MAXK);
    if (V == 0) return NBX_OK;
    hipLaunchKernelGGL(eqv2_rmsnorm_kernel, dim3(nblk(V, 4)), dim3(256), 0, (hipStream_t)stream, V, C, X, weight, bias,
                       eps, Y, save);
    NBX_LAUNCH_CHECK("eqv2_rms_norm");
    return NBX_OK;
}

extern "C" int nbx_eqv2_rms_norm_backward(int64_t V, int32_t C, const float* X, const float* weight, const float* save,
                                          const float* dY, float* dX, float* G, void* stream) {
    NBX_CHECK_ARG(V >= 0 && C >= 1 && C <= 64 * RMS_MAXK, "nbx_eqv2_rms_norm_backward: need 1 <= C <= %d",
                  64 * RMS_MAXK);
    if (V == 0) return NBX_OK;
    hipLaunchKernelGGL(eqv2_rmsnorm_bwd_kernel, dim3(nblk(V, 4)), dim3(256), 0, (hipStream_t)stream, V, C, X, weight,
                       save, dY, dX, G);
    NBX_LAUNCH_CHECK("eqv2_rms_norm_backward");
    return NBX_OK;
}
