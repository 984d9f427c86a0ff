// EquiformerV2 at general degrees (ABI 13): lmax <= 6, mmax <= lmax — the reference constructor's
// default lmax_list = [6], mmax_list = [2] (equiformer_v2_nbody.py:122-123) and every other single-
// resolution choice.  The composed forward / training step (eqv2_train.py) runs on these operators
// plus the generic ones (nbx_gemm_f32, nbx_bias_act, nbx_layernorm_*, nbx_gather_rows /
// nbx_segment_sum, nbx_segment_softmax, nbx_eqv2_s2_act):
//   * nbx_eqv2_wigner: the kept (|m| <= mmax) rows of every degree's Wigner block D^l(R) of the edge
//     frame R (SO3_Rotation.set_wigner, so3.py:485-531).  D^0 = 1, D^1 = R, and for l >= 2
//     D^l = [Y^l(R u_k)]_k P_l over the probe vectors u_k and P_l = pinv([Y^l(u_k)]_k) of the host
//     table (so3.py wigner_table): exact because Y^l(R u) = D^l(R) Y^l(u), no Euler angles, so no
//     gimbal singularity (the reference goes through xyz_to_angles + Jd.pt: the same matrix);
//   * nbx_eqv2_rotate_general: rotate (D_sel x) / rotate_inv (D_sel^T y, times get_rotate_inv_rescale's
//     sqrt((2l+1)/(2 mmax+1)) for l > mmax, so3.py:160-185) — each the other's adjoint;
//   * nbx_eqv2_rms_norm_general (+ backward): EquivariantRMSNormArraySphericalHarmonicsV2
//     (layer_norm.py:327-441) at any lmax and channel count.
// Layouts: node irreps [V][(lmax+1)^2][C], edge irreps [E][R][C] with R kept coefficients (l-primary),
// channels contiguous; dsel [E][S] with degree blocks [2 min(l, mmax)+1][2l+1] back to back
// (S = so3.Layout.dsel_floats).  Every reduction runs in a fixed order (bit-reproducible).
#include <algorithm>
#include <cmath>

#include "nbx_internal.h"

namespace {

constexpr int GL_MAX = 6;                 // largest degree
constexpr int GN_MAX = 2 * GL_MAX + 1;    // coefficients of one degree

unsigned nblk(int64_t n, int t = 256) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    return x;
}

__device__ __forceinline__ int kept(int l, int mmax) { return 2 * (l < mmax ? l : mmax) + 1; }

// e3nn real harmonic Y_lm (component normalisation, y polar, no Condon-Shortley phase) at unit v,
// without the degree's constant sqrt(2l+1) sqrt((l-|m|)!/(l+|m|)!) (applied by the caller)
__device__ float sh_lm_unnormed(int l, int m, float x, float y, float z) {
    const int am = m < 0 ? -m : m;
    float re = 1.f, im = 0.f;                     // (z + i x)^|m|
    for (int k = 0; k < am; ++k) {
        const float nr = re * z - im * x, ni = re * x + im * z;
        re = nr;
        im = ni;
    }
    float a = 1.f;                                // Q_|m|^|m| = (2|m| - 1)!!
    for (int k = 2 * am - 1; k > 0; k -= 2) a *= (float)k;
    float q = a;
    if (l > am) {
        float b = (float)(2 * am + 1) * y * a;
        for (int k = am + 2; k <= l; ++k) {
            const float c = ((float)(2 * k - 1) * y * b - (float)(k + am - 1) * a) / (float)(k - am);
            a = b;
            b = c;
        }
        q = b;
    }
    const float ang = m > 0 ? 1.4142135623730951f * re : (m < 0 ? 1.4142135623730951f * im : 1.f);
    return q * ang;
}

// thread = (edge, kept row of some degree); dsel[e][off_l + i (2l+1) + j] = D^l[l + m_i][j]
__global__ void eqv2_wigner_kernel(int64_t E, int lmax, int mmax, int rows, int S, const float* __restrict__ rot,
                                   int64_t ld_rot, const float* __restrict__ table, float* __restrict__ dsel) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= E * rows) return;
    const int64_t e = t / rows;
    int r = (int)(t - e * rows);
    int l = 0, off = 0, toff = 0;
    while (r >= kept(l, mmax)) {                  // locate the degree of this kept row
        r -= kept(l, mmax);
        off += kept(l, mmax) * (2 * l + 1);
        if (l >= 2) toff += (l + 1) * (2 * l + 1) * (2 * l + 4);
        ++l;
    }
    const int mm = l < mmax ? l : mmax;
    const int m = r - mm;                         // order of this row
    const int n = 2 * l + 1;
    float R[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = rot[e * ld_rot + k];
    float* out = dsel + e * S + off + r * n;
    if (l == 0) {
        out[0] = 1.f;
        return;
    }
    if (l == 1) {                                 // D^1 = R in e3nn's (x, y, z) basis
#pragma unroll
        for (int j = 0; j < 3; ++j) out[j] = R[3 * (m + 1) + j];
        return;
    }
    const int K = (l + 1) * n;
    const float* u = table + toff;
    const float* P = u + 3 * K;
    const int am = m < 0 ? -m : m;
    float ratio = 1.f;
    for (int k = l - am + 1; k <= l + am; ++k) ratio /= (float)k;
    const float nrm = sqrtf((float)n * ratio);
    float acc[GN_MAX];
#pragma unroll
    for (int j = 0; j < GN_MAX; ++j) acc[j] = 0.f;
    for (int k = 0; k < K; ++k) {
        const float ux = u[3 * k], uy = u[3 * k + 1], uz = u[3 * k + 2];
        const float vx = R[0] * ux + R[1] * uy + R[2] * uz;
        const float vy = R[3] * ux + R[4] * uy + R[5] * uz;
        const float vz = R[6] * ux + R[7] * uy + R[8] * uz;
        const float y = nrm * sh_lm_unnormed(l, m, vx, vy, vz);
        const float* p = P + k * n;
#pragma unroll
        for (int j = 0; j < GN_MAX; ++j)
            if (j < n) acc[j] += y * p[j];
    }
#pragma unroll
    for (int j = 0; j < GN_MAX; ++j)
        if (j < n) out[j] = acc[j];
}

// get_rotate_inv_rescale: float32(sqrt((2l+1)/(2 mmax+1))) for l > mmax
__device__ __forceinline__ float inv_rescale(int l, int mmax) {
    return l > mmax ? (float)sqrt((double)(2 * l + 1) / (double)(2 * mmax + 1)) : 1.f;
}

// MODE 0 (rotate):     out [E][R][C]          = D_sel in (x rescale), in [E][(lmax+1)^2][C] (ld_in per edge)
// MODE 1 (rotate_inv): out [E][(lmax+1)^2][C] = D_sel^T in (x rescale), in [E][R][C] (ld_in per edge)
// order (nullable): the edge-side row of kept coefficient k (l-primary) is order[k] -- e.g. the
// m-primary order of SO2_Convolution, so the SO(2) blocks read contiguous rows without a permutation.
// UNI (C a multiple of 64): a wave's lanes share one edge, made explicit with readfirstlane, so the
// edge's Wigner block and the row order are read once per wave through the scalar cache instead of
// once per lane (455 per-lane loads per output channel at lmax 6 / mmax 2).
// GATHER (MODE 0): in is the node array [V][(lmax+1)^2][C / 2] (ld_in floats per node) and edge e's
// input is [in[src[e]] | in[dst[e]]] per coefficient -- the attention's gathered message, read in
// place instead of materialised (nbx_eqv2_rotate_gather)
// rad (GATHER, nullable): output row j of edge e is multiplied by rad[e ld_rad + radrow[j] C + c], the
// SO(2) convolution's radial weights applied in the epilogue (inference; the same single rounding as
// the separate product)
// LDSD (C < 64 dividing the 256-thread block, not UNI): the block's 256 / C edges share a wave, so their
// Wigner blocks are staged once in the LDS (coalesced) and read from there, not per lane from memory
template <int MODE, bool UNI, bool GATHER = false, bool LDSD = false>
__global__ void eqv2_rotate_general_kernel(int64_t E, int C, int lmax, int mmax, int S, int R,
                                           const float* __restrict__ D, const float* __restrict__ in, int64_t ld_in,
                                           float* __restrict__ out, int rescale, const int* __restrict__ order,
                                           const int* __restrict__ src = nullptr,
                                           const int* __restrict__ dst = nullptr,
                                           const float* __restrict__ rad = nullptr, int64_t ld_rad = 0,
                                           const int* __restrict__ radrow = nullptr) {
    extern __shared__ float rot_lds[];
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * (blockDim.x / C);   // LDSD: the block's first edge
    if constexpr (LDSD) {
        const int64_t n = std::min<int64_t>(blockDim.x / C, E - e0) * S;
        for (int64_t k = threadIdx.x; k < n; k += blockDim.x) rot_lds[k] = D[e0 * S + k];
        __syncthreads();
    }
    if (t >= E * C) return;
    const int64_t e = UNI ? (int64_t)__builtin_amdgcn_readfirstlane((int)(t / C)) : t / C;
    const int c = (int)(t - e * C);
    const float* d;
    if constexpr (LDSD) d = rot_lds + (e - e0) * S;
    else d = D + e * S;
    const int half = C >> 1;
    const float* x = GATHER ? (c < half ? in + (int64_t)src[e] * ld_in + c : in + (int64_t)dst[e] * ld_in + (c - half))
                            : in + e * ld_in + c;
    const int xs = GATHER ? half : C;   // stride between the coefficient rows of x
    const int K = (lmax + 1) * (lmax + 1);
    float* o = out + e * (int64_t)(MODE == 0 ? R : K) * C + c;
    int doff = 0, roff = 0;
    for (int l = 0; l <= lmax; ++l) {
        const int n = 2 * l + 1, kl = kept(l, mmax);
        const float s = rescale ? inv_rescale(l, mmax) : 1.f;     // MODE 0 with rescale: rotate_inv's adjoint
        if (MODE == 0) {
            float v[GN_MAX];
#pragma unroll
            for (int j = 0; j < GN_MAX; ++j) v[j] = j < n ? x[(int64_t)(l * l + j) * xs] : 0.f;
            for (int i = 0; i < kl; ++i) {
                const float* di = d + doff + i * n;
                float a = 0.f;
#pragma unroll
                for (int j = 0; j < GN_MAX; ++j)
                    if (j < n) a += di[j] * v[j];
                const int j = order ? order[roff + i] : roff + i;
                const float y = s * a;
                o[(int64_t)j * C] = (GATHER && rad) ? y * rad[e * ld_rad + (int64_t)radrow[j] * C + c] : y;
            }
        } else {
            float v[GN_MAX];
#pragma unroll
            for (int i = 0; i < GN_MAX; ++i) v[i] = i < kl ? x[(int64_t)(order ? order[roff + i] : roff + i) * C] : 0.f;
            for (int j = 0; j < n; ++j) {
                float a = 0.f;
#pragma unroll
                for (int i = 0; i < GN_MAX; ++i)
                    if (i < kl) a += d[doff + i * n + j] * v[i];
                o[(int64_t)(l * l + j) * C] = s * a;
            }
        }
        doff += kl * n;
        roff += kl;
    }
}

// ---------------------------------------------------------------- RMS norm at any lmax / C
// one wave per node; lanes stride the channels.  bal(l) = float32(1/(2l+1)) / (lmax+1) in float32
// (the reference's default-dtype balance_degree_weight buffer, layer_norm.py:370-378)
__device__ __forceinline__ float bal_of(int l, int lmax) { return (1.0f / (float)(2 * l + 1)) / (float)(lmax + 1); }

__global__ __launch_bounds__(256) void eqv2_rmsnorm_general_kernel(int64_t V, int lmax, int C,
                                                                  const float* __restrict__ X,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ b, float eps,
                                                                  float* __restrict__ Y, float* __restrict__ save) {
    const int lane = threadIdx.x & 63;
    const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= V) return;
    const int K = (lmax + 1) * (lmax + 1);
    const float* x = X + v * K * C;
    float m0 = 0.f;
    for (int c = lane; c < C; c += 64) m0 += x[c];
    m0 = wave_sum(m0) / (float)C;
    float q = 0.f;
    for (int l = 0; l <= lmax; ++l) {
        const float bl = bal_of(l, lmax);
        for (int j = 0; j < 2 * l + 1; ++j) {
            const int i = l * l + j;
            for (int c = lane; c < C; c += 64) {
                const float xc = x[(int64_t)i * C + c] - (i == 0 ? m0 : 0.f);
                q += bl * xc * xc;
            }
        }
    }
    const float s = 1.0f / sqrtf(wave_sum(q) / (float)C + eps);
    float* y = Y + v * K * C;
    for (int l = 0; l <= lmax; ++l)
        for (int j = 0; j < 2 * l + 1; ++j) {
            const int i = l * l + j;
            for (int c = lane; c < C; c += 64)
                y[(int64_t)i * C + c] = (x[(int64_t)i * C + c] - (i == 0 ? m0 : 0.f)) * s * w[l * C + c] +
                                        (i == 0 ? b[c] : 0.f);
        }
    if (lane == 0) {
        save[v] = m0;
        save[V + v] = s;
    }
}

// dX, and G [V][(lmax+2) C] = (sum over degree l's coefficients of dY xc s, l = 0..lmax | dY[0]):
// the column sums of G are dweight [lmax+1][C] | dbias [C]
__global__ __launch_bounds__(256) void eqv2_rmsnorm_general_bwd_kernel(int64_t V, int lmax, int C,
                                                                      const float* __restrict__ X,
                                                                      const float* __restrict__ w,
                                                                      const float* __restrict__ save,
                                                                      const float* __restrict__ dY,
                                                                      float* __restrict__ dX, float* __restrict__ G) {
    const int lane = threadIdx.x & 63;
    const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (v >= V) return;
    const int K = (lmax + 1) * (lmax + 1);
    const float m0 = save[v], s = save[V + v];
    const float* x = X + v * K * C;
    const float* dy = dY + v * K * C;
    float* gr = G + v * (int64_t)(lmax + 2) * C;
    float dot = 0.f;
    for (int c = lane; c < C; c += 64) {
        for (int l = 0; l <= lmax; ++l) {
            float gw = 0.f;
            const float wl = w[l * C + c];
            for (int j = 0; j < 2 * l + 1; ++j) {
                const int i = l * l + j;
                const float xc = x[(int64_t)i * C + c] - (i == 0 ? m0 : 0.f);
                const float d = dy[(int64_t)i * C + c];
                gw += d * xc * s;
                dot += d * wl * xc;
            }
            gr[l * C + c] = gw;
        }
        gr[(lmax + 1) * C + c] = dy[c];
    }
    const float coef = s * s * s / (float)C * wave_sum(dot);
    // d xc[i][c] = s g[i][c] - coef bal(i) xc[i][c]; the l = 0 row then minus its channel mean
    const float b0 = bal_of(0, lmax);
    float dm = 0.f;
    for (int c = lane; c < C; c += 64) dm += s * dy[c] * w[c] - coef * b0 * (x[c] - m0);
    dm = wave_sum(dm) / (float)C;
    float* dx = dX + v * K * C;
    for (int l = 0; l <= lmax; ++l) {
        const float bl = bal_of(l, lmax);
        for (int j = 0; j < 2 * l + 1; ++j) {
            const int i = l * l + j;
            for (int c = lane; c < C; c += 64) {
                const float xc = x[(int64_t)i * C + c] - (i == 0 ? m0 : 0.f);
                dx[(int64_t)i * C + c] = s * dy[(int64_t)i * C + c] * w[l * C + c] - coef * bl * xc - (i == 0 ? dm : 0.f);
            }
        }
    }
}

int dsel_floats(int lmax, int mmax) {
    int s = 0;
    for (int l = 0; l <= lmax; ++l) s += (2 * std::min(l, mmax) + 1) * (2 * l + 1);
    return s;
}

int kept_rows(int lmax, int mmax) {
    int s = 0;
    for (int l = 0; l <= lmax; ++l) s += 2 * std::min(l, mmax) + 1;
    return s;
}

}  // namespace

// ======================================================================== C ABI (include/nbx.h)
extern "C" int nbx_eqv2_wigner_table_floats(int32_t lmax, int64_t* floats) {
    NBX_CHECK_ARG(floats && lmax >= 0 && lmax <= GL_MAX, "nbx_eqv2_wigner_table_floats: need 0 <= lmax <= %d", GL_MAX);
    int64_t n = 0;
    for (int l = 2; l <= lmax; ++l) n += (int64_t)(l + 1) * (2 * l + 1) * (2 * l + 4);
    *floats = n;
    return NBX_OK;
}

extern "C" int nbx_eqv2_dsel_floats(int32_t lmax, int32_t mmax, int64_t* floats) {
    NBX_CHECK_ARG(floats && mmax >= 0 && mmax <= lmax && lmax <= GL_MAX,
                  "nbx_eqv2_dsel_floats: need 0 <= mmax <= lmax <= %d", GL_MAX);
    *floats = dsel_floats(lmax, mmax);
    return NBX_OK;
}

extern "C" int nbx_eqv2_wigner(int64_t E, int32_t lmax, int32_t mmax, const float* rot, int64_t ld_rot,
                               const float* table, float* dsel, void* stream) {
    NBX_CHECK_ARG(E >= 0 && mmax >= 0 && mmax <= lmax && lmax <= GL_MAX && ld_rot >= 9,
                  "nbx_eqv2_wigner: need 0 <= mmax <= lmax <= %d, ld_rot >= 9", GL_MAX);
    NBX_CHECK_ARG(E == 0 || (rot && dsel && (lmax < 2 || table)), "nbx_eqv2_wigner: null operand");
    if (E == 0) return NBX_OK;
    const int rows = kept_rows(lmax, mmax);
    hipLaunchKernelGGL(eqv2_wigner_kernel, dim3(nblk(E * rows)), dim3(256), 0, (hipStream_t)stream, E, lmax, mmax,
                       rows, dsel_floats(lmax, mmax), rot, ld_rot, table, dsel);
    NBX_LAUNCH_CHECK("eqv2_wigner");
    return NBX_OK;
}

extern "C" int nbx_eqv2_rotate_general(int64_t E, int32_t C, int32_t lmax, int32_t mmax, const float* dsel,
                                       const float* in, int64_t ld_in, float* out, int32_t inverse, int32_t rescale,
                                       const int32_t* order, void* stream) {
    NBX_CHECK_ARG(E >= 0 && C >= 1 && mmax >= 0 && mmax <= lmax && lmax <= GL_MAX,
                  "nbx_eqv2_rotate_general: need C >= 1, 0 <= mmax <= lmax <= %d", GL_MAX);
    const int R = kept_rows(lmax, mmax), K = (lmax + 1) * (lmax + 1);
    NBX_CHECK_ARG(ld_in >= (int64_t)(inverse ? R : K) * C, "nbx_eqv2_rotate_general: ld_in too small");
    if (E == 0) return NBX_OK;
    NBX_CHECK_ARG(dsel && in && out, "nbx_eqv2_rotate_general: null operand");
    hipStream_t st = (hipStream_t)stream;
    const int S = dsel_floats(lmax, mmax);
    NBX_CHECK_ARG(E * C < ((int64_t)1 << 31), "nbx_eqv2_rotate_general: E C >= 2^31");
    const bool uni = C % 64 == 0;
    const size_t lds = (size_t)(256 / C) * S * sizeof(float);
    const bool ldsd = !uni && 256 % C == 0 && lds <= 64 * 1024;
    auto go = [&](auto kern, size_t shm) {
        hipLaunchKernelGGL(kern, dim3(nblk(E * C)), dim3(256), shm, st, E, C, lmax, mmax, S, R, dsel, in, ld_in, out,
                           rescale, order, (const int*)nullptr, (const int*)nullptr, (const float*)nullptr, (int64_t)0,
                           (const int*)nullptr);
    };
    if (inverse) {
        if (uni) go(eqv2_rotate_general_kernel<1, true>, 0);
        else if (ldsd) go(eqv2_rotate_general_kernel<1, false, false, true>, lds);
        else go(eqv2_rotate_general_kernel<1, false>, 0);
    } else {
        if (uni) go(eqv2_rotate_general_kernel<0, true>, 0);
        else if (ldsd) go(eqv2_rotate_general_kernel<0, false, false, true>, lds);
        else go(eqv2_rotate_general_kernel<0, false>, 0);
    }
    NBX_LAUNCH_CHECK("eqv2_rotate_general");
    return NBX_OK;
}

extern "C" int nbx_eqv2_rotate_gather(int64_t E, int32_t C, int32_t lmax, int32_t mmax, const float* dsel,
                                      const float* X, int64_t ld_x, const int32_t* src, const int32_t* dst, float* out,
                                      int32_t rescale, const int32_t* order, const float* rad, int64_t ld_rad,
                                      const int32_t* radrow, void* stream) {
    NBX_CHECK_ARG(E >= 0 && C >= 1 && mmax >= 0 && mmax <= lmax && lmax <= GL_MAX,
                  "nbx_eqv2_rotate_gather: need C >= 1, 0 <= mmax <= lmax <= %d", GL_MAX);
    const int R = kept_rows(lmax, mmax), K = (lmax + 1) * (lmax + 1);
    NBX_CHECK_ARG(ld_x >= (int64_t)K * C, "nbx_eqv2_rotate_gather: ld_x too small");
    if (E == 0) return NBX_OK;
    NBX_CHECK_ARG(dsel && X && src && dst && out, "nbx_eqv2_rotate_gather: null operand");
    NBX_CHECK_ARG(!rad || (radrow && ld_rad >= 2 * C), "nbx_eqv2_rotate_gather: rad needs radrow and ld_rad >= 2 C");
    NBX_CHECK_ARG(2 * E * C < ((int64_t)1 << 31), "nbx_eqv2_rotate_gather: 2 E C >= 2^31");
    hipStream_t st = (hipStream_t)stream;
    const int S = dsel_floats(lmax, mmax), C2 = 2 * C;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(nblk(E * C2)), dim3(256), 0, st, E, C2, lmax, mmax, S, R, dsel, X, ld_x, out,
                           rescale, order, src, dst, rad, ld_rad, radrow);
    };
    if (C % 64 == 0) go(eqv2_rotate_general_kernel<0, true, true>);
    else go(eqv2_rotate_general_kernel<0, false, true>);
    NBX_LAUNCH_CHECK("eqv2_rotate_gather");
    return NBX_OK;
}

extern "C" int nbx_eqv2_rms_norm_general(int64_t V, int32_t lmax, int32_t C, const float* X, const float* weight,
                                         const float* bias, float eps, float* Y, float* save, void* stream) {
    NBX_CHECK_ARG(V >= 0 && C >= 1 && lmax >= 0 && lmax <= GL_MAX, "nbx_eqv2_rms_norm_general: need C >= 1, lmax <= %d",
                  GL_MAX);
    if (V == 0) return NBX_OK;
    NBX_CHECK_ARG(X && weight && bias && Y && save, "nbx_eqv2_rms_norm_general: null operand");
    hipLaunchKernelGGL(eqv2_rmsnorm_general_kernel, dim3(nblk(V, 4)), dim3(256), 0, (hipStream_t)stream, V, lmax, C, X,
                       weight, bias, eps, Y, save);
    NBX_LAUNCH_CHECK("eqv2_rms_norm_general");
    return NBX_OK;
}

extern "C" int nbx_eqv2_rms_norm_general_backward(int64_t V, int32_t lmax, int32_t C, const float* X,
                                                  const float* weight, const float* save, const float* dY, float* dX,
                                                  float* G, void* stream) {
    NBX_CHECK_ARG(V >= 0 && C >= 1 && lmax >= 0 && lmax <= GL_MAX,
                  "nbx_eqv2_rms_norm_general_backward: need C >= 1, lmax <= %d", GL_MAX);
    if (V == 0) return NBX_OK;
    NBX_CHECK_ARG(X && weight && save && dY && dX && G, "nbx_eqv2_rms_norm_general_backward: null operand");
    hipLaunchKernelGGL(eqv2_rmsnorm_general_bwd_kernel, dim3(nblk(V, 4)), dim3(256), 0, (hipStream_t)stream, V, lmax, C,
                       X, weight, save, dY, dX, G);
    NBX_LAUNCH_CHECK("eqv2_rms_norm_general_backward");
    return NBX_OK;
}
