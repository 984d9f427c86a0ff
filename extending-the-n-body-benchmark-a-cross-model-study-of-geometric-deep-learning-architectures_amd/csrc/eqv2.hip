// EquiformerV2 N-body forward + device-resident self-feed rollout (fp32; GEMMs on the fp16x2
// split-precision MFMA path of lin.h, the bf16x3 images with NBX_EQ_SPLIT=x3).
//
// Reference (models/equiformer_v2/architecture/): equiformer_v2_nbody.py:428-575 (forward),
// edge_rot_mat.py:6-63, so3.py:30-185 / 485-531 / 695-745, so2_ops.py:13-238,
// transformer_block.py:22-728, input_block.py:83-138, layer_norm.py:327-441, activation.py:62-202.
// Oracle: oracle/equiformer_v2.py (pinned to the reference by tests/golden/eqv2.npz).
//
// Data layout in HBM (V = B N nodes, E = V (N-1) edges in the fully-connected order of
// build_graph_with_knn, src = edge_index[0], dst = edge_index[1]):
//   X, XN  [V][9][C]        node irreps (l-major coefficients, channels contiguous), XN = normed
//   rot    [E][32]          R (edge frame, rows) | D^2 rows m = -1, 0, +1 | |pos_src - pos_dst|
//   H2     [E][He]          second radial hidden layer
//   A0/A1  [E][3 2C] / [2E][2 2C]   rad * rotated message, m = 0 / (m = +1 row, m = -1 row)
//   Y0/Y1  [E][ld0] / [2E][4H]      so2_conv_1 outputs (alpha | gating | m0 coefficients; x_r | x_i)
//   Z0/Z1  [E][3H] / [2E][2H]       separable-S2-activated message (so2_conv_2 input, m-primary)
//   L      [E][nh]                  attention logits
//   V0/V1  [E][ldv0] / [2E][ldv1]   so2_conv_2 outputs (values)
// Per attention: radial MLP (one fp16x2 launch, eqv2_radial_h2_kernel) -> radial GEMM with the
// message-building epilogue (LIN_EQMSG)
// -> two SO(2) GEMMs -> S2 activation + alpha kernel -> two GEMMs -> per-system node kernel
// (segment softmax over the N-1 incoming edges, inverse rotation, sum, projection, residual, norm,
// the whole FFN and the next norm), so node features make one HBM round trip per block.
#include <cstdlib>
#include <cstring>

#include "lin.h"
#include "nbx_internal.h"
#include "rollout_state.h"

namespace {

constexpr int ROT = 32;                              // floats per edge record
constexpr float kAvgDegree = 23.395238876342773f;    // equiformer_v2_nbody.py:36
constexpr float kRescale2 = 1.2909944487358056f;     // sqrt(5 / 3): get_rotate_inv_rescale, l = 2 > mmax = 1
constexpr int GA = 18, GF = 42;                      // SO3_Grid(2,1): 6 x 3 points; SO3_Grid(2,2): 6 x 7

// x * sigmoid(x) with the hardware reciprocal (1 ulp) instead of an IEEE division sequence
__device__ inline float silu(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

__device__ inline float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ inline int lidx(int i) { return i == 0 ? 0 : (i < 4 ? 1 : 2); }

// counter-based uniform [0, 1) (splitmix64 finaliser), the device stand-in for torch.rand_like
__device__ inline float hash_uniform(uint64_t seed, uint64_t ctr) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (ctr + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)(z >> 40) * (1.0f / 16777216.0f);
}

__device__ inline void edge_nodes(int64_t e, int N, int64_t& src, int64_t& dst) {
    const int64_t per = (int64_t)N * (N - 1);
    const int64_t b = e / per, rr = e - b * per, i = rr / (N - 1), jj = rr - i * (N - 1);
    src = b * N + i;
    dst = b * N + (jj < i ? jj : jj + 1);
}

// ---- edge frame: init_edge_rot_mat (edge_rot_mat.py:6-63) and the Wigner blocks the rotations use
// (SO3_Rotation, so3.py:485-531).  D^1 = R; D^2_ij = 2/3 tr((R^T Q_i R) Q_j) over e3nn's symmetric
// traceless basis Q (oracle/e3nn_so3.py documents the basis; the reference goes through Euler angles
// and Jd.pt, which is the same matrix).
__global__ void eqv2_edge_kernel(const float* __restrict__ pos, const float* __restrict__ mass,
                                 const float* __restrict__ gauge, uint64_t seed, uint64_t frame, int64_t V, int N,
                                 int num_elements, float* __restrict__ rot, int* __restrict__ zn) {
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t E = V * (N - 1);
    if (e < V) {
        int z = (int)mass[e];                         // atomic_numbers = charges.int() (tuple branch)
        zn[e] = z < 0 ? 0 : (z >= num_elements ? num_elements - 1 : z);
    }
    if (e >= E) return;
    int64_t s, d;
    edge_nodes(e, N, s, d);
    const float vx = pos[3 * s] - pos[3 * d], vy = pos[3 * s + 1] - pos[3 * d + 1], vz = pos[3 * s + 2] - pos[3 * d + 2];
    const float dist = sqrtf(vx * vx + vy * vy + vz * vz);
    const float nx[3] = {vx / dist, vy / dist, vz / dist};
    float g[3];
    for (int k = 0; k < 3; ++k)
        g[k] = gauge ? gauge[3 * e + k] : hash_uniform(seed, ((uint64_t)frame * (uint64_t)E + (uint64_t)e) * 3 + k);
    float v2[3] = {g[0] - 0.5f, g[1] - 0.5f, g[2] - 0.5f};
    float n2 = sqrtf(v2[0] * v2[0] + v2[1] * v2[1] + v2[2] * v2[2]);
    for (int k = 0; k < 3; ++k) v2[k] /= n2;
    auto adot = [&](const float* a) { return fabsf(a[0] * nx[0] + a[1] * nx[1] + a[2] * nx[2]); };
    // both 90-degree alternatives are rotations of the ORIGINAL draw (edge_rot_mat.py:27-43)
    const float vb[3] = {-v2[1], v2[0], v2[2]};
    const float vc[3] = {v2[0], -v2[2], v2[1]};
    if (adot(v2) > adot(vb)) { v2[0] = vb[0]; v2[1] = vb[1]; v2[2] = vb[2]; }
    if (adot(v2) > adot(vc)) { v2[0] = vc[0]; v2[1] = vc[1]; v2[2] = vc[2]; }
    float nz[3] = {nx[1] * v2[2] - nx[2] * v2[1], nx[2] * v2[0] - nx[0] * v2[2], nx[0] * v2[1] - nx[1] * v2[0]};
    for (int pass = 0; pass < 2; ++pass) {
        const float nn = sqrtf(nz[0] * nz[0] + nz[1] * nz[1] + nz[2] * nz[2]);
        for (int k = 0; k < 3; ++k) nz[k] /= nn;
    }
    float ny[3] = {nx[1] * nz[2] - nx[2] * nz[1], nx[2] * nz[0] - nx[0] * nz[2], nx[0] * nz[1] - nx[1] * nz[0]};
    const float nyn = sqrtf(ny[0] * ny[0] + ny[1] * ny[1] + ny[2] * ny[2]);
    float R[3][3];
    for (int k = 0; k < 3; ++k) {
        R[0][k] = nz[k];
        R[1][k] = nx[k];
        R[2][k] = -ny[k] / nyn;
    }
    float* out = rot + e * ROT;
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) out[3 * a + b] = R[a][b];
    const float s3h = 0.8660254037844386f;   // sqrt3 / 2
    for (int row = 1; row <= 3; ++row) {     // D^2 rows m = -1 (xy), 0, +1 (yz)
        float M[3][3];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                if (row == 1) M[a][b] = s3h * (R[0][a] * R[1][b] + R[1][a] * R[0][b]);
                else if (row == 2) M[a][b] = -0.5f * R[0][a] * R[0][b] + R[1][a] * R[1][b] - 0.5f * R[2][a] * R[2][b];
                else M[a][b] = s3h * (R[1][a] * R[2][b] + R[2][a] * R[1][b]);
            }
        const float t = 2.0f / 3.0f, s3 = 1.7320508075688772f;
        float* o = out + 9 + 5 * (row - 1);
        o[0] = t * s3 * M[0][2];
        o[1] = t * s3 * M[0][1];
        o[2] = t * (-0.5f * M[0][0] + M[1][1] - 0.5f * M[2][2]);
        o[3] = t * s3 * M[1][2];
        o[4] = t * 0.5f * s3 * (M[2][2] - M[0][0]);
    }
    out[24] = dist;
}

// ---- RadialFunction first hidden layer (radial_function.py:5-32), first Linear folded:
// H1 = SiLU(LN(d a + c + us[z_src] + ut[z_dst])).  One wave per edge, lane = channel.  The second
// hidden layer (Linear + LN + SiLU) is a GEMM with the LIN_LNSILU epilogue (lin.h).
template <int HE>
__global__ __launch_bounds__(256) void eqv2_radial_kernel(const float* __restrict__ rot, const int* __restrict__ zn,
                                                         const nbx_eqv2_radial W, int64_t E, int N,
                                                         float* __restrict__ H1) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool on = lane < HE;
    const int c = on ? lane : 0;
    const float a = W.a[c], cc = W.c[c], g1 = W.ln1_w[c], bb1 = W.ln1_b[c];
    const float inv = 1.0f / HE;
    for (int64_t e = blockIdx.x * 4 + wave; e < E; e += (int64_t)gridDim.x * 4) {
        int64_t s, t;
        edge_nodes(e, N, s, t);
        const float d = rot[e * ROT + 24];
        const float v = on ? d * a + cc + W.us[zn[s] * HE + c] + W.ut[zn[t] * HE + c] : 0.f;
        const float mu = wave_sum(v) * inv;
        const float dv = on ? v - mu : 0.f;
        const float var = wave_sum(dv * dv) * inv;
        if (on) H1[e * HE + c] = silu(dv / sqrtf(var + 1e-5f) * g1 + bb1);
    }
}

// ---- both RadialFunction hidden layers in one launch on the fp16x2 path (net.3 image W.w1_h2): a wave
// owns a 32-edge tile.  Lane (r, h) forms the first layer of edge r at k = 32 c + 16 h + [0, 16) (chunk
// c) in registers -- the A-fragment layout of v_mfma_f32_32x32x16_f16 (lin.h lin_kernel: lane (r, h)
// holds k = 16 h + 4 q + e of a 32-deep chunk) -- with the row's LayerNorm statistics from the lane's
// values plus one shuffle with its partner half; then net.3 on the fp16x2 image in LDS and the
// LIN_LNSILU epilogue (bias, LayerNorm over the He columns, SiLU).  H1 never leaves registers.
constexpr int RAD_WAVES = 4;
template <int HE>
__global__ __launch_bounds__(64 * RAD_WAVES, 2) void eqv2_radial_h2_kernel(const float* __restrict__ rot,
                                                                       const int* __restrict__ zn,
                                                                       const nbx_eqv2_radial W, int64_t E, int N,
                                                                       float* __restrict__ H2, int* range_flag) {
    constexpr int NC = HE / 32;                  // K chunks = output column tiles
    constexpr int BLK = nbx::LIN_H2_BLK;
    using SP = nbx::SplitP<2>;
    using SPT = SP::T;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* cst = lds + NC * NC * BLK;            // a | c | ln1_w | ln1_b, HE floats each
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, r = lane & 31, h = lane >> 5;
    nbx::tp_dma_image<RAD_WAVES>(static_cast<const float*>(W.w1_h2), lds, NC * NC * BLK);
    for (int i = t; i < 4 * HE; i += 64 * RAD_WAVES) {
        const int q = i / HE, k = i - q * HE;
        cst[i] = (q == 0 ? W.a : q == 1 ? W.c : q == 2 ? W.ln1_w : W.ln1_b)[k];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float bb[NC], gw[NC], gb[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        bb[j] = W.b1[32 * j + r];
        gw[j] = W.ln2_w[32 * j + r];
        gb[j] = W.ln2_b[32 * j + r];
    }
    const float inv = 1.0f / HE;
    const SPT* ldsx = reinterpret_cast<const SPT*>(lds);
    const __amdgpu_buffer_rsrc_t rsH2 = __builtin_amdgcn_make_buffer_rsrc((void*)H2, (short)0, 0x7FFFFFF0, 0x00020000);
    const int64_t tiles = (E + 31) >> 5;
    float zguard = 0.f;
    for (int64_t tile = (int64_t)blockIdx.x * RAD_WAVES + wave; tile < tiles; tile += (int64_t)gridDim.x * RAD_WAVES) {
        const int64_t e = tile * 32 + r;
        const int64_t ee = e < E ? e : E - 1;
        int64_t s, tt;
        edge_nodes(ee, N, s, tt);
        const float d = rot[ee * ROT + 24];
        const float* us = W.us + (size_t)zn[s] * HE + 16 * h;
        const float* ut = W.ut + (size_t)zn[tt] * HE + 16 * h;
        // first layer: v = d a + c + us[z_src] + ut[z_dst] (eqv2_radial_kernel's order)
        float v[NC][16];
        float sum = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 u = *reinterpret_cast<const float4*>(us + 32 * c + 4 * q);
                const float4 w = *reinterpret_cast<const float4*>(ut + 32 * c + 4 * q);
                const float4 a = *reinterpret_cast<const float4*>(cst + 32 * c + 16 * h + 4 * q);
                const float4 cc = *reinterpret_cast<const float4*>(cst + HE + 32 * c + 16 * h + 4 * q);
                v[c][4 * q + 0] = d * a.x + cc.x + u.x + w.x;
                v[c][4 * q + 1] = d * a.y + cc.y + u.y + w.y;
                v[c][4 * q + 2] = d * a.z + cc.z + u.z + w.z;
                v[c][4 * q + 3] = d * a.w + cc.w + u.w + w.w;
#pragma unroll
                for (int i = 0; i < 4; ++i) sum += v[c][4 * q + i];
                if (q == 3) __builtin_amdgcn_sched_barrier(0);   // one chunk's loads live at a time (VGPR budget)
            }
        sum += __shfl_xor(sum, 32);
        const float mu = sum * inv;
        float sq = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                v[c][i] -= mu;
                sq += v[c][i] * v[c][i];
            }
        sq += __shfl_xor(sq, 32);
        const float rsd = 1.0f / sqrtf(sq * inv + 1e-5f);
        nbx::floatx16 acc[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            float hv[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 g = *reinterpret_cast<const float4*>(cst + 2 * HE + 32 * c + 16 * h + 4 * q);
                const float4 b = *reinterpret_cast<const float4*>(cst + 3 * HE + 32 * c + 16 * h + 4 * q);
                hv[4 * q + 0] = silu(v[c][4 * q + 0] * rsd * g.x + b.x);
                hv[4 * q + 1] = silu(v[c][4 * q + 1] * rsd * g.y + b.y);
                hv[4 * q + 2] = silu(v[c][4 * q + 2] * rsd * g.z + b.z);
                hv[4 * q + 3] = silu(v[c][4 * q + 3] * rsd * g.w + b.w);
            }
#pragma unroll
            for (int m = 0; m < 2; ++m) {   // MFMA m takes k = 16 h + 8 m + [0, 8)
                SPT a[SP::NP];
                SP::split(make_float4(hv[8 * m], hv[8 * m + 1], hv[8 * m + 2], hv[8 * m + 3]),
                          make_float4(hv[8 * m + 4], hv[8 * m + 5], hv[8 * m + 6], hv[8 * m + 7]), a);
#pragma unroll
                for (int j = 0; j < NC; ++j) {
                    const SPT* bp = ldsx + (j * NC + c) * (BLK / 4) + lane;
                    SPT b[SP::NP];
#pragma unroll
                    for (int p3 = 0; p3 < SP::NP; ++p3) b[p3] = bp[(2 * p3 + m) * 64];
#pragma unroll
                    for (int tt3 = 0; tt3 < SP::NT; ++tt3) acc[j] = nbx::mfma32x32(a[SP::TA[tt3]], b[SP::TB[tt3]], acc[j]);
                }
            }
        }
        // epilogue (lin.h LIN_LNSILU): undo the weight scale, guard, bias, LayerNorm over HE, SiLU
#pragma unroll
        for (int j = 0; j < NC; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                acc[j][i] *= W.w1_sinv;
                zguard = nbx::tp_nonfinite_fold(zguard, acc[j][i]);
            }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int64_t row = tile * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
            float y[NC], sm = 0.f;
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                y[j] = acc[j][i] + bb[j];
                sm += y[j];
            }
            for (int o = 16; o > 0; o >>= 1) sm += __shfl_xor(sm, o);   // the 32 lanes of this row
            const float m2 = sm * inv;
            float q2 = 0.f;
#pragma unroll
            for (int j = 0; j < NC; ++j) q2 += (y[j] - m2) * (y[j] - m2);
            for (int o = 16; o > 0; o >>= 1) q2 += __shfl_xor(q2, o);
            const float rs = 1.0f / sqrtf(q2 * inv + 1e-5f);
#pragma unroll
            for (int j = 0; j < NC; ++j) {   // 32-bit offsets (E HE < 2^29, eqv2_prepare), rows past E dropped
                const float z = (y[j] - m2) * rs * gw[j] + gb[j];
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, z * __builtin_amdgcn_rcpf(1.0f + __expf(-z))), rsH2,
                                                      row < E ? (uint32_t)((row * HE + 32 * j + r) * 4) : 0x7FFFFFF0u,
                                                      0, 0);
            }
        }
    }
    nbx::tp_range_flag(range_flag, zguard);
}

// softmax over a node's deg incoming edges for head `lane` (segment softmax + 1e-16, PyG): alpha[q] ->
// sal[q * 8 + lane].  Up to 32 edges the logits are loaded in one predicated batch into registers (the
// loop form waited one memory latency per edge, twice); the arithmetic and its order are unchanged.
template <class EdgeOf>
__device__ __forceinline__ void edge_softmax(const float* __restrict__ L, int nh, int lane, int deg, EdgeOf edge_of,
                                             float* sal) {
    if (deg <= 32) {
        float lv[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) lv[q] = q < deg ? L[edge_of(q) * nh + lane] : -INFINITY;
        float mx = -INFINITY;
#pragma unroll
        for (int q = 0; q < 32; ++q) mx = fmaxf(mx, lv[q]);
        float sum = 0.f;
#pragma unroll
        for (int q = 0; q < 32; ++q)
            if (q < deg) {
                lv[q] = __expf(lv[q] - mx);
                sum += lv[q];
            }
        const float inv = 1.0f / (sum + 1e-16f);
#pragma unroll
        for (int q = 0; q < 32; ++q)
            if (q < deg) sal[q * 8 + lane] = lv[q] * inv;
        return;
    }
    float mx = -INFINITY;
    for (int q = 0; q < deg; ++q) mx = fmaxf(mx, L[edge_of(q) * nh + lane]);
    float sum = 0.f;
    for (int q = 0; q < deg; ++q) {
        const float ex = __expf(L[edge_of(q) * nh + lane] - mx);
        sal[q * 8 + lane] = ex;
        sum += ex;
    }
    const float inv = 1.0f / (sum + 1e-16f);
    for (int q = 0; q < deg; ++q) sal[q * 8 + lane] *= inv;
}

// ---- separable S2 activation of the so2_conv_1 output + attention logits
// (transformer_block.py:287-339; activation.py:155-202; so2_ops.py:61-75 complex combine):
// one wave per edge, lane = hidden channel.
struct S2Args {
    const float* Y0; int ld0;     // [E][ld0]: alpha (nh na) | gating (H) | m0 coefficients (3H)
    const float* Y1;              // [2E][4H]: x_r (2H) | x_i (2H) per row (m = +1 input row, m = -1 input row)
    const float* gto; const float* gfrom;   // [18][7]
    const float* an_w; const float* an_b; const float* adot;
    int nh, na, H;
    int64_t E;
    float* Z0; float* Z1; float* L;
};

// NA: attn_alpha_channels as a compile-time count (8 at C4, 16), so the head's alpha row and LayerNorm
// parameters are loaded in one batch; 0 = run-time count (a serial load per element: the lanes h < nh
// of every wave waited ~3 NA memory latencies, which bounded the kernel)
template <int NA>
__global__ __launch_bounds__(256) void eqv2_s2act_kernel(const S2Args A) {
    // one thread per (edge, hidden channel); the grid matrices are read with uniform addresses
    // (scalar loads, SGPR operands): no LDS traffic in the 18-point loop
    const float* __restrict__ gt = A.gto;
    const float* __restrict__ gf = A.gfrom;
    const int H = A.H, ex = A.nh * A.na;
    const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t e = gid / H;
    const int h = (int)(gid - e * H);
    if (e >= A.E) return;
    const float* y0 = A.Y0 + e * A.ld0;
    const float* yr = A.Y1 + 2 * e * 4 * H;
    const float* yi = yr + 4 * H;
    float v[7];
    v[0] = y0[ex + H + h];
    v[2] = y0[ex + 2 * H + h];
    v[5] = y0[ex + 3 * H + h];
    v[3] = yr[h] - yi[2 * H + h];            // m = +1, l = 1
    v[6] = yr[H + h] - yi[3 * H + h];        // m = +1, l = 2
    v[1] = yi[h] + yr[2 * H + h];            // m = -1, l = 1
    v[4] = yi[H + h] + yr[3 * H + h];        // m = -1, l = 2
    const float gate = y0[ex + h];
    float o[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < GA; ++p) {
        float gv = 0.f;
#pragma unroll
        for (int i = 0; i < 7; ++i) gv += gt[p * 7 + i] * v[i];
        const float sg = silu(gv);
#pragma unroll
        for (int i = 0; i < 7; ++i) o[i] += gf[p * 7 + i] * sg;
    }
    o[0] = silu(gate);
    float* z0 = A.Z0 + e * 3 * H + h;
    z0[0] = o[0];
    z0[H] = o[2];
    z0[2 * H] = o[5];
    float* z1 = A.Z1 + 2 * e * 2 * H + h;
    z1[0] = o[3];
    z1[H] = o[6];
    z1[2 * H] = o[1];
    z1[3 * H] = o[4];
    if (h < A.nh) {   // alpha_norm (LayerNorm), SmoothLeakyReLU(0.2), alpha_dot for head h
        const float* xa = y0 + h * A.na;
        if constexpr (NA > 0) {
            float xs[NA], w[NA], b[NA], d[NA];
#pragma unroll
            for (int k = 0; k < NA; ++k) {
                xs[k] = xa[k];
                w[k] = A.an_w[k];
                b[k] = A.an_b[k];
                d[k] = A.adot[h * NA + k];
            }
            float mu = 0.f;
#pragma unroll
            for (int k = 0; k < NA; ++k) mu += xs[k];
            mu /= NA;
            float var = 0.f;
#pragma unroll
            for (int k = 0; k < NA; ++k) var += (xs[k] - mu) * (xs[k] - mu);
            const float rs = 1.0f / sqrtf(var / NA + 1e-5f);
            float lg = 0.f;
#pragma unroll
            for (int k = 0; k < NA; ++k) {
                const float y = (xs[k] - mu) * rs * w[k] + b[k];
                const float sg = __builtin_amdgcn_rcpf(1.0f + __expf(-y));
                lg += (0.6f * y + 0.4f * y * (2.0f * sg - 1.0f)) * d[k];
            }
            A.L[e * A.nh + h] = lg;
        } else {
            float xs[16];
            float mu = 0.f;
            for (int k = 0; k < A.na; ++k) {
                xs[k] = xa[k];
                mu += xs[k];
            }
            mu /= A.na;
            float var = 0.f;
            for (int k = 0; k < A.na; ++k) var += (xs[k] - mu) * (xs[k] - mu);
            const float rs = 1.0f / sqrtf(var / A.na + 1e-5f);
            float lg = 0.f;
            for (int k = 0; k < A.na; ++k) {
                const float y = (xs[k] - mu) * rs * A.an_w[k] + A.an_b[k];
                const float sg = __builtin_amdgcn_rcpf(1.0f + __expf(-y));
                lg += (0.6f * y + 0.4f * y * (2.0f * sg - 1.0f)) * A.adot[h * A.na + k];
            }
            A.L[e * A.nh + h] = lg;
        }
    }
}

// ---- per-system node kernel: attention aggregation (segment softmax over edge_index[1],
// inverse rotation, sum, proj), residual, norm_2, FFN (gating + so3_linear_1 + S2 activation on
// SO3_Grid(2,2) + so3_linear_2), residual, next norm (transformer_block.py:669-728).  MODE 1 is the
// force block's output head, MODE 2 the input embedding + EdgeDegreeEmbedding (input_block.py:83-138,
// equiformer_v2_nbody.py:486-546).  One workgroup per system, one wave per node, lane = channel.
enum NodeMode : int { NODE_BLOCK = 0, NODE_FORCE = 1, NODE_INIT = 2 };

struct NodeArgs {
    const float* L; const float* V0; const float* V1; int ldv0, ldv1, nh, nv;
    const float* rot;
    const float* proj_t; const float* proj_b; int cout;
    float* X; float* XN;
    const float* norm2_w; const float* norm2_b;
    const float* gate_t; const float* gate_b;
    const float* lin1_t; const float* lin1_b;
    const float* lin2_t; const float* lin2_b;
    const float* gto; const float* gfrom;   // [42][9]
    const float* nnorm_w; const float* nnorm_b;
    const float* Red;                       // edge-degree radial output [E][3C]
    const float* semb; const float* vel; const float* vel_t; const float* vel_b; const int* zn;
    float* out;
    int C, F, N;
};

// EquivariantRMSNormArraySphericalHarmonicsV2 of x[9] (lane = channel c < C)
__device__ inline void rms_norm(const float (&x)[9], float (&y)[9], const float* w, const float* b, int c, bool on,
                                int C) {
    const float mean0 = wave_sum(on ? x[0] : 0.f) / C;
    const float f0 = x[0] - mean0;
    float s = f0 * f0 * (1.0f / 3.0f);
#pragma unroll
    for (int i = 1; i < 4; ++i) s += x[i] * x[i] * (1.0f / 9.0f);
#pragma unroll
    for (int i = 4; i < 9; ++i) s += x[i] * x[i] * (1.0f / 15.0f);
    const float nrm = wave_sum(on ? s : 0.f) / C;
    const float sc = 1.0f / sqrtf(nrm + 1e-5f);
    if (!on) return;
    y[0] = f0 * sc * w[c] + b[c];
#pragma unroll
    for (int i = 1; i < 9; ++i) y[i] = x[i] * sc * w[lidx(i) * C + c];
}

template <int MODE>
__global__ __launch_bounds__(64) void eqv2_node_kernel(const NodeArgs A) {
    // one single-wave workgroup per node (lane = channel): enough waves in flight to hide the
    // gathers; the per-node weight reads come from L2
    __shared__ float s_alpha[64 * 8];
    __shared__ float s_vec[9 * 64];
    __shared__ float s_vec2[9 * 64];
    __shared__ float s_gt[GF * 9], s_gf[GF * 9];
    const int lane = threadIdx.x;
    const int C = A.C, F = A.F, N = A.N, deg = N - 1;
    const int64_t node = blockIdx.x;
    const int64_t sys = node / N;
    const int t = (int)(node - sys * N);
    if (MODE == NODE_BLOCK) {
        for (int i = lane; i < GF * 9; i += 64) {
            s_gt[i] = A.gto[i];
            s_gf[i] = A.gfrom[i];
        }
    }
    __syncthreads();
    const int c = lane < C ? lane : 0;
    const bool on = lane < C;
    const bool active = true;
    {
        auto edge_of = [&](int q) -> int64_t {   // q-th incoming edge of node t (source q' != t)
            const int s = q < t ? q : q + 1;
            return sys * N * deg + (int64_t)s * deg + (t < s ? t : t - 1);
        };
        float x[9];
        if (MODE == NODE_INIT) {
            // EdgeDegreeEmbedding: m = 0 coefficients rotated back and summed / AVG_DEGREE
            float ed[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (active && on) {
                for (int q = 0; q < deg; ++q) {
                    const int64_t e = edge_of(q);
                    const float* rr = A.Red + e * 3 * C + c;
                    const float* D = A.rot + e * ROT;
                    const float v0 = rr[0], v1 = rr[C], v2 = rr[2 * C];
                    ed[0] += v0;
#pragma unroll
                    for (int k = 0; k < 3; ++k) ed[1 + k] += D[3 + k] * v1;
#pragma unroll
                    for (int k = 0; k < 5; ++k) ed[4 + k] += kRescale2 * D[14 + k] * v2;
                }
            }
            const float* vv = A.vel + 3 * node;
#pragma unroll
            for (int i = 0; i < 9; ++i) x[i] = ed[i] / kAvgDegree;
            x[0] += A.semb[A.zn[node] * C + c];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int o = j * C + c;
                x[1 + j] += A.vel_b[o] + vv[0] * A.vel_t[o] + vv[1] * A.vel_t[3 * C + o] + vv[2] * A.vel_t[6 * C + o];
            }
        } else {
            // ---- attention: softmax over the N-1 incoming edges per head
            const int KV = A.nh * A.nv;
            float* sal = s_alpha;
            if (active && lane < A.nh) edge_softmax(A.L, A.nh, lane, deg, edge_of, sal);
            __syncthreads();
            // ---- values * alpha, rotated back (Wigner^T with the l = 2 rescale), summed over edges
            const int G = 64 / KV, k = lane % KV, qg = lane / KV, hd = k / A.nv;
            float agg[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (active) {
                for (int q = qg; q < deg; q += G) {
                    const int64_t e = edge_of(q);
                    const float a = sal[q * 8 + hd];
                    const float* v0 = A.V0 + e * A.ldv0 + k;
                    const float* vr = A.V1 + 2 * e * A.ldv1 + k;
                    const float* vi = vr + A.ldv1;
                    const float m0 = v0[0] * a, m1 = v0[KV] * a, m2 = v0[2 * KV] * a;
                    const float re1 = (vr[0] - vi[2 * KV]) * a, re2 = (vr[KV] - vi[3 * KV]) * a;
                    const float im1 = (vi[0] + vr[2 * KV]) * a, im2 = (vi[KV] + vr[3 * KV]) * a;
                    const float* D = A.rot + e * ROT;
                    agg[0] += m0;
#pragma unroll
                    for (int j = 0; j < 3; ++j) agg[1 + j] += D[j] * im1 + D[3 + j] * m1 + D[6 + j] * re1;
#pragma unroll
                    for (int j = 0; j < 5; ++j)
                        agg[4 + j] += kRescale2 * (D[9 + j] * im2 + D[14 + j] * m2 + D[19 + j] * re2);
                }
            }
#pragma unroll
            for (int i = 0; i < 9; ++i)
                for (int o = KV; o < 64; o <<= 1) agg[i] += __shfl_xor(agg[i], o);
            float* sag = s_vec;
            if (lane < KV)
#pragma unroll
                for (int i = 0; i < 9; ++i) sag[i * KV + lane] = agg[i];
            __syncthreads();
            // ---- proj (SO3_LinearV2 nh nv -> cout)
            const int co = lane < A.cout ? lane : 0;
            float y[9];
#pragma unroll
            for (int i = 0; i < 9; ++i) y[i] = 0.f;
            for (int kk = 0; kk < KV; ++kk) {
                const float w0 = A.proj_t[kk * A.cout + co], w1 = A.proj_t[(KV + kk) * A.cout + co],
                            w2 = A.proj_t[(2 * KV + kk) * A.cout + co];
                y[0] += sag[kk] * w0;
#pragma unroll
                for (int i = 1; i < 4; ++i) y[i] += sag[i * KV + kk] * w1;
#pragma unroll
                for (int i = 4; i < 9; ++i) y[i] += sag[i * KV + kk] * w2;
            }
            y[0] += A.proj_b[co];
            if (MODE == NODE_FORCE) {
                // pred = proj output: channel 0 l = 1 -> delta pos, channel 1 l = 1 -> vel
                if (lane < 2)
                    for (int j = 0; j < 3; ++j) A.out[node * 6 + 3 * lane + j] = y[1 + j];
                return;
            }
            const float* xo = A.X + node * 9 * C + c;
#pragma unroll
            for (int i = 0; i < 9; ++i) x[i] = xo[i * C] + y[i];
            // ---- norm_2 + FFN
            float xn[9];
            rms_norm(x, xn, A.norm2_w, A.norm2_b, c, on, C);
            float* sx = s_vec;
            __syncthreads();
            if (on)
#pragma unroll
                for (int i = 0; i < 9; ++i) sx[i * C + c] = xn[i];
            __syncthreads();
            const bool fon = lane < F;
            const int f = fon ? lane : 0;
            float gate = A.gate_b[f];
            float h[9];
            h[0] = A.lin1_b[f];
#pragma unroll
            for (int i = 1; i < 9; ++i) h[i] = 0.f;
            for (int cc = 0; cc < C; ++cc) {
                const float w0 = A.lin1_t[cc * F + f], w1 = A.lin1_t[(C + cc) * F + f],
                            w2 = A.lin1_t[(2 * C + cc) * F + f];
                gate += sx[cc] * A.gate_t[cc * F + f];
                h[0] += sx[cc] * w0;
#pragma unroll
                for (int i = 1; i < 4; ++i) h[i] += sx[i * C + cc] * w1;
#pragma unroll
                for (int i = 4; i < 9; ++i) h[i] += sx[i * C + cc] * w2;
            }
            float o[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            for (int p = 0; p < GF; ++p) {
                float gv = 0.f;
#pragma unroll
                for (int i = 0; i < 9; ++i) gv += s_gt[p * 9 + i] * h[i];
                const float sg = silu(gv);
#pragma unroll
                for (int i = 0; i < 9; ++i) o[i] += s_gf[p * 9 + i] * sg;
            }
            o[0] = silu(gate);
            float* sa = s_vec2;
            if (fon)
#pragma unroll
                for (int i = 0; i < 9; ++i) sa[i * F + f] = o[i];
            __syncthreads();
            float h2[9];
            h2[0] = A.lin2_b[c];
#pragma unroll
            for (int i = 1; i < 9; ++i) h2[i] = 0.f;
            for (int ff = 0; ff < F; ++ff) {
                const float w0 = A.lin2_t[ff * C + c], w1 = A.lin2_t[(F + ff) * C + c],
                            w2 = A.lin2_t[(2 * F + ff) * C + c];
                h2[0] += sa[ff] * w0;
#pragma unroll
                for (int i = 1; i < 4; ++i) h2[i] += sa[i * F + ff] * w1;
#pragma unroll
                for (int i = 4; i < 9; ++i) h2[i] += sa[i * F + ff] * w2;
            }
#pragma unroll
            for (int i = 0; i < 9; ++i) x[i] += h2[i];
        }
        float xn[9];
        rms_norm(x, xn, A.nnorm_w, A.nnorm_b, c, on, C);
        if (active && on) {
            float* xw = A.X + node * 9 * C + c;
            float* xnw = A.XN + node * 9 * C + c;
#pragma unroll
            for (int i = 0; i < 9; ++i) {
                xw[i * C] = x[i];
                xnw[i * C] = xn[i];
            }
        }
    }
}

// NODE_BLOCK on NPW nodes per wave (lane = channel): the attention aggregation runs node by
// node, then proj, the FFN's gate / so3_linear_1 and so3_linear_2 walk their weights once for
// all NPW nodes (each weight load feeds NPW nodes' FMAs, so the chains of dependent L2 weight
// reads that bound the one-node kernel are NPW times shorter).  Per node the arithmetic and its
// order are those of eqv2_node_kernel<NODE_BLOCK>.  Needs KV <= 16.
// NB_ROWS: weight rows per load batch (1: the default, 121 VGPRs; 4: 124 VGPRs; 8: 190 VGPRs)
template <int NPW, int NB_ROWS = 1>
__global__ __launch_bounds__(64) void eqv2_node_block_kernel(const NodeArgs A, int64_t V) {
    __shared__ float s_alpha[64 * 8];
    __shared__ float s_ag[NPW][9 * 16];
    __shared__ float s_x[NPW][9 * 64];
    __shared__ float s_gt[GF * 9], s_gf[GF * 9];
    const int lane = threadIdx.x;
    const int C = A.C, F = A.F, N = A.N, deg = N - 1, KV = A.nh * A.nv;
    const int64_t node0 = (int64_t)blockIdx.x * NPW;
    for (int i = lane; i < GF * 9; i += 64) {
        s_gt[i] = A.gto[i];
        s_gf[i] = A.gfrom[i];
    }
    const int c = lane < C ? lane : 0;
    const bool on = lane < C;
    // ---- attention aggregation, node by node (softmax over the N-1 incoming edges per head,
    // values * alpha rotated back and summed) -> s_ag[n]
#pragma unroll
    for (int n = 0; n < NPW; ++n) {
        const int64_t node = node0 + n;
        __syncthreads();   // s_alpha of the previous node is consumed
        if (node >= V) continue;
        const int64_t sys = node / N;
        const int t = (int)(node - sys * N);
        auto edge_of = [&](int q) -> int64_t {
            const int s = q < t ? q : q + 1;
            return sys * N * deg + (int64_t)s * deg + (t < s ? t : t - 1);
        };
        if (lane < A.nh) edge_softmax(A.L, A.nh, lane, deg, edge_of, s_alpha);
        __syncthreads();
        const int G = 64 / KV, k = lane % KV, qg = lane / KV, hd = k / A.nv;
        float agg[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int q = qg; q < deg; q += G) {
            const int64_t e = edge_of(q);
            const float a = s_alpha[q * 8 + hd];
            const float* v0 = A.V0 + e * A.ldv0 + k;
            const float* vr = A.V1 + 2 * e * A.ldv1 + k;
            const float* vi = vr + A.ldv1;
            const float m0 = v0[0] * a, m1 = v0[KV] * a, m2 = v0[2 * KV] * a;
            const float re1 = (vr[0] - vi[2 * KV]) * a, re2 = (vr[KV] - vi[3 * KV]) * a;
            const float im1 = (vi[0] + vr[2 * KV]) * a, im2 = (vi[KV] + vr[3 * KV]) * a;
            const float* D = A.rot + e * ROT;
            agg[0] += m0;
#pragma unroll
            for (int j = 0; j < 3; ++j) agg[1 + j] += D[j] * im1 + D[3 + j] * m1 + D[6 + j] * re1;
#pragma unroll
            for (int j = 0; j < 5; ++j) agg[4 + j] += kRescale2 * (D[9 + j] * im2 + D[14 + j] * m2 + D[19 + j] * re2);
        }
#pragma unroll
        for (int i = 0; i < 9; ++i)
            for (int o = KV; o < 64; o <<= 1) agg[i] += __shfl_xor(agg[i], o);
        if (lane < KV)
#pragma unroll
            for (int i = 0; i < 9; ++i) s_ag[n][i * KV + lane] = agg[i];
    }
    __syncthreads();
    // ---- proj (SO3_LinearV2 nh nv -> C), residual, norm_2 -> s_x[n]
    float x[NPW][9];
    {
        float y[NPW][9];
#pragma unroll
        for (int n = 0; n < NPW; ++n)
#pragma unroll
            for (int i = 0; i < 9; ++i) y[n][i] = 0.f;
        // weight loops in groups of NB_ROWS rows: the group's weight loads are issued together into
        // registers before its FMAs (one L2 round trip per group instead of per row or two); the
        // accumulation order is unchanged
        auto proj_rows = [&](int k0, auto nrows) {
            constexpr int R = decltype(nrows)::value;
            float w0[R], w1[R], w2[R];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int kk = k0 + u;
                w0[u] = A.proj_t[kk * C + c];
                w1[u] = A.proj_t[(KV + kk) * C + c];
                w2[u] = A.proj_t[(2 * KV + kk) * C + c];
            }
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int kk = k0 + u;
#pragma unroll
                for (int n = 0; n < NPW; ++n) {
                    y[n][0] += s_ag[n][kk] * w0[u];
#pragma unroll
                    for (int i = 1; i < 4; ++i) y[n][i] += s_ag[n][i * KV + kk] * w1[u];
#pragma unroll
                    for (int i = 4; i < 9; ++i) y[n][i] += s_ag[n][i * KV + kk] * w2[u];
                }
            }
        };
        {
            int k0 = 0;
            for (; k0 + NB_ROWS <= KV; k0 += NB_ROWS) proj_rows(k0, std::integral_constant<int, NB_ROWS>{});
            for (; k0 < KV; ++k0) proj_rows(k0, std::integral_constant<int, 1>{});
        }
        const float pb = A.proj_b[c];
#pragma unroll
        for (int n = 0; n < NPW; ++n) {
            const int64_t node = node0 + n < V ? node0 + n : V - 1;
            y[n][0] += pb;
            const float* xo = A.X + node * 9 * C + c;
#pragma unroll
            for (int i = 0; i < 9; ++i) x[n][i] = xo[i * C] + y[n][i];
            float xn[9];
            rms_norm(x[n], xn, A.norm2_w, A.norm2_b, c, on, C);
            if (on)
#pragma unroll
                for (int i = 0; i < 9; ++i) s_x[n][i * C + c] = xn[i];
        }
    }
    __syncthreads();
    // ---- FFN: gating + so3_linear_1, S2 activation on the grid -> s_x[n] (reused), so3_linear_2
    {
        const bool fon = lane < F;
        const int f = fon ? lane : 0;
        float gate[NPW], h[NPW][9];
#pragma unroll
        for (int n = 0; n < NPW; ++n) {
            gate[n] = A.gate_b[f];
            h[n][0] = A.lin1_b[f];
#pragma unroll
            for (int i = 1; i < 9; ++i) h[n][i] = 0.f;
        }
        auto lin1_rows = [&](int c0, auto nrows) {
            constexpr int R = decltype(nrows)::value;
            float wg[R], w0[R], w1[R], w2[R];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int cc = c0 + u;
                wg[u] = A.gate_t[cc * F + f];
                w0[u] = A.lin1_t[cc * F + f];
                w1[u] = A.lin1_t[(C + cc) * F + f];
                w2[u] = A.lin1_t[(2 * C + cc) * F + f];
            }
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int cc = c0 + u;
#pragma unroll
                for (int n = 0; n < NPW; ++n) {
                    gate[n] += s_x[n][cc] * wg[u];
                    h[n][0] += s_x[n][cc] * w0[u];
#pragma unroll
                    for (int i = 1; i < 4; ++i) h[n][i] += s_x[n][i * C + cc] * w1[u];
#pragma unroll
                    for (int i = 4; i < 9; ++i) h[n][i] += s_x[n][i * C + cc] * w2[u];
                }
            }
        };
        {
            int c0 = 0;
            for (; c0 + NB_ROWS <= C; c0 += NB_ROWS) lin1_rows(c0, std::integral_constant<int, NB_ROWS>{});
            for (; c0 < C; ++c0) lin1_rows(c0, std::integral_constant<int, 1>{});
        }
        __syncthreads();   // s_x is rewritten with the activation below
#pragma unroll
        for (int n = 0; n < NPW; ++n) {
            float o[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            for (int p = 0; p < GF; ++p) {
                float gv = 0.f;
#pragma unroll
                for (int i = 0; i < 9; ++i) gv += s_gt[p * 9 + i] * h[n][i];
                const float sg = silu(gv);
#pragma unroll
                for (int i = 0; i < 9; ++i) o[i] += s_gf[p * 9 + i] * sg;
            }
            o[0] = silu(gate[n]);
            if (fon)
#pragma unroll
                for (int i = 0; i < 9; ++i) s_x[n][i * F + f] = o[i];
        }
    }
    __syncthreads();
    {
        float h2[NPW][9];
        const float b2 = A.lin2_b[c];
#pragma unroll
        for (int n = 0; n < NPW; ++n) {
            h2[n][0] = b2;
#pragma unroll
            for (int i = 1; i < 9; ++i) h2[n][i] = 0.f;
        }
        auto lin2_rows = [&](int f0, auto nrows) {
            constexpr int R = decltype(nrows)::value;
            float w0[R], w1[R], w2[R];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int ff = f0 + u;
                w0[u] = A.lin2_t[ff * C + c];
                w1[u] = A.lin2_t[(F + ff) * C + c];
                w2[u] = A.lin2_t[(2 * F + ff) * C + c];
            }
#pragma unroll
            for (int u = 0; u < R; ++u) {
                const int ff = f0 + u;
#pragma unroll
                for (int n = 0; n < NPW; ++n) {
                    h2[n][0] += s_x[n][ff] * w0[u];
#pragma unroll
                    for (int i = 1; i < 4; ++i) h2[n][i] += s_x[n][i * F + ff] * w1[u];
#pragma unroll
                    for (int i = 4; i < 9; ++i) h2[n][i] += s_x[n][i * F + ff] * w2[u];
                }
            }
        };
        {
            int f0 = 0;
            for (; f0 + NB_ROWS <= F; f0 += NB_ROWS) lin2_rows(f0, std::integral_constant<int, NB_ROWS>{});
            for (; f0 < F; ++f0) lin2_rows(f0, std::integral_constant<int, 1>{});
        }
#pragma unroll
        for (int n = 0; n < NPW; ++n) {
            const int64_t node = node0 + n;
#pragma unroll
            for (int i = 0; i < 9; ++i) x[n][i] += h2[n][i];
            float xn[9];
            rms_norm(x[n], xn, A.nnorm_w, A.nnorm_b, c, on, C);
            if (node < V && on) {
                float* xw = A.X + node * 9 * C + c;
                float* xnw = A.XN + node * 9 * C + c;
#pragma unroll
                for (int i = 0; i < 9; ++i) {
                    xw[i * C] = x[n][i];
                    xnw[i * C] = xn[i];
                }
            }
        }
    }
}

struct EqWs {
    float *rot, *H2, *A0, *A1, *Y0, *Y1, *Z0, *Z1, *L, *V0, *V1, *X, *XN, *out;
    int* zn;
    int* RANGE;   // [64]: the call's fp16x2 range flag (tp_fused.h tp_range_flag)
    int ld0, ldv0, ldv1;
};

inline int ceil32(int x) { return (x + 31) & ~31; }

// ---- per-kind timing for nbx_eqv2_forward_timed: HIP event pairs around each launch group on the
// launch stream, with the group's algorithmic flops (2 x MACs of the fp32-accurate products) and
// HBM bytes (its tensor inputs + outputs once).  Kinds: 0 radial hidden layers, 1 radial output GEMM
// + message epilogue, 2 SO(2) conv 1 m = 0 GEMM, 3 SO(2) conv 1 m = 1 GEMM, 4 S2 activation +
// logits, 5 SO(2) conv 2 GEMMs, 6 node kernels, 7 edge frame + edge-degree embedding.
constexpr int EQ_KINDS = 8;
struct EqTimer {
    static constexpr int MAXR = 512;
    hipEvent_t ev[2 * MAXR];
    int kind[MAXR];
    int n = 0;
    double flops[EQ_KINDS] = {}, bytes[EQ_KINDS] = {};
};
thread_local EqTimer* g_timer = nullptr;
struct TScope {
    hipStream_t st;
    bool on = false;
    TScope(int k, hipStream_t s, double fl, double by) : st(s) {
        EqTimer* T = g_timer;
        if (T && T->n < EqTimer::MAXR - 1) {
            on = hipEventRecord(T->ev[2 * T->n], st) == hipSuccess;
            T->kind[T->n] = k;
            T->flops[k] += fl;
            T->bytes[k] += by;
        }
    }
    ~TScope() {
        if (on) {
            (void)hipEventRecord(g_timer->ev[2 * g_timer->n + 1], st);
            g_timer->n++;
        }
    }
};

size_t eqv2_carve(EqWs* ws, void* base, const nbx_eqv2_weights* w, int64_t B, int64_t N) {
    const int C = w->sphere_channels, H = w->attn_hidden, He = w->edge_channels, KV = w->num_heads * w->value_channels;
    const int64_t V = B * N, E = V * (N - 1);
    EqWs s;
    s.ld0 = std::max(ceil32(w->num_heads * w->alpha_channels + 4 * H), 3 * C);
    s.ldv0 = ceil32(3 * KV);
    s.ldv1 = ceil32(4 * KV);
    size_t off = 0;
    auto take = [&](size_t n, size_t el) -> void* {
        off = (off + 255) & ~size_t(255);
        void* p = base ? (void*)((char*)base + off) : nullptr;
        off += n * el;
        return p;
    };
    s.rot = (float*)take(E * ROT, 4);
    s.zn = (int*)take(V, 4);
    s.H2 = (float*)take(E * He, 4);
    s.A0 = (float*)take(E * 6 * C, 4);
    s.A1 = (float*)take(2 * E * 4 * C, 4);
    s.Y0 = (float*)take(E * s.ld0, 4);
    s.Y1 = (float*)take(2 * E * 4 * H, 4);
    s.Z0 = (float*)take(E * 3 * H, 4);
    s.Z1 = (float*)take(2 * E * 2 * H, 4);
    s.L = (float*)take(E * w->num_heads, 4);
    s.V0 = (float*)take(E * s.ldv0, 4);
    s.V1 = (float*)take(2 * E * s.ldv1, 4);
    s.X = (float*)take(V * 9 * C, 4);
    s.XN = (float*)take(V * 9 * C, 4);
    s.out = (float*)take(V * 6, 4);
    s.RANGE = (int*)take(64, 4);
    if (ws) *ws = s;
    return (off + 255) & ~size_t(255);
}

unsigned g1(int64_t n) { return (unsigned)nbx::ceil_div(n > 0 ? n : 1, 256); }
unsigned gwave(int64_t n) { return (unsigned)std::min<int64_t>(nbx::ceil_div(n > 0 ? n : 1, 4), 8192); }

// H2 = SiLU(LN(W1 SiLU(LN(h1_pre)) + b1)): the per-edge first layer, then an MFMA GEMM with the
// LayerNorm + SiLU epilogue (He = 32 or 64 columns: one column chunk).  H1 lives in the A0 buffer.
bool eq_h2_enabled();

int radial(const nbx_eqv2_weights* w, const nbx_eqv2_radial& R, const EqWs& ws, int64_t E, int N, hipStream_t st) {
    const int He = w->edge_channels;
    static const bool two = getenv("NBX_EQ_RAD2") && getenv("NBX_EQ_RAD2")[0] == '1';   // A/B: the two-launch form
    if (R.w1_h2 && eq_h2_enabled() && !two) {   // one launch (eqv2_radial_h2_kernel)
        const int64_t tiles = (E + 31) / 32;
        const unsigned blocks = (unsigned)std::min<int64_t>(nbx::ceil_div(tiles, RAD_WAVES), 4096);
        const size_t lds = ((size_t)(He / 32) * (He / 32) * nbx::LIN_H2_BLK + 4 * He) * 4;
        if (He == 64)
            hipLaunchKernelGGL(eqv2_radial_h2_kernel<64>, dim3(blocks), dim3(64 * RAD_WAVES), lds, st, ws.rot, ws.zn, R,
                               E, N, ws.H2, ws.RANGE);
        else
            hipLaunchKernelGGL(eqv2_radial_h2_kernel<32>, dim3(blocks), dim3(64 * RAD_WAVES), lds, st, ws.rot, ws.zn, R,
                               E, N, ws.H2, ws.RANGE);
        NBX_LAUNCH_CHECK("eqv2 radial (fp16x2, one launch)");
        return NBX_OK;
    }
    float* H1 = ws.A0;
    if (He == 64)
        hipLaunchKernelGGL(eqv2_radial_kernel<64>, dim3(gwave(E)), dim3(256), 0, st, ws.rot, ws.zn, R, E, N, H1);
    else
        hipLaunchKernelGGL(eqv2_radial_kernel<32>, dim3(gwave(E)), dim3(256), 0, st, ws.rot, ws.zn, R, E, N, H1);
    NBX_LAUNCH_CHECK("eqv2 radial");
    nbx::LinProb p = nbx::lin_dense(H1, He, He, (int)E, R.w1, He, He, R.b1, ws.H2, He);
    p.ln_w = R.ln2_w;
    p.ln_b = R.ln2_b;
    if (He == 64) return nbx::lin_launch<2, nbx::ACT_NONE, nbx::LIN_LNSILU>(p, st);
    return nbx::lin_launch<1, nbx::ACT_NONE, nbx::LIN_LNSILU>(p, st);
}

// the fp16x2 images when the weights carry them (NBX_EQ_SPLIT=x3: the bf16x3 images, A/B only)
bool eq_h2_enabled() {
    static const bool on = !(getenv("NBX_EQ_SPLIT") && (getenv("NBX_EQ_SPLIT")[0] == 'x' || getenv("NBX_EQ_SPLIT")[0] == '1'));
    return on;
}

// split-precision GEMM: Y[rows][ldy] = A[rows][K] W^T (+ bias), N padded to 32; on the fp16x2 image (Wh2,
// descaled by sinv, raising `flag` on a non-finite tile) when given and enabled, else the bf16x3 one
int gemm_x3(const float* A, int K, int rows, const void* Wx3, const void* Wh2, float sinv, int* flag, int N,
            const float* bias, float* Y, int ldy, hipStream_t st) {
    nbx::LinProb p = nbx::lin_dense(A, K, K, rows, nullptr, K, N, bias, Y, ldy);
    p.Wx3 = Wx3;
    if (Wh2 && eq_h2_enabled()) {
        p.Wh2 = Wh2;
        p.h2_sinv = sinv;
        p.range_flag = flag;
        return nbx::lin_launch<2, nbx::ACT_NONE, nbx::LIN_STORE, 2>(p, st);
    }
    return nbx::lin_launch<2, nbx::ACT_NONE, nbx::LIN_STORE, 1>(p, st);
}

// row-panel split-precision GEMM over all N = 32 ntiles columns (chunk-major image; lin.h lin_rp_kernel)
template <int PREC>
int gemm_rp_p(const nbx::LinRpProb& p, int ntiles, hipStream_t st) {
    switch (ntiles) {
        case 4: return nbx::lin_rp_launch<4, nbx::ACT_NONE, PREC>(p, st);
        case 5: return nbx::lin_rp_launch<5, nbx::ACT_NONE, PREC>(p, st);
        case 8: return nbx::lin_rp_launch<8, nbx::ACT_NONE, PREC>(p, st);
        case 9: return nbx::lin_rp_launch<9, nbx::ACT_NONE, PREC>(p, st);
        default:
            nbx::set_error("eqv2: no row-panel GEMM for %d column tiles", ntiles);
            return NBX_E_UNSUPPORTED;
    }
}
int gemm_rp(const float* A, int K, int rows, const void* Wx3, const void* Wh2, float sinv, int* flag, int ntiles,
            const float* bias, float* Y, int ldy, hipStream_t st) {
    const bool h2 = Wh2 && eq_h2_enabled();
    nbx::LinRpProb p{A, K, rows, K, h2 ? Wh2 : Wx3, bias, Y, ldy, 32 * ntiles, nullptr, 0, nullptr, sinv, flag};
    return h2 ? gemm_rp_p<2>(p, ntiles, st) : gemm_rp_p<1>(p, ntiles, st);
}

// SO2EquivariantGraphAttention (transformer_block.py:226-370) up to the per-edge values and logits
int attention_edges(const nbx_eqv2_weights* w, const nbx_eqv2_attn& Aw, const EqWs& ws, int64_t B, int N,
                    hipStream_t st) {
    const int C = w->sphere_channels, H = w->attn_hidden, He = w->edge_channels;
    const int nh = w->num_heads, KV = nh * w->value_channels;
    const int64_t V = B * N, E = V * (N - 1);
    const int iE = (int)E;
    const double e = (double)E, f4 = 4.0;
    const int na = w->alpha_channels, n0r = nh * na + 4 * H;
    {
        TScope ts(0, st, 2.0 * e * He * He, f4 * e * (2 * He + 2 * He + 1));
        if (int rc = radial(w, Aw.rad, ws, E, N, st)) return rc;
    }
    {   // rad = H2 W2^T + b2 (columns permuted), epilogue: A0/A1 = rad * rotated [x_src | x_dst]
        TScope ts(1, st, 2.0 * e * He * 10 * C, f4 * e * (He + 14 * C + 25));
        nbx::LinProb p = nbx::lin_dense(ws.H2, He, He, iE, nullptr, He, 10 * C, Aw.rad.b2, nullptr, 0);
        p.Wx3 = Aw.rad.w2_x3;
        p.Wh2 = Aw.w2_h2;
        p.h2_sinv = Aw.w2_sinv;
        p.range_flag = ws.RANGE;
        p.eq_x = ws.XN;
        p.eq_rot = ws.rot;
        p.eq_a0 = ws.A0;
        p.eq_a1 = ws.A1;
        p.eq_C = C;
        p.eq_nodes = N;
        const int rc = p.Wh2 && eq_h2_enabled() ? nbx::lin_launch<5, nbx::ACT_NONE, nbx::LIN_EQMSG, 2>(p, st)
                                                : nbx::lin_launch<5, nbx::ACT_NONE, nbx::LIN_EQMSG, 1>(p, st);
        if (rc) return rc;
    }
    const int n0 = ceil32(nh * w->alpha_channels + 4 * H);
    {
        TScope ts(2, st, 2.0 * e * 6 * C * n0r, f4 * e * (6 * C + n0r));
        if (int rc = gemm_rp(ws.A0, 6 * C, iE, Aw.fc0_x3, Aw.fc0_h2, Aw.fc0_sinv, ws.RANGE, n0 / 32, Aw.fc0_b, ws.Y0,
                             ws.ld0, st))
            return rc;
    }
    {
        TScope ts(3, st, 2.0 * 2 * e * 4 * C * 4 * H, f4 * 2 * e * (4 * C + 4 * H));
        if (int rc = gemm_rp(ws.A1, 4 * C, 2 * iE, Aw.fc1_x3, Aw.fc1_h2, Aw.fc1_sinv, ws.RANGE, 4 * H / 32, nullptr,
                             ws.Y1, 4 * H, st))
            return rc;
    }
    S2Args s{ws.Y0, ws.ld0, ws.Y1, w->grid_attn_to, w->grid_attn_from, Aw.alpha_norm_w, Aw.alpha_norm_b,
             Aw.alpha_dot, nh, w->alpha_channels, H, E, ws.Z0, ws.Z1, ws.L};
    {
        TScope ts(4, st, 2.0 * e * H * GA * 14, f4 * e * (n0r + 8 * H + 7 * H + nh));
        // NBX_EQV2_S2_NA0=1: the run-time alpha count (A/B)
        static const bool rt = getenv("NBX_EQV2_S2_NA0") && getenv("NBX_EQV2_S2_NA0")[0] == '1';
        if (!rt && s.na == 8)
            hipLaunchKernelGGL(eqv2_s2act_kernel<8>, dim3(g1(E * H)), dim3(256), 0, st, s);
        else if (!rt && s.na == 16)
            hipLaunchKernelGGL(eqv2_s2act_kernel<16>, dim3(g1(E * H)), dim3(256), 0, st, s);
        else
            hipLaunchKernelGGL(eqv2_s2act_kernel<0>, dim3(g1(E * H)), dim3(256), 0, st, s);
        NBX_LAUNCH_CHECK("eqv2 s2act");
    }
    {
        TScope ts(5, st, 2.0 * e * (3 * H * 3 * KV + 2 * 2 * H * 4 * KV), f4 * e * (7 * H + 11 * KV));
        if (int rc = gemm_x3(ws.Z0, 3 * H, iE, Aw.c20_x3, Aw.c20_h2, Aw.c20_sinv, ws.RANGE, ws.ldv0, Aw.c20_b, ws.V0,
                             ws.ldv0, st))
            return rc;
        if (int rc = gemm_x3(ws.Z1, 2 * H, 2 * iE, Aw.c21_x3, Aw.c21_h2, Aw.c21_sinv, ws.RANGE, ws.ldv1, nullptr, ws.V1,
                             ws.ldv1, st))
            return rc;
    }
    (void)KV;
    return NBX_OK;
}

NodeArgs node_args(const nbx_eqv2_weights* w, const EqWs& ws, int N) {
    NodeArgs a;
    memset(&a, 0, sizeof(a));
    a.L = ws.L; a.V0 = ws.V0; a.V1 = ws.V1; a.ldv0 = ws.ldv0; a.ldv1 = ws.ldv1;
    a.nh = w->num_heads; a.nv = w->value_channels;
    a.rot = ws.rot; a.X = ws.X; a.XN = ws.XN;
    a.gto = w->grid_ffn_to; a.gfrom = w->grid_ffn_from;
    a.C = w->sphere_channels; a.F = w->ffn_hidden; a.N = N;
    return a;
}

int eqv2_forward_impl(const nbx_eqv2_weights* w, const float* pos, const float* vel, const float* mass, int64_t B,
                      int64_t N64, const float* gauge, uint64_t seed, uint64_t frame, float* out, const EqWs& ws,
                      hipStream_t st) {
    const int N = (int)N64, C = w->sphere_channels, He = w->edge_channels;
    const int64_t V = B * N, E = V * (N - 1);
    const int F = w->ffn_hidden, KV = w->num_heads * w->value_channels;
    const double e = (double)E, v = (double)V, f4 = 4.0;
    // node kernel per block: proj + FFN flops, reads V0/V1/L/rot + X, writes X, XN
    const double node_fl = 2.0 * v * (9.0 * KV * C + C * F + 9.0 * C * F * 2 + GF * 18.0 * F) +
                           2.0 * e * (25.0 + 7.0) * KV;
    const double node_by = f4 * (e * (11.0 * KV + w->num_heads + 25) + v * 27.0 * C);
    {
    TScope ts_all(7, st, 2.0 * e * He * (He + 3 * C), f4 * (e * (32 + 2 * He + 3 * C) + v * 19.0 * C));
    hipLaunchKernelGGL(eqv2_edge_kernel, dim3(g1(std::max(V, E))), dim3(256), 0, st, pos, mass, gauge, seed, frame, V,
                       N, w->num_elements, ws.rot, ws.zn);
    NBX_LAUNCH_CHECK("eqv2 edge");
    // EdgeDegreeEmbedding radial -> [E][3C] (Y0 as scratch), then the embedding node pass
    if (int rc = radial(w, w->edge_degree, ws, E, N, st)) return rc;
    {
        nbx::LinProb p = nbx::lin_dense(ws.H2, He, He, (int)E, w->edge_degree.w2, He, 3 * C, w->edge_degree.b2, ws.Y0,
                                        3 * C);
        if (w->edge_degree.w2_h2 && eq_h2_enabled()) {   // fp16x2 (3C % 32 == 0: C is 32 or 64)
            p.Wh2 = w->edge_degree.w2_h2;
            p.h2_sinv = w->edge_degree.w2_sinv;
            p.range_flag = ws.RANGE;
            if (int rc = nbx::lin_launch<2, nbx::ACT_NONE, nbx::LIN_STORE, 2>(p, st)) return rc;
        } else if (int rc = nbx::lin_launch<2, nbx::ACT_NONE>(p, st)) {
            return rc;
        }
    }
    {
        NodeArgs a = node_args(w, ws, N);
        a.Red = ws.Y0; a.semb = w->sphere_emb; a.vel = vel; a.vel_t = w->vel_t; a.vel_b = w->vel_b; a.zn = ws.zn;
        a.nnorm_w = w->num_layers ? w->blocks[0].norm1_w : w->norm_w;
        a.nnorm_b = w->num_layers ? w->blocks[0].norm1_b : w->norm_b;
        hipLaunchKernelGGL(eqv2_node_kernel<NODE_INIT>, dim3((unsigned)(B * N)), dim3(64), 0, st, a);
        NBX_LAUNCH_CHECK("eqv2 node init");
    }
    }
    for (int l = 0; l < w->num_layers; ++l) {
        const nbx_eqv2_block& Bk = w->blocks[l];
        if (int rc = attention_edges(w, Bk.ga, ws, B, N, st)) return rc;
        NodeArgs a = node_args(w, ws, N);
        a.proj_t = Bk.ga.proj_t; a.proj_b = Bk.ga.proj_b; a.cout = C;
        a.norm2_w = Bk.norm2_w; a.norm2_b = Bk.norm2_b;
        a.gate_t = Bk.gate_t; a.gate_b = Bk.gate_b;
        a.lin1_t = Bk.lin1_t; a.lin1_b = Bk.lin1_b;
        a.lin2_t = Bk.lin2_t; a.lin2_b = Bk.lin2_b;
        const bool last = l + 1 == w->num_layers;
        a.nnorm_w = last ? w->norm_w : w->blocks[l + 1].norm1_w;
        a.nnorm_b = last ? w->norm_b : w->blocks[l + 1].norm1_b;
        TScope ts(6, st, node_fl, node_by);
        // two nodes per wave (measured at C4: 98.7 us against 100.4-101.1 us for one node per wave and
        // 139 us for four, whose 158 VGPRs cut the occupancy); NBX_EQ_NPW=1 keeps the one-node kernel
        static const int npw = getenv("NBX_EQ_NPW") ? atoi(getenv("NBX_EQ_NPW")) : 2;
        const int64_t V = B * N;
        if (npw == 2 && w->num_heads * w->value_channels <= 16)
        {
            // NBX_EQ_NB: weight rows per load batch (A/B: 1, 4, 8; measured at C4: 237.0 / 236.3, 234.8 /
            // 235.2, 226.8 / 228.7 steps/s -- the compiler's own schedule of one row per step is best)
            static const int nb = getenv("NBX_EQ_NB") ? atoi(getenv("NBX_EQ_NB")) : 1;
            if (nb == 8)
                hipLaunchKernelGGL((eqv2_node_block_kernel<2, 8>), dim3((unsigned)((V + 1) / 2)), dim3(64), 0, st, a, V);
            else if (nb == 4)
                hipLaunchKernelGGL((eqv2_node_block_kernel<2, 4>), dim3((unsigned)((V + 1) / 2)), dim3(64), 0, st, a, V);
            else
                hipLaunchKernelGGL((eqv2_node_block_kernel<2, 1>), dim3((unsigned)((V + 1) / 2)), dim3(64), 0, st, a, V);
        }
        else
            hipLaunchKernelGGL(eqv2_node_kernel<NODE_BLOCK>, dim3((unsigned)V), dim3(64), 0, st, a);
        NBX_LAUNCH_CHECK("eqv2 node block");
    }
    if (int rc = attention_edges(w, w->force, ws, B, N, st)) return rc;
    NodeArgs a = node_args(w, ws, N);
    a.proj_t = w->force.proj_t; a.proj_b = w->force.proj_b; a.cout = 2; a.out = out;
    TScope ts(6, st, 2.0 * e * 32.0 * KV + 2.0 * v * 9.0 * KV * 2, f4 * (e * (11.0 * KV + w->num_heads + 25) + v * 6));
    hipLaunchKernelGGL(eqv2_node_kernel<NODE_FORCE>, dim3((unsigned)(B * N)), dim3(64), 0, st, a);
    NBX_LAUNCH_CHECK("eqv2 node force");
    return NBX_OK;
}

int eqv2_prepare(const nbx_eqv2_weights* w, int64_t B, int64_t N, void* ws_ptr, size_t bytes, EqWs* ws) {
    NBX_CHECK_ARG(w, "eqv2: null weights");
    const int C = w->sphere_channels, H = w->attn_hidden, F = w->ffn_hidden, He = w->edge_channels;
    const int KV = w->num_heads * w->value_channels;
    NBX_CHECK_ARG(C == 32 || C == 64, "eqv2: sphere_channels must be 32 or 64 (got %d)", C);
    NBX_CHECK_ARG(H == 32 || H == 64, "eqv2: attn_hidden_channels must be 32 or 64 (got %d)", H);
    NBX_CHECK_ARG(F == 32 || F == 64, "eqv2: ffn_hidden_channels must be 32 or 64 (got %d)", F);
    NBX_CHECK_ARG(He == 32 || He == 64, "eqv2: edge_channels must be 32 or 64 (got %d)", He);
    NBX_CHECK_ARG(KV == 8 || KV == 16 || KV == 32, "eqv2: num_heads * attn_value_channels must be 8, 16 or 32");
    NBX_CHECK_ARG(w->num_heads >= 1 && w->num_heads <= 8 && w->alpha_channels >= 1 && w->alpha_channels <= 16,
                  "eqv2: num_heads <= 8, attn_alpha_channels <= 16");
    NBX_CHECK_ARG(w->num_layers >= 0 && w->num_layers <= NBX_EQV2_MAX_LAYERS, "eqv2: bad num_layers");
    NBX_CHECK_ARG(w->num_elements >= 1, "eqv2: num_elements");
    NBX_CHECK_ARG(B >= 1 && N >= 2 && N <= 64 && B * N * (N - 1) * 8 * C < ((int64_t)1 << 31),
                  "eqv2: need B >= 1, 2 <= N <= 64 and E * 8C < 2^31");
    const size_t need = eqv2_carve(ws, ws_ptr, w, B, N);
    if (!ws_ptr || bytes < need) {
        nbx::set_error("eqv2: workspace too small (%zu < %zu bytes)", bytes, need);
        return NBX_E_WORKSPACE;
    }
    return NBX_OK;
}

// ---- training step (eqv2_train.py): the reduced Wigner rows of every edge as a dense [7][9] block
// (rows l = 0; l = 1, m = -1, 0, 1; l = 2, m = -1, 0, 1 — the |m| <= mmax = 1 coefficients in l-primary
// order, so3.py:30-115; columns the 9 l-primary coefficients) and |pos_src - pos_dst|, from the same
// edge records the inference path uses (eqv2_edge_kernel).
__global__ void eqv2_dsel_kernel(int64_t E, const float* __restrict__ rot, float* __restrict__ dsel,
                                 float* __restrict__ dist) {
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (e >= E) return;
    const float* r = rot + e * ROT;
    dist[e] = r[24];
    if (!dsel) return;                                // nbx_eqv2_edges: frames and distances only
    float* d = dsel + e * 63;
#pragma unroll
    for (int i = 0; i < 63; ++i) d[i] = 0.f;
    d[0] = 1.f;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) d[(1 + a) * 9 + 1 + b] = r[3 * a + b];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 5; ++b) d[(4 + a) * 9 + 4 + b] = r[9 + 5 * a + b];
}

}  // namespace

extern "C" int nbx_eqv2_workspace_bytes(const nbx_eqv2_weights* w, int64_t B, int64_t N, size_t* bytes) {
    NBX_CHECK_ARG(w && bytes && B >= 1 && N >= 2, "nbx_eqv2_workspace_bytes: bad arguments");
    *bytes = eqv2_carve(nullptr, nullptr, w, B, N);
    return NBX_OK;
}

extern "C" int nbx_eqv2_forward(const nbx_eqv2_weights* w, const float* pos, const float* vel, const float* mass,
                                int64_t B, int64_t N, const float* gauge, uint64_t seed, float* out, void* workspace,
                                size_t workspace_bytes, void* stream) {
    EqWs ws;
    if (int rc = eqv2_prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    NBX_HIP(hipMemsetAsync(ws.RANGE, 0, sizeof(int), (hipStream_t)stream));
    return eqv2_forward_impl(w, pos, vel, mass, B, N, gauge, seed, 0, out, ws, (hipStream_t)stream);
}

extern "C" int nbx_eqv2_forward_timed(const nbx_eqv2_weights* w, const float* pos, const float* vel,
                                      const float* mass, int64_t B, int64_t N, const float* gauge, uint64_t seed,
                                      float* out, void* workspace, size_t workspace_bytes, void* stream,
                                      float kind_ms[8], int32_t kind_launches[8], double kind_flops[8],
                                      double kind_bytes[8], float* total_ms) {
    EqWs ws;
    if (int rc = eqv2_prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    hipStream_t st = (hipStream_t)stream;
    NBX_HIP(hipMemsetAsync(ws.RANGE, 0, sizeof(int), st));
    static EqTimer T;
    static bool made = false;
    if (!made) {
        for (auto& ev : T.ev) NBX_HIP(hipEventCreate(&ev));
        made = true;
    }
    T.n = 0;
    for (int k = 0; k < EQ_KINDS; ++k) T.flops[k] = T.bytes[k] = 0.0;
    hipEvent_t t0 = T.ev[2 * EqTimer::MAXR - 2], t1 = T.ev[2 * EqTimer::MAXR - 1];
    NBX_HIP(hipEventRecord(t0, st));
    g_timer = &T;
    const int rc = eqv2_forward_impl(w, pos, vel, mass, B, N, gauge, seed, 0, out, ws, st);
    g_timer = nullptr;
    if (rc) return rc;
    NBX_HIP(hipEventRecord(t1, st));
    NBX_HIP(hipEventSynchronize(t1));
    for (int k = 0; k < EQ_KINDS; ++k) {
        kind_ms[k] = 0.f;
        kind_launches[k] = 0;
        kind_flops[k] = T.flops[k];
        kind_bytes[k] = T.bytes[k];
    }
    for (int i = 0; i < T.n && i < EqTimer::MAXR - 1; ++i) {
        float ms = 0.f;
        NBX_HIP(hipEventElapsedTime(&ms, T.ev[2 * i], T.ev[2 * i + 1]));
        kind_ms[T.kind[i]] += ms;
        kind_launches[T.kind[i]] += 1;
    }
    NBX_HIP(hipEventElapsedTime(total_ms, t0, t1));
    return NBX_OK;
}

extern "C" int nbx_eqv2_rollout(const nbx_eqv2_weights* w, float* pos, float* vel, const float* mass, int64_t B,
                                int64_t N, int64_t num_frames, int32_t flags, uint64_t seed, float* traj_pos,
                                float* traj_vel, void* workspace, size_t workspace_bytes, void* stream) {
    EqWs ws;
    if (int rc = eqv2_prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    NBX_CHECK_ARG(num_frames >= 1, "nbx_eqv2_rollout: frames >= 1");
    hipStream_t st = (hipStream_t)stream;
    NBX_HIP(hipMemsetAsync(ws.RANGE, 0, sizeof(int), st));
    const int64_t V = B * N;
    hipLaunchKernelGGL(nbx::rollout_state_kernel, dim3(g1(3 * V)), dim3(256), 0, st, pos, vel, ws.out, V, (int)N,
                       (int64_t)0, num_frames, traj_pos, traj_vel, flags & NBX_ROLLOUT_ABSOLUTE);
    for (int64_t f = 1; f < num_frames; ++f) {
        if (int rc = eqv2_forward_impl(w, pos, vel, mass, B, N, nullptr, seed, (uint64_t)(f - 1), ws.out, ws, st))
            return rc;
        hipLaunchKernelGGL(nbx::rollout_state_kernel, dim3(g1(3 * V)), dim3(256), 0, st, pos, vel, ws.out, V, (int)N,
                           f, num_frames, traj_pos, traj_vel, flags & NBX_ROLLOUT_ABSOLUTE);
    }
    NBX_LAUNCH_CHECK("eqv2 rollout");
    return NBX_OK;
}

extern "C" int nbx_eqv2_train_edges(int64_t B, int64_t N, const float* pos, const float* mass, const float* gauge,
                                    uint64_t seed, int32_t num_elements, float* rot_scratch, float* dsel, float* dist,
                                    int32_t* zn, void* stream) {
    NBX_CHECK_ARG(B >= 1 && N >= 2 && num_elements >= 1, "nbx_eqv2_train_edges: bad sizes");
    NBX_CHECK_ARG(pos && mass && rot_scratch && dsel && dist && zn, "nbx_eqv2_train_edges: null operand");
    hipStream_t st = (hipStream_t)stream;
    const int64_t V = B * N, E = V * (N - 1);
    hipLaunchKernelGGL(eqv2_edge_kernel, dim3(g1(std::max(V, E))), dim3(256), 0, st, pos, mass, gauge, seed,
                       (uint64_t)0, V, (int)N, num_elements, rot_scratch, zn);
    NBX_LAUNCH_CHECK("eqv2 train edge");
    hipLaunchKernelGGL(eqv2_dsel_kernel, dim3(g1(E)), dim3(256), 0, st, E, rot_scratch, dsel, dist);
    NBX_LAUNCH_CHECK("eqv2 dsel");
    return NBX_OK;
}

extern "C" int nbx_eqv2_edges(int64_t B, int64_t N, const float* pos, const float* mass, const float* gauge,
                              uint64_t seed, int64_t frame, int32_t num_elements, float* rot_scratch, float* dist,
                              int32_t* zn, void* stream) {
    NBX_CHECK_ARG(B >= 1 && N >= 2 && num_elements >= 1 && frame >= 0, "nbx_eqv2_edges: bad sizes");
    NBX_CHECK_ARG(pos && mass && rot_scratch && dist && zn, "nbx_eqv2_edges: null operand");
    hipStream_t st = (hipStream_t)stream;
    const int64_t V = B * N, E = V * (N - 1);
    hipLaunchKernelGGL(eqv2_edge_kernel, dim3(g1(std::max(V, E))), dim3(256), 0, st, pos, mass, gauge, seed,
                       (uint64_t)frame, V, (int)N, num_elements, rot_scratch, zn);
    NBX_LAUNCH_CHECK("eqv2 edges");
    hipLaunchKernelGGL(eqv2_dsel_kernel, dim3(g1(E)), dim3(256), 0, st, E, rot_scratch, nullptr, dist);
    NBX_LAUNCH_CHECK("eqv2 edge distances");
    return NBX_OK;
}

extern "C" int nbx_eqv2_range_check(const nbx_eqv2_weights* w, const void* workspace, size_t workspace_bytes, int64_t B,
                                    int64_t N, void* stream) {
    EqWs ws;
    if (int rc = eqv2_prepare(w, B, N, const_cast<void*>(workspace), workspace_bytes, &ws)) return rc;
    int flag = 0;
    NBX_HIP(hipMemcpyAsync(&flag, ws.RANGE, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
    NBX_HIP(hipStreamSynchronize((hipStream_t)stream));
    if (flag) {
        nbx::set_error("eqv2: a GEMM operand left the fp16 range of the fp16x2 split path (|a| >= 65520) or the "
                       "input is not finite; the bf16x3 path (NBX_EQ_SPLIT=x3) keeps the fp32 exponent range");
        return NBX_E_RANGE;
    }
    return NBX_OK;
}
