// SEGNN forward + device-resident self-feed rollout (fp32).
//
// Reference: models/segnn/segnn.py:17-304, models/segnn/o3_building_blocks.py:10-278,
// helper_scripts/infer_self_feed.py:99-194.  Math restated in DESIGN.md §SEGNN.
//
// Data layout in HBM (V = B*N nodes, E = V*(N-1) edges, M = mul):
//   X    [4][V][M]   node features, plane 0 = 0e channels, planes 1..3 = x/y/z of 1o channels
//   NA   [V][4]      node attribute (1, na_x, na_y, na_z)  (na_0 forced to 1: catch_isolated_nodes)
//   EG   [Ep][8]     per edge slot (dst-major): rhat xyz, |rel|, m_src*m_dst
//   edges are enumerated dst-major in G = next_pow2(N-1) slots per destination:
//   slot e = dst*G + q, q < N-1 is the edge from the q-th other node of the system,
//   q >= N-1 is padding (zero rows, masked).  General graphs (a kNN graph of
//   build_graph_with_knn, any simple within-system graph): SLOT [V][G] int32 names the source
//   (local index) of slot q of each destination, sources ascending, -1 past the node's in-degree
//   DEG[dst]; padding slots carry |rel| = -1 in EG.  A node's messages are then G
//   consecutive rows, i.e. registers of one lane in the MFMA accumulator tile,
//   and aggregate without atomics (Ep = V*G; G = 4 at N = 5: no padding).
// Every O(3) tensor product with l <= 1 is split into a "scalar-row" GEMM
// [x_s | x_v.y] -> [s | t] and a "vector-row" GEMM x_v[:,k] -> v (one row per
// component); the constants of e3nn's path normalisation, the SEGNN rescale and
// the spherical-harmonic prefactors are folded into the packed weights.
// The x_i / x_j halves of message_layer_1 are linear in node features, so they
// are computed once per node (node_pre GEMM) and combined per edge.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "nbx_internal.h"
#include "tp16.h"
#include "tp_fused.h"
#include "msg_pre.h"

namespace {

using nbx::kC_SIGMOID;
using nbx::kC_SILU;
using nbx::kSH_C1;

__device__ inline float silu_f(float x) { return x / (1.0f + expf(-x)); }
__device__ inline float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }

// Elementwise kernels use block (32, 8): threadIdx.x = channel within a 32-chunk,
// threadIdx.y = row lane; a block covers ROWS_PER_BLOCK rows x 32 channels.
constexpr int EW_X = 32, EW_Y = 8, ROWS_PER_BLOCK = 16;

// ---------------------------------------------------------------- featurise + embedding
// O3Transform (o3_building_blocks.py:231-278) + catch_isolated_nodes (segnn.py:136-148), then
// embedding_layer: O3TensorProduct(2x1o+1x0e -> hidden, node attrs) (segnn.py:69-71,170).
// featurise + embedding in one launch: a block of FE_NODES nodes first runs O3Transform /
// catch_isolated_nodes per node (thread = node; NA and EG to HBM, X0 kept in LDS), then the
// embedding TP per (node, channel).
constexpr int FE_NODES = 8;   // nodes per block: V / 8 blocks fill the chip at the C2 size
// Featurise + embed the nodes [n0, n0 + nn) of whole systems.  lpos / lvel hold the positions
// and velocities from node pbase on: the global arrays (pbase 0) in featurize_embed_kernel, the
// block's LDS copy of the updated state in the rollout's fused pre_pool2 (rollout_pp2_kernel).
template <int NB>
__device__ __forceinline__ void featurize_nodes(const float* lpos, const float* lvel, int64_t pbase,
                                                const float* __restrict__ mass, int64_t V, int N, int G,
                                                const float* __restrict__ emb, const float* __restrict__ emb_b, int M,
                                                float* __restrict__ NA, float* __restrict__ EG, float* __restrict__ X,
                                                float* __restrict__ XD, int64_t n0, int nn,
                                                const int* __restrict__ slot, const float* __restrict__ degv) {
    __shared__ float sx0[NB][8];
    __shared__ float sna[NB][4];
    __shared__ float shs[NB][32][3];   // per (node, edge slot) kSH_C1 * rhat
    const int t = threadIdx.x;
    // edge geometry: one thread per (node, slot) pair (G <= 32; larger systems: one thread per node)
    const bool par = G <= 32;
    for (int pq = t; par && pq < nn * G; pq += blockDim.x) {
        const int ln = pq / G, q = pq - ln * G;
        const int64_t node = n0 + ln;
        float* eg = EG + (node * G + q) * 8;
        const int64_t b = node / N;
        const int d = (int)(node - b * N);
        const int sq = slot ? slot[node * G + q] : (q < N - 1 ? (q < d ? q : q + 1) : -1);
        if (sq < 0) {   // padding slot (general graphs mark it with |rel| = -1)
            eg[0] = eg[1] = eg[2] = eg[4] = 0.f;
            eg[3] = slot ? -1.f : 0.f;
            shs[ln][q][0] = shs[ln][q][1] = shs[ln][q][2] = 0.f;
            continue;
        }
        const int64_t s2 = b * N + sq;
        const float* ps = lpos + 3 * (s2 - pbase);
        const float* pd = lpos + 3 * (node - pbase);
        const float rx = ps[0] - pd[0], ry = ps[1] - pd[1];
        const float rz = ps[2] - pd[2];
        const float dist = sqrtf(rx * rx + ry * ry + rz * rz);
        const float inv = 1.0f / fmaxf(dist, 1e-12f);
        const float hx = rx * inv, hy = ry * inv, hz = rz * inv;
        eg[0] = hx; eg[1] = hy; eg[2] = hz; eg[3] = dist; eg[4] = mass[s2] * mass[node];
        shs[ln][q][0] = kSH_C1 * hx; shs[ln][q][1] = kSH_C1 * hy; shs[ln][q][2] = kSH_C1 * hz;
    }
    __syncthreads();
    if (t < nn) {
        const int64_t node = n0 + t;
        const float* pp = lpos + 3 * (node - pbase);
        const float* pv = lvel + 3 * (node - pbase);
        const float px = pp[0], py = pp[1], pz = pp[2];
        const float vx = pv[0], vy = pv[1], vz = pv[2];
        float sxh = 0.f, syh = 0.f, szh = 0.f;
        if (par) {
            for (int q = 0; q < (slot ? G : N - 1); ++q) {
                sxh += shs[t][q][0]; syh += shs[t][q][1]; szh += shs[t][q][2];
            }
        } else {
            const int64_t b = node / N;
            const int d = (int)(node - b * N);
            const float m = mass[node];
            for (int q = 0; q < N - 1; ++q) {
                const int64_t s2 = b * N + (q < d ? q : q + 1);
                const float* ps = lpos + 3 * (s2 - pbase);
                const float rx = ps[0] - px, ry = ps[1] - py, rz = ps[2] - pz;
                const float dist = sqrtf(rx * rx + ry * ry + rz * rz);
                const float inv = 1.0f / fmaxf(dist, 1e-12f);
                const float hx = rx * inv, hy = ry * inv, hz = rz * inv;
                float* eg = EG + (node * G + q) * 8;
                eg[0] = hx; eg[1] = hy; eg[2] = hz; eg[3] = dist; eg[4] = mass[s2] * m;
                sxh += kSH_C1 * hx; syh += kSH_C1 * hy; szh += kSH_C1 * hz;
            }
            for (int q = N - 1; q < G; ++q) {
                float* eg = EG + (node * G + q) * 8;
                eg[0] = eg[1] = eg[2] = eg[3] = eg[4] = 0.f;
            }
        }
        // scatter(reduce="mean") at edge_index[1]: a node without incoming edges gets 0
        const float cnt = slot ? degv[node] : (float)(N - 1);
        const float inv_cnt = cnt > 0.f ? 1.0f / cnt : 0.f;
        const float vn = sqrtf(vx * vx + vy * vy + vz * vz);
        const float vden = fmaxf(vn, 1e-12f);
        const float na1 = sxh * inv_cnt + kSH_C1 * (vx / vden), na2 = syh * inv_cnt + kSH_C1 * (vy / vden);
        const float na3 = szh * inv_cnt + kSH_C1 * (vz / vden);
        NA[4 * node + 0] = 1.0f; NA[4 * node + 1] = na1; NA[4 * node + 2] = na2; NA[4 * node + 3] = na3;
        sna[t][0] = 1.0f; sna[t][1] = na1; sna[t][2] = na2; sna[t][3] = na3;
        const float mp = (px + py + pz) / 3.0f;  // pos.mean(1): mean over xyz (reference quirk)
        sx0[t][0] = px - mp; sx0[t][1] = py - mp; sx0[t][2] = pz - mp;
        sx0[t][3] = vx; sx0[t][4] = vy; sx0[t][5] = vz; sx0[t][6] = vn; sx0[t][7] = 0.f;
    }
    __syncthreads();
    // thread = (channel w, node lane): the embedding coefficients of w are loaded once
    const int lanes = (int)blockDim.x >= M ? (int)blockDim.x / M : 1;
    const int l0 = lanes > 1 ? t / M : 0;
    if (l0 >= lanes) return;
    for (int w = lanes > 1 ? t % M : t; w < M; w += lanes > 1 ? M : (int)blockDim.x) {
    const float a0 = emb[w], a1 = emb[M + w], b0 = emb[2 * M + w], b1 = emb[3 * M + w];
    const float c = emb[4 * M + w], dd = emb[5 * M + w], bias = emb_b[w];
    for (int ln = l0; ln < nn; ln += lanes) {
        const int64_t n = n0 + ln;
        const float* x0 = sx0[ln];
        const float* na = sna[ln];
        const float u0n = x0[0] * na[1] + x0[1] * na[2] + x0[2] * na[3];
        const float u1n = x0[3] * na[1] + x0[4] * na[2] + x0[5] * na[3];
        X[n * M + w] = b0 * u0n + b1 * u1n + c * x0[6] + bias;
        float xd = 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float xv = a0 * x0[k] + a1 * x0[3 + k] + dd * x0[6] * na[1 + k];
            X[((1 + k) * V + n) * M + w] = xv;
            xd += xv * na[1 + k];
        }
        if (XD) XD[n * M + w] = xd;
    }
    }
}

__global__ void featurize_embed_kernel(const float* __restrict__ pos, const float* __restrict__ vel,
                                       const float* __restrict__ mass, int64_t V, int N, int G,
                                       const float* __restrict__ emb, const float* __restrict__ emb_b, int M,
                                       float* __restrict__ NA, float* __restrict__ EG, float* __restrict__ X,
                                       float* __restrict__ XD, double* __restrict__ zsum, int nzero,
                                       const int* __restrict__ slot, const float* __restrict__ degv,
                                       int* __restrict__ range_flag) {
    // zero the forward's atomic BatchNorm sums (nzero = 0: not in use) and, at the first frame of a call,
    // its fp16x2 range flag (null: a later frame, which accumulates into the call's flag)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nzero; i += gridDim.x * blockDim.x) zsum[i] = 0.0;
    if (range_flag && blockIdx.x == 0 && threadIdx.x == 0) *range_flag = 0;
    const int64_t n0 = (int64_t)blockIdx.x * FE_NODES;
    const int nn = (int)(V - n0 < FE_NODES ? V - n0 : FE_NODES);
    featurize_nodes<FE_NODES>(pos, vel, 0, mass, V, N, G, emb, emb_b, M, NA, EG, X, XD, n0, nn, slot, degv);
}

// ---------------------------------------------------------------- message
// message_layer_1 per (edge, channel) from the per-node precomputation NP
// NP rows: [V scalar rows | 3V vector rows] x 6M columns:
//   scalar row  [P_dst(2M) | R_dst(M) | P_src(2M) | R_src(M)]
//   vector row  [Q_dst(2M) | S_dst(M) | Q_src(2M) | S_src(M)]
// then Gate -> M1S [E][2M] = [m_s | m_v . rhat], M1V [3][E][M] = m_v
__global__ void msg1_kernel(const float* __restrict__ NP, const float* __restrict__ EG,
                            const float* __restrict__ amfw, const float* __restrict__ bias, int64_t V, int N, int G,
                            int M, float* __restrict__ M1S, float* __restrict__ M1V, const int* __restrict__ slot) {
    const int w = blockIdx.y * EW_X + threadIdx.x;
    if (w >= M) return;
    const int64_t E = V * G;
    const int ld = 6 * M;
    const float ea0 = amfw[w], eg0 = amfw[M + w], et0 = amfw[2 * M + w];
    const float ea1 = amfw[3 * M + w], eg1 = amfw[4 * M + w], et1 = amfw[5 * M + w];
    const float ba = bias[w], bg = bias[M + w];
    for (int64_t e = blockIdx.x * (int64_t)ROWS_PER_BLOCK + threadIdx.y; e < E && e < (blockIdx.x + 1) * (int64_t)ROWS_PER_BLOCK; e += EW_Y) {
        const int64_t dn = e / G;
        const int q = (int)(e - dn * G);
        const int64_t b = dn / N;
        const int d = (int)(dn - b * N);
        const int sq = slot ? slot[e] : (q < N - 1 ? (q < d ? q : q + 1) : -1);
        if (sq < 0) {  // padding slot
            M1S[e * 2 * M + w] = 0.f;
            M1S[e * 2 * M + M + w] = 0.f;
            for (int k = 0; k < 3; ++k) M1V[((int64_t)k * E + e) * M + w] = 0.f;
            continue;
        }
        const int64_t sn = b * N + sq;
        const float* eg = EG + e * 8;
        const float hx = eg[0], hy = eg[1], hz = eg[2], dist = eg[3], pm = eg[4];
        const float* sd = NP + dn * ld;
        const float* ss = NP + sn * ld;
        float sa = sd[w] + ss[3 * M + w] + ea0 * dist + ea1 * pm + ba;
        float sg = sd[M + w] + ss[4 * M + w] + eg0 * dist + eg1 * pm + bg;
        const float t = sd[2 * M + w] + ss[5 * M + w] + et0 * dist + et1 * pm;
        float v[3];
        const float hk[3] = {hx, hy, hz};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float* vd = NP + ((1 + k) * V + dn) * ld;
            const float* vs = NP + ((1 + k) * V + sn) * ld;
            sa += hk[k] * (vd[w] + vs[3 * M + w]);
            sg += hk[k] * (vd[M + w] + vs[4 * M + w]);
            v[k] = hk[k] * t + vd[2 * M + w] + vs[5 * M + w];
        }
        const float g = kC_SIGMOID * sigmoid_f(sg);
        float dot = 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float mv = g * v[k];
            M1V[((int64_t)k * E + e) * M + w] = mv;
            dot += mv * hk[k];
        }
        M1S[e * 2 * M + w] = kC_SILU * silu_f(sa);
        M1S[e * 2 * M + M + w] = dot;
    }
}

// e3nn BatchNorm (train mode) finalisation: one block per channel chunk of the producing
// TP kernel. The chunk's partial rows [wpc][3][cw] are read coalesced (thread = (row phase,
// column), all loads of a thread issued back to back), the row phases are combined in LDS in a
// fixed order (deterministic), then one thread per channel computes scale/shift and the
// running-stat update r <- (1-m) r + m * batch_stat.  The per-channel parameters are loaded
// before the reduction so their latency overlaps it.
// coef layout: [0..2M) scale (0e then 1o channels), [2M..3M) shift (0e).
constexpr int BNF_THREADS = 1024;
__global__ __launch_bounds__(BNF_THREADS) void bn_finalize_kernel(
        const double* __restrict__ partial, int wpc, int cw, double count, int M, int training, float eps,
        float momentum, const float* __restrict__ weight, const float* __restrict__ bias,
        float* __restrict__ rmean, float* __restrict__ rvar, float* __restrict__ coef) {
    __shared__ double red[BNF_THREADS];
    const int chunk = blockIdx.x, t = threadIdx.x;
    const int ncol = 3 * cw, phases = BNF_THREADS / ncol;
    // finalising threads: t < cw -> 0e channel, cw <= t < 2cw -> 1o channel
    const bool scalar = t < cw;
    const int c = chunk * cw + (scalar ? t : t - cw);
    const bool fin = t < 2 * cw && c < M;
    float wgt = 0.f, bs = 0.f, rm = 0.f, rv = 0.f;
    if (fin) {
        wgt = weight[scalar ? c : M + c];
        rv = rvar[scalar ? c : M + c];
        if (scalar) { bs = bias[c]; rm = rmean[c]; }
    }
    double a = 0.0, b = 0.0;
    if (training) {
        const int col = t % ncol, ph = t / ncol;
        double acc = 0.0;
        if (ph < phases) {
            const double* p = partial + (size_t)chunk * wpc * ncol + col;
#pragma unroll 8
            for (int i = ph; i < wpc; i += phases) acc += p[(size_t)i * ncol];
        }
        red[t] = acc;
        __syncthreads();
        if (fin) {
            const int ca = scalar ? t : 2 * cw + (t - cw);
            for (int q = 0; q < phases; ++q) a += red[q * ncol + ca];
            if (scalar)
                for (int q = 0; q < phases; ++q) b += red[q * ncol + cw + t];
        }
    }
    if (!fin) return;
    if (scalar) {
        double mu, var;
        if (training) {
            mu = a / count;
            var = b / count - mu * mu;
            if (var < 0.0) var = 0.0;
            rmean[c] = (1.0f - momentum) * rm + momentum * (float)mu;
            rvar[c] = (1.0f - momentum) * rv + momentum * (float)var;
        } else {
            mu = rm;
            var = rv;
        }
        const float sc = (float)(1.0 / sqrt(var + (double)eps)) * wgt;
        coef[c] = sc;
        coef[2 * M + c] = bs - sc * (float)mu;
    } else {
        double n;
        if (training) {
            n = a / (3.0 * count);
            rvar[M + c] = (1.0f - momentum) * rv + momentum * (float)n;
        } else {
            n = rv;
        }
        coef[M + c] = (float)(1.0 / sqrt(n + (double)eps)) * wgt;
    }
}

// Deterministic BatchNorm sums (nbx_segnn_weights.deterministic, and the SyncBN path of general
// graphs): the producing kernel's partial rows [chunk][wpc][3][cw] are summed in a fixed order into
// sums [3][M] (sum s, sum s^2 over the 0e channels, sum |v|^2 over the 1o channels) -- the layout
// the atomic path accumulates -- so the consumers (or bn_coef_kernel) finalise from the same slot
// and a SyncBN all-reduce can run between the two.
__global__ __launch_bounds__(BNF_THREADS) void bn_reduce_kernel(const double* __restrict__ partial, int wpc, int cw,
                                                               int M, double* __restrict__ sums) {
    __shared__ double red[BNF_THREADS];
    const int chunk = blockIdx.x, t = threadIdx.x;
    const int ncol = 3 * cw, phases = BNF_THREADS / ncol;
    const int col = t % ncol, ph = t / ncol;
    double acc = 0.0;
    if (ph < phases) {
        const double* p = partial + (size_t)chunk * wpc * ncol + col;
#pragma unroll 8
        for (int i = ph; i < wpc; i += phases) acc += p[(size_t)i * ncol];
    }
    red[t] = acc;
    __syncthreads();
    if (t < ncol) {
        double a = 0.0;
        for (int q = 0; q < phases; ++q) a += red[q * ncol + t];
        const int st = t / cw, c = chunk * cw + (t - st * cw);
        if (c < M) sums[st * M + c] = a;
    }
}

// coefficients [sc_s | sc_v | sh] (and the running-stat update) from finalised sums, for the
// consumers that read ws.coef_* (general graphs under SyncBN): one thread per (part, channel)
__global__ void bn_coef_kernel(nbx::BnSrc b, int M) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 3 * M) return;
    const int part = i / M, k = i - part * M;
    (void)nbx::bn_coef(b, M, part, k, true);
}

// ---------------------------------------------------------------- update
// message BatchNorm applied to the aggregate (BN is affine per channel, so
// sum_j BN(m_ij) = scale * sum_j m_ij + deg * shift), then the update_layer_1
// GEMM inputs: U1S [V][4M] = [x_s | a_s | x_v.na | a_v.na], U1V [3][V][2M] = [x_v[:,k] | a_v[:,k]]
__global__ void upd_pre_kernel(const float* __restrict__ X, const float* __restrict__ AGG,
                               const float* __restrict__ NA, const float* __restrict__ coef,
                               const float* __restrict__ xcoef, float deg, int64_t V, int M,
                               float* __restrict__ U1S, float* __restrict__ U1V, const float* __restrict__ degv) {
    const int w = blockIdx.y * EW_X + threadIdx.x;
    if (w >= M) return;
    const float sc_s = coef[w], sc_v = coef[M + w], sh1 = coef[2 * M + w];
    // pending feature BatchNorm of X (previous layer; identity for layer 0)
    const float xs_sc = xcoef ? xcoef[w] : 1.f, xv_sc = xcoef ? xcoef[M + w] : 1.f;
    const float xs_sh = xcoef ? xcoef[2 * M + w] : 0.f;
    for (int64_t n = blockIdx.x * (int64_t)ROWS_PER_BLOCK + threadIdx.y; n < V && n < (blockIdx.x + 1) * (int64_t)ROWS_PER_BLOCK; n += EW_Y) {
        const float* na = NA + 4 * n;
        const float xs = fmaf(xs_sc, X[n * M + w], xs_sh);
        const float as = sc_s * AGG[n * M + w] + sh1 * (degv ? degv[n] : deg);   // deg: in-degree
        float xdot = 0.f, adot = 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float xv = xv_sc * X[((1 + k) * V + n) * M + w];
            const float av = sc_v * AGG[((1 + k) * V + n) * M + w];
            xdot += xv * na[1 + k];
            adot += av * na[1 + k];
            U1V[((int64_t)k * V + n) * 2 * M + w] = xv;
            U1V[((int64_t)k * V + n) * 2 * M + M + w] = av;
        }
        float* u = U1S + n * 4 * M;
        u[w] = xs; u[M + w] = as; u[2 * M + w] = xdot; u[3 * M + w] = adot;
    }
}

// feature BatchNorm apply (in place on X)
__global__ void bn_apply_kernel(float* __restrict__ X, const float* __restrict__ coef, int64_t V, int M,
                                float* __restrict__ XD) {
    const int w = blockIdx.y * EW_X + threadIdx.x;
    if (w >= M) return;
    const float sc_s = coef[w], sc_v = coef[M + w], sh = coef[2 * M + w];
    for (int64_t n = blockIdx.x * (int64_t)ROWS_PER_BLOCK + threadIdx.y; n < V && n < (blockIdx.x + 1) * (int64_t)ROWS_PER_BLOCK; n += EW_Y) {
        X[n * M + w] = sc_s * X[n * M + w] + sh;
#pragma unroll
        for (int k = 0; k < 3; ++k) X[((1 + k) * V + n) * M + w] *= sc_v;
        if (XD) XD[n * M + w] *= sc_v;   // x_v . na is linear in x_v
    }
}

// pre_pool1 inputs from X with the last layer's pending feature BatchNorm applied (coef, or
// identity when null): U1S [V][2M] = [x_s | x_v.na], U1V [3][V][M] = x_v
__global__ void pp_pre_kernel(const float* __restrict__ X, const float* __restrict__ NA,
                              const float* __restrict__ coef, int64_t V, int M, float* __restrict__ U1S,
                              float* __restrict__ U1V) {
    const int w = blockIdx.y * EW_X + threadIdx.x;
    if (w >= M) return;
    const float sc_s = coef ? coef[w] : 1.f, sc_v = coef ? coef[M + w] : 1.f, sh = coef ? coef[2 * M + w] : 0.f;
    for (int64_t n = blockIdx.x * (int64_t)ROWS_PER_BLOCK + threadIdx.y; n < V && n < (blockIdx.x + 1) * (int64_t)ROWS_PER_BLOCK; n += EW_Y) {
        const float* na = NA + 4 * n;
        float dot = 0.f;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float xv = sc_v * X[((1 + k) * V + n) * M + w];
            U1V[((int64_t)k * V + n) * M + w] = xv;
            dot += xv * na[1 + k];
        }
        U1S[n * 2 * M + w] = fmaf(sc_s, X[n * M + w], sh);
        U1S[n * 2 * M + M + w] = dot;
    }
}

// Optional fused self-feed state update (infer_self_feed.py:182-211, target pos_dt+vel):
// pos += out[:3], vel = out[3:], and the new state is written as trajectory frame `frame`.
struct RolloutUpdate {
    float* pos;
    float* vel;
    float* traj_pos;
    float* traj_vel;
    int64_t frame, num_frames;
    int N;
    int featurize_next;   // rollout_pp2_kernel: also featurise + embed the next frame's input
    int absolute;         // target "pos+vel" (NBX_ROLLOUT_ABSOLUTE): pos = out[:3] instead of pos += out[:3]
};

// pre_pool2 of node n by one wave (lanes over M); lanes 0-2 write out[n] and, in a rollout, the
// updated state (also to sp / sv when non-null)
__device__ __forceinline__ void pp2_node(const float* __restrict__ H2S, const float* __restrict__ H2V,
                                         const float* __restrict__ NA, const float* __restrict__ W, int64_t V, int M,
                                         float* __restrict__ out, const RolloutUpdate& U, int64_t n, int lane,
                                         float* sp, float* sv) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // t0, t1, v0xyz, v1xyz
    for (int u = lane; u < M; u += 64) {
        const float hs = H2S[n * 2 * M + u];
        acc[0] += W[u] * hs;
        acc[1] += W[M + u] * hs;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float hv = H2V[((int64_t)k * V + n) * M + u];
            acc[2 + k] += W[2 * M + u] * hv;
            acc[5 + k] += W[3 * M + u] * hv;
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
        for (int off = 32; off > 0; off >>= 1) acc[i] += __shfl_xor(acc[i], off);
    if (lane < 3) {
        const int k = lane;
        const float* na = NA + 4 * n;
        const float dp = na[1 + k] * acc[0] + acc[2 + k];
        const float nv = na[1 + k] * acc[1] + acc[5 + k];
        out[6 * n + k] = dp;
        out[6 * n + 3 + k] = nv;
        if (U.pos) {
            const float p = U.absolute ? dp : U.pos[3 * n + k] + dp;
            U.pos[3 * n + k] = p;
            U.vel[3 * n + k] = nv;
            const int64_t b = n / U.N, d = n - b * U.N;
            const int64_t o = ((b * U.num_frames + U.frame) * U.N + d) * 3 + k;
            U.traj_pos[o] = p;
            U.traj_vel[o] = nv;
            if (sp) { sp[k] = p; sv[k] = nv; }
        }
    }
}

__global__ void pp2_kernel(const float* __restrict__ H2S, const float* __restrict__ H2V,
                           const float* __restrict__ NA, const float* __restrict__ W, int64_t V, int M,
                           float* __restrict__ out, RolloutUpdate U) {
    const int64_t n = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
    if (n >= V) return;
    pp2_node(H2S, H2V, NA, W, V, M, out, U, n, threadIdx.x & 63, nullptr, nullptr);
}

// Rollout frames before the last: pre_pool2 + the state update of this frame, then the next
// frame's featurisation + embedding (featurize_embed_kernel's work) from the updated state, in
// one launch.  A block owns nb nodes = whole systems (one wave per node), so every position a
// system's edges need is in the block's LDS after the barrier.
constexpr int RPP2_MAX = 16;   // nodes (waves) per block
__global__ __launch_bounds__(64 * RPP2_MAX) void rollout_pp2_kernel(
    const float* __restrict__ H2S, const float* __restrict__ H2V, float* __restrict__ NA, const float* __restrict__ W,
    int64_t V, int M, float* __restrict__ out, RolloutUpdate U, int nb, const float* __restrict__ mass, int N, int G,
    const float* __restrict__ emb, const float* __restrict__ emb_b, float* __restrict__ EG, float* __restrict__ X,
    float* __restrict__ XD, double* __restrict__ zsum, int nzero) {
    __shared__ float spos[RPP2_MAX][3], svel[RPP2_MAX][3];
    // zero the next forward's atomic BatchNorm sums (this forward's last consumer, pre_pool1, is done)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nzero; i += gridDim.x * blockDim.x) zsum[i] = 0.0;
    const int64_t n0 = blockIdx.x * (int64_t)nb;
    const int wv = threadIdx.x >> 6;
    const int nn = (int)(V - n0 < nb ? V - n0 : nb);
    if (wv < nn) pp2_node(H2S, H2V, NA, W, V, M, out, U, n0 + wv, threadIdx.x & 63, spos[wv], svel[wv]);
    __syncthreads();   // all of this block's NA reads are done before featurize_nodes rewrites it
    featurize_nodes<RPP2_MAX>(&spos[0][0], &svel[0][0], n0, mass, V, N, G, emb, emb_b, M, NA, EG, X, XD, n0, nn,
                              nullptr, nullptr);
}

// self-feed state update (infer_self_feed.py:182-194, target pos_dt+vel) and trajectory write
__global__ void rollout_update_kernel(float* __restrict__ pos, float* __restrict__ vel, const float* __restrict__ out,
                                      int64_t V, int N, int64_t frame, int64_t num_frames,
                                      float* __restrict__ traj_pos, float* __restrict__ traj_vel) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= V * 3) return;
    const int64_t node = i / 3;
    const int k = (int)(i - node * 3);
    float p = pos[i], v = vel[i];
    if (frame > 0) {
        p = p + out[6 * node + k];
        v = out[6 * node + 3 + k];
        pos[i] = p;
        vel[i] = v;
    }
    const int64_t b = node / N, d = node - b * N;
    const int64_t o = ((b * num_frames + frame) * N + d) * 3 + k;
    traj_pos[o] = p;
    traj_vel[o] = v;
}

// ---------------------------------------------------------------- host side
int next_pow2(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

struct Dims {
    int64_t B, N, V, G, Ep;  // Ep = V * G padded edge slots
    int M, chunks;
};

Dims dims_of(int64_t B, int64_t N, int M) {
    Dims d;
    d.B = B; d.N = N; d.V = B * N;
    d.G = N > 1 ? next_pow2((int)(N - 1)) : 1;
    d.Ep = d.V * d.G;
    d.M = M;
    d.chunks = (M + 31) / 32;
    return d;
}

// Upper bound of waves per chunk over every fused launch (partials buffer size).
// Upper bound of (chunks x waves per chunk x 3 x chunk width) over every fused
// launch: the BN partial-sum buffer size in doubles.
int64_t partial_doubles(const Dims& d) {
    const int64_t tiles = (std::max(d.Ep, d.V) + 15) / 16;
    const int64_t waves = std::min<int64_t>(tiles, 2 * 256 * 8);  // <= 2 blocks/CU x 8 waves per group
    const int64_t chunks16 = (d.M + 15) / 16;
    return std::max<int64_t>(1, (chunks16 + 1) * (waves + 8)) * 3 * 32;
}

struct Workspace {
    float *X, *NA, *EG, *NP, *M1S, *M1V, *AGG, *U1S, *U1V, *U2S, *U2V, *coef_msg, *coef_feat, *out;
    float *XD, *AD;   // x_v . na and aggregated a_v . na per node and channel (segmented update_layer_1)
    int* SLOT;        // general graphs: [Ep] source of each slot (-1 padding)
    float* DEG;       // general graphs: [V] in-degree
    unsigned long long* ADJ;   // general graphs: [V] source bit masks
    int* ERR;         // general graphs: [64] validation flags
    int* RANGE;       // fp16x2 range flag of the call (tp_fused.h tp_range_flag), zeroed by its first featurisation
    double* partial;
    double* bn_sums;  // atomic-mode BatchNorm sums: [2 x NBX_SEGNN_MAX_LAYERS][3][M] (message, feature per layer)
    size_t bytes;
};

size_t carve(Workspace* ws, void* base, int64_t B, int64_t N, int M) {
    const Dims d = dims_of(B, N, M);
    const int64_t V = d.V, Ep = d.Ep;
    size_t off = 0;
    auto take = [&](size_t n_elems, size_t elem) -> void* {
        off = (off + 255) & ~size_t(255);
        void* p = base ? (void*)((char*)base + off) : nullptr;
        off += n_elems * elem;
        return p;
    };
    Workspace w;
    w.partial = (double*)take((size_t)partial_doubles(d), 8);
    w.bn_sums = (double*)take((size_t)2 * NBX_SEGNN_MAX_LAYERS * 3 * M, 8);
    w.X = (float*)take(4 * V * M, 4);
    w.NA = (float*)take(4 * V, 4);
    w.EG = (float*)take(8 * Ep, 4);
    w.NP = (float*)take(4 * V * 6 * M, 4);
    w.M1S = (float*)take(Ep * 2 * M, 4);
    w.M1V = (float*)take(3 * Ep * M, 4);
    w.AGG = (float*)take(4 * V * M, 4);
    w.U1S = (float*)take(V * 4 * M, 4);
    w.U1V = (float*)take(3 * V * 2 * M, 4);
    w.U2S = (float*)take(V * 2 * M, 4);
    w.U2V = (float*)take(3 * V * M, 4);
    w.coef_msg = (float*)take(3 * M, 4);
    w.coef_feat = (float*)take(3 * M, 4);
    w.out = (float*)take(6 * V, 4);
    w.XD = (float*)take(V * M, 4);
    w.AD = (float*)take(V * M, 4);
    w.SLOT = (int*)take(Ep, 4);
    w.DEG = (float*)take(V, 4);
    w.ADJ = (unsigned long long*)take(V, 8);
    w.ERR = (int*)take(64, 4);
    w.RANGE = (int*)take(64, 4);
    w.bytes = (off + 255) & ~size_t(255);
    if (ws) *ws = w;
    return w.bytes;
}

int check_weights(const nbx_segnn_weights* w) {
    NBX_CHECK_ARG(w != nullptr, "segnn: null weights");
    NBX_CHECK_ARG(w->mul > 0 && w->mul % 4 == 0, "segnn: mul must be a positive multiple of 4 (got %d)", w->mul);
    NBX_CHECK_ARG(w->num_layers >= 0 && w->num_layers <= NBX_SEGNN_MAX_LAYERS, "segnn: bad num_layers %d",
                  w->num_layers);
    return NBX_OK;
}

dim3 ew_grid(int64_t rows, int M) {
    return dim3((unsigned)nbx::ceil_div(rows > 0 ? rows : 1, ROWS_PER_BLOCK), (unsigned)nbx::ceil_div(M, EW_X));
}

// Optional per-launch timing of the dominant kernel (nbx_segnn_forward_timed):
// an event pair around every tp_fused launch on the launch stream.
// Kinds: 0 = TP_PLAIN (node_pre), 1 = TP_MSG, 2 = TP_GATE_NODE, 3 = TP_RESID.
struct KernelTiming {
    std::vector<hipEvent_t> ev;
    std::vector<int> kind;
    double flops[4] = {0, 0, 0, 0};
    int launches[4] = {0, 0, 0, 0};
};

template <int NS, int NV, int EPI, int WAVES = nbx::TP_WAVES, int D = 2, class SK = nbx::DynSK>
int run_tp(nbx::TpProb& p, hipStream_t st, KernelTiming* tm) {
    p.NS = NS;
    p.NV = NV;
    p.epi = EPI;
    nbx::tp_geometry(p, WAVES, 256, SK::PREC);
    if (!tm) return nbx::tp_launch<NS, NV, EPI, WAVES, D, SK>(p, st);
    hipEvent_t a, b;
    NBX_HIP(hipEventCreate(&a));
    NBX_HIP(hipEventCreate(&b));
    tm->ev.push_back(a);
    tm->ev.push_back(b);
    nbx::armed_events() = {a, b};   // the launch below records the kernel's own begin / end
    if (int rc = nbx::tp_launch<NS, NV, EPI, WAVES, D, SK>(p, st)) return rc;
    NBX_HIP(nbx::disarm_events(st));
    double k = 0;
    for (int j = 0; j < NS; ++j) k += p.K[j];
    k += NV ? 3.0 * p.Kv : 0.0;
    tm->kind.push_back(EPI);
    tm->flops[EPI] += 2.0 * p.rows * 32.0 * p.chunks * k;  // executed MACs x 2 (incl. channel padding)
    tm->launches[EPI] += 1;
    return NBX_OK;
}

// The node TPs run a fully unrolled K loop when their chunk counts match one of the static
// schedules compiled here (the C2 width mul = 96 and mul = 32), else the run-time-shaped loop.
// NBX_STATIC=0 forces the run-time loop (A/B only).
// BatchNorm statistics by fp64 atomics, finalised inside the consuming kernel (no finalize
// launch; NBX_BN_ATOMIC=0 restores the partial rows + bn_finalize_kernel path)
bool bn_atomic_enabled() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("NBX_BN_ATOMIC");
        v = (e && e[0] == '0') ? 0 : 1;
    }
    return v == 1;
}

bool static_enabled() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("NBX_STATIC");
        v = (e && e[0] == '0') ? 0 : 1;
    }
    return v == 1;
}

template <class SK>
bool sk_matches(const nbx::TpProb& p, int NS, int NV) {
    auto kc = [](int K) { return (K + 31) / 32; };
    return kc(p.K[0]) == SK::K0 && (NS < 2 || kc(p.K[1]) == SK::K1) && (NS < 3 || kc(p.K[2]) == SK::K2) &&
           (NV ? kc(p.Kv) : 0) == SK::KV;
}

// K chunk schedules per TP at mul = 96 and mul = 32
using SK_UPD1 = nbx::StatSK<12, 12, 6, 6>;
using SK_UPD1_32 = nbx::StatSK<4, 4, 2, 2>;
using SK_UPD1_SEG = nbx::StatSK<12, 12, 6, 6, 4>;
using SK_UPD1_SEG_X3 = nbx::StatSKX3<12, 12, 6, 6, 4>;
using SK_UPD1_32_SEG = nbx::StatSK<4, 4, 2, 2, 4>;
using SK_UPD2 = nbx::StatSK<6, 3, 0, 3>;
using SK_UPD2_32 = nbx::StatSK<2, 1, 0, 1>;
using SK_GATE = nbx::StatSK<6, 6, 3, 3>;     // pre_pool1 (and message_layer_2's shape)
using SK_GATE_32 = nbx::StatSK<2, 2, 1, 1>;
using SK_PP1_SEG = nbx::StatSK<6, 6, 3, 3, 2>;   // pre_pool1 reading [x_s | x_v.na] + x_v from X / XD
using SK_PP1_32_SEG = nbx::StatSK<2, 2, 1, 1, 2>;
using SK_MSG2_X3 = nbx::StatSKX3<6, 6, 3, 3>;
using SK_MSG2_32_X3 = nbx::StatSKX3<2, 2, 1, 1>;
// fp16x2 split path (include/nbx.h "fp16x2 images")
using SK_MSG2_H2 = nbx::StatSKH2<6, 6, 3, 3>;
using SK_MSG2_32_H2 = nbx::StatSKH2<2, 2, 1, 1>;
using SK_MSG2_H2_DV = nbx::StatSKH2<6, 6, 3, 3, 0, 1>;     // dot half of M1S formed in registers
using SK_MSG2_32_H2_DV = nbx::StatSKH2<2, 2, 1, 1, 0, 1>;
using SK_UPD1_SEG_H2 = nbx::StatSKH2<12, 12, 6, 6, 4>;
using SK_UPD1_32_SEG_H2 = nbx::StatSKH2<4, 4, 2, 2, 4>;
using SK_UPD2_H2 = nbx::StatSKH2<6, 3, 0, 3>;
using SK_UPD2_32_H2 = nbx::StatSKH2<2, 1, 0, 1>;
using SK_PP1_SEG_H2 = nbx::StatSKH2<6, 6, 3, 3, 2>;
using SK_PP1_32_SEG_H2 = nbx::StatSKH2<2, 2, 1, 1, 2>;
// (register-formed x_v . na / a_v . na chunks: tp_fused.h TpStream)
using SK_UPD1_SEG_H2_DV = nbx::StatSKH2<12, 12, 6, 6, 4, 1>;
using SK_UPD1_32_SEG_H2_DV = nbx::StatSKH2<4, 4, 2, 2, 4, 1>;
using SK_PP1_SEG_H2_DV = nbx::StatSKH2<6, 6, 3, 3, 2, 1>;
using SK_PP1_32_SEG_H2_DV = nbx::StatSKH2<2, 2, 1, 1, 2, 1>;
using SK_UPD2_H2_DV = nbx::StatSKH2<6, 3, 0, 3, 0, 1>;   // [h_s | h_v . na]: the dot half from U2V
using SK_UPD2_32_H2_DV = nbx::StatSKH2<2, 1, 0, 1, 0, 1>;

// message_layer_2 on the split-precision MFMA path when the weights carry a bf16x3 image
// (NBX_X3=0: fp32 MFMA path, A/B only)
bool x3_enabled() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("NBX_X3");
        v = (e && e[0] == '0') ? 0 : 1;
    }
    return v == 1;
}

// Split-precision MFMA path of the SEGNN TPs: 2 = the fp16x2 images (default, when present),
// 1 = the bf16x3 images, 0 = fp32 MFMA.  NBX_SPLIT=x3 / NBX_X3=0 select 1 / 0 (A/B only).
int split_prec() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("NBX_SPLIT");
        v = !x3_enabled() ? 0 : (e && (e[0] == 'x' || e[0] == '1')) ? 1 : (e && e[0] == '0') ? 0 : 2;
    }
    return v;
}

// NBX_TP_DEBUG: per-wave phase clocks scratch buffer (tuning only)
unsigned long long* tp_dbg_buf(hipStream_t st) {
    static unsigned long long* dbg = nullptr;
    if (!dbg && hipMalloc(&dbg, sizeof(unsigned long long) * 4 * 65536) != hipSuccess) return nullptr;
    if (hipMemsetAsync(dbg, 0, sizeof(unsigned long long) * 4 * 65536, st) != hipSuccess) return nullptr;
    return dbg;
}

// NBX_TP_DEBUG=1: per-wave phase clocks of the message kernel printed to stderr (tuning only)
int tp_debug_dump(const nbx::TpProb& p, hipStream_t st, int waves) {
    const int n = p.chunks * p.blocks_per_chunk * waves;
    std::vector<unsigned long long> h((size_t)n * 6);
    NBX_HIP(hipStreamSynchronize(st));
    NBX_HIP(hipMemcpy(h.data(), p.dbg, h.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long w0 = ~0ull, w1 = 0;
    double s01 = 0, s12 = 0, s23 = 0, sw = 0, sc = 0;
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
        const unsigned long long* d = &h[(size_t)i * 6];
        if (!d[3]) continue;
        w0 = std::min(w0, d[4]);
        w1 = std::max(w1, d[5]);
        sw += (double)(d[5] - d[4]);
        sc += (double)(d[3] - d[0]);
        if (d[2]) { s01 += d[1] - d[0]; s12 += d[2] - d[1]; s23 += d[3] - d[2]; ++cnt; }
    }
    // wall_clock64 ticks at 100 MHz on every XCD: the waves' span and the shader clock rate
    fprintf(stderr, "tp_debug waves=%d stage=%.0f loop=%.0f epi=%.0f (avg clocks) waves_span=%.2fus wave_avg=%.2fus clk=%.2fGHz\n",
            cnt, s01 / std::max(cnt, 1), s12 / std::max(cnt, 1), s23 / std::max(cnt, 1), (w1 - w0) / 100.0,
            sw / std::max(cnt, 1) / 100.0, sw > 0 ? sc / sw * 0.1 : 0.0);
    return NBX_OK;
}

// message_layer_2 forms the dot half of its scalar operand (M1S [m_s | m_v . rhat]) from M1V in
// registers (tp_fused.h TpStream, DV) instead of reading it, and msg_pre does not write it: 20 %
// fewer A bytes per edge.  Requires the fp16x2 static schedule (mul 96 or 32); NBX_MSG_DV=0: the
// dot half is written and read (A/B only).
bool msg_dv(int64_t M, int64_t N, bool h2_img) {
    static const bool on = !(getenv("NBX_MSG_DV") && getenv("NBX_MSG_DV")[0] == '0');
    return on && h2_img && static_enabled() && split_prec() == 2 && N > 1 && (M == 96 || M == 32);
}

// update_layer_1 and pre_pool1 form their x_v . na / a_v . na operand chunks from the vector planes
// in registers (tp_fused.h TpStream, DV), so XD / AD are neither written (update_layer_2, message_layer_2,
// featurisation) nor read: requires the fp16x2 segmented schedules of every layer (mul 96 or 32);
// NBX_UPD_DV=0: XD / AD are materialised (A/B only).
bool upd_dv(const nbx_segnn_weights* w, int64_t M, bool seg_upd) {
    static const bool on = !(getenv("NBX_UPD_DV") && getenv("NBX_UPD_DV")[0] == '0');
    if (!on || !seg_upd || split_prec() != 2 || !(M == 96 || M == 32) || !w->pp1_img_h2) return false;
    for (int l = 0; l < w->num_layers; ++l)
        if (!w->layers[l].upd1_img_h2) return false;
    return true;
}

template <int NS, int NV, int EPI>
int run_tp_msg_sel(nbx::TpProb& p, hipStream_t st, KernelTiming* tm, const void* img_x3, const void* img_h2,
                   float h2_descale, bool dv) {
    // message_layer_2 at mul = 96 / 32: fully unrolled static chunk schedule
    if (dv) {   // (msg_dv: the M1S dot half was not written)
        if constexpr (EPI == nbx::TP_MSG && NS == 3 && NV == 1) {
            p.B = static_cast<const float*>(img_h2);
            p.bscale = h2_descale;
            if (sk_matches<SK_MSG2_H2_DV>(p, NS, NV)) return run_tp<NS, NV, EPI, 8, 2, SK_MSG2_H2_DV>(p, st, tm);
            if (sk_matches<SK_MSG2_32_H2_DV>(p, NS, NV)) return run_tp<NS, NV, EPI, 8, 3, SK_MSG2_32_H2_DV>(p, st, tm);
        }
        nbx::set_error("message_layer_2: no register-dot schedule for this shape");
        return NBX_E_UNSUPPORTED;
    }
    if (static_enabled()) {
        if (img_h2 && split_prec() == 2) {
            const float* fp32_img = p.B;
            p.B = static_cast<const float*>(img_h2);
            p.bscale = h2_descale;
            // (A-ring depth 3: 4 and 5 measured no faster, r05 profiles/r05/pf)
            if (sk_matches<SK_MSG2_H2>(p, NS, NV)) return run_tp<NS, NV, EPI, 8, 3, SK_MSG2_H2>(p, st, tm);
            if (sk_matches<SK_MSG2_32_H2>(p, NS, NV)) return run_tp<NS, NV, EPI, 8, 3, SK_MSG2_32_H2>(p, st, tm);
            p.B = fp32_img;
        }
        if (img_x3 && split_prec() == 1) {
            const float* fp32_img = p.B;
            p.B = static_cast<const float*>(img_x3);
            if (sk_matches<SK_MSG2_X3>(p, NS, NV)) {
                return run_tp<NS, NV, EPI, 8, 3, SK_MSG2_X3>(p, st, tm);
            }
            if (sk_matches<SK_MSG2_32_X3>(p, NS, NV)) return run_tp<NS, NV, EPI, 8, 3, SK_MSG2_32_X3>(p, st, tm);
            p.B = fp32_img;
        }
        if (sk_matches<SK_GATE>(p, NS, NV)) return run_tp<NS, NV, EPI, 8, 3, SK_GATE>(p, st, tm);
        if (sk_matches<SK_GATE_32>(p, NS, NV)) return run_tp<NS, NV, EPI, 8, 3, SK_GATE_32>(p, st, tm);
    }
    return run_tp<NS, NV, EPI, 8, 3>(p, st, tm);
}

template <int NS, int NV, int EPI>
int run_tp_msg(nbx::TpProb& p, hipStream_t st, KernelTiming* tm, const void* img_x3 = nullptr,
               const void* img_h2 = nullptr, float h2_descale = 1.f, bool dv = false) {
    static const bool debug = getenv("NBX_TP_DEBUG") != nullptr;
    if (debug) p.dbg = tp_dbg_buf(st);
    const int rc = run_tp_msg_sel<NS, NV, EPI>(p, st, tm, img_x3, img_h2, h2_descale, dv);
    if (rc || !debug) return rc;
    return tp_debug_dump(p, st, 8);
}


int tp16_debug_dump(const unsigned long long* dbg, int n, hipStream_t st, const char* label) {
    std::vector<unsigned long long> h((size_t)n * 6);
    NBX_HIP(hipStreamSynchronize(st));
    NBX_HIP(hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost));
    double s01 = 0, s12 = 0, s23 = 0, sw = 0;
    unsigned long long w0 = ~0ull, w1 = 0;
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
        const unsigned long long* d = &h[(size_t)i * 6];
        if (!d[1]) continue;
        s01 += d[1] - d[0]; s12 += d[2]; s23 += d[3]; ++cnt;
        w0 = std::min(w0, d[4]);
        w1 = std::max(w1, d[5]);
        sw += (double)(d[5] - d[4]);
    }
    fprintf(stderr,
            "tp_debug %s waves=%d/%d stage=%.0f loop=%.0f epi=%.0f (avg clocks per wave, loop/epi summed over its "
            "tiles) waves_span=%.2fus wave_avg=%.2fus\n",
            label, cnt, n, s01 / std::max(cnt, 1), s12 / std::max(cnt, 1), s23 / std::max(cnt, 1), (w1 - w0) / 100.0,
            sw / std::max(cnt, 1) / 100.0);
    return NBX_OK;
}

template <int NS, int NV, int EPI, int CG, int WAVES, int PF, int KS, class SK = nbx::DynSK>
int run_tp16_w(nbx::TpProb& p, hipStream_t st, KernelTiming* tm) {
    static const bool debug = getenv("NBX_TP_DEBUG") != nullptr;
    if (debug) {
        p.dbg = tp_dbg_buf(st);
        if (int rc = nbx::tp16_launch<NS, NV, EPI, CG, WAVES, PF, KS, SK>(p, st)) return rc;
        int n = ((p.chunks + CG - 1) / CG) * p.blocks_per_chunk * WAVES;
        char lab[32];
        snprintf(lab, sizeof lab, "tp16<%d,%d,%d,%d,KS%d>", NS, NV, EPI, CG, KS);
        return tp16_debug_dump(p.dbg, n, st, lab);
    }
    if (!tm) return nbx::tp16_launch<NS, NV, EPI, CG, WAVES, PF, KS, SK>(p, st);
    hipEvent_t a, b;
    NBX_HIP(hipEventCreate(&a));
    NBX_HIP(hipEventCreate(&b));
    tm->ev.push_back(a);
    tm->ev.push_back(b);
    nbx::armed_events() = {a, b};   // the launch below records the kernel's own begin / end
    if (int rc = nbx::tp16_launch<NS, NV, EPI, CG, WAVES, PF, KS, SK>(p, st)) return rc;
    NBX_HIP(nbx::disarm_events(st));
    double k = 0;
    for (int j = 0; j < NS; ++j) k += p.K[j];
    k += NV ? 3.0 * p.Kv : 0.0;
    constexpr int kind = EPI;
    tm->kind.push_back(kind);
    tm->flops[kind] += 2.0 * p.rows * 16.0 * p.chunks * k;
    tm->launches[kind] += 1;
    return NBX_OK;
}


int run_msg_pre(nbx::MsgPreProb& p, hipStream_t st, KernelTiming* tm) {
    static const bool debug = getenv("NBX_TP_DEBUG") != nullptr;
    if (debug) {
        p.dbg = tp_dbg_buf(st);
        if (int rc = nbx::msg_pre_launch(p, st)) return rc;
        const int n = p.chunks * p.per_chunk * 8;
        std::vector<unsigned long long> h((size_t)n * 4);
        NBX_HIP(hipStreamSynchronize(st));
        NBX_HIP(hipMemcpy(h.data(), p.dbg, h.size() * 8, hipMemcpyDeviceToHost));
        // waves 0-3 of a block run the GEMM, 4-7 the edges: average each counter over its role
        double s[4] = {0, 0, 0, 0}, exg = 0, exe = 0;
        for (int i = 0; i < n; ++i) {
            for (int k = 0; k < 4; ++k) s[k] += (double)h[(size_t)i * 4 + k];
            ((i & 7) < 4 ? exg : exe) += (double)h[(size_t)i * 4 + 2];
        }
        const double half = n / 2.0;
        fprintf(stderr,
                "tp_debug msg_pre waves=%d slabs=%d per_chunk=%d stage=%.0f gemm=%.0f ex(gemm waves)=%.0f edge=%.0f "
                "ex(edge waves)=%.0f (avg clocks per wave of the role)\n",
                n, p.n_slabs, p.per_chunk, s[0] / n, s[1] / half, exg / half, s[3] / half, exe / half);
        return NBX_OK;
    }
    if (!tm) return nbx::msg_pre_launch(p, st);
    hipEvent_t a, b;
    NBX_HIP(hipEventCreate(&a));
    NBX_HIP(hipEventCreate(&b));
    tm->ev.push_back(a);
    tm->ev.push_back(b);
    nbx::armed_events() = {a, b};   // the launch below records the kernel's own begin / end
    if (int rc = nbx::msg_pre_launch(p, st)) return rc;
    NBX_HIP(nbx::disarm_events(st));
    tm->kind.push_back(nbx::TP_PLAIN);   // reported as the message_layer_1 kind
    tm->flops[nbx::TP_PLAIN] += 2.0 * 4.0 * p.V * p.M * 6.0 * p.M;   // the node GEMM's useful MACs x 2
    tm->launches[nbx::TP_PLAIN] += 1;
    return NBX_OK;
}

template <int NS, int NV, int EPI, int CG>
int run_tp16_pair(nbx::TpProb& p0, nbx::TpProb& p1, hipStream_t st, KernelTiming* tm) {
    static const bool debug = getenv("NBX_TP_DEBUG") != nullptr;
    if (debug) {
        p0.dbg = p1.dbg = tp_dbg_buf(st);
        if (int rc = nbx::tp16_launch2<NS, NV, EPI, CG, 8, 3, 1>(p0, p1, st)) return rc;
        const int n = ((p0.chunks + CG - 1) / CG) * p0.blocks_per_chunk * 8;   // first problem's blocks
        return tp16_debug_dump(p0.dbg, n, st, "tp16 node_pre pair (scalar-row part)");
    }
    if (!tm) return nbx::tp16_launch2<NS, NV, EPI, CG, 8, 3, 1>(p0, p1, st);
    hipEvent_t a, b;
    NBX_HIP(hipEventCreate(&a));
    NBX_HIP(hipEventCreate(&b));
    tm->ev.push_back(a);
    tm->ev.push_back(b);
    nbx::armed_events() = {a, b};   // the launch below records the kernel's own begin / end
    if (int rc = nbx::tp16_launch2<NS, NV, EPI, CG, 8, 3, 1>(p0, p1, st)) return rc;
    NBX_HIP(nbx::disarm_events(st));
    for (const nbx::TpProb* p : {&p0, &p1}) {
        double k = 0;
        for (int j = 0; j < NS; ++j) k += p->K[j];
        k += NV ? 3.0 * p->Kv : 0.0;
        tm->flops[EPI] += 2.0 * p->rows * 16.0 * p->chunks * k;
    }
    tm->kind.push_back(EPI);
    tm->launches[EPI] += 1;
    return NBX_OK;
}

// KS > 1 splits each row tile's K loop over KS waves of the block (partials folded through
// LDS before the epilogue).  Measured on MI355X at C2: it pays only for update_layer_2
// (30 -> 24 us); the other node TPs lose to the extra block rounds.
template <int NS, int NV, int EPI, int CG, int KS, class SK, class... Rest>
int run_tp16_try(nbx::TpProb& p, hipStream_t st, KernelTiming* tm) {
    if (static_enabled() && sk_matches<SK>(p, NS, NV)) return run_tp16_w<NS, NV, EPI, CG, 8, 3, KS, SK>(p, st, tm);
    if constexpr (sizeof...(Rest) > 0) return run_tp16_try<NS, NV, EPI, CG, KS, Rest...>(p, st, tm);
    else return run_tp16_w<NS, NV, EPI, CG, 8, 3, KS, nbx::DynSK>(p, st, tm);
}

nbx::TpProb tp_base(int rows, const Dims& d) {
    nbx::TpProb p;
    memset(&p, 0, sizeof(p));
    p.rows = rows;
    p.M = d.M;
    p.chunks = d.chunks;
    return p;
}

// A general (non fully-connected) graph as slot tables in the workspace (ws.SLOT / ws.DEG),
// `edges` real edges in total.
struct GraphSlots {
    double edges;
    bool regular;   // every node is the source of the same number of edges (a kNN graph): SyncBN can scale counts
};

int forward_impl(const nbx_segnn_weights* w, const float* pos, const float* vel, const float* mass, int64_t B,
                 int64_t N, float* out, const Workspace& ws, hipStream_t st, KernelTiming* tm = nullptr,
                 const RolloutUpdate* upd = nullptr, bool featurized = false, const GraphSlots* gr = nullptr) {
    const int M = w->mul;
    const Dims d = dims_of(B, N, M);
    const int64_t V = d.V, Ep = d.Ep;
    const dim3 ewb(EW_X, EW_Y);
    // every tensor-product problem of the forward raises the call's fp16x2 range flag
    auto tp_flagged = [&](int rows, const Dims& dd) {
        nbx::TpProb p = tp_base(rows, dd);
        p.range_flag = ws.RANGE;
        return p;
    };


    // update_layer_1 reads its [x | BN(agg)] input straight from X / AGG and the two dot buffers
    // (no materialised U1) when the static segmented schedule applies (mul = 96 or 32)
    // (general graphs: the segmented input folds the message BN shift x a constant degree, so
    // they take the materialised path with per-node in-degrees)
    const bool seg_upd = static_enabled() && (M == 96 || M == 32) && !gr;
    const bool dv_upd = upd_dv(w, M, seg_upd);   // x_v . na / a_v . na formed in registers, XD / AD unused
    const int* slot = gr ? ws.SLOT : nullptr;
    const float* degv = gr ? ws.DEG : nullptr;
    // block: whole multiples of the channel count (192 threads at mul = 96), >= FE_NODES
    const unsigned fe_threads = (unsigned)std::max(64, std::min(1024, M * std::max(1, 256 / M)));
    // Lazy feature BatchNorm: X in HBM holds each layer's pre-normalisation output and its
    // consumers in the next layer (message_layer_1, the update inputs, the residual) apply
    // the pending per-channel scale/shift (ws.coef_feat) as they read it; null = identity.
    const bool fused_msg = N > 1 && nbx::msg_pre_group((int)N) > 0 && M <= 128;
    // atomic BatchNorm statistics: the message BN is finalised by update_layer_1 (segmented input),
    // the feature BN of layers 0..L-2 by the next layer's message_layer_1, the last layer's by
    // pre_pool1 (segmented input); the sums are zeroed by the featurising kernel of the forward
    // consumer-finalised BatchNorm (the segmented path): the producers' sums land in a [3][M] slot per
    // BN instance, by fp64 atomics (default) or, deterministic, as partial rows summed in a fixed order
    // by bn_reduce_kernel (one small launch per BN instance)
    const bool bn_slot = fused_msg && seg_upd && (w->deterministic || bn_atomic_enabled());
    const bool bn_atomic = bn_slot && !w->deterministic;
    auto sums_of = [&](int l, int kind) { return ws.bn_sums + ((size_t)2 * l + kind) * 3 * M; };
    // SyncBN (w->bn_comm: an RCCL all-reduce the library enqueues itself; or the w->bn_allreduce hook):
    // the batch statistics are summed over every rank between the producing kernel and the finalising
    // consumer, and normalised by the global counts
    const bool sync = (w->bn_comm != nullptr || w->bn_allreduce != nullptr) && w->training;
    const int64_t Bg = sync && w->bn_global_batch > 0 ? w->bn_global_batch : B;
    // general graphs: the real edge count (a kNN rollout's V k scales to the global batch under SyncBN)
    const double cnt_nodes = (double)(Bg * N);
    const double cnt_edges = gr ? gr->edges * ((double)Bg / (double)B) : (double)(Bg * N * (N - 1));
    if (sync && gr && !gr->regular) {
        nbx::set_error("segnn: SyncBN over a general edge_index needs a regular (kNN) graph");
        return NBX_E_UNSUPPORTED;
    }
    auto sync_bn = [&](double* sums) -> int {
        if (!sync) return NBX_OK;
        if (w->bn_comm) return nbx::comm_allreduce_f64(sums, (int64_t)3 * M, w->bn_comm, st);
        if (w->bn_allreduce(sums, (int64_t)3 * M, (void*)st, w->bn_allreduce_ctx) != 0) {
            nbx::set_error("segnn: bn_allreduce hook failed");
            return NBX_E_HIP;
        }
        return NBX_OK;
    };
    // non-atomic sums of the slot or general-graph paths: partial rows -> fixed-order reduction ->
    // (SyncBN) all-reduce
    auto reduce_sums = [&](int wpc, int cw, double* sums) -> int {
        hipLaunchKernelGGL(bn_reduce_kernel, dim3((unsigned)nbx::ceil_div(M, cw)), dim3(BNF_THREADS), 0, st,
                           ws.partial, wpc, cw, M, sums);
        NBX_LAUNCH_CHECK("bn_reduce");
        return sync_bn(sums);
    };
    // general-graph / non-segmented path under SyncBN: reduce, all-reduce, coefficients from the sums
    auto finalize_sync = [&](int wpc, int cw, double* sums, const nbx::BnSrc& src) -> int {
        if (int rc = reduce_sums(wpc, cw, sums)) return rc;
        hipLaunchKernelGGL(bn_coef_kernel, dim3((unsigned)nbx::ceil_div(3 * M, 256)), dim3(256), 0, st, src, M);
        NBX_LAUNCH_CHECK("bn_coef");
        return NBX_OK;
    };
    // (featurized: the previous rollout_pp2_kernel zeroed them)
    const int nzero = bn_atomic ? 2 * w->num_layers * 3 * M : 0;
    // (featurized: a rollout's previous rollout_pp2_kernel already wrote NA / EG / X / XD)
    if (!featurized) {
        hipLaunchKernelGGL(featurize_embed_kernel, dim3((unsigned)nbx::ceil_div(V, FE_NODES)), dim3(fe_threads), 0, st,
                           pos, vel, mass, V, (int)N, (int)d.G, w->emb, w->emb_bias, M, ws.NA, ws.EG, ws.X,
                           seg_upd && !dv_upd ? ws.XD : nullptr, ws.bn_sums, nzero, slot, degv,
                           upd == nullptr || upd->frame <= 1 ? ws.RANGE : nullptr);
        NBX_LAUNCH_CHECK("embed");
    }

    for (int l = 0; l < w->num_layers; ++l) {
        const nbx_segnn_layer& L = w->layers[l];
        const float* xprev = l > 0 ? ws.coef_feat : nullptr;
        if (xprev && !fused_msg && N > 1) {
            // the unfused message path reads X directly: normalise it in place first
            hipLaunchKernelGGL(bn_apply_kernel, ew_grid(V, M), ewb, 0, st, ws.X, ws.coef_feat, V, M,
                               seg_upd && !dv_upd ? ws.XD : nullptr);
            NBX_LAUNCH_CHECK("bn_apply");
            xprev = nullptr;
        }
        const bool msg2_dv = msg_dv(M, N, L.msg2_img_h2 != nullptr);
        // update_layer_2 forms the [h_v . na] half of its scalar operand from U2V (TpStream DV), so
        // update_layer_1's gate epilogue skips writing it (same switch as dv_upd)
        const bool upd2_dv = dv_upd && L.upd2_img_h2 != nullptr;
        if (fused_msg) {
            // message_layer_1: node precomputation + edge combination + gate in one kernel
            nbx::MsgPreProb mp;
            memset(&mp, 0, sizeof(mp));
            mp.X = ws.X; mp.Simg = L.node_pre_s_img; mp.Vimg = L.node_pre_v_img; mp.EG = ws.EG;
            mp.amf = L.msg1_amf; mp.bias = L.msg1_bias; mp.M1S = ws.M1S; mp.M1V = ws.M1V; mp.xcoef = xprev;
            mp.V = V; mp.N = (int)N; mp.G = (int)d.G; mp.M = M; mp.NG = nbx::msg_pre_group((int)N);
            mp.slot = slot;
            if (bn_slot && l > 0) {
                const nbx_segnn_layer& Lp = w->layers[l - 1];
                mp.xbn = nbx::BnSrc{sums_of(l - 1, 1), Lp.feat_bn_weight, Lp.feat_bn_bias, Lp.feat_bn_running_mean,
                                    Lp.feat_bn_running_var, ws.coef_feat, cnt_nodes, w->bn_eps, w->bn_momentum,
                                    w->training, 1};
            }
            // split-precision node GEMM when its two bf16x3 images and the exchange buffers fit the
            // LDS (mul <= 96); wider layers run the fp32 MFMA node GEMM
            if (L.node_pre_s_img_h2 && L.node_pre_v_img_h2 && split_prec() == 2 && M <= 96) {
                mp.Simg = static_cast<const float*>(L.node_pre_s_img_h2);
                mp.Vimg = static_cast<const float*>(L.node_pre_v_img_h2);
                mp.prec = 2;
                mp.bscale = L.node_pre_h2_descale;
            } else if (L.node_pre_s_img_x3 && L.node_pre_v_img_x3 && split_prec() == 1 && M <= 96) {
                mp.Simg = static_cast<const float*>(L.node_pre_s_img_x3);
                mp.Vimg = static_cast<const float*>(L.node_pre_v_img_x3);
                mp.prec = 1;
            }
            mp.no_dot = msg2_dv ? 1 : 0;
            mp.range_flag = ws.RANGE;
            if (int rc = run_msg_pre(mp, st, tm)) return rc;
        } else if (N > 1) {
            // systems larger than a 16-row tile: node precomputation (plain GEMM, part-major
            // columns of NP: parts 0-2 and 3-5 of the 6-part image in two paired launches), then
            // the per-edge combination
            const int KC = (M + 31) / 32, F6 = 6 * KC * 512;
            for (int half = 0; half < 2; ++half) {
                nbx::TpProb pp[2];
                for (int part = 0; part < 2; ++part) {
                    nbx::TpProb& p = pp[part];
                    p = tp_flagged(part == 0 ? (int)V : (int)(3 * V), d);
                    p.As = ws.X + (part ? V * M : 0);
                    p.lda_s = M;
                    p.B = (part ? L.node_pre_v_img : L.node_pre_s_img) + half * 3 * KC * 512;
                    p.img_stride = F6;
                    p.K[0] = p.K[1] = p.K[2] = M;
                    p.chunks = (M + 15) / 16;
                    p.col_part_stride = M;
                    p.col_part0 = 3 * half;
                    p.C = ws.NP + (part ? V * 6 * M : 0);
                    p.ldc = 6 * M;
                    p.ncols = 6 * M;
                }
                if (int rc = run_tp16_pair<3, 0, nbx::TP_PLAIN, 2>(pp[0], pp[1], st, tm)) return rc;
            }
            hipLaunchKernelGGL(msg1_kernel, ew_grid(Ep, M), ewb, 0, st, ws.NP, ws.EG, L.msg1_amf, L.msg1_bias, V,
                               (int)N, (int)d.G, M, ws.M1S, ws.M1V, slot);
            NBX_LAUNCH_CHECK("msg1");
        }
        int wpc_msg = 1, cw_msg = 16;
        {
            // message_layer_2 + gate + aggregation + message-BN partial sums
            nbx::TpProb p = tp_flagged((int)Ep, d);
            p.As = ws.M1S; p.lda_s = 2 * M; p.B = L.msg2_img;
            p.K[0] = 2 * M; p.K[1] = 2 * M; p.K[2] = M;
            p.Av = ws.M1V; p.lda_v = M; p.plane_stride = Ep * M; p.Kv = M;
            p.bias = L.msg2_bias; p.geom = ws.EG; p.group = (int)d.G;
            p.valid_per_group = gr ? (int)d.G : (int)(N - 1);   // general graphs: padding rows have |rel| < 0
            p.out_s = ws.AGG; p.out_v = ws.AGG + V * M; p.out_plane = V * M; p.partial = ws.partial;
            if (seg_upd && !dv_upd) { p.na = ws.NA; p.out_dot = ws.AD; }
            if (bn_atomic) p.bn_sums = sums_of(l, 0);
            if (N > 1) {  // 32x32 tiles: edge rows are plentiful, and a tile holds whole destinations
                if (int rc = run_tp_msg<3, 1, nbx::TP_MSG>(p, st, tm, L.msg2_img_x3, L.msg2_img_h2, L.msg2_h2_descale,
                                                           msg2_dv))
                    return rc;
                wpc_msg = p.waves_per_chunk;
                cw_msg = 32;
                if (bn_atomic) {
                    if (int rc = sync_bn(sums_of(l, 0))) return rc;
                } else if (bn_slot) {
                    if (int rc = reduce_sums(wpc_msg, cw_msg, sums_of(l, 0))) return rc;
                }
            } else {
                NBX_HIP(hipMemsetAsync(ws.AGG, 0, sizeof(float) * 4 * V * M, st));
                NBX_HIP(hipMemsetAsync(ws.AD, 0, sizeof(float) * V * M, st));
                NBX_HIP(hipMemsetAsync(ws.partial, 0, sizeof(double) * 48 * ((M + 15) / 16), st));
            }
        }
        if (!bn_slot && sync) {
            if (int rc = finalize_sync(wpc_msg, cw_msg, sums_of(l, 0),
                                       nbx::BnSrc{sums_of(l, 0), L.msg_bn_weight, L.msg_bn_bias, L.msg_bn_running_mean,
                                                  L.msg_bn_running_var, ws.coef_msg, std::max(1.0, cnt_edges),
                                                  w->bn_eps, w->bn_momentum, w->training, 1}))
                return rc;
        } else if (!bn_slot) {
            hipLaunchKernelGGL(bn_finalize_kernel, dim3((unsigned)nbx::ceil_div(M, cw_msg)), dim3(BNF_THREADS), 0, st,
                               ws.partial, wpc_msg, cw_msg, std::max(1.0, cnt_edges), M, w->training,
                               w->bn_eps, w->bn_momentum, L.msg_bn_weight, L.msg_bn_bias, L.msg_bn_running_mean,
                               L.msg_bn_running_var, ws.coef_msg);
            NBX_LAUNCH_CHECK("bn_finalize(msg)");
        }
        if (seg_upd) {
            // update_layer_1 + gate, input segments [x_s | a_s | x_v.na | a_v.na] and [x_v | a_v]
            // read from X / AGG / XD / AD with the pending feature BN and the message BN applied
            // per (segment, channel) as the A chunks are consumed
            nbx::TpProb p = tp_flagged((int)V, d);
            p.K[0] = 4 * M; p.K[1] = 4 * M; p.K[2] = 2 * M; p.Kv = 2 * M;
            p.lda_s = 4 * M; p.lda_v = 2 * M;
            p.seg_s[0] = ws.X; p.seg_s[1] = ws.AGG; p.seg_s[2] = ws.XD; p.seg_s[3] = ws.AD;
            p.seg_v[0] = ws.X + V * M; p.seg_v[1] = ws.AGG + V * M; p.seg_vplane = V * M;
            p.xcoef = xprev; p.mcoef = ws.coef_msg; p.deg = (float)(N - 1);
            if (bn_slot)
                p.mbn = nbx::BnSrc{sums_of(l, 0), L.msg_bn_weight, L.msg_bn_bias, L.msg_bn_running_mean,
                                   L.msg_bn_running_var, ws.coef_msg, cnt_edges, w->bn_eps,
                                   w->bn_momentum, w->training, 1};
            p.B = L.upd1_img;
            p.bias = L.upd1_bias; p.geom = ws.NA; p.out_s = ws.U2S; p.out_v = ws.U2V; p.out_plane = V * M;
            p.chunks = (M + 15) / 16;
            p.skip_gate_dot = upd2_dv ? 1 : 0;
            if ((M == 96 || M == 32) && L.upd1_img_h2 && split_prec() == 2) {
                p.B = static_cast<const float*>(L.upd1_img_h2);
                p.bscale = L.upd1_h2_descale;
                // (A-ring depth 3: 5 and 7 measured slower, r05 profiles/r05/pf)
                // (r06 A/B, profiles/r06/upd_variants: two 16-channel chunks per 4-wave block, ring 3 or 5,
                // 17.5-18.1 us against 17.8 us and fewer steps/s -- the single-tile latency chain, not the
                // 6x L2 re-read, bounds this kernel)
                const int rc =
                    dv_upd ? (M == 96 ? run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_UPD1_SEG_H2_DV>(p, st, tm)
                                        : run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_UPD1_32_SEG_H2_DV>(p, st, tm))
                    : M == 96 ? run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_UPD1_SEG_H2>(p, st, tm)
                              : run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_UPD1_32_SEG_H2>(p, st, tm);
                if (rc) return rc;
            } else if (dv_upd) {   // (upd_dv implies the branch above; XD / AD were not written)
                nbx::set_error("segnn: internal: register-dot update_layer_1 decision without its schedule");
                return NBX_E_INVAL;
            } else if (M == 96 && L.upd1_img_x3 && split_prec() == 1) {
                p.B = static_cast<const float*>(L.upd1_img_x3);
                if (int rc = run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_UPD1_SEG_X3>(p, st, tm)) return rc;
            } else if (M == 96) {
                if (int rc = run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_UPD1_SEG>(p, st, tm)) return rc;
            } else {
                if (int rc = run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_UPD1_32_SEG>(p, st, tm)) return rc;
            }
        } else {
            hipLaunchKernelGGL(upd_pre_kernel, ew_grid(V, M), ewb, 0, st, ws.X, ws.AGG, ws.NA, ws.coef_msg, xprev,
                               (float)(N - 1), V, M, ws.U1S, ws.U1V, degv);
            NBX_LAUNCH_CHECK("upd_pre");
            {
                // update_layer_1 + gate -> inputs of update_layer_2
                nbx::TpProb p = tp_flagged((int)V, d);
                p.As = ws.U1S; p.lda_s = 4 * M; p.B = L.upd1_img;
                p.K[0] = 4 * M; p.K[1] = 4 * M; p.K[2] = 2 * M;
                p.Av = ws.U1V; p.lda_v = 2 * M; p.plane_stride = V * 2 * M;
                p.Kv = 2 * M;
                p.bias = L.upd1_bias; p.geom = ws.NA; p.out_s = ws.U2S; p.out_v = ws.U2V; p.out_plane = V * M;
                p.chunks = (M + 15) / 16;
                if (int rc = run_tp16_try<3, 1, nbx::TP_GATE_NODE, 1, 1, SK_UPD1, SK_UPD1_32>(p, st, tm)) return rc;
            }
        }
        int wpc_feat;
        {
            // update_layer_2 + residual + feature-BN partial sums
            nbx::TpProb p = tp_flagged((int)V, d);
            p.As = ws.U2S; p.lda_s = 2 * M; p.B = L.upd2_img;
            p.K[0] = 2 * M; p.K[1] = M;
            p.Av = ws.U2V; p.lda_v = M; p.plane_stride = V * M; p.Kv = M;
            p.bias = L.upd2_bias; p.geom = ws.NA; p.out_s = ws.X; p.out_v = ws.X + V * M; p.out_plane = V * M;
            p.partial = ws.partial;
            const bool feat_atomic = bn_atomic;
            if (feat_atomic) p.bn_sums = sums_of(l, 1);
            p.xcoef = xprev;
            if (seg_upd && !dv_upd) { p.out_dot = ws.XD; }
            p.chunks = (M + 15) / 16;
            // update_layer_2: one 16-channel chunk per wave, full K (CG 1, KS 1; r02 measured it against
            // CG 2 / KS 2, CG 1 / KS 2, CG 2 / KS 1, CG 1 / KS 4: 15.1 vs 17.8 / 16.3 / 19.5 / 20.9 us)
            if ((M == 96 || M == 32) && L.upd2_img_h2 && split_prec() == 2 && static_enabled()) {
                p.B = static_cast<const float*>(L.upd2_img_h2);
                p.bscale = L.upd2_h2_descale;
                // (r06 A/B, profiles/r06/upd_variants: CG 2 / 4 waves with ring 3 or 5: 12.3-12.4 us against
                // 11.5 us; CG 3 / 2 waves needs a 144-thread BN reduction and was not kept)
                const int rc =
                    upd2_dv ? (M == 96 ? run_tp16_w<2, 1, nbx::TP_RESID, 1, 8, 3, 1, SK_UPD2_H2_DV>(p, st, tm)
                                       : run_tp16_w<2, 1, nbx::TP_RESID, 1, 8, 3, 1, SK_UPD2_32_H2_DV>(p, st, tm))
                    : M == 96 ? run_tp16_w<2, 1, nbx::TP_RESID, 1, 8, 3, 1, SK_UPD2_H2>(p, st, tm)
                              : run_tp16_w<2, 1, nbx::TP_RESID, 1, 8, 3, 1, SK_UPD2_32_H2>(p, st, tm);
                if (rc) return rc;
            } else if (upd2_dv) {   // (update_layer_1 skipped the [h_v . na] half this consumer would read)
                nbx::set_error("segnn: internal: register-dot update_layer_2 decision without its schedule");
                return NBX_E_INVAL;
            } else {
                if (int rc = run_tp16_try<2, 1, nbx::TP_RESID, 1, 1, SK_UPD2, SK_UPD2_32>(p, st, tm)) return rc;
            }
            wpc_feat = p.waves_per_chunk;
            if (bn_atomic) {
                if (int rc = sync_bn(sums_of(l, 1))) return rc;
            } else if (bn_slot) {
                if (int rc = reduce_sums(wpc_feat, 16, sums_of(l, 1))) return rc;
            }
        }
        if (!bn_slot && sync) {
            if (int rc = finalize_sync(wpc_feat, 16, sums_of(l, 1),
                                       nbx::BnSrc{sums_of(l, 1), L.feat_bn_weight, L.feat_bn_bias,
                                                  L.feat_bn_running_mean, L.feat_bn_running_var, ws.coef_feat,
                                                  cnt_nodes, w->bn_eps, w->bn_momentum, w->training, 1}))
                return rc;
        } else if (!bn_slot) {
            hipLaunchKernelGGL(bn_finalize_kernel, dim3((unsigned)nbx::ceil_div(M, 16)), dim3(BNF_THREADS), 0, st,
                               ws.partial, wpc_feat, 16, (double)V, M, w->training, w->bn_eps, w->bn_momentum,
                               L.feat_bn_weight, L.feat_bn_bias, L.feat_bn_running_mean, L.feat_bn_running_var,
                               ws.coef_feat);
        }
    }

    // pre_pool1 (gate TP) and pre_pool2 (-> 2x1o)
    // pre_pool1 inputs with the last layer's pending feature BatchNorm applied: read segment by
    // segment from X and XD (x_v . na) with the scale / shift applied as the A chunks are consumed
    // (static schedules at mul 96 / 32), else materialised by pp_pre_kernel
    if (seg_upd) {
        nbx::TpProb p = tp_flagged((int)V, d);
        p.K[0] = 2 * M; p.K[1] = 2 * M; p.K[2] = M; p.Kv = M;
        p.lda_s = 2 * M; p.lda_v = M;
        p.seg_s[0] = ws.X; p.seg_s[1] = ws.XD; p.seg_v[0] = ws.X + V * M; p.seg_vplane = V * M;
        p.xcoef = w->num_layers > 0 ? ws.coef_feat : nullptr;
        if (bn_slot && w->num_layers > 0) {
            const nbx_segnn_layer& Lp = w->layers[w->num_layers - 1];
            p.xbn = nbx::BnSrc{sums_of(w->num_layers - 1, 1), Lp.feat_bn_weight, Lp.feat_bn_bias,
                               Lp.feat_bn_running_mean, Lp.feat_bn_running_var, ws.coef_feat, cnt_nodes, w->bn_eps,
                               w->bn_momentum, w->training, 1};
        }
        p.B = w->pp1_img;
        p.bias = w->pp1_bias; p.geom = ws.NA; p.out_s = ws.U2S; p.out_v = ws.U2V; p.out_plane = V * M;
        p.chunks = (M + 15) / 16;
        p.skip_gate_dot = 1;   // pre_pool2 (pp2_node) reads only the h_s half of U2S
        if (w->pp1_img_h2 && split_prec() == 2) {
            p.B = static_cast<const float*>(w->pp1_img_h2);
            p.bscale = w->pp1_h2_descale;
            const int rc =
                dv_upd ? (M == 96 ? run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_PP1_SEG_H2_DV>(p, st, tm)
                                  : run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_PP1_32_SEG_H2_DV>(p, st, tm))
                : M == 96 ? run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_PP1_SEG_H2>(p, st, tm)
                          : run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_PP1_32_SEG_H2>(p, st, tm);
            if (rc) return rc;
        } else if (dv_upd) {   // (upd_dv implies the branch above; XD was not written)
            nbx::set_error("segnn: internal: register-dot pre_pool1 decision without its schedule");
            return NBX_E_INVAL;
        } else if (M == 96) {
            if (int rc = run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_PP1_SEG>(p, st, tm)) return rc;
        } else {
            if (int rc = run_tp16_w<3, 1, nbx::TP_GATE_NODE, 1, 8, 3, 1, SK_PP1_32_SEG>(p, st, tm)) return rc;
        }
    } else {
    hipLaunchKernelGGL(pp_pre_kernel, ew_grid(V, M), ewb, 0, st, ws.X, ws.NA,
                       w->num_layers > 0 ? ws.coef_feat : nullptr, V, M, ws.U1S, ws.U1V);
    {
        nbx::TpProb p = tp_flagged((int)V, d);
        p.As = ws.U1S; p.lda_s = 2 * M; p.B = w->pp1_img;
        p.K[0] = 2 * M; p.K[1] = 2 * M; p.K[2] = M;
        p.Av = ws.U1V; p.lda_v = M; p.plane_stride = V * M; p.Kv = M;
        p.bias = w->pp1_bias; p.geom = ws.NA; p.out_s = ws.U2S; p.out_v = ws.U2V; p.out_plane = V * M;
        p.chunks = (M + 15) / 16;
        // pre_pool1: CG 1 / KS 1 (r02: CG 2 measured -0.8 % step time)
        if (int rc = run_tp16_try<3, 1, nbx::TP_GATE_NODE, 1, 1, SK_GATE, SK_GATE_32>(p, st, tm)) return rc;
    }
    }
    if (upd && upd->featurize_next && !gr) {
        const int nb = (int)N * std::max(1, 8 / (int)N);   // whole systems, N <= RPP2_MAX
        hipLaunchKernelGGL(rollout_pp2_kernel, dim3((unsigned)nbx::ceil_div(V, nb)), dim3(64 * nb), 0, st, ws.U2S,
                           ws.U2V, ws.NA, w->pp2, V, M, out, *upd, nb, mass, (int)N, (int)d.G, w->emb, w->emb_bias,
                           ws.EG, ws.X, seg_upd && !dv_upd ? ws.XD : nullptr, ws.bn_sums, nzero);
        NBX_LAUNCH_CHECK("pre_pool2 + next featurise");
        return NBX_OK;
    }
    RolloutUpdate none{};
    hipLaunchKernelGGL(pp2_kernel, dim3((unsigned)nbx::ceil_div(V, 4)), dim3(256), 0, st, ws.U2S, ws.U2V, ws.NA,
                       w->pp2, V, M, out, upd ? *upd : none);
    NBX_LAUNCH_CHECK("pre_pool2");
    return NBX_OK;
}

int prepare(const nbx_segnn_weights* w, int64_t B, int64_t N, void* workspace, size_t bytes, Workspace* ws) {
    if (int rc = check_weights(w)) return rc;
    NBX_CHECK_ARG(B >= 1 && N >= 1, "segnn: need B >= 1 and N >= 1");
    NBX_CHECK_ARG(N <= 33, "segnn: native path supports systems of at most 33 nodes (got %lld)", (long long)N);
    NBX_CHECK_ARG(B * N * 32 < (int64_t)1 << 30, "segnn: graph too large");
    const size_t need = carve(ws, workspace, B, N, w->mul);
    if (bytes < need || workspace == nullptr) {
        nbx::set_error("segnn: workspace too small (%zu < %zu bytes)", bytes, need);
        return NBX_E_WORKSPACE;
    }
    return NBX_OK;
}

}  // namespace

extern "C" int nbx_segnn_workspace_bytes(int64_t B, int64_t N, int32_t mul, size_t* bytes) {
    NBX_CHECK_ARG(bytes != nullptr && B >= 1 && N >= 1 && mul > 0, "nbx_segnn_workspace_bytes: bad arguments");
    *bytes = carve(nullptr, nullptr, B, N, mul);
    return NBX_OK;
}

extern "C" int nbx_segnn_forward(const nbx_segnn_weights* w, const float* pos, const float* vel, const float* mass,
                                 int64_t B, int64_t N, float* out, void* workspace, size_t workspace_bytes,
                                 void* stream) {
    Workspace ws;
    if (int rc = prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    return forward_impl(w, pos, vel, mass, B, N, out, ws, (hipStream_t)stream);
}

extern "C" int nbx_segnn_rollout(const nbx_segnn_weights* w, float* pos, float* vel, const float* mass, int64_t B,
                                 int64_t N, int64_t num_frames, int32_t flags, float* traj_pos, float* traj_vel,
                                 void* workspace, size_t workspace_bytes, void* stream) {
    Workspace ws;
    if (int rc = prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    NBX_CHECK_ARG(num_frames >= 1, "nbx_segnn_rollout: num_frames must be >= 1");
    hipStream_t st = (hipStream_t)stream;
    const int64_t V = B * N;
    const unsigned ub = (unsigned)nbx::ceil_div(V * 3, 256);
    hipLaunchKernelGGL(rollout_update_kernel, dim3(ub), dim3(256), 0, st, pos, vel, ws.out, V, (int)N, (int64_t)0,
                       num_frames, traj_pos, traj_vel);
    NBX_LAUNCH_CHECK("rollout_update");
    // whole systems per rollout_pp2_kernel block: the next frame's featurisation fused into pre_pool2
    const bool fuse = N <= RPP2_MAX;
    for (int64_t f = 1; f < num_frames; ++f) {
        // the state update + trajectory write of frame f is fused into pre_pool2's epilogue, and
        // (fuse) so is the featurisation of frame f + 1's input
        const RolloutUpdate upd{pos, vel, traj_pos, traj_vel, f, num_frames, (int)N, fuse && f + 1 < num_frames,
                                (flags & NBX_ROLLOUT_ABSOLUTE) ? 1 : 0};
        if (int rc = forward_impl(w, pos, vel, mass, B, N, ws.out, ws, st, nullptr, &upd, fuse && f >= 2)) return rc;
    }
    return NBX_OK;
}

namespace {

// Slot tables of a graph given as an edge_index (validated; one host synchronisation) or as the
// kNN graph of the current positions (csrc/graph.hip).
int slots_from_edges(const int64_t* ei, int64_t E, int64_t B, int64_t N, const Workspace& ws, hipStream_t st) {
    const Dims d = dims_of(B, N, 4);
    return nbx::graph_slots_from_edges(ei, E, d.V, (int)N, (int)d.G, ws.ADJ, ws.SLOT, ws.DEG, ws.ERR, st);
}

int slots_from_knn(const float* pos, int64_t B, int64_t N, int k, const Workspace& ws, hipStream_t st) {
    const Dims d = dims_of(B, N, 4);
    return nbx::graph_slots_from_knn(pos, d.V, (int)N, (int)d.G, k, ws.ADJ, ws.SLOT, ws.DEG, ws.ERR, st);
}

}  // namespace

extern "C" int nbx_segnn_forward_graph(const nbx_segnn_weights* w, const float* pos, const float* vel,
                                       const float* mass, int64_t B, int64_t N, const int64_t* edge_index,
                                       int64_t num_edges, float* out, void* workspace, size_t workspace_bytes,
                                       void* stream) {
    Workspace ws;
    if (int rc = prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    NBX_CHECK_ARG(num_edges >= 1 && edge_index != nullptr, "nbx_segnn_forward_graph: need at least one edge");
    hipStream_t st = (hipStream_t)stream;
    if (int rc = slots_from_edges(edge_index, num_edges, B, N, ws, st)) return rc;
    const GraphSlots gr{(double)num_edges, false};
    return forward_impl(w, pos, vel, mass, B, N, out, ws, st, nullptr, nullptr, false, &gr);
}

extern "C" int nbx_segnn_rollout_knn(const nbx_segnn_weights* w, float* pos, float* vel, const float* mass, int64_t B,
                                     int64_t N, int64_t num_frames, int32_t flags, int64_t num_neighbors,
                                     float* traj_pos, float* traj_vel, void* workspace, size_t workspace_bytes,
                                     void* stream) {
    if (num_neighbors < 0) num_neighbors = N - 1;   // the reference's None
    NBX_CHECK_ARG(num_neighbors < N, "Graph cannot have more neighbors than there are nodes in simulation - 1");
    if (num_neighbors == N - 1)   // build_graph_with_knn returns the fully-connected pattern
        return nbx_segnn_rollout(w, pos, vel, mass, B, N, num_frames, flags, traj_pos, traj_vel, workspace,
                                 workspace_bytes, stream);
    NBX_CHECK_ARG(num_neighbors >= 1, "nbx_segnn_rollout_knn: num_neighbors must be >= 1");
    Workspace ws;
    if (int rc = prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    NBX_CHECK_ARG(num_frames >= 1, "nbx_segnn_rollout_knn: num_frames must be >= 1");
    hipStream_t st = (hipStream_t)stream;
    const int64_t V = B * N;
    hipLaunchKernelGGL(rollout_update_kernel, dim3((unsigned)nbx::ceil_div(V * 3, 256)), dim3(256), 0, st, pos, vel,
                       ws.out, V, (int)N, (int64_t)0, num_frames, traj_pos, traj_vel);
    NBX_LAUNCH_CHECK("rollout_update");
    const GraphSlots gr{(double)(V * num_neighbors), true};
    for (int64_t f = 1; f < num_frames; ++f) {
        // the graph is rebuilt from each frame's positions (infer_self_feed.py:121-123)
        if (int rc = slots_from_knn(pos, B, N, (int)num_neighbors, ws, st)) return rc;
        const RolloutUpdate upd{pos, vel, traj_pos, traj_vel, f, num_frames, (int)N, 0,
                                (flags & NBX_ROLLOUT_ABSOLUTE) ? 1 : 0};
        if (int rc = forward_impl(w, pos, vel, mass, B, N, ws.out, ws, st, nullptr, &upd, false, &gr)) return rc;
    }
    return NBX_OK;
}

extern "C" int nbx_segnn_range_check(const void* workspace, size_t workspace_bytes, int64_t B, int64_t N, int32_t mul,
                                     void* stream) {
    NBX_CHECK_ARG(workspace != nullptr && B >= 1 && N >= 1 && mul > 0, "nbx_segnn_range_check: bad arguments");
    Workspace ws;
    const size_t need = carve(&ws, const_cast<void*>(workspace), B, N, mul);
    NBX_CHECK_ARG(workspace_bytes >= need, "nbx_segnn_range_check: workspace too small (%zu < %zu bytes)",
                  workspace_bytes, need);
    int flag = 0;
    NBX_HIP(hipMemcpyAsync(&flag, ws.RANGE, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
    NBX_HIP(hipStreamSynchronize((hipStream_t)stream));
    if (flag) {
        nbx::set_error("segnn: a tensor-product operand left the fp16 range of the fp16x2 split path (|a| >= 65520) "
                       "or the input is not finite; the bf16x3 path (NBX_SPLIT=x3) keeps the fp32 exponent range");
        return NBX_E_RANGE;
    }
    return NBX_OK;
}

extern "C" int nbx_segnn_forward_timed(const nbx_segnn_weights* w, const float* pos, const float* vel,
                                       const float* mass, int64_t B, int64_t N, float* out, void* workspace,
                                       size_t workspace_bytes, void* stream, float* kind_ms, int32_t* kind_launches,
                                       double* kind_flops, float* total_ms) {
    Workspace ws;
    if (int rc = prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    hipStream_t st = (hipStream_t)stream;
    KernelTiming tm;
    hipEvent_t t0, t1;
    NBX_HIP(hipEventCreate(&t0));
    NBX_HIP(hipEventCreate(&t1));
    NBX_HIP(hipEventRecord(t0, st));
    int rc = forward_impl(w, pos, vel, mass, B, N, out, ws, st, &tm);
    NBX_HIP(hipEventRecord(t1, st));
    NBX_HIP(hipEventSynchronize(t1));
    float acc[4] = {0, 0, 0, 0};
    for (size_t i = 0; i + 1 < tm.ev.size(); i += 2) {
        float ms = 0.f;
        NBX_HIP(hipEventElapsedTime(&ms, tm.ev[i], tm.ev[i + 1]));
        acc[tm.kind[i / 2]] += ms;
    }
    float tot = 0.f;
    NBX_HIP(hipEventElapsedTime(&tot, t0, t1));
    for (hipEvent_t e : tm.ev) (void)hipEventDestroy(e);
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    if (rc) return rc;
    for (int k = 0; k < 4; ++k) {
        if (kind_ms) kind_ms[k] = acc[k];
        if (kind_launches) kind_launches[k] = tm.launches[k];
        if (kind_flops) kind_flops[k] = tm.flops[k];
    }
    if (total_ms) *total_ms = tot;
    return NBX_OK;
}
