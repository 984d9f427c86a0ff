// EGNN-MC forward + device-resident self-feed rollout (fp32).
//
// Reference: dataloaders/egnn_mc_n_body_dataloader.py:8-56 (preprocess_batch),
// models/egnn_mc/egnn_mc.py:45-295 (_EGNNMessageBlock, _VectorHead, EGNNMultiChannel),
// helper_scripts/infer_self_feed.py:161-194 (rollout branch).
//
// Edges keep the reference's fully-connected order (row-major over i, then
// j != i), so the N-1 edges that EGNN aggregates at row = edge_index[0] are
// consecutive.  Every Linear is the weight-stationary MFMA kernel of lin.h; the
// edge MLP's input [h_row | h_col | radial, edge_attr] is gathered inside the
// kernel's A loader (no concatenated edge tensor is materialised), and the two
// 128 -> 1 heads (coord_mlp, coord_mlp_vel) are row dot products in the epilogue.
#include <cstdlib>
#include <cstring>

#include "lin.h"
#include "rollout_state.h"
#include "nbx_internal.h"

namespace {

// x = [|vel|, mass, 0, 0]; per-edge static attrs EA [E][4]; edge index arrays (reference order).
__global__ void egnn_prep_kernel(const float* __restrict__ pos, const float* __restrict__ vel,
                                 const float* __restrict__ mass, int64_t V, int N, float* __restrict__ X4,
                                 float* __restrict__ EA, int64_t* __restrict__ erow, int64_t* __restrict__ ecol) {
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t E = V * (N - 1);
    if (e < V) {
        const float vx = vel[3 * e], vy = vel[3 * e + 1], vz = vel[3 * e + 2];
        X4[4 * e] = sqrtf(vx * vx + vy * vy + vz * vz);
        X4[4 * e + 1] = mass[e];
        X4[4 * e + 2] = 0.f;
        X4[4 * e + 3] = 0.f;
    }
    if (e >= E) return;
    const int64_t per = (int64_t)N * (N - 1);
    const int64_t b = e / per, rr = e - b * per, i = rr / (N - 1), jj = rr - i * (N - 1);
    const int64_t j = jj < i ? jj : jj + 1;
    const int64_t row = b * N + i, col = b * N + j;
    erow[e] = row;
    ecol[e] = col;
    const float dx = pos[3 * row] - pos[3 * col], dy = pos[3 * row + 1] - pos[3 * col + 1],
                dz = pos[3 * row + 2] - pos[3 * col + 2];
    const float d2 = dx * dx + dy * dy + dz * dz;
    const float dist = fmaxf(sqrtf(d2), 1e-12f);
    const float hx = dx / dist, hy = dy / dist, hz = dz / dist;
    EA[4 * e + 0] = mass[row] * mass[col];
    EA[4 * e + 1] = vel[3 * row] * hx + vel[3 * row + 1] * hy + vel[3 * row + 2] * hz;
    EA[4 * e + 2] = vel[3 * col] * hx + vel[3 * col + 1] * hy + vel[3 * col + 2] * hz;
    EA[4 * e + 3] = d2;
}

// coord2radial (egnn_mc.py:155-164): ER [E][8] = (radial, edge_attr[4], 0, 0, 0), DIFF [E][4]
__global__ void egnn_radial_kernel(const float* __restrict__ coord, const int64_t* __restrict__ erow,
                                   const int64_t* __restrict__ ecol, const float* __restrict__ EA, int64_t E,
                                   int norm_diff, float* __restrict__ ER, float* __restrict__ DIFF,
                                   float* __restrict__ cdot) {
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int64_t r = erow[e], c = ecol[e];
    float dx = coord[3 * r] - coord[3 * c], dy = coord[3 * r + 1] - coord[3 * c + 1],
          dz = coord[3 * r + 2] - coord[3 * c + 2];
    const float radial = dx * dx + dy * dy + dz * dz;
    if (norm_diff) {
        const float nrm = fmaxf(sqrtf(radial), 1.0f);
        dx /= nrm; dy /= nrm; dz /= nrm;
    }
    float* er = ER + 8 * e;
    er[0] = radial;
    er[1] = EA[4 * e]; er[2] = EA[4 * e + 1]; er[3] = EA[4 * e + 2]; er[4] = EA[4 * e + 3];
    er[5] = er[6] = er[7] = 0.f;
    DIFF[4 * e] = dx; DIFF[4 * e + 1] = dy; DIFF[4 * e + 2] = dz; DIFF[4 * e + 3] = 0.f;
    cdot[e] = 0.f;
}

// _unsorted_segment_mean over row = edge_index[0] (N-1 consecutive edges per node)
__global__ void egnn_segmean_kernel(const float* __restrict__ EF, int64_t V, int deg, int H, float* __restrict__ AGG) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= V * H) return;
    const int64_t v = i / H;
    const int c = (int)(i - v * H);
    float s = 0.f;
    for (int q = 0; q < deg; ++q) s += EF[(v * deg + q) * H + c];
    AGG[i] = deg > 0 ? s / (float)deg : 0.f;
}

// coord_model + velocity term (egnn_mc.py:135-153, 178-183):
// coord += mean_q clamp(diff * tanh(c), +-100) * w + (cv + b) * vel
__global__ void egnn_coord_kernel(float* __restrict__ coord, const float* __restrict__ vel,
                                  const float* __restrict__ DIFF, const float* __restrict__ cdot,
                                  const float* __restrict__ vdot, float vbias, int64_t V, int deg, int use_tanh,
                                  float coords_weight) {
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= V) return;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int q = 0; q < deg; ++q) {
        const int64_t e = v * deg + q;
        float c = cdot[e];
        if (use_tanh) c = tanhf(c);
        a0 += fminf(fmaxf(DIFF[4 * e] * c, -100.f), 100.f);
        a1 += fminf(fmaxf(DIFF[4 * e + 1] * c, -100.f), 100.f);
        a2 += fminf(fmaxf(DIFF[4 * e + 2] * c, -100.f), 100.f);
    }
    const float inv = deg > 0 ? 1.0f / (float)deg : 0.f;
    const float cv = vdot[v] + vbias;
    coord[3 * v] += a0 * inv * coords_weight + cv * vel[3 * v];
    coord[3 * v + 1] += a1 * inv * coords_weight + cv * vel[3 * v + 1];
    coord[3 * v + 2] += a2 * inv * coords_weight + cv * vel[3 * v + 2];
}

// head input tail: [coord - pos, vel, 0, 0]
__global__ void egnn_headin_kernel(const float* __restrict__ coord, const float* __restrict__ pos,
                                   const float* __restrict__ vel, int64_t V, float* __restrict__ HX) {
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= V) return;
    for (int k = 0; k < 3; ++k) {
        HX[8 * v + k] = coord[3 * v + k] - pos[3 * v + k];
        HX[8 * v + 3 + k] = vel[3 * v + k];
    }
    HX[8 * v + 6] = HX[8 * v + 7] = 0.f;
}

// ===================================================================================================
// Persistent per-system path: one workgroup per system runs preprocessing, every layer, both heads
// and (for a rollout) every frame with the system's state in LDS — one launch per rollout instead of
// ~60 per step.  GEMMs are block-wide fp32 FMA GEMMs over LDS activations (rows = the system's
// N(N-1) <= 56 edges or N <= 8 nodes): thread (n, s) owns output column n and K-slice s, partial sums
// are reduced through LDS in a fixed order (deterministic).  Weights come input-major from the
// persist blob (include/nbx.h), each weight read once per workgroup per layer (coalesced over n).
constexpr int EP_THREADS = 512, EP_NMAX = 8, EP_EMAX = EP_NMAX * (EP_NMAX - 1), EP_RC = 12;

struct EgnnPersist {
    const float* blob;
    int L, N, heads, recurrent, norm_diff, use_tanh;
    float coords_weight;
    float* pos; float* vel; const float* mass;   // [B N 3], [B N 3], [B N]; pos / vel updated in place
    int64_t frames;                              // 0: one forward into out; >= 1: rollout frames
    int absolute;
    float* traj_pos; float* traj_vel;            // [B][frames][N][3]
    float* out;                                  // [B N][3 heads]
    int knn;                                     // 0: fully connected; k >= 1: k edges per row node
    const int* nbr;                              // [B N][k] local neighbour of each edge (forward on a
                                                 // given graph); nullptr with knn: kNN of each frame
};

__device__ inline float ep_silu(float x) { return x / (1.0f + __expf(-x)); }

// Y[r][n] = act(bias[n] + sum_k X[r][k] Wi[k][n]), r < rows, n < H; X, Y in LDS (row strides ldx, ldy,
// ldx % 4 == 0), K % 4 == 0.  Register-blocked: a thread owns 4 adjacent columns and a K-slice, so each
// broadcast LDS read of 4 k-values of a row feeds 16 FMAs; the K-slices held by one wave are summed
// with lane shuffles, the 8 waves' partials through LDS in a fixed order.  All threads call it.
template <int H>
__device__ void ep_gemm(const float* X, int rows, int ldx, int K, const float* __restrict__ Wi,
                        const float* __restrict__ bias, float* Y, int ldy, bool silu_act, float* part) {
    constexpr int CG = H / 4;                  // column groups per wave (32, 16, 8)
    constexpr int SPW = 64 / CG;               // K-slices per wave (2, 4, 8)
    constexpr int S = SPW * (EP_THREADS / 64); // K-slices in the workgroup
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cg = lane % CG, s = wave * SPW + lane / CG, n0 = 4 * cg;
    const int Kc = (((K + S - 1) / S) + 3) & ~3;
    const int k0 = min(K, s * Kc), k1 = min(K, k0 + Kc);
    for (int r0 = 0; r0 < rows; r0 += EP_RC) {
        const int rc = min(EP_RC, rows - r0);
        float4 acc[EP_RC];
#pragma unroll
        for (int r = 0; r < EP_RC; ++r) acc[r] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int k = k0; k < k1; k += 4) {
            const float4 w0 = *reinterpret_cast<const float4*>(&Wi[(size_t)k * H + n0]);
            const float4 w1 = *reinterpret_cast<const float4*>(&Wi[(size_t)(k + 1) * H + n0]);
            const float4 w2 = *reinterpret_cast<const float4*>(&Wi[(size_t)(k + 2) * H + n0]);
            const float4 w3 = *reinterpret_cast<const float4*>(&Wi[(size_t)(k + 3) * H + n0]);
#pragma unroll
            for (int r = 0; r < EP_RC; ++r) {
                if (r < rc) {
                    const float4 x = *reinterpret_cast<const float4*>(&X[(r0 + r) * ldx + k]);
                    acc[r].x += x.x * w0.x + x.y * w1.x + x.z * w2.x + x.w * w3.x;
                    acc[r].y += x.x * w0.y + x.y * w1.y + x.z * w2.y + x.w * w3.y;
                    acc[r].z += x.x * w0.z + x.y * w1.z + x.z * w2.z + x.w * w3.z;
                    acc[r].w += x.x * w0.w + x.y * w1.w + x.z * w2.w + x.w * w3.w;
                }
            }
        }
#pragma unroll
        for (int r = 0; r < EP_RC; ++r) {
            if (r < rc) {
#pragma unroll
                for (int o = CG; o < 64; o <<= 1) {       // the wave's K-slices (fixed order)
                    acc[r].x += __shfl_xor(acc[r].x, o);
                    acc[r].y += __shfl_xor(acc[r].y, o);
                    acc[r].z += __shfl_xor(acc[r].z, o);
                    acc[r].w += __shfl_xor(acc[r].w, o);
                }
                if (lane < CG) *reinterpret_cast<float4*>(&part[(wave * EP_RC + r) * H + n0]) = acc[r];
            }
        }
        __syncthreads();
        for (int o = tid; o < rc * H; o += EP_THREADS) {
            const int r = o / H, nn = o - r * H;
            float v = bias ? bias[nn] : 0.f;
            for (int w = 0; w < EP_THREADS / 64; ++w) v += part[(w * EP_RC + r) * H + nn];
            Y[(r0 + r) * ldy + nn] = silu_act ? ep_silu(v) : v;
        }
        __syncthreads();
    }
}

template <int H>
__global__ __launch_bounds__(EP_THREADS, 1) void egnn_persist_kernel(const EgnnPersist P) {
    constexpr int LD_E = 2 * H + 8, LD_H8 = H + 8;
    constexpr int LAYER = 8 * H * H + 16 * H + 4, HEAD = 2 * H * H + 14 * H + 4;
    constexpr int S = EP_THREADS / 64;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* sA = lds;                                 // [EMAX][2H + 8]: edge input, later EF [E][H]
    float* sB = sA + EP_EMAX * LD_E;                 // [EMAX][H]: EF1 / c0 out / v0 out / n0 out / head hidden
    float* sH = sB + EP_EMAX * H;                    // [NMAX][H]
    float* sHn = sH + EP_NMAX * H;                   // [NMAX][H]
    float* sX = sHn + EP_NMAX * H;                   // [NMAX][2H]: node input [h | agg], heads [h | hx]
    float* sP = sX + EP_NMAX * 2 * H;                // [S][RC][H] partial sums
    float* sm = sP + S * EP_RC * H;                  // small state
    float* pos0 = sm;             // [N][3]
    float* coord = pos0 + 3 * EP_NMAX;
    float* velv = coord + 3 * EP_NMAX;
    float* mass = velv + 3 * EP_NMAX;            // [N]
    float* ea = mass + EP_NMAX;                  // [E][4]
    float* diff = ea + 4 * EP_EMAX;              // [E][3]
    float* cdot = diff + 3 * EP_EMAX;            // [E]
    float* vdot = cdot + EP_EMAX;                // [N]
    float* pred = vdot + EP_NMAX;                // [N][6]
    int* snbr = reinterpret_cast<int*>(pred + 6 * EP_NMAX);   // [E]: kNN graphs, col of edge (i, q) = snbr[i k + q]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int N = P.N, deg = P.knn > 0 ? P.knn : N - 1, E = N * deg;
    const int64_t sys = blockIdx.x;
    const float* emb_i = P.blob;
    const float* emb_b = emb_i + 2 * H;
    const float* layer0 = emb_b + H;
    const float* head0 = layer0 + (size_t)P.L * LAYER;
    auto erow = [&](int e) { return e / deg; };
    auto ecol = [&](int e) {
        if (P.knn > 0) return snbr[e];
        const int i = e / deg, j = e - i * deg;
        return j < i ? j : j + 1;
    };

    for (int i = tid; i < 3 * N; i += EP_THREADS) {
        pos0[i] = P.pos[sys * N * 3 + i];
        velv[i] = P.vel[sys * N * 3 + i];
    }
    for (int i = tid; i < N; i += EP_THREADS) mass[i] = P.mass[sys * N + i];
    __syncthreads();
    auto write_frame = [&](int64_t f) {
        for (int i = tid; i < 3 * N; i += EP_THREADS) {
            P.traj_pos[((sys * P.frames) + f) * N * 3 + i] = pos0[i];
            P.traj_vel[((sys * P.frames) + f) * N * 3 + i] = velv[i];
        }
    };
    if (P.frames >= 1) write_frame(0);
    const int64_t steps = P.frames >= 1 ? P.frames - 1 : 1;
    for (int64_t f = 1; f <= steps; ++f) {
        // ---- graph (egnn_mc_n_body_dataloader.py:13-28): the given kNN table, or build_graph_with_knn
        // of this frame's positions (utils/build_fully_connected_graph.py:42-80): node i's k nearest
        // others by (fp64 distance, index), the first pick (self) dropped -- graph.hip's selection
        if (P.knn > 0) {
            if (P.nbr) {
                for (int e = tid; e < E; e += EP_THREADS) snbr[e] = P.nbr[sys * E + e];
            } else if (tid < N) {
                double d[EP_NMAX];
                const double xi = pos0[3 * tid], yi = pos0[3 * tid + 1], zi = pos0[3 * tid + 2];
                for (int j = 0; j < N; ++j) {
                    const double dx = xi - (double)pos0[3 * j], dy = yi - (double)pos0[3 * j + 1],
                                 dz = zi - (double)pos0[3 * j + 2];
                    d[j] = sqrt(dx * dx + dy * dy + dz * dz);
                }
                unsigned taken = 0;
                for (int s = 0; s <= deg; ++s) {
                    int best = -1;
                    for (int j = 0; j < N; ++j) {
                        if ((taken >> j) & 1u) continue;
                        if (best < 0 || d[j] < d[best]) best = j;
                    }
                    taken |= 1u << best;
                    if (s > 0) snbr[tid * deg + s - 1] = best;
                }
            }
            __syncthreads();
        }
        // ---- preprocess_batch (egnn_mc_n_body_dataloader.py:8-56): x = [|vel|, mass], edge_attr
        for (int o = tid; o < N * H; o += EP_THREADS) {
            const int i = o / H, n = o - i * H;
            const float vx = velv[3 * i], vy = velv[3 * i + 1], vz = velv[3 * i + 2];
            sH[i * H + n] = emb_b[n] + sqrtf(vx * vx + vy * vy + vz * vz) * emb_i[n] + mass[i] * emb_i[H + n];
        }
        for (int e = tid; e < E; e += EP_THREADS) {
            const int r = erow(e), c = ecol(e);
            const float dx = pos0[3 * r] - pos0[3 * c], dy = pos0[3 * r + 1] - pos0[3 * c + 1],
                        dz = pos0[3 * r + 2] - pos0[3 * c + 2];
            const float d2 = dx * dx + dy * dy + dz * dz, d = fmaxf(sqrtf(d2), 1e-12f);
            const float hx = dx / d, hy = dy / d, hz = dz / d;
            ea[4 * e] = mass[r] * mass[c];
            ea[4 * e + 1] = velv[3 * r] * hx + velv[3 * r + 1] * hy + velv[3 * r + 2] * hz;
            ea[4 * e + 2] = velv[3 * c] * hx + velv[3 * c + 1] * hy + velv[3 * c + 2] * hz;
            ea[4 * e + 3] = d2;
        }
        for (int i = tid; i < 3 * N; i += EP_THREADS) coord[i] = pos0[i];
        __syncthreads();
        float* h = sH;
        float* hn = sHn;
        for (int l = 0; l < P.L; ++l) {
            const float* Wl = layer0 + (size_t)l * LAYER;
            const float *e0_i = Wl, *e0_b = e0_i + LD_E * H, *e1_i = e0_b + H, *e1_b = e1_i + H * H,
                        *c0_i = e1_b + H, *c0_b = c0_i + H * H, *c1_w = c0_b + H, *v0_i = c1_w + H,
                        *v0_b = v0_i + H * H, *v1_w = v0_b + H, *v1_b = v1_w + H, *n0_i = v1_b + 4,
                        *n0_b = n0_i + 2 * H * H, *n1_i = n0_b + H, *n1_b = n1_i + H * H;
            // coord2radial (egnn_mc.py:155-164) + edge input [h_row | h_col | radial, edge_attr]
            for (int e = tid; e < E; e += EP_THREADS) {
                const int r = erow(e), c = ecol(e);
                float dx = coord[3 * r] - coord[3 * c], dy = coord[3 * r + 1] - coord[3 * c + 1],
                      dz = coord[3 * r + 2] - coord[3 * c + 2];
                const float radial = dx * dx + dy * dy + dz * dz;
                if (P.norm_diff) {
                    const float nrm = fmaxf(sqrtf(radial), 1.0f);
                    dx /= nrm; dy /= nrm; dz /= nrm;
                }
                diff[3 * e] = dx; diff[3 * e + 1] = dy; diff[3 * e + 2] = dz;
                float* x = sA + e * LD_E + 2 * H;
                x[0] = radial; x[1] = ea[4 * e]; x[2] = ea[4 * e + 1]; x[3] = ea[4 * e + 2]; x[4] = ea[4 * e + 3];
                x[5] = x[6] = x[7] = 0.f;
            }
            for (int o = tid; o < E * H; o += EP_THREADS) {
                const int e = o / H, n = o - e * H;
                sA[e * LD_E + n] = h[erow(e) * H + n];
                sA[e * LD_E + H + n] = h[ecol(e) * H + n];
            }
            __syncthreads();
            ep_gemm<H>(sA, E, LD_E, LD_E, e0_i, e0_b, sB, H, true, sP);       // edge_mlp[0] + SiLU
            ep_gemm<H>(sB, E, H, H, e1_i, e1_b, sA, H, true, sP);             // edge_mlp[2] + SiLU -> EF
            ep_gemm<H>(sA, E, H, H, c0_i, c0_b, sB, H, true, sP);             // coord_mlp[0] + SiLU
            for (int e = wave; e < E; e += EP_THREADS / 64) {                   // coord_mlp[2] (no bias)
                float v = 0.f;
                for (int n = lane; n < H; n += 64) v += sB[e * H + n] * c1_w[n];
                for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
                if (lane == 0) cdot[e] = P.use_tanh ? tanhf(v) : v;
            }
            __syncthreads();
            ep_gemm<H>(h, N, H, H, v0_i, v0_b, sB, H, true, sP);              // coord_mlp_vel[0] + SiLU
            for (int i = wave; i < N; i += EP_THREADS / 64) {
                float v = 0.f;
                for (int n = lane; n < H; n += 64) v += sB[i * H + n] * v1_w[n];
                for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
                if (lane == 0) vdot[i] = v + v1_b[0];
            }
            for (int o = tid; o < N * H; o += EP_THREADS) {                   // node input [h | mean_j EF]
                const int i = o / H, n = o - i * H;
                float a = 0.f;
                for (int q = 0; q < deg; ++q) a += sA[(i * deg + q) * H + n];
                sX[i * 2 * H + n] = h[i * H + n];
                sX[i * 2 * H + H + n] = deg > 0 ? a / (float)deg : 0.f;
            }
            __syncthreads();
            ep_gemm<H>(sX, N, 2 * H, 2 * H, n0_i, n0_b, sB, H, true, sP);     // node_mlp[0] + SiLU
            ep_gemm<H>(sB, N, H, H, n1_i, n1_b, hn, H, false, sP);            // node_mlp[2]
            if (P.recurrent)
                for (int o = tid; o < N * H; o += EP_THREADS) hn[o] += h[o];
            // coord_model + velocity term (egnn_mc.py:135-153, 178-183)
            for (int o = tid; o < 3 * N; o += EP_THREADS) {
                const int i = o / 3, k = o - 3 * i;
                float a = 0.f;
                for (int q = 0; q < deg; ++q) {
                    const int e = i * deg + q;
                    a += fminf(fmaxf(diff[3 * e + k] * cdot[e], -100.f), 100.f);
                }
                coord[o] += (deg > 0 ? a / (float)deg : 0.f) * P.coords_weight + vdot[i] * velv[o];
            }
            __syncthreads();
            float* t = h; h = hn; hn = t;
        }
        // ---- vector heads: [h | coord - pos, vel, 0, 0] -> SiLU -> SiLU -> 3
        for (int o = tid; o < N * LD_H8; o += EP_THREADS) {
            const int i = o / LD_H8, k = o - i * LD_H8;
            float v = 0.f;
            if (k < H) v = h[i * H + k];
            else if (k < H + 3) v = coord[3 * i + k - H] - pos0[3 * i + k - H];
            else if (k < H + 6) v = velv[3 * i + k - H - 3];
            sX[i * LD_H8 + k] = v;
        }
        __syncthreads();
        for (int t = 0; t < P.heads; ++t) {
            const float* Wh = head0 + (size_t)t * HEAD;
            const float *w0_i = Wh, *b0 = w0_i + LD_H8 * H, *w1_i = b0 + H, *b1 = w1_i + H * H, *w2_i = b1 + H,
                        *b2 = w2_i + 4 * H;
            ep_gemm<H>(sX, N, LD_H8, LD_H8, w0_i, b0, sB, H, true, sP);
            ep_gemm<H>(sB, N, H, H, w1_i, b1, sA, H, true, sP);
            for (int i = wave; i < N; i += EP_THREADS / 64) {
                float v0 = 0.f, v1 = 0.f, v2 = 0.f;
                for (int n = lane; n < H; n += 64) {
                    const float x = sA[i * H + n];
                    v0 += x * w2_i[4 * n];
                    v1 += x * w2_i[4 * n + 1];
                    v2 += x * w2_i[4 * n + 2];
                }
                for (int o = 32; o > 0; o >>= 1) {
                    v0 += __shfl_xor(v0, o);
                    v1 += __shfl_xor(v1, o);
                    v2 += __shfl_xor(v2, o);
                }
                if (lane == 0) {
                    pred[6 * i + 3 * t] = v0 + b2[0];
                    pred[6 * i + 3 * t + 1] = v1 + b2[1];
                    pred[6 * i + 3 * t + 2] = v2 + b2[2];
                }
            }
            __syncthreads();
        }
        if (P.frames == 0) {
            for (int o = tid; o < N * 3 * P.heads; o += EP_THREADS) {
                const int i = o / (3 * P.heads), k = o - i * 3 * P.heads;
                P.out[(sys * N + i) * 3 * P.heads + k] = pred[6 * i + k];
            }
            return;
        }
        // ---- self-feed state update (infer_self_feed.py:182-194)
        for (int o = tid; o < 3 * N; o += EP_THREADS) {
            const int i = o / 3, k = o - 3 * i;
            pos0[o] = P.absolute ? pred[6 * i + k] : pos0[o] + pred[6 * i + k];
            velv[o] = pred[6 * i + 3 + k];
        }
        __syncthreads();
        write_frame(f);
    }
    for (int i = tid; i < 3 * N; i += EP_THREADS) {
        P.pos[sys * N * 3 + i] = pos0[i];
        P.vel[sys * N * 3 + i] = velv[i];
    }
}

size_t ep_lds_bytes(int H) {
    const int S = EP_THREADS / 64;
    const size_t fl = (size_t)EP_EMAX * (2 * H + 8) + EP_EMAX * H + 2 * EP_NMAX * H + EP_NMAX * 2 * H +
                      (size_t)S * EP_RC * H + 3 * 3 * EP_NMAX + EP_NMAX + 4 * EP_EMAX + 3 * EP_EMAX + EP_EMAX +
                      EP_NMAX + 6 * EP_NMAX + EP_EMAX;
    return fl * 4;
}

bool ep_usable(const nbx_egnn_weights* w, int64_t N) {
    static const bool off = getenv("NBX_EGNN_PERSIST") && getenv("NBX_EGNN_PERSIST")[0] == '0';
    return !off && w->persist_blob && (w->hidden == 32 || w->hidden == 64 || w->hidden == 128) && N >= 2 &&
           N <= EP_NMAX && w->num_heads >= 1 && w->num_heads <= 2;
}

template <int H>
int ep_launch_h(const EgnnPersist& p, int64_t B, hipStream_t st) {
    const size_t lds = ep_lds_bytes(H);
    NBX_LDS_160K(egnn_persist_kernel<H>);
    hipLaunchKernelGGL(egnn_persist_kernel<H>, dim3((unsigned)B), dim3(EP_THREADS), lds, st, p);
    NBX_HIP(hipGetLastError());
    return NBX_OK;
}

int ep_launch(const nbx_egnn_weights* w, float* pos, float* vel, const float* mass, int64_t B, int64_t N,
              int64_t frames, int absolute, float* traj_pos, float* traj_vel, float* out, hipStream_t st,
              int knn = 0, const int* nbr = nullptr) {
    EgnnPersist p{w->persist_blob, w->num_layers, (int)N, w->num_heads, w->recurrent, w->norm_diff, w->use_tanh,
                  w->coords_weight, pos, vel, mass, frames, absolute, traj_pos, traj_vel, out, knn, nbr};
    switch (w->hidden) {
        case 32: return ep_launch_h<32>(p, B, st);
        case 64: return ep_launch_h<64>(p, B, st);
        default: return ep_launch_h<128>(p, B, st);
    }
}

struct EgnnWs {
    float *X4, *EA, *ER, *DIFF, *cdot, *vdot, *H, *H2, *EF1, *EF, *AGG, *N1, *coord, *HX, *T1, *T2, *out;
    int64_t *erow, *ecol;
};

size_t egnn_carve(EgnnWs* ws, void* base, int64_t B, int64_t N, int H) {
    const int64_t V = B * N, E = V * (N - 1);
    size_t off = 0;
    auto take = [&](size_t n, size_t el) -> void* {
        off = (off + 255) & ~size_t(255);
        void* p = base ? (void*)((char*)base + off) : nullptr;
        off += n * el;
        return p;
    };
    EgnnWs w;
    w.erow = (int64_t*)take(E, 8);
    w.ecol = (int64_t*)take(E, 8);
    w.X4 = (float*)take(4 * V, 4);
    w.EA = (float*)take(4 * E, 4);
    w.ER = (float*)take(8 * E, 4);
    w.DIFF = (float*)take(4 * E, 4);
    w.cdot = (float*)take(E, 4);
    w.vdot = (float*)take(V, 4);
    w.H = (float*)take(V * H, 4);
    w.H2 = (float*)take(V * H, 4);
    w.EF1 = (float*)take(E * H, 4);
    w.EF = (float*)take(E * H, 4);
    w.AGG = (float*)take(V * H, 4);
    w.N1 = (float*)take(V * H, 4);
    w.coord = (float*)take(3 * V, 4);
    w.HX = (float*)take(8 * V, 4);
    w.T1 = (float*)take(V * H, 4);
    w.T2 = (float*)take(V * H, 4);
    w.out = (float*)take(6 * V, 4);
    if (ws) *ws = w;
    return (off + 255) & ~size_t(255);
}

unsigned g1(int64_t n) { return (unsigned)nbx::ceil_div(n > 0 ? n : 1, 256); }

int egnn_forward_impl(const nbx_egnn_weights* w, const float* pos, const float* vel, const float* mass, int64_t B,
                      int64_t N, float* out, const EgnnWs& ws, hipStream_t st) {
    using nbx::LinProb;
    const int H = w->hidden;
    const int64_t V = B * N, E = V * (N - 1);
    const int deg = (int)(N - 1);
    const int iV = (int)V, iE = (int)E;
    hipLaunchKernelGGL(egnn_prep_kernel, dim3(g1(std::max(V, E))), dim3(256), 0, st, pos, vel, mass, V, (int)N, ws.X4,
                       ws.EA, ws.erow, ws.ecol);
    NBX_HIP(hipMemcpyAsync(ws.coord, pos, sizeof(float) * 3 * V, hipMemcpyDeviceToDevice, st));
    {   // embedding: Linear(node_input_dim -> H)
        LinProb p = nbx::lin_dense(ws.X4, 4, 4, iV, w->emb_t, 32, H, w->emb_b, ws.H, H);
        if (int rc = nbx::lin_launch<4, nbx::ACT_NONE>(p, st)) return rc;
    }
    float* h = ws.H;
    float* h_next = ws.H2;
    for (int l = 0; l < w->num_layers; ++l) {
        const nbx_egnn_layer& L = w->layers[l];
        hipLaunchKernelGGL(egnn_radial_kernel, dim3(g1(E)), dim3(256), 0, st, ws.coord, ws.erow, ws.ecol, ws.EA, E,
                           w->norm_diff, ws.ER, ws.DIFF, ws.cdot);
        NBX_HIP(hipMemsetAsync(ws.vdot, 0, sizeof(float) * V, st));
        if (E > 0) {
            // edge_mlp[0]: SiLU(W [h_row | h_col | radial, attrs] + b)
            LinProb p;
            memset(&p, 0, sizeof(p));
            p.seg[0] = nbx::LinSeg{h, ws.erow, H, (H + 31) & ~31, H};
            p.seg[1] = nbx::LinSeg{h, ws.ecol, H, (H + 31) & ~31, H};
            p.seg[2] = nbx::LinSeg{ws.ER, nullptr, 8, 32, 8};
            p.nseg = 3;
            p.rows = iE; p.N = H; p.Ktot = 2 * ((H + 31) & ~31) + 32;
            p.Wt = L.e0_t; p.ldw = p.Ktot; p.bias = L.e0_b; p.Y = ws.EF1; p.ldy = H;
            if (int rc = nbx::lin_launch<4, nbx::ACT_SILU>(p, st)) return rc;
            // edge_mlp[2]
            LinProb q = nbx::lin_dense(ws.EF1, H, H, iE, L.e1_t, (H + 31) & ~31, H, L.e1_b, ws.EF, H);
            if (int rc = nbx::lin_launch<4, nbx::ACT_SILU>(q, st)) return rc;
            // coord_mlp: SiLU(W0 ef + b0) . w1  (no bias; tanh applied in egnn_coord_kernel)
            LinProb c = nbx::lin_dense(ws.EF, H, H, iE, L.c0_t, (H + 31) & ~31, H, L.c0_b, nullptr, 0);
            c.dotw = L.c1_w;
            c.rowdot = ws.cdot;
            if (int rc = nbx::lin_launch<4, nbx::ACT_SILU>(c, st)) return rc;
        }
        {   // coord_mlp_vel: SiLU(V0 h + b) . v1 + b1
            LinProb p = nbx::lin_dense(h, H, H, iV, L.v0_t, (H + 31) & ~31, H, L.v0_b, nullptr, 0);
            p.dotw = L.v1_w;
            p.rowdot = ws.vdot;
            if (int rc = nbx::lin_launch<4, nbx::ACT_SILU>(p, st)) return rc;
        }
        hipLaunchKernelGGL(egnn_segmean_kernel, dim3(g1(V * H)), dim3(256), 0, st, ws.EF, V, deg, H, ws.AGG);
        {   // node_mlp: h' = h + W1 SiLU(W0 [h | agg] + b0) + b1
            LinProb p;
            memset(&p, 0, sizeof(p));
            p.seg[0] = nbx::LinSeg{h, nullptr, H, (H + 31) & ~31, H};
            p.seg[1] = nbx::LinSeg{ws.AGG, nullptr, H, (H + 31) & ~31, H};
            p.nseg = 2;
            p.rows = iV; p.N = H; p.Ktot = 2 * ((H + 31) & ~31);
            p.Wt = L.n0_t; p.ldw = p.Ktot; p.bias = L.n0_b; p.Y = ws.N1; p.ldy = H;
            if (int rc = nbx::lin_launch<4, nbx::ACT_SILU>(p, st)) return rc;
            LinProb q = nbx::lin_dense(ws.N1, H, H, iV, L.n1_t, (H + 31) & ~31, H, L.n1_b, h_next, H);
            if (w->recurrent) {
                q.resid = h;
                q.ldr = H;
            }
            if (int rc = nbx::lin_launch<4, nbx::ACT_NONE>(q, st)) return rc;
        }
        hipLaunchKernelGGL(egnn_coord_kernel, dim3(g1(V)), dim3(256), 0, st, ws.coord, vel, ws.DIFF, ws.cdot, ws.vdot,
                           L.v1_b, V, deg, w->use_tanh, w->coords_weight);
        NBX_LAUNCH_CHECK("egnn layer");
        std::swap(h, h_next);
    }
    // heads: [h | coord - pos, vel] -> SiLU -> SiLU -> 3, concatenated in target order
    hipLaunchKernelGGL(egnn_headin_kernel, dim3(g1(V)), dim3(256), 0, st, ws.coord, pos, vel, V, ws.HX);
    for (int t = 0; t < w->num_heads; ++t) {
        LinProb p;
        memset(&p, 0, sizeof(p));
        p.seg[0] = nbx::LinSeg{h, nullptr, H, (H + 31) & ~31, H};
        p.seg[1] = nbx::LinSeg{ws.HX, nullptr, 8, 32, 8};
        p.nseg = 2;
        p.rows = iV; p.N = H; p.Ktot = ((H + 31) & ~31) + 32;
        p.Wt = w->heads[t].w0_t; p.ldw = p.Ktot; p.bias = w->heads[t].b0; p.Y = ws.T1; p.ldy = H;
        if (int rc = nbx::lin_launch<4, nbx::ACT_SILU>(p, st)) return rc;
        LinProb q = nbx::lin_dense(ws.T1, H, H, iV, w->heads[t].w1_t, (H + 31) & ~31, H, w->heads[t].b1, ws.T2, H);
        if (int rc = nbx::lin_launch<4, nbx::ACT_SILU>(q, st)) return rc;
        LinProb o = nbx::lin_dense(ws.T2, H, H, iV, w->heads[t].w2_t, (H + 31) & ~31, 3, w->heads[t].b2, out + 3 * t,
                                   3 * w->num_heads);
        if (int rc = nbx::lin_launch<1, nbx::ACT_NONE>(o, st)) return rc;
    }
    NBX_LAUNCH_CHECK("egnn heads");
    return NBX_OK;
}

int egnn_prepare(const nbx_egnn_weights* w, int64_t B, int64_t N, void* ws_ptr, size_t bytes, EgnnWs* ws) {
    NBX_CHECK_ARG(w && w->hidden > 0 && w->hidden % 4 == 0 && w->hidden <= 160, "egnn: hidden must be 4..160, %%4");
    NBX_CHECK_ARG(w->num_layers >= 0 && w->num_layers <= NBX_EGNN_MAX_LAYERS, "egnn: bad num_layers");
    NBX_CHECK_ARG(w->num_heads >= 1 && w->num_heads <= 2, "egnn: 1 or 2 vector heads");
    NBX_CHECK_ARG(B >= 1 && N >= 2 && B * N * N < ((int64_t)1 << 31), "egnn: need B >= 1, N >= 2");
    const size_t need = egnn_carve(ws, ws_ptr, B, N, w->hidden);
    if (!ws_ptr || bytes < need) {
        nbx::set_error("egnn: workspace too small (%zu < %zu bytes)", bytes, need);
        return NBX_E_WORKSPACE;
    }
    return NBX_OK;
}

}  // namespace

extern "C" int nbx_egnn_workspace_bytes(int64_t B, int64_t N, int32_t hidden, size_t* bytes) {
    NBX_CHECK_ARG(bytes && B >= 1 && N >= 1 && hidden > 0, "nbx_egnn_workspace_bytes: bad arguments");
    *bytes = egnn_carve(nullptr, nullptr, B, N, hidden);
    return NBX_OK;
}

extern "C" int nbx_egnn_forward(const nbx_egnn_weights* w, const float* pos, const float* vel, const float* mass,
                                int64_t B, int64_t N, float* out, void* workspace, size_t workspace_bytes,
                                void* stream) {
    EgnnWs ws;
    if (int rc = egnn_prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    if (ep_usable(w, N))   // frames = 0: one forward, pos / vel read only
        return ep_launch(w, const_cast<float*>(pos), const_cast<float*>(vel), mass, B, N, 0, 0, nullptr, nullptr, out,
                         (hipStream_t)stream);
    return egnn_forward_impl(w, pos, vel, mass, B, N, out, ws, (hipStream_t)stream);
}

extern "C" int nbx_egnn_rollout(const nbx_egnn_weights* w, float* pos, float* vel, const float* mass, int64_t B,
                                int64_t N, int64_t num_frames, int32_t flags, float* traj_pos, float* traj_vel, void* workspace,
                                size_t workspace_bytes, void* stream) {
    EgnnWs ws;
    if (int rc = egnn_prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    NBX_CHECK_ARG(num_frames >= 1 && w->num_heads == 2, "nbx_egnn_rollout: needs 2 heads (pos_dt, vel), frames >= 1");
    hipStream_t st = (hipStream_t)stream;
    if (ep_usable(w, N))   // the whole rollout in one launch
        return ep_launch(w, pos, vel, mass, B, N, num_frames, flags & NBX_ROLLOUT_ABSOLUTE, traj_pos, traj_vel, nullptr,
                         st);
    const int64_t V = B * N;
    hipLaunchKernelGGL(nbx::rollout_state_kernel, dim3(g1(3 * V)), dim3(256), 0, st, pos, vel, ws.out, V, (int)N, (int64_t)0,
                       num_frames, traj_pos, traj_vel, flags & NBX_ROLLOUT_ABSOLUTE);
    for (int64_t f = 1; f < num_frames; ++f) {
        if (int rc = egnn_forward_impl(w, pos, vel, mass, B, N, ws.out, ws, st)) return rc;
        hipLaunchKernelGGL(nbx::rollout_state_kernel, dim3(g1(3 * V)), dim3(256), 0, st, pos, vel, ws.out, V, (int)N, f,
                           num_frames, traj_pos, traj_vel, flags & NBX_ROLLOUT_ABSOLUTE);
    }
    NBX_LAUNCH_CHECK("egnn rollout");
    return NBX_OK;
}

// kNN graphs (egnn_mc_n_body_dataloader.py:13-28 hands the model build_graph_with_knn's
// graph when args.num_neighbors < N - 1): the persistent kernel with an explicit neighbour table.
namespace {
int egnn_knn_check(const nbx_egnn_weights* w, int64_t N, int64_t k, const char* fn) {
    NBX_CHECK_ARG(k >= 1 && k < N, "%s: need 1 <= num_neighbors < N (got %lld, N = %lld)", fn, (long long)k,
                  (long long)N);
    if (!ep_usable(w, N)) {
        nbx::set_error("%s: kNN graphs run on the persistent kernel only (hidden 32 / 64 / 128, 2 <= N <= %d)", fn,
                       EP_NMAX);
        return NBX_E_UNSUPPORTED;
    }
    return NBX_OK;
}
}  // namespace

extern "C" int nbx_egnn_forward_graph(const nbx_egnn_weights* w, const float* pos, const float* vel,
                                      const float* mass, int64_t B, int64_t N, int64_t k, const int32_t* nbr,
                                      float* out, void* workspace, size_t workspace_bytes, void* stream) {
    EgnnWs ws;
    if (int rc = egnn_prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    if (k == N - 1 && !nbr) return nbx_egnn_forward(w, pos, vel, mass, B, N, out, workspace, workspace_bytes, stream);
    if (int rc = egnn_knn_check(w, N, k, "nbx_egnn_forward_graph")) return rc;
    NBX_CHECK_ARG(nbr != nullptr, "nbx_egnn_forward_graph: null neighbour table");
    return ep_launch(w, const_cast<float*>(pos), const_cast<float*>(vel), mass, B, N, 0, 0, nullptr, nullptr, out,
                     (hipStream_t)stream, (int)k, nbr);
}

extern "C" int nbx_egnn_rollout_knn(const nbx_egnn_weights* w, float* pos, float* vel, const float* mass, int64_t B,
                                    int64_t N, int64_t num_frames, int32_t flags, int64_t k, float* traj_pos,
                                    float* traj_vel, void* workspace, size_t workspace_bytes, void* stream) {
    if (k == N - 1)
        return nbx_egnn_rollout(w, pos, vel, mass, B, N, num_frames, flags, traj_pos, traj_vel, workspace,
                                workspace_bytes, stream);
    EgnnWs ws;
    if (int rc = egnn_prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    NBX_CHECK_ARG(num_frames >= 1 && w->num_heads == 2, "nbx_egnn_rollout_knn: needs 2 heads (pos_dt, vel), frames >= 1");
    if (int rc = egnn_knn_check(w, N, k, "nbx_egnn_rollout_knn")) return rc;
    return ep_launch(w, pos, vel, mass, B, N, num_frames, flags & NBX_ROLLOUT_ABSOLUTE, traj_pos, traj_vel, nullptr,
                     (hipStream_t)stream, (int)k, nullptr);
}
