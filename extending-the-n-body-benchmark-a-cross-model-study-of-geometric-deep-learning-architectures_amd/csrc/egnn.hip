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
    return egnn_forward_impl(w, pos, vel, mass, B, N, out, ws, (hipStream_t)stream);
}

extern "C" int nbx_egnn_rollout(const nbx_egnn_weights* w, float* pos, float* vel, const float* mass, int64_t B,
                                int64_t N, int64_t num_frames, int32_t flags, float* traj_pos, float* traj_vel, void* workspace,
                                size_t workspace_bytes, void* stream) {
    EgnnWs ws;
    if (int rc = egnn_prepare(w, B, N, workspace, workspace_bytes, &ws)) return rc;
    NBX_CHECK_ARG(num_frames >= 1 && w->num_heads == 2, "nbx_egnn_rollout: needs 2 heads (pos_dt, vel), frames >= 1");
    hipStream_t st = (hipStream_t)stream;
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
