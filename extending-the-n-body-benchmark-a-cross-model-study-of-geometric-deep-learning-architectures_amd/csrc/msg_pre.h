// Fused message_layer_1 (node precomputation GEMM + per-edge combination + Gate) for SEGNN.
//
// message_layer_1 acts on [x_i, x_j, amf] (segnn.py:264-284, o3_building_blocks.py:170-203).
// Its x_i / x_j halves are linear in node features, so per node and plane (0e row, x/y/z rows
// of the 1o channels) the GEMM  X[plane][node] (K = M) x W_plane -> 6 parts of M columns
//   scalar plane: [P_dst s | P_dst gate | R_dst t | P_src s | P_src gate | R_src t]
//   vector plane: [Q_dst s | Q_dst gate | S_dst v | Q_src s | Q_src gate | S_src v]
// is shared by the N-1 edges of the node (2.6x fewer FLOPs than contracting per edge),
// then every edge (dst d, src s) combines d's dst parts with s's src parts, the amf and bias
// terms and the edge's rhat, and applies the gate -> M1S [E][2M] = [m_s | m_v . rhat],
// M1V [3][E][M] = m_v: the A operands of message_layer_2.
//
// Here both steps run in one kernel.  A block owns one 16-channel chunk c (its 6 parts x 16
// columns of both weight images stay in LDS) and walks node groups; a group is the largest
// number of whole systems that fits a 16-row MFMA tile (N <= 16), so every edge of a group is
// computed from the group's own tile.  The block's waves split by role and run a two-stage
// pipeline over a double-buffered LDS exchange:
//   waves 0-3 (one per plane): the 16-row tile of group i through v_mfma_f32_16x16x4_f32
//     (6 independent accumulators, 144 MFMAs at M = 96), results -> exchange[i % 2];
//   waves 4-7: the edges of group i-1 from exchange[(i-1) % 2]; thread = (edge slot, 4
//     channels), ds_read_b128 operands, float4 stores of M1S / M1V;
// one barrier per stage.  The per-node precomputation never goes to HBM.
#pragma once
#include "tp_fused.h"

namespace nbx {

struct MsgPreProb {
    const float* X;      // [4][V][M]
    const float* Simg;   // [c16][F] image of node_pre_s: 6 parts x 16 channels per chunk (CW = 16)
    const float* Vimg;   // [c16][F] image of node_pre_v
                         // (x3: the bf16x3 images, include/nbx.h "bf16x3 images")
    const float* EG;     // [V*G][8] per edge slot: rhat xyz, |rel|, m_src m_dst
    const float* amf;    // [2][3M] (dist, m_i m_j) -> (s, gate, t)
    const float* bias;   // [2M]   (s, gate)
    const float* xcoef;  // pending feature BatchNorm of X (previous layer): [sc_s(M) | sc_v(M) | sh(M)], or null
    BnSrc xbn;           // xbn.sums non-null: that BatchNorm finalised here from atomic sums (xcoef unused);
                         // block 0 stores the coefficients to xbn.coef_out for the layer's later consumers
    float* M1S;          // [V*G][2M]
    float* M1V;          // [3][V*G][M]
    const int* slot;     // general graphs: [V*G] source (local index) per slot, -1 padding; null = fully connected
    long V;
    int N, G, M;
    int NG;              // nodes per group (whole systems, <= 16)
    int n_slabs;         // node groups: ceil(V / NG)
    int chunks;          // ceil(M / 16)
    int per_chunk;       // persistent blocks per chunk
    int img_floats;      // F = 6 * ceil(M/32) * 512 (x3: * 768)
    int prec;            // node GEMM: 0 fp32 MFMA, 1 bf16x3 images, 2 fp16x2 images (descaled by bscale)
    float bscale;        // fp16x2: the factor that undoes the images' power-of-two weight scale
    int xcd_group;       // block id -> (chunk, slab) so a slab's chunk blocks share one XCD (per_chunk % 8 == 0)
    unsigned long long* dbg;  // optional per-wave phase clocks (tuning only)
    int no_dot;               // 1: M1S's dot half is not written (message_layer_2 forms it: TpStream DV)
    int* range_flag;          // fp16x2 range guard (tp_fused.h tp_range_flag), null: off
    unsigned* check;          // NBX_MP_CHECK builds: hand-off invariant violations are counted here
};

// helpers (defined in msg_pre.hip, compiled with packed-fp32 VALU disabled: the edge step's
// arithmetic runs beside the other wave's MFMAs, where v_pk_* ops cost more than plain ones)
inline int msg_pre_group(int N) { return (N >= 2 && N <= 16) ? (16 / N) * N : 0; }
int msg_pre_launch(MsgPreProb& p, hipStream_t st, int num_cus = 256);

}  // namespace nbx
