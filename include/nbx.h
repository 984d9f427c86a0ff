/*
 * nbx.h — C ABI of the MI355X-native N-body hot path (libnbx.so).
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t passed
 * as `void*`; nothing here owns memory (callers allocate outputs and the
 * workspace).  Return value: 0 on success, otherwise a nonzero code; the message
 * is available from nbx_last_error() (thread-local).  Launches are asynchronous
 * on `stream` unless stated otherwise and never synchronise the device, so a
 * caller may capture them into a hipGraph.
 *
 * Each declaration cites the reference interface (file:line, paths relative to
 * the reference repository) whose behaviour it reproduces.  The reference is
 * pure Python; the binding a maintainer would add is shown in INTEGRATION.md.
 */
#ifndef NBX_H
#define NBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NBX_ABI_VERSION 19

#define NBX_OK 0
#define NBX_E_INVAL 1      /* bad argument (shape, size, pointer) */
#define NBX_E_UNSUPPORTED 2 /* configuration outside the native path */
#define NBX_E_HIP 3        /* HIP runtime error (message has details) */
#define NBX_E_WORKSPACE 4  /* workspace too small */
#define NBX_E_RANGE 5      /* an fp16x2 tensor-product operand left the fp16 range (nbx_segnn_range_check) */

/* rollout flags */
#define NBX_ROLLOUT_ABSOLUTE 1 /* the model predicts absolute positions: pos = pred[:, :3] (every dataset target
                                  other than "pos_dt+vel", infer_self_feed.py:185-186); default pos += pred[:, :3] */

int nbx_abi_version(void);
const char* nbx_last_error(void);

/* ------------------------------------------------------------------------
 * A1 — graph builder.
 * Replaces utils/build_fully_connected_graph.py:4-20 (_build_fully_connected_edge_index)
 * and the fully-connected branch of build_graph_with_knn (:23-40).
 * edge_index: int64 [2, B*N*(N-1)], row-major over i then j != i, system offset b*N.
 * Bit-exact with the reference.
 */
int nbx_fc_edge_index(int64_t batch_size, int64_t num_nodes, int64_t* edge_index, void* stream);

/* kNN branch of build_graph_with_knn (:42-80): per system, the k nearest other
 * nodes by Euclidean distance in ascending order (index order breaks ties);
 * edge_index = [i, neighbour] + b*N, int64 [2, B*N*k].  loc fp32 [B*N, 3]
 * (dtype 0) or fp64 (dtype 1).  Returns NBX_E_INVAL if k >= N (the reference
 * raises ValueError), requires N <= 64. */
int nbx_knn_edge_index(const void* loc, int32_t dtype, int64_t batch_size, int64_t num_nodes, int64_t k,
                       int64_t* edge_index, void* stream);

/* ------------------------------------------------------------------------
 * A20-A22 — GravitySim ground-truth integrator (fp64).
 * Replaces datasets/nbody/dataset/synthetic_sim.py:318-340 (compute_acceleration).
 * pos [S,N,3], mass [S,N]; acc [S,N,3] = G * sum_j m_j (x_j - x_i)(|x_j-x_i|^2+eps^2)^-1.5
 */
int nbx_gravity_acceleration(const double* pos, const double* mass, int64_t num_systems, int64_t num_nodes,
                             double G, double softening, double* acc, void* stream);

/* Replaces synthetic_sim.py:383-408 (the sample_trajectory KDK loop, noise_var=0):
 * from initial (pos, vel) [S,N,3] run T kick-drift-kick steps of size dt,
 * saving (pos, vel, acc*mass) every sample_freq steps BEFORE stepping into
 * pos_save/vel_save/force_save [S, T/sample_freq, N, 3].  pos/vel are
 * overwritten with the final state.  The whole loop runs inside one kernel per
 * system tile (state in LDS).  Requires T % sample_freq == 0, N <= 1024. */
int nbx_gravity_sample(double* pos, double* vel, const double* mass, int64_t num_systems, int64_t num_nodes,
                       int64_t T, int64_t sample_freq, double dt, double G, double softening,
                       double* pos_save, double* vel_save, double* force_save, void* stream);

/* Trainer._compute_nbody_energies (trainer.py:888-927) on the device: loc/vel
 * [B, T, N, 3] fp64 -> kinetic/potential [B, T] per frame (unit masses) and, when
 * the pointers are non-NULL, their means over the B systems [T]. */
int nbx_nbody_energies(const double* loc, const double* vel, int64_t batch_size, int64_t num_frames,
                       int64_t num_nodes, double G, double softening, double* kinetic, double* potential,
                       double* mean_kinetic, double* mean_potential, void* stream);

/* Self-feed macro statistics (utils/ks_utils.py:7-17 `_ks_p`, driven by
 * trainer.py:668-722): for each of num_pairs pairs (a[p, :na], b[p, :nb]) (rows lda / ldb
 * doubles apart, device memory) the two-sample Kolmogorov-Smirnov statistic of the non-NaN
 * values, D = max_x |F_a(x) - F_b(x)| with F(x) = #{<= x} / n over every sample (scipy
 * ks_2samp's statistic, bit-exact) -> d_out[p] (NaN if either side has no numbers) and, if
 * n_out is non-NULL, the non-NaN counts n_out[2p], n_out[2p+1].  One workgroup per pair;
 * na, nb <= 8192.  The p-value is a host-side function of (D, n_a, n_b). */
int nbx_ks_2samp_stat(const double* a, int64_t na, int64_t lda, const double* b, int64_t nb, int64_t ldb,
                      int64_t num_pairs, double* d_out, int64_t* n_out, void* stream);

/* ------------------------------------------------------------------------
 * SEGNN (models/segnn/segnn.py:17-304, o3_building_blocks.py:10-278) — fp32.
 *
 * Native scope: task="node", norm="batch", lmax_h = lmax_attr = 1, input irreps
 * 2x1o+1x0e, output 2x1o, additional message irreps 2x0e, fully-connected
 * systems of N nodes.  Hidden irreps are mul x 0e + mul x 1o (mul % 4 == 0).
 *
 * Weights are the reference's e3nn parameters re-packed once on the device by
 * the host module (see the package's segnn.py::packed_matrices for the exact
 * formulas).  Matrices named *_t are stored transposed, [N_out][K_in], row-major.
 *
 * TP operand images (*_img; built by segnn.py::tp_images).  Every O(3) tensor
 * product is a scalar-row GEMM with sub-tiles j (output part j: s, gate, t;
 * contraction length K_j) plus, for the gate/update TPs, a vector-row GEMM
 * (length Kv).  Its image is [chunks][F] fp32, one chunk = CW output channels of
 * every part, copied verbatim into LDS by the kernel:
 *   F = (sum_j KC_j + KC_v) * 32 * CW,  KC = ceil(K / 32);
 *   inside a chunk: the sub-tile blocks j = 0.. then the vector block, each
 *   [KC][32 * CW] in MFMA fragment order, zero past K and past the real channels:
 *     CW = 16 (v_mfma_f32_16x16x4_f32): [half 2][qd 4][c 16][e 4] = W[c][32 kc + 8 qd + 4 half + e]
 *     CW = 32 (v_mfma_f32_32x32x2_f32): [q 4][h 2][c 32][e 4]     = W[c][32 kc + 16 h + 4 q + e]
 *   so lane l of a wave reads 16 contiguous bytes per ds_read_b128 (bank-conflict free).
 * msg2_img uses CW = 32 with ceil(mul/32) chunks; every other image CW = 16 with
 * ceil(mul/16) chunks rounded up to a multiple of 4.  node_pre: 6 parts of mul
 * columns (P_dst s, gate, t, P_src s, gate, t), chunk c = channels [16 c, 16 c + 16) of each.
 *
 * bf16x3 images (*_img_x3, optional, NULL = fp32 MFMA path): the split-precision
 * path writes every weight as W = hi + mid + lo, each part rounded to bf16
 * (|W - hi - mid - lo| <= 2^-27 |W|), and every activation the same way as it is
 * loaded; a product accumulates in fp32 the six terms hi.hi + hi.mid + mid.hi +
 * hi.lo + mid.mid + lo.hi (dropped terms <= 2^-24 relative), fp32-level accuracy
 * on v_mfma_f32_32x32x16_bf16 / 16x16x32_bf16.  Layout per sub-tile block and
 * 32-deep K chunk kc:
 *   CW = 32: [part p 3][m 2][lane 64][j 8] bf16 = part p of
 *            W[c = 32 chunk + (lane & 31)][k = 32 kc + 16 (lane >> 5) + 8 m + j];
 *   CW = 16: [part p 3][lane 64][j 8] bf16 = part p of
 *            W[c = 16 chunk + (lane & 15)][k = 32 kc + 8 (lane >> 4) + j].
 *
 * fp16x2 images (*_img_h2, ABI 15, NULL = no fp16x2 path): the weights of one TP are scaled by a
 * power of two s (max |W s| in [2^9, 2^10)) and written as W s = hi + lo, hi = fp16(W s) (RNE),
 * lo = fp16(W s - hi); activations are split the same way as they are loaded (unscaled).  A product
 * accumulates in fp32 the three terms hi.lo + lo.hi + hi.hi on v_mfma_f32_32x32x16_f16 /
 * 16x16x32_f16 and the kernel multiplies the accumulator by *_h2_descale = 1/s.  Per product the
 * representation error is <= ~2^-22 |a||b|, below the fp32 accumulation error of the K >= 96
 * contractions it feeds.  Layout: the bf16x3 layout above with two parts (hi, lo) of fp16:
 *   CW = 32: [part p 2][m 2][lane 64][j 8];  CW = 16: [part p 2][lane 64][j 8]  (fp16),
 * i.e. the same bytes per block as the fp32 image.
 */
#define NBX_SEGNN_MAX_LAYERS 64

/* Cross-rank sum hook: sums `count` doubles at device address `buf` over all ranks in place;
 * the reduction must be ordered after the work already enqueued on `stream` and before the work
 * enqueued after the call returns.  Returns 0 on success. */
typedef int (*nbx_allreduce_fn)(double* buf, int64_t count, void* stream, void* ctx);

typedef struct nbx_segnn_layer {
    const float* node_pre_s_img; /* image of [6*mul][mul] x_s -> [P_dst(2mul) R_dst(mul) P_src(2mul) R_src(mul)] */
    const float* node_pre_v_img; /* image of [6*mul][mul] x_v[:,k] -> [Q_dst(2mul) S_dst(mul) Q_src(2mul) S_src(mul)] */
    const void* node_pre_s_img_x3; /* bf16x3 images of the same (CW = 16), or NULL */
    const void* node_pre_v_img_x3;
    const float* msg1_amf;     /* [2][3*mul]    amf (dist, m_i m_j) -> [s(2mul) t(mul)] */
    const float* msg1_bias;    /* [2*mul] */
    const float* msg2_img;     /* parts of [3*mul][2*mul] [m_s | m_v.rhat] -> [s | gate | t] + [mul][mul] m_v[:,k] -> v */
    const void* msg2_img_x3;   /* the same operand as a bf16x3 split image ("bf16x3 images"), or NULL */
    const float* msg2_bias;    /* [2*mul] */
    const float* upd1_img;     /* [3*mul][4*mul] [x_s a_s x_v.na a_v.na] -> [s | gate | t] + [mul][2*mul] -> v */
    const void* upd1_img_x3;   /* bf16x3 image of the same (CW = 16), or NULL */
    const float* upd1_bias;    /* [2*mul] */
    const float* upd2_img;     /* [2*mul][2*mul] [h_s | h_v.na] -> [s | t] + [mul][mul] -> v */
    const float* upd2_bias;    /* [mul] */
    /* e3nn BatchNorm(hidden): weight [2mul], bias [mul], running_mean [mul],
       running_var [2mul]; running stats are updated in place in train mode. */
    const float* msg_bn_weight;
    const float* msg_bn_bias;
    float* msg_bn_running_mean;
    float* msg_bn_running_var;
    const float* feat_bn_weight;
    const float* feat_bn_bias;
    float* feat_bn_running_mean;
    float* feat_bn_running_var;
    /* ABI 15: fp16x2 images ("fp16x2 images") of node_pre (both images share one scale, CW = 16),
     * msg2 (CW = 32), upd1 and upd2 (CW = 16), and the factors that undo their weight scales */
    const void* node_pre_s_img_h2;
    const void* node_pre_v_img_h2;
    const void* msg2_img_h2;
    const void* upd1_img_h2;
    const void* upd2_img_h2;
    float node_pre_h2_descale;
    float msg2_h2_descale;
    float upd1_h2_descale;
    float upd2_h2_descale;
} nbx_segnn_layer;

typedef struct nbx_segnn_weights {
    int32_t mul;        /* hidden multiplicity: hidden irreps = mul x 0e + mul x 1o */
    int32_t num_layers; /* <= NBX_SEGNN_MAX_LAYERS */
    int32_t training;   /* 1: BatchNorm uses batch statistics (the reference rollout), 0: running stats */
    float bn_eps;       /* 1e-5 */
    float bn_momentum;  /* 0.1 */
    const float* emb;      /* [6][mul]: W_a[0], W_a[1], W_b[0]/sqrt3, W_b[1]/sqrt3, W_c, W_d */
    const float* emb_bias; /* [mul] */
    const float* pp1_img;  /* pre_pool1 (gate TP, node attrs): [3*mul][2*mul] + [mul][mul] */
    const float* pp1_bias; /* [2*mul] */
    const float* pp2;      /* [2][2][mul]: (s->1o, v->1o) x (out channel 0, 1) */
    /* SyncBN (the multi-GPU form of the reference's train-mode BatchNorm, models/segnn/segnn.py:233-235,
     * 257-261, 282-283): when non-NULL and training, the library calls bn_allreduce after each
     * producing kernel to sum a layer's [3][mul] fp64 BatchNorm sums (sum s, sum s^2 over the 0e
     * channels, sum |v|^2 over the 1o channels) over every rank, in place, ordered on `stream`
     * (e.g. an RCCL all-reduce enqueued on it), and normalises by the global counts of
     * bn_global_batch systems (0: this call's batch).  12 calls per forward at 6 layers.  Requires
     * the atomic BatchNorm path (mul 96 or 32, 2 <= N <= 16); NBX_E_UNSUPPORTED otherwise. */
    nbx_allreduce_fn bn_allreduce;
    void* bn_allreduce_ctx;
    int64_t bn_global_batch;
    /* ABI 10.  bn_comm: an RCCL communicator from nbx_comm_init.  When non-NULL and training, the
     * library enqueues the SyncBN all-reduce itself (ncclAllReduce of the [3][mul] fp64 sums on
     * `stream`; takes precedence over bn_allreduce): no host round trip, graph-capturable.  Also
     * available on general (kNN) graphs, through the fixed-order reduction below.
     * deterministic: 1 = the BatchNorm batch sums are reduced from per-block partial rows in a fixed
     * order (one small launch per BatchNorm) instead of fp64 atomics, so train-mode forwards and
     * rollouts are bit-reproducible (measured cost: DESIGN.md §3.3); 0 = atomics (default). */
    void* bn_comm;
    int32_t deterministic;
    int32_t reserved0;
    /* ABI 15: pre_pool1's fp16x2 image (CW = 16) and descale, or NULL */
    const void* pp1_img_h2;
    float pp1_h2_descale;
    int32_t reserved1;
    nbx_segnn_layer layers[NBX_SEGNN_MAX_LAYERS];
} nbx_segnn_weights;

/* RCCL communicators for nbx_segnn_weights.bn_comm (ABI 10), one process per GPU: rank 0 calls
 * nbx_comm_unique_id, the id (NBX_COMM_ID_BYTES opaque bytes) travels to every rank over any
 * channel (torch.distributed.broadcast_object_list), then every rank calls nbx_comm_init with its
 * rank and HIP device (collective: blocks until all ranks arrive).  nbx_comm_allreduce_f64 sums
 * `count` doubles in place on `stream`.  No reference counterpart: the reference runs one
 * process on one GPU (SURVEY §2.1 "Parallelism strategies"). */
#define NBX_COMM_ID_BYTES 128
int nbx_comm_unique_id(void* id_out);
int nbx_comm_init(const void* id, int32_t nranks, int32_t rank, int32_t device, void** comm_out);
int nbx_comm_destroy(void* comm);
int nbx_comm_allreduce_f64(double* buf, int64_t count, void* comm, void* stream);

/* Bytes of device workspace nbx_segnn_forward / nbx_segnn_rollout need. */
int nbx_segnn_workspace_bytes(int64_t batch_size, int64_t num_nodes, int32_t mul, size_t* bytes);

/* O3Transform + catch_isolated_nodes + SEGNN.forward in one call
 * (infer_self_feed.py:115-130 graph build and model(graph)).
 * pos/vel [B*N,3], mass [B*N] fp32 -> out [B*N, 6] = (2x1o: delta-pos, vel).
 * Train mode (w->training = 1): the BatchNorm batch statistics are fp64 sums accumulated
 * with device-scope atomics, so repeated calls can differ in the last float bits (eval mode
 * is bit-reproducible; w->deterministic = 1 makes train mode bit-reproducible too); the running
 * statistics are updated in place as in the reference. */
int nbx_segnn_forward(const nbx_segnn_weights* w, const float* pos, const float* vel, const float* mass,
                      int64_t batch_size, int64_t num_nodes, float* out, void* workspace, size_t workspace_bytes,
                      void* stream);

/* Diagnostic variant of nbx_segnn_forward used by bench.py: records a HIP event
 * pair around every launch of the fused tensor-product kernels on `stream`,
 * synchronises at the end (so it is NOT graph-capturable) and reports, per
 * kernel kind (0 node_pre, 1 edge message, 2 gated node TP, 3 residual node TP),
 * the summed time (ms), the launch count and the executed FLOPs (2*MACs), plus
 * the whole forward's time.  Arrays have 4 entries. */
int nbx_segnn_forward_timed(const nbx_segnn_weights* w, const float* pos, const float* vel, const float* mass,
                            int64_t batch_size, int64_t num_nodes, float* out, void* workspace, size_t workspace_bytes,
                            void* stream, float* kind_ms, int32_t* kind_launches, double* kind_flops, float* total_ms);

/* Device-resident self-feed rollout (helper_scripts/infer_self_feed.py:99-194,
 * force zeroed, mass constant): starting from pos/vel [B,N,3] it runs num_frames-1
 * model steps; traj_pos/traj_vel [B, num_frames, N, 3] receive frame 0 = the initial
 * state and frame t = the state after t steps.  flags: 0 (target "pos_dt+vel":
 * pos += pred[:, :3]) or NBX_ROLLOUT_ABSOLUTE (pos = pred[:, :3]); vel = pred[:, 3:].
 * pos/vel are updated to the final state.  No host synchronisation inside (except
 * what a SyncBN hook does). */
int nbx_segnn_rollout(const nbx_segnn_weights* w, float* pos, float* vel, const float* mass,
                      int64_t batch_size, int64_t num_nodes, int64_t num_frames, int32_t flags,
                      float* traj_pos, float* traj_vel, void* workspace, size_t workspace_bytes, void* stream);

/* General graphs (ABI 8).  nbx_segnn_forward on the graph `edge_index` (int64 [2][num_edges],
 * device memory, row = source, col = target: the layout of build_graph_with_knn,
 * utils/build_fully_connected_graph.py:23-80, e.g. its kNN branch with num_neighbors < N-1) instead
 * of the fully-connected pattern: messages flow source -> target and aggregate at the target
 * (MessagePassing aggr="add"), node attributes average the edge attributes over a node's incoming
 * edges (0 for a node without any, O3Transform's scatter mean), the message BatchNorm counts the real
 * edges.  Every edge must join two different nodes of one system, without duplicates; returns
 * NBX_E_INVAL otherwise.  Synchronises `stream` once (the validation).  Not with SyncBN. */
int nbx_segnn_forward_graph(const nbx_segnn_weights* w, const float* pos, const float* vel, const float* mass,
                            int64_t batch_size, int64_t num_nodes, const int64_t* edge_index, int64_t num_edges,
                            float* out, void* workspace, size_t workspace_bytes, void* stream);

/* nbx_segnn_rollout with the reference's num_neighbors (infer_self_feed.py:58,121-123): every frame's
 * graph is the kNN graph of that frame's positions (build_graph_with_knn's kNN branch, selected on
 * the device as nbx_knn_edge_index does).  num_neighbors = N-1 or < 0 (None): the fully-connected
 * nbx_segnn_rollout; >= N: NBX_E_INVAL (the reference's ValueError). */
int nbx_segnn_rollout_knn(const nbx_segnn_weights* w, float* pos, float* vel, const float* mass,
                          int64_t batch_size, int64_t num_nodes, int64_t num_frames, int32_t flags,
                          int64_t num_neighbors, float* traj_pos, float* traj_vel, void* workspace,
                          size_t workspace_bytes, void* stream);

/* fp16x2 range guard (ABI 17).  The fp16x2 split tensor products (include/nbx.h "fp16x2 images", the
 * default SEGNN path) represent an fp32 operand a as hi + lo, both fp16: fp32-accurate for |a| < 65504,
 * while an operand at |a| >= 65520 rounds to an fp16 infinity.  Every split-precision kernel of a
 * nbx_segnn_forward / _forward_graph / _rollout / _rollout_knn call raises a flag in the call's
 * workspace when one of its output tiles is not finite (such an operand, or a non-finite input);
 * the flag covers every frame of a rollout.  This call waits for `stream`, reads the flag of the last
 * call made with `workspace` and returns NBX_E_RANGE (with a message) if it is set, NBX_OK otherwise.
 * The fp32 MFMA and bf16x3 paths (NBX_X3=0, NBX_SPLIT=x3) have the fp32 exponent range.  Synchronises. */
int nbx_segnn_range_check(const void* workspace, size_t workspace_bytes, int64_t batch_size, int64_t num_nodes,
                          int32_t mul, void* stream);

/* Diagnosis of msg_pre's exchange-buffer hand-off (ABI 17).  With the environment variable
 * NBX_MP_CHECK=1 set before the first SEGNN call, the fp16x2 message_layer_1 kernel runs an instantiation in
 * which every wave checks the stage tag of the exchange buffer it consumes (the group its hand-off
 * counters promise) and counts and printfs each mismatch; NBX_MP_CHECK=2 also drops the edge waves' wait
 * (fault injection, for the test that the check fires).  Writes the count so far (0 when the check is
 * off) and resets it if `reset`.  Synchronises the device. */
int nbx_debug_msg_pre_check(uint32_t* mismatches, int32_t reset);


/* ------------------------------------------------------------------------
 * SEGNN training step (ABI 10; SURVEY §8(f)4: trainer.py:233-358, pred = model(graph) with the
 * train-mode BatchNorm of models/segnn/segnn.py:233-235, loss.backward()).  The training forward and
 * backward are composed (segnn_train.py, autograd) of the operators below; every O(3) tensor product
 * of SEGNN (o3_building_blocks.py:10-203) is one canonical form
 *   S_in = [XS | sum_k XV[k] * Y3[:, k]],  Zs = S_in Ws^T,  Zv[k] = XV[k] Wv^T,
 *   OS = Zs[:, :Ms] + b (gated: c_silu SiLU), OV[k] = Y3[:, k] Zs[:, NSc + w] + Zv[k]
 *        (gated: times c_sig sigmoid(Zs[:, Ms + w] + b[Ms + w]); NSc = Ms (+ Nt gates))
 * with e3nn's path constants and the SH prefactors folded into Ws / Wv (segnn.py train_matrices).
 * Layouts: row-major, vector features as 3 component planes [3][rows][C].  All reductions run in a
 * fixed order (bit-reproducible).  fp32. */

/* C = op(A) op(B) (+ C if beta = 1), C [M][N] (ldc); op(A) [M][K]: A stored [M][K] (lda) or, with
 * NBX_GEMM_TRANS_A, [K][M]; op(B) [K][N]: B stored [K][N] (ldb) or, with NBX_GEMM_TRANS_B, [N][K].
 * fp32 MFMA (v_mfma_f32_32x32x2_f32), 64 x 64 tiles; small-M N, long-K products (weight gradients)
 * split K over the workspace (nbx_gemm_f32_workspace_bytes) and sum the splits in order.  Large
 * C = A B^T products (flags exactly NBX_GEMM_TRANS_B, plain rows, no K split, K >= 64, N >= 96, >= 2^30
 * multiply-adds, 16-byte aligned operands; in a batched / grouped launch: when every problem qualifies)
 * run on the bf16x3 split MFMA since r06: six bf16 products per fp32 product, fp32 accumulation,
 * fp32-level accuracy but not bitwise the fp32-MFMA result; NBX_GEMM_X3=0 keeps them on fp32 MFMA. */
#define NBX_GEMM_TRANS_A 1
#define NBX_GEMM_TRANS_B 2
/* op(B) gains a last column of ones (n = N - 1 reads 1, not memory; B holds N - 1 columns): C's last
 * column is then the row sums of op(A) -- a bias gradient from the weight-gradient GEMM (ABI 14) */
#define NBX_GEMM_B_ONES 4
/* with NBX_GEMM_B_ONES: C's last column (the row sums) is stored as the contiguous vector C + M ldc
 * instead of column N - 1 (ldc >= N - 1), so a weight gradient [M][N - 1] (ldc = N - 1) and its bias
 * gradient [M] both come out contiguous, one buffer of M N floats (ABI 16) */
#define NBX_GEMM_ONES_TAIL 8
int nbx_gemm_f32_workspace_bytes(int64_t M, int64_t N, int64_t K, size_t* bytes);
/* ABI 12.  Up to 4 (ABI 16: 8) independent nbx_gemm_f32 problems in one launch (plus one launch for every split-K
 * sum): problem i has flags[i], dims[6 i ..] = (M, N, K, lda, ldb, ldc), A[i], B[i], C[i], beta[i]
 * (0 or 1), each with the operand layouts, blocking and split-K order of nbx_gemm_f32, so its result
 * is bit-identical.  Host arrays; workspace from nbx_gemm_f32_batched_workspace_bytes.  Replaces the
 * separate launches of one tensor product's GEMMs in the training step (segnn_train.py). */
int nbx_gemm_f32_batched_workspace_bytes(int32_t count, const int64_t* dims, size_t* bytes);
int nbx_gemm_f32_batched(int32_t count, const int32_t* flags, const int64_t* dims, const float* const* A,
                         const float* const* B, float* const* C, const float* beta, void* workspace,
                         size_t workspace_bytes, void* stream);
int nbx_gemm_f32(int32_t flags, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* B,
                 int64_t ldb, float* C, int64_t ldc, float beta, void* workspace, size_t workspace_bytes, void* stream);
/* ABI 16.  nbx_gemm_f32_batched with two-level rows: dims[10 i ..] = (M, N, K, lda, ldb, ldc, rdiv, oa, ob,
 * oc); row r of a row-major operand (A's [M][K] or [K][M] rows, B's [K][N] or [N][K] rows, C's rows)
 * whose outer stride (oa / ob / oc) is non-zero sits at (r / rdiv) outer + (r % rdiv) ld (outer >=
 * rdiv ld), so the 2l + 1 rows of degree l of every node of an [nodes][(lmax + 1)^2][C] array are one
 * operand of nodes (2l + 1) rows: SO3_LinearV2 (equiformer_v2 so3.py:695-745) forward and backward for
 * all degrees in one launch, without per-degree copies (eqv2_train.py _SO3LinearFn).  Up to 8
 * problems (both grouped entry points since ABI 16); NBX_GEMM_ONES_TAIL needs oc = 0.  bias (host array of
 * count device pointers, or NULL): C(r, n) = op(A) op(B) + bias[i][n] (+ C), the nn.Linear bias in the
 * GEMM's epilogue / split-K sum (not with NBX_GEMM_B_ONES). */
int nbx_gemm_f32_grouped_workspace_bytes(int32_t count, const int64_t* dims, size_t* bytes);
int nbx_gemm_f32_grouped(int32_t count, const int32_t* flags, const int64_t* dims, const float* const* A,
                         const float* const* B, float* const* C, const float* beta, const float* const* bias,
                         void* workspace, size_t workspace_bytes, void* stream);

/* S_in [rows][Ks + Kv] from XS (rows x Ks, leading dimension ldxs), XV [3][rows][Kv], Y3 [rows][3];
 * backward: dXS = dS[:, :Ks] (written when non-NULL), dXV[k] += Y3[:, k] dS[:, Ks:] (accumulated). */
int nbx_tp_prep(int64_t rows, int32_t Ks, int32_t Kv, const float* XS, int64_t ldxs, const float* XV, const float* Y3,
                float* S, void* stream);
int nbx_tp_prep_backward(int64_t rows, int32_t Ks, int32_t Kv, const float* dS, const float* Y3, float* dXS,
                         int64_t lddxs, float* dXV, void* stream);

/* The TP epilogue: Zs [rows][NSc + Nt], Zv [3][rows][Nt] -> OS [rows][Ms], OV [3][rows][Nt] (+ the
 * optional residuals RS / RV: x + update, segnn.py:303); gate = e3nn Gate(SiLU, sigmoid)
 * (o3_building_blocks.py:187-203).  Backward: dOS, dOV -> dZs, dZv (the bias gradient is the column
 * sum of dZs[:, :NSc], nbx_colsum). */
int nbx_tp_post(int64_t rows, int32_t Ms, int32_t Nt, int32_t gate, const float* Zs, const float* Zv, const float* Y3,
                const float* bias, const float* RS, const float* RV, float* OS, float* OV, void* stream);
int nbx_tp_post_backward(int64_t rows, int32_t Ms, int32_t Nt, int32_t gate, const float* Zs, const float* Zv,
                         const float* Y3, const float* bias, const float* dOS, const float* dOV, float* dZs, float* dZv,
                         void* stream);

/* out[c] (+)= sum over rows of X[r][c] (fixed order, fp64 partials). */
int nbx_colsum_workspace_bytes(int64_t rows, int32_t cols, size_t* bytes);
int nbx_colsum(int64_t rows, int32_t cols, const float* X, int64_t ld, float* out, int32_t accumulate, void* workspace,
               size_t workspace_bytes, void* stream);

/* e3nn BatchNorm with batch statistics (train mode) of M 0e channels S [rows][M]
 * and M 1o channels V [3][rows][M]: OS = (S - mu) w / sqrt(var + eps) + b, OV = V w_v / sqrt(n + eps),
 * n = mean over rows and components of V^2; running stats updated in place (momentum) when non-NULL;
 * save [3][M] = (mu, 1/sqrt(var + eps), 1/sqrt(n + eps)) for the backward, which returns dS, dV and
 * the parameter gradients dweight [2M] (0e then 1o), dbias [M]. */
int nbx_bn_train_workspace_bytes(int64_t rows, int32_t M, size_t* bytes);
int nbx_bn_train_forward(int64_t rows, int32_t M, const float* S, const float* V, const float* weight, const float* bias,
                         float* running_mean, float* running_var, float eps, float momentum, float* save, float* OS,
                         float* OV, void* workspace, size_t workspace_bytes, void* stream);
int nbx_bn_train_backward(int64_t rows, int32_t M, const float* S, const float* V, const float* weight,
                          const float* save, const float* dOS, const float* dOV, float* dS, float* dV, float* dweight,
                          float* dbias, void* workspace, size_t workspace_bytes, void* stream);

/* SyncBN training step (sharded train-mode BatchNorm; the reference trains on one device, so the
 * statistics of a sharded step are those of the whole global batch): nbx_bn_train_sums writes
 * sums [3M + 1] fp64 -- the forward sums (sum s, sum s^2, sum |v|^2) when dOS / dOV are NULL, the
 * backward sums (sum dy_s, sum dy_s xhat, sum dy_v . v) otherwise -- and sums[3M] = rows; the caller
 * all-reduces them over the ranks (one collective of 3M + 1 doubles); nbx_bn_train_apply /
 * nbx_bn_train_backward_apply then normalise / back-propagate with the all-reduced sums and count.
 * nbx_bn_train_param_grads: dweight / dbias from the LOCAL backward sums (the data-parallel gradient
 * all-reduce sums them over the ranks); scratch [3M] doubles. */
int nbx_bn_train_sums(int64_t rows, int32_t M, const float* S, const float* V, const float* dOS, const float* dOV,
                      const float* save, double* sums, void* workspace, size_t workspace_bytes, void* stream);
int nbx_bn_train_apply(int64_t rows, int32_t M, const float* S, const float* V, const float* weight, const float* bias,
                       const double* sums, float* running_mean, float* running_var, float eps, float momentum,
                       float* save, float* OS, float* OV, void* stream);
int nbx_bn_train_param_grads(int32_t M, const float* save, const double* local_sums, double* scratch, float* dweight,
                             float* dbias, void* stream);
int nbx_bn_train_backward_apply(int64_t rows, int32_t M, const float* S, const float* V, const float* weight,
                                const float* save, const double* sums, const float* dOS, const float* dOV, float* dS,
                                float* dV, void* stream);

/* Message passing (MessagePassing aggr="add", segnn.py:249): out[r] = in[idx[r]] per plane (x_i = x[dst],
 * x_j = x[src]) and out[n] (+)= sum over j in [ptr[n], ptr[n+1]) of in[eid[j]] (a CSR of the edges by
 * destination / source; the aggregation and the gathers' adjoint).  planes: component planes, strides
 * plane_in / plane_out. */
int nbx_gather_rows(int64_t n, int32_t cols, const int32_t* idx, const float* in, int64_t ld_in, int64_t plane_in,
                    float* out, int64_t ld_out, int64_t plane_out, int32_t planes, void* stream);
int nbx_segment_sum(int64_t n, int32_t cols, const int32_t* ptr, const int32_t* eid, const float* in, int64_t ld_in,
                    int64_t plane_in, float* out, int64_t ld_out, int64_t plane_out, int32_t planes,
                    int32_t accumulate, void* stream);

/* O3Transform + catch_isolated_nodes on an edge list (src, dst int32 [E]; dst_ptr [V+1] / dst_eid [E]:
 * the edges grouped by destination): na3 [V][3] (the l=1 node attribute), xs0 [V] = |vel|,
 * xv0 [3][V][2] = (pos - mean_xyz(pos), vel), rhat [E][3], amf [E][2] = (|rel|, m_src m_dst). */
int nbx_segnn_train_featurize(int64_t V, int64_t E, const float* pos, const float* vel, const float* mass,
                              const int32_t* src, const int32_t* dst, const int32_t* dst_ptr, const int32_t* dst_eid,
                              float* na3, float* xs0, float* xv0, float* rhat, float* amf, void* stream);

/* ------------------------------------------------------------------------
 * PONITA training step (ABI 11; SURVEY §8(f)4: trainer.py:233-358 on PONITA_NBODY,
 * models/ponita/models/ponita_pg.py:134-192, nn/conv.py:103-133, nn/convnext.py:18-32).  The training
 * forward and backward (ponita_train.py, autograd) are composed of nbx_gemm_f32 (every nn.Linear),
 * nbx_colsum (bias / LayerNorm parameter gradients), the CSRs of nbx_segment_sum's convention and
 * the operators below, on the fibre-bundle layout: node rows [V][O][C], edge rows [E][O][*], fibre
 * rows [O][O][*] (o major).  fp32; every reduction in a fixed order (bit-reproducible).
 */
#define NBX_ACT_NONE 0
#define NBX_ACT_GELU 1   /* nn.GELU(): 0.5 x (1 + erf(x / sqrt 2)) */
#define NBX_ACT_SILU 2   /* nn.SiLU(): x sigmoid(x) */
#define NBX_ACT_SLRELU 3 /* SmoothLeakyReLU(0.2): 0.6 x + 0.4 x (2 sigmoid(x) - 1) */

/* Invariants + degree-3 polynomial features (no gradient): attr [E*O][16] (16-byte aligned) =
 * poly(r.o, |r - (r.o) o|) (14 features, 2 zero pads), r = pos[src] - pos[dst]; fiber [O*O][4] =
 * (s, s^2, s^3, 0), s = o_p . o_o; lift [V*O][2] = (mass, vel . o). */
int nbx_ponita_train_featurize(int64_t V, int64_t E, int32_t O, const float* pos, const float* vel, const float* mass,
                               const float* ori_grid, const int32_t* src, const int32_t* dst, float* attr, float* fiber,
                               float* lift, void* stream);

/* Y[r][c] = act(Z[r][c] + bias[c]) (bias may be NULL); backward dZ = dY act'(Z + bias), dY / dZ
 * contiguous [rows][cols]. */
int nbx_bias_act(int64_t rows, int32_t cols, const float* Z, int64_t ldz, const float* bias, int32_t act, float* Y,
                 int64_t ldy, void* stream);
int nbx_bias_act_backward(int64_t rows, int32_t cols, const float* Z, int64_t ldz, const float* bias, int32_t act,
                          const float* dY, float* dZ, void* stream);

/* Separable spatial message, aggr "add" at edge_index[1]: X1[v][o][c] = sum over the edges e into v
 * (dst CSR) of K[e][o][c] H[src_e][o][c].  Backward: dK[e] = dX1[dst_e] H[src_e] (NULL: skipped) and
 * dH[u] = sum over the edges out of u (src CSR) of dX1[dst_e] K[e] (NULL: skipped). */
int nbx_po_message(int64_t V, int32_t O, int32_t C, const int32_t* dst_ptr, const int32_t* dst_eid, const int32_t* src,
                   const float* K, const float* H, float* X1, void* stream);
int nbx_po_message_backward(int64_t V, int64_t E, int32_t O, int32_t C, const int32_t* src, const int32_t* dst,
                            const int32_t* src_ptr, const int32_t* src_eid, const float* K, const float* H,
                            const float* dX1, float* dK, float* dH, void* stream);

/* Depth-wise fibre convolution X2[v][p][c] = (sum_o X1[v][o][c] FK[o][p][c]) / O + bias[c];
 * backward dX1 (NULL: skipped) and dFK (summed over the nodes in fixed chunks; workspace). */
int nbx_po_fiber_conv(int64_t V, int32_t O, int32_t C, const float* X1, const float* FK, const float* bias, float* X2,
                      void* stream);
int nbx_po_fiber_conv_workspace_bytes(int64_t V, int32_t O, int32_t C, size_t* bytes);
int nbx_po_fiber_conv_backward(int64_t V, int32_t O, int32_t C, const float* X1, const float* FK, const float* dX2,
                               float* dX1, float* dFK, void* workspace, size_t workspace_bytes, void* stream);

/* LayerNorm over C <= 1024 channels (biased variance): save [2][rows] = (mean, 1/sqrt(var + eps));
 * backward dX and G [rows][2C] = (dY xhat | dY), whose column sums are dweight | dbias. */
int nbx_layernorm_forward(int64_t rows, int32_t C, const float* X, const float* weight, const float* bias, float eps,
                          float* Y, float* save, void* stream);
int nbx_layernorm_backward(int64_t rows, int32_t C, const float* X, const float* weight, const float* save,
                           const float* dY, float* dX, float* G, void* stream);

/* ------------------------------------------------------------------------
 * EquiformerV2 training step (ABI 11; SURVEY §8(f)4: trainer.py:233-358 on EquiformerV2_nbody,
 * equiformer_v2_nbody.py:392-575, lmax 2 / mmax 1).  The training forward and backward
 * (eqv2_train.py, autograd) are composed of nbx_gemm_f32, nbx_bias_act (SiLU, SmoothLeakyReLU),
 * nbx_layernorm_*, nbx_colsum, nbx_gather_rows / nbx_segment_sum and the operators below.  Layout:
 * node irreps [V][9][C] (l-primary coefficients, channels contiguous), edge irreps [E][7][C] (the
 * |m| <= 1 coefficients, l-primary), fully-connected edges in build_graph_with_knn order.
 */

/* Edge frames (edge_rot_mat.py:6-63 with the gauge draws of nbx_eqv2_forward: `gauge` [E][3] or the
 * device hash of `seed`): dsel [E][7][9] = the |m| <= 1 rows of the block Wigner matrix
 * (so3.py:485-531), dist [E] = |pos_src - pos_dst|, zn [V] = clamp(int(mass)); rot_scratch [E][32]. */
int nbx_eqv2_train_edges(int64_t B, int64_t N, const float* pos, const float* mass, const float* gauge, uint64_t seed,
                         int32_t num_elements, float* rot_scratch, float* dsel, float* dist, int32_t* zn, void* stream);

/* SO3_Rotation.rotate (inverse = 0: out [E][7][C] = dsel in, in [E][9][C] with `ld_in` floats per edge)
 * and rotate_inv (inverse = 1: out [E][9][C] = dsel^T in, in [E][7][C]); rescale = 1 multiplies the
 * l = 2 block by sqrt(5/3) (get_rotate_inv_rescale, so3.py:160-185).  Each is the other's adjoint. */
int nbx_eqv2_rotate(int64_t E, int32_t C, const float* dsel, const float* in, int64_t ld_in, float* out,
                    int32_t inverse, int32_t rescale, void* stream);

/* Separable S2 activation, grid part (activation.py:155-202): out[r][i][h] = sum_p F[p][i]
 * SiLU(sum_j T[p][j] X[r][j][h]), X / out [rows][I][H], T / F [P][I] (SO3_Grid to / from grid
 * matrices), I <= 49, P <= 240 (ABI 13; lmax 6: SO3_Grid(6, 6) has 14 x 15 points); backward dX from dOut. */
int nbx_eqv2_s2_act(int64_t rows, int32_t I, int32_t P, int32_t H, const float* to_grid, const float* from_grid,
                    const float* X, float* out, void* stream);
int nbx_eqv2_s2_act_backward(int64_t rows, int32_t I, int32_t P, int32_t H, const float* to_grid,
                             const float* from_grid, const float* X, const float* dOut, float* dX, void* stream);

/* torch_geometric softmax of logits [E][nh] over edge_index[1] (dst CSR), + 1e-16 in the denominator
 * (transformer_block.py:331-339), and its backward. */
int nbx_segment_softmax(int64_t V, int32_t nh, const int32_t* dst_ptr, const int32_t* dst_eid, const float* logits,
                        float* alpha, void* stream);
int nbx_segment_softmax_backward(int64_t V, int32_t nh, const int32_t* dst_ptr, const int32_t* dst_eid,
                                 const float* alpha, const float* dalpha, float* dlogits, void* stream);

/* EquivariantRMSNormArraySphericalHarmonicsV2 (layer_norm.py:327-441, lmax 2, C <= 128) of X [V][9][C]:
 * weight [3][C], bias [C]; save [2][V]; backward dX and G [V][4C] whose column sums are
 * dweight [3][C] | dbias [C]. */
int nbx_eqv2_rms_norm(int64_t V, int32_t C, const float* X, const float* weight, const float* bias, float eps, float* Y,
                      float* save, void* stream);
int nbx_eqv2_rms_norm_backward(int64_t V, int32_t C, const float* X, const float* weight, const float* save,
                               const float* dY, float* dX, float* G, void* stream);

/* ------------------------------------------------------------------------
 * EquiformerV2 at general degrees (ABI 13; lmax <= 6, mmax <= lmax: the reference constructor's
 * default lmax_list = [6], mmax_list = [2], equiformer_v2_nbody.py:122-123).  The composed forward
 * and training step (eqv2_train.py) use these with the operators above.  Layout: node irreps
 * [V][(lmax+1)^2][C] (l-primary), edge irreps [E][R][C] with the R kept (|m| <= mmax) coefficients
 * (l-primary, coefficient_idx of so3.py:117-157), dsel [E][S]: per degree l the kept rows of D^l,
 * [2 min(l, mmax)+1][2l+1], back to back (S from nbx_eqv2_dsel_floats).
 */

/* nbx_eqv2_train_edges without the lmax-2 rows and with the gauge counter's frame index (the draws
 * of nbx_eqv2_rollout's frame `frame`): rot_scratch [E][32] (R, the edge frame, in floats 0..8),
 * dist [E], zn [V]. */
int nbx_eqv2_edges(int64_t B, int64_t N, const float* pos, const float* mass, const float* gauge, uint64_t seed,
                   int64_t frame, int32_t num_elements, float* rot_scratch, float* dist, int32_t* zn, void* stream);

/* Sizes: the probe table of nbx_eqv2_wigner (host-built: so3.py wigner_table) and S. */
int nbx_eqv2_wigner_table_floats(int32_t lmax, int64_t* floats);
int nbx_eqv2_dsel_floats(int32_t lmax, int32_t mmax, int64_t* floats);

/* Kept Wigner rows of every edge frame (SO3_Rotation.set_wigner, so3.py:485-531; Y(R u) = D(R) Y(u)
 * in e3nn's basis): R = rot[e * ld_rot + 0..8] (rows), D^0 = 1, D^1 = R, D^l = [Y^l(R u_k)]_k P_l from
 * the table's probe vectors u_k and P_l = pinv([Y^l(u_k)]_k). */
int nbx_eqv2_wigner(int64_t E, int32_t lmax, int32_t mmax, const float* rot, int64_t ld_rot, const float* table,
                    float* dsel, void* stream);

/* rotate (inverse = 0: out [E][R][C] = dsel in, in [E][(lmax+1)^2][C] with ld_in floats per edge) and
 * rotate_inv (inverse = 1: out [E][(lmax+1)^2][C] = dsel^T in, in [E][R][C]); rescale = 1 multiplies
 * degree l > mmax by float32(sqrt((2l+1)/(2 mmax+1))) (get_rotate_inv_rescale, so3.py:160-185), so
 * each direction with the same rescale is the other's adjoint.  order [R] (nullable): the row of the
 * [E][R][C] side that holds kept coefficient k (l-primary) -- the m-primary order of SO2_Convolution
 * (so3.py:30-115 to_m) keeps the SO(2) blocks contiguous. */
int nbx_eqv2_rotate_general(int64_t E, int32_t C, int32_t lmax, int32_t mmax, const float* dsel, const float* in,
                            int64_t ld_in, float* out, int32_t inverse, int32_t rescale, const int32_t* order,
                            void* stream);

/* ABI 19.  The attention's gathered message rotated in one pass (transformer_block.py:281-289 then
 * SO3_Rotation.rotate): out [E][R][2C] = rotate of in'[e] = [X[src[e]] | X[dst[e]]] per coefficient,
 * X [V][(lmax+1)^2][C] with ld_x floats per node, src / dst int32 [E]; rescale and order as
 * nbx_eqv2_rotate_general with inverse = 0, and bit-identical to it on the materialised in' (which is
 * never written).  Its adjoint is nbx_eqv2_rotate_general (inverse = 1) followed by the segment sums of
 * the gather.  rad (nullable, inference): out[e][j][c] is multiplied by rad[e ld_rad + radrow[j] 2C + c],
 * SO2_Convolution's radial weights (so2_ops.py:118-121, one per (m, coefficient, channel), shared by the
 * +m / -m rows; radrow int32 [R] maps each output row to its radial block row), bit-identical to the
 * separate product. */
int nbx_eqv2_rotate_gather(int64_t E, int32_t C, int32_t lmax, int32_t mmax, const float* dsel, const float* X,
                           int64_t ld_x, const int32_t* src, const int32_t* dst, float* out, int32_t rescale,
                           const int32_t* order, const float* rad, int64_t ld_rad, const int32_t* radrow,
                           void* stream);

/* EquivariantRMSNormArraySphericalHarmonicsV2 (layer_norm.py:327-441) of X [V][(lmax+1)^2][C], any C:
 * weight [lmax+1][C], bias [C], balance weights float32(1/(2l+1)) / (lmax+1); save [2][V]; backward
 * dX and G [V][(lmax+2) C] whose column sums are dweight [lmax+1][C] | dbias [C]. */
int nbx_eqv2_rms_norm_general(int64_t V, int32_t lmax, int32_t C, const float* X, const float* weight,
                              const float* bias, float eps, float* Y, float* save, void* stream);
int nbx_eqv2_rms_norm_general_backward(int64_t V, int32_t lmax, int32_t C, const float* X, const float* weight,
                                       const float* save, const float* dY, float* dX, float* G, void* stream);

/* ------------------------------------------------------------------------
 * EGNN-MC (models/egnn_mc/egnn_mc.py:45-295 with the preprocessing of
 * dataloaders/egnn_mc_n_body_dataloader.py:8-56) — fp32.
 *
 * Native scope: SiLU activation, num_vectors_in = num_vectors_out = 1, attention
 * off, hidden_node_dim = hidden_edge_dim = hidden_coord_dim = hidden <= 128,
 * node_input_dim 2, edge_attr_dim 4, fully-connected systems.  Linear weights
 * are stored as W [out][K] (nn.Linear layout) with K zero-padded per input
 * segment to a multiple of 32; `Kp = ceil32(hidden)`:
 *   e0_t [hidden][2 Kp + 32]  (h_row | h_col | radial, edge_attr[4], 0...)
 *   n0_t [hidden][2 Kp]       (h | mean edge features)
 *   w0_t [hidden][Kp + 32]    (h | coord - pos, vel, 0...)
 *   emb_t [hidden][32]        (|vel|, mass, 0...)
 *   other *_t [out][Kp]; c1_w / v1_w [hidden] (the 128 -> 1 linears).
 */
#define NBX_EGNN_MAX_LAYERS 64

typedef struct nbx_egnn_layer {
    const float* e0_t; const float* e0_b;  /* edge_mlp.0 */
    const float* e1_t; const float* e1_b;  /* edge_mlp.2 */
    const float* c0_t; const float* c0_b;  /* coord_mlp.0 */
    const float* c1_w;                     /* coord_mlp.2 (no bias) */
    const float* v0_t; const float* v0_b;  /* coord_mlp_vel.0 */
    const float* v1_w; float v1_b;         /* coord_mlp_vel.2 */
    const float* n0_t; const float* n0_b;  /* node_mlp.0 */
    const float* n1_t; const float* n1_b;  /* node_mlp.2 */
} nbx_egnn_layer;

typedef struct nbx_egnn_head {
    const float* w0_t; const float* b0;   /* net.0 */
    const float* w1_t; const float* b1;   /* net.2 */
    const float* w2_t; const float* b2;   /* net.4 (-> 3) */
} nbx_egnn_head;

/* persist_blob (optional; NULL = the per-layer GEMM path): every weight once more, input-major
 * ([K][out], "_i"), contiguous, for the persistent per-system kernel (one workgroup per system runs
 * every layer, the heads and the whole rollout on chip; hidden in {32, 64, 128}, N <= 8):
 *   emb_i [2][H] | emb_b [H]
 *   per layer: e0_i [2H + 8][H] (h_row | h_col | radial, edge_attr[4], 0, 0, 0) | e0_b [H] | e1_i [H][H] |
 *              e1_b | c0_i [H][H] | c0_b | c1_w [H] | v0_i [H][H] | v0_b | v1_w [H] | v1_b [4] (1 used) |
 *              n0_i [2H][H] (h | agg) | n0_b | n1_i [H][H] | n1_b            (8 H^2 + 16 H + 4 floats)
 *   per head:  w0_i [H + 8][H] (h | coord - pos, vel, 0, 0) | b0 [H] | w1_i [H][H] | b1 [H] |
 *              w2_i [H][4] (3 used) | b2 [4]                                  (2 H^2 + 14 H + 4 floats) */
typedef struct nbx_egnn_weights {
    int32_t hidden, num_layers, num_heads, recurrent, norm_diff, use_tanh;
    float coords_weight;
    const float* emb_t; const float* emb_b;
    const float* persist_blob;
    nbx_egnn_head heads[2];
    nbx_egnn_layer layers[NBX_EGNN_MAX_LAYERS];
} nbx_egnn_weights;

int nbx_egnn_workspace_bytes(int64_t batch_size, int64_t num_nodes, int32_t hidden, size_t* bytes);

/* preprocess_batch + EGNNMultiChannel.forward: pos/vel [B*N,3], mass [B*N] ->
 * out [B*N, 3*num_heads] (heads in target order, e.g. pos_dt | vel). */
int nbx_egnn_forward(const nbx_egnn_weights* w, const float* pos, const float* vel, const float* mass,
                     int64_t batch_size, int64_t num_nodes, float* out, void* workspace, size_t workspace_bytes,
                     void* stream);

/* Device-resident self-feed rollout with the EGNN-MC branch of
 * infer_self_feed.py:161-194 (two heads: pos_dt, vel); same contract as
 * nbx_segnn_rollout. */
int nbx_egnn_rollout(const nbx_egnn_weights* w, float* pos, float* vel, const float* mass, int64_t batch_size,
                     int64_t num_nodes, int64_t num_frames, int32_t flags, float* traj_pos, float* traj_vel, void* workspace,
                     size_t workspace_bytes, void* stream);

/* kNN graphs (ABI 9; dataloaders/egnn_mc_n_body_dataloader.py:13-28 builds build_graph_with_knn's
 * graph when args.num_neighbors < N - 1; EGNNMultiChannel aggregates at row = edge_index[0], so every
 * node has exactly k edges).  nbx_egnn_forward_graph: nbx_egnn_forward on the graph whose edges
 * (b N + i, b N + nbr[(b N + i) k + q]), q < k, are node i's (int32 local indices, [B N][k]);
 * k == N - 1 with nbr == NULL is nbx_egnn_forward.  nbx_egnn_rollout_knn: nbx_egnn_rollout with
 * every frame's graph the kNN graph of that frame's positions (k == N - 1: nbx_egnn_rollout).
 * Both need 1 <= k < N and the persistent kernel's shapes (hidden 32 / 64 / 128, N <= 8), else
 * NBX_E_INVAL / NBX_E_UNSUPPORTED. */
int nbx_egnn_forward_graph(const nbx_egnn_weights* w, const float* pos, const float* vel, const float* mass,
                           int64_t batch_size, int64_t num_nodes, int64_t k, const int32_t* nbr, float* out,
                           void* workspace, size_t workspace_bytes, void* stream);
int nbx_egnn_rollout_knn(const nbx_egnn_weights* w, float* pos, float* vel, const float* mass, int64_t batch_size,
                         int64_t num_nodes, int64_t num_frames, int32_t flags, int64_t k, float* traj_pos,
                         float* traj_vel, void* workspace, size_t workspace_bytes, void* stream);

/* EGNN-MC training step (trainer.py:233-358: pred = model(graph); loss.backward()), ABI 7.
 * nbx_egnn_train_forward runs the forward of `batch_size` fully-connected systems of 2..8 bodies
 * (hidden % 4 == 0; the LDS bound allows N <= 6 at hidden 128) from the persist blob and keeps the
 * activations the backward needs in `workspace` (nbx_egnn_train_workspace_bytes: B x the per-system
 * save area + the backward's partial gradient slices); out [B N][3 heads] as nbx_egnn_forward.
 * nbx_egnn_train_backward, given dL/dout [B N][3 heads] and the same workspace, writes dL/dblob
 * (grad_blob: the persist blob's length and layout; every entry written, padding included) —
 * the gradient of every weight of models/egnn_mc/egnn_mc.py:211-295 through the embedding, all
 * _EGNNMessageBlock layers (edge / coord / velocity / node MLPs, the clamped coordinate update and
 * the coordinate geometry) and the vector heads.  Inputs (pos, vel, mass) are data: no gradient. */
int nbx_egnn_train_workspace_bytes(const nbx_egnn_weights* w, int64_t batch_size, int64_t num_nodes, size_t* bytes);
int nbx_egnn_train_forward(const nbx_egnn_weights* w, const float* pos, const float* vel, const float* mass,
                           int64_t batch_size, int64_t num_nodes, float* out, void* workspace, size_t workspace_bytes,
                           void* stream);
int nbx_egnn_train_backward(const nbx_egnn_weights* w, const float* pos, const float* vel, const float* mass,
                            int64_t batch_size, int64_t num_nodes, const float* grad_out, float* grad_blob,
                            void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * PONITA fibre bundle (models/ponita/ponita_nbody.py:9-95,
 * models/ponita/models/ponita_pg.py:56-192, nn/conv.py:65-140,
 * nn/convnext.py:4-32, transforms/, geometry/invariants.py:9-51) — fp32.
 *
 * Scope: num_ori orientations on S2 (<= 24), hidden C in {32, 64, 128},
 * basis_dim % 4 == 0, degree 3, in = (mass, vel), out = 2 vector channels,
 * radius None (identity window), fully-connected systems.  Weights as
 * W [out][K] with K zero-padded to a multiple of 32 (`Kp(x) = ceil32(x)`):
 *   basis1_t / fbasis1_t [C][32]        (14 / 3 polynomial features valid)
 *   basis2_t / fbasis2_t [Bk][Kp(C)]    (Bk = basis_dim)
 *   fiber_t  [L*C][Kp(Bk)]              (conv.fiber_kernel of every layer, stacked)
 *   kernel_t [C][Kp(Bk)]; lin1_t [4C][Kp(C)]; lin2_t [C][Kp(4C)]
 *   embed_w  [C][2] (x_embedder, no bias); readout_w [2][C].
 * The orientation grid ori_grid [O][3] is an input like any weight (the
 * reference draws it from the RNG at construction and does not persist it).
 */
#define NBX_PONITA_MAX_LAYERS 64

typedef struct nbx_ponita_layer {
    const float* kernel_t;            /* conv.kernel (no bias) */
    const float* conv_bias;           /* conv.bias [C] */
    const float* norm_w; const float* norm_b;   /* LayerNorm(C), eps 1e-5 */
    const float* lin1_t; const float* lin1_b;   /* linear_1 -> GELU */
    const float* lin2_t; const float* lin2_b;   /* linear_2 */
    const float* layer_scale;         /* [C] or NULL */
    const float* readout_w; const float* readout_b;  /* read_out_layers[i] or NULL */
    /* optional bf16x3 images of kernel_t / lin1_t / lin2_t (NULL: fp32 MFMA path): the
     * "bf16x3 images" layout with CW = 32 and one sub-tile, [N/32][K/32][3][2][64][8] bf16;
     * lin2's image is chunk-major, [K/32][N/32][3][2][64][8] (the row-panel GEMM streams K chunks) */
    const void* kernel_img_x3;
    const void* lin1_img_x3;
    const void* lin2_img_x3;
    /* optional (ABI 7): the fused ConvNext MLP's slabs, one per 32-wide hidden chunk j (NULL: the
     * two-GEMM path): [linear_1 rows 32j..32j+31 as (C/32) K-chunk blocks [3][2][64][8] bf16 (the
     * "bf16x3 images" block with the hidden units as rows)] [linear_2 columns of chunk j for the C/32
     * output tiles, same block layout, with the hidden index inside the chunk permuted: image slot
     * 16 h + 8 m + i holds hidden unit (i & 3) + 16 m + 8 (i >> 2) + 4 h]; used when hidden C is 64
     * or 128 and 4C <= 1024 (ponita.py _ffn_image); lin1_b / lin2_b / layer_scale as above */
    const void* ffn_img_x3;
    /* optional (ABI 17): fp16x2 images ("fp16x2 images": W s = hi + lo, both fp16, s a power of two per
     * matrix; block [part 2][m 2][lane 64][8] fp16 in place of the bf16x3 block) of the fused ConvNext MLP
     * (the ffn_img_x3 layout; linear_1 scaled by 1 / ffn_h2_s1inv, linear_2 by 1 / ffn_h2_s2inv) and of
     * kernel_t (the kernel_img_x3 layout, scaled by 1 / kernel_h2_sinv); used in place of the bf16x3 images
     * when present (NBX_PO_SPLIT=x3: the bf16x3 images) */
    const void* ffn_img_h2;
    const void* kernel_img_h2;
    float ffn_h2_s1inv, ffn_h2_s2inv, kernel_h2_sinv, h2_pad;
} nbx_ponita_layer;

typedef struct nbx_ponita_weights {
    int32_t hidden, basis_dim, widening, num_layers, num_ori;
    const float* ori_grid;
    const float* basis1_t; const float* basis1_b;
    const float* basis2_t; const float* basis2_b;
    const float* fbasis1_t; const float* fbasis1_b;
    const float* fbasis2_t; const float* fbasis2_b;
    const float* fiber_t;
    const float* embed_w;
    const void* basis2_img_x3;   /* optional bf16x3 image of basis2_t (as the layer images) */
    /* optional (ABI 10): both kernel-basis layers in one kernel (hidden width = hidden, basis_dim 64 or
     * 128): per 32-wide hidden chunk one slab [basis1_t rows of the chunk | basis2_t columns of the
     * chunk, K order permuted], the ffn_img_x3 layout with one 32-deep input chunk; the [E O][hidden]
     * activation between the layers never reaches HBM */
    const void* basis_ffn_img_x3;
    /* optional (ABI 17): the fp16x2 image of the fused kernel-basis MLP (basis_ffn_img_x3 layout, the
     * ffn_img_h2 scales) */
    const void* basis_ffn_img_h2;
    float basis_ffn_h2_s1inv, basis_ffn_h2_s2inv;
    nbx_ponita_layer layers[NBX_PONITA_MAX_LAYERS];
} nbx_ponita_weights;

int nbx_ponita_workspace_bytes(const nbx_ponita_weights* w, int64_t batch_size, int64_t num_nodes, size_t* bytes);

/* fp16x2 range guard of the PONITA calls (ABI 17), as nbx_segnn_range_check: waits for `stream`, reads the
 * flag the fp16x2 kernels of the last nbx_ponita_forward / _forward_graph / _rollout / _rollout_knn call made
 * with `workspace` raised, and returns NBX_E_RANGE if an operand left the fp16 range (or an input was not
 * finite).  Synchronises. */
int nbx_ponita_range_check(const nbx_ponita_weights* w, const void* workspace, size_t workspace_bytes,
                           int64_t batch_size, int64_t num_nodes, void* stream);

/* PONITA_NBODY.forward on the graph of infer_self_feed.py:131-147
 * (x = mass, vec = vel, rel_pos = pos[src] - pos[dst]): out [B*N, 6].
 * calib_moments: NULL, or a device buffer of num_layers*6 doubles that receives per layer
 * (sum, sum of squares) of the layer input, x_1 and x_2 (before the bias) — the
 * statistics FiberBundleConv.callibrate (conv.py:115-117,134-140) needs on the first
 * training-mode forward; the caller rescales the weights. */
int nbx_ponita_forward(const nbx_ponita_weights* w, const float* pos, const float* vel, const float* mass,
                       int64_t batch_size, int64_t num_nodes, float* out, double* calib_moments, void* workspace,
                       size_t workspace_bytes, void* stream);

/* nbx_ponita_forward with HIP events around the main launches, on `stream`:
 * per kind k (0 spatial conv, 1 ConvNext linear_1, 2 linear_2, 3 basis MLP,
 * 4 fibre conv + LayerNorm) the summed kernel time, launch count and the
 * algorithmic flops / bytes; total_ms = the whole forward. */
int nbx_ponita_forward_timed(const nbx_ponita_weights* w, const float* pos, const float* vel, const float* mass,
                             int64_t batch_size, int64_t num_nodes, float* out, void* workspace,
                             size_t workspace_bytes, void* stream, float kind_ms[8], int32_t kind_launches[8],
                             double kind_flops[8], double kind_bytes[8], float* total_ms);

/* Device-resident self-feed rollout with the PONITA branch of
 * infer_self_feed.py:131-147,182-194; same contract as nbx_segnn_rollout. */
int nbx_ponita_rollout(const nbx_ponita_weights* w, float* pos, float* vel, const float* mass, int64_t batch_size,
                       int64_t num_nodes, int64_t num_frames, int32_t flags, float* traj_pos, float* traj_vel, void* workspace,
                       size_t workspace_bytes, void* stream);

/* General graphs (ABI 8), as nbx_segnn_forward_graph: nbx_ponita_forward on `edge_index` (int64
 * [2][num_edges], row = source, col = target, e.g. build_graph_with_knn's kNN branch,
 * infer_self_feed.py:137-142): FiberBundleConv sums the messages of a node's incoming edges, a node
 * without any receives zero.  Edges must join different nodes of one system, without duplicates
 * (NBX_E_INVAL otherwise); synchronises `stream` once. */
int nbx_ponita_forward_graph(const nbx_ponita_weights* w, const float* pos, const float* vel, const float* mass,
                             int64_t batch_size, int64_t num_nodes, const int64_t* edge_index, int64_t num_edges,
                             float* out, double* calib_moments, void* workspace, size_t workspace_bytes, void* stream);

/* nbx_ponita_rollout with the reference's num_neighbors: each frame's kNN graph built on the device
 * (contract of nbx_segnn_rollout_knn). */
int nbx_ponita_rollout_knn(const nbx_ponita_weights* w, float* pos, float* vel, const float* mass,
                           int64_t batch_size, int64_t num_nodes, int64_t num_frames, int32_t flags,
                           int64_t num_neighbors, float* traj_pos, float* traj_vel, void* workspace,
                           size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * EquiformerV2 (models/equiformer_v2/architecture/equiformer_v2_nbody.py:57-575 on the tuple
 * branch of helper_scripts/infer_self_feed.py:178-181, eval mode) — fp32.
 *
 * Scope: lmax_list = [2], mmax_list = [1] (one resolution), norm_type "rms_norm_sh",
 * distance_function "projection", use_atom_edge_embedding (not shared), use_m_share_rad False,
 * separable S2 activations, sphere_channels C in {32, 64}, attn_hidden H and ffn_hidden F in {32, 64},
 * edge_channels He in {32, 64}, num_heads * attn_alpha_channels <= 64 (alpha <= 16),
 * num_heads * attn_value_channels in {8, 16, 32}, fully-connected systems of N <= 64 nodes.
 * Atomic numbers are (int) mass, clamped to [0, num_elements).
 *
 * Radial functions (RadialFunction [1024 + 2 He, He, He, R]) are passed with their first Linear
 * folded over the input it sees: x_edge = [distance_expansion(d) | source_emb[z_s] | target_emb[z_t]]
 * (an affine function of d plus two table lookups), so h1 = d * a + c + us[z_s] + ut[z_t]:
 *   a = W0[:, :1024] w_de, c = W0[:, :1024] b_de + b0, us = (W0[:, 1024:1024+He] E_s^T)^T [Z][He],
 *   ut likewise.  The last Linear (He -> R) is a bf16x3 image (CW = 32, "bf16x3 images" above) of
 * its weight with rows permuted: attention radials R = 10 C, output column
 * n = 160 cb + 32 g + i <- original row g * 2C + 32 cb + i (g = 0..4 = m0 l0, m0 l1, m0 l2, m1 l1,
 * m1 l2; cb = 32-channel block of the message [x_src | x_dst]); bias permuted alike.  The edge-degree
 * radial (R = 3 C) keeps its row order and is a plain fp32 matrix [3C][He].
 * GEMM images (*_x3) are bf16x3 images of nn.Linear weights [out][in] with out zero-padded to a
 * multiple of 32 (biases padded alike).  Node-side matrices are stored input-major ("_t": [in][out]):
 *   proj_t [3][nh nv][Cout], gate_t [C][F], lin1_t [3][C][F], lin2_t [3][F][C], vel_t [3][3C].
 * Grids: SO3_Grid(2, 1) (attention) and SO3_Grid(2, 2) (FFN) to/from matrices [points][coeffs]
 * (so3.py:543-618; 18 x 7 and 42 x 9).
 */
#define NBX_EQV2_MAX_LAYERS 32

typedef struct nbx_eqv2_radial {
    const float* a; const float* c;        /* [He] */
    const float* us; const float* ut;      /* [num_elements][He] */
    const float* ln1_w; const float* ln1_b;
    const float* w1; const float* b1;      /* net.3 [He][He] (nn.Linear layout), [He] */
    const float* ln2_w; const float* ln2_b;
    const void* w2_x3;                     /* net.6 image (attention radials, permuted), or NULL */
    const float* w2;                       /* net.6 [R][He] fp32 (edge-degree radial) */
    const float* b2;                       /* [R] */
    /* optional (ABI 18): fp16x2 images (nbx_eqv2_attn "fp16x2 images", the lin_kernel block order) of
     * net.3 -- with it the hidden layers run as one launch: the first layer formed in the GEMM's operand
     * registers, net.3 on fp16x2 MFMA, LayerNorm + SiLU in its epilogue -- and, edge-degree radial only,
     * of net.6 (the attention radials' net.6 image is nbx_eqv2_attn.w2_h2); with their 1 / s */
    const void* w1_h2; const void* w2_h2;
    float w1_sinv, w2_sinv;
} nbx_eqv2_radial;

typedef struct nbx_eqv2_attn {             /* SO2EquivariantGraphAttention */
    nbx_eqv2_radial rad;                   /* so2_conv_1.rad_func (with this module's atom embeddings) */
    /* so2_conv_1 weights as CHUNK-MAJOR bf16x3 images [K/32][N/32][3][2][64][8] (the blocks of the
     * "bf16x3 images" layout with the K-chunk index outermost): the row-panel GEMM streams one K
     * chunk of every column tile per step */
    const void* fc0_x3; const float* fc0_b;  /* so2_conv_1.fc_m0 [nh na + H + 3 H][3 * 2C] */
    const void* fc1_x3;                      /* so2_conv_1.so2_m_conv.0.fc [4H][2 * 2C] */
    const void* c20_x3; const float* c20_b;  /* so2_conv_2.fc_m0 [3 nh nv][3H] */
    const void* c21_x3;                      /* so2_conv_2.so2_m_conv.0.fc [4 nh nv][2H] */
    const float* alpha_norm_w; const float* alpha_norm_b;   /* [na] */
    const float* alpha_dot;                  /* [nh][na] */
    const float* proj_t; const float* proj_b;  /* proj (SO3_LinearV2) [3][nh nv][Cout], [Cout] */
    /* optional (ABI 17): fp16x2 images (W s = hi + lo, both fp16, s a power of two per matrix; block
     * [part 2][m 2][lane 64][8] fp16 in place of the bf16x3 block, same orders: fc0 / fc1 chunk-major)
     * of rad.w2, fc0, fc1, c20, c21 with their 1 / s; used in place of the bf16x3 images when present
     * (NBX_EQ_SPLIT=x3: the bf16x3 images) */
    const void* w2_h2; const void* fc0_h2; const void* fc1_h2; const void* c20_h2; const void* c21_h2;
    float w2_sinv, fc0_sinv, fc1_sinv, c20_sinv, c21_sinv, h2_pad;
} nbx_eqv2_attn;

typedef struct nbx_eqv2_block {            /* TransBlockV2 */
    const float* norm1_w; const float* norm1_b;   /* [3][C], [C] */
    nbx_eqv2_attn ga;
    const float* norm2_w; const float* norm2_b;
    const float* gate_t; const float* gate_b;     /* ffn.gating_linear */
    const float* lin1_t; const float* lin1_b;     /* ffn.so3_linear_1 */
    const float* lin2_t; const float* lin2_b;     /* ffn.so3_linear_2 */
} nbx_eqv2_block;

typedef struct nbx_eqv2_weights {
    int32_t sphere_channels, attn_hidden, num_heads, alpha_channels, value_channels, ffn_hidden,
        edge_channels, num_layers, num_elements;
    const float* grid_attn_to; const float* grid_attn_from;   /* [18][7] */
    const float* grid_ffn_to; const float* grid_ffn_from;     /* [42][9] */
    const float* sphere_emb;                  /* [num_elements][C] */
    const float* vel_t; const float* vel_b;   /* velocity_embedding [3][3C], [3C] */
    nbx_eqv2_radial edge_degree;              /* R = 3C (m = 0 coefficients of l = 0, 1, 2) */
    const float* norm_w; const float* norm_b; /* final norm */
    nbx_eqv2_attn force;                      /* force_block (Cout = 2) */
    nbx_eqv2_block blocks[NBX_EQV2_MAX_LAYERS];
} nbx_eqv2_weights;

int nbx_eqv2_workspace_bytes(const nbx_eqv2_weights* w, int64_t batch_size, int64_t num_nodes, size_t* bytes);

/* EquiformerV2_nbody.forward((pos, vel, force, mass, pos), batch): pos/vel [B*N,3], mass [B*N] ->
 * out [B*N, 6] (delta pos | vel).  init_edge_rot_mat (edge_rot_mat.py:21) draws one random vector per
 * edge; `gauge` supplies them (fp32 [E][3], uniform [0,1), E = B*N*(N-1) in the fully-connected
 * order) or, when NULL, they are drawn on the device from a counter-based hash of (seed, edge). */
int nbx_eqv2_forward(const nbx_eqv2_weights* w, const float* pos, const float* vel, const float* mass,
                     int64_t batch_size, int64_t num_nodes, const float* gauge, uint64_t seed, float* out,
                     void* workspace, size_t workspace_bytes, void* stream);

/* nbx_eqv2_forward with HIP event pairs around each launch group on `stream` (synchronises; not
 * graph-capturable): per kind k (0 radial hidden layers, 1 radial output GEMM + message epilogue,
 * 2 SO(2) conv 1 m=0 GEMM, 3 SO(2) conv 1 m=1 GEMM, 4 S2 activation + logits, 5 SO(2) conv 2 GEMMs,
 * 6 node kernels, 7 edge frame + edge-degree embedding) the summed time, launch-group count, and the
 * algorithmic flops (2 x MACs of fp32-accurate products) and HBM bytes (inputs + outputs once);
 * total_ms = the whole forward. */
int nbx_eqv2_forward_timed(const nbx_eqv2_weights* w, const float* pos, const float* vel, const float* mass,
                           int64_t batch_size, int64_t num_nodes, const float* gauge, uint64_t seed, float* out,
                           void* workspace, size_t workspace_bytes, void* stream, float kind_ms[8],
                           int32_t kind_launches[8], double kind_flops[8], double kind_bytes[8], float* total_ms);

/* Device-resident self-feed rollout through the tuple branch (infer_self_feed.py:99-194), same
 * contract as nbx_segnn_rollout; step t draws its gauges from the hash of (seed, t, edge). */
int nbx_eqv2_rollout(const nbx_eqv2_weights* w, float* pos, float* vel, const float* mass, int64_t batch_size,
                     int64_t num_nodes, int64_t num_frames, int32_t flags, uint64_t seed, float* traj_pos,
                     float* traj_vel, void* workspace, size_t workspace_bytes, void* stream);

/* fp16x2 range guard of the EquiformerV2 calls (ABI 17), as nbx_segnn_range_check: waits for `stream`, reads
 * the flag of the last nbx_eqv2_forward / _forward_timed / _rollout call made with `workspace`; NBX_E_RANGE
 * if an operand of an fp16x2 GEMM left the fp16 range (or an input was not finite).  Synchronises. */
int nbx_eqv2_range_check(const nbx_eqv2_weights* w, const void* workspace, size_t workspace_bytes, int64_t batch_size,
                         int64_t num_nodes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NBX_H */
