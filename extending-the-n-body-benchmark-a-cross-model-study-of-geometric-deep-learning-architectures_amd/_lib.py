"""ctypes binding of libnbx.so (include/nbx.h).

The product path has NO CPU fallback: every op goes through this library and
raises if it is missing or if a tensor is not on a HIP device.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NBX_LIB") or os.path.join(_HERE, "lib", "libnbx.so")  # NBX_LIB: A/B builds only
ABI_VERSION = 19
COMM_ID_BYTES = 128
ROLLOUT_ABSOLUTE = 1   # NBX_ROLLOUT_ABSOLUTE
GEMM_TRANS_A, GEMM_TRANS_B, GEMM_B_ONES, GEMM_ONES_TAIL = 1, 2, 4, 8
ACT_NONE, ACT_GELU, ACT_SILU, ACT_SLRELU = 0, 1, 2, 3
MAX_LAYERS = 64

c_i64, c_i32, c_f, c_d, c_p, c_sz = (ctypes.c_int64, ctypes.c_int32, ctypes.c_float, ctypes.c_double,
                                     ctypes.c_void_p, ctypes.c_size_t)


class SegnnLayer(ctypes.Structure):
    _fields_ = [(n, c_p) for n in (
        "node_pre_s_img", "node_pre_v_img", "node_pre_s_img_x3", "node_pre_v_img_x3", "msg1_amf", "msg1_bias", "msg2_img", "msg2_img_x3", "msg2_bias",
        "upd1_img", "upd1_img_x3", "upd1_bias", "upd2_img", "upd2_bias",
        "msg_bn_weight", "msg_bn_bias", "msg_bn_running_mean", "msg_bn_running_var",
        "feat_bn_weight", "feat_bn_bias", "feat_bn_running_mean", "feat_bn_running_var",
        "node_pre_s_img_h2", "node_pre_v_img_h2", "msg2_img_h2", "upd1_img_h2", "upd2_img_h2")] + [
        (n, c_f) for n in ("node_pre_h2_descale", "msg2_h2_descale", "upd1_h2_descale", "upd2_h2_descale")]


# nbx_allreduce_fn: int (*)(double* buf, int64_t count, void* stream, void* ctx)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, c_p, c_i64, c_p, c_p)


class SegnnWeights(ctypes.Structure):
    _fields_ = [("mul", c_i32), ("num_layers", c_i32), ("training", c_i32), ("bn_eps", c_f),
                ("bn_momentum", c_f)] + [(n, c_p) for n in (
                    "emb", "emb_bias", "pp1_img", "pp1_bias", "pp2")] + [
                ("bn_allreduce", ALLREDUCE_FN), ("bn_allreduce_ctx", c_p), ("bn_global_batch", c_i64),
                ("bn_comm", c_p), ("deterministic", c_i32), ("reserved0", c_i32),
                ("pp1_img_h2", c_p), ("pp1_h2_descale", c_f), ("reserved1", c_i32),
                ("layers", SegnnLayer * MAX_LAYERS)]


EGNN_MAX_LAYERS = 64


class EgnnLayer(ctypes.Structure):
    _fields_ = [("e0_t", c_p), ("e0_b", c_p), ("e1_t", c_p), ("e1_b", c_p), ("c0_t", c_p), ("c0_b", c_p),
                ("c1_w", c_p), ("v0_t", c_p), ("v0_b", c_p), ("v1_w", c_p), ("v1_b", c_f), ("n0_t", c_p),
                ("n0_b", c_p), ("n1_t", c_p), ("n1_b", c_p)]


class EgnnHead(ctypes.Structure):
    _fields_ = [(n, c_p) for n in ("w0_t", "b0", "w1_t", "b1", "w2_t", "b2")]


class EgnnWeights(ctypes.Structure):
    _fields_ = [(n, c_i32) for n in ("hidden", "num_layers", "num_heads", "recurrent", "norm_diff", "use_tanh")] + [
        ("coords_weight", c_f), ("emb_t", c_p), ("emb_b", c_p), ("persist_blob", c_p), ("heads", EgnnHead * 2),
        ("layers", EgnnLayer * EGNN_MAX_LAYERS)]


PONITA_MAX_LAYERS = 64


class PonitaLayer(ctypes.Structure):
    _fields_ = [(n, c_p) for n in ("kernel_t", "conv_bias", "norm_w", "norm_b", "lin1_t", "lin1_b", "lin2_t",
                                   "lin2_b", "layer_scale", "readout_w", "readout_b", "kernel_img_x3",
                                   "lin1_img_x3", "lin2_img_x3", "ffn_img_x3", "ffn_img_h2", "kernel_img_h2")] + [
        (n, c_f) for n in ("ffn_h2_s1inv", "ffn_h2_s2inv", "kernel_h2_sinv", "h2_pad")]


class PonitaWeights(ctypes.Structure):
    _fields_ = [(n, c_i32) for n in ("hidden", "basis_dim", "widening", "num_layers", "num_ori")] + [
        (n, c_p) for n in ("ori_grid", "basis1_t", "basis1_b", "basis2_t", "basis2_b", "fbasis1_t", "fbasis1_b",
                           "fbasis2_t", "fbasis2_b", "fiber_t", "embed_w", "basis2_img_x3", "basis_ffn_img_x3",
                           "basis_ffn_img_h2")] + [
        ("basis_ffn_h2_s1inv", c_f), ("basis_ffn_h2_s2inv", c_f), ("layers", PonitaLayer * PONITA_MAX_LAYERS)]


EQV2_MAX_LAYERS = 32


class Eqv2Radial(ctypes.Structure):
    _fields_ = [(n, c_p) for n in ("a", "c", "us", "ut", "ln1_w", "ln1_b", "w1", "b1", "ln2_w", "ln2_b", "w2_x3", "w2",
                                   "b2", "w1_h2", "w2_h2")] + [(n, c_f) for n in ("w1_sinv", "w2_sinv")]


class Eqv2Attn(ctypes.Structure):
    _fields_ = [("rad", Eqv2Radial)] + [(n, c_p) for n in (
        "fc0_x3", "fc0_b", "fc1_x3", "c20_x3", "c20_b", "c21_x3", "alpha_norm_w", "alpha_norm_b", "alpha_dot",
        "proj_t", "proj_b", "w2_h2", "fc0_h2", "fc1_h2", "c20_h2", "c21_h2")] + [
        (n, c_f) for n in ("w2_sinv", "fc0_sinv", "fc1_sinv", "c20_sinv", "c21_sinv", "h2_pad")]


class Eqv2Block(ctypes.Structure):
    _fields_ = [("norm1_w", c_p), ("norm1_b", c_p), ("ga", Eqv2Attn)] + [(n, c_p) for n in (
        "norm2_w", "norm2_b", "gate_t", "gate_b", "lin1_t", "lin1_b", "lin2_t", "lin2_b")]


class Eqv2Weights(ctypes.Structure):
    _fields_ = [(n, c_i32) for n in ("sphere_channels", "attn_hidden", "num_heads", "alpha_channels", "value_channels",
                                     "ffn_hidden", "edge_channels", "num_layers", "num_elements")] + [
        (n, c_p) for n in ("grid_attn_to", "grid_attn_from", "grid_ffn_to", "grid_ffn_from", "sphere_emb", "vel_t",
                           "vel_b")] + [
        ("edge_degree", Eqv2Radial), ("norm_w", c_p), ("norm_b", c_p), ("force", Eqv2Attn),
        ("blocks", Eqv2Block * EQV2_MAX_LAYERS)]


_SIGNATURES = {
    "nbx_abi_version": (ctypes.c_int, []),
    "nbx_last_error": (ctypes.c_char_p, []),
    "nbx_fc_edge_index": (ctypes.c_int, [c_i64, c_i64, c_p, c_p]),
    "nbx_knn_edge_index": (ctypes.c_int, [c_p, c_i32, c_i64, c_i64, c_i64, c_p, c_p]),
    "nbx_gravity_acceleration": (ctypes.c_int, [c_p, c_p, c_i64, c_i64, c_d, c_d, c_p, c_p]),
    "nbx_gravity_sample": (ctypes.c_int, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_d, c_d, c_d,
                                          c_p, c_p, c_p, c_p]),
    "nbx_nbody_energies": (ctypes.c_int, [c_p, c_p, c_i64, c_i64, c_i64, c_d, c_d, c_p, c_p, c_p, c_p, c_p]),
    "nbx_ks_2samp_stat": (ctypes.c_int, [c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p]),
    "nbx_comm_unique_id": (ctypes.c_int, [c_p]),
    "nbx_comm_init": (ctypes.c_int, [c_p, c_i32, c_i32, c_i32, ctypes.POINTER(c_p)]),
    "nbx_comm_destroy": (ctypes.c_int, [c_p]),
    "nbx_comm_allreduce_f64": (ctypes.c_int, [c_p, c_i64, c_p, c_p]),
    "nbx_gemm_f32_workspace_bytes": (ctypes.c_int, [c_i64, c_i64, c_i64, ctypes.POINTER(c_sz)]),
    "nbx_gemm_f32": (ctypes.c_int, [c_i32, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_f, c_p, c_sz, c_p]),
    "nbx_gemm_f32_batched_workspace_bytes": (ctypes.c_int, [c_i32, c_p, ctypes.POINTER(c_sz)]),
    "nbx_gemm_f32_batched": (ctypes.c_int, [c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "nbx_gemm_f32_grouped_workspace_bytes": (ctypes.c_int, [c_i32, c_p, ctypes.POINTER(c_sz)]),
    "nbx_gemm_f32_grouped": (ctypes.c_int, [c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "nbx_tp_prep": (ctypes.c_int, [c_i64, c_i32, c_i32, c_p, c_i64, c_p, c_p, c_p, c_p]),
    "nbx_tp_prep_backward": (ctypes.c_int, [c_i64, c_i32, c_i32, c_p, c_p, c_p, c_i64, c_p, c_p]),
    "nbx_tp_post": (ctypes.c_int, [c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "nbx_tp_post_backward": (ctypes.c_int, [c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "nbx_colsum_workspace_bytes": (ctypes.c_int, [c_i64, c_i32, ctypes.POINTER(c_sz)]),
    "nbx_colsum": (ctypes.c_int, [c_i64, c_i32, c_p, c_i64, c_p, c_i32, c_p, c_sz, c_p]),
    "nbx_bn_train_workspace_bytes": (ctypes.c_int, [c_i64, c_i32, ctypes.POINTER(c_sz)]),
    "nbx_bn_train_forward": (ctypes.c_int, [c_i64, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_f, c_f, c_p, c_p, c_p, c_p,
                                            c_sz, c_p]),
    "nbx_bn_train_backward": (ctypes.c_int, [c_i64, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_sz,
                                             c_p]),
    "nbx_bn_train_sums": (ctypes.c_int, [c_i64, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "nbx_bn_train_apply": (ctypes.c_int, [c_i64, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_f, c_f, c_p, c_p, c_p,
                                          c_p]),
    "nbx_bn_train_param_grads": (ctypes.c_int, [c_i32, c_p, c_p, c_p, c_p, c_p, c_p]),
    "nbx_bn_train_backward_apply": (ctypes.c_int, [c_i64, c_i32] + [c_p] * 10),
    "nbx_gather_rows": (ctypes.c_int, [c_i64, c_i32, c_p, c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_i32, c_p]),
    "nbx_segment_sum": (ctypes.c_int, [c_i64, c_i32, c_p, c_p, c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_i32, c_i32, c_p]),
    "nbx_segnn_train_featurize": (ctypes.c_int, [c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                                 c_p, c_p]),
    "nbx_ponita_train_featurize": (ctypes.c_int, [c_i64, c_i64, c_i32] + [c_p] * 10),
    "nbx_bias_act": (ctypes.c_int, [c_i64, c_i32, c_p, c_i64, c_p, c_i32, c_p, c_i64, c_p]),
    "nbx_bias_act_backward": (ctypes.c_int, [c_i64, c_i32, c_p, c_i64, c_p, c_i32, c_p, c_p, c_p]),
    "nbx_po_message": (ctypes.c_int, [c_i64, c_i32, c_i32] + [c_p] * 7),
    "nbx_po_message_backward": (ctypes.c_int, [c_i64, c_i64, c_i32, c_i32] + [c_p] * 10),
    "nbx_po_fiber_conv": (ctypes.c_int, [c_i64, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p]),
    "nbx_po_fiber_conv_workspace_bytes": (ctypes.c_int, [c_i64, c_i32, c_i32, ctypes.POINTER(c_sz)]),
    "nbx_po_fiber_conv_backward": (ctypes.c_int, [c_i64, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "nbx_layernorm_forward": (ctypes.c_int, [c_i64, c_i32, c_p, c_p, c_p, c_f, c_p, c_p, c_p]),
    "nbx_layernorm_backward": (ctypes.c_int, [c_i64, c_i32] + [c_p] * 7),
    "nbx_eqv2_train_edges": (ctypes.c_int, [c_i64, c_i64, c_p, c_p, c_p, ctypes.c_uint64, c_i32, c_p, c_p, c_p, c_p,
                                            c_p]),
    "nbx_eqv2_rotate": (ctypes.c_int, [c_i64, c_i32, c_p, c_p, c_i64, c_p, c_i32, c_i32, c_p]),
    "nbx_eqv2_s2_act": (ctypes.c_int, [c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p]),
    "nbx_eqv2_s2_act_backward": (ctypes.c_int, [c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p]),
    "nbx_segment_softmax": (ctypes.c_int, [c_i64, c_i32, c_p, c_p, c_p, c_p, c_p]),
    "nbx_segment_softmax_backward": (ctypes.c_int, [c_i64, c_i32, c_p, c_p, c_p, c_p, c_p, c_p]),
    "nbx_eqv2_rms_norm": (ctypes.c_int, [c_i64, c_i32, c_p, c_p, c_p, c_f, c_p, c_p, c_p]),
    "nbx_eqv2_rms_norm_backward": (ctypes.c_int, [c_i64, c_i32] + [c_p] * 7),
    "nbx_eqv2_edges": (ctypes.c_int, [c_i64, c_i64, c_p, c_p, c_p, ctypes.c_uint64, c_i64, c_i32, c_p, c_p, c_p, c_p]),
    "nbx_eqv2_wigner_table_floats": (ctypes.c_int, [c_i32, ctypes.POINTER(c_i64)]),
    "nbx_eqv2_dsel_floats": (ctypes.c_int, [c_i32, c_i32, ctypes.POINTER(c_i64)]),
    "nbx_eqv2_wigner": (ctypes.c_int, [c_i64, c_i32, c_i32, c_p, c_i64, c_p, c_p, c_p]),
    "nbx_eqv2_rotate_general": (ctypes.c_int, [c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_i64, c_p, c_i32, c_i32, c_p,
                                                c_p]),
    "nbx_eqv2_rotate_gather": (ctypes.c_int, [c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_i64, c_p, c_p, c_p, c_i32,
                                               c_p, c_p, c_i64, c_p, c_p]),
    "nbx_eqv2_rms_norm_general": (ctypes.c_int, [c_i64, c_i32, c_i32, c_p, c_p, c_p, c_f, c_p, c_p, c_p]),
    "nbx_eqv2_rms_norm_general_backward": (ctypes.c_int, [c_i64, c_i32, c_i32] + [c_p] * 7),
    "nbx_segnn_workspace_bytes": (ctypes.c_int, [c_i64, c_i64, c_i32, ctypes.POINTER(c_sz)]),
    "nbx_segnn_forward": (ctypes.c_int, [ctypes.POINTER(SegnnWeights), c_p, c_p, c_p, c_i64, c_i64, c_p,
                                         c_p, c_sz, c_p]),
    "nbx_segnn_forward_timed": (ctypes.c_int, [ctypes.POINTER(SegnnWeights), c_p, c_p, c_p, c_i64, c_i64, c_p,
                                               c_p, c_sz, c_p, c_f * 4, c_i32 * 4, c_d * 4, ctypes.POINTER(c_f)]),
    "nbx_egnn_workspace_bytes": (ctypes.c_int, [c_i64, c_i64, c_i32, ctypes.POINTER(c_sz)]),
    "nbx_egnn_forward": (ctypes.c_int, [ctypes.POINTER(EgnnWeights), c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_sz,
                                        c_p]),
    "nbx_egnn_rollout": (ctypes.c_int, [ctypes.POINTER(EgnnWeights), c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_p, c_p,
                                        c_p, c_sz, c_p]),
    "nbx_egnn_forward_graph": (ctypes.c_int, [ctypes.POINTER(EgnnWeights), c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p,
                                              c_p, c_p, c_sz, c_p]),
    "nbx_egnn_rollout_knn": (ctypes.c_int, [ctypes.POINTER(EgnnWeights), c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32,
                                            c_i64, c_p, c_p, c_p, c_sz, c_p]),
    "nbx_egnn_train_workspace_bytes": (ctypes.c_int, [ctypes.POINTER(EgnnWeights), c_i64, c_i64, ctypes.POINTER(c_sz)]),
    "nbx_egnn_train_forward": (ctypes.c_int, [ctypes.POINTER(EgnnWeights), c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_sz,
                                              c_p]),
    "nbx_egnn_train_backward": (ctypes.c_int, [ctypes.POINTER(EgnnWeights), c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_p,
                                               c_sz, c_p]),
    "nbx_segnn_rollout": (ctypes.c_int, [ctypes.POINTER(SegnnWeights), c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32,
                                         c_p, c_p, c_p, c_sz, c_p]),
    "nbx_segnn_forward_graph": (ctypes.c_int, [ctypes.POINTER(SegnnWeights), c_p, c_p, c_p, c_i64, c_i64, c_p,
                                               c_i64, c_p, c_p, c_sz, c_p]),
    "nbx_segnn_rollout_knn": (ctypes.c_int, [ctypes.POINTER(SegnnWeights), c_p, c_p, c_p, c_i64, c_i64, c_i64,
                                             c_i32, c_i64, c_p, c_p, c_p, c_sz, c_p]),
    "nbx_segnn_range_check": (ctypes.c_int, [c_p, c_sz, c_i64, c_i64, c_i32, c_p]),
    "nbx_ponita_range_check": (ctypes.c_int, [ctypes.POINTER(PonitaWeights), c_p, c_sz, c_i64, c_i64, c_p]),
    "nbx_eqv2_range_check": (ctypes.c_int, [ctypes.POINTER(Eqv2Weights), c_p, c_sz, c_i64, c_i64, c_p]),
    "nbx_debug_msg_pre_check": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32), c_i32]),
    "nbx_ponita_workspace_bytes": (ctypes.c_int, [ctypes.POINTER(PonitaWeights), c_i64, c_i64,
                                                  ctypes.POINTER(c_sz)]),
    "nbx_ponita_forward": (ctypes.c_int, [ctypes.POINTER(PonitaWeights), c_p, c_p, c_p, c_i64, c_i64, c_p, c_p,
                                          c_p, c_sz, c_p]),
    "nbx_ponita_forward_graph": (ctypes.c_int, [ctypes.POINTER(PonitaWeights), c_p, c_p, c_p, c_i64, c_i64, c_p,
                                                c_i64, c_p, c_p, c_p, c_sz, c_p]),
    "nbx_ponita_rollout_knn": (ctypes.c_int, [ctypes.POINTER(PonitaWeights), c_p, c_p, c_p, c_i64, c_i64, c_i64,
                                              c_i32, c_i64, c_p, c_p, c_p, c_sz, c_p]),
    "nbx_ponita_forward_timed": (ctypes.c_int, [ctypes.POINTER(PonitaWeights), c_p, c_p, c_p, c_i64, c_i64, c_p,
                                                c_p, c_sz, c_p, c_f * 8, c_i32 * 8, c_d * 8, c_d * 8,
                                                ctypes.POINTER(c_f)]),
    "nbx_ponita_rollout": (ctypes.c_int, [ctypes.POINTER(PonitaWeights), c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32,
                                          c_p, c_p, c_p, c_sz, c_p]),
    "nbx_eqv2_workspace_bytes": (ctypes.c_int, [ctypes.POINTER(Eqv2Weights), c_i64, c_i64, ctypes.POINTER(c_sz)]),
    "nbx_eqv2_forward": (ctypes.c_int, [ctypes.POINTER(Eqv2Weights), c_p, c_p, c_p, c_i64, c_i64, c_p, ctypes.c_uint64,
                                        c_p, c_p, c_sz, c_p]),
    "nbx_eqv2_forward_timed": (ctypes.c_int, [ctypes.POINTER(Eqv2Weights), c_p, c_p, c_p, c_i64, c_i64, c_p,
                                              ctypes.c_uint64, c_p, c_p, c_sz, c_p, c_f * 8, c_i32 * 8, c_d * 8,
                                              c_d * 8, ctypes.POINTER(c_f)]),
    "nbx_eqv2_rollout": (ctypes.c_int, [ctypes.POINTER(Eqv2Weights), c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i32,
                                        ctypes.c_uint64, c_p, c_p, c_p, c_sz, c_p]),
}

_lib = None


class NbxError(RuntimeError):
    pass


def lib():
    """Load libnbx.so (once).  Raises NbxError if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NbxError(f"HIP extension not built: {LIB_PATH} is missing (run __graft_entry__.build())")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype, fn.argtypes = res, args
        if handle.nbx_abi_version() != ABI_VERSION:
            raise NbxError("libnbx ABI version mismatch")
        _lib = handle
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        raise NbxError(f"{what}: {lib().nbx_last_error().decode()} (code {rc})")


def dev_ptr(t: torch.Tensor, dtype=None) -> int:
    """Device pointer of a contiguous HIP tensor (raises on CPU tensors: no fallback)."""
    if not t.is_cuda:
        raise NbxError("nbx ops run on the HIP device only; got a CPU tensor")
    if dtype is not None and t.dtype != dtype:
        raise NbxError(f"expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise NbxError("expected a contiguous tensor")
    return t.data_ptr()


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
