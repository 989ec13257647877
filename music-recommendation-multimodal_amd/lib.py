"""ctypes binding of libttmi.so (include/ttmi.h).

The library is built in-tree (``make`` at the repo root, or ``__graft_entry__.build()``)
into ``lib/libttmi.so`` next to this file.  ``load()`` raises if it is missing: there is no
CPU or eager-PyTorch fallback on the product path.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libttmi.so")

F32, BF16 = 0, 1
ABI_VERSION = 22

c_i, c_i64, c_u64, c_f, c_p = (ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float,
                               ctypes.c_void_p)


class GemmDesc(ctypes.Structure):
    """ttmi_gemm_desc (include/ttmi.h)."""
    _fields_ = [
        ("dtype", c_i),
        ("M", c_i64), ("N", c_i64), ("K", c_i64),
        ("A", c_p), ("lda", c_i64), ("a_kmajor", c_i),
        ("B", c_p), ("ldb", c_i64), ("b_kmajor", c_i),
        ("C", c_p), ("ldc", c_i64), ("c_dtype", c_i), ("c_mode", c_i),
        ("alpha", c_f),
        ("bias", c_p),
        ("act", c_i),
        ("drop_p", c_f), ("drop_seed", c_p), ("ld_drop", c_i64),
        ("gate", c_p), ("gate_dtype", c_i), ("ld_gate", c_i64), ("gate_scale", c_f),
        ("residual", c_p), ("ld_res", c_i64),
        ("colsum", c_p),
        ("split_k", c_i),
        ("drop_rows", c_p),
        ("rowsum_a", c_p),
        ("pre_out", c_p),
    ]


class WgradDesc(ctypes.Structure):
    """ttmi_wgrad_desc (include/ttmi.h)."""
    _fields_ = [("R", c_i64), ("M", c_i64), ("N", c_i64),
                ("dy", c_p), ("ld_dy", c_i64),
                ("x", c_p), ("ld_x", c_i64),
                ("dw", c_p), ("ld_dw", c_i64),
                ("db", c_p),
                ("alpha", c_f),
                ("accumulate", c_i),
                ("workspace", c_p), ("workspace_bytes", c_i64),
                ("defer", c_i)]


class ConvDesc(ctypes.Structure):
    """ttmi_conv_desc (include/ttmi.h)."""
    _fields_ = [("mode", c_i), ("N", c_i), ("H", c_i), ("W", c_i), ("C", c_i), ("Cin", c_i),
                ("Co", c_i), ("KH", c_i), ("KW", c_i), ("stride", c_i), ("pad", c_i),
                ("x", c_p), ("dy", c_p), ("w", c_p), ("out", c_p), ("addend", c_p),
                ("colsum", c_p), ("colsumsq", c_p), ("workspace", c_p),
                ("workspace_bytes", ctypes.c_int64),
                ("bn_gate", c_p), ("bn_x", c_p), ("bn_mean", c_p), ("bn_rstd", c_p),
                ("bn_sums", c_p)]


class ConvWPrep(ctypes.Structure):
    """ttmi_conv_wprep (include/ttmi.h)."""
    _fields_ = [("Co", c_i), ("Cin", c_i), ("Cp", c_i), ("KH", c_i), ("KW", c_i), ("s2d", c_i),
                ("w", c_p), ("wf", c_p), ("wd", c_p)]


class DisAttnDesc(ctypes.Structure):
    """ttmi_dis_attn_desc (include/ttmi.h)."""
    _fields_ = [("B", c_i), ("S", c_i), ("nh", c_i), ("d_head", c_i), ("npos", c_i),
                ("q", c_p), ("k", c_p), ("v", c_p), ("ldqkv", ctypes.c_int64),
                ("posq", c_p), ("posk", c_p), ("ldpos", ctypes.c_int64),
                ("mask", c_p), ("delta", c_p), ("inv_scale", ctypes.c_float),
                ("drop_p", ctypes.c_float), ("drop_seed", c_p),
                ("ctx", c_p), ("ldctx", ctypes.c_int64), ("lse", c_p),
                ("dctx", c_p), ("lddctx", ctypes.c_int64),
                ("dq", c_p), ("dk", c_p), ("dv", c_p), ("lddqkv", ctypes.c_int64),
                ("lora_u", c_p), ("lora_bq", c_p), ("lora_hu", c_p), ("lora_pb", c_p),
                ("dq_scratch", c_p), ("lora_pbx", c_p), ("order", c_p)]


class ItemHeadDesc(ctypes.Structure):
    """ttmi_item_head_desc (include/ttmi.h, ABI 14; stages ABI 15)."""
    _fields_ = [("B", c_i), ("K", c_i), ("N1", c_i), ("D", c_i),
                ("modal", c_p), ("w0", c_p), ("b0", c_p),
                ("bn_w", c_p), ("bn_b", c_p), ("bn_eps", ctypes.c_float), ("momentum", ctypes.c_float),
                ("running_mean", c_p), ("running_var", c_p), ("num_batches_tracked", c_p),
                ("drop_p", ctypes.c_float), ("drop_seed", c_p),
                ("w4", c_p), ("b4", c_p), ("ln_w", c_p), ("ln_b", c_p), ("ln_eps", ctypes.c_float),
                ("modal16", c_p), ("z", c_p), ("bn_mean", c_p), ("bn_rstd", c_p), ("y1", c_p), ("y2", c_p),
                ("out", c_p), ("m5", c_p), ("r5", c_p), ("ws", c_p),
                ("out_hat", c_p), ("out_norm", c_p), ("bn_part", c_p), ("bn_cnt", c_p)]


class BnBwdDesc(ctypes.Structure):
    """ttmi_bn_bwd_desc (include/ttmi.h, ABI 18)."""
    _fields_ = [("dtype", c_i), ("B", c_i), ("C", c_i),
                ("dy", c_p), ("z", c_p), ("w", c_p), ("mean", c_p), ("rstd", c_p),
                ("y", c_p), ("gate_scale", c_f), ("gated", c_i),
                ("dz", c_p), ("dw", c_p), ("db", c_p), ("dz16", c_p)]


class ItemHeadBwdDesc(ctypes.Structure):
    """ttmi_item_head_bwd_desc (include/ttmi.h, ABI 15)."""
    _fields_ = [("B", c_i), ("D", c_i), ("N1", c_i),
                ("dout", c_p), ("y2", c_p), ("m5", c_p), ("r5", c_p), ("ln_w", c_p),
                ("w4t", c_p), ("dy2", c_p), ("dy1", c_p), ("ws", c_p)]


class UserHeadDesc(ctypes.Structure):
    """ttmi_user_head_desc (include/ttmi.h)."""
    _fields_ = [("B", c_i), ("D", c_i), ("F", c_i), ("dg", c_i), ("dc", c_i),
                ("eps", ctypes.c_float),
                ("ctx", c_p), ("res", c_p), ("drop_rows", c_p),
                ("wo", c_p), ("bo", c_p), ("n2w", c_p), ("n2b", c_p),
                ("w1", c_p), ("b1", c_p), ("w2", c_p), ("b2", c_p),
                ("gender", c_p), ("G", c_p), ("country", c_p), ("C", c_p),
                ("wf0", c_p), ("bf0", c_p), ("lnw", c_p), ("lnb", c_p),
                ("wf3", c_p), ("bf3", c_p),
                ("d1_p", ctypes.c_float), ("d1_seed", c_p),
                ("dff_p", ctypes.c_float), ("dff_seed", c_p),
                ("d2_p", ctypes.c_float), ("d2_seed", c_p),
                ("x1", c_p), ("a2", c_p), ("m2", c_p), ("r2", c_p), ("h", c_p), ("comb", c_p),
                ("rows", c_p), ("z", c_p), ("az", c_p), ("mz", c_p), ("rz", c_p), ("u", c_p),
                ("u_hat", c_p), ("u_norm", c_p),
                ("n_genders", c_i), ("n_countries", c_i), ("id_err", c_p), ("ffn_ws", c_p)]


class AttnBlockDesc(ctypes.Structure):
    """ttmi_attn_block_desc (include/ttmi.h, ABI 21)."""
    _fields_ = [("B", c_i), ("L", c_i), ("H", c_i), ("Dh", c_i),
                ("a", c_p), ("w_in", c_p), ("b_in", c_p), ("key_valid", c_p),
                ("drop_p", ctypes.c_float), ("drop_seed", c_p),
                ("qkv", c_p), ("ctx", c_p), ("lse", c_p),
                ("wo", c_p), ("bo", c_p), ("res", c_p), ("n2w", c_p), ("n2b", c_p),
                ("eps", ctypes.c_float),
                ("drop1_p", ctypes.c_float), ("drop1_seed", c_p),
                ("x1", c_p), ("a2", c_p), ("m2", c_p), ("r2", c_p)]


class Q1KvBwdDesc(ctypes.Structure):
    """ttmi_q1_kv_bwd_desc (include/ttmi.h, ABI 21)."""
    _fields_ = [("B", c_i), ("L", c_i), ("H", c_i), ("Dh", c_i),
                ("qkv", c_p), ("key_valid", c_p), ("rows", c_p), ("lse", c_p), ("dctx", c_p),
                ("drop_p", ctypes.c_float), ("drop_seed", c_p),
                ("dqkv", c_p), ("wqt", c_p), ("ld_wqt", ctypes.c_int64), ("a_in", c_p),
                ("dq_rows", c_p), ("a_rows", c_p), ("dyq", c_p), ("bn", c_p)]


class FfnBlockDesc(ctypes.Structure):
    """ttmi_ffn_block_desc (include/ttmi.h, ABI 21; kv fields ABI 22)."""
    _fields_ = [("M", c_i), ("D", c_i), ("F", c_i),
                ("a", c_p), ("w1", c_p), ("b1", c_p), ("w2", c_p), ("b2", c_p), ("res", c_p),
                ("dropf_p", ctypes.c_float), ("dropf_seed", c_p),
                ("drop2_p", ctypes.c_float), ("drop2_seed", c_p),
                ("h", c_p), ("x2", c_p), ("lnw", c_p), ("lnb", c_p), ("eps", ctypes.c_float),
                ("y", c_p), ("mean", c_p), ("rstd", c_p),
                ("wkv", c_p), ("bkv", c_p), ("kv", c_p), ("ld_kv", c_i64)]


class FfnBlockBwdDesc(ctypes.Structure):
    """ttmi_ffn_block_bwd_desc (include/ttmi.h, ABI 21)."""
    _fields_ = [("M", c_i), ("D", c_i), ("F", c_i),
                ("dy2", c_p), ("w2t", c_p), ("w1t", c_p), ("h", c_p), ("gate_scale", ctypes.c_float),
                ("dz1", c_p), ("x1", c_p), ("m2", c_p), ("r2", c_p), ("n2w", c_p), ("res", c_p),
                ("dx1", c_p), ("dy1", c_p), ("drop1_p", ctypes.c_float), ("drop1_seed", c_p),
                ("sum_ws", c_p)]


class UserHeadBwdDesc(ctypes.Structure):
    """ttmi_user_head_bwd_desc (include/ttmi.h)."""
    _fields_ = [("B", c_i), ("D", c_i), ("F", c_i), ("dg", c_i), ("dc", c_i),
                ("ffn_scale", ctypes.c_float),
                ("du", c_p), ("az", c_p), ("z", c_p), ("mz", c_p), ("rz", c_p),
                ("h", c_p), ("x1", c_p), ("m2", c_p), ("r2", c_p),
                ("drop_rows", c_p), ("gender", c_p), ("country", c_p),
                ("wf3t", c_p), ("wf0t", c_p), ("w2t", c_p), ("w1t", c_p), ("wot", c_p),
                ("lnw", c_p), ("n2w", c_p),
                ("d1_p", ctypes.c_float), ("d1_seed", c_p),
                ("d2_p", ctypes.c_float), ("d2_seed", c_p),
                ("dG", c_p), ("dC", c_p),
                ("dz16", c_p), ("dy2", c_p), ("dz1", c_p), ("dx1", c_p), ("dy1", c_p),
                ("dctx", c_p), ("ws", c_p),
                ("n_genders", c_i), ("n_countries", c_i), ("ffn_ws", c_p)]


class LnBwdDesc(ctypes.Structure):
    """ttmi_linear_ln_bwd_desc (include/ttmi.h)."""
    _fields_ = [("M", ctypes.c_int64), ("N", ctypes.c_int64), ("K", ctypes.c_int64),
                ("dh", ctypes.c_void_p), ("ld_dh", ctypes.c_int64),
                ("wt", ctypes.c_void_p), ("ld_wt", ctypes.c_int64),
                ("x", ctypes.c_void_p), ("ldx", ctypes.c_int64),
                ("mean", ctypes.c_void_p), ("rstd", ctypes.c_void_p), ("ln_w", ctypes.c_void_p),
                ("res", ctypes.c_void_p), ("ld_res", ctypes.c_int64),
                ("dx", ctypes.c_void_p), ("lddx", ctypes.c_int64),
                ("next", ctypes.c_void_p), ("ld_next", ctypes.c_int64),
                ("drop_p", ctypes.c_float), ("drop_seed", ctypes.c_void_p),
                ("ld_drop", ctypes.c_int64), ("drop_rows", ctypes.c_void_p),
                ("ln_dw", ctypes.c_void_p), ("ln_db", ctypes.c_void_p),
                ("sum_ws", ctypes.c_void_p),
                ("res_rows", ctypes.c_void_p), ("res_L", ctypes.c_int64),
                ("dy_add", ctypes.c_void_p), ("ld_add", ctypes.c_int64)]


class FoldDesc(ctypes.Structure):
    """ttmi_fold_desc (include/ttmi.h)."""
    _fields_ = [("part", c_p), ("S", c_i64), ("s_stride", c_i64), ("M", c_i64), ("N", c_i64),
                ("C", c_p), ("ldc", c_i64), ("accumulate", c_i), ("fx_shift", c_i)]


class FoldPlan(ctypes.Structure):
    """ttmi_fold_plan (include/ttmi.h, ABI 19): opaque fold segments for ttmi_adamw_folded."""
    _fields_ = [("n", ctypes.c_int32), ("reserved", ctypes.c_int32), ("seg", c_u64 * (32 * 16))]


class ResLnDesc(ctypes.Structure):
    """ttmi_linear_res_ln_desc (include/ttmi.h)."""
    _fields_ = [("M", ctypes.c_int64), ("N", ctypes.c_int64), ("K", ctypes.c_int64),
                ("x", ctypes.c_void_p), ("ldx", ctypes.c_int64),
                ("w", ctypes.c_void_p), ("ldw", ctypes.c_int64),
                ("bias", ctypes.c_void_p),
                ("drop_p", ctypes.c_float), ("drop_seed", ctypes.c_void_p), ("ld_drop", ctypes.c_int64),
                ("residual", ctypes.c_void_p), ("ld_res", ctypes.c_int64),
                ("out", ctypes.c_void_p), ("ld_out", ctypes.c_int64),
                ("ln_w", ctypes.c_void_p), ("ln_b", ctypes.c_void_p), ("eps", ctypes.c_float),
                ("y", ctypes.c_void_p), ("ldy", ctypes.c_int64),
                ("mean", ctypes.c_void_p), ("rstd", ctypes.c_void_p)]


# name -> (restype, argtypes); mirrors include/ttmi.h one-to-one.
SIGNATURES = {
    "ttmi_last_error": (ctypes.c_char_p, []),
    "ttmi_abi_version": (c_i, []),
    "ttmi_gemm": (c_i, [ctypes.POINTER(GemmDesc), c_p]),
    "ttmi_catalogue_rows": (c_i, [c_i, c_i, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p]),
    "ttmi_wgrad_workspace": (c_i64, [c_i64, c_i64, c_i64, c_i64, c_i64]),
    "ttmi_wgrad": (c_i, [ctypes.POINTER(WgradDesc), c_p]),
    "ttmi_wgrad_fold": (c_i, [c_i, ctypes.POINTER(ctypes.POINTER(WgradDesc)), c_i,
                              ctypes.POINTER(FoldDesc), c_p]),
    "ttmi_linear_ln_bwd_sum_blocks": (c_i64, [c_i64]),
    "ttmi_linear_ln_bwd_sum_blocks_n": (c_i64, [c_i64, c_i64]),
    "ttmi_wgrad_batch": (c_i, [c_i, ctypes.POINTER(ctypes.POINTER(WgradDesc)), c_i,
                               ctypes.POINTER(FoldDesc), c_p]),
    "ttmi_wgrad_batch_plan": (c_i, [c_i, ctypes.POINTER(ctypes.POINTER(WgradDesc)), c_i,
                                    ctypes.POINTER(FoldDesc), ctypes.POINTER(FoldPlan), c_p]),
    "ttmi_adamw_folded_skip": (c_i, [c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_p, c_i64, c_i64, c_i,
                                     ctypes.POINTER(FoldPlan), c_i64, c_i64, c_p, c_p]),
    "ttmi_fold_plan_merge": (c_i, [ctypes.POINTER(FoldPlan), ctypes.POINTER(FoldPlan), c_p]),
    "ttmi_fold_plan_run": (c_i, [ctypes.POINTER(FoldPlan), c_p]),
    "ttmi_adamw_folded": (c_i, [c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_p, c_i64, c_i64, c_i,
                                ctypes.POINTER(FoldPlan), c_p, c_p]),
    "ttmi_layernorm_fwd": (c_i, [c_i64, c_i, c_p, c_i64, c_p, c_p, c_f, c_i, c_f, c_p, c_p, c_i,
                                 c_i64, c_p, c_p, c_p]),
    "ttmi_layernorm_bwd_workspace": (c_i64, [c_i]),
    "ttmi_layernorm_bwd_folds": (c_i, [c_i, c_p, c_p, c_p, c_p]),
    "ttmi_layernorm_bwd": (c_i, [c_i64, c_i, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_i, c_i64,
                                 c_f, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64, c_f, c_p, c_i, c_p]),
    "ttmi_seq_embed_fwd": (c_i, [c_i, c_i, c_i, c_p, c_p, c_i64, c_p, c_p, c_p, c_f, c_f, c_p, c_p,
                                 c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_seq_embed_bwd_workspace": (c_i64, [c_i64, c_i, c_i]),
    "ttmi_seq_embed_bwd_folds": (c_i, [c_i64, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_seq_embed_bwd": (c_i, [c_i, c_i, c_i, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_f, c_p, c_p,
                                 c_p, c_p, c_p, c_p, c_i64, c_p, c_i, c_p]),
    "ttmi_mha_fwd": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_f, c_p, c_p, c_p, c_p]),
    "ttmi_mha_bwd": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_p]),
    "ttmi_mha_generic_fwd": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_f, c_p, c_p, c_p, c_p]),
    "ttmi_mha_generic_bwd": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_p, c_p]),
    "ttmi_qkv_attn_supported": (c_i, [c_i, c_i, c_i, c_i]),
    "ttmi_mha_bwd_dy": (c_i, [c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_p]),
    "ttmi_attn_block_fwd": (c_i, [c_p, c_p]),
    "ttmi_ffn_block_supported": (c_i, [c_i, c_i, c_i]),
    "ttmi_ffn_block_bwd_supported": (c_i, [c_i, c_i, c_i]),
    "ttmi_ffn_block_fwd": (c_i, [c_p, c_p]),
    "ttmi_ffn_block_bwd_sum_blocks": (c_i, [c_i]),
    "ttmi_ffn_block_bwd": (c_i, [c_p, c_p]),
    "ttmi_mha_q1_proj_gather_fwd": (c_i, [c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_f, c_p,
                                          c_p, c_p, c_p, c_p]),
    "ttmi_qkv_attn_fwd": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_p, c_p,
                                c_p]),
    "ttmi_user_concat_fwd": (c_i, [c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_i, c_p, c_p, c_i, c_p,
                                   c_p, c_i, c_i, c_p, c_p]),
    "ttmi_user_concat_bwd": (c_i, [c_i, c_i, c_p, c_p, c_p, c_i, c_p, c_i, c_p, c_p, c_p, c_i, c_i,
                                   c_i, c_p]),
    "ttmi_batchnorm_fwd": (c_i, [c_i, c_i, c_i, c_p, c_p, c_p, c_f, c_f, c_p, c_p, c_p, c_i, c_i,
                                 c_f, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_batchnorm_bwd": (c_i, [c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_f, c_i, c_p, c_p, c_p,
                                 c_p, c_p]),
    "ttmi_infonce_workspace": (c_i64, [c_i, c_i]),
    "ttmi_infonce_fwd": (c_i, [c_i, c_i, c_p, c_p, c_p, c_f, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_infonce_fwd_acc": (c_i, [c_i, c_i, c_p, c_p, c_p, ctypes.c_float, c_p, c_p, c_p, c_p, c_p, c_p,
                                   c_p, c_p, c_p, c_p]),
    "ttmi_infonce_fwd_pre": (c_i, [c_i, c_i, c_p, ctypes.c_float, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                   c_p]),
    "ttmi_infonce_counter_bytes": (ctypes.c_int64, [c_i]),
    "ttmi_infonce_bwd": (c_i, [c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_infonce_bwd16": (c_i, [c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_infonce_bwd_fused": (c_i, [c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_p, c_p, c_p,
                                     c_p, c_p]),
    "ttmi_infonce_bwd_counter_bytes": (ctypes.c_int64, [c_i]),
    "ttmi_adamw": (c_i, [c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_p, c_p]),
    "ttmi_adamw_fx": (c_i, [c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_p, c_i64, c_i64, c_i,
                            c_p, c_p]),
    "ttmi_batch_copy": (c_i, [c_i, c_p, c_p, c_p, c_p]),
    "ttmi_transpose_bf16_batch": (c_i, [c_i, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_transpose_bf16_batch_seeds": (c_i, [c_i, c_p, c_p, c_p, c_p, c_u64, c_p, c_p, c_i, c_i, c_p]),
    "ttmi_step_prologue": (c_i, [c_i, c_p, c_p, c_p, c_i, c_p, c_p, c_p, c_p, c_u64, c_p, c_p, c_i,
                                 c_i, c_p]),
    "ttmi_linear_ln_bwd": (c_i, [c_p, c_p]),
    "ttmi_linear_res_ln": (c_i, [c_p, c_p]),
    "ttmi_deb_embed_fwd": (c_i, [c_i64, c_i, c_p, c_p, c_p, c_p, ctypes.c_float, c_p,
                                 ctypes.c_float, c_p, c_p, c_p, c_i64, c_i64, c_p, c_p]),
    "ttmi_deb_ln_fwd": (c_i, [c_i64, c_i, c_p, c_p, c_p, c_f, c_p, c_p, c_i64, c_p, c_p, c_p, c_p,
                               c_f, c_p, c_p, c_p]),
    "ttmi_deb_gelu": (c_i, [c_i64, c_p, c_p, c_p]),
    "ttmi_topk_rows": (c_i, [c_i, c_i, c_i, c_p, c_i64, c_i, c_p, c_p, c_p]),
    "ttmi_rank_of": (c_i, [c_i, c_i, c_p, c_p, c_p, c_p]),
    "ttmi_mask_items": (c_i, [c_i, c_i, c_p, c_i64, c_p, c_i, c_p]),
    "ttmi_dis_attn_fwd": (c_i, [c_p, c_p]),
    "ttmi_dis_attn_bwd": (c_i, [c_p, c_p]),
    "ttmi_dis_attn_pbx_floats": (ctypes.c_int64, [c_i, c_i, c_i]),
    "ttmi_dis_attn_order": (c_i, [c_p, c_i, c_i, c_p, c_p]),
    "ttmi_user_head_fwd": (c_i, [c_p, c_p]),
    "ttmi_user_head_bwd": (c_i, [c_p, c_p]),
    "ttmi_user_head_bwd_ws_floats": (ctypes.c_int64, [c_i]),
    "ttmi_item_head_fwd": (c_i, [c_p, c_p]),
    "ttmi_item_head_fwd_stages": (c_i, [c_p, c_i, c_p]),
    "ttmi_user_item_head_fwd": (c_i, [c_p, c_p, c_p]),
    "ttmi_user_item_head_fwd_c": (c_i, [c_p, c_p, c_p]),
    "ttmi_user_item_head_fwd_ac": (c_i, [c_p, c_p, c_p]),
    "ttmi_item_head_bwd_c": (c_i, [c_p, c_p]),
    "ttmi_item_head_bn_part_floats": (ctypes.c_int64, [c_i]),
    "ttmi_item_head_bn_counter_bytes": (ctypes.c_int64, [c_i]),
    "ttmi_user_head_ffn_ws_bytes": (ctypes.c_int64, [c_i, c_i]),
    "ttmi_item_head_bwd_ws_floats": (ctypes.c_int64, [c_i]),
    "ttmi_user_item_head_bwd": (c_i, [c_p, c_p, c_p]),
    "ttmi_deb_pool_fwd": (c_i, [c_i, c_i, c_i, c_p, c_p, c_p, c_p]),
    "ttmi_deb_pool_bwd": (c_i, [c_i, c_i, c_i, c_p, c_p, c_p, c_p]),
    "ttmi_skinny_wgrad": (c_i, [c_i64, c_i, c_p, c_i64, c_p, c_i, c_i64, c_i, c_i, ctypes.c_float, c_p,
                                c_i64, c_i64, c_p, c_p]),
    "ttmi_mel_power": (c_i, [c_i, c_i64, c_p, c_i64, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_mel_db_minmax": (c_i, [c_i, c_i64, ctypes.c_float, ctypes.c_float, c_p, c_p]),
    "ttmi_cover_prep": (c_i, [c_i, c_i, c_i, c_p, c_i64, c_i, c_i, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_lora_dx": (c_i, [c_i64, c_i, c_p, c_i64, c_p, c_p, ctypes.c_float, ctypes.c_float, c_p, c_p,
                           c_i64, c_p, c_i64, c_p]),
    "ttmi_conv2d": (c_i, [c_p, c_p]),
    "ttmi_conv2d_workspace": (ctypes.c_int64, [c_p]),
    "ttmi_conv_weight_prep": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p]),
    "ttmi_nchw_to_nhwc": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p]),
    "ttmi_conv_weight_prep_batch": (c_i, [c_i, c_p, c_p]),
    "ttmi_stem_s2d": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p]),
    "ttmi_stem_weight_prep": (c_i, [c_i, c_i, c_i, c_p, c_p, c_p]),
    "ttmi_bn2d_fwd": (c_i, [c_i64, c_i, c_p, c_p, c_p, c_p, c_p, c_f, c_f, c_p, c_p, c_p, c_p, c_i,
                            c_p, c_p, c_p, c_p]),
    "ttmi_bn2d_bwd": (c_i, [c_i64, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_bn2d_bwd_reduce": (c_i, [c_i64, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_bn2d_bwd_apply": (c_i, [c_i64, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_maxpool_fwd": (c_i, [c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p]),
    "ttmi_maxpool_bwd": (c_i, [c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p]),
    "ttmi_stem_pool_fwd": (c_i, [c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_f, c_f, c_p, c_p, c_p,
                                 c_p, c_p, c_p, c_p, c_p]),
    "ttmi_stem_pool_bwd": (c_i, [c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                                 c_p, c_p, c_p]),
    "ttmi_avgpool_fwd": (c_i, [c_i, c_i, c_i, c_p, c_p, c_p]),
    "ttmi_avgpool_bwd": (c_i, [c_i, c_i, c_i, c_p, c_i, c_p, c_p, c_p]),
    "ttmi_l2norm_fwd": (c_i, [c_i, c_i, c_p, c_p, c_p, c_p]),
    "ttmi_l2norm_bwd": (c_i, [c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_rowce_fwd": (c_i, [c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_i64, c_f, c_p, c_p, c_p, c_p]),
    "ttmi_rowce_workspace": (c_i64, [c_i, c_i]),
    "ttmi_rowce_bwd": (c_i, [c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_f, c_p, c_f,
                             c_p, c_p, c_p, c_p]),
    "ttmi_sum_scaled": (c_i, [c_i, c_p, c_f, c_p, c_p]),
    "ttmi_step_inc": (c_i, [c_p, c_p]),
    "ttmi_dropout_seeds": (c_i, [c_u64, c_p, c_p, c_i, c_i, c_p]),
    "ttmi_cast_f32_bf16": (c_i, [c_i64, c_p, c_p, c_p]),
    "ttmi_dropout_bwd": (c_i, [c_i, c_i64, c_i, c_p, c_i64, c_f, c_p, c_i64, c_p, c_p, c_i64, c_p,
                               c_p]),
    "ttmi_last_rows": (c_i, [c_i, c_i, c_p, c_p, c_p]),
    "ttmi_last_rows_gather": (c_i, [c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p]),
    "ttmi_gather_rows": (c_i, [c_i, c_i, c_p, c_p, c_p, c_p]),
    "ttmi_scatter_add_rows": (c_i, [c_i, c_i, c_p, c_p, c_p, c_p]),
    "ttmi_mha_q1_fwd": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_f, c_p, c_p, c_p, c_p]),
    "ttmi_mha_q1_gather_fwd": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_f, c_p, c_p,
                                     c_p, c_p]),
    "ttmi_mha_q1_bwd": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_p]),
    "ttmi_mha_q1_kv_bwd": (c_i, [c_p, c_p]),
    "ttmi_mha_q1_bnr_bwd": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_f, c_p, c_p, c_p,
                                  c_p]),
    "ttmi_mha_q1_gather_item_fwd": (c_i, [c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_p, c_p, c_p, c_f, c_p,
                                          c_p, c_p, c_p, c_p]),
    "ttmi_colsum": (c_i, [c_i, c_i64, c_i, c_p, c_i64, c_p, c_p]),
}

_lib = None
_lock = threading.Lock()


class TTMIError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libttmi.so and bind every entry point.  Raises if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise TTMIError(
                f"libttmi.so not found at {path}: build it with `make` at the repo root "
                "(or __graft_entry__.build()).  There is no fallback path.")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.ttmi_abi_version()
        if v != ABI_VERSION:
            raise TTMIError(f"libttmi.so ABI {v} != expected {ABI_VERSION}; rebuild")
        _lib = lib
        return lib


def call(name: str, *args):
    """Invoke an entry point; raise TTMIError with ttmi_last_error() on failure."""
    lib = _lib if _lib is not None else load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.ttmi_last_error().decode(errors="replace")
        raise TTMIError(f"{name} failed (rc={rc}): {msg}")
    return rc
