"""ctypes binding of libgwn.so (include/gwn.h).

The library is the only compute path of this package: if it is missing or fails to load, every
product entry point raises (there is no CPU or eager-PyTorch fallback).  PyTorch is used only as
the device-memory / stream provider: tensors are passed as raw device pointers together with
``torch.cuda.current_stream().cuda_stream``.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# GWN_LIB: alternative build of the same library (kernel experiments, tools/); default in-tree
LIB_PATH = os.environ.get("GWN_LIB") or os.path.join(_HERE, "libgwn.so")

c_int, c_long, c_float, c_void_p, c_u64 = (ctypes.c_int, ctypes.c_long, ctypes.c_float,
                                          ctypes.c_void_p, ctypes.c_ulonglong)


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("A", c_void_p), ("lda_m", c_long), ("lda_k", c_long), ("a_ko_stride", c_long),
        ("a_kin", c_int), ("a_row_shift", c_int), ("a_rows", c_int),
        ("B", c_void_p), ("ldb_k", c_long), ("ldb_n", c_long), ("b_ko_stride", c_long),
        ("b_no_stride", c_long), ("b_kin", c_int), ("b_nin", c_int),
        ("C", c_void_p), ("ldc_m", c_long), ("ldc_n", c_long), ("c_no_stride", c_long), ("c_nin", c_int),
        ("C0", c_void_p), ("ldc0_m", c_long), ("ldc0_n", c_long), ("c0_no_stride", c_long), ("beta", c_float),
        ("bias_n", c_void_p),
        ("mask", c_void_p), ("ldmask_m", c_long),
        ("M", c_int), ("N", c_int), ("K", c_int),
        ("alpha", c_float),
        ("epi", c_int), ("relu", c_int),
        ("aux", c_void_p), ("ld_aux", c_long),
        ("aux2", c_void_p), ("ld_aux2", c_long), ("aux2_row0", c_int),
        ("seed_ptr", c_void_p), ("seed_salt", c_u64), ("drop_p", c_float),
        ("ksplit", c_int), ("kchunk", c_int), ("part", c_void_p), ("ones_out", c_void_p),
        ("batch", c_int), ("a_bstride", c_long), ("b_bstride", c_long), ("c_bstride", c_long),
    ]


class TcnArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("t_in", c_int), ("P", c_int), ("c", c_int), ("dilation", c_int),
        ("w_fg", c_void_p), ("b_fg", c_void_p),
        ("xg", c_void_p), ("ld_xg", c_long),
        ("fg", c_void_p),
        ("skipcat", c_void_p), ("ld_skip", c_long), ("skip_row0", c_int),
        ("x_mean", c_void_p),
        ("ntaps", c_int), ("c_out", c_int),
        ("bn", c_void_p), ("bn_partials", c_void_p), ("bn_nparts", c_int),
    ]


class TcnBwdArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("t_in", c_int), ("P", c_int), ("c", c_int), ("dilation", c_int),
        ("w_fg", c_void_p), ("fg", c_void_p),
        ("dxg", c_void_p), ("ld_dxg", c_long),
        ("dskip", c_void_p), ("ld_dskip", c_long), ("skip_row0", c_int),
        ("dfg", c_void_p),
        ("dw_fg", c_void_p), ("db_fg", c_void_p),
        ("dx", c_void_p), ("accumulate_dx", c_int),
        ("workspace", c_void_p),
        ("skip_weight_grads", c_int),
        ("dfg_ready", c_int), ("acc_row0", c_long),
        ("bn_z", c_void_p), ("bn_mean", c_void_p), ("bn_rstd", c_void_p), ("bn_sums", c_void_p),
        ("x_mean", c_void_p), ("x_scale", c_void_p), ("x_shift", c_void_p),
        ("ntaps", c_int), ("c_out", c_int),
    ]


class BnFold(ctypes.Structure):
    _fields_ = [
        ("gamma", c_void_p), ("beta", c_void_p), ("running_mean", c_void_p), ("running_var", c_void_p),
        ("momentum", c_float), ("eps", c_float),
        ("save_mean", c_void_p), ("save_rstd", c_void_p), ("scale", c_void_p),
        ("w_next", c_void_p), ("b_next", c_void_p), ("w_fold", c_void_p), ("b_fold", c_void_p),
        ("num_batches_tracked", c_void_p),
    ]


class GcnArgs(ctypes.Structure):
    _fields_ = [
        ("rows", c_int), ("n", c_int), ("c", c_int), ("nsup", c_int),
        ("sup", ctypes.POINTER(c_void_p)), ("ld_sup", c_int),
        ("h", c_void_p), ("ld_h", c_long),
        ("w_mlp", c_void_p), ("b_mlp", c_void_p),
        ("residual", c_void_p),
        ("z", c_void_p),
        ("seed_ptr", c_void_p), ("salt", c_u64), ("drop_p", c_float),
        ("bn_partials", c_void_p),
        ("no_pieces", c_int),
        ("bn_running_mean", c_void_p), ("bn_running_var", c_void_p), ("bn_weight", c_void_p),
        ("bn_bias", c_void_p), ("bn_eps", c_float), ("bn_out", c_void_p),
        ("layout", c_int),
        ("split_planes", c_int),
        ("sup_bstride", c_long), ("sup_batch", c_int),
        ("residual_mean", c_void_p), ("residual_scale", c_void_p), ("residual_shift", c_void_p),
        ("ksplit", c_int), ("ksplit_ws", c_void_p), ("ksplit_count", c_void_p),
        ("sup2", ctypes.POINTER(c_void_p)),
        ("w_mlp_t", c_void_p),
        ("c_out", c_int),
        ("sup_g4", ctypes.POINTER(c_void_p)),
        ("sup_g4b", ctypes.POINTER(c_void_p)),
        ("xg4", c_void_p), ("xg4_support", c_int),
        ("pieces_bf16", c_void_p), ("ld_pb", c_long),
        ("bn_fold", ctypes.POINTER(BnFold)),
        ("tcn", ctypes.POINTER(TcnArgs)),
        ("clock", c_void_p),
        ("bn_slots_used", ctypes.POINTER(c_int)),
    ]


class ReduceSeg(ctypes.Structure):
    _fields_ = [
        ("part", c_void_p), ("nparts", c_int), ("part_stride", c_long),
        ("J", c_int), ("Kc", c_int),
        ("out", c_void_p), ("ld_out", c_long), ("out2", c_void_p),
        ("db_off", c_long),
    ]


class WgradProblem(ctypes.Structure):
    _fields_ = [
        ("dY", c_void_p), ("ldy", c_long),
        ("X", c_void_p), ("ldx", c_long), ("x_rows", c_long), ("shift", c_long),
        ("x_mean", c_void_p), ("x_scale", c_void_p), ("x_shift", c_void_p),
        ("part", c_void_p),
        ("R", c_int),
        ("Xb", c_void_p), ("ldxb", c_long),
    ]


class GramLayer(ctypes.Structure):
    _fields_ = [("x1", c_void_p), ("t1", c_void_p), ("x2", c_void_p), ("t2", c_void_p), ("slices", c_int)]


class GcnBwdArgs(ctypes.Structure):
    _fields_ = [
        ("rows", c_int), ("n", c_int), ("c", c_int), ("nsup", c_int),
        ("sup", ctypes.POINTER(c_void_p)), ("ld_sup", c_int),
        ("h", c_void_p), ("ld_h", c_long),
        ("w_mlp", c_void_p),
        ("dh", c_void_p),
        ("dhcat", c_void_p), ("ld_dhcat", c_long),
        ("dw_mlp", c_void_p), ("db_mlp", c_void_p),
        ("adp_index", c_int), ("dadp", c_void_p), ("accumulate_dadp", c_int),
        ("workspace", c_void_p),
        ("sup_t", ctypes.POINTER(c_void_p)),
        ("skip_weight_grads", c_int),
        ("bn_dy", c_void_p), ("bn_z", c_void_p), ("bn_gamma", c_void_p), ("bn_mean", c_void_p),
        ("bn_rstd", c_void_p), ("bn_sums", c_void_p), ("bn_dgamma", c_void_p), ("bn_dbeta", c_void_p),
        ("dres", c_void_p), ("dh_out", c_void_p),
        ("seed_ptr", c_void_p), ("salt", c_u64), ("drop_p", c_float),
        ("fg", c_void_p), ("dskip", c_void_p), ("ld_dskip", c_long), ("skip_row0", c_int),
        ("dfg", c_void_p),
        ("layout", c_int),
        ("sup_bstride", c_long), ("sup_batch", c_int),
        ("split_planes", c_int),
        ("ksplit", c_int), ("ksplit_ws", c_void_p), ("ksplit_count", c_void_p),
        ("sup2_t", ctypes.POINTER(c_void_p)),
        ("c_out", c_int),
        ("sup_g4_t", ctypes.POINTER(c_void_p)),
        ("sup_g4b_t", ctypes.POINTER(c_void_p)),
        ("tg4", c_void_p),
    ]

# ctypes mirrors checked against the library's own sizeof (gwn_abi_sizeof) at load time
_STRUCTS = {"gwn_gemm_desc": GemmDesc, "gwn_tcn_args": TcnArgs, "gwn_tcn_bwd_args": TcnBwdArgs,
            "gwn_gcn_args": GcnArgs, "gwn_gcn_bwd_args": GcnBwdArgs, "gwn_reduce_seg": ReduceSeg,
            "gwn_wgrad_problem": WgradProblem, "gwn_gram_layer": GramLayer,
            "gwn_bn_fold": BnFold}


# (name, restype, argtypes) of every exported entry point declared in include/gwn.h
_SIGS = [
    ("gwn_version", c_int, []),
    ("gwn_set_sync_check", None, [c_int]),
    ("gwn_last_error", ctypes.c_char_p, []),
    ("gwn_abi_sizeof", c_long, [ctypes.c_char_p]),
    ("gwn_gemm", c_int, [ctypes.POINTER(GemmDesc), c_void_p]),
    ("gwn_gemm_nt", c_int, [c_void_p, c_long, c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_int,
                            c_void_p, c_int, c_void_p, c_long, c_void_p]),
    ("gwn_gemm_nt_bf16", c_int, [c_void_p, c_long, c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_int,
                                 c_void_p, c_int, c_void_p, c_long, c_void_p]),
    ("gwn_gemm_workspace_floats", c_long, [c_int, c_int, c_int]),
    ("gwn_nconv", c_int, [c_void_p, c_int, c_int, c_void_p, c_long, c_void_p, c_long, c_void_p, c_long,
                          c_int, c_int, c_int, c_void_p]),
    ("gwn_nconv_adj_grad", c_int, [c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_int, c_void_p,
                                   c_int, c_int, c_void_p, c_void_p]),
    ("gwn_nconv_adj_grad_workspace_floats", c_long, [c_int, c_int, c_int]),
    ("gwn_adaptive_adj_fwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p]),
    ("gwn_adaptive_adj_bwd", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                     c_void_p, c_void_p, c_void_p, c_void_p]),
    ("gwn_start_conv_fwd", c_int, [c_void_p, c_long, c_long, c_long, c_long, c_int, c_int, c_int, c_int,
                                   c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    ("gwn_gated_tcn_fwd", c_int, [ctypes.POINTER(TcnArgs), c_void_p]),
    ("gwn_gated_tcn_bwd", c_int, [ctypes.POINTER(TcnBwdArgs), c_void_p]),
    ("gwn_gated_tcn_bwd_workspace_floats", c_long, [c_int, c_int, c_int, c_int]),
    ("gwn_gated_tcn_bwd_workspace_floats_ex", c_long, [c_int, c_int, c_int, c_int, c_int, c_int]),
    ("gwn_nconv2", c_int, [c_void_p, c_int, c_long, c_int, c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_int,
                           c_int, c_void_p]),
    ("gwn_nconv2_adj_grad", c_int, [c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                    c_long, c_int, c_void_p]),
    ("gwn_gcn_fwd", c_int, [ctypes.POINTER(GcnArgs), c_void_p]),
    ("gwn_gcn_tcn_fused", c_int, [ctypes.POINTER(GcnArgs)]),
    ("gwn_wall_clock_khz", c_int, []),
    ("gwn_gcn_bn_partial_count", c_long, [c_int, c_int, c_int, c_int, c_int]),
    ("gwn_gcn_t16b_supported", c_int, [c_int, c_int]),
    ("gwn_gcn_bwd", c_int, [ctypes.POINTER(GcnBwdArgs), c_void_p]),
    ("gwn_gcn_bwd_workspace_floats", c_long, [c_int, c_int, c_int, c_int]),
    ("gwn_gcn_bwd_workspace_floats_ex", c_long, [c_int, c_int, c_int, c_int, c_int]),
    ("gwn_gcn_ksplit_ws_floats", c_long, [c_int, c_int, c_int]),
    ("gwn_wgrad", c_int, [c_void_p, c_long, c_int, c_void_p, c_long, c_long, c_int, c_int, c_long, c_int,
                          c_void_p, c_long, c_void_p, c_void_p, c_void_p]),
    ("gwn_wgrad_workspace_floats", c_long, [c_int, c_int, c_int]),
    ("gwn_wgrad_partial_count", c_int, [c_int, c_int, c_int]),
    ("gwn_wgrad_partials", c_int, [c_void_p, c_long, c_int, c_void_p, c_long, c_long, c_int, c_int, c_long, c_int,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("gwn_reduce_partials", c_int, [ctypes.POINTER(ReduceSeg), c_int, c_void_p]),
    ("gwn_wgrad_bf16_partial_count", c_int, [c_int, c_int, c_int]),
    ("gwn_wgrad_bf16_partials", c_int, [c_void_p, c_long, c_int, c_void_p, c_long, c_int, c_int, c_void_p, c_void_p]),
    ("gwn_wgrad_group_supported", c_int, [c_int, c_int, c_int]),
    ("gwn_gram_group_workspace_floats", c_long, [c_int, ctypes.POINTER(c_int), c_int]),
    ("gwn_gram_group", c_int, [ctypes.POINTER(GramLayer), c_int, c_long, c_long, c_int, c_void_p, c_int, c_int,
                               c_void_p, c_void_p]),
    ("gwn_gram_g4_group_workspace_floats", c_long, [c_int, ctypes.POINTER(c_int), c_int]),
    ("gwn_gram_g4_group", c_int, [ctypes.POINTER(GramLayer), c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    ("gwn_wgrad_group_plan", c_int, [ctypes.POINTER(c_int), c_int, c_int, c_int, c_int, ctypes.POINTER(c_int)]),
    ("gwn_wgrad_group", c_int, [ctypes.POINTER(WgradProblem), c_int, c_int, c_int, c_int, c_void_p]),
    ("gwn_wgrad_bn", c_int, [c_void_p, c_long, c_int, c_void_p, c_long, c_long, c_int, c_int, c_long, c_int,
                             c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_void_p]),
    ("gwn_gram", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_long, c_int, c_int, c_void_p, c_int,
                         c_int, c_void_p, c_void_p]),
    ("gwn_masked_loss_rows", c_int, [c_void_p, c_int, c_void_p, c_long, c_long, c_long, c_int, c_int, c_int, c_int,
                                     c_float, c_float, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    ("gwn_gather_sum", c_int, [c_void_p, c_void_p, c_void_p, c_long, c_long, c_int, c_int, c_long, c_void_p]),
    ("gwn_gram_workspace_floats", c_long, [c_int, c_int]),
    ("gwn_gram_g4_bf16", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                            c_void_p]),
    ("gwn_gram_g4_workspace_floats", c_long, [c_int, c_int]),
    ("gwn_gram_bf16", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_long, c_int, c_int, c_void_p, c_int,
                              c_int, c_void_p, c_void_p]),
    ("gwn_batchnorm_fwd", c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float,
                                  c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("gwn_batchnorm_workspace_floats", c_long, [c_int, c_int]),
    ("gwn_batchnorm_fwd_partials", c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p]),
    ("gwn_batchnorm_fwd_fold", c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float,
                                       c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p]),
    ("gwn_fused_occupancy", c_int, [c_int, c_int, c_int]),
    ("gwn_support_square", c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("gwn_support_square_g4", c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_long,
                                      c_int, c_void_p]),
    ("gwn_support_g4_floats", c_long, [c_int]),
    ("gwn_support_g4_bf16_elems", c_long, [c_int]),
    ("gwn_support_g4_bf16", c_int, [ctypes.POINTER(c_void_p), c_int, c_int, c_int, c_void_p, c_long, c_void_p]),
    ("gwn_support_g4", c_int, [ctypes.POINTER(c_void_p), c_int, c_int, c_int, c_void_p, c_long, c_void_p]),
    ("gwn_transpose", c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p]),
    ("gwn_pad_square", c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p]),
    ("gwn_pad_square_batched", c_int, [c_void_p, c_int, c_long, c_int, c_int, c_void_p, c_int, c_int, c_long, c_int,
                                       c_void_p]),
    ("gwn_adaptive_adj_fwd_batched", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_long,
                                             c_void_p]),
    ("gwn_batchnorm_bwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_u64, c_float, c_int,
                                  c_void_p, c_void_p]),
    ("gwn_colsum", c_int, [c_void_p, c_int, c_int, c_long, c_void_p, c_int, c_void_p, c_void_p]),
    ("gwn_colsum_workspace_floats", c_long, [c_int, c_int]),
    ("gwn_masked_loss", c_int, [c_void_p, c_void_p, c_long, c_long, c_long, c_int, c_int, c_int, c_int,
                                c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("gwn_masked_loss_workspace_floats", c_long, [c_int, c_int, c_int, c_int]),
    ("gwn_clip_adam", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_long,
                              c_float, c_float, c_float, c_float, c_float, c_float, c_void_p, c_void_p,
                              c_void_p, c_void_p]),
    ("gwn_clip_adam_workspace_floats", c_long, [c_long]),
    ("gwn_adam_clipped", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_long,
                                 c_float, c_float, c_float, c_float, c_float, c_float, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_u64, c_void_p]),
    ("gwn_gather_sqnorm", c_int, [c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_void_p]),
    ("gwn_sqnorm_partials", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_long, c_void_p, c_void_p]),
    ("gwn_gather", c_int, [c_void_p, c_void_p, c_void_p, c_long, c_void_p]),
    ("gwn_to_nchw", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    ("gwn_from_nchw", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    ("gwn_from_nchw_ld", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    ("gwn_sum_vectors", c_int, [c_void_p, c_int, c_int, c_long, c_void_p, c_void_p]),
    ("gwn_increment_u64", c_int, [c_void_p, c_u64, c_void_p]),
    ("gwn_horizon_metrics", c_int, [c_void_p, c_long, c_long, c_long, c_void_p, c_long, c_long, c_long, c_int,
                                    c_int, c_int, c_float, c_float, c_void_p, c_void_p, c_void_p]),
    ("gwn_horizon_metrics_workspace_floats", c_long, [c_int]),
    ("gwn_gather_rows", c_int, [c_void_p, c_long, c_void_p, c_int, c_void_p, c_void_p]),
    ("gwn_window_batch", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                 c_int, ctypes.c_double, ctypes.c_double, c_int, c_void_p, c_void_p, c_void_p]),
]

EXPORTED = [s[0] for s in _SIGS]

_lib = None


class GwnError(RuntimeError):
    pass


def load():
    """Load libgwn.so (raises if it is missing: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise GwnError("libgwn.so not found at %s; run build.sh (or __graft_entry__.build())" % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        for name, res, args in _SIGS:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        for cname, st in _STRUCTS.items():
            if lib.gwn_abi_sizeof(cname.encode()) != ctypes.sizeof(st):
                raise GwnError("libgwn.so ABI mismatch: sizeof(%s) = %d, ctypes mirror %d (stale build?)"
                               % (cname, lib.gwn_abi_sizeof(cname.encode()), ctypes.sizeof(st)))
        _lib = lib
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = load().gwn_last_error().decode(errors="replace")
        raise GwnError("libgwn %s failed (%d): %s" % (what, rc, msg))


def ptr(t):
    """Raw device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


_SYNC_CHECK = os.environ.get("GWN_SYNC_CHECK", "0") == "1"


def call(name, *args):
    """Invoke an int-returning entry point and raise on failure.  With GWN_SYNC_CHECK=1 (debugging)
    the library synchronises after every kernel, except while the stream is being captured."""
    lib = load()
    if _SYNC_CHECK:
        import torch
        lib.gwn_set_sync_check(2 if torch.cuda.is_current_stream_capturing() else 1)
    rc = getattr(lib, name)(*args)
    check(rc, name)
