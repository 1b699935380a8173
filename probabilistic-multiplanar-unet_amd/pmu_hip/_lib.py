"""ctypes binding of libpmunet_hip.so (the C ABI declared in include/pmunet_hip.h).

The library is loaded after ``import torch`` so that its ``libamdhip64.so.7`` dependency
binds to the HIP runtime torch already loaded (same SONAME) — one runtime, one set of
streams.  There is no fallback: if the library or a GPU is missing, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_longlong, c_size_t, c_void_p

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

# PMU_LIB=debug selects the bounds-checked debug build (csrc: make DEBUG=1; see pmu_debug_read);
# PMU_LIB=exp a kernel-variant A/B build (csrc: make EXPERIMENTS=1 BLD=build_exp
# OUT=../pmu_hip/libpmunet_hip_exp.so; not shipped, tools/ and scripts/ only)
# PMU_LIB=prev: a previous revision's release build placed there by an A/B script (scripts/gpu_r4_dma.sh)
LIB_NAME = {"debug": "libpmunet_hip_debug.so", "exp": "libpmunet_hip_exp.so",
            "prev": "libpmunet_hip_prev.so"}.get(os.environ.get("PMU_LIB", ""), "libpmunet_hip.so")
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
HEADER_PATH = os.path.normpath(
    os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "include", "pmunet_hip.h"))
EXP_HEADER_PATH = os.path.join(os.path.dirname(HEADER_PATH), "pmunet_hip_experiments.h")
EXP_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpmunet_hip_exp.so")

PMU_OK = 0
PMU_ERR_ARG = 1001
SRC_RAW, SRC_BNRELU, SRC_BNBWD = 0, 1, 2
POOL_NONE, POOL_MAX2, POOL_AVG2CEIL = 0, 1, 2
DT_X_BF16, DT_Z_BF16 = 1, 2


class PmuSrc(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("z", c_void_p), ("coef", c_void_p), ("mode", c_int), ("pool", c_int),
                ("C", c_int), ("H", c_int), ("W", c_int), ("off_h", c_int), ("off_w", c_int), ("dtype", c_int)]


class PmuFrame(ctypes.Structure):
    _fields_ = [("src", PmuSrc * 2), ("nsrc", c_int), ("N", c_int), ("H", c_int), ("W", c_int)]


class PmuPackJob(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("dst", c_void_p), ("Cout", c_int), ("Cin", c_int), ("block0", c_int),
                ("nblocks", c_int)]


class PmuSgdChunk(ctypes.Structure):
    _fields_ = [("tensor", c_int), ("len", c_int), ("start", c_longlong)]


_FP = POINTER(PmuFrame)
# name -> (restype, argtypes)
SIGNATURES = {
    "pmu_conv3x3_tiles": (c_int, [c_int, c_int, c_int]),
    "pmu_conv3x3_wgrad_ws": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "pmu_conv3x3_wgrad": (c_int, [_FP, _FP, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pmu_conv3x3_packed_size_wino": (c_size_t, [c_int, c_int, c_int]),
    "pmu_conv3x3_pack_wino": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_conv3x3_tiles_wino": (c_int, [c_int, c_int, c_int]),
    "pmu_conv3x3_fwd_wino": (c_int, [_FP, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_wino": (c_int, [_FP, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_packed_size_wino2h": (c_size_t, [c_int, c_int, c_int]),
    "pmu_conv3x3_pack_wino2h": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_conv3x3_tiles_wino2h": (c_int, [c_int, c_int, c_int]),
    "pmu_conv3x3_fwd_wino2h": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                       c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_wino2h": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                                         c_void_p, c_void_p]),
    "pmu_conv3x3_packed_size_wino4": (c_size_t, [c_int, c_int, c_int]),
    "pmu_conv3x3_pack_wino4": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_conv3x3_tiles_wino4": (c_int, [c_int, c_int, c_int]),
    "pmu_conv3x3_dgrad_wino4": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                                        c_void_p, c_void_p]),
    "pmu_conv3x3_wgrad_ws_wino": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "pmu_conv3x3_wgrad_wino": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                       c_size_t, c_void_p]),
    "pmu_conv3x3_packed_size_bf16": (c_size_t, [c_int, c_int, c_int]),
    "pmu_conv3x3_pack_bf16": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_conv3x3_fwd_bf16": (c_int, [_FP, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_bf16": (c_int, [_FP, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_packed_size_raw": (c_size_t, [c_int, c_int, c_int]),
    "pmu_conv3x3_tiles_raw": (c_int, [c_int, c_int, c_int, c_int]),
    "pmu_conv3x3_pack_raw": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_conv3x3_fwd_raw": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                    c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_raw": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                                      c_void_p, c_void_p]),
    "pmu_frame_to_bf16": (c_int, [_FP, c_int, c_void_p, c_void_p]),
    "pmu_frame_to_f32": (c_int, [_FP, c_void_p, c_void_p]),
    "pmu_frame_to_f32_ld": (c_int, [_FP, c_void_p, c_int, c_void_p]),
    "pmu_frame_to_bf16_ld": (c_int, [_FP, c_int, c_void_p, c_int, c_void_p]),
    "pmu_frame_pool_skip_ok": (c_int, [_FP]),
    "pmu_frame_to_bf16_pool_skip": (c_int, [_FP, c_void_p, c_void_p, c_int, c_void_p]),
    "pmu_frame_to_f32_pool_skip": (c_int, [_FP, c_void_p, c_void_p, c_int, c_void_p]),
    "pmu_conv3x3_wgrad_ws_bf16": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "pmu_conv3x3_wgrad_bf16": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                       c_size_t, c_void_p]),
    "pmu_convT2x2_wgrad_ws_bf16": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "pmu_convT2x2_wgrad_bf16": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                        c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pmu_occupancy_conv3x3_raw": (c_int, [POINTER(c_int)]),
    "pmu_occupancy_wgrad3x3_bf16": (c_int, [POINTER(c_int)]),
    "pmu_conv_first_fwd": (c_int, [POINTER(c_void_p), c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                                   c_void_p, c_void_p, c_void_p]),
    "pmu_conv_first_tiles": (c_int, [c_int, c_int, c_int]),
    "pmu_conv_first_wgrad_ws": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "pmu_conv_first_wgrad": (c_int, [_FP, POINTER(c_void_p), c_int, c_int, c_void_p, c_void_p, c_size_t,
                                     c_void_p]),
    "pmu_colsum_f64": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p]),
    "pmu_colsum_groups": (c_int, [c_int]),
    "pmu_bn_fwd_finalize": (c_int, [c_void_p, c_int, c_int, c_double, c_void_p, c_void_p, c_float, c_float,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_bn_eval_coef": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int, c_void_p, c_void_p]),
    "pmu_bn_bwd_reduce": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                  c_void_p]),
    "pmu_bn_bwd_tiles": (c_int, [c_int, c_int]),
    "pmu_bn_bwd_finalize": (c_int, [c_void_p, c_int, c_int, c_double, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_bnrelu_apply": (c_int, [c_void_p, c_void_p, c_longlong, c_int, c_void_p, c_void_p]),
    "pmu_maxpool2_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                 c_void_p]),
    "pmu_maxpool2_bwd_bnr_tiles": (c_int, [c_int, c_int, c_int, c_int]),
    "pmu_maxpool2_bwd_bnr": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                     c_void_p, c_int, c_void_p, c_void_p]),
    "pmu_avgpool2_bwd": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_avgpool2_bwd_bnr": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                     c_void_p, c_void_p, c_void_p]),
    "pmu_spatial_mean_bwd_bnr": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                         c_int, c_void_p, c_void_p, c_void_p]),
    "pmu_convT2x2_packed_size": (c_size_t, [c_int, c_int]),
    "pmu_convT2x2_pack": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_convT2x2_fwd": (c_int, [_FP, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "pmu_convT2x2_fwd_ld_ok": (c_int, [_FP, c_int]),
    "pmu_convT2x2_fwd_ld": (c_int, [_FP, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "pmu_convT2x2_dgrad": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                   c_int, c_int, c_void_p, c_void_p]),
    "pmu_convT2x2_wgrad_ws": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "pmu_convT2x2_wgrad": (c_int, [c_void_p, c_int, c_int, c_int, c_int, _FP, c_int, c_void_p, c_void_p,
                                   c_void_p, c_size_t, c_void_p]),
    "pmu_head1x1_fwd": (c_int, [_FP, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "pmu_head1x1_bwd": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                c_void_p, c_void_p, c_void_p]),
    "pmu_head1x1_bwd_bnr_ok": (c_int, [c_int, c_int, c_int, c_int]),
    "pmu_head1x1_bwd_tiles": (c_int, [c_int, c_int, c_int]),
    "pmu_head1x1_bwd_bnr": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_size_t, c_void_p]),
    "pmu_head1x1_bwd_dz": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                   c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "pmu_wgrad1x1_ws": (c_size_t, [c_int, c_int, c_int]),
    "pmu_wgrad1x1": (c_int, [c_void_p, _FP, c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pmu_sgd_clip": (c_int, [c_void_p, c_int, c_void_p, c_float, c_float, c_float, c_float, c_void_p]),
    "pmu_loss_ws": (c_size_t, [c_longlong]),
    "pmu_bce_fwd": (c_int, [c_void_p, c_void_p, c_longlong, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_bce_bwd": (c_int, [c_void_p, c_void_p, c_longlong, c_int, c_void_p, c_void_p, c_void_p]),
    "pmu_ce_fwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_longlong, c_int, c_longlong, c_void_p, c_void_p,
                           c_void_p, c_void_p]),
    "pmu_ce_bwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_longlong, c_int, c_longlong, c_void_p, c_void_p,
                           c_void_p, c_void_p]),
    "pmu_dice_counts": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_dice_counts_many": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_dice_sums": (c_int, [c_void_p, c_void_p, c_longlong, c_void_p, c_void_p]),
    "pmu_slice_view_layout": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                      c_void_p]),
    "pmu_slice_max": (c_int, [c_void_p, c_int, c_longlong, c_void_p, c_void_p]),
    "pmu_gather_slices": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_longlong, c_int, c_void_p, c_void_p]),
    "pmu_fuse3view": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                              c_void_p, c_void_p, c_void_p]),
    "pmu_spatial_mean": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_spatial_mean_bwd": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_linear_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_linear_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                               c_void_p]),
    "pmu_fcomb_zbias": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_fcomb_fwd": (c_int, [c_void_p, c_void_p, POINTER(c_void_p), POINTER(c_void_p), c_void_p, c_void_p,
                              c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_fcomb_bwd_ws": (c_size_t, [c_int, c_int, c_int]),
    "pmu_fcomb_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, POINTER(c_void_p), POINTER(c_void_p),
                              c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                              c_void_p, POINTER(c_void_p), POINTER(c_void_p), c_void_p, c_void_p, c_void_p,
                              c_size_t, c_void_p]),
    "pmu_conv3x3_dma_ok": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "pmu_conv3x3_tiles_dma": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "pmu_conv3x3_packed_size_dma": (c_size_t, [c_int, c_int, c_int]),
    "pmu_conv3x3_pack_dma": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_conv3x3_fwd_dma": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                    c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_dma": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                                      c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_dma_x1b": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                                          c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_dma_x1b_sum": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int,
                                              c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_convT2x2_dbias_rows_ws": (c_size_t, [c_int]),
    "pmu_convT2x2_dbias_rows": (c_int, [c_void_p, c_int, c_longlong, c_int, c_void_p, c_void_p, c_void_p]),
    "pmu_convT2x2_dma_ok": (c_int, [c_int, c_int, c_int]),
    "pmu_convT2x2_packed_size_dma": (c_size_t, [c_int, c_int]),
    "pmu_convT2x2_pack_dma": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_convT2x2_fwd_dma": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int,
                                     c_void_p, c_void_p]),
    "pmu_convT2x2_fwd_dma_ldb": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int,
                                         c_void_p, c_int, c_void_p]),
    "pmu_convT2x2_dgrad_dma": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int,
                                       c_int, c_int, c_void_p, c_void_p]),
    "pmu_convT2x2_dgrad_dma_dxb": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int,
                                           c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_wino2h_bnr": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p,
                                             c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_wino4_bnr": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p,
                                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_dma_bnr": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_dma_dxb": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                                          c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_dma_x1b_dxb": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int,
                                              c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_dma_x1b_sum_dxb": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int,
                                                  c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_dma_bnr_dxb": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p,
                                              c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_wgrad_dma_ok": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "pmu_conv3x3_wgrad_ws_bf16_dma": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "pmu_conv3x3_wgrad_bf16_dma": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                           c_size_t, c_void_p]),
    "pmu_bn_bwd_reduce_dxb": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                      c_void_p]),
    "pmu_maxpool2_bwd_bnr_dxb": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                         c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "pmu_maxpool2_bwd_bnr_stats_dxb": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                               c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_maxpool2_bwd_bnbwd_dxb": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                           c_int, c_int, c_void_p, c_void_p]),
    "pmu_maxpool2_bwd_bnr_stats": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                           c_int, c_int, c_void_p, c_void_p]),
    "pmu_maxpool2_bwd_bnbwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                       c_int, c_void_p, c_void_p]),
    "pmu_conv3x3_pack_wino2h_blocks": (c_int, [c_int, c_int, c_int]),
    "pmu_conv3x3_pack_wino2h_multi": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p]),
    "pmu_conv3x3_pack_wino4_blocks": (c_int, [c_int, c_int, c_int]),
    "pmu_conv3x3_pack_wino4_multi": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p]),
    "pmu_convT2x2_pack_blocks": (c_int, [c_int, c_int, c_int]),
    "pmu_convT2x2_pack_multi": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p]),
    "pmu_conv3x3_pack_dma_blocks": (c_int, [c_int, c_int, c_int]),
    "pmu_conv3x3_pack_dma_multi": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p]),
    "pmu_convT2x2_pack_dma_blocks": (c_int, [c_int, c_int, c_int]),
    "pmu_convT2x2_pack_dma_multi": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p]),
    "pmu_build_flags": (c_int, []),
    "pmu_debug_read": (c_int, [POINTER(c_int), POINTER(ctypes.c_char_p)]),
    "pmu_debug_reset": (c_int, []),
}
# The experiments build's extra entries (include/pmunet_hip_experiments.h; csrc make EXPERIMENTS=1): bound
# when the loaded library exports them, never by the shipped one.
EXP_SIGNATURES = {
    "pmu_conv3x3_fwd": (c_int, [_FP, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_packed_size": (c_size_t, [c_int, c_int, c_int]),
    "pmu_conv3x3_pack": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad": (c_int, [_FP, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_fwd_wino_raw": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                         c_void_p, c_void_p]),
    "pmu_conv3x3_dgrad_wino_raw": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                                           c_void_p, c_void_p]),
    "pmu_conv3x3_fwd_wino4": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                      c_void_p, c_void_p]),
    "pmu_convT2x2_pack_bf16": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pmu_convT2x2_bf16_ok": (c_int, [_FP, c_int]),
    "pmu_convT2x2_fwd_bf16": (c_int, [_FP, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "pmu_convT2x2_dgrad_bf16": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int,
                                        c_int, c_void_p, c_void_p]),
    "pmu_occupancy_conv3x3_pipe": (c_int, [POINTER(c_int)]),
    "pmu_conv3x3_dma_persistent": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "pmu_bn_bwd_reduce_zb": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                     c_void_p]),
    "pmu_maxpool2_bwd_zb": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                    c_void_p]),
    "pmu_conv3x3_fwd_dma_zb": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                       c_void_p, c_void_p, c_void_p]),
    "pmu_bn_center": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "pmu_conv3x3_wgrad_ws_wino4": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "pmu_conv3x3_wgrad_wino4": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                        c_size_t, c_void_p]),
    "pmu_conv3x3_dgrad_dma_bnr_zb": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p,
                                             c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
}

# The entry points whose kernels issue MFMAs (every other entry is VALU / memory work).  bench.py's
# KernelTimer counts exactly these, each with a FLOP formula; tests/test_cpu_host.py checks that every
# one of them has a non-zero formula and is declared in SIGNATURES.
MFMA_ENTRY_POINTS = (
    # fp32 direct-sum and Winograd 3x3 convs (conv3x3*.hip, wgrad3x3*.hip)
    "pmu_conv3x3_fwd", "pmu_conv3x3_dgrad", "pmu_conv3x3_wgrad",
    "pmu_conv3x3_fwd_wino", "pmu_conv3x3_dgrad_wino", "pmu_conv3x3_wgrad_wino",
    "pmu_conv3x3_fwd_wino_raw", "pmu_conv3x3_dgrad_wino_raw",
    "pmu_conv3x3_fwd_wino2h", "pmu_conv3x3_dgrad_wino2h", "pmu_conv3x3_dgrad_wino2h_bnr",
    "pmu_conv3x3_fwd_wino4", "pmu_conv3x3_dgrad_wino4", "pmu_conv3x3_dgrad_wino4_bnr", "pmu_conv3x3_wgrad_wino4",
    # bf16 3x3 convs
    "pmu_conv3x3_fwd_bf16", "pmu_conv3x3_dgrad_bf16", "pmu_conv3x3_wgrad_bf16", "pmu_conv3x3_wgrad_bf16_dma",
    "pmu_conv3x3_fwd_raw", "pmu_conv3x3_dgrad_raw",
    "pmu_conv3x3_fwd_dma", "pmu_conv3x3_fwd_dma_zb", "pmu_conv3x3_dgrad_dma", "pmu_conv3x3_dgrad_dma_bnr",
    "pmu_conv3x3_dgrad_dma_bnr_zb", "pmu_conv3x3_dgrad_dma_x1b", "pmu_conv3x3_dgrad_dma_x1b_sum",
    "pmu_conv3x3_dgrad_dma_dxb", "pmu_conv3x3_dgrad_dma_bnr_dxb", "pmu_conv3x3_dgrad_dma_x1b_dxb",
    "pmu_conv3x3_dgrad_dma_x1b_sum_dxb",
    # transposed convs
    "pmu_convT2x2_fwd", "pmu_convT2x2_fwd_ld", "pmu_convT2x2_dgrad", "pmu_convT2x2_wgrad",
    "pmu_convT2x2_fwd_bf16", "pmu_convT2x2_dgrad_bf16", "pmu_convT2x2_wgrad_bf16",
    "pmu_convT2x2_fwd_dma", "pmu_convT2x2_fwd_dma_ldb", "pmu_convT2x2_dgrad_dma", "pmu_convT2x2_dgrad_dma_dxb",
    # the Probabilistic U-Net's Fcomb
    "pmu_fcomb_fwd", "pmu_fcomb_bwd",
)

_LIB = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load the shared library and declare every signature (no GPU needed)."""
    if not os.path.exists(path):
        raise ImportError(
            f"{LIB_NAME} not found at {path}: build it with `make -C csrc` (or __graft_entry__.build()). "
            "There is no CPU fallback for the PMU hot path.")
    cdll = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(cdll, name)  # AttributeError if the export is missing
        fn.restype = res
        fn.argtypes = args
    for name, (res, args) in EXP_SIGNATURES.items():
        if hasattr(cdll, name):
            fn = getattr(cdll, name)
            fn.restype = res
            fn.argtypes = args
    return cdll


def lib() -> ctypes.CDLL:
    """The loaded library; raises unless a ROCm GPU is present (the product path never runs on CPU)."""
    global _LIB
    if _LIB is None:
        if not torch.cuda.is_available():
            raise RuntimeError("pmu_hip requires an AMD GPU (gfx950); torch.cuda.is_available() is False. "
                               "There is no CPU fallback for the PMU hot path.")
        _LIB = load_library()
    return _LIB


_HIP_ERR = {1: "hipErrorInvalidValue", 2: "hipErrorOutOfMemory", 98: "hipErrorInvalidDeviceFunction",
            209: "hipErrorNoBinaryForGpu", 700: "hipErrorIllegalAddress"}


def check(rc: int, name: str) -> None:
    if rc != PMU_OK:
        what = "invalid argument" if rc == PMU_ERR_ARG else _HIP_ERR.get(rc, f"hipError {rc}")
        raise RuntimeError(f"{name} failed: {what} (code {rc})")


_OBSERVER = None


def set_call_observer(fn) -> None:
    """Install fn(name, args, start_event, end_event) around every launch (None to remove).
    Used by bench.py to time kernels with HIP events on the launch stream."""
    global _OBSERVER
    _OBSERVER = fn


def call(name: str, *args) -> None:
    obs = _OBSERVER
    if obs is None:
        check(getattr(lib(), name)(*args), name)
        return
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    check(getattr(lib(), name)(*args), name)
    e1.record()
    obs(name, args, e0, e1)


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


BUILD_EXPERIMENTS, BUILD_DEBUG = 1, 2


def build_flags() -> int:
    """pmu_build_flags() of the loaded library (cached on it: the engine asks per conv)."""
    cdll = lib()
    f = cdll.__dict__.get("_pmu_flags")
    if f is None:
        f = int(cdll.pmu_build_flags())
        cdll.__dict__["_pmu_flags"] = f
    return f


def experiments_build() -> bool:
    """True for a `make EXPERIMENTS=1` library (kernel-variant A/B switches honoured)."""
    return bool(build_flags() & BUILD_EXPERIMENTS)


def debug_build() -> bool:
    """True when the bounds-checked debug library (PMU_LIB=debug) is loaded."""
    return bool(build_flags() & BUILD_DEBUG)


DBG_CODES = {1: "operand read outside the operand tensor", 2: "store outside the output tensor",
             3: "workgroup mapped outside the problem", 4: "data-dependent index out of range",
             5: "workspace row out of range"}


def debug_check(reset: bool = True) -> None:
    """Debug build: raise if any kernel recorded an index-bound violation since the last reset
    (synchronises the device).  No-op with the release library."""
    out = (c_int * 5)()
    tu = ctypes.c_char_p()
    check(lib().pmu_debug_read(out, ctypes.byref(tu)), "pmu_debug_read")
    if out[3]:
        if reset:
            check(lib().pmu_debug_reset(), "pmu_debug_reset")
        where = tu.value.decode() if tu.value else "?"
        raise RuntimeError(f"PMU debug build: {DBG_CODES.get(out[0], out[0])} at {os.path.basename(where)}:{out[1]} "
                           f"(workgroup {out[2]})")
