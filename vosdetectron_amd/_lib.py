"""ctypes binding of libvosdet.so (the C ABI in include/vosdet.h).

The library is the product: every operator in this package calls into it and
there is no CPU or PyTorch fallback.  If the shared object is missing the first
call raises ``RuntimeError`` (run ``python -c "import __graft_entry__ as g;
g.build()"`` or ``make -C vosdetectron_amd/csrc``).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libvosdet.so")
# research builds (make VD_RESEARCH=1 OUT=...) are loaded by tools/research via this
# override; the product and the tests use the in-tree library
if os.environ.get("VOSDET_RESEARCH_LIB"):
    LIB_PATH = os.environ["VOSDET_RESEARCH_LIB"]
# pinned per-shape GEMM kernel choices (csrc/gemm_epi.cpp): the same file for
# every process -- GPU tests, bench, all ranks -- so they compute the same numbers
GEMM_PLANS = os.path.join(_HERE, "gemm_plans.txt")
os.environ.setdefault("VOSDET_GEMM_PLANS", GEMM_PLANS)

VD_OK, VD_ERR_ARG, VD_ERR_SHAPE, VD_ERR_LAUNCH, VD_ERR_WORKSPACE = range(5)
VD_LAYOUT_NCHW, VD_LAYOUT_NHWC = 0, 1
VD_MAX_LEVELS = 5
VD_ACT_NONE, VD_ACT_RELU, VD_ACT_SIGMOID, VD_ACT_TANH = range(4)

_lock = threading.Lock()
_lib = None


class VdFeatLevel(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("H", ctypes.c_int), ("W", ctypes.c_int),
                ("spatial_scale", ctypes.c_float)]


class VdRpnLevel(ctypes.Structure):
    _fields_ = [("cls_prob", ctypes.c_void_p), ("bbox_pred", ctypes.c_void_p),
                ("anchors", ctypes.c_void_p), ("A", ctypes.c_int), ("H", ctypes.c_int),
                ("W", ctypes.c_int), ("spatial_scale", ctypes.c_float)]


# name -> (restype, argtypes)
_P, _I, _F, _S, _L = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_int64
SIGNATURES = {
    "vd_version": (_I, []),
    "vd_status_string": (ctypes.c_char_p, [_I]),
    "vd_roi_align_forward": (_I, [_I, _I, _F, _I, _P, _I, _I, _I, _I, _P, _I, _I, _P, _P]),
    "vd_roi_align_backward": (_I, [_I, _I, _F, _I, _P, _I, _I, _I, _I, _P, _I, _I, _P, _P]),
    "vd_roi_align_fpn_forward": (_I, [ctypes.POINTER(VdFeatLevel), _I, _I, _I, _I, _P, _P, _P,
                                      _I, _I, _I, _I, _I, _P, _P]),
    "vd_roi_align_fpn_tiled_workspace_size": (_S, [ctypes.POINTER(VdFeatLevel), _I, _I, _I, _I,
                                                   _I]),
    "vd_roi_align_fpn_tiled_forward": (_I, [ctypes.POINTER(VdFeatLevel), _I, _I, _I, _P, _P, _I,
                                            _I, _I, _P, _P, _S, _P]),
    "vd_gemm_workspace_size": (_S, []),
    "vd_gemm_plans_key": (_I, [_P, _I]),
    "vd_gemm_plan_list": (_I, [_P, _I]),
    "vd_gemm_bias_act": (_I, [_P, _I, _I, _P, _I, _P, _P, _I, _P, _P, _S, _P]),
    "vd_gemm_dual_bias_act": (_I, [_P, _I, _P, _I, _I, _P, _I, _P, _I, _P, _P]),
    "vd_gemm_split3_weight_size": (_S, [_I, _I]),
    "vd_mask_head_upconv_logits": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _I, _P, _P]),
    "vd_gemm_split3_weight": (_I, [_P, _I, _I, _P, _P]),
    "vd_gemm_split3_bias_act": (_I, [_P, _I, _I, _P, _I, _P, _P, _I, _P, _P, _I, _I, _I, _I,
                                    _I, _P, _I, _P]),
    "vd_fpn_lateral_weight": (_I, [_P, _I, _I, _P, _P]),
    "vd_fpn_lateral_topdown": (_I, [_P, _L, _I, _P, _I, _P, _P, _I, _I, _P, _P]),
    "vd_conv3x3_bias_act": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P]),
    "vd_conv3x3_wino_weight": (_I, [_P, _I, _I, _P, _P]),
    "vd_conv3x3_wino_bias_act": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P]),
    "vd_conv3x3_wino4_weight": (_I, [_P, _I, _I, _P, _P]),
    "vd_conv3x3_wino4_bias_act": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P]),
    "vd_conv3x3_wino4_mosaic_bias_act": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P]),
    "vd_conv3x3_wino4_rows_bias_act": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P]),
    "vd_conv3x3_wino4_grid_bias_act": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P]),
    "vd_conv3x3_wino4_dilated2_bias_act": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _I, _P, _I,
                                                _P]),
    "vd_conv3x3_wino4_grouped_bias_act": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _I, _P, _I,
                                               _P]),
    "vd_conv3x3_wino_seg_bias_act": (_I, [_P, _I, _I, _I, _P, _I, _P, _I, _I, _P, _P]),
    "vd_conv3x3_wino_mosaic_bias_act": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _I, _P, _P]),
    "vd_roi_align_legacy_forward": (_I, [_I, _I, _F, _P, _I, _I, _I, _I, _P, _I, _P, _P]),
    "vd_roi_pool_forward": (_I, [_I, _I, _F, _P, _I, _I, _I, _I, _P, _I, _P, _P, _P]),
    "vd_roi_pool_backward": (_I, [_P, _P, _L, _P, _P]),
    "vd_roi_crop_forward": (_I, [_P, _I, _I, _I, _I, _P, _I, _I, _I, _P, _P]),
    "vd_nms_workspace_size": (_S, [_I]),
    "vd_nms": (_I, [_P, _I, _I, _F, _P, _P, _P, _S, _P]),
    "vd_map_rois_to_fpn_levels": (_I, [_P, _I, _I, _I, _I, _I, _F, _F, _P, _P]),
    "vd_mask_rois": (_I, [_P, _P, _P, _I, _I, _P, _I, _I, _I, _I, _F, _F, _P, _P, _P, _P, _P]),
    "vd_generate_proposals_workspace_size": (_S, [ctypes.POINTER(VdRpnLevel), _I, _I, _I]),
    "vd_generate_proposals": (_I, [ctypes.POINTER(VdRpnLevel), _I, _I, _P, _I, _I, _F, _F, _P,
                                   _P, _P, _P, _S, _P]),
    "vd_collect_distribute": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "vd_box_detections_workspace_size": (_S, [_I, _I, _I]),
    "vd_box_detections": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _P, _F, _F, _I, _P, _I, _P, _P,
                               _P, _P, _S, _P]),
    "vd_box_detections_ex": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _P, _F, _F, _I, _P,
                                  _I, _F, _F, _I, _F, _F, _I, _P, _P, _P, _P, _S, _P]),
    "vd_stem_weight_size": (_S, []),
    "vd_stem_weight_pack": (_I, [_P, _P, _P]),
    "vd_stem_conv_pool": (_I, [_P, _I, _I, _I, _P, _P, _P, _P]),
    "vd_stem_split_weight_size": (_S, []),
    "vd_stem_split_weight_pack": (_I, [_P, _P, _P]),
    "vd_stem_split_conv_pool": (_I, [_P, _I, _I, _I, _P, _P, _P, _P]),
    "vd_soft_nms": (_I, [_P, _I, _I, _F, _F, _F, _I, _P, _P, _P, _P]),
    "vd_box_voting": (_I, [_P, _I, _I, _P, _I, _I, _F, _I, _F, _P, _P]),
    "vd_image_to_blob": (_I, [_P, _I, _I, _I, _P, _I, _I, _I, _P, _P]),
    "vd_image_resize_to_blob": (_I, [_P, _I, _I, _I, _P, ctypes.c_double, _I, _I, _I, _I, _I,
                                     _P, _P]),
    "vd_nchw_to_nhwc": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "vd_bias_act": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "vd_detections_postfilter": (_I, [_P, _P, _P, _I, _I, _F, _I, _P]),
    "vd_mask_iou_nms_workspace_size": (_S, [_I, _I, _I]),
    "vd_mask_iou_nms": (_I, [_P, _I, _I, _I, _P, _I, _P, ctypes.c_double, _I, _P, _P, _P, _S,
                             _P]),
    "vd_detections_prev_box_filter": (_I, [_P, _P, _P, _I, _I, _P, _P, _P, _I, _F, _F, _P]),
    # segm_results (paste + binarize + RLE counts)
    "vd_paste_masks": (_I, [_P, _I, _I, _P, _I, _I, _I, _F, _P, _P]),
    "vd_mask_rle": (_I, [_P, _I, _I, _I, _P, _I, _P, _P]),
    "vd_bias_relu_maxpool": (_I, [_P, _P, _I, _I, _I, _I, _P, _P]),
    "vd_rpn_head": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "vd_segm_rle": (_I, [_P, _I, _I, _P, _I, _I, _I, _F, _P, _I, _P, _P]),
    "vd_rle_strings": (_I, [_P, _P, _I, _I, _P, _P, _P]),
    # VOS temporal path
    "vd_flow_align_forward": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "vd_flow_align_backward": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P]),
    "vd_group_norm_workspace_size": (_S, [_I, _I]),
    "vd_group_norm_act": (_I, [_P, _P, _I, _I, _I, _I, _I, _F, _P, _P, _P, _I, _P, _P, _I, _I,
                               _P, _P, _S, _P]),
    "vd_convgru_gates": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _F, _P, _P, _P, _P, _I,
                              _P, _P, _P, _S, _P]),
    "vd_convgru_update": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _F, _P, _P, _I, _P, _P,
                               _S, _P]),
}


def lib():
    """Load libvosdet.so once; raise loudly if it is absent."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(
                        "vosdetectron_amd: %s is missing -- build the HIP library first "
                        "(__graft_entry__.build()); there is no CPU fallback." % LIB_PATH)
                L = ctypes.CDLL(LIB_PATH)
                for name, (res, args) in SIGNATURES.items():
                    fn = getattr(L, name)
                    fn.restype = res
                    fn.argtypes = args
                _lib = L
    return _lib


class VosdetError(RuntimeError):
    pass


def check(status: int, what: str) -> None:
    if status != VD_OK:
        msg = lib().vd_status_string(status).decode()
        raise VosdetError("%s failed: %s (status %d)" % (what, msg, status))
