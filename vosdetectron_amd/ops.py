"""Torch-facing wrappers over the C ABI (libvosdet.so).

Every function takes device tensors, launches on torch's current HIP stream and
returns device tensors; shapes and dtypes are checked here, and any kernel
status other than VD_OK raises.  PyTorch is used for allocation and streams
only -- all arithmetic happens in the HIP kernels.
"""
from __future__ import annotations

import ctypes
import os
import sys
import weakref
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import VD_ERR_SHAPE, check, lib


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _need(t: torch.Tensor, name: str, dtype=torch.float32) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError("%s must be a torch.Tensor" % name)
    if not t.is_cuda:
        raise ValueError("%s must be a device (HIP) tensor; there is no CPU path" % name)
    if t.dtype != dtype:
        raise TypeError("%s must be %s, got %s" % (name, dtype, t.dtype))
    return t.contiguous()


def _ws(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


# --------------------------------------------------------------------------- #
# RoIAlign (Caffe2)                                                            #
# --------------------------------------------------------------------------- #
def roi_align_forward(features, rois, aligned_height, aligned_width, spatial_scale,
                      sampling_ratio):
    """RoIAlignFunction.forward (roi_xfrom/roi_align/functions/roi_align.py:16-32) on
    NCHW features; returns R x C x ah x aw."""
    f = _need(features, "features")
    r = _need(rois, "rois")
    if f.dim() != 4 or r.dim() != 2:
        raise ValueError("features must be 4-D NCHW and rois 2-D")
    B, C, H, W = f.shape
    R = r.shape[0]
    out = torch.empty((R, C, aligned_height, aligned_width), dtype=torch.float32, device=f.device)
    if R == 0:
        return out
    check(lib().vd_roi_align_forward(int(aligned_height), int(aligned_width),
                                     float(spatial_scale), int(sampling_ratio), f.data_ptr(),
                                     B, C, H, W, r.data_ptr(), R, r.shape[1], out.data_ptr(),
                                     _stream()), "vd_roi_align_forward")
    return out


def roi_align_backward(top_grad, rois, feat_shape, spatial_scale, sampling_ratio):
    g = _need(top_grad, "top_grad")
    r = _need(rois, "rois")
    B, C, H, W = feat_shape
    R, _, ah, aw = g.shape
    out = torch.zeros((B, C, H, W), dtype=torch.float32, device=g.device)
    if R == 0:
        return out
    check(lib().vd_roi_align_backward(ah, aw, float(spatial_scale), int(sampling_ratio),
                                      g.data_ptr(), B, C, H, W, r.data_ptr(), R, r.shape[1],
                                      out.data_ptr(), _stream()), "vd_roi_align_backward")
    return out


class _RoIAlignAutograd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, features, rois, ah, aw, scale, sr):
        ctx.save_for_backward(rois)
        ctx.meta = (tuple(features.shape), scale, sr)
        return roi_align_forward(features, rois, ah, aw, scale, sr)

    @staticmethod
    def backward(ctx, grad_out):
        (rois,) = ctx.saved_tensors
        shape, scale, sr = ctx.meta
        g = roi_align_backward(grad_out, rois, shape, scale, sr)
        return g, None, None, None, None, None


class RoIAlignFunction:
    """Drop-in for the reference's old-style ``RoIAlignFunction(aligned_height,
    aligned_width, spatial_scale, sampling_ratio)(features, rois)``
    (lib/modeling/roi_xfrom/roi_align/functions/roi_align.py:7-48).  The
    reference raises NotImplementedError for CPU tensors (:29-30); so does this
    one (there is no CPU path)."""

    def __init__(self, aligned_height, aligned_width, spatial_scale, sampling_ratio):
        self.aligned_width = int(aligned_width)
        self.aligned_height = int(aligned_height)
        self.spatial_scale = float(spatial_scale)
        self.sampling_ratio = int(sampling_ratio)

    def __call__(self, features, rois):
        if not features.is_cuda:
            raise NotImplementedError("RoIAlign has no CPU implementation")
        return _RoIAlignAutograd.apply(features, rois, self.aligned_height, self.aligned_width,
                                       self.spatial_scale, self.sampling_ratio)

    forward = __call__


class RoIAlign(torch.nn.Module):
    """modules/roi_align.py:6-17 counterpart."""

    def __init__(self, aligned_height, aligned_width, spatial_scale, sampling_ratio):
        super().__init__()
        self.fn = RoIAlignFunction(aligned_height, aligned_width, spatial_scale, sampling_ratio)

    def forward(self, features, rois):
        return self.fn(features, rois)


def roi_align_fpn(levels: Sequence[torch.Tensor], spatial_scales: Sequence[float],
                  rois: torch.Tensor, roi_level: Optional[torch.Tensor], resolution: int,
                  sampling_ratio: int, layout: str = "nhwc",
                  roi_order: Optional[torch.Tensor] = None,
                  out: Optional[torch.Tensor] = None, out_layout: str = "nchw") -> torch.Tensor:
    """One-launch multi-level RoIAlign (replaces the per-level loop + cat + restore
    of model_builder.py:252-303).  levels: finest first, each B x H x W x C
    (layout 'nhwc') or B x C x H x W ('nchw', single level only).  roi_level[r]
    is the index into ``levels``.  Output row r belongs to rois[r]; out_layout
    'nchw' -> R x C x P x P (the reference's), 'nhwc' -> R x P x P x C."""
    if len(levels) < 1 or len(levels) > _lib.VD_MAX_LEVELS:
        raise ValueError("1..%d levels" % _lib.VD_MAX_LEVELS)
    r = _need(rois, "rois")
    nhwc = layout == "nhwc"
    if r.dim() != 2 or r.shape[1] != 5:
        raise ValueError("rois must be R x 5, got %s" % (tuple(r.shape),))
    descs = (_lib.VdFeatLevel * len(levels))()
    keep = []
    BC = None
    for i, (t, sc) in enumerate(zip(levels, spatial_scales)):
        t = _need(t, "levels[%d]" % i)
        if t.dim() != 4:
            raise ValueError("levels[%d] must be 4-D" % i)
        keep.append(t)
        if nhwc:
            B, H, W, C = t.shape
        else:
            B, C, H, W = t.shape
        if BC is not None and (B, C) != BC:
            raise ValueError("levels[%d] has B, C = %s; levels[0] has %s" % (i, (B, C), BC))
        BC = (B, C)
        descs[i] = _lib.VdFeatLevel(t.data_ptr(), H, W, float(sc))
    R = r.shape[0]
    onhwc = out_layout == "nhwc"
    shape = (R, resolution, resolution, C) if onhwc else (R, C, resolution, resolution)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=r.device)
    elif (tuple(out.shape) != shape or out.dtype != torch.float32 or not out.is_contiguous()
          or out.device != r.device):
        raise ValueError("out must be a contiguous float32 %s tensor on %s, got %s %s"
                         % (shape, r.device, tuple(out.shape), out.dtype))
    if R == 0:
        return out
    if roi_level is not None and tuple(roi_level.shape) != (R,):
        raise ValueError("roi_level must have R = %d entries" % R)
    if roi_order is not None and tuple(roi_order.shape) != (R,):
        raise ValueError("roi_order must have R = %d entries" % R)
    lv = _need(roi_level, "roi_level", torch.int32) if roi_level is not None else None
    od = _need(roi_order, "roi_order", torch.int32) if roi_order is not None else None
    if nhwc and onhwc and int(sampling_ratio) == 2 and roi_align_variant() == "30" \
            and (len(levels) == 1 or lv is not None):
        # tile-binned LDS-staged kernel (csrc/roi_align_tile.hip): bit-identical to the
        # reference's per-sample arithmetic; roi_order does not apply (tiles set the order)
        L = len(levels)
        nws = lib().vd_roi_align_fpn_tiled_workspace_size(descs, L, B, C, R, resolution)
        if nws:
            ws = torch.empty((nws,), dtype=torch.uint8, device=r.device)
            st = lib().vd_roi_align_fpn_tiled_forward(
                descs, L, B, C, r.data_ptr(), lv.data_ptr() if lv is not None else None, R,
                resolution, 2, out.data_ptr(), ws.data_ptr(), nws, _stream())
            if st != _lib.VD_ERR_SHAPE:
                check(st, "vd_roi_align_fpn_tiled_forward")
                return out
    check(lib().vd_roi_align_fpn_forward(
        descs, len(levels), B, C, _lib.VD_LAYOUT_NHWC if nhwc else _lib.VD_LAYOUT_NCHW,
        r.data_ptr(), lv.data_ptr() if lv is not None else None,
        od.data_ptr() if od is not None else None, R, resolution, resolution,
        int(sampling_ratio), _lib.VD_LAYOUT_NHWC if onhwc else _lib.VD_LAYOUT_NCHW,
        out.data_ptr(), _stream()), "vd_roi_align_fpn_forward")
    return out


_ORDER_CACHE = {}

# FPN RoIAlign kernel for NHWC in/out (VOSDET_ROIALIGN_VARIANT overrides):
# "30" tile-binned LDS-staged (roi_align_tile.hip), "10" register-gather separable
# (roi_align.hip), "3" reference-order rows.
ROI_ALIGN_DEFAULT_VARIANT = "10"


def roi_align_variant() -> str:
    return os.environ.get("VOSDET_ROIALIGN_VARIANT", ROI_ALIGN_DEFAULT_VARIANT)


def _spread16(v: torch.Tensor) -> torch.Tensor:
    """Bits 0..15 of v to the even bit positions 0..30."""
    v = (v | (v << 8)) & 0x00FF00FF
    v = (v | (v << 4)) & 0x0F0F0F0F
    v = (v | (v << 2)) & 0x33333333
    return (v | (v << 1)) & 0x55555555


def _morton16(y: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """Z-order index of 16-bit (y, x): x on the even bits, y on the odd bits."""
    return _spread16(x) | (_spread16(y) << 1)


def _deal(n: int, n_xcd: int, window: Optional[int]) -> np.ndarray:
    """Block b -> position in the sorted order: inside each window of `window`
    consecutive positions (the whole order by default), XCD k (b % n_xcd == k)
    takes the k-th contiguous slice."""
    p = np.empty(n, np.int64)
    w = n if not window else int(window)
    for start in range(0, n, w):
        m = min(w, n - start)
        per = -(-m // n_xcd)
        b = np.arange(m)
        slot = (b % n_xcd) * per + b // n_xcd
        ok = slot < m
        q = np.empty(m, np.int64)
        q[ok] = slot[ok]
        q[~ok] = np.setdiff1d(np.arange(m), slot[ok])
        p[start:start + m] = q + start
    return p


def xcd_roi_order(rois: torch.Tensor, roi_level: torch.Tensor, n_xcd: Optional[int] = None,
                  band: int = 8, window: Optional[int] = None,
                  curve: Optional[str] = None) -> torch.Tensor:
    """Scheduling permutation for roi_align_fpn (never changes results): RoIs
    sorted by (image, level, position) and dealt so that the blocks of one XCD
    (b % 8 equal) walk one contiguous slice of that order -- spatial
    neighbours, whose footprints overlap, run on the same L2.  `curve` orders
    the positions: 'band' (y-band of `band` level pixels, then x) or 'morton'
    (Z-order of the level-pixel centre: consecutive RoIs stay inside a square,
    so the RoIs resident on an XCD at one time share more of their footprint;
    tools/research/ra_l2_sim.py models the L2 misses of both).  The default is
    VOSDET_RA_CURVE or 'morton'.  With `window` the dealing restarts every
    `window` positions (e.g. one frame's RoIs), so all XCDs work on the same
    frame at a time; n_xcd=1 is the plain spatial sort."""
    curve = curve or os.environ.get("VOSDET_RA_CURVE", "morton")
    n_xcd = 8 if n_xcd is None else n_xcd
    r = rois
    lv = roi_level.to(torch.int64)
    scale = torch.pow(2.0, -(lv + 2).to(torch.float32))
    cy = (r[:, 2] + r[:, 4]) * 0.5 * scale
    cx = (r[:, 1] + r[:, 3]) * 0.5 * scale
    head = r[:, 0].to(torch.int64) * 8 + lv
    if curve == "band":
        key = (head * 4096 + (cy / band).to(torch.int64)) * 65536 \
            + cx.clamp(0, 65535).to(torch.int64)
    elif curve == "morton":
        key = head * (1 << 32) + _morton16(cy.clamp(0, 65535).to(torch.int64),
                                           cx.clamp(0, 65535).to(torch.int64))
    else:
        raise ValueError("curve must be 'band' or 'morton', got %r" % (curve,))
    srt = torch.argsort(key)
    n = r.shape[0]
    if n_xcd <= 1:
        return srt.to(torch.int32).contiguous()
    perm = _ORDER_CACHE.get((n, n_xcd, window, r.device))
    if perm is None:
        perm = torch.from_numpy(_deal(n, n_xcd, window)).to(r.device)
        _ORDER_CACHE[(n, n_xcd, window, r.device)] = perm
    return srt[perm].to(torch.int32).contiguous()


# --------------------------------------------------------------------------- #
# lib/model ops: legacy RoIAlign, RoIPool, RoICrop                             #
# --------------------------------------------------------------------------- #
def roi_align_legacy(features, rois, aligned_height, aligned_width, spatial_scale):
    """jwyang RoIAlignFunction (lib/model/roi_align/functions/roi_align.py)."""
    f = _need(features, "features")
    r = _need(rois, "rois")
    B, C, H, W = f.shape
    R = r.shape[0]
    out = torch.zeros((R, C, aligned_height, aligned_width), dtype=torch.float32, device=f.device)
    if R:
        check(lib().vd_roi_align_legacy_forward(aligned_height, aligned_width,
                                                float(spatial_scale), f.data_ptr(), B, C, H, W,
                                                r.data_ptr(), R, out.data_ptr(), _stream()),
              "vd_roi_align_legacy_forward")
    return out


class _RoIPoolAutograd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, features, rois, ph, pw, scale):
        f = _need(features, "features")
        r = _need(rois, "rois")
        B, C, H, W = f.shape
        R = r.shape[0]
        out = torch.zeros((R, C, ph, pw), dtype=torch.float32, device=f.device)
        arg = torch.full((R, C, ph, pw), -1, dtype=torch.int32, device=f.device)
        if R:
            check(lib().vd_roi_pool_forward(ph, pw, float(scale), f.data_ptr(), B, C, H, W,
                                            r.data_ptr(), R, out.data_ptr(), arg.data_ptr(),
                                            _stream()), "vd_roi_pool_forward")
        ctx.save_for_backward(arg)
        ctx.shape = (B, C, H, W)
        return out, arg

    @staticmethod
    def backward(ctx, grad_out, _grad_arg):
        (arg,) = ctx.saved_tensors
        g = _need(grad_out, "grad_out")
        bottom = torch.zeros(ctx.shape, dtype=torch.float32, device=g.device)
        check(lib().vd_roi_pool_backward(g.data_ptr(), arg.data_ptr(), g.numel(),
                                         bottom.data_ptr(), _stream()), "vd_roi_pool_backward")
        return bottom, None, None, None, None


class RoIPoolFunction:
    """``RoIPoolFunction(pooled_height, pooled_width, spatial_scale)(features, rois)``
    (lib/model/roi_pooling/functions/roi_pool.py:6-38), CUDA-kernel semantics."""

    def __init__(self, pooled_height, pooled_width, spatial_scale):
        self.pooled_height = int(pooled_height)
        self.pooled_width = int(pooled_width)
        self.spatial_scale = float(spatial_scale)
        self.argmax = None

    def __call__(self, features, rois):
        out, self.argmax = _RoIPoolAutograd.apply(features, rois, self.pooled_height,
                                                  self.pooled_width, self.spatial_scale)
        return out


class RoICropFunction:
    """``RoICropFunction()(input_BCHW, grid_yx)`` (lib/model/roi_crop/functions/roi_crop.py:7-15)."""

    def __call__(self, input1, input2):
        f = _need(input1, "input")
        g = _need(input2, "grid")
        B, C, H, W = f.shape
        R, GH, GW, two = g.shape
        if two != 2:
            raise ValueError("grid must be R x GH x GW x 2 (y, x)")
        out = torch.zeros((R, C, GH, GW), dtype=torch.float32, device=f.device)
        if R:
            check(lib().vd_roi_crop_forward(f.data_ptr(), B, C, H, W, g.data_ptr(), R, GH, GW,
                                            out.data_ptr(), _stream()), "vd_roi_crop_forward")
        return out


# --------------------------------------------------------------------------- #
# NMS / levels                                                                 #
# --------------------------------------------------------------------------- #
def nms(dets: torch.Tensor, thresh: float) -> torch.Tensor:
    """cython_nms.nms semantics on device: dets N x (>=5) fp32 -> kept indices
    (int64, ascending)."""
    d = _need(dets, "dets")
    n = d.shape[0]
    keep = torch.empty((max(n, 1),), dtype=torch.int64, device=d.device)
    num = torch.zeros((1,), dtype=torch.int32, device=d.device)
    wsb = lib().vd_nms_workspace_size(n)
    ws = _ws(wsb, d.device)
    check(lib().vd_nms(d.data_ptr() if n else None, n, d.shape[1] if d.dim() == 2 else 5,
                       float(np.float32(thresh)), keep.data_ptr(), num.data_ptr(),
                       ws.data_ptr(), ws.numel(), _stream()), "vd_nms")
    return keep[: int(num.item())]


def soft_nms(dets: torch.Tensor, sigma: float = 0.5, overlap_thresh: float = 0.3,
             score_thresh: float = 0.001, method: str = "linear"):
    """utils.boxes.soft_nms on the device (vd_soft_nms): dets N x (>=5) fp32 ->
    (rows [N',5] with decayed scores in the reference's order, keep int64 [N'])."""
    d = _need(dets, "dets")
    n = d.shape[0]
    if method not in SOFT_NMS_METHODS:
        raise ValueError("Unknown soft_nms method: {}".format(method))  # boxes.py:344
    out = torch.empty((max(n, 1), 5), dtype=torch.float32, device=d.device)
    keep = torch.empty((max(n, 1),), dtype=torch.int64, device=d.device)
    num = torch.zeros((1,), dtype=torch.int32, device=d.device)
    check(lib().vd_soft_nms(d.data_ptr() if n else None, n, d.shape[1] if d.dim() == 2 else 5,
                            float(np.float32(sigma)), float(np.float32(overlap_thresh)),
                            float(np.float32(score_thresh)), SOFT_NMS_METHODS[method],
                            out.data_ptr(), keep.data_ptr(), num.data_ptr(), _stream()),
          "vd_soft_nms")
    k = int(num.item())
    return out[:k], keep[:k]


def box_voting(top_dets: torch.Tensor, all_dets: torch.Tensor, thresh: float,
               scoring_method: str = "ID", beta: float = 1.0) -> torch.Tensor:
    """utils.boxes.box_voting on the device (vd_box_voting): top [n,>=5], all
    [m,>=5] fp32 -> [n,5]."""
    t, a = _need(top_dets, "top_dets"), _need(all_dets, "all_dets")
    out = torch.empty((t.shape[0], 5), dtype=torch.float32, device=t.device)
    if t.shape[0]:
        check(lib().vd_box_voting(t.data_ptr(), t.shape[0], t.shape[1], a.data_ptr(),
                                  a.shape[0], a.shape[1], float(np.float32(thresh)),
                                  bbox_vote_method(scoring_method, beta), float(beta),
                                  out.data_ptr(), _stream()), "vd_box_voting")
    return out


def map_rois_to_fpn_levels(rois: torch.Tensor, k_min: int, k_max: int, col0: int = 1,
                           canonical_scale: float = 224., canonical_level: float = 4.):
    """utils/fpn.py:11-28 on device; returns int32 levels (k_min..k_max)."""
    r = _need(rois, "rois")
    R = r.shape[0]
    out = torch.empty((R,), dtype=torch.int32, device=r.device)
    if R:
        check(lib().vd_map_rois_to_fpn_levels(r.data_ptr(), r.shape[1], col0, R, k_min, k_max,
                                              float(canonical_scale), float(canonical_level),
                                              out.data_ptr(), _stream()),
              "vd_map_rois_to_fpn_levels")
    return out


def mask_rois(dets: torch.Tensor, classes: torch.Tensor, counts: torch.Tensor,
              im_scale: torch.Tensor, rows: int, k_min: int, k_max: int, row0: int = 0,
              canonical_scale: float = 224., canonical_level: float = 4.):
    """The mask-head batch of all frames without a host read (vd_mask_rois):
    dets [F, D, 5], classes [F, D] int32, counts [F] int32, im_scale [F] float64
    -> rois [rows, 5], levels [rows] (level - k_min), classes [rows] int32 and the
    device total [1] int32; global rows [row0, row0 + rows), frame-major, padding
    past the total."""
    d, c, n = _need(dets, "dets"), _need(classes, "classes", torch.int32), \
        _need(counts, "counts", torch.int32)
    sc = _need(im_scale, "im_scale", torch.float64)
    F, D = d.shape[0], d.shape[1]
    if tuple(c.shape) != (F, D) or n.numel() != F or sc.numel() != F:
        raise ValueError("mask_rois: dets %s classes %s counts %s im_scale %s"
                         % (tuple(d.shape), tuple(c.shape), tuple(n.shape), tuple(sc.shape)))
    rois = torch.empty((rows, 5), dtype=torch.float32, device=d.device)
    lvl = torch.empty((rows,), dtype=torch.int32, device=d.device)
    cls = torch.empty((rows,), dtype=torch.int32, device=d.device)
    total = torch.empty((1,), dtype=torch.int32, device=d.device)
    check(lib().vd_mask_rois(d.data_ptr(), c.data_ptr(), n.data_ptr(), F, D, sc.data_ptr(),
                             int(row0), int(rows), k_min, k_max, float(canonical_scale),
                             float(canonical_level), rois.data_ptr(), lvl.data_ptr(),
                             cls.data_ptr(), total.data_ptr(), _stream()), "vd_mask_rois")
    return rois, lvl, cls, total


def nchw_to_nhwc(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    t = _need(x, "x")
    B, C, H, W = t.shape
    if out is None:
        out = torch.empty((B, H, W, C), dtype=torch.float32, device=t.device)
    check(lib().vd_nchw_to_nhwc(t.data_ptr(), B, C, H, W, out.data_ptr(), _stream()),
          "vd_nchw_to_nhwc")
    return out


def bias_act_(x: torch.Tensor, bias: Optional[torch.Tensor], residual=None, residual_bias=None,
              relu: bool = True, upsample_residual: bool = False) -> torch.Tensor:
    """In-place conv epilogue x = act((x + bias) + residual[+residual_bias]) (vd_bias_act).
    x: N x C x H x W, contiguous or channels_last; residual in the same memory format."""
    N, C, H, W = x.shape
    if x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous():
        nhwc = 1
    elif x.is_contiguous():
        nhwc = 0
    else:
        raise ValueError("x must be contiguous (NCHW or channels_last)")
    if not x.is_cuda or x.dtype != torch.float32:
        raise ValueError("x must be a float32 device tensor")
    for v in (bias, residual_bias):
        if v is not None and (v.numel() != C or not v.is_contiguous() or v.dtype != torch.float32):
            raise ValueError("bias vectors must be contiguous float32 of length C")
    mode = 0
    if residual is not None:
        mode = 2 if upsample_residual else 1
        want_shape = (N, C, H // 2, W // 2) if upsample_residual else (N, C, H, W)
        if tuple(residual.shape) != want_shape or residual.dtype != torch.float32:
            raise ValueError("residual shape %s, expected %s" % (tuple(residual.shape),
                                                                 want_shape))
        want = torch.channels_last if nhwc else torch.contiguous_format
        if not residual.is_contiguous(memory_format=want):
            residual = residual.contiguous(memory_format=want)
    check(lib().vd_bias_act(x.data_ptr(), bias.data_ptr() if bias is not None else None,
                            residual.data_ptr() if residual is not None else None,
                            residual_bias.data_ptr() if residual_bias is not None else None,
                            N, C, H, W, nhwc, mode, int(relu), _stream()), "vd_bias_act")
    return x


_GEMM_WS = {}


def gemm_workspace(device) -> torch.Tensor:
    """The hipBLASLt workspace for one vd_gemm_bias_act launch.  Algorithms with
    a workspace keep inter-workgroup state in it (split-K partials, stream-K
    fix-up flags; vd_gemm_plan_list shows which plans use one), so two GEMMs
    that can run at the same time must not share it.  A captured step bakes the
    pointer into its graph: the two captured steps of bench.capture_graphs,
    replayed concurrently on two streams, shared the one per-device workspace of
    round 4 and stopped making progress.  So:
      * while the current stream is capturing, every call takes its workspace
        from the graph's private memory pool (freed after the call, the caching
        allocator hands the same block to the next GEMM of the same capture:
        one workspace per graph, stream-ordered inside it);
      * eager launches use one workspace per (device, stream)."""
    device = torch.device(device)
    if torch.cuda.is_current_stream_capturing():
        return _ws(lib().vd_gemm_workspace_size(), device)
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    ws = _GEMM_WS.get(key)
    if ws is None:
        ws = _GEMM_WS[key] = _ws(lib().vd_gemm_workspace_size(), device)
    return ws


def gemm_plan_list() -> list:
    """(M, N, K, relu, has_res, 'own' | 'blas', workspace_bytes) for every GEMM
    shape this process has planned (vd_gemm_plan_list)."""
    n = 1 << 16
    while True:
        buf = ctypes.create_string_buffer(n)
        st = lib().vd_gemm_plan_list(buf, n)
        if st != _lib.VD_ERR_WORKSPACE:
            break
        n *= 4
    check(st, "vd_gemm_plan_list")
    rows = []
    for line in buf.value.decode().splitlines():
        M, N, K, relu, res, what, ws = line.split()
        rows.append((int(M), int(N), int(K), int(relu), int(res), what, int(ws)))
    return rows


# K from which a GEMM with a split-bf16 route runs it there (gemm_split3_bias_act):
# below it the GEMMs are HBM-bound and the fp32 kernels are as fast
# (profiles/r06/gemm_split3/)
SPLIT3_MIN_K = 128
# id(weight tensor) -> (weakref to it, key, split image); an entry leaves with its tensor
_split3_cache = {}


def split3_enabled() -> bool:
    """VOSDET_GEMM_SPLIT3=0 keeps every GEMM on the fp32-MFMA kernels (A/B runs)."""
    return os.environ.get("VOSDET_GEMM_SPLIT3", "1") != "0"


def split3_weight_cached(w: torch.Tensor) -> Optional[torch.Tensor]:
    """gemm_split3_weight(w), made once per weight tensor and remade when the tensor
    changes (its storage or version counter: an in-place update, load_state_dict)."""
    key = (w.data_ptr(), w._version, tuple(w.shape))
    i = id(w)
    ent = _split3_cache.get(i)
    if ent is not None and ent[0]() is w and ent[1] == key:
        return ent[2]
    def _drop(r, i=i):
        if _split3_cache.get(i, (None,))[0] is r:
            del _split3_cache[i]
    ref = weakref.ref(w, _drop)
    if os.environ.get("VOSDET_SPLIT3_TRACE") == "1":  # research: report every (re)split
        import traceback
        sys.stderr.write("split3 weight %s (cache %s)\n%s" % (
            tuple(w.shape), "stale" if ent is not None else "miss",
            "".join(traceback.format_stack(limit=6)[:-1])))
    wp = gemm_split3_weight(w)
    _split3_cache[i] = (ref, key, wp)
    return wp


def gemm_bias_act(a: torch.Tensor, w: torch.Tensor, bias: torch.Tensor,
                  residual: Optional[torch.Tensor] = None, relu: bool = True,
                  out: Optional[torch.Tensor] = None,
                  a_bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """act(a @ w.T + bias (+ residual)) in one GEMM launch: a [M,K], w [N,K], bias [N],
    residual / out [M,N], all fp32 contiguous.  From K = SPLIT3_MIN_K (N a multiple
    of 64) on the bf16 matrix cores at fp32 accuracy (gemm_split3_bias_act, the
    weight's split image cached per tensor); otherwise vd_gemm_bias_act (hipBLASLt
    with the epilogue fused, or the hand-written fp32 MFMA kernel where it is
    faster).  a_bias [K]: a enters as relu(a + a_bias) (fused into the split GEMM's A
    load; a separate pass before the other kernels).  Returns None when nothing serves
    the shape (the caller falls back, a_bias not applied)."""
    a_ = _need(a, "a")
    w_ = _need(w, "w")
    b_ = _need(bias, "bias")
    M, K = a_.shape
    N = w_.shape[0]
    if w_.shape[1] != K or b_.numel() != N:
        raise ValueError("gemm_bias_act: a %s, w %s, bias %s" % (tuple(a_.shape), tuple(w_.shape),
                                                                 tuple(b_.shape)))
    r_ = None
    if residual is not None:
        r_ = _need(residual, "residual")
        if tuple(r_.shape) != (M, N):
            raise ValueError("residual must be %s, got %s" % ((M, N), tuple(r_.shape)))
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a_.device)
    elif tuple(out.shape) != (M, N) or not out.is_contiguous():
        raise ValueError("out must be a contiguous %s tensor" % ((M, N),))
    if K >= SPLIT3_MIN_K and N % 64 == 0 and K % 16 == 0 and M > 0 and split3_enabled():
        wp = split3_weight_cached(w if w.is_contiguous() else w_)
        if wp is not None:
            return gemm_split3_bias_act(a_, wp, b_, residual=r_, relu=relu, out=out,
                                        a_bias=a_bias)
    if a_bias is not None:
        a_ = torch.relu(a_ + _need(a_bias, "a_bias"))
    if os.environ.get("VOSDET_GEMM_TRACE") == "1":  # research: the fp32-kernel GEMMs
        sys.stderr.write("fp32 gemm M=%d N=%d K=%d res=%d\n" % (M, N, K, r_ is not None))
    ws = gemm_workspace(a_.device)
    st = lib().vd_gemm_bias_act(a_.data_ptr(), M, K, w_.data_ptr(), N, b_.data_ptr(),
                                r_.data_ptr() if r_ is not None else None, int(relu),
                                out.data_ptr(), ws.data_ptr(), ws.numel(), _stream())
    if st == VD_ERR_SHAPE:  # no hipBLASLt algorithm and no MFMA kernel for the shape
        return None
    check(st, "vd_gemm_bias_act")
    return out


def gemm_split3_weight(w: torch.Tensor) -> Optional[torch.Tensor]:
    """W [N, K] fp32 (a 1x1 conv / Linear weight) -> the three-piece bf16 split image
    vd_gemm_split3_bias_act reads (once per model; N * K * 6 bytes).  None when the
    shape is not served (K a multiple of 32, N of 64)."""
    w_ = _need(w.reshape(w.shape[0], -1), "w")
    N, K = w_.shape
    nbytes = lib().vd_gemm_split3_weight_size(N, K)
    if not nbytes:
        return None
    wp = torch.empty(nbytes, dtype=torch.uint8, device=w_.device)
    check(lib().vd_gemm_split3_weight(w_.data_ptr(), N, K, wp.data_ptr(), _stream()),
          "vd_gemm_split3_weight")
    wp.split3_shape = (N, K)
    return wp


def gemm_split3_bias_act(a: torch.Tensor, wp: torch.Tensor, bias: torch.Tensor,
                         residual: Optional[torch.Tensor] = None, relu: bool = True,
                         out: Optional[torch.Tensor] = None, cfg: int = 0,
                         up_hw: Optional[Sequence[int]] = None,
                         sub_hw: Optional[Sequence[int]] = None,
                         a2: Optional[torch.Tensor] = None,
                         a_bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """act(a @ w.T + bias (+ residual)) with the fp32 operands split into three bf16
    pieces on the bf16 matrix cores (vd_gemm_split3_bias_act, fp32 accuracy):
    a [M,K], wp from gemm_split3_weight(w [N,K]), bias [N], out [M,N]; residual
    [M,N], or with up_hw = (H, W) the top-down map [M / (H W), H/2, W/2, N] of an
    FPN level added at the nearest-2x row of each pixel (FPN.py:292-300).  With
    sub_hw = (H, W): a is an images x H x W map's rows [images H W, K] read at
    stride 2, M = images x ceil(H/2) x ceil(W/2) output rows (a stride-2 1x1 conv).
    With a2 [M, K2]: w's last K2 input channels multiply a2 (a is [M, K - K2]): two
    1x1 convs of two inputs summed in one GEMM.  With a_bias [K - K2]: a enters as
    relu(a + a_bias) (the producing layer's bias + ReLU, fused into the A load)."""
    a_ = _need(a, "a")
    N, K = wp.split3_shape
    M = a_.shape[0]
    K2, a2_ = 0, None
    if a2 is not None:
        a2_ = _need(a2, "a2")
        K2 = a2_.shape[1]
        if a2_.shape[0] != M or a_.shape[1] + K2 != K or K2 % 16 or sub_hw is not None:
            raise ValueError("gemm_split3_bias_act: a %s + a2 %s vs w (%d, %d)"
                             % (tuple(a_.shape), tuple(a2_.shape), N, K))
    sh = sw = 0
    if sub_hw is not None:
        sh, sw = int(sub_hw[0]), int(sub_hw[1])
        if sh < 1 or sw < 1 or M % (sh * sw):
            raise ValueError("a %s is not a stack of %s maps" % (tuple(a_.shape), (sh, sw)))
        M = M // (sh * sw) * ((sh + 1) // 2) * ((sw + 1) // 2)
    b_ = _need(bias, "bias")
    if a_.dim() != 2 or a_.shape[1] + K2 != K or b_.numel() != N:
        raise ValueError("gemm_split3_bias_act: a %s, w (%d, %d), bias %s"
                         % (tuple(a_.shape), N, K, tuple(b_.shape)))
    ab_ = None
    if a_bias is not None:
        ab_ = _need(a_bias, "a_bias")
        if ab_.numel() != K - K2:
            raise ValueError("a_bias must have %d entries, got %d" % (K - K2, ab_.numel()))
    r_ = None
    uh = uw = 0
    if residual is not None:
        r_ = _need(residual, "residual")
        if up_hw is not None:
            uh, uw = int(up_hw[0]), int(up_hw[1])
            if uh % 2 or uw % 2 or uh < 2 or uw < 2 or M % (uh * uw) or \
                    r_.numel() != (M // 4) * N:
                raise ValueError("top-down map %s does not match %d pixels of %s maps"
                                 % (tuple(r_.shape), M, (uh, uw)))
        elif tuple(r_.shape) != (M, N):
            raise ValueError("residual must be %s, got %s" % ((M, N), tuple(r_.shape)))
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a_.device)
    elif tuple(out.shape) != (M, N) or not out.is_contiguous():
        raise ValueError("out must be a contiguous %s tensor" % ((M, N),))
    check(lib().vd_gemm_split3_bias_act(a_.data_ptr(), M, K,
                                        a2_.data_ptr() if a2_ is not None else None, K2,
                                        ab_.data_ptr() if ab_ is not None else None,
                                        wp.data_ptr(), N, b_.data_ptr(),
                                        r_.data_ptr() if r_ is not None else None, uh, uw,
                                        sh, sw, int(relu), out.data_ptr(), int(cfg), _stream()),
          "vd_gemm_split3_bias_act")
    return out


def mask_head_upconv_logits(x: torch.Tensor, wp: torch.Tensor, bias: torch.Tensor,
                            cls_w: torch.Tensor, cls_b: torch.Tensor, roi_ch: torch.Tensor,
                            P: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The mask head's upconv5 + ReLU and the class-selected mask logits + sigmoid in one
    split-bf16 launch (vd_mask_head_upconv_logits): x [R P P, 256] NHWC RoI map rows,
    wp = gemm_split3_weight of the upconv weight as [(i, j, co), 256], bias [1024],
    cls_w [classes, 256], cls_b [classes], roi_ch [R] (int32 class channels).  Returns
    [R, 2P, 2P] mask probabilities."""
    x_ = _need(x, "x")
    R = int(roi_ch.numel())
    if x_.dim() != 2 or x_.shape[0] != R * P * P or tuple(wp.split3_shape) != (1024, x_.shape[1]):
        raise ValueError("mask_head_upconv_logits: x %s, %d RoIs of %d x %d, w %s"
                         % (tuple(x_.shape), R, P, P, wp.split3_shape))
    cw = _need(cls_w, "cls_w")
    if cw.dim() != 2 or cw.shape[1] != 256:
        raise ValueError("cls_w must be [classes, 256], got %s" % (tuple(cw.shape),))
    ch = _need(roi_ch, "roi_ch", torch.int32)
    if out is None:
        out = torch.empty((R, 2 * P, 2 * P), dtype=torch.float32, device=x_.device)
    check(lib().vd_mask_head_upconv_logits(x_.data_ptr(), x_.shape[0], x_.shape[1], wp.data_ptr(),
                                           _need(bias, "bias").data_ptr(), cw.data_ptr(),
                                           _need(cls_b, "cls_b").data_ptr(), ch.data_ptr(), P,
                                           out.data_ptr(), _stream()),
          "vd_mask_head_upconv_logits")
    return out


def conv3x3_weight(w: torch.Tensor) -> torch.Tensor:
    """PyTorch conv weight [Cout][Cin][3][3] -> the [Cout][3][3][Cin] layout
    vd_conv3x3_bias_act reads (once per model, at prepare time)."""
    return w.permute(0, 2, 3, 1).contiguous()


def conv3x3_bias_act(x: torch.Tensor, w2: torch.Tensor, bias: Optional[torch.Tensor],
                     relu: bool = False, out: Optional[torch.Tensor] = None):
    """act(conv3x3(x, pad 1) + bias) on a channels_last fp32 tensor in one MFMA
    implicit-GEMM kernel (vd_conv3x3_bias_act); w2 from conv3x3_weight.  Returns
    None for a shape the kernel does not serve (the caller falls back)."""
    if x.dim() != 4 or not x.is_cuda or x.dtype != torch.float32 or \
            not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv3x3_bias_act: x must be a channels_last fp32 CUDA tensor")
    N, C, H, W = x.shape
    w_ = _need(w2, "w2")
    Cout = w_.shape[0]
    if tuple(w_.shape) != (Cout, 3, 3, C):
        raise ValueError("w2 must be [Cout][3][3][Cin], got %s" % (tuple(w_.shape),))
    b_ = _need(bias, "bias") if bias is not None else None
    if b_ is not None and b_.numel() != Cout:
        raise ValueError("bias must have %d elements" % Cout)
    if out is None:
        out = torch.empty((N, Cout, H, W), dtype=torch.float32, device=x.device,
                          memory_format=torch.channels_last)
    elif tuple(out.shape) != (N, Cout, H, W) or \
            not out.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("out must be a channels_last %s tensor" % ((N, Cout, H, W),))
    st = lib().vd_conv3x3_bias_act(x.data_ptr(), N, H, W, C, w_.data_ptr(), Cout,
                                   b_.data_ptr() if b_ is not None else None, int(relu),
                                   out.data_ptr(), _stream())
    if st == VD_ERR_SHAPE:
        return None
    check(st, "vd_conv3x3_bias_act")
    return out


WINO_MAX_CIN = 4096  # csrc/conv3x3_wino.hip: the zero lanes' DMA source holds 4096 floats


def conv3x3_wino_weight(w: torch.Tensor) -> Optional[torch.Tensor]:
    """PyTorch conv weight [Cout][Cin][3][3] -> the Winograd F(2x2,3x3) operand
    U = G g G^T in the kernel's register-fragment order [Cout/64][Cin/8][2][16][64][4]
    (32-channel group, fragment, lane, 2 positions x 2 channels;
    vd_conv3x3_wino_weight; once per model).  None for
    a shape the kernel does not serve (Cout % 64, Cin % 8, Cin > WINO_MAX_CIN)."""
    w_ = _need(w, "w")
    if w_.dim() != 4 or tuple(w_.shape[2:]) != (3, 3):
        raise ValueError("conv3x3_wino_weight: weight %s" % (tuple(w_.shape),))
    Cout, C = w_.shape[:2]
    if Cout % 64 or C % 8 or Cout == 0 or C == 0 or C > WINO_MAX_CIN:
        return None
    u = torch.empty((Cout // 64, C // 8, 2, 16, 64, 4), dtype=torch.float32, device=w_.device)
    check(lib().vd_conv3x3_wino_weight(w_.data_ptr(), Cout, C, u.data_ptr(), _stream()),
          "vd_conv3x3_wino_weight")
    return u


def conv3x3_wino_bias_act(x: torch.Tensor, u: torch.Tensor, bias: Optional[torch.Tensor],
                          relu: bool = False, out: Optional[torch.Tensor] = None,
                          mosaic: bool = False):
    """act(conv3x3(x, pad 1) + bias) on a channels_last fp32 tensor by Winograd
    F(2x2,3x3) on the MFMA pipes (vd_conv3x3_wino_bias_act); u from
    conv3x3_wino_weight.  mosaic=True runs the N images as one N*H-row image with
    per-image zero padding (vd_conv3x3_wino_seg_bias_act; H even): bit-identical,
    fewer idle block rows on small maps.  mosaic="2d" also packs maps side by side
    (vd_conv3x3_wino_mosaic_bias_act; an odd side padded by a phantom row / column
    per map): no idle block columns either.
    Returns None for a shape the kernel does not serve."""
    if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 4 \
            or not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("x must be a channels_last fp32 device tensor")
    if u is None:
        return None
    u_ = _need(u, "u")
    N, C, H, W = x.shape
    if u_.dim() != 6 or tuple(u_.shape[1:]) != (C // 8, 2, 16, 64, 4) or C % 8:
        raise ValueError("u must be [Cout/64][%d][2][16][64][4], got %s" % (C // 8, tuple(u_.shape)))
    Cout = u_.shape[0] * 64
    b_ = _need(bias, "bias") if bias is not None else None
    if out is None:
        out = torch.empty((N, Cout, H, W), dtype=torch.float32, device=x.device,
                          memory_format=torch.channels_last)
    if mosaic == "2d" and N > 0:
        st = lib().vd_conv3x3_wino_mosaic_bias_act(x.data_ptr(), N, H, W, C, u_.data_ptr(), Cout,
                                                   b_.data_ptr() if b_ is not None else None,
                                                   int(relu), out.data_ptr(), _stream())
    elif mosaic and N > 0:
        st = lib().vd_conv3x3_wino_seg_bias_act(x.data_ptr(), N * H, W, C, u_.data_ptr(), Cout,
                                                b_.data_ptr() if b_ is not None else None,
                                                int(relu), H, out.data_ptr(), _stream())
    else:
        st = lib().vd_conv3x3_wino_bias_act(x.data_ptr(), N, H, W, C, u_.data_ptr(), Cout,
                                            b_.data_ptr() if b_ is not None else None,
                                            int(relu), out.data_ptr(), _stream())
    if st == VD_ERR_SHAPE:
        return None
    check(st, "vd_conv3x3_wino_bias_act")
    return out


def conv3x3_wino4_weight(w: torch.Tensor) -> Optional[torch.Tensor]:
    """PyTorch conv weight [Cout][Cin][3][3] -> the Winograd F(4x4,3x3) operand
    U = G g G^T (6 x 6 positions) in the kernel's fragment order
    [Cout/64][Cin/8][4][18][64][4] (vd_conv3x3_wino4_weight; once per model).  None
    for a shape the kernel does not serve."""
    w_ = _need(w, "w")
    if w_.dim() != 4 or tuple(w_.shape[2:]) != (3, 3):
        raise ValueError("conv3x3_wino4_weight: weight %s" % (tuple(w_.shape),))
    Cout, C = w_.shape[:2]
    if Cout % 64 or C % 8 or Cout == 0 or C == 0 or C > WINO_MAX_CIN:
        return None
    u = torch.empty((Cout // 64, C // 8, 4, 18, 64, 4), dtype=torch.float32, device=w_.device)
    check(lib().vd_conv3x3_wino4_weight(w_.data_ptr(), Cout, C, u.data_ptr(), _stream()),
          "vd_conv3x3_wino4_weight")
    return u


def conv3x3_wino4_grouped_weight(w: torch.Tensor, groups: int) -> Optional[torch.Tensor]:
    """A grouped conv's weight [C][C / groups][3][3] (C / groups dividing 64) -> U for
    vd_conv3x3_wino4_grouped_bias_act: the block-diagonal expansion to [C][64][3][3]
    (each output channel's 64-channel input block, zeros outside its group) through
    conv3x3_wino4_weight (once per model).  None for a shape the kernel does not serve."""
    w_ = _need(w, "w")
    C, cpg = int(w_.shape[0]), int(w_.shape[1])
    if groups < 2 or cpg * groups != C or C % 64 or 64 % cpg or tuple(w_.shape[2:]) != (3, 3):
        return None
    G = 64 // cpg  # groups per 64-channel block
    wd = torch.zeros((C // 64, G, cpg, G, cpg, 3, 3), dtype=w_.dtype, device=w_.device)
    wg = w_.view(C // 64, G, cpg, cpg, 3, 3)
    for i in range(G):
        wd[:, i, :, i] = wg[:, i]
    return conv3x3_wino4_weight(wd.view(C, 64, 3, 3))


def conv3x3_wino4_bias_act(x: torch.Tensor, u: torch.Tensor, bias: Optional[torch.Tensor],
                           relu: bool = False, out: Optional[torch.Tensor] = None,
                           mosaic=False, groups: int = 1):
    """act(conv3x3(x, pad 1) + bias) on a channels_last fp32 tensor by Winograd
    F(4x4,3x3) (vd_conv3x3_wino4_bias_act); u from conv3x3_wino4_weight.  mosaic
    True / "pair": maps of at most 15 x 15 two per output block
    (vd_conv3x3_wino4_mosaic_bias_act); "rows": the maps stacked in one column at a
    4-row pitch (vd_conv3x3_wino4_rows_bias_act); both bit-identical.  "grid": the
    maps as a 2-D grid at an (H + 1) x (W + 1) pitch (vd_conv3x3_wino4_grid_bias_act;
    equal within Winograd rounding).  groups > 1: a grouped conv (u from
    conv3x3_wino4_grouped_weight; mosaic False or "rows").  None for a shape the kernel
    does not serve."""
    if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 4 \
            or not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("x must be a channels_last fp32 device tensor")
    if u is None:
        return None
    u_ = _need(u, "u")
    N, C, H, W = x.shape
    if groups > 1:
        if u_.dim() != 6 or tuple(u_.shape) != (C // 64, 8, 4, 18, 64, 4) or C % 64:
            raise ValueError("grouped u must be [%d][8][4][18][64][4], got %s"
                             % (C // 64, tuple(u_.shape)))
        if mosaic not in (False, None, "rows"):
            return None
        b_ = _need(bias, "bias") if bias is not None else None
        if out is None:
            out = torch.empty((N, C, H, W), dtype=torch.float32, device=x.device,
                              memory_format=torch.channels_last)
        st = lib().vd_conv3x3_wino4_grouped_bias_act(
            x.data_ptr(), N, H, W, C, u_.data_ptr(), int(groups),
            b_.data_ptr() if b_ is not None else None, int(relu), out.data_ptr(),
            int(mosaic == "rows"), _stream())
        if st == VD_ERR_SHAPE:
            return None
        check(st, "vd_conv3x3_wino4_grouped_bias_act")
        return out
    if u_.dim() != 6 or tuple(u_.shape[1:]) != (C // 8, 4, 18, 64, 4) or C % 8:
        raise ValueError("u must be [Cout/64][%d][4][18][64][4], got %s" % (C // 8, tuple(u_.shape)))
    Cout = u_.shape[0] * 64
    b_ = _need(bias, "bias") if bias is not None else None
    if out is None:
        out = torch.empty((N, Cout, H, W), dtype=torch.float32, device=x.device,
                          memory_format=torch.channels_last)
    fn = {False: lib().vd_conv3x3_wino4_bias_act, True: lib().vd_conv3x3_wino4_mosaic_bias_act,
          "pair": lib().vd_conv3x3_wino4_mosaic_bias_act,
          "rows": lib().vd_conv3x3_wino4_rows_bias_act,
          "grid": lib().vd_conv3x3_wino4_grid_bias_act}[mosaic]
    st = fn(x.data_ptr(), N, H, W, C, u_.data_ptr(), Cout,
            b_.data_ptr() if b_ is not None else None, int(relu), out.data_ptr(), _stream())
    if st == VD_ERR_SHAPE:
        return None
    check(st, "vd_conv3x3_wino4_bias_act (mosaic %r)" % (mosaic,))
    return out


def conv3x3_wino4_dilated2_bias_act(x: torch.Tensor, u: torch.Tensor,
                                    bias: Optional[torch.Tensor], relu: bool = False,
                                    out: Optional[torch.Tensor] = None, layout=False):
    """act(conv3x3(x, dilation 2, pad 2) + bias) of channels_last fp32 maps (H, W even)
    on the F(4x4) kernel as the plain conv of the polyphase sub-maps, read and written in
    place (vd_conv3x3_wino4_dilated2_bias_act); u from conv3x3_wino4_weight.  None for a
    shape the kernel does not serve.  layout: the sub-maps' block layout, False (one
    per block), "pair" (pairs / octets) or "grid"."""
    if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 4 \
            or not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("x must be a channels_last fp32 device tensor")
    lay = {False: 0, None: 0, "pair": 1, True: 1, "grid": 2}.get(layout)
    if lay is None:
        return None
    u_ = _need(u, "u")
    N, C, H, W = x.shape
    if u_.dim() != 6 or tuple(u_.shape[1:]) != (C // 8, 4, 18, 64, 4) or C % 8 or H % 2 or W % 2:
        return None
    Cout = u_.shape[0] * 64
    b_ = _need(bias, "bias") if bias is not None else None
    if out is None:
        out = torch.empty((N, Cout, H, W), dtype=torch.float32, device=x.device,
                          memory_format=torch.channels_last)
    st = lib().vd_conv3x3_wino4_dilated2_bias_act(
        x.data_ptr(), N, H, W, C, u_.data_ptr(), Cout, b_.data_ptr() if b_ is not None else None,
        int(relu), out.data_ptr(), lay, _stream())
    if st == VD_ERR_SHAPE:
        return None
    check(st, "vd_conv3x3_wino4_dilated2_bias_act")
    return out


def gemm_dual_bias_act(a1: torch.Tensor, a2: torch.Tensor, w: torch.Tensor, bias: torch.Tensor,
                       relu: bool = True, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """act(a1 @ w[:, :K1].T + a2 @ w[:, K1:].T + bias) in one MFMA kernel
    (vd_gemm_dual_bias_act): a1 [M,K1], a2 [M,K2], w [N,K1+K2], bias [N].
    Returns None for a shape the kernel does not serve (the caller falls back)."""
    a1_, a2_ = _need(a1, "a1"), _need(a2, "a2")
    w_, b_ = _need(w, "w"), _need(bias, "bias")
    M, K1 = a1_.shape
    K2 = a2_.shape[1]
    N = w_.shape[0]
    if a2_.shape[0] != M or w_.shape[1] != K1 + K2 or b_.numel() != N:
        raise ValueError("gemm_dual_bias_act: a1 %s, a2 %s, w %s, bias %s"
                         % (tuple(a1_.shape), tuple(a2_.shape), tuple(w_.shape), tuple(b_.shape)))
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a1_.device)
    elif tuple(out.shape) != (M, N) or not out.is_contiguous():
        raise ValueError("out must be a contiguous %s tensor" % ((M, N),))
    st = lib().vd_gemm_dual_bias_act(a1_.data_ptr(), K1, a2_.data_ptr(), K2, M, w_.data_ptr(), N,
                                     b_.data_ptr(), int(relu), out.data_ptr(), _stream())
    if st == VD_ERR_SHAPE:
        return None
    check(st, "vd_gemm_dual_bias_act")
    return out


FPN_LATERAL_K = (256, 512, 1024)  # csrc/gemm_lateral.hip (N = 256)


def fpn_lateral_weight(w: torch.Tensor) -> Optional[torch.Tensor]:
    """The lateral 1x1 conv weight [256][K] (or [256][K][1][1]) -> the fragment order
    vd_fpn_lateral_topdown reads (vd_fpn_lateral_weight; once per model).  None for a
    shape the kernel does not serve (N != 256 or K not in FPN_LATERAL_K)."""
    w_ = _need(w, "w").reshape(w.shape[0], -1).contiguous()
    N, K = w_.shape
    if N != 256 or K not in FPN_LATERAL_K:
        return None
    wf = torch.empty((K // 32, 16, 2, 64, 4), dtype=torch.float32, device=w_.device)
    check(lib().vd_fpn_lateral_weight(w_.data_ptr(), N, K, wf.data_ptr(), _stream()),
          "vd_fpn_lateral_weight")
    return wf


def fpn_lateral_topdown(lateral: torch.Tensor, wf: torch.Tensor, bias: torch.Tensor,
                        top: Optional[torch.Tensor]) -> torch.Tensor:
    """FPN.py topdown_lateral_module.forward (:292-300) in one MFMA launch
    (vd_fpn_lateral_topdown): conv_lateral(lateral) + nearest-2x(top), the sum in the
    reference's order ((conv + bias) + top).  lateral: channels_last N x K x H x W fp32;
    top: channels_last N x 256 x H/2 x W/2 (None: the lateral conv alone); wf from
    fpn_lateral_weight.  Returns a channels_last N x 256 x H x W tensor."""
    if not lateral.is_cuda or lateral.dtype != torch.float32 or lateral.dim() != 4 \
            or not lateral.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("lateral must be a channels_last fp32 device tensor")
    N, K, H, W = lateral.shape
    wf_ = _need(wf, "wf")
    b_ = _need(bias, "bias")
    if tuple(wf_.shape) != (K // 32, 16, 2, 64, 4) or b_.numel() != 256:
        raise ValueError("fpn_lateral_topdown: wf %s / bias %s for K = %d"
                         % (tuple(wf_.shape), tuple(b_.shape), K))
    t_ = None
    if top is not None:
        if tuple(top.shape) != (N, 256, H // 2, W // 2) or H % 2 or W % 2:
            raise ValueError("top must be %s, got %s" % ((N, 256, H // 2, W // 2),
                                                         tuple(top.shape)))
        if not top.is_cuda or top.dtype != torch.float32:
            raise ValueError("top must be a float32 device tensor")
        # (not _need: its .contiguous() would copy a channels_last tensor to NCHW)
        t_ = top if top.is_contiguous(memory_format=torch.channels_last) else \
            top.contiguous(memory_format=torch.channels_last)
    out = torch.empty((N, 256, H, W), dtype=torch.float32, device=lateral.device,
                      memory_format=torch.channels_last)
    check(lib().vd_fpn_lateral_topdown(lateral.data_ptr(), N * H * W, K, wf_.data_ptr(), 256,
                                       b_.data_ptr(), t_.data_ptr() if t_ is not None else None,
                                       H, W, out.data_ptr(), _stream()),
          "vd_fpn_lateral_topdown")
    return out


def pixel_lut(pixel_means=(102.9801, 115.9465, 122.7717)) -> np.ndarray:
    """float32(u - mean_c) for u in 0..255 exactly as numpy computes
    ``im.astype(float32); im -= PIXEL_MEANS`` (float64 subtraction, float32 store,
    lib/utils/blob.py:126-127)."""
    u = np.arange(256, dtype=np.float32).astype(np.float64)
    return np.stack([(u - m).astype(np.float32) for m in pixel_means]).reshape(-1)


def image_to_blob(frames: torch.Tensor, lut: torch.Tensor, Hp: int, Wp: int, nhwc: bool = False,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    fr = _need(frames, "frames", torch.uint8)
    F, H, W, three = fr.shape
    lt = _need(lut, "lut")
    if out is None:
        shape = (F, Hp, Wp, 3) if nhwc else (F, 3, Hp, Wp)
        out = torch.empty(shape, dtype=torch.float32, device=fr.device)
    check(lib().vd_image_to_blob(fr.data_ptr(), F, H, W, lt.data_ptr(), Hp, Wp, int(nhwc),
                                 out.data_ptr(), _stream()), "vd_image_to_blob")
    return out


def target_scale(im_h: int, im_w: int, target_size: float, max_size: float) -> float:
    """lib/utils/blob.py:153-160 get_target_scale (Python floats = doubles)."""
    smin, smax = min(im_h, im_w), max(im_h, im_w)
    s = float(target_size) / float(smin)
    if np.round(s * smax) > max_size:
        s = float(max_size) / float(smax)
    return s


def resized_hw(im_h: int, im_w: int, im_scale: float):
    """cv::resize's dsize for fx = fy = im_scale: saturate_cast<int> rounds half
    to even, as Python's round does."""
    return int(round(im_h * im_scale)), int(round(im_w * im_scale))


def image_resize_to_blob(frames: torch.Tensor, lut: torch.Tensor, im_scale: float, Hp: int,
                         Wp: int, nhwc: bool = False, out: Optional[torch.Tensor] = None):
    """prep_im_for_blob + im_list_to_blob at any scale (vd_image_resize_to_blob)."""
    fr = _need(frames, "frames", torch.uint8)
    F, H, W, three = fr.shape
    Hr, Wr = resized_hw(H, W, im_scale)
    if Hp < Hr or Wp < Wr:
        raise ValueError("blob %dx%d smaller than the resized frame %dx%d" % (Hp, Wp, Hr, Wr))
    lt = _need(lut, "lut")
    if out is None:
        shape = (F, Hp, Wp, 3) if nhwc else (F, 3, Hp, Wp)
        out = torch.empty(shape, dtype=torch.float32, device=fr.device)
    check(lib().vd_image_resize_to_blob(fr.data_ptr(), F, H, W, lt.data_ptr(), float(im_scale),
                                        Hr, Wr, Hp, Wp, int(nhwc), out.data_ptr(), _stream()),
          "vd_image_resize_to_blob")
    return out


# --------------------------------------------------------------------------- #
# Proposals, collect/distribute, detections                                    #
# --------------------------------------------------------------------------- #
def generate_proposals(cls_probs: Sequence[torch.Tensor], bbox_preds: Sequence[torch.Tensor],
                       anchors: Sequence[torch.Tensor], spatial_scales: Sequence[float],
                       im_info: torch.Tensor, pre_nms_topN: int, post_nms_topN: int,
                       nms_thresh: float, min_size: float, out=None):
    """GenerateProposalsOp over all levels / images.  Returns (rois [N,L,post,5],
    probs [N,L,post], counts int32 [N,L])."""
    L = len(cls_probs)
    descs = (_lib.VdRpnLevel * L)()
    keep = []
    N = cls_probs[0].shape[0]
    for i in range(L):
        p = _need(cls_probs[i], "cls_prob")
        d = _need(bbox_preds[i], "bbox_pred")
        a = _need(anchors[i], "anchors", torch.float64)
        keep += [p, d, a]
        _, A, H, W = p.shape
        descs[i] = _lib.VdRpnLevel(p.data_ptr(), d.data_ptr(), a.data_ptr(), A, H, W,
                                   float(spatial_scales[i]))
    info = _need(im_info, "im_info")
    dev = info.device
    if out is None:
        rois = torch.zeros((N, L, post_nms_topN, 5), dtype=torch.float32, device=dev)
        probs = torch.zeros((N, L, post_nms_topN), dtype=torch.float32, device=dev)
        counts = torch.zeros((N, L), dtype=torch.int32, device=dev)
    else:
        rois, probs, counts = out
    wsb = lib().vd_generate_proposals_workspace_size(descs, L, N, pre_nms_topN)
    ws = _ws(wsb, dev)
    check(lib().vd_generate_proposals(descs, L, N, info.data_ptr(), int(pre_nms_topN),
                                      int(post_nms_topN), float(np.float32(nms_thresh)),
                                      float(min_size), rois.data_ptr(), probs.data_ptr(),
                                      counts.data_ptr(), ws.data_ptr(), ws.numel(), _stream()),
          "vd_generate_proposals")
    return rois, probs, counts


COUNT_SELECT_FAILED, COUNT_PREV_BOXES = -1, -2  # include/vosdet.h VD_COUNT_*


def raise_on_failed_counts(counts, what: str = "frame"):
    """-1 in a per-image count means a device kernel could not complete that
    image (generate_proposals' top-k threshold search could not bracket
    pre_nms_topN within its candidate capacity; collect_distribute and
    box_detections pass the -1 on).  Raise instead of dropping proposals."""
    prev = [i for i, c in enumerate(counts) if c == COUNT_PREV_BOXES]
    if prev:
        raise _lib.VosdetError(
            "TEST.NMS_SMALL_BOX_IOU: the previous result of %s(s) %s holds more than one box "
            "of a class (lib_vos/tools/vos_test.py:848 asserts < 2; set "
            "TEST.NUM_DET_PER_CLASS_POST = 1 or TEST.NMS_WITH_MASK_IOU)" % (what, prev))
    bad = [i for i, c in enumerate(counts) if c < 0]
    if bad:
        raise _lib.VosdetError(
            "proposal selection failed for %s(s) %s: the pre_nms_topN threshold search "
            "could not bracket its candidates (count -1)" % (what, bad))


def collect_distribute(level_rois, level_probs, level_counts, post_nms_topN: int, k_min: int = 2,
                       k_max: int = 5, out=None):
    """collect + distribute per image: returns (rois [N,post,5], lvl idx int32
    [N,post] (level - k_min), counts int32 [N])."""
    lr = _need(level_rois, "level_rois")
    lp = _need(level_probs, "level_probs")
    lc = _need(level_counts, "level_counts", torch.int32)
    N, L, cap, _ = lr.shape
    if out is None:
        rois = torch.zeros((N, post_nms_topN, 5), dtype=torch.float32, device=lr.device)
        lvl = torch.zeros((N, post_nms_topN), dtype=torch.int32, device=lr.device)
        cnt = torch.zeros((N,), dtype=torch.int32, device=lr.device)
    else:
        rois, lvl, cnt = out
    check(lib().vd_collect_distribute(lr.data_ptr(), lp.data_ptr(), lc.data_ptr(), L, cap, N,
                                      int(post_nms_topN), k_min, k_max, rois.data_ptr(),
                                      lvl.data_ptr(), cnt.data_ptr(), _stream()),
          "vd_collect_distribute")
    return rois, lvl, cnt


SOFT_NMS_METHODS = {"hard": 0, "linear": 1, "gaussian": 2}  # utils/boxes.py:344
BBOX_VOTE_METHODS = {"ID": 0, "AVG": 1, "IOU_AVG": 2, "QUASI_SUM": 3}


def bbox_vote_method(scoring_method: str, beta: float = 1.0) -> int:
    """TEST.BBOX_VOTE.SCORING_METHOD -> vd_box_detections_ex's code; GENERALIZED_AVG
    at beta 1 is AVG (mean(ws**1)**1).  TEMP_AVG (numpy's float32 log / exp) and
    GENERALIZED_AVG at other betas raise NotImplementedError."""
    if scoring_method == "GENERALIZED_AVG" and float(beta) == 1.0:
        return BBOX_VOTE_METHODS["AVG"]
    if scoring_method not in BBOX_VOTE_METHODS:
        raise NotImplementedError("TEST.BBOX_VOTE.SCORING_METHOD=%r (beta %r) is not implemented"
                                  % (scoring_method, beta))
    return BBOX_VOTE_METHODS[scoring_method]


def box_detections(rois, cls_prob, bbox_pred, roi_count, im_scale, im_hw, score_thresh=0.05,
                   nms_thresh=0.5, dets_per_im=100, bbox_reg_weights=(10., 10., 5., 5.),
                   det_cap=256, out=None, nms_cross_class=0., num_det_per_class_pre=0,
                   soft_nms=None, soft_nms_sigma=0.5, bbox_vote=None, bbox_vote_thresh=0.8,
                   bbox_vote_beta=1.0):
    """Decode + clip + per-class NMS + detections limit.  rois [N,R,5],
    cls_prob [N,R,K], bbox_pred [N,R,4K] -> (dets [N,cap,5], cls int32 [N,cap],
    counts int32 [N]).  soft_nms: TEST.SOFT_NMS.METHOD ('hard' / 'linear' /
    'gaussian') instead of the NMS; bbox_vote: TEST.BBOX_VOTE.SCORING_METHOD
    (lib/core/test.py:756-776, vd_box_detections_ex)."""
    r = _need(rois, "rois")
    p = _need(cls_prob, "cls_prob")
    d = _need(bbox_pred, "bbox_pred")
    c = _need(roi_count, "roi_count", torch.int32)
    s = _need(im_scale, "im_scale")
    hw = _need(im_hw, "im_hw", torch.int32)
    N, R, K = p.shape
    if out is None:
        dets = torch.zeros((N, det_cap, 5), dtype=torch.float32, device=r.device)
        cls = torch.zeros((N, det_cap), dtype=torch.int32, device=r.device)
        cnt = torch.zeros((N,), dtype=torch.int32, device=r.device)
    else:
        dets, cls, cnt = out
    wsb = lib().vd_box_detections_workspace_size(R, N, K)
    ws = _ws(wsb, r.device)
    w = (ctypes.c_float * 4)(*[float(np.float32(x)) for x in bbox_reg_weights])
    if soft_nms is None and bbox_vote is None:
        check(lib().vd_box_detections(r.data_ptr(), p.data_ptr(), d.data_ptr(), c.data_ptr(), R,
                                      N, K, s.data_ptr(), hw.data_ptr(),
                                      float(np.float32(score_thresh)),
                                      float(np.float32(nms_thresh)), int(dets_per_im),
                                      ctypes.cast(w, ctypes.c_void_p), det_cap, dets.data_ptr(),
                                      cls.data_ptr(), cnt.data_ptr(), ws.data_ptr(), ws.numel(),
                                      _stream()), "vd_box_detections")
    else:
        sm = -1 if soft_nms is None else SOFT_NMS_METHODS[soft_nms]
        vm = -1 if bbox_vote is None else bbox_vote_method(bbox_vote, bbox_vote_beta)
        check(lib().vd_box_detections_ex(
            r.data_ptr(), p.data_ptr(), d.data_ptr(), c.data_ptr(), R, N, K, s.data_ptr(),
            hw.data_ptr(), float(np.float32(score_thresh)), float(np.float32(nms_thresh)),
            int(dets_per_im), ctypes.cast(w, ctypes.c_void_p), sm,
            float(np.float32(soft_nms_sigma)), float(np.float32(0.0001)), vm,
            float(np.float32(bbox_vote_thresh)), float(bbox_vote_beta), det_cap, dets.data_ptr(),
            cls.data_ptr(), cnt.data_ptr(), ws.data_ptr(), ws.numel(), _stream()),
            "vd_box_detections_ex")
    if nms_cross_class > 0 or num_det_per_class_pre > 0:  # the fork's vos_test.py:805-833
        check(lib().vd_detections_postfilter(dets.data_ptr(), cls.data_ptr(), cnt.data_ptr(), N,
                                             det_cap, float(np.float32(nms_cross_class)),
                                             int(num_det_per_class_pre), _stream()),
              "vd_detections_postfilter")
    return dets, cls, cnt


def detections_prev_box_filter(dets: torch.Tensor, classes: torch.Tensor, counts: torch.Tensor,
                               prev_dets: torch.Tensor, prev_classes: torch.Tensor,
                               prev_counts: torch.Tensor, iou_thresh: float,
                               score_thresh: float) -> None:
    """TEST.NMS_SMALL_BOX_IOU (lib_vos/tools/vos_test.py:845-860) in place on the
    device detections (vd_detections_prev_box_filter): dets [F,cap,5], classes /
    counts as box_detections writes them; prev_* the previous frame's final result
    of each row ([F,pcap,5], [F,pcap], [F]).  A row whose previous result holds
    two boxes of one class gets count -1 (the reference asserts)."""
    d, c, n = _need(dets, "dets"), _need(classes, "classes", torch.int32), \
        _need(counts, "counts", torch.int32)
    pd, pc, pn = _need(prev_dets, "prev_dets"), _need(prev_classes, "prev_classes", torch.int32), \
        _need(prev_counts, "prev_counts", torch.int32)
    F, cap = d.shape[0], d.shape[1]
    if tuple(pd.shape[:1]) != (F,) or pd.shape[2] != 5 or tuple(pc.shape) != tuple(pd.shape[:2]) \
            or pn.numel() != F:
        raise ValueError("prev_* must be [F,pcap,5], [F,pcap], [F] for F = %d" % F)
    check(lib().vd_detections_prev_box_filter(
        d.data_ptr(), c.data_ptr(), n.data_ptr(), F, cap, pd.data_ptr(), pc.data_ptr(),
        pn.data_ptr(), pd.shape[1], float(np.float32(iou_thresh)),
        float(np.float32(score_thresh)), _stream()), "vd_detections_prev_box_filter")


def mask_iou_nms(planes: torch.Tensor, dets: torch.Tensor, classes: torch.Tensor,
                 iou_th: float, max_per_class: int) -> torch.Tensor:
    """nms_with_mask_iou (lib_vos/tools/vos_test.py:985-1029) on one frame
    (vd_mask_iou_nms): planes [n,H,W] uint8 binary masks, dets [n,>=5], classes
    [n] int32, in cls_boxes order.  Returns the kept indices (int64) in the
    reference's output order (class ascending, then score order)."""
    pl = _need(planes, "planes", torch.uint8)
    d, c = _need(dets, "dets"), _need(classes, "classes", torch.int32)
    n = d.shape[0]
    if pl.shape[0] != n or c.numel() != n:
        raise ValueError("planes, dets and classes must have the same n")
    H, W = (pl.shape[1], pl.shape[2]) if pl.dim() == 3 else (1, 1)
    keep = torch.empty((max(n, 1),), dtype=torch.int64, device=d.device)
    num = torch.zeros((1,), dtype=torch.int32, device=d.device)
    ws = _ws(lib().vd_mask_iou_nms_workspace_size(n, H, W), d.device)
    check(lib().vd_mask_iou_nms(pl.data_ptr() if n else None, n, H, W,
                                d.data_ptr() if n else None, d.shape[1] if d.dim() == 2 else 5,
                                c.data_ptr() if n else None, float(iou_th), int(max_per_class),
                                keep.data_ptr(), num.data_ptr(), ws.data_ptr(), ws.numel(),
                                _stream()), "vd_mask_iou_nms")
    return keep[: int(num.item())]


# --------------------------------------------------------------------------- #
# segm_results: paste + binarize + RLE counts      #
# --------------------------------------------------------------------------- #
def paste_masks(masks: torch.Tensor, boxes: torch.Tensor, im_h: int, im_w: int,
                thresh: float = 0.5, out=None) -> torch.Tensor:
    """masks [M,R,R] fp32 (class-selected probabilities), boxes [M,>=4] fp32 image
    coordinates -> [M,im_h,im_w] uint8 binary masks (segm_results' expand_boxes +
    cv2.resize + `> THRESH_BINARIZE` + paste, lib/core/test.py:801-835)."""
    m = _need(masks, "masks")
    b = _need(boxes, "boxes")
    M, R = m.shape[0], m.shape[-1]
    if b.shape[0] != M or b.dim() != 2 or b.shape[1] < 4:
        raise ValueError("boxes must be M x >=4, got %s" % (tuple(b.shape),))
    if out is None:
        out = torch.empty((M, im_h, im_w), dtype=torch.uint8, device=m.device)
    check(lib().vd_paste_masks(m.data_ptr(), M, R, b.data_ptr(), b.shape[1], int(im_h),
                               int(im_w), float(np.float32(thresh)), out.data_ptr(), _stream()),
          "vd_paste_masks")
    return out


def mask_rle_counts(planes: torch.Tensor, cap: Optional[int] = None):
    """pycocotools mask.encode run lengths (column-major, zeros first) of each
    [H,W] uint8 plane: returns (counts int32 [M,cap'], n int32 [M]); runs are
    < H*W <= 2^31, so int32 holds the kernel's uint32 counts."""
    p = _need(planes, "planes", torch.uint8)
    M, H, W = p.shape
    cap = int(cap or (8 * W + 2))
    while True:
        counts = torch.empty((M, cap), dtype=torch.int32, device=p.device)
        n = torch.empty((M,), dtype=torch.int32, device=p.device)
        check(lib().vd_mask_rle(p.data_ptr(), M, H, W, counts.data_ptr(), cap, n.data_ptr(),
                                _stream()), "vd_mask_rle")
        need = int((-n).max().item()) if M else 0
        if need <= cap:
            return counts, n
        cap = need


def bias_relu_maxpool(x_raw: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """ResNet stem tail (vd_bias_relu_maxpool): MaxPool2d(3, 2, 1)(relu(x + b)) of
    a channels_last N x C x H x W tensor; returns channels_last N x C x Ho x Wo."""
    N, C, H, W = x_raw.shape
    if not (x_raw.is_cuda and x_raw.dtype == torch.float32
            and x_raw.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError("x_raw must be a channels_last float32 device tensor")
    b = _need(bias, "bias")
    if b.numel() != C:
        raise ValueError("bias must have C = %d entries" % C)
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    out = torch.empty((N, C, Ho, Wo), dtype=torch.float32, device=x_raw.device,
                      memory_format=torch.channels_last)
    check(lib().vd_bias_relu_maxpool(x_raw.data_ptr(), b.data_ptr(), N, C, H, W,
                                     out.data_ptr(), _stream()), "vd_bias_relu_maxpool")
    return out


def stem_pack(weight: torch.Tensor, split: bool = False) -> torch.Tensor:
    """conv1's weight [64, 3, 7, 7] in vd_stem_conv_pool's register order (once), or
    (split) its three-piece bf16 image for vd_stem_split_conv_pool (a uint8 tensor)."""
    w = _need(weight, "weight")
    if tuple(w.shape) != (64, 3, 7, 7):
        raise ValueError("stem weight must be 64 x 3 x 7 x 7, got %s" % (tuple(w.shape),))
    if split:
        out = torch.empty((lib().vd_stem_split_weight_size(),), dtype=torch.uint8,
                          device=w.device)
        check(lib().vd_stem_split_weight_pack(w.data_ptr(), out.data_ptr(), _stream()),
              "vd_stem_split_weight_pack")
        return out
    out = torch.empty((lib().vd_stem_weight_size() // 4,), dtype=torch.float32, device=w.device)
    check(lib().vd_stem_weight_pack(w.data_ptr(), out.data_ptr(), _stream()),
          "vd_stem_weight_pack")
    return out


def stem_conv_pool(x: torch.Tensor, packed: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """ResNet stem in one kernel (vd_stem_conv_pool, or vd_stem_split_conv_pool for a
    split image from stem_pack(w, split=True)): MaxPool2d(3, 2, 1)(relu(conv1 7x7/2
    pad 3 (x) + bias)) for a channels_last N x 3 x H x W blob; returns channels_last
    N x 64 x Ho x Wo (the conv output never leaves LDS)."""
    N, C, H, W = x.shape
    if not (x.is_cuda and x.dtype == torch.float32 and C == 3
            and x.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError("x must be a channels_last float32 N x 3 x H x W device tensor")
    b = _need(bias, "bias")
    if b.numel() != 64:
        raise ValueError("bias must have 64 entries")
    split = packed.dtype == torch.uint8
    need = lib().vd_stem_split_weight_size() if split else lib().vd_stem_weight_size()
    if not packed.is_cuda or packed.numel() * packed.element_size() != need:
        raise ValueError("packed must be stem_pack's device image (%d bytes)" % need)
    Hc, Wc = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    Ho, Wo = (Hc - 1) // 2 + 1, (Wc - 1) // 2 + 1
    out = torch.empty((N, 64, Ho, Wo), dtype=torch.float32, device=x.device,
                      memory_format=torch.channels_last)
    fn = lib().vd_stem_split_conv_pool if split else lib().vd_stem_conv_pool
    check(fn(x.data_ptr(), N, H, W, packed.data_ptr(), b.data_ptr(), out.data_ptr(), _stream()),
          "vd_stem_split_conv_pool" if split else "vd_stem_conv_pool")
    return out


def rpn_head(x_raw: torch.Tensor, conv_bias: torch.Tensor, w: torch.Tensor, b: torch.Tensor,
             num_anchors: int):
    """FPN RPN head of one level (vd_rpn_head): x_raw = the shared 3x3 conv's
    output without bias, N x C x H x W in channels_last memory; w [5A, C] (cls
    then bbox 1x1 weights), b [5A].  Returns (cls_prob N x A x H x W after the
    sigmoid, bbox_pred N x 4A x H x W), both contiguous NCHW."""
    N, C, H, W = x_raw.shape
    if not (x_raw.is_cuda and x_raw.dtype == torch.float32
            and x_raw.is_contiguous(memory_format=torch.channels_last)):
        raise ValueError("x_raw must be a channels_last float32 device tensor")
    A = int(num_anchors)
    cb = _need(conv_bias, "conv_bias")
    wt = _need(w, "w")
    bt = _need(b, "b")
    if tuple(wt.shape) != (5 * A, C) or bt.numel() != 5 * A or cb.numel() != C:
        raise ValueError("w must be [5A, C] = [%d, %d], b [5A], conv_bias [C]" % (5 * A, C))
    cls = torch.empty((N, A, H, W), dtype=torch.float32, device=x_raw.device)
    box = torch.empty((N, 4 * A, H, W), dtype=torch.float32, device=x_raw.device)
    check(lib().vd_rpn_head(x_raw.data_ptr(), cb.data_ptr(), wt.data_ptr(), bt.data_ptr(), N, H,
                            W, C, A, cls.data_ptr(), box.data_ptr(), _stream()), "vd_rpn_head")
    return cls, box


def segm_rle_counts(masks: torch.Tensor, boxes: torch.Tensor, im_h: int, im_w: int,
                    thresh: float = 0.5, cap: Optional[int] = None):
    """paste_masks + mask_rle_counts fused (vd_segm_rle): the same counts and n
    without materialising the M x im_h x im_w planes.  Frames wider than the
    fused kernel's LDS column table (VD_ERR_SHAPE) take the two-pass planes path
    (paste_masks, then mask_rle_counts), which has no width limit."""
    m = _need(masks, "masks")
    b = _need(boxes, "boxes")
    M, R = m.shape[0], m.shape[-1]
    if b.shape[0] != M or b.dim() != 2 or b.shape[1] < 4:
        raise ValueError("boxes must be M x >=4, got %s" % (tuple(b.shape),))
    cap = int(cap or (4 * im_w + 2))
    while True:
        counts = torch.empty((M, cap), dtype=torch.int32, device=m.device)
        n = torch.empty((M,), dtype=torch.int32, device=m.device)
        st = lib().vd_segm_rle(m.data_ptr(), M, R, b.data_ptr(), b.shape[1], int(im_h),
                               int(im_w), float(np.float32(thresh)), counts.data_ptr(), cap,
                               n.data_ptr(), _stream())
        if st == VD_ERR_SHAPE:
            return mask_rle_counts(paste_masks(m, b, im_h, im_w, thresh))
        check(st, "vd_segm_rle")
        need = int((-n).max().item()) if M else 0
        if need <= cap:
            return counts, n
        cap = need


def rle_strings(counts: torch.Tensor, n: torch.Tensor) -> list:
    """pycocotools rleToString of each row's counts[:n] on the device
    (vd_rle_strings): list of M ASCII strings, as segm_results stores them."""
    c = _need(counts, "counts", torch.int32)
    nn = _need(n, "n", torch.int32)
    M, cap = c.shape
    if M == 0:
        return []
    lens = torch.empty((M,), dtype=torch.int32, device=c.device)
    check(lib().vd_rle_strings(c.data_ptr(), nn.data_ptr(), M, cap, lens.data_ptr(), None,
                               _stream()), "vd_rle_strings")
    offs = np.zeros(M + 1, np.int64)
    np.cumsum(lens.cpu().numpy(), out=offs[1:])
    total = int(offs[-1])
    if total >= 2 ** 31:
        raise ValueError("RLE strings of %d detections exceed 2 GiB" % M)
    chars = torch.empty((max(total, 1),), dtype=torch.uint8, device=c.device)
    check(lib().vd_rle_strings(c.data_ptr(), nn.data_ptr(), M, cap, lens.data_ptr(),
                               chars.data_ptr(), _stream()), "vd_rle_strings")
    buf = chars[:total].cpu().numpy().tobytes()
    return [buf[offs[i]:offs[i + 1]].decode("ascii") for i in range(M)]


# --------------------------------------------------------------------------- #
# VOS temporal path: FlowAlign, GroupNorm epilogues, ConvGRU gates             #
# --------------------------------------------------------------------------- #
def _fmt(x: torch.Tensor, name: str) -> int:
    """Memory format of a 4-D fp32 device tensor as a vosdet layout code."""
    if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 4:
        raise ValueError("%s must be a 4-D float32 device tensor" % name)
    if x.is_contiguous():
        return _lib.VD_LAYOUT_NCHW
    if x.is_contiguous(memory_format=torch.channels_last):
        return _lib.VD_LAYOUT_NHWC
    raise ValueError("%s must be contiguous (NCHW or channels_last)" % name)


def _like(x: torch.Tensor, layout: int, name: str) -> torch.Tensor:
    """x in the memory format `layout` (a copy only if it is not already)."""
    want = torch.channels_last if layout == _lib.VD_LAYOUT_NHWC else torch.contiguous_format
    if not x.is_cuda or x.dtype != torch.float32:
        raise ValueError("%s must be a float32 device tensor" % name)
    return x if x.is_contiguous(memory_format=want) else x.contiguous(memory_format=want)


def _empty_as(x: torch.Tensor, layout: int, shape=None) -> torch.Tensor:
    shape = tuple(x.shape) if shape is None else shape
    fmt = torch.channels_last if layout == _lib.VD_LAYOUT_NHWC else torch.contiguous_format
    return torch.empty(shape, dtype=torch.float32, device=x.device, memory_format=fmt)


def flow_align(features: torch.Tensor, flow: torch.Tensor) -> torch.Tensor:
    """FlowAlignFunction.forward (lib_vos/vos_model/flow_align/functions/flow_align.py:13-30):
    features B x C x H x W (NCHW, or channels_last -> the NHWC kernel), flow
    B x 2 x H x W at the feature resolution.  Output in the features' format."""
    lay = _fmt(features, "features")
    fl = _need(flow, "flow")
    B, C, H, W = features.shape
    if tuple(fl.shape) != (B, 2, H, W):
        raise ValueError("flow must be B x 2 x H x W = %s, got %s" % ((B, 2, H, W),
                                                                      tuple(fl.shape)))
    out = _empty_as(features, lay)
    check(lib().vd_flow_align_forward(features.data_ptr(), fl.data_ptr(), B, C, H, W, lay,
                                      out.data_ptr(), _stream()), "vd_flow_align_forward")
    return out


def flow_align_backward(grad_out, features, flow):
    g = _need(grad_out, "grad_out")
    f = _need(features, "features")
    fl = _need(flow, "flow")
    B, C, H, W = f.shape
    gf = torch.zeros_like(f)
    gfl = torch.zeros((B, 2, H, W), dtype=torch.float32, device=f.device)
    check(lib().vd_flow_align_backward(g.data_ptr(), f.data_ptr(), fl.data_ptr(), B, C, H, W,
                                       gf.data_ptr(), gfl.data_ptr(), _stream()),
          "vd_flow_align_backward")
    return gf, gfl


class FlowAlignFunction(torch.autograd.Function):
    """functions/flow_align.py:7-45 (static autograd Function, as the reference).
    CPU tensors raise like the reference's NotImplementedError branch (:28-29)."""

    @staticmethod
    def forward(ctx, features, flows):
        if not features.is_cuda:
            raise NotImplementedError
        ctx.save_for_backward(features, flows)
        return flow_align(features, flows)

    @staticmethod
    def backward(ctx, grad_output):
        features, flows = ctx.saved_tensors
        return flow_align_backward(grad_output, features, flows)


_ACT = {None: 0, "none": 0, "relu": 1, "sigmoid": 2, "tanh": 3}


def group_norm_act(x: torch.Tensor, num_groups: int, gamma: torch.Tensor, beta: torch.Tensor,
                   eps: float = 1e-5, x2: Optional[torch.Tensor] = None, residual=None,
                   residual_gn=None, upsample_residual: bool = False, act=None,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """act(GN(x [+ x2]) + residual) in one statistics + one apply pass
    (vd_group_norm_act).  residual_gn = (gamma_r, beta_r) normalises the residual
    with its own statistics (basic_gn_shortcut).  Works on NCHW or channels_last
    tensors; the output keeps x's memory format.  out may be x (in place)."""
    lay = _fmt(x, "x")
    B, C, H, W = x.shape
    if x2 is not None:
        x2 = _like(x2, lay, "x2")
    mode = 0
    res = None
    if residual is not None:
        mode = 3 if residual_gn is not None else (2 if upsample_residual else 1)
        want = (B, C, H // 2, W // 2) if mode == 2 else (B, C, H, W)
        if tuple(residual.shape) != want:
            raise ValueError("residual shape %s, expected %s" % (tuple(residual.shape), want))
        res = _like(residual, lay, "residual")
    if out is None:
        out = _empty_as(x, lay)
    rg, rb = residual_gn if residual_gn is not None else (None, None)
    nws = lib().vd_group_norm_workspace_size(B, num_groups) * (2 if mode == 3 else 1)
    ws = _ws(nws, x.device)
    check(lib().vd_group_norm_act(
        x.data_ptr(), x2.data_ptr() if x2 is not None else None, B, C, H, W, int(num_groups),
        float(eps), gamma.data_ptr(), beta.data_ptr(), res.data_ptr() if res is not None else None,
        mode, rg.data_ptr() if rg is not None else None, rb.data_ptr() if rb is not None else None,
        _ACT[act], lay, out.data_ptr(), ws.data_ptr(), ws.numel(), _stream()),
        "vd_group_norm_act")
    return out


def convgru_gates(zx, rx, h, zh, rh, num_groups, gamma_z, beta_z, gamma_r, beta_r, eps=1e-5):
    """(z, h*r) of convgrucell.py:85-87 from the six convolution outputs; with
    h None (zero state) returns (z, None)."""
    lay = _fmt(zx, "zx")
    B, C, H, W = zx.shape
    z = _empty_as(zx, lay)
    hr = _empty_as(zx, lay) if h is not None else None
    ws = _ws(2 * lib().vd_group_norm_workspace_size(B, num_groups), zx.device)
    ptr = lambda t: _like(t, lay, "t").data_ptr() if t is not None else None  # noqa: E731
    check(lib().vd_convgru_gates(
        ptr(zh), zx.data_ptr(), ptr(rh), ptr(rx), ptr(h), B, C, H, W, int(num_groups),
        float(eps), gamma_z.data_ptr(), beta_z.data_ptr(), gamma_r.data_ptr(), beta_r.data_ptr(),
        lay, z.data_ptr(), hr.data_ptr() if hr is not None else None, ws.data_ptr(), ws.numel(),
        _stream()), "vd_convgru_gates")
    return z, hr


def convgru_update(hx, hh, z, h, num_groups, gamma_h, beta_h, finer=None, eps=1e-5,
                   out: Optional[torch.Tensor] = None):
    """hn = (1-z)*h + z*tanh(GN_h(hh + hx)) (convgrucell.py:88-91), fused with the
    VOS fusion hn/2 + bilinear_0.5x(finer)/2 (vos_model_builder.py:341-342)."""
    lay = _fmt(hx, "hx")
    B, C, H, W = hx.shape
    if finer is not None and tuple(finer.shape) != (B, C, 2 * H, 2 * W):
        raise ValueError("finer level must be %s, got %s" % ((B, C, 2 * H, 2 * W),
                                                             tuple(finer.shape)))
    if out is None:
        out = _empty_as(hx, lay)
    ws = _ws(lib().vd_group_norm_workspace_size(B, num_groups), hx.device)
    ptr = lambda t: _like(t, lay, "t").data_ptr() if t is not None else None  # noqa: E731
    check(lib().vd_convgru_update(
        ptr(hh), hx.data_ptr(), ptr(z), ptr(h), ptr(finer), B, C, H, W, int(num_groups),
        float(eps), gamma_h.data_ptr(), beta_h.data_ptr(), lay, out.data_ptr(), ws.data_ptr(),
        ws.numel(), _stream()), "vd_convgru_update")
    return out
