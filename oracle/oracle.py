"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY (the parity checker).

CPU restatement of the reference's per-frame Mask R-CNN hot path, used to check
the HIP kernels in ``vosdetectron_amd``.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import this module; the product path
never does (it fails loudly when its HIP library is missing).

Byte/index semantics follow the reference functions cited on each function, as
executed by numpy 2.2 (this image).  Two deliberate, documented readings:

* Sorting.  The reference uses numpy's default (unstable) ``argsort`` /
  ``argpartition``; with tied keys their order is implementation-defined.  The
  oracle uses the *stable* reading: ``argsort(-s)`` keeps ties in index order,
  ``s.argsort()[::-1]`` (the NMS order) visits ties highest-index-first -- the
  order the survey observed for the reference (``keep=[1, 2]`` for two
  identical boxes).  Golden fixtures generated from the reference itself use
  tie-free scores, where every reading agrees.
* dtype promotion.  ``BBOX_XFORM_CLIP`` is an ``np.float64`` scalar
  (``lib/core/config.py:1009``), so under numpy 2 (NEP 50) ``np.minimum(dw,
  clip)`` promotes ``dw``/``dh`` -- and with them ``exp(dw) * w`` and the box
  corners -- to float64 before the float32 store.  The oracle (and the HIP
  decode kernel) reproduce that.

Pinning: the functions marked ``[pinned]`` are checked against golden vectors
produced by importing the reference's own Python (``tools/gen_goldens.py`` ->
``tests/golden/``) and against the anchor known-answer table in
``lib/modeling/generate_anchors.py:26-51``.  The C kernels in ``roi_ops.c`` are
"parity unpinned" against an executed reference (see that file's header).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

BBOX_XFORM_CLIP = np.log(1000. / 16.)  # lib/core/config.py:1009 (np.float64)
PIXEL_MEANS = np.array([[[102.9801, 115.9465, 122.7717]]])  # config.py:1015


def build(force: bool = False) -> str:
    """Compile roi_ops.c into oracle/liboracle.so (gcc, no FMA contraction)."""
    src = os.path.join(_HERE, "roi_ops.c")
    if force or not os.path.exists(_LIB_PATH) or \
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        f32p = ctypes.POINTER(ctypes.c_float)
        i32p = ctypes.POINTER(ctypes.c_int32)
        i64p = ctypes.POINTER(ctypes.c_int64)
        ci, cf = ctypes.c_int, ctypes.c_float
        L.or_roi_align_fwd.argtypes = [f32p, ci, ci, ci, ci, f32p, ci, ci, ci, cf, ci, f32p]
        L.or_roi_align_bwd.argtypes = [f32p, ci, ci, ci, ci, f32p, ci, ci, ci, cf, ci, f32p]
        L.or_roi_align_legacy_fwd.argtypes = [f32p, ci, ci, ci, ci, f32p, ci, ci, ci, cf, f32p]
        L.or_roi_pool_fwd.argtypes = [f32p, ci, ci, ci, ci, f32p, ci, ci, ci, cf, f32p, i32p]
        L.or_roi_crop_fwd.argtypes = [f32p, ci, ci, ci, ci, f32p, ci, ci, ci, f32p]
        L.or_flow_align_fwd.argtypes = [f32p, f32p, ci, ci, ci, ci, f32p]
        L.or_flow_align_bwd.argtypes = [f32p, f32p, f32p, ci, ci, ci, ci, f32p, f32p]
        L.or_nms.argtypes = [f32p, ci, ci, cf, i64p]
        L.or_nms.restype = ci
        _lib = L
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _p(a, t=ctypes.c_float):
    return a.ctypes.data_as(ctypes.POINTER(t))


# --------------------------------------------------------------------------- #
# RoI operators (C restatements, see roi_ops.c)                                #
# --------------------------------------------------------------------------- #
def roi_align(features, rois, ph, pw, spatial_scale, sampling_ratio):
    """Caffe2 RoIAlign fwd, roi_align_kernel.cu:65-121. features NCHW f32."""
    f, r = _f32(features), _f32(rois)
    B, C, H, W = f.shape
    R = r.shape[0]
    out = np.zeros((R, C, ph, pw), np.float32)
    if R:
        lib().or_roi_align_fwd(_p(f), B, C, H, W, _p(r), R, ph, pw,
                               float(spatial_scale), int(sampling_ratio), _p(out))
    return out


def flow_align(features, flow):
    """FlowAlign fwd, lib_vos/vos_model/flow_align/src/flow_align_cuda_kernel.cu:15-55.
    features B x C x H x W f32, flow B x 2 x H x W f32."""
    f, fl = _f32(features), _f32(flow)
    B, C, H, W = f.shape
    out = np.zeros_like(f)
    lib().or_flow_align_fwd(_p(f), _p(fl), B, C, H, W, _p(out))
    return out


def flow_align_backward(top_diff, features, flow):
    """FlowAlign bwd, flow_align_cuda_kernel.cu:57-117 (serial accumulation)."""
    g, f, fl = _f32(top_diff), _f32(features), _f32(flow)
    B, C, H, W = f.shape
    gf = np.zeros_like(f)
    gfl = np.zeros((B, 2, H, W), np.float32)
    lib().or_flow_align_bwd(_p(g), _p(f), _p(fl), B, C, H, W, _p(gf), _p(gfl))
    return gf, gfl


def flow_downsample(flow, spatial_scale):
    """FlowAlign.conv_flow_downsample (modules/flow_align.py:12-25): a 2->2
    conv, kernel = stride = 1/scale, weight diag = scale**3, no bias (float32
    torch conv, as the reference module computes it)."""
    import torch
    k = int(1.0 / spatial_scale)
    w = torch.zeros((2, 2, k, k), dtype=torch.float32)
    for i in range(2):
        w[i, i] = spatial_scale ** 3
    return torch.nn.functional.conv2d(torch.as_tensor(flow, dtype=torch.float32), w,
                                      stride=k).numpy()


def roi_align_backward(top_diff, rois, feat_shape, spatial_scale, sampling_ratio):
    """Caffe2 RoIAlign bwd, roi_align_kernel.cu:195-270 (serial sum order)."""
    g, r = _f32(top_diff), _f32(rois)
    B, C, H, W = feat_shape
    R, _, ph, pw = g.shape
    out = np.zeros((B, C, H, W), np.float32)
    if R:
        lib().or_roi_align_bwd(_p(g), B, C, H, W, _p(r), R, ph, pw,
                               float(spatial_scale), int(sampling_ratio), _p(out))
    return out


def roi_align_legacy(features, rois, ph, pw, spatial_scale):
    """jwyang RoIAlign fwd, lib/model/roi_align/src/roi_align_kernel.cu:15-70."""
    f, r = _f32(features), _f32(rois)
    B, C, H, W = f.shape
    R = r.shape[0]
    out = np.zeros((R, C, ph, pw), np.float32)
    if R:
        lib().or_roi_align_legacy_fwd(_p(f), B, C, H, W, _p(r), R, ph, pw,
                                      float(spatial_scale), _p(out))
    return out


def roi_pool(features, rois, ph, pw, spatial_scale):
    """RoIPool fwd (CUDA semantics), roi_pooling_kernel.cu:24-93."""
    f, r = _f32(features), _f32(rois)
    B, C, H, W = f.shape
    R = r.shape[0]
    out = np.zeros((R, C, ph, pw), np.float32)
    arg = np.zeros((R, C, ph, pw), np.int32)
    if R:
        lib().or_roi_pool_fwd(_p(f), B, C, H, W, _p(r), R, ph, pw,
                              float(spatial_scale), _p(out), _p(arg, ctypes.c_int32))
    return out, arg


def roi_crop(features, grid_yx):
    """RoICrop bilinear sampler fwd, roi_crop_cuda_kernel.cu:47-109."""
    f, g = _f32(features), _f32(grid_yx)
    B, C, H, W = f.shape
    R, GH, GW, _ = g.shape
    out = np.zeros((R, C, GH, GW), np.float32)
    if R:
        lib().or_roi_crop_fwd(_p(f), B, C, H, W, _p(g), R, GH, GW, _p(out))
    return out


def nms(dets, thresh):
    """utils.boxes.nms -> cython_nms.nms (boxes.py:329-333, cython_nms.pyx:37-87).

    Returns kept indices, ascending, int64 (``[]`` -> empty array)."""
    d = _f32(dets)
    n = d.shape[0]
    if n == 0:
        return np.zeros((0,), np.int64)
    keep = np.empty((n,), np.int64)
    k = lib().or_nms(_p(d), n, d.shape[1], float(np.float32(thresh)),
                     _p(keep, ctypes.c_int64))
    return keep[:k]


# --------------------------------------------------------------------------- #
# Anchors, box decode, proposals                                   [pinned]    #
# --------------------------------------------------------------------------- #
def generate_anchors(stride=16, sizes=(32, 64, 128, 256, 512), aspect_ratios=(0.5, 1, 2)):
    """lib/modeling/generate_anchors.py:54-123 (float64)."""
    scales = np.array(sizes, dtype=np.float64) / stride
    ratios = np.array(aspect_ratios, dtype=np.float64)
    anchor = np.array([1, 1, stride, stride], dtype=np.float64) - 1

    def whctrs(a):
        w = a[2] - a[0] + 1
        h = a[3] - a[1] + 1
        return w, h, a[0] + 0.5 * (w - 1), a[1] + 0.5 * (h - 1)

    def mk(ws, hs, xc, yc):
        ws, hs = ws[:, None], hs[:, None]
        return np.hstack((xc - 0.5 * (ws - 1), yc - 0.5 * (hs - 1),
                          xc + 0.5 * (ws - 1), yc + 0.5 * (hs - 1)))

    w, h, xc, yc = whctrs(anchor)
    ws = np.round(np.sqrt(w * h / ratios))
    hs = np.round(ws * ratios)
    base = mk(ws, hs, xc, yc)
    out = []
    for i in range(base.shape[0]):
        w, h, xc, yc = whctrs(base[i])
        out.append(mk(w * scales, h * scales, xc, yc))
    return np.vstack(out)


def fpn_level_anchors(lvl, k_min=2, start_size=32, ratios=(0.5, 1, 2)):
    """Per-level anchors as built in lib/modeling/FPN.py:340-350."""
    return generate_anchors(stride=2. ** lvl, sizes=(start_size * 2. ** (lvl - k_min),),
                            aspect_ratios=ratios)


def bbox_transform(boxes, deltas, weights=(1.0, 1.0, 1.0, 1.0), clip=BBOX_XFORM_CLIP):
    """lib/utils/boxes.py:156-205, numpy-2 promotion semantics (see module doc)."""
    if boxes.shape[0] == 0:
        return np.zeros((0, deltas.shape[1]), dtype=deltas.dtype)
    boxes = boxes.astype(deltas.dtype, copy=False)
    widths = boxes[:, 2] - boxes[:, 0] + 1.0
    heights = boxes[:, 3] - boxes[:, 1] + 1.0
    ctr_x = boxes[:, 0] + 0.5 * widths
    ctr_y = boxes[:, 1] + 0.5 * heights
    wx, wy, ww, wh = weights
    dx = deltas[:, 0::4] / wx
    dy = deltas[:, 1::4] / wy
    dw = np.minimum(deltas[:, 2::4] / ww, clip)
    dh = np.minimum(deltas[:, 3::4] / wh, clip)
    pred_ctr_x = dx * widths[:, None] + ctr_x[:, None]
    pred_ctr_y = dy * heights[:, None] + ctr_y[:, None]
    pred_w = np.maximum(np.exp(dw) * widths[:, None], 1.0)
    pred_h = np.maximum(np.exp(dh) * heights[:, None], 1.0)
    out = np.zeros(deltas.shape, dtype=deltas.dtype)
    out[:, 0::4] = pred_ctr_x - 0.5 * pred_w
    out[:, 1::4] = pred_ctr_y - 0.5 * pred_h
    out[:, 2::4] = pred_ctr_x + 0.5 * pred_w - 1
    out[:, 3::4] = pred_ctr_y + 0.5 * pred_h - 1
    return out


def clip_tiled_boxes(boxes, im_shape):
    """lib/utils/boxes.py:138-153 (in place, returns boxes)."""
    boxes[:, 0::4] = np.maximum(np.minimum(boxes[:, 0::4], im_shape[1] - 1), 0)
    boxes[:, 1::4] = np.maximum(np.minimum(boxes[:, 1::4], im_shape[0] - 1), 0)
    boxes[:, 2::4] = np.maximum(np.minimum(boxes[:, 2::4], im_shape[1] - 1), 0)
    boxes[:, 3::4] = np.maximum(np.minimum(boxes[:, 3::4], im_shape[0] - 1), 0)
    return boxes


def filter_boxes(boxes, min_size, im_info):
    """lib/modeling/generate_proposals.py:171-182."""
    min_size = min_size * im_info[2]
    ws = boxes[:, 2] - boxes[:, 0] + 1
    hs = boxes[:, 3] - boxes[:, 1] + 1
    x_ctr = boxes[:, 0] + ws / 2.
    y_ctr = boxes[:, 1] + hs / 2.
    return np.where((ws >= min_size) & (hs >= min_size) &
                    (x_ctr < im_info[1]) & (y_ctr < im_info[0]))[0]


def shifted_anchors(anchors, feat_stride, height, width):
    """generate_proposals.py:69-89: (K*A, 4) float64, rows ordered (h, w, a)."""
    sx = np.arange(0, width) * feat_stride
    sy = np.arange(0, height) * feat_stride
    sx, sy = np.meshgrid(sx, sy, copy=False)
    shifts = np.vstack((sx.ravel(), sy.ravel(), sx.ravel(), sy.ravel())).transpose()
    A, K = anchors.shape[0], shifts.shape[0]
    return (anchors[None, :, :] + shifts[:, None, :]).reshape((K * A, 4))


def proposals_for_one_image(im_info, all_anchors, bbox_deltas, scores,
                            pre_nms_topN, post_nms_topN, nms_thresh, min_size):
    """generate_proposals.py:104-168 (stable top-k reading)."""
    bbox_deltas = bbox_deltas.transpose((1, 2, 0)).reshape((-1, 4))
    scores = scores.transpose((1, 2, 0)).reshape((-1, 1))
    order = np.argsort(-scores.squeeze(axis=1), kind="stable")
    if not (pre_nms_topN <= 0 or pre_nms_topN >= len(scores)):
        order = order[:pre_nms_topN]
    bbox_deltas = bbox_deltas[order, :]
    all_anchors = all_anchors[order, :]
    scores = scores[order]
    proposals = bbox_transform(all_anchors, bbox_deltas, (1.0, 1.0, 1.0, 1.0))
    proposals = clip_tiled_boxes(proposals, im_info[:2])
    keep = filter_boxes(proposals, min_size, im_info)
    proposals = proposals[keep, :]
    scores = scores[keep]
    if nms_thresh > 0:
        keep = nms(np.hstack((proposals, scores)), nms_thresh)
        if post_nms_topN > 0:
            keep = keep[:post_nms_topN]
        proposals = proposals[keep, :]
        scores = scores[keep]
    return proposals, scores


def generate_proposals(anchors, spatial_scale, cls_prob, bbox_pred, im_info,
                       pre_nms_topN=1000, post_nms_topN=1000, nms_thresh=0.7, min_size=0):
    """GenerateProposalsOp.forward (generate_proposals.py:20-102) on ndarrays."""
    scores = np.asarray(cls_prob, np.float32)
    deltas = np.asarray(bbox_pred, np.float32)
    im_info = np.asarray(im_info, np.float32)
    height, width = scores.shape[-2:]
    all_anchors = shifted_anchors(anchors, 1. / spatial_scale, height, width)
    rois = np.empty((0, 5), np.float32)
    probs = np.empty((0, 1), np.float32)
    for i in range(scores.shape[0]):
        b, p = proposals_for_one_image(im_info[i, :], all_anchors, deltas[i], scores[i],
                                       pre_nms_topN, post_nms_topN, nms_thresh, min_size)
        bi = i * np.ones((b.shape[0], 1), dtype=np.float32)
        rois = np.append(rois, np.hstack((bi, b)), axis=0)
        probs = np.append(probs, p, axis=0)
    return rois, probs


def collect(roi_list, score_list, post_nms_topN=1000):
    """collect_and_distribute_fpn_rpn_proposals.py:91-106 (stable)."""
    rois = np.concatenate(roi_list)
    scores = np.concatenate(score_list).squeeze(axis=1)
    inds = np.argsort(-scores, kind="stable")[:post_nms_topN]
    return rois[inds, :]


def map_rois_to_fpn_levels(rois, k_min, k_max, s0=224, lvl0=4):
    """lib/utils/fpn.py:11-28 (float32 arithmetic as numpy evaluates it)."""
    w = rois[:, 2] - rois[:, 0] + 1
    h = rois[:, 3] - rois[:, 1] + 1
    areas = w * h
    areas[areas < 0] = 0
    s = np.sqrt(areas)
    lv = np.floor(lvl0 + np.log2(s / s0 + 1e-6))
    return np.clip(lv, k_min, k_max)


def distribute(rois, lvl_min=2, lvl_max=5, prefix="rois"):
    """distribute() (collect_and_distribute...py:109-138) / add_multilevel_roi_blobs
    (lib/utils/fpn.py:31-58): per-level rois + int32 restore index."""
    lvls = map_rois_to_fpn_levels(rois[:, 1:5], lvl_min, lvl_max)
    out = {prefix: rois}
    order = np.empty((0,))
    for lvl in range(lvl_min, lvl_max + 1):
        idx = np.where(lvls == lvl)[0]
        out[prefix + "_fpn" + str(lvl)] = rois[idx, :]
        order = np.concatenate((order, idx))
    out[prefix + "_idx_restore_int32"] = np.argsort(order, kind="stable").astype(np.int32)
    return out


def roi_feature_transform(blobs_in, rpn_ret, blob_rois, resolution, spatial_scales,
                          sampling_ratio, k_min=2, k_max=5):
    """Generalized_RCNN.roi_feature_transform, RoIAlign FPN branch
    (lib/modeling/model_builder.py:252-303): blobs_in coarsest first."""
    outs = []
    for lvl in range(k_min, k_max + 1):
        bl = blobs_in[k_max - lvl]
        sc = spatial_scales[k_max - lvl]
        r = rpn_ret[blob_rois + "_fpn" + str(lvl)]
        if len(r):
            outs.append(roi_align(bl, r, resolution, resolution, sc, sampling_ratio))
    sh = np.concatenate(outs, axis=0)
    return sh[rpn_ret[blob_rois + "_idx_restore_int32"].astype(np.int64)]


# --------------------------------------------------------------------------- #
# Detection post-processing                                                    #
# --------------------------------------------------------------------------- #
def bb_iou_vos(a, b):
    """lib_vos/tools/vos_test.py:961-982 bb_intersection_over_union on float32 box
    rows as numpy 2 evaluates it: every product / sum in float32 (Python ints and
    the float() of a float32 are weak scalars), the division float32 too."""
    a = [np.float32(v) for v in a[:4]]
    b = [np.float32(v) for v in b[:4]]
    xA, yA = max(a[0], b[0]), max(a[1], b[1])
    xB, yB = min(a[2], b[2]), min(a[3], b[3])
    inter = max(0, xB - xA + 1) * max(0, yB - yA + 1)
    area_a = (a[2] - a[0] + 1) * (a[3] - a[1] + 1)
    area_b = (b[2] - b[0] + 1) * (b[3] - b[1] + 1)
    return inter / float(area_a + area_b - inter)


def small_box_filter(cls_boxes, prev_cls_boxes, iou_thresh, score_thresh):
    """lib_vos/tools/vos_test.py:845-860 (TEST.NMS_SMALL_BOX_IOU > 0): for every
    class j whose previous-frame result holds exactly one box (the reference
    asserts < 2) with score >= score_thresh, drop this frame's class-j boxes whose
    IoU with it is below iou_thresh; order kept."""
    if prev_cls_boxes is None:
        return cls_boxes
    for j in range(1, len(cls_boxes)):
        pj = prev_cls_boxes[j] if j < len(prev_cls_boxes) else []
        assert len(pj) < 2, "number of prev boxes should <2."
        if len(pj) != 1 or pj[0][-1] < score_thresh:
            continue
        keep = [k for k in range(len(cls_boxes[j]))
                if not bb_iou_vos(pj[0], cls_boxes[j][k]) < iou_thresh]
        cls_boxes[j] = cls_boxes[j][keep, :] if len(cls_boxes[j]) else cls_boxes[j]
    return cls_boxes


def nms_with_mask_iou(dets, classes, masks, iou_th, max_per_class):
    """lib_vos/tools/vos_test.py:985-1029 on a frame's detections in cls_boxes
    (class-major) order: dets [n,5], classes [n], masks [n,H,W] binary (the
    decoded segms).  Processing order = score descending (np.argsort(-s), read
    stably); position j is discarded by an earlier kept position i when
    inter / (|m_i| + 1e-6) > iou_th or inter / (|m_j| + 1e-6) > iou_th (float64,
    as numpy divides its integer sums); the kept detections are appended to
    their class while it holds fewer than max_per_class.  Returns the kept input
    indices in the reference's output order (class ascending, then append order)."""
    n = len(dets)
    if n == 0:
        return np.zeros(0, np.int64)
    order = np.argsort(-np.asarray(dets)[:, -1], kind="stable")
    m = np.asarray(masks).reshape(n, -1).astype(bool)[order]
    area = m.sum(1).astype(np.int64)
    discard = np.zeros(n, bool)
    for i in range(n):
        if discard[i]:
            continue
        inter = (m[i + 1:] & m[i]).sum(1).astype(np.int64)
        iou1 = inter / (area[i] + 1e-6)
        iou2 = inter / (area[i + 1:] + 1e-6)
        discard[i + 1:] |= (iou1 > iou_th) | (iou2 > iou_th)
    kept = order[~discard]
    per = {}
    out = []
    for k in kept:
        c = int(classes[k])
        if per.get(c, 0) < max_per_class:
            per[c] = per.get(c, 0) + 1
            out.append(k)
    out = sorted(out, key=lambda k: (int(classes[k]), out.index(k)))
    return np.asarray(out, np.int64)


def _cy_area(x1, y1, x2, y2):
    """(x2 - x1 + 1) * (y2 - y1 + 1) on C floats as the compiled .pyx evaluates it:
    Cython 3 emits the literal 1 as 1.0, so each side is (double)(x2 - x1) + 1.0,
    the product in double, rounded to float on assignment."""
    f, d = np.float32, np.float64
    return f((d(f(x2 - x1)) + 1.0) * (d(f(y2 - y1)) + 1.0))


def _cy_iou(a, b, area_b):
    """iw / ih / ua / ov of cython_nms.soft_nms (:166-171) and cython_bbox
    (bbox_overlaps) for float32 boxes a (the kept / top box) and b: 0 when they
    do not overlap (iw or ih <= 0)."""
    f, d = np.float32, np.float64
    iw = f(d(f(min(a[2], b[2]) - max(a[0], b[0]))) + 1.0)
    if not iw > 0:
        return None
    ih = f(d(f(min(a[3], b[3]) - max(a[1], b[1]))) + 1.0)
    if not ih > 0:
        return None
    ua = f((d(f(a[2] - a[0])) + 1.0) * (d(f(a[3] - a[1])) + 1.0) + d(area_b) - d(f(iw * ih)))
    return f(f(iw * ih) / ua)


def soft_nms(dets, sigma=0.5, overlap_thresh=0.3, score_thresh=0.001, method="linear"):
    """lib/utils/boxes.py:336-355 -> cython_nms.soft_nms (lib/utils/cython_nms.pyx:
    98-203) as compiled here (Cython 3, see _cy_area): repeatedly move the
    highest remaining score (first maximum by position) to the front, decay the
    scores of the boxes after it that overlap it (linear: 1 - ov when ov > Nt;
    gaussian: exp(-ov^2 / sigma) in double, stored as float; hard: 0 when
    ov > Nt), and drop a decayed box whose score falls below score_thresh by
    moving the last box into its place.  Returns (dets [N,5] float32, inds)."""
    f = np.float32
    if len(dets) == 0:
        return dets, []
    meth = {"hard": 0, "linear": 1, "gaussian": 2}[method]
    b = np.array(dets, np.float32)
    sigma, Nt, thr = f(sigma), f(overlap_thresh), f(score_thresh)
    N = len(b)
    inds = np.arange(N)
    for i in range(len(b)):  # range() is evaluated once; the iterations i >= N are no-ops
        if i >= N:
            break
        mp = i + int(np.argmax(b[i:N, 4]))  # `maxscore < s`: the first maximum
        b[[i, mp]] = b[[mp, i]]
        inds[[i, mp]] = inds[[mp, i]]
        t = b[i].copy()
        pos = i + 1
        while pos < N:
            x = b[pos]
            ov = _cy_iou(t, x, _cy_area(x[0], x[1], x[2], x[3]))
            if ov is not None:
                if meth == 1:
                    w = f(1) - ov if ov > Nt else f(1)
                elif meth == 2:
                    w = f(np.exp(np.float64(f(-(ov * ov)) / sigma)))
                else:
                    w = f(0) if ov > Nt else f(1)
                b[pos, 4] = f(w * b[pos, 4])
                if b[pos, 4] < thr:
                    b[pos] = b[N - 1]
                    inds[pos] = inds[N - 1]
                    N -= 1
                    pos -= 1
            pos += 1
    return b[:N], inds[:N]


def np_pairwise_sum_f32(x):
    """numpy's float32 add-reduce along a contiguous axis (loops_utils.h
    pairwise_sum: < 8 sequential; <= 128 eight strided accumulators combined
    ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the tail; else halves split at a
    multiple of 8), after the reduction's initial 0."""
    f = np.float32
    x = [f(v) for v in x]

    def pw(a):
        n = len(a)
        if n < 8:
            r = f(0)
            for v in a:
                r = f(r + v)
            return r
        if n <= 128:
            r = list(a[:8])
            i = 8
            while i < n - n % 8:
                for k in range(8):
                    r[k] = f(r[k] + a[i + k])
                i += 8
            res = f(f(f(r[0] + r[1]) + f(r[2] + r[3])) + f(f(r[4] + r[5]) + f(r[6] + r[7])))
            for v in a[i:]:
                res = f(res + v)
            return res
        n2 = n // 2
        n2 -= n2 % 8
        return f(pw(a[:n2]) + pw(a[n2:]))
    return f(f(0) + pw(x))


def box_voting(top_dets, all_dets, thresh, scoring_method="ID", beta=1.0):
    """lib/utils/boxes.py:277-333 on float32 rows: the voters of top box k are
    the rows of all_dets with bbox_overlaps (cython_bbox, float32; _cy_iou) >=
    thresh, in row order; the box becomes np.average(voters, weights=scores)
    = (sequential float32 sum of box * w down the rows) / (pairwise float32 sum
    of w).  Scores: ID keeps it; AVG = mean(w); IOU_AVG = np.average(w,
    weights=overlaps) (both sums pairwise along the 1-D axis); QUASI_SUM =
    sum(w) / float(n) ** beta; GENERALIZED_AVG at beta == 1 is AVG.  TEMP_AVG
    (float32 log / exp of numpy's SIMD library) is not restated."""
    f = np.float32
    out = np.array(top_dets, np.float32)
    a = np.asarray(all_dets, np.float32)
    areas = [_cy_area(*r[:4]) for r in a]
    for k in range(len(out)):
        t = out[k].copy()
        vi, vo = [], []
        for i in range(len(a)):
            ov = _cy_iou(t, a[i], areas[i])
            ov = f(0) if ov is None else ov
            if ov >= f(thresh):
                vi.append(i)
                vo.append(ov)
        ws = [a[i, 4] for i in vi]
        scl = np_pairwise_sum_f32(ws)
        for c in range(4):
            acc = f(0)
            for i, w in zip(vi, ws):
                acc = f(acc + f(a[i, c] * w))
            out[k, c] = f(acc / scl)
        n = len(ws)
        if scoring_method == "ID":
            pass
        elif scoring_method == "AVG" or (scoring_method == "GENERALIZED_AVG" and beta == 1.0):
            out[k, 4] = f(scl / f(n))
        elif scoring_method == "IOU_AVG":
            out[k, 4] = f(np_pairwise_sum_f32([f(w * o) for w, o in zip(ws, vo)])
                          / np_pairwise_sum_f32(vo))
        elif scoring_method == "QUASI_SUM":
            out[k, 4] = f(scl / f(float(n) ** beta))
        else:
            raise NotImplementedError(scoring_method)
    return out


def box_results_with_nms_and_limit(scores, boxes, num_classes=81, score_thresh=0.05,
                                   nms_thresh=0.5, dets_per_im=100, nms_cross_class=0.,
                                   num_det_per_class_pre=0, prev_cls_boxes=None,
                                   small_box_iou=0., small_box_score_thresh=0.,
                                   soft_nms_method=None, soft_nms_sigma=0.5,
                                   bbox_vote=None, bbox_vote_th=0.8, bbox_vote_beta=1.0):
    """lib/core/test.py:733-797 with the fork's NUM_DET_PER_CLASS fix and its
    post-limit steps (lib_vos/tools/vos_test.py:748-865): TEST.NMS_CROSS_CLASS
    (:810-827), TEST.NUM_DET_PER_CLASS_PRE (:829-833; np.argsort(-s) read
    stably, kind="stable") and TEST.NMS_SMALL_BOX_IOU against the previous
    frame's result (:845-860, small_box_filter).  TEST.SOFT_NMS (soft_nms_method
    'hard' / 'linear' / 'gaussian', score_thresh 0.0001, test.py:756-763) and
    TEST.BBOX_VOTE (bbox_vote = the scoring method, test.py:769-776)."""
    cls_boxes = [[] for _ in range(num_classes)]
    for j in range(1, num_classes):
        inds = np.where(scores[:, j] >= score_thresh)[0]
        sj = scores[inds, j]
        bj = boxes[inds, j * 4:(j + 1) * 4]
        dj = np.hstack((bj, sj[:, None])).astype(np.float32, copy=False)
        if soft_nms_method is not None:
            nms_dets, _ = soft_nms(dj, soft_nms_sigma, nms_thresh, 0.0001, soft_nms_method)
        else:
            nms_dets = dj[nms(dj, nms_thresh), :]
        if bbox_vote is not None and len(nms_dets):
            nms_dets = box_voting(nms_dets, dj, bbox_vote_th, bbox_vote, bbox_vote_beta)
        cls_boxes[j] = nms_dets
    if dets_per_im > 0:
        image_scores = np.hstack([cls_boxes[j][:, -1] for j in range(1, num_classes)])
        if len(image_scores) > dets_per_im:
            thr = np.sort(image_scores)[-dets_per_im]
            for j in range(1, num_classes):
                keep = np.where(cls_boxes[j][:, -1] >= thr)[0]
                cls_boxes[j] = cls_boxes[j][keep, :]
    if nms_cross_class > 0.:
        all_dets = np.vstack([cls_boxes[j] for j in range(1, num_classes)])
        class_ids = np.vstack([np.ones(shape=(len(cls_boxes[j]), 1)) * j
                               for j in range(1, num_classes)])
        keep = nms(all_dets, nms_cross_class)
        all_dets, class_ids = all_dets[keep, :], class_ids[keep, :]
        for j in range(1, num_classes):
            cls_boxes[j] = all_dets[np.where(class_ids == j)[0], :]
    if num_det_per_class_pre > 0:
        for j in range(1, num_classes):
            keep = np.argsort(-cls_boxes[j][:, -1], kind="stable")[:num_det_per_class_pre]
            cls_boxes[j] = cls_boxes[j][keep, :]
    if small_box_iou > 0:
        cls_boxes = small_box_filter(cls_boxes, prev_cls_boxes, small_box_iou,
                                     small_box_score_thresh)
    im_results = np.vstack([cls_boxes[j] for j in range(1, num_classes)])
    return im_results[:, -1], im_results[:, :-1], cls_boxes


def cv2_resize_fx(src, fx, fy=None):
    """cv2.resize(src, None, None, fx=fx, fy=fy, interpolation=INTER_LINEAR) for an
    H x W x C float32 image, restating OpenCV's scalar float path: dsize =
    (round(W*fx), round(H*fy)) (saturate_cast<int>, half to even), scale = 1/fx
    (cv::resize keeps inv_scale = fx when dsize is derived from it), coefficient
    tables and the horizontal-then-vertical passes as cv2_resize_linear.
    cv2 is not importable here: parity against an executed cv2 is unpinned."""
    fy = fx if fy is None else fy
    src = np.asarray(src, np.float32)
    sh, sw = src.shape[:2]
    w, h = int(round(sw * fx)), int(round(sh * fy))
    scale_x, scale_y = 1. / fx, 1. / fy
    if scale_x == 2.0 and scale_y == 2.0:
        return _area2(src, h, w)
    dx = np.arange(w)
    fxs = ((dx + 0.5) * scale_x - 0.5).astype(np.float32)
    sx = np.floor(fxs).astype(np.int64)
    fxs = (fxs - sx.astype(np.float32)).astype(np.float32)
    lo = sx < 0
    fxs[lo], sx[lo] = 0, 0
    hi = sx >= sw - 1
    fxs[hi], sx[hi] = 0, sw - 1
    a0, a1 = (np.float32(1) - fxs).astype(np.float32), fxs
    sx1 = np.minimum(sx + 1, sw - 1)
    ex = (slice(None),) + (None,) * (src.ndim - 2)
    D = src[:, sx] * a0[ex] + src[:, sx1] * a1[ex]  # HResizeLinear, every source row
    dy = np.arange(h)
    fys = ((dy + 0.5) * scale_y - 0.5).astype(np.float32)
    sy = np.floor(fys).astype(np.int64)
    fys = (fys - sy.astype(np.float32)).astype(np.float32)
    r0, r1 = np.clip(sy, 0, sh - 1), np.clip(sy + 1, 0, sh - 1)
    b0, b1 = (np.float32(1) - fys).astype(np.float32), fys
    ey = (slice(None),) + (None,) * (src.ndim - 1)
    return (D[r0] * b0[ey] + D[r1] * b1[ey]).astype(np.float32)  # VResizeLinear


def target_scale(im_size_min, im_size_max, target_size, max_size):
    """lib/utils/blob.py:153-160 get_target_scale."""
    scale = float(target_size) / float(im_size_min)
    if np.round(scale * im_size_max) > max_size:
        scale = float(max_size) / float(im_size_max)
    return scale


def get_image_blob(im, target_scale=800, max_size=1333, stride=32):
    """lib/utils/blob.py:37-161: prep_im_for_blob (mean subtraction, then the
    INTER_LINEAR resize restated by cv2_resize_fx when the scale is not 1) and
    im_list_to_blob's zero padding to `stride` (1 = no padding, as without FPN)."""
    im = im.astype(np.float32, copy=False) - PIXEL_MEANS
    im = im.astype(np.float32)
    smin, smax = min(im.shape[:2]), max(im.shape[:2])
    scale = float(target_scale) / float(smin)
    if np.round(scale * smax) > max_size:
        scale = float(max_size) / float(smax)
    if scale != 1.0:
        im = cv2_resize_fx(im, scale)
    H = int(np.ceil(im.shape[0] / stride) * stride)
    W = int(np.ceil(im.shape[1] / stride) * stride)
    blob = np.zeros((1, H, W, 3), np.float32)
    blob[0, :im.shape[0], :im.shape[1], :] = im
    blob = blob.transpose(0, 3, 1, 2)
    im_info = np.array([[H, W, scale]], np.float32)
    return blob, scale, im_info


# --------------------------------------------------------------------------- #
# segm_results (lib/core/test.py:801-855).  cv2 and pycocotools are absent
# here, so the two third-party steps are restated from their published
# algorithms -- "parity unpinned" against an executed cv2/pycocotools:
#   * cv2.resize(src_f32, (w, h)) INTER_LINEAR, OpenCV's scalar float path
#     (imgproc/src/resize.cpp: coefficient tables of cv::resize, HResizeLinear,
#     VResizeLinear); IPP/SIMD builds may round differently;
#   * pycocotools mask.encode (maskApi.c rleEncode + rleToString).
# --------------------------------------------------------------------------- #
def expand_boxes(boxes, scale):
    """lib/utils/boxes.py:242-258 (float32 inputs stay float32 in numpy 2)."""
    w_half = (boxes[:, 2] - boxes[:, 0]) * .5
    h_half = (boxes[:, 3] - boxes[:, 1]) * .5
    x_c = (boxes[:, 2] + boxes[:, 0]) * .5
    y_c = (boxes[:, 3] + boxes[:, 1]) * .5
    w_half *= scale
    h_half *= scale
    boxes_exp = np.zeros(boxes.shape)
    boxes_exp[:, 0] = x_c - w_half
    boxes_exp[:, 2] = x_c + w_half
    boxes_exp[:, 1] = y_c - h_half
    boxes_exp[:, 3] = y_c + h_half
    return boxes_exp


def _area2(src, h, w):
    """OpenCV's resize dispatch runs INTER_AREA's fast path for INTER_LINEAR when
    both scales are exactly 2: each output is the mean of its 2 x 2 source block,
    summed ((a + b) + c) + d in float and times 0.25f (a partial block at an odd
    edge: the sum of the taps inside / their count).  Restated from OpenCV's
    resize.cpp as published; cv2 absent here, so unpinned."""
    src = np.asarray(src, np.float32)
    sh, sw = src.shape[:2]
    out = np.zeros((h, w) + src.shape[2:], np.float32)
    fh, fw = min(h, sh // 2), min(w, sw // 2)  # blocks entirely inside the image
    a, b = src[0:2 * fh:2, 0:2 * fw:2], src[0:2 * fh:2, 1:2 * fw:2]
    c, d = src[1:2 * fh:2, 0:2 * fw:2], src[1:2 * fh:2, 1:2 * fw:2]
    out[:fh, :fw] = (((a + b) + c) + d) * np.float32(0.25)
    for y in range(h):  # partial blocks at odd edges
        for x in range(w):
            if y < fh and x < fw:
                continue
            taps = [src[2 * y + dy, 2 * x + dx] for dy in (0, 1) for dx in (0, 1)
                    if 2 * y + dy < sh and 2 * x + dx < sw]
            acc = np.zeros(src.shape[2:], np.float32)
            for t in taps:
                acc = (acc + t).astype(np.float32)
            out[y, x] = acc / np.float32(len(taps))
    return out


def cv2_resize_linear(src, w, h):
    """cv2.resize(src, (w, h)) for a single-channel float32 image, INTER_LINEAR."""
    src = np.asarray(src, np.float32)
    sh, sw = src.shape
    scale_x = 1. / (float(w) / sw)
    scale_y = 1. / (float(h) / sh)
    if scale_x == 2.0 and scale_y == 2.0:
        return _area2(src, h, w)
    dx = np.arange(w)
    fx = ((dx + 0.5) * scale_x - 0.5).astype(np.float32)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx.astype(np.float32)).astype(np.float32)
    lo = sx < 0
    fx[lo], sx[lo] = 0, 0
    hi = sx >= sw - 1
    fx[hi], sx[hi] = 0, sw - 1
    a0, a1 = (np.float32(1) - fx).astype(np.float32), fx
    sx1 = np.minimum(sx + 1, sw - 1)
    D = src[:, sx] * a0 + src[:, sx1] * a1  # HResizeLinear, every source row
    dy = np.arange(h)
    fy = ((dy + 0.5) * scale_y - 0.5).astype(np.float32)
    sy = np.floor(fy).astype(np.int64)
    fy = (fy - sy.astype(np.float32)).astype(np.float32)
    r0, r1 = np.clip(sy, 0, sh - 1), np.clip(sy + 1, 0, sh - 1)
    b0, b1 = (np.float32(1) - fy).astype(np.float32), fy
    return (D[r0] * b0[:, None] + D[r1] * b1[:, None]).astype(np.float32)  # VResizeLinear


def paste_masks(masks, boxes, im_h, im_w, thresh=0.5):
    """segm_results' per-detection loop (test.py:808-835) up to im_mask:
    masks [M,R,R] class-selected, boxes [M,>=4] float32 -> [M,im_h,im_w] u8."""
    M = masks.shape[-1]
    scale = (M + 2.0) / M
    ref_boxes = expand_boxes(np.asarray(boxes, np.float32)[:, :4], scale).astype(np.int32)
    padded = np.zeros((M + 2, M + 2), dtype=np.float32)
    out = np.zeros((len(masks), im_h, im_w), np.uint8)
    for i in range(len(masks)):
        padded[1:-1, 1:-1] = masks[i]
        rb = ref_boxes[i]
        w = max(rb[2] - rb[0] + 1, 1)
        h = max(rb[3] - rb[1] + 1, 1)
        mask = np.array(cv2_resize_linear(padded, w, h) > thresh, dtype=np.uint8)
        x_0, x_1 = max(rb[0], 0), min(rb[2] + 1, im_w)
        y_0, y_1 = max(rb[1], 0), min(rb[3] + 1, im_h)
        out[i, y_0:y_1, x_0:x_1] = mask[(y_0 - rb[1]):(y_1 - rb[1]), (x_0 - rb[0]):(x_1 - rb[0])]
    return out


def rle_to_string(cnts):
    """pycocotools maskApi.c rleToString: each count after the second
    delta-coded against cnts[i-2] (signed), 5 bits per char low bits first,
    0x20 = more, + 48; stops at 0 (or -1 with the sign bit 0x10 set)."""
    s = []
    for i in range(len(cnts)):
        x = int(cnts[i]) - (int(cnts[i - 2]) if i > 2 else 0)
        while True:
            c = x & 0x1f
            x >>= 5
            more = x != -1 if c & 0x10 else x != 0
            s.append(chr((c | (0x20 if more else 0)) + 48))
            if not more:
                break
    return "".join(s)


def rle_encode(im_mask):
    """pycocotools mask.encode of one H x W u8 mask: {'size', 'counts' (str)}
    plus the raw run lengths (maskApi.c rleEncode over Fortran order)."""
    flat = np.asarray(im_mask, np.uint8).flatten(order="F")
    change = np.flatnonzero(np.diff(np.concatenate([[0], flat])) != 0)
    bounds = np.concatenate([[0], change, [flat.size]])
    cnts = np.diff(bounds).astype(np.int64)
    return ({"size": [int(im_mask.shape[0]), int(im_mask.shape[1])],
             "counts": rle_to_string(cnts)}, cnts)
