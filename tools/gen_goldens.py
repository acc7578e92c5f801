#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by importing the REFERENCE's
own Python (read-only, from /root/reference) in this container.

Only data (inputs + expected outputs) is written; no reference source is copied.
Runs here only -- /root/reference does not exist on the GPU box; the committed
.npz fixtures travel instead.

Runtime-only import shims (nothing under /root/reference is modified):
  * ``np.float`` / ``np.int`` aliases (removed in numpy >= 1.24; used by
    generate_anchors.py:63,72, core/test.py:904-905);
  * ``torch._six`` stub (lib/nn/parallel/scatter_gather.py:7);
  * ``utils.cython_nms``: the REFERENCE's own ``lib/utils/cython_nms.pyx``,
    compiled by tools/ref_cython_nms.py from a /tmp scratch copy with the
    two-token dtype substitution of SURVEY Appendix A (``np.int_t`` ->
    ``np.intp_t``, ``dtype=np.int)`` -> ``dtype=np.intp)``: the same 64-bit
    integer on Linux; numpy 2's .pxd dropped the old spelling).  Every fixture
    that runs through NMS (proposals, C4 proposals, collect/distribute, the
    fork's post-filter) therefore runs the executed reference NMS, and
    ``nms.npz`` pins it directly.  ``utils.cython_bbox``: the reference's own
    ``lib/utils/cython_bbox.pyx``, compiled unmodified the same way (box voting).
  * ``cv2`` / ``pycocotools`` stubs (imported at module level by core/test.py,
    never called on the functions used here; vos_post.npz's mask-IoU NMS gets a
    decode / encode stub that carries binary masks, see gen_vos_post_fixture);
  * ``np.delete`` accepting an integral float64 index array (vos_test.py:1011,
    what numpy of the reference's era did), for vos_post.npz only.

Usage: python tools/gen_goldens.py   (writes tests/golden/*.npz)
       python tools/gen_goldens.py vos_post   (only tests/golden/vos_post.npz)
       python tools/gen_goldens.py soft_nms   (only tests/golden/soft_nms.npz)
"""
import os
import sys
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)


def install_shims():
    np.float = float
    np.int = int
    sys.path.insert(0, os.path.join(REF, "lib"))
    six_mod = types.ModuleType("torch._six")
    six_mod.string_classes = (str, bytes)
    six_mod.int_classes = int
    sys.modules["torch._six"] = six_mod
    import torch.utils.data.dataloader as dl
    if not hasattr(dl, "numpy_type_map"):
        dl.numpy_type_map = {}
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from ref_cython_nms import load as load_ref_nms, load_bbox
    sys.modules["utils.cython_nms"] = load_ref_nms()
    sys.modules["utils.cython_bbox"] = load_bbox()  # box voting's bbox_overlaps
    cv2 = types.ModuleType("cv2")
    cv2.INTER_LINEAR = 1
    sys.modules["cv2"] = cv2
    class _Stub(types.ModuleType):
        def __getattr__(self, attr):  # any attribute: an inert placeholder
            if attr.startswith("__"):
                raise AttributeError(attr)
            return type(attr, (), {})
    for name in ("pycocotools", "pycocotools.mask", "pycocotools.coco",
                 "pycocotools.cocoeval", "scipy.misc", "imdb", "imdb.vos",
                 "imdb.vos.davis_db", "datasets.json_dataset"):
        sys.modules[name] = _Stub(name)
    sys.modules["imdb.vos"].davis_db = sys.modules["imdb.vos.davis_db"]
    import yaml
    _load = yaml.load
    yaml.load = lambda s, Loader=yaml.SafeLoader: _load(s, Loader=Loader)


def distinct_scores(rng, n):
    """Tie-free scores in (0, 1): a random permutation of n distinct float32s."""
    vals = np.linspace(0.001, 0.999, n, dtype=np.float64).astype(np.float32)
    vals = np.unique(vals)
    assert vals.size == n
    return rng.permutation(vals).astype(np.float32)


def main():
    install_shims()
    from core.config import cfg
    from modeling.generate_anchors import generate_anchors
    import utils.boxes as box_utils
    import utils.fpn as fpn_utils
    from modeling.generate_proposals import GenerateProposalsOp
    import modeling.collect_and_distribute_fpn_rpn_proposals as cdp

    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(20241015)

    # ---- anchors: reference output + the comment KAT (generate_anchors.py:26-51)
    kat_comment = np.array([[-83, -39, 100, 56], [-175, -87, 192, 104], [-359, -183, 376, 200],
                            [-55, -55, 72, 72], [-119, -119, 136, 136], [-247, -247, 264, 264],
                            [-35, -79, 52, 96], [-79, -167, 96, 184], [-167, -343, 184, 360]],
                           np.float64)
    kat_ref = generate_anchors(stride=16, sizes=(128, 256, 512), aspect_ratios=(0.5, 1, 2))
    lvl_anchors = {}
    for lvl in range(2, 7):
        lvl_anchors["fpn%d" % lvl] = generate_anchors(
            stride=2. ** lvl, sizes=(32 * 2. ** (lvl - 2),), aspect_ratios=(0.5, 1, 2))
    np.savez(os.path.join(OUT, "anchors.npz"), kat_comment=kat_comment, kat_ref=kat_ref,
             **lvl_anchors)

    # ---- bbox_transform + clip_tiled_boxes (boxes.py:138-205)
    N = 512
    xy = rng.uniform(-50, 1300, (N, 2))
    wh = rng.uniform(0.5, 400, (N, 2))
    boxes = np.hstack([xy, xy + wh]).astype(np.float32)
    deltas1 = rng.normal(0, 1.0, (N, 4)).astype(np.float32)
    deltas1[:8, 2:] = 9.0  # exercise BBOX_XFORM_CLIP
    deltas81 = rng.normal(0, 2.0, (128, 4 * 81)).astype(np.float32)
    cfg.immutable(False) if hasattr(cfg, "immutable") else None
    out1 = box_utils.bbox_transform(boxes.astype(np.float64), deltas1, (1.0, 1.0, 1.0, 1.0))
    out81 = box_utils.bbox_transform(boxes[:128], deltas81, (10., 10., 5., 5.))
    im_info = np.array([800, 1344, 1.0], np.float32)
    clip1 = box_utils.clip_tiled_boxes(out1.copy(), im_info[:2])
    clip81 = box_utils.clip_tiled_boxes(out81.copy(), (800, 1333, 3))
    np.savez(os.path.join(OUT, "bbox_transform.npz"), boxes=boxes, deltas1=deltas1,
             deltas81=deltas81, out1=out1, out81=out81, clip1=clip1, clip81=clip81)

    # ---- map_rois_to_fpn_levels (utils/fpn.py:11-28), incl. near-boundary sizes
    s = np.concatenate([np.exp(rng.uniform(np.log(4), np.log(1400), 2000)),
                        224. * 2. ** np.arange(-3, 3) - 1, 224. * 2. ** np.arange(-3, 3)])
    a = np.exp(rng.uniform(np.log(0.5), np.log(2), s.size))
    w, h = s / np.sqrt(a), s * np.sqrt(a)
    cx, cy = rng.uniform(0, 1333, s.size), rng.uniform(0, 800, s.size)
    lv_boxes = np.stack([cx - w / 2, cy - h / 2, cx + w / 2 - 1, cy + h / 2 - 1], 1).astype(np.float32)
    square = np.array(224. * 2. ** np.arange(-3, 3), np.float32)
    sq = np.stack([np.zeros_like(square), np.zeros_like(square), square - 1, square - 1], 1)
    lv_boxes = np.concatenate([lv_boxes, sq]).astype(np.float32)
    lvls = fpn_utils.map_rois_to_fpn_levels(lv_boxes, 2, 5)
    np.savez(os.path.join(OUT, "fpn_levels.npz"), boxes=lv_boxes, lvls=lvls)

    # ---- GenerateProposalsOp per FPN level (generate_proposals.py:20-168)
    cfg.TEST.RPN_PRE_NMS_TOP_N = 1000
    cfg.TEST.RPN_POST_NMS_TOP_N = 1000
    cfg.TEST.RPN_NMS_THRESH = 0.7
    cfg.TEST.RPN_MIN_SIZE = 0
    prop = {}
    im_info = np.array([[800, 1344, 1.0]], np.float32)
    shapes = {2: (100, 168), 3: (50, 84), 4: (25, 42), 5: (13, 21), 6: (7, 11)}
    per_level_rois, per_level_probs = [], []
    # one pool of distinct values so scores are tie-free across levels too
    total = sum(3 * H * W for (H, W) in shapes.values())
    pool, used = distinct_scores(rng, total), 0
    for lvl, (H, W) in shapes.items():
        anchors = generate_anchors(stride=2. ** lvl, sizes=(32 * 2. ** (lvl - 2),),
                                   aspect_ratios=(0.5, 1, 2))
        A = anchors.shape[0]
        probs = pool[used:used + A * H * W].reshape(1, A, H, W)
        used += A * H * W
        deltas = rng.normal(0, 0.3, (1, 4 * A, H, W)).astype(np.float32)
        op = GenerateProposalsOp(anchors, 1. / 2 ** lvl)
        op.eval()
        import torch
        rois, rprobs = op(torch.from_numpy(probs), torch.from_numpy(deltas), torch.from_numpy(im_info))
        prop["probs_fpn%d" % lvl] = probs
        prop["deltas_fpn%d" % lvl] = deltas
        prop["rois_fpn%d" % lvl] = rois
        prop["roi_probs_fpn%d" % lvl] = rprobs
        per_level_rois.append(rois)
        per_level_probs.append(rprobs)
    prop["im_info"] = im_info
    np.savez(os.path.join(OUT, "proposals.npz"), **prop)

    # ---- collect + distribute (collect_and_distribute...py:91-138)
    cfg.FPN.RPN_COLLECT_SCALE = 1
    cfg.FPN.RPN_MIN_LEVEL, cfg.FPN.RPN_MAX_LEVEL = 2, 6
    cfg.FPN.ROI_MIN_LEVEL, cfg.FPN.ROI_MAX_LEVEL = 2, 5
    cfg.FPN.FPN_ON = True
    cfg.FPN.MULTILEVEL_ROIS = True
    cfg.MODEL.KEYPOINTS_ON = False
    cfg.MODEL.MASK_ON = False
    # collect() needs the score inputs tie-free across levels too
    rois_c = cdp.collect(per_level_rois + per_level_probs, False)
    dist = cdp.distribute(rois_c, None)
    np.savez(os.path.join(OUT, "collect_distribute.npz"), collected=rois_c,
             **{k: np.asarray(v) for k, v in dist.items()})

    # ---- add_multilevel_roi_blobs (mask rois path, utils/fpn.py:31-58)
    blobs = {}
    mrois = np.hstack([np.zeros((100, 1), np.float32), lv_boxes[:100]]).astype(np.float32)
    lv = fpn_utils.map_rois_to_fpn_levels(mrois[:, 1:5], 2, 5)
    fpn_utils.add_multilevel_roi_blobs(blobs, "mask_rois", mrois, lv, 2, 5)
    np.savez(os.path.join(OUT, "multilevel_mask_rois.npz"), mask_rois=mrois,
             **{k: np.asarray(v) for k, v in blobs.items()})

    # ---- single-scale C4 RPN (rpn_heads.single_scale_rpn_outputs, :38-55 and
    # GenerateProposalsOp with e2e_mask_rcnn_R-50-C4_1x.yaml TEST pre/post
    # 6000/1000): 15 anchors at stride 16 on a 50x84 res4 map
    rng4 = np.random.default_rng(20241016)
    cfg.TEST.RPN_PRE_NMS_TOP_N = 6000
    cfg.TEST.RPN_POST_NMS_TOP_N = 1000
    anchors = generate_anchors(stride=16, sizes=(32, 64, 128, 256, 512),
                               aspect_ratios=(0.5, 1, 2))
    A, H, W = anchors.shape[0], 50, 84
    probs = distinct_scores(rng4, A * H * W).reshape(1, A, H, W)
    deltas = rng4.normal(0, 0.3, (1, 4 * A, H, W)).astype(np.float32)
    op = GenerateProposalsOp(anchors, 1. / 16)
    op.eval()
    import torch
    rois, rprobs = op(torch.from_numpy(probs), torch.from_numpy(deltas), torch.from_numpy(im_info))
    np.savez(os.path.join(OUT, "proposals_c4.npz"), anchors=anchors, probs=probs, deltas=deltas,
             rois=rois, roi_probs=rprobs, im_info=im_info, pre_nms=6000, post_nms=1000)
    cfg.TEST.RPN_PRE_NMS_TOP_N = 1000

    # ---- the fork's box_results_with_nms_and_limit post-limit steps
    # (lib_vos/tools/vos_test.py:748-865): TEST.NMS_CROSS_CLASS and
    # TEST.NUM_DET_PER_CLASS_PRE, executed by the reference module itself
    sys.path.insert(0, os.path.join(REF, "lib_vos", "tools"))
    import vos_test
    rng5 = np.random.default_rng(20241017)
    R, K = 400, 81
    xy = rng5.uniform(0, 700, (R, 2))
    wh = rng5.uniform(8, 200, (R, 2))
    base = np.hstack([xy, xy + wh])
    jitter = rng5.normal(0, 6, (R, 4 * K))
    boxes_cls = (np.tile(base, K) + jitter).astype(np.float32)
    logits = rng5.normal(0, 2.5, (R, K))
    e = np.exp(logits - logits.max(1, keepdims=True))
    scores = (e / e.sum(1, keepdims=True)).astype(np.float32)  # continuous: tie-free
    cfg.MODEL.NUM_CLASSES = K  # reference default -1
    cfg.TEST.SCORE_THRESH, cfg.TEST.NMS, cfg.TEST.DETECTIONS_PER_IM = 0.05, 0.5, 100
    cfg.TEST.SOFT_NMS.ENABLED, cfg.TEST.BBOX_VOTE.ENABLED = False, False
    cfg.TEST.NMS_SMALL_BOX_IOU = 0.
    post = {"scores": scores, "boxes": boxes_cls}
    for tag, cross, pre in (("cross04_pre2", 0.4, 2), ("cross0_pre50", 0., 50),
                            ("cross06_pre0", 0.6, 0), ("cross0_pre0", 0., 0)):
        cfg.TEST.NMS_CROSS_CLASS, cfg.TEST.NUM_DET_PER_CLASS_PRE = cross, pre
        _, _, cls_b = vos_test.box_results_with_nms_and_limit(scores, boxes_cls)
        post[tag + "_dets"] = np.vstack([cls_b[j] for j in range(1, K)]).astype(np.float32)
        post[tag + "_cls"] = np.concatenate(
            [[j] * len(cls_b[j]) for j in range(1, K)]).astype(np.int32)
    cfg.TEST.NMS_CROSS_CLASS, cfg.TEST.NUM_DET_PER_CLASS_PRE = 0., 0
    np.savez(os.path.join(OUT, "detections_postfilter.npz"), **post)

    gen_nms_fixture(sys.modules["utils.cython_nms"])
    print("wrote", sorted(os.listdir(OUT)))


def _clustered_dets(rng, n, span=1300.):
    """RPN / class-NMS-like boxes: jittered copies around n/8+1 centres (heavy
    overlap) mixed with free boxes; 1-2 px boxes and exact duplicates included."""
    k = max(1, n // 8)
    centres = np.hstack([rng.uniform(0, span, (k, 2)), rng.uniform(4, 300, (k, 2))])
    pick = rng.integers(0, k, n)
    c = centres[pick]
    jit = rng.normal(0, 1, (n, 4)) * (0.08 * c[:, 2:4].repeat(2, 1))
    x1 = c[:, 0] - c[:, 2] / 2 + jit[:, 0]
    y1 = c[:, 1] - c[:, 3] / 2 + jit[:, 1]
    x2 = c[:, 0] + c[:, 2] / 2 + jit[:, 2]
    y2 = c[:, 1] + c[:, 3] / 2 + jit[:, 3]
    free = rng.uniform(0, 1, n) < 0.25
    fxy = rng.uniform(0, span, (n, 2))
    fwh = rng.uniform(0, 150, (n, 2))
    x1 = np.where(free, fxy[:, 0], x1)
    y1 = np.where(free, fxy[:, 1], y1)
    x2 = np.where(free, fxy[:, 0] + fwh[:, 0], np.maximum(x2, x1))
    y2 = np.where(free, fxy[:, 1] + fwh[:, 1], np.maximum(y2, y1))
    d = np.stack([x1, y1, x2, y2, np.zeros(n)], 1).astype(np.float32)
    if n >= 8:
        d[1] = d[0]                        # exact duplicate box
        d[2, 2:4] = d[2, 0:2]              # 1x1 box (+1 convention)
    return d


def gen_nms_fixture(cy):
    """tests/golden/nms.npz: the executed reference ``cython_nms.nms``
    (lib/utils/cython_nms.pyx:37-87) on
      * tie-free sets at N in {1, 64, 65, 1000, 4381, 5000} x thresh {0.3, 0.5, 0.7};
      * exact-threshold IoU pairs (IoU == fl32(thresh) suppresses, one ulp
        below does not) at each threshold;
      * tie-bearing sets (scores quantised to 1/8): the reference's keep AND its
        processing order ``scores.argsort()[::-1]`` as numpy computed it on the
        generating host.  Tie order is host-dependent (numpy's unstable SIMD
        argsort), so the tests pin the NMS given that
        order: rescoring the rows by their rank in ``order`` must reproduce
        ``keep`` bit for bit."""
    rng = np.random.default_rng(20261017)
    out, i = {}, 0
    for n in (1, 64, 65, 1000, 4381, 5000):
        for thr in (0.3, 0.5, 0.7):
            d = _clustered_dets(rng, n)
            d[:, 4] = distinct_scores(rng, n) if n > 1 else np.float32(0.5)
            out["dets_%d" % i] = d
            out["thresh_%d" % i] = np.float32(thr)
            out["keep_%d" % i] = np.asarray(cy.nms(d, np.float32(thr)), np.int64)
            out["kind_%d" % i] = np.array("tie_free")
            i += 1
    # exact-threshold pairs: a 10x10 box against 10 x h boxes inside it,
    # IoU = 10h / 100 exactly representable as fl32(h / 10)
    for thr, h in ((0.3, 3), (0.5, 5), (0.7, 7)):
        rows = [[0, 0, 9, 9, 0.9],
                [0, 0, 9, h - 1, 0.8],          # IoU == fl32(thr): suppressed
                [40, 0, 49, 9, 0.7],
                [40, 0, 49, h - 1 - 1e-3, 0.6],  # IoU a hair below: kept
                [80, 0, 89, 9, 0.5],
                [80, 0, 89, h - 1 + 1e-3, 0.4]]  # a hair above: suppressed
        d = np.array(rows, np.float32)
        out["dets_%d" % i] = d
        out["thresh_%d" % i] = np.float32(thr)
        out["keep_%d" % i] = np.asarray(cy.nms(d, np.float32(thr)), np.int64)
        out["kind_%d" % i] = np.array("exact_threshold")
        i += 1
    for n, thr in ((5, 0.5), (16, 0.5), (17, 0.7), (300, 0.3), (1000, 0.7), (3000, 0.5)):
        d = _clustered_dets(rng, n)
        d[:, 4] = np.round(rng.uniform(0, 1, n) * 8) / 8
        out["dets_%d" % i] = d
        out["thresh_%d" % i] = np.float32(thr)
        out["keep_%d" % i] = np.asarray(cy.nms(d, np.float32(thr)), np.int64)
        out["order_%d" % i] = d[:, 4].argsort()[::-1].astype(np.int64)
        out["kind_%d" % i] = np.array("ties")
        i += 1
    out["count"] = np.int64(i)
    np.savez_compressed(os.path.join(OUT, "nms.npz"), **out)


def _blob_mask(rng, H, W, box):
    """A filled ellipse / rectangle inside box (x1, y1, x2, y2) on an H x W frame."""
    m = np.zeros((H, W), np.uint8)
    x1, y1, x2, y2 = [int(round(v)) for v in box]
    x1, y1 = max(x1, 0), max(y1, 0)
    x2, y2 = min(x2, W - 1), min(y2, H - 1)
    if x2 < x1 or y2 < y1:
        return m
    if rng.uniform() < 0.5:
        m[y1:y2 + 1, x1:x2 + 1] = 1
    else:
        yy, xx = np.mgrid[0:H, 0:W]
        cy, cx = (y1 + y2) / 2, (x1 + x2) / 2
        ry, rx = max((y2 - y1) / 2, .5), max((x2 - x1) / 2, .5)
        m[((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1] = 1
    return m


def gen_vos_post_fixture():
    """tests/golden/vos_post.npz: the fork's two detection heuristics of the VOS
    frame loop, executed by the reference's own lib_vos/tools/vos_test.py:
      * nms_with_mask_iou (:985-1029; called at :113-118 when
        TEST.NMS_WITH_MASK_IOU > 0): masks decoded from the segms, greedy in
        score order discarding j when inter / |m_i| or inter / |m_j| > iou_th,
        then at most TEST.NUM_DET_PER_CLASS_POST per class.  pycocotools is
        absent: a runtime stub decodes a segm to the binary mask it carries and
        encodes a mask back to the index of the input mask it equals, so the
        fixture records which detections the reference keeps, in its order;
      * box_results_with_nms_and_limit(..., prev_cls_boxes) with
        TEST.NMS_SMALL_BOX_IOU > 0 (:845-860): a class's boxes whose IoU with the
        previous frame's (single, confident) box of that class is below the
        threshold are dropped, after the cross-class NMS and the per-class cap."""
    install_shims()
    from core.config import cfg
    sys.path.insert(0, os.path.join(REF, "lib_vos", "tools"))
    import vos_test
    rng = np.random.default_rng(20261018)
    out = {}
    # ---- nms_with_mask_iou
    H, W, K = 48, 64, 81
    cfg.MODEL.NUM_CLASSES = K
    masks_in = []

    class _MaskUtil:
        @staticmethod
        def decode(segms):
            return np.stack([sg["m"] for sg in segms], axis=2)

        @staticmethod
        def encode(arr):
            m = np.asarray(arr)[:, :, 0]
            idx = [i for i, mi in enumerate(masks_in) if np.array_equal(mi, m)]
            return [{"counts": str(idx[0]).encode("ascii"), "size": [H, W]}]
    vos_test.mask_util = _MaskUtil
    # nms_with_mask_iou collects discarded positions in np.array([]) (float64) and
    # passes it to np.delete (:999-1011), which numpy of the reference's era accepted
    # (integral floats as indices) and numpy 2 rejects: a runtime shim casts such an
    # index array to intp -- the positions the reference meant
    _np_delete = np.delete

    def _delete(arr, obj, axis=None):
        if isinstance(obj, np.ndarray) and obj.dtype.kind == "f":
            assert np.all(obj == np.round(obj))
            obj = obj.astype(np.intp)
        return _np_delete(arr, obj, axis)
    np.delete = _delete
    ci = 0
    for case, (n, iou_th, per_cls) in enumerate(((40, 0.5, 1), (40, 0.7, 2), (60, 0.9, 0),
                                                 (30, 1.0, 1), (50, 0.3, 3), (1, 0.5, 1))):
        classes = np.sort(rng.choice([1, 2, 3, 7, 15, 40, 80], n))
        centres = rng.uniform([4, 4], [W - 4, H - 4], (max(1, n // 3), 2))
        c = centres[rng.integers(0, len(centres), n)] + rng.normal(0, 3, (n, 2))
        wh = rng.uniform(3, 30, (n, 2))
        boxes = np.hstack([c - wh / 2, c + wh / 2]).astype(np.float32)
        scores = distinct_scores(rng, max(n, 2))[:n]
        masks = [_blob_mask(rng, H, W, b) for b in boxes]
        for i in range(1, n, 7):  # nested masks: a smaller copy inside another
            j = i - 1
            inner = masks[j].copy()
            ys, xs = np.nonzero(inner)
            if len(ys) > 4:
                inner[ys.min():ys.min() + (ys.max() - ys.min()) // 2 + 1] = 0
                masks[i] = inner
        if n > 5:
            masks[5] = np.zeros((H, W), np.uint8)  # an empty mask
        # no two input masks equal (the encode stub identifies masks by value)
        seen = []
        for i in range(n):
            while any(np.array_equal(masks[i], m) for m in seen):
                y, x = rng.integers(0, H), rng.integers(0, W)
                masks[i][y, x] ^= 1
            seen.append(masks[i])
        masks_in[:] = masks
        cls_boxes = [[] for _ in range(K)]
        cls_segms = [[] for _ in range(K)]
        for j in range(1, K):
            idx = np.where(classes == j)[0]
            if len(idx):
                cls_boxes[j] = np.hstack([boxes[idx], scores[idx, None]]).astype(np.float32)
                cls_segms[j] = [{"m": masks[i]} for i in idx]
        nb, ns = vos_test.nms_with_mask_iou(cls_boxes, cls_segms, iou_th=iou_th,
                                            max_per_class=per_cls)
        kept_idx, kept_cls, kept_box = [], [], []
        for j in range(K):
            for b, sg in zip(nb[j], ns[j]):
                kept_idx.append(int(sg["counts"]))
                kept_cls.append(j)
                kept_box.append(np.asarray(b, np.float32))
        out["mask_%d_classes" % case] = classes.astype(np.int32)
        out["mask_%d_dets" % case] = np.hstack([boxes, scores[:, None]]).astype(np.float32)
        out["mask_%d_masks" % case] = np.stack(masks).astype(np.uint8)
        out["mask_%d_iou_th" % case] = np.float64(iou_th)
        out["mask_%d_per_class" % case] = np.int32(per_cls)
        out["mask_%d_keep" % case] = np.asarray(kept_idx, np.int32)
        out["mask_%d_keep_cls" % case] = np.asarray(kept_cls, np.int32)
        out["mask_%d_keep_dets" % case] = (np.stack(kept_box) if kept_box
                                           else np.zeros((0, 5), np.float32))
        ci = case + 1
    out["mask_count"] = np.int32(ci)
    # ---- NMS_SMALL_BOX_IOU inside box_results_with_nms_and_limit
    R = 300
    xy = rng.uniform(0, 700, (R, 2))
    wh = rng.uniform(8, 200, (R, 2))
    base = np.hstack([xy, xy + wh])
    boxes_cls = (np.tile(base, K) + rng.normal(0, 6, (R, 4 * K))).astype(np.float32)
    logits = rng.normal(0, 2.5, (R, K))
    e = np.exp(logits - logits.max(1, keepdims=True))
    scores = (e / e.sum(1, keepdims=True)).astype(np.float32)
    cfg.TEST.SCORE_THRESH, cfg.TEST.NMS, cfg.TEST.DETECTIONS_PER_IM = 0.05, 0.5, 100
    cfg.TEST.SOFT_NMS.ENABLED, cfg.TEST.BBOX_VOTE.ENABLED = False, False
    out["small_scores"], out["small_boxes"] = scores, boxes_cls
    cases = ((0.3, 0.2, 0, 0.), (0.5, 0.2, 2, 0.), (0.1, 0.0, 0, 0.4), (0.7, 0.5, 1, 0.))
    for case, (iou, sthr, pre, cross) in enumerate(cases):
        cfg.TEST.NMS_SMALL_BOX_IOU = 0.
        cfg.TEST.NMS_CROSS_CLASS, cfg.TEST.NUM_DET_PER_CLASS_PRE = cross, pre
        _, _, cls_b = vos_test.box_results_with_nms_and_limit(scores, boxes_cls)
        prev = [[] for _ in range(K)]
        pd, pc = [], []
        for j in range(1, K):
            u = rng.uniform()
            if len(cls_b[j]) and u < 0.6:  # a jittered copy of one of this frame's boxes
                b = cls_b[j][rng.integers(0, len(cls_b[j]))][:4] + rng.normal(0, 25, 4)
            elif u < 0.7:  # a box anywhere
                p0 = rng.uniform(0, 700, 2)
                b = np.hstack([p0, p0 + rng.uniform(8, 200, 2)])
            else:
                continue
            row = np.hstack([b, rng.uniform(0, 1)]).astype(np.float32)
            prev[j] = row[None]
            pd.append(row)
            pc.append(j)
        cfg.TEST.NMS_SMALL_BOX_IOU = iou
        cfg.TEST.NMS_SMALL_BOX_SCORE_THRESHOLD = sthr
        _, _, cls_f = vos_test.box_results_with_nms_and_limit(scores, boxes_cls,
                                                             prev_cls_boxes=prev)
        out["small_%d_cfg" % case] = np.array([iou, sthr, pre, cross], np.float64)
        out["small_%d_prev_dets" % case] = np.asarray(pd, np.float32).reshape(-1, 5)
        out["small_%d_prev_cls" % case] = np.asarray(pc, np.int32)
        out["small_%d_dets" % case] = np.vstack(
            [cls_f[j] for j in range(1, K)]).astype(np.float32).reshape(-1, 5)
        out["small_%d_cls" % case] = np.concatenate(
            [[j] * len(cls_f[j]) for j in range(1, K)]).astype(np.int32)
        out["small_%d_unfiltered" % case] = np.int32(sum(len(cls_b[j]) for j in range(1, K)))
    out["small_count"] = np.int32(len(cases))
    cfg.TEST.NMS_SMALL_BOX_IOU, cfg.TEST.NMS_CROSS_CLASS, cfg.TEST.NUM_DET_PER_CLASS_PRE = 0., 0., 0
    np.savez_compressed(os.path.join(OUT, "vos_post.npz"), **out)
    print("wrote vos_post.npz:", {k: v.shape for k, v in out.items() if k.endswith(("keep", "_dets"))})


def gen_soft_nms_fixture():
    """tests/golden/soft_nms.npz: TEST.SOFT_NMS and TEST.BBOX_VOTE executed by the
    reference itself (lib/core/test.py:756-776):
      * soft_%d: utils/boxes.py soft_nms -> the compiled cython_nms.soft_nms
        (cython_nms.pyx:98-203) on clustered boxes with exact duplicates (scores
        decayed to 0 and removed), tied scores, N up to 1000, each method at
        overlap 0.3 / 0.5: output rows and keep indices;
      * vote_%d: utils/boxes.py box_voting (bbox_overlaps = the compiled
        cython_bbox.pyx) on the NMS / soft-NMS rows of a set, every scoring
        method this path builds, including a 400-box cluster (> 128 voters:
        numpy's pairwise summation splits);
      * det_%d: box_results_with_nms_and_limit (the fork's, lib_vos/tools/vos_test.py:
        748-865; core/test.py:789 reads TEST.NUM_DET_PER_CLASS, absent from the
        config) on decoded boxes
        (box_utils.bbox_transform + clip_tiled_boxes of rois / deltas, as
        im_detect_bbox does) with SOFT_NMS / BBOX_VOTE enabled."""
    install_shims()
    from core.config import cfg
    import utils.boxes as box_utils
    sys.path.insert(0, os.path.join(REF, "lib_vos", "tools"))
    import vos_test as ref_test  # the fork's box_results (core/test.py:789 names a missing key)
    rng = np.random.default_rng(20261019)
    out = {}
    i = 0
    for si, n in enumerate((1, 2, 9, 64, 300, 1000)):
        d = _clustered_dets(rng, n)
        d[:, 4] = distinct_scores(rng, n) if n > 1 else np.float32(0.5)
        if n >= 64:
            d[10:20, :4] = d[9, :4]                        # exact duplicates: ov = 1
            d[30:40, 4] = np.round(d[30:40, 4] * 4) / 4    # tied scores
        for method in ("hard", "linear", "gaussian"):
            for th in (0.3, 0.5):
                r, keep = box_utils.soft_nms(d, sigma=0.5, overlap_thresh=th,
                                             score_thresh=0.0001, method=method)
                out["soft_in_%d" % si] = d
                out["soft_%d_in" % i] = np.int64(si)
                out["soft_%d_cfg" % i] = np.array([["hard", "linear", "gaussian"].index(method),
                                                   th, 0.5], np.float64)
                out["soft_%d_out" % i] = np.asarray(r, np.float32)
                out["soft_%d_keep" % i] = np.asarray(keep, np.int64)
                i += 1
    out["soft_count"] = np.int64(i)
    # ---- box voting
    i = 0
    dense = np.array([[100, 100, 180, 160]], np.float64) + rng.normal(0, 1.0, (400, 4))
    dense = np.hstack([dense, distinct_scores(rng, 400)[:, None]]).astype(np.float32)
    sets = [("cluster300", _clustered_dets(rng, 300)), ("dense400", dense)]
    sets[0][1][:, 4] = distinct_scores(rng, 300)
    max_voters = 0
    ntop = 0
    for si, (name, d) in enumerate(sets):
        out["vote_set_%d" % si] = d
        tops = {"nms": d[box_utils.nms(d, 0.5), :],
                "soft": box_utils.soft_nms(d, 0.5, 0.3, 0.0001, "linear")[0]}
        for tname, top in tops.items():
            out["vote_top_%d" % ntop] = np.asarray(top, np.float32)
            ov = sys.modules["utils.cython_bbox"].bbox_overlaps(
                np.ascontiguousarray(top[:, :4]), np.ascontiguousarray(d[:, :4]))
            for vth in (0.5, 0.8, 0.95):
                max_voters = max(max_voters, int((ov >= np.float32(vth)).sum(1).max()))
                for sm, beta in (("ID", 1.0), ("AVG", 1.0), ("IOU_AVG", 1.0),
                                 ("QUASI_SUM", 1.0), ("QUASI_SUM", 2.0),
                                 ("GENERALIZED_AVG", 1.0)):
                    v = box_utils.box_voting(top, d, vth, scoring_method=sm, beta=beta)
                    out["vote_%d_sets" % i] = np.array([si, ntop], np.int64)
                    out["vote_%d_cfg" % i] = np.array([vth, beta], np.float64)
                    out["vote_%d_method" % i] = np.array(sm)
                    out["vote_%d_out" % i] = np.asarray(v, np.float32)
                    i += 1
            ntop += 1
    assert max_voters > 128, max_voters
    out["vote_count"] = np.int64(i)
    # ---- box_results_with_nms_and_limit with the options, on decoded boxes
    R, K, im_h, im_w = 300, 81, 480, 854
    xy = rng.uniform(0, 800, (R, 2))
    wh = rng.uniform(8, 200, (R, 2))
    rois = np.zeros((R, 5), np.float32)
    rois[:, 1:3] = xy
    rois[:, 3:5] = np.minimum(xy + wh, [im_w + 9, im_h - 1])
    logits = rng.normal(0, 2.5, (R, K))
    e = np.exp(logits - logits.max(1, keepdims=True))
    scores = (e / e.sum(1, keepdims=True)).astype(np.float32)
    deltas = rng.normal(0, 0.25, (R, 4 * K)).astype(np.float32)
    boxes = box_utils.bbox_transform(rois[:, 1:5], deltas, (10., 10., 5., 5.))
    boxes = box_utils.clip_tiled_boxes(boxes, (im_h, im_w, 3))
    out.update(det_rois=rois, det_scores=scores, det_deltas=deltas,
               det_im_hw=np.array([im_h, im_w], np.int32))
    cfg.MODEL.NUM_CLASSES = K
    cfg.TEST.SCORE_THRESH, cfg.TEST.NMS, cfg.TEST.DETECTIONS_PER_IM = 0.05, 0.5, 100
    i = 0
    for soft, vote, vth in ((None, None, 0.8), ("linear", None, 0.8), ("gaussian", None, 0.8),
                            ("hard", None, 0.8), (None, "ID", 0.8), (None, "IOU_AVG", 0.5),
                            ("linear", "AVG", 0.5), ("gaussian", "QUASI_SUM", 0.8)):
        cfg.TEST.SOFT_NMS.ENABLED = soft is not None
        cfg.TEST.SOFT_NMS.METHOD = soft or "linear"
        cfg.TEST.SOFT_NMS.SIGMA = 0.5
        cfg.TEST.BBOX_VOTE.ENABLED = vote is not None
        cfg.TEST.BBOX_VOTE.SCORING_METHOD = vote or "ID"
        cfg.TEST.BBOX_VOTE.VOTE_TH = vth
        _, _, cls_b = ref_test.box_results_with_nms_and_limit(scores, boxes)
        out["det_%d_cfg" % i] = np.array([str(soft), str(vote), str(vth)])
        out["det_%d_dets" % i] = np.vstack([cls_b[j] for j in range(1, K)]).astype(
            np.float32).reshape(-1, 5)
        out["det_%d_cls" % i] = np.concatenate(
            [[j] * len(cls_b[j]) for j in range(1, K)]).astype(np.int32)
        i += 1
    out["det_count"] = np.int64(i)
    cfg.TEST.SOFT_NMS.ENABLED, cfg.TEST.BBOX_VOTE.ENABLED = False, False
    np.savez_compressed(os.path.join(OUT, "soft_nms.npz"), **out)
    print("wrote soft_nms.npz: %d soft, %d vote, %d det cases, max voters %d"
          % (out["soft_count"], out["vote_count"], out["det_count"], max_voters))


if __name__ == "__main__":
    if sys.argv[1:] == ["vos_post"]:
        gen_vos_post_fixture()
    elif sys.argv[1:] == ["soft_nms"]:
        gen_soft_nms_fixture()
    else:
        main()
        gen_vos_post_fixture()
        gen_soft_nms_fixture()
