"""Shared GPU-engine parity checks (imported by the -m gpu test modules).

Stage-wise parity feeds each HIP stage the GPU's own upstream tensors and
compares it with the oracle on the same inputs (proposals and detections
bit-exact; RoIAlign within north_star's 1e-4); the e2e check matches the
engine's detections against the fully independent CPU pipeline
(oracle/pipeline.py: torch-CPU convolutions, numpy proposals, C RoIAlign/NMS)."""
import numpy as np
import torch

from oracle import oracle as orc

LEVEL_SCALES = [1. / 32, 1. / 16, 1. / 8, 1. / 4]  # blobs_in order [P5, P4, P3, P2]


def _nchw(mf, C):
    if mf.ndim == 4 and mf.shape[-1] == C and mf.shape[1] != C:
        return mf.transpose(0, 3, 1, 2)  # NHWC product layout
    return mf


def stagewise(cfg, pipe, out, frame, f=0):
    """Frame f of an engine output (run with keep_intermediates=True)."""
    from vosdetectron_amd import ops
    _, im_scale, im_info = orc.get_image_blob(frame, target_scale=cfg.TEST.SCALE,
                                              max_size=cfg.TEST.MAX_SIZE,
                                              stride=cfg.FPN.COARSEST_STRIDE)
    tst = cfg.TEST
    rl, pl = [], []
    for i, lvl in enumerate(range(cfg.FPN.RPN_MIN_LEVEL, cfg.FPN.RPN_MAX_LEVEL + 1)):
        p = out["rpn_probs"][i][f:f + 1].cpu().numpy()
        d = out["rpn_deltas"][i][f:f + 1].cpu().numpy()
        an = pipe.anchors[i].cpu().numpy()
        r, pr = orc.generate_proposals(an, 1. / 2 ** lvl, p, d, im_info,
                                       tst.RPN_PRE_NMS_TOP_N, tst.RPN_POST_NMS_TOP_N,
                                       tst.RPN_NMS_THRESH, tst.RPN_MIN_SIZE)
        rl.append(r)
        pl.append(pr)
    post = int(tst.RPN_POST_NMS_TOP_N * cfg.FPN.RPN_COLLECT_SCALE + 0.5)
    rois = orc.collect(rl, pl, post)
    n = int(out["roi_counts"][f].item())
    assert n == len(rois), (n, len(rois))
    rois_gpu = out["rois"][f, :n].cpu().numpy()
    assert np.array_equal(rois_gpu[:, 1:], rois[:, 1:])
    # box RoIAlign through the reference operator API on the GPU pyramid
    rpn_ret = orc.distribute(rois)
    blobs = [t[f:f + 1].cpu().numpy() for t in out["feats"][1:]]
    P, sr = cfg.FAST_RCNN.ROI_XFORM_RESOLUTION, cfg.FAST_RCNN.ROI_XFORM_SAMPLING_RATIO
    bf_ref = orc.roi_feature_transform(blobs, rpn_ret, "rois", P, LEVEL_SCALES, sr)
    pyr = [t[f:f + 1] for t in out["pyramid"]]
    lv = orc.map_rois_to_fpn_levels(rois[:, 1:5], 2, 5).astype(np.int32) - 2
    r0 = rois.copy()
    r0[:, 0] = 0
    got = ops.roi_align_fpn(pyr, pipe.roi_scales, torch.from_numpy(r0).to(pyr[0].device),
                            torch.from_numpy(lv).to(pyr[0].device), P, sr)
    np.testing.assert_allclose(got.cpu().numpy(), bf_ref, rtol=1e-4, atol=1e-4)
    # detections from the GPU's own head outputs
    K = cfg.MODEL.NUM_CLASSES
    sc = out["cls_prob"].view(-1, post, K)[f, :n].cpu().numpy()
    dl = out["bbox_pred"].view(-1, post, out["bbox_pred"].shape[-1])[f, :n].cpu().numpy()
    pred = orc.clip_tiled_boxes(orc.bbox_transform(rois[:, 1:5] / im_scale, dl,
                                                   tuple(cfg.MODEL.BBOX_REG_WEIGHTS)), frame.shape)
    s_ref, b_ref, _ = orc.box_results_with_nms_and_limit(
        sc, pred, K, tst.SCORE_THRESH, tst.NMS, tst.DETECTIONS_PER_IM,
        nms_cross_class=tst.NMS_CROSS_CLASS, num_det_per_class_pre=tst.NUM_DET_PER_CLASS_PRE)
    k = out["counts_host"][f]
    assert k == len(s_ref)
    dets = out["dets"][f, :k].cpu().numpy()
    assert np.array_equal(dets[:, :4], b_ref) and np.array_equal(dets[:, 4], s_ref)
    # mask RoIAlign from the GPU detections
    o = int(sum(out["counts_host"][:f]))
    mrois = out["mask_rois"][o:o + k].cpu().numpy().copy()
    mrois[:, 0] = 0
    mret = orc.distribute(mrois, prefix="mask_rois")
    mc = cfg.MRCNN
    mf_ref = orc.roi_feature_transform(blobs, mret, "mask_rois", mc.ROI_XFORM_RESOLUTION,
                                       LEVEL_SCALES, mc.ROI_XFORM_SAMPLING_RATIO)
    mf = _nchw(out["mask_feat"][o:o + k].cpu().numpy(), mf_ref.shape[1])
    np.testing.assert_allclose(mf, mf_ref, rtol=1e-4, atol=1e-4)
    return rois, blobs


def match(gd, gc, gm, sc, bx, cl, masks, iou_min=0.95):
    """Detections matched by class + IoU; max |mask diff| of each matched pair."""
    matched, mask_err = 0, []
    for i in range(len(sc)):
        same = np.where(gc == cl[i])[0]
        if not len(same):
            continue
        b = gd[same, :4]
        xx1 = np.maximum(b[:, 0], bx[i, 0]); yy1 = np.maximum(b[:, 1], bx[i, 1])
        xx2 = np.minimum(b[:, 2], bx[i, 2]); yy2 = np.minimum(b[:, 3], bx[i, 3])
        inter = np.maximum(0, xx2 - xx1 + 1) * np.maximum(0, yy2 - yy1 + 1)
        a1 = (b[:, 2] - b[:, 0] + 1) * (b[:, 3] - b[:, 1] + 1)
        a2 = (bx[i, 2] - bx[i, 0] + 1) * (bx[i, 3] - bx[i, 1] + 1)
        iou = inter / (a1 + a2 - inter)
        j = int(np.argmax(iou))
        if iou[j] > iou_min:
            matched += 1
            mask_err.append(np.abs(gm[same[j]] - masks[i]).max())
    return matched, mask_err


def e2e_vs_cpu(out, ref_out, f=0, count_tol=0.02, match_min=0.98, mask_tol=1e-3):
    """Frame f of the GPU engine vs the independent CPU pipeline: detection
    counts within 2 % (>= 2), >= 98 % of the CPU detections matched by class and
    IoU > 0.95, median max-|mask diff| of the matched pairs < 1e-3.  The two
    pipelines' convolutions (MIOpen / hand-written MFMA vs oneDNN, folded vs
    unfolded AffineChannel) round differently, so a detection whose score sits
    at the 0.05 threshold or the 100th place can flip; everything else must
    agree (the stage-wise checks hold each HIP stage bit-exact / 1e-4)."""
    sc, bx, cl, masks, _ = ref_out
    k = out["counts_host"][f]
    o = int(sum(out["counts_host"][:f]))
    gd = out["dets"][f, :k].cpu().numpy()
    gc = out["classes"][f, :k].cpu().numpy()
    gm = out["masks"][o:o + k].cpu().numpy()
    assert abs(k - len(sc)) <= max(2, count_tol * len(sc)), (k, len(sc))
    matched, mask_err = match(gd, gc, gm, sc, bx, cl, masks)
    assert matched >= match_min * len(sc), (matched, len(sc))
    assert np.median(mask_err) < mask_tol, np.median(mask_err)
    print("e2e frame %d: %d/%d CPU detections matched, GPU count %d, median mask err %.2e"
          % (f, matched, len(sc), k, float(np.median(mask_err))))
    return matched
