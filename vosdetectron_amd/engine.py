"""Device-resident per-frame inference engine (the hot path).

Replaces the host-driven chain of lib/core/test.py im_detect_all (:50-111):
im_detect_bbox (:128-190) -> box_results_with_nms_and_limit (:733-797) ->
im_detect_mask (:366-402), for a batch of F frames already resident in HBM:

  u8 frames --vd_image_to_blob--> blob --PyTorch ResNet-FPN--> P2..P6
  --PyTorch RPN convs--> vd_generate_proposals (all levels, all frames)
  --> vd_collect_distribute --> vd_roi_align_fpn (one launch, NHWC pyramid)
  --> PyTorch fc6/fc7/cls/bbox --> vd_box_detections (decode, clip, class NMS,
  top-100) --> vd_mask_rois (mask batch of F x DETECTIONS_PER_IM rows from the
  device counts) --> vd_roi_align_fpn 14x14 --> PyTorch mask head -->
  class-selected 28x28.

The reference crosses host<->device 5+5 times in proposals alone and twice per
roi_feature_transform; here nothing inside the step reads the host: the
detection counts are read once after the step is queued (complete()).  Outputs match the reference's
`cls_boxes` rows (class-major, proposal order) and the class-selected masks
that segm_results consumes; `frame_segms` runs segm_results' paste + RLE on
the device (segm.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import ops


class StageTimer:
    """utils/timer.Timer's accounting (total_time, calls, average_time) fed with
    HIP-event stage times instead of time.time() tic/toc."""

    def __init__(self, name: str):
        self.name = name
        self.total_time = 0.
        self.calls = 0
        self.average_time = 0.

    def add(self, seconds: float):
        self.total_time += seconds
        self.calls += 1
        self.average_time = self.total_time / self.calls


def nms_options(cfg) -> dict:
    """TEST.SOFT_NMS / TEST.BBOX_VOTE (lib/core/test.py:756-776) as box_detections
    keywords (empty when both are off: the stock vd_box_detections).  The
    reference never passes TEST.BBOX_VOTE.SCORING_METHOD_BETA to box_voting
    (test.py:770-775, vos_test.py:786-791), so beta stays 1.0 here too."""
    tst = cfg.TEST
    opts = {}
    if tst.SOFT_NMS.ENABLED:
        opts.update(soft_nms=tst.SOFT_NMS.METHOD, soft_nms_sigma=tst.SOFT_NMS.SIGMA)
    if tst.BBOX_VOTE.ENABLED:
        opts.update(bbox_vote=tst.BBOX_VOTE.SCORING_METHOD,
                    bbox_vote_thresh=tst.BBOX_VOTE.VOTE_TH,
                    bbox_vote_beta=1.0)
    return opts


class FramePipeline:
    ASYNC = True  # run(sync=False) queues a step with no host read (see run())
    def __init__(self, model, cfg, frame_hw=(800, 1333), batch=1, channels_last=False,
                 det_cap=256, device="cuda"):
        self.model = model
        self.cfg = cfg
        self.F = batch
        self.H, self.W = frame_hw
        self.device = torch.device(device)
        self.channels_last = channels_last
        self.det_cap = det_cap
        self._nms_options = nms_options(cfg)
        # blob geometry (lib/utils/blob.py:37-161): get_target_scale, cv2.resize
        # to round(H*s) x round(W*s) (done on the device when s != 1), pad to
        # FPN.COARSEST_STRIDE (get_max_shape; the C4 pipeline does not pad)
        scale = ops.target_scale(self.H, self.W, cfg.TEST.SCALE, cfg.TEST.MAX_SIZE)
        self.im_scale = scale
        self.Hr, self.Wr = ops.resized_hw(self.H, self.W, scale)
        st = cfg.FPN.COARSEST_STRIDE
        self.Hp = int(math.ceil(self.Hr / st) * st)
        self.Wp = int(math.ceil(self.Wr / st) * st)
        self.lut = torch.from_numpy(ops.pixel_lut(cfg.PIXEL_MEANS)).to(self.device)
        F = batch
        self.im_info = torch.tensor([[self.Hp, self.Wp, scale]] * F, dtype=torch.float32,
                                    device=self.device)
        self.im_scale_t = torch.full((F,), scale, dtype=torch.float32, device=self.device)
        self.im_scale_d = torch.full((F,), scale, dtype=torch.float64, device=self.device)
        self.im_hw = torch.tensor([[self.H, self.W]] * F, dtype=torch.int32, device=self.device)
        if cfg.FPN.FPN_ON:
            k_min, k_max = cfg.FPN.RPN_MIN_LEVEL, cfg.FPN.RPN_MAX_LEVEL
            self.rpn_levels = list(range(k_min, k_max + 1))
            self.anchors = [getattr(model, "anchors_fpn%d" % l).to(self.device)
                            for l in self.rpn_levels]
            self.rpn_scales = [1. / 2 ** l for l in self.rpn_levels]
            self.roi_levels = list(range(cfg.FPN.ROI_MIN_LEVEL, cfg.FPN.ROI_MAX_LEVEL + 1))
            self.roi_scales = [1. / 2 ** l for l in self.roi_levels]
        self.timers = None  # enable_timers(): per-stage HIP-event timing
        self._marks = None

    # ------------------------------------------------------------------ #
    # tracing: the reference threads a defaultdict(Timer) through im_detect_all
    # (lib/core/test.py:62-107, utils/timer.py:11-35, wall clock); here each
    # stage boundary records a HIP event on the launch stream, so the stage
    # times are device times and timing never adds a synchronisation.
    def enable_timers(self, on: bool = True):
        self.timers = {} if on else None
        return self

    def _mark(self, name: str):
        if self._marks is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._marks.append((name, ev))

    def _collect_marks(self):
        marks, self._marks = self._marks, None
        if not marks:
            return
        marks[-1][1].synchronize()
        for (_, a), (name, b) in zip(marks[:-1], marks[1:]):
            t = self.timers.setdefault(name, StageTimer(name))
            t.add(a.elapsed_time(b) / 1e3)

    def timer_summary(self):
        """{stage: average seconds per call} (Timer.average_time of the reference)."""
        return {k: v.average_time for k, v in (self.timers or {}).items()}

    def make_blob(self, frames):
        """get_image_blob on the device: identity scale -> vd_image_to_blob, else
        vd_image_resize_to_blob (mean subtraction + INTER_LINEAR resize + pad)."""
        nhwc = self.channels_last
        if self.im_scale == 1.0:
            blob = ops.image_to_blob(frames, self.lut, self.Hp, self.Wp, nhwc=nhwc)
        else:
            blob = ops.image_resize_to_blob(frames, self.lut, self.im_scale, self.Hp, self.Wp,
                                            nhwc=nhwc)
        return blob.permute(0, 3, 1, 2) if nhwc else blob  # NCHW view

    def backbone(self, frames):
        return self.model.Conv_Body(self.make_blob(frames))  # [P6, P5, P4, P3, P2]

    def nhwc_pyramid(self, feats):
        """P2..P5 as B x H x W x C (a free view when the body ran channels_last)."""
        out = []
        for lvl in self.roi_levels:
            t = feats[len(feats) - 1 - (lvl - self.rpn_levels[0])]
            if t.is_contiguous(memory_format=torch.channels_last):
                out.append(t.permute(0, 2, 3, 1))
            else:
                out.append(ops.nchw_to_nhwc(t))
        return out

    @torch.no_grad()
    def run(self, frames: torch.Tensor, keep_intermediates: bool = False, sync: bool = True):
        """frames: F x H x W x 3 uint8 BGR on the device.  Returns a dict of device
        tensors: dets [F,cap,5] (x1,y1,x2,y2,score), classes [F,cap], counts [F],
        masks [M,28,28] for the M = sum(counts) detections in (frame, class,
        proposal) order, and counts_host.  sync=False queues the step without
        any host read (graph-capturable): masks then has mask_rows(F) rows of
        which the first M are real, and complete(out) later reads the counts and
        trims.  Stage marks (enable_timers): conv_body, proposals, box_head
        (together the reference's im_detect_bbox), misc_bbox, im_detect_mask."""
        if self.timers is not None:
            self._marks = []
            self._mark("start")
        try:
            return self._run(frames, keep_intermediates, sync)
        finally:
            if self.timers is not None:
                self._collect_marks()

    def _run(self, frames: torch.Tensor, keep_intermediates: bool = False, sync: bool = True):
        cfg = self.cfg
        F = frames.shape[0]
        feats = self.backbone(frames)
        self._mark("conv_body")
        # RPN heads on P2..P6 (finest first for the proposal kernel)
        probs, deltas = [], []
        for lvl in self.rpn_levels:
            t = feats[len(feats) - 1 - (lvl - self.rpn_levels[0])]
            p, d = self.model.RPN.level_outputs(t)
            probs.append(p.contiguous())
            deltas.append(d.contiguous())
        tst = cfg.TEST
        lrois, lprobs, lcnt = ops.generate_proposals(
            probs, deltas, self.anchors, self.rpn_scales, self.im_info[:F],
            tst.RPN_PRE_NMS_TOP_N, tst.RPN_POST_NMS_TOP_N, tst.RPN_NMS_THRESH, tst.RPN_MIN_SIZE)
        post = int(tst.RPN_POST_NMS_TOP_N * cfg.FPN.RPN_COLLECT_SCALE + 0.5)
        rois, rlvl, rcnt = ops.collect_distribute(lrois, lprobs, lcnt, post,
                                                  cfg.FPN.ROI_MIN_LEVEL, cfg.FPN.ROI_MAX_LEVEL)
        self._mark("proposals")
        pyr = self.nhwc_pyramid(feats)
        fr = cfg.FAST_RCNN
        flat_rois, flat_lvl = rois.view(-1, 5), rlvl.view(-1)
        fast = self.channels_last and getattr(self.model.Box_Head, "nhwc_ready", False)
        box_feat = ops.roi_align_fpn(pyr, self.roi_scales, flat_rois, flat_lvl,
                                     fr.ROI_XFORM_RESOLUTION, fr.ROI_XFORM_SAMPLING_RATIO,
                                     roi_order=ops.xcd_roi_order(flat_rois, flat_lvl),
                                     out_layout="nhwc" if fast else "nchw")
        x = self.model.Box_Head.mlp_nhwc(box_feat) if fast else self.model.Box_Head.mlp(box_feat)
        cls_prob, bbox_pred = self.model.Box_Outs(x)
        self._mark("box_head")
        K = cls_prob.shape[1]
        bbox_pred = self.model.Box_Outs.per_class_deltas(bbox_pred, K)
        dets, dcls, dcnt = ops.box_detections(
            rois, cls_prob.view(F, post, K), bbox_pred.view(F, post, 4 * K), rcnt,
            self.im_scale_t[:F], self.im_hw[:F], tst.SCORE_THRESH, tst.NMS,
            tst.DETECTIONS_PER_IM, cfg.MODEL.BBOX_REG_WEIGHTS, self.det_cap,
            nms_cross_class=tst.NMS_CROSS_CLASS, num_det_per_class_pre=tst.NUM_DET_PER_CLASS_PRE,
            **self._nms_options)
        self._post_detections(dets, dcls, dcnt)
        self._mark("misc_bbox")
        out = {"dets": dets, "classes": dcls, "counts": dcnt, "rois": rois, "roi_counts": rcnt,
               "cls_prob": cls_prob, "bbox_pred": bbox_pred}
        if keep_intermediates:  # for stage-wise parity tests
            out.update(feats=feats, rpn_probs=probs, rpn_deltas=deltas, pyramid=pyr)
        # the mask batch: F x DETECTIONS_PER_IM rows (padded to 64), built on the
        # device from the device counts -- no host read inside the step
        # (box_results_with_nms_and_limit keeps <= DETECTIONS_PER_IM per frame
        # barring exact score ties at the limit; complete() runs the rest)
        cap = self.mask_rows(F)
        mrois, mlvl, mcls, mtotal = ops.mask_rois(
            dets, dcls, dcnt, self.im_scale_d[:F], cap, cfg.FPN.ROI_MIN_LEVEL,
            cfg.FPN.ROI_MAX_LEVEL)
        out["masks"], out["mask_feat"] = self._mask_batch(pyr, mrois, mlvl, mcls, fast)
        out["mask_rois"], out["mask_total"] = mrois, mtotal
        # the pyramid stays referenced only until complete() (the rare overflow
        # batch reads it); complete() drops it so a kept result does not pin ~1.5 GB
        out["_pyr"], out["_fast"] = pyr, fast
        self._mark("im_detect_mask")
        if sync:
            self.complete(out)
        return out

    def _post_detections(self, dets, classes, counts):
        """Hook after box_results_with_nms_and_limit's device steps (the VOS loop
        adds its previous-frame filter)."""

    def mask_rows(self, F: int) -> int:
        """Rows of the step's mask batch: F x DETECTIONS_PER_IM, a multiple of 64
        (a handful of stable shapes for the convolution algorithm search)."""
        return -(-F * int(self.cfg.TEST.DETECTIONS_PER_IM) // 64) * 64

    def _mask_batch(self, pyr, mrois, mlvl, mcls, fast):
        """Mask RoIAlign + mask head + class-selected masks for a padded batch
        (padding rows are zero boxes whose outputs are never read)."""
        mc = self.cfg.MRCNN
        if fast and getattr(self.model.Mask_Head, "nhwc_ready", False):
            mfeat = ops.roi_align_fpn(pyr, self.roi_scales, mrois, mlvl, mc.ROI_XFORM_RESOLUTION,
                                      mc.ROI_XFORM_SAMPLING_RATIO, out_layout="nhwc")
            masks = self.model.Mask_Head.masks_nhwc(mfeat, self.model.Mask_Outs, mcls)
            return masks, mfeat.permute(0, 3, 1, 2)
        mfeat = ops.roi_align_fpn(pyr, self.roi_scales, mrois, mlvl, mc.ROI_XFORM_RESOLUTION,
                                  mc.ROI_XFORM_SAMPLING_RATIO)
        mh = self.model.Mask_Head.head(mfeat)
        return self.model.Mask_Outs.selected(mh, mcls), mfeat

    def complete(self, out: dict) -> dict:
        """The step's one host read, after everything is queued: the detection
        counts (failure / capacity checks), the masks of detections beyond the
        padded batch (exact score ties at DETECTIONS_PER_IM), and the outputs
        trimmed to the M = sum(counts) real detections.  Idempotent."""
        if "counts_host" in out:
            return out
        counts = out["counts"].cpu().tolist()
        ops.raise_on_failed_counts(counts)
        if max(counts, default=0) > self.det_cap:
            raise RuntimeError("detections exceed det_cap=%d: %s" % (self.det_cap, counts))
        M, cap = sum(counts), out["masks"].shape[0]
        if M > cap:  # rows [cap, M): a second, rare batch
            extra = -(-(M - cap) // 64) * 64
            F = len(counts)
            r2, l2, c2, _ = ops.mask_rois(out["dets"], out["classes"], out["counts"],
                                          self.im_scale_d[:F], extra, self.cfg.FPN.ROI_MIN_LEVEL,
                                          self.cfg.FPN.ROI_MAX_LEVEL, row0=cap)
            m2, f2 = self._mask_batch(out["_pyr"], r2, l2, c2, out["_fast"])
            out["masks"] = torch.cat([out["masks"], m2])
            out["mask_feat"] = torch.cat([out["mask_feat"], f2])
            out["mask_rois"] = torch.cat([out["mask_rois"], r2])
        out.pop("_pyr", None)
        out.pop("_fast", None)
        out["masks"] = out["masks"][:M]
        out["mask_feat"] = out["mask_feat"][:M]
        out["mask_rois"] = out["mask_rois"][:M]
        out["counts_host"] = counts
        return out


def frame_segms(pipe: FramePipeline, out: dict, num_classes: int = 81):
    """segm_results for every frame of a pipeline output: one fused paste + RLE
    launch and one rleToString pass over all frames' detections
    (vosdetectron_amd/segm.py), then the per-frame class grouping.  Returns a
    list over frames of cls_segms."""
    from . import segm
    if isinstance(pipe, VOSPipeline) and pipe.heuristics_on():
        raise ValueError("frame_segms skips TEST.NMS_WITH_MASK_IOU / NMS_SMALL_BOX_IOU: use "
                         "VOSPipeline.frame_results for this config")
    ks = [int(k) for k in out["counts_host"]]
    total = sum(ks)
    if total == 0:
        return [[[] for _ in range(num_classes)] for _ in ks]
    boxes = torch.cat([out["dets"][f, :k] for f, k in enumerate(ks)])
    classes = torch.cat([out["classes"][f, :k] for f, k in enumerate(ks)]).cpu().tolist()
    rles = segm.encode_masks(out["masks"][:total], boxes, pipe.H, pipe.W,
                             pipe.cfg.MRCNN.THRESH_BINARIZE)
    res, start = [], 0
    for k in ks:
        res.append(segm.group_by_class(rles[start:start + k], classes[start:start + k],
                                       num_classes))
        start += k
    return res


class VOSPipeline(FramePipeline):
    """The VOS frame loop (lib_vos/tools/infer_davis_sequential.py:134-149 driving
    Generalized_VOS_RCNN._forward, vos_model_builder.py:289-447) for F sequences
    in lockstep: batch row b of every step is the next frame of sequence b, and
    the ConvGRU hidden states (one B x H x W x C tensor per level, in HBM) carry
    each sequence's state to its next frame.  `reset` starts new sequences
    (clean_hidden_states, :279-281)."""

    def __init__(self, model, cfg, frame_hw=(480, 854), batch=1, channels_last=False,
                 det_cap=256, device="cuda"):
        super().__init__(model, cfg, frame_hw, batch, channels_last, det_cap, device)
        self._flow = None
        # each sequence row's previous-frame result (prev_cls_boxes of the
        # reference loop, train_davis_online.py:591-592), for NMS_SMALL_BOX_IOU
        F = batch
        self.prev_dets = torch.zeros((F, det_cap, 5), dtype=torch.float32, device=self.device)
        self.prev_classes = torch.zeros((F, det_cap), dtype=torch.int32, device=self.device)
        self.prev_counts = torch.zeros((F,), dtype=torch.int32, device=self.device)
        # a step whose result frame_results has not yet recorded as the previous
        # frame (only tracked while a heuristic reads the previous result)
        self._unfinalized = False

    def heuristics_on(self) -> bool:
        """TEST.NMS_WITH_MASK_IOU / NMS_SMALL_BOX_IOU (vos_test.py:113-118, 845-860):
        both need frame_results, the step's mask-IoU NMS and the previous frame's
        final result."""
        tst = self.cfg.TEST
        return float(tst.NMS_WITH_MASK_IOU) > 0 or float(tst.NMS_SMALL_BOX_IOU) > 0

    def reset(self, rows=None):
        """Zero the hidden states (and forget the previous-frame results) of batch
        rows `rows` (all when None).  Resetting every row also drops the pending
        'unfinalized step' guard: no row's next frame reads that result any more."""
        if rows is None:
            self.prev_counts.zero_()
        else:
            self.prev_counts[list(rows)] = 0
        if rows is None or set(range(self.prev_counts.shape[0])) <= set(int(r) for r in rows):
            self._unfinalized = False
        hs = self.model.hidden_states
        if rows is None or all(h is None for h in hs):
            self.model.clean_hidden_states()
            return
        for h in hs:
            if h is not None:
                h[list(rows)] = 0

    def _post_detections(self, dets, classes, counts):
        """TEST.NMS_SMALL_BOX_IOU (lib_vos/tools/vos_test.py:845-860): each row's
        detections against its previous frame's final result, on the device.  Rows
        without a previous result (a new sequence) pass unchanged."""
        tst = self.cfg.TEST
        if float(tst.NMS_SMALL_BOX_IOU) > 0:
            F = dets.shape[0]
            ops.detections_prev_box_filter(dets, classes, counts, self.prev_dets[:F],
                                           self.prev_classes[:F], self.prev_counts[:F],
                                           tst.NMS_SMALL_BOX_IOU,
                                           tst.NMS_SMALL_BOX_SCORE_THRESHOLD)

    def frame_results(self, out: dict, num_classes: int = None):
        """The tail of the VOS im_detect_all (lib_vos/tools/vos_test.py:50-120) for
        every row of a completed step: segm_results, then nms_with_mask_iou when
        TEST.NMS_WITH_MASK_IOU > 0 (:113-118: masks pasted on the device, the mask
        IoU NMS and the per-class cap of NUM_DET_PER_CLASS_POST on the device).
        Returns a list over rows of (cls_boxes, cls_segms) -- cls_boxes[j] an
        [n_j, 5] float32 array -- and records each row's result as the previous
        frame of its sequence (prev_cls_boxes, for NMS_SMALL_BOX_IOU)."""
        from . import segm
        K = num_classes or int(self.cfg.MODEL.NUM_CLASSES)
        tst = self.cfg.TEST
        self.complete(out)
        self._unfinalized = False
        ks = [int(k) for k in out["counts_host"]]
        thr = self.cfg.MRCNN.THRESH_BINARIZE
        res, start = [], 0
        mask_nms = float(tst.NMS_WITH_MASK_IOU) > 0
        for f, k in enumerate(ks):
            dets = out["dets"][f, :k]
            classes = out["classes"][f, :k]
            masks = out["masks"][start:start + k]
            start += k
            rles = segm.encode_masks(masks, dets, self.H, self.W, thr)
            keep = torch.arange(k, device=self.device)
            if mask_nms and k:
                planes = ops.paste_masks(masks, dets, self.H, self.W, thr)
                keep = ops.mask_iou_nms(planes, dets, classes, float(tst.NMS_WITH_MASK_IOU),
                                        int(tst.NUM_DET_PER_CLASS_POST))
            kd, kc = dets[keep], classes[keep]
            n = kd.shape[0]
            self.prev_dets[f, :n] = kd
            self.prev_classes[f, :n] = kc
            self.prev_counts[f] = n
            kd_h, kc_h = kd.cpu().numpy(), kc.cpu().tolist()
            kept = keep.cpu().tolist()
            cls_boxes = [np.zeros((0, 5), np.float32) for _ in range(K)]
            cls_segms = [[] for _ in range(K)]
            for j in sorted(set(kc_h)):
                rows = [i for i, c in enumerate(kc_h) if c == j]
                cls_boxes[j] = kd_h[rows]
                cls_segms[j] = [rles[kept[i]] for i in rows]
            res.append((cls_boxes, cls_segms))
        return res

    def backbone(self, frames):
        feats = super().backbone(frames)
        return self.model.temporal_fusion(feats, self._flow)

    @torch.no_grad()
    def run(self, frames: torch.Tensor, flow: torch.Tensor = None, keep_intermediates=False,
            sync: bool = True):
        """frames: F x H x W x 3 u8 (frame t of each sequence); flow: optional
        F x 2 x Hp x Wp optical flow at blob resolution (flo_to_blob, data_flow);
        sync as FramePipeline.run (False: complete() reads the counts later).
        With TEST.NMS_WITH_MASK_IOU / NMS_SMALL_BOX_IOU on, every step's result
        must pass through frame_results before the next step runs (the filter
        reads the previous frame's final result): raises otherwise."""
        if self._unfinalized and self.heuristics_on():
            raise RuntimeError(
                "VOSPipeline.run: the previous step's result has not been through "
                "frame_results(); TEST.NMS_WITH_MASK_IOU / NMS_SMALL_BOX_IOU need it as the "
                "next frame's previous result (lib_vos/tools/vos_test.py:113-118, 845-860)")
        self._flow = flow
        try:
            out = super().run(frames, keep_intermediates, sync=sync)
        finally:
            self._flow = None
        self._unfinalized = True
        return out
