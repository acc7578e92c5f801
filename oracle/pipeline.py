"""oracle/pipeline.py -- TEST INFRASTRUCTURE ONLY.

The reference's pure-CPU per-frame path, restated: PyTorch-CPU convolutions in
the reference's module order (ResNet.py / FPN.py / fast_rcnn_heads.py /
mask_rcnn_heads.py, AffineChannel2d applied as y = x*w + b, nothing folded)
plus the oracle's numpy proposal path and C RoIAlign / NMS, driven the way
lib/core/test.py im_detect_all (:50-111) drives the model:

  get_image_blob -> Conv_Body -> per-level RPN + GenerateProposalsOp ->
  collect/distribute -> roi_feature_transform (box, 7x7) -> fc6/fc7/cls/bbox ->
  bbox_transform + clip -> box_results_with_nms_and_limit ->
  _add_multilevel_rois_for_test -> roi_feature_transform (mask, 14x14) ->
  mask head -> sigmoid (R x 81 x 28 x 28).

Used (a) as the e2e parity checker for the HIP engine and (b) by bench.py's
cpu_baseline leg.  It consumes a state_dict with the reference's parameter
names; it does not import the product package.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import oracle as orc


class RefCPUPipeline:
    def __init__(self, sd, block_counts=(3, 4, 6, 3), groups=1, num_classes=81,
                 pre_nms=1000, post_nms=1000, rpn_nms=0.7, test_nms=0.5, score_thresh=0.05,
                 dets_per_im=100, box_res=7, box_sr=2, mask_res=14, mask_sr=2, mask_dilation=1):
        self.sd = {k: v.detach().cpu().float() for k, v in sd.items()}
        self.block_counts = block_counts
        self.groups = groups
        self.K = num_classes
        self.pre_nms, self.post_nms, self.rpn_nms = pre_nms, post_nms, rpn_nms
        self.test_nms, self.score_thresh, self.dets_per_im = test_nms, score_thresh, dets_per_im
        self.box_res, self.box_sr = box_res, box_sr
        self.mask_res, self.mask_sr, self.mask_dil = mask_res, mask_sr, mask_dilation
        self.anchors = {l: orc.fpn_level_anchors(l) for l in range(2, 7)}

    # ---------------------------------------------------------------- body
    def _aff(self, x, p):
        return x * self.sd[p + ".weight"].view(1, -1, 1, 1) + self.sd[p + ".bias"].view(1, -1, 1, 1)

    def _conv(self, x, p, stride=1, padding=0, dilation=1, groups=1, bias=True):
        b = self.sd.get(p + ".bias") if bias else None
        return F.conv2d(x, self.sd[p + ".weight"], b, stride, padding, dilation, groups)

    def backbone(self, blob):
        s = self.sd
        pre = "Conv_Body.conv_body."
        x = self._conv(blob, pre + "res1.conv1", 2, 3, bias=False)
        x = F.relu(self._aff(x, pre + "res1.bn1"))
        x = F.max_pool2d(x, 3, 2, 1)
        outs = [x]
        for si, n in enumerate(self.block_counts):
            for b in range(n):
                p = pre + "res%d.%d." % (si + 2, b)
                stride = 2 if (b == 0 and si > 0) else 1
                o = F.relu(self._aff(self._conv(x, p + "conv1", stride, bias=False), p + "bn1"))
                o = F.relu(self._aff(self._conv(o, p + "conv2", 1, 1, groups=self.groups,
                                                bias=False), p + "bn2"))
                o = self._aff(self._conv(o, p + "conv3", bias=False), p + "bn3")
                if (p + "downsample.0.weight") in s:
                    r = self._aff(self._conv(x, p + "downsample.0", stride, bias=False),
                                  p + "downsample.1")
                else:
                    r = x
                x = F.relu(o + r)
            outs.append(x)
        c = outs  # res1..res5
        inner = [self._conv(c[-1], "Conv_Body.conv_top")]
        for i in range(3):
            lat = self._conv(c[-(i + 2)], "Conv_Body.topdown_lateral_modules.%d.conv_lateral" % i)
            inner.append(lat + F.interpolate(inner[-1], scale_factor=2, mode="nearest"))
        fpn = [self._conv(inner[i], "Conv_Body.posthoc_modules.%d" % i, 1, 1) for i in range(4)]
        fpn.insert(0, F.max_pool2d(fpn[0], 1, 2, 0))
        return fpn  # [P6, P5, P4, P3, P2]

    # ---------------------------------------------------------------- frame
    @torch.no_grad()
    def __call__(self, im_u8):
        """im_u8: H x W x 3 uint8 BGR.  Returns (scores, boxes, classes, masks, extra)."""
        blob, im_scale, im_info = orc.get_image_blob(im_u8)
        fpn = self.backbone(torch.from_numpy(blob))
        rois_l, probs_l = [], []
        extra = {"probs": {}, "deltas": {}}
        for lvl in range(2, 7):
            t = fpn[6 - lvl]
            h = F.relu(self._conv(t, "RPN.FPN_RPN_conv", 1, 1))
            cls = torch.sigmoid(self._conv(h, "RPN.FPN_RPN_cls_score")).numpy()
            dl = self._conv(h, "RPN.FPN_RPN_bbox_pred").numpy()
            extra["probs"][lvl], extra["deltas"][lvl] = cls, dl
            r, p = orc.generate_proposals(self.anchors[lvl], 1. / 2 ** lvl, cls, dl, im_info,
                                          self.pre_nms, self.post_nms, self.rpn_nms, 0)
            rois_l.append(r)
            probs_l.append(p)
        rois = orc.collect(rois_l, probs_l, self.post_nms)
        rpn_ret = orc.distribute(rois)
        blobs = [f.numpy() for f in fpn[1:]]  # [P5, P4, P3, P2]
        scales = [1. / 32, 1. / 16, 1. / 8, 1. / 4]
        bf = orc.roi_feature_transform(blobs, rpn_ret, "rois", self.box_res, scales, self.box_sr)
        x = torch.from_numpy(bf).reshape(bf.shape[0], -1)
        x = F.relu(F.linear(x, self.sd["Box_Head.fc1.weight"], self.sd["Box_Head.fc1.bias"]))
        x = F.relu(F.linear(x, self.sd["Box_Head.fc2.weight"], self.sd["Box_Head.fc2.bias"]))
        scores = F.softmax(F.linear(x, self.sd["Box_Outs.cls_score.weight"],
                                    self.sd["Box_Outs.cls_score.bias"]), dim=1).numpy()
        deltas = F.linear(x, self.sd["Box_Outs.bbox_pred.weight"],
                          self.sd["Box_Outs.bbox_pred.bias"]).numpy()
        boxes = rois[:, 1:5] / im_scale
        pred = orc.bbox_transform(boxes, deltas, (10., 10., 5., 5.))
        pred = orc.clip_tiled_boxes(pred, im_u8.shape)
        sc, bx, cls_boxes = orc.box_results_with_nms_and_limit(
            scores, pred, self.K, self.score_thresh, self.test_nms, self.dets_per_im)
        classes = np.concatenate([[j] * len(cls_boxes[j]) for j in range(1, self.K)] +
                                 [np.zeros((0,))]).astype(np.int32)
        extra.update(rois=rois, scores_all=scores, deltas_all=deltas)
        if bx.shape[0] == 0:
            return sc, bx, classes, np.zeros((0, 28, 28), np.float32), extra
        mrois = np.hstack([np.zeros((bx.shape[0], 1)), bx.astype(np.float64) * im_scale])
        mrois = mrois.astype(np.float32)
        mret = orc.distribute(mrois, prefix="mask_rois")
        mf = orc.roi_feature_transform(blobs, mret, "mask_rois", self.mask_res, scales,
                                       self.mask_sr)
        y = torch.from_numpy(mf)
        for i in range(4):
            y = F.relu(self._conv(y, "Mask_Head.conv_fcn.%d" % (2 * i), 1, self.mask_dil,
                                  self.mask_dil))
        y = F.relu(F.conv_transpose2d(y, self.sd["Mask_Head.upconv.weight"],
                                      self.sd["Mask_Head.upconv.bias"], 2))
        m = torch.sigmoid(self._conv(y, "Mask_Outs.classify")).numpy()
        masks = m[np.arange(len(classes)), classes]
        extra.update(mask_rois=mrois, mask_feat=mf)
        return sc, bx, classes, masks, extra


class RefCPUPipelineC4(RefCPUPipeline):
    """The reference's CPU im_detect_all for e2e_mask_rcnn_R-50-C4 (no FPN):
    ResNet50_conv4_body (ResNet.py:17-116) -> single_scale_rpn_outputs
    (rpn_heads.py:37-126) -> GenerateProposalsOp (15 anchors, pre/post
    6000/1000) -> roi_feature_transform single blob (model_builder.py:304-322,
    RoIAlign 14x14, adaptive sr 0) -> ResNet_roi_conv5_head (res5, avgpool 7) ->
    fast_rcnn_outputs -> box_results_with_nms_and_limit -> mask RoIAlign 14x14
    -> shared res5 -> upconv5 + ReLU (mask_rcnn_fcn_head_v0upshare,
    mask_rcnn_heads.py:263-331) -> sigmoid (R x 81 x 14 x 14)."""

    def __init__(self, sd, block_counts=(3, 4, 6), pre_nms=6000, post_nms=1000,
                 test_scale=800, **kw):
        self.test_scale = test_scale  # TEST.SCALE (get_image_blob resizes when != 1)
        kw.setdefault("box_res", 14)
        kw.setdefault("box_sr", 0)
        kw.setdefault("mask_res", 14)
        kw.setdefault("mask_sr", 0)
        super().__init__(sd, block_counts=block_counts, pre_nms=pre_nms, post_nms=post_nms,
                         **kw)
        self.anchors = orc.generate_anchors(16, (32, 64, 128, 256, 512), (0.5, 1, 2))

    def _block(self, x, p, stride):
        o = F.relu(self._aff(self._conv(x, p + "conv1", stride, bias=False), p + "bn1"))
        o = F.relu(self._aff(self._conv(o, p + "conv2", 1, 1, groups=self.groups, bias=False),
                             p + "bn2"))
        o = self._aff(self._conv(o, p + "conv3", bias=False), p + "bn3")
        if (p + "downsample.0.weight") in self.sd:
            r = self._aff(self._conv(x, p + "downsample.0", stride, bias=False),
                          p + "downsample.1")
        else:
            r = x
        return F.relu(o + r)

    def backbone(self, blob):
        pre = "Conv_Body."
        x = self._conv(blob, pre + "res1.conv1", 2, 3, bias=False)
        x = F.relu(self._aff(x, pre + "res1.bn1"))
        x = F.max_pool2d(x, 3, 2, 1)
        for si, n in enumerate(self.block_counts):
            for b in range(n):
                x = self._block(x, pre + "res%d.%d." % (si + 2, b),
                                2 if (b == 0 and si > 0) else 1)
        return x  # res4, 1/16

    def res5(self, x):
        for b in range(3):
            x = self._block(x, "Box_Head.res5.%d." % b, 2 if b == 0 else 1)
        return x

    @torch.no_grad()
    def __call__(self, im_u8):
        """im_u8: H x W x 3 uint8 BGR.  Returns (scores, boxes, classes, masks, extra)."""
        blob, im_scale, im_info = orc.get_image_blob(im_u8, self.test_scale,
                                                     stride=1)  # no FPN padding
        res4 = self.backbone(torch.from_numpy(blob))
        h = F.relu(self._conv(res4, "RPN.RPN_conv", 1, 1))
        cls = torch.sigmoid(self._conv(h, "RPN.RPN_cls_score")).numpy()
        dl = self._conv(h, "RPN.RPN_bbox_pred").numpy()
        rois, _ = orc.generate_proposals(self.anchors, 1. / 16, cls, dl, im_info, self.pre_nms,
                                         self.post_nms, self.rpn_nms, 0)
        extra = {"probs": cls, "deltas": dl, "rois": rois}
        feat = res4.numpy()
        bf = orc.roi_align(feat, rois, self.box_res, self.box_res, 1. / 16, self.box_sr)
        x = F.avg_pool2d(self.res5(torch.from_numpy(bf)), 7).flatten(1)
        scores = F.softmax(F.linear(x, self.sd["Box_Outs.cls_score.weight"],
                                    self.sd["Box_Outs.cls_score.bias"]), dim=1).numpy()
        deltas = F.linear(x, self.sd["Box_Outs.bbox_pred.weight"],
                          self.sd["Box_Outs.bbox_pred.bias"]).numpy()
        boxes = rois[:, 1:5] / im_scale
        pred = orc.bbox_transform(boxes, deltas, (10., 10., 5., 5.))
        pred = orc.clip_tiled_boxes(pred, im_u8.shape)
        sc, bx, cls_boxes = orc.box_results_with_nms_and_limit(
            scores, pred, self.K, self.score_thresh, self.test_nms, self.dets_per_im)
        classes = np.concatenate([[j] * len(cls_boxes[j]) for j in range(1, self.K)] +
                                 [np.zeros((0,))]).astype(np.int32)
        extra.update(scores_all=scores, deltas_all=deltas, box_feat=bf)
        R = self.mask_res
        if bx.shape[0] == 0:
            return sc, bx, classes, np.zeros((0, R, R), np.float32), extra
        mrois = np.hstack([np.zeros((bx.shape[0], 1)), bx.astype(np.float64) * im_scale])
        mrois = mrois.astype(np.float32)
        mf = orc.roi_align(feat, mrois, self.mask_res, self.mask_res, 1. / 16, self.mask_sr)
        y = F.relu(F.conv_transpose2d(self.res5(torch.from_numpy(mf)),
                                      self.sd["Mask_Head.upconv5.weight"],
                                      self.sd["Mask_Head.upconv5.bias"], 2))
        m = torch.sigmoid(self._conv(y, "Mask_Outs.classify")).numpy()
        masks = m[np.arange(len(classes)), classes]
        extra.update(mask_rois=mrois, mask_feat=mf)
        return sc, bx, classes, masks, extra
