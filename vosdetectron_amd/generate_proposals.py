"""Drop-in for the reference's ``GenerateProposalsOp`` (lib/modeling/generate_proposals.py:13-102).

Same constructor (anchors ndarray A x 4, spatial_scale), same forward arguments
(rpn_cls_prob N x A x H x W, rpn_bbox_pred N x 4A x H x W, im_info N x 3) and the
same return value: host ndarrays ``rois`` (R, 5) float32 ``[batch, x1, y1, x2,
y2]`` and ``roi_probs`` (R, 1) float32, images in batch order.  The work --
shifted anchors, decode (bbox_transform, boxes.py:156-205), clip, min-size
filter, top pre_nms_topN, NMS, keep[:post_nms_topN] -- is one
vd_generate_proposals launch over every image (proposals.hip); only the final
per-image rows are copied back, because the reference's callers consume
ndarrays.  Mode-dependent config (TRAIN / TEST RPN_* keys) is read from the
package's global cfg (vosdetectron_amd.config.cfg), as the reference reads
core.config.cfg.

Error behaviour as the reference: NaN deltas raise ValueError('bbox_deltas nan')
(:62-63).  CPU tensors raise NotImplementedError (there is no CPU path).
A level whose top-k selection cannot complete raises (VosdetError) instead of
returning fewer proposals.
"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn

from . import config as vcfg
from . import ops


class GenerateProposalsOp(nn.Module):
    def __init__(self, anchors, spatial_scale, cfg=None):
        super().__init__()
        self._anchors = np.asarray(anchors, np.float64)
        self._num_anchors = self._anchors.shape[0]
        self._feat_stride = 1. / spatial_scale
        self._spatial_scale = float(spatial_scale)
        self._cfg = cfg
        self._dev_anchors = {}

    def _anchors_on(self, device):
        a = self._dev_anchors.get(device)
        if a is None:
            a = torch.from_numpy(self._anchors).to(device)
            self._dev_anchors[device] = a
        return a

    def forward(self, rpn_cls_prob, rpn_bbox_pred, im_info):
        cfg = self._cfg if self._cfg is not None else vcfg.cfg
        c = cfg.TRAIN if (self.training and "TRAIN" in cfg) else cfg.TEST
        p = rpn_cls_prob.detach() if isinstance(rpn_cls_prob, torch.Tensor) else None
        d = rpn_bbox_pred.detach() if isinstance(rpn_bbox_pred, torch.Tensor) else None
        if p is None or d is None or not p.is_cuda or not d.is_cuda:
            raise NotImplementedError("GenerateProposalsOp runs on device tensors only")
        N, A, H, W = p.shape
        if A != self._num_anchors or tuple(d.shape) != (N, 4 * A, H, W):
            raise ValueError("rpn_cls_prob %s / rpn_bbox_pred %s do not match %d anchors"
                             % (tuple(p.shape), tuple(d.shape), self._num_anchors))
        if bool(torch.isnan(d).any()):
            raise ValueError("bbox_deltas nan")
        info = torch.as_tensor(np.asarray(im_info.cpu() if isinstance(im_info, torch.Tensor)
                                          else im_info, np.float32), device=p.device)
        rois, probs, counts = ops.generate_proposals(
            [p.float().contiguous()], [d.float().contiguous()], [self._anchors_on(p.device)],
            [self._spatial_scale], info, int(c.RPN_PRE_NMS_TOP_N), int(c.RPN_POST_NMS_TOP_N),
            float(c.RPN_NMS_THRESH), float(c.RPN_MIN_SIZE))
        cnt = counts[:, 0].cpu().tolist()
        ops.raise_on_failed_counts(cnt, "image")
        rois_h, probs_h = rois[:, 0].cpu().numpy(), probs[:, 0].cpu().numpy()
        out_r = [rois_h[i, :k] for i, k in enumerate(cnt)]
        out_p = [probs_h[i, :k, None] for i, k in enumerate(cnt)]
        return (np.concatenate(out_r).astype(np.float32, copy=False) if out_r
                else np.empty((0, 5), np.float32),
                np.concatenate(out_p).astype(np.float32, copy=False) if out_p
                else np.empty((0, 1), np.float32))
