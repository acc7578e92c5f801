"""Drop-in for the reference's ``CollectAndDistributeFpnRpnProposalsOp``
(lib/modeling/collect_and_distribute_fpn_rpn_proposals.py:46-88) and its
module functions ``collect`` (:91-106) and ``distribute`` (:109-138).

``op(inputs, roidb, im_info)`` takes the reference's input list
``[rpn_rois_fpn2 .. rpn_rois_fpn6, rpn_roi_probs_fpn2 .. rpn_roi_probs_fpn6]``
(host ndarrays, as GenerateProposalsOp returns them) and returns the reference's
inference blob dict: ``rois`` (R, 5), ``rois_fpn2 .. rois_fpn5`` and
``rois_idx_restore_int32`` -- the ``rpn_ret`` entries roi_feature_transform
consumes.  The top-post_nms_topN selection over all levels and the FPN level map
(utils/fpn.py:11-28) run on the device (vd_collect_distribute); the per-level
split of the selected rows and the restore permutation are the dict's host
formatting.  As in the reference, collect() ranks every input row together
(all images of the batch at once).  Training (roidb labels) is out of scope and
raises NotImplementedError.
"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn

from . import config as vcfg
from . import ops


def _device():
    return torch.device("cuda", torch.cuda.current_device())


def collect_device(inputs, cfg, device=None):
    """collect(): returns (rois [R,5] device, level index int32 [R] device) of the
    global top post_nms_topN over every level's rows."""
    k_min, k_max = cfg.FPN.RPN_MIN_LEVEL, cfg.FPN.RPN_MAX_LEVEL
    L = k_max - k_min + 1
    if len(inputs) != 2 * L:
        raise ValueError("expected %d inputs (rois and probs of levels %d..%d), got %d"
                         % (2 * L, k_min, k_max, len(inputs)))
    post = int(cfg.TEST.RPN_POST_NMS_TOP_N * cfg.FPN.RPN_COLLECT_SCALE + 0.5)
    rois_l = [np.asarray(r, np.float32).reshape(-1, 5) for r in inputs[:L]]
    probs_l = [np.asarray(p, np.float32).reshape(-1) for p in inputs[L:]]
    cap = max(1, max(len(r) for r in rois_l))
    if L * cap > 8192:
        raise ValueError("collect: %d levels x %d rows exceed the device kernel's 8192 "
                         "candidates" % (L, cap))
    lr = np.zeros((1, L, cap, 5), np.float32)
    lp = np.zeros((1, L, cap), np.float32)
    lc = np.zeros((1, L), np.int32)
    for i, (r, p) in enumerate(zip(rois_l, probs_l)):
        lr[0, i, :len(r)] = r
        lp[0, i, :len(p)] = p
        lc[0, i] = len(r)
    dev = device or _device()
    rois, lvl, cnt = ops.collect_distribute(torch.from_numpy(lr).to(dev),
                                            torch.from_numpy(lp).to(dev),
                                            torch.from_numpy(lc).to(dev), post,
                                            cfg.FPN.ROI_MIN_LEVEL, cfg.FPN.ROI_MAX_LEVEL)
    n = int(cnt[0].item())
    return rois[0, :n], lvl[0, :n]


def collect(inputs, is_training, cfg=None):
    """collect_and_distribute_fpn_rpn_proposals.collect (:91-106) -> rois ndarray."""
    if is_training:
        raise NotImplementedError("training-time collect is out of scope")
    rois, _ = collect_device(inputs, cfg if cfg is not None else vcfg.cfg)
    return rois.cpu().numpy()


def _blobs(rois, lvls, lvl_min, lvl_max, prefix="rois"):
    """The reference's output dict from rows + their level (utils/fpn.py's
    rois_idx_restore = argsort(concat(per-level indices)))."""
    out = {prefix: rois}
    order = []
    for lvl in range(lvl_min, lvl_max + 1):
        idx = np.where(lvls == lvl)[0]
        out[prefix + "_fpn" + str(lvl)] = rois[idx, :]
        order.append(idx)
    order = np.concatenate(order) if order else np.zeros((0,), np.int64)
    restore = np.empty(len(order), np.int32)
    restore[order] = np.arange(len(order), dtype=np.int32)
    out[prefix + "_idx_restore_int32"] = restore
    return out


def distribute(rois, label_blobs, cfg=None):
    """distribute (:109-138): level map on the device, per-level blobs + restore."""
    cfg = cfg if cfg is not None else vcfg.cfg
    r = np.ascontiguousarray(rois, np.float32)
    if len(r) == 0:
        lv = np.zeros((0,), np.int32)
    else:
        lv = ops.map_rois_to_fpn_levels(torch.from_numpy(r).to(_device()),
                                        cfg.FPN.ROI_MIN_LEVEL, cfg.FPN.ROI_MAX_LEVEL).cpu().numpy()
    return _blobs(r, lv, cfg.FPN.ROI_MIN_LEVEL, cfg.FPN.ROI_MAX_LEVEL)


class CollectAndDistributeFpnRpnProposalsOp(nn.Module):
    def __init__(self, cfg=None):
        super().__init__()
        self._cfg = cfg

    def forward(self, inputs, roidb=None, im_info=None):
        if self.training:
            raise NotImplementedError("training-time proposal labelling is out of scope")
        cfg = self._cfg if self._cfg is not None else vcfg.cfg
        rois, lvl = collect_device(inputs, cfg)
        lv = lvl.cpu().numpy() + cfg.FPN.ROI_MIN_LEVEL
        return _blobs(rois.cpu().numpy(), lv, cfg.FPN.ROI_MIN_LEVEL, cfg.FPN.ROI_MAX_LEVEL)
