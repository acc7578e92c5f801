"""Drop-ins for the reference's ``utils.boxes`` NMS entry points (lib/utils/boxes.py:
277-355: nms, soft_nms, box_voting).

``nms(dets, thresh)`` keeps the reference's host signature -- dets an (N, >=5)
float32 ndarray ``[x1, y1, x2, y2, score]``, thresh a float -- and returns the
kept row indices as an int64 ndarray in ascending order (``[]`` for no rows),
with cython_nms.nms semantics (``+1`` areas, fp32 IoU, suppress on
``>= thresh``; lib/utils/cython_nms.pyx:37-87).  The suppression runs on the
device (vd_nms: wave-ballot bitmask + single-wave resolve, nms.hip); the rows go
up and the indices come back because the reference's callers hold ndarrays.
Device tensors are accepted as well and stay on the device.

``soft_nms`` (vd_soft_nms) and ``box_voting`` (vd_box_voting) keep the
reference's signatures and return ndarrays the same way.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops


def nms(dets, thresh):
    """Apply classic DPM-style greedy NMS (cython_nms semantics) on the device."""
    if isinstance(dets, torch.Tensor):
        if not dets.is_cuda:
            raise NotImplementedError("nms: CPU tensors have no path; pass an ndarray "
                                      "or a device tensor")
        return ops.nms(dets.float().contiguous(), thresh)
    d = np.asarray(dets)
    if d.shape[0] == 0:
        return []
    if d.ndim != 2 or d.shape[1] < 5:
        raise ValueError("dets must be N x >=5, got %s" % (d.shape,))
    t = torch.from_numpy(np.ascontiguousarray(d, np.float32)).to(
        torch.device("cuda", torch.cuda.current_device()))
    return ops.nms(t, thresh).cpu().numpy()


def _dev(d):
    return torch.from_numpy(np.ascontiguousarray(d, np.float32)).to(
        torch.device("cuda", torch.cuda.current_device()))


def soft_nms(dets, sigma=0.5, overlap_thresh=0.3, score_thresh=0.001, method="linear"):
    """Apply the soft NMS algorithm from https://arxiv.org/abs/1704.04503 (device)."""
    d = np.asarray(dets)
    if d.shape[0] == 0:
        return dets, []
    rows, keep = ops.soft_nms(_dev(d), sigma, overlap_thresh, score_thresh, method)
    return rows.cpu().numpy(), keep.cpu().numpy()


def box_voting(top_dets, all_dets, thresh, scoring_method="ID", beta=1.0):
    """Refine top_dets by voting with all_dets (https://arxiv.org/abs/1505.01749)."""
    t = np.asarray(top_dets)
    if t.shape[0] == 0:
        return t.copy()
    return ops.box_voting(_dev(t), _dev(all_dets), thresh, scoring_method, beta).cpu().numpy()
