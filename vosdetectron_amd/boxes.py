"""Drop-ins for the reference's ``utils.boxes`` NMS entry point (lib/utils/boxes.py:329-333).

``nms(dets, thresh)`` keeps the reference's host signature -- dets an (N, >=5)
float32 ndarray ``[x1, y1, x2, y2, score]``, thresh a float -- and returns the
kept row indices as an int64 ndarray in ascending order (``[]`` for no rows),
with cython_nms.nms semantics (``+1`` areas, fp32 IoU, suppress on
``>= thresh``; lib/utils/cython_nms.pyx:37-87).  The suppression runs on the
device (vd_nms: wave-ballot bitmask + single-wave resolve, nms.hip); the rows go
up and the indices come back because the reference's callers hold ndarrays.
Device tensors are accepted as well and stay on the device.
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
