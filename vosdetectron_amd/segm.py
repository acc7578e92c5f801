"""segm_results on the device (lib/core/test.py:801-855, fork
lib_vos/tools/vos_test.py:867-921): the per-detection host loop of
expand_boxes + cv2.resize + threshold + paste + pycocotools RLE + rleToString
becomes three launches over every detection of a batch -- vd_segm_rle (paste
and run lengths fused: the pasted values are evaluated inside each clipped box
and turned into column-major runs without writing the frame-sized planes) and
vd_rle_strings (rleToString, lengths then packed chars).  The host only slices
the packed ASCII buffer into one string per detection and groups them by class,
as the reference's `rle['counts'].decode('ascii')` + `cls_segms[j].append`."""
from __future__ import annotations

from typing import List, Sequence

import torch

from . import ops


def encode_masks(masks: torch.Tensor, boxes: torch.Tensor, im_h: int, im_w: int,
                 thresh: float = 0.5) -> List[dict]:
    """[M,R,R] class-selected mask probabilities + [M,>=4] boxes -> the
    pycocotools-style RLE dicts of their pasted, binarised frame masks."""
    M = masks.shape[0]
    if M == 0:
        return []
    counts, n = ops.segm_rle_counts(masks, boxes, im_h, im_w, thresh)
    size = [int(im_h), int(im_w)]
    return [{"size": size, "counts": s} for s in ops.rle_strings(counts, n)]


def encode_planes(planes: torch.Tensor) -> List[dict]:
    """[M,H,W] uint8 device planes -> pycocotools-style RLE dicts (counts as str)."""
    M, H, W = planes.shape
    if M == 0:
        return []
    counts, n = ops.mask_rle_counts(planes)
    return [{"size": [int(H), int(W)], "counts": s} for s in ops.rle_strings(counts, n)]


def group_by_class(rles: Sequence[dict], classes: Sequence[int], num_classes: int = 81):
    """cls_segms[j] = the RLEs of class j, in detection order (test.py:840-842)."""
    cls_segms = [[] for _ in range(num_classes)]
    for r, c in zip(rles, classes):
        cls_segms[int(c)].append(r)
    return cls_segms


def segm_results(dets: torch.Tensor, classes: torch.Tensor, masks: torch.Tensor, im_h: int,
                 im_w: int, num_classes: int = 81, thresh: float = 0.5):
    """The reference's segm_results(cls_boxes, masks, ref_boxes, im_h, im_w) for
    one frame of the device pipeline: dets [k,>=4] (the cls_boxes rows in
    class-major order), classes [k] int, masks [k,R,R] class-selected mask
    probabilities.  Returns cls_segms: list over classes of RLE dicts."""
    rles = encode_masks(masks, dets, im_h, im_w, thresh)
    return group_by_class(rles, classes.cpu().tolist(), num_classes)
