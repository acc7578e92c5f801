"""segm_results on the device (lib/core/test.py:801-855, fork
lib_vos/tools/vos_test.py:867-921): the per-detection host loop of
expand_boxes + cv2.resize + threshold + paste + pycocotools RLE becomes two
launches (vd_paste_masks, vd_mask_rle) over every detection of a batch; only
the run lengths -> ASCII step (pycocotools rleToString, maskApi.c) is host
formatting, as the reference's `rle['counts'].decode('ascii')` is."""
from __future__ import annotations

from typing import List, Sequence

import torch

from . import ops


def rle_to_string(counts: Sequence[int]) -> str:
    """pycocotools maskApi.c rleToString: LEB128-like, 6 bits per char in
    ASCII 48..111, each count after the second delta-coded against counts[i-2]."""
    out = []
    for i, c in enumerate(counts):
        x = int(c)
        if i > 2:
            x -= int(counts[i - 2])
        more = True
        while more:
            ch = x & 0x1f
            x >>= 5
            more = (x != -1) if (ch & 0x10) else (x != 0)
            if more:
                ch |= 0x20
            out.append(chr(ch + 48))
    return "".join(out)


def encode_planes(planes: torch.Tensor) -> List[dict]:
    """[M,H,W] uint8 device planes -> pycocotools-style RLE dicts (counts as str)."""
    M, H, W = planes.shape
    if M == 0:
        return []
    counts, n = ops.mask_rle_counts(planes)
    counts, n = counts.cpu().numpy(), n.cpu().numpy()
    return [{"size": [int(H), int(W)], "counts": rle_to_string(counts[i, :n[i]])}
            for i in range(M)]


def segm_results(dets: torch.Tensor, classes: torch.Tensor, masks: torch.Tensor, im_h: int,
                 im_w: int, num_classes: int = 81, thresh: float = 0.5):
    """The reference's segm_results(cls_boxes, masks, ref_boxes, im_h, im_w) for
    one frame of the device pipeline: dets [k,>=4] (the cls_boxes rows in
    class-major order), classes [k] int, masks [k,R,R] class-selected mask
    probabilities.  Returns (cls_segms: list over classes of RLE dicts, planes
    [k,im_h,im_w] uint8 on the device)."""
    planes = ops.paste_masks(masks, dets, im_h, im_w, thresh)
    rles = encode_planes(planes)
    cls_segms = [[] for _ in range(num_classes)]
    for r, c in zip(rles, classes.cpu().tolist()):
        cls_segms[int(c)].append(r)
    return cls_segms, planes
