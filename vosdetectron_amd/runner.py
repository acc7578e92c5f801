"""Frame-sharded multi-GPU inference.

The reference range-shards a dataset over per-GPU subprocesses and collates
pickled `all_boxes` / `all_segms` in the parent (lib/core/test_engine.py:168-213,
lib/utils/subprocess.py:41-115).  Here every rank (one process per GPU,
torch.distributed over RCCL/xGMI) runs the device-resident engine on its own
frames, and ONE collective per step -- all_gather of fixed-size padded tensors --
gives every rank all results (no reduction, so the gathered rows are bit-identical
to the per-rank rows).  The same code runs on the gloo backend with CPU tensors,
which is how the N>1 path is tested in a CPU container.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np
import torch
import torch.distributed as dist


def shard_frames(n_frames: int, world: int, rank: int) -> Sequence[int]:
    """Contiguous ranges, np.array_split like lib/utils/subprocess.py:56."""
    return [int(i) for i in np.array_split(np.arange(n_frames), world)[rank]]


class ResultGatherer:
    """Pads each rank's per-frame results to fixed shapes and all-gathers them."""

    def __init__(self, frames_per_rank: int, det_cap: int, mask_res: int, world: int,
                 device, with_masks: bool = True):
        F, D = frames_per_rank, det_cap
        self.F, self.D, self.world, self.with_masks = F, D, world, with_masks
        self.pad_masks = torch.zeros((F, D, mask_res, mask_res), device=device)
        self.g_dets = torch.zeros((world * F, D, 5), device=device)
        self.g_cls = torch.zeros((world * F, D), dtype=torch.int32, device=device)
        self.g_cnt = torch.zeros((world * F,), dtype=torch.int32, device=device)
        self.g_masks = torch.zeros((world * F, D, mask_res, mask_res), device=device)

    def pack_masks(self, masks: torch.Tensor, counts: List[int]) -> torch.Tensor:
        self.pad_masks.zero_()
        o = 0
        for f, c in enumerate(counts):
            if c:
                self.pad_masks[f, :c] = masks[o:o + c]
            o += c
        return self.pad_masks

    def gather(self, dets: torch.Tensor, classes: torch.Tensor, counts: torch.Tensor,
               masks: torch.Tensor, counts_host: List[int]) -> Dict[str, torch.Tensor]:
        """dets [F,D,5], classes [F,D] int32, counts [F] int32, masks [M,R,R]."""
        if self.world == 1:
            return {"dets": dets, "classes": classes, "counts": counts,
                    "masks": self.pack_masks(masks, counts_host) if self.with_masks else None}
        dist.all_gather_into_tensor(self.g_dets, dets.contiguous())
        dist.all_gather_into_tensor(self.g_cls, classes.contiguous())
        dist.all_gather_into_tensor(self.g_cnt, counts.contiguous())
        if self.with_masks:
            dist.all_gather_into_tensor(self.g_masks, self.pack_masks(masks, counts_host))
        return {"dets": self.g_dets, "classes": self.g_cls, "counts": self.g_cnt,
                "masks": self.g_masks if self.with_masks else None}
