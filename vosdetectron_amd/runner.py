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


class PendingGather:
    """An in-flight all_gather (async_op) of one buffer slot."""

    def __init__(self, work, gatherer, rbuf):
        self.work, self.g, self.rbuf = work, gatherer, rbuf

    def wait(self, views: bool = True) -> Dict[str, torch.Tensor]:
        """Orders the caller's stream after the collective; returns the gathered
        results ([world*F, ...], rank-major) unless views=False."""
        if self.work is not None:
            self.work.wait()
            self.work = None
        return self.g._views(self.rbuf) if views else {}


class ResultGatherer:
    """Packs each rank's per-frame results -- dets [F,D,5], classes [F,D], counts
    [F], class-selected masks padded to [F,D,R,R] -- into ONE flat fp32 buffer
    (int32 fields bit-cast) and all-gathers it in a single collective.  Two
    buffer slots alternate, so `gather_async` of step t can run on RCCL's stream
    while step t+1 computes; `wait()` before the slot is reused (the caller
    keeps at most one gather in flight)."""

    def __init__(self, frames_per_rank: int, det_cap: int, mask_res: int, world: int,
                 device, with_masks: bool = True):
        F, D, R = frames_per_rank, det_cap, mask_res
        self.F, self.D, self.R, self.world, self.with_masks = F, D, R, world, with_masks
        self.o_cls = F * D * 5
        self.o_cnt = self.o_cls + F * D
        self.o_msk = self.o_cnt + F
        self.L = self.o_msk + (F * D * R * R if with_masks else 0)
        self.send = [torch.zeros((self.L,), device=device) for _ in range(2)]
        self.recv = [torch.zeros((world, self.L), device=device) for _ in range(2)]
        self.slot = 0

    def _pack(self, buf, dets, classes, counts, masks, counts_host):
        F, D, R = self.F, self.D, self.R
        buf[:self.o_cls].copy_(dets.reshape(-1))
        buf[self.o_cls:self.o_cnt].view(torch.int32).copy_(classes.reshape(-1))
        buf[self.o_cnt:self.o_msk].view(torch.int32).copy_(counts.reshape(-1))
        if self.with_masks:
            pm = buf[self.o_msk:].view(F, D, R, R)
            pm.zero_()
            o = 0
            for f, c in enumerate(counts_host):
                if c:
                    pm[f, :c] = masks[o:o + c]
                o += c

    def _views(self, rb):
        W, F, D, R = rb.shape[0], self.F, self.D, self.R
        v = {"dets": rb[:, :self.o_cls].reshape(W * F, D, 5),
             "classes": rb[:, self.o_cls:self.o_cnt].contiguous().view(torch.int32)
                        .reshape(W * F, D),
             "counts": rb[:, self.o_cnt:self.o_msk].contiguous().view(torch.int32).reshape(W * F),
             "masks": rb[:, self.o_msk:].reshape(W * F, D, R, R) if self.with_masks else None}
        return v

    def gather_async(self, dets: torch.Tensor, classes: torch.Tensor, counts: torch.Tensor,
                     masks: torch.Tensor, counts_host: List[int]) -> PendingGather:
        """dets [F,D,5], classes [F,D] int32, counts [F] int32, masks [M,R,R]."""
        s = self.slot
        self.slot ^= 1
        self._pack(self.send[s], dets, classes, counts, masks, counts_host)
        if self.world == 1:
            return PendingGather(None, self, self.send[s].view(1, -1))
        work = dist.all_gather_into_tensor(self.recv[s].view(-1), self.send[s], async_op=True)
        return PendingGather(work, self, self.recv[s])

    def gather(self, dets, classes, counts, masks, counts_host) -> Dict[str, torch.Tensor]:
        return self.gather_async(dets, classes, counts, masks, counts_host).wait()
