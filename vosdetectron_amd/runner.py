"""Frame-sharded multi-GPU inference.

The reference range-shards a dataset over per-GPU subprocesses and collates
pickled `all_boxes` / `all_segms` in the parent (lib/core/test_engine.py:168-213,
lib/utils/subprocess.py:41-115).  Here every rank (one process per GPU,
torch.distributed over RCCL/xGMI) runs the device-resident engine on its own
frames, and ONE collective per step -- all_gather of a fixed-size packed buffer
-- gives every rank all results (no reduction, so the gathered rows are
bit-identical to the per-rank rows).  The same code runs on the gloo backend
with CPU tensors, which is how the N>1 path is tested in a CPU container.

Also here: `FrameUploader`, the per-step host->device frame upload that the
§8d FPS definition puts inside the timed region (pinned host batches, copied on
a side stream one step ahead of the compute that consumes them).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist


def shard_frames(n_frames: int, world: int, rank: int) -> Sequence[int]:
    """Contiguous ranges, np.array_split like lib/utils/subprocess.py:56."""
    return [int(i) for i in np.array_split(np.arange(n_frames), world)[rank]]


class PendingGather:
    """An in-flight all_gather (async_op) of one buffer slot.

    The views `wait()` returns alias the gatherer's receive slot (the send slot
    without a process group).  Slots alternate, so a view stays valid until the
    gather_async call after next; `wait(clone=True)` returns private copies for
    callers that keep results longer.  A `wait()` on a slot that a later
    gather_async has reused raises (generation check); views returned by an
    earlier `wait()` are NOT guarded -- they alias the buffer and show the
    later step's rows once it is reused."""

    def __init__(self, work, gatherer, rbuf, slot, gen, over=None):
        self.work, self.g, self.rbuf, self.slot, self.gen = work, gatherer, rbuf, slot, gen
        self.over = over  # this rank's mask rows past mask_rows (not in the packet)

    def wait(self, views: bool = True, clone: bool = False) -> Dict[str, torch.Tensor]:
        """Orders the caller's stream after the collective; returns the gathered
        results (rank-major) unless views=False."""
        if self.work is not None:
            self.work.wait()
            self.work = None
        if not views:
            return {}
        if self.g.gen[self.slot] != self.gen:
            raise RuntimeError("gathered results of slot %d were overwritten by a later "
                               "gather_async; wait(clone=True) keeps a private copy" % self.slot)
        v = self.g._views(self.rbuf)
        return {k: t.clone() for k, t in v.items()} if clone else v

    def finish(self, masks_full: Optional[torch.Tensor] = None, clone: bool = False
               ) -> Dict[str, torch.Tensor]:
        """wait() plus the mask rows past the packet's mask_rows, on every rank.
        Collective: call it on all ranks for the same step.  After the packet
        lands every rank reads the gathered counts (one small D2H) and so takes
        the same decision: when some rank has M > mask_rows (detections tied at
        DETECTIONS_PER_IM, or the engine's complete() adding rows after the packet
        was sent), ONE more all_gather ships each rank's extra rows, zero-padded to
        the largest overflow, as views["masks_extra"] [W, max_overflow, R, R];
        frame_masks reads them.  masks_full: this rank's complete M-row masks
        (after FramePipeline.complete); default: the rows gather_async could not
        pack."""
        v = self.wait(clone=clone)
        g = self.g
        if not g.with_masks:
            return v
        W = v["counts"].shape[0] // g.F
        M = v["counts"].view(W, g.F).to(torch.int64).sum(1).cpu().tolist()
        over = [max(0, m - g.mask_rows) for m in M]
        mo = max(over, default=0)
        if mo == 0:
            return v
        rank = dist.get_rank() if g.collective else 0
        mine = masks_full[g.mask_rows:M[rank]] if masks_full is not None else self.over
        if over[rank] and (mine is None or mine.shape[0] != over[rank]):
            raise RuntimeError("rank %d has %d mask rows past the packet, %s given"
                               % (rank, over[rank], None if mine is None else mine.shape[0]))
        dev = g.send[0].device
        send = torch.zeros((mo, g.R, g.R), dtype=torch.float32, device=dev)
        if over[rank]:
            send[:over[rank]].copy_(mine.reshape(-1, g.R, g.R))
        if g.collective:
            recv = torch.empty((W, mo, g.R, g.R), dtype=torch.float32, device=dev)
            dist.all_gather_into_tensor(recv.view(-1), send.view(-1))
        else:
            recv = send.view(1, mo, g.R, g.R)
        v = dict(v)
        v["masks_extra"] = recv
        return v


class ResultGatherer:
    """Packs each rank's per-step results into ONE flat fp32 buffer and
    all-gathers it in a single collective:

      dets [F, D, 5] | classes [F, D] (int32 bit-cast) | counts [F] (int32) |
      masks [mask_rows, R, R]  (the class-selected fp32 masks of the step's
                                M = sum(counts) detections, frame-major, as the
                                engine produces them; rows >= M are padding)

    Packing is three device copies (no host loop, no per-frame work): the
    engine's masks are already frame-contiguous, so a frame's rows start at the
    exclusive prefix sum of the counts, which receivers recompute on the device
    (`frame_offsets`).  mask_rows defaults to F x DETECTIONS_PER_IM (100), the
    most box_results_with_nms_and_limit keeps per frame barring exact score ties
    at the 100th place; a step whose M exceeds it raises (never truncates).
    With F = 16 that is 5.0 MB per rank per step (vs 12.8 MB for masks padded to
    the engine's det_cap of 256 rows per frame), still exact fp32 -- the
    reference's segm_results resizes the probabilities before thresholding, so a
    pre-binarised mask would change its output.  Rows past mask_rows are not
    dropped: PendingGather.finish() ships them in a second all_gather, only on
    steps where some rank has them.

    Two buffer slots alternate, so `gather_async` of step t can run on RCCL's
    stream while step t+1 computes; the caller keeps at most one gather in
    flight (`wait()` before issuing the next).  The collective is issued
    whenever a process group is initialised -- including a one-rank RCCL group,
    so world 1 exercises the same all_gather_into_tensor -- and skipped (the
    send slot is the result) only without one."""

    def __init__(self, frames_per_rank: int, det_cap: int, mask_res: int, world: int,
                 device, with_masks: bool = True, mask_rows: Optional[int] = None):
        F, D, R = frames_per_rank, det_cap, mask_res
        self.F, self.D, self.R, self.world, self.with_masks = F, D, R, world, with_masks
        self.mask_rows = int(mask_rows if mask_rows is not None else F * 100) if with_masks else 0
        self.o_cls = F * D * 5
        self.o_cnt = self.o_cls + F * D
        self.o_msk = self.o_cnt + F
        self.L = self.o_msk + self.mask_rows * R * R
        self.send = [torch.zeros((self.L,), device=device) for _ in range(2)]
        self.recv = [torch.zeros((world, self.L), device=device) for _ in range(2)]
        self.slot = 0
        self.gen = [0, 0]
        self.collective = dist.is_available() and dist.is_initialized()
        if self.collective and dist.get_world_size() != world:
            raise ValueError("ResultGatherer(world=%d) but the process group has %d ranks"
                             % (world, dist.get_world_size()))

    @property
    def bytes_per_rank(self) -> int:
        return 4 * self.L

    def _pack(self, buf, dets, classes, counts, masks):
        buf[:self.o_cls].copy_(dets.reshape(-1))
        buf[self.o_cls:self.o_cnt].view(torch.int32).copy_(classes.reshape(-1))
        buf[self.o_cnt:self.o_msk].view(torch.int32).copy_(counts.reshape(-1))
        if self.with_masks:
            M = min(masks.shape[0], self.mask_rows)  # the rest: PendingGather.finish
            if M:
                buf[self.o_msk:self.o_msk + M * self.R * self.R].copy_(masks[:M].reshape(-1))

    def _views(self, rb):
        W, F, D, R = rb.shape[0], self.F, self.D, self.R
        counts = rb[:, self.o_cnt:self.o_msk].contiguous().view(torch.int32)
        v = {"dets": rb[:, :self.o_cls].reshape(W * F, D, 5),
             "classes": rb[:, self.o_cls:self.o_cnt].contiguous().view(torch.int32)
                        .reshape(W * F, D),
             "counts": counts.reshape(W * F)}
        if self.with_masks:
            v["masks"] = rb[:, self.o_msk:].reshape(W, self.mask_rows, R, R)
            v["mask_offsets"] = self.frame_offsets(counts)
        return v

    @staticmethod
    def frame_offsets(counts: torch.Tensor) -> torch.Tensor:
        """counts [W, F] int32 -> first mask row of every frame within its rank's
        mask rows ([W, F] int64, exclusive prefix sum, on the counts' device)."""
        c = counts.to(torch.int64)
        return torch.cumsum(c, 1) - c

    def gather_async(self, dets: torch.Tensor, classes: torch.Tensor, counts: torch.Tensor,
                     masks: torch.Tensor, counts_host: Optional[List[int]] = None
                     ) -> PendingGather:
        """dets [F,D,5], classes [F,D] int32, counts [F] int32, masks [M,R,R] (the
        engine's class-selected masks, frame-major).  counts_host is unused (kept
        for callers of the round-1 signature)."""
        s = self.slot
        self.slot ^= 1
        self.gen[s] += 1
        self._pack(self.send[s], dets, classes, counts, masks)
        over = masks[self.mask_rows:] if self.with_masks and masks.shape[0] > self.mask_rows \
            else None
        if not self.collective:
            return PendingGather(None, self, self.send[s].view(1, -1), s, self.gen[s], over)
        work = dist.all_gather_into_tensor(self.recv[s].view(-1), self.send[s], async_op=True)
        return PendingGather(work, self, self.recv[s], s, self.gen[s], over)

    def gather(self, dets, classes, counts, masks, counts_host=None) -> Dict[str, torch.Tensor]:
        return self.gather_async(dets, classes, counts, masks).wait()


def frame_masks(views: Dict[str, torch.Tensor], frames_per_rank: int, frame: int
                ) -> torch.Tensor:
    """The gathered masks of global frame index `frame` (rank-major order); rows
    past the packet's mask rows come from views["masks_extra"]
    (PendingGather.finish), and raise if the views lack them."""
    r, f = divmod(frame, frames_per_rank)
    o = int(views["mask_offsets"][r, f])
    k = int(views["counts"][frame])
    cap = views["masks"].shape[1]
    if o + k <= cap:
        return views["masks"][r, o:o + k]
    extra = views.get("masks_extra")
    if extra is None or o + k - cap > extra.shape[1]:
        raise RuntimeError("frame %d's masks (rows %d..%d) exceed the %d gathered mask rows "
                           "(PendingGather.finish ships the rest)" % (frame, o, o + k, cap))
    head = views["masks"][r, o:cap] if o < cap else views["masks"][r, :0]
    return torch.cat([head, extra[r, max(0, o - cap):o + k - cap]])


class FrameUploader:
    """Per-step H2D of the u8 frames (SURVEY.md §8d puts "H2D of the u8 frame"
    inside the timed region).  Host batches live in pinned memory; `get(t)`
    returns batch t's device copy with the current stream ordered after it, and
    issues batch t+1's copy on a side stream so PCIe overlaps step t's compute.
    Two device slots alternate; the copy into a slot waits for the compute
    stream's event recorded after the step that last read it (`release`)."""

    def __init__(self, host_batches: Sequence[np.ndarray], device):
        self.device = torch.device(device)
        self.host = [torch.from_numpy(np.ascontiguousarray(b)).pin_memory() for b in host_batches]
        shape = self.host[0].shape
        self.dev = [torch.empty(shape, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self.stream = torch.cuda.Stream(device=self.device)
        self.ready = [torch.cuda.Event() for _ in range(2)]
        self.free = [None, None]
        self.issued = -1
        self.nbytes = int(self.host[0].numel())

    def _issue(self, t: int):
        s = t % 2
        with torch.cuda.stream(self.stream):
            if self.free[s] is not None:
                self.stream.wait_event(self.free[s])
            self.dev[s].copy_(self.host[t % len(self.host)], non_blocking=True)
            self.ready[s].record(self.stream)
        self.issued = t

    def get(self, t: int, prefetch: bool = True) -> torch.Tensor:
        """prefetch=False on a timed region's last step (and a warm-up's): the
        next region's first upload is then issued, and timed, inside it."""
        if self.issued < t:
            self._issue(t)
        s = t % 2
        torch.cuda.current_stream().wait_event(self.ready[s])
        if prefetch:
            self._issue(t + 1)  # overlaps this step's compute
        return self.dev[s]

    def release(self, t: int):
        """Call after step t's work is queued: its slot may be overwritten once
        the compute stream passes this point."""
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self.free[t % 2] = ev


class StepWatchdog:
    """Per-rank watchdog over a timed step loop (a stalled step must
    end the run with its index, not at the launcher's time limit).  The loop
    calls start_step(i) / end_step() around each iteration; a daemon thread
    checks the running iteration against max(factor x the median of the
    iterations done so far, floor_s) -- first_s until three have finished -- and
    on a trip prints the rank, iteration and times and exits the process with
    status 3 (os._exit: no re-exec, no cleanup that could block on the stalled
    device).  With graph replay an iteration mostly waits in the previous step's
    host read, so a stalled step t trips at iteration t or t + 1.  The reference
    has no equivalent (its per-GPU subprocesses are joined without a timeout,
    lib/utils/subprocess.py:84-101)."""

    def __init__(self, rank: int = 0, factor: float = 10.0, floor_s: float = 2.0,
                 first_s: float = 120.0, poll_s: float = 0.05, on_trip=None):
        import threading
        self.rank, self.factor, self.floor_s, self.first_s = rank, factor, floor_s, first_s
        self.poll_s = poll_s
        self.on_trip = on_trip
        self.durations: List[float] = []
        self.current = None  # (iteration, start time)
        self.tripped = None
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._watch, daemon=True)
        self._thread.start()

    def limit(self) -> float:
        with self._lock:
            d = list(self.durations)
        if len(d) < 3:
            return self.first_s
        return max(self.factor * float(np.median(d)), self.floor_s)

    def start_step(self, i: int):
        import time
        with self._lock:
            self.current = (i, time.perf_counter())

    def end_step(self):
        import time
        with self._lock:
            if self.current is not None:
                self.durations.append(time.perf_counter() - self.current[1])
            self.current = None

    def stop(self):
        self._stop.set()
        self._thread.join(timeout=5.0)

    def _watch(self):
        import os
        import sys
        import time
        while not self._stop.wait(self.poll_s):
            lim = self.limit()
            with self._lock:
                cur = self.current
                med = float(np.median(self.durations)) if self.durations else None
            if cur is None:
                continue
            ran = time.perf_counter() - cur[1]
            if ran <= lim:
                continue
            self.tripped = (cur[0], ran, lim)
            print("watchdog: rank %d, timed iteration %d has run %.2f s > limit %.2f s "
                  "(median iteration %s): stopping the rank"
                  % (self.rank, cur[0], ran, lim,
                     "%.1f ms" % (med * 1e3) if med is not None else "n/a"),
                  file=sys.stderr, flush=True)
            if self.on_trip is not None:
                self.on_trip(*self.tripped)
                return
            os._exit(3)
