#!/usr/bin/env python3
"""Where the ring RoIAlign kernel (variant 60) spends its time, from the research
build's per-wave cycle accounting (VOSDET_RESEARCH_LIB=.../libvosdet_research.so):
loaders -- waiting for a slot to retire, waiting for their DMA; consumers --
waiting for a slot to be published, working on it.  One 8-frame launch (bench's
roofline workload) after warm-up."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("VOSDET_ROIALIGN_VARIANT", "60")
from bench import fpn_levels_np, synthetic_rois  # noqa: E402
from vosdetectron_amd import _lib, ops  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda")
    sizes = [(200, 336), (100, 168), (50, 84), (25, 42)]
    scales = [1. / 4, 1. / 8, 1. / 16, 1. / 32]
    g = torch.Generator(device=dev).manual_seed(1)
    pyr = [torch.randn((8, h, w, 256), generator=g, device=dev) for h, w in sizes]
    rois = np.concatenate([synthetic_rois(f, 1000, batch_idx=f) for f in range(8)])
    lv = fpn_levels_np(rois) - 2
    rt, lt = torch.from_numpy(rois).to(dev), torch.from_numpy(lv.astype(np.int32)).to(dev)
    out = torch.empty((8000, 7, 7, 256), device=dev)
    for _ in range(3):
        ops.roi_align_fpn(pyr, scales, rt, lt, 7, 2, out=out, out_layout="nhwc")
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (256 * 16 * 4))()
    _lib.check(_lib.lib().vd_research_ring_stats(buf, len(buf)), "stats")
    a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 16, 4).astype(np.float64)
    nl = int(os.environ.get("RING_NL", "5"))
    L, C = a[:, :nl], a[:, nl:]
    res = {"cycles_total_max": float(a[:, :, 0].max()),
           "loader": {"total": float(L[..., 0].mean()), "wait_retire": float(L[..., 1].mean()),
                      "wait_dma": float(L[..., 2].mean()), "items": float(L[..., 3].mean()),
                      "dma_cycles_per_item": float(L[..., 2].sum() / L[..., 3].sum())},
           "consumer": {"total": float(C[..., 0].mean()), "wait_publish": float(C[..., 1].mean()),
                        "work": float(C[..., 2].mean()), "tasks": float(C[..., 3].mean()),
                        "work_cycles_per_task": float(C[..., 2].sum() / max(C[..., 3].sum(), 1))}}
    print(json.dumps(res))
