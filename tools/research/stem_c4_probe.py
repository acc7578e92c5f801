#!/usr/bin/env python3
"""Stem 7x7/2 conv (16 x 800 x 1344 frames, 64 outputs) on MIOpen: 3 input channels
vs the blob padded to 4 (a zero channel with zero weights: the same convolution),
NCHW and channels_last; HIP-event ms per call and max |diff| vs the 3-channel result."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import vosdetectron_amd  # noqa: E402,F401  (MIOpen find-db / mode defaults)


def timed(f, iters=10):
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


g = torch.Generator(device="cuda").manual_seed(0)
x3 = torch.randn(16, 3, 800, 1344, device="cuda", generator=g)
w3 = torch.randn(64, 3, 7, 7, device="cuda", generator=g) * 0.1
x4 = torch.cat([x3, torch.zeros_like(x3[:, :1])], 1)
w4 = torch.cat([w3, torch.zeros_like(w3[:, :1])], 1)
ref = F.conv2d(x3.contiguous(memory_format=torch.channels_last), w3, None, 2, 3)
for name, x, w in (("c3", x3, w3), ("c4", x4, w4)):
    for cl in (False, True):
        xx = x.contiguous(memory_format=torch.channels_last) if cl else x.contiguous()
        y = F.conv2d(xx, w, None, 2, 3)
        rec = {"input": name, "channels_last": cl,
               "ms": round(timed(lambda: F.conv2d(xx, w, None, 2, 3)), 4),
               "max_abs_diff_vs_c3_cl": float((y - ref).abs().max())}
        print(json.dumps(rec), flush=True)
