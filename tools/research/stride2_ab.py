#!/usr/bin/env python3
"""The ResNet stages' first-block strided 1x1 convs (conv1 + downsample, stride 2,
16 frames at 800 x 1333): MIOpen / CK strided convs vs the every-other-pixel copy +
two hipBLASLt GEMMs (modeling._subsample, _gemm_conv1x1); HIP events, one process."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from vosdetectron_amd import modeling  # noqa: E402


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


for (C, inner, out, H, W) in [(256, 128, 512, 200, 336), (512, 256, 1024, 100, 168),
                              (1024, 512, 2048, 50, 84)]:
    x = torch.randn(16, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    w1 = torch.randn(inner, C, 1, 1, device="cuda") / C ** .5
    wd = torch.randn(out, C, 1, 1, device="cuda") / C ** .5
    b1, bd = torch.randn(inner, device="cuda"), torch.randn(out, device="cuda")
    w1_, wd_ = w1.view(inner, C).contiguous(), wd.view(out, C).contiguous()

    def conv():
        return F.relu(F.conv2d(x, w1, b1, stride=2)), F.conv2d(x, wd, bd, stride=2)

    def gemm():
        xs = modeling._subsample(x, (2, 2))
        return (modeling._gemm_conv1x1(xs, w1_, b1, relu=True),
                modeling._gemm_conv1x1(xs, wd_, bd, relu=False))

    a, b = conv(), gemm()
    rec = {"C": C, "inner": inner, "out": out, "H": H, "W": W,
           "conv_ms": round(timed(conv), 4), "gemm_ms": round(timed(gemm), 4),
           "subsample_ms": round(timed(lambda: modeling._subsample(x, (2, 2))), 4),
           "max_rel": [float(((p - q).abs().max() / q.abs().max())) for p, q in zip(b, a)]}
    print(json.dumps(rec), flush=True)
