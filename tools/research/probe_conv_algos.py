#!/usr/bin/env python3
"""Which convolution algorithm MIOpen picks (Find, cudnn.benchmark) for the
benched 3x3 shapes in NCHW and NHWC, against the hand-written MFMA implicit
GEMM (ops.conv3x3_bias_act).  HIP-event times; prints one JSON line per shape.
usage: MIOPEN_LOG_LEVEL=4 tools/probe_conv_algos.py 2> miopen.log
(wino_TFs counts the direct convolution's FLOPs: Winograd does 1/2.25 of them.)"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402


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


def main():
    torch.backends.cudnn.benchmark = True
    shapes = [(16, 256, 200, 336), (16, 256, 100, 168), (16, 256, 50, 84), (1600, 256, 14, 14),
              (16, 64, 200, 336), (16, 128, 100, 168)]
    for N, C, H, W in shapes:
        x = torch.randn(N, C, H, W, device="cuda")
        w = torch.randn(C, C, 3, 3, device="cuda") / (9 * C) ** .5
        flop = 2.0 * N * H * W * C * C * 9
        rec = {"shape": [N, C, H, W]}
        rec["miopen_nchw_ms"] = round(timed(lambda: F.conv2d(x, w, padding=1)), 3)
        xl = x.contiguous(memory_format=torch.channels_last)
        rec["miopen_nhwc_ms"] = round(timed(lambda: F.conv2d(xl, w, padding=1)), 3)
        w2 = ops.conv3x3_weight(w)
        if ops.conv3x3_bias_act(xl, w2, None) is not None:
            rec["mfma_ms"] = round(timed(lambda: ops.conv3x3_bias_act(xl, w2, None)), 3)
        u = ops.conv3x3_wino_weight(w)
        y = ops.conv3x3_wino_bias_act(xl, u, None)
        if y is not None:
            rec["wino_ms"] = round(timed(lambda: ops.conv3x3_wino_bias_act(xl, u, None)), 3)
            ref = F.conv2d(xl, w, padding=1)
            rec["wino_rel_err"] = float((y - ref).abs().max() / ref.abs().max())
        for k in [k for k in rec if k.endswith("_ms")]:
            rec[k.replace("_ms", "_TFs")] = round(flop / rec[k] / 1e9, 1)
        print(json.dumps(rec), flush=True)
        del x, xl


if __name__ == "__main__":
    main()
