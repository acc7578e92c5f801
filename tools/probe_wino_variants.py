#!/usr/bin/env python3
"""A/B of the Winograd kernel's schedule variants (VOSDET_WINO_VARIANT, see
csrc/conv3x3_wino.hip) in ONE process on one box (MFMA loops differ by up to
~12 % across MI355X devices, so cross-box comparisons are not A/B): HIP-event
times per shape and the max relative error vs torch fp32 conv2d."""
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
    variants = [int(v) for v in (sys.argv[1:] or ["9", "1", "0", "8", "11", "13", "6"])]
    shapes = [(16, 256, 200, 336), (16, 256, 100, 168), (1600, 256, 14, 14), (16, 64, 200, 336)]
    for N, C, H, W in shapes:
        x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
        w = torch.randn(C, C, 3, 3, device="cuda") / (9 * C) ** .5
        b = torch.randn(C, device="cuda")
        ref = F.relu(F.conv2d(x, w, b, padding=1))
        u = ops.conv3x3_wino_weight(w)
        rec = {"shape": [N, C, H, W]}
        for v in variants:
            os.environ["VOSDET_WINO_VARIANT"] = str(v)
            y = ops.conv3x3_wino_bias_act(x, u, b, relu=True)
            err = float((y - ref).abs().max() / ref.abs().max())
            ms = timed(lambda: ops.conv3x3_wino_bias_act(x, u, b, relu=True))
            rec["v%d" % v] = [round(ms, 3), "%.1e" % err]
        print(json.dumps(rec), flush=True)
        del x, ref, y


if __name__ == "__main__":
    main()
