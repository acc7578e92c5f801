#!/usr/bin/env python3
"""Winograd F(4x4,3x3) (csrc/conv3x3_wino4.hip) vs F(2x2,3x3) (conv3x3_wino.hip) on
the step's 3x3 shapes [N, C, H, W, Cout] (32-frame R-50-FPN step): HIP-event us per
call, executed-MFMA fraction of the 157.3 TF/s fp32 matrix peak (F(2x2): 16
positions per 4 outputs; F(4x4): 36 per 16), direct-conv TF/s, max|err| / max|y| vs
torch fp32.  usage: tools/bench_wino4.py [SHAPES...]  (e.g. 32x256x200x336x256)"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402

PEAK = 157.3e12
DEFAULT = ["32x256x200x336x256", "32x256x100x168x256", "32x256x50x84x256",
           "32x128x100x168x128", "32x512x25x42x512", "32x64x200x336x64"]


def timed(fn, iters=10):
    s = torch.cuda.current_stream()
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    shapes = [[int(v) for v in a.split("x")] for a in (sys.argv[1:] or DEFAULT)]
    for N, C, H, W, Co in shapes:
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
            memory_format=torch.channels_last)
        w = torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (9 * C) ** .5
        b = torch.randn(Co, device="cuda", generator=g)
        direct = 2.0 * N * H * W * C * Co * 9
        row = {"shape": [N, C, H, W, Co]}
        ref = F.relu(F.conv2d(x[:2], w, b, padding=1))
        scale = float(ref.abs().max())
        for name, wf, cf, exe in (("wino2", ops.conv3x3_wino_weight, ops.conv3x3_wino_bias_act,
                                   direct * 16 / 36),
                                  ("wino4", ops.conv3x3_wino4_weight,
                                   lambda *a, **k: ops.conv3x3_wino4_bias_act(
                                       *a, mosaic=os.environ.get("WINO4_MOSAIC") or False, **k),
                                   direct * 36 / 144)):
            u = wf(w)
            y = cf(x, u, b, relu=True)
            err = float((y[:2] - ref).abs().max()) / scale
            us = timed(lambda: cf(x, u, b, relu=True, out=y))
            row[name + "_us"] = round(us, 1)
            row[name + "_exec_frac"] = round(exe / (us * 1e-6) / PEAK, 3)
            row[name + "_direct_TFs"] = round(direct / (us * 1e-6) / 1e12, 1)
            row[name + "_rel_err"] = float("%.2e" % err)
            del y
        print(json.dumps(row), flush=True)
        del x


if __name__ == "__main__":
    main()
