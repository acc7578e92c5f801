#!/usr/bin/env python3
"""A/B of the 256 -> 256 3x3 convolutions of a 16-frame R-50-FPN step: the
hand-written MFMA implicit GEMM with the bias (+ReLU) epilogue (csrc/conv3x3.hip)
vs what the engine runs today (MIOpen conv without bias + vd_bias_act).  HIP
events; fraction of the 157.3 TF/s fp32 matrix peak.  usage: tools/bench_conv3x3.py [out.json]"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402

PEAK = 157.3e12
SHAPES = [(int(v) for v in t.split("x")) for t in os.environ["CONV3X3_SHAPES"].split(",")] \
    if os.environ.get("CONV3X3_SHAPES") else [(16, 256, 200, 336, 256), (16, 256, 100, 168, 256), (16, 256, 50, 84, 256),
          (1600, 256, 14, 14, 256), (16, 256, 25, 42, 256), (16, 128, 100, 168, 128),
          (16, 64, 200, 336, 64)]


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
    torch.backends.cudnn.benchmark = True
    rows = []
    for N, C, H, W, Co in SHAPES:
        x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Co, C, 3, 3, device="cuda") / (9 * C) ** .5).contiguous(
            memory_format=torch.channels_last)
        b = torch.randn(Co, device="cuda")
        w2 = ops.conv3x3_weight(w)
        y = torch.empty(N, Co, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
        flops = 2 * N * H * W * C * Co * 9
        t_ref = timed(lambda: ops.bias_act_(F.conv2d(x, w, None, padding=1), b, relu=True))
        ref = ops.bias_act_(F.conv2d(x, w, None, padding=1), b, relu=True)
        row = {"shape": [N, C, H, W, Co], "miopen_plus_bias_act_us": round(t_ref, 1),
               "miopen_frac": round(flops / (t_ref * 1e-6) / PEAK, 3)}
        for v in os.environ.get("CONV3X3_VARIANTS", "1,2").split(","):
            os.environ["VOSDET_CONV3X3_VARIANT"] = v
            t_own = timed(lambda: ops.conv3x3_bias_act(x, w2, b, relu=True, out=y))
            row["mfma_v%s_us" % v] = round(t_own, 1)
            row["mfma_v%s_frac" % v] = round(flops / (t_own * 1e-6) / PEAK, 3)
            row["maxdiff_v%s" % v] = float((y - ref).abs().max())
        os.environ.pop("VOSDET_CONV3X3_VARIANT")
        print(json.dumps(row), flush=True)
        rows.append(row)
        del x, y, ref
        torch.cuda.empty_cache()
    if len(sys.argv) > 1:
        json.dump(rows, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
