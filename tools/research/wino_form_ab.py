#!/usr/bin/env python3
"""Winograd F(2x2,3x3) forms A/B (csrc/conv3x3_wino.hip): form 2 (32 tiles, 4 waves,
2 stages, two workgroups per CU) vs form 3 (64 tiles, 8 waves, 3 stages, one per
CU) at the benched shapes in the layout the engine picks (modeling.conv3x3_route).
Checks the two forms are bit-identical and both within 2e-5 of torch fp32; HIP
events per launch; executed-MFMA fraction of the 157.3 TF/s fp32 peak (4/9 of
the direct-conv FLOPs).  usage: tools/wino_form_ab.py [out.json]"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import modeling, ops  # noqa: E402

PEAK = 157.3e12
SHAPES = [(16, 256, 200, 336), (16, 256, 100, 168), (16, 256, 50, 84), (1600, 256, 14, 14),
          (16, 64, 200, 336), (16, 128, 100, 168), (16, 512, 25, 42), (16, 256, 25, 42),
          (16, 256, 13, 21)]


def timed(fn, iters=10):
    for _ in range(2):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    rows = []
    forms = os.environ.get("WINO_FORMS", "2,3").split(",")
    for N, C, H, W in SHAPES:
        algo, mos = modeling.conv3x3_route(N, C, C, H, W)
        g = torch.Generator(device="cuda").manual_seed(N + C + H)
        x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
            memory_format=torch.channels_last)
        w = torch.randn(C, C, 3, 3, device="cuda", generator=g) / (3. * C ** .5)
        b = torch.randn(C, device="cuda", generator=g)
        u = ops.conv3x3_wino_weight(w)
        ref = F.relu(F.conv2d(x, w, b, padding=1))
        scale = max(1., float(ref.abs().max()))
        exe = 2.0 * N * H * W * C * C * 4
        row = {"shape": [N, C, H, W], "route": [algo, mos]}
        outs = {}
        for f in forms:
            os.environ["VOSDET_WINO_FORM"] = f
            y = ops.conv3x3_wino_bias_act(x, u, b, relu=True, mosaic=mos)
            torch.cuda.synchronize()
            outs[f] = y.clone()
            t = timed(lambda: ops.conv3x3_wino_bias_act(x, u, b, relu=True, mosaic=mos, out=y))
            row["form%s_us" % f] = round(t, 1)
            row["form%s_frac" % f] = round(exe / (t * 1e-6) / PEAK, 4)
            row["form%s_err" % f] = float((outs[f] - ref).abs().max()) / scale
        os.environ.pop("VOSDET_WINO_FORM", None)
        if len(forms) > 1:
            row["bit_identical"] = bool(torch.equal(outs[forms[0]], outs[forms[1]]))
        print(json.dumps(row), flush=True)
        rows.append(row)
        del x, y, ref, outs
        torch.cuda.empty_cache()
    if len(sys.argv) > 1:
        json.dump(rows, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
