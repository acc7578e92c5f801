#!/usr/bin/env python3
"""Why C4's res5-head 3x3 (8000 RoI maps of 7 x 7, 512 -> 512) runs at ~0.34 of the
executed-MFMA peak in the Winograd 2-D mosaic: variants of the shape and launch
mapping, HIP-event ms per call."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from vosdetectron_amd import ops  # noqa: E402


def timed(f, iters=10):
    for _ in range(2):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def run(N, C, H, W, env=None, mosaic="2d"):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    w = torch.randn(C, C, 3, 3, device="cuda", generator=g) / (9 * C) ** .5
    b = torch.randn(C, device="cuda", generator=g)
    u = ops.conv3x3_wino_weight(w)
    out = torch.empty_like(x)
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        t = timed(lambda: ops.conv3x3_wino_bias_act(x, u, b, relu=True, out=out, mosaic=mosaic))
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    tiles = -(-H // 2) * -(-W // 2) * N
    tf = tiles * 16 * C * C * 2 / t / 1e9
    return {"shape": [N, C, H, W], "env": env or {}, "mosaic": mosaic, "ms": round(t, 3),
            "executed_TFs": round(tf, 1)}


for args in [((8000, 512, 7, 7),), ((8000, 512, 7, 7), {"VOSDET_WINO_MAP": "0"}),
             ((8000, 512, 8, 8),), ((8000, 256, 7, 7),), ((2000, 512, 7, 7),),
             ((8000, 512, 14, 14),), ((16, 512, 200, 336),)]:
    print(json.dumps(run(*args[0], *args[1:])), flush=True)
    torch.cuda.empty_cache()
