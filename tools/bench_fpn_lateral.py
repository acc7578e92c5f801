#!/usr/bin/env python3
"""FPN top-down lateral step at the benched 32-frame shapes: the fused MFMA kernel
(vd_fpn_lateral_topdown) vs the previous route (vd_gemm_bias_act -- pinned plan /
search -- then vd_bias_act's nearest-2x add), HIP events over 20 launches each.
One JSON line per shape: ms, TF/s and fraction of the 157.3 TF/s fp32 matrix peak."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402

PEAK = 157.3


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


F_ = int(sys.argv[1]) if len(sys.argv) > 1 else 32
TAG = os.environ.get("VOSDET_LATERAL_NB", "auto")
for K, H, W in [(256, 200, 336), (512, 100, 168), (1024, 50, 84)]:
    g = torch.Generator(device="cuda").manual_seed(K)
    lat = torch.randn(F_, K, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(256, K, device="cuda", generator=g) / K ** .5
    b = torch.randn(256, device="cuda", generator=g)
    t = torch.randn(F_, 256, H // 2, W // 2, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    wf = ops.fpn_lateral_weight(w)
    M = F_ * H * W
    a2 = lat.permute(0, 2, 3, 1).reshape(M, K)

    def old():
        y = ops.gemm_bias_act(a2, w, b, relu=False)
        y = y.view(F_, H, W, 256).permute(0, 3, 1, 2)
        return ops.bias_act_(y, None, t, relu=False, upsample_residual=True)

    def gemm_only():
        return ops.gemm_bias_act(a2, w, b, relu=False)

    def new():
        return ops.fpn_lateral_topdown(lat, wf, b, t)

    def new_notop():
        return ops.fpn_lateral_topdown(lat, wf, b, None)

    ref = old()
    got = new()
    torch.cuda.synchronize()
    err = float((got - ref).abs().max())
    gf = 2. * M * K * 256 / 1e9
    r = {"nb": TAG, "K": K, "H": H, "W": W, "frames": F_, "gflop": round(gf, 1), "max_abs_diff": err}
    for name, fn in (("fused", new), ("fused_no_top", new_notop), ("old_gemm_plus_add", old),
                     ("old_gemm_only", gemm_only)):
        ms = timed(fn)
        r[name + "_ms"] = round(ms, 4)
        r[name + "_frac"] = round(gf / ms / PEAK, 3)
    print(json.dumps(r), flush=True)
    del lat, t, ref, got, a2
