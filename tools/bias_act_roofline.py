#!/usr/bin/env python3
"""Roofline of the remaining vd_bias_act launches of one bench step (VERDICT r1
weak #3): record every ops.bias_act_ call of one e2e_mask_rcnn_R-50-FPN_1x
step (16 frames, channels_last, GEMM epilogue on), then replay each distinct
shape alone with HIP events.  Algorithmic bytes per launch: read x + write x
(4 B each per element) + the residual (mode 1: same shape, mode 2: nearest-2x
source, a quarter) + bias vectors.  Prints/writes one JSON record.

usage: python tools/bias_act_roofline.py [out.json]"""
import collections
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from vosdetectron_amd import ops  # noqa: E402


def main():
    from bench import synthetic_frames
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.engine import FramePipeline
    from vosdetectron_amd.weights import build_model
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
    model, _ = build_model(cfg, device=dev, channels_last=True)
    F = 16
    pipe = FramePipeline(model, cfg, batch=F, channels_last=True, device=dev)
    frames = torch.from_numpy(synthetic_frames(F, 1)).to(dev)
    pipe.run(frames)  # warm-up (algorithm search)
    calls = []
    orig = ops.bias_act_

    def rec(x, bias, residual=None, residual_bias=None, relu=True, upsample_residual=False):
        mode = 0 if residual is None else (2 if upsample_residual else 1)
        calls.append((tuple(x.shape), mode, residual_bias is not None, bool(relu)))
        return orig(x, bias, residual, residual_bias, relu, upsample_residual)

    ops.bias_act_ = rec
    try:
        pipe.run(frames)
    finally:
        ops.bias_act_ = orig
    torch.cuda.synchronize()
    shapes = collections.Counter(calls)
    rows, tot_t, tot_b = [], 0., 0
    for (shape, mode, rb, relu), n in sorted(shapes.items(), key=lambda kv: -np.prod(kv[0][0])):
        N, C, H, W = shape
        x = torch.randn(shape, device=dev).contiguous(memory_format=torch.channels_last)
        b = torch.randn(C, device=dev)
        res = None
        if mode == 1:
            res = torch.randn(shape, device=dev).contiguous(memory_format=torch.channels_last)
        elif mode == 2:
            res = torch.randn((N, C, H // 2, W // 2), device=dev).contiguous(
                memory_format=torch.channels_last)
        rbias = torch.randn(C, device=dev) if rb else None
        for _ in range(3):
            orig(x, b, res, rbias, relu, mode == 2)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            orig(x, b, res, rbias, relu, mode == 2)
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / reps
        el = N * C * H * W
        nbytes = 8 * el + (4 * el if mode == 1 else el if mode == 2 else 0) + 4 * C * (1 + rb)
        rows.append({"shape_nchw": list(shape), "residual_mode": mode, "calls_per_step": n,
                     "bytes_per_launch": int(nbytes), "us_per_launch": round(t * 1e6, 2),
                     "GBs": round(nbytes / t / 1e9, 1), "frac_of_8TBs": round(nbytes / t / 8e12, 3)})
        tot_t += n * t
        tot_b += n * nbytes
    rec_ = {"step": "e2e_mask_rcnn_R-50-FPN_1x, 16 frames 800x1333, channels_last, "
                    "GEMM epilogue %s" % os.environ.get("VOSDET_GEMM_EPILOGUE", "1"),
            "launches_per_step": len(calls), "ms_per_step_replayed": round(tot_t * 1e3, 3),
            "bytes_per_step": int(tot_b), "GBs_overall": round(tot_b / tot_t / 1e9, 1),
            "frac_overall": round(tot_b / tot_t / 8e12, 3), "launches": rows}
    print(json.dumps(rec_, indent=1))
    if len(sys.argv) > 1:
        json.dump(rec_, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
