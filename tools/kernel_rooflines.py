#!/usr/bin/env python3
"""HBM rooflines of the hand-written epilogue / head / segm kernels, each replayed
alone on its bench shape (16 frames of 800x1333, R-50-FPN) with HIP events on
the launch stream.  Algorithmic bytes per launch are stated per kernel; peak
8 TB/s (MI355X HBM3E).  usage: tools/kernel_rooflines.py [OUT.json]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402

PEAK = 8000.0


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def line(name, nbytes, us, formula):
    gbs = nbytes / us / 1e3
    return {"kernel": name, "algorithmic_bytes": int(nbytes), "bytes_formula": formula,
            "avg_launch_us": round(us, 2), "achieved_GBs": round(gbs, 1),
            "frac": round(gbs / PEAK, 3)}


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    F, C = 16, 256
    out = []
    # RPN head on P2 (16 x 200 x 336): read 4C B, write 4 * 5A B per pixel
    for (H, W) in [(200, 336), (100, 168)]:
        x = torch.randn(F, C, H, W, generator=g, device=dev).contiguous(
            memory_format=torch.channels_last)
        cb = torch.randn(C, generator=g, device=dev)
        w = torch.randn(15, C, generator=g, device=dev) / 16
        b = torch.randn(15, generator=g, device=dev)
        us = timed(lambda: ops.rpn_head(x, cb, w, b, 3))
        npix = F * H * W
        out.append(line("vd::rpn_head_kernel P%dx%d" % (H, W), npix * (4 * C + 4 * 15), us,
                        "pixels * (4*C read + 4*5A written)"))
        del x
    # stem tail: read 16 x 400 x 672 x 64 raw conv1, write 16 x 200 x 336 x 64
    x = torch.randn(F, 64, 400, 672, generator=g, device=dev).contiguous(
        memory_format=torch.channels_last)
    cb = torch.randn(64, generator=g, device=dev)
    us = timed(lambda: ops.bias_relu_maxpool(x, cb))
    out.append(line("vd::bias_relu_maxpool_nhwc4_kernel", x.numel() * 4 + x.numel(), us,
                    "input read once (4 B/elem) + output (1/4 of the elements, 4 B)"))
    del x
    # segm: fused paste+RLE and strings for 16 frames x 100 detections
    M, R = 1600, 28
    masks = torch.rand(M, R, R, generator=g, device=dev)
    xy = torch.rand(M, 2, generator=g, device=dev) * torch.tensor([1200., 700.], device=dev)
    wh = torch.rand(M, 2, generator=g, device=dev) * 300 + 8
    boxes = torch.cat([xy, torch.minimum(xy + wh, torch.tensor([1332., 799.], device=dev)),
                       torch.ones(M, 1, device=dev)], 1).contiguous()
    us = timed(lambda: ops.segm_rle_counts(masks, boxes, 800, 1333), iters=5)
    out.append({"kernel": "vd::segm_rle_kernel (+host retry check)", "detections": M,
                "avg_launch_us": round(us, 2), "us_per_frame": round(us / F, 2),
                "note": "latency-bound per detection (column walks), no frame planes written"})
    json.dump(out, open(sys.argv[1], "w") if len(sys.argv) > 1 else sys.stdout, indent=1)
    if len(sys.argv) > 1:
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
