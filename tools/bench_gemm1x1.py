#!/usr/bin/env python3
"""A/B of the bottleneck 1x1-conv GEMMs with the fused epilogue (16 frames,
R-50-FPN shapes): the hand-written MFMA kernel (csrc/gemm1x1.hip,
VOSDET_GEMM_MFMA=1) vs hipBLASLt's best searched algorithm (VOSDET_GEMM_MFMA=0).
HIP events per launch; algorithmic bytes (A + W + R + D) and flops give the
per-shape roofline fractions.  usage: tools/bench_gemm1x1.py [out.json]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402

HBM, MFMA = 8000e9, 157.3e12
SHAPES = [  # (M, K, N, residual): P2 / P3 bottleneck GEMMs of a 16-frame step
    (16 * 200 * 336, 64, 256, True),   # res2 conv3 + identity / downsample residual
    (16 * 200 * 336, 256, 64, False),  # res2 conv1 (blocks 1, 2)
    (16 * 200 * 336, 64, 64, False),   # res2 block 0 conv1
    (16 * 200 * 336, 64, 256, False),  # res2 downsample shape
    (16 * 100 * 168, 128, 512, True),  # res3 conv3 + residual (N split over 4 workgroups)
]


def timed(fn, iters=20):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    rows = []
    for M, K, N, res in SHAPES:
        a = torch.randn(M, K, device="cuda", generator=g)
        w = torch.randn(N, K, device="cuda", generator=g) / K ** .5
        b = torch.randn(N, device="cuda", generator=g)
        r = torch.randn(M, N, device="cuda", generator=g) if res else None
        d = torch.empty(M, N, device="cuda")
        row = {"M": M, "K": K, "N": N, "residual": res}
        nbytes = 4 * (M * K + N * K + M * N * (2 if res else 1))
        flops = 2 * M * N * K
        outs = {}
        for mode in ("0", "1"):
            os.environ["VOSDET_GEMM_MFMA"] = mode[0]
            us = timed(lambda: ops.gemm_bias_act(a, w, b, residual=r, relu=True, out=d))
            outs[mode] = d.clone()
            key = {"0": "hipblaslt", "1": "mfma"}[mode]
            row[key + "_us"] = round(us, 1)
            row[key + "_hbm_frac"] = round(nbytes / (us * 1e-6) / HBM, 3)
            row[key + "_mfma_frac"] = round(flops / (us * 1e-6) / MFMA, 3)
        row["maxdiff"] = float((outs["0"] - outs["1"]).abs().max())
        row["bound_us"] = round(max(nbytes / HBM, flops / MFMA) * 1e6, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
        del a, w, b, r, d, outs
        torch.cuda.empty_cache()
    # res2 block 0 tail: MIOpen downsample conv + GEMM with that residual vs the
    # two-operand MFMA GEMM (conv3 + downsample summed in the accumulators)
    import torch.nn.functional as F
    M = 16 * 200 * 336
    h = torch.randn(M, 64, device="cuda", generator=g)
    x = torch.randn(16, 64, 200, 336, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    x2 = x.permute(0, 2, 3, 1).reshape(M, 64)
    w3 = torch.randn(256, 64, device="cuda", generator=g) / 8
    wd = torch.randn(256, 64, device="cuda", generator=g) / 8
    b = torch.randn(256, device="cuda", generator=g)
    wcat = torch.cat([w3, wd], 1).contiguous()
    d = torch.empty(M, 256, device="cuda")

    def two_step():
        r = F.conv2d(x, wd.view(256, 64, 1, 1)).permute(0, 2, 3, 1).reshape(M, 256)
        ops.gemm_bias_act(h, w3, b, residual=r, relu=True, out=d)
    row = {"what": "res2 block-0 tail (16 frames)", "downsample_conv_plus_gemm_us":
           round(timed(two_step), 1),
           "dual_mfma_us": round(timed(lambda: ops.gemm_dual_bias_act(h, x2, wcat, b, out=d)),
                                 1)}
    print(json.dumps(row), flush=True)
    rows.append(row)
    if len(sys.argv) > 1:
        json.dump(rows, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
