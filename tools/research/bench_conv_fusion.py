#!/usr/bin/env python3
"""Microbenchmark: conv + bias + relu (+ residual) variants on MI355X, channels_last fp32."""
import json, sys, time
import os

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = "cuda"

def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3

shapes = [  # (N, Cin, H, W, Cout, k, stride)
    (16, 64, 200, 336, 64, 3, 1),
    (16, 256, 200, 336, 64, 1, 1),
    (16, 64, 200, 336, 256, 1, 1),
    (16, 128, 100, 168, 128, 3, 1),
    (16, 256, 50, 84, 256, 3, 1),
    (16, 256, 200, 336, 256, 3, 1),
    (1600, 256, 14, 14, 256, 3, 1),
    (16, 3, 800, 1344, 64, 7, 2),
]
res = []
for (N, Ci, H, W, Co, k, s) in shapes:
    x = torch.randn(N, Ci, H, W, device=dev).to(memory_format=torch.channels_last)
    w = torch.randn(Co, Ci, k, k, device=dev).to(memory_format=torch.channels_last) * 0.05
    b = torch.randn(Co, device=dev)
    p = k // 2
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    z = torch.randn(N, Co, Ho, Wo, device=dev).to(memory_format=torch.channels_last)
    r = {"shape": [N, Ci, H, W, Co, k, s]}
    r["conv_nobias"] = timeit(lambda: F.conv2d(x, w, None, s, p))
    r["conv_vdepi"] = timeit(lambda: ops.bias_act_(F.conv2d(x, w, None, s, p), b, relu=True))
    r["conv_vdepi_res"] = timeit(lambda: ops.bias_act_(F.conv2d(x, w, None, s, p), b, z, relu=True))
    r["conv_bias_relu"] = timeit(lambda: F.relu_(F.conv2d(x, w, b, s, p)))
    r["conv_bias_add_relu"] = timeit(lambda: F.relu_(F.conv2d(x, w, b, s, p).add_(z)))
    try:
        r["miopen_conv_relu"] = timeit(lambda: torch.miopen_convolution_relu(x, w, b, (s, s), (p, p), (1, 1), 1))
        r["miopen_conv_add_relu"] = timeit(lambda: torch.miopen_convolution_add_relu(x, w, z, 1.0, b, (s, s), (p, p), (1, 1), 1))
        a = torch.miopen_convolution_relu(x, w, b, (s, s), (p, p), (1, 1), 1)
        ref = F.relu(F.conv2d(x, w, b, s, p))
        r["miopen_relu_maxdiff"] = float((a - ref).abs().max())
    except Exception as e:
        r["miopen_err"] = str(e)[:200]
    r["gflop"] = 2 * N * Co * Ho * Wo * Ci * k * k / 1e9
    res.append(r)
    print(json.dumps(r), flush=True)
