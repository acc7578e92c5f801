#!/usr/bin/env python3
"""1x1 convolutions of the R-50-FPN body (channels_last fp32, 8 frames): MIOpen
conv + vd_bias_act epilogue vs one hipBLASLt GEMM with a fused bias(+ReLU)
epilogue (torch._addmm_activation) on the NHWC view."""
import json
import os
import sys
import time

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


N = 8
shapes = [(64, 200, 336, 256), (256, 200, 336, 64), (256, 200, 336, 256), (512, 100, 168, 128),
          (128, 100, 168, 512), (1024, 50, 84, 256), (256, 50, 84, 1024), (2048, 25, 42, 512),
          (512, 25, 42, 2048), (256, 100, 168, 256)]
for ci, h, w, co in shapes:
    x = torch.randn(N, ci, h, w, device=dev).to(memory_format=torch.channels_last)
    wt = (torch.randn(co, ci, 1, 1, device=dev) / ci ** .5).to(memory_format=torch.channels_last)
    b = torch.randn(co, device=dev)
    x2 = x.permute(0, 2, 3, 1).reshape(-1, ci)
    wm = wt.view(co, ci).t()
    r = {"shape": [N, ci, h, w, co], "gflop": 2 * N * h * w * ci * co / 1e9}
    r["conv_biasact_ms"] = timeit(lambda: ops.bias_act_(F.conv2d(x, wt), b, relu=True))
    r["gemm_bias_relu_ms"] = timeit(lambda: torch._addmm_activation(b, x2, wm))
    r["gemm_bias_ms"] = timeit(lambda: torch.addmm(b, x2, wm))
    a = ops.bias_act_(F.conv2d(x, wt), b, relu=True).permute(0, 2, 3, 1).reshape(-1, co)
    r["maxdiff"] = float((a - torch._addmm_activation(b, x2, wm)).abs().max())
    print(json.dumps(r), flush=True)
