#!/usr/bin/env python3
"""Run one 3x3 convolution shape a few times (for rocprofv3 PMC passes).
usage: tools/conv_shape_run.py {wino,direct} N C H W [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vosdetectron_amd import ops  # noqa: E402

algo = sys.argv[1]
N, C, H, W = (int(v) for v in sys.argv[2:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 5
x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
w = torch.randn(C, C, 3, 3, device="cuda") / (9 * C) ** .5
if algo == "wino":
    u = ops.conv3x3_wino_weight(w)
    for _ in range(iters):
        ops.conv3x3_wino_bias_act(x, u, None)
else:
    w2 = ops.conv3x3_weight(w)
    for _ in range(iters):
        ops.conv3x3_bias_act(x, w2, None)
torch.cuda.synchronize()
