#!/usr/bin/env python3
"""Driver for PMC passes over the MFMA 3x3 conv alone (P2 shape, 5 launches)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from vosdetectron_amd import ops  # noqa: E402

x = torch.randn(16, 256, 200, 336, device="cuda").contiguous(memory_format=torch.channels_last)
w2 = ops.conv3x3_weight(torch.randn(256, 256, 3, 3, device="cuda") / 48)
b = torch.randn(256, device="cuda")
y = torch.empty_like(x)
for _ in range(5):
    ops.conv3x3_bias_act(x, w2, b, relu=True, out=y)
torch.cuda.synchronize()
print("ok")
