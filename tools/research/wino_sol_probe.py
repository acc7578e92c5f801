#!/usr/bin/env python3
"""Speed-of-light probes of the Winograd kernel (VOSDET_WINO_PROBE, wrong results
by design): times the P2 shape with parts of the chunk loop removed, one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from vosdetectron_amd import ops  # noqa: E402


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


N, C, H, W = 16, 256, 200, 336
x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
u = ops.conv3x3_wino_weight(torch.randn(C, C, 3, 3, device="cuda"))
rec = {}
for pr in os.environ.get("PROBES", "0,2,4,8,32,36,12,46").split(","):
    os.environ["VOSDET_WINO_PROBE"] = pr
    rec[pr] = round(timed(lambda: ops.conv3x3_wino_bias_act(x, u, None)), 3)
print(json.dumps({"shape": [N, C, H, W], "probe_ms": rec,
                  "legend": "2 no patch reads, 4 no barrier, 8 no U loads, 32 no patch DMA"}))
