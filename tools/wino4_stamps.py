#!/usr/bin/env python3
"""Where a F(4x4) chunk's time goes: the STAMP form (VOSDET_WINO4_STAMP=1) of the P2
conv records s_memtime at six points of chunks 8..11 in workgroups < 512; this prints
the mean cycles per phase for the transforming waves (0-3) and the others (4-7):
DMA issue, transform, MFMA loop, end-of-chunk vmcnt wait, barrier."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["VOSDET_WINO4_STAMP"] = "1"
from vosdetectron_amd import ops, _lib  # noqa: E402

shape = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "32x256x200x336x256").split("x")]
N, C, H, W, Co = shape
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
w = torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (3. * C ** .5)
u = ops.conv3x3_wino4_weight(w)
for _ in range(3):
    y = ops.conv3x3_wino4_bias_act(x, u, None)
torch.cuda.synchronize()
lib = ctypes.CDLL(_lib.LIB_PATH)
n = 512 * 8 * 4 * 6
buf = (ctypes.c_ulonglong * n)()
assert lib.vd_research_wino4_stamps(buf, n) == 0
t = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(512, 8, 4, 6)
d = np.diff(t, axis=-1)  # dma, transform, mfma, wait, barrier
names = ["dma_issue", "transform", "mfma_loop", "vmcnt_wait", "barrier"]
rec = {"shape": shape}
for grp, sl in (("waves0_3", slice(0, 4)), ("waves4_7", slice(4, 8))):
    dd = d[:, sl].reshape(-1, 5)
    rec[grp] = {k: round(float(np.median(dd[:, i])), 1) for i, k in enumerate(names)}
    rec[grp]["chunk"] = round(float(np.median(dd.sum(1))), 1)
    rec[grp]["mfma_loop_p90"] = round(float(np.percentile(dd[:, 2], 90)), 1)
print(json.dumps(rec))
