#!/usr/bin/env python3
"""Which convolutions of one eager 16-frame FPN step still go to torch (MIOpen / CK):
wraps F.conv2d / F.conv_transpose2d / F.linear and prints their shapes and the
3x3 route counts (modeling.ROUTE_COUNTS).  One process, one GPU."""
import collections
import json
import os
import sys

import torch
import torch.nn.functional as Fn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from vosdetectron_amd import config as vcfg, modeling  # noqa: E402
from vosdetectron_amd.weights import build_model  # noqa: E402

calls = collections.Counter()


def wrap(name, fn):
    def f(x, w, *a, **k):
        calls[(name, tuple(x.shape), tuple(w.shape), str(a[1:3] if len(a) > 1 else k))] += 1
        return fn(x, w, *a, **k)
    return f


dev = torch.device("cuda", 0)
cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
model, sd = build_model(cfg, seed=0, device=dev, channels_last=True)
pipe, fh, fw = bench.make_pipeline(cfg, model, 16, "nhwc", dev)
frames = torch.from_numpy(bench.synthetic_frames(16, 1, fh, fw)).to(dev)
pipe.run(frames)
torch.cuda.synchronize()
Fn.conv2d = wrap("conv2d", Fn.conv2d)
Fn.conv_transpose2d = wrap("conv_transpose2d", Fn.conv_transpose2d)
torch.nn.functional.conv2d = Fn.conv2d
modeling.ROUTE_COUNTS.clear()
pipe.run(frames)
torch.cuda.synchronize()
for k, n in sorted(calls.items()):
    print(json.dumps({"op": k[0], "x": k[1], "w": k[2], "args": k[3], "n": n}))
print(json.dumps({"routes": modeling.ROUTE_COUNTS}))
