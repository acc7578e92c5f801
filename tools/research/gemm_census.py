#!/usr/bin/env python3
"""Every GEMM of one eager F-frame FPN step (F = argv[1], default 32) (ops.gemm_bias_act / gemm_dual_bias_act,
F.linear, torch._addmm_activation): shape, calls, and its time alone with HIP events
(pinned plans), as TF/s against the 157.3 TF/s fp32 matrix peak.  One process."""
import collections
import json
import os
import sys

import torch
import torch.nn.functional as Fn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from vosdetectron_amd import config as vcfg, ops  # noqa: E402
from vosdetectron_amd.weights import build_model  # noqa: E402

seen = collections.OrderedDict()


def log(kind, M, N, K, fn):
    key = (kind, M, N, K)
    if key not in seen:
        seen[key] = [0, fn]
    seen[key][0] += 1


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


dev = torch.device("cuda", 0)
cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
model, sd = build_model(cfg, seed=0, device=dev, channels_last=True)
NF = int(sys.argv[1]) if len(sys.argv) > 1 else 32
pipe, fh, fw = bench.make_pipeline(cfg, model, NF, "nhwc", dev)
frames = torch.from_numpy(bench.synthetic_frames(NF, 1, fh, fw)).to(dev)
pipe.run(frames)
torch.cuda.synchronize()

g0, gd0, lin0, addmm0 = ops.gemm_bias_act, ops.gemm_dual_bias_act, Fn.linear, torch._addmm_activation
fl0 = ops.fpn_lateral_topdown


def fl(lat, wf, bias, top):
    c = (lat.clone(), wf.clone(), bias.clone(), None if top is None else top.clone())
    N, K, H, W = lat.shape
    log("fpn_lateral" + ("+top" if top is not None else ""), N * H * W, 256, K, lambda: fl0(*c))
    return fl0(lat, wf, bias, top)


def g(a, w, bias, residual=None, relu=True, out=None):
    a_, w_, b_ = a.clone(), w.clone(), bias.clone()
    r_ = residual.clone() if residual is not None else None
    log("gemm_bias_act" + ("+res" if residual is not None else ""), a.shape[0], w.shape[0],
        a.shape[1], lambda: g0(a_, w_, b_, residual=r_, relu=relu))
    return g0(a, w, bias, residual=residual, relu=relu, out=out)


def gd(a1, a2, w, bias, *args, **kw):
    c = (a1.clone(), a2.clone(), w.clone(), bias.clone())
    log("gemm_dual", a1.shape[0], w.shape[0], w.shape[1], lambda: gd0(*c))
    return gd0(a1, a2, w, bias, *args, **kw)


def lin(x, w, b=None):
    c = (x.clone(), w.clone(), None if b is None else b.clone())
    log("linear", x.shape[0], w.shape[0], w.shape[1], lambda: lin0(*c))
    return lin0(x, w, b)


def addmm(b, x, w, **kw):
    c = (b.clone(), x.clone(), w.clone())
    log("addmm_act", x.shape[0], w.shape[1], x.shape[1], lambda: addmm0(*c, **kw))
    return addmm0(b, x, w, **kw)


ops.gemm_bias_act, ops.gemm_dual_bias_act, Fn.linear, torch._addmm_activation = g, gd, lin, addmm
ops.fpn_lateral_topdown = fl
pipe.run(frames)
torch.cuda.synchronize()
ops.gemm_bias_act, ops.gemm_dual_bias_act, Fn.linear, torch._addmm_activation = g0, gd0, lin0, addmm0
ops.fpn_lateral_topdown = fl0
tot_ms = tot_gf = 0.0
for (kind, M, N, K), (n, fn) in seen.items():
    ms = timed(fn)
    gf = 2.0 * M * N * K / 1e9
    tot_ms += ms * n
    tot_gf += gf * n
    print(json.dumps({"kind": kind, "M": M, "N": N, "K": K, "calls": n, "ms": round(ms, 4),
                      "TFs": round(gf / ms, 1), "frac": round(gf / ms / 157.3, 3)}), flush=True)
print(json.dumps({"total_ms": round(tot_ms, 3), "total_gflop": round(tot_gf, 1),
                  "TFs": round(tot_gf / tot_ms, 1)}))
