#!/usr/bin/env python3
"""Per-convolution / GEMM roofline of one bench step (e2e_mask_rcnn_R-50-FPN_1x,
16 frames 800x1333, channels_last, GEMM epilogue on).  F.conv2d,
F.conv_transpose2d and F.linear are wrapped for one steady-state step: each
call is bracketed by HIP events on the current stream and its FLOPs are
2 * (output elements) * Cin/groups * kh * kw (2*M*N*K for linear).  The
C-ABI routes -- the GEMM-epilogue 1x1 convs (ops.gemm_bias_act: hipBLASLt or
csrc/gemm1x1.hip), the two-operand GEMM (ops.gemm_dual_bias_act), the MFMA
3x3 conv (ops.conv3x3_bias_act, csrc/conv3x3.hip), the Winograd 3x3 conv
(ops.conv3x3_wino_bias_act, csrc/conv3x3_wino.hip: FLOPs counted as the
direct convolution's, so its TF/s can exceed the fp32 peak) and the RPN head
(ops.rpn_head) -- are wrapped the same way.  Peak:
157.3 TFLOP/s fp32 MFMA (MI355X_MICROARCH.md; no xf32 on gfx950).

usage: python tools/conv_roofline.py [out.json]"""
import collections
import json
import os
import sys

import torch
import torch.nn.functional as Fn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = 157.3e12


def main():
    from bench import synthetic_frames
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd import ops
    from vosdetectron_amd.engine import FramePipeline
    from vosdetectron_amd.weights import build_model
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    cfg = vcfg.get(os.environ.get("CFG", "e2e_mask_rcnn_R-50-FPN_1x"))
    model, _ = build_model(cfg, device=dev, channels_last=True)
    F = int(os.environ.get("FRAMES", "16"))
    pipe = FramePipeline(model, cfg, batch=F, channels_last=True, device=dev)
    frames = torch.from_numpy(synthetic_frames(F, 1)).to(dev)
    for _ in range(2):
        pipe.run(frames)
    torch.cuda.synchronize()
    recs = []

    def timed(kind, fn, flops_of):
        def w(*a, **k):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            y = fn(*a, **k)
            e1.record()
            recs.append((kind, e0, e1, flops_of(y, *a, **k)))
            return y
        return w

    def conv_key(y, x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
        kh, kw = w.shape[2:]
        fl = 2.0 * y.numel() * (w.shape[1]) * kh * kw
        return fl, "x%s w%s s%s g%d" % (list(x.shape), list(w.shape), stride, groups)

    def convt_key(y, x, w, b=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1):
        kh, kw = w.shape[2:]
        fl = 2.0 * x.numel() * w.shape[1] * kh * kw
        return fl, "x%s w%s (transposed)" % (list(x.shape), list(w.shape))

    def lin_key(y, x, w, b=None):
        return 2.0 * y.numel() * w.shape[1], "x%s w%s" % (list(x.shape), list(w.shape))

    def gemm_key(y, A, M, K, Wt, N, *a, **k):
        return 2.0 * M * N * K, "gemm M%d N%d K%d" % (M, N, K)

    orig = (Fn.conv2d, Fn.conv_transpose2d, Fn.linear, getattr(ops, "_gemm_launch", None))
    Fn.conv2d = timed("conv", orig[0], conv_key)
    Fn.conv_transpose2d = timed("deconv", orig[1], convt_key)
    Fn.linear = timed("linear", orig[2], lin_key)
    gl = getattr(ops, "gemm_bias_act", None)
    if gl is not None:
        def gk(y, A, W, bias, residual=None, relu=True, out=None):
            M, K = A.shape
            return 2.0 * M * W.shape[0] * K, "gemm_bias_act M%d N%d K%d%s" % (
                M, W.shape[0], K, " +res" if residual is not None else "")
        ops.gemm_bias_act = timed("gemm_epi", gl, gk)
    cl = ops.conv3x3_bias_act

    def ck(y, x, w2, bias, relu=False, out=None):
        if y is None:
            return 0.0, "conv3x3 (fell back)"
        N, C, H, W = x.shape
        return 2.0 * N * H * W * y.shape[1] * C * 9, "conv3x3_mfma x%s Cout%d%s" % (
            list(x.shape), y.shape[1], " +bias" if bias is not None else "")
    ops.conv3x3_bias_act = timed("conv3x3_mfma", cl, ck)
    wl = ops.conv3x3_wino_bias_act

    def wk(y, x, u, bias, relu=False, out=None, mosaic=False):
        if y is None:
            return 0.0, "conv3x3_wino (fell back)"
        N, C, H, W = x.shape
        return 2.0 * N * H * W * y.shape[1] * C * 9, "conv3x3_wino x%s Cout%d%s%s" % (
            list(x.shape), y.shape[1], " +bias" if bias is not None else "",
            " mosaic" if mosaic else "")
    ops.conv3x3_wino_bias_act = timed("conv3x3_wino", wl, wk)
    dl = ops.gemm_dual_bias_act

    def dk(y, a1, a2, w, bias, relu=True, out=None):
        M = a1.shape[0]
        return 2.0 * M * w.shape[0] * w.shape[1], "gemm_dual M%d N%d K%d+%d" % (
            M, w.shape[0], a1.shape[1], a2.shape[1])
    ops.gemm_dual_bias_act = timed("gemm_dual", dl, dk)
    rl = ops.rpn_head

    def rk(y, x_raw, conv_bias, w, b, *a, **k):
        N, C, H, W = x_raw.shape
        return 2.0 * N * H * W * C * w.shape[0], "rpn_head x[%d,%d,%d,%d] 5A=%d" % (
            N, C, H, W, w.shape[0])
    ops.rpn_head = timed("rpn_head", rl, rk)
    try:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        pipe.run(frames)
        e1.record()
        torch.cuda.synchronize()
    finally:
        Fn.conv2d, Fn.conv_transpose2d, Fn.linear = orig[:3]
        if gl is not None:
            ops.gemm_bias_act = gl
        ops.conv3x3_bias_act, ops.gemm_dual_bias_act, ops.rpn_head = cl, dl, rl
        ops.conv3x3_wino_bias_act = wl
    step_ms = e0.elapsed_time(e1)
    agg = collections.OrderedDict()
    for kind, a, b, (fl, key) in recs:
        t = a.elapsed_time(b) * 1e3
        r = agg.setdefault((kind, key), [0, 0.0, 0.0])
        r[0] += 1
        r[1] += t
        r[2] += fl
    rows, tot_us, tot_fl = [], 0.0, 0.0
    for (kind, key), (n, us, fl) in agg.items():
        rows.append({"kind": kind, "shape": key, "calls": n, "us": round(us, 1),
                     "GFLOP": round(fl / 1e9, 2), "TFs": round(fl / (us * 1e-6) / 1e12, 1),
                     "frac_of_peak": round(fl / (us * 1e-6) / PEAK, 3)})
        tot_us += us
        tot_fl += fl
    rows.sort(key=lambda r: -r["us"])
    rec = {"step": "%s, %d frames 800x1333, channels_last" % (cfg.MODEL.TYPE if hasattr(cfg, "MODEL")
                                                              else "model", F),
           "config": os.environ.get("CFG", "e2e_mask_rcnn_R-50-FPN_1x"),
           "step_ms_instrumented": round(step_ms, 2), "conv_gemm_ms": round(tot_us / 1e3, 2),
           "conv_gemm_TFLOP": round(tot_fl / 1e12, 3),
           "conv_gemm_TFs": round(tot_fl / (tot_us * 1e-6) / 1e12, 1),
           "peak_TFs": PEAK / 1e12, "ops": rows}
    print(json.dumps(rec, indent=1))
    if len(sys.argv) > 1:
        json.dump(rec, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
