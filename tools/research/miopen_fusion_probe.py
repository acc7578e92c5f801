#!/usr/bin/env python3
"""Probe: does MIOpen's fusion API (conv -> bias -> ReLU as one plan; solvers
ConvCKIgemmFwdBiasActivFused / ConvCKIgemmGrpFwdBiasActivFused) compile for
the fp32 NHWC 3x3 convs of this path, and how fast is it against the unfused
conv + vd_bias_act the engine runs?  Uses torch's own libMIOpen (ctypes)."""
import ctypes
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from vosdetectron_amd import ops  # noqa: E402

L = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libMIOpen.so"))
P = ctypes.c_void_p


def ok(st, what):
    if st != 0:
        raise RuntimeError("%s: miopen status %d" % (what, st))


def tdesc(shape_nchw, nhwc=True):
    d = P()
    ok(L.miopenCreateTensorDescriptor(ctypes.byref(d)), "create desc")
    n, c, h, w = shape_nchw
    strides = (h * w * c, 1, w * c, c) if nhwc else (c * h * w, h * w, w, 1)
    dims = (ctypes.c_int * 4)(*shape_nchw)
    st = (ctypes.c_int * 4)(*strides)
    ok(L.miopenSetTensorDescriptor(d, 1, 4, dims, st), "set desc")
    return d


def timed(fn, iters=10):
    s = torch.cuda.current_stream()
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def probe(N, C, H, W, K, ksz=3, pad=1):
    x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, ksz, ksz, device="cuda") / (C * ksz * ksz) ** .5).contiguous(
        memory_format=torch.channels_last)
    b = torch.randn(K, device="cuda")
    y = torch.empty(N, K, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    h = P()
    ok(L.miopenCreateWithStream(ctypes.byref(h), P(torch.cuda.current_stream().cuda_stream)),
       "handle")
    xd, yd = tdesc((N, C, H, W)), tdesc((N, K, H, W))
    wd = tdesc((K, C, ksz, ksz))
    bd = tdesc((1, K, 1, 1), nhwc=False)
    cd = P()
    ok(L.miopenCreateConvolutionDescriptor(ctypes.byref(cd)), "conv desc")
    ok(L.miopenInitConvolutionDescriptor(cd, 0, pad, pad, 1, 1, 1, 1), "init conv")
    plan = P()
    ok(L.miopenCreateFusionPlan(ctypes.byref(plan), 0, xd), "plan")
    cop, bop, aop = P(), P(), P()
    ok(L.miopenCreateOpConvForward(plan, ctypes.byref(cop), cd, wd), "conv op")
    ok(L.miopenCreateOpBiasForward(plan, ctypes.byref(bop), bd), "bias op")
    ok(L.miopenCreateOpActivationForward(plan, ctypes.byref(aop), 3), "activ op")
    res = {"shape": [N, C, H, W, K, ksz]}
    st = L.miopenCompileFusionPlan(h, plan)
    res["compile_status"] = st
    ref = F.relu(F.conv2d(x, w, b, padding=pad))
    res["unfused_us"] = round(timed(lambda: ops.bias_act_(F.conv2d(x, w, None, padding=pad), b)), 1)
    if st == 0:
        args = P()
        ok(L.miopenCreateOperatorArgs(ctypes.byref(args)), "args")
        one, zero = ctypes.c_float(1.), ctypes.c_float(0.)
        ok(L.miopenSetOpArgsConvForward(args, cop, ctypes.byref(one), ctypes.byref(zero),
                                        P(w.data_ptr())), "conv args")
        ok(L.miopenSetOpArgsBiasForward(args, bop, ctypes.byref(one), ctypes.byref(zero),
                                        P(b.data_ptr())), "bias args")
        ok(L.miopenSetOpArgsActivForward(args, aop, ctypes.byref(one), ctypes.byref(zero),
                                         ctypes.c_double(0.), ctypes.c_double(0.),
                                         ctypes.c_double(0.)), "activ args")

        def fused():
            ok(L.miopenExecuteFusionPlan(h, plan, xd, P(x.data_ptr()), yd, P(y.data_ptr()), args),
               "execute")
        res["fused_us"] = round(timed(fused), 1)
        res["maxdiff"] = float((y - ref).abs().max())
    print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    torch.backends.cudnn.benchmark = True
    out = [probe(16, 256, 100, 168, 256), probe(16, 256, 200, 336, 256),
           probe(1600, 256, 14, 14, 256), probe(16, 64, 200, 336, 64)]
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)
