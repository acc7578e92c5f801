"""Characterise the split-bf16 GEMM's rounding: error (in ulps of the fp64-exact
result rounded to fp32) of one 16-deep step (six bf16 MFMAs) and of K-deep sums,
signed and non-negative operands; torch's fp32 matmul beside it."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def ulps(x, ref):
    r32 = ref.float()
    ulp = (torch.nextafter(r32.abs(), torch.tensor(float("inf"), device=r32.device)) - r32.abs()).double()
    return (x.double() - ref) / ulp


def main():
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(1)
    for K in (16, 32, 256, 1024):
        for signed in (True, False):
            M, N = 8192, 256
            a = torch.randn(M, K, device="cuda", generator=g)
            if not signed:
                a = a.abs()
            w = torch.randn(N, K, device="cuda", generator=g)
            if not signed:
                w = w.abs()
            b = torch.zeros(N, device="cuda")
            ref = a.double() @ w.double().t()
            s3 = ops.gemm_split3_bias_act(a, ops.gemm_split3_weight(w), b, relu=False)
            t = a @ w.t()
            torch.cuda.synchronize()
            out = {"K": K, "signed": signed}
            for name, x in (("split3", s3), ("torch", t)):
                u = ulps(x, ref)
                e = (x.double() - ref)
                sc = float(ref.abs().max())
                out[name] = {"abs_mean_rel": float(e.abs().mean()) / sc,
                             "abs_max_rel": float(e.abs().max()) / sc,
                             "bias_rel": float(e.mean()) / sc,
                             "mean_ulp": float(u.mean()), "mean_abs_ulp": float(u.abs().mean()),
                             "max_abs_ulp": float(u.abs().max()),
                             "frac_exact": float((x.double() == ref.float().double()).double().mean())}
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
