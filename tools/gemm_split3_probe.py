"""Split-bf16 GEMM (csrc/gemm_split3.hip) vs the fp32 GEMM path (vd_gemm_bias_act:
hipBLASLt / gemm1x1 as pinned) on the benched 32-frame step's GEMM shapes
(profiles/r05/gemm_census_f32.jsonl): time (HIP events) and error against an fp64
reference on the first rows.  One JSON line per (shape, path).

    python tools/gemm_split3_probe.py [--shapes all|quick] [--reps 10] > out.jsonl
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (M, N, K, residual) -- relu on, as the step's
    (2150400, 64, 256, False), (537600, 128, 256, False), (537600, 512, 256, False),
    (537600, 512, 128, True), (537600, 128, 512, False), (134400, 256, 512, False),
    (134400, 1024, 512, False), (134400, 1024, 256, True), (134400, 256, 1024, False),
    (33600, 512, 1024, False), (33600, 2048, 1024, False), (33600, 2048, 512, True),
    (33600, 512, 2048, False), (33600, 256, 2048, False), (32000, 1024, 12544, False),
    (32000, 1024, 1024, False), (627200, 1024, 256, False), (537600, 256, 512, False),
    (134400, 256, 1024, False), (537600, 512, 128, False), (2150400, 256, 256, False),
]
QUICK = [SHAPES[i] for i in (6, 8, 14, 16)]
SMALLK = [(2150400, 64, 64, False), (2150400, 256, 64, True), (537600, 512, 128, True),
          (537600, 128, 256, False), (134400, 256, 512, False)]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="all")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cfgs", default="1,2,3")
    ap.add_argument("--check-rows", type=int, default=4096)
    args = ap.parse_args()
    from vosdetectron_amd import ops
    shapes = {"quick": QUICK, "smallk": SMALLK}.get(args.shapes, SHAPES)
    g = torch.Generator(device="cuda").manual_seed(0)
    for (M, N, K, res) in shapes:
        a = torch.randn(M, K, device="cuda", generator=g).relu_()  # post-ReLU activations
        w = torch.randn(N, K, device="cuda", generator=g) / K ** .5
        b = torch.randn(N, device="cuda", generator=g) * .1
        r = torch.randn(M, N, device="cuda", generator=g) if res else None
        rows = min(M, args.check_rows)
        ref = a[:rows].double() @ w.double().t() + b.double()
        if res:
            ref = ref + r[:rows].double()
        ref = ref.relu()
        scale = float(ref.abs().max())
        flop = 2.0 * M * N * K

        def report(path, ms, d):
            e = (d[:rows].double() - ref).abs()
            print(json.dumps({"M": M, "N": N, "K": K, "res": res, "path": path, "ms": round(ms, 4),
                              "TFs": round(flop / ms / 1e9, 1),
                              "max_err_rel": float(e.max()) / scale,
                              "mean_err_rel": float(e.mean()) / scale}), flush=True)

        out = torch.empty(M, N, device="cuda")
        ms = timed(lambda: ops.gemm_bias_act(a, w, b, residual=r, relu=True, out=out), args.reps)
        report("auto", ms, out)
        os.environ["VOSDET_GEMM_SPLIT3"] = "0"
        ms = timed(lambda: ops.gemm_bias_act(a, w, b, residual=r, relu=True, out=out), args.reps)
        del os.environ["VOSDET_GEMM_SPLIT3"]
        report("fp32", ms, out)
        wp = ops.gemm_split3_weight(w)
        for cfg in [int(c) for c in args.cfgs.split(",")]:
            if (cfg in (1, 11, 12, 13, 19) and N % 256) or (cfg in (2, 14, 15, 16, 17, 18) and N % 128) or \
                    (cfg >= 10 and r is not None):
                continue
            out.zero_()
            ms = timed(lambda: ops.gemm_split3_bias_act(a, wp, b, residual=r, relu=True, out=out,
                                                        cfg=cfg), args.reps)
            report("split3_cfg%d" % cfg, ms, out)
        del a, w, r, out, ref, wp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
