"""Research: split-bf16 GEMM tile configs 2 (256 x 128, two per CU) vs 5 (256 x 256,
eight waves) on the 64-frame step's shapes, HIP events, same process."""
import torch

from vosdetectron_amd import ops

dev = torch.device("cuda")
for (M, N, K, res) in [(268800, 1024, 1024, False), (268800, 1024, 1024, True),
                       (268800, 1024, 256, True), (268800, 256, 1024, False),
                       (1075200, 512, 128, True), (1075200, 128, 512, False),
                       (67200, 2048, 512, True), (67200, 512, 2048, False)]:
    a = torch.randn(M, K, device=dev).relu_()
    w = torch.randn(N, K, device=dev) / K ** .5
    b = torch.randn(N, device=dev)
    r = torch.randn(M, N, device=dev) if res else None
    wp = ops.gemm_split3_weight(w)
    out = torch.empty(M, N, device=dev)
    t = {}
    for cfg in (0, 2, 4, 5):
        try:
            for _ in range(3):
                ops.gemm_split3_bias_act(a, wp, b, residual=r, out=out, cfg=cfg)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ops.gemm_split3_bias_act(a, wp, b, residual=r, out=out, cfg=cfg)
            e1.record()
            torch.cuda.synchronize()
            t[cfg] = round(e0.elapsed_time(e1) / 10, 3)
        except Exception as ex:  # noqa
            t[cfg] = None
    print((M, N, K, res), t, flush=True)
    del a, w, r, out, wp
