"""HIP-event time of the ResNet stem at the benched blob (16 x 800 x 1344): the fused
vd_stem_conv_pool vs MIOpen conv1 + vd_bias_relu_maxpool (the previous route)."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from vosdetectron_amd import ops  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
x = (torch.rand((16, 800, 1344, 3), device=dev) * 255 - 120).permute(0, 3, 1, 2)
w = torch.randn((64, 3, 7, 7), device=dev) / 147 ** 0.5
b = torch.randn((64,), device=dev)
pk = ops.stem_pack(w)


def fused():
    return ops.stem_conv_pool(x, pk, b)


def miopen():
    h = F.conv2d(x, w, None, 2, 3)
    return ops.bias_relu_maxpool(h.contiguous(memory_format=torch.channels_last), b)


def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


a, m = t(fused), t(miopen)
err = float((fused() - miopen()).abs().max())
gflop = 2 * 16 * 400 * 672 * 64 * 147 / 1e9
print(json.dumps({"fused_ms": round(a, 3), "miopen_plus_pool_ms": round(m, 3),
                  "fused_TFs_direct": round(gflop / a, 1), "max_abs_diff": err}))
