"""X-101-32x8d's grouped 3x3 convs (conv2 of every bottleneck, 32 groups) at the
32-frame step shapes: MIOpen's conv + our bias/ReLU pass (the engine's route) against
torch.miopen_convolution_relu (MIOpen's fused conv + bias + activation).  Times with
HIP events and the max difference between the two."""
import torch
import torch.nn.functional as F

from vosdetectron_amd import ops

dev = torch.device("cuda")
F_ = 32
for (C, H, W, s) in [(256, 200, 336, 1), (512, 100, 168, 1), (1024, 50, 84, 1), (2048, 25, 42, 1),
                     (512, 200, 336, 2), (1024, 100, 168, 2), (2048, 50, 84, 2)]:
    n = F_ if C <= 1024 else F_
    x = torch.randn(n, C, H, W, device=dev).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, C // 32, 3, 3, device=dev) / (3 * (C // 32) ** .5)).contiguous(
        memory_format=torch.channels_last)
    b = torch.randn(C, device=dev)

    def a():
        y = F.conv2d(x, w, None, s, 1, 1, 32)
        return ops.bias_act_(y, b, relu=True)

    def f():
        return torch.miopen_convolution_relu(x, w, b, (s, s), (1, 1), (1, 1), 32)

    res = {}
    for name, fn in (("conv+bias_act", a), ("miopen_conv_relu", f)):
        try:
            for _ in range(3):
                y = fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                y = fn()
            e1.record()
            torch.cuda.synchronize()
            res[name] = (e0.elapsed_time(e1) / 10, y)
        except Exception as ex:  # noqa
            res[name] = (None, repr(ex)[:120])
    d = None
    if all(isinstance(v[1], torch.Tensor) for v in res.values()):
        d = float((res["conv+bias_act"][1] - res["miopen_conv_relu"][1]).abs().max())
    print(C, H, W, s, {k: (v[0] if v[0] is not None else v[1]) for k, v in res.items()}, "maxdiff", d,
          flush=True)
    del x, w, res
