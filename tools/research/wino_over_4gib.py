#!/usr/bin/env python3
"""The Winograd kernel's >= 4 GiB input fallback (64-bit DMA pointers, zero-buffer
source) vs torch fp32 -- kept as a script until it has run on a GPU box (the round-4
session ended with the pool unavailable); move it into tests/test_conv3x3_gpu.py once
it has passed there.  usage: python tools/research/wino_over_4gib.py"""
import torch
import torch.nn.functional as F


def check_wino_input_over_4gib():
    """The Winograd kernel's patch DMA reads X through 32-bit byte offsets; an input
    of 4 GiB or more takes the 64-bit-pointer form with the zero-buffer source
    (csrc/conv3x3_wino.hip, launch_wino).  2 x 256 x 1536 x 1408 fp32 = 4.43 GB,
    vs torch fp32 at 2e-5 of the output range, borders included."""
    import os, sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from vosdetectron_amd import ops
    N, C, H, W = 2, 256, 1536, 1408
    assert N * C * H * W * 4 >= 1 << 32
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(C, C, 3, 3, device="cuda", generator=g) / (3. * C ** .5)
    b = torch.randn(C, device="cuda", generator=g)
    got = ops.conv3x3_wino_bias_act(x, ops.conv3x3_wino_weight(w), b, relu=True)
    ref = F.relu(F.conv2d(x, w, b, padding=1))
    torch.cuda.synchronize()
    err = float((got - ref).abs().max())
    assert err <= 2e-5 * max(1., float(ref.abs().max())), err
    # the image borders (first / last rows and columns) are where the zero taps live
    for sl in ((slice(None), slice(None), 0), (slice(None), slice(None), H - 1),
               (slice(None), slice(None), slice(None), 0), (slice(None), slice(None), slice(None), W - 1)):
        e = float((got[sl] - ref[sl]).abs().max())
        assert e <= 2e-5 * max(1., float(ref.abs().max())), (sl, e)
    del x, got, ref
    torch.cuda.empty_cache()


if __name__ == "__main__":
    check_wino_input_over_4gib()
    print("ok")
