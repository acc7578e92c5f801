"""vd_conv3x3_bias_act (hand-written MFMA implicit-GEMM 3x3 conv, csrc/conv3x3.hip)
against a plain torch fp32 reference of the same op: conv2d(pad 1) + bias (+ ReLU)
on channels_last tensors, incl. borders, a ragged pixel tail and Cout > 128."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,C,H,W,Cout", [(2, 64, 9, 13, 128), (1, 256, 14, 14, 256),
                                          (3, 128, 1, 1, 128), (1, 256, 25, 42, 256),
                                          (5, 256, 7, 7, 384), (2, 64, 30, 41, 64),
                                          (1, 128, 5, 3, 64)])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("variant", ["1", "2", "6"])
def test_conv3x3_vs_torch(monkeypatch, N, C, H, W, Cout, relu, variant):
    from vosdetectron_amd import ops
    monkeypatch.setenv("VOSDET_CONV3X3_VARIANT", variant)
    g = torch.Generator(device="cpu").manual_seed(N * 1000 + C + H + Cout)
    x = torch.randn(N, C, H, W, generator=g).cuda().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** .5).cuda()
    b = torch.randn(Cout, generator=g).cuda()
    ref = F.conv2d(x, w, b, padding=1)
    if relu:
        ref = F.relu(ref)
    got = ops.conv3x3_bias_act(x, ops.conv3x3_weight(w), b, relu=relu)
    torch.cuda.synchronize()
    assert got.is_contiguous(memory_format=torch.channels_last)
    assert float((got - ref).abs().max()) <= 2e-5 * max(1., float(ref.abs().max()))


def test_conv3x3_no_bias_and_unsupported_shape():
    from vosdetectron_amd import ops
    x = torch.randn(1, 64, 5, 6, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(128, 64, 3, 3, device="cuda") / 24
    got = ops.conv3x3_bias_act(x, ops.conv3x3_weight(w), None)
    ref = F.conv2d(x, w, None, padding=1)
    assert float((got - ref).abs().max()) <= 2e-5 * max(1., float(ref.abs().max()))
    w2 = torch.randn(96, 64, 3, 3, device="cuda")  # Cout neither 64 nor a multiple of 128
    assert ops.conv3x3_bias_act(x, ops.conv3x3_weight(w2), None) is None
