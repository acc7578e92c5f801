"""vd_conv3x3_bias_act (hand-written MFMA implicit-GEMM 3x3 conv, csrc/conv3x3.hip)
against a plain torch fp32 reference of the same op: conv2d(pad 1) + bias (+ ReLU)
on channels_last tensors, incl. borders, a ragged pixel tail and Cout > 128."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,C,H,W,Cout", [(37, 256, 14, 14, 256), (5, 64, 6, 20, 128),
                                          (3, 8, 2, 9, 64), (9, 128, 14, 14, 64),
                                          (1, 64, 14, 14, 64), (100, 256, 14, 14, 256),
                                          (16, 64, 4, 6, 64), (7, 64, 8, 24, 64),
                                          (16, 64, 25, 42, 64), (5, 64, 13, 21, 128),
                                          (9, 64, 7, 7, 64)])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("mode", [True, "2d"])
def test_conv3x3_wino_mosaic_bit_exact(N, C, H, W, Cout, relu, mode):
    """The N maps as one mosaic with per-map zero padding give bit for bit the
    per-map Winograd result, and stay within the conv tolerance of torch fp32:
    mode True stacks them in one (N * H)-row column (vd_conv3x3_wino_seg_bias_act),
    "2d" also packs 16 / gcd(W, 16) maps side by side per mosaic row
    (vd_conv3x3_wino_mosaic_bias_act; a partly filled last row when N is not a
    multiple of it; odd sides padded by a phantom row / column per map).  The row
    mosaic refuses an odd H."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cpu").manual_seed(13 * N + C + H + W + Cout)
    x = torch.randn(N, C, H, W, generator=g).cuda().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** .5).cuda()
    b = torch.randn(Cout, generator=g).cuda()
    u = ops.conv3x3_wino_weight(w)
    per = ops.conv3x3_wino_bias_act(x, u, b, relu=relu)
    mos = ops.conv3x3_wino_bias_act(x, u, b, relu=relu, mosaic=mode)
    torch.cuda.synchronize()
    if mode is True and H % 2:
        assert mos is None
        return
    assert mos.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(per, mos)
    ref = F.conv2d(x, w, b, padding=1)
    if relu:
        ref = F.relu(ref)
    assert float((mos - ref).abs().max()) <= 2e-5 * max(1., float(ref.abs().max()))
