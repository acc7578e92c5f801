"""vd_bias_act (fused conv epilogue) against the unfused PyTorch sequence it
replaces: bias add, residual add (same-shape or nearest-2x upsampled, with an
optional residual bias), ReLU.  Same association order, so bit-exact."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x, b, res, rb, relu, up):
    y = x + b.view(1, -1, 1, 1) if b is not None else x.clone()
    if res is not None:
        if up:
            res = F.interpolate(res, scale_factor=2, mode="nearest")
        t = res + rb.view(1, -1, 1, 1) if rb is not None else res
        y = y + t
    return F.relu(y) if relu else y


@pytest.mark.parametrize("cl", [False, True])
@pytest.mark.parametrize("mode", ["none", "same", "same_bias", "up"])
@pytest.mark.parametrize("relu", [False, True])
def test_bias_act_matches_unfused(cl, mode, relu):
    from vosdetectron_amd import ops
    g = torch.Generator(device="cpu").manual_seed(7)
    N, C, H, W = 2, 36, 10, 14
    fmt = torch.channels_last if cl else torch.contiguous_format
    x = torch.randn(N, C, H, W, generator=g).cuda().contiguous(memory_format=fmt)
    b = torch.randn(C, generator=g).cuda()
    res = rb = None
    up = mode == "up"
    if mode != "none":
        shape = (N, C, H // 2, W // 2) if up else (N, C, H, W)
        res = torch.randn(*shape, generator=g).cuda().contiguous(memory_format=fmt)
    if mode == "same_bias":
        rb = torch.randn(C, generator=g).cuda()
    exp = _ref(x, b, res, rb, relu, up)
    got = ops.bias_act_(x.clone(memory_format=fmt), b, res, rb, relu=relu, upsample_residual=up)
    torch.cuda.synchronize()
    assert torch.equal(got, exp)


def test_bias_act_rejects_bad_shapes():
    from vosdetectron_amd import ops
    x = torch.zeros(1, 8, 6, 6, device="cuda")
    with pytest.raises(ValueError):
        ops.bias_act_(x, torch.zeros(7, device="cuda"))
    with pytest.raises(ValueError):
        ops.bias_act_(x, None, torch.zeros(1, 8, 4, 3, device="cuda"), upsample_residual=True)


def test_bias_act_large_odd_grid():
    """More elements than one grid-stride pass (exercises the loop)."""
    from vosdetectron_amd import ops
    N, C, H, W = 4, 256, 200, 336
    x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    b = torch.randn(C, device="cuda")
    r = torch.randn_like(x)
    exp = F.relu((x + b.view(1, -1, 1, 1)) + r)
    got = ops.bias_act_(x.clone(memory_format=torch.channels_last), b, r)
    assert torch.equal(got, exp)
