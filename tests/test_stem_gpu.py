"""The fused ResNet stem (vd_stem_conv_pool, csrc/stem.hip): conv1 7x7/2 pad 3 on
the MFMA pipes + folded bias + ReLU + MaxPool 3x3/2 pad 1 in one kernel
(basic_bn_stem, lib/modeling/ResNet.py:224-230) vs the torch fp32 module sequence,
at the benched blob (16 x 800 x 1344) and at ragged sizes (tile edges, odd conv
and pool extents, the C4 demo frame's 800 x 1133 blob)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _ref(x, w, b):
    y = F.conv2d(x, w, None, 2, 3)
    return F.max_pool2d(F.relu(y + b.view(1, -1, 1, 1)), 3, 2, 1)


@pytest.mark.parametrize("shape", [(16, 800, 1344), (1, 800, 1133), (2, 37, 45), (3, 64, 96),
                                   (1, 7, 9), (1, 1, 1)])
def test_stem_conv_pool_vs_torch(shape):
    """max |err| / max |y| <= 2e-5 (fp32 accumulation order differs from MIOpen's)."""
    from vosdetectron_amd import ops
    N, H, W = shape
    g = torch.Generator(device="cpu").manual_seed(H * 1000 + W)
    x = (torch.rand((N, H, W, 3), generator=g) * 255 - 120).to(DEV).permute(0, 3, 1, 2)
    w = (torch.randn((64, 3, 7, 7), generator=g) / 147 ** 0.5).to(DEV)
    b = torch.randn((64,), generator=g).to(DEV)
    got = ops.stem_conv_pool(x, ops.stem_pack(w), b)
    torch.backends.cudnn.allow_tf32 = False
    want = _ref(x.contiguous(), w, b)
    assert got.shape == want.shape
    assert got.is_contiguous(memory_format=torch.channels_last)
    err = float((got - want).abs().max())
    scale = float(want.abs().max())
    assert err <= 2e-5 * scale, (shape, err, scale)


def test_stem_rejects_bad_input():
    from vosdetectron_amd import ops
    w = torch.zeros((64, 3, 7, 7), device=DEV)
    with pytest.raises(ValueError):
        ops.stem_conv_pool(torch.zeros((1, 3, 8, 8), device=DEV), ops.stem_pack(w),
                           torch.zeros(64, device=DEV))  # NCHW, not channels_last
    with pytest.raises(ValueError):
        ops.stem_pack(torch.zeros((64, 3, 3, 3), device=DEV))


def test_model_stem_routes_to_fused_kernel(monkeypatch):
    """The folded R-50 body's stem takes the fused kernel by default and agrees with
    the MIOpen conv + epilogue route (VOSDET_STEM=miopen) within 2e-5."""
    from vosdetectron_amd import config as vcfg, ops
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.e2e_mask_rcnn_R_50_FPN_1x()
    model, _ = build_model(cfg, seed=0, device=DEV, channels_last=True)
    stems = [m for m in model.modules() if type(m).__name__ == "_StemEpilogue"]
    assert len(stems) == 1
    stem = stems[0]
    x = (torch.rand((2, 3, 160, 224)) * 255 - 120).to(DEV).contiguous(
        memory_format=torch.channels_last)
    monkeypatch.setenv("VOSDET_STEM", "fused")
    calls = []
    orig = ops.stem_conv_pool
    monkeypatch.setattr(ops, "stem_conv_pool", lambda *a: calls.append(1) or orig(*a))
    with torch.no_grad():
        fused = stem(x)
        assert calls == [1]
        monkeypatch.setenv("VOSDET_STEM", "miopen")
        ref = stem(x)
    assert calls == [1]
    err = float((fused - ref).abs().max())
    assert err <= 2e-5 * float(ref.abs().max()), err
