"""The fused ResNet stem (vd_stem_conv_pool, csrc/stem.hip): conv1 7x7/2 pad 3 on
the MFMA pipes + folded bias + ReLU + MaxPool 3x3/2 pad 1 in one kernel
(basic_bn_stem, lib/modeling/ResNet.py:224-230) vs the torch fp32 module sequence,
at the benched blob (16 x 800 x 1344) and at ragged sizes (tile edges, odd conv
and pool extents, the C4 demo frame's 800 x 1133 blob) -- both conv1 cores: the
split-bf16 one (vd_stem_split_conv_pool, the default) and the fp32 one."""
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
@pytest.mark.parametrize("split", [True, False])
def test_stem_conv_pool_vs_torch(shape, split):
    """max |err| / max |y| <= 2e-5 (fp32 accumulation order differs from MIOpen's)."""
    from vosdetectron_amd import ops
    N, H, W = shape
    g = torch.Generator(device="cpu").manual_seed(H * 1000 + W)
    x = (torch.rand((N, H, W, 3), generator=g) * 255 - 120).to(DEV).permute(0, 3, 1, 2)
    w = (torch.randn((64, 3, 7, 7), generator=g) / 147 ** 0.5).to(DEV)
    b = torch.randn((64,), generator=g).to(DEV)
    got = ops.stem_conv_pool(x, ops.stem_pack(w, split=split), b)
    torch.backends.cudnn.allow_tf32 = False
    want = _ref(x.contiguous(), w, b)
    assert got.shape == want.shape
    assert got.is_contiguous(memory_format=torch.channels_last)
    err = float((got - want).abs().max())
    scale = float(want.abs().max())
    assert err <= 2e-5 * scale, (shape, err, scale)


def test_stem_split_as_accurate_as_fp32():
    """Against a float64 evaluation, the split-bf16 stem's error is no larger than the
    fp32 MFMA stem's (mean within 1.5x, max within 3x), and it is deterministic."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cpu").manual_seed(7)
    x = (torch.rand((2, 240, 320, 3), generator=g) * 255 - 120).to(DEV).permute(0, 3, 1, 2)
    w = (torch.randn((64, 3, 7, 7), generator=g) / 147 ** 0.5).to(DEV)
    b = torch.randn((64,), generator=g).to(DEV)
    want = _ref(x.contiguous().double().cpu(), w.double().cpu(), b.double().cpu())
    e = {}
    for split in (True, False):
        got = ops.stem_conv_pool(x, ops.stem_pack(w, split=split), b)
        e[split] = (got.double().cpu() - want).abs()
        if split:
            assert torch.equal(got, ops.stem_conv_pool(x, ops.stem_pack(w, split=True), b))
    assert float(e[True].mean()) <= 1.5 * float(e[False].mean()) + 1e-12, (
        float(e[True].mean()), float(e[False].mean()))
    assert float(e[True].max()) <= 3 * float(e[False].max()) + 1e-12


def test_stem_split_weight_image_is_the_rne_split():
    """vd_stem_split_weight_pack's image: [k-step 5][co block 4][piece 3][lane 64][8 bf16],
    lane = 16 (k-group) + co % 16, k = (ky, kx, ci) zero-padded to 160, pieces the
    round-to-nearest-even three-way bf16 split (torch's conversion)."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cpu").manual_seed(3)
    w = torch.randn((64, 3, 7, 7), generator=g) * 0.3
    img = ops.stem_pack(w.to(DEV), split=True).cpu()
    wk = torch.zeros((64, 160))
    wk[:, :147] = w.permute(0, 2, 3, 1).reshape(64, 147)
    p0 = wk.to(torch.bfloat16)
    r1 = wk - p0.float()
    p1 = r1.to(torch.bfloat16)
    p2 = (r1 - p1.float()).to(torch.bfloat16)
    pieces = torch.stack([p0, p1, p2])  # [3][co 64][k 160]
    # [piece][b][j][s][q][8] -> [s][b][piece][q][j][8]
    want = pieces.view(3, 4, 16, 5, 4, 8).permute(3, 1, 0, 4, 2, 5).contiguous()
    assert torch.equal(img.view(torch.bfloat16).view(-1), want.view(-1))


def test_stem_rejects_bad_input():
    from vosdetectron_amd import ops
    w = torch.zeros((64, 3, 7, 7), device=DEV)
    with pytest.raises(ValueError):
        ops.stem_conv_pool(torch.zeros((1, 3, 8, 8), device=DEV), ops.stem_pack(w),
                           torch.zeros(64, device=DEV))  # NCHW, not channels_last
    with pytest.raises(ValueError):
        ops.stem_pack(torch.zeros((64, 3, 3, 3), device=DEV))


@pytest.mark.parametrize("mode", ["split", "fused", None])
def test_model_stem_routes_to_fused_kernel(monkeypatch, mode):
    """The folded R-50 body's stem takes the fused kernel (split-bf16 by default) and
    agrees with the MIOpen conv + epilogue route (VOSDET_STEM=miopen) within 2e-5."""
    from vosdetectron_amd import config as vcfg, ops
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.e2e_mask_rcnn_R_50_FPN_1x()
    model, _ = build_model(cfg, seed=0, device=DEV, channels_last=True)
    stems = [m for m in model.modules() if type(m).__name__ == "_StemEpilogue"]
    assert len(stems) == 1
    stem = stems[0]
    x = (torch.rand((2, 3, 160, 224)) * 255 - 120).to(DEV).contiguous(
        memory_format=torch.channels_last)
    if mode is None:
        monkeypatch.delenv("VOSDET_STEM", raising=False)
    else:
        monkeypatch.setenv("VOSDET_STEM", mode)
    calls = []
    orig = ops.stem_conv_pool
    monkeypatch.setattr(ops, "stem_conv_pool", lambda *a: calls.append(a[1].dtype) or orig(*a))
    with torch.no_grad():
        fused = stem(x)
        want = torch.float32 if mode == "fused" else torch.uint8  # the split image is bytes
        assert calls == [want]
        monkeypatch.setenv("VOSDET_STEM", "miopen")
        ref = stem(x)
    assert calls == [want]
    err = float((fused - ref).abs().max())
    assert err <= 2e-5 * float(ref.abs().max()), err
