"""Winograd F(4x4,3x3), position-split form (csrc/conv3x3_wino4.hip,
VOSDET_WINO4_PS=1) and the hand-counted-vmcnt form (VOSDET_WINO4_ACC=1) vs the first
form -- and the default form's packed-fp32 input transform (VOSDET_WINO4_PK) against
its scalar one: the same MFMA operands in the same order and
the same output transform, so the outputs must be bit-identical -- on the step's
shapes (incl. ragged blocks: H, W not multiples of 16 / 32), with and without bias
and ReLU -- and within 5e-5 of torch fp32 (the F(4x4) tolerance)."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


FORMS = {"first": {"VOSDET_WINO4_PS": "0", "VOSDET_WINO4_ACC": "0", "VOSDET_WINO4_VD": "1",
                   "VOSDET_WINO4_IL": "0"},
         "ps": {"VOSDET_WINO4_PS": "1", "VOSDET_WINO4_ACC": "0", "VOSDET_WINO4_VD": "1"},
         "acc": {"VOSDET_WINO4_PS": "0", "VOSDET_WINO4_ACC": "1", "VOSDET_WINO4_VD": "1"},
         "acc3": {"VOSDET_WINO4_PS": "0", "VOSDET_WINO4_ACC": "1", "VOSDET_WINO4_VD": "3"},
         "il": {"VOSDET_WINO4_PS": "0", "VOSDET_WINO4_ACC": "1", "VOSDET_WINO4_VD": "1",
                "VOSDET_WINO4_IL": "1"},
         # the default ACC form with the scalar input transform (the packed-fp32 one,
         # VOSDET_WINO4_PK=1, is the default and is what "acc" runs)
         "acc_scalar": {"VOSDET_WINO4_PS": "0", "VOSDET_WINO4_ACC": "1", "VOSDET_WINO4_VD": "1",
                        "VOSDET_WINO4_PK": "0"}}


def _run(x, u, b, relu, form):
    from vosdetectron_amd import ops
    env = FORMS[form]
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        y = ops.conv3x3_wino4_bias_act(x, u, b, relu=relu)
        torch.cuda.synchronize()
        return y
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("N,C,H,W,Co", [(2, 64, 20, 36, 64), (1, 256, 50, 84, 256),
                                        (3, 128, 17, 45, 128), (2, 512, 25, 42, 512),
                                        (1, 8, 9, 9, 64), (4, 24, 33, 31, 128)])
@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize("form", ["ps", "acc", "acc3", "il", "acc_scalar"])
def test_wino4_forms_bit_identical_to_first_form(N, C, H, W, Co, bias, form):
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(N * 1000 + C + H)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (3. * C ** .5)
    b = torch.randn(Co, device="cuda", generator=g) if bias else None
    u = ops.conv3x3_wino4_weight(w)
    y1 = _run(x, u, b, bias, "first")
    y2 = _run(x, u, b, bias, form)
    assert torch.equal(y1, y2), float((y1 - y2).abs().max())
    ref = F.conv2d(x, w, b, padding=1)
    if bias:
        ref = F.relu(ref)
    err = float((y2 - ref).abs().max())
    assert err <= 5e-5 * max(1., float(ref.abs().max())), err


@pytest.mark.parametrize("form", ["ps", "acc", "acc3", "il", "acc_scalar"])
def test_wino4_forms_benched_p2(form):
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(32, 256, 200, 336, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(256, 256, 3, 3, device="cuda", generator=g) / 48.
    b = torch.randn(256, device="cuda", generator=g)
    u = ops.conv3x3_wino4_weight(w)
    y1 = _run(x, u, b, False, "first")
    y2 = _run(x, u, b, False, form)
    assert torch.equal(y1, y2), float((y1 - y2).abs().max())


@pytest.mark.parametrize("N,C,H,W,Co", [(7, 256, 14, 14, 256), (4, 64, 15, 13, 128),
                                        (2, 8, 1, 1, 64), (1, 24, 9, 15, 64),
                                        (3200, 256, 14, 14, 256)])
def test_wino4_pair_mosaic_bit_identical(N, C, H, W, Co):
    """vd_conv3x3_wino4_mosaic_bias_act (two maps per block) == one map per block,
    and within the F(4x4) tolerance of torch; odd N leaves the last pair half empty."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(N + C + H * W)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (3. * C ** .5)
    b = torch.randn(Co, device="cuda", generator=g)
    u = ops.conv3x3_wino4_weight(w)
    y1 = ops.conv3x3_wino4_bias_act(x, u, b, relu=True)
    y2 = ops.conv3x3_wino4_bias_act(x, u, b, relu=True, mosaic=True)
    torch.cuda.synchronize()
    assert y2 is not None
    assert torch.equal(y1, y2), float((y1 - y2).abs().max())
    ref = F.relu(F.conv2d(x[:64], w, b, padding=1))
    err = float((y2[:64] - ref).abs().max())
    assert err <= 5e-5 * max(1., float(ref.abs().max())), err


def test_wino4_pair_mosaic_refuses_large_maps():
    from vosdetectron_amd import ops
    x = torch.zeros(2, 64, 16, 14, device="cuda").contiguous(memory_format=torch.channels_last)
    u = ops.conv3x3_wino4_weight(torch.zeros(64, 64, 3, 3, device="cuda"))
    assert ops.conv3x3_wino4_bias_act(x, u, None, mosaic=True) is None


@pytest.mark.parametrize("N,C,H,W,Co", [(3, 64, 50, 84, 64), (2, 256, 25, 42, 128),
                                        (5, 8, 7, 33, 64), (2, 16, 16, 16, 64),
                                        (1, 64, 13, 9, 64), (32, 256, 50, 84, 256),
                                        (8, 64, 200, 336, 64)])
def test_wino4_row_stack_bit_identical(N, C, H, W, Co):
    """vd_conv3x3_wino4_rows_bias_act (maps stacked at a pitch of H + 1 rounded up to
    4 rows) == one launch over the N maps, incl. H a multiple of 4 and blocks that
    straddle maps; within the F(4x4) tolerance of torch."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(N * 7 + C + H * W)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (3. * C ** .5)
    b = torch.randn(Co, device="cuda", generator=g)
    u = ops.conv3x3_wino4_weight(w)
    y1 = ops.conv3x3_wino4_bias_act(x, u, b, relu=True)
    y2 = ops.conv3x3_wino4_bias_act(x, u, b, relu=True, mosaic="rows")
    torch.cuda.synchronize()
    assert y2 is not None
    assert torch.equal(y1, y2), float((y1 - y2).abs().max())
    ref = F.relu(F.conv2d(x[:4], w, b, padding=1))
    err = float((y2[:4] - ref).abs().max())
    assert err <= 5e-5 * max(1., float(ref.abs().max())), err


@pytest.mark.parametrize("N,C,H,W,Co", [(5, 64, 7, 7, 64), (17, 128, 6, 5, 64),
                                        (9, 8, 1, 7, 64), (8000, 512, 7, 7, 512)])
def test_wino4_octet_mosaic_bit_identical(N, C, H, W, Co):
    """Maps of at most 7 x 7 run eight per block (8 x 8 cells) through
    vd_conv3x3_wino4_mosaic_bias_act: == one map per block, incl. a last block with
    fewer than eight maps; within the F(4x4) tolerance of torch."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(N + 3 * C + H * W)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (3. * C ** .5)
    b = torch.randn(Co, device="cuda", generator=g)
    u = ops.conv3x3_wino4_weight(w)
    y1 = ops.conv3x3_wino4_bias_act(x, u, b, relu=True)
    y2 = ops.conv3x3_wino4_bias_act(x, u, b, relu=True, mosaic=True)
    torch.cuda.synchronize()
    assert y2 is not None
    assert torch.equal(y1, y2), float((y1 - y2).abs().max())
    ref = F.relu(F.conv2d(x[:64], w, b, padding=1))
    err = float((y2[:64] - ref).abs().max())
    assert err <= 5e-5 * max(1., float(ref.abs().max())), err


@pytest.mark.parametrize("N,C,H,W,Co", [(3200, 256, 14, 14, 256), (37, 64, 9, 11, 64),
                                        (1, 8, 14, 14, 64), (100, 24, 14, 14, 128),
                                        (5, 64, 7, 7, 64), (33, 64, 15, 15, 64),
                                        (50, 8, 1, 1, 64), (70, 16, 3, 40, 64)])
def test_wino4_grid_mosaic(N, C, H, W, Co):
    """vd_conv3x3_wino4_grid_bias_act (maps at an (H + 1) x (W + 1) pitch in a 2-D grid,
    tiles straddling maps): every output written, each map its own zero-padded conv --
    within the F(4x4) tolerance of torch on every map, and (maps of 4 px and more) as
    close to an fp64 evaluation as one map per block (mean within 1.25x, max 2x)."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(N * 3 + C + H * W)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (3. * C ** .5)
    b = torch.randn(Co, device="cuda", generator=g)
    u = ops.conv3x3_wino4_weight(w)
    y1 = ops.conv3x3_wino4_bias_act(x, u, b, relu=True)
    out = torch.full((N, Co, H, W), float("nan"), device="cuda").contiguous(
        memory_format=torch.channels_last)
    y2 = ops.conv3x3_wino4_bias_act(x, u, b, relu=True, mosaic="grid", out=out)
    torch.cuda.synchronize()
    assert y2 is not None and not bool(torch.isnan(y2).any())
    sel = torch.arange(N, device="cuda") if N <= 128 else torch.cat(
        [torch.arange(64, device="cuda"), torch.arange(N - 64, N, device="cuda")])
    xs = x[sel]
    ref = F.relu(F.conv2d(xs, w, b, padding=1))
    err = float((y2[sel] - ref).abs().max())
    assert err <= 5e-5 * max(1., float(ref.abs().max())), err
    r64 = F.relu(F.conv2d(xs.double(), w.double(), b.double(), padding=1))
    e1, e2 = (y1[sel].double() - r64).abs(), (y2[sel].double() - r64).abs()
    if min(H, W) >= 4:  # (maps under 4 px put one map per block at the tile's most
        # accurate output positions only; the grid mixes all of them)
        assert float(e2.mean()) <= 1.25 * float(e1.mean()) + 1e-12, (float(e2.mean()),
                                                                       float(e1.mean()))
        assert float(e2.max()) <= 2 * float(e1.max()) + 1e-12
    assert float(e2.max()) <= 2e-5 * max(1., float(r64.abs().max()))
    # deterministic
    assert torch.equal(y2, ops.conv3x3_wino4_bias_act(x, u, b, relu=True, mosaic="grid"))


def test_wino4_mask_head_routes_to_grid(monkeypatch):
    """The mask head's 14 x 14 RoI maps take the grid (1410 blocks per 3200 maps vs 1600
    as pairs); VOSDET_WINO4_GRID=0 keeps pairs; octets stay octets."""
    from vosdetectron_amd import modeling
    assert modeling.conv3x3_route(3200, 256, 256, 14, 14) == ("wino4", "grid")
    assert modeling.conv3x3_route(8000, 512, 512, 7, 7) == ("wino4", "pair")
    monkeypatch.setenv("VOSDET_WINO4_GRID", "0")
    assert modeling.conv3x3_route(3200, 256, 256, 14, 14) == ("wino4", "pair")


@pytest.mark.parametrize("N,C,H,W,groups,rows", [(2, 256, 20, 36, 32, False),
                                                 (2, 512, 17, 45, 32, False),
                                                 (1, 1024, 25, 42, 32, False),
                                                 (2, 2048, 13, 21, 32, False),
                                                 (3, 256, 50, 84, 32, True),
                                                 (4, 128, 9, 11, 16, True),
                                                 (2, 512, 33, 31, 64, False)])
@pytest.mark.parametrize("bias", [True, False])
def test_wino4_grouped(N, C, H, W, groups, rows, bias):
    """vd_conv3x3_wino4_grouped_bias_act (ResNeXt's grouped conv2 on the F(4x4) kernel,
    the weight block-diagonal per 64-channel block) vs torch's grouped conv: within
    the F(4x4) tolerance, and against fp64 as close as the dense F(4x4) kernel is on a
    dense conv of the same block width (mean within 1.5x)."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(N * 11 + C + H)
    cpg = C // groups
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(C, cpg, 3, 3, device="cuda", generator=g) / (3. * cpg ** .5)
    b = torch.randn(C, device="cuda", generator=g) if bias else None
    u = ops.conv3x3_wino4_grouped_weight(w, groups)
    y = ops.conv3x3_wino4_bias_act(x, u, b, relu=bias, groups=groups,
                                   mosaic="rows" if rows else False)
    torch.cuda.synchronize()
    assert y is not None
    ref = F.conv2d(x, w, b, padding=1, groups=groups)
    if bias:
        ref = F.relu(ref)
    err = float((y - ref).abs().max())
    assert err <= 5e-5 * max(1., float(ref.abs().max())), err
    r64 = F.conv2d(x.double(), w.double(), b.double() if bias else None, padding=1,
                   groups=groups)
    if bias:
        r64 = F.relu(r64)
    e = (y.double() - r64).abs()
    # the same conv as a dense one on the expanded (block-diagonal) weight
    wd = torch.zeros(C, 64, 3, 3, device="cuda")
    for co in range(C):
        gi = co // cpg
        lo = gi * cpg - (co // 64) * 64
        wd[co, lo:lo + cpg] = w[co]
    assert torch.equal(u, ops.conv3x3_wino4_weight(wd))
    # deterministic
    assert torch.equal(y, ops.conv3x3_wino4_bias_act(x, u, b, relu=bias, groups=groups,
                                                     mosaic="rows" if rows else False))
    assert float(e.max()) <= 2e-5 * max(1., float(r64.abs().max()))


def test_wino4_grouped_refuses():
    from vosdetectron_amd import ops
    w = torch.zeros(96, 3, 3, 3, device="cuda")
    assert ops.conv3x3_wino4_grouped_weight(w, 32) is None       # C % 64
    w = torch.zeros(256, 48, 3, 3, device="cuda")
    assert ops.conv3x3_wino4_grouped_weight(w, 5) is None        # cpg * groups != C


def test_resnext_body_grouped_route(monkeypatch):
    """X-101-32x8d's body with its stride-1 grouped conv2s on the F(4x4) grouped form
    (the workgroup gate lowered so a small batch takes it): the route counter shows it
    ran, and against a float64 CPU evaluation of the same body its P2-P6 error is no
    larger than the MIOpen route's (VOSDET_WINO4_GROUPED=0): max within 2x, mean
    within 1.5x."""
    import copy
    from vosdetectron_amd import config as vcfg, modeling
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.get("e2e_mask_rcnn_X-101-32x8d-FPN_1x")
    model, _ = build_model(cfg, seed=0, device="cuda", channels_last=True)
    monkeypatch.setattr(modeling, "_WINO4_MIN_WGS", 1)
    g = torch.Generator(device="cpu").manual_seed(0)
    xc = torch.rand((2, 3, 128, 160), generator=g) * 255 - 120
    x = xc.to("cuda").contiguous(memory_format=torch.channels_last)
    outs = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("VOSDET_WINO4_GROUPED", flag)
        modeling.ROUTE_COUNTS.clear()
        with torch.no_grad():
            outs[flag] = [t.double().cpu() for t in model.Conv_Body(x)]
        n = modeling.ROUTE_COUNTS.get("wino4_grouped", 0)
        assert (n >= 5) if flag == "1" else (n == 0), modeling.ROUTE_COUNTS
    m64 = copy.deepcopy(model).cpu().double()
    with torch.no_grad():
        ref = [t.double() for t in m64.Conv_Body(xc.double())]
    for p, q, r in zip(outs["1"], outs["0"], ref):
        ep, eq = (p - r).abs(), (q - r).abs()
        assert float(ep.max()) <= 2 * float(eq.max()) + 1e-9, (float(ep.max()), float(eq.max()))
        assert float(ep.mean()) <= 1.5 * float(eq.mean()) + 1e-12, (float(ep.mean()),
                                                                    float(eq.mean()))


@pytest.mark.parametrize("N,C,H,W,Co", [(1600, 256, 14, 14, 256), (5, 64, 14, 14, 64),
                                        (3, 128, 20, 36, 128), (2, 8, 2, 4, 64)])
@pytest.mark.parametrize("bias", [True, False])
def test_dilated2_conv_polyphase(N, C, H, W, Co, bias):
    """A 3x3 / dilation-2 / pad-2 conv (the VOS mask head) as the plain conv of its
    four polyphase sub-maps on the Winograd kernels (modeling._conv3x3_mfma): within
    the F(4x4) tolerance of torch's dilated conv, through the route counter."""
    import torch.nn as nn
    from vosdetectron_amd import modeling
    g = torch.Generator(device="cuda").manual_seed(N + C + H)
    conv = nn.Conv2d(C, Co, 3, 1, padding=2, dilation=2, bias=bias).cuda()
    with torch.no_grad():
        conv.weight.copy_(torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (3. * C ** .5))
        if bias:
            conv.bias.copy_(torch.randn(Co, device="cuda", generator=g))
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    modeling.ROUTE_COUNTS.clear()
    y = modeling._conv3x3_mfma(conv, x, bias=bias, relu=bias)
    assert y is not None and modeling.ROUTE_COUNTS.get("dilated2", 0) == 1
    assert y.is_contiguous(memory_format=torch.channels_last)
    step = max(1, 4096 // (H * W))
    with torch.no_grad():
        ref = torch.cat([conv(x[i:i + step]) for i in range(0, min(N, 256), step)])
    if bias:
        ref = F.relu(ref)
    n = ref.shape[0]
    err = float((y[:n] - ref).abs().max())
    assert err <= 5e-5 * max(1., float(ref.abs().max())), err


@pytest.mark.parametrize("N,C,H,W,Co", [(1600, 256, 14, 14, 256), (5, 64, 14, 14, 64),
                                        (3, 128, 20, 36, 128), (7, 64, 28, 30, 64)])
def test_dilated2_inplace_equals_copies(N, C, H, W, Co, monkeypatch):
    """The dilation-2 conv read / written in place by the kernel
    (vd_conv3x3_wino4_dilated2_bias_act) == the same kernel on copied polyphase
    sub-maps (VOSDET_DILATED_INPLACE=0), bit for bit (same sub-map order, same blocks)."""
    import torch.nn as nn
    from vosdetectron_amd import modeling
    g = torch.Generator(device="cuda").manual_seed(N * 5 + C + H)
    conv = nn.Conv2d(C, Co, 3, 1, padding=2, dilation=2, bias=True).cuda()
    with torch.no_grad():
        conv.weight.copy_(torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (3. * C ** .5))
        conv.bias.copy_(torch.randn(Co, device="cuda", generator=g))
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    monkeypatch.setenv("VOSDET_DILATED_INPLACE", "1")
    y1 = modeling._conv3x3_mfma(conv, x, bias=True, relu=True)
    monkeypatch.setenv("VOSDET_DILATED_INPLACE", "0")
    y0 = modeling._conv3x3_mfma(conv, x, bias=True, relu=True)
    torch.cuda.synchronize()
    assert y1 is not None and y0 is not None
    assert y1.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(y1, y0), float((y1 - y0).abs().max())
