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
