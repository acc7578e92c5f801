"""Winograd F(4x4,3x3), position-split form (csrc/conv3x3_wino4.hip,
VOSDET_WINO4_PS=1) vs the first form: the same MFMA operands in the same order and
the same output transform, so the outputs must be bit-identical -- on the step's
shapes (incl. ragged blocks: H, W not multiples of 16 / 32), with and without bias
and ReLU -- and within 5e-5 of torch fp32 (the F(4x4) tolerance)."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _run(x, u, b, relu, ps):
    from vosdetectron_amd import ops
    old = os.environ.get("VOSDET_WINO4_PS")
    os.environ["VOSDET_WINO4_PS"] = "1" if ps else "0"
    try:
        y = ops.conv3x3_wino4_bias_act(x, u, b, relu=relu)
        torch.cuda.synchronize()
        return y
    finally:
        if old is None:
            del os.environ["VOSDET_WINO4_PS"]
        else:
            os.environ["VOSDET_WINO4_PS"] = old


@pytest.mark.parametrize("N,C,H,W,Co", [(2, 64, 20, 36, 64), (1, 256, 50, 84, 256),
                                        (3, 128, 17, 45, 128), (2, 512, 25, 42, 512),
                                        (1, 8, 9, 9, 64), (4, 24, 33, 31, 128)])
@pytest.mark.parametrize("bias", [True, False])
def test_wino4ps_bit_identical_to_first_form(N, C, H, W, Co, bias):
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(N * 1000 + C + H)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(Co, C, 3, 3, device="cuda", generator=g) / (3. * C ** .5)
    b = torch.randn(Co, device="cuda", generator=g) if bias else None
    u = ops.conv3x3_wino4_weight(w)
    y1 = _run(x, u, b, bias, False)
    y2 = _run(x, u, b, bias, True)
    assert torch.equal(y1, y2), float((y1 - y2).abs().max())
    ref = F.conv2d(x, w, b, padding=1)
    if bias:
        ref = F.relu(ref)
    err = float((y2 - ref).abs().max())
    assert err <= 5e-5 * max(1., float(ref.abs().max())), err


def test_wino4ps_benched_p2():
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(32, 256, 200, 336, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(256, 256, 3, 3, device="cuda", generator=g) / 48.
    b = torch.randn(256, device="cuda", generator=g)
    u = ops.conv3x3_wino4_weight(w)
    y1 = _run(x, u, b, False, False)
    y2 = _run(x, u, b, False, True)
    assert torch.equal(y1, y2), float((y1 - y2).abs().max())
