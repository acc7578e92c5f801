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


def test_gemm_bias_act_vs_torch():
    """vd_gemm_bias_act (hipBLASLt, epilogue fused) vs a plain torch fp32
    reference of the same op: relu(a @ w.T + b + r) / (a @ w.T + b)."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(3)
    for M, K, N in [(4096, 64, 256), (1000, 256, 64), (777, 512, 2048), (1, 128, 32)]:
        a = torch.randn(M, K, device="cuda", generator=g)
        w = torch.randn(N, K, device="cuda", generator=g) / K ** .5
        b = torch.randn(N, device="cuda", generator=g)
        r = torch.randn(M, N, device="cuda", generator=g)
        ref = torch.relu(a @ w.t() + b + r)
        got = ops.gemm_bias_act(a, w, b, residual=r, relu=True)
        assert float((got - ref).abs().max()) <= 2e-5 * max(1., float(ref.abs().max()))
        ref2 = a @ w.t() + b
        got2 = ops.gemm_bias_act(a, w, b, relu=False)
        assert float((got2 - ref2).abs().max()) <= 2e-5 * max(1., float(ref2.abs().max()))


@pytest.mark.parametrize("K,N", [(64, 256), (64, 64), (256, 64), (128, 512)])
@pytest.mark.parametrize("M", [4096, 1003, 16, 1])
def test_gemm1x1_mfma_vs_torch(monkeypatch, K, N, M):
    """The hand-written MFMA 1x1-conv GEMM (csrc/gemm1x1.hip, forced with
    VOSDET_GEMM_MFMA=1) vs a plain torch fp32 reference: relu(a @ w.T + b + r),
    relu(a @ w.T + b), a @ w.T + b + r and a @ w.T + b, incl. a ragged pixel tail."""
    from vosdetectron_amd import ops
    monkeypatch.setenv("VOSDET_GEMM_MFMA", "1")
    g = torch.Generator(device="cuda").manual_seed(K + N + M)
    a = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) / K ** .5
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g)
    for res in (r, None):
        for relu in (True, False):
            ref = a @ w.t() + b + (res if res is not None else 0.)
            if relu:
                ref = torch.relu(ref)
            got = ops.gemm_bias_act(a, w, b, residual=res, relu=relu)
            tol = 2e-5 * max(1., float(ref.abs().max()))
            assert float((got - ref).abs().max()) <= tol, (M, K, N, res is not None, relu)


@pytest.mark.parametrize("M", [4096, 1003, 1])
def test_gemm_dual_vs_torch(M):
    """vd_gemm_dual_bias_act (conv3 + stride-1 downsample as one two-operand MFMA
    GEMM) vs torch fp32: relu(a1 @ w[:, :64].T + a2 @ w[:, 64:].T + b); shapes the
    kernel does not serve return None (the caller falls back)."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(M)
    a1 = torch.randn(M, 64, device="cuda", generator=g)
    a2 = torch.randn(M, 64, device="cuda", generator=g)
    w = torch.randn(256, 128, device="cuda", generator=g) / 128 ** .5
    b = torch.randn(256, device="cuda", generator=g)
    for relu in (True, False):
        ref = a1 @ w[:, :64].t() + a2 @ w[:, 64:].t() + b
        if relu:
            ref = torch.relu(ref)
        got = ops.gemm_dual_bias_act(a1, a2, w, b, relu=relu)
        assert float((got - ref).abs().max()) <= 2e-5 * max(1., float(ref.abs().max()))
    assert ops.gemm_dual_bias_act(a1, a2[:, :32].contiguous(), w[:, :96].contiguous(), b) is None


def test_bottleneck_gemm_path_matches_conv_path(monkeypatch):
    """A folded Bottleneck on channels_last input: the GEMM-epilogue path equals
    the MIOpen conv + vd_bias_act path within fp32 accumulation-order noise
    (identity and downsample residuals, stride 1 and 2)."""
    from vosdetectron_amd.modeling import Bottleneck, prepare_bottlenecks
    torch.manual_seed(0)
    for cin, cout, inner, stride in [(256, 256, 64, 1), (64, 256, 64, 1), (256, 512, 128, 2)]:
        blk = Bottleneck(cin, cout, inner, stride, 1).cuda().eval()
        for m in blk.modules():
            if isinstance(m, torch.nn.Conv2d):
                torch.nn.init.normal_(m.weight, 0, (2. / m.weight[0].numel()) ** .5)
        prepare_bottlenecks([blk])
        x = torch.randn(2, cin, 40, 56, device="cuda").contiguous(
            memory_format=torch.channels_last)
        with torch.no_grad():
            y = blk(x)
            monkeypatch.setenv("VOSDET_GEMM_EPILOGUE", "0")
            y0 = blk(x)
            monkeypatch.delenv("VOSDET_GEMM_EPILOGUE")
        assert y.is_contiguous(memory_format=torch.channels_last)
        assert float((y - y0).abs().max()) <= 1e-4 * max(1., float(y0.abs().max()))


@pytest.mark.parametrize("N,C,H,W,A", [(2, 256, 50, 84, 3), (3, 64, 7, 11, 1), (1, 128, 1, 1, 3),
                                       (16, 256, 13, 21, 3)])
def test_rpn_head_vs_torch(N, C, H, W, A):
    """vd_rpn_head (bias + ReLU + cls/bbox 1x1 + sigmoid in one pass over the raw
    RPN conv output) against the unfused fp32 PyTorch sequence of FPN.py:376-422;
    tile tails (N*H*W not a multiple of 64) included."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cpu").manual_seed(N * 1000 + C + H)
    x = torch.randn(N, C, H, W, generator=g).cuda().contiguous(memory_format=torch.channels_last)
    cb = (torch.randn(C, generator=g) * 0.5).cuda()
    w = (torch.randn(5 * A, C, generator=g) / C ** 0.5).cuda()
    b = torch.randn(5 * A, generator=g).cuda()
    h = F.relu(x + cb.view(1, -1, 1, 1))
    o = F.conv2d(h.contiguous(), w.view(5 * A, C, 1, 1), b)
    cls, box = ops.rpn_head(x, cb, w, b, A)
    torch.cuda.synchronize()
    assert cls.shape == (N, A, H, W) and box.shape == (N, 4 * A, H, W) and cls.is_contiguous()
    torch.testing.assert_close(cls, torch.sigmoid(o[:, :A]), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(box, o[:, A:], rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("N,C,H,W", [(2, 64, 40, 66), (1, 64, 13, 7), (3, 8, 1, 2), (1, 64, 400, 672)])
def test_bias_relu_maxpool_bit_exact(N, C, H, W):
    """vd_bias_relu_maxpool == vd_bias_act(relu) + MaxPool2d(3, 2, 1) bit for bit
    (basic_bn_stem's tail, ResNet.py:224-230), odd sizes included."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cpu").manual_seed(H * W + C)
    x = torch.randn(N, C, H, W, generator=g).cuda().contiguous(memory_format=torch.channels_last)
    b = torch.randn(C, generator=g).cuda()
    ref = F.max_pool2d(ops.bias_act_(x.clone(memory_format=torch.channels_last), b, relu=True),
                       kernel_size=3, stride=2, padding=1)
    got = ops.bias_relu_maxpool(x, b)
    torch.cuda.synchronize()
    assert got.shape == ref.shape and got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(got, ref)
