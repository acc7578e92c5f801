"""The split-bf16 GEMM (csrc/gemm_split3.hip, vd_gemm_split3_bias_act): fp32
operands split into three bf16 pieces, the six largest piece products accumulated
in fp32 on the bf16 matrix cores.  Its accuracy claim is "fp32's": on every shape
the error against an fp64 reference stays at torch's own fp32 GEMM error (mean
within 1.5x, max within 3x: the max of a few hundred rows is a noisy statistic)
and within the 2e-5 relative bound the fp32 GEMM tests use.
Also: every tile configuration, ragged pixel counts, residual / ReLU epilogues,
determinism, graph replay, the weight cache following in-place updates, and the
routing rule of ops.gemm_bias_act."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _case(M, N, K, res, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = torch.randn(M, K, device=DEV, generator=g).relu_()
    w = torch.randn(N, K, device=DEV, generator=g) / K ** .5
    b = torch.randn(N, device=DEV, generator=g) * .1
    r = torch.randn(M, N, device=DEV, generator=g) if res else None
    return a, w, b, r


def _ref64(a, w, b, r, relu):
    y = a.double() @ w.double().t() + b.double()
    if r is not None:
        y = y + r.double()
    return y.relu() if relu else y


def _errs(got, ref):
    e = (got.double() - ref).abs()
    s = float(ref.abs().max())
    return float(e.max()) / s, float(e.mean()) / s


@pytest.mark.parametrize("M,N,K,res,relu", [
    (1000, 64, 256, False, True), (777, 128, 512, True, True), (4099, 256, 1024, False, False),
    (3000, 512, 2048, True, True), (2048, 1024, 256, False, True), (513, 2048, 512, True, False),
    (333, 1024, 12544, False, True), (64, 64, 16, False, True), (1, 256, 32, True, True)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5])
def test_split3_fp32_accuracy(M, N, K, res, relu, cfg):
    from vosdetectron_amd import ops
    if (cfg in (1, 5) and N % 256) or (cfg in (2, 4) and N % 128):
        pytest.skip("tile needs N %% %d" % (256 if cfg in (1, 5) else 128))
    a, w, b, r = _case(M, N, K, res, M + N + K)
    ref = _ref64(a, w, b, r, relu)
    got = ops.gemm_split3_bias_act(a, ops.gemm_split3_weight(w), b, residual=r, relu=relu,
                                   cfg=cfg)
    t32 = a @ w.t() + b
    if r is not None:
        t32 = t32 + r
    if relu:
        t32 = t32.relu()
    torch.cuda.synchronize()
    mx, mean = _errs(got, ref)
    tmx, tmean = _errs(t32, ref)
    assert mx <= 2e-5, mx
    assert mx <= 3 * tmx + 1e-7 and mean <= 1.5 * tmean + 1e-9, (mx, mean, tmx, tmean)


def test_split3_deterministic_and_graph_replay():
    from vosdetectron_amd import ops
    a, w, b, r = _case(5000, 256, 512, True, 5)
    wp = ops.gemm_split3_weight(w)
    y0 = ops.gemm_split3_bias_act(a, wp, b, residual=r)
    y1 = ops.gemm_split3_bias_act(a, wp, b, residual=r)
    assert torch.equal(y0, y1)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            out = ops.gemm_split3_bias_act(a, wp, b, residual=r)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, y0)


def test_gemm_bias_act_routes_and_cache():
    """K >= SPLIT3_MIN_K runs split (matches the direct split call bit for bit);
    the cached split image follows an in-place weight update; VOSDET_GEMM_SPLIT3=0
    and K below the threshold keep the fp32 kernels (within 2e-5 of torch)."""
    import os
    from vosdetectron_amd import ops
    a, w, b, _ = _case(3000, 256, 512, False, 9)
    y = ops.gemm_bias_act(a, w, b, relu=True)
    assert torch.equal(y, ops.gemm_split3_bias_act(a, ops.gemm_split3_weight(w), b))
    with torch.no_grad():
        w.mul_(0.5)
    y2 = ops.gemm_bias_act(a, w, b, relu=True)
    ref = (a @ w.t() + b).relu()
    torch.cuda.synchronize()
    assert float((y2 - ref).abs().max()) <= 2e-5 * float(ref.abs().max())
    os.environ["VOSDET_GEMM_SPLIT3"] = "0"
    try:
        y3 = ops.gemm_bias_act(a, w, b, relu=True)
    finally:
        del os.environ["VOSDET_GEMM_SPLIT3"]
    torch.cuda.synchronize()
    assert float((y3 - ref).abs().max()) <= 2e-5 * float(ref.abs().max())
    assert not torch.equal(y3, y2)  # the fp32 kernels sum in another order


def test_split3_rejects_bad_shapes():
    from vosdetectron_amd import _lib, ops
    assert ops.gemm_split3_weight(torch.randn(96, 64, device=DEV)) is None   # N % 64
    assert ops.gemm_split3_weight(torch.randn(64, 40, device=DEV)) is None   # K % 16
    wp = ops.gemm_split3_weight(torch.randn(128, 64, device=DEV))
    with pytest.raises(ValueError):
        ops.gemm_split3_bias_act(torch.randn(10, 32, device=DEV), wp, torch.zeros(128, device=DEV))
    with pytest.raises(_lib.VosdetError):  # a 256-channel tile on N = 128
        ops.gemm_split3_bias_act(torch.randn(10, 64, device=DEV), wp,
                                 torch.zeros(128, device=DEV), cfg=1)


@pytest.mark.parametrize("n,K,H,W", [(2, 256, 16, 20), (3, 512, 10, 14), (1, 1024, 6, 8),
                                     (32, 256, 200, 336)])
def test_split3_fpn_topdown_lateral(n, K, H, W):
    """The FPN top-down step (FPN.py:292-300: conv_lateral(lateral) + nearest-2x
    upsample of top) in one split-bf16 launch, vs fp64 (and within 2x of torch
    fp32's own error); through the module (modeling.TopdownLateral) as well."""
    import torch.nn.functional as F
    from vosdetectron_amd import modeling, ops
    g = torch.Generator(device="cuda").manual_seed(K + H)
    lat = torch.randn(n, K, H, W, device=DEV, generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(256, K, 1, 1, device=DEV, generator=g) / K ** .5
    b = torch.randn(256, device=DEV, generator=g)
    top = torch.randn(n, 256, H // 2, W // 2, device=DEV, generator=g).contiguous(
        memory_format=torch.channels_last)
    rows = min(n * H * W, 20000)
    a2 = lat.permute(0, 2, 3, 1).reshape(-1, K)
    up = F.interpolate(top, scale_factor=2, mode="nearest").permute(0, 2, 3, 1).reshape(-1, 256)
    ref = (a2[:rows].double() @ w.view(256, K).double().t() + b.double()) + up[:rows].double()
    got = ops.gemm_split3_bias_act(a2, ops.gemm_split3_weight(w.view(256, K)), b,
                                   residual=top.permute(0, 2, 3, 1).reshape(-1, 256),
                                   relu=False, up_hw=(H, W))
    # torch's fp32 GEMM of the same sum (MIOpen's conv2d can reduce K in a tree, a
    # different error class from any K-ordered GEMM, so the GEMM is the comparison)
    t32 = (a2[:rows] @ w.view(256, K).t() + b) + up[:rows]
    torch.cuda.synchronize()
    mx, mean = _errs(got[:rows], ref)
    tmx, tmean = _errs(t32, ref)
    assert mx <= 2e-5 and mx <= 3 * tmx + 1e-7 and mean <= 1.5 * tmean + 1e-9, \
        (mx, mean, tmx, tmean)
    m = modeling.TopdownLateral(256, K).to(DEV)
    with torch.no_grad():
        m.conv_lateral.weight.copy_(w)
        m.conv_lateral.bias.copy_(b)
    modeling.prepare_topdown_lateral(m)
    y = m(top, lat)
    torch.cuda.synchronize()
    assert y.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(y.permute(0, 2, 3, 1).reshape(-1, 256), got)
    del lat, top, got, t32, y, up, a2


@pytest.mark.parametrize("n,C,H,W,N", [(2, 256, 20, 34, 128), (3, 512, 11, 17, 1024),
                                       (32, 256, 200, 336, 512)])
def test_split3_stride2_rows(n, C, H, W, N):
    """A stride-2 pad-0 1x1 conv read at stride 2 by the GEMM itself (sub_hw): equal
    bit for bit to the same GEMM over the subsampled copy, odd sizes included."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(C + H)
    x = torch.randn(n, C, H, W, device=DEV, generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(N, C, device=DEV, generator=g) / C ** .5
    b = torch.randn(N, device=DEV, generator=g)
    wp = ops.gemm_split3_weight(w)
    xs = x[:, :, ::2, ::2].contiguous(memory_format=torch.channels_last)
    want = ops.gemm_split3_bias_act(xs.permute(0, 2, 3, 1).reshape(-1, C), wp, b)
    got = ops.gemm_split3_bias_act(x.permute(0, 2, 3, 1).reshape(-1, C), wp, b, sub_hw=(H, W))
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    del x, xs, want, got


@pytest.mark.parametrize("R,ncls", [(64, 81), (333, 81), (7, 1)])
@torch.no_grad()
def test_mask_head_upconv_logits_fused(R, ncls):
    """The mask head's upconv5 + ReLU + class-selected logits + sigmoid in one launch
    (vd_mask_head_upconv_logits) vs the unfused path (the upconv GEMM's output written,
    then the per-RoI class dot product of MaskRCNNOutputs.selected_from_up) and vs
    an fp64 reference: within 1e-5 (probabilities)."""
    from vosdetectron_amd import modeling, ops
    from vosdetectron_amd import config as vcfg
    cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
    g = torch.Generator(device="cuda").manual_seed(R + ncls)
    head = modeling.MaskHeadV1upXconvs(256, None, 1. / 16, cfg).to(DEV)
    outs = modeling.MaskRCNNOutputs(256, ncls).to(DEV)
    with torch.no_grad():
        head.upconv.weight.copy_(torch.randn(256, 256, 2, 2, device=DEV, generator=g) / 16)
        head.upconv.bias.copy_(torch.randn(256, device=DEV, generator=g) * .1)
        outs.classify.weight.copy_(torch.randn(ncls, 256, 1, 1, device=DEV, generator=g) / 16)
        outs.classify.bias.copy_(torch.randn(ncls, device=DEV, generator=g))
    head.prepare()
    P = 14
    x = torch.randn(R * P * P, 256, device=DEV, generator=g).relu_()
    cls = torch.randint(0, 81, (R,), device=DEV, generator=g, dtype=torch.int32)
    ch = outs._channel(cls).to(torch.int32)
    got = ops.mask_head_upconv_logits(x, ops.gemm_split3_weight(head.up_wt), head.up_b,
                                      outs.classify.weight.view(ncls, -1), outs.classify.bias,
                                      ch, P)
    unf = outs.selected_from_up(head._upconv_nhwc(x, R, P), cls)
    # fp64: upconv as the GEMM over (i, j, co), relu, the class dot product, sigmoid
    y = (x.double() @ head.up_wt.double().t() + head.up_b.double()).relu()
    y = y.view(R, P, P, 2, 2, 256)
    w = outs.classify.weight.view(ncls, 256).double()[ch.long()]
    z = torch.einsum("rhwijc,rc->rhiwj", y, w).reshape(R, 2 * P, 2 * P)
    ref = torch.sigmoid(z + outs.classify.bias.double()[ch.long()].view(-1, 1, 1))
    torch.cuda.synchronize()
    assert got.shape == (R, 2 * P, 2 * P)
    assert float((got.double() - ref).abs().max()) <= 1e-5
    assert float((got - unf).abs().max()) <= 1e-5


@pytest.mark.parametrize("M,K1,K2,N", [(5000, 64, 64, 256), (2150400 // 16, 64, 64, 256),
                                       (777, 128, 256, 512)])
def test_split3_two_operands(M, K1, K2, N):
    """A2: the last K2 input channels from a second operand -- a stage's first block
    (conv3 of h + the stride-1 downsample of x) in one GEMM: equal bit for bit to the
    same GEMM over the concatenated [h | x] rows, at torch fp32's error level."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(M + K1)
    h = torch.randn(M, K1, device=DEV, generator=g).relu_()
    x = torch.randn(M, K2, device=DEV, generator=g).relu_()
    w = torch.randn(N, K1 + K2, device=DEV, generator=g) / (K1 + K2) ** .5
    b = torch.randn(N, device=DEV, generator=g)
    wp = ops.gemm_split3_weight(w)
    got = ops.gemm_split3_bias_act(h, wp, b, a2=x)
    want = ops.gemm_split3_bias_act(torch.cat([h, x], 1), wp, b)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    ref = (torch.cat([h, x], 1).double() @ w.double().t() + b.double()).relu()
    mx, _ = _errs(got, ref)
    assert mx <= 2e-5, mx


def test_split3_weight_image_is_the_rne_split():
    """vd_gemm_split3_weight's image holds, bit for bit, the round-to-nearest-even bf16
    pieces torch's own conversion gives (tests/test_split3_cpu.py's arithmetic), in the
    [K/16][N/32][piece][lane = 32 h + r][8] order: W[32 t + r][16 s + 8 h + j]."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(7)
    N, K = 128, 64
    w = (torch.randn(N, K, device=DEV, generator=g) *
         torch.logspace(-20, 20, K, device=DEV)[None, :])
    img = ops.gemm_split3_weight(w).view(torch.int16).view(K // 16, N // 32, 3, 2, 32, 8)
    x0 = w.to(torch.bfloat16).float()
    x1 = (w - x0).to(torch.bfloat16).float()
    x2 = (w - x0 - x1).to(torch.bfloat16).float()
    for p, piece in enumerate((x0, x1, x2)):
        ref = piece.to(torch.bfloat16).view(torch.int16)           # [N][K]
        ref = ref.view(N // 32, 32, K // 16, 2, 8).permute(2, 0, 3, 1, 4)  # [s][t][h][r][j]
        assert torch.equal(img[:, :, p], ref), p


@pytest.mark.parametrize("M,K,N,cfg", [(5000, 256, 256, 0), (1237, 512, 1024, 0),
                                       (4099, 1024, 256, 2), (999, 256, 128, 3),
                                       (3000, 512, 512, 4), (2048, 2048, 512, 5)])
def test_split3_a_bias_prologue_bit_identical(M, K, N, cfg):
    """a_bias: A enters as relu(A + a_bias) -- bit-identical to applying the bias + ReLU
    in a separate fp32 pass and splitting that (ResNeXt's grouped conv2 epilogue fused
    into conv3's A load), with and without a residual; with a second operand the bias
    touches A's channels only; with a stride-2 A as well."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(M + K)
    a = torch.randn(M, K, device=DEV, generator=g)  # raw conv output: both signs
    ab = torch.randn(K, device=DEV, generator=g) * .5
    w = torch.randn(N, K, device=DEV, generator=g) / K ** .5
    b = torch.randn(N, device=DEV, generator=g) * .1
    r = torch.randn(M, N, device=DEV, generator=g)
    wp = ops.gemm_split3_weight(w)
    pre = torch.relu(a + ab)
    for res in (None, r):
        got = ops.gemm_split3_bias_act(a, wp, b, residual=res, cfg=cfg, a_bias=ab)
        want = ops.gemm_split3_bias_act(pre, wp, b, residual=res, cfg=cfg)
        torch.cuda.synchronize()
        assert torch.equal(got, want), float((got - want).abs().max())
    # the ops.gemm_bias_act route passes it through
    assert torch.equal(ops.gemm_bias_act(a, w, b, relu=True, a_bias=ab),
                       ops.gemm_bias_act(pre, w, b, relu=True))
    # two operands: the bias covers A's K1 channels, not A2's
    K1 = K // 2
    got = ops.gemm_split3_bias_act(a[:, :K1].contiguous(), wp, b,
                                   a2=a[:, K1:].contiguous(), a_bias=ab[:K1].contiguous())
    want = ops.gemm_split3_bias_act(pre[:, :K1].contiguous(), wp, b,
                                    a2=a[:, K1:].contiguous())
    assert torch.equal(got, want)
    with pytest.raises(ValueError):
        ops.gemm_split3_bias_act(a, wp, b, a_bias=ab[:K1].contiguous())


def test_split3_a_bias_stride2():
    from vosdetectron_amd import ops
    g = torch.Generator(device="cuda").manual_seed(5)
    n, C, H, W, N = 3, 256, 21, 34, 512
    x = torch.randn(n, H, W, C, device=DEV, generator=g)
    ab = torch.randn(C, device=DEV, generator=g)
    w = torch.randn(N, C, device=DEV, generator=g) / C ** .5
    b = torch.randn(N, device=DEV, generator=g)
    wp = ops.gemm_split3_weight(w)
    got = ops.gemm_split3_bias_act(x.reshape(-1, C), wp, b, sub_hw=(H, W), a_bias=ab)
    want = ops.gemm_split3_bias_act(torch.relu(x + ab).reshape(-1, C), wp, b, sub_hw=(H, W))
    assert torch.equal(got, want)


def test_resnext_block_conv2_prologue_bit_identical(monkeypatch):
    """X-101-32x8d's body (grouped conv2 on MIOpen): conv2's bias + ReLU applied by
    conv3's split GEMM (the default) == the separate bias / ReLU pass
    (VOSDET_CONV2_PROLOGUE=0), bit for bit, on the res2-res5 stages."""
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.get("e2e_mask_rcnn_X-101-32x8d-FPN_1x")
    model, _ = build_model(cfg, seed=0, device=DEV, channels_last=True)
    x = (torch.rand((2, 3, 256, 320)) * 255 - 120).to(DEV).contiguous(
        memory_format=torch.channels_last)
    outs = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("VOSDET_CONV2_PROLOGUE", flag)
        with torch.no_grad():
            outs[flag] = [t.clone() for t in model.Conv_Body(x)]
    for p, q in zip(outs["1"], outs["0"]):
        assert torch.equal(p, q), float((p - q).abs().max())
