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


@pytest.mark.parametrize("N,C,H,W,Cout", [(1, 256, 25, 42, 256), (2, 256, 14, 14, 128)])
def test_conv3x3_mid_tiles_vs_torch(monkeypatch, N, C, H, W, Cout):
    """The opt-in 64 x 128-tile variant (VOSDET_CONV3X3_MID=1, used below 4096
    big tiles) vs torch fp32, with and without bias / ReLU."""
    from vosdetectron_amd import ops
    monkeypatch.setenv("VOSDET_CONV3X3_MID", "1")
    g = torch.Generator(device="cpu").manual_seed(N + C + H + W)
    x = torch.randn(N, C, H, W, generator=g).cuda().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** .5).cuda()
    b = torch.randn(Cout, generator=g).cuda()
    for bias, relu in ((b, True), (None, False)):
        ref = F.conv2d(x, w, bias, padding=1)
        if relu:
            ref = F.relu(ref)
        got = ops.conv3x3_bias_act(x, ops.conv3x3_weight(w), bias, relu=relu)
        assert float((got - ref).abs().max()) <= 2e-5 * max(1., float(ref.abs().max()))


@pytest.mark.parametrize("N,C,H,W,Cout", [(2, 64, 9, 13, 128), (1, 256, 14, 14, 256),
                                          (3, 128, 1, 1, 128), (1, 256, 25, 42, 256),
                                          (5, 256, 7, 7, 64), (2, 64, 30, 41, 64),
                                          (1, 8, 5, 3, 64), (1, 256, 17, 70, 192)])
@pytest.mark.parametrize("relu", [False, True])
def test_conv3x3_wino_vs_torch(N, C, H, W, Cout, relu):
    """Winograd F(2x2,3x3) MFMA kernel (csrc/conv3x3_wino.hip) vs a plain torch
    fp32 conv2d(pad 1) + bias (+ ReLU): odd sizes (partial tiles and tile
    blocks; both block shapes), a 1x1 image, Cin 8..256, Cout 64..256."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cpu").manual_seed(7 * N + C + H + W + Cout)
    x = torch.randn(N, C, H, W, generator=g).cuda().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** .5).cuda()
    b = torch.randn(Cout, generator=g).cuda()
    for bias in (b, None):
        ref = F.conv2d(x, w, bias, padding=1)
        if relu:
            ref = F.relu(ref)
        got = ops.conv3x3_wino_bias_act(x, ops.conv3x3_wino_weight(w), bias, relu=relu)
        torch.cuda.synchronize()
        assert got.is_contiguous(memory_format=torch.channels_last)
        err = float((got - ref).abs().max())
        assert err <= 2e-5 * max(1., float(ref.abs().max())), err


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


def test_conv3x3_wino_input_over_4gib():
    """The Winograd kernel's patch DMA reads X through 32-bit byte offsets; an input
    of 4 GiB or more takes the 64-bit-pointer form with the zero-buffer source
    (csrc/conv3x3_wino.hip, launch_wino).  2 x 256 x 1536 x 1408 fp32 = 4.43 GB,
    vs torch fp32 at 2e-5 of the output range, borders included."""
    from vosdetectron_amd import ops
    N, C, H, W = 2, 256, 1536, 1408
    assert N * C * H * W * 4 >= 1 << 32
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(C, C, 3, 3, device="cuda", generator=g) / (3. * C ** .5)
    b = torch.randn(C, device="cuda", generator=g)
    got = ops.conv3x3_wino_bias_act(x, ops.conv3x3_wino_weight(w), b, relu=True)
    ref = F.relu(F.conv2d(x, w, b, padding=1))
    torch.cuda.synchronize()
    err = float((got - ref).abs().max())
    assert err <= 2e-5 * max(1., float(ref.abs().max())), err
    # the image borders (first / last rows and columns) are where the zero taps live
    for sl in ((slice(None), slice(None), 0), (slice(None), slice(None), H - 1),
               (slice(None), slice(None), slice(None), 0), (slice(None), slice(None), slice(None), W - 1)):
        e = float((got[sl] - ref[sl]).abs().max())
        assert e <= 2e-5 * max(1., float(ref.abs().max())), (sl, e)
    del x, got, ref
    torch.cuda.empty_cache()



@pytest.mark.parametrize("N,C,H,W,Cout", [(2, 64, 9, 13, 128), (1, 256, 14, 14, 256),
                                          (3, 128, 1, 1, 128), (1, 256, 25, 42, 256),
                                          (5, 256, 7, 7, 64), (2, 64, 30, 41, 64),
                                          (1, 8, 5, 3, 64), (1, 256, 17, 70, 192),
                                          (2, 256, 50, 84, 256), (1, 512, 33, 65, 128)])
@pytest.mark.parametrize("relu", [False, True])
def test_conv3x3_wino4_vs_torch(N, C, H, W, Cout, relu):
    """Winograd F(4x4,3x3) MFMA kernel (csrc/conv3x3_wino4.hip) vs a plain torch fp32
    conv2d(pad 1) + bias (+ ReLU): partial 4x4 tiles and 16 x 32 blocks, a 1x1
    image, Cin 8..512, Cout 64..256.  Tolerance 5e-5 of max|y| (the F(4x4)
    transforms scale by up to 8: ~2-4e-6 measured on these random data)."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cpu").manual_seed(11 * N + C + H + W + Cout)
    x = torch.randn(N, C, H, W, generator=g).cuda().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, C, 3, 3, generator=g) / (9 * C) ** .5).cuda()
    b = torch.randn(Cout, generator=g).cuda()
    u = ops.conv3x3_wino4_weight(w)
    for bias in (b, None):
        ref = F.conv2d(x, w, bias, padding=1)
        if relu:
            ref = F.relu(ref)
        got = ops.conv3x3_wino4_bias_act(x, u, bias, relu=relu)
        torch.cuda.synchronize()
        assert got.is_contiguous(memory_format=torch.channels_last)
        err = float((got - ref).abs().max())
        assert err <= 5e-5 * max(1., float(ref.abs().max())), err


def test_conv3x3_wino4_graph_replay_bit_exact():
    """The F(4x4) launch captured into a hipGraph (as bench.py replays the step)
    writes exactly what the direct launch writes: its 126 KiB of LDS is a static
    allocation (a > 64 KiB dynamic one, set by hipFuncSetAttribute, left a
    replayed launch's output unwritten), and nothing else is baked in at capture.
    Replayed twice, with new input copied into the captured buffer in between."""
    from vosdetectron_amd import ops
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(2, 64, 40, 70, generator=g).cuda().contiguous(
        memory_format=torch.channels_last)
    x2 = torch.randn(2, 64, 40, 70, generator=g).cuda().contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(128, 64, 3, 3, generator=g) / 24.).cuda()
    b = torch.randn(128, generator=g).cuda()
    u = ops.conv3x3_wino4_weight(w)
    eager = [ops.conv3x3_wino4_bias_act(xx, u, b, relu=True) for xx in (x, x2)]
    xs = x.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.conv3x3_wino4_bias_act(xs, u, b, relu=True)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        out = ops.conv3x3_wino4_bias_act(xs, u, b, relu=True)
    for xx, ref in ((x, eager[0]), (x2, eager[1])):
        xs.copy_(xx)
        out.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
