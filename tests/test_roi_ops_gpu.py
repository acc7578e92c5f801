"""GPU parity of the RoI operators (HIP, through the C ABI) against the oracle.

Bit-exact where the kernel keeps the reference's evaluation order (RoIAlign
fwd NCHW / NHWC, RoIPool, RoICrop, legacy RoIAlign); the atomics-based backward
is compared within fp32 tolerance (sum order differs, as it does between two
runs of the reference's own atomicAdd kernel)."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda"


def make_rois(rng, n, img_w, img_h, batch=1, edge=True):
    s = np.exp(rng.uniform(np.log(4), np.log(600), n))
    a = np.exp(rng.uniform(np.log(0.5), np.log(2), n))
    w, h = s / np.sqrt(a), s * np.sqrt(a)
    cx, cy = rng.uniform(-20, img_w + 20, n), rng.uniform(-20, img_h + 20, n)
    b = rng.integers(0, batch, n)
    r = np.stack([b, cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], 1).astype(np.float32)
    if edge:
        extra = np.array([
            [0, -50, -50, -10, -10],        # fully outside (top-left)
            [0, img_w + 5, img_h + 5, img_w + 40, img_h + 40],  # fully outside
            [0, 10, 10, 10, 10],            # degenerate -> 1x1
            [0, 30, 30, 20, 20],            # malformed x2<x1
            [0, 0, 0, img_w - 1, img_h - 1],  # whole image
            [0, img_w - 2, img_h - 2, img_w + 3, img_h + 3],  # straddles the far edge
            [0, -0.75, -0.75, 2.2, 2.2],    # straddles the near edge
        ], np.float32)
        extra[:, 0] = np.minimum(extra[:, 0], batch - 1)
        r = np.concatenate([r, extra])
    return r


@pytest.mark.parametrize("P,sr", [(7, 2), (14, 2), (7, 0), (5, 2)])
def test_roi_align_nchw_bit_exact(P, sr):
    from vosdetectron_amd import ops
    rng = np.random.default_rng(P * 10 + sr)
    B, C, H, W = 2, 24, 37, 51
    f = rng.standard_normal((B, C, H, W)).astype(np.float32)
    rois = make_rois(rng, 60, W * 8, H * 8, batch=B)
    scale = 1. / 8
    ref = orc.roi_align(f, rois, P, P, scale, sr)
    out = ops.roi_align_forward(torch.from_numpy(f).to(DEV), torch.from_numpy(rois).to(DEV), P, P,
                                scale, sr).cpu().numpy()
    assert np.array_equal(out, ref)


def _pyramid(rng, B, C, sizes):
    return [rng.standard_normal((B, C, h, w)).astype(np.float32) for (h, w) in sizes]


@pytest.mark.parametrize("P,sr,C", [(7, 2, 256), (14, 2, 256), (7, 0, 256), (7, 2, 64),
                                    (14, 2, 520), (6, 2, 128)])
def test_roi_align_fpn_nhwc_bit_exact(P, sr, C, monkeypatch):
    """One launch over 4 levels vs the reference per-level loop + restore
    (model_builder.py:252-303) evaluated by the oracle.  Kernel variant 3 keeps
    the reference's per-sample arithmetic order: bit-exact."""
    from vosdetectron_amd import ops
    monkeypatch.setenv("VOSDET_ROIALIGN_VARIANT", "3")
    rng = np.random.default_rng(1000 + P + sr + C)
    B = 2
    sizes = [(50, 84), (25, 42), (13, 21), (7, 11)]
    scales = [1. / 4, 1. / 8, 1. / 16, 1. / 32]
    feats = _pyramid(rng, B, C, sizes)
    rois = make_rois(rng, 120, 336, 200, batch=B)
    lv = orc.map_rois_to_fpn_levels(rois[:, 1:5], 2, 5).astype(np.int32) - 2
    d = {"rois": rois}
    order = np.empty((0,))
    for k in range(4):
        idx = np.where(lv == k)[0]
        d["rois_fpn%d" % (k + 2)] = rois[idx]
        order = np.concatenate([order, idx])
    d["rois_idx_restore_int32"] = np.argsort(order, kind="stable").astype(np.int32)
    ref = orc.roi_feature_transform(feats[::-1], d, "rois", P, scales[::-1], sr)
    nhwc = [torch.from_numpy(x).to(DEV).permute(0, 2, 3, 1).contiguous() for x in feats]
    out = ops.roi_align_fpn(nhwc, scales, torch.from_numpy(rois).to(DEV),
                            torch.from_numpy(lv).to(DEV), P, sr).cpu().numpy()
    assert np.array_equal(out, ref)
    # NHWC output layout (product path) holds the same numbers
    if P in (7, 14):
        o2 = ops.roi_align_fpn(nhwc, scales, torch.from_numpy(rois).to(DEV),
                               torch.from_numpy(lv).to(DEV), P, sr, out_layout="nhwc")
        assert np.array_equal(o2.permute(0, 3, 1, 2).cpu().numpy(), ref)
    # scheduling permutation must not move outputs
    perm = torch.from_numpy(rng.permutation(len(rois)).astype(np.int32)).to(DEV)
    if P in (7, 14):
        out2 = ops.roi_align_fpn(nhwc, scales, torch.from_numpy(rois).to(DEV),
                                 torch.from_numpy(lv).to(DEV), P, sr, roi_order=perm)
        assert np.array_equal(out2.cpu().numpy(), ref)


def test_roi_align_function_api_and_backward():
    from vosdetectron_amd.ops import RoIAlignFunction
    rng = np.random.default_rng(7)
    B, C, H, W = 1, 8, 20, 30
    f = rng.standard_normal((B, C, H, W)).astype(np.float32)
    rois = make_rois(rng, 30, W * 4, H * 4, batch=B)
    ft = torch.from_numpy(f).to(DEV).requires_grad_(True)
    out = RoIAlignFunction(7, 7, 0.25, 2)(ft, torch.from_numpy(rois).to(DEV))
    g = rng.standard_normal(out.shape).astype(np.float32)
    out.backward(torch.from_numpy(g).to(DEV))
    ref = orc.roi_align_backward(g, rois, f.shape, 0.25, 2)
    np.testing.assert_allclose(ft.grad.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    with pytest.raises(NotImplementedError):
        RoIAlignFunction(7, 7, 0.25, 2)(torch.from_numpy(f), torch.from_numpy(rois))


def test_roi_align_rejects_bad_rois():
    from vosdetectron_amd import ops
    from vosdetectron_amd._lib import VosdetError
    f = torch.zeros((1, 4, 8, 8), device=DEV)
    with pytest.raises(VosdetError):
        ops.roi_align_forward(f, torch.zeros((3, 4), device=DEV), 7, 7, 1., 2)
    out = ops.roi_align_forward(f, torch.zeros((0, 5), device=DEV), 7, 7, 1., 2)
    assert out.shape == (0, 4, 7, 7)


def test_legacy_pool_crop_bit_exact():
    from vosdetectron_amd import ops
    rng = np.random.default_rng(11)
    B, C, H, W = 2, 16, 23, 31
    f = rng.standard_normal((B, C, H, W)).astype(np.float32)
    rois = make_rois(rng, 40, W * 16, H * 16, batch=B)
    ft, rt = torch.from_numpy(f).to(DEV), torch.from_numpy(rois).to(DEV)
    ref = orc.roi_align_legacy(f, rois, 7, 7, 1. / 16)
    assert np.array_equal(ops.roi_align_legacy(ft, rt, 7, 7, 1. / 16).cpu().numpy(), ref)
    ref_o, ref_a = orc.roi_pool(f, rois, 7, 7, 1. / 16)
    fn = ops.RoIPoolFunction(7, 7, 1. / 16)
    out = fn(ft, rt)
    assert np.array_equal(out.cpu().numpy(), ref_o)
    assert np.array_equal(fn.argmax.cpu().numpy(), ref_a)
    # RoICrop: grids from the reference's affine_grid_gen shape, incl. outside taps
    R, G = 8, 14
    grid = rng.uniform(-1.3, 1.3, (R, G, G, 2)).astype(np.float32)
    ref_c = orc.roi_crop(f, grid)
    out_c = ops.RoICropFunction()(ft, torch.from_numpy(grid).to(DEV)).cpu().numpy()
    assert np.array_equal(out_c, ref_c)


def test_roi_pool_backward_matches_scatter():
    from vosdetectron_amd import ops
    rng = np.random.default_rng(5)
    f = rng.standard_normal((1, 4, 12, 12)).astype(np.float32)
    rois = make_rois(rng, 10, 48, 48, edge=False)
    ft = torch.from_numpy(f).to(DEV).requires_grad_(True)
    fn = ops.RoIPoolFunction(3, 3, 0.25)
    out = fn(ft, torch.from_numpy(rois).to(DEV))
    g = np.ones(out.shape, np.float32)
    out.backward(torch.from_numpy(g).to(DEV))
    _, arg = orc.roi_pool(f, rois, 3, 3, 0.25)
    ref = np.zeros(f.size, np.float32)
    np.add.at(ref, arg[arg >= 0].ravel(), 1.0)
    assert np.array_equal(ft.grad.cpu().numpy().ravel(), ref)


@pytest.mark.parametrize("variant", [None, "3", "11"])
@pytest.mark.parametrize("P,C", [(7, 256), (14, 256), (7, 64), (14, 520)])
def test_roi_align_fpn_separable_within_tolerance(P, C, variant, monkeypatch):
    """Separable NHWC kernels (variants 8 / 10): same sampling, summation
    re-associated as sum_x w_x sum_y w_y F, so they hold the reference to 1e-4
    (north_star's RoIAlign tolerance), not bit-for-bit."""
    from vosdetectron_amd import ops
    rng = np.random.default_rng(2000 + P + C)
    B = 2
    sizes = [(50, 84), (25, 42), (13, 21), (7, 11)]
    scales = [1. / 4, 1. / 8, 1. / 16, 1. / 32]
    feats = _pyramid(rng, B, C, sizes)
    rois = make_rois(rng, 150, 336, 200, batch=B)
    rois[:4, 1:5] = [[-30, -20, 40, 30], [300, 180, 400, 260], [0, 0, 0.5, 0.5],
                     [330, 190, 335.9, 199.9]]  # partly outside / degenerate / at the edge
    lv = orc.map_rois_to_fpn_levels(rois[:, 1:5], 2, 5).astype(np.int32) - 2
    d = {"rois": rois}
    order = np.empty((0,))
    for k in range(4):
        idx = np.where(lv == k)[0]
        d["rois_fpn%d" % (k + 2)] = rois[idx]
        order = np.concatenate([order, idx])
    d["rois_idx_restore_int32"] = np.argsort(order, kind="stable").astype(np.int32)
    ref = orc.roi_feature_transform(feats[::-1], d, "rois", P, scales[::-1], 2)
    nhwc = [torch.from_numpy(x).to(DEV).permute(0, 2, 3, 1).contiguous() for x in feats]
    if variant is None:  # the product default
        monkeypatch.delenv("VOSDET_ROIALIGN_VARIANT", raising=False)
    else:
        monkeypatch.setenv("VOSDET_ROIALIGN_VARIANT", variant)
    args = (nhwc, scales, torch.from_numpy(rois).to(DEV), torch.from_numpy(lv).to(DEV), P, 2)
    o1 = ops.roi_align_fpn(*args).cpu().numpy()
    o2 = ops.roi_align_fpn(*args, out_layout="nhwc").permute(0, 3, 1, 2).cpu().numpy()
    np.testing.assert_allclose(o1, ref, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(o2, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("P", [7, 14])
def test_roi_align_fpn_schedules_and_edges(P):
    """The product kernel on 3 frames of the 800x1333 pyramid: any RoI schedule
    (none, spatially sorted, XCD-dealt, frame-windowed) gives bit-identical
    output, including RoIs off the map, degenerate, at the border and very wide
    (167 level px); one frame against the oracle's per-level loop (1e-4)."""
    from vosdetectron_amd import ops
    from bench import fpn_levels_np, synthetic_rois
    C, F = 256, 3
    g = torch.Generator(device=DEV).manual_seed(7)
    sizes = [(200, 336), (100, 168), (50, 84), (25, 42)]
    pyr = [torch.randn((F, h, w, C), generator=g, device=DEV) for h, w in sizes]
    rois = np.concatenate([synthetic_rois(f, 500, batch_idx=f) for f in range(F)])
    rois[:6, 1:5] = [[-30, -20, 40, 30], [1300, 780, 1400, 900], [0, 0, 0.5, 0.5],
                     [1320, 790, 1332.9, 799.9], [0, 400, 1332, 420],  # 167 px wide at P3
                     [-200, 100, 1500, 140]]
    lv = fpn_levels_np(rois) - 2
    rt, lt = torch.from_numpy(rois).to(DEV), torch.from_numpy(lv).to(DEV)
    scales = [1. / 4, 1. / 8, 1. / 16, 1. / 32]
    ref = ops.roi_align_fpn(pyr, scales, rt, lt, P, 2, out_layout="nhwc").cpu().numpy()
    for order in (ops.xcd_roi_order(rt, lt, n_xcd=1), ops.xcd_roi_order(rt, lt),
                  ops.xcd_roi_order(rt, lt, window=500)):
        got = ops.roi_align_fpn(pyr, scales, rt, lt, P, 2, roi_order=order,
                                out_layout="nhwc").cpu().numpy()
        assert np.array_equal(got, ref)
    # variant 8 (global loads), variants 11 / 13 (the pipelined sweep) and candidate kernels
    # (VOSDET_TEST_RA_VARIANTS="..."): bit-identical to variant 10 (buffer loads)
    import os
    for variant in ["8", "11", "13"] + os.environ.get("VOSDET_TEST_RA_VARIANTS", "").split():
        os.environ["VOSDET_ROIALIGN_VARIANT"] = variant
        try:
            got = ops.roi_align_fpn(pyr, scales, rt, lt, P, 2, out_layout="nhwc").cpu().numpy()
        finally:
            del os.environ["VOSDET_ROIALIGN_VARIANT"]
        assert np.array_equal(got, ref), variant
    # the product kernel's general form (runtime row segments / workgroup parts, the
    # C > 256 path) vs its specialised default launch: bit-identical
    for env in ({"VOSDET_RA_GENERAL": "1"}, {"VOSDET_RA_SEGS": "2"},
                {"VOSDET_RA_SEGS": "4", "VOSDET_RA_PARTS": "2"}):
        os.environ.update(env)
        try:
            got = ops.roi_align_fpn(pyr, scales, rt, lt, P, 2, roi_order=ops.xcd_roi_order(rt, lt),
                                    out_layout="nhwc").cpu().numpy()
        finally:
            for k in env:
                del os.environ[k]
        assert np.array_equal(got, ref), env
    sel = rois[:, 0] == 0
    r1 = rois[sel].copy()
    d = orc.distribute(r1)
    feats = [p[0:1].permute(0, 3, 1, 2).cpu().numpy() for p in pyr]
    oref = orc.roi_feature_transform(feats[::-1], d, "rois", P, scales[::-1], 2)
    np.testing.assert_allclose(ref[sel].transpose(0, 3, 1, 2), oref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("P", [7, 14])
def test_roi_align_rows_bit_exact(P):
    """The reference-order row kernel (variant 3) computes every output with the
    reference's arithmetic: bit-identical to the oracle's per-level loop and the
    same for any RoI schedule, on 3 frames of the 800x1333 pyramid incl. RoIs off
    the map, degenerate, at the border, tall and wide."""
    import os
    from vosdetectron_amd import ops
    from bench import fpn_levels_np, synthetic_rois
    C, F = 256, 3
    g = torch.Generator(device=DEV).manual_seed(11)
    sizes = [(200, 336), (100, 168), (50, 84), (25, 42)]
    pyr = [torch.randn((F, h, w, C), generator=g, device=DEV) for h, w in sizes]
    rois = np.concatenate([synthetic_rois(f + 5, 400, batch_idx=f) for f in range(F)])
    rois[:8, 1:5] = [[-30, -20, 40, 30], [1300, 780, 1400, 900], [0, 0, 0.5, 0.5],
                     [1320, 790, 1332.9, 799.9], [0, 400, 1332, 420],  # 167 px wide at P3: direct
                     [-200, 100, 1500, 140], [10, 10, 450, 890],  # tall: several bands
                     [600, -50, 620, 1000]]
    lv = fpn_levels_np(rois) - 2
    rt, lt = torch.from_numpy(rois).to(DEV), torch.from_numpy(lv).to(DEV)
    scales = [1. / 4, 1. / 8, 1. / 16, 1. / 32]

    def run(variant, order=None):
        os.environ["VOSDET_ROIALIGN_VARIANT"] = variant
        try:
            return ops.roi_align_fpn(pyr, scales, rt, lt, P, 2, roi_order=order,
                                     out_layout="nhwc").cpu().numpy()
        finally:
            del os.environ["VOSDET_ROIALIGN_VARIANT"]
    ref = run("3")
    for order in (None, ops.xcd_roi_order(rt, lt), ops.xcd_roi_order(rt, lt, n_xcd=1),
                  ops.xcd_roi_order(rt, lt, window=400)):
        got = run("3", order)
        assert np.array_equal(got, ref)
    sel = rois[:, 0] == 0
    d = orc.distribute(rois[sel].copy())
    feats = [p[0:1].permute(0, 3, 1, 2).cpu().numpy() for p in pyr]
    oref = orc.roi_feature_transform(feats[::-1], d, "rois", P, scales[::-1], 2)
    assert np.array_equal(ref[sel].transpose(0, 3, 1, 2), oref)


@pytest.mark.parametrize("variant", ["30"])
@pytest.mark.parametrize("P", [7, 14])
def test_roi_align_tiled_bit_exact(P, variant):
    """The tile-binned LDS-staged kernel (variant 30, roi_align_tile.hip) computes
    every output with the reference's per-sample arithmetic: bit-identical to the
    reference-order row kernel (variant 3) and to the oracle's per-level loop, on
    3 frames of the 800x1333 pyramid incl. RoIs off the map (zero bins), degenerate,
    at the border, wider than a tile window (direct bins), a dense pile of RoIs on
    one tile (chunked items) and out-of-range level / batch indices (zeros)."""
    import os
    from vosdetectron_amd import ops
    from bench import fpn_levels_np, synthetic_rois
    C, F = 256, 3
    g = torch.Generator(device=DEV).manual_seed(13)
    sizes = [(200, 336), (100, 168), (50, 84), (25, 42)]
    pyr = [torch.randn((F, h, w, C), generator=g, device=DEV) for h, w in sizes]
    rois = np.concatenate([synthetic_rois(f + 9, 400, batch_idx=f) for f in range(F)])
    rois[:8, 1:5] = [[-30, -20, 40, 30], [1300, 780, 1400, 900], [0, 0, 0.5, 0.5],
                     [1320, 790, 1332.9, 799.9], [0, 400, 1332, 420],  # 167 px wide at P3
                     [-200, 100, 1500, 140], [0, 0, 1332, 799],  # whole frame at P5: direct
                     [600, -50, 620, 1000]]
    rng = np.random.default_rng(5)
    xy = rng.uniform(500, 560, (60, 2))  # 60 small boxes on one P2 tile: > 128 bins
    rois[8:68, 1:5] = np.hstack([xy, xy + rng.uniform(4, 30, (60, 2))])
    lv = fpn_levels_np(rois) - 2
    lv[68], lv[69] = 7, -1  # malformed level indices pool to zero
    rois[70, 0] = 5  # batch index past the pyramid
    rt, lt = torch.from_numpy(rois).to(DEV), torch.from_numpy(lv).to(DEV)
    scales = [1. / 4, 1. / 8, 1. / 16, 1. / 32]

    def run(variant, **kw):
        os.environ["VOSDET_ROIALIGN_VARIANT"] = variant
        try:
            return ops.roi_align_fpn(pyr, scales, rt, lt, P, 2, out_layout="nhwc",
                                     **kw).cpu().numpy()
        finally:
            del os.environ["VOSDET_ROIALIGN_VARIANT"]
    ref = run("3")
    assert not ref[68:71].any()
    got = run(variant)
    assert np.array_equal(got, ref)
    os.environ["VOSDET_RA_CHUNK"] = "16"  # every tile split into many items
    try:
        assert np.array_equal(run(variant), ref)
    finally:
        del os.environ["VOSDET_RA_CHUNK"]
    sel = (rois[:, 0] == 0) & (np.arange(len(rois)) < 68)
    d = orc.distribute(rois[sel].copy())
    feats = [p[0:1].permute(0, 3, 1, 2).cpu().numpy() for p in pyr]
    oref = orc.roi_feature_transform(feats[::-1], d, "rois", P, scales[::-1], 2)
    assert np.array_equal(got[sel].transpose(0, 3, 1, 2), oref)


def test_roi_align_tiled_shapes():
    """Variant 30 on other shapes: C = 64 / 96 (fewer slices), one level, B = 1,
    a single RoI, and a shape it does not serve (C % 32 != 0 -> the register-gather
    kernel), all against the reference-order kernel."""
    import os
    from vosdetectron_amd import ops
    rng = np.random.default_rng(21)
    for C, sizes, n in ((64, [(50, 84), (25, 42)], 90), (96, [(37, 61)], 1),
                        (256, [(13, 21)], 40), (40, [(25, 42), (13, 21)], 30)):
        L = len(sizes)
        feats = _pyramid(rng, 1, C, sizes)
        nhwc = [torch.from_numpy(x).to(DEV).permute(0, 2, 3, 1).contiguous() for x in feats]
        scales = [1. / 2 ** (k + 2) for k in range(L)]
        rois = make_rois(rng, n, 336, 200, batch=1)
        lv = (orc.map_rois_to_fpn_levels(rois[:, 1:5], 2, 1 + L).astype(np.int32) - 2)
        args = (nhwc, scales, torch.from_numpy(rois).to(DEV), torch.from_numpy(lv).to(DEV), 7, 2)
        outs = {}
        for v in ("3", "30"):
            os.environ["VOSDET_ROIALIGN_VARIANT"] = v
            try:
                outs[v] = ops.roi_align_fpn(*args, out_layout="nhwc").cpu().numpy()
            finally:
                del os.environ["VOSDET_ROIALIGN_VARIANT"]
        for v in ("30",):
            if C % 32 == 0:
                assert np.array_equal(outs[v], outs["3"]), (C, v)
            else:
                np.testing.assert_allclose(outs[v], outs["3"], rtol=1e-4, atol=1e-4)
