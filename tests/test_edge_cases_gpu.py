"""Edge cases on the GPU: empty inputs, everything
filtered, RoIs off the map, all-tied scores, and the size limits of each entry
point (largest accepted, first rejected) -- each against the oracle."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_roi_align_empty_and_off_map():
    from vosdetectron_amd import ops
    f = torch.randn(1, 16, 20, 30, device=DEV)
    z = torch.zeros((0, 5), device=DEV)
    assert ops.roi_align_forward(f, z, 7, 7, 0.25, 2).shape == (0, 16, 7, 7)
    lv = torch.zeros((0,), dtype=torch.int32, device=DEV)
    nhwc = f.permute(0, 2, 3, 1).contiguous()
    assert ops.roi_align_fpn([nhwc], [0.25], z, lv, 7, 2, out_layout="nhwc").shape == (0, 7, 7, 16)
    # RoIs wholly outside the map (samples y < -1 or > H) pool to exactly zero
    rois = np.array([[0, -500, -500, -300, -300], [0, 400, 300, 900, 700],
                     [0, -8, -8, -4.1, -4.1]], np.float32)
    ref = orc.roi_align(f.cpu().numpy(), rois, 7, 7, 0.25, 2)
    out = ops.roi_align_forward(f, torch.from_numpy(rois).to(DEV), 7, 7, 0.25, 2)
    assert np.array_equal(out.cpu().numpy(), ref)
    lv = torch.zeros((3,), dtype=torch.int32, device=DEV)
    o2 = ops.roi_align_fpn([nhwc], [0.25], torch.from_numpy(rois).to(DEV), lv, 7, 2)
    np.testing.assert_allclose(o2.cpu().numpy(), ref, atol=1e-6)


def test_nms_size_limits():
    from vosdetectron_amd import ops
    from vosdetectron_amd._lib import VosdetError
    rng = np.random.default_rng(7)
    n = 8192  # kNmsMaxN
    xy = rng.uniform(0, 2000, (n, 2))
    d = np.hstack([xy, xy + rng.uniform(1, 80, (n, 2)),
                   np.round(rng.uniform(0, 1, (n, 1)) * 64) / 64]).astype(np.float32)
    assert np.array_equal(ops.nms(torch.from_numpy(d).to(DEV), 0.5).cpu().numpy(),
                          orc.nms(d, 0.5))
    with pytest.raises(VosdetError):
        ops.nms(torch.zeros((n + 1, 5), device=DEV), 0.5)


def test_proposals_everything_filtered_and_all_tied():
    from vosdetectron_amd import ops
    rng = np.random.default_rng(3)
    H, W = 25, 42
    an = orc.fpn_level_anchors(4)
    info = np.array([[800, 1344, 1.0], [800, 1344, 1.0]], np.float32)
    p = np.full((2, 3, H, W), 0.5, np.float32)  # every score tied
    d = rng.normal(0, 0.3, (2, 12, H, W)).astype(np.float32)
    d[1] = -20.0  # image 1: every box collapses to width/height 1 -> min_size drops all
    min_size = 2
    rois, pr, cnt = [t.cpu().numpy() for t in ops.generate_proposals(
        [torch.from_numpy(p).to(DEV)], [torch.from_numpy(d).to(DEV)],
        [torch.from_numpy(an).to(DEV)], [1. / 16], torch.from_numpy(info).to(DEV), 1000, 1000,
        0.7, min_size)]
    ref_r, ref_p = orc.generate_proposals(an, 1. / 16, p, d, info, 1000, 1000, 0.7, min_size)
    for img in range(2):
        sel = ref_r[:, 0] == img
        assert cnt[img, 0] == sel.sum()
        assert np.array_equal(rois[img, 0, :cnt[img, 0]], ref_r[sel])
    assert cnt[1, 0] == 0
    # collect/distribute with an image that has no proposals at all
    cr, clv, ccnt = ops.collect_distribute(*[torch.from_numpy(x).to(DEV)
                                             for x in (rois, pr, cnt)], 1000, 2, 5)
    assert int(ccnt[1].item()) == 0 and int(ccnt[0].item()) == cnt[0, 0]


def test_box_detections_nothing_above_threshold():
    from vosdetectron_amd import ops
    N, R, K = 2, 50, 81
    rois = torch.zeros((N, R, 5), device=DEV)
    rois[:, :, 3:] = 40.
    cls = torch.full((N, R, K), 1. / K, device=DEV)  # 0.0123 < SCORE_THRESH 0.05
    pred = torch.zeros((N, R, 4 * K), device=DEV)
    cnt = torch.tensor([R, 0], dtype=torch.int32, device=DEV)
    dets, dcls, dcnt = ops.box_detections(rois, cls, pred, cnt, torch.ones(N, device=DEV),
                                          torch.tensor([[100, 100]] * N, dtype=torch.int32,
                                                       device=DEV))
    assert dcnt.cpu().tolist() == [0, 0]


def test_segm_empty_and_degenerate():
    from vosdetectron_amd import ops, segm
    planes = ops.paste_masks(torch.zeros((0, 28, 28), device=DEV), torch.zeros((0, 5), device=DEV),
                             40, 60)
    assert planes.shape == (0, 40, 60) and segm.encode_planes(planes) == []
    m = np.random.default_rng(1).uniform(0, 1, (3, 28, 28)).astype(np.float32)
    b = np.array([[5, 5, 5, 5, 1], [0, 0, 59, 39, 1], [58.9, 38.9, 59, 39, 1]], np.float32)
    got = ops.paste_masks(torch.from_numpy(m).to(DEV), torch.from_numpy(b).to(DEV), 40, 60)
    assert np.array_equal(got.cpu().numpy(), orc.paste_masks(m, b, 40, 60))
    assert segm.encode_planes(got) == [orc.rle_encode(x)[0] for x in orc.paste_masks(m, b, 40, 60)]


def test_pipeline_with_no_detections():
    """A frame whose every class score is under TEST.SCORE_THRESH: zero counts, an
    empty mask batch, and empty segm results (the reference's empty cls_boxes)."""
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.engine import FramePipeline, frame_segms
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
    cfg.TEST.SCORE_THRESH = 1.01
    model, _ = build_model(cfg, device=DEV, channels_last=True)
    pipe = FramePipeline(model, cfg, batch=2, device=DEV, channels_last=True)
    fr = np.random.RandomState(2).randint(0, 256, (2, 800, 1333, 3), np.uint8)
    out = pipe.run(torch.from_numpy(fr).to(DEV))
    assert out["counts_host"] == [0, 0] and out["masks"].shape == (0, 28, 28)
    assert all(not any(s) for s in frame_segms(pipe, out))


def test_proposals_size_limits():
    """pre_nms_topN up to 8192 (the large-candidate kernel's limit, incl. take-all at
    exactly 8192 anchors) matches the oracle; 8193 is rejected."""
    from vosdetectron_amd import ops
    from vosdetectron_amd._lib import VosdetError
    rng = np.random.default_rng(11)
    an = orc.generate_anchors(16, (32, 64, 128, 256, 512), (0.5, 1, 2))
    for (H, W, pre) in [(16, 34, 0), (40, 60, 8192)]:  # 16*34*15 = 8160 take-all; pre cap
        p = rng.uniform(0, 1, (1, 15, H, W)).astype(np.float32)
        d = rng.normal(0, 0.3, (1, 60, H, W)).astype(np.float32)
        info = np.array([[H * 16, W * 16, 1.0]], np.float32)
        rois, _, cnt = [t.cpu().numpy() for t in ops.generate_proposals(
            [torch.from_numpy(p).to(DEV)], [torch.from_numpy(d).to(DEV)],
            [torch.from_numpy(an).to(DEV)], [1. / 16], torch.from_numpy(info).to(DEV), pre,
            1000, 0.7, 0)]
        ref, _ = orc.generate_proposals(an, 1. / 16, p, d, info, pre, 1000, 0.7, 0)
        assert cnt[0, 0] == len(ref) and np.array_equal(rois[0, 0, :cnt[0, 0]], ref)
    with pytest.raises(VosdetError):
        z = torch.zeros((1, 15, 40, 60), device=DEV)
        ops.generate_proposals([z], [torch.zeros((1, 60, 40, 60), device=DEV)],
                               [torch.from_numpy(an).to(DEV)], [1. / 16],
                               torch.tensor([[640., 960., 1.]], device=DEV), 8193, 1000, 0.7, 0)


def test_proposals_unbracketable_topk_fails_loudly(monkeypatch):
    """a score map on which the one-workgroup top-k threshold search
    (VOSDET_RPN_PRESEL=0) cannot bracket pre_nms_topN within its candidate
    capacity (the sampled anchors score 0 but four, every other anchor 0.5: 197k
    candidates tie between two adjacent sample keys) must not drop the level
    silently -- its count is -1, which collect_distribute and box_detections pass
    on and the engine raises on.  The default multi-workgroup radix select
    resolves the same map exactly (its index digits split the tie): checked
    against the oracle."""
    from vosdetectron_amd import ops
    from vosdetectron_amd._lib import VosdetError
    monkeypatch.setenv("VOSDET_RPN_PRESEL", "0")
    H, W, A = 200, 336, 3
    n_all, S = H * W * A, 2048  # kSampleMax
    flat = np.full(n_all, 0.5, np.float32)  # element order e = (h*W + w)*A + a
    samp = (np.arange(S, dtype=np.int64) * n_all) // S
    flat[samp] = 0.0
    flat[samp[:4]] = 1.0
    p = flat.reshape(H * W, A).T.reshape(1, A, H, W).copy()
    d = np.zeros((1, 4 * A, H, W), np.float32)
    an = orc.fpn_level_anchors(2)
    info = torch.tensor([[800., 1344., 1.]], device=DEV)
    rois, pr, cnt = ops.generate_proposals(
        [torch.from_numpy(p).to(DEV)], [torch.from_numpy(d).to(DEV)],
        [torch.from_numpy(an).to(DEV)], [1. / 4], info, 1000, 1000, 0.7, 0)
    assert cnt.cpu().tolist() == [[-1]]
    cr, clv, ccnt = ops.collect_distribute(rois, pr, cnt, 1000, 2, 5)
    assert ccnt.cpu().tolist() == [-1]
    K = 81
    dets, dcls, dcnt = ops.box_detections(
        cr, torch.full((1, 1000, K), 0.5, device=DEV), torch.zeros((1, 1000, 4 * K), device=DEV),
        ccnt, torch.ones(1, device=DEV), torch.tensor([[800, 1333]], dtype=torch.int32,
                                                      device=DEV))
    assert dcnt.cpu().tolist() == [-1]
    with pytest.raises(VosdetError):
        ops.raise_on_failed_counts(dcnt.cpu().tolist())
    monkeypatch.setenv("VOSDET_RPN_PRESEL", "1")
    rois, pr, cnt = ops.generate_proposals(
        [torch.from_numpy(p).to(DEV)], [torch.from_numpy(d).to(DEV)],
        [torch.from_numpy(an).to(DEV)], [1. / 4], info, 1000, 1000, 0.7, 0)
    ref_r, ref_p = orc.generate_proposals(an, 1. / 4, p, d, info.cpu().numpy(), 1000, 1000,
                                          0.7, 0)
    k = int(cnt[0, 0])
    assert k == len(ref_r) and k > 0
    assert np.array_equal(rois[0, 0, :k].cpu().numpy(), ref_r)
    assert np.array_equal(pr[0, 0, :k].cpu().numpy(), ref_p[:, 0])


def test_roi_align_fpn_malformed_indices_pool_to_zero():
    """out-of-range level / batch indices from a caller of the public C
    ABI pool to exactly zero (no out-of-bounds read); well-formed RoIs of the
    same launch are unaffected; mismatched level shapes are rejected on the host."""
    from vosdetectron_amd import ops
    C = 256
    lv0 = torch.randn(2, 20, 30, C, device=DEV)
    lv1 = torch.randn(2, 10, 15, C, device=DEV)
    rois = torch.tensor([[0, 4, 4, 60, 50], [5, 4, 4, 60, 50], [-1, 4, 4, 60, 50],
                         [1, 10, 8, 70, 60], [0, 4, 4, 60, 50]], dtype=torch.float32,
                        device=DEV)
    lvl = torch.tensor([0, 0, 1, 1, 7], dtype=torch.int32, device=DEV)
    for variant in ("10", "8", "3"):
        import os
        os.environ["VOSDET_ROIALIGN_VARIANT"] = variant
        try:
            out = ops.roi_align_fpn([lv0, lv1], [0.25, 0.125], rois, lvl, 7, 2, out_layout="nhwc")
        finally:
            del os.environ["VOSDET_ROIALIGN_VARIANT"]
        o = out.cpu().numpy()
        assert not o[1].any() and not o[2].any() and not o[4].any()
        good = ops.roi_align_fpn([lv0, lv1], [0.25, 0.125], rois[[0, 3]], lvl[[0, 3]], 7, 2,
                                 out_layout="nhwc").cpu().numpy()
        np.testing.assert_allclose(o[[0, 3]], good, rtol=1e-5, atol=1e-6)
    f = torch.randn(2, 8, 10, 12, device=DEV)
    got = ops.roi_align_forward(f, torch.tensor([[3., 0, 0, 20, 20]], device=DEV), 7, 7, 0.5, 2)
    assert not got.cpu().numpy().any()
    with pytest.raises(ValueError):
        ops.roi_align_fpn([lv0, torch.randn(1, 10, 15, C, device=DEV)], [0.25, 0.125], rois,
                          lvl, 7, 2)
