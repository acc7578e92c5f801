"""GPU parity of NMS, FPN level map, RPN proposals, collect/distribute and the
box-head post-processing against the oracle and the reference-generated golden
fixtures.  Index selection must be bit-exact."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rand_dets(rng, n, ties=False, span=800):
    xy = rng.uniform(0, span, (n, 2))
    wh = rng.uniform(1, 120, (n, 2))
    s = rng.uniform(0, 1, n)
    if ties:
        s = np.round(s * 8) / 8  # heavy ties
    d = np.hstack([xy, xy + wh, s[:, None]]).astype(np.float32)
    return d


@pytest.mark.parametrize("n,thr,ties", [(1, 0.5, False), (7, 0.5, True), (300, 0.7, False),
                                        (1000, 0.7, True), (2500, 0.5, False), (64, 0.3, True),
                                        (65, 0.3, False), (5000, 0.6, True)])
def test_nms_bit_exact(n, thr, ties):
    from vosdetectron_amd import ops
    rng = np.random.default_rng(n + int(thr * 10))
    d = rand_dets(rng, n, ties)
    ref = orc.nms(d, thr)
    out = ops.nms(torch.from_numpy(d).to(DEV), thr).cpu().numpy()
    assert np.array_equal(out, ref)


def test_nms_edge_cases():
    from vosdetectron_amd import ops
    same = np.array([[0, 0, 10, 10, 0.9]] * 5, np.float32)
    assert ops.nms(torch.from_numpy(same).to(DEV), 0.5).cpu().tolist() == [4]
    assert ops.nms(torch.zeros((0, 5), device=DEV), 0.5).numel() == 0
    # threshold equality suppresses (>=)
    d = np.array([[0, 0, 10, 10, 0.9], [0, 0, 10, 21, 0.8]], np.float32)
    assert ops.nms(torch.from_numpy(d).to(DEV), 0.5).cpu().tolist() == [0]


def test_nms_vs_executed_reference(golden):
    """vd_nms (ops.nms) and the ndarray drop-in boxes.nms against the EXECUTED
    reference cython_nms.nms (tests/golden/nms.npz, tools/ref_cython_nms.py):
    tie-free sets at N in {1, 64, 65, 1000, 4381, 5000} x {0.3, 0.5, 0.7},
    exact-threshold IoU pairs, and tie sets given the reference's processing
    order.  Bit-exact index selection (north_star)."""
    from tests.test_oracle_golden import _nms_cases
    from vosdetectron_amd import boxes, ops
    g = golden("nms")
    n_cases = 0
    for kind, d, thr, keep in _nms_cases(g):
        out = ops.nms(torch.from_numpy(d).to(DEV), thr).cpu().numpy()
        assert np.array_equal(out, keep), (kind, len(d), thr)
        assert np.array_equal(np.asarray(boxes.nms(d, thr), np.int64), keep), (kind, len(d))
        n_cases += 1
    assert n_cases == int(g["count"])


def test_fpn_levels_golden(golden):
    from vosdetectron_amd import ops
    g = golden("fpn_levels")
    rois = np.hstack([np.zeros((len(g["boxes"]), 1), np.float32), g["boxes"]])
    out = ops.map_rois_to_fpn_levels(torch.from_numpy(rois).to(DEV), 2, 5).cpu().numpy()
    assert np.array_equal(out, g["lvls"].astype(np.int32))


def _anchors(lvl):
    return torch.from_numpy(orc.fpn_level_anchors(lvl)).to(DEV)


@pytest.mark.parametrize("split", ["1", "0"])
def test_generate_proposals_golden(golden, split, monkeypatch):
    """Reference-executed GenerateProposalsOp per level (tests/golden/proposals.npz),
    through the split NMS (default) and the single-kernel small variant
    (VOSDET_RPN_SPLIT=0)."""
    from vosdetectron_amd import ops
    monkeypatch.setenv("VOSDET_RPN_SPLIT", split)
    g = golden("proposals")
    lv = list(range(2, 7))
    probs = [torch.from_numpy(g["probs_fpn%d" % l]).to(DEV) for l in lv]
    deltas = [torch.from_numpy(g["deltas_fpn%d" % l]).to(DEV) for l in lv]
    rois, pr, cnt = ops.generate_proposals(probs, deltas, [_anchors(l) for l in lv],
                                           [1. / 2 ** l for l in lv],
                                           torch.from_numpy(g["im_info"]).to(DEV), 1000, 1000,
                                           0.7, 0)
    rois, pr, cnt = rois.cpu().numpy(), pr.cpu().numpy(), cnt.cpu().numpy()
    for i, l in enumerate(lv):
        ref_r, ref_p = g["rois_fpn%d" % l], g["roi_probs_fpn%d" % l]
        k = cnt[0, i]
        assert k == len(ref_r), (l, k, len(ref_r))
        assert np.array_equal(rois[0, i, :k], ref_r), l
        assert np.array_equal(pr[0, i, :k], ref_p[:, 0]), l
    # collect + distribute against the reference's collect/distribute outputs
    c = golden("collect_distribute")
    cr, clv, ccnt = ops.collect_distribute(torch.from_numpy(rois).to(DEV),
                                           torch.from_numpy(pr).to(DEV),
                                           torch.from_numpy(cnt).to(DEV), 1000)
    cr, clv = cr.cpu().numpy()[0], clv.cpu().numpy()[0]
    assert int(ccnt.item()) == 1000
    assert np.array_equal(cr, c["collected"])
    for k in range(4):
        sel = cr[clv == k]
        assert np.array_equal(sel, c["rois_fpn%d" % (k + 2)])


def test_generate_proposals_c4_golden(golden):
    """Single-scale C4 RPN (15 anchors, pre 6000 -> the large-candidate kernel)
    against the reference-executed GenerateProposalsOp (proposals_c4.npz)."""
    from vosdetectron_amd import ops
    g = golden("proposals_c4")
    rois, pr, cnt = ops.generate_proposals(
        [torch.from_numpy(g["probs"]).to(DEV)], [torch.from_numpy(g["deltas"]).to(DEV)],
        [torch.from_numpy(g["anchors"]).to(DEV)], [1. / 16],
        torch.from_numpy(g["im_info"]).to(DEV), 6000, 1000, 0.7, 0)
    k = int(cnt[0, 0].item())
    assert k == len(g["rois"])
    assert np.array_equal(rois[0, 0, :k].cpu().numpy(), g["rois"])
    assert np.array_equal(pr[0, 0, :k].cpu().numpy(), g["roi_probs"][:, 0])


@pytest.mark.parametrize("seed,pre,A,H,W", [(0, 6000, 15, 50, 84), (1, 6000, 15, 50, 84),
                                           (2, 8192, 15, 38, 60), (3, 3000, 9, 25, 42),
                                           (4, 0, 15, 20, 25)])
def test_generate_proposals_large_vs_oracle(seed, pre, A, H, W):
    """Large-candidate variant with ties, two images (seed 1/4: heavy ties; pre=0 and
    n_all = 7500 <= 8192: take-all)."""
    from vosdetectron_amd import ops
    rng = np.random.default_rng(100 + seed)
    N = 2
    an = orc.generate_anchors(16, (32, 64, 128, 256, 512)[:A // 3], (0.5, 1, 2))
    p = rng.uniform(0, 1, (N, A, H, W)).astype(np.float32)
    if seed in (1, 4):
        p = (np.round(p * 256) / 256).astype(np.float32)
    d = rng.normal(0, 0.5, (N, 4 * A, H, W)).astype(np.float32)
    info = np.array([[H * 16, W * 16, 1.0]] * N, np.float32)
    rois, pr, cnt = [t.cpu().numpy() for t in ops.generate_proposals(
        [torch.from_numpy(p).to(DEV)], [torch.from_numpy(d).to(DEV)],
        [torch.from_numpy(an).to(DEV)], [1. / 16], torch.from_numpy(info).to(DEV), pre, 1000,
        0.7, 0)]
    ref_r, ref_p = orc.generate_proposals(an, 1. / 16, p, d, info, pre, 1000, 0.7, 0)
    for img in range(N):
        sel = ref_r[:, 0] == img
        k = cnt[img, 0]
        assert k == sel.sum(), img
        assert np.array_equal(rois[img, 0, :k], ref_r[sel]), img
        assert np.array_equal(pr[img, 0, :k], ref_p[sel, 0]), img


@pytest.mark.parametrize("presel", ["1", "0"])
@pytest.mark.parametrize("seed,ties", [(0, False), (1, True), (2, True)])
def test_generate_proposals_vs_oracle_batched(seed, ties, presel, monkeypatch):
    """Two images, full-size P2..P6 of an 800x1344 blob, tied scores; through the
    multi-workgroup radix select (default) and round 4's one-workgroup select
    (VOSDET_RPN_PRESEL=0)."""
    from vosdetectron_amd import ops
    monkeypatch.setenv("VOSDET_RPN_PRESEL", presel)
    rng = np.random.default_rng(seed)
    N = 2
    shapes = {2: (200, 336), 3: (100, 168), 4: (50, 84), 5: (25, 42), 6: (13, 21)}
    im_info = np.array([[800, 1344, 1.0], [800, 1344, 1.0]], np.float32)
    probs, deltas = [], []
    for l, (H, W) in shapes.items():
        p = rng.uniform(0, 1, (N, 3, H, W)).astype(np.float32)
        if ties:
            p = (np.round(p * 512) / 512).astype(np.float32)
        probs.append(p)
        deltas.append(rng.normal(0, 0.5, (N, 12, H, W)).astype(np.float32))
    lv = list(shapes)
    out = ops.generate_proposals([torch.from_numpy(p).to(DEV) for p in probs],
                                 [torch.from_numpy(d).to(DEV) for d in deltas],
                                 [_anchors(l) for l in lv], [1. / 2 ** l for l in lv],
                                 torch.from_numpy(im_info).to(DEV), 1000, 1000, 0.7, 0)
    rois, pr, cnt = [t.cpu().numpy() for t in out]
    for i, l in enumerate(lv):
        ref_r, ref_p = orc.generate_proposals(orc.fpn_level_anchors(l), 1. / 2 ** l, probs[i],
                                              deltas[i], im_info)
        for img in range(N):
            sel = ref_r[:, 0] == img
            k = cnt[img, i]
            assert k == sel.sum(), (l, img)
            assert np.array_equal(rois[img, i, :k], ref_r[sel]), (l, img)
            assert np.array_equal(pr[img, i, :k], ref_p[sel, 0]), (l, img)
    # per-image collect/distribute
    cr, clv, ccnt = [t.cpu().numpy() for t in ops.collect_distribute(
        *[torch.from_numpy(x).to(DEV) for x in (rois, pr, cnt)], 1000)]
    for img in range(N):
        rl = [rois[img, i, :cnt[img, i]] for i in range(5)]
        pl = [pr[img, i, :cnt[img, i], None] for i in range(5)]
        col = orc.collect(rl, pl, 1000)
        assert np.array_equal(cr[img, :ccnt[img]], col)
        lvls = orc.map_rois_to_fpn_levels(col[:, 1:5], 2, 5).astype(np.int32) - 2
        assert np.array_equal(clv[img, :ccnt[img]], lvls)


@pytest.mark.parametrize("case", ["all_equal", "two_values", "just_above_pre", "negative",
                                  "pre_eq_cap"])
def test_radix_select_edge_cases(case):
    """The multi-workgroup radix select where its passes run deepest: every score
    equal (the boundary is fixed by the index digits alone, all six passes),
    two distinct values, n_all = pre + 1, negative and zero scores (sign-flipped
    float keys), and pre = 2048 on a level of 3 x 200 x 336 (candidate capacity
    = 2 x pre).  Bit-exact vs the oracle (lower index wins ties)."""
    from vosdetectron_amd import ops
    rng = np.random.default_rng(7)
    A, H, W, pre = 3, 200, 336, 1000
    if case == "just_above_pre":
        H, W = 7, 48  # 1008 anchors, pre 1000 -> 1007 would be take-all
        pre = 1000
    p = rng.uniform(0, 1, (1, A, H, W)).astype(np.float32)
    if case == "all_equal":
        p[:] = np.float32(0.5)
    elif case == "two_values":
        p = np.where(p < 0.5, np.float32(0.25), np.float32(0.75)).astype(np.float32)
    elif case == "negative":
        p = -np.abs(rng.normal(0, 1, (1, A, H, W))).astype(np.float32)
        p[0, 0, :5] = 0.0
        p[0, 1, :5] = -0.0
    elif case == "pre_eq_cap":
        pre = 2048
    d = rng.normal(0, 0.5, (1, 4 * A, H, W)).astype(np.float32)
    info = np.array([[H * 4, W * 4, 1.0]], np.float32)
    an = orc.fpn_level_anchors(2)
    rois, pr, cnt = [t.cpu().numpy() for t in ops.generate_proposals(
        [torch.from_numpy(p).to(DEV)], [torch.from_numpy(d).to(DEV)],
        [torch.from_numpy(an).to(DEV)], [1. / 4], torch.from_numpy(info).to(DEV), pre, 1000,
        0.7, 0)]
    ref_r, ref_p = orc.generate_proposals(an, 1. / 4, p, d, info, pre, 1000, 0.7, 0)
    k = cnt[0, 0]
    assert k == len(ref_r), (k, len(ref_r))
    assert np.array_equal(rois[0, 0, :k], ref_r)
    assert np.array_equal(pr[0, 0, :k], ref_p[:, 0])


@pytest.mark.parametrize("seed", [0, 1])
def test_box_detections_vs_oracle(seed):
    """Decode (weights 10,10,5,5) + clip to the original image + per-class NMS +
    top-100 (core/test.py:157-184, 733-797) vs the oracle."""
    from vosdetectron_amd import ops
    rng = np.random.default_rng(seed)
    N, R, K = 2, 1000, 81
    im_h, im_w = 800, 1333
    rois = np.zeros((N, R, 5), np.float32)
    for i in range(N):
        xy = rng.uniform(0, 1300, (R, 2))
        wh = rng.uniform(4, 300, (R, 2))
        rois[i, :, 0] = i
        rois[i, :, 1:3] = xy
        rois[i, :, 3:5] = np.minimum(xy + wh, [1343, 799])
    logits = rng.normal(0, 2.5, (N, R, K)).astype(np.float32)
    e = np.exp(logits - logits.max(-1, keepdims=True))
    cls = (e / e.sum(-1, keepdims=True)).astype(np.float32)
    if seed == 1:
        cls = (np.round(cls * 256) / 256).astype(np.float32)  # ties in scores
    pred = rng.normal(0, 1.0, (N, R, 4 * K)).astype(np.float32)
    counts = np.array([R, R - 37], np.int32)
    out = ops.box_detections(*[torch.from_numpy(x).to(DEV) for x in (rois, cls, pred, counts)],
                             torch.tensor([1.0, 1.0], device=DEV),
                             torch.tensor([[im_h, im_w]] * N, dtype=torch.int32, device=DEV),
                             det_cap=8192)
    dets, dcls, dcnt = [t.cpu().numpy() for t in out]
    for i in range(N):
        r = counts[i]
        boxes = rois[i, :r, 1:5] / 1.0
        pb = orc.bbox_transform(boxes, pred[i, :r], (10., 10., 5., 5.))
        pb = orc.clip_tiled_boxes(pb, (im_h, im_w, 3))
        sc, bx, cls_boxes = orc.box_results_with_nms_and_limit(cls[i, :r], pb)
        n = dcnt[i]
        assert n == len(sc)
        assert np.array_equal(dets[i, :n, :4], bx)
        assert np.array_equal(dets[i, :n, 4], sc)
        ref_cls = np.concatenate([[j] * len(cls_boxes[j]) for j in range(1, K)]).astype(np.int32)
        assert np.array_equal(dcls[i, :n], ref_cls)


@pytest.mark.parametrize("seed,cross,pre,dets_per_im", [(0, 0.3, 0, 100), (1, 0., 2, 100),
                                                        (2, 0.5, 1, 100), (3, 0.4, 50, 300),
                                                        (4, 0.7, 3, 400)])
def test_detections_postfilter_vs_oracle(seed, cross, pre, dets_per_im):
    """The fork's post-limit steps (vos_test.py:805-833): cross-class NMS and the
    per-class top-k (NUM_DET_PER_CLASS_PRE, e.g. 50 in
    R-101-FPN_3x_gn_train_online.yaml), on vd_box_detections' outputs; seeds 1, 3
    with tied scores."""
    from vosdetectron_amd import ops
    rng = np.random.default_rng(50 + seed)
    N, R, K = 2, 600, 81
    im_h, im_w = 480, 854
    rois = np.zeros((N, R, 5), np.float32)
    for i in range(N):
        xy = rng.uniform(0, 800, (R, 2))
        wh = rng.uniform(8, 200, (R, 2))
        rois[i, :, 0] = i
        rois[i, :, 1:3] = xy
        rois[i, :, 3:5] = np.minimum(xy + wh, [863, 479])
    logits = rng.normal(0, 2.5, (N, R, K)).astype(np.float32)
    e = np.exp(logits - logits.max(-1, keepdims=True))
    cls = (e / e.sum(-1, keepdims=True)).astype(np.float32)
    if seed in (1, 3):
        cls = (np.round(cls * 64) / 64).astype(np.float32)
    pred = rng.normal(0, 1.0, (N, R, 4 * K)).astype(np.float32)
    counts = np.array([R, R - 11], np.int32)
    out = ops.box_detections(*[torch.from_numpy(x).to(DEV) for x in (rois, cls, pred, counts)],
                             torch.tensor([1.0, 1.0], device=DEV),
                             torch.tensor([[im_h, im_w]] * N, dtype=torch.int32, device=DEV),
                             dets_per_im=dets_per_im, det_cap=512, nms_cross_class=cross,
                             num_det_per_class_pre=pre)
    dets, dcls, dcnt = [t.cpu().numpy() for t in out]
    for i in range(N):
        r = counts[i]
        pb = orc.clip_tiled_boxes(orc.bbox_transform(rois[i, :r, 1:5], pred[i, :r],
                                                     (10., 10., 5., 5.)), (im_h, im_w, 3))
        sc, bx, cls_boxes = orc.box_results_with_nms_and_limit(
            cls[i, :r], pb, dets_per_im=dets_per_im, nms_cross_class=cross,
            num_det_per_class_pre=pre)
        n = dcnt[i]
        assert n == len(sc), (n, len(sc))
        assert np.array_equal(dets[i, :n, :4], bx)
        assert np.array_equal(dets[i, :n, 4], sc)
        ref_cls = np.concatenate([[j] * len(cls_boxes[j]) for j in range(1, K)]).astype(np.int32)
        assert np.array_equal(dcls[i, :n], ref_cls)


def test_detections_postfilter_golden(golden):
    """vd_detections_postfilter on the stock limit's output reproduces the
    reference-executed fork steps (detections_postfilter.npz)."""
    import ctypes
    from vosdetectron_amd._lib import check, lib
    g = golden("detections_postfilter")
    sc, bx, cls_boxes = orc.box_results_with_nms_and_limit(g["scores"], g["boxes"])
    cls = np.concatenate([[j] * len(cls_boxes[j]) for j in range(1, 81)]).astype(np.int32)
    cap = 256
    for tag, cross, pre in (("cross04_pre2", 0.4, 2), ("cross0_pre50", 0., 50),
                            ("cross06_pre0", 0.6, 0), ("cross0_pre0", 0., 0)):
        dets = torch.zeros((1, cap, 5), device=DEV)
        dets[0, :len(sc), :4] = torch.from_numpy(bx).to(DEV)
        dets[0, :len(sc), 4] = torch.from_numpy(sc).to(DEV)
        dcls = torch.zeros((1, cap), dtype=torch.int32, device=DEV)
        dcls[0, :len(sc)] = torch.from_numpy(cls).to(DEV)
        cnt = torch.tensor([len(sc)], dtype=torch.int32, device=DEV)
        check(lib().vd_detections_postfilter(dets.data_ptr(), dcls.data_ptr(), cnt.data_ptr(), 1,
                                             cap, ctypes.c_float(cross), pre,
                                             torch.cuda.current_stream().cuda_stream),
              "vd_detections_postfilter")
        n = int(cnt.item())
        assert n == len(g[tag + "_dets"]), tag
        assert np.array_equal(dets[0, :n].cpu().numpy(), g[tag + "_dets"]), tag
        assert np.array_equal(dcls[0, :n].cpu().numpy(), g[tag + "_cls"]), tag


def test_proposals_tie_fixture(golden):
    """The reference-executed tie study (tools/tie_study.py): on tie-bearing
    scores the HIP kernel reproduces the package's stable reading bit for bit,
    and the reference's output rows as a set wherever the reference's unstable
    numpy order left the set unchanged (see tests/golden/proposals_ties.json)."""
    import json
    import os
    from tests.conftest import GOLDEN
    from vosdetectron_amd import ops
    info = json.load(open(os.path.join(GOLDEN, "proposals_ties.json")))
    g = golden("proposals_ties")
    for c in info["cases"]:
        tag = c["case"]
        if tag + "_probs" not in g.files:
            continue
        lvl = int(tag.split("fpn")[1])
        an = orc.fpn_level_anchors(lvl)
        p, d = g[tag + "_probs"], g[tag + "_deltas"]
        rois, _, cnt = ops.generate_proposals(
            [torch.from_numpy(p).to(DEV)], [torch.from_numpy(d).to(DEV)],
            [torch.from_numpy(an).to(DEV)], [1. / 2 ** lvl],
            torch.from_numpy(g["im_info"]).to(DEV), 1000, 1000, 0.7, 0)
        k = int(cnt[0, 0].item())
        got = rois[0, 0, :k].cpu().numpy()
        stable, _ = orc.generate_proposals(an, 1. / 2 ** lvl, p, d, g["im_info"])
        assert np.array_equal(got, stable), tag
        if c["same_rows_as_a_set"]:
            key = lambda a: a[np.lexsort(a.T[::-1])]  # noqa: E731
            assert np.array_equal(key(got), key(g[tag + "_ref_rois"])), tag


def test_generate_proposals_graph_replays_like_eager():
    """vd_generate_proposals (multi-workgroup radix select) captured into a hipGraph
    and replayed three times, then with new scores: every replay equals an eager
    call.  Its selection counters are re-zeroed by a kernel inside the step (a
    captured hipMemsetAsync did not run again at replay on this ROCm: every replay
    after the first returned count -1, round 5)."""
    import torch
    from vosdetectron_amd import ops
    dev = torch.device("cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    F, A = 4, 3
    shapes = [(200, 336), (100, 168), (50, 84), (25, 42), (13, 21)]
    scales = [1 / 4., 1 / 8., 1 / 16., 1 / 32., 1 / 64.]
    cls = [torch.rand(F, A, h, w, device=dev, generator=g) for h, w in shapes]
    box = [torch.randn(F, 4 * A, h, w, device=dev, generator=g) * .1 for h, w in shapes]
    anc = [torch.rand(h * w * A, 4, device=dev, generator=g, dtype=torch.float64) * 500
           for h, w in shapes]
    for a in anc:
        a[:, 2:] += a[:, :2] + 16
    info = torch.tensor([[800., 1344., 1.]] * F, device=dev)
    args = (cls, box, anc, scales, info, 1000, 1000, 0.7, 0.)
    eager = ops.generate_proposals(*args)
    assert int(eager[2].min()) > 0
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.generate_proposals(*args)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        out = ops.generate_proposals(*args)
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        assert all(torch.equal(a, b) for a, b in zip(out, eager))
    for c in cls:
        c.uniform_(generator=g)
    eager2 = ops.generate_proposals(*args)
    graph.replay()
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(out, eager2))
