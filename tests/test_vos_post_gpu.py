"""The VOS frame loop's detection heuristics on the device:
TEST.NMS_SMALL_BOX_IOU (lib_vos/tools/vos_test.py:845-860, vd_detections_prev_box_filter)
and nms_with_mask_iou (:985-1029, vd_mask_iou_nms), against the fixtures the
reference's own vos_test produced (tests/golden/vos_post.npz, tools/gen_goldens.py)
and, inside engine.VOSPipeline, stage-wise against the oracle on the GPU's own
detections over a 3-frame, 2-sequence run."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
K = 81


def test_mask_iou_nms_vs_executed_reference(golden):
    from vosdetectron_amd import ops
    g = golden("vos_post")
    for c in range(int(g["mask_count"])):
        masks = torch.from_numpy(g["mask_%d_masks" % c]).to(DEV)
        dets = torch.from_numpy(g["mask_%d_dets" % c]).to(DEV)
        cls = torch.from_numpy(g["mask_%d_classes" % c]).to(DEV)
        keep = ops.mask_iou_nms(masks, dets, cls, float(g["mask_%d_iou_th" % c]),
                                int(g["mask_%d_per_class" % c]))
        assert keep.cpu().tolist() == g["mask_%d_keep" % c].tolist(), c


def test_mask_iou_nms_edges():
    """No detections; masks touching the last pixel; a frame width not a multiple of
    32 (packed words straddle rows); score ties read by index."""
    from vosdetectron_amd import ops
    e = ops.mask_iou_nms(torch.zeros((0, 5, 7), dtype=torch.uint8, device=DEV),
                         torch.zeros((0, 5), device=DEV),
                         torch.zeros((0,), dtype=torch.int32, device=DEV), 0.5, 1)
    assert e.numel() == 0
    rng = np.random.default_rng(3)
    H, W, n = 37, 45, 30
    masks = (rng.uniform(0, 1, (n, H, W)) < 0.3).astype(np.uint8)
    masks[3] = masks[2]
    masks[4, -1, -1] = 1
    dets = np.hstack([rng.uniform(0, 40, (n, 4)), np.round(rng.uniform(0, 1, (n, 1)) * 4) / 4])
    dets = dets.astype(np.float32)
    cls = np.sort(rng.integers(1, 5, n)).astype(np.int32)
    for th, cap in ((0.2, 2), (0.31, 5), (0.9, 1)):
        want = orc.nms_with_mask_iou(dets, cls, masks, th, cap)
        got = ops.mask_iou_nms(torch.from_numpy(masks).to(DEV), torch.from_numpy(dets).to(DEV),
                               torch.from_numpy(cls).to(DEV), th, cap)
        assert got.cpu().tolist() == want.tolist(), (th, cap)


def _postfilter_inputs(g, c):
    """The fixture case's detections before the previous-frame filter (the
    oracle's box_results_with_nms_and_limit, pinned by detections_postfilter.npz)."""
    iou, sthr, pre, cross = g["small_%d_cfg" % c]
    _, _, cb = orc.box_results_with_nms_and_limit(g["small_scores"], g["small_boxes"], K,
                                                  nms_cross_class=cross,
                                                  num_det_per_class_pre=int(pre))
    dets = np.vstack([cb[j] for j in range(1, K)]).reshape(-1, 5).astype(np.float32)
    cls = np.concatenate([[j] * len(cb[j]) for j in range(1, K)]).astype(np.int32)
    return dets, cls, iou, sthr


def test_prev_box_filter_vs_executed_reference(golden):
    from vosdetectron_amd import ops
    g = golden("vos_post")
    cap, pcap = 256, 96
    for c in range(int(g["small_count"])):
        dets, cls, iou, sthr = _postfilter_inputs(g, c)
        n = len(dets)
        assert n == int(g["small_%d_unfiltered" % c])
        D = torch.zeros((2, cap, 5), device=DEV)
        C = torch.zeros((2, cap), dtype=torch.int32, device=DEV)
        D[1, :n], C[1, :n] = torch.from_numpy(dets), torch.from_numpy(cls)
        N = torch.tensor([0, n], dtype=torch.int32, device=DEV)
        pd, pc = g["small_%d_prev_dets" % c], g["small_%d_prev_cls" % c]
        PD = torch.zeros((2, pcap, 5), device=DEV)
        PC = torch.zeros((2, pcap), dtype=torch.int32, device=DEV)
        PD[1, :len(pd)], PC[1, :len(pc)] = torch.from_numpy(pd), torch.from_numpy(pc)
        PN = torch.tensor([0, len(pd)], dtype=torch.int32, device=DEV)
        ops.detections_prev_box_filter(D, C, N, PD, PC, PN, iou, sthr)
        k = int(N[1])
        assert int(N[0]) == 0
        assert np.array_equal(D[1, :k].cpu().numpy(), g["small_%d_dets" % c]), c
        assert C[1, :k].cpu().tolist() == g["small_%d_cls" % c].tolist(), c


def test_prev_box_filter_no_prev_and_assert():
    """A row without a previous result passes unchanged; two previous boxes of one
    class (the reference asserts for every class, vos_test.py:846-848) fail the row
    with VD_COUNT_PREV_BOXES -- also when the current frame has no box of that
    class (row 2) -- and complete()'s check names the heuristic."""
    from vosdetectron_amd import _lib, ops
    D = torch.rand((3, 8, 5), device=DEV) * 100
    D[..., 2:4] += D[..., 0:2]
    C = torch.tensor([[1, 1, 2, 3, 3, 3, 4, 5]] * 3, dtype=torch.int32, device=DEV)
    N = torch.tensor([8, 8, 8], dtype=torch.int32, device=DEV)
    D0 = D.clone()
    PD = torch.zeros((3, 4, 5), device=DEV)
    PC = torch.tensor([[3, 0, 0, 0], [3, 3, 0, 0], [1, 7, 7, 0]], dtype=torch.int32, device=DEV)
    PN = torch.tensor([0, 2, 3], dtype=torch.int32, device=DEV)
    ops.detections_prev_box_filter(D, C, N, PD, PC, PN, 0.3, 0.0)
    assert int(N[0]) == 8 and torch.equal(D[0], D0[0])
    assert int(N[1]) == ops.COUNT_PREV_BOXES == -2
    assert int(N[2]) == ops.COUNT_PREV_BOXES
    with pytest.raises(_lib.VosdetError, match="NMS_SMALL_BOX_IOU"):
        ops.raise_on_failed_counts(N.cpu().tolist())


@pytest.fixture(scope="module")
def vos_seq():
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.engine import VOSPipeline
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.get("vos_R-101-FPN_3x_gn_dynamic_davis")
    cfg.TEST.NMS_SMALL_BOX_IOU = 0.3
    # random-init scores sit near SCORE_THRESH; the fixtures cover the threshold
    cfg.TEST.NMS_SMALL_BOX_SCORE_THRESHOLD = 0.0
    cfg.TEST.NMS_WITH_MASK_IOU = 0.5
    cfg.TEST.NUM_DET_PER_CLASS_POST = 1
    vcfg.check_supported(cfg)
    frames = [np.stack([np.random.RandomState(600 + 10 * i + r).randint(0, 256, (480, 854, 3),
                                                                      np.uint8)
                        for r in range(2)]) for i in range(3)]
    model, sd = build_model(cfg, device=DEV, channels_last=True, calibrate_frame=frames[0][0])
    pipe = VOSPipeline(model, cfg, frame_hw=(480, 854), batch=2, device=DEV, channels_last=True)
    return cfg, pipe, frames


def test_vos_pipeline_heuristics_stagewise(vos_seq):
    """Two sequences, three frames each, both heuristics on.  Frame t's device
    detections equal the oracle's box_results_with_nms_and_limit on the GPU's own
    class scores / deltas with the previous frame's final boxes of the same row;
    frame_results' boxes equal the oracle's nms_with_mask_iou over the oracle's
    paste of the GPU masks; a reset row forgets its previous frame."""
    cfg, pipe, frames = vos_seq
    tst = cfg.TEST
    K = int(cfg.MODEL.NUM_CLASSES)  # 145 (the fork's class-agnostic VOS heads)
    pipe.reset()
    prev = [None, None]
    filtered_any = False
    for t, fr in enumerate(frames):
        if t == 2:
            pipe.reset(rows=[1])  # row 1 starts a new sequence
            prev[1] = None
        out = pipe.run(torch.from_numpy(fr).to(DEV), keep_intermediates=True)
        res = pipe.frame_results(out)
        post = out["rois"].shape[1]
        start = 0
        for f in range(2):
            n = int(out["roi_counts"][f].item())
            rois = out["rois"][f, :n].cpu().numpy()
            sc = out["cls_prob"].view(2, post, K)[f, :n].cpu().numpy()
            dl = out["bbox_pred"].view(2, post, -1)[f, :n].cpu().numpy()
            pred = orc.clip_tiled_boxes(orc.bbox_transform(rois[:, 1:5] / pipe.im_scale, dl,
                                                           tuple(cfg.MODEL.BBOX_REG_WEIGHTS)),
                                        fr[f].shape)
            kw = dict(nms_cross_class=tst.NMS_CROSS_CLASS,
                      num_det_per_class_pre=tst.NUM_DET_PER_CLASS_PRE)
            _, _, cb0 = orc.box_results_with_nms_and_limit(sc, pred, K, tst.SCORE_THRESH,
                                                           tst.NMS, tst.DETECTIONS_PER_IM, **kw)
            _, _, cb = orc.box_results_with_nms_and_limit(
                sc, pred, K, tst.SCORE_THRESH, tst.NMS, tst.DETECTIONS_PER_IM,
                prev_cls_boxes=prev[f], small_box_iou=tst.NMS_SMALL_BOX_IOU,
                small_box_score_thresh=tst.NMS_SMALL_BOX_SCORE_THRESHOLD, **kw)
            want = np.vstack([cb[j] for j in range(1, K)]).reshape(-1, 5)
            wcls = np.concatenate([[j] * len(cb[j]) for j in range(1, K)]).astype(np.int32)
            filtered_any |= len(want) < sum(len(cb0[j]) for j in range(1, K))
            k = out["counts_host"][f]
            assert k == len(want), (t, f, k, len(want))
            assert np.array_equal(out["dets"][f, :k].cpu().numpy(), want), (t, f)
            assert out["classes"][f, :k].cpu().tolist() == wcls.tolist(), (t, f)
            # the mask-IoU NMS over the oracle's paste of the GPU's own masks
            masks = out["masks"][start:start + k].cpu().numpy()
            start += k
            planes = orc.paste_masks(masks, want, 480, 854, cfg.MRCNN.THRESH_BINARIZE)
            keep = orc.nms_with_mask_iou(want, wcls, planes, tst.NMS_WITH_MASK_IOU,
                                         tst.NUM_DET_PER_CLASS_POST)
            cls_boxes, cls_segms = res[f]
            got = np.vstack([cls_boxes[j] for j in range(K)]).reshape(-1, 5)
            assert np.array_equal(got, want[keep]), (t, f)
            assert all(len(cls_segms[j]) == len(cls_boxes[j]) for j in range(K))
            fin = [[] for _ in range(K)]
            for j in range(K):
                if len(cls_boxes[j]):
                    fin[j] = cls_boxes[j]
            prev[f] = fin
    assert filtered_any, "the previous-frame filter never removed a detection"


def test_vos_heuristics_refuse_unfinalized_steps(vos_seq):
    """with NMS_WITH_MASK_IOU / NMS_SMALL_BOX_IOU on, a second run()
    before frame_results(previous) would filter against the wrong frame, and
    frame_segms would skip the mask-IoU NMS: both raise instead."""
    from vosdetectron_amd.engine import frame_segms
    cfg, pipe, frames = vos_seq
    pipe.reset()
    out = pipe.run(torch.from_numpy(frames[0]).to(DEV))
    with pytest.raises(RuntimeError, match="frame_results"):
        pipe.run(torch.from_numpy(frames[1]).to(DEV))
    with pytest.raises(ValueError, match="frame_results"):
        frame_segms(pipe, out, int(cfg.MODEL.NUM_CLASSES))
    pipe.frame_results(out)
    pipe.frame_results(pipe.run(torch.from_numpy(frames[1]).to(DEV)))  # now allowed
    # a dropped step followed by a reset of every row starts new
    # sequences, so the guard no longer applies; a partial reset keeps it
    pipe.run(torch.from_numpy(frames[0]).to(DEV))
    pipe.reset(rows=[0])
    with pytest.raises(RuntimeError, match="frame_results"):
        pipe.run(torch.from_numpy(frames[1]).to(DEV))
    pipe.reset(rows=[0, 1])
    pipe.frame_results(pipe.run(torch.from_numpy(frames[1]).to(DEV)))
    pipe.run(torch.from_numpy(frames[2]).to(DEV))
    pipe.reset()
    pipe.frame_results(pipe.run(torch.from_numpy(frames[0]).to(DEV)))


def test_prev_box_filter_keeps_failed_counts():
    """a frame an upstream kernel failed (count -1, e.g. an
    unbracketable proposal select) keeps its code through the previous-frame
    filter instead of becoming an empty frame, and its rows are untouched."""
    from vosdetectron_amd import _lib, ops
    D = torch.rand((3, 8, 5), device=DEV) * 100
    D[..., 2:4] += D[..., 0:2]
    C = torch.tensor([[1, 1, 2, 3, 3, 3, 4, 5]] * 3, dtype=torch.int32, device=DEV)
    N = torch.tensor([-1, 8, ops.COUNT_PREV_BOXES], dtype=torch.int32, device=DEV)
    D0, C0 = D.clone(), C.clone()
    PD = D.clone()[:, :4].contiguous()
    PC = torch.tensor([[1, 2, 0, 0], [3, 0, 0, 0], [1, 2, 0, 0]], dtype=torch.int32, device=DEV)
    PN = torch.tensor([2, 1, 2], dtype=torch.int32, device=DEV)
    ops.detections_prev_box_filter(D, C, N, PD, PC, PN, 0.3, 0.0)
    got = N.cpu().tolist()
    assert got[0] == -1 and got[2] == ops.COUNT_PREV_BOXES
    assert 0 <= got[1] <= 8
    assert torch.equal(D[0], D0[0]) and torch.equal(C[0], C0[0])
    assert torch.equal(D[2], D0[2]) and torch.equal(C[2], C0[2])
    with pytest.raises(_lib.VosdetError):
        ops.raise_on_failed_counts(got)
