"""TEST.SOFT_NMS and TEST.BBOX_VOTE on the device (lib/core/test.py:756-776):
vd_soft_nms / vd_box_voting (the utils.boxes drop-ins) and vd_box_detections_ex
(the options inside the per-class kernel) against the fixtures the compiled
reference produced (tests/golden/soft_nms.npz, tools/gen_goldens.py soft_nms),
then a FramePipeline step with both options on, stage-wise against the oracle."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
METHODS = ["hard", "linear", "gaussian"]


def test_soft_nms_vs_executed_reference(golden):
    from vosdetectron_amd import ops
    g = golden("soft_nms")
    for c in range(int(g["soft_count"])):
        d = torch.from_numpy(g["soft_in_%d" % int(g["soft_%d_in" % c])]).to(DEV)
        m, th, sigma = g["soft_%d_cfg" % c]
        rows, keep = ops.soft_nms(d, sigma, th, 0.0001, METHODS[int(m)])
        assert np.array_equal(rows.cpu().numpy(), g["soft_%d_out" % c]), c
        assert keep.cpu().tolist() == g["soft_%d_keep" % c].tolist(), c


def test_soft_nms_drop_in_edges():
    """boxes.soft_nms keeps the reference's host signature: no rows pass through;
    every row removed (exact duplicates at hard / linear) leaves the first."""
    from vosdetectron_amd import boxes
    e = np.zeros((0, 5), np.float32)
    r, k = boxes.soft_nms(e)
    assert r is e and k == []
    d = np.array([[0, 0, 9, 9, .9]] * 5, np.float32)
    for m in ("hard", "linear"):
        r, k = boxes.soft_nms(d, overlap_thresh=0.3, score_thresh=0.0001, method=m)
        want_r, want_k = orc.soft_nms(d, 0.5, 0.3, 0.0001, m)
        assert np.array_equal(r, want_r) and list(k) == list(want_k) == [0]
    with pytest.raises(ValueError):
        boxes.soft_nms(d, method="cubic")


def test_box_voting_vs_executed_reference(golden):
    from vosdetectron_amd import ops
    g = golden("soft_nms")
    for c in range(int(g["vote_count"])):
        si, ti = g["vote_%d_sets" % c]
        vth, beta = g["vote_%d_cfg" % c]
        out = ops.box_voting(torch.from_numpy(g["vote_top_%d" % ti]).to(DEV),
                             torch.from_numpy(g["vote_set_%d" % si]).to(DEV), vth,
                             str(g["vote_%d_method" % c]), beta)
        assert np.array_equal(out.cpu().numpy(), g["vote_%d_out" % c]), \
            (c, str(g["vote_%d_method" % c]))


def test_box_detections_options_vs_executed_reference(golden):
    """vd_box_detections_ex decodes the fixture's rois / deltas on the device and
    runs soft-NMS and / or box voting inside the per-class kernel: the class-major
    rows after the limit equal the fork's box_results_with_nms_and_limit."""
    from vosdetectron_amd import ops
    g = golden("soft_nms")
    R = g["det_rois"].shape[0]
    rois = torch.from_numpy(g["det_rois"][None]).to(DEV)
    cls = torch.from_numpy(g["det_scores"][None]).to(DEV)
    pred = torch.from_numpy(g["det_deltas"][None]).to(DEV)
    cnt = torch.tensor([R], dtype=torch.int32, device=DEV)
    hw = torch.from_numpy(g["det_im_hw"][None]).to(DEV)
    for c in range(int(g["det_count"])):
        soft, vote, vth = [str(v) for v in g["det_%d_cfg" % c]]
        dets, dcls, dcnt = ops.box_detections(
            rois, cls, pred, cnt, torch.tensor([1.0], device=DEV), hw, det_cap=256,
            soft_nms=None if soft == "None" else soft,
            bbox_vote=None if vote == "None" else vote, bbox_vote_thresh=float(vth))
        n = int(dcnt[0])
        assert np.array_equal(dets[0, :n].cpu().numpy(), g["det_%d_dets" % c]), (c, soft, vote)
        assert dcls[0, :n].cpu().tolist() == g["det_%d_cls" % c].tolist(), (c, soft, vote)


@pytest.mark.parametrize("soft,vote", [("linear", "IOU_AVG"), ("gaussian", None),
                                       (None, "AVG")])
def test_pipeline_soft_nms_vote_stagewise(soft, vote):
    """A 2-frame FramePipeline step at 480 x 640 with the options from the
    config: the device detections equal the oracle's box_results (same options)
    on the GPU's own class scores and deltas."""
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.engine import FramePipeline
    from vosdetectron_amd.weights import build_model
    ov = {"TEST.SCALE": 480, "TEST.SOFT_NMS.ENABLED": soft is not None,
          "TEST.SOFT_NMS.METHOD": soft or "linear", "TEST.BBOX_VOTE.ENABLED": vote is not None,
          "TEST.BBOX_VOTE.SCORING_METHOD": vote or "ID", "TEST.BBOX_VOTE.VOTE_TH": 0.5}
    cfg = vcfg.e2e_mask_rcnn_R_50_FPN_1x()
    for k, v in ov.items():
        d = cfg
        for p in k.split(".")[:-1]:
            d = d[p]
        d[k.split(".")[-1]] = v
    vcfg.check_supported(cfg)
    model, _ = build_model(cfg, seed=0, device=DEV, channels_last=True)
    pipe = FramePipeline(model, cfg, frame_hw=(480, 640), batch=2, device=DEV,
                         channels_last=True)
    frames = np.stack([np.random.RandomState(900 + r).randint(0, 256, (480, 640, 3), np.uint8)
                       for r in range(2)])
    out = pipe.run(torch.from_numpy(frames).to(DEV))
    tst, K = cfg.TEST, cfg.MODEL.NUM_CLASSES
    post = out["rois"].shape[1]
    total = 0
    for f in range(2):
        n = int(out["roi_counts"][f].item())
        rois = out["rois"][f, :n].cpu().numpy()
        sc = out["cls_prob"].view(2, post, K)[f, :n].cpu().numpy()
        dl = out["bbox_pred"].view(2, post, -1)[f, :n].cpu().numpy()
        pred = orc.clip_tiled_boxes(orc.bbox_transform(rois[:, 1:5] / pipe.im_scale, dl,
                                                       tuple(cfg.MODEL.BBOX_REG_WEIGHTS)),
                                    frames[f].shape)
        s_ref, b_ref, _ = orc.box_results_with_nms_and_limit(
            sc, pred, K, tst.SCORE_THRESH, tst.NMS, tst.DETECTIONS_PER_IM,
            soft_nms_method=soft, soft_nms_sigma=tst.SOFT_NMS.SIGMA, bbox_vote=vote,
            bbox_vote_th=tst.BBOX_VOTE.VOTE_TH)
        k = out["counts_host"][f]
        assert k == len(s_ref), (f, k, len(s_ref))
        dets = out["dets"][f, :k].cpu().numpy()
        assert np.array_equal(dets[:, :4], b_ref) and np.array_equal(dets[:, 4], s_ref), f
        total += k
    assert total > 0
