"""The reference's Python operator API, mirrored over the HIP kernels, called the
way the reference calls it:

* GenerateProposalsOp(anchors, spatial_scale)(rpn_cls_prob, rpn_bbox_pred, im_info)
  (lib/modeling/generate_proposals.py:13-102) vs the fixtures the reference's own
  op produced (tests/golden/proposals.npz, tools/gen_goldens.py);
* CollectAndDistributeFpnRpnProposalsOp()(inputs, roidb, im_info)
  (collect_and_distribute_fpn_rpn_proposals.py:46-88) vs the reference's
  collect + distribute output dict (collect_distribute.npz);
* utils.boxes.nms(ndarray, thresh) (lib/utils/boxes.py:329-333) vs the oracle;
* Generalized_RCNN.roi_feature_transform(blobs_in, rpn_ret, ...) for RoIAlign and
  the config default RoIPoolF (model_builder.py:252-324, config.py:632) vs the
  oracle's per-level loop, and the heads' roi_xform forward path."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def test_generate_proposals_op_vs_reference_fixture(golden):
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.generate_proposals import GenerateProposalsOp
    g = golden("proposals")
    cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
    cfg.TEST.RPN_MIN_SIZE = 0
    for lvl in range(2, 7):
        an = orc.fpn_level_anchors(lvl)
        op = GenerateProposalsOp(an, 1. / 2 ** lvl, cfg=cfg)
        op.eval()
        rois, probs = op(torch.from_numpy(g["probs_fpn%d" % lvl]).to(DEV),
                         torch.from_numpy(g["deltas_fpn%d" % lvl]).to(DEV),
                         torch.from_numpy(g["im_info"]))  # im_info stays on the host
        assert isinstance(rois, np.ndarray) and rois.dtype == np.float32
        assert np.array_equal(rois, g["rois_fpn%d" % lvl]), lvl
        assert np.array_equal(probs, g["roi_probs_fpn%d" % lvl]), lvl
    # the reference's NaN guard (generate_proposals.py:62-63) and the no-CPU rule
    d = torch.from_numpy(g["deltas_fpn6"]).to(DEV)
    d[0, 0, 0, 0] = float("nan")
    with pytest.raises(ValueError, match="bbox_deltas nan"):
        op(torch.from_numpy(g["probs_fpn6"]).to(DEV), d, torch.from_numpy(g["im_info"]))
    with pytest.raises(NotImplementedError):
        op(torch.from_numpy(g["probs_fpn6"]), torch.from_numpy(g["deltas_fpn6"]),
           torch.from_numpy(g["im_info"]))


def test_generate_proposals_op_two_images():
    """N = 2 images in one call: rows per image in batch order, batch column set."""
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.generate_proposals import GenerateProposalsOp
    rng = np.random.default_rng(4)
    cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
    an = orc.fpn_level_anchors(4)
    p = rng.uniform(0, 1, (2, 3, 25, 42)).astype(np.float32)
    d = rng.normal(0, 0.3, (2, 12, 25, 42)).astype(np.float32)
    info = np.array([[800, 1344, 1.0], [640, 1024, 1.0]], np.float32)
    rois, probs = GenerateProposalsOp(an, 1. / 16, cfg=cfg).eval()(
        torch.from_numpy(p).to(DEV), torch.from_numpy(d).to(DEV), info)
    ref_r, ref_p = orc.generate_proposals(an, 1. / 16, p, d, info)
    assert np.array_equal(rois, ref_r) and np.array_equal(probs, ref_p)
    assert set(np.unique(rois[:, 0])) == {0., 1.}


def test_collect_and_distribute_op_vs_reference_fixture(golden):
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.collect_and_distribute_fpn_rpn_proposals import (
        CollectAndDistributeFpnRpnProposalsOp, collect, distribute)
    gp, gc = golden("proposals"), golden("collect_distribute")
    cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
    inputs = [gp["rois_fpn%d" % l] for l in range(2, 7)] + \
             [gp["roi_probs_fpn%d" % l] for l in range(2, 7)]
    op = CollectAndDistributeFpnRpnProposalsOp(cfg=cfg).eval()
    blobs = op(inputs, None, torch.from_numpy(gp["im_info"]))
    assert set(blobs) == {"rois", "rois_fpn2", "rois_fpn3", "rois_fpn4", "rois_fpn5",
                          "rois_idx_restore_int32"}
    for k, v in blobs.items():
        assert v.dtype == gc[k].dtype and np.array_equal(v, gc[k]), k
    assert np.array_equal(collect(inputs, False, cfg), gc["collected"])
    d2 = distribute(gc["collected"], None, cfg)
    for k, v in d2.items():
        assert np.array_equal(v, gc[k]), k
    with pytest.raises(NotImplementedError):
        op.train()(inputs, None, None)


def test_boxes_nms_ndarray_api():
    from vosdetectron_amd import boxes
    rng = np.random.default_rng(9)
    for n, q in ((0, 0), (1, 0), (300, 0), (2000, 16)):
        xy = rng.uniform(0, 500, (n, 2))
        s = rng.uniform(0, 1, (n, 1))
        if q:
            s = np.round(s * q) / q  # ties
        d = np.hstack([xy, xy + rng.uniform(4, 120, (n, 2)), s]).astype(np.float32)
        keep = boxes.nms(d, 0.5)
        if n == 0:
            assert keep == []
            continue
        assert keep.dtype == np.int64 and np.array_equal(keep, orc.nms(d, 0.5))
    dt = torch.from_numpy(d).to(DEV)
    assert np.array_equal(boxes.nms(dt, 0.3).cpu().numpy(), orc.nms(d, 0.3))


@pytest.fixture(scope="module")
def rcnn():
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.modeling import Generalized_RCNN
    cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
    return Generalized_RCNN(cfg).to(DEV).eval()


def _pyramid_and_rois(seed=3, R=300):
    rng = np.random.default_rng(seed)
    sizes = [(25, 42), (50, 84), (100, 168), (200, 336)]  # P5..P4..P2 (blobs_in order)
    feats = [rng.standard_normal((1, 256, h, w), dtype=np.float32) for h, w in sizes]
    s = np.exp(rng.uniform(np.log(16), np.log(600), R))
    xy = rng.uniform(0, 1200, (R, 2))
    rois = np.hstack([np.zeros((R, 1)), xy, np.minimum(xy + s[:, None], 1330)]).astype(np.float32)
    return feats, rois


def test_roi_feature_transform_roialign_and_roipoolf(rcnn):
    feats, rois = _pyramid_and_rois()
    rpn_ret = orc.distribute(rois)
    assert min(len(rpn_ret["rois_fpn%d" % l]) for l in range(2, 6)) > 0
    blobs = [torch.from_numpy(f).to(DEV) for f in feats]
    scales = [1. / 32, 1. / 16, 1. / 8, 1. / 4]
    got = rcnn.roi_feature_transform(blobs, rpn_ret, blob_rois="rois", method="RoIAlign",
                                     resolution=7, spatial_scale=scales, sampling_ratio=2)
    ref = orc.roi_feature_transform(feats, rpn_ret, "rois", 7, scales, 2)
    assert np.array_equal(got.cpu().numpy(), ref)  # NCHW drop-in kernel: bit-exact
    # RoIPoolF, the config default method (config.py:632): per-level RoIPool +
    # cat + restore, as model_builder.py:271-303 composes it
    got_p = rcnn.roi_feature_transform(blobs, rpn_ret, blob_rois="rois", method="RoIPoolF",
                                       resolution=7, spatial_scale=scales)
    outs = []
    for lvl in range(2, 6):
        r = rpn_ret["rois_fpn%d" % lvl]
        outs.append(orc.roi_pool(feats[5 - lvl], r, 7, 7, scales[5 - lvl])[0])
    ref_p = np.concatenate(outs)[rpn_ret["rois_idx_restore_int32"].astype(np.int64)]
    assert np.array_equal(got_p.cpu().numpy(), ref_p)
    with pytest.raises(AttributeError):  # the reference's dead RoICrop branch
        rcnn.roi_feature_transform(blobs, rpn_ret, method="RoICrop")


def test_heads_roi_xform_forward_path(rcnn):
    """Box_Head.forward(x, rpn_ret) and Mask_Head.forward(x, rpn_ret): the
    reference-API path (roi_xform = roi_feature_transform) equals the engine's
    fused path (one FPN launch) on the same rois within RoIAlign's 1e-4."""
    from vosdetectron_amd import ops
    feats, rois = _pyramid_and_rois(seed=5, R=200)
    blobs = [torch.from_numpy(f).to(DEV) for f in feats]
    rpn_ret = orc.distribute(rois)
    rpn_ret.update(orc.distribute(rois[:64], prefix="mask_rois"))
    with torch.no_grad():
        x_ref = rcnn.Box_Head(blobs, rpn_ret)
        pyr = [b.permute(0, 2, 3, 1).contiguous() for b in blobs[::-1]]
        lv = orc.map_rois_to_fpn_levels(rois[:, 1:5], 2, 5).astype(np.int32) - 2
        bf = ops.roi_align_fpn(pyr, [1. / 4, 1. / 8, 1. / 16, 1. / 32],
                               torch.from_numpy(rois).to(DEV), torch.from_numpy(lv).to(DEV), 7, 2)
        x_eng = rcnn.Box_Head.mlp(bf)
        assert float((x_ref - x_eng).abs().max()) <= 1e-3 * max(1., float(x_ref.abs().max()))
        m_ref = rcnn.Mask_Head(blobs, rpn_ret)
        mf = ops.roi_align_fpn(pyr, [1. / 4, 1. / 8, 1. / 16, 1. / 32],
                               torch.from_numpy(rois[:64]).to(DEV),
                               torch.from_numpy(lv[:64]).to(DEV), 14, 2)
        m_eng = rcnn.Mask_Head.head(mf)
        assert float((m_ref - m_eng).abs().max()) <= 1e-3 * max(1., float(m_ref.abs().max()))
