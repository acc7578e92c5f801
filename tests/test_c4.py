"""e2e_mask_rcnn_R-50-C4 (BASELINE.json configs[0]): the single-scale family.

CPU: the module tree carries the reference's parameter names and its dense
parts equal the oracle's C4 pipeline; the oracle's C4 pipeline runs a frame
end to end.  GPU: C4FramePipeline stage by stage against the oracle (proposals
and detections bit-exact from the GPU's own head outputs, the adaptive-sr
14x14 RoIAlign on the 1024-channel res4 map within north_star's 1e-4), then
end to end against the independent CPU pipeline."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

FRAME_HW = (320, 480)  # TEST.SCALE 320 -> identity scale; res4 20 x 30 x 15 = 9000 anchors


def _cfg(post=300):
    from vosdetectron_amd import config as vcfg
    cfg = vcfg.get("e2e_mask_rcnn_R-50-C4_1x")
    cfg.TEST.SCALE = FRAME_HW[0]
    cfg.TEST.RPN_POST_NMS_TOP_N = post
    return cfg


def _frame(seed=7):
    return np.random.RandomState(seed).randint(0, 256, FRAME_HW + (3,), np.uint8)


def test_c4_config_and_names():
    from vosdetectron_amd.c4 import Generalized_RCNN_C4
    cfg = _cfg()
    assert not cfg.FPN.FPN_ON and cfg.TEST.RPN_PRE_NMS_TOP_N == 6000
    m = Generalized_RCNN_C4(cfg)
    names = set(m.state_dict())
    for k in ["Conv_Body.res1.conv1.weight", "Conv_Body.res4.5.conv3.weight",
              "RPN.RPN_conv.weight", "RPN.RPN_cls_score.weight", "RPN.RPN_bbox_pred.bias",
              "Box_Head.res5.0.downsample.0.weight", "Box_Head.res5.2.bn3.bias",
              "Box_Outs.cls_score.weight", "Box_Outs.bbox_pred.weight",
              "Mask_Head.upconv5.weight", "Mask_Outs.classify.weight"]:
        assert k in names, k
    assert "Conv_Body.res5.0.conv1.weight" not in names
    assert m.RPN.RPN_cls_score.out_channels == 15 and m.RPN.RPN_bbox_pred.out_channels == 60
    assert m.Mask_Head.res5 is m.Box_Head.res5  # share_res5_module
    np.testing.assert_array_equal(m.anchors.numpy(),
                                  orc.generate_anchors(16, (32, 64, 128, 256, 512)))


def test_c4_module_tree_vs_oracle_cpu():
    from oracle.pipeline import RefCPUPipelineC4
    from vosdetectron_amd.weights import build_model
    cfg = _cfg(post=50)
    torch.manual_seed(0)
    model, sd = build_model(cfg, device="cpu", fold=False, calibrate_frame=_frame(1))
    ref = RefCPUPipelineC4(sd, post_nms=50, test_scale=FRAME_HW[0])
    frame = _frame()
    blob, _, im_info = orc.get_image_blob(frame, target_scale=FRAME_HW[0], stride=1)
    assert blob.shape == (1, 3) + FRAME_HW  # no padding without FPN
    with torch.no_grad():
        x = torch.from_numpy(blob)
        a, b = model.Conv_Body(x), ref.backbone(x)
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
        p, d = model.RPN.outputs(a)
        rois = np.zeros((4, 5), np.float32)
        rois[:, 1:] = [[0, 0, 63, 63], [10, 20, 200, 150], [100, 50, 479, 319], [5, 5, 40, 300]]
        bf = orc.roi_align(a.numpy(), rois, 14, 14, 1. / 16, 0)
        h1 = model.Box_Head.head(torch.from_numpy(bf))
        h2 = torch.nn.functional.avg_pool2d(ref.res5(torch.from_numpy(bf)), 7).flatten(1)
        torch.testing.assert_close(h1, h2, rtol=1e-5, atol=1e-5)
    torch.set_num_threads(8)
    sc, bx, cl, masks, extra = ref(frame)
    assert len(extra["rois"]) == 50
    assert masks.shape[1:] == (14, 14) and len(masks) == len(sc) == len(cl)


@pytest.fixture(scope="module")
def gpu_setup():
    from vosdetectron_amd.c4 import C4FramePipeline
    from vosdetectron_amd.weights import build_model
    dev = torch.device("cuda")
    cfg = _cfg()
    model, sd = build_model(cfg, device=dev, channels_last=True, calibrate_frame=_frame(1))
    frame = _frame()
    pipe = C4FramePipeline(model, cfg, frame_hw=FRAME_HW, batch=1, device=dev,
                           channels_last=True)
    out = pipe.run(torch.from_numpy(frame[None]).to(dev), keep_intermediates=True)
    return cfg, model, sd, pipe, frame, out


@pytest.mark.gpu
def test_c4_stagewise_parity(gpu_setup):
    cfg, model, sd, pipe, frame, out = gpu_setup
    post = cfg.TEST.RPN_POST_NMS_TOP_N
    _, _, im_info = orc.get_image_blob(frame, target_scale=FRAME_HW[0], stride=1)
    p, d = out["rpn_probs"][0].cpu().numpy(), out["rpn_deltas"][0].cpu().numpy()
    rois, _ = orc.generate_proposals(orc.generate_anchors(16), 1. / 16, p, d, im_info, 6000,
                                     post, 0.7, 0)
    n = int(out["roi_counts"][0].item())
    assert n == len(rois)
    assert np.array_equal(out["rois"][0, :n].cpu().numpy(), rois)
    # adaptive-sr RoIAlign (14x14, C=1024) on the GPU's own res4
    res4 = out["feats"].float().contiguous().cpu().numpy()
    from vosdetectron_amd import ops
    lvl = torch.zeros((n,), dtype=torch.int32, device="cuda")
    nhwc = out["feats"].permute(0, 2, 3, 1).contiguous()
    bf = ops.roi_align_fpn([nhwc], [1. / 16], torch.from_numpy(rois).cuda(), lvl, 14, 0,
                           out_layout="nhwc").permute(0, 3, 1, 2).cpu().numpy()
    bf_ref = orc.roi_align(res4, rois, 14, 14, 1. / 16, 0)
    np.testing.assert_allclose(bf, bf_ref, rtol=1e-4, atol=1e-4)
    # drop-in NCHW operator (reference decomposition): bit-exact
    nchw = ops.RoIAlignFunction(14, 14, 1. / 16, 0)(torch.from_numpy(res4).cuda(),
                                                    torch.from_numpy(rois).cuda())
    assert np.array_equal(nchw.cpu().numpy(), bf_ref)
    # detections from the GPU's own head outputs
    sc = out["cls_prob"][:n].cpu().numpy()
    dl = out["bbox_pred"][:n].cpu().numpy()
    pred = orc.clip_tiled_boxes(orc.bbox_transform(rois[:, 1:5], dl, (10., 10., 5., 5.)),
                                frame.shape)
    s_ref, b_ref, _ = orc.box_results_with_nms_and_limit(sc, pred)
    k = out["counts_host"][0]
    assert k == len(s_ref)
    dets = out["dets"][0, :k].cpu().numpy()
    assert np.array_equal(dets[:, :4], b_ref) and np.array_equal(dets[:, 4], s_ref)
    if k:
        mf_ref = orc.roi_align(res4, out["mask_rois"].cpu().numpy(), 14, 14, 1. / 16, 0)
        np.testing.assert_allclose(out["mask_feat"].cpu().numpy(), mf_ref, rtol=1e-4,
                                   atol=1e-4)


@pytest.mark.gpu
def test_c4_end_to_end_vs_independent_cpu(gpu_setup):
    cfg, model, sd, pipe, frame, out = gpu_setup
    from oracle.pipeline import RefCPUPipelineC4
    torch.set_num_threads(16)
    sc, bx, cl, masks, _ = RefCPUPipelineC4(sd, post_nms=cfg.TEST.RPN_POST_NMS_TOP_N,
                                            test_scale=FRAME_HW[0])(frame)
    assert len(sc) > 0
    from tests.engine_checks import e2e_vs_cpu
    e2e_vs_cpu(out, (sc, bx, cl, masks, None))
