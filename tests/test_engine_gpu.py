"""End-to-end engine on the GPU vs the oracle pipeline.

Stage-wise parity: each HIP stage is fed the GPU's own upstream tensors and
compared with the oracle run on the same inputs -- proposals from the GPU's RPN
outputs and the detections from the GPU's class scores / deltas bit-exact; the
box RoIAlign from the GPU's pyramid and rois and the mask RoIAlign from the GPU
detections within north_star's 1e-4 (the product's separable kernel), and
bit-exact through the reference-order kernel (variant 3).  The dense PyTorch parts (convs: MIOpen vs oneDNN, folded vs
unfolded AffineChannel) are compared within fp32 tolerance, and the final
detections are matched against the fully independent CPU pipeline."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


@pytest.fixture(scope="module", params=["nchw", "nhwc"])
def setup(request):
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.engine import FramePipeline
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.get("e2e_mask_rcnn_R-50-FPN_1x")
    cl = request.param == "nhwc"
    model, sd = build_model(cfg, device=DEV, channels_last=cl)
    frame = np.random.RandomState(1000).randint(0, 256, (800, 1333, 3), np.uint8)
    pipe = FramePipeline(model, cfg, batch=1, device=DEV, channels_last=cl)
    out = pipe.run(torch.from_numpy(frame[None]).to(DEV), keep_intermediates=True)
    return cfg, model, sd, pipe, frame, out


def test_stagewise_parity(setup, monkeypatch):
    cfg, model, sd, pipe, frame, out = setup
    # blob (image_to_blob) vs get_image_blob
    blob_ref, _, im_info = orc.get_image_blob(frame)
    from vosdetectron_amd import ops
    blob = ops.image_to_blob(torch.from_numpy(frame[None]).to(DEV), pipe.lut, pipe.Hp, pipe.Wp)
    assert np.array_equal(blob.cpu().numpy(), blob_ref)
    # the exact tensors the engine consumed (convolution algorithms may differ
    # between two calls, so a rerun would not be bit-identical)
    feats = out["feats"]
    rl, pl = [], []
    for i, lvl in enumerate(range(2, 7)):
        p, d = out["rpn_probs"][i], out["rpn_deltas"][i]
        r, pr = orc.generate_proposals(orc.fpn_level_anchors(lvl), 1. / 2 ** lvl,
                                       p.cpu().numpy(), d.cpu().numpy(), im_info)
        rl.append(r)
        pl.append(pr)
    rois = orc.collect(rl, pl, 1000)
    n = int(out["roi_counts"][0].item())
    assert n == len(rois)
    assert np.array_equal(out["rois"][0, :n].cpu().numpy(), rois)
    # box RoIAlign through the reference operator API on the GPU pyramid
    rpn_ret = orc.distribute(rois)
    blobs = [f.cpu().numpy() for f in feats[1:]]
    bf_ref = orc.roi_feature_transform(blobs, rpn_ret, "rois", 7, [1. / 32, 1. / 16, 1. / 8, 1. / 4], 2)
    pyr = out["pyramid"]
    lv = orc.map_rois_to_fpn_levels(rois[:, 1:5], 2, 5).astype(np.int32) - 2
    args = (pyr, pipe.roi_scales, torch.from_numpy(rois).to(DEV), torch.from_numpy(lv).to(DEV),
            7, 2)
    np.testing.assert_allclose(ops.roi_align_fpn(*args).cpu().numpy(), bf_ref, rtol=1e-4,
                               atol=1e-4)
    monkeypatch.setenv("VOSDET_ROIALIGN_VARIANT", "3")
    assert np.array_equal(ops.roi_align_fpn(*args).cpu().numpy(), bf_ref)
    # the LDS-staged tile-binned kernel on the engine's own pyramid and proposals:
    # bit-identical to the reference operator API
    for v in ("30",):
        monkeypatch.setenv("VOSDET_ROIALIGN_VARIANT", v)
        got = ops.roi_align_fpn(*args, out_layout="nhwc").permute(0, 3, 1, 2).cpu().numpy()
        assert np.array_equal(got, bf_ref), v
    monkeypatch.delenv("VOSDET_ROIALIGN_VARIANT")
    # detections from the GPU's own head outputs
    sc = out["cls_prob"][:n].cpu().numpy()
    dl = out["bbox_pred"][:n].cpu().numpy()
    pred = orc.clip_tiled_boxes(orc.bbox_transform(rois[:, 1:5] / 1.0, dl, (10., 10., 5., 5.)),
                                frame.shape)
    s_ref, b_ref, cls_boxes = orc.box_results_with_nms_and_limit(sc, pred)
    k = out["counts_host"][0]
    assert k == len(s_ref)
    dets = out["dets"][0, :k].cpu().numpy()
    assert np.array_equal(dets[:, :4], b_ref) and np.array_equal(dets[:, 4], s_ref)
    # mask RoIAlign from the GPU detections
    mret = orc.distribute(out["mask_rois"].cpu().numpy(), prefix="mask_rois")
    mf_ref = orc.roi_feature_transform(blobs, mret, "mask_rois", 14,
                                       [1. / 32, 1. / 16, 1. / 8, 1. / 4], 2)
    mf = out["mask_feat"].cpu().numpy()
    if mf.ndim == 4 and mf.shape[-1] == mf_ref.shape[1] and mf.shape[1] != mf_ref.shape[1]:
        mf = mf.transpose(0, 3, 1, 2)  # NHWC product layout
    np.testing.assert_allclose(mf, mf_ref, rtol=1e-4, atol=1e-4)


def test_model_outputs_vs_cpu_torch(setup):
    """Dense parts within tolerance: folded GPU body vs the oracle's unfolded CPU body."""
    cfg, model, sd, pipe, frame, out = setup
    from oracle.pipeline import RefCPUPipeline
    ref = RefCPUPipeline(sd)
    blob_ref, _, _ = orc.get_image_blob(frame)
    with torch.no_grad():
        f_ref = ref.backbone(torch.from_numpy(blob_ref))
        f_gpu = pipe.backbone(torch.from_numpy(frame[None]).to(DEV))
    for a, b in zip(f_gpu, f_ref):
        a = a.cpu()
        rel = (a - b).abs().max() / b.abs().max()
        assert rel < 1e-3, rel


def test_end_to_end_vs_independent_cpu(setup):
    """Full CPU pipeline (independent convs) vs the GPU engine: detections match
    by class + IoU (>= 98 %); masks of matched detections agree to tolerance."""
    cfg, model, sd, pipe, frame, out = setup
    from oracle.pipeline import RefCPUPipeline
    from tests.engine_checks import e2e_vs_cpu
    torch.set_num_threads(16)
    e2e_vs_cpu(out, RefCPUPipeline(sd)(frame))


def test_stage_timers(setup):
    """HIP-event stage timers (the reference's im_detect_all timers dict)."""
    cfg, model, sd, pipe, frame, out = setup
    pipe.enable_timers()
    try:
        for _ in range(2):
            pipe.run(torch.from_numpy(frame[None]).to(DEV))
        s = pipe.timer_summary()
        assert set(s) == {"conv_body", "proposals", "box_head", "misc_bbox", "im_detect_mask"}
        assert all(v > 0 for v in s.values()) and pipe.timers["conv_body"].calls == 2
    finally:
        pipe.enable_timers(False)
