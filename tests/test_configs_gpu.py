"""BASELINE.json configs[2..4] on the GPU at their full sizes vs the oracle.

configs[2] e2e_mask_rcnn_R-101-FPN_2x and configs[4] e2e_mask_rcnn_X-101-32x8d-FPN_1x
(grouped 3x3 convolutions, 1000 proposals per image) on a synthetic 800x1333 frame:
stage-wise parity of every HIP stage fed the GPU's own upstream tensors
(proposals + collect and detections bit-exact, box / mask RoIAlign within 1e-4)
and e2e detections + masks vs the independent CPU pipeline.  configs[4]'s
"RoIAlign LDS stress" -- P=14 over the frame's 1000 proposals -- is checked
against the oracle's roi_feature_transform.  configs[3]: the dynamic VOS model
on 480x854 DAVIS-shaped frames, three frames of one sequence with the ConvGRU
hidden states carried (lib_vos/tools/infer_davis_sequential.py:134-149,
vos_model_builder.py:289-447) vs the CPU VOS pipeline.
Reference: lib/core/test.py:50-111 (im_detect_all)."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from tests.engine_checks import LEVEL_SCALES, e2e_vs_cpu, match, stagewise

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


@pytest.fixture(scope="module", params=["e2e_mask_rcnn_R-101-FPN_2x",
                                        "e2e_mask_rcnn_X-101-32x8d-FPN_1x"])
def fpn_setup(request):
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.engine import FramePipeline
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.get(request.param)
    assert cfg.TEST.RPN_POST_NMS_TOP_N == 1000
    model, sd = build_model(cfg, device=DEV, channels_last=True)
    frame = np.random.RandomState(1001).randint(0, 256, (800, 1333, 3), np.uint8)
    pipe = FramePipeline(model, cfg, batch=1, device=DEV, channels_last=True)
    out = pipe.run(torch.from_numpy(frame[None]).to(DEV), keep_intermediates=True)
    return request.param, cfg, sd, pipe, frame, out


def test_fpn_config_stagewise(fpn_setup):
    name, cfg, sd, pipe, frame, out = fpn_setup
    rois, blobs = stagewise(cfg, pipe, out, frame)
    assert len(rois) == 1000, len(rois)  # a full 1000-proposal frame
    if "X-101" in name:
        # configs[4] stress: 14x14 RoIAlign over all 1000 proposals (NHWC product
        # kernel, one launch over the four levels) vs the reference operator API
        from vosdetectron_amd import ops
        rpn_ret = orc.distribute(rois)
        ref = orc.roi_feature_transform(blobs, rpn_ret, "rois", 14, LEVEL_SCALES, 2)
        lv = orc.map_rois_to_fpn_levels(rois[:, 1:5], 2, 5).astype(np.int32) - 2
        rt = torch.from_numpy(rois).to(DEV)
        lt = torch.from_numpy(lv).to(DEV)
        got = ops.roi_align_fpn(out["pyramid"], pipe.roi_scales, rt, lt, 14, 2,
                                roi_order=ops.xcd_roi_order(rt, lt), out_layout="nhwc")
        np.testing.assert_allclose(got.cpu().numpy().transpose(0, 3, 1, 2), ref, rtol=1e-4,
                                   atol=1e-4)
        assert np.bincount(lv, minlength=4).min() > 0  # every level exercised


def test_fpn_config_e2e_vs_cpu(fpn_setup):
    name, cfg, sd, pipe, frame, out = fpn_setup
    from oracle.pipeline import RefCPUPipeline
    from vosdetectron_amd.modeling import _stage_counts
    torch.set_num_threads(16)
    ref = RefCPUPipeline(sd, block_counts=_stage_counts(cfg.MODEL.CONV_BODY),
                         groups=cfg.RESNETS.NUM_GROUPS)
    e2e_vs_cpu(out, ref(frame))


@pytest.fixture(scope="module")
def vos480():
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.engine import VOSPipeline
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.get("vos_R-101-FPN_3x_gn_dynamic_davis")
    assert cfg.TEST.SCALE == 480  # 480 x 854 frames: identity scale, blob 512 x 896
    frames = [np.random.RandomState(400 + i).randint(0, 256, (480, 854, 3), np.uint8)
              for i in range(3)]
    model, sd = build_model(cfg, device=DEV, channels_last=True, calibrate_frame=frames[0])
    pipe = VOSPipeline(model, cfg, frame_hw=(480, 854), batch=1, device=DEV, channels_last=True)
    return cfg, sd, pipe, frames


def test_vos_480x854_sequence_vs_cpu_oracle(vos480):
    """configs[3] at DAVIS size: three frames, hidden states carried, dynamic model;
    frame 0's HIP stages stage-wise, every frame e2e vs the CPU VOS pipeline."""
    cfg, sd, pipe, frames = vos480
    from oracle.vos_pipeline import RefCPUVOSPipeline
    torch.set_num_threads(16)
    ref = RefCPUVOSPipeline(sd, target_scale=480, max_size=cfg.TEST.MAX_SIZE)
    pipe.reset()
    for t, fr in enumerate(frames):
        out = pipe.run(torch.from_numpy(fr[None]).to(DEV), keep_intermediates=True)
        assert tuple(out["feats"][-1].shape[-2:]) == (128, 224)  # P2 of the 512 x 896 blob
        if t == 0:
            stagewise(cfg, pipe, out, fr)
        sc, bx, cl, masks, ex = ref(fr)
        for a, b in zip(out["feats"], ex["fpn"]):
            rel = float((a.cpu() - b).abs().max() / b.abs().max())
            assert rel < 2e-3, (t, rel)
        k = out["counts_host"][0]
        assert abs(k - len(sc)) <= max(2, 0.02 * len(sc)), (t, k, len(sc))
        gd = out["dets"][0, :k].cpu().numpy()
        gc = out["classes"][0, :k].cpu().numpy()
        gm = out["masks"][:k].cpu().numpy()
        assert gm.shape[1:] == (56, 56)
        matched, mask_err = match(gd, gc, gm, sc, bx, cl, masks)
        print("VOS frame %d: %d/%d matched, count %d" % (t, matched, len(sc), k))
        assert matched >= 0.98 * len(sc), (t, matched, len(sc))
        assert np.median(mask_err) < 2e-3, (t, np.median(mask_err))
