"""The restated configurations equal the reference's YAML files merged over the
defaults, for every key the hot path reads.  Reads /root/reference as text
(YAML, safe loader) when it is present -- this container only; skipped on the
GPU box, where the reference does not exist."""
import os

import pytest

from vosdetectron_amd import config as vcfg

REF = "/root/reference"
CASES = {
    "e2e_mask_rcnn_R-50-C4_1x": "configs/baselines/e2e_mask_rcnn_R-50-C4_1x.yaml",
    "e2e_mask_rcnn_R-50-FPN_1x": "configs/baselines/e2e_mask_rcnn_R-50-FPN_1x.yaml",
    "e2e_mask_rcnn_R-101-FPN_2x": "configs/baselines/e2e_mask_rcnn_R-101-FPN_2x.yaml",
    "e2e_mask_rcnn_X-101-32x8d-FPN_1x": "configs/baselines/e2e_mask_rcnn_X-101-32x8d-FPN_1x.yaml",
}
KEYS = ["MODEL.CONV_BODY", "MODEL.MASK_ON", "FAST_RCNN.ROI_BOX_HEAD", "FAST_RCNN.ROI_XFORM_METHOD",
        "FAST_RCNN.ROI_XFORM_RESOLUTION", "FAST_RCNN.ROI_XFORM_SAMPLING_RATIO",
        "MRCNN.ROI_MASK_HEAD", "MRCNN.RESOLUTION", "MRCNN.ROI_XFORM_RESOLUTION",
        "MRCNN.ROI_XFORM_SAMPLING_RATIO", "MRCNN.DILATION", "RESNETS.NUM_GROUPS",
        "RESNETS.WIDTH_PER_GROUP", "TEST.SCALE", "TEST.MAX_SIZE", "TEST.NMS",
        "TEST.RPN_PRE_NMS_TOP_N", "TEST.RPN_POST_NMS_TOP_N", "RPN.SIZES", "FPN.FPN_ON"]


def _get(cfg, key):
    for p in key.split("."):
        cfg = cfg[p]
    return cfg


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree absent")
@pytest.mark.parametrize("name", sorted(CASES))
def test_config_matches_reference_yaml(name):
    path = os.path.join(REF, CASES[name])
    if not os.path.exists(path):
        pytest.skip("yaml absent")
    ours = vcfg.get(name)
    ref = vcfg.load_cfg(path)
    for k in KEYS:
        a, b = _get(ours, k), _get(ref, k)
        if isinstance(a, (list, tuple)):
            a, b = tuple(a), tuple(b)
        assert a == b, (name, k, a, b)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree absent")
@pytest.mark.parametrize("yml,keys", [
    ("configs/baselines/e2e_mask_rcnn_X-152-32x8d-FPN-IN5k_1.44x.yaml",
     ["TEST.BBOX_AUG.ENABLED", "TEST.MASK_AUG.ENABLED"]),
])
def test_unsupported_options_raise(yml, keys):
    """A reference YAML that enables an inference option this path does not build
    (test-time augmentation, ...) raises and names the keys, through both
    load_cfg and merge_cfg_from_file; the global cfg is left unchanged."""
    path = os.path.join(REF, yml)
    with pytest.raises(NotImplementedError) as e:
        vcfg.load_cfg(path)
    for k in keys:
        assert k in str(e.value), (k, str(e.value))
    before = vcfg.copy.deepcopy(vcfg.cfg)
    with pytest.raises(NotImplementedError):
        vcfg.merge_cfg_from_file(path)
    assert vcfg.cfg == before


def test_unsupported_overrides_raise():
    for key, val in (("MODEL.USE_DELTA_FLOW", True), ("TEST.KPS_AUG.ENABLED", True)):
        with pytest.raises(NotImplementedError, match=key.replace(".", r"\.")):
            vcfg.load_cfg(overrides={key: val})
    with pytest.raises(NotImplementedError, match="BBOX_VOTE"):
        vcfg.merge_cfg_from_list(["TEST.BBOX_VOTE.ENABLED", "True",
                                  "TEST.BBOX_VOTE.SCORING_METHOD", "TEMP_AVG"])
    with pytest.raises(NotImplementedError, match="SOFT_NMS"):
        vcfg.load_cfg(overrides={"TEST.SOFT_NMS.ENABLED": True, "TEST.SOFT_NMS.METHOD": "cubic"})
    # disabled values are accepted
    vcfg.load_cfg(overrides={"TEST.SOFT_NMS.ENABLED": False, "TEST.BBOX_VOTE.ENABLED": False})


def test_soft_nms_and_box_voting_are_built():
    """TEST.SOFT_NMS (every method) and TEST.BBOX_VOTE (ID / AVG / IOU_AVG /
    QUASI_SUM, GENERALIZED_AVG at beta 1) load and map onto vd_box_detections_ex."""
    from vosdetectron_amd.engine import nms_options
    for m in ("hard", "linear", "gaussian"):
        c = vcfg.load_cfg(overrides={"TEST.SOFT_NMS.ENABLED": True, "TEST.SOFT_NMS.METHOD": m})
        assert nms_options(c) == {"soft_nms": m, "soft_nms_sigma": 0.5}
    for sm in ("ID", "AVG", "IOU_AVG", "QUASI_SUM", "GENERALIZED_AVG"):
        c = vcfg.load_cfg(overrides={"TEST.BBOX_VOTE.ENABLED": True,
                                     "TEST.BBOX_VOTE.SCORING_METHOD": sm})
        assert nms_options(c)["bbox_vote"] == sm
    # SCORING_METHOD_BETA never reaches box_voting in the reference (test.py:770-775,
    # vos_test.py:786-791): beta stays 1, GENERALIZED_AVG at any beta is AVG
    for sm in ("QUASI_SUM", "GENERALIZED_AVG"):
        c = vcfg.load_cfg(overrides={"TEST.BBOX_VOTE.ENABLED": True,
                                     "TEST.BBOX_VOTE.SCORING_METHOD": sm,
                                     "TEST.BBOX_VOTE.SCORING_METHOD_BETA": 2.0})
        assert nms_options(c)["bbox_vote_beta"] == 1.0
    assert nms_options(vcfg.load_cfg()) == {}
    c = vcfg.load_cfg(os.path.join(REF, "lib_vos/tools/R-101-FPN_3x_gn_train_online.yaml")) \
        if os.path.isdir(REF) else None
    if c is not None:  # the fork's ablation setting (disabled there)
        assert (c.TEST.BBOX_VOTE.VOTE_TH, c.TEST.BBOX_VOTE.SCORING_METHOD) == (0.5, "IOU_AVG")


def test_vos_heuristics_are_built():
    """TEST.NMS_WITH_MASK_IOU and TEST.NMS_SMALL_BOX_IOU (the VOS
    frame loop's heuristics, lib_vos/tools/vos_test.py:113-118, 845-860) are
    implemented by engine.VOSPipeline: enabling them loads."""
    c = vcfg.load_cfg(overrides={"TEST.NMS_WITH_MASK_IOU": 0.9, "TEST.NMS_SMALL_BOX_IOU": 0.3,
                                 "TEST.NMS_SMALL_BOX_SCORE_THRESHOLD": 0.2,
                                 "TEST.NUM_DET_PER_CLASS_POST": 1})
    assert c.TEST.NMS_WITH_MASK_IOU == 0.9 and c.TEST.NMS_SMALL_BOX_IOU == 0.3
    assert c.TEST.NMS_SMALL_BOX_SCORE_THRESHOLD == 0.2


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree absent")
def test_train_online_yaml_loads():
    """The fork's online-training VOS config (NMS_WITH_MASK_IOU 1.0,
    NUM_DET_PER_CLASS_POST 1, NMS_SMALL_BOX_SCORE_THRESHOLD 0.2) loads."""
    c = vcfg.load_cfg(os.path.join(REF, "lib_vos/tools/R-101-FPN_3x_gn_train_online.yaml"))
    assert c.TEST.NMS_WITH_MASK_IOU == 1.0 and c.TEST.NUM_DET_PER_CLASS_POST == 1
    assert c.TEST.NMS_SMALL_BOX_SCORE_THRESHOLD == 0.2