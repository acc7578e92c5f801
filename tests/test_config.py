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
