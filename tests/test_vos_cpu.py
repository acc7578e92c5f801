"""VOS path on the host: the oracle's FlowAlign restatement against known
answers, and the product's module tree (GN ResNet-101 + GN FPN + ConvGRUs,
reference-semantics forward on CPU) against the oracle's CPU VOS pipeline,
frame after frame with hidden states carried (dynamic) or reset (static)."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc


def test_flow_align_oracle_affine_ramp_is_exact():
    """Bilinear sampling reproduces an affine function exactly wherever the
    displaced point stays inside [0, H-1) x [0, W-1)."""
    B, C, H, W = 1, 2, 7, 9
    yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    f = np.stack([2 * yy + 0.5 * xx, -yy + 3 * xx]).astype(np.float32)[None]
    rng = np.random.default_rng(0)
    fl = rng.uniform(-2, 2, (B, 2, H, W)).astype(np.float32)
    out = orc.flow_align(f, fl)
    py, px = yy + fl[0, 1], xx + fl[0, 0]
    inside = (py >= 0) & (py < H - 1) & (px >= 0) & (px < W - 1)
    np.testing.assert_allclose(out[0, 0][inside], (2 * py + 0.5 * px)[inside], rtol=0, atol=2e-5)
    np.testing.assert_allclose(out[0, 1][inside], (-py + 3 * px)[inside], rtol=0, atol=2e-5)
    assert np.all(out[0][:, ~inside] == 0)


def test_flow_align_oracle_integer_shift():
    f = np.random.default_rng(1).standard_normal((2, 3, 6, 8)).astype(np.float32)
    fl = np.zeros((2, 2, 6, 8), np.float32)
    fl[:, 0] = 1.0  # x + 1
    out = orc.flow_align(f, fl)
    np.testing.assert_array_equal(out[..., :-1, :-2], f[..., :-1, 1:-1])
    assert np.all(out[..., -2:] == 0) and np.all(out[..., -1, :] == 0)


def test_flow_downsample_is_scaled_block_mean():
    rng = np.random.default_rng(2)
    fl = rng.standard_normal((1, 2, 16, 24)).astype(np.float32)
    d = orc.flow_downsample(fl, 0.25)
    blk = fl.reshape(1, 2, 4, 4, 6, 4).mean(axis=(3, 5)) * 0.25
    np.testing.assert_allclose(d, blk, rtol=1e-5, atol=1e-6)


@pytest.fixture(scope="module", params=["vos_R-101-FPN_3x_gn_dynamic_davis",
                                        "vos_R-101-FPN_3x_gn_static_davis"])
def vos_cpu(request):
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.get(request.param)
    cfg.TEST.SCALE = 128
    frames = [np.random.RandomState(50 + i).randint(0, 256, (128, 228, 3), np.uint8)
              for i in range(3)]
    torch.set_num_threads(8)
    model, sd = build_model(cfg, device="cpu", fold=False, calibrate_frame=frames[0])
    return cfg, model, sd, frames


def test_vos_modules_match_oracle_pipeline(vos_cpu):
    """Parameter names + module order of Generalized_VOS_RCNN: its reference-
    semantics forward (FPN body -> temporal_fusion) reproduces the oracle's
    restated VOS pyramid bit for bit on CPU, with the hidden states of frame t
    feeding frame t+1 (dynamic) or reset every frame (static)."""
    cfg, model, sd, frames = vos_cpu
    from oracle.vos_pipeline import RefCPUVOSPipeline
    dyn = cfg.CONVGRU.DYNAMIC_MODEL
    ref = RefCPUVOSPipeline(sd, dynamic=dyn, target_scale=128, max_size=cfg.TEST.MAX_SIZE)
    model.clean_hidden_states()
    outs = []
    for fr in frames:
        sc, bx, cl, masks, ex = ref(fr)
        blob, _, _ = orc.get_image_blob(fr, 128, cfg.TEST.MAX_SIZE, cfg.FPN.COARSEST_STRIDE)
        with torch.no_grad():
            feats = model.temporal_fusion(model.Conv_Body(torch.from_numpy(blob)), fused=False)
        for a, b in zip(feats, ex["fpn"]):
            assert torch.equal(a, b)
        assert masks.shape[1:] == (56, 56)
        outs.append(feats[-1].clone())
    assert (model.hidden_states[0] is not None) == dyn
    # the dynamic model's state changes the pyramid of a repeated frame
    with torch.no_grad():
        blob, _, _ = orc.get_image_blob(frames[-1], 128, cfg.TEST.MAX_SIZE, 64)
        again = model.temporal_fusion(model.Conv_Body(torch.from_numpy(blob)), fused=False)[-1]
    assert torch.equal(again, outs[-1]) != dyn
