"""VOS temporal path on the GPU: FlowAlign vs the oracle's C restatement
(bit-exact fwd, 1e-5 bwd), GroupNorm epilogues and the fused ConvGRU vs torch
fp32 module math (tolerance stated per test), and the VOSPipeline frame loop
(hidden states carried across frames) vs the independent CPU oracle pipeline."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _flow(rng, B, H, W, amp):
    return rng.uniform(-amp, amp, (B, 2, H, W)).astype(np.float32)


@pytest.mark.parametrize("B,C,H,W,amp", [(1, 3, 5, 6, 0.0), (2, 5, 9, 13, 2.5),
                                         (2, 256, 16, 28, 4.0), (1, 8, 1, 7, 1.0)])
def test_flow_align_forward_bitexact(B, C, H, W, amp):
    from vosdetectron_amd import ops
    rng = np.random.default_rng(B * 100 + C)
    f = rng.standard_normal((B, C, H, W)).astype(np.float32)
    fl = _flow(rng, B, H, W, amp)
    fl[:, :, ::3] = np.round(fl[:, :, ::3])  # integer displacements: exact taps + borders
    ref = orc.flow_align(f, fl)
    ft, flt = torch.from_numpy(f).to(DEV), torch.from_numpy(fl).to(DEV)
    assert np.array_equal(ops.flow_align(ft, flt).cpu().numpy(), ref)
    if C % 4 == 0:  # NHWC product kernel (channels_last input)
        out = ops.flow_align(ft.contiguous(memory_format=torch.channels_last), flt)
        assert out.is_contiguous(memory_format=torch.channels_last)
        assert np.array_equal(out.contiguous().cpu().numpy(), ref)


def test_flow_align_zero_flow_zeroes_last_row_and_column():
    """The reference's strict `>= H-1` / `>= W-1` test drops the last row/column
    even for zero flow (flow_align_cuda_kernel.cu:33)."""
    from vosdetectron_amd import ops
    f = torch.arange(2 * 4 * 5, dtype=torch.float32, device=DEV).view(1, 2, 4, 5)
    out = ops.flow_align(f, torch.zeros((1, 2, 4, 5), device=DEV))
    assert torch.equal(out[..., :-1, :-1], f[..., :-1, :-1])
    assert float(out[..., -1, :].abs().sum()) == 0 and float(out[..., :, -1].abs().sum()) == 0


def test_flow_align_backward_vs_oracle():
    from vosdetectron_amd import ops
    rng = np.random.default_rng(7)
    f = rng.standard_normal((2, 4, 9, 11)).astype(np.float32)
    fl = _flow(rng, 2, 9, 11, 3.0)
    g = rng.standard_normal(f.shape).astype(np.float32)
    gf_ref, gfl_ref = orc.flow_align_backward(g, f, fl)
    gf, gfl = ops.flow_align_backward(torch.from_numpy(g).to(DEV), torch.from_numpy(f).to(DEV),
                                      torch.from_numpy(fl).to(DEV))
    np.testing.assert_allclose(gf.cpu().numpy(), gf_ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(gfl.cpu().numpy(), gfl_ref, rtol=1e-5, atol=1e-5)


def test_flow_align_module_downsample():
    """FlowAlign module = frozen block-mean conv (scale**3 diag) + the kernel."""
    from vosdetectron_amd.vos import FlowAlign
    rng = np.random.default_rng(3)
    feat = rng.standard_normal((1, 8, 8, 14)).astype(np.float32)
    flow = rng.uniform(-12, 12, (1, 2, 64, 112)).astype(np.float32)
    m = FlowAlign(1. / 8).to(DEV)
    out = m(torch.from_numpy(feat).to(DEV), torch.from_numpy(flow).to(DEV)).cpu().numpy()
    ref = orc.flow_align(feat, orc.flow_downsample(flow, 1. / 8))
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-5)


# --------------------------------------------------------------------------- GN
@pytest.mark.parametrize("cl", [False, True])
@pytest.mark.parametrize("case", ["plain", "relu", "res", "res_up", "res_gn", "x2_sigmoid"])
def test_group_norm_act_vs_torch(cl, case):
    """|GPU - torch fp32| <= 2e-5 (unit-scale data): statistics in double, the
    normalisation in fp32 like torch."""
    from vosdetectron_amd import ops
    g = torch.Generator(device=DEV).manual_seed(11)
    B, C, H, W, G = 3, 64, 10, 14, 32
    x = torch.randn((B, C, H, W), generator=g, device=DEV) * 3 + 1
    gamma = torch.randn(C, generator=g, device=DEV)
    beta = torch.randn(C, generator=g, device=DEV)
    fmt = torch.channels_last if cl else torch.contiguous_format
    xx = x.contiguous(memory_format=fmt)
    ref = F.group_norm(x, G, gamma, beta, 1e-5)
    kw = {}
    if case == "relu":
        ref, kw = F.relu(ref), {"act": "relu"}
    elif case == "res":
        r = torch.randn((B, C, H, W), generator=g, device=DEV)
        ref, kw = F.relu(ref + r), {"act": "relu", "residual": r}
    elif case == "res_up":
        r = torch.randn((B, C, H // 2, W // 2), generator=g, device=DEV)
        ref = ref + F.interpolate(r, scale_factor=2, mode="nearest")
        kw = {"residual": r, "upsample_residual": True}
    elif case == "res_gn":
        r = torch.randn((B, C, H, W), generator=g, device=DEV) * 2
        gr, br = torch.randn(C, generator=g, device=DEV), torch.randn(C, generator=g, device=DEV)
        ref = F.relu(ref + F.group_norm(r, G, gr, br, 1e-5))
        kw = {"act": "relu", "residual": r, "residual_gn": (gr, br)}
    elif case == "x2_sigmoid":
        x2 = torch.randn((B, C, H, W), generator=g, device=DEV)
        ref = torch.sigmoid(F.group_norm(x + x2, G, gamma, beta, 1e-5))
        kw = {"act": "sigmoid", "x2": x2}
    out = ops.group_norm_act(xx, G, gamma, beta, 1e-5, **kw)
    assert out.is_contiguous(memory_format=fmt)
    err = float((out - ref).abs().max())
    assert err <= 2e-5, err


@pytest.mark.parametrize("zero_state", [False, True])
@pytest.mark.parametrize("cl", [False, True])
def test_convgru_fused_vs_module(zero_state, cl):
    """ConvGRUCell2d.fused (HIP gates/update + fusion) vs the reference module math
    on the same device convs, fp32: |diff| <= 1e-5."""
    from vosdetectron_amd.vos import ConvGRUCell2d
    torch.manual_seed(5)
    cell = ConvGRUCell2d(64, 64, GN_groups=32).to(DEV).eval()
    for p in cell.parameters():
        torch.nn.init.normal_(p, 0, 0.05)
    fmt = torch.channels_last if cl else torch.contiguous_format
    if cl:
        cell.to(memory_format=torch.channels_last)
    x = torch.randn((2, 64, 12, 18), device=DEV).contiguous(memory_format=fmt)
    h = None if zero_state else torch.randn_like(x).contiguous(memory_format=fmt)
    finer = torch.randn((2, 64, 24, 36), device=DEV).contiguous(memory_format=fmt)
    with torch.no_grad():
        ref = cell((x, torch.zeros_like(x) if h is None else h))
        ref = ref / 2.0 + F.interpolate(finer, scale_factor=0.5, mode="bilinear",
                                        align_corners=False) / 2.0
        out = cell.fused(x, h, finer)
        out0 = cell.fused(x, h, None)
        ref0 = cell((x, torch.zeros_like(x) if h is None else h))
    assert float((out - ref).abs().max()) <= 1e-5
    assert float((out0 - ref0).abs().max()) <= 1e-5


# --------------------------------------------------------------------------- e2e
@pytest.fixture(scope="module")
def vos_setup():
    from vosdetectron_amd import config as vcfg
    from vosdetectron_amd.engine import VOSPipeline
    from vosdetectron_amd.weights import build_model
    cfg = vcfg.get("vos_R-101-FPN_3x_gn_dynamic_davis")
    cfg.TEST.SCALE = 240  # 240 x 427 frames: identity scale, blob 256 x 448
    frames = [np.random.RandomState(300 + i).randint(0, 256, (240, 427, 3), np.uint8)
              for i in range(3)]
    model, sd = build_model(cfg, device=DEV, channels_last=True, calibrate_frame=frames[0])
    pipe = VOSPipeline(model, cfg, frame_hw=(240, 427), batch=1, device=DEV, channels_last=True)
    return cfg, model, sd, pipe, frames


def _match(gd, gc, gm, sc, bx, cl, masks):
    matched, mask_err = 0, []
    for i in range(len(sc)):
        same = np.where(gc == cl[i])[0]
        if not len(same):
            continue
        b = gd[same, :4]
        xx1 = np.maximum(b[:, 0], bx[i, 0]); yy1 = np.maximum(b[:, 1], bx[i, 1])
        xx2 = np.minimum(b[:, 2], bx[i, 2]); yy2 = np.minimum(b[:, 3], bx[i, 3])
        inter = np.maximum(0, xx2 - xx1 + 1) * np.maximum(0, yy2 - yy1 + 1)
        a1 = (b[:, 2] - b[:, 0] + 1) * (b[:, 3] - b[:, 1] + 1)
        a2 = (bx[i, 2] - bx[i, 0] + 1) * (bx[i, 3] - bx[i, 1] + 1)
        iou = inter / (a1 + a2 - inter)
        j = int(np.argmax(iou))
        if iou[j] > 0.95:
            matched += 1
            mask_err.append(np.abs(gm[same[j]] - masks[i]).max())
    return matched, mask_err


def test_vos_sequence_vs_cpu_oracle(vos_setup):
    """Three frames of one sequence (hidden states carried, dynamic model): the
    fused pyramid, the detections and the class-agnostic 56x56 masks of the
    GPU engine vs the independent CPU pipeline (torch-CPU convs/GroupNorm)."""
    cfg, model, sd, pipe, frames = vos_setup
    from oracle.vos_pipeline import RefCPUVOSPipeline
    torch.set_num_threads(16)
    ref = RefCPUVOSPipeline(sd, target_scale=240, max_size=cfg.TEST.MAX_SIZE)
    pipe.reset()
    for t, fr in enumerate(frames):
        out = pipe.run(torch.from_numpy(fr[None]).to(DEV), keep_intermediates=True)
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
        matched, mask_err = _match(gd, gc, gm, sc, bx, cl, masks)
        print("VOS frame %d: %d/%d matched, count %d" % (t, matched, len(sc), k))
        assert matched >= 0.98 * len(sc), (t, matched, len(sc))
        assert np.median(mask_err) < 2e-3, (t, np.median(mask_err))


def test_vos_batch_rows_are_independent_sequences(vos_setup):
    """Batch row b carries sequence b: two sequences in lockstep give the same
    per-row results as each run alone (frame-sharding across sequences)."""
    cfg, model, sd, _, frames = vos_setup
    from vosdetectron_amd.engine import VOSPipeline
    two = VOSPipeline(model, cfg, frame_hw=(240, 427), batch=2, device=DEV, channels_last=True)
    one = VOSPipeline(model, cfg, frame_hw=(240, 427), batch=1, device=DEV, channels_last=True)
    seq_b = [np.ascontiguousarray(f[::-1]) for f in frames]
    two.reset()
    outs2 = [two.run(torch.from_numpy(np.stack([a, b])).to(DEV), keep_intermediates=True)
             for a, b in zip(frames, seq_b)]
    one.reset()
    outs1 = [one.run(torch.from_numpy(b[None]).to(DEV), keep_intermediates=True) for b in seq_b]
    for o2, o1 in zip(outs2, outs1):
        for f2, f1 in zip(o2["feats"], o1["feats"]):
            rel = float((f2[1] - f1[0]).abs().max() / f1[0].abs().max())
            assert rel < 1e-4, rel
