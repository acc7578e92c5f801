"""Deterministic synthetic weights (no checkpoints ship with the reference and
there is no network).

1. Every parameter of the reference's state_dict is drawn from
   ``numpy.random.default_rng(crc32(name) ^ seed)``: N(0, 1/fan_in) for conv /
   linear weights (fan_in = prod(shape[1:])), zeros for biases, gamma=1 / beta=0
   for AffineChannel2d (SURVEY.md §8d "Weights").
2. Raw random ResNets without normalisation blow activations up (RPN scores
   saturate at 0/1, deltas hit BBOX_XFORM_CLIP and every proposal collapses to
   the image border), which is not the workload a trained detector presents.
   ``calibrate`` therefore runs ONE synthetic frame through the body and sets
   each frozen AffineChannel2d to whiten its input (what a trained BN does) and
   rescales the FPN / RPN convs to unit output; the heads get fixed gains
   (RPN objectness logits ~N(-1.5, 1.5^2), deltas ~0.2, class logits ~3x, mask
   logits ~2x).  The result is a fixed dict that both the HIP engine and the
   CPU oracle pipeline load, so both run the identical network.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch


def synthetic_state_dict(model: torch.nn.Module, seed: int = 0) -> dict:
    sd = {}
    for name, p in model.state_dict().items():
        shape = tuple(p.shape)
        if "conv_flow_downsample" in name:  # frozen, fixed by construction
            sd[name] = p.detach().clone().cpu()
            continue
        is_affine = name.endswith(".weight") and len(shape) == 1
        if is_affine:  # AffineChannel2d scale
            sd[name] = torch.ones(shape)
        elif name.endswith(".bias"):
            sd[name] = torch.zeros(shape)
        else:
            rng = np.random.default_rng(zlib.crc32(name.encode()) ^ seed)
            fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
            w = rng.standard_normal(shape, dtype=np.float32) / np.float32(np.sqrt(fan_in))
            sd[name] = torch.from_numpy(w)
    return sd


@torch.no_grad()
def calibrate(model, frame_u8: np.ndarray, device):
    """Whiten the frozen AffineChannel2d layers and unit-scale the FPN/RPN convs on
    one frame (see module doc).  Mutates ``model`` in place."""
    from .modeling import AffineChannel2d
    means = torch.tensor(model.cfg.PIXEL_MEANS, dtype=torch.float32, device=device)
    im = torch.from_numpy(frame_u8).to(device).float() - means
    H, W = im.shape[:2]
    st = model.cfg.FPN.COARSEST_STRIDE
    Hp, Wp = -(-H // st) * st, -(-W // st) * st
    blob = torch.zeros((1, 3, Hp, Wp), device=device)
    blob[0, :, :H, :W] = im.permute(2, 0, 1)
    hooks = []

    def affine_pre(mod, inp):
        x = inp[0]
        m = x.mean(dim=(0, 2, 3))
        s = x.std(dim=(0, 2, 3)).clamp_min(1e-3)
        mod.weight.copy_(1.0 / s)
        mod.bias.copy_(-m / s)

    def unit_out(target_std=1.0, target_mean=0.0):
        def hook(mod, inp, out):
            if getattr(mod, "_calibrated", False):
                return None
            s = out.std().clamp_min(1e-6)
            g = target_std / s
            mod.weight.mul_(g)
            if mod.bias is not None:
                mod.bias.mul_(g).add_(target_mean - out.mean() * g)
            mod._calibrated = True
            return (out - out.mean()) * g + target_mean
        return hook

    if not model.cfg.FPN.FPN_ON:
        return _calibrate_c4(model, blob[:, :, :H, :W], affine_pre, unit_out)
    for m in model.Conv_Body.conv_body.modules():
        if isinstance(m, AffineChannel2d):
            hooks.append(m.register_forward_pre_hook(affine_pre))
    body = model.Conv_Body
    if not body.use_gn:  # GroupNorm FPN outputs are already unit-scale
        hooks.append(body.conv_top.register_forward_hook(unit_out()))
        for t in body.topdown_lateral_modules:
            hooks.append(t.conv_lateral.register_forward_hook(unit_out()))
        for p in body.posthoc_modules:
            hooks.append(p.register_forward_hook(unit_out()))
    rpn = model.RPN
    hooks.append(rpn.FPN_RPN_conv.register_forward_hook(unit_out()))
    hooks.append(rpn.FPN_RPN_cls_score.register_forward_hook(unit_out(1.5, -1.5)))
    hooks.append(rpn.FPN_RPN_bbox_pred.register_forward_hook(unit_out(0.2)))
    feats = body(blob)
    if hasattr(model, "temporal_fusion"):  # VOS: the RPN sees the ConvGRU-fused pyramid
        feats = model.temporal_fusion(feats, fused=False)
        model.clean_hidden_states()
    rpn.level_outputs(feats[-1])  # calibrate the shared RPN convs on P2
    for h in hooks:
        h.remove()
    for m in model.modules():
        if hasattr(m, "_calibrated"):
            del m._calibrated
    # fixed head gains (inputs are ~unit after the FPN calibration)
    model.Box_Outs.cls_score.weight.mul_(6.0)
    model.Mask_Outs.classify.weight.mul_(4.0)
    return model


@torch.no_grad()
def _calibrate_c4(model, blob, affine_pre, unit_out):
    """C4 family (no FPN): whiten the body's and the res5 head's AffineChannel2d
    (the head on the whole res4 map, a stand-in for its RoI features), unit-scale
    the RPN convs; same head gains as the FPN models."""
    from .modeling import AffineChannel2d
    hooks = []
    for mod in (model.Conv_Body, model.Box_Head.res5):
        for m in mod.modules():
            if isinstance(m, AffineChannel2d):
                hooks.append(m.register_forward_pre_hook(affine_pre))
    rpn = model.RPN
    hooks.append(rpn.RPN_conv.register_forward_hook(unit_out()))
    hooks.append(rpn.RPN_cls_score.register_forward_hook(unit_out(1.5, -1.5)))
    hooks.append(rpn.RPN_bbox_pred.register_forward_hook(unit_out(0.2)))
    res4 = model.Conv_Body(blob)
    rpn.outputs(res4)
    model.Box_Head.res5(res4)
    for h in hooks:
        h.remove()
    for m in model.modules():
        if hasattr(m, "_calibrated"):
            del m._calibrated
    model.Box_Outs.cls_score.weight.mul_(6.0)
    model.Mask_Outs.classify.weight.mul_(4.0)
    return model


def build_model(cfg, seed: int = 0, device="cuda", fold=True, channels_last=False,
                calibrate_frame: np.ndarray | None = None):
    """Generalized_RCNN (Generalized_VOS_RCNN for the VOS configs, i.e. when
    cfg.CONVGRU is set and the config names a VOS model) with synthetic
    (calibrated) weights in eval mode.  Returns (model, state_dict) where
    state_dict has the reference's names and the unfolded AffineChannel
    parameters (what the oracle pipelines load)."""
    from .c4 import Generalized_RCNN_C4
    from .modeling import Generalized_RCNN
    from .vos import Generalized_VOS_RCNN
    vos = bool(cfg.get("VOS", False))
    c4 = not cfg.FPN.FPN_ON
    m = (Generalized_VOS_RCNN if vos else Generalized_RCNN_C4 if c4 else Generalized_RCNN)(cfg)
    sd = synthetic_state_dict(m, seed)
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    m.eval()
    m.to(device)
    for p in m.parameters():
        p.requires_grad_(False)
    if calibrate_frame is None:
        hw = (480, 854) if vos else (800, 1333)
        calibrate_frame = np.random.RandomState(0).randint(0, 256, hw + (3,), np.uint8)
    calibrate(m, calibrate_frame, device)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    if fold:
        m.fold_affine()
    if channels_last:
        m.Conv_Body.to(memory_format=torch.channels_last)
        m.RPN.to(memory_format=torch.channels_last)
        if c4:
            m.Box_Head.to(memory_format=torch.channels_last)
            m.Mask_Head.upconv5.to(memory_format=torch.channels_last)
        else:
            m.Mask_Head.conv_fcn.to(memory_format=torch.channels_last)
        if vos:
            m.ConvGRUs.to(memory_format=torch.channels_last)
    return m, sd
