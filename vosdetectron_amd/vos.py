"""Generalized_VOS_RCNN: the VOS fork's per-frame model with temporal ConvGRU
fusion of the FPN pyramid (lib_vos/vos_modeling/vos_model_builder.py:70-447).

Module tree and parameter names follow the reference (ConvGRUs.i.Wz_h ...,
FlowAligns.i.conv_flow_downsample) so its checkpoints load.  The convolutions
run on PyTorch-ROCm; everything between them is HIP:

  * ConvGRUCell2d (lib_vos/vos_nn/convgrucell.py:14-92): the GroupNorm + sigmoid
    gates and h*r run as vd_convgru_gates, the candidate GroupNorm + tanh, the
    (1-z)h + z h_ update and the pyramid fusion blob/2 + bilinear_0.5x(finer)/2
    (vos_model_builder.py:335-345) as one vd_convgru_update.  A zero hidden state
    (the static model every frame; the first frame of a sequence) skips the four
    convolutions whose outputs are exactly zero (W*h, W*(h*r)) -- same result.
  * FlowAlign (lib_vos/vos_model/flow_align): vd_flow_align_forward warps the
    hidden states by the (downsampled) optical flow.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .modeling import Generalized_RCNN, _conv3x3_mfma, _conv_nb


def _gru_conv(conv, x):
    """A ConvGRU gate conv (3x3, no bias) on the hand-written Winograd kernels where
    they serve it (modeling.conv3x3_route: F(4x4) at the P2 / P3 level sizes), else
    MIOpen (round 6: MIOpen's kernel took 11 ms per P2 gate conv of a 16-frame 480p
    step).  VOSDET_GRU_WINO=0 keeps MIOpen for all of them."""
    import os
    if os.environ.get("VOSDET_GRU_WINO", "1") != "0":
        y = _conv3x3_mfma(conv, x, bias=False, relu=False)
        if y is not None:
            return y
    return _conv_nb(conv, x)


class ConvGRUCell2d(nn.Module):
    """lib_vos/vos_nn/convgrucell.py:14-92 (use_GN=True: bz/br/bh are GroupNorms)."""

    def __init__(self, i_channels, h_channels, kernel_size=3, stride=1, dilation=1, groups=1,
                 use_GN=True, GN_groups=32):
        super().__init__()
        if not use_GN:
            raise NotImplementedError("ConvGRUCell2d(use_GN=False) is not on the VOS configs")
        pad = kernel_size // 2
        conv = lambda ci: nn.Conv2d(ci, h_channels, kernel_size, stride, pad, dilation,  # noqa
                                    groups, bias=False)
        self.Wz_h, self.Wz_x = conv(h_channels), conv(i_channels)
        self.Wr_h, self.Wr_x = conv(h_channels), conv(i_channels)
        self.Wh_h, self.Wh_x = conv(h_channels), conv(i_channels)
        self.bz = nn.GroupNorm(GN_groups, h_channels)
        self.br = nn.GroupNorm(GN_groups, h_channels)
        self.bh = nn.GroupNorm(GN_groups, h_channels)
        self.h_channels = h_channels

    def forward(self, x):
        """Reference semantics, x = (input, hidden_state) (convgrucell.py:73-92)."""
        inp, h = x
        z = torch.sigmoid(self.bz(self.Wz_h(h) + self.Wz_x(inp)))
        r = torch.sigmoid(self.br(self.Wr_h(h) + self.Wr_x(inp)))
        h_ = torch.tanh(self.bh(self.Wh_h(torch.mul(h, r)) + self.Wh_x(inp)))
        return torch.mul(1 - z, h) + torch.mul(z, h_)

    def fused(self, inp, h=None, finer=None):
        """The GRU step + the VOS pyramid fusion on the device.  h None = zero
        state.  Returns hn/2 + bilinear_0.5x(finer)/2 (or hn when finer is None)."""
        g = self.bz.num_groups
        zx = _gru_conv(self.Wz_x, inp)
        hx = _gru_conv(self.Wh_x, inp)
        if h is None:
            z, _ = ops.convgru_gates(zx, None, None, None, None, g, self.bz.weight, self.bz.bias,
                                     self.br.weight, self.br.bias, self.bz.eps)
            return ops.convgru_update(hx, None, z, None, g, self.bh.weight, self.bh.bias,
                                      finer=finer, eps=self.bh.eps)
        rx = _gru_conv(self.Wr_x, inp)
        zh = _gru_conv(self.Wz_h, h)
        rh = _gru_conv(self.Wr_h, h)
        z, hr = ops.convgru_gates(zx, rx, h, zh, rh, g, self.bz.weight, self.bz.bias,
                                  self.br.weight, self.br.bias, self.bz.eps)
        hh = _gru_conv(self.Wh_h, hr)
        return ops.convgru_update(hx, hh, z, h, g, self.bh.weight, self.bh.bias, finer=finer,
                                  eps=self.bh.eps)


class FlowAlign(nn.Module):
    """lib_vos/vos_model/flow_align/modules/flow_align.py:5-37: a frozen 2->2
    conv (kernel = stride = 1/scale, diagonal weight scale**3) brings the
    image-resolution flow to the level, then FlowAlignFunction warps."""

    def __init__(self, spatial_scale):
        super().__init__()
        assert spatial_scale <= 1.0 and spatial_scale in [1.0, 0.5, 0.25, 0.125, 0.0625,
                                                          0.03125, 1. / 64.]
        self.spatial_scale = spatial_scale
        k = int(1.0 / spatial_scale)
        self.conv_flow_downsample = nn.Conv2d(2, 2, k, k, 0, 1, 1, bias=False)
        w = torch.zeros(self.conv_flow_downsample.weight.shape)
        for i in range(2):
            w[i, i] = spatial_scale ** 3
        self.conv_flow_downsample.weight = nn.Parameter(w, requires_grad=False)

    def forward(self, features, flows):
        f = self.conv_flow_downsample(flows) if self.spatial_scale != 1.0 else flows
        return ops.FlowAlignFunction.apply(features, f.contiguous())


class Generalized_VOS_RCNN(Generalized_RCNN):
    """vos_model_builder.py:70-447 (inference).  Inherits the detector (body, RPN,
    heads, roi_feature_transform) and adds the ConvGRUs, the FlowAligns and the
    hidden-state management of the reference (:258-297)."""

    def __init__(self, cfg):
        super().__init__(cfg)
        g = cfg.CONVGRU
        dim = cfg.FPN.DIM
        self.ConvGRUs = nn.ModuleList([
            ConvGRUCell2d(dim, g.HIDDEN_STATE_CHANNELS[i], kernel_size=g.KERNEL_SIZE,
                          stride=g.STRIDE, dilation=g.DILATION, groups=g.GROUPS, use_GN=g.USE_GN,
                          GN_groups=g.GN_GROUPS) for i in range(5)])
        if g.DYNAMIC_MODEL:
            self.fpn_scales = [1. / 64., 1. / 32., 1. / 16., 1. / 8., 1. / 4.]
            self.FlowAligns = nn.ModuleList([FlowAlign(s) for s in self.fpn_scales])
        self.hidden_states = [None] * 5
        self.update_hidden_states = True

    # -- hidden-state management (vos_model_builder.py:258-297) ---------------- #
    def clean_hidden_states(self):
        self.hidden_states = [None] * 5

    def set_update_hidden_states(self, update=True):
        self.update_hidden_states = update

    def temporal_fusion(self, blob_conv, data_flow=None, fused=None):
        """vos_model_builder.py:318-345 on the FPN outputs [P6..P2]: warp the
        hidden states by the flow (dynamic model), run each level's ConvGRU from the
        finest (P2) to the coarsest, fusing each with the bilinear-downsampled finer
        result; the fused levels become the new hidden states (dynamic model)."""
        cfg = self.cfg
        dynamic = cfg.CONVGRU.DYNAMIC_MODEL
        if fused is None:
            fused = blob_conv[0].is_cuda
        hs = self.hidden_states if dynamic else [None] * 5
        if dynamic and data_flow is not None:
            hs = [self.FlowAligns[i](hs[i], data_flow) if hs[i] is not None else None
                  for i in range(5)]
        out = list(blob_conv)
        for i in range(4, -1, -1):
            finer = out[i + 1] if i < 4 else None
            if fused:
                out[i] = self.ConvGRUs[i].fused(out[i], hs[i], finer)
            else:
                h = hs[i] if hs[i] is not None else torch.zeros_like(out[i])
                y = self.ConvGRUs[i]((out[i], h))
                if finer is not None:
                    y = y / 2.0 + F.interpolate(finer, scale_factor=0.5, mode="bilinear",
                                                align_corners=False) / 2.0
                out[i] = y
            if self.update_hidden_states and dynamic:
                self.hidden_states[i] = out[i]
        return out
