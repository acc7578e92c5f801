"""Generalized_RCNN for the per-frame Mask R-CNN hot path on PyTorch-ROCm.

Module tree and parameter names mirror the reference so its state_dicts load
unchanged (lib/modeling/model_builder.py:71-124; ResNet.py; FPN.py;
fast_rcnn_heads.py; mask_rcnn_heads.py).  The dense convolutions and linear
layers stay on PyTorch (MIOpen / hipBLASLt, fp32 -> MFMA); every custom op of the
reference goes through the HIP library:

  * ``roi_feature_transform`` keeps the reference's signature
    (model_builder.py:252-324) and dispatches to ops.RoIAlignFunction /
    RoIPoolFunction / RoICropFunction per level, exactly like the reference;
  * the device-resident engine (engine.py) instead calls ``roi_align_fpn`` once
    over all levels on the NHWC pyramid.

Inference-time MI355X choices: frozen AffineChannel2d is folded into the
preceding conv (``fold_affine``), the RPN's cls/bbox 1x1 convs are fused into one
15-channel conv, and the backbone can run channels_last.
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops


class AffineChannel2d(nn.Module):
    """lib/nn/modules/affine.py:5-17: y = x * weight + bias (frozen BN)."""

    def __init__(self, num_features):
        super().__init__()
        self.num_features = num_features
        self.weight = nn.Parameter(torch.ones(num_features), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(num_features), requires_grad=False)

    def forward(self, x):
        return x * self.weight.view(1, -1, 1, 1) + self.bias.view(1, -1, 1, 1)


def _conv_nb(conv: nn.Conv2d, x):
    """The convolution of `conv` without its bias (added by the fused epilogue):
    the MFMA 3x3 kernel where it applies (_conv3x3_mfma), else MIOpen."""
    y = _conv3x3_mfma(conv, x, bias=False)
    if y is not None:
        return y
    return F.conv2d(x, conv.weight, None, conv.stride, conv.padding, conv.dilation, conv.groups)


def _conv_epi(conv: nn.Conv2d, x, relu=True, res=None, res_bias=None, up=False):
    """conv -> one vd_bias_act pass: act((conv(x) + b) + (res [+ res_bias])).  Same
    association order as the module code it replaces (bias kernel after the MIOpen
    conv, then the residual add, then ReLU), so the results are bit-identical."""
    return ops.bias_act_(_conv_nb(conv, x), conv.bias, res, res_bias, relu=relu,
                         upsample_residual=up)


_CONV3X3_MIN_PIXELS = 1 << 18  # below this CK's kernels fill the chip better
_WINO_MIN_PIXELS = 1 << 12  # res5 / P5 / P6 of a 16-frame batch included (beats MIOpen / CK)
# Winograd workgroups cover 8 x 16 or 4 x 32 output pixels (the kernel takes the
# shape that wastes less): the C4 head's 7 x 7 RoI maps one per block are 49 / 128
# real work, which lost to the implicit GEMM (69 -> 60 frames/s); as a 2-D mosaic of
# 8 x 8-pitch maps they are 77 % real and beat it, 9.99 vs 13.24 ms per 8000-map conv
# (profiles/r03/wino_mosaic2d/odd_shapes_probe.json)
_WINO_MIN_BLOCK_USE = 0.6


def _wino_block_area(H: int, W: int) -> int:
    """Pixels of the Winograd pixel blocks covering an H x W image, for the block
    shape the kernel picks (csrc/conv3x3_wino.hip, launch_conv3x3_wino)."""
    return min(-(-H // br) * br * -(-W // bc) * bc for br, bc in ((8, 16), (4, 32)))


def _wino_block_use(H: int, W: int) -> float:
    """Fraction of the Winograd kernel's pixel blocks that is real output."""
    return H * W / float(_wino_block_area(H, W))


def _mosaic_dims(N: int, H: int, W: int, mos):
    """(rows, columns) of the image the Winograd kernel sees: one map, the maps
    stacked (mosaic rows), or g = 16 / gcd(W', 16) maps of H' x W' side by side per
    mosaic row, H' / W' = H / W rounded up to even (launch_conv3x3_wino_mosaic)."""
    if mos == "2d":
        ph, pw = H + H % 2, W + W % 2
        g = min(16 // math.gcd(pw, 16), N)
        return -(-N // g) * ph, g * pw
    return (N * H, W) if mos else (H, W)


def _pick_mosaic(N: int, H: int, W: int, allow=True):
    """The Winograd layout of a batch with the most real output per pixel block:
    one launch over the N images as they are (False), stacked in one column (True),
    or tiled 2-D ("2d"); ties keep the simpler layout.  VOSDET_WINO_MOSAIC: 0 off,
    1 rows at most, 2 (default) any."""
    env = os.environ.get("VOSDET_WINO_MOSAIC", "2")
    best = (False, _wino_block_use(H, W))
    if not allow or env == "0" or N < 2:
        return best
    cands = ([True] if H % 2 == 0 else []) + (["2d"] if env == "2" else [])
    for m in cands:  # real pixels over block pixels (phantom rows / columns are waste)
        u = N * H * W / float(_wino_block_area(*_mosaic_dims(N, H, W, m)))
        if u > best[1] + 1e-9:
            best = (m, u)
    return best


# Winograd F(4x4,3x3) (csrc/conv3x3_wino4.hip): 16 x 32-pixel x 64-channel workgroups,
# one per CU (120 KiB of LDS), 1.78x fewer MFMA multiplies than F(2x2).  Faster than
# F(2x2) on every 32-frame step shape with >= 4 workgroups per CU and blocks >= 50 %
# real output (profiles/r05/wino4/ab_v3.jsonl: P2 7.41 vs 9.31 ms, P3 2.13 vs 2.61,
# P4 0.65 vs 0.81, res2 0.63 vs 0.85, res5 0.79 vs 0.91); below that its coarse blocks
# leave CUs idle.  The mask head's 14 x 14 RoI maps run two per block (_wino4_pair_ok).
_WINO4_MIN_WGS = 1024
_WINO4_MIN_BLOCK_USE = 0.5


def _wino4_block_use(H: int, W: int) -> float:
    """Fraction of the F(4x4) kernel's 16 x 32 output-pixel blocks that is real output."""
    return H * W / float(-(-H // 16) * 16 * -(-W // 32) * 32)


def _wino4_rows_use(N: int, H: int, W: int) -> float:
    """Real-output share of the F(4x4) blocks over the row stack (maps at a pitch of
    H + 1 rounded up to 4 rows, vd_conv3x3_wino4_rows_bias_act)."""
    hp = (H + 4) // 4 * 4
    return N * H * W / float(-(-N * hp // 16) * 16 * -(-W // 32) * 32)


def _wino4_mode(N: int, Cin: int, Cout: int, H: int, W: int):
    """conv3x3_route's F(4x4) gate: None (not F(4x4)), False (one map per block
    column) or "rows" (the row stack, where it wastes less of the blocks: 50 x 84 maps
    84 % vs 68 %, 25 x 42 59 % vs 51 %; VOSDET_WINO4_ROWS=0 turns it off).
    VOSDET_WINO4=0 turns F(4x4) off."""
    if os.environ.get("VOSDET_WINO4", "1") == "0":
        return None
    if Cout % 64 or Cin % 8 or Cout == 0 or Cin == 0 or Cin > ops.WINO_MAX_CIN:
        return None
    if H * W * Cin >= (1 << 31):
        return None
    use = _wino4_block_use(H, W)
    wgs = N * -(-H // 16) * -(-W // 32) * (Cout // 64)
    plain = wgs >= _WINO4_MIN_WGS and use >= _WINO4_MIN_BLOCK_USE
    if (os.environ.get("VOSDET_WINO4_ROWS", "1") != "0" and N > 1
            and N * H * W * Cin < (1 << 31)):
        # measured (profiles/r05/wino4_rows/): P3 2.09 -> 2.00 ms, P4 0.63 -> 0.53, res3
        # 0.64 -> 0.60, res5 0.79 -> 0.75 (896 workgroups, fewer than one map per block
        # column gives, and still faster)
        ru = _wino4_rows_use(N, H, W)
        rwgs = -(-N * ((H + 4) // 4 * 4) // 16) * -(-W // 32) * (Cout // 64)
        # (P2 200 x 336: 0.918 -> 0.936, 7.15 -> 7.11 ms, res2 0.64 -> 0.64 ms)
        if (ru > use + 0.015 and ru >= _WINO4_MIN_BLOCK_USE
                and (rwgs >= _WINO4_MIN_WGS or (plain and rwgs >= _WINO4_MIN_WGS // 2))):
            return "rows"
    return False if plain else None


def _wino4_ok(N: int, Cin: int, Cout: int, H: int, W: int) -> bool:
    """conv3x3_route's F(4x4) gate (VOSDET_WINO4=0 turns it off)."""
    return _wino4_mode(N, Cin, Cout, H, W) is not None


def _wino4_pair_ok(N: int, Cin: int, Cout: int, H: int, W: int) -> bool:
    """F(4x4) over small maps two per 16 x 32 block (vd_conv3x3_wino4_mosaic_bias_act;
    the mask head's 14 x 14 RoI maps: 77 % of each block real output; 2.43 vs 2.87 ms
    per 3200-map conv for F(2x2) on its 2-D mosaic, profiles/r05/wino4_pair/).  Maps
    of at most 7 x 7 (C4's res5 head) run eight per block in 8 x 8 cells
    (VOSDET_WINO4_OCTET=0 keeps them on the F(2x2) mosaic).  VOSDET_WINO4_MOSAIC=0
    turns both off."""
    if os.environ.get("VOSDET_WINO4_MOSAIC", "1") == "0" or os.environ.get("VOSDET_WINO4", "1") == "0":
        return False
    if Cout % 64 or Cin % 8 or Cout == 0 or Cin == 0 or Cin > ops.WINO_MAX_CIN:
        return False
    cell, per = (8, 8) if (H <= 7 and W <= 7) else (16, 2)  # octets / pairs per block
    if cell == 8 and os.environ.get("VOSDET_WINO4_OCTET", "1") == "0":
        return False
    if H > 15 or W > 15 or per * H * W * Cin >= (1 << 31) or H * W < 0.5 * cell * cell:
        return False
    return -(-N // per) * (Cout // 64) >= _WINO4_MIN_WGS


def _wino4_grid_blocks(N: int, H: int, W: int) -> int:
    """16 x 32 output blocks of the F(4x4) grid layout (launch_conv3x3_wino4, mos 4):
    maps at an (H + 1) x (W + 1) pitch, g per grid row for the fewest blocks."""
    return min(-(-(-(-N // g) * (H + 1)) // 16) * -(-(g * (W + 1)) // 32)
               for g in range(1, min(64, N) + 1))


def _wino4_grid_better(N: int, Cin: int, H: int, W: int) -> bool:
    """The map-pair / octet mosaic's maps as a shared-separator grid instead, where
    that needs fewer blocks (14 x 14 RoI maps: 1410 vs 1600 blocks per 3200 maps).
    VOSDET_WINO4_GRID=0 keeps pairs / octets."""
    if (os.environ.get("VOSDET_WINO4_GRID", "1") == "0" or N * H * W * Cin >= (1 << 31)
            or H > 255 or W > 255):
        return False
    cells = -(-N // 8) if (H <= 7 and W <= 7) else -(-N // 2)
    return _wino4_grid_blocks(N, H, W) < cells


def conv3x3_route(N: int, Cin: int, Cout: int, H: int, W: int, mosaic=True):
    """(algorithm, mosaic) the engine runs a 3x3 / stride-1 / pad-1 fp32 conv of an
    N x Cin x H x W channels_last batch with: ('wino4', None) -- Winograd F(4x4,3x3),
    csrc/conv3x3_wino4.hip, where _wino4_ok holds -- else ('wino', layout) -- Winograd
    F(2x2,3x3), csrc/conv3x3_wino.hip, from 2^12 output pixels where its blocks are
    >= 60 % real output (Cout % 64, Cin % 8) -- else ('igemm', None), the implicit
    GEMM (csrc/conv3x3.hip), from 2^18 pixels, else (None, None): MIOpen / CK.
    One rule for the engine (_conv3x3_mfma) and the bench's executed-FLOP count."""
    npx = N * H * W
    mos, use = _pick_mosaic(N, H, W, mosaic)
    wino = (os.environ.get("VOSDET_CONV3X3_ALGO", CONV3X3_ALGO) == "wino" and Cout % 64 == 0
            and Cin % 8 == 0 and Cout > 0 and Cin <= ops.WINO_MAX_CIN)
    w4 = _wino4_mode(N, Cin, Cout, H, W) if wino else None
    if w4 is not None:
        return "wino4", (w4 or None)
    if wino and mosaic and _wino4_pair_ok(N, Cin, Cout, H, W):
        return "wino4", ("grid" if _wino4_grid_better(N, Cin, H, W) else "pair")
    if wino and npx >= _WINO_MIN_PIXELS and use >= _WINO_MIN_BLOCK_USE:
        return "wino", mos
    if npx < _CONV3X3_MIN_PIXELS:
        # below the implicit GEMM's range the alternative is MIOpen, whose small-map
        # solvers split K with atomics (igemm_fwd_gtcx35_..._gkgs): a 3-frame step's
        # P6 RPN conv differed run to run.  Winograd is deterministic, and at these
        # sizes its idle block share costs microseconds.
        return ("wino", mos) if wino else (None, None)
    return "igemm", None


def conv3x3_grouped_route(N: int, C: int, Cout: int, H: int, W: int, groups: int):
    """The layout a grouped 3x3 / stride-1 conv (ResNeXt's conv2) runs with on the
    F(4x4) kernel's grouped form (each 64-channel output block reading the 64 input
    channels of its groups, the weight block-diagonal: 64 / (C / groups) x the
    multiplies of the grouped conv, still fewer than MIOpen / CK spend on these
    shapes): False (plain) or "rows" -- the dense rule of _wino4_mode -- or None (not
    served: C != Cout, C / groups not dividing 64, small batches; VOSDET_WINO4_GROUPED=0)."""
    if os.environ.get("VOSDET_WINO4_GROUPED", "1") == "0" or groups < 2:
        return None
    if C != Cout or C % 64 or C % groups or 64 % (C // groups):
        return None
    return _wino4_mode(N, C, Cout, H, W)


# conv3x3 launches per route since the last reset (host-side, also counted while a
# hipGraph is captured): 'wino4', 'wino', 'wino_rows', 'wino_2d', 'igemm', 'miopen'
ROUTE_COUNTS = {}


def _count_route(name: str):
    ROUTE_COUNTS[name] = ROUTE_COUNTS.get(name, 0) + 1


def _dilated2_ok(conv: nn.Conv2d, x) -> bool:
    """A 3x3 / dilation-2 / pad-2 conv (the VOS mask head, MRCNN.DILATION = 2) of
    even-sized channels_last maps, which _conv3x3_mfma runs as the plain 3x3 conv of
    its four polyphase sub-maps (VOSDET_WINO_DILATED=0 keeps MIOpen)."""
    return (conv.dilation == (2, 2) and conv.padding == (2, 2) and conv.stride == (1, 1)
            and conv.kernel_size == (3, 3) and conv.groups == 1 and x.dim() == 4
            and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0 and x.is_cuda
            and x.dtype == torch.float32 and x.is_contiguous(memory_format=torch.channels_last)
            and os.environ.get("VOSDET_WINO_DILATED", "1") != "0"
            and os.environ.get("VOSDET_CONV3X3_MFMA", "1") != "0")


def _conv3x3_mfma(conv: nn.Conv2d, x, bias=True, relu=False, mosaic=True):
    """conv (3x3, stride 1, pad 1) of a channels_last fp32 tensor on the
    hand-written MFMA kernels with the bias (+ ReLU) epilogue, or None where
    they do not apply (other geometry, VOSDET_CONV3X3_MFMA=0).  The algorithm
    is conv3x3_route's.  mosaic=True lets Winograd run the batch as a mosaic of
    maps with per-map zero padding (_pick_mosaic): the mask head's 14 x 14 RoI
    maps 8 side by side per 112-column row -- every 8 x 16-pixel block real
    output (77 % one map per block, 87.5 % stacked in one column) -- and the
    16-frame P3 / P4 maps 2 / 4 per row; bit-identical results.  The transformed
    weights are cached on the module.  A dilation-2 / pad-2 3x3 conv of even-sized
    maps (round 6) is the plain pad-1 conv of its four polyphase sub-maps -- output
    (2i + a, 2j + b) reads only inputs of parity (a, b), the dilated taps are that
    sub-map's neighbours and its zero padding is one sub-pixel: space-to-batch, the
    same kernels on 4N maps of H/2 x W/2 (the VOS mask head's 14 x 14 RoI maps become
    7 x 7 octets), batch-to-space."""
    if _dilated2_ok(conv, x):
        N, C, H, W = x.shape
        algo, mos = conv3x3_route(4 * N, C, conv.weight.shape[0], H // 2, W // 2, mosaic)
        if (algo == "wino4" and mos in ("pair", "grid", None)
                and os.environ.get("VOSDET_DILATED_INPLACE", "1") != "0"):
            # the kernel reads / writes the sub-maps in place: no polyphase copies
            w = conv.weight
            key = (w.data_ptr(), w._version)
            if getattr(conv, "_vd_u4_key", None) != key:
                conv._vd_u4 = ops.conv3x3_wino4_weight(w.detach())
                conv._vd_u4_key = key
            b = conv.bias.detach() if (bias and conv.bias is not None) else None
            y = ops.conv3x3_wino4_dilated2_bias_act(x, conv._vd_u4, b, relu=relu,
                                                    layout=mos or False)
            if y is not None:
                _count_route("dilated2")
                return y
        xs = x.permute(0, 2, 3, 1).reshape(N, H // 2, 2, W // 2, 2, C).permute(
            2, 4, 0, 1, 3, 5).reshape(4 * N, H // 2, W // 2, C).permute(0, 3, 1, 2)
        y = _conv3x3_mfma_core(conv, xs, bias, relu, mosaic, as_plain=True)
        if y is None:
            return None
        Co = y.shape[1]
        y = y.permute(0, 2, 3, 1).reshape(2, 2, N, H // 2, W // 2, Co).permute(
            2, 3, 0, 4, 1, 5).reshape(N, H, W, Co).permute(0, 3, 1, 2)
        _count_route("dilated2")
        return y
    return _conv3x3_mfma_core(conv, x, bias, relu, mosaic)


def _conv3x3_mfma_core(conv: nn.Conv2d, x, bias=True, relu=False, mosaic=True,
                       as_plain=False):
    """_conv3x3_mfma's body; as_plain: a dilation-2 / pad-2 conv taken as the pad-1 conv
    it is on polyphase sub-maps (the caller has split x)."""
    dil = (1, 1) if as_plain else conv.dilation
    pad = (1, 1) if as_plain else conv.padding
    if (conv.groups > 1 and os.environ.get("VOSDET_CONV3X3_MFMA", "1") != "0" and x.is_cuda
            and conv.kernel_size == (3, 3) and conv.stride == (1, 1) and pad == (1, 1)
            and dil == (1, 1) and x.dtype == torch.float32
            and x.is_contiguous(memory_format=torch.channels_last)):
        mode = conv3x3_grouped_route(x.shape[0], x.shape[1], conv.weight.shape[0], x.shape[2],
                                     x.shape[3], conv.groups)
        if mode is not None:
            w = conv.weight
            key = (w.data_ptr(), w._version)
            if getattr(conv, "_vd_u4g_key", None) != key:
                conv._vd_u4g = ops.conv3x3_wino4_grouped_weight(w.detach(), conv.groups)
                conv._vd_u4g_key = key
            b = conv.bias.detach() if (bias and conv.bias is not None) else None
            if conv._vd_u4g is not None:
                y = ops.conv3x3_wino4_bias_act(x, conv._vd_u4g, b, relu=relu,
                                               mosaic=mode or False, groups=conv.groups)
                if y is not None:
                    _count_route("wino4_grouped")
                    return y
    if (os.environ.get("VOSDET_CONV3X3_MFMA", "1") == "0" or not x.is_cuda
            or conv.kernel_size != (3, 3) or conv.stride != (1, 1) or pad != (1, 1)
            or dil != (1, 1) or conv.groups != 1 or x.dtype != torch.float32
            or not x.is_contiguous(memory_format=torch.channels_last)):
        if conv.kernel_size == (3, 3):
            _count_route("miopen")
        return None
    w = conv.weight
    key = (w.data_ptr(), w._version)
    b = conv.bias.detach() if (bias and conv.bias is not None) else None
    algo, mos = conv3x3_route(x.shape[0], x.shape[1], w.shape[0], x.shape[2], x.shape[3],
                              mosaic)
    if algo == "wino4":
        if getattr(conv, "_vd_u4_key", None) != key:
            conv._vd_u4 = ops.conv3x3_wino4_weight(w.detach())
            conv._vd_u4_key = key
        y = ops.conv3x3_wino4_bias_act(x, conv._vd_u4, b, relu=relu, mosaic=mos or False)
        if y is not None:
            _count_route({"pair": "wino4_pair", "rows": "wino4_rows",
                          "grid": "wino4_grid"}.get(mos, "wino4"))
            return y
        algo, mos = "wino", _pick_mosaic(x.shape[0], x.shape[2], x.shape[3], mosaic)[0]
    if algo == "wino":
        if getattr(conv, "_vd_u_key", None) != key:
            conv._vd_u = ops.conv3x3_wino_weight(w.detach())
            conv._vd_u_key = key
        y = ops.conv3x3_wino_bias_act(x, conv._vd_u, b, relu=relu, mosaic=mos)
        if y is not None:
            _count_route({False: "wino", True: "wino_rows", "2d": "wino_2d"}[mos])
            return y
        algo = "igemm" if x.shape[0] * x.shape[2] * x.shape[3] >= _CONV3X3_MIN_PIXELS else None
    if algo is None:
        _count_route("miopen")
        return None
    if getattr(conv, "_vd_w2_key", None) != key:
        conv._vd_w2 = ops.conv3x3_weight(w.detach())
        conv._vd_w2_key = key
    y = ops.conv3x3_bias_act(x, conv._vd_w2, b, relu=relu)
    _count_route("igemm" if y is not None else "miopen")
    return y


CONV3X3_ALGO = "wino"  # the 3x3 algorithm the engine uses (VOSDET_CONV3X3_ALGO overrides)


def _stage_counts(conv_body: str):
    return {"FPN.fpn_ResNet50_conv5_body": (3, 4, 6, 3),
            "FPN.fpn_ResNet101_conv5_body": (3, 4, 23, 3),
            "FPN.fpn_ResNet152_conv5_body": (3, 8, 36, 3)}[conv_body]


class Bottleneck(nn.Module):
    """ResNet.py bottleneck_transformation (STRIDE_1X1 -> stride on the 1x1)."""

    def __init__(self, inplanes, outplanes, innerplanes, stride, group, stride_1x1=True):
        super().__init__()
        s1, s3 = (stride, 1) if stride_1x1 else (1, stride)
        self.conv1 = nn.Conv2d(inplanes, innerplanes, 1, s1, bias=False)
        self.bn1 = AffineChannel2d(innerplanes)
        self.conv2 = nn.Conv2d(innerplanes, innerplanes, 3, s3, 1, bias=False, groups=group)
        self.bn2 = AffineChannel2d(innerplanes)
        self.conv3 = nn.Conv2d(innerplanes, outplanes, 1, 1, bias=False)
        self.bn3 = AffineChannel2d(outplanes)
        self.downsample = None
        if stride != 1 or inplanes != outplanes:
            self.downsample = nn.Sequential(nn.Conv2d(inplanes, outplanes, 1, stride, bias=False),
                                            AffineChannel2d(outplanes))
        self.fused = False
        self.epilogue = False

    def forward(self, x):
        if self.fused and self.epilogue and x.is_cuda:
            if _gemm_ok(x):
                return self._forward_gemm(x)
            out = _conv_epi(self.f1, x)
            out = _conv_epi(self.f2, out)
            if self.downsample is not None:
                return _conv_epi(self.f3, out, res=_conv_nb(self.fd, x), res_bias=self.fd.bias)
            return _conv_epi(self.f3, out, res=x)
        if self.fused:
            out = F.relu(self.f1(x), inplace=True)
            out = F.relu(self.f2(out), inplace=True)
            out = self.f3(out)
            res = self.fd(x) if self.downsample is not None else x
            return F.relu_(out.add_(res))
        out = F.relu(self.bn1(self.conv1(x)), inplace=True)
        out = F.relu(self.bn2(self.conv2(out)), inplace=True)
        out = self.bn3(self.conv3(out))
        res = self.downsample(x) if self.downsample is not None else x
        return F.relu(out + res, inplace=True)


    def _forward_gemm(self, x):
        """channels_last: the stride-1 1x1 convs run as hipBLASLt GEMMs with their
        epilogue fused -- conv1: relu(x W1^T + b1); conv3: relu(h W3^T + b3 + r)
        with the residual r (identity, or the downsample conv whose bias is
        folded into b3) read by the GEMM itself (ops.gemm_bias_act)."""
        # a stage's first block (stride 2 on the 1x1s): the strided 1x1 convs are
        # GEMMs over the every-other-pixel copy of x (a quarter of its bytes, one
        # copy kernel) instead of MIOpen / CK strided convs: 2.78 -> 2.27 ms per
        # 16-frame step over res3-res5 (profiles/r04/stride2/ab.jsonl)
        xs = None
        strided = self.downsample is not None and self.fd.stride != (1, 1) and _is_1x1(self.fd)
        # round 6: the split-bf16 GEMM reads x at stride 2 itself (no subsampled copy)
        s2 = strided and self.fd.stride == (2, 2) and _split3_s2_ok(x, self.wd)
        if strided and not s2:
            xs = _subsample(x, self.fd.stride)
        out = None
        if self.f1.stride == (1, 1):
            out = _gemm_conv1x1(x, self.w1, self.f1.bias, relu=True)
        elif s2 and self.f1.stride == (2, 2) and _is_1x1(self.f1) and _split3_s2_ok(x, self.w1):
            out = _gemm_conv1x1_s2(x, self.w1, self.f1.bias, relu=True)
        elif strided and self.f1.stride == self.fd.stride and _is_1x1(self.f1):
            if xs is None:
                xs = _subsample(x, self.fd.stride)
            out = _gemm_conv1x1(xs, self.w1, self.f1.bias, relu=True)
        if out is None:
            out = _conv_epi(self.f1, x)
        y = _conv3x3_mfma(self.f2, out, relu=True)  # res2 / res3 3x3s (>= 2^18 px)
        pre = None  # conv2's bias, applied (+ ReLU) by conv3's split GEMM as it loads A
        if y is not None:
            out = y
        elif _conv2_prologue_ok(self.f2, self.w3):
            # ResNeXt's grouped conv2 (MIOpen, no epilogue): its bias + ReLU ride on
            # conv3's A load instead of a separate pass over the conv2 output
            out, pre = _conv_nb(self.f2, out), self.f2.bias
        else:
            out = _conv_epi(self.f2, out)
        if self.downsample is not None:
            if self.fd.stride == (1, 1) and x.is_contiguous(memory_format=torch.channels_last):
                # conv3 and the stride-1 downsample as one two-operand MFMA GEMM
                N, _, H, W = out.shape
                K = self.w3d.shape[1]
                if ops.split3_enabled() and K >= ops.SPLIT3_MIN_K and K % 16 == 0 and \
                        out.shape[1] % 16 == 0 and self.w3d.shape[0] % 64 == 0:
                    # round 6: on the bf16 matrix cores at fp32 accuracy (split GEMM, A2)
                    y = ops.gemm_split3_bias_act(_nhwc2d(out), ops.split3_weight_cached(self.w3d),
                                                 self.b3d, a2=_nhwc2d(x), a_bias=pre)
                else:
                    if pre is not None:
                        out, pre = ops.bias_act_(out, pre, relu=True), None
                    y = ops.gemm_dual_bias_act(_nhwc2d(out), _nhwc2d(x), self.w3d, self.b3d)
                if y is not None:
                    return y.view(N, H, W, -1).permute(0, 3, 1, 2)
            if s2:  # relu(h W3^T + b3 + (x[::2, ::2] Wd^T + bd))
                r = _gemm_conv1x1_s2(x, self.wd, self.fd.bias, relu=False)
                return _gemm_conv1x1(out, self.w3, self.f3.bias, relu=True, res=r, a_bias=pre)
            if xs is not None:  # relu(h W3^T + b3 + (xs Wd^T + bd))
                r = _gemm_conv1x1(xs, self.wd, self.fd.bias, relu=False)
                return _gemm_conv1x1(out, self.w3, self.f3.bias, relu=True, res=r, a_bias=pre)
            return _gemm_conv1x1(out, self.w3, self.b3d, relu=True, res=_conv_nb(self.fd, x),
                                 a_bias=pre)
        return _gemm_conv1x1(out, self.w3, self.f3.bias, relu=True, res=x, a_bias=pre)


def _is_1x1(conv: nn.Conv2d) -> bool:
    return conv.kernel_size == (1, 1) and conv.padding == (0, 0) and conv.groups == 1


def _subsample(x, stride):
    """x[:, :, ::sh, ::sw] as a channels_last tensor: the pixels a pad-0 strided 1x1
    conv reads (output size ceil(H / s), as the conv's)."""
    return x[:, :, ::stride[0], ::stride[1]].contiguous(memory_format=torch.channels_last)


def _split3_s2_ok(x, w2d) -> bool:
    """A stride-2 1x1 conv of x runs as a split-bf16 GEMM reading x at stride 2."""
    return (ops.split3_enabled() and x.shape[1] >= ops.SPLIT3_MIN_K and x.shape[1] % 16 == 0
            and w2d.shape[0] % 64 == 0 and _gemm_ok(x))


def _gemm_conv1x1_s2(x, w2d, bias, relu=True, res=None):
    """Stride-2 pad-0 1x1 conv of a channels_last NCHW tensor as act(x[::2, ::2] W^T + b
    [+ res]) in one split-bf16 GEMM that reads x at stride 2 (no subsampled copy)."""
    N, C, H, W = x.shape
    wp = ops.split3_weight_cached(w2d)
    r = None
    if res is not None:
        r = _nhwc2d(res.contiguous(memory_format=torch.channels_last))
    y = ops.gemm_split3_bias_act(_nhwc2d(x), wp, bias, residual=r, relu=relu, sub_hw=(H, W))
    return y.view(N, (H + 1) // 2, (W + 1) // 2, w2d.shape[0]).permute(0, 3, 1, 2)


def _gemm_ok(x) -> bool:
    """GEMM epilogue path: channels_last fp32 activations (VOSDET_GEMM_EPILOGUE=0
    switches it off for A/B measurements)."""
    import os
    return (os.environ.get("VOSDET_GEMM_EPILOGUE", "1") != "0" and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous()
            and x.dtype == torch.float32)


def _nhwc2d(x):
    N, C, H, W = x.shape
    return x.permute(0, 2, 3, 1).reshape(N * H * W, C)


def _conv2_prologue_ok(conv2: nn.Conv2d, w3) -> bool:
    """A grouped conv2 (ResNeXt, on MIOpen) whose bias + ReLU conv3's split-bf16 GEMM
    applies as it loads its input (ops.gemm_split3_bias_act a_bias), instead of a
    separate pass: conv3 must take the split GEMM (K = conv2's channels >= SPLIT3_MIN_K,
    K % 16, N % 64).  VOSDET_CONV2_PROLOGUE=0 keeps the separate pass."""
    import os
    k = conv2.out_channels
    return (conv2.groups > 1 and conv2.bias is not None and ops.split3_enabled()
            and k >= ops.SPLIT3_MIN_K and k % 16 == 0 and w3.shape[0] % 64 == 0
            and w3.shape[1] == k and os.environ.get("VOSDET_CONV2_PROLOGUE", "1") != "0")


def _gemm_conv1x1(x, w2d, bias, relu=True, res=None, a_bias=None):
    """Stride-1 1x1 conv of a channels_last NCHW tensor as act(X W^T + b [+ res]);
    a_bias: X enters as relu(X + a_bias) (the producing conv's epilogue, fused)."""
    N, C, H, W = x.shape
    r = None
    if res is not None:
        if not res.is_contiguous(memory_format=torch.channels_last):
            res = res.contiguous(memory_format=torch.channels_last)
        r = _nhwc2d(res)
    y = ops.gemm_bias_act(_nhwc2d(x), w2d, bias, residual=r, relu=relu, a_bias=a_bias)
    if y is None:  # no GEMM algorithm for the shape: MIOpen's 1x1 conv + torch epilogue
        if a_bias is not None:
            x = ops.bias_act_(x, a_bias, relu=True)
        y = F.conv2d(x, w2d.view(w2d.shape[0], C, 1, 1), bias)
        if res is not None:
            y = y + res
        return F.relu(y) if relu else y
    return y.view(N, H, W, w2d.shape[0]).permute(0, 3, 1, 2)


def group_gn(dim: int, cfg) -> int:
    """utils/net.py get_group_gn (:208-226)."""
    dpg, ng = cfg.GROUP_NORM.DIM_PER_GP, cfg.GROUP_NORM.NUM_GROUPS
    assert dpg == -1 or ng == -1, "GroupNorm: can only specify G or C/G."
    if dpg > 0:
        assert dim % dpg == 0
        return dim // dpg
    assert dim % ng == 0
    return ng


def _gn(dim: int, cfg) -> nn.GroupNorm:
    return nn.GroupNorm(group_gn(dim, cfg), dim, eps=cfg.GROUP_NORM.EPSILON)


def _gn_conv1x1(conv: nn.Conv2d, x):
    """A GN model's bias-free 1x1 conv (stride 1, or 2 read in place) as a split-bf16
    GEMM (a zero bias; the GroupNorm follows), or None where the GEMM does not serve it
    (MIOpen then: with its NHWC layout copies around a CK kernel, round 6's VOS trace)."""
    if (not _is_1x1(conv) or conv.bias is not None or not x.is_cuda
            or x.dtype != torch.float32 or not x.is_contiguous(memory_format=torch.channels_last)
            or not ops.split3_enabled()):
        return None
    w = conv.weight
    if getattr(conv, "_vd_gn_src", None) is not w:
        conv._vd_gn_w2d = w.detach().reshape(w.shape[0], -1)
        conv._vd_gn_zb = torch.zeros(w.shape[0], dtype=w.dtype, device=w.device)
        conv._vd_gn_src = w
    w2d = conv._vd_gn_w2d
    K, N = w2d.shape[1], w2d.shape[0]
    if K < ops.SPLIT3_MIN_K or K % 16 or N % 64 or x.shape[1] != K:
        return None
    if conv.stride == (1, 1):
        return _gemm_conv1x1(x, w2d, conv._vd_gn_zb, relu=False)
    if conv.stride == (2, 2) and _split3_s2_ok(x, w2d):
        return _gemm_conv1x1_s2(x, w2d, conv._vd_gn_zb, relu=False)
    return None


def _gn_epi(conv: nn.Conv2d, gn: nn.GroupNorm, x, act="relu", res=None, res_gn=None, up=False):
    """conv (no bias) -> one vd_group_norm_act: act(GN(conv(x)) + res), the residual
    optionally normalised by its own GroupNorm (res_gn) or nearest-2x upsampled.  A
    3x3 / stride-1 conv takes the hand-written Winograd kernels where they serve it
    (conv3x3_route; VOSDET_GN_WINO=0 keeps MIOpen)."""
    y = None
    if os.environ.get("VOSDET_GN_WINO", "1") != "0":
        y = _conv3x3_mfma(conv, x, bias=False, relu=False)
    if y is None and os.environ.get("VOSDET_GN_GEMM", "1") != "0":
        y = _gn_conv1x1(conv, x)
    if y is None:
        y = _conv_nb(conv, x)
    return ops.group_norm_act(y, gn.num_groups, gn.weight, gn.bias, gn.eps, residual=res,
                              residual_gn=(res_gn.weight, res_gn.bias) if res_gn is not None
                              else None, upsample_residual=up, act=act, out=y)


class BottleneckGN(nn.Module):
    """ResNet.py bottleneck_gn_transformation (:296-345) with basic_gn_shortcut
    (:208-218).  GPU path: each conv's GroupNorm (+ shortcut GroupNorm, residual
    add, ReLU) runs as one vd_group_norm_act."""

    def __init__(self, inplanes, outplanes, innerplanes, stride, group, stride_1x1, cfg):
        super().__init__()
        s1, s3 = (stride, 1) if stride_1x1 else (1, stride)
        self.conv1 = nn.Conv2d(inplanes, innerplanes, 1, s1, bias=False)
        self.gn1 = _gn(innerplanes, cfg)
        self.conv2 = nn.Conv2d(innerplanes, innerplanes, 3, s3, 1, bias=False, groups=group)
        self.gn2 = _gn(innerplanes, cfg)
        self.conv3 = nn.Conv2d(innerplanes, outplanes, 1, 1, bias=False)
        self.gn3 = _gn(outplanes, cfg)
        self.downsample = None
        if stride != 1 or inplanes != outplanes:
            self.downsample = nn.Sequential(nn.Conv2d(inplanes, outplanes, 1, stride, bias=False),
                                            _gn(outplanes, cfg))
        self.epilogue = False

    def forward(self, x):
        if self.epilogue and x.is_cuda:
            out = _gn_epi(self.conv1, self.gn1, x)
            out = _gn_epi(self.conv2, self.gn2, out)
            if self.downsample is not None:
                return _gn_epi(self.conv3, self.gn3, out, res=_conv_nb(self.downsample[0], x),
                               res_gn=self.downsample[1])
            return _gn_epi(self.conv3, self.gn3, out, res=x)
        out = F.relu(self.gn1(self.conv1(x)), inplace=True)
        out = F.relu(self.gn2(self.conv2(out)), inplace=True)
        out = self.gn3(self.conv3(out))
        res = self.downsample(x) if self.downsample is not None else x
        return F.relu(out + res, inplace=True)


class _StemGN(nn.Module):
    """basic_gn_stem (ResNet.py:233-241) with the GroupNorm + ReLU fused."""

    def __init__(self, conv1, gn1, maxpool):
        super().__init__()
        self.conv1, self.gn1, self.maxpool = conv1, gn1, maxpool

    def forward(self, x):
        if x.is_cuda:
            return self.maxpool(_gn_epi(self.conv1, self.gn1, x))
        return self.maxpool(F.relu(self.gn1(self.conv1(x)), inplace=True))


def _fold(conv: nn.Conv2d, aff: AffineChannel2d) -> nn.Conv2d:
    f = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride,
                  conv.padding, conv.dilation, conv.groups, bias=True).to(conv.weight.device)
    with torch.no_grad():
        f.weight.copy_(conv.weight * aff.weight.view(-1, 1, 1, 1))
        f.bias.copy_(aff.bias if conv.bias is None else conv.bias * aff.weight + aff.bias)
    f.weight.requires_grad_(False)
    f.bias.requires_grad_(False)
    return f


class _StemEpilogue(nn.Module):
    """Folded stem: conv1 + bias + ReLU + max-pool in one MFMA kernel
    (VOSDET_STEM=split, the default: vd_stem_split_conv_pool, conv1 on the bf16 matrix
    cores at fp32 accuracy; =fused: vd_stem_conv_pool, fp32 MFMA; =miopen: conv1 on
    MIOpen + one epilogue pass)."""

    def __init__(self, conv1, maxpool):
        super().__init__()
        self.conv1, self.maxpool = conv1, maxpool

    def _fused_ok(self, x):
        c = self.conv1
        return (os.environ.get("VOSDET_STEM", "split") in ("split", "fused")
                and c.bias is not None
                and tuple(c.weight.shape) == (64, 3, 7, 7) and c.stride == (2, 2)
                and c.padding == (3, 3) and c.dilation == (1, 1) and c.groups == 1
                and x.shape[1] == 3 and x.is_contiguous(memory_format=torch.channels_last)
                and x.dtype == torch.float32)

    def forward(self, x):
        if x.is_cuda:
            if self._fused_ok(x):  # conv + bias + ReLU + max-pool in one MFMA kernel
                split = os.environ.get("VOSDET_STEM", "split") == "split"
                key = (self.conv1.weight.data_ptr(), self.conv1.weight._version, split)
                if getattr(self, "_stem_key", None) != key:
                    self._stem_packed = ops.stem_pack(self.conv1.weight, split=split)
                    self._stem_key = key
                return ops.stem_conv_pool(x, self._stem_packed, self.conv1.bias)
            h = _conv_nb(self.conv1, x)
            if (h.is_contiguous(memory_format=torch.channels_last) and not h.is_contiguous()
                    and h.shape[1] % 4 == 0 and os.environ.get("VOSDET_STEM_FUSED", "1") != "0"):
                return ops.bias_relu_maxpool(h, self.conv1.bias)  # one pass, bit-identical
            return self.maxpool(ops.bias_act_(h, self.conv1.bias, relu=True))
        return self.maxpool(F.relu(self.conv1(x), inplace=True))


class ResNetBody(nn.Module):
    """ResNet.py ResNet_convX_body (res1..res5) with basic_bn_stem /
    bottleneck_transformation, or (cfg given and RESNETS.USE_GN) basic_gn_stem /
    bottleneck_gn_transformation / basic_gn_shortcut."""

    def __init__(self, block_counts, groups=1, width_per_group=64, stride_1x1=True, cfg=None):
        super().__init__()
        self.block_counts = block_counts
        self.convX = len(block_counts) + 1
        self.use_gn = bool(cfg is not None and cfg.RESNETS.USE_GN)
        norm = ("gn1", _gn(64, cfg)) if self.use_gn else ("bn1", AffineChannel2d(64))
        self.res1 = nn.Sequential(OrderedDict([
            ("conv1", nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)),
            norm,
            ("relu", nn.ReLU(inplace=True)),
            ("maxpool", nn.MaxPool2d(kernel_size=3, stride=2, padding=1))]))
        inner = groups * width_per_group
        dim_in = 64
        specs = [(256, inner, 1), (512, inner * 2, 2), (1024, inner * 4, 2), (2048, inner * 8, 2)]
        for i, (n, (out, innerp, stride)) in enumerate(zip(block_counts, specs)):
            blocks = []
            for b in range(n):
                st = stride if b == 0 else 1
                blocks.append(BottleneckGN(dim_in, out, innerp, st, groups, stride_1x1, cfg)
                              if self.use_gn else
                              Bottleneck(dim_in, out, innerp, st, groups, stride_1x1))
                dim_in = out
            setattr(self, "res%d" % (i + 2), nn.Sequential(*blocks))
        self.dim_out = dim_in

    def forward_stages(self, x):
        outs = []
        for i in range(self.convX):
            x = getattr(self, "res%d" % (i + 1))(x)
            outs.append(x)
        return outs


class TopdownLateral(nn.Module):
    """FPN.py topdown_lateral_module (:261-299): lateral 1x1 (+ GroupNorm with
    FPN.USE_GN) + nearest 2x top-down."""

    def __init__(self, dim_top, dim_lateral, cfg=None):
        super().__init__()
        self.use_gn = bool(cfg is not None and cfg.FPN.USE_GN)
        if self.use_gn:
            self.conv_lateral = nn.Sequential(nn.Conv2d(dim_lateral, dim_top, 1, 1, 0, bias=False),
                                              _gn(dim_top, cfg))
        else:
            self.conv_lateral = nn.Conv2d(dim_lateral, dim_top, 1, 1, 0)
        self.epilogue = False

    def forward(self, top, lateral):
        if self.epilogue and lateral.is_cuda:
            if self.use_gn:
                return _gn_epi(self.conv_lateral[0], self.conv_lateral[1], lateral, act=None,
                               res=top, up=True)
            c = self.conv_lateral
            w2d = getattr(self, "_vd_w2d", None)
            if w2d is None or w2d.data_ptr() != c.weight.data_ptr():
                # one persistent 2-D view of the weight (ops caches its split image)
                w2d = self._vd_w2d = c.weight.reshape(c.out_channels, -1)
            if ops.split3_enabled() and c.in_channels >= ops.SPLIT3_MIN_K and \
                    c.out_channels % 64 == 0 and c.bias is not None and _is_1x1(c) and \
                    c.stride == (1, 1) and _gemm_ok(lateral) and top.is_cuda and \
                    top.shape[2] * 2 == lateral.shape[2] and top.shape[3] * 2 == lateral.shape[3]:
                # the lateral 1x1, its bias and the nearest-2x top-down add in one launch
                # on the bf16 matrix cores at fp32 accuracy (csrc/gemm_split3.hip)
                wp = ops.split3_weight_cached(w2d)
                if wp is not None:
                    n, _, H, W = lateral.shape
                    t = top if top.is_contiguous(memory_format=torch.channels_last) else \
                        top.contiguous(memory_format=torch.channels_last)
                    y = ops.gemm_split3_bias_act(_nhwc2d(lateral), wp, c.bias,
                                                 residual=_nhwc2d(t), relu=False, up_hw=(H, W))
                    _count_route("fpn_lateral_split3")
                    return y.view(n, H, W, -1).permute(0, 3, 1, 2)
            wf = getattr(self, "_vd_wf", None)
            if wf is not None:
                # the packed weight follows the live one (a load_state_dict after
                # prepare_fpn_body), as the Winograd routes' U keys do
                w = c.weight
                key = (w.data_ptr(), w._version)
                if self._vd_wf_key != key:
                    wf = self._vd_wf = ops.fpn_lateral_weight(w.detach())
                    self._vd_wf_key = key
            if wf is not None and _gemm_ok(lateral) and top.shape[2] * 2 == lateral.shape[2] \
                    and top.shape[3] * 2 == lateral.shape[3]:
                # the lateral 1x1, its bias and the nearest-2x top-down add in one
                # MFMA launch (csrc/gemm_lateral.hip): no separate pass over the sum
                _count_route("fpn_lateral")
                return ops.fpn_lateral_topdown(lateral, wf, c.bias, top)
            if _gemm_ok(lateral) and _is_1x1(c) and c.stride == (1, 1):
                # the lateral 1x1 as a GEMM with its bias fused, then the nearest-2x
                # top-down add (MIOpen / CK took it before; at small batches their
                # solvers were not run-to-run deterministic)
                y = _gemm_conv1x1(lateral, w2d, c.bias, relu=False)
                return ops.bias_act_(y, None, top, relu=False, upsample_residual=True)
            return _conv_epi(c, lateral, relu=False, res=top, up=True)
        return self.conv_lateral(lateral) + F.interpolate(top, scale_factor=2, mode="nearest")


class FPNBody(nn.Module):
    """FPN.py fpn (P2..P5 + P6 by 1x1/2 max-pool; outputs coarsest first)."""

    def __init__(self, cfg):
        super().__init__()
        counts = _stage_counts(cfg.MODEL.CONV_BODY)
        self.conv_body = ResNetBody(counts, cfg.RESNETS.NUM_GROUPS, cfg.RESNETS.WIDTH_PER_GROUP,
                                    cfg.RESNETS.STRIDE_1X1, cfg)
        dim = cfg.FPN.DIM
        lat_dims = (2048, 1024, 512, 256)
        self.use_gn = bool(cfg.FPN.USE_GN)
        if self.use_gn:  # FPN.py:96-101, 113-120
            self.conv_top = nn.Sequential(nn.Conv2d(lat_dims[0], dim, 1, 1, 0, bias=False),
                                          _gn(dim, cfg))
            self.posthoc_modules = nn.ModuleList(
                [nn.Sequential(nn.Conv2d(dim, dim, 3, 1, 1, bias=False), _gn(dim, cfg))
                 for _ in range(4)])
        else:
            self.conv_top = nn.Conv2d(lat_dims[0], dim, 1, 1, 0)
            self.posthoc_modules = nn.ModuleList([nn.Conv2d(dim, dim, 3, 1, 1) for _ in range(4)])
        self.topdown_lateral_modules = nn.ModuleList(
            [TopdownLateral(dim, lat_dims[i + 1], cfg) for i in range(3)])
        self.spatial_scale = [1. / 64, 1. / 32, 1. / 16, 1. / 8, 1. / 4]  # incl. P6
        self.dim_out = dim
        self.epilogue = False

    def _gn_seq(self, m, x):
        if self.epilogue and x.is_cuda:
            return _gn_epi(m[0], m[1], x, act=None)
        return m(x)

    def forward(self, x):
        c = self.conv_body.forward_stages(x)  # res1..res5
        if self.use_gn:
            inner = [self._gn_seq(self.conv_top, c[-1])]
        elif self.epilogue and c[-1].is_cuda and _gemm_ok(c[-1]):
            # one persistent 2-D view of the weight (the split-bf16 image is cached per
            # tensor object; a fresh view per call would re-split it every step)
            cw = self.conv_top.weight
            if getattr(self, "_vd_top_src", None) is not cw:
                self._vd_top_w2d = cw.reshape(self.conv_top.out_channels, -1)
                self._vd_top_src = cw
            inner = [_gemm_conv1x1(c[-1], self._vd_top_w2d, self.conv_top.bias, relu=False)]
        else:
            inner = [self.conv_top(c[-1])]
        for i in range(3):
            inner.append(self.topdown_lateral_modules[i](inner[-1], c[-(i + 2)]))
        if self.use_gn:
            outs = [self._gn_seq(self.posthoc_modules[i], inner[i]) for i in range(4)]
        else:
            outs = []
            for i in range(4):
                y = _conv3x3_mfma(self.posthoc_modules[i], inner[i]) if self.epilogue else None
                outs.append(y if y is not None else self.posthoc_modules[i](inner[i]))
        outs.insert(0, F.max_pool2d(outs[0], kernel_size=1, stride=2, padding=0))  # P6
        return outs  # [P6, P5, P4, P3, P2]


class FPNRPNOutputs(nn.Module):
    """FPN.py fpn_rpn_outputs: shared 3x3 conv + cls/bbox 1x1 on every level."""

    def __init__(self, dim_in, num_anchors=3):
        super().__init__()
        self.FPN_RPN_conv = nn.Conv2d(dim_in, dim_in, 3, 1, 1)
        self.FPN_RPN_cls_score = nn.Conv2d(dim_in, num_anchors, 1, 1, 0)
        self.FPN_RPN_bbox_pred = nn.Conv2d(dim_in, 4 * num_anchors, 1, 1, 0)
        self.num_anchors = num_anchors
        self.fused = None
        self.fused_w2d = None

    def fuse(self):
        A = self.num_anchors
        f = nn.Conv2d(self.FPN_RPN_conv.out_channels, 5 * A, 1, 1, 0).to(
            self.FPN_RPN_cls_score.weight.device)
        with torch.no_grad():
            f.weight.copy_(torch.cat([self.FPN_RPN_cls_score.weight,
                                      self.FPN_RPN_bbox_pred.weight]))
            f.bias.copy_(torch.cat([self.FPN_RPN_cls_score.bias, self.FPN_RPN_bbox_pred.bias]))
        self.fused = f
        self.fused_w2d = f.weight.detach().reshape(5 * A, -1).contiguous()

    def level_outputs(self, x):
        """(sigmoid cls probs N x A x H x W, bbox deltas N x 4A x H x W)."""
        A = self.num_anchors
        if (self.fused is not None and x.is_cuda and _gemm_ok(x) and 5 * A <= 16
                and x.shape[1] % 64 == 0 and os.environ.get("VOSDET_RPN_HEAD", "1") != "0"):
            # conv without bias, then bias + ReLU + both 1x1s + sigmoid in one pass
            h = _conv3x3_mfma(self.FPN_RPN_conv, x, bias=False)
            if h is None:
                h = _conv_nb(self.FPN_RPN_conv, x)
            if not h.is_contiguous(memory_format=torch.channels_last):
                h = h.contiguous(memory_format=torch.channels_last)
            return ops.rpn_head(h, self.FPN_RPN_conv.bias.detach(), self.fused_w2d,
                                self.fused.bias.detach(), A)
        if self.fused is not None and x.is_cuda:
            h = _conv_epi(self.FPN_RPN_conv, x)
        else:
            h = F.relu(self.FPN_RPN_conv(x), inplace=True)
        if self.fused is not None:
            if _gemm_ok(h):  # the fused cls + bbox 1x1 as one GEMM with the bias epilogue
                o = _gemm_conv1x1(h, self.fused_w2d, self.fused.bias.detach(), relu=False)
            else:
                o = self.fused(h)
            return torch.sigmoid(o[:, :A]).contiguous(), o[:, A:].contiguous()
        return torch.sigmoid(self.FPN_RPN_cls_score(h)), self.FPN_RPN_bbox_pred(h)


class Roi2MLPHead(nn.Module):
    """fast_rcnn_heads.roi_2mlp_head."""

    def __init__(self, dim_in, roi_xform, spatial_scale, cfg):
        super().__init__()
        self.roi_xform = roi_xform
        self.spatial_scale = spatial_scale
        self.cfg = cfg
        res = cfg.FAST_RCNN.ROI_XFORM_RESOLUTION
        hid = cfg.FAST_RCNN.MLP_HEAD_DIM
        self.fc1 = nn.Linear(dim_in * res ** 2, hid)
        self.fc2 = nn.Linear(hid, hid)
        self.dim_out = hid

    def mlp(self, x):
        x = F.relu(self.fc1(x.view(x.size(0), -1)), inplace=True)
        return F.relu(self.fc2(x), inplace=True)

    def mlp_nhwc(self, x):
        """fc6/fc7 on R x P x P x C RoI features: fc6's weight columns are permuted
        once (prepare) from the reference's (c, ph, pw) flattening to (ph, pw, c)."""
        x = x.reshape(x.size(0), -1)
        if x.is_cuda and x.dtype == torch.float32 and x.size(0) > 0:
            # ReLU in the GEMM epilogue, the plan pinned per shape (ops.gemm_bias_act)
            y = ops.gemm_bias_act(x.contiguous(), self.fc1_nhwc_weight, self.fc1.bias, relu=True)
            if y is not None:
                z = ops.gemm_bias_act(y, self.fc2.weight, self.fc2.bias, relu=True)
                if z is not None:
                    return z
        x = F.relu(F.linear(x, self.fc1_nhwc_weight, self.fc1.bias), inplace=True)
        return F.relu(self.fc2(x), inplace=True)

    @torch.no_grad()
    def prepare(self):
        res = self.cfg.FAST_RCNN.ROI_XFORM_RESOLUTION
        w = self.fc1.weight
        C = w.shape[1] // (res * res)
        self.fc1_nhwc_weight = (w.view(w.shape[0], C, res, res).permute(0, 2, 3, 1)
                                .reshape(w.shape[0], -1).contiguous())
        self.nhwc_ready = True

    def forward(self, x, rpn_ret):
        c = self.cfg.FAST_RCNN
        x = self.roi_xform(x, rpn_ret, blob_rois="rois", method=c.ROI_XFORM_METHOD,
                           resolution=c.ROI_XFORM_RESOLUTION, spatial_scale=self.spatial_scale,
                           sampling_ratio=c.ROI_XFORM_SAMPLING_RATIO)
        return self.mlp(x)


class RoiXconv1fcGNHead(nn.Module):
    """fast_rcnn_heads.roi_Xconv1fc_gn_head (:227-290): NUM_STACKED_CONVS x
    (conv 3x3, GroupNorm, ReLU) + fc + ReLU.  The NHWC path runs each
    GroupNorm + ReLU as one vd_group_norm_act on the R x P x P x C RoI features
    straight from the RoIAlign kernel; fc's columns are permuted once to match."""

    def __init__(self, dim_in, roi_xform, spatial_scale, cfg):
        super().__init__()
        self.roi_xform = roi_xform
        self.spatial_scale = spatial_scale
        self.cfg = cfg
        hid = cfg.FAST_RCNN.CONV_HEAD_DIM
        mods = []
        for _ in range(cfg.FAST_RCNN.NUM_STACKED_CONVS):
            mods += [nn.Conv2d(dim_in, hid, 3, 1, 1, bias=False), _gn(hid, cfg),
                     nn.ReLU(inplace=True)]
            dim_in = hid
        self.convs = nn.Sequential(*mods)
        res = cfg.FAST_RCNN.ROI_XFORM_RESOLUTION
        self.dim_out = cfg.FAST_RCNN.MLP_HEAD_DIM
        self.fc = nn.Linear(dim_in * res * res, self.dim_out)

    def mlp(self, x):
        x = self.convs(x)
        return F.relu(self.fc(x.reshape(x.size(0), -1)), inplace=True)

    def mlp_nhwc(self, x):
        R = x.shape[0]
        y = x.permute(0, 3, 1, 2)  # NCHW view, channels_last memory
        for i in range(0, len(self.convs), 3):
            y = _gn_epi(self.convs[i], self.convs[i + 1], y)
        y = y.permute(0, 2, 3, 1).reshape(R, -1)
        # fc + ReLU in one GEMM launch (split-bf16 at K = 12,544; torch's hipBLASLt GEMM
        # took 2.7 ms per 16-frame VOS step)
        z = ops.gemm_bias_act(y.contiguous(), self.fc_nhwc_weight, self.fc.bias, relu=True)
        if z is not None:
            return z
        return F.relu(F.linear(y, self.fc_nhwc_weight, self.fc.bias), inplace=True)

    @torch.no_grad()
    def prepare(self):
        res = self.cfg.FAST_RCNN.ROI_XFORM_RESOLUTION
        w = self.fc.weight
        C = w.shape[1] // (res * res)
        self.fc_nhwc_weight = (w.view(w.shape[0], C, res, res).permute(0, 2, 3, 1)
                               .reshape(w.shape[0], -1).contiguous())
        self.convs.to(memory_format=torch.channels_last)
        self.nhwc_ready = True

    def forward(self, x, rpn_ret):
        c = self.cfg.FAST_RCNN
        x = self.roi_xform(x, rpn_ret, blob_rois="rois", method=c.ROI_XFORM_METHOD,
                           resolution=c.ROI_XFORM_RESOLUTION, spatial_scale=self.spatial_scale,
                           sampling_ratio=c.ROI_XFORM_SAMPLING_RATIO)
        return self.mlp(x)


class FastRCNNOutputs(nn.Module):
    """fast_rcnn_heads.fast_rcnn_outputs (:13-84; softmax at inference).  With
    CLS_AGNOSTIC_BBOX_REG the box head predicts 2 x 4 deltas (bg, fg)."""

    def __init__(self, dim_in, num_classes, cls_agnostic=False):
        super().__init__()
        self.cls_score = nn.Linear(dim_in, num_classes)
        self.bbox_pred = nn.Linear(dim_in, 4 * (2 if cls_agnostic else num_classes))
        self.cls_agnostic = cls_agnostic

    def forward(self, x):
        if x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.shape[0] > 0 and \
                ops.split3_enabled() and x.shape[1] >= ops.SPLIT3_MIN_K and x.shape[1] % 16 == 0:
            # cls_score and bbox_pred as ONE GEMM over the concatenated weights (N = 81 +
            # 324 padded to 448: a multiple of the 64-channel tile) on the split-bf16
            # kernel; hipBLASLt ran the two skinny GEMMs at ~0.1 of the fp32 peak
            w, b = self._cat_weights()
            y = ops.gemm_bias_act(x.contiguous(), w, b, relu=False)
            if y is not None:
                nc, nb = self.cls_score.out_features, self.bbox_pred.out_features
                return F.softmax(y[:, :nc], dim=1), y[:, nc:nc + nb].contiguous()
        return F.softmax(self.cls_score(x), dim=1), self.bbox_pred(x)

    @torch.no_grad()
    def _cat_weights(self):
        ws = (self.cls_score.weight, self.bbox_pred.weight, self.cls_score.bias,
              self.bbox_pred.bias)
        key = tuple((t.data_ptr(), t._version) for t in ws)
        if getattr(self, "_vd_cat_key", None) != key:
            n = ws[0].shape[0] + ws[1].shape[0]
            npad = (n + 63) // 64 * 64
            w = torch.zeros((npad, ws[0].shape[1]), dtype=ws[0].dtype, device=ws[0].device)
            b = torch.zeros((npad,), dtype=ws[0].dtype, device=ws[0].device)
            w[:n] = torch.cat([ws[0], ws[1]])
            b[:n] = torch.cat([ws[2], ws[3]])
            self._vd_cat, self._vd_cat_key = (w, b), key
        return self._vd_cat

    def per_class_deltas(self, bbox_pred, num_classes):
        """vos_test.py:179-190 decodes the fg deltas once and tiles the boxes over
        the classes; decoding the tiled deltas per class gives the same boxes."""
        if not self.cls_agnostic:
            return bbox_pred
        return bbox_pred[:, -4:].repeat(1, num_classes)


class MaskHeadV1upXconvs(nn.Module):
    """mask_rcnn_heads.mask_rcnn_fcn_head_v1upXconvs."""

    def __init__(self, dim_in, roi_xform, spatial_scale, cfg, num_convs=4):
        super().__init__()
        self.roi_xform = roi_xform
        self.spatial_scale = spatial_scale
        self.cfg = cfg
        d = cfg.MRCNN.DILATION
        inner = cfg.MRCNN.DIM_REDUCED
        mods = []
        for _ in range(num_convs):
            mods += [nn.Conv2d(dim_in, inner, 3, 1, padding=d, dilation=d), nn.ReLU(inplace=True)]
            dim_in = inner
        self.conv_fcn = nn.Sequential(*mods)
        self.upconv = nn.ConvTranspose2d(inner, inner, 2, 2, 0)
        self.dim_out = inner

    def head(self, x):
        return F.relu(self.upconv(self.conv_fcn(x)), inplace=True)

    @torch.no_grad()
    def prepare(self):
        """ConvTranspose2d(k=2, s=2) has no overlapping taps, so it is one GEMM
        [M*H*W, Cin] x [Cin, 2*2*Cout] followed by a depth-to-space shuffle."""
        w = self.upconv.weight  # Cin x Cout x 2 x 2
        self.up_w = w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous()  # Cin x (i,j,co)
        self.up_b = self.upconv.bias.repeat(4).contiguous()
        self.up_wt = self.up_w.t().contiguous()  # (i,j,co) x Cin: ops.gemm_bias_act's W
        self.nhwc_ready = True

    def head_nhwc(self, x_nhwc):
        """x_nhwc: M x P x P x C RoI features.  Returns M x P x P x 2 x 2 x C
        (relu'd upconv output; (h, w, i, j) -> pixel (2h+i, 2w+j))."""
        M, P, _, C = x_nhwc.shape
        x = self._convs_nhwc(x_nhwc.permute(0, 3, 1, 2))  # NCHW view, channels_last
        x = x.permute(0, 2, 3, 1).reshape(M * P * P, -1)
        # bias + ReLU in the GEMM epilogue (hipBLASLt, the plan pinned per shape by
        # ops.gemm_bias_act's timing search) instead of a separate pass over the
        # (M*P*P x 4C) upconv output
        y = ops.gemm_bias_act(x.contiguous(), self.up_wt, self.up_b, relu=True)
        if y is None:
            y = torch._addmm_activation(self.up_b, x, self.up_w)
        return y.view(M, P, P, 2, 2, -1)

    def masks_nhwc(self, x_nhwc, outs, cls_idx):
        """x_nhwc: M x P x P x C RoI features -> M x 2P x 2P mask probabilities at each
        RoI's class (outs: the MaskRCNNOutputs).  With the split-bf16 GEMM on, the upconv
        and the class-selected logits run as ONE launch (ops.mask_head_upconv_logits):
        the M x P x P x 1024 relu'd upconv output never reaches HBM."""
        M, P, _, C = x_nhwc.shape
        cw = outs.classify.weight
        if ops.split3_enabled() and C == 256 and tuple(self.up_wt.shape) == (1024, 256) and \
                cw.shape[1] == 256 and M > 0:
            x = self._convs_nhwc(x_nhwc.permute(0, 3, 1, 2))
            x = x.permute(0, 2, 3, 1).reshape(M * P * P, -1)
            wp = ops.split3_weight_cached(self.up_wt)
            if wp is not None:
                ch = outs._channel(cls_idx).to(torch.int32)
                return ops.mask_head_upconv_logits(x.contiguous(), wp, self.up_b,
                                                   cw.view(cw.shape[0], -1), outs.classify.bias,
                                                   ch, P)
            return outs.selected_from_up(self._upconv_nhwc(x, M, P), cls_idx)
        return outs.selected_from_up(self.head_nhwc(x_nhwc), cls_idx)

    def _upconv_nhwc(self, x, M, P):
        y = ops.gemm_bias_act(x.contiguous(), self.up_wt, self.up_b, relu=True)
        if y is None:
            y = torch._addmm_activation(self.up_b, x, self.up_w)
        return y.view(M, P, P, 2, 2, -1)

    def _convs_nhwc(self, x):
        for m in self.conv_fcn:
            if isinstance(m, nn.Conv2d):
                y = _conv3x3_mfma(m, x, relu=True, mosaic=True)  # N x 14 x 14 RoI maps
                x = y if y is not None else _conv_epi(m, x)
        return x

    def forward(self, x, rpn_ret):
        c = self.cfg.MRCNN
        x = self.roi_xform(x, rpn_ret, blob_rois="mask_rois", method=c.ROI_XFORM_METHOD,
                           resolution=c.ROI_XFORM_RESOLUTION, spatial_scale=self.spatial_scale,
                           sampling_ratio=c.ROI_XFORM_SAMPLING_RATIO)
        return self.head(x)


class MaskHeadV1upXconvsGN(MaskHeadV1upXconvs):
    """mask_rcnn_heads.mask_rcnn_fcn_head_v1upXconvs_gn (:191-255): X x (conv 3x3
    no bias, GroupNorm, ReLU), ConvTranspose 2x2 + ReLU."""

    def __init__(self, dim_in, roi_xform, spatial_scale, cfg, num_convs=4):
        super().__init__(dim_in, roi_xform, spatial_scale, cfg, num_convs)
        d = cfg.MRCNN.DILATION
        inner = cfg.MRCNN.DIM_REDUCED
        mods = []
        for _ in range(num_convs):
            mods += [nn.Conv2d(dim_in, inner, 3, 1, padding=d, dilation=d, bias=False),
                     _gn(inner, cfg), nn.ReLU(inplace=True)]
            dim_in = inner
        self.conv_fcn = nn.Sequential(*mods)

    def _convs_nhwc(self, x):
        for i in range(0, len(self.conv_fcn), 3):
            x = _gn_epi(self.conv_fcn[i], self.conv_fcn[i + 1], x)
        return x


class MaskRCNNOutputs(nn.Module):
    """mask_rcnn_heads.mask_rcnn_outputs (sigmoid at inference).  The
    reference's stock builder passes one argument (model_builder.py:114, a
    crash); the fork passes NUM_CLASSES (vos_model_builder.py:144), as here."""

    def __init__(self, dim_in, num_classes):
        super().__init__()
        self.classify = nn.Conv2d(dim_in, num_classes, 1, 1, 0)

    def forward(self, x):
        return torch.sigmoid(self.classify(x))

    def _channel(self, cls_idx):
        """Mask channel of each RoI: its class, or 0 for a class-agnostic head
        (MRCNN.CLS_SPECIFIC_MASK False, mask_rcnn_heads.py:26; segm_results
        reads masks[i, 0], vos_test.py:885-888)."""
        if self.classify.out_channels == 1:
            return torch.zeros_like(cls_idx, dtype=torch.long)
        return cls_idx.long()

    def selected(self, x, cls_idx):
        """Sigmoid of only the channel of each RoI's class: the per-RoI dot
        product with the selected 1x1 filter (what segm_results consumes)."""
        ch = self._channel(cls_idx)
        w = self.classify.weight[ch, :, 0, 0]  # M x D
        b = self.classify.bias[ch]
        y = torch.einsum("mdhw,md->mhw", x, w) + b.view(-1, 1, 1)
        return torch.sigmoid(y)

    def selected_from_up(self, up, cls_idx):
        """up: M x P x P x 2 x 2 x D (MaskHead.head_nhwc) -> M x 2P x 2P masks."""
        M, P = up.shape[0], up.shape[1]
        ch = self._channel(cls_idx)
        w = self.classify.weight[ch, :, 0, 0]  # M x D
        b = self.classify.bias[ch]
        y = torch.bmm(up.view(M, P * P * 4, -1), w.unsqueeze(2)).view(M, P, P, 2, 2)
        y = y.permute(0, 1, 3, 2, 4).reshape(M, 2 * P, 2 * P) + b.view(-1, 1, 1)
        return torch.sigmoid(y)


# cfg.FAST_RCNN.ROI_BOX_HEAD / cfg.MRCNN.ROI_MASK_HEAD names -> modules (the
# reference resolves them with get_func, model_builder.py:33-49)
BOX_HEADS = {"fast_rcnn_heads.roi_2mlp_head": Roi2MLPHead,
             "fast_rcnn_heads.roi_Xconv1fc_gn_head": RoiXconv1fcGNHead}
MASK_HEADS = {"mask_rcnn_heads.mask_rcnn_fcn_head_v1up4convs": (MaskHeadV1upXconvs, 4),
              "mask_rcnn_heads.mask_rcnn_fcn_head_v1up": (MaskHeadV1upXconvs, 2),
              "mask_rcnn_heads.mask_rcnn_fcn_head_v1up4convs_gn": (MaskHeadV1upXconvsGN, 4),
              "mask_rcnn_heads.mask_rcnn_fcn_head_v1up_gn": (MaskHeadV1upXconvsGN, 2)}


class Generalized_RCNN(nn.Module):
    """lib/modeling/model_builder.py:71-369 (inference)."""

    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.Conv_Body = FPNBody(cfg)
        self.RPN = FPNRPNOutputs(self.Conv_Body.dim_out, len(cfg.FPN.RPN_ASPECT_RATIOS))
        self.num_roi_levels = cfg.FPN.ROI_MAX_LEVEL - cfg.FPN.ROI_MIN_LEVEL + 1
        roi_scales = self.Conv_Body.spatial_scale[-self.num_roi_levels:]
        self.roi_spatial_scale = roi_scales  # coarsest first, as the reference
        self.Box_Head = BOX_HEADS[cfg.FAST_RCNN.ROI_BOX_HEAD](
            self.Conv_Body.dim_out, self.roi_feature_transform, roi_scales, cfg)
        self.Box_Outs = FastRCNNOutputs(self.Box_Head.dim_out, cfg.MODEL.NUM_CLASSES,
                                        cfg.MODEL.CLS_AGNOSTIC_BBOX_REG)
        mk, nconv = MASK_HEADS[cfg.MRCNN.ROI_MASK_HEAD]
        self.Mask_Head = mk(self.Conv_Body.dim_out, self.roi_feature_transform, roi_scales, cfg,
                            nconv)
        self.Mask_Outs = MaskRCNNOutputs(
            self.Mask_Head.dim_out, cfg.MODEL.NUM_CLASSES if cfg.MRCNN.CLS_SPECIFIC_MASK else 1)
        anchors = []
        k_min, k_max = cfg.FPN.RPN_MIN_LEVEL, cfg.FPN.RPN_MAX_LEVEL
        for lvl in range(k_min, k_max + 1):
            anchors.append(torch.from_numpy(generate_anchors(
                stride=2. ** lvl, sizes=(cfg.FPN.RPN_ANCHOR_START_SIZE * 2. ** (lvl - k_min),),
                aspect_ratios=cfg.FPN.RPN_ASPECT_RATIOS)))
        for i, a in enumerate(anchors):
            self.register_buffer("anchors_fpn%d" % (k_min + i), a, persistent=False)

    # -- the reference's operator API -------------------------------------- #
    def roi_feature_transform(self, blobs_in, rpn_ret, blob_rois="rois", method="RoIPoolF",
                              resolution=7, spatial_scale=1. / 16., sampling_ratio=0):
        """model_builder.py:252-324, same arguments and rpn_ret keys (ndarrays on the
        host).  Each level's op is the HIP kernel behind RoIAlignFunction /
        RoIPoolFunction / RoICropFunction."""
        assert method in {"RoIPoolF", "RoICrop", "RoIAlign"}, \
            "Unknown pooling method: {}".format(method)
        if method == "RoICrop":
            # model_builder.py:283 uses self.grid_size, which the reference never
            # assigns: the branch raises there too.
            raise AttributeError("'Generalized_RCNN' object has no attribute 'grid_size'")
        cfg = self.cfg
        if isinstance(blobs_in, list):
            dev = blobs_in[0].device
            k_max, k_min = cfg.FPN.ROI_MAX_LEVEL, cfg.FPN.ROI_MIN_LEVEL
            assert len(blobs_in) == k_max - k_min + 1
            outs = []
            for lvl in range(k_min, k_max + 1):
                bl_in = blobs_in[k_max - lvl]
                sc = spatial_scale[k_max - lvl]
                r = rpn_ret[blob_rois + "_fpn" + str(lvl)]
                if len(r):
                    rois = torch.as_tensor(np.ascontiguousarray(r, np.float32), device=dev)
                    if method == "RoIPoolF":
                        outs.append(ops.RoIPoolFunction(resolution, resolution, sc)(bl_in, rois))
                    else:
                        outs.append(ops.RoIAlignFunction(resolution, resolution, sc,
                                                         sampling_ratio)(bl_in, rois))
            shuffled = torch.cat(outs, dim=0)
            restore = torch.as_tensor(
                rpn_ret[blob_rois + "_idx_restore_int32"].astype(np.int64), device=dev)
            return shuffled[restore]
        rois = torch.as_tensor(np.ascontiguousarray(rpn_ret[blob_rois], np.float32),
                               device=blobs_in.device)
        if method == "RoIPoolF":
            return ops.RoIPoolFunction(resolution, resolution, spatial_scale)(blobs_in, rois)
        return ops.RoIAlignFunction(resolution, resolution, spatial_scale,
                                    sampling_ratio)(blobs_in, rois)

    # -- inference-time fusion ---------------------------------------------- #
    @torch.no_grad()
    def fold_affine(self, epilogue: bool = True):
        """Fold the frozen AffineChannel2d into conv weight + bias; with `epilogue`
        the bias/residual/ReLU after each conv run as one vd_bias_act pass (GN
        bodies: each GroupNorm + residual + ReLU as one vd_group_norm_act)."""
        prepare_fpn_body(self.Conv_Body, epilogue)
        self.RPN.fuse()
        self.Box_Head.prepare()
        self.Mask_Head.prepare()
        return self


@torch.no_grad()
def prepare_bottlenecks(blocks, epilogue: bool = True):
    """Fold each BN Bottleneck's AffineChannel2d into its convs and switch on the
    fused bias/residual/ReLU epilogue (GN blocks: the fused GroupNorm epilogue)."""
    for blk in blocks:
        if isinstance(blk, Bottleneck):
            blk.f1 = _fold(blk.conv1, blk.bn1)
            blk.f2 = _fold(blk.conv2, blk.bn2)
            blk.f3 = _fold(blk.conv3, blk.bn3)
            if blk.downsample is not None:
                blk.fd = _fold(blk.downsample[0], blk.downsample[1])
                blk.b3d = (blk.f3.bias + blk.fd.bias).contiguous()
            # 2-D weights of the 1x1 convs for the GEMM epilogue path
            blk.w1 = blk.f1.weight.reshape(blk.f1.out_channels, -1).contiguous()
            blk.w3 = blk.f3.weight.reshape(blk.f3.out_channels, -1).contiguous()
            if blk.downsample is not None:  # [W3 | Wd] for the two-operand GEMM
                blk.wd = blk.fd.weight.reshape(blk.fd.out_channels, -1).contiguous()
                blk.w3d = torch.cat([blk.w3, blk.wd], 1).contiguous()
            blk.fused = True
        blk.epilogue = epilogue


@torch.no_grad()
def prepare_resnet_body(body: ResNetBody, epilogue: bool = True):
    """Inference-time rewrite of a ResNetBody (stem + every stage)."""
    stem = body.res1
    if body.use_gn:
        body.res1 = _StemGN(stem.conv1, stem.gn1, stem.maxpool) if epilogue else stem
    elif epilogue:
        body.res1 = _StemEpilogue(_fold(stem.conv1, stem.bn1), stem.maxpool)
    else:
        body.res1 = nn.Sequential(OrderedDict([
            ("conv1", _fold(stem.conv1, stem.bn1)), ("relu", nn.ReLU(inplace=True)),
            ("maxpool", stem.maxpool)]))
    for i in range(2, body.convX + 1):
        prepare_bottlenecks(getattr(body, "res%d" % i), epilogue)
    return body


@torch.no_grad()
def _fpn_lateral_fused_k():
    """Lateral input widths whose top-down step runs as ONE fused MFMA launch
    (ops.fpn_lateral_topdown).  Measured at the benched 32-frame shapes
    (profiles/r05/fpn_lateral/ab.jsonl): P2 (K = 256) 2.64 ms fused vs 3.13 ms for
    hipBLASLt + the add pass; P3 (512) even; P4 (1024) 0.68 vs 0.55 -- so P2 only by
    default.  VOSDET_FPN_LATERAL = 0 (none) | all | comma-separated K list."""
    v = os.environ.get("VOSDET_FPN_LATERAL", "256").strip().lower()
    if v in ("0", "", "none"):
        return ()
    if v == "all":
        return ops.FPN_LATERAL_K
    return tuple(int(k) for k in v.split(","))


def prepare_topdown_lateral(m: TopdownLateral, epilogue: bool = True):
    """One top-down lateral module: the fused-lateral weight (fragment order, keyed
    by the live weight so a later load_state_dict repacks it) and the epilogue flag."""
    m._vd_wf = m._vd_wf_key = None
    c = m.conv_lateral
    if epilogue and not m.use_gn and c.weight.is_cuda and _is_1x1(c) and c.stride == (1, 1) \
            and c.bias is not None and c.in_channels in _fpn_lateral_fused_k():
        m._vd_wf = ops.fpn_lateral_weight(c.weight.detach())
        m._vd_wf_key = (c.weight.data_ptr(), c.weight._version)
    m.epilogue = epilogue


def prepare_fpn_body(fpn: FPNBody, epilogue: bool = True):
    """Inference-time rewrite of an FPNBody: AffineChannel2d folded into the
    convs (BN bodies) and the fused HIP epilogues switched on."""
    prepare_resnet_body(fpn.conv_body, epilogue)
    for m in fpn.topdown_lateral_modules:
        prepare_topdown_lateral(m, epilogue)
    fpn.epilogue = epilogue
    return fpn


def generate_anchors(stride=16, sizes=(32, 64, 128, 256, 512), aspect_ratios=(0.5, 1, 2)):
    """lib/modeling/generate_anchors.py:54-123 (float64, 0-based)."""
    scales = np.array(sizes, dtype=np.float64) / stride
    ratios = np.array(aspect_ratios, dtype=np.float64)
    base = np.array([1, 1, stride, stride], dtype=np.float64) - 1

    def whctrs(a):
        w, h = a[2] - a[0] + 1, a[3] - a[1] + 1
        return w, h, a[0] + 0.5 * (w - 1), a[1] + 0.5 * (h - 1)

    def mk(ws, hs, xc, yc):
        ws, hs = ws[:, None], hs[:, None]
        return np.hstack((xc - 0.5 * (ws - 1), yc - 0.5 * (hs - 1),
                          xc + 0.5 * (ws - 1), yc + 0.5 * (hs - 1)))

    w, h, xc, yc = whctrs(base)
    ws = np.round(np.sqrt(w * h / ratios))
    ratio_anchors = mk(ws, np.round(ws * ratios), xc, yc)
    out = []
    for a in ratio_anchors:
        w, h, xc, yc = whctrs(a)
        out.append(mk(w * scales, h * scales, xc, yc))
    return np.vstack(out)
