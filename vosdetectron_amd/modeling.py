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
    """The convolution of `conv` without its bias (added by the fused epilogue)."""
    return F.conv2d(x, conv.weight, None, conv.stride, conv.padding, conv.dilation, conv.groups)


def _conv_epi(conv: nn.Conv2d, x, relu=True, res=None, res_bias=None, up=False):
    """conv -> one vd_bias_act pass: act((conv(x) + b) + (res [+ res_bias])).  Same
    association order as the module code it replaces (bias kernel after the MIOpen
    conv, then the residual add, then ReLU), so the results are bit-identical."""
    return ops.bias_act_(_conv_nb(conv, x), conv.bias, res, res_bias, relu=relu,
                         upsample_residual=up)


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
    """Folded stem: conv1 (+ bias + ReLU in one epilogue pass) + max-pool."""

    def __init__(self, conv1, maxpool):
        super().__init__()
        self.conv1, self.maxpool = conv1, maxpool

    def forward(self, x):
        if x.is_cuda:
            return self.maxpool(_conv_epi(self.conv1, x))
        return self.maxpool(F.relu(self.conv1(x), inplace=True))


class ResNetBody(nn.Module):
    """ResNet.py ResNet_convX_body with basic_bn_stem (res1..res5)."""

    def __init__(self, block_counts, groups=1, width_per_group=64, stride_1x1=True):
        super().__init__()
        self.block_counts = block_counts
        self.convX = len(block_counts) + 1
        self.res1 = nn.Sequential(OrderedDict([
            ("conv1", nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)),
            ("bn1", AffineChannel2d(64)),
            ("relu", nn.ReLU(inplace=True)),
            ("maxpool", nn.MaxPool2d(kernel_size=3, stride=2, padding=1))]))
        inner = groups * width_per_group
        dim_in = 64
        specs = [(256, inner, 1), (512, inner * 2, 2), (1024, inner * 4, 2), (2048, inner * 8, 2)]
        for i, (n, (out, innerp, stride)) in enumerate(zip(block_counts, specs)):
            blocks = []
            for b in range(n):
                blocks.append(Bottleneck(dim_in, out, innerp, stride if b == 0 else 1, groups,
                                         stride_1x1))
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
    """FPN.py topdown_lateral_module: lateral 1x1 + nearest 2x top-down."""

    def __init__(self, dim_top, dim_lateral):
        super().__init__()
        self.conv_lateral = nn.Conv2d(dim_lateral, dim_top, 1, 1, 0)
        self.epilogue = False

    def forward(self, top, lateral):
        if self.epilogue and lateral.is_cuda:
            return _conv_epi(self.conv_lateral, lateral, relu=False, res=top, up=True)
        return self.conv_lateral(lateral) + F.interpolate(top, scale_factor=2, mode="nearest")


class FPNBody(nn.Module):
    """FPN.py fpn (P2..P5 + P6 by 1x1/2 max-pool; outputs coarsest first)."""

    def __init__(self, cfg):
        super().__init__()
        counts = _stage_counts(cfg.MODEL.CONV_BODY)
        self.conv_body = ResNetBody(counts, cfg.RESNETS.NUM_GROUPS, cfg.RESNETS.WIDTH_PER_GROUP,
                                    cfg.RESNETS.STRIDE_1X1)
        dim = cfg.FPN.DIM
        lat_dims = (2048, 1024, 512, 256)
        self.conv_top = nn.Conv2d(lat_dims[0], dim, 1, 1, 0)
        self.topdown_lateral_modules = nn.ModuleList(
            [TopdownLateral(dim, lat_dims[i + 1]) for i in range(3)])
        self.posthoc_modules = nn.ModuleList([nn.Conv2d(dim, dim, 3, 1, 1) for _ in range(4)])
        self.spatial_scale = [1. / 64, 1. / 32, 1. / 16, 1. / 8, 1. / 4]  # incl. P6
        self.dim_out = dim

    def forward(self, x):
        c = self.conv_body.forward_stages(x)  # res1..res5
        inner = [self.conv_top(c[-1])]
        for i in range(3):
            inner.append(self.topdown_lateral_modules[i](inner[-1], c[-(i + 2)]))
        outs = [self.posthoc_modules[i](inner[i]) for i in range(4)]
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

    def fuse(self):
        A = self.num_anchors
        f = nn.Conv2d(self.FPN_RPN_conv.out_channels, 5 * A, 1, 1, 0).to(
            self.FPN_RPN_cls_score.weight.device)
        with torch.no_grad():
            f.weight.copy_(torch.cat([self.FPN_RPN_cls_score.weight,
                                      self.FPN_RPN_bbox_pred.weight]))
            f.bias.copy_(torch.cat([self.FPN_RPN_cls_score.bias, self.FPN_RPN_bbox_pred.bias]))
        self.fused = f

    def level_outputs(self, x):
        """(sigmoid cls probs N x A x H x W, bbox deltas N x 4A x H x W)."""
        if self.fused is not None and x.is_cuda:
            h = _conv_epi(self.FPN_RPN_conv, x)
        else:
            h = F.relu(self.FPN_RPN_conv(x), inplace=True)
        A = self.num_anchors
        if self.fused is not None:
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
        x = F.relu(F.linear(x.reshape(x.size(0), -1), self.fc1_nhwc_weight, self.fc1.bias),
                   inplace=True)
        return F.relu(self.fc2(x), inplace=True)

    @torch.no_grad()
    def prepare(self):
        res = self.cfg.FAST_RCNN.ROI_XFORM_RESOLUTION
        w = self.fc1.weight
        C = w.shape[1] // (res * res)
        self.fc1_nhwc_weight = (w.view(w.shape[0], C, res, res).permute(0, 2, 3, 1)
                                .reshape(w.shape[0], -1).contiguous())

    def forward(self, x, rpn_ret):
        c = self.cfg.FAST_RCNN
        x = self.roi_xform(x, rpn_ret, blob_rois="rois", method=c.ROI_XFORM_METHOD,
                           resolution=c.ROI_XFORM_RESOLUTION, spatial_scale=self.spatial_scale,
                           sampling_ratio=c.ROI_XFORM_SAMPLING_RATIO)
        return self.mlp(x)


class FastRCNNOutputs(nn.Module):
    """fast_rcnn_heads.fast_rcnn_outputs (softmax at inference)."""

    def __init__(self, dim_in, num_classes):
        super().__init__()
        self.cls_score = nn.Linear(dim_in, num_classes)
        self.bbox_pred = nn.Linear(dim_in, 4 * num_classes)

    def forward(self, x):
        return F.softmax(self.cls_score(x), dim=1), self.bbox_pred(x)


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

    def head_nhwc(self, x_nhwc):
        """x_nhwc: M x P x P x C RoI features.  Returns M x P x P x 2 x 2 x C
        (relu'd upconv output; (h, w, i, j) -> pixel (2h+i, 2w+j))."""
        M, P, _, C = x_nhwc.shape
        x = x_nhwc.permute(0, 3, 1, 2)  # NCHW view with channels_last strides
        for m in self.conv_fcn:
            if isinstance(m, nn.Conv2d):
                x = _conv_epi(m, x)
        x = x.permute(0, 2, 3, 1).reshape(M * P * P, -1)
        y = torch.addmm(self.up_b, x, self.up_w)
        return F.relu_(y).view(M, P, P, 2, 2, -1)

    def forward(self, x, rpn_ret):
        c = self.cfg.MRCNN
        x = self.roi_xform(x, rpn_ret, blob_rois="mask_rois", method=c.ROI_XFORM_METHOD,
                           resolution=c.ROI_XFORM_RESOLUTION, spatial_scale=self.spatial_scale,
                           sampling_ratio=c.ROI_XFORM_SAMPLING_RATIO)
        return self.head(x)


class MaskRCNNOutputs(nn.Module):
    """mask_rcnn_heads.mask_rcnn_outputs (sigmoid at inference).  The
    reference's stock builder passes one argument (model_builder.py:114, a
    crash); the fork passes NUM_CLASSES (vos_model_builder.py:144), as here."""

    def __init__(self, dim_in, num_classes):
        super().__init__()
        self.classify = nn.Conv2d(dim_in, num_classes, 1, 1, 0)

    def forward(self, x):
        return torch.sigmoid(self.classify(x))

    def selected(self, x, cls_idx):
        """Sigmoid of only the channel of each RoI's class: the per-RoI dot
        product with the selected 1x1 filter (what segm_results consumes)."""
        w = self.classify.weight[cls_idx.long(), :, 0, 0]  # M x D
        b = self.classify.bias[cls_idx.long()]
        y = torch.einsum("mdhw,md->mhw", x, w) + b.view(-1, 1, 1)
        return torch.sigmoid(y)

    def selected_from_up(self, up, cls_idx):
        """up: M x P x P x 2 x 2 x D (MaskHead.head_nhwc) -> M x 2P x 2P masks."""
        M, P = up.shape[0], up.shape[1]
        w = self.classify.weight[cls_idx.long(), :, 0, 0]  # M x D
        b = self.classify.bias[cls_idx.long()]
        y = torch.bmm(up.view(M, P * P * 4, -1), w.unsqueeze(2)).view(M, P, P, 2, 2)
        y = y.permute(0, 1, 3, 2, 4).reshape(M, 2 * P, 2 * P) + b.view(-1, 1, 1)
        return torch.sigmoid(y)


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
        self.Box_Head = Roi2MLPHead(self.Conv_Body.dim_out, self.roi_feature_transform,
                                    roi_scales, cfg)
        self.Box_Outs = FastRCNNOutputs(self.Box_Head.dim_out, cfg.MODEL.NUM_CLASSES)
        self.Mask_Head = MaskHeadV1upXconvs(self.Conv_Body.dim_out, self.roi_feature_transform,
                                            roi_scales, cfg)
        self.Mask_Outs = MaskRCNNOutputs(self.Mask_Head.dim_out, cfg.MODEL.NUM_CLASSES)
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
        the bias/residual/ReLU after each conv run as one vd_bias_act pass."""
        body = self.Conv_Body.conv_body
        stem = body.res1
        if epilogue:
            body.res1 = _StemEpilogue(_fold(stem.conv1, stem.bn1), stem.maxpool)
        else:
            body.res1 = nn.Sequential(OrderedDict([
                ("conv1", _fold(stem.conv1, stem.bn1)), ("relu", nn.ReLU(inplace=True)),
                ("maxpool", stem.maxpool)]))
        for i in range(2, body.convX + 1):
            for blk in getattr(body, "res%d" % i):
                blk.f1 = _fold(blk.conv1, blk.bn1)
                blk.f2 = _fold(blk.conv2, blk.bn2)
                blk.f3 = _fold(blk.conv3, blk.bn3)
                if blk.downsample is not None:
                    blk.fd = _fold(blk.downsample[0], blk.downsample[1])
                blk.fused = True
                blk.epilogue = epilogue
        for m in self.Conv_Body.topdown_lateral_modules:
            m.epilogue = epilogue
        self.RPN.fuse()
        self.Box_Head.prepare()
        self.Mask_Head.prepare()
        return self


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
