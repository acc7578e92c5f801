"""e2e_mask_rcnn_R-50-C4 (BASELINE.json configs[0]): the single-scale model family.

Reference module tree (configs/baselines/e2e_mask_rcnn_R-50-C4_1x.yaml):
  Conv_Body  ResNet.ResNet50_conv4_body         lib/modeling/ResNet.py:17-116 (res1..res4, 1/16)
  RPN        rpn_heads.single_scale_rpn_outputs lib/modeling/rpn_heads.py:37-126 (15 anchors)
  Box_Head   ResNet.ResNet_roi_conv5_head       lib/modeling/ResNet.py:118-155 (RoIAlign 14x14,
             res5 with stride 2, avgpool 7)
  Box_Outs   fast_rcnn_heads.fast_rcnn_outputs
  Mask_Head  mask_rcnn_heads.mask_rcnn_fcn_head_v0upshare  mask_rcnn_heads.py:263-331 (res5
             shared with the box head, upconv5 2x2 + ReLU)
  Mask_Outs  mask_rcnn_heads.mask_rcnn_outputs  (14x14 masks, MRCNN.RESOLUTION 14)

Parameter names follow the reference's module tree so its state dicts load.
The device path (C4FramePipeline) mirrors lib/core/test.py im_detect_all for a
non-FPN model: no blob padding (blob.py:104-114 pads only with FPN_ON), one
proposal level through the large-candidate vd_generate_proposals
(TEST.RPN_PRE_NMS_TOP_N 6000), RoIAlign with the adaptive sampling ratio
(sr 0, roi_align_kernel.cu:98-101) on the NHWC res4 map.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .engine import FramePipeline
from .modeling import (Bottleneck, FastRCNNOutputs, Generalized_RCNN, MaskRCNNOutputs,
                       ResNetBody, _conv_epi, generate_anchors, prepare_bottlenecks,
                       prepare_resnet_body)


def _conv4_counts(conv_body: str):
    return {"ResNet.ResNet50_conv4_body": (3, 4, 6),
            "ResNet.ResNet101_conv4_body": (3, 4, 23)}[conv_body]


class ResNetConv4Body(ResNetBody):
    """ResNet.py ResNet_convX_body with convX = 4 (:40-116): output res4, 1/16."""

    def __init__(self, cfg):
        r = cfg.RESNETS
        super().__init__(_conv4_counts(cfg.MODEL.CONV_BODY), r.NUM_GROUPS, r.WIDTH_PER_GROUP,
                         r.STRIDE_1X1)
        self.spatial_scale = 1. / 16.

    def forward(self, x):
        for i in range(self.convX):
            x = getattr(self, "res%d" % (i + 1))(x)
        return x


class SingleScaleRPNOutputs(nn.Module):
    """rpn_heads.single_scale_rpn_outputs (:37-126), sigmoid activation."""

    def __init__(self, dim_in, num_anchors):
        super().__init__()
        self.RPN_conv = nn.Conv2d(dim_in, dim_in, 3, 1, 1)  # RPN.OUT_DIM_AS_IN_DIM
        self.RPN_cls_score = nn.Conv2d(dim_in, num_anchors, 1, 1, 0)
        self.RPN_bbox_pred = nn.Conv2d(dim_in, num_anchors * 4, 1, 1, 0)
        self.epilogue = False

    def outputs(self, x):
        h = _conv_epi(self.RPN_conv, x) if (self.epilogue and x.is_cuda) else \
            F.relu(self.RPN_conv(x))
        return torch.sigmoid(self.RPN_cls_score(h)), self.RPN_bbox_pred(h)


def _res5_stage(dim_in, cfg, stride_init):
    """ResNet.py add_stage(dim_in, 2048, dim_bottleneck * 8, 3, stride_init) (:158-173)."""
    r = cfg.RESNETS
    inner = r.NUM_GROUPS * r.WIDTH_PER_GROUP * 8
    blocks, d = [], dim_in
    for b in range(3):
        blocks.append(Bottleneck(d, 2048, inner, stride_init if b == 0 else 1, r.NUM_GROUPS,
                                 r.STRIDE_1X1))
        d = 2048
    return nn.Sequential(*blocks)


class ResNetRoIConv5Head(nn.Module):
    """ResNet.ResNet_roi_conv5_head (ResNet.py:118-155)."""

    def __init__(self, dim_in, roi_xform, spatial_scale, cfg):
        super().__init__()
        self.roi_xform = roi_xform
        self.spatial_scale = spatial_scale
        self.cfg = cfg
        self.res5 = _res5_stage(dim_in, cfg, cfg.FAST_RCNN.ROI_XFORM_RESOLUTION // 7)
        self.avgpool = nn.AvgPool2d(7)
        self.dim_out = 2048

    def prepare(self):
        prepare_bottlenecks(self.res5)

    def head(self, x):
        """RoI features (R x 1024 x 14 x 14, any memory format) -> R x 2048."""
        return self.avgpool(self.res5(x)).flatten(1)

    def forward(self, x, rpn_ret):
        c = self.cfg.FAST_RCNN
        x = self.roi_xform(x, rpn_ret, blob_rois="rois", method=c.ROI_XFORM_METHOD,
                           resolution=c.ROI_XFORM_RESOLUTION, spatial_scale=self.spatial_scale,
                           sampling_ratio=c.ROI_XFORM_SAMPLING_RATIO)
        return self.avgpool(self.res5(x))


class MaskHeadV0upshare(nn.Module):
    """mask_rcnn_heads.mask_rcnn_fcn_head_v0upshare (:263-331): res5 shared with
    the box head (share_res5_module), upconv5 2x2 stride 2 + ReLU."""

    SHARE_RES5 = True

    def __init__(self, dim_in, roi_xform, spatial_scale, cfg):
        super().__init__()
        self.roi_xform = roi_xform
        self.spatial_scale = spatial_scale
        self.cfg = cfg
        self.res5 = None
        self.dim_out = cfg.MRCNN.DIM_REDUCED
        self.upconv5 = nn.ConvTranspose2d(2048, self.dim_out, 2, 2, 0)

    def share_res5_module(self, res5_target):
        self.res5 = res5_target

    def prepare(self):
        pass  # res5 is prepared through the box head

    def head(self, x):
        h = self.res5(x)
        if (h.is_cuda and h.dim() == 4 and h.is_contiguous(memory_format=torch.channels_last)
                and os.environ.get("VOSDET_C4_UPCONV_GEMM", "1") != "0"):
            y = self._upconv_gemm(h)
            if y is not None:
                return y
        return F.relu(self.upconv5(h))

    def _upconv_gemm(self, h):
        """upconv5 (ConvTranspose2d k 2, s 2: no overlapping taps) + ReLU as ONE GEMM
        [R H W, 2048] x [2048, 2 x 2 x 256] with the bias + ReLU epilogue (the split-bf16
        kernel; MIOpen's transposed conv took 3.6 ms per 16-frame step), then the
        depth-to-space shuffle; None where no GEMM serves the shape."""
        w = self.upconv5.weight  # Cin x Cout x 2 x 2
        key = (w.data_ptr(), w._version)
        if getattr(self, "_vd_up_key", None) != key:
            self._vd_up_wt = w.detach().permute(2, 3, 1, 0).reshape(4 * w.shape[1],
                                                                    w.shape[0]).contiguous()
            self._vd_up_b = self.upconv5.bias.detach().repeat(4).contiguous()
            self._vd_up_key = key
        R, C, H, W = h.shape
        y = ops.gemm_bias_act(h.permute(0, 2, 3, 1).reshape(R * H * W, C), self._vd_up_wt,
                              self._vd_up_b, relu=True)
        if y is None:
            return None
        co = self._vd_up_wt.shape[0] // 4
        y = y.view(R, H, W, 2, 2, co).permute(0, 1, 3, 2, 4, 5).reshape(R, 2 * H, 2 * W, co)
        return y.permute(0, 3, 1, 2)

    def forward(self, x, rpn_ret):
        c = self.cfg.MRCNN
        x = self.roi_xform(x, rpn_ret, blob_rois="mask_rois", method=c.ROI_XFORM_METHOD,
                           resolution=c.ROI_XFORM_RESOLUTION, spatial_scale=self.spatial_scale,
                           sampling_ratio=c.ROI_XFORM_SAMPLING_RATIO)
        return self.head(x)


class Generalized_RCNN_C4(nn.Module):
    """lib/modeling/model_builder.py:71-369 with FPN.FPN_ON False (inference)."""

    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.Conv_Body = ResNetConv4Body(cfg)
        anchors = generate_anchors(stride=1. / self.Conv_Body.spatial_scale,
                                   sizes=cfg.RPN.SIZES, aspect_ratios=cfg.RPN.ASPECT_RATIOS)
        self.RPN = SingleScaleRPNOutputs(self.Conv_Body.dim_out, anchors.shape[0])
        self.Box_Head = ResNetRoIConv5Head(self.Conv_Body.dim_out, self.roi_feature_transform,
                                           self.Conv_Body.spatial_scale, cfg)
        self.Box_Outs = FastRCNNOutputs(self.Box_Head.dim_out, cfg.MODEL.NUM_CLASSES,
                                        cfg.MODEL.CLS_AGNOSTIC_BBOX_REG)
        self.Mask_Head = MaskHeadV0upshare(self.Conv_Body.dim_out, self.roi_feature_transform,
                                           self.Conv_Body.spatial_scale, cfg)
        self.Mask_Head.share_res5_module(self.Box_Head.res5)  # model_builder.py:112-113
        self.Mask_Outs = MaskRCNNOutputs(
            self.Mask_Head.dim_out, cfg.MODEL.NUM_CLASSES if cfg.MRCNN.CLS_SPECIFIC_MASK else 1)
        self.register_buffer("anchors", torch.from_numpy(anchors), persistent=False)

    # the reference's single-blob branch of roi_feature_transform (:304-322)
    roi_feature_transform = Generalized_RCNN.roi_feature_transform

    @torch.no_grad()
    def fold_affine(self, epilogue: bool = True):
        prepare_resnet_body(self.Conv_Body, epilogue)
        self.RPN.epilogue = epilogue
        self.Box_Head.prepare()
        return self


class C4FramePipeline(FramePipeline):
    """Device-resident im_detect_all (lib/core/test.py:50-111) for the C4 family:

      u8 frames --vd_image_to_blob (no padding)--> res1..res4 --> RPN convs
      --> vd_generate_proposals (1 level, 15 anchors, pre 6000 / post 1000)
      --> vd_roi_align_fpn (1 level, NHWC res4, 14x14, adaptive sr) --> res5 +
      avgpool + cls/bbox --> vd_box_detections --> [detection counts D2H] -->
      mask RoIAlign 14x14 --> shared res5 --> upconv5 + ReLU --> class-selected
      14x14 masks.
    """
    ASYNC = False  # run() always reads the counts (the C4 mask batch is host-sized)

    def __init__(self, model, cfg, frame_hw=(800, 1333), batch=1, channels_last=False,
                 det_cap=256, device="cuda"):
        super().__init__(model, cfg, frame_hw, batch, channels_last, det_cap, device)
        self.Hp, self.Wp = self.Hr, self.Wr  # get_max_shape pads only with FPN_ON
        F_ = batch
        self.im_info = torch.tensor([[self.Hp, self.Wp, self.im_scale]] * F_,
                                    dtype=torch.float32, device=self.device)
        self.anchors = [model.anchors.to(self.device)]
        self.scale = model.Conv_Body.spatial_scale

    def backbone(self, frames):
        return self.model.Conv_Body(self.make_blob(frames))

    def _roi_feat(self, res4_nhwc, rois, res, sr, order=None):
        lvl = torch.zeros((rois.shape[0],), dtype=torch.int32, device=self.device)
        out = ops.roi_align_fpn([res4_nhwc], [self.scale], rois, lvl, res, sr,
                                roi_order=order, out_layout="nhwc")
        return out.permute(0, 3, 1, 2)  # NCHW view, channels_last memory

    def _run(self, frames: torch.Tensor, keep_intermediates: bool = False, sync: bool = True):
        # the C4 family sizes its mask batch from the host counts (one read after
        # the box stage); sync is accepted for the FramePipeline interface
        cfg, tst = self.cfg, self.cfg.TEST
        F_ = frames.shape[0]
        res4 = self.backbone(frames)
        self._mark("conv_body")
        prob, delta = self.model.RPN.outputs(res4)
        lrois, lprobs, lcnt = ops.generate_proposals(
            [prob.contiguous()], [delta.contiguous()], self.anchors, [self.scale],
            self.im_info[:F_], tst.RPN_PRE_NMS_TOP_N, tst.RPN_POST_NMS_TOP_N,
            tst.RPN_NMS_THRESH, tst.RPN_MIN_SIZE)
        self._mark("proposals")
        post = tst.RPN_POST_NMS_TOP_N
        rois, rcnt = lrois[:, 0].contiguous(), lcnt[:, 0].contiguous()
        res4_nhwc = res4.permute(0, 2, 3, 1)
        if not res4_nhwc.is_contiguous():
            res4_nhwc = ops.nchw_to_nhwc(res4)
        # padded proposal slots (count < post) are zero RoIs whose scores are
        # ignored by vd_box_detections (roi_count)
        flat = rois.view(-1, 5)
        fr = cfg.FAST_RCNN
        bf = self._roi_feat(res4_nhwc, flat, fr.ROI_XFORM_RESOLUTION, fr.ROI_XFORM_SAMPLING_RATIO)
        x = self.model.Box_Head.head(bf)
        cls_prob, bbox_pred = self.model.Box_Outs(x)
        self._mark("box_head")
        K = cls_prob.shape[1]
        bbox_pred = self.model.Box_Outs.per_class_deltas(bbox_pred, K)
        dets, dcls, dcnt = ops.box_detections(
            rois, cls_prob.view(F_, post, K), bbox_pred.view(F_, post, 4 * K), rcnt,
            self.im_scale_t[:F_], self.im_hw[:F_], tst.SCORE_THRESH, tst.NMS,
            tst.DETECTIONS_PER_IM, cfg.MODEL.BBOX_REG_WEIGHTS, self.det_cap,
            nms_cross_class=tst.NMS_CROSS_CLASS, num_det_per_class_pre=tst.NUM_DET_PER_CLASS_PRE)
        counts = dcnt.cpu().tolist()
        ops.raise_on_failed_counts(counts)
        self._mark("misc_bbox")
        if max(counts) > self.det_cap:
            raise RuntimeError("detections exceed det_cap=%d: %s" % (self.det_cap, counts))
        out = {"dets": dets, "classes": dcls, "counts": dcnt, "counts_host": counts,
               "rois": rois, "roi_counts": rcnt, "cls_prob": cls_prob, "bbox_pred": bbox_pred}
        if keep_intermediates:
            out.update(feats=res4, rpn_probs=[prob], rpn_deltas=[delta])
        M = sum(counts)
        R = cfg.MRCNN.RESOLUTION
        if M == 0:
            out["masks"] = torch.zeros((0, R, R), device=self.device)
            return out
        sel = torch.cat([torch.arange(c, device=self.device) + f * self.det_cap
                         for f, c in enumerate(counts)])
        d = dets.view(-1, 5).index_select(0, sel)
        bidx = torch.cat([torch.full((c,), f, dtype=torch.float32, device=self.device)
                          for f, c in enumerate(counts)])
        boxes = (d[:, :4].double() * self.im_scale).float()  # _get_rois_blob, test.py:877-906
        mrois = torch.cat([bidx[:, None], boxes], 1).contiguous()
        mcls = dcls.view(-1).index_select(0, sel)
        mc = cfg.MRCNN
        mf = self._roi_feat(res4_nhwc, mrois, mc.ROI_XFORM_RESOLUTION,
                            mc.ROI_XFORM_SAMPLING_RATIO)
        y = self.model.Mask_Head.head(mf)
        out["masks"] = self.model.Mask_Outs.selected(y, mcls)
        out["mask_rois"] = mrois
        out["mask_feat"] = mf
        self._mark("im_detect_mask")
        return out
