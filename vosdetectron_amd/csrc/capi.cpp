// extern "C" surface of libvosdet.so (declared in include/vosdet.h).
// Argument validation happens here; the kernels assume validated shapes.
#include <hip/hip_runtime.h>

#include "vosdet_internal.hpp"

using namespace vd;

#define VD_STREAM(s) reinterpret_cast<hipStream_t>(s)

extern "C" {

int vd_version(void) { return 1; }

const char *vd_status_string(int status) {
    switch (status) {
        case VD_OK: return "ok";
        case VD_ERR_ARG: return "invalid argument";
        case VD_ERR_SHAPE: return "unsupported shape";
        case VD_ERR_LAUNCH: return "kernel launch failed";
        case VD_ERR_WORKSPACE: return "workspace too small";
        default: return "unknown status";
    }
}

static bool bad_feat(const void *p, int B, int C, int H, int W) {
    return !p || B < 1 || C < 1 || H < 1 || W < 1;
}

int vd_roi_align_forward(int ah, int aw, float spatial_scale, int sampling_ratio,
                         const float *features, int B, int C, int H, int W, const float *rois,
                         int num_rois, int roi_cols, float *output, void *stream) {
    if (roi_cols != 5) return VD_ERR_ARG;
    if (num_rois == 0) return VD_OK;
    if (bad_feat(features, B, C, H, W) || !rois || !output || ah < 1 || aw < 1 || num_rois < 0)
        return VD_ERR_ARG;
    return launch_roi_align_fwd_nchw(features, B, C, H, W, rois, num_rois, ah, aw, spatial_scale,
                                     sampling_ratio, output, VD_STREAM(stream));
}

int vd_roi_align_backward(int ah, int aw, float spatial_scale, int sampling_ratio,
                          const float *top_grad, int B, int C, int H, int W, const float *rois,
                          int num_rois, int roi_cols, float *bottom_grad, void *stream) {
    if (roi_cols != 5) return VD_ERR_ARG;
    if (num_rois == 0) return VD_OK;
    if (bad_feat(bottom_grad, B, C, H, W) || !rois || !top_grad || ah < 1 || aw < 1)
        return VD_ERR_ARG;
    return launch_roi_align_bwd_nchw(top_grad, B, C, H, W, rois, num_rois, ah, aw, spatial_scale,
                                     sampling_ratio, bottom_grad, VD_STREAM(stream));
}

static int fpn_levels(const VdFeatLevel *levels, int num_levels, int B, int C, int num_rois,
                      FpnLevels &fa) {
    if (!levels || num_levels < 1 || num_levels > VD_MAX_LEVELS || B < 1 || C < 1 ||
        num_rois < 0)
        return VD_ERR_ARG;
    fa = FpnLevels{};
    for (int l = 0; l < num_levels; ++l) {
        if (bad_feat(levels[l].data, B, C, levels[l].H, levels[l].W)) return VD_ERR_ARG;
        fa.feat[l] = levels[l].data;
        fa.H[l] = levels[l].H;
        fa.W[l] = levels[l].W;
        fa.scale[l] = levels[l].spatial_scale;
    }
    fa.L = num_levels;
    fa.B = B;
    fa.R = num_rois;
    return VD_OK;
}

int vd_roi_align_fpn_forward(const VdFeatLevel *levels, int num_levels, int B, int C, int layout,
                             const float *rois, const int32_t *roi_level,
                             const int32_t *roi_order, int num_rois, int ah, int aw,
                             int sampling_ratio, int output_layout, float *output,
                             void *stream) {
    if (num_rois == 0) return VD_OK;
    if (!rois || !output || ah < 1 || aw < 1) return VD_ERR_ARG;
    if (num_levels > 1 && !roi_level) return VD_ERR_ARG;
    FpnLevels fa;
    const int st = fpn_levels(levels, num_levels, B, C, num_rois, fa);
    if (st != VD_OK) return st;
    if (output_layout != VD_LAYOUT_NCHW && output_layout != VD_LAYOUT_NHWC) return VD_ERR_ARG;
    if (layout == VD_LAYOUT_NHWC)
        return launch_roi_align_fpn_nhwc(fa, C, rois, roi_level, roi_order, num_rois, ah, aw,
                                         sampling_ratio, output_layout == VD_LAYOUT_NHWC, output,
                                         VD_STREAM(stream));
    if (layout != VD_LAYOUT_NCHW || output_layout != VD_LAYOUT_NCHW) return VD_ERR_ARG;
    if (num_levels != 1) return VD_ERR_SHAPE;  // multi-level NCHW: use per-level calls
    return launch_roi_align_fwd_nchw(fa.feat[0], B, C, fa.H[0], fa.W[0], rois, num_rois, ah, aw,
                                     fa.scale[0], sampling_ratio, output, VD_STREAM(stream));
}

size_t vd_roi_align_fpn_tiled_workspace_size(const VdFeatLevel *levels, int num_levels, int B,
                                             int C, int num_rois, int aligned_size) {
    FpnLevels fa;
    if (aligned_size < 1 || fpn_levels(levels, num_levels, B, C, num_rois, fa) != VD_OK) return 0;
    return roi_align_tiled_workspace_bytes(fa, num_rois, aligned_size, C);
}

int vd_roi_align_fpn_tiled_forward(const VdFeatLevel *levels, int num_levels, int B, int C,
                                   const float *rois, const int32_t *roi_level, int num_rois,
                                   int aligned_size, int sampling_ratio, float *output,
                                   void *workspace, size_t workspace_bytes, void *stream) {
    if (num_rois == 0) return VD_OK;
    if (!rois || !output || aligned_size < 1) return VD_ERR_ARG;
    if (num_levels > 1 && !roi_level) return VD_ERR_ARG;
    FpnLevels fa;
    const int st = fpn_levels(levels, num_levels, B, C, num_rois, fa);
    if (st != VD_OK) return st;
    if (B > 64 || !roi_align_tiled_supported(fa, C, aligned_size, sampling_ratio))
        return VD_ERR_SHAPE;
    return launch_roi_align_fpn_tiled(fa, C, rois, roi_level, num_rois, aligned_size,
                                      sampling_ratio, output, workspace, workspace_bytes,
                                      VD_STREAM(stream));
}

size_t vd_gemm_workspace_size(void) { return gemm_epi_workspace_bytes(); }

int vd_gemm_plans_key(char *buf, int n) {
    if (!buf || n < 16) return VD_ERR_ARG;
    return gemm_plans_key(buf, n);
}

int vd_gemm_plan_list(char *buf, int n) { return gemm_plan_list(buf, n); }

int vd_gemm_bias_act(const float *A, int M, int K, const float *W, int N, const float *bias,
                     const float *residual, int relu, float *D, void *workspace,
                     size_t workspace_bytes, void *stream) {
    if (M < 0 || K < 1 || N < 1 || !W || !bias || !D || (M > 0 && !A)) return VD_ERR_ARG;
    return launch_gemm_bias_act(A, M, K, W, N, bias, residual, relu, D, workspace,
                                workspace_bytes, VD_STREAM(stream));
}

size_t vd_gemm_split3_weight_size(int N, int K) {
    return (N > 0 && K > 0 && gemm_split3_supported(K, N)) ? gemm_split3_weight_bytes(N, K) : 0;
}

int vd_gemm_split3_weight(const float *W, int N, int K, void *Wp, void *stream) {
    if (N < 1 || K < 1 || !W || !Wp) return VD_ERR_ARG;
    return launch_gemm_split3_weight(W, N, K, Wp, VD_STREAM(stream));
}

int vd_gemm_split3_bias_act(const float *A, int M, int K, const float *A2, int K2,
                            const float *a_bias, const void *Wp, int N, const float *bias,
                            const float *residual, int up_h, int up_w, int sub_h, int sub_w,
                            int relu, float *D, int cfg, void *stream) {
    if (M < 0 || K < 1 || N < 1 || !Wp || !bias || !D || (M > 0 && !A) || cfg < 0 || cfg > 19)
        return VD_ERR_ARG;
    return launch_gemm_split3(A, M, K, A2, K2, Wp, N, bias, residual, up_h, up_w, sub_h, sub_w,
                              relu, D, cfg, VD_STREAM(stream), a_bias);
}

int vd_mask_head_upconv_logits(const float *X, int M, int K, const void *Wp, const float *bias,
                               const float *cls_w, const float *cls_b, const int32_t *roi_ch,
                               int P, float *masks, void *stream) {
    if (M < 0 || K < 1 || P < 1 || !Wp || !bias || !masks || (M > 0 && !X)) return VD_ERR_ARG;
    return launch_gemm_split3_mask_logits(X, M, K, Wp, 1024, bias, cls_w, cls_b, roi_ch, P, masks,
                                          VD_STREAM(stream));
}

int vd_conv3x3_bias_act(const float *X, int N, int H, int W, int C, const float *W2, int Cout,
                        const float *bias, int relu, float *Y, void *stream) {
    if (N < 0 || H < 1 || W < 1 || C < 1 || Cout < 1 || !W2 || !Y || (N > 0 && !X))
        return VD_ERR_ARG;
    return launch_conv3x3_mfma(X, N, H, W, C, W2, Cout, bias, relu, Y, VD_STREAM(stream));
}

int vd_conv3x3_wino_weight(const float *w, int Cout, int Cin, float *U, void *stream) {
    if (Cout < 1 || Cin < 1 || !w || !U) return VD_ERR_ARG;
    return launch_conv3x3_wino_weight(w, Cout, Cin, U, VD_STREAM(stream));
}

int vd_conv3x3_wino_bias_act(const float *X, int N, int H, int W, int C, const float *U,
                             int Cout, const float *bias, int relu, float *Y, void *stream) {
    if (N < 0 || H < 1 || W < 1 || C < 1 || Cout < 1 || !U || !Y || (N > 0 && !X))
        return VD_ERR_ARG;
    return launch_conv3x3_wino(X, N, H, W, C, U, Cout, bias, relu, Y, VD_STREAM(stream));
}

int vd_conv3x3_wino4_weight(const float *w, int Cout, int Cin, float *U, void *stream) {
    if (Cout < 1 || Cin < 1 || !w || !U) return VD_ERR_ARG;
    return launch_conv3x3_wino4_weight(w, Cout, Cin, U, VD_STREAM(stream));
}

int vd_conv3x3_wino4_bias_act(const float *X, int N, int H, int W, int C, const float *U,
                              int Cout, const float *bias, int relu, float *Y, void *stream) {
    if (N < 0 || H < 1 || W < 1 || C < 1 || Cout < 1 || !U || !Y || (N > 0 && !X))
        return VD_ERR_ARG;
    return launch_conv3x3_wino4(X, N, H, W, C, U, Cout, bias, relu, Y, VD_STREAM(stream));
}

int vd_conv3x3_wino4_mosaic_bias_act(const float *X, int N, int H, int W, int C, const float *U,
                                     int Cout, const float *bias, int relu, float *Y,
                                     void *stream) {
    if (N < 0 || H < 1 || W < 1 || C < 1 || Cout < 1 || !U || !Y || (N > 0 && !X))
        return VD_ERR_ARG;
    return launch_conv3x3_wino4(X, N, H, W, C, U, Cout, bias, relu, Y, VD_STREAM(stream), 1);
}

int vd_conv3x3_wino4_rows_bias_act(const float *X, int N, int H, int W, int C, const float *U,
                                   int Cout, const float *bias, int relu, float *Y,
                                   void *stream) {
    if (N < 0 || H < 1 || W < 1 || C < 1 || Cout < 1 || !U || !Y || (N > 0 && !X))
        return VD_ERR_ARG;
    return launch_conv3x3_wino4(X, N, H, W, C, U, Cout, bias, relu, Y, VD_STREAM(stream), 2);
}

int vd_conv3x3_wino4_grouped_bias_act(const float *X, int N, int H, int W, int C,
                                      const float *U, int groups, const float *bias, int relu,
                                      float *Y, int rows, void *stream) {
    if (N < 0 || H < 1 || W < 1 || C < 1 || groups < 1 || !U || !Y || (N > 0 && !X))
        return VD_ERR_ARG;
    return launch_conv3x3_wino4(X, N, H, W, C, U, C, bias, relu, Y, VD_STREAM(stream),
                                rows ? 2 : 0, groups);
}

int vd_conv3x3_wino4_dilated2_bias_act(const float *X, int N, int H, int W, int C,
                                       const float *U, int Cout, const float *bias, int relu,
                                       float *Y, int layout, void *stream) {
    if (N < 0 || H < 2 || W < 2 || (H & 1) || (W & 1) || C < 1 || Cout < 1 || !U || !Y ||
        (N > 0 && !X))
        return VD_ERR_ARG;
    if ((int64_t)N * H * W == 0) return VD_OK;
    if ((int64_t)4 * N >= ((int64_t)1 << 30)) return VD_ERR_SHAPE;
    const int h = H / 2, w = W / 2;
    // layout of the sub-maps: 0 one per block, 1 pairs / octets (h, w <= 15), 2 the
    // shared-separator grid
    if (layout < 0 || layout > 2 || (layout == 1 && (h > 15 || w > 15))) return VD_ERR_ARG;
    return launch_conv3x3_wino4(X, 4 * N, h, w, C, U, Cout, bias, relu, Y, VD_STREAM(stream),
                                layout == 2 ? 4 : layout, -2);
}

int vd_conv3x3_wino4_grid_bias_act(const float *X, int N, int H, int W, int C, const float *U,
                                   int Cout, const float *bias, int relu, float *Y,
                                   void *stream) {
    if (N < 0 || H < 1 || W < 1 || C < 1 || Cout < 1 || !U || !Y || (N > 0 && !X))
        return VD_ERR_ARG;
    return launch_conv3x3_wino4(X, N, H, W, C, U, Cout, bias, relu, Y, VD_STREAM(stream), 4);
}

int vd_conv3x3_wino_seg_bias_act(const float *X, int H, int W, int C, const float *U, int Cout,
                                 const float *bias, int relu, int seg_h, float *Y, void *stream) {
    if (H < 1 || W < 1 || C < 1 || Cout < 1 || seg_h < 2 || !U || !Y || !X) return VD_ERR_ARG;
    return launch_conv3x3_wino(X, 1, H, W, C, U, Cout, bias, relu, Y, VD_STREAM(stream), seg_h);
}

int vd_conv3x3_wino_mosaic_bias_act(const float *X, int R, int H, int W, int C, const float *U,
                                    int Cout, const float *bias, int relu, float *Y, void *stream) {
    return launch_conv3x3_wino_mosaic(X, R, H, W, C, U, Cout, bias, relu, Y, VD_STREAM(stream));
}

int vd_fpn_lateral_weight(const float *W, int N, int K, float *Wf, void *stream) {
    if (!W || !Wf) return VD_ERR_ARG;
    return launch_fpn_lateral_weight(W, N, K, Wf, VD_STREAM(stream));
}

int vd_fpn_lateral_topdown(const float *A, int64_t M, int K, const float *Wf, int N,
                           const float *bias, const float *top, int H, int W, float *D,
                           void *stream) {
    if (M < 0 || !Wf || !bias || !D || (M > 0 && !A)) return VD_ERR_ARG;
    return launch_fpn_lateral(A, M, K, Wf, N, bias, top, H, W, D, VD_STREAM(stream));
}

int vd_gemm_dual_bias_act(const float *A1, int K1, const float *A2, int K2, int M, const float *W,
                          int N, const float *bias, int relu, float *D, void *stream) {
    if (M < 0 || K1 < 1 || K2 < 1 || N < 1 || !W || !bias || !D || (M > 0 && (!A1 || !A2)))
        return VD_ERR_ARG;
    return launch_gemm1x1_dual(A1, K1, A2, K2, M, W, N, bias, relu, D, VD_STREAM(stream));
}

int vd_roi_align_legacy_forward(int ah, int aw, float spatial_scale, const float *features,
                                int B, int C, int H, int W, const float *rois, int num_rois,
                                float *output, void *stream) {
    if (num_rois == 0) return VD_OK;
    if (bad_feat(features, B, C, H, W) || !rois || !output || num_rois < 0) return VD_ERR_ARG;
    if (H < 2 || W < 2) return VD_ERR_SHAPE;  // the kernel reads the 2x2 block at <= (H-2, W-2)
    return launch_roi_align_legacy_fwd(features, B, C, H, W, rois, num_rois, ah, aw,
                                       spatial_scale, output, VD_STREAM(stream));
}

int vd_roi_pool_forward(int ph, int pw, float spatial_scale, const float *features, int B, int C,
                        int H, int W, const float *rois, int num_rois, float *output,
                        int32_t *argmax, void *stream) {
    if (num_rois == 0) return VD_OK;
    if (bad_feat(features, B, C, H, W) || !rois || !output || ph < 1 || pw < 1 || num_rois < 0)
        return VD_ERR_ARG;
    return launch_roi_pool_fwd(features, B, C, H, W, rois, num_rois, ph, pw, spatial_scale,
                               output, argmax, VD_STREAM(stream));
}

int vd_roi_pool_backward(const float *top_grad, const int32_t *argmax, int64_t num_outputs,
                         float *bottom_grad, void *stream) {
    if (num_outputs == 0) return VD_OK;
    if (!top_grad || !argmax || !bottom_grad || num_outputs < 0) return VD_ERR_ARG;
    return launch_roi_pool_bwd(top_grad, argmax, num_outputs, bottom_grad, VD_STREAM(stream));
}

int vd_roi_crop_forward(const float *input, int B, int C, int H, int W, const float *grid_yx,
                        int num_rois, int GH, int GW, float *output, void *stream) {
    if (num_rois == 0) return VD_OK;
    if (bad_feat(input, B, C, H, W) || !grid_yx || !output || GH < 1 || GW < 1) return VD_ERR_ARG;
    return launch_roi_crop_fwd(input, B, C, H, W, grid_yx, num_rois, GH, GW, output,
                               VD_STREAM(stream));
}

size_t vd_nms_workspace_size(int n) { return nms_workspace_bytes(n); }

int vd_nms(const float *dets, int n, int det_stride, float thresh, int64_t *keep_out,
           int32_t *num_out, void *workspace, size_t workspace_bytes, void *stream) {
    if (!num_out || (n > 0 && (!dets || !keep_out))) return VD_ERR_ARG;
    return launch_nms(dets, n, det_stride, thresh, keep_out, num_out, workspace, workspace_bytes,
                      VD_STREAM(stream));
}

int vd_map_rois_to_fpn_levels(const float *rois, int roi_stride, int col0, int R, int k_min,
                              int k_max, float canonical_scale, float canonical_level,
                              int32_t *lvl_out, void *stream) {
    if (R == 0) return VD_OK;
    if (!rois || !lvl_out || R < 0 || roi_stride < col0 + 4 || col0 < 0 || k_min > k_max)
        return VD_ERR_ARG;
    return launch_map_levels(rois, roi_stride, col0, R, k_min, k_max, canonical_scale,
                             canonical_level, lvl_out, VD_STREAM(stream));
}

int vd_mask_rois(const float *dets, const int32_t *classes, const int32_t *counts,
                 int num_images, int det_cap, const double *im_scale, int row0, int rows,
                 int k_min, int k_max, float canonical_scale, float canonical_level,
                 float *rois_out, int32_t *lvl_out, int32_t *cls_out, int32_t *total_out,
                 void *stream) {
    if (num_images == 0 || (rows == 0 && !total_out)) return VD_OK;
    if (!dets || !classes || !counts || !im_scale || num_images < 0 || det_cap < 1 || row0 < 0 ||
        rows < 0 || k_min > k_max || (rows > 0 && (!rois_out || !lvl_out || !cls_out)))
        return VD_ERR_ARG;
    return launch_mask_rois(dets, classes, counts, num_images, det_cap, im_scale, row0, rows,
                            k_min, k_max, canonical_scale, canonical_level, rois_out, lvl_out,
                            cls_out, total_out, VD_STREAM(stream));
}

size_t vd_generate_proposals_workspace_size(const VdRpnLevel *levels, int num_levels,
                                            int num_images, int pre_nms_topN) {
    return rpn_workspace_bytes(levels, num_levels, num_images, pre_nms_topN);
}

int vd_generate_proposals(const VdRpnLevel *levels, int num_levels, int num_images,
                          const float *im_info, int pre_nms_topN, int post_nms_topN,
                          float nms_thresh, float min_size, float *rois_out, float *probs_out,
                          int32_t *counts_out, void *workspace, size_t workspace_bytes,
                          void *stream) {
    if (!levels || !im_info || !rois_out || !probs_out || !counts_out) return VD_ERR_ARG;
    for (int l = 0; l < num_levels && l < VD_MAX_LEVELS; ++l)
        if (!levels[l].cls_prob || !levels[l].bbox_pred || !levels[l].anchors ||
            levels[l].A < 1 || levels[l].H < 1 || levels[l].W < 1 ||
            !(levels[l].spatial_scale > 0.f))
            return VD_ERR_ARG;
    return launch_rpn_proposals(levels, num_levels, num_images, im_info, pre_nms_topN,
                                post_nms_topN, nms_thresh, min_size, rois_out, probs_out,
                                counts_out, workspace, workspace_bytes, VD_STREAM(stream));
}

int vd_collect_distribute(const float *level_rois, const float *level_probs,
                          const int32_t *level_counts, int num_levels, int level_cap,
                          int num_images, int post_nms_topN, int k_min, int k_max,
                          float *rois_out, int32_t *lvl_out, int32_t *count_out, void *stream) {
    if (!level_rois || !level_probs || !level_counts || !rois_out || !lvl_out || !count_out ||
        level_cap < 1 || k_min > k_max)
        return VD_ERR_ARG;
    return launch_collect_distribute(level_rois, level_probs, level_counts, num_levels,
                                     level_cap, num_images, post_nms_topN, k_min, k_max,
                                     rois_out, lvl_out, count_out, VD_STREAM(stream));
}

size_t vd_box_detections_workspace_size(int R_cap, int num_images, int num_classes) {
    return box_detections_workspace_bytes(R_cap, num_images, num_classes);
}

int vd_box_detections(const float *rois, const float *cls_prob, const float *bbox_pred,
                      const int32_t *roi_count, int R_cap, int num_images, int num_classes,
                      const float *im_scale, const int32_t *im_hw, float score_thresh,
                      float nms_thresh, int dets_per_im, const float *bbox_reg_weights,
                      int det_cap, float *dets_out, int32_t *det_cls_out,
                      int32_t *det_count_out, void *workspace, size_t workspace_bytes,
                      void *stream) {
    if (!rois || !cls_prob || !bbox_pred || !roi_count || !im_scale || !im_hw ||
        !bbox_reg_weights || !dets_out || !det_cls_out || !det_count_out)
        return VD_ERR_ARG;
    return launch_box_detections(rois, cls_prob, bbox_pred, roi_count, R_cap, num_images,
                                 num_classes, im_scale, im_hw, score_thresh, nms_thresh,
                                 dets_per_im, bbox_reg_weights, -1, 0.5f, 0.0001f, -1, 0.8f,
                                 1.0f, det_cap, dets_out, det_cls_out, det_count_out, workspace,
                                 workspace_bytes, VD_STREAM(stream));
}

int vd_box_detections_ex(const float *rois, const float *cls_prob, const float *bbox_pred,
                         const int32_t *roi_count, int R_cap, int num_images, int num_classes,
                         const float *im_scale, const int32_t *im_hw, float score_thresh,
                         float nms_thresh, int dets_per_im, const float *bbox_reg_weights,
                         int soft_nms_method, float soft_nms_sigma, float soft_nms_min_score,
                         int bbox_vote_method, float bbox_vote_thresh, float bbox_vote_beta,
                         int det_cap, float *dets_out, int32_t *det_cls_out,
                         int32_t *det_count_out, void *workspace, size_t workspace_bytes,
                         void *stream) {
    if (!rois || !cls_prob || !bbox_pred || !roi_count || !im_scale || !im_hw ||
        !bbox_reg_weights || !dets_out || !det_cls_out || !det_count_out)
        return VD_ERR_ARG;
    return launch_box_detections(rois, cls_prob, bbox_pred, roi_count, R_cap, num_images,
                                 num_classes, im_scale, im_hw, score_thresh, nms_thresh,
                                 dets_per_im, bbox_reg_weights, soft_nms_method, soft_nms_sigma,
                                 soft_nms_min_score, bbox_vote_method, bbox_vote_thresh,
                                 bbox_vote_beta, det_cap, dets_out, det_cls_out, det_count_out,
                                 workspace, workspace_bytes, VD_STREAM(stream));
}

size_t vd_stem_weight_size(void) { return stem_weight_floats() * sizeof(float); }

int vd_stem_weight_pack(const float *w, float *packed, void *stream) {
    if (!w || !packed) return VD_ERR_ARG;
    return launch_stem_weight(w, packed, VD_STREAM(stream));
}

int vd_stem_conv_pool(const float *x, int N, int H, int W, const float *packed, const float *bias,
                      float *y, void *stream) {
    if ((int64_t)N * H * W > 0 && (!x || !packed || !bias || !y)) return VD_ERR_ARG;
    return launch_stem_conv_pool(x, N, H, W, packed, bias, y, 0, VD_STREAM(stream));
}

size_t vd_stem_split_weight_size(void) { return stem_weight_split_bytes(); }

int vd_stem_split_weight_pack(const float *w, void *packed, void *stream) {
    if (!w || !packed) return VD_ERR_ARG;
    return launch_stem_weight_split(w, packed, VD_STREAM(stream));
}

int vd_stem_split_conv_pool(const float *x, int N, int H, int W, const void *packed,
                            const float *bias, float *y, void *stream) {
    if ((int64_t)N * H * W > 0 && (!x || !packed || !bias || !y)) return VD_ERR_ARG;
    return launch_stem_conv_pool(x, N, H, W, static_cast<const float *>(packed), bias, y, 0,
                                 VD_STREAM(stream), true);
}

int vd_soft_nms(const float *dets, int n, int dets_stride, float sigma, float overlap_thresh,
                float score_thresh, int method, float *dets_out, int64_t *keep_out,
                int32_t *count_out, void *stream) {
    if ((n > 0 && (!dets || !dets_out || !keep_out)) || !count_out) return VD_ERR_ARG;
    return launch_soft_nms(dets, n, dets_stride, sigma, overlap_thresh, score_thresh, method,
                           dets_out, keep_out, count_out, VD_STREAM(stream));
}

int vd_box_voting(const float *top_dets, int n_top, int top_stride, const float *all_dets,
                  int n_all, int all_stride, float thresh, int scoring_method, float beta,
                  float *out, void *stream) {
    if (n_top > 0 && (!top_dets || !all_dets || !out)) return VD_ERR_ARG;
    return launch_box_voting(top_dets, n_top, top_stride, all_dets, n_all, all_stride, thresh,
                             scoring_method, beta, out, VD_STREAM(stream));
}

int vd_image_to_blob(const uint8_t *frames, int F, int H, int W, const float *lut, int Hp,
                     int Wp, int nhwc, float *blob, void *stream) {
    if (!frames || !lut || !blob || H < 1 || W < 1) return VD_ERR_ARG;
    return launch_image_to_blob(frames, F, H, W, lut, Hp, Wp, nhwc, blob, VD_STREAM(stream));
}

int vd_image_resize_to_blob(const uint8_t *frames, int F, int H, int W, const float *lut,
                            double im_scale, int Hr, int Wr, int Hp, int Wp, int nhwc,
                            float *blob, void *stream) {
    if (!frames || !lut || !blob) return VD_ERR_ARG;
    return launch_resize_to_blob(frames, F, H, W, lut, im_scale, Hr, Wr, Hp, Wp, nhwc, blob,
                                 VD_STREAM(stream));
}

int vd_bias_act(float *x, const float *bias, const float *residual, const float *residual_bias,
                int N, int C, int H, int W, int nhwc, int residual_mode, int relu, void *stream) {
    if (!x || N < 1 || C < 1 || H < 1 || W < 1 || residual_mode < 0 || residual_mode > 2 ||
        (residual_mode && !residual))
        return VD_ERR_ARG;
    return launch_bias_act(x, bias, residual, residual_bias, (int64_t)N * C * H * W, C, H, W,
                           nhwc, residual_mode, relu, VD_STREAM(stream));
}

int vd_nchw_to_nhwc(const float *in, int B, int C, int H, int W, float *out, void *stream) {
    if (!in || !out) return VD_ERR_ARG;
    return launch_nchw_to_nhwc(in, B, C, H, W, out, VD_STREAM(stream));
}


// ---------------------------------------------------------------- VOS path
int vd_flow_align_forward(const float *features, const float *flow, int B, int C, int H, int W,
                          int layout, float *output, void *stream) {
    if (bad_feat(features, B, C, H, W) || !flow || !output) return VD_ERR_ARG;
    if (layout != VD_LAYOUT_NCHW && layout != VD_LAYOUT_NHWC) return VD_ERR_ARG;
    return launch_flow_align_fwd(features, flow, B, C, H, W, layout == VD_LAYOUT_NHWC, output,
                                 VD_STREAM(stream));
}

int vd_flow_align_backward(const float *top_grad, const float *features, const float *flow,
                           int B, int C, int H, int W, float *features_grad, float *flow_grad,
                           void *stream) {
    if (bad_feat(features, B, C, H, W) || !top_grad || !flow || !features_grad || !flow_grad)
        return VD_ERR_ARG;
    return launch_flow_align_bwd(top_grad, features, flow, B, C, H, W, features_grad, flow_grad,
                                 VD_STREAM(stream));
}

size_t vd_group_norm_workspace_size(int B, int G) { return gn_workspace_bytes(B, G, 1); }

static bool bad_gn(const float *x, int B, int C, int H, int W, int G, int layout) {
    if (bad_feat(x, B, C, H, W) || G < 1 || G > 64 || C % G) return true;
    if (layout != VD_LAYOUT_NCHW && layout != VD_LAYOUT_NHWC) return true;
    return false;
}

int vd_group_norm_act(const float *x, const float *x2, int B, int C, int H, int W, int G,
                      float eps, const float *gamma, const float *beta, const float *residual,
                      int residual_mode, const float *res_gamma, const float *res_beta, int act,
                      int layout, float *out, void *workspace, size_t ws_bytes, void *stream) {
    if (bad_gn(x, B, C, H, W, G, layout) || !gamma || !beta || !out || !workspace)
        return VD_ERR_ARG;
    if (residual_mode < 0 || residual_mode > 3 || act < 0 || act > 3) return VD_ERR_ARG;
    if (residual_mode && !residual) return VD_ERR_ARG;
    if (residual_mode == 3 && (!res_gamma || !res_beta)) return VD_ERR_ARG;
    if (residual_mode == 2 && ((H & 1) || (W & 1))) return VD_ERR_SHAPE;
    const int nsets = residual_mode == 3 ? 2 : 1;
    if (ws_bytes < gn_workspace_bytes(B, G, nsets)) return VD_ERR_WORKSPACE;
    double *ws = static_cast<double *>(workspace);
    const size_t per = (size_t)B * G * 2;
    GnSets sets = {};
    sets.s[0] = {x, x2, ws};
    sets.s[1] = {residual, nullptr, ws + per};
    hipStream_t s = VD_STREAM(stream);
    const int nhwc = layout == VD_LAYOUT_NHWC;
    int st = launch_gn_stats(sets, nsets, B, C, H * W, G, nhwc, s);
    if (st != VD_OK) return st;
    GnApply a = {};
    a.x = x;
    a.x2 = x2;
    a.ws = ws;
    a.gamma = gamma;
    a.beta = beta;
    a.res = residual;
    a.res_ws = residual_mode == 3 ? ws + per : nullptr;
    a.res_gamma = res_gamma;
    a.res_beta = res_beta;
    a.out = out;
    a.mode = VD_GN_ACT;
    a.act = act;
    a.res_mode = residual_mode;
    a.eps = eps;
    return launch_gn_apply(a, B, C, H, W, G, nhwc, s);
}

int vd_convgru_gates(const float *zh, const float *zx, const float *rh, const float *rx,
                     const float *h, int B, int C, int H, int W, int G, float eps,
                     const float *gamma_z, const float *beta_z, const float *gamma_r,
                     const float *beta_r, int layout, float *z, float *hr, void *workspace,
                     size_t ws_bytes, void *stream) {
    if (bad_gn(zx, B, C, H, W, G, layout) || !gamma_z || !beta_z || !z || !workspace)
        return VD_ERR_ARG;
    if (h && (!zh || !rh || !rx || !gamma_r || !beta_r || !hr)) return VD_ERR_ARG;
    if (ws_bytes < gn_workspace_bytes(B, G, 2)) return VD_ERR_WORKSPACE;
    double *ws = static_cast<double *>(workspace);
    const size_t per = (size_t)B * G * 2;
    GnSets sets = {};
    sets.s[0] = {zx, h ? zh : nullptr, ws};
    sets.s[1] = {rx, rh, ws + per};
    hipStream_t s = VD_STREAM(stream);
    const int nhwc = layout == VD_LAYOUT_NHWC;
    int st = launch_gn_stats(sets, h ? 2 : 1, B, C, H * W, G, nhwc, s);
    if (st != VD_OK) return st;
    GnApply a = {};
    a.x = zx;
    a.x2 = h ? zh : nullptr;
    a.ws = ws;
    a.gamma = gamma_z;
    a.beta = beta_z;
    a.out = z;
    a.mode = VD_GN_GRU_Z;
    a.eps = eps;
    st = launch_gn_apply(a, B, C, H, W, G, nhwc, s);
    if (st != VD_OK || !h) return st;
    a.x = rx;
    a.x2 = rh;
    a.ws = ws + per;
    a.gamma = gamma_r;
    a.beta = beta_r;
    a.res = h;
    a.out = hr;
    a.mode = VD_GN_GRU_R;
    return launch_gn_apply(a, B, C, H, W, G, nhwc, s);
}

int vd_convgru_update(const float *hh, const float *hx, const float *z, const float *h,
                      const float *finer, int B, int C, int H, int W, int G, float eps,
                      const float *gamma_h, const float *beta_h, int layout, float *out,
                      void *workspace, size_t ws_bytes, void *stream) {
    if (bad_gn(hx, B, C, H, W, G, layout) || !z || !gamma_h || !beta_h || !out || !workspace)
        return VD_ERR_ARG;
    if (h && !hh) return VD_ERR_ARG;
    if (ws_bytes < gn_workspace_bytes(B, G, 1)) return VD_ERR_WORKSPACE;
    GnSets sets = {};
    sets.s[0] = {hx, h ? hh : nullptr, static_cast<double *>(workspace)};
    hipStream_t s = VD_STREAM(stream);
    const int nhwc = layout == VD_LAYOUT_NHWC;
    int st = launch_gn_stats(sets, 1, B, C, H * W, G, nhwc, s);
    if (st != VD_OK) return st;
    GnApply a = {};
    a.x = hx;
    a.x2 = h ? hh : nullptr;
    a.ws = static_cast<double *>(workspace);
    a.gamma = gamma_h;
    a.beta = beta_h;
    a.res = h;
    a.z = z;
    a.finer = finer;
    a.out = out;
    a.mode = VD_GN_GRU_H;
    a.eps = eps;
    return launch_gn_apply(a, B, C, H, W, G, nhwc, s);
}

int vd_paste_masks(const float *masks, int M, int R, const float *boxes, int box_stride,
                   int im_h, int im_w, float thresh, uint8_t *out, void *stream) {
    if (M == 0) return VD_OK;
    if (!masks || !boxes || !out || M < 0 || R < 1 || box_stride < 4 || im_h < 1 || im_w < 1)
        return VD_ERR_ARG;
    return launch_paste_masks(masks, M, R, boxes, box_stride, im_h, im_w, thresh, out,
                              VD_STREAM(stream));
}

int vd_mask_rle(const uint8_t *masks, int M, int H, int W, uint32_t *counts, int cap,
                int32_t *ncounts, void *stream) {
    if (M == 0) return VD_OK;
    if (!masks || !counts || !ncounts || M < 0 || H < 1 || W < 1 || cap < 1 ||
        (int64_t)H * W > 0xffffffffll)
        return VD_ERR_ARG;
    return launch_mask_rle(masks, M, H, W, counts, cap, ncounts, VD_STREAM(stream));
}

int vd_segm_rle(const float *masks, int M, int R, const float *boxes, int box_stride,
                int im_h, int im_w, float thresh, uint32_t *counts, int cap, int32_t *ncounts,
                void *stream) {
    if (M == 0) return VD_OK;
    if (!masks || !boxes || !counts || !ncounts || M < 0 || R < 1 || box_stride < 4 ||
        im_h < 1 || im_w < 1 || cap < 1 || (int64_t)im_h * im_w > 0xffffffffll)
        return VD_ERR_ARG;
    return launch_segm_rle(masks, M, R, boxes, box_stride, im_h, im_w, thresh, counts, cap,
                           ncounts, VD_STREAM(stream));
}

int vd_rle_strings(const uint32_t *counts, const int32_t *ncounts, int M, int cap,
                   int32_t *lens, uint8_t *chars, void *stream) {
    if (M == 0) return VD_OK;
    if (!counts || !ncounts || !lens || M < 0 || cap < 1) return VD_ERR_ARG;
    return launch_rle_strings(counts, ncounts, M, cap, lens, chars, VD_STREAM(stream));
}

int vd_bias_relu_maxpool(const float *x, const float *bias, int N, int C, int H, int W,
                         float *out, void *stream) {
    if (!x || !bias || !out || N < 0 || C < 0 || H < 0 || W < 0) return VD_ERR_ARG;
    return launch_bias_relu_maxpool(x, bias, N, C, H, W, out, VD_STREAM(stream));
}

int vd_rpn_head(const float *x, const float *conv_bias, const float *w, const float *b, int N,
                int H, int W, int C, int A, float *cls_prob, float *bbox_pred, void *stream) {
    if (!x || !conv_bias || !w || !b || !cls_prob || !bbox_pred || N < 0 || H < 0 || W < 0)
        return VD_ERR_ARG;
    return launch_rpn_head(x, conv_bias, w, b, N, H, W, C, A, cls_prob, bbox_pred,
                           VD_STREAM(stream));
}

int vd_detections_postfilter(float *dets, int32_t *classes, int32_t *counts, int num_images,
                             int det_cap, float nms_cross_class, int num_det_per_class_pre,
                             void *stream) {
    if (!dets || !classes || !counts) return VD_ERR_ARG;
    return launch_detections_postfilter(dets, classes, counts, num_images, det_cap,
                                        nms_cross_class, num_det_per_class_pre,
                                        VD_STREAM(stream));
}

size_t vd_mask_iou_nms_workspace_size(int n, int im_h, int im_w) {
    return mask_iou_nms_workspace_bytes(n, im_h, im_w);
}

int vd_mask_iou_nms(const uint8_t *planes, int n, int im_h, int im_w, const float *dets,
                    int det_stride, const int32_t *classes, double iou_th, int max_per_class,
                    int64_t *keep_out, int32_t *num_out, void *workspace, size_t workspace_bytes,
                    void *stream) {
    if (n < 0 || !num_out || (n > 0 && (!planes || !dets || !classes || !keep_out)))
        return VD_ERR_ARG;
    return launch_mask_iou_nms(planes, n, im_h, im_w, dets, det_stride, classes, iou_th,
                               max_per_class, keep_out, num_out, workspace, workspace_bytes,
                               VD_STREAM(stream));
}

int vd_detections_prev_box_filter(float *dets, int32_t *classes, int32_t *counts, int F,
                                  int det_cap, const float *prev_dets,
                                  const int32_t *prev_classes, const int32_t *prev_counts,
                                  int prev_cap, float iou_thresh, float score_thresh,
                                  void *stream) {
    if (F < 0 || (F > 0 && (!dets || !classes || !counts || !prev_counts ||
                            (prev_cap > 0 && (!prev_dets || !prev_classes)))))
        return VD_ERR_ARG;
    return launch_prev_box_filter(dets, classes, counts, F, det_cap, prev_dets, prev_classes,
                                  prev_counts, prev_cap, iou_thresh, score_thresh,
                                  VD_STREAM(stream));
}

}  // extern "C"
