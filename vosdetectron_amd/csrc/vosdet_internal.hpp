// Internal launcher declarations shared between the kernel translation units
// and the C-ABI (capi.cpp).  Not part of the public interface (include/vosdet.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vosdet.h"

namespace vd {

struct FpnLevels {
    const float *feat[VD_MAX_LEVELS];
    int H[VD_MAX_LEVELS];
    int W[VD_MAX_LEVELS];
    float scale[VD_MAX_LEVELS];
    int L;  // levels in use
    int B;  // images per level
    int R;  // RoIs of the launch (bounds roi_order entries)
};

// Zero `bytes` at p with a kernel on stream s.  Used instead of
// hipMemsetAsync for workspaces a captured step re-zeroes: on this ROCm a captured
// hipMemsetAsync did not run again at hipGraph replay (the radix select's counters
// kept the previous replay's values; tools/research/graph_prop_dbg.py, round 5).
int zero_async(void *p, size_t bytes, hipStream_t s);

int launch_roi_align_fwd_nchw(const float *feat, int B, int C, int H, int W, const float *rois,
                              int R, int PH, int PW, float scale, int sr, float *out,
                              hipStream_t s);
int launch_roi_align_bwd_nchw(const float *top_diff, int B, int C, int H, int W,
                              const float *rois, int R, int PH, int PW, float scale, int sr,
                              float *bottom_diff, hipStream_t s);
int launch_roi_align_fpn_nhwc(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                              const int *order, int R, int PH, int PW, int sr, int out_nhwc,
                              float *out, hipStream_t s);

bool roi_align_tiled_supported(const FpnLevels &fa, int C, int P, int sr);
size_t roi_align_tiled_workspace_bytes(const FpnLevels &fa, int R, int P, int C);
int launch_roi_align_fpn_tiled(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                               int R, int P, int sr, float *out, void *ws, size_t ws_bytes,
                               hipStream_t s);

size_t mask_iou_nms_workspace_bytes(int n, int im_h, int im_w);
int launch_mask_iou_nms(const uint8_t *planes, int n, int im_h, int im_w, const float *dets,
                        int det_stride, const int32_t *classes, double iou_th, int max_per_class,
                        int64_t *keep_out, int32_t *num_out, void *ws, size_t ws_bytes,
                        hipStream_t s);
int launch_prev_box_filter(float *dets, int32_t *classes, int32_t *counts, int F, int det_cap,
                           const float *prev_dets, const int32_t *prev_classes,
                           const int32_t *prev_counts, int prev_cap, float iou_thresh,
                           float score_thresh, hipStream_t s);
size_t gemm_epi_workspace_bytes();
int gemm_plans_key(char *buf, int n);
int gemm_plan_list(char *buf, int n);
int launch_gemm_bias_act(const float *A, int M, int K, const float *W, int N, const float *bias,
                         const float *R, int relu, float *D, void *ws, size_t ws_bytes,
                         hipStream_t s);
bool gemm_split3_supported(int K, int N);
size_t gemm_split3_weight_bytes(int N, int K);
int launch_gemm_split3_weight(const float *W, int N, int K, void *Wp, hipStream_t s);
int launch_gemm_split3(const float *A, int M, int K, const float *A2, int K2, const void *Wp,
                       int N, const float *bias, const float *R, int up_h, int up_w, int sub_h,
                       int sub_w, int relu, float *D, int cfg, hipStream_t s,
                       const float *a_bias = nullptr);
int launch_gemm_split3_mask_logits(const float *A, int M, int K, const void *Wp, int N,
                                   const float *bias, const float *cls_w, const float *cls_b,
                                   const int32_t *roi_ch, int P, float *masks, hipStream_t s);
bool gemm1x1_mfma_supported(int K, int N);
bool conv3x3_mfma_supported(int C, int Cout);
int launch_conv3x3_mfma(const float *X, int N, int H, int W, int C, const float *W2, int Cout,
                        const float *bias, int relu, float *Y, hipStream_t s);
bool conv3x3_wino_supported(int C, int Cout);
bool conv3x3_wino4_supported(int C, int Cout);
int launch_conv3x3_wino4_weight(const float *w, int Cout, int C, float *U, hipStream_t s);
int launch_conv3x3_wino4(const float *X, int N, int H, int W, int C, const float *U, int Cout,
                         const float *bias, int relu, float *Y, hipStream_t s, int mos = 0,
                         int groups = 1);
int launch_conv3x3_wino_weight(const float *w, int Cout, int C, float *U, hipStream_t s);
int launch_conv3x3_wino(const float *X, int N, int H, int W, int C, const float *U, int Cout,
                        const float *bias, int relu, float *Y, hipStream_t s, int seg_h = 0);
int launch_conv3x3_wino_mosaic(const float *X, int R, int H, int W, int C, const float *U,
                               int Cout, const float *bias, int relu, float *Y, hipStream_t s);
bool gemm1x1_dual_supported(int K1, int K2, int N);
int launch_gemm1x1_dual(const float *A1, int K1, const float *A2, int K2, int M, const float *W,
                        int N, const float *bias, int relu, float *D, hipStream_t s);
int launch_gemm1x1_mfma(const float *A, int M, int K, const float *W, int N, const float *bias,
                        const float *R, int relu, float *D, hipStream_t s);
bool fpn_lateral_supported(int K, int N);
int launch_fpn_lateral_weight(const float *W, int N, int K, float *Wf, hipStream_t s);
int launch_fpn_lateral(const float *A, int64_t M, int K, const float *Wf, int N, const float *bias,
                       const float *T, int H, int Wd, float *D, hipStream_t s);

int launch_roi_align_legacy_fwd(const float *feat, int B, int C, int H, int W, const float *rois,
                                int R, int PH, int PW, float scale, float *out, hipStream_t s);
int launch_roi_pool_fwd(const float *feat, int B, int C, int H, int W, const float *rois, int R,
                        int PH, int PW, float scale, float *out, int32_t *argmax, hipStream_t s);
int launch_roi_pool_bwd(const float *top_diff, const int32_t *argmax, int64_t n_out,
                        float *bottom_diff, hipStream_t s);
int launch_roi_crop_fwd(const float *in, int B, int C, int H, int W, const float *grid, int R,
                        int GH, int GW, float *out, hipStream_t s);

int launch_nms(const float *dets, int n, int stride, float thresh, int64_t *keep, int32_t *nkeep,
               void *workspace, size_t ws_bytes, hipStream_t s);
size_t nms_workspace_bytes(int n);

int launch_map_levels(const float *rois, int roi_stride, int col0, int R, int k_min, int k_max,
                      float s0, float lvl0, int32_t *lvl_out, hipStream_t s);

int launch_mask_rois(const float *dets, const int32_t *classes, const int32_t *counts, int F,
                     int det_cap, const double *im_scale, int row0, int rows, int k_min,
                     int k_max, float s0, float lvl0, float *rois_out, int32_t *lvl_out,
                     int32_t *cls_out, int32_t *total_out, hipStream_t s);

int launch_rpn_proposals(const VdRpnLevel *levels, int num_levels, int num_images,
                         const float *im_info, int pre_nms_topN, int post_nms_topN,
                         float nms_thresh, float min_size, float *rois_out, float *probs_out,
                         int32_t *counts_out, void *workspace, size_t ws_bytes, hipStream_t s);
size_t rpn_workspace_bytes(const VdRpnLevel *levels, int num_levels, int num_images,
                           int pre_nms_topN);

int launch_collect_distribute(const float *level_rois, const float *level_probs,
                              const int32_t *level_counts, int num_levels, int level_cap,
                              int num_images, int post_nms_topN, int k_min, int k_max,
                              float *rois_out, int32_t *lvl_out, int32_t *count_out,
                              hipStream_t s);

int launch_box_detections(const float *rois, const float *cls_prob, const float *bbox_pred,
                          const int32_t *roi_count, int R_cap, int num_images, int num_classes,
                          const float *im_scale, const int32_t *im_hw, float score_thresh,
                          float nms_thresh, int dets_per_im, const float *bbox_weights,
                          int soft_method, float soft_sigma, float soft_min, int vote_method,
                          float vote_th, float vote_beta, int det_cap, float *dets_out,
                          int32_t *det_cls_out, int32_t *det_count_out, void *workspace,
                          size_t ws_bytes, hipStream_t s);
size_t box_detections_workspace_bytes(int R_cap, int num_images, int num_classes);
size_t stem_weight_floats();
int launch_stem_weight(const float *w, float *Wp, hipStream_t s);
size_t stem_weight_split_bytes();
int launch_stem_weight_split(const float *w, void *Wp3, hipStream_t s);
int launch_stem_conv_pool(const float *X, int N, int H, int W, const float *Wp, const float *bias,
                          float *Y, int num_cus, hipStream_t s, bool split = false);
int launch_soft_nms(const float *dets, int n, int stride, float sigma, float overlap_thresh,
                    float score_thresh, int method, float *dets_out, int64_t *keep_out,
                    int32_t *count_out, hipStream_t s);
int launch_box_voting(const float *top, int n_top, int top_stride, const float *all, int n_all,
                      int all_stride, float thresh, int method, float beta, float *out,
                      hipStream_t s);

int launch_image_to_blob(const uint8_t *frames, int F, int H, int W, const float *lut,
                         int Hp, int Wp, int nhwc, float *blob, hipStream_t s);
int launch_resize_to_blob(const uint8_t *frames, int F, int H, int W, const float *lut,
                          double im_scale, int Hr, int Wr, int Hp, int Wp, int nhwc, float *blob,
                          hipStream_t s);
int launch_bias_act(float *x, const float *bias, const float *z, const float *bias2, int64_t n,
                    int C, int H, int W, int nhwc, int mode, int relu, hipStream_t s);
int launch_nchw_to_nhwc(const float *in, int B, int C, int H, int W, float *out, hipStream_t s);

// ---- VOS temporal path (vos.hip)
// GroupNorm statistics: ws[n][g] = {sum, sum of squares} (double) of x (+ x2).
struct GnSet {
    const float *x;
    const float *x2;  // optional: statistics of x + x2 (torch's a + b, then GN)
    double *ws;
};
struct GnSets {
    GnSet s[3];
};
// GroupNorm apply + fused epilogue (modes VD_GN_* of vosdet.h, see vos.hip).
struct GnApply {
    const float *x, *x2;
    const double *ws;
    const float *gamma, *beta;
    const float *res;      // residual (VD_GN_ACT) or the hidden state h (GRU modes)
    const double *res_ws;  // res_mode 3: statistics of res
    const float *res_gamma, *res_beta;
    const float *z;      // VD_GN_GRU_H: update gate
    const float *finer;  // VD_GN_GRU_H: finer fused level (2H x 2W), or NULL
    float *out;
    int mode, act, res_mode;
    float eps;
};
int launch_flow_align_fwd(const float *feat, const float *flow, int B, int C, int H, int W,
                          int nhwc, float *out, hipStream_t s);
int launch_flow_align_bwd(const float *top_diff, const float *feat, const float *flow, int B,
                          int C, int H, int W, float *feat_diff, float *flow_diff, hipStream_t s);
size_t gn_workspace_bytes(int B, int G, int sets);
int launch_gn_stats(const GnSets &sets, int nsets, int B, int C, int HW, int G, int nhwc,
                    hipStream_t s);
int launch_gn_apply(const GnApply &a, int B, int C, int H, int W, int G, int nhwc, hipStream_t s);

int launch_paste_masks(const float *masks, int M, int R, const float *boxes, int box_stride,
                       int im_h, int im_w, float thresh, uint8_t *out, hipStream_t s);
int launch_mask_rle(const uint8_t *planes, int M, int H, int W, uint32_t *counts, int cap,
                    int32_t *ncounts, hipStream_t s);
int launch_segm_rle(const float *masks, int M, int R, const float *boxes, int box_stride,
                    int im_h, int im_w, float thresh, uint32_t *counts, int cap,
                    int32_t *ncounts, hipStream_t s);
int launch_rle_strings(const uint32_t *counts, const int32_t *ncounts, int M, int cap,
                       int32_t *lens, uint8_t *chars, hipStream_t s);

int launch_bias_relu_maxpool(const float *x, const float *bias, int N, int C, int H, int W,
                             float *out, hipStream_t s);
int launch_rpn_head(const float *x, const float *conv_bias, const float *w, const float *b,
                    int N, int H, int W, int C, int A, float *cls_prob, float *bbox_pred,
                    hipStream_t s);

int launch_detections_postfilter(float *dets, int32_t *cls, int32_t *counts, int num_images,
                                 int det_cap, float nms_cross_class, int num_det_per_class_pre,
                                 hipStream_t s);

}  // namespace vd
