/*
 * vosdet.h -- C ABI of the MI355X (gfx950) per-frame Mask R-CNN hot path.
 *
 * Library: vosdetectron_amd/libvosdet.so (built by __graft_entry__.build()).
 * Plain C: raw device pointers, sizes and an explicit stream (a hipStream_t
 * passed as void*, NULL = the null stream).  No torch types.  Every call is
 * asynchronous on `stream`, performs no allocation, no host<->device copy and
 * no synchronisation (graph-capturable), and returns a status code instead of
 * the reference's fprintf + exit(-1) (roi_align_kernel.cu:135-139).
 *
 * Each entry point cites the reference interface it replaces.  Numerics follow
 * the reference functions cited in the kernel sources; see DESIGN.md.
 */
#ifndef VOSDET_H_
#define VOSDET_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VD_MAX_LEVELS 5

enum {
    VD_OK = 0,
    VD_ERR_ARG = 1,       /* bad argument (e.g. rois row width != 5) */
    VD_ERR_SHAPE = 2,     /* shape outside what the kernel supports */
    VD_ERR_LAUNCH = 3,    /* kernel launch failed */
    VD_ERR_WORKSPACE = 4  /* workspace too small */
};

enum { VD_LAYOUT_NCHW = 0, VD_LAYOUT_NHWC = 1 };

/* Per-frame failure codes written in place of a device count (never a valid
 * count; downstream kernels treat a negative count as an empty frame and keep it):
 *   VD_COUNT_SELECT_FAILED   the proposal top-k could not bracket pre_nms_topN
 *   VD_COUNT_PREV_BOXES      NMS_SMALL_BOX_IOU: the previous frame kept more
 *                            than one box of a class (vos_test.py:848 asserts) */
#define VD_COUNT_SELECT_FAILED (-1)
#define VD_COUNT_PREV_BOXES (-2)

int vd_version(void);
const char *vd_status_string(int status);

/* ---------------------------------------------------------------------------
 * RoIAlign (Caffe2-exact).  Replaces
 *   int roi_align_forward_cuda(int aligned_height, int aligned_width,
 *       float spatial_scale, int sampling_ratio, THCudaTensor *features,
 *       THCudaTensor *rois, THCudaTensor *output)
 *   lib/modeling/roi_xfrom/roi_align/src/roi_align_cuda.h:1-2, .c:7-40.
 * features: B x C x H x W fp32 NCHW contiguous; rois: num_rois x roi_cols fp32
 * [batch, x1, y1, x2, y2] in input-image coordinates; output: num_rois x C x
 * aligned_height x aligned_width (written entirely).  roi_cols != 5 ->
 * VD_ERR_ARG (the reference silently returns 0 with the output untouched).
 * ------------------------------------------------------------------------- */
int vd_roi_align_forward(int aligned_height, int aligned_width, float spatial_scale,
                         int sampling_ratio, const float *features, int B, int C, int H, int W,
                         const float *rois, int num_rois, int roi_cols, float *output,
                         void *stream);

/* Replaces roi_align_backward_cuda (roi_align_cuda.h:4-5, .c:42-76).
 * bottom_grad (B x C x H x W) must be zero-filled by the caller (as the
 * reference's RoIAlignFunction.backward does, functions/roi_align.py:40-45);
 * contributions are accumulated with fp32 atomics. */
int vd_roi_align_backward(int aligned_height, int aligned_width, float spatial_scale,
                          int sampling_ratio, const float *top_grad, int B, int C, int H, int W,
                          const float *rois, int num_rois, int roi_cols, float *bottom_grad,
                          void *stream);

/* Multi-level FPN RoIAlign: the whole per-level loop + cat + unshuffle of
 * Generalized_RCNN.roi_feature_transform (lib/modeling/model_builder.py:252-303)
 * in one launch.  Level l of the pyramid is levels[l]; roi r is pooled from
 * levels[roi_level[r]] (roi_level == NULL -> level 0) and written to output
 * row r, i.e. already in the order the reference restores with
 * `_idx_restore_int32`.  layout: VD_LAYOUT_NHWC (B x H x W x C, the product
 * layout; C % 4 == 0) or VD_LAYOUT_NCHW.  roi_order (optional): a permutation
 * that only changes the order in which RoIs are scheduled (L2 locality), never
 * the output placement.  output_layout: VD_LAYOUT_NCHW -> num_rois x C x ah x aw
 * (the reference's layout), VD_LAYOUT_NHWC -> num_rois x ah x aw x C (NHWC
 * input, ah == aw in {7, 14}; what channels_last heads consume). */
typedef struct {
    const float *data;
    int H;
    int W;
    float spatial_scale;
} VdFeatLevel;

int vd_roi_align_fpn_forward(const VdFeatLevel *levels, int num_levels, int B, int C, int layout,
                             const float *rois, const int32_t *roi_level,
                             const int32_t *roi_order, int num_rois, int aligned_height,
                             int aligned_width, int sampling_ratio, int output_layout,
                             float *output, void *stream);

/* Tile-binned, LDS-staged multi-level RoIAlign: the same operation as
 * vd_roi_align_fpn_forward(layout = output_layout = VD_LAYOUT_NHWC,
 * aligned_height = aligned_width = aligned_size) -- the per-level loop + cat +
 * unshuffle of roi_feature_transform (lib/modeling/model_builder.py:252-303)
 * over the Caffe2 RoIAlign of lib/modeling/roi_xfrom/roi_align/src/
 * roi_align_kernel.cu:65-121 -- computed in the reference's per-sample
 * arithmetic (bit-identical to it).  Serves sampling_ratio 2, C % 32 == 0,
 * B <= 64, aligned_size <= 64; returns VD_ERR_SHAPE otherwise (callers then use
 * vd_roi_align_fpn_forward).  workspace: >= vd_roi_align_fpn_tiled_workspace_size()
 * bytes of device memory, stream-ordered (no host sync, graph-capturable). */
size_t vd_roi_align_fpn_tiled_workspace_size(const VdFeatLevel *levels, int num_levels, int B,
                                             int C, int num_rois, int aligned_size);
int vd_roi_align_fpn_tiled_forward(const VdFeatLevel *levels, int num_levels, int B, int C,
                                   const float *rois, const int32_t *roi_level, int num_rois,
                                   int aligned_size, int sampling_ratio, float *output,
                                   void *workspace, size_t workspace_bytes, void *stream);

/* jwyang RoIAlign (legacy, lib/model/roi_align).  Replaces
 * roi_align_forward_cuda(int aligned_height, int aligned_width, float
 * spatial_scale, THCudaTensor *features, THCudaTensor *rois, THCudaTensor
 * *output)  lib/model/roi_align/src/roi_align_cuda.c. */
int vd_roi_align_legacy_forward(int aligned_height, int aligned_width, float spatial_scale,
                                const float *features, int B, int C, int H, int W,
                                const float *rois, int num_rois, float *output, void *stream);

/* RoIPool.  Replaces roi_pooling_forward_cuda(int pooled_height, int
 * pooled_width, float spatial_scale, THCudaTensor *features, THCudaTensor
 * *rois, THCudaTensor *output, THCudaIntTensor *argmax)
 * lib/model/roi_pooling/src/roi_pooling_cuda.c:7.  argmax may be NULL. */
int vd_roi_pool_forward(int pooled_height, int pooled_width, float spatial_scale,
                        const float *features, int B, int C, int H, int W, const float *rois,
                        int num_rois, float *output, int32_t *argmax, void *stream);
/* Replaces roi_pooling_backward_cuda (roi_pooling_cuda.c): scatter top_grad
 * into the zero-filled bottom_grad at argmax (fp32 atomics). */
int vd_roi_pool_backward(const float *top_grad, const int32_t *argmax, int64_t num_outputs,
                         float *bottom_grad, void *stream);

/* RoICrop bilinear sampler.  Replaces BilinearSamplerBHWD_updateOutput_cuda(
 * THCudaTensor *inputImages, THCudaTensor *grids, THCudaTensor *output)
 * lib/model/roi_crop/src/roi_crop_cuda.c:15.  input B x C x H x W, grid
 * R x GH x GW x 2 in (y, x) order in [-1, 1]; output R x C x GH x GW must be
 * zero-filled by the caller (samples with every tap outside keep the zero). */
int vd_roi_crop_forward(const float *input, int B, int C, int H, int W, const float *grid_yx,
                        int num_rois, int GH, int GW, float *output, void *stream);

/* 1x1 convolution on channels_last tensors as a GEMM with the conv epilogue
 * fused (hipBLASLt): D[M][N] = act(A[M][K] . W[N][K]^T + bias[N] (+ R[M][N])),
 * row-major fp32, act = ReLU when relu != 0.  With bias = the folded frozen-BN
 * shift and R = the block input, this is the whole tail of the reference's
 * bottleneck_transformation (lib/modeling/ResNet.py:246-294: conv3 ->
 * AffineChannel2d -> + residual -> ReLU) in one kernel.  residual may be NULL.
 * workspace: >= vd_gemm_workspace_size() bytes, stream-ordered.  Not a
 * replacement for a reference custom op (those convs run in PyTorch there);
 * it removes the separate epilogue pass over the conv output. */
size_t vd_gemm_workspace_size(void);
/* The key under which this process applies pinned GEMM plans (VOSDET_GEMM_PLANS):
 * "<arch> hipblaslt-<version>-<git revision> cu<CUs>" of the current device; a
 * plans file's "# key ..." line must equal it for the pins below it to apply. */
int vd_gemm_plans_key(char *buf, int n);
/* The GEMM plans this process has made, one line per shape:
 * "M N K relu has_res own|blas workspace_bytes".  A plan with workspace_bytes > 0
 * keeps inter-workgroup state (split-K partials, stream-K fix-up flags) in the
 * caller's workspace, so two launches that may run concurrently (two captured
 * steps replayed on two streams) must be given different workspaces.
 * VD_ERR_WORKSPACE when n bytes cannot hold the list. */
int vd_gemm_plan_list(char *buf, int n);
int vd_gemm_bias_act(const float *A, int M, int K, const float *W, int N, const float *bias,
                     const float *residual, int relu, float *D, void *workspace,
                     size_t workspace_bytes, void *stream);

/* The same GEMM (D[M][N] = act(A[M][K] . W[N][K]^T + bias[N] (+ R[M][N])), fp32
 * in and out) on the bf16 matrix cores at fp32 accuracy: every operand is split
 * into three bf16 pieces carrying its 24-bit significand and the six largest piece
 * products are accumulated in fp32 (csrc/gemm_split3.hip; error measured against
 * fp64 beside torch's fp32 GEMM in tests/test_gemm_split3_gpu.py).  Wp is the
 * weight in split form, vd_gemm_split3_weight_size(N, K) bytes, made once per
 * model by vd_gemm_split3_weight.  K a multiple of 32, N of 64 (VD_ERR_SHAPE
 * otherwise); residual may be NULL.  A2 / K2 > 0 (a multiple of 16): the last K2 of the K
 * input channels come from a second [M][K2] operand (A is then [M][K - K2]): a stage's
 * first block, conv3 of h and the stride-1 downsample of x as ONE GEMM (ResNet.py:246-294
 * with basic_bn_shortcut :195-205).  up_h, up_w > 0 (both even): residual is the
 * top-down map of an FPN level, images x up_h/2 x up_w/2 x N, added at the nearest-2x
 * row of each of the M = images x up_h x up_w pixels after the bias -- the FPN
 * top-down lateral step (FPN.py:292-300) in one launch.  sub_h, sub_w > 0: A is an
 * images x sub_h x sub_w NHWC map read at stride 2 (M = images x ceil(sub_h/2) x
 * ceil(sub_w/2)): a stage's stride-2 1x1 convs (ResNet.py:246-294 with STRIDE_1X1, and
 * the downsample shortcut) without the subsampled copy.  cfg 0 picks the tile shape
 * (1: 256 pixels x 256 channels, 2: 256 x 128, 3: 256 x 64, 4: 128 x 128, 5: 256 x 256 in
 * eight waves per workgroup;
 * VD_ERR_SHAPE when N does not divide by the tile's channels).  a_bias (K - K2 floats,
 * or NULL): A's channels enter as relu(A + a_bias[k]) -- the bias + ReLU of the layer
 * that produced A, applied in fp32 before the split (bit-identical to a separate
 * pass; ResNeXt's grouped conv2 runs on MIOpen without them).  Replaces the same
 * fp32 convolutions / Linear layers as vd_gemm_bias_act (ResNet.py:246-294
 * bottleneck 1x1s, fast_rcnn_heads.py fc6 / fc7, mask_rcnn_heads.py upconv5). */
size_t vd_gemm_split3_weight_size(int N, int K);
int vd_gemm_split3_weight(const float *W, int N, int K, void *Wp, void *stream);
int vd_gemm_split3_bias_act(const float *A, int M, int K, const float *A2, int K2,
                            const float *a_bias, const void *Wp, int N, const float *bias,
                            const float *residual, int up_h, int up_w, int sub_h, int sub_w,
                            int relu, float *D, int cfg, void *stream);

/* The mask head's tail in one split-bf16 GEMM launch: the 2x2 / 2 transposed conv
 * upconv5 + ReLU (mask_rcnn_heads.py:62-68) and the class-selected 1x1 mask logits +
 * sigmoid (mask_rcnn_outputs, mask_rcnn_heads.py:20-35, at each RoI's class as
 * segm_results reads them, test.py:801-855): X = the RoI maps, M = RoIs x P x P
 * NHWC rows of K = 256 channels; Wp = vd_gemm_split3_weight of the upconv weight as
 * [(i, j, co) = 1024][K]; bias [1024] = the upconv bias per (i, j); cls_w [classes][256],
 * cls_b [classes]; roi_ch [RoIs] the class channel of each RoI; masks [RoIs][2P][2P]
 * = sigmoid(sum_co relu(upconv)[2y+i][2x+j][co] * cls_w[ch][co] + cls_b[ch]).  The
 * M x 1024 upconv output never reaches HBM. */
int vd_mask_head_upconv_logits(const float *X, int M, int K, const void *Wp, const float *bias,
                               const float *cls_w, const float *cls_b, const int32_t *roi_ch,
                               int P, float *masks, void *stream);

/* 3x3 stride-1 pad-1 convolution of a channels_last (NHWC) fp32 tensor with
 * the bias (+ ReLU) epilogue fused, one hand-written MFMA implicit-GEMM kernel:
 * Y[n][y][x][co] = act(sum_{ky,kx,ci} X[n][y+ky-1][x+kx-1][ci] W2[co][ky][kx][ci]
 * + bias[co]), out-of-image taps zero.  W2 is the PyTorch weight [Cout][Cin][3][3]
 * permuted to [Cout][3][3][Cin].  bias may be NULL.  The FPN posthoc convs
 * (lib/modeling/FPN.py:227-258), the RPN conv (FPN.py:376-422) and the mask head
 * convs (mask_rcnn_heads.py:178-188) run in PyTorch in the reference.
 * Requires Cin % 64 == 0 and Cout % 128 == 0 or Cout == 64 (VD_ERR_SHAPE otherwise). */
int vd_conv3x3_bias_act(const float *X, int N, int H, int W, int C, const float *W2, int Cout,
                        const float *bias, int relu, float *Y, void *stream);

/* The same convolution by Winograd F(2x2, 3x3) on the MFMA pipes (2.25x fewer
 * multiplies; the transforms add, subtract and halve): U from
 * vd_conv3x3_wino_weight (16 x Cout x Cin fp32 in an opaque chunk-blocked order,
 * once per model) replaces W2.  Both require Cin % 8 == 0 and Cout % 64 == 0
 * (VD_ERR_SHAPE otherwise).  Results agree with the direct form within fp32
 * rounding (not bit for bit). */
int vd_conv3x3_wino_weight(const float *w, int Cout, int Cin, float *U, void *stream);
int vd_conv3x3_wino_bias_act(const float *X, int N, int H, int W, int C, const float *U,
                             int Cout, const float *bias, int relu, float *Y, void *stream);

/* The same convolution by Winograd F(4x4, 3x3) (round 5; 4x fewer multiplies than
 * the direct form, 1.78x fewer than F(2x2); transforms scale by up to 8, so a few
 * times F(2x2)'s rounding error): U from vd_conv3x3_wino4_weight (36 x Cout x Cin
 * fp32, opaque fragment order).  Cin % 8 == 0, Cin <= 4096, Cout % 64 == 0
 * (VD_ERR_SHAPE otherwise).  Replaces the same PyTorch convolutions as above. */
int vd_conv3x3_wino4_weight(const float *w, int Cout, int Cin, float *U, void *stream);
int vd_conv3x3_wino4_bias_act(const float *X, int N, int H, int W, int C, const float *U,
                              int Cout, const float *bias, int relu, float *Y, void *stream);
/* The same over N small maps (H, W <= 15: the mask head's 14 x 14 RoI features,
 * mask_rcnn_heads.py:178-188), two maps per 16 x 32 output block -- eight in 8 x 8
 * cells when H, W <= 7 (C4's res5 head on 7 x 7 RoI maps, ResNet.py:17-155) -- each
 * padded by its own zeros: bit-identical to vd_conv3x3_wino4_bias_act, which gives
 * every map a block of its own.  VD_ERR_SHAPE for larger maps. */
int vd_conv3x3_wino4_mosaic_bias_act(const float *X, int N, int H, int W, int C, const float *U,
                                     int Cout, const float *bias, int relu, float *Y,
                                     void *stream);
/* The same over N maps stacked in one column at a pitch of H + 1 rounded up to 4 rows
 * (each map padded by its own zeros), so the 16-row output blocks run on through the
 * stack: for heights that leave most of a map's last block row empty (50 x 84 res4 /
 * P4, 25 x 42 res5).  Bit-identical to vd_conv3x3_wino4_bias_act; VD_ERR_SHAPE when
 * N H W C >= 2^31. */
int vd_conv3x3_wino4_rows_bias_act(const float *X, int N, int H, int W, int C, const float *U,
                                   int Cout, const float *bias, int relu, float *Y,
                                   void *stream);
/* A grouped 3x3 convolution (ResNeXt's conv2, ResNet.py:246-294 with groups > 1; C
 * in = out channels, C / groups dividing 64) by the same F(4x4) kernel: every 64-channel
 * output block reads only the 64 input channels of its groups.  U =
 * vd_conv3x3_wino4_weight of the block-diagonal expansion of the [C][C / groups][3][3]
 * weight to [C][64][3][3] (zeros between groups; Cin = 64).  rows != 0: the N maps as
 * the row stack of vd_conv3x3_wino4_rows_bias_act.  VD_ERR_SHAPE for other shapes. */
int vd_conv3x3_wino4_grouped_bias_act(const float *X, int N, int H, int W, int C,
                                      const float *U, int groups, const float *bias, int relu,
                                      float *Y, int rows, void *stream);
/* A 3x3 convolution with dilation 2 and padding 2 (the VOS mask head, MRCNN.DILATION = 2,
 * mask_rcnn_heads.py:178-188) of N maps of H x W (H, W even) by the same F(4x4) kernel:
 * it is the plain pad-1 conv of the 4 N polyphase sub-maps of H/2 x W/2 (output (2i +
 * a, 2j + b) reads only parity-(a, b) inputs at sub-map distance 1), which the kernel
 * reads and writes in place in the full maps.  layout: the sub-maps one per block (0),
 * as pairs / octets (1, H/2, W/2 <= 15) or as the shared-separator grid (2).  U from
 * vd_conv3x3_wino4_weight of the same weight. */
int vd_conv3x3_wino4_dilated2_bias_act(const float *X, int N, int H, int W, int C,
                                       const float *U, int Cout, const float *bias, int relu,
                                       float *Y, int layout, void *stream);
/* The same over N maps laid out as a 2-D grid at a pitch of (H + 1) x (W + 1) -- one
 * zero row / column shared between neighbours, g maps per grid row chosen for the
 * fewest 16 x 32 output blocks (round 6; the mask head's 14 x 14 RoI maps: 32 per
 * 480-column row, 87 % of each block real output against 77 % for map pairs).  Tiles
 * straddle maps, so the result equals vd_conv3x3_wino4_bias_act's within Winograd
 * rounding, not bitwise; each output is still its own map's zero-padded convolution.
 * VD_ERR_SHAPE when N H W C >= 2^31 or H, W > 255. */
int vd_conv3x3_wino4_grid_bias_act(const float *X, int N, int H, int W, int C, const float *U,
                                   int Cout, const float *bias, int relu, float *Y,
                                   void *stream);

/* The Winograd convolution of R images of seg_h x W pixels stored back to back
 * (R x seg_h x W x C, i.e. one H = R * seg_h image), each padded by its own zeros:
 * the mask head's RoI maps run as one mosaic, so the 8 x 16-pixel blocks are not
 * split at every 14-row map.  seg_h even, H % seg_h == 0; bit-identical to
 * vd_conv3x3_wino_bias_act on the R images. */
int vd_conv3x3_wino_seg_bias_act(const float *X, int H, int W, int C, const float *U, int Cout,
                                 const float *bias, int relu, int seg_h, float *Y, void *stream);

/* The Winograd convolution of R maps of H x W pixels (R x H x W x C, each padded by
 * its own zeros) run as one 2-D mosaic: g maps side by side per mosaic row, g the
 * least count with g * W a multiple of 16, so neither the 8-row nor the 16-column
 * side of a pixel block is split at a map edge (the mask head's 14 x 14 RoI maps:
 * 8 per row, 112 columns).  An odd H or W gets one phantom row / column per map
 * (reads 0, never stored).  Output in the input's R x H x W layout; bit-identical to
 * vd_conv3x3_wino_bias_act on the R maps. */
int vd_conv3x3_wino_mosaic_bias_act(const float *X, int R, int H, int W, int C, const float *U,
                                    int Cout, const float *bias, int relu, float *Y, void *stream);

/* Two 1x1 convolutions of two channels_last inputs summed, with the epilogue:
 * D[M][N] = act(A1[M][K1] . W[:, :K1]^T + A2[M][K2] . W[:, K1:]^T + bias[N]),
 * W = [W1 | W2] as N x (K1 + K2) row-major.  With A1 = the bottleneck's conv2
 * output, A2 = the block input, W = [W3 | Wdownsample] and bias = b3 + bd, this
 * is a ResNet stage's first block tail (ResNet.py:246-294 with the stride-1
 * basic_bn_shortcut, :195-205) without the downsample tensor's HBM round trip.
 * One hand-written MFMA kernel (K1 = K2 = 64, N = 256: res2 of the R-50/R-101
 * FPN bodies); other shapes return VD_ERR_SHAPE (callers use vd_gemm_bias_act
 * with the downsample output as the residual). */
int vd_gemm_dual_bias_act(const float *A1, int K1, const float *A2, int K2, int M, const float *W,
                          int N, const float *bias, int relu, float *D, void *stream);

/* The FPN top-down lateral step in one MFMA GEMM with the nearest-2x add fused
 * (replaces lib/modeling/FPN.py:292-300 topdown_lateral_module.forward, which runs
 * in PyTorch in the reference: lat = conv_lateral(lateral); td = F.upsample(top,
 * scale_factor=2, mode='nearest'); return lat + td):
 *   D[p][co] = (A[p] . W[co] + bias[co]) + top[up(p)][co]
 * A: M x K NHWC rows of the lateral (M = images x H x W), top: images x H/2 x W/2 x N
 * (NULL: no top-down term), D: M x N.  H, W even.  Wf from vd_fpn_lateral_weight
 * (W [N][K] row-major -> an opaque fragment order, K x N fp32, once per model).
 * N == 256 and K in {256, 512, 1024}; VD_ERR_SHAPE otherwise. */
int vd_fpn_lateral_weight(const float *W, int N, int K, float *Wf, void *stream);
int vd_fpn_lateral_topdown(const float *A, int64_t M, int K, const float *Wf, int N,
                           const float *bias, const float *top, int H, int W, float *D,
                           void *stream);

/* ---------------------------------------------------------------------------
 * NMS with the semantics of the NMS the reference executes,
 * utils.boxes.nms -> cython_nms.nms (lib/utils/boxes.py:329-333,
 * lib/utils/cython_nms.pyx:37-87): dets n x det_stride fp32 [x1,y1,x2,y2,score,..],
 * processing order score-descending (ties: higher index first), suppression
 * when IoU (+1 convention) >= thresh, kept indices written ascending to
 * keep_out (int64), their count to *num_out (device int32).  n <= 8192.
 * Stands in for the reference's unused GPU path nms_cuda(THCudaIntTensor
 * *keep_out, THCudaTensor *boxes, THCudaIntTensor *num_out, float thresh)
 * (lib/model/nms/src/nms_cuda.c:8-19) WITH THE CYTHON SEMANTICS above: it is
 * not a drop-in for nms_cuda's own rule, which suppresses on IoU > thresh
 * (strict) over pre-sorted input (lib/model/nms/src/nms_cuda_kernel.cu:78). */
size_t vd_nms_workspace_size(int n);
int vd_nms(const float *dets, int n, int det_stride, float thresh, int64_t *keep_out,
           int32_t *num_out, void *workspace, size_t workspace_bytes, void *stream);

/* The VOS fork's mask-IoU NMS, lib_vos/tools/vos_test.py:985-1029
 * nms_with_mask_iou (applied at :113-118 when TEST.NMS_WITH_MASK_IOU > 0) on one
 * frame's n detections (n <= 1024) in cls_boxes (class-major) order:
 * planes n x im_h x im_w uint8 (the pasted, thresholded segms, nonzero = set),
 * dets n x det_stride fp32 (score at column 4), classes n int32.  Score order
 * (np.argsort(-s), ties by index), position j discarded by an earlier kept i
 * when inter / (|m_i| + 1e-6) or inter / (|m_j| + 1e-6) > iou_th (float64), then
 * at most max_per_class (TEST.NUM_DET_PER_CLASS_POST) per class.  Writes the
 * kept detection indices in the reference's output order (class ascending, then
 * score order) to keep_out and their count to *num_out (device int32).
 * workspace: >= vd_mask_iou_nms_workspace_size(n, im_h, im_w) bytes. */
size_t vd_mask_iou_nms_workspace_size(int n, int im_h, int im_w);
int vd_mask_iou_nms(const uint8_t *planes, int n, int im_h, int im_w, const float *dets,
                    int det_stride, const int32_t *classes, double iou_th, int max_per_class,
                    int64_t *keep_out, int32_t *num_out, void *workspace, size_t workspace_bytes,
                    void *stream);

/* TEST.NMS_SMALL_BOX_IOU of the fork's box_results_with_nms_and_limit
 * (lib_vos/tools/vos_test.py:845-860), in place on the device detections of F
 * frames (dets [F][det_cap][5], classes, counts, class-major as vd_box_detections
 * writes them): for each class whose previous-frame result (prev_* of the same
 * row, [F][prev_cap]) holds one box with score >= score_thresh, the class's
 * boxes with IoU (bb_intersection_over_union, float32) < iou_thresh are dropped;
 * order kept.  A previous result with several boxes of one class (the reference
 * asserts for every class, vos_test.py:846-848) sets the frame's count to
 * VD_COUNT_PREV_BOXES.  det_cap <= 1024. */
int vd_detections_prev_box_filter(float *dets, int32_t *classes, int32_t *counts, int F,
                                  int det_cap, const float *prev_dets,
                                  const int32_t *prev_classes, const int32_t *prev_counts,
                                  int prev_cap, float iou_thresh, float score_thresh,
                                  void *stream);

/* FPN level of each RoI: utils/fpn.py:11-28 map_rois_to_fpn_levels
 * (floor(lvl0 + log2(sqrt(area)/s0 + 1e-6)) clipped to [k_min, k_max]).
 * rois: R x roi_stride, the box at columns [col0, col0+4). */
int vd_map_rois_to_fpn_levels(const float *rois, int roi_stride, int col0, int R, int k_min,
                              int k_max, float canonical_scale, float canonical_level,
                              int32_t *lvl_out, void *stream);

/* The mask-head batch of im_detect_mask for all frames of a step, sized
 * without a host read of the detection counts (lib/core/test.py:366-402:
 * _get_rois_blob :877-906 -- box * im_scale as a float64 product stored as
 * float32 -- and _add_multilevel_rois_for_test :909-927).  Detection j of
 * frame f (j < counts[f], vd_box_detections' outputs) is global row
 * prefix(counts)[f] + j, frame-major; rows [row0, row0 + rows) are written:
 * rois_out [rows][5] = (f, x1, y1, x2, y2), lvl_out = FPN level - k_min,
 * cls_out = its class.  Output rows past the total are padding (zero box,
 * level 0, class 1).  total_out[0] = sum(counts) (may exceed row0 + rows: the
 * caller runs a second batch from row0 = rows for those).  im_scale: F doubles. */
int vd_mask_rois(const float *dets, const int32_t *classes, const int32_t *counts,
                 int num_images, int det_cap, const double *im_scale, int row0, int rows,
                 int k_min, int k_max, float canonical_scale, float canonical_level,
                 float *rois_out, int32_t *lvl_out, int32_t *cls_out, int32_t *total_out,
                 void *stream);

/* ---------------------------------------------------------------------------
 * RPN proposals for all FPN levels and images in one launch: per (image,
 * level) GenerateProposalsOp.forward / proposals_for_one_image
 * (lib/modeling/generate_proposals.py:20-168): top pre_nms_topN by score,
 * anchor shift + bbox_transform (boxes.py:156-205), clip to im_info
 * (boxes.py:138-153), _filter_boxes (:171-182), NMS, keep[:post_nms_topN].
 * cls_prob: N x A x H x W, bbox_pred: N x 4A x H x W (conv outputs, NCHW),
 * anchors: A x 4 float64 (generate_anchors.py), im_info: N x 3 device fp32.
 * Outputs per (image i, level l), slot base (i*num_levels + l)*post_nms_topN:
 * rois_out [.][5] = (i, x1, y1, x2, y2), probs_out [.], counts_out[i*L+l].
 * pre_nms_topN <= 2048 per level. */
typedef struct {
    const float *cls_prob;
    const float *bbox_pred;
    const double *anchors;
    int A;
    int H;
    int W;
    float spatial_scale;
} VdRpnLevel;

size_t vd_generate_proposals_workspace_size(const VdRpnLevel *levels, int num_levels,
                                            int num_images, int pre_nms_topN);
int vd_generate_proposals(const VdRpnLevel *levels, int num_levels, int num_images,
                          const float *im_info, int pre_nms_topN, int post_nms_topN,
                          float nms_thresh, float min_size, float *rois_out, float *probs_out,
                          int32_t *counts_out, void *workspace, size_t workspace_bytes,
                          void *stream);

/* collect() + distribute() of CollectAndDistributeFpnRpnProposalsOp at
 * inference (lib/modeling/collect_and_distribute_fpn_rpn_proposals.py:91-138),
 * per image: concatenate the per-level proposals (level-major), keep the top
 * post_nms_topN by score (ties: lower concatenation index first), and give
 * each kept RoI its FPN level (utils/fpn.py:11-28).  Inputs are the outputs of
 * vd_generate_proposals (level_cap = its post_nms_topN).  Outputs per image i:
 * rois_out[i*post_nms_topN + r][5], lvl_out[.] (level index k - k_min),
 * count_out[i]. */
int vd_collect_distribute(const float *level_rois, const float *level_probs,
                          const int32_t *level_counts, int num_levels, int level_cap,
                          int num_images, int post_nms_topN, int k_min, int k_max,
                          float *rois_out, int32_t *lvl_out, int32_t *count_out, void *stream);

/* Box-head post-processing for each image: im_detect_bbox's decode + clip
 * (lib/core/test.py:157-184; bbox_transform with BBOX_REG_WEIGHTS, clip to the
 * original image) followed by box_results_with_nms_and_limit (test.py:733-797;
 * fork fix lib_vos/tools/vos_test.py:748-865): per class j >= 1 score >=
 * score_thresh, NMS, then the top dets_per_im over all classes (score >= the
 * dets_per_im-th largest).  rois: num_images x R_cap x 5 (first roi_count[i]
 * valid), cls_prob: . x R_cap x K, bbox_pred: . x R_cap x 4K, im_scale[i],
 * im_hw[i] = original (height, width) as int32.  Outputs per image i (det_cap
 * slots): dets_out[.][5] = (x1, y1, x2, y2, score) ordered by class then
 * proposal index (np.vstack order), det_cls_out[.] class id,
 * det_count_out[i]. */
size_t vd_box_detections_workspace_size(int R_cap, int num_images, int num_classes);
int vd_box_detections(const float *rois, const float *cls_prob, const float *bbox_pred,
                      const int32_t *roi_count, int R_cap, int num_images, int num_classes,
                      const float *im_scale, const int32_t *im_hw, float score_thresh,
                      float nms_thresh, int dets_per_im, const float *bbox_reg_weights,
                      int det_cap, float *dets_out, int32_t *det_cls_out,
                      int32_t *det_count_out, void *workspace, size_t workspace_bytes,
                      void *stream);

/* vd_box_detections with the inference options of box_results_with_nms_and_limit
 * (lib/core/test.py:756-776):
 *  soft_nms_method  -1 = the NMS above; 0 hard / 1 linear / 2 gaussian =
 *                   TEST.SOFT_NMS (utils/boxes.py:336-355 -> cython_nms.soft_nms,
 *                   cython_nms.pyx:98-203; overlap threshold nms_thresh, sigma,
 *                   min score 0.0001 at test.py:760): the class's rows in soft-NMS
 *                   output order with decayed scores;
 *  bbox_vote_method -1 = off; 0 ID / 1 AVG / 2 IOU_AVG / 3 QUASI_SUM =
 *                   TEST.BBOX_VOTE.SCORING_METHOD (utils/boxes.py:277-333, voters:
 *                   bbox_overlaps >= bbox_vote_thresh among the class's candidates;
 *                   QUASI_SUM's beta = bbox_vote_beta).  GENERALIZED_AVG at beta 1
 *                   is AVG; TEMP_AVG is not offered.
 * Bit-exact to the compiled reference in this container (tests/golden/soft_nms.npz). */
int vd_box_detections_ex(const float *rois, const float *cls_prob, const float *bbox_pred,
                         const int32_t *roi_count, int R_cap, int num_images, int num_classes,
                         const float *im_scale, const int32_t *im_hw, float score_thresh,
                         float nms_thresh, int dets_per_im, const float *bbox_reg_weights,
                         int soft_nms_method, float soft_nms_sigma, float soft_nms_min_score,
                         int bbox_vote_method, float bbox_vote_thresh, float bbox_vote_beta,
                         int det_cap, float *dets_out, int32_t *det_cls_out,
                         int32_t *det_count_out, void *workspace, size_t workspace_bytes,
                         void *stream);

/* ResNet stem in one pass (basic_bn_stem, lib/modeling/ResNet.py:224-230, with
 * the AffineChannel folded into the bias): MaxPool 3x3/2 pad 1 (ReLU (conv1 7x7/2
 * pad 3 (x) + bias)), conv1 3 -> 64 channels on the MFMA pipes; the conv output
 * stays in LDS.  x: N x H x W x 3 fp32 (NHWC, the channels_last blob); y: N x Ho x
 * Wo x 64 (Ho = ((H - 1) / 2) / 2 + 1 ...).  vd_stem_weight_pack reorders the
 * PyTorch weight [64][3][7][7] into vd_stem_weight_size() bytes once. */
size_t vd_stem_weight_size(void);
int vd_stem_weight_pack(const float *w, float *packed, void *stream);
int vd_stem_conv_pool(const float *x, int N, int H, int W, const float *packed, const float *bias,
                      float *y, void *stream);

/* The same stem with conv1 on the bf16 matrix cores at fp32 accuracy (round 6; the
 * three-piece bf16 split of gemm_split3, six piece products per fp32 product, fp32
 * accumulate): vd_stem_split_weight_pack splits the PyTorch weight [64][3][7][7] into
 * vd_stem_split_weight_size() bytes once; vd_stem_split_conv_pool takes that image and
 * is otherwise vd_stem_conv_pool. */
size_t vd_stem_split_weight_size(void);
int vd_stem_split_weight_pack(const float *w, void *packed, void *stream);
int vd_stem_split_conv_pool(const float *x, int N, int H, int W, const void *packed,
                            const float *bias, float *y, void *stream);

/* utils.boxes.soft_nms (lib/utils/boxes.py:336-355 -> cython_nms.soft_nms,
 * cython_nms.pyx:98-203) on the device: dets n x dets_stride (>= 5) float32
 * [x1, y1, x2, y2, score]; method 0 hard / 1 linear / 2 gaussian.  Writes the
 * count_out[0] = N surviving rows (dets_out N x 5, decayed scores, in the
 * reference's output order) and their input indices (keep_out).  n <= 4096;
 * one wavefront (the reference loop is sequential in its selections). */
int vd_soft_nms(const float *dets, int n, int dets_stride, float sigma, float overlap_thresh,
                float score_thresh, int method, float *dets_out, int64_t *keep_out,
                int32_t *count_out, void *stream);

/* utils.boxes.box_voting (lib/utils/boxes.py:277-333): every top row becomes
 * the score-weighted average of the rows of all_dets whose bbox_overlaps
 * (cython_bbox.pyx, float32) with it is >= thresh, in numpy's summation order;
 * scoring_method 0 ID / 1 AVG / 2 IOU_AVG / 3 QUASI_SUM (beta).  out: n_top x 5.
 * n_all <= 4096. */
int vd_box_voting(const float *top_dets, int n_top, int top_stride, const float *all_dets,
                  int n_all, int all_stride, float thresh, int scoring_method, float beta,
                  float *out, void *stream);

/* Frame preparation, lib/utils/blob.py:37-114 at identity scale (im_scale 1): u8 BGR frames
 * (F x H x W x 3) -> fp32 blob minus PIXEL_MEANS, zero-padded to Hp x Wp
 * (multiples of FPN.COARSEST_STRIDE).  lut[3*256] = float32(u - mean_c) for
 * every byte value (numpy's float64 subtraction, then the float32 store).
 * nhwc = 0 -> F x 3 x Hp x Wp, 1 -> F x Hp x Wp x 3. */
int vd_image_to_blob(const uint8_t *frames, int F, int H, int W, const float *lut, int Hp,
                     int Wp, int nhwc, float *blob, void *stream);

/* Frame preparation at any scale: prep_im_for_blob (lib/utils/blob.py:117-139,
 * driven by get_image_blob :37-60 and tools/infer_simple.py:142-149) --
 * float32(BGR) - PIXEL_MEANS, cv2.resize(fx = fy = im_scale, INTER_LINEAR) to
 * Hr x Wr (= rint(H * im_scale), rint(W * im_scale), cv::resize's dsize) --
 * then zero-padded to Hp x Wp like vd_image_to_blob.  The resize restates
 * OpenCV's scalar float INTER_LINEAR path (scale = 1 / im_scale in double,
 * coefficient tables, horizontal then vertical pass, see misc.hip); cv2 is not
 * importable in the build container, so this step's parity against an executed
 * cv2 is unpinned (it is pinned against the numpy restatement and known answers). */
int vd_image_resize_to_blob(const uint8_t *frames, int F, int H, int W, const float *lut,
                            double im_scale, int Hr, int Wr, int Hp, int Wp, int nhwc,
                            float *blob, void *stream);

/* Convolution epilogue, in place on x (N x C x H x W logical, physical NHWC when
 * nhwc = 1):  x = act((x + bias[c]) + r),  r = 0 (residual_mode 0), residual
 * (+ residual_bias[c]) of the same shape (mode 1), or residual nearest-2x
 * upsampled from (H/2, W/2) (+ residual_bias[c]) (mode 2: the FPN top-down add,
 * lib/modeling/FPN.py:293-299).  act = ReLU if relu.  One pass instead of the
 * bias / residual / ReLU passes after a bias-free convolution (the frozen
 * AffineChannel2d of ResNet.py:276-294 folded into conv weight + bias).
 * bias / residual_bias may be NULL; N*C*H*W < 2^31. */
int vd_bias_act(float *x, const float *bias, const float *residual, const float *residual_bias,
                int N, int C, int H, int W, int nhwc, int residual_mode, int relu, void *stream);

/* B x C x H x W -> B x H x W x C (pyramid relayout for the NHWC RoIAlign). */
int vd_nchw_to_nhwc(const float *in, int B, int C, int H, int W, float *out, void *stream);


/* ===========================================================================
 * VOS temporal path (lib_vos): FlowAlign, GroupNorm epilogues, ConvGRU gates.
 * ======================================================================== */

/* FlowAlign.  Replaces
 *   int flow_align_forward_cuda(THCudaTensor *bottom, THCudaTensor *flow,
 *                               THCudaTensor *top)
 *   lib_vos/vos_model/flow_align/src/flow_align_cuda.c:7-23 (kernel
 *   flow_align_cuda_kernel.cu:15-55).
 * features: B x C x H x W (layout VD_LAYOUT_NCHW, the reference's) or
 * B x H x W x C (VD_LAYOUT_NHWC, C % 4 == 0); flow: B x 2 x H x W fp32 (x, y
 * displacement in level pixels, already downsampled by the module's
 * conv_flow_downsample); output: same layout/shape as features, written
 * entirely (0 where the displaced position leaves [0, H-1) x [0, W-1)). */
int vd_flow_align_forward(const float *features, const float *flow, int B, int C, int H, int W,
                          int layout, float *output, void *stream);

/* Replaces flow_align_backward_cuda (flow_align_cuda.c:25-44, kernel :57-117).
 * NCHW only.  features_grad (B x C x H x W) and flow_grad (B x 2 x H x W) must
 * be zero-filled by the caller (functions/flow_align.py:36-39); contributions
 * are accumulated with fp32 atomics. */
int vd_flow_align_backward(const float *top_grad, const float *features, const float *flow,
                           int B, int C, int H, int W, float *features_grad, float *flow_grad,
                           void *stream);

/* GroupNorm + fused epilogue.  Replaces the nn.GroupNorm (+ residual add,
 * + ReLU) module sequences of the GN ResNet / FPN / heads (ResNet.py:208-345,
 * FPN.py:96-120,268-274, fast_rcnn_heads.py:228-290,
 * mask_rcnn_heads.py:191-255) with one statistics pass and one apply pass:
 *   out = act(GN(x [+ x2]; gamma, beta) + r),  r per residual_mode:
 *     0: none; 1: residual (same shape); 2: residual nearest-2x upsampled
 *     (B x H/2 x W/2); 3: GN(residual; res_gamma, res_beta) (its own
 *     statistics, the basic_gn_shortcut branch).
 * act: VD_ACT_*.  G groups over C channels (C % G == 0; NHWC needs
 * (C / G) % 4 == 0).  Statistics in double, normalisation in fp32.
 * workspace: vd_group_norm_workspace_size(B, G) bytes (x2 for residual_mode 3).
 * out may alias x (in place) but not residual. */
enum { VD_ACT_NONE = 0, VD_ACT_RELU = 1, VD_ACT_SIGMOID = 2, VD_ACT_TANH = 3 };
enum { VD_GN_ACT = 0, VD_GN_GRU_Z = 1, VD_GN_GRU_R = 2, VD_GN_GRU_H = 3 };

size_t vd_group_norm_workspace_size(int B, int G);

int vd_group_norm_act(const float *x, const float *x2, int B, int C, int H, int W, int G,
                      float eps, const float *gamma, const float *beta, const float *residual,
                      int residual_mode, const float *res_gamma, const float *res_beta, int act,
                      int layout, float *out, void *workspace, size_t ws_bytes, void *stream);

/* ConvGRU gates (lib_vos/vos_nn/convgrucell.py:73-92, use_GN branch):
 *   z  = sigmoid(GN_z(Wz_h(h) + Wz_x(x)))
 *   hr = h * sigmoid(GN_r(Wr_h(h) + Wr_x(x)))
 * zh/zx/rh/rx are the convolution outputs (B x C x H x W in `layout`); h the
 * hidden state.  h == NULL means the zero state (first frame of a sequence, or
 * the static model's fresh state): zh/rh/hr are then unused (the h-side
 * convolutions of a zero state are exactly zero) and only z is produced.
 * workspace: 2 * vd_group_norm_workspace_size(B, G). */
int vd_convgru_gates(const float *zh, const float *zx, const float *rh, const float *rx,
                     const float *h, int B, int C, int H, int W, int G, float eps,
                     const float *gamma_z, const float *beta_z, const float *gamma_r,
                     const float *beta_r, int layout, float *z, float *hr, void *workspace,
                     size_t ws_bytes, void *stream);

/* ConvGRU update + VOS top-down fusion (convgrucell.py:88-91;
 * vos_model_builder.py:335-345):
 *   hn  = (1 - z) * h + z * tanh(GN_h(Wh_h(h * r) + Wh_x(x)))   (h == NULL: z * tanh(..))
 *   out = finer ? hn / 2 + bilinear_0.5x(finer) / 2 : hn
 * hh may be NULL with h (zero state).  finer: the already-fused next-finer level
 * (B x C x 2H x 2W in `layout`), or NULL for the finest level. */
int vd_convgru_update(const float *hh, const float *hx, const float *z, const float *h,
                      const float *finer, int B, int C, int H, int W, int G, float eps,
                      const float *gamma_h, const float *beta_h, int layout, float *out,
                      void *workspace, size_t ws_bytes, void *stream);

/* The fork's steps after the detections limit in box_results_with_nms_and_limit
 * (lib_vos/tools/vos_test.py:805-833), in place on vd_box_detections' outputs:
 * nms_cross_class > 0 -> one NMS (cython semantics) over all classes'
 * detections, survivors regrouped by class in row order (TEST.NMS_CROSS_CLASS);
 * num_det_per_class_pre > 0 -> per class the top-k by score, rows reordered by
 * score (TEST.NUM_DET_PER_CLASS_PRE; ties by row order).  Both off -> no-op.
 * det_cap <= 512. */
int vd_detections_postfilter(float *dets, int32_t *classes, int32_t *counts, int num_images,
                             int det_cap, float nms_cross_class, int num_det_per_class_pre,
                             void *stream);

/* vd_bias_relu_maxpool: the stem tail of basic_bn_stem (lib/modeling/ResNet.py:
 * 224-230) after a bias-free conv1: out = MaxPool2d(3, 2, 1)(relu(x + bias[c])),
 * x N x H x W x C (NHWC), out N x Ho x Wo x C with Ho = (H - 1) / 2 + 1,
 * Wo = (W - 1) / 2 + 1.  Bit-identical to vd_bias_act followed by the max-pool.
 * C % 4 == 0. */
int vd_bias_relu_maxpool(const float *x, const float *bias, int N, int C, int H, int W,
                         float *out, void *stream);

/* vd_rpn_head: the FPN RPN head of one level after its shared 3x3 conv
 * (lib/modeling/FPN.py:376-422, test branch): x = the conv's raw output WITHOUT
 * its bias, N x H x W x C (NHWC, contiguous); conv_bias [C]; w [5A][C] = the
 * cls_score (A rows) then bbox_pred (4A rows) 1x1 weights, b [5A] their biases.
 * Writes cls_prob N x A x H x W = sigmoid(w_cls . relu(x + conv_bias) + b_cls)
 * and bbox_pred N x 4A x H x W (NCHW), the layouts vd_generate_proposals reads.
 * C % 64 == 0, 5A <= 16 (else VD_ERR_SHAPE). */
int vd_rpn_head(const float *x, const float *conv_bias, const float *w, const float *b, int N,
                int H, int W, int C, int A, float *cls_prob, float *bbox_pred, void *stream);

/* ---------------------------------------------------------------------------
 * segm_results (lib/core/test.py:801-855; fork lib_vos/tools/vos_test.py:867-921)
 * on the device, SURVEY.md section 8f row 3.
 *
 * vd_paste_masks: masks M x R x R fp32 (each detection's class-selected mask
 * probabilities, i.e. masks[mask_ind, j]), boxes M x box_stride fp32
 * (x1, y1, x2, y2 in image coordinates, the cls_boxes rows) -> out M x im_h x
 * im_w u8 (row-major, every byte written): box_utils.expand_boxes by
 * (R+2)/R (boxes.py:242-258) + astype(int32), cv2.resize(padded_mask, (w, h))
 * INTER_LINEAR (OpenCV's scalar float path, restated), `> thresh`
 * (MRCNN.THRESH_BINARIZE), pasted into the clipped box.  R <= 62.
 *
 * vd_mask_rle: pycocotools mask.encode counts of each M x H x W u8 plane in
 * column-major (Fortran) order: counts[m][0..n) with n = ncounts[m], the
 * first run counting zeros.  If a plane needs more than `cap` runs,
 * ncounts[m] = -n and its counts are not written (call again with cap >= n).
 * The run lengths -> ASCII string step (rleToString) is vd_rle_strings.
 * ------------------------------------------------------------------------- */
int vd_paste_masks(const float *masks, int M, int R, const float *boxes, int box_stride,
                   int im_h, int im_w, float thresh, uint8_t *out, void *stream);
int vd_mask_rle(const uint8_t *masks, int M, int H, int W, uint32_t *counts, int cap,
                int32_t *ncounts, void *stream);

/* vd_segm_rle: vd_paste_masks followed by vd_mask_rle in one launch, without
 * the M x im_h x im_w planes: each detection's pasted values are evaluated in
 * its clipped box only (everything outside is 0) and turned into the same
 * counts / ncounts (retry contract as vd_mask_rle).  im_w <= 8192.
 *
 * vd_rle_strings: pycocotools rleToString (maskApi.c) of each detection's
 * counts[m][0..ncounts[m]).  chars == NULL: lens[m] = the string's length
 * (0 for ncounts[m] <= 0).  chars != NULL: lens must hold those lengths
 * (sum < 2^31); detection m's ASCII string is written at
 * chars[lens[0] + ... + lens[m-1]], unterminated.  Replaces the host-side
 * mask_util.encode(...)['counts'].decode('ascii') of segm_results
 * (lib/core/test.py:844-847). */
int vd_segm_rle(const float *masks, int M, int R, const float *boxes, int box_stride,
                int im_h, int im_w, float thresh, uint32_t *counts, int cap, int32_t *ncounts,
                void *stream);
int vd_rle_strings(const uint32_t *counts, const int32_t *ncounts, int M, int cap,
                   int32_t *lens, uint8_t *chars, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* VOSDET_H_ */
