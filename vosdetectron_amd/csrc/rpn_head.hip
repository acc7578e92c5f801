// FPN RPN head outputs on the raw shared-conv output, one pass over HBM.
//
// Reference: lib/modeling/FPN.py:376-422 fpn_rpn_outputs (test branch):
//   conv_rpn = relu(FPN_RPN_conv(x) + b)          (3x3, dim_in -> dim_in)
//   cls_prob  = sigmoid(FPN_RPN_cls_score(conv_rpn))   (1x1, -> A)
//   bbox_pred = FPN_RPN_bbox_pred(conv_rpn)            (1x1, -> 4A)
// The 3x3 conv stays on MIOpen (MFMA) and is run WITHOUT its bias; this kernel
// reads its NHWC output once, applies bias + ReLU on the way into LDS, and
// evaluates both 1x1 convs (5A <= 16 outputs) and the sigmoid, writing the
// NCHW cls_prob / bbox_pred planes vd_generate_proposals reads.  That replaces
// the bias+ReLU read-modify-write pass, the 15-wide GEMM's read of the same
// tensor and the slicing / sigmoid copies: HBM bytes per pixel 4*C read +
// 4*5A written (memory-bound, 16 flop/B at C = 256).
//
// Work: a workgroup stages 64 consecutive pixels (64 x C floats, contiguous
// in NHWC) in LDS, pixel p's 16-byte chunk k stored at chunk k ^ (p & 15) so a
// lane-per-pixel ds_read_b128 is bank-conflict free without padding (64 KiB +
// 16 KiB of weights: two workgroups per CU); wave w then computes outputs 4w..4w+3
// for the 64 pixels (lane = pixel, channel-uniform weights from a transposed
// [C][16] copy held in LDS and read as broadcasts).  Sums run over the
// channels in order with FMA (the 1x1 convolutions' summation order is the
// library's in the reference: tolerance, not bit parity).
#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

static constexpr int kRpnTile = 64;

__global__ __launch_bounds__(256) void rpn_head_kernel(
    const float *__restrict__ x, const float *__restrict__ conv_bias,
    const float *__restrict__ w, const float *__restrict__ b, int C, int A, int64_t npix,
    int HW, float *__restrict__ cls_prob, float *__restrict__ bbox_pred) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float *tile = lds;                  // [64][C], chunks XOR-swizzled by pixel
    float *wt = lds + kRpnTile * C;     // [C][16] transposed weights
    const int cout = 5 * A;
    const int64_t p0 = (int64_t)blockIdx.x * kRpnTile;
    const int np = (int)min((int64_t)kRpnTile, npix - p0);
    const int C4 = C / 4;
    for (int i = threadIdx.x; i < C * 16; i += blockDim.x) {
        const int c = i >> 4, j = i & 15;
        wt[i] = j < cout ? w[(int64_t)j * C + c] : 0.f;
    }
    const float *src = x + p0 * C;
    for (int i = threadIdx.x; i < np * C4; i += blockDim.x) {
        const int p = i / C4, c = (i - p * C4) * 4;
        float4 v = *reinterpret_cast<const float4 *>(src + (int64_t)i * 4);
        const float4 cb = *reinterpret_cast<const float4 *>(conv_bias + c);
        v.x = fmaxf(v.x + cb.x, 0.f);
        v.y = fmaxf(v.y + cb.y, 0.f);
        v.z = fmaxf(v.z + cb.z, 0.f);
        v.w = fmaxf(v.w + cb.w, 0.f);
        *reinterpret_cast<float4 *>(tile + p * C + (((c >> 2) ^ (p & 15)) << 2)) = v;
    }
    __syncthreads();
    const int lane = lane_id(), j0 = 4 * wave_id();
    if (j0 >= cout || lane >= np) return;
    const float *row = tile + lane * C;
    const int sw = lane & 15;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
    for (int c = 0; c < C; c += 4) {
        const float4 v = *reinterpret_cast<const float4 *>(row + (((c >> 2) ^ sw) << 2));
        const float xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 wk = *reinterpret_cast<const float4 *>(wt + (c + k) * 16 + j0);
            acc0 = fmaf(wk.x, xs[k], acc0);
            acc1 = fmaf(wk.y, xs[k], acc1);
            acc2 = fmaf(wk.z, xs[k], acc2);
            acc3 = fmaf(wk.w, xs[k], acc3);
        }
    }
    const int64_t pp = p0 + lane;
    const int64_t n = pp / HW, q = pp - n * HW;
    const float accs[4] = {acc0, acc1, acc2, acc3};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = j0 + k;
        if (j >= cout) break;
        const float o = accs[k] + b[j];
        if (j < A)
            cls_prob[(n * A + j) * HW + q] = 1.f / (1.f + expf(-o));
        else
            bbox_pred[(n * 4 * A + (j - A)) * HW + q] = o;
    }
}

int launch_rpn_head(const float *x, const float *conv_bias, const float *w, const float *b,
                    int N, int H, int W, int C, int A, float *cls_prob, float *bbox_pred,
                    hipStream_t s) {
    const int64_t npix = (int64_t)N * H * W;
    if (npix == 0) return VD_OK;
    if (C % 64 != 0 || A < 1 || 5 * A > 16) return VD_ERR_SHAPE;  // swizzle: 16 | C/4
    const size_t lds = ((size_t)kRpnTile * C + (size_t)C * 16) * 4;
    if (lds > 160 * 1024) return VD_ERR_SHAPE;
    const int64_t blocks = (npix + kRpnTile - 1) / kRpnTile;
    hipLaunchKernelGGL(rpn_head_kernel, dim3((unsigned)blocks), dim3(256), lds, s, x, conv_bias,
                       w, b, C, A, npix, H * W, cls_prob, bbox_pred);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
