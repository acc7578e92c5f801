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
#include <stdlib.h>

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
    // tile fill: 16 float4 loads per thread (the whole 64 KiB tile at C = 256)
    // in flight before any is stored (a load -> store loop waits one HBM round
    // trip per float4)
    const float4 *src = reinterpret_cast<const float4 *>(x + p0 * C);
    const int n4 = np * C4, bd = blockDim.x;
    auto put = [&](int i, float4 v) {
        const int p = i / C4, c = (i - p * C4) * 4;
        const float4 cb = *reinterpret_cast<const float4 *>(conv_bias + c);
        v.x = fmaxf(v.x + cb.x, 0.f);
        v.y = fmaxf(v.y + cb.y, 0.f);
        v.z = fmaxf(v.z + cb.z, 0.f);
        v.w = fmaxf(v.w + cb.w, 0.f);
        *reinterpret_cast<float4 *>(tile + p * C + (((c >> 2) ^ (p & 15)) << 2)) = v;
    };
    constexpr int U = 16;
    int i = threadIdx.x;
    for (; i + (U - 1) * bd < n4; i += U * bd) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = src[i + u * bd];
#pragma unroll
        for (int u = 0; u < U; ++u) put(i + u * bd, v[u]);
    }
    for (; i < n4; i += bd) put(i, src[i]);
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

// MFMA form (C = 256, 5A <= 16): a wave computes 16 pixels x 16 outputs per
// step with v_mfma_f32_16x16x4_f32, straight from global memory, no LDS tile.
// Lane l: pixel (block base + l % 16), channel group kq = l / 16.  For step s
// (0..15) the lane loads the float4 of channels 16 s + 4 kq .. + 3 of its pixel
// (the 4 lane groups read 64 contiguous bytes of each pixel; over the 16 steps
// every byte of the 1 KiB pixel once), applies bias + ReLU, and feeds the 4
// values to 4 MFMAs as A[pixel][k = kq]; B[k = kq][n = l % 16] is the matching
// weight, held in 64 VGPRs for the whole launch.  The k order is a permutation
// of the channels, shared by A and B, so D = relu(x + b_conv) . W^T exactly up
// to summation order.  D: lane l, register r = output n = l % 16 of pixel
// 4 kq + r.  16 loads (16 KiB per wave) are in flight per step block.
__global__ __launch_bounds__(256) void rpn_head_mfma_kernel(
    const float *__restrict__ x, const float *__restrict__ conv_bias,
    const float *__restrict__ w, const float *__restrict__ b, int A, int64_t npix, int HW,
    float *__restrict__ cls_prob, float *__restrict__ bbox_pred) {
    constexpr int C = 256, S = C / 16;
    typedef float f4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) float cb_s[C];
    for (int i = threadIdx.x; i < C; i += blockDim.x) cb_s[i] = conv_bias[i];
    __syncthreads();
    const int lane = lane_id(), n = lane & 15, kq = lane >> 4;
    const int cout = 5 * A;
    float4 wr[S];
#pragma unroll
    for (int s = 0; s < S; ++s)
        wr[s] = n < cout ? *reinterpret_cast<const float4 *>(w + (int64_t)n * C + 16 * s + 4 * kq)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
    const float bn = n < cout ? b[n] : 0.f;
    const int64_t nblk = (npix + 15) / 16;
    const int64_t wave0 = (int64_t)blockIdx.x * num_waves() + wave_id();
    const int64_t nwaves = (int64_t)gridDim.x * num_waves();
    for (int64_t blk = wave0; blk < nblk; blk += nwaves) {
        int64_t p = blk * 16 + n;
        if (p >= npix) p = npix - 1;  // tail lanes read a valid pixel, result dropped
        const float4 *xp = reinterpret_cast<const float4 *>(x + p * C + 4 * kq);
        float4 a[S];
#pragma unroll
        for (int s = 0; s < S; ++s) a[s] = xp[4 * s];
        f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const float4 cb = *reinterpret_cast<const float4 *>(cb_s + 16 * s + 4 * kq);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fmaxf(a[s].x + cb.x, 0.f), wr[s].x, acc,
                                                      0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fmaxf(a[s].y + cb.y, 0.f), wr[s].y, acc,
                                                      0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fmaxf(a[s].z + cb.z, 0.f), wr[s].z, acc,
                                                      0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fmaxf(a[s].w + cb.w, 0.f), wr[s].w, acc,
                                                      0, 0, 0);
        }
        if (n >= cout) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t pp = blk * 16 + 4 * kq + r;
            if (pp >= npix) break;
            const int64_t img = pp / HW, q = pp - img * HW;
            const float o = acc[r] + bn;
            if (n < A)
                cls_prob[(img * A + n) * HW + q] = 1.f / (1.f + expf(-o));
            else
                bbox_pred[(img * 4 * A + (n - A)) * HW + q] = o;
        }
    }
}

int launch_rpn_head(const float *x, const float *conv_bias, const float *w, const float *b,
                    int N, int H, int W, int C, int A, float *cls_prob, float *bbox_pred,
                    hipStream_t s) {
    const int64_t npix = (int64_t)N * H * W;
    if (npix == 0) return VD_OK;
    if (C % 64 != 0 || A < 1 || 5 * A > 16) return VD_ERR_SHAPE;  // swizzle: 16 | C/4
    const size_t lds = ((size_t)kRpnTile * C + (size_t)C * 16) * 4;
    if (lds > VD_LDS_BYTES) return VD_ERR_SHAPE;
    const char *e = getenv("VOSDET_RPN_HEAD_MFMA");
    if (C == 256 && !(e && e[0] == '0')) {
        const int64_t waves = (npix + 15) / 16;
        int64_t grid = (waves + 3) / 4;
        if (grid > 256 * 8) grid = 256 * 8;  // grid-stride over 16-pixel blocks
        hipLaunchKernelGGL(rpn_head_mfma_kernel, dim3((unsigned)grid), dim3(256), 0, s, x,
                           conv_bias, w, b, A, npix, H * W, cls_prob, bbox_pred);
        return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
    }
    const int64_t blocks = (npix + kRpnTile - 1) / kRpnTile;
    hipLaunchKernelGGL(rpn_head_kernel, dim3((unsigned)blocks), dim3(256), lds, s, x, conv_bias,
                       w, b, C, A, npix, H * W, cls_prob, bbox_pred);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
