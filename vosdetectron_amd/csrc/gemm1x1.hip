// Stride-1 1x1 convolutions of the ResNet bottlenecks as a hand-written fp32
// MFMA GEMM with the conv epilogue fused, for the skinny shapes hipBLASLt
// leaves far from their roofline (profiles/r02_conv_roofline_search.json: the
// P2-level M = 16*200*336 GEMMs with K = 64 run at 0.33-0.38 of the fp32
// matrix peak, memory-bound on the residual read and the output write).
//
//   D[M][N] = act(A[M][K] . W[N][K]^T + bias[N] (+ R[M][N]))
//
// A, R, D are NHWC activations (row = pixel, contiguous channels), W the conv
// weight [Cout][Cin] with the frozen-BN AffineChannel folded in (reference:
// lib/modeling/ResNet.py:246-294 bottleneck_transformation, conv1 -> relu,
// conv3 + residual -> relu).
//
// Mapping (v_mfma_f32_16x16x4_f32, D[i][j] = sum_k A[i][k] B[k][j] + C):
// the MFMA's A operand is the weight tile (i = output channel), its B operand
// the pixel tile (j = pixel), so a lane's 4 accumulators are 4 CONSECUTIVE
// output channels of one pixel: the residual is read and D written as one
// float4 per lane (the 4 lanes of a pixel cover 64 contiguous bytes; the 16
// channel tiles of a 16-pixel block cover its rows completely).
//   lane l: pixel j = l % 16 of the block, k-group q = l / 16.
//   For channel block kb (16 input channels), the lane holds the float4 of
//   channels 16 kb + 4 q .. + 3 of its pixel; MFMA c (= .x .y .z .w) sums over
//   q the channels 16 kb + 4 q + c -- a permutation of the K axis shared by
//   both operands, so the result is A . W^T up to summation order.
//   The weight operand of (channel tile t, block kb) is the float4
//   W[16 t + l % 16][16 kb + 4 q ..] -- staged once per workgroup in LDS in
//   exactly that per-lane order, so every read is one conflict-free
//   ds_read_b128 at lane * 16 bytes.
// A wave keeps its pixel block's K inputs in registers for all N / 16 channel
// tiles (KB float4s), accumulates one tile at a time (4 VGPRs) and finishes it
// with bias (+ residual) + ReLU straight to HBM.  Workgroups are persistent
// (grid = CUs x resident workgroups) and walk 16-pixel blocks.
#include <stdlib.h>

#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));

template <int K, int N, bool RES, bool RELU>
__global__ __launch_bounds__(512, 4) void gemm1x1_mfma_kernel(const float *__restrict__ A,
                                                           const float *__restrict__ W,
                                                           const float *__restrict__ bias,
                                                           const float *__restrict__ R,
                                                           float *__restrict__ D, int64_t M) {
    constexpr int NT = N / 16, KB = K / 16;
    extern __shared__ __attribute__((aligned(16))) float4 wfrag[];  // [NT][KB][64] + bias[N]
    float *bias_s = reinterpret_cast<float *>(wfrag + NT * KB * 64);
    for (int i = threadIdx.x; i < NT * KB * 64; i += blockDim.x) {
        const int l = i & 63, tk = i >> 6;
        const int t = tk / KB, kb = tk - t * KB;
        wfrag[i] = *reinterpret_cast<const float4 *>(W + (int64_t)(16 * t + (l & 15)) * K +
                                                     16 * kb + 4 * (l >> 4));
    }
    for (int i = threadIdx.x; i < N; i += blockDim.x) bias_s[i] = bias ? bias[i] : 0.f;
    __syncthreads();
    const int lane = lane_id(), pj = lane & 15, q = lane >> 4;
    const int64_t nblk = (M + 15) / 16;
    const int64_t nw = (int64_t)gridDim.x * num_waves();
    for (int64_t blk = (int64_t)blockIdx.x * num_waves() + wave_id(); blk < nblk; blk += nw) {
        int64_t p = blk * 16 + pj;
        const bool live = p < M;
        if (!live) p = M - 1;  // tail lanes compute on a valid pixel; their stores are dropped
        const float *ap = A + p * K + 4 * q;
        float4 x[KB];
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) x[kb] = *reinterpret_cast<const float4 *>(ap + 16 * kb);
        const int64_t orow = p * N + 4 * q;
        // the residual of tile t + 1 is loaded while tile t's MFMAs run
        float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
        if (RES) r = *reinterpret_cast<const float4 *>(R + orow);
#pragma unroll 1
        for (int t = 0; t < NT; ++t) {
            float4 rn = make_float4(0.f, 0.f, 0.f, 0.f);
            if (RES && t + 1 < NT) rn = *reinterpret_cast<const float4 *>(R + orow + 16 * (t + 1));
            f4v acc = {0.f, 0.f, 0.f, 0.f};
            const float4 *wt = wfrag + t * KB * 64 + lane;
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                const float4 w = wt[kb * 64];
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, x[kb].x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, x[kb].y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, x[kb].z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, x[kb].w, acc, 0, 0, 0);
            }
            const float4 b = *reinterpret_cast<const float4 *>(bias_s + 16 * t + 4 * q);
            float4 o = make_float4(acc[0] + b.x, acc[1] + b.y, acc[2] + b.z, acc[3] + b.w);
            if (RES) {
                o.x += r.x;
                o.y += r.y;
                o.z += r.z;
                o.w += r.w;
                r = rn;
            }
            if (RELU) {
                o.x = fmaxf(o.x, 0.f);
                o.y = fmaxf(o.y, 0.f);
                o.z = fmaxf(o.z, 0.f);
                o.w = fmaxf(o.w, 0.f);
            }
            if (live) *reinterpret_cast<float4 *>(D + orow + 16 * t) = o;
        }
    }
}

template <int K, int N, bool RES, bool RELU>
int launch_shape(const float *A, int64_t M, const float *W, const float *bias, const float *R,
                 float *D, hipStream_t s) {
    constexpr size_t lds = (size_t)N * K * 4 + (size_t)N * 4;
    static_assert(lds <= 80 * 1024, "two workgroups per CU");
    auto kern = gemm1x1_mfma_kernel<K, N, RES, RELU>;
    static bool attr = [&] {
        return hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds) == hipSuccess;
    }();
    if (!attr) return VD_ERR_LAUNCH;
    const int64_t blocks16 = (M + 15) / 16;
    int64_t grid = 256 * 2;  // persistent: 2 workgroups (16 waves) per CU
    if (grid * 8 > blocks16) grid = (blocks16 + 7) / 8;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(512), lds, s, A, W, bias, R, D, M);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace

bool gemm1x1_mfma_supported(int K, int N) {
    return (K == 64 && (N == 64 || N == 256)) || (K == 256 && N == 64);
}

int launch_gemm1x1_mfma(const float *A, int M, int K, const float *W, int N, const float *bias,
                        const float *R, int relu, float *D, hipStream_t s) {
    if (M == 0) return VD_OK;
#define VD_G1(KK, NN)                                                                     \
    if (K == KK && N == NN) {                                                             \
        if (R) return relu ? launch_shape<KK, NN, true, true>(A, M, W, bias, R, D, s)     \
                           : launch_shape<KK, NN, true, false>(A, M, W, bias, R, D, s);   \
        return relu ? launch_shape<KK, NN, false, true>(A, M, W, bias, R, D, s)           \
                    : launch_shape<KK, NN, false, false>(A, M, W, bias, R, D, s);         \
    }
    VD_G1(64, 256)
    VD_G1(64, 64)
    VD_G1(256, 64)
#undef VD_G1
    return VD_ERR_SHAPE;
}

}  // namespace vd
