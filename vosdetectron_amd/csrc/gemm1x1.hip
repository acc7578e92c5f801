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


// S > 1 splits the N output channels over S workgroups of the same XCD
// (block b runs on XCD b % 8; the S splits of a pixel range are blocks
// 8 (S w + s) + xcd), each staging an N / S-channel weight slice, so the
// slices fit LDS and the pixel rows they share are read from one L2.
//
// K2 > 0: a second input operand A2 [M][K2] contributes the last K2 of the K
// input channels (W = [W1 | W2], K = K1 + K2): the ResNet stage's first block
// as ONE kernel, conv3 and the stride-1 downsample of the block input summed
// in the accumulators -- relu(h W3^T + x Wd^T + b3 + bd) -- instead of the
// downsample conv's output written and read back as the residual.
template <int K, int K2, int NFULL, int S, bool RES, bool RELU>
__global__ __launch_bounds__(512, 4) void gemm1x1_mfma_kernel(const float *__restrict__ A,
                                                           const float *__restrict__ A2,
                                                           const float *__restrict__ W,
                                                           const float *__restrict__ bias,
                                                           const float *__restrict__ R,
                                                           float *__restrict__ D, int64_t M) {
    constexpr int N = NFULL / S, NT = N / 16, KB = K / 16;
    extern __shared__ __attribute__((aligned(16))) float4 wfrag[];  // [NT][KB][64] + bias[N]
    float *bias_s = reinterpret_cast<float *>(wfrag + NT * KB * 64);
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int split = slot % S;
    const int n0 = split * N;
    const int64_t worker = (int64_t)(slot / S) * 8 + xcd, nworkers = gridDim.x / S;
    for (int i = threadIdx.x; i < NT * KB * 64; i += blockDim.x) {
        const int l = i & 63, tk = i >> 6;
        const int t = tk / KB, kb = tk - t * KB;
        wfrag[i] = *reinterpret_cast<const float4 *>(W + (int64_t)(n0 + 16 * t + (l & 15)) * K +
                                                     16 * kb + 4 * (l >> 4));
    }
    for (int i = threadIdx.x; i < N; i += blockDim.x) bias_s[i] = bias ? bias[n0 + i] : 0.f;
    __syncthreads();
    const int lane = lane_id(), pj = lane & 15, q = lane >> 4;
    const int64_t nblk = (M + 15) / 16;
    const int64_t nw = nworkers * num_waves();
    // the next block's inputs are loaded while this block's groups run
    constexpr int K1 = K - K2, KB1 = K1 / 16;
    auto load_x = [&](int64_t blk, float4 (&x)[KB]) {
        const int64_t p = min(blk * 16 + pj, M - 1);
        const float *ap = A + p * K1 + 4 * q;
        const float *ap2 = A2 + p * K2 + 4 * q;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
            x[kb] = kb < KB1 ? *reinterpret_cast<const float4 *>(ap + 16 * kb)
                             : *reinterpret_cast<const float4 *>(ap2 + 16 * (kb - KB1));
    };
    int64_t blk = worker * num_waves() + wave_id();
    float4 x[KB];
    if (blk < nblk) load_x(blk, x);
    for (; blk < nblk; blk += nw) {
        int64_t p = blk * 16 + pj;
        const bool live = p < M;
        if (!live) p = M - 1;  // tail lanes compute on a valid pixel; their stores are dropped
        float4 xn[KB];
        if (blk + nw < nblk) load_x(blk + nw, xn);
        const int64_t orow = p * NFULL + n0 + 4 * q;
        // channel tiles in groups of G: a group's residual / output float4s of a
        // pixel are G x 64 contiguous bytes touched by back-to-back instructions
        // (whole 128-byte lines while they are in L2); the next group's residual
        // is loaded while this group's MFMAs run
        constexpr int G = (NT >= 8 && K <= 64) ? 4 : (NT >= 2 ? 2 : 1), NG = NT / G;
        float4 r[G], rn[G];
#pragma unroll
        for (int u = 0; u < G; ++u)
            r[u] = RES ? *reinterpret_cast<const float4 *>(R + orow + 16 * u)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 1
        for (int g = 0; g < NG; ++g) {
#pragma unroll
            for (int u = 0; u < G; ++u)
                rn[u] = (RES && g + 1 < NG)
                            ? *reinterpret_cast<const float4 *>(R + orow + 16 * (G * (g + 1) + u))
                            : make_float4(0.f, 0.f, 0.f, 0.f);
            f4v acc[G];
#pragma unroll
            for (int u = 0; u < G; ++u) {
                acc[u] = f4v{0.f, 0.f, 0.f, 0.f};
                const float4 *wt = wfrag + (G * g + u) * KB * 64 + lane;
#pragma unroll
                for (int kb = 0; kb < KB; ++kb) {
                    const float4 w = wt[kb * 64];
                    acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, x[kb].x, acc[u], 0, 0, 0);
                    acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, x[kb].y, acc[u], 0, 0, 0);
                    acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, x[kb].z, acc[u], 0, 0, 0);
                    acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, x[kb].w, acc[u], 0, 0, 0);
                }
            }
#pragma unroll
            for (int u = 0; u < G; ++u) {
                const int t = G * g + u;
                const float4 b = *reinterpret_cast<const float4 *>(bias_s + 16 * t + 4 * q);
                float4 o = make_float4(acc[u][0] + b.x + r[u].x, acc[u][1] + b.y + r[u].y,
                                       acc[u][2] + b.z + r[u].z, acc[u][3] + b.w + r[u].w);
                if (RELU) {
                    o.x = fmaxf(o.x, 0.f);
                    o.y = fmaxf(o.y, 0.f);
                    o.z = fmaxf(o.z, 0.f);
                    o.w = fmaxf(o.w, 0.f);
                }
                if (live) *reinterpret_cast<float4 *>(D + orow + 16 * t) = o;
                r[u] = rn[u];
            }
        }
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) x[kb] = xn[kb];
    }
}

// K >= 128: the K axis is walked in chunks of 64 input channels with the
// accumulators of all N / 16 tiles live (N <= 128), the next chunk's (or the
// next block's first chunk's) inputs loaded while the current chunk's MFMAs
// run -- a flattened (block, chunk) loop, so the prefetch crosses blocks.
template <int K, int N, bool RES, bool RELU>
__global__ __launch_bounds__(512) void gemm1x1_mfma_chunk_kernel(const float *__restrict__ A,
                                                                 const float *__restrict__,
                                                                 const float *__restrict__ W,
                                                                 const float *__restrict__ bias,
                                                                 const float *__restrict__ R,
                                                                 float *__restrict__ D, int64_t M) {
    constexpr int NT = N / 16, KB = K / 16, CH = 4, NCH = KB / CH;
    static_assert(KB % CH == 0 && NT <= 8, "chunked shape");
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
    const int64_t blk0 = (int64_t)blockIdx.x * num_waves() + wave_id();
    if (blk0 >= nblk) return;
    const int64_t nmine = (nblk - blk0 + nw - 1) / nw;  // blocks this wave walks
    auto pixel = [&](int64_t blk) {
        const int64_t p = blk * 16 + pj;
        return p < M ? p : M - 1;  // tail lanes compute on a valid pixel; stores dropped
    };
    auto load_chunk = [&](int64_t blk, int c, float4 (&x)[CH]) {
        const float *ap = A + pixel(blk) * K + 64 * c + 4 * q;
#pragma unroll
        for (int kb = 0; kb < CH; ++kb) x[kb] = *reinterpret_cast<const float4 *>(ap + 16 * kb);
    };
    float4 xc[CH];
    load_chunk(blk0, 0, xc);
    f4v acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f4v{0.f, 0.f, 0.f, 0.f};
    const int64_t steps = nmine * NCH;
#pragma unroll 1
    for (int64_t st = 0; st < steps; ++st) {
        const int64_t blk = blk0 + (st / NCH) * nw;
        const int c = (int)(st % NCH);
        float4 xn[CH];
        if (st + 1 < steps)
            load_chunk(blk0 + ((st + 1) / NCH) * nw, (int)((st + 1) % NCH), xn);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const float4 *wt = wfrag + (t * KB + c * CH) * 64 + lane;
#pragma unroll
            for (int kb = 0; kb < CH; ++kb) {
                const float4 w = wt[kb * 64];
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, xc[kb].x, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, xc[kb].y, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, xc[kb].z, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, xc[kb].w, acc[t], 0, 0, 0);
            }
        }
        if (c == NCH - 1) {
            const int64_t p = blk * 16 + pj;
            const int64_t orow = pixel(blk) * N + 4 * q;
            float4 r[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t)
                r[t] = RES ? *reinterpret_cast<const float4 *>(R + orow + 16 * t)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const float4 b = *reinterpret_cast<const float4 *>(bias_s + 16 * t + 4 * q);
                float4 o = make_float4(acc[t][0] + b.x + r[t].x, acc[t][1] + b.y + r[t].y,
                                       acc[t][2] + b.z + r[t].z, acc[t][3] + b.w + r[t].w);
                if (RELU) {
                    o.x = fmaxf(o.x, 0.f);
                    o.y = fmaxf(o.y, 0.f);
                    o.z = fmaxf(o.z, 0.f);
                    o.w = fmaxf(o.w, 0.f);
                }
                if (p < M) *reinterpret_cast<float4 *>(D + orow + 16 * t) = o;
                acc[t] = f4v{0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int kb = 0; kb < CH; ++kb) xc[kb] = xn[kb];
    }
}

template <int K, int N, int S, bool RES, bool RELU, int K2 = 0>
int launch_shape(const float *A, int64_t M, const float *W, const float *bias, const float *R,
                 float *D, hipStream_t s, const float *A2 = nullptr) {
    constexpr size_t lds = (size_t)(N / S) * K * 4 + (size_t)(N / S) * 4;
    static_assert(lds <= 80 * 1024, "two workgroups per CU");
    constexpr bool chunked = K >= 128 && S == 1 && K2 == 0;
    void (*kern)(const float *, const float *, const float *, const float *, const float *,
                 float *, int64_t);
    if constexpr (chunked)
        kern = gemm1x1_mfma_chunk_kernel<K, N, RES, RELU>;
    else
        kern = gemm1x1_mfma_kernel<K, K2, N, S, RES, RELU>;
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)lds) == hipSuccess;
    if (!attr) return VD_ERR_LAUNCH;
    // persistent: 2 workgroups of 8 waves per CU (LDS: a weight slice + bias each);
    // a multiple of 8 * S blocks so every split of every XCD exists
    const int64_t blocks16 = (M + 15) / 16;
    int64_t grid = 256 * 2;
    const int64_t need = (blocks16 + 7) / 8 * S;
    if (grid > need) grid = need;
    grid = (grid + 8 * S - 1) / (8 * S) * (8 * S);
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(512), lds, s, A, A2, W, bias, R, D, M);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace

bool gemm1x1_mfma_supported(int K, int N) {
    return (K == 64 && (N == 64 || N == 256)) || (K == 256 && N == 64) || (K == 128 && N == 512);
}

int launch_gemm1x1_mfma(const float *A, int M, int K, const float *W, int N, const float *bias,
                        const float *R, int relu, float *D, hipStream_t s) {
    if (M == 0) return VD_OK;
#define VD_G1(KK, NN, SS)                                                                 \
    if (K == KK && N == NN) {                                                             \
        if (R) return relu ? launch_shape<KK, NN, SS, true, true>(A, M, W, bias, R, D, s) \
                           : launch_shape<KK, NN, SS, true, false>(A, M, W, bias, R, D, s); \
        return relu ? launch_shape<KK, NN, SS, false, true>(A, M, W, bias, R, D, s)       \
                    : launch_shape<KK, NN, SS, false, false>(A, M, W, bias, R, D, s);     \
    }
    VD_G1(64, 256, 1)
    VD_G1(64, 64, 1)
    VD_G1(256, 64, 1)
    VD_G1(128, 512, 4)
#undef VD_G1
    return VD_ERR_SHAPE;
}

bool gemm1x1_dual_supported(int K1, int K2, int N) { return K1 == 64 && K2 == 64 && N == 256; }

int launch_gemm1x1_dual(const float *A1, int K1, const float *A2, int K2, int M, const float *W,
                        int N, const float *bias, int relu, float *D, hipStream_t s) {
    if (M == 0) return VD_OK;
    if (!gemm1x1_dual_supported(K1, K2, N)) return VD_ERR_SHAPE;
    return relu ? launch_shape<128, 256, 2, false, true, 64>(A1, M, W, bias, nullptr, D, s, A2)
                : launch_shape<128, 256, 2, false, false, 64>(A1, M, W, bias, nullptr, D, s, A2);
}

}  // namespace vd
