// The FPN top-down lateral step as ONE hand-written fp32 MFMA GEMM with the
// nearest-2x top-down add in its epilogue (reference: lib/modeling/FPN.py:292-300
// topdown_lateral_module.forward: lat = conv_lateral(lateral) (1x1 + bias);
// td = F.upsample(top, scale_factor=2, mode='nearest'); return lat + td):
//
//   D[p][co] = (A[p][0..K) . W[co][0..K) + bias[co]) + T[up(p)][co],  co < 256
//   p = (n * H + y) * Wd + x,  up(p) = (n * H/2 + y/2) * Wd/2 + x/2
//
// A = the lateral (res2..res4 output, NHWC rows), T = the coarser level's
// inner map (NHWC, H/2 x Wd/2), D = this level's inner map.  Before this kernel
// the step ran hipBLASLt's GEMM (D written) and a separate pass that read D and
// T and wrote D again: at P2 of a 32-frame step 2.2 GB read + 2.2 GB written for
// the add alone.
//
// Shape of the work: K in {256, 512, 1024} input channels, N = 256 output
// channels (cfg.FPN.DIM), M = F * H * Wd pixels.  2 M K N flops against
// 4 (M K + M N + M N / 4) bytes: MFMA-bound at every level (P2: 282 GFLOP vs
// 5.0 GB per 32 frames, 1.79 ms at the fp32 matrix peak vs 0.62 ms at 8 TB/s).
//
// Mapping (v_mfma_f32_16x16x4_f32, as gemm1x1.hip): the MFMA's A operand is a
// 16-output-channel weight tile, its B operand a 16-pixel block; lane l holds
// pixel l % 16 and the float4 of input channels 4 (l / 16) .. + 3 of each
// 16-channel group kb, and its 4 accumulators are 4 consecutive output
// channels of its pixel (D and T move as float4s).
//   * A workgroup of 4 waves owns a tile of 4 x NB x 16 pixels and all 256
//     output channels: a wave keeps NB x 16 tiles x 4 accumulators for the
//     whole K loop (NB = 1 for the top-down form: the 16 top-down float4s of a
//     block must fit beside them in the 256 registers of two waves per SIMD).
//   * W streams through LDS in 32-input-channel chunks (32 KiB each, double
//     buffered: 64 KiB, two workgroups per CU), pre-arranged once per model in
//     the per-lane fragment order (vd_fpn_lateral_weight), so a chunk is one
//     contiguous LDS-DMA (global_load_lds_dwordx4, no registers) and every LDS
//     read one conflict-free ds_read_b128 at lane * 16 bytes.  Each weight
//     float4 read from LDS feeds NB x 4 MFMAs.
//   * Workgroups are persistent (two per CU) and walk (tile, chunk) steps as one
//     flattened loop: the next chunk's weights and pixel inputs are in flight
//     while this chunk's MFMAs run, across tile boundaries too; the top-down
//     rows of a tile are loaded during its last step's MFMAs.
//   * vmcnt discipline: the compiler counts only its own loads, not the asm DMA,
//     so every DMA is issued after the step's first use of each input register
//     (pinned by a scheduling barrier), and the epilogue step is a separate
//     straight-line copy of the step (no merged counts at a join).
//   * XCD-aware: workgroup b runs on XCD b % 8; workers are numbered
//     (b % 8) * (G / 8) + b / 8, so the tiles one XCD walks at a time are
//     neighbours and the top-down rows two output rows share come from one L2.
// Measured (profiles/r05/fpn_lateral/ab.jsonl, 32 frames): P2 (K = 256) 2.64 ms
// vs 3.13 ms for hipBLASLt's GEMM + the separate add; P3 even; P4 slower (the
// engine fuses P2 only, modeling._fpn_lateral_fused_k).
#include <stdlib.h>

#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kN = 256;                     // output channels
constexpr int kNT = kN / 16;                // 16-channel output tiles
constexpr int kChunk = 32;                  // input channels per LDS chunk
constexpr int kKB = kChunk / 16;            // 16-channel groups per chunk
constexpr int kChunkF4 = kNT * kKB * 64;    // float4s per chunk (32 KiB)
constexpr int kWaves = 4, kThreads = 64 * kWaves;

__device__ __forceinline__ void lat_dma_1k(const float4 *src, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(lds)
        : "memory");
}

// vmcnt waits as immediates
template <int N>
__device__ __forceinline__ void wait_vm() {
    if constexpr (N == 0)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 1)
        asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
}

// Two workgroups of 4 waves per CU (64 KiB of LDS each), so one workgroup's
// epilogue -- the top-down reads, latency-bound -- runs while the other's MFMAs
// keep the matrix pipes busy.
template <int K, int NB, bool UP>
__global__ __launch_bounds__(kThreads, 2) void fpn_lateral_kernel(
    const float *__restrict__ A, const float4 *__restrict__ Wf, const float *__restrict__ bias,
    const float *__restrict__ T, float *__restrict__ D, int64_t M, int H, int Wd, int tprobe) {
    constexpr int NC = K / kChunk, TP = kWaves * NB * 16;  // chunks per tile, pixels per tile
    __shared__ __attribute__((aligned(16))) float4 wbuf[2][kChunkF4];
    __shared__ float bias_s[kN];
    for (int i = threadIdx.x; i < kN; i += kThreads) bias_s[i] = bias[i];

    const int lane = lane_id(), pj = lane & 15, q = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int G = gridDim.x;  // a multiple of 8
    const int worker = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
    const int64_t ntiles = (M + TP - 1) / TP;
    if (worker >= ntiles) return;  // whole workgroup: no barrier is skipped by part of it
    const int64_t nmine = (ntiles - worker + G - 1) / G;
    const int64_t steps = nmine * NC;

    auto pix = [&](int64_t tile, int b) {
        const int64_t p = tile * TP + (wv * NB + b) * 16 + pj;
        return p < M ? p : M - 1;  // tail lanes compute on a valid pixel; stores dropped
    };
    // a chunk's 32 KiB of weights straight from L2 into LDS: 32 wave instructions of
    // 1 KiB, 8 per wave, no registers
    const uint32_t wbase = (uint32_t)(uintptr_t)&wbuf[0][0];
    auto dma_w = [&](int64_t st) {
        const float4 *src = Wf + (size_t)(st % NC) * kChunkF4 + lane;
        const uint32_t dst = wbase + (uint32_t)((st & 1) * kChunkF4 * 16);
#pragma unroll
        for (int e = 0; e < kChunkF4 / 64 / kWaves; ++e) {
            const int k = wv + kWaves * e;
            lat_dma_1k(src + k * 64, dst + (uint32_t)(k * 1024));
        }
    };

    float4 x[NB][kKB];
    dma_w(0);
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int kb = 0; kb < kKB; ++kb)
            x[b][kb] = *reinterpret_cast<const float4 *>(A + pix(worker, b) * K + 4 * q + 16 * kb);
    wait_vm<0>();
    __syncthreads();

    f4v acc[NB][kNT];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int t = 0; t < kNT; ++t) acc[b][t] = f4v{0.f, 0.f, 0.f, 0.f};

    // the top-down rows of one 16-pixel block: 16 float4 (channels 16 t + 4 q ..)
    auto load_top = [&](int64_t tile, int b, float4 (&r)[kNT]) {
        const int64_t p = pix(tile, b);
        const int64_t hw = (int64_t)H * Wd;
        const int64_t n = p / hw;
        const int rem = (int)(p - n * hw);
        const int y = rem / Wd, xx = rem - y * Wd;
        int64_t trow = (n * (H >> 1) + (y >> 1)) * (int64_t)(Wd >> 1) + (xx >> 1);
        // research probes (VOSDET_LATERAL_PROBE, wrong results): 1 one row for all,
        // 2 no loads, 4 row p / 4 (no division)
        if (tprobe & 1) trow = 0;
        if (tprobe & 4) trow = p >> 2;
        const float *tr = T + trow * kN + 4 * q;
        if (tprobe & 2) {
#pragma unroll
            for (int t = 0; t < kNT; ++t) r[t] = make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
#pragma unroll
            for (int t = 0; t < kNT; ++t) r[t] = *reinterpret_cast<const float4 *>(tr + 16 * t);
        }
    };

    // One step = one 32-channel chunk of one tile.  The body exists twice, for plain
    // steps and for a tile's last (epilogue) step, so each copy is straight-line code
    // and the compiler's vmcnt counts never merge two paths' pending loads (a merge
    // takes the stricter count: a conditional load before a use would be waited for).
#define VD_LAT_STEP(EPI_)                                                                    \
    {                                                                                        \
        constexpr bool EPI = EPI_;                                                           \
        const int64_t ntile = worker + ((st + 1) / NC) * G;                                 \
        const int nc = (int)((st + 1) % NC);                                                \
        const int64_t tile = worker + (st / NC) * G;                                        \
        /* NB = 1: the top-down rows, issued after the first use of this step's inputs */   \
        /* and before its MFMAs: the step's MFMAs hide their latency (the CU's two */       \
        /* workgroups run in lockstep -- the same work per step -- so neither covers */     \
        /* the other's epilogue) */                                                         \
        float4 r[kNT];                                                                      \
        const float4 *wl = wbuf[st & 1] + lane;                                             \
_Pragma("unroll")                                                                           \
        for (int kb = 0; kb < kKB; ++kb) {                                                  \
_Pragma("unroll")                                                                           \
            for (int t = 0; t < kNT; ++t) {                                                 \
                /* The next chunk's weights (into the other buffer, whose last readers */   \
                /* passed the previous barrier) are issued only after this step's first */  \
                /* use of every x register: the compiler's vmcnt waits count its own */     \
                /* loads, not this asm, so a DMA issued before a load it waits on would */  \
                /* be waited for too.  After the last step: a valid chunk into a buffer */  \
                /* nobody reads. */                                                         \
                if (kb == kKB - 1 && t == 1) {                                              \
                    __builtin_amdgcn_sched_barrier(0); /* after x's first uses */        \
                    dma_w(st + 1);                                                          \
                    if (EPI && UP && NB == 1) {                                             \
                        load_top(tile, 0, r);                                               \
                        __builtin_amdgcn_sched_barrier(0); /* kept here, not sunk */        \
                    }                                                                       \
                }                                                                           \
                const float4 w = wl[(t * kKB + kb) * 64];                                   \
_Pragma("unroll")                                                                           \
                for (int b = 0; b < NB; ++b) {                                              \
                    acc[b][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.x, x[b][kb].x, acc[b][t], 0, 0, 0);\
                    acc[b][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.y, x[b][kb].y, acc[b][t], 0, 0, 0);\
                    acc[b][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.z, x[b][kb].z, acc[b][t], 0, 0, 0);\
                    acc[b][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w.w, x[b][kb].w, acc[b][t], 0, 0, 0);\
                }                                                                           \
            }                                                                               \
            /* x[.][kb] is dead for this step: the next step's inputs go into its registers */\
            /* (after the last step: clamped to a valid pixel, never used) */               \
_Pragma("unroll")                                                                           \
            for (int b = 0; b < NB; ++b)                                                    \
                x[b][kb] = *reinterpret_cast<const float4 *>(A + pix(ntile, b) * K + kChunk * nc +\
                                                             4 * q + 16 * kb);              \
        }                                                                                   \
        if constexpr (EPI) { /* the tile's epilogue: + bias (+ the upsampled top) -> D */  \
            /* NB = 2: block 1's top-down rows are loaded before block 0's stores, so */    \
            /* waiting for them never waits for a store (vmcnt retires loads and stores */  \
            /* in issue order) */                                                           \
            if (UP && NB > 1) load_top(tile, 0, r);                                         \
            __builtin_amdgcn_sched_barrier(0);                                              \
_Pragma("unroll")                                                                           \
            for (int b = 0; b < NB; ++b) {                                                  \
                /* tail lanes (past M) computed pixel M - 1 exactly as its own lane */   \
                /* did (same inputs, same MFMA column arithmetic) and store the same */  \
                /* bits there: unconditional stores, so the compiler cannot sink the */ \
                /* epilogue and the top-down loads into a branch */                      \
                const int64_t p = pix(tile, b);                                          \
                float *dr = D + p * kN + 4 * q;                                             \
_Pragma("unroll")                                                                           \
                for (int t = 0; t < kNT; ++t) {                                             \
                    const float4 bb = *reinterpret_cast<const float4 *>(bias_s + 16 * t + 4 * q);\
                    /* (conv + bias) + top-down: the reference's evaluation order */        \
                    const float4 rt = UP ? r[t] : make_float4(0.f, 0.f, 0.f, 0.f);          \
                    acc[b][t] = f4v{(acc[b][t][0] + bb.x) + rt.x, (acc[b][t][1] + bb.y) + rt.y,\
                                    (acc[b][t][2] + bb.z) + rt.z, (acc[b][t][3] + bb.w) + rt.w};\
                }                                                                           \
                if (UP && b + 1 < NB) {                                                     \
                    load_top(tile, b + 1, r);                                               \
                    __builtin_amdgcn_sched_barrier(0);                                      \
                }                                                                           \
_Pragma("unroll")                                                                           \
                for (int t = 0; t < kNT; ++t)                                               \
                    *reinterpret_cast<f4v *>(dr + 16 * t) = acc[b][t];                      \
                __builtin_amdgcn_sched_barrier(0);                                          \
_Pragma("unroll")                                                                           \
                for (int t = 0; t < kNT; ++t) acc[b][t] = f4v{0.f, 0.f, 0.f, 0.f};          \
            }                                                                               \
            /* its loads and stores came after the next chunk's weights */                  \
            wait_vm<0>();                                                                   \
        } else {                                                                            \
            /* the next chunk's weights must have landed in LDS before the barrier; the */  \
            /* NB input loads issued after them (the last x group) may stay in flight */    \
            /* (vmcnt counts in issue order) */                                             \
            wait_vm<NB>();                                                                  \
        }                                                                                   \
        __syncthreads();                                                                    \
    }

    for (int64_t st = 0; st < steps;) {
#pragma unroll 1
        for (int c = 0; c < NC - 1; ++c, ++st) VD_LAT_STEP(false)
        VD_LAT_STEP(true)
        ++st;
    }
#undef VD_LAT_STEP
}

// W [256][K] (the conv weight, row-major) -> Wf [K/32][16 t][2 kb][64 lanes] float4,
// lane l = 16 q + r holding W[16 t + r][32 c + 16 kb + 4 q .. + 3]
__global__ void fpn_lateral_weight_kernel(const float *__restrict__ W, int K,
                                          float4 *__restrict__ Wf) {
    const int64_t n = (int64_t)(K / kChunk) * kChunkF4;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i / kChunkF4), j = (int)(i % kChunkF4);
        const int l = j & 63, tk = j >> 6, t = tk / kKB, kb = tk % kKB;
        Wf[i] = *reinterpret_cast<const float4 *>(W + (int64_t)(16 * t + (l & 15)) * K + kChunk * c +
                                                  16 * kb + 4 * (l >> 4));
    }
}

int tprobe() {
    static const int p = [] {
        const char *e = getenv("VOSDET_LATERAL_PROBE");
        return e ? atoi(e) : 0;
    }();
    return p;
}

template <int K, int NB, bool UP>
int launch_k(const float *A, int64_t M, const float4 *Wf, const float *bias, const float *T,
             float *D, int H, int Wd, int cus, hipStream_t s) {
    constexpr int TP = kWaves * NB * 16;
    const int64_t ntiles = (M + TP - 1) / TP;
    int64_t grid = 2 * (int64_t)cus;  // two resident workgroups per CU
    if (grid > ntiles) grid = ntiles;
    grid = (grid + 7) / 8 * 8;
    hipLaunchKernelGGL((fpn_lateral_kernel<K, NB, UP>), dim3((unsigned)grid), dim3(kThreads), 0, s,
                       A, Wf, bias, T, D, M, H, Wd, tprobe());
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int cu_count() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        hipDeviceProp_t prop;
        n = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
                ? prop.multiProcessorCount
                : 256;
    }
    return n;
}

}  // namespace

bool fpn_lateral_supported(int K, int N) { return N == kN && (K == 256 || K == 512 || K == 1024); }

int launch_fpn_lateral_weight(const float *W, int N, int K, float *Wf, hipStream_t s) {
    if (!fpn_lateral_supported(K, N)) return VD_ERR_SHAPE;
    hipLaunchKernelGGL(fpn_lateral_weight_kernel, dim3(256), dim3(256), 0, s, W, K,
                       reinterpret_cast<float4 *>(Wf));
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int launch_fpn_lateral(const float *A, int64_t M, int K, const float *Wf, int N, const float *bias,
                       const float *T, int H, int Wd, float *D, hipStream_t s) {
    if (!fpn_lateral_supported(K, N)) return VD_ERR_SHAPE;
    if (M == 0) return VD_OK;
    if (T && ((H & 1) || (Wd & 1) || H <= 0 || Wd <= 0 || M % ((int64_t)H * Wd))) return VD_ERR_ARG;
    const float4 *wf = reinterpret_cast<const float4 *>(Wf);
    const int cus = cu_count();
    // 128-pixel tiles (NB = 2) when there are >= 4 per workgroup slot and no top-down
    // term (with it, NB = 2 needs more than the 256 registers of two waves per SIMD);
    // else 64 (NB = 1).  VOSDET_LATERAL_NB=1|2 forces one (A/B measurements).
    static const int force_nb = [] {
        const char *e = getenv("VOSDET_LATERAL_NB");
        return e ? atoi(e) : 0;
    }();
    const bool big = force_nb ? force_nb == 2 : (!T && M >= (int64_t)cus * 2 * 128 * 4);
#define VD_LAT(KK)                                                                            \
    if (K == KK) {                                                                            \
        if (big) return T ? launch_k<KK, 2, true>(A, M, wf, bias, T, D, H, Wd, cus, s)        \
                          : launch_k<KK, 2, false>(A, M, wf, bias, T, D, H, Wd, cus, s);      \
        return T ? launch_k<KK, 1, true>(A, M, wf, bias, T, D, H, Wd, cus, s)                 \
                 : launch_k<KK, 1, false>(A, M, wf, bias, T, D, H, Wd, cus, s);               \
    }
    VD_LAT(256)
    VD_LAT(512)
    VD_LAT(1024)
#undef VD_LAT
    return VD_ERR_SHAPE;
}

}  // namespace vd
