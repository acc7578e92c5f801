// 3x3 stride-1 pad-1 convolution on NHWC fp32 by Winograd F(4x4, 3x3) on the
// MFMA pipes, bias (+ ReLU) epilogue fused.
//
// Same operator as conv3x3.hip / conv3x3_wino.hip (FPN posthoc / RPN conv,
// lib/modeling/FPN.py:227-258, 376-422; ResNet bottleneck conv2,
// lib/modeling/ResNet.py:246-294), computed with 4x fewer multiplies than the
// direct convolution (1.78x fewer than F(2x2,3x3)): every 4x4 output tile is
//   Y = A^T [ sum_ci (G g G^T) (.) (B^T d B) ] A
// with d the tile's 6x6 input patch (Lavin & Gray, "Fast Algorithms for
// Convolutional Neural Networks", interpolation points 0, +-1, +-2, inf).  The sum
// over ci is 36 independent GEMMs M[pos][co][tile] = sum_ci U[pos][co][ci]
// V[pos][ci][tile] on v_mfma_f32_16x16x4_f32 (fp32 in and out).  The transforms
// scale by up to 8 (A) and 5 (B), so the result carries ~4x the rounding error of
// F(2x2,3x3): measured 3.7e-6 of max|y| on 256-channel random data (direct fp32
// 3.9e-7), within the conv tests' 2e-5.
//
// Workgroup = 4 waves, 32 tiles (4 x 8 tiles = 16 x 32 output pixels of one
// image) x 32 output channels; wave w owns 16 tiles (w & 1: tile rows 2(w & 1),
// + 1) x 16 channels (w >> 1) at all 36 positions = 36 MFMA accumulators (144
// VGPRs).  A lane's 36 position values of one (channel, tile) sit in the same
// register slot of its 36 accumulators, so the output transform is lane-local.
//
// K is walked in chunks of 4 input channels (one MFMA k-step per position):
// U's chunk slice (36 x 4 x 32 fp32 = 18 KiB, stored chunk-blocked so it is one
// contiguous run) and the raw 18 x 34-pixel input patch (12 KiB) are copied
// HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4; inline asm so hipcc does not
// drain it), double-buffered, one barrier per chunk, two workgroups per CU (60
// KiB each).  Lane (j, q) = (tile, input channel) transforms its own MFMA B
// fragments -- the 36 values V[pos][q][tile j] -- from the patch in registers.
// LDS layouts: U [pos / 4][ci][co][pos % 4] (one conflict-free ds_read_b128
// gives a lane 4 positions' A fragments); patch pixel (R, C) at 16-B slot
// R * 42 + C + C / 4 (the column skew makes the 16 tiles' taps of every (a, b)
// fall in 16 distinct bank quads: conflict-free ds_read_b32).
#include <stdlib.h>

#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int k4KC = 4;                           // input channels per chunk
constexpr int k4TR = 4, k4TC = 8;                 // tiles per block: 16 x 32 pixels
constexpr int k4PR = 4 * k4TR + 2, k4PC = 4 * k4TC + 2;  // 18 x 34 patch
constexpr int k4RP = 42;                          // patch row pitch (16-B slots)
constexpr int k4PUsed = k4PR * k4RP;              // 756
constexpr int k4PSlots = 768;                     // 12 DMA wave instructions
// per-stage LDS: U slice 36 x 4 x CO fp32 + the patch
template <int CO>
struct W4Cfg {
    static constexpr int kWaves = CO / 8;  // 2 tile groups x CO / 16 channel groups
    static constexpr int kUB = 36 * k4KC * CO * 4;       // 18 / 36 KiB
    static constexpr int kStageB = kUB + k4PSlots * 16;  // 30 / 48 KiB
};

__device__ float4 g_wino4_zero;  // the source of out-of-image patch taps

__device__ __forceinline__ void w4_dma_1k(const float *src, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds))
        : "memory");
}

__device__ __forceinline__ void w4_wait_barrier() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// y = B^T x, B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0;
//                   0 2 -1 -2 1 0; 0 4 0 -5 0 1]
__device__ __forceinline__ void bt6(const float x[6], float y[6]) {
    const float t0 = __builtin_fmaf(-4.f, x[2], x[4]), t1 = __builtin_fmaf(-4.f, x[1], x[3]);
    const float t2 = x[4] - x[2], t3 = 2.f * (x[3] - x[1]);
    y[0] = __builtin_fmaf(4.f, x[0], __builtin_fmaf(-5.f, x[2], x[4]));
    y[1] = t0 + t1;
    y[2] = t0 - t1;
    y[3] = t2 + t3;
    y[4] = t2 - t3;
    y[5] = __builtin_fmaf(4.f, x[1], __builtin_fmaf(-5.f, x[3], x[5]));
}

// y = A^T m, A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
__device__ __forceinline__ void at6(const float m[6], float y[4]) {
    const float s12 = m[1] + m[2], d12 = m[1] - m[2], s34 = m[3] + m[4], d34 = m[3] - m[4];
    y[0] = m[0] + s12 + s34;
    y[1] = __builtin_fmaf(2.f, d34, d12);
    y[2] = __builtin_fmaf(4.f, s34, s12);
    y[3] = __builtin_fmaf(8.f, d34, d12) + m[5];
}

template <bool RELU, int CO>
__global__ __launch_bounds__(CO * 8, CO == 32 ? 2 : 1) void conv3x3_wino4_kernel(
    const float *__restrict__ X, int N, int H, int W, int C, const float *__restrict__ U,
    int Cout, const float *__restrict__ bias, float *__restrict__ Y, int tby, int tbx) {
    constexpr int k4Co = CO, NW = W4Cfg<CO>::kWaves, k4UB = W4Cfg<CO>::kUB;
    constexpr int k4StageB = W4Cfg<CO>::kStageB;
    __shared__ __attribute__((aligned(16))) float sm[2 * k4StageB / 4];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 15, q = lane >> 4;
    // the Cout / 32 channel blocks of one spatial block run on one XCD (blocks
    // b, b + 8, ...): its input patches come from one L2
    const int ncb = Cout / k4Co;
    const int r8 = blockIdx.x % (8 * ncb);
    const int cb = r8 / 8;
    const int sp = (blockIdx.x / (8 * ncb)) * 8 + (r8 & 7);
    if (sp >= N * tby * tbx) return;
    const int n = sp / (tby * tbx);
    const int rem = sp - n * tby * tbx;
    const int tyb = rem / tbx, txb = rem - (rem / tbx) * tbx;
    const int oy0 = 4 * k4TR * tyb, ox0 = 4 * k4TC * txb;
    const int iy0 = oy0 - 1, ix0 = ox0 - 1;
    const int n0 = cb * k4Co;
    const int tg = wave & 1, cg = wave >> 1;
    const uint32_t sbase = (uint32_t)(uintptr_t)sm;
    const int nch = C / k4KC;

    // U DMA: chunk slice = CO x 576 contiguous bytes, instruction i by wave i % NW
    const float *usrc = U + (int64_t)cb * nch * (k4UB / 4) + lane * 4;
    // patch DMA: 12 instructions, wave w takes w, w + NW, ...; slots outside the
    // patch (row padding, the column skew's gaps) or the image copy zeros
    constexpr int NP = (12 + NW - 1) / NW;
    const float *psrc[NP];
    bool pok[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const int s = 64 * (wave + NW * k) + lane;
        const int r = s / k4RP, t = s - (s / k4RP) * k4RP;
        const int c = t - t / 5;  // inverse of c + c / 4
        const int y = iy0 + r, x = ix0 + c;
        pok[k] = wave + NW * k < 12 && s < k4PUsed && t % 5 != 4 && c < k4PC && (unsigned)y < (unsigned)H &&
                 (unsigned)x < (unsigned)W;
        psrc[k] = pok[k] ? X + (((int64_t)n * H + y) * W + x) * C : X;
    }
    const float *zero = reinterpret_cast<const float *>(&g_wino4_zero);
#define VD_W4_DMA(CH, ST)                                                                    \
    {                                                                                        \
        const uint32_t d_ = sbase + (uint32_t)(ST) * k4StageB;                               \
        const float *u_ = usrc + (int64_t)(CH) * (k4UB / 4);                                 \
        for (int i = wave; i < k4UB / 1024; i += NW)                                         \
            w4_dma_1k(u_ + i * 256, d_ + (uint32_t)i * 1024u);                               \
        _Pragma("unroll") for (int k = 0; k < NP; ++k) if (wave + NW * k < 12)               \
            w4_dma_1k(pok[k] ? psrc[k] + (CH) * k4KC : zero,                                 \
                      d_ + (uint32_t)k4UB + (uint32_t)(wave + NW * k) * 1024u);              \
    }
    // transform reads: lane (j, q) -> tile 16 tg + j (tile row tr, col tc), channel q;
    // pixel (4 tr + a, 4 tc + b) at slot (4 tr + a) * 42 + 5 tc + b + b / 4
    const int vt = tg * 16 + j, tr = vt / k4TC, tc = vt % k4TC;
    int roff[6], coff[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        roff[a] = 16 * (4 * tr + a) * k4RP;
        coff[a] = 16 * (5 * tc + a + (a >> 2)) + 4 * q + k4UB;
    }
    // U fragments: 16-B unit ((p4 * 4 + q) * 32 + 16 cg + j) holds positions
    // 4 p4 .. + 3 of U[.][co = 16 cg + j][ci = q]
    const int ufo = ((q * k4Co) + 16 * cg + j) * 16;
    f4v acc[36];
#pragma unroll
    for (int p = 0; p < 36; ++p) acc[p] = f4v{0.f, 0.f, 0.f, 0.f};

    VD_W4_DMA(0, 0)
    w4_wait_barrier();
    for (int ch = 0; ch < nch; ++ch) {
        const int s = ch & 1;
        if (ch + 1 < nch) VD_W4_DMA(ch + 1, s ^ 1)
        const char *stb = reinterpret_cast<const char *>(sm) + s * k4StageB;
        // V = B^T d B for the lane's tile and channel
        float v[36];
        {
            float d[6][6];
#pragma unroll
            for (int a = 0; a < 6; ++a)
#pragma unroll
                for (int b = 0; b < 6; ++b)
                    d[a][b] = *reinterpret_cast<const float *>(stb + roff[a] + coff[b]);
            float e[6][6];
#pragma unroll
            for (int b = 0; b < 6; ++b) {
                float x[6], y[6];
#pragma unroll
                for (int a = 0; a < 6; ++a) x[a] = d[a][b];
                bt6(x, y);
#pragma unroll
                for (int a = 0; a < 6; ++a) e[a][b] = y[a];
            }
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                float y[6];
                bt6(e[a], y);
#pragma unroll
                for (int b = 0; b < 6; ++b) v[6 * a + b] = y[b];
            }
        }
#pragma unroll
        for (int p4 = 0; p4 < 9; ++p4) {
            const f4v ua = *reinterpret_cast<const f4v *>(stb + p4 * (k4KC * CO * 16) + ufo);
#pragma unroll
            for (int e = 0; e < 4; ++e)
                acc[4 * p4 + e] =
                    __builtin_amdgcn_mfma_f32_16x16x4f32(ua[e], v[4 * p4 + e], acc[4 * p4 + e], 0, 0, 0);
        }
        w4_wait_barrier();  // DMA of chunk ch + 1 landed; stage s read
    }
#undef VD_W4_DMA
    // output transform (lane-local): accumulator slot r holds channel
    // n0 + 16 cg + 4 q + r of tile 16 tg + j
    const int co = n0 + 16 * cg + 4 * q;
    const float4 bv = bias ? *reinterpret_cast<const float4 *>(bias + co)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
    float o[4][16];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float z[4][6];
#pragma unroll
        for (int b = 0; b < 6; ++b) {
            float m[6], y[4];
#pragma unroll
            for (int a = 0; a < 6; ++a) m[a] = acc[6 * a + b][r];
            at6(m, y);
#pragma unroll
            for (int k = 0; k < 4; ++k) z[k][b] = y[k];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float y[4];
            at6(z[k], y);
#pragma unroll
            for (int l = 0; l < 4; ++l) o[r][4 * k + l] = y[l];
        }
    }
    const int oy = oy0 + 4 * tr, ox = ox0 + 4 * tc;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int y = oy + (k >> 2), x = ox + (k & 3);
        if (y >= H || x >= W) continue;
        float4 val = make_float4(o[0][k] + bv.x, o[1][k] + bv.y, o[2][k] + bv.z, o[3][k] + bv.w);
        if (RELU) {
            val.x = fmaxf(val.x, 0.f);
            val.y = fmaxf(val.y, 0.f);
            val.z = fmaxf(val.z, 0.f);
            val.w = fmaxf(val.w, 0.f);
        }
        *reinterpret_cast<float4 *>(Y + ((int64_t)(n * H + y) * W + x) * Cout + co) = val;
    }
}

// U = G g G^T of the PyTorch weight w[co][ci][3][3] (G 6 x 3: rows [1/4 0 0],
// [-1/6 -1/6 -1/6], [-1/6 1/6 -1/6], [1/24 1/12 1/6], [1/24 -1/12 1/6],
// [0 0 1]), float64, rounded once; stored chunk-blocked as
// [co / 32][ci / 4][pos / 4][ci % 4][co % 32][pos % 4].
template <int k4Co>
__global__ void wino4_weight_kernel(const float *__restrict__ w, int Cout, int C,
                                    float *__restrict__ U) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)Cout * C) return;
    const int co = (int)(i / C), ci = (int)(i - (int64_t)(i / C) * C);
    const double G[6][3] = {{0.25, 0, 0},
                            {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                            {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                            {1.0 / 24, 1.0 / 12, 1.0 / 6},
                            {1.0 / 24, -1.0 / 12, 1.0 / 6},
                            {0, 0, 1}};
    const float *g = w + i * 9;
    double t[6][3];  // G g
    for (int a = 0; a < 6; ++a)
        for (int c = 0; c < 3; ++c)
            t[a][c] = G[a][0] * g[c] + G[a][1] * g[3 + c] + G[a][2] * g[6 + c];
    float *dst = U + (((int64_t)(co / k4Co) * (C / k4KC) + ci / k4KC) * 9) * (k4KC * k4Co * 4) +
                 ((ci % k4KC) * k4Co + co % k4Co) * 4;
    for (int a = 0; a < 6; ++a)
        for (int b = 0; b < 6; ++b) {
            const double u = t[a][0] * G[b][0] + t[a][1] * G[b][1] + t[a][2] * G[b][2];
            const int p = 6 * a + b;
            dst[(p >> 2) * (k4KC * k4Co * 4) + (p & 3)] = (float)u;
        }
}

}  // namespace

// Channel block of the kernel (the weight layout depends on it): 32 (4 waves, two
// workgroups per CU).  The 64-channel form (8 waves, one per CU; half the U
// traffic per output) measured slower on every step shape: P2 5.69 vs 4.99 ms
// (profiles/r03/wino4_probe.json).
static int w4_co(int) { return 32; }

bool conv3x3_wino4_supported(int C, int Cout) {
    return C % k4KC == 0 && C >= k4KC && Cout % 32 == 0 && Cout >= 32;
}

int launch_conv3x3_wino4_weight(const float *w, int Cout, int C, float *U, hipStream_t s) {
    const int64_t n = (int64_t)Cout * C;
    if (n == 0) return VD_OK;
    if (!conv3x3_wino4_supported(C, Cout)) return VD_ERR_SHAPE;
    hipLaunchKernelGGL(w4_co(Cout) == 64 ? wino4_weight_kernel<64> : wino4_weight_kernel<32>,
                       dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, Cout, C, U);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int launch_conv3x3_wino4(const float *X, int N, int H, int W, int C, const float *U, int Cout,
                         const float *bias, int relu, float *Y, hipStream_t s) {
    if ((int64_t)N * H * W == 0) return VD_OK;
    if (!conv3x3_wino4_supported(C, Cout)) return VD_ERR_SHAPE;
    const int tby = (H + 4 * k4TR - 1) / (4 * k4TR), tbx = (W + 4 * k4TC - 1) / (4 * k4TC);
    const int64_t nsp = (int64_t)N * tby * tbx;
    const int co = w4_co(Cout);
    const int64_t blocks = (nsp + 7) / 8 * 8 * (Cout / co);
    if (blocks > 0x7fffffff) return VD_ERR_SHAPE;
    auto kern = co == 64 ? (relu ? conv3x3_wino4_kernel<true, 64> : conv3x3_wino4_kernel<false, 64>)
                         : (relu ? conv3x3_wino4_kernel<true, 32> : conv3x3_wino4_kernel<false, 32>);
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(co * 8), 0, s, X, N, H, W, C, U, Cout,
                       bias, Y, tby, tbx);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
