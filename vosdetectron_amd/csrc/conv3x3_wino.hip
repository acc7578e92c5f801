// 3x3 stride-1 pad-1 convolution on NHWC fp32 by Winograd F(2x2, 3x3) on the
// MFMA pipes, bias (+ ReLU) epilogue fused.
//
// Same operator as conv3x3.hip (FPN posthoc / RPN conv, lib/modeling/FPN.py:
// 227-258, 376-422; mask head convs, mask_rcnn_heads.py:178-188), computed with
// 2.25x fewer multiplies (Lavin & Gray, "Fast Algorithms for Convolutional Neural
// Networks"): every 2x2 output tile is
//   Y = A^T [ sum_ci (G g G^T) (.) (B^T d B) ] A
// with d the tile's 4x4 input patch.  The sum over ci is 16 independent GEMMs,
// M[pos][co][tile] = sum_ci U[pos][co][ci] V[pos][ci][tile] (pos = the 16
// transform positions), run with v_mfma_f32_16x16x4_f32 (fp32 in, fp32 out: the
// reference's precision; the transforms only add / subtract and scale by 0.5).
//
// Workgroup (8 waves, one per CU: 150 KiB of LDS): 64 tiles (4 tile rows x 16
// tile columns = 8 x 32 output pixels of one image) x 64 output channels.
// Wave w owns tile row w & 3 and 32 channels (w >> 2), i.e. ALL 16 positions of
// its 16 tiles x 32 channels: 128 accumulator registers per lane, and a lane's
// 16 position values of one (channel, tile) sit in the same register slot of its
// 16 accumulators, so the output transform is lane-local.
// K is walked in chunks of 8 input channels; per chunk the raw 10 x 34 pixel
// patch and U's slice are staged in LDS, every thread transforms one (tile,
// channel) of the NEXT chunk's patch into V while the MFMAs of this chunk run,
// and the loads of the chunks after that are in flight: two LDS stages, one
// barrier per chunk.  K permutation (both operands): lane group q at k-step s
// holds channel 2q + s, so each fragment is one ds_read_b64.
#include <stdlib.h>

#include <mutex>
#include <set>

#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int kTiles = 64;                 // tiles per workgroup: TR x TC (4 x 16 or 8 x 8)
constexpr int kCo = 64;                    // output channels per workgroup
constexpr int kKC = 8;                     // input channels per chunk
constexpr int kPatchMaxF4 = 680;           // the larger patch (10 x 34 pixels x 8 channels)
constexpr int kVsF = 16 * kTiles * kKC;    // 8192 floats: V [pos][tile][8]
constexpr int kUsF = 16 * kCo * kKC;       // 8192 floats: U [pos][co][8]
// patch pixels are kPixF floats apart (8 channels + 4 pad): the transform's
// ds_read_b32 lanes (4 tiles, 2 pixels apart, x 8 channels per 32-lane group)
// then fall on 32 distinct banks (a stride of 8 would be 2-way)
constexpr int kPixF = 12;
constexpr int kPatchF = kPatchMaxF4 / 2 * kPixF + 4;  // patch [row][col][12] + a pad
constexpr int kStageF = kVsF + kUsF + kPatchF;
constexpr size_t kLdsBytes = 2 * (size_t)kStageF * 4;  // 163,744 B
constexpr int kThreads = 512;

// Row-half swizzle of the [.][8] rows: rows r and r + 8 of a 16-row MFMA block
// put their two float4 halves in opposite order, so a ds_read_b64 fragment read
// (lanes j = 0..15 x q = 0..1 per 32-lane group) touches 32 distinct banks.
__device__ __forceinline__ int sw_half(int row) { return (row >> 3) & 1; }

// TC tile columns x (64 / TC) tile rows per workgroup: 16 (8 x 32 output pixels)
// for feature maps, 8 (16 x 16 pixels: one 14 x 14 mask-head RoI) for small ones.
// Schedule variants (VOSDET_WINO_VARIANT, A/B in one process): bit 0 = two
// barriers per chunk (stores of chunk + 2 between them) instead of one; bit 1 =
// opaque position stride (plain ds_read_b64 fragment reads, no read2 pairing);
// bit 2 = sched_group_barrier interleave of transform / staging with the MFMAs;
// bit 3 = four positions per MFMA group instead of two.
template <bool RELU, int TC, int V>
__global__ __launch_bounds__(kThreads, 1) void conv3x3_wino_kernel(
    const float *__restrict__ X, int N, int H, int W, int C, const float *__restrict__ U,
    int Cout, const float *__restrict__ bias, float *__restrict__ Y, int tby, int tbx) {
    constexpr int kTC = TC, kTR = kTiles / TC;
    constexpr int kPR = 2 * kTR + 2, kPC = 2 * kTC + 2;  // input patch (pixels)
    constexpr int kPatchF4 = kPR * kPC * kKC / 4;
    static_assert(kPatchF4 <= kPatchMaxF4, "patch fits its LDS region");
    extern __shared__ __attribute__((aligned(16))) float lds[];  // [2][kStageF]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 15, q = lane >> 4;
    // the Cout / 64 channel blocks of one spatial block run on one XCD (blocks
    // b, b + 8, ...): its input patches come from one L2
    const int ncb = Cout / kCo;
    const int r8 = blockIdx.x % (8 * ncb);
    const int cb = r8 / 8;
    const int sp = (blockIdx.x / (8 * ncb)) * 8 + (r8 & 7);
    const int nsp = N * tby * tbx;
    if (sp >= nsp) return;
    const int n = sp / (tby * tbx);
    const int rem = sp - n * tby * tbx;
    const int tyb = rem / tbx, txb = rem - (rem / tbx) * tbx;
    const int oy0 = 2 * kTR * tyb, ox0 = 2 * kTC * txb;  // first output pixel
    const int iy0 = oy0 - 1, ix0 = ox0 - 1;              // first patch pixel
    const int n0 = cb * kCo;
    const int tg = wave & 3, cg = wave >> 2;  // wave: tiles 16 tg .. + 15, 32-channel group

    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(X), (short)0, (int)((int64_t)N * H * W * C * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(U), (short)0, (int)((int64_t)16 * Cout * C * 4), 0x00020000);

    // staging assignment: patch float4 f = tid + 512 i (i < 2, f < 680);
    // U float4 f = tid + 512 i (i < 4): row f >> 1 = (pos, co), half f & 1
    int poff[2], uoff[4], pdst[2], udst[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int f = tid + kThreads * i;
        const int px = f >> 1, h = f & 1;
        const int prow = px / kPC, pcol = px - (px / kPC) * kPC;
        const int y = iy0 + prow, x = ix0 + pcol;
        const bool ok = f < kPatchF4 && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
        // out-of-image taps read past the buffer's range: zeros
        poff[i] = ok ? (((n * H + y) * W + x) * C + 4 * h) * 4 : 0x7ffffff0;
        // lanes past the patch store into the region's pad (no branch)
        pdst[i] = kVsF + kUsF + (f < kPatchF4 ? px * kPixF + 4 * h : kPatchF - 4);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int f = tid + kThreads * i;
        const int row = f >> 1, h = f & 1;
        const int pos = row >> 6, co = row & 63;
        uoff[i] = ((pos * Cout + n0 + co) * C + 4 * h) * 4;
        udst[i] = kVsF + row * kKC + 4 * (h ^ sw_half(co));
    }
    float4 pr[2], urg[4];
#define VD_W_LOADP(CH)                                                                       \
    {                                                                                        \
        const int cb4_ = (CH) * kKC * 4;                                                     \
        _Pragma("unroll") for (int i = 0; i < 2; ++i) pr[i] = __builtin_bit_cast(            \
            float4, __builtin_amdgcn_raw_buffer_load_b128(                                   \
                        xr, poff[i] == 0x7ffffff0 ? poff[i] : poff[i] + cb4_, 0, 0));        \
    }
#define VD_W_LOADU(CH)                                                                       \
    {                                                                                        \
        const int cb4_ = (CH) * kKC * 4;                                                     \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) urg[i] = __builtin_bit_cast(           \
            float4, __builtin_amdgcn_raw_buffer_load_b128(ur, uoff[i] + cb4_, 0, 0));        \
    }
#define VD_W_STOREP(STG)                                                                     \
    {                                                                                        \
        float *s_ = lds + (STG) * kStageF;                                                   \
        _Pragma("unroll") for (int i = 0; i < 2; ++i)                                        \
            *reinterpret_cast<float4 *>(s_ + pdst[i]) = pr[i];                               \
    }
#define VD_W_STOREU(STG)                                                                     \
    {                                                                                        \
        float *s_ = lds + (STG) * kStageF;                                                   \
        _Pragma("unroll") for (int i = 0; i < 4; ++i)                                        \
            *reinterpret_cast<float4 *>(s_ + udst[i]) = urg[i];                              \
    }
    // input transform of one (tile, channel) of stage STG's patch into its V:
    // V = B^T d B, B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]
    const int xt = tid >> 3, xc = tid & 7;  // tile, channel
    const int xtr = xt / kTC, xtc = xt % kTC;
    const int vdst = xt * kKC + 4 * ((xc >> 2) ^ sw_half(xt)) + (xc & 3);
#define VD_W_XFORM(STG)                                                                      \
    {                                                                                        \
        const float *p_ = lds + (STG) * kStageF + kVsF + kUsF;                               \
        float d_[4][4];                                                                      \
        _Pragma("unroll") for (int a = 0; a < 4; ++a)                                        \
            _Pragma("unroll") for (int c = 0; c < 4; ++c)                                    \
                d_[a][c] = p_[((2 * xtr + a) * kPC + 2 * xtc + c) * kPixF + xc];               \
        float r_[4][4];                                                                      \
        _Pragma("unroll") for (int c = 0; c < 4; ++c) {                                      \
            r_[0][c] = d_[0][c] - d_[2][c];                                                  \
            r_[1][c] = d_[1][c] + d_[2][c];                                                  \
            r_[2][c] = d_[2][c] - d_[1][c];                                                  \
            r_[3][c] = d_[1][c] - d_[3][c];                                                  \
        }                                                                                    \
        float *v_ = lds + (STG) * kStageF + vdst;                                            \
        _Pragma("unroll") for (int a = 0; a < 4; ++a) {                                      \
            v_[(4 * a + 0) * kTiles * kKC] = r_[a][0] - r_[a][2];                            \
            v_[(4 * a + 1) * kTiles * kKC] = r_[a][1] + r_[a][2];                            \
            v_[(4 * a + 2) * kTiles * kKC] = r_[a][2] - r_[a][1];                            \
            v_[(4 * a + 3) * kTiles * kKC] = r_[a][1] - r_[a][3];                            \
        }                                                                                    \
    }
    // fragment offsets (floats within a stage): V of tile tg*16 + j, U of channel
    // cg*32 + 16 tc + j; channels 2q, 2q + 1 of the chunk
    const int vt = tg * 16 + j;
    const int vfo = vt * kKC + 4 * ((q >> 1) ^ sw_half(vt)) + 2 * (q & 1);
    int ufo[2];
#pragma unroll
    for (int tc = 0; tc < 2; ++tc) {
        const int co = cg * 32 + 16 * tc + j;
        ufo[tc] = kVsF + co * kKC + 4 * ((q >> 1) ^ sw_half(co)) + 2 * (q & 1);
    }
    f4v acc[16][2];
#pragma unroll
    for (int p = 0; p < 16; ++p)
#pragma unroll
        for (int tc = 0; tc < 2; ++tc) acc[p][tc] = f4v{0.f, 0.f, 0.f, 0.f};

    const int nch = C / kKC;
    // Before phase ch: V(ch), U(ch) in stage ch & 1, patch(ch + 1) in stage
    // (ch + 1) & 1.  Phase ch reads V / U of stage s = ch & 1 and the patch of
    // stage s ^ 1, and writes V and U of stage s ^ 1 (V(ch + 1), U(ch + 1)) and
    // the patch of stage s (patch(ch + 2)): nothing it writes is read in the
    // phase, so one barrier per chunk.  Loads / stores past the last chunk
    // re-stage it harmlessly, keeping the body branch-free (one basic block,
    // so the transform and the staging interleave with the MFMAs).
    constexpr bool kTwoBar = V & 1, kOpaque = V & 2, kInterleave = V & 4;
    constexpr int kPG = (V & 8) ? 4 : 2;  // positions per MFMA group
    if (kTwoBar) {
        // before phase ch: V(ch), U(ch), patch(ch + 1) staged; phase ch: MFMA(ch),
        // transform patch(ch + 1), barrier, store U / patch of chunk ch + 2, barrier
        VD_W_LOADP(0)
        VD_W_LOADU(0)
        VD_W_STOREP(0)
        VD_W_STOREU(0)
        __syncthreads();
        VD_W_XFORM(0)
        VD_W_LOADP(nch > 1 ? 1 : 0)
        VD_W_LOADU(nch > 1 ? 1 : 0)
        VD_W_STOREP(1)
        VD_W_STOREU(1)
        __syncthreads();
    } else {
        VD_W_LOADP(0)
        VD_W_LOADU(0)
        VD_W_STOREP(0)
        VD_W_STOREU(0)
        __syncthreads();
        VD_W_XFORM(0)
        VD_W_LOADP(nch > 1 ? 1 : 0)
        VD_W_STOREP(1)
        __syncthreads();
    }
    for (int ch = 0; ch < nch; ++ch) {
        const int s = ch & 1;
        const int c1 = ch + 1 < nch ? ch + 1 : nch - 1, c2 = ch + 2 < nch ? ch + 2 : nch - 1;
        if (kTwoBar) {
            VD_W_LOADU(c2)
        } else {
            VD_W_LOADU(c1)
        }
        VD_W_LOADP(c2)
        const float *st = lds + s * kStageF;
        // with kOpaque, an opaque position stride: hipcc would otherwise pair the
        // fragment reads of two positions into ds_read2st64_b64, whose 16-lane /
        // 32-bank groups are 2-way conflicted on this layout (ds_read_b64 is not)
        int vps = kTiles * kKC, ups = kCo * kKC;
        if (kOpaque) asm volatile("" : "+v"(vps), "+v"(ups));
        // kPG positions at a time: 2 kPG independent MFMAs between the two k-steps
        // of one accumulator (dependent latency 40 cycles)
#pragma unroll
        for (int p0 = 0; p0 < 16; p0 += kPG) {
            f2v b[kPG], a[kPG][2];
#pragma unroll
            for (int i = 0; i < kPG; ++i) {
                const int vo = (p0 + i) * vps + vfo, uo = (p0 + i) * ups;  // 32-bit LDS offsets
                b[i] = *reinterpret_cast<const f2v *>(st + vo);
                a[i][0] = *reinterpret_cast<const f2v *>(st + uo + ufo[0]);
                a[i][1] = *reinterpret_cast<const f2v *>(st + uo + ufo[1]);
            }
#pragma unroll
            for (int i = 0; i < kPG; ++i)
#pragma unroll
                for (int tc = 0; tc < 2; ++tc)
                    acc[p0 + i][tc] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                        a[i][tc].x, b[i].x, acc[p0 + i][tc], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < kPG; ++i)
#pragma unroll
                for (int tc = 0; tc < 2; ++tc)
                    acc[p0 + i][tc] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                        a[i][tc].y, b[i].y, acc[p0 + i][tc], 0, 0, 0);
        }
        VD_W_XFORM(s ^ 1)  // patch(ch + 1) -> V(ch + 1)
        if (kTwoBar) {
            __syncthreads();    // stage s fully read; V(ch + 1) written
            VD_W_STOREU(s)      // U(ch + 2)
            VD_W_STOREP(s)      // patch(ch + 2)
        } else {
            VD_W_STOREU(s ^ 1)  // U(ch + 1)
            VD_W_STOREP(s)      // patch(ch + 2)
        }
        if (kInterleave) {
            // transform / staging instructions into the issue shadows of the
            // MFMAs (32 cycles each on the SIMD) instead of after them
#pragma unroll
            for (int k = 0; k < 40; ++k) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 LDS read
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // 1 VALU
                __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // 1 LDS write
            }
        }
        __syncthreads();
    }
#undef VD_W_LOADP
#undef VD_W_LOADU
#undef VD_W_STOREP
#undef VD_W_STOREU
#undef VD_W_XFORM
    // output transform (lane-local): A^T = [1 1 1 0; 0 1 -1 -1]; lane (j, q),
    // accumulator slot r holds channel n0 + cg*32 + 16 tc + 4 q + r of tile (tg, j)
    const int vtile = tg * 16 + j;
    const int oy = oy0 + 2 * (vtile / kTC), ox = ox0 + 2 * (vtile % kTC);
#pragma unroll
    for (int tc = 0; tc < 2; ++tc) {
        const int co = n0 + cg * 32 + 16 * tc + 4 * q;
        const float4 bv = bias ? *reinterpret_cast<const float4 *>(bias + co)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
        float o[4][4];  // [output pixel dy*2+dx][slot r]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float s0[4], s1[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                s0[c] = acc[c][tc][r] + acc[4 + c][tc][r] + acc[8 + c][tc][r];
                s1[c] = acc[4 + c][tc][r] - acc[8 + c][tc][r] - acc[12 + c][tc][r];
            }
            o[0][r] = s0[0] + s0[1] + s0[2];
            o[1][r] = s0[1] - s0[2] - s0[3];
            o[2][r] = s1[0] + s1[1] + s1[2];
            o[3][r] = s1[1] - s1[2] - s1[3];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int y = oy + (k >> 1), x = ox + (k & 1);
            if (y >= H || x >= W) continue;
            float4 v = make_float4(o[k][0] + bv.x, o[k][1] + bv.y, o[k][2] + bv.z,
                                   o[k][3] + bv.w);
            if (RELU) {
                v.x = fmaxf(v.x, 0.f);
                v.y = fmaxf(v.y, 0.f);
                v.z = fmaxf(v.z, 0.f);
                v.w = fmaxf(v.w, 0.f);
            }
            *reinterpret_cast<float4 *>(Y + ((int64_t)(n * H + y) * W + x) * Cout + co) = v;
        }
    }
}

// U[pos][co][ci] = (G g G^T)[pos / 4][pos % 4] of the PyTorch weight
// w[co][ci][3][3]; G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]; float64, rounded once.
__global__ void wino_weight_kernel(const float *__restrict__ w, int Cout, int C,
                                   float *__restrict__ U) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)Cout * C) return;
    const int co = (int)(i / C), ci = (int)(i - (int64_t)(i / C) * C);
    const float *g = w + i * 9;
    double t[4][3];  // G g
    for (int c = 0; c < 3; ++c) {
        const double g0 = g[c], g1 = g[3 + c], g2 = g[6 + c];
        t[0][c] = g0;
        t[1][c] = 0.5 * (g0 + g1 + g2);
        t[2][c] = 0.5 * (g0 - g1 + g2);
        t[3][c] = g2;
    }
    for (int a = 0; a < 4; ++a) {
        const double u[4] = {t[a][0], 0.5 * (t[a][0] + t[a][1] + t[a][2]),
                             0.5 * (t[a][0] - t[a][1] + t[a][2]), t[a][2]};
        for (int b = 0; b < 4; ++b)
            U[((int64_t)(4 * a + b) * Cout + co) * C + ci] = (float)u[b];
    }
}

bool allow_lds_wino(const void *kern) {  // > 64 KiB of dynamic LDS, once per kernel
    static std::mutex mu;
    static std::set<const void *> done;
    std::lock_guard<std::mutex> lk(mu);
    if (done.count(kern)) return true;
    if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes) !=
        hipSuccess)
        return false;
    done.insert(kern);
    return true;
}

}  // namespace

bool conv3x3_wino_supported(int C, int Cout) {
    return C % kKC == 0 && C >= kKC && Cout % kCo == 0 && Cout >= kCo;
}

int launch_conv3x3_wino_weight(const float *w, int Cout, int C, float *U, hipStream_t s) {
    const int64_t n = (int64_t)Cout * C;
    if (n == 0) return VD_OK;
    hipLaunchKernelGGL(wino_weight_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w,
                       Cout, C, U);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

typedef void (*wino_kern_t)(const float *, int, int, int, int, const float *, int,
                            const float *, float *, int, int);

template <int V>
wino_kern_t pick_v(bool relu, bool sq) {
    return sq ? (relu ? conv3x3_wino_kernel<true, 8, V> : conv3x3_wino_kernel<false, 8, V>)
              : (relu ? conv3x3_wino_kernel<true, 16, V> : conv3x3_wino_kernel<false, 16, V>);
}

wino_kern_t pick_kernel(bool relu, bool sq, int v) {
    switch (v) {
        case 0: return pick_v<0>(relu, sq);   // one barrier, read2 pairs, 2-pos groups
        case 1: return pick_v<1>(relu, sq);   // two barriers
        case 6: return pick_v<6>(relu, sq);   // one barrier, plain b64 reads, interleave
        case 8: return pick_v<8>(relu, sq);   // one barrier, 4-pos groups
        case 9: return pick_v<9>(relu, sq);   // two barriers, 4-pos groups (round-3 first form)
        case 11: return pick_v<11>(relu, sq); // two barriers, plain b64, 4-pos groups
        case 13: return pick_v<13>(relu, sq); // two barriers, interleave, 4-pos groups
        default: return nullptr;
    }
}

constexpr int kDefaultVariant = 0;

int launch_conv3x3_wino(const float *X, int N, int H, int W, int C, const float *U, int Cout,
                        const float *bias, int relu, float *Y, hipStream_t s) {
    if ((int64_t)N * H * W == 0) return VD_OK;
    if (!conv3x3_wino_supported(C, Cout)) return VD_ERR_SHAPE;
    if ((int64_t)N * H * W * C * 4 >= 0x7ffffff0ll || (int64_t)16 * Cout * C * 4 >= 0x7ffffff0ll)
        return VD_ERR_SHAPE;  // 32-bit buffer offsets
    const bool sq = W <= 16;  // small maps (the 14 x 14 mask-head RoIs): 16 x 16-pixel blocks
    const int tby = sq ? (H + 15) / 16 : (H + 7) / 8;  // else 8 x 32-pixel blocks
    const int tbx = sq ? (W + 15) / 16 : (W + 31) / 32;
    const int64_t nsp = (int64_t)N * tby * tbx;
    const int64_t blocks = (nsp + 7) / 8 * 8 * (Cout / kCo);
    if (blocks > 0x7fffffff) return VD_ERR_SHAPE;
    // schedule variant (see the kernel): default 0 = one barrier per chunk, read2
    // fragment pairs, two positions per MFMA group -- best or tied-best on all four
    // benched shapes in one-process A/B (tools/probe_wino_variants.py)
    const char *ev = getenv("VOSDET_WINO_VARIANT");
    const int v = ev ? atoi(ev) : kDefaultVariant;
    auto kern = pick_kernel(relu != 0, sq, v);
    if (!kern) return VD_ERR_ARG;
    if (!allow_lds_wino(reinterpret_cast<const void *>(kern))) return VD_ERR_LAUNCH;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kThreads), kLdsBytes, s, X, N, H, W, C,
                       U, Cout, bias, Y, tby, tbx);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
