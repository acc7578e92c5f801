// fp32 GEMMs of the 1x1 convolutions and fully connected layers on the bf16
// matrix cores, at fp32 accuracy, with the conv epilogue fused:
//
//   D[M][N] = act(A[M][K] . W[N][K]^T + bias[N] (+ R[M][N]))      (fp32 in / out)
//
// gfx950 has no xf32 MFMA: fp32 operands run on v_mfma_f32_*_f32 at the fp32
// VALU rate (157 TF/s), 1/16 of the bf16 MFMA rate.  Every fp32 operand here is
// split EXACTLY-ish into three bf16 pieces x = x0 + x1 + x2 (x0 = bf16(x),
// x1 = bf16(x - x0), x2 = bf16(x - x0 - x1), round-to-nearest: |x - x0 - x1 - x2|
// <= 2^-24 |x|, i.e. the three pieces carry fp32's 24-bit significand), and the
// product is the six largest of the nine piece products
//
//   a.b ~= a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0)
//
// (the three dropped ones are <= 2^-24 |a b| together), accumulated in fp32 by
// v_mfma_f32_32x32x16_bf16 (every bf16 x bf16 product is exact in fp32).
// Six bf16 MFMAs cost 6/16 of one fp32 MFMA of the same shape: the error stays
// at fp32's level (tests/test_gemm_split3_gpu.py measures it against fp64 next
// to torch's own fp32 GEMM) while the matrix-core time drops 2.67x.  This is
// the bf16x6 scheme of Henry, Tang & Heinecke, "Leveraging the bfloat16
// Artificial Intelligence Datatype For Higher-Precision Computations" (ARITH
// 2019), whose bf16x6 matched fp32 SGEMM accuracy.
//
// Reference: the convolutions and fc layers of lib/modeling/ResNet.py:246-294
// (bottleneck 1x1s + AffineChannel + residual + ReLU), fast_rcnn_heads.py
// roi_2mlp_head fc6/fc7, mask_rcnn_heads.py upconv5, FPN.py laterals -- fp32
// PyTorch convs / Linear layers there.
//
// Mapping (v_mfma_f32_32x32x16_bf16; lane l = (h = l >> 5, r = l & 31) holds
// A-operand row r / B-operand column r, k = 8 h .. 8 h + 7 of a 16-deep step):
// the MFMA's A operand is the weight tile (row = output channel), its B operand
// the pixel tile (column = pixel), so a lane's accumulator registers 4g..4g+3
// are output channels 8 g + 4 h .. + 3 of one pixel: bias, residual and the
// store are float4s.  Both operands sit in LDS as lane-linear 1 KiB fragments
// ([piece][tile][kstep][lane][8 bf16]): every fragment read is one ds_read_b128
// at lane * 16 B.  The weights are split once (vd_gemm_split3_weight) into that
// exact image per 32-deep K chunk, so the weight fill is a straight copy; the
// activations are split while they are written to LDS.
//
// Workgroup: 8 waves, BM pixels x BN channels, each wave (BM / WM) x (BN / WN)
// as TPM x TPN 32 x 32 tiles.  K walks in 32-deep chunks through two LDS
// buffers: chunk c + 2's global loads are in registers while chunk c computes,
// and chunk c + 1 (loaded one iteration earlier) is split into the other buffer
// after chunk c's MFMAs, one barrier per chunk.
#include <stdlib.h>

#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int kStep = 16;           // fp32 K per pipeline stage (one MFMA k-step)
constexpr int kFragBytes = 1024;    // one lane-linear 32 x 16 bf16 fragment

// Two fp32 -> three packed bf16 pairs (piece 0, 1, 2), round to nearest even.
__device__ __forceinline__ void split_pair(float x0, float x1, uint32_t &p0, uint32_t &p1,
                                           uint32_t &p2) {
    const f2v x = {x0, x1};
    const bf16x2 h = __builtin_convertvector(x, bf16x2);
    const uint32_t uh = __builtin_bit_cast(uint32_t, h);
    const f2v hf = {__uint_as_float(uh << 16), __uint_as_float(uh & 0xffff0000u)};
    const f2v r1 = x - hf;  // exact
    const bf16x2 m = __builtin_convertvector(r1, bf16x2);
    const uint32_t um = __builtin_bit_cast(uint32_t, m);
    const f2v mf = {__uint_as_float(um << 16), __uint_as_float(um & 0xffff0000u)};
    const f2v r2 = r1 - mf;  // exact
    const bf16x2 l = __builtin_convertvector(r2, bf16x2);
    p0 = uh;
    p1 = um;
    p2 = __builtin_bit_cast(uint32_t, l);
}

// W [N][K] fp32 -> Wp: [K / 16][N / 32][piece 3][lane 64][8] bf16, lane l = 32 h + r
// holding W[32 t + r][16 s + 8 h .. + 7] of k-step s, tile t.
__global__ void split3_weight_kernel(const float *__restrict__ W, int N, int K,
                                     uint4 *__restrict__ Wp) {
    const int64_t cells = (int64_t)(K / kStep) * (N / 32) * 64;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < cells;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int lane = (int)(i & 63);
        const int64_t st = i >> 6;
        const int t = (int)(st % (N / 32)), s = (int)(st / (N / 32));
        const int n = 32 * t + (lane & 31), k = kStep * s + 8 * (lane >> 5);
        const float *w = W + (int64_t)n * K + k;
        uint32_t q[3][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) split_pair(w[2 * j], w[2 * j + 1], q[0][j], q[1][j], q[2][j]);
#pragma unroll
        for (int p = 0; p < 3; ++p)
            Wp[(st * 3 + p) * 64 + lane] = make_uint4(q[p][0], q[p][1], q[p][2], q[p][3]);
    }
}

// Workgroup: 4 waves (one per SIMD), BM pixels x BN channels; wave (wm, wn) owns
// TPM x TPN 32 x 32 tiles (up to 4 x 4: 256 accumulator registers).  OCC = 2: two
// workgroups per CU (<= 256 registers a wave), so each SIMD interleaves two waves.  K walks in
// 16-deep stages through two LDS buffers; stage c + 2's global loads are issued
// into registers right after stage c + 1's registers were split into the other
// buffer, all inside stage c's MFMA stream (one basic block, so the scheduler
// interleaves them), one barrier per stage.
// RES: 0 none, 1 R[M][N] (the identity residual), 2 R = the top-down map of an FPN
// level, images x H/2 x W/2 x N, read at the nearest-2x row of pixel p (FPN.py:292-300).
// RES 3: the mask head's upconv with the class-selected 1x1 mask logits fused
// (mask_rcnn_heads.py:62-68 + the MaskRCNNOutputs classify conv at each RoI's class,
// sigmoid): BN = 256 = one (i, j) tap group of the 2x2 / 2 transposed conv, R = the
// classify weights [classes][256], cb its bias, rch each RoI's class channel, H = P
// (the RoI map side), D = masks [RoIs][2P][2P]; the relu'd upconv output never leaves
// the workgroup.
template <int BM, int BN, int TPM, int TPN, int RES, bool RELU, int PROBE = 0, int OCC = 1,
          int NW = 4, bool APRO = false>
__global__ __launch_bounds__(64 * NW, OCC) void gemm_split3_kernel(
    const float *__restrict__ A, const uint4 *__restrict__ Wp, const float *__restrict__ bias,
    const float *__restrict__ R, float *__restrict__ D, int M, int N, int K, int tiles_n,
    int num_tiles, int H, int W, int SH, int SW, const float *__restrict__ cb,
    const int32_t *__restrict__ rch, const float *__restrict__ A2, int K2,
    const float *__restrict__ abias) {
    constexpr int WM = BM / (32 * TPM), WN = BN / (32 * TPN), NTH = 64 * NW;
    static_assert(WM * WN == NW, "one (pixel, channel) block per wave");
    constexpr int PT = BM / 32, NTW = BN / 32;                 // pixel / channel tiles
    constexpr int A_BYTES = 3 * PT * kFragBytes;               // [piece][pt][lane]
    constexpr int W_BYTES = NTW * 3 * kFragBytes;              // [tw][piece][lane]
    constexpr int BUF = A_BYTES + W_BYTES;
    constexpr int AL = BM * kStep / 4 / NTH;                   // A float4 loads per thread
    constexpr int RPJ = NTH / 4;                               // A rows per load round
    constexpr int WCELLS = W_BYTES / 16, WL = (WCELLS + NTH - 1) / NTH;
    static_assert(AL >= 1 && BM % RPJ == 0, "A rows per thread");
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    // XCD-aware tile order: XCD x walks the x-th contiguous slice of the
    // (pixel tile, channel tile) list, channel tiles fastest: the workgroups on
    // one XCD at a time share pixel tiles (A) and channel slices (W) in its L2
    const int xcd = blockIdx.x & 7, per = (num_tiles + 7) >> 3;
    const int tile = xcd * per + (int)(blockIdx.x >> 3);
    if (tile >= num_tiles) return;
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int64_t m0 = (int64_t)tm * BM;
    const int n0 = tn * BN;

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = w % WM, wn = w / WM;
    const int nsteps = K / kStep;

    // this thread's A rows / K quads (row = t / 4 + RPJ j, kq = t % 4)
    const int kq = t & 3;
    // A2 (K2 > 0): the last K2 of the K input channels come from a second operand
    // [M][K2] (a stage's first block: conv3 of h and the downsample of x, one GEMM)
    const int K1 = K - K2;
    const float *arow[AL], *arow2[AL];
#pragma unroll
    for (int j = 0; j < AL; ++j) {
        int64_t m = m0 + (t >> 2) + RPJ * j;
        if (m >= M) m = M - 1;
        if (SH > 0) {  // A read at stride 2 from images x SH x SW (a strided 1x1 conv)
            const int Ho = (SH + 1) >> 1, Wo = (SW + 1) >> 1;
            const int64_t hw = (int64_t)Ho * Wo, n = m / hw;
            const int rem = (int)(m - n * hw), y = rem / Wo, x = rem - y * Wo;
            m = (n * SH + 2 * y) * (int64_t)SW + 2 * x;
        }
        arow[j] = A + m * K1 + 4 * kq;
        arow2[j] = K2 ? A2 + m * K2 + 4 * kq : arow[j];
    }
    // the workgroup's weight slice of stage s: NTW consecutive (s, t) blocks
    const uint4 *wsrc = Wp + (int64_t)(n0 / 32) * (3 * 64);
    const int64_t wstep = (int64_t)(N / 32) * (3 * 64);

    float4 ar[AL];
    uint4 wr[WL];
    // abias (A prologue): A's first K1 channels enter as relu(A + abias[k]) -- the
    // bias + ReLU of the layer that produced A (a grouped 3x3 conv MIOpen runs without
    // them), applied in fp32 before the split, so bit-identical to a separate pass
    float4 abr = make_float4(0.f, 0.f, 0.f, 0.f);
    bool aon = false;
    // stage s's A rows and weight slice into registers (s clamped: the loads past
    // the last stage reread it and are never stored)
#define S3_LOAD(s_)                                                                       \
    do {                                                                                  \
        const int s = (s_) < nsteps ? (s_) : nsteps - 1;                                  \
        const int k0_ = kStep * s;                                                        \
        _Pragma("unroll") for (int j = 0; j < AL; ++j) ar[j] =                            \
            *reinterpret_cast<const float4 *>(k0_ < K1 ? arow[j] + k0_ : arow2[j] + (k0_ - K1)); \
        if constexpr (APRO) {                                                             \
            aon = k0_ < K1;                                                               \
            if (aon) abr = *reinterpret_cast<const float4 *>(abias + k0_ + 4 * kq);        \
        }                                                                                 \
        _Pragma("unroll") for (int j = 0; j < WL; ++j) {                                  \
            const int i = t + NTH * j;                                                    \
            wr[j] = (WCELLS % NTH == 0 || i < WCELLS) ? wsrc[s * wstep + i]               \
                                                           : make_uint4(0u, 0u, 0u, 0u);  \
        }                                                                                 \
    } while (0)
    // the registers into LDS buffer `buf` (A split into three pieces; W copied)
#define S3_STORE(buf)                                                                     \
    do {                                                                                  \
        unsigned char *base_ = lds + (buf) * BUF;                                         \
        if (APRO && aon) {                                                                \
            _Pragma("unroll") for (int j = 0; j < AL; ++j) {                              \
                ar[j].x = fmaxf(ar[j].x + abr.x, 0.f);                                    \
                ar[j].y = fmaxf(ar[j].y + abr.y, 0.f);                                    \
                ar[j].z = fmaxf(ar[j].z + abr.z, 0.f);                                    \
                ar[j].w = fmaxf(ar[j].w + abr.w, 0.f);                                    \
            }                                                                             \
        }                                                                                 \
        _Pragma("unroll") for (int j = 0; j < AL; ++j) {                                  \
            const int row = (t >> 2) + RPJ * j, pt = row >> 5, r = row & 31;              \
            uint32_t p00, p10, p20, p01, p11, p21;                                        \
            split_pair(ar[j].x, ar[j].y, p00, p10, p20);                                  \
            split_pair(ar[j].z, ar[j].w, p01, p11, p21);                                  \
            const int off = (pt * 64 + (kq >> 1) * 32 + r) * 16 + (kq & 1) * 8;           \
            *reinterpret_cast<uint2 *>(base_ + off) = make_uint2(p00, p01);               \
            *reinterpret_cast<uint2 *>(base_ + PT * kFragBytes + off) = make_uint2(p10, p11); \
            *reinterpret_cast<uint2 *>(base_ + 2 * PT * kFragBytes + off) =               \
                make_uint2(p20, p21);                                                     \
        }                                                                                 \
        _Pragma("unroll") for (int j = 0; j < WL; ++j) {                                  \
            const int i = t + NTH * j;                                                    \
            if (WCELLS % NTH == 0 || i < WCELLS)                                          \
                *reinterpret_cast<uint4 *>(base_ + A_BYTES + 16 * i) = wr[j];             \
        }                                                                                 \
    } while (0)

    f32x16 acc[TPM][TPN];
#pragma unroll
    for (int a = 0; a < TPM; ++a)
#pragma unroll
        for (int b = 0; b < TPN; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

    S3_LOAD(0);
    S3_STORE(0);
    S3_LOAD(1);
    __syncthreads();
    bf16x8 wf[TPN][3], af[TPM][3];
#pragma unroll 1
    for (int c = 0; c < nsteps; ++c) {
        const unsigned char *base = lds + (c & 1) * BUF;
        // research probes 4 / 5: the fragments read once (MFMA stream alone, without /
        // with the per-stage barrier)
        if (PROBE < 4 || c == 0) {
#pragma unroll
        for (int a = 0; a < TPM; ++a)
#pragma unroll
            for (int q = 0; q < 3; ++q)
                af[a][q] = *reinterpret_cast<const bf16x8 *>(
                    base + (q * PT + wm * TPM + a) * kFragBytes + lane * 16);
#pragma unroll
        for (int b = 0; b < TPN; ++b)
#pragma unroll
            for (int q = 0; q < 3; ++q)
                wf[b][q] = *reinterpret_cast<const bf16x8 *>(
                    base + A_BYTES + ((wn * TPN + b) * 3 + q) * kFragBytes + lane * 16);
        }
#pragma unroll
        for (int b = 0; b < TPN; ++b)
#pragma unroll
            for (int a = 0; a < TPM; ++a) {
                if (PROBE == 1) {
                    acc[a][b][0] += (float)wf[b][0][0] * (float)af[a][0][0];
                    continue;
                }
                f32x16 x = acc[a][b];
                x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[b][2], af[a][0], x, 0, 0, 0);
                x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[b][1], af[a][1], x, 0, 0, 0);
                x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[b][0], af[a][2], x, 0, 0, 0);
                x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[b][1], af[a][0], x, 0, 0, 0);
                x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[b][0], af[a][1], x, 0, 0, 0);
                x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[b][0], af[a][0], x, 0, 0, 0);
                acc[a][b] = x;
            }
        // stage c + 1 (its loads issued one stage ago) into the other buffer, whose
        // last readers passed the previous barrier; then stage c + 2's loads.  After
        // the last stage: a clamped copy into a buffer nobody reads.
        if (PROBE != 2 && PROBE < 4) S3_STORE((c + 1) & 1);
        if (PROBE != 3 && PROBE < 4) S3_LOAD(c + 2);
        if (PROBE != 4) __syncthreads();
    }
#undef S3_LOAD
#undef S3_STORE

    // epilogue: lane = pixel (r), registers 4g..4g+3 = channels 8g + 4h .. + 3
    const int h = lane >> 5, r = lane & 31;
    if constexpr (RES == 3) {
        static_assert(BN == 256 && RELU, "one (i, j) group per workgroup");
        // per pixel: sum over this wave's 128 channels of relu(acc + b) * Wc[class][co],
        // the two lane halves' channel sets added by a shuffle, the two channel waves
        // through LDS (the K loop's last barrier has passed: the buffers are free)
        float *part = reinterpret_cast<float *>(lds);  // [WN - 1][BM] partials, waves wn >= 1
        float dot[TPM];
#pragma unroll
        for (int a = 0; a < TPM; ++a) {
            const int64_t p = min(m0 + (wm * TPM + a) * 32 + r, (int64_t)M - 1);
            const int roi = (int)(p / (H * H));
            const float *wc = R + (int64_t)rch[roi] * BN;
            float sacc = 0.f;
#pragma unroll
            for (int b = 0; b < TPN; ++b) {
                const int cl = (wn * TPN + b) * 32 + 4 * h;  // channel within the group
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 bb = *reinterpret_cast<const float4 *>(bias + n0 + cl + 8 * g);
                    const float4 ww = *reinterpret_cast<const float4 *>(wc + cl + 8 * g);
                    sacc += fmaxf(acc[a][b][4 * g] + bb.x, 0.f) * ww.x;
                    sacc += fmaxf(acc[a][b][4 * g + 1] + bb.y, 0.f) * ww.y;
                    sacc += fmaxf(acc[a][b][4 * g + 2] + bb.z, 0.f) * ww.z;
                    sacc += fmaxf(acc[a][b][4 * g + 3] + bb.w, 0.f) * ww.w;
                }
            }
            dot[a] = sacc + __shfl_xor(sacc, 32);
        }
        if (wn >= 1 && h == 0) {
#pragma unroll
            for (int a = 0; a < TPM; ++a) part[(wn - 1) * BM + (wm * TPM + a) * 32 + r] = dot[a];
        }
        __syncthreads();
        if (wn == 0 && h == 0) {
            const int P = H, ij = tn;  // tap group (i, j) = (ij / 2, ij % 2)
#pragma unroll
            for (int a = 0; a < TPM; ++a) {
                const int64_t p = m0 + (wm * TPM + a) * 32 + r;
                if (p >= M) continue;
                const int roi = (int)(p / (P * P)), hw = (int)(p - (int64_t)roi * P * P);
                const int y = hw / P, x = hw - y * P;
                float z = dot[a];
#pragma unroll
                for (int u = 1; u < WN; ++u) z += part[(u - 1) * BM + (wm * TPM + a) * 32 + r];
                z += cb[rch[roi]];
                D[((int64_t)roi * 2 * P + 2 * y + (ij >> 1)) * 2 * P + 2 * x + (ij & 1)] =
                    1.f / (1.f + __expf(-z));
            }
        }
        return;
    }
#pragma unroll
    for (int a = 0; a < TPM; ++a) {
        const int64_t p = m0 + (wm * TPM + a) * 32 + r;
        if (p >= M) continue;
        int64_t rrow = p;
        if (RES == 2) {  // the nearest-2x source row of pixel p in the top-down map
            const int64_t hw = (int64_t)H * W, n = p / hw;
            const int rem = (int)(p - n * hw), y = rem / W, x = rem - y * W;
            rrow = (n * (H >> 1) + (y >> 1)) * (int64_t)(W >> 1) + (x >> 1);
        }
#pragma unroll
        for (int b = 0; b < TPN; ++b) {
            const int cb = n0 + (wn * TPN + b) * 32 + 4 * h;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int ch = cb + 8 * g;
                const float4 bb = *reinterpret_cast<const float4 *>(bias + ch);
                float4 o = make_float4(acc[a][b][4 * g] + bb.x, acc[a][b][4 * g + 1] + bb.y,
                                       acc[a][b][4 * g + 2] + bb.z, acc[a][b][4 * g + 3] + bb.w);
                if (RES) {  // (conv + bias) + residual: the reference's order
                    const float4 rr = *reinterpret_cast<const float4 *>(R + rrow * N + ch);
                    o.x += rr.x;
                    o.y += rr.y;
                    o.z += rr.z;
                    o.w += rr.w;
                }
                if (RELU) {
                    o.x = fmaxf(o.x, 0.f);
                    o.y = fmaxf(o.y, 0.f);
                    o.z = fmaxf(o.z, 0.f);
                    o.w = fmaxf(o.w, 0.f);
                }
                *reinterpret_cast<float4 *>(D + p * N + ch) = o;
            }
        }
    }
}

template <int BM, int BN, int TPM, int TPN, int RES, bool RELU, int PROBE = 0, int OCC = 1,
          int NW = 4, bool APRO = false>
int launch_cfg(const float *A, int M, int K, const uint4 *Wp, int N, const float *bias,
               const float *R, float *D, int H, int W, int SH, int SW, hipStream_t s,
               const float *cb = nullptr, const int32_t *rch = nullptr,
               const float *A2 = nullptr, int K2 = 0, const float *abias = nullptr) {
    constexpr int PT = BM / 32, NTW = BN / 32;
    constexpr size_t lds = 2 * (size_t)(3 * PT + NTW * 3) * kFragBytes;
    static_assert(lds <= VD_LDS_BYTES, "LDS");
    auto kern = gemm_split3_kernel<BM, BN, TPM, TPN, RES, RELU, PROBE, OCC, NW, APRO>;
    static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)lds) == hipSuccess;
    if (!attr) return VD_ERR_LAUNCH;
    const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;
    const int64_t num_tiles = (int64_t)tiles_m * tiles_n;
    if (num_tiles >= (1ll << 31) - 8) return VD_ERR_SHAPE;
    const int64_t grid = (num_tiles + 7) / 8 * 8;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * NW), lds, s, A, Wp, bias, R, D, M, N,
                       K, tiles_n, (int)num_tiles, H, W, SH, SW, cb, rch, A2, K2, abias);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

template <int BM, int BN, int TPM, int TPN, int OCC, int NW = 4>
int launch_epi(const float *A, int M, int K, const uint4 *Wp, int N, const float *bias,
               const float *R, int relu, float *D, int H, int W, int SH, int SW, hipStream_t s,
               const float *A2, int K2, const float *abias) {
#define VD_S3_RELU(RES_)                                                                       \
    return relu ? launch_cfg<BM, BN, TPM, TPN, RES_, true, 0, OCC, NW>(                        \
                      A, M, K, Wp, N, bias, R, D, H, W, SH, SW, s, nullptr, nullptr, A2, K2,   \
                      abias)                                                                   \
                : launch_cfg<BM, BN, TPM, TPN, RES_, false, 0, OCC, NW>(                       \
                      A, M, K, Wp, N, bias, R, D, H, W, SH, SW, s, nullptr, nullptr, A2, K2,   \
                      abias)
    if (abias) {  // the A prologue: compiled only where it is used (conv3 after a
                  // grouped conv2: ReLU, with or without a residual)
        if (!relu || (R && H > 0)) return VD_ERR_ARG;
        if (R)
            return launch_cfg<BM, BN, TPM, TPN, 1, true, 0, OCC, NW, true>(
                A, M, K, Wp, N, bias, R, D, H, W, SH, SW, s, nullptr, nullptr, A2, K2, abias);
        return launch_cfg<BM, BN, TPM, TPN, 0, true, 0, OCC, NW, true>(
            A, M, K, Wp, N, bias, R, D, H, W, SH, SW, s, nullptr, nullptr, A2, K2, abias);
    }
    if (R && H > 0) VD_S3_RELU(2);
    if (R) VD_S3_RELU(1);
    VD_S3_RELU(0);
#undef VD_S3_RELU
}

}  // namespace

bool gemm_split3_supported(int K, int N) { return K >= kStep && K % kStep == 0 && N % 64 == 0; }

size_t gemm_split3_weight_bytes(int N, int K) { return (size_t)N * K * 6; }

int launch_gemm_split3_weight(const float *W, int N, int K, void *Wp, hipStream_t s) {
    if (!gemm_split3_supported(K, N)) return VD_ERR_SHAPE;
    const int64_t cells = (int64_t)(K / kStep) * (N / 32) * 64;
    const int64_t blocks = (cells + 255) / 256;
    hipLaunchKernelGGL(split3_weight_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)),
                       dim3(256), 0, s, W, N, K, reinterpret_cast<uint4 *>(Wp));
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// cfg: 0 = auto, 1 = 256 x 256 (one workgroup per CU), 2 = 256 x 128, 3 = 256 x 64 (two
// per CU), 4 = 128 x 128 (three per CU), 5 = 256 x 256 with 8 waves (one per CU) --
// pixels x channels per workgroup; waves of 128 x 128 / 128 x 64 / 128 x 32 / 64 x 64 /
// 128 x 64
// up_h / up_w > 0: R is the top-down map of an images x up_h x up_w level (M = images
// x up_h x up_w, both even), read at the nearest-2x row of each pixel.  sub_h / sub_w
// > 0: A is an images x sub_h x sub_w map read at stride 2 (M = images x ceil(sub_h / 2)
// x ceil(sub_w / 2)): a stride-2 pad-0 1x1 convolution without the subsampled copy.
// a_bias (K - K2 floats, or null): A's channels enter as relu(A + a_bias[k]).
int launch_gemm_split3(const float *A, int M, int K, const float *A2, int K2, const void *Wp,
                       int N, const float *bias, const float *R, int up_h, int up_w, int sub_h,
                       int sub_w, int relu, float *D, int cfg, hipStream_t s,
                       const float *a_bias) {
    if (M == 0) return VD_OK;
    if (!gemm_split3_supported(K, N)) return VD_ERR_SHAPE;
    if (K2 < 0 || K2 >= K || (K2 && (!A2 || K2 % kStep || sub_h || sub_w))) return VD_ERR_ARG;
    if (!K2) A2 = nullptr;
    if (sub_h || sub_w) {
        if (sub_h < 1 || sub_w < 1 || M % ((int64_t)((sub_h + 1) / 2) * ((sub_w + 1) / 2)))
            return VD_ERR_ARG;
    }
    if (up_h || up_w) {
        if (!R || up_h < 2 || up_w < 2 || (up_h & 1) || (up_w & 1) ||
            M % ((int64_t)up_h * up_w))
            return VD_ERR_ARG;
    }
    const uint4 *w = reinterpret_cast<const uint4 *>(Wp);
    if (cfg == 0) {
        // 256 x 128 tiles at two workgroups per CU (two waves per SIMD hide each
        // other's LDS / barrier stalls: 10-20 % faster than one 256 x 256 workgroup on
        // the step's shapes), the 256 x 256 single workgroup only for very deep K
        // (fc6, K = 12,544: 4 % faster), 256 x 64 where N is not a multiple of 128
        // (profiles/r06/gemm_split3/)
        cfg = N % 128 == 0 ? 2 : 3;
        // 256 x 256 tiles with eight 128 x 64 waves (one workgroup per CU, the A split
        // shared by twice the channels) for deep K, large M, and fc7-like shapes: 2-7 %
        // faster than 256 x 128 there, slower on the few-tile res4 / res5 shapes
        // (VOSDET_SPLIT3_WIDE=0 keeps 256 x 128: A/B runs)
        static const bool wide = [] {
            const char *e = getenv("VOSDET_SPLIT3_WIDE");
            return !(e && e[0] == '0');
        }();
        // (N, K >= 1024 at any M: ResNeXt's 1024-wide res4 1x1s at 64 frames, 2.76 ->
        // 2.51 ms, profiles/r06/split3_cfg/)
        if (wide && N % 256 == 0 &&
            (K >= 4096 || M >= 500000 || (N >= 1024 && K >= 1024)))
            cfg = 5;
        // 128 x 128 tiles at three workgroups per CU where 256 x 128 would give fewer
        // than three workgroups per slot (res4 / res5 at 32 frames, N <= 512): more
        // workgroups in flight, 5-15 % faster there (profiles/r06/gemm_split3/)
        if (cfg == 2 && N <= 512 && (int64_t)((M + 255) / 256) * (N / 128) < 1536) cfg = 4;
    }
    switch (cfg) {
    case 1:
        if (N % 256) return VD_ERR_SHAPE;
        return launch_epi<256, 256, 4, 4, 1>(A, M, K, w, N, bias, R, relu, D, up_h, up_w, sub_h, sub_w,
                                             s, A2, K2, a_bias);
    case 2:
        if (N % 128) return VD_ERR_SHAPE;
        return launch_epi<256, 128, 4, 2, 2>(A, M, K, w, N, bias, R, relu, D, up_h, up_w, sub_h, sub_w,
                                             s, A2, K2, a_bias);
    case 5:
        if (N % 256) return VD_ERR_SHAPE;
        return launch_epi<256, 256, 4, 2, 1, 8>(A, M, K, w, N, bias, R, relu, D, up_h, up_w, sub_h,
                                                sub_w, s, A2, K2, a_bias);
    case 4:
        if (N % 128) return VD_ERR_SHAPE;
        return launch_epi<128, 128, 2, 2, 3>(A, M, K, w, N, bias, R, relu, D, up_h, up_w, sub_h, sub_w,
                                             s, A2, K2, a_bias);
    case 3:
        return launch_epi<256, 64, 4, 1, 2>(A, M, K, w, N, bias, R, relu, D, up_h, up_w, sub_h, sub_w,
                                             s, A2, K2, a_bias);
#ifdef VD_RESEARCH_PROBES
    case 11: case 12: case 13:  // speed-of-light probes of cfg 1 (wrong results by design)
        if (N % 256 || R || !relu) return VD_ERR_SHAPE;
        if (cfg == 11) return launch_cfg<256, 256, 4, 4, 0, true, 1>(A, M, K, w, N, bias, R, D, 0, 0, 0, 0, s);
        if (cfg == 12) return launch_cfg<256, 256, 4, 4, 0, true, 2>(A, M, K, w, N, bias, R, D, 0, 0, 0, 0, s);
        return launch_cfg<256, 256, 4, 4, 0, true, 3>(A, M, K, w, N, bias, R, D, 0, 0, 0, 0, s);
    case 14: case 15:  // cfg 2: MFMA stream alone (fragments read once), without / with barriers
        if (N % 128 || R || !relu) return VD_ERR_SHAPE;
        if (cfg == 14) return launch_cfg<256, 128, 4, 2, 0, true, 4, 2>(A, M, K, w, N, bias, R, D, 0, 0, 0, 0, s);
        return launch_cfg<256, 128, 4, 2, 0, true, 5, 2>(A, M, K, w, N, bias, R, D, 0, 0, 0, 0, s);
    case 16: case 17: case 18:  // the same probes of cfg 2
        if (N % 128 || R || !relu) return VD_ERR_SHAPE;
        if (cfg == 16) return launch_cfg<256, 128, 4, 2, 0, true, 1, 2>(A, M, K, w, N, bias, R, D, 0, 0, 0, 0, s);
        if (cfg == 17) return launch_cfg<256, 128, 4, 2, 0, true, 2, 2>(A, M, K, w, N, bias, R, D, 0, 0, 0, 0, s);
        return launch_cfg<256, 128, 4, 2, 0, true, 3, 2>(A, M, K, w, N, bias, R, D, 0, 0, 0, 0, s);
#endif
    default:
        return VD_ERR_ARG;
    }
}

int launch_gemm_split3_mask_logits(const float *A, int M, int K, const void *Wp, int N,
                                   const float *bias, const float *cls_w, const float *cls_b,
                                   const int32_t *roi_ch, int P, float *masks, hipStream_t s) {
    if (M == 0) return VD_OK;
    if (N != 4 * 256 || !gemm_split3_supported(K, N)) return VD_ERR_SHAPE;
    if (P < 1 || M % (P * P) || !cls_w || !cls_b || !roi_ch || !masks) return VD_ERR_ARG;
    return launch_cfg<256, 256, 4, 2, 3, true, 0, 1, 8>(A, M, K,
                                                        reinterpret_cast<const uint4 *>(Wp), N,
                                                        bias, cls_w, masks, P, P, 0, 0, s, cls_b,
                                                        roi_ch);
}

}  // namespace vd
