// ResNet stem in one pass: conv1 7x7 / 2 pad 3 (3 -> 64 channels) on the MFMA
// pipes, the folded AffineChannel bias, ReLU and MaxPool 3x3 / 2 pad 1
// (basic_bn_stem, lib/modeling/ResNet.py:224-230; conv1 + bn1 + relu + maxpool).
//
// The conv output (N x 400 x 672 x 64 fp32 for an 800 x 1344 blob, 1.1 GB) never
// reaches HBM: a workgroup computes the 15 x 17 conv pixels under a 7 x 8 tile of
// pooled outputs (one conv row / column of halo recomputed, 13.8 %), keeps them in
// LDS and writes only the pooled tile (4.3x fewer bytes than the conv).
//
// GEMM view per tile: D[co][pixel] = sum_k W[co][k] P[k][pixel], K = 7 x 7 x 3 =
// 147 (+1 zero) ordered (ky, kx, ci) so that a k row of 21 is contiguous in the
// NHWC input patch; v_mfma_f32_16x16x4_f32 (fp32 in / out: the reference's
// precision).  4 waves, one per SIMD: wave w owns conv-pixel blocks 4w .. 4w + 3
// (16 pixels each, 255 real) x all 4 blocks of 16 output channels; the weights
// (37 k-steps x 4 blocks = 148 values per lane) stay in registers for the
// workgroup's lifetime (a persistent grid walks the tiles), so a k-step costs four
// LDS reads (the pixels' patch values) per sixteen MFMAs.
#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));

// two fp32 -> three packed bf16 pairs, round to nearest even (gemm_split3.hip)
__device__ __forceinline__ void split_pair(float x0, float x1, uint32_t &p0, uint32_t &p1,
                                           uint32_t &p2) {
    const f2v x = {x0, x1};
    const uint32_t uh = __builtin_bit_cast(uint32_t, __builtin_convertvector(x, bf16x2));
    const f2v r1 = x - f2v{__uint_as_float(uh << 16), __uint_as_float(uh & 0xffff0000u)};
    const uint32_t um = __builtin_bit_cast(uint32_t, __builtin_convertvector(r1, bf16x2));
    const f2v r2 = r1 - f2v{__uint_as_float(um << 16), __uint_as_float(um & 0xffff0000u)};
    p0 = uh;
    p1 = um;
    p2 = __builtin_bit_cast(uint32_t, __builtin_convertvector(r2, bf16x2));
}

constexpr int kPY = 7, kPX = 8;                       // pooled outputs per tile
constexpr int kCY = 2 * kPY + 1, kCX = 2 * kPX + 1;   // 15 x 17 conv outputs
constexpr int kCP = kCY * kCX;                        // 255
constexpr int kIY = 2 * (kCY - 1) + 7, kIX = 2 * (kCX - 1) + 7;  // 35 x 39 input pixels
constexpr int kRow = 3 * kIX;                         // 117 floats per patch row
constexpr int kPatch = kIY * kRow;                    // 4095 floats
constexpr int kKS = 37;                               // k-steps of 4 (K = 147 + 1 zero)
constexpr int kKS3 = 5;                               // SPLIT: k-steps of 32 (K = 160)
constexpr int kThreadsF = 256;                        // fp32 core: 4 waves of 4 pixel blocks
constexpr int kThreadsS = 512;                        // SPLIT: 8 waves (2 a SIMD) of 2
constexpr int kOutPitch = 68;                         // floats per conv pixel in LDS

// patch offset (floats) of k = (ky, kx, ci) = 21 ky + 3 kx + ci; k = 147 is the
// zero-weight pad and reads k = 146's (finite) value
__device__ __forceinline__ int koff(int k) {
    k = k < 146 ? k : 146;
    const int ky = k / 21;
    return k + (kRow - 21) * ky;
}

// SPLIT (round 6, the default): conv1 on the bf16 matrix cores at fp32 accuracy --
// v_mfma_f32_16x16x32_bf16 over K = 160 (5 k-steps; k >= 147 zero weights), every fp32
// operand split into three bf16 pieces and the six largest piece products accumulated
// (gemm_split3.hip's scheme): the weights pre-split once (stem_weight_split_kernel,
// 240 dwords a lane held for the workgroup's lifetime), each pixel's eight patch
// values of a k-step split as they are read.  6 x 80 bf16 MFMAs of 16 cycles per
// wave and tile against 592 fp32 MFMAs of 32.
template <bool SPLIT, int NT>
__global__ __launch_bounds__(NT, 1) void stem_conv_pool_kernel(
    const float *__restrict__ X, int N, int H, int W, const float *__restrict__ Wp,
    const float *__restrict__ bias, float *__restrict__ Y, int Hc, int Wc, int Hp, int Wp_,
    int tiles_y, int tiles_x, int ntiles) {
    __shared__ __attribute__((aligned(16))) float patch[kPatch + 1];
    __shared__ __attribute__((aligned(16))) float outs[256 * kOutPitch];
    constexpr int kThreads = NT;
    constexpr int kPB = 1024 / NT;  // conv-pixel blocks per wave (16 blocks of 16)
    constexpr int kPer = (kPatch + NT - 1) / NT;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 15, q = lane >> 4;

    // the lane's weights: A[co = 16 b + j][k = 4 s + q] (fp32), or (SPLIT) the three
    // bf16 pieces of A[co = 16 b + j][k = 32 s + 8 q .. + 7]
    constexpr int kWS = SPLIT ? 1 : kKS;
    float wr[kWS][4];
    // (SPLIT: the 61 KiB split image sits in LDS, lane-linear 16-byte fragments read
    // with ds_read_b128 -- held in registers it spills)
    __shared__ __attribute__((aligned(16))) uint4 wl[SPLIT ? kKS3 * 4 * 3 * 64 : 1];
    if constexpr (SPLIT) {
        const uint4 *w4 = reinterpret_cast<const uint4 *>(Wp);
        for (int i = tid; i < kKS3 * 4 * 3 * 64; i += kThreads) wl[i] = w4[i];
    } else {
#pragma unroll
        for (int s = 0; s < kKS; ++s)
#pragma unroll
            for (int b = 0; b < 4; ++b) wr[s][b] = Wp[(s * 4 + b) * 64 + lane];
    }

    // the lane's conv pixels (column j of blocks kPB wave + pb): patch base
    // offsets; pixel 255 is padding and reads pixel 254
    int pbase[kPB];
#pragma unroll
    for (int pb = 0; pb < kPB; ++pb) {
        int t = (kPB * wave + pb) * 16 + j;
        t = t < kCP ? t : kCP - 1;
        const int ty = t / kCX, tx = t - (t / kCX) * kCX;
        pbase[pb] = 2 * ty * kRow + 6 * tx;
    }

    // XCD-aware walk: blocks b, b + 8, ... (one XCD) take a contiguous tile range
    const int nx = 8, xcd = blockIdx.x % nx, per = gridDim.x / nx;
    const int slot = blockIdx.x / nx;
    const int lo = (int)((int64_t)ntiles * xcd / nx), hi = (int)((int64_t)ntiles * (xcd + 1) / nx);

    auto tile_origin = [&](int t, int &n, int &py0, int &px0) {
        n = t / (tiles_y * tiles_x);
        const int r = t - n * tiles_y * tiles_x;
        py0 = (r / tiles_x) * kPY;
        px0 = (r - (r / tiles_x) * tiles_x) * kPX;
    };
    auto load_patch = [&](int t, float (&v)[kPer]) {
        int n, py0, px0;
        tile_origin(t, n, py0, px0);
        const int iy0 = 4 * py0 - 5, ix0 = 4 * px0 - 5;
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int e = tid + i * kThreads;
            const int r = e / kRow, cc = e - (e / kRow) * kRow;
            const int y = iy0 + r, x = ix0 + cc / 3;
            const bool ok = e < kPatch && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
            v[i] = ok ? X[((int64_t)(n * H + y) * W + ix0) * 3 + cc] : 0.f;
        }
    };

    float pre[kPer];
    int t = lo + slot;
    if (t < hi) {
        load_patch(t, pre);
#pragma unroll
        for (int i = 0; i < kPer; ++i)
            if (tid + i * kThreads < kPatch) patch[tid + i * kThreads] = pre[i];
    }
    __syncthreads();
    for (; t < hi; t += per) {
        const int tn = t + per;
        if (tn < hi) load_patch(tn, pre);  // lands while the MFMAs run
        f4v acc[kPB][4];
#pragma unroll
        for (int pb = 0; pb < kPB; ++pb)
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[pb][b] = f4v{0.f, 0.f, 0.f, 0.f};
        if constexpr (SPLIT) {
#pragma unroll
            for (int s = 0; s < kKS3; ++s) {
                int ko[8];  // patch offsets of the lane's k values
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) ko[jj] = koff(32 * s + 8 * q + jj);
                bf16x8 bp[kPB][3];  // the pixels' pieces
#pragma unroll
                for (int pb = 0; pb < kPB; ++pb) {
                    float v[8];
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) v[jj] = patch[pbase[pb] + ko[jj]];
                    uint32_t p0[4], p1[4], p2[4];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        split_pair(v[2 * jj], v[2 * jj + 1], p0[jj], p1[jj], p2[jj]);
                    bp[pb][0] = __builtin_bit_cast(bf16x8, make_uint4(p0[0], p0[1], p0[2], p0[3]));
                    bp[pb][1] = __builtin_bit_cast(bf16x8, make_uint4(p1[0], p1[1], p1[2], p1[3]));
                    bp[pb][2] = __builtin_bit_cast(bf16x8, make_uint4(p2[0], p2[1], p2[2], p2[3]));
                }
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    bf16x8 w[3];
#pragma unroll
                    for (int pc = 0; pc < 3; ++pc)
                        w[pc] = __builtin_bit_cast(bf16x8, wl[((s * 4 + b) * 3 + pc) * 64 + lane]);
#pragma unroll
                    for (int pb = 0; pb < kPB; ++pb) {
                        f4v x = acc[pb][b];
                        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2], bp[pb][0], x, 0, 0, 0);
                        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], bp[pb][1], x, 0, 0, 0);
                        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], bp[pb][2], x, 0, 0, 0);
                        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], bp[pb][0], x, 0, 0, 0);
                        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], bp[pb][1], x, 0, 0, 0);
                        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], bp[pb][0], x, 0, 0, 0);
                        acc[pb][b] = x;
                    }
                }
            }
        } else {
#pragma unroll
        for (int s = 0; s < kKS; ++s) {
            const int o = koff(4 * s + q);
            float v[kPB];
#pragma unroll
            for (int pb = 0; pb < kPB; ++pb) v[pb] = patch[pbase[pb] + o];
#pragma unroll
            for (int pb = 0; pb < kPB; ++pb)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[pb][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[s][b], v[pb], acc[pb][b],
                                                                      0, 0, 0);
        }
        }
        // D[co = 16 b + 4 q + r][pixel j] -> outs[pixel][co]
#pragma unroll
        for (int pb = 0; pb < kPB; ++pb) {
            const int p = (kPB * wave + pb) * 16 + j;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                *reinterpret_cast<f4v *>(&outs[p * kOutPitch + 16 * b + 4 * q]) = acc[pb][b];
        }
        __syncthreads();  // conv tile complete; every patch read retired
        if (tn < hi) {
#pragma unroll
            for (int i = 0; i < kPer; ++i)
                if (tid + i * kThreads < kPatch) patch[tid + i * kThreads] = pre[i];
        }
        // max-pool 3 x 3 / 2 pad 1 over the conv tile (conv origin 2 py0 - 1,
        // 2 px0 - 1; positions outside the conv map are the pool's padding), then
        // bias + ReLU (max(v) + b = max(v + b): rounding is monotonic)
        int n, py0, px0;
        tile_origin(t, n, py0, px0);
        for (int task = tid; task < kPY * kPX * 16; task += kThreads) {
            const int p = task >> 4, c4 = task & 15;
            const int pyl = p / kPX, pxl = p - (p / kPX) * kPX;
            const int py = py0 + pyl, px = px0 + pxl;
            if (py >= Hp || px >= Wp_) continue;
            f4v m = f4v{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                const int cy = 2 * py - 1 + dy;
                if ((unsigned)cy >= (unsigned)Hc) continue;
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    const int cx = 2 * px - 1 + dx;
                    if ((unsigned)cx >= (unsigned)Wc) continue;
                    const f4v v = *reinterpret_cast<const f4v *>(
                        &outs[((2 * pyl + dy) * kCX + 2 * pxl + dx) * kOutPitch + 4 * c4]);
                    m.x = fmaxf(m.x, v.x);
                    m.y = fmaxf(m.y, v.y);
                    m.z = fmaxf(m.z, v.z);
                    m.w = fmaxf(m.w, v.w);
                }
            }
            const float4 bv = reinterpret_cast<const float4 *>(bias)[c4];
            const float4 o = make_float4(fmaxf(m.x + bv.x, 0.f), fmaxf(m.y + bv.y, 0.f),
                                         fmaxf(m.z + bv.z, 0.f), fmaxf(m.w + bv.w, 0.f));
            reinterpret_cast<float4 *>(Y)[((int64_t)(n * Hp + py) * Wp_ + px) * 16 + c4] = o;
        }
        __syncthreads();  // pooled reads of outs done; the next patch visible
    }
}

// Wp[s][b][lane] = w[co = 16 b + lane % 16][k = 4 s + lane / 16], k = (ky, kx, ci),
// from the PyTorch weight w[64][3][7][7]; k = 147 -> 0
__global__ void stem_weight_kernel(const float *__restrict__ w, float *__restrict__ Wp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kKS * 4 * 64) return;
    const int lane = i & 63, b = (i >> 6) & 3, s = i >> 8;
    const int co = 16 * b + (lane & 15), k = 4 * s + (lane >> 4);
    float v = 0.f;
    if (k < 147) {
        const int ky = k / 21, r = k - (k / 21) * 21, kx = r / 3, ci = r - (r / 3) * 3;
        v = w[((co * 3 + ci) * 7 + ky) * 7 + kx];
    }
    Wp[i] = v;
}

// SPLIT weights: Wp3[s][b][piece][lane][8 bf16] = piece of w[co = 16 b + lane % 16]
// [k = 32 s + 8 (lane / 16) + j], k = (ky, kx, ci); k >= 147 -> 0
__global__ void stem_weight_split_kernel(const float *__restrict__ w, uint4 *__restrict__ Wp3) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kKS3 * 4 * 64) return;
    const int lane = i & 63, b = (i >> 6) & 3, s = i >> 8;
    const int co = 16 * b + (lane & 15), k0 = 32 * s + 8 * (lane >> 4);
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
        const int k = k0 + jj;
        v[jj] = 0.f;
        if (k < 147) {
            const int ky = k / 21, r = k - (k / 21) * 21, kx = r / 3, ci = r - (r / 3) * 3;
            v[jj] = w[((co * 3 + ci) * 7 + ky) * 7 + kx];
        }
    }
    uint32_t p[3][4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) split_pair(v[2 * jj], v[2 * jj + 1], p[0][jj], p[1][jj], p[2][jj]);
#pragma unroll
    for (int pc = 0; pc < 3; ++pc)
        Wp3[((s * 4 + b) * 3 + pc) * 64 + lane] = make_uint4(p[pc][0], p[pc][1], p[pc][2], p[pc][3]);
}

}  // namespace

size_t stem_weight_floats() { return (size_t)kKS * 4 * 64; }

size_t stem_weight_split_bytes() { return (size_t)kKS3 * 4 * 3 * 64 * 16; }

int launch_stem_weight_split(const float *w, void *Wp3, hipStream_t s) {
    hipLaunchKernelGGL(stem_weight_split_kernel, dim3((kKS3 * 256 + 255) / 256), dim3(256), 0, s,
                       w, reinterpret_cast<uint4 *>(Wp3));
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int launch_stem_weight(const float *w, float *Wp, hipStream_t s) {
    hipLaunchKernelGGL(stem_weight_kernel, dim3((kKS * 256 + 255) / 256), dim3(256), 0, s, w, Wp);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int launch_stem_conv_pool(const float *X, int N, int H, int W, const float *Wp, const float *bias,
                          float *Y, int num_cus, hipStream_t s, bool split) {
    if (N < 0 || H < 0 || W < 0) return VD_ERR_SHAPE;
    if ((int64_t)N * H * W == 0) return VD_OK;
    const int Hc = (H - 1) / 2 + 1, Wc = (W - 1) / 2 + 1;   // (H + 6 - 7) / 2 + 1
    const int Hp = (Hc - 1) / 2 + 1, Wp_ = (Wc - 1) / 2 + 1;  // (Hc + 2 - 3) / 2 + 1
    const int tiles_y = (Hp + kPY - 1) / kPY, tiles_x = (Wp_ + kPX - 1) / kPX;
    const int64_t ntiles = (int64_t)N * tiles_y * tiles_x;
    if (ntiles > 0x3fffffff || (int64_t)N * H * W * 3 >= ((int64_t)1 << 31) ||
        (int64_t)N * Hp * Wp_ * 16 >= ((int64_t)1 << 31))
        return VD_ERR_SHAPE;
    // one persistent workgroup per CU (86 KB of LDS), a multiple of the 8 XCDs
    if (num_cus <= 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                hipSuccess)
            num_cus = 256;
    }
    int g = num_cus;
    g = g / 8 * 8;
    if (g < 8) g = 8;
    if (split)
        hipLaunchKernelGGL((stem_conv_pool_kernel<true, kThreadsS>), dim3(g), dim3(kThreadsS), 0, s,
                           X, N, H, W,
                           Wp, bias, Y, Hc, Wc, Hp, Wp_, tiles_y, tiles_x, (int)ntiles);
    else
        hipLaunchKernelGGL((stem_conv_pool_kernel<false, kThreadsF>), dim3(g), dim3(kThreadsF), 0, s,
                           X, N, H, W,
                           Wp, bias, Y, Hc, Wc, Hp, Wp_, tiles_y, tiles_x, (int)ntiles);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
