// 3x3 stride-1 pad-1 convolution on NHWC fp32 as an MFMA implicit GEMM with the
// bias (+ ReLU) epilogue fused.
//
// The 256 -> 256 3x3 convolutions are half of a Mask R-CNN step: FPN posthoc
// (lib/modeling/FPN.py:227-258, conv + bias), the RPN conv (FPN.py:376-422),
// the mask head's four convs (mask_rcnn_heads.py:178-188, conv + bias + ReLU)
// and res4's conv2.  Implicit GEMM:
//   D[m][co] = sum_{t = (ky,kx), ci} X[pixel m shifted by (ky-1, kx-1)][ci] . W2[co][t][ci]
// with out-of-image taps reading zero; W2 = the weight permuted to
// [Cout][3][3][Cin] once on the host side (k = 9 taps x Cin contiguous per co).
//
// Tiling: a workgroup (4 waves, one per SIMD) computes 128 pixels x 128 output
// channels; wave w owns 64 x 64 (pixels (w & 1) * 64, channels (w >> 1) * 64)
// as 4 x 4 tiles of v_mfma_f32_16x16x4_f32 in the transposed orientation (MFMA
// A operand = weights, B operand = pixels), so each lane's accumulators are 4
// consecutive output channels of one pixel and the epilogue stores float4s.
// The K axis (9 x Cin) is walked in chunks of 64 input channels of one tap:
// the chunk's pixel rows (128 x 256 B) and weight rows (128 x 256 B) are
// staged in LDS, 16-byte chunk c of row r at c ^ (r & 15) so every fragment
// read (lane = row, 4 lanes per 64 contiguous bytes) is a conflict-free
// ds_read_b128; the next chunk's global loads are in flight while the current
// chunk's 256 MFMAs per wave run; one LDS stage per workgroup and two
// workgroups per CU, so one's store phase overlaps the other's MFMAs.
// Per 16 input channels (kb) a lane holds channels 16 kb + 4 q .. + 3 (q = lane
// / 16) of its row in both operands: a K permutation shared by A and B.
#include <stdlib.h>

#include <mutex>
#include <set>

#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kTM = 128, kTN = 128;  // tile: pixels x output channels

// KC input channels per K chunk, STAGES LDS stages per workgroup.  Row r of a
// stage holds KC / 4 float4s, float4 c stored at c ^ swz(r): conflict-free
// ds_read_b128 for 16 lanes reading 16 consecutive rows at one c.
template <int KC>
__device__ __forceinline__ int swz(int r) {
    return KC == 64 ? (r & 15) : ((r >> 1) & 7);
}

// TM x TN: the workgroup tile (pixels x output channels), 4 waves of 64 x 64:
// 128 x 128 (2 x 2 waves) or 256 x 64 (4 x 1, for Cout = 64).
// WTP x WTC: a wave's 16 x 16 MFMA tiles along pixels x channels (4 x 4 = 64 x 64;
// 2 x 4 = 32 x 64 for the 64 x 128 workgroup tile of the mid-size shapes, which
// runs three workgroups per CU).
template <bool RELU, int KC, int STAGES, int TM = kTM, int TN = kTN, int WTP = 4, int WTC = 4,
          int WGS = 2>
__global__ __launch_bounds__(256, WGS) void conv3x3_mfma_kernel(
    const float *__restrict__ X, int N, int H, int W, int C, const float *__restrict__ W2,
    int Cout, const float *__restrict__ bias, float *__restrict__ Y, int mtiles) {
    constexpr int R4 = KC / 4;               // float4s per staged row
    constexpr int STAGE = (TM + TN) * R4;    // float4s per stage
    constexpr int RP = 256 / R4;             // rows per staging pass
    constexpr int NI = TM / RP, NB = TN / RP;  // passes for pixel / weight rows
    constexpr int WPX = TM / (16 * WTP);     // waves along the pixels
    static_assert(WPX * (TN / (16 * WTC)) == 4, "four waves per workgroup");
    extern __shared__ __attribute__((aligned(16))) float4 lds[];  // [STAGES][TM + TN][R4]
    const int64_t M = (int64_t)N * H * W;
    const int tid = threadIdx.x, lane = lane_id(), wave = wave_id();
    const int j = lane & 15, q = lane >> 4;
    // the Cout / TN channel tiles of a pixel tile are blocks b, b + 8, ... --
    // the same XCD (block b runs on XCD b % 8), so its pixel rows come from one L2
    const int ntiles = Cout / TN;
    const int r16 = blockIdx.x % (8 * ntiles);
    const int nt = r16 / 8, mt = (blockIdx.x / (8 * ntiles)) * 8 + (r16 & 7);
    if (mt >= mtiles) return;
    const int64_t m0 = (int64_t)mt * TM;
    const int n0 = nt * TN;
    // staging: thread t moves float4 sc = t % R4 of rows sr0 + RP i (i < NI)
    const int sc = tid % R4, sr0 = tid / R4;
    int py[NI], px[NI], pix[NI];  // pixel row / column / linear index (M * C < 2^29)
    bool pv[NI];
    const int HW = H * W;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int m = (int)m0 + sr0 + RP * i;
        pv[i] = m < M;
        pix[i] = pv[i] ? m : 0;
        const int rem = pix[i] % HW;
        py[i] = rem / W;
        px[i] = rem - py[i] * W;
    }
    const int K9 = 9 * C;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(X), (short)0, (int)(M * C * 4), 0x00020000);
    const int cblocks = C / KC, nchunks = 9 * cblocks;
    // weight rows n0 + sr0 + RP i, float4 sc of the chunk's KC k (buffer offsets)
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(W2), (short)0, Cout * K9 * 4, 0x00020000);
    const int wrow0 = (n0 + sr0) * K9 + 4 * sc;
    f4v acc[WTC][WTP];
#pragma unroll
    for (int tc = 0; tc < WTC; ++tc)
#pragma unroll
        for (int tp = 0; tp < WTP; ++tp) acc[tc][tp] = f4v{0.f, 0.f, 0.f, 0.f};
    const int pw0 = (wave % WPX) * 16 * WTP, cw0 = (wave / WPX) * 16 * WTC;
    // chunk ch = (tap, channel block): its pixel / weight float4s in registers
#define VD_LOAD_CHUNK(CH)                                                                   \
    {                                                                                       \
        const int tap_ = (CH) / cblocks, cb_ = (CH) - tap_ * cblocks;                       \
        const int dy_ = tap_ / 3 - 1, dx_ = tap_ % 3 - 1;                                   \
        const int koff_ = tap_ * C + cb_ * KC;                                              \
        _Pragma("unroll") for (int i = 0; i < NI; ++i) {                                    \
            const int y_ = py[i] + dy_, x_ = px[i] + dx_;                                   \
            const bool ok_ = pv[i] & ((unsigned)y_ < (unsigned)H) & ((unsigned)x_ < (unsigned)W); \
            /* out-of-image taps read past the buffer's range: zeros, no branch */         \
            const int off_ = ok_ ? ((pix[i] + dy_ * W + dx_) * C + cb_ * KC + 4 * sc) * 4    \
                                 : 0x7ffffff0;                                              \
            ra[i] = __builtin_bit_cast(float4,                                              \
                                       __builtin_amdgcn_raw_buffer_load_b128(xr, off_, 0, 0)); \
        }                                                                                   \
        _Pragma("unroll") for (int i = 0; i < NB; ++i)                                      \
            rb[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(             \
                        wr, (wrow0 + RP * i * K9 + koff_) * 4, 0, 0));                      \
    }
#define VD_STORE_CHUNK(BUF)                                                                 \
    {                                                                                       \
        float4 *a_ = lds + (BUF) * STAGE;                                                   \
        _Pragma("unroll") for (int i = 0; i < NI; ++i) {                                    \
            const int r_ = sr0 + RP * i;                                                    \
            a_[r_ * R4 + (sc ^ swz<KC>(r_))] = ra[i];                                       \
        }                                                                                   \
        _Pragma("unroll") for (int i = 0; i < NB; ++i) {                                    \
            const int r_ = sr0 + RP * i;                                                    \
            a_[(TM + r_) * R4 + (sc ^ swz<KC>(r_))] = rb[i];                                \
        }                                                                                   \
    }
    // STAGES == 1: one stage per workgroup, the next chunk stored between two
    // barriers; STAGES == 2: double-buffered, one barrier per chunk.  Either way
    // two workgroups share a CU, so one's store phase overlaps the other's MFMAs.
    {
        float4 ra[NI], rb[NB];
        VD_LOAD_CHUNK(0)
        VD_STORE_CHUNK(0)
    }
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
        const int buf = STAGES == 2 ? (ch & 1) : 0;
        const int nxt = ch + 1 < nchunks ? ch + 1 : ch;
        float4 ra[NI], rb[NB];
        VD_LOAD_CHUNK(nxt)
        // keep the next chunk's loads here, a whole chunk of MFMAs ahead of their
        // use (the scheduler would otherwise sink them next to the LDS stores)
        __builtin_amdgcn_sched_barrier(0);
        const float4 *a = lds + buf * STAGE;
        const float4 *b = a + TM * R4;
        // fragments of block kb + 1 are read while block kb's MFMAs run
        float4 pf[WTP], wf[WTC];
#pragma unroll
        for (int t = 0; t < WTP; ++t) pf[t] = a[(pw0 + 16 * t + j) * R4 + (q ^ swz<KC>(j))];
#pragma unroll
        for (int t = 0; t < WTC; ++t) wf[t] = b[(cw0 + 16 * t + j) * R4 + (q ^ swz<KC>(j))];
#pragma unroll
        for (int kb = 0; kb < KC / 16; ++kb) {
            float4 pn[WTP], wn[WTC];
            if (kb + 1 < KC / 16) {
                const int c = ((kb + 1) * 4 + q) ^ swz<KC>(j);
#pragma unroll
                for (int t = 0; t < WTP; ++t) pn[t] = a[(pw0 + 16 * t + j) * R4 + c];
#pragma unroll
                for (int t = 0; t < WTC; ++t) wn[t] = b[(cw0 + 16 * t + j) * R4 + c];
            }
            // component-major: 16 independent accumulators between two uses of one
#define VD_MF(COMP)                                                                         \
    _Pragma("unroll") for (int tc = 0; tc < WTC; ++tc)                                      \
        _Pragma("unroll") for (int tp = 0; tp < WTP; ++tp) acc[tc][tp] =                    \
            __builtin_amdgcn_mfma_f32_16x16x4f32(wf[tc].COMP, pf[tp].COMP, acc[tc][tp], 0, 0, 0);
            VD_MF(x)
            VD_MF(y)
            VD_MF(z)
            VD_MF(w)
#undef VD_MF
            if (kb + 1 < KC / 16) {
#pragma unroll
                for (int t = 0; t < WTP; ++t) pf[t] = pn[t];
#pragma unroll
                for (int t = 0; t < WTC; ++t) wf[t] = wn[t];
            }
        }
        if (STAGES == 1) __syncthreads();  // every wave is done reading the stage
        VD_STORE_CHUNK(STAGES == 2 ? (buf ^ 1) : 0)
        __syncthreads();  // the next chunk is visible
    }
#undef VD_LOAD_CHUNK
#undef VD_STORE_CHUNK
    // epilogue: lane (j, q), tile (tc, tp) holds channels n0 + cw0 + 16 tc + 4 q .. + 3
    // of pixel m0 + pw0 + 16 tp + j
#pragma unroll
    for (int tc = 0; tc < WTC; ++tc) {
        const int co = n0 + cw0 + 16 * tc + 4 * q;
        const float4 bv = bias ? *reinterpret_cast<const float4 *>(bias + co)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int tp = 0; tp < WTP; ++tp) {
            const int64_t m = m0 + pw0 + 16 * tp + j;
            if (m >= M) continue;
            float4 o = make_float4(acc[tc][tp][0] + bv.x, acc[tc][tp][1] + bv.y,
                                   acc[tc][tp][2] + bv.z, acc[tc][tp][3] + bv.w);
            if (RELU) {
                o.x = fmaxf(o.x, 0.f);
                o.y = fmaxf(o.y, 0.f);
                o.z = fmaxf(o.z, 0.f);
                o.w = fmaxf(o.w, 0.f);
            }
            *reinterpret_cast<float4 *>(Y + m * Cout + co) = o;
        }
    }
}

// The dynamic-LDS opt-in (> 64 KiB) once per kernel instance, not per launch.
bool allow_lds(const void *kern, size_t lds) {
    static std::mutex mu;
    static std::set<const void *> done;
    std::lock_guard<std::mutex> lk(mu);
    if (done.count(kern)) return true;
    if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
        return false;
    done.insert(kern);
    return true;
}

}  // namespace

bool conv3x3_mfma_supported(int C, int Cout) {
    return C % 64 == 0 && C >= 64 && (Cout % kTN == 0 || Cout == 64);
}

int launch_conv3x3_mfma(const float *X, int N, int H, int W, int C, const float *W2, int Cout,
                        const float *bias, int relu, float *Y, hipStream_t s) {
    const int64_t M = (int64_t)N * H * W;
    if (M == 0) return VD_OK;
    if (!conv3x3_mfma_supported(C, Cout)) return VD_ERR_SHAPE;
    if (M * C * 4 >= 0x7ffffff0ll || (int64_t)Cout * 9 * C * 4 >= 0x7ffffff0ll)
        return VD_ERR_SHAPE;  // 32-bit buffer offsets
    const bool narrow = Cout == 64;  // 256 x 64 tiles (res2's 64-channel conv2)
    // mid-size shapes (fewer than 8 rounds of 128 x 128 tiles over 512 slots):
    // 64 x 128 tiles, three workgroups per CU
    const char *em = getenv("VOSDET_CONV3X3_MID");
    const int64_t big_tiles = (M + kTM - 1) / kTM * (Cout / kTN);
    const bool mid = !narrow && em && atoi(em) != 0 && big_tiles < 4096;  // opt-in (A/B)
    const int tm = narrow ? 256 : (mid ? 64 : kTM), tn = narrow ? 64 : kTN;
    const int64_t mtiles = (M + tm - 1) / tm;
    const int64_t blocks = (mtiles + 7) / 8 * 8 * (Cout / tn);
    if (blocks > 0x7fffffff) return VD_ERR_SHAPE;
    // variant (profiles/r02c/README.md): 6 (default) = K chunk 32, one 32 KiB stage,
    // THREE workgroups per CU -- while one stores its next chunk between its two
    // barriers, two others keep the MFMA pipes fed (0.87 of peak at P2); 1 = K chunk
    // 64, one 64 KiB stage, two per CU (0.84); 2 = K chunk 32 double-buffered, two
    // per CU (0.84).  Four per CU spills (0.69); one double-buffered per CU 0.73;
    // s_setprio over the MFMA phase cost 1-4 %.
    const char *e = getenv("VOSDET_CONV3X3_VARIANT");
    const int v = e ? atoi(e) : 6;
    void (*kern)(const float *, int, int, int, int, const float *, int, const float *, float *,
                 int);
    size_t lds;
    if (narrow) {
        kern = relu ? conv3x3_mfma_kernel<true, 64, 1, 256, 64>
                    : conv3x3_mfma_kernel<false, 64, 1, 256, 64>;
        lds = (size_t)(256 + 64) * 16 * sizeof(float4);  // 80 KiB
    } else if (mid) {
        kern = relu ? conv3x3_mfma_kernel<true, 64, 1, 64, 128, 2, 4, 3>
                    : conv3x3_mfma_kernel<false, 64, 1, 64, 128, 2, 4, 3>;
        lds = (size_t)(64 + 128) * 16 * sizeof(float4);  // 48 KiB: three per CU
    } else if (v == 6) {  // K chunk 32, one 32 KiB stage, three workgroups per CU
        kern = relu ? conv3x3_mfma_kernel<true, 32, 1, kTM, kTN, 4, 4, 3>
                    : conv3x3_mfma_kernel<false, 32, 1, kTM, kTN, 4, 4, 3>;
        lds = (size_t)(kTM + kTN) * 8 * sizeof(float4);
    } else if (v == 2) {
        kern = relu ? conv3x3_mfma_kernel<true, 32, 2> : conv3x3_mfma_kernel<false, 32, 2>;
        lds = 2 * (size_t)(kTM + kTN) * 8 * sizeof(float4);
    } else {
        kern = relu ? conv3x3_mfma_kernel<true, 64, 1> : conv3x3_mfma_kernel<false, 64, 1>;
        lds = (size_t)(kTM + kTN) * 16 * sizeof(float4);
    }
    if (!allow_lds(reinterpret_cast<const void *>(kern), lds)) return VD_ERR_LAUNCH;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), lds, s, X, N, H, W, C, W2, Cout,
                       bias, Y, (int)mtiles);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
