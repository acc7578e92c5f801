// RoIAlign forward, LDS-staged (variant 20): the product FPN kernel.
//
// Reference semantics: lib/modeling/roi_xfrom/roi_align/src/roi_align_kernel.cu
//   bilinear_interpolate :16-63, ROIAlignForward :65-121 (per output element: the
//   grid of SR x SR samples, w1*v1 + w2*v2 + w3*v3 + w4*v4 per sample, iy-major
//   accumulation, final / count).  Every output element here is computed with
//   exactly that arithmetic (no re-association, no FMA contraction), so the
//   result is bit-identical to the C restatement oracle/roi_ops.c and to the
//   row kernel of roi_align.hip (variant 3).
//
// Layout: NHWC pyramid (a pixel = C = 256 fp32 = 1 KiB), output [R][P][P][C].
//
// Schedule.  One persistent workgroup per CU (8 waves) walks its share of the
// XCD-dealt RoI order (ops.xcd_roi_order: the 32 workgroups of an XCD work on
// 32 spatially consecutive RoIs of one image at a time, so their footprints
// meet in that XCD's L2).  A RoI is cut into ITEMS = (band of output rows,
// 32-channel slice): the band's WINDOW -- the pixel rows its samples tap x the
// RoI's tap columns, 128 B per pixel for the slice -- is copied HBM/L2 -> LDS
// by LDS-DMA (global_load_lds_dwordx4: one wave instruction moves 8 pixels'
// slices, no VGPR round trip), three windows in a ring: while the workgroup
// computes item i from LDS, the DMA of items i+1 and i+2 is in flight.  One
// barrier per item; the DMA is issued in inline asm so the compiler does not
// drain it (hipcc waits vmcnt(0) before LDS reads that may alias an LDS-DMA it
// knows of), and each wave retires exactly its own copies of item i with a
// counted vmcnt(N) before that barrier (N = the ops it issued after them).
//
// Compute: a wave takes one output row of the band (P = 7; two half rows for
// P = 14); lane = (bin pw, 4-channel quad q), 8 lanes per bin, 7-8 bins per
// wave.  The row's y taps are wave-uniform, the bin's x taps per lane; every
// tap is one ds_read_b128 of the window.  Each pixel of the RoI's footprint
// crosses the CU once per slice (band splits re-read at most the shared tap
// rows), against ~1.27x that for the register-gather kernel that re-loads the
// tap rows shared by adjacent output rows.
//
// A RoI whose single output row needs more window pixels than a buffer holds
// (> kCapPx; e.g. a box spanning the whole frame at P2) is computed straight
// from global memory by the same code (direct mode), so any box is accepted.
#include <stdlib.h>

#include "common.hpp"
#include "roi_geom.hpp"
#include "vosdet_internal.hpp"

namespace vd {
namespace ralds {

constexpr int kC = 256;                 // channels (the FPN dimension)
constexpr int kG = 32;                  // channels per item (slice)
constexpr int kNS = kC / kG;            // slices per RoI
constexpr int kWaves = 8;               // waves per workgroup
constexpr int kBuf = 3;                 // window ring depth
constexpr int kCapPx = 416;             // pixels per window buffer (multiple of 8)
constexpr int kSlotB = kG * 4;          // bytes per pixel slice
constexpr int kBufB = kCapPx * kSlotB;  // 53,248 B; 3 buffers = 156 KiB of the CU's 160

// RoI state shared by the fill and compute cursors (wave-uniform values).
struct Roi {
    int r;               // RoI index (< 0: past the end of this workgroup's walk)
    const float *img;    // its image in its level (NHWC)
    int H, W;
    float sw, sh, bw, bh;
    int cx0, ncols;      // tap columns of the whole RoI (ncols 0: no sample in range)
    int direct;          // 1: an output row's window exceeds a buffer
};

struct Cursor {
    Roi g;
    int t;               // RoI ordinal in this workgroup's walk
    int a, b;            // output rows [a, b) of the current item
    int wy0, nrows;      // window rows of the band
    int s;               // channel slice
};

// Sample row (ph, iy): the reference's y and its taps (roi_align_kernel.cu:19-48).
template <int P, int SR>
__device__ __forceinline__ float sample_y(const Roi &g, int ph, int iy) {
    return g.sh + ph * g.bh + (iy + .5f) * g.bh / SR;
}
template <int P, int SR>
__device__ __forceinline__ float sample_x(const Roi &g, int pw, int ix) {
    return g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
}
// Clamped taps of one coordinate; returns false for a sample outside [-1, N].
__device__ __forceinline__ bool taps1(float v, int N, int &lo, int &hi, float &l) {
    const bool ok = !(v < -1.0f || v > (float)N);
    if (v <= 0) v = 0;
    lo = (int)v;
    if (lo >= N - 1) {
        hi = lo = N - 1;
        v = (float)lo;
    } else {
        hi = lo + 1;
    }
    l = v - lo;
    return ok;
}

// Window rows [lo, hi] of output row ph (false: no sample of the row in range).
template <int P, int SR>
__device__ __forceinline__ bool row_span(const Roi &g, int ph, int &lo, int &hi) {
    bool any = false;
#pragma unroll
    for (int iy = 0; iy < SR; ++iy) {
        int yl, yh;
        float ly;
        if (taps1(sample_y<P, SR>(g, ph, iy), g.H, yl, yh, ly)) {
            if (!any) lo = yl;
            hi = yh;  // samples are non-decreasing in (ph, iy)
            any = true;
        }
    }
    return any;
}

template <int P, int SR>
__device__ __forceinline__ void load_roi(Roi &g, const FpnLevels &fa, const float *__restrict__ rois,
                                         const int *__restrict__ roi_level,
                                         const int *__restrict__ roi_order, int p) {
    if (p >= fa.R) {
        g.r = -1;
        return;
    }
    int r = roi_order ? roi_order[p] : p;
    r = __builtin_amdgcn_readfirstlane(r);
    if (r < 0 || r >= fa.R) {  // malformed schedule entry: skipped (writes nothing)
        g.r = -2;
        return;
    }
    g.r = r;
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom rg = roi_geom(fa, kC, rois + (int64_t)r * 5, li, P, P, SR);
    g.img = rg.feat;
    g.H = rg.H;
    g.W = rg.W;
    g.sw = rg.sw;
    g.sh = rg.sh;
    g.bw = rg.bw;
    g.bh = rg.bh;
    // tap columns: x samples are non-decreasing in (pw, ix), so the window runs
    // from the first in-range sample's low tap to the last one's high tap
    int c0 = 0, c1 = -1;
    bool any = false;
    for (int j = 0; j < P * SR; ++j) {
        int xl, xh;
        float lx;
        if (taps1(sample_x<P, SR>(g, j / SR, j % SR), g.W, xl, xh, lx)) {
            if (!any) c0 = xl;
            c1 = xh;
            any = true;
        }
    }
    g.cx0 = c0;
    g.ncols = any ? c1 - c0 + 1 : 0;
    g.direct = 0;
    if (g.ncols > 0) {
        for (int ph = 0; ph < P; ++ph) {
            int lo, hi;
            if (row_span<P, SR>(g, ph, lo, hi) && (hi - lo + 1) * g.ncols > kCapPx) g.direct = 1;
        }
    }
}

// Band [a, b) starting at a: as many output rows as fit one buffer.
template <int P, int SR>
__device__ __forceinline__ void make_band(Cursor &c) {
    const Roi &g = c.g;
    int lo = 0, hi = -1;
    bool any = false;
    int b = c.a;
    while (b < P) {
        int l2, h2;
        if (g.direct || g.ncols == 0 || !row_span<P, SR>(g, b, l2, h2)) {
            ++b;  // no window rows needed for this output row
            continue;
        }
        const int nlo = any ? lo : l2;
        if (any && (h2 - nlo + 1) * g.ncols > kCapPx) break;
        lo = nlo;
        hi = h2;
        any = true;
        ++b;
    }
    c.b = b;
    c.wy0 = lo;
    c.nrows = any ? hi - lo + 1 : 0;
}

template <int P, int SR>
__device__ __forceinline__ void cursor_roi(Cursor &c, const FpnLevels &fa, const float *rois,
                                           const int *roi_level, const int *roi_order,
                                           int nblk) {
    for (;;) {
        load_roi<P, SR>(c.g, fa, rois, roi_level, roi_order, blockIdx.x + nblk * c.t);
        if (c.g.r != -2 && !(c.g.r >= 0 && c.g.direct)) break;
        ++c.t;  // malformed entry, or a direct-mode RoI (the second kernel's): next position
    }
    c.a = 0;
    c.s = 0;
    if (c.g.r >= 0) make_band<P, SR>(c);
}

template <int P, int SR>
__device__ __forceinline__ void cursor_next(Cursor &c, const FpnLevels &fa, const float *rois,
                                            const int *roi_level, const int *roi_order,
                                            int nblk) {
    if (++c.s < kNS) return;
    c.s = 0;
    c.a = c.b;
    if (c.a < P) {
        make_band<P, SR>(c);
        return;
    }
    ++c.t;
    cursor_roi<P, SR>(c, fa, rois, roi_level, roi_order, nblk);
}

// One LDS-DMA wave instruction: 64 lanes x 16 B from per-lane global addresses
// into 1 KiB of LDS at the wave-uniform byte address `lds` (lane-linear).
// Inline asm so that hipcc neither counts nor drains it (see the file comment);
// M0 carries the LDS base and is restored within the statement.
__device__ __forceinline__ void dma_1k(const float *src, uint32_t lds) {
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

// Wait until at most n of this wave's vector-memory ops are outstanding, retire
// its LDS reads, then the workgroup barrier.  n is wave-uniform.
__device__ __forceinline__ void wait_barrier(int n) {
#define VD_WB(k)                                                                   \
    case k:                                                                        \
        asm volatile("s_waitcnt vmcnt(" #k ") lgkmcnt(0)\n\ts_barrier" ::: "memory"); \
        break;
    switch (n) {
        VD_WB(1) VD_WB(2) VD_WB(3) VD_WB(4) VD_WB(5) VD_WB(6) VD_WB(7) VD_WB(8) VD_WB(9)
        VD_WB(10) VD_WB(11) VD_WB(12) VD_WB(13) VD_WB(14) VD_WB(15) VD_WB(16) VD_WB(17)
        VD_WB(18) VD_WB(19) VD_WB(20)
        default:
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            break;
    }
#undef VD_WB
}

// Issue this wave's share of item c's window copy into buffer `buf`; returns
// the number of DMA instructions issued.
__device__ __forceinline__ int fill(const Cursor &c, uint32_t lds_base, int buf, int wave,
                                    int lane) {
    if (c.g.r < 0 || c.g.direct) return 0;
    const int npx = c.nrows * c.g.ncols;
    const int npc = (npx + 7) >> 3;
    if (wave >= npc) return 0;
    const float inv = 1.f / (float)c.g.ncols;
    const float *src0 = c.g.img + c.s * kG + (lane & 7) * 4;
    const uint32_t dst0 = lds_base + (uint32_t)buf * kBufB;
    int n = 0;
    for (int pc = wave; pc < npc; pc += kWaves) {
        int pix = pc * 8 + (lane >> 3);
        pix = pix < npx ? pix : npx - 1;
        // pix / ncols exactly: the fraction (x + 0.5) / ncols stays >= 1/(2 ncols)
        // away from an integer, far more than the float error at these sizes
        const int yy = (int)(((float)pix + 0.5f) * inv);
        const int xx = pix - yy * c.g.ncols;
        const float *src = src0 + ((int64_t)(c.wy0 + yy) * c.g.W + (c.g.cx0 + xx)) * kC;
        dma_1k(src, __builtin_amdgcn_readfirstlane(dst0 + (uint32_t)pc * 1024u));
        ++n;
    }
    return n;
}

template <bool NT>
__device__ __forceinline__ void store4(float *dst, float4 v) {
    if (NT) {
        vf4 u = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(u, reinterpret_cast<vf4 *>(dst));
    } else {
        *reinterpret_cast<float4 *>(dst) = v;
    }
}

__device__ __forceinline__ float4 bil4(float w1, float w2, float w3, float w4, float4 a,
                                       float4 b, float4 c, float4 d) {
    // w1*v1 + w2*v2 + w3*v3 + w4*v4, left to right (roi_align_kernel.cu:60)
    return make_float4(w1 * a.x + w2 * b.x + w3 * c.x + w4 * d.x,
                       w1 * a.y + w2 * b.y + w3 * c.y + w4 * d.y,
                       w1 * a.z + w2 * b.z + w3 * c.z + w4 * d.z,
                       w1 * a.w + w2 * b.w + w3 * c.w + w4 * d.w);
}

typedef __attribute__((address_space(3))) const vf4 lds_f4;

__device__ __forceinline__ float4 lds4(lds_f4 *p) {
    const vf4 v = *p;
    return make_float4(v.x, v.y, v.z, v.w);
}

// Compute item c from window buffer `win` (float4 units): this wave's tasks;
// returns the number of output stores issued.
template <int P, int SR, bool NT, bool DIRECT>
__device__ __forceinline__ int compute(const Cursor &c, lds_f4 *win, int wave, int lane,
                                       float *__restrict__ out, int waves = kWaves) {
    if (c.g.r < 0) return 0;
    constexpr int TPR = (P + 7) / 8;  // tasks (8-bin runs) per output row
    const int ntask = (c.b - c.a) * TPR;
    const Roi &g = c.g;
    const int q = lane & 7;
    int n = 0;
    for (int task = wave; task < ntask; task += waves) {
        const int ph = c.a + task / TPR;
        const int pw_raw = (task % TPR) * 8 + (lane >> 3);
        const bool lane_on = pw_raw < P;
        const int pw = lane_on ? pw_raw : P - 1;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int iy = 0; iy < SR; ++iy) {
            int yl, yh;
            float ly;
            const bool vy = taps1(sample_y<P, SR>(g, ph, iy), g.H, yl, yh, ly);
            const float hy = 1.f - ly;
            int rl = 0, rh = 0;  // window row offsets (pixels)
            if (!DIRECT) {
                const int mr = c.nrows > 0 ? c.nrows - 1 : 0;
                rl = min(max(yl - c.wy0, 0), mr) * g.ncols;
                rh = min(max(yh - c.wy0, 0), mr) * g.ncols;
            }
#pragma unroll
            for (int ix = 0; ix < SR; ++ix) {
                int xl, xh;
                float lx;
                const bool vx = taps1(sample_x<P, SR>(g, pw, ix), g.W, xl, xh, lx);
                const float hx = 1.f - lx;
                float4 v1, v2, v3, v4;
                if (!DIRECT) {
                    const int mc = g.ncols > 0 ? g.ncols - 1 : 0;
                    const int cl = min(max(xl - g.cx0, 0), mc), ch = min(max(xh - g.cx0, 0), mc);
                    v1 = lds4(win + (rl + cl) * 8 + q);
                    v2 = lds4(win + (rl + ch) * 8 + q);
                    v3 = lds4(win + (rh + cl) * 8 + q);
                    v4 = lds4(win + (rh + ch) * 8 + q);
                } else {
                    const float *base = g.img + c.s * kG + q * 4;
                    v1 = ld4(base + ((int64_t)yl * g.W + xl) * kC);
                    v2 = ld4(base + ((int64_t)yl * g.W + xh) * kC);
                    v3 = ld4(base + ((int64_t)yh * g.W + xl) * kC);
                    v4 = ld4(base + ((int64_t)yh * g.W + xh) * kC);
                }
                const float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
                float4 val = bil4(w1, w2, w3, w4, v1, v2, v3, v4);
                if (!(vy && vx)) val = make_float4(0.f, 0.f, 0.f, 0.f);
                acc.x += val.x;
                acc.y += val.y;
                acc.z += val.z;
                acc.w += val.w;
            }
        }
        const float count = (float)(SR * SR);
        acc = make_float4(acc.x / count, acc.y / count, acc.z / count, acc.w / count);
        if (lane_on)
            store4<NT>(out + (((int64_t)g.r * P + ph) * P + pw) * kC + c.s * kG + q * 4, acc);
        ++n;
    }
    return n;
}

template <int P, int SR, bool NT>
__global__ __launch_bounds__(kWaves * 64) void roi_align_fpn_lds_kernel(
    FpnLevels fa, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) float4 lds[kBuf * kBufB / 16];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int nblk = gridDim.x;
    const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
    Cursor F, K;
    F.t = 0;
    cursor_roi<P, SR>(F, fa, rois, roi_level, roi_order, nblk);
    K = F;
    // prologue: windows of items 0 and 1
    fill(F, lds_base, 0, wave, lane);
    cursor_next<P, SR>(F, fa, rois, roi_level, roi_order, nblk);
    int d_next = fill(F, lds_base, 1, wave, lane);  // D(i+1)
    cursor_next<P, SR>(F, fa, rois, roi_level, roi_order, nblk);
    int s_prev2 = 0, s_prev = 0;                    // S(i-2), S(i-1)
    for (int i = 0; K.g.r >= 0; ++i) {
        // retire D(i): younger ops are S(i-2), D(i+1), S(i-1)
        wait_barrier(s_prev2 + d_next + s_prev);
        const int d2 = fill(F, lds_base, (i + 2) % kBuf, wave, lane);
        cursor_next<P, SR>(F, fa, rois, roi_level, roi_order, nblk);
        const int s_i = compute<P, SR, NT, false>(
            K, (lds_f4 *)lds + (i % kBuf) * (kBufB / 16), wave, lane, out);
        cursor_next<P, SR>(K, fa, rois, roi_level, roi_order, nblk);
        s_prev2 = s_prev;
        s_prev = s_i;
        d_next = d2;
    }
    // no LDS-DMA may land after the workgroup's LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// RoIs in direct mode (skipped by the kernel above): one wave per RoI, every
// (output row, slice) item computed from global memory with the same arithmetic.
template <int P, int SR, bool NT>
__global__ __launch_bounds__(256) void roi_align_fpn_direct_kernel(
    FpnLevels fa, const float *__restrict__ rois, const int *__restrict__ roi_level,
    float *__restrict__ out) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= fa.R) return;
    Cursor c;
    load_roi<P, SR>(c.g, fa, rois, roi_level, nullptr, r);
    if (c.g.r < 0 || !c.g.direct) return;
    c.a = 0;
    c.b = P;
    c.wy0 = 0;
    c.nrows = 0;
    for (c.s = 0; c.s < kNS; ++c.s)
        compute<P, SR, NT, true>(c, nullptr, 0, threadIdx.x & 63, out, 1);
}

static int num_cus() {
    static int n = 0;
    if (n == 0) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            v > 0)
            n = v;
        else
            n = 256;
    }
    return n;
}

}  // namespace ralds

// C = 256, sr = 2, P in {7, 14}, NHWC out; VD_ERR_SHAPE otherwise (the caller
// falls back to the register-gather kernels).
int launch_roi_align_fpn_lds(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                             const int *order, int R, int P, int sr, float *out, hipStream_t s) {
    using namespace ralds;
    if (C != kC || sr != 2 || (P != 7 && P != 14)) return VD_ERR_SHAPE;
    for (int l = 0; l < fa.L; ++l)  // 32-bit window arithmetic per image
        if ((int64_t)fa.H[l] * fa.W[l] >= (1ll << 23)) return VD_ERR_SHAPE;
    if (R == 0) return VD_OK;
    int nblk = num_cus();
    nblk = nblk / 8 * 8;  // block b -> XCD b % 8: whole XCD groups
    if (nblk < 8) nblk = 8;
    const int per = (R + nblk - 1) / nblk;
    if (per < 2 && R < nblk) nblk = (R + 7) / 8 * 8;  // small launches: fewer workgroups
    const int ndir = (R + 3) / 4;
    if (P == 7) {
        hipLaunchKernelGGL((roi_align_fpn_lds_kernel<7, 2, true>), dim3(nblk), dim3(kWaves * 64),
                           0, s, fa, rois, lvl, order, out);
        hipLaunchKernelGGL((roi_align_fpn_direct_kernel<7, 2, true>), dim3(ndir), dim3(256), 0, s,
                           fa, rois, lvl, out);
    } else {
        hipLaunchKernelGGL((roi_align_fpn_lds_kernel<14, 2, true>), dim3(nblk),
                           dim3(kWaves * 64), 0, s, fa, rois, lvl, order, out);
        hipLaunchKernelGGL((roi_align_fpn_direct_kernel<14, 2, true>), dim3(ndir), dim3(256), 0,
                           s, fa, rois, lvl, out);
    }
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
