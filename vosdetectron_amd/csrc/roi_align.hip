// RoIAlign (Caffe2-exact) for gfx950.
//
// Reference semantics: lib/modeling/roi_xfrom/roi_align/src/roi_align_kernel.cu
//   bilinear_interpolate :16-63, ROIAlignForward :65-121, ROIAlignBackward :195-270.
//
// Two forward layouts:
//  * NCHW (the reference's tensor layout, used by the drop-in RoIAlignFunction
//    on arbitrary caller tensors): one lane per output element, the reference's
//    decomposition, kept as the compatibility path.
//  * NHWC multi-level FPN (the product path): one launch for every RoI of every
//    FPN level on the NHWC pyramid (one 1 KiB coalesced wave load per pixel,
//    lane = 4 channels).  The default kernel (roi_align_fpn_nhwc_sep_kernel,
//    variant 8) factors the bilinear sampling into a row pass and a column pass
//    so each pixel is fetched ~once per output row; it re-associates the sums,
//    so it holds the reference to 1e-4 (north_star's RoIAlign tolerance).  The
//    row kernel (variant 3, VOSDET_ROIALIGN_VARIANT=3) keeps the reference's
//    per-sample order -- sample positions, weights, w1*v1+w2*v2+w3*v3+w4*v4,
//    iy-major accumulation, final /count, no FMA contraction -- and is
//    bit-identical to the C restatement in oracle/roi_ops.c, as are the NCHW
//    kernels.
#include <stdlib.h>

#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

// --------------------------------------------------------------------------
// NCHW forward: one thread per output element (n, c, ph, pw).
// --------------------------------------------------------------------------
__device__ __forceinline__ float bilinear_nchw(const float *__restrict__ plane, int H, int W,
                                               float y, float x) {
    if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) return 0.f;
    if (y <= 0) y = 0;
    if (x <= 0) x = 0;
    int yl = (int)y, xl = (int)x, yh, xh;
    if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
    if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
    float ly = y - yl, lx = x - xl;
    float hy = 1.f - ly, hx = 1.f - lx;
    float v1 = plane[yl * W + xl], v2 = plane[yl * W + xh];
    float v3 = plane[yh * W + xl], v4 = plane[yh * W + xh];
    float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
    return (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4);
}

__global__ __launch_bounds__(256) void roi_align_fwd_nchw_kernel(
    int64_t nthreads, const float *__restrict__ feat, float scale, int H, int W, int C,
    int PH, int PW, int sr, const float *__restrict__ rois, float *__restrict__ out) {
    for (int64_t index = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; index < nthreads;
         index += (int64_t)blockDim.x * gridDim.x) {
        int pw = (int)(index % PW);
        int ph = (int)((index / PW) % PH);
        int c = (int)((index / PW / PH) % C);
        int64_t n = index / PW / PH / C;
        const float *r = rois + n * 5;
        int b = (int)r[0];
        float sw = r[1] * scale, sh = r[2] * scale, ew = r[3] * scale, eh = r[4] * scale;
        float rw = fmaxf(ew - sw, 1.f), rh = fmaxf(eh - sh, 1.f);
        float bh = rh / PH, bw = rw / PW;
        const float *plane = feat + ((int64_t)b * C + c) * (int64_t)H * W;
        int gh = sr > 0 ? sr : (int)ceilf(rh / PH);
        int gw = sr > 0 ? sr : (int)ceilf(rw / PW);
        const float count = (float)(gh * gw);
        float acc = 0.f;
        for (int iy = 0; iy < gh; iy++) {
            const float y = sh + ph * bh + (iy + .5f) * bh / gh;
            for (int ix = 0; ix < gw; ix++) {
                const float x = sw + pw * bw + (ix + .5f) * bw / gw;
                acc += bilinear_nchw(plane, H, W, y, x);
            }
        }
        acc /= count;
        out[index] = acc;
    }
}

// --------------------------------------------------------------------------
// NCHW backward (training path): reference decomposition with f32 atomics into
// the zero-filled bottom_diff (sum order is arrival order, as in the reference).
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void roi_align_bwd_nchw_kernel(
    int64_t nthreads, const float *__restrict__ top_diff, float scale, int H, int W, int C,
    int PH, int PW, int sr, const float *__restrict__ rois, float *__restrict__ bottom_diff) {
    for (int64_t index = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; index < nthreads;
         index += (int64_t)blockDim.x * gridDim.x) {
        int pw = (int)(index % PW);
        int ph = (int)((index / PW) % PH);
        int c = (int)((index / PW / PH) % C);
        int64_t n = index / PW / PH / C;
        const float *r = rois + n * 5;
        int b = (int)r[0];
        float sw = r[1] * scale, sh = r[2] * scale, ew = r[3] * scale, eh = r[4] * scale;
        float rw = fmaxf(ew - sw, 1.f), rh = fmaxf(eh - sh, 1.f);
        float bh = rh / PH, bw = rw / PW;
        float *plane = bottom_diff + ((int64_t)b * C + c) * (int64_t)H * W;
        const float g = top_diff[index];
        int gh = sr > 0 ? sr : (int)ceilf(rh / PH);
        int gw = sr > 0 ? sr : (int)ceilf(rw / PW);
        const float count = (float)(gh * gw);
        for (int iy = 0; iy < gh; iy++) {
            const float y0 = sh + ph * bh + (iy + .5f) * bh / gh;
            for (int ix = 0; ix < gw; ix++) {
                float y = y0;
                float x = sw + pw * bw + (ix + .5f) * bw / gw;
                if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) continue;
                if (y <= 0) y = 0;
                if (x <= 0) x = 0;
                int yl = (int)y, xl = (int)x, yh, xh;
                if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
                if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
                float ly = y - yl, lx = x - xl;
                float hy = 1.f - ly, hx = 1.f - lx;
                float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
                atomicAdd(plane + yl * W + xl, g * w1 / count);
                atomicAdd(plane + yl * W + xh, g * w2 / count);
                atomicAdd(plane + yh * W + xl, g * w3 / count);
                atomicAdd(plane + yh * W + xh, g * w4 / count);
            }
        }
    }
}

// --------------------------------------------------------------------------
// NHWC multi-level forward.
// --------------------------------------------------------------------------
struct RoiGeom {
    const float *feat;  // this RoI's image base in its level
    int H, W;
    float sw, sh, bw, bh;
    int gh, gw;
    float count;
};

__device__ __forceinline__ RoiGeom roi_geom(const FpnLevels &fa, int C, const float *roi,
                                            int li, int PH, int PW, int sr) {
    RoiGeom g;
    g.H = fa.H[li];
    g.W = fa.W[li];
    const float scale = fa.scale[li];
    const int b = (int)roi[0];
    g.feat = fa.feat[li] + (int64_t)b * g.H * g.W * C;
    g.sw = roi[1] * scale;
    g.sh = roi[2] * scale;
    float ew = roi[3] * scale, eh = roi[4] * scale;
    float rw = fmaxf(ew - g.sw, 1.f), rh = fmaxf(eh - g.sh, 1.f);
    g.bh = rh / PH;
    g.bw = rw / PW;
    g.gh = sr > 0 ? sr : (int)ceilf(rh / PH);
    g.gw = sr > 0 ? sr : (int)ceilf(rw / PW);
    g.count = (float)(g.gh * g.gw);
    return g;
}

__device__ __forceinline__ void bilerp_acc(float4 &acc, float w1, float w2, float w3, float w4,
                                           const float4 &a, const float4 &b, const float4 &c,
                                           const float4 &d) {
    acc.x += (w1 * a.x + w2 * b.x + w3 * c.x + w4 * d.x);
    acc.y += (w1 * a.y + w2 * b.y + w3 * c.y + w4 * d.y);
    acc.z += (w1 * a.z + w2 * b.z + w3 * c.z + w4 * d.z);
    acc.w += (w1 * a.w + w2 * b.w + w3 * c.w + w4 * d.w);
}

__device__ __forceinline__ float4 ld4(const float *p) {
    return *reinterpret_cast<const float4 *>(p);
}

// One wave computes output row `ph` for 256 channels starting at c0 (lane owns
// c0 + 4*lane .. +3); acc[P] lives in registers.
template <int P>
__device__ __forceinline__ void nhwc_row(const RoiGeom &g, int C, int ph, int cbase, bool active,
                                         float4 (&acc)[P]) {
#pragma unroll
    for (int pw = 0; pw < P; ++pw) acc[pw] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int H = g.H, W = g.W;
    const int64_t rowstride = (int64_t)W * C;
    for (int iy = 0; iy < g.gh; ++iy) {
        float y = g.sh + ph * g.bh + (iy + .5f) * g.bh / g.gh;
        if (y < -1.0f || y > (float)H) continue;  // every x of this sample row reads 0
        if (y <= 0) y = 0;
        int yl = (int)y, yh;
        if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
        const float ly = y - yl, hy = 1.f - ly;
        const float *top = g.feat + yl * rowstride + cbase;
        const float *bot = g.feat + yh * rowstride + cbase;
        int cl = -1, ch = -1;  // columns currently held in (tl,bl) / (tr,br)
        float4 tl = make_float4(0.f, 0.f, 0.f, 0.f), tr = tl, bl = tl, br = tl;
#pragma unroll
        for (int pw = 0; pw < P; ++pw) {
            for (int ix = 0; ix < g.gw; ++ix) {
                float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / g.gw;
                if (x < -1.0f || x > (float)W) continue;
                if (x <= 0) x = 0;
                int xl = (int)x, xh;
                if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
                const float lx = x - xl, hx = 1.f - lx;
                if (!(xl == cl && xh == ch)) {
                    if (xl == ch) {  // slide right by one column: keep the shared column
                        tl = tr;
                        bl = br;
                    } else if (active) {
                        tl = ld4(top + (int64_t)xl * C);
                        bl = ld4(bot + (int64_t)xl * C);
                    }
                    if (active) {
                        tr = ld4(top + (int64_t)xh * C);
                        br = ld4(bot + (int64_t)xh * C);
                    }
                    cl = xl;
                    ch = xh;
                }
                const float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
                bilerp_acc(acc[pw], w1, w2, w3, w4, tl, tr, bl, br);
            }
        }
    }
}

// Compile-time sampling ratio: every sample of the row is unrolled and
// branch-free (invalid samples are masked with a select, taps clamped in
// range), so the compiler can keep dozens of 1 KiB tap loads in flight per wave
// instead of waiting on each sample's taps.
template <int P, int SR, int D>
__device__ __forceinline__ void nhwc_row_sr(const RoiGeom &g, int C, int ph, int cbase,
                                            float4 (&acc)[P]) {
#pragma unroll
    for (int pw = 0; pw < P; ++pw) acc[pw] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int H = g.H, W = g.W;
    const int64_t rowstride = (int64_t)W * C;
    // x geometry of the row's P*SR samples: identical for every sample row
    int xo_l[P * SR], xo_h[P * SR];
    float lxs[P * SR];
    bool vxs[P * SR];
#pragma unroll
    for (int j = 0; j < P * SR; ++j) {
        const int pw = j / SR, ix = j % SR;
        float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
        vxs[j] = !(x < -1.0f || x > (float)W);
        if (x <= 0) x = 0;
        int xl = (int)x, xh;
        if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
        lxs[j] = x - xl;
        xo_l[j] = xl * C;
        xo_h[j] = xh * C;
    }
    // D - 1 samples' taps (4 x 1 KiB each) are in flight ahead of the math
#pragma unroll
    for (int iy = 0; iy < SR; ++iy) {
        float y = g.sh + ph * g.bh + (iy + .5f) * g.bh / SR;
        if (y < -1.0f || y > (float)H) continue;  // wave-uniform
        if (y <= 0) y = 0;
        int yl = (int)y, yh;
        if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
        const float ly = y - yl, hy = 1.f - ly;
        const float *top = g.feat + yl * rowstride + cbase;
        const float *bot = g.feat + yh * rowstride + cbase;
        float4 buf[D][4];
#pragma unroll
        for (int j = 0; j < D - 1; ++j) {
            buf[j][0] = ld4(top + xo_l[j]);
            buf[j][1] = ld4(top + xo_h[j]);
            buf[j][2] = ld4(bot + xo_l[j]);
            buf[j][3] = ld4(bot + xo_h[j]);
        }
#pragma unroll
        for (int j = 0; j < P * SR; ++j) {
            const int jn = j + D - 1;
            if (jn < P * SR) {
                buf[jn % D][0] = ld4(top + xo_l[jn]);
                buf[jn % D][1] = ld4(top + xo_h[jn]);
                buf[jn % D][2] = ld4(bot + xo_l[jn]);
                buf[jn % D][3] = ld4(bot + xo_h[jn]);
            }
            const float lx = lxs[j], hx = 1.f - lx;
            const float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
            float4 t = acc[j / SR];
            bilerp_acc(t, w1, w2, w3, w4, buf[j % D][0], buf[j % D][1], buf[j % D][2],
                       buf[j % D][3]);
            if (vxs[j]) acc[j / SR] = t;  // out-of-range sample contributes exactly 0
        }
    }
}

// --------------------------------------------------------------------------
// Separable NHWC forward.  Bilinear sampling on a tensor-product grid factors:
//   sum_{iy,ix} [hy hx F(yl,xl) + hy lx F(yl,xh) + ly hx F(yh,xl) + ly lx F(yh,xh)]
//     = sum_ix [hx V(xl) + lx V(xh)],   V(x) = sum_iy [hy F(yl,x) + ly F(yh,x)],
// with out-of-range samples dropping out of either sum.  Per output row the
// 2*SR y taps are merged into distinct pixel rows (usually 2-3), and V(x) is
// computed once per distinct column while the x samples sweep left to right
// (their columns are non-decreasing), so a 1 KiB pixel is fetched ~once per row
// instead of once per tap: ~4x fewer vector-memory instructions than
// nhwc_row_sr, which is what bounds the gather (texture-addresser issue).  Each
// bin is finished and stored before the next starts, so no per-row accumulator
// array is live (low VGPRs, high occupancy).  Rounding differs from the
// reference's per-sample order by a few ulp (north_star's RoIAlign tolerance is
// 1e-4 fp32); the bit-exact kernels above stay selectable.
// --------------------------------------------------------------------------
template <int SR>
struct RowTaps {
    int row[2 * SR];
    float w[2 * SR];
    bool alive[2 * SR];
};

template <int SR>
__device__ __forceinline__ RowTaps<SR> row_taps(const RoiGeom &g, int ph) {
    RowTaps<SR> t;
    const int H = g.H;
#pragma unroll
    for (int iy = 0; iy < SR; ++iy) {
        float y = g.sh + ph * g.bh + (iy + .5f) * g.bh / SR;
        const bool ok = !(y < -1.0f || y > (float)H);
        if (y <= 0) y = 0;
        int yl = (int)y, yh;
        if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
        const float ly = y - yl;
        t.row[2 * iy] = yl;
        t.w[2 * iy] = 1.f - ly;
        t.alive[2 * iy] = ok;
        t.row[2 * iy + 1] = yh;
        t.w[2 * iy + 1] = ly;
        t.alive[2 * iy + 1] = ok;
    }
#pragma unroll
    for (int k = 1; k < 2 * SR; ++k)
#pragma unroll
        for (int k2 = 0; k2 < k; ++k2)
            if (t.alive[k] && t.alive[k2] && t.row[k2] == t.row[k]) {
                t.w[k2] += t.w[k];
                t.alive[k] = false;
            }
    return t;
}

__device__ __forceinline__ float4 fma4(float w, const float4 &a, const float4 &c) {
    return make_float4(fmaf(w, a.x, c.x), fmaf(w, a.y, c.y), fmaf(w, a.z, c.z), fmaf(w, a.w, c.w));
}

template <int SR>
struct TapCol {
    float4 f[2 * SR];
};

template <int SR>
__device__ __forceinline__ TapCol<SR> load_column(const RowTaps<SR> &t, const float *base,
                                                  int64_t rowstride, int64_t xoff) {
    TapCol<SR> c;
#pragma unroll
    for (int k = 0; k < 2 * SR; ++k)
        if (t.alive[k]) c.f[k] = ld4(base + t.row[k] * rowstride + xoff);
    return c;
}

template <int SR, bool FMA>
__device__ __forceinline__ float4 combine_column(const RowTaps<SR> &t, const TapCol<SR> &c) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < 2 * SR; ++k)
        if (t.alive[k]) {
            if (FMA) {
                v = fma4(t.w[k], c.f[k], v);
            } else {
                v.x += t.w[k] * c.f[k].x;
                v.y += t.w[k] * c.f[k].y;
                v.z += t.w[k] * c.f[k].z;
                v.w += t.w[k] * c.f[k].w;
            }
        }
    return v;
}

// PF: while the bins consume column x, the taps of column x+1 (the next one the
// left-to-right sweep needs unless it skips) are already in flight.
typedef float vf4 __attribute__((ext_vector_type(4)));

// NT: output rows are written once and never re-read by this launch; storing
// them non-temporal keeps them from evicting pyramid lines that overlapping
// RoIs on the same XCD are about to re-read from L2.
template <int SR, bool FMA, bool PF, bool NT = false>
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_sep_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, int out_nhwc, float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float tile[];  // [C][P][P] (NCHW out)
    const int r = roi_order ? roi_order[blockIdx.x] : (int)blockIdx.x;
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
    const int chunks = (C + 255) / 256;
    const int lane = lane_id();
    const int W = g.W;
    const int64_t rowstride = (int64_t)W * C;
    const float inv = 1.f / g.count;  // count = SR*SR, a power of two for SR=2: exact
    for (int u = wave_id(); u < P * chunks; u += num_waves()) {
        const int ph = u / chunks;
        const int ck = u - ph * chunks;
        const int c0 = ck * 256 + lane * 4;
        const bool active = c0 < C;
        const float *base = g.feat + (active ? c0 : 0);
        const RowTaps<SR> taps = row_taps<SR>(g, ph);
        int cl = -1, ch = -1, pfc = -1;
        float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
        TapCol<SR> pf;
        auto column = [&](int x) -> float4 {
            if (PF) {
                TapCol<SR> cur;
                if (x == pfc) cur = pf;
                else cur = load_column<SR>(taps, base, rowstride, (int64_t)x * C);
                pfc = min(x + 1, W - 1);
                pf = load_column<SR>(taps, base, rowstride, (int64_t)pfc * C);
                return combine_column<SR, FMA>(taps, cur);
            }
            return combine_column<SR, FMA>(taps,
                                           load_column<SR>(taps, base, rowstride, (int64_t)x * C));
        };
        for (int pw = 0; pw < P; ++pw) {
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int ix = 0; ix < SR; ++ix) {
                float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
                if (x < -1.0f || x > (float)W) continue;  // wave-uniform
                if (x <= 0) x = 0;
                int xl = (int)x, xh;
                if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
                const float lx = x - xl, hx = 1.f - lx;
                if (xl != cl || xh != ch) {
                    if (xl == ch) va = vb;
                    else va = column(xl);
                    vb = (xh == xl) ? va : column(xh);
                    cl = xl;
                    ch = xh;
                }
                if (FMA) {
                    acc = fma4(hx, va, acc);
                    acc = fma4(lx, vb, acc);
                } else {
                    acc.x += hx * va.x + lx * vb.x;
                    acc.y += hx * va.y + lx * vb.y;
                    acc.z += hx * va.z + lx * vb.z;
                    acc.w += hx * va.w + lx * vb.w;
                }
            }
            acc = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
            if (!active) continue;
            if (out_nhwc) {
                float *dst = out + (((int64_t)r * P + ph) * P + pw) * C + c0;
                if (NT) {
                    vf4 v = {acc.x, acc.y, acc.z, acc.w};
                    __builtin_nontemporal_store(v, reinterpret_cast<vf4 *>(dst));
                } else {
                    *reinterpret_cast<float4 *>(dst) = acc;
                }
            } else {
                float *t = tile + (int64_t)c0 * P * P + ph * P + pw;
                t[0] = acc.x;
                t[P * P] = acc.y;
                t[2 * P * P] = acc.z;
                t[3 * P * P] = acc.w;
            }
        }
    }
    if (out_nhwc) return;
    __syncthreads();
    const int n4 = (C * P * P) / 4;
    float4 *o4 = reinterpret_cast<float4 *>(out + (int64_t)r * C * P * P);
    const float4 *t4 = reinterpret_cast<const float4 *>(tile);
    for (int i = threadIdx.x; i < n4; i += blockDim.x) o4[i] = t4[i];
    float *o = out + (int64_t)r * C * P * P;
    for (int i = n4 * 4 + threadIdx.x; i < C * P * P; i += blockDim.x) o[i] = tile[i];
}

// --------------------------------------------------------------------------
// XCD channel-sliced separable forward, one workgroup per (RoI, slice) with
// one wave per output row.  Keeping ~P waves per RoI keeps the number of RoIs
// an XCD has in flight at what the full-pixel kernel has (~128), while the
// bytes each RoI pulls into that XCD's L2 shrink 8x: the in-flight footprint
// window (~3 MB of 128-B pixel slices) fits the 4 MiB L2, so overlapping RoIs
// re-read from L2 instead of the fabric.  Per output row the wave
//   1. loads its tap columns 8 at a time (lane group g = column slot, lane
//      q = channel quad): one 1 KiB instruction = 8 pixel slices of one tap
//      row; the vertical combine V(x) = sum_k w_k F(row_k, x) is lane-local;
//   2. parks V in LDS (wave-private), then lane group g computes bin pw = g
//      (g + 8 ...) from V(xl), V(xh) of its samples and stores 128 B.
// Column slots: the contiguous range [xmin, xmax] of tap columns when it fits
// NS slots (every RoI with sample spacing <= 1 px), else one slot per tap
// (2 P SR <= NS).  Arithmetic order as roi_align_fpn_nhwc_sep_kernel.
// Measured (variant 16, profiles/r01_roialign_pmc/xslice_v16.txt): fabric reads
// drop to 642 MB per launch (= the compulsory 0.66 GB; variant 8 reads 1.17 GB)
// and the L2 hit rate rises 0.54 -> 0.69, but the kernel runs 8x the waves
// with the per-RoI prologue replicated per slice: 2.7x the VALU instructions
// of variant 8, VALU-issue bound at ~510 us vs 306 us.  Kept as the record of
// the locality experiment (and its persistent / slice-per-row-group cousins,
// both slower); variant 8 stays the product kernel.
// --------------------------------------------------------------------------
struct SampleX {
    int xl, xh;
    float lx;
    bool ok;
};

template <int SR>
__device__ __forceinline__ SampleX sample_x(const RoiGeom &g, int j) {
    const int pw = j / SR, ix = j - (j / SR) * SR;
    float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
    SampleX sx;
    sx.ok = !(x < -1.0f || x > (float)g.W);
    if (x <= 0) x = 0;
    int xl = (int)x, xh;
    if (xl >= g.W - 1) { xh = xl = g.W - 1; x = (float)xl; } else xh = xl + 1;
    sx.xl = xl;
    sx.xh = xh;
    sx.lx = x - xl;
    return sx;
}

template <int SR, int NS>
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_xslice2_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, float *__restrict__ out) {
    __shared__ float4 vcol[8][NS][8];  // [wave][column slot][channel quad]
    const int S = C >> 5;
    const int s = blockIdx.x % S;
    const int i = blockIdx.x / S;
    int r = roi_order ? roi_order[i] : i;
    r = __builtin_amdgcn_readfirstlane(r);
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
    const int lane = lane_id(), wv = wave_id();
    const int grp = lane >> 3, q = lane & 7;
    const int c0 = s * 32 + q * 4;
    const float *base = g.feat + c0;
    const int64_t rowstride = (int64_t)g.W * C;
    const float inv = 1.f / g.count;
    const int nsamp = P * SR;
    // valid samples are a contiguous run [j0, j1] (x increases with j)
    int j0 = 0, j1 = nsamp - 1;
    while (j0 < nsamp && !sample_x<SR>(g, j0).ok) ++j0;
    while (j1 >= j0 && !sample_x<SR>(g, j1).ok) --j1;
    int xmin = 0, nslot = 0;
    bool contiguous = true;
    if (j0 <= j1) {
        xmin = sample_x<SR>(g, j0).xl;
        const int span = sample_x<SR>(g, j1).xh - xmin + 1;
        contiguous = span <= NS;
        nslot = contiguous ? span : 2 * nsamp;
    }
    float4 *vw = &vcol[wv][0][0];
    for (int ph = wv; ph < P; ph += num_waves()) {
        const RowTaps<SR> taps = row_taps<SR>(g, ph);
        for (int c8 = 0; c8 < nslot; c8 += 8) {
            const int slot = c8 + grp;
            int col;
            if (contiguous) {
                col = xmin + slot;
            } else {
                const SampleX sx = sample_x<SR>(g, min(slot >> 1, nsamp - 1));
                col = (slot & 1) ? sx.xh : sx.xl;
            }
            col = min(col, g.W - 1);
            const bool ok = slot < nslot;
            const float *p = base + (int64_t)col * C;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int k = 0; k < 2 * SR; ++k)
                if (taps.alive[k] && ok) {
                    const float4 f = ld4(p + taps.row[k] * rowstride);
                    v.x += taps.w[k] * f.x;
                    v.y += taps.w[k] * f.y;
                    v.z += taps.w[k] * f.z;
                    v.w += taps.w[k] * f.w;
                }
            vw[slot * 8 + q] = v;
        }
        __builtin_amdgcn_wave_barrier();
        for (int pw = grp; pw < P; pw += 8) {
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int ix = 0; ix < SR; ++ix) {
                const int j = pw * SR + ix;
                const SampleX sx = sample_x<SR>(g, j);
                if (!sx.ok) continue;
                const int sa = contiguous ? sx.xl - xmin : 2 * j;
                const int sb = contiguous ? sx.xh - xmin : 2 * j + 1;
                const float4 va = vw[sa * 8 + q], vb = vw[sb * 8 + q];
                const float lx = sx.lx, hx = 1.f - lx;
                acc.x += hx * va.x + lx * vb.x;
                acc.y += hx * va.y + lx * vb.y;
                acc.z += hx * va.z + lx * vb.z;
                acc.w += hx * va.w + lx * vb.w;
            }
            *reinterpret_cast<float4 *>(out + (((int64_t)r * P + ph) * P + pw) * C + c0) =
                make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Column-streamed separable row: the row's tap columns form the contiguous
// range [xa, xb] (sample spacing bw/SR <= 1 px for every RoI the FPN level map
// sends to P2-P5 at 7x7 / SR 2, except the largest on P5), so the wave walks it
// left to right with the taps of the next DEPTH columns already in flight (a
// static ring of raw loads: the memory-level parallelism the dependent
// column-by-column fetch of roi_align_fpn_nhwc_sep_kernel lacks).  Samples are
// consumed as soon as their right column has arrived; a bin is stored when its
// last sample is done.
template <int SR, int DEPTH>
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_stream_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, int out_nhwc, float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float tile[];  // [C][P][P] (NCHW out)
    constexpr int T = 2 * SR;
    const int r = roi_order ? roi_order[blockIdx.x] : (int)blockIdx.x;
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
    const int chunks = (C + 255) / 256;
    const int lane = lane_id();
    const int W = g.W;
    const int64_t rowstride = (int64_t)W * C;
    const float inv = 1.f / g.count;
    const int NS = P * SR;
    // x geometry of sample j (identical for every row)
    auto sample = [&](int j, int &xl, int &xh, float &lx) -> bool {
        const int pw = j / SR, ix = j - pw * SR;
        float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
        if (x < -1.0f || x > (float)W) return false;
        if (x <= 0) x = 0;
        xl = (int)x;
        if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
        lx = x - xl;
        return true;
    };
    // valid samples are a contiguous index range [ja, jb); columns [xa, xb]
    int ja = 0, jb = NS, xa = 0, xb = -1;
    {
        int xl, xh;
        float lx;
        while (ja < NS && !sample(ja, xl, xh, lx)) ++ja;
        if (ja < NS) xa = xl;
        while (jb > ja && !sample(jb - 1, xl, xh, lx)) --jb;
        if (jb > ja) xb = xh;
    }
    const int ncols = xb - xa + 1;
    for (int u = wave_id(); u < P * chunks; u += num_waves()) {
        const int ph = u / chunks;
        const int ck = u - ph * chunks;
        const int c0 = ck * 256 + lane * 4;
        const bool active = c0 < C;
        const float *base = g.feat + (active ? c0 : 0);
        const RowTaps<SR> taps = row_taps<SR>(g, ph);
        const float *rp[T];
#pragma unroll
        for (int k = 0; k < T; ++k) rp[k] = base + taps.row[k] * rowstride;
        auto store = [&](int pw, float4 a) {
            if (!active) return;
            a = make_float4(a.x * inv, a.y * inv, a.z * inv, a.w * inv);
            if (out_nhwc) {
                *reinterpret_cast<float4 *>(out + (((int64_t)r * P + ph) * P + pw) * C + c0) = a;
            } else {
                float *t = tile + (int64_t)c0 * P * P + ph * P + pw;
                t[0] = a.x;
                t[P * P] = a.y;
                t[2 * P * P] = a.z;
                t[3 * P * P] = a.w;
            }
        };
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        int j = 0;
        // leading out-of-range samples (contribute 0)
        for (; j < ja; ++j)
            if (j % SR == SR - 1) { store(j / SR, acc); acc = make_float4(0.f, 0.f, 0.f, 0.f); }
        float4 raw[DEPTH][T];
        auto issue = [&](float4 (&dst)[T], int col) {
            const int64_t off = (int64_t)min(col, xb) * C;
#pragma unroll
            for (int k = 0; k < T; ++k)
                if (taps.alive[k]) dst[k] = ld4(rp[k] + off);
        };
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) issue(raw[d], xa + d);
        float4 vprev = make_float4(0.f, 0.f, 0.f, 0.f);
        // consume column xa + k from ring slot d, refill the slot with column + DEPTH
        auto step = [&](int k, float4 (&slot)[T]) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int t = 0; t < T; ++t)
                if (taps.alive[t]) {
                    v.x += taps.w[t] * slot[t].x;
                    v.y += taps.w[t] * slot[t].y;
                    v.z += taps.w[t] * slot[t].z;
                    v.w += taps.w[t] * slot[t].w;
                }
            if (k + DEPTH < ncols) issue(slot, xa + k + DEPTH);
            const int x = xa + k;
            int xl, xh;
            float lx;
            while (j < jb) {
                sample(j, xl, xh, lx);
                if (xh != x) break;
                const float hx = 1.f - lx;
                const float4 va = (xl == x) ? v : vprev;
                acc.x += hx * va.x + lx * v.x;
                acc.y += hx * va.y + lx * v.y;
                acc.z += hx * va.z + lx * v.z;
                acc.w += hx * va.w + lx * v.w;
                if (j % SR == SR - 1) {
                    store(j / SR, acc);
                    acc = make_float4(0.f, 0.f, 0.f, 0.f);
                }
                ++j;
            }
            vprev = v;
        };
        for (int k = 0; k < ncols; k += DEPTH) {
#pragma unroll
            for (int d = 0; d < DEPTH; ++d)
                if (k + d < ncols) step(k + d, raw[d]);
        }
        // trailing out-of-range samples
        for (; j < NS; ++j)
            if (j % SR == SR - 1) { store(j / SR, acc); acc = make_float4(0.f, 0.f, 0.f, 0.f); }
    }
    if (out_nhwc) return;
    __syncthreads();
    const int n4 = (C * P * P) / 4;
    float4 *o4 = reinterpret_cast<float4 *>(out + (int64_t)r * C * P * P);
    const float4 *t4 = reinterpret_cast<const float4 *>(tile);
    for (int i = threadIdx.x; i < n4; i += blockDim.x) o4[i] = t4[i];
    float *o = out + (int64_t)r * C * P * P;
    for (int i = n4 * 4 + threadIdx.x; i < C * P * P; i += blockDim.x) o[i] = tile[i];
}

template <int P, int SR, int D>
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int R, int sr, int rows_per_block, int out_nhwc,
    float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float tile[];
    const int r = roi_order ? roi_order[blockIdx.x] : (int)blockIdx.x;
    const int row0 = blockIdx.y * rows_per_block;
    const int rows = min(rows_per_block, P - row0);
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, sr);
    const int chunks = (C + 255) / 256;
    const int units = rows * chunks;
    const int seg = rows * P;
    const int lane = lane_id();
    for (int u = wave_id(); u < units; u += num_waves()) {
        const int prow = u / chunks;
        const int ck = u - prow * chunks;
        const int c0 = ck * 256 + lane * 4;
        const bool active = c0 < C;
        float4 acc[P];
        if (SR > 0)
            nhwc_row_sr<P, (SR > 0 ? SR : 1), D>(g, C, row0 + prow, active ? c0 : 0, acc);
        else
            nhwc_row<P>(g, C, row0 + prow, active ? c0 : 0, active, acc);
        if (active && out_nhwc) {  // [R][P][P][C]: one coalesced 1 KiB store per bin
            float *o = out + (((int64_t)r * P + row0 + prow) * P) * C + c0;
#pragma unroll
            for (int pw = 0; pw < P; ++pw) {
                const float4 a = acc[pw];
                *reinterpret_cast<float4 *>(o + (int64_t)pw * C) =
                    make_float4(a.x / g.count, a.y / g.count, a.z / g.count, a.w / g.count);
            }
        } else if (active) {
#pragma unroll
            for (int pw = 0; pw < P; ++pw) {
                float *t = tile + (int64_t)c0 * seg + prow * P + pw;
                t[0] = acc[pw].x / g.count;
                t[seg] = acc[pw].y / g.count;
                t[2 * seg] = acc[pw].z / g.count;
                t[3 * seg] = acc[pw].w / g.count;
            }
        }
    }
    if (out_nhwc) return;
    __syncthreads();
    float *o = out + (int64_t)r * C * P * P + row0 * P;
    if (rows == P) {  // whole RoI: one contiguous C*P*P block
        const int n4 = (C * P * P) / 4;
        float4 *o4 = reinterpret_cast<float4 *>(o);
        const float4 *t4 = reinterpret_cast<const float4 *>(tile);
        for (int i = threadIdx.x; i < n4; i += blockDim.x) o4[i] = t4[i];
        for (int i = n4 * 4 + threadIdx.x; i < C * P * P; i += blockDim.x) o[i] = tile[i];
    } else {
        for (int i = threadIdx.x; i < C * seg; i += blockDim.x) {
            const int c = i / seg, rem = i - c * seg;
            o[(int64_t)c * P * P + rem] = tile[i];
        }
    }
}

// --------------------------------------------------------------------------
// NHWC forward with the RoI footprint staged in LDS (C == 256, fixed P, SR).
//
// The P*SR x-samples of a RoI touch a sorted set of distinct columns D and the
// P*SR y-samples a sorted set of distinct rows Y; every bilinear tap is a pixel
// of the Y x D grid.  The grid is loaded into LDS once per RoI (one 1 KiB
// global_load_lds per pixel = 256 fp32 channels), window by window when it is
// larger than the LDS budget, and every one of the 4*P*P*SR*SR taps is then an
// LDS read.  Each pixel crosses the L2/MALL once per RoI instead of once per
// tap (4x-8x fewer fetches for the small RoIs that dominate P2).  Wave w owns
// output column pw = w and accumulates acc[ph] in the reference's order.
// --------------------------------------------------------------------------
struct FootMeta {
    int ncol, nrow;
    int col[64], row[64];            // distinct tap columns / rows (pixel coords)
    int xs_l[32], xs_h[32];          // per x-sample: slots in col[]
    int ys_l[32], ys_h[32];          // per y-sample: slots in row[]
    float lx[32], ly[32];
    int vx[32], vy[32];
};

template <int NS>
__device__ inline void build_axis(int n_lim, float start, float bin, int (&slots_l)[32],
                                  int (&slots_h)[32], float (&frac)[32], int (&valid)[32],
                                  int (&list)[64], int &count, int SRv) {
    // serial, one lane: positions are non-decreasing, so the union of {lo, hi}
    // over valid samples is built sorted by appending
    int cnt = 0, last = -1;
    for (int j = 0; j < NS; ++j) {
        const int p = j / SRv, ix = j - p * SRv;
        float v = start + p * bin + (ix + .5f) * bin / SRv;
        const bool ok = !(v < -1.0f || v > (float)n_lim);
        if (v <= 0) v = 0;
        int lo = (int)v, hi;
        if (lo >= n_lim - 1) { hi = lo = n_lim - 1; v = (float)lo; } else hi = lo + 1;
        frac[j] = v - lo;
        valid[j] = ok;
        if (!ok) { slots_l[j] = slots_h[j] = 0; continue; }
        if (lo > last) { list[cnt++] = lo; last = lo; }
        slots_l[j] = (list[cnt - 1] == lo) ? cnt - 1 : cnt - 2;
        if (hi > last) { list[cnt++] = hi; last = hi; }
        slots_h[j] = (list[cnt - 1] == hi) ? cnt - 1 : cnt - 2;
    }
    count = cnt;
}

template <int P, int SR>
__global__ __launch_bounds__(P * 64) void roi_align_fpn_nhwc_lds_kernel(
    FpnLevels fa, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int budget_px, float *__restrict__ out) {
    constexpr int C = 256;
    constexpr int NS = P * SR;
    extern __shared__ __attribute__((aligned(16))) float4 sm[];
    __shared__ FootMeta meta;
    const int r = roi_order ? roi_order[blockIdx.x] : (int)blockIdx.x;
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
    const int wave = wave_id(), lane = lane_id();
    if (threadIdx.x == 0)
        build_axis<NS>(g.W, g.sw, g.bw, meta.xs_l, meta.xs_h, meta.lx, meta.vx, meta.col,
                       meta.ncol, SR);
    if (threadIdx.x == 64)
        build_axis<NS>(g.H, g.sh, g.bh, meta.ys_l, meta.ys_h, meta.ly, meta.vy, meta.row,
                       meta.nrow, SR);
    __syncthreads();
    const int ncol = meta.ncol, nrow = meta.nrow;
    const int M = ncol > 0 ? budget_px / ncol : 0;  // rows per LDS window (>= 2)
    const float *fbase = g.feat + lane * 4;
    // this wave's column of bins: samples j = pw*SR + ix
    const int pw = wave;
    int xl[SR], xh[SR];
    float lxv[SR];
    bool vxv[SR];
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
        const int j = pw * SR + ix;
        xl[ix] = meta.xs_l[j];
        xh[ix] = meta.xs_h[j];
        lxv[ix] = meta.lx[j];
        vxv[ix] = meta.vx[j] != 0;
    }
    float4 acc[P];
#pragma unroll
    for (int ph = 0; ph < P; ++ph) acc[ph] = make_float4(0.f, 0.f, 0.f, 0.f);
    int w0 = 0, w1 = 0;  // rows [w0, w1) of row[] are resident
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        if (!meta.vy[i]) continue;  // whole sample row reads 0 (uniform)
        const int yl = meta.ys_l[i], yh = meta.ys_h[i];
        if (yh >= w1 || yl < w0) {  // slide the window (uniform across the block)
            __syncthreads();
            w0 = yl;
            w1 = min(w0 + M, nrow);
            const int npx = (w1 - w0) * ncol;
            for (int p = wave; p < npx; p += P) {
                const int ry = w0 + p / ncol, cx = p - (p / ncol) * ncol;
                const float *src = fbase + ((int64_t)meta.row[ry] * g.W + meta.col[cx]) * C;
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)src,
                    (__attribute__((address_space(3))) void *)(sm + p * 64), 16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        const float ly = meta.ly[i], hy = 1.f - ly;
        const float4 *top = sm + (yl - w0) * ncol * 64 + lane;
        const float4 *bot = sm + (yh - w0) * ncol * 64 + lane;
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) {
            const float lx = lxv[ix], hx = 1.f - lx;
            const float4 a = top[xl[ix] * 64], b = top[xh[ix] * 64];
            const float4 c = bot[xl[ix] * 64], d = bot[xh[ix] * 64];
            float4 t = acc[i / SR];
            bilerp_acc(t, hy * hx, hy * lx, ly * hx, ly * lx, a, b, c, d);
            if (vxv[ix]) acc[i / SR] = t;
        }
    }
    __syncthreads();  // the window buffer becomes the [C][P][P] output tile
    float *tile = reinterpret_cast<float *>(sm);
#pragma unroll
    for (int ph = 0; ph < P; ++ph) {
        float *t = tile + (lane * 4) * (P * P) + ph * P + pw;
        t[0] = acc[ph].x / g.count;
        t[P * P] = acc[ph].y / g.count;
        t[2 * P * P] = acc[ph].z / g.count;
        t[3 * P * P] = acc[ph].w / g.count;
    }
    __syncthreads();
    float4 *o4 = reinterpret_cast<float4 *>(out + (int64_t)r * C * P * P);
    for (int i = threadIdx.x; i < C * P * P / 4; i += blockDim.x) o4[i] = sm[i];
}

// --------------------------------------------------------------------------
// NHWC forward, channel-sliced per XCD (the product kernel for C % 32 == 0).
//
// Overlapping RoIs of one frame re-read the same pyramid pixels ~4.5x (sum of
// per-RoI footprints / union), and a whole-pixel (1 KiB) working
// set of the RoIs in flight does not fit a 4 MiB XCD L2, so those re-reads go
// to the Infinity Cache.  Here block b pools channel slice s = b % S (32
// channels = one 128-B line per pixel) of RoI order[b / S]: all blocks of a
// slice land on one XCD (blocks b and b+8 share an XCD), so each XCD's L2 only
// holds 1/8 of every pixel and the spatially sorted RoI stream re-reads it from
// L2.  A lane group of 8 lanes (float4 each) owns one output bin; every tap is
// one 128-B line, all 4*SR*SR taps of a bin are in flight together.  The bin
// values are staged in LDS as [32][P*P] and written as one contiguous block.
// --------------------------------------------------------------------------
template <int SR>
__device__ __forceinline__ float4 bin_value(const RoiGeom &g, int C, const float *base, int ph,
                                            int pw, int gh, int gw) {
    const int H = g.H, W = g.W;
    const int64_t rowstride = (int64_t)W * C;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (SR > 0) {
        constexpr int NK = SR > 0 ? SR * SR : 1;
        float4 v[NK][4];
        float wts[NK][4];
        bool ok[NK];
#pragma unroll
        for (int iy = 0; iy < SR; ++iy) {
            float y = g.sh + ph * g.bh + (iy + .5f) * g.bh / SR;
            const bool vy = !(y < -1.0f || y > (float)H);
            if (y <= 0) y = 0;
            int yl = (int)y, yh;
            if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
            const float ly = y - yl, hy = 1.f - ly;
#pragma unroll
            for (int ix = 0; ix < SR; ++ix) {
                float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
                const bool vx = !(x < -1.0f || x > (float)W);
                if (x <= 0) x = 0;
                int xl = (int)x, xh;
                if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
                const float lx = x - xl, hx = 1.f - lx;
                const int k = iy * SR + ix;
                v[k][0] = ld4(base + yl * rowstride + (int64_t)xl * C);
                v[k][1] = ld4(base + yl * rowstride + (int64_t)xh * C);
                v[k][2] = ld4(base + yh * rowstride + (int64_t)xl * C);
                v[k][3] = ld4(base + yh * rowstride + (int64_t)xh * C);
                wts[k][0] = hy * hx;
                wts[k][1] = hy * lx;
                wts[k][2] = ly * hx;
                wts[k][3] = ly * lx;
                ok[k] = vy && vx;
            }
        }
#pragma unroll
        for (int k = 0; k < SR * SR; ++k) {
            float4 t = acc;
            bilerp_acc(t, wts[k][0], wts[k][1], wts[k][2], wts[k][3], v[k][0], v[k][1], v[k][2],
                       v[k][3]);
            if (ok[k]) acc = t;
        }
        return acc;
    }
    for (int iy = 0; iy < gh; ++iy) {
        float y = g.sh + ph * g.bh + (iy + .5f) * g.bh / gh;
        for (int ix = 0; ix < gw; ++ix) {
            float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / gw;
            float yy = y;
            if (yy < -1.0f || yy > (float)H || x < -1.0f || x > (float)W) continue;
            if (yy <= 0) yy = 0;
            if (x <= 0) x = 0;
            int yl = (int)yy, xl = (int)x, yh, xh;
            if (yl >= H - 1) { yh = yl = H - 1; yy = (float)yl; } else yh = yl + 1;
            if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
            const float ly = yy - yl, lx = x - xl, hy = 1.f - ly, hx = 1.f - lx;
            bilerp_acc(acc, hy * hx, hy * lx, ly * hx, ly * lx,
                       ld4(base + yl * rowstride + (int64_t)xl * C),
                       ld4(base + yl * rowstride + (int64_t)xh * C),
                       ld4(base + yh * rowstride + (int64_t)xl * C),
                       ld4(base + yh * rowstride + (int64_t)xh * C));
        }
    }
    return acc;
}

template <int SR>
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_sliced_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int PH, int PW, int sr, float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) float tile[32 * 196];
    const int S = C / 32;
    const int slice = blockIdx.x % S;
    const int ri = blockIdx.x / S;
    const int r = roi_order ? roi_order[ri] : ri;
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, PH, PW, sr);
    const int lane = lane_id();
    const int grp = lane >> 3, q = lane & 7;
    const int PP = PH * PW;
    const float *base = g.feat + slice * 32 + q * 4;
    for (int b0 = wave_id() * 8; b0 < PP; b0 += num_waves() * 8) {
        const int bin = b0 + grp;
        if (bin < PP) {
            const int ph = bin / PW, pw = bin - (bin / PW) * PW;
            const float4 a = bin_value<SR>(g, C, base, ph, pw, g.gh, g.gw);
            float *t = tile + (q * 4) * PP + bin;
            t[0] = a.x / g.count;
            t[PP] = a.y / g.count;
            t[2 * PP] = a.z / g.count;
            t[3 * PP] = a.w / g.count;
        }
    }
    __syncthreads();
    float *o = out + ((int64_t)r * C + slice * 32) * PP;
    const int n = 32 * PP;
    // 32*PP floats: a multiple of 4, and o is 16-B aligned (C % 32 == 0)
    for (int i = threadIdx.x; i < n / 4; i += blockDim.x)
        reinterpret_cast<float4 *>(o)[i] = reinterpret_cast<const float4 *>(tile)[i];
}

// Any pooled size: one wave per (bin, 256-channel chunk), accumulator per bin.
__global__ __launch_bounds__(256) void roi_align_fpn_nhwc_generic_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    int R, int PH, int PW, int sr, float *__restrict__ out) {
    const int r = blockIdx.x;
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, PH, PW, sr);
    const int chunks = (C + 255) / 256;
    const int lane = lane_id();
    const int64_t rowstride = (int64_t)g.W * C;
    for (int u = wave_id(); u < PH * PW * chunks; u += num_waves()) {
        const int bin = u / chunks, ck = u - bin * chunks;
        const int ph = bin / PW, pw = bin - ph * PW;
        const int c0 = ck * 256 + lane * 4;
        if (c0 >= C) continue;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int iy = 0; iy < g.gh; ++iy) {
            float y = g.sh + ph * g.bh + (iy + .5f) * g.bh / g.gh;
            for (int ix = 0; ix < g.gw; ++ix) {
                float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / g.gw;
                float yy = y;
                if (yy < -1.0f || yy > (float)g.H || x < -1.0f || x > (float)g.W) continue;
                if (yy <= 0) yy = 0;
                if (x <= 0) x = 0;
                int yl = (int)yy, xl = (int)x, yh, xh;
                if (yl >= g.H - 1) { yh = yl = g.H - 1; yy = (float)yl; } else yh = yl + 1;
                if (xl >= g.W - 1) { xh = xl = g.W - 1; x = (float)xl; } else xh = xl + 1;
                float ly = yy - yl, lx = x - xl, hy = 1.f - ly, hx = 1.f - lx;
                const float *base = g.feat + c0;
                float4 a = ld4(base + yl * rowstride + (int64_t)xl * C);
                float4 b = ld4(base + yl * rowstride + (int64_t)xh * C);
                float4 c = ld4(base + yh * rowstride + (int64_t)xl * C);
                float4 d = ld4(base + yh * rowstride + (int64_t)xh * C);
                bilerp_acc(acc, hy * hx, hy * lx, ly * hx, ly * lx, a, b, c, d);
            }
        }
        float *o = out + ((int64_t)r * C + c0) * PH * PW + ph * PW + pw;
        o[0] = acc.x / g.count;
        o[PH * PW] = acc.y / g.count;
        o[2 * PH * PW] = acc.z / g.count;
        o[3 * PH * PW] = acc.w / g.count;
    }
}

// --------------------------------------------------------------------------
// Launchers
// --------------------------------------------------------------------------
static int grid_1d(int64_t n, int block) {
    int64_t g = (n + block - 1) / block;
    if (g > 65536) g = 65536;  // grid-stride the rest (memory-bound)
    return (int)(g < 1 ? 1 : g);
}

int launch_roi_align_fwd_nchw(const float *feat, int B, int C, int H, int W, const float *rois,
                              int R, int PH, int PW, float scale, int sr, float *out,
                              hipStream_t s) {
    (void)B;
    int64_t n = (int64_t)R * C * PH * PW;
    if (n == 0) return VD_OK;
    hipLaunchKernelGGL(roi_align_fwd_nchw_kernel, dim3(grid_1d(n, 256)), dim3(256), 0, s, n, feat,
                       scale, H, W, C, PH, PW, sr, rois, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int launch_roi_align_bwd_nchw(const float *top_diff, int B, int C, int H, int W,
                              const float *rois, int R, int PH, int PW, float scale, int sr,
                              float *bottom_diff, hipStream_t s) {
    (void)B;
    int64_t n = (int64_t)R * C * PH * PW;
    if (n == 0) return VD_OK;
    hipLaunchKernelGGL(roi_align_bwd_nchw_kernel, dim3(grid_1d(n, 256)), dim3(256), 0, s, n,
                       top_diff, scale, H, W, C, PH, PW, sr, rois, bottom_diff);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

static constexpr int kTileBudget = 64 * 1024;  // LDS bytes per workgroup (2-3 WGs/CU)

template <int P, int SR, int D = 3>
static int launch_rows(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                       const int *order, int R, int sr, float *out, hipStream_t s,
                       int out_nhwc = 0) {
    const int row_bytes = C * P * 4;
    int rows = kTileBudget / row_bytes;
    if (rows < 1) rows = 1;
    if (rows > P || out_nhwc) rows = P;
    if (!out_nhwc && (int64_t)rows * row_bytes > 160 * 1024) return VD_ERR_SHAPE;
    const int chunks = (C + 255) / 256;
    int waves = rows * chunks;
    if (waves > 8) waves = 8;  // __launch_bounds__(512): <= 256 VGPRs, acc[P] stays in registers
    const size_t lds = out_nhwc ? 0 : (size_t)rows * row_bytes;
    dim3 grid(R, (P + rows - 1) / rows);
    hipLaunchKernelGGL((roi_align_fpn_nhwc_kernel<P, SR, D>), grid, dim3(64 * waves), lds, s, fa,
                       C, rois, lvl, order, R, sr, rows, out_nhwc, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

static int roialign_variant() {  // read per launch so tests can switch kernels
    const char *e = getenv("VOSDET_ROIALIGN_VARIANT");
    // 8: separable kernel (product default, RoIAlign tolerance 1e-4);
    // 3: bit-exact row kernel (the reference's per-sample arithmetic order)
    return e ? atoi(e) : 8;
}

template <int SR, bool FMA, bool PF, bool NT = false>
static void launch_sep_t(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                         const int *order, int R, int P, int out_nhwc, float *out, hipStream_t s,
                         int waves, size_t lds) {
    hipLaunchKernelGGL((roi_align_fpn_nhwc_sep_kernel<SR, FMA, PF, NT>), dim3(R), dim3(64 * waves),
                       lds, s, fa, C, rois, lvl, order, P, out_nhwc, out);
}

static int launch_sep(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                      const int *order, int R, int P, int out_nhwc, float *out, hipStream_t s) {
    const size_t lds = out_nhwc ? 0 : (size_t)C * P * P * 4;
    if (lds > 160 * 1024) return VD_ERR_SHAPE;
    int waves = P * ((C + 255) / 256);
    if (waves > 8) waves = 8;
    const int v = roialign_variant();
    if (v == 9)
        hipLaunchKernelGGL((roi_align_fpn_nhwc_stream_kernel<2, 2>), dim3(R), dim3(64 * waves), lds,
                           s, fa, C, rois, lvl, order, P, out_nhwc, out);
    else if (v == 13)
        launch_sep_t<2, true, false>(fa, C, rois, lvl, order, R, P, out_nhwc, out, s, waves, lds);
    else if (v == 14)
        launch_sep_t<2, true, true>(fa, C, rois, lvl, order, R, P, out_nhwc, out, s, waves, lds);
    else if (v == 20)  // plain (write-back) output stores: 306 us vs 297 us with NT
        launch_sep_t<2, false, false>(fa, C, rois, lvl, order, R, P, out_nhwc, out, s, waves,
                                      lds);
    else if (v == 22)
        launch_sep_t<2, true, false, true>(fa, C, rois, lvl, order, R, P, out_nhwc, out, s, waves,
                                           lds);
    else  // product default (variant 8): non-temporal output stores
        launch_sep_t<2, false, false, true>(fa, C, rois, lvl, order, R, P, out_nhwc, out, s, waves,
                                            lds);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}


int launch_roi_align_fpn_nhwc(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                              const int *order, int R, int PH, int PW, int sr, int out_nhwc,
                              float *out, hipStream_t s) {
    if (R == 0) return VD_OK;
    if (C % 4 != 0) return VD_ERR_SHAPE;
    const int variant = roialign_variant();
    if (out_nhwc) {  // product path: [R][P][P][C] written straight from registers
        if (variant == 16 && sr == 2 && PH == PW && C % 32 == 0 && PH <= 16) {
            const int64_t blocks = (int64_t)R * (C / 32);
            const int waves = PH < 8 ? PH : 8;
            if (PH <= 8)
                hipLaunchKernelGGL((roi_align_fpn_nhwc_xslice2_kernel<2, 32>),
                                   dim3((unsigned)blocks), dim3(64 * waves), 0, s, fa, C, rois,
                                   lvl, order, PH, out);
            else
                hipLaunchKernelGGL((roi_align_fpn_nhwc_xslice2_kernel<2, 64>),
                                   dim3((unsigned)blocks), dim3(64 * waves), 0, s, fa, C, rois,
                                   lvl, order, PH, out);
            return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
        }
        if (variant >= 8 && sr == 2 && PH == PW)
            return launch_sep(fa, C, rois, lvl, order, R, PH, 1, out, s);
        if (PH == PW && PH == 7)
            return sr == 2 ? launch_rows<7, 2, 2>(fa, C, rois, lvl, order, R, sr, out, s, 1)
                           : launch_rows<7, 0>(fa, C, rois, lvl, order, R, sr, out, s, 1);
        if (PH == PW && PH == 14)
            return sr == 2 ? launch_rows<14, 2, 2>(fa, C, rois, lvl, order, R, sr, out, s, 1)
                           : launch_rows<14, 0>(fa, C, rois, lvl, order, R, sr, out, s, 1);
        return VD_ERR_SHAPE;
    }
    if (variant >= 8 && sr == 2 && PH == PW && (int64_t)C * PH * PW * 4 <= 160 * 1024)
        return launch_sep(fa, C, rois, lvl, order, R, PH, 0, out, s);
    if (C % 32 == 0 && PH * PW <= 196 && (variant == 0 || variant == 7)) {
        const int bins = PH * PW;
        int waves = (bins + 7) / 8;
        if (waves > 8) waves = 8;
        const dim3 grid((unsigned)((int64_t)R * (C / 32)));
        if (sr == 2)
            hipLaunchKernelGGL((roi_align_fpn_nhwc_sliced_kernel<2>), grid, dim3(64 * waves), 0, s,
                               fa, C, rois, lvl, order, PH, PW, sr, out);
        else
            hipLaunchKernelGGL((roi_align_fpn_nhwc_sliced_kernel<0>), grid, dim3(64 * waves), 0, s,
                               fa, C, rois, lvl, order, PH, PW, sr, out);
        return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
    }
    if (PH == PW && (PH == 7 || PH == 14)) {
        const bool unrolled = sr == 2 && variant >= 2;
        if (PH == 7 && sr == 2 && C == 256 && variant == 6) {
            // LDS footprint staging: budget >= 2 rows x 28 columns and >= the output tile
            const int budget_px = 72;
            hipLaunchKernelGGL((roi_align_fpn_nhwc_lds_kernel<7, 2>), dim3(R), dim3(7 * 64),
                               (size_t)budget_px * 1024, s, fa, rois, lvl, order, budget_px, out);
            return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
        }
        if (PH == 7 && unrolled) {
            switch (variant) {
                case 3: return launch_rows<7, 2, 2>(fa, C, rois, lvl, order, R, sr, out, s);
                case 4: return launch_rows<7, 2, 4>(fa, C, rois, lvl, order, R, sr, out, s);
                case 5: return launch_rows<7, 2, 6>(fa, C, rois, lvl, order, R, sr, out, s);
                default: return launch_rows<7, 2, 3>(fa, C, rois, lvl, order, R, sr, out, s);
            }
        }
        if (PH == 7) return launch_rows<7, 0>(fa, C, rois, lvl, order, R, sr, out, s);
        return unrolled ? launch_rows<14, 2>(fa, C, rois, lvl, order, R, sr, out, s)
                        : launch_rows<14, 0>(fa, C, rois, lvl, order, R, sr, out, s);
    }
    if (order) return VD_ERR_ARG;  // the generic path writes in RoI order only
    hipLaunchKernelGGL(roi_align_fpn_nhwc_generic_kernel, dim3(R), dim3(256), 0, s, fa, C, rois,
                       lvl, R, PH, PW, sr, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
