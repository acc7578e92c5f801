// RoI geometry shared by the NHWC RoIAlign kernels (roi_align.hip,
// roi_align_tiled.hip): the reference's per-RoI sample grid
// (lib/modeling/roi_xfrom/roi_align/src/roi_align_kernel.cu:65-121) and the
// separable row-tap decomposition of the product kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vosdet_internal.hpp"

namespace vd {

__device__ __forceinline__ float4 ld4(const float *p) {
    return *reinterpret_cast<const float4 *>(p);
}

struct RoiGeom {
    const float *feat;  // this RoI's image base in its level
    int H, W;
    float sw, sh, bw, bh;
    int gh, gw;
    float count;
};

// A RoI whose level index or batch index is out of range (a malformed caller of
// the public C ABI) pools to exactly zero instead of reading out of bounds: its
// box is moved far off the map, where every sample is out of range (y < -1).
__device__ __forceinline__ RoiGeom roi_geom(const FpnLevels &fa, int C, const float *roi,
                                            int li, int PH, int PW, int sr) {
    RoiGeom g;
    const int b = (int)roi[0];
    const bool ok = li >= 0 && li < fa.L && b >= 0 && b < fa.B;
    if (!ok) li = 0;
    g.H = fa.H[li];
    g.W = fa.W[li];
    const float scale = fa.scale[li];
    g.feat = fa.feat[li] + (ok ? (int64_t)b * g.H * g.W * C : 0);
    const float kOff = -1e30f;
    g.sw = ok ? roi[1] * scale : kOff;
    g.sh = ok ? roi[2] * scale : kOff;
    float ew = ok ? roi[3] * scale : kOff, eh = ok ? roi[4] * scale : kOff;
    float rw = fmaxf(ew - g.sw, 1.f), rh = fmaxf(eh - g.sh, 1.f);
    g.bh = rh / PH;
    g.bw = rw / PW;
    g.gh = sr > 0 ? sr : (int)ceilf(rh / PH);
    g.gw = sr > 0 ? sr : (int)ceilf(rw / PW);
    g.count = (float)(g.gh * g.gw);
    return g;
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

template <int SR>
__device__ __forceinline__ float4 combine_column(const RowTaps<SR> &t, const TapCol<SR> &c) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < 2 * SR; ++k)
        if (t.alive[k]) {
            v.x += t.w[k] * c.f[k].x;
            v.y += t.w[k] * c.f[k].y;
            v.z += t.w[k] * c.f[k].z;
            v.w += t.w[k] * c.f[k].w;
        }
    return v;
}

typedef float vf4 __attribute__((ext_vector_type(4)));

}  // namespace vd
