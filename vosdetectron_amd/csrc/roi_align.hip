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
//    lane = 4 channels).  The default kernel (roi_align_fpn_nhwc_sep_buf_kernel,
//    variant 10; variant 8 is the same sweep through global loads) factors the
//    bilinear sampling into a row pass and a column pass so each pixel is
//    fetched ~once per output row; it re-associates the sums, so it holds the
//    reference to 1e-4 (north_star's RoIAlign tolerance).  The
//    row kernel (variant 3, VOSDET_ROIALIGN_VARIANT=3) keeps the reference's
//    per-sample order -- sample positions, weights, w1*v1+w2*v2+w3*v3+w4*v4,
//    iy-major accumulation, final /count, no FMA contraction -- and is
//    bit-identical to the C restatement in oracle/roi_ops.c, as are the NCHW
//    kernels.
#include <stdlib.h>

#include "common.hpp"
#include "roi_geom.hpp"
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
    int64_t nthreads, const float *__restrict__ feat, float scale, int B, int H, int W, int C,
    int PH, int PW, int sr, const float *__restrict__ rois, float *__restrict__ out) {
    for (int64_t index = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; index < nthreads;
         index += (int64_t)blockDim.x * gridDim.x) {
        int pw = (int)(index % PW);
        int ph = (int)((index / PW) % PH);
        int c = (int)((index / PW / PH) % C);
        int64_t n = index / PW / PH / C;
        const float *r = rois + n * 5;
        int b = (int)r[0];
        if (b < 0 || b >= B) {  // out-of-range batch index: zero, never an OOB read
            out[index] = 0.f;
            continue;
        }
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

__device__ __forceinline__ void bilerp_acc(float4 &acc, float w1, float w2, float w3, float w4,
                                           const float4 &a, const float4 &b, const float4 &c,
                                           const float4 &d) {
    acc.x += (w1 * a.x + w2 * b.x + w3 * c.x + w4 * d.x);
    acc.y += (w1 * a.y + w2 * b.y + w3 * c.y + w4 * d.y);
    acc.z += (w1 * a.z + w2 * b.z + w3 * c.z + w4 * d.z);
    acc.w += (w1 * a.w + w2 * b.w + w3 * c.w + w4 * d.w);
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



// One output row of the separable sweep (roi_geom.hpp): the x samples of
// every output column left to right, V(x) = column(x) computed once per
// distinct column (cl, ch reuse), store(pw, acc) per finished bin.
// Bins [pw0, pw1) of the row; V(x) of a column does not depend on which
// sweep computed it, so splitting a row into segments is bit-identical.
template <int SR, class Column, class Store>
__device__ __forceinline__ void sep_row_sweep(const RoiGeom &g, int pw0, int pw1, Column column,
                                              Store store) {
    const int W = g.W;
    const float inv = 1.f / g.count;  // count = SR*SR, a power of two for SR=2: exact
    int cl = -1, ch = -1;
    float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
    for (int pw = pw0; pw < pw1; ++pw) {
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
            acc.x += hx * va.x + lx * vb.x;
            acc.y += hx * va.y + lx * vb.y;
            acc.z += hx * va.z + lx * vb.z;
            acc.w += hx * va.w + lx * vb.w;
        }
        store(pw, make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv));
    }
}

template <bool NT>
__device__ __forceinline__ void store_bin(float *dst, float4 acc) {
    if (NT) {
        vf4 v = {acc.x, acc.y, acc.z, acc.w};
        __builtin_nontemporal_store(v, reinterpret_cast<vf4 *>(dst));
    } else {
        *reinterpret_cast<float4 *>(dst) = acc;
    }
}

// Separable NHWC forward (variant 8): see roi_geom.hpp for the row-tap /
// column decomposition it uses.
// NT: output rows are written once and never re-read by this launch; storing
// them non-temporal keeps them from evicting pyramid lines that overlapping
// RoIs on the same XCD are about to re-read from L2.
template <int SR, bool NT>
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_sep_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, int out_nhwc, float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float tile[];  // [C][P][P] (NCHW out)
    const int r = roi_order ? roi_order[blockIdx.x] : (int)blockIdx.x;
    if (r < 0 || r >= fa.R) return;  // malformed schedule entry: write nothing
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
    const int chunks = (C + 255) / 256;
    const int lane = lane_id();
    const int64_t rowstride = (int64_t)g.W * C;
    for (int u = wave_id(); u < P * chunks; u += num_waves()) {
        const int ph = u / chunks;
        const int ck = u - ph * chunks;
        const int c0 = ck * 256 + lane * 4;
        const bool active = c0 < C;
        const float *base = g.feat + (active ? c0 : 0);
        const RowTaps<SR> taps = row_taps<SR>(g, ph);
        float *orow = out + (((int64_t)r * P + ph) * P) * C + c0;
        auto column = [&](int x) -> float4 {
            return combine_column<SR>(taps,
                                      load_column<SR>(taps, base, rowstride, (int64_t)x * C));
        };
        sep_row_sweep<SR>(g, 0, P, column, [&](int pw, float4 acc) {
            if (!active) return;
            if (out_nhwc) {
                store_bin<NT>(orow + (int64_t)pw * C, acc);
            } else {
                float *t = tile + (int64_t)c0 * P * P + ph * P + pw;
                t[0] = acc.x;
                t[P * P] = acc.y;
                t[2 * P * P] = acc.z;
                t[3 * P * P] = acc.w;
            }
        });
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

// Separable NHWC forward, buffer-load form (variant 10): variant 8's sweep
// bin for bin (bit-identical), with the tap loads issued as
// buffer_load_dwordx4 against a per-RoI buffer resource (the RoI's image in
// its level): every address term but the lane's 16-byte channel offset is
// wave-uniform, so it travels in the scalar offset -- no per-lane 64-bit
// address arithmetic or pointer registers -- and a tap outside the image
// reads 0 from the hardware range check instead of faulting.
//
// segs > 1 splits every output row into `segs` runs of bins, one wave each:
// a RoI then occupies P*segs waves, so fewer RoIs are resident per XCD at the
// same occupancy and the union of their footprints stays closer to the 4 MiB
// L2 (tools/research/ra_l2_sim.py); each run re-reads at most one boundary
// column of its neighbour.
//
// SIMPLE: the default launch (C <= 256, segs = parts = 1) -- wave w computes
// output row w with no runtime divisions ahead of its first tap load.
template <int SR, bool NT, bool SIMPLE>
__global__ __launch_bounds__(1024) void roi_align_fpn_nhwc_sep_buf_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, int segs, int parts, float *__restrict__ out) {
    if (SIMPLE) {
        segs = 1;
        parts = 1;
    }
    // parts > 1: a RoI's units are spread over `parts` consecutive workgroups of
    // the same XCD (block b runs on XCD b % 8): b -> schedule position p.
    const int b = blockIdx.x;
    const int p = parts == 1 ? b : (b / 8 / parts) * 8 + (b & 7);
    const int part = parts == 1 ? 0 : (b / 8) % parts;
    if (p >= fa.R) return;
    const int r = roi_order ? roi_order[p] : p;
    if (r < 0 || r >= fa.R) return;  // malformed schedule entry: write nothing
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
    const int chunks = SIMPLE ? 1 : (C + 255) / 256;
    const int lane = lane_id();
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(g.feat), (short)0, g.H * g.W * C * 4, 0x00020000);
    const int rowbytes = g.W * C * 4, colbytes = C * 4;
    const int units = P * chunks * segs, per = (units + parts - 1) / parts;
    const int u1 = min(units, (part + 1) * per);
    for (int u = part * per + wave_id(); u < u1; u += num_waves()) {
        const int ph = SIMPLE ? u : u / (chunks * segs);
        const int rem = SIMPLE ? 0 : u - ph * chunks * segs;
        const int ck = SIMPLE ? 0 : rem / segs;
        const int sg = SIMPLE ? 0 : rem - ck * segs;
        const int c0 = ck * 256 + lane * 4;
        const bool active = c0 < C;
        const int voff = (active ? c0 : 0) * 4;
        const RowTaps<SR> taps = row_taps<SR>(g, ph);
        int rowoff[2 * SR];
#pragma unroll
        for (int k = 0; k < 2 * SR; ++k)
            rowoff[k] = __builtin_amdgcn_readfirstlane(taps.row[k] * rowbytes);
        float *orow = out + (((int64_t)r * P + ph) * P) * C + c0;
        auto column = [&](int x) -> float4 {
            const int xo = __builtin_amdgcn_readfirstlane(x * colbytes);
            TapCol<SR> c;
#pragma unroll
            for (int k = 0; k < 2 * SR; ++k)
                if (taps.alive[k])
                    c.f[k] = __builtin_bit_cast(
                        float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, rowoff[k] + xo, 0));
            return combine_column<SR>(taps, c);
        };
        const int pw0 = SIMPLE ? 0 : sg * P / segs, pw1 = SIMPLE ? P : (sg + 1) * P / segs;
        sep_row_sweep<SR>(g, pw0, pw1, column, [&](int pw, float4 acc) {
            if (active) store_bin<NT>(orow + (int64_t)pw * C, acc);
        });
    }
}

// Pipelined separable sweep (variant 11, round 5): variant 10's sweep bin for bin
// (bit-identical: the same V(x), the same per-bin sums in the same order), with
// the row's distinct columns listed up front so that column k + 2's tap loads
// are issued before column k is combined.  Variant 10 loads a column only when
// the sweep reaches it, each tap behind a wave-uniform branch, and drains
// (vmcnt 0) before combining it: <= 4 KiB in flight per wave, ~2.5 on average
// (2-3 distinct tap rows per output row), about half of what an HBM miss needs
// at 28 resident waves per CU (profiles/r05/roialign/README.md).  Here every
// column issues exactly NR (= the row's distinct tap rows, 2..4) loads -- a
// padding tap reads pixel (0, 0) and is skipped by the combine -- so the loop is
// branch-free and two columns' loads stay outstanding while one is combined.
//   Column list: lane 2 j + h holds sample j's column xl (h = 0) / xh (h = 1);
//   a valid lane's column is new iff it exceeds every earlier valid lane's
//   (prefix max; ballot + prefix count give its index), the list is strictly
//   increasing, and sample j is finished when column index(xh_j) is combined
//   (xl_j = xh_j - 1 is the entry before it, or xh_j itself when clamped at the
//   right edge).
typedef int ra_v4i __attribute__((ext_vector_type(4)));
typedef float ra_f4 __attribute__((ext_vector_type(4)));

// One 16-B tap load per lane against the RoI image's buffer descriptor (SGPR quad):
// vector offset = the lane's channel bytes, scalar offset = the tap's row + column.
// Inline asm so the compiler neither waits on it nor reuses its destination
// early; the tied operand keeps the slot in one register across the loop (an
// untied output let the register allocator copy a loop-carried slot at the back
// edge -- a read of the register before the load landed).  The caller counts
// vmcnt (ra_wait).
// The scalar offset usually comes straight from v_readfirstlane (a VALU write of
// an SGPR), which a VMEM instruction may read only 5 wait states later; the
// compiler's hazard recognizer does not look inside the asm, so the asm pads
// them itself (without it the load read the previous column's offset).
__device__ __forceinline__ void ra_load(ra_f4 &r, ra_v4i desc, int voff, int soff) {
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, %3 offen"
                 : "+v"(r)
                 : "v"(voff), "s"(desc), "s"(soff)
                 : "memory");
}
// All but the last N vector-memory ops retired; the slot's registers pass through
// so nothing reads them above the wait.
template <int N, int NR>
__device__ __forceinline__ void ra_wait(ra_f4 (&a)[NR]) {
    if constexpr (NR == 2)
        asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a[0]), "+v"(a[1]) : "i"(N) : "memory");
    else if constexpr (NR == 3)
        asm volatile("s_waitcnt vmcnt(%3)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]) : "i"(N) : "memory");
    else
        asm volatile("s_waitcnt vmcnt(%4)"
                     : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3])
                     : "i"(N)
                     : "memory");
}

template <int NR, bool NT, int D>
__device__ __forceinline__ void pipe_row(const RoiGeom &g, ra_v4i desc, int voff,
                                         const int (&roff)[4], const float (&rw)[4], int nr,
                                         const int *cols, int nc, int ns, int colbytes, int xh_k,
                                         int xinfo, float lxv, bool active, float *orow, int C) {
    constexpr int SR = 2;
    const float inv = 1.f / g.count;
    // a padding tap (r >= nr, or a column past the list) loads pixel (0, 0) of the
    // image -- in range, one cached line -- and is left out of the combine
    auto issue = [&](int k, ra_f4 (&sl)[NR]) {
        const bool live = k < nc;
        const int xo = __builtin_amdgcn_readfirstlane(live ? cols[k] * colbytes : 0);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const bool real = live && r < nr;
            ra_load(sl[r], desc, voff, __builtin_amdgcn_readfirstlane(real ? roff[r] + xo : 0));
        }
    };
    ra_f4 s0[NR], s1[NR], s2[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) s0[r] = s1[r] = s2[r] = ra_f4{0.f, 0.f, 0.f, 0.f};
    issue(0, s0);
    if (D == 2) issue(1, s1);
    float4 vprev = make_float4(0.f, 0.f, 0.f, 0.f), vcur = vprev, acc = vprev;
    int s = 0;  // the next sample to finish
    auto finish = [&](int k) {  // every sample whose xh column is k (or invalid) in order
        while (s < ns) {
            const int fin = __builtin_amdgcn_readlane(xh_k, 2 * s + 1);
            const int info = __builtin_amdgcn_readlane(xinfo, 2 * s + 1);  // 1 valid, 2 xl == xh
            if ((info & 1) && fin > k) break;
            if (info & 1) {
                const float lx = __builtin_bit_cast(
                    float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lxv), 2 * s + 1));
                const float hx = 1.f - lx;
                const float4 va = (info & 2) ? vcur : vprev;
                acc.x += hx * va.x + lx * vcur.x;
                acc.y += hx * va.y + lx * vcur.y;
                acc.z += hx * va.z + lx * vcur.z;
                acc.w += hx * va.w + lx * vcur.w;
            }
            if (s % SR == SR - 1) {
                if (active)
                    store_bin<NT>(orow + (int64_t)(s / SR) * C,
                                  make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv));
                acc = make_float4(0.f, 0.f, 0.f, 0.f);
            }
            ++s;
        }
    };
    // column k's loads were issued two columns ago; after them came column k + 1's
    // and k + 2's (NR each) and the bin stores of one finish: vmcnt(2 NR) retires
    // them (and at most those stores' worth of k + 1's loads early)
    auto consume = [&](int k, ra_f4 (&sl)[NR]) {
        ra_wait<D * NR>(sl);
        vprev = vcur;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int r = 0; r < NR; ++r) {  // combine_column's sum, tap order
            if (r < nr) {                // wave-uniform: padding taps are skipped
                v.x += rw[r] * sl[r][0];
                v.y += rw[r] * sl[r][1];
                v.z += rw[r] * sl[r][2];
                v.w += rw[r] * sl[r][3];
            }
        }
        vcur = v;
        finish(k);
    };
    if constexpr (D == 2) {
        for (int k = 0; k < nc; k += 3) {
            issue(k + 2, s2);
            consume(k, s0);
            if (k + 1 >= nc) break;
            issue(k + 3, s0);
            consume(k + 1, s1);
            if (k + 2 >= nc) break;
            issue(k + 4, s1);
            consume(k + 2, s2);
        }
    } else {  // one column ahead (fewer VGPRs, more resident waves)
        for (int k = 0; k < nc; k += 2) {
            issue(k + 1, s1);
            consume(k, s0);
            if (k + 1 >= nc) break;
            issue(k + 2, s0);
            consume(k + 1, s1);
        }
    }
    finish(0x7fffffff);  // samples past the last column: all invalid; their bins store 0
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no load outlives the row's slots
}

template <bool NT, int D>
__global__ __launch_bounds__(1024) void roi_align_fpn_nhwc_sep_pipe_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, float *__restrict__ out) {
    constexpr int SR = 2;
    __shared__ int s_cols[16][64];
    const int b = blockIdx.x;
    if (b >= fa.R) return;
    const int r = roi_order ? roi_order[b] : b;
    if (r < 0 || r >= fa.R) return;  // malformed schedule entry: write nothing
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
    const int lane = lane_id(), wave = wave_id();
    // raw buffer descriptor (stride 0, range = the RoI's image), as
    // __builtin_amdgcn_make_buffer_rsrc builds it for variant 10
    const uint64_t fb = (uint64_t)(uintptr_t)g.feat;
    ra_v4i desc;
    desc.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)fb);
    desc.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(fb >> 32) & 0xffff);
    desc.z = __builtin_amdgcn_readfirstlane(g.H * g.W * C * 4);
    desc.w = 0x00020000;
    const int rowbytes = g.W * C * 4, colbytes = C * 4;
    const int c0 = lane * 4;
    const bool active = c0 < C;
    const int voff = (active ? c0 : 0) * 4;
    const int ns = P * SR;  // samples per row (<= 32: two column candidates per lane pair)
    // the row's x geometry does not depend on the row: sample j = lane >> 1
    const int j = lane >> 1;
    int xl = 0, xh = 0;
    float lx = 0.f;
    bool valid = false;
    if (j < ns) {
        const int pw = j / SR, ix = j % SR;
        float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
        valid = !(x < -1.0f || x > (float)g.W);
        if (x <= 0) x = 0;
        xl = (int)x;
        if (xl >= g.W - 1) { xh = xl = g.W - 1; x = (float)xl; } else xh = xl + 1;
        lx = x - xl;
    }
    // the lanes' columns are NOT monotone (xl_1 < xh_0 when two samples share a
    // pixel pair), but each valid lane's column is a new one iff it exceeds every
    // earlier valid lane's: an exclusive prefix max over the wave
    const int cand = (lane & 1) ? xh : xl;
    int incl = valid ? cand : -1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl = incl > v ? incl : v;
    }
    int excl = __shfl_up(incl, 1);
    if (lane == 0) excl = -1;
    const bool distinct = valid && cand > excl;
    const uint64_t dm = ballot(distinct);
    const int rank = __popcll(dm & ((1ull << lane) - 1ull));
    const int nc = __popcll(dm);
    const int xh_k = distinct ? rank : rank - 1;  // this lane's column index in the list
    const int xinfo = (valid ? 1 : 0) | (xl == xh ? 2 : 0);
    if (distinct) s_cols[wave][rank] = cand;
    __builtin_amdgcn_wave_barrier();
    for (int ph = wave; ph < P; ph += num_waves()) {
        const RowTaps<SR> taps = row_taps<SR>(g, ph);
        int roff[4] = {0, 0, 0, 0}, nr = 0;
        float rw[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 2 * SR; ++k)
            if (taps.alive[k]) {  // wave-uniform; the alive taps in tap order
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (q == nr) {
                        roff[q] = __builtin_amdgcn_readfirstlane(taps.row[k] * rowbytes);
                        rw[q] = taps.w[k];
                    }
                ++nr;
            }
        float *orow = out + (((int64_t)r * P + ph) * P) * C + c0;
        if (nr <= 2)
            pipe_row<2, NT, D>(g, desc, voff, roff, rw, nr, s_cols[wave], nc, ns, colbytes, xh_k,
                                xinfo, lx, active, orow, C);
        else if (nr == 3)
            pipe_row<3, NT, D>(g, desc, voff, roff, rw, nr, s_cols[wave], nc, ns, colbytes, xh_k,
                                xinfo, lx, active, orow, C);
        else
            pipe_row<4, NT, D>(g, desc, voff, roff, rw, nr, s_cols[wave], nc, ns, colbytes, xh_k,
                                xinfo, lx, active, orow, C);
    }
}

template <int P, int SR, int D>
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int R, int sr, int rows_per_block, int out_nhwc,
    float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float tile[];
    const int r = roi_order ? roi_order[blockIdx.x] : (int)blockIdx.x;
    if (r < 0 || r >= fa.R) return;  // malformed schedule entry: write nothing
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
    int64_t n = (int64_t)R * C * PH * PW;
    if (n == 0) return VD_OK;
    hipLaunchKernelGGL(roi_align_fwd_nchw_kernel, dim3(grid_1d(n, 256)), dim3(256), 0, s, n, feat,
                       scale, B, H, W, C, PH, PW, sr, rois, out);
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
    if (!out_nhwc && (int64_t)rows * row_bytes > VD_LDS_BYTES) return VD_ERR_SHAPE;
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
    // 10: separable kernel with buffer loads (product default, NHWC out; RoIAlign
    //    tolerance 1e-4 vs the reference's per-sample order); 8: the same sweep
    //    with global loads (bit-identical to 10; also the NCHW-out path);
    //    11 / 13: variant 10's sweep pipelined two / one column(s) ahead (bit-
    //    identical to 10, 8-9 % slower at half the occupancy: profiles/r05/roialign/);
    //    3: bit-exact row kernel (the reference's per-sample arithmetic order).  Round-2 alternatives (XCD channel slices,
    //    tile-binned LDS windows, a pipelined column ring) are in tools/research/
    //    with their measurements (profiles/r02_roialign/README.md).
    return e ? atoi(e) : 10;
}

static int launch_sep_buf(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                          const int *order, int R, int P, float *out, hipStream_t s) {
    for (int l = 0; l < fa.L; ++l)  // 32-bit buffer offsets: every image of a level < 2 GiB
        if ((int64_t)fa.H[l] * fa.W[l] * C * 4 >= (1ll << 31)) return VD_ERR_SHAPE;
    // Row segments x workgroups per RoI (VOSDET_RA_SEGS / VOSDET_RA_PARTS, both 1
    // in the product): bit-identical schedules that keep fewer RoIs resident per
    // XCD.  Measured (profiles/r02_roialign/README.md): fabric reads fall from
    // 1.12 to 0.71 GB (1.04x the algorithmic bytes) at segs = parts = 4, but the
    // launch slows from 301 to 364 us -- the extra boundary loads cost more than
    // the L2 hits save, the kernel being bound by its vector-memory wave loads.
    const char *es = getenv("VOSDET_RA_SEGS");
    int segs = es ? atoi(es) : 1;
    if (segs < 1 || segs > P) segs = 1;
    const char *ep = getenv("VOSDET_RA_PARTS");
    int parts = ep ? atoi(ep) : 1;
    if (parts < 1) parts = 1;
    const int units = P * ((C + 255) / 256) * segs;
    int waves = (units + parts - 1) / parts;
    if (waves > 16) waves = 16;
    if (segs == 1 && parts == 1 && waves > 8) waves = 8;
    const int nblk = parts == 1 ? R : (R + 7) / 8 * 8 * parts;
    if (segs == 1 && parts == 1 && C <= 256 && getenv("VOSDET_RA_GENERAL") == nullptr)
        hipLaunchKernelGGL((roi_align_fpn_nhwc_sep_buf_kernel<2, true, true>), dim3(nblk),
                           dim3(64 * waves), 0, s, fa, C, rois, lvl, order, P, 1, 1, out);
    else
        hipLaunchKernelGGL((roi_align_fpn_nhwc_sep_buf_kernel<2, true, false>), dim3(nblk),
                           dim3(64 * waves), 0, s, fa, C, rois, lvl, order, P, segs, parts, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

static int launch_sep_pipe(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                           const int *order, int R, int P, float *out, hipStream_t s,
                           bool depth1) {
    if (C > 256 || P > 16) return VD_ERR_SHAPE;
    for (int l = 0; l < fa.L; ++l)  // 32-bit buffer offsets: every image of a level < 2 GiB
        if ((int64_t)fa.H[l] * fa.W[l] * C * 4 >= (1ll << 31)) return VD_ERR_SHAPE;
    const int waves = P < 8 ? P : 8;
    if (depth1)
        hipLaunchKernelGGL((roi_align_fpn_nhwc_sep_pipe_kernel<true, 1>), dim3(R),
                           dim3(64 * waves), 0, s, fa, C, rois, lvl, order, P, out);
    else
        hipLaunchKernelGGL((roi_align_fpn_nhwc_sep_pipe_kernel<true, 2>), dim3(R),
                           dim3(64 * waves), 0, s, fa, C, rois, lvl, order, P, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

static int launch_sep(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                      const int *order, int R, int P, int out_nhwc, float *out, hipStream_t s) {
    const size_t lds = out_nhwc ? 0 : (size_t)C * P * P * 4;
    if (lds > VD_LDS_BYTES) return VD_ERR_SHAPE;
    int waves = P * ((C + 255) / 256);
    if (waves > 8) waves = 8;
    // non-temporal output stores (297 us vs 306 us write-back on the 8-frame launch)
    hipLaunchKernelGGL((roi_align_fpn_nhwc_sep_kernel<2, true>), dim3(R), dim3(64 * waves), lds,
                       s, fa, C, rois, lvl, order, P, out_nhwc, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}


int launch_roi_align_fpn_nhwc(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                              const int *order, int R, int PH, int PW, int sr, int out_nhwc,
                              float *out, hipStream_t s) {
    if (R == 0) return VD_OK;
    if (C % 4 != 0) return VD_ERR_SHAPE;
    const int variant = roialign_variant();
    if (out_nhwc) {  // product path: [R][P][P][C] written straight from registers
        if ((variant == 11 || variant == 13) && sr == 2 && PH == PW) {  // pipelined gathers
            const int st = launch_sep_pipe(fa, C, rois, lvl, order, R, PH, out, s, variant == 13);
            if (st != VD_ERR_SHAPE) return st;
        }
        if (variant >= 10 && sr == 2 && PH == PW) {  // register gathers
            const int st = launch_sep_buf(fa, C, rois, lvl, order, R, PH, out, s);
            if (st != VD_ERR_SHAPE) return st;
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
    if (variant >= 8 && sr == 2 && PH == PW && (int64_t)C * PH * PW * 4 <= VD_LDS_BYTES)
        return launch_sep(fa, C, rois, lvl, order, R, PH, 0, out, s);
    if (PH == PW && (PH == 7 || PH == 14)) {
        const bool unrolled = sr == 2 && variant >= 2;
        if (PH == 7 && unrolled)
            return variant == 3 ? launch_rows<7, 2, 2>(fa, C, rois, lvl, order, R, sr, out, s)
                                : launch_rows<7, 2, 3>(fa, C, rois, lvl, order, R, sr, out, s);
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
