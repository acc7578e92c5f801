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
//    FPN level.  A 64-lane wave owns 256 channels of one output row (ph): each
//    lane loads float4 (16 B) of the 4 bilinear taps, so every tap is a fully
//    coalesced 1 KiB wave load of one pyramid pixel.  The sample geometry is
//    wave-uniform (scalar), so re-use of the previous sample's tap columns along
//    x is a uniform branch, not divergence.  Results are transposed through LDS
//    into the reference's [R][C][P][P] output and written as contiguous rows.
//
// Arithmetic order (sample positions, weights, w1*v1+w2*v2+w3*v3+w4*v4, the
// iy-major accumulation and the final /count) is the reference's, and the file
// is compiled without FMA contraction, so results are bit-identical to the C
// restatement in oracle/roi_ops.c.
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

template <int P>
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int R, int sr, int rows_per_block,
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
        nhwc_row<P>(g, C, row0 + prow, active ? c0 : 0, active, acc);
        if (active) {
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

template <int P>
static int launch_rows(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                       const int *order, int R, int sr, float *out, hipStream_t s) {
    const int row_bytes = C * P * 4;
    int rows = kTileBudget / row_bytes;
    if (rows < 1) rows = 1;
    if (rows > P) rows = P;
    if ((int64_t)rows * row_bytes > 160 * 1024) return VD_ERR_SHAPE;
    const int chunks = (C + 255) / 256;
    int waves = rows * chunks;
    if (waves > 8) waves = 8;  // __launch_bounds__(512): <= 256 VGPRs, acc[P] stays in registers
    const size_t lds = (size_t)rows * row_bytes;
    dim3 grid(R, (P + rows - 1) / rows);
    hipLaunchKernelGGL(roi_align_fpn_nhwc_kernel<P>, grid, dim3(64 * waves), lds, s, fa, C, rois,
                       lvl, order, R, sr, rows, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int launch_roi_align_fpn_nhwc(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                              const int *order, int R, int PH, int PW, int sr, float *out,
                              hipStream_t s) {
    if (R == 0) return VD_OK;
    if (C % 4 != 0) return VD_ERR_SHAPE;
    if (PH == PW) {
        switch (PH) {
            case 7: return launch_rows<7>(fa, C, rois, lvl, order, R, sr, out, s);
            case 14: return launch_rows<14>(fa, C, rois, lvl, order, R, sr, out, s);
            default: break;
        }
    }
    if (order) return VD_ERR_ARG;  // the generic path writes in RoI order only
    hipLaunchKernelGGL(roi_align_fpn_nhwc_generic_kernel, dim3(R), dim3(256), 0, s, fa, C, rois,
                       lvl, R, PH, PW, sr, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
