// Round 2, variant 50 v2 (profiles/r02_roialign/README.md): tile-binned
// RoIAlign with LDS-DMA window fills and one-unit-per-lane-group sweeps.
// 520 us per launch (tile kernel 468 us, VALU-bound: 162 M instructions, 2.1x
// variant 8's) vs 304 us for the product kernel, although its fabric traffic
// is 1.07x the algorithmic bytes (variant 8: 1.39x).  Bit-identical to
// variant 8 on the GPU tests.  NOT part of libvosdet.so; it compiled as
// vosdetectron_amd/csrc/roi_align_tiled.hip with roi_geom.hpp and was reached
// through VOSDET_ROIALIGN_VARIANT=50 (launch_roi_align_fpn_tiled_own_ws).
//
// Tile-binned RoIAlign forward (FPN, NHWC in and out, sampling ratio 2),
// round-2 variant 50 v2 (VOSDET_ROIALIGN_VARIANT=50; see profiles/r02_roialign).
//
// Reference semantics: lib/modeling/roi_xfrom/roi_align/src/roi_align_kernel.cu
// :16-121 (Caffe2 RoIAlign).  Every output bin is computed in exactly the order
// of the separable product kernel (roi_align.hip, roi_align_fpn_nhwc_sep_kernel):
// V(x) = combine_column(taps, F(taps, x)) over the merged tap rows, swept left
// to right with the same (cl, ch) column reuse, acc += hx V(xl) + lx V(xh) per
// sample, times 1/count -- so the two kernels are bit-identical.
//
// Why: the product kernel fetches every RoI's footprint separately, ~2.9 GB of
// 1 KiB wave loads for 0.66 GB of distinct pyramid bytes at the section-8(d)
// workload (the RoIs' footprints overlap 4.5x).  Here the overlap is served
// from LDS: a counting sort of "units" (one RoI output row x a run of its
// columns whose taps fall in one 16 x 16 level tile) by tile, then one
// workgroup per (tile, 32-channel slice) stages the tile's (16+4)^2-pixel
// window with LDS-DMA (global_load_lds_dwordx4, no VGPR round trip), and each
// 8-lane group sweeps one unit from LDS.
//   1. roi_units     one lane per (RoI, output row): tap-row tile, column runs,
//                    slot = atomicAdd(count[tile]); taps overrunning the window
//                    or dead rows/columns -> fallback bins.
//   2. tile_scan     exclusive prefix sum of the tile counts (one workgroup).
//   3. unit_scatter  list[offset[tile] + slot] = unit.
//   4. tile_units    workgroup (tile, slice): window fill, barrier, units.
//                    Slice s = block % 8 lands on XCD s, so an XCD only caches
//                    its 128 B of each pixel and the window halos hit its L2.
//   5. fallback      one wave per fallback bin, taps from global memory.
// Steps 4 and 5 write disjoint bins; nothing accumulates across workgroups, so
// the result is deterministic.
#include <mutex>

#include "common.hpp"
#include "roi_geom.hpp"
#include "vosdet_internal.hpp"

namespace vd {

namespace {

constexpr int kTile = 16, kHalo = 4, kWin = kTile + kHalo;
constexpr int kWinPix = (kWin * kWin + 7) / 8 * 8;  // glds moves 8 pixels per wave
constexpr int kSlice = 32;                           // channels per workgroup (128 B/pixel)
constexpr int kMaxP = 16;                            // pooled sizes served by this path
constexpr int kThreads = 256;

struct TileGrid {
    int ty[VD_MAX_LEVELS], tx[VD_MAX_LEVELS];
    int base[VD_MAX_LEVELS + 1];  // first tile index of level l (all images)
};

template <int SR>
__device__ __forceinline__ bool row_extent(const RowTaps<SR> &t, int &y0, int &y1) {
    y0 = 1 << 30;
    y1 = -1;
#pragma unroll
    for (int k = 0; k < 2 * SR; ++k)
        if (t.alive[k]) {
            y0 = min(y0, t.row[k]);
            y1 = max(y1, t.row[k]);
        }
    return y1 >= 0;
}

// Column extent of output column pw (the x samples exactly as the separable
// kernel computes them); false: no in-range sample, the bin pools to 0.
template <int SR>
__device__ __forceinline__ bool col_extent(const RoiGeom &g, int pw, int &x0, int &x1) {
    x0 = 1 << 30;
    x1 = -1;
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
        float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
        if (x < -1.0f || x > (float)g.W) continue;
        if (x <= 0) x = 0;
        int xl = (int)x, xh;
        if (xl >= g.W - 1) xh = xl = g.W - 1; else xh = xl + 1;
        x0 = min(x0, xl);
        x1 = max(x1, xh);
    }
    return x1 >= 0;
}

// 1. One lane per (RoI, output row).
template <int SR>
__global__ __launch_bounds__(256) void roi_units_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level, int P,
    TileGrid tg, int *__restrict__ count, int4 *__restrict__ unit, int *__restrict__ nunit,
    int *__restrict__ fb_count, int *__restrict__ fb_list) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= fa.R * P) return;
    const int r = i / P, ph = i - r * P;
    const int li = roi_level ? roi_level[r] : 0;
    const float *roi = rois + (int64_t)r * 5;
    const int b = (int)roi[0];
    const bool roi_ok = li >= 0 && li < fa.L && b >= 0 && b < fa.B;
    const RoiGeom g = roi_geom(fa, C, roi, li, P, P, SR);
    int y0, y1;
    const bool live = roi_ok && row_extent<SR>(row_taps<SR>(g, ph), y0, y1);
    const int ty = live ? y0 / kTile : -1;
    const bool row_ok = live && y1 < ty * kTile + kWin;
    int4 *my = unit + (int64_t)i * P;
    int n = 0, prev = -1, pw0 = 0;
    auto emit = [&](int tx, int a, int e) {
        const int tile = tg.base[li] + (b * tg.ty[li] + ty) * tg.tx[li] + tx;
        my[n++] = make_int4(r, ph | (a << 8) | (e << 16), tile, atomicAdd(count + tile, 1));
    };
    auto fallback = [&](int pw) { fb_list[atomicAdd(fb_count, 1)] = (r * P + ph) * P + pw; };
    for (int pw = 0; pw < P; ++pw) {
        int tx = -1, x0, x1;
        if (row_ok && col_extent<SR>(g, pw, x0, x1)) {
            tx = x0 / kTile;
            if (x1 >= tx * kTile + kWin) tx = -1;
        }
        if (tx != prev) {
            if (prev >= 0) emit(prev, pw0, pw - 1);
            pw0 = pw;
            prev = tx;
        }
        if (tx < 0) fallback(pw);
    }
    if (prev >= 0) emit(prev, pw0, P - 1);
    nunit[i] = n;
}

// 2. Exclusive prefix sum of count[0..T) into offset[0..T) (one workgroup).
__global__ __launch_bounds__(1024) void tile_scan_kernel(const int *__restrict__ count, int T,
                                                          int *__restrict__ offset) {
    __shared__ int part[1024];
    const int t = threadIdx.x, nt = blockDim.x;
    const int per = (T + nt - 1) / nt;
    const int a = min(t * per, T), e = min(a + per, T);
    int s = 0;
    for (int i = a; i < e; ++i) s += count[i];
    part[t] = s;
    __syncthreads();
    for (int off = 1; off < nt; off <<= 1) {
        const int v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = part[t] - s;
    for (int i = a; i < e; ++i) {
        offset[i] = run;
        run += count[i];
    }
}

// 3. Units into per-tile lists (one lane per (RoI, output row)).
__global__ __launch_bounds__(256) void unit_scatter_kernel(int RP, int P,
                                                            const int4 *__restrict__ unit,
                                                            const int *__restrict__ nunit,
                                                            const int *__restrict__ offset,
                                                            int2 *__restrict__ list) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= RP) return;
    const int n = nunit[i];
    for (int k = 0; k < n; ++k) {
        const int4 u = unit[(int64_t)i * P + k];
        list[offset[u.z] + u.w] = make_int2(u.x, u.y);
    }
}

// 4. Workgroup (tile, slice): LDS-DMA window fill, then 8-lane groups sweep the
// tile's units from LDS.
template <int SR, bool NT>
__global__ __launch_bounds__(kThreads) void tile_units_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, int P, TileGrid tg, int nslice,
    const int *__restrict__ count, const int *__restrict__ offset, const int2 *__restrict__ list,
    float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) float win[kWinPix * kSlice];  // 51.2 KB
    const int tile = blockIdx.x / nslice, s = blockIdx.x - tile * nslice;
    const int n = count[tile];
    if (n == 0) return;
    int li = 0;
    while (li + 1 < fa.L && tile >= tg.base[li + 1]) ++li;
    const int local = tile - tg.base[li];
    const int per_img = tg.ty[li] * tg.tx[li];
    const int b = local / per_img, rem = local - b * per_img;
    const int ty = rem / tg.tx[li], tx = rem - ty * tg.tx[li];
    const int H = fa.H[li], W = fa.W[li];
    const int y0 = ty * kTile, x0 = tx * kTile;
    const int lane = lane_id(), q = lane & 7;
    const int wv = __builtin_amdgcn_readfirstlane(wave_id());
    {
        const float *src = fa.feat[li] + (int64_t)b * H * W * C + s * kSlice + q * 4;
        for (int p8 = wv * 8; p8 < kWinPix; p8 += (kThreads / 64) * 8) {
            const int pix = p8 + (lane >> 3);
            const int yy = pix / kWin, xx = pix - yy * kWin;
            const int gy = min(y0 + yy, H - 1), gx = min(x0 + xx, W - 1);  // clamped: unused
            __builtin_amdgcn_global_load_lds(
                (const void *)(src + ((int64_t)gy * W + gx) * C),
                (__attribute__((address_space(3))) void *)(win + p8 * kSlice), 16, 0, 0);
        }
    }
    const int off = offset[tile];
    const float inv = 1.f / (float)(SR * SR);
    const float *wq = win + q * 4;
    __syncthreads();  // window resident
    for (int ub = wv * 8; ub < n; ub += (kThreads / 64) * 8) {
        const int u = ub + (lane >> 3);
        if (u >= n) continue;
        const int2 en = list[off + u];
        const int r = en.x, ph = en.y & 255, pw0 = (en.y >> 8) & 255, pw1 = (en.y >> 16) & 255;
        const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
        const RowTaps<SR> taps = row_taps<SR>(g, ph);
        int roff[2 * SR];
#pragma unroll
        for (int k = 0; k < 2 * SR; ++k) roff[k] = (taps.row[k] - y0) * kWin * kSlice;
        auto column = [&](int x) -> float4 {
            TapCol<SR> c;
            const float *cp = wq + (x - x0) * kSlice;
#pragma unroll
            for (int k = 0; k < 2 * SR; ++k)
                if (taps.alive[k]) c.f[k] = *reinterpret_cast<const float4 *>(cp + roff[k]);
            return combine_column<SR>(taps, c);
        };
        int cl = -1, ch = -1;
        float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
        float *dst = out + (((int64_t)r * P + ph) * P) * C + s * kSlice + q * 4;
        for (int pw = pw0; pw <= pw1; ++pw) {
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int ix = 0; ix < SR; ++ix) {
                float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
                if (x < -1.0f || x > (float)W) continue;
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
            acc = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
            if (NT) {
                vf4 v = {acc.x, acc.y, acc.z, acc.w};
                __builtin_nontemporal_store(v, reinterpret_cast<vf4 *>(dst + (int64_t)pw * C));
            } else {
                *reinterpret_cast<float4 *>(dst + (int64_t)pw * C) = acc;
            }
        }
    }
}

// 5. One wave per fallback bin, every channel, taps from global memory; a bin
// with no in-range sample (or an out-of-range RoI) writes zeros.  Grid-stride
// over the device-side count, so every wave reaches the exit.
template <int SR>
__global__ __launch_bounds__(256) void fallback_bins_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level, int P,
    const int *__restrict__ fb_count, const int *__restrict__ fb_list, float *__restrict__ out) {
    const int n = *fb_count;
    const int lane = lane_id();
    const int waves = gridDim.x * num_waves();
    for (int i = blockIdx.x * num_waves() + wave_id(); i < n; i += waves) {
        const int bin = fb_list[i];
        const int PP = P * P;
        const int r = bin / PP, rr = bin - r * PP;
        const int ph = rr / P, pw = rr - ph * P;
        const int li = roi_level ? roi_level[r] : 0;
        const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
        const RowTaps<SR> taps = row_taps<SR>(g, ph);
        const int64_t rowstride = (int64_t)g.W * C;
        for (int c0 = lane * 4; c0 < C; c0 += 256) {
            const float *base = g.feat + c0;
            auto column = [&](int x) -> float4 {
                return combine_column<SR>(taps,
                                          load_column<SR>(taps, base, rowstride, (int64_t)x * C));
            };
            // column values are pure functions of x, so starting the sweep
            // cache at this bin gives the product kernel's values exactly
            int cl = -1, ch = -1;
            float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va, acc = va;
#pragma unroll
            for (int ix = 0; ix < SR; ++ix) {
                float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
                if (x < -1.0f || x > (float)g.W) continue;
                if (x <= 0) x = 0;
                int xl = (int)x, xh;
                if (xl >= g.W - 1) { xh = xl = g.W - 1; x = (float)xl; } else xh = xl + 1;
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
            const float inv = 1.f / g.count;
            *reinterpret_cast<float4 *>(out + (int64_t)bin * C + c0) =
                make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
        }
    }
}

TileGrid tile_grid(const FpnLevels &fa) {
    TileGrid tg = {};
    int base = 0;
    for (int l = 0; l < fa.L; ++l) {
        tg.ty[l] = (fa.H[l] + kTile - 1) / kTile;
        tg.tx[l] = (fa.W[l] + kTile - 1) / kTile;
        tg.base[l] = base;
        base += fa.B * tg.ty[l] * tg.tx[l];
    }
    tg.base[fa.L] = base;
    return tg;
}

size_t align256(size_t n) { return (n + 255) & ~(size_t)255; }

}  // namespace

size_t roi_align_tiled_workspace_bytes(const FpnLevels &fa, int R, int P) {
    const TileGrid tg = tile_grid(fa);
    const size_t T = (size_t)tg.base[fa.L];
    const size_t RP = (size_t)R * P;
    return align256(T * 4) * 2 + align256(RP * P * 16) + align256(RP * 4) + align256(RP * P * 8) +
           align256(RP * P * 4) + 256;
}

bool roi_align_tiled_supported(int C, int PH, int PW, int sr, int out_nhwc) {
    return out_nhwc && sr == 2 && PH == PW && PH <= kMaxP && C % kSlice == 0;
}

int launch_roi_align_fpn_tiled(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                               int R, int P, int sr, float *out, void *ws, size_t ws_bytes,
                               hipStream_t s) {
    if (R == 0) return VD_OK;
    if (!roi_align_tiled_supported(C, P, P, sr, 1)) return VD_ERR_SHAPE;
    if (!ws || ws_bytes < roi_align_tiled_workspace_bytes(fa, R, P)) return VD_ERR_WORKSPACE;
    const TileGrid tg = tile_grid(fa);
    const int T = tg.base[fa.L];
    const size_t RP = (size_t)R * P;
    char *p = (char *)ws;
    int *count = (int *)p;
    p += align256((size_t)T * 4);
    int *offset = (int *)p;
    p += align256((size_t)T * 4);
    int4 *unit = (int4 *)p;
    p += align256(RP * P * 16);
    int *nunit = (int *)p;
    p += align256(RP * 4);
    int2 *list = (int2 *)p;
    p += align256(RP * P * 8);
    int *fb_list = (int *)p;
    p += align256(RP * P * 4);
    int *fb_count = (int *)p;
    if (hipMemsetAsync(count, 0, (size_t)T * 4, s) != hipSuccess) return VD_ERR_LAUNCH;
    if (hipMemsetAsync(fb_count, 0, 4, s) != hipSuccess) return VD_ERR_LAUNCH;
    const unsigned blk = (unsigned)((RP + 255) / 256);
    hipLaunchKernelGGL((roi_units_kernel<2>), dim3(blk), dim3(256), 0, s, fa, C, rois, lvl, P, tg,
                       count, unit, nunit, fb_count, fb_list);
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, count, T, offset);
    hipLaunchKernelGGL(unit_scatter_kernel, dim3(blk), dim3(256), 0, s, (int)RP, P, unit, nunit,
                       offset, list);
    const int nslice = C / kSlice;
    hipLaunchKernelGGL((tile_units_kernel<2, true>), dim3((unsigned)((int64_t)T * nslice)),
                       dim3(kThreads), 0, s, fa, C, rois, P, tg, nslice, count, offset, list, out);
    hipLaunchKernelGGL((fallback_bins_kernel<2>), dim3(256), dim3(256), 0, s, fa, C, rois, lvl, P,
                       fb_count, fb_list, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// Variant-50 experiments reach the tiled path through vd_roi_align_fpn_forward
// with a library-held workspace (grown on demand; not stream-ordered across
// concurrent streams -- experiment use only).
int launch_roi_align_fpn_tiled_own_ws(const FpnLevels &fa, int C, const float *rois,
                                      const int *lvl, int R, int P, int sr, float *out,
                                      hipStream_t s) {
    static std::mutex mu;
    static void *buf = nullptr;
    static size_t cap = 0;
    std::lock_guard<std::mutex> lk(mu);
    const size_t need = roi_align_tiled_workspace_bytes(fa, R, P);
    if (need > cap) {
        if (buf && hipStreamSynchronize(s) != hipSuccess) return VD_ERR_LAUNCH;
        if (buf) (void)hipFree(buf);
        buf = nullptr;
        cap = 0;
        if (hipMalloc(&buf, need) != hipSuccess) return VD_ERR_LAUNCH;
        cap = need;
    }
    return launch_roi_align_fpn_tiled(fa, C, rois, lvl, R, P, sr, out, buf, cap, s);
}

}  // namespace vd
