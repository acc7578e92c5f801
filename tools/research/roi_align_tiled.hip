// Round 2, variant 50c (profiles/r02_roialign/README.md): tile-binned RoIAlign.
// 524 us per launch (tile kernel 469 us + binning ~55 us) vs 300 us for the
// product separable kernel; kept as the record of the experiment, NOT part of
// libvosdet.so.  It compiled as vosdetectron_amd/csrc/roi_align_tiled.hip with
// roi_geom.hpp and was reached through vd_roi_align_fpn_forward_ws.
//
// Tile-binned RoIAlign forward (FPN, NHWC in and out, compile-time sampling
// ratio): the inter-RoI footprint overlap (4.5x at the §8d workload) is served
// from LDS instead of being re-fetched per RoI.
//
// Reference semantics: lib/modeling/roi_xfrom/roi_align/src/roi_align_kernel.cu
// :16-121 (Caffe2 RoIAlign).  Every output bin is computed in exactly the order
// of the separable product kernel (roi_align.hip, roi_align_fpn_nhwc_sep_kernel):
// V(x) = sum_k w_k F(row_k, x) over the merged tap rows, acc += hx V(xl) +
// lx V(xh) per sample, times 1/count -- so the two kernels' outputs are
// bit-identical and the tolerance story (1e-4 vs the reference's per-sample
// order) is unchanged.
//
// Work decomposition (a counting sort of output bins by the level tile their
// taps fall in, then one workgroup per (tile, channel slice)):
//   1. bin_tiles   one lane per output bin (RoI, ph, pw): the bin's tap box;
//                  its anchor tile = (first tap row, first tap column) / 16 on
//                  its image and level; slot = atomicAdd(count[tile]).  Bins
//                  whose taps overrun the tile's 20 x 20 window (bins wider than
//                  ~8 level pixels) and bins with no in-range sample go to a
//                  fallback list.
//   2. tile_scan   exclusive prefix sum of the tile counts (one workgroup).
//   3. bin_scatter list[offset[tile] + slot] = bin.
//   4. tile_bins   workgroup (tile, slice s): the 20 x 20 window of 32
//                  channels (51 KB) is staged once in LDS, then every bin of the
//                  tile is computed from LDS (lane group of 8 = one bin, lane =
//                  4 channels).  Slice s = block % 8 lands on XCD s, so each XCD
//                  only ever caches its 128 B of a pixel and the windows'
//                  overlap (halo) re-reads hit its L2.
//   5. fallback    one wave per fallback bin, taps from global memory.
// Steps 4 and 5 write disjoint bins; nothing is accumulated across workgroups,
// so the result is deterministic.
#include "common.hpp"
#include "roi_geom.hpp"
#include "vosdet_internal.hpp"

namespace vd {

static constexpr int kTile = 16, kHalo = 3, kWin = kTile + kHalo;
static constexpr int kSlice = 32;    // channels per workgroup (128 B of a pixel)
static constexpr int kMaxEnt = 32;   // (tile, rectangle) entries per RoI, else fallback
static constexpr int kEntBatch = 8;  // entries staged per pass of a tile workgroup
static constexpr int kMaxP = 16;     // pooled size supported by the tiled path

struct TileGrid {
    int ty[VD_MAX_LEVELS], tx[VD_MAX_LEVELS];
    int base[VD_MAX_LEVELS + 1];  // first tile index of level l (all images)
};

// Tap-row extent of output row ph (false: no live tap, the row pools to 0).
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

struct ColSamples {
    int xl[2], xh[2];
    float lx[2];
    bool ok[2];
};

// The SR (<= 2) x samples of output column pw, exactly as the separable kernel.
template <int SR>
__device__ __forceinline__ ColSamples col_samples(const RoiGeom &g, int pw) {
    ColSamples c;
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
        float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
        c.ok[ix] = !(x < -1.0f || x > (float)g.W);
        if (x <= 0) x = 0;
        int xl = (int)x, xh;
        if (xl >= g.W - 1) { xh = xl = g.W - 1; x = (float)xl; } else xh = xl + 1;
        c.xl[ix] = xl;
        c.xh[ix] = xh;
        c.lx[ix] = x - xl;
    }
    return c;
}

template <int SR>
__device__ __forceinline__ bool col_extent(const ColSamples &c, int &x0, int &x1) {
    x0 = 1 << 30;
    x1 = -1;
#pragma unroll
    for (int ix = 0; ix < SR; ++ix)
        if (c.ok[ix]) {
            x0 = min(x0, c.xl[ix]);
            x1 = max(x1, c.xh[ix]);
        }
    return x1 >= 0;
}

// 1. One lane per RoI: the tile of every output row (by its first tap row) and
// column (by its first tap column); runs of rows / columns with the same tile
// whose taps fit that tile's 20 x 20 window give (tile, rectangle) entries.
// Rows / columns that are dead (pool to 0) or overrun the window make their
// bins fallback bins.
template <int SR>
__global__ __launch_bounds__(256) void roi_tiles_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level, int P,
    TileGrid tg, int *__restrict__ count, int4 *__restrict__ ent, int *__restrict__ nent,
    int *__restrict__ fb_count, int *__restrict__ fb_list) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= fa.R) return;
    const int li = roi_level ? roi_level[r] : 0;
    const float *roi = rois + (int64_t)r * 5;
    const int b = (int)roi[0];
    const bool roi_ok = li >= 0 && li < fa.L && b >= 0 && b < fa.B;
    const RoiGeom g = roi_geom(fa, C, roi, li, P, P, SR);
    int rty[kMaxP], ctx[kMaxP];  // tile row / column, -1: fallback
    for (int ph = 0; ph < P; ++ph) {
        int y0, y1;
        const bool live = roi_ok && row_extent<SR>(row_taps<SR>(g, ph), y0, y1);
        const int ty = live ? y0 / kTile : -1;
        rty[ph] = (live && y1 < ty * kTile + kWin) ? ty : -1;
    }
    for (int pw = 0; pw < P; ++pw) {
        int x0, x1;
        const bool live = roi_ok && col_extent<SR>(col_samples<SR>(g, pw), x0, x1);
        const int tx = live ? x0 / kTile : -1;
        ctx[pw] = (live && x1 < tx * kTile + kWin) ? tx : -1;
    }
    int n = 0;
    bool overflow = false;
    for (int ph0 = 0; ph0 < P && !overflow;) {
        int ph1 = ph0;
        while (ph1 + 1 < P && rty[ph1 + 1] == rty[ph0]) ++ph1;
        if (rty[ph0] >= 0) {
            for (int pw0 = 0; pw0 < P;) {
                int pw1 = pw0;
                while (pw1 + 1 < P && ctx[pw1 + 1] == ctx[pw0]) ++pw1;
                if (ctx[pw0] >= 0) {
                    if (n == kMaxEnt) {
                        overflow = true;
                        break;
                    }
                    const int tile = tg.base[li] + (b * tg.ty[li] + rty[ph0]) * tg.tx[li] +
                                     ctx[pw0];
                    ent[(int64_t)r * kMaxEnt + n] =
                        make_int4(r, ph0 | (ph1 << 8) | (pw0 << 16) | (pw1 << 24), tile,
                                  atomicAdd(count + tile, 1));
                    ++n;
                }
                pw0 = pw1 + 1;
            }
        }
        ph0 = ph1 + 1;
    }
    if (overflow) {  // pathological RoI: all of it through the fallback (n entries stay
        // listed; mark them void so the scatter skips them)
        for (int k = 0; k < n; ++k) ent[(int64_t)r * kMaxEnt + k].y = -1;
    }
    nent[r] = n;
    // fallback bins: rows or columns without a tile (all bins if overflow)
    int nfb = 0;
    for (int ph = 0; ph < P; ++ph)
        for (int pw = 0; pw < P; ++pw) nfb += overflow || rty[ph] < 0 || ctx[pw] < 0;
    if (nfb) {
        int pos = atomicAdd(fb_count, nfb);
        for (int ph = 0; ph < P; ++ph)
            for (int pw = 0; pw < P; ++pw)
                if (overflow || rty[ph] < 0 || ctx[pw] < 0) fb_list[pos++] = (r * P + ph) * P + pw;
    }
}

// Exclusive prefix sum of count[0..T) into offset[0..T) (one workgroup).
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

// 3. Entries into per-tile lists (one lane per RoI).
__global__ __launch_bounds__(256) void entry_scatter_kernel(int R, const int4 *__restrict__ ent,
                                                             const int *__restrict__ nent,
                                                             const int *__restrict__ offset,
                                                             int2 *__restrict__ list) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const int n = nent[r];
    for (int k = 0; k < n; ++k) {
        const int4 e = ent[(int64_t)r * kMaxEnt + k];
        // void entries (overflowed RoI) keep their slot with an empty rectangle
        list[offset[e.z] + e.w] = make_int2(e.x, e.y);
    }
}

struct RowDesc {  // one output row of an entry: LDS float offsets of its tap rows
    float w[4];
    int off[4];  // (row - y0) * kWin * kSlice, -1 = dead tap
};
struct ColDesc {  // one output column of an entry, columns relative to the window
    float lx[2];
    int cols;  // xl0, xh0, xl1, xh1 as int8 (255 = sample out of range)
};

// 4. Workgroup (tile, slice): stage the window, then every bin of the tile's
// entries from LDS, kEntBatch entries per pass.  Dynamic LDS: the window, the
// batch's row / column descriptors and a bin map (bin -> entry, local index).
template <int SR, bool NT>
__global__ __launch_bounds__(512) void tile_bins_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, int P, TileGrid tg, int nslice,
    const int *__restrict__ count, const int *__restrict__ offset, const int2 *__restrict__ list,
    float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *win = smem;                                                      // kWin^2 x 32
    RowDesc *rdesc = reinterpret_cast<RowDesc *>(win + kWin * kWin * kSlice);  // [kEntBatch][P]
    ColDesc *cdesc = reinterpret_cast<ColDesc *>(rdesc + kEntBatch * P);       // [kEntBatch][P]
    int2 *bent = reinterpret_cast<int2 *>(cdesc + kEntBatch * P);              // [kEntBatch]
    int *boff = reinterpret_cast<int *>(bent + kEntBatch);                     // [kEntBatch + 1]
    uint16_t *bmap = reinterpret_cast<uint16_t *>(boff + kEntBatch + 1);       // [kEntBatch*P*P]
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
    const int wy = min(kWin, H - y0), wx = min(kWin, W - x0);
    const float *src = fa.feat[li] + (int64_t)b * H * W * C + s * kSlice;
    for (int i = threadIdx.x; i < wy * wx * 8; i += blockDim.x) {
        const int pix = i >> 3, q = i & 7;
        const int yy = pix / wx, xx = pix - yy * wx;
        *reinterpret_cast<float4 *>(win + (yy * kWin + xx) * kSlice + q * 4) =
            ld4(src + ((int64_t)(y0 + yy) * W + (x0 + xx)) * C + q * 4);
    }
    const int off = offset[tile];
    const int lane = lane_id(), grp = lane >> 3, q = lane & 7;
    const int c0 = s * kSlice + q * 4;
    const float inv = 1.f / (float)(SR * SR);
    const float *wq = win + q * 4;
    for (int e0 = 0; e0 < n; e0 += kEntBatch) {
        const int ne = min(kEntBatch, n - e0);
        // entry descriptors: thread (entry e, item it): it < 32 -> row ph0 + it,
        // else column pw0 + it - 32 (64 items per entry)
        {
            const int e = threadIdx.x >> 6, it = threadIdx.x & 63;
            if (e < ne) {
                const int2 en = list[off + e0 + e];
                const int ph0 = en.y & 255, ph1 = (en.y >> 8) & 255;
                const int pw0 = (en.y >> 16) & 255, pw1 = (en.y >> 24) & 255;
                const bool void_ent = en.y == -1;
                if (it == 0) {
                    bent[e] = en;
                    boff[e + 1] = void_ent ? 0 : (ph1 - ph0 + 1) * (pw1 - pw0 + 1);
                }
                const bool row_item = it < 32 && ph0 + it <= ph1;
                const bool col_item = it >= 32 && pw0 + it - 32 <= pw1;
                if (!void_ent && (row_item || col_item)) {
                    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)en.x * 5, li, P, P, SR);
                    if (row_item) {
                        const RowTaps<SR> t = row_taps<SR>(g, ph0 + it);
                        RowDesc d;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const bool a = k < 2 * SR && t.alive[k];
                            d.w[k] = a ? t.w[k] : 0.f;
                            d.off[k] = a ? (t.row[k] - y0) * kWin * kSlice : -1;
                        }
                        rdesc[e * P + it] = d;
                    } else {
                        const ColSamples cs = col_samples<SR>(g, pw0 + it - 32);
                        ColDesc d;
                        int packed = 0;
#pragma unroll
                        for (int ix = 0; ix < 2; ++ix) {
                            const bool a = ix < SR && cs.ok[ix];
                            d.lx[ix] = a ? cs.lx[ix] : 0.f;
                            packed |= ((a ? cs.xl[ix] - x0 : 255) & 255) << (16 * ix);
                            packed |= ((a ? cs.xh[ix] - x0 : 255) & 255) << (16 * ix + 8);
                        }
                        d.cols = packed;
                        cdesc[e * P + it - 32] = d;
                    }
                }
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            boff[0] = 0;
            for (int e = 0; e < ne; ++e) boff[e + 1] += boff[e];
        }
        __syncthreads();
        {  // bin map: bin j of the batch -> (entry, index in its rectangle)
            const int e = threadIdx.x >> 6, it = threadIdx.x & 63;
            if (e < ne)
                for (int k = it; k < boff[e + 1] - boff[e]; k += 64)
                    bmap[boff[e] + k] = (uint16_t)((e << 12) | k);
        }
        __syncthreads();
        const int nb = boff[ne];
        for (int j = wave_id() * 8 + grp; j - grp < nb; j += num_waves() * 8) {
            if (j >= nb) continue;
            const int m = bmap[j];
            const int e = m >> 12, k = m & 4095;
            const int2 en = bent[e];
            const int ph0 = en.y & 255, pw0 = (en.y >> 16) & 255, pw1 = (en.y >> 24) & 255;
            const int nw = pw1 - pw0 + 1;
            const int dr = k / nw, dc = k - dr * nw;
            const RowDesc rd = rdesc[e * P + dr];
            const ColDesc cd = cdesc[e * P + dc];
            auto column = [&](int xr) -> float4 {
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                const float *cp = wq + xr * kSlice;
#pragma unroll
                for (int t = 0; t < 2 * SR; ++t) {
                    if (rd.off[t] >= 0) {
                        const float4 f = *reinterpret_cast<const float4 *>(cp + rd.off[t]);
                        v.x += rd.w[t] * f.x;
                        v.y += rd.w[t] * f.y;
                        v.z += rd.w[t] * f.z;
                        v.w += rd.w[t] * f.w;
                    }
                }
                return v;
            };
            int cl = -1, ch = -1;
            float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va, acc = va;
#pragma unroll
            for (int ix = 0; ix < SR; ++ix) {
                const int xl = (cd.cols >> (16 * ix)) & 255, xh = (cd.cols >> (16 * ix + 8)) & 255;
                if (xl == 255) continue;
                const float lx = cd.lx[ix], hx = 1.f - lx;
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
            float *dst = out + (((int64_t)en.x * P + ph0 + dr) * P + pw0 + dc) * C + c0;
            if (NT) {
                vf4 v = {acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv};
                __builtin_nontemporal_store(v, reinterpret_cast<vf4 *>(dst));
            } else {
                *reinterpret_cast<float4 *>(dst) =
                    make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
            }
        }
        __syncthreads();  // descriptors of this batch consumed
    }
}

static size_t tile_bins_lds(int P) {
    return (size_t)kWin * kWin * kSlice * 4 + kEntBatch * P * (sizeof(RowDesc) + sizeof(ColDesc)) +
           kEntBatch * sizeof(int2) + (kEntBatch + 1) * 4 + (size_t)kEntBatch * P * P * 2 + 16;
}

// One wave per fallback bin, every channel, taps from global memory; a bin
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

static TileGrid tile_grid(const FpnLevels &fa) {
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

static size_t align256(size_t n) { return (n + 255) & ~(size_t)255; }

size_t roi_align_tiled_workspace_bytes(const FpnLevels &fa, int R, int P) {
    const TileGrid tg = tile_grid(fa);
    const size_t T = (size_t)tg.base[fa.L];
    const size_t ne = (size_t)R * kMaxEnt;
    return align256(T * 4) * 2 + align256(ne * 16) + align256((size_t)R * 4) +
           align256(ne * 8) + align256((size_t)R * P * P * 4) + 256;
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
    const size_t ne = (size_t)R * kMaxEnt;
    char *p = (char *)ws;
    int *count = (int *)p;
    p += align256((size_t)T * 4);
    int *offset = (int *)p;
    p += align256((size_t)T * 4);
    int4 *ent = (int4 *)p;
    p += align256(ne * 16);
    int *nent = (int *)p;
    p += align256((size_t)R * 4);
    int2 *list = (int2 *)p;
    p += align256(ne * 8);
    int *fb_list = (int *)p;
    p += align256((size_t)R * P * P * 4);
    int *fb_count = (int *)p;
    if (hipMemsetAsync(count, 0, (size_t)T * 4, s) != hipSuccess) return VD_ERR_LAUNCH;
    if (hipMemsetAsync(fb_count, 0, 4, s) != hipSuccess) return VD_ERR_LAUNCH;
    const unsigned rblk = (unsigned)((R + 255) / 256);
    hipLaunchKernelGGL((roi_tiles_kernel<2>), dim3(rblk), dim3(256), 0, s, fa, C, rois, lvl, P, tg,
                       count, ent, nent, fb_count, fb_list);
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, count, T, offset);
    hipLaunchKernelGGL(entry_scatter_kernel, dim3(rblk), dim3(256), 0, s, R, ent, nent, offset,
                       list);
    const int nslice = C / kSlice;
    hipLaunchKernelGGL((tile_bins_kernel<2, true>), dim3((unsigned)((int64_t)T * nslice)),
                       dim3(512), tile_bins_lds(P), s, fa, C, rois, P, tg, nslice, count, offset,
                       list, out);
    hipLaunchKernelGGL((fallback_bins_kernel<2>), dim3(256), dim3(256), 0, s, fa, C, rois, lvl, P,
                       fb_count, fb_list, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
