// RoIAlign forward, tile-binned and LDS-staged: the product FPN kernel path
// (VOSDET_ROIALIGN_VARIANT 30).
//
// Reference semantics: lib/modeling/roi_xfrom/roi_align/src/roi_align_kernel.cu
//   bilinear_interpolate :16-63, ROIAlignForward :65-121.  Every output element
//   is computed with exactly that arithmetic -- per sample (iy, ix) the weights
//   hy*hx, hy*lx, ly*hx, ly*lx, val = w1*v1 + w2*v2 + w3*v3 + w4*v4 left to
//   right, iy-major accumulation, / count -- so the result is bit-identical to
//   oracle/roi_ops.c and to the row kernel of roi_align.hip (variant 3).
//
// Why tiles.  The 1000 RoIs of a frame overlap ~4x on the pyramid: fetched per
// RoI (the register-gather kernel, variant 10) every pixel crosses the L2 ->
// CU path ~4 times and, because the in-flight footprint of an XCD's resident
// RoIs exceeds its 4 MiB L2, ~1.5x the compulsory bytes cross the fabric.
// Here the unit of staging is a 16 x 16 TILE of one level image: each pixel is
// copied into LDS once per tile window (plus a small halo), and every bin of
// every RoI whose taps fall in that window is computed from LDS.
//
// Pipeline (one launch sequence, all stream-ordered, no host sync):
//  0. memset   tile counters / extents, direct-list and item counters.
//  1. bin_count    one lane per output bin (r, ph, pw): the reference's sample
//                  geometry; the bin goes to the tile of its top-left tap when
//                  all its taps fit that tile's 20 x 20 window, else to the
//                  direct list; a bin with no sample in range (or a malformed
//                  RoI) is written as zeros right here.  Lanes of a wave that
//                  share a tile aggregate into one atomicAdd (slot) and one
//                  64-bit atomicOr (window extent bits).
//  2. tile_scan    one workgroup: exclusive prefix of the tile counts
//                  (descriptor offsets), chunking of dense tiles, and the
//                  ITEM list (tile, 32-channel slice, chunk) in (image, level,
//                  slice, tile row, tile col) order -- the order in which an
//                  XCD's workgroups sweep it, so window halos are L2 hits.
//  3. bin_scatter  the same geometry again; each bin's 24-byte descriptor
//                  (output row, window-relative tap rows / columns, validity,
//                  ly / lx) is stored contiguously per tile.
//  4. tile kernel  persistent, one 8-wave workgroup per CU: wave 0 is the
//                  LOADER -- it copies item windows (rows x cols x 128 B) from
//                  HBM/L2 into a 3-slot LDS ring by LDS-DMA
//                  (global_load_lds_dwordx4, 8 pixels' slices per wave
//                  instruction), two items ahead of the compute; waves 1..7
//                  compute 8 bins x 32 channels per task from the resident
//                  window (16 ds_read_b128 per lane per bin) and store 128 B
//                  per bin and slice.  One barrier per item; the loader alone
//                  issues DMAs and waits for them with a counted vmcnt.
//  5. direct       one wave per direct-list bin, taps from global memory.
//
// Kernel 4 and 5 write disjoint bins and nothing accumulates across waves, so
// the output is deterministic and independent of the schedule.
#include <stdio.h>
#include <stdlib.h>

#include "common.hpp"
#include "roi_geom.hpp"
#include "vosdet_internal.hpp"

namespace vd {
namespace ratile {

constexpr int kT = 16;                  // tile edge (level pixels)
constexpr int kWin = 20;                // window edge cap: tile + halo 4
constexpr int kG = 32;                  // channels per slice (128 B per pixel)
constexpr int kSlotPx = kWin * kWin;    // 400 pixels
constexpr int kWinB = kSlotPx * kG * 4;   // 51,200 B of window
constexpr int kMaxChunk = 128;          // bins per item (descriptors staged with the window)
constexpr int kDescB = kMaxChunk * 24 + 16;  // 3,088 B: 24-B descriptors + alignment slack
constexpr int kSlotB = kWinB + kDescB;  // 54,288 B per ring slot
constexpr int kSlots = 3;               // 162,864 B of the CU's 160 KiB

// Bin kinds of the binning passes.
constexpr int kTiled = 0, kDirect = 1, kZero = 2;

struct TileGrid {
    int ty[VD_MAX_LEVELS], tx[VD_MAX_LEVELS];
    int base[VD_MAX_LEVELS + 1];  // first tile index of level l (all images)
};

// One work item of the tile kernel (32 B, read by the loader with scalar loads,
// one record ahead of its use).
struct ItemRec {
    const float *base;  // window origin pixel of the item's image / level, + slice
    int rstride;        // bytes per level row (W * C * 4)
    int nrc;            // nrows | ncols << 8 | slice << 16
    int start;          // first descriptor
    int count;          // descriptors (bins) of this item
    int pad0, pad1;
};

// Window-resident item metadata the loader publishes in LDS next to a slot:
// {count (bins; -1: no more items), first descriptor, ncols, slice}.
typedef int vi4 __attribute__((ext_vector_type(4)));

struct BinGeom {
    int kind;
    int tile;
    uint64_t ext;   // bit (ymax - y0) in the low word, bit (xmax - x0) in the high word
    int pk;         // packed window-relative taps and validity
    float4 lw;      // ly0, ly1, lx0, lx1
};

// Clamped taps of one coordinate (roi_align_kernel.cu:19-48); false for a
// sample outside [-1, N].
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

// Geometry of output bin (r, ph, pw) with sampling ratio 2 (the reference's
// sample positions: roi_align_kernel.cu:84-105), its tile and descriptor.
__device__ __forceinline__ BinGeom bin_geom(const FpnLevels &fa, const TileGrid &tg,
                                            const float *__restrict__ rois,
                                            const int *__restrict__ roi_level, int P, int r,
                                            int ph, int pw) {
    BinGeom o;
    o.kind = kZero;
    o.tile = 0;
    o.ext = 0;
    o.pk = 0;
    o.lw = make_float4(0.f, 0.f, 0.f, 0.f);
    const float *roi = rois + (int64_t)r * 5;
    const int li = roi_level ? roi_level[r] : 0;
    const int b = (int)roi[0];
    if (li < 0 || li >= fa.L || b < 0 || b >= fa.B) return o;  // malformed: pools to 0
    const int H = fa.H[li], W = fa.W[li];
    const float scale = fa.scale[li];
    const float sw = roi[1] * scale, sh = roi[2] * scale;
    const float rw = fmaxf(roi[3] * scale - sw, 1.f), rh = fmaxf(roi[4] * scale - sh, 1.f);
    const float bh = rh / P, bw = rw / P;
    int yl[2], yh[2], xl[2], xh[2];
    float ly[2], lx[2];
    bool vy[2], vx[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        vy[i] = taps1(sh + ph * bh + (i + .5f) * bh / 2, H, yl[i], yh[i], ly[i]);
        vx[i] = taps1(sw + pw * bw + (i + .5f) * bw / 2, W, xl[i], xh[i], lx[i]);
    }
    if (!(vy[0] || vy[1]) || !(vx[0] || vx[1])) return o;  // every sample out of range
    // invalid samples borrow the valid one's taps (their value is discarded)
    if (!vy[0]) { yl[0] = yl[1]; yh[0] = yh[1]; }
    if (!vy[1]) { yl[1] = yl[0]; yh[1] = yh[0]; }
    if (!vx[0]) { xl[0] = xl[1]; xh[0] = xh[1]; }
    if (!vx[1]) { xl[1] = xl[0]; xh[1] = xh[0]; }
    const int ymin = min(yl[0], yl[1]), ymax = max(yh[0], yh[1]);
    const int xmin = min(xl[0], xl[1]), xmax = max(xh[0], xh[1]);
    const int ty = ymin / kT, tx = xmin / kT;
    const int y0 = ty * kT, x0 = tx * kT;
    o.kind = kDirect;
    if (ymax - y0 >= kWin || xmax - x0 >= kWin) return o;
    o.kind = kTiled;
    o.tile = tg.base[li] + (b * tg.ty[li] + ty) * tg.tx[li] + tx;
    o.ext = (1ull << (ymax - y0)) | ((1ull << (xmax - x0)) << 32);
    o.pk = (yl[0] - y0) | (yl[1] - y0) << 5 | (xl[0] - x0) << 10 | (xl[1] - x0) << 15 |
           (yh[0] - yl[0]) << 20 | (yh[1] - yl[1]) << 21 | (xh[0] - xl[0]) << 22 |
           (xh[1] - xl[1]) << 23 | (int)vy[0] << 24 | (int)vy[1] << 25 | (int)vx[0] << 26 |
           (int)vx[1] << 27;
    o.lw = make_float4(ly[0], ly[1], lx[0], lx[1]);
    return o;
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v |= shfl_xor64(v, m);
    return v;
}

// 1. One lane per output bin.
__global__ __launch_bounds__(256) void bin_count_kernel(FpnLevels fa, TileGrid tg, int C,
                                                        const float *__restrict__ rois,
                                                        const int *__restrict__ roi_level, int P,
                                                        int *__restrict__ cnt,
                                                        unsigned long long *__restrict__ ext,
                                                        int *__restrict__ slot,
                                                        int *__restrict__ dir_cnt,
                                                        int *__restrict__ dir_list,
                                                        float *__restrict__ out) {
    const int PP = P * P;
    const int64_t nb = (int64_t)fa.R * PP;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = g < nb;
    BinGeom bg;
    bg.kind = -1;
    if (act) {
        const int r = (int)(g / PP), rem = (int)(g - (int64_t)r * PP);
        const int ph = rem / P, pw = rem - ph * P;
        bg = bin_geom(fa, tg, rois, roi_level, P, r, ph, pw);
    }
    const int lane = lane_id();
    // tiled bins: the lanes of each distinct tile of the wave elect their lowest
    // lane, which issues ONE atomicAdd (slots) and ONE atomicOr (extent bits)
    // for the group; all leaders' atomics go out together (one round trip).
    int leader = -1, rank = 0, gsize = 0;
    uint64_t gext = 0;
    uint64_t pend = ballot(bg.kind == kTiled);
    while (pend) {
        const int ld = __ffsll((unsigned long long)pend) - 1;
        const int lt = __builtin_amdgcn_readlane(bg.tile, ld);
        const bool mine = bg.kind == kTiled && bg.tile == lt;
        const uint64_t same = ballot(mine);
        const uint64_t e = wave_or64(mine ? bg.ext : 0ull);
        if (mine) {
            leader = ld;
            rank = lane_prefix(same);
            gsize = (int)__popcll(same);
            gext = e;
        }
        pend &= ~same;
    }
    int base = 0;
    if (leader == lane) {
        base = atomicAdd(cnt + bg.tile, gsize);
        atomicOr(ext + bg.tile, (unsigned long long)gext);
    }
    base = __shfl(base, leader < 0 ? lane : leader);
    const int my_slot = leader >= 0 ? base + rank : -1;
    // direct bins: one atomicAdd per wave
    const uint64_t dmask = ballot(bg.kind == kDirect);
    if (dmask) {
        const int leader = __ffsll((unsigned long long)dmask) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(dir_cnt, (int)__popcll(dmask));
        base = __builtin_amdgcn_readlane(base, leader);
        if (bg.kind == kDirect) dir_list[base + lane_prefix(dmask)] = (int)g;
    }
    if (act) slot[g] = my_slot;
    if (bg.kind == kZero) {  // output_val = 0 / count
        float4 *dst = reinterpret_cast<float4 *>(out + g * C);
        for (int c = 0; c < C / 4; ++c) dst[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// 2. One workgroup: exclusive prefix of the tile counts (descriptor offsets),
//    of the tiles' chunk counts (chunk_pre[T + 1]), and the (image, level)
//    group table grp = {chunks of group g, first item of group g} that fixes the
//    item order: image, level, slice, tile row, tile col, chunk.
__global__ __launch_bounds__(1024) void tile_scan_kernel(FpnLevels fa, TileGrid tg, int S,
                                                         int chunk, const int *__restrict__ cnt,
                                                         int *__restrict__ offset,
                                                         int *__restrict__ chunk_pre,
                                                         int2 *__restrict__ grp,
                                                         int *__restrict__ n_items) {
    __shared__ int part[2][1024];
    __shared__ int gch[VD_MAX_LEVELS * 64];
    const int T = tg.base[fa.L];
    const int t = threadIdx.x, nt = blockDim.x;
    const int per = (T + nt - 1) / nt;
    const int a = min(t * per, T), e = min(a + per, T);
    int s_cnt = 0, s_chk = 0;
    for (int i = a; i < e; ++i) {
        const int c = cnt[i];
        s_cnt += c;
        s_chk += (c + chunk - 1) / chunk;
    }
    part[0][t] = s_cnt;
    part[1][t] = s_chk;
    __syncthreads();
    for (int off = 1; off < nt; off <<= 1) {  // Hillis-Steele over both arrays
        const int v0 = t >= off ? part[0][t - off] : 0, v1 = t >= off ? part[1][t - off] : 0;
        __syncthreads();
        part[0][t] += v0;
        part[1][t] += v1;
        __syncthreads();
    }
    int r0 = part[0][t] - s_cnt, r1 = part[1][t] - s_chk;
    for (int i = a; i < e; ++i) {
        const int c = cnt[i];
        offset[i] = r0;
        chunk_pre[i] = r1;
        r0 += c;
        r1 += (c + chunk - 1) / chunk;
    }
    if (t == nt - 1) chunk_pre[T] = r1;
    __syncthreads();
    const int ng = fa.B * fa.L;
    for (int gi = t; gi < ng; gi += nt) {  // groups (image b, level l): contiguous tiles
        const int b = gi / fa.L, l = gi - b * fa.L;
        const int t0 = tg.base[l] + b * tg.ty[l] * tg.tx[l], t1 = t0 + tg.ty[l] * tg.tx[l];
        gch[gi] = chunk_pre[t1] - chunk_pre[t0];
    }
    __syncthreads();
    if (t == 0) {
        int sum = 0;
        for (int gi = 0; gi < ng; ++gi) {
            grp[gi] = make_int2(gch[gi], sum);
            sum += S * gch[gi];
        }
        *n_items = sum;
    }
}

// A bin's descriptor (24 B): output bin (r * P + ph) * P + pw, packed
// window-relative taps, ly0, ly1, lx0, lx1 (as float bits).
struct Desc {
    int o, pk;
    float ly0, ly1, lx0, lx1;
};

// 3. Descriptors into per-tile contiguous storage.
//    Blocks past the bins' emit the item records: one lane per tile.
__global__ __launch_bounds__(256) void bin_scatter_kernel(
    FpnLevels fa, TileGrid tg, int C, int S, int chunk, const float *__restrict__ rois,
    const int *__restrict__ roi_level, int P, const int *__restrict__ slot,
    const int *__restrict__ cnt, const unsigned long long *__restrict__ ext,
    const int *__restrict__ offset, const int *__restrict__ chunk_pre,
    const int2 *__restrict__ grp, unsigned bin_blocks, int slice_inner, Desc *__restrict__ desc,
    ItemRec *__restrict__ items) {
    const int PP = P * P;
    const int64_t nb = (int64_t)fa.R * PP;
    if (blockIdx.x >= bin_blocks) {
        const int i = (blockIdx.x - bin_blocks) * blockDim.x + threadIdx.x;
        if (i >= tg.base[fa.L]) return;
        const int c = cnt[i];
        if (c == 0) return;
        int l = 0;
        while (l + 1 < fa.L && i >= tg.base[l + 1]) ++l;
        const int local = i - tg.base[l];
        const int per_img = tg.ty[l] * tg.tx[l];
        const int b = local / per_img, rem = local - b * per_img;
        const int ty = rem / tg.tx[l], tx = rem - ty * tg.tx[l];
        const int2 gr = grp[b * fa.L + l];
        const int within = chunk_pre[i] - chunk_pre[tg.base[l] + b * per_img];
        const unsigned long long ex = ext[i];
        const int nrows = 32 - __clz((int)(uint32_t)ex), ncols = 32 - __clz((int)(uint32_t)(ex >> 32));
        const int H = fa.H[l], W = fa.W[l];
        const float *org = fa.feat[l] + (((int64_t)b * H + ty * kT) * W + tx * kT) * C;
        const int nch = (c + chunk - 1) / chunk;
        for (int sl = 0; sl < S; ++sl)
            for (int k = 0; k < nch; ++k) {
                ItemRec it;
                it.base = org + sl * kG;
                it.rstride = W * C * 4;
                it.nrc = nrows | ncols << 8 | sl << 16;
                it.start = offset[i] + k * chunk;
                it.count = min(chunk, c - k * chunk);
                it.pad0 = it.pad1 = 0;
                items[gr.y + (slice_inner ? (within + k) * S + sl : sl * gr.x + within + k)] =
                    it;
            }
        return;
    }
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nb) return;
    const int sl = slot[g];
    if (sl < 0) return;
    const int r = (int)(g / PP), rem = (int)(g - (int64_t)r * PP);
    const int ph = rem / P, pw = rem - ph * P;
    const BinGeom bg = bin_geom(fa, tg, rois, roi_level, P, r, ph, pw);
    const int d = offset[bg.tile] + sl;
    desc[d] = Desc{(int)g, bg.pk, bg.lw.x, bg.lw.y, bg.lw.z, bg.lw.w};
}

// One LDS-DMA wave instruction: lane i copies 16 B from sbase + voff into LDS
// byte address lds + 16 i.  Inline asm so that hipcc neither counts nor drains
// it; M0 carries the LDS address and is restored within the statement.
__device__ __forceinline__ void dma_1k(const float *sbase, uint32_t voff, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(sbase), "s"(lds)
        : "memory");
}

// s_waitcnt vmcnt(n) (n wave-uniform, clamped to the 6-bit field: waiting for
// fewer outstanding operations is always safe since loads complete in order),
// lgkmcnt(0), then the workgroup barrier.
__device__ __forceinline__ void wait_barrier(int n) {
#define VD_W1(k)                                                                   \
    case k:                                                                        \
        asm volatile("s_waitcnt vmcnt(" #k ") lgkmcnt(0)\n\ts_barrier" ::: "memory"); \
        break;
#define VD_W8(k) VD_W1(k) VD_W1(k + 1) VD_W1(k + 2) VD_W1(k + 3) VD_W1(k + 4) VD_W1(k + 5) \
    VD_W1(k + 6) VD_W1(k + 7)
    n = __builtin_amdgcn_readfirstlane(n);
    switch (n < 63 ? n : 63) {
        VD_W8(0) VD_W8(8) VD_W8(16) VD_W8(24) VD_W8(32) VD_W8(40) VD_W8(48) VD_W8(56)
        default:
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            break;
    }
#undef VD_W8
#undef VD_W1
}

typedef __attribute__((address_space(3))) const vf4 lds_f4;
typedef __attribute__((address_space(3))) vi4 lds_meta;

// Loader wave w of NL: issue its share (chunks c = w mod NL) of item `it`'s
// window DMA and descriptor DMA into the slot at `slot_lds`; loader 0 publishes
// the slot meta.  Returns the DMA instructions this wave issued (wave-uniform).
template <int NL, int MODE>
__device__ __forceinline__ int load_item(int C, const ItemRec &it, bool live,
                                         const Desc *__restrict__ desc, uint32_t slot_lds,
                                         lds_meta *meta, int w, int lane) {
    if (!live) {
        if (w == 0 && lane == 0) *meta = vi4{-1, 0, 0, 0};
        return 0;
    }
    const int nrows = it.nrc & 255, ncols = (it.nrc >> 8) & 255, sl = it.nrc >> 16;
    const int npx = nrows * ncols;
    const int nchunk = (npx + 7) >> 3;
    const uint32_t magic = (65536u + (uint32_t)ncols - 1u) / (uint32_t)ncols;
    const int q = lane & 7;
    const uint32_t pstride = (uint32_t)C * 4u;
    int n = 0;
    if (MODE != 2) {
        for (int c = w; c < nchunk; c += NL) {
            const int p = c * 8 + (lane >> 3);
            const int yy = (int)(((uint32_t)p * magic) >> 16);
            const int xx = p - yy * ncols;
            const uint32_t voff = (uint32_t)yy * (uint32_t)it.rstride + (uint32_t)xx * pstride +
                                  (uint32_t)q * 16u;
            if (p < npx) dma_1k(it.base, voff, slot_lds + (uint32_t)c * 1024u);  // lanes past
            ++n;                                                                // the window:
        }                                                                       // masked
    }
    // the item's descriptors, 16-B aligned copy of [start * 24, (start + count) * 24)
    const int64_t b0 = (int64_t)it.start * 24;
    const int delta = (int)(b0 & 15);
    const char *dsrc = reinterpret_cast<const char *>(desc) + (b0 - delta);
    const int n16 = (delta + it.count * 24 + 15) >> 4;
    const int nd = (n16 + 63) >> 6;
    for (int c = w; c < nd; c += NL) {
        const int j = c * 64 + lane;
        if (j < n16)
            dma_1k(reinterpret_cast<const float *>(dsrc), (uint32_t)j * 16u,
                   slot_lds + kWinB + (uint32_t)c * 1024u);
        ++n;
    }
    if (w == 0 && lane == 0) *meta = vi4{it.count, delta, ncols, sl};
    return n;
}

__device__ __forceinline__ float4 lds4(lds_f4 *p) {
    const vf4 v = *p;
    return make_float4(v.x, v.y, v.z, v.w);
}

// w1*v1 + w2*v2 + w3*v3 + w4*v4, left to right (roi_align_kernel.cu:60)
__device__ __forceinline__ float4 bil4(float w1, float w2, float w3, float w4, float4 a,
                                       float4 b, float4 c, float4 d) {
    return make_float4(w1 * a.x + w2 * b.x + w3 * c.x + w4 * d.x,
                       w1 * a.y + w2 * b.y + w3 * c.y + w4 * d.y,
                       w1 * a.z + w2 * b.z + w3 * c.z + w4 * d.z,
                       w1 * a.w + w2 * b.w + w3 * c.w + w4 * d.w);
}

// One compute task: 8 bins (lane >> 3) x 32 channels (lane & 7 = channel quad).
__device__ __forceinline__ void bin_task(int pk, const float4 lw, lds_f4 *win, int ncols, int q,
                                         float *__restrict__ dst) {
    const int yo[2] = {pk & 31, (pk >> 5) & 31};
    const int xo[2] = {(pk >> 10) & 31, (pk >> 15) & 31};
    const int dy[2] = {(pk >> 20) & 1, (pk >> 21) & 1};
    const int dx[2] = {(pk >> 22) & 1, (pk >> 23) & 1};
    const bool vy[2] = {((pk >> 24) & 1) != 0, ((pk >> 25) & 1) != 0};
    const bool vx[2] = {((pk >> 26) & 1) != 0, ((pk >> 27) & 1) != 0};
    const float ly[2] = {lw.x, lw.y}, lx[2] = {lw.z, lw.w};
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int iy = 0; iy < 2; ++iy) {
        const int rl = yo[iy] * ncols, rh = (yo[iy] + dy[iy]) * ncols;
        const float hy = 1.f - ly[iy];
#pragma unroll
        for (int ix = 0; ix < 2; ++ix) {
            const int cl = xo[ix], ch = xo[ix] + dx[ix];
            const float hx = 1.f - lx[ix];
            const float4 v1 = lds4(win + (rl + cl) * 8 + q);
            const float4 v2 = lds4(win + (rl + ch) * 8 + q);
            const float4 v3 = lds4(win + (rh + cl) * 8 + q);
            const float4 v4 = lds4(win + (rh + ch) * 8 + q);
            const float w1 = hy * hx, w2 = hy * lx[ix], w3 = ly[iy] * hx, w4 = ly[iy] * lx[ix];
            float4 val = bil4(w1, w2, w3, w4, v1, v2, v3, v4);
            if (!(vy[iy] && vx[ix])) val = make_float4(0.f, 0.f, 0.f, 0.f);
            acc.x += val.x;
            acc.y += val.y;
            acc.z += val.z;
            acc.w += val.w;
        }
    }
    const float count = 4.f;
    const vf4 r = {acc.x / count, acc.y / count, acc.z / count, acc.w / count};
    __builtin_nontemporal_store(r, reinterpret_cast<vf4 *>(dst));
}

// 4. Persistent tile kernel: grid = a multiple of 8 workgroups (block b runs on
// XCD b % 8); XCD x sweeps items [x N / 8, (x + 1) N / 8), its k-th workgroup
// takes every K-th of them.  Waves 0..NL-1 load, the others compute.  MODE
// (diagnostics): 0 product, 1 no compute, 2 no window DMA.
template <int NL, int NW, int MODE>
__global__ __launch_bounds__(NW * 64) void tile_kernel(int C,
                                                           const ItemRec *__restrict__ items,
                                                           const int *__restrict__ n_items,
                                                           const Desc *__restrict__ desc,
                                                           float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) float4 lds[kSlots * kSlotB / 16];
    __shared__ vi4 meta[kSlots];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int N = __builtin_amdgcn_readfirstlane(*n_items);
    const int xcd = blockIdx.x & 7, K = gridDim.x >> 3, k = blockIdx.x >> 3;
    const int lo = (int)((int64_t)N * xcd / 8), hi = (int)((int64_t)N * (xcd + 1) / 8);
    const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
    lds_meta *metap = (lds_meta *)meta;
    const bool loader = wave < NL;
    int next = lo + k;  // loader cursor: the record in `nxt`
    int d_next = 0;     // this loader's DMA instructions of item i + 1
    ItemRec nxt = {};
    if (loader) {
        if (next < hi) nxt = items[next];
        for (int j = 0; j < 2; ++j) {
            const ItemRec cur = nxt;
            const bool live = next < hi;
            next += K;
            if (next < hi) nxt = items[next];
            const int n = load_item<NL, MODE>(C, cur, live, desc, lds_base + j * kSlotB,
                                              metap + j, wave, lane);
            if (j == 1) d_next = n;
        }
    }
    for (int i = 0;; ++i) {
        // loaders retire item i's DMA (younger: item i + 1's), then all sync
        wait_barrier(loader ? d_next : 63);
        const int sl = i % kSlots;
        const vi4 m = meta[sl];
        const int count = __builtin_amdgcn_readfirstlane(m.x);
        if (count < 0) break;
        if (loader) {
            const ItemRec cur = nxt;
            const bool live = next < hi;
            next += K;
            const int s2 = (i + 2) % kSlots;
            d_next = load_item<NL, MODE>(C, cur, live, desc, lds_base + s2 * kSlotB,
                                         metap + s2, wave, lane);
            if (next < hi) nxt = items[next];  // lands before the next barrier
        } else if (MODE != 1) {
            const int delta = __builtin_amdgcn_readfirstlane(m.y);
            const int ncols = __builtin_amdgcn_readfirstlane(m.z);
            const int slice = __builtin_amdgcn_readfirstlane(m.w);
            lds_f4 *win = (lds_f4 *)lds + sl * (kSlotB / 16);
            const int q = lane & 7;
            const int ntask = (count + 7) >> 3;
            for (int t = wave - NL; t < ntask; t += NW - NL) {
                const int j = t * 8 + (lane >> 3);
                const bool on = j < count;
                // descriptor j: three 8-B LDS reads (broadcast to the bin's 8 lanes)
                typedef int vi2 __attribute__((ext_vector_type(2)));
                typedef __attribute__((address_space(3))) const vi2 lds_i2;
                lds_i2 *dp = (lds_i2 *)((__attribute__((address_space(3))) const char *)win +
                                        kWinB + delta + (on ? j : 0) * 24);
                const vi2 a = dp[0], l01 = dp[1], l23 = dp[2];
                const float4 lw = make_float4(__int_as_float(l01.x), __int_as_float(l01.y),
                                              __int_as_float(l23.x), __int_as_float(l23.y));
                if (on)
                    bin_task(a.y, lw, win, ncols, q,
                             out + (int64_t)a.x * C + slice * kG + q * 4);
            }
        }
    }
    // no LDS-DMA may land after the workgroup's LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// 5. Direct-list bins: one wave per bin, every channel from global memory, the
// same per-sample arithmetic.  Grid-stride over the device-side count.
__global__ __launch_bounds__(256) void direct_kernel(FpnLevels fa, TileGrid tg, int C,
                                                     const float *__restrict__ rois,
                                                     const int *__restrict__ roi_level, int P,
                                                     const int *__restrict__ dir_cnt,
                                                     const int *__restrict__ dir_list,
                                                     float *__restrict__ out) {
    const int n = *dir_cnt;
    const int lane = lane_id();
    const int waves = gridDim.x * num_waves();
    const int PP = P * P;
    for (int i = blockIdx.x * num_waves() + wave_id(); i < n; i += waves) {
        const int g = dir_list[i];
        const int r = g / PP, rem = g - r * PP;
        const int ph = rem / P, pw = rem - ph * P;
        const float *roi = rois + (int64_t)r * 5;
        const int li = roi_level ? roi_level[r] : 0;
        const int b = (int)roi[0];
        const int H = fa.H[li], W = fa.W[li];
        const float scale = fa.scale[li];
        const float sw = roi[1] * scale, sh = roi[2] * scale;
        const float rw = fmaxf(roi[3] * scale - sw, 1.f), rh = fmaxf(roi[4] * scale - sh, 1.f);
        const float bh = rh / P, bw = rw / P;
        const float *img = fa.feat[li] + (int64_t)b * H * W * C;
        for (int c0 = lane * 4; c0 < C; c0 += 256) {
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int iy = 0; iy < 2; ++iy) {
                int yl, yh;
                float ly;
                const bool vy = taps1(sh + ph * bh + (iy + .5f) * bh / 2, H, yl, yh, ly);
                const float hy = 1.f - ly;
                for (int ix = 0; ix < 2; ++ix) {
                    int xl, xh;
                    float lx;
                    const bool vx = taps1(sw + pw * bw + (ix + .5f) * bw / 2, W, xl, xh, lx);
                    if (!(vy && vx)) continue;
                    const float hx = 1.f - lx;
                    const float4 v1 = ld4(img + ((int64_t)yl * W + xl) * C + c0);
                    const float4 v2 = ld4(img + ((int64_t)yl * W + xh) * C + c0);
                    const float4 v3 = ld4(img + ((int64_t)yh * W + xl) * C + c0);
                    const float4 v4 = ld4(img + ((int64_t)yh * W + xh) * C + c0);
                    const float4 val = bil4(hy * hx, hy * lx, ly * hx, ly * lx, v1, v2, v3, v4);
                    acc.x += val.x;
                    acc.y += val.y;
                    acc.z += val.z;
                    acc.w += val.w;
                }
            }
            const float count = 4.f;
            *reinterpret_cast<float4 *>(out + (int64_t)g * C + c0) =
                make_float4(acc.x / count, acc.y / count, acc.z / count, acc.w / count);
        }
    }
}

TileGrid tile_grid(const FpnLevels &fa) {
    TileGrid tg = {};
    int base = 0;
    for (int l = 0; l < fa.L; ++l) {
        tg.ty[l] = (fa.H[l] + kT - 1) / kT;
        tg.tx[l] = (fa.W[l] + kT - 1) / kT;
        tg.base[l] = base;
        base += fa.B * tg.ty[l] * tg.tx[l];
    }
    tg.base[fa.L] = base;
    return tg;
}

int chunk_bins() {
    const char *e = getenv("VOSDET_RA_CHUNK");
    const int c = e ? atoi(e) : ratile::kMaxChunk;
    return c >= 8 && c <= ratile::kMaxChunk ? c : ratile::kMaxChunk;
}

size_t a256(size_t n) { return (n + 255) & ~(size_t)255; }

struct Ws {
    int *cnt;
    unsigned long long *ext;
    int *dir_cnt, *n_items;
    int *slot, *offset, *chunk_pre, *dir_list;
    int2 *grp;
    ItemRec *items;
    Desc *desc;
    size_t zero_bytes, total;
};

Ws carve(const FpnLevels &fa, int R, int P, int C, char *p) {
    const TileGrid tg = tile_grid(fa);
    const size_t T = (size_t)tg.base[fa.L];
    const size_t nb = (size_t)R * P * P;
    const size_t S = (size_t)C / kG;
    const size_t max_items = S * (T + nb / 8 + 1);  // chunks of >= 8 bins
    Ws w;
    char *p0 = p;
    w.ext = (unsigned long long *)p;  // zeroed region first: ext, cnt, dir_cnt, n_items
    p += a256(T * 8);
    w.cnt = (int *)p;
    p += a256(T * 4);
    w.dir_cnt = (int *)p;
    w.n_items = w.dir_cnt + 1;
    p += 256;
    w.zero_bytes = (size_t)(p - p0);
    w.slot = (int *)p;
    p += a256(nb * 4);
    w.offset = (int *)p;
    p += a256(T * 4);
    w.chunk_pre = (int *)p;
    p += a256((T + 1) * 4);
    w.dir_list = (int *)p;
    p += a256(nb * 4);
    w.grp = (int2 *)p;
    p += a256((size_t)fa.B * fa.L * 8);
    w.items = (ItemRec *)p;
    p += a256(max_items * sizeof(ItemRec));
    w.desc = (Desc *)p;
    p += a256(nb * sizeof(Desc) + 16);
    w.total = (size_t)(p - p0);
    return w;
}

int num_cus() {
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

}  // namespace ratile

bool roi_align_tiled_supported(const FpnLevels &fa, int C, int P, int sr) {
    using namespace ratile;
    if (sr != 2 || P < 1 || P > 64 || C % kG != 0 || C / kG > 255) return false;
    for (int l = 0; l < fa.L; ++l)  // 32-bit per-lane DMA offsets within an image
        if ((int64_t)fa.H[l] * fa.W[l] * C * 4 >= (1ll << 31)) return false;
    return (int64_t)fa.R * P * P < (1ll << 31) / 2;
}

size_t roi_align_tiled_workspace_bytes(const FpnLevels &fa, int R, int P, int C) {
    return ratile::carve(fa, R, P, C, nullptr).total;
}

int launch_roi_align_fpn_tiled(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                               int R, int P, int sr, float *out, void *ws, size_t ws_bytes,
                               hipStream_t s) {
    using namespace ratile;
    if (R == 0) return VD_OK;
    if (!roi_align_tiled_supported(fa, C, P, sr)) return VD_ERR_SHAPE;
    const Ws w = carve(fa, R, P, C, (char *)ws);
    if (!ws || ws_bytes < w.total) return VD_ERR_WORKSPACE;
    const TileGrid tg = tile_grid(fa);
    const int64_t nb = (int64_t)R * P * P;
    const int S = C / kG;
    if (zero_async(w.ext, w.zero_bytes, s) != VD_OK) return VD_ERR_LAUNCH;
    const unsigned blk = (unsigned)((nb + 255) / 256);
    const int chunk = chunk_bins();
    const int T = tg.base[fa.L];
    const char *eo = getenv("VOSDET_RA_ORDER");  // 1: slice-inner item order
    const int order = eo ? atoi(eo) : 0;
    hipLaunchKernelGGL(bin_count_kernel, dim3(blk), dim3(256), 0, s, fa, tg, C, rois, lvl, P,
                       w.cnt, w.ext, w.slot, w.dir_cnt, w.dir_list, out);
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, fa, tg, S, chunk, w.cnt,
                       w.offset, w.chunk_pre, w.grp, w.n_items);
    hipLaunchKernelGGL(bin_scatter_kernel, dim3(blk + (unsigned)((T + 255) / 256)), dim3(256), 0,
                       s, fa, tg, C, S, chunk, rois, lvl, P, w.slot, w.cnt, w.ext, w.offset,
                       w.chunk_pre, w.grp, blk, order, w.desc, w.items);
    int nblk = num_cus() / 8 * 8;
    if (nblk < 8) nblk = 8;
    // VOSDET_RA_CFG="loaders,waves,mode" (diagnostics / tuning; default below)
    int nl = 4, nw = 16, mode = 0;  // measured best of the sweep (profiles/r03/roialign_tiled)
    if (const char *e = getenv("VOSDET_RA_CFG")) sscanf(e, "%d,%d,%d", &nl, &nw, &mode);
    const int cfg = nl * 100 + nw * 10 / 4 + mode;  // nw in {8, 12, 16}, mode < 3
#define VD_TK(NL, NW, M)                                                                  \
    case NL * 100 + NW * 10 / 4 + M:                                                      \
        hipLaunchKernelGGL((tile_kernel<NL, NW, M>), dim3(nblk), dim3(NW * 64), 0, s, C,  \
                           w.items, w.n_items, w.desc, out);                              \
        break;
#define VD_TK3(NL, NW) VD_TK(NL, NW, 0) VD_TK(NL, NW, 1) VD_TK(NL, NW, 2)
    switch (cfg) {
        VD_TK3(1, 8) VD_TK3(2, 12) VD_TK3(4, 12) VD_TK3(4, 16) VD_TK3(8, 16)
        default:
            return VD_ERR_ARG;
    }
#undef VD_TK3
#undef VD_TK
    hipLaunchKernelGGL(direct_kernel, dim3(256), dim3(256), 0, s, fa, tg, C, rois, lvl, P,
                       w.dir_cnt, w.dir_list, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
