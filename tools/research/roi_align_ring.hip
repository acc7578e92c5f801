// RoIAlign forward, tile-binned and LDS-staged through a per-CU ring of windows
// with flag hand-offs: the product FPN kernel path (VOSDET_ROIALIGN_VARIANT 60).
//
// Reference semantics: lib/modeling/roi_xfrom/roi_align/src/roi_align_kernel.cu
//   bilinear_interpolate :16-63, ROIAlignForward :65-121.  Every output element
//   is computed with exactly that arithmetic -- per sample (iy, ix) the weights
//   hy*hx, hy*lx, ly*hx, ly*lx, val = w1*v1 + w2*v2 + w3*v3 + w4*v4 left to
//   right, iy-major accumulation, / count -- so the result is bit-identical to
//   oracle/roi_ops.c and to the row kernel of roi_align.hip (variant 3).
//
// Why tiles.  The 1000 RoIs of a frame overlap ~4x on the pyramid.  Fetched per
// RoI (the register-gather kernel, variant 10) every pixel crosses the L2 -> CU
// path ~4 times (3.0 M 1 KiB wave loads per 8-frame launch, ~100 us per million)
// and ~1.7x the compulsory bytes cross the fabric.  Here the unit of staging is
// a 16 x 16 TILE of one level image: each pixel slice is copied into LDS once
// per tile window (tile + 4-pixel halo), and every bin of every RoI whose taps
// fall in that window is computed from LDS.
//
// Channel slices pinned to XCDs.  A window carries one 16-channel slice (64 B
// of each pixel's 1 KiB); XCD x computes slices 2x and 2x+1 of every tile, so
// one 128-B line of each pixel is only ever fetched by one XCD and that XCD's
// L2 holds 1/8 of every pixel: the halos of neighbouring tiles (swept by the
// XCD's 32 CUs together) and the sibling slice are L2 hits, and the fabric sees
// each pixel line about once.
//
// Pipeline (one launch sequence, all stream-ordered, no host sync):
//  0. memset      tile counters / extents, direct-list and chunk counters.
//  1. bin_count   one lane per output bin: the reference's sample geometry; the
//                 bin goes to the tile of its top-left tap when all its taps
//                 fit that tile's 20 x 20 window, else to the direct list; a bin
//                 with no sample in range is written as zeros right here.
//  2. tile_scan   one workgroup: prefix of the tile counts (descriptor offsets)
//                 and of the tiles' chunk counts (chunks of <= 192 bins).
//  3. bin_scatter each bin's 24-byte descriptor into per-tile contiguous storage;
//                 one lane per tile writes its chunk records.
//  4. ring kernel persistent, one 16-wave workgroup per CU.  Five LOADER waves,
//                 one per slot of a 5-slot LDS ring, copy item windows (rows x
//                 cols x 64 B) and descriptors into their slot by LDS-DMA and
//                 publish it by writing its sequence number once their own DMA
//                 landed.  Eleven CONSUMER waves poll the slot, compute their
//                 share of its 16-bin tasks (task t goes to consumer (t - item)
//                 mod 11) from LDS and count themselves out of the slot; its
//                 loader refills it once all eleven have left.  No workgroup
//                 barrier: consumers drift up to the ring depth apart.
//  5. direct      one wave per direct-list bin, taps from global memory.
//
// Kernels 4 and 5 write disjoint bins and nothing accumulates across waves, so
// the output is deterministic and independent of the schedule.
#include <stdio.h>
#include <stdlib.h>

#include "common.hpp"
#include "roi_geom.hpp"
#include "vosdet_internal.hpp"

namespace vd {
namespace raring {

constexpr int kT = 16;                   // tile edge (level pixels)
constexpr int kWin = 20;                 // window edge cap: tile + halo 4
constexpr int kG = 16;                   // channels per slice (64 B per pixel)
constexpr int kPxB = kG * 4;             // 64 B
constexpr int kWinB = kWin * kWin * kPxB;  // 25,600 B of window
constexpr int kMaxChunk = 192;           // bins per item
constexpr int kDescB = kMaxChunk * 24 + 32;  // 4,640 B: descriptors + alignment slack
constexpr int kSlotB = 30720;            // window + descriptors, 1 KiB multiple
static_assert(kWinB + kDescB <= kSlotB, "slot holds its window and descriptors");
constexpr int kSlots = 5;                // 153,600 B of the CU's 160 KiB
constexpr int kNL = kSlots;              // loader waves: one per slot
constexpr int kNC = 11;                  // consumer waves (16 waves per workgroup)
constexpr int kTaskBins = 16;            // bins per consumer task (4 lanes per bin)

// Bin kinds of the binning passes.
constexpr int kTiled = 0, kDirect = 1, kZero = 2;

struct TileGrid {
    int ty[VD_MAX_LEVELS], tx[VD_MAX_LEVELS];
    int base[VD_MAX_LEVELS + 1];  // first tile index of level l (all images)
};

// One chunk of one tile (every slice of it is an item of the ring kernel).
struct ChunkRec {
    const float *base;  // window origin pixel of the tile's image / level (slice 0)
    int rstride;        // bytes per level row (W * C * 4)
    int nrc;            // nrows | ncols << 8
    int start;          // first descriptor
    int count;          // descriptors (bins) of this chunk
    int pad0, pad1;
};

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
    const uint64_t dmask = ballot(bg.kind == kDirect);
    if (dmask) {
        const int dl = __ffsll((unsigned long long)dmask) - 1;
        int db = 0;
        if (lane == dl) db = atomicAdd(dir_cnt, (int)__popcll(dmask));
        db = __builtin_amdgcn_readlane(db, dl);
        if (bg.kind == kDirect) dir_list[db + lane_prefix(dmask)] = (int)g;
    }
    if (act) slot[g] = my_slot;
    if (bg.kind == kZero) {  // output_val = 0 / count
        float4 *dst = reinterpret_cast<float4 *>(out + g * C);
        for (int c = 0; c < C / 4; ++c) dst[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// 2. One workgroup: exclusive prefix of the tile counts (descriptor offsets) and
//    of the tiles' chunk counts; chunk_pre[T] = the number of chunks.
__global__ __launch_bounds__(1024) void tile_scan_kernel(int T, int chunk,
                                                         const int *__restrict__ cnt,
                                                         int *__restrict__ offset,
                                                         int *__restrict__ chunk_pre) {
    __shared__ int part[2][1024];
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
}

// A bin's descriptor (24 B): output bin (r * P + ph) * P + pw, packed
// window-relative taps, ly0, ly1, lx0, lx1 (as float bits).
struct Desc {
    int o, pk;
    float ly0, ly1, lx0, lx1;
};

// 3. Descriptors into per-tile contiguous storage; blocks past the bins' write
//    the chunk records (one lane per tile), in tile order = (level, image, tile
//    row, tile column): the order the XCDs' CUs sweep them.
__global__ __launch_bounds__(256) void bin_scatter_kernel(
    FpnLevels fa, TileGrid tg, int C, int chunk, const float *__restrict__ rois,
    const int *__restrict__ roi_level, int P, const int *__restrict__ slot,
    const int *__restrict__ cnt, const unsigned long long *__restrict__ ext,
    const int *__restrict__ offset, const int *__restrict__ chunk_pre, unsigned bin_blocks,
    Desc *__restrict__ desc, ChunkRec *__restrict__ chunks) {
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
        const unsigned long long ex = ext[i];
        const int nrows = 32 - __clz((int)(uint32_t)ex), ncols = 32 - __clz((int)(uint32_t)(ex >> 32));
        const int H = fa.H[l], W = fa.W[l];
        const float *org = fa.feat[l] + (((int64_t)b * H + ty * kT) * W + tx * kT) * C;
        const int nch = (c + chunk - 1) / chunk;
        for (int k = 0; k < nch; ++k) {
            ChunkRec it;
            it.base = org;
            it.rstride = W * C * 4;
            it.nrc = nrows | ncols << 8;
            it.start = offset[i] + k * chunk;
            it.count = min(chunk, c - k * chunk);
            it.pad0 = it.pad1 = 0;
            chunks[chunk_pre[i] + k] = it;
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
__device__ __forceinline__ void dma_1k(const void *sbase, uint32_t voff, uint32_t lds) {
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

// s_waitcnt vmcnt(n): all but this wave's n youngest vector-memory operations
// done (n wave-uniform, clamped to the 6-bit field: waiting for fewer
// outstanding operations is always safe since they complete in issue order).
__device__ __forceinline__ void wait_vm(int n) {
#define VD_W1(k)                                                 \
    case k:                                                      \
        asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory");    \
        break;
#define VD_W8(k) VD_W1(k) VD_W1(k + 1) VD_W1(k + 2) VD_W1(k + 3) VD_W1(k + 4) VD_W1(k + 5) \
    VD_W1(k + 6) VD_W1(k + 7)
    n = __builtin_amdgcn_readfirstlane(n);
    switch (n < 63 ? n : 63) {
        VD_W8(0) VD_W8(8) VD_W8(16) VD_W8(24) VD_W8(32) VD_W8(40) VD_W8(48) VD_W8(56)
        default:
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            break;
    }
#undef VD_W8
#undef VD_W1
}

typedef __attribute__((address_space(3))) const vf4 lds_f4;
typedef int vi2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const vi2 lds_i2;
typedef __attribute__((address_space(3))) volatile int lds_vi;

// Per-slot hand-off words in LDS.
struct Ring {
    int seq[kSlots];    // item index + 1 once the slot's window and descriptors landed
    int done[kSlots];   // consumers that have left the slot's current item
    int retired[kSlots];  // item index + 1 of the slot's last item every consumer left
    int count[kSlots];  // bins of the slot's item
    int ncols[kSlots];  // window columns
    int delta[kSlots];  // descriptor byte offset (16-B aligned DMA of the descriptors)
};

// Issue item (chunk record `it`, slice `sl`) into LDS slot byte address `slot`:
// the window (nrows x ncols pixels x 64 B, 16 pixels per wave instruction) and
// the 16-B aligned run of its descriptors.  Returns the DMA instructions issued.
__device__ __forceinline__ int issue_item(int C, const ChunkRec &it, int sl,
                                          const Desc *__restrict__ desc, uint32_t slot,
                                          int lane, int &delta_out) {
    const int nrows = it.nrc & 255, ncols = (it.nrc >> 8) & 255;
    const int npx = nrows * ncols;
    const int ninst = (npx + 15) >> 4;
    const uint32_t magic = (65536u + (uint32_t)ncols - 1u) / (uint32_t)ncols;
    const int q = lane & 3;
    const uint32_t pstride = (uint32_t)C * 4u;
    const float *wbase = it.base + sl * kG;
    int n = 0;
    for (int c = 0; c < ninst; ++c) {
        const int p = c * 16 + (lane >> 2);
        const int yy = (int)(((uint32_t)p * magic) >> 16);
        const int xx = p - yy * ncols;
        const uint32_t voff = (uint32_t)yy * (uint32_t)it.rstride + (uint32_t)xx * pstride +
                              (uint32_t)q * 16u;
        if (p < npx) dma_1k(wbase, voff, slot + (uint32_t)c * 1024u);  // lanes past the
        ++n;                                                          // window: masked
    }
    const int64_t b0 = (int64_t)it.start * 24;
    const int delta = (int)(b0 & 15);
    const char *dsrc = reinterpret_cast<const char *>(desc) + (b0 - delta);
    const int n16 = (delta + it.count * 24 + 15) >> 4;
    const int nd = (n16 + 63) >> 6;
    for (int c = 0; c < nd; ++c) {
        const int j = c * 64 + lane;
        if (j < n16) dma_1k(dsrc, (uint32_t)j * 16u, slot + kWinB + (uint32_t)c * 1024u);
        ++n;
    }
    delta_out = delta;
    return n;
}

// w1*v1 + w2*v2 + w3*v3 + w4*v4, left to right (roi_align_kernel.cu:60)
__device__ __forceinline__ float4 bil4(float w1, float w2, float w3, float w4, float4 a,
                                       float4 b, float4 c, float4 d) {
    return make_float4(w1 * a.x + w2 * b.x + w3 * c.x + w4 * d.x,
                       w1 * a.y + w2 * b.y + w3 * c.y + w4 * d.y,
                       w1 * a.z + w2 * b.z + w3 * c.z + w4 * d.z,
                       w1 * a.w + w2 * b.w + w3 * c.w + w4 * d.w);
}

__device__ __forceinline__ float4 lds4(lds_f4 *p) {
    const vf4 v = *p;
    return make_float4(v.x, v.y, v.z, v.w);
}

// One bin of a task: 4 channels (quad q of the slice) of bin descriptor (pk, lw).
__device__ __forceinline__ void bin_task(int pk, const float4 lw, lds_f4 *win, int ncols, int q,
                                         float *__restrict__ dst) {
    const int yo[2] = {pk & 31, (pk >> 5) & 31};
    const int xo[2] = {(pk >> 10) & 31, (pk >> 15) & 31};
    const int dy[2] = {(pk >> 20) & 1, (pk >> 21) & 1};
    const int dx[2] = {(pk >> 22) & 1, (pk >> 23) & 1};
    const bool vy[2] = {((pk >> 24) & 1) != 0, ((pk >> 25) & 1) != 0};
    const bool vx[2] = {((pk >> 26) & 1) != 0, ((pk >> 27) & 1) != 0};
    const float ly[2] = {lw.x, lw.y}, lx[2] = {lw.z, lw.w};
    float4 v[2][2][4];
#pragma unroll
    for (int iy = 0; iy < 2; ++iy) {
        const int rl = yo[iy] * ncols, rh = (yo[iy] + dy[iy]) * ncols;
#pragma unroll
        for (int ix = 0; ix < 2; ++ix) {
            const int cl = xo[ix], ch = xo[ix] + dx[ix];
            v[iy][ix][0] = lds4(win + (rl + cl) * 4 + q);
            v[iy][ix][1] = lds4(win + (rl + ch) * 4 + q);
            v[iy][ix][2] = lds4(win + (rh + cl) * 4 + q);
            v[iy][ix][3] = lds4(win + (rh + ch) * 4 + q);
        }
    }
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int iy = 0; iy < 2; ++iy) {
        const float hy = 1.f - ly[iy];
#pragma unroll
        for (int ix = 0; ix < 2; ++ix) {
            const float hx = 1.f - lx[ix];
            const float w1 = hy * hx, w2 = hy * lx[ix], w3 = ly[iy] * hx, w4 = ly[iy] * lx[ix];
            float4 val = bil4(w1, w2, w3, w4, v[iy][ix][0], v[iy][ix][1], v[iy][ix][2],
                              v[iy][ix][3]);
            if (!(vy[iy] && vx[ix])) val = make_float4(0.f, 0.f, 0.f, 0.f);
            acc.x += val.x;
            acc.y += val.y;
            acc.z += val.z;
            acc.w += val.w;
        }
    }
    const float count = 4.f;
    *reinterpret_cast<float4 *>(dst) =
        make_float4(acc.x / count, acc.y / count, acc.z / count, acc.w / count);
}

__device__ __forceinline__ void nap() { __builtin_amdgcn_s_sleep(1); }

#ifdef VD_RESEARCH_PROBES
// Per-wave cycle accounting of the ring (research build only; read by
// vd_research_ring_stats): [workgroup][wave][total, wait, work, items]
__device__ unsigned long long g_ring_stats[256][16][4];
#define VD_T(x) const unsigned long long x = __builtin_amdgcn_s_memtime()
#define VD_ACC(i, v) acc_[i] += (v)
#else
#define VD_T(x)
#define VD_ACC(i, v)
#endif

// 4. Persistent ring kernel: grid = 8 x K workgroups, block b on XCD x = b % 8,
// k = b / 8.  XCD x computes slices 2x, 2x + 1; its item list is (chunk, slice
// parity) in chunk order, and workgroup k takes items k, k + K8, ... with K8 =
// 8 x (K / 8)... here simply k + K m: chunk (k + K m) / 2, slice 2x + (k & 1)
// (K even).  Waves 0..kNL-1 load, the others compute.  MODE (diagnostics):
// 0 product, 1 no compute, 2 no window DMA.
template <int MODE>
__global__ __launch_bounds__((kNL + kNC) * 64) void ring_kernel(
    int C, const ChunkRec *__restrict__ chunks, const int *__restrict__ n_chunks,
    const Desc *__restrict__ desc, float *__restrict__ out) {
    __shared__ __attribute__((aligned(1024))) char lds[kSlots * kSlotB];
    __shared__ Ring ring;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int xcd = blockIdx.x & 7, K = gridDim.x >> 3, k = blockIdx.x >> 3;
    const int nchunk = __builtin_amdgcn_readfirstlane(*n_chunks);
    const int n_items = 2 * nchunk;              // this XCD's items: chunk x slice parity
    const int n_mine = k < n_items ? (n_items - k + K - 1) / K : 0;
    const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
    lds_vi *seqw = (lds_vi *)ring.seq;
    lds_vi *retw = (lds_vi *)ring.retired;
    if (threadIdx.x < kSlots) {
        ring.seq[threadIdx.x] = 0;
        ring.done[threadIdx.x] = 0;
        ring.retired[threadIdx.x] = 0;
    }
    __syncthreads();
#ifdef VD_RESEARCH_PROBES
    unsigned long long acc_[4] = {0, 0, 0, 0};
    VD_T(t_begin);
#endif
    if (wave < kNL) {
        // LOADER w owns slot w: items m = w, w + kSlots, ...  It refills its slot
        // once every consumer has left the slot's previous item, prefetches its
        // next chunk record while the DMA is in flight, waits for its own DMA
        // only and publishes.  kSlots loaders keep every free slot in flight.
        const int j = wave;
        ChunkRec it = {};
        if (j < n_mine) it = chunks[(k + K * j) >> 1];
        for (int m = j; m < n_mine; m += kSlots) {
            VD_T(t0);
            if (m >= kSlots)
                while (retw[j] != m - kSlots + 1) nap();  // item m - kSlots retired
            VD_T(t1);
            VD_ACC(1, t1 - t0);
            const int idx = k + K * m;
            const int sl = 2 * xcd + (idx & 1);
            int delta = 0;
            if (MODE != 2) {
                issue_item(C, it, sl, desc, lds_base + (uint32_t)j * kSlotB, lane, delta);
            } else {  // descriptors only
                ChunkRec d = it;
                d.nrc = 0;
                issue_item(C, d, sl, desc, lds_base + (uint32_t)j * kSlotB, lane, delta);
            }
            if (lane == 0) {
                ring.done[j] = 0;
                ring.count[j] = it.count;
                ring.ncols[j] = (it.nrc >> 8) & 255;
                ring.delta[j] = delta;
            }
            const int mn = m + kSlots;
            ChunkRec nx = it;
            if (mn < n_mine) nx = chunks[(k + K * mn) >> 1];  // lands during the DMA
            VD_T(t2);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            VD_T(t3);
            VD_ACC(2, t3 - t2);
            VD_ACC(3, 1);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) seqw[j] = m + 1;
            it = nx;
        }
#ifdef VD_RESEARCH_PROBES
        VD_T(t_end);
        if (lane == 0 && blockIdx.x < 256) {
            g_ring_stats[blockIdx.x][wave][0] = t_end - t_begin;
            for (int i = 1; i < 4; ++i) g_ring_stats[blockIdx.x][wave][i] = acc_[i];
        }
#endif
        return;
    }
    // CONSUMER c: tasks t of item m with (t - m) mod kNC == c
    const int c = wave - kNL;
    const int q = lane & 3, bsub = lane >> 2;
    for (int m = 0; m < n_mine; ++m) {
        const int j = m % kSlots;
        VD_T(t0);
        while (seqw[j] != m + 1) nap();
        VD_T(t1);
        VD_ACC(1, t1 - t0);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int count = __builtin_amdgcn_readfirstlane(ring.count[j]);
        const int ncols = __builtin_amdgcn_readfirstlane(ring.ncols[j]);
        const int delta = __builtin_amdgcn_readfirstlane(ring.delta[j]);
        const int idx = k + K * m;
        const int sl = 2 * xcd + (idx & 1);
        const int ntask = (count + kTaskBins - 1) / kTaskBins;
        lds_f4 *win = (lds_f4 *)(lds + j * kSlotB);
        int t = c - m % kNC;
        if (t < 0) t += kNC;
        if (MODE != 1) {
            for (; t < ntask; t += kNC) {
                const int bi = t * kTaskBins + bsub;
                const bool on = bi < count;
                lds_i2 *dp = (lds_i2 *)((__attribute__((address_space(3))) const char *)win +
                                        kWinB + delta + (on ? bi : 0) * 24);
                const vi2 a = dp[0], l01 = dp[1], l23 = dp[2];
                const float4 lw = make_float4(__int_as_float(l01.x), __int_as_float(l01.y),
                                              __int_as_float(l23.x), __int_as_float(l23.y));
                if (on)
                    bin_task(a.y, lw, win, ncols, q, out + (int64_t)a.x * C + sl * kG + q * 4);
            }
        }
        // this wave's reads of the slot are done; the last consumer out retires it
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0 && atomicAdd((int *)&ring.done[j], 1) == kNC - 1) retw[j] = m + 1;
        VD_T(t2);
        VD_ACC(2, t2 - t1);
        VD_ACC(3, ntask > 0 ? (ntask - 1 - (c - m % kNC + kNC) % kNC) / kNC + 1 : 0);
    }
#ifdef VD_RESEARCH_PROBES
    VD_T(t_end);
    if (lane == 0 && blockIdx.x < 256) {
        g_ring_stats[blockIdx.x][wave][0] = t_end - t_begin;
        for (int i = 1; i < 4; ++i) g_ring_stats[blockIdx.x][wave][i] = acc_[i];
    }
#endif
}

// 5. Direct-list bins: one wave per bin, every channel from global memory, the
// same per-sample arithmetic.  Grid-stride over the device-side count.
__global__ __launch_bounds__(256) void direct_kernel(FpnLevels fa, int C,
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

size_t a256(size_t n) { return (n + 255) & ~(size_t)255; }

struct Ws {
    int *cnt;
    unsigned long long *ext;
    int *dir_cnt;
    int *slot, *offset, *chunk_pre, *dir_list;
    ChunkRec *chunks;
    Desc *desc;
    size_t zero_bytes, total;
};

Ws carve(const FpnLevels &fa, int R, int P, char *p) {
    const TileGrid tg = tile_grid(fa);
    const size_t T = (size_t)tg.base[fa.L];
    const size_t nb = (size_t)R * P * P;
    const size_t max_chunks = T + nb / 8 + 1;
    Ws w;
    char *p0 = p;
    w.ext = (unsigned long long *)p;  // zeroed region first: ext, cnt, dir_cnt
    p += a256(T * 8);
    w.cnt = (int *)p;
    p += a256(T * 4);
    w.dir_cnt = (int *)p;
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
    w.chunks = (ChunkRec *)p;
    p += a256(max_chunks * sizeof(ChunkRec));
    w.desc = (Desc *)p;
    p += a256(nb * sizeof(Desc) + 64);
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

}  // namespace raring

#ifdef VD_RESEARCH_PROBES
// Research build: copy the last ring launch's per-wave cycle accounting out.
extern "C" int vd_research_ring_stats(unsigned long long *host, int n) {
    const size_t bytes = sizeof(raring::g_ring_stats);
    if (!host || (size_t)n * 8 < bytes) return VD_ERR_ARG;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(raring::g_ring_stats), bytes, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}
#endif

bool roi_align_ring_supported(const FpnLevels &fa, int C, int P, int sr) {
    using namespace raring;
    // XCD x computes slices 2x, 2x + 1: exactly 16 slices of 16 channels
    if (sr != 2 || P < 1 || P > 64 || C != 16 * kG) return false;
    for (int l = 0; l < fa.L; ++l)  // 32-bit per-lane DMA offsets within an image
        if ((int64_t)fa.H[l] * fa.W[l] * C * 4 >= (1ll << 31)) return false;
    return (int64_t)fa.R * P * P < (1ll << 31) / 2;
}

size_t roi_align_ring_workspace_bytes(const FpnLevels &fa, int R, int P) {
    return raring::carve(fa, R, P, nullptr).total;
}

int launch_roi_align_fpn_ring(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                              int R, int P, int sr, float *out, void *ws, size_t ws_bytes,
                              hipStream_t s) {
    using namespace raring;
    if (R == 0) return VD_OK;
    if (!roi_align_ring_supported(fa, C, P, sr)) return VD_ERR_SHAPE;
    const Ws w = carve(fa, R, P, (char *)ws);
    if (!ws || ws_bytes < w.total) return VD_ERR_WORKSPACE;
    const TileGrid tg = tile_grid(fa);
    const int64_t nb = (int64_t)R * P * P;
    if (hipMemsetAsync(w.ext, 0, w.zero_bytes, s) != hipSuccess) return VD_ERR_LAUNCH;
    const unsigned blk = (unsigned)((nb + 255) / 256);
    const int T = tg.base[fa.L];
    const char *ec = getenv("VOSDET_RA_CHUNK");  // tests: smaller chunks, more items
    int chunk = ec ? atoi(ec) : kMaxChunk;
    if (chunk < 8 || chunk > kMaxChunk) chunk = kMaxChunk;
    hipLaunchKernelGGL(bin_count_kernel, dim3(blk), dim3(256), 0, s, fa, tg, C, rois, lvl, P,
                       w.cnt, w.ext, w.slot, w.dir_cnt, w.dir_list, out);
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, T, chunk, w.cnt,
                       w.offset, w.chunk_pre);
    hipLaunchKernelGGL(bin_scatter_kernel, dim3(blk + (unsigned)((T + 255) / 256)), dim3(256), 0,
                       s, fa, tg, C, chunk, rois, lvl, P, w.slot, w.cnt, w.ext, w.offset,
                       w.chunk_pre, blk, w.desc, w.chunks);
    int nblk = num_cus() / 16 * 16;  // K = nblk / 8 workgroups per XCD, K even
    if (nblk < 16) nblk = 16;
    const char *em = getenv("VOSDET_RA_RING_MODE");  // diagnostics: 1 no compute, 2 no DMA
    const int mode = em ? atoi(em) : 0;
    if (mode == 1)
        hipLaunchKernelGGL(ring_kernel<1>, dim3(nblk), dim3((kNL + kNC) * 64), 0, s, C, w.chunks,
                           w.chunk_pre + T, w.desc, out);
    else if (mode == 2)
        hipLaunchKernelGGL(ring_kernel<2>, dim3(nblk), dim3((kNL + kNC) * 64), 0, s, C, w.chunks,
                           w.chunk_pre + T, w.desc, out);
    else
        hipLaunchKernelGGL(ring_kernel<0>, dim3(nblk), dim3((kNL + kNC) * 64), 0, s, C, w.chunks,
                           w.chunk_pre + T, w.desc, out);
    hipLaunchKernelGGL(direct_kernel, dim3(256), dim3(256), 0, s, fa, C, rois, lvl, P, w.dir_cnt,
                       w.dir_list, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
