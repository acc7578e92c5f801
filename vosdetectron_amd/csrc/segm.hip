// segm_results on the device: paste + binarize + COCO RLE counts.
//
// Reference: lib/core/test.py:801-855 segm_results (fork copy
// lib_vos/tools/vos_test.py:867-921), box_utils.expand_boxes
// (lib/utils/boxes.py:242-258), cv2.resize INTER_LINEAR on float32 and
// pycocotools mask.encode (column-major run lengths).
//
// paste_masks_kernel: grid (detection, row band).  The (R+2)^2 zero-padded
// mask sits in LDS; each lane produces one image byte of its band, so a
// detection's whole frame plane is written once, coalesced, zeros included
// (the reference's np.zeros + slice assignment).  The resize is OpenCV's
// scalar INTER_LINEAR for float images, restated:
//   x: fx = (float)((dx + 0.5) * scale_x - 0.5), sx = floor(fx), fx -= sx,
//      sx < 0 -> (sx, fx) = (0, 0); sx >= S-1 -> (S-1, 0)  (resize.cpp tables),
//      row value D = S[sx] * (1 - fx) + S[sx+1] * fx  (HResizeLinear; the right
//      border uses S[sx] * 1 only, the same float result);
//   y: fy likewise, rows clip(sy, 0, S-1), clip(sy + 1, 0, S-1), no fy clamp,
//      value = D0 * (1 - fy) + D1 * fy  (VResizeLinear);
//   scale = 1 / (dsize / ssize) in double, as cv::resize computes it.
// Built with -ffp-contract=off, so every product and sum rounds as the numpy
// restatement in oracle/oracle.py does.
//
// mask_rle_kernel: one workgroup per detection; a lane walks whole columns of
// the pasted plane (column-major = pycocotools' Fortran order), counts value
// changes, a block scan places each change position, and the positions are
// differenced in place into run lengths starting with a zero run, exactly
// rleEncode's counts.
#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

static constexpr int kPasteMaxR = 62;  // (R+2)^2 floats in LDS

// One detection's paste geometry (expand_boxes, the clipped box, OpenCV's
// resize scales) and its pixel function over the zero-padded mask in LDS.
struct PasteGeom {
    int S, bx0, by0, x_0, x_1, y_0, y_1;
    double scale_x, scale_y;
    bool area2;
};

__device__ __forceinline__ PasteGeom paste_geom(const float *b, int R, int im_h, int im_w) {
    PasteGeom g;
    g.S = R + 2;
    // expand_boxes in float32 (numpy: float32 array op python float), then
    // astype(int32) truncates toward zero
    const float scale = (float)((R + 2.0) / R);
    float w_half = (b[2] - b[0]) * .5f, h_half = (b[3] - b[1]) * .5f;
    const float x_c = (b[2] + b[0]) * .5f, y_c = (b[3] + b[1]) * .5f;
    w_half *= scale;
    h_half *= scale;
    const int bx0 = (int)(x_c - w_half), bx2 = (int)(x_c + w_half);
    const int by0 = (int)(y_c - h_half), by2 = (int)(y_c + h_half);
    const int w = max(bx2 - bx0 + 1, 1), h = max(by2 - by0 + 1, 1);
    g.bx0 = bx0;
    g.by0 = by0;
    g.x_0 = max(bx0, 0);
    g.x_1 = min(bx2 + 1, im_w);
    g.y_0 = max(by0, 0);
    g.y_1 = min(by2 + 1, im_h);
    g.scale_x = 1. / ((double)w / (double)g.S);
    g.scale_y = 1. / ((double)h / (double)g.S);
    // OpenCV's resize dispatch turns INTER_LINEAR into INTER_AREA's fast path
    // when both scales are exactly 2 (a 15 x 15 box for R = 28): the mean of
    // each 2 x 2 block, ((a + b) + c) + d) * 0.25f in its scalar loop order
    // (restated from OpenCV's resize.cpp as remembered; cv2 absent: unpinned)
    g.area2 = g.scale_x == 2.0 && g.scale_y == 2.0;
    return g;
}

struct PasteRow {  // VResizeLinear taps of one output row
    int r0, r1;
    float b0, b1;
};

__device__ __forceinline__ PasteRow paste_row(const PasteGeom &g, int y) {
    PasteRow r;
    const int dy = y - g.by0;
    float fy = (float)((dy + 0.5) * g.scale_y - 0.5);
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    r.r0 = min(max(sy, 0), g.S - 1);
    r.r1 = min(max(sy + 1, 0), g.S - 1);
    r.b0 = 1.f - fy;
    r.b1 = fy;
    return r;
}

struct PasteCol {  // HResizeLinear taps of one output column
    int sx, sx1;
    float a0, a1;
};

__device__ __forceinline__ PasteCol paste_col(const PasteGeom &g, int x) {
    PasteCol c;
    const int dx = x - g.bx0;
    float fx = (float)((dx + 0.5) * g.scale_x - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) { fx = 0.f; sx = 0; }
    if (sx >= g.S - 1) { fx = 0.f; sx = g.S - 1; }
    c.sx = sx;
    c.sx1 = min(sx + 1, g.S - 1);
    c.a0 = 1.f - fx;
    c.a1 = fx;
    return c;
}

// Binarised pasted value of in-box pixel (x, y): cv2.resize(...) > thresh.
__device__ __forceinline__ int paste_pixel(const float *pm, const PasteGeom &g, const PasteRow &r,
                                           const PasteCol &c, int x, int y, float thresh) {
    const int S = g.S;
    if (g.area2) {
        const int dx = x - g.bx0, dy = y - g.by0;
        const float *p0 = pm + (2 * dy) * S + 2 * dx, *p1 = p0 + S;
        const float val = (((p0[0] + p0[1]) + p1[0]) + p1[1]) * 0.25f;
        return val > thresh ? 1 : 0;
    }
    const float d0 = pm[r.r0 * S + c.sx] * c.a0 + pm[r.r0 * S + c.sx1] * c.a1;
    const float d1 = pm[r.r1 * S + c.sx] * c.a0 + pm[r.r1 * S + c.sx1] * c.a1;
    const float val = d0 * r.b0 + d1 * r.b1;
    return val > thresh ? 1 : 0;
}

// (R+2)^2 zero-padded mask of detection m into LDS
__device__ __forceinline__ void load_padded(float *pm, const float *src, int R) {
    const int S = R + 2;
    for (int i = threadIdx.x; i < S * S; i += blockDim.x) {
        const int y = i / S, x = i - y * S;
        pm[i] = (y >= 1 && y <= R && x >= 1 && x <= R) ? src[(y - 1) * R + (x - 1)] : 0.f;
    }
}

__global__ __launch_bounds__(256) void paste_masks_kernel(
    const float *__restrict__ masks, int R, const float *__restrict__ boxes, int box_stride,
    int im_h, int im_w, int rows_per_band, float thresh, uint8_t *__restrict__ out) {
    __shared__ float pm[(kPasteMaxR + 2) * (kPasteMaxR + 2)];
    const int m = blockIdx.x;
    load_padded(pm, masks + (int64_t)m * R * R, R);
    __syncthreads();
    const PasteGeom g = paste_geom(boxes + (int64_t)m * box_stride, R, im_h, im_w);
    const int ybeg = blockIdx.y * rows_per_band;
    const int yend = min(ybeg + rows_per_band, im_h);
    uint8_t *plane = out + (int64_t)m * im_h * im_w;
    for (int y = ybeg; y < yend; ++y) {
        const bool yin = y >= g.y_0 && y < g.y_1;
        const PasteRow r = paste_row(g, yin ? y : g.y_0);
        for (int x = threadIdx.x; x < im_w; x += blockDim.x) {
            uint8_t v = 0;
            if (yin && x >= g.x_0 && x < g.x_1)
                v = (uint8_t)paste_pixel(pm, g, r, paste_col(g, x), x, y, thresh);
            plane[(int64_t)y * im_w + x] = v;
        }
    }
}

int launch_paste_masks(const float *masks, int M, int R, const float *boxes, int box_stride,
                       int im_h, int im_w, float thresh, uint8_t *out, hipStream_t s) {
    if (M == 0) return VD_OK;
    if (R < 1 || R > kPasteMaxR) return VD_ERR_SHAPE;
    const int rows = 16;
    const dim3 grid(M, (im_h + rows - 1) / rows);
    hipLaunchKernelGGL(paste_masks_kernel, grid, dim3(256), 0, s, masks, R, boxes, box_stride,
                       im_h, im_w, rows, thresh, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// --------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void mask_rle_kernel(const uint8_t *__restrict__ planes,
                                                         int H, int W, uint32_t *__restrict__ counts,
                                                         int cap, int32_t *__restrict__ ncounts) {
    __shared__ int scan[1024];
    const int m = blockIdx.x;
    const uint8_t *p = planes + (int64_t)m * H * W;
    uint32_t *cnt = counts + (int64_t)m * cap;
    const int t = threadIdx.x, nt = blockDim.x;
    // columns [c0, c1) of this lane (contiguous split keeps positions ordered by lane)
    const int per = (W + nt - 1) / nt;
    const int c0 = min(t * per, W), c1 = min(c0 + per, W);
    auto prev_of = [&](int x) -> uint8_t {  // element before (0, x) in column-major order
        return x == 0 ? (uint8_t)0 : p[(int64_t)(H - 1) * W + (x - 1)];
    };
    int changes = 0;
    for (int x = c0; x < c1; ++x) {
        uint8_t prev = prev_of(x);
        for (int y = 0; y < H; ++y) {
            const uint8_t v = p[(int64_t)y * W + x];
            changes += v != prev;
            prev = v;
        }
    }
    // inclusive block scan of the per-lane change counts
    scan[t] = changes;
    __syncthreads();
    for (int off = 1; off < nt; off <<= 1) {
        const int v = t >= off ? scan[t - off] : 0;
        __syncthreads();
        scan[t] += v;
        __syncthreads();
    }
    const int total = scan[nt - 1];
    const int n = total + 1;  // runs: the leading (possibly empty) zero run + one per change
    if (t == 0) ncounts[m] = n <= cap ? n : -n;
    if (n > cap) return;  // caller retries with cap >= n
    // positions of the changes at cnt[1..total]
    int k = scan[t] - changes + 1;
    for (int x = c0; x < c1; ++x) {
        uint8_t prev = prev_of(x);
        for (int y = 0; y < H; ++y) {
            const uint8_t v = p[(int64_t)y * W + x];
            if (v != prev) cnt[k++] = (uint32_t)((int64_t)x * H + y);
            prev = v;
        }
    }
    if (t == 0) cnt[0] = 0;
    __threadfence_block();
    __syncthreads();
    // run lengths: counts[i] = pos[i+1] - pos[i] with pos[0] = 0, pos[n] = H*W.
    // In place, lowest chunk first: a chunk reads its own slots and the first slot
    // of the next chunk, none of which an earlier chunk rewrote.
    const uint32_t hw = (uint32_t)((int64_t)H * W);
    const int nchunks = (n + nt - 1) / nt;
    for (int c = 0; c < nchunks; ++c) {
        const int i = c * nt + t;
        uint32_t a = 0, bnext = 0;
        if (i < n) {
            a = cnt[i];
            bnext = i + 1 < n ? cnt[i + 1] : hw;
        }
        __threadfence_block();
        __syncthreads();
        if (i < n) cnt[i] = bnext - a;
        __threadfence_block();
        __syncthreads();
    }
}

int launch_mask_rle(const uint8_t *planes, int M, int H, int W, uint32_t *counts, int cap,
                    int32_t *ncounts, hipStream_t s) {
    if (M == 0) return VD_OK;
    hipLaunchKernelGGL(mask_rle_kernel, dim3(M), dim3(1024), 0, s, planes, H, W, counts, cap,
                       ncounts);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// --------------------------------------------------------------------------
// Fused segm_results RLE: the pycocotools counts of every detection's pasted
// plane without writing the plane.  Outside the clipped box the plane is 0, so
// in column-major order every change lies in a box column x at a position
// x*H + y with y in [y_0, y_1] (y_1: the 1 -> 0 step below the box, or, for a
// full-height box, the first pixel of the next column).  One wave walks one
// box column 64 rows at a time: each lane evaluates its pixel from the padded
// mask in LDS (paste_pixel, bit-identical to vd_paste_masks), compares it
// with the lane above (DPP shift; lane 0 takes the previous chunk's last
// value) and a ballot counts / places the changes.  Pass 1 counts per column,
// a block scan orders the columns, pass 2 writes the positions, and they are
// differenced into run lengths as mask_rle_kernel does.
// --------------------------------------------------------------------------
static constexpr int kSegmMaxW = 8192;

template <bool WRITE>
__device__ int segm_column_changes(const float *pm, const PasteGeom &g, int x, int H, int W,
                                   float thresh, uint32_t *pos) {
    const int lane = lane_id();
    const PasteCol c = paste_col(g, x);
    int prev = 0;  // the plane value just before (x, y_0) in column-major order
    if (g.y_0 == 0 && g.y_1 == H && x > g.x_0)
        prev = paste_pixel(pm, g, paste_row(g, H - 1), paste_col(g, x - 1), x - 1, H - 1, thresh);
    int cnt = 0;
    for (int yb = g.y_0; yb < g.y_1; yb += VD_WAVE) {
        const int y = yb + lane;
        const bool in = y < g.y_1;
        const int v = in ? paste_pixel(pm, g, paste_row(g, y), c, x, y, thresh) : 0;
        int vp = __shfl_up(v, 1);
        if (lane == 0) vp = prev;
        const bool ch = in && v != vp;
        const uint64_t b = ballot(ch);
        if (WRITE && ch) pos[cnt + lane_prefix(b)] = (uint32_t)((int64_t)x * H + y);
        cnt += __popcll(b);
        prev = __shfl(v, min(VD_WAVE - 1, g.y_1 - 1 - yb));
    }
    // 1 -> 0 after the column's last box pixel, unless that next position is the
    // first pixel of the next box column (which compares against it itself)
    const int64_t q = (int64_t)x * H + g.y_1;
    if (prev == 1 && q < (int64_t)H * W && !(g.y_1 == H && g.y_0 == 0 && x + 1 < g.x_1)) {
        if (WRITE && lane == 0) pos[cnt] = (uint32_t)q;
        ++cnt;
    }
    return cnt;
}

__global__ __launch_bounds__(256) void segm_rle_kernel(
    const float *__restrict__ masks, int R, const float *__restrict__ boxes, int box_stride,
    int H, int W, float thresh, uint32_t *__restrict__ counts, int cap,
    int32_t *__restrict__ ncounts) {
    __shared__ float pm[(kPasteMaxR + 2) * (kPasteMaxR + 2)];
    __shared__ int colofs[kSegmMaxW + 1];
    __shared__ int part[256];
    const int m = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    load_padded(pm, masks + (int64_t)m * R * R, R);
    __syncthreads();
    const PasteGeom g = paste_geom(boxes + (int64_t)m * box_stride, R, H, W);
    const int ncol = (g.y_1 > g.y_0 && g.x_1 > g.x_0) ? g.x_1 - g.x_0 : 0;
    uint32_t *cnt = counts + (int64_t)m * cap;
    const int wv = wave_id(), nw = num_waves();
    for (int ci = wv; ci < ncol; ci += nw) {
        const int k = segm_column_changes<false>(pm, g, g.x_0 + ci, H, W, thresh, nullptr);
        if (lane_id() == 0) colofs[ci] = k;
    }
    __syncthreads();
    // exclusive scan of the per-column counts: contiguous chunk per thread
    const int per = (ncol + nt - 1) / nt;
    const int a0 = min(t * per, ncol), a1 = min(a0 + per, ncol);
    int sum = 0;
    for (int i = a0; i < a1; ++i) sum += colofs[i];
    part[t] = sum;
    __syncthreads();
    for (int off = 1; off < nt; off <<= 1) {
        const int v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const int total = part[nt - 1];
    int run = part[t] - sum;
    for (int i = a0; i < a1; ++i) {
        const int k = colofs[i];
        colofs[i] = run;
        run += k;
    }
    const int n = total + 1;
    if (t == 0) ncounts[m] = n <= cap ? n : -n;
    if (n > cap) return;  // caller retries with cap >= n
    __syncthreads();
    for (int ci = wv; ci < ncol; ci += nw)
        segm_column_changes<true>(pm, g, g.x_0 + ci, H, W, thresh, cnt + 1 + colofs[ci]);
    if (t == 0) cnt[0] = 0;
    __threadfence_block();
    __syncthreads();
    const uint32_t hw = (uint32_t)((int64_t)H * W);
    const int nchunks = (n + nt - 1) / nt;
    for (int c = 0; c < nchunks; ++c) {
        const int i = c * nt + t;
        uint32_t a = 0, bnext = 0;
        if (i < n) {
            a = cnt[i];
            bnext = i + 1 < n ? cnt[i + 1] : hw;
        }
        __threadfence_block();
        __syncthreads();
        if (i < n) cnt[i] = bnext - a;
        __threadfence_block();
        __syncthreads();
    }
}

int launch_segm_rle(const float *masks, int M, int R, const float *boxes, int box_stride,
                    int im_h, int im_w, float thresh, uint32_t *counts, int cap,
                    int32_t *ncounts, hipStream_t s) {
    if (M == 0) return VD_OK;
    if (R < 1 || R > kPasteMaxR || im_w > kSegmMaxW) return VD_ERR_SHAPE;
    hipLaunchKernelGGL(segm_rle_kernel, dim3(M), dim3(256), 0, s, masks, R, boxes, box_stride,
                       im_h, im_w, thresh, counts, cap, ncounts);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// --------------------------------------------------------------------------
// rleToString (pycocotools maskApi.c) on the device.  Count i becomes
// x = cnts[i] - cnts[i-2] (i > 2; signed 64-bit), emitted 5 bits per char
// low bits first, 0x20 = "more", char + 48, stopping when the rest is 0 (or
// -1 with the sign bit 0x10 set in the last char).  Per detection one
// workgroup: chunk of 256 counts -> char lengths -> block scan -> chars.
// lengths mode (chars == NULL) writes lens[m]; write mode places detection
// m's string at sum(lens[0..m)) of one packed buffer.
// --------------------------------------------------------------------------
__device__ __forceinline__ int64_t rle_delta(const uint32_t *c, int i) {
    int64_t x = (int64_t)c[i];
    if (i > 2) x -= (int64_t)c[i - 2];
    return x;
}

__device__ __forceinline__ int rle_char_len(int64_t x) {
    int len = 0;
    bool more = true;
    while (more) {
        const int ch = (int)(x & 0x1f);
        x >>= 5;
        more = (ch & 0x10) ? x != -1 : x != 0;
        ++len;
    }
    return len;
}

__global__ __launch_bounds__(256) void rle_string_kernel(const uint32_t *__restrict__ counts,
                                                         const int32_t *__restrict__ ncounts,
                                                         int cap, int32_t *__restrict__ lens,
                                                         uint8_t *__restrict__ chars) {
    __shared__ int part[256];
    __shared__ long long base_s;
    const int m = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    const int n = ncounts[m];
    const uint32_t *c = counts + (int64_t)m * cap;
    if (chars) {  // this detection's offset in the packed buffer
        long long b = 0;
        for (int j = t; j < m; j += nt) b += lens[j];
        part[t] = (int)b;  // lens sum < 2^31 (checked by the host)
        __syncthreads();
        if (t == 0) {
            long long tot = 0;
            for (int j = 0; j < nt; ++j) tot += part[j];
            base_s = tot;
        }
        __syncthreads();
    }
    const long long base = chars ? base_s : 0;
    int run = 0;
    const int nn = n > 0 ? n : 0;
    for (int c0 = 0; c0 < nn; c0 += nt) {
        const int i = c0 + t;
        const int64_t x = i < nn ? rle_delta(c, i) : 0;
        const int len = i < nn ? rle_char_len(x) : 0;
        __syncthreads();
        part[t] = len;
        __syncthreads();
        for (int off = 1; off < nt; off <<= 1) {
            const int v = t >= off ? part[t - off] : 0;
            __syncthreads();
            part[t] += v;
            __syncthreads();
        }
        if (chars && i < nn) {
            uint8_t *o = chars + base + run + part[t] - len;
            int64_t y = x;
            bool more = true;
            while (more) {
                int ch = (int)(y & 0x1f);
                y >>= 5;
                more = (ch & 0x10) ? y != -1 : y != 0;
                if (more) ch |= 0x20;
                *o++ = (uint8_t)(ch + 48);
            }
        }
        run += part[nt - 1];
    }
    if (!chars && t == 0) lens[m] = run;
}

int launch_rle_strings(const uint32_t *counts, const int32_t *ncounts, int M, int cap,
                       int32_t *lens, uint8_t *chars, hipStream_t s) {
    if (M == 0) return VD_OK;
    hipLaunchKernelGGL(rle_string_kernel, dim3(M), dim3(256), 0, s, counts, ncounts, cap, lens,
                       chars);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
