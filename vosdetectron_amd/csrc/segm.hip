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
#include "vosdet_internal.hpp"

namespace vd {

static constexpr int kPasteMaxR = 62;  // (R+2)^2 floats in LDS

__global__ __launch_bounds__(256) void paste_masks_kernel(
    const float *__restrict__ masks, int R, const float *__restrict__ boxes, int box_stride,
    int im_h, int im_w, int rows_per_band, float thresh, uint8_t *__restrict__ out) {
    __shared__ float pm[(kPasteMaxR + 2) * (kPasteMaxR + 2)];
    const int m = blockIdx.x;
    const int S = R + 2;
    const float *src = masks + (int64_t)m * R * R;
    for (int i = threadIdx.x; i < S * S; i += blockDim.x) {
        const int y = i / S, x = i - y * S;
        pm[i] = (y >= 1 && y <= R && x >= 1 && x <= R) ? src[(y - 1) * R + (x - 1)] : 0.f;
    }
    __syncthreads();
    // expand_boxes in float32 (numpy: float32 array op python float), then
    // astype(int32) truncates toward zero
    const float *b = boxes + (int64_t)m * box_stride;
    const float scale = (float)((R + 2.0) / R);
    float w_half = (b[2] - b[0]) * .5f, h_half = (b[3] - b[1]) * .5f;
    const float x_c = (b[2] + b[0]) * .5f, y_c = (b[3] + b[1]) * .5f;
    w_half *= scale;
    h_half *= scale;
    const int bx0 = (int)(x_c - w_half), bx2 = (int)(x_c + w_half);
    const int by0 = (int)(y_c - h_half), by2 = (int)(y_c + h_half);
    const int w = max(bx2 - bx0 + 1, 1), h = max(by2 - by0 + 1, 1);
    const int x_0 = max(bx0, 0), x_1 = min(bx2 + 1, im_w);
    const int y_0 = max(by0, 0), y_1 = min(by2 + 1, im_h);
    const double scale_x = 1. / ((double)w / (double)S), scale_y = 1. / ((double)h / (double)S);
    // OpenCV's resize dispatch turns INTER_LINEAR into INTER_AREA's fast path
    // when both scales are exactly 2 (a 15 x 15 box for R = 28): the mean of
    // each 2 x 2 block, ((a + b) + c) + d) * 0.25f in its scalar loop order
    // (restated from OpenCV's resize.cpp as remembered; cv2 absent: unpinned)
    const bool area2 = scale_x == 2.0 && scale_y == 2.0;

    const int ybeg = blockIdx.y * rows_per_band;
    const int yend = min(ybeg + rows_per_band, im_h);
    uint8_t *plane = out + (int64_t)m * im_h * im_w;
    for (int y = ybeg; y < yend; ++y) {
        const bool yin = y >= y_0 && y < y_1;
        int r0 = 0, r1 = 0;
        float b0 = 0.f, b1 = 0.f;
        if (yin) {
            const int dy = y - by0;
            float fy = (float)((dy + 0.5) * scale_y - 0.5);
            const int sy = (int)floorf(fy);
            fy -= (float)sy;
            r0 = min(max(sy, 0), S - 1);
            r1 = min(max(sy + 1, 0), S - 1);
            b0 = 1.f - fy;
            b1 = fy;
        }
        for (int x = threadIdx.x; x < im_w; x += blockDim.x) {
            uint8_t v = 0;
            if (yin && x >= x_0 && x < x_1 && area2) {
                const int dx = x - bx0, dy = y - by0;
                const float *p0 = pm + (2 * dy) * S + 2 * dx, *p1 = p0 + S;
                const float val = (((p0[0] + p0[1]) + p1[0]) + p1[1]) * 0.25f;
                v = val > thresh ? 1 : 0;
            } else if (yin && x >= x_0 && x < x_1) {
                const int dx = x - bx0;
                float fx = (float)((dx + 0.5) * scale_x - 0.5);
                int sx = (int)floorf(fx);
                fx -= (float)sx;
                if (sx < 0) { fx = 0.f; sx = 0; }
                if (sx >= S - 1) { fx = 0.f; sx = S - 1; }
                const float a0 = 1.f - fx, a1 = fx;
                const int sx1 = min(sx + 1, S - 1);
                const float d0 = pm[r0 * S + sx] * a0 + pm[r0 * S + sx1] * a1;
                const float d1 = pm[r1 * S + sx] * a0 + pm[r1 * S + sx1] * a1;
                const float val = d0 * b0 + d1 * b1;
                v = val > thresh ? 1 : 0;
            }
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

}  // namespace vd
