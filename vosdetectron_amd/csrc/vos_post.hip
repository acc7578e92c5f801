// The VOS fork's two frame-level detection heuristics on the device
// (lib_vos/tools/vos_test.py):
//
//  * NMS_SMALL_BOX_IOU (:845-860, inside box_results_with_nms_and_limit): a
//    class's boxes whose IoU with the PREVIOUS frame's single, confident box of
//    that class is below the threshold are dropped.  IoU as
//    bb_intersection_over_union (:961-982) evaluates it on float32 box rows under
//    numpy 2: differences, +1 widths, products, sums and the division all in
//    float32; the comparison with the threshold in float32 too.
//  * nms_with_mask_iou (:985-1029, called at :113-118 after segm_results): the
//    frame's binary masks (the pasted, thresholded segms), greedy in score order:
//    position j is discarded by an earlier kept i when inter / (|m_i| + 1e-6) or
//    inter / (|m_j| + 1e-6) exceeds iou_th (float64, as numpy divides its integer
//    sums), then at most max_per_class detections per class, output class-major.
//
// Masks are bit-packed once (32 pixels per word, row-major over the frame), pair
// intersections are popcounts over the rows both masks occupy, and the greedy
// pass runs in one workgroup with the discard flags in LDS.
#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

namespace {

constexpr int kMaxMaskNms = 1024;

__global__ void zero_count_kernel(int32_t *p) { *p = 0; }

struct MaskWs {
    uint32_t *bits;  // [n][nw]
    int64_t *area;   // [n]
    int *row0, *row1;  // [n] first / last row with a set pixel (row0 > row1: empty)
    int32_t *inter;  // [n][n], i < j
};

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

MaskWs carve_mask_ws(void *p, int n, int nw, size_t *total) {
    char *c = (char *)p;
    MaskWs w;
    size_t off = 0;
    w.bits = (uint32_t *)(c + off);
    off += align256((size_t)n * nw * 4);
    w.area = (int64_t *)(c + off);
    off += align256((size_t)n * 8);
    w.row0 = (int *)(c + off);
    off += align256((size_t)n * 4);
    w.row1 = (int *)(c + off);
    off += align256((size_t)n * 4);
    w.inter = (int32_t *)(c + off);
    off += align256((size_t)n * n * 4);
    if (total) *total = off;
    return w;
}

// One workgroup per mask: pack 32 pixels per word, count the set pixels, find
// the first / last occupied row.
__global__ __launch_bounds__(256) void mask_pack_kernel(const uint8_t *__restrict__ planes,
                                                        int HW, int W, int nw, MaskWs ws) {
    const int m = blockIdx.x;
    const uint8_t *p = planes + (int64_t)m * HW;
    uint32_t *bits = ws.bits + (int64_t)m * nw;
    __shared__ unsigned long long red[256];
    __shared__ int rmin[256], rmax[256];
    unsigned long long cnt = 0;
    int lo = 0x7fffffff, hi = -1;
    for (int w = threadIdx.x; w < nw; w += blockDim.x) {
        uint32_t v = 0;
        const int p0 = w * 32;
#pragma unroll 8
        for (int b = 0; b < 32; ++b) {
            const int px = p0 + b;
            if (px < HW && p[px]) v |= 1u << b;
        }
        bits[w] = v;
        if (v) {
            cnt += __popc(v);
            const int first = p0 + __ffs(v) - 1, last = p0 + 31 - __clz(v);
            lo = min(lo, first / W);
            hi = max(hi, last / W);
        }
    }
    red[threadIdx.x] = cnt;
    rmin[threadIdx.x] = lo;
    rmax[threadIdx.x] = hi;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            red[threadIdx.x] += red[threadIdx.x + s];
            rmin[threadIdx.x] = min(rmin[threadIdx.x], rmin[threadIdx.x + s]);
            rmax[threadIdx.x] = max(rmax[threadIdx.x], rmax[threadIdx.x + s]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        ws.area[m] = (int64_t)red[0];
        ws.row0[m] = rmin[0];
        ws.row1[m] = rmax[0];
    }
}

// One workgroup per pair (i < j): popcount of the AND over the words of the rows
// both masks occupy.
__global__ __launch_bounds__(256) void mask_inter_kernel(int n, int W, int nw, MaskWs ws) {
    const int i = blockIdx.x / n, j = blockIdx.x - (blockIdx.x / n) * n;
    if (j <= i) return;
    const int r0 = max(ws.row0[i], ws.row0[j]), r1 = min(ws.row1[i], ws.row1[j]);
    int total = 0;
    if (r0 <= r1) {
        const int w0 = (int)(((int64_t)r0 * W) / 32);
        const int w1 = min(nw - 1, (int)(((int64_t)(r1 + 1) * W - 1) / 32));
        const uint32_t *a = ws.bits + (int64_t)i * nw, *b = ws.bits + (int64_t)j * nw;
        for (int w = w0 + threadIdx.x; w <= w1; w += blockDim.x) total += __popc(a[w] & b[w]);
    }
    __shared__ int red[256];
    red[threadIdx.x] = total;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) ws.inter[(int64_t)i * n + j] = red[0];
}

// One workgroup: the score order, the greedy discard pass, the per-class cap and
// the class-major output order.
__global__ __launch_bounds__(1024) void mask_nms_kernel(int n, const float *__restrict__ dets,
                                                        int stride,
                                                        const int32_t *__restrict__ classes,
                                                        double iou_th, int max_per_class,
                                                        MaskWs ws, int64_t *__restrict__ keep_out,
                                                        int32_t *__restrict__ num_out) {
    __shared__ int order[kMaxMaskNms];   // position -> detection
    __shared__ int disc[kMaxMaskNms];    // by position
    __shared__ int sel[kMaxMaskNms];     // by position: kept and under the class cap
    const int t = threadIdx.x;
    // np.argsort(-scores), read stably: rank = #{k: s_k > s_t or (s_k == s_t, k < t)}
    for (int d = t; d < n; d += blockDim.x) {
        const float s = dets[(int64_t)d * stride + 4];
        int rank = 0;
        for (int k = 0; k < n; ++k) {
            const float sk = dets[(int64_t)k * stride + 4];
            rank += (sk > s) || (sk == s && k < d);
        }
        order[rank] = d;
    }
    for (int q = t; q < n; q += blockDim.x) disc[q] = 0;
    __syncthreads();
    for (int p = 0; p < n; ++p) {
        if (!disc[p]) {  // uniform: read after the barrier
            const int i = order[p];
            const double ai = (double)ws.area[i] + 1e-6;
            for (int q = p + 1 + t; q < n; q += blockDim.x) {
                const int j = order[q];
                const int inter = ws.inter[(int64_t)min(i, j) * n + max(i, j)];
                const double iou1 = (double)inter / ai;
                const double iou2 = (double)inter / ((double)ws.area[j] + 1e-6);
                if (iou1 > iou_th || iou2 > iou_th) disc[q] = 1;
            }
        }
        __syncthreads();
    }
    // the per-class cap in score order over the kept positions
    for (int q = t; q < n; q += blockDim.x) {
        int ok = 0;
        if (!disc[q]) {
            const int c = classes[order[q]];
            int before = 0;
            for (int u = 0; u < q; ++u) before += !disc[u] && classes[order[u]] == c;
            ok = before < max_per_class;
        }
        sel[q] = ok;
    }
    __syncthreads();
    // class-major output: class ascending, then score order
    int nsel = 0;
    for (int q = t; q < n; q += blockDim.x) {
        if (!sel[q]) continue;
        const int c = classes[order[q]];
        int pos = 0;
        for (int u = 0; u < n; ++u) {
            if (!sel[u]) continue;
            const int cu = classes[order[u]];
            pos += cu < c || (cu == c && u < q);
        }
        keep_out[pos] = order[q];
    }
    for (int q = 0; q < n; ++q) nsel += sel[q];
    if (t == 0) *num_out = nsel;
}

// box rows as float32, bb_intersection_over_union's expression order
__device__ __forceinline__ float iou_vos(const float *a, const float *b) {
    const float xA = fmaxf(a[0], b[0]), yA = fmaxf(a[1], b[1]);
    const float xB = fminf(a[2], b[2]), yB = fminf(a[3], b[3]);
    const float iw = fmaxf(0.f, (xB - xA) + 1.f), ih = fmaxf(0.f, (yB - yA) + 1.f);
    const float inter = iw * ih;
    const float aa = ((a[2] - a[0]) + 1.f) * ((a[3] - a[1]) + 1.f);
    const float ab = ((b[2] - b[0]) + 1.f) * ((b[3] - b[1]) + 1.f);
    return inter / ((aa + ab) - inter);
}

// One workgroup per frame: filter the frame's detections against the previous
// frame's result, stable compaction in place.  A class with more than one
// previous box (the reference asserts len(prev_cls_boxes[j]) < 2 for EVERY
// class j, vos_test.py:846-848, whether or not the current frame has one) fails
// the frame with its own code: count VD_COUNT_PREV_BOXES (-2).
__global__ __launch_bounds__(1024) void prev_box_filter_kernel(
    float *__restrict__ dets, int32_t *__restrict__ classes, int32_t *__restrict__ counts,
    int det_cap, const float *__restrict__ prev_dets, const int32_t *__restrict__ prev_classes,
    const int32_t *__restrict__ prev_counts, int prev_cap, float iou_thresh, float score_thresh) {
    const int f = blockIdx.x, t = threadIdx.x;
    // A frame an upstream kernel already failed (negative count) keeps its code:
    // propagate, never hide (vosdet.h).  Every thread reads it before thread 0's
    // only write below, so the whole workgroup leaves together.
    const int c0 = counts[f];
    if (c0 < 0) return;
    const int n = min(c0, det_cap);
    const int np_ = prev_counts[f] > 0 ? min(prev_counts[f], prev_cap) : 0;
    float *d = dets + (int64_t)f * det_cap * 5;
    int32_t *c = classes + (int64_t)f * det_cap;
    const float *pd = prev_dets + (int64_t)f * prev_cap * 5;
    const int32_t *pc = prev_classes + (int64_t)f * prev_cap;
    __shared__ int bad;
    __shared__ int pref[1024];
    if (t == 0) bad = 0;
    __syncthreads();
    float row[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    int cls = 0, keep = 0;
    if (t < n) {
        for (int k = 0; k < 5; ++k) row[k] = d[t * 5 + k];
        cls = c[t];
        int found = -1, nprev = 0;
        for (int k = 0; k < np_; ++k)
            if (pc[k] == cls) {
                ++nprev;
                found = k;
            }
        keep = 1;
        if (nprev == 1 && !(pd[found * 5 + 4] < score_thresh))
            keep = !(iou_vos(pd + found * 5, row) < iou_thresh);
    }
    for (int u = t; u < np_; u += blockDim.x)  // every previous class, present here or not
        for (int k = 0; k < u; ++k)
            if (pc[k] == pc[u]) atomicOr(&bad, 1);
    pref[t] = keep;
    __syncthreads();
    for (int s = 1; s < (int)blockDim.x; s <<= 1) {  // inclusive scan
        const int v = t >= s ? pref[t - s] : 0;
        __syncthreads();
        pref[t] += v;
        __syncthreads();
    }
    if (t < n && keep) {
        const int o = pref[t] - 1;
        for (int k = 0; k < 5; ++k) d[o * 5 + k] = row[k];
        c[o] = cls;
    }
    __syncthreads();
    if (t == 0) counts[f] = bad ? VD_COUNT_PREV_BOXES : (n ? pref[n - 1] : 0);
}

}  // namespace

size_t mask_iou_nms_workspace_bytes(int n, int im_h, int im_w) {
    if (n <= 0) return 0;
    const int nw = (int)(((int64_t)im_h * im_w + 31) / 32);
    size_t total = 0;
    carve_mask_ws(nullptr, n, nw, &total);
    return total;
}

int launch_mask_iou_nms(const uint8_t *planes, int n, int im_h, int im_w, const float *dets,
                        int det_stride, const int32_t *classes, double iou_th, int max_per_class,
                        int64_t *keep_out, int32_t *num_out, void *ws, size_t ws_bytes,
                        hipStream_t s) {
    if (n < 0 || n > kMaxMaskNms || im_h < 1 || im_w < 1 || det_stride < 5) return VD_ERR_SHAPE;
    if (n == 0) {
        hipLaunchKernelGGL(zero_count_kernel, dim3(1), dim3(1), 0, s, num_out);
        return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
    }
    const int64_t HW = (int64_t)im_h * im_w;
    if (HW >= (1ll << 31) - 64) return VD_ERR_SHAPE;
    const int nw = (int)((HW + 31) / 32);
    size_t total = 0;
    const MaskWs w = carve_mask_ws(ws, n, nw, &total);
    if (!ws || ws_bytes < total) return VD_ERR_WORKSPACE;
    hipLaunchKernelGGL(mask_pack_kernel, dim3(n), dim3(256), 0, s, planes, (int)HW, im_w, nw, w);
    hipLaunchKernelGGL(mask_inter_kernel, dim3((unsigned)n * n), dim3(256), 0, s, n, im_w, nw, w);
    hipLaunchKernelGGL(mask_nms_kernel, dim3(1), dim3(1024), 0, s, n, dets, det_stride, classes,
                       iou_th, max_per_class, w, keep_out, num_out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int launch_prev_box_filter(float *dets, int32_t *classes, int32_t *counts, int F, int det_cap,
                           const float *prev_dets, const int32_t *prev_classes,
                           const int32_t *prev_counts, int prev_cap, float iou_thresh,
                           float score_thresh, hipStream_t s) {
    if (F <= 0) return VD_OK;
    if (det_cap < 1 || det_cap > 1024 || prev_cap < 0) return VD_ERR_SHAPE;
    const int threads = (det_cap + 63) / 64 * 64;
    hipLaunchKernelGGL(prev_box_filter_kernel, dim3(F), dim3(threads), 0, s, dets, classes, counts,
                       det_cap, prev_dets, prev_classes, prev_counts, prev_cap, iou_thresh,
                       score_thresh);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
