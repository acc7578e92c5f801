// Box-head post-processing on device.
//
// Reference (host numpy per frame):
//   im_detect_bbox decode + clip           lib/core/test.py:157-184
//     bbox_transform(boxes=rois/im_scale, deltas, BBOX_REG_WEIGHTS)  boxes.py:156-205
//     clip_tiled_boxes(pred_boxes, im.shape)                          boxes.py:138-153
//   box_results_with_nms_and_limit          lib/core/test.py:733-797
//     (fork fix of the NUM_DET_PER_CLASS crash: lib_vos/tools/vos_test.py:748-865)
//
// Kernel 1: one workgroup per (class j >= 1, image): ordered compaction of the
//   proposals with score >= thresh, decode of the class-j box, NMS (cython
//   semantics), survivors ascending -> per-class slots in the workspace.
// Kernel 2: one workgroup per image: the dets_per_im-th largest score over all
//   classes (radix select), keep score >= it, emit in class-major order.
// Kernel 3 (optional, vd_detections_postfilter): the fork's steps after the
//   limit (lib_vos/tools/vos_test.py:805-833): TEST.NMS_CROSS_CLASS (one NMS
//   over every class's detections, survivors regrouped by class) and
//   TEST.NUM_DET_PER_CLASS_PRE (per class, the top-k by score, rows reordered
//   by score -- np.argsort(-s) read stably: ties by row order).
#include "nms_block.hpp"
#include "vosdet_internal.hpp"

namespace vd {

static constexpr int kDetRMax = 2048;
static constexpr double kClip = 4.135166556742356;  // np.log(1000. / 16.)

__host__ __device__ inline size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

struct DetWs {
    float *cls_dets;     // [img][K][R_cap][5]
    int32_t *cls_count;  // [img][K]
    uint64_t *mask;      // [img][K][R_cap*words]
};

__host__ __device__ inline DetWs det_ws(void *base, int R_cap, int num_images, int K) {
    DetWs w;
    char *p = (char *)base;
    const size_t nd = (size_t)num_images * K * R_cap * 5 * sizeof(float);
    w.cls_dets = (float *)p;
    p += al256(nd);
    w.cls_count = (int32_t *)p;
    p += al256((size_t)num_images * K * sizeof(int32_t));
    w.mask = (uint64_t *)p;
    return w;
}

size_t box_detections_workspace_bytes(int R_cap, int num_images, int K) {
    const size_t words = (size_t)(R_cap + 63) / 64;
    return al256((size_t)num_images * K * R_cap * 5 * sizeof(float)) +
           al256((size_t)num_images * K * sizeof(int32_t)) +
           al256((size_t)num_images * K * R_cap * words * sizeof(uint64_t));
}

__device__ __forceinline__ void decode_box_w(float bx1, float by1, float bx2, float by2,
                                             const float *d, const float *wts, float &x1,
                                             float &y1, float &x2, float &y2) {
    const float widths = bx2 - bx1 + 1.0f;
    const float heights = by2 - by1 + 1.0f;
    const float ctr_x = bx1 + 0.5f * widths;
    const float ctr_y = by1 + 0.5f * heights;
    const float dx = d[0] / wts[0], dy = d[1] / wts[1];
    const double dw = fmin((double)(d[2] / wts[2]), kClip);
    const double dh = fmin((double)(d[3] / wts[3]), kClip);
    const float pcx = dx * widths + ctr_x;
    const float pcy = dy * heights + ctr_y;
    const double pw = fmax(exp(dw) * (double)widths, 1.0);
    const double ph = fmax(exp(dh) * (double)heights, 1.0);
    x1 = (float)((double)pcx - 0.5 * pw);
    y1 = (float)((double)pcy - 0.5 * ph);
    x2 = (float)((double)pcx + 0.5 * pw - 1.0);
    y2 = (float)((double)pcy + 0.5 * ph - 1.0);
}

// Per-workgroup LDS, sized for cap = next_pow2(R_cap) candidates at launch
// (55 KiB at R_cap = 1000, two workgroups per CU; a fixed kDetRMax layout
// took 110 KiB and serialised the (class, image) workgroups one per CU).
struct ClsLds {
    uint64_t *keys;
    int *cand;
    float *cx1, *cy1, *cx2, *cy2, *csc, *ox1, *oy1, *ox2, *oy2, *oar;
    uint8_t *keep_rank, *keep_t;
    float *wts;
    int *scratch;
};

__host__ __device__ inline size_t cls_lds_bytes(int cap) {
    return (size_t)cap * (8 + 4 + 10 * 4 + 2) + 4 * 4 + 32 * 4;
}

__device__ inline ClsLds cls_lds(char *p, int cap) {
    ClsLds L;
    L.keys = reinterpret_cast<uint64_t *>(p);
    p += (size_t)cap * 8;
    L.cand = reinterpret_cast<int *>(p);
    p += (size_t)cap * 4;
    float **f[10] = {&L.cx1, &L.cy1, &L.cx2, &L.cy2, &L.csc, &L.ox1, &L.oy1, &L.ox2, &L.oy2, &L.oar};
    for (int i = 0; i < 10; ++i) {
        *f[i] = reinterpret_cast<float *>(p);
        p += (size_t)cap * 4;
    }
    L.wts = reinterpret_cast<float *>(p);
    p += 16;
    L.scratch = reinterpret_cast<int *>(p);
    p += 128;
    L.keep_rank = reinterpret_cast<uint8_t *>(p);
    L.keep_t = L.keep_rank + cap;
    return L;
}

__global__ __launch_bounds__(1024) void class_nms_kernel(
    const float *__restrict__ rois, const float *__restrict__ cls_prob,
    const float *__restrict__ bbox_pred, const int32_t *__restrict__ roi_count, int R_cap, int K,
    const float *__restrict__ im_scale, const int32_t *__restrict__ im_hw, float score_thresh,
    float nms_thresh, float4 bbox_w, DetWs ws) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    const ClsLds L = cls_lds(lds_raw, next_pow2(R_cap < 64 ? 64 : R_cap));
    const int j = blockIdx.x + 1, img = blockIdx.y;
    const int R = min(roi_count[img], R_cap);
    if (threadIdx.x == 0) {
        L.wts[0] = bbox_w.x;
        L.wts[1] = bbox_w.y;
        L.wts[2] = bbox_w.z;
        L.wts[3] = bbox_w.w;
    }
    const float *prob = cls_prob + (size_t)img * R_cap * K;
    const float *pred = bbox_pred + (size_t)img * R_cap * 4 * K;
    const float *ri = rois + (size_t)img * R_cap * 5;
    const float scale = im_scale[img];
    const float hm1 = (float)(im_hw[img * 2 + 0] - 1), wm1 = (float)(im_hw[img * 2 + 1] - 1);
    __syncthreads();
    const int m = block_compact(
        R, [&](int r) { return prob[(size_t)r * K + j] >= score_thresh; },
        [&](int t, int r) { L.cand[t] = r; }, L.scratch);
    for (int t = threadIdx.x; t < m; t += blockDim.x) {
        const int r = L.cand[t];
        const float *rb = ri + (size_t)r * 5;
        const float bx1 = rb[1] / scale, by1 = rb[2] / scale;
        const float bx2 = rb[3] / scale, by2 = rb[4] / scale;
        float x1, y1, x2, y2;
        decode_box_w(bx1, by1, bx2, by2, pred + (size_t)r * 4 * K + 4 * j, L.wts, x1, y1, x2, y2);
        L.cx1[t] = fmaxf(fminf(x1, wm1), 0.f);
        L.cy1[t] = fmaxf(fminf(y1, hm1), 0.f);
        L.cx2[t] = fmaxf(fminf(x2, wm1), 0.f);
        L.cy2[t] = fmaxf(fminf(y2, hm1), 0.f);
        const float sc = prob[(size_t)r * K + j];
        L.csc[t] = sc;
    }
    const int np2 = next_pow2(m < 1 ? 1 : m);
    for (int t = threadIdx.x; t < np2; t += blockDim.x)
        L.keys[t] = t < m ? ((uint64_t)float_key(L.csc[t]) << 32) | (uint32_t)t : 0ull;
    __syncthreads();
    if (m > 1) bitonic_sort_desc(L.keys, np2);
    for (int rk = threadIdx.x; rk < m; rk += blockDim.x) {
        const int t = (int)(uint32_t)L.keys[rk];
        const float a = L.cx1[t], b = L.cy1[t], c = L.cx2[t], e = L.cy2[t];
        L.ox1[rk] = a;
        L.oy1[rk] = b;
        L.ox2[rk] = c;
        L.oy2[rk] = e;
        L.oar[rk] = (c - a + 1) * (e - b + 1);
    }
    __syncthreads();
    const size_t slot = (size_t)img * K + j;
    const size_t words = (size_t)(R_cap + 63) / 64;
    uint64_t *mask = ws.mask + slot * (size_t)R_cap * words;
    nms_build_mask_rows(L.ox1, L.oy1, L.ox2, L.oy2, L.oar, m, nms_thresh, mask, wave_id(),
                        num_waves());
    __threadfence_block();
    __syncthreads();
    if (wave_id() == 0) nms_resolve_wave(mask, m, L.keep_rank);
    __syncthreads();
    for (int rk = threadIdx.x; rk < m; rk += blockDim.x)
        L.keep_t[(int)(uint32_t)L.keys[rk]] = L.keep_rank[rk];
    __syncthreads();
    float *dst = ws.cls_dets + slot * (size_t)R_cap * 5;
    const int kept = block_compact(
        m, [&](int t) { return L.keep_t[t] != 0; },
        [&](int u, int t) {
            dst[u * 5 + 0] = L.cx1[t];
            dst[u * 5 + 1] = L.cy1[t];
            dst[u * 5 + 2] = L.cx2[t];
            dst[u * 5 + 3] = L.cy2[t];
            dst[u * 5 + 4] = L.csc[t];
        },
        L.scratch);
    if (threadIdx.x == 0) ws.cls_count[slot] = kept;
}

__global__ __launch_bounds__(1024) void det_limit_kernel(const int32_t *__restrict__ roi_count,
                                                          int R_cap, int K, int dets_per_im,
                                                          int det_cap, DetWs ws,
                                                          float *__restrict__ dets_out,
                                                          int32_t *__restrict__ det_cls_out,
                                                          int32_t *__restrict__ det_count_out) {
    __shared__ int offs[1025];
    __shared__ uint32_t hist[256];
    __shared__ int scratch[32];
    const int img = blockIdx.x;
    if (roi_count[img] < 0) {  // proposal selection failed upstream: propagate, never hide
        if (threadIdx.x == 0) det_count_out[img] = -1;
        return;
    }
    // prefix over classes 1..K-1 (K <= 1024)
    if (threadIdx.x == 0) {
        int o = 0;
        offs[0] = 0;
        for (int j = 1; j < K; ++j) {
            o += ws.cls_count[(size_t)img * K + j];
            offs[j] = o;
        }
    }
    __syncthreads();
    const int total = offs[K - 1];
    auto at = [&](int q, int &jj, int &u) {
        int lo = 1, hi = K - 1;  // first j with offs[j] > q
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (offs[mid] > q) hi = mid; else lo = mid + 1;
        }
        jj = lo;
        u = q - offs[lo - 1];
    };
    auto score = [&](int q) -> float {
        int jj, u;
        at(q, jj, u);
        return ws.cls_dets[(((size_t)img * K + jj) * R_cap + u) * 5 + 4];
    };
    bool limit = dets_per_im > 0 && total > dets_per_im;
    float thr = 0.f;
    if (limit) {
        const uint32_t kk = block_kth_largest(
            total, dets_per_im, [&](int q) { return float_key(score(q)); }, hist, scratch);
        thr = key_float(kk);
    }
    const int n = block_compact(
        total, [&](int q) { return !limit || score(q) >= thr; },
        [&](int d, int q) {
            if (d < det_cap) {
                int jj, u;
                at(q, jj, u);
                const float *src = ws.cls_dets + (((size_t)img * K + jj) * R_cap + u) * 5;
                float *o = dets_out + ((size_t)img * det_cap + d) * 5;
                o[0] = src[0];
                o[1] = src[1];
                o[2] = src[2];
                o[3] = src[3];
                o[4] = src[4];
                det_cls_out[(size_t)img * det_cap + d] = jj;
            }
        },
        scratch);
    if (threadIdx.x == 0) det_count_out[img] = n;
}

int launch_box_detections(const float *rois, const float *cls_prob, const float *bbox_pred,
                          const int32_t *roi_count, int R_cap, int num_images, int K,
                          const float *im_scale, const int32_t *im_hw, float score_thresh,
                          float nms_thresh, int dets_per_im, const float *bbox_weights,
                          int det_cap, float *dets_out, int32_t *det_cls_out,
                          int32_t *det_count_out, void *workspace, size_t ws_bytes,
                          hipStream_t s) {
    if (K < 2 || K > 1024 || num_images < 1 || R_cap < 1 || det_cap < 1) return VD_ERR_ARG;
    if (R_cap > kDetRMax) return VD_ERR_SHAPE;
    if (!workspace || ws_bytes < box_detections_workspace_bytes(R_cap, num_images, K))
        return VD_ERR_WORKSPACE;
    DetWs ws = det_ws(workspace, R_cap, num_images, K);
    const float4 bw = make_float4(bbox_weights[0], bbox_weights[1], bbox_weights[2], bbox_weights[3]);
    const int cap = next_pow2(R_cap < 64 ? 64 : R_cap);
    hipLaunchKernelGGL(class_nms_kernel, dim3(K - 1, num_images), dim3(1024), cls_lds_bytes(cap), s,
                       rois, cls_prob, bbox_pred, roi_count, R_cap, K, im_scale, im_hw,
                       score_thresh, nms_thresh, bw, ws);
    hipLaunchKernelGGL(det_limit_kernel, dim3(num_images), dim3(1024), 0, s, roi_count, R_cap, K,
                       dets_per_im, det_cap, ws, dets_out, det_cls_out, det_count_out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// --------------------------------------------------------------------------
// Kernel 3: in-place post-filter of one image's detections (class-major rows).
// --------------------------------------------------------------------------
static constexpr int kPostMax = 512;

struct PostLds {
    float x1[kPostMax], y1[kPostMax], x2[kPostMax], y2[kPostMax], sc[kPostMax];
    float ox1[kPostMax], oy1[kPostMax], ox2[kPostMax], oy2[kPostMax], oar[kPostMax];
    int cl[kPostMax], rank[kPostMax], pos[kPostMax];
    uint64_t keys[kPostMax];
    uint64_t mask[kPostMax * (kPostMax / 64)];
    uint8_t keep_rank[kPostMax], alive[kPostMax];
    int scratch[32];
};

__global__ __launch_bounds__(512) void det_postfilter_kernel(float *__restrict__ dets,
                                                              int32_t *__restrict__ cls,
                                                              int32_t *__restrict__ counts,
                                                              int det_cap, float cross_thresh,
                                                              int per_class_pre) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    PostLds &L = *reinterpret_cast<PostLds *>(lds_raw);
    const int img = blockIdx.x, t = threadIdx.x;
    if (counts[img] < 0) return;  // upstream failure stays visible (-1)
    const int k = min((int)counts[img], det_cap);  // det_cap <= kPostMax (launcher)
    float *d = dets + (size_t)img * det_cap * 5;
    int32_t *c = cls + (size_t)img * det_cap;
    for (int i = t; i < k; i += blockDim.x) {
        L.x1[i] = d[i * 5 + 0];
        L.y1[i] = d[i * 5 + 1];
        L.x2[i] = d[i * 5 + 2];
        L.y2[i] = d[i * 5 + 3];
        L.sc[i] = d[i * 5 + 4];
        L.cl[i] = c[i];
        L.alive[i] = 1;
    }
    __syncthreads();
    if (cross_thresh > 0.f && k > 1) {
        // utils.boxes.nms(all_dets, NMS_CROSS_CLASS): processing order (score
        // desc, higher row first), cython_nms semantics
        const int np2 = next_pow2(k);
        for (int i = t; i < np2; i += blockDim.x)
            L.keys[i] = i < k ? ((uint64_t)float_key(L.sc[i]) << 32) | (uint32_t)i : 0ull;
        __syncthreads();
        bitonic_sort_desc(L.keys, np2);
        for (int r = t; r < k; r += blockDim.x) {
            const int i = (int)(uint32_t)L.keys[r];
            L.ox1[r] = L.x1[i];
            L.oy1[r] = L.y1[i];
            L.ox2[r] = L.x2[i];
            L.oy2[r] = L.y2[i];
            L.oar[r] = (L.x2[i] - L.x1[i] + 1) * (L.y2[i] - L.y1[i] + 1);
        }
        __syncthreads();
        nms_build_mask_rows(L.ox1, L.oy1, L.ox2, L.oy2, L.oar, k, cross_thresh, L.mask,
                            wave_id(), num_waves());
        __syncthreads();
        if (wave_id() == 0) nms_resolve_wave(L.mask, k, L.keep_rank);
        __syncthreads();
        for (int r = t; r < k; r += blockDim.x) L.alive[(int)(uint32_t)L.keys[r]] = L.keep_rank[r];
        __syncthreads();
    }
    // rank within the class: by (score desc, row asc) with the per-class top-k,
    // else by row (the order is unchanged)
    for (int i = t; i < k; i += blockDim.x) {
        int rk = 0;
        if (L.alive[i]) {
            for (int j = 0; j < k; ++j) {
                if (!L.alive[j] || L.cl[j] != L.cl[i]) continue;
                if (per_class_pre > 0)
                    rk += (L.sc[j] > L.sc[i]) || (L.sc[j] == L.sc[i] && j < i);
                else
                    rk += j < i;
            }
        }
        L.rank[i] = rk;
    }
    __syncthreads();
    if (per_class_pre > 0)
        for (int i = t; i < k; i += blockDim.x)
            if (L.rank[i] >= per_class_pre) L.alive[i] = 0;
    __syncthreads();
    for (int i = t; i < k; i += blockDim.x) {
        int p = -1;
        if (L.alive[i]) {
            p = 0;
            for (int j = 0; j < k; ++j)
                p += L.alive[j] && (L.cl[j] < L.cl[i] || (L.cl[j] == L.cl[i] && L.rank[j] < L.rank[i]));
        }
        L.pos[i] = p;
    }
    __syncthreads();
    int n = 0;
    for (int i = t; i < k; i += blockDim.x) n += L.alive[i];
    n = block_sum(n, L.scratch);
    for (int i = t; i < k; i += blockDim.x) {
        const int p = L.pos[i];
        if (p < 0) continue;
        d[p * 5 + 0] = L.x1[i];
        d[p * 5 + 1] = L.y1[i];
        d[p * 5 + 2] = L.x2[i];
        d[p * 5 + 3] = L.y2[i];
        d[p * 5 + 4] = L.sc[i];
        c[p] = L.cl[i];
    }
    if (t == 0) counts[img] = n;
}

int launch_detections_postfilter(float *dets, int32_t *cls, int32_t *counts, int num_images,
                                 int det_cap, float nms_cross_class, int num_det_per_class_pre,
                                 hipStream_t s) {
    if (num_images < 1 || det_cap < 1) return VD_ERR_ARG;
    if (det_cap > kPostMax) return VD_ERR_SHAPE;
    if (!(nms_cross_class > 0.f) && num_det_per_class_pre <= 0) return VD_OK;
    hipLaunchKernelGGL(det_postfilter_kernel, dim3(num_images), dim3(512), sizeof(PostLds), s,
                       dets, cls, counts, det_cap, nms_cross_class, num_det_per_class_pre);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
