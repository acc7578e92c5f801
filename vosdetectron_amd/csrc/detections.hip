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
//   Options of lib/core/test.py:756-776 in the same workgroup: TEST.SOFT_NMS
//   (cython_nms.soft_nms, one wave, instead of the NMS) and TEST.BBOX_VOTE
//   (utils/boxes.py box_voting, one thread per kept box) -- DetOpts.
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

// TEST.SOFT_NMS / TEST.BBOX_VOTE (lib/core/test.py:756-776).
struct DetOpts {
    int soft_method;  // -1: cython NMS; 0 hard, 1 linear, 2 gaussian (cython_nms.soft_nms)
    float soft_sigma, soft_min;  // sigma, score_thresh (0.0001 at test.py:760)
    int vote_method;  // -1 off; 0 ID, 1 AVG, 2 IOU_AVG, 3 QUASI_SUM (boxes.py:277-333)
    float vote_th, vote_beta;
};

// The compiled .pyx arithmetic (cython_nms.soft_nms :166-171, cython_bbox.bbox_overlaps):
// Cython emits the literal 1 of `x2 - x1 + 1` as 1.0, so each side is the float
// difference widened to double, products / sums in double, rounded to float on
// assignment; iw * ih is a float product; ov a float division.
__device__ __forceinline__ float cy_area(float x1, float y1, float x2, float y2) {
    return (float)(((double)(x2 - x1) + 1.0) * ((double)(y2 - y1) + 1.0));
}

// IoU of a kept / top box a with box b (area_b = cy_area(b)); false when they
// do not overlap (iw or ih <= 0: soft_nms leaves the box, bbox_overlaps 0).
__device__ __forceinline__ bool cy_iou(float ax1, float ay1, float ax2, float ay2, float bx1,
                                       float by1, float bx2, float by2, float area_b,
                                       float &ov) {
    const float iw = (float)((double)(fminf(ax2, bx2) - fmaxf(ax1, bx1)) + 1.0);
    if (!(iw > 0.f)) return false;
    const float ih = (float)((double)(fminf(ay2, by2) - fmaxf(ay1, by1)) + 1.0);
    if (!(ih > 0.f)) return false;
    const float inter = iw * ih;
    const float ua = (float)(((double)(ax2 - ax1) + 1.0) * ((double)(ay2 - ay1) + 1.0) +
                             (double)area_b - (double)inter);
    ov = inter / ua;
    return true;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// cython_nms.soft_nms (cython_nms.pyx:98-203) by one wave over the m boxes in
// (x1, y1, x2, y2, s), rearranged in place as the reference rearranges its copy:
// step i swaps the first maximum of s[i, N) to i; every later box that overlaps
// it is decayed (each box is decayed once per step wherever the sequential loop
// would meet it, so the decays run in parallel); a decayed score below soft_min
// removes the box by moving the current last box into its place and looking at
// that one again (the holes are filled in ascending order by the wave's lane 0).
// rem: LDS byte per position; ind (optional) follows the rows (the keep indices).
// Returns N, the boxes kept in [0, N).
__device__ int soft_nms_wave(float *x1, float *y1, float *x2, float *y2, float *s, uint8_t *rem,
                             int *ind, int m, float Nt, const DetOpts &o) {
    const int lane = lane_id();
    int N = m;
    for (int i = 0; i < N; ++i) {
        float best = -INFINITY;
        int bp = 0x7fffffff;
        for (int p = i + lane; p < N; p += VD_WAVE) {
            const float v = s[p];
            if (v > best) {
                best = v;
                bp = p;
            }
        }
        for (int off = VD_WAVE / 2; off > 0; off >>= 1) {
            const float ob = __shfl_xor(best, off);
            const int op = __shfl_xor(bp, off);
            if (ob > best || (ob == best && op < bp)) {
                best = ob;
                bp = op;
            }
        }
        if (bp != i && lane == 0) {
            float t;
            t = x1[i]; x1[i] = x1[bp]; x1[bp] = t;
            t = y1[i]; y1[i] = y1[bp]; y1[bp] = t;
            t = x2[i]; x2[i] = x2[bp]; x2[bp] = t;
            t = y2[i]; y2[i] = y2[bp]; y2[bp] = t;
            t = s[i]; s[i] = s[bp]; s[bp] = t;
            if (ind) {
                const int k = ind[i];
                ind[i] = ind[bp];
                ind[bp] = k;
            }
        }
        wave_sync();
        const float tx1 = x1[i], ty1 = y1[i], tx2 = x2[i], ty2 = y2[i];
        for (int p = i + 1 + lane; p < N; p += VD_WAVE) {
            const float bx1 = x1[p], by1 = y1[p], bx2 = x2[p], by2 = y2[p];
            float ov;
            uint8_t r = 0;
            if (cy_iou(tx1, ty1, tx2, ty2, bx1, by1, bx2, by2, cy_area(bx1, by1, bx2, by2), ov)) {
                float w;
                if (o.soft_method == 1)
                    w = ov > Nt ? 1.f - ov : 1.f;
                else if (o.soft_method == 2)
                    w = (float)exp((double)((-(ov * ov)) / o.soft_sigma));
                else
                    w = ov > Nt ? 0.f : 1.f;
                const float ns = w * s[p];
                s[p] = ns;
                r = ns < o.soft_min;
            }
            rem[p] = r;
        }
        wave_sync();
        for (int base = i + 1; base < N; base += VD_WAVE) {
            const int p = base + lane;
            uint64_t mask = ballot(p < N && rem[p]);
            while (mask) {
                const int q = base + __ffsll((unsigned long long)mask) - 1;
                mask &= mask - 1;
                if (q >= N) break;
                for (;;) {  // boxes[q] = boxes[N-1]; N -= 1; look at q again
                    const int last = N - 1;
                    if (lane == 0 && last != q) {
                        x1[q] = x1[last];
                        y1[q] = y1[last];
                        x2[q] = x2[last];
                        y2[q] = y2[last];
                        s[q] = s[last];
                        rem[q] = rem[last];
                        if (ind) ind[q] = ind[last];
                    }
                    N = last;
                    wave_sync();
                    if (q >= N || !rem[q]) break;
                }
            }
        }
    }
    return N;
}

// box_voting's sums for one top box, in numpy's order: the voters (rows of the
// class's candidates with bbox_overlaps >= vote_th, ascending) stream by; the
// weighted box sums run sequentially down the rows (a (n,4) axis-0 reduction),
// the 1-D sums (weights, weight * overlap, overlap) in numpy's pairwise order.
struct VoteAcc {
    float w, wo, o;
};

__device__ __forceinline__ VoteAcc va_add(VoteAcc a, VoteAcc b) {
    return {a.w + b.w, a.wo + b.wo, a.o + b.o};
}

struct VoteStream {
    const float *x1, *y1, *x2, *y2, *s;
    int cur;
    float tx1, ty1, tx2, ty2, th;
    float c0, c1, c2, c3;
    __device__ float overlap(int i) const {
        float ov;
        return cy_iou(tx1, ty1, tx2, ty2, x1[i], y1[i], x2[i], y2[i],
                      cy_area(x1[i], y1[i], x2[i], y2[i]), ov) ? ov : 0.f;
    }
    __device__ VoteAcc next() {  // the caller asks for exactly the counted voters
        for (;; ++cur) {
            const float ov = overlap(cur);
            if (ov >= th) {
                const int i = cur++;
                const float w = s[i];
                c0 = c0 + x1[i] * w;
                c1 = c1 + y1[i] * w;
                c2 = c2 + x2[i] * w;
                c3 = c3 + y2[i] * w;
                return {w, w * ov, ov};
            }
        }
    }
};

// numpy pairwise_sum (loops_utils.h): < 8 sequential from 0; <= 128 eight strided
// accumulators ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the tail; else halves at
// a multiple of 8.  D bounds the recursion (n <= 128 << D).
template <int D>
__device__ VoteAcc pw_sum(VoteStream &st, int n) {
    if (n < 8) {
        VoteAcc r = {0.f, 0.f, 0.f};
        for (int i = 0; i < n; ++i) r = va_add(r, st.next());
        return r;
    }
    if constexpr (D > 0) {
        if (n > 128) {
            int n2 = n / 2;
            n2 -= n2 % 8;
            const VoteAcc a = pw_sum<D - 1>(st, n2);
            const VoteAcc b = pw_sum<D - 1>(st, n - n2);
            return va_add(a, b);
        }
    }
    VoteAcc r[8];
    for (int k = 0; k < 8; ++k) r[k] = st.next();
    int i = 8;
    for (; i < n - n % 8; i += 8)
        for (int k = 0; k < 8; ++k) r[k] = va_add(r[k], st.next());
    VoteAcc res = va_add(va_add(va_add(r[0], r[1]), va_add(r[2], r[3])),
                         va_add(va_add(r[4], r[5]), va_add(r[6], r[7])));
    for (; i < n; ++i) res = va_add(res, st.next());
    return res;
}

// box_voting (boxes.py:277-333) of one top row against the m candidates.
__device__ void vote_box(const float *x1, const float *y1, const float *x2, const float *y2,
                         const float *s, int m, const DetOpts &o, float *row) {
    VoteStream st{x1, y1, x2, y2, s, 0, row[0], row[1], row[2], row[3], o.vote_th,
                  0.f, 0.f, 0.f, 0.f};
    int n = 0;
    for (int i = 0; i < m; ++i) n += st.overlap(i) >= o.vote_th;
    if (n == 0) return;  // numpy raises (weights sum to zero); never for a top row itself
    const VoteAcc sum = pw_sum<5>(st, n);
    const float scl = 0.f + sum.w;
    row[0] = st.c0 / scl;
    row[1] = st.c1 / scl;
    row[2] = st.c2 / scl;
    row[3] = st.c3 / scl;
    if (o.vote_method == 1)
        row[4] = scl / (float)n;
    else if (o.vote_method == 2)
        row[4] = (0.f + sum.wo) / (0.f + sum.o);
    else if (o.vote_method == 3)
        row[4] = scl / (float)pow((double)n, (double)o.vote_beta);
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
    float nms_thresh, float4 bbox_w, DetOpts opt, DetWs ws) {
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
    const size_t slot = (size_t)img * K + j;
    float *dst = ws.cls_dets + slot * (size_t)R_cap * 5;
    __syncthreads();
    int kept;
    if (opt.soft_method >= 0) {
        // soft-NMS on a copy (the candidates stay box_voting's all_dets)
        for (int t = threadIdx.x; t < m; t += blockDim.x) {
            L.ox1[t] = L.cx1[t];
            L.oy1[t] = L.cy1[t];
            L.ox2[t] = L.cx2[t];
            L.oy2[t] = L.cy2[t];
            L.oar[t] = L.csc[t];
        }
        __syncthreads();
        if (wave_id() == 0) {
            const int n = soft_nms_wave(L.ox1, L.oy1, L.ox2, L.oy2, L.oar, L.keep_rank, nullptr,
                                        m, nms_thresh, opt);
            if (lane_id() == 0) L.scratch[16] = n;
        }
        __syncthreads();
        kept = L.scratch[16];
    } else {
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
        if (opt.vote_method < 0) {  // survivors ascending straight to the class slot
            kept = block_compact(
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
            return;
        }
        kept = block_compact(  // the top rows for box voting
            m, [&](int t) { return L.keep_t[t] != 0; },
            [&](int u, int t) {
                L.ox1[u] = L.cx1[t];
                L.oy1[u] = L.cy1[t];
                L.ox2[u] = L.cx2[t];
                L.oy2[u] = L.cy2[t];
                L.oar[u] = L.csc[t];
            },
            L.scratch);
    }
    for (int u = threadIdx.x; u < kept; u += blockDim.x) {
        float row[5] = {L.ox1[u], L.oy1[u], L.ox2[u], L.oy2[u], L.oar[u]};
        if (opt.vote_method >= 0) vote_box(L.cx1, L.cy1, L.cx2, L.cy2, L.csc, m, opt, row);
        for (int c = 0; c < 5; ++c) dst[u * 5 + c] = row[c];
    }
    if (threadIdx.x == 0) ws.cls_count[slot] = kept;
}

static constexpr int kLimStage = 16384;  // scores staged in LDS by det_limit_kernel

__global__ __launch_bounds__(1024) void det_limit_kernel(const int32_t *__restrict__ roi_count,
                                                          int R_cap, int K, int dets_per_im,
                                                          int det_cap, DetWs ws,
                                                          float *__restrict__ dets_out,
                                                          int32_t *__restrict__ det_cls_out,
                                                          int32_t *__restrict__ det_count_out) {
    __shared__ int offs[1025];
    __shared__ uint32_t hist[256];
    __shared__ int scratch[32];
    __shared__ float stage[kLimStage];
    const int img = blockIdx.x;
    if (roi_count[img] < 0) {  // proposal selection failed upstream: propagate, never hide
        if (threadIdx.x == 0) det_count_out[img] = -1;
        return;
    }
    // prefix over classes 1..K-1 (K <= 1024): the counts loaded by K threads at
    // once (a serial loop waited out one global-load latency per class), then one
    // thread sums them in LDS
    for (int j = threadIdx.x; j < K; j += blockDim.x)
        offs[j] = j ? ws.cls_count[(size_t)img * K + j] : 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        int o = 0;
        for (int j = 1; j < K; ++j) {
            o += offs[j];
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
    // the radix select reads every score four times and the compaction once:
    // staged in LDS (one parallel gather) when they fit, else read in place
    const bool staged = total <= kLimStage;
    if (staged) {
        for (int q = threadIdx.x; q < total; q += blockDim.x) {
            int jj, u;
            at(q, jj, u);
            stage[q] = ws.cls_dets[(((size_t)img * K + jj) * R_cap + u) * 5 + 4];
        }
        __syncthreads();
    }
    auto score = [&](int q) -> float {
        if (staged) return stage[q];
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
                          int soft_method, float soft_sigma, float soft_min, int vote_method,
                          float vote_th, float vote_beta, int det_cap, float *dets_out,
                          int32_t *det_cls_out, int32_t *det_count_out, void *workspace,
                          size_t ws_bytes, hipStream_t s) {
    if (K < 2 || K > 1024 || num_images < 1 || R_cap < 1 || det_cap < 1) return VD_ERR_ARG;
    if (R_cap > kDetRMax) return VD_ERR_SHAPE;
    if (soft_method < -1 || soft_method > 2 || vote_method < -1 || vote_method > 3)
        return VD_ERR_ARG;
    if (!workspace || ws_bytes < box_detections_workspace_bytes(R_cap, num_images, K))
        return VD_ERR_WORKSPACE;
    DetWs ws = det_ws(workspace, R_cap, num_images, K);
    const float4 bw = make_float4(bbox_weights[0], bbox_weights[1], bbox_weights[2], bbox_weights[3]);
    const int cap = next_pow2(R_cap < 64 ? 64 : R_cap);
    hipLaunchKernelGGL(class_nms_kernel, dim3(K - 1, num_images), dim3(1024), cls_lds_bytes(cap), s,
                       rois, cls_prob, bbox_pred, roi_count, R_cap, K, im_scale, im_hw,
                       score_thresh, nms_thresh, bw,
                       DetOpts{soft_method, soft_sigma, soft_min, vote_method, vote_th, vote_beta},
                       ws);
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

// --------------------------------------------------------------------------
// Standalone utils.boxes.soft_nms / box_voting (vd_soft_nms, vd_box_voting).
// --------------------------------------------------------------------------
static constexpr int kSoftMax = 4096;

__global__ __launch_bounds__(64) void soft_nms_kernel(const float *__restrict__ dets, int n,
                                                      int stride, float Nt, DetOpts opt,
                                                      float *__restrict__ out,
                                                      int64_t *__restrict__ keep,
                                                      int32_t *__restrict__ count) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    float *x1 = reinterpret_cast<float *>(lds_raw);
    float *y1 = x1 + n, *x2 = y1 + n, *y2 = x2 + n, *s = y2 + n;
    int *ind = reinterpret_cast<int *>(s + n);
    uint8_t *rem = reinterpret_cast<uint8_t *>(ind + n);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float *d = dets + (size_t)i * stride;
        x1[i] = d[0];
        y1[i] = d[1];
        x2[i] = d[2];
        y2[i] = d[3];
        s[i] = d[4];
        ind[i] = i;
    }
    wave_sync();
    const int N = soft_nms_wave(x1, y1, x2, y2, s, rem, ind, n, Nt, opt);
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        out[i * 5 + 0] = x1[i];
        out[i * 5 + 1] = y1[i];
        out[i * 5 + 2] = x2[i];
        out[i * 5 + 3] = y2[i];
        out[i * 5 + 4] = s[i];
        keep[i] = ind[i];
    }
    if (threadIdx.x == 0) *count = N;
}

int launch_soft_nms(const float *dets, int n, int stride, float sigma, float overlap_thresh,
                    float score_thresh, int method, float *dets_out, int64_t *keep_out,
                    int32_t *count_out, hipStream_t s) {
    if (n < 0 || stride < 5 || method < 0 || method > 2) return VD_ERR_ARG;
    if (n > kSoftMax) return VD_ERR_SHAPE;
    const size_t lds = (size_t)n * (5 * 4 + 4 + 1) + 16;
    hipLaunchKernelGGL(soft_nms_kernel, dim3(1), dim3(64), lds, s, dets, n, stride,
                       overlap_thresh, DetOpts{method, sigma, score_thresh, -1, 0.f, 1.f},
                       dets_out, keep_out, count_out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

__global__ __launch_bounds__(256) void box_voting_kernel(const float *__restrict__ top, int n_top,
                                                         int top_stride,
                                                         const float *__restrict__ all,
                                                         int n_all, int all_stride,
                                                         DetOpts opt, float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    float *x1 = reinterpret_cast<float *>(lds_raw);
    float *y1 = x1 + n_all, *x2 = y1 + n_all, *y2 = x2 + n_all, *s = y2 + n_all;
    for (int i = threadIdx.x; i < n_all; i += blockDim.x) {
        const float *d = all + (size_t)i * all_stride;
        x1[i] = d[0];
        y1[i] = d[1];
        x2[i] = d[2];
        y2[i] = d[3];
        s[i] = d[4];
    }
    __syncthreads();
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_top) return;
    float row[5];
    for (int c = 0; c < 5; ++c) row[c] = top[(size_t)k * top_stride + c];
    vote_box(x1, y1, x2, y2, s, n_all, opt, row);
    for (int c = 0; c < 5; ++c) out[(size_t)k * 5 + c] = row[c];
}

int launch_box_voting(const float *top, int n_top, int top_stride, const float *all, int n_all,
                      int all_stride, float thresh, int method, float beta, float *out,
                      hipStream_t s) {
    if (n_top < 0 || n_all < 0 || top_stride < 5 || all_stride < 5 || method < 0 || method > 3)
        return VD_ERR_ARG;
    if (n_all > kSoftMax) return VD_ERR_SHAPE;
    if (n_top == 0) return VD_OK;
    const size_t lds = (size_t)n_all * 5 * 4 + 16;
    hipLaunchKernelGGL(box_voting_kernel, dim3((n_top + 255) / 256), dim3(256), lds, s, top,
                       n_top, top_stride, all, n_all, all_stride,
                       DetOpts{-1, 0.5f, 0.f, method, thresh, beta}, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
