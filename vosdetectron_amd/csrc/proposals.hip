// RPN proposal generation + FPN collect/distribute, device resident.
//
// Reference (per image, per FPN level, host numpy in the reference):
//   GenerateProposalsOp.forward / proposals_for_one_image
//     lib/modeling/generate_proposals.py:20-168
//   bbox_transform lib/utils/boxes.py:156-205, clip_tiled_boxes :138-153,
//   _filter_boxes generate_proposals.py:171-182, nms -> cython_nms.pyx:37-87
//   collect / distribute lib/modeling/collect_and_distribute_fpn_rpn_proposals.py:91-138
//   map_rois_to_fpn_levels lib/utils/fpn.py:11-28
//
// select  -- top pre_nms_topN of the H*W*A scores by the unique 64-bit key
//            (score, ~index).  Multi-workgroup radix select (round 5): every
//            (level, image) score map is split into 4096-score chunks, one
//            256-thread workgroup each (~2200 workgroups for 32 frames);
//            rpn_sel_hist_kernel passes build 11-bit digit histograms of the
//            keys still inside the boundary prefix, until the keys above the
//            boundary bin fit the candidate capacity; rpn_sel_compact_kernel
//            writes them to a per-slot candidate list.  Then one workgroup
//            (1024 threads) per (level, image) does the rest of the chain in
//            LDS: candidates bitonic-sorted, first pre taken.  Equals numpy's
//            argpartition+argsort top-k with ties broken by lower index (the
//            stable reading).  VOSDET_RPN_PRESEL=0 keeps round 4's single-
//            workgroup select (a strided sample fixes a threshold whose
//            candidate set is exact-superset-checked by count passes).
//   decode  -- anchors + shifts (float64, as numpy) -> float32 boxes; the
//              delta decode reproduces numpy 2's float64 promotion of dw/dh by
//              the float64 BBOX_XFORM_CLIP; clip; min-size/centre filter.
//   nms     -- processing order (score desc, position desc), ballot bitmask,
//              single-wave resolve; survivors ascending, first post_nms_topN.
#include <stdlib.h>

#include "nms_block.hpp"
#include "vosdet_internal.hpp"

namespace vd {

static constexpr int kSelCap = 8192;      // candidate keys held in LDS
static constexpr int kPreMax = 2048;      // pre_nms_topN per level
static constexpr int kSampleMax = 2048;
// Large variant (single-scale C4 RPN: 15 anchors, TEST.RPN_PRE_NMS_TOP_N 6000,
// e2e_mask_rcnn_R-50-C4_1x.yaml): 128 KiB of candidate keys in LDS, the
// per-candidate box arrays in the global workspace.
static constexpr int kSelCapL = 16384;
static constexpr int kPreMaxL = 8192;
static_assert(sizeof(uint64_t) * kSelCapL + 2 * kPreMaxL + 128 <= VD_LDS_BYTES, "LDS");
static constexpr double kBboxXformClip = 4.135166556742356;  // np.log(1000. / 16.)

struct RpnArgs {
    VdRpnLevel lv[VD_MAX_LEVELS];
};

__host__ __device__ inline size_t a256(size_t b) { return (b + 255) & ~(size_t)255; }
static inline size_t rpn_mask_bytes(int pre) {
    return a256(sizeof(uint64_t) * (size_t)pre * (size_t)((pre + 63) / 64));
}

static inline size_t rpn_box_bytes(int pre) { return a256(sizeof(float) * 10 * (size_t)pre); }
// large variant: NMS processing-order keys + the candidate count m, handed from the
// select/decode kernel to the mask-build and resolve kernels
static inline size_t rpn_key_bytes(int pre) { return a256(sizeof(uint64_t) * (size_t)pre) + 256; }

// pre_nms_topN actually used per level and whether the large variant is needed
static bool rpn_plan(const VdRpnLevel *levels, int num_levels, int pre_nms_topN, int *max_pre,
                     bool *large) {
    *max_pre = 0;
    *large = false;
    for (int l = 0; l < num_levels; ++l) {
        const int n_all = levels[l].A * levels[l].H * levels[l].W;
        const bool take_all = pre_nms_topN <= 0 || pre_nms_topN >= n_all;
        const int pre = take_all ? n_all : pre_nms_topN;
        if (pre > kPreMax || (take_all && n_all > kSelCap)) *large = true;
        if (pre > kPreMaxL || (take_all && n_all > kSelCapL)) return false;
        *max_pre = pre > *max_pre ? pre : *max_pre;
    }
    return true;
}

// Split NMS (the mask built by many workgroups, resolved by a third kernel):
// always for the large variant; for the small one unless VOSDET_RPN_SPLIT=0.
static bool rpn_split(bool large) {
    if (large) return true;
    const char *e = getenv("VOSDET_RPN_SPLIT");
    return !(e && e[0] == '0');
}

static inline size_t rpn_slot_bytes(int max_pre, bool large) {
    const int p = max_pre < 64 ? 64 : max_pre;
    return large ? rpn_mask_bytes(p) + rpn_box_bytes(p) + rpn_key_bytes(p) : rpn_mask_bytes(p);
}

size_t sel_slot_bytes(int cap);

// Multi-workgroup select (default; VOSDET_RPN_PRESEL=0: round 4's one-workgroup
// sample-and-count select) and its candidate capacity per slot: twice the
// power of two above pre (the boundary bin then usually closes after two
// passes), at most the kernel's LDS key capacity.
static bool rpn_presel() {
    const char *e = getenv("VOSDET_RPN_PRESEL");
    return !(e && e[0] == '0');
}
// Mask build of the split NMS: the one-wave-per-row kernel (default) or the
// LDS-staged row-block kernel (VOSDET_RPN_MASK_LDS=1), which measured slower:
// 174 vs 132 us for P2-P6 x 32 images (profiles/r05/proposals_breakdown.txt) --
// the build is VALU-bound on the IoU tests, and the LDS form's 4 waves per 64-row
// block leave the long first blocks on few SIMDs
static bool rpn_mask_lds() {
    const char *e = getenv("VOSDET_RPN_MASK_LDS");
    return e && e[0] == '1';
}
static int rpn_sel_cap(int max_pre, bool large) {
    const int sel_cap = large ? kSelCapL : kSelCap;
    const int c = 2 * next_pow2(max_pre < 64 ? 64 : max_pre);
    return c < sel_cap ? c : sel_cap;
}

size_t rpn_workspace_bytes(const VdRpnLevel *levels, int num_levels, int num_images,
                           int pre_nms_topN) {
    int max_pre;
    bool large;
    if (num_levels < 1 || !rpn_plan(levels, num_levels, pre_nms_topN, &max_pre, &large))
        return 256;
    const size_t slots = (size_t)num_levels * (size_t)num_images;
    size_t b = rpn_slot_bytes(max_pre, rpn_split(large)) * slots + 256;
    if (rpn_presel()) b += sel_slot_bytes(rpn_sel_cap(max_pre, large)) * slots;
    return b;
}

// numpy-2 bbox_transform of one box with weights (wx, wy, ww, wh): returns
// x1, y1, x2, y2 as the float32 store of numpy's (partly float64) arithmetic.
__device__ __forceinline__ void decode_box(float bx1, float by1, float bx2, float by2, float d0,
                                           float d1, float d2, float d3, float wx, float wy,
                                           float ww, float wh, float &x1, float &y1, float &x2,
                                           float &y2) {
    const float widths = bx2 - bx1 + 1.0f;
    const float heights = by2 - by1 + 1.0f;
    const float ctr_x = bx1 + 0.5f * widths;
    const float ctr_y = by1 + 0.5f * heights;
    const float dx = d0 / wx, dy = d1 / wy;
    const double dw = fmin((double)(d2 / ww), kBboxXformClip);
    const double dh = fmin((double)(d3 / wh), kBboxXformClip);
    const float pcx = dx * widths + ctr_x;
    const float pcy = dy * heights + ctr_y;
    const double pw = fmax(exp(dw) * (double)widths, 1.0);
    const double ph = fmax(exp(dh) * (double)heights, 1.0);
    x1 = (float)((double)pcx - 0.5 * pw);
    y1 = (float)((double)pcy - 0.5 * ph);
    x2 = (float)((double)pcx + 0.5 * pw - 1.0);
    y2 = (float)((double)pcy + 0.5 * ph - 1.0);
}

__device__ __forceinline__ float clip_coord(float v, float hi) {  // max(min(v, hi), 0)
    return fmaxf(fminf(v, hi), 0.f);
}

// utils/fpn.py:11-28 in numpy's float32 arithmetic
__device__ __forceinline__ int fpn_level(float x1, float y1, float x2, float y2, int k_min,
                                         int k_max, float s0, float lvl0) {
    const float w = x2 - x1 + 1.0f, h = y2 - y1 + 1.0f;
    float area = w * h;
    if (area < 0.f) area = 0.f;
    const float s = sqrtf(area);
    const float t = s / s0 + 1e-6f;
    const float l2 = (float)log2((double)t);  // correctly rounded float32 log2
    float lv = floorf(lvl0 + l2);
    lv = fminf(fmaxf(lv, (float)k_min), (float)k_max);
    return (int)lv;
}

// Small variant: everything in LDS.  Large variant (GB = true): the ten
// per-candidate float arrays live in the slot's global workspace.
template <int SelCap, int PreMax, bool GB>
struct RpnLds {
    uint64_t keys[SelCap];           // candidates, later NMS order keys
    float box[GB ? 1 : 10][GB ? 1 : PreMax];
    uint8_t keep_rank[PreMax];
    uint8_t keep_pos[PreMax];
    int scratch[32];
};

// Block-strided walk over probs[0, n) in memory order, 8 loads per thread in
// flight before any is consumed (a plain strided loop waits on every load:
// ~200 dependent HBM round trips per pass over a P2 score map).  f(m, s) is
// called for every m with s = probs[m], each wave's lanes on consecutive m;
// in the last partial row the lanes past n call f(-1, 0) so that every lane of
// a wave with work takes part in f's ballots.
#ifdef VD_PROF
#define PROF_DECL __shared__ long long prof_t[16]; int prof_n = 0;
#define PROF_MARK() do { __syncthreads(); if (threadIdx.x == 0) prof_t[prof_n] = wall_clock64(); ++prof_n; } while (0)
#define PROF_DUMP(tag) do { if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) { \
    for (int i_ = 1; i_ < prof_n; ++i_) printf("%s phase %d: %.1f us\n", tag, i_, (prof_t[i_] - prof_t[i_ - 1]) * 0.01); } } while (0)
#else
#define PROF_DECL
#define PROF_MARK()
#define PROF_DUMP(tag)
#endif

#ifndef VD_SWEEP_U
#define VD_SWEEP_U 8
#endif
template <class F>
__device__ inline void sweep_probs(const float *__restrict__ probs, int n, F f) {
    constexpr int U = VD_SWEEP_U;
    const int bd = blockDim.x;
    int m = threadIdx.x;
    // full batches: every lane of the block has all U elements
    const int full = (n / (U * bd)) * (U * bd);
    for (; m < full; m += U * bd) {
        float v[U];
#pragma unroll
        for (int i = 0; i < U; ++i) v[i] = probs[m + i * bd];
#pragma unroll
        for (int i = 0; i < U; ++i) f(m + i * bd, v[i]);
    }
    // tail: whole waves step together (ballots inside f stay wave-uniform)
    for (int base = full; base < n; base += bd) {
        const int i = base + (int)threadIdx.x;
        if (base + (int)(threadIdx.x & ~63u) >= n) break;  // this wave has no element
        const float v = i < n ? probs[i] : 0.f;
        if (i < n) f(i, v);
        else f(-1, 0.f);
    }
}

// ---------------------------------------------------------------------------
// Multi-workgroup radix select of the top `pre` 64-bit keys of every
// (level, image) slot.  Key of element e (score s):
//   key = float_key(s) << 32 | ~e          (unique; larger = earlier in the order)
// Pass q histograms the q-th digit (11 bits; the last pass 9) of the keys whose
// higher digits equal the boundary prefix fixed by passes < q.  From the
// histograms every workgroup derives the same state: walking the bins from the
// top, the boundary bin b of pass q holds the pre-th largest key; if the keys
// at or above it (above + cum(b)) fit the candidate capacity, the select is
// done with threshold "top bits >= prefix.b", else b extends the prefix.  Keys
// are unique, so the last pass always ends it (one key per bin).
static constexpr int kSelChunk = 4096;    // scores per select workgroup
static constexpr int kSelThreads = 256;
static constexpr int kSelPer = kSelChunk / kSelThreads;
static constexpr int kRadixBins = 2048;   // 11-bit digits
static constexpr int kRadixPasses = 6;    // 11 x 5 + 9 = 64 bits

__host__ __device__ constexpr int radix_width(int q) { return q < 5 ? 11 : 9; }
__host__ __device__ constexpr int radix_shift(int q) { return q < 5 ? 53 - 11 * q : 0; }

struct SelState {
    uint64_t prefix;  // fixed top `pbits` bits of the boundary
    int pbits;
    int above;        // keys strictly above the prefix range
    int done;         // 1: candidates = keys whose top `pbits` bits >= prefix
    int ncand;
};

struct SelSlot {  // per (image, level) slot; the candidate keys follow
    uint32_t hist[kRadixPasses][kRadixBins];
    SelState state[kRadixPasses];  // state[q]: after passes [0, q), by pass q's chunk 0
    int32_t count;
};
size_t sel_slot_bytes(int cap) {
    return a256(sizeof(SelSlot)) + a256(sizeof(uint64_t) * (size_t)cap);
}

struct SelLevels {  // per-level chunk offsets of the flattened grid
    int chunk0[VD_MAX_LEVELS + 1];
};

// Apply pass q's histogram to the state after passes [0, q): identical in every
// workgroup of the slot.  lds: int[16].  kSelThreads threads.
__device__ inline void sel_step(const SelSlot *__restrict__ st, int q, int pre, int cap, int *lds,
                                SelState &S) {
    const int t = threadIdx.x, lane = lane_id(), wave = wave_id();
    // thread t owns bins top - 8t - 0 .. top - 8t - 7 (highest first)
    uint32_t h[8];
    int tot = 0;
    const int top = kRadixBins - 1 - 8 * t;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        h[i] = st->hist[q][top - i];
        tot += (int)h[i];
    }
    int incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == 63) lds[wave] = incl;
    __syncthreads();
    int wbase = 0;
    for (int w = 0; w < wave; ++w) wbase += lds[w];
    const int excl = wbase + incl - tot;
    const int need = pre - S.above;  // >= 1, <= this prefix's key count
    if (excl < need && excl + tot >= need) {
        int acc = excl, i = 0;
        for (; i < 7; ++i) {
            if (acc + (int)h[i] >= need) break;
            acc += (int)h[i];
        }
        lds[8] = top - i;  // boundary bin
        lds[9] = acc;      // keys above it (within the prefix)
        lds[10] = (int)h[i];
    }
    __syncthreads();
    const int b = lds[8], cum_excl = lds[9], hb = lds[10];
    __syncthreads();
    const int w = radix_width(q);
    S.prefix = (S.prefix << w) | (uint64_t)b;
    S.pbits += w;
    if (S.above + cum_excl + hb <= cap) {
        S.done = 1;
        S.ncand = S.above + cum_excl + hb;
    } else {
        S.above += cum_excl;
    }
}

// The state after passes [0, q): pass q - 1's saved state plus its histogram.
__device__ inline SelState sel_state(const SelSlot *__restrict__ st, int q, int pre, int cap,
                                     int *lds) {
    if (q == 0) return SelState{0ull, 0, 0, 0, 0};
    SelState S = st->state[q - 1];
    if (!S.done) sel_step(st, q - 1, pre, cap, lds, S);
    return S;
}

__device__ __forceinline__ void sel_locate(const SelLevels &lvls, int num_levels, int &l,
                                           int &chunk) {
    const int bx = blockIdx.x;
    l = 0;
    while (l + 1 < num_levels && bx >= lvls.chunk0[l + 1]) ++l;
    chunk = bx - lvls.chunk0[l];
}

__device__ __forceinline__ uint64_t sel_key(const VdRpnLevel &lv, int m, float s) {
    const int K = lv.H * lv.W;
    const int a = m / K, hw = m - a * K;
    const int e = hw * lv.A + a;
    return ((uint64_t)float_key(s) << 32) | (uint32_t)(0xffffffffu - (uint32_t)e);
}

// top `bits` bits of key == / >= prefix, testing the float key first (the
// index part, an integer division, only when the score bits alone tie)
__device__ __forceinline__ int sel_cmp(const VdRpnLevel &lv, int m, float s, uint64_t prefix,
                                       int bits) {  // -1 below, 0 equal, 1 above
    if (bits == 0) return 0;
    const uint32_t fk = float_key(s);
    if (bits <= 32) {
        const uint32_t v = fk >> (32 - bits), p = (uint32_t)prefix;
        return v == p ? 0 : (v > p ? 1 : -1);
    }
    const uint32_t ph = (uint32_t)(prefix >> (bits - 32));
    if (fk != ph) return fk > ph ? 1 : -1;
    const uint64_t v = sel_key(lv, m, s) >> (64 - bits);
    return v == prefix ? 0 : (v > prefix ? 1 : -1);
}

__device__ __forceinline__ int sel_pre(int pre_nms_topN, int n_all) {
    return (pre_nms_topN <= 0 || pre_nms_topN >= n_all) ? n_all : pre_nms_topN;
}

__global__ __launch_bounds__(kSelThreads) void rpn_sel_hist_kernel(
    RpnArgs args, SelLevels lvls, int num_levels, int pre_nms_topN, int cap, int pass,
    char *__restrict__ sel_ws, size_t sel_slot_b) {
    __shared__ uint32_t lh[kRadixBins];
    __shared__ int lds[16];
    int l, chunk;
    sel_locate(lvls, num_levels, l, chunk);
    const int img = blockIdx.y;
    const VdRpnLevel lv = args.lv[l];
    const int K = lv.H * lv.W, n_all = K * lv.A;
    const int pre = sel_pre(pre_nms_topN, n_all);
    SelSlot *st = reinterpret_cast<SelSlot *>(sel_ws + (size_t)(img * num_levels + l) * sel_slot_b);
    const SelState S = sel_state(st, pass, pre, cap, lds);
    if (chunk == 0 && threadIdx.x == 0) st->state[pass] = S;  // for pass + 1
    if (S.done) return;
    for (int b = threadIdx.x; b < kRadixBins; b += kSelThreads) lh[b] = 0;
    __syncthreads();
    const float *probs = lv.cls_prob + (int64_t)img * n_all;
    const int m0 = chunk * kSelChunk + threadIdx.x;
    float v[kSelPer];
#pragma unroll
    for (int i = 0; i < kSelPer; ++i) {
        const int m = m0 + i * kSelThreads;
        v[i] = m < n_all ? probs[m] : 0.f;
    }
    const int sh = radix_shift(pass);
    const uint32_t dmask = (1u << radix_width(pass)) - 1u;
#pragma unroll
    for (int i = 0; i < kSelPer; ++i) {
        const int m = m0 + i * kSelThreads;
        if (m >= n_all) continue;
        if (pass == 0) {
            atomicAdd(&lh[float_key(v[i]) >> 21], 1u);
        } else if (sel_cmp(lv, m, v[i], S.prefix, S.pbits) == 0) {
            const uint64_t key = sel_key(lv, m, v[i]);
            atomicAdd(&lh[(uint32_t)(key >> sh) & dmask], 1u);
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kRadixBins; b += kSelThreads)
        if (lh[b]) atomicAdd(&st->hist[pass][b], lh[b]);
}

__global__ __launch_bounds__(kSelThreads) void rpn_sel_compact_kernel(
    RpnArgs args, SelLevels lvls, int num_levels, int pre_nms_topN, int cap,
    char *__restrict__ sel_ws, size_t sel_slot_b) {
    __shared__ int lds[16];
    int l, chunk;
    sel_locate(lvls, num_levels, l, chunk);
    const int img = blockIdx.y;
    const VdRpnLevel lv = args.lv[l];
    const int K = lv.H * lv.W, n_all = K * lv.A;
    const int pre = sel_pre(pre_nms_topN, n_all);
    char *slot = sel_ws + (size_t)(img * num_levels + l) * sel_slot_b;
    SelSlot *st = reinterpret_cast<SelSlot *>(slot);
    uint64_t *cand = reinterpret_cast<uint64_t *>(slot + a256(sizeof(SelSlot)));
    const SelState S = sel_state(st, kRadixPasses, pre, cap, lds);
    if (!S.done) {  // unreachable for unique keys; the slot's kernel reports it
        if (chunk == 0 && threadIdx.x == 0) st->count = -(1 << 30);
        return;
    }
    const float *probs = lv.cls_prob + (int64_t)img * n_all;
    const int m0 = chunk * kSelChunk + threadIdx.x;
    float v[kSelPer];
#pragma unroll
    for (int i = 0; i < kSelPer; ++i) {
        const int m = m0 + i * kSelThreads;
        v[i] = m < n_all ? probs[m] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < kSelPer; ++i) {
        const int m = m0 + i * kSelThreads;
        const bool p = m < n_all && sel_cmp(lv, m, v[i], S.prefix, S.pbits) >= 0;
        const uint64_t b = ballot(p);
        if (!b) continue;
        const int leader = __ffsll((unsigned long long)b) - 1;
        int base = 0;
        if (lane_id() == leader) base = atomicAdd(&st->count, __popcll(b));
        base = __shfl(base, leader);
        const int pos = base + lane_prefix(b);
        if (p && pos < cap) cand[pos] = sel_key(lv, m, v[i]);
    }
}

template <int SelCap, int PreMax, bool GB>
__global__ __launch_bounds__(1024) void rpn_proposals_kernel(
    RpnArgs args, int num_levels, const float *__restrict__ im_info, int pre_nms_topN,
    int post_nms_topN, float nms_thresh, float min_size, float *__restrict__ rois_out,
    float *__restrict__ probs_out, int32_t *__restrict__ counts_out, char *__restrict__ ws,
    size_t slot_bytes, size_t mask_bytes, size_t box_bytes, const char *__restrict__ sel_ws,
    size_t sel_slot_b) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    auto &L = *reinterpret_cast<RpnLds<SelCap, PreMax, GB> *>(lds_raw);
    PROF_DECL
    PROF_MARK();
    const int l = blockIdx.x, img = blockIdx.y;
    const VdRpnLevel lv = args.lv[l];
    const int A = lv.A, H = lv.H, W = lv.W, K = H * W;
    const int n_all = K * A;
    const float *probs = lv.cls_prob + (int64_t)img * A * K;
    const float *deltas = lv.bbox_pred + (int64_t)img * 4 * A * K;
    const int slot = img * num_levels + l;
    uint64_t *mask = reinterpret_cast<uint64_t *>(ws + (size_t)slot * slot_bytes);
    float *boxes = GB ? reinterpret_cast<float *>(ws + (size_t)slot * slot_bytes + mask_bytes)
                      : &L.box[0][0];
    // box-array stride: the slot's box region holds >= max_pre entries (rpn_box_bytes)
    const int bstride = GB ? (int)(box_bytes / (10 * sizeof(float))) : PreMax;
    uint64_t *gkeys = reinterpret_cast<uint64_t *>(ws + (size_t)slot * slot_bytes + mask_bytes +
                                                   box_bytes);
    int32_t *gm = reinterpret_cast<int32_t *>(gkeys + bstride);
    float *const px1 = boxes, *const py1 = boxes + bstride, *const px2 = boxes + 2 * bstride;
    float *const py2 = boxes + 3 * bstride, *const psc = boxes + 4 * bstride;
    float *const ox1 = boxes + 5 * bstride, *const oy1 = boxes + 6 * bstride;
    float *const ox2 = boxes + 7 * bstride, *const oy2 = boxes + 8 * bstride;
    float *const oar = boxes + 9 * bstride;

    // element e = (h*W + w)*A + a lives at probs[a*K + h*W + w]
    auto key_of = [&](int e) -> uint64_t {
        const int a = e % A, hw = e / A;
        const float s = probs[(int64_t)a * K + hw];
        return ((uint64_t)float_key(s) << 32) | (uint32_t)(0xffffffffu - (uint32_t)e);
    };
    // memory-order walk for coalesced count passes: m = a*K + hw  ->  e
    auto key_at = [&](int m, float s) -> uint64_t {
        const int a = m / K, hw = m - a * K;
        const int e = hw * A + a;
        return ((uint64_t)float_key(s) << 32) | (uint32_t)(0xffffffffu - (uint32_t)e);
    };

    // key_at(m, s) >= thr, the index part (an integer division) only on a
    // score tie with the threshold
    auto ge_thr = [&](int m, float s, uint64_t thr) -> bool {
        const uint32_t fk = float_key(s), th = (uint32_t)(thr >> 32);
        return fk != th ? fk > th : key_at(m, s) >= thr;
    };

    const bool take_all = pre_nms_topN <= 0 || pre_nms_topN >= n_all;
    const int pre = take_all ? n_all : pre_nms_topN;
    int ncand;
    if (take_all) {
        for (int e = threadIdx.x; e < n_all; e += blockDim.x) L.keys[e] = key_of(e);
        ncand = n_all;
        __syncthreads();
    } else if (sel_ws) {
        // candidates from the multi-workgroup radix select
        const char *sl = sel_ws + (size_t)slot * sel_slot_b;
        const uint64_t *cand = reinterpret_cast<const uint64_t *>(sl + a256(sizeof(SelSlot)));
        ncand = reinterpret_cast<const SelSlot *>(sl)->count;
        if (ncand < pre || ncand > SelCap) {  // cannot happen for unique keys: report
            if (threadIdx.x == 0) {
                counts_out[slot] = -1;
                if (GB) *gm = -1;
            }
            return;
        }
        for (int i = threadIdx.x; i < ncand; i += blockDim.x) L.keys[i] = cand[i];
        __syncthreads();
    } else {
        // ---- sample + threshold search
        const int S = min(kSampleMax, n_all);
        for (int j = threadIdx.x; j < kSampleMax; j += blockDim.x)
            L.keys[j] = j < S ? key_of((int)(((int64_t)j * n_all) / S)) : 0ull;
        __syncthreads();
        PROF_MARK();
        bitonic_sort_desc(L.keys, kSampleMax);
        PROF_MARK();
        int lo = 0, hi = S - 1;  // rank window in the sorted sample
        // threshold at ~1.5x pre expected candidates: <= 2048 keys to sort for
        // pre = 1000 (P2: rank 16 of the 2048-sample, ~4 % need a second count)
        int rank = (int)(((int64_t)3 * pre * S + 2 * (int64_t)n_all - 1) / (2 * (int64_t)n_all));
        if (rank > S - 1) rank = S - 1;
        uint64_t thr = 0;
        ncand = -1;
        for (int it = 0; it < 24; ++it) {
            thr = L.keys[rank];
            __syncthreads();
            int c = 0;
            sweep_probs(probs, n_all, [&](int m, float s) { c += m >= 0 && ge_thr(m, s, thr); });
            c = block_sum(c, L.scratch);
            if (c >= pre && c <= SelCap) { ncand = c; break; }
            if (c < pre) lo = rank + 1; else hi = rank - 1;
            if (lo > hi) break;
            rank = (lo + hi) >> 1;
        }
        if (ncand < 0) {  // cannot bracket: count -1, which collect_distribute and the
                          // detections propagate to the engine's host read (raises)
            if (threadIdx.x == 0) {
                counts_out[slot] = -1;
                if (GB) *gm = -1;
            }
            return;
        }
        PROF_MARK();
        // unordered compaction (the candidates are sorted by their unique keys
        // next): one LDS atomic per wave and batch, no barrier per element row
        if (threadIdx.x == 0) L.scratch[31] = 0;
        __syncthreads();
        sweep_probs(probs, n_all, [&](int m, float s) {
            const bool p = m >= 0 && ge_thr(m, s, thr);
            const uint64_t b = ballot(p);
            if (!b) return;
            const uint64_t k = p ? key_at(m, s) : 0ull;
            int base = 0;
            if (lane_id() == __ffsll((unsigned long long)b) - 1)
                base = atomicAdd(&L.scratch[31], __popcll(b));
            base = __shfl(base, __ffsll((unsigned long long)b) - 1);
            if (p) L.keys[base + lane_prefix(b)] = k;
        });
        __syncthreads();
    }
    {
        const int np2 = next_pow2(ncand);
        for (int i = ncand + threadIdx.x; i < np2; i += blockDim.x) L.keys[i] = 0ull;
        __syncthreads();
        PROF_MARK();
        bitonic_sort_desc(L.keys, np2);
        PROF_MARK();
    }

    // ---- decode + clip + filter (positions in score order)
    const float im_h = im_info[img * 3 + 0], im_w = im_info[img * 3 + 1];
    const float ms = min_size * im_info[img * 3 + 2];
    const double stride = 1.0 / (double)lv.spatial_scale;
    for (int t = threadIdx.x; t < pre; t += blockDim.x) {
        const uint64_t k = L.keys[t];
        const int e = (int)(0xffffffffu - (uint32_t)k);
        const int a = e % A, hw = e / A, h = hw / W, w = hw - h * W;
        const double sx = (double)w * stride, sy = (double)h * stride;
        const double *an = lv.anchors + a * 4;
        const float bx1 = (float)(an[0] + sx), by1 = (float)(an[1] + sy);
        const float bx2 = (float)(an[2] + sx), by2 = (float)(an[3] + sy);
        const float *d = deltas + (int64_t)(4 * a) * K + hw;
        float x1, y1, x2, y2;
        decode_box(bx1, by1, bx2, by2, d[0], d[K], d[2 * K], d[3 * K], 1.f, 1.f, 1.f, 1.f, x1, y1,
                   x2, y2);
        x1 = clip_coord(x1, im_w - 1.f);
        y1 = clip_coord(y1, im_h - 1.f);
        x2 = clip_coord(x2, im_w - 1.f);
        y2 = clip_coord(y2, im_h - 1.f);
        ox1[t] = x1;
        oy1[t] = y1;
        ox2[t] = x2;
        oy2[t] = y2;
        oar[t] = key_float((uint32_t)(k >> 32));
    }
    __syncthreads();
    const int m = block_compact(
        pre,
        [&](int t) {
            const float ws_ = ox2[t] - ox1[t] + 1.f, hs = oy2[t] - oy1[t] + 1.f;
            const float xc = ox1[t] + ws_ / 2.f, yc = oy1[t] + hs / 2.f;
            return (ws_ >= ms) && (hs >= ms) && (xc < im_w) && (yc < im_h);
        },
        [&](int p, int t) {
            px1[p] = ox1[t];
            py1[p] = oy1[t];
            px2[p] = ox2[t];
            py2[p] = oy2[t];
            psc[p] = oar[t];
        },
        L.scratch);

    const int cap = post_nms_topN > 0 ? post_nms_topN : pre;
    float *ro = rois_out + (size_t)slot * cap * 5;
    float *po = probs_out + (size_t)slot * cap;
    if (nms_thresh <= 0.f) {
        const int n_out = min(m, cap);
        for (int p = threadIdx.x; p < n_out; p += blockDim.x) {
            ro[p * 5 + 0] = (float)img;
            ro[p * 5 + 1] = px1[p];
            ro[p * 5 + 2] = py1[p];
            ro[p * 5 + 3] = px2[p];
            ro[p * 5 + 4] = py2[p];
            po[p] = psc[p];
        }
        if (threadIdx.x == 0) {
            counts_out[slot] = n_out;
            if (GB) *gm = -1;
        }
        return;
    }

    // ---- NMS: processing order = scores.argsort()[::-1] on the sorted array
    {
        // psc is non-increasing (candidates sorted by score); only equal scores
        // can reorder, so without ties the processing order is the identity
        int ties = 0;
        for (int p = threadIdx.x; p + 1 < m; p += blockDim.x)
            ties |= float_key(psc[p]) == float_key(psc[p + 1]);
        ties = block_sum(ties, L.scratch);
        const int np2 = next_pow2(m);
        for (int p = threadIdx.x; p < np2; p += blockDim.x)
            L.keys[p] = p < m ? ((uint64_t)float_key(psc[p]) << 32) | (uint32_t)p : 0ull;
        __syncthreads();
        PROF_MARK();
        if (m > 1 && ties) bitonic_sort_desc(L.keys, np2);
        PROF_MARK();
    }
    for (int r = threadIdx.x; r < m; r += blockDim.x) {
        const int p = (int)(uint32_t)L.keys[r];
        const float a = px1[p], b = py1[p], c = px2[p], e = py2[p];
        ox1[r] = a;
        oy1[r] = b;
        ox2[r] = c;
        oy2[r] = e;
        oar[r] = (c - a + 1) * (e - b + 1);
        if (GB) gkeys[r] = L.keys[r];
    }
    if (GB) {  // mask rows and resolve run as rpn_nms_mask_kernel / rpn_nms_finish_kernel
        PROF_MARK();
        PROF_DUMP("select");
        if (threadIdx.x == 0) *gm = m;
        return;
    }
    __syncthreads();
    nms_build_mask_rows(ox1, oy1, ox2, oy2, oar, m, nms_thresh, mask, wave_id(),
                        num_waves());
    __threadfence_block();
    __syncthreads();
    if (wave_id() == 0) nms_resolve_wave(mask, m, L.keep_rank);
    __syncthreads();
    for (int r = threadIdx.x; r < m; r += blockDim.x)
        L.keep_pos[(int)(uint32_t)L.keys[r]] = L.keep_rank[r];
    __syncthreads();
    const int kept = block_compact(
        m, [&](int p) { return L.keep_pos[p] != 0; },
        [&](int pos, int p) {
            if (pos < cap) {
                ro[pos * 5 + 0] = (float)img;
                ro[pos * 5 + 1] = px1[p];
                ro[pos * 5 + 2] = py1[p];
                ro[pos * 5 + 3] = px2[p];
                ro[pos * 5 + 4] = py2[p];
                po[pos] = psc[p];
            }
        },
        L.scratch);
    if (threadIdx.x == 0) counts_out[slot] = min(kept, cap);
}

// Large variant, phase 2: the suppression mask of every slot built by many
// workgroups (one wave per row, as the standalone vd_nms) instead of the 16
// waves of the slot's own workgroup.
__global__ __launch_bounds__(1024) void rpn_nms_mask_kernel(char *__restrict__ ws,
                                                             size_t slot_bytes, size_t mask_bytes,
                                                             size_t box_bytes, float nms_thresh) {
    const int slot = blockIdx.y;
    char *base = ws + (size_t)slot * slot_bytes;
    const int bstride = (int)(box_bytes / (10 * sizeof(float)));
    const float *boxes = reinterpret_cast<const float *>(base + mask_bytes);
    const int32_t m = *reinterpret_cast<const int32_t *>(
        reinterpret_cast<const uint64_t *>(base + mask_bytes + box_bytes) + bstride);
    if (m < 1) return;
    const int wpb = blockDim.x / 64;
    nms_build_mask_rows(boxes + 5 * bstride, boxes + 6 * bstride, boxes + 7 * bstride,
                        boxes + 8 * bstride, boxes + 9 * bstride, m, nms_thresh,
                        reinterpret_cast<uint64_t *>(base), blockIdx.x * wpb + wave_id(),
                        gridDim.x * wpb);
}

// Split NMS, phase 2 (round 5): one 256-thread workgroup per (64-row block,
// slot) with the slot's boxes from the block's first row on staged in LDS, so
// the IoU tests read LDS instead of one global load per lane and box; each
// wave builds 16 rows, a row's words stored by the lanes in one coalesced
// write.  Opt-in (VOSDET_RPN_MASK_LDS=1): measured 1.3x slower than the
// one-wave-per-row form above, which stays the default.
static constexpr int kMaskLdsMaxBoxes = 3200;  // 5 x 4 B x 3200 = 62.5 KiB

__global__ __launch_bounds__(256) void rpn_nms_mask_lds_kernel(char *__restrict__ ws,
                                                               size_t slot_bytes,
                                                               size_t mask_bytes,
                                                               size_t box_bytes, float nms_thresh) {
    extern __shared__ __attribute__((aligned(16))) float lbox[];
    const int slot = blockIdx.y;
    char *base = ws + (size_t)slot * slot_bytes;
    const int bstride = (int)(box_bytes / (10 * sizeof(float)));
    const float *boxes = reinterpret_cast<const float *>(base + mask_bytes);
    const int32_t m = *reinterpret_cast<const int32_t *>(
        reinterpret_cast<const uint64_t *>(base + mask_bytes + box_bytes) + bstride);
    const int r0 = blockIdx.x * 64;
    if (m < 1 || r0 >= m) return;
    const int n = m - r0;  // boxes [r0, m): this block's rows and every later column
    float *X1 = lbox, *Y1 = lbox + n, *X2 = lbox + 2 * n, *Y2 = lbox + 3 * n, *AR = lbox + 4 * n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        X1[i] = boxes[5 * bstride + r0 + i];
        Y1[i] = boxes[6 * bstride + r0 + i];
        X2[i] = boxes[7 * bstride + r0 + i];
        Y2[i] = boxes[8 * bstride + r0 + i];
        AR[i] = boxes[9 * bstride + r0 + i];
    }
    __syncthreads();
    uint64_t *mask = reinterpret_cast<uint64_t *>(base);
    const int words = (m + 63) >> 6;
    const int lane = lane_id();
    const int w0 = blockIdx.x;  // the diagonal word of every row of this block
    for (int rr = wave_id(); rr < 64 && r0 + rr < m; rr += num_waves()) {
        const int i = r0 + rr;
        const float ix1 = X1[rr], iy1 = Y1[rr], ix2 = X2[rr], iy2 = Y2[rr], ia = AR[rr];
        uint64_t mine = 0;
        for (int w = w0; w < words; ++w) {
            const int j = (w << 6) + lane;  // column; local index j - r0
            bool sup = false;
            if (j > i && j < m) {
                const int q = j - r0;
                sup = suppresses(ix1, iy1, ix2, iy2, ia, X1[q], Y1[q], X2[q], Y2[q], AR[q],
                                 nms_thresh);
            }
            const uint64_t b = ballot(sup);
            if (lane == w - w0) mine = b;
        }
        if (lane < words - w0) mask[(int64_t)i * words + w0 + lane] = mine;
    }
}

// Split NMS, phase 3: greedy resolve (one wave) + ascending compaction.  The
// slot's mask is first copied into LDS by the whole workgroup when it fits
// (m <= ~1300 at 160 KiB): the resolve then waits on LDS, not on a global
// round trip per 64-row block.  LDS: keys[cap] u64 | keep_rank[cap] |
// keep_pos[cap] | scratch int[32] | mask (optional).
__host__ __device__ inline size_t finish_lds_base(int cap) {
    return a256((size_t)cap * 8 + 2 * (size_t)cap) + 32 * sizeof(int);
}

__global__ __launch_bounds__(1024) void rpn_nms_finish_kernel(
    int num_levels, int post_nms_topN, float *__restrict__ rois_out,
    float *__restrict__ probs_out, int32_t *__restrict__ counts_out, char *__restrict__ ws,
    size_t slot_bytes, size_t mask_bytes, size_t box_bytes, int cap_keys, int lds_mask_rows) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    uint64_t *keys = reinterpret_cast<uint64_t *>(lds_raw);
    uint8_t *keep_rank = reinterpret_cast<uint8_t *>(keys + cap_keys);
    uint8_t *keep_pos = keep_rank + cap_keys;
    const size_t base_bytes = finish_lds_base(cap_keys);
    int *scratch = reinterpret_cast<int *>(lds_raw + base_bytes - 32 * sizeof(int));
    uint64_t *lmask = reinterpret_cast<uint64_t *>(lds_raw + base_bytes);
    PROF_DECL
    PROF_MARK();
    const int l = blockIdx.x, img = blockIdx.y;
    const int slot = img * num_levels + l;
    char *base = ws + (size_t)slot * slot_bytes;
    const int bstride = (int)(box_bytes / (10 * sizeof(float)));
    const float *boxes = reinterpret_cast<const float *>(base + mask_bytes);
    const uint64_t *gkeys = reinterpret_cast<const uint64_t *>(base + mask_bytes + box_bytes);
    const int32_t m = *reinterpret_cast<const int32_t *>(gkeys + bstride);
    if (m < 0) return;  // finished in phase 1 (no NMS, or could not bracket)
    const float *px1 = boxes, *py1 = boxes + bstride, *px2 = boxes + 2 * bstride;
    const float *py2 = boxes + 3 * bstride, *psc = boxes + 4 * bstride;
    for (int r = threadIdx.x; r < m; r += blockDim.x) keys[r] = gkeys[r];
    const uint64_t *gmask = reinterpret_cast<const uint64_t *>(base);
    const bool in_lds = m <= lds_mask_rows;
    if (in_lds) {  // whole mask (m rows x words) into LDS
        const int n = m * ((m + 63) >> 6);
        for (int i = threadIdx.x; i < n; i += blockDim.x) lmask[i] = gmask[i];
    }
    __syncthreads();
    PROF_MARK();
    if (wave_id() == 0 && m > 0) {  // two inlined copies: ds_read / global_load
        if (in_lds)
            nms_resolve_wave(lmask, m, keep_rank);
        else
            nms_resolve_wave(gmask, m, keep_rank);
    }
    __syncthreads();
    PROF_MARK();
    for (int r = threadIdx.x; r < m; r += blockDim.x)
        keep_pos[(int)(uint32_t)keys[r]] = keep_rank[r];
    __syncthreads();
    const int cap = post_nms_topN;
    float *ro = rois_out + (size_t)slot * cap * 5;
    float *po = probs_out + (size_t)slot * cap;
    const int kept = block_compact(
        m, [&](int p) { return keep_pos[p] != 0; },
        [&](int pos, int p) {
            if (pos < cap) {
                ro[pos * 5 + 0] = (float)img;
                ro[pos * 5 + 1] = px1[p];
                ro[pos * 5 + 2] = py1[p];
                ro[pos * 5 + 3] = px2[p];
                ro[pos * 5 + 4] = py2[p];
                po[pos] = psc[p];
            }
        },
        scratch);
    PROF_MARK();
    PROF_DUMP("finish");
    if (threadIdx.x == 0) counts_out[slot] = min(kept, cap);
}

int launch_rpn_proposals(const VdRpnLevel *levels, int num_levels, int num_images,
                         const float *im_info, int pre_nms_topN, int post_nms_topN,
                         float nms_thresh, float min_size, float *rois_out, float *probs_out,
                         int32_t *counts_out, void *workspace, size_t ws_bytes, hipStream_t s) {
    if (num_levels < 1 || num_levels > VD_MAX_LEVELS || num_images < 1) return VD_ERR_ARG;
    if (post_nms_topN <= 0) return VD_ERR_ARG;  // output capacity is post_nms_topN
    RpnArgs args;
    for (int l = 0; l < num_levels; ++l) args.lv[l] = levels[l];
    int max_pre;
    bool large;
    if (!rpn_plan(levels, num_levels, pre_nms_topN, &max_pre, &large)) return VD_ERR_SHAPE;
    const bool split = rpn_split(large);
    const int p = max_pre < 64 ? 64 : max_pre;
    const size_t mb = rpn_mask_bytes(p);
    const size_t bb = split ? rpn_box_bytes(p) : 0;
    const size_t sb = rpn_slot_bytes(max_pre, split);
    if (!workspace || ws_bytes < sb * (size_t)num_levels * (size_t)num_images)
        return VD_ERR_WORKSPACE;
    const dim3 grid(num_levels, num_images);
    // multi-workgroup select of every slot that keeps fewer than all its anchors
    const char *sel_ws = nullptr;
    size_t selb = 0;
    if (rpn_presel()) {
        SelLevels sl;
        int nch = 0;
        for (int l = 0; l < num_levels; ++l) {
            sl.chunk0[l] = nch;
            const int n_all = levels[l].A * levels[l].H * levels[l].W;
            const bool take_all = pre_nms_topN <= 0 || pre_nms_topN >= n_all;
            nch += take_all ? 0 : (n_all + kSelChunk - 1) / kSelChunk;
        }
        sl.chunk0[num_levels] = nch;
        const int cap = rpn_sel_cap(max_pre, large);
        selb = sel_slot_bytes(cap);
        const size_t slots = (size_t)num_levels * (size_t)num_images;
        if (ws_bytes < sb * slots + selb * slots) return VD_ERR_WORKSPACE;
        char *sw = (char *)workspace + sb * slots;
        sel_ws = sw;
        if (nch > 0) {
            if (zero_async(sw, selb * slots, s) != VD_OK) return VD_ERR_LAUNCH;
            const dim3 sgrid(nch, num_images);
            for (int pass = 0; pass < kRadixPasses; ++pass)
                hipLaunchKernelGGL(rpn_sel_hist_kernel, sgrid, dim3(kSelThreads), 0, s, args, sl,
                                   num_levels, pre_nms_topN, cap, pass, sw, selb);
            hipLaunchKernelGGL(rpn_sel_compact_kernel, sgrid, dim3(kSelThreads), 0, s, args, sl,
                               num_levels, pre_nms_topN, cap, sw, selb);
        }
    }
    if (split) {
        if (large) {
            using Lds = RpnLds<kSelCapL, kPreMaxL, true>;
            hipLaunchKernelGGL((rpn_proposals_kernel<kSelCapL, kPreMaxL, true>), grid,
                               dim3(1024), sizeof(Lds), s, args, num_levels, im_info,
                               pre_nms_topN, post_nms_topN, nms_thresh, min_size, rois_out,
                               probs_out, counts_out, (char *)workspace, sb, mb, bb, sel_ws, selb);
        } else {
            using Lds = RpnLds<kSelCap, kPreMax, true>;
            hipLaunchKernelGGL((rpn_proposals_kernel<kSelCap, kPreMax, true>), grid, dim3(1024),
                               sizeof(Lds), s, args, num_levels, im_info, pre_nms_topN,
                               post_nms_topN, nms_thresh, min_size, rois_out, probs_out,
                               counts_out, (char *)workspace, sb, mb, bb, sel_ws, selb);
        }
        if (nms_thresh > 0.f) {
            if (rpn_mask_lds() && p <= kMaskLdsMaxBoxes && (p + 63) / 64 <= 64) {
                const dim3 mgrid((p + 63) / 64, num_levels * num_images);
                hipLaunchKernelGGL(rpn_nms_mask_lds_kernel, mgrid, dim3(256),
                                   5 * sizeof(float) * (size_t)p, s, (char *)workspace, sb, mb,
                                   bb, nms_thresh);
            } else {
                const int rows_per_block = 16;  // 16 waves, one row each per pass
                const dim3 mgrid((p + rows_per_block - 1) / rows_per_block,
                                 num_levels * num_images);
                hipLaunchKernelGGL(rpn_nms_mask_kernel, mgrid, dim3(64 * rows_per_block), 0, s,
                                   (char *)workspace, sb, mb, bb, nms_thresh);
            }
            // keys / keep arrays for p candidates, plus the mask when it fits
            const size_t lbase = finish_lds_base(p);
            const int words = (p + 63) / 64;
            const size_t lmask = (size_t)p * words * 8;
            const bool in_lds = lbase + lmask <= VD_LDS_BYTES;
            hipLaunchKernelGGL(rpn_nms_finish_kernel, grid, dim3(1024),
                               lbase + (in_lds ? lmask : 0), s, num_levels, post_nms_topN,
                               rois_out, probs_out, counts_out, (char *)workspace, sb, mb, bb,
                               p, in_lds ? p : 0);
        }
    } else {
        using Lds = RpnLds<kSelCap, kPreMax, false>;
        hipLaunchKernelGGL((rpn_proposals_kernel<kSelCap, kPreMax, false>), grid, dim3(1024),
                           sizeof(Lds), s, args, num_levels, im_info, pre_nms_topN,
                           post_nms_topN, nms_thresh, min_size, rois_out, probs_out, counts_out,
                           (char *)workspace, sb, mb, bb, sel_ws, selb);
    }
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// --------------------------------------------------------------------------
// collect + distribute (per image)
// --------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void collect_distribute_kernel(
    const float *__restrict__ level_rois, const float *__restrict__ level_probs,
    const int32_t *__restrict__ level_counts, int num_levels, int level_cap, int post_nms_topN,
    int k_min, int k_max, float *__restrict__ rois_out, int32_t *__restrict__ lvl_out,
    int32_t *__restrict__ count_out) {
    __shared__ uint64_t keys[kSelCap];
    __shared__ int offs[VD_MAX_LEVELS + 1];
    __shared__ int failed;
    const int img = blockIdx.x;
    if (threadIdx.x == 0) {
        int o = 0;
        failed = 0;
        for (int l = 0; l < num_levels; ++l) {
            offs[l] = o;
            const int c = level_counts[img * num_levels + l];
            failed |= c < 0;  // a level's selection could not bracket its top-k
            o += c > 0 ? c : 0;
        }
        offs[num_levels] = o;
        if (failed) count_out[img] = -1;
    }
    __syncthreads();
    if (failed) return;
    const int n = offs[num_levels];
    const int np2 = next_pow2(n < 1 ? 1 : n);
    for (int q = threadIdx.x; q < np2; q += blockDim.x) {
        uint64_t k = 0;
        if (q < n) {
            int l = 0;
            while (q >= offs[l + 1]) ++l;
            const int t = q - offs[l];
            const float p = level_probs[((size_t)img * num_levels + l) * level_cap + t];
            k = ((uint64_t)float_key(p) << 32) | (uint32_t)(0xffffffffu - (uint32_t)q);
        }
        keys[q] = k;
    }
    __syncthreads();
    bitonic_sort_desc(keys, np2);
    const int R = min(n, post_nms_topN);
    for (int r = threadIdx.x; r < R; r += blockDim.x) {
        const int q = (int)(0xffffffffu - (uint32_t)keys[r]);
        int l = 0;
        while (q >= offs[l + 1]) ++l;
        const int t = q - offs[l];
        const float *src = level_rois + (((size_t)img * num_levels + l) * level_cap + t) * 5;
        float *dst = rois_out + ((size_t)img * post_nms_topN + r) * 5;
        const float b = src[0], x1 = src[1], y1 = src[2], x2 = src[3], y2 = src[4];
        dst[0] = b;
        dst[1] = x1;
        dst[2] = y1;
        dst[3] = x2;
        dst[4] = y2;
        lvl_out[(size_t)img * post_nms_topN + r] =
            fpn_level(x1, y1, x2, y2, k_min, k_max, 224.f, 4.f) - k_min;
    }
    if (threadIdx.x == 0) count_out[img] = R;
}

int launch_collect_distribute(const float *level_rois, const float *level_probs,
                              const int32_t *level_counts, int num_levels, int level_cap,
                              int num_images, int post_nms_topN, int k_min, int k_max,
                              float *rois_out, int32_t *lvl_out, int32_t *count_out,
                              hipStream_t s) {
    if (num_levels < 1 || num_levels > VD_MAX_LEVELS || num_images < 1 || post_nms_topN < 1)
        return VD_ERR_ARG;
    if ((int64_t)num_levels * level_cap > kSelCap) return VD_ERR_SHAPE;
    hipLaunchKernelGGL(collect_distribute_kernel, dim3(num_images), dim3(1024), 0, s, level_rois,
                       level_probs, level_counts, num_levels, level_cap, post_nms_topN, k_min,
                       k_max, rois_out, lvl_out, count_out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// --------------------------------------------------------------------------
// stand-alone level map
// --------------------------------------------------------------------------
__global__ void map_levels_kernel(const float *__restrict__ rois, int stride, int col0, int R,
                                  int k_min, int k_max, float s0, float lvl0,
                                  int32_t *__restrict__ out) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const float *b = rois + (int64_t)r * stride + col0;
    out[r] = fpn_level(b[0], b[1], b[2], b[3], k_min, k_max, s0, lvl0);
}

// --------------------------------------------------------------------------
// mask-head batch without a host read (im_detect_mask's _get_rois_blob +
// _add_multilevel_rois_for_test, lib/core/test.py:877-927): block f writes
// frame f's detections at global rows prefix(counts)[f] + j; rows [row0,
// row0 + rows) land in the outputs, the rest of them is padding.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mask_rois_kernel(
    const float *__restrict__ dets, const int32_t *__restrict__ classes,
    const int32_t *__restrict__ counts, int F, int det_cap, const double *__restrict__ im_scale,
    int row0, int rows, int k_min, int k_max, float s0, float lvl0, float *__restrict__ rois_out,
    int32_t *__restrict__ lvl_out, int32_t *__restrict__ cls_out, int32_t *__restrict__ total_out) {
    const int f = blockIdx.x;
    int pre = 0, total = 0;
    for (int i = 0; i < F; ++i) {  // F is small (frames per step); negative = failed frame
        const int c = counts[i] > 0 ? min(counts[i], det_cap) : 0;
        pre += i < f ? c : 0;
        total += c;
    }
    const int n = counts[f] > 0 ? min(counts[f], det_cap) : 0;
    const double sc = im_scale[f];
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
        const int o = pre + j - row0;
        if (o < 0 || o >= rows) continue;
        const float *d = dets + ((int64_t)f * det_cap + j) * 5;
        // float64 product, float32 store (_project_im_rois, test.py:893-906)
        const float x1 = (float)((double)d[0] * sc), y1 = (float)((double)d[1] * sc);
        const float x2 = (float)((double)d[2] * sc), y2 = (float)((double)d[3] * sc);
        float *r = rois_out + (int64_t)o * 5;
        r[0] = (float)f;
        r[1] = x1;
        r[2] = y1;
        r[3] = x2;
        r[4] = y2;
        lvl_out[o] = fpn_level(x1, y1, x2, y2, k_min, k_max, s0, lvl0) - k_min;
        cls_out[o] = classes[(int64_t)f * det_cap + j];
    }
    const int pad0 = max(total - row0, 0);
    for (int o = pad0 + f * blockDim.x + threadIdx.x; o < rows; o += F * blockDim.x) {
        float *r = rois_out + (int64_t)o * 5;
        r[0] = 0.f;
        r[1] = r[2] = r[3] = r[4] = 0.f;
        lvl_out[o] = 0;
        cls_out[o] = 1;
    }
    if (f == 0 && threadIdx.x == 0 && total_out) total_out[0] = total;
}

int launch_mask_rois(const float *dets, const int32_t *classes, const int32_t *counts, int F,
                     int det_cap, const double *im_scale, int row0, int rows, int k_min,
                     int k_max, float s0, float lvl0, float *rois_out, int32_t *lvl_out,
                     int32_t *cls_out, int32_t *total_out, hipStream_t s) {
    if (F <= 0) return VD_OK;
    hipLaunchKernelGGL(mask_rois_kernel, dim3(F), dim3(256), 0, s, dets, classes, counts, F,
                       det_cap, im_scale, row0, rows, k_min, k_max, s0, lvl0, rois_out, lvl_out,
                       cls_out, total_out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int launch_map_levels(const float *rois, int roi_stride, int col0, int R, int k_min, int k_max,
                      float s0, float lvl0, int32_t *lvl_out, hipStream_t s) {
    if (R <= 0) return VD_OK;
    hipLaunchKernelGGL(map_levels_kernel, dim3((R + 255) / 256), dim3(256), 0, s, rois,
                       roi_stride, col0, R, k_min, k_max, s0, lvl0, lvl_out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
