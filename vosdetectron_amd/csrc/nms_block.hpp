// Block-level greedy NMS building blocks (device code), shared by the
// standalone vd_nms, the RPN proposal kernel and the class-NMS kernel.
//
// Semantics: lib/utils/cython_nms.pyx:37-87.  Boxes are given in PROCESSING
// order (rank 0 first).  Phase 1 builds the upper-triangular suppression
// bitmask with one wave ballot per (row, 64-column word) -- a row's word is the
// 64 IoU tests of its 64 lanes.  Phase 2 is the greedy resolution by one wave:
// per 64-row block the diagonal word is resolved with scalar bit ops on
// readlane'd rows (no memory round trip), then every kept row of the block is
// OR-ed into the "removed" words that lanes hold for the later blocks.
// Result: keep flag per rank, identical to the sequential cython loop (a
// suppressed box never suppresses, and "i suppresses j" is only ever tested
// for i processed before j).
#pragma once

#include "common.hpp"

namespace vd {

static constexpr int kNmsMaxWordsPerLane = 4;  // words <= 256  ->  n <= 16384

// Phase 1.  mask: global (or LDS) buffer of m*words u64.  Rows are spread over
// `row_stride` waves starting at `row_begin`; pass the block's wave id / count
// for an in-block build, or a global wave index for a multi-workgroup build.
__device__ inline void nms_build_mask_rows(const float *__restrict__ x1, const float *__restrict__ y1,
                                           const float *__restrict__ x2, const float *__restrict__ y2,
                                           const float *__restrict__ area, int m, float thresh,
                                           uint64_t *__restrict__ mask, int row_begin,
                                           int row_stride) {
    const int words = (m + 63) >> 6;
    const int lane = lane_id();
    for (int i = row_begin; i < m; i += row_stride) {
        const float ix1 = x1[i], iy1 = y1[i], ix2 = x2[i], iy2 = y2[i], ia = area[i];
        for (int w = i >> 6; w < words; ++w) {
            const int j = (w << 6) + lane;
            bool s = false;
            if (j > i && j < m)
                s = suppresses(ix1, iy1, ix2, iy2, ia, x1[j], y1[j], x2[j], y2[j], area[j], thresh);
            const uint64_t b = ballot(s);
            if (lane == 0) mask[(int64_t)i * words + w] = b;
        }
    }
}

// Phase 2, executed by ONE wave (all 64 lanes).  keep[rank] = 1/0.  Forced
// inline: as an out-of-line call the 64-bit state spills to scratch and every
// LDS mask read goes through flat addressing.
__device__ __forceinline__ void nms_resolve_wave(const uint64_t *__restrict__ mask, int m,
                                                 uint8_t *__restrict__ keep) {
    const int words = (m + 63) >> 6;
    const int lane = lane_id();
    uint64_t remv[kNmsMaxWordsPerLane];
#pragma unroll
    for (int q = 0; q < kNmsMaxWordsPerLane; ++q) remv[q] = 0;
    for (int blk = 0; blk < words; ++blk) {
        const int row = (blk << 6) + lane;
        const uint64_t diag = row < m ? mask[(int64_t)row * words + blk] : 0ull;
        // the removed-word of this block lives in lane (blk & 63), slot blk >> 6
        uint64_t cur = 0;
#pragma unroll
        for (int q = 0; q < kNmsMaxWordsPerLane; ++q)
            if (q == (blk >> 6)) cur = readlane64(remv[q], blk & 63);
        // Greedy inside the block, visiting only rows that can change it: a
        // row with an empty diagonal word suppresses nothing here, so the loop
        // steps (find-first-set) through the not-yet-removed rows that do have
        // suppression edges; every row left unremoved at the end is kept.
        const int nrows = min(64, m - (blk << 6));
        const uint64_t valid = nrows == 64 ? ~0ull : ((1ull << nrows) - 1ull);
        const uint64_t nz = ballot(diag != 0ull);
        uint64_t todo = nz & ~cur & valid;
        while (todo) {
            const int t = __ffsll((unsigned long long)todo) - 1;
            cur |= readlane64(diag, t);  // bits > t only (upper triangle)
            todo &= ~cur & (~1ull << t);
        }
        const uint64_t kept = ~cur & valid;
        if (row < m) keep[row] = (uint8_t)((kept >> lane) & 1ull);
        // OR the kept rows of this block into the later words: 16 rows' words
        // loaded before any is used (a dependent load per kept row made this
        // loop one memory round trip per kept box)
#pragma unroll
        for (int q = 0; q < kNmsMaxWordsPerLane; ++q) {
            const int w = lane + (q << 6);
            if (w > blk && w < words) {
                uint64_t acc = 0;
                const uint64_t *col = mask + (int64_t)(blk << 6) * words + w;
                for (int t0 = 0; t0 < nrows; t0 += 16) {
                    const uint64_t kb = (kept >> t0) & 0xffffull;
                    if (!kb) continue;  // wave-uniform
                    uint64_t v[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        v[i] = col[(int64_t)min(t0 + i, nrows - 1) * words];
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        if ((kb >> i) & 1ull) acc |= v[i];
                }
                remv[q] |= acc;
            }
        }
    }
}

}  // namespace vd
