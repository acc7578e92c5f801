// RoIAlign research kernels of round 1, kept as the record of the experiments
// DESIGN.md section 4 reports (NOT part of libvosdet.so; not built by build()).
// Variant 16: XCD channel-sliced separable forward (reached the compulsory
// fabric bytes but 2.7x the VALU of the product kernel, 510 us vs 306 us).
// Variant 30: speed-of-light probe -- reads each RoI's footprint once, no
// sampling arithmetic (NOT RoIAlign).  They compiled inside roi_align.hip
// (same helpers: RoiGeom, row_taps, ld4, lane_id/wave_id) and were selected by
// VOSDET_ROIALIGN_VARIANT=16/30 in launch_roi_align_fpn_nhwc:
//
//         if (variant == 30 && PH == PW && C % 256 == 0) {  // speed-of-light probe (not RoIAlign)
//             hipLaunchKernelGGL(roi_footprint_probe_kernel, dim3(R), dim3(64 * (PH < 8 ? PH : 8)),
//                                0, s, fa, C, rois, lvl, order, PH, out);
//             return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
//         }
//         if (variant == 16 && sr == 2 && PH == PW && C % 32 == 0 && PH <= 16) {
//             const int64_t blocks = (int64_t)R * (C / 32);
//             const int waves = PH < 8 ? PH : 8;
//             if (PH <= 8)
//                 hipLaunchKernelGGL((roi_align_fpn_nhwc_xslice2_kernel<2, 32>),
//                                    dim3((unsigned)blocks), dim3(64 * waves), 0, s, fa, C, rois,
//                                    lvl, order, PH, out);
//             else
//                 hipLaunchKernelGGL((roi_align_fpn_nhwc_xslice2_kernel<2, 64>),
//                                    dim3((unsigned)blocks), dim3(64 * waves), 0, s, fa, C, rois,
//                                    lvl, order, PH, out);
//             return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
//         }

// --------------------------------------------------------------------------
// XCD channel-sliced separable forward, one workgroup per (RoI, slice) with
// one wave per output row.  Keeping ~P waves per RoI keeps the number of RoIs
// an XCD has in flight at what the full-pixel kernel has (~128), while the
// bytes each RoI pulls into that XCD's L2 shrink 8x: the in-flight footprint
// window (~3 MB of 128-B pixel slices) fits the 4 MiB L2, so overlapping RoIs
// re-read from L2 instead of the fabric.  Per output row the wave
//   1. loads its tap columns 8 at a time (lane group g = column slot, lane
//      q = channel quad): one 1 KiB instruction = 8 pixel slices of one tap
//      row; the vertical combine V(x) = sum_k w_k F(row_k, x) is lane-local;
//   2. parks V in LDS (wave-private), then lane group g computes bin pw = g
//      (g + 8 ...) from V(xl), V(xh) of its samples and stores 128 B.
// Column slots: the contiguous range [xmin, xmax] of tap columns when it fits
// NS slots (every RoI with sample spacing <= 1 px), else one slot per tap
// (2 P SR <= NS).  Arithmetic order as roi_align_fpn_nhwc_sep_kernel.
// Measured (variant 16, profiles/r01_roialign_pmc/xslice_v16.txt): fabric reads
// drop to 642 MB per launch (= the compulsory 0.66 GB; variant 8 reads 1.17 GB)
// and the L2 hit rate rises 0.54 -> 0.69, but the kernel runs 8x the waves
// with the per-RoI prologue replicated per slice: 2.7x the VALU instructions
// of variant 8, VALU-issue bound at ~510 us vs 306 us.  Kept as the record of
// the locality experiment (and its persistent / slice-per-row-group cousins,
// both slower); variant 8 stays the product kernel.
// --------------------------------------------------------------------------
struct SampleX {
    int xl, xh;
    float lx;
    bool ok;
};

template <int SR>
__device__ __forceinline__ SampleX sample_x(const RoiGeom &g, int j) {
    const int pw = j / SR, ix = j - (j / SR) * SR;
    float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
    SampleX sx;
    sx.ok = !(x < -1.0f || x > (float)g.W);
    if (x <= 0) x = 0;
    int xl = (int)x, xh;
    if (xl >= g.W - 1) { xh = xl = g.W - 1; x = (float)xl; } else xh = xl + 1;
    sx.xl = xl;
    sx.xh = xh;
    sx.lx = x - xl;
    return sx;
}

template <int SR, int NS>
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_xslice2_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, float *__restrict__ out) {
    __shared__ float4 vcol[8][NS][8];  // [wave][column slot][channel quad]
    const int S = C >> 5;
    const int s = blockIdx.x % S;
    const int i = blockIdx.x / S;
    int r = roi_order ? roi_order[i] : i;
    r = __builtin_amdgcn_readfirstlane(r);
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
    const int lane = lane_id(), wv = wave_id();
    const int grp = lane >> 3, q = lane & 7;
    const int c0 = s * 32 + q * 4;
    const float *base = g.feat + c0;
    const int64_t rowstride = (int64_t)g.W * C;
    const float inv = 1.f / g.count;
    const int nsamp = P * SR;
    // valid samples are a contiguous run [j0, j1] (x increases with j)
    int j0 = 0, j1 = nsamp - 1;
    while (j0 < nsamp && !sample_x<SR>(g, j0).ok) ++j0;
    while (j1 >= j0 && !sample_x<SR>(g, j1).ok) --j1;
    int xmin = 0, nslot = 0;
    bool contiguous = true;
    if (j0 <= j1) {
        xmin = sample_x<SR>(g, j0).xl;
        const int span = sample_x<SR>(g, j1).xh - xmin + 1;
        contiguous = span <= NS;
        nslot = contiguous ? span : 2 * nsamp;
    }
    float4 *vw = &vcol[wv][0][0];
    for (int ph = wv; ph < P; ph += num_waves()) {
        const RowTaps<SR> taps = row_taps<SR>(g, ph);
        for (int c8 = 0; c8 < nslot; c8 += 8) {
            const int slot = c8 + grp;
            int col;
            if (contiguous) {
                col = xmin + slot;
            } else {
                const SampleX sx = sample_x<SR>(g, min(slot >> 1, nsamp - 1));
                col = (slot & 1) ? sx.xh : sx.xl;
            }
            col = min(col, g.W - 1);
            const bool ok = slot < nslot;
            const float *p = base + (int64_t)col * C;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int k = 0; k < 2 * SR; ++k)
                if (taps.alive[k] && ok) {
                    const float4 f = ld4(p + taps.row[k] * rowstride);
                    v.x += taps.w[k] * f.x;
                    v.y += taps.w[k] * f.y;
                    v.z += taps.w[k] * f.z;
                    v.w += taps.w[k] * f.w;
                }
            vw[slot * 8 + q] = v;
        }
        __builtin_amdgcn_wave_barrier();
        for (int pw = grp; pw < P; pw += 8) {
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int ix = 0; ix < SR; ++ix) {
                const int j = pw * SR + ix;
                const SampleX sx = sample_x<SR>(g, j);
                if (!sx.ok) continue;
                const int sa = contiguous ? sx.xl - xmin : 2 * j;
                const int sb = contiguous ? sx.xh - xmin : 2 * j + 1;
                const float4 va = vw[sa * 8 + q], vb = vw[sb * 8 + q];
                const float lx = sx.lx, hx = 1.f - lx;
                acc.x += hx * va.x + lx * vb.x;
                acc.y += hx * va.y + lx * vb.y;
                acc.z += hx * va.z + lx * vb.z;
                acc.w += hx * va.w + lx * vb.w;
            }
            *reinterpret_cast<float4 *>(out + (((int64_t)r * P + ph) * P + pw) * C + c0) =
                make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Speed-of-light probe (variant 30, measurement only -- NOT RoIAlign): the same
// grid, block shape, RoI order and output writes as the separable kernel, but
// each RoI reads its compulsory footprint (the SURVEY 8d rectangle of level
// pixels) exactly once, one row per wave, with no sampling arithmetic.  Its time
// is what any kernel that fetches per RoI pays for the memory traffic alone.
__global__ __launch_bounds__(512) void roi_footprint_probe_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, float *__restrict__ out) {
    const int r = roi_order ? roi_order[blockIdx.x] : (int)blockIdx.x;
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const float *roi = rois + (int64_t)r * 5;
    const int H = fa.H[li], W = fa.W[li];
    const float s = fa.scale[li];
    const float *feat = fa.feat[li] + (int64_t)(int)roi[0] * H * W * C;
    const float x1 = roi[1] * s, y1 = roi[2] * s, x2 = roi[3] * s, y2 = roi[4] * s;
    const int xa = max((int)floorf(x1), 0), xb = min((int)floorf(fmaxf(x2, x1 + 1.f)) + 1, W - 1);
    const int ya = max((int)floorf(y1), 0), yb = min((int)floorf(fmaxf(y2, y1 + 1.f)) + 1, H - 1);
    const int lane = lane_id();
    for (int c0 = 0; c0 < C; c0 += 256) {
        const int c = c0 + lane * 4;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int y = ya + wave_id(); y <= yb; y += num_waves())
            for (int x = xa; x <= xb; ++x) {
                const float4 v = ld4(feat + ((int64_t)y * W + x) * C + c);
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            }
        for (int ph = wave_id(); ph < P; ph += num_waves())
            for (int pw = 0; pw < P; ++pw) {
                vf4 v = {acc.x, acc.y, acc.z, acc.w};
                __builtin_nontemporal_store(
                    v, reinterpret_cast<vf4 *>(out + (((int64_t)r * P + ph) * P + pw) * C + c));
            }
    }
}



// ==========================================================================
// Round 2, variant 40b (profiles/r02_roialign/README.md): XCD channel slices,
// lane group = tap column, LDS row exchange.  436 us vs 300 us for variant 8.
// Launched as: blocks = ceil(R / 4) * (C / 32), 256 threads, roi_order =
// xcd_roi_order(n_xcd=1).
// ==========================================================================
// --------------------------------------------------------------------------
// XCD-sliced separable forward (variant 40).  Channel slice s (32 channels =
// 128 B of every pyramid pixel) of every RoI runs on XCD s: block b takes slice
// b % 8, which the round-robin dispatch places on XCD b % 8, so an XCD's 4 MiB
// L2 only caches 1/8 of each pixel and the footprints of the RoIs it has in
// flight (spatially sorted, xcd_roi_order with n_xcd = 1) fit in it: the 4.5x
// inter-RoI footprint overlap is served from L2 and the fabric moves about the
// compulsory bytes (variant 8 re-fetches ~1.6x of them).
// One wave owns one (RoI, slice) and walks the P output rows.  Per row it loads
// the RoI's tap columns [xmin, xmax] eight at a time -- lane group g = lane / 8
// holds column xmin + 8c + g, lane q = lane % 8 four channels, so one 1 KiB wave
// load fetches eight pixel slices and every pixel slice is fetched once per row
// (the separable kernel's sliding-window count) -- and combines the live tap
// rows into V(x) = sum_k w_k F(row_k, x) in registers.  V goes to a
// wave-private LDS row; then lane group g computes bin pw = g (+8, ...) as
// acc += hx V(xl) + lx V(xh) per sample.  Same arithmetic, same order as
// roi_align_fpn_nhwc_sep_kernel: bit-identical outputs.
// --------------------------------------------------------------------------
static constexpr int kXcdMaxSpan = 64;  // tap columns per RoI row held in LDS

template <int SR>
__global__ __launch_bounds__(256) void roi_align_fpn_nhwc_xcd_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, int nslice, float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) float4 vrow[4][kXcdMaxSpan][8];
    const int s = blockIdx.x % nslice;
    const int wv = wave_id();
    const int i = (blockIdx.x / nslice) * num_waves() + wv;
    if (i >= fa.R) return;  // wave-uniform; no block-wide barrier below
    int r = roi_order ? roi_order[i] : i;
    r = __builtin_amdgcn_readfirstlane(r);
    if (r < 0 || r >= fa.R) return;
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
    const int lane = lane_id();
    const int grp = lane >> 3, q = lane & 7;
    const int c0 = s * 32 + q * 4;
    const float *base = g.feat + c0;
    const int W = g.W;
    const int64_t rowstride = (int64_t)W * C;
    const float inv = 1.f / g.count;
    // tap-column range of the valid samples (x grows with the sample index)
    int xmin = 1 << 30, xmax = -1;
    for (int j = 0; j < P * SR; ++j) {
        const int pw = j / SR, ix = j - pw * SR;
        float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
        if (x < -1.0f || x > (float)W) continue;
        if (x <= 0) x = 0;
        int a = (int)x, b;
        if (a >= W - 1) { b = a = W - 1; } else b = a + 1;
        xmin = min(xmin, a);
        xmax = max(xmax, b);
    }
    const int span = xmax >= xmin ? xmax - xmin + 1 : 0;
    if (span > kXcdMaxSpan) {
        // RoIs wider than the LDS row (extreme aspect ratios): each lane group
        // fetches its own bin's tap columns straight from memory (same order)
        for (int ph = 0; ph < P; ++ph) {
            const RowTaps<SR> taps = row_taps<SR>(g, ph);
            for (int pw = grp; pw < P; pw += 8) {
                auto column = [&](int x) -> float4 {
                    return combine_column<SR>(
                        taps, load_column<SR>(taps, base, rowstride, (int64_t)x * C));
                };
                int cl = -1, ch = -1;
                float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va, acc = va;
#pragma unroll
                for (int ix = 0; ix < SR; ++ix) {
                    float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
                    if (x < -1.0f || x > (float)W) continue;
                    if (x <= 0) x = 0;
                    int xl = (int)x, xh;
                    if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
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
                vf4 o = {acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv};
                __builtin_nontemporal_store(
                    o, reinterpret_cast<vf4 *>(out + (((int64_t)r * P + ph) * P + pw) * C + c0));
            }
        }
        return;
    }
    const int nchunk = (span + 7) >> 3;
    float4(*vw)[8] = vrow[wv];
    for (int ph = 0; ph < P; ++ph) {
        const RowTaps<SR> taps = row_taps<SR>(g, ph);
        for (int c = 0; c < nchunk; ++c) {
            const int col = xmin + c * 8 + grp;
            const bool in = col <= xmax;
            const float *p = base + (int64_t)(in ? col : xmin) * C;
            float4 f[2 * SR];
#pragma unroll
            for (int k = 0; k < 2 * SR; ++k)
                if (taps.alive[k]) f[k] = ld4(p + taps.row[k] * rowstride);
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int k = 0; k < 2 * SR; ++k)
                if (taps.alive[k]) {
                    v.x += taps.w[k] * f[k].x;
                    v.y += taps.w[k] * f[k].y;
                    v.z += taps.w[k] * f[k].z;
                    v.w += taps.w[k] * f[k].w;
                }
            vw[c * 8 + grp][q] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int pw = grp; pw < P; pw += 8) {
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int ix = 0; ix < SR; ++ix) {
                float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
                if (x < -1.0f || x > (float)W) continue;
                if (x <= 0) x = 0;
                int xl = (int)x, xh;
                if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
                const float lx = x - xl, hx = 1.f - lx;
                const float4 va = vw[xl - xmin][q], vb = vw[xh - xmin][q];
                acc.x += hx * va.x + lx * vb.x;
                acc.y += hx * va.y + lx * vb.y;
                acc.z += hx * va.z + lx * vb.z;
                acc.w += hx * va.w + lx * vb.w;
            }
            vf4 o = {acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv};
            __builtin_nontemporal_store(
                o, reinterpret_cast<vf4 *>(out + (((int64_t)r * P + ph) * P + pw) * C + c0));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

