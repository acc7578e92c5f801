// Round-4 RoIAlign experiments, kept for the record (NOT built into libvosdet.so;
// measurements: profiles/r04/roialign/README.md).  These were kernels of
// vosdetectron_amd/csrc/roi_align.hip (same includes / helpers: roi_geom.hpp,
// sep_row_sweep, store_bin) selected by VOSDET_ROIALIGN_VARIANT 12 / 14 / 16:
//  12 / 14  channel-pinned separable sweep (G = 2 / 4 XCD groups, G adjacent
//           columns per 1 KiB wave load): 340 / 476 us vs 289-293 us (variant 10)
//  16       variant 10 in frame-window order + prefetch blocks streaming the next
//           frame's pyramid into the Infinity Cache: 756-2945 us (stride 8..32);
//           frame-window order alone 321-326 us
//  18       variant 10 + one TOUCH wave per block loading one dword per 128-B line of
//           the footprint of the RoI its XCD runs `ahead` positions later: 417-494 us
//           (ahead 16..256) vs 293 us -- the eighth wave per block costs occupancy
// Channel-pinned separable NHWC forward (variants 12: G = 2, 14: G = 4), C = 256.
// The 8 XCDs form G groups of 8 / G; group g computes channels [g * 256 / G,
// (g + 1) * 256 / G) of EVERY RoI, so a pixel's line set is split over the groups
// and each XCD's 4 MiB L2 holds 1 / G of every pixel it touches -- G times the
// spatial reach before overlapping RoIs' re-reads miss to the fabric
// (tools/research/ra_l2_sim.py: misses 1.97x -> 1.40x / 1.05x the compulsory
// pixels for G = 2 / 4 at 128 resident RoIs per XCD).  A wave still moves 1 KiB
// per load: its G lane sub-groups (64 / G lanes, 4 channels each) take G
// ADJACENT columns, so the separable sweep advances G columns per load; each
// sub-group accumulates the weighted columns it holds and the G partial sums of
// a bin are added across sub-groups (v_permlane16/32_swap) when the bin
// completes.  Sub-group s stores bin (G-bin block + s): one store instruction
// per G bins.  Same sample geometry as variant 10; sums re-associated (1e-4).
template <int G>
__device__ __forceinline__ float4 pin_reduce(float4 v) {
    float4 r = v;
#define VD_SWAP(F, x)                                                                        \
    {                                                                                        \
        auto t_ = F(__float_as_uint(x), __float_as_uint(x), false, false);                   \
        x = __uint_as_float(t_[0]) + __uint_as_float(t_[1]);                                 \
    }
    if (G == 4) {
        VD_SWAP(__builtin_amdgcn_permlane16_swap, r.x)
        VD_SWAP(__builtin_amdgcn_permlane16_swap, r.y)
        VD_SWAP(__builtin_amdgcn_permlane16_swap, r.z)
        VD_SWAP(__builtin_amdgcn_permlane16_swap, r.w)
    }
    VD_SWAP(__builtin_amdgcn_permlane32_swap, r.x)
    VD_SWAP(__builtin_amdgcn_permlane32_swap, r.y)
    VD_SWAP(__builtin_amdgcn_permlane32_swap, r.z)
    VD_SWAP(__builtin_amdgcn_permlane32_swap, r.w)
#undef VD_SWAP
    return r;
}

template <int G>
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_pin_kernel(
    FpnLevels fa, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, float *__restrict__ out) {
    constexpr int C = 256, NX = 8 / G, LG = 64 / G;
    const int b = blockIdx.x, xcd = b & 7;
    const int grp = xcd / NX;
    const int ig = (b >> 3) * NX + xcd % NX;  // position in this group's RoI order
    if (ig >= fa.R) return;
    const int r = roi_order ? roi_order[ig] : ig;
    if (r < 0 || r >= fa.R) return;  // malformed schedule entry: write nothing
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, 2);
    const int ph = wave_id();
    if (ph >= P) return;
    const int lane = lane_id();
    const int sub = lane / LG;                         // column within a G-column block
    const int c0 = grp * (C / G) + (lane % LG) * 4;   // this lane's 4 channels
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(g.feat), (short)0, g.H * g.W * C * 4, 0x00020000);
    const int rowbytes = g.W * C * 4, colbytes = C * 4;
    const int voff = c0 * 4 + sub * colbytes;
    const RowTaps<2> taps = row_taps<2>(g, ph);
    int rowoff[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) rowoff[k] = __builtin_amdgcn_readfirstlane(taps.row[k] * rowbytes);
    auto block_v = [&](int p) -> float4 {  // V(column G p + sub) for this lane's channels
        const int xo = __builtin_amdgcn_readfirstlane(p * G * colbytes);
        TapCol<2> c;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (taps.alive[k])
                c.f[k] = __builtin_bit_cast(
                    float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, rowoff[k] + xo, 0));
        return combine_column<2>(taps, c);
    };
    float *orow = out + (((int64_t)r * P + ph) * P) * C + c0;
    const int W = g.W;
    int pa = -1;
    bool vb_ok = false;
    float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va, mine = va;
    for (int pw = 0; pw < P; ++pw) {
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int ix = 0; ix < 2; ++ix) {
            float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / 2;
            if (x < -1.0f || x > (float)W) continue;  // wave-uniform
            if (x <= 0) x = 0;
            int xl = (int)x, xh;
            if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
            const float lx = x - xl, hx = 1.f - lx;
            const int pl = xl / G, pr = xh / G;
            if (pl != pa) {
                if (vb_ok && pl == pa + 1) va = vb;
                else va = block_v(pl);
                pa = pl;
                vb_ok = false;
            }
            if (pr != pa && !vb_ok) {
                vb = block_v(pa + 1);
                vb_ok = true;
            }
            const int cl = G * pa + sub;
            // selects, not products with a zero weight: a column past the map edge
            // holds another pixel's (finite or not) values and must not enter
            const float4 t0 = make_float4(hx * va.x, hx * va.y, hx * va.z, hx * va.w);
            const float4 t1 = make_float4(lx * va.x, lx * va.y, lx * va.z, lx * va.w);
            const float4 t2 = make_float4(lx * vb.x, lx * vb.y, lx * vb.z, lx * vb.w);
            if (cl == xl) { acc.x += t0.x; acc.y += t0.y; acc.z += t0.z; acc.w += t0.w; }
            if (cl == xh) { acc.x += t1.x; acc.y += t1.y; acc.z += t1.z; acc.w += t1.w; }
            if (cl + G == xh) { acc.x += t2.x; acc.y += t2.y; acc.z += t2.z; acc.w += t2.w; }
        }
        const float4 tot = pin_reduce<G>(acc);
        if (sub == pw % G) mine = make_float4(tot.x * .25f, tot.y * .25f, tot.z * .25f, tot.w * .25f);
        if (pw % G == G - 1 || pw == P - 1) {
            const int pw0 = pw - pw % G;
            if (sub <= pw % G) store_bin<true>(orow + (int64_t)(pw0 + sub) * C, mine);
        }
    }
}

// Variant 16 (experiment): variant 10's default launch in frame-window order
// (all XCDs on one frame at a time: xcd_roi_order(window = RoIs per frame)) with
// one PREFETCH block every `stride` blocks streaming the NEXT frame's pyramid
// from HBM into the Infinity Cache / L2 (LDS-DMA into a scratch line of LDS, the
// data discarded), so the compute blocks' first-touch misses are cache hits
// (tools/research/ra_floor_probe.py: 299 us with the pyramid in HBM, 191 us
// with it cache-resident, same kernel and wave loads).
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_pf_kernel(
    FpnLevels fa, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, int stride, int n_pf, float *__restrict__ out) {
    constexpr int C = 256;
    __shared__ __attribute__((aligned(1024))) char scratch[8 * 1024];
    const int b = blockIdx.x;
    if (b % stride == stride - 1) {  // prefetch block k of n_pf
        const int k = b / stride;
        int64_t fbytes = 0;
        for (int l = 0; l < fa.L; ++l) fbytes += (int64_t)fa.H[l] * fa.W[l] * C * 4;
        const int64_t total = (int64_t)(fa.B - 1) * fbytes;  // frames 1 .. B-1
        if (total <= 0) return;
        const int64_t u0 = (total / 1024) * k / n_pf, u1 = (total / 1024) * (k + 1) / n_pf;
        const int w = __builtin_amdgcn_readfirstlane(wave_id()), nw = num_waves();
        const uint32_t lds = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)scratch + (uint32_t)(w & 7) * 1024u);
        int n = 0;
        for (int64_t u = u0 + w; u < u1; u += nw) {
            int64_t off = u * 1024;
            const int f = 1 + (int)(off / fbytes);
            int64_t rem = off - (int64_t)(f - 1) * fbytes;
            int l = 0;
            while (l + 1 < fa.L && rem >= (int64_t)fa.H[l] * fa.W[l] * C * 4) {
                rem -= (int64_t)fa.H[l] * fa.W[l] * C * 4;
                ++l;
            }
            // wave-uniform: w came through readfirstlane, everything else is uniform
            const char *src = reinterpret_cast<const char *>(fa.feat[l]) +
                              (int64_t)f * fa.H[l] * fa.W[l] * C * 4 + rem;
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\t"
                "s_mov_b32 m0, %3\n\t"
                "s_nop 0\n\t"
                "global_load_lds_dwordx4 %1, %2\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"((uint32_t)lane_id() * 16u), "s"(src), "s"(lds)
                : "memory");
            if (++n == 16) {  // at most 16 KiB in flight per wave
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                n = 8;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // before the LDS is released
        return;
    }
    const int p = (b / stride) * (stride - 1) + b % stride;
    if (p >= fa.R) return;
    const int r = roi_order ? roi_order[p] : p;
    if (r < 0 || r >= fa.R) return;
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, 2);
    const int lane = lane_id();
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(g.feat), (short)0, g.H * g.W * C * 4, 0x00020000);
    const int rowbytes = g.W * C * 4, colbytes = C * 4;
    const int ph = wave_id();
    if (ph >= P) return;
    const int c0 = lane * 4;
    const int voff = c0 * 4;
    const RowTaps<2> taps = row_taps<2>(g, ph);
    int rowoff[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) rowoff[k] = __builtin_amdgcn_readfirstlane(taps.row[k] * rowbytes);
    float *orow = out + (((int64_t)r * P + ph) * P) * C + c0;
    auto column = [&](int x) -> float4 {
        const int xo = __builtin_amdgcn_readfirstlane(x * colbytes);
        TapCol<2> c;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (taps.alive[k])
                c.f[k] = __builtin_bit_cast(
                    float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, rowoff[k] + xo, 0));
        return combine_column<2>(taps, c);
    };
    sep_row_sweep<2>(g, 0, P, column, [&](int pw, float4 acc) {
        store_bin<true>(orow + (int64_t)pw * C, acc);
    });
}


// ---- dispatch (was in launch_roi_align_fpn_nhwc) ----
        if ((variant == 12 || variant == 14) && sr == 2 && PH == PW && C == 256) {
            bool fits = true;  // 32-bit buffer offsets: every image of a level < 2 GiB
            for (int l = 0; l < fa.L; ++l)
                fits &= (int64_t)fa.H[l] * fa.W[l] * C * 4 < (1ll << 31);
            if (fits && PH <= 8) {
                const int G = variant == 12 ? 2 : 4, NX = 8 / G;
                const int nblk = (R + NX - 1) / NX * 8;
                if (G == 2)
                    hipLaunchKernelGGL(roi_align_fpn_nhwc_pin_kernel<2>, dim3(nblk), dim3(64 * PH),
                                       0, s, fa, rois, lvl, order, PH, out);
                else
                    hipLaunchKernelGGL(roi_align_fpn_nhwc_pin_kernel<4>, dim3(nblk), dim3(64 * PH),
                                       0, s, fa, rois, lvl, order, PH, out);
                return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
            }
        }
        if (variant == 16 && sr == 2 && PH == PW && C == 256 && PH <= 8) {
            bool fits = true;
            for (int l = 0; l < fa.L; ++l)
                fits &= (int64_t)fa.H[l] * fa.W[l] * C * 4 < (1ll << 31);
            if (fits) {
                const char *e = getenv("VOSDET_RA_PF_STRIDE");
                int stride = e ? atoi(e) : 16;
                if (stride < 2) stride = 2;
                const int nblk = (R + stride - 2) / (stride - 1) * stride;
                hipLaunchKernelGGL(roi_align_fpn_nhwc_pf_kernel, dim3(nblk), dim3(64 * PH), 0, s,
                                   fa, rois, lvl, order, PH, stride, nblk / stride, out);
                return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
            }
        }

// ===================== variant 18: touch wave =====================
__device__ float g_touch_sink;

// TOUCH (experiment, variant 18): one extra wave per block that touches every
// 128-B line of the footprint of the RoI its XCD will run `ahead` schedule
// positions later (blocks b and b + 8 ahead run on the same XCD, its slice of
// the dealt order), so that RoI's first-touch misses are taken by a wave nobody
// waits on and its compute waves hit the Infinity Cache / L2
// (profiles/r04/roialign: 299 us with the pyramid in HBM, 191 us cache-resident).
__device__ __forceinline__ void touch_roi(const FpnLevels &fa, int C, const float *roi, int li,
                                          int P) {
    const RoiGeom g = roi_geom(fa, C, roi, li, P, P, 2);
    const int y0 = max(0, (int)floorf(g.sh)), x0 = max(0, (int)floorf(g.sw));
    const int y1 = min(g.H - 1, (int)floorf(g.sh + g.bh * P) + 1);
    const int x1 = min(g.W - 1, (int)floorf(g.sw + g.bw * P) + 1);
    if (y1 < y0 || x1 < x0 || g.sh < -1e29f) return;
    const int nx = x1 - x0 + 1, np = (y1 - y0 + 1) * nx;
    const int lines = C / 32;  // 128-B lines per pixel
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(g.feat), (short)0, g.H * g.W * C * 4, 0x00020000);
    const int lane = lane_id(), total = np * lines;
    float sum = 0.f;
    for (int t0 = 0; t0 < total; t0 += 64 * 8) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int t = t0 + i * 64 + lane;
            const int pix = t / lines, ln = t - (t / lines) * lines;
            const int yy = y0 + pix / nx, xx = x0 + pix - (pix / nx) * nx;
            const int voff = t < total ? ((yy * g.W + xx) * C + ln * 32) * 4 : 0x7ffffff0;
            v[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) sum += v[i];
    }
    if (__float_as_uint(sum) == 0x7fbadbadu) g_touch_sink = sum;  // keeps the loads alive
}


// ---- in the kernel, before the RoI geometry ----
    if (TOUCH && wave_id() == P) {
        const int pt = p + 8 * ahead;
        if (pt < fa.R) {
            const int rt = roi_order ? roi_order[pt] : pt;
            if (rt >= 0 && rt < fa.R) {
                const int lt = __builtin_amdgcn_readfirstlane(roi_level ? roi_level[rt] : 0);
                if (lt >= 0 && lt < fa.L) touch_roi(fa, C, rois + (int64_t)rt * 5, lt, P);
            }
        }
        return;
    }

// ---- launch ----
    const char *et = getenv("VOSDET_RA_TOUCH_AHEAD");  // variant 18 (experiment)
    if (roialign_variant() == 18 && segs == 1 && parts == 1 && C <= 256 && P <= 8)
        hipLaunchKernelGGL((roi_align_fpn_nhwc_sep_buf_kernel<2, true, true, true>), dim3(nblk),
                           dim3(64 * (P + 1)), 0, s, fa, C, rois, lvl, order, P, 1, 1, out,
                           et ? atoi(et) : 64);
