// Round 2, variant 9 (profiles/r02_roialign/README.md): the separable kernel
// with per-RoI x-sample geometry (lane = output column, read back with
// readlane) and a register ring of column loads meant to keep the next
// columns in flight.  Bit-identical to variant 8 on the GPU tests but slower
// (325-364 us vs 304 us): every step issues all 2*SR tap loads (dead or merged
// taps re-read a live row) so the waits could be counted, and the compiler
// still copies loaded registers across the unrolled ring and drains vmcnt to
// zero -- more wave loads with no overlap gained.  NOT part of libvosdet.so;
// it compiled inside vosdetectron_amd/csrc/roi_align.hip next to
// sep_row_sweep / store_bin.

// Pipelined separable NHWC forward (variant 9): the arithmetic of variant 8
// bin for bin (bit-identical), restructured for the gather's latency.
//  - The x samples are the same for every output row of a RoI: lane pw
//    computes output column pw's SR samples once per RoI (variant 8 recomputes
//    them serially in every row), and the row sweeps read them with readlane.
//  - The distinct columns a row needs form a 64-bit mask relative to the
//    first sample's column; the sweep walks it with the next two columns'
//    tap loads already in flight (a 3-deep register ring, unrolled so nothing
//    is indexed dynamically), instead of loading each column when a sample
//    first asks for it.
// A RoI whose columns span more than 64 level pixels (out of the canonical
// level ranges) sweeps as variant 8.
template <bool NT, int DEPTH>
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_pipe_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, float *__restrict__ out) {
    constexpr int SR = 2;
    const int r = roi_order ? roi_order[blockIdx.x] : (int)blockIdx.x;
    if (r < 0 || r >= fa.R) return;  // malformed schedule entry: write nothing
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
    const int chunks = (C + 255) / 256;
    const int lane = lane_id();
    const int W = g.W;
    const int64_t rowstride = (int64_t)W * C;
    const float inv = 1.f / g.count;
    // x samples of output column pw = lane, exactly as sep_row_sweep computes them
    int sxl[SR], sxh[SR];
    float slx[SR];
    bool sok[SR];
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
        float x = g.sw + lane * g.bw + (ix + .5f) * g.bw / SR;
        sok[ix] = lane < P && !(x < -1.0f || x > (float)W);
        if (x <= 0) x = 0;
        int xl = (int)x, xh;
        if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
        sxl[ix] = xl;
        sxh[ix] = xh;
        slx[ix] = x - xl;
    }
    const uint64_t ok0 = ballot(sok[0]), ok1 = ballot(sok[1]);
    const uint64_t any = ok0 | ok1;
    int xbase = 0;
    uint64_t cols = 0;
    bool fits = true;
    if (any) {  // samples are monotone in (pw, ix): the first live one has the least column
        const int first = __builtin_ctzll(any);
        xbase = __builtin_amdgcn_readlane(sok[0] ? sxl[0] : sxl[1], first);
        uint64_t m = 0;
        bool over = false;
#pragma unroll
        for (int ix = 0; ix < SR; ++ix)
            if (sok[ix]) {
                const int a = sxl[ix] - xbase, b = sxh[ix] - xbase;
                if (b >= 64) over = true;
                else m |= (1ull << a) | (1ull << b);
            }
        fits = ballot(over) == 0;
        for (int o = 32; o > 0; o >>= 1) m |= __shfl_xor(m, o);
        cols = readlane64(m, 0);
    }
    if (!fits) {
        for (int u = wave_id(); u < P * chunks; u += num_waves()) {
            const int ph = u / chunks;
            const int c0 = (u - ph * chunks) * 256 + lane * 4;
            const bool active = c0 < C;
            float *orow = out + (((int64_t)r * P + ph) * P) * C + c0;
            sep_row_sweep<SR>(g, row_taps<SR>(g, ph), g.feat + (active ? c0 : 0), rowstride, C, P,
                              [&](int pw, float4 acc) {
                                  if (active) store_bin<NT>(orow + (int64_t)pw * C, acc);
                              });
        }
        return;
    }
    extern __shared__ __attribute__((aligned(16))) float4 rowbufs[];  // [waves][P][64]
    float4 *rowbuf = rowbufs + wave_id() * P * 64 + lane;
    for (int u = wave_id(); u < P * chunks; u += num_waves()) {
        const int ph = u / chunks;
        const int ck = u - ph * chunks;
        const int c0 = ck * 256 + lane * 4;
        const bool active = c0 < C;
        const float *base = g.feat + (active ? c0 : 0);
        const RowTaps<SR> taps = row_taps<SR>(g, ph);
        float *orow = out + (((int64_t)r * P + ph) * P) * C + c0;
        uint64_t gen = cols;
        auto next_col = [&]() -> int {
            if (!gen) return -1;
            const int c = xbase + __builtin_ctzll(gen);
            gen &= gen - 1;
            return c;
        };
        // Every step issues exactly 2*SR loads (dead or merged taps re-read a
        // live row -- every tap row is clamped into the map -- and past the
        // last column the first one is re-read), so the wait before a column's
        // combine is a fixed vmcnt that leaves the younger columns in flight.
        const int x_any = xbase;
        auto load = [&](int x) {
            TapCol<SR> c;
            const int64_t xo = (int64_t)(x < 0 ? x_any : x) * C;
#pragma unroll
            for (int k = 0; k < 2 * SR; ++k) c.f[k] = ld4(base + taps.row[k] * rowstride + xo);
            return c;
        };
        TapCol<SR> ra, rb, rc;
        int ca = next_col(), cb = next_col(), cc = DEPTH > 2 ? next_col() : -1;
        // (sched barriers keep the columns' loads in issue order, so the
        // waits below are per column)
        ra = load(ca);
        __builtin_amdgcn_sched_barrier(0);
        rb = load(cb);
        __builtin_amdgcn_sched_barrier(0);
        if (DEPTH > 2) rc = load(cc);
        __builtin_amdgcn_sched_barrier(0);
        float4 vprev = make_float4(0.f, 0.f, 0.f, 0.f), vcur = vprev, acc = vprev;
        int ccur = -1, s = 0;
        // every sample whose columns are available, in (pw, ix) order
        auto drain = [&]() {
            while (s < SR * P) {
                const int pw = s >> 1, ix = s & 1;
                if ((((ix ? ok1 : ok0) >> pw) & 1) != 0) {
                    const int xh = __builtin_amdgcn_readlane(ix ? sxh[1] : sxh[0], pw);
                    if (xh > ccur) return;
                    const int xl = __builtin_amdgcn_readlane(ix ? sxl[1] : sxl[0], pw);
                    const float lx = __int_as_float(
                        __builtin_amdgcn_readlane(__float_as_int(ix ? slx[1] : slx[0]), pw));
                    const float hx = 1.f - lx;
                    // xl < ccur means xl is the previous distinct column (xh = xl + 1)
                    const float4 va = xl == ccur ? vcur : vprev, vb = vcur;
                    acc.x += hx * va.x + lx * vb.x;
                    acc.y += hx * va.y + lx * vb.y;
                    acc.z += hx * va.z + lx * vb.z;
                    acc.w += hx * va.w + lx * vb.w;
                }
                if (ix == SR - 1) {  // bins wait in LDS: no store between the loads
                    rowbuf[pw * 64] = make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
                    acc = make_float4(0.f, 0.f, 0.f, 0.f);
                }
                ++s;
            }
        };
        drain();  // leading out-of-range samples
        // register ring, unrolled so no column is moved or indexed dynamically:
        // each step waits only for its own column's loads
        auto step = [&](TapCol<SR> &reg, int &cx) -> bool {
            if (cx < 0) return false;
            vprev = vcur;
            vcur = combine_column<SR>(taps, reg);
            ccur = cx;
            cx = next_col();
            __builtin_amdgcn_sched_barrier(0);
            reg = load(cx);
            __builtin_amdgcn_sched_barrier(0);
            drain();
            return true;
        };
        if (DEPTH > 2) {
            while (step(ra, ca) && step(rb, cb) && step(rc, cc)) {
            }
        } else {
            while (step(ra, ca) && step(rb, cb)) {
            }
        }
        ccur = 1 << 30;  // only trailing out-of-range samples remain
        drain();
        if (active)
            for (int pw = 0; pw < P; ++pw) store_bin<NT>(orow + (int64_t)pw * C, rowbuf[pw * 64]);
    }
}


static int launch_pipe(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                       const int *order, int R, int P, float *out, hipStream_t s) {
    const char *e = getenv("VOSDET_RA_PIPE");  // experiment knobs: "<depth><waves>", e.g. 24
    const int depth = e && e[0] == '3' ? 3 : 2;
    int waves = e && e[0] && e[1] ? e[1] - '0' : 4;
    const int units = P * ((C + 255) / 256);
    if (waves > units) waves = units;
    if (waves < 1 || waves > 8) waves = 4;
    const size_t lds = (size_t)waves * P * 64 * 16;
    if (depth == 3)
        hipLaunchKernelGGL((roi_align_fpn_nhwc_pipe_kernel<true, 3>), dim3(R), dim3(64 * waves),
                           lds, s, fa, C, rois, lvl, order, P, out);
    else
        hipLaunchKernelGGL((roi_align_fpn_nhwc_pipe_kernel<true, 2>), dim3(R), dim3(64 * waves),
                           lds, s, fa, C, rois, lvl, order, P, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

