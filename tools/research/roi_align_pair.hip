// Round 2, variant 11 (profiles/r02_roialign/README.md): the buffer-load
// separable kernel with one wave sweeping two adjacent output rows and the
// second row's duplicate tap rows taken from the first row's registers.
// Bit-identical to the product kernel; 10% fewer wave loads (2.69 M vs
// 3.00 M) but 110 VGPRs (4 waves/SIMD) and 83 M VALU: 299 us vs 295 us.
// NOT part of libvosdet.so; it compiled inside roi_align.hip next to
// roi_align_fpn_nhwc_sep_buf_kernel.

// Row-pair form of the buffer-load kernel (variant 11): one wave sweeps two
// adjacent output rows a, b.  Their x samples -- and so the column sequence
// and the (cl, ch) reuse -- are identical, and b's first tap rows are usually
// a's last ones.  Tap slots 0..3 are a's merged taps, 4..7 b's; a b tap whose
// row a already has is not loaded: its weight moves onto a's slot.  b's taps
// are increasing in row and its duplicates are its lowest rows, so summing
// b's weights over slots 0..3 then 4..7 is b's own k order: both rows' V(x)
// are bit-identical to combine_column (variants 8 / 10), with ~25% fewer
// 1 KiB wave loads and the x geometry computed once per pair.
template <int SR, bool NT>
__global__ __launch_bounds__(512) void roi_align_fpn_nhwc_sep_pair_kernel(
    FpnLevels fa, int C, const float *__restrict__ rois, const int *__restrict__ roi_level,
    const int *__restrict__ roi_order, int P, float *__restrict__ out) {
    constexpr int T = 2 * SR;
    const int r = roi_order ? roi_order[blockIdx.x] : (int)blockIdx.x;
    if (r < 0 || r >= fa.R) return;  // malformed schedule entry: write nothing
    int li = roi_level ? roi_level[r] : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const RoiGeom g = roi_geom(fa, C, rois + (int64_t)r * 5, li, P, P, SR);
    const int chunks = (C + 255) / 256;
    const int pairs = (P + 1) / 2;
    const int lane = lane_id();
    const int W = g.W;
    const float inv = 1.f / g.count;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(g.feat), (short)0, g.H * g.W * C * 4, 0x00020000);
    const int rowbytes = g.W * C * 4, colbytes = C * 4;
    for (int u = wave_id(); u < pairs * chunks; u += num_waves()) {
        const int pr = u / chunks;
        const int ck = u - pr * chunks;
        const int c0 = ck * 256 + lane * 4;
        const bool active = c0 < C;
        const int voff = (active ? c0 : 0) * 4;
        const int pa = 2 * pr, pb = pa + 1;
        const bool has_b = pb < P;
        const RowTaps<SR> ta = row_taps<SR>(g, pa);
        const RowTaps<SR> tb = row_taps<SR>(g, has_b ? pb : pa);
        float wdup[T];     // b's weight on a's slot k (b tap merged onto a's row)
        bool dup_on[T];    // slot k carries a b weight
        bool own[T];       // b tap k loaded into its own slot
        int offa[T], offb[T];
#pragma unroll
        for (int k = 0; k < T; ++k) {
            wdup[k] = 0.f;
            dup_on[k] = false;
        }
#pragma unroll
        for (int k = 0; k < T; ++k) {
            bool d = false;
#pragma unroll
            for (int i = 0; i < T; ++i)
                if (has_b && tb.alive[k] && ta.alive[i] && ta.row[i] == tb.row[k]) {
                    wdup[i] = tb.w[k];
                    dup_on[i] = true;
                    d = true;
                }
            own[k] = has_b && tb.alive[k] && !d;
            offa[k] = __builtin_amdgcn_readfirstlane(ta.row[k] * rowbytes);
            offb[k] = __builtin_amdgcn_readfirstlane(tb.row[k] * rowbytes);
        }
        float *orow_a = out + (((int64_t)r * P + pa) * P) * C + c0;
        float *orow_b = orow_a + (int64_t)P * C;
        auto column = [&](int x, float4 &vb_out) -> float4 {
            const int xo = __builtin_amdgcn_readfirstlane(x * colbytes);
            float4 f[2 * T];
#pragma unroll
            for (int k = 0; k < T; ++k) {
                if (ta.alive[k])
                    f[k] = __builtin_bit_cast(
                        float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, offa[k] + xo, 0));
                if (own[k])
                    f[T + k] = __builtin_bit_cast(
                        float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, offb[k] + xo, 0));
            }
            float4 va_ = make_float4(0.f, 0.f, 0.f, 0.f), vb_ = va_;
#pragma unroll
            for (int k = 0; k < T; ++k)
                if (ta.alive[k]) {
                    va_.x += ta.w[k] * f[k].x;
                    va_.y += ta.w[k] * f[k].y;
                    va_.z += ta.w[k] * f[k].z;
                    va_.w += ta.w[k] * f[k].w;
                }
#pragma unroll
            for (int k = 0; k < T; ++k)
                if (dup_on[k]) {
                    vb_.x += wdup[k] * f[k].x;
                    vb_.y += wdup[k] * f[k].y;
                    vb_.z += wdup[k] * f[k].z;
                    vb_.w += wdup[k] * f[k].w;
                }
#pragma unroll
            for (int k = 0; k < T; ++k)
                if (own[k]) {
                    vb_.x += tb.w[k] * f[T + k].x;
                    vb_.y += tb.w[k] * f[T + k].y;
                    vb_.z += tb.w[k] * f[T + k].z;
                    vb_.w += tb.w[k] * f[T + k].w;
                }
            vb_out = vb_;
            return va_;
        };
        int cl = -1, ch = -1;
        float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        float4 va = z, vb = z, wa = z, wb = z;  // v*: row a, w*: row b
        for (int pw = 0; pw < P; ++pw) {
            float4 acc = z, acc2 = z;
#pragma unroll
            for (int ix = 0; ix < SR; ++ix) {
                float x = g.sw + pw * g.bw + (ix + .5f) * g.bw / SR;
                if (x < -1.0f || x > (float)W) continue;  // wave-uniform
                if (x <= 0) x = 0;
                int xl = (int)x, xh;
                if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
                const float lx = x - xl, hx = 1.f - lx;
                if (xl != cl || xh != ch) {
                    if (xl == ch) {
                        va = vb;
                        wa = wb;
                    } else {
                        va = column(xl, wa);
                    }
                    if (xh == xl) {
                        vb = va;
                        wb = wa;
                    } else {
                        vb = column(xh, wb);
                    }
                    cl = xl;
                    ch = xh;
                }
                acc.x += hx * va.x + lx * vb.x;
                acc.y += hx * va.y + lx * vb.y;
                acc.z += hx * va.z + lx * vb.z;
                acc.w += hx * va.w + lx * vb.w;
                acc2.x += hx * wa.x + lx * wb.x;
                acc2.y += hx * wa.y + lx * wb.y;
                acc2.z += hx * wa.z + lx * wb.z;
                acc2.w += hx * wa.w + lx * wb.w;
            }
            if (active) {
                store_bin<NT>(orow_a + (int64_t)pw * C,
                              make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv));
                if (has_b)
                    store_bin<NT>(orow_b + (int64_t)pw * C, make_float4(acc2.x * inv, acc2.y * inv,
                                                                        acc2.z * inv, acc2.w * inv));
            }
        }
    }
}

static int launch_sep_pair(const FpnLevels &fa, int C, const float *rois, const int *lvl,
                           const int *order, int R, int P, float *out, hipStream_t s) {
    for (int l = 0; l < fa.L; ++l)  // 32-bit buffer offsets: every image of a level < 2 GiB
        if ((int64_t)fa.H[l] * fa.W[l] * C * 4 >= (1ll << 31)) return VD_ERR_SHAPE;
    int waves = ((P + 1) / 2) * ((C + 255) / 256);
    if (waves > 8) waves = 8;
    hipLaunchKernelGGL((roi_align_fpn_nhwc_sep_pair_kernel<2, true>), dim3(R), dim3(64 * waves),
                       0, s, fa, C, rois, lvl, order, P, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

