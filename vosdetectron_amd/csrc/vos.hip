// VOS temporal path for gfx950: FlowAlign, GroupNorm (+ fused epilogues) and the
// ConvGRU gate math of Generalized_VOS_RCNN.
//
// Reference:
//   FlowAlign    lib_vos/vos_model/flow_align/src/flow_align_cuda_kernel.cu:15-55 (fwd),
//                :57-117 (bwd); wrapper flow_align_cuda.c:7-44; module
//                modules/flow_align.py:5-37 (conv_flow_downsample + FlowAlignFunction).
//   GroupNorm    torch.nn.GroupNorm as used by ResNet.py basic_gn_stem / bottleneck_gn_transformation
//                / basic_gn_shortcut (:208-345), FPN.py USE_GN (:96-120, :268-274),
//                fast_rcnn_heads.roi_Xconv1fc_gn_head (:228-290),
//                mask_rcnn_heads.mask_rcnn_fcn_head_v1upXconvs_gn (:191-255).
//   ConvGRU      lib_vos/vos_nn/convgrucell.py:73-92 (use_GN branch) and the fusion of
//                vos_model_builder.py:335-345 (blob/2 + bilinear-0.5x(finer)/2).
//
// FlowAlign keeps the reference's arithmetic exactly: float position, float
// ratios, and the reference's mixed float/double tap expression (the `1.`
// literals promote some products to double, others stay float) -- bit-identical
// to the C restatement, which compiles the same expression text.
// GroupNorm statistics are accumulated in double (sum, sum of squares) and the
// normalisation runs in fp32; it matches torch's fp32 GroupNorm to rounding.
#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

static int grid_for(int64_t n, int bs, int cap = 65536) {
    int64_t g = (n + bs - 1) / bs;
    if (g > cap) g = cap;
    return (int)(g < 1 ? 1 : g);
}

// ============================================================ FlowAlign
// out(n,c,h,w) = bilinear sample of feat(n,c) at (h + flow_y, w + flow_x);
// 0 when the position is outside [0, H-1) x [0, W-1) (strict, as the reference).
struct FlowTap {
    bool ok;
    int off;       // (h_start * W + w_start)
    float hr, wr;  // h_ratio, w_ratio
};

__device__ __forceinline__ FlowTap flow_tap(const float *flow, int n, int h, int w, int H, int W) {
    const int64_t HW = (int64_t)H * W;
    const float flo_x = flow[(int64_t)n * HW * 2 + (int64_t)h * W + w];
    const float flo_y = flow[(int64_t)n * HW * 2 + HW + (int64_t)h * W + w];
    const float w_flo = w + flo_x;
    const float h_flo = h + flo_y;
    FlowTap t;
    t.ok = !(h_flo < 0 || h_flo >= H - 1 || w_flo < 0 || w_flo >= W - 1);
    const int h_start = (int)floorf(h_flo);
    const int w_start = (int)floorf(w_flo);
    t.hr = h_flo - (float)h_start;
    t.wr = w_flo - (float)w_start;
    t.off = t.ok ? w_start + W * h_start : 0;
    return t;
}

// The reference expression verbatim (flow_align_cuda_kernel.cu:46-49): C's
// usual conversions make f1, f2 terms double, f3 * hr a float product promoted
// by (1. - wr), and f4 * hr * wr an all-float product -- summed in double.
__device__ __forceinline__ float flow_blend(float f1, float f2, float f3, float f4, float hr,
                                            float wr) {
    return (float)(f1 * (1. - hr) * (1. - wr) + f2 * (1. - hr) * (wr) + f3 * (hr) * (1. - wr) +
                   f4 * (hr) * (wr));
}

// Reference decomposition (NCHW, one lane per output element).
__global__ __launch_bounds__(256) void flow_align_fwd_nchw_kernel(int64_t n_out, int H, int W,
                                                                  int C,
                                                                  const float *__restrict__ feat,
                                                                  const float *__restrict__ flow,
                                                                  float *__restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_out;
         i += (int64_t)blockDim.x * gridDim.x) {
        const int w = (int)(i % W);
        const int h = (int)((i / W) % H);
        const int64_t nc = i / W / H;
        const int n = (int)(nc / C);
        const FlowTap t = flow_tap(flow, n, h, w, H, W);
        if (!t.ok) {
            out[i] = 0.f;
            continue;
        }
        const float *p = feat + nc * H * W + t.off;
        out[i] = flow_blend(p[0], p[1], p[W], p[W + 1], t.hr, t.wr);
    }
}

// NHWC (product layout of the hidden states): one wave per pixel, lane = 4
// channels, the pixel's flow read once; each tap is a coalesced 1 KiB row.
__global__ __launch_bounds__(256) void flow_align_fwd_nhwc_kernel(int B, int H, int W, int C,
                                                                  const float *__restrict__ feat,
                                                                  const float *__restrict__ flow,
                                                                  float *__restrict__ out) {
    const int64_t npix = (int64_t)B * H * W;
    const int C4 = C >> 2;
    for (int64_t pix = (int64_t)blockIdx.x * num_waves() + wave_id(); pix < npix;
         pix += (int64_t)gridDim.x * num_waves()) {
        const int w = (int)(pix % W);
        const int h = (int)((pix / W) % H);
        const int n = (int)(pix / W / H);
        const FlowTap t = flow_tap(flow, n, h, w, H, W);
        float4 *o = reinterpret_cast<float4 *>(out + pix * C);
        const float4 *b = reinterpret_cast<const float4 *>(feat + ((int64_t)n * H * W + t.off) * C);
        const int64_t rs = (int64_t)W * C4;
        for (int c = lane_id(); c < C4; c += VD_WAVE) {
            if (!t.ok) {
                o[c] = make_float4(0.f, 0.f, 0.f, 0.f);
                continue;
            }
            const float4 a = b[c], bb = b[C4 + c], cc = b[rs + c], d = b[rs + C4 + c];
            o[c] = make_float4(flow_blend(a.x, bb.x, cc.x, d.x, t.hr, t.wr),
                               flow_blend(a.y, bb.y, cc.y, d.y, t.hr, t.wr),
                               flow_blend(a.z, bb.z, cc.z, d.z, t.hr, t.wr),
                               flow_blend(a.w, bb.w, cc.w, d.w, t.hr, t.wr));
        }
    }
}

// Backward (training path, reference decomposition): fp32 atomics into the
// zero-filled feature and flow gradients; same double-promoted products.
__global__ __launch_bounds__(256) void flow_align_bwd_nchw_kernel(
    int64_t n_out, int H, int W, int C, const float *__restrict__ top_diff,
    const float *__restrict__ feat, const float *__restrict__ flow, float *__restrict__ feat_diff,
    float *__restrict__ flow_diff) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_out;
         i += (int64_t)blockDim.x * gridDim.x) {
        const int w = (int)(i % W);
        const int h = (int)((i / W) % H);
        const int64_t nc = i / W / H;
        const int n = (int)(nc / C);
        const FlowTap t = flow_tap(flow, n, h, w, H, W);
        if (!t.ok) continue;
        const int64_t HW = (int64_t)H * W;
        const float hr = t.hr, wr = t.wr;  // float, as the reference (promotions matter)
        const float g = top_diff[i];
        float *bd = feat_diff + nc * HW + t.off;
        atomicAdd(bd, (float)(g * (1. - hr) * (1. - wr)));
        atomicAdd(bd + 1, (float)(g * (1. - hr) * (wr)));
        atomicAdd(bd + W, (float)(g * (hr) * (1. - wr)));
        atomicAdd(bd + W + 1, (float)(g * (hr) * (wr)));
        const float *p = feat + nc * HW + t.off;
        const float f1 = p[0], f2 = p[1], f3 = p[W], f4 = p[W + 1];
        const float dx = (float)(-f1 * (1. - hr) + f2 * (1. - hr) - f3 * (hr) + f4 * (hr));
        const float dy = (float)(-f1 * (1. - wr) - f2 * (wr) + f3 * (1. - wr) + f4 * (wr));
        atomicAdd(flow_diff + (int64_t)n * HW * 2 + (int64_t)h * W + w, g * dx);
        atomicAdd(flow_diff + (int64_t)n * HW * 2 + HW + (int64_t)h * W + w, g * dy);
    }
}

int launch_flow_align_fwd(const float *feat, const float *flow, int B, int C, int H, int W,
                          int nhwc, float *out, hipStream_t s) {
    const int64_t n = (int64_t)B * C * H * W;
    if (n == 0) return VD_OK;
    if (nhwc) {
        if (C % 4) return VD_ERR_SHAPE;
        const int64_t npix = (int64_t)B * H * W;
        hipLaunchKernelGGL(flow_align_fwd_nhwc_kernel, dim3(grid_for(npix, 4)), dim3(256), 0, s,
                           B, H, W, C, feat, flow, out);
    } else {
        hipLaunchKernelGGL(flow_align_fwd_nchw_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, n,
                           H, W, C, feat, flow, out);
    }
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int launch_flow_align_bwd(const float *top_diff, const float *feat, const float *flow, int B,
                          int C, int H, int W, float *feat_diff, float *flow_diff,
                          hipStream_t s) {
    const int64_t n = (int64_t)B * C * H * W;
    if (n == 0) return VD_OK;
    hipLaunchKernelGGL(flow_align_bwd_nchw_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, n, H,
                       W, C, top_diff, feat, flow, feat_diff, flow_diff);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// ============================================================ GroupNorm
// Statistics: ws[set][n][g] = {sum, sum of squares} (double) of x (+ x2) over
// the group's C/G channels x H*W pixels.  Up to 3 independent tensors per
// launch (blockIdx.z = set): the ConvGRU's update and reset gates share one.
// NHWC, C % 4 == 0, C <= 1024, G <= 64.  Thread t owns channel quad t % C4 of
// pixels t / C4, t / C4 + ppi, ...; the four lanes of its quad are summed
// separately and folded into their groups at the end, so any C / G works
// (the GN ResNet's 64-channel stages have 2 channels per group).
__global__ __launch_bounds__(256) void gn_stats_nhwc_kernel(GnSets sets, int HW, int C, int G,
                                                            int pix_per_block) {
    __shared__ double red[2][64];  // per group (G <= 64)
    const GnSet st = sets.s[blockIdx.z];
    const int n = blockIdx.y;
    const int C4 = C >> 2;
    const int cg = C / G;
    for (int i = threadIdx.x; i < 2 * 64; i += blockDim.x) red[i / 64][i % 64] = 0.0;
    __syncthreads();
    const int p0 = blockIdx.x * pix_per_block;
    const int p1 = min(p0 + pix_per_block, HW);
    const float4 *x = reinterpret_cast<const float4 *>(st.x) + (int64_t)n * HW * C4;
    const float4 *x2 =
        st.x2 ? reinterpret_cast<const float4 *>(st.x2) + (int64_t)n * HW * C4 : nullptr;
    for (int q0 = 0; q0 < C4; q0 += blockDim.x) {  // C4 > 256: several quad blocks
        const int nq = min(C4 - q0, (int)blockDim.x);
        const int ppi = blockDim.x / nq;  // pixels per block iteration
        const int q = q0 + (int)threadIdx.x % nq;
        if ((int)threadIdx.x >= ppi * nq) continue;
        double s[4] = {0, 0, 0, 0}, ss[4] = {0, 0, 0, 0};
        for (int p = p0 + (int)threadIdx.x / nq; p < p1; p += ppi) {
            float4 v = x[(int64_t)p * C4 + q];
            if (x2) {
                const float4 u = x2[(int64_t)p * C4 + q];
                v.x = v.x + u.x; v.y = v.y + u.y; v.z = v.z + u.z; v.w = v.w + u.w;
            }
            s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
            ss[0] += (double)v.x * v.x; ss[1] += (double)v.y * v.y;
            ss[2] += (double)v.z * v.z; ss[3] += (double)v.w * v.w;
        }
        if (cg % 4 == 0) {
            const int g = (q * 4) / cg;
            atomicAdd(&red[0][g], (s[0] + s[1]) + (s[2] + s[3]));
            atomicAdd(&red[1][g], (ss[0] + ss[1]) + (ss[2] + ss[3]));
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int g = (q * 4 + k) / cg;
                atomicAdd(&red[0][g], s[k]);
                atomicAdd(&red[1][g], ss[k]);
            }
        }
    }
    __syncthreads();
    for (int g = threadIdx.x; g < G; g += blockDim.x) {
        atomicAdd(st.ws + ((int64_t)n * G + g) * 2, red[0][g]);
        atomicAdd(st.ws + ((int64_t)n * G + g) * 2 + 1, red[1][g]);
    }
}

// NCHW (or any layout where a group is one contiguous run of cg * HW floats).
__global__ __launch_bounds__(256) void gn_stats_nchw_kernel(GnSets sets, int HW, int C, int G,
                                                            int chunk) {
    __shared__ double red[2][4];
    const GnSet st = sets.s[blockIdx.z];
    const int ng = blockIdx.y;  // n * G + g
    const int64_t len = (int64_t)(C / G) * HW;
    const int64_t base = (int64_t)ng * len;
    const int64_t i0 = (int64_t)blockIdx.x * chunk;
    const int64_t i1 = min(i0 + chunk, len);
    double s = 0.0, ss = 0.0;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
        float v = st.x[base + i];
        if (st.x2) v = v + st.x2[base + i];
        s += v;
        ss += (double)v * v;
    }
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o);
        ss += __shfl_xor(ss, o);
    }
    if (lane_id() == 0) {
        red[0][wave_id()] = s;
        red[1][wave_id()] = ss;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < num_waves(); ++w) {
            s += red[0][w];
            ss += red[1][w];
        }
        atomicAdd(st.ws + (int64_t)ng * 2, s);
        atomicAdd(st.ws + (int64_t)ng * 2 + 1, ss);
    }
}

// Normalisation constants of group (n, g): mean, rstd = 1/sqrt(var + eps).
__device__ __forceinline__ float2 gn_consts(const double *ws, int n, int G, int g, double count,
                                            float eps) {
    const double s = ws[((int64_t)n * G + g) * 2], ss = ws[((int64_t)n * G + g) * 2 + 1];
    const double mean = s / count;
    double var = ss / count - mean * mean;
    if (var < 0.0) var = 0.0;
    const float rstd = 1.f / sqrtf((float)var + eps);
    return make_float2((float)mean, rstd);
}

__device__ __forceinline__ float gn_norm(float v, float2 mr, float gamma, float beta) {
    return (v - mr.x) * mr.y * gamma + beta;
}

__device__ __forceinline__ float sigmoidf_(float v) { return 1.f / (1.f + expf(-v)); }

// Apply modes (GnApply.mode):
//   VD_GN_ACT:  out = act(GN(x [+ x2]) + res_term), res_term:
//               res_mode 0: none, 1: res, 2: res nearest-2x upsampled, 3: GN_r(res)
//   VD_GN_GRU_Z: out = sigmoid(GN(x + x2))                              (update gate)
//   VD_GN_GRU_R: out = h * sigmoid(GN(x + x2))                          (h * reset gate)
//   VD_GN_GRU_H: hn = (1 - z) * h + z * tanh(GN(x + x2))   (h == NULL: 0 state)
//               out = finer ? hn / 2 + bilinear_0.5x(finer) / 2 : hn
template <bool NHWC>
__device__ __forceinline__ float gn_apply_one(const GnApply &a, int64_t i, int n, int c, int h,
                                              int w, int H, int W, int C, int G, double count,
                                              float2 mr) {
    const int g = c / (C / G);
    float v = a.x[i];
    if (a.x2) v = v + a.x2[i];
    v = gn_norm(v, mr, a.gamma[c], a.beta[c]);
    if (a.mode == VD_GN_ACT) {
        if (a.res_mode == 1) {
            v = v + a.res[i];
        } else if (a.res_mode == 2) {
            const int64_t j = NHWC ? (((int64_t)n * (H / 2) + h / 2) * (W / 2) + w / 2) * C + c
                                   : (((int64_t)n * C + c) * (H / 2) + h / 2) * (W / 2) + w / 2;
            v = v + a.res[j];
        } else if (a.res_mode == 3) {
            const float2 rm = gn_consts(a.res_ws, n, G, g, count, a.eps);
            v = v + gn_norm(a.res[i], rm, a.res_gamma[c], a.res_beta[c]);
        }
        if (a.act == 1) v = fmaxf(v, 0.f);
        else if (a.act == 2) v = sigmoidf_(v);
        else if (a.act == 3) v = tanhf(v);
        return v;
    }
    if (a.mode == VD_GN_GRU_Z) return sigmoidf_(v);
    if (a.mode == VD_GN_GRU_R) return a.res ? a.res[i] * sigmoidf_(v) : 0.f;
    // VD_GN_GRU_H
    const float hh = tanhf(v);
    const float zz = a.z[i];
    float hn = a.res ? (1.f - zz) * a.res[i] + zz * hh : zz * hh;
    if (a.finer) {
        const int W2 = 2 * W, H2 = 2 * H;
        const float *f = a.finer;
        float x00, x01, x10, x11;
        if (NHWC) {
            const int64_t b0 = (((int64_t)n * H2 + 2 * h) * W2 + 2 * w) * C + c;
            x00 = f[b0]; x01 = f[b0 + C];
            x10 = f[b0 + (int64_t)W2 * C]; x11 = f[b0 + (int64_t)W2 * C + C];
        } else {
            const int64_t b0 = (((int64_t)n * C + c) * H2 + 2 * h) * W2 + 2 * w;
            x00 = f[b0]; x01 = f[b0 + 1]; x10 = f[b0 + W2]; x11 = f[b0 + W2 + 1];
        }
        // F.upsample(scale_factor=0.5, mode='bilinear'): source 2*d + 0.5,
        // both lambdas 0.5 (align_corners=False)
        const float down = 0.5f * (0.5f * x00 + 0.5f * x01) + 0.5f * (0.5f * x10 + 0.5f * x11);
        hn = hn / 2.0f + down / 2.0f;
    }
    return hn;
}

__global__ __launch_bounds__(256) void gn_apply_nhwc_kernel(GnApply a, int B, int H, int W,
                                                            int C, int G) {
    const int64_t HW = (int64_t)H * W;
    const int64_t n_el = B * HW * C;
    const double count = (double)(C / G) * HW;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_el;
         i += (int64_t)blockDim.x * gridDim.x) {
        const int c = (int)(i % C);
        const int64_t pix = i / C;
        const int w = (int)(pix % W);
        const int h = (int)((pix / W) % H);
        const int n = (int)(pix / HW);
        const float2 mr = gn_consts(a.ws, n, G, c / (C / G), count, a.eps);
        a.out[i] = gn_apply_one<true>(a, i, n, c, h, w, H, W, C, G, count, mr);
    }
}

__global__ __launch_bounds__(256) void gn_apply_nchw_kernel(GnApply a, int B, int H, int W,
                                                            int C, int G) {
    const int64_t HW = (int64_t)H * W;
    const int64_t n_el = B * HW * C;
    const double count = (double)(C / G) * HW;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_el;
         i += (int64_t)blockDim.x * gridDim.x) {
        const int w = (int)(i % W);
        const int h = (int)((i / W) % H);
        const int c = (int)((i / HW) % C);
        const int n = (int)(i / HW / C);
        const float2 mr = gn_consts(a.ws, n, G, c / (C / G), count, a.eps);
        a.out[i] = gn_apply_one<false>(a, i, n, c, h, w, H, W, C, G, count, mr);
    }
}


// NHWC, C % 4 == 0 (product path): one image per blockIdx.y, the per-channel
// mean / rstd of that image staged in LDS once per block (instead of being
// rebuilt from the double sums per element), one float4 = 4 channels per
// thread step.  Same arithmetic per element as gn_apply_one.
__device__ __forceinline__ float gn_act_(float v, int act) {
    if (act == 1) return fmaxf(v, 0.f);
    if (act == 2) return sigmoidf_(v);
    if (act == 3) return tanhf(v);
    return v;
}

__global__ __launch_bounds__(256) void gn_apply_nhwc4_kernel(GnApply a, int H, int W, int C, int G,
                                                             int pix_per_block) {
    extern __shared__ float cst[];  // [4][C]: mean, rstd, residual mean, residual rstd
    const int n = blockIdx.y;
    const int cg = C / G;
    const int HW = H * W;
    const double count = (double)cg * HW;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const float2 mr = gn_consts(a.ws, n, G, c / cg, count, a.eps);
        cst[c] = mr.x;
        cst[C + c] = mr.y;
        if (a.res_mode == 3) {
            const float2 rm = gn_consts(a.res_ws, n, G, c / cg, count, a.eps);
            cst[2 * C + c] = rm.x;
            cst[3 * C + c] = rm.y;
        }
    }
    __syncthreads();
    const int C4 = C >> 2;
    const int p0 = blockIdx.x * pix_per_block;
    const int p1 = min(p0 + pix_per_block, HW);
    const int64_t img4 = (int64_t)n * HW * C4;
    const float4 *x4 = reinterpret_cast<const float4 *>(a.x);
    const float4 *x24 = reinterpret_cast<const float4 *>(a.x2);
    const float4 *r4 = reinterpret_cast<const float4 *>(a.res);
    const float4 *z4 = reinterpret_cast<const float4 *>(a.z);
    const float4 *g4 = reinterpret_cast<const float4 *>(a.gamma);
    const float4 *b4 = reinterpret_cast<const float4 *>(a.beta);
    float4 *o4 = reinterpret_cast<float4 *>(a.out);
    for (int64_t e = (int64_t)p0 * C4 + threadIdx.x; e < (int64_t)p1 * C4; e += blockDim.x) {
        const int q = (int)(e % C4);
        const int p = (int)(e / C4);
        const int c = q * 4;
        const int64_t i4 = img4 + e;
        float v[4], y[4];
        {
            float4 t = x4[i4];
            if (a.x2) {
                const float4 u = x24[i4];
                t.x = t.x + u.x; t.y = t.y + u.y; t.z = t.z + u.z; t.w = t.w + u.w;
            }
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        }
        const float4 gg = g4[q], bb = b4[q];
        const float gk[4] = {gg.x, gg.y, gg.z, gg.w}, bk[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            y[k] = (v[k] - cst[c + k]) * cst[C + c + k] * gk[k] + bk[k];
        if (a.mode == VD_GN_ACT) {
            if (a.res_mode) {
                int64_t j4 = i4;
                if (a.res_mode == 2) {
                    const int h = p / W, w = p - (p / W) * W;
                    j4 = (((int64_t)n * (H / 2) + h / 2) * (W / 2) + w / 2) * C4 + q;
                }
                const float4 rt = r4[j4];
                float rv[4] = {rt.x, rt.y, rt.z, rt.w};
                if (a.res_mode == 3) {
                    const float4 rg = reinterpret_cast<const float4 *>(a.res_gamma)[q];
                    const float4 rb = reinterpret_cast<const float4 *>(a.res_beta)[q];
                    const float rgk[4] = {rg.x, rg.y, rg.z, rg.w}, rbk[4] = {rb.x, rb.y, rb.z, rb.w};
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        rv[k] = (rv[k] - cst[2 * C + c + k]) * cst[3 * C + c + k] * rgk[k] + rbk[k];
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) y[k] = y[k] + rv[k];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) y[k] = gn_act_(y[k], a.act);
        } else if (a.mode == VD_GN_GRU_Z) {
#pragma unroll
            for (int k = 0; k < 4; ++k) y[k] = sigmoidf_(y[k]);
        } else if (a.mode == VD_GN_GRU_R) {
            const float4 ht = a.res ? r4[i4] : make_float4(0.f, 0.f, 0.f, 0.f);
            const float hk[4] = {ht.x, ht.y, ht.z, ht.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) y[k] = a.res ? hk[k] * sigmoidf_(y[k]) : 0.f;
        } else {  // VD_GN_GRU_H
            const float4 zt = z4[i4];
            const float zk[4] = {zt.x, zt.y, zt.z, zt.w};
            float hk[4] = {0.f, 0.f, 0.f, 0.f};
            if (a.res) {
                const float4 ht = r4[i4];
                hk[0] = ht.x; hk[1] = ht.y; hk[2] = ht.z; hk[3] = ht.w;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float hh = tanhf(y[k]);
                y[k] = a.res ? (1.f - zk[k]) * hk[k] + zk[k] * hh : zk[k] * hh;
            }
            if (a.finer) {
                const int h = p / W, w = p - (p / W) * W;
                const int W2 = 2 * W, H2 = 2 * H;
                const float4 *f4 = reinterpret_cast<const float4 *>(a.finer);
                const int64_t b0 = (((int64_t)n * H2 + 2 * h) * W2 + 2 * w) * C4 + q;
                const float4 t00 = f4[b0], t01 = f4[b0 + C4];
                const float4 t10 = f4[b0 + (int64_t)W2 * C4], t11 = f4[b0 + (int64_t)W2 * C4 + C4];
                const float f00[4] = {t00.x, t00.y, t00.z, t00.w},
                            f01[4] = {t01.x, t01.y, t01.z, t01.w},
                            f10[4] = {t10.x, t10.y, t10.z, t10.w},
                            f11[4] = {t11.x, t11.y, t11.z, t11.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float down = 0.5f * (0.5f * f00[k] + 0.5f * f01[k]) +
                                       0.5f * (0.5f * f10[k] + 0.5f * f11[k]);
                    y[k] = y[k] / 2.0f + down / 2.0f;
                }
            }
        }
        o4[i4] = make_float4(y[0], y[1], y[2], y[3]);
    }
}

size_t gn_workspace_bytes(int B, int G, int sets) { return (size_t)sets * B * G * 2 * sizeof(double); }

int launch_gn_stats(const GnSets &sets, int nsets, int B, int C, int HW, int G, int nhwc,
                    hipStream_t s) {
    if (B == 0 || HW == 0) return VD_OK;
    for (int k = 0; k < nsets; ++k)
        if (zero_async(sets.s[k].ws, (size_t)B * G * 2 * sizeof(double), s) != VD_OK)
            return VD_ERR_LAUNCH;
    if (nhwc && C % 4 == 0 && G <= 64) {
        const int C4 = C / 4;
        const int ppi = C4 >= 256 ? 1 : 256 / C4;
        const int ppb = ppi * 32;  // 32 iterations per thread
        const dim3 grid((HW + ppb - 1) / ppb, B, nsets);
        hipLaunchKernelGGL(gn_stats_nhwc_kernel, grid, dim3(256), 0, s, sets, HW, C, G, ppb);
    } else if (!nhwc) {
        const int64_t len = (int64_t)(C / G) * HW;
        const int chunk = 256 * 32;
        const dim3 grid((unsigned)((len + chunk - 1) / chunk), B * G, nsets);
        hipLaunchKernelGGL(gn_stats_nchw_kernel, grid, dim3(256), 0, s, sets, HW, C, G, chunk);
    } else {
        return VD_ERR_SHAPE;
    }
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int launch_gn_apply(const GnApply &a, int B, int C, int H, int W, int G, int nhwc,
                    hipStream_t s) {
    const int64_t n = (int64_t)B * C * H * W;
    if (n == 0) return VD_OK;
    if (nhwc && C % 4 == 0) {
        const int ppb = max(1, 4096 / (C / 4));  // ~16 float4 per thread
        const dim3 grid((H * W + ppb - 1) / ppb, B);
        hipLaunchKernelGGL(gn_apply_nhwc4_kernel, grid, dim3(256), (size_t)4 * C * sizeof(float),
                           s, a, H, W, C, G, ppb);
    } else if (nhwc)
        hipLaunchKernelGGL(gn_apply_nhwc_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, a, B, H,
                           W, C, G);
    else
        hipLaunchKernelGGL(gn_apply_nchw_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, a, B, H,
                           W, C, G);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
