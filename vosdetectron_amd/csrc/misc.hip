// The remaining RoI operators of the reference's lib/model (API completeness,
// selectable through FAST_RCNN.ROI_XFORM_METHOD) and the frame/pyramid layout
// kernels of the product path.
//
//   jwyang RoIAlign   lib/model/roi_align/src/roi_align_kernel.cu:15-70
//   RoIPool fwd/bwd   lib/model/roi_pooling/src/roi_pooling_kernel.cu:24-93,128-203
//   RoICrop fwd       lib/model/roi_crop/src/roi_crop_cuda_kernel.cu:11-109,201-255
//   image -> blob     lib/utils/blob.py:37-114 (identity scale)
#include <float.h>

#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

static int blocks_for(int64_t n, int bs) {
    int64_t g = (n + bs - 1) / bs;
    if (g > 65536) g = 65536;
    return (int)(g < 1 ? 1 : g);
}

// ---------------------------------------------------------------- legacy
__global__ __launch_bounds__(256) void roi_align_legacy_kernel(
    int64_t nthreads, const float *__restrict__ feat, float scale, int H, int W, int C, int PH,
    int PW, const float *__restrict__ rois, float *__restrict__ out) {
    for (int64_t index = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; index < nthreads;
         index += (int64_t)blockDim.x * gridDim.x) {
        const int pw = (int)(index % PW);
        const int ph = (int)((index / PW) % PH);
        const int c = (int)((index / PW / PH) % C);
        const int64_t n = index / PW / PH / C;
        const float *r = rois + n * 5;
        const int b = (int)r[0];  // reference multiplies a float batch index (:30,:46)
        const float sw = r[1] * scale, sh = r[2] * scale, ew = r[3] * scale, eh = r[4] * scale;
        const float rw = fmaxf((float)((double)(ew - sw) + 1.), 0.f);
        const float rh = fmaxf((float)((double)(eh - sh) + 1.), 0.f);
        const float bh = (float)(rh / (PH - 1.));
        const float bw = (float)(rw / (PW - 1.));
        const float h = (float)ph * bh + sh;
        const float w = (float)pw * bw + sw;
        const int hstart = (int)fminf(floorf(h), (float)(H - 2));
        const int wstart = (int)fminf(floorf(w), (float)(W - 2));
        if (h < 0 || h >= H || w < 0 || w >= W) {
            out[index] = 0.f;
            continue;
        }
        const float hr = h - (float)hstart, wr = w - (float)wstart;
        const int64_t ul = (int64_t)b * C * H * W + ((int64_t)c * H + hstart) * W + wstart;
        const int64_t ur = ul + 1, dl = ul + W, dr = dl + 1;
        out[index] = (float)(feat[ul] * (1. - hr) * (1. - wr) + feat[ur] * (1. - hr) * wr +
                             feat[dl] * hr * (1. - wr) + feat[dr] * hr * wr);
    }
}

int launch_roi_align_legacy_fwd(const float *feat, int B, int C, int H, int W, const float *rois,
                                int R, int PH, int PW, float scale, float *out, hipStream_t s) {
    (void)B;
    const int64_t n = (int64_t)R * C * PH * PW;
    if (n == 0) return VD_OK;
    if (PH < 2 || PW < 2) return VD_ERR_ARG;
    hipLaunchKernelGGL(roi_align_legacy_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, n, feat,
                       scale, H, W, C, PH, PW, rois, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// ---------------------------------------------------------------- RoIPool
__global__ __launch_bounds__(256) void roi_pool_fwd_kernel(
    int64_t nthreads, const float *__restrict__ feat, float scale, int H, int W, int C, int PH,
    int PW, const float *__restrict__ rois, float *__restrict__ out, int32_t *__restrict__ argmax) {
    for (int64_t index = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; index < nthreads;
         index += (int64_t)blockDim.x * gridDim.x) {
        const int pw = (int)(index % PW);
        const int ph = (int)((index / PW) % PH);
        const int c = (int)((index / PW / PH) % C);
        const int64_t n = index / PW / PH / C;
        const float *r = rois + n * 5;
        const int b = (int)r[0];
        const int rsw = (int)roundf(r[1] * scale), rsh = (int)roundf(r[2] * scale);
        const int rew = (int)roundf(r[3] * scale), reh = (int)roundf(r[4] * scale);
        const int rw = (int)fmaxf((float)(rew - rsw + 1), 1.f);
        const int rh = (int)fmaxf((float)(reh - rsh + 1), 1.f);
        const float bh = (float)rh / (float)PH, bw = (float)rw / (float)PW;
        int hs = (int)floorf((float)ph * bh), ws = (int)floorf((float)pw * bw);
        int he = (int)ceilf((float)(ph + 1) * bh), we = (int)ceilf((float)(pw + 1) * bw);
        hs = (int)fminf(fmaxf((float)(hs + rsh), 0.f), (float)H);
        he = (int)fminf(fmaxf((float)(he + rsh), 0.f), (float)H);
        ws = (int)fminf(fmaxf((float)(ws + rsw), 0.f), (float)W);
        we = (int)fminf(fmaxf((float)(we + rsw), 0.f), (float)W);
        const bool empty = (he <= hs) || (we <= ws);
        float maxval = empty ? 0.f : -FLT_MAX;
        int maxidx = -1;
        const int64_t off = ((int64_t)b * C + c) * (int64_t)H * W;
        for (int h = hs; h < he; ++h)
            for (int w = ws; w < we; ++w) {
                const float v = feat[off + (int64_t)h * W + w];
                if (v > maxval) {
                    maxval = v;
                    maxidx = (int)(off + (int64_t)h * W + w);
                }
            }
        out[index] = maxval;
        if (argmax) argmax[index] = maxidx;
    }
}

__global__ __launch_bounds__(256) void roi_pool_bwd_kernel(int64_t n,
                                                           const float *__restrict__ top_diff,
                                                           const int32_t *__restrict__ argmax,
                                                           float *__restrict__ bottom_diff) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)blockDim.x * gridDim.x) {
        const int a = argmax[i];
        if (a >= 0) atomicAdd(bottom_diff + a, top_diff[i]);
    }
}

int launch_roi_pool_fwd(const float *feat, int B, int C, int H, int W, const float *rois, int R,
                        int PH, int PW, float scale, float *out, int32_t *argmax, hipStream_t s) {
    (void)B;
    const int64_t n = (int64_t)R * C * PH * PW;
    if (n == 0) return VD_OK;
    hipLaunchKernelGGL(roi_pool_fwd_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, n, feat,
                       scale, H, W, C, PH, PW, rois, out, argmax);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int launch_roi_pool_bwd(const float *top_diff, const int32_t *argmax, int64_t n,
                        float *bottom_diff, hipStream_t s) {
    if (n == 0) return VD_OK;
    hipLaunchKernelGGL(roi_pool_bwd_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, n,
                       top_diff, argmax, bottom_diff);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// ---------------------------------------------------------------- RoICrop
__device__ __forceinline__ void top_left(float x, int width, int &point, float &weight) {
    const float xcoord = (x + 1) * (width - 1) / 2;
    point = (int)floorf(xcoord);
    weight = 1 - (xcoord - point);
}
__device__ __forceinline__ bool between(int v, int lo, int hi) { return v >= lo && v <= hi; }

__global__ __launch_bounds__(256) void roi_crop_fwd_kernel(
    int64_t nthreads, const float *__restrict__ in, int C, int H, int W,
    const float *__restrict__ grid, int GH, int GW, int roi_per_image, float *__restrict__ out) {
    for (int64_t index = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; index < nthreads;
         index += (int64_t)blockDim.x * gridDim.x) {
        const int xo = (int)(index % GW);
        const int yo = (int)((index / GW) % GH);
        const int c = (int)((index / GW / GH) % C);
        const int64_t b = index / GW / GH / C;
        const int64_t bi = b / roi_per_image;
        const float *g = grid + ((b * GH + yo) * GW + xo) * 2;
        const float yf = g[0], xf = g[1];
        int yTL, xTL;
        float yW, xW;
        top_left(xf, W, xTL, xW);
        top_left(yf, H, yTL, yW);
        const bool tl = between(xTL, 0, W - 1) && between(yTL, 0, H - 1);
        const bool tr = between(xTL + 1, 0, W - 1) && between(yTL, 0, H - 1);
        const bool bl = between(xTL, 0, W - 1) && between(yTL + 1, 0, H - 1);
        const bool br = between(xTL + 1, 0, W - 1) && between(yTL + 1, 0, H - 1);
        if (!tl && !tr && !bl && !br) continue;
        const float *plane = in + (bi * C + c) * (int64_t)H * W;
        const float vTL = tl ? plane[(int64_t)yTL * W + xTL] : 0.f;
        const float vTR = tr ? plane[(int64_t)yTL * W + xTL + 1] : 0.f;
        const float vBL = bl ? plane[(int64_t)(yTL + 1) * W + xTL] : 0.f;
        const float vBR = br ? plane[(int64_t)(yTL + 1) * W + xTL + 1] : 0.f;
        out[index] = xW * yW * vTL + (1 - xW) * yW * vTR + xW * (1 - yW) * vBL +
                     (1 - xW) * (1 - yW) * vBR;
    }
}

int launch_roi_crop_fwd(const float *in, int B, int C, int H, int W, const float *grid, int R,
                        int GH, int GW, float *out, hipStream_t s) {
    const int64_t n = (int64_t)R * C * GH * GW;
    if (n == 0) return VD_OK;
    if (B < 1 || R < B) return VD_ERR_ARG;  // roiPerImage = ob / ib (launcher :217)
    hipLaunchKernelGGL(roi_crop_fwd_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, n, in, C,
                       H, W, grid, GH, GW, R / B, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// ---------------------------------------------------------------- frames
// One thread per 4 padded pixels of one row; u8 BGR triplets -> LUT floats.
__global__ __launch_bounds__(256) void image_to_blob_kernel(const uint8_t *__restrict__ frames,
                                                            int H, int W,
                                                            const float *__restrict__ lut, int Hp,
                                                            int Wp, int nhwc,
                                                            float *__restrict__ blob) {
    __shared__ float slut[768];
    for (int i = threadIdx.x; i < 768; i += blockDim.x) slut[i] = lut[i];
    __syncthreads();
    const int f = blockIdx.z, y = blockIdx.y;
    const uint8_t *src = frames + ((int64_t)f * H + y) * W * 3;
    for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < Wp; x += gridDim.x * blockDim.x) {
        float b = 0.f, g = 0.f, r = 0.f;
        if (y < H && x < W) {
            b = slut[src[x * 3 + 0]];
            g = slut[256 + src[x * 3 + 1]];
            r = slut[512 + src[x * 3 + 2]];
        }
        if (nhwc) {
            float *d = blob + (((int64_t)f * Hp + y) * Wp + x) * 3;
            d[0] = b;
            d[1] = g;
            d[2] = r;
        } else {
            const int64_t plane = (int64_t)Hp * Wp;
            float *d = blob + (int64_t)f * 3 * plane + (int64_t)y * Wp + x;
            d[0] = b;
            d[plane] = g;
            d[2 * plane] = r;
        }
    }
}

int launch_image_to_blob(const uint8_t *frames, int F, int H, int W, const float *lut, int Hp,
                         int Wp, int nhwc, float *blob, hipStream_t s) {
    if (F < 1 || Hp < H || Wp < W) return VD_ERR_ARG;
    dim3 grid((Wp + 255) / 256, Hp, F);
    hipLaunchKernelGGL(image_to_blob_kernel, grid, dim3(256), 0, s, frames, H, W, lut, Hp, Wp,
                       nhwc, blob);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// prep_im_for_blob with a non-identity scale (lib/utils/blob.py:117-139):
//   im = float32(BGR u8) - PIXEL_MEANS;  cv2.resize(im, None, fx=s, fy=s,
//   INTER_LINEAR);  zero-pad to (Hp, Wp) (im_list_to_blob, :86-110).
// The resize restates OpenCV's scalar float INTER_LINEAR path (cv::resize with
// dsize from fx/fy keeps inv_scale = s, so scale = 1/s in double):
//   fx = (float)((dx + 0.5) * scale - 0.5), sx = floor(fx), fx -= sx;
//   sx < 0 -> (0, 0); sx >= W-1 -> (W-1, 0)         (coefficient tables)
//   row value  D = S[sx] * (1 - fx) + S[sx+1] * fx   (HResizeLinear)
//   fy likewise, rows clip(sy, 0, H-1), clip(sy+1, 0, H-1), no fy clamp,
//   value      D0 * (1 - fy) + D1 * fy              (VResizeLinear)
// per channel on the mean-subtracted float image (the LUT holds numpy's
// float32(u - mean)).  -ffp-contract=off keeps every product and sum rounded
// as the scalar path and the numpy restatement in oracle/oracle.py round them;
// OpenCV's SIMD builds may fuse a multiply-add (parity unpinned: cv2 absent).
__global__ __launch_bounds__(256) void resize_to_blob_kernel(
    const uint8_t *__restrict__ frames, int H, int W, const float *__restrict__ lut,
    double scale_x, double scale_y, int Hr, int Wr, int Hp, int Wp, int nhwc,
    float *__restrict__ blob) {
    __shared__ float slut[768];
    for (int i = threadIdx.x; i < 768; i += blockDim.x) slut[i] = lut[i];
    __syncthreads();
    const int f = blockIdx.z, y = blockIdx.y;
    // both scales exactly 2: OpenCV runs INTER_AREA's fast path instead (mean of
    // each 2 x 2 block, scalar loop order; a partial block at an odd edge
    // averages the taps inside the image)
    const bool area2 = scale_x == 2.0 && scale_y == 2.0;
    if (area2) {
        for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < Wp; x += gridDim.x * blockDim.x) {
            float v[3] = {0.f, 0.f, 0.f};
            if (y < Hr && x < Wr) {
                const int ys = 2 * y, xs = 2 * x;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float *L = slut + 256 * c;
                    float sum = 0.f;
                    int cnt = 0;
                    for (int dy = 0; dy < 2 && ys + dy < H; ++dy)
                        for (int dx = 0; dx < 2 && xs + dx < W; ++dx) {
                            sum += L[frames[(((int64_t)f * H + ys + dy) * W + xs + dx) * 3 + c]];
                            ++cnt;
                        }
                    v[c] = cnt == 4 ? sum * 0.25f : sum / (float)cnt;
                }
            }
            if (nhwc) {
                float *d = blob + (((int64_t)f * Hp + y) * Wp + x) * 3;
                d[0] = v[0];
                d[1] = v[1];
                d[2] = v[2];
            } else {
                const int64_t plane = (int64_t)Hp * Wp;
                float *d = blob + (int64_t)f * 3 * plane + (int64_t)y * Wp + x;
                d[0] = v[0];
                d[plane] = v[1];
                d[2 * plane] = v[2];
            }
        }
        return;
    }
    int r0 = 0, r1 = 0;
    float b0 = 0.f, b1 = 0.f;
    if (y < Hr) {
        float fy = (float)((y + 0.5) * scale_y - 0.5);
        const int sy = (int)floorf(fy);
        fy -= (float)sy;
        r0 = min(max(sy, 0), H - 1);
        r1 = min(max(sy + 1, 0), H - 1);
        b0 = 1.f - fy;
        b1 = fy;
    }
    const uint8_t *row0 = frames + ((int64_t)f * H + r0) * W * 3;
    const uint8_t *row1 = frames + ((int64_t)f * H + r1) * W * 3;
    for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < Wp; x += gridDim.x * blockDim.x) {
        float v[3] = {0.f, 0.f, 0.f};
        if (y < Hr && x < Wr) {
            float fx = (float)((x + 0.5) * scale_x - 0.5);
            int sx = (int)floorf(fx);
            fx -= (float)sx;
            if (sx < 0) { fx = 0.f; sx = 0; }
            if (sx >= W - 1) { fx = 0.f; sx = W - 1; }
            const int sx1 = min(sx + 1, W - 1);
            const float a0 = 1.f - fx, a1 = fx;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float *L = slut + 256 * c;
                const float d0 = L[row0[sx * 3 + c]] * a0 + L[row0[sx1 * 3 + c]] * a1;
                const float d1 = L[row1[sx * 3 + c]] * a0 + L[row1[sx1 * 3 + c]] * a1;
                v[c] = d0 * b0 + d1 * b1;
            }
        }
        if (nhwc) {
            float *d = blob + (((int64_t)f * Hp + y) * Wp + x) * 3;
            d[0] = v[0];
            d[1] = v[1];
            d[2] = v[2];
        } else {
            const int64_t plane = (int64_t)Hp * Wp;
            float *d = blob + (int64_t)f * 3 * plane + (int64_t)y * Wp + x;
            d[0] = v[0];
            d[plane] = v[1];
            d[2 * plane] = v[2];
        }
    }
}

int launch_resize_to_blob(const uint8_t *frames, int F, int H, int W, const float *lut,
                          double im_scale, int Hr, int Wr, int Hp, int Wp, int nhwc, float *blob,
                          hipStream_t s) {
    if (F < 1 || H < 1 || W < 1 || !(im_scale > 0.0) || Hr < 1 || Wr < 1 || Hp < Hr || Wp < Wr)
        return VD_ERR_ARG;
    const double scale = 1.0 / im_scale;  // cv::resize: scale_x = 1 / inv_scale_x
    dim3 grid((Wp + 255) / 256, Hp, F);
    hipLaunchKernelGGL(resize_to_blob_kernel, grid, dim3(256), 0, s, frames, H, W, lut, scale,
                       scale, Hr, Wr, Hp, Wp, nhwc, blob);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// B x C x HW -> B x HW x C through a 64x64 LDS tile (+1 pad against bank conflicts).
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const float *__restrict__ in, int C,
                                                           int HW, float *__restrict__ out) {
    __shared__ float tile[64][65];
    const int b = blockIdx.z;
    const int c0 = blockIdx.y * 64, p0 = blockIdx.x * 64;
    const float *src = in + (int64_t)b * C * HW;
    float *dst = out + (int64_t)b * C * HW;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
    for (int k = ty; k < 64; k += 4) {
        const int c = c0 + k, p = p0 + tx;
        tile[k][tx] = (c < C && p < HW) ? src[(int64_t)c * HW + p] : 0.f;
    }
    __syncthreads();
    for (int k = ty; k < 64; k += 4) {
        const int p = p0 + k, c = c0 + tx;
        if (p < HW && c < C) dst[(int64_t)p * C + c] = tile[tx][k];
    }
}

int launch_nchw_to_nhwc(const float *in, int B, int C, int H, int W, float *out, hipStream_t s) {
    const int HW = H * W;
    if (B < 1 || C < 1 || HW < 1) return VD_ERR_ARG;
    dim3 grid((HW + 63) / 64, (C + 63) / 64, B);
    hipLaunchKernelGGL(nchw_to_nhwc_kernel, grid, dim3(256), 0, s, in, C, HW, out);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// ---------------------------------------------------------------- conv epilogue
// out = act((x + bias[c]) + res_term), in place on x, where res_term is
//   mode 0: 0, mode 1: z (+ bias2[c]), mode 2: z nearest-2x-upsampled (+ bias2[c]).
// One read of x (and z), one write: replaces the bias-add, residual-add and
// ReLU passes PyTorch runs after each MIOpen convolution (each a full HBM
// round trip of the activation).  Same association order as the unfused
// module code ((conv + bias) + residual), so results are bit-identical to it.
// NHWC, C % 4 == 0: one float4 = 4 consecutive channels of one pixel.
__global__ __launch_bounds__(256) void bias_act_nhwc4_kernel(
    float *__restrict__ x, const float *__restrict__ bias, const float *__restrict__ z,
    const float *__restrict__ bias2, uint32_t n4, uint32_t C4, uint32_t H, uint32_t W, int mode,
    int relu) {
    for (uint32_t i4 = blockIdx.x * blockDim.x + threadIdx.x; i4 < n4;
         i4 += blockDim.x * gridDim.x) {
        const uint32_t c4 = i4 % C4;
        float4 v = reinterpret_cast<float4 *>(x)[i4];
        if (bias) {
            const float4 bb = reinterpret_cast<const float4 *>(bias)[c4];
            v.x = v.x + bb.x; v.y = v.y + bb.y; v.z = v.z + bb.z; v.w = v.w + bb.w;
        }
        if (mode) {
            uint32_t zi = i4;
            if (mode == 2) {  // i4 = ((n*H + h)*W + w)*C4 + c4
                const uint32_t pix = i4 / C4;
                const uint32_t w = pix % W, nh = pix / W;
                const uint32_t h = nh % H, nn = nh / H;
                zi = ((nn * (H / 2) + h / 2) * (W / 2) + w / 2) * C4 + c4;
            }
            float4 t = reinterpret_cast<const float4 *>(z)[zi];
            if (bias2) {
                const float4 bb = reinterpret_cast<const float4 *>(bias2)[c4];
                t.x = t.x + bb.x; t.y = t.y + bb.y; t.z = t.z + bb.z; t.w = t.w + bb.w;
            }
            v.x = v.x + t.x; v.y = v.y + t.y; v.z = v.z + t.z; v.w = v.w + t.w;
        }
        if (relu) {
            v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f);
            v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
        }
        reinterpret_cast<float4 *>(x)[i4] = v;
    }
}

// Any layout / C: one element per thread.
__global__ __launch_bounds__(256) void bias_act_scalar_kernel(
    float *__restrict__ x, const float *__restrict__ bias, const float *__restrict__ z,
    const float *__restrict__ bias2, uint32_t n, uint32_t C, uint32_t H, uint32_t W, int nhwc,
    int mode, int relu) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += blockDim.x * gridDim.x) {
        uint32_t c, w, h, nn;
        if (nhwc) {  // i = ((n*H + h)*W + w)*C + c
            c = i % C;
            const uint32_t pix = i / C;
            w = pix % W;
            h = (pix / W) % H;
            nn = pix / W / H;
        } else {  // i = ((n*C + c)*H + h)*W + w
            w = i % W;
            h = (i / W) % H;
            c = (i / W / H) % C;
            nn = i / W / H / C;
        }
        float y = x[i];
        if (bias) y = y + bias[c];
        if (mode) {
            uint32_t zi = i;
            if (mode == 2)
                zi = nhwc ? ((nn * (H / 2) + h / 2) * (W / 2) + w / 2) * C + c
                          : ((nn * C + c) * (H / 2) + h / 2) * (W / 2) + w / 2;
            float t = z[zi];
            if (bias2) t = t + bias2[c];
            y = y + t;
        }
        if (relu) y = fmaxf(y, 0.f);
        x[i] = y;
    }
}

int launch_bias_act(float *x, const float *bias, const float *z, const float *bias2, int64_t n,
                    int C, int H, int W, int nhwc, int mode, int relu, hipStream_t s) {
    if (n == 0) return VD_OK;
    if (n >= (int64_t)1 << 31 || (mode == 2 && ((H & 1) || (W & 1)))) return VD_ERR_SHAPE;
    if (nhwc && C % 4 == 0) {
        const int64_t n4 = n / 4;
        hipLaunchKernelGGL(bias_act_nhwc4_kernel, dim3(blocks_for(n4, 256)), dim3(256), 0, s, x,
                           bias, z, bias2, (uint32_t)n4, (uint32_t)(C / 4), (uint32_t)H,
                           (uint32_t)W, mode, relu);
    } else {
        hipLaunchKernelGGL(bias_act_scalar_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, x,
                           bias, z, bias2, (uint32_t)n, (uint32_t)C, (uint32_t)H, (uint32_t)W,
                           nhwc, mode, relu);
    }
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// ---------------------------------------------------------------- stem epilogue
// basic_bn_stem's tail (lib/modeling/ResNet.py:224-230) after the bias-free
// conv1: AffineChannel bias + ReLU + MaxPool2d(3, stride 2, pad 1) in one pass,
// NHWC in and out.  Each window element is relu(x + b) exactly as vd_bias_act
// computes it, and the max of those is what max_pool2d returns (padding never
// wins: every window holds at least one in-image pixel), so the result is
// bit-identical to bias_act + max_pool2d while the full-resolution activation
// is read once instead of written and read again (HBM bytes per output pixel:
// ~2.25 x 4C read through L2 for 4C written).
__global__ __launch_bounds__(256) void bias_relu_maxpool_nhwc4_kernel(
    const float *__restrict__ x, const float *__restrict__ bias, float *__restrict__ out,
    uint32_t n4, uint32_t C4, uint32_t H, uint32_t W, uint32_t Ho, uint32_t Wo) {
    for (uint32_t i4 = blockIdx.x * blockDim.x + threadIdx.x; i4 < n4;
         i4 += blockDim.x * gridDim.x) {
        const uint32_t c4 = i4 % C4, pix = i4 / C4;
        const uint32_t wo = pix % Wo, t = pix / Wo;
        const uint32_t ho = t % Ho, n = t / Ho;
        const float4 b = reinterpret_cast<const float4 *>(bias)[c4];
        float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
            const int y = 2 * (int)ho - 1 + dy;
            if (y < 0 || y >= (int)H) continue;
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                const int xx = 2 * (int)wo - 1 + dx;
                if (xx < 0 || xx >= (int)W) continue;
                const float4 v = reinterpret_cast<const float4 *>(
                    x)[((uint64_t)(n * H + y) * W + xx) * C4 + c4];
                m.x = fmaxf(m.x, fmaxf(v.x + b.x, 0.f));
                m.y = fmaxf(m.y, fmaxf(v.y + b.y, 0.f));
                m.z = fmaxf(m.z, fmaxf(v.z + b.z, 0.f));
                m.w = fmaxf(m.w, fmaxf(v.w + b.w, 0.f));
            }
        }
        reinterpret_cast<float4 *>(out)[i4] = m;
    }
}

int launch_bias_relu_maxpool(const float *x, const float *bias, int N, int C, int H, int W,
                             float *out, hipStream_t s) {
    if ((int64_t)N * H * W == 0) return VD_OK;
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;  // (H + 2 - 3) / 2 + 1
    const int64_t n4 = (int64_t)N * Ho * Wo * (C / 4);
    if (C % 4 != 0 || (int64_t)N * H * W * C >= ((int64_t)1 << 32) || n4 >= ((int64_t)1 << 31))
        return VD_ERR_SHAPE;
    hipLaunchKernelGGL(bias_relu_maxpool_nhwc4_kernel, dim3(blocks_for(n4, 256)), dim3(256), 0, s,
                       x, bias, out, (uint32_t)n4, (uint32_t)(C / 4), (uint32_t)H, (uint32_t)W,
                       (uint32_t)Ho, (uint32_t)Wo);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

// [p, p + bytes): the 16-B aligned middle as uint4 stores, the < 16-B head and tail
// bytes by workgroup 0
__global__ void zero_kernel(uint8_t *head, int nhead, uint4 *mid, size_t n16, uint8_t *tail,
                            int ntail) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
        mid[i] = make_uint4(0u, 0u, 0u, 0u);
    if (blockIdx.x == 0) {
        if ((int)threadIdx.x < nhead) head[threadIdx.x] = 0;
        if ((int)threadIdx.x < ntail) tail[threadIdx.x] = 0;
    }
}

int zero_async(void *p, size_t bytes, hipStream_t s) {
    if (bytes == 0) return VD_OK;
    uint8_t *b = reinterpret_cast<uint8_t *>(p);
    size_t nhead = (16 - ((uintptr_t)b & 15)) & 15;
    if (nhead > bytes) nhead = bytes;
    const size_t n16 = (bytes - nhead) / 16;
    const size_t ntail = bytes - nhead - n16 * 16;
    size_t blocks = (n16 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(zero_kernel, dim3((unsigned)blocks), dim3(256), 0, s, b, (int)nhead,
                       reinterpret_cast<uint4 *>(b + nhead), n16, b + nhead + n16 * 16,
                       (int)ntail);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
