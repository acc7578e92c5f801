// Standalone NMS (drop-in for utils.boxes.nms -> cython_nms.nms,
// lib/utils/boxes.py:329-333, lib/utils/cython_nms.pyx:37-87).
//
// Three launches on the caller's stream, all device-resident (the reference's
// GPU path nms_cuda_compute copies the whole mask to the host and resolves it
// there, lib/model/nms/src/nms_cuda_kernel.cu:111-145):
//   1. prep   (1 WG):  processing order = keys (score, index) sorted
//                      descending -> score desc, ties higher index first;
//                      boxes gathered in that order, areas in fp32.
//   2. mask   (n/16 WGs): one wave per row, one ballot per 64-column word.
//   3. resolve(1 WG):  one wave resolves the mask; the block maps ranks back
//                      to input indices and compacts them ascending.
#include "nms_block.hpp"
#include "vosdet_internal.hpp"

namespace vd {

static constexpr int kNmsMaxN = 8192;

struct NmsWs {
    float *x1, *y1, *x2, *y2, *area;
    int32_t *order;
    uint64_t *mask;
};

__host__ __device__ inline size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

__host__ __device__ inline NmsWs nms_ws(void *base, int n) {
    NmsWs w;
    char *p = (char *)base;
    const size_t fb = align256(sizeof(float) * (size_t)n);
    w.x1 = (float *)p; p += fb;
    w.y1 = (float *)p; p += fb;
    w.x2 = (float *)p; p += fb;
    w.y2 = (float *)p; p += fb;
    w.area = (float *)p; p += fb;
    w.order = (int32_t *)p; p += align256(sizeof(int32_t) * (size_t)n);
    w.mask = (uint64_t *)p;
    return w;
}

size_t nms_workspace_bytes(int n) {
    if (n <= 0) return 256;
    const size_t words = (size_t)(n + 63) / 64;
    return 5 * align256(sizeof(float) * (size_t)n) + align256(sizeof(int32_t) * (size_t)n) +
           align256(sizeof(uint64_t) * (size_t)n * words);
}

__global__ __launch_bounds__(1024) void nms_prep_kernel(const float *__restrict__ dets, int n,
                                                         int stride, NmsWs ws) {
    extern __shared__ __attribute__((aligned(16))) uint64_t keys[];
    const int np2 = next_pow2(n);
    for (int i = threadIdx.x; i < np2; i += blockDim.x)
        keys[i] = i < n ? ((uint64_t)float_key(dets[(int64_t)i * stride + 4]) << 32) | (uint32_t)i
                        : 0ull;
    __syncthreads();
    bitonic_sort_desc(keys, np2);
    for (int r = threadIdx.x; r < n; r += blockDim.x) {
        const int i = (int)(uint32_t)keys[r];
        const float *d = dets + (int64_t)i * stride;
        const float a = d[0], b = d[1], c = d[2], e = d[3];
        ws.x1[r] = a;
        ws.y1[r] = b;
        ws.x2[r] = c;
        ws.y2[r] = e;
        ws.area[r] = (c - a + 1) * (e - b + 1);  // cython_nms.pyx:44
        ws.order[r] = i;
    }
}

__global__ __launch_bounds__(1024) void nms_mask_kernel(int n, float thresh, NmsWs ws) {
    const int waves_per_block = blockDim.x / 64;
    nms_build_mask_rows(ws.x1, ws.y1, ws.x2, ws.y2, ws.area, n, thresh, ws.mask,
                        blockIdx.x * waves_per_block + wave_id(), gridDim.x * waves_per_block);
}

// in_lds: the whole mask is first copied into LDS by the block (coalesced), so
// the resolving wave's row reads cost LDS latency instead of one L2 round trip
// per 16-row batch (N = 1000: 128 KB, 37 -> ~10 us)
__global__ __launch_bounds__(1024) void nms_resolve_kernel(int n, NmsWs ws,
                                                            int64_t *__restrict__ keep_out,
                                                            int32_t *__restrict__ num_out,
                                                            int in_lds) {
    __shared__ uint8_t keep_rank[kNmsMaxN];
    __shared__ uint8_t keep_idx[kNmsMaxN];
    __shared__ int scratch[16];
    extern __shared__ __attribute__((aligned(16))) uint64_t lmask[];
    if (in_lds) {
        const int cnt = n * ((n + 63) >> 6);
        for (int i = threadIdx.x; i < cnt; i += blockDim.x) lmask[i] = ws.mask[i];
        __syncthreads();
        if (wave_id() == 0) nms_resolve_wave(lmask, n, keep_rank);
    } else if (wave_id() == 0) {
        nms_resolve_wave(ws.mask, n, keep_rank);
    }
    __syncthreads();
    for (int r = threadIdx.x; r < n; r += blockDim.x) keep_idx[ws.order[r]] = keep_rank[r];
    __syncthreads();
    const int cnt = block_compact(
        n, [&](int i) { return keep_idx[i] != 0; },
        [&](int pos, int i) { keep_out[pos] = (int64_t)i; }, scratch);
    if (threadIdx.x == 0) *num_out = cnt;
}

__global__ void zero_i32_kernel(int32_t *p) { *p = 0; }

int launch_nms(const float *dets, int n, int stride, float thresh, int64_t *keep, int32_t *nkeep,
               void *workspace, size_t ws_bytes, hipStream_t s) {
    if (n < 0 || stride < 5) return VD_ERR_ARG;
    if (n > kNmsMaxN) return VD_ERR_SHAPE;
    if (n == 0) {
        hipLaunchKernelGGL(zero_i32_kernel, dim3(1), dim3(1), 0, s, nkeep);
        return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
    }
    if (ws_bytes < nms_workspace_bytes(n) || !workspace) return VD_ERR_WORKSPACE;
    NmsWs ws = nms_ws(workspace, n);
    const size_t lds = sizeof(uint64_t) * (size_t)next_pow2(n);
    hipLaunchKernelGGL(nms_prep_kernel, dim3(1), dim3(1024), lds, s, dets, n, stride, ws);
    const int rows_per_block = 16;
    hipLaunchKernelGGL(nms_mask_kernel, dim3((n + rows_per_block - 1) / rows_per_block),
                       dim3(64 * rows_per_block), 0, s, n, thresh, ws);
    const size_t mask_bytes = sizeof(uint64_t) * (size_t)n * (size_t)((n + 63) / 64);
    const int in_lds = mask_bytes + 2 * kNmsMaxN + 256 <= VD_LDS_BYTES;
    hipLaunchKernelGGL(nms_resolve_kernel, dim3(1), dim3(1024), in_lds ? mask_bytes : 0, s, n, ws,
                       keep, nkeep, in_lds);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
