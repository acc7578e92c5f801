// Shared device helpers for the gfx950 kernels of vosdetectron_amd.
//
// Every translation unit is compiled with -ffp-contract=off: the hot-path
// arithmetic (RoIAlign sample positions / bilinear weights, box decode, IoU)
// must round exactly like the reference's evaluation order, so no a*b+c is
// fused unless a kernel asks for it explicitly with __builtin_fmaf.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define VD_WAVE 64

// gfx950 only: the launches size LDS for its 160 KiB per workgroup (NMS resolve
// in LDS, det_limit's staged rows, soft-NMS at kSoftMax, the proposal select's
// candidate keys) and the MFMA kernels use its instruction set.
#define VD_LDS_BYTES (160 * 1024)
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "vosdetectron_amd kernels target gfx950 (160 KiB LDS per workgroup) only"
#endif

namespace vd {

// Orderable 32-bit key of a float: unsigned comparison of keys == numeric
// comparison of values (-0.0 is folded onto +0.0 so that, as in numpy, the
// two compare equal and fall back to the index tie-break).
__device__ __forceinline__ uint32_t float_key(float f) {
    uint32_t u = __float_as_uint(f);
    if (u == 0x80000000u) u = 0u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_float(uint32_t k) {
    uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    return __uint_as_float(u);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (VD_WAVE - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x / VD_WAVE; }
__device__ __forceinline__ int num_waves() { return (blockDim.x + VD_WAVE - 1) / VD_WAVE; }

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// popcount of the ballot bits below this lane (exclusive lane prefix)
__device__ __forceinline__ int lane_prefix(uint64_t bits) {
    return __popcll(bits & ((1ull << lane_id()) - 1ull));
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
    uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int mask) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, mask);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), mask);
    return ((uint64_t)hi << 32) | lo;
}

// Register form of the bitonic network below: thread t holds elements
// t + e*T (T = blockDim.x, e < E).  Compare-exchange partners i ^ j are another
// lane of the same wave for j < 64 (shuffle, no barrier), another element of
// the same thread for j >= T (register), and otherwise go through LDS (one
// barrier pair per stage).  Every pair ends with (max, min) or (min, max) by
// the same rule as the LDS network, so the sorted array is identical.
template <int E>
__device__ __forceinline__ void bitonic_sort_desc_reg(uint64_t *keys, int n) {
    const int T = blockDim.x, t = threadIdx.x;
    const bool act = t < n;  // n < T: only the first n threads (whole waves) hold data
    uint64_t v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = act ? keys[t + e * T] : 0ull;
    for (int k = 2; k <= n; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= T) {
                const int je = j / T;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int pe = e ^ je;
                    if (pe > e) {
                        const bool desc = ((t + e * T) & k) == 0;
                        const uint64_t a = v[e], b = v[pe];
                        const uint64_t mx = a > b ? a : b, mn = a > b ? b : a;
                        v[e] = desc ? mx : mn;
                        v[pe] = desc ? mn : mx;
                    }
                }
            } else if (j >= 64) {
                __syncthreads();
                if (act) {
#pragma unroll
                    for (int e = 0; e < E; ++e) keys[t + e * T] = v[e];
                }
                __syncthreads();
                if (act) {
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        const int i = t + e * T;
                        const uint64_t b = keys[i ^ j];
                        const bool take_max = ((i & j) == 0) == ((i & k) == 0);
                        v[e] = take_max ? (v[e] > b ? v[e] : b) : (v[e] > b ? b : v[e]);
                    }
                }
            } else if (act) {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const int i = t + e * T;
                    const uint64_t b = shfl_xor64(v[e], j);
                    const bool take_max = ((i & j) == 0) == ((i & k) == 0);
                    v[e] = take_max ? (v[e] > b ? v[e] : b) : (v[e] > b ? b : v[e]);
                }
            }
        }
    }
    __syncthreads();
    if (act) {
#pragma unroll
        for (int e = 0; e < E; ++e) keys[t + e * T] = v[e];
    }
    __syncthreads();
}

__device__ __forceinline__ void bitonic_sort_desc_lds(uint64_t *keys, int n);

// Block-wide descending bitonic sort of n (power of two) 64-bit keys in LDS.
// Register network when blockDim.x is a power of two >= 64, n >= 64 and
// n <= 8 * blockDim.x; the all-LDS network otherwise.
// Forced inline: out of line, the LDS pointer becomes generic (flat accesses).
__device__ __forceinline__ void bitonic_sort_desc(uint64_t *keys, int n) {
    const int T = blockDim.x;
    if (n >= 64 && T >= 64 && (T & (T - 1)) == 0 && (n <= T || n % T == 0)) {
        const int E = n <= T ? 1 : n / T;
        if (E == 1) return bitonic_sort_desc_reg<1>(keys, n);
        if (E == 2) return bitonic_sort_desc_reg<2>(keys, n);
        if (E == 4) return bitonic_sort_desc_reg<4>(keys, n);
        if (E == 8) return bitonic_sort_desc_reg<8>(keys, n);
    }
    bitonic_sort_desc_lds(keys, n);
}

__device__ __forceinline__ void bitonic_sort_desc_lds(uint64_t *keys, int n) {
    for (int k = 2; k <= n; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                int ixj = i ^ j;
                if (ixj > i) {
                    uint64_t a = keys[i], b = keys[ixj];
                    bool desc = (i & k) == 0;
                    if (desc ? (a < b) : (a > b)) {
                        keys[i] = b;
                        keys[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
}

__host__ __device__ inline int next_pow2(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

// Block-wide ORDERED compaction: calls out(pos, i) for every i in [0, n) with
// pred(i) true, pos = rank of i among those (ascending i).  Returns the count
// (same value in every thread).  scratch: LDS int[16] (<= 16 waves).
template <class Pred, class Out>
__device__ inline int block_compact(int n, Pred pred, Out out, int *scratch) {
    const int lane = lane_id(), wave = wave_id(), nw = num_waves();
    int base = 0;
    for (int start = 0; start < n; start += blockDim.x) {
        const int i = start + threadIdx.x;
        const bool p = i < n && pred(i);
        const uint64_t b = ballot(p);
        if (lane == 0) scratch[wave] = __popcll(b);
        __syncthreads();
        int off = base, total = 0;
        for (int w = 0; w < nw; ++w) {
            const int c = scratch[w];
            if (w < wave) off += c;
            total += c;
        }
        if (p) out(off + lane_prefix(b), i);
        base += total;
        __syncthreads();
    }
    return base;
}

// Block-wide sum of one int per thread.  scratch: LDS int[16].
__device__ inline int block_sum(int v, int *scratch) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane_id() == 0) scratch[wave_id()] = v;
    __syncthreads();
    int t = 0;
    for (int w = 0; w < num_waves(); ++w) t += scratch[w];
    __syncthreads();
    return t;
}

// k-th largest (1-based) of n 32-bit keys, by 4 passes of 8-bit radix select
// with wave-aggregated LDS histogram updates.  hist: LDS uint32[256].
template <class Key>
__device__ inline uint32_t block_kth_largest(int n, int k, Key key, uint32_t *hist,
                                             int *scratch) {
    uint32_t prefix = 0, pmask = 0;
    int need = k;
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0;
        __syncthreads();
        for (int start = 0; start < n; start += blockDim.x) {
            const int i = start + threadIdx.x;
            bool act = false;
            uint32_t d = 0;
            if (i < n) {
                const uint32_t kv = key(i);
                act = (kv & pmask) == prefix;
                d = (kv >> shift) & 0xffu;
            }
            uint64_t pending = ballot(act);
            while (pending) {  // one LDS add per distinct digit in the wave
                const int leader = __ffsll((unsigned long long)pending) - 1;
                const uint32_t dl = __builtin_amdgcn_readlane(d, leader);
                const uint64_t same = ballot(act && d == dl);
                if (lane_id() == leader) atomicAdd(&hist[dl], (uint32_t)__popcll(same));
                pending &= ~same;
                if (d == dl) act = false;
            }
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            // the digit holding the need-th largest key, by the first wave: lane l
            // owns bins 255 - 4l .. 252 - 4l (highest first), a wave prefix sum over
            // the lanes' totals, and the first lane whose prefix reaches `need`
            // walks its four bins (one thread walking all 256 bins serially cost
            // ~40 us per launch in LDS round trips)
            const int l = threadIdx.x;
            int h[4], tot = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                h[i] = (int)hist[255 - 4 * l - i];
                tot += h[i];
            }
            int incl = tot;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int v = __shfl_up(incl, o);
                if (l >= o) incl += v;
            }
            const int excl = incl - tot;
            const uint64_t hit = ballot(incl >= need);
            const int first = hit ? __ffsll((unsigned long long)hit) - 1 : 63;
            if (l == first) {
                int acc = excl, digit = 255 - 4 * l - 3;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (acc + h[i] >= need) { digit = 255 - 4 * l - i; break; }
                    acc += h[i];
                }
                scratch[0] = digit;
                scratch[1] = need - acc;
            }
        }
        __syncthreads();
        prefix |= (uint32_t)scratch[0] << shift;
        pmask |= 0xffu << shift;
        need = scratch[1];
        __syncthreads();
    }
    return prefix;
}

// cython_nms.pyx:28-32 max/min (a if a >= b else b), float32
__device__ __forceinline__ float cy_max(float a, float b) { return a >= b ? a : b; }
__device__ __forceinline__ float cy_min(float a, float b) { return a <= b ? a : b; }

// IoU test of cython_nms.pyx:76-85 between the box being kept (i) and a later
// box (j) in processing order.  Exact float32 op order, no contraction.
__device__ __forceinline__ bool suppresses(float ix1, float iy1, float ix2, float iy2, float iarea,
                                           float jx1, float jy1, float jx2, float jy2, float jarea,
                                           float thresh) {
    float xx1 = cy_max(ix1, jx1);
    float yy1 = cy_max(iy1, jy1);
    float xx2 = cy_min(ix2, jx2);
    float yy2 = cy_min(iy2, jy2);
    float w = cy_max(0.0f, xx2 - xx1 + 1.0f);
    float h = cy_max(0.0f, yy2 - yy1 + 1.0f);
    float inter = w * h;
    // Disjoint boxes (most pairs of an NMS) have inter = 0, so ovr = +-0 or NaN:
    // never >= a positive thresh.  A wave with no overlapping pair skips the
    // IEEE division (~10 VALU with a quarter-rate rcp); the result is unchanged.
    if (thresh > 0.f && ballot(inter > 0.f) == 0ull) return false;
    float ovr = inter / (iarea + jarea - inter);
    return ovr >= thresh;
}

}  // namespace vd
