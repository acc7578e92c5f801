// 3x3 stride-1 pad-1 convolution on NHWC fp32 by Winograd F(4x4, 3x3) on the MFMA
// pipes, bias (+ ReLU) epilogue fused (round 5).
//
// Same operator as conv3x3_wino.hip's F(2x2, 3x3) kernel (FPN posthoc / RPN conv,
// lib/modeling/FPN.py:227-258, 376-422; mask head convs, mask_rcnn_heads.py:178-188),
// with every 4x4 output tile computed as
//   Y = A^T [ sum_ci (G g G^T) (.) (B^T d B) ] A        (d: the tile's 6 x 6 patch)
// -- 36 transform positions per 16 outputs instead of 16 per 4: 1.78x fewer MFMA
// multiplies than F(2x2).  Interpolation points 0, +-1, +-2, inf (Lavin & Gray);
// the transforms scale by up to 8 (A) and 5 (B), so the result carries a few times
// F(2x2)'s rounding error (2-4e-6 of max|y| on random 64-256-channel data, vs 2e-6
// for F(2x2) and 4e-7 for a direct fp32 conv).
//
// What keeps F(4x4) on the matrix pipe is the input transform: ~170 flops per (tile,
// input channel), 4x F(2x2)'s.  Round 3's research kernel (tools/research/
// conv3x3_wino4.hip) let every wave transform the patches of its own tiles, 4x
// redundantly across the workgroup's channel groups, and ran at 0.40 of the fp32
// matrix peak.  Here each (tile, channel) is transformed ONCE per workgroup, into
// LDS, and read back by all the waves that need it:
//
//   workgroup = 8 waves (2 per SIMD), 32 tiles (4 x 8 = 16 x 32 output pixels) x 64
//   output channels; wave (tg, cg) owns tiles 16 tg .. + 15 x channels 16 cg .. + 15 at
//   all 36 positions (36 MFMA accumulators, 144 registers; the output transform is
//   lane-local).  K walked in chunks of 8 input channels, three-stage pipeline:
//     patch DMA (LDS-DMA, chunk ch + 2)  |  transform (waves 0-3, chunk ch + 1,
//     patch -> V in LDS)  |  MFMAs (all waves, chunk ch, V from LDS, U from L2)
//   one barrier per chunk.  Waves 0-3 and 4-7 share the SIMDs pairwise, so the
//   partner wave's MFMAs fill a transforming wave's VALU time.
// Per chunk and wave: 72 v_mfma_f32_16x16x4_f32, 36 ds_read_b64 (V), 18 U loads
// (1 KiB each); per transforming lane: 36 ds_read_b32 (patch), ~170 VALU, 36
// ds_write_b32 (V).
//
// Default form (ACC, round 5): the U loads are inline asm with the loop's own vmcnt
// accounting, so no U wait covers a patch DMA piece (the compiler cannot see the asm
// DMAs and, vmcnt retiring in issue order, its own waits did from the fourth position
// of every chunk); the patch DMA is spread over all 8 waves (3 pieces each); V is
// stored [pos][tg][ch / 2][tile % 16][ch & 1] with an XOR swizzle, which makes the
// MFMA waves' V reads conflict-free (the first form's were 4-way conflicted: 66 % of
// its LDS-array cycles).  Bit-identical to the first form (VOSDET_WINO4_ACC=0); P2
// 7.33 -> 7.16 ms, MFMA busy 0.61 -> 0.64 (profiles/r05/wino4acc/).
//
// LDS (120 KiB, one workgroup per CU):
//   V [2][36 pos][32 tiles][8 ch] fp32 (36 KiB a stage): a wave's B fragment of a
//     position is one conflict-free ds_read_b64 (lane (j, q) -> tile 16 tg + j,
//     channels 2q, 2q + 1: the K permutation shared with U, as in F(2x2));
//   patch [2][18 rows][84 16-B slots]: pixel column C's two 4-channel halves at slots
//     2C + C/2 + half (a pad slot every other pixel), so the 64 lanes of a transform
//     read (8 tiles of a tile row x 8 channels) fall in 64 distinct banks.
#include <stdlib.h>

#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int k4Co = 64;             // output channels per workgroup
constexpr int k4KC = 8;              // input channels per chunk
constexpr int k4Threads = 512;       // 8 waves
constexpr int k4TR = 4, k4TC = 8;    // tiles per block: 16 x 32 output pixels
constexpr int k4PR = 4 * k4TR + 2;   // 18 patch rows
constexpr int k4PC = 4 * k4TC + 2;   // 34 patch columns
constexpr int k4RP = 84;             // 16-B slots per patch row
constexpr int k4PSlots = 1536;       // 24 DMA wave instructions (18 x 84 = 1512 used)
constexpr int k4PStageB = k4PSlots * 16;        // 24 KiB
constexpr int k4VStageB = 36 * 32 * k4KC * 4;   // 36 KiB
constexpr int k4ZeroF4 = 1024;                  // zero source for C <= 4096
constexpr int k4LdsB = 2 * k4VStageB + 2 * k4PStageB + 6 * 256 * 4;  // + DMA offsets

__device__ float4 g_wino4_zero[k4ZeroF4];

__device__ __forceinline__ void w4_dma_1k(const float *src, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(lds)
        : "memory");
}

// ACC form: the U fragments through inline-asm buffer loads with the loop's own vmcnt
// accounting.  The compiler cannot see the (inline-asm) patch DMAs, so its own waits
// for compiler-issued U loads undercount the queue by the DMA pieces and, vmcnt
// retiring in issue order, from the fourth position of a chunk every U wait also waits
// for the patch's HBM fetch.  Counted by hand, a DMA is waited for only at the chunk's
// end barrier.
typedef int w4i4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void w4_uload_asm(f4v &r, w4i4 rsrc, uint32_t voff, uint32_t soff) {
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen"
                 : "+v"(r)
                 : "v"(voff), "s"(rsrc), "s"(soff)
                 : "memory");
}
// all but the N youngest vector-memory ops of this wave retired; the fragment passes
// through so its MFMAs cannot be scheduled above the wait
template <int N>
__device__ __forceinline__ void w4_wait_u(f4v &a) {
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(a) : "n"(N) : "memory");
}

// y = B^T x, B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0;
//                   0 2 -1 -2 1 0; 0 4 0 -5 0 1]
__device__ __forceinline__ void w4_bt6(const float (&x)[6], float (&y)[6]) {
    const float t0 = __builtin_fmaf(-4.f, x[2], x[4]), t1 = __builtin_fmaf(-4.f, x[1], x[3]);
    const float t2 = x[4] - x[2], d = x[3] - x[1];
    y[0] = __builtin_fmaf(4.f, x[0], __builtin_fmaf(-5.f, x[2], x[4]));
    y[1] = t0 + t1;
    y[2] = t0 - t1;
    // t2 +- 2 d with 2 d exact: one rounding either way, as t2 +- (2 d) -- 12 VALU a call
    y[3] = __builtin_fmaf(2.f, d, t2);
    y[4] = __builtin_fmaf(-2.f, d, t2);
    y[5] = __builtin_fmaf(4.f, x[1], __builtin_fmaf(-5.f, x[3], x[5]));
}

// w4_bt6 on two independent vectors at once (packed fp32: v_pk_fma_f32 / v_pk_add_f32,
// two lanes' worth of the same IEEE operations, so bit-identical to two w4_bt6 calls)
__device__ __forceinline__ f2v w4_pfma(float a, f2v b, f2v c) {
    return __builtin_elementwise_fma(f2v{a, a}, b, c);
}
__device__ __forceinline__ void w4_bt6v(const f2v (&x)[6], f2v (&y)[6]) {
    const f2v t0 = w4_pfma(-4.f, x[2], x[4]), t1 = w4_pfma(-4.f, x[1], x[3]);
    const f2v t2 = x[4] - x[2], d = x[3] - x[1];
    y[0] = w4_pfma(4.f, x[0], w4_pfma(-5.f, x[2], x[4]));
    y[1] = t0 + t1;
    y[2] = t0 - t1;
    y[3] = w4_pfma(2.f, d, t2);
    y[4] = w4_pfma(-2.f, d, t2);
    y[5] = w4_pfma(4.f, x[1], w4_pfma(-5.f, x[3], x[5]));
}

// y = A^T m, A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
__device__ __forceinline__ void w4_at6(const float (&m)[6], float (&y)[4]) {
    const float s12 = m[1] + m[2], d12 = m[1] - m[2], s34 = m[3] + m[4], d34 = m[3] - m[4];
    y[0] = m[0] + s12 + s34;
    y[1] = __builtin_fmaf(2.f, d34, d12);
    y[2] = __builtin_fmaf(4.f, s34, s12);
    y[3] = __builtin_fmaf(8.f, d34, d12) + m[5];
}

// PROBE (research timing only, VOSDET_WINO4_PROBE; results are wrong when set): bit 0
// no transform, bit 1 no MFMA, bit 2 no patch DMA, bit 3 no U reloads.
// ACC: U loads and their waits counted by hand (w4_uload_asm), the patch DMA spread over
// all 8 waves (3 pieces each, a zero-page piece where no chunk is left) so every wave's
// queue has the same shape
// STAMP (research, VOSDET_WINO4_STAMP=1; outputs unchanged): lane 0 of every wave of
// workgroups < 512 records s_memtime at six points of chunks 8..11 into
// g_wino4_stamps (vd_research_wino4_stamps copies them out)
constexpr int kStampWg = 512, kStampCh0 = 8, kStampNch = 4;
__device__ unsigned long long g_wino4_stamps[kStampWg * 8 * kStampNch * 6];

// IL (ACC form, VOSDET_WINO4_IL): the next chunk's transform interleaved with the
// transforming wave's own MFMAs -- column c of B^T d after position c's MFMAs (its patch
// reads issued one position ahead), row a of (B^T d) B and its V writes after position
// 6 + a -- instead of one block before them (the chunk stamps: 3.6 k cycles of
// transform, during which the SIMD's MFMA pipe is fed by the partner wave alone)
// PK (round 6, the default; VOSDET_WINO4_PK=0 keeps the scalar transform): the input
// transform in packed fp32, bit-identical
template <bool RELU, int PROBE, bool ACC = false, int VD = 1, bool STAMP = false, bool IL = false,
          bool PK = false>
__global__ __launch_bounds__(k4Threads) void conv3x3_wino4_kernel(
    const float *__restrict__ X, int N, int H, int W, int C, const float *__restrict__ U,
    int Cout, const float *__restrict__ bias, float *__restrict__ Y, int tby, int tbx,
    int cb_per_xcd, int probe_hi, int mos, int gin) {
    // static, not dynamic: a > 64 KiB dynamic allocation is honoured by a direct launch
    // after hipFuncSetAttribute but not by the same launch captured into a hipGraph
    // (every replayed P2 conv came out unwritten, round 5)
    __shared__ __attribute__((aligned(16))) char w4_lds[k4LdsB];
    float *const vst = reinterpret_cast<float *>(w4_lds);                  // [2][36][32][8]
    char *const pst = w4_lds + 2 * k4VStageB;                              // [2][1536][16 B]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ncb = Cout / k4Co;
    int cb, sp;
    if (cb_per_xcd) {  // XCD x computes channel block x % ncb: its L2 holds one U block
        const int xcd = blockIdx.x & 7;
        cb = xcd % ncb;
        sp = (blockIdx.x >> 3) * (8 / ncb) + xcd / ncb;
    } else {
        const int r8 = blockIdx.x % (8 * ncb);
        cb = r8 / 8;
        sp = (blockIdx.x / (8 * ncb)) * 8 + (r8 & 7);
    }
    // mos: map-pair mosaic (H, W <= 15, vd_conv3x3_wino4_mosaic_bias_act) -- block sp
    // holds maps 2 sp (columns 0..15) and 2 sp + 1 (columns 16..31), each at the
    // origin of its 16 x 16 cell; taps outside a map read zero, so every output is
    // the map's own padded convolution, bit-identical to one map per block
    // mos >= 4: row stack (vd_conv3x3_wino4_rows_bias_act) -- the N maps stacked at a
    // pitch of hp = mos >> 2 rows (a multiple of 4, > H: every tile inside one map's
    // pitch, the rows past a map zero), one image of N hp rows
    // mos == 3: octets -- maps of at most 7 x 7, eight per block in 8 x 8 cells (2 rows
    // of 4), map n + 4 (y >> 3) + (x >> 3)
    // (mos & 3) == 2: grid (vd_conv3x3_wino4_grid_bias_act, round 6) -- the maps at a
    // pitch of (H + 1) x (W + 1) in rows of gG = mos >> 2 (map gG gy + gx at row gy,
    // column gx), one zero row / column between neighbours: tiles straddle maps, taps
    // in a separator or past the last map read zero and separator outputs are not
    // stored, so every output is its map's own padded convolution (in other tile
    // positions than one map per block: equal within Winograd rounding, not bitwise)
    const bool pair = mos == 1, oct = mos == 3, grid = (mos & 3) == 2;
    const int hp = (mos & 3) == 0 ? mos >> 2 : 0;
    const int gG = grid ? mos >> 2 : 0, gPh = H + 1, gPw = W + 1;
    if (sp >= (pair ? (N + 1) >> 1 : oct ? (N + 7) >> 3 : ((hp || grid) ? tby * tbx : N * tby * tbx))) return;
    const int n = pair ? 2 * sp : oct ? 8 * sp : ((hp || grid) ? 0 : sp / (tby * tbx));
    const int rem = (pair || oct) ? 0 : sp - n * tby * tbx;
    const int tyb = rem / tbx, txb = rem - (rem / tbx) * tbx;
    const int oy0 = 4 * k4TR * tyb, ox0 = 4 * k4TC * txb;
    const int iy0 = oy0 - 1, ix0 = ox0 - 1;
    // gin (grouped, round 6): a workgroup's 64 output channels read only the 64 input
    // channels of their groups -- input channels 64 cb .. + 63 at pixel stride C, U the
    // block-diagonal expansion (zeros between groups) with Cin = 64
    const int nch = ((gin & 1) ? 64 : C) / k4KC;
    const uint32_t pbase = (uint32_t)(uintptr_t)pst;

    // ---- patch DMA (waves 0-3 only, so the U loads of waves 4-7 never wait behind a
    // patch piece): instructions i = wave + 4 k (k < 6) of 24; slot s -> row R, column
    // C = 2 m + (rem >> 1), half rem & 1 (rem = 4: the pad slot).  Sources as 32-bit
    // float offsets in frame n (bit 31: the zero page)
    // gin bit 1 (polyphase, round 6): the N maps are the 4 polyphase sub-maps (parity a,
    // b = sub-map / (N / 4)) of N / 4 maps of 2H x 2W -- a dilation-2 conv run as the
    // plain conv of its sub-maps, read and written at their places in the full maps
    const bool pph = (gin & 2) != 0;
    const int pNr = N >> 2;
    const float *const Xn = X + (pph ? 0 : (int64_t)n * H * W * C) + ((gin & 1) ? 64 * cb : 0);
    // element offset of (sub-)map m, row y, column x
    auto px_off = [&](int m, int y, int x) -> int64_t {
        if (pph) {
            const int ab = m / pNr, nr = m - ab * pNr;
            return (((int64_t)nr * 2 * H + 2 * y + (ab >> 1)) * (2 * W) + 2 * x + (ab & 1));
        }
        return ((int64_t)m * H + y) * W + x;
    };
    // kept in LDS (after the patch stages), not in six registers the MFMA phase needs
    uint32_t *const poff = reinterpret_cast<uint32_t *>(pst + 2 * k4PStageB) + tid;
    constexpr int kDW = ACC ? 8 : 4;  // waves issuing the patch DMA
    constexpr int kDK = 24 / kDW;     // its wave instructions per issuing wave
    constexpr int kPS = ACC ? 512 : 256;
    const float *const zero = reinterpret_cast<const float *>(g_wino4_zero);
    // ACC: each piece's chunk-0 source kept per lane (2 VGPRs a piece; zero-page lanes
    // point into the zero page, which holds C floats, so they may advance with the
    // chunk too): a chunk's DMA address is one 64-bit add per piece, not the ~15 VALU of
    // offset decode and selects per piece the first form spends
    const float *srcp[kDK];
#pragma unroll
    for (int k = 0; k < kDK; ++k) {
        if (!ACC && wave >= 4) break;
        const int s = 64 * (wave + kDW * k) + lane;
        const int R = s / k4RP, u = s - R * k4RP;
        const int m = u / 5, r5 = u - 5 * m;
        const int Cc = 2 * m + (r5 >> 1), hf = r5 & 1;
        const int y = iy0 + R, x = ix0 + Cc;
        // grid: map column gx = x / (W + 1), map row gy = y / (H + 1)
        const int gx = (grid && x >= 0) ? x / gPw : 0, gy = (grid && y >= 0) ? y / gPh : 0;
        // mosaic: cell x >> 4 (map n + cell), column x & 15 of that map
        const int cell = pair ? (x >> 4) : oct ? (x >> 3) : grid ? gx : 0;
        const int xm = pair ? (x & 15) : oct ? (x & 7) : grid ? x - gx * gPw : x;
        // row stack: map y / hp, its row y % hp (octets: map row 4 (y >> 3), row y & 7)
        const int mr = (hp && y >= 0) ? y / hp : (oct && y >= 0) ? 4 * (y >> 3) : grid ? gG * gy : 0;
        const int ly = hp ? y - mr * hp : oct ? (y & 7) : grid ? y - gy * gPh : y;
        const bool ok = R < k4PR && r5 < 4 && Cc < k4PC && (unsigned)ly < (unsigned)H &&
                        y >= 0 && x >= 0 && (unsigned)xm < (unsigned)W && n + cell + mr < N &&
                        (!oct || (cell < 4 && mr < 8)) && (!grid || gx < gG);
        const int64_t po = pph ? px_off(n + cell + mr, ly, xm) : px_off(cell + mr, ly, xm);
        poff[kPS * k] = ok ? (uint32_t)(po * C + 4 * hf)
                           : 0x80000000u | (uint32_t)(4 * hf);
        srcp[k] = ok ? Xn + po * C + 4 * hf : zero + 4 * hf;
    }
    auto dma = [&](int ch, int stage) {
        if constexpr (ACC) {  // ch: the chunk whose data the pieces copy (clamped by the caller)
#pragma unroll
            for (int k = 0; k < kDK; ++k)
                w4_dma_1k(srcp[k] + ch * k4KC,
                          pbase + (uint32_t)(stage * k4PStageB + (wave + kDW * k) * 1024));
            return;
        }  // ch < 0 (ACC): zero-page pieces, queue shape only
        uint32_t oo[kDK];  // all offsets read before the first DMA (one LDS round trip)
#pragma unroll
        for (int k = 0; k < kDK; ++k) oo[k] = poff[kPS * k];
#pragma unroll
        for (int k = 0; k < kDK; ++k) {
            const uint32_t o = oo[k];
            const float *src = (o & 0x80000000u) ? zero + (o & 7u) : Xn + o + ch * k4KC;
            if (ACC && ch < 0) src = zero;
            w4_dma_1k(src, pbase + (uint32_t)(stage * k4PStageB + (wave + kDW * k) * 1024));
        }
    };

    // ---- transform (waves 0-3): lane -> tile (tile row = wave, column tc = lane >> 3),
    // channel ci = lane & 7; reads pixel (4 tr + r, 4 tc + c), channel ci (slot
    // (4 tr + r) * 84 + 10 tc + 2 c + c / 2 + ci / 4, word ci % 4), writes V[pos][tile][ci]
    const int ttc = lane >> 3, tci = lane & 7;
    const float *const tread =
        reinterpret_cast<const float *>(pst) + ((4 * wave) * k4RP + 10 * ttc + (tci >> 2)) * 4 +
        (tci & 3);
    // V[pos][tile][ch] (first form), or (ACC) V[pos][tg][q = ch / 2][j = tile % 16][ch & 1]
    // with the 32-dword row XOR-swizzled by 8 q: the MFMA waves' ds_read2st64_b64 (16-lane
    // groups, bank = dword mod 32) and the transform's ds_write_b32 (32-lane groups) are
    // both conflict-free -- the first form's reads are 4-way conflicted (PMC: 66 % of
    // the LDS-array cycles were conflict cycles)
    const int wtile_j = 8 * (wave & 1) + ttc;
    float *const twrite =
        ACC ? vst + (wave >> 1) * 128 + 32 * (tci >> 1) + ((2 * wtile_j + (tci & 1)) ^ (8 * (tci >> 1)))
            : vst + 64 * wave + lane;
    auto transform = [&](int stage) {
        const float *tp = tread + stage * (k4PStageB / 4);
        float *vp = twrite + stage * (k4VStageB / 4);
        if (PK) {  // packed fp32: columns (c, c + 1), then rows (a, a + 1), in pairs
            f2v t[6][3];  // B^T d: t[a][c / 2] = {row a col c, row a col c + 1}
#pragma unroll
            for (int c = 0; c < 6; c += 2) {
                f2v x[6], y[6];
#pragma unroll
                for (int r = 0; r < 6; ++r)
                    x[r] = f2v{tp[(r * k4RP + 2 * c + (c >> 1)) * 4],
                               tp[(r * k4RP + 2 * (c + 1) + ((c + 1) >> 1)) * 4]};
                w4_bt6v(x, y);
#pragma unroll
                for (int a = 0; a < 6; ++a) t[a][c >> 1] = y[a];
            }
#pragma unroll
            for (int a = 0; a < 6; a += 2) {
                f2v x[6], y[6];
#pragma unroll
                for (int c = 0; c < 6; ++c)
                    x[c] = f2v{t[a][c >> 1][c & 1], t[a + 1][c >> 1][c & 1]};
                w4_bt6v(x, y);
#pragma unroll
                for (int b = 0; b < 6; ++b) {
                    vp[(6 * a + b) * 256] = y[b][0];
                    vp[(6 * (a + 1) + b) * 256] = y[b][1];
                }
            }
            return;
        }
        float t[6][6];  // B^T d: column c's 6 values
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            float x[6], y[6];
#pragma unroll
            for (int r = 0; r < 6; ++r) x[r] = tp[(r * k4RP + 2 * c + (c >> 1)) * 4];
            w4_bt6(x, y);
#pragma unroll
            for (int a = 0; a < 6; ++a) t[a][c] = y[a];
        }
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            float y[6];
            w4_bt6(t[a], y);
#pragma unroll
            for (int b = 0; b < 6; ++b) vp[(6 * a + b) * 256] = y[b];
        }
    };

    // ---- MFMAs: wave (tg = wave >> 2, cg = wave & 3), lane (j, q): V fragment of tile
    // 16 tg + j, channels 2q, 2q + 1; U fragment of channel 16 cg + j (U's layout
    // [Cout/64][C/8][cg][pp = pos / 2][lane][4], element 2 (pos & 1) + (ci & 1),
    // conv3x3_wino4_weight_kernel)
    const int tg = wave >> 2, cg = wave & 3;
    const int j = lane & 15, q = lane >> 4;
    const f2v *const vread = reinterpret_cast<const f2v *>(
        ACC ? vst + 128 * tg + 32 * q + ((2 * j) ^ (8 * q)) : vst + (16 * tg + j) * 8 + 2 * q);
    // U through a buffer resource: wave-uniform base and per-position offsets in scalar
    // registers, one VGPR (the lane's 16 B) for all loads
    const __amdgpu_buffer_rsrc_t urs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(U) + (int64_t)__builtin_amdgcn_readfirstlane(
                                     (cb * nch * 4 + cg) * (18 * 64)) * 4,
        (short)0, nch * 4 * 18 * 64 * 16, 0x00020000);
    const int uvoff = lane * 16;
    auto uload = [&](int ch, int pos) {  // chunk ch, position pair pos
        return __builtin_bit_cast(
            f4v, __builtin_amdgcn_raw_buffer_load_b128(urs, uvoff,
                                                       (ch * 4 * 18 + pos) * 1024, 0));
    };
    // the same resource as four SGPR words for the inline-asm loads (ACC)
    const uintptr_t uaddr = (uintptr_t)(U + (int64_t)__builtin_amdgcn_readfirstlane(
                                                (cb * nch * 4 + cg) * (18 * 64)) * 4);
    const w4i4 ursv = {__builtin_amdgcn_readfirstlane((int)(uint32_t)uaddr),
                       __builtin_amdgcn_readfirstlane((int)(uint32_t)(uaddr >> 32) & 0xffff),
                       __builtin_amdgcn_readfirstlane(nch * 4 * 18 * 64 * 16), 0x00020000};
    auto uload_acc = [&](f4v &r, int ch, int pos) {
        w4_uload_asm(r, ursv, (uint32_t)uvoff,
                     (uint32_t)__builtin_amdgcn_readfirstlane((ch * 4 * 18 + pos) * 1024));
    };
    f4v acc[36];
#pragma unroll
    for (int p = 0; p < 36; ++p) acc[p] = f4v{0.f, 0.f, 0.f, 0.f};
    // U fragments: a ring of 9 (positions 2 pp, 2 pp + 1 each); after the MFMAs of pp
    // its slot is reloaded with pp + 9 of this chunk, then with pp - 9 of the next
    // chunk, so the next chunk's first half is in flight across the barrier
    constexpr int kUR = 9;  // divides 18: position q of every chunk in slot q % kUR
    f4v u[kUR];
    // V fragments are read one position ahead; a scheduling barrier after every
    // position keeps the U reloads where they are written (left to itself the compiler
    // sinks them next to their use, and each of the second half's positions then waits
    // a full L2 round trip) and the V read of position pp + 1 ahead of pp's MFMAs.
    // xon (waves 0-3): the next chunk's transform rides along -- column c of B^T d at
    // position c (its patch reads one position ahead), row a of (B^T d) B and its V
    // writes at position 6 + a -- so its VALU issues between this wave's own MFMAs and
    // the four SIMDs' two waves reach the barrier together.
    auto mfma_chunk = [&](bool xon, int stage, int ch, int chn, int tstage) {
        const f2v *vp = vread + stage * (k4VStageB / 8);
        const float *tpi = tread + tstage * (k4PStageB / 4);
        float *vpw = twrite + tstage * (k4VStageB / 4);
        float xc[6], tt[6][6];
        if (IL && xon) {
#pragma unroll
            for (int r = 0; r < 6; ++r) xc[r] = tpi[(r * k4RP) * 4];
        }
        if (!IL && xon) {
            // probe_hi bit 1 (VOSDET_WINO4_PRIO=1): the transform at wave priority 1
            if (probe_hi & 2) asm volatile("s_setprio 1" ::: "memory");
            transform(tstage);
            if (probe_hi & 2) asm volatile("s_setprio 0" ::: "memory");
        }
        // V of positions pp .. pp + VD - 1 in a ring (VD > 1: more LDS latency hidden
        // behind one wave's own MFMAs while its SIMD partner transforms)
        f2v vq[VD][2];
#pragma unroll
        for (int d = 0; d < VD; ++d) {
            vq[d][0] = vp[(2 * d) * 128];
            vq[d][1] = vp[(2 * d + 1) * 128];
        }
        f2v b0 = vq[0][0], b1 = vq[0][1];
#pragma unroll
        for (int pp = 0; pp < 18; ++pp) {
            f2v n0, n1;
            if (pp + VD < 18) {
                n0 = vp[(2 * (pp + VD)) * 128];
                n1 = vp[(2 * (pp + VD) + 1) * 128];
            }
            if constexpr (ACC) {
                // younger than U(ch, pp <= 8) (issued last chunk): its 8 - pp successors,
                // the 3 DMA pieces, this chunk's pp reloads; U(ch, pp >= 9): 8 reloads
                if (pp < kUR)
                    w4_wait_u<kUR - 1 + kDK>(u[pp % kUR]);
                else
                    w4_wait_u<kUR - 1>(u[pp % kUR]);
            }
            const f4v uf = u[pp % kUR];
            if constexpr (!(PROBE & 2)) {
            acc[2 * pp] = __builtin_amdgcn_mfma_f32_16x16x4f32(uf.x, b0.x, acc[2 * pp], 0, 0, 0);
            acc[2 * pp] = __builtin_amdgcn_mfma_f32_16x16x4f32(uf.y, b0.y, acc[2 * pp], 0, 0, 0);
            acc[2 * pp + 1] =
                __builtin_amdgcn_mfma_f32_16x16x4f32(uf.z, b1.x, acc[2 * pp + 1], 0, 0, 0);
            acc[2 * pp + 1] =
                __builtin_amdgcn_mfma_f32_16x16x4f32(uf.w, b1.y, acc[2 * pp + 1], 0, 0, 0);
            } else {
                acc[2 * pp][0] += b0.x + b1.y;
            }
            if constexpr (ACC) {
                if (pp + kUR < 18)
                    uload_acc(u[pp % kUR], ch, pp + kUR);
                else
                    uload_acc(u[pp % kUR], chn, pp + kUR - 18);
            } else if constexpr (!(PROBE & 8)) {
                if (pp + kUR < 18)
                    u[pp % kUR] = uload(ch, pp + kUR);
                else
                    u[pp % kUR] = uload(chn, pp + kUR - 18);
            }
            if constexpr (IL) {
                if (xon && pp < 6) {  // column pp of B^T d, then column pp + 1's reads
                    float y[6];
                    w4_bt6(xc, y);
#pragma unroll
                    for (int a = 0; a < 6; ++a) tt[a][pp] = y[a];
                    if (pp < 5) {
                        const int c = pp + 1;
#pragma unroll
                        for (int r = 0; r < 6; ++r) xc[r] = tpi[(r * k4RP + 2 * c + (c >> 1)) * 4];
                    }
                } else if (xon && pp < 12) {  // row pp - 6 of (B^T d) B -> V
                    const int a = pp - 6;
                    float y[6];
                    w4_bt6(tt[a], y);
#pragma unroll
                    for (int b = 0; b < 6; ++b) vpw[(6 * a + b) * 256] = y[b];
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            if (pp + VD < 18) {
                vq[pp % VD][0] = n0;
                vq[pp % VD][1] = n1;
            }
            if (pp < 17) {
                b0 = vq[(pp + 1) % VD][0];
                b1 = vq[(pp + 1) % VD][1];
            }
        }
    };

    // ---- pipeline: prologue (chunk 0 transformed, chunk 1's patch landed)
    if constexpr (ACC) {
#pragma unroll
        for (int i = 0; i < kUR; ++i) {
            u[i] = f4v{0.f, 0.f, 0.f, 0.f};
            uload_acc(u[i], 0, i);
        }
        // chunks 0 and 1 fetched together: one HBM round trip in the prologue, not two
        dma(0, 0);
        dma(nch > 1 ? 1 : 0, 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kDK) : "memory");  // U and chunk 0 landed
        __syncthreads();
        if (wave < 4) transform(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int ch = 0; ch < nch; ++ch) {
            const int sv = ch & 1;
            const int chn = ch + 1 < nch ? ch + 1 : ch;
            if constexpr (STAMP) {
                const bool st = blockIdx.x < kStampWg && ch >= kStampCh0 && ch < kStampCh0 + kStampNch;
                unsigned long long *sp_ = g_wino4_stamps +
                    ((blockIdx.x * 8 + wave) * kStampNch + (ch - kStampCh0)) * 6;
                unsigned long long t[6];
                t[0] = __builtin_amdgcn_s_memtime();
                dma(ch + 2 < nch ? ch + 2 : nch - 1, sv);
                t[1] = __builtin_amdgcn_s_memtime();
                if (!IL && wave < 4 && ch + 1 < nch) transform(sv ^ 1);
                t[2] = __builtin_amdgcn_s_memtime();
                mfma_chunk(IL && wave < 4 && ch + 1 < nch, sv, ch, chn, sv ^ 1);
                t[3] = __builtin_amdgcn_s_memtime();
                asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
                t[4] = __builtin_amdgcn_s_memtime();
                __syncthreads();
                t[5] = __builtin_amdgcn_s_memtime();
                if (st && lane == 0) {
#pragma unroll
                    for (int i = 0; i < 6; ++i) sp_[i] = t[i];
                }
                continue;
            }
            // every wave, every chunk: 3 pieces (past the last chunk, a copy of it into
            // the stage no transform reads again, so the queue keeps its shape)
            dma(ch + 2 < nch ? ch + 2 : nch - 1, sv);
            mfma_chunk(wave < 4 && ch + 1 < nch, sv, ch, chn, sv ^ 1);
            asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
            __syncthreads();
        }
    } else {
#pragma unroll
    for (int i = 0; i < kUR; ++i) u[i] = uload(0, i);
    if (wave < 4) dma(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wave < 4) transform(0);
    if (wave < 4 && nch > 1) dma(1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
        const int sv = ch & 1;
        const int chn = ch + 1 < nch ? ch + 1 : ch;
        if (!(PROBE & 4) && wave < 4 && ch + 2 < nch) dma(ch + 2, sv);  // stage sv: chunk ch, transformed
        // one code path for all waves (a separate transform-free copy of the loop
        // doubles the live ranges the register allocator sees across the branch)
        mfma_chunk(!(PROBE & 1) && wave < 4 && ch + 1 < nch, sv, ch, chn, sv ^ 1);
        // chunk ch + 2's patch (issued before the 18 U loads of this chunk's MFMA
        // phase) landed; the next chunk's 9 U loads may stay in flight
        asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        __syncthreads();
    }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- output transform (lane-local): accumulator slot r of lane (j, q) holds output
    // channel 64 cb + 16 cg + 4 q + r of tile 16 tg + j
    const int tile = 16 * tg + j, tr = tile >> 3, tc = tile & 7;
    const int co = cb * k4Co + 16 * cg + 4 * q;
    const float4 bv = bias ? *reinterpret_cast<const float4 *>(bias + co)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
    float o[16][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float tt[4][6];
#pragma unroll
        for (int b = 0; b < 6; ++b) {
            float m[6], y[4];
#pragma unroll
            for (int a = 0; a < 6; ++a) m[a] = acc[6 * a + b][r];
            w4_at6(m, y);
#pragma unroll
            for (int i = 0; i < 4; ++i) tt[i][b] = y[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float y[4];
            w4_at6(tt[i], y);
#pragma unroll
            for (int k = 0; k < 4; ++k) o[4 * i + k][r] = y[k];
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int yv = oy0 + 4 * tr + i;
        const int gy = grid ? yv / gPh : 0;
        const int mr = hp ? yv / hp : oct ? 4 * (yv >> 3) : grid ? gG * gy : 0;
        const int yy = hp ? yv - mr * hp : oct ? (yv & 7) : grid ? yv - gy * gPh : yv;
        if (yy >= H || n + mr >= N) continue;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int xc = ox0 + 4 * tc + k;
            const int gx = grid ? xc / gPw : 0;
            const int ncell = pair ? n + (xc >> 4) : oct ? n + mr + (xc >> 3) : n + mr + gx;
            const int xx = pair ? (xc & 15) : oct ? (xc & 7) : grid ? xc - gx * gPw : xc;
            if (xx >= W || ncell >= N || (grid && gx >= gG)) continue;
            float4 v = make_float4(o[4 * i + k][0] + bv.x, o[4 * i + k][1] + bv.y,
                                   o[4 * i + k][2] + bv.z, o[4 * i + k][3] + bv.w);
            if (RELU) {
                v.x = fmaxf(v.x, 0.f);
                v.y = fmaxf(v.y, 0.f);
                v.z = fmaxf(v.z, 0.f);
                v.w = fmaxf(v.w, 0.f);
            }
            // probe_hi bit 0 (research, VOSDET_WINO4_PROBE bit 4): no output stores (a
            // store the data never takes keeps the values live)
            if (!(probe_hi & 1) || v.x == 1234.5678f)
                *reinterpret_cast<float4 *>(Y + px_off(ncell, yy, xx) * Cout + co) = v;
        }
    }
}

// ---------------------------------------------------------------------------------
// Position-split form (round 5, VOSDET_WINO4_PS): the same block (32 tiles x 64 output
// channels, 8-channel chunks, patch DMA -> transform -> MFMA pipeline), but a wave owns
// a set of transform POSITIONS for all 64 channels x 32 tiles instead of all 36
// positions for 16 channels x 16 tiles:
//   waves 0-3: positions 5 w .. 5 w + 4 (MFMAs only), waves 4-7: positions 20 + 4 v ..
//   + 3 (and the patch DMA + transform); each SIMD pairs a 5- and a 4-position wave:
//   144 MFMAs per SIMD per chunk, as before.
//   per position and chunk: 2 V fragments (ds_read_b64) and 4 U fragments (b64 buffer
//   loads) feed 16 MFMAs (was 2 + 1 b128 for 4): a quarter of the V reads and half the
//   U bytes per workgroup, and 16 independent MFMAs between dependences instead of 4.
// The output transform needs all 36 positions of a (tile, channel): after the K loop
// the accumulators go through LDS in four 16-channel rounds (positions 0-15 in the V
// stage 0 array, 16-31 in V stage 1, 32-35 in patch stage 0), one (tile, channel) per
// thread.  The MFMA operands, their order and the output transform are the first
// form's, so the results are bit-identical to it.
// Patch fill through registers (three LDS stages: loaded at the end of one chunk,
// written at the end of the next), not LDS-DMA: the asm DMA is invisible to the
// compiler's vmcnt bookkeeping, so a wait for a U load issued before a DMA also waited
// for the DMA; the builtin is counted but makes every barrier wait for all loads.
constexpr int k4VStageF = 36 * 32 * k4KC;  // floats per V stage
constexpr int k4XS = 32 * 16;              // exchange floats per position (16 ch x 32 tiles)

template <bool RELU, int NP, bool XW, int PP>
__device__ __forceinline__ void wino4ps_body(
    const float *__restrict__ Xn, int H, int W, int C, const float *__restrict__ U, int Cout,
    const float *__restrict__ bias, float *__restrict__ Y, int n, int cb, int oy0, int ox0,
    float4 *pst, float *vs, uint32_t *poff, int wave, int lane) {
    const int nch = C / k4KC;
    const int p0 = XW ? 20 + 4 * (wave - 4) : 5 * wave;
    const int tw = wave & 3;  // XW: transform tile row / DMA instruction group
    const int j = lane & 15, q = lane >> 4;
    const int tid = wave * 64 + lane;

    // ---- patch fill (XW waves): slot group i = tw + 4 k (k < 6) of 24, sources from the
    // offsets in poff (bit 31: the zero page), loaded into registers at the start of a
    // chunk and written to the stage at its end: ordinary compiler-counted loads, so no
    // wait ever covers more than it needs (an LDS-DMA either hid from the compiler's
    // vmcnt counts -- asm -- or, as the builtin, made it wait for everything at each
    // barrier)
    const float *const zero = reinterpret_cast<const float *>(g_wino4_zero);
    // (inline in the chunk body, not lambdas over a captured array: a captured
    // register array is kept in scratch memory)
#define VD_W4PS_PLOAD(CH, PR)                                                              \
    {                                                                                      \
        uint32_t oo_[6];                                                                   \
        _Pragma("unroll") for (int k = 0; k < 6; ++k) oo_[k] = poff[256 * k + (tid - 256)]; \
        _Pragma("unroll") for (int k = 0; k < 6; ++k) {                                    \
            const uint32_t o = oo_[k];                                                     \
            const float *src = (o & 0x80000000u) ? zero + (o & 7u) : Xn + o + (CH) * k4KC; \
            PR[k] = *reinterpret_cast<const f4v *>(src);                                   \
        }                                                                                  \
    }
#define VD_W4PS_PSTORE(STAGE, PR)                                                          \
    _Pragma("unroll") for (int k = 0; k < 6; ++k)                                          \
        *reinterpret_cast<f4v *>((STAGE) + (tw + 4 * k) * 64 + lane) = PR[k];
    // ---- transform (XW waves): as the first form's, tile row tw
    const int ttc = lane >> 3, tci = lane & 7;
    const int tro = ((4 * tw) * k4RP + 10 * ttc + (tci >> 2)) * 4 + (tci & 3);
    auto transform = [&](const float4 *pstage, float *vstage) {
        const float *tp = reinterpret_cast<const float *>(pstage) + tro;
        float t[6][6];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            float x[6], y[6];
#pragma unroll
            for (int r = 0; r < 6; ++r) x[r] = tp[(r * k4RP + 2 * c + (c >> 1)) * 4];
            w4_bt6(x, y);
#pragma unroll
            for (int a = 0; a < 6; ++a) t[a][c] = y[a];
        }
        float *vp = vstage + 64 * tw + lane;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            float y[6];
            w4_bt6(t[a], y);
#pragma unroll
            for (int b = 0; b < 6; ++b) vp[(6 * a + b) * 256] = y[b];
        }
    };

    // ---- U: the first form's layout [Cout/64][C/8][cg][pp][lane][4], element
    // 2 (pos & 1) + (ci & 1): co-tile i of position p is the float2 at
    // (((ch * 4 + i) * 18 + p / 2) * 64 + lane) * 4 + 2 (p & 1)
    const __amdgpu_buffer_rsrc_t urs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(U) + (int64_t)__builtin_amdgcn_readfirstlane(cb * nch * 4 * 18 * 256),
        (short)0, nch * 4 * 18 * 64 * 16, 0x00020000);
    const int uvoff = lane * 16;
    auto uload = [&](int ch, int p, int i) {
        return __builtin_bit_cast(
            f2v, __builtin_amdgcn_raw_buffer_load_b64(
                     urs, uvoff + 8 * (p & 1), ((ch * 4 + i) * 18 + (p >> 1)) * 1024, 0));
    };
    // U: a whole chunk's positions in registers.  MFMA-only waves reload position k's
    // slot for the next chunk right after its MFMAs; the transforming waves load the
    // next chunk's batch at the end of the chunk, BEFORE their patch loads: vmcnt
    // retires loads in issue order, so a U load issued after a patch load (HBM, the
    // longest latency here) could not be waited for without waiting for the patch
    constexpr int UR = NP;
    f2v ub[UR][4];
#pragma unroll
    for (int k = 0; k < UR; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) ub[k][i] = uload(0, p0 + k, i);

    f4v acc[NP][4][2];
#pragma unroll
    for (int k = 0; k < NP; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int g = 0; g < 2; ++g) acc[k][i][g] = f4v{0.f, 0.f, 0.f, 0.f};

    // V fragment of position p, tile group g: lane (j, q) -> tile 16 g + j, channels 2q, 2q+1
    const int vro = (16 * 0 + j) * 8 + 2 * q;
    // Patch pipeline, three stages: the registers loaded at the END of chunk ch (patch
    // of chunk ch + 3, the last memory loads the chunk issues, so no U wait ever sits
    // behind them) are written to their stage at the end of chunk ch + 1 and
    // transformed during chunk ch + 2.
    f4v pr[6];  // f4v, not float4: an array of the struct type stays in scratch
    auto chunk = [&](int ch) {
        if (XW) {
            // no scheduling barrier: the compiler interleaves the transform's VALU and
            // LDS traffic with this wave's first MFMAs (serialised it cost 1.8 ms at P2)
            if (!(PP & 1) && ch + 1 < nch)
                transform(pst + ((ch + 1) % 3) * k4PSlots, vs + ((ch + 1) & 1) * k4VStageF);
        }
        const int chn = ch + 1 < nch ? ch + 1 : ch;
        const f2v *vp = reinterpret_cast<const f2v *>(vs + (ch & 1) * k4VStageF + vro);
        f2v v0 = vp[(p0 * 256) / 2], v1 = vp[(p0 * 256 + 128) / 2];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const int p = p0 + k;
            f2v n0, n1;
            if (k + 1 < NP) {
                n0 = vp[((p + 1) * 256) / 2];
                n1 = vp[((p + 1) * 256 + 128) / 2];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const f2v u = ub[k][i];
                if constexpr (PP & 2) {  // research probe: no MFMAs
                    acc[k][i][0][0] += u.x + v0.x + v1.y;
                } else {
                acc[k][i][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(u.x, v0.x, acc[k][i][0], 0, 0, 0);
                acc[k][i][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(u.y, v0.y, acc[k][i][0], 0, 0, 0);
                acc[k][i][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(u.x, v1.x, acc[k][i][1], 0, 0, 0);
                acc[k][i][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(u.y, v1.y, acc[k][i][1], 0, 0, 0);
                }
            }
            if (!XW) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (!(PP & 8)) ub[k][i] = uload(chn, p, i);
            }
            __builtin_amdgcn_sched_barrier(0);
            if (k + 1 < NP) {
                v0 = n0;
                v1 = n1;
            }
        }
        if (XW) {
#pragma unroll
            for (int k = 0; k < NP; ++k)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (!(PP & 8)) ub[k][i] = uload(chn, p0 + k, i);
            __builtin_amdgcn_sched_barrier(0);
            // unconditional (past the last chunk: the last chunk's patch again, into a
            // stage nothing reads)
            if constexpr (!(PP & 4)) {
                VD_W4PS_PSTORE(pst + ((ch + 2) % 3) * k4PSlots, pr)
                VD_W4PS_PLOAD(ch + 3 < nch ? ch + 3 : nch - 1, pr)
            }
        }
        __syncthreads();
    };

    // ---- prologue: patches 0 and 1 in their stages, chunk 0 transformed, patch 2 in
    // the registers
    if (XW) {
        VD_W4PS_PLOAD(0, pr)
        VD_W4PS_PSTORE(pst, pr)
        VD_W4PS_PLOAD(nch > 1 ? 1 : 0, pr)
        VD_W4PS_PSTORE(pst + k4PSlots, pr)
    }
    __syncthreads();
    if (XW) {
        VD_W4PS_PLOAD(nch > 2 ? 2 : nch - 1, pr)
        transform(pst, vs);
    }
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) chunk(ch);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef VD_W4PS_PLOAD
#undef VD_W4PS_PSTORE

    // ---- output: four rounds of 16 channels (co-tile rr) through LDS, then one
    // (tile, channel) per thread: tile = tid >> 4, channel 16 rr + (tid & 15)
    float *const xs0 = vs, *const xs1 = vs + k4VStageF, *const xs2 = reinterpret_cast<float *>(pst);
    auto xpos = [&](int p) {  // exchange base of position p
        return p < 16 ? xs0 + p * k4XS : (p < 32 ? xs1 + (p - 16) * k4XS : xs2 + (p - 32) * k4XS);
    };
    const int otile = tid >> 4, och = tid & 15;
    const int otr = otile >> 3, otc = otile & 7;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
#pragma unroll
        for (int k = 0; k < NP; ++k)
#pragma unroll
            for (int g = 0; g < 2; ++g)
                *reinterpret_cast<f4v *>(xpos(p0 + k) + (16 * g + j) * 16 + 4 * q) = acc[k][rr][g];
        __syncthreads();
        float m[36];
#pragma unroll
        for (int p = 0; p < 36; ++p) m[p] = xpos(p)[otile * 16 + och];
        float tt[4][6];
#pragma unroll
        for (int b = 0; b < 6; ++b) {
            float mm[6], y[4];
#pragma unroll
            for (int a = 0; a < 6; ++a) mm[a] = m[6 * a + b];
            w4_at6(mm, y);
#pragma unroll
            for (int i = 0; i < 4; ++i) tt[i][b] = y[i];
        }
        const int co = cb * k4Co + 16 * rr + och;
        const float bv = bias ? bias[co] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float y[4];
            w4_at6(tt[i], y);
            const int yy = oy0 + 4 * otr + i;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int xx = ox0 + 4 * otc + k;
                float v = y[k] + bv;
                if (RELU) v = fmaxf(v, 0.f);
                if (yy < H && xx < W && (!(PP & 16) || v == 1234.5678f))
                    Y[(((int64_t)n * H + yy) * W + xx) * Cout + co] = v;
            }
        }
        __syncthreads();
    }
}

// PP: research probes (VOSDET_WINO4_PSPROBE; wrong results when set): 1 no transform,
// 2 no MFMAs, 4 no patch loads / stores, 8 no U reloads, 16 no output stores
template <bool RELU, int PP>
__global__ __launch_bounds__(k4Threads) void conv3x3_wino4ps_kernel(
    const float *__restrict__ X, int N, int H, int W, int C, const float *__restrict__ U,
    int Cout, const float *__restrict__ bias, float *__restrict__ Y, int tby, int tbx,
    int cb_per_xcd) {
    __shared__ __attribute__((aligned(16))) float4 pst[3 * k4PSlots];
    __shared__ __attribute__((aligned(16))) float vs[2 * k4VStageF];
    __shared__ uint32_t poff[6 * 256];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ncb = Cout / k4Co;
    int cb, sp;
    if (cb_per_xcd) {
        const int xcd = blockIdx.x & 7;
        cb = xcd % ncb;
        sp = (blockIdx.x >> 3) * (8 / ncb) + xcd / ncb;
    } else {
        const int r8 = blockIdx.x % (8 * ncb);
        cb = r8 / 8;
        sp = (blockIdx.x / (8 * ncb)) * 8 + (r8 & 7);
    }
    if (sp >= N * tby * tbx) return;
    const int n = sp / (tby * tbx);
    const int rem = sp - n * tby * tbx;
    const int tyb = rem / tbx, txb = rem - (rem / tbx) * tbx;
    const int oy0 = 4 * k4TR * tyb, ox0 = 4 * k4TC * txb;
    const int iy0 = oy0 - 1, ix0 = ox0 - 1;
    // DMA source offsets of the XW waves (4-7): slot s of instruction tw + 4 k, as the
    // first form's
    if (wave >= 4) {
        const int tw = wave & 3;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int s = 64 * (tw + 4 * k) + lane;
            const int R = s / k4RP, u = s - R * k4RP;
            const int m = u / 5, r5 = u - 5 * m;
            const int Cc = 2 * m + (r5 >> 1), hf = r5 & 1;
            const int y = iy0 + R, x = ix0 + Cc;
            const bool ok = R < k4PR && r5 < 4 && Cc < k4PC && (unsigned)y < (unsigned)H &&
                            (unsigned)x < (unsigned)W;
            poff[256 * k + (tid - 256)] =
                ok ? (uint32_t)((y * W + x) * C + 4 * hf) : 0x80000000u | (uint32_t)(4 * hf);
        }
    }
    const float *const Xn = X + (int64_t)n * H * W * C;
    if (wave < 4)
        wino4ps_body<RELU, 5, false, PP>(Xn, H, W, C, U, Cout, bias, Y, n, cb, oy0, ox0, pst, vs, poff,
                                     wave, lane);
    else
        wino4ps_body<RELU, 4, true, PP>(Xn, H, W, C, U, Cout, bias, Y, n, cb, oy0, ox0, pst, vs, poff,
                                    wave, lane);
}

// U = G g G^T of the PyTorch weight w[co][ci][3][3], G = [1/4 0 0; -1/6 -1/6 -1/6;
// -1/6 1/6 -1/6; 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1], float64, rounded once; stored
// in the kernel's fragment order [co / 64][ci / 8][cg = co % 64 / 16][pp = pos / 2]
// [lane = 16 (ci % 8 / 2) + co % 16][2 (pos & 1) + (ci & 1)], pos = 6 a + b.
__global__ void wino4_weight_kernel(const float *__restrict__ w, int Cout, int C,
                                    float *__restrict__ U) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)Cout * C) return;
    const int co = (int)(i / C), ci = (int)(i - (int64_t)(i / C) * C);
    const int cl = co % k4Co, nch = C / k4KC;
    const int lane = 16 * ((ci & 7) >> 1) + (cl & 15);
    float *dst = U + ((((int64_t)(co / k4Co) * nch + ci / k4KC) * 4 + (cl >> 4)) * 18) * 256 +
                 lane * 4 + (ci & 1);
    const float *g = w + i * 9;
    const double Gm[6][3] = {{0.25, 0., 0.},
                             {-1. / 6, -1. / 6, -1. / 6},
                             {-1. / 6, 1. / 6, -1. / 6},
                             {1. / 24, 1. / 12, 1. / 6},
                             {1. / 24, -1. / 12, 1. / 6},
                             {0., 0., 1.}};
    double t[6][3];  // G g
    for (int a = 0; a < 6; ++a)
        for (int c = 0; c < 3; ++c)
            t[a][c] = Gm[a][0] * g[c] + Gm[a][1] * g[3 + c] + Gm[a][2] * g[6 + c];
    for (int a = 0; a < 6; ++a)
        for (int b = 0; b < 6; ++b) {
            const double u = t[a][0] * Gm[b][0] + t[a][1] * Gm[b][1] + t[a][2] * Gm[b][2];
            const int pos = 6 * a + b;
            dst[(pos >> 1) * 256 + (pos & 1) * 2] = (float)u;
        }
}

}  // namespace

bool conv3x3_wino4_supported(int C, int Cout) {
    return C % k4KC == 0 && C >= k4KC && C <= 4 * k4ZeroF4 && Cout % k4Co == 0 && Cout >= k4Co;
}

size_t conv3x3_wino4_weight_floats(int Cout, int C) { return (size_t)Cout * C * 36; }

int launch_conv3x3_wino4_weight(const float *w, int Cout, int C, float *U, hipStream_t s) {
    const int64_t n = (int64_t)Cout * C;
    if (n == 0) return VD_OK;
    if (!conv3x3_wino4_supported(C, Cout)) return VD_ERR_SHAPE;
    hipLaunchKernelGGL(wino4_weight_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w,
                       Cout, C, U);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

int launch_conv3x3_wino4(const float *X, int N, int H, int W, int C, const float *U, int Cout,
                         const float *bias, int relu, float *Y, hipStream_t s, int mos,
                         int groups) {
    if ((int64_t)N * H * W == 0) return VD_OK;
    if (!conv3x3_wino4_supported(C, Cout)) return VD_ERR_SHAPE;
    // grouped: C == Cout, 64 input channels per 64-channel output block (C / groups
    // divides 64); the pair / octet / grid mosaics stay dense-only
    // groups == -2: polyphase (X / Y are N / 4 maps of 2H x 2W; the N sub-maps of H x W
    // their parity planes): plain, pair / octet layouts only
    int gin = groups > 1;
    if (groups == -2) {
        if (N % 4 || mos == 2 || (int64_t)N * H * W * (C > Cout ? C : Cout) >=
                                                 ((int64_t)1 << 31))
            return VD_ERR_SHAPE;
        gin = 2;
    } else if (gin && (groups < 1 || C != Cout || C % 64 || C % groups ||
                       64 % (C / groups) || mos == 1 || mos == 4)) {
        return VD_ERR_SHAPE;
    }
    if ((int64_t)N * H * W * C >= ((int64_t)1 << 40) || (int64_t)H * W * C >= ((int64_t)1 << 31))
        return VD_ERR_SHAPE;
    // the map-pair mosaic: two maps of at most 15 x 15 per 16 x 32 block (the 16 x 16
    // cell keeps a zero column / row after each map), 2 H W C floats of offsets < 2^31
    if (mos == 1 && (H > 15 || W > 15 || (int64_t)2 * H * W * C >= ((int64_t)1 << 31)))
        return VD_ERR_SHAPE;
    if (mos == 1 && H <= 7 && W <= 7) mos = 3;  // octets: eight maps per block
    if (mos == 3 && (int64_t)8 * H * W * C >= ((int64_t)1 << 31)) return VD_ERR_SHAPE;
    // the row stack: pitch = H + 1 rounded up to 4 (a zero row after every map), one
    // image whose offsets stay 32-bit
    const int hp = (H + 1 + 3) / 4 * 4;
    if (mos == 2) {
        if ((int64_t)N * H * W * C >= ((int64_t)1 << 31) || (int64_t)N * hp >= ((int64_t)1 << 30))
            return VD_ERR_SHAPE;
        mos = hp << 2;
    }
    // the grid: maps at a (H + 1) x (W + 1) pitch, g per mosaic row, g chosen for the
    // fewest 16 x 32 blocks (14 x 14: 32 maps = 480 columns = 15 blocks exactly)
    int gG = 0;
    if (mos == 4) {
        if ((int64_t)N * H * W * C >= ((int64_t)1 << 31) || H > 255 || W > 255) return VD_ERR_SHAPE;
        int64_t best = -1;
        for (int g = 1; g <= 64 && g <= N; ++g) {
            const int64_t rows = (int64_t)(N + g - 1) / g * (H + 1);
            const int64_t b = (rows + 4 * k4TR - 1) / (4 * k4TR) *
                              (((int64_t)g * (W + 1) + 4 * k4TC - 1) / (4 * k4TC));
            if (best < 0 || b < best) best = b, gG = g;
        }
        if ((int64_t)(N + gG - 1) / gG * (H + 1) >= ((int64_t)1 << 30)) return VD_ERR_SHAPE;
    }
    const bool cells = mos == 1 || mos == 3;
    const int tby = cells ? 1
                    : gG ? (int)(((int64_t)(N + gG - 1) / gG * (H + 1) + 4 * k4TR - 1) / (4 * k4TR))
                         : ((mos ? N * hp : H) + 4 * k4TR - 1) / (4 * k4TR);
    const int tbx = cells ? 1 : ((gG ? gG * (W + 1) : W) + 4 * k4TC - 1) / (4 * k4TC);
    if (gG) mos = (gG << 2) | 2;
    const int64_t nsp = mos == 1 ? ((int64_t)N + 1) / 2
                                 : mos == 3 ? ((int64_t)N + 7) / 8
                                            : (int64_t)(mos ? 1 : N) * tby * tbx;
    const int ncb = Cout / k4Co;
    // VOSDET_WINO4_CBX=0: the four channel blocks of a spatial block on one XCD (the
    // patch then comes from that XCD's L2 three times in four), not one channel block
    // per XCD (its U in that L2)
    const char *cbxe = getenv("VOSDET_WINO4_CBX");
    const int cbx = (8 % ncb == 0) && !(cbxe && cbxe[0] == '0');
    const int64_t blocks = cbx ? (nsp + 8 / ncb - 1) / (8 / ncb) * 8 : (nsp + 7) / 8 * 8 * ncb;
    if (blocks > 0x7fffffff) return VD_ERR_SHAPE;
    static_assert(k4LdsB <= VD_LDS_BYTES, "LDS");
    static const int probe = [] {
        const char *e = getenv("VOSDET_WINO4_PROBE");
        return e ? atoi(e) & 15 : 0;
    }();
    static const int probe_hi = [] {
        const char *e = getenv("VOSDET_WINO4_PROBE");
        return e ? (atoi(e) >> 4) & 1 : 0;
    }();
    typedef void (*kern_t)(const float *, int, int, int, int, const float *, int, const float *,
                           float *, int, int, int, int, int, int);
    static const kern_t table[2][16] = {
        {conv3x3_wino4_kernel<false, 0>, conv3x3_wino4_kernel<false, 1>,
         conv3x3_wino4_kernel<false, 2>, conv3x3_wino4_kernel<false, 3>,
         conv3x3_wino4_kernel<false, 4>, conv3x3_wino4_kernel<false, 5>,
         conv3x3_wino4_kernel<false, 6>, conv3x3_wino4_kernel<false, 7>,
         conv3x3_wino4_kernel<false, 8>, conv3x3_wino4_kernel<false, 9>,
         conv3x3_wino4_kernel<false, 10>, conv3x3_wino4_kernel<false, 11>,
         conv3x3_wino4_kernel<false, 12>, conv3x3_wino4_kernel<false, 13>,
         conv3x3_wino4_kernel<false, 14>, conv3x3_wino4_kernel<false, 15>},
        {conv3x3_wino4_kernel<true, 0>, conv3x3_wino4_kernel<true, 1>,
         conv3x3_wino4_kernel<true, 2>, conv3x3_wino4_kernel<true, 3>,
         conv3x3_wino4_kernel<true, 4>, conv3x3_wino4_kernel<true, 5>,
         conv3x3_wino4_kernel<true, 6>, conv3x3_wino4_kernel<true, 7>,
         conv3x3_wino4_kernel<true, 8>, conv3x3_wino4_kernel<true, 9>,
         conv3x3_wino4_kernel<true, 10>, conv3x3_wino4_kernel<true, 11>,
         conv3x3_wino4_kernel<true, 12>, conv3x3_wino4_kernel<true, 13>,
         conv3x3_wino4_kernel<true, 14>, conv3x3_wino4_kernel<true, 15>}};
    // read at every launch (a few us of host time), so one process can A/B the forms
    const char *pse = getenv("VOSDET_WINO4_PS");
    const bool ps = pse && pse[0] == '1';
    if (ps && !probe && !mos && !gin) {
        typedef void (*kps_t)(const float *, int, int, int, int, const float *, int,
                              const float *, float *, int, int, int);
        const char *ppe = getenv("VOSDET_WINO4_PSPROBE");
        const int pp = ppe ? atoi(ppe) : 0;
#define VD_PSK(P) (relu ? conv3x3_wino4ps_kernel<true, P> : conv3x3_wino4ps_kernel<false, P>)
        kps_t kp = VD_PSK(0);
        if (pp == 1) kp = VD_PSK(1);
        if (pp == 2) kp = VD_PSK(2);
        if (pp == 4) kp = VD_PSK(4);
        if (pp == 8) kp = VD_PSK(8);
        if (pp == 16) kp = VD_PSK(16);
        if (pp == 18) kp = VD_PSK(18);
        if (pp == 31) kp = VD_PSK(31);
        if (pp == 5) kp = VD_PSK(5);
        if (pp == 12) kp = VD_PSK(12);
#undef VD_PSK
        hipLaunchKernelGGL(kp, dim3((unsigned)blocks), dim3(k4Threads), 0, s, X, N, H, W, C, U,
                           Cout, bias, Y, tby, tbx, cbx);
        return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
    }
    // the ACC form (hand-counted vmcnt, conflict-free V layout) is the default;
    // VOSDET_WINO4_ACC=0 selects the first form (bit-identical, 2-6 % slower)
    const char *acce = getenv("VOSDET_WINO4_ACC");
    const bool acc = !(acce && acce[0] == '0');
    // VOSDET_WINO4_VD (ACC form): V fragments read 1-3 positions ahead
    const char *vde = getenv("VOSDET_WINO4_VD");
    const int vd = vde ? atoi(vde) : 1;
    const char *pke = getenv("VOSDET_WINO4_PK");
    const bool pk = !(pke && pke[0] == '0');
    kern_t kacc = relu ? conv3x3_wino4_kernel<true, 0, true, 1> : conv3x3_wino4_kernel<false, 0, true, 1>;
    if (pk)
        kacc = relu ? conv3x3_wino4_kernel<true, 0, true, 1, false, false, true>
                    : conv3x3_wino4_kernel<false, 0, true, 1, false, false, true>;
    if (vd == 2)
        kacc = relu ? conv3x3_wino4_kernel<true, 0, true, 2> : conv3x3_wino4_kernel<false, 0, true, 2>;
    if (vd == 3)
        kacc = relu ? conv3x3_wino4_kernel<true, 0, true, 3> : conv3x3_wino4_kernel<false, 0, true, 3>;
    const char *pre = getenv("VOSDET_WINO4_PRIO");
    const int prio = (pre && pre[0] == '1') ? 2 : 0;
    const char *ste = getenv("VOSDET_WINO4_STAMP");
    if (ste && ste[0] == '1')
        kacc = relu ? conv3x3_wino4_kernel<true, 0, true, 1, true>
                    : conv3x3_wino4_kernel<false, 0, true, 1, true>;
    const char *ile = getenv("VOSDET_WINO4_IL");
    if (ile && ile[0] == '1')
        kacc = relu ? conv3x3_wino4_kernel<true, 0, true, 1, false, true>
                    : conv3x3_wino4_kernel<false, 0, true, 1, false, true>;
    if (ile && ile[0] == '2')  // interleaved + stamps
        kacc = relu ? conv3x3_wino4_kernel<true, 0, true, 1, true, true>
                    : conv3x3_wino4_kernel<false, 0, true, 1, true, true>;
    const kern_t kern = (acc && !probe) ? kacc : table[relu ? 1 : 0][probe];
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(k4Threads), 0, s, X, N, H, W, C, U,
                       Cout, bias, Y, tby, tbx, cbx, probe_hi | prio, mos, gin);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd

// research: the STAMP form's timestamps [512 workgroups][8 waves][4 chunks][6]
extern "C" int vd_research_wino4_stamps(unsigned long long *host, int n) {
    const int cap = vd::kStampWg * 8 * vd::kStampNch * 6;
    if (n > cap) n = cap;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(vd::g_wino4_stamps), (size_t)n * 8, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
