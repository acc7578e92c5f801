// 3x3 stride-1 pad-1 convolution on NHWC fp32 by Winograd F(2x2, 3x3) on the
// MFMA pipes, bias (+ ReLU) epilogue fused.
//
// Same operator as conv3x3.hip (FPN posthoc / RPN conv, lib/modeling/FPN.py:
// 227-258, 376-422; mask head convs, mask_rcnn_heads.py:178-188), computed with
// 2.25x fewer multiplies (Lavin & Gray, "Fast Algorithms for Convolutional Neural
// Networks"): every 2x2 output tile is
//   Y = A^T [ sum_ci (G g G^T) (.) (B^T d B) ] A
// with d the tile's 4x4 input patch.  The sum over ci is 16 independent GEMMs,
// M[pos][co][tile] = sum_ci U[pos][co][ci] V[pos][ci][tile] (pos = the 16
// transform positions), run with v_mfma_f32_16x16x4_f32 (fp32 in, fp32 out: the
// reference's precision; the transforms only add / subtract and scale by 0.5).
//
// Workgroup = 4 waves, 32 tiles (2 x 16 tiles = 4 x 32 output pixels of one
// image, or 4 x 8 tiles = 8 x 16 pixels for maps <= 16 wide: the 14 x 14 mask-head
// RoIs) x 64 output channels, two waves per SIMD (248-252 VGPRs), so TWO workgroups share a CU and the
// barrier / transform gaps of one are filled by the MFMAs of the other (the
// round-3 one-per-CU 8-wave form, 64 tiles and 150 KiB, ran 7-12 % slower on every
// benched shape in one-process A/B: profiles/r03_wino_ab.json).  Wave w owns 16 tiles (w & 1) x
// 32 channels (w >> 1), ALL 16 positions: 128 accumulator registers per lane,
// and a lane's 16 position values of one (channel, tile) sit in the same register
// slot of its 16 accumulators, so the output transform is lane-local.
//
// K is walked in chunks of 8 input channels.  Per chunk the raw input patch is
// copied HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR round trip),
// double-buffered (2 x 9 KiB), one barrier per chunk; each wave's U operand (the 16
// positions x its 32 channels x 8 input channels, 64 VGPRs) comes straight from L2
// into registers, each fragment reloaded for the next chunk right after its MFMAs
// consumed it.  (U through LDS -- its 32 KiB slice LDS-DMA'd per chunk and read back
// -- ran 5-13 % slower on every benched shape, bit-identical:
// profiles/r04/wino_ureg_ab.jsonl.)  All of the loop's vector-memory ops are inline
// asm, so hipcc neither drains them at LDS reads nor counts them: the loop waits
// with its own vmcnt.  The input transform needs no LDS round
// trip: the MFMA B fragment of lane (j, q) is V[pos][channels 2q, 2q + 1][tile j]
// -- the 4 x 4 transform of tile j's patch for those two channels -- so every lane
// transforms its own fragment from the patch into registers (v_pk_add_f32 on the
// channel pair).  K permutation (both operands): lane group q at k-step s holds
// channel 2q + s, so each fragment is one 8-byte LDS read.
#include <stdlib.h>

#include <type_traits>

#include "common.hpp"
#include "vosdet_internal.hpp"

namespace vd {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int kCo = 64;  // output channels per workgroup
constexpr int kKC = 8;   // input channels per chunk
constexpr int k2Tiles = 32;
constexpr int k2Threads = 256;
constexpr int k2PDma = 512;               // patch slots copied per chunk (480 used)
constexpr int k2PSlots = 576;             // + the all-zero row the masked taps read
constexpr int k2StageB = k2PSlots * 16;  // 9 KiB; two stages
constexpr int kUChunk = 16 * kCo * kKC;  // floats of U per (channel block, chunk)

constexpr int kZeroF4 = 1024;  // 4096 floats: the zero lanes' DMA source for C <= 4096
__device__ float4 g_wino_zero[kZeroF4];  // the source of out-of-image patch taps

template <int TC, bool SK = (TC == 16)>
struct Patch2 {  // patch [row][half][column] in 16-B slots
    static constexpr int kTR = k2Tiles / TC, kPR = 2 * kTR + 2, kPC = 2 * TC + 2;
    static constexpr int kHP = TC == 16 ? 37 : 20, kRP = TC == 16 ? 80 : 48;
    static_assert(kPR * kRP <= k2PDma, "patch fits its DMA'd LDS region");
    static_assert(kPR * kRP + kRP <= k2PSlots, "the zero row fits past it");
    // first slot of a row past both halves (unused, so the DMA copies zeros there)
    static constexpr int kZC = 2 * kHP;
    static_assert(kZC + 3 <= kRP && kHP >= 2 * TC + 4, "zero column slots (+ half + row skew)");
    static_assert(kRP % 16 == 0, "row pitch: whole bank sweeps");
    // TC = 16, (p >> 4): columns 16 apart land 17 slots apart, so the 16 tiles of one
    // fragment read (pixel columns 2j + c) fall in distinct 16-B bank groups (one
    // 2-way pair for c >= 2); ((r >> 1) & 1): rows two apart are shifted by one
    // slot, so a TC = 8 read (8 tiles on each of two tile rows) is conflict-free
    // with no column skew at all (the skew there cost a 2-way conflict on half the
    // reads: SQ_LDS_BANK_CONFLICT = 1 cycle per ds_read, profiles/r04/wino_pmc/;
    // without it bit-identical, 0.5-2 % faster, profiles/r04/wino_noskew/)
    __device__ static int col(int p) { return SK ? p + (p >> 4) : p; }
    __device__ static int col_inv(int u) { return !SK || u < 16 ? u : (u < 33 ? u - 1 : u - 2); }
    __device__ static int slot(int r, int h, int p) {
        return r * kRP + h * kHP + col(p) + ((r >> 1) & 1);
    }
};

// One LDS-DMA wave instruction: 64 lanes x 16 B from per-lane global addresses to
// 1 KiB of LDS at the wave-uniform byte address `lds`, lane-linear (M0 carries the
// LDS base and is restored within the statement).
__device__ __forceinline__ void wino_dma_1k(const float *src, uint32_t lds) {
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

// The same from a wave-uniform SGPR base + a per-lane 32-bit byte offset.
__device__ __forceinline__ void wino_dma_1k_off(const float *base, uint32_t voff, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(base), "s"(lds)
        : "memory");
}

// This wave's LDS-DMAs landed and LDS reads retired, then the workgroup barrier.
__device__ __forceinline__ void wino_wait_barrier() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Packed fp32 a + b / a - b on a channel pair (v_pk_add_f32: both halves IEEE adds,
// bit-identical to two v_add_f32; hipcc otherwise splits half the transform into
// scalar adds)
__device__ __forceinline__ f2v pk_add(f2v a, f2v b) {
    f2v r;
    asm("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f2v pk_sub(f2v a, f2v b) {
    f2v r;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// One 16-B U fragment per lane, global -> VGPR: wave-uniform SGPR base + lane
// offset (no per-load 64-bit VALU address arithmetic).  Inline asm so the
// compiler neither drains it nor moves it around the LDS-DMAs; the tied operand
// keeps the fragment in the register its MFMAs read.  The caller counts vmcnt.
__device__ __forceinline__ void wino_load_u(f4v &r, const float *ub, uint32_t voff) {
    asm volatile("global_load_dwordx4 %0, %1, %2" : "+v"(r) : "v"(voff), "s"(ub) : "memory");
}
template <int OFF>  // + an immediate byte offset (< 4 KiB): one SGPR base per 4 fragments
__device__ __forceinline__ void wino_load_u_off(f4v &r, const float *ub, uint32_t voff) {
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3"
                 : "+v"(r)
                 : "v"(voff), "s"(ub), "i"(OFF)
                 : "memory");
}
// All but the last 16 vector-memory ops of this wave retired; the two fragments
// pass through so their MFMAs cannot be scheduled above the wait.
__device__ __forceinline__ void wino_wait_u(f4v &a, f4v &b) {
    asm volatile("s_waitcnt vmcnt(16)" : "+v"(a), "+v"(b) : : "memory");
}
// One 8-byte LDS read per lane at a precomputed address + an immediate (the stage);
// inline asm so the stage offset stays an immediate -- the caller waits lgkmcnt.
template <int OFF>
__device__ __forceinline__ f2v wino_ds_read(uint32_t addr) {
    f2v r;
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
    return r;
}
__device__ __forceinline__ void wino_wait_lds(f2v (&d)[4][4]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(d[0][0]), "+v"(d[0][1]), "+v"(d[0][2]), "+v"(d[0][3]), "+v"(d[1][0]),
                   "+v"(d[1][1]), "+v"(d[1][2]), "+v"(d[1][3]), "+v"(d[2][0]), "+v"(d[2][1]),
                   "+v"(d[2][2]), "+v"(d[2][3]), "+v"(d[3][0]), "+v"(d[3][1]), "+v"(d[3][2]),
                   "+v"(d[3][3]));
}
__device__ __forceinline__ void wino_wait16_barrier() {
    asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}


template <bool RELU, int TC, int PR = 0, bool SK = (TC == 16), bool RD = false, bool PRIO = true>
__global__ __launch_bounds__(k2Threads, 2) void conv3x3_wino2_kernel(
    const float *__restrict__ X, int N, int H, int W, int C, const float *__restrict__ U,
    int Cout, const float *__restrict__ bias, float *__restrict__ Y, int tby, int tbx,
    int cb_per_xcd, int seg_h, int seg_w, int gx, int nmaps, int map_h, int map_w) {
    using PG = Patch2<TC, SK>;
    __shared__ __attribute__((aligned(16))) float sm[2 * k2StageB / 4];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 15, q = lane >> 4;
    // the Cout / 64 channel blocks of one spatial block run on one XCD (blocks
    // b, b + 8, ...): its input patches come from one L2
    const int ncb = Cout / kCo;
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
    if (sp >= N * tby * tbx) return;
    const int n = sp / (tby * tbx);
    const int rem = sp - n * tby * tbx;
    const int tyb = rem / tbx, txb = rem - (rem / tbx) * tbx;
    const int oy0 = 2 * PG::kTR * tyb, ox0 = 2 * TC * txb;
    const int iy0 = oy0 - 1, ix0 = ox0 - 1;
    const int n0 = cb * kCo;
    const int tg = wave & 1, cg = wave >> 1;  // wave: tiles 16 tg .. + 15, 32-channel group
    const uint32_t sbase = (uint32_t)(uintptr_t)sm;

    const int nch = C / kKC;
    // patch DMA: blocks b = wave + 4 i (i < 2); slots outside the patch or the
    // image copy zeros
    const float *psrc[2];
    uint32_t poff[2];  // RD: byte offsets from X (invalid lanes copy X[0..3], never read)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int s = 64 * (wave + 4 * i) + lane;
        const int r = s / PG::kRP, t = s - (s / PG::kRP) * PG::kRP;
        const int h = t >= PG::kHP;
        const int u = t - h * PG::kHP - ((r >> 1) & 1);
        const int p = PG::col_inv(u);
        const int y = iy0 + r, x = ix0 + p;
        bool ok = r < PG::kPR && u >= 0 && p < PG::kPC && PG::slot(r, h, p) == s &&
                  (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
        int64_t pix = ((int64_t)n * H + y) * W + x;
        if (seg_w > 0 && ok) {  // 2-D mosaic pixel (y, x) -> map, row, column in X
            const int m = (y / seg_h) * gx + x / seg_w, my = y % seg_h, mx = x % seg_w;
            ok = m < nmaps && my < map_h && mx < map_w;  // a map's phantom row / column: 0
            pix = ((int64_t)m * map_h + my) * map_w + mx;
        }
        psrc[i] = ok ? X + pix * C + 4 * h : reinterpret_cast<const float *>(g_wino_zero);
        poff[i] = ok ? (uint32_t)((pix * C + 4 * h) * 4) : 0u;
    }
    // transform reads: lane (j, q) -> tile 16 tg + j, channels 2q, 2q + 1 (half
    // q >> 1, dwords 2 (q & 1) ..): byte offsets within a stage
    const int vt = tg * 16 + j, tr = vt / TC, tc = vt % TC;
    // segmented rows (seg_h > 0: the image is a vertical mosaic of seg_h-row
    // images, e.g. [R][14][14][C] as [1][14 R][14][C]): the patch row above / below
    // a tile at a segment edge belongs to the neighbouring image and reads as the
    // zero padding of its own (seg_h even: a 2x2 tile never straddles an edge)
    const int toy = oy0 + 2 * tr;  // the tile's first output row
    const bool zero_top = seg_h > 0 && toy % seg_h == 0;
    const bool zero_bot = seg_h > 0 && (toy + 2) % seg_h == 0;
    // 2-D mosaic (seg_w > 0: gx maps side by side per mosaic row): the same for the
    // patch columns left / right of a tile at a map's side (seg_w even)
    const int tox = ox0 + 2 * tc;
    const bool zero_left = seg_w > 0 && tox % seg_w == 0;
    const bool zero_right = seg_w > 0 && (tox + 2) % seg_w == 0;
    int roff[4], coff[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const int r = 2 * tr + a, p = 2 * tc + a;
        roff[a] = 16 * (r * PG::kRP + ((r >> 1) & 1));
        coff[a] = 16 * PG::col(p) + 16 * (q >> 1) * PG::kHP + 8 * (q & 1);
    }
    // the masked taps read zeros from LDS rather than being zeroed per chunk: a masked
    // row reads the all-zero row kPR (past the DMA'd slots, zeroed once here), a
    // masked column the unused, DMA-zeroed slots kZC, kZC + 1 of its row (bit-identical
    // to the per-chunk v_cndmask form it replaced, 2-6 % faster with the packed
    // transform: profiles/r04/wino_zs/)
    if (zero_top) roff[0] = 16 * PG::kPR * PG::kRP;
    if (zero_bot) roff[3] = 16 * PG::kPR * PG::kRP;
    if (zero_left) coff[0] = 16 * (PG::kZC + (q >> 1)) + 8 * (q & 1);
    if (zero_right) coff[3] = 16 * (PG::kZC + (q >> 1)) + 8 * (q & 1);
    if (tid < 2 * (k2PSlots - k2PDma))
        reinterpret_cast<float4 *>(sm)[(tid / (k2PSlots - k2PDma)) * k2PSlots + k2PDma +
                                       tid % (k2PSlots - k2PDma)] = make_float4(0.f, 0.f, 0.f, 0.f);
    f4v acc[16][2];
#pragma unroll
    for (int p = 0; p < 16; ++p)
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2) acc[p][t2] = f4v{0.f, 0.f, 0.f, 0.f};

    // the wave's U fragments of one chunk (weight order [Cout / 64][C / 8][cg][l][lane][4],
    // wino_weight_kernel): fragment l = 2 pp + t2 holds positions 2 pp, 2 pp + 1 x
    // channels 2q, 2q + 1 of output channel cg*32 + 16 t2 + j -- 1 KiB per wave load
    f4v ur[16];
    const float *ursrc = U + ((int64_t)cb * nch * 2 + cg) * (kUChunk / 2);
    const uint32_t uvoff = (uint32_t)lane * 16u;
#pragma unroll
    for (int l = 0; l < 16; ++l) ur[l] = f4v{0.f, 0.f, 0.f, 0.f};
    // V = B^T d B for the lane's two channels, B^T = [1 0 -1 0; 0 1 1 0;
    // 0 -1 1 0; 0 1 0 -1]
    auto transform = [&](f2v(&d)[4][4], f2v(&b)[16]) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const f2v r0 = pk_sub(d[0][c], d[2][c]), r1 = pk_add(d[1][c], d[2][c]);
            const f2v r2 = pk_sub(d[2][c], d[1][c]), r3 = pk_sub(d[1][c], d[3][c]);
            d[0][c] = r0;
            d[1][c] = r1;
            d[2][c] = r2;
            d[3][c] = r3;
        }
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            b[4 * a + 0] = pk_sub(d[a][0], d[a][2]);
            b[4 * a + 1] = pk_add(d[a][1], d[a][2]);
            b[4 * a + 2] = pk_sub(d[a][2], d[a][1]);
            b[4 * a + 3] = pk_sub(d[a][1], d[a][3]);
        }
    };
    // positions 2 pp, 2 pp + 1 of one chunk: their U fragments landed (after them this
    // wave issued the other 14, the current chunk's 2 patch DMAs and 2 pp U loads:
    // vmcnt(16)), 8 MFMAs, then the fragments' reload for chunk `un`
    auto mfma_pair = [&](int pp, const f2v(&b)[16], const float *un) {
        wino_wait_u(ur[2 * pp], ur[2 * pp + 1]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
                acc[2 * pp + i][t2] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                    i ? ur[2 * pp + t2].z : ur[2 * pp + t2].x, b[2 * pp + i].x,
                    acc[2 * pp + i][t2], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
                acc[2 * pp + i][t2] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                    i ? ur[2 * pp + t2].w : ur[2 * pp + t2].y, b[2 * pp + i].y,
                    acc[2 * pp + i][t2], 0, 0, 0);
        if (!(PR & 8)) {
            const float *ub = un + (pp >> 1) * 1024;
            if (pp & 1) {
                wino_load_u_off<2048>(ur[2 * pp], ub, uvoff);
                wino_load_u_off<3072>(ur[2 * pp + 1], ub, uvoff);
            } else {
                wino_load_u_off<0>(ur[2 * pp], ub, uvoff);
                wino_load_u_off<1024>(ur[2 * pp + 1], ub, uvoff);
            }
        }
    };
    // The chunk loop, unrolled by the two stages: the stage is an immediate of the 16
    // LDS reads (their addresses precomputed), the zero lanes' DMA reads the zero
    // buffer at the chunk's offset (no per-chunk select), one SGPR base per 4 U
    // fragments.  Every chunk issues 2 patch DMAs, then 16 U loads (the last chunk
    // re-copies itself into the idle stage and reloads its own U), so in-order vmcnt
    // makes every wait vmcnt(16).  (Loop VALU 56 -> 34, SALU 80 -> 47 per chunk:
    // bit-identical, 1-5 % faster, profiles/r04/wino_v2/.  A three-stage ring with
    // the next chunk's patch read during this chunk's MFMAs: 0-1 %, not kept:
    // profiles/r04/wino_pf/.)
    {
        uint32_t radr[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int c = 0; c < 4; ++c) radr[a][c] = sbase + roff[a] + coff[c];
        if constexpr (RD) {
            // every tap outside the image (or a map's phantom row / column, or a
            // mosaic neighbour -- the masks above) reads the zero row past the DMA'd
            // slots, so the DMA never has to write zeros: its invalid lanes copy
            // X[0..3] into slots no tap reads
            const uint32_t zaddr = sbase + 16u * k2PDma + 8u * (q & 1);
            // 2-D mosaic: the tile's rows / columns within its map (a tile never
            // straddles maps; the taps past a map's side are the masks above)
            const int ty = seg_w > 0 ? toy % seg_h : 0, tx = seg_w > 0 ? tox % seg_w : 0;
            uint32_t badr = 0, badc = 0;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const int y = toy - 1 + a, x = tox - 1 + a;
                if ((unsigned)y >= (unsigned)H || (seg_w > 0 && ty - 1 + a >= map_h)) badr |= 1u << a;
                if ((unsigned)x >= (unsigned)W || (seg_w > 0 && tx - 1 + a >= map_w)) badc |= 1u << a;
            }
            if (zero_top) badr |= 1u;
            if (zero_bot) badr |= 8u;
            if (zero_left) badc |= 1u;
            if (zero_right) badc |= 8u;
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (((badr >> a) | (badc >> c)) & 1u) radr[a][c] = zaddr;
        }
        const uint32_t dbase = sbase + (uint32_t)wave * 1024u;
        auto chunk = [&](int ch, auto stc) {
            constexpr int S = decltype(stc)::value;
            const int nxt = ch + 1 < nch ? ch + 1 : ch;
            if (!(PR & 32)) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    if constexpr (RD)
                        wino_dma_1k_off(X + nxt * kKC, poff[i],
                                        dbase + (uint32_t)((S ^ 1) * k2StageB + i * 4096));
                    else
                        wino_dma_1k(psrc[i] + nxt * kKC, dbase + (uint32_t)((S ^ 1) * k2StageB + i * 4096));
                }
            }
            f2v d[4][4], b[16];
            // the reads + transform at wave priority 1: the partner wave on the SIMD
            // keeps the matrix pipe while this one gets back to its MFMAs sooner
            // (bit-identical, 0.3-2 % per benched shape, +0.4 % bench:
            // profiles/r04/wino_prio/)
            if constexpr (PRIO) asm volatile("s_setprio 1" ::: "memory");
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    d[a][c] = (PR & 2) ? f2v{(float)radr[a][c], 0.f}
                                       : wino_ds_read<S * k2StageB>(radr[a][c]);
            wino_wait_lds(d);
            transform(d, b);
            if constexpr (PRIO) {
                // the transform's results pass through, so it cannot sink below
                asm volatile("s_setprio 0" : "+v"(b[0]), "+v"(b[15]) : : "memory");
            }
            const float *un = ursrc + (int64_t)nxt * kUChunk;
#pragma unroll
            for (int pp = 0; pp < 8; ++pp) mfma_pair(pp, b, un);
            // the next chunk's patch DMAs landed (16 U loads were issued after them)
            // and stage S read by every wave
            if (!(PR & 4)) wino_wait16_barrier();
        };
        for (int l = 0; l < 2; ++l) {
            if constexpr (RD)
                wino_dma_1k_off(X, poff[l], dbase + (uint32_t)(l * 4096));
            else
                wino_dma_1k(psrc[l], dbase + (uint32_t)(l * 4096));
        }
#pragma unroll
        for (int l = 0; l < 16; ++l) wino_load_u(ur[l], ursrc + l * 256, uvoff);
        wino_wait_barrier();
        for (int ch = 0; ch < nch; ch += 2) {
            chunk(ch, std::integral_constant<int, 0>{});
            if (ch + 1 < nch) chunk(ch + 1, std::integral_constant<int, 1>{});
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the wave
    // output transform (lane-local): A^T = [1 1 1 0; 0 1 -1 -1]; lane (j, q),
    // accumulator slot r holds channel n0 + cg*32 + 16 t2 + 4 q + r of tile 16 tg + j
    const int oy = oy0 + 2 * tr, ox = ox0 + 2 * tc;
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
        const int co = n0 + cg * 32 + 16 * t2 + 4 * q;
        const float4 bv = bias ? *reinterpret_cast<const float4 *>(bias + co)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
        float o[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float s0[4], s1[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                s0[c] = acc[c][t2][r] + acc[4 + c][t2][r] + acc[8 + c][t2][r];
                s1[c] = acc[4 + c][t2][r] - acc[8 + c][t2][r] - acc[12 + c][t2][r];
            }
            o[0][r] = s0[0] + s0[1] + s0[2];
            o[1][r] = s0[1] - s0[2] - s0[3];
            o[2][r] = s1[0] + s1[1] + s1[2];
            o[3][r] = s1[1] - s1[2] - s1[3];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int y = oy + (k >> 1), x = ox + (k & 1);
            if (y >= H || x >= W) continue;
            int64_t pix = (int64_t)(n * H + y) * W + x;
            if (seg_w > 0) {
                const int m = (y / seg_h) * gx + x / seg_w, my = y % seg_h, mx = x % seg_w;
                if (m >= nmaps || my >= map_h || mx >= map_w) continue;
                pix = ((int64_t)m * map_h + my) * map_w + mx;
            }
            float4 v = make_float4(o[k][0] + bv.x, o[k][1] + bv.y, o[k][2] + bv.z,
                                   o[k][3] + bv.w);
            if (RELU) {
                v.x = fmaxf(v.x, 0.f);
                v.y = fmaxf(v.y, 0.f);
                v.z = fmaxf(v.z, 0.f);
                v.w = fmaxf(v.w, 0.f);
            }
            *reinterpret_cast<float4 *>(Y + pix * Cout + co) = v;
        }
    }
}

// U = G g G^T of the PyTorch weight w[co][ci][3][3], G = [1 0 0; .5 .5 .5;
// .5 -.5 .5; 0 0 1], float64, rounded once; stored in the kernel's register-fragment
// order [co / 64][ci / 8][cg][l][lane][4]: cg = co % 64 / 32, fragment l = 2 (pos / 2)
// + co % 32 / 16, lane = 16 (ci % 8 / 2) + co % 16, element 2 (pos & 1) + (ci & 1).
__global__ void wino_weight_kernel(const float *__restrict__ w, int Cout, int C,
                                   float *__restrict__ U) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)Cout * C) return;
    const int co = (int)(i / C), ci = (int)(i - (int64_t)(i / C) * C);
    const int cl = co % kCo;
    float *dst = U + ((int64_t)(co / kCo) * (C / kKC) + ci / kKC) * kUChunk + (cl >> 5) * 4096 +
                 ((cl >> 4) & 1) * 256 + (16 * ((ci & 7) >> 1) + (cl & 15)) * 4 + (ci & 1);
    const float *g = w + i * 9;
    double t[4][3];  // G g
    for (int c = 0; c < 3; ++c) {
        const double g0 = g[c], g1 = g[3 + c], g2 = g[6 + c];
        t[0][c] = g0;
        t[1][c] = 0.5 * (g0 + g1 + g2);
        t[2][c] = 0.5 * (g0 - g1 + g2);
        t[3][c] = g2;
    }
    for (int a = 0; a < 4; ++a) {
        const double u[4] = {t[a][0], 0.5 * (t[a][0] + t[a][1] + t[a][2]),
                             0.5 * (t[a][0] - t[a][1] + t[a][2]), t[a][2]};
        for (int b = 0; b < 4; ++b) {
            const int pos = 4 * a + b;
            dst[(pos >> 1) * 512 + (pos & 1) * 2] = (float)u[b];
        }
    }
}

}  // namespace

bool conv3x3_wino_supported(int C, int Cout) {
    return C % kKC == 0 && C >= kKC && C <= 4 * kZeroF4 && Cout % kCo == 0 && Cout >= kCo;
}

int launch_conv3x3_wino_weight(const float *w, int Cout, int C, float *U, hipStream_t s) {
    const int64_t n = (int64_t)Cout * C;
    if (n == 0) return VD_OK;
    if (!conv3x3_wino_supported(C, Cout)) return VD_ERR_SHAPE;
    hipLaunchKernelGGL(wino_weight_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w,
                       Cout, C, U);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

namespace {

int launch_wino(const float *X, int N, int H, int W, int C, const float *U, int Cout,
                const float *bias, int relu, float *Y, hipStream_t s, int seg_h, int seg_w, int gx,
                int nmaps, int map_h, int map_w) {
    // block shape: 8 x 16 or 4 x 32 output pixels, whichever wastes less of the map
    // (measured, profiles/r03/wino_small_probe.json: 8 x 16 wins on res5 / P5
    // 25 x 42 maps and at P3, 4 x 32 at P4); VOSDET_WINO_SQ=1/0 forces one
    const double use_sq = (double)H * W / ((double)((H + 7) / 8 * 8) * ((W + 15) / 16 * 16));
    const double use_wide = (double)H * W / ((double)((H + 3) / 4 * 4) * ((W + 31) / 32 * 32));
    const char *esq = getenv("VOSDET_WINO_SQ");
    const bool sq = esq ? atoi(esq) == 1 : use_sq > use_wide;
    const int tby = sq ? (H + 7) / 8 : (H + 3) / 4;
    const int tbx = sq ? (W + 15) / 16 : (W + 31) / 32;
    const int64_t nsp = (int64_t)N * tby * tbx;
    const int ncb = Cout / kCo;
    // XCD x computes channel block x % ncb (its L2 keeps one U block instead of
    // all of them): bit-identical, P3 1.66 -> 1.51 ms, P2 / mask head 1-3 %
    // (profiles/r03/wino_map_probe.json); VOSDET_WINO_MAP=0 restores the
    // channel-blocks-of-a-spatial-block-on-one-XCD order
    const char *em = getenv("VOSDET_WINO_MAP");
    const int cbx = (!em || atoi(em) != 0) && 8 % ncb == 0;
    const int64_t blocks = cbx ? (nsp + 8 / ncb - 1) / (8 / ncb) * 8
                               : (nsp + 7) / 8 * 8 * ncb;
    if (blocks > 0x7fffffff) return VD_ERR_SHAPE;
    // the DMA reads X through 32-bit byte offsets (taps outside the image redirected to
    // a zero row, so no zero source per lane: bit-identical, 0-3.5 % faster on the
    // benched shapes, profiles/r04/wino_rd/); an X of 4 GiB or more takes the
    // 64-bit-pointer form with the zero-buffer source
    const int64_t xbytes = (seg_w > 0 ? (int64_t)nmaps * map_h * map_w : (int64_t)N * H * W) * C * 4;
    auto kern = sq ? (relu ? conv3x3_wino2_kernel<true, 8, 0, false, true> : conv3x3_wino2_kernel<false, 8, 0, false, true>)
                   : (relu ? conv3x3_wino2_kernel<true, 16, 0, true, true> : conv3x3_wino2_kernel<false, 16, 0, true, true>);
    if (xbytes >= ((int64_t)1 << 32))
        kern = sq ? (relu ? conv3x3_wino2_kernel<true, 8> : conv3x3_wino2_kernel<false, 8>)
                  : (relu ? conv3x3_wino2_kernel<true, 16> : conv3x3_wino2_kernel<false, 16>);
#ifdef VD_RESEARCH_PROBES
    // speed-of-light probes (wrong results; tools/research/wino_sol_probe.py): 2 no
    // patch reads, 4 no barrier, 8 no U loads, 32 no patch DMA (round-4 probe 64, the
    // DMA from lane-contiguous addresses: profiles/r04/wino_sol_probe_dma.json).  Only in a research build
    // (make VD_RESEARCH=1), never in the product library: a stray environment
    // variable must not be able to corrupt a product convolution.
    const char *pe = getenv("VOSDET_WINO_PROBE");
    switch (pe && !relu ? atoi(pe) : 0) {
#define VD_PROBE_CASE(B) \
        case B: kern = sq ? conv3x3_wino2_kernel<false, 8, B, false, true> : conv3x3_wino2_kernel<false, 16, B, true, true>; break;
        VD_PROBE_CASE(2) VD_PROBE_CASE(4) VD_PROBE_CASE(8) VD_PROBE_CASE(32) VD_PROBE_CASE(36)
        VD_PROBE_CASE(12) VD_PROBE_CASE(46)
#undef VD_PROBE_CASE
        default: break;
    }
#endif
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(k2Threads), 0, s, X, N, H, W, C, U, Cout,
                       bias, Y, tby, tbx, cbx, seg_h, seg_w, gx, nmaps, map_h, map_w);
    return hipGetLastError() == hipSuccess ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace

int launch_conv3x3_wino(const float *X, int N, int H, int W, int C, const float *U, int Cout,
                        const float *bias, int relu, float *Y, hipStream_t s, int seg_h) {
    if ((int64_t)N * H * W == 0) return VD_OK;
    if (!conv3x3_wino_supported(C, Cout)) return VD_ERR_SHAPE;
    if (seg_h < 0 || (seg_h > 0 && (seg_h % 2 || H % seg_h))) return VD_ERR_SHAPE;
    return launch_wino(X, N, H, W, C, U, Cout, bias, relu, Y, s, seg_h, 0, 0, 0, 0, 0);
}

// R maps of H x W pixels ([R][H][W][C]) as one 2-D mosaic: each map on an even
// pitch (an odd side gets one phantom row / column that reads 0 and is not stored,
// which is what the map's own zero padding gives that tile), gx maps side by side per
// mosaic row, gx the least count that makes the mosaic width a multiple of 16 (the
// 8 x 16-pixel block: 14 x 14 maps -> gx = 8, 112 columns, no idle block columns);
// the last mosaic row may be partly empty (its pixels read 0 and are not stored)
int launch_conv3x3_wino_mosaic(const float *X, int R, int H, int W, int C, const float *U,
                               int Cout, const float *bias, int relu, float *Y, hipStream_t s) {
    if (R < 0 || H < 0 || W < 0) return VD_ERR_SHAPE;
    if ((int64_t)R * H * W == 0) return VD_OK;
    if (!conv3x3_wino_supported(C, Cout)) return VD_ERR_SHAPE;
    const int ph = H + (H & 1), pw = W + (W & 1);
    int g = 16;
    for (int w = pw; w % 2 == 0 && g > 1; w /= 2) g /= 2;  // 16 / gcd(pw, 16)
    if (g > R) g = R;
    const int64_t Hm = (int64_t)(R + g - 1) / g * ph, Wm = (int64_t)g * pw;
    if (Hm > 0x3fffffff || Wm > 0x3fffffff) return VD_ERR_SHAPE;
    return launch_wino(X, 1, (int)Hm, (int)Wm, C, U, Cout, bias, relu, Y, s, ph, pw, g, R, H, W);
}

}  // namespace vd
