// mmq8.hip — quantized mat-mat (prefill, ne11 > 8) on the int8 matrix cores, all five types.
//
// The integer form of the reference's MMQ (src/ggml-cuda/mmq.cuh:3134 mul_mat_q; int8 tiles
// mma.cuh:515-569; the per-type tile loaders load_tiles_q4_0 / _q8_0 / _q4_K / _q5_K / _q6_K,
// mmq.cuh:2027 for Q6_K) with the arithmetic of ggml-cpu's block dots
// (src/ggml-cpu/quants.c ggml_vec_dot_q4_K_q8_K / _q6_K_q8_K / _q8_0_q8_0), built for gfx950:
//
//   1. mmq8_quant_x: activations -> int8 blocks of 256 exactly as quantize_row_q8_K_ref
//      (src/ggml-quants.c:2555-2591: d = max/-127 of the signed largest-|x| value,
//      q = nearest_int(x * -127/max) clamped to 127, 16-element block sums). The output is not
//      a row-major array but, per (token tile of 64, super-block of 256 k), the exact LDS image
//      the tile kernel consumes, so the kernel copies it with LDS-DMA (buffer_load ... lds, no
//      VGPR round trip, no ds_write) in whole 1-KiB pieces.
//   2. mmq8_kernel<T>: 128 weight rows x 64 tokens per workgroup, 8 waves = 2 K-groups x
//      (2 row halves x 2 token halves); a wave owns 64 rows x 32 tokens, i.e. two 32x32 MFMA
//      tiles that share the token (A) fragment. Per super-block the weight rows are loaded with
//      16-B buffer loads into registers one stage ahead, decoded to int8 codes (Q4_0: q-8,
//      Q4_K: q, Q5_K: q | qh<<4, Q6_K: q-32, Q8_0 as is) and written to LDS in MFMA-fragment
//      order with an XOR swizzle meant to spread the staging writes and fragment reads over the
//      banks (the counters still show 0.14 M SQ_LDS_BANK_CONFLICT cycles per Q8_0 4096 x 4096 x
//      512 call, profiles/r04_mmq8_pmc.txt; the repacked tile below has none). K-group g takes
//      blocks 4g..4g+3 of every super-block.
//        Q8_0 / Q4_0: v_mfma_i32_32x32x32_i8 per 32-k block with C = 0x4B400000: the int32
//          result R + 0x4B400000 IS the f32 bit pattern of 12582912 + R (|R| < 2^22), so one
//          fma per output and block applies the weight scale: p += (12582912 + R) * d_w; the
//          constant 12582912 * sum(d_w) leaves once per super-block.
//        Q4_K / Q5_K: p_i += sc_j * R_j in int32 (v_mad_i32_i24: the 6-bit sub-block scales
//          are integers, as ggml_vec_dot_q4_K_q8_K sums them); the min term sum_j m_j * bsum_j
//          as one f16 MFMA on exact integers; p = d * p_i - dmin * mins.
//        Q6_K: scales are per 16 weights, so one v_mfma_i32_32x32x16_i8 per scale group and
//          p_i += sc_g * R_g (signed); p = d * p_i.
//      and acc += d_x[token] * p once per super-block (the activation scale is per 256).
//   Split-K over workgroups (fixed-order reduce kernel) when the tile grid alone cannot fill
//   the chip; the workgroup -> tile map keeps the token tiles of one row tile on one XCD so
//   that XCD's L2 serves the weight rows to all of them.
//   The integer dot products are those of the CPU backend bit for bit (Q8_K activation blocks,
//   i.e. the CPU's own for the K-quants); only the fp32 order of the scale accumulation differs.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "dispatch.h"
#include "qcommon.h"
#include "settings.h"
#include <string>

namespace mi355x {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void *lds_ptr_t;

constexpr uint32_t Q8_RSRC_W3 = 0x00020000u;   // raw buffer, dword3 for gfx9-class descriptors
constexpr int Q8_QK = 256;                     // activation block = one super-block of k
constexpr int Q8_TOK = 64;                     // tokens per activation image
// TR = weight rows per workgroup (128, or 64 for two workgroups per CU), 4 TR threads
constexpr uint32_t Q8_MAGIC_I = 0x4B400000u;   // f32 bits of 12582912 = 1.5 * 2^23
constexpr float Q8_MAGIC_F = 12582912.0f;
// measurement builds only (scripts/mmq8_exp.sh): 1 no scale epilogue (Q8_0 / Q4_0), 2 no weight
// decode + store, 4 no weight loads, 8 no MFMA phase, 16 no activation DMA. Results are wrong.
#ifndef MMQ8_EXP
#define MMQ8_EXP 0
#endif
#ifndef MMQ8R_EXP
#define MMQ8R_EXP 0
#endif
// repacked tile: the producers also touch (one dword load per 128-B line, result unused) the
// operands RP_TOUCH steps ahead, so that the LDS-DMA of a step two steps ahead finds them in the
// XCD's L2 instead of waiting out an Infinity-Cache / HBM miss (0 = off; measurements)
#ifndef RP_TOUCH
#define RP_TOUCH 0
#endif
// repacked tile: workgroup (row tile r, token tile t) walks its super-blocks starting at
// (RP_ROT_R * r + RP_ROT_T * t) mod steps, so that the workgroups sharing a weight row tile (or an
// activation tile) do not all request the same lines at the same moment (0, 0 = all start at 0)
#ifndef RP_ROT_R
#define RP_ROT_R 3
#endif
#ifndef RP_ROT_T
#define RP_ROT_T 2
#endif

// ---- activation image of one (token tile, super-block): the LDS bytes, 1-KiB pieces ----
//   codes  [blk 8][h 2][tok 64][16 B]            (Q6_K: [blk 8][h 2][hl 2][tok 64][8 B])
//   dx     [tok 64] f32                          at XI_DX
//   bsums  [hl 2][tok 64][8 f16], k16-sums 8hl.. at XI_BS (Q4_K / Q5_K)
constexpr int XI_DX = 16384, XI_BS = 16640;
template <int T> constexpr bool q8_has_min() { return T == T_Q4_K || T == T_Q5_K; }
template <int T> constexpr int ximg_bytes() { return q8_has_min<T>() ? 19456 : 17408; }
// ---- MUL_MAT_ID: expert-sorted (slot, token) pairs (moe_prep below), 64-pair token tiles
//   offsets[e] .. offsets[e+1]: sorted positions of expert e's pairs; tile_off[e]: first tile of
//   expert e (prefix sum of ceil(count / 64)); pos_pair[q]: pair t * n_used + slot at position q
struct Moe8 {
    const int *offsets, *tile_off, *pos_pair;
    int n_expert, n_used;
};
// tile j -> expert e, first sorted position q0, pairs in the tile; false past the last tile.
// The largest e with tile_off[e] <= j is the non-empty expert holding j (empty experts share
// their successor's offset).
__device__ __forceinline__ bool moe8_tile(const Moe8 &m, int j, int &e, int &q0, int &cnt) {
    if (j >= m.tile_off[m.n_expert]) return false;
    int lo = 0, hi = m.n_expert - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (m.tile_off[mid] <= j) lo = mid; else hi = mid - 1;
    }
    e = lo;
    q0 = m.offsets[e] + (j - m.tile_off[e]) * 64;
    cnt = min(64, m.offsets[e + 1] - q0);
    return true;
}

// ---- weight image: codes [blk 8][h 2][row TR][16 B] (Q6_K [blk][h][hl][row][8 B]) + meta [kg][row][16 B]
template <int TR> constexpr int wi_meta() { return 256 * TR; }
template <int TR> constexpr int wi_bytes() { return 288 * TR; }

// 16-B code piece (blk, h) of weight row `row`. The XOR permutes rows inside a group of 16, so a
// fragment read (16 lanes = 16 consecutive rows of one piece) still touches every LDS bank once;
// the XOR pattern is chosen per staging map so that the 16 lanes of a staging write, which hold
// different pieces of few rows, land on 16 distinct 16-B slots as well.
template <int T> __device__ __forceinline__ int swz16(int blk, int h) {
    return q8_has_min<T>() ? (4 * h + 8 * ((blk >> 1) & 1)) : (blk + 8 * h);
}
template <int T, int TR> __device__ __forceinline__ uint32_t wslot16(int blk, int h, int row) {
    return (uint32_t)(blk * 32 * TR + h * 16 * TR + ((row ^ swz16<T>(blk, h)) << 4));
}
// Q6_K: 8-B piece (blk, h, hl) (one 16-weight scale group per 32x32x16 MFMA); rows permuted
// inside groups of 32 (a 32-lane ds_read_b64 reads 32 consecutive rows)
__device__ __forceinline__ int swz8(int blk, int h) { return 8 * (2 * (blk >> 2) + h); }
template <int TR> __device__ __forceinline__ uint32_t wslot8(int blk, int h, int hl, int row) {
    return (uint32_t)(blk * 32 * TR + h * 16 * TR + hl * 8 * TR + ((row ^ swz8(blk, h)) << 3));
}

__device__ __forceinline__ u32x4v bl128(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t bl32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ void st128(uint8_t *p, u32x4v v) { *reinterpret_cast<u32x4v *>(p) = v; }
__device__ __forceinline__ void st64(uint8_t *p, u32x2v v) { *reinterpret_cast<u32x2v *>(p) = v; }
__device__ __forceinline__ u32x4v ld128(const uint8_t *p) { return *reinterpret_cast<const u32x4v *>(p); }
__device__ __forceinline__ u32x2v ld64(const uint8_t *p) { return *reinterpret_cast<const u32x2v *>(p); }
__device__ __forceinline__ float uf(uint32_t u) { return __builtin_bit_cast(float, u); }
__device__ __forceinline__ uint32_t fu(float f) { return __builtin_bit_cast(uint32_t, f); }
__device__ __forceinline__ i32x4 as_i4(u32x4v v) { return __builtin_bit_cast(i32x4, v); }
__device__ __forceinline__ long as_l(u32x2v v) { return __builtin_bit_cast(long, v); }

// 16 B per lane from the buffer straight into LDS at lds_dst + 16 * lane (lds_dst wave-uniform)
__device__ __forceinline__ void q8_dma16(__amdgpu_buffer_rsrc_t r, uint8_t *lds_dst, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds_dst, 16, voff, 0, 0, 0);
}

// ------------------------------------------------------------------------------------------
// activations -> Q8_K blocks, written as stage images (restates quantize_row_q8_K_ref,
// src/ggml-quants.c:2555-2591). One wave per (token, super-block): lane l holds k = 4l..4l+3,
// one coalesced 16-B load (a token's 1 KB per wave instruction); the largest |x| over the 256
// values by DPP / permlane exchanges, no LDS; lane l writes its 4 codes (one dword of a 16-B
// code piece) and, per 16-element block, the lane of the piece's first dword its sum.
// ------------------------------------------------------------------------------------------
// MOE: token index = position in the tile-padded pair list (tile tok / 64 of moe), its column
// gathered from src1 (slot % ne11, token) as mmq_convert_x does; padding positions are zeros.
// zero_dst: also clear dst (the 2-way split-K kernel adds both halves into it): the wave of
// (token, super-block sb) clears columns [sb * ceil(N / n_sb), ...) of the token's row.
// grid.x = (64-token images) * 16 * n_sb: 4 tokens (waves) of one super-block per workgroup.
template <int T, bool MOE = false>
__global__ __launch_bounds__(256) void mmq8_quant_x(const MmArgs a, uint8_t *__restrict__ ximg, int n_tt, int n_sb,
                                                    const Moe8 moe, int zero_dst) {
    constexpr int XB = ximg_bytes<T>();
    const int lane = threadIdx.x & 63;
    const int tok = (blockIdx.x / n_sb) * 4 + (threadIdx.x >> 6), sb = blockIdx.x % n_sb;
    const int slice = blockIdx.y;
    const int i12 = slice % a.ne12, i13 = slice / a.ne12;
    if (!MOE && zero_dst && tok < a.M) {
        const int chunk = (a.N + n_sb - 1) / n_sb, c1 = min(a.N, (sb + 1) * chunk);
        float *drow = reinterpret_cast<float *>(a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3 + (int64_t)tok * a.nb1);
        for (int c = sb * chunk + lane; c < c1; c += 64) drow[c] = 0.f;
    }
    const uint8_t *row = nullptr;
    if constexpr (MOE) {
        int e, q0, cnt;
        if (!moe8_tile(moe, tok >> 6, e, q0, cnt)) return;   // (uniform: 4 tokens of one tile)
        if ((tok & 63) < cnt) {
            const int pair = moe.pos_pair[q0 + (tok & 63)];
            row = a.x + (int64_t)((pair % moe.n_used) % a.ne11_b) * a.nb11 + (int64_t)(pair / moe.n_used) * a.nb12;
        }
    } else if (tok < a.M) {
        row = a.x + (int64_t)i12 * a.nb12 + (int64_t)i13 * a.nb13 + (int64_t)tok * a.nb11;
    }
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    const int k0 = sb * Q8_QK + 4 * lane;
    if (row != nullptr && k0 < a.K) {   // (K % 32 == 0: a lane's 4 values are all in or all out)
        const float *src = reinterpret_cast<const float *>(row) + k0;
        if (a.x_aligned16) {
            const float4 f = *reinterpret_cast<const float4 *>(src);
            v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = src[i];
        }
    }
    // the signed value of largest |x|, first k on ties (the reference's strict '>'): (|x|, k, x)
    // reduced with max |x|, then min k — a total order, so the butterfly gives every lane the
    // same winner
    float am = fabsf(v[0]), mx = v[0];
    int idx = 4 * lane;
#pragma unroll
    for (int i = 1; i < 4; ++i)
        if (fabsf(v[i]) > am) { am = fabsf(v[i]); mx = v[i]; idx = 4 * lane + i; }
    auto take = [&](float am2, float mx2, int idx2) {
        if (am2 > am || (am2 == am && idx2 < idx)) { am = am2; mx = mx2; idx = idx2; }
    };
#define Q8X_STEP(D) take(xchg<D>(am), xchg<D>(mx), __builtin_bit_cast(int, xchg<D>(__builtin_bit_cast(float, idx))))
    Q8X_STEP(1); Q8X_STEP(2); Q8X_STEP(4); Q8X_STEP(8); Q8X_STEP(16); Q8X_STEP(32);
#undef Q8X_STEP
    uint32_t w = 0u;
    int s = 0;
    float d = 0.f;
    if (am != 0.f) {
        const float iscale = -127.f / mx;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int q = min(127, (int)__builtin_rintf(iscale * v[i]));
            s += q;
            w |= (uint32_t)(q & 0xff) << (8 * i);
        }
        d = 1.f / iscale;
    }
    uint8_t *img = ximg + (((int64_t)slice * n_tt + (tok >> 6)) * n_sb + sb) * XB;
    const int tl = tok & 63, p = lane >> 2, blk = p >> 1, h = p & 1;   // p: 16-element piece
    if constexpr (T == T_Q6_K)
        *reinterpret_cast<uint32_t *>(img + blk * 2048 + h * 1024 + ((lane >> 1) & 1) * 512 + tl * 8 + (lane & 1) * 4) = w;
    else
        *reinterpret_cast<uint32_t *>(img + blk * 2048 + h * 1024 + tl * 16 + (lane & 3) * 4) = w;
    if constexpr (q8_has_min<T>()) {
        float fs = (float)s;   // |sums| <= 16 * 127: exact
        fs += xchg<1>(fs);
        fs += xchg<2>(fs);
        if ((lane & 3) == 0) *reinterpret_cast<_Float16 *>(img + XI_BS + (p >> 3) * 1024 + tl * 16 + 2 * (p & 7)) = (_Float16)fs;
    }
    if (lane == 0) *reinterpret_cast<float *>(img + XI_DX + tl * 4) = d;
}

// ------------------------------------------------------------------------------------------
// weight staging. Every thread loads its tasks of the row tile's super-block into registers one
// stage ahead and, after the stage's MFMAs, decodes them into the LDS image. Tasks run along the
// rows (consecutive lanes = consecutive blocks / chunks of one row), so a wave's 16-B loads
// cover a few whole rows (coalesced) instead of one window of many rows.
// ------------------------------------------------------------------------------------------
// first row of the tile, rows of the matrix, row pitch, super-block offset (plus the matrix's
// misalignment below a dword: the buffer base is the dword floor of the matrix), and the 32-blocks
// of a row left from this super-block on (Q4_0 / Q8_0: K need not be a multiple of 256; blocks
// past the row's end get a zero scale)
struct RowTile {
    int row0, N;
    uint32_t nb01, sboff;
    int blk_left;
    __device__ __forceinline__ uint32_t rb(int row) const {
        return (uint32_t)min(row0 + row, N - 1) * nb01 + sboff;
    }
};

template <int T> struct WStage8;

// Q8_0: task (row, block) = (t >> 3, t & 7), t = tid + 512 e. Blocks are 2-byte aligned (34-B
// blocks, rows and matrices at any even offset): a block starting at 0 mod 4 has its codes at +2,
// one starting at 2 mod 4 has them dword-aligned; one v_perm per dword realigns either, chosen
// per lane from the block's own offset.
template <> struct WStage8<T_Q8_0> {
    static constexpr int VMEM = 6;   // vector-memory instructions of one load()
    uint32_t w[2][9];
    template <int TR> __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, const RowTile &R, int tid) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int t = tid + 4 * TR * e;
            const uint32_t o4 = (R.rb(t >> 3) + 34u * (t & 7)) & ~3u;
            const u32x4v a0 = bl128(rs, o4), a1 = bl128(rs, o4 + 16);
            w[e][0] = a0[0]; w[e][1] = a0[1]; w[e][2] = a0[2]; w[e][3] = a0[3];
            w[e][4] = a1[0]; w[e][5] = a1[1]; w[e][6] = a1[2]; w[e][7] = a1[3];
            w[e][8] = bl32(rs, o4 + 32);
        }
    }
    template <int TR> __device__ __forceinline__ void store(uint8_t *W, const RowTile &R, int tid) const {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int t = tid + 4 * TR * e, row = t >> 3, blk = t & 7;
            const int odd = ((R.rb(row) >> 1) ^ blk) & 1;   // the block starts at 2 mod 4
            const uint32_t sel = odd ? 0x07060504u : 0x05040302u;
            uint32_t c[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_perm(w[e][i + 1], w[e][i], sel);
            const float d = blk < R.blk_left ? h2f((uint16_t)(odd ? w[e][0] >> 16 : w[e][0] & 0xffffu)) : 0.f;
            st128(W + wslot16<T_Q8_0, TR>(blk, 0, row), u32x4v{c[0], c[1], c[2], c[3]});
            st128(W + wslot16<T_Q8_0, TR>(blk, 1, row), u32x4v{c[4], c[5], c[6], c[7]});
            *reinterpret_cast<float *>(W + wi_meta<TR>() + (blk >> 2) * 16 * TR + row * 16 + 4 * (blk & 3)) = d;
        }
    }
};

// Q4_0: as Q8_0 with 18-B blocks; codes decoded to q - 8
template <> struct WStage8<T_Q4_0> {
    static constexpr int VMEM = 4;
    uint32_t w[2][5];
    template <int TR> __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, const RowTile &R, int tid) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int t = tid + 4 * TR * e;
            const uint32_t o4 = (R.rb(t >> 3) + 18u * (t & 7)) & ~3u;
            const u32x4v a0 = bl128(rs, o4);
            w[e][0] = a0[0]; w[e][1] = a0[1]; w[e][2] = a0[2]; w[e][3] = a0[3];
            w[e][4] = bl32(rs, o4 + 16);
        }
    }
    template <int TR> __device__ __forceinline__ void store(uint8_t *W, const RowTile &R, int tid) const {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int t = tid + 4 * TR * e, row = t >> 3, blk = t & 7;
            const int odd = ((R.rb(row) >> 1) ^ blk) & 1;
            const uint32_t sel = odd ? 0x07060504u : 0x05040302u;
            uint32_t lo[4], hi[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t n = __builtin_amdgcn_perm(w[e][i + 1], w[e][i], sel);
                lo[i] = sub8_bytes(n & 0x0F0F0F0Fu);          // k 0..15
                hi[i] = sub8_bytes((n >> 4) & 0x0F0F0F0Fu);   // k 16..31
            }
            const float d = blk < R.blk_left ? h2f((uint16_t)(odd ? w[e][0] >> 16 : w[e][0] & 0xffffu)) : 0.f;
            st128(W + wslot16<T_Q4_0, TR>(blk, 0, row), u32x4v{lo[0], lo[1], lo[2], lo[3]});
            st128(W + wslot16<T_Q4_0, TR>(blk, 1, row), u32x4v{hi[0], hi[1], hi[2], hi[3]});
            *reinterpret_cast<float *>(W + wi_meta<TR>() + (blk >> 2) * 16 * TR + row * 16 + 4 * (blk & 3)) = d;
        }
    }
};

// Q4_K / Q5_K (16-B aligned super-blocks): task (row, q) = (tid >> 2, tid & 3): qs chunks q and
// q+4 (64-weight chunk c = q>>1 (+2), half h = q&1: low nibbles -> block 2c, high -> 2c+1);
// Q5_K adds qh chunk h; q == 0 the header. meta [kg][row] = {d, dmin, sc (4 B), m (4 B)} of
// sub-blocks 4kg..4kg+3
template <int T> struct WStageK8 {
    static constexpr bool Q5 = T == T_Q5_K;
    static constexpr uint32_t QS = Q5 ? 48 : 16;
    static constexpr int VMEM = Q5 ? 4 : 3;
    u32x4v c[2], qh, hd;
    template <int TR> __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, const RowTile &R, int tid) {
        const int q = tid & 3;
        const uint32_t rb = R.rb(tid >> 2);
        c[0] = bl128(rs, rb + QS + 16u * q);
        c[1] = bl128(rs, rb + QS + 16u * (q + 4));
        if constexpr (Q5) qh = bl128(rs, rb + 16 + 16u * (q & 1));
        hd = bl128(rs, rb);   // every lane (one line per row): no load under a branch
    }
    template <int TR> __device__ __forceinline__ void store(uint8_t *W, const RowTile &, int tid) const {
        const int q = tid & 3, row = tid >> 2, h = q & 1;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int cc = (q >> 1) + 2 * e;   // 64-weight chunk
            u32x4v lo, hi;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                lo[i] = c[e][i] & 0x0F0F0F0Fu;
                hi[i] = (c[e][i] >> 4) & 0x0F0F0F0Fu;
                if constexpr (Q5) {
                    lo[i] |= ((qh[i] >> (2 * cc)) & 0x01010101u) << 4;
                    hi[i] |= ((qh[i] >> (2 * cc + 1)) & 0x01010101u) << 4;
                }
            }
            st128(W + wslot16<T, TR>(2 * cc, h, row), lo);
            st128(W + wslot16<T, TR>(2 * cc + 1, h, row), hi);
        }
        if (q == 0) {   // get_scale_min_k4 (src/ggml-quants.c:703-710) in the packed form of quants.c:580-585
            const uint32_t S0 = hd[1], S1 = hd[2], S2 = hd[3];
            const uint32_t sc_lo = S0 & 0x3f3f3f3fu;
            const uint32_t sc_hi = (S2 & 0x0f0f0f0fu) | (((S0 >> 6) & 0x03030303u) << 4);
            const uint32_t mn_lo = S1 & 0x3f3f3f3fu;
            const uint32_t mn_hi = ((S2 >> 4) & 0x0f0f0f0fu) | (((S1 >> 6) & 0x03030303u) << 4);
            const uint32_t d = fu(h2f((uint16_t)(hd[0] & 0xffffu))), dmin = fu(h2f((uint16_t)(hd[0] >> 16)));
            st128(W + wi_meta<TR>() + row * 16, u32x4v{d, dmin, sc_lo, mn_lo});
            st128(W + wi_meta<TR>() + 16 * TR + row * 16, u32x4v{d, dmin, sc_hi, mn_hi});
        }
    }
};
template <> struct WStage8<T_Q4_K> : WStageK8<T_Q4_K> {};
template <> struct WStage8<T_Q5_K> : WStageK8<T_Q5_K> {};

// Q6_K (210-B super-blocks, 2-byte aligned): task (row, q) = (tid >> 2, tid & 3), half hf = q>>1,
// k-half h = q&1 of each of the four 32-blocks 4hf..4hf+3: ql[64hf+16h..], ql[64hf+32+16h..],
// qh[32hf+16h..] (16 B each), decoded as dequantize_row_q6_K (src/ggml-quants.c:1762-1791) to
// q - 32; q == 0 also the scales and d. meta [kg = hf][row] = {d, sc[8kg .. 8kg+7] (int8), 0}
template <> struct WStage8<T_Q6_K> {
    static constexpr int VMEM = 8;
    uint32_t w[3][5], s[5];
    template <int TR> __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, const RowTile &R, int tid) {
        const int q = tid & 3;
        const uint32_t rb = R.rb(tid >> 2), hf = q >> 1, h = q & 1;
        const uint32_t po[3] = {64 * hf + 16 * h, 64 * hf + 32 + 16 * h, 128 + 32 * hf + 16 * h};
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const uint32_t o4 = (rb + po[p]) & ~3u;
            const u32x4v a0 = bl128(rs, o4);
            w[p][0] = a0[0]; w[p][1] = a0[1]; w[p][2] = a0[2]; w[p][3] = a0[3];
            w[p][4] = bl32(rs, o4 + 16);
        }
        {   // scales + d, every lane (no load under a branch)
            const uint32_t o4 = (rb + 192) & ~3u;
            const u32x4v a0 = bl128(rs, o4);
            s[0] = a0[0]; s[1] = a0[1]; s[2] = a0[2]; s[3] = a0[3];
            s[4] = bl32(rs, o4 + 16);
        }
    }
    template <int TR> __device__ __forceinline__ void store(uint8_t *W, const RowTile &R, int tid) const {
        const int q = tid & 3, row = tid >> 2, hf = q >> 1, h = q & 1;
        const uint32_t sel = (R.rb(row) & 2) ? 0x05040302u : 0x03020100u;   // realign by 0 or 2 bytes
        uint32_t la[4], lb[4], qh[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            la[i] = __builtin_amdgcn_perm(w[0][i + 1], w[0][i], sel);
            lb[i] = __builtin_amdgcn_perm(w[1][i + 1], w[1][i], sel);
            qh[i] = __builtin_amdgcn_perm(w[2][i + 1], w[2][i], sel);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            uint32_t v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t x;
                if (t == 0) x = (la[i] & 0x0F0F0F0Fu) | ((qh[i] << 4) & 0x30303030u);
                else if (t == 1) x = (lb[i] & 0x0F0F0F0Fu) | ((qh[i] << 2) & 0x30303030u);
                else if (t == 2) x = ((la[i] >> 4) & 0x0F0F0F0Fu) | (qh[i] & 0x30303030u);
                else x = ((lb[i] >> 4) & 0x0F0F0F0Fu) | ((qh[i] >> 2) & 0x30303030u);
                v[i] = sub32_bytes(x);
            }
            const int blk = 4 * hf + t;
            st64(W + wslot8<TR>(blk, h, 0, row), u32x2v{v[0], v[1]});
            st64(W + wslot8<TR>(blk, h, 1, row), u32x2v{v[2], v[3]});
        }
        if (q == 0) {
            uint32_t sc[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) sc[i] = __builtin_amdgcn_perm(s[i + 1], s[i], sel);
            const uint32_t dd = __builtin_amdgcn_perm(s[4], s[4], sel) & 0xffffu;
            const uint32_t d = fu(h2f((uint16_t)dd));
            st128(W + wi_meta<TR>() + row * 16, u32x4v{d, sc[0], sc[1], 0u});
            st128(W + wi_meta<TR>() + 16 * TR + row * 16, u32x4v{d, sc[2], sc[3], 0u});
        }
    }
};

// ------------------------------------------------------------------------------------------
// one super-block of one wave: NG K-groups of 4 blocks starting at group g0 (NG = 1: the
// workgroup splits the super-block between two K-groups of waves; NG = 2: the wave takes all 8
// blocks), tokens 32tg.. of the activation image X x rows 64rg.. (two 32x32 tiles).
// acc[ti][i]: token 32tg + 8(i>>2) + 4hl + (i&3), weight row 64rg + 32ti + (lane & 31)
// Software pipeline of depth one: the MFMAs of step s are issued before the results of step s-1
// are consumed, and a scheduling barrier per step keeps the compiler from hoisting every step's
// MFMAs (their int32 results would not fit the register budget of 2 waves / SIMD).
// ------------------------------------------------------------------------------------------
template <int T, int NG, int TR>
__device__ __forceinline__ void q8_sb_compute(const uint8_t *W, const uint8_t *X, int g0, int rg, int tg, int lane,
                                              f32x16 &acc0, f32x16 &acc1) {
    const int r = lane & 31, hl = lane >> 5;
    const int row0 = 64 * rg + r, row1 = row0 + 32, tok = 32 * tg + r;
    f32x16 p0, p1;
    i32x16 zero;
#pragma unroll
    for (int i = 0; i < 16; ++i) { p0[i] = 0.f; p1[i] = 0.f; zero[i] = 0; }
    if constexpr (T == T_Q8_0 || T == T_Q4_0) {
        i32x16 magic;
#pragma unroll
        for (int i = 0; i < 16; ++i) magic[i] = (int)Q8_MAGIC_I;
        asm volatile("" : "+v"(magic));   // opaque: not rematerialized, so the pin below holds its registers
        // the magic constant's share, -12582912 * sum(d_w), starts the sums (folded into the first
        // fma of every output instead of a subtraction at the end)
        // (NG = 2 reads the meta again per group rather than holding 16 more registers)
        float dsum0 = 0.f, dsum1 = 0.f;
#pragma unroll
        for (int g = g0; g < g0 + NG; ++g) {
            const u32x4v m0 = ld128(W + wi_meta<TR>() + g * 16 * TR + row0 * 16);
            const u32x4v m1 = ld128(W + wi_meta<TR>() + g * 16 * TR + row1 * 16);
            dsum0 += (uf(m0[0]) + uf(m0[1])) + (uf(m0[2]) + uf(m0[3]));
            dsum1 += (uf(m1[0]) + uf(m1[1])) + (uf(m1[2]) + uf(m1[3]));
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) { p0[i] = -Q8_MAGIC_F * dsum0; p1[i] = -Q8_MAGIC_F * dsum1; }
#pragma unroll
        for (int g = g0; g < g0 + NG; ++g) {
            const u32x4v m0 = ld128(W + wi_meta<TR>() + g * 16 * TR + row0 * 16);
            const u32x4v m1 = ld128(W + wi_meta<TR>() + g * 16 * TR + row1 * 16);
            auto issue = [&](int bi, i32x16 &R0, i32x16 &R1) {
                const int blk = 4 * g + bi;
                const u32x4v A = ld128(X + blk * 2048 + hl * 1024 + tok * 16);
                const u32x4v B0 = ld128(W + wslot16<T, TR>(blk, hl, row0));
                const u32x4v B1 = ld128(W + wslot16<T, TR>(blk, hl, row1));
                R0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(as_i4(A), as_i4(B0), magic, 0, 0, 0);
                R1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(as_i4(A), as_i4(B1), magic, 0, 0, 0);
            };
            auto consume = [&](int bi, const i32x16 &R0, const i32x16 &R1) {
                if constexpr (MMQ8_EXP & 1) { asm volatile("" ::"v"(R0), "v"(R1)); return; }
                const float d0 = uf(m0[bi]), d1 = uf(m1[bi]);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    p0[i] = __builtin_fmaf(uf((uint32_t)R0[i]), d0, p0[i]);
                    p1[i] = __builtin_fmaf(uf((uint32_t)R1[i]), d1, p1[i]);
                }
                asm volatile("" : "+v"(p0), "+v"(p1));
            };
            i32x16 Ra0, Ra1, Rb0, Rb1;
            issue(0, Ra0, Ra1);
            issue(1, Rb0, Rb1);
            consume(0, Ra0, Ra1);
            __builtin_amdgcn_sched_barrier(0);
            issue(2, Ra0, Ra1);
            consume(1, Rb0, Rb1);
            __builtin_amdgcn_sched_barrier(0);
            issue(3, Rb0, Rb1);
            consume(2, Ra0, Ra1);
            __builtin_amdgcn_sched_barrier(0);
            consume(3, Rb0, Rb1);
        }
        // keep the C-input registers allocated past the last MFMA that reads them (without this
        // the compiler recycles them as epilogue destinations 7 wait states after that MFMA)
        asm volatile("" ::"v"(magic));
    } else {   // K-quants: integer sub-block (or 16-group) scales, exact int32 sums
        i32x16 pi0, pi1;
#pragma unroll
        for (int i = 0; i < 16; ++i) { pi0[i] = 0; pi1[i] = 0; }
        auto consume = [&](int s0, int s1, const i32x16 &R0, const i32x16 &R1) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                pi0[i] += __mul24(R0[i], s0);
                pi1[i] += __mul24(R1[i], s1);
            }
            // integer adds may be reassociated: without this the compiler multiplies every step's
            // results first and keeps all of them live (spills); pin the accumulators per step
            asm volatile("" : "+v"(pi0), "+v"(pi1));
        };
        float dd0 = 0.f, dd1 = 0.f, dm0 = 0.f, dm1 = 0.f;
#pragma unroll
        for (int g = g0; g < g0 + NG; ++g) {
            const u32x4v m0 = ld128(W + wi_meta<TR>() + g * 16 * TR + row0 * 16);
            const u32x4v m1 = ld128(W + wi_meta<TR>() + g * 16 * TR + row1 * 16);
            dd0 = uf(m0[0]); dd1 = uf(m1[0]); dm0 = uf(m0[1]); dm1 = uf(m1[1]);
            if constexpr (T == T_Q4_K || T == T_Q5_K) {
                auto issue = [&](int bi, i32x16 &R0, i32x16 &R1) {
                    const int blk = 4 * g + bi;
                    const u32x4v A = ld128(X + blk * 2048 + hl * 1024 + tok * 16);
                    const u32x4v B0 = ld128(W + wslot16<T, TR>(blk, hl, row0));
                    const u32x4v B1 = ld128(W + wslot16<T, TR>(blk, hl, row1));
                    R0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(as_i4(A), as_i4(B0), zero, 0, 0, 0);
                    R1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(as_i4(A), as_i4(B1), zero, 0, 0, 0);
                };
                auto sc = [&](const u32x4v &m, int bi) { return (int)((m[2] >> (8 * bi)) & 0xffu); };
                i32x16 Ra0, Ra1, Rb0, Rb1;
                issue(0, Ra0, Ra1);
                issue(1, Rb0, Rb1);
                consume(sc(m0, 0), sc(m1, 0), Ra0, Ra1);
                __builtin_amdgcn_sched_barrier(0);
                issue(2, Ra0, Ra1);
                consume(sc(m0, 1), sc(m1, 1), Rb0, Rb1);
                __builtin_amdgcn_sched_barrier(0);
                issue(3, Rb0, Rb1);
                consume(sc(m0, 2), sc(m1, 2), Ra0, Ra1);
                __builtin_amdgcn_sched_barrier(0);
                consume(sc(m0, 3), sc(m1, 3), Rb0, Rb1);
            } else {   // Q6_K: 8 scale groups q = 2 bi + h per K-group, one 32x32x16 MFMA each
                auto issue = [&](int q, i32x16 &R0, i32x16 &R1) {
                    const int blk = 4 * g + (q >> 1), h = q & 1;
                    const u32x2v A = ld64(X + blk * 2048 + h * 1024 + hl * 512 + tok * 8);
                    const u32x2v B0 = ld64(W + wslot8<TR>(blk, h, hl, row0));
                    const u32x2v B1 = ld64(W + wslot8<TR>(blk, h, hl, row1));
                    R0 = __builtin_amdgcn_mfma_i32_32x32x16_i8(as_l(A), as_l(B0), zero, 0, 0, 0);
                    R1 = __builtin_amdgcn_mfma_i32_32x32x16_i8(as_l(A), as_l(B1), zero, 0, 0, 0);
                };
                auto sc = [&](const u32x4v &m, int q) {
                    return (int)(int8_t)(uint8_t)((q < 4 ? m[1] : m[2]) >> (8 * (q & 3)));
                };
                i32x16 Ra0, Ra1, Rb0, Rb1;
                issue(0, Ra0, Ra1);
#pragma unroll
                for (int q = 1; q < 8; ++q) {
                    if (q & 1) issue(q, Rb0, Rb1);
                    else issue(q, Ra0, Ra1);
                    if (q & 1) consume(sc(m0, q - 1), sc(m1, q - 1), Ra0, Ra1);
                    else consume(sc(m0, q - 1), sc(m1, q - 1), Rb0, Rb1);
                    __builtin_amdgcn_sched_barrier(0);
                }
                consume(sc(m0, 7), sc(m1, 7), Rb0, Rb1);
            }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) { p0[i] = dd0 * (float)pi0[i]; p1[i] = dd1 * (float)pi1[i]; }
        if constexpr (T == T_Q4_K || T == T_Q5_K) {
            // sum_j m_j * bsum_j over all 8 sub-blocks (k16-sum e pairs with m_(e>>1)) as one f16
            // MFMA on exact integers per tile; the two K-groups take one tile each (the partials
            // meet in the K-group reduction), a wave holding both groups (NG = 2) both tiles
            const f16x8 As = __builtin_bit_cast(f16x8, ld128(X + XI_BS + hl * 1024 + tok * 16));
            f32x16 zf;
#pragma unroll
            for (int i = 0; i < 16; ++i) zf[i] = 0.f;
            auto mins_of = [&](int row) {
                const uint32_t mw = *reinterpret_cast<const uint32_t *>(W + wi_meta<TR>() + hl * 16 * TR + row * 16 + 12);
                u32x4v bm;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t hb = __builtin_bit_cast(uint16_t, (_Float16)(float)((mw >> (8 * k)) & 0xffu));
                    bm[k] = hb | (hb << 16);
                }
                return __builtin_amdgcn_mfma_f32_32x32x16_f16(As, __builtin_bit_cast(f16x8, bm), zf, 0, 0, 0);
            };
            if (NG == 2 || g0 == 0) {
                const f32x16 mins0 = mins_of(row0);
#pragma unroll
                for (int i = 0; i < 16; ++i) p0[i] = __builtin_fmaf(-dm0, mins0[i], p0[i]);
            }
            if (NG == 2 || g0 != 0) {
                const f32x16 mins1 = mins_of(row1);
#pragma unroll
                for (int i = 0; i < 16; ++i) p1[i] = __builtin_fmaf(-dm1, mins1[i], p1[i]);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const u32x4v dx = ld128(X + XI_DX + 4 * (32 * tg + 8 * q + 4 * hl));
        const float dv[4] = {uf(dx[0]), uf(dx[1]), uf(dx[2]), uf(dx[3])};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            acc0[4 * q + c] = __builtin_fmaf(p0[4 * q + c], dv[c], acc0[4 * q + c]);
            acc1[4 * q + c] = __builtin_fmaf(p1[4 * q + c], dv[c], acc1[4 * q + c]);
        }
    }
}

// 4 B per lane from the buffer into LDS at lds_dst + 4 * lane (a 256-B piece per wave)
__device__ __forceinline__ void q8_dma4(__amdgpu_buffer_rsrc_t r, uint8_t *lds_dst, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds_dst, 4, voff, 0, 0, 0);
}

// copy one activation image into LDS with the same instruction count in every wave (the
// counted vmcnt waits below rely on it): the 16 KiB of codes as 1-KiB pieces w, w+NW, ..; the
// 256-B dx row by every wave (identical bytes to the same place); the 2-KiB bsums (Q4_K / Q5_K)
// as 256-B shares w, w+NW, ..
template <int T, int NW> constexpr int q8_x_vmem() { return 16 / NW + 1 + (q8_has_min<T>() ? 8 / NW : 0); }
template <int T, int NW>
__device__ __forceinline__ void q8_x_dma(__amdgpu_buffer_rsrc_t xr, uint32_t img_off, uint8_t *X, int wave, int lane) {
#pragma unroll
    for (int p = 0; p < 16 / NW; ++p) {
        const int pc = wave + p * NW;
        q8_dma16(xr, X + pc * 1024, img_off + pc * 1024 + lane * 16);
    }
    q8_dma4(xr, X + XI_DX, img_off + XI_DX + lane * 4);
    if constexpr (q8_has_min<T>()) {
#pragma unroll
        for (int s = 0; s < 8 / NW; ++s) {
            const int sh = wave + s * NW;
            q8_dma4(xr, X + XI_BS + sh * 256, img_off + XI_BS + sh * 256 + lane * 4);
        }
    }
}

// stream-K state (SK kernels): per-tile arrival counters (zero between launches: the second
// arrival re-arms its tile's), two partial slots per tile, the tile count of one slice
struct StreamK {
    int *cnt;
    float *part;
    int n_tiles;
};
constexpr int MMQ8_SK_WGS = 256;   // stream-K grid: one workgroup per CU (the 128-row tiles hold ~136 KB of LDS)

// one (row tile, token tile, super-block range) of mmq8_kernel: stages, steps, K-group
// reduction and the epilogue (plain store, the 2-way split-K atomic add, the split-K partial, or
// the stream-K hand-off)
template <int T, int TT, int TR, bool MOE, bool SK>
__device__ __forceinline__ void mmq8_job(const MmArgs &a, const uint8_t *__restrict__ ximg, int n_tt, uint32_t w_extent,
                                         float *__restrict__ part, int xcd_remap, const Moe8 &moe, const StreamK &sk,
                                         uint8_t *lds, int rt, int tt, int sb0, int sb1, int ksplit, int ks, int slice) {
    constexpr int NW = TR / 16;                    // waves
    constexpr int WB = wi_bytes<TR>();
    constexpr int XB = ximg_bytes<T>();
    constexpr int NI = TT / Q8_TOK;                // activation images per stage
    constexpr int N_XS = (TT == 64 && TR == 128) ? 3 : 2;   // activation stage ring
    constexpr int DX = N_XS - 1;                   // activation DMA distance (super-blocks ahead)
    uint8_t *const Xs = lds + 2 * WB;
    const int n_sb = (a.K + Q8_QK - 1) / Q8_QK;
    const int i12 = slice % a.ne12, i13 = slice / a.ne12;
    int ex = 0, q0 = 0, n_tok = a.M;   // MOE: expert, first sorted pair, pairs of the tile
    if constexpr (MOE)
        if (!moe8_tile(moe, slice, ex, q0, n_tok)) return;   // (uniform, before any barrier)
    const uint8_t *wmat = MOE ? a.w + (int64_t)ex * a.nb02
                              : a.w + (int64_t)(i12 / a.r2) * a.nb02 + (int64_t)(i13 / a.r3) * a.nb03;
    // buffer base = the dword floor of the matrix, so that every window below is dword-aligned
    const uint32_t wmis = (uint32_t)(reinterpret_cast<uintptr_t>(wmat) & 3);
    // (w_extent: bytes from the matrix start to its last row's end; rounded up to the dword
    // holding that end, so no window reaches into a later dword)
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void *)(wmat - wmis), 0, (w_extent + wmis + 3) & ~3u, Q8_RSRC_W3);
    // the NI consecutive 64-token images of this tile: [slice][64-token tile][sb][image]
    const uint8_t *xbase = ximg + ((int64_t)slice * n_tt * NI + (int64_t)tt * NI) * n_sb * XB;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc((void *)xbase, 0, (uint32_t)(NI * n_sb * XB), Q8_RSRC_W3);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (scalar) roles
    // wave roles: rg = 64-row group, tg = 32-token group, kg = K-group (TT = 64)
    constexpr int NRG = TR / 64, NTG = TT / 32, NKG = NW / (NRG * NTG);
    static_assert(NKG == (TT == 64 ? 2 : 1), "wave layout");
    const int rg = wave % NRG, tg = (wave / NRG) % NTG, kg = wave / (NRG * NTG);
    constexpr uint32_t SBB = (uint32_t)QT<T>::bytes * (Q8_QK / QT<T>::blck);   // bytes of one row's super-block
    constexpr int NXV = NI * q8_x_vmem<T, NW>();   // vector-memory instructions of one activation stage
    auto rowtile = [&](int sb) {
        return RowTile{rt * TR, a.N, (uint32_t)a.nb01, (uint32_t)sb * SBB + wmis, a.K / 32 - 8 * sb};
    };

    f32x16 acc0, acc1;
#pragma unroll
    for (int i = 0; i < 16; ++i) { acc0[i] = 0.f; acc1[i] = 0.f; }

    // Every load below is issued unconditionally (past the last super-block the source is the
    // last one again and the destination a stage nobody reads any more): a load under a branch
    // makes the compiler's in-order vmcnt bookkeeping fall back to draining everything.
    auto x_issue = [&](int it_dst, int sb) {   // activation images of sb into ring slot it_dst
        uint8_t *dst = Xs + (it_dst % N_XS) * NI * XB;
#pragma unroll
        for (int i = 0; i < NI; ++i) q8_x_dma<T, NW>(xr, (uint32_t)((i * n_sb + sb) * XB), dst + i * XB, wave, lane);
    };
    const int n_steps = sb1 - sb0;
    if (n_steps <= 0) return;   // (uniform: a whole workgroup with no k range)
    auto sbc = [&](int it) { return sb0 + min(it, n_steps - 1); };
    WStage8<T> wa, wb;
#pragma unroll
    for (int d = 0; d < DX; ++d) x_issue(d, sbc(d));
    wa.template load<TR>(wr, rowtile(sbc(0)), tid);
    wb.template load<TR>(wr, rowtile(sbc(1)), tid);
    wa.template store<TR>(lds, rowtile(sbc(0)), tid);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    // step it: X(it+DX) DMA and W(it+2) loads into `ld` (the set that held it), MFMAs of it,
    // decode of W(it+1) from `st` into its stage, wait for X(it+1), one barrier
    auto step = [&](int it, WStage8<T> &ld, WStage8<T> &st) {
        if constexpr (!(MMQ8_EXP & 16)) x_issue(it + DX, sbc(it + DX));
        if constexpr (!(MMQ8_EXP & 4)) ld.template load<TR>(wr, rowtile(sbc(it + 2)), tid);
        const uint8_t *Xc = Xs + (it % N_XS) * NI * XB;
        if constexpr (MMQ8_EXP & 8) {
        } else if constexpr (TT == 64)
            q8_sb_compute<T, 1, TR>(lds + (it & 1) * WB, Xc, kg, rg, tg, lane, acc0, acc1);
        else
            q8_sb_compute<T, 2, TR>(lds + (it & 1) * WB, Xc + (tg >> 1) * XB, 0, rg, tg & 1, lane, acc0, acc1);
        if constexpr (!(MMQ8_EXP & 2)) st.template store<TR>(lds + ((it + 1) & 1) * WB, rowtile(sbc(it + 1)), tid);
        // X(it+1) must have landed: younger than it are this step's W(it+2) loads and (DX = 2)
        // this step's X(it+2) pieces
        if constexpr (DX == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WStage8<T>::VMEM + NXV) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WStage8<T>::VMEM) : "memory");
        lds_barrier();
    };
    for (int it = 0; it < n_steps; it += 2) {
        step(it, wa, wb);
        if (it + 1 < n_steps) step(it + 1, wb, wa);
    }
    // the clamped prefetches of the last steps land before the workgroup can leave
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // K-group reduction through LDS (the stages are free after the loop's last barrier)
    if constexpr (NKG == 2) {
        float *red = reinterpret_cast<float *>(lds);
        const int wl = wave % (NW / 2);
        if (kg == 1) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                red[((wl * 2 + 0) * 16 + i) * 64 + lane] = acc0[i];
                red[((wl * 2 + 1) * 16 + i) * 64 + lane] = acc1[i];
            }
        }
        lds_barrier();
        if (kg == 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                acc0[i] += red[((wl * 2 + 0) * 16 + i) * 64 + lane];
                acc1[i] += red[((wl * 2 + 1) * 16 + i) * 64 + lane];
            }
        }
    }
    const bool out_wave = NKG == 1 || kg == 0;   // the waves holding the sums
    if constexpr (SK) {
        // a tile shared by two workgroups: each stores its partial write-through (sc1, one
        // 256-B wave row per register), drains, and one lane adds to the tile's counter (agent
        // scope); the workgroup whose add returns 1 came second: it loads the other partial with
        // sc1 loads, adds it (two operands: the same sum in either order) and stores dst; it
        // also re-arms the counter (MI355X_MICROARCH.md inter-workgroup visibility, first form).
        // Ordering: the compiler cannot move the partial loads above the counter add, because
        // lds_barrier() is an asm statement with a "memory" clobber between them (and the loads
        // sit behind the branch on the add's result); on the hardware, sc1 stores drained by
        // vmcnt(0) before the add and sc1 loads after it are the guide's measured valid form. An
        // acquire-release add would instead cost an L2 write-back and an L1 invalidate (~1.7 us)
        // per tile.
        const int n_sb2 = (a.K + Q8_QK - 1) / Q8_QK;
        if (sb0 != 0 || sb1 != n_sb2) {
            const int tile = rt * n_tt + tt;
            const int me = sb0 == 0 ? 0 : 1;
            constexpr int OW = NW / NKG;           // output waves
            const int ow = NKG == 1 ? wave : wave % OW;
            auto slot = [&](int who) {
                return reinterpret_cast<uint32_t *>(sk.part) + (((int64_t)tile * 2 + who) * OW + ow) * 32 * 64;
            };
            if (out_wave) {
                // (f32 values, no bit_cast: ROCm 7.2's clang lowers __builtin_bit_cast of an
                // ext_vector element, acc0[i], to element 0 for every i, or to an undefined value:
                // scripts/bitcast_vec_elem.hip)
                float *mine = reinterpret_cast<float *>(slot(me));
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float v0 = acc0[i], v1 = acc1[i];
                    __hip_atomic_store(mine + i * 64 + lane, v0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(mine + (16 + i) * 64 + lane, v1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
            __shared__ int sk_order;
            lds_barrier();
            if (threadIdx.x == 0)
                sk_order = __hip_atomic_fetch_add(sk.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lds_barrier();
            if (sk_order == 0) return;             // (uniform) the other half finishes the tile
            if (out_wave) {
                const float *other = reinterpret_cast<const float *>(slot(me ^ 1));
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    acc0[i] += __hip_atomic_load(other + i * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    acc1[i] += __hip_atomic_load(other + (16 + i) * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (threadIdx.x == 0) __hip_atomic_store(sk.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (!out_wave) return;
    const int r = lane & 31, hl = lane >> 5;
    const int tok0 = tt * TT + 32 * tg + 4 * hl;
    const int rowA = rt * TR + 64 * rg + r, rowB = rowA + 32;
    uint8_t *dbase;
    int64_t ldd;
    const bool atomic = !SK && (xcd_remap & 4) != 0;   // 2-way split-K: both halves add into dst (zeroed)
    if (!SK && ksplit > 1 && !atomic) {   // part[ks][slice][token][row]
        dbase = reinterpret_cast<uint8_t *>(part + ((int64_t)ks * gridDim.y + slice) * a.M * a.N);
        ldd = (int64_t)a.N * 4;
    } else {
        dbase = a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3;
        ldd = a.nb1;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int tok = tok0 + 8 * (i >> 2) + (i & 3);
        if (tok < n_tok) {
            float *drow;
            if constexpr (MOE) {   // scatter to dst[slot][token] of the pair
                const int pair = moe.pos_pair[q0 + tok];
                drow = reinterpret_cast<float *>(a.dst + (int64_t)(pair % moe.n_used) * a.nb1 +
                                                 (int64_t)(pair / moe.n_used) * a.nb2);
            } else {
                drow = reinterpret_cast<float *>(dbase + (int64_t)tok * ldd);
            }
            if (atomic) {   // 0 + a + b == 0 + b + a: deterministic for exactly two halves
                if (rowA < a.N) unsafeAtomicAdd(drow + rowA, acc0[i]);
                if (rowB < a.N) unsafeAtomicAdd(drow + rowB, acc1[i]);
                continue;
            }
            if (rowA < a.N) drow[rowA] = acc0[i];
            if (rowB < a.N) drow[rowB] = acc1[i];
        }
    }
}

// grid.x = n_rt * ksplit * n_tt (token tiles fastest; XCD-remapped when a multiple of 8),
// grid.y = slices. TR weight rows x TT tokens per workgroup, TR / 16 waves of 64 rows x 32
// tokens:
//   TT = 64:  two K-groups of waves split every super-block (blocks 0-3 / 4-7), reduced through
//             LDS at the end;
//   TT = 128: every wave takes whole super-blocks (the weight stage serves twice the tokens).
//   TR = 64 halves the workgroup (4 waves, ~70 KB of LDS) so that two run on one CU and their
//   load / compute phases interleave.
// SK (stream-K, the reference's CDNA decomposition, src/ggml-cuda/mmq.cu:115 / mmq.cuh:3374):
// grid.x workgroups split the (tile, super-block) units evenly, a tile's two halves meet
// through a write-through partial and a counter (mmq8_job).
template <int T, int TT, int TR, bool MOE = false, bool SK = false>
__global__ __launch_bounds__(4 * TR) void mmq8_kernel(const MmArgs a, const uint8_t *__restrict__ ximg, int n_tt,
                                                      int ksplit, int sb_per, uint32_t w_extent,
                                                      float *__restrict__ part, int xcd_remap, const Moe8 moe,
                                                      const StreamK sk) {
    constexpr int WB = wi_bytes<TR>();
    constexpr int XB = ximg_bytes<T>();
    constexpr int NI = TT / Q8_TOK;                // activation images per stage
    constexpr int N_XS = (TT == 64 && TR == 128) ? 3 : 2;   // activation stage ring
    // LDS: two weight stages (decoded one super-block ahead from registers loaded two ahead) and
    // the activation ring (LDS-DMA DX super-blocks ahead)
    __shared__ __align__(16) uint8_t lds[2 * WB + N_XS * NI * XB];
    const int n_sb = (a.K + Q8_QK - 1) / Q8_QK;
    int v = blockIdx.x;
    if (xcd_remap & 1) v = (v & 7) * (int)(gridDim.x >> 3) + (v >> 3);
    const int slice = blockIdx.y;   // MOE: the token tile
    if constexpr (SK) {
        // stream-K: this workgroup's share [u0, u1) of the (tile, super-block) units, tiles in
        // (row tile, token tile) order, token tiles fastest (neighbours share weights and, after
        // the XCD remap, an L2); at most two workgroups share a tile (host: units per workgroup
        // >= super-blocks per tile)
        const int64_t U = (int64_t)sk.n_tiles * n_sb;
        const int u0 = (int)((int64_t)v * U / gridDim.x), u1 = (int)((int64_t)(v + 1) * U / gridDim.x);
        for (int u = u0; u < u1;) {
            const int tile = u / n_sb, k0 = u - tile * n_sb, k1 = min(n_sb, k0 + (u1 - u));
            mmq8_job<T, TT, TR, MOE, SK>(a, ximg, n_tt, w_extent, part, xcd_remap, moe, sk, lds, tile / n_tt, tile % n_tt,
                                         k0, k1, 1, 0, slice);
            u += k1 - k0;
            lds_barrier();   // (the next job's stages overwrite the reduction / stage LDS)
        }
        return;
    }
    const int tt = v % n_tt;
    v /= n_tt;
    const int ks = v % ksplit, rt = v / ksplit;
    const int sb0 = ks * sb_per, sb1 = min(n_sb, sb0 + sb_per);
    mmq8_job<T, TT, TR, MOE, SK>(a, ximg, n_tt, w_extent, part, xcd_remap, moe, sk, lds, rt, tt, sb0, sb1, ksplit, ks, slice);
}

// dst[slice][token][row] = sum over s of part[s][slice][token][row], in s order
__global__ __launch_bounds__(256) void mmq8_split_reduce(const MmArgs a, const float *__restrict__ part, int ksplit,
                                                         int slices) {
    const int64_t per_slice = (int64_t)a.M * a.N;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= per_slice * slices) return;
    const int slice = (int)(i / per_slice);
    const int64_t rem = i % per_slice;
    const int tok = (int)(rem / a.N), row = (int)(rem % a.N);
    float v = 0.f;
    for (int s = 0; s < ksplit; ++s) v += part[((int64_t)s * slices + slice) * per_slice + rem];
    const int i12 = slice % a.ne12, i13 = slice / a.ne12;
    reinterpret_cast<float *>(a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3 + (int64_t)tok * a.nb1)[row] = v;
}

// ==========================================================================================
// Repacked weights (the optional repacked weight layout): the int8 tile's B
// operands stored once in MFMA-fragment order, so the tile kernel moves them into LDS by
// LDS-DMA, 1 KiB per wave instruction, with no VGPR round trip, no decode and no realignment.
// (Reference analogue: the CPU backend's repack extra buffer type, src/ggml-cpu/repack.cpp:1967,
// which re-lays Q4_0 / Q4_K blocks for its SIMD kernels at set_tensor time.)
//   codes [mat][rt32][sb][blk 8][1 KiB]  the int8 codes of 32 rows x one 32-block, in the order a
//         v_mfma_i32_32x32x32_i8 B operand reads them: lane l holds row l&31, k 16(l>>5)..+15 at
//         bytes 16l..16l+15. Q6_K: two 512-B v_mfma_i32_32x32x16_i8 operands per block, group g
//         of 16 k: lane l holds row l&31, k 16g+8(l>>5)..+7 at bytes 512g+8l..
//         Codes: Q4_0 q-8, Q8_0 q, Q4_K q, Q5_K q | qh<<4, Q6_K q-32.
//   meta  [mat][rt32][sb][row 32][K-half 2][16 B]  what one lane needs for its row and its half
//         (blocks 4h..4h+3) of a super-block, in one 16-B load:
//           Q4_0 / Q8_0: f32 d of the four blocks;
//           Q4_K / Q5_K: f32 d, f32 dmin, u8 sc[4], u8 m[4] (get_scale_min_k4, ggml-quants.c:703-710);
//           Q6_K:        f32 d, i8 sc[8] (the 16-groups of the four blocks), 4 B zero.
// Rows are padded to 32 and K to whole super-blocks with zero codes and zero scales, so the tile
// kernel never tests a bound inside its loop.
// ==========================================================================================
template <int T> constexpr bool rp_has_mins() { return T == T_Q4_K || T == T_Q5_K; }

struct RpArgs {
    const uint8_t *codes;
    const uint8_t *meta;
    int n_rt, n_sb;          // 32-row tiles and super-blocks per matrix
    int ne02;                // matrix index = i03 * ne02 + i02
};

struct RpSrc {               // the ggml tensor being repacked
    const uint8_t *w;
    int64_t nb01, nb02, nb03;
    int K, N, ne02, n_mat;
};

__device__ __forceinline__ uint32_t ld_u16(const uint8_t *p) { return *reinterpret_cast<const uint16_t *>(p); }
// 4 bytes at a 2-byte-aligned address
__device__ __forceinline__ uint32_t ld_u32a2(const uint8_t *p) { return ld_u16(p) | (ld_u16(p + 2) << 16); }

// one thread per (matrix, row, 32-block), the row fastest: consecutive threads write consecutive
// 16-B pieces of one fragment; the thread of a K-half's first block writes that half's meta
template <int T>
__global__ __launch_bounds__(256) void repack_kernel(const RpSrc s, const RpArgs r) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int rr = (int)(t & 31);
    int64_t q = t >> 5;
    const int blk = (int)(q & 7);
    q >>= 3;
    const int sb = (int)(q % r.n_sb);
    q /= r.n_sb;
    const int rt = (int)(q % r.n_rt);
    const int mat = (int)(q / r.n_rt);
    if (mat >= s.n_mat) return;
    const int row = rt * 32 + rr, b = sb * 8 + blk;   // 32-block index in the row
    const bool live = row < s.N && b * 32 < s.K;
    const uint8_t *wrow = s.w + (int64_t)(mat % s.ne02) * s.nb02 + (int64_t)(mat / s.ne02) * s.nb03 + (int64_t)row * s.nb01;
    uint32_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};        // 32 codes, little-endian bytes
    u32x4v meta = u32x4v{0u, 0u, 0u, 0u};           // (the K-half's, written by blk % 4 == 0)
    float d = 0.f;                                  // Q4_0 / Q8_0 block scale
    if (live) {
        if constexpr (T == T_Q8_0) {
            const uint8_t *p = wrow + (int64_t)b * 34;
            d = h2f((uint16_t)ld_u16(p));
#pragma unroll
            for (int i = 0; i < 8; ++i) c[i] = ld_u32a2(p + 2 + 4 * i);
        } else if constexpr (T == T_Q4_0) {
            const uint8_t *p = wrow + (int64_t)b * 18;
            d = h2f((uint16_t)ld_u16(p));
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t n = ld_u32a2(p + 2 + 4 * i);
                c[i] = sub8_bytes(n & 0x0F0F0F0Fu);            // k 4i..4i+3
                c[4 + i] = sub8_bytes((n >> 4) & 0x0F0F0F0Fu); // k 16+4i..
            }
        } else if constexpr (T == T_Q4_K || T == T_Q5_K) {
            constexpr int BB = T == T_Q4_K ? 144 : 176, QS = T == T_Q4_K ? 16 : 48;
            const uint8_t *p = wrow + (int64_t)sb * BB;      // 16-B aligned rows (checked on the host)
            const int cc = blk >> 1, hi = blk & 1;           // 64-chunk, nibble
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t n = *reinterpret_cast<const uint32_t *>(p + QS + 32 * cc + 4 * i);
                uint32_t v = hi ? (n >> 4) & 0x0F0F0F0Fu : n & 0x0F0F0F0Fu;
                if constexpr (T == T_Q5_K) {
                    const uint32_t h = *reinterpret_cast<const uint32_t *>(p + 16 + 4 * i);
                    v |= ((h >> blk) & 0x01010101u) << 4;
                }
                c[i] = v;
            }
            if ((blk & 3) == 0) {   // get_scale_min_k4 (src/ggml-quants.c:703-710) for blocks blk..blk+3
                const uint32_t h0 = *reinterpret_cast<const uint32_t *>(p);
                const uint8_t *scs = p + 4;
                uint32_t sc = 0, m = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int jj = blk + j;
                    const uint32_t scv = jj < 4 ? scs[jj] & 63 : (scs[jj + 4] & 0xF) | ((scs[jj - 4] >> 6) << 4);
                    const uint32_t mv = jj < 4 ? scs[jj + 4] & 63 : (scs[jj + 4] >> 4) | ((scs[jj] >> 6) << 4);
                    sc |= scv << (8 * j);
                    m |= mv << (8 * j);
                }
                meta = u32x4v{fu(h2f((uint16_t)(h0 & 0xffffu))), fu(h2f((uint16_t)(h0 >> 16))), sc, m};
            }
        } else {   // Q6_K: 32-block blk = 4h + k of the super-block (dequantize_row_q6_K, src/ggml-quants.c:1762-1791)
            const uint8_t *p = wrow + (int64_t)sb * 210;     // 2-byte aligned
            const int h = blk >> 2, k = blk & 3;
            const uint8_t *ql = p + 64 * h + (k & 1) * 32, *qh = p + 128 + 32 * h;
            const int sh = 2 * k;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t l = ld_u32a2(ql + 4 * i), hb = ld_u32a2(qh + 4 * i);
                const uint32_t lo = (k >> 1) ? (l >> 4) & 0x0F0F0F0Fu : l & 0x0F0F0F0Fu;
                c[i] = sub32_bytes(lo | (((hb >> sh) & 0x03030303u) << 4));
            }
            if (k == 0) {   // groups of blocks 4h..4h+3: scale of block 4h + k, group g is sc[8h + g + 2k]
                const float dd = h2f((uint16_t)ld_u16(p + 208));
                uint32_t s0 = 0, s1 = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    s0 |= (uint32_t)p[192 + 8 * h + j] << (8 * j);
                    s1 |= (uint32_t)p[192 + 8 * h + 4 + j] << (8 * j);
                }
                meta = u32x4v{fu(dd), s0, s1, 0u};   // sc bytes in (block, group) order = 2k + g
            }
        }
    }
    const int64_t tile = ((int64_t)mat * r.n_rt + rt) * r.n_sb + sb;
    uint8_t *cb = const_cast<uint8_t *>(r.codes) + (tile * 8 + blk) * 1024;
    uint8_t *mb = const_cast<uint8_t *>(r.meta) + ((tile * 32 + rr) * 2 + (blk >> 2)) * 16;
    if constexpr (T == T_Q6_K) {   // group g = k/16, k-half kg = (k/8)&1: 8 B at 512g + 256kg + 8rr
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int kg = 0; kg < 2; ++kg)
                *reinterpret_cast<u32x2v *>(cb + 512 * g + 256 * kg + 8 * rr) = u32x2v{c[4 * g + 2 * kg], c[4 * g + 2 * kg + 1]};
    } else {
        st128(cb + 16 * rr, u32x4v{c[0], c[1], c[2], c[3]});
        st128(cb + 512 + 16 * rr, u32x4v{c[4], c[5], c[6], c[7]});
    }
    if constexpr (T == T_Q4_0 || T == T_Q8_0) *reinterpret_cast<float *>(mb + 4 * (blk & 3)) = d;
    else if ((blk & 3) == 0) st128(mb, meta);
}

// ------------------------------------------------------------------------------------------
// the tile kernel on repacked weights: 128 rows x 64 tokens per workgroup, 8 waves in two roles,
// one of each per SIMD (a workgroup's waves 0-3 land on four different SIMDs, and so do 4-7):
//   consumers (waves 0-3): a wave owns 32 rows x 64 tokens over the whole super-block, i.e. two
//     32x32 MFMA tiles sharing the weight (B) fragment, 16 MFMAs + their scale epilogue per step;
//     it also loads its rows' meta (16 B per K-half) into a 3-deep register ring;
//   producers (waves 4-7): move the next steps' operands into a 3-slot LDS ring by LDS-DMA, two
//     steps ahead (row group p's 8 KiB of weight fragments, a quarter of the activation image),
//     and wait for the next step's pieces before each barrier.
// One s_barrier per step orders the ring (a slot is refilled one step after its last read). With
// the roles split, one wave of each SIMD issues the DMA (its issue cost, ~100+ cycles per 1 KiB
// piece, is the partner's VALU / MFMA time) while the other computes: a step costs the larger of
// the two instead of their sum (measured decomposition: scripts/mmq8r_exp.sh).
// Scale arithmetic as mmq8_kernel:
//   Q4_0 / Q8_0: the MFMA's C input 0x4B400000 makes the int32 result the f32 12582912 + R, one
//     fma per output and block applies d; -12582912 * sum(d) starts the sums;
//   K-quants: exact int32 sums p_i += sc * R (v_mad_i32_i24), then d * p_i, and for Q4_K / Q5_K
//     minus dmin * sum_j m_j * bsum_j as one f16 MFMA per tile and K-half on exact integers;
// then acc += dx[token] * p per super-block.
// ------------------------------------------------------------------------------------------
constexpr int RP_WB = 32768;   // weight bytes of one ring slot: 4 row groups x 8 blocks x 1 KiB

template <int T> constexpr int rp_slot_bytes() { return RP_WB + ximg_bytes<T>(); }
// vector-memory instructions of one producer wave per step (identical in every producer)
// step order: DMA of it+2, touch of it+2+RP_TOUCH; before the barrier the DMA of it+1 must have
// landed, younger than it: the touch of it+1+RP_TOUCH, the DMA of it+2 and its touch
template <int T> constexpr int rp_prod_wait() { return 8 + q8_x_vmem<T, 4>() + (RP_TOUCH > 0 ? 4 : 0); }

template <int T>
__global__ __launch_bounds__(512) void mmq8r_kernel(const MmArgs a, const RpArgs r, const uint8_t *__restrict__ ximg,
                                                    int n_tt, int ksplit, int sb_per, float *__restrict__ part, int flags) {
    constexpr int XB = ximg_bytes<T>();
    constexpr int SLOT = rp_slot_bytes<T>();
    constexpr bool F32S = T == T_Q4_0 || T == T_Q8_0;   // float block scales (else integer sub-block scales)
    __shared__ __align__(16) uint8_t lds[3 * SLOT];
    const int n_sb = r.n_sb;
    int v = blockIdx.x;
    if (flags & 1) v = (v & 7) * (int)(gridDim.x >> 3) + (v >> 3);
    const int tt = v % n_tt;
    v /= n_tt;
    const int ks = v % ksplit, rt128 = v / ksplit;
    const int sb0 = ks * sb_per, sb1 = min(n_sb, sb0 + sb_per);
    const int n_steps = sb1 - sb0;
    if (n_steps <= 0) return;   // (uniform)
    const int slice = blockIdx.y;
    const int i12 = slice % a.ne12, i13 = slice / a.ne12;
    const int mat = (i13 / a.r3) * r.ne02 + (i12 / a.r2);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool producer = wave >= 4;
    const int rg = wave & 3;              // consumer: its row group; producer: its share
    const int rr = lane & 31, hl = lane >> 5;
    const int64_t mat_tiles = (int64_t)mat * r.n_rt;
    const int my_rt = min(4 * rt128 + rg, r.n_rt - 1);   // (rows past N: the last tile, never stored)
    // super-block of step it (steps past the end: a valid super-block again, a dead prefetch)
    const int rot = (RP_ROT_R * rt128 + RP_ROT_T * tt) % n_steps;
    auto sbc = [&](int it) { return sb0 + (rot + it) % n_steps; };

    if (producer) {
        // ---------------- producer: DMA two steps ahead, one barrier per step ----------------
        const uint32_t codes_bytes = (uint32_t)r.n_rt * (uint32_t)n_sb * 8192u;
        const __amdgpu_buffer_rsrc_t wr =
            __builtin_amdgcn_make_buffer_rsrc((void *)(r.codes + mat_tiles * n_sb * 8192), 0, codes_bytes, Q8_RSRC_W3);
        const uint8_t *xbase = ximg + ((int64_t)slice * n_tt + tt) * n_sb * XB;
        const __amdgpu_buffer_rsrc_t xr =
            __builtin_amdgcn_make_buffer_rsrc((void *)xbase, 0, (uint32_t)(n_sb * XB), Q8_RSRC_W3);
        const uint32_t wbase = (uint32_t)my_rt * (uint32_t)n_sb * 8192u + (uint32_t)lane * 16u;
        // touch of super-block sb: lane i loads one dword of line i of this wave's 8 KiB of weights
        // and of line i of its quarter of the activation image (the results are never read)
        const uint32_t xq = (uint32_t)((XB + 511) / 512) * 128u;   // a quarter of the image, 128-B lines
        auto touch = [&](int sb) {
            if constexpr (RP_TOUCH > 0) {
                uint32_t t0 = bl32(wr, wbase - (uint32_t)lane * 16u + (uint32_t)sb * 8192u + (uint32_t)lane * 128u);
                uint32_t t1 = bl32(xr, (uint32_t)(sb * XB) + min((uint32_t)rg * xq + (uint32_t)lane * 128u, (uint32_t)XB - 4u));
                asm volatile("" ::"v"(t0), "v"(t1));   // keep the loads; nothing waits for them but the counted vmcnt
            }
        };
        auto issue = [&](int slot, int sb) {
            uint8_t *dst = lds + slot * SLOT;
            if constexpr (!(MMQ8R_EXP & 1)) {
#pragma unroll
                for (int i = 0; i < 8; ++i) q8_dma16(wr, dst + (rg * 8 + i) * 1024, wbase + (uint32_t)sb * 8192u + i * 1024u);
            }
            if constexpr (!(MMQ8R_EXP & 2)) q8_x_dma<T, 4>(xr, (uint32_t)(sb * XB), dst + RP_WB, rg, lane);
        };
        // per step: DMA of it+2 then the touch of it+2+RP_TOUCH (counted in rp_prod_wait)
        for (int d = 2; d < RP_TOUCH; ++d) touch(sbc(d));   // (uncounted: issued before everything below)
        issue(0, sbc(0));
        touch(sbc(RP_TOUCH));
        issue(1, sbc(1));
        touch(sbc(RP_TOUCH + 1));
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(rp_prod_wait<T>()) : "memory");   // step 0 landed
        lds_barrier();
        for (int it = 0; it < n_steps; ++it) {
            issue((it + 2) % 3, sbc(it + 2));
            touch(sbc(it + 2 + RP_TOUCH));
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(rp_prod_wait<T>()) : "memory");   // step it+1 landed
            lds_barrier();
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the clamped prefetches land before the exit
        return;
    }

    // ---------------- consumer ----------------
    const uint8_t *mrow = r.meta + ((mat_tiles + my_rt) * n_sb * 32 + rr) * 32;
    struct Meta { u32x4v h[2]; };   // this lane's row: K-half 0 and 1 of one super-block
    auto load_meta = [&](int sb, Meta &g) {
        const u32x4v *p = reinterpret_cast<const u32x4v *>(mrow + (int64_t)sb * 32 * 32);
        g.h[0] = p[0];
        g.h[1] = p[1];
    };

    f32x16 acc0, acc1;
    i32x16 cin;   // MFMA C input: the magic constant (float scales) or zero (integer scales)
#pragma unroll
    for (int i = 0; i < 16; ++i) { acc0[i] = 0.f; acc1[i] = 0.f; cin[i] = F32S ? (int)Q8_MAGIC_I : 0; }
    asm volatile("" : "+v"(cin));   // opaque: not rematerialized, so the pins after the MFMAs hold its registers

    auto compute = [&](int slot, const Meta &g) {
        if constexpr ((MMQ8R_EXP & 4) != 0) {
            asm volatile("" ::"v"(g.h[0]), "v"(g.h[1]));
            return;
        }
        const uint8_t *W = lds + slot * SLOT + rg * 8192;
        const uint8_t *X = lds + slot * SLOT + RP_WB;
        // step q: (block, group); A fragments of both token tiles and one B fragment, read from LDS
        // one step ahead of their MFMAs (one wave per SIMD computes: nothing else hides the latency)
        constexpr int NQ = T == T_Q6_K ? 16 : 8;
        struct Frag { u32x4v A0, A1, B; };
        auto load = [&](int q, Frag &f) {
            if constexpr (T == T_Q6_K) {
                const int blk = q >> 1, gq = q & 1;
                const uint8_t *xa = X + blk * 2048 + gq * 1024 + hl * 512 + rr * 8;
                const u32x2v a0 = ld64(xa), a1 = ld64(xa + 256), b = ld64(W + blk * 1024 + gq * 512 + lane * 8);
                f.A0 = u32x4v{a0[0], a0[1], 0u, 0u};
                f.A1 = u32x4v{a1[0], a1[1], 0u, 0u};
                f.B = u32x4v{b[0], b[1], 0u, 0u};
            } else {
                const uint8_t *xa = X + q * 2048 + hl * 1024 + rr * 16;
                f.A0 = ld128(xa);
                f.A1 = ld128(xa + 512);
                f.B = ld128(W + q * 1024 + lane * 16);
            }
        };
        auto mfma2 = [&](const Frag &f, i32x16 &R0, i32x16 &R1) {
            if constexpr (T == T_Q6_K) {
                const long A0 = as_l(u32x2v{f.A0[0], f.A0[1]}), A1 = as_l(u32x2v{f.A1[0], f.A1[1]});
                const long B = as_l(u32x2v{f.B[0], f.B[1]});
                R0 = __builtin_amdgcn_mfma_i32_32x32x16_i8(A0, B, cin, 0, 0, 0);
                R1 = __builtin_amdgcn_mfma_i32_32x32x16_i8(A1, B, cin, 0, 0, 0);
            } else {
                R0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(as_i4(f.A0), as_i4(f.B), cin, 0, 0, 0);
                R1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(as_i4(f.A1), as_i4(f.B), cin, 0, 0, 0);
            }
        };
        f32x16 p0, p1;
        i32x16 pi0, pi1;
        float c0 = 0.f;
        if constexpr (F32S)
            c0 = -Q8_MAGIC_F * (((uf(g.h[0][0]) + uf(g.h[0][1])) + (uf(g.h[0][2]) + uf(g.h[0][3]))) +
                                ((uf(g.h[1][0]) + uf(g.h[1][1])) + (uf(g.h[1][2]) + uf(g.h[1][3]))));
        auto consume = [&](int q, const i32x16 &R0, const i32x16 &R1) {
            if constexpr (F32S) {
                const float sq = uf(g.h[q >> 2][q & 3]);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    p0[i] = __builtin_fmaf(uf((uint32_t)R0[i]), sq, q == 0 ? c0 : p0[i]);
                    p1[i] = __builtin_fmaf(uf((uint32_t)R1[i]), sq, q == 0 ? c0 : p1[i]);
                }
                asm volatile("" : "+v"(p0), "+v"(p1));
            } else {
                // Q4_K / Q5_K: sc of block q (unsigned 6-bit) in byte q&3 of half q>>2's word 2;
                // Q6_K: sc of step q (signed) in byte q&3 of half q>>3's words 1..2
                int sc;
                if constexpr (T == T_Q6_K) sc = (int)(int8_t)(uint8_t)(g.h[q >> 3][1 + ((q >> 2) & 1)] >> (8 * (q & 3)));
                else sc = (int)((g.h[q >> 2][2] >> (8 * (q & 3))) & 0xffu);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    pi0[i] = q == 0 ? __mul24(R0[i], sc) : pi0[i] + __mul24(R0[i], sc);
                    pi1[i] = q == 0 ? __mul24(R1[i], sc) : pi1[i] + __mul24(R1[i], sc);
                }
                asm volatile("" : "+v"(pi0), "+v"(pi1));
            }
        };
        i32x16 Ra0, Ra1, Rb0, Rb1;
        u32x4v dxv[8];
        Frag fa, fb;
        load(0, fa);
        load(1, fb);
        mfma2(fa, Ra0, Ra1);
        load(2, fa);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 1; q < NQ; ++q) {
            // fragments of q are in (q & 1 ? fb : fa); those of q+1 go into the other set after
            // the MFMAs of q have read theirs
            if (q & 1) mfma2(fb, Rb0, Rb1);
            else mfma2(fa, Ra0, Ra1);
            if (q + 2 < NQ) {
                if (q & 1) load(q + 2, fb);
                else load(q + 2, fa);
            }
            if (q == NQ - 1) {   // tile 0's token scales: read now, used after the last epilogues
#pragma unroll
                for (int k = 0; k < 4; ++k) dxv[k] = ld128(X + XI_DX + 4 * (8 * k + 4 * hl));
            }
            if (q & 1) consume(q - 1, Ra0, Ra1);
            else consume(q - 1, Rb0, Rb1);
            __builtin_amdgcn_sched_barrier(0);
        }
        consume(NQ - 1, Rb0, Rb1);
        asm volatile("" ::"v"(cin));   // C-input registers stay allocated past the last MFMA (see q8_sb_compute)
#pragma unroll
        for (int k = 0; k < 4; ++k) dxv[4 + k] = ld128(X + XI_DX + 4 * (32 + 8 * k + 4 * hl));   // tile 1's
        if constexpr (!F32S) {
            // one d per super-block (both halves carry it)
            const float dd = uf(g.h[0][0]);
#pragma unroll
            for (int i = 0; i < 16; ++i) { p0[i] = dd * (float)pi0[i]; p1[i] = dd * (float)pi1[i]; }
        }
        if constexpr (rp_has_mins<T>()) {
            // sum over sub-blocks j of m_j * bsum_j, per K-half kh: k16-sums 8kh..8kh+7 of the image
            // (half kh of its bsums), lane k-group (l>>5) takes four of them; m_j for k16-sum e is
            // m_(e>>1). Exact integers in f16, f32 sums.
            typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
            f32x16 zf;
#pragma unroll
            for (int i = 0; i < 16; ++i) zf[i] = 0.f;
#pragma unroll
            for (int kh = 0; kh < 2; ++kh) {
                const u32x2v bs0 = ld64(X + XI_BS + kh * 1024 + rr * 16 + hl * 8);
                const u32x2v bs1 = ld64(X + XI_BS + kh * 1024 + (32 + rr) * 16 + hl * 8);
                const uint32_t mw = g.h[kh][3];
                const uint32_t m0 = (mw >> (16 * hl)) & 0xffu, m1 = (mw >> (16 * hl + 8)) & 0xffu;
                const uint32_t h0 = __builtin_bit_cast(uint16_t, (_Float16)(float)m0);
                const uint32_t h1 = __builtin_bit_cast(uint16_t, (_Float16)(float)m1);
                const f16x4 Bm = __builtin_bit_cast(f16x4, u32x2v{h0 | (h0 << 16), h1 | (h1 << 16)});
                const f32x16 mn0 = __builtin_amdgcn_mfma_f32_32x32x8f16(__builtin_bit_cast(f16x4, bs0), Bm, zf, 0, 0, 0);
                const f32x16 mn1 = __builtin_amdgcn_mfma_f32_32x32x8f16(__builtin_bit_cast(f16x4, bs1), Bm, zf, 0, 0, 0);
                const float ndmin = -uf(g.h[0][1]);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    p0[i] = __builtin_fmaf(ndmin, mn0[i], p0[i]);
                    p1[i] = __builtin_fmaf(ndmin, mn1[i], p1[i]);
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                acc0[4 * q + c] = __builtin_fmaf(p0[4 * q + c], uf(dxv[q][c]), acc0[4 * q + c]);
                acc1[4 * q + c] = __builtin_fmaf(p1[4 * q + c], uf(dxv[4 + q][c]), acc1[4 * q + c]);
            }
        }
    };

    // this lane's meta of step it+1 is loaded while step it computes (a 2-deep register ring)
    Meta g0, g1;
    load_meta(sbc(0), g0);
    lds_barrier();   // (the producers' step-0 barrier)
    auto step = [&](int it, int slot, const Meta &gc, Meta &gi) {
        load_meta(sbc(it + 1), gi);
        compute(slot, gc);
        lds_barrier();
    };
    // (slots rotate by 3, the meta ring by 2: unrolled by 6)
    for (int it = 0; it < n_steps; it += 6) {
        step(it, 0, g0, g1);
        if (it + 1 < n_steps) step(it + 1, 1, g1, g0);
        if (it + 2 < n_steps) step(it + 2, 2, g0, g1);
        if (it + 3 < n_steps) step(it + 3, 0, g1, g0);
        if (it + 4 < n_steps) step(it + 4, 1, g0, g1);
        if (it + 5 < n_steps) step(it + 5, 2, g1, g0);
    }

    const int row = rt128 * 128 + rg * 32 + rr;
    if (row >= a.N) return;
    const bool atomic = (flags & 4) != 0;
    uint8_t *dbase;
    int64_t ldd;
    if (ksplit > 1 && !atomic) {
        dbase = reinterpret_cast<uint8_t *>(part + ((int64_t)ks * gridDim.y + slice) * a.M * a.N);
        ldd = (int64_t)a.N * 4;
    } else {
        dbase = a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3;
        ldd = a.nb1;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int tok = tt * 64 + 32 * t + 8 * (i >> 2) + 4 * hl + (i & 3);
            if (tok < a.M) {
                float *drow = reinterpret_cast<float *>(dbase + (int64_t)tok * ldd);
                const float val = t ? acc1[i] : acc0[i];
                if (atomic) unsafeAtomicAdd(drow + row, val);
                else drow[row] = val;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
static int ximg_bytes_rt(int type) {
    switch (type) {
        case T_Q4_K: case T_Q5_K: return ximg_bytes<T_Q4_K>();
        default: return ximg_bytes<T_Q8_0>();
    }
}

// Every K the block size divides (Q4_0 / Q8_0: a partial last super-block, its missing blocks
// with zero activation codes and zero weight scales) and every 2-byte-aligned layout of Q4_0 /
// Q8_0 / Q6_K (windows realigned per lane from the block's own offset, the buffer based at the
// matrix's dword floor). Q4_K / Q5_K rows are 144 / 176 B, so their super-blocks are 16-B aligned
// whenever the tensor is; a K-quant view at a finer offset takes the mat-vec.
bool mmq8_images_fit(int type, const MmArgs &a);
bool mmq8_supported(int type, const MmArgs &a) {
    if (!(type == T_Q4_0 || type == T_Q8_0 || type == T_Q4_K || type == T_Q5_K || type == T_Q6_K)) return false;
    if (a.K <= 0 || a.K % type_blck(type) != 0 || a.M <= 0) return false;
    const uintptr_t al = (type == T_Q4_K || type == T_Q5_K) ? 15 : 1;
    // (the matrix strides matter only where there is more than one matrix)
    const bool many2 = a.ne12 / a.r2 > 1, many3 = a.ne13 / a.r3 > 1;
    if ((reinterpret_cast<uintptr_t>(a.w) & al) || (a.nb01 & al) || (many2 && (a.nb02 & al)) || (many3 && (a.nb03 & al)))
        return false;
    const int64_t row_b = (int64_t)a.K / type_blck(type) * type_bytes(type);
    const int64_t n_sb = (a.K + Q8_QK - 1) / Q8_QK;
    // the last super-block's windows reach past a short row by up to one super-block
    const int64_t w_span = (int64_t)a.N * a.nb01 + n_sb * Q8_QK / type_blck(type) * type_bytes(type) + 8;
    return a.nb01 >= row_b && w_span < (1LL << 32) && mmq8_images_fit(type, a);
}

// one slice's activation images stay below 2 GiB (32-bit buffer offsets), counted for the
// 128-token tile, which allocates two 64-token images per tile (ceil(M / 128) * 2 >= ceil(M / 64));
// the repacked tile's images are the same
bool mmq8_images_fit(int type, const MmArgs &a) {
    const int64_t n_sb = (a.K + Q8_QK - 1) / Q8_QK;
    const int64_t n_img = (a.M + 127) / 128 * 2;
    return n_img * n_sb * ximg_bytes_rt(type) < (1LL << 31);
}

template <int T>
static void launch8(const MmArgs &a, uint8_t *ximg, int tr_rows, int tt_tok, int n_tt, int slices, int ksplit,
                    int sb_per, float *part, bool atomic, const StreamK &sk, hipStream_t st) {
    const int n_sb = (a.K + Q8_QK - 1) / Q8_QK;
    const int n_img = n_tt * (tt_tok / Q8_TOK);   // 64-token images per slice (tokens past M: zeros)
    hipLaunchKernelGGL(mmq8_quant_x<T>, dim3((unsigned)(n_img * (Q8_TOK / 4) * n_sb), slices), dim3(256), 0, st, a, ximg,
                       n_img, n_sb, Moe8{}, atomic ? 1 : 0);
    const int64_t row_b = (int64_t)a.K / QT<T>::blck * QT<T>::bytes;
    const uint32_t w_extent = (uint32_t)((int64_t)(a.N - 1) * a.nb01 + row_b);   // (the kernel rounds it up)
    const int n_rt = (a.N + tr_rows - 1) / tr_rows;
    if (sk.cnt != nullptr) {   // stream-K: one workgroup per CU, the units split evenly
        const unsigned gx = MMQ8_SK_WGS;
        if (tt_tok == 128)
            hipLaunchKernelGGL((mmq8_kernel<T, 128, 128, false, true>), dim3(gx, 1), dim3(512), 0, st, a, (const uint8_t *)ximg,
                               n_tt, 1, n_sb, w_extent, part, 1, Moe8{}, sk);
        else
            hipLaunchKernelGGL((mmq8_kernel<T, 64, 128, false, true>), dim3(gx, 1), dim3(512), 0, st, a, (const uint8_t *)ximg,
                               n_tt, 1, n_sb, w_extent, part, 1, Moe8{}, sk);
        return;
    }
    const unsigned gx = (unsigned)(n_rt * ksplit * n_tt);
    const int remap = ((gx % 8 == 0) ? 1 : 0) | (atomic ? 4 : 0);
    const dim3 grid(gx, slices);
#define Q8_LAUNCH(TTv, TRv)                                                                                          \
    hipLaunchKernelGGL((mmq8_kernel<T, TTv, TRv>), grid, dim3(4 * TRv), 0, st, a, (const uint8_t *)ximg, n_tt, ksplit, \
                       sb_per, w_extent, part, remap, Moe8{}, StreamK{})
    if (tt_tok == 128) Q8_LAUNCH(128, 128);
    else if (tr_rows == 128) Q8_LAUNCH(64, 128);
    else Q8_LAUNCH(64, 64);   // measured slower than 128 rows at every shape; kept for A/B
#undef Q8_LAUNCH
    if (ksplit > 1 && !atomic) {
        const int64_t n = (int64_t)slices * a.M * a.N;
        hipLaunchKernelGGL(mmq8_split_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, (const float *)part,
                           ksplit, slices);
    }
}

// rows x tokens per workgroup of the in-place tile: 128-token tiles (the weight stage then serves
// twice the tokens) once more than 128 of them fill the chip without split-K: 4096 x 4096 x 576
// (160 tiles) 53 vs 67 us, x 768 54 vs 71, 4096 x 6144 x 512 54 vs 70, Q6_K 4096 x 4096 x 768
// 79 vs 101 (profiles/r04_mmq8_tt_sweep2.txt). At 128 tiles (4096 x 4096 x 512) the 128-token
// tile needs 2-way split-K and is slower: 44.9-45.1 vs 41.3 us (profiles/r03_mmq8_split2_atomic.txt)
int64_t mmq8_tiles128(const MmArgs &a) {
    return (int64_t)((a.N + 127) / 128) * ((a.M + 127) / 128) * a.ne12 * a.ne13;
}
int mmq8_tile_tokens(const MmArgs &a) { return mmq8_tiles128(a) > 128 ? 128 : 64; }

// the in-place tile's launch plan (pure: the launcher and the dispatch description share it)
struct Mmq8Plan {
    int tt_tok, tr_rows, n_rt, n_tt, ksplit, sb_per;
    int64_t tiles;
    bool atomic, use_sk;
};
static Mmq8Plan mmq8_plan(const MmArgs &a) {
    const Settings &S = settings();
    Mmq8Plan p{};
    const int slices = a.ne12 * a.ne13;
    const int n_sb = (a.K + Q8_QK - 1) / Q8_QK;
    // GGML_MI355X_MMQ8_TT / _TR override (measurements; 128 tokens always run 128 rows)
    p.tt_tok = mmq8_tile_tokens(a);
    if (S.mmq8_tt != 0) p.tt_tok = S.mmq8_tt == 128 ? 128 : 64;
    p.tr_rows = (S.mmq8_tr == 64 && p.tt_tok == 64) ? 64 : 128;
    p.n_rt = (a.N + p.tr_rows - 1) / p.tr_rows;
    p.n_tt = (a.M + p.tt_tok - 1) / p.tt_tok;
    // split-K over workgroups while the tile grid leaves CUs idle (>= 2 super-blocks per split)
    p.tiles = (int64_t)p.n_rt * p.n_tt * slices;
    int ksplit = 1;
    while (p.tiles * ksplit * 2 <= 256 && n_sb >= 4 * ksplit) ksplit *= 2;
    if (S.mmq8_ksplit > 0) ksplit = std::max(1, std::min(S.mmq8_ksplit, n_sb));
    p.sb_per = (n_sb + ksplit - 1) / ksplit;
    p.ksplit = (n_sb + p.sb_per - 1) / p.sb_per;
    // exactly two halves add into dst atomically (order-independent); more go through part[]
    p.atomic = p.ksplit == 2 && !S.mmq8_no_atomic;
    // stream-K (one slice, no split-K, 128-row tiles) where whole rounds of one tile per CU would
    // leave the last round mostly idle: e.g. 4096 x 11008 x 512, 344 128-token tiles = 1.34
    // rounds. A tile's units are then split between at most two workgroups (units per
    // workgroup >= super-blocks per tile, since tiles > workgroups). GGML_MI355X_MMQ8_SK: 0 never
    // (A/B), 1 whenever the tiles outnumber the workgroups
    const int64_t rounds = (p.tiles + MMQ8_SK_WGS - 1) / MMQ8_SK_WGS;
    const bool can_sk = slices == 1 && p.ksplit == 1 && p.tr_rows == 128 && p.tiles > MMQ8_SK_WGS && p.tiles <= Scratch::COUNTERS;
    p.use_sk = S.mmq8_sk >= 0 ? (S.mmq8_sk == 1 && can_sk) : (can_sk && (double)p.tiles / (double)(rounds * MMQ8_SK_WGS) < 0.85);
    return p;
}

std::string mmq8_plan_text(const MmArgs &a) {
    const Mmq8Plan p = mmq8_plan(a);
    return "mmq8 tile=" + std::to_string(p.tr_rows) + "x" + std::to_string(p.tt_tok) + " tiles=" + std::to_string(p.tiles) +
           " ksplit=" + std::to_string(p.ksplit) + (p.atomic ? " atomic" : "") + (p.use_sk ? " stream-k" : "");
}

hipError_t mmq8_launch(int type, const MmArgs &a, hipStream_t st, Scratch &scratch) {
    const int slices = a.ne12 * a.ne13;
    const int n_sb = (a.K + Q8_QK - 1) / Q8_QK;
    const Mmq8Plan pl = mmq8_plan(a);
    const int tt_tok = pl.tt_tok, tr_rows = pl.tr_rows, n_tt = pl.n_tt, ksplit = pl.ksplit, sb_per = pl.sb_per;
    const int64_t tiles = pl.tiles;
    const bool atomic = pl.atomic;
    const size_t img_bytes = ((size_t)slices * n_tt * (tt_tok / Q8_TOK) * n_sb * ximg_bytes_rt(type) + 255) & ~(size_t)255;
    size_t part_bytes = ksplit > 1 && !atomic ? (size_t)ksplit * slices * a.M * a.N * sizeof(float) : 0;
    StreamK sk{};
    if (pl.use_sk) {
        sk.cnt = scratch.counters(st);
        sk.n_tiles = (int)tiles;
        if (sk.cnt) part_bytes = (size_t)tiles * 2 * (tt_tok == 128 ? 8 : 4) * 32 * 64 * sizeof(float);
    }
    uint8_t *buf = static_cast<uint8_t *>(scratch.get(img_bytes + part_bytes, st));
    if (!buf) return hipErrorOutOfMemory;
    float *part = reinterpret_cast<float *>(buf + img_bytes);
    sk.part = part;
    switch (type) {
        case T_Q4_0: launch8<T_Q4_0>(a, buf, tr_rows, tt_tok, n_tt, slices, ksplit, sb_per, part, atomic, sk, st); break;
        case T_Q8_0: launch8<T_Q8_0>(a, buf, tr_rows, tt_tok, n_tt, slices, ksplit, sb_per, part, atomic, sk, st); break;
        case T_Q4_K: launch8<T_Q4_K>(a, buf, tr_rows, tt_tok, n_tt, slices, ksplit, sb_per, part, atomic, sk, st); break;
        case T_Q5_K: launch8<T_Q5_K>(a, buf, tr_rows, tt_tok, n_tt, slices, ksplit, sb_per, part, atomic, sk, st); break;
        case T_Q6_K: launch8<T_Q6_K>(a, buf, tr_rows, tt_tok, n_tt, slices, ksplit, sb_per, part, atomic, sk, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// MUL_MAT_ID on the int8 tile (prefill / many tokens): moe_prep groups the (slot, token) pairs
// by expert, mmq8_quant_x gathers and quantizes their columns into one 64-token image per
// tile, and every tile runs the 128 x 64 kernel on its expert's matrix, the epilogue scattering
// rows to dst[slot][token]. grid.y is the bound ceil(P / 64) + n_expert; surplus workgroups
// exit at once, so nothing waits on the host. (Reference: ggml_cuda_mul_mat_id,
// src/ggml-cuda/ggml-cuda.cu:2092-2230, which runs its int8 MMQ per expert.)
// ------------------------------------------------------------------------------------------
constexpr int MOE8_MAX_EXPERTS = 1024;   // moe_prep's LDS counters

// counting sort of the (slot, token) pairs by expert in LDS (one 1024-thread workgroup): per
// expert the offset of its pairs and of its 64-pair token tiles, and the sorted pair list — the
// expert grouping of ggml_compute_forward_mul_mat_id (src/ggml-cpu/ggml-cpu.c:1564-1579)
__global__ __launch_bounds__(1024) void moe_prep(const MmArgs a, int *offsets, int *tile_off, int *pos_pair) {
    __shared__ int cnt[MOE8_MAX_EXPERTS], cur[MOE8_MAX_EXPERTS];
    const int E = a.n_expert, P = a.n_used * a.n_tok;
    for (int e = threadIdx.x; e < E; e += 1024) cnt[e] = 0;
    __syncthreads();
    auto expert_of = [&](int p) {
        const int slot = p % a.n_used, t = p / a.n_used;
        const int ex = *reinterpret_cast<const int32_t *>(reinterpret_cast<const uint8_t *>(a.ids) + slot * a.ids_nb0 +
                                                          (int64_t)t * a.ids_nb1);
        return min(max(ex, 0), E - 1);     // host validates ids; never index out of bounds
    };
    for (int p = threadIdx.x; p < P; p += 1024) atomicAdd(&cnt[expert_of(p)], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        int o = 0, tl = 0;
        for (int e = 0; e < E; ++e) {
            offsets[e] = o;
            tile_off[e] = tl;
            cur[e] = o;
            o += cnt[e];
            tl += (cnt[e] + Q8_TOK - 1) / Q8_TOK;
        }
        offsets[E] = o;
        tile_off[E] = tl;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += 1024) pos_pair[atomicAdd(&cur[expert_of(p)], 1)] = p;
}

static hipError_t moe_prep_launch(const MmArgs &a, int *offsets, int *tile_off, int *pos_pair, hipStream_t st) {
    hipLaunchKernelGGL(moe_prep, dim3(1), dim3(1024), 0, st, a, offsets, tile_off, pos_pair);
    return hipGetLastError();
}

static int64_t moe8_tiles(const MmArgs &a) { return ((int64_t)a.n_used * a.n_tok + 63) / 64 + a.n_expert; }

bool mmq8_id_supported(int type, const MmArgs &a) {
    if (a.n_expert > MOE8_MAX_EXPERTS || a.n_expert < 1) return false;
    MmArgs b = a;
    b.M = a.n_used * a.n_tok;
    b.ne12 = a.n_expert; b.ne13 = 1; b.r2 = 1; b.r3 = 1;   // every expert matrix: alignment of nb02
    if (!mmq8_supported(type, b)) return false;
    return moe8_tiles(a) <= 65535 && moe8_tiles(a) * ((a.K + Q8_QK - 1) / Q8_QK) * ximg_bytes_rt(type) < (1LL << 31);
}

template <int T>
static void launch8_id(const MmArgs &a, uint8_t *ximg, int n_tiles, const Moe8 &moe, hipStream_t st) {
    const int n_sb = (a.K + Q8_QK - 1) / Q8_QK;
    hipLaunchKernelGGL((mmq8_quant_x<T, true>), dim3((unsigned)(n_tiles * (Q8_TOK / 4) * n_sb), 1), dim3(256), 0, st, a,
                       ximg, n_tiles, n_sb, moe, 0);
    const int64_t row_b = (int64_t)a.K / QT<T>::blck * QT<T>::bytes;
    const uint32_t w_extent = (uint32_t)((int64_t)(a.N - 1) * a.nb01 + row_b);
    const unsigned gx = (unsigned)((a.N + 127) / 128);
    const int remap = (gx % 8 == 0) ? 1 : 0;
    hipLaunchKernelGGL((mmq8_kernel<T, 64, 128, true>), dim3(gx, (unsigned)n_tiles), dim3(512), 0, st, a,
                       (const uint8_t *)ximg, 1, 1, n_sb, w_extent, (float *)nullptr, remap, moe, StreamK{});
}

hipError_t mmq8_id_launch(int type, const MmArgs &a, hipStream_t st, Scratch &scratch) {
    const int P = a.n_used * a.n_tok, E = a.n_expert, n_sb = (a.K + Q8_QK - 1) / Q8_QK;
    const int n_tiles = (int)moe8_tiles(a);
    const size_t img_bytes = ((size_t)n_tiles * n_sb * ximg_bytes_rt(type) + 255) & ~(size_t)255;
    const size_t map_bytes = sizeof(int) * (2 * (size_t)(E + 1) + P);
    uint8_t *buf = static_cast<uint8_t *>(scratch.get(img_bytes + map_bytes, st));
    if (!buf) return hipErrorOutOfMemory;
    int *offsets = reinterpret_cast<int *>(buf + img_bytes);
    int *tile_off = offsets + (E + 1);
    int *pos_pair = tile_off + (E + 1);
    hipError_t e = moe_prep_launch(a, offsets, tile_off, pos_pair, st);
    if (e != hipSuccess) return e;
    const Moe8 moe{offsets, tile_off, pos_pair, E, a.n_used};
    switch (type) {
        case T_Q4_0: launch8_id<T_Q4_0>(a, buf, n_tiles, moe, st); break;
        case T_Q8_0: launch8_id<T_Q8_0>(a, buf, n_tiles, moe, st); break;
        case T_Q4_K: launch8_id<T_Q4_K>(a, buf, n_tiles, moe, st); break;
        case T_Q5_K: launch8_id<T_Q5_K>(a, buf, n_tiles, moe, st); break;
        case T_Q6_K: launch8_id<T_Q6_K>(a, buf, n_tiles, moe, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// repacked operand: geometry, the repack launch and the tile launch
// ------------------------------------------------------------------------------------------
static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

RpLayout rp_layout(int type, int K, int N, int n_mat) {
    RpLayout L{};
    L.n_rt = (N + 31) / 32;
    L.n_sb = (K + Q8_QK - 1) / Q8_QK;
    const size_t tiles = (size_t)n_mat * L.n_rt * L.n_sb;
    L.off_meta = al256(tiles * 8192);
    L.bytes = L.off_meta + al256(tiles * 32 * 2 * 16);
    return L;
}

bool repack_supported(int type, const RpSrcView &s) {
    if (!(type == T_Q4_0 || type == T_Q8_0 || type == T_Q4_K || type == T_Q5_K || type == T_Q6_K)) return false;
    if (s.K <= 0 || s.N <= 0 || s.n_mat <= 0 || s.K % type_blck(type) != 0) return false;
    // K-quant headers and qs are read as dwords: 16-B aligned super-blocks (144 / 176 B)
    const uintptr_t al = (type == T_Q4_K || type == T_Q5_K) ? 15 : 1;
    if ((reinterpret_cast<uintptr_t>(s.w) & al) || (s.nb01 & al) || (s.n_mat > s.ne02 && (s.nb03 & al)) || (s.ne02 > 1 && (s.nb02 & al)))
        return false;
    const RpLayout L = rp_layout(type, s.K, s.N, s.n_mat);
    return L.bytes < (1ull << 40) && (int64_t)L.n_rt * L.n_sb * 8192 < (1ll << 32);
}

static RpArgs rp_args(const RpLayout &L, const void *base, int ne02) {
    RpArgs r{};
    r.codes = static_cast<const uint8_t *>(base);
    r.meta = static_cast<const uint8_t *>(base) + L.off_meta;
    r.n_rt = L.n_rt;
    r.n_sb = L.n_sb;
    r.ne02 = ne02;
    return r;
}

hipError_t repack_launch(int type, const RpSrcView &v, void *dst, hipStream_t st) {
    const RpLayout L = rp_layout(type, v.K, v.N, v.n_mat);
    const RpArgs r = rp_args(L, dst, v.ne02);
    const RpSrc s{static_cast<const uint8_t *>(v.w), v.nb01, v.nb02, v.nb03, v.K, v.N, v.ne02, v.n_mat};
    const int64_t threads = (int64_t)v.n_mat * L.n_rt * L.n_sb * 8 * 32;
    const dim3 grid((unsigned)((threads + 255) / 256));
    switch (type) {
        case T_Q4_0: hipLaunchKernelGGL(repack_kernel<T_Q4_0>, grid, dim3(256), 0, st, s, r); break;
        case T_Q8_0: hipLaunchKernelGGL(repack_kernel<T_Q8_0>, grid, dim3(256), 0, st, s, r); break;
        case T_Q4_K: hipLaunchKernelGGL(repack_kernel<T_Q4_K>, grid, dim3(256), 0, st, s, r); break;
        case T_Q5_K: hipLaunchKernelGGL(repack_kernel<T_Q5_K>, grid, dim3(256), 0, st, s, r); break;
        case T_Q6_K: hipLaunchKernelGGL(repack_kernel<T_Q6_K>, grid, dim3(256), 0, st, s, r); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int T>
static void launch8r(const MmArgs &a, const RpArgs &r, uint8_t *ximg, int n_tt, int slices, int ksplit, int sb_per,
                     float *part, bool atomic, hipStream_t st) {
    const int n_sb = r.n_sb;
    hipLaunchKernelGGL(mmq8_quant_x<T>, dim3((unsigned)(n_tt * (Q8_TOK / 4) * n_sb), slices), dim3(256), 0, st, a, ximg,
                       n_tt, n_sb, Moe8{}, atomic ? 1 : 0);
    const int n_rt128 = (a.N + 127) / 128;
    const unsigned gx = (unsigned)(n_rt128 * ksplit * n_tt);
    const int flags = ((gx % 8 == 0) ? 1 : 0) | (atomic ? 4 : 0);
    hipLaunchKernelGGL(mmq8r_kernel<T>, dim3(gx, slices), dim3(512), 0, st, a, r, (const uint8_t *)ximg, n_tt, ksplit,
                       sb_per, part, flags);
    if (ksplit > 1 && !atomic) {
        const int64_t n = (int64_t)slices * a.M * a.N;
        hipLaunchKernelGGL(mmq8_split_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, (const float *)part,
                           ksplit, slices);
    }
}

// the tile on a repacked operand (rp = its base, laid out by rp_layout for the matrices of a);
// repack_first: repack a.w into scratch first (the per-call form)
hipError_t mmq8r_launch(int type, const MmArgs &a, const void *rp, int ne02, int n_mat, hipStream_t st, Scratch &scratch) {
    const int slices = a.ne12 * a.ne13;
    const RpLayout L = rp_layout(type, a.K, a.N, n_mat);
    const int n_sb = L.n_sb;
    const int n_tt = (a.M + Q8_TOK - 1) / Q8_TOK;
    const int n_rt128 = (a.N + 127) / 128;
    const int64_t tiles = (int64_t)n_rt128 * n_tt * slices;
    int ksplit = 1;
    while (tiles * ksplit * 2 <= 256 && n_sb >= 4 * ksplit) ksplit *= 2;
    if (settings().mmq8_ksplit > 0) ksplit = std::max(1, std::min(settings().mmq8_ksplit, n_sb));
    const int sb_per = (n_sb + ksplit - 1) / ksplit;
    ksplit = (n_sb + sb_per - 1) / sb_per;
    const bool atomic = ksplit == 2 && !settings().mmq8_no_atomic;
    const size_t img_bytes = al256((size_t)slices * n_tt * n_sb * ximg_bytes_rt(type));
    const size_t part_bytes = ksplit > 1 && !atomic ? al256((size_t)ksplit * slices * a.M * a.N * sizeof(float)) : 0;
    const size_t rp_bytes = rp ? 0 : L.bytes;
    uint8_t *buf = static_cast<uint8_t *>(scratch.get(img_bytes + part_bytes + rp_bytes, st));
    if (!buf) return hipErrorOutOfMemory;
    float *part = reinterpret_cast<float *>(buf + img_bytes);
    if (!rp) {
        RpSrcView v{a.w, a.nb01, a.nb02, a.nb03, a.K, a.N, ne02, n_mat};
        const hipError_t e = repack_launch(type, v, buf + img_bytes + part_bytes, st);
        if (e != hipSuccess) return e;
        rp = buf + img_bytes + part_bytes;
    }
    const RpArgs r = rp_args(L, rp, ne02);
    switch (type) {
        case T_Q4_0: launch8r<T_Q4_0>(a, r, buf, n_tt, slices, ksplit, sb_per, part, atomic, st); break;
        case T_Q8_0: launch8r<T_Q8_0>(a, r, buf, n_tt, slices, ksplit, sb_per, part, atomic, st); break;
        case T_Q4_K: launch8r<T_Q4_K>(a, r, buf, n_tt, slices, ksplit, sb_per, part, atomic, st); break;
        case T_Q5_K: launch8r<T_Q5_K>(a, r, buf, n_tt, slices, ksplit, sb_per, part, atomic, st); break;
        case T_Q6_K: launch8r<T_Q6_K>(a, r, buf, n_tt, slices, ksplit, sb_per, part, atomic, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace mi355x
