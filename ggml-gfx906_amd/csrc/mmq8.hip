// mmq8.hip — quantized mat-mat (prefill, ne11 > 8) on the int8 matrix cores.
//
// The integer form of the reference's MMQ (src/ggml-cuda/mmq.cuh:3134 mul_mat_q, mma.cuh:515-569
// int8 tiles; the arithmetic of ggml-cpu's block dot products, src/ggml-cpu/quants.c
// ggml_vec_dot_q4_K_q8_K / _q8_0_q8_0), built for gfx950:
//
//   1. mmq8_quant_x: activations -> int8 blocks of 256 exactly as quantize_row_q8_K_ref
//      (src/ggml-quants.c:2555-2591: d = max/-127 of the signed largest-|x| value, q =
//      nearest_int(x * -127/max) clamped to 127) plus the 16-element block sums, one wave per
//      (token, 256-k block). Layout x8[slice][Mpad][K], xd[slice][Mpad][K/256],
//      xbs[slice][Mpad][K/256][16] (f16: sums of 16 int8 are exact in f16).
//   2. mmq8_kernel: 64 weight rows x 64 tokens per workgroup, 4 waves of one 32x32 tile each,
//      KG K-groups (split-K inside the workgroup, reduced through LDS). Per 256-k block the
//      workgroup stages the raw weight bytes and the int8 activations through LDS (coalesced
//      16-B global loads into registers, realigned and written as 32-B rows with a 16-B XOR
//      swizzle that makes every ds_read_b128 fragment read conflict-free), then each wave runs
//      v_mfma_i32_32x32x32_i8 per 32-k block: the B operand is one weight row per lane (so the
//      row's block scale is a per-lane scalar), the A operand 32 tokens.
//        Q8_0 / Q4_0: R_b (int32, exact) -> p += d_b * R_b  (Q4_0 codes decoded to q-8)
//        Q4_K / Q5_K: p_i += sc_j * R_j in int32 (v_mad_i32_i24: the 6-bit sub-block scales
//                     are integers, as ggml_vec_dot_q4_K_q8_K sums them), and the min term
//                     sum_j m_j * bsum_j as one f16 MFMA per block on exact integers;
//                     per block p = d * p_i - dmin * mins.
//      and acc += d8[token] * p once per 256-k block.
//   The integer dot products are those of the CPU backend bit for bit; only the fp32 order of
//   the per-block scale accumulation differs (K-quants: identical activation blocks too).
#include <cstdlib>
#include <cstring>

#include "dispatch.h"
#include "qcommon.h"

namespace mi355x {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

constexpr uint32_t Q8_RSRC_W3 = 0x00020000u;   // raw buffer, dword3 for gfx9-class descriptors
constexpr int Q8_QK = 256;                     // activation block (Q8_K super-block)
constexpr int Q8_TILE = 64;                    // weight rows = tokens per workgroup

// ------------------------------------------------------------------------------------------
// activations -> Q8_K-style int8 blocks (restates quantize_row_q8_K_ref, src/ggml-quants.c:2555)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mmq8_quant_x(const MmArgs a, int8_t *__restrict__ x8, float *__restrict__ xd,
                                                    _Float16 *__restrict__ xbs, int Mpad, int n_sb) {
    const int lane = threadIdx.x & 63;
    const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (item >= (int64_t)Mpad * n_sb) return;   // whole wave
    const int tok = (int)(item / n_sb), sb = (int)(item % n_sb);
    const int slice = blockIdx.y;
    const int i12 = slice % a.ne12, i13 = slice / a.ne12;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (tok < a.M) {
        const float *src = reinterpret_cast<const float *>(a.x + (int64_t)i12 * a.nb12 + (int64_t)i13 * a.nb13 +
                                                           (int64_t)tok * a.nb11) +
                           sb * Q8_QK + lane * 4;
        if (a.x_aligned16) {
            const float4 f = *reinterpret_cast<const float4 *>(src);
            v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = src[i];
        }
    }
    // largest |x| and the first k reaching it (the reference's strict '>' keeps the first)
    float am = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
#pragma unroll
    for (int o = 32; o; o >>= 1) am = fmaxf(am, __shfl_xor(am, o));
    int idx = 1 << 30;
#pragma unroll
    for (int i = 3; i >= 0; --i)
        if (fabsf(v[i]) == am) idx = lane * 4 + i;
#pragma unroll
    for (int o = 32; o; o >>= 1) idx = min(idx, __shfl_xor(idx, o));
    const int sel = idx & 3;
    const float mine = sel == 0 ? v[0] : sel == 1 ? v[1] : sel == 2 ? v[2] : v[3];
    const float mx = __shfl(mine, (idx >> 2) & 63);
    int q[4] = {0, 0, 0, 0};
    float d = 0.f;
    if (am != 0.f) {
        const float iscale = -127.f / mx;
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = min(127, (int)__builtin_rintf(iscale * v[i]));
        d = 1.f / iscale;
    }
    const int64_t rowi = (int64_t)slice * Mpad + tok;
    const uint32_t packed = (uint32_t)(q[0] & 0xff) | (uint32_t)(q[1] & 0xff) << 8 | (uint32_t)(q[2] & 0xff) << 16 |
                            (uint32_t)(q[3] & 0xff) << 24;
    reinterpret_cast<uint32_t *>(x8 + rowi * ((int64_t)n_sb * Q8_QK) + sb * Q8_QK)[lane] = packed;
    int s = q[0] + q[1] + q[2] + q[3];
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    if ((lane & 3) == 0) xbs[(rowi * n_sb + sb) * 16 + (lane >> 2)] = (_Float16)s;
    if (lane == 0) xd[rowi * n_sb + sb] = d;
}

// ------------------------------------------------------------------------------------------
// LDS image of one 256-k block (per K-group):
//   XQ  8 planes x 64 tokens x 32 B  int8 activations, plane b = k 32b..32b+31
//   XD  64 f32                        activation block scales
//   XB  64 tokens x 32 B              16 f16 block sums (K-quants)
//   W   per type (below)
// A 32-B plane row holds two 16-B halves (k 0..15, 16..31); half h of row r sits at
// 16 * (h ^ (r >> 4 & 1)), which spreads every 16-lane ds_read_b128 group over all 64 banks.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pl_off(int r, int h) { return (uint32_t)(r * 32 + 16 * (h ^ ((r >> 4) & 1))); }

constexpr int L_XQ = 0, L_XD = 8 * 2048, L_XB = L_XD + 256, L_W = L_XB + 2048;

template <int T> struct W8;
// Q8_0: WQ 8 planes x 64 rows x 32 B (int8 codes), WD 64 rows x 8 f32 (block scales)
template <> struct W8<T_Q8_0> {
    static constexpr int SBB = 272, WQ = 0, WD = 8 * 2048, BYTES = WD + 2048, NREG = 2 * 9;
};
// Q4_0: WQ 8 planes x 64 rows x 16 B (nibbles), WD as Q8_0
template <> struct W8<T_Q4_0> {
    static constexpr int SBB = 144, WQ = 0, WD = 8 * 1024, BYTES = WD + 2048, NREG = 2 * 5;
};
// Q4_K: WQ 4 planes x 64 rows x 32 B (nibble pairs), WH 64 rows x 16 B header (d, dmin, scales)
template <> struct W8<T_Q4_K> {
    static constexpr int SBB = 144, WQ = 0, WH = 4 * 2048, BYTES = WH + 1024, NREG = 3 * 4, NCH = 9;
};
// Q5_K: as Q4_K plus QH 64 rows x 32 B high bits
template <> struct W8<T_Q5_K> {
    static constexpr int SBB = 176, WQ = 0, WH = 4 * 2048, QH = WH + 1024, BYTES = QH + 2048, NREG = 3 * 4, NCH = 11;
};

template <int T> constexpr int stage_bytes() { return (L_W + W8<T>::BYTES + 15) / 16 * 16; }

__device__ __forceinline__ u32x4v bl128(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t bl32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ void lds_st128(uint8_t *p, u32x4v v) { *reinterpret_cast<u32x4v *>(p) = v; }
__device__ __forceinline__ u32x4v lds_ld128(const uint8_t *p) { return *reinterpret_cast<const u32x4v *>(p); }

// ---- weight staging: global -> registers (issued early) -> LDS (after the block's compute) ----
// j: thread index in the K-group (0..255); wbase: byte offset of this tile's first row + the
// 256-k block within the row
template <int T> struct WStage;

template <> struct WStage<T_Q8_0> {   // task (row, block): 9 dwords covering the 34-B block
    uint32_t w[2][9];
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, uint32_t wbase, uint32_t nb01, int j) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int task = j + 256 * t, row = task >> 3, blk = task & 7;
            const uint32_t off = wbase + (uint32_t)row * nb01 + 34u * blk;
            const uint32_t o4 = off & ~3u;
            const u32x4v a0 = bl128(rs, o4), a1 = bl128(rs, o4 + 16);
            w[t][0] = a0[0]; w[t][1] = a0[1]; w[t][2] = a0[2]; w[t][3] = a0[3];
            w[t][4] = a1[0]; w[t][5] = a1[1]; w[t][6] = a1[2]; w[t][7] = a1[3];
            w[t][8] = bl32(rs, o4 + 32);
        }
    }
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 9; ++i) w[t][i] = 0;
    }
    __device__ __forceinline__ void store(uint8_t *W, uint32_t wbase, uint32_t nb01, int j) const {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int task = j + 256 * t, row = task >> 3, blk = task & 7;
            const bool odd = ((wbase + (uint32_t)row * nb01 + 34u * blk) & 2u) != 0;   // block at +2 in w[0]
            // odd: d = hi16(w0), codes = w1..w8; even: d = lo16(w0), codes = bytes 2..33
            const uint32_t dbits = odd ? (w[t][0] >> 16) : (w[t][0] & 0xffffu);
            uint32_t q[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) q[i] = odd ? w[t][i + 1] : __builtin_amdgcn_alignbyte(w[t][i + 1], w[t][i], 2);
            uint8_t *WQ = W + W8<T_Q8_0>::WQ + blk * 2048;
            lds_st128(WQ + pl_off(row, 0), u32x4v{q[0], q[1], q[2], q[3]});
            lds_st128(WQ + pl_off(row, 1), u32x4v{q[4], q[5], q[6], q[7]});
            *reinterpret_cast<float *>(W + W8<T_Q8_0>::WD + pl_off(row, blk >> 2) + 4 * (blk & 3)) = h2f((uint16_t)dbits);
        }
    }
};

template <> struct WStage<T_Q4_0> {   // task (row, block): 5 dwords covering the 18-B block
    uint32_t w[2][5];
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, uint32_t wbase, uint32_t nb01, int j) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int task = j + 256 * t, row = task >> 3, blk = task & 7;
            const uint32_t off = wbase + (uint32_t)row * nb01 + 18u * blk;
            const uint32_t o4 = off & ~3u;
            const u32x4v a0 = bl128(rs, o4);
            w[t][0] = a0[0]; w[t][1] = a0[1]; w[t][2] = a0[2]; w[t][3] = a0[3];
            w[t][4] = bl32(rs, o4 + 16);
        }
    }
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 5; ++i) w[t][i] = 0;
    }
    __device__ __forceinline__ void store(uint8_t *W, uint32_t wbase, uint32_t nb01, int j) const {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int task = j + 256 * t, row = task >> 3, blk = task & 7;
            const bool odd = ((wbase + (uint32_t)row * nb01 + 18u * blk) & 2u) != 0;
            const uint32_t dbits = odd ? (w[t][0] >> 16) : (w[t][0] & 0xffffu);
            uint32_t q[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) q[i] = odd ? w[t][i + 1] : __builtin_amdgcn_alignbyte(w[t][i + 1], w[t][i], 2);
            lds_st128(W + W8<T_Q4_0>::WQ + blk * 1024 + row * 16, u32x4v{q[0], q[1], q[2], q[3]});
            *reinterpret_cast<float *>(W + W8<T_Q4_0>::WD + pl_off(row, blk >> 2) + 4 * (blk & 3)) = h2f((uint16_t)dbits);
        }
    }
};

// K-quants: the row's 256-k block is 16-B aligned; task (row, 16-B chunk)
template <int T> struct WStageK {
    static constexpr int NCH = W8<T>::NCH, NT = 64 * NCH;
    u32x4v w[3];
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, uint32_t wbase, uint32_t nb01, int j) {
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int task = j + 256 * t;
            const int row = task / NCH, ch = task % NCH;
            // tasks past the block (t = 2 for some threads) read an in-range dummy, never stored
            w[t] = bl128(rs, wbase + (uint32_t)min(row, 63) * nb01 + 16u * ch);
        }
    }
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int t = 0; t < 3; ++t) w[t] = u32x4v{0, 0, 0, 0};
    }
    __device__ __forceinline__ void store(uint8_t *W, uint32_t, uint32_t, int j) const {
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int task = j + 256 * t;
            if (task >= NT) break;
            const int row = task / NCH, ch = task % NCH;
            uint8_t *dst;
            if (ch == 0) {
                dst = W + W8<T>::WH + row * 16;
            } else if (T == T_Q5_K && ch <= 2) {
                dst = W + W8<T_Q5_K>::QH + pl_off(row, ch - 1);
            } else {
                const int c16 = ch - (T == T_Q5_K ? 3 : 1);
                dst = W + W8<T>::WQ + (c16 >> 1) * 2048 + pl_off(row, c16 & 1);
            }
            lds_st128(dst, w[t]);
        }
    }
};
template <> struct WStage<T_Q4_K> : WStageK<T_Q4_K> {};
template <> struct WStage<T_Q5_K> : WStageK<T_Q5_K> {};

// ---- activation staging: 64 tokens x 256 B + scales (+ block sums) ----
struct XStage {
    u32x4v q[4];
    float d;
    u32x4v bs;
    __device__ __forceinline__ void load(const int8_t *x8, const float *xd, const _Float16 *xbs, int64_t row0, int K,
                                         int n_sb, int sb, int j, bool ksum) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int task = j + 256 * i, tok = task >> 4, c16 = task & 15;
            q[i] = *reinterpret_cast<const u32x4v *>(x8 + (row0 + tok) * K + sb * Q8_QK + 16 * c16);
        }
        d = j < 64 ? xd[(row0 + j) * n_sb + sb] : 0.f;
        if (ksum && j < 128)
            bs = *reinterpret_cast<const u32x4v *>(xbs + ((row0 + (j >> 1)) * n_sb + sb) * 16 + 8 * (j & 1));
    }
    __device__ __forceinline__ void store(uint8_t *S, int j, bool ksum) const {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int task = j + 256 * i, tok = task >> 4, c16 = task & 15;
            lds_st128(S + L_XQ + (c16 >> 1) * 2048 + pl_off(tok, c16 & 1), q[i]);
        }
        if (j < 64) reinterpret_cast<float *>(S + L_XD)[j] = d;
        if (ksum && j < 128) lds_st128(S + L_XB + pl_off(j >> 1, j & 1), bs);
    }
};

__device__ __forceinline__ i32x4 as_i4(u32x4v v) { return __builtin_bit_cast(i32x4, v); }

// ---- compute of one 256-k block by one wave: 32 tokens (A) x 32 weight rows (B) ----
// acc[i]: token 32*tg + (i & 3) + 8 * (i >> 2) + 4 * h, weight row 32*rg + (lane & 31)
template <int T>
__device__ __forceinline__ void block_compute(const uint8_t *S, int rg, int tg, int lane, f32x16 &acc) {
    const int r = lane & 31, h = lane >> 5;
    const int wrow = 32 * rg + r, atok = 32 * tg + r;
    const uint8_t *W = S + L_W;
    const i32x16 zero16 = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    f32x16 p;
    if constexpr (T == T_Q8_0 || T == T_Q4_0) {
        const float4 d0 = *reinterpret_cast<const float4 *>(W + W8<T>::WD + pl_off(wrow, 0));
        const float4 d1 = *reinterpret_cast<const float4 *>(W + W8<T>::WD + pl_off(wrow, 1));
        const float dw[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
        for (int i = 0; i < 16; ++i) p[i] = 0.f;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            u32x4v bq;
            if constexpr (T == T_Q8_0) {
                bq = lds_ld128(W + W8<T>::WQ + b * 2048 + pl_off(wrow, h));
            } else {   // Q4_0: k 0..15 low nibbles, 16..31 high nibbles, codes q - 8
                const u32x4v raw = lds_ld128(W + W8<T>::WQ + b * 1024 + wrow * 16);
#pragma unroll
                for (int i = 0; i < 4; ++i) bq[i] = sub8_bytes((raw[i] >> (4 * h)) & 0x0F0F0F0Fu);
            }
            const u32x4v aq = lds_ld128(S + L_XQ + b * 2048 + pl_off(atok, h));
            const i32x16 R = __builtin_amdgcn_mfma_i32_32x32x32_i8(as_i4(aq), as_i4(bq), zero16, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; ++i) p[i] = __builtin_fmaf((float)R[i], dw[b], p[i]);
        }
    } else {   // Q4_K / Q5_K
        const u32x4v hd = lds_ld128(W + W8<T>::WH + wrow * 16);
        const uint32_t S3[3] = {hd[1], hd[2], hd[3]};
        uint32_t sc[8], mn[8];
#pragma unroll
        for (int c = 0; c < 4; ++c) k4_scale_min_pair(S3, c, sc[2 * c], sc[2 * c + 1], mn[2 * c], mn[2 * c + 1]);
        u32x4v qh = {0, 0, 0, 0};
        if constexpr (T == T_Q5_K) qh = lds_ld128(W + W8<T_Q5_K>::QH + pl_off(wrow, h));
        i32x16 pi = zero16;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const u32x4v raw = lds_ld128(W + W8<T>::WQ + c * 2048 + pl_off(wrow, h));
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int j = 2 * c + e;
                u32x4v bq;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    uint32_t v = (raw[i] >> (4 * e)) & 0x0F0F0F0Fu;
                    if constexpr (T == T_Q5_K) v |= ((qh[i] >> j) & 0x01010101u) << 4;
                    bq[i] = v;
                }
                const u32x4v aq = lds_ld128(S + L_XQ + j * 2048 + pl_off(atok, h));
                const i32x16 R = __builtin_amdgcn_mfma_i32_32x32x32_i8(as_i4(aq), as_i4(bq), zero16, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 16; ++i) pi[i] += __mul24(R[i], (int)sc[j]);
            }
        }
        // sum_j m_j * bsum_j: A = the token's 16 block sums of 16 (k = 8h + i), B = m_(k/2)
        const u32x4v bsr = lds_ld128(S + L_XB + pl_off(atok, h));
        const f16x8 am = __builtin_bit_cast(f16x8, bsr);
        f16x8 bm;
#pragma unroll
        for (int i = 0; i < 8; ++i) bm[i] = (_Float16)(float)mn[4 * h + (i >> 1)];
        const f32x16 zf = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const f32x16 mins = __builtin_amdgcn_mfma_f32_32x32x16_f16(am, bm, zf, 0, 0, 0);
        const float d = h2f((uint16_t)(hd[0] & 0xffff)), dmin = h2f((uint16_t)(hd[0] >> 16));
#pragma unroll
        for (int i = 0; i < 16; ++i) p[i] = __builtin_fmaf(d, (float)pi[i], -dmin * mins[i]);
    }
    const float *XD = reinterpret_cast<const float *>(S + L_XD);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float4 dx = *reinterpret_cast<const float4 *>(XD + 32 * tg + 8 * g + 4 * h);
        acc[4 * g + 0] = __builtin_fmaf(p[4 * g + 0], dx.x, acc[4 * g + 0]);
        acc[4 * g + 1] = __builtin_fmaf(p[4 * g + 1], dx.y, acc[4 * g + 1]);
        acc[4 * g + 2] = __builtin_fmaf(p[4 * g + 2], dx.z, acc[4 * g + 2]);
        acc[4 * g + 3] = __builtin_fmaf(p[4 * g + 3], dx.w, acc[4 * g + 3]);
    }
}

// grid: (ceil(N / 64), Mpad / 64, slices); KG K-groups of 4 waves
template <int T, int KG>
__global__ __launch_bounds__(256 * KG) void mmq8_kernel(const MmArgs a, const int8_t *__restrict__ x8,
                                                        const float *__restrict__ xd,
                                                        const _Float16 *__restrict__ xbs, int Mpad, uint32_t w_extent) {
    constexpr int SBYTES = stage_bytes<T>();
    constexpr bool KSUM = T == T_Q4_K || T == T_Q5_K;
    __shared__ __align__(16) uint8_t lds[KG * SBYTES];
    const int K = a.K, n_sb = K / Q8_QK;
    const int slice = blockIdx.z;
    const int i12 = slice % a.ne12, i13 = slice / a.ne12;
    const uint8_t *wmat = a.w + (int64_t)(i12 / a.r2) * a.nb02 + (int64_t)(i13 / a.r3) * a.nb03;
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void *)wmat, 0, w_extent, Q8_RSRC_W3);
    const int row0 = blockIdx.x * Q8_TILE, tok0 = blockIdx.y * Q8_TILE;
    const int64_t xrow0 = (int64_t)slice * Mpad + tok0;
    const uint32_t nb01 = (uint32_t)a.nb01;

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int kg = wave >> 2, rg = wave & 1, tg = (wave >> 1) & 1;
    const int j = threadIdx.x & 255;
    uint8_t *S = lds + kg * SBYTES;

    WStage<T> ws;
    XStage xs;
    const int iters = (n_sb + KG - 1) / KG;
    auto load = [&](int sb) {
        if (sb < n_sb) {
            ws.load(wr, (uint32_t)row0 * nb01 + (uint32_t)sb * W8<T>::SBB, nb01, j);
            xs.load(x8, xd, xbs, xrow0, K, n_sb, sb, j, KSUM);
        }
    };
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    load(kg);
    for (int it = 0; it < iters; ++it) {
        const int sb = kg + it * KG;
        __syncthreads();   // the previous block's compute is done with the LDS image
        if (sb < n_sb) {
            ws.store(S + L_W, (uint32_t)row0 * nb01 + (uint32_t)sb * W8<T>::SBB, nb01, j);
            xs.store(S, j, KSUM);
        }
        __syncthreads();
        load(sb + KG);     // next block's global loads fly during this block's MFMAs
        if (sb < n_sb) block_compute<T>(S, rg, tg, lane, acc);
    }
    // K-group reduction through LDS, then the store: dst[token][row] (coalesced rows per i)
    if constexpr (KG > 1) {
        __syncthreads();
        float *red = reinterpret_cast<float *>(lds);
        if (kg > 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) red[(((kg - 1) * 4 + (wave & 3)) * 16 + i) * 64 + lane] = acc[i];
        }
        __syncthreads();
        if (kg > 0) return;
#pragma unroll
        for (int g = 1; g < KG; ++g)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] += red[(((g - 1) * 4 + wave) * 16 + i) * 64 + lane];
    }
    const int row = row0 + 32 * rg + (lane & 31);
    if (row >= a.N) return;
    uint8_t *dmat = a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int tok = tok0 + 32 * tg + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
        if (tok < a.M) reinterpret_cast<float *>(dmat + (int64_t)tok * a.nb1)[row] = acc[i];
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
bool mmq8_supported(int type, const MmArgs &a) {
    if (!(type == T_Q4_0 || type == T_Q8_0 || type == T_Q4_K || type == T_Q5_K)) return false;
    if (a.K % Q8_QK != 0 || a.M <= 0) return false;
    // dword-aligned rows (Q4_0 / Q8_0 windows), 16-B aligned 256-k row segments (K-quants)
    const uintptr_t al = (type == T_Q4_K || type == T_Q5_K) ? 15 : 3;
    if ((reinterpret_cast<uintptr_t>(a.w) & al) || (a.nb01 & al) || (a.nb02 & al) || (a.nb03 & al)) return false;
    const int64_t row_b = (int64_t)a.K / type_blck(type) * type_bytes(type);
    const int64_t w_span = (int64_t)(a.N + Q8_TILE) * a.nb01 + row_b;
    const int64_t slices = (int64_t)a.ne12 * a.ne13;
    const int64_t mpad = (a.M + Q8_TILE - 1) / Q8_TILE * Q8_TILE;
    return a.nb01 >= row_b && w_span < (1LL << 32) && slices * mpad * a.K < (1LL << 31);
}

template <int T, int KG>
static void launch8(const MmArgs &a, const int8_t *x8, const float *xd, const _Float16 *xbs, int Mpad, int slices,
                    hipStream_t st) {
    const dim3 grid((a.N + Q8_TILE - 1) / Q8_TILE, Mpad / Q8_TILE, slices);
    const int64_t row_b = (int64_t)a.K / QT<T>::blck * QT<T>::bytes;
    // windows of the last block may reach 2 bytes past the row: round the range up to a dword
    const uint32_t w_extent = (uint32_t)(((int64_t)(a.N - 1) * a.nb01 + row_b + 3) & ~(int64_t)3);
    hipLaunchKernelGGL((mmq8_kernel<T, KG>), grid, dim3(256 * KG), 0, st, a, x8, xd, xbs, Mpad, w_extent);
}

template <int T>
static void launch8_kg(int kg, const MmArgs &a, const int8_t *x8, const float *xd, const _Float16 *xbs, int Mpad,
                       int slices, hipStream_t st) {
    if (kg >= 2) launch8<T, 2>(a, x8, xd, xbs, Mpad, slices, st);
    else launch8<T, 1>(a, x8, xd, xbs, Mpad, slices, st);
}

hipError_t mmq8_launch(int type, const MmArgs &a, hipStream_t st, Scratch &scratch) {
    const int slices = a.ne12 * a.ne13;
    const int Mpad = (a.M + Q8_TILE - 1) / Q8_TILE * Q8_TILE;
    const int n_sb = a.K / Q8_QK;
    const size_t x8_bytes = ((size_t)slices * Mpad * a.K + 255) & ~(size_t)255;
    const size_t xd_bytes = ((size_t)slices * Mpad * n_sb * sizeof(float) + 255) & ~(size_t)255;
    const size_t xb_bytes = (size_t)slices * Mpad * n_sb * 16 * sizeof(_Float16);
    uint8_t *buf = static_cast<uint8_t *>(scratch.get(x8_bytes + xd_bytes + xb_bytes, st));
    if (!buf) return hipErrorOutOfMemory;
    int8_t *x8 = reinterpret_cast<int8_t *>(buf);
    float *xd = reinterpret_cast<float *>(buf + x8_bytes);
    _Float16 *xbs = reinterpret_cast<_Float16 *>(buf + x8_bytes + xd_bytes);
    const int64_t items = (int64_t)Mpad * n_sb;
    hipLaunchKernelGGL(mmq8_quant_x, dim3((unsigned)((items + 3) / 4), slices), dim3(256), 0, st, a, x8, xd, xbs, Mpad,
                       n_sb);
    // K-groups: split K inside the workgroup while the grid alone leaves CUs short of 2 workgroups
    static const char *env = getenv("GGML_MI355X_MMQ8_KG");
    const int64_t wgs = (int64_t)((a.N + Q8_TILE - 1) / Q8_TILE) * (Mpad / Q8_TILE) * slices;
    int kg = (wgs < 1024 && n_sb >= 2) ? 2 : 1;
    if (env) kg = atoi(env);
    switch (type) {
        case T_Q4_0: launch8_kg<T_Q4_0>(kg, a, x8, xd, xbs, Mpad, slices, st); break;
        case T_Q8_0: launch8_kg<T_Q8_0>(kg, a, x8, xd, xbs, Mpad, slices, st); break;
        case T_Q4_K: launch8_kg<T_Q4_K>(kg, a, x8, xd, xbs, Mpad, slices, st); break;
        case T_Q5_K: launch8_kg<T_Q5_K>(kg, a, x8, xd, xbs, Mpad, slices, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace mi355x
