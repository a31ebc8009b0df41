// mmvq_impl.h — quantized mat-vec kernel template (decode, ne11 <= 8) for gfx950.
//
// Replaces the reference's mul_mat_vec_q / quantize_q8_1 pair (src/ggml-cuda/mmvq.cu:139-226,
// quantize.cu:4-48) with a CDNA4-first design:
//
//  * one 512-thread workgroup = 8 waves; each wave owns RPW consecutive weight rows;
//  * a lane owns a fixed 64-weight "slot" of K for every row it touches (Q4_0/Q8_0: two
//    32-blocks; Q4_K/Q5_K: one 64-chunk of a super-block; Q6_K: a quarter of a 128-half), so
//    a wave's weight stream is a handful of wide (dwordx4) loads per row, issued for all RPW
//    rows up front, straight to VGPRs (no LDS round trip for the once-read weights);
//  * src1 is quantized to int8 per 32-block (d = amax/127, round-to-nearest-even) once per
//    workgroup into LDS, in a slot-interleaved layout so lane s reads its 64 activations with
//    4 conflict-free ds_read_b128. Quantization is ~2 VALU per value: one FMA against the
//    1.5*2^23 magic constant rounds and biases, v_perm_b32 packs bytes, v_dot4_u32_u8 sums;
//  * beside the bytes sit d, d*sum(q) per 32-block and d*sum(q) per 16-run, so the zero-point
//    terms of Q4_0 (q-8), Q6_K (q-32) and the Q4_K/Q5_K mins cost one FMA per block instead of
//    a per-byte fix-up;
//  * integer block dots on v_dot4_i32_i8, fp32 scale accumulation per block — the reference's
//    per-block arithmetic (src/ggml-cpu/quants.c:115-758);
//  * cross-lane reduction by a butterfly transpose on DPP / permlane swaps: RPW*NC partial
//    sums per lane collapse to one value per lane without touching LDS.
//
// Templated on <type, NC columns, RPW rows per wave, IDS = MUL_MAT_ID routing, RAG, XA>.
#pragma once
#include <algorithm>
#include <cstdlib>

#include "qcommon.h"
#include "qmm_args.h"

namespace mi355x {

// measurement builds only (scripts/mmvq_exp.sh): 1 = no activation loads, 2 = no quantization
// into LDS, 4 = no weight loads, 8 = no barrier before the dots, 16 = no issue-order barrier
// (profiles/r06_single_launch_decomposition.txt)
#ifndef MMVQ_EXP
#define MMVQ_EXP 0
#endif

constexpr int MMVQ_WAVES = 8;
constexpr int MMVQ_THREADS = MMVQ_WAVES * WAVE;

// ------------------------------------------------------------------------------------------
// slot geometry: K-chunk (16 activations) q  <->  (slot s, part j)
// ------------------------------------------------------------------------------------------
template <int T> struct SlotMap {
    // slot s covers activations [64 s, 64 s + 64): parts are consecutive 16-chunks
    __device__ static inline void place(int q, int &s, int &j) { s = q >> 2; j = q & 3; }
};
template <> struct SlotMap<T_Q6_K> {
    // slot s = 4 sb + 2 h + p covers 256 sb + 128 h + 16 p + 32 j + [0,16), j = 0..3
    __device__ static inline void place(int q, int &s, int &j) {
        const int sb = q >> 4, r = q & 15, h = r >> 3, r2 = r & 7;
        j = r2 >> 1;
        s = 4 * sb + 2 * h + (r2 & 1);
    }
};

// ------------------------------------------------------------------------------------------
// activation quantization into LDS (per column m, Kpad = K rounded up to 64):
//   xq  : int8 [Kpad]      slot-interleaved: chunk (s, j) at (j * nslots + s) * 16
//   xd  : f32  [Kpad/32]   block scale d = amax / 127
//   xs  : f32  [Kpad/32]   d * sum(q) over the 32-block
//   x16 : f32  [Kpad/16]   d * sum(q) over each 16-run
// Work split: 4 lanes per 32-block (8 values each, DPP inside the quad); a round covers
// MMVQ_THREADS/4 blocks; loads of a round are issued before its arithmetic.
// ------------------------------------------------------------------------------------------
struct XSmem {
    int8_t *xq;
    float *xd, *xs, *x16;
};

__device__ __forceinline__ XSmem xsmem(uint8_t *smem, int Kpad, int nc) {
    XSmem s;
    s.xq = reinterpret_cast<int8_t *>(smem);
    s.xd = reinterpret_cast<float *>(smem + (size_t)nc * Kpad);
    s.xs = s.xd + nc * (Kpad / 32);
    s.x16 = s.xs + nc * (Kpad / 32);
    return s;
}

constexpr int XR_STRIDE = MMVQ_THREADS / 4;

// Branch-free: the address is clamped into the row, so every lane issues the same loads (a
// load under a branch makes the compiler's in-order vmcnt bookkeeping ambiguous and it then
// waits for ALL outstanding loads). The loaded values are NOT touched here: out-of-range
// lanes are zeroed by xblock_mask once the weight stream is in flight too — a select right
// behind the load would make the compiler wait for the activations before it issues the
// weights, serializing two memory latencies.
template <bool XA>
__device__ __forceinline__ void xblock_load(const MmArgs &a, const uint8_t *xcol, int kb, float4 &v0, float4 &v1) {
    const int k0 = kb * 32 + (threadIdx.x & 3) * 8;
    const float *src = reinterpret_cast<const float *>(xcol) + min(k0, a.K - 8);
    if constexpr (XA) {
        v0 = reinterpret_cast<const float4 *>(src)[0];
        v1 = reinterpret_cast<const float4 *>(src)[1];
    } else {
        v0 = make_float4(src[0], src[1], src[2], src[3]);
        v1 = make_float4(src[4], src[5], src[6], src[7]);
    }
}

__device__ __forceinline__ void xblock_mask(const MmArgs &a, int kb, float4 &v0, float4 &v1) {
    const bool in = kb * 32 + (int)(threadIdx.x & 3) * 8 < a.K;
    v0.x = in ? v0.x : 0.f; v0.y = in ? v0.y : 0.f; v0.z = in ? v0.z : 0.f; v0.w = in ? v0.w : 0.f;
    v1.x = in ? v1.x : 0.f; v1.y = in ? v1.y : 0.f; v1.z = in ? v1.z : 0.f; v1.w = in ? v1.w : 0.f;
}

// FUSE, a.attn_part != nullptr: the 8 activations of this lane are elements k0 .. k0+7 of the
// attention output of column `col` (one head: k0 % 8 == 0), merged from the ATTN_SPLITS
// partials by the usual rescaling: O = sum_i e^(m_i - M) o_i / sum_i e^(m_i - M) l_i.
// Loaded in the issue phase (attn_part_load), combined after the weights are in flight.
struct AttnPart {
    float m[ATTN_SPLITS], l[ATTN_SPLITS];
    float4 o0[ATTN_SPLITS], o1[ATTN_SPLITS];
};

__device__ __forceinline__ void attn_part_load(const MmArgs &a, int col, int kb, AttnPart &p) {
    const int k0 = min(kb * 32 + (int)(threadIdx.x & 3) * 8, a.K - 8);
    const int h = k0 >> 6, d0 = k0 & 63;
    const float *pb = a.attn_part + (int64_t)(col * a.n_head + h) * ATTN_SPLITS * ATTN_PART_STRIDE;
#pragma unroll
    for (int i = 0; i < ATTN_SPLITS; ++i) {
        const float *q = pb + i * ATTN_PART_STRIDE;
        p.m[i] = q[0];
        p.l[i] = q[1];
        p.o0[i] = *reinterpret_cast<const float4 *>(q + 4 + d0);
        p.o1[i] = *reinterpret_cast<const float4 *>(q + 8 + d0);
    }
}

__device__ __forceinline__ void attn_part_combine(const AttnPart &p, float4 &v0, float4 &v1) {
    float M = -INFINITY;
#pragma unroll
    for (int i = 0; i < ATTN_SPLITS; ++i) M = p.l[i] > 0.f ? fmaxf(M, p.m[i]) : M;
    float L = 0.f;
    v0 = make_float4(0.f, 0.f, 0.f, 0.f);
    v1 = v0;
#pragma unroll
    for (int i = 0; i < ATTN_SPLITS; ++i) {
        const float w = p.l[i] > 0.f ? expf(p.m[i] - M) : 0.f;
        L += w * p.l[i];
        v0.x += w * p.o0[i].x; v0.y += w * p.o0[i].y; v0.z += w * p.o0[i].z; v0.w += w * p.o0[i].w;
        v1.x += w * p.o1[i].x; v1.y += w * p.o1[i].y; v1.z += w * p.o1[i].z; v1.w += w * p.o1[i].w;
    }
    const float inv = 1.0f / L;
    v0 = make_float4(v0.x * inv, v0.y * inv, v0.z * inv, v0.w * inv);
    v1 = make_float4(v1.x * inv, v1.y * inv, v1.z * inv, v1.w * inv);
}

template <int T>
__device__ __forceinline__ void xblock_store(int Kpad, int kb, const float4 &v0, const float4 &v1, int8_t *xq,
                                             float *xd, float *xs, float *x16) {
    const int sub = threadIdx.x & 3;
    float amax = fmaxf(fmaxf(fmaxf(fabsf(v0.x), fabsf(v0.y)), fmaxf(fabsf(v0.z), fabsf(v0.w))),
                       fmaxf(fmaxf(fabsf(v1.x), fabsf(v1.y)), fmaxf(fabsf(v1.z), fabsf(v1.w))));
    amax = fmaxf(amax, dpp_f<DPP_XOR1>(amax));
    amax = fmaxf(amax, dpp_f<DPP_XOR2>(amax));
    const float d = amax * (1.0f / 127.f);
    const float id = amax > 0.f ? 127.f * __builtin_amdgcn_rcpf(amax) : 0.f;
    // t = x*id + (1.5*2^23 + 128): the FMA rounds to nearest-even into the mantissa, so the
    // low byte of t's bits is 128 + q with q in [-127, 127]
    constexpr float MAGIC = 12582912.0f + 128.0f;
    const uint32_t b0 = __builtin_bit_cast(uint32_t, __builtin_fmaf(v0.x, id, MAGIC));
    const uint32_t b1 = __builtin_bit_cast(uint32_t, __builtin_fmaf(v0.y, id, MAGIC));
    const uint32_t b2 = __builtin_bit_cast(uint32_t, __builtin_fmaf(v0.z, id, MAGIC));
    const uint32_t b3 = __builtin_bit_cast(uint32_t, __builtin_fmaf(v0.w, id, MAGIC));
    const uint32_t b4 = __builtin_bit_cast(uint32_t, __builtin_fmaf(v1.x, id, MAGIC));
    const uint32_t b5 = __builtin_bit_cast(uint32_t, __builtin_fmaf(v1.y, id, MAGIC));
    const uint32_t b6 = __builtin_bit_cast(uint32_t, __builtin_fmaf(v1.z, id, MAGIC));
    const uint32_t b7 = __builtin_bit_cast(uint32_t, __builtin_fmaf(v1.w, id, MAGIC));
    const uint32_t w0 = __builtin_amdgcn_perm(__builtin_amdgcn_perm(b3, b2, 0x0c0c0400u), __builtin_amdgcn_perm(b1, b0, 0x0c0c0400u), 0x05040100u);
    const uint32_t w1 = __builtin_amdgcn_perm(__builtin_amdgcn_perm(b7, b6, 0x0c0c0400u), __builtin_amdgcn_perm(b5, b4, 0x0c0c0400u), 0x05040100u);
    // biased bytes (128 + q): sum(q) = udot4(bytes, 1) - 4*128 per dword
    const int qs = (int)__builtin_amdgcn_udot4(w0, 0x01010101u, __builtin_amdgcn_udot4(w1, 0x01010101u, 0u, false), false) - 1024;
    int s, j;
    SlotMap<T>::place(kb * 2 + (sub >> 1), s, j);
    const int nslots = Kpad / 64;
    *reinterpret_cast<uint2 *>(xq + (size_t)(j * nslots + s) * 16 + (sub & 1) * 8) = make_uint2(w0 ^ 0x80808080u, w1 ^ 0x80808080u);
    float fs = (float)qs;
    fs += dpp_f<DPP_XOR1>(fs);              // 16-run sum (lane pairs 0-1 / 2-3)
    if ((sub & 1) == 0) x16[kb * 2 + (sub >> 1)] = d * fs;
    fs += dpp_f<DPP_XOR2>(fs);              // 32-block sum
    if (sub == 0) {
        xd[kb] = d;
        xs[kb] = d * fs;
    }
}

// ------------------------------------------------------------------------------------------
// per-type weight fragment: load (raw bytes of one slot of one row) and dot with a column.
//   X  : 16 dwords = the slot's 64 int8 activations (parts j = 0..3)
//   dx : block scales of the slot's 32-blocks (2, or 4 for Q6_K)
//   sx : d*sum(q): per 32-block (Q4_0, Q4_K, Q5_K) or per 16-run (Q6_K)
// ------------------------------------------------------------------------------------------
template <int T> struct Frag;

// Q4_0: slot = blocks 2s, 2s+1 (36 contiguous bytes); sum (q-8)*x = sum q*x - 8 sum x
template <> struct Frag<T_Q4_0> {
    uint32_t D[9];
    template <bool RAG>
    __device__ inline void load(const uint8_t *row, int s, int nblk) {
        const uint8_t *p = row + (size_t)s * 36;
        ld16(p, D);
        if (!RAG || 2 * s + 1 < nblk) {
            ld16(p + 16, D + 4);
            D[8] = ld4(p + 32);
        } else {                     // ragged tail: K % 64 == 32, second block absent
            D[4] = ld2(p + 16);
            D[5] = D[6] = D[7] = D[8] = 0;
        }
    }
    __device__ inline void zero() { for (int i = 0; i < 9; ++i) D[i] = 0; }
    __device__ inline float dot(const uint32_t X[16], const float *dx, const float *sx) const {
        const float d0 = h2f((uint16_t)(D[0] & 0xffff));
        const float d1 = h2f((uint16_t)(D[4] >> 16));
        int s0 = 0, s1 = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t q0 = align2(D[i + 1], D[i]);      // qs of block 0 at byte 2
            s0 = dot4(q0 & 0x0f0f0f0fu, X[i], s0);
            s0 = dot4((q0 >> 4) & 0x0f0f0f0fu, X[4 + i], s0);
            const uint32_t q1 = D[5 + i];                   // qs of block 1 at byte 20
            s1 = dot4(q1 & 0x0f0f0f0fu, X[8 + i], s1);
            s1 = dot4((q1 >> 4) & 0x0f0f0f0fu, X[12 + i], s1);
        }
        return d0 * __builtin_fmaf(dx[0], (float)s0, -8.f * sx[0]) + d1 * __builtin_fmaf(dx[1], (float)s1, -8.f * sx[1]);
    }
};

// Q8_0: slot = blocks 2s, 2s+1 (68 contiguous bytes)
template <> struct Frag<T_Q8_0> {
    uint32_t D[17];
    template <bool RAG>
    __device__ inline void load(const uint8_t *row, int s, int nblk) {
        const uint8_t *p = row + (size_t)s * 68;
        ld16(p, D);
        ld16(p + 16, D + 4);
        if (!RAG || 2 * s + 1 < nblk) {
            ld16(p + 32, D + 8);
            ld16(p + 48, D + 12);
            D[16] = ld4(p + 64);
        } else {
            D[8] = ld2(p + 32);
            for (int i = 9; i < 17; ++i) D[i] = 0;
        }
    }
    __device__ inline void zero() { for (int i = 0; i < 17; ++i) D[i] = 0; }
    __device__ inline float dot(const uint32_t X[16], const float *dx, const float *) const {
        const float d0 = h2f((uint16_t)(D[0] & 0xffff));
        const float d1 = h2f((uint16_t)(D[8] >> 16));
        int s0 = 0, s1 = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            s0 = dot4(align2(D[i + 1], D[i]), X[i], s0);
            s1 = dot4(D[9 + i], X[8 + i], s1);
        }
        return (d0 * dx[0]) * (float)s0 + (d1 * dx[1]) * (float)s1;
    }
};

// Q4_K: slot = (super-block s/4, 64-chunk c = s%4): header 16 B + qs[32c .. 32c+32)
template <> struct Frag<T_Q4_K> {
    uint32_t H[4], Q[8];
    int c;
    template <bool RAG>
    __device__ inline void load(const uint8_t *row, int s, int) {
        const uint8_t *p = row + (size_t)(s >> 2) * 144;
        c = s & 3;
        ld16(p, H);
        ld16(p + 16 + 32 * c, Q);
        ld16(p + 32 + 32 * c, Q + 4);
    }
    __device__ inline void zero() { for (int i = 0; i < 4; ++i) H[i] = 0; for (int i = 0; i < 8; ++i) Q[i] = 0; c = 0; }
    __device__ inline float dot(const uint32_t X[16], const float *dx, const float *sx) const {
        const float d = h2f((uint16_t)(H[0] & 0xffff)), dmin = h2f((uint16_t)(H[0] >> 16));
        const uint32_t S[3] = {H[1], H[2], H[3]};
        uint32_t sc0, sc1, m0, m1;
        k4_scale_min_pair(S, c, sc0, sc1, m0, m1);
        int s0 = 0, s1 = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            s0 = dot4(Q[i] & 0x0f0f0f0fu, X[i], s0);
            s1 = dot4((Q[i] >> 4) & 0x0f0f0f0fu, X[8 + i], s1);
        }
        return d * ((float)sc0 * dx[0] * (float)s0 + (float)sc1 * dx[1] * (float)s1) -
               dmin * ((float)m0 * sx[0] + (float)m1 * sx[1]);
    }
};

// Q5_K: as Q4_K plus the 32-byte qh (bit 2c / 2c+1 of qh[l] is the 5th bit)
template <> struct Frag<T_Q5_K> {
    uint32_t H[4], QH[8], Q[8];
    int c;
    template <bool RAG>
    __device__ inline void load(const uint8_t *row, int s, int) {
        const uint8_t *p = row + (size_t)(s >> 2) * 176;
        c = s & 3;
        ld16(p, H);
        ld16(p + 16, QH);
        ld16(p + 32, QH + 4);
        ld16(p + 48 + 32 * c, Q);
        ld16(p + 64 + 32 * c, Q + 4);
    }
    __device__ inline void zero() {
        for (int i = 0; i < 4; ++i) H[i] = 0;
        for (int i = 0; i < 8; ++i) QH[i] = Q[i] = 0;
        c = 0;
    }
    __device__ inline float dot(const uint32_t X[16], const float *dx, const float *sx) const {
        const float d = h2f((uint16_t)(H[0] & 0xffff)), dmin = h2f((uint16_t)(H[0] >> 16));
        const uint32_t S[3] = {H[1], H[2], H[3]};
        uint32_t sc0, sc1, m0, m1;
        k4_scale_min_pair(S, c, sc0, sc1, m0, m1);
        int s0 = 0, s1 = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t lo = (Q[i] & 0x0f0f0f0fu) | (((QH[i] >> (2 * c)) & 0x01010101u) << 4);
            const uint32_t hi = ((Q[i] >> 4) & 0x0f0f0f0fu) | (((QH[i] >> (2 * c + 1)) & 0x01010101u) << 4);
            s0 = dot4(lo, X[i], s0);
            s1 = dot4(hi, X[8 + i], s1);
        }
        return d * ((float)sc0 * dx[0] * (float)s0 + (float)sc1 * dx[1] * (float)s1) -
               dmin * ((float)m0 * sx[0] + (float)m1 * sx[1]);
    }
};

// Q6_K: slot = (super-block sb = s/4, half h = (s/2)%2, part p = s%2); lane handles
// positions 128h + 16p + 32k + [0,16) for k = 0..3, i.e. ql[64h+16p..], ql[64h+32+16p..],
// qh[32h+16p..] and scales 8h + p + 2k; sum (q-32)*x = sum q*x - 32 sum x per 16-run.
template <> struct Frag<T_Q6_K> {
    // raw 4-byte-aligned windows, realigned in dot(): load() only issues loads, so the
    // prefetched unit stays in flight until the dot product needs it
    uint32_t R0[5], R1[5], RQ[5], RS[5];
    uint32_t sh;
    int p, h;
    // a super-block starts 2-byte aligned when sb is odd; 2-byte-misaligned 16-B loads stream
    // ~16 % slower on MI355X (scripts/hbm_probe.hip), 4-byte aligned ones at full rate, so
    // every piece is loaded from its 4-byte-aligned floor (all pieces of a block share the
    // block's alignment) and funnel-shifted into place.
    // (pointer arithmetic, not an integer round trip: a pointer rebuilt from an integer loses
    // its global address space, every load becomes a flat load, and a flat load's wait drains
    // the whole prefetch stream)
    __device__ static inline void ld20(const uint8_t *pa, uint32_t *o) {
        const uint4 w = *reinterpret_cast<const uint4 *>(pa);    // 4-B aligned dwordx4
        o[0] = w.x; o[1] = w.y; o[2] = w.z; o[3] = w.w;
        o[4] = *reinterpret_cast<const uint32_t *>(pa + 16);
    }
    __device__ static inline void al16(const uint32_t *w, uint32_t sh, uint32_t *o) {
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
    }
    template <bool RAG>
    __device__ inline void load(const uint8_t *row, int s, int) {
        const uint8_t *b = row + (size_t)(s >> 2) * 210;
        h = (s >> 1) & 1;
        p = s & 1;
        sh = (uint32_t)(reinterpret_cast<uintptr_t>(b) & 3);
        const uint8_t *ba = b - sh;
        ld20(ba + 64 * h + 16 * p, R0);
        ld20(ba + 64 * h + 32 + 16 * p, R1);
        ld20(ba + 128 + 32 * h + 16 * p, RQ);
        // the 16 scale bytes and d (bytes 192..209) in one 20-B window: the last dword ends at
        // byte 209 + (2 - sh), i.e. at most 2 bytes past the block, inside its dword
        ld20(ba + 192, RS);
    }
    __device__ inline void zero() {
        for (int i = 0; i < 5; ++i) R0[i] = R1[i] = RQ[i] = RS[i] = 0;
        sh = 0;
        p = h = 0;
    }
    // dx: d of the four 32-blocks 4h + k; sx: d*sum(q) of the four 16-runs
    __device__ inline float dot(const uint32_t X[16], const float *dx, const float *sx) const {
        uint32_t L0[4], L1[4], QH[4], SC[2];
        al16(R0, sh, L0);
        al16(R1, sh, L1);
        al16(RQ, sh, QH);
        SC[0] = __builtin_amdgcn_alignbyte(h ? RS[3] : RS[1], h ? RS[2] : RS[0], sh);
        SC[1] = __builtin_amdgcn_alignbyte(h ? RS[4] : RS[2], h ? RS[3] : RS[1], sh);
        const uint16_t dh = (uint16_t)(RS[4] >> (8 * sh));   // d: block bytes 208..209
        int s[4] = {0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const uint32_t w0 = (L0[t] & 0x0f0f0f0fu) | ((QH[t] & 0x03030303u) << 4);
            const uint32_t w1 = (L1[t] & 0x0f0f0f0fu) | ((QH[t] & 0x0c0c0c0cu) << 2);
            const uint32_t w2 = ((L0[t] >> 4) & 0x0f0f0f0fu) | (QH[t] & 0x30303030u);
            const uint32_t w3 = ((L1[t] >> 4) & 0x0f0f0f0fu) | ((QH[t] & 0xc0c0c0c0u) >> 2);
            s[0] = dot4(w0, X[t], s[0]);
            s[1] = dot4(w1, X[4 + t], s[1]);
            s[2] = dot4(w2, X[8 + t], s[2]);
            s[3] = dot4(w3, X[12 + t], s[3]);
        }
        // scales sc[8h + p + 2k]: byte (p + 2k) of the 8 loaded scale bytes
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int byte = p + 2 * k;
            const int8_t sc = (int8_t)((SC[byte >> 2] >> (8 * (byte & 3))) & 0xff);
            acc += (float)sc * __builtin_fmaf(dx[k], (float)s[k], -32.f * sx[k]);
        }
        return h2f(dh) * acc;
    }
};

template <int T> struct XdCount { static constexpr int n = 2; };
template <> struct XdCount<T_Q6_K> { static constexpr int n = 4; };

// ------------------------------------------------------------------------------------------
// butterfly-transpose reduction over groups of LPR lanes (LPR = 16 / 32 / 64, lane bits
// 0 .. log2(LPR)-1): V (power of two, <= LPR) partial sums per lane. Distances run from LPR/2
// down to 1, so the exchanges never leave the group. On return lane L holds the group's full
// sum of value index ((L % LPR) >> (log2(LPR) - log2(V))).
// ------------------------------------------------------------------------------------------
template <int x> struct Log2 { static constexpr int v = 1 + Log2<x / 2>::v; };
template <> struct Log2<1> { static constexpr int v = 0; };
constexpr int pow2ceil(int x) { return x <= 1 ? 1 : 2 * pow2ceil((x + 1) / 2); }

template <int V, int DIST, int HALF>
__device__ __forceinline__ void butterfly_step(float (&v)[V], int lane) {
    const bool upper = (lane & DIST) != 0;
#pragma unroll
    for (int i = 0; i < HALF; ++i) {
        const float send = upper ? v[i] : v[i + HALF];
        const float keep = upper ? v[i + HALF] : v[i];
        v[i] = keep + xchg<DIST>(send);
    }
}

template <int V, int LPR, int DIST>
__device__ __forceinline__ float reduce_rest(float (&v)[V], int lane, float r) {
    if constexpr (DIST == 0) {
        return r;
    } else {
        // the transposing steps consume log2(V) distances from the top; the rest plain-sum
        constexpr int STEP = Log2<LPR>::v - 1 - Log2<DIST>::v;   // 0 for DIST = LPR/2
        if constexpr (STEP < Log2<V>::v) {
            butterfly_step<V, DIST, (V >> (STEP + 1))>(v, lane);
            return reduce_rest<V, LPR, DIST / 2>(v, lane, v[0]);
        } else {
            r += xchg<DIST>(r);
            return reduce_rest<V, LPR, DIST / 2>(v, lane, r);
        }
    }
}

template <int V, int LPR>
__device__ inline float group_reduce_transpose(float (&v)[V]) {
    static_assert(V <= LPR, "more partial sums than lanes in the group");
    const int lane = threadIdx.x & 63;
    return reduce_rest<V, LPR, LPR / 2>(v, lane, v[0]);
}

// ------------------------------------------------------------------------------------------
// fused layer-norm prologue (FUSE kernels): normalizes the register-resident columns in place.
// xa/xb[m][r] hold values k0 .. k0+7 of column m, k0 = (kb0 + r*XR_STRIDE)*32 + (tid&3)*8.
// ------------------------------------------------------------------------------------------
template <int NC, int PRE>
__device__ __forceinline__ void layer_norm_cols(const MmArgs &a, int kb0, float4 (&xa)[NC][PRE], float4 (&xb)[NC][PRE],
                                                const float4 (&g)[PRE][2], const float4 (&bb)[PRE][2], const float (&shift)[NC]) {
    // one pass over the register-resident column: sums of (x - c) and (x - c)^2 with c = the
    // column's first value (so E[(x-c)^2] - E[x-c]^2 does not cancel), ONE workgroup
    // reduction. gamma / beta arrived with the activations (issued at kernel start).
    __shared__ float red[MMVQ_WAVES][NC][2];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float mean[NC], rstd[NC];
#pragma unroll
    for (int m = 0; m < NC; ++m) {
        const float c = shift[m];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int r = 0; r < PRE; ++r) {
            const int k0 = (kb0 + r * XR_STRIDE) * 32 + (threadIdx.x & 3) * 8;
            if (k0 < a.K) {
                const float v[8] = {xa[m][r].x - c, xa[m][r].y - c, xa[m][r].z - c, xa[m][r].w - c,
                                    xb[m][r].x - c, xb[m][r].y - c, xb[m][r].z - c, xb[m][r].w - c};
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    s1 += v[i];
                    s2 = __builtin_fmaf(v[i], v[i], s2);
                }
            }
        }
        s1 = wave_sum(s1);
        s2 = wave_sum(s2);
        if (lane == 0) {
            red[wave][m][0] = s1;
            red[wave][m][1] = s2;
        }
    }
    lds_barrier();   // weights stay in flight
#pragma unroll
    for (int m = 0; m < NC; ++m) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int w = 0; w < MMVQ_WAVES; ++w) {
            t1 += red[w][m][0];
            t2 += red[w][m][1];
        }
        const float d = t1 / (float)a.K;                 // E[x - c]
        mean[m] = shift[m] + d;
        const float var = fmaxf(t2 / (float)a.K - d * d, 0.f);
        rstd[m] = 1.0f / sqrtf(var + a.ln_eps);
    }
#pragma unroll
    for (int r = 0; r < PRE; ++r) {
        const int k0 = (kb0 + r * XR_STRIDE) * 32 + (threadIdx.x & 3) * 8;
        const bool in = k0 < a.K;
        const float4 g0 = g[r][0], g1 = g[r][1], b0 = bb[r][0], b1 = bb[r][1];
#pragma unroll
        for (int m = 0; m < NC; ++m) {
            const float mu = mean[m], rs = rstd[m];
            auto f = [&](float x, float gg, float b) { return in ? (x - mu) * rs * gg + b : 0.f; };
            float4 &p = xa[m][r], &q = xb[m][r];
            p = make_float4(f(p.x, g0.x, b0.x), f(p.y, g0.y, b0.y), f(p.z, g0.z, b0.z), f(p.w, g0.w, b0.w));
            q = make_float4(f(q.x, g1.x, b1.x), f(q.y, g1.y, b1.y), f(q.z, g1.z, b1.z), f(q.w, g1.w, b1.w));
        }
    }
}

// ------------------------------------------------------------------------------------------
// fused argmax epilogue (FUSE kernels, a.epi & EPI_ARGMAX): every thread offers the best
// (value, row) it stored for its column (col < 0: stored nothing); wave 0 reduces them per
// column and writes the workgroup's partial. Ties go to the lowest row (greedy sampling of
// the reference's examples take the first maximum).
// ------------------------------------------------------------------------------------------
template <int NC>
__device__ __forceinline__ void argmax_epilogue(const MmArgs &a, float bv, int bi, int col) {
    __shared__ float sv[MMVQ_THREADS];
    __shared__ int si[MMVQ_THREADS], sc[MMVQ_THREADS];
    sv[threadIdx.x] = bv;
    si[threadIdx.x] = bi;
    sc[threadIdx.x] = col;
    __syncthreads();
    if (threadIdx.x >= WAVE) return;
    const int lane = threadIdx.x;
#pragma unroll
    for (int m = 0; m < NC; ++m) {
        float v = -INFINITY;
        int i = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < MMVQ_WAVES; ++k) {
            const int t = lane + k * WAVE;
            const float tv = sv[t];
            const int ti = si[t];
            if (sc[t] == m && (tv > v || (tv == v && ti < i))) { v = tv; i = ti; }
        }
#pragma unroll
        for (int d = 1; d < WAVE; d <<= 1) {
            const float ov = __shfl_xor(v, d);
            const int oi = __shfl_xor(i, d);
            if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
        }
        if (lane == 0) {
            const int c = blockIdx.z * NC + m;
            a.amax_v[c * ARGMAX_SLOTS + blockIdx.x] = v;
            a.amax_i[c * ARGMAX_SLOTS + blockIdx.x] = i;
        }
    }
}

// ------------------------------------------------------------------------------------------
// the kernel
//   LPR : lanes per weight row (16 or 64). A wave covers 64/LPR rows side by side; a lane walks
//         K slots s = lane % LPR + it * LPR, it < n_it = ceil(nslots / LPR). Small K (GPT-2's
//         768: 12 slots) uses 16-lane rows so 75% of the lanes carry weights instead of 19%.
//   RAG : K % 64 == 32 (only possible for the 32-block types): last slot holds one block
//   XA  : src1 rows and strides are 16-byte aligned (float4 activation loads)
//
// Work: blockIdx.y selects the matrix / column group (batch entry, or (expert, token) for
// MUL_MAT_ID); the workgroup quantizes that column group into LDS ONCE, then walks row groups
// g = blockIdx.x, blockIdx.x + gridDim.x, ... (8 waves x 64/LPR x RPW rows each). Each unit of
// work = (row group, K iteration); the weights of unit u+1 are in flight while unit u is
// computed (two register buffers). The unit walk is incremental (no integer division in the
// kernel: n_it comes from the host), and a workgroup with a single unit — the single-matrix
// decode shapes — takes a straight-line path with no prefetch.
// ------------------------------------------------------------------------------------------
template <int T, int NC, int LPR, int RPW, bool IDS, bool RAG, bool XA, bool BIGK, bool FUSE = false, bool ATTN = false>
__global__ __launch_bounds__(MMVQ_THREADS) void mmvq_kernel(const MmArgs a) {
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr int NX = XdCount<T>::n;
    constexpr int V = pow2ceil(RPW * NC);
    constexpr int GPW = WAVE / LPR;                       // row groups side by side in a wave
    constexpr int ROWS_PER_WAVE = GPW * RPW;
    constexpr int ROWS_PER_GROUP = MMVQ_WAVES * ROWS_PER_WAVE;
    static_assert(V <= LPR, "RPW * NC partial sums must fit the lanes of a row");

    const int Kpad = (a.K + 63) & ~63;
    const int nslots = Kpad / 64;
    const int nblk = a.K / QT<T>::blck;           // quant blocks per row
    const int nxblk = Kpad / 32;
    const int n_it = a.n_it;                      // host: ceil(nslots / LPR)
    const XSmem sm = xsmem(smem, Kpad, NC);

    // ---- which matrix / columns this workgroup serves
    const uint8_t *wmat;
    const uint8_t *xcol0;
    uint8_t *dcol0;
    if constexpr (IDS) {
        // one (expert slot e, token t) pair per blockIdx.y, NC == 1
        const int e = blockIdx.y % a.n_used, t = blockIdx.y / a.n_used;
        int ex = *reinterpret_cast<const int32_t *>(reinterpret_cast<const uint8_t *>(a.ids) + e * a.ids_nb0 + t * a.ids_nb1);
        ex = min(max(ex, 0), a.n_expert - 1);     // host validates ids; never index out of bounds
        wmat = a.w + (int64_t)ex * a.nb02;
        xcol0 = a.x + (int64_t)(e % a.ne11_b) * a.nb11 + (int64_t)t * a.nb12;
        dcol0 = a.dst + (int64_t)e * a.nb1 + (int64_t)t * a.nb2;
    } else {
        const int i12 = blockIdx.y % a.ne12, i13 = blockIdx.y / a.ne12;
        wmat = a.w + (int64_t)(i12 / a.r2) * a.nb02 + (int64_t)(i13 / a.r3) * a.nb03;
        xcol0 = a.x + (int64_t)i12 * a.nb12 + (int64_t)i13 * a.nb13 + (int64_t)blockIdx.z * NC * a.nb11;
        dcol0 = a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3 + (int64_t)blockIdx.z * NC * a.nb1;
    }

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int sl = lane % LPR;                    // slot lane inside the row group
    const int wrow = wave * ROWS_PER_WAVE + (lane / LPR) * RPW;   // this lane's first row in a group
    const int n_groups = (a.N + ROWS_PER_GROUP - 1) / ROWS_PER_GROUP;
    const bool stamp = a.stamps != nullptr && threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0;
    if (stamp) { a.stamps[blockIdx.x * 8 + 0] = __builtin_amdgcn_s_memrealtime(); a.stamps[blockIdx.x * 8 + 4] = __builtin_amdgcn_s_memtime(); }
    // diagnostics: per-wave stamps (lane 0 of every wave of the stamped grid row)
    const bool wstamp = a.stamps != nullptr && (threadIdx.x & 63) == 0 && blockIdx.y == 0 && blockIdx.z == 0;
    unsigned long long *const wst = a.stamps + 4 * 65536 + ((int64_t)blockIdx.x * MMVQ_WAVES + (threadIdx.x >> 6)) * 4;
    if (wstamp) wst[0] = __builtin_amdgcn_s_memrealtime();

    // unit (g, it): rows g * ROWS_PER_GROUP + wrow + r, slot sl + it * LPR (clamped: dead
    // lanes / rows read valid memory and are masked out of the sums)
    auto load_unit = [&](Frag<T> (&f)[RPW], int g, int it) {
        const int r0 = g * ROWS_PER_GROUP + wrow;
        const int s = min(sl + it * LPR, nslots - 1);
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            if constexpr (MMVQ_EXP & 4) f[r].zero();
            else f[r].template load<RAG>(wmat + (int64_t)min(r0 + r, a.N - 1) * a.nb01, s, nblk);
        }
    };

    // fused epilogue operands of this lane's output (bias[row], and dst[row] for the residual
    // add), loaded with the weights of the unit so the epilogue waits on nothing. Lanes that
    // store nothing, and launches without bias / residual, re-read valid addresses.
    constexpr int ESHIFT = Log2<LPR>::v - Log2<V>::v;
    const int eidx = sl >> ESHIFT;                               // this lane's (row, column) slot
    const int er = min(eidx, RPW * NC - 1) / NC, em = min(eidx, RPW * NC - 1) % NC;
    struct EpiOps { float bias, resid; };
    auto load_epi = [&](int gg) -> EpiOps {
        const int row = min(gg * ROWS_PER_GROUP + wrow + er, a.N - 1);
        const float *bp = a.bias != nullptr ? a.bias + row : reinterpret_cast<const float *>(dcol0 + (int64_t)em * a.nb1) + row;
        EpiOps e;
        e.bias = *bp;
        e.resid = a.resid != nullptr ? reinterpret_cast<const float *>(a.resid + (int64_t)(blockIdx.z * NC + em) * a.resid_nb1)[row]
                                     : reinterpret_cast<const float *>(dcol0 + (int64_t)em * a.nb1)[row];
        return e;
    };

    // ---- activation loads of the first round first (L2/MALL hits), then the weight stream of
    // unit 0, so the quantization waits only for the activations (vmcnt is in-order) while the
    // weights stay in flight.
    // up to two rounds (K <= 8192) are preloaded; BIGK kernels loop over the rest
    const int kb0 = threadIdx.x >> 2;
    // activation rounds held in registers: 2 (K <= 8192) for narrow column groups; wide groups
    // (NC >= 4) keep one round (K <= 4096, mmvq_max_k_for_nc) so their registers stay unspilled
    constexpr int PRE = (BIGK || NC >= 4) ? 1 : 2;
    float4 xa[NC][PRE], xb[NC][PRE];
    // FUSE + attn_part: the activations are merged attention partials (K = n_embd <= 4096:
    // one round); their loads are issued here and combined after the weights
    // (80 registers of partials per column: held across the weight issue for NC <= 2 only;
    // wider column groups merge each column before the weights are issued)
    // ATTN kernels only (a template flag: the partial registers would otherwise weigh on every
    // fused instantiation's occupancy)
    static_assert(!ATTN || (FUSE && !BIGK), "attention merge is a fused-prologue variant");
    constexpr bool AP_PRE = ATTN && NC <= 2;
    constexpr int NAP = AP_PRE ? NC : 1;
    [[maybe_unused]] AttnPart ap[NAP];
    constexpr bool attn = ATTN;
    if constexpr (attn) {
        if constexpr (AP_PRE) {
#pragma unroll
            for (int m = 0; m < NAP; ++m) attn_part_load(a, (int)blockIdx.z * NC + m, kb0, ap[m]);
        } else {
#pragma unroll
            for (int m = 0; m < NC; ++m) {
                attn_part_load(a, (int)blockIdx.z * NC + m, kb0, ap[0]);
                attn_part_combine(ap[0], xa[m][0], xb[m][0]);
                if constexpr (PRE > 1) xa[m][1] = xb[m][1] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    } else {
#pragma unroll
        for (int m = 0; m < NC; ++m) {
#pragma unroll
            for (int r = 0; r < PRE; ++r) {
                if constexpr (MMVQ_EXP & 1) xa[m][r] = xb[m][r] = make_float4(1.f, 2.f, 3.f, (float)threadIdx.x);
                else xblock_load<XA>(a, xcol0 + (int64_t)m * a.nb11, kb0 + r * XR_STRIDE, xa[m][r], xb[m][r]);
            }
        }
    }

    // fused prologue operands, issued with the activations: gamma / beta of this lane's 8
    // values per round and each column's first value (the layer norm's shift). Without a layer
    // norm the loads re-read the activations (valid addresses, no branch around a load).
    // (wide column groups hold NC x PRE x 8 activations already: they load gamma / beta after
    // the weights instead of keeping 32 more registers live across the weight issue)
    [[maybe_unused]] float4 lg[PRE][2], lb[PRE][2];
    [[maybe_unused]] float lshift[NC];
    auto load_ln = [&]() {
        const bool ln = a.ln_g != nullptr;
        const float *gp = ln ? a.ln_g : reinterpret_cast<const float *>(a.x);
        const float *bp = ln ? a.ln_b : reinterpret_cast<const float *>(a.x);
#pragma unroll
        for (int r = 0; r < PRE; ++r) {
            const int kc = min((kb0 + r * XR_STRIDE) * 32 + (int)(threadIdx.x & 3) * 8, a.K - 8);
            lg[r][0] = reinterpret_cast<const float4 *>(gp + kc)[0];
            lg[r][1] = reinterpret_cast<const float4 *>(gp + kc)[1];
            lb[r][0] = reinterpret_cast<const float4 *>(bp + kc)[0];
            lb[r][1] = reinterpret_cast<const float4 *>(bp + kc)[1];
        }
#pragma unroll
        for (int m = 0; m < NC; ++m) lshift[m] = *reinterpret_cast<const float *>(xcol0 + (int64_t)m * a.nb11);
    };
    if constexpr (FUSE && NC <= 2) load_ln();

    Frag<T> fa[RPW], fb[RPW];
    int g = blockIdx.x, it = 0;                   // the unit being computed (grid.x <= n_groups)
    // issue order: every wave's activation loads ahead of every wave's weight loads. A plain
    // s_barrier (no waitcnt: gfx950 barriers do not drain memory) between the two; without it the
    // late waves' activations queue in the CU's load path behind the early waves' weights, and
    // the workgroup's quantization barrier waits for them (single 4096 x 4096 Q4_K launch:
    // activations in registers 1080 -> 720 ns after the wave's start, 5.96 -> 5.74 us; batched
    // launches within +-1 %, profiles/r06_mmvq_barrier_batched.txt). Not Q6_K: 24 stacked
    // 4096 x 11008 matrices 167-169 us with it, 164-167 without.
    if constexpr (!FUSE && T != T_Q6_K && !(MMVQ_EXP & 16)) asm volatile("s_barrier" ::: "memory");
    load_unit(fa, g, it);
    [[maybe_unused]] EpiOps ea{}, eb{};
    if constexpr (FUSE) ea = load_epi(g);
    __builtin_amdgcn_sched_barrier(0);            // ---- everything above is in flight; consume below

    if constexpr (AP_PRE) {
#pragma unroll
        for (int m = 0; m < NAP; ++m) {
            attn_part_combine(ap[m], xa[m][0], xb[m][0]);
            if constexpr (PRE > 1) xa[m][1] = xb[m][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
#pragma unroll
    for (int m = 0; m < NC; ++m)
#pragma unroll
        for (int r = 0; r < PRE; ++r) xblock_mask(a, kb0 + r * XR_STRIDE, xa[m][r], xb[m][r]);
    if (wstamp) {   // diagnostics: the activations have arrived (the mask consumed them)
        __builtin_amdgcn_sched_barrier(0);
        float probe = xa[0][0].x + xb[0][PRE - 1].w;
        asm volatile("" : "+v"(probe));
        wst[1] = __builtin_amdgcn_s_memrealtime() + (probe == 12345.f);
    }

    // fused prologue: layer norm of each column over its K values (ggml_norm, reference
    // src/ggml-cpu/ops.cpp ggml_compute_forward_norm_f32: mean, then mean of squared
    // deviations, scale 1/sqrt(var + eps)), then * g + b (ggml_mul / ggml_add). The whole
    // column is already in registers (K <= 8192, no BIGK); out-of-range values are zero.
    if constexpr (FUSE) {
        if constexpr (NC > 2) load_ln();
        if (a.ln_g != nullptr) layer_norm_cols<NC, PRE>(a, kb0, xa, xb, lg, lb, lshift);
    }

#pragma unroll
    for (int r = 0; r < PRE; ++r) {
        const int kb = kb0 + r * XR_STRIDE;
        if (kb < nxblk && !(MMVQ_EXP & 2)) {
#pragma unroll
            for (int m = 0; m < NC; ++m)
                xblock_store<T>(Kpad, kb, xa[m][r], xb[m][r], sm.xq + (size_t)m * Kpad, sm.xd + m * nxblk,
                                sm.xs + m * nxblk, sm.x16 + m * 2 * nxblk);
        }
    }
    if constexpr (BIGK) {
        for (int kb = kb0 + XR_STRIDE; kb < nxblk; kb += XR_STRIDE) {
#pragma unroll
            for (int m = 0; m < NC; ++m) {
                xblock_load<XA>(a, xcol0 + (int64_t)m * a.nb11, kb, xa[m][0], xb[m][0]);
                xblock_mask(a, kb, xa[m][0], xb[m][0]);
                xblock_store<T>(Kpad, kb, xa[m][0], xb[m][0], sm.xq + (size_t)m * Kpad, sm.xd + m * nxblk,
                                sm.xs + m * nxblk, sm.x16 + m * 2 * nxblk);
            }
        }
    }
    if (wstamp) wst[2] = __builtin_amdgcn_s_memrealtime();   // quantized, at the barrier
#ifdef MMVQ_FENCE_BARRIER   // A/B measurement builds only (scripts/ab_singles.sh)
    __syncthreads();
#else
    if constexpr (!(MMVQ_EXP & 8)) lds_barrier();
#endif
    if (stamp) a.stamps[blockIdx.x * 8 + 1] = __builtin_amdgcn_s_memrealtime();

    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    float best_v = -INFINITY;                     // EPI_ARGMAX: this lane's best stored value
    int best_i = 0x7fffffff, best_c = -1;

    auto compute_unit = [&](const Frag<T> (&f)[RPW], int gg, int itt, const EpiOps &eo) {
        const int s_raw = sl + itt * LPR;
        const int s = min(s_raw, nslots - 1);
        const float live = s_raw < nslots ? 1.f : 0.f;
        int xb0, x16b;
        if constexpr (T == T_Q6_K) {
            xb0 = 8 * (s >> 2) + 4 * ((s >> 1) & 1);
            x16b = 16 * (s >> 2) + 8 * ((s >> 1) & 1) + (s & 1);
        } else {
            xb0 = 2 * s;
            x16b = 0;
        }
#pragma unroll
        for (int m = 0; m < NC; ++m) {
            uint32_t X[16];
            const int8_t *xm = sm.xq + (size_t)m * Kpad;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint4 t4 = *reinterpret_cast<const uint4 *>(xm + (size_t)(j * nslots + s) * 16);
                X[4 * j + 0] = t4.x; X[4 * j + 1] = t4.y; X[4 * j + 2] = t4.z; X[4 * j + 3] = t4.w;
            }
            float dx[NX], sx[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) dx[i] = sm.xd[m * nxblk + xb0 + i];
            if constexpr (T == T_Q6_K) {
#pragma unroll
                for (int i = 0; i < NX; ++i) sx[i] = sm.x16[m * 2 * nxblk + x16b + 2 * i];
            } else {
#pragma unroll
                for (int i = 0; i < NX; ++i) sx[i] = sm.xs[m * nxblk + xb0 + i];
            }
#pragma unroll
            for (int r = 0; r < RPW; ++r) acc[r * NC + m] += live * f[r].dot(X, dx, sx);
        }
        // last K iteration of this row group: reduce across the row's lanes and store
        if (itt == n_it - 1) {
            const float sum = group_reduce_transpose<V, LPR>(acc);
            constexpr int SHIFT = Log2<LPR>::v - Log2<V>::v;
            const int idx = sl >> SHIFT;
            const int r0 = gg * ROWS_PER_GROUP + wrow;
            if ((sl & ((1 << SHIFT) - 1)) == 0 && idx < RPW * NC) {
                const int r = idx / NC, m = idx % NC;
                if (r0 + r < a.N) {
                    float *out = reinterpret_cast<float *>(dcol0 + (int64_t)m * a.nb1) + r0 + r;
                    float v = sum;
                    if constexpr (FUSE) {
                        // fused epilogue, in ggml's node order: + bias, gelu, + residual
                        // (operands prefetched with the unit's weights: eo)
                        if (a.bias != nullptr) v += eo.bias;
                        if (a.epi & EPI_GELU) v = gelu_ggml(v);
                        if (a.epi & EPI_RESID) v += eo.resid;
                        if (a.epi & EPI_ARGMAX) {
                            if (v > best_v || best_c < 0) { best_v = v; best_i = r0 + r; }   // rows ascend per lane
                            best_c = m;
                        }
#pragma unroll
                        for (int cpi = 0; cpi < 2; ++cpi) {   // copy-out (graph_compute's cache writes)
                            const unsigned cr = (unsigned)(r0 + r - a.cp_r0[cpi]);
                            if (a.cp_dst[cpi] != nullptr && cr < (unsigned)a.cp_n[cpi])
                                reinterpret_cast<float *>(reinterpret_cast<uint8_t *>(a.cp_dst[cpi]) +
                                                          (int64_t)(blockIdx.z * NC + m) * a.cp_nb1[cpi])[cr] = v;
                        }
                    }
                    *out = v;
                }
            }
#pragma unroll
            for (int i = 0; i < V; ++i) acc[i] = 0.f;
        }
    };

    // next unit after (g, it); uniform scalar arithmetic
    int ng = g, nit = it + 1;
    if (nit == n_it) { nit = 0; ng += gridDim.x; }
    if (ng >= n_groups) {
        // single unit per workgroup (e.g. a 4096-row matrix at K <= 4096): no prefetch at all
        compute_unit(fa, g, it, ea);
        if (wstamp) wst[3] = __builtin_amdgcn_s_memrealtime();   // diagnostics: dots stored
    } else {
        // prefetches are unconditional (clamped to the current unit once the walk ends: a
        // repeat of addresses already in flight, served on-chip) so the load stream never sits
        // under a branch; sched_barrier pins each prefetch ahead of the compute that follows it
        // (left alone, the scheduler sinks the loads below the compute to save registers and
        // the overlap is lost)
        for (;;) {
            bool more = ng < n_groups;
            load_unit(fb, more ? ng : g, more ? nit : it);
            if constexpr (FUSE) eb = load_epi(more ? ng : g);
            __builtin_amdgcn_sched_barrier(0);
            compute_unit(fa, g, it, ea);
            if (!more) break;
            g = ng; it = nit;
            if (++nit == n_it) { nit = 0; ng += gridDim.x; }
            more = ng < n_groups;
            load_unit(fa, more ? ng : g, more ? nit : it);
            if constexpr (FUSE) ea = load_epi(more ? ng : g);
            __builtin_amdgcn_sched_barrier(0);
            compute_unit(fb, g, it, eb);
            if (!more) break;
            g = ng; it = nit;
            if (++nit == n_it) { nit = 0; ng += gridDim.x; }
        }
    }
    if constexpr (FUSE) {
        if (a.epi & EPI_ARGMAX) argmax_epilogue<NC>(a, best_v, best_i, best_c);
    }
    if (stamp) { a.stamps[blockIdx.x * 8 + 2] = a.stamps[blockIdx.x * 8 + 3] = __builtin_amdgcn_s_memrealtime(); a.stamps[blockIdx.x * 8 + 5] = __builtin_amdgcn_s_memtime(); }
}

}  // namespace mi355x
