// mmvq_mma.hip — the quantized mat-vec for 2..16 src1 columns on the int8 matrix cores.
//
// The reference streams the weights once for up to 8 columns with per-column dp4a dot products
// (mul_mat_vec_q<type, ncols_dst>, src/ggml-cuda/mmvq.cu:139-226). On gfx950 the per-column VALU
// dots (mmvq_impl.h / mmvq_ring.hip) grow with the column count, and so do the LDS reads of the
// quantized columns, which every wave re-reads: at 8 columns a CU spends as long on them as on
// its share of the weight stream, and the two do not overlap (profiles/r05_ring_depth_ab.txt:
// 8 columns take 2.2x one column at K = 14336). Here the columns are the N side of
// v_mfma_i32_16x16x32_i8 and the weight rows its M side:
//
//  * one 32-weight block (Q4_0 / Q8_0) or 32-weight sub-block (K-quants) = one MFMA K step;
//    the integer dot of 16 rows x 16 columns is one instruction, the block scales are applied
//    to its int32 results in fp32 (per block, as ggml-cpu's vec_dot does);
//  * a wave owns 16 weight rows and a contiguous range of K; lane (r = l & 15, g = l >> 4)
//    loads row r's bytes for k-group g, straight to registers (no LDS staging of weights);
//    Q4_0 / Q8_0 lanes load one whole block each and a 4 x 4 transpose across the lanes of a
//    row (two permlane swaps) hands every lane its k-group of all four blocks;
//  * the columns were quantized once per call by mma_prequant into the B-fragment order
//    (int8 per 32-block, d = amax/127, round-to-nearest-even, exactly as the other mat-vec
//    kernels), so lane (t, g) reads its 4 blocks of column t as 32 contiguous bytes;
//  * the row scales reach the output lanes (column t, rows 4G..4G+3) through a 256-B per-wave
//    LDS slot; the K ranges of a workgroup's waves are summed through LDS in a fixed order.
//
// A workgroup = KS waves on the same 16 rows (KS = 4, 8 or 16, so that the grid holds ~16
// waves per CU at any N); MUL_MAT batch slices on grid.y.
#include <type_traits>

#include "mmvq_impl.h"

namespace mi355x {

typedef int i32x4_t __attribute__((ext_vector_type(4)));

constexpr int MMA_STEP_K = 128;   // K per step: 4 MFMA K steps of 32

// activation image of one (slice, step), one record per column t: codes [g 4][j 4][8 B] (int8,
// the B-fragment byte order of the type), d [4] f32, and for Q4_K / Q5_K d * sum(q) [4] f32.
// The record stride (144 / 160 B) also spreads the columns' 16-B LDS reads over distinct banks.
template <int T> __host__ __device__ constexpr int mma_rec_bytes() { return (T == T_Q4_K || T == T_Q5_K) ? 160 : 144; }
template <int T, int TOK> __host__ __device__ constexpr int mma_step_bytes() { return TOK * mma_rec_bytes<T>(); }

// element of a 32-block held by byte i (0..7) of k-group g: Q4_0 pairs each nibble byte's low
// and high halves (byte 4g + i holds elements 4g + i and 4g + i + 16), the others are in order
template <int T> __device__ __forceinline__ int mma_elem(int g, int i) {
    if constexpr (T == T_Q4_0) return i < 4 ? 4 * g + i : 4 * g + 12 + i;
    else return 8 * g + i;
}

// grid (steps, slices), TOK * 16 threads: thread (t, j, g) quantizes k-group g of block j of
// column t; the quad of a block shares amax and sum(q) through DPP
template <int T, int TOK>
__global__ __launch_bounds__(TOK * 16) void mma_prequant(const MmArgs a, uint8_t *__restrict__ img) {
    const int s = blockIdx.x, z = blockIdx.y;
    const int i12 = z % a.ne12, i13 = z / a.ne12;
    const int g = threadIdx.x & 3, j = (threadIdx.x >> 2) & 3, t = threadIdx.x >> 4;
    const int kb = s * MMA_STEP_K + 32 * j;   // first element of the block
    const float *col = reinterpret_cast<const float *>(a.x + (int64_t)i12 * a.nb12 + (int64_t)i13 * a.nb13 +
                                                       (int64_t)min(t, a.M - 1) * a.nb11);
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int k = kb + mma_elem<T>(g, i);
        const float x = col[min(k, a.K - 1)];
        v[i] = (k < a.K && t < a.M) ? x : 0.f;
    }
    // the quantization of mmvq_impl.h's xblock_store, bit for bit
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
    amax = fmaxf(amax, dpp_f<DPP_XOR1>(amax));
    amax = fmaxf(amax, dpp_f<DPP_XOR2>(amax));
    const float d = amax * (1.0f / 127.f);
    const float id = amax > 0.f ? 127.f * __builtin_amdgcn_rcpf(amax) : 0.f;
    constexpr float MAGIC = 12582912.0f + 128.0f;
    uint32_t b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = __float_as_uint(__builtin_fmaf(v[i], id, MAGIC));
    const uint32_t w0 = __builtin_amdgcn_perm(__builtin_amdgcn_perm(b[3], b[2], 0x0c0c0400u), __builtin_amdgcn_perm(b[1], b[0], 0x0c0c0400u), 0x05040100u);
    const uint32_t w1 = __builtin_amdgcn_perm(__builtin_amdgcn_perm(b[7], b[6], 0x0c0c0400u), __builtin_amdgcn_perm(b[5], b[4], 0x0c0c0400u), 0x05040100u);
    const int qs = (int)__builtin_amdgcn_udot4(w0, 0x01010101u, __builtin_amdgcn_udot4(w1, 0x01010101u, 0u, false), false) - 1024;
    float fs = (float)qs;
    fs += dpp_f<DPP_XOR1>(fs);
    fs += dpp_f<DPP_XOR2>(fs);
    uint8_t *rec = img + ((int64_t)z * gridDim.x + s) * mma_step_bytes<T, TOK>() + t * mma_rec_bytes<T>();
    *reinterpret_cast<uint2 *>(rec + g * 32 + j * 8) = make_uint2(w0 ^ 0x80808080u, w1 ^ 0x80808080u);
    if (g == 0) {
        float *ds = reinterpret_cast<float *>(rec + 128);
        ds[j] = d;
        if constexpr (mma_rec_bytes<T>() == 160) ds[4 + j] = d * fs;
    }
}

// ------------------------------------------------------------------------------------------
// per-type weight fragment of one step for lane (row r, k-group g)
//   load  : issue the loads (no use of the data: the next step's loads stay in flight)
//   frags : the 8 int8 weights of k-group g of every MFMA of the step
//   sc   : the row scale(s) this lane publishes for the epilogue
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void swap32(uint32_t &lo_src, uint32_t &hi_dst) {
    // upper 32 lanes of hi_dst <-> lower 32 lanes of lo_src
    const auto r = __builtin_amdgcn_permlane32_swap(hi_dst, lo_src, false, false);
    hi_dst = r[0];
    lo_src = r[1];
}
__device__ __forceinline__ void swap16(uint32_t &even_src, uint32_t &odd_dst) {
    // odd 16-lane rows of odd_dst <-> even rows of even_src
    const auto r = __builtin_amdgcn_permlane16_swap(odd_dst, even_src, false, false);
    odd_dst = r[0];
    even_src = r[1];
}
// 4 x 4 transpose across the lanes g = 0..3 of a row: lane g ends with q[j] = lane j's q[g]
__device__ __forceinline__ void transpose4(uint32_t (&q)[4]) {
    swap32(q[2], q[0]);
    swap32(q[3], q[1]);
    swap16(q[1], q[0]);
    swap16(q[3], q[2]);
}
__device__ __forceinline__ long pack2(uint32_t lo, uint32_t hi) { return (long)(((uint64_t)hi << 32) | lo); }

// An empty volatile asm that "modifies" a loaded register: arithmetic on the value cannot be
// placed before it, and a volatile asm keeps its place after the scheduling barrier. Without it
// the selection DAG hoists a step's MFMAs (which only read registers) next to their loads, above
// the barrier that issues the following step's loads first, and the wait for them drains both.
template <typename V> __device__ __forceinline__ void pin(V &v) {
    static_assert(sizeof(V) % 4 == 0, "dword registers");
    uint32_t *u = reinterpret_cast<uint32_t *>(&v);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(V) / 4); ++i) asm volatile("" : "+v"(u[i]));
}

template <int T> struct MmaW;

// Q4_0: lane g loads block 4s + g of its row (a 20-byte window from the dword floor)
template <> struct MmaW<T_Q4_0> {
    static constexpr int NMF = 4, NSC = 1;
    uint32_t W[5];
    uint32_t sh;
    __device__ inline void load(const uint8_t *row, int s, int g, int nblk) {
        const uint8_t *p = row + (size_t)min(4 * s + g, nblk - 1) * 18;
        sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
        const uint8_t *pa = p - sh;
        const uint4 w = *reinterpret_cast<const uint4 *>(pa);
        W[0] = w.x; W[1] = w.y; W[2] = w.z; W[3] = w.w;
        W[4] = *reinterpret_cast<const uint32_t *>(pa + 16);
    }
    __device__ inline void frags(long (&A)[NMF]) {
        pin(W);
        uint32_t q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = sh ? W[k + 1] : align2(W[k + 1], W[k]);
        transpose4(q);
#pragma unroll
        for (int j = 0; j < 4; ++j) A[j] = pack2(sub8_bytes(q[j] & 0x0f0f0f0fu), sub8_bytes((q[j] >> 4) & 0x0f0f0f0fu));
    }
    __device__ inline void sc(float *o) const { o[0] = h2f((uint16_t)(W[0] >> (8 * sh))); }
};

// Q8_0: lane g loads block 4s + g (a 36-byte window); k-group g' = qs dwords 2g', 2g'+1
template <> struct MmaW<T_Q8_0> {
    static constexpr int NMF = 4, NSC = 1;
    uint32_t W[9];
    uint32_t sh;
    __device__ inline void load(const uint8_t *row, int s, int g, int nblk) {
        const uint8_t *p = row + (size_t)min(4 * s + g, nblk - 1) * 34;
        sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
        const uint8_t *pa = p - sh;
        const uint4 w0 = *reinterpret_cast<const uint4 *>(pa);
        const uint4 w1 = *reinterpret_cast<const uint4 *>(pa + 16);
        W[0] = w0.x; W[1] = w0.y; W[2] = w0.z; W[3] = w0.w;
        W[4] = w1.x; W[5] = w1.y; W[6] = w1.z; W[7] = w1.w;
        W[8] = *reinterpret_cast<const uint32_t *>(pa + 32);
    }
    __device__ inline void frags(long (&A)[NMF]) {
        pin(W);
        uint32_t qe[4], qo[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            qe[k] = sh ? W[2 * k + 1] : align2(W[2 * k + 1], W[2 * k]);
            qo[k] = sh ? W[2 * k + 2] : align2(W[2 * k + 2], W[2 * k + 1]);
        }
        transpose4(qe);
        transpose4(qo);
#pragma unroll
        for (int j = 0; j < 4; ++j) A[j] = pack2(qe[j], qo[j]);
    }
    __device__ inline void sc(float *o) const { o[0] = h2f((uint16_t)(W[0] >> (8 * sh))); }
};

// Q4_K: step s = half h = s & 1 of super-block s >> 1: sub-blocks 4h .. 4h+3 are the low / high
// nibbles of qs chunks 2h and 2h+1; lane g loads its 8 bytes of each chunk and the 16-B header
template <> struct MmaW<T_Q4_K> {
    static constexpr int NMF = 4, NSC = 2;
    uint32_t H[4], QA[2], QB[2];
    int h;
    __device__ inline void load(const uint8_t *row, int s, int g, int) {
        const uint8_t *p = row + (size_t)(s >> 1) * 144;
        h = s & 1;
        ld16(p, H);
        ld8(p + 16 + 64 * h + 8 * g, QA);
        ld8(p + 48 + 64 * h + 8 * g, QB);
    }
    __device__ inline void frags(long (&A)[NMF]) {
        pin(H);
        pin(QA);
        pin(QB);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t *Q = j < 2 ? QA : QB;
            const int shf = (j & 1) * 4;
            A[j] = pack2((Q[0] >> shf) & 0x0f0f0f0fu, (Q[1] >> shf) & 0x0f0f0f0fu);
        }
    }
    // d * sc and dmin * m of sub-block 4h + g
    __device__ inline void sc(float *o, int g) const {
        const uint32_t S[3] = {H[1], H[2], H[3]};
        uint32_t sc0, sc1, m0, m1;
        k4_scale_min_pair(S, 2 * h + (g >> 1), sc0, sc1, m0, m1);
        const float d = h2f((uint16_t)(H[0] & 0xffff)), dmin = h2f((uint16_t)(H[0] >> 16));
        o[0] = d * (float)(g & 1 ? sc1 : sc0);
        o[1] = dmin * (float)(g & 1 ? m1 : m0);
    }
};

// Q5_K: as Q4_K plus the 5th bits: qh byte 8g + i, bit (4h + j) for sub-block 4h + j
template <> struct MmaW<T_Q5_K> {
    static constexpr int NMF = 4, NSC = 2;
    uint32_t H[4], QH[2], QA[2], QB[2];
    int h;
    __device__ inline void load(const uint8_t *row, int s, int g, int) {
        const uint8_t *p = row + (size_t)(s >> 1) * 176;
        h = s & 1;
        ld16(p, H);
        ld8(p + 16 + 8 * g, QH);
        ld8(p + 48 + 64 * h + 8 * g, QA);
        ld8(p + 80 + 64 * h + 8 * g, QB);
    }
    __device__ inline void frags(long (&A)[NMF]) {
        pin(H);
        pin(QH);
        pin(QA);
        pin(QB);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t *Q = j < 2 ? QA : QB;
            const int shf = (j & 1) * 4, hb = 4 * h + j;
            const uint32_t lo = ((Q[0] >> shf) & 0x0f0f0f0fu) | (((QH[0] >> hb) & 0x01010101u) << 4);
            const uint32_t hi = ((Q[1] >> shf) & 0x0f0f0f0fu) | (((QH[1] >> hb) & 0x01010101u) << 4);
            A[j] = pack2(lo, hi);
        }
    }
    __device__ inline void sc(float *o, int g) const {
        const uint32_t S[3] = {H[1], H[2], H[3]};
        uint32_t sc0, sc1, m0, m1;
        k4_scale_min_pair(S, 2 * h + (g >> 1), sc0, sc1, m0, m1);
        const float d = h2f((uint16_t)(H[0] & 0xffff)), dmin = h2f((uint16_t)(H[0] >> 16));
        o[0] = d * (float)(g & 1 ? sc1 : sc0);
        o[1] = dmin * (float)(g & 1 ? m1 : m0);
    }
};

// Q6_K: step s = half h of super-block s >> 1; sub-block q of the half: low 4 bits from
// ql[64h + 32 (q & 1) + l] (nibble q >> 1), high 2 bits from qh[32h + l] >> 2q; scales per 16
// (k-groups 0-1 / 2-3), so each sub-block is two MFMAs with the other run's weights zeroed
// (dequantize_row_q6_K, reference src/ggml-quants.c:1762)
template <> struct MmaW<T_Q6_K> {
    static constexpr int NMF = 8, NSC = 2;
    // 4-byte-aligned windows from the dword floor of the (2-byte aligned) super-block, as
    // mmvq_impl.h's Frag<Q6_K>: ql (two 12-B windows), qh (12 B), scales + d (20 B)
    uint32_t L0[3], L1[3], QH[3], RS[5];
    uint32_t sh;
    int h, g;
    __device__ static inline void ld12(const uint8_t *pa, uint32_t *o) {
        const uint2 w = *reinterpret_cast<const uint2 *>(pa);
        o[0] = w.x; o[1] = w.y;
        o[2] = *reinterpret_cast<const uint32_t *>(pa + 8);
    }
    __device__ inline void load(const uint8_t *row, int s, int g_, int) {
        const uint8_t *p = row + (size_t)(s >> 1) * 210;
        h = s & 1;
        g = g_;
        sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
        const uint8_t *pa = p - sh;
        ld12(pa + 64 * h + 8 * g, L0);
        ld12(pa + 64 * h + 32 + 8 * g, L1);
        ld12(pa + 128 + 32 * h + 8 * g, QH);
        const uint4 w = *reinterpret_cast<const uint4 *>(pa + 192);
        RS[0] = w.x; RS[1] = w.y; RS[2] = w.z; RS[3] = w.w;
        RS[4] = *reinterpret_cast<const uint32_t *>(pa + 208);
    }
    __device__ inline void frags(long (&A)[NMF]) {
        pin(L0);
        pin(L1);
        pin(QH);
        pin(RS);
        uint32_t l0[2], l1[2], qh[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            l0[k] = __builtin_amdgcn_alignbyte(L0[k + 1], L0[k], sh);
            l1[k] = __builtin_amdgcn_alignbyte(L1[k + 1], L1[k], sh);
            qh[k] = __builtin_amdgcn_alignbyte(QH[k + 1], QH[k], sh);
        }
        // MFMA m = 2 q + run; this lane's k-group belongs to run g >> 1, the other run is zero
#pragma unroll
        for (int m = 0; m < NMF; ++m) {
            const int q = m >> 1, run = m & 1;
            const uint32_t keep = 0u - (uint32_t)(run == (g >> 1));   // (a mask, not a branch)
            const uint32_t *L = (q & 1) ? l1 : l0;
            const int shf = (q >> 1) * 4, hs = 2 * q;
            const uint32_t lo = ((L[0] >> shf) & 0x0f0f0f0fu) | (((qh[0] >> hs) & 0x03030303u) << 4);
            const uint32_t hi = ((L[1] >> shf) & 0x0f0f0f0fu) | (((qh[1] >> hs) & 0x03030303u) << 4);
            A[m] = pack2(sub32_bytes(lo) & keep, sub32_bytes(hi) & keep);
        }
    }
    // d * sc[8h + 2g + run] for run 0, 1 (sub-block q = g): bytes sh + 8h + 2g of the scale window
    __device__ inline void sc(float *o, int) const {
        const uint32_t ob = sh + 8 * h + 2 * g;   // even, <= 16: both bytes in one dword
        const uint32_t wi = ob >> 2;
        const uint32_t wd = wi == 0 ? RS[0] : wi == 1 ? RS[1] : wi == 2 ? RS[2] : wi == 3 ? RS[3] : RS[4];
        const uint32_t sc2 = wd >> (8 * (ob & 3));
        const float d = h2f((uint16_t)(RS[4] >> (8 * sh)));
        o[0] = d * (float)(int8_t)(sc2 & 0xff);
        o[1] = d * (float)(int8_t)((sc2 >> 8) & 0xff);
    }
};

// ------------------------------------------------------------------------------------------
// weight sets per wave (DEPTH - 1 steps in flight). XL (the slice's activation image copied to
// LDS once per workgroup): the sets hold only weights, so they go deep; otherwise the sets hold
// the activation fragments too, 2 deep.
template <int T, bool XL> __host__ __device__ constexpr int mma_depth() {
    if constexpr (!XL) return 2;
    else return T == T_Q4_0 ? 6 : (T == T_Q8_0 || T == T_Q4_K) ? 4 : T == T_Q5_K ? 3 : 2;
}

// Workgroup = KS waves on one 16-row tile at a time, each wave a contiguous K range of it
// (persistent over tiles when XL: the image is copied once); the row scales reach the output
// lanes through a per-wave LDS slot; the K ranges are summed through LDS in a fixed order.
template <int T, int TOK, int KS, bool XL>
__global__ __launch_bounds__(KS * WAVE) void mmvq_mma_kernel(const MmArgs a, const uint8_t *__restrict__ img, int n_steps,
                                                           int n_tiles) {
    constexpr int NMF = MmaW<T>::NMF;
    constexpr int NSC = MmaW<T>::NSC;
    constexpr int RB = mma_rec_bytes<T>();
    constexpr int SB = mma_step_bytes<T, TOK>();
    constexpr int D = mma_depth<T, XL>();
    constexpr bool SX = RB == 160;
    extern __shared__ __align__(16) uint8_t xsm[];   // XL: n_steps * SB bytes
    // per wave: the row scales of the step being finished, [row 16][4 j][NSC] floats; the K-split
    // partial sums of the live lanes (column < TOK) [wave][g 4][t TOK][4]
    __shared__ __align__(16) float wsc[KS][16 * 4 * NSC];
    __shared__ __align__(16) float red[KS][4 * TOK * 4];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane & 15, g = lane >> 4;
    const int z = blockIdx.y;
    const int i12 = z % a.ne12, i13 = z / a.ne12;
    const uint8_t *wmat = a.w + (int64_t)(i12 / a.r2) * a.nb02 + (int64_t)(i13 / a.r3) * a.nb03;
    const int nblk = a.K / QT<T>::blck;
    const uint8_t *xs = img + (int64_t)z * n_steps * SB;
    const int tl = r & (TOK - 1);   // this lane's column (lanes past TOK repeat a column)
    const int s0 = (int)((int64_t)wave * n_steps / KS), s1 = (int)((int64_t)(wave + 1) * n_steps / KS);
    const uint8_t *xsrc = XL ? xsm : xs;   // (generic pointer: global or LDS)

    struct Xf {
        uint4 c0, c1;   // codes of 4 blocks (8 B each)
        float4 d, sx;   // d and d * sum(q) of the 4 blocks, this lane's column
    };
    auto read_x = [&](Xf &x, int s) __attribute__((always_inline)) {
        if constexpr (XL) {
            const uint8_t *rec = xsm + s * SB + tl * RB;
            x.c0 = *reinterpret_cast<const uint4 *>(rec + g * 32);
            x.c1 = *reinterpret_cast<const uint4 *>(rec + g * 32 + 16);
            x.d = *reinterpret_cast<const float4 *>(rec + 128);
            if constexpr (SX) x.sx = *reinterpret_cast<const float4 *>(rec + 144);
        } else {
            const uint8_t *rec = xs + (int64_t)s * SB + tl * RB;
            x.c0 = *reinterpret_cast<const uint4 *>(rec + g * 32);
            x.c1 = *reinterpret_cast<const uint4 *>(rec + g * 32 + 16);
            x.d = *reinterpret_cast<const float4 *>(rec + 128);
            if constexpr (SX) x.sx = *reinterpret_cast<const float4 *>(rec + 144);
        }
    };
    (void)xsrc;
    float acc[4];
    auto compute = [&](MmaW<T> &w, Xf &x, float live) __attribute__((always_inline)) {
        long A[NMF];
        w.frags(A);
        pin(x.c0);
        pin(x.c1);
        pin(x.d);
        if constexpr (SX) pin(x.sx);
        const long xb[4] = {pack2(x.c0.x, x.c0.y), pack2(x.c0.z, x.c0.w), pack2(x.c1.x, x.c1.y), pack2(x.c1.z, x.c1.w)};
        i32x4_t R[NMF];
        const i32x4_t zero = {0, 0, 0, 0};
#pragma unroll
        for (int m = 0; m < NMF; ++m) R[m] = __builtin_amdgcn_mfma_i32_16x16x32_i8(A[m], xb[NMF == 8 ? m >> 1 : m], zero, 0, 0, 0);
        // publish this lane's row scales: [r][j = g][NSC]
        float o[NSC];
        if constexpr (NSC == 1) w.sc(o);
        else w.sc(o, g);
        float *ws = wsc[wave];
#pragma unroll
        for (int k = 0; k < NSC; ++k) ws[(r * 4 + g) * NSC + k] = o[k];
        // read the scales of rows 4G + i (G = g): 4 * NSC floats per row
        const float xd[4] = {x.d.x, x.d.y, x.d.z, x.d.w};
        // (the padding step's live = 0 is applied to its finished sums: a factor on the loaded
        // scales would be hoisted next to their loads, and its wait would drain the prefetch)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float c;
            const float *rs = ws + (4 * g + i) * 4 * NSC;
            if constexpr (T == T_Q4_0 || T == T_Q8_0) {
                const float4 dw = *reinterpret_cast<const float4 *>(rs);
                c = (dw.x * xd[0]) * (float)R[0][i] + (dw.y * xd[1]) * (float)R[1][i] +
                    (dw.z * xd[2]) * (float)R[2][i] + (dw.w * xd[3]) * (float)R[3][i];
            } else if constexpr (T == T_Q6_K) {
                const float4 lo = *reinterpret_cast<const float4 *>(rs), hi = *reinterpret_cast<const float4 *>(rs + 4);
                // [q][run]: lo = q0r0 q0r1 q1r0 q1r1, hi = q2r0 q2r1 q3r0 q3r1
                c = xd[0] * (lo.x * (float)R[0][i] + lo.y * (float)R[1][i]) +
                    xd[1] * (lo.z * (float)R[2][i] + lo.w * (float)R[3][i]) +
                    xd[2] * (hi.x * (float)R[4][i] + hi.y * (float)R[5][i]) +
                    xd[3] * (hi.z * (float)R[6][i] + hi.w * (float)R[7][i]);
            } else {
                const float4 lo = *reinterpret_cast<const float4 *>(rs), hi = *reinterpret_cast<const float4 *>(rs + 4);
                // [j][sc, m]: lo = sc0 m0 sc1 m1, hi = sc2 m2 sc3 m3
                const float sx[4] = {x.sx.x, x.sx.y, x.sx.z, x.sx.w};
                c = (lo.x * (xd[0] * (float)R[0][i]) - lo.y * sx[0]) + (lo.z * (xd[1] * (float)R[1][i]) - lo.w * sx[1]) +
                    (hi.x * (xd[2] * (float)R[2][i]) - hi.y * sx[2]) + (hi.z * (xd[3] * (float)R[3][i]) - hi.w * sx[3]);
            }
            acc[i] = __builtin_fmaf(live, c, acc[i]);
        }
    };

    bool copied = !XL;
    for (int tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int row0 = tile * 16;
        const uint8_t *wrow = wmat + (int64_t)min(row0 + r, a.N - 1) * a.nb01;
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = 0.f;
        // DEPTH - 1 steps in flight per wave: step s computes from set s % DEPTH while the loads
        // of s + DEPTH - 1 go into the set step s - 1 used (clamped repeats past s1 - 1). A CU's
        // whole weight stream is the steps its waves hold in flight (a wave owns a few steps of
        // ~1 KiB each), so the depth sets the bandwidth. The step count is padded to a multiple
        // of DEPTH with repeats that add nothing (live = 0): no exit inside the unrolled body.
        // The scheduling barriers keep each step's loads ahead of the previous step's
        // arithmetic, with pin() (see there) keeping that arithmetic behind them.
        MmaW<T> F[D];
        Xf X[D];
        const bool work = s1 > s0;
        if (work) {
#pragma unroll
            for (int d = 0; d < D - 1; ++d) {
                F[d].load(wrow, min(s0 + d, s1 - 1), g, nblk);
                if constexpr (!XL) read_x(X[d], min(s0 + d, s1 - 1));
            }
        }
        if (!copied) {   // XL, first tile: the slice's image into LDS behind the weight prologue
            const uint4 *src = reinterpret_cast<const uint4 *>(xs);
            uint4 *dst = reinterpret_cast<uint4 *>(xsm);
            const int n16 = n_steps * SB / 16;
            constexpr int B = 8;   // loads issued before the writes that wait for them
            for (int i0 = threadIdx.x; i0 < n16; i0 += B * KS * WAVE) {
                uint4 v[B];
#pragma unroll
                for (int b = 0; b < B; ++b) v[b] = src[min(i0 + b * KS * WAVE, n16 - 1)];
#pragma unroll
                for (int b = 0; b < B; ++b) dst[min(i0 + b * KS * WAVE, n16 - 1)] = v[b];   // (clamped: a repeat of the last)
            }
            lds_barrier();
            copied = true;
        }
        if (work) {
            const int n_pad = (s1 - s0 + D - 1) / D * D;
            auto step = [&](auto k_c, int s) __attribute__((always_inline)) {
                constexpr int k = decltype(k_c)::value;
                const int sl = min(s + D - 1, s1 - 1);
                F[(k + D - 1) % D].load(wrow, sl, g, nblk);
                if constexpr (!XL) read_x(X[(k + D - 1) % D], sl);
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (XL) read_x(X[k], min(s, s1 - 1));
                compute(F[k], X[k], s < s1 ? 1.f : 0.f);
            };
            for (int it = 0; it < n_pad; it += D) {
                const int s = s0 + it;
                step(std::integral_constant<int, 0>{}, s);
                if constexpr (D > 1) step(std::integral_constant<int, 1 % D>{}, s + 1);
                if constexpr (D > 2) step(std::integral_constant<int, 2 % D>{}, s + 2);
                if constexpr (D > 3) step(std::integral_constant<int, 3 % D>{}, s + 3);
                if constexpr (D > 4) step(std::integral_constant<int, 4 % D>{}, s + 4);
                if constexpr (D > 5) step(std::integral_constant<int, 5 % D>{}, s + 5);
            }
        }
        // K-split reduction over the waves, fixed order (live lanes: column t < TOK)
        if (r < TOK) {
#pragma unroll
            for (int i = 0; i < 4; ++i) red[wave][(g * TOK + r) * 4 + i] = acc[i];
        }
        lds_barrier();
        if (wave == 0 && r < TOK) {
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = red[0][(g * TOK + r) * 4 + i];
#pragma unroll
            for (int w = 1; w < KS; ++w)
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] += red[w][(g * TOK + r) * 4 + i];
            if (r < a.M) {
                float *dst = reinterpret_cast<float *>(a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3 + (int64_t)r * a.nb1);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = row0 + 4 * g + i;
                    if (row < a.N) dst[row] = v[i];
                }
            }
        }
        lds_barrier();   // (red is rewritten by the next tile)
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
static int mma_steps(const MmArgs &a) { return (a.K + MMA_STEP_K - 1) / MMA_STEP_K; }

template <int T> static size_t img_bytes_t(const MmArgs &a) {
    return (size_t)mma_steps(a) * (a.M <= 8 ? mma_step_bytes<T, 8>() : mma_step_bytes<T, 16>()) * a.ne12 * a.ne13;
}

size_t mmvq_mma_img_bytes(int type, const MmArgs &a) {
    switch (type) {
        case T_Q4_0: return img_bytes_t<T_Q4_0>(a);
        case T_Q8_0: return img_bytes_t<T_Q8_0>(a);
        case T_Q4_K: return img_bytes_t<T_Q4_K>(a);
        case T_Q5_K: return img_bytes_t<T_Q5_K>(a);
        case T_Q6_K: return img_bytes_t<T_Q6_K>(a);
        default: return 0;
    }
}

template <int T, int TOK, int KS, bool XL>
static hipError_t mma_launch_k(const MmArgs &a, uint8_t *img, int S, int tiles, int slices, size_t xl_bytes, hipStream_t st) {
    const void *kern = reinterpret_cast<const void *>(mmvq_mma_kernel<T, TOK, KS, XL>);
    if constexpr (XL) {
        static bool attr_set = false;   // per instantiation; set only once the call succeeded
        if (!attr_set) {
            hipFuncAttributes fa{};
            hipError_t e = hipFuncGetAttributes(&fa, kern);
            if (e == hipSuccess) e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(160 * 1024 - fa.sharedSizeBytes));
            if (e != hipSuccess) {
                (void)hipGetLastError();
                return e;
            }
            attr_set = true;
        }
    }
    // XL: one workgroup per CU, persistent over the slice's tiles (the image copy is paid once)
    const int gx = XL ? std::max(1, std::min(tiles, 256 / std::max(1, slices))) : tiles;
    hipLaunchKernelGGL((mmvq_mma_kernel<T, TOK, KS, XL>), dim3(gx, slices), dim3(KS * WAVE), XL ? xl_bytes : 0, st, a,
                       (const uint8_t *)img, S, tiles);
    return hipGetLastError();
}

template <int T, int TOK>
static hipError_t mma_tok(const MmArgs &a, uint8_t *img, hipStream_t st) {
    const int S = mma_steps(a);
    const int slices = a.ne12 * a.ne13;
    const int tiles = (a.N + 15) / 16;
    hipLaunchKernelGGL((mma_prequant<T, TOK>), dim3(S, slices), dim3(TOK * 16), 0, st, a, img);
    // ~16 waves per CU over the whole grid; never more waves than steps
    const char *kse = getenv("GGML_MI355X_MMA_KS");   // per call: tests switch it
    const int ks_env = kse ? atoi(kse) : 0;
    const int64_t waves_per_tile = std::max<int64_t>(1, (256 * 16) / ((int64_t)tiles * slices));
    int ks = ks_env > 0 ? ks_env : waves_per_tile >= 16 ? 16 : waves_per_tile >= 8 ? 8 : 4;
    while (ks > 4 && ks > S) ks >>= 1;
    if (T == T_Q6_K && ks > 8) ks = 8;   // (its fragments need more than the 128 VGPRs of 16 waves)
    // the image in LDS when it fits beside the static arrays (<= 16 KiB); GGML_MI355X_MMA_XL=0: never
    const char *xle = getenv("GGML_MI355X_MMA_XL");
    const size_t xl_bytes = (size_t)S * mma_step_bytes<T, TOK>();
    // (not Q6_K: its deeper fragment sets spill)
    const bool xl = T != T_Q6_K && !(xle && atoi(xle) == 0) && xl_bytes <= 144 * 1024;
    // XL: 8 waves per workgroup (one per CU, persistent): the deep weight sets need the 256
    // VGPRs of 2 waves per SIMD; 16 waves would spill them
    if (xl) return ks >= 8 ? mma_launch_k<T, TOK, 8, true>(a, img, S, tiles, slices, xl_bytes, st)
                           : mma_launch_k<T, TOK, 4, true>(a, img, S, tiles, slices, xl_bytes, st);
    if (ks >= 16 && (T == T_Q4_0 || T == T_Q8_0))   // (the K-quants' sets spill at 16 waves)
        return mma_launch_k<T, TOK, 16, false>(a, img, S, tiles, slices, xl_bytes, st);
    if (ks >= 8) return mma_launch_k<T, TOK, 8, false>(a, img, S, tiles, slices, xl_bytes, st);
    return mma_launch_k<T, TOK, 4, false>(a, img, S, tiles, slices, xl_bytes, st);
}

template <int T>
static hipError_t mma_type(const MmArgs &a, uint8_t *img, hipStream_t st) {
    return a.M <= 8 ? mma_tok<T, 8>(a, img, st) : mma_tok<T, 16>(a, img, st);
}

// plain MUL_MAT with 1 <= M <= 16 columns, img = mmvq_mma_img_bytes(type, a) of scratch
hipError_t mmvq_mma_launch(int type, const MmArgs &a, uint8_t *img, hipStream_t st) {
    if (a.M < 1 || a.M > 16 || img == nullptr) return hipErrorInvalidValue;
    switch (type) {
        case T_Q4_0: return mma_type<T_Q4_0>(a, img, st);
        case T_Q8_0: return mma_type<T_Q8_0>(a, img, st);
        case T_Q4_K: return mma_type<T_Q4_K>(a, img, st);
        case T_Q5_K: return mma_type<T_Q5_K>(a, img, st);
        case T_Q6_K: return mma_type<T_Q6_K>(a, img, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mi355x
