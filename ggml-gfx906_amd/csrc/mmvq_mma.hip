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

// measurement builds only (scripts/mma_exp.sh; results wrong by design): bit 1 = no activation
// loads (the records quantize zeros), bit 2 = no weight loads, bit 4 = no K-part hand-off
#ifndef MMA_EXP
#define MMA_EXP 0
#endif

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

// k-group g of block j of step s of column t (zeros past K or M), loaded, then quantized into
// its record `rec` (the record of (s, t)); the 4 threads of a block (g = 0..3) are consecutive
// lanes and share amax and sum(q) through DPP. The arithmetic of mmvq_impl.h's xblock_store,
// bit for bit.
// (the loads only: the zeroing past K / M is applied by mma_quant once every load of the batch
// is issued; a select right behind a load makes the compiler wait for it before the next load)
template <int T, bool XA>
__device__ __forceinline__ void mma_xload(const MmArgs &a, const float *col, int s, int j, int g, float (&v)[8]) {
    const int kb = s * MMA_STEP_K + 32 * j;   // first element of the block
    if constexpr (XA) {   // rows 16-B aligned, K % 4 == 0 (runs of 4 clamped as a whole)
        const float4 lo = *reinterpret_cast<const float4 *>(col + min(kb + mma_elem<T>(g, 0), a.K - 4));
        const float4 hi = *reinterpret_cast<const float4 *>(col + min(kb + mma_elem<T>(g, 4), a.K - 4));
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
        v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = col[min(kb + mma_elem<T>(g, i), a.K - 1)];
    }
}
template <int T, bool SX>
__device__ __forceinline__ void mma_quant(const MmArgs &a, float (&v)[8], int s, int j, int t, int g, uint8_t *rec, bool store) {
    const int kb = s * MMA_STEP_K + 32 * j;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (kb + mma_elem<T>(g, i) < a.K && t < a.M) ? v[i] : 0.f;
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
    if (store) *reinterpret_cast<uint2 *>(rec + g * 32 + j * 8) = make_uint2(w0 ^ 0x80808080u, w1 ^ 0x80808080u);
    float fs = 0.f;
    if constexpr (SX) {
        const int qs = (int)__builtin_amdgcn_udot4(w0, 0x01010101u, __builtin_amdgcn_udot4(w1, 0x01010101u, 0u, false), false) - 1024;
        fs = (float)qs;
        fs += dpp_f<DPP_XOR1>(fs);
        fs += dpp_f<DPP_XOR2>(fs);
    }
    if (g == 0 && store) {
        float *ds = reinterpret_cast<float *>(rec + 128);
        ds[j] = d;
        if constexpr (SX) ds[4 + j] = d * fs;
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
// weight sets per wave (DEPTH - 1 steps in flight; the activations come from LDS): as deep as
// the register budget of 16 waves per CU allows without spills
template <int T> __host__ __device__ constexpr int mma_depth() {
    return T == T_Q4_0 ? 5 : (T == T_Q8_0 || T == T_Q4_K) ? 3 : 2;
}

// One launch, no pre-pass. Workgroup (row group rg, K part kp, slice z) = 8 waves, wave w on the
// 16-row tile 8 rg + w, all waves over the same K part:
//  1. the workgroup quantizes its K part of the src1 columns into LDS (records of mma_quant),
//     while the first weight steps of every wave are already in flight;
//  2. each wave streams its tile's weights over the K part, DEPTH - 1 steps ahead in registers,
//     one MFMA per 32-block against the LDS records;
//  3. with one K part the wave stores its tile; otherwise it stores a partial (write-through
//     sc1 stores), the workgroup adds one to its row group's counter (agent scope) and the
//     workgroup that arrives last sums the parts in K order and stores dst
//     (MI355X_MICROARCH.md inter-workgroup visibility, the counter row), then re-arms it.
template <int D, typename F, int... Is>
__device__ __forceinline__ void mma_run_steps(F &&f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is % D>{}, Is), ...);
}

template <int T, int TOK, int D, int NSTEP, bool XA>
__global__ __launch_bounds__(8 * WAVE) void mmvq_mma_kernel(const MmArgs a, int n_steps, int n_kp, float *__restrict__ part,
                                                          int *__restrict__ cnt) {
    constexpr int NMF = MmaW<T>::NMF;
    constexpr int NSC = MmaW<T>::NSC;
    constexpr int RB = mma_rec_bytes<T>();
    constexpr int SB = mma_step_bytes<T, TOK>();
    constexpr bool SX = RB == 160;
    extern __shared__ __align__(16) uint8_t xsm[];   // the K part's records: steps * SB bytes
    __shared__ __align__(16) float wsc[8][16 * 4 * NSC];
    __shared__ int order;

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane & 15, g = lane >> 4;
    const int rg = blockIdx.x, kp = blockIdx.y, z = blockIdx.z;
    const int i12 = z % a.ne12, i13 = z / a.ne12;
    const int k0 = kp * NSTEP, k1 = min(n_steps, k0 + NSTEP);   // this K part's steps (NSTEP per part)
    const int tile = rg * 8 + wave;
    const int row0 = tile * 16;
    const uint8_t *wrow = a.w + (int64_t)(i12 / a.r2) * a.nb02 + (int64_t)(i13 / a.r3) * a.nb03 +
                          (int64_t)min(row0 + r, a.N - 1) * a.nb01;
    const int nblk = a.K / QT<T>::blck;
    const int tl = r & (TOK - 1);   // this lane's column (lanes past TOK repeat a column)

    // 1. weight prologue, then the K part's activations into LDS (16-B loads: the 8 values of a
    // unit are two runs of 4 consecutive floats in either element order)
    MmaW<T> F[D];
#pragma unroll
    for (int d = 0; d < D - 1; ++d)
        if constexpr (!(MMA_EXP & 2)) F[d].load(wrow, min(k0 + d, k1 - 1), g, nblk);
    {
        const float *xz = reinterpret_cast<const float *>(a.x + (int64_t)i12 * a.nb12 + (int64_t)i13 * a.nb13);
        const int units = (k1 - k0) * 4 * TOK * 4;   // (step, t, j, g), g fastest
        constexpr int QU = 4;   // units per thread whose loads are issued together
        for (int u0 = threadIdx.x; u0 < units; u0 += QU * 8 * WAVE) {
            float v[QU][8];
#pragma unroll
            for (int q = 0; q < QU; ++q) {
                const int u = min(u0 + q * 8 * WAVE, units - 1);
                const int j = (u >> 2) & 3, t = (u >> 4) % TOK, sl = (u >> 4) / TOK;
                const float *col = reinterpret_cast<const float *>(reinterpret_cast<const uint8_t *>(xz) + (int64_t)min(t, a.M - 1) * a.nb11);
                if constexpr (MMA_EXP & 1) {
                    for (int c = 0; c < 8; ++c) v[q][c] = 0.f;
                    (void)col;
                } else {
                    mma_xload<T, XA>(a, col, k0 + sl, j, u & 3, v[q]);
                }
            }
#pragma unroll
            for (int q = 0; q < QU; ++q) {
                // (units past the end, whole quads since units % 4 == 0, quantize the clamped
                // repeat without storing it: a quad of repeats has the wrong amax)
                const int u = min(u0 + q * 8 * WAVE, units - 1);
                const int j = (u >> 2) & 3, t = (u >> 4) % TOK, sl = (u >> 4) / TOK;
                mma_quant<T, SX>(a, v[q], k0 + sl, j, t, u & 3, xsm + sl * SB + t * RB, u0 + q * 8 * WAVE < units);
            }
        }
    }
    lds_barrier();

    // 2. the weight stream: step s computes from set s % D while the loads of s + D - 1 go into
    // the set step s - 1 used (clamped repeats past k1 - 1); the step count is padded to a
    // multiple of D with repeats that add nothing (live = 0). The scheduling barriers keep each
    // step's loads ahead of the previous step's arithmetic, pin() keeps that arithmetic behind.
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    auto compute = [&](MmaW<T> &w, int s, float live) __attribute__((always_inline)) {
        long A[NMF];
        w.frags(A);
        const uint8_t *rec = xsm + (s - k0) * SB + tl * RB;
        const uint4 c0 = *reinterpret_cast<const uint4 *>(rec + g * 32);
        const uint4 c1 = *reinterpret_cast<const uint4 *>(rec + g * 32 + 16);
        const float4 xdv = *reinterpret_cast<const float4 *>(rec + 128);
        float4 sxv = {0.f, 0.f, 0.f, 0.f};
        if constexpr (SX) sxv = *reinterpret_cast<const float4 *>(rec + 144);
        const long xb[4] = {pack2(c0.x, c0.y), pack2(c0.z, c0.w), pack2(c1.x, c1.y), pack2(c1.z, c1.w)};
        i32x4_t R[NMF];
        const i32x4_t zero = {0, 0, 0, 0};
#pragma unroll
        for (int m = 0; m < NMF; ++m) R[m] = __builtin_amdgcn_mfma_i32_16x16x32_i8(A[m], xb[NMF == 8 ? m >> 1 : m], zero, 0, 0, 0);
        // publish this lane's row scales [r][j = g][NSC]; read those of rows 4G + i (G = g)
        float o[NSC];
        if constexpr (NSC == 1) w.sc(o);
        else w.sc(o, g);
        float *ws = wsc[wave];
#pragma unroll
        for (int k = 0; k < NSC; ++k) ws[(r * 4 + g) * NSC + k] = o[k];
        const float xd[4] = {xdv.x, xdv.y, xdv.z, xdv.w};
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
                c = (lo.x * (xd[0] * (float)R[0][i]) - lo.y * sxv.x) + (lo.z * (xd[1] * (float)R[1][i]) - lo.w * sxv.y) +
                    (hi.x * (xd[2] * (float)R[2][i]) - hi.y * sxv.z) + (hi.z * (xd[3] * (float)R[3][i]) - hi.w * sxv.w);
            }
            acc[i] = __builtin_fmaf(live, c, acc[i]);
        }
    };
    // straight-line: NSTEP steps (the last part's steps past k1 are clamped repeats with
    // live = 0), no loop, so no register set crosses a back-edge (the copies the register
    // allocator puts on a back-edge move sets whose loads are still in flight, and each copy
    // waits for its load: one memory latency per step)
    auto step = [&](auto k_c, int i) __attribute__((always_inline)) {
        constexpr int k = decltype(k_c)::value;
        const int s = k0 + i;
        if constexpr (!(MMA_EXP & 2))
            if (i + D - 1 < NSTEP) F[(k + D - 1) % D].load(wrow, min(s + D - 1, k1 - 1), g, nblk);
        __builtin_amdgcn_sched_barrier(0);
        compute(F[k], min(s, k1 - 1), s < k1 ? 1.f : 0.f);
    };
    mma_run_steps<D>(step, std::make_integer_sequence<int, NSTEP>{});

    // 3. store (live lanes: column t < TOK, rows 4G + i)
    const bool live_lane = r < TOK;
    float *dcol = reinterpret_cast<float *>(a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3 + (int64_t)r * a.nb1);
    if (n_kp == 1 || (MMA_EXP & 4)) {
        if (live_lane && r < a.M)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (row0 + 4 * g + i < a.N) dcol[row0 + 4 * g + i] = acc[i];
        return;
    }
    // partial of (slice, K part, tile): [lane (g, t < TOK)][4] floats
    const int n_tiles8 = gridDim.x * 8;
    auto slot = [&](int k) { return part + (((int64_t)z * n_kp + k) * n_tiles8 + tile) * (TOK * 4 * 4) + (g * TOK + tl) * 4; };
    if (live_lane) {
        float *p = slot(kp);
#pragma unroll
        for (int i = 0; i < 4; ++i) __hip_atomic_store(p + i, acc[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
    lds_barrier();
    int *c = cnt + (int64_t)z * gridDim.x + rg;
    if (threadIdx.x == 0) order = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lds_barrier();
    if (order != n_kp - 1) return;   // (uniform) a later workgroup finishes the row group
    if (live_lane) {
        // the parts in K order, loads of 8 parts issued before their sums (one latency per 8)
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        for (int k0p = 0; k0p < n_kp; k0p += 8) {
            float pv[8][4];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float *p = slot(min(k0p + k, n_kp - 1));
#pragma unroll
                for (int i = 0; i < 4; ++i) pv[k][i] = __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] += k0p + k < n_kp ? pv[k][i] : 0.f;
        }
        if (r < a.M)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (row0 + 4 * g + i < a.N) dcol[row0 + 4 * g + i] = v[i];
    }
    if (threadIdx.x == 0) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
static int mma_steps(const MmArgs &a) { return (a.K + MMA_STEP_K - 1) / MMA_STEP_K; }

// K parts of NSTEP steps: 8 (1024 K) when that still gives ~2 workgroups per CU over the grid
// (row groups x slices x parts), else 4
static int mma_nstep(const MmArgs &a) {
    const int S = mma_steps(a);
    const int64_t groups = (a.N + 127) / 128, slices = (int64_t)a.ne12 * a.ne13;
    const char *e = getenv("GGML_MI355X_MMA_NSTEP");   // per call: tests switch it
    if (e) return atoi(e) <= 4 ? 4 : 8;
    return groups * slices * ((S + 7) / 8) >= 384 ? 8 : 4;
}

template <int T, int TOK> static void mma_geometry(const MmArgs &a, int &groups, int &n_kp, size_t &lds) {
    const int S = mma_steps(a);
    const int ns = mma_nstep(a);
    groups = (a.N + 127) / 128;
    n_kp = (S + ns - 1) / ns;
    lds = (size_t)ns * mma_step_bytes<T, TOK>();
}

size_t mmvq_mma_part_bytes(int type, const MmArgs &a) {
    int groups = 0, n_kp = 1;
    size_t lds = 0;
    const bool t8 = a.M <= 8;
    switch (type) {
        case T_Q4_0: t8 ? mma_geometry<T_Q4_0, 8>(a, groups, n_kp, lds) : mma_geometry<T_Q4_0, 16>(a, groups, n_kp, lds); break;
        case T_Q8_0: t8 ? mma_geometry<T_Q8_0, 8>(a, groups, n_kp, lds) : mma_geometry<T_Q8_0, 16>(a, groups, n_kp, lds); break;
        case T_Q4_K: t8 ? mma_geometry<T_Q4_K, 8>(a, groups, n_kp, lds) : mma_geometry<T_Q4_K, 16>(a, groups, n_kp, lds); break;
        case T_Q5_K: t8 ? mma_geometry<T_Q5_K, 8>(a, groups, n_kp, lds) : mma_geometry<T_Q5_K, 16>(a, groups, n_kp, lds); break;
        default: return 0;
    }
    if (n_kp == 1) return 0;
    // [slice][part][tile][g 4][t TOK][4] floats
    return (size_t)a.ne12 * a.ne13 * n_kp * groups * 8 * (t8 ? 8 : 16) * 16 * sizeof(float);
}

template <int T, int TOK>
static hipError_t mma_tok(const MmArgs &a, float *part, int *cnt, hipStream_t st) {
    int groups = 0, n_kp = 1;
    size_t lds = 0;
    mma_geometry<T, TOK>(a, groups, n_kp, lds);
    const int slices = a.ne12 * a.ne13;
    if (n_kp > 1 && (part == nullptr || cnt == nullptr || (int64_t)groups * slices > 16384)) return hipErrorInvalidValue;
    const char *de = getenv("GGML_MI355X_MMA_D");   // measurements: 2 = one step ahead
    const bool d2 = de && atoi(de) == 2;
    const bool n8 = mma_nstep(a) == 8;
    const dim3 grid(groups, n_kp, slices);
    const int S = mma_steps(a);
    // (16-B activation loads when the rows are 16-B aligned; K is a multiple of 32 for every type)
#define MMA_GO(DV, NS)                                                                                                \
    if (a.x_aligned16) hipLaunchKernelGGL((mmvq_mma_kernel<T, TOK, DV, NS, true>), grid, dim3(8 * WAVE), lds, st, a, S, n_kp, part, cnt); \
    else hipLaunchKernelGGL((mmvq_mma_kernel<T, TOK, DV, NS, false>), grid, dim3(8 * WAVE), lds, st, a, S, n_kp, part, cnt)
    if (d2) {
        if (n8) MMA_GO(2, 8);
        else MMA_GO(2, 4);
    } else {
        if (n8) MMA_GO(mma_depth<T>(), 8);
        else MMA_GO(mma_depth<T>(), 4);
    }
#undef MMA_GO
    return hipGetLastError();
}

template <int T>
static hipError_t mma_type(const MmArgs &a, float *part, int *cnt, hipStream_t st) {
    return a.M <= 8 ? mma_tok<T, 8>(a, part, cnt, st) : mma_tok<T, 16>(a, part, cnt, st);
}

// plain MUL_MAT with 1 <= M <= 16 columns. part: mmvq_mma_part_bytes(type, a) bytes of scratch
// (nullptr when that is 0), cnt: zeroed counters (Scratch::counters) when part is set
hipError_t mmvq_mma_launch(int type, const MmArgs &a, float *part, int *cnt, hipStream_t st) {
    if (a.M < 1 || a.M > 16) return hipErrorInvalidValue;
    switch (type) {
        case T_Q4_0: return mma_type<T_Q4_0>(a, part, cnt, st);
        case T_Q8_0: return mma_type<T_Q8_0>(a, part, cnt, st);
        case T_Q4_K: return mma_type<T_Q4_K>(a, part, cnt, st);
        case T_Q5_K: return mma_type<T_Q5_K>(a, part, cnt, st);
        default: return hipErrorInvalidValue;   // (Q6_K: its eight MFMAs per step spill; the VALU kernels take it)
    }
}

}  // namespace mi355x
