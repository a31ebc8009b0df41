// mmvq_mma.hip — the quantized mat-vec for 1..8 src1 columns on the int8 matrix cores.
//
// The reference streams the weights once for up to 8 columns with per-column dp4a dot products
// (mul_mat_vec_q<type, ncols_dst>, src/ggml-cuda/mmvq.cu:139-226). On gfx950 the per-column VALU
// dots (mmvq_impl.h / mmvq_ring.hip) grow with the column count: at 8 columns a CU spends as
// long on them as on its share of the weight stream (profiles/r05_ring_depth_ab.txt: 8 columns
// take 2.2x one column at K = 14336). Here the dots run on v_mfma_i32_16x16x32_i8, weight rows
// on its M side, and the VALU only unpacks weights and applies the block scales.
//
// An MFMA's 16 columns would leave most of the scale work on padding columns (a lane owns 4
// outputs of one column; at 4 tokens 12 of 16 columns are empty). So the columns are packed
// block-diagonally: with TOK tokens, column c holds token c % TOK of block group c / TOK, and
// the 32-wide contraction is split into 16 / TOK ranges, one per block group; each lane's
// B fragment is zero outside its group's range. Every output is then a (row, token, block)
// dot, and the scale epilogue does no padding work:
//
//  * TOK = 4 (1..4 columns): 4 blocks per MFMA, 8 K of each; 4 MFMAs make a step of 4 blocks
//    (128 K) and lane (row r, k-group g) owns block g of row r for the whole step;
//  * TOK = 8 (5..8 columns): 2 blocks per MFMA, 16 K of each; two pairs of MFMAs per step,
//    lane g holds half g & 1 of block g >> 1 of the pair (Q4_0 / Q8_0: a permlane exchange of
//    the halves of the blocks the lanes loaded whole; K-quants: each lane loads its own qs run's
//    half and trades the other run's half with lane g ^ 2);
//  * the B fragments come from the columns' images (int8 per 32-block, d = amax / 127,
//    round-to-nearest-even, exactly as the other mat-vec kernels), quantized once per call by
//    mma_prequant and staged per workgroup in LDS; lanes outside their group's range read a
//    zero region after the image;
//  * the row scales reach the output lanes through a per-wave LDS slot; Q4_0 codes stay
//    unsigned (0..15) and the - 8 comes back through d * sum(q) of the column block;
//  * a workgroup = RT 16-row tiles sharing the column fragments x one of KH K parts, 16 waves
//    striding its steps in straight-line code; the block groups are summed across lanes (DPP),
//    the waves through LDS in a fixed order, and two K parts add into the zeroed dst (two terms:
//    order-free), so results repeat bit for bit;
//  * weight loads go through a per-step buffer descriptor (scalar base, per-lane constant
//    offsets; steps past K have no records, so they read zeros); the number of load
//    instructions per step is what bounds the kernel, so Q4_0 / Q8_0 at long K
//    load two adjacent blocks per lane for two steps at once (paired steps), and Q4_K at long K
//    and 1..4 columns loads a super-block's qs row-contiguously and permutes it (MmaPair<T_Q4_K>);
//  * Q6_K has a scale per 16 weights: one MFMA chain per 16-element half of a block (MmaW<T_Q6_K>).
#include <type_traits>

// measurement builds only (scripts/mma_exp.sh; results wrong by design): bit 1 = no activation
// loads (pre-pass and records), bit 2 = no weight loads, bit 4 = Q4_K weight loads reading 8 rows x
// 128 contiguous bytes per instruction (scripts/gpu_r06_rowc.sh)
#ifndef MMA_EXP
#define MMA_EXP 0
#endif

#include "mmvq_impl.h"
#include "settings.h"

#include <string>

namespace mi355x {

typedef int i32x4_t __attribute__((ext_vector_type(4)));

constexpr int MMA_STEP_K = 128;   // K per step: 4 blocks of 32
constexpr int MMA_KS = 16;        // waves per workgroup
constexpr uint32_t MMA_RSRC_W3 = 0x00020000u;   // raw buffer descriptor dword 3 (as mmq8.hip)

// activation image of one (slice, step): codes [t TOK][block 4][32 B] in chunk order, then
// [t][block] {d, d * sum(q)} f32
template <int TOK> __host__ __device__ constexpr int mma_step_bytes() { return TOK * 160; }

// element of a 32-block at byte i (0..7) of chunk m (0..3): chunks 0 / 1 are elements 0..7 /
// 16..23, chunks 2 / 3 are 8..15 / 24..31, so a chunk pair {2a, 2a + 1} is the low and high
// nibbles of Q4_0 qs bytes 8a .. 8a + 7 (and of a K-quant's 32-byte qs run)
__host__ __device__ constexpr int mma_elem(int m, int i) { return 8 * (m >> 1) + 16 * (m & 1) + i; }

// chunk m of block j of step s of column t (zeros past K or M), loaded, quantized and stored into
// the step's image; the 4 threads of a block are consecutive lanes and share amax and sum(q)
// through DPP. The arithmetic of mmvq_impl.h's xblock_store, bit for bit.
// (the loads only: the zeroing past K / M is applied by mma_quant once every load of the batch
// is issued; a select right behind a load makes the compiler wait for it before the next load)
template <bool XA>
__device__ __forceinline__ void mma_xload(const MmArgs &a, const float *col, int s, int j, int m, float (&v)[8]) {
    const int k0 = s * MMA_STEP_K + 32 * j + mma_elem(m, 0);   // 8 consecutive elements
    if constexpr (XA) {   // rows 16-B aligned, K % 4 == 0 (runs of 4 clamped as a whole)
        const float4 lo = *reinterpret_cast<const float4 *>(col + min(k0, a.K - 4));
        const float4 hi = *reinterpret_cast<const float4 *>(col + min(k0 + 4, a.K - 4));
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
        v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = col[min(k0 + i, a.K - 1)];
    }
}
template <int TOK>
__device__ __forceinline__ void mma_quant(const MmArgs &a, float (&v)[8], int s, int j, int t, int m, uint8_t *step) {
    const int k0 = s * MMA_STEP_K + 32 * j + mma_elem(m, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (k0 + i < a.K && t < a.M) ? v[i] : 0.f;
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
    *reinterpret_cast<uint2 *>(step + (t * 4 + j) * 32 + m * 8) = make_uint2(w0 ^ 0x80808080u, w1 ^ 0x80808080u);
    const int qs = (int)__builtin_amdgcn_udot4(w0, 0x01010101u, __builtin_amdgcn_udot4(w1, 0x01010101u, 0u, false), false) - 1024;
    float fs = (float)qs;
    fs += dpp_f<DPP_XOR1>(fs);
    fs += dpp_f<DPP_XOR2>(fs);
    if (m == 0) *reinterpret_cast<float2 *>(step + TOK * 128 + (t * 4 + j) * 8) = make_float2(d, d * fs);
}

// ------------------------------------------------------------------------------------------
// helpers
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

constexpr uint32_t NIB = 0x0f0f0f0fu;

// Q4_0 / Q8_0 with 8 tokens: lane g loaded block g whole; lane g needs half g & 1 of block
// 2p + (g >> 1) for pair p. With X = the lane's lower half and Y = its upper half (n dwords
// each), two swaps leave pair 0's half in X and pair 1's in Y:
//   X = L0 L1 L2 L3, Y = H0 H1 H2 H3  --swap16-->  X = L0 H0 L2 H2, Y = L1 H1 L3 H3
//                                     --swap32-->  X = L0 H0 L1 H1, Y = L2 H2 L3 H3
template <int n> __device__ __forceinline__ void halves_to_pairs(uint32_t (&X)[n], uint32_t (&Y)[n]) {
#pragma unroll
    for (int k = 0; k < n; ++k) {
        swap16(Y[k], X[k]);
        swap32(Y[k], X[k]);
    }
}

typedef uint32_t mma_u4 __attribute__((ext_vector_type(4)));
typedef uint32_t mma_u2 __attribute__((ext_vector_type(2)));
typedef float mma_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void bl16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t *o) {
    const mma_u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3];
}
__device__ __forceinline__ void bl8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t *o) {
    const mma_u2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    o[0] = v[0]; o[1] = v[1];
}

// K-quants with 8 tokens: lane g loaded half g & 1 of qs run 2h + (g >> 1); pair p needs half
// g & 1 of run 2h + p. Lanes g and g ^ 2 (32 apart) trade their own halves: afterwards X holds
// run 2h's half and Y run 2h + 1's on every lane.
__device__ __forceinline__ void runs_to_pairs(const uint32_t (&own)[4], uint32_t (&X)[4], uint32_t (&Y)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        X[k] = own[k];
        Y[k] = own[k];
        swap32(Y[k], X[k]);   // upper lanes' X <- lower lanes' own, lower lanes' Y <- upper lanes' own
    }
}

// ------------------------------------------------------------------------------------------
// per-type weights of one step for lane (row r, k-group g), loaded through a per-step buffer
// descriptor (base = the tile at the step's first byte; no records at all for a step past K,
// so those loads return zeros) at offsets fixed per lane:
//   lanes : the lane's offsets in the tile (row r, k-group g, half h of a K-quant super-block)
//   load  : issue the loads (no use of the data: the next steps' loads stay in flight)
//   frags : A[p][q], the int8 weights of MFMA q of pair p (TOK 4: p = 0, q = chunk of the
//           lane's block; TOK 8: q = chunk 2 (g & 1) + q of block 2p + (g >> 1))
//   sc    : the scale(s) of block g of the step (sub-block 4h + g for the K-quants)
// Q4_0 / Q8_0 blocks are 2-byte aligned: their qs come from a dword-aligned window and a
// per-lane funnel shift (unaligned 16-byte loads cost about twice the memory-pipeline time).
// ------------------------------------------------------------------------------------------
struct MmaLanes {
    uint32_t a, b, c;
};
template <int T, int TOK> struct MmaW;

template <int TOK> struct MmaW<T_Q4_0, TOK> {
    static constexpr int NSC = 1;
    uint32_t V[5], d;
    int h;   // (unused)
    __device__ static uint32_t step_off(int s) { return 72u * s; }
    // a = the block, b = the dword floor of its qs (a 20-byte window), c = the qs offset in it
    __device__ static MmaLanes lanes(int r, int g, int, uint32_t nb01, uint32_t mis) {
        const uint32_t blk = r * nb01 + 18u * g, o = (mis + blk + 2) & 3;
        return {blk, blk + 2 - o, o};
    }
    __device__ inline void load(__amdgpu_buffer_rsrc_t rs, const MmaLanes &lo) {
        bl16(rs, lo.b, V);
        // (the window's last dword is only used for its low 2 bytes, the block's last two: a 2-byte
        // load keeps the tensor's last block inside the descriptor's range)
        V[4] = __builtin_amdgcn_raw_buffer_load_b16(rs, lo.a + 16, 0, 0);
        d = __builtin_amdgcn_raw_buffer_load_b16(rs, lo.a, 0, 0);
    }
    __device__ inline void frags(long (&A)[4], int, const MmaLanes &lo) {
        pin(V);
        uint32_t q[4];   // qs dwords
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = __builtin_amdgcn_alignbyte(V[k + 1], V[k], lo.c);
        frags_q(q, A);
    }
    // A fragments from the block's 16 qs bytes (lane g owns block g of the step)
    __device__ static inline void frags_q(const uint32_t (&q)[4], long (&A)[4]) {
        if constexpr (TOK == 4) {
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int a = m >> 1, sft = 4 * (m & 1);
                A[m] = pack2((q[2 * a] >> sft) & NIB, (q[2 * a + 1] >> sft) & NIB);
            }
        } else {
            uint32_t X[2] = {q[0], q[1]}, Y[2] = {q[2], q[3]};
            halves_to_pairs(X, Y);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                A[h] = pack2((X[0] >> (4 * h)) & NIB, (X[1] >> (4 * h)) & NIB);
                A[2 + h] = pack2((Y[0] >> (4 * h)) & NIB, (Y[1] >> (4 * h)) & NIB);
            }
        }
    }
    __device__ inline void sc(float *o, int) {
        pin(d);
        o[0] = h2f((uint16_t)d);
    }
};

// Q8_0: chunk m = qs dwords 2 (m >> 1) + 4 (m & 1)
template <int TOK> struct MmaW<T_Q8_0, TOK> {
    static constexpr int NSC = 1;
    uint32_t V[9], d;
    int h;   // (unused)
    __device__ static uint32_t step_off(int s) { return 136u * s; }
    __device__ static MmaLanes lanes(int r, int g, int, uint32_t nb01, uint32_t mis) {
        const uint32_t blk = r * nb01 + 34u * g, o = (mis + blk + 2) & 3;
        return {blk, blk + 2 - o, o};
    }
    __device__ inline void load(__amdgpu_buffer_rsrc_t rs, const MmaLanes &lo) {
        bl16(rs, lo.b, V);
        bl16(rs, lo.b + 16, V + 4);
        V[8] = __builtin_amdgcn_raw_buffer_load_b16(rs, lo.a + 32, 0, 0);   // (as Q4_0)
        d = __builtin_amdgcn_raw_buffer_load_b16(rs, lo.a, 0, 0);
    }
    __device__ inline void frags(long (&A)[4], int, const MmaLanes &lo) {
        pin(V);
        uint32_t q[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = __builtin_amdgcn_alignbyte(V[k + 1], V[k], lo.c);
        frags_q(q, A);
    }
    __device__ static inline void frags_q(const uint32_t (&q)[8], long (&A)[4]) {
        if constexpr (TOK == 4) {
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int o = 2 * (m >> 1) + 4 * (m & 1);
                A[m] = pack2(q[o], q[o + 1]);
            }
        } else {
            // half a = chunks 2a, 2a + 1 = dwords {2a, 2a + 1, 2a + 4, 2a + 5}
            uint32_t X[4] = {q[0], q[1], q[4], q[5]}, Y[4] = {q[2], q[3], q[6], q[7]};
            halves_to_pairs(X, Y);
            A[0] = pack2(X[0], X[1]);
            A[1] = pack2(X[2], X[3]);
            A[2] = pack2(Y[0], Y[1]);
            A[3] = pack2(Y[2], Y[3]);
        }
    }
    __device__ inline void sc(float *o, int) {
        pin(d);
        o[0] = h2f((uint16_t)d);
    }
};

// Q4_K: step s = half h = s & 1 of super-block s >> 1 (h is the wave's: s = wave + 16 i); sub-block
// 4h + b is nibble b & 1 of qs run 2h + (b >> 1) (32 B at 16 + 32 (2h + (b >> 1))); every lane
// loads the 16-B header.
//   TOK 4: lane g loads the 32-B run of its sub-block g;
//   TOK 8: lane g loads bytes 8 (g & 1) + 16 q .. + 8 (q = 0, 1) of run 2h + p for both pairs
// K-quant runs: lanes g and g ^ 1 (adjacent 16-lane rows) each load one 16-byte half of a 32-byte
// run and trade the other half by one permlane16 swap per dword.
// whole run (4 tokens): both lanes want all 32 bytes. With A = B = the lane's own half, the swap
// leaves B = bytes 0..15 and A = bytes 16..31 on both lanes (the even lane's B and the odd lane's
// A are their own halves, the others the partner's).
__device__ __forceinline__ void run_whole(const uint32_t (&own)[4], uint32_t (&q)[8]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t A = own[k], B = own[k];
        swap16(A, B);
        q[k] = B;
        q[4 + k] = A;
    }
}
// half g & 1 of a run (8 tokens): lane a = g & 1 wants bytes 8a..8a+7 and 16+8a..16+8a+7; it
// loaded 16a..16a+15. With X = own dwords 2, 3 and Y = own dwords 0, 1, the swap leaves
// {Y, X} = the wanted 16 bytes on both lanes.
__device__ __forceinline__ void run_half(const uint32_t (&own)[4], uint32_t (&q)[4]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        uint32_t X = own[2 + k], Y = own[k];
        swap16(X, Y);
        q[k] = Y;
        q[2 + k] = X;
    }
}

// Q4_K: step s = half h = s & 1 of super-block s >> 1 (h is the wave's: s = wave + 16 i); sub-block
// 4h + b is nibble b & 1 of qs run 2h + (b >> 1) (32 B at 16 + 32 (2h + (b >> 1))); every lane
// loads the 16-B header and half g & 1 of the run of its sub-block g (run_whole / run_half).
//   TOK 4: lane g uses the whole run of sub-block g;
//   TOK 8: lane g uses half g & 1 of run 2h + (g >> 1), and trades it for run 2h + 1 - (g >> 1)'s
//          with lane g ^ 2 (runs_to_pairs)
template <int TOK> struct MmaW<T_Q4_K, TOK> {
    static constexpr int NSC = 2;
    uint32_t H[4], QV[4];
    int h;
    __device__ static uint32_t step_off(int s) { return 144u * (uint32_t)(s >> 1); }
    __device__ static MmaLanes lanes(int r, int g, int h, uint32_t nb01, uint32_t) {
        const uint32_t row = r * nb01;
        return {row, row + 16 + 32 * (2 * h + (g >> 1)) + 16 * (g & 1), 0};
    }
    __device__ inline void load(__amdgpu_buffer_rsrc_t rs, const MmaLanes &lo) {
        bl16(rs, lo.a, H);
        bl16(rs, lo.b, QV);
    }
    __device__ inline void frags(long (&A)[4], int g, const MmaLanes &) {
        pin(H);
        pin(QV);
        if constexpr (TOK == 4) {
            uint32_t Q[8];
            run_whole(QV, Q);
            const int sft = 4 * (g & 1);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int o = 2 * (m >> 1) + 4 * (m & 1);
                A[m] = pack2((Q[o] >> sft) & NIB, (Q[o + 1] >> sft) & NIB);
            }
        } else {
            uint32_t Q[4], X[4], Y[4];
            run_half(QV, Q);
            runs_to_pairs(Q, X, Y);
            const int sft = 4 * (g >> 1);
            A[0] = pack2((X[0] >> sft) & NIB, (X[1] >> sft) & NIB);
            A[1] = pack2((X[2] >> sft) & NIB, (X[3] >> sft) & NIB);
            A[2] = pack2((Y[0] >> sft) & NIB, (Y[1] >> sft) & NIB);
            A[3] = pack2((Y[2] >> sft) & NIB, (Y[3] >> sft) & NIB);
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

// Q5_K: as Q4_K (runs at 48 + 32 c) plus the 5th bits: qh byte e (32 B at 16), bit 4h + b for
// sub-block 4h + b; the qh run is split and traded the same way
template <int TOK> struct MmaW<T_Q5_K, TOK> {
    static constexpr int NSC = 2;
    uint32_t H[4], QV[4], QHV[4];
    int h;
    __device__ static uint32_t step_off(int s) { return 176u * (uint32_t)(s >> 1); }
    __device__ static MmaLanes lanes(int r, int g, int h, uint32_t nb01, uint32_t) {
        const uint32_t row = r * nb01;
        return {row, row + 48 + 32 * (2 * h + (g >> 1)) + 16 * (g & 1), row + 16 + 16 * (g & 1)};
    }
    __device__ inline void load(__amdgpu_buffer_rsrc_t rs, const MmaLanes &lo) {
        bl16(rs, lo.a, H);
        bl16(rs, lo.b, QV);
        bl16(rs, lo.c, QHV);
    }
    __device__ inline void frags(long (&A)[4], int g, const MmaLanes &) {
        pin(H);
        pin(QV);
        pin(QHV);
        if constexpr (TOK == 4) {
            uint32_t Q[8], QH[8];
            run_whole(QV, Q);
            run_whole(QHV, QH);
            const int sft = 4 * (g & 1), hb = 4 * h + g;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int o = 2 * (m >> 1) + 4 * (m & 1);
                A[m] = pack2(((Q[o] >> sft) & NIB) | (((QH[o] >> hb) & 0x01010101u) << 4),
                             ((Q[o + 1] >> sft) & NIB) | (((QH[o + 1] >> hb) & 0x01010101u) << 4));
            }
        } else {
            uint32_t Q[4], QH[4], X[4], Y[4];
            run_half(QV, Q);
            run_half(QHV, QH);
            runs_to_pairs(Q, X, Y);
            const int sft = 4 * (g >> 1);
#pragma unroll
            for (int pq = 0; pq < 4; ++pq) {
                const uint32_t *R = pq < 2 ? X : Y;
                const int hb = 4 * h + 2 * (pq >> 1) + (g >> 1), o = 2 * (pq & 1);
                A[pq] = pack2(((R[o] >> sft) & NIB) | (((QH[o] >> hb) & 0x01010101u) << 4),
                              ((R[o + 1] >> sft) & NIB) | (((QH[o + 1] >> hb) & 0x01010101u) << 4));
            }
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

// Q6_K: step s = half h = s & 1 of super-block s >> 1 (128 elements: ql bytes 64h .. 64h + 63,
// qh bytes 128 + 32h .. + 31, scales 192 + 8h .. + 7, d at 208). Block j of the half is element
// l = 0..31 of quadrant j: the low (j < 2) or high nibble of ql run j & 1 (32 B at 64h + 32 (j & 1)),
// bits 2j, 2j + 1 of qh byte l, scale 8h + 2j + l / 16 (so each 32-block has two scales, one per
// 16-element half). Codes are stored signed (q - 32 fits int8), so no offset term is left.
// Two 16-B loads per lane and step (the load instructions bound the kernel: separate 2-byte scale
// and d loads cost 15 %, profiles/r06_q6k_mma.txt):
//   ql: TOK 4: lane g (block g) loads half g >> 1 of run g & 1 and trades with lane g ^ 2
//       (run_whole32); TOK 8: lane g (half g & 1 of block 2p + (g >> 1) for pairs p = 0, 1: the
//       same run, nibble p) loads bytes 16 (g & 1) .. + 15 of run g >> 1, then run_half;
//   second piece: lanes 0 / 1 the qh run's halves, lane 2 the scale bytes 192..207, lane 3 bytes
//       194..209 (the last 14 scales and d); one swap32 leaves qh half g & 1 and the scale window
//       of lane 2 + (g & 1) on every lane, and in either window block g's two scales are dword
//       2h + (g >> 1), low half; d reaches the even lanes by one swap16.
// Super-blocks are 2-byte aligned, so the 16-B pieces may be too (the memory path takes them at
// the same rate here: 4-byte aligned pieces measured no faster).
__device__ __forceinline__ void run_whole32(const uint32_t (&own)[4], uint32_t (&q)[8]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t A = own[k], B = own[k];
        swap32(A, B);   // (lanes g < 2 loaded bytes 0..15, g >= 2 bytes 16..31)
        q[k] = B;
        q[4 + k] = A;
    }
}
// 4 signed codes (q - 32) from 4 ql nibbles at shift sft and 4 qh bit pairs at shift hb
__device__ __forceinline__ uint32_t q6_codes(uint32_t ql, uint32_t qh, int sft, int hb) {
    const uint32_t u = ((ql >> sft) & NIB) | (((qh >> hb) & 0x03030303u) << 4);   // 0..63 per byte
    return (u + 0x60606060u) ^ 0x80808080u;                                         // (u + 96) - 128
}
template <int TOK> struct MmaW<T_Q6_K, TOK> {
    static constexpr int NSC = 2;
    uint32_t QV[4], MV[4], S, D;
    int h;
    __device__ static uint32_t step_off(int s) { return 210u * (uint32_t)(s >> 1); }
    // a = the ql piece, b = the second piece
    __device__ static MmaLanes lanes(int r, int g, int h, uint32_t nb01, uint32_t) {
        const uint32_t row = r * nb01;
        const uint32_t ql = TOK == 4 ? 32 * (g & 1) + 16 * (g >> 1) : 32 * (g >> 1) + 16 * (g & 1);
        const uint32_t m = g < 2 ? 128 + 32 * h + 16 * g : 192 + 2 * (g - 2);
        return {row + 64 * h + ql, row + m, 0};
    }
    __device__ inline void load(__amdgpu_buffer_rsrc_t rs, const MmaLanes &lo) {
        bl16(rs, lo.a, QV);
        bl16(rs, lo.b, MV);
    }
    __device__ inline void frags(long (&A)[4], int g, const MmaLanes &) {
        pin(QV);
        pin(MV);
        uint32_t H[4], W[4];   // qh half g & 1; the scale window of lane 2 + (g & 1)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t a = MV[k], b = MV[k];
            swap32(a, b);
            H[k] = b;
            W[k] = a;
        }
        uint32_t dw = W[3], dn = W[3];
        swap16(dw, dn);   // (even lanes: the odd partner's bytes 206..209; odd lanes keep their own)
        D = dw >> 16;
        const uint32_t w0 = h ? W[2] : W[0], w1 = h ? W[3] : W[1];
        S = (g & 2 ? w1 : w0) & 0xffffu;
        if constexpr (TOK == 4) {
            uint32_t Q[8], QH[8];
            run_whole32(QV, Q);
            run_whole(H, QH);
            const int sft = 4 * (g >> 1), hb = 2 * g;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int o = 2 * (m >> 1) + 4 * (m & 1);
                A[m] = pack2(q6_codes(Q[o], QH[o], sft, hb), q6_codes(Q[o + 1], QH[o + 1], sft, hb));
            }
        } else {
            uint32_t Q[4], QH[4];
            run_half(QV, Q);
            run_half(H, QH);
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int sft = 4 * p, hb = 2 * (2 * p + (g >> 1));
                A[2 * p] = pack2(q6_codes(Q[0], QH[0], sft, hb), q6_codes(Q[1], QH[1], sft, hb));
                A[2 * p + 1] = pack2(q6_codes(Q[2], QH[2], sft, hb), q6_codes(Q[3], QH[3], sft, hb));
            }
        }
    }
    // d * sc of the two halves of block g (S, D: from frags)
    __device__ inline void sc(float *o, int) const {
        const float d = h2f((uint16_t)D);
        o[0] = d * (float)(int8_t)(S & 0xff);
        o[1] = d * (float)(int8_t)(S >> 8);
    }
};

// ------------------------------------------------------------------------------------------
// Paired steps (Q4_0 / Q8_0, 4-byte-aligned contiguous rows): lane g loads blocks 2g and 2g + 1
// of a double step (8 blocks of its row, 256 k) as one aligned window — half the load
// instructions of one block per step — and two permlane swaps per dword hand every lane its
// block of each of the two steps:
//   F = block 2g, S = block 2g + 1:  g0 F0 S0 | g1 F1 S1 | g2 F2 S2 | g3 F3 S3
//   --swap16-->  X: F0 S0 F2 S2 / Y: F1 S1 F3 S3  --swap32-->  X: F0 S0 F1 S1 (step 2j: blocks 0..3)
//                                                            Y: F2 S2 F3 S3 (step 2j + 1: 4..7)
// ------------------------------------------------------------------------------------------
template <int T, int TOK> struct MmaHalf {   // one step's block of a lane, in registers
    static constexpr int NQ = T == T_Q4_0 ? 4 : 8;
    static constexpr int NSC = 1;
    uint32_t q[NQ], d;
    int h;   // (unused)
    __device__ inline void frags(long (&A)[4], int, const MmaLanes &) { MmaW<T, TOK>::frags_q(q, A); }
    __device__ inline void sc(float *o, int) { o[0] = h2f((uint16_t)d); }
};
template <int T, int TOK> struct MmaPair {
    static constexpr int NQ = T == T_Q4_0 ? 4 : 8;
    static constexpr int NV = T == T_Q4_0 ? 9 : 17;   // 36 / 68 bytes
    uint32_t V[NV];
    __device__ static MmaLanes lanes(int r, int g, uint32_t nb01) { return {r * nb01 + (2u * QT<T>::bytes) * g, 0, 0}; }
    __device__ inline void load(__amdgpu_buffer_rsrc_t rs, const MmaLanes &lo, uint32_t) {
#pragma unroll
        for (int k = 0; k + 4 <= NV; k += 4) bl16(rs, lo.a + 4 * k, V + k);
        V[NV - 1] = __builtin_amdgcn_raw_buffer_load_b32(rs, lo.a + 4 * (NV - 1), 0, 0);
    }
    // the two steps' blocks of this lane (X: step 2j, Y: step 2j + 1)
    __device__ inline void split(MmaHalf<T, TOK> &X, MmaHalf<T, TOK> &Y) {
        pin(V);
        // F = bytes 0..QT-1 (d at 0, qs from 2: funnel by 2), S = the next block (d in the high half
        // of dword NQ, qs dword-aligned after it)
        X.d = V[0] & 0xffff;
#pragma unroll
        for (int k = 0; k < NQ; ++k) X.q[k] = __builtin_amdgcn_alignbyte(V[k + 1], V[k], 2);
        Y.d = V[NQ] >> 16;
#pragma unroll
        for (int k = 0; k < NQ; ++k) Y.q[k] = V[NQ + 1 + k];
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            swap16(Y.q[k], X.q[k]);
            swap32(Y.q[k], X.q[k]);
        }
        swap16(Y.d, X.d);
        swap32(Y.d, X.d);
    }
};

// Q4_K paired steps (the two halves of a super-block): the 128 qs bytes of the tile's 16 rows are
// loaded row-contiguously, 8 rows x 128 bytes per wave instruction (instruction i: lane l holds
// row 8i + l / 8, piece l % 8), where the unpaired form gathers 16 rows x 64 bytes per instruction
// per step (the gather shape costs 8-12 % of the kernel, profiles/r06_mma_rowcontig_exp.txt);
// each lane then takes the piece MmaW<Q4_K> would have loaded for each half (piece 4h + g of row
// c) by ds_bpermute from the instruction holding row c, and the 16-B header is loaded once for
// both halves: 3 load instructions per super-block instead of 4.
// Q5_K likewise (qs at 48), its qh piece (half g & 1 of the 32 qh bytes, the same for both halves
// of the super-block) loaded once per super-block too: 4 load instructions instead of 6.
template <int T, int TOK> struct MmaPairK {
    static constexpr bool QH = T == T_Q5_K;
    static constexpr uint32_t QS = QH ? 48 : 16;
    uint32_t H[4], P0[4], P1[4], QHV[QH ? 4 : 1];
    __device__ static MmaLanes lanes(int r, int g, uint32_t nb01) {
        const uint32_t tile = (uint32_t)(r & ~15) * nb01, row = tile + (uint32_t)(r & 15) * nb01;
        const int l = (r & 15) + 16 * g;
        return {row, tile + (uint32_t)(l >> 3) * nb01 + QS + 16 * (l & 7), row + 16 + 16 * (g & 1)};
    }
    __device__ inline void load(__amdgpu_buffer_rsrc_t rs, const MmaLanes &lo, uint32_t nb01) {
        bl16(rs, lo.a, H);
        bl16(rs, lo.b, P0);
        bl16(rs, lo.b + 8 * nb01, P1);
        if constexpr (QH) bl16(rs, lo.c, QHV);
    }
    __device__ inline void split(MmaW<T, TOK> &X, MmaW<T, TOK> &Y) {
        pin(H);
        pin(P0);
        pin(P1);
        if constexpr (QH) {
            pin(QHV);
#pragma unroll
            for (int k = 0; k < 4; ++k) X.QHV[k] = Y.QHV[k] = QHV[k];
        }
        const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
        const int src0 = 4 * (8 * (c & 7) + g), src1 = src0 + 16;   // (byte addresses: piece g, 4 + g)
        const bool hi = c >= 8;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t a0 = __builtin_amdgcn_ds_bpermute(src0, P0[k]), b0 = __builtin_amdgcn_ds_bpermute(src0, P1[k]);
            const uint32_t a1 = __builtin_amdgcn_ds_bpermute(src1, P0[k]), b1 = __builtin_amdgcn_ds_bpermute(src1, P1[k]);
            X.QV[k] = hi ? b0 : a0;
            Y.QV[k] = hi ? b1 : a1;
            X.H[k] = Y.H[k] = H[k];
        }
        X.h = 0;
        Y.h = 1;
    }
};
template <int T, int TOK> struct PairOf { using type = MmaPair<T, TOK>; using half = MmaHalf<T, TOK>; };
template <int TOK> struct PairOf<T_Q4_K, TOK> { using type = MmaPairK<T_Q4_K, TOK>; using half = MmaW<T_Q4_K, TOK>; };
template <int TOK> struct PairOf<T_Q5_K, TOK> { using type = MmaPairK<T_Q5_K, TOK>; using half = MmaW<T_Q5_K, TOK>; };

// ------------------------------------------------------------------------------------------
// step sets in flight per wave (D - 1 steps ahead), within the 128 VGPRs of 16 waves per CU
#ifdef MMA_D
template <int T, int TOK, int RT> __host__ __device__ constexpr int mma_depth() { return MMA_D; }   // (measurement builds)
#else
template <int T, int TOK, int RT> __host__ __device__ constexpr int mma_depth() {
    return (T == T_Q5_K && TOK == 4) || (RT == 2 && T != T_Q4_0) ? 2 : 3;
}
#endif

template <int D, typename F, int... Is>
__device__ __forceinline__ void mma_run_steps(F &&f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is % D>{}, Is), ...);
}

// the columns' images once per call: grid (steps, slices), TOK * 16 threads, thread (t, j, m)
// quantizes chunk m of block j of column t (zeros past K and M); zero_dst: also clear dst (the
// two K halves of the main kernel add into it)
template <int TOK, bool XA>
__global__ __launch_bounds__(TOK * 16) void mma_prequant(const MmArgs a, uint8_t *__restrict__ img, int zero_dst) {
    const int s = blockIdx.x, z = blockIdx.y;
    const int i12 = z % a.ne12, i13 = z / a.ne12;
    const int m = threadIdx.x & 3, j = (threadIdx.x >> 2) & 3, t = threadIdx.x >> 4;
    const float *col = reinterpret_cast<const float *>(a.x + (int64_t)i12 * a.nb12 + (int64_t)i13 * a.nb13 +
                                                       (int64_t)min(t, a.M - 1) * a.nb11);
    float v[8];
    if constexpr (MMA_EXP & 1) {
        for (int c = 0; c < 8; ++c) v[c] = 0.f;
    } else {
        mma_xload<XA>(a, col, s, j, m, v);
    }
    if (zero_dst) {
        uint8_t *dz = a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3;
        for (int r = s * blockDim.x + threadIdx.x; r < a.N; r += gridDim.x * blockDim.x)
            for (int c = 0; c < a.M; ++c) reinterpret_cast<float *>(dz + (int64_t)c * a.nb1)[r] = 0.f;
    }
    mma_quant<TOK>(a, v, s, j, t, m, img + ((int64_t)z * gridDim.x + s) * mma_step_bytes<TOK>());
}

// Workgroup = RT 16-row tiles x one K part (grid.z of them, 1 or 2: two halves add into the
// zeroed dst, and 0 + a + b == 0 + b + a, so the result stays deterministic), 16 waves, wave w the
// part's steps w, w + 16, w + 32, ..., so that the workgroup's loads in flight are 16 consecutive
// steps of each row. The RT tiles of a wave share its column fragments: the column image a CU
// stages and the LDS reads per weight byte both fall with RT x K parts (the column image is
// most of the memory-pipeline work otherwise: 8 columns of K are more bytes than 16 weight rows).
// Steps past the part load through empty descriptors (zero weights) against the part's last
// column step. Straight-line code, no loop, so no register set crosses a back-edge (the copies
// the allocator puts on a back-edge move sets whose loads are still in flight, and each copy
// waits for its load). Each step loads its weights D - 1 steps ahead; all weight addresses are
// per-lane constants plus the step's descriptor base (scalar arithmetic).
template <int T, int TOK, int RT, int NSTEP, bool PR>
__global__ __launch_bounds__(MMA_KS * WAVE) void mmvq_mma_kernel(const MmArgs a, const uint8_t *__restrict__ img, int n_steps, int part_steps) {
    using W = MmaW<T, TOK>;
    static_assert(!PR || (T != T_Q6_K && NSTEP % 2 == 0), "paired steps: not Q6_K, even runs");
    constexpr int G = 16 / TOK;   // block groups per MFMA
    constexpr int L = 4 / G;      // k-groups per block group
    constexpr int P = 4 / G;      // MFMA outputs per step
    constexpr int Qn = G;         // MFMAs per output
    constexpr int NSC = W::NSC;
    constexpr int SB = mma_step_bytes<TOK>();
    constexpr int D = mma_depth<T, TOK, RT>();
    __shared__ __align__(16) float wsc[MMA_KS][RT][4 * NSC * 16];   // [wave][tile][block][k][row]
    __shared__ __align__(16) float red[MMA_KS][RT][4 * TOK * 4];
    extern __shared__ __align__(16) uint8_t xl[];   // [part steps][SB] column image, then 128 zero bytes

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int z = blockIdx.y;
    const int i12 = z % a.ne12, i13 = z / a.ne12;
    const int row0 = blockIdx.x * 16 * RT;
    const int s0 = blockIdx.z * part_steps;                     // the part's first step (even)
    const int n_loc = min(part_steps, n_steps - s0);            // its steps
    if (n_loc <= 0) return;                                     // (uniform: nothing to add)
    const uint8_t *wtile = a.w + (int64_t)(i12 / a.r2) * a.nb02 + (int64_t)(i13 / a.r3) * a.nb03 + (int64_t)row0 * a.nb01;
    const uint32_t nb01 = (uint32_t)a.nb01;
    const uint32_t tile_bytes = (uint32_t)(min(16 * RT, a.N - row0) - 1) * nb01 + (uint32_t)(a.K / QT<T>::blck) * QT<T>::bytes;
#if MMA_EXP & 4   // (measurement: Q4_K weight loads of 8 rows x 128 contiguous bytes per instruction)
    const uint32_t xrow = (uint32_t)((lane >> 3) + 8 * (wave & 1)) * nb01;   // (a wave pair: both halves of 16 rows)
    const MmaLanes lo0 = T == T_Q4_K ? MmaLanes{xrow, xrow + 16 + 16 * (lane & 7), 0}
                                     : W::lanes(c, g, wave & 1, nb01, (uint32_t)(reinterpret_cast<uintptr_t>(wtile) & 3));
#else
    const MmaLanes lo0 = W::lanes(c, g, wave & 1, nb01, (uint32_t)(reinterpret_cast<uintptr_t>(wtile) & 3));
#endif
    MmaLanes lo[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
        const uint32_t dt = 16 * t * nb01;
        lo[t] = {lo0.a + dt, lo0.b + dt, lo0.c + (T == T_Q5_K ? dt : 0u)};
    }
    if constexpr (T == T_Q4_0 || T == T_Q8_0) {
#pragma unroll
        for (int t = 0; t < RT; ++t) lo[t].c = lo0.c;   // (the funnel shift: 16 rows apart keep the alignment)
    }
    auto wrs = [&](int sl) __attribute__((always_inline)) {   // local step sl
        const uint32_t so = W::step_off(s0 + sl);
        return __builtin_amdgcn_make_buffer_rsrc((void *)(wtile + so), 0, sl < n_loc ? tile_bytes - so : 0u, MMA_RSRC_W3);
    };
    // the part's column image, staged in LDS once: 16-B pieces, thread t the pieces t + 1024 k
    // (issued before the weight prefetch, so the LDS writes wait for these loads only)
    const uint32_t nbx = (uint32_t)(n_loc * SB);
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc((void *)(img + ((int64_t)z * n_steps + s0) * SB), 0, nbx, MMA_RSRC_W3);
    constexpr int NP = (MMA_KS * NSTEP * SB + 16383) / 16384;
    uint32_t stg[NP][4];
    if constexpr (!(MMA_EXP & 1)) {
#pragma unroll
        for (int k = 0; k < NP; ++k) bl16(xr, threadIdx.x * 16 + k * 16384, stg[k]);
    }
    // B role: column c = token bt of block group bg; codes only where k-group g is in bg's range
    // (the other lanes read the zero bytes after the image, at a fixed address)
    const int bt = c % TOK, bg = c / TOK;
    const bool xlive = g / L == bg;
    const uint32_t xc = xlive ? (uint32_t)((bt * 4 + bg) * 32 + (g % L) * Qn * 8) : nbx;
    const uint32_t xstep = xlive ? (uint32_t)SB : 0u;
    const uint32_t xsc = (uint32_t)(TOK * 128 + (bt * 4 + bg) * 8);
    // (paired: wave w the double steps w, w + 16, ..., i.e. steps 2w, 2w + 1, 2w + 32, ...)
    auto step_of = [&](int i) { return PR ? 2 * (wave + MMA_KS * (i >> 1)) + (i & 1) : wave + MMA_KS * i; };

    struct Xf {
        uint32_t c[8];   // codes: TOK 4: 4 chunks of 8 B; TOK 8: pair p's 2 chunks at 4p
        float2 s[P];     // {d, d * sum(q)} of the output lane's (token, block) per pair
    };
    // (steps past the part read the zero bytes after the image: zero codes and zero scales)
    auto load_x = [&](Xf &x, int sl) __attribute__((always_inline)) {
        const bool live = sl < n_loc;
        const uint8_t *cp = live ? xl + xc + (uint32_t)sl * xstep : xl + nbx;
        const uint8_t *sp = live ? xl + xsc + (uint32_t)sl * SB : xl + nbx;
#pragma unroll
        for (int p = 0; p < P; ++p) {
            if constexpr (TOK == 4) {
                const uint4 v0 = *reinterpret_cast<const uint4 *>(cp), v1 = *reinterpret_cast<const uint4 *>(cp + 16);
                x.c[0] = v0.x; x.c[1] = v0.y; x.c[2] = v0.z; x.c[3] = v0.w;
                x.c[4] = v1.x; x.c[5] = v1.y; x.c[6] = v1.z; x.c[7] = v1.w;
            } else {
                const uint4 v = *reinterpret_cast<const uint4 *>(cp + p * G * 32);
                x.c[4 * p] = v.x; x.c[4 * p + 1] = v.y; x.c[4 * p + 2] = v.z; x.c[4 * p + 3] = v.w;
            }
            x.s[p] = *reinterpret_cast<const float2 *>(sp + p * G * 8);
        }
    };
    mma_f2 acc[RT][2] = {};   // tile t, rows 4g + {0, 1}, {2, 3}
    // sl: the local step. Its blocks past K (the last step of a Q4_0 / Q8_0 row whose K is not a
    // multiple of 128) were loaded from whatever follows the row (the next row, a view's padding):
    // their codes meet zero activation codes, and their weight scales are zeroed here, so a
    // non-finite f16 there cannot turn 0 * d into NaN
    auto compute = [&](auto &w, Xf &x, int sl) __attribute__((always_inline)) {
        pin(x.c);
        pin(x.s);
        const bool blk_live = T == T_Q4_0 || T == T_Q8_0 ? ((s0 + sl) * MMA_STEP_K + 32 * g < a.K) : true;
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            long A[4];
            w[t].frags(A, g, lo[t]);
            // publish this lane's block-g scales, [block g][k][row c]
            float o[NSC];
            w[t].sc(o, g);
#pragma unroll
            for (int k = 0; k < NSC; ++k) o[k] = blk_live ? o[k] : 0.f;
            float *ws = wsc[wave][t];
#pragma unroll
            for (int k = 0; k < NSC; ++k) ws[(g * NSC + k) * 16 + c] = o[k];
            const i32x4_t zero = {0, 0, 0, 0};
#pragma unroll
            for (int p = 0; p < P; ++p) {
                if constexpr (T == T_Q6_K) {
                    // a block's two 16-element halves have scales of their own: one MFMA chain per
                    // half (TOK 4: chunks 0, 2 | 1, 3; TOK 8: MFMA q is half q), then
                    // acc += dx * (s0 * R0 + s1 * R1) for rows 4g + i, token bt, block p G + bg
                    i32x4_t R0 = zero, R1 = zero;
#pragma unroll
                    for (int q = 0; q < Qn; ++q) {
                        const int ci = TOK == 4 ? 2 * q : 4 * p + 2 * q;
                        const long B = pack2(x.c[ci], x.c[ci + 1]);
                        if ((TOK == 4 ? q & 1 : q) == 0) R0 = __builtin_amdgcn_mfma_i32_16x16x32_i8(A[p * Qn + q], B, R0, 0, 0, 0);
                        else R1 = __builtin_amdgcn_mfma_i32_16x16x32_i8(A[p * Qn + q], B, R1, 0, 0, 0);
                    }
                    const float *rs = ws + (p * G + bg) * NSC * 16 + 4 * g;
                    const float4 s4 = *reinterpret_cast<const float4 *>(rs), t4 = *reinterpret_cast<const float4 *>(rs + 16);
                    const mma_f2 xd = {x.s[p].x, x.s[p].x};
                    const mma_f2 s0[2] = {{s4.x, s4.y}, {s4.z, s4.w}}, s1[2] = {{t4.x, t4.y}, {t4.z, t4.w}};
                    const mma_f2 r0[2] = {{(float)R0[0], (float)R0[1]}, {(float)R0[2], (float)R0[3]}};
                    const mma_f2 r1[2] = {{(float)R1[0], (float)R1[1]}, {(float)R1[2], (float)R1[3]}};
#pragma unroll
                    for (int h = 0; h < 2; ++h) acc[t][h] = __builtin_elementwise_fma(xd, __builtin_elementwise_fma(s0[h], r0[h], s1[h] * r1[h]), acc[t][h]);
                    continue;
                }
                i32x4_t R = zero;
#pragma unroll
                for (int q = 0; q < Qn; ++q) {
                    const int ci = TOK == 4 ? 2 * q : 4 * p + 2 * q;
                    R = __builtin_amdgcn_mfma_i32_16x16x32_i8(A[p * Qn + q], pack2(x.c[ci], x.c[ci + 1]), R, 0, 0, 0);
                }
                // outputs: rows 4g + i, token bt, block p G + bg, two rows at a time (the object is
                // built without packed-f32 ops, as mmq8.o: scalar fmas beside the MFMAs, Makefile)
                const float *rs = ws + (p * G + bg) * NSC * 16 + 4 * g;
                const mma_f2 xd = {x.s[p].x, x.s[p].x};
                const mma_f2 r[2] = {{(float)R[0], (float)R[1]}, {(float)R[2], (float)R[3]}};
                if constexpr (T == T_Q4_0 || T == T_Q8_0) {
                    const float4 dw = *reinterpret_cast<const float4 *>(rs);
                    const mma_f2 dv[2] = {{dw.x, dw.y}, {dw.z, dw.w}};
                    const float o8 = T == T_Q4_0 ? -8.f * x.s[p].y : 0.f;
                    const mma_f2 off = {o8, o8};
#pragma unroll
                    for (int h = 0; h < 2; ++h) acc[t][h] = __builtin_elementwise_fma(dv[h], __builtin_elementwise_fma(xd, r[h], off), acc[t][h]);
                } else {
                    const float4 s4 = *reinterpret_cast<const float4 *>(rs), m4 = *reinterpret_cast<const float4 *>(rs + 16);
                    const mma_f2 sv[2] = {{s4.x, s4.y}, {s4.z, s4.w}}, nm[2] = {{-m4.x, -m4.y}, {-m4.z, -m4.w}};
                    const mma_f2 sx = {x.s[p].y, x.s[p].y};
#pragma unroll
                    for (int h = 0; h < 2; ++h) acc[t][h] = __builtin_elementwise_fma(sv[h], xd * r[h], __builtin_elementwise_fma(nm[h], sx, acc[t][h]));
                }
            }
        }
        // (without the pins the scale sums of every step sink below the last step, each step's
        // MFMA results stay live to the end, and the registers spill)
        pin(acc);
    };

    auto stage_x = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const uint32_t o = threadIdx.x * 16 + k * 16384;
            if (o < nbx) {
                if constexpr (MMA_EXP & 1) *reinterpret_cast<uint4 *>(xl + o) = make_uint4(o, 1, 2, 3);
                else *reinterpret_cast<uint4 *>(xl + o) = make_uint4(stg[k][0], stg[k][1], stg[k][2], stg[k][3]);
            }
        }
        if (threadIdx.x < 8) *reinterpret_cast<uint4 *>(xl + nbx + threadIdx.x * 16) = make_uint4(0, 0, 0, 0);
        lds_barrier();
    };
    if constexpr (!PR) {
        W F[D][RT];
        Xf X[D];
#pragma unroll
        for (int d = 0; d < D - 1; ++d)
#pragma unroll
            for (int t = 0; t < RT; ++t) {
                if constexpr (!(MMA_EXP & 2)) F[d][t].load(wrs(step_of(d)), lo[t]);
                F[d][t].h = wave & 1;
            }
        stage_x();
#pragma unroll
        for (int d = 0; d < D - 1; ++d) load_x(X[d], step_of(d));
        auto step = [&](auto k_c, int i) __attribute__((always_inline)) {
            constexpr int k = decltype(k_c)::value;
            if (i + D - 1 < NSTEP) {
                const int sl = step_of(i + D - 1);
#pragma unroll
                for (int t = 0; t < RT; ++t) {
                    if constexpr (!(MMA_EXP & 2)) F[(k + D - 1) % D][t].load(wrs(sl), lo[t]);
                    F[(k + D - 1) % D][t].h = wave & 1;
                }
                load_x(X[(k + D - 1) % D], sl);
            }
            __builtin_amdgcn_sched_barrier(0);
            compute(F[k], X[k], step_of(i));
        };
        mma_run_steps<D>(step, std::make_integer_sequence<int, NSTEP>{});
    } else {
        // one pair (two steps) ahead; a pair's descriptor is its first step's (the second step's
        // blocks follow in the row; past the part its columns are zero)
        constexpr int DP = 2;
        using WP = typename PairOf<T, TOK>::type;
        MmaLanes lp[RT];
#pragma unroll
        for (int t = 0; t < RT; ++t) lp[t] = WP::lanes(c + 16 * t, g, nb01);
        WP F[DP][RT];
        Xf X[DP][2];
#pragma unroll
        for (int t = 0; t < RT; ++t)
            if constexpr (!(MMA_EXP & 2)) F[0][t].load(wrs(step_of(0)), lp[t], nb01);
        stage_x();
        load_x(X[0][0], step_of(0));
        load_x(X[0][1], step_of(1));
        auto pstep = [&](auto k_c, int j) __attribute__((always_inline)) {
            constexpr int k = decltype(k_c)::value;
            if (j + 1 < NSTEP / 2) {
#pragma unroll
                for (int t = 0; t < RT; ++t)
                    if constexpr (!(MMA_EXP & 2)) F[(k + 1) % DP][t].load(wrs(step_of(2 * j + 2)), lp[t], nb01);
                load_x(X[(k + 1) % DP][0], step_of(2 * j + 2));
                load_x(X[(k + 1) % DP][1], step_of(2 * j + 3));
            }
            __builtin_amdgcn_sched_barrier(0);
            typename PairOf<T, TOK>::half H0[RT], H1[RT];
#pragma unroll
            for (int t = 0; t < RT; ++t) F[k][t].split(H0[t], H1[t]);
            compute(H0, X[k][0], step_of(2 * j));
            compute(H1, X[k][1], step_of(2 * j + 1));
        };
        mma_run_steps<DP>(pstep, std::make_integer_sequence<int, NSTEP / 2>{});
    }

    // sum the block groups (columns c, c + TOK, ... of the 16-lane row), then the waves in order
#pragma unroll
    for (int t = 0; t < RT; ++t) {
        float v[4] = {acc[t][0].x, acc[t][0].y, acc[t][1].x, acc[t][1].y};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if constexpr (TOK == 4) v[i] += dpp_f<DPP_ROR4>(v[i]);
            v[i] += dpp_f<DPP_ROR8>(v[i]);
        }
        if (c < TOK) {
#pragma unroll
            for (int i = 0; i < 4; ++i) red[wave][t][(g * TOK + c) * 4 + i] = v[i];
        }
    }
    lds_barrier();
    if (wave >= RT || c >= TOK || c >= a.M) return;   // wave t sums tile t
    const int t = wave;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = red[0][t][(g * TOK + c) * 4 + i];
#pragma unroll
    for (int w = 1; w < MMA_KS; ++w)
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] += red[w][t][(g * TOK + c) * 4 + i];
    float *dcol = reinterpret_cast<float *>(a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3 + (int64_t)c * a.nb1);
    const int r0 = row0 + 16 * t + 4 * g;
    if (gridDim.z == 2) {   // 0 + a + b == 0 + b + a: deterministic for exactly two parts
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (r0 + i < a.N) unsafeAtomicAdd(dcol + r0 + i, v[i]);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (r0 + i < a.N) dcol[r0 + i] = v[i];
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
static int mma_steps(const MmArgs &a) { return (a.K + MMA_STEP_K - 1) / MMA_STEP_K; }
static int mma_tok_of(const MmArgs &a) { return a.M <= 4 ? 4 : 8; }
// steps of a K part (even: a K-quant super-block's two halves stay in one part)
static int mma_part_steps(const MmArgs &a, int kh) {
    const int S = mma_steps(a);
    return kh == 1 ? S : ((S + 1) / 2 + 1) & ~1;
}

// Q4_0 / Q8_0 rows contiguous and 4-byte aligned (paired steps load aligned 36 / 68-byte windows)
static bool mma_pair_aligned(int type, const MmArgs &a) {
    if (type == T_Q4_K || type == T_Q5_K) return true;   // (rows loaded one by one: any row stride)
    if (type != T_Q4_0 && type != T_Q8_0) return false;
    const int64_t row = (int64_t)(a.K / 32) * (type == T_Q4_0 ? 18 : 34);
    return a.nb01 == row && row % 4 == 0 && a.nb02 % 4 == 0 && a.nb03 % 4 == 0 && (reinterpret_cast<uintptr_t>(a.w) & 3) == 0;
}

// steps per wave: the smallest run that covers the part over the 16 waves (0: too long)
static constexpr int MMA_RUNS[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14};
static int mma_nstep(int part) {
    for (int ns : MMA_RUNS)
        if (MMA_KS * ns >= part) return ns;
    return 0;
}
// the run mma_run launches for a part: pairs round it up to an even length (0: none fits)
static int mma_run_len(int part, bool pr) {
    const int ns = mma_nstep(part);
    return pr && ns > 0 ? (ns + 1) & ~1 : ns;
}

// the column image of a part lives in LDS next to the kernel's static arrays (wsc: 4 KiB x RT x
// scales per block, red: 1 KiB x RT x TOK), after which come the 128 zero bytes; 256 bytes of
// slack for alignment
static constexpr int mma_nsc(int type) { return type == T_Q4_K || type == T_Q5_K || type == T_Q6_K ? 2 : 1; }
static constexpr int mma_lds_img(int nsc, int tok, int rt) { return 160 * 1024 - (4096 * nsc + 1024 * tok) * rt - 128 - 256; }

// exactly the launcher's conditions for a part of `part` steps: a run for it, its image in LDS,
// and the run's steps within the image mma_main accepts (paired runs of part 97..102 at 8
// tokens, or 193..204 at 4, round past it with two tiles: e.g. Q4_0 K = 25600 at 5..8 columns,
// Q4_K K = 49408 at 3)
static bool mma_part_fits(int type, const MmArgs &a, int part, bool pr, int rt) {
    const int ns = mma_run_len(part, pr), tok = mma_tok_of(a), sb = tok * 160;   // mma_step_bytes<TOK>()
    const int img = mma_lds_img(mma_nsc(type), tok, rt);
    return ns > 0 && part * sb <= img && MMA_KS * ns * sb <= img + 16 * sb;
}

// the launch plan, from hipGraph periods of back-to-back calls (scripts/mv_graph.py through
// scripts/mv_sweep.sh: 4 types x 10 shapes x 3..8 columns, weights Infinity-Cache-cold and warm,
// profiles/r06_mma_plan_sweep.txt; round 5 chose from eager launches, whose period the host's
// launch rate bounded):
//   pr  paired steps: Q4_0 always, Q8_0 below K = 8192 and from 12288 (at 11008 the unpaired
//       form with two tiles wins), where the rows allow it; the K-quant pairs where rows are
//       whole 128-B lines apart (K = 11008: 43 super-blocks, rows 48 / 16 B off a line, pairs
//       4-6 % slower): Q4_K at 1..4 columns from K = 12288 (28672 x 4096 at 3 columns 20.3 vs
//       22.3 us, 12288 x 4096 12.7 vs 13.1; at 5..8 columns 6-10 % slower,
//       profiles/r06_q4k_pairs.txt), Q5_K at any column count where the whole K fits one part
//       (28672 x 4096 at 3..4 columns 23.4-25.2 vs 28.5, 12288 x 4096 14.3-15.0 vs 15.7-15.9,
//       4096 x 14336 at 5..8 16.7-18.7 vs 18.4-21.0; two parts paired were 1-5 % slower on one
//       box of two, profiles/r06_q5k_pairs.txt);
//   kh  one K part wherever the whole column image fits the workgroup's LDS: 0.85-0.95x the
//       two-part time (no dst zeroing in the pre-pass, no atomic adds, a wave walks twice the
//       steps); two parts only for images that do not fit (e.g. Q4_0 at 5..8 columns from K =
//       15104 with one tile, 13184 with two),
//       as before where each part keeps >= 32 steps for pairs, >= 16 unpaired, and for Q5_K with
//       K and N below 8192 (one tile per workgroup: 512 two-part workgroups beat 256);
//   rt  16-row tiles per workgroup: Q5_K and Q8_0 pairs 1 (registers); with one K part 2 when
//       N >= 8192 at K >= 8192, or N >= 12288, else 1 (one tile per workgroup doubles the
//       workgroups: Q8_0 11008 x 4096 15.6 vs 23.3 us with two); with two parts 2.
// GGML_MI355X_MMA_PAIR / _KH / _RT force (measurements: _KH=1 one part, =2 two parts where the
// steps allow; _RT=1/2)
struct MmaPlan {
    int kh, rt;
    bool pr;
};
static MmaPlan mma_plan(int type, const MmArgs &a) {
    const int S = mma_steps(a);
    MmaPlan p;
    const int pe = settings().mma_pair;
    const bool lines = a.nb01 % 128 == 0;   // (K-quant pairs: rows whole 128-B lines apart)
    const bool want = pe >= 0 ? pe == 1
                              : (type == T_Q4_0 || (type == T_Q8_0 && (a.K < 8192 || a.K >= 12288)) ||
                                 (type == T_Q4_K && lines && a.M <= 4 && a.K >= 12288) ||
                                 (type == T_Q5_K && lines && mma_part_fits(type, a, S, true, 1)));
    p.pr = want && mma_pair_aligned(type, a);
    const bool two_ok = p.pr ? S >= 64 : S >= 32;
    const int ke = settings().mma_kh, re = settings().mma_rt;
    auto rt_of = [&](int want) { return type == T_Q5_K || type == T_Q6_K || (type == T_Q8_0 && p.pr) ? 1 : re == 1 || re == 2 ? re : want; };
    const int rt1 = rt_of((a.N >= 8192 && a.K >= 8192) || a.N >= 12288 ? 2 : 1);
    if (ke == 1) p.kh = 1;
    else if (ke == 2) p.kh = two_ok ? 2 : 1;
    else if ((type == T_Q5_K || type == T_Q6_K) && a.K < 8192 && a.N < 8192) p.kh = two_ok ? 2 : 1;   // (one tile per workgroup: 512 beat 256)
    else p.kh = two_ok && !mma_part_fits(type, a, S, p.pr, rt1) ? 2 : 1;
    p.rt = p.kh == 1 ? rt1 : rt_of(2);
    return p;
}

// the plan keeps the K range in one part / takes paired steps (dispatch.cpp use_mma)
bool mmvq_mma_one_part(int type, const MmArgs &a) { return mma_plan(type, a).kh == 1; }
bool mmvq_mma_paired(int type, const MmArgs &a) { return mma_plan(type, a).pr; }

bool mmvq_mma_supported(int type, const MmArgs &a) {
    if (!(type == T_Q4_0 || type == T_Q8_0 || type == T_Q4_K || type == T_Q5_K || type == T_Q6_K) || a.M < 1 || a.M > 8) return false;
    const MmaPlan pl = mma_plan(type, a);
    return mma_part_fits(type, a, mma_part_steps(a, pl.kh), pl.pr, pl.rt);
}

// the launch mma_tok makes (the dispatch description, ggml_mi355x_mul_mat_plan)
std::string mmvq_mma_plan_text(int type, const MmArgs &a) {
    const MmaPlan pl = mma_plan(type, a);
    const int part = mma_part_steps(a, pl.kh);
    int rt = pl.rt;
    if (type == T_Q5_K || type == T_Q6_K || (type == T_Q8_0 && pl.pr)) rt = 1;
    return "mma tok=" + std::to_string(mma_tok_of(a)) + " kh=" + std::to_string(pl.kh) + " rt=" + std::to_string(rt) +
           (pl.pr ? " paired" : "") + " run=" + std::to_string(mma_run_len(part, pl.pr)) + " cols=" + std::to_string(a.M);
}

size_t mmvq_mma_img_bytes(int, const MmArgs &a) {
    return (size_t)mma_steps(a) * mma_tok_of(a) * 160 * a.ne12 * a.ne13;
}

template <int T, int TOK, int RT, int NS, bool PR>
static hipError_t mma_main(const MmArgs &a, const uint8_t *img, int S, int part, int kh, hipStream_t st) {
    constexpr int IMG = mma_lds_img(MmaW<T, TOK>::NSC, TOK, RT);
    if constexpr (MMA_KS * NS * mma_step_bytes<TOK>() > IMG + 16 * mma_step_bytes<TOK>()) {
        return hipErrorInvalidValue;   // (runs whose image cannot fit: never selected)
    } else {
        auto kern = mmvq_mma_kernel<T, TOK, RT, NS, PR>;
        const size_t lds = (size_t)part * mma_step_bytes<TOK>() + 128;
        static LdsAttr attr;   // per instantiation and device; > 64 KB of dynamic LDS needs the attribute
        if (lds > 64 * 1024)
            if (const hipError_t e = lds_attr_once(reinterpret_cast<const void *>(kern), attr); e != hipSuccess) return e;
        hipLaunchKernelGGL(kern, dim3((a.N + 16 * RT - 1) / (16 * RT), a.ne12 * a.ne13, kh), dim3(MMA_KS * WAVE), lds, st, a, img, S, part);
        return hipSuccess;
    }
}

template <int T, int TOK, int RT, bool PR>
static hipError_t mma_run(const MmArgs &a, const uint8_t *img, int S, int part, int kh, hipStream_t st) {
    switch (mma_run_len(part, PR)) {   // (pairs: even runs)
        case 1: if constexpr (!PR) return mma_main<T, TOK, RT, 1, PR>(a, img, S, part, kh, st); else break;
        case 2: return mma_main<T, TOK, RT, 2, PR>(a, img, S, part, kh, st);
        case 3: if constexpr (!PR) return mma_main<T, TOK, RT, 3, PR>(a, img, S, part, kh, st); else break;
        case 4: return mma_main<T, TOK, RT, 4, PR>(a, img, S, part, kh, st);
        case 5: if constexpr (!PR) return mma_main<T, TOK, RT, 5, PR>(a, img, S, part, kh, st); else break;
        case 6: return mma_main<T, TOK, RT, 6, PR>(a, img, S, part, kh, st);
        case 7: if constexpr (!PR) return mma_main<T, TOK, RT, 7, PR>(a, img, S, part, kh, st); else break;
        case 8: return mma_main<T, TOK, RT, 8, PR>(a, img, S, part, kh, st);
        case 10: return mma_main<T, TOK, RT, 10, PR>(a, img, S, part, kh, st);
        case 12: return mma_main<T, TOK, RT, 12, PR>(a, img, S, part, kh, st);
        case 14: return mma_main<T, TOK, RT, 14, PR>(a, img, S, part, kh, st);
        default: break;
    }
    return hipErrorInvalidValue;
}

template <int T, int TOK>
static hipError_t mma_tok(const MmArgs &a, uint8_t *img, hipStream_t st) {
    const MmaPlan pl = mma_plan(T, a);
    const int S = mma_steps(a), kh = pl.kh, part = mma_part_steps(a, kh);
    const dim3 pg(S, a.ne12 * a.ne13);
    if (settings().diag & 256) {   // (measurement: no pre-pass)
    } else if (a.x_aligned16) hipLaunchKernelGGL((mma_prequant<TOK, true>), pg, dim3(TOK * 16), 0, st, a, img, kh == 2);
    else hipLaunchKernelGGL((mma_prequant<TOK, false>), pg, dim3(TOK * 16), 0, st, a, img, kh == 2);
    hipError_t e;
    if constexpr (T == T_Q6_K) e = mma_run<T, TOK, 1, false>(a, img, S, part, kh, st);
    else if constexpr (T == T_Q5_K) e = pl.pr ? mma_run<T, TOK, 1, true>(a, img, S, part, kh, st) : mma_run<T, TOK, 1, false>(a, img, S, part, kh, st);
    else if constexpr (T == T_Q8_0) {
        if (pl.pr) e = mma_run<T, TOK, 1, true>(a, img, S, part, kh, st);   // (two tiles of pairs would spill)
        else e = pl.rt == 2 ? mma_run<T, TOK, 2, false>(a, img, S, part, kh, st) : mma_run<T, TOK, 1, false>(a, img, S, part, kh, st);
    } else if constexpr (T == T_Q4_0) {
        if (pl.pr) e = pl.rt == 2 ? mma_run<T, TOK, 2, true>(a, img, S, part, kh, st) : mma_run<T, TOK, 1, true>(a, img, S, part, kh, st);
        else e = pl.rt == 2 ? mma_run<T, TOK, 2, false>(a, img, S, part, kh, st) : mma_run<T, TOK, 1, false>(a, img, S, part, kh, st);
    } else if constexpr (T == T_Q4_K) {
        if (pl.pr) e = pl.rt == 2 ? mma_run<T, TOK, 2, true>(a, img, S, part, kh, st) : mma_run<T, TOK, 1, true>(a, img, S, part, kh, st);
        else e = pl.rt == 2 ? mma_run<T, TOK, 2, false>(a, img, S, part, kh, st) : mma_run<T, TOK, 1, false>(a, img, S, part, kh, st);
    } else e = pl.rt == 2 ? mma_run<T, TOK, 2, false>(a, img, S, part, kh, st) : mma_run<T, TOK, 1, false>(a, img, S, part, kh, st);
    return e != hipSuccess ? e : hipGetLastError();
}

template <int T>
static hipError_t mma_type(const MmArgs &a, uint8_t *img, hipStream_t st) {
    return mma_tok_of(a) == 4 ? mma_tok<T, 4>(a, img, st) : mma_tok<T, 8>(a, img, st);
}

// plain MUL_MAT with 1 <= M <= 8 columns (mmvq_mma_supported), img = mmvq_mma_img_bytes of scratch
hipError_t mmvq_mma_launch(int type, const MmArgs &a, uint8_t *img, hipStream_t st) {
    if (!mmvq_mma_supported(type, a) || img == nullptr) return hipErrorInvalidValue;
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
