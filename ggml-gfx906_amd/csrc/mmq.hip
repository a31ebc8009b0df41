// mmq.hip — quantized mat-mat (prefill, ne11 > 8) on gfx950 matrix cores.
//
// Replaces the reference's MMQ path (quantize_mmq_q8_1 + mul_mat_q, src/ggml-cuda/mmq.cuh:3134,
// quantize.cu:50-146). Design choice for CDNA4 (reasoning and numbers in DESIGN.md §MMQ):
//
//   The ggml block formats carry one scale per 16-32 weights. An int8 MFMA
//   (v_mfma_i32_32x32x32_i8) spans exactly one 32-block per instruction, so every output
//   element needs its own cvt + scale-multiply + FMA after every MFMA: ~48 VALU issues
//   (~190 cycles for one wave) per 32-cycle MFMA, which caps int8 well below the f16 rate.
//   Dequantizing each weight ONCE per tile into f16 (exact integer codes, one rounding of
//   d*q) and running v_mfma_f32_32x32x16_f16 with fp32 accumulation needs no per-block
//   epilogue: the dequant (~1.7 packed VALU per weight) is amortized over the tile's tokens,
//   and the matrix pipe runs at the dense f16 rate. Activations are converted to f16 once
//   per launch with a per-token power-of-two prescale (no overflow, no subnormals), which is
//   more accurate than the reference's own int8 activation blocks.
//
// Tile: BM weight rows x BN tokens per 256-thread workgroup (4 waves as 2 x 2, each
// BM/2 x BN/2 = (BM/64) x (BN/64) MFMA 32x32 tiles), BK = 64 per step. Staging is a 2-deep
// register ring (raw quant bytes + f16 activations for steps s+1 and s+2 in flight while the
// MFMAs of step s run) into 2 LDS buffers; LDS rows are 128 B with a 16-B XOR swizzle that
// makes the ds_read_b128 fragment reads conflict-free.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "dispatch.h"
#include "qcommon.h"

namespace mi355x {

typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // SROA-friendly 16-B register

constexpr int MQ_BK = 64;        // K per step = one 128-B LDS row of f16
constexpr int MQ_THREADS = 256;

__device__ __forceinline__ h2v as_h2(uint32_t u) { return __builtin_bit_cast(h2v, u); }
__device__ __forceinline__ uint32_t as_u(h2v v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ h2v splat_h2(float f) {
    const _Float16 h = (_Float16)f;
    return h2v{h, h};
}

// Register "launder": the asm produces v, so nothing computed from v can be scheduled above it.
// Used to keep the decode of a ring slot in its store phase (the pre-RA scheduler otherwise
// floats that pure VALU work up into the load phase and waits on the loads it just issued).
__device__ __forceinline__ void pin(uint32_t &v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(u32x4 &v) { asm volatile("" : "+v"(v)); }
template <int N> __device__ __forceinline__ void pin(uint32_t (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) pin(v[i]);
}

// 4 unsigned bytes -> f16 pairs holding (1024 + byte): 0x64XX is 1024 + XX exactly
__device__ __forceinline__ void bytes_f16(uint32_t b, uint32_t &lo, uint32_t &hi) {
    lo = __builtin_amdgcn_perm(0x64646464u, b, 0x04010400u);
    hi = __builtin_amdgcn_perm(0x64646464u, b, 0x04030402u);
}

// 16 byte codes in c[4] -> 16 f16 weights (c - bias) * d, packed in o[8]; one rounding
template <int BIAS>
__device__ __forceinline__ void emit_scaled(const uint32_t c[4], h2v d, uint32_t o[8]) {
    const h2v bias = splat_h2(1024.f + BIAS);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t lo, hi;
        bytes_f16(c[i], lo, hi);
        o[2 * i] = as_u((as_h2(lo) - bias) * d);
        o[2 * i + 1] = as_u((as_h2(hi) - bias) * d);
    }
}

// 16 byte codes -> c * d1 - m1 (affine K-quant form)
__device__ __forceinline__ void emit_affine(const uint32_t c[4], h2v d1, h2v m1, uint32_t o[8]) {
    const h2v bias = splat_h2(1024.f);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t lo, hi;
        bytes_f16(c[i], lo, hi);
        o[2 * i] = as_u(__builtin_elementwise_fma(as_h2(lo) - bias, d1, -m1));
        o[2 * i + 1] = as_u(__builtin_elementwise_fma(as_h2(hi) - bias, d1, -m1));
    }
}

// ------------------------------------------------------------------------------------------
// 16-weight dequant units: raw registers loaded ahead (load), decoded at LDS-store time (emit).
// Formulas restate src/ggml-quants.c dequantize_row_* (:307, :401, :1352, :1554, :1762).
// ------------------------------------------------------------------------------------------
template <int T> struct Deq16;

template <> struct Deq16<T_Q4_0> {
    uint32_t q[4], d;
    int sh;
    __device__ __forceinline__ void pin_all() { pin(q); pin(d); }
    __device__ __forceinline__ void load(const uint8_t *row, int k0) {
        const uint8_t *b = row + (k0 >> 5) * 18;
        d = ld2(b);
        ld16(b + 2, q);
        sh = (k0 & 16) ? 4 : 0;
    }
    __device__ __forceinline__ void emit(uint32_t o[8]) const {
        uint32_t c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = (q[i] >> sh) & 0x0F0F0F0Fu;
        emit_scaled<8>(c, splat_h2(h2f((uint16_t)d)), o);
    }
};

template <> struct Deq16<T_Q8_0> {
    uint32_t q[4], d;
    __device__ __forceinline__ void pin_all() { pin(q); pin(d); }
    __device__ __forceinline__ void load(const uint8_t *row, int k0) {
        const uint8_t *b = row + (k0 >> 5) * 34;
        d = ld2(b);
        ld16(b + 2 + (k0 & 16), q);
    }
    __device__ __forceinline__ void emit(uint32_t o[8]) const {
        uint32_t c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = q[i] ^ 0x80808080u;   // int8 -> 128 + q
        emit_scaled<128>(c, splat_h2(h2f((uint16_t)d)), o);
    }
};

template <> struct Deq16<T_Q4_K> {
    uint32_t q[4], dm, S[3];
    int j;
    __device__ __forceinline__ void pin_all() { pin(q); pin(dm); pin(S); }
    __device__ __forceinline__ void load(const uint8_t *row, int k0) {
        const uint8_t *b = row + (k0 >> 8) * 144;
        const int w = k0 & 255, c = w >> 6;
        j = w >> 5;
        dm = ld4(b);
        S[0] = ld4(b + 4); S[1] = ld4(b + 8); S[2] = ld4(b + 12);
        ld16(b + 16 + 32 * c + (w & 31), q);
    }
    __device__ __forceinline__ void emit(uint32_t o[8]) const {
        uint32_t sc0, sc1, m0, m1;
        k4_scale_min_pair(S, j >> 1, sc0, sc1, m0, m1);
        const bool hi = j & 1;
        const float d1 = h2f((uint16_t)dm) * (float)(hi ? sc1 : sc0);
        const float mm = h2f((uint16_t)(dm >> 16)) * (float)(hi ? m1 : m0);
        const int sh = hi ? 4 : 0;
        uint32_t c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = (q[i] >> sh) & 0x0F0F0F0Fu;
        emit_affine(c, splat_h2(d1), splat_h2(mm), o);
    }
};

template <> struct Deq16<T_Q5_K> {
    uint32_t q[4], h[4], dm, S[3];
    int j;
    __device__ __forceinline__ void pin_all() { pin(q); pin(h); pin(dm); pin(S); }
    __device__ __forceinline__ void load(const uint8_t *row, int k0) {
        const uint8_t *b = row + (k0 >> 8) * 176;
        const int w = k0 & 255, c = w >> 6;
        j = w >> 5;
        dm = ld4(b);
        S[0] = ld4(b + 4); S[1] = ld4(b + 8); S[2] = ld4(b + 12);
        ld16(b + 16 + (w & 31), h);
        ld16(b + 48 + 32 * c + (w & 31), q);
    }
    __device__ __forceinline__ void emit(uint32_t o[8]) const {
        uint32_t sc0, sc1, m0, m1;
        k4_scale_min_pair(S, j >> 1, sc0, sc1, m0, m1);
        const bool hi = j & 1;
        const float d1 = h2f((uint16_t)dm) * (float)(hi ? sc1 : sc0);
        const float mm = h2f((uint16_t)(dm >> 16)) * (float)(hi ? m1 : m0);
        const int sh = hi ? 4 : 0;
        uint32_t c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = ((q[i] >> sh) & 0x0F0F0F0Fu) | (((h[i] >> j) & 0x01010101u) << 4);
        emit_affine(c, splat_h2(d1), splat_h2(mm), o);
    }
};

template <> struct Deq16<T_Q6_K> {
    uint32_t ql[4], qh[4], d;
    int k;
    __device__ __forceinline__ void pin_all() { pin(ql); pin(qh); pin(d); }
    __device__ __forceinline__ void load(const uint8_t *row, int k0) {
        const uint8_t *b = row + (k0 >> 8) * 210;
        const int w = k0 & 255, hh = w >> 7, r = w & 127, l0 = r & 31;
        k = r >> 5;
        ld16(b + 64 * hh + l0 + 32 * (k & 1), ql);
        ld16(b + 128 + 32 * hh + l0, qh);
        const uint32_t sc = b[192 + 8 * hh + (l0 >> 4) + 2 * k];   // int8 scale of these 16
        d = (uint32_t)ld2(b + 208) | (sc << 16);
    }
    __device__ __forceinline__ void emit(uint32_t o[8]) const {
        const float ds = h2f((uint16_t)d) * (float)(int8_t)(d >> 16);
        const int sh = (k >> 1) * 4, hs = 2 * k;
        uint32_t c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = ((ql[i] >> sh) & 0x0F0F0F0Fu) | (((qh[i] >> hs) & 0x03030303u) << 4);
        emit_scaled<32>(c, splat_h2(ds), o);
    }
};

// ------------------------------------------------------------------------------------------
// activations: f32 (strided) -> f16 [slice][M][Kpad]; per-token power-of-two prescale puts the
// largest |x| in (2^13, 2^14] (no f16 overflow, no subnormals); xinv[slice][M] undoes it
// ------------------------------------------------------------------------------------------
// one wave per token: float4 loads (scalar when src1 rows are not 16-B aligned), 8-B stores
__global__ __launch_bounds__(256) void mmq_convert_x(const MmArgs a, _Float16 *x16, float *xinv, int Kpad) {
    const int lane = threadIdx.x & 63;
    const int tok = blockIdx.x * 4 + (threadIdx.x >> 6), slice = blockIdx.y;
    if (tok >= a.M) return;   // whole wave; no barriers below
    const int i12 = slice % a.ne12, i13 = slice / a.ne12;
    const float *src = reinterpret_cast<const float *>(a.x + (int64_t)i12 * a.nb12 + (int64_t)i13 * a.nb13 +
                                                       (int64_t)tok * a.nb11);
    auto ld4f = [&](int k) -> float4 {
        if (a.x_aligned16) return *reinterpret_cast<const float4 *>(src + k);
        return make_float4(src[k], src[k + 1], src[k + 2], src[k + 3]);
    };
    float amax = 0.f;
    for (int k = lane * 4; k < a.K; k += 256) {   // K % 32 == 0
        const float4 v = ld4f(k);
        amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    amax = fmaxf(amax, xchg<1>(amax));
    amax = fmaxf(amax, xchg<2>(amax));
    amax = fmaxf(amax, xchg<4>(amax));
    amax = fmaxf(amax, xchg<8>(amax));
    amax = fmaxf(amax, xchg<16>(amax));
    amax = fmaxf(amax, xchg<32>(amax));
    const int e = amax > 0.f ? (int)ceilf(log2f(amax)) - 14 : 0;
    const float s = ldexpf(1.f, -e);
    _Float16 *dst = x16 + ((int64_t)slice * a.M + tok) * Kpad;
    for (int k = lane * 4; k < Kpad; k += 256) {
        const float4 v = k < a.K ? ld4f(k) : make_float4(0.f, 0.f, 0.f, 0.f);
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<h4 *>(dst + k) = h4{(_Float16)(v.x * s), (_Float16)(v.y * s), (_Float16)(v.z * s), (_Float16)(v.w * s)};
    }
    if (lane == 0) xinv[(int64_t)slice * a.M + tok] = ldexpf(1.f, e);
}

// byte offset of 16-B chunk c of LDS row r (128-B rows, XOR swizzle over row pairs)
__device__ __forceinline__ int swz(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// ------------------------------------------------------------------------------------------
// the tile kernel
// ------------------------------------------------------------------------------------------
template <int T, int BM, int BN>
__global__ __launch_bounds__(MQ_THREADS) void mmq_kernel(const MmArgs a, const _Float16 *__restrict__ x16,
                                                         const float *__restrict__ xinv, int Kpad) {
    constexpr int U = BM / 64;          // 16-weight units per thread per step
    constexpr int V = BN / 32;          // 16-B activation chunks per thread per step
    constexpr int TM = BM / 64;         // MFMA tiles per wave along weight rows
    constexpr int TN = BN / 64;         // MFMA tiles per wave along tokens
    constexpr int BUF = (BM + BN) * 128;
    __shared__ __align__(16) uint8_t lds[2 * BUF];

    const int slice = blockIdx.z;
    const int i12 = slice % a.ne12, i13 = slice / a.ne12;
    const uint8_t *wmat = a.w + (int64_t)(i12 / a.r2) * a.nb02 + (int64_t)(i13 / a.r3) * a.nb03;
    const _Float16 *xs = x16 + (int64_t)slice * a.M * Kpad;
    uint8_t *dmat = a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3;

    const int wrow0 = blockIdx.x * BM;
    const int tok0 = blockIdx.y * BN;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int nsteps = Kpad / MQ_BK;

    // staging roles (dead rows / tokens are clamped: they only feed outputs that are not stored)
    const uint8_t *w_row[U];
    int w_r[U], w_c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int g = tid + MQ_THREADS * u;
        w_r[u] = g >> 2;
        w_c[u] = (g & 3) * 16;
        w_row[u] = wmat + (int64_t)min(wrow0 + w_r[u], a.N - 1) * a.nb01;
    }
    const u32x4 *x_src[V];
    int x_r[V], x_c[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int g = tid + MQ_THREADS * v;
        x_r[v] = g >> 3;
        x_c[v] = g & 7;
        x_src[v] = reinterpret_cast<const u32x4 *>(xs + (int64_t)min(tok0 + x_r[v], a.M - 1) * Kpad) + x_c[v];
    }

    // one ring slot: raw weight units + activation chunks of one K-step
    auto load = [&](Deq16<T> (&w)[U], u32x4 (&x)[V], int step) {
        const int k0 = step * MQ_BK;
#pragma unroll
        for (int v = 0; v < V; ++v) x[v] = x_src[v][k0 / 8];
#pragma unroll
        for (int u = 0; u < U; ++u) w[u].load(w_row[u], min(k0 + w_c[u], a.K - 16));
    };
    auto store = [&](Deq16<T> (&w)[U], u32x4 (&x)[V], int step, int buf) {
        const int k0 = step * MQ_BK;
#pragma unroll
        for (int v = 0; v < V; ++v) pin(x[v]);
#pragma unroll
        for (int u = 0; u < U; ++u) w[u].pin_all();
        uint8_t *W = lds + buf * BUF;
        uint8_t *X = W + BM * 128;
#pragma unroll
        for (int v = 0; v < V; ++v) *reinterpret_cast<u32x4 *>(X + swz(x_r[v], x_c[v])) = x[v];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint32_t o[8];
            w[u].emit(o);
            if (k0 + w_c[u] >= a.K) {   // ragged K tail (32-block types): zero weights
#pragma unroll
                for (int i = 0; i < 8; ++i) o[i] = 0;
            }
            *reinterpret_cast<u32x4 *>(W + swz(w_r[u], w_c[u] / 8)) = u32x4{o[0], o[1], o[2], o[3]};
            *reinterpret_cast<u32x4 *>(W + swz(w_r[u], w_c[u] / 8 + 1)) = u32x4{o[4], o[5], o[6], o[7]};
        }
    };

    float16v acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int fr = lane & 31, fh = lane >> 5;
    auto compute = [&](int buf) {
        const uint8_t *W = lds + buf * BUF;
        const uint8_t *X = W + BM * 128;
#pragma unroll
        for (int ks = 0; ks < MQ_BK / 16; ++ks) {
            const int c = 2 * ks + fh;
            half8 bw[TM], ax[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                bw[i] = *reinterpret_cast<const half8 *>(W + swz(wm * (BM / 2) + 32 * i + fr, c));
#pragma unroll
            for (int j = 0; j < TN; ++j)
                ax[j] = *reinterpret_cast<const half8 *>(X + swz(wn * (BN / 2) + 32 * j + fr, c));
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax[j], bw[i], acc[i][j], 0, 0, 0);
        }
    };

    // 2-deep register ring: loads for step s+2 are issued before the MFMAs of step s and
    // written to LDS after those of step s+1. Loads and stores are unconditional (clamped step)
    // so the compiler keeps counted vmcnt waits instead of draining the ring.
    Deq16<T> wa[U], wb[U];
    u32x4 xa[V], xb[V];
    load(wa, xa, 0);
    load(wb, xb, min(1, nsteps - 1));
    store(wa, xa, 0, 0);
    __syncthreads();
    int s = 0;
    // sched_barrier pins the phases: without it the scheduler hoists the decode of the slot just
    // loaded into the current phase and waits vmcnt(0) for it, collapsing the ring to depth 1
    for (; s + 1 < nsteps; s += 2) {
        load(wa, xa, min(s + 2, nsteps - 1));
        __builtin_amdgcn_sched_barrier(0);
        compute(0);
        __builtin_amdgcn_sched_barrier(0);
        store(wb, xb, s + 1, 1);
        __syncthreads();
        load(wb, xb, min(s + 3, nsteps - 1));
        __builtin_amdgcn_sched_barrier(0);
        compute(1);
        __builtin_amdgcn_sched_barrier(0);
        store(wa, xa, s + 2, 0);
        __syncthreads();
    }
    if (s < nsteps) compute(0);   // odd step count: the last step sits in buffer 0

    // epilogue: lane holds weight row (lane & 31) of each B tile and 16 tokens of each A tile;
    // token scales are read before any store (dst may alias nothing, but the compiler cannot know)
    float inv[TN][16];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int tok = tok0 + wn * (BN / 2) + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * fh;
            inv[j][r] = xinv[(int64_t)slice * a.M + min(tok, a.M - 1)];
        }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int orow = wrow0 + wm * (BM / 2) + 32 * i + fr;
        if (orow >= a.N) continue;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int tok = tok0 + wn * (BN / 2) + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * fh;
                if (tok < a.M) reinterpret_cast<float *>(dmat + (int64_t)tok * a.nb1)[orow] = acc[i][j][r] * inv[j][r];
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
bool mmq_supported(int type, const MmArgs &a) {
    (void)a;
    return type == T_Q4_0 || type == T_Q8_0 || type == T_Q4_K || type == T_Q5_K || type == T_Q6_K;
}

template <int T, int BM, int BN>
static void launch_tile(const MmArgs &a, const _Float16 *x16, const float *xinv, int Kpad, int slices, hipStream_t st) {
    const dim3 grid((a.N + BM - 1) / BM, (a.M + BN - 1) / BN, slices);
    hipLaunchKernelGGL((mmq_kernel<T, BM, BN>), grid, dim3(MQ_THREADS), 0, st, a, x16, xinv, Kpad);
}

template <int T>
static void launch_type(int tile, const MmArgs &a, const _Float16 *x16, const float *xinv, int Kpad, int slices,
                        hipStream_t st) {
    switch (tile) {
        case 0: launch_tile<T, 64, 128>(a, x16, xinv, Kpad, slices, st); break;
        case 1: launch_tile<T, 128, 64>(a, x16, xinv, Kpad, slices, st); break;
        default: launch_tile<T, 128, 128>(a, x16, xinv, Kpad, slices, st); break;
    }
}

// tile shape: the largest tile that still gives every CU a workgroup; GGML_MI355X_MMQ_TILE
// (64x128 | 128x64 | 128x128) overrides it for measurements
static int pick_tile(const MmArgs &a, int slices) {
    static const char *env = getenv("GGML_MI355X_MMQ_TILE");
    if (env) {
        if (!strcmp(env, "64x128")) return 0;
        if (!strcmp(env, "128x64")) return 1;
        if (!strcmp(env, "128x128")) return 2;
    }
    auto wgs = [&](int bm, int bn) { return (int64_t)((a.N + bm - 1) / bm) * ((a.M + bn - 1) / bn) * slices; };
    if (wgs(128, 128) >= 256) return 2;
    return a.M <= 64 ? 1 : (wgs(128, 64) >= 256 ? 1 : 0);
}

hipError_t mmq_launch(int type, const MmArgs &a, hipStream_t st, Scratch &scratch) {
    const int Kpad = (a.K + MQ_BK - 1) / MQ_BK * MQ_BK;
    const int slices = a.ne12 * a.ne13;
    const size_t x16_bytes = ((size_t)slices * a.M * Kpad * sizeof(_Float16) + 255) & ~(size_t)255;
    const size_t inv_bytes = (size_t)slices * a.M * sizeof(float);
    uint8_t *buf = static_cast<uint8_t *>(scratch.get(x16_bytes + inv_bytes, st));
    if (!buf) return hipErrorOutOfMemory;
    _Float16 *x16 = reinterpret_cast<_Float16 *>(buf);
    float *xinv = reinterpret_cast<float *>(buf + x16_bytes);
    hipLaunchKernelGGL(mmq_convert_x, dim3((a.M + 3) / 4, slices), dim3(256), 0, st, a, x16, xinv, Kpad);
    const int tile = pick_tile(a, slices);
    switch (type) {
        case T_Q4_0: launch_type<T_Q4_0>(tile, a, x16, xinv, Kpad, slices, st); break;
        case T_Q8_0: launch_type<T_Q8_0>(tile, a, x16, xinv, Kpad, slices, st); break;
        case T_Q4_K: launch_type<T_Q4_K>(tile, a, x16, xinv, Kpad, slices, st); break;
        case T_Q5_K: launch_type<T_Q5_K>(tile, a, x16, xinv, Kpad, slices, st); break;
        case T_Q6_K: launch_type<T_Q6_K>(tile, a, x16, xinv, Kpad, slices, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace mi355x
