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
constexpr int MQ_THREADS = 512;

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

// ------------------------------------------------------------------------------------------
// 8-weight dequant units: raw registers loaded ahead through a buffer resource (32-bit offsets,
// out-of-range reads return zero), decoded at LDS-store time (emit -> one 16-B f16 chunk).
// Formulas restate src/ggml-quants.c dequantize_row_* (:307, :401, :1352, :1554, :1762).
// ------------------------------------------------------------------------------------------
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void pin(u32x2 &v) { asm volatile("" : "+v"(v)); }

__device__ __forceinline__ u32x4 bl128(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ u32x2 bl64(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t bl16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t bl8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
}

// 8 byte codes (2 dwords) -> 8 f16 weights (c - bias) * d; one rounding of the exact product
template <int BIAS>
__device__ __forceinline__ u32x4 emit8_scaled(uint32_t c0, uint32_t c1, h2v d) {
    const h2v bias = splat_h2(1024.f + BIAS);
    uint32_t l0, h0, l1, h1;
    bytes_f16(c0, l0, h0);
    bytes_f16(c1, l1, h1);
    return u32x4{as_u((as_h2(l0) - bias) * d), as_u((as_h2(h0) - bias) * d), as_u((as_h2(l1) - bias) * d),
                 as_u((as_h2(h1) - bias) * d)};
}
// 8 byte codes -> c * d1 - m1 (K-quant affine form)
__device__ __forceinline__ u32x4 emit8_affine(uint32_t c0, uint32_t c1, h2v d1, h2v m1) {
    const h2v bias = splat_h2(1024.f);
    uint32_t l0, h0, l1, h1;
    bytes_f16(c0, l0, h0);
    bytes_f16(c1, l1, h1);
    auto f = [&](uint32_t v) { return as_u(__builtin_elementwise_fma(as_h2(v) - bias, d1, -m1)); };
    return u32x4{f(l0), f(h0), f(l1), f(h1)};
}

template <int T> struct Deq8;

template <> struct Deq8<T_Q4_0> {
    u32x2 q;
    uint32_t d;
    int sh;
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t row, int k0) {
        const uint32_t b = row + (uint32_t)(k0 >> 5) * 18;
        d = bl16(r, b);
        q = bl64(r, b + 2 + (k0 & 15));
        sh = (k0 & 16) ? 4 : 0;
    }
    __device__ __forceinline__ void pin_all() { pin(q); pin(d); }
    __device__ __forceinline__ u32x4 emit() const {
        return emit8_scaled<8>((q[0] >> sh) & 0x0F0F0F0Fu, (q[1] >> sh) & 0x0F0F0F0Fu, splat_h2(h2f((uint16_t)d)));
    }
};

template <> struct Deq8<T_Q8_0> {
    u32x2 q;
    uint32_t d;
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t row, int k0) {
        const uint32_t b = row + (uint32_t)(k0 >> 5) * 34;
        d = bl16(r, b);
        q = bl64(r, b + 2 + (k0 & 31));
    }
    __device__ __forceinline__ void pin_all() { pin(q); pin(d); }
    __device__ __forceinline__ u32x4 emit() const {   // int8 -> 128 + q
        return emit8_scaled<128>(q[0] ^ 0x80808080u, q[1] ^ 0x80808080u, splat_h2(h2f((uint16_t)d)));
    }
};

// Q4_K / Q5_K header: d, dmin (fp16) and the 12 packed 6-bit scale/min bytes -> (d*sc, dmin*m)
// of sub-block j (get_scale_min_k4, src/ggml-quants.c:703-710)
__device__ __forceinline__ void k4_sub_scale(const u32x4 &hd, int j, h2v &d1, h2v &m1) {
    const uint32_t S[3] = {hd[1], hd[2], hd[3]};
    uint32_t sc0, sc1, m0, m1v;
    k4_scale_min_pair(S, j >> 1, sc0, sc1, m0, m1v);
    const bool hi = j & 1;
    d1 = splat_h2(h2f((uint16_t)hd[0]) * (float)(hi ? sc1 : sc0));
    m1 = splat_h2(h2f((uint16_t)(hd[0] >> 16)) * (float)(hi ? m1v : m0));
}

template <> struct Deq8<T_Q4_K> {
    u32x4 hd;
    u32x2 q;
    int j;
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t row, int k0) {
        const uint32_t b = row + (uint32_t)(k0 >> 8) * 144;
        const int w = k0 & 255;
        j = w >> 5;
        hd = bl128(r, b);
        q = bl64(r, b + 16 + 32 * (w >> 6) + (w & 31));
    }
    __device__ __forceinline__ void pin_all() { pin(hd); pin(q); }
    __device__ __forceinline__ u32x4 emit() const {
        h2v d1, m1;
        k4_sub_scale(hd, j, d1, m1);
        const int sh = (j & 1) * 4;
        return emit8_affine((q[0] >> sh) & 0x0F0F0F0Fu, (q[1] >> sh) & 0x0F0F0F0Fu, d1, m1);
    }
};

template <> struct Deq8<T_Q5_K> {
    u32x4 hd;
    u32x2 q, h;
    int j;
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t row, int k0) {
        const uint32_t b = row + (uint32_t)(k0 >> 8) * 176;
        const int w = k0 & 255;
        j = w >> 5;
        hd = bl128(r, b);
        h = bl64(r, b + 16 + (w & 31));
        q = bl64(r, b + 48 + 32 * (w >> 6) + (w & 31));
    }
    __device__ __forceinline__ void pin_all() { pin(hd); pin(q); pin(h); }
    __device__ __forceinline__ u32x4 emit() const {
        h2v d1, m1;
        k4_sub_scale(hd, j, d1, m1);
        const int sh = (j & 1) * 4;
        const uint32_t c0 = ((q[0] >> sh) & 0x0F0F0F0Fu) | (((h[0] >> j) & 0x01010101u) << 4);
        const uint32_t c1 = ((q[1] >> sh) & 0x0F0F0F0Fu) | (((h[1] >> j) & 0x01010101u) << 4);
        return emit8_affine(c0, c1, d1, m1);
    }
};

template <> struct Deq8<T_Q6_K> {
    u32x2 ql, qh;
    uint32_t d, sc;
    int k;
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t row, int k0) {
        const uint32_t b = row + (uint32_t)(k0 >> 8) * 210;
        const int w = k0 & 255, hh = w >> 7, rr = w & 127, l = rr & 31;
        k = rr >> 5;
        ql = bl64(r, b + 64 * hh + l + 32 * (k & 1));
        qh = bl64(r, b + 128 + 32 * hh + l);
        sc = bl8(r, b + 192 + 8 * hh + (l >> 4) + 2 * k);   // int8 scale of this 16-group
        d = bl16(r, b + 208);
    }
    __device__ __forceinline__ void pin_all() { pin(ql); pin(qh); pin(d); pin(sc); }
    __device__ __forceinline__ u32x4 emit() const {
        const float ds = h2f((uint16_t)d) * (float)(int8_t)sc;
        const int sh = (k >> 1) * 4, hs = 2 * k;
        const uint32_t c0 = ((ql[0] >> sh) & 0x0F0F0F0Fu) | (((qh[0] >> hs) & 0x03030303u) << 4);
        const uint32_t c1 = ((ql[1] >> sh) & 0x0F0F0F0Fu) | (((qh[1] >> hs) & 0x03030303u) << 4);
        return emit8_scaled<32>(c0, c1, splat_h2(ds));
    }
};

// ------------------------------------------------------------------------------------------
// activations: f32 (strided) -> f16 [slice][M][Kpad]; per-token power-of-two prescale puts the
// largest |x| in (2^13, 2^14] (no f16 overflow, no subnormals); xinv[slice][M] undoes it
// ------------------------------------------------------------------------------------------
// one workgroup per token (K spread over 256 threads, 4 float4 loads in flight per thread);
// scalar loads when src1 rows are not 16-B aligned; 8-B stores
// MUL_MAT_ID grouping (expert-sorted (slot, token) pairs), built on the device by moe_prep:
//   offsets[e] .. offsets[e+1]  : sorted positions of expert e's pairs
//   tile_off[e]                 : first token tile of expert e (prefix sum of ceil(count / BN))
//   pos_pair[pos]               : pair index t * n_used + slot at sorted position pos
struct MoeMap {
    const int *offsets, *tile_off, *pos_pair;
    int n_expert, n_used;
};

// pos_pair == nullptr: plain MUL_MAT (row tok of slice blockIdx.y); otherwise row pos of the
// expert-sorted pair list, gathered from src1 column (slot % ne11, token)
__global__ __launch_bounds__(256) void mmq_convert_x(const MmArgs a, _Float16 *x16, float *xinv, int Kpad,
                                                     const int *pos_pair) {
    const int tok = blockIdx.x, slice = blockIdx.y;
    const float *src;
    if (pos_pair) {
        const int pair = pos_pair[tok];
        const int slot = pair % a.n_used, t = pair / a.n_used;
        src = reinterpret_cast<const float *>(a.x + (int64_t)(slot % a.ne11_b) * a.nb11 + (int64_t)t * a.nb12);
    } else {
        const int i12 = slice % a.ne12, i13 = slice / a.ne12;
        src = reinterpret_cast<const float *>(a.x + (int64_t)i12 * a.nb12 + (int64_t)i13 * a.nb13 + (int64_t)tok * a.nb11);
    }
    auto ld4f = [&](int k) -> float4 {
        if (k >= a.K) return make_float4(0.f, 0.f, 0.f, 0.f);   // K % 4 == 0
        if (a.x_aligned16) return *reinterpret_cast<const float4 *>(src + k);
        return make_float4(src[k], src[k + 1], src[k + 2], src[k + 3]);
    };
    const int t4 = threadIdx.x * 4;
    float amax = 0.f;
    for (int k0 = 0; k0 < a.K; k0 += 4096) {
        float4 v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = ld4f(k0 + 1024 * i + t4);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v[i].x), fabsf(v[i].y)), fmaxf(fabsf(v[i].z), fabsf(v[i].w))));
    }
    amax = fmaxf(amax, xchg<1>(amax));
    amax = fmaxf(amax, xchg<2>(amax));
    amax = fmaxf(amax, xchg<4>(amax));
    amax = fmaxf(amax, xchg<8>(amax));
    amax = fmaxf(amax, xchg<16>(amax));
    amax = fmaxf(amax, xchg<32>(amax));
    __shared__ float red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const int e = amax > 0.f ? (int)ceilf(log2f(amax)) - 14 : 0;
    const float s = ldexpf(1.f, -e);
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    _Float16 *dst = x16 + ((int64_t)slice * a.M + tok) * Kpad;
    for (int k0 = 0; k0 < Kpad; k0 += 4096) {
        float4 v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = ld4f(k0 + 1024 * i + t4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = k0 + 1024 * i + t4;
            if (k < Kpad)
                *reinterpret_cast<h4 *>(dst + k) =
                    h4{(_Float16)(v[i].x * s), (_Float16)(v[i].y * s), (_Float16)(v[i].z * s), (_Float16)(v[i].w * s)};
        }
    }
    if (threadIdx.x == 0) xinv[(int64_t)slice * a.M + tok] = ldexpf(1.f, e);
}

// byte offset of 16-B chunk c of LDS row r (128-B rows, XOR swizzle over row pairs)
__device__ __forceinline__ int swz(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// ------------------------------------------------------------------------------------------
// the tile kernel: 8 waves (two per SIMD, so one wave's dequant VALU overlaps the other's
// MFMAs), wave grid (BM/32) x (8/(BM/32)), wave tile 32 weight rows x TN*32 tokens.
//
// Per K-step (BK = 64) of phase s:
//   1. weight units of step s+2 -> registers (buffer loads, 2 register slots)
//   2. activations of step s+2 -> LDS X ring slot (s+2)%3 by LDS-DMA (buffer_load ... lds):
//      no VGPR round trip and no ds_write issue cost (the ds_write path, ~80 B/clk/CU, was the
//      bottleneck of register staging); the 16-B XOR swizzle is applied on the source address
//   3. MFMAs of step s from W slot s%2 and X slot s%3
//   4. decode the weight units of step s+1 (loaded one phase ago) into W slot (s+1)%2
//   5. s_waitcnt vmcnt(<this phase's loads>) retires the DMA of step s+1, then one barrier
// ------------------------------------------------------------------------------------------
constexpr uint32_t RSRC_W3 = 0x00020000u;   // raw buffer, dword3 for gfx9-class descriptors

template <int T> struct LoadsPerUnit;   // VMEM instructions one Deq8<T>::load issues
template <> struct LoadsPerUnit<T_Q4_0> { static constexpr int n = 2; };
template <> struct LoadsPerUnit<T_Q8_0> { static constexpr int n = 2; };
template <> struct LoadsPerUnit<T_Q4_K> { static constexpr int n = 2; };
template <> struct LoadsPerUnit<T_Q5_K> { static constexpr int n = 3; };
template <> struct LoadsPerUnit<T_Q6_K> { static constexpr int n = 4; };

template <int N> __device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef __attribute__((address_space(3))) void *lds_ptr_t;

// 16 B per lane from the buffer straight into LDS at lds_dst + 16 * lane (lds_dst wave-uniform).
// (A plain device function: used directly inside the kernel's lambdas, this builtin makes the
// ROCm 7.2 host pass drop the kernel's launch stub.)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint8_t *lds_dst, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds_dst, 16, voff, 0, 0, 0);
}

// NW waves per workgroup; each wave owns TM x TN MFMA tiles of 32 x 32 (weight rows x tokens).
// TM = TN = 2 (64 x 64 per wave) reads one LDS fragment per MFMA instead of two.
template <int T, int BM, int BN, bool STAMP = false, bool IDS = false, int NW = 8, int TM = 1>
__global__ __launch_bounds__(NW * 64) void mmq_kernel(const MmArgs a, const _Float16 *__restrict__ x16,
                                                      const float *__restrict__ xinv, int Kpad, uint32_t w_extent,
                                                      const MoeMap moe) {
    constexpr int THREADS = NW * 64;
    constexpr int WGM = BM / (32 * TM);          // waves along weight rows
    constexpr int WGN = NW / WGM;                // waves along tokens
    constexpr int TN = BN / WGN / 32;            // MFMA tiles per wave along tokens
    constexpr int U = BM * 8 / THREADS;          // 8-weight units per thread per step
    constexpr int V = BN / 8 / NW;               // 1-KiB activation pieces per wave per step
    constexpr int WB = BM * 128, XB = BN * 128;  // bytes of one W / X slot
    constexpr int VM_PHASE = U * LoadsPerUnit<T>::n + V;   // VMEM ops one wave issues per phase
    static_assert(WGM * WGN == NW && TN >= 1 && U >= 1 && V >= 1 && VM_PHASE < 64, "tile shape");
    __shared__ __align__(16) uint8_t lds[2 * WB + 3 * XB];   // one array: see the .s traps in the guide
    uint8_t *const wslot = lds;
    uint8_t *const xslot = lds + 2 * WB;

    const int slice = blockIdx.z;
    const int i12 = slice % a.ne12, i13 = slice / a.ne12;
    const uint8_t *wmat;
    const _Float16 *xs;
    uint8_t *dmat;
    int tok0, tok_end;   // token rows [tok0, tok_end) of xs feed this workgroup
    if constexpr (IDS) {
        // grid.y is an upper bound on the token tiles of all experts; tile -> expert by a search
        // of the prefix sums (empty experts share their successor's start, so "last e with
        // tile_off[e] <= tile" is the non-empty one)
        const int tile = blockIdx.y;
        if (tile >= moe.tile_off[moe.n_expert]) return;   // whole workgroup, before any barrier
        int lo = 0, hi = moe.n_expert - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (moe.tile_off[mid] <= tile) lo = mid; else hi = mid - 1;
        }
        wmat = a.w + (int64_t)lo * a.nb02;
        xs = x16;
        dmat = a.dst;
        tok0 = moe.offsets[lo] + (tile - moe.tile_off[lo]) * BN;
        tok_end = moe.offsets[lo + 1];
    } else {
        wmat = a.w + (int64_t)(i12 / a.r2) * a.nb02 + (int64_t)(i13 / a.r3) * a.nb03;
        xs = x16 + (int64_t)slice * a.M * Kpad;
        dmat = a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3;
        tok0 = blockIdx.y * BN;
        tok_end = a.M;
    }
    // rows past N and tokens past tok_end read as zeros (buffer range check)
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void *)wmat, 0, w_extent, RSRC_W3);
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc((void *)xs, 0, (uint32_t)tok_end * (uint32_t)Kpad * 2u, RSRC_W3);

    const int wrow0 = blockIdx.x * BM;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave % WGM, wn = wave / WGM;
    const int nsteps = Kpad / MQ_BK;
    // diagnostic build only (GGML_MI355X_STAMPS): per-wave s_memtime cycles spent in each phase
    uint64_t st_seg[5] = {0, 0, 0, 0, 0}, st_t = 0, st_start = 0;
    auto stamp = [&](int seg) {
        if constexpr (STAMP) {
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t t = __builtin_amdgcn_s_memtime();
            if (seg >= 0) st_seg[seg] += t - st_t;
            st_t = t;
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    stamp(-1);
    st_start = st_t;

    uint32_t w_row[U];
    int w_r[U], w_c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int g = tid + THREADS * u;
        w_r[u] = g >> 3;
        w_c[u] = (g & 7) * 8;
        w_row[u] = (uint32_t)(wrow0 + w_r[u]) * (uint32_t)a.nb01;
    }
    // activation pieces: wave piece p = wave + 8v covers tile rows 8p..8p+7; lane -> (row, LDS
    // chunk lane&7) fetching the global chunk that the swizzle maps there
    uint32_t x_off[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int r = 8 * (wave + NW * v) + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        x_off[v] = ((uint32_t)(tok0 + r) * (uint32_t)Kpad + (uint32_t)c * 8u) * 2u;
    }

    auto load_w = [&](Deq8<T> (&w)[U], int step) {
        const int k0 = step * MQ_BK;
        // the K tail of the 32-block types re-reads the row's last unit: finite weights times
        // the zero-padded activations contribute exactly 0
#pragma unroll
        for (int u = 0; u < U; ++u) w[u].load(wr, w_row[u], min(k0 + w_c[u], a.K - 8));
    };
    auto dma_x = [&](int step, int slot) {
        const uint32_t k2 = (uint32_t)step * MQ_BK * 2u;
#pragma unroll
        for (int v = 0; v < V; ++v)
            dma16(xr, xslot + slot * XB + (wave + NW * v) * 1024, x_off[v] + k2);
    };
    auto store_w = [&](Deq8<T> (&w)[U], int slot) {
#pragma unroll
        for (int u = 0; u < U; ++u) w[u].pin_all();
        uint8_t *W = wslot + slot * WB;
#pragma unroll
        for (int u = 0; u < U; ++u)
            *reinterpret_cast<u32x4 *>(W + swz(w_r[u], w_c[u] / 8)) = w[u].emit();
    };

    float16v acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int fr = lane & 31, fh = lane >> 5;
    auto compute = [&](int wsl, int xsl) {
        const uint8_t *W = wslot + wsl * WB;
        const uint8_t *X = xslot + xsl * XB;
#pragma unroll
        for (int ks = 0; ks < MQ_BK / 16; ++ks) {
            const int c = 2 * ks + fh;
            half8 bw[TM], ax[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                bw[i] = *reinterpret_cast<const half8 *>(W + swz(wm * (TM * 32) + 32 * i + fr, c));
#pragma unroll
            for (int j = 0; j < TN; ++j)
                ax[j] = *reinterpret_cast<const half8 *>(X + swz(wn * (TN * 32) + 32 * j + fr, c));
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax[j], bw[i], acc[i][j], 0, 0, 0);
        }
    };
    auto barrier = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's ds_writes landed
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    Deq8<T> wa[U], wb[U];
    // prologue: steps 0 and 1 in flight, step 0 decoded
    load_w(wa, 0);
    dma_x(0, 0);
    load_w(wb, min(1, nsteps - 1));
    dma_x(min(1, nsteps - 1), 1);
    __builtin_amdgcn_sched_barrier(0);
    store_w(wa, 0);
    wait_vmcnt<VM_PHASE>();   // retires step 0's DMA
    barrier();

    // phase body; W register slot parity is static (loop unrolled by 2), X slots rotate by 3
    auto phase = [&](Deq8<T> (&wnext)[U], Deq8<T> (&wdec)[U], int s, int xs0) {
        const int xs1 = xs0 == 2 ? 0 : xs0 + 1, xs2 = xs1 == 2 ? 0 : xs1 + 1;
        stamp(4);
        // the raw units of step s+1 arrived during the previous phase: take them now, so their
        // decode VALU is interleaved by the scheduler with this step's MFMAs (+2-6 % measured)
#pragma unroll
        for (int u = 0; u < U; ++u) wdec[u].pin_all();
        load_w(wnext, min(s + 2, nsteps - 1));
        dma_x(min(s + 2, nsteps - 1), xs2);
        __builtin_amdgcn_sched_barrier(0);
        stamp(0);
        u32x4 dec[U];
#pragma unroll
        for (int u = 0; u < U; ++u) dec[u] = wdec[u].emit();
        compute(s & 1, xs0);
        uint8_t *W = wslot + ((s + 1) & 1) * WB;
#pragma unroll
        for (int u = 0; u < U; ++u) *reinterpret_cast<u32x4 *>(W + swz(w_r[u], w_c[u] / 8)) = dec[u];
        stamp(1);
        stamp(2);
        wait_vmcnt<VM_PHASE>();   // retires step s+1's DMA (issued one phase ago)
        stamp(3);
        barrier();
        return xs1;
    };
    int s = 0, xsl = 0;
    for (; s + 1 < nsteps; s += 2) {
        xsl = phase(wa, wb, s, xsl);
        xsl = phase(wb, wa, s + 1, xsl);
    }
    if (s < nsteps) compute(s & 1, xsl);   // odd step count: the last step
    wait_vmcnt<0>();   // no LDS-DMA may still be landing when the workgroup's LDS is released
    stamp(4);
    if constexpr (STAMP) {
        if (lane == 0 && a.stamps) {
            const int g = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
            unsigned long long *o = a.stamps + ((size_t)g * 8 + wave) * 8;
            o[0] = st_start;
            for (int i = 0; i < 5; ++i) o[1 + i] = st_seg[i];
            o[6] = st_t;
            o[7] = nsteps;
        }
    }

    // epilogue: lane holds weight row (lane & 31) and 16 tokens of each A tile; token scales are
    // read before any store (the compiler cannot prove dst does not alias them)
    const float *xinv_s = IDS ? xinv : xinv + (int64_t)slice * a.M;
    float inv[TN][16];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int tok = tok0 + wn * (TN * 32) + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * fh;
            inv[j][r] = xinv_s[min(tok, tok_end - 1)];
        }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
    const int orow = wrow0 + wm * (TM * 32) + 32 * i + fr;
    if (orow < a.N) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int tok = tok0 + wn * (TN * 32) + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * fh;
                if (tok < tok_end) {
                    uint8_t *drow;
                    if constexpr (IDS) {   // scatter back to dst[slot][token]
                        const int pair = moe.pos_pair[tok];
                        drow = dmat + (int64_t)(pair % moe.n_used) * a.nb1 + (int64_t)(pair / moe.n_used) * a.nb2;
                    } else {
                        drow = dmat + (int64_t)tok * a.nb1;
                    }
                    reinterpret_cast<float *>(drow)[orow] = acc[i][j][r] * inv[j][r];
                }
            }
        }
    }
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
static int64_t row_bytes(int type, int K) { return (int64_t)K / type_blck(type) * type_bytes(type); }

// buffer offsets are 32-bit: one weight matrix (plus a tile of rows past its end) and one
// slice of converted activations must each stay below 4 GiB; larger problems use the mat-vec
bool mmq_supported(int type, const MmArgs &a) {
    if (!(type == T_Q4_0 || type == T_Q8_0 || type == T_Q4_K || type == T_Q5_K || type == T_Q6_K)) return false;
    const int64_t kpad = (a.K + MQ_BK - 1) / MQ_BK * MQ_BK;
    const int64_t w_span = (int64_t)(a.N + 128) * a.nb01 + row_bytes(type, a.K);
    return a.nb01 >= row_bytes(type, a.K) && w_span < (1LL << 32) && (int64_t)(a.M + 128) * kpad * 2 < (1LL << 32);
}

template <int T, int BM, int BN, int NW = 8, int TM = 1>
static void launch_tile(const MmArgs &a, const _Float16 *x16, const float *xinv, int Kpad, int slices, hipStream_t st) {
    const dim3 grid((a.N + BM - 1) / BM, (a.M + BN - 1) / BN, slices);
    const uint32_t w_extent = (uint32_t)((int64_t)(a.N - 1) * a.nb01 + row_bytes(T, a.K));
    const MoeMap none{};
    if (a.stamps && (size_t)grid.x * grid.y * grid.z * 64 <= 8 * 65536)
        hipLaunchKernelGGL((mmq_kernel<T, BM, BN, true, false, NW, TM>), grid, dim3(NW * 64), 0, st, a, x16, xinv, Kpad, w_extent, none);
    else
        hipLaunchKernelGGL((mmq_kernel<T, BM, BN, false, false, NW, TM>), grid, dim3(NW * 64), 0, st, a, x16, xinv, Kpad, w_extent, none);
}

template <int T>
static void launch_type(int tile, const MmArgs &a, const _Float16 *x16, const float *xinv, int Kpad, int slices,
                        hipStream_t st) {
    switch (tile) {
        case 0: launch_tile<T, 64, 128>(a, x16, xinv, Kpad, slices, st); break;
        case 1: launch_tile<T, 128, 64>(a, x16, xinv, Kpad, slices, st); break;
        case 3: launch_tile<T, 128, 128, 4, 2>(a, x16, xinv, Kpad, slices, st); break;
        case 4: launch_tile<T, 64, 128, 4, 1>(a, x16, xinv, Kpad, slices, st); break;
        default: launch_tile<T, 128, 128>(a, x16, xinv, Kpad, slices, st); break;
    }
}

// tile shape; GGML_MI355X_MMQ_TILE (64x128 | 128x64 | 128x128 | 128x128w4 | 64x128w4, the w4
// forms with 4 waves of 64 x 64 or 32 x 128 tiles) overrides it for measurements
static int pick_tile(const MmArgs &a, int slices) {
    static const char *env = getenv("GGML_MI355X_MMQ_TILE");
    if (env) {
        if (!strcmp(env, "64x128")) return 0;
        if (!strcmp(env, "128x64")) return 1;
        if (!strcmp(env, "128x128")) return 2;
        if (!strcmp(env, "128x128w4")) return 3;
        if (!strcmp(env, "64x128w4")) return 4;
    }
    auto wgs = [&](int bm, int bn) { return (int64_t)((a.N + bm - 1) / bm) * ((a.M + bn - 1) / bn) * slices; };
    // measured on MI355X (scripts/mmq_sweep.sh): 128x128 once it fills the chip, otherwise the
    // 64-row tile (twice the workgroups) unless there are too few tokens for 128-token tiles
    if (wgs(128, 128) >= 256) return 2;
    return a.M > 64 ? 0 : 1;
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
    hipLaunchKernelGGL(mmq_convert_x, dim3(a.M, slices), dim3(256), 0, st, a, x16, xinv, Kpad, (const int *)nullptr);
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

// ------------------------------------------------------------------------------------------
// MUL_MAT_ID on the MFMA tiles (prefill / many tokens): the (slot, token) pairs are grouped by
// expert on the device (counting sort in LDS), their activation columns gathered into f16 rows
// in that order, and every expert's rows run as token tiles of the same kernel; the epilogue
// scatters each row back to dst[slot][token]. No host synchronisation: grid.y is the upper
// bound ceil(P / BN) + n_expert and surplus workgroups exit at once. (Reference: the expert
// grouping of ggml_compute_forward_mul_mat_id, src/ggml-cpu/ggml-cpu.c:1564-1579, and
// ggml_cuda_mul_mat_id, src/ggml-cuda/ggml-cuda.cu:2092-2230.)
// ------------------------------------------------------------------------------------------
constexpr int MOE_MAX_EXPERTS = 1024;
constexpr int MOE_BN = 64;                // token tile of the grouped path (128 x 64 tiles)

__global__ __launch_bounds__(1024) void moe_prep(const MmArgs a, int *offsets, int *tile_off, int *pos_pair) {
    __shared__ int cnt[MOE_MAX_EXPERTS], cur[MOE_MAX_EXPERTS];
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
            tl += (cnt[e] + MOE_BN - 1) / MOE_BN;
        }
        offsets[E] = o;
        tile_off[E] = tl;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += 1024) pos_pair[atomicAdd(&cur[expert_of(p)], 1)] = p;
}

bool mmq_id_supported(int type, const MmArgs &a) {
    const int P = a.n_used * a.n_tok;
    MmArgs b = a;
    b.M = P;
    return a.n_expert <= MOE_MAX_EXPERTS && mmq_supported(type, b);
}

hipError_t mmq_id_launch(int type, const MmArgs &a, hipStream_t st, Scratch &scratch) {
    const int Kpad = (a.K + MQ_BK - 1) / MQ_BK * MQ_BK;
    const int P = a.n_used * a.n_tok, E = a.n_expert;
    const size_t x16_bytes = ((size_t)P * Kpad * sizeof(_Float16) + 255) & ~(size_t)255;
    const size_t inv_bytes = ((size_t)P * sizeof(float) + 255) & ~(size_t)255;
    const size_t map_bytes = sizeof(int) * (2 * (size_t)(E + 1) + P);
    uint8_t *buf = static_cast<uint8_t *>(scratch.get(x16_bytes + inv_bytes + map_bytes, st));
    if (!buf) return hipErrorOutOfMemory;
    _Float16 *x16 = reinterpret_cast<_Float16 *>(buf);
    float *xinv = reinterpret_cast<float *>(buf + x16_bytes);
    int *offsets = reinterpret_cast<int *>(buf + x16_bytes + inv_bytes);
    int *tile_off = offsets + (E + 1);
    int *pos_pair = tile_off + (E + 1);
    hipLaunchKernelGGL(moe_prep, dim3(1), dim3(1024), 0, st, a, offsets, tile_off, pos_pair);
    hipLaunchKernelGGL(mmq_convert_x, dim3(P, 1), dim3(256), 0, st, a, x16, xinv, Kpad, (const int *)pos_pair);
    const MoeMap moe{offsets, tile_off, pos_pair, E, a.n_used};
    const dim3 grid((a.N + 127) / 128, (P + MOE_BN - 1) / MOE_BN + E, 1);
    const uint32_t w_extent = (uint32_t)((int64_t)(a.N - 1) * a.nb01 + row_bytes(type, a.K));
    switch (type) {
#define MQ_ID(TT) case TT: hipLaunchKernelGGL((mmq_kernel<TT, 128, MOE_BN, false, true>), grid, dim3(MQ_THREADS), 0, st, a, x16, xinv, Kpad, w_extent, moe); break;
        MQ_ID(T_Q4_0) MQ_ID(T_Q8_0) MQ_ID(T_Q4_K) MQ_ID(T_Q5_K) MQ_ID(T_Q6_K)
#undef MQ_ID
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace mi355x
