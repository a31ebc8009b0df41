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
#include <type_traits>

#include "dispatch.h"
#include "qcommon.h"

namespace mi355x {

typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // SROA-friendly 16-B register

constexpr uint32_t RSRC_W3 = 0x00020000u;   // raw buffer, dword3 for gfx9-class descriptors
constexpr int MQ_BK = 64;                 // K per step = one 128-B LDS row of f16
constexpr int MQ_WIN = 4;                 // K-steps per offset MFMA of mmq_wave_kernel
constexpr float MQ_SUM_SCALE = 1.f / 16;  // activation run sums are stored x 1/16
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
// expert-sorted pair list, gathered from src1 column (slot % ne11, token).
// One single-wave workgroup per row (spread over every CU, no barrier): up to 4096 values are held in registers,
// so the row is read once (16 x 16-B loads in flight per lane), its |x|max reduced across the
// wave, and written as f16 with coalesced 8-B stores. Longer rows are re-read per 4096 chunk.
constexpr int CVT_T = 256;  // threads per token row (4 waves: 4x the loads in flight of one wave)
constexpr int CVT_R = 4;    // float4 per lane held across the reduction
// WAVE (mmq_wave_kernel's operand): values stored in order (0,2,1,3) within each 4 k, and each
// 16-k group's sum of the prescaled values, x 1/16, into xsum[row][window of 256 k][16] at the
// slot the kernel's correction fragment reads (see mmq_wave_kernel)
template <bool WAVE>
__global__ __launch_bounds__(CVT_T) void mmq_convert_x(const MmArgs a, _Float16 *x16, float *xinv, int Kpad,
                                                    const int *pos_pair, int n_rows, _Float16 *xsum) {
    const int tok = blockIdx.x, slice = blockIdx.y, lane = threadIdx.x & 63, tid = threadIdx.x;
    if (tok >= n_rows) return;
    const float *src;
    if (pos_pair) {
        const int pair = pos_pair[tok];
        const int slot = pair % a.n_used, t = pair / a.n_used;
        src = reinterpret_cast<const float *>(a.x + (int64_t)(slot % a.ne11_b) * a.nb11 + (int64_t)t * a.nb12);
    } else {
        const int i12 = slice % a.ne12, i13 = slice / a.ne12;
        src = reinterpret_cast<const float *>(a.x + (int64_t)i12 * a.nb12 + (int64_t)i13 * a.nb13 + (int64_t)tok * a.nb11);
    }
    // branch-free loads: a buffer resource over the row returns zeros past K (and takes any
    // 4-B alignment), so all CVT_R loads of a chunk are in flight together
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, (uint32_t)a.K * 4u, RSRC_W3);
    auto ld4f = [&](int k) -> float4 {
        return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, (uint32_t)k * 4u, 0, 0));
    };
    constexpr int CH = 4 * CVT_T * CVT_R;   // values per chunk
    const int t4 = tid * 4;
    float4 v[CVT_R];
    float amax = 0.f;
    for (int k0 = 0; k0 < a.K; k0 += CH) {
#pragma unroll
        for (int i = 0; i < CVT_R; ++i) v[i] = ld4f(k0 + 4 * CVT_T * i + t4);
#pragma unroll
        for (int i = 0; i < CVT_R; ++i)
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v[i].x), fabsf(v[i].y)), fmaxf(fabsf(v[i].z), fabsf(v[i].w))));
    }
    amax = fmaxf(amax, xchg<1>(amax));
    amax = fmaxf(amax, xchg<2>(amax));
    amax = fmaxf(amax, xchg<4>(amax));
    amax = fmaxf(amax, xchg<8>(amax));
    amax = fmaxf(amax, xchg<16>(amax));
    amax = fmaxf(amax, xchg<32>(amax));
    __shared__ float wmax[CVT_T / 64];
    if (lane == 0) wmax[tid >> 6] = amax;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < CVT_T / 64; ++w) amax = fmaxf(amax, wmax[w]);
    const int e = amax > 0.f ? (int)ceilf(log2f(amax)) - 14 : 0;
    const float sc = ldexpf(1.f, -e);
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const int64_t row_id = (int64_t)slice * (pos_pair ? n_rows : a.M) + tok;
    const int nrec = (Kpad + 511) / 512 * 2;   // mmq_wave_kernel's run-sum records
    _Float16 *dst = x16 + row_id * Kpad;
    for (int k0 = 0; k0 < Kpad; k0 += CH) {
        if (Kpad > CH) {   // the registers hold the last chunk only: re-read
#pragma unroll
            for (int i = 0; i < CVT_R; ++i) v[i] = ld4f(k0 + 4 * CVT_T * i + t4);
        }
#pragma unroll
        for (int i = 0; i < CVT_R; ++i) {
            const int k = k0 + 4 * CVT_T * i + t4;
            const float4 y = make_float4(v[i].x * sc, v[i].y * sc, v[i].z * sc, v[i].w * sc);
            if constexpr (WAVE) {
                const h4 hv = h4{(_Float16)y.x, (_Float16)y.z, (_Float16)y.y, (_Float16)y.w};
                // 32-k group = 8 consecutive lanes: sum of the values as stored (f16), kept as an
                // f16 hi + lo pair so the kernel's offset term uses the same activations exactly
                float gs = ((float)hv[0] + (float)hv[1]) + ((float)hv[2] + (float)hv[3]);
                gs += xchg<1>(gs);
                gs += xchg<2>(gs);
                gs += xchg<4>(gs);
                if (k < Kpad) {
                    *reinterpret_cast<h4 *>(dst + k) = hv;
                    if ((lane & 7) == 0) {
                        const int g = k >> 5, st = g >> 1;   // 32-run g = step st, half g & 1
                        const float sv = gs * MQ_SUM_SCALE;
                        const _Float16 hi = (_Float16)sv, lo = (_Float16)(sv - (float)hi);
                        _Float16 *o = xsum + row_id * nrec * 16 + ((st >> 3) * 2 + (st & 1)) * 16 + (g & 1) * 8 +
                                      ((st & 7) >> 1) * 2;
                        o[0] = hi;
                        o[1] = lo;
                    }
                }
            } else if (k < Kpad) {
                *reinterpret_cast<h4 *>(dst + k) = h4{(_Float16)y.x, (_Float16)y.y, (_Float16)y.z, (_Float16)y.w};
            }
        }
    }
    if constexpr (WAVE) {   // runs past Kpad (phantom steps of the last records): zero sums
        for (int g = Kpad / 32 + tid; g < nrec * 8; g += CVT_T) {
            const int st = g >> 1;
            _Float16 *o = xsum + row_id * nrec * 16 + ((st >> 3) * 2 + (st & 1)) * 16 + (g & 1) * 8 + ((st & 7) >> 1) * 2;
            o[0] = o[1] = (_Float16)0.f;
        }
    }
    if (tid == 0) xinv[row_id] = ldexpf(1.f, e);
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
// mmq_wave_kernel: weights decoded straight into MFMA fragments (no weight LDS traffic).
//
// Lane (fr = lane & 31, fh = lane >> 5) of wave w owns weight row wrow0 + 32w + fr and, in
// K-step s (64 weights), the contiguous 32-weight run k = 64s + 32fh .. +31: one Q4_0 / Q8_0
// block, one K-quant sub-block, two Q6_K scale groups. The MFMA k-slot (ks, fh, e) of a step
// carries run weight 8ks + pi(e), pi = (0,2,1,3) within each 4 (the order in which packed
// decodes produce pairs); mmq_convert_x stores the activations in the same order, and the
// fragment of slot (ks, fh) is LDS chunk 4fh + ks of the token row. Each wave owns distinct
// rows (4 waves x 32 = 128 rows per workgroup), so every weight is fetched and decoded once per
// token tile; only activations (BN tokens x 64 k, f16) go through LDS, by LDS-DMA into a 3-slot
// ring shared by the 4 waves.
//
// Decode in "code x scale - correction" form. Every type's weight is w = d * n - c with n a
// small unsigned code (nibble, 5/6-bit code, or int8 + 128), d the block scale and c the
// block's offset (8d, 128d, dmin*m, 32d*sc). The fragment holds d * n, made exactly by one
// v_pk_fma_f16 per pair: (1024 + n) * d - 1024 * d, where 1024 + n is the code dropped into an
// f16 mantissa (and_or / perm) and 1024 * d is exact. The offsets go into ONE extra MFMA per 4
// K-steps: per 16-weight group, B = -16 c (f16) and A = the group's activation sum / 16 (f16,
// mmq_convert_x), so sum_k w_k x_k = sum d n x - sum_g c_g S_g. (The reference folds its mins
// the same way, with q8_1 block sums: vec_dot_q4_K_q8_1 in src/ggml-cuda/vecdotq.cuh.)
//
// f16 range guard: a block whose d * 1024, d * n or 16 c could leave the f16 range sets a flag;
// a wave with any flagged lane recomputes its tile in fp32 on the VALU (slow, exact; real
// quantized weights are many orders of magnitude inside the range) before the epilogue.
// ------------------------------------------------------------------------------------------

// f32 Q4_K/Q5_K sub-block scale and min (get_scale_min_k4, src/ggml-quants.c:703-710)
__device__ __forceinline__ void k4_sub_scale_f(const u32x4 &hd, int j, float &d1, float &m1) {
    const uint32_t S[3] = {hd[1], hd[2], hd[3]};
    uint32_t sc0, sc1, m0, m1v;
    k4_scale_min_pair(S, j >> 1, sc0, sc1, m0, m1v);
    const bool hi = j & 1;
    d1 = h2f((uint16_t)hd[0]) * (float)(hi ? sc1 : sc0);
    m1 = h2f((uint16_t)(hd[0] >> 16)) * (float)(hi ? m1v : m0);
}
__device__ __forceinline__ uint32_t byte_of(const u32x4 &lo, const u32x4 &hi, int e) {   // byte e of 32
    const u32x4 &q = e < 16 ? lo : hi;
    return (q[(e & 15) >> 2] >> (8 * (e & 3))) & 0xFFu;
}
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t m, uint32_t o) { return (a & m) | o; }
// Decode constants held in registers: gfx950 VOP3 takes no literals, so with literal operands
// (a & m) | o splits into v_and + v_or; from an SGPR mask and a VGPR base it is one v_and_or_b32.
struct DecK {
    uint32_t m4, m1, m3;   // 0x000F000F, 0x00100010, 0x00300030 (SGPRs)
    uint32_t f1024;        // 0x64006400: f16 pair (1024, 1024) (VGPR)
    __device__ __forceinline__ static DecK make() {
        DecK k{0x000F000Fu, 0x00100010u, 0x00300030u, 0x64006400u};
        asm volatile("" : "+s"(k.m4), "+s"(k.m1), "+s"(k.m3), "+v"(k.f1024));
        return k;
    }
};
// 4 nibbles (bits sh..sh+3 of each byte of v) -> f16 pairs (1024 + n): (byte0, byte2), (byte1, byte3)
__device__ __forceinline__ void nib_pairs(uint32_t v, int sh, uint32_t &p02, uint32_t &p13, const DecK &K) {
    const uint32_t t = v >> sh;
    p02 = and_or(t, K.m4, K.f1024);
    p13 = and_or(t >> 8, K.m4, K.f1024);
}
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
// running max of the |scale| bit patterns (f16 pairs): v_pk_max_u16
__device__ __forceinline__ void track_scale(uint32_t &mx, uint32_t bits) {
    mx = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, mx),
                                                                __builtin_bit_cast(u16x2, bits & 0x7FFF7FFFu)));
}
// f16 pair math: (1024 + n) * d - 1024 * d = n * d, one rounding
struct Scale2 {
    h2v mul, add;
    __device__ __forceinline__ void set(float d) {
        mul = splat_h2(d);
        add = splat_h2(-1024.f * d);
    }
    __device__ __forceinline__ uint32_t operator()(uint32_t p) const {
        return as_u(__builtin_elementwise_fma(as_h2(p), mul, add));
    }
};
// f16 range: the decode needs 1024 * scale, (q + 128) * d, 16 * offset and the Q6_K products
// inside f16. All hold while every raw block scale (d, dmin) is below 1 in magnitude (the
// sub-block factors are <= 63, codes <= 255); prep() tracks the largest raw scale bit pattern and
// the kernel takes its fp32 path for a wave whose rows hold one >= 1.0 (0x3C00).
constexpr uint32_t F16_ONE = 0x3C00u;

template <int T> struct Deq32;

// Each type: at(row, kr) fixes the run's addresses; part(r, p) issues vector-memory load p of
// NLOADS (the phase spreads them between MFMAs); prep(bad, c) derives the scale once the loads
// landed, returns the run's two group offsets as an f16 pair (-16 c per group) and flags range
// trouble; frag(ks) decodes run weights 8ks..8ks+7 (order pi) as d * n; w32(e) is the exact
// fp32 weight e for the guard's slow path.
// Blocks of 18 / 34 bytes start 2-byte aligned. Their bytes are fetched as dword-aligned windows
// (multi-dword buffer loads at 2-byte offsets fetch slowly and were seen to break the in-order
// retirement that counted vmcnt waits rely on) and realigned by a 64-bit funnel shift.
__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t bits) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> bits);
}
__device__ __forceinline__ uint32_t bl32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
// LDS reads of staged weight rows (mmq_wl_kernel): 16-B aligned, or dword aligned
__device__ __forceinline__ u32x4 lds16(const uint8_t *p) { return *reinterpret_cast<const u32x4 *>(p); }
__device__ __forceinline__ uint32_t lds1(const uint8_t *p) { return *reinterpret_cast<const uint32_t *>(p); }
__device__ __forceinline__ u32x4 lds4u(const uint8_t *p) { return u32x4{lds1(p), lds1(p + 4), lds1(p + 8), lds1(p + 12)}; }

template <> struct Deq32<T_Q4_0> {   // block: d (f16), 16 B of nibbles (w[i] low, w[i+16] high)
    static constexpr int NLOADS = 2;
    uint32_t b;       // dword-aligned window start; the block starts at b + 2 * odd
    uint32_t odd;     // block start is 2 mod 4
    u32x4 w0;
    uint32_t w4;
    Scale2 s;
    __device__ __forceinline__ void at(uint32_t row, int kr) {
        const uint32_t o = row + (uint32_t)(kr >> 5) * 18;
        b = o & ~3u;
        odd = (o >> 1) & 1;
    }
    __device__ __forceinline__ void part(__amdgpu_buffer_rsrc_t r, int p) {
        if (p == 0) w0 = bl128(r, b);
        else w4 = bl32(r, b + 16);
    }
    static constexpr int SB = 144;   // bytes of 8 blocks (256 k) of one row, staged per row in LDS
    __device__ __forceinline__ void lds(const uint8_t *rp, int kr) {   // rp: the row's 16-B aligned segment
        const uint32_t o = (uint32_t)((kr >> 5) & 7) * 18;
        b = o & ~3u;
        odd = (o >> 1) & 1;
        w0 = lds4u(rp + b);
        w4 = lds1(rp + b + 16);
    }
    __device__ __forceinline__ uint32_t d16() const { return (w0[0] >> (16 * odd)) & 0xFFFFu; }
    // dword i of the 16 nibble bytes: window bytes 2 + 2 odd + 4i ..
    __device__ __forceinline__ uint32_t qw(int i) const { return funnel(w0[i], i + 1 < 4 ? w0[i + 1] : w4, 16 + 16 * odd); }
    __device__ __forceinline__ uint32_t prep(uint32_t &bad) {
        const float df = h2f((uint16_t)d16());
        track_scale(bad, d16());
        s.set(df);
        return as_u(splat_h2(-16.f * 8.f * df));
    }
    __device__ __forceinline__ u32x4 frag(int ks, const DecK &K) const {
        const int sh = (ks >> 1) * 4, i = (ks & 1) * 2;
        uint32_t a0, a1, b0, b1;
        nib_pairs(qw(i), sh, a0, a1, K);
        nib_pairs(qw(i + 1), sh, b0, b1, K);
        return u32x4{s(a0), s(a1), s(b0), s(b1)};
    }
    __device__ __forceinline__ float w32(int e) const {
        const uint32_t v = (qw((e & 15) >> 2) >> (8 * (e & 3))) & 0xFFu;
        return (float)((int)((v >> (4 * (e >> 4))) & 15) - 8) * h2f((uint16_t)d16());
    }
};

template <> struct Deq32<T_Q8_0> {   // block: d (f16), 32 int8
    static constexpr int NLOADS = 3;
    uint32_t b, odd;
    u32x4 w0, w4;
    uint32_t w8;
    Scale2 s;
    __device__ __forceinline__ void at(uint32_t row, int kr) {
        const uint32_t o = row + (uint32_t)(kr >> 5) * 34;
        b = o & ~3u;
        odd = (o >> 1) & 1;
    }
    __device__ __forceinline__ void part(__amdgpu_buffer_rsrc_t r, int p) {
        if (p == 0) w0 = bl128(r, b);
        else if (p == 1) w4 = bl128(r, b + 16);
        else w8 = bl32(r, b + 32);
    }
    static constexpr int SB = 272;
    __device__ __forceinline__ void lds(const uint8_t *rp, int kr) {
        const uint32_t o = (uint32_t)((kr >> 5) & 7) * 34;
        b = o & ~3u;
        odd = (o >> 1) & 1;
        w0 = lds4u(rp + b);
        w4 = lds4u(rp + b + 16);
        w8 = lds1(rp + b + 32);
    }
    __device__ __forceinline__ uint32_t win(int i) const { return i < 4 ? w0[i] : i < 8 ? w4[i - 4] : w8; }
    __device__ __forceinline__ uint32_t d16() const { return (w0[0] >> (16 * odd)) & 0xFFFFu; }
    // dword i of the 32 quant bytes: window bytes 2 + 2 odd + 4i ..
    __device__ __forceinline__ uint32_t qw(int i) const { return funnel(win(i), win(i + 1), 16 + 16 * odd); }
    __device__ __forceinline__ uint32_t prep(uint32_t &bad) {
        const float df = h2f((uint16_t)d16());
        track_scale(bad, d16());
        s.set(df);
        return as_u(splat_h2(-16.f * 128.f * df));
    }
    __device__ __forceinline__ u32x4 frag(int ks, const DecK &K) const {
        const uint32_t u0 = qw(2 * ks) ^ 0x80808080u, u1 = qw(2 * ks + 1) ^ 0x80808080u;   // q + 128
        return u32x4{s(__builtin_amdgcn_perm(0x64646464u, u0, 0x04020400u)),
                     s(__builtin_amdgcn_perm(0x64646464u, u0, 0x04030401u)),
                     s(__builtin_amdgcn_perm(0x64646464u, u1, 0x04020400u)),
                     s(__builtin_amdgcn_perm(0x64646464u, u1, 0x04030401u))};
    }
    __device__ __forceinline__ float w32(int e) const {
        return (float)(int8_t)((qw(e >> 2) >> (8 * (e & 3))) & 0xFFu) * h2f((uint16_t)d16());
    }
};

template <> struct Deq32<T_Q4_K> {   // super-block 144 B: d, dmin, 12 B scales, 128 B nibbles
    static constexpr int NLOADS = 3;
    uint32_t b;
    int j;   // sub-block: bytes 32 (j >> 1) .. +31 of the nibbles, nibble j & 1
    u32x4 hd, q0, q1;
    Scale2 s;
    __device__ __forceinline__ void at(uint32_t row, int kr) {
        b = row + (uint32_t)(kr >> 8) * 144;
        j = (kr & 255) >> 5;
    }
    __device__ __forceinline__ void part(__amdgpu_buffer_rsrc_t r, int p) {
        if (p == 0) hd = bl128(r, b);
        else if (p == 1) q0 = bl128(r, b + 16 + 32 * (j >> 1));
        else q1 = bl128(r, b + 32 + 32 * (j >> 1));
    }
    static constexpr int SB = 144;
    __device__ __forceinline__ void lds(const uint8_t *rp, int kr) {
        j = (kr & 255) >> 5;
        hd = lds16(rp);
        q0 = lds16(rp + 16 + 32 * (j >> 1));
        q1 = lds16(rp + 32 + 32 * (j >> 1));
    }
    __device__ __forceinline__ uint32_t prep(uint32_t &bad) {
        float d1, m1;
        k4_sub_scale_f(hd, j, d1, m1);
        const h2v dq = splat_h2(d1);   // the scale is an f16 product, as the reference rounds it
        const float dr = (float)dq[0];
        track_scale(bad, hd[0]);
        s.set(dr);
        return as_u(splat_h2(-16.f * m1));
    }
    __device__ __forceinline__ u32x4 frag(int ks, const DecK &K) const {
        const u32x4 &q = ks < 2 ? q0 : q1;
        const int i = (ks & 1) * 2, sh = (j & 1) * 4;
        uint32_t a0, a1, b0, b1;
        nib_pairs(q[i], sh, a0, a1, K);
        nib_pairs(q[i + 1], sh, b0, b1, K);
        return u32x4{s(a0), s(a1), s(b0), s(b1)};
    }
    __device__ __forceinline__ float w32(int e) const {
        float d1, m1;
        k4_sub_scale_f(hd, j, d1, m1);
        return (float)((byte_of(q0, q1, e) >> (4 * (j & 1))) & 15) * d1 - m1;
    }
};

template <> struct Deq32<T_Q5_K> {   // super-block 176 B: d, dmin, 12 B scales, 32 B high bits, 128 B nibbles
    static constexpr int NLOADS = 5;
    uint32_t b;
    int j;
    u32x4 hd, h0, h1, q0, q1;
    Scale2 s;
    __device__ __forceinline__ void at(uint32_t row, int kr) {
        b = row + (uint32_t)(kr >> 8) * 176;
        j = (kr & 255) >> 5;
    }
    __device__ __forceinline__ void part(__amdgpu_buffer_rsrc_t r, int p) {
        if (p == 0) hd = bl128(r, b);
        else if (p == 1) q0 = bl128(r, b + 48 + 32 * (j >> 1));
        else if (p == 2) q1 = bl128(r, b + 64 + 32 * (j >> 1));
        else if (p == 3) h0 = bl128(r, b + 16);
        else h1 = bl128(r, b + 32);
    }
    static constexpr int SB = 176;
    __device__ __forceinline__ void lds(const uint8_t *rp, int kr) {
        j = (kr & 255) >> 5;
        hd = lds16(rp);
        h0 = lds16(rp + 16);
        h1 = lds16(rp + 32);
        q0 = lds16(rp + 48 + 32 * (j >> 1));
        q1 = lds16(rp + 64 + 32 * (j >> 1));
    }
    __device__ __forceinline__ uint32_t prep(uint32_t &bad) {
        float d1, m1;
        k4_sub_scale_f(hd, j, d1, m1);
        const h2v dq = splat_h2(d1);
        const float dr = (float)dq[0];
        track_scale(bad, hd[0]);
        s.set(dr);
        return as_u(splat_h2(-16.f * m1));
    }
    __device__ __forceinline__ u32x4 frag(int ks, const DecK &K) const {
        const u32x4 &q = ks < 2 ? q0 : q1;
        const u32x4 &h = ks < 2 ? h0 : h1;
        const int i = (ks & 1) * 2, sh = (j & 1) * 4;
        u32x4 o;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            uint32_t p02, p13;
            nib_pairs(q[i + t], sh, p02, p13, K);
            const uint32_t u = __builtin_amdgcn_alignbit(h[i + t], h[i + t], (j - 4) & 31);   // bit j -> bit 4
            o[2 * t] = s(and_or(u, K.m1, p02));
            o[2 * t + 1] = s(and_or(u >> 8, K.m1, p13));
        }
        return o;
    }
    __device__ __forceinline__ float w32(int e) const {
        float d1, m1;
        k4_sub_scale_f(hd, j, d1, m1);
        const uint32_t c = ((byte_of(q0, q1, e) >> (4 * (j & 1))) & 15) | (((byte_of(h0, h1, e) >> j) & 1) << 4);
        return (float)c * d1 - m1;
    }
};

template <> struct Deq32<T_Q6_K> {   // super-block 210 B: ql 128, qh 64, int8 scales 16, d
    // 210-B super-blocks start 2-byte aligned: the two 32-byte runs (low nibbles, high bits) are
    // fetched as dword-aligned 36-byte windows, the scale pair and d as 16-bit loads
    static constexpr int NLOADS = 8;
    uint32_t b, odd;
    int hh, k;   // 128-half, and quarter of it: nibble (k >> 1), high-bit pair 2k
    u32x4 l0, l4, h0, h4;
    uint32_t l8, h8, sc, d;
    __device__ __forceinline__ void at(uint32_t row, int kr) {
        const uint32_t o = row + (uint32_t)(kr >> 8) * 210;
        b = o & ~3u;
        odd = (o >> 1) & 1;
        hh = (kr & 255) >> 7;
        k = (kr & 127) >> 5;
    }
    __device__ __forceinline__ void part(__amdgpu_buffer_rsrc_t r, int p) {
        const uint32_t lb = b + 64 * hh + 32 * (k & 1), hb = b + 128 + 32 * hh;
        if (p == 0) d = bl16(r, b + 2 * odd + 208);
        else if (p == 1) sc = bl16(r, b + 2 * odd + 192 + 8 * hh + 2 * k);
        else if (p == 2) l0 = bl128(r, lb);
        else if (p == 3) l4 = bl128(r, lb + 16);
        else if (p == 4) l8 = bl32(r, lb + 32);
        else if (p == 5) h0 = bl128(r, hb);
        else if (p == 6) h4 = bl128(r, hb + 16);
        else h8 = bl32(r, hb + 32);
    }
    __device__ __forceinline__ static uint32_t pick(const u32x4 &w0, const u32x4 &w4, uint32_t w8, int i) {
        return i < 4 ? w0[i] : i < 8 ? w4[i - 4] : w8;
    }
    __device__ __forceinline__ uint32_t lw(int i) const { return funnel(pick(l0, l4, l8, i), pick(l0, l4, l8, i + 1), 16 * odd); }
    __device__ __forceinline__ uint32_t hw(int i) const { return funnel(pick(h0, h4, h8, i), pick(h0, h4, h8, i + 1), 16 * odd); }
    __device__ __forceinline__ float dsc(int half) const {
        return (float)(_Float16)(h2f((uint16_t)d) * (float)(int8_t)(sc >> (8 * half)));   // f16 product
    }
    // Q6_K keeps the exact affine form (code - 32) * scale per pair, (1024 + c) - 1056 being
    // exact in f16: its two scale groups per run would need two offset slots per step
    h2v ds0, ds1;
    __device__ __forceinline__ uint32_t prep(uint32_t &bad) {
        const float a0 = dsc(0), a1 = dsc(1);
        track_scale(bad, d);
        ds0 = splat_h2(a0);
        ds1 = splat_h2(a1);
        return 0u;
    }
    __device__ __forceinline__ u32x4 frag(int ks, const DecK &K) const {
        const h2v ds = ks < 2 ? ds0 : ds1;
        const h2v bias = splat_h2(1056.f);
        auto s = [&](uint32_t p) { return as_u((as_h2(p) - bias) * ds); };
        const int sh = (k >> 1) * 4;
        u32x4 o;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            uint32_t p02, p13;
            nib_pairs(lw(2 * ks + t), sh, p02, p13, K);
            const uint32_t hv = hw(2 * ks + t);
            const uint32_t u = __builtin_amdgcn_alignbit(hv, hv, (2 * k - 4) & 31);   // bits 2k,2k+1 -> 4,5
            o[2 * t] = s(and_or(u, K.m3, p02));
            o[2 * t + 1] = s(and_or(u >> 8, K.m3, p13));
        }
        return o;
    }
    __device__ __forceinline__ float w32(int e) const {
        const uint32_t lb = (lw(e >> 2) >> (8 * (e & 3))) & 0xFFu, hb = (hw(e >> 2) >> (8 * (e & 3))) & 0xFFu;
        const uint32_t c = ((lb >> ((k >> 1) * 4)) & 15) | (((hb >> (2 * k)) & 3) << 4);
        return (float)((int)c - 32) * (h2f((uint16_t)d) * (float)(int8_t)(sc >> (8 * (e >> 4))));
    }
};

// The workgroup is 8 waves in two K-groups: waves 4g .. 4g+3 own the same 128 rows x BN tokens
// and take the even (g = 0) or odd (g = 1) K-steps, each group with its own activation ring.
// Two waves per SIMD then interleave: one wave's decode VALU and loads issue while its partner's
// MFMAs run. The groups' accumulators are summed through LDS at the end.
// Activation run sums (for the offset MFMA) are laid out per group and per 4 of the group's
// steps: record (step / 8) * 2 + (step & 1) of 16 f16, slot fh * 8 + 2 * ((step % 8) / 2) + hi/lo.
// Split-K (few tokens, so few token tiles): blockIdx.z = slice * n_split + split; split s runs
// phases [s * split_np, (s + 1) * split_np) and, with n_split > 1, writes its scaled partial tile
// to part[split][slice][token][row] for mmq_split_reduce.
template <int T, int TN, bool IDS, bool STAMP = false>
__global__ __launch_bounds__(512) void mmq_wave_kernel(const MmArgs a, const _Float16 *__restrict__ x16,
                                                       const _Float16 *__restrict__ xsum, const float *__restrict__ xinv,
                                                       int Kpad, uint32_t w_extent, const MoeMap moe, int n_split,
                                                       int split_np, float *__restrict__ part) {
    constexpr int BN = 32 * TN;                 // tokens per workgroup
    constexpr int XB = BN * 128;                // bytes of one activation slot (BK = 64 f16)
    constexpr int V = TN;                       // 1-KiB activation pieces per wave per step
    constexpr int NLW = Deq32<T>::NLOADS;
    constexpr int VM_PHASE = NLW + V;           // vector-memory ops of a plain phase
    static_assert(VM_PHASE + TN < 64, "vmcnt range");
    static_assert(6 * XB >= 128 * BN * 4, "accumulator exchange fits the rings");
    __shared__ __align__(16) uint8_t lds[6 * XB];   // [group][3 slots][XB]
    __shared__ uint32_t g1_bad[4];

    const int slice = blockIdx.z / n_split, split = blockIdx.z % n_split;
    const int i12 = slice % a.ne12, i13 = slice / a.ne12;
    const uint8_t *wmat;
    const _Float16 *xs, *ss;
    uint8_t *dmat;
    int tok0, tok_end;
    const int nrec = (Kpad + 511) / 512 * 2;    // run-sum records per token row (Kpad % 128 == 0)
    if constexpr (IDS) {   // token tile -> expert (see mmq_kernel)
        const int tile = blockIdx.y;
        if (tile >= moe.tile_off[moe.n_expert]) return;
        int lo = 0, hi = moe.n_expert - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (moe.tile_off[mid] <= tile) lo = mid; else hi = mid - 1;
        }
        wmat = a.w + (int64_t)lo * a.nb02;
        xs = x16;
        ss = xsum;
        dmat = a.dst;
        tok0 = moe.offsets[lo] + (tile - moe.tile_off[lo]) * BN;
        tok_end = moe.offsets[lo + 1];
    } else {
        wmat = a.w + (int64_t)(i12 / a.r2) * a.nb02 + (int64_t)(i13 / a.r3) * a.nb03;
        xs = x16 + (int64_t)slice * a.M * Kpad;
        ss = xsum + (int64_t)slice * a.M * nrec * 16;
        dmat = a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3;
        tok0 = blockIdx.y * BN;
        tok_end = a.M;
    }
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void *)wmat, 0, w_extent, RSRC_W3);
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc((void *)xs, 0, (uint32_t)tok_end * (uint32_t)Kpad * 2u, RSRC_W3);
    const __amdgpu_buffer_rsrc_t sr =
        __builtin_amdgcn_make_buffer_rsrc((void *)ss, 0, (uint32_t)tok_end * (uint32_t)nrec * 32u, RSRC_W3);

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int grp = wave >> 2, wq = wave & 3;
    const int fr = lane & 31, fh = lane >> 5;
    const int row = blockIdx.x * 128 + 32 * wq + fr;
    const uint32_t wrow = (uint32_t)row * (uint32_t)a.nb01;   // rows >= N read as zeros
    const int p0 = split * split_np;                             // first phase of this split
    const int np = min(split_np, Kpad / (2 * MQ_BK) - p0);       // phases (steps per group)
    uint8_t *const xslot = lds + grp * 3 * XB;
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

    uint32_t x_off[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int r = 8 * (wq + 4 * v) + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        x_off[v] = ((uint32_t)(tok0 + r) * (uint32_t)Kpad + (uint32_t)c * 8u) * 2u;
    }
    auto step_of = [&](int p) { return 2 * (p0 + p) + grp; };
    // a K tail (32-block types, K % 128 != 0) re-reads the row's last block: its codes meet zero
    // activations and zero run sums, so it adds exactly 0
    auto at_w = [&](Deq32<T> &w, int p) { w.at(wrow, min(step_of(p) * MQ_BK + 32 * fh, a.K - 32)); };
    auto load_w = [&](Deq32<T> &w, int p) {
        at_w(w, p);
#pragma unroll
        for (int q = 0; q < NLW; ++q) w.part(wr, q);
    };
    auto dma_piece = [&](int p, int slot, int v) {
        dma16(xr, xslot + slot * XB + (wq + 4 * v) * 1024, x_off[v] + (uint32_t)step_of(p) * MQ_BK * 2u);
    };
    // run-sum fragment of this group's window w (phases 4w .. 4w+3) for token tile j
    u32x4 sfrag[TN];
    auto load_sums = [&](int w) {   // w counts this split's windows (p0 is a multiple of MQ_WIN)
        const uint32_t rec = (uint32_t)(2 * (w + p0 / MQ_WIN) + grp);
#pragma unroll
        for (int j = 0; j < TN; ++j)
            sfrag[j] = bl128(sr, ((uint32_t)(tok0 + 32 * j + fr) * (uint32_t)nrec + rec) * 32u + 16u * fh);
    };

    float16v acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    auto compute = [&](const u32x4 (&f)[4], int xsl) {
        const uint8_t *X = xslot + xsl * XB;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            half8 ax[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) ax[j] = *reinterpret_cast<const half8 *>(X + swz(32 * j + fr, 4 * fh + ks));
            const half8 bw = __builtin_bit_cast(half8, f[ks]);
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax[j], bw, acc[j], 0, 0, 0);
        }
    };
    u32x4 cw = {0u, 0u, 0u, 0u};   // -16 c of the current window: dword = phase slot
    auto correct = [&]() {
#pragma unroll
        for (int j = 0; j < TN; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, sfrag[j]), __builtin_bit_cast(half8, cw),
                                                            acc[j], 0, 0, 0);
        cw = u32x4{0u, 0u, 0u, 0u};
    };
    auto barrier = [&]() {   // compiler fences on both sides: no LDS access or DMA crosses it
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };

    uint32_t bad = 0;   // largest raw block-scale bit pattern seen (f16 pair)
    const DecK DK = DecK::make();
    Deq32<T> ra, rb;
    u32x4 F[4], G[4];
    load_sums(0);
    load_w(ra, 0);
#pragma unroll
    for (int v = 0; v < V; ++v) dma_piece(0, 0, v);
    load_w(rb, min(1, np - 1));
#pragma unroll
    for (int v = 0; v < V; ++v) dma_piece(min(1, np - 1), 1, v);
    cw[0] = ra.prep(bad);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) F[ks] = ra.frag(ks, DK);
    wait_vmcnt<VM_PHASE>();   // phase 0's activations landed (this wave's pieces)
    barrier();

    // phase p (SP = slot of phase p+1 in its window): loads of phase p+2 out, decode of phase
    // p+1 (raw registers loaded one phase ago) beside the MFMAs of phase p, then the activations
    // of phase p+1 retire and one barrier. Laid out in NMF chunks fenced by sched_barrier: chunk
    // i = MFMA i, its share of the vector-memory instructions and of the decode; all activation
    // fragments of the step are read from LDS first. When phase p+1 completes a window (SP == 3)
    // the offset MFMA follows and the next window's sums load.
    constexpr int NMF = 4 * TN;
    auto phase = [&](auto SPc, Deq32<T> &rdec, Deq32<T> &rload, const u32x4 (&fcur)[4], u32x4 (&fnext)[4], int p,
                     int xs0) {
        constexpr int SP = decltype(SPc)::value;
        const int xs1 = xs0 == 2 ? 0 : xs0 + 1, xs2 = xs1 == 2 ? 0 : xs1 + 1;
        const int pl = min(p + 2, np - 1);
        stamp(3);
        const uint8_t *X = xslot + xs0 * XB;
        half8 ax[4][TN];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
            for (int j = 0; j < TN; ++j) ax[ks][j] = *reinterpret_cast<const half8 *>(X + swz(32 * j + fr, 4 * fh + ks));
        at_w(rload, pl);
        stamp(0);
#pragma unroll
        for (int i = 0; i < NMF; ++i) {
            const int ks = i / TN, j = i % TN;
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax[ks][j], __builtin_bit_cast(half8, fcur[ks]), acc[j], 0, 0, 0);
#pragma unroll
            for (int l = i * VM_PHASE / NMF; l < (i + 1) * VM_PHASE / NMF; ++l) {
                if (l < NLW) rload.part(wr, l);
                else dma_piece(pl, xs2, l - NLW);
            }
            constexpr int PER = NMF / 4;   // MFMAs per decoded fragment
            if (i % PER == PER - 1) {
                if (i == PER - 1) cw[SP] = rdec.prep(bad);
                fnext[i / PER] = rdec.frag(i / PER, DK);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (SP == MQ_WIN - 1) {
            correct();
            load_sums((p + 2) / MQ_WIN);   // phase p+2 opens the next window
        }
        stamp(1);
        // retire the activations of phase p+1, issued last in the previous phase: younger are
        // this phase's loads, plus the window sums issued after them in a closing phase
        wait_vmcnt<VM_PHASE + (SP == MQ_WIN - 1 || SP == 0 ? TN : 0)>();
        stamp(2);
        barrier();
        return xs1;
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I0 = std::integral_constant<int, 0>;
    int p = 0, xsl = 0;
    for (; p + MQ_WIN <= np - 1; p += MQ_WIN) {   // phases p .. p+3 decode phases p+1 .. p+4
        xsl = phase(I1{}, rb, ra, F, G, p, xsl);
        xsl = phase(I2{}, ra, rb, G, F, p + 1, xsl);
        xsl = phase(I3{}, rb, ra, F, G, p + 2, xsl);
        xsl = phase(I0{}, ra, rb, G, F, p + 3, xsl);
    }
    const int rem = np - 1 - p;   // 0..3 phases left; the last step is in F or G
    if (rem >= 1) xsl = phase(I1{}, rb, ra, F, G, p, xsl);
    if (rem >= 2) xsl = phase(I2{}, ra, rb, G, F, p + 1, xsl);
    if (rem >= 3) xsl = phase(I3{}, rb, ra, F, G, p + 2, xsl);
    if (rem & 1) compute(G, xsl);
    else compute(F, xsl);
    if (rem != 3) correct();   // the last window is partial (rem == 3: it closed in its phase)
    wait_vmcnt<0>();   // no LDS-DMA may still be landing when the rings are reused below
    stamp(3);
    if constexpr (STAMP) {
        if (lane == 0 && a.stamps) {
            const int g = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
            unsigned long long *o = a.stamps + ((size_t)g * 8 + wave) * 8;
            o[0] = st_start;
            for (int i = 0; i < 5; ++i) o[1 + i] = st_seg[i];
            o[6] = st_t;
            o[7] = np;
        }
    }

    // sum the groups: group 1 parks its accumulators (and range flag) in the rings, group 0 adds
    const bool bad_here = (bad & 0xFFFFu) >= F16_ONE || (bad >> 16) >= F16_ONE;
    float4 *park = reinterpret_cast<float4 *>(lds) + (size_t)(wq * 64 + lane) * 4 * TN;
    barrier();   // every wave is done reading the rings
    if (grp == 1) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                park[4 * j + q] = make_float4(acc[j][4 * q], acc[j][4 * q + 1], acc[j][4 * q + 2], acc[j][4 * q + 3]);
        const bool b1 = __builtin_amdgcn_ballot_w64(bad_here) != 0;
        if (lane == 0) g1_bad[wq] = b1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();
    if (grp == 1) return;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 o = park[4 * j + q];
            acc[j][4 * q] += o.x;
            acc[j][4 * q + 1] += o.y;
            acc[j][4 * q + 2] += o.z;
            acc[j][4 * q + 3] += o.w;
        }

    // token of accumulator element (j, r) of this lane
    auto tok_of = [&](int j, int r) { return tok0 + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * fh; };
    if ((__builtin_amdgcn_ballot_w64(bad_here) != 0) || g1_bad[wq]) {
        // a block scale >= 1.0 in this wave's rows: recompute the tile in fp32 (exact; far outside
        // what quantized weights hold). Activations are read back in their stored order pi.
        for (int j = 0; j < TN; ++j)
            for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
        for (int kr = p0 * 2 * MQ_BK; kr < min(a.K, (p0 + np) * 2 * MQ_BK); kr += 32) {   // this split's K
            Deq32<T> w;
            w.at(wrow, kr);
            for (int q = 0; q < NLW; ++q) w.part(wr, q);
            for (int e = 0; e < 32; ++e) {
                const float wf = w.w32(e);
                const int ke = kr + (e & ~3) + ((e & 3) == 1 ? 2 : (e & 3) == 2 ? 1 : (e & 3));
                for (int j = 0; j < TN; ++j)
                    for (int r = 0; r < 16; ++r) {
                        const int t = min(tok_of(j, r), tok_end - 1);
                        acc[j][r] += wf * (float)xs[(int64_t)t * Kpad + ke];
                    }
            }
        }
    }

    const float *xinv_s = IDS ? xinv : xinv + (int64_t)slice * a.M;
    float inv[TN][16];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) inv[j][r] = xinv_s[min(tok_of(j, r), tok_end - 1)];
    if (row < a.N) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int tok = tok_of(j, r);
                if (tok < tok_end) {
                    uint8_t *drow;
                    if constexpr (IDS) {
                        const int pair = moe.pos_pair[tok];
                        drow = dmat + (int64_t)(pair % moe.n_used) * a.nb1 + (int64_t)(pair / moe.n_used) * a.nb2;
                    } else if (n_split > 1) {
                        drow = reinterpret_cast<uint8_t *>(part + (((int64_t)split * gridDim.z / n_split + slice) * a.M + tok) * a.N);
                    } else {
                        drow = dmat + (int64_t)tok * a.nb1;
                    }
                    reinterpret_cast<float *>(drow)[row] = acc[j][r] * inv[j][r];
                }
            }
    }
}

// ------------------------------------------------------------------------------------------
// mmq_wl_kernel: mmq_wave_kernel with the weights staged through LDS. The register-decode
// kernel's per-lane row loads touch 32 rows (32 cache lines) per wave instruction and keep the
// texture unit busy (§4.2 of DESIGN.md). Here all 8 waves copy each 256-k super-block of the
// workgroup's 128 rows into an LDS ring with 16-B LDS-DMA pieces that walk the rows in order
// (a piece covers ~7 consecutive row segments), and each lane then reads its own run from LDS.
// Needs every row's 256-k segment 16-B aligned: Q4_0 / Q8_0 / Q4_K / Q5_K with K % 256 == 0.
//   ring: 3 slots of 128 rows x SB bytes; super-block b is consumed by phases 2b, 2b+1 (both
//   K-groups), its pieces are issued in phases 2b-4 and 2b-3 (half each) and retire with the
//   activations of phase 2b-2, one barrier before the first decode reads them.
// ------------------------------------------------------------------------------------------
template <int T, int TN, bool STAMP = false>
__global__ __launch_bounds__(512) void mmq_wl_kernel(const MmArgs a, const _Float16 *__restrict__ x16,
                                                     const _Float16 *__restrict__ xsum, const float *__restrict__ xinv,
                                                     int Kpad, uint32_t w_extent, int n_split, int split_np,
                                                     float *__restrict__ part) {
    constexpr int BN = 32 * TN, XB = BN * 128, V = TN;
    constexpr int SB = Deq32<T>::SB;            // bytes of one row's 256-k segment
    constexpr int WSLOT = 128 * SB;             // one ring slot
    constexpr int NPIECE = WSLOT / 1024;        // 1-KiB pieces per slot
    static_assert(WSLOT % 1024 == 0 && SB % 16 == 0, "slot made of whole pieces");
    constexpr int TMAX = (NPIECE + 7) / 8;      // pieces of the busiest wave per slot
    constexpr int TMIN = NPIECE / 8;            // pieces of the least busy wave per slot
    constexpr int WMAX0 = (TMAX + 1) / 2, WMAX1 = TMAX / 2;   // per half (even / odd phase)
    constexpr int WLOW0 = (TMIN + 1) / 2, WLOW1 = TMIN / 2;
    static_assert(WMAX0 + V + 2 * TN < 64, "vmcnt range");
    __shared__ __align__(16) uint8_t lds[6 * XB + 3 * WSLOT];   // [group][3][XB] | [3][WSLOT]
    __shared__ uint32_t g1_bad[4];

    const int slice = blockIdx.z / n_split, split = blockIdx.z % n_split;
    const int i12 = slice % a.ne12, i13 = slice / a.ne12;
    const int nrec = (Kpad + 511) / 512 * 2;
    const uint8_t *wmat = a.w + (int64_t)(i12 / a.r2) * a.nb02 + (int64_t)(i13 / a.r3) * a.nb03;
    const _Float16 *xs = x16 + (int64_t)slice * a.M * Kpad;
    const _Float16 *ss = xsum + (int64_t)slice * a.M * nrec * 16;
    uint8_t *dmat = a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3;
    const int tok0 = blockIdx.y * BN, tok_end = a.M;
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void *)wmat, 0, w_extent, RSRC_W3);
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc((void *)xs, 0, (uint32_t)tok_end * (uint32_t)Kpad * 2u, RSRC_W3);
    const __amdgpu_buffer_rsrc_t sr =
        __builtin_amdgcn_make_buffer_rsrc((void *)ss, 0, (uint32_t)tok_end * (uint32_t)nrec * 32u, RSRC_W3);

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int grp = wave >> 2, wq = wave & 3;
    const int fr = lane & 31, fh = lane >> 5;
    const int row0 = blockIdx.x * 128;
    const int row = row0 + 32 * wq + fr;
    const uint32_t wrow = (uint32_t)row * (uint32_t)a.nb01;
    const int p0 = split * split_np;                        // first (global) phase of this split
    const int np = min(split_np, Kpad / (2 * MQ_BK) - p0);   // phases of this split (even)
    const int sb_last = (p0 + np - 1) / 2;                  // last super-block of this split
    uint8_t *const xslot = lds + grp * 3 * XB;
    uint8_t *const wslot = lds + 6 * XB;
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

    uint32_t x_off[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int r = 8 * (wq + 4 * v) + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        x_off[v] = ((uint32_t)(tok0 + r) * (uint32_t)Kpad + (uint32_t)c * 8u) * 2u;
    }
    auto step_of = [&](int p) { return 2 * (p0 + p) + grp; };
    auto dma_x = [&](int p, int slot, int v) {
        dma16(xr, xslot + slot * XB + (wq + 4 * v) * 1024, x_off[v] + (uint32_t)step_of(p) * MQ_BK * 2u);
    };
    // piece q of super-block gsb (data of min(gsb, sb_last)) into ring slot gsb % 3: chunk
    // c = 64 q + lane is 16-B piece i of row r's segment, rows in order
    auto dma_w = [&](int gsb, int q) {
        const int c = q * 64 + lane, r = c / (SB / 16), i = c % (SB / 16);
        const uint32_t off = (uint32_t)(row0 + r) * (uint32_t)a.nb01 + (uint32_t)min(gsb, sb_last) * SB + 16u * i;
        dma16(wr, wslot + (gsb % 3) * WSLOT + q * 1024, off);
    };
    // the wave's pieces of a slot are q = wave + 8t; half h takes t = h, h + 2, ...
    auto w_count = [&](int h) { const int tw = (NPIECE - wave + 7) / 8; return (tw - h + 1) / 2; };
    u32x4 sfrag[TN];
    auto load_sums = [&](int w) {
        const uint32_t rec = (uint32_t)(2 * (w + p0 / MQ_WIN) + grp);
#pragma unroll
        for (int j = 0; j < TN; ++j)
            sfrag[j] = bl128(sr, ((uint32_t)(tok0 + 32 * j + fr) * (uint32_t)nrec + rec) * 32u + 16u * fh);
    };
    // this lane's run of local phase p, read from the ring
    auto fetch = [&](Deq32<T> &w, int p) {
        const int st = step_of(p), gsb = st >> 2;
        w.lds(wslot + (gsb % 3) * WSLOT + (32 * wq + fr) * SB, st * MQ_BK + 32 * fh);
    };

    float16v acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    auto compute = [&](const u32x4 (&f)[4], int xsl) {
        const uint8_t *X = xslot + xsl * XB;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            half8 ax[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) ax[j] = *reinterpret_cast<const half8 *>(X + swz(32 * j + fr, 4 * fh + ks));
            const half8 bw = __builtin_bit_cast(half8, f[ks]);
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax[j], bw, acc[j], 0, 0, 0);
        }
    };
    u32x4 cw = {0u, 0u, 0u, 0u};
    auto correct = [&]() {
#pragma unroll
        for (int j = 0; j < TN; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, sfrag[j]), __builtin_bit_cast(half8, cw),
                                                            acc[j], 0, 0, 0);
        cw = u32x4{0u, 0u, 0u, 0u};
    };
    auto barrier = [&]() {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };

    uint32_t bad = 0;
    const DecK DK = DecK::make();
    Deq32<T> rw;
    u32x4 F[4], G[4];
    // prologue: the split's first two super-blocks, the activations of phases 0 and 1
    const int gsb0 = p0 / 2;
    load_sums(0);
#pragma unroll
    for (int t = 0; t < TMAX; ++t)
        if (wave + 8 * t < NPIECE) {
            dma_w(gsb0, wave + 8 * t);
            dma_w(gsb0 + 1, wave + 8 * t);
        }
#pragma unroll
    for (int v = 0; v < V; ++v) dma_x(0, 0, v);
#pragma unroll
    for (int v = 0; v < V; ++v) dma_x(min(1, np - 1), 1, v);
    wait_vmcnt<V>();   // everything but phase 1's activations
    barrier();
    fetch(rw, 0);
    cw[0] = rw.prep(bad);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) F[ks] = rw.frag(ks, DK);

    // phase p (SP = window slot of phase p+1, H = half of the super-block pieces it issues):
    // LDS reads (this step's activation fragments, next step's weight run) first, then NMF chunks
    // of one MFMA, a share of the DMA pieces (weights for super-block (P/2)+2, then the
    // activations of phase p+2) and of the decode; the activations of phase p+1 retire and one
    // barrier ends the phase
    constexpr int NMF = 4 * TN;
    auto phase = [&](auto SPc, const u32x4 (&fcur)[4], u32x4 (&fnext)[4], int p, int xs0) {
        constexpr int SP = decltype(SPc)::value;
        constexpr int H = (SP + 1) & 1;          // p % 2 (p0 is a multiple of MQ_WIN)
        constexpr int WMX = H ? WMAX1 : WMAX0, WLOW = H ? WLOW1 : WLOW0;
        constexpr int VMX = WMX + V;
        const int xs1 = xs0 == 2 ? 0 : xs0 + 1, xs2 = xs1 == 2 ? 0 : xs1 + 1;
        const int pl = min(p + 2, np - 1);
        const int gsb_dma = (p0 + p) / 2 + 2;
        const int wcnt = w_count(H);
        stamp(3);
        const uint8_t *X = xslot + xs0 * XB;
        half8 ax[4][TN];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
            for (int j = 0; j < TN; ++j) ax[ks][j] = *reinterpret_cast<const half8 *>(X + swz(32 * j + fr, 4 * fh + ks));
        fetch(rw, p + 1);
        stamp(0);
#pragma unroll
        for (int i = 0; i < NMF; ++i) {
            const int ks = i / TN, j = i % TN;
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax[ks][j], __builtin_bit_cast(half8, fcur[ks]), acc[j], 0, 0, 0);
#pragma unroll
            for (int l = i * VMX / NMF; l < (i + 1) * VMX / NMF; ++l) {
                if (l < WMX) {
                    if (l < wcnt) dma_w(gsb_dma, wave + 8 * (H + 2 * l));
                } else {
                    dma_x(pl, xs2, l - WMX);
                }
            }
            constexpr int PER = NMF / 4;
            if (i % PER == PER - 1) {
                if (i == PER - 1) cw[SP] = rw.prep(bad);
                fnext[i / PER] = rw.frag(i / PER, DK);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (SP == MQ_WIN - 1) {
            correct();
            load_sums((p + 2) / MQ_WIN);
        }
        stamp(1);
        // retire phase p+1's activations (issued last in the previous phase, after its weight
        // pieces): younger are at least this phase's pieces and the sums of a closing phase
        wait_vmcnt<V + WLOW + (SP == MQ_WIN - 1 || SP == 0 ? TN : 0)>();
        stamp(2);
        barrier();
        return xs1;
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I0 = std::integral_constant<int, 0>;
    int p = 0, xsl = 0;
    for (; p + MQ_WIN <= np - 1; p += MQ_WIN) {
        xsl = phase(I1{}, F, G, p, xsl);
        xsl = phase(I2{}, G, F, p + 1, xsl);
        xsl = phase(I3{}, F, G, p + 2, xsl);
        xsl = phase(I0{}, G, F, p + 3, xsl);
    }
    const int rem = np - 1 - p;
    if (rem >= 1) xsl = phase(I1{}, F, G, p, xsl);
    if (rem >= 2) xsl = phase(I2{}, G, F, p + 1, xsl);
    if (rem >= 3) xsl = phase(I3{}, F, G, p + 2, xsl);
    if (rem & 1) compute(G, xsl);
    else compute(F, xsl);
    if (rem != 3) correct();
    wait_vmcnt<0>();
    stamp(3);
    if constexpr (STAMP) {
        if (lane == 0 && a.stamps) {
            const int g = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
            unsigned long long *o = a.stamps + ((size_t)g * 8 + wave) * 8;
            o[0] = st_start;
            for (int i = 0; i < 5; ++i) o[1 + i] = st_seg[i];
            o[6] = st_t;
            o[7] = np;
        }
    }

    const bool bad_here = (bad & 0xFFFFu) >= F16_ONE || (bad >> 16) >= F16_ONE;
    float4 *park = reinterpret_cast<float4 *>(lds) + (size_t)(wq * 64 + lane) * 4 * TN;
    barrier();
    if (grp == 1) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                park[4 * j + q] = make_float4(acc[j][4 * q], acc[j][4 * q + 1], acc[j][4 * q + 2], acc[j][4 * q + 3]);
        const bool b1 = __builtin_amdgcn_ballot_w64(bad_here) != 0;
        if (lane == 0) g1_bad[wq] = b1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();
    if (grp == 1) return;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 o = park[4 * j + q];
            acc[j][4 * q] += o.x;
            acc[j][4 * q + 1] += o.y;
            acc[j][4 * q + 2] += o.z;
            acc[j][4 * q + 3] += o.w;
        }

    auto tok_of = [&](int j, int r) { return tok0 + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * fh; };
    if ((__builtin_amdgcn_ballot_w64(bad_here) != 0) || g1_bad[wq]) {   // fp32 path, as mmq_wave_kernel
        for (int j = 0; j < TN; ++j)
            for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
        for (int kr = p0 * 2 * MQ_BK; kr < min(a.K, (p0 + np) * 2 * MQ_BK); kr += 32) {
            Deq32<T> w;
            w.at(wrow, kr);
            for (int q = 0; q < Deq32<T>::NLOADS; ++q) w.part(wr, q);
            for (int e = 0; e < 32; ++e) {
                const float wf = w.w32(e);
                const int ke = kr + (e & ~3) + ((e & 3) == 1 ? 2 : (e & 3) == 2 ? 1 : (e & 3));
                for (int j = 0; j < TN; ++j)
                    for (int r = 0; r < 16; ++r) {
                        const int t = min(tok_of(j, r), tok_end - 1);
                        acc[j][r] += wf * (float)xs[(int64_t)t * Kpad + ke];
                    }
            }
        }
    }
    const float *xinv_s = xinv + (int64_t)slice * a.M;
    float inv[TN][16];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) inv[j][r] = xinv_s[min(tok_of(j, r), tok_end - 1)];
    if (row < a.N) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int tok = tok_of(j, r);
                if (tok < tok_end) {
                    float *drow = n_split > 1 ? part + (((int64_t)split * (gridDim.z / n_split) + slice) * a.M + tok) * a.N
                                              : reinterpret_cast<float *>(dmat + (int64_t)tok * a.nb1);
                    drow[row] = acc[j][r] * inv[j][r];
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
    const int64_t kpad = (a.K + 2 * MQ_BK - 1) / (2 * MQ_BK) * (2 * MQ_BK);   // the larger of both paths' padding
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

// dst[slice][token][row] = sum of the split-K partial tiles (mmq_wave_kernel with n_split > 1)
__global__ __launch_bounds__(256) void mmq_split_reduce(const MmArgs a, const float *__restrict__ part, int n_split,
                                                        int slices) {
    const int64_t per_slice = (int64_t)a.M * a.N;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= per_slice * slices) return;
    const int slice = (int)(i / per_slice);
    const int64_t rem = i % per_slice;
    const int tok = (int)(rem / a.N), row = (int)(rem % a.N);
    float v = 0.f;
    for (int s = 0; s < n_split; ++s) v += part[((int64_t)s * slices + slice) * per_slice + rem];
    const int i12 = slice % a.ne12, i13 = slice / a.ne12;
    reinterpret_cast<float *>(a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3 + (int64_t)tok * a.nb1)[row] = v;
}

template <int T, int TN>
static void launch_wave(const MmArgs &a, const _Float16 *x16, const _Float16 *xsum, const float *xinv, int Kpad, int slices,
                        int n_split, int split_np, float *part, hipStream_t st) {
    const dim3 grid((a.N + 127) / 128, (a.M + 32 * TN - 1) / (32 * TN), slices * n_split);
    // dword-aligned windows may end 2 bytes past the last block: round the range up to a dword
    // (buffer range checks are per dword; the extra bytes never leave the last page)
    const uint32_t w_extent = (uint32_t)(((int64_t)(a.N - 1) * a.nb01 + row_bytes(T, a.K) + 3) & ~(int64_t)3);
    const MoeMap none{};
    if (a.stamps && (size_t)grid.x * grid.y * grid.z * 64 <= 8 * 65536)
        hipLaunchKernelGGL((mmq_wave_kernel<T, TN, false, true>), grid, dim3(512), 0, st, a, x16, xsum, xinv, Kpad, w_extent, none,
                           n_split, split_np, part);
    else
        hipLaunchKernelGGL((mmq_wave_kernel<T, TN, false, false>), grid, dim3(512), 0, st, a, x16, xsum, xinv, Kpad, w_extent, none,
                           n_split, split_np, part);
}

template <int T, int TN>
static void launch_wl(const MmArgs &a, const _Float16 *x16, const _Float16 *xsum, const float *xinv, int Kpad, int slices,
                      int n_split, int split_np, float *part, hipStream_t st) {
    const dim3 grid((a.N + 127) / 128, (a.M + 32 * TN - 1) / (32 * TN), slices * n_split);
    const uint32_t w_extent = (uint32_t)(((int64_t)(a.N - 1) * a.nb01 + row_bytes(T, a.K) + 3) & ~(int64_t)3);
    if (a.stamps && (size_t)grid.x * grid.y * grid.z * 64 <= 8 * 65536)
        hipLaunchKernelGGL((mmq_wl_kernel<T, TN, true>), grid, dim3(512), 0, st, a, x16, xsum, xinv, Kpad, w_extent, n_split,
                           split_np, part);
    else
        hipLaunchKernelGGL((mmq_wl_kernel<T, TN, false>), grid, dim3(512), 0, st, a, x16, xsum, xinv, Kpad, w_extent, n_split,
                           split_np, part);
}

// mmq_wl_kernel needs every row's 256-k segment 16-B aligned
static bool wl_ok(int type, const MmArgs &a) {
    if (!(type == T_Q4_0 || type == T_Q8_0 || type == T_Q4_K || type == T_Q5_K)) return false;
    return a.K % 256 == 0 && (reinterpret_cast<uintptr_t>(a.w) & 15) == 0 && a.nb01 % 16 == 0 && a.nb02 % 16 == 0 &&
           a.nb03 % 16 == 0;
}

template <int T>
static void launch_wave_tn(int tile, const MmArgs &a, const _Float16 *x16, const _Float16 *xsum, const float *xinv, int Kpad,
                           int slices, int n_split, int split_np, float *part, hipStream_t st) {
    switch (tile) {
        case 20: if constexpr (T != T_Q6_K) launch_wl<T, 1>(a, x16, xsum, xinv, Kpad, slices, n_split, split_np, part, st); break;
        case 21: if constexpr (T != T_Q6_K) launch_wl<T, 2>(a, x16, xsum, xinv, Kpad, slices, n_split, split_np, part, st); break;
        case 10: launch_wave<T, 1>(a, x16, xsum, xinv, Kpad, slices, n_split, split_np, part, st); break;
        case 12: launch_wave<T, 4>(a, x16, xsum, xinv, Kpad, slices, n_split, split_np, part, st); break;
        default: launch_wave<T, 2>(a, x16, xsum, xinv, Kpad, slices, n_split, split_np, part, st); break;
    }
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
static int pick_tile(int type, const MmArgs &a, int slices) {
    static const char *env = getenv("GGML_MI355X_MMQ_TILE");
    if (env) {
        if (!strcmp(env, "64x128")) return 0;
        if (!strcmp(env, "128x64")) return 1;
        if (!strcmp(env, "128x128")) return 2;
        if (!strcmp(env, "128x128w4")) return 3;
        if (!strcmp(env, "64x128w4")) return 4;
        if (!strcmp(env, "wave32")) return 10;
        if (!strcmp(env, "wave64")) return 11;
        if (!strcmp(env, "wave128")) return 12;
        if (!strcmp(env, "wl32")) return wl_ok(type, a) ? 20 : 10;
        if (!strcmp(env, "wl64")) return wl_ok(type, a) ? 21 : 11;
    }
    auto wgs = [&](int bm, int bn) { return (int64_t)((a.N + bm - 1) / bm) * ((a.M + bn - 1) / bn) * slices; };
    // register-decode kernels (scripts/mmq_tiles.sh, round 2): with the weights staged through
    // LDS (mmq_wl_kernel, 16-B aligned 256-k row segments) for Q4_0 / Q4_K / Q5_K below a full
    // chip of 128x128 tiles and for any of the four at M <= 64 (Q4_K M=32 20 us vs 47,
    // M=512 45 vs 50); the per-lane-load variant for few tokens of misaligned Q4_0 / Q4_K / Q8_0.
    // Beyond, Q8_0 above 64 tokens and Q6_K: the LDS-staged f16 tiles.
    const bool wl = wl_ok(type, a);
    if (wl && a.M <= 64) return 20;
    if (wl && type != T_Q8_0 && wgs(128, 128) < 256) return a.M <= 128 ? 20 : 21;
    const bool light = type == T_Q4_0 || type == T_Q4_K || type == T_Q8_0;
    if (light && a.M <= 128 && (a.M <= 64 || type != T_Q8_0)) return 10;
    // LDS-staged tiles (scripts/mmq_sweep.sh): 128x128 once it fills the chip, otherwise the
    // 64-row tile (twice the workgroups) unless there are too few tokens for 128-token tiles
    if (wgs(128, 128) >= 256) return 2;
    return a.M > 64 ? 0 : 1;
}

hipError_t mmq_launch(int type, const MmArgs &a, hipStream_t st, Scratch &scratch) {
    const int slices = a.ne12 * a.ne13;
    const int tile = pick_tile(type, a, slices);
    const bool wave = tile >= 10;
    const int kq = wave ? 2 * MQ_BK : MQ_BK;   // the wave kernel's two K-groups take step pairs
    const int Kpad = (a.K + kq - 1) / kq * kq;
    // split-K for the wave kernel: workgroups for every CU, splits of whole run-sum windows
    // (MQ_WIN phases = 512 k each)
    int n_split = 1, split_np = Kpad / kq;
    if (wave) {
        const int tn = (tile == 10 || tile == 20) ? 1 : tile == 12 ? 4 : 2;
        const int64_t wgs = (int64_t)((a.N + 127) / 128) * ((a.M + 32 * tn - 1) / (32 * tn)) * slices;
        const int windows = (split_np + MQ_WIN - 1) / MQ_WIN;
        while (wgs * n_split < 256 && windows >= 2 * n_split) n_split *= 2;
        split_np = (windows + n_split - 1) / n_split * MQ_WIN;
        n_split = (Kpad / kq + split_np - 1) / split_np;
    }
    const size_t x16_bytes = ((size_t)slices * a.M * Kpad * sizeof(_Float16) + 255) & ~(size_t)255;
    const size_t sum_bytes = wave ? (((size_t)slices * a.M * ((Kpad + 511) / 512 * 2) * 32 + 255) & ~(size_t)255) : 0;
    const size_t part_bytes = n_split > 1 ? (((size_t)n_split * slices * a.M * a.N * sizeof(float) + 255) & ~(size_t)255) : 0;
    const size_t inv_bytes = (size_t)slices * a.M * sizeof(float);
    uint8_t *buf = static_cast<uint8_t *>(scratch.get(x16_bytes + sum_bytes + part_bytes + inv_bytes, st));
    if (!buf) return hipErrorOutOfMemory;
    _Float16 *x16 = reinterpret_cast<_Float16 *>(buf);
    _Float16 *xsum = reinterpret_cast<_Float16 *>(buf + x16_bytes);
    float *part = reinterpret_cast<float *>(buf + x16_bytes + sum_bytes);
    float *xinv = reinterpret_cast<float *>(buf + x16_bytes + sum_bytes + part_bytes);
    const dim3 cgrid(a.M, slices);
    if (wave) {
        hipLaunchKernelGGL(mmq_convert_x<true>, cgrid, dim3(CVT_T), 0, st, a, x16, xinv, Kpad, (const int *)nullptr, a.M, xsum);
        switch (type) {
            case T_Q4_0: launch_wave_tn<T_Q4_0>(tile, a, x16, xsum, xinv, Kpad, slices, n_split, split_np, part, st); break;
            case T_Q8_0: launch_wave_tn<T_Q8_0>(tile, a, x16, xsum, xinv, Kpad, slices, n_split, split_np, part, st); break;
            case T_Q4_K: launch_wave_tn<T_Q4_K>(tile, a, x16, xsum, xinv, Kpad, slices, n_split, split_np, part, st); break;
            case T_Q5_K: launch_wave_tn<T_Q5_K>(tile, a, x16, xsum, xinv, Kpad, slices, n_split, split_np, part, st); break;
            case T_Q6_K: launch_wave_tn<T_Q6_K>(tile, a, x16, xsum, xinv, Kpad, slices, n_split, split_np, part, st); break;
            default: return hipErrorInvalidValue;
        }
        if (n_split > 1) {
            const int64_t n = (int64_t)slices * a.M * a.N;
            hipLaunchKernelGGL(mmq_split_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, (const float *)part,
                               n_split, slices);
        }
        return hipGetLastError();
    }
    hipLaunchKernelGGL(mmq_convert_x<false>, cgrid, dim3(CVT_T), 0, st, a, x16, xinv, Kpad, (const int *)nullptr, a.M,
                       (_Float16 *)nullptr);
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

hipError_t moe_prep_launch(const MmArgs &a, int *offsets, int *tile_off, int *pos_pair, hipStream_t st) {
    hipLaunchKernelGGL(moe_prep, dim3(1), dim3(1024), 0, st, a, offsets, tile_off, pos_pair);
    return hipGetLastError();
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
    hipLaunchKernelGGL(mmq_convert_x<false>, dim3(P, 1), dim3(CVT_T), 0, st, a, x16, xinv, Kpad, (const int *)pos_pair, P,
                       (_Float16 *)nullptr);
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
