// qcommon.h — shared device-side definitions for the MI355X quantized MUL_MAT path.
//
// Block layouts are the ggml on-disk/in-memory formats (reference src/ggml-common.h:170-344);
// the kernels read them in place (no repacking), so a ggml tensor uploaded by set_tensor is
// consumed byte-for-byte.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi355x {

// ggml type ids (reference include/ggml.h:372-412)
enum : int {
    T_F32 = 0, T_F16 = 1, T_Q4_0 = 2, T_Q8_0 = 8, T_Q4_K = 12, T_Q5_K = 13, T_Q6_K = 14, T_I32 = 26,
};

constexpr int WAVE = 64;

template <int T> struct QT;
template <> struct QT<T_Q4_0> { static constexpr int blck = 32,  bytes = 18;  };
template <> struct QT<T_Q8_0> { static constexpr int blck = 32,  bytes = 34;  };
template <> struct QT<T_Q4_K> { static constexpr int blck = 256, bytes = 144; };
template <> struct QT<T_Q5_K> { static constexpr int blck = 256, bytes = 176; };
template <> struct QT<T_Q6_K> { static constexpr int blck = 256, bytes = 210; };

// 16-byte / 8-byte / 4-byte loads that only assume 2-byte alignment. gfx950 runs with
// unaligned global access enabled (HSA default), so these still lower to one
// global_load_dwordx4/x2/dword; the hot configurations are 4- or 16-byte aligned anyway.
struct __attribute__((packed, aligned(2))) u32x4_a2 { uint32_t v[4]; };
struct __attribute__((packed, aligned(2))) u32x2_a2 { uint32_t v[2]; };
struct __attribute__((packed, aligned(2))) u32x1_a2 { uint32_t v; };

__device__ __forceinline__ void ld16(const uint8_t *p, uint32_t *o) {
    const u32x4_a2 t = *reinterpret_cast<const u32x4_a2 *>(p);
    o[0] = t.v[0]; o[1] = t.v[1]; o[2] = t.v[2]; o[3] = t.v[3];
}
__device__ __forceinline__ void ld8(const uint8_t *p, uint32_t *o) {
    const u32x2_a2 t = *reinterpret_cast<const u32x2_a2 *>(p);
    o[0] = t.v[0]; o[1] = t.v[1];
}
__device__ __forceinline__ uint32_t ld4(const uint8_t *p) { return reinterpret_cast<const u32x1_a2 *>(p)->v; }
__device__ __forceinline__ uint16_t ld2(const uint8_t *p) { return *reinterpret_cast<const uint16_t *>(p); }

__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }

// 4-way int8 dot with int32 accumulate (v_dot4_i32_i8)
__device__ __forceinline__ int dot4(uint32_t a, uint32_t b, int c) {
    return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

// bytewise (b - 8) for b in [0,15]  -> int8 in [-8,7]    (no inter-byte carries)
__device__ __forceinline__ uint32_t sub8_bytes(uint32_t v) { return (v + 0x78787878u) ^ 0x80808080u; }
// bytewise (b - 32) for b in [0,63] -> int8 in [-32,31]
__device__ __forceinline__ uint32_t sub32_bytes(uint32_t v) { return (v + 0x60606060u) ^ 0x80808080u; }

// funnel: bytes [off, off+4) of the 8-byte little-endian pair (lo, hi)
__device__ __forceinline__ uint32_t align2(uint32_t hi, uint32_t lo) { return __builtin_amdgcn_alignbyte(hi, lo, 2); }

// Q4_K / Q5_K 6-bit (scale, min) for sub-blocks 2c and 2c+1 of a super-block whose 12
// scale bytes are S[0..2] (restates get_scale_min_k4, reference src/ggml-quants.c:703-710,
// in the 32-bit form of src/ggml-cpu/quants.c:580-585, branch-free for per-lane c).
__device__ __forceinline__ void k4_scale_min_pair(const uint32_t S[3], int c, uint32_t &sc0, uint32_t &sc1,
                                                  uint32_t &m0, uint32_t &m1) {
    const uint32_t sc_lo = S[0] & 0x3f3f3f3fu;                                         // scales j=0..3
    const uint32_t sc_hi = (S[2] & 0x0f0f0f0fu) | (((S[0] >> 6) & 0x03030303u) << 4);   // scales j=4..7
    const uint32_t mn_lo = S[1] & 0x3f3f3f3fu;                                         // mins   j=0..3
    const uint32_t mn_hi = ((S[2] >> 4) & 0x0f0f0f0fu) | (((S[1] >> 6) & 0x03030303u) << 4);
    const uint32_t sw = c < 2 ? sc_lo : sc_hi;
    const uint32_t mw = c < 2 ? mn_lo : mn_hi;
    const int sh = (c & 1) * 16;
    sc0 = (sw >> sh) & 0xff;
    sc1 = (sw >> (sh + 8)) & 0xff;
    m0  = (mw >> sh) & 0xff;
    m1  = (mw >> (sh + 8)) & 0xff;
}

// ------------------------------------------------------------------------------------------
// cross-lane exchange without the LDS pipe: DPP within rows of 16, permlane swaps across
// rows / halves (gfx950 v_permlane16_swap / v_permlane32_swap). Each returns the value of
// lane (lane ^ mask) for the listed partner pattern.
//   xor1  quad_perm [1,0,3,2]        xor2  quad_perm [2,3,0,1]
//   mir7  row_half_mirror (lane ^ 7 inside each 8)
//   mir15 row_mirror      (lane ^ 15 inside each 16)
//   sw16  lane ^ 16                    sw32  lane ^ 32
// The mirrors flip the low bits too; reductions that only combine symmetric partial sums
// (and the butterfly below, which consumes the bits from high to low) stay exact.
// ------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, dpp_u<CTRL>(__builtin_bit_cast(uint32_t, v)));
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_MIR7 = 0x141, DPP_MIR15 = 0x140;
constexpr int DPP_ROR4 = 0x124, DPP_ROR8 = 0x128;   // row_ror: rotate within 16-lane rows

__device__ __forceinline__ float swap16_f(float v) {
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return __builtin_bit_cast(float, (threadIdx.x & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ float swap32_f(float v) {
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return __builtin_bit_cast(float, (threadIdx.x & 32) ? r[0] : r[1]);
}

// partner value for butterfly distance D (D = 32, 16, 8, 4, 2, 1)
template <int D> __device__ __forceinline__ float xchg(float v);
template <> __device__ __forceinline__ float xchg<32>(float v) { return swap32_f(v); }
template <> __device__ __forceinline__ float xchg<16>(float v) { return swap16_f(v); }
template <> __device__ __forceinline__ float xchg<8>(float v) { return dpp_f<DPP_MIR15>(v); }
template <> __device__ __forceinline__ float xchg<4>(float v) { return dpp_f<DPP_MIR7>(v); }
template <> __device__ __forceinline__ float xchg<2>(float v) { return dpp_f<DPP_XOR2>(v); }
template <> __device__ __forceinline__ float xchg<1>(float v) { return dpp_f<DPP_XOR1>(v); }

// Workgroup barrier for LDS hand-offs only: this wave's LDS operations complete, then s_barrier.
// __syncthreads() is a release/acquire fence at workgroup scope, which also waits for every
// outstanding global load (vmcnt(0)) — it would drain a weight stream issued ahead of the
// barrier. No kernel here passes data between waves through global memory. Both instructions
// sit in ONE asm statement with a "memory" clobber: __builtin_amdgcn_s_barrier() alone is
// modelled as touching no memory, so LDS accesses could legally be moved across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// full 64-lane sum, result in every lane
__device__ __forceinline__ float wave_sum(float v) {
    v += xchg<1>(v);
    v += xchg<2>(v);
    v += xchg<4>(v);
    v += xchg<8>(v);
    v += xchg<16>(v);
    v += xchg<32>(v);
    return v;
}

// fp32 -> fp16 RNE keeping the sign of zero (GGML_FP32_TO_FP16, reference src/ggml-impl.h:358-405)
__device__ __forceinline__ uint16_t f2h_rne(float f) {
    const uint16_t h = __builtin_bit_cast(uint16_t, (_Float16)f);
    return (uint16_t)(h | ((__builtin_bit_cast(uint32_t, f) >> 16) & 0x8000u));
}

// GELU as ggml-cpu evaluates it (src/ggml-cpu/vec.h:601-646 with GGML_GELU_FP16): x <= -10 -> 0,
// x >= 10 -> x, else the fp16 table entry, i.e. fp16(gelu_tanh(fp16(x))) with the table built
// in f32 (src/ggml-cpu/ggml-cpu.c:3542).
__device__ __forceinline__ float gelu_ggml(float x) {
    constexpr float GELU_COEF_A = 0.044715f;
    constexpr float SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
    if (x <= -10.0f) return 0.0f;
    if (x >= 10.0f) return x;
    const float xh = h2f(f2h_rne(x));
    return h2f(f2h_rne(0.5f * xh * (1.0f + tanhf(SQRT_2_OVER_PI * xh * (1.0f + GELU_COEF_A * xh * xh)))));
}

}  // namespace mi355x
