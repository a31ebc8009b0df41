// mmvq_solo.hip — the single-column mat-vec as one wave per workgroup, for the single-matrix
// decode shape (one src1 column, K <= 4096, K % 64 == 0): the north-star launch (Q4_K 4096 x
// 4096, M = 1) and BASELINE configs[1] / [2].
//
// The 8-wave kernel of mmvq_impl.h shares one quantized copy of the column between its waves
// through LDS: each wave quantizes an eighth of K, and a workgroup barrier waits for the last
// one before any dot. In a single launch that barrier is the critical path: the slowest wave's
// activations queue in the CU's load path behind the other waves' weight loads, and the
// weights of every wave then wait for it (profiles/r06_single_launch_decomposition.txt: without
// the barrier the launch is 1.2 us shorter; with activations, quantization and weights removed
// it is 2.2 us shorter). Here lane l of every wave owns slot l of every row (64 weights), so it
// needs only the 64 activations of that slot: it loads them itself (16-B loads, L2 hits after the
// first wave), quantizes them in its own registers — per 32-block d = amax / 127 and
// round-to-nearest-even, the arithmetic of xblock_store bit for bit (Q6_K: a slot holds half of
// each of four 32-blocks, the other half is lane l ^ 1's, one DPP exchange per block) — and dots
// its slot of R rows. No LDS, no barrier: each wave depends on its own loads only. The cost is
// more activation traffic per CU (every wave reads the whole column: 16 KB against 9-18 KB of
// weights per wave).
//
// Same arithmetic as the 8-wave kernel: the same int8 activation blocks and block dots; the R row
// sums of a lane meet across the 64 lanes in its butterfly transpose (group_reduce_transpose), so
// with R rows per wave a row's sum equals that kernel's at RPW = R bit for bit.
#include "mmvq_impl.h"
#include "settings.h"

#include <string>

namespace mi355x {

namespace {

// the K positions of part j (16 values) of slot s: 64 s + 16 j, or Q6_K's interleave
template <int T>
__device__ __forceinline__ int slot_part_k(int s, int j) {
    if constexpr (T == T_Q6_K) return 256 * (s >> 2) + 128 * ((s >> 1) & 1) + 16 * (s & 1) + 32 * j;
    else return 64 * s + 16 * j;
}

// quantize 32 values (two 16-value parts, lo = elements 0..15, hi = 16..31 of one 32-block) the
// way xblock_store does: d = amax / 127, t = x * (127 / amax) + (1.5 * 2^23 + 128), code = low
// byte - 128; returns the 8 code dwords (lo: 0..3, hi: 4..7), d and sum(q) of each 16-run
__device__ __forceinline__ void q32(const float (&lo)[16], const float (&hi)[16], float amax, uint32_t (&w)[8], float &d, int &s_lo,
                                    int &s_hi) {
    d = amax * (1.0f / 127.f);
    const float id = amax > 0.f ? 127.f * __builtin_amdgcn_rcpf(amax) : 0.f;
    constexpr float MAGIC = 12582912.0f + 128.0f;
    auto pack = [&](const float *v) {
        uint32_t b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) b[i] = __builtin_bit_cast(uint32_t, __builtin_fmaf(v[i], id, MAGIC));
        return __builtin_amdgcn_perm(__builtin_amdgcn_perm(b[3], b[2], 0x0c0c0400u), __builtin_amdgcn_perm(b[1], b[0], 0x0c0c0400u),
                                     0x05040100u);
    };
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        w[i] = pack(lo + 4 * i);
        w[4 + i] = pack(hi + 4 * i);
    }
    s_lo = (int)__builtin_amdgcn_udot4(w[0], 0x01010101u, __builtin_amdgcn_udot4(w[1], 0x01010101u,
             __builtin_amdgcn_udot4(w[2], 0x01010101u, __builtin_amdgcn_udot4(w[3], 0x01010101u, 0u, false), false), false), false) - 2048;
    s_hi = (int)__builtin_amdgcn_udot4(w[4], 0x01010101u, __builtin_amdgcn_udot4(w[5], 0x01010101u,
             __builtin_amdgcn_udot4(w[6], 0x01010101u, __builtin_amdgcn_udot4(w[7], 0x01010101u, 0u, false), false), false), false) - 2048;
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] ^= 0x80808080u;
}

__device__ __forceinline__ float amax16(const float (&v)[16]) {
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) m = fmaxf(m, fabsf(v[i]));
    return m;
}

// one wave = one workgroup; R rows per wave, lane l = slot l (K <= 4096: nslots <= 64)
template <int T, int R, bool XA>
__global__ __launch_bounds__(WAVE) void mmvq_solo_kernel(const MmArgs a) {
    constexpr int NX = XdCount<T>::n;
    constexpr int V = pow2ceil(R);
    const int lane = threadIdx.x;
    const int nslots = a.K / 64;
    const int s = min(lane, nslots - 1);                 // (lanes past K repeat the last slot, masked)
    const int r0 = blockIdx.x * R;
    const uint8_t *wmat = a.w;
    const float *x = reinterpret_cast<const float *>(a.x);
    const int nblk = a.K / QT<T>::blck;
    // diagnostics (GGML_MI355X_STAMPS): per wave start / activations in registers / quantized /
    // end (s_memrealtime) and the shader clock (s_memtime), scripts/solo_stamps.py
    unsigned long long *const st = a.stamps != nullptr && lane == 0 ? a.stamps + (int64_t)blockIdx.x * 8 : nullptr;
    if (st) { st[0] = __builtin_amdgcn_s_memrealtime(); st[4] = __builtin_amdgcn_s_memtime(); }

    // ---- the slot's 64 activations first (four 16-value parts), then the R rows' weights
    float xv[4][16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float *p = x + slot_part_k<T>(s, j);
        if constexpr (XA) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 f = reinterpret_cast<const float4 *>(p)[q];
                xv[j][4 * q] = f.x; xv[j][4 * q + 1] = f.y; xv[j][4 * q + 2] = f.z; xv[j][4 * q + 3] = f.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) xv[j][q] = p[q];
        }
    }
    Frag<T> f[R];
#pragma unroll
    for (int r = 0; r < R; ++r) f[r].template load<false>(wmat + (int64_t)min(r0 + r, a.N - 1) * a.nb01, s, nblk);
    __builtin_amdgcn_sched_barrier(0);

    // ---- quantize the slot in registers: X[16] dwords in part order (parts 0..3 = the Frag's
    // j), dx / sx as Frag::dot expects them
    if (st) {   // (the probe consumes this lane's first and last activation: all have landed)
        float probe = xv[0][0] + xv[3][15];
        asm volatile("" : "+v"(probe));
        st[1] = __builtin_amdgcn_s_memrealtime() + (probe == 12345.f);
    }
    uint32_t X[16];
    float dx[NX], sx[NX];
    if constexpr (T == T_Q6_K) {
        // part j of slot s is the (s & 1) half of 32-block 8 sb + 4 h + j: amax over the block
        // needs the partner lane's half (lane ^ 1); sx = d * sum(q) per 16-run (this lane's)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float am = amax16(xv[j]);
            am = fmaxf(am, dpp_f<DPP_XOR1>(am));
            const float d = am * (1.0f / 127.f);
            const float id = am > 0.f ? 127.f * __builtin_amdgcn_rcpf(am) : 0.f;
            constexpr float MAGIC = 12582912.0f + 128.0f;
            uint32_t w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t b[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) b[k] = __builtin_bit_cast(uint32_t, __builtin_fmaf(xv[j][4 * i + k], id, MAGIC));
                w[i] = __builtin_amdgcn_perm(__builtin_amdgcn_perm(b[3], b[2], 0x0c0c0400u), __builtin_amdgcn_perm(b[1], b[0], 0x0c0c0400u),
                                             0x05040100u);
            }
            const int qs = (int)__builtin_amdgcn_udot4(w[0], 0x01010101u, __builtin_amdgcn_udot4(w[1], 0x01010101u,
                             __builtin_amdgcn_udot4(w[2], 0x01010101u, __builtin_amdgcn_udot4(w[3], 0x01010101u, 0u, false), false), false), false) - 2048;
#pragma unroll
            for (int i = 0; i < 4; ++i) X[4 * j + i] = w[i] ^ 0x80808080u;
            dx[j] = d;
            sx[j] = d * (float)qs;
        }
    } else {
        // parts 0, 1 = block 2s, parts 2, 3 = block 2s + 1
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const float am = fmaxf(amax16(xv[2 * b]), amax16(xv[2 * b + 1]));
            uint32_t w[8];
            float d;
            int s_lo, s_hi;
            q32(xv[2 * b], xv[2 * b + 1], am, w, d, s_lo, s_hi);
#pragma unroll
            for (int i = 0; i < 8; ++i) X[8 * b + i] = w[i];
            dx[b] = d;
            sx[b] = d * (float)(s_lo + s_hi);
        }
    }

    if (st) {
        uint32_t probe = X[0] ^ X[15];
        asm volatile("" : "+v"(probe));
        st[2] = __builtin_amdgcn_s_memrealtime() + (probe == 12345u);
    }
    // ---- dots and the cross-lane sum
    const float live = lane < nslots ? 1.f : 0.f;
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = live * f[r].dot(X, dx, sx);
    const float sum = group_reduce_transpose<V, 64>(acc);
    constexpr int SHIFT = 6 - Log2<V>::v;
    const int idx = lane >> SHIFT;
    if ((lane & ((1 << SHIFT) - 1)) == 0 && idx < R && r0 + idx < a.N) reinterpret_cast<float *>(a.dst)[r0 + idx] = sum;
    if (st) { st[3] = __builtin_amdgcn_s_memrealtime(); st[5] = __builtin_amdgcn_s_memtime(); }
}

template <int T, int R>
hipError_t solo_one(const MmArgs &a, hipStream_t st) {
    const dim3 grid((a.N + R - 1) / R);
    if (a.x_aligned16) hipLaunchKernelGGL((mmvq_solo_kernel<T, R, true>), grid, dim3(WAVE), 0, st, a);
    else hipLaunchKernelGGL((mmvq_solo_kernel<T, R, false>), grid, dim3(WAVE), 0, st, a);
    return hipGetLastError();
}

template <int T>
hipError_t solo_type(const MmArgs &a, int rows, hipStream_t st) {
    switch (rows) {
        case 2: return solo_one<T, 2>(a, st);
        case 4: return solo_one<T, 4>(a, st);
        case 8: return solo_one<T, 8>(a, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

// shapes it takes: one column, one matrix, K a multiple of 64 up to 4096 (one slot per lane)
bool mmvq_solo_supported(const MmArgs &a) {
    return a.M == 1 && a.ne12 == 1 && a.ne13 == 1 && a.K % 64 == 0 && a.K >= 64 && a.K <= 4096;
}

// the default (settings().solo < 0): Q8_0 and Q6_K from K = 1536 (or up to 1024 rows), Q4_K /
// Q5_K from 8192 rows. Measured first as
// rocprof kernel durations (profiles/r06_solo_singles_ab.txt: 8 rows per wave Q4_0 4096^2
// 5.14-5.20 vs 5.33-5.39 us for the 8-wave kernel, Q4_K 4096^2 5.30-5.32 vs 5.47-5.54), then as
// hipGraph periods of back-to-back calls, what a decode graph runs (profiles/r06_valu_plan_sweep.txt):
// there the 8-wave kernel is ahead at 4096 rows (Q4_0 4096^2 4.51 vs 4.75 us, Q4_K 4.67 vs 4.90,
// Q5_K 5.23 vs 5.74, and Q4_0 at 11008 rows) and this kernel from 11008 rows for the K-quants
// (Q4_K 4096 x 11008 8.48 vs 8.83, Q5_K 10.17 vs 10.32, Q6_K 11.12 vs 12.18, and at 14336 rows;
// Q6_K already at 4096 rows: 2048 x 4096 4.98 vs 5.51, 4096^2 5.62 vs 5.73, and short
// matrices: 3072 x 768 3.4 vs 4.0 with 64-lane rows; Q8_0 at every shape measured: 4096^2 5.26
// vs 5.55, 3072 x 768 3.19 vs 3.41, 4096 x 11008 11.56 vs 12.16; but at K = 768, where a wave
// has 12 slots, 768 x 50257 16.4 vs 10.2). Q4_0 / Q4_K / Q5_K below 8192 rows: the 8-wave kernel
// with 64-lane rows is ahead (mmvq.hip lanes_per_row).
// Two rows per wave are 1.4-1.7x slower (the column is re-read per wave).
bool mmvq_solo_default(int type, const MmArgs &a) {
    const int s = settings().solo;
    if (s == 0 || !mmvq_solo_supported(a)) return false;
    if (s > 0) return true;
    if (type == T_Q8_0 || type == T_Q6_K) return a.K >= 1536 || a.N <= 1024;   // (K = 768: 12 of 64 lanes live)
    return a.N >= 8192 && (type == T_Q4_K || type == T_Q5_K);
}

static int solo_rows_default(int type) { return type == T_Q6_K ? 4 : 8; }
int mmvq_solo_rows(int type, const MmArgs &) { return settings().solo > 1 ? settings().solo : solo_rows_default(type); }

std::string mmvq_solo_plan_text(int type, const MmArgs &a) {
    const int r = mmvq_solo_rows(type, a);
    return "mmvq-solo rows=" + std::to_string(r) + " grid=" + std::to_string((a.N + r - 1) / r);
}

hipError_t mmvq_solo_launch(int type, const MmArgs &a, hipStream_t st) {
    if (!mmvq_solo_supported(a)) return hipErrorInvalidValue;
    const int r = mmvq_solo_rows(type, a);
    switch (type) {
        case T_Q4_0: return solo_type<T_Q4_0>(a, r, st);
        case T_Q8_0: return solo_type<T_Q8_0>(a, r, st);
        case T_Q4_K: return solo_type<T_Q4_K>(a, r, st);
        case T_Q5_K: return solo_type<T_Q5_K>(a, r, st);
        case T_Q6_K: return solo_type<T_Q6_K>(a, r, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mi355x
