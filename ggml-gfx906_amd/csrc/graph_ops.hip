// graph_ops.hip — the non-matmul f32 ops of the GPT-2 graph, so that a
// ggml_backend_sched split keeps whole layers on an MI355X instead of bouncing to the CPU
// backend between the quantized MUL_MATs. Reference graph: examples/gpt-2/main-sched.cpp:590-858.
//
// Each kernel mirrors the ggml-cpu arithmetic it stands in for (cited per kernel), including
// where the CPU accumulates in double (NORM, SOFT_MAX) or rounds through fp16 (GELU's table),
// so the results are bit-identical to ggml-cpu wherever the CPU is itself order-independent.
// All of them are HBM/latency-bound elementwise or row-reduction kernels; none belongs on MFMA.
// Layouts are ggml's: ne/nb per dimension, any byte strides, dim 0 innermost.
#include "../../include/ggml-mi355x.h"
#include "dispatch.h"
#include "qcommon.h"
#include "settings.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace mi355x {

namespace {

struct DevT {
    char *p;
    int64_t ne[4];
    int64_t nb[4];
};

DevT dev(const TensorView &v) {
    DevT d;
    d.p = static_cast<char *>(v.data);
    for (int i = 0; i < 4; ++i) {
        d.ne[i] = v.ne[i];
        d.nb[i] = (int64_t)v.nb[i];
    }
    return d;
}

int64_t nrows(const TensorView &v) { return v.ne[1] * v.ne[2] * v.ne[3]; }
int64_t nelem(const TensorView &v) { return v.ne[0] * v.ne[1] * v.ne[2] * v.ne[3]; }
bool same_shape(const TensorView &a, const TensorView &b) {
    for (int i = 0; i < 4; ++i)
        if (a.ne[i] != b.ne[i]) return false;
    return true;
}
bool contiguous_rows(const TensorView &v, int esize) { return (int64_t)v.nb[0] == esize; }
bool is_contiguous(const TensorView &v, int esize) {
    int64_t s = esize;
    for (int i = 0; i < 4; ++i) {
        if (v.ne[i] != 1 && (int64_t)v.nb[i] != s) return false;
        s *= v.ne[i];
    }
    return true;
}

// row index -> (i1, i2, i3)
__device__ __forceinline__ void row_coords(int64_t r, const int64_t *ne, int64_t &i1, int64_t &i2, int64_t &i3) {
    i1 = r % ne[1];
    r /= ne[1];
    i2 = r % ne[2];
    i3 = r / ne[2];
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// block-wide reduction over 256 threads (4 waves) through LDS; every thread gets the result
template <typename F, typename R>
__device__ __forceinline__ R block_reduce(R v, R *lds, F op) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
    __syncthreads();
    if (lane == 0) lds[w] = v;
    __syncthreads();
    R r = lds[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = op(r, lds[i]);
    return r;
}

__device__ __forceinline__ float h2f_dev(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ uint16_t f2h_dev(float f) {
    // RNE, sign of zero kept (GGML_FP32_TO_FP16)
    const uint16_t h = __builtin_bit_cast(uint16_t, (_Float16)f);
    return (uint16_t)(h | ((__builtin_bit_cast(uint32_t, f) >> 16) & 0x8000u));
}

constexpr unsigned MAX_GRID = 1u << 20;

unsigned grid_for(int64_t n, int per) {
    const int64_t g = (n + per - 1) / per;
    return (unsigned)(g < (int64_t)MAX_GRID ? (g < 1 ? 1 : g) : MAX_GRID);
}

// ------------------------------------------------------------------------------------------
// binary ADD / SUB / MUL / DIV with src1 repeated over src0 (ggml_can_repeat), f32.
// ggml-cpu/binary-ops.cpp apply_binary_op: i1x = i0x % ne1x.
// ------------------------------------------------------------------------------------------
enum BinOp { B_ADD, B_SUB, B_MUL, B_DIV };

template <int OP>
__global__ __launch_bounds__(256) void binary_kernel(const DevT d, const DevT a, const DevT b, int64_t rows) {
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
        int64_t i1, i2, i3;
        row_coords(r, d.ne, i1, i2, i3);
        const char *pa = a.p + i1 * a.nb[1] + i2 * a.nb[2] + i3 * a.nb[3];
        const char *pb = b.p + (i1 % b.ne[1]) * b.nb[1] + (i2 % b.ne[2]) * b.nb[2] + (i3 % b.ne[3]) * b.nb[3];
        char *pd = d.p + i1 * d.nb[1] + i2 * d.nb[2] + i3 * d.nb[3];
        for (int64_t i0 = threadIdx.x; i0 < d.ne[0]; i0 += 256) {
            const float x = *reinterpret_cast<const float *>(pa + i0 * a.nb[0]);
            const float y = *reinterpret_cast<const float *>(pb + (i0 % b.ne[0]) * b.nb[0]);
            float z;
            if constexpr (OP == B_ADD) z = x + y;
            else if constexpr (OP == B_SUB) z = x - y;
            else if constexpr (OP == B_MUL) z = x * y;
            else z = x / y;
            *reinterpret_cast<float *>(pd + i0 * d.nb[0]) = z;
        }
    }
}

// ------------------------------------------------------------------------------------------
// NORM (ggml-cpu/ops.cpp:4067-4116): mean and variance accumulated in double like the CPU's
// ggml_float, v = x - mean in f32, y = v * (1/sqrtf(var + eps)). One wave per row.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void norm_kernel(const DevT d, const DevT a, int64_t rows, float eps) {
    const int lane = threadIdx.x & 63;
    const int64_t n0 = a.ne[0];
    for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (int64_t)gridDim.x * 4) {
        int64_t i1, i2, i3;
        row_coords(r, d.ne, i1, i2, i3);
        const char *pa = a.p + i1 * a.nb[1] + i2 * a.nb[2] + i3 * a.nb[3];
        char *pd = d.p + i1 * d.nb[1] + i2 * d.nb[2] + i3 * d.nb[3];
        double s = 0.0;
        for (int64_t i = lane; i < n0; i += 64) s += (double)*reinterpret_cast<const float *>(pa + i * a.nb[0]);
        s = wave_sum(s);
        const float mean = (float)(s / (double)n0);
        double s2 = 0.0;
        for (int64_t i = lane; i < n0; i += 64) {
            const float v = *reinterpret_cast<const float *>(pa + i * a.nb[0]) - mean;
            s2 += (double)(v * v);
        }
        s2 = wave_sum(s2);
        const float variance = (float)(s2 / (double)n0);
        const float scale = 1.0f / sqrtf(variance + eps);
        for (int64_t i = lane; i < n0; i += 64) {
            const float v = *reinterpret_cast<const float *>(pa + i * a.nb[0]) - mean;
            *reinterpret_cast<float *>(pd + i * d.nb[0]) = v * scale;
        }
    }
}

// ------------------------------------------------------------------------------------------
// SCALE (ggml-cpu/ops.cpp:4802-4852): y = x*s, or x*s + b when b != 0.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void scale_kernel(const DevT d, const DevT a, int64_t rows, float s, float bias) {
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
        int64_t i1, i2, i3;
        row_coords(r, d.ne, i1, i2, i3);
        const char *pa = a.p + i1 * a.nb[1] + i2 * a.nb[2] + i3 * a.nb[3];
        char *pd = d.p + i1 * d.nb[1] + i2 * d.nb[2] + i3 * d.nb[3];
        for (int64_t i0 = threadIdx.x; i0 < d.ne[0]; i0 += 256) {
            const float x = *reinterpret_cast<const float *>(pa + i0 * a.nb[0]);
            *reinterpret_cast<float *>(pd + i0 * d.nb[0]) = bias == 0.f ? x * s : fmaf(x, s, bias);
        }
    }
}

// ------------------------------------------------------------------------------------------
// DIAG_MASK_INF / DIAG_MASK_ZERO (ggml-cpu/ops.cpp:5597-5650): element (i0, i1) is replaced by
// `value` when i0 > n_past + i1; everything else is copied.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void diag_mask_kernel(const DevT d, const DevT a, int64_t rows, int n_past, float value) {
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
        int64_t i1, i2, i3;
        row_coords(r, d.ne, i1, i2, i3);
        const char *pa = a.p + i1 * a.nb[1] + i2 * a.nb[2] + i3 * a.nb[3];
        char *pd = d.p + i1 * d.nb[1] + i2 * d.nb[2] + i3 * d.nb[3];
        for (int64_t i0 = threadIdx.x; i0 < d.ne[0]; i0 += 256) {
            const float x = *reinterpret_cast<const float *>(pa + i0 * a.nb[0]);
            *reinterpret_cast<float *>(pd + i0 * d.nb[0]) = i0 > n_past + i1 ? value : x;
        }
    }
}

// ------------------------------------------------------------------------------------------
// SOFT_MAX (ggml-cpu/ops.cpp:5685-5795): w = x*scale + slope*mask (mask f32 or f16, broadcast
// over dims 2/3 by modulo, ALiBi slope from max_bias), optional per-head sink logits (src[2]);
// y = exp(w - max) / sum, the sum accumulated in double. One 256-thread workgroup per row.
// ------------------------------------------------------------------------------------------
struct SoftMaxP {
    float scale, max_bias, m0, m1;
    uint32_t n_head_log2;
    int mask_type;  // -1 none, 0 f32, 1 f16
    bool sinks;
    // fused SCALE -> DIAG_MASK_INF producers (backend graph fusion): x <- x * pre_s (+ pre_b),
    // then -inf where i0 > n_past + i1 (pre_n_past >= 0), exactly as scale_kernel /
    // diag_mask_kernel write their outputs
    bool pre;
    float pre_s, pre_b;
    int pre_n_past;
};

__global__ __launch_bounds__(256) void soft_max_kernel(const DevT d, const DevT a, const DevT m, const DevT sk, int64_t rows,
                                                       const SoftMaxP p) {
    __shared__ float red_f[4];
    __shared__ double red_d[4];
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
        int64_t i1, i2, i3;
        row_coords(r, a.ne, i1, i2, i3);
        const char *pa = a.p + i1 * a.nb[1] + i2 * a.nb[2] + i3 * a.nb[3];
        char *pd = d.p + i1 * d.nb[1] + i2 * d.nb[2] + i3 * d.nb[3];
        const char *pm = nullptr;
        if (p.mask_type >= 0) pm = m.p + i1 * m.nb[1] + (i2 % m.ne[2]) * m.nb[2] + (i3 % m.ne[3]) * m.nb[3];
        const uint32_t h = (uint32_t)i2;
        const float slope = p.max_bias > 0.f ? (h < p.n_head_log2 ? powf(p.m0, (float)(h + 1))
                                                                  : powf(p.m1, (float)(2 * (h - p.n_head_log2) + 1)))
                                             : 1.f;
        auto w_at = [&](int64_t i) {
            float x = *reinterpret_cast<const float *>(pa + i * a.nb[0]);
            if (p.pre) {
                x = p.pre_b == 0.f ? x * p.pre_s : fmaf(x, p.pre_s, p.pre_b);
                if (p.pre_n_past >= 0 && i > p.pre_n_past + i1) x = -INFINITY;
            }
            float w = x * p.scale;
            if (pm) {
                const float mv = p.mask_type == 0 ? *reinterpret_cast<const float *>(pm + i * m.nb[0])
                                                  : h2f_dev(*reinterpret_cast<const uint16_t *>(pm + i * m.nb[0]));
                w += slope * mv;
            }
            return w;
        };
        float mx = -INFINITY;
        for (int64_t i = threadIdx.x; i < a.ne[0]; i += 256) mx = fmaxf(mx, w_at(i));
        mx = block_reduce(mx, red_f, [](float x, float y) { return fmaxf(x, y); });
        const float snk = p.sinks ? *reinterpret_cast<const float *>(sk.p + i2 * sk.nb[0]) : 0.f;
        if (p.sinks) mx = fmaxf(mx, snk);
        double s = 0.0;
        for (int64_t i = threadIdx.x; i < a.ne[0]; i += 256) s += (double)expf(w_at(i) - mx);
        s = block_reduce(s, red_d, [](double x, double y) { return x + y; });
        if (p.sinks) s += (double)expf(snk - mx);
        const float inv = (float)(1.0 / s);
        for (int64_t i = threadIdx.x; i < a.ne[0]; i += 256)
            *reinterpret_cast<float *>(pd + i * d.nb[0]) = expf(w_at(i) - mx) * inv;
    }
}

// ------------------------------------------------------------------------------------------
// UNARY GELU (ggml-cpu/vec.h:601-646 with GGML_GELU_FP16): x <= -10 -> 0, x >= 10 -> x, else
// the fp16 table lookup, i.e. fp16(gelu_tanh(fp16(x))) with the table built in f32
// (ggml-cpu.c:3542).
// ------------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void gelu_kernel(const DevT d, const DevT a, int64_t rows) {
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
        int64_t i1, i2, i3;
        row_coords(r, d.ne, i1, i2, i3);
        const char *pa = a.p + i1 * a.nb[1] + i2 * a.nb[2] + i3 * a.nb[3];
        char *pd = d.p + i1 * d.nb[1] + i2 * d.nb[2] + i3 * d.nb[3];
        for (int64_t i0 = threadIdx.x; i0 < d.ne[0]; i0 += 256) {
            const float x = *reinterpret_cast<const float *>(pa + i0 * a.nb[0]);
            *reinterpret_cast<float *>(pd + i0 * d.nb[0]) = gelu_ggml(x);
        }
    }
}

// ------------------------------------------------------------------------------------------
// CPY / CONT / DUP between f32 and f16 (ggml-cpu/ops.cpp ggml_compute_forward_dup_*): element
// e of src in ggml's flattened order goes to element e of dst in dst's flattened order. When
// the shapes agree (CONT, DUP, permuted copies) one coordinate decomposition serves both.
// ------------------------------------------------------------------------------------------
template <typename TS, typename TD>
__device__ __forceinline__ TD cvt(TS v);
template <> __device__ __forceinline__ float cvt<float, float>(float v) { return v; }
template <> __device__ __forceinline__ uint16_t cvt<float, uint16_t>(float v) { return f2h_dev(v); }
template <> __device__ __forceinline__ float cvt<uint16_t, float>(uint16_t v) { return h2f_dev(v); }
template <> __device__ __forceinline__ uint16_t cvt<uint16_t, uint16_t>(uint16_t v) { return v; }

// up to two independent copies per launch (blockIdx.y picks one): the backend pairs adjacent
// CPY nodes such as GPT-2's K and V cache writes (main-sched.cpp:654-655)
struct CpyPair {
    DevT d0, a0, d1, a1;
    int64_t rows0, rows1;
};

template <typename TS, typename TD, bool SAME>
__global__ __launch_bounds__(256) void cpy_kernel(const CpyPair c) {
    const bool second = blockIdx.y != 0;
    const DevT d = second ? c.d1 : c.d0, a = second ? c.a1 : c.a0;
    const int64_t rows = second ? c.rows1 : c.rows0;
    // iterate over src rows; dst coordinates follow from the flattened index
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
        int64_t i1, i2, i3;
        row_coords(r, a.ne, i1, i2, i3);
        const char *pa = a.p + i1 * a.nb[1] + i2 * a.nb[2] + i3 * a.nb[3];
        if constexpr (SAME) {
            char *pd = d.p + i1 * d.nb[1] + i2 * d.nb[2] + i3 * d.nb[3];
            for (int64_t i0 = threadIdx.x; i0 < a.ne[0]; i0 += 256)
                *reinterpret_cast<TD *>(pd + i0 * d.nb[0]) = cvt<TS, TD>(*reinterpret_cast<const TS *>(pa + i0 * a.nb[0]));
        } else {
            const int64_t base = r * a.ne[0];
            for (int64_t i0 = threadIdx.x; i0 < a.ne[0]; i0 += 256) {
                int64_t e = base + i0;
                const int64_t j0 = e % d.ne[0]; e /= d.ne[0];
                const int64_t j1 = e % d.ne[1]; e /= d.ne[1];
                const int64_t j2 = e % d.ne[2];
                const int64_t j3 = e / d.ne[2];
                *reinterpret_cast<TD *>(d.p + j0 * d.nb[0] + j1 * d.nb[1] + j2 * d.nb[2] + j3 * d.nb[3]) =
                    cvt<TS, TD>(*reinterpret_cast<const TS *>(pa + i0 * a.nb[0]));
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// float MUL_MAT: src0 f32/f16 [K, N, ne02, ne03] x src1 f32 [K, M, ne12, ne13] -> dst f32
// [N, M, ne12, ne13], src0 broadcast over dims 2/3 (ggml-cpu.c:1133-1134). These are GPT-2's
// attention products KQ and KQV (main-sched.cpp:687, 726): K of 64 or n_kv, tiny N/M per head.
// One wave per (src0 row, 4 columns); lanes stride K and reduce with DPP shuffles.
// ------------------------------------------------------------------------------------------
template <typename TA>
__global__ __launch_bounds__(256) void mm_float_kernel(const DevT d, const DevT a, const DevT b) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t c0 = (int64_t)blockIdx.y * 4;
    const int64_t i12 = blockIdx.z % b.ne[2], i13 = blockIdx.z / b.ne[2];
    if (row >= a.ne[1]) return;
    const int64_t i02 = i12 / (b.ne[2] / a.ne[2]), i03 = i13 / (b.ne[3] / a.ne[3]);
    const char *pa = a.p + row * a.nb[1] + i02 * a.nb[2] + i03 * a.nb[3];
    const char *pb = b.p + i12 * b.nb[2] + i13 * b.nb[3];
    const int nc = (int)min<int64_t>(4, b.ne[1] - c0);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int64_t k = lane; k < a.ne[0]; k += 64) {
        float w;
        if constexpr (sizeof(TA) == 4) w = *reinterpret_cast<const float *>(pa + k * a.nb[0]);
        else w = h2f_dev(*reinterpret_cast<const uint16_t *>(pa + k * a.nb[0]));
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (c < nc) acc[c] = fmaf(w, *reinterpret_cast<const float *>(pb + (c0 + c) * b.nb[1] + k * b.nb[0]), acc[c]);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float s = wave_sum(acc[c]);
        if (lane == c && c < nc)
            *reinterpret_cast<float *>(d.p + row * d.nb[0] + (c0 + c) * d.nb[1] + i12 * d.nb[2] + i13 * d.nb[3]) = s;
    }
}


// ------------------------------------------------------------------------------------------
// fused attention (backend graph fusion, see AttnView): one workgroup per (query, head).
//   scores: 16 lanes per key, lane l reads d = l, l+16, ... (64-B runs of a key row), 4 DPP/
//     shuffle steps reduce them; the scalar chain per score is the one ggml applies node by
//     node: (dot * s [+ b]) -> -inf above the causal diagonal -> * soft_max scale.
//   soft_max: block max, exp, sum in double (as soft_max_kernel / ggml-cpu ops.cpp:5685-5795).
//   output: lane = d (256-B V^T row segments), 4 waves over keys, LDS sum, * 1/sum.
// Latency-bound at decode sizes (n_q * H workgroups of n_kv * D * 8 bytes of K and V).
// ------------------------------------------------------------------------------------------
template <typename T> __device__ __forceinline__ float ldf(const char *p);
template <> __device__ __forceinline__ float ldf<float>(const char *p) { return *reinterpret_cast<const float *>(p); }
template <> __device__ __forceinline__ float ldf<uint16_t>(const char *p) { return h2f_dev(*reinterpret_cast<const uint16_t *>(p)); }

template <typename TK, typename TV>
__global__ __launch_bounds__(256) void attn_kernel(const AttnView a) {
    extern __shared__ float sc[];                  // [n_kv] scores, then exp(score - max)
    __shared__ float qs[ATTN_MAX_D];
    __shared__ float red_f[4];
    __shared__ double red_d[4];
    __shared__ float part[4][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = tid & 15;
    const int i = blockIdx.x, h = blockIdx.y, hk = h / (a.H / a.Hk);
    const char *qp = static_cast<const char *>(a.q) + i * a.q_i + h * a.q_h;
    for (int d = tid; d < a.D; d += 256) qs[d] = *reinterpret_cast<const float *>(qp + d * a.q_d);
    __syncthreads();
    const char *kb = static_cast<const char *>(a.k) + hk * a.k_h;
    float mx = -INFINITY;
    for (int j0 = 0; j0 < a.n_kv; j0 += 16) {
        const int j = j0 + (tid >> 4);
        float acc = 0.f;
        if (j < a.n_kv) {
            const char *kp = kb + (int64_t)j * a.k_j;
            for (int d = l16; d < a.D; d += 16) acc = fmaf(ldf<TK>(kp + d * a.k_d), qs[d], acc);
        }
        acc += __shfl_xor(acc, 8, 64);
        acc += __shfl_xor(acc, 4, 64);
        acc += __shfl_xor(acc, 2, 64);
        acc += __shfl_xor(acc, 1, 64);
        if (j < a.n_kv) {
            float x = a.pre_b == 0.f ? acc * a.pre_s : fmaf(acc, a.pre_s, a.pre_b);
            if (a.n_past >= 0 && j > a.n_past + i) x = -INFINITY;
            const float w = x * a.sm_scale;
            if (l16 == 0) sc[j] = w;
            mx = fmaxf(mx, w);
        }
    }
    mx = block_reduce(mx, red_f, [](float x, float y) { return fmaxf(x, y); });
    double sum = 0.0;
    for (int j = tid; j < a.n_kv; j += 256) {
        const float e = expf(sc[j] - mx);
        sc[j] = e;
        sum += (double)e;
    }
    sum = block_reduce(sum, red_d, [](double x, double y) { return x + y; });   // (its barriers publish sc)
    const float inv = (float)(1.0 / sum);
    const char *vb = static_cast<const char *>(a.v) + hk * a.v_h;
    char *ob = static_cast<char *>(a.o) + i * a.o_i + h * a.o_h;
    for (int d0 = 0; d0 < a.D; d0 += 64) {
        const int d = d0 + lane;
        float o = 0.f;
        if (d < a.D)
            for (int j = wave; j < a.n_kv; j += 4) o = fmaf(sc[j] * inv, ldf<TV>(vb + (int64_t)j * a.v_j + d * a.v_d), o);
        part[wave][lane] = o;
        __syncthreads();
        if (wave == 0 && d < a.D)
            *reinterpret_cast<float *>(ob + d * a.o_d) = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
        __syncthreads();
    }
}

// D = 64, f32 K / V with unit d stride and 16-B aligned rows (GPT-2's caches): the same
// arithmetic with one dependent memory round trip at decode sizes. Every load that does not
// depend on a score is issued first: q, this thread's key row (16 float4) and the first
// ATTN_VPRE V^T rows of its output slot; the softmax runs while they land.
//   scores: one key per thread (more keys: further rounds of 256)
//   output: 16 lanes x float4 cover d, 16 key slots per workgroup
constexpr int ATTN_VPRE = 8;   // V^T rows prefetched per slot: n_kv <= 128 needs no further loads

__global__ __launch_bounds__(256) void attn_kernel_d64(const AttnView a) {
    extern __shared__ float sc[];
    __shared__ float4 q4[16];
    __shared__ float red_f[4];
    __shared__ double red_d[4];
    __shared__ float4 part[4][16];
    const int tid = threadIdx.x, wave = tid >> 6, l16 = tid & 15, slot = tid >> 4;
    const int i = blockIdx.x, h = blockIdx.y, hk = h / (a.H / a.Hk);
    const char *qp = static_cast<const char *>(a.q) + i * a.q_i + h * a.q_h;
    const char *kb = static_cast<const char *>(a.k) + hk * a.k_h;
    const char *vb = static_cast<const char *>(a.v) + hk * a.v_h + l16 * 16;
    const int n_kv = a.n_kv;
    float qv = 0.f;
    if (tid < 64) qv = *reinterpret_cast<const float *>(qp + tid * a.q_d);
    float4 kv[16];
    {
        const float4 *kr = reinterpret_cast<const float4 *>(kb + (int64_t)min(tid, n_kv - 1) * a.k_j);
#pragma unroll
        for (int u = 0; u < 16; ++u) kv[u] = kr[u];
    }
    float4 vv[ATTN_VPRE];
#pragma unroll
    for (int u = 0; u < ATTN_VPRE; ++u)
        vv[u] = *reinterpret_cast<const float4 *>(vb + (int64_t)min(slot + 16 * u, n_kv - 1) * a.v_j);
    if (tid < 64) reinterpret_cast<float *>(q4)[tid] = qv;
    __syncthreads();
    auto score = [&](int j, const float4 (&k)[16]) {
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const float4 q = q4[u];
            acc = fmaf(k[u].x, q.x, acc);
            acc = fmaf(k[u].y, q.y, acc);
            acc = fmaf(k[u].z, q.z, acc);
            acc = fmaf(k[u].w, q.w, acc);
        }
        float x = a.pre_b == 0.f ? acc * a.pre_s : fmaf(acc, a.pre_s, a.pre_b);
        if (a.n_past >= 0 && j > a.n_past + i) x = -INFINITY;
        return x * a.sm_scale;
    };
    float mx = -INFINITY;
    if (tid < n_kv) {
        const float w = score(tid, kv);
        sc[tid] = w;
        mx = w;
    }
    for (int j = tid + 256; j < n_kv; j += 256) {
        const float4 *kr = reinterpret_cast<const float4 *>(kb + (int64_t)j * a.k_j);
#pragma unroll
        for (int u = 0; u < 16; ++u) kv[u] = kr[u];
        const float w = score(j, kv);
        sc[j] = w;
        mx = fmaxf(mx, w);
    }
    mx = block_reduce(mx, red_f, [](float x, float y) { return fmaxf(x, y); });
    double sum = 0.0;
    for (int j = tid; j < n_kv; j += 256) {   // the keys this thread scored
        const float e = expf(sc[j] - mx);
        sc[j] = e;
        sum += (double)e;
    }
    sum = block_reduce(sum, red_d, [](double x, double y) { return x + y; });   // (its barriers publish sc)
    const float inv = (float)(1.0 / sum);
    float4 o0 = make_float4(0.f, 0.f, 0.f, 0.f), o1 = o0;
    auto acc4 = [](float4 &o, float p, float4 v) {
        o.x = fmaf(p, v.x, o.x); o.y = fmaf(p, v.y, o.y); o.z = fmaf(p, v.z, o.z); o.w = fmaf(p, v.w, o.w);
    };
#pragma unroll
    for (int u = 0; u < ATTN_VPRE; ++u) {
        const int j = slot + 16 * u;
        if (j < n_kv) acc4((u & 1) ? o1 : o0, sc[j] * inv, vv[u]);
    }
    int j = slot + 16 * ATTN_VPRE;
    for (; j + 16 < n_kv; j += 32) {
        const float4 v0 = *reinterpret_cast<const float4 *>(vb + (int64_t)j * a.v_j);
        const float4 v1 = *reinterpret_cast<const float4 *>(vb + (int64_t)(j + 16) * a.v_j);
        acc4(o0, sc[j] * inv, v0);
        acc4(o1, sc[j + 16] * inv, v1);
    }
    if (j < n_kv) acc4(o0, sc[j] * inv, *reinterpret_cast<const float4 *>(vb + (int64_t)j * a.v_j));
    float4 o = make_float4(o0.x + o1.x, o0.y + o1.y, o0.z + o1.z, o0.w + o1.w);
    // the 4 key slots of a wave: lanes l16, l16+16, l16+32, l16+48
#pragma unroll
    for (int sh = 16; sh <= 32; sh <<= 1) {
        o.x += __shfl_xor(o.x, sh, 64);
        o.y += __shfl_xor(o.y, sh, 64);
        o.z += __shfl_xor(o.z, sh, 64);
        o.w += __shfl_xor(o.w, sh, 64);
    }
    if ((tid & 63) < 16) part[wave][l16] = o;
    __syncthreads();
    if (tid < 64) {
        const int d = tid;   // 64 outputs, one per lane of wave 0
        const float *pp = reinterpret_cast<const float *>(part);
        const float r = (pp[d] + pp[64 + d]) + (pp[128 + d] + pp[192 + d]);
        *reinterpret_cast<float *>(static_cast<char *>(a.o) + i * a.o_i + h * a.o_h + d * a.o_d) = r;
    }
}

bool f32(const TensorView &v) { return v.type == T_F32; }
bool f32_or_f16(const TensorView &v) { return v.type == T_F32 || v.type == T_F16; }
int esize(int t) { return t == T_F16 ? 2 : 4; }

float fparam(const GraphOp &g, int i) {
    float f;
    std::memcpy(&f, &g.params[i], sizeof f);
    return f;
}

}  // namespace

int check_graph_op(const GraphOp &g) {
    const TensorView &d = g.dst, &a = g.src[0];
    if (!g.has_src[0]) return GGML_MI355X_EINVAL;
    for (int i = 0; i < 4; ++i)
        if (d.ne[i] < 0 || a.ne[i] < 0) return GGML_MI355X_EINVAL;
    switch (g.op) {
        case GOP_ADD: case GOP_SUB: case GOP_MUL: case GOP_DIV: {
            if (!g.has_src[1]) return GGML_MI355X_EINVAL;
            const TensorView &b = g.src[1];
            if (!f32(d) || !f32(a) || !f32(b) || !same_shape(a, d)) return GGML_MI355X_EINVAL;
            for (int i = 0; i < 4; ++i)
                if (b.ne[i] <= 0 || a.ne[i] % b.ne[i] != 0) return GGML_MI355X_EINVAL;
            return GGML_MI355X_OK;
        }
        case GOP_NORM:
        case GOP_SCALE:
        case GOP_DIAG_MASK_INF:
        case GOP_DIAG_MASK_ZERO:
        case GOP_GELU:
            return f32(d) && f32(a) && same_shape(a, d) ? GGML_MI355X_OK : GGML_MI355X_EINVAL;
        case GOP_SOFT_MAX: {
            if (!f32(d) || !f32(a) || !same_shape(a, d)) return GGML_MI355X_EINVAL;
            if (g.has_src[1]) {
                const TensorView &m = g.src[1];
                if (!f32_or_f16(m) || m.ne[0] != a.ne[0] || m.ne[1] < a.ne[1]) return GGML_MI355X_EINVAL;
                if (m.ne[2] <= 0 || m.ne[3] <= 0 || a.ne[2] % m.ne[2] != 0 || a.ne[3] % m.ne[3] != 0) return GGML_MI355X_EINVAL;
            }
            if (g.has_src[2] && (!f32(g.src[2]) || g.src[2].ne[0] < a.ne[2])) return GGML_MI355X_EINVAL;
            return GGML_MI355X_OK;
        }
        case GOP_CPY:
            if (!f32_or_f16(a) || !f32_or_f16(d) || nelem(a) != nelem(d)) return GGML_MI355X_EINVAL;
            return GGML_MI355X_OK;
        case GOP_MUL_MAT: {
            if (!g.has_src[1]) return GGML_MI355X_EINVAL;
            const TensorView &b = g.src[1];
            if (!f32_or_f16(a) || !f32(b) || !f32(d)) return GGML_MI355X_EINVAL;
            if (a.ne[0] != b.ne[0] || d.ne[0] != a.ne[1] || d.ne[1] != b.ne[1] || d.ne[2] != b.ne[2] || d.ne[3] != b.ne[3])
                return GGML_MI355X_EINVAL;
            if (a.ne[2] <= 0 || a.ne[3] <= 0 || b.ne[2] % a.ne[2] != 0 || b.ne[3] % a.ne[3] != 0) return GGML_MI355X_EINVAL;
            if (b.ne[2] * b.ne[3] > 65535 || (b.ne[1] + 3) / 4 > 65535) return GGML_MI355X_EINVAL;
            return GGML_MI355X_OK;
        }
        default:
            return GGML_MI355X_EINVAL;
    }
}

int run_graph_op(const GraphOp &g, hipStream_t st) { return run_graph_op_pre(g, nullptr, st); }

namespace {
int cpy_key(const GraphOp &g) { return (g.src[0].type == T_F16 ? 2 : 0) + (g.dst.type == T_F16 ? 1 : 0); }
}  // namespace

bool cpy_pairable(const GraphOp &g0, const GraphOp &g1) {
    return g0.op == GOP_CPY && g1.op == GOP_CPY && check_graph_op(g0) == GGML_MI355X_OK && check_graph_op(g1) == GGML_MI355X_OK &&
           cpy_key(g0) == cpy_key(g1) && same_shape(g0.src[0], g0.dst) == same_shape(g1.src[0], g1.dst);
}

// one CPY, or two pairable ones (cpy_pairable; the caller checked they are independent) in one launch
int run_cpy_pair(const GraphOp &g0, const GraphOp *g1, hipStream_t st) {
    int rc = check_graph_op(g0);
    if (rc == GGML_MI355X_OK && g1) rc = cpy_pairable(g0, *g1) ? GGML_MI355X_OK : GGML_MI355X_EINVAL;
    if (rc != GGML_MI355X_OK) return rc;
    CpyPair c{};
    c.d0 = dev(g0.dst);
    c.a0 = dev(g0.src[0]);
    c.rows0 = nelem(g0.dst) == 0 ? 0 : nrows(g0.src[0]);
    if (g1) {
        c.d1 = dev(g1->dst);
        c.a1 = dev(g1->src[0]);
        c.rows1 = nelem(g1->dst) == 0 ? 0 : nrows(g1->src[0]);
    }
    const int64_t rows = std::max(c.rows0, c.rows1);
    if (rows == 0) return GGML_MI355X_OK;
    const dim3 grid(grid_for(rows, 1), g1 ? 2 : 1);
    const bool same = same_shape(g0.src[0], g0.dst);
#define CPY_CASE(K, TS, TD)                                                                     \
    case K:                                                                                     \
        if (same) hipLaunchKernelGGL((cpy_kernel<TS, TD, true>), grid, dim3(256), 0, st, c);   \
        else hipLaunchKernelGGL((cpy_kernel<TS, TD, false>), grid, dim3(256), 0, st, c);       \
        break;
    switch (cpy_key(g0)) {
        CPY_CASE(0, float, float)
        CPY_CASE(1, float, uint16_t)
        CPY_CASE(2, uint16_t, float)
        CPY_CASE(3, uint16_t, uint16_t)
    }
#undef CPY_CASE
    return hipGetLastError() == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
}

int run_attention(const AttnView &a, hipStream_t st) {
    if (a.D < 1 || a.D > ATTN_MAX_D || a.n_kv < 1 || a.n_kv > ATTN_MAX_KV || a.n_q < 1 || a.H < 1 || a.Hk < 1 ||
        a.H % a.Hk != 0 || a.n_q > 65535 || a.H > 65535)
        return GGML_MI355X_EINVAL;
    const dim3 grid((unsigned)a.n_q, (unsigned)a.H);
    const size_t lds = (size_t)a.n_kv * sizeof(float);
    auto al16 = [](const void *p, int64_t s1, int64_t s2) { return (uintptr_t)p % 16 == 0 && s1 % 16 == 0 && s2 % 16 == 0; };
    const bool generic = settings().attn_generic;   // A/B switch
    if (!generic && a.D == 64 && !a.k_f16 && !a.v_f16 && a.k_d == 4 && a.v_d == 4 && al16(a.k, a.k_j, a.k_h) &&
        al16(a.v, a.v_j, a.v_h)) {
        hipLaunchKernelGGL(attn_kernel_d64, grid, dim3(256), lds, st, a);
    } else if (a.k_f16 && a.v_f16) hipLaunchKernelGGL((attn_kernel<uint16_t, uint16_t>), grid, dim3(256), lds, st, a);
    else if (a.k_f16) hipLaunchKernelGGL((attn_kernel<uint16_t, float>), grid, dim3(256), lds, st, a);
    else if (a.v_f16) hipLaunchKernelGGL((attn_kernel<float, uint16_t>), grid, dim3(256), lds, st, a);
    else hipLaunchKernelGGL((attn_kernel<float, float>), grid, dim3(256), lds, st, a);
    return hipGetLastError() == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
}

// SCALE -> DIAG_MASK_INF -> SOFT_MAX as one launch (backend fusion): g is the SOFT_MAX node with
// src[0] replaced by the SCALE node's input
int run_soft_max_pre(const GraphOp &g, const SoftmaxPre &pre, hipStream_t st) {
    if (g.op != GOP_SOFT_MAX) return GGML_MI355X_EINVAL;
    return run_graph_op_pre(g, &pre, st);
}

int run_graph_op_pre(const GraphOp &g, const SoftmaxPre *pre, hipStream_t st) {
    const int rc = check_graph_op(g);
    if (rc != GGML_MI355X_OK) return rc;
    const TensorView &dv = g.dst, &av = g.src[0];
    if (nelem(dv) == 0) return GGML_MI355X_OK;
    const DevT d = dev(dv), a = dev(av);
    const int64_t rows = nrows(dv);
    const dim3 blk(256);
    switch (g.op) {
        case GOP_ADD: case GOP_SUB: case GOP_MUL: case GOP_DIV: {
            const DevT b = dev(g.src[1]);
            const dim3 grid(grid_for(rows, 1));
            switch (g.op) {
                case GOP_ADD: hipLaunchKernelGGL(binary_kernel<B_ADD>, grid, blk, 0, st, d, a, b, rows); break;
                case GOP_SUB: hipLaunchKernelGGL(binary_kernel<B_SUB>, grid, blk, 0, st, d, a, b, rows); break;
                case GOP_MUL: hipLaunchKernelGGL(binary_kernel<B_MUL>, grid, blk, 0, st, d, a, b, rows); break;
                default: hipLaunchKernelGGL(binary_kernel<B_DIV>, grid, blk, 0, st, d, a, b, rows); break;
            }
            break;
        }
        case GOP_NORM:
            hipLaunchKernelGGL(norm_kernel, dim3(grid_for(rows, 4)), blk, 0, st, d, a, rows, fparam(g, 0));
            break;
        case GOP_SCALE:
            hipLaunchKernelGGL(scale_kernel, dim3(grid_for(rows, 1)), blk, 0, st, d, a, rows, fparam(g, 0), fparam(g, 1));
            break;
        case GOP_DIAG_MASK_INF:
        case GOP_DIAG_MASK_ZERO:
            hipLaunchKernelGGL(diag_mask_kernel, dim3(grid_for(rows, 1)), blk, 0, st, d, a, rows, g.params[0],
                               g.op == GOP_DIAG_MASK_INF ? -INFINITY : 0.0f);
            break;
        case GOP_SOFT_MAX: {
            SoftMaxP p{};
            if (pre) {
                p.pre = true;
                p.pre_s = pre->scale;
                p.pre_b = pre->bias;
                p.pre_n_past = pre->n_past;
            }
            p.scale = fparam(g, 0);
            p.max_bias = fparam(g, 1);
            const uint32_t n_head = (uint32_t)av.ne[2];
            p.n_head_log2 = 1u << (uint32_t)std::floor(std::log2((double)n_head));
            p.m0 = std::pow(2.0f, -(p.max_bias) / p.n_head_log2);
            p.m1 = std::pow(2.0f, -(p.max_bias / 2.0f) / p.n_head_log2);
            p.mask_type = g.has_src[1] ? (g.src[1].type == T_F16 ? 1 : 0) : -1;
            p.sinks = g.has_src[2];
            const DevT m = g.has_src[1] ? dev(g.src[1]) : DevT{};
            const DevT sk = g.has_src[2] ? dev(g.src[2]) : DevT{};
            hipLaunchKernelGGL(soft_max_kernel, dim3(grid_for(rows, 1)), blk, 0, st, d, a, m, sk, rows, p);
            break;
        }
        case GOP_GELU:
            hipLaunchKernelGGL(gelu_kernel, dim3(grid_for(rows, 1)), blk, 0, st, d, a, rows);
            break;
        case GOP_CPY:
            return run_cpy_pair(g, nullptr, st);
        case GOP_MUL_MAT: {
            const DevT b = dev(g.src[1]);
            const dim3 grid((unsigned)((av.ne[1] + 3) / 4), (unsigned)((g.src[1].ne[1] + 3) / 4),
                            (unsigned)(g.src[1].ne[2] * g.src[1].ne[3]));
            if (av.type == T_F16) hipLaunchKernelGGL(mm_float_kernel<uint16_t>, grid, blk, 0, st, d, a, b);
            else hipLaunchKernelGGL(mm_float_kernel<float>, grid, blk, 0, st, d, a, b);
            break;
        }
        default:
            return GGML_MI355X_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
}

}  // namespace mi355x
