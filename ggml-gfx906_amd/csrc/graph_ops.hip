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

#include <cmath>
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

template <typename TS, typename TD, bool SAME>
__global__ __launch_bounds__(256) void cpy_kernel(const DevT d, const DevT a, int64_t rows) {
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
        case GOP_CPY: {
            const int64_t srows = nrows(av);
            const dim3 grid(grid_for(srows, 1));
            const bool same = same_shape(av, dv);
            const int key = (av.type == T_F16 ? 2 : 0) + (dv.type == T_F16 ? 1 : 0);
#define CPY_CASE(K, TS, TD)                                                                                     \
    case K:                                                                                                     \
        if (same) hipLaunchKernelGGL((cpy_kernel<TS, TD, true>), grid, blk, 0, st, d, a, srows);              \
        else hipLaunchKernelGGL((cpy_kernel<TS, TD, false>), grid, blk, 0, st, d, a, srows);                  \
        break;
            switch (key) {
                CPY_CASE(0, float, float)
                CPY_CASE(1, float, uint16_t)
                CPY_CASE(2, uint16_t, float)
                CPY_CASE(3, uint16_t, uint16_t)
            }
#undef CPY_CASE
            break;
        }
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
