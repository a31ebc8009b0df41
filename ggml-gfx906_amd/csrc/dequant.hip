// dequant.hip — device dequantization, bit-exact with the reference's dequantize_row_*
// (src/ggml-quants.c:307-323, 401-415, 1352-1374, 1554-1579, 1762-1791).
//
// Each product/difference is formed with explicitly rounded IEEE ops (__fmul_rn / __fsub_rn)
// so the compiler cannot contract d*q - m into an FMA: the reference's ggml-base is built
// without FMA, and the oracle tests require identical bits.
#include "deq.h"

namespace mi355x {

template <int T>
__global__ void dequant_kernel(const uint8_t *__restrict__ src, float *__restrict__ dst, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t b = i / QT<T>::blck;
    dst[i] = deq_one<T>(src + b * QT<T>::bytes, (int)(i - b * QT<T>::blck));
}

hipError_t dequant_launch(int type, const void *src, float *dst, int64_t n, hipStream_t st) {
    const int threads = 256;
    const dim3 grid((unsigned)((n + threads - 1) / threads));
    const uint8_t *s = static_cast<const uint8_t *>(src);
    switch (type) {
        case T_Q4_0: hipLaunchKernelGGL(dequant_kernel<T_Q4_0>, grid, dim3(threads), 0, st, s, dst, n); break;
        case T_Q8_0: hipLaunchKernelGGL(dequant_kernel<T_Q8_0>, grid, dim3(threads), 0, st, s, dst, n); break;
        case T_Q4_K: hipLaunchKernelGGL(dequant_kernel<T_Q4_K>, grid, dim3(threads), 0, st, s, dst, n); break;
        case T_Q5_K: hipLaunchKernelGGL(dequant_kernel<T_Q5_K>, grid, dim3(threads), 0, st, s, dst, n); break;
        case T_Q6_K: hipLaunchKernelGGL(dequant_kernel<T_Q6_K>, grid, dim3(threads), 0, st, s, dst, n); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// GET_ROWS: dst[i12][i11][i10][:] = dequantize_row(src0 row idx[i12][i11][i10] of matrix
// (i11, i12)) — src/ggml-cpu/ops.cpp:5121-5163 (get_rows_q), src/ggml.c:3617-3637 (shapes).
// Bit-exact: the same per-element formulas as dequantize_row_*. An index outside [0, ne01) is
// the reference's GGML_ASSERT (ops.cpp:5157): the kernel raises the device error word (a
// vector store into host-mapped memory, read by the host after the stream synchronizes) and
// writes nothing for that row, so it never reads outside src0.
// ------------------------------------------------------------------------------------------
struct RowsArgs {
    const uint8_t *src; int64_t nb01, nb02, nb03, ne01;
    const uint8_t *idx; int64_t nb10, nb11, nb12, ne10, ne11;
    uint8_t *dst; int64_t nb1, nb2, nb3;
    int64_t ne00;
    int *err;
};

__device__ __forceinline__ bool row_in_range(int64_t r, const RowsArgs &a) {
    if (r >= 0 && r < a.ne01) return true;
    __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return false;
}

template <int T>
__global__ __launch_bounds__(256) void get_rows_kernel(const RowsArgs a) {
    const int64_t row = blockIdx.y;                      // flattened (i10, i11, i12)
    const int64_t i12 = row / (a.ne10 * a.ne11);
    const int64_t i11 = (row - i12 * a.ne10 * a.ne11) / a.ne10;
    const int64_t i10 = row - i12 * a.ne10 * a.ne11 - i11 * a.ne10;
    const int64_t i01 = *reinterpret_cast<const int32_t *>(a.idx + i10 * a.nb10 + i11 * a.nb11 + i12 * a.nb12);
    if (!row_in_range(i01, a)) return;
    const uint8_t *srow = a.src + i01 * a.nb01 + i11 * a.nb02 + i12 * a.nb03;
    float *drow = reinterpret_cast<float *>(a.dst + i10 * a.nb1 + i11 * a.nb2 + i12 * a.nb3);
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.ne00) return;
    if constexpr (T == T_F32) {
        drow[i] = reinterpret_cast<const float *>(srow)[i];
    } else {
        const int64_t b = i / QT<T>::blck;
        drow[i] = deq_one<T>(srow + b * QT<T>::bytes, (int)(i - b * QT<T>::blck));
    }
}

// GET_ROWS(a) + GET_ROWS(b) -> ADD in one launch (the GPT-2 embedding, main-sched.cpp:589-595:
// wte rows + wpe rows): each output element is the same dequantized values and the same single
// fp32 addition as the three nodes, so the result is bit-identical. b is f32; both index one
// 2-D matrix with a 1-D row list (the host checks).
template <int T>
__global__ __launch_bounds__(256) void get_rows_add_kernel(const RowsArgs a, const RowsArgs b) {
    const int64_t row = blockIdx.y;
    const int64_t ia = *reinterpret_cast<const int32_t *>(a.idx + row * a.nb10);
    const int64_t ib = *reinterpret_cast<const int32_t *>(b.idx + row * b.nb10);
    if (!row_in_range(ia, a) || !row_in_range(ib, b)) return;
    const uint8_t *sa = a.src + ia * a.nb01;
    const float *sb = reinterpret_cast<const float *>(b.src + ib * b.nb01);
    float *drow = reinterpret_cast<float *>(a.dst + row * a.nb1);
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.ne00) return;
    float va;
    if constexpr (T == T_F32) {
        va = reinterpret_cast<const float *>(sa)[i];
    } else {
        const int64_t bl = i / QT<T>::blck;
        va = deq_one<T>(sa + bl * QT<T>::bytes, (int)(i - bl * QT<T>::blck));
    }
    drow[i] = __fadd_rn(va, sb[i]);
}

hipError_t get_rows_add_launch(int type, const RowsArgs &a, const RowsArgs &b, int64_t nrows, hipStream_t st) {
    const dim3 grid((unsigned)((a.ne00 + 255) / 256), (unsigned)nrows);
    switch (type) {
        case T_F32: hipLaunchKernelGGL(get_rows_add_kernel<T_F32>, grid, dim3(256), 0, st, a, b); break;
        case T_Q4_0: hipLaunchKernelGGL(get_rows_add_kernel<T_Q4_0>, grid, dim3(256), 0, st, a, b); break;
        case T_Q8_0: hipLaunchKernelGGL(get_rows_add_kernel<T_Q8_0>, grid, dim3(256), 0, st, a, b); break;
        case T_Q4_K: hipLaunchKernelGGL(get_rows_add_kernel<T_Q4_K>, grid, dim3(256), 0, st, a, b); break;
        case T_Q5_K: hipLaunchKernelGGL(get_rows_add_kernel<T_Q5_K>, grid, dim3(256), 0, st, a, b); break;
        case T_Q6_K: hipLaunchKernelGGL(get_rows_add_kernel<T_Q6_K>, grid, dim3(256), 0, st, a, b); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t get_rows_launch(int type, const RowsArgs &a, int64_t nrows, hipStream_t st) {
    const dim3 grid((unsigned)((a.ne00 + 255) / 256), (unsigned)nrows);
    switch (type) {
        case T_F32: hipLaunchKernelGGL(get_rows_kernel<T_F32>, grid, dim3(256), 0, st, a); break;
        case T_Q4_0: hipLaunchKernelGGL(get_rows_kernel<T_Q4_0>, grid, dim3(256), 0, st, a); break;
        case T_Q8_0: hipLaunchKernelGGL(get_rows_kernel<T_Q8_0>, grid, dim3(256), 0, st, a); break;
        case T_Q4_K: hipLaunchKernelGGL(get_rows_kernel<T_Q4_K>, grid, dim3(256), 0, st, a); break;
        case T_Q5_K: hipLaunchKernelGGL(get_rows_kernel<T_Q5_K>, grid, dim3(256), 0, st, a); break;
        case T_Q6_K: hipLaunchKernelGGL(get_rows_kernel<T_Q6_K>, grid, dim3(256), 0, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// f32 -> Q4_0 / Q8_0 (GGML_OP_CPY into a quantized tensor; the reference GPU path is
// cpy_f32_q, src/ggml-cuda/cpy.cu:66-94). One thread per 32-block, bit-exact with
// quantize_row_q4_0_ref / quantize_row_q8_0_ref (src/ggml-quants.c:36-71, 199-222): the same
// sequential max search, correctly rounded division, and separately rounded mul / add.
// ------------------------------------------------------------------------------------------
struct QuantArgs {
    const uint8_t *src; int64_t nb01, nb02, nb03;        // f32 rows (nb00 == 4)
    uint8_t *dst; int64_t nb1, nb2, nb3;                  // quantized rows (nb0 == block bytes)
    int64_t ne0, ne1, ne2, ne3;
};

template <int T>
__global__ __launch_bounds__(256) void quantize_kernel(const QuantArgs a) {
    const int64_t nb = a.ne0 / 32;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nblocks = nb * a.ne1 * a.ne2 * a.ne3;
    if (t >= nblocks) return;
    int64_t r = t / nb;
    const int64_t ib = t - r * nb;
    const int64_t i1 = r % a.ne1; r /= a.ne1;
    const int64_t i2 = r % a.ne2;
    const int64_t i3 = r / a.ne2;
    const float *x = reinterpret_cast<const float *>(a.src + i1 * a.nb01 + i2 * a.nb02 + i3 * a.nb03) + ib * 32;
    uint8_t *y = a.dst + i1 * a.nb1 + i2 * a.nb2 + i3 * a.nb3 + ib * QT<T>::bytes;
    float v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = x[j];
    if constexpr (T == T_Q4_0) {
        float amax = 0.f, mx = 0.f;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if (amax < fabsf(v[j])) { amax = fabsf(v[j]); mx = v[j]; }
        }
        // max / -8 is an exact power-of-two scaling: -(max * 0.125) rounds identically and keeps
        // the -0.0 an all-zero block gets from the reference (d = 0.0f / -8)
        const float d = -__fmul_rn(mx, 0.125f);
        const float id = d != 0.f ? __fdiv_rn(1.f, d) : 0.f;
        const uint16_t dh = f2h_rne(d);
        y[0] = (uint8_t)(dh & 0xff);
        y[1] = (uint8_t)(dh >> 8);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int xi0 = min(15, (int)(int8_t)(int)__fadd_rn(__fmul_rn(v[j], id), 8.5f));
            const int xi1 = min(15, (int)(int8_t)(int)__fadd_rn(__fmul_rn(v[16 + j], id), 8.5f));
            y[2 + j] = (uint8_t)(xi0 | (xi1 << 4));
        }
    } else {
        float amax = 0.f;
#pragma unroll
        for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(v[j]));
        const float d = __fdiv_rn(amax, 127.f);
        const float id = d != 0.f ? __fdiv_rn(1.f, d) : 0.f;
        const uint16_t dh = f2h_rne(d);
        y[0] = (uint8_t)(dh & 0xff);
        y[1] = (uint8_t)(dh >> 8);
#pragma unroll
        for (int j = 0; j < 32; ++j) y[2 + j] = (uint8_t)(int8_t)roundf(__fmul_rn(v[j], id));
    }
}

hipError_t quantize_launch(int type, const QuantArgs &a, hipStream_t st) {
    const int64_t n = a.ne0 / 32 * a.ne1 * a.ne2 * a.ne3;
    const dim3 grid((unsigned)((n + 255) / 256));
    switch (type) {
        case T_Q4_0: hipLaunchKernelGGL(quantize_kernel<T_Q4_0>, grid, dim3(256), 0, st, a); break;
        case T_Q8_0: hipLaunchKernelGGL(quantize_kernel<T_Q8_0>, grid, dim3(256), 0, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// GGML_OP_CPY out of a quantized tensor (the reference GPU path is cpy_q_f32,
// src/ggml-cuda/cpy.cu:94, dispatched at :362-366; the CPU one is dup_q, ops.cpp:1105-1154).
//   hot -> f32: element i of src (row-major over ne00..ne02) is dequantized bit-exactly, as
//     dequantize_row_* would, and lands at dup_q's position: the dst offset of the first element
//     of its 32/256-block (i10..i13 from the block start over ne0..ne2) plus 4 * (i % blck).
//     One thread per element, 4-byte coalesced stores; a grid-stride loop covers any count.
//   hot -> same hot: whole blocks are moved (dup_bytes, ops.cpp:956-1103), block b of src in
//     row-major block order to block b of dst; one thread per block in 2-byte units (every block
//     size here is even and ggml block rows are 2-byte aligned).
// ------------------------------------------------------------------------------------------
struct CpyQArgs {
    const uint8_t *src; int64_t ne00, ne01, ne02; int64_t nb00, nb01, nb02, nb03;
    uint8_t *dst; int64_t ne0, ne1, ne2; int64_t nb0, nb1, nb2, nb3;
    int64_t n;    // elements (to f32) or blocks (same type)
};

template <int T>
__global__ __launch_bounds__(256) void cpy_q_f32_kernel(const CpyQArgs a) {
    constexpr int QK = QT<T>::blck;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += stride) {
        const int64_t j = i % QK;
        const int64_t b0 = i - j;                               // first element of the block
        int64_t r = b0;
        const int64_t i00 = r % a.ne00; r /= a.ne00;
        const int64_t i01 = r % a.ne01; r /= a.ne01;
        const int64_t i02 = r % a.ne02;
        const int64_t i03 = r / a.ne02;
        const uint8_t *blk = a.src + (i00 / QK) * a.nb00 + i01 * a.nb01 + i02 * a.nb02 + i03 * a.nb03;
        r = b0;
        const int64_t i10 = r % a.ne0; r /= a.ne0;
        const int64_t i11 = r % a.ne1; r /= a.ne1;
        const int64_t i12 = r % a.ne2;
        const int64_t i13 = r / a.ne2;
        float *d = reinterpret_cast<float *>(a.dst + i10 * a.nb0 + i11 * a.nb1 + i12 * a.nb2 + i13 * a.nb3);
        d[j] = deq_one<T>(blk, (int)j);
    }
}

template <int T>
__global__ __launch_bounds__(256) void cpy_q_q_kernel(const CpyQArgs a) {
    constexpr int QK = QT<T>::blck, HW = QT<T>::bytes / 2;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < a.n; b += stride) {
        const int64_t nbr0 = a.ne00 / QK, nbr1 = a.ne0 / QK;   // blocks per row
        int64_t r = b;
        const int64_t i00 = r % nbr0; r /= nbr0;
        const int64_t i01 = r % a.ne01; r /= a.ne01;
        const int64_t i02 = r % a.ne02;
        const int64_t i03 = r / a.ne02;
        const uint16_t *s = reinterpret_cast<const uint16_t *>(a.src + i00 * a.nb00 + i01 * a.nb01 + i02 * a.nb02 + i03 * a.nb03);
        r = b;
        const int64_t i10 = r % nbr1; r /= nbr1;
        const int64_t i11 = r % a.ne1; r /= a.ne1;
        const int64_t i12 = r % a.ne2;
        const int64_t i13 = r / a.ne2;
        uint16_t *d = reinterpret_cast<uint16_t *>(a.dst + i10 * a.nb0 + i11 * a.nb1 + i12 * a.nb2 + i13 * a.nb3);
#pragma unroll 8
        for (int k = 0; k < HW; ++k) d[k] = s[k];
    }
}

template <int T>
static void cpy_q_one(bool to_f32, const CpyQArgs &a, hipStream_t st) {
    const int64_t want = (a.n + 255) / 256;
    const dim3 grid((unsigned)(want < 65536 * 16 ? want : 65536 * 16));
    if (to_f32) hipLaunchKernelGGL(cpy_q_f32_kernel<T>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(cpy_q_q_kernel<T>, grid, dim3(256), 0, st, a);
}

hipError_t cpy_q_launch(int type, bool to_f32, const CpyQArgs &a, hipStream_t st) {
    if (a.n <= 0) return hipSuccess;
    switch (type) {
        case T_Q4_0: cpy_q_one<T_Q4_0>(to_f32, a, st); break;
        case T_Q8_0: cpy_q_one<T_Q8_0>(to_f32, a, st); break;
        case T_Q4_K: cpy_q_one<T_Q4_K>(to_f32, a, st); break;
        case T_Q5_K: cpy_q_one<T_Q5_K>(to_f32, a, st); break;
        case T_Q6_K: cpy_q_one<T_Q6_K>(to_f32, a, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace mi355x
