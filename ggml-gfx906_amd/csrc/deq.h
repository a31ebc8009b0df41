// deq.h — per-element dequantization, bit-exact with the reference's dequantize_row_*
// (src/ggml-quants.c:307-323, 401-415, 1352-1374, 1554-1579, 1762-1791): explicitly rounded
// IEEE ops (__fmul_rn / __fsub_rn), never a contracted FMA. Shared by dequant.hip (DEQUANTIZE,
// GET_ROWS) and gpt2_ops.hip (token embedding rows).
#pragma once
#include "qcommon.h"

namespace mi355x {

template <int T>
__device__ inline float deq_one(const uint8_t *blk, int i);

template <> __device__ inline float deq_one<T_Q4_0>(const uint8_t *b, int i) {
    const float d = h2f(ld2(b));
    const int q = i < 16 ? (b[2 + i] & 0x0f) - 8 : (b[2 + i - 16] >> 4) - 8;
    return __fmul_rn((float)q, d);
}

template <> __device__ inline float deq_one<T_Q8_0>(const uint8_t *b, int i) {
    return __fmul_rn((float)(int8_t)b[2 + i], h2f(ld2(b)));
}

__device__ inline void scale_min_k4(int j, const uint8_t *q, int &d, int &m) {
    if (j < 4) {
        d = q[j] & 63;
        m = q[j + 4] & 63;
    } else {
        d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
    }
}

template <> __device__ inline float deq_one<T_Q4_K>(const uint8_t *b, int i) {
    const int c = i >> 6, r = i & 63, hi = r >> 5, l = r & 31;
    int sc, m;
    scale_min_k4(2 * c + hi, b + 4, sc, m);
    const float d1 = __fmul_rn(h2f(ld2(b)), (float)sc);
    const float m1 = __fmul_rn(h2f(ld2(b + 2)), (float)m);
    const uint8_t qb = b[16 + 32 * c + l];
    const int q = hi ? (qb >> 4) : (qb & 0xF);
    return __fsub_rn(__fmul_rn(d1, (float)q), m1);
}

template <> __device__ inline float deq_one<T_Q5_K>(const uint8_t *b, int i) {
    const int c = i >> 6, r = i & 63, hi = r >> 5, l = r & 31;
    int sc, m;
    scale_min_k4(2 * c + hi, b + 4, sc, m);
    const float d1 = __fmul_rn(h2f(ld2(b)), (float)sc);
    const float m1 = __fmul_rn(h2f(ld2(b + 2)), (float)m);
    const uint8_t qb = b[48 + 32 * c + l];
    const int bit = (b[16 + l] >> (2 * c + hi)) & 1;
    const int q = (hi ? (qb >> 4) : (qb & 0xF)) + (bit ? 16 : 0);
    return __fsub_rn(__fmul_rn(d1, (float)q), m1);
}

template <> __device__ inline float deq_one<T_Q6_K>(const uint8_t *b, int i) {
    const int h = i >> 7, r = i & 127, k = r >> 5, l = r & 31;
    const uint8_t *ql = b + 64 * h, *qh = b + 128 + 32 * h;
    const int8_t *sc = reinterpret_cast<const int8_t *>(b + 192) + 8 * h;
    const int lo = (k & 1) ? ql[l + 32] : ql[l];
    const int nib = (k >> 1) ? (lo >> 4) : (lo & 0xF);
    const int q = (int)(int8_t)(nib | (((qh[l] >> (2 * k)) & 3) << 4)) - 32;
    const float d = h2f(ld2(b + 208));
    return __fmul_rn(__fmul_rn(d, (float)sc[l / 16 + 2 * k]), (float)q);
}

}  // namespace mi355x
