/*
 * oracle/qref.h — CPU restatement of the reference's quantized MUL_MAT path.
 *
 * TEST INFRASTRUCTURE ONLY. This is the parity checker ("oracle") for the MI355X backend:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The
 * product (libggml-hip-mi355x.so) never links or calls it.
 *
 * Every function restates the algorithm of the upstream ggml CPU path (file:line cited
 * next to each definition in qref.c). Parity of this restatement is PINNED against the real
 * reference: tests/golden/ holds vectors produced by oracle/gen_golden.cpp linked against
 * the reference sources compiled in place (oracle/ref.mk), and tests/test_oracle_golden.py
 * checks this library against them bit-for-bit (quantize / dequantize / activation
 * quantization / generic vec_dot) and within tolerance (mul_mat vs the SIMD CPU backend).
 *
 * Type ids are ggml's (include/ggml.h:372-412 of the reference).
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    QREF_F32  = 0,
    QREF_F16  = 1,
    QREF_Q4_0 = 2,
    QREF_Q8_0 = 8,
    QREF_Q8_1 = 9,
    QREF_Q4_K = 12,
    QREF_Q5_K = 13,
    QREF_Q6_K = 14,
    QREF_Q8_K = 15,
    QREF_I32  = 26,
};

/* activation-quantizer flavour used for src1 (ggml-cpu quantizes src1 to the vec_dot type) */
enum {
    QREF_ACT_REF  = 0, /* quantize_row_q8_0_ref: d = amax/127, q = roundf(x * (1/d))          */
    QREF_ACT_X86  = 1, /* arch/x86 AVX2 quantize_row_q8_0: q = rint(x * (127/amax))            */
};

int64_t qref_blck_size(int type);
size_t  qref_type_size(int type);
size_t  qref_row_size(int type, int64_t ne);
int     qref_vec_dot_type(int type);

uint16_t qref_fp32_to_fp16(float f);
float    qref_fp16_to_fp32(uint16_t h);

/* deterministic portable input generator (splitmix64 counter mode); identical in numpy */
void qref_fill_uniform(float *dst, int64_t n, uint64_t seed, float lo, float hi);

/* weight quantization: mirrors ggml_quantize_chunk(type, src, dst, start, nrows, n_per_row, imatrix) */
size_t qref_quantize_chunk(int type, const float *src, void *dst, int64_t start, int64_t nrows,
                           int64_t n_per_row, const float *imatrix);
/* `_ref` quantizer of one contiguous run of k values */
void   qref_quantize_row_ref(int type, const float *x, void *y, int64_t k);
void   qref_dequantize_row(int type, const void *x, float *y, int64_t k);

/* activation quantization to Q8_0 / Q8_K / Q8_1 */
void   qref_quantize_act(int type, const float *x, void *y, int64_t k, int flavour);

/* generic-order block dot of n values: weights `x` of `type`, activations `y` of vec_dot_type */
float  qref_vec_dot(int type, int n, const void *x, const void *y);

/* ggml-shaped view of a tensor: ne = elements per dim, nb = byte strides */
typedef struct {
    int      type;
    void    *data;
    int64_t  ne[4];
    size_t   nb[4];
} qref_tensor;

/* dst = mul_mat(src0, src1) with ggml semantics (broadcast over dims 2/3, strided views).
 * src0 quantized (or f32), src1 f32, dst f32. n_threads <= 0 selects all cores. */
int qref_mul_mat(const qref_tensor *src0, const qref_tensor *src1, qref_tensor *dst,
                 int act_flavour, int n_threads);

/* dst = mul_mat_id(as, b, ids): as [K,N,n_expert], b [K, n_used|1, T], ids i32 [n_used, T] */
int qref_mul_mat_id(const qref_tensor *as, const qref_tensor *b, const qref_tensor *ids,
                    qref_tensor *dst, int act_flavour, int n_threads);

#ifdef __cplusplus
}
#endif
