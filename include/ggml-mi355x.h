/*
 * ggml-mi355x.h — C-ABI boundary of the MI355X (gfx950) quantized MUL_MAT backend.
 *
 * One shared library, libggml-hip-mi355x.so, exports two layers:
 *
 *  1. The ggml dynamic-backend entry points. These are exactly what the reference's loader
 *     binds (src/ggml-backend-reg.cpp:239-283 dlsym()s "ggml_backend_score" and
 *     "ggml_backend_init" and checks api_version == 1), so the library is a drop-in for
 *     upstream test-backend-ops / examples via GGML_BACKEND_PATH or ggml_backend_load().
 *     The returned registry fills the vtables of src/ggml-backend-impl.h:17-207
 *     (buffer type, buffer, backend/stream, device, reg) — see INTEGRATION.md.
 *
 *  2. A direct kernel API on device pointers, for hosts without ggml (the repo's harness and
 *     bench on the GPU box). It takes ggml tensor geometry verbatim and runs the same
 *     dispatch as graph_compute does for GGML_OP_MUL_MAT / GGML_OP_MUL_MAT_ID.
 *
 * No torch or HIP types cross this boundary: plain pointers, sizes and an opaque stream.
 */
#ifndef GGML_MI355X_H
#define GGML_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GGML_MI355X_API __attribute__((visibility("default")))

/* ---- 1. ggml dynamic-backend boundary -------------------------------------------------- */

struct ggml_backend_reg;

/* Replaces GGML_BACKEND_DL_IMPL(ggml_backend_cuda_reg) (reference src/ggml-cuda/ggml-cuda.cu:3819,
 * macro src/ggml-backend-impl.h:220-251). Returns a registry with api_version == 1. */
GGML_MI355X_API struct ggml_backend_reg *ggml_backend_init(void);

/* Replaces GGML_BACKEND_DL_SCORE_IMPL: 0 = no usable gfx950 device (loader skips the library,
 * src/ggml-backend-reg.cpp:248-254), otherwise a positive score. */
GGML_MI355X_API int ggml_backend_score(void);

/* Replaces ggml_backend_cuda_reg() (reference include/ggml-cuda.h) for static linking. */
GGML_MI355X_API struct ggml_backend_reg *ggml_backend_mi355x_reg(void);

/* ---- 2. direct kernel API ---------------------------------------------------------------- */

/* ggml type ids used here (reference include/ggml.h:372-412) */
enum ggml_mi355x_type {
    GGML_MI355X_F32  = 0,
    GGML_MI355X_Q4_0 = 2,
    GGML_MI355X_Q8_0 = 8,
    GGML_MI355X_Q4_K = 12,
    GGML_MI355X_Q5_K = 13,
    GGML_MI355X_Q6_K = 14,
    GGML_MI355X_I32  = 26,
};

/* error codes (0 = success) */
enum ggml_mi355x_status {
    GGML_MI355X_OK          = 0,
    GGML_MI355X_EINVAL      = -1, /* unsupported type or inconsistent shapes / strides        */
    GGML_MI355X_ENOMEM      = -2, /* scratch allocation failed                                */
    GGML_MI355X_EHIP        = -3, /* a HIP runtime call or kernel launch failed               */
    GGML_MI355X_ENODEV      = -4, /* no gfx950 device                                         */
};

/* A ggml tensor view on device memory: ne = elements per dim, nb = byte strides
 * (same meaning as struct ggml_tensor ne/nb, reference include/ggml.h:614-646). */
typedef struct {
    int32_t type;
    void   *data;
    int64_t ne[4];
    size_t  nb[4];
} ggml_mi355x_tensor;

/* dst = src0 x src1 with GGML_OP_MUL_MAT semantics (ggml_mul_mat, reference src/ggml.c:3015-3031;
 * CPU definition src/ggml-cpu/ggml-cpu.c:1202-1394): src0 quantized (Q4_0/Q8_0/Q4_K/Q5_K/Q6_K),
 * src1 and dst f32; broadcast of src0 over dims 2/3; strided src0/src1 rows (permutes/views).
 * Replaces ggml_cuda_mul_mat (src/ggml-cuda/ggml-cuda.cu:2007-2090). `stream` is a hipStream_t
 * (NULL = default stream); the call is asynchronous with respect to the host. */
GGML_MI355X_API int ggml_mi355x_mul_mat(const ggml_mi355x_tensor *src0, const ggml_mi355x_tensor *src1,
                                        ggml_mi355x_tensor *dst, void *stream);

/* dst = mul_mat_id(as, b, ids) with GGML_OP_MUL_MAT_ID semantics (reference src/ggml.c:3043-3081,
 * src/ggml-cpu/ggml-cpu.c:1476-1655): as [K,N,n_expert], b [K, n_used|1, T] f32,
 * ids [n_used, T] i32, dst [N, n_used, T] f32. Replaces ggml_cuda_mul_mat_id
 * (src/ggml-cuda/ggml-cuda.cu:2092-2230). Expert ids must be in [0, n_expert). */
GGML_MI355X_API int ggml_mi355x_mul_mat_id(const ggml_mi355x_tensor *as, const ggml_mi355x_tensor *b,
                                           const ggml_mi355x_tensor *ids, ggml_mi355x_tensor *dst, void *stream);

/* dst[k] = dequantize_row_<type>(src, k) on the device, bit-exact with the reference's
 * dequantize_row_* (src/ggml-quants.c:307, 401, 1352, 1554, 1762); replaces the
 * dequantize_block_* kernels of src/ggml-cuda/convert.cu:82-266. n = number of values,
 * a multiple of the block size. */
GGML_MI355X_API int ggml_mi355x_dequantize(int32_t type, const void *src, float *dst, int64_t n, void *stream);

/* dst = get_rows(src0, rows) with GGML_OP_GET_ROWS semantics (ggml_get_rows, reference
 * src/ggml.c:3617-3637; CPU src/ggml-cpu/ops.cpp:5121-5163): src0 [ne00, ne01, ne02, ne03] of a
 * hot quant type or f32, rows [r, ne02, ne03] i32, dst [ne00, r, ne02, ne03] f32, each row the
 * bit-exact dequantize_row_* of the selected src0 row. Replaces get_rows_cuda
 * (src/ggml-cuda/getrows.cu). An index outside [0, ne01) (the reference GGML_ASSERTs,
 * src/ggml-cpu/ops.cpp:5157) writes nothing for that row and raises the device error word that
 * ggml_mi355x_device_error() returns once the stream has synchronized. */
GGML_MI355X_API int ggml_mi355x_get_rows(const ggml_mi355x_tensor *src0, const ggml_mi355x_tensor *rows,
                                         ggml_mi355x_tensor *dst, void *stream);

/* Returns and clears the device error word (nonzero: a kernel met a precondition the reference
 * asserts on, e.g. a GET_ROWS index out of range). Call after the stream synchronized. */
GGML_MI355X_API int ggml_mi355x_device_error(void);

/* dst = src with GGML_OP_CPY semantics (ggml_cpy, reference src/ggml.c; CPU dup_q
 * src/ggml-cpu/ops.cpp:1105-1154 and dup_bytes :956-1103) between this path's types:
 *   f32 -> Q4_0 / Q8_0     as ggml_mi355x_quantize (same shapes);
 *   Q4_0/Q8_0/Q4_K/Q5_K/Q6_K -> f32   bit-exact dequantize_row_* of every block, placed where
 *                          dup_q places it (same element count; dst rows hold whole blocks or
 *                          dst is contiguous);
 *   hot type -> same type  block copy (same element count, whole blocks per row).
 * Replaces ggml_cpy_q4_0_f32_cuda / ggml_cpy_q8_0_f32_cuda (src/ggml-cuda/cpy.cu:94, :362-366). */
GGML_MI355X_API int ggml_mi355x_cpy(const ggml_mi355x_tensor *src, ggml_mi355x_tensor *dst, void *stream);

/* dst = src converted f32 -> Q4_0 or Q8_0 (GGML_OP_CPY into a quantized tensor), bit-exact with
 * quantize_row_q4_0_ref / quantize_row_q8_0_ref (reference src/ggml-quants.c:36-71, 199-222).
 * Same shapes, strided 4-d views with contiguous rows; ne0 a multiple of 32. Replaces
 * ggml_cpy_f32_q4_0_cuda / ggml_cpy_f32_q8_0_cuda (src/ggml-cuda/cpy.cu). */
GGML_MI355X_API int ggml_mi355x_quantize(const ggml_mi355x_tensor *src, ggml_mi355x_tensor *dst, void *stream);

/* Repacked weights for the int8 mat-mat tile (the reference's analogue is the CPU
 * backend's repack extra buffer type, src/ggml-cpu/repack.cpp:1967): the quantized codes of src0 as
 * int8 in MFMA-fragment order plus f32 block scales, made once (e.g. at weight upload) so that
 * MUL_MAT with many tokens streams them with no per-call decode. ggml_mi355x_repack_size gives the
 * bytes for src0 (every matrix of a 3-d / 4-d tensor), ggml_mi355x_repack writes them to `dst`
 * (device memory) on `stream`; ggml_mi355x_mul_mat_repacked is ggml_mi355x_mul_mat with that copy
 * beside src0 (src0 itself still serves the mat-vec shapes, ne11 <= 8, and the shapes where
 * the in-place tile's 128-token tiles are faster than the copy's 64-token ones). The copy must
 * be remade when src0's bytes change. */
GGML_MI355X_API int ggml_mi355x_repack_size(const ggml_mi355x_tensor *src0, size_t *bytes);
GGML_MI355X_API int ggml_mi355x_repack(const ggml_mi355x_tensor *src0, void *dst, size_t bytes, void *stream);
GGML_MI355X_API int ggml_mi355x_mul_mat_repacked(const ggml_mi355x_tensor *src0, const void *repacked,
                                                 const ggml_mi355x_tensor *src1, ggml_mi355x_tensor *dst, void *stream);

/* Same predicate the backend's supports_op uses for MUL_MAT / MUL_MAT_ID on these operands
 * (replaces the MUL_MAT arm of ggml_backend_cuda_device_supports_op, ggml-cuda.cu:3270-3330). */
GGML_MI355X_API int ggml_mi355x_supports_mul_mat(const ggml_mi355x_tensor *src0, const ggml_mi355x_tensor *src1);

/* Same predicate the backend's supports_op uses for MUL_MAT_ID (the MUL_MAT_ID arm of
 * ggml_backend_cuda_device_supports_op, ggml-cuda.cu:3270-3330): as [K,N,n_expert], b, ids as for
 * ggml_mi355x_mul_mat_id; true exactly when ggml_mi355x_mul_mat_id accepts the geometry. */
GGML_MI355X_API int ggml_mi355x_supports_mul_mat_id(const ggml_mi355x_tensor *as, const ggml_mi355x_tensor *b,
                                                    const ggml_mi355x_tensor *ids);

/* The kernel launches ggml_mi355x_mul_mat (repacked != 0: ggml_mi355x_mul_mat_repacked) would make
 * for these operands, as text into buf (e.g. "mmvq nc=1 lpr=64 rpw=1 grid=512x1x1", "mma tok=8 ...",
 * "mmq8 tile=128x64 ..."). Launches nothing and touches no device memory (data pointers are only
 * checked for alignment), so it runs without a GPU: tests pin the dispatch of the benchmark and
 * reference-perf shapes with it. No reference counterpart (the CUDA backend's choice is internal). */
GGML_MI355X_API int ggml_mi355x_mul_mat_plan(const ggml_mi355x_tensor *src0, const ggml_mi355x_tensor *src1, int repacked,
                                             char *buf, size_t len);

/* Re-read the GGML_MI355X_* tuning and diagnostics variables (read once otherwise):
 * tests and benches that switch one between calls call this after changing the environment. */
GGML_MI355X_API int ggml_mi355x_reload_settings(void);

/* number of gfx950 devices visible to this process */
GGML_MI355X_API int ggml_mi355x_device_count(void);

/* short text for a status code */
GGML_MI355X_API const char *ggml_mi355x_strerror(int status);

#ifdef __cplusplus
}
#endif

#endif /* GGML_MI355X_H */
