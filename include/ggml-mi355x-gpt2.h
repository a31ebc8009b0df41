/*
 * ggml-mi355x-gpt2.h — C-ABI of the MI355X GPT-2 decode engine (libggml-hip-mi355x.so).
 *
 * The reference runs GPT-2 as a ggml graph (examples/gpt-2/main-sched.cpp) whose nodes a
 * backend executes one by one. This engine is the same model run natively on gfx950: the
 * reference's per-layer node chain is collapsed into five launches (fused mat-vecs carrying the
 * layer norms, biases, GELU and residual adds, plus one attention kernel), one decode step is a
 * replayable hipGraph, and positions / next tokens stay in device memory.
 *
 * Pipeline parallelism: a model object holds ONE STAGE, the layer range
 * [layer_begin, layer_end) of one process / GPU. The first stage also owns the embeddings
 * (wte, wpe), the last stage ln_f and lm_head. The host moves each stage's hidden state
 * (n_seq x n_embd f32, see ggml_mi355x_gpt2_ctx_buffers) to the next stage — over RCCL
 * send/recv in ggml-gfx906_amd/gpt2.py — the role ggml_backend_sched's cpy_tensor_async plays
 * between the reference's backends (src/ggml-backend.cpp:1383).
 *
 * Conventions: 0 = success, negative = ggml_mi355x_status (ggml-mi355x.h). Device memory is
 * allocated on the HIP device current at *_init time; every call must run with that device
 * current. `stream` is a hipStream_t (NULL = default stream).
 */
#ifndef GGML_MI355X_GPT2_H
#define GGML_MI355X_GPT2_H

#include <stdint.h>

#include "ggml-mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

/* gpt2_hparams (reference examples/gpt-2/main-sched.cpp:44-52); ftype with the quantization
 * version already stripped (ftype % GGML_QNT_VERSION_FACTOR, :196-199). */
typedef struct {
    int32_t n_vocab, n_ctx, n_embd, n_head, n_layer, ftype;
} ggml_mi355x_gpt2_hparams;

typedef struct ggml_mi355x_gpt2_model ggml_mi355x_gpt2_model;
typedef struct ggml_mi355x_gpt2_ctx ggml_mi355x_gpt2_ctx;

/* Read the header of a legacy ggml GPT-2 file (magic 0x67676d6c, hparams, vocab;
 * gpt2_model_load, main-sched.cpp:155-223). Host only. -1 = not a GPT-2 ggml file. */
GGML_MI355X_API int ggml_mi355x_gpt2_read_hparams(const char *fname, ggml_mi355x_gpt2_hparams *hp);

/* Allocate one pipeline stage's weights on the current device, layers [layer_begin,
 * layer_end) (the reference's per-layer backend placement, main-sched.cpp:300-340). Weight
 * matrices have type ggml_ftype_to_ggml_type(hp->ftype): Q4_0, Q8_0, Q4_K, Q5_K or Q6_K
 * (f32 also accepted); head dimension n_embd / n_head must be 64. Contents are undefined
 * until loaded or filled through ggml_mi355x_gpt2_model_tensor. */
GGML_MI355X_API int ggml_mi355x_gpt2_model_init(const ggml_mi355x_gpt2_hparams *hp, int32_t layer_begin, int32_t layer_end,
                                                ggml_mi355x_gpt2_model **out);

/* Upload this stage's tensors from a legacy ggml GPT-2 file, enforcing the reference loader's
 * checks (known names, element counts, shapes, byte sizes; main-sched.cpp:429-517) and its
 * tied-embedding rule (lm_head := wte when the file has no model/lm_head, :503-510). */
GGML_MI355X_API int ggml_mi355x_gpt2_model_load(ggml_mi355x_gpt2_model *model, const char *fname);

/* Device pointer, ggml type and shape of a tensor of this stage by its legacy name
 * ("model/wte", "model/h3/mlp/c_fc/w", ... main-sched.cpp:256-297). -1 = not in this stage. */
GGML_MI355X_API int ggml_mi355x_gpt2_model_tensor(ggml_mi355x_gpt2_model *model, const char *name, void **data, int32_t *type,
                                                  int64_t ne[2]);

/* Bytes of device memory held by the stage's weights. */
GGML_MI355X_API int64_t ggml_mi355x_gpt2_model_bytes(const ggml_mi355x_gpt2_model *model);

GGML_MI355X_API void ggml_mi355x_gpt2_model_free(ggml_mi355x_gpt2_model *model);

/* A decode context: n_seq independent sequences (1..64) decoded together, with their KV cache
 * for this stage's layers ([layer][seq][n_ctx][n_embd] f32 K and V, the reference's
 * memory_k / memory_v, main-sched.cpp:384-420), positions and activation buffers.
 * For Q4_0 / Q8_0 stages on the two-launch layer, ctx_init also (re)makes the model's one shared
 * set of head-/slice-major c_proj and MLP-projection copies from the current weights: weights
 * written through ggml_mi355x_gpt2_model_tensor after a context exists reach decoding once a
 * context is created after the write (every context of the model then reads the new copies).
 * ctx_init waits for the device to drain before rewriting them; it must not run concurrently with
 * decode calls on the same model from another thread. */
GGML_MI355X_API int ggml_mi355x_gpt2_ctx_init(ggml_mi355x_gpt2_model *model, int32_t n_seq, ggml_mi355x_gpt2_ctx **out);

/* Device buffers of the context:
 *   tokens [n_seq] i32  : input token per sequence (first stage); the last stage writes the
 *                         greedy next token here at the end of each step
 *   pos    [n_seq] i32  : position of the token being decoded (= n_past), advanced by each step
 *   hidden [n_seq][n_embd] f32 : the residual stream — the stage's output, and the input of a
 *                         non-first stage
 *   logits [n_seq][n_vocab] f32 : last stage only (NULL otherwise) */
GGML_MI355X_API int ggml_mi355x_gpt2_ctx_buffers(ggml_mi355x_gpt2_ctx *ctx, int32_t **tokens, int32_t **pos, float **hidden,
                                                 float **logits);

/* One decode step of this stage for all n_seq sequences: [embed] -> layers -> [ln_f, lm_head,
 * argmax] -> pos += 1 (gpt2_eval with N = 1, main-sched.cpp:867-905, plus greedy sampling).
 * use_graph != 0 captures the step into a hipGraph on the first call for `stream` and replays
 * it afterwards (every step reads its position from device memory). Asynchronous. Positions
 * must stay below n_ctx (the kernels clamp; the caller checks). */
GGML_MI355X_API int ggml_mi355x_gpt2_decode(ggml_mi355x_gpt2_ctx *ctx, void *stream, int32_t use_graph);

GGML_MI355X_API void ggml_mi355x_gpt2_ctx_free(ggml_mi355x_gpt2_ctx *ctx);

/* Stream-ordered copy between any two of host / this device / a peer device (unified
 * addressing; hipMemcpyAsync with hipMemcpyDefault). Used by the host driver to move token
 * ids, positions and stage activations in and out of a context's buffers. */
GGML_MI355X_API int ggml_mi355x_memcpy(void *dst, const void *src, size_t bytes, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* GGML_MI355X_GPT2_H */
