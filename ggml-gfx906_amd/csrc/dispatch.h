// dispatch.h — internal host interface between the ggml backend glue (backend.cpp), the
// direct C API and the kernel launchers.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <mutex>

#include "qmm_args.h"

namespace mi355x {

struct TensorView {
    int type;
    void *data;
    int64_t ne[4];
    size_t nb[4];
};

// grow-only device scratch owned by ONE (device, stream) pair: only work queued on that stream
// touches it, so growing it (synchronize that stream, free, allocate) never races another
// stream. Growing is refused (nullptr, the launch then fails with GGML_MI355X_ENOMEM) while the
// stream is being captured into a hipGraph: hipFree / hipMalloc are not capturable, so a
// captured launch must have been run once eagerly on the same stream first.
//
// Several host threads may share one stream (torch's default stream is handle 0 on every
// thread, and ctypes releases the GIL during a call), so mul_mat / mul_mat_id hold `mu` from
// get() until every kernel that uses the buffer is queued: a second thread that must grow the
// buffer then synchronizes the stream behind those kernels before it frees the old one.
//
// `gen` counts reallocations: a hipGraph captured while the buffer had generation g holds its
// address, so the graph may be replayed only while gen is still g (backend.cpp checks it).
struct Scratch {
    std::mutex mu;
    void *ptr = nullptr;
    size_t cap = 0;
    int device = -1;
    uint64_t gen = 0;
    // set when get() had to refuse a larger buffer inside a stream capture. Some users then take
    // a slower path that needs no scratch (the mat-vec's pre-quantized forms), so the capture
    // itself succeeds; the backend checks this flag and runs eagerly instead (which grows the
    // buffer), so the graph it captures next holds the fast path
    bool short_in_capture = false;
    void *get(size_t bytes, hipStream_t st);
    // stream-K tile counters (mmq8.hip): a separate zeroed allocation of COUNTERS ints, made once
    // (outside any capture) and never moved; every launch leaves them zero
    static constexpr int COUNTERS = 16384;
    int *cnt = nullptr;
    int *counters(hipStream_t st);
    void release();                   // free now (on the current device)
    ~Scratch();
};

// the process-wide scratch of (current device, st) for callers without a backend object
Scratch &scratch_for(hipStream_t st);

int type_blck(int t);
int type_bytes(int t);
bool is_hot_quant(int t);

// repacked weights for the int8 mat-mat tile (mmq8.hip): int8 codes in MFMA-fragment order +
// f32 block scales (+ K-quant mins), laid out per matrix by rp_layout
struct RpLayout {
    int n_rt, n_sb;          // 32-row tiles, super-blocks per row
    size_t off_meta, bytes;
};
struct RpSrcView {           // a ggml weight tensor: n_mat = ne02 * ne03 matrices of N rows x K
    const void *w;
    int64_t nb01, nb02, nb03;
    int K, N, ne02, n_mat;
};
RpLayout rp_layout(int type, int K, int N, int n_mat);
bool repack_supported(int type, const RpSrcView &s);
hipError_t repack_launch(int type, const RpSrcView &s, void *dst, hipStream_t st);
int repack(const TensorView &w, void *dst, size_t bytes, hipStream_t st);
size_t repack_size(const TensorView &w);
// MUL_MAT with src0 also available repacked at `rp` (nullptr: plain mul_mat)
int mul_mat_rp(const TensorView &a, const void *rp, const TensorView &b, const TensorView &d, hipStream_t st,
               Scratch &scratch);

int check_mul_mat(const TensorView &a, const TensorView &b, const TensorView &d);
int check_mul_mat_id(const TensorView &as, const TensorView &b, const TensorView &ids, const TensorView &d);

int mul_mat(const TensorView &a, const TensorView &b, const TensorView &d, hipStream_t st, Scratch &scratch);
int mul_mat_id(const TensorView &as, const TensorView &b, const TensorView &ids, const TensorView &d, hipStream_t st,
               Scratch &scratch);
int dequantize(int type, const void *src, float *dst, int64_t n, hipStream_t st);
int check_get_rows(const TensorView &a, const TensorView &rows, const TensorView &d);
int get_rows(const TensorView &a, const TensorView &rows, const TensorView &d, hipStream_t st);
int get_rows_add(const TensorView &a, const TensorView &ra, const TensorView &b, const TensorView &rb, const TensorView &d,
                 hipStream_t st);
// device error word (host-mapped): raised by kernels on a failed device-side precondition;
// take_device_error() returns and clears it (call after the stream synchronized)
int *device_error_word();
int take_device_error(int device);   // device < 0: all devices
int check_quantize(const TensorView &src, const TensorView &d);
// GGML_OP_CPY between this path's types: f32 -> Q4_0 / Q8_0, hot -> f32, hot -> same hot
int check_cpy(const TensorView &src, const TensorView &d);
int cpy(const TensorView &src, const TensorView &d, hipStream_t st);
int quantize(const TensorView &src, const TensorView &d, hipStream_t st);

// the f32 graph ops around the matmuls (graph_ops.hip)
enum GraphOpKind {
    GOP_ADD, GOP_SUB, GOP_MUL, GOP_DIV, GOP_NORM, GOP_SCALE, GOP_DIAG_MASK_INF, GOP_DIAG_MASK_ZERO,
    GOP_SOFT_MAX, GOP_GELU, GOP_CPY, GOP_MUL_MAT,
};
struct GraphOp {
    int op;                 // GraphOpKind
    int32_t params[4];      // the node's op_params[0..3] (eps, scale/bias, n_past, ...)
    TensorView dst;
    TensorView src[3];
    bool has_src[3];
};
int check_graph_op(const GraphOp &g);
int run_graph_op(const GraphOp &g, hipStream_t st);
// fused producers of a SOFT_MAX (backend graph fusion of SCALE -> DIAG_MASK_INF -> SOFT_MAX)
struct SoftmaxPre {
    float scale, bias;   // SCALE's op_params
    int n_past;          // DIAG_MASK_INF's n_past (-1: no mask node)
};
int run_graph_op_pre(const GraphOp &g, const SoftmaxPre *pre, hipStream_t st);
// two CPY nodes in one launch (same type pair and shape relation); independence is the caller's
bool cpy_pairable(const GraphOp &g0, const GraphOp &g1);
int run_cpy_pair(const GraphOp &g0, const GraphOp *g1, hipStream_t st);
int run_soft_max_pre(const GraphOp &g, const SoftmaxPre &pre, hipStream_t st);

// attention over strided views (backend graph fusion of MUL_MAT(K, Q) -> [SCALE] ->
// [DIAG_MASK_INF] -> SOFT_MAX -> MUL_MAT(V^T, .) [-> PERMUTE -> CONT]); byte strides, per
// (query i, head h): O[:, i, h] = sum_j softmax_j(w_j) V^T[j, :, hk], hk = h / (H / Hk),
// w_j = ((K[:, j, hk] . Q[:, i, h]) * pre_s (+ pre_b), -inf where j > n_past + i) * sm_scale
struct AttnView {
    const void *q;  int64_t q_d, q_i, q_h;              // f32
    const void *k;  int k_f16; int64_t k_d, k_j, k_h;   // f32 or f16
    const void *v;  int v_f16; int64_t v_j, v_d, v_h;   // f32 or f16 (V^T[j, d, hk])
    void *o;        int64_t o_d, o_i, o_h;              // f32
    int D, n_q, n_kv, H, Hk;
    float pre_s, pre_b, sm_scale;
    int n_past;                                         // -1: no causal mask
};
constexpr int ATTN_MAX_D = 256, ATTN_MAX_KV = 14336;   // scores of one row live in LDS
int run_attention(const AttnView &a, hipStream_t st);

// quantized mat-vec with the decode-layer fusions (mmvq_fused.hip): layer-norm prologue,
// bias / GELU / residual epilogue (MmArgs fields); nc columns per launch column group
hipError_t mmvq_fused_launch(int type, const MmArgs &a, int nc, int rpw, hipStream_t st);
hipError_t mmvq_fused_prepare(int type);
int mmvq_fused_pick_nc(int M, int K);

// the GPT-2 two-launch layer (gpt2_block.hip): used by the decode engine (gpt2.cpp) and by the
// plugin's graph fusion of whole GPT-2 layers (backend.cpp)
bool gpt2_block_supported(int n_embd, int n_head);
int gpt2_block_mlp_slices(int n_embd);
hipError_t gpt2_attn_block_launch(int layer, int type, const float *base, const float *bias_in, const float *parts_in, int n_parts_in,
                                  float *x_out, const float *ln_g, const float *ln_b, float eps, const uint8_t *w_qkv,
                                  int64_t nb_qkv, const float *b_qkv, float *kc, float *vc, const int32_t *pos, float scale,
                                  int n_ctx, const uint8_t *w_o, int64_t nb_o, float *parts_out, int E, int n_head, int n_seq,
                                  const uint8_t *wte, int64_t wte_nb, const float *wpe, const int32_t *tokens, int n_vocab,
                                  hipStream_t st);
bool gpt2_block_embeds(int type);
hipError_t gpt2_mlp_block_launch(int layer, int type, const float *base, const float *bias_in, const float *parts_in, int n_parts_in,
                                 float *x_out, const float *ln_g, const float *ln_b, float eps, const uint8_t *w_fc,
                                 int64_t nb_fc, const float *b_fc, const uint8_t *w_mp, int64_t nb_mp, float *parts_out, int E,
                                 int n_head, int n_seq, hipStream_t st);
bool gpt2_block_repacks(int type);
hipError_t gpt2_block_repack(int type, int E, const uint8_t *w_o, uint8_t *o_dst, const uint8_t *w_mp, uint8_t *mp_dst,
                             size_t *o_bytes, size_t *mp_bytes, hipStream_t st);
hipError_t gpt2_resid_launch(const float *base, const float *bias_in, const float *parts_in, int n_parts_in, float *x_out, int E,
                             int n_seq, hipStream_t st);

}  // namespace mi355x
