// qmm_args.h — launch descriptors shared by the host dispatch and the kernels.
//
// A descriptor carries ggml tensor geometry verbatim (ne / nb in elements and bytes), so the
// kernels honour every layout test-backend-ops produces: broadcast over dims 2/3 (r2, r3),
// permuted src0/src1 (arbitrary nb01..nb03, nb11..nb13) and views (reference
// src/ggml-cpu/ggml-cpu.c:1133-1191 defines the semantics).
#pragma once
#include <stdint.h>

namespace mi355x {

enum { EPI_GELU = 1, EPI_RESID = 2, EPI_ARGMAX = 4 };

// EPI_ARGMAX: per-workgroup partial argmax slots per output column (GPT-2 greedy sampling)
constexpr int ARGMAX_SLOTS = 2048;

// decode attention: key splits per (sequence, head) and the partial record (m, l, o[64])
constexpr int ATTN_SPLITS = 4;
constexpr int ATTN_PART_STRIDE = 4 + 64;   // m, l, 2 pad (16-B aligned o), o[64]

struct MmArgs {
    const uint8_t *w;      // src0, quantized rows (nb00 == block bytes)
    int64_t nb01, nb02, nb03;
    const uint8_t *x;      // src1, f32 rows (nb10 == 4)
    int64_t nb11, nb12, nb13;
    uint8_t *dst;          // dst, f32 rows (nb0 == 4)
    int64_t nb1, nb2, nb3;
    int K;                 // ne00 == ne10
    int N;                 // ne01: weight rows = dst ne0
    int M;                 // ne11: src1 columns handled by this launch
    int ne12, ne13;        // batch dims of src1 / dst
    int r2, r3;            // ne12/ne02, ne13/ne03
    // MUL_MAT_ID (ids != nullptr): dst[e, t] = as[ids[e,t]] @ b[:, e % ne11_b, t]
    const int32_t *ids;
    int64_t ids_nb0, ids_nb1;
    int n_used;            // ids->ne[0]
    int n_tok;             // ids->ne[1]
    int ne11_b;            // b->ne[1]
    int n_expert;          // as->ne[2]
    int x_aligned16;       // src1 rows / strides are 16-byte aligned
    int n_it;              // mat-vec: K iterations per row = ceil(ceil(K/64) / lanes per row)
    // fused decode-layer variant (gpt2.cpp; plain MUL_MAT leaves all of these zero):
    //   prologue, ln_g != nullptr: each src1 column is layer-normalized before quantization,
    //     x <- (x - mean) / sqrt(var + ln_eps) * ln_g + ln_b  (ggml_norm + mul + add)
    //   epilogue: v <- v + bias[row]; epi & EPI_GELU: v <- gelu(v); epi & EPI_RESID: dst += v
    const float *ln_g, *ln_b;
    float ln_eps;
    const float *bias;
    int epi;
    //   EPI_RESID reads the residual from `resid` (column stride resid_nb1 bytes) when set,
    //     else from dst itself (dst += v)
    const uint8_t *resid;
    int64_t resid_nb1;
    //   epi & EPI_ARGMAX: every workgroup also writes the (max, lowest row) of the rows it
    //     produced, per column c, to amax_v / amax_i [c * ARGMAX_SLOTS + blockIdx.x]
    float *amax_v;
    int32_t *amax_i;
    //   attn_part != nullptr: the activations are the decode attention output, merged here
    //     from ATTN_SPLITS flash-decoding partials per (column, head) (gpt2_ops.hip):
    //     part[((col * n_head + h) * ATTN_SPLITS + i) * ATTN_PART_STRIDE + {0: m, 1: l, 4..67: o}]
    const float *attn_part;
    int n_head;
    //   copy-out (graph_compute: the K / V cache writes that follow a fused qkv mat-vec,
    //     main-sched.cpp:648-655): output rows [cp_r0[i], cp_r0[i] + cp_n[i]) of column m are
    //     also stored to cp_dst[i] + m * cp_nb1[i] bytes + (row - cp_r0[i]) floats
    float *cp_dst[2];
    int cp_r0[2], cp_n[2];
    int64_t cp_nb1[2];
    int fused;
    // diagnostics (GGML_MI355X_STAMPS): per-workgroup s_memrealtime stamps, or nullptr
    unsigned long long *stamps;
    int diag;              // diagnostics: bit0 = skip activation loads, bit1 = skip weight loads
};

}  // namespace mi355x
