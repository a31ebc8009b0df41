// gpt2_ops.hip — the non-matmul kernels of the GPT-2 decode engine (gpt2.cpp).
//
// The matmuls and everything that can ride on them (layer norms, biases, GELU, residual adds)
// run inside the fused mat-vec (mmvq_fused.hip). What is left is here:
//   * embed_kernel     : inpL = get_rows(wte, token) + get_rows(wpe, pos)
//                        (examples/gpt-2/main-sched.cpp:589-595; dequantized rows bit-exact,
//                        src/ggml-cpu/ops.cpp get_rows_q)
//   * attn_decode_kernel: one query token per sequence against its KV cache: stores K/V of the
//                        new token (main-sched.cpp:648-655), KQ = K.Q scaled by 1/sqrt(d)
//                        (:685-694), softmax (:700-703; nothing to mask for a single query at
//                        the end of the sequence, :696-698), KQV = V^T.softmax merged back to
//                        [n_embd] (:705-735). Layout, per layer: cache[seq][n_ctx][n_embd] f32,
//                        the reference's memory_k/memory_v rows (:388-396) with a sequence axis.
//   * argmax_kernel    : greedy next token (lowest index on ties) for the device-resident loop
//   * advance_kernel   : pos[s] += 1 after a step
// Positions live in device memory, so one captured hipGraph replays every decode step.
#include <hip/hip_runtime.h>

#include "deq.h"

namespace mi355x {

namespace {

constexpr int HEAD_DIM = 64;   // every GPT-2 size (117M .. 1.5B) uses 64-wide heads

template <int T>
__global__ __launch_bounds__(256) void embed_kernel(const uint8_t *__restrict__ wte, int64_t wte_nb1, const float *__restrict__ wpe,
                                                    const int32_t *__restrict__ tokens, const int32_t *__restrict__ pos,
                                                    float *__restrict__ x, int n_embd, int n_vocab, int n_ctx) {
    const int s = blockIdx.x;
    const int t = min(max(tokens[s], 0), n_vocab - 1);
    const int p = min(max(pos[s], 0), n_ctx - 1);
    const uint8_t *row = wte + (int64_t)t * wte_nb1;
    for (int i = threadIdx.x; i < n_embd; i += blockDim.x) {
        float e;
        if constexpr (T == T_F32) {
            e = reinterpret_cast<const float *>(row)[i];
        } else {
            const int b = i / QT<T>::blck;
            e = deq_one<T>(row + (int64_t)b * QT<T>::bytes, i - b * QT<T>::blck);
        }
        x[(int64_t)s * n_embd + i] = e + wpe[(int64_t)p * n_embd + i];
    }
}

// grid (n_head, n_seq), 256 threads = 4 waves; dynamic LDS: n_ctx floats of scores
__global__ __launch_bounds__(256) void attn_decode_kernel(const float *__restrict__ qkv, float *__restrict__ kc, float *__restrict__ vc,
                                                          const int32_t *__restrict__ pos, float *__restrict__ out, int n_embd,
                                                          int n_ctx, float scale) {
    extern __shared__ float sc[];
    __shared__ float red[4][HEAD_DIM];
    __shared__ float rmax[4], rsum[4];
    const int h = blockIdx.x, s = blockIdx.y;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int p = min(max(pos[s], 0), n_ctx - 1);
    const float *q = qkv + (int64_t)s * 3 * n_embd + h * HEAD_DIM;
    const float *kcur = q + n_embd;
    const float *vcur = q + 2 * n_embd;
    float *K = kc + (int64_t)s * n_ctx * n_embd + h * HEAD_DIM;
    float *V = vc + (int64_t)s * n_ctx * n_embd + h * HEAD_DIM;

    // store the new token's K and V (the reference's ggml_cpy into memory_k / memory_v)
    if (tid < HEAD_DIM) {
        K[(int64_t)p * n_embd + tid] = kcur[tid];
        V[(int64_t)p * n_embd + tid] = vcur[tid];
    }

    // scores: 4 lanes per key, 16 dims each (float4 x 4); 16 keys per wave per pass
    const int g = lane >> 2, sub = lane & 3;
    float4 qv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) qv[i] = reinterpret_cast<const float4 *>(q + sub * 16)[i];
    float lmax = -INFINITY;
    for (int j = wave * 16 + g; j <= p; j += 64) {
        const float *kr = (j == p ? kcur : K + (int64_t)j * n_embd) + sub * 16;
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float4 kv = reinterpret_cast<const float4 *>(kr)[i];
            d += qv[i].x * kv.x + qv[i].y * kv.y + qv[i].z * kv.z + qv[i].w * kv.w;
        }
        d += dpp_f<DPP_XOR1>(d);
        d += dpp_f<DPP_XOR2>(d);
        d *= scale;
        if (sub == 0) sc[j] = d;
        lmax = fmaxf(lmax, d);
    }
    // softmax over [0, p] (src/ggml-cpu/ops.cpp soft_max: max, exp(x - max), 1/sum)
    lmax = fmaxf(lmax, xchg<1>(lmax)); lmax = fmaxf(lmax, xchg<2>(lmax)); lmax = fmaxf(lmax, xchg<4>(lmax));
    lmax = fmaxf(lmax, xchg<8>(lmax)); lmax = fmaxf(lmax, xchg<16>(lmax)); lmax = fmaxf(lmax, xchg<32>(lmax));
    if (lane == 0) rmax[wave] = lmax;
    __syncthreads();
    const float mx = fmaxf(fmaxf(rmax[0], rmax[1]), fmaxf(rmax[2], rmax[3]));
    float lsum = 0.f;
    for (int j = tid; j <= p; j += 256) {
        const float e = expf(sc[j] - mx);
        sc[j] = e;
        lsum += e;
    }
    lsum = wave_sum(lsum);
    if (lane == 0) rsum[wave] = lsum;
    __syncthreads();
    const float inv = 1.0f / ((rsum[0] + rsum[1]) + (rsum[2] + rsum[3]));

    // KQV: wave w sums keys j = w, w+4, ...; lane = head dimension (coalesced 256-B rows)
    float acc = 0.f;
    for (int j = wave; j <= p; j += 4) acc += sc[j] * (j == p ? vcur[lane] : V[(int64_t)j * n_embd + lane]);
    red[wave][lane] = acc;
    __syncthreads();
    if (wave == 0) out[(int64_t)s * n_embd + h * HEAD_DIM + lane] = ((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane])) * inv;
}

__global__ __launch_bounds__(1024) void argmax_kernel(const float *__restrict__ logits, int n_vocab, int32_t *__restrict__ tokens) {
    __shared__ float bv[16];
    __shared__ int bi[16];
    const int s = blockIdx.x;
    const float *l = logits + (int64_t)s * n_vocab;
    float v = -INFINITY;
    int idx = 0x7fffffff;
    for (int i = threadIdx.x; i < n_vocab; i += blockDim.x) {
        const float x = l[i];
        if (x > v) { v = x; idx = i; }   // strided scan: a later i only wins when strictly greater
    }
    for (int d = 1; d < 64; d <<= 1) {
        const float ov = __shfl_xor(v, d);
        const int oi = __shfl_xor(idx, d);
        if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { bv[wave] = v; bi[wave] = idx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
            if (bv[w] > v || (bv[w] == v && bi[w] < idx)) { v = bv[w]; idx = bi[w]; }
        tokens[s] = idx == 0x7fffffff ? 0 : idx;
    }
}

__global__ void advance_kernel(int32_t *pos, int n_seq) {
    const int s = threadIdx.x;
    if (s < n_seq) pos[s] += 1;
}

}  // namespace

hipError_t gpt2_embed_launch(int wtype, const void *wte, int64_t wte_nb1, const float *wpe, const int32_t *tokens,
                             const int32_t *pos, float *x, int n_seq, int n_embd, int n_vocab, int n_ctx, hipStream_t st) {
    const auto *w = static_cast<const uint8_t *>(wte);
    switch (wtype) {
        case T_F32: hipLaunchKernelGGL(embed_kernel<T_F32>, dim3(n_seq), dim3(256), 0, st, w, wte_nb1, wpe, tokens, pos, x, n_embd, n_vocab, n_ctx); break;
        case T_Q4_0: hipLaunchKernelGGL(embed_kernel<T_Q4_0>, dim3(n_seq), dim3(256), 0, st, w, wte_nb1, wpe, tokens, pos, x, n_embd, n_vocab, n_ctx); break;
        case T_Q8_0: hipLaunchKernelGGL(embed_kernel<T_Q8_0>, dim3(n_seq), dim3(256), 0, st, w, wte_nb1, wpe, tokens, pos, x, n_embd, n_vocab, n_ctx); break;
        case T_Q4_K: hipLaunchKernelGGL(embed_kernel<T_Q4_K>, dim3(n_seq), dim3(256), 0, st, w, wte_nb1, wpe, tokens, pos, x, n_embd, n_vocab, n_ctx); break;
        case T_Q5_K: hipLaunchKernelGGL(embed_kernel<T_Q5_K>, dim3(n_seq), dim3(256), 0, st, w, wte_nb1, wpe, tokens, pos, x, n_embd, n_vocab, n_ctx); break;
        case T_Q6_K: hipLaunchKernelGGL(embed_kernel<T_Q6_K>, dim3(n_seq), dim3(256), 0, st, w, wte_nb1, wpe, tokens, pos, x, n_embd, n_vocab, n_ctx); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t gpt2_attn_launch(const float *qkv, float *kc, float *vc, const int32_t *pos, float *out, int n_seq, int n_head,
                            int n_embd, int n_ctx, float scale, hipStream_t st) {
    if (n_embd != n_head * HEAD_DIM) return hipErrorInvalidValue;
    hipLaunchKernelGGL(attn_decode_kernel, dim3(n_head, n_seq), dim3(256), (size_t)n_ctx * sizeof(float), st, qkv, kc, vc, pos, out,
                       n_embd, n_ctx, scale);
    return hipGetLastError();
}

hipError_t gpt2_argmax_launch(const float *logits, int n_seq, int n_vocab, int32_t *tokens, hipStream_t st) {
    hipLaunchKernelGGL(argmax_kernel, dim3(n_seq), dim3(1024), 0, st, logits, n_vocab, tokens);
    return hipGetLastError();
}

hipError_t gpt2_advance_launch(int32_t *pos, int n_seq, hipStream_t st) {
    hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(64 * ((n_seq + 63) / 64)), 0, st, pos, n_seq);
    return hipGetLastError();
}

}  // namespace mi355x
