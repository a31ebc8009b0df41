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

#include <algorithm>

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

// Split-key decode attention ("flash decoding"): grid (n_head, n_seq, nsplit), 256 threads.
// Workgroup (h, s, c) takes keys [c*chunk, min(p+1, (c+1)*chunk)), chunk = ceil((p+1)/nsplit)
// with p = pos[s] read on the device, so one captured launch serves every position and all
// nsplit*n_head*n_seq workgroups stream the cache in parallel. Each writes (max, sum, o[64])
// of its keys; the last to finish (device-scope counter, release/acquire fences across the 8
// XCDs' L2s) merges them with the usual rescaling and resets the counter for the next launch.
// Dynamic LDS: chunk_max floats of scores.
__global__ __launch_bounds__(256) void attn_decode_kernel(const float *__restrict__ qkv, float *__restrict__ kc, float *__restrict__ vc,
                                                          const int32_t *__restrict__ pos, float *__restrict__ out, float *__restrict__ part,
                                                          uint32_t *__restrict__ counter, int n_embd, int n_ctx, float scale) {
    extern __shared__ float sc[];
    __shared__ float red[4][HEAD_DIM];
    __shared__ float rmax[4], rsum[4];
    __shared__ bool is_last;
    const int h = blockIdx.x, s = blockIdx.y, c = blockIdx.z, nsplit = gridDim.z;
    const int n_head = gridDim.x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int p = min(max(pos[s], 0), n_ctx - 1);
    const int nk = p + 1;
    const int chunk = (nk + nsplit - 1) / nsplit;
    const int j0 = c * chunk, j1 = min(nk, j0 + chunk);
    const float *q = qkv + (int64_t)s * 3 * n_embd + h * HEAD_DIM;
    const float *kcur = q + n_embd;
    const float *vcur = q + 2 * n_embd;
    float *K = kc + (int64_t)s * n_ctx * n_embd + h * HEAD_DIM;
    float *V = vc + (int64_t)s * n_ctx * n_embd + h * HEAD_DIM;
    float *pm = part + ((int64_t)(s * n_head + h) * nsplit + c) * (HEAD_DIM + 2);

    // the new token's K and V go to the cache once (the reference's ggml_cpy into memory_k/v);
    // this launch reads them from qkv, later launches from the cache
    if (c == 0 && tid < HEAD_DIM) {
        K[(int64_t)p * n_embd + tid] = kcur[tid];
        V[(int64_t)p * n_embd + tid] = vcur[tid];
    }

    float mx = -INFINITY, l = 0.f;
    if (j0 < j1) {
        // scores: 4 lanes per key (16 dims each), 64 keys per pass
        const int g = tid >> 2, sub = tid & 3;
        float4 qv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) qv[i] = reinterpret_cast<const float4 *>(q + sub * 16)[i];
        float lmax = -INFINITY;
        for (int j = j0 + g; j < j1; j += 64) {
            const float *kr = (j == p ? kcur : K + (int64_t)j * n_embd) + sub * 16;
            float4 kv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) kv[i] = reinterpret_cast<const float4 *>(kr)[i];
            float d = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) d += qv[i].x * kv[i].x + qv[i].y * kv[i].y + qv[i].z * kv[i].z + qv[i].w * kv[i].w;
            d += dpp_f<DPP_XOR1>(d);
            d += dpp_f<DPP_XOR2>(d);
            d *= scale;
            if (sub == 0) sc[j - j0] = d;
            lmax = fmaxf(lmax, d);
        }
        lmax = fmaxf(lmax, xchg<1>(lmax)); lmax = fmaxf(lmax, xchg<2>(lmax)); lmax = fmaxf(lmax, xchg<4>(lmax));
        lmax = fmaxf(lmax, xchg<8>(lmax)); lmax = fmaxf(lmax, xchg<16>(lmax)); lmax = fmaxf(lmax, xchg<32>(lmax));
        if (lane == 0) rmax[wave] = lmax;
        __syncthreads();
        mx = fmaxf(fmaxf(rmax[0], rmax[1]), fmaxf(rmax[2], rmax[3]));
        float lsum = 0.f;
        for (int j = j0 + tid; j < j1; j += 256) {
            const float e = expf(sc[j - j0] - mx);
            sc[j - j0] = e;
            lsum += e;
        }
        lsum = wave_sum(lsum);
        if (lane == 0) rsum[wave] = lsum;
        __syncthreads();
        l = (rsum[0] + rsum[1]) + (rsum[2] + rsum[3]);

        // o = sum_j e_j V_j: lane = (key slot ks = lane >> 4, dims 4*(lane & 15) .. +3), a wave
        // covers 4 keys per pass (coalesced 256-B rows), the workgroup 16; 2 passes in flight
        const int ks = lane >> 4, dq = (lane & 15) * 4;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int j = j0 + wave * 4 + ks; j < j1; j += 16) {
            const float e = sc[j - j0];
            const float4 v = *reinterpret_cast<const float4 *>((j == p ? vcur : V + (int64_t)j * n_embd) + dq);
            acc.x += e * v.x; acc.y += e * v.y; acc.z += e * v.z; acc.w += e * v.w;
        }
        acc.x += xchg<16>(acc.x); acc.y += xchg<16>(acc.y); acc.z += xchg<16>(acc.z); acc.w += xchg<16>(acc.w);
        acc.x += xchg<32>(acc.x); acc.y += xchg<32>(acc.y); acc.z += xchg<32>(acc.z); acc.w += xchg<32>(acc.w);
        if (lane < 16) *reinterpret_cast<float4 *>(&red[wave][dq]) = acc;
        __syncthreads();
        if (tid < HEAD_DIM) pm[2 + tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
    } else if (tid < HEAD_DIM) {
        pm[2 + tid] = 0.f;
    }
    if (tid == 0) {
        pm[0] = mx;
        pm[1] = l;
    }

    // last-arriving workgroup of (h, s) merges the nsplit partials
    __threadfence();
    __syncthreads();
    if (tid == 0) {
        const uint32_t prev = atomicAdd(&counter[s * n_head + h], 1u);
        is_last = prev == (uint32_t)nsplit - 1;
    }
    __syncthreads();
    if (!is_last) return;
    __threadfence();
    if (tid < HEAD_DIM) {
        const float *pb = part + (int64_t)(s * n_head + h) * nsplit * (HEAD_DIM + 2);
        float M = -INFINITY;
        for (int i = 0; i < nsplit; ++i) M = fmaxf(M, __builtin_nontemporal_load(pb + i * (HEAD_DIM + 2)));
        float L = 0.f, O = 0.f;
        for (int i = 0; i < nsplit; ++i) {
            const float *pi = pb + i * (HEAD_DIM + 2);
            const float li = __builtin_nontemporal_load(pi + 1);
            if (li > 0.f) {
                const float w = expf(__builtin_nontemporal_load(pi) - M);
                L += w * li;
                O += w * __builtin_nontemporal_load(pi + 2 + tid);
            }
        }
        out[(int64_t)s * n_embd + h * HEAD_DIM + tid] = O / L;
    }
    if (tid == 0) counter[s * n_head + h] = 0u;
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

// keys per split: at most 64 (the score pass width); n_ctx = 1024 -> 16 splits
int gpt2_attn_nsplit(int n_ctx) { return std::min(64, std::max(1, (n_ctx + 63) / 64)); }

hipError_t gpt2_attn_launch(const float *qkv, float *kc, float *vc, const int32_t *pos, float *out, float *part, uint32_t *counter,
                            int n_seq, int n_head, int n_embd, int n_ctx, float scale, hipStream_t st) {
    if (n_embd != n_head * HEAD_DIM) return hipErrorInvalidValue;
    const int nsplit = gpt2_attn_nsplit(n_ctx);
    const int chunk_max = (n_ctx + nsplit - 1) / nsplit;
    hipLaunchKernelGGL(attn_decode_kernel, dim3(n_head, n_seq, nsplit), dim3(256), (size_t)chunk_max * sizeof(float), st, qkv, kc, vc,
                       pos, out, part, counter, n_embd, n_ctx, scale);
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
