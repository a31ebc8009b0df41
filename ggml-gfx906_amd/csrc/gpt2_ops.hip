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
#include "mmvq_impl.h"   // group_reduce_transpose

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

// Decode attention as flash-decoding partials: workgroup (h, s, c) of 4 waves takes split c of
// the p + 1 visible keys (p = pos[s], read on the device, so one captured launch serves every
// position), cut into ATTN_SPLITS contiguous chunks and each chunk into 4 wave ranges. Inside a
// wave every lane owns keys j = j0 + lane + 64 t with its own online-softmax state (running max
// m, sum l, o = sum_j e^(s_j - m) V_j as 64 registers); one butterfly transpose merges the lanes
// (lane d ends with o[d]), LDS merges the 4 waves, and the workgroup writes its (m, l, o[64])
// record. The consumer — the c_proj mat-vec's prologue (mmvq_impl.h attn_merge_load) — merges
// the ATTN_SPLITS records per head, so the attention output never makes its own HBM round trip
// and no workgroup waits on another. K and V rows are read once, 16 dwordx4 per lane each, in
// flight together. Numerically: softmax(K.q * scale) . V of main-sched.cpp:685-735, evaluated in
// the rescaling order of online softmax.
__global__ __launch_bounds__(256) void attn_partial_kernel(const float *__restrict__ qkv, float *__restrict__ kc, float *__restrict__ vc,
                                                           const int32_t *__restrict__ pos, float *__restrict__ part, int n_embd, int n_ctx,
                                                           float scale) {
    __shared__ float4 qs[HEAD_DIM / 4];
    __shared__ float wo[4][HEAD_DIM];
    __shared__ float wm[4], wl[4];
    const int h = blockIdx.x, s = blockIdx.y, c = blockIdx.z, n_head = gridDim.x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int p = min(max(pos[s], 0), n_ctx - 1);
    const int nk = p + 1;
    const float *q = qkv + (int64_t)s * 3 * n_embd + h * HEAD_DIM;
    const float *kcur = q + n_embd;
    const float *vcur = q + 2 * n_embd;
    float *K = kc + (int64_t)s * n_ctx * n_embd + h * HEAD_DIM;
    float *V = vc + (int64_t)s * n_ctx * n_embd + h * HEAD_DIM;

    // q (pre-scaled) to LDS; split 0 stores the new token's K and V into the cache (the
    // reference's ggml_cpy into memory_k / memory_v); this launch reads them from qkv
    if (tid < HEAD_DIM / 4) {
        float4 v = reinterpret_cast<const float4 *>(q)[tid];
        v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
        qs[tid] = v;
    } else if (c == 0 && tid >= 64 && tid < 64 + HEAD_DIM / 4) {
        const int i = tid - 64;
        reinterpret_cast<float4 *>(K + (int64_t)p * n_embd)[i] = reinterpret_cast<const float4 *>(kcur)[i];
        reinterpret_cast<float4 *>(V + (int64_t)p * n_embd)[i] = reinterpret_cast<const float4 *>(vcur)[i];
    }
    __syncthreads();

    const int chunk = (nk + ATTN_SPLITS - 1) / ATTN_SPLITS;
    const int c0 = min(nk, c * chunk), c1 = min(nk, c0 + chunk);
    const int wchunk = (c1 - c0 + 3) >> 2;
    const int j0 = min(c1, c0 + wave * wchunk), j1 = min(c1, j0 + wchunk);
    float m = -INFINITY, l = 0.f;
    float o[HEAD_DIM];
#pragma unroll
    for (int d = 0; d < HEAD_DIM; ++d) o[d] = 0.f;
    for (int jb = j0; jb < j1; jb += 64) {
        const int j = jb + lane;
        const bool live = j < j1;
        const int jc = live ? j : j0;                     // dead lanes re-read a live row
        const float *kr = jc == p ? kcur : K + (int64_t)jc * n_embd;
        const float *vr = jc == p ? vcur : V + (int64_t)jc * n_embd;
        float4 kv[HEAD_DIM / 4], vv[HEAD_DIM / 4];
#pragma unroll
        for (int i = 0; i < HEAD_DIM / 4; ++i) kv[i] = reinterpret_cast<const float4 *>(kr)[i];
#pragma unroll
        for (int i = 0; i < HEAD_DIM / 4; ++i) vv[i] = reinterpret_cast<const float4 *>(vr)[i];
        float sc = 0.f;
#pragma unroll
        for (int i = 0; i < HEAD_DIM / 4; ++i) {
            const float4 qv = qs[i];
            sc += qv.x * kv[i].x + qv.y * kv[i].y + qv.z * kv[i].z + qv.w * kv[i].w;
        }
        if (live) {
            const float mn = fmaxf(m, sc);
            const float cr = expf(m - mn);                // 0 on the first key (m = -inf)
            const float e = expf(sc - mn);
            l = l * cr + e;
#pragma unroll
            for (int i = 0; i < HEAD_DIM / 4; ++i) {
                o[4 * i + 0] = o[4 * i + 0] * cr + e * vv[i].x;
                o[4 * i + 1] = o[4 * i + 1] * cr + e * vv[i].y;
                o[4 * i + 2] = o[4 * i + 2] * cr + e * vv[i].z;
                o[4 * i + 3] = o[4 * i + 3] * cr + e * vv[i].w;
            }
            m = mn;
        }
    }
    // wave merge: rescale every lane to the wave max, then one transpose reduction
    float M = m;
    M = fmaxf(M, xchg<1>(M)); M = fmaxf(M, xchg<2>(M)); M = fmaxf(M, xchg<4>(M));
    M = fmaxf(M, xchg<8>(M)); M = fmaxf(M, xchg<16>(M)); M = fmaxf(M, xchg<32>(M));
    const float f = l > 0.f ? expf(m - M) : 0.f;
    l = wave_sum(l * f);
#pragma unroll
    for (int d = 0; d < HEAD_DIM; ++d) o[d] *= f;
    const float od = group_reduce_transpose<HEAD_DIM, 64>(o);   // lane d: sum over the wave's keys
    wo[wave][lane] = od;
    if (lane == 0) { wm[wave] = M; wl[wave] = l; }
    __syncthreads();
    if (wave == 0) {
        float MX = -INFINITY;
#pragma unroll
        for (int w = 0; w < 4; ++w) if (wl[w] > 0.f) MX = fmaxf(MX, wm[w]);
        float L = 0.f, O = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            if (wl[w] > 0.f) {
                const float g = expf(wm[w] - MX);
                L += g * wl[w];
                O += g * wo[w][lane];
            }
        }
        float *rec = part + ((int64_t)(s * n_head + h) * ATTN_SPLITS + c) * ATTN_PART_STRIDE;
        rec[4 + lane] = O;                                // unnormalized: the consumer divides by sum l
        if (lane == 0) {
            rec[0] = MX;
            rec[1] = L;                                   // 0 for an empty split (skipped by the merge)
        }
    }
}

// greedy next token from the lm_head's per-workgroup partials (EPI_ARGMAX, mmvq_impl.h):
// ARGMAX_SLOTS (value, row) pairs per sequence, unused slots hold (-inf, INT_MAX). Lowest row
// on ties. Also advances the sequence's position (the step's last launch).
__global__ __launch_bounds__(256) void argmax_final_kernel(const float *__restrict__ pv, const int32_t *__restrict__ pi,
                                                           int32_t *__restrict__ tokens, int32_t *__restrict__ pos) {
    __shared__ float bv[4];
    __shared__ int bi[4];
    const int s = blockIdx.x;
    float v = -INFINITY;
    int idx = 0x7fffffff;
    // every slot pair of this thread is loaded before any is compared (one memory round trip,
    // not ARGMAX_SLOTS / 256 dependent ones)
    constexpr int PER = ARGMAX_SLOTS / 256;
    float xs[PER];
    int is[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        xs[u] = pv[(int64_t)s * ARGMAX_SLOTS + threadIdx.x + 256 * u];
        is[u] = pi[(int64_t)s * ARGMAX_SLOTS + threadIdx.x + 256 * u];
    }
#pragma unroll
    for (int u = 0; u < PER; ++u)
        if (xs[u] > v || (xs[u] == v && is[u] < idx)) { v = xs[u]; idx = is[u]; }
    for (int d = 1; d < 64; d <<= 1) {
        const float ov = __shfl_xor(v, d);
        const int oi = __shfl_xor(idx, d);
        if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { bv[wave] = v; bi[wave] = idx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w)
            if (bv[w] > v || (bv[w] == v && bi[w] < idx)) { v = bv[w]; idx = bi[w]; }
        tokens[s] = idx == 0x7fffffff ? 0 : idx;
        pos[s] += 1;
    }
}

// reset the partial slots to (-inf, INT_MAX) (once per context)
__global__ void argmax_reset_kernel(float *pv, int32_t *pi, int64_t n) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) { pv[k] = -INFINITY; pi[k] = 0x7fffffff; }
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

hipError_t gpt2_attn_launch(const float *qkv, float *kc, float *vc, const int32_t *pos, float *part, int n_seq, int n_head,
                            int n_embd, int n_ctx, float scale, hipStream_t st) {
    if (n_embd != n_head * HEAD_DIM) return hipErrorInvalidValue;
    hipLaunchKernelGGL(attn_partial_kernel, dim3(n_head, n_seq, ATTN_SPLITS), dim3(256), 0, st, qkv, kc, vc, pos, part, n_embd,
                       n_ctx, scale);
    return hipGetLastError();
}

hipError_t gpt2_argmax_launch(const float *pv, const int32_t *pi, int n_seq, int32_t *tokens, int32_t *pos, hipStream_t st) {
    hipLaunchKernelGGL(argmax_final_kernel, dim3(n_seq), dim3(256), 0, st, pv, pi, tokens, pos);
    return hipGetLastError();
}

hipError_t gpt2_argmax_reset(float *pv, int32_t *pi, int n_seq, hipStream_t st) {
    const int64_t n = (int64_t)n_seq * ARGMAX_SLOTS;
    hipLaunchKernelGGL(argmax_reset_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, pv, pi, n);
    return hipGetLastError();
}

hipError_t gpt2_advance_launch(int32_t *pos, int n_seq, hipStream_t st) {
    hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(64 * ((n_seq + 63) / 64)), 0, st, pos, n_seq);
    return hipGetLastError();
}

}  // namespace mi355x
