// gpt2_block.hip — GPT-2 decode layer as TWO launches (attention block, MLP block).
//
// The five-launch layer of gpt2.cpp (qkv mat-vec, attention, c_proj, fc, mlp proj) spends most
// of each launch waiting: the kernel boundary, then one memory latency for the activations,
// then a few hundred nanoseconds of work on ~1 MB of weights. Here every workgroup owns a
// piece of the layer that needs no other workgroup's output until the next launch:
//
//   attn block, workgroup (head h, sequence s):
//     x      = base + bias + sum_i part_in[i]          (previous block's residual + partials)
//     q,k,v  = W_attn[rows of head h] . LN1(x) + b     (192 rows, mat-vec on the int8 path)
//     o      = softmax(K.q / sqrt(64)) . V             (cache keys 0..p-1, key p from LDS;
//                                                       stores the new K/V row of head h)
//     part_out[h] = W_proj[:, cols of head h] . o      (the c_proj product restricted to the
//                                                       head's 64 columns: a K-split of c_proj)
//   mlp block, workgroup (slice j of 128 hidden units, sequence s):
//     y      = x + b_proj + sum_h part_attn[h]
//     h_j    = gelu(W_fc[rows of slice j] . LN2(y) + b_fc)
//     part_out[j] = W_mlp[:, cols of slice j] . h_j     (K-split of the MLP projection)
//
// The K-splits are exact restatements of the reference's single mat-vecs
// (examples/gpt-2/main-sched.cpp:706-730 c_proj, :760-808 fc / gelu / proj): each 32-block of
// the activation vector lies inside one head / one slice, so its int8 quantization
// (quantize_row_q8_0/1, the block the dot products use) is the same block the full vector
// would give; only the order of the fp32 sums over the K-splits differs. The partial sums are
// kept as f32 slabs [split][seq][n_embd] and summed in a fixed order by the next launch's
// prologue (resid_issue / resid_finish), so results are deterministic and independent of the grid.
// Workgroup 0 of every block also writes the summed residual ("materialized" x), which the
// next-but-one block uses as its base. For Q4_0 / Q8_0 the K-split streams of c_proj and the
// MLP projection come from head- / slice-major copies (gpt2_block_repack), so they are
// contiguous. Measured choices: 128-unit slices beat 256 (4207 vs 3850
// tokens/s, GPT-2 117M Q4_0), LDS-only barriers keep weight streams in flight.
#include <algorithm>
#include <type_traits>

#include "mmvq_impl.h"

namespace mi355x {

unsigned long long *stamps_buffer();

namespace {

constexpr int HD = 64;                     // head dim of every GPT-2 size
constexpr int BT = MMVQ_THREADS;           // 512 threads = 8 waves
constexpr int NW = MMVQ_WAVES;
constexpr int E_MAX = 1024;                // n_embd bound of these kernels (GPT-2 117M / 345M; wider
                                           // models keep the five-launch layer: one slot pass per row here)
constexpr int MLP_SLICE = 128;             // hidden units per mlp workgroup (two whole slots of every type;
                                           // Q6_K: one 128-half of a super-block)

// 32-block types: the engine repacks c_proj and the MLP projection into head- / slice-major
// copies whose K-splits are contiguous (gpt2.cpp, gpt2_block_repack); K-quant slots are not
// contiguous byte ranges (header + chunk), so those read the ggml rows in place
template <int T> constexpr bool REPACK = T == T_Q4_0 || T == T_Q8_0;
constexpr bool REPACK_TYPE(int t) { return t == T_Q4_0 || t == T_Q8_0; }

// LDS bytes of one quantized activation vector of K values (XSmem layout, nc = 1)
constexpr int xs_bytes(int K) { return K + 4 * (K / 32) * 2 + 4 * (K / 16); }

struct BlockArgs {
    // residual input: x = base + bias + sum_{i < n_parts_in} parts_in[i][s]  (bias / parts optional)
    const float *base, *bias_in, *parts_in;
    int n_parts_in;
    float *x_out;                          // materialized x, written by workgroups with blockIdx.x == 0
    const float *ln_g, *ln_b;
    float eps;
    // attn block
    const uint8_t *w_qkv;
    int64_t nb_qkv;
    const float *b_qkv;
    float *kc, *vc;                        // this layer's caches [seq][n_ctx][n_embd]
    const int32_t *pos;
    float scale;
    int n_ctx;
    const uint8_t *w_o;                    // c_proj [n_embd][n_embd]
    int64_t nb_o;
    // mlp block
    const uint8_t *w_fc;
    int64_t nb_fc;
    const float *b_fc;
    const uint8_t *w_mp;                   // mlp proj [n_embd][4 n_embd]
    int64_t nb_mp;
    float *parts_out;                      // [blockIdx.x][n_seq][n_embd]
    int E, n_head, n_seq;
    // diagnostics (GGML_MI355X_STAMPS): s_memrealtime phase stamps of workgroups (x, 0),
    // slot ((2 * layer + kind) * 64 + x) * 16 + phase; nullptr when off
    unsigned long long *stamps;
    int layer;
    // layer 0 of a first stage, Q4_0 / Q8_0 (EMB kernels): the residual is the token embedding
    // wte[tokens[s]] + wpe[pos[s]] (main-sched.cpp:589-595), dequantized in the prologue
    const uint8_t *wte;
    int64_t wte_nb;
    const float *wpe;
    const int32_t *tokens;
    int n_vocab;
};

__device__ __forceinline__ void stamp(const BlockArgs &a, int kind, int phase) {
    if (a.stamps != nullptr && threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < 64)
        a.stamps[((2 * a.layer + kind) * 64 + blockIdx.x) * 16 + phase] = __builtin_amdgcn_s_memrealtime();
}
// shader-clock stamp (s_memtime) into a free slot: the in-kernel clock is
// (memtime_end - memtime_start) / (realtime_end - realtime_start) x 100 MHz
__device__ __forceinline__ void stamp_clk(const BlockArgs &a, int kind, int slot) {
    if (a.stamps != nullptr && threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < 64)
        a.stamps[((2 * a.layer + kind) * 64 + blockIdx.x) * 16 + slot] = __builtin_amdgcn_s_memtime();
}

// The residual of sequence s: rows (base[s], bias, parts[0][s], parts[1][s], ...) summed. All
// 512 threads load: thread t takes the 8-float chunk c = t % (E/8) of rows rg, rg + G, rg + 2G,
// ... (row group rg = t / (E/8), G = 512 / (E/8) groups), so one issue round covers up to
// G * RROWS rows; each thread sums its rows in order, the row groups meet in LDS and are
// summed in order rg = 0 .. G-1. The order depends only on (E, number of rows): the resid
// kernel and every prologue give bit-identical x for the same inputs.
constexpr int RROWS = 6;                   // max rows per thread: one issue round covers G * RR rows
constexpr int RED_FLOATS = 4096;           // LDS floats of the row-group partials (G * E <= 4096)

template <int RR>
struct Resid {
    float4 v[RR][2];
};

__device__ __forceinline__ int resid_rows(const BlockArgs &a) { return 1 + (a.bias_in != nullptr) + a.n_parts_in; }

// branch-free (selects only): a load under a branch makes the compiler's in-order vmcnt
// bookkeeping ambiguous, and it then drains every load in flight (the weight stream) first
__device__ __forceinline__ const float *resid_row(const BlockArgs &a, int s, int r) {
    const int hb = a.bias_in != nullptr ? 1 : 0;
    const float *pp = a.parts_in + ((int64_t)max(r - 1 - hb, 0) * a.n_seq + s) * a.E;
    const float *p = (hb && r == 1) ? a.bias_in : pp;
    return r == 0 ? a.base + (int64_t)s * a.E : p;
}

template <int RR>
__device__ __forceinline__ void resid_issue(const BlockArgs &a, int s, int round, Resid<RR> &R) {
    const int nch = a.E / 8, G = BT / nch;
    const int c = (int)threadIdx.x % nch, rg = min((int)threadIdx.x / nch, G - 1);
    const int nrows = resid_rows(a);
#pragma unroll
    for (int i = 0; i < RR; ++i) {
        const int r = min(rg + G * (round * RR + i), nrows - 1);
        const float *p = resid_row(a, s, r) + 8 * c;
        R.v[i][0] = reinterpret_cast<const float4 *>(p)[0];
        R.v[i][1] = reinterpret_cast<const float4 *>(p)[1];
    }
}

template <int RR>
__device__ __forceinline__ void resid_accum(const BlockArgs &a, int round, const Resid<RR> &R, float4 &s0, float4 &s1) {
    const int nch = a.E / 8, G = BT / nch;
    const int rg = (int)threadIdx.x / nch;
    const int nrows = resid_rows(a);
#pragma unroll
    for (int i = 0; i < RR; ++i) {
        if (rg < G && rg + G * (round * RR + i) < nrows) {
            s0.x += R.v[i][0].x; s0.y += R.v[i][0].y; s0.z += R.v[i][0].z; s0.w += R.v[i][0].w;
            s1.x += R.v[i][1].x; s1.y += R.v[i][1].y; s1.z += R.v[i][1].z; s1.w += R.v[i][1].w;
        }
    }
}


// finish: the loads R were issued by the caller (before its weight stream); the host
// guarantees one round covers every row (gpt2_block_supported). Thread t < E/8 returns
// x[8t .. 8t+8) (others zeros). Contains a workgroup barrier.
template <int RR>
__device__ __forceinline__ void resid_finish(const BlockArgs &a, int s, const Resid<RR> &R0, float *red, float4 &x0, float4 &x1) {
    const int nch = a.E / 8, G = BT / nch;
    const int c = (int)threadIdx.x % nch, rg = (int)threadIdx.x / nch;
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
    resid_accum(a, 0, R0, s0, s1);
    if (rg < G) {
        reinterpret_cast<float4 *>(red + rg * a.E + 8 * c)[0] = s0;
        reinterpret_cast<float4 *>(red + rg * a.E + 8 * c)[1] = s1;
    }
    lds_barrier();
    x0 = x1 = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((int)threadIdx.x < nch) {
        for (int g = 0; g < G; ++g) {
            const float4 p0 = reinterpret_cast<const float4 *>(red + g * a.E + 8 * threadIdx.x)[0];
            const float4 p1 = reinterpret_cast<const float4 *>(red + g * a.E + 8 * threadIdx.x)[1];
            x0.x += p0.x; x0.y += p0.y; x0.z += p0.z; x0.w += p0.w;
            x1.x += p1.x; x1.y += p1.y; x1.z += p1.z; x1.w += p1.w;
        }
    }
}

// x[0] of the sequence from the row-group partials (the layer norm's shift; every thread)
__device__ __forceinline__ float resid_first(const BlockArgs &a, const float *red) {
    const int G = BT / (a.E / 8);
    float v = 0.f;
    for (int g = 0; g < G; ++g) v += red[g * a.E];
    return v;
}

__device__ __forceinline__ bool resid_in(const BlockArgs &a) { return (int)threadIdx.x < a.E / 8; }

__device__ __forceinline__ void store_resid(const BlockArgs &a, int s, const float4 &v0, const float4 &v1) {
    if (!resid_in(a)) return;
    float *o = a.x_out + (int64_t)s * a.E + 8 * threadIdx.x;
    reinterpret_cast<float4 *>(o)[0] = v0;
    reinterpret_cast<float4 *>(o)[1] = v1;
}

// ------------------------------------------------------------------------------------------
// rows of a quantized matrix dotted with a quantized activation vector in LDS, restricted to
// the slots [s0, s0 + ns) of each row (a K-split). LPR lanes per row, RPW rows per lane,
// NIT slot iterations per lane; one pass covers NW * (64 / LPR) * RPW rows. load() issues the
// weight stream (so it can be in flight while the activations are prepared), compute() dots
// and reduces; out(row, value) runs on the lane holding the row's sum.
// ------------------------------------------------------------------------------------------
template <int T, int LPR, int RPW, int NIT>
struct RowsDot {
    static constexpr int RPP = NW * (WAVE / LPR) * RPW;
    Frag<T> f[NIT][RPW];
    int r0, s0, ns;

    // s0_: first activation slot; ws0: first slot within the weight row (the same unless the
    // rows are a repacked slice, which starts at slot 0)
    template <class RowPtr>
    __device__ __forceinline__ void load(RowPtr rowptr, int nrows, int base, int s0_, int ns_, int ws0 = -1) {
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, sl = lane % LPR;
        s0 = s0_;
        ns = ns_;
        r0 = base + wave * (WAVE / LPR) * RPW + (lane / LPR) * RPW;
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int s = (ws0 < 0 ? s0 : ws0) + min(sl + it * LPR, ns - 1);
#pragma unroll
            for (int r = 0; r < RPW; ++r) f[it][r].template load<false>(rowptr(min(r0 + r, nrows - 1)), s, 0);
        }
    }

    template <class Out>
    __device__ __forceinline__ void compute(const XSmem &sm, int Kpad, int nrows, Out out) const {
        constexpr int NX = XdCount<T>::n;
        // V <= LPR: butterfly transpose (one row's sum per lane); otherwise (few lanes per row)
        // every row is summed over its LPR lanes and the row's first lane stores them all
        constexpr bool TRANSPOSE = LPR > 1 && pow2ceil(RPW) <= LPR;
        constexpr int V = TRANSPOSE ? pow2ceil(RPW) : RPW;
        const int lane = threadIdx.x & 63, sl = lane % LPR;
        const int nslots = Kpad / 64;
        float acc[V];
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int s_raw = sl + it * LPR;
            const int s = s0 + min(s_raw, ns - 1);
            const float live = s_raw < ns ? 1.f : 0.f;
            int xb0, x16b;
            if constexpr (T == T_Q6_K) {
                xb0 = 8 * (s >> 2) + 4 * ((s >> 1) & 1);
                x16b = 16 * (s >> 2) + 8 * ((s >> 1) & 1) + (s & 1);
            } else {
                xb0 = 2 * s;
                x16b = 0;
            }
            uint32_t X[16];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint4 t4 = *reinterpret_cast<const uint4 *>(sm.xq + (size_t)(j * nslots + s) * 16);
                X[4 * j + 0] = t4.x; X[4 * j + 1] = t4.y; X[4 * j + 2] = t4.z; X[4 * j + 3] = t4.w;
            }
            float dx[NX], sx[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) dx[i] = sm.xd[xb0 + i];
#pragma unroll
            for (int i = 0; i < NX; ++i) sx[i] = T == T_Q6_K ? sm.x16[x16b + 2 * i] : sm.xs[xb0 + i];
#pragma unroll
            for (int r = 0; r < RPW; ++r) acc[r] += live * f[it][r].dot(X, dx, sx);
        }
        if constexpr (!TRANSPOSE) {
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                if constexpr (LPR >= 2) acc[r] += xchg<1>(acc[r]);
                if constexpr (LPR >= 4) acc[r] += xchg<2>(acc[r]);
                if constexpr (LPR >= 8) acc[r] += xchg<4>(acc[r]);
                if constexpr (LPR >= 16) acc[r] += xchg<8>(acc[r]);
            }
            if (sl == 0) {
#pragma unroll
                for (int r = 0; r < RPW; ++r)
                    if (r0 + r < nrows) out(r0 + r, acc[r]);
            }
        } else {
            const float sum = group_reduce_transpose<V, LPR>(acc);
            constexpr int SHIFT = Log2<LPR>::v - Log2<V>::v;
            const int idx = sl >> SHIFT;
            if ((sl & ((1 << SHIFT) - 1)) == 0 && idx < RPW && r0 + idx < nrows) out(r0 + idx, sum);
        }
    }
};

// token embedding of sequence s for this thread's 8-value chunk (thread t < E/8: values
// 8t .. 8t+7; the others repeat a valid chunk): the block's raw scale and 8 code bytes and the
// wpe row are issued here; token and position are uniform per workgroup (scalar loads), so the
// vector loads wait on nothing in flight. embed_finish decodes exactly as dequantize_row_q4_0 /
// _q8_0 (src/ggml-quants.c:307-323, 401-415) and adds wpe (the ggml_add of :589-595).
struct Emb {
    uint32_t d;
    uint32_t q[2];
    float4 w[2];
};

template <int T>
__device__ __forceinline__ void embed_issue(const BlockArgs &a, int s, Emb &e) {
    const int nch = a.E / 8, k = 8 * ((int)threadIdx.x % nch);
    const int tok = min(max(a.tokens[s], 0), a.n_vocab - 1);
    const int p = min(max(a.pos[s], 0), a.n_ctx - 1);
    const uint8_t *blk = a.wte + (int64_t)tok * a.wte_nb + (int64_t)(k >> 5) * QT<T>::bytes;
    e.d = ld2(blk);
    ld8(blk + 2 + (T == T_Q4_0 ? (k & 15) : (k & 31)), e.q);
    const float *wp = a.wpe + (int64_t)p * a.E + k;
    e.w[0] = reinterpret_cast<const float4 *>(wp)[0];
    e.w[1] = reinterpret_cast<const float4 *>(wp)[1];
}

template <int T>
__device__ __forceinline__ void embed_finish(const BlockArgs &a, const Emb &e, float4 &x0, float4 &x1) {
    const int k = 8 * ((int)threadIdx.x % (a.E / 8));
    const float d = h2f((uint16_t)e.d);
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t byte = (e.q[i >> 2] >> (8 * (i & 3))) & 0xffu;
        const int q = T == T_Q4_0 ? (int)((k & 31) >= 16 ? byte >> 4 : byte & 0x0fu) - 8 : (int)(int8_t)byte;
        v[i] = __fmul_rn((float)q, d);
    }
    x0 = make_float4(v[0] + e.w[0].x, v[1] + e.w[0].y, v[2] + e.w[0].z, v[3] + e.w[0].w);
    x1 = make_float4(v[4] + e.w[1].x, v[5] + e.w[1].y, v[6] + e.w[1].z, v[7] + e.w[1].w);
    if (!resid_in(a)) x0 = x1 = make_float4(0.f, 0.f, 0.f, 0.f);
}

// LN of the register-resident residual (layer_norm_cols, shift = x[0] of the sequence) and its
// int8 quantization into `sm` (K = E). Ends with a workgroup barrier.
template <int T>
__device__ __forceinline__ void ln_quantize(const BlockArgs &a, float4 (&xa)[1][1], float4 (&xb)[1][1], const float4 (&g)[1][2],
                                            const float4 (&bb)[1][2], const XSmem &sm, float shift0) {
    const int kb0 = threadIdx.x >> 2;
    const float shift[1] = {shift0};
    MmArgs la{};
    la.K = a.E;
    la.ln_eps = a.eps;
    layer_norm_cols<1, 1>(la, kb0, xa, xb, g, bb, shift);
    if (kb0 < a.E / 32) xblock_store<T>(a.E, kb0, xa[0][0], xb[0][0], sm.xq, sm.xd, sm.xs, sm.x16);
    lds_barrier();
}

__device__ __forceinline__ void load_ln(const float *gp, const float *bp, int E, float4 (&g)[1][2], float4 (&bb)[1][2]) {
    const int k0 = min((int)(threadIdx.x >> 2) * 32 + (int)(threadIdx.x & 3) * 8, E - 8);
    // only the waves holding a thread t < E / 8 (the threads whose block kb0 = t / 4 exists)
    // load: the prologue's issue phase is paced by the CU's vector-memory instruction rate, so a
    // wave-instruction of clamped duplicates costs about what a useful one does (2 of 8 waves at
    // n_embd 768: attention block 9.07 -> 8.69 us, engine +1.7 %, profiles/r06_gpt2_prologue_ab.txt).
    // Skipping the duplicate residual slots, bias loads or q/k/v rows the same way measured slower
    // (branches between the residual and weight issues), and is not done.
    g[0][0] = g[0][1] = bb[0][0] = bb[0][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (__builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6) * WAVE >= E / 8) return;
    g[0][0] = reinterpret_cast<const float4 *>(gp + k0)[0];
    g[0][1] = reinterpret_cast<const float4 *>(gp + k0)[1];
    bb[0][0] = reinterpret_cast<const float4 *>(bp + k0)[0];
    bb[0][1] = reinterpret_cast<const float4 *>(bp + k0)[1];
}


// ------------------------------------------------------------------------------------------
// attention block: grid (n_head, n_seq)
// ------------------------------------------------------------------------------------------
constexpr int AGROUPS = NW * 4;            // 16-lane key groups per workgroup
constexpr int AU = 8;                      // keys per group in flight per round

template <int T, int QNIT, int RR, bool EMB = false>
__global__ __launch_bounds__(BT) void attn_block_kernel(const BlockArgs a) {
    __shared__ __align__(16) uint8_t lds_x[xs_bytes(E_MAX)];   // LN1(x), quantized
    __shared__ __align__(16) uint8_t lds_o[xs_bytes(E_MAX)];   // head h's attention output, quantized
    __shared__ __align__(16) float red[RED_FLOATS];            // residual row-group partials
    __shared__ __align__(16) float qkv_s[3 * HD];
    __shared__ __align__(16) float qb_s[3 * HD];
    __shared__ __align__(16) float go[AGROUPS][HD];
    __shared__ float gm[AGROUPS], gl[AGROUPS], gw_s[AGROUPS];
    __shared__ __align__(16) float o_s[HD];
    const int h = blockIdx.x, s = blockIdx.y, E = a.E;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const XSmem sx = xsmem(lds_x, E, 1), so = xsmem(lds_o, E, 1);
    stamp(a, 0, 0);

    // ---- issue: residual rows (layer 0 of a first stage: the token embedding), LN params, q/k/v
    // bias, position; then the qkv weight stream
    [[maybe_unused]] Resid<RR> R0;
    [[maybe_unused]] Emb em;
    if constexpr (EMB) embed_issue<T>(a, s, em);
    else resid_issue(a, s, 0, R0);
    float4 g[1][2], bb[1][2];
    load_ln(a.ln_g, a.ln_b, E, g, bb);
    const int vr_b = min(tid, 3 * HD - 1);
    const float qb = a.b_qkv[(vr_b >> 6) * E + h * HD + (vr_b & 63)];
    const int p = min(max(a.pos[s], 0), a.n_ctx - 1);
    RowsDot<T, 16, 6, QNIT> qd;
    qd.load([&](int vr) { return a.w_qkv + (int64_t)((vr >> 6) * E + h * HD + (vr & 63)) * a.nb_qkv; }, 3 * HD, 0, 0, E / 64);
    __builtin_amdgcn_sched_barrier(0);
    stamp(a, 0, 8);
    if (a.stamps != nullptr) {   // diagnostics: when this wave's first residual row has landed
        float probe = R0.v[0][0].x;
        asm volatile("" : "+v"(probe));
        if (probe == 1.2345e-30f) stamp(a, 0, 10);
        stamp(a, 0, 9);
    }

    if (tid < 3 * HD) qb_s[tid] = qb;
    for (int i = tid; i < xs_bytes(E) / 4; i += BT) reinterpret_cast<uint32_t *>(lds_o)[i] = 0u;   // c_proj K-split: zeros outside head h
    float4 xa[1][1], xb[1][1];
    float shift0;
    if constexpr (EMB) {
        embed_finish<T>(a, em, xa[0][0], xb[0][0]);
        if (tid == 0) red[0] = xa[0][0].x;
        lds_barrier();
        shift0 = red[0];
    } else {
        resid_finish(a, s, R0, red, xa[0][0], xb[0][0]);
        shift0 = resid_first(a, red);
    }
    stamp(a, 0, 1);
    if (h == 0) store_resid(a, s, xa[0][0], xb[0][0]);
    ln_quantize<T>(a, xa, xb, g, bb, sx, shift0);
    stamp(a, 0, 2);

    // ---- q, k, v of head h (+ bias)
    if (a.stamps != nullptr) {   // diagnostics: this wave's last q/k/v weight fragment has landed
        uint32_t probe = reinterpret_cast<const uint32_t *>(&qd.f[0][5])[0];
        asm volatile("" : "+v"(probe));
        if (probe == 0x12345u && threadIdx.x == 999) stamp(a, 0, 12);
        stamp(a, 0, 11);
    }
    qd.compute(sx, E, 3 * HD, [&](int vr, float v) { qkv_s[vr] = v + qb_s[vr]; });
    lds_barrier();
    stamp(a, 0, 3);

    // ---- the new token's K / V row of head h into the cache (the reference's ggml_cpy into
    // memory_k / memory_v, main-sched.cpp:648-655); attention reads key p from LDS
    float *K = a.kc + (int64_t)s * a.n_ctx * E + h * HD;
    float *Vc = a.vc + (int64_t)s * a.n_ctx * E + h * HD;
    if (tid < 16) reinterpret_cast<float4 *>(K + (int64_t)p * E)[tid] = reinterpret_cast<const float4 *>(qkv_s + HD)[tid];
    else if (tid < 32) reinterpret_cast<float4 *>(Vc + (int64_t)p * E)[tid - 16] = reinterpret_cast<const float4 *>(qkv_s + 2 * HD)[tid - 16];

    // ---- keys 0 .. p-1 (softmax(K.q * scale) . V, main-sched.cpp:685-735, in the rescaling
    // order of online softmax): a 16-lane group owns one key at a time, lane d4 the dims
    // 4 d4 .. 4 d4 + 3 (16-B coalesced row reads); 32 groups x AU keys in flight per round
    const int grp = wave * 4 + (lane >> 4), d4 = lane & 15;
    const int nk = p;
    const float4 q4 = reinterpret_cast<const float4 *>(qkv_s)[d4];
    float m = -INFINITY, l = 0.f;
    float4 o4 = make_float4(0.f, 0.f, 0.f, 0.f);
    // a wave issues only the key slots u that hold a key of one of its four groups (the wave's
    // first group is the lowest; no other load is in flight here, so the branch costs no wait):
    // at short contexts most of a round's AU slots lie past nk. Skipped slots read zeros (their
    // scores are -inf and their weights 0, so the values must be finite). Measured neutral
    // (profiles/r06_gpt2_prologue_ab.txt), kept with the layer-norm trim it was measured beside.
    const int wg0 = __builtin_amdgcn_readfirstlane(wave) * 4;
    for (int jb = 0; jb < nk; jb += AGROUPS * AU) {
        float4 kk[AU], vv[AU];
#pragma unroll
        for (int u = 0; u < AU; ++u) {
            const int jc = min(jb + u * AGROUPS + grp, nk - 1);
            kk[u] = vv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (jb + u * AGROUPS + wg0 < nk) {
                kk[u] = reinterpret_cast<const float4 *>(K + (int64_t)jc * E)[d4];
                vv[u] = reinterpret_cast<const float4 *>(Vc + (int64_t)jc * E)[d4];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        float sc[AU];
        float mn = m;
#pragma unroll
        for (int u = 0; u < AU; ++u) {
            float t = q4.x * kk[u].x + q4.y * kk[u].y + q4.z * kk[u].z + q4.w * kk[u].w;
            t += xchg<1>(t);
            t += xchg<2>(t);
            t += xchg<4>(t);
            t += xchg<8>(t);
            sc[u] = jb + u * AGROUPS + grp < nk ? t * a.scale : -INFINITY;
            mn = fmaxf(mn, sc[u]);
        }
        if (mn > -INFINITY) {   // uniform in the group
            const float cr = expf(m - mn);
            l *= cr;
            o4.x *= cr; o4.y *= cr; o4.z *= cr; o4.w *= cr;
#pragma unroll
            for (int u = 0; u < AU; ++u) {
                const float e = expf(sc[u] - mn);
                l += e;
                o4.x += e * vv[u].x; o4.y += e * vv[u].y; o4.z += e * vv[u].z; o4.w += e * vv[u].w;
            }
            m = mn;
        }
    }
    reinterpret_cast<float4 *>(go[grp])[d4] = o4;
    if (d4 == 0) { gm[grp] = m; gl[grp] = l; }

    // c_proj K-split weights: the slots holding head h's 64 columns (Q6_K: halves of two slots).
    // Q4_0 / Q8_0: the engine's head-major copy [head][row][one slot] (gpt2.cpp), a contiguous
    // stream; K-quants read the ggml rows in place
    constexpr int OLPR = T == T_Q6_K ? 2 : 1;
    const int os0 = T == T_Q6_K ? 4 * (h >> 2) + 2 * ((h & 3) >> 1) : h;
    const int ows0 = REPACK<T> ? 0 : -1;
    auto orow = [&](int r) {
        return REPACK<T> ? a.w_o + ((int64_t)h * E + r) * (2 * QT<T>::bytes) : a.w_o + (int64_t)r * a.nb_o;
    };
    RowsDot<T, OLPR, 2, 1> od0;
    od0.load(orow, E, 0, os0, OLPR, ows0);
    stamp(a, 0, 4);
    lds_barrier();

    // ---- merge the key groups and key p (wave 0: lane g < 32 scores group g, then lane d
    // owns o[d]); straight-line, every LDS read of a step issued together
    if (wave == 0) {
        const float sp = wave_sum(qkv_s[lane] * qkv_s[HD + lane]) * a.scale;
        const int g = lane & (AGROUPS - 1);
        const float gmv = gm[g], glv = gl[g];
        float mx = glv > 0.f ? gmv : -INFINITY;
        mx = fmaxf(mx, xchg<1>(mx)); mx = fmaxf(mx, xchg<2>(mx)); mx = fmaxf(mx, xchg<4>(mx));
        mx = fmaxf(mx, xchg<8>(mx)); mx = fmaxf(mx, xchg<16>(mx)); mx = fmaxf(mx, xchg<32>(mx));
        const float MX = fmaxf(mx, sp);
        const float wg = glv > 0.f ? expf(gmv - MX) : 0.f;
        const float ep = expf(sp - MX);
        const float L = wave_sum(lane < AGROUPS ? wg * glv : 0.f) + ep;
        if (lane < AGROUPS) gw_s[lane] = wg;
        float O = ep * qkv_s[2 * HD + lane];
#pragma unroll
        for (int w = 0; w < AGROUPS; ++w) O += gw_s[w] * go[w][lane];
        o_s[lane] = O / L;
        // quantize o (blocks 2h, 2h+1) in the same wave: its LDS accesses run in order
        if (lane < 8) {
            const int q0 = (lane >> 2) * 32 + (lane & 3) * 8;
            const float4 v0 = reinterpret_cast<const float4 *>(o_s + q0)[0];
            const float4 v1 = reinterpret_cast<const float4 *>(o_s + q0)[1];
            xblock_store<T>(E, 2 * h + (lane >> 2), v0, v1, so.xq, so.xd, so.xs, so.x16);
        }
    }
    lds_barrier();
    stamp(a, 0, 5);

    // ---- c_proj partial of head h: part_out[h][s][row]
    float *po = a.parts_out + ((int64_t)h * a.n_seq + s) * E;
    auto out = [&](int r, float v) { po[r] = v; };
    od0.compute(so, E, E, out);
    for (int base = RowsDot<T, OLPR, 2, 1>::RPP; base < E; base += RowsDot<T, OLPR, 2, 1>::RPP) {
        RowsDot<T, OLPR, 2, 1> odn;
        odn.load(orow, E, base, os0, OLPR, ows0);
        odn.compute(so, E, E, out);
    }
    stamp(a, 0, 6);
}

// ------------------------------------------------------------------------------------------
// MLP block: grid (4 n_embd / MLP_SLICE, n_seq)
// ------------------------------------------------------------------------------------------
template <int T, int FNIT, int RR>
__global__ __launch_bounds__(BT) void mlp_block_kernel(const BlockArgs a) {
    __shared__ __align__(16) uint8_t lds_x[xs_bytes(E_MAX)];       // LN2(y), quantized
    __shared__ __align__(16) uint8_t lds_h[xs_bytes(4 * E_MAX)];   // slice j of gelu(fc), quantized (K = 4E)
    __shared__ __align__(16) float red[RED_FLOATS];
    __shared__ __align__(16) float h_s[MLP_SLICE];
    __shared__ float fb_s[MLP_SLICE];
    const int j = blockIdx.x, s = blockIdx.y, E = a.E;
    const int tid = threadIdx.x;
    const XSmem sx = xsmem(lds_x, E, 1), sh = xsmem(lds_h, 4 * E, 1);
    stamp(a, 1, 0);
    stamp_clk(a, 1, 6);

    Resid<RR> R0;
    resid_issue(a, s, 0, R0);
    float4 g[1][2], bb[1][2];
    load_ln(a.ln_g, a.ln_b, E, g, bb);
    const float fb = a.b_fc[j * MLP_SLICE + min(tid, MLP_SLICE - 1)];
    // fc rows: n_embd 768 (FNIT 3): 4 lanes per row, 3 slots each, one row per lane (every lane
    // and every wave live: 8 waves x 16 rows = the slice's 128); otherwise (FNIT 1): 16 lanes per
    // row, one slot each, four rows per lane
    using FD = std::conditional_t<FNIT == 1, RowsDot<T, 16, MLP_SLICE / 32, 1>, RowsDot<T, 4, MLP_SLICE / 128, FNIT>>;
    FD fd;
    fd.load([&](int r) { return a.w_fc + (int64_t)(j * MLP_SLICE + r) * a.nb_fc; }, MLP_SLICE, 0, 0, E / 64);
    __builtin_amdgcn_sched_barrier(0);
    stamp(a, 1, 8);

    if (tid < MLP_SLICE) fb_s[tid] = fb;
    float4 xa[1][1], xb[1][1];
    resid_finish(a, s, R0, red, xa[0][0], xb[0][0]);
    stamp(a, 1, 1);
    if (j == 0) store_resid(a, s, xa[0][0], xb[0][0]);
    ln_quantize<T>(a, xa, xb, g, bb, sx, resid_first(a, red));
    stamp(a, 1, 2);

    if (a.stamps != nullptr) {   // diagnostics: this wave's fc weights have landed
        uint32_t probe = reinterpret_cast<const uint32_t *>(&fd.f[0][FNIT == 1 ? MLP_SLICE / 32 - 1 : 0])[0];
        asm volatile("" : "+v"(probe));
        if (probe == 0x12345u && threadIdx.x == 999) stamp(a, 1, 10);
        stamp(a, 1, 9);
    }
    fd.compute(sx, E, MLP_SLICE, [&](int r, float v) { h_s[r] = gelu_ggml(v + fb_s[r]); });
    stamp(a, 1, 11);

    // mlp proj K-split weights: slots [SL j, SL j + SL) of every row (the slice's columns); one
    // pass covers 8 waves x 32 x 3 = 768 rows
    constexpr int SL = MLP_SLICE / 64;
    using MD = RowsDot<T, SL, 3, 1>;
    MD md0;
    // Q4_0 / Q8_0: the engine's slice-major copy [slice][row][SL slots] (a contiguous stream)
    const int mws0 = REPACK<T> ? 0 : -1;
    auto mrow = [&](int r) {
        return REPACK<T> ? a.w_mp + ((int64_t)j * E + r) * (SL * 2 * QT<T>::bytes) : a.w_mp + (int64_t)r * a.nb_mp;
    };
    md0.load(mrow, E, 0, SL * j, SL, mws0);
    stamp(a, 1, 3);
    lds_barrier();
    if (tid < MLP_SLICE / 8) {
        const int q0 = (tid >> 2) * 32 + (tid & 3) * 8;
        const float4 v0 = reinterpret_cast<const float4 *>(h_s + q0)[0];
        const float4 v1 = reinterpret_cast<const float4 *>(h_s + q0)[1];
        xblock_store<T>(4 * E, j * (MLP_SLICE / 32) + (tid >> 2), v0, v1, sh.xq, sh.xd, sh.xs, sh.x16);
    }
    lds_barrier();

    stamp(a, 1, 4);
    float *po = a.parts_out + ((int64_t)j * a.n_seq + s) * E;
    auto out = [&](int r, float v) { po[r] = v; };
    md0.compute(sh, 4 * E, E, out);
    for (int base = MD::RPP; base < E; base += MD::RPP) {
        MD mdn;
        mdn.load(mrow, E, base, SL * j, SL, mws0);
        mdn.compute(sh, 4 * E, E, out);
    }
    stamp(a, 1, 5);
    stamp_clk(a, 1, 7);
}

// x_out = base + bias + sum parts (the residual leaving a stage): grid (n_seq)
template <int RR>
__global__ __launch_bounds__(BT) void resid_kernel(const BlockArgs a) {
    __shared__ __align__(16) float red[RED_FLOATS];
    Resid<RR> R0;
    resid_issue(a, blockIdx.x, 0, R0);
    float4 v0, v1;
    resid_finish(a, blockIdx.x, R0, red, v0, v1);
    store_resid(a, blockIdx.x, v0, v1);
}

// residual rows per thread of one issue round (3 covers GPT-2 117M: 14 rows over 5 row groups)
int resid_rr(const BlockArgs &a) {
    const int G = BT / (a.E / 8);
    return (1 + (a.bias_in != nullptr) + a.n_parts_in + G - 1) / G <= 3 ? 3 : RROWS;   // 117M: 26 rows -> 6
}

template <int T, int RR>
hipError_t launch_pair(bool attn, const BlockArgs &a, hipStream_t st) {
    if (attn && a.wte != nullptr) {
        if constexpr (REPACK<T>) hipLaunchKernelGGL((attn_block_kernel<T, 1, 3, true>), dim3(a.n_head, a.n_seq), dim3(BT), 0, st, a);
        else return hipErrorInvalidValue;
    } else if (attn) hipLaunchKernelGGL((attn_block_kernel<T, 1, RR>), dim3(a.n_head, a.n_seq), dim3(BT), 0, st, a);
    else {
        if constexpr (REPACK<T>) {
            if (a.E == 768) {
                hipLaunchKernelGGL((mlp_block_kernel<T, 3, RR>), dim3(4 * a.E / MLP_SLICE, a.n_seq), dim3(BT), 0, st, a);
                return hipGetLastError();
            }
        }
        hipLaunchKernelGGL((mlp_block_kernel<T, 1, RR>), dim3(4 * a.E / MLP_SLICE, a.n_seq), dim3(BT), 0, st, a);
    }
    return hipGetLastError();
}

template <int T>
hipError_t launch_type(bool attn, const BlockArgs &a, hipStream_t st) {
    return resid_rr(a) == 3 ? launch_pair<T, 3>(attn, a, st) : launch_pair<T, RROWS>(attn, a, st);
}

hipError_t launch_block(int type, bool attn, const BlockArgs &a, hipStream_t st) {
    switch (type) {
        case T_Q4_0: return launch_type<T_Q4_0>(attn, a, st);
        case T_Q8_0: return launch_type<T_Q8_0>(attn, a, st);
        case T_Q4_K: return launch_type<T_Q4_K>(attn, a, st);
        case T_Q5_K: return launch_type<T_Q5_K>(attn, a, st);
        case T_Q6_K: return launch_type<T_Q6_K>(attn, a, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

// shapes these kernels serve: 64-wide heads, n_embd <= E_MAX, whole 4 n_embd / 256 slices
bool gpt2_block_supported(int n_embd, int n_head) {
    if (n_embd != HD * n_head || n_embd > E_MAX || n_embd % 64 != 0 || (4 * n_embd) % MLP_SLICE != 0) return false;
    const int G = BT / (n_embd / 8);
    // one issue round of the residual prologue: base + bias + the larger partial count
    return G * n_embd <= RED_FLOATS && 2 + std::max(n_head, 4 * n_embd / MLP_SLICE) <= G * RROWS;
}

int gpt2_block_mlp_slices(int n_embd) { return 4 * n_embd / MLP_SLICE; }

// layer 0 of a first stage can take the token embedding in its prologue (32-block types)
bool gpt2_block_embeds(int type) { return REPACK_TYPE(type); }

// head-major c_proj ([head][row][2 blocks]) and slice-major MLP projection
// ([slice][row][MLP_SLICE / 32 blocks]) copies of one layer, for the 32-block types; bytes of
// each through *_bytes (dst == nullptr: sizes only)
bool gpt2_block_repacks(int type) { return type == T_Q4_0 || type == T_Q8_0; }

hipError_t gpt2_block_repack(int type, int E, const uint8_t *w_o, uint8_t *o_dst, const uint8_t *w_mp, uint8_t *mp_dst,
                             size_t *o_bytes, size_t *mp_bytes, hipStream_t st) {
    const int bs = type == T_Q4_0 ? QT<T_Q4_0>::bytes : QT<T_Q8_0>::bytes;
    const size_t wo = 2 * (size_t)bs, wm = (MLP_SLICE / 32) * (size_t)bs;     // bytes of one row's K-split
    const size_t ro = (size_t)E / 32 * bs, rm = (size_t)4 * E / 32 * bs;     // ggml row bytes
    if (o_bytes) *o_bytes = wo * E * (E / HD);
    if (mp_bytes) *mp_bytes = wm * E * (4 * E / MLP_SLICE);
    if (!o_dst) return hipSuccess;
    for (int h = 0; h < E / HD; ++h) {
        const hipError_t e = hipMemcpy2DAsync(o_dst + h * wo * E, wo, w_o + h * wo, ro, wo, E, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return e;
    }
    for (int j = 0; j < 4 * E / MLP_SLICE; ++j) {
        const hipError_t e = hipMemcpy2DAsync(mp_dst + j * wm * E, wm, w_mp + j * wm, rm, wm, E, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t gpt2_attn_block_launch(int layer, int type, const float *base, const float *bias_in, const float *parts_in, int n_parts_in,
                                  float *x_out, const float *ln_g, const float *ln_b, float eps, const uint8_t *w_qkv,
                                  int64_t nb_qkv, const float *b_qkv, float *kc, float *vc, const int32_t *pos, float scale,
                                  int n_ctx, const uint8_t *w_o, int64_t nb_o, float *parts_out, int E, int n_head, int n_seq,
                                  const uint8_t *wte, int64_t wte_nb, const float *wpe, const int32_t *tokens, int n_vocab,
                                  hipStream_t st) {
    if (!gpt2_block_supported(E, n_head)) return hipErrorInvalidValue;
    BlockArgs a{};
    a.base = base; a.bias_in = bias_in; a.parts_in = parts_in; a.n_parts_in = parts_in ? n_parts_in : 0;
    a.x_out = x_out; a.ln_g = ln_g; a.ln_b = ln_b; a.eps = eps;
    a.w_qkv = w_qkv; a.nb_qkv = nb_qkv; a.b_qkv = b_qkv; a.kc = kc; a.vc = vc; a.pos = pos; a.scale = scale; a.n_ctx = n_ctx;
    a.w_o = w_o; a.nb_o = nb_o; a.parts_out = parts_out;
    a.E = E; a.n_head = n_head; a.n_seq = n_seq;
    a.layer = layer; a.stamps = stamps_buffer();
    a.wte = wte; a.wte_nb = wte_nb; a.wpe = wpe; a.tokens = tokens; a.n_vocab = n_vocab;
    return launch_block(type, true, a, st);
}

hipError_t gpt2_mlp_block_launch(int layer, int type, const float *base, const float *bias_in, const float *parts_in, int n_parts_in,
                                 float *x_out, const float *ln_g, const float *ln_b, float eps, const uint8_t *w_fc,
                                 int64_t nb_fc, const float *b_fc, const uint8_t *w_mp, int64_t nb_mp, float *parts_out, int E,
                                 int n_head, int n_seq, hipStream_t st) {
    if (!gpt2_block_supported(E, n_head)) return hipErrorInvalidValue;
    BlockArgs a{};
    a.base = base; a.bias_in = bias_in; a.parts_in = parts_in; a.n_parts_in = parts_in ? n_parts_in : 0;
    a.x_out = x_out; a.ln_g = ln_g; a.ln_b = ln_b; a.eps = eps;
    a.w_fc = w_fc; a.nb_fc = nb_fc; a.b_fc = b_fc; a.w_mp = w_mp; a.nb_mp = nb_mp; a.parts_out = parts_out;
    a.E = E; a.n_head = n_head; a.n_seq = n_seq;
    a.layer = layer; a.stamps = stamps_buffer();
    return launch_block(type, false, a, st);
}

hipError_t gpt2_resid_launch(const float *base, const float *bias_in, const float *parts_in, int n_parts_in, float *x_out, int E,
                             int n_seq, hipStream_t st) {
    if (E % 8 != 0 || E / 8 > BT || (BT / (E / 8)) * E > RED_FLOATS) return hipErrorInvalidValue;
    if (1 + (bias_in != nullptr) + (parts_in ? n_parts_in : 0) > (BT / (E / 8)) * RROWS) return hipErrorInvalidValue;
    BlockArgs a{};
    a.base = base; a.bias_in = bias_in; a.parts_in = parts_in; a.n_parts_in = parts_in ? n_parts_in : 0;
    a.x_out = x_out; a.E = E; a.n_seq = n_seq;
    if (resid_rr(a) == 3) hipLaunchKernelGGL(resid_kernel<3>, dim3(n_seq), dim3(BT), 0, st, a);
    else hipLaunchKernelGGL(resid_kernel<RROWS>, dim3(n_seq), dim3(BT), 0, st, a);
    return hipGetLastError();
}

}  // namespace mi355x
