// mmvq_ring.hip — the quantized mat-vec for several columns at any K: one pass over the weights
// for up to 8 src1 columns, as the reference's mul_mat_vec_q<type, ncols_dst> streams them once
// for ncols_dst = 1..8 (src/ggml-cuda/mmvq.cu:139-226, tables :85-137).
//
// The plain mat-vec (mmvq_impl.h) quantizes a column group's whole K into LDS once per workgroup
// and then walks its rows. That holds NC x K x 1.5 B of LDS and NC x 8 x (K / 4096) activation
// registers per lane, so wide column groups at large K (the reference's perf shapes, K = 14336,
// bs 2..8; LLaMA's FFN-down) had to be split into several passes over the weights. Here K runs
// in chunks of 4096 (64 slots of 64 weights = one K iteration of a 64-lane row):
//
//  * LDS holds a ring of two chunk images (NC x 6 KiB each, the layout of mmvq_impl.h's XSmem
//    with Kpad = 4096); unit (row group g, chunk it) reads ring slot (unit count & 1);
//  * per unit, the f32 activations of the NEXT unit's chunk are issued first, then its weights,
//    then this unit's dot products run out of LDS; the next chunk is quantized into the other
//    ring slot once this unit is done (the activation loads were issued first, so waiting for
//    them does not wait for the weights: vmcnt retires in order), and one barrier per unit
//    hands it over. The quantization is the same xblock_store as the plain kernel's, so the
//    results are bit-identical to it at any K;
//  * columns past the launch's live count (M not a multiple of NC) re-read the last live column
//    and store nothing.
#include <type_traits>

#include "mmvq_impl.h"
#include "settings.h"

#include <string>

namespace mi355x {

constexpr int RING_K = 4096;                   // K per chunk
constexpr int RING_XBLK = RING_K / 32;         // 32-blocks per chunk (= XR_STRIDE: one per lane quad)
static_assert(RING_XBLK == XR_STRIDE, "one 32-block per lane quad and chunk");

__host__ __device__ constexpr int ring_slot_bytes(int nc) { return nc * RING_K + 4 * nc * (RING_K / 32) * 4; }

typedef __attribute__((address_space(3))) void *lds_ptr_t;

// PRE: the column group's activations were quantized once per call by mmvq_prequant into the
// ring-slot image of every chunk, [batch][chunk][slot image of NC columns] in global memory; the
// kernel copies chunk images into the ring by LDS-DMA (buffer_load ... lds: no VGPRs, no
// quantization in the workgroup). Without PRE every workgroup quantizes every chunk of its
// column group from f32 (NC x 4 B per K per workgroup read from L2), which costs more than the
// weight stream itself from 4 columns on (profiles/r05_tbo_perf_mul_mat.txt).
template <int T, bool XA, int NC>
__global__ __launch_bounds__(512) void mmvq_prequant(const MmArgs a, uint8_t *__restrict__ img) {
    // grid (chunk, column, batch); lane quad q quantizes the chunk's 32-block q
    const int c = blockIdx.x, m = blockIdx.y, z = blockIdx.z;
    const int i12 = z % a.ne12, i13 = z / a.ne12;
    const int kbl = threadIdx.x >> 2;
    const uint8_t *col = a.x + (int64_t)i12 * a.nb12 + (int64_t)i13 * a.nb13 + (int64_t)min(m, a.M - 1) * a.nb11;
    float4 v0, v1;
    xblock_load<XA>(a, col, c * RING_XBLK + kbl, v0, v1);
    xblock_mask(a, m < a.M ? c * RING_XBLK + kbl : (1 << 29), v0, v1);   // (columns past M: zeros)
    const XSmem sm = xsmem(img + ((int64_t)z * a.n_it + c) * ring_slot_bytes(NC), RING_K, NC);
    xblock_store<T>(RING_K, kbl, v0, v1, sm.xq + (size_t)m * RING_K, sm.xd + m * RING_XBLK, sm.xs + m * RING_XBLK,
                    sm.x16 + m * 2 * RING_XBLK);
}

// WAVES = 8 or 16 per workgroup: with 16, a row group has twice the rows for the same LDS ring
// and each lane quad quantizes half of the columns (8 columns: 32 activation registers instead of
// 64), so a 8-column kernel keeps one row per wave and no spills
template <int T, int NC, int RPW, bool RAG, bool XA, int WAVES>
__global__ __launch_bounds__(WAVES * WAVE) void mmvq_ring_kernel(const MmArgs a) {
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr int LPR = 64;
    constexpr int NX = XdCount<T>::n;
    constexpr int V = pow2ceil(RPW * NC);
    constexpr int ROWS_PER_GROUP = WAVES * RPW;
    constexpr int SLOT = ring_slot_bytes(NC);
    constexpr int CSETS = WAVES / 8;               // column sets: lane quads per (chunk block, column)
    constexpr int NCQ = (NC + CSETS - 1) / CSETS;  // columns quantized by one lane quad
    static_assert(V <= LPR, "RPW * NC partial sums must fit the lanes of a row");
    static_assert(NC % CSETS == 0, "column sets split the columns evenly");

    const int Kpad = (a.K + 63) & ~63;
    const int nslots = Kpad / 64;
    const int nblk = a.K / QT<T>::blck;
    const int n_it = a.n_it;                       // host: chunks = ceil(nslots / 64)

    const int i12 = blockIdx.y % a.ne12, i13 = blockIdx.y / a.ne12;
    const uint8_t *wmat = a.w + (int64_t)(i12 / a.r2) * a.nb02 + (int64_t)(i13 / a.r3) * a.nb03;
    const int c0 = (int)blockIdx.z * NC;
    const int ncl = min(NC, a.M - c0);             // live columns of this workgroup
    const uint8_t *xcol0 = a.x + (int64_t)i12 * a.nb12 + (int64_t)i13 * a.nb13 + (int64_t)c0 * a.nb11;
    uint8_t *dcol0 = a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3 + (int64_t)c0 * a.nb1;

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int wrow = wave * RPW;
    const int n_groups = (a.N + ROWS_PER_GROUP - 1) / ROWS_PER_GROUP;
    const int kbl = (threadIdx.x >> 2) % RING_XBLK;   // this lane quad's 32-block inside a chunk
    const int cq0 = (threadIdx.x >> 2) / RING_XBLK * NCQ;   // and its first column

    float4 xa[NCQ], xb[NCQ];
    auto load_x = [&](int it) {
#pragma unroll
        for (int i = 0; i < NCQ; ++i)
            xblock_load<XA>(a, xcol0 + (int64_t)min(cq0 + i, ncl - 1) * a.nb11, it * RING_XBLK + kbl, xa[i], xb[i]);
    };
    // (the ring slot is a compile-time constant at every call, so LDS addresses fold into
    // instruction offsets instead of per-column address registers)
    auto store_x = [&](int it, auto slot_c) {
        const XSmem sm = xsmem(smem + decltype(slot_c)::value * SLOT, RING_K, NC);
#pragma unroll
        for (int i = 0; i < NCQ; ++i) {
            const int m = cq0 + i;
            xblock_mask(a, it * RING_XBLK + kbl, xa[i], xb[i]);
            xblock_store<T>(RING_K, kbl, xa[i], xb[i], sm.xq + (size_t)m * RING_K, sm.xd + m * RING_XBLK,
                            sm.xs + m * RING_XBLK, sm.x16 + m * 2 * RING_XBLK);
        }
    };
    // unit (g, it): rows g * ROWS_PER_GROUP + wrow + r, slot lane + 64 it (clamped: dead lanes
    // and rows read valid memory and are masked out of the sums)
    auto load_unit = [&](Frag<T> (&f)[RPW], int g, int it) {
        const int r0 = g * ROWS_PER_GROUP + wrow;
        const int s = min(lane + it * LPR, nslots - 1);
#pragma unroll
        for (int r = 0; r < RPW; ++r) f[r].template load<RAG>(wmat + (int64_t)min(r0 + r, a.N - 1) * a.nb01, s, nblk);
    };

    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;

    auto compute_unit = [&](const Frag<T> (&f)[RPW], int gg, int itt, auto slot_c) {
        const float live = lane + itt * LPR < nslots ? 1.f : 0.f;
        const int s = lane;                        // the slot inside the chunk
        int xb0, x16b;
        if constexpr (T == T_Q6_K) {
            xb0 = 8 * (s >> 2) + 4 * ((s >> 1) & 1);
            x16b = 16 * (s >> 2) + 8 * ((s >> 1) & 1) + (s & 1);
        } else {
            xb0 = 2 * s;
            x16b = 0;
        }
        const XSmem sm = xsmem(smem + decltype(slot_c)::value * SLOT, RING_K, NC);
#pragma unroll
        for (int m = 0; m < NC; ++m) {
            if (m >= ncl) continue;                // (uniform; a `break` here doubles the registers)
            uint32_t X[16];
            const int8_t *xm = sm.xq + (size_t)m * RING_K;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint4 t4 = *reinterpret_cast<const uint4 *>(xm + (size_t)(j * 64 + s) * 16);
                X[4 * j + 0] = t4.x; X[4 * j + 1] = t4.y; X[4 * j + 2] = t4.z; X[4 * j + 3] = t4.w;
            }
            float dx[NX], sx[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) dx[i] = sm.xd[m * RING_XBLK + xb0 + i];
            if constexpr (T == T_Q6_K) {
#pragma unroll
                for (int i = 0; i < NX; ++i) sx[i] = sm.x16[m * 2 * RING_XBLK + x16b + 2 * i];
            } else {
#pragma unroll
                for (int i = 0; i < NX; ++i) sx[i] = sm.xs[m * RING_XBLK + xb0 + i];
            }
#pragma unroll
            for (int r = 0; r < RPW; ++r) acc[r * NC + m] += live * f[r].dot(X, dx, sx);
        }
        if (itt == n_it - 1) {                     // the row group's last chunk: reduce, store
            const float sum = group_reduce_transpose<V, LPR>(acc);
            constexpr int SHIFT = Log2<LPR>::v - Log2<V>::v;
            const int idx = lane >> SHIFT;
            const int r0 = gg * ROWS_PER_GROUP + wrow;
            if ((lane & ((1 << SHIFT) - 1)) == 0 && idx < RPW * NC) {
                const int r = idx / NC, m = idx % NC;
                if (r0 + r < a.N && m < ncl) reinterpret_cast<float *>(dcol0 + (int64_t)m * a.nb1)[r0 + r] = sum;
            }
#pragma unroll
            for (int i = 0; i < V; ++i) acc[i] = 0.f;
        }
    };

    // prologue: chunk 0's activations first, then unit 0's weights; quantize; hand over
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    Frag<T> fa[RPW], fb[RPW];
    int g = blockIdx.x, it = 0;                    // the unit being computed (grid.x <= n_groups)
    load_x(it);
    load_unit(fa, g, it);
    __builtin_amdgcn_sched_barrier(0);
    store_x(it, S0{});
    lds_barrier();

    int ng = g, nit = it + 1;
    if (nit == n_it) { nit = 0; ng += gridDim.x; }
    // every load is unconditional (past the last unit: the current unit again, an on-chip
    // repeat) so the load stream never sits under a branch; each unit: next activations, next
    // weights, this unit's dots, quantize the next chunk into the other slot, one barrier.
    // Units alternate (fa, slot 0) and (fb, slot 1).
    for (;;) {
        bool more = ng < n_groups;
        load_x(more ? nit : it);
        load_unit(fb, more ? ng : g, more ? nit : it);
        __builtin_amdgcn_sched_barrier(0);
        compute_unit(fa, g, it, S0{});
        if (!more) break;
        store_x(nit, S1{});
        lds_barrier();
        g = ng; it = nit;
        if (++nit == n_it) { nit = 0; ng += gridDim.x; }
        more = ng < n_groups;
        load_x(more ? nit : it);
        load_unit(fa, more ? ng : g, more ? nit : it);
        __builtin_amdgcn_sched_barrier(0);
        compute_unit(fb, g, it, S1{});
        if (!more) break;
        store_x(nit, S0{});
        lds_barrier();
        g = ng; it = nit;
        if (++nit == n_it) { nit = 0; ng += gridDim.x; }
    }
}

// The pre-quantized form (PRE): CW compute waves and one loader wave. The loader copies chunk
// images from the mmvq_prequant output into the LDS ring by LDS-DMA, one unit ahead, and waits
// for its own copies (vmcnt is per wave) before each hand-off barrier; the compute waves issue
// only weight loads, so no wait of theirs ever covers a DMA (a wave that issues LDS-DMA gets a
// compiler wait for all of it before its next LDS read, which would drain the weight prefetch).
// Both walk the same unit sequence and meet at the same barriers.
template <int T, int NC, int RPW, bool RAG, int CW, int DEPTH>
__global__ __launch_bounds__((CW + 1) * WAVE) void mmvq_ring_pre_kernel(const MmArgs a, const uint8_t *__restrict__ img) {
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr int LPR = 64;
    constexpr int NX = XdCount<T>::n;
    constexpr int V = pow2ceil(RPW * NC);
    constexpr int ROWS_PER_GROUP = CW * RPW;
    constexpr int SLOT = ring_slot_bytes(NC);
    static_assert(SLOT % 1024 == 0, "whole 1-KiB pieces");
    static_assert(V <= LPR, "RPW * NC partial sums must fit the lanes of a row");
    static_assert(DEPTH == 2 || DEPTH == 3, "weight sets in flight");

    const int Kpad = (a.K + 63) & ~63;
    const int nslots = Kpad / 64;
    const int nblk = a.K / QT<T>::blck;
    const int n_it = a.n_it;
    const int i12 = blockIdx.y % a.ne12, i13 = blockIdx.y / a.ne12;
    const int ncl = min(NC, a.M);
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int n_groups = (a.N + ROWS_PER_GROUP - 1) / ROWS_PER_GROUP;

    if (wave == CW) {   // ---- loader: chunk images into the ring, one unit ahead
        const __amdgpu_buffer_rsrc_t xr =
            __builtin_amdgcn_make_buffer_rsrc((void *)(img + (int64_t)blockIdx.y * n_it * SLOT), 0, (uint32_t)(n_it * SLOT), 0x00020000);
        auto dma = [&](int it, int slot) {
            uint8_t *dst = smem + slot * SLOT;
#pragma unroll
            for (int p = 0; p < SLOT / 1024; ++p)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_ptr_t)(dst + p * 1024), 16, (uint32_t)(it * SLOT + p * 1024 + lane * 16),
                                                         0, 0, 0);
            __builtin_amdgcn_s_waitcnt(0x3f70);   // vmcnt(0): this wave's copies have landed
        };
        int g = blockIdx.x, it = 0, slot = 0;
        dma(it, slot);
        lds_barrier();
        for (;;) {
            if (++it == n_it) { it = 0; g += gridDim.x; }
            if (g >= n_groups) break;
            slot ^= 1;
            dma(it, slot);
            lds_barrier();
        }
        return;
    }

    // ---- compute waves
    const uint8_t *wmat = a.w + (int64_t)(i12 / a.r2) * a.nb02 + (int64_t)(i13 / a.r3) * a.nb03;
    uint8_t *dcol0 = a.dst + (int64_t)i12 * a.nb2 + (int64_t)i13 * a.nb3;
    const int wrow = wave * RPW;
    auto load_unit = [&](Frag<T> (&f)[RPW], int g, int it) __attribute__((always_inline)) {
        const int r0 = g * ROWS_PER_GROUP + wrow;
        const int s = min(lane + it * LPR, nslots - 1);
#pragma unroll
        for (int r = 0; r < RPW; ++r) f[r].template load<RAG>(wmat + (int64_t)min(r0 + r, a.N - 1) * a.nb01, s, nblk);
    };
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    auto compute_unit = [&](const Frag<T> (&f)[RPW], int gg, int itt, auto slot_c) __attribute__((always_inline)) {
        const float live = lane + itt * LPR < nslots ? 1.f : 0.f;
        const int s = lane;
        int xb0, x16b;
        if constexpr (T == T_Q6_K) {
            xb0 = 8 * (s >> 2) + 4 * ((s >> 1) & 1);
            x16b = 16 * (s >> 2) + 8 * ((s >> 1) & 1) + (s & 1);
        } else {
            xb0 = 2 * s;
            x16b = 0;
        }
        const XSmem sm = xsmem(smem + decltype(slot_c)::value * SLOT, RING_K, NC);
#pragma unroll
        for (int m = 0; m < NC; ++m) {
            if (m >= ncl) continue;                // (uniform)
            uint32_t X[16];
            const int8_t *xm = sm.xq + (size_t)m * RING_K;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint4 t4 = *reinterpret_cast<const uint4 *>(xm + (size_t)(j * 64 + s) * 16);
                X[4 * j + 0] = t4.x; X[4 * j + 1] = t4.y; X[4 * j + 2] = t4.z; X[4 * j + 3] = t4.w;
            }
            float dx[NX], sx[NX];
#pragma unroll
            for (int i = 0; i < NX; ++i) dx[i] = sm.xd[m * RING_XBLK + xb0 + i];
            if constexpr (T == T_Q6_K) {
#pragma unroll
                for (int i = 0; i < NX; ++i) sx[i] = sm.x16[m * 2 * RING_XBLK + x16b + 2 * i];
            } else {
#pragma unroll
                for (int i = 0; i < NX; ++i) sx[i] = sm.xs[m * RING_XBLK + xb0 + i];
            }
#pragma unroll
            for (int r = 0; r < RPW; ++r) acc[r * NC + m] += live * f[r].dot(X, dx, sx);
        }
        if (itt == n_it - 1) {
            const float sum = group_reduce_transpose<V, LPR>(acc);
            constexpr int SHIFT = Log2<LPR>::v - Log2<V>::v;
            const int idx = lane >> SHIFT;
            const int r0 = gg * ROWS_PER_GROUP + wrow;
            if ((lane & ((1 << SHIFT) - 1)) == 0 && idx < RPW * NC) {
                const int r = idx / NC, m = idx % NC;
                if (r0 + r < a.N && m < ncl) reinterpret_cast<float *>(dcol0 + (int64_t)m * a.nb1)[r0 + r] = sum;
            }
#pragma unroll
            for (int i = 0; i < V; ++i) acc[i] = 0.f;
        }
    };
    // weights DEPTH - 1 units ahead: unit u computes from F[u % DEPTH] out of ring slot u % 2 and
    // issues the loads of unit u + DEPTH - 1 into the set unit u - 1 used (past the last unit
    // the last one again: an on-chip repeat, so no load sits under a branch). One unit in flight
    // (DEPTH 2) leaves a CU's weight stream idle for a memory latency per unit, since a unit is
    // only ~4 K cycles of the CU's HBM share; DEPTH 3 keeps the next two in flight.
    struct Cur {
        int g, it;
    };
    auto adv = [&](Cur c) __attribute__((always_inline)) {
        if (++c.it == n_it) { c.it = 0; c.g += gridDim.x; }
        return c;
    };
    Frag<T> F[DEPTH][RPW];
    Cur cur{(int)blockIdx.x, 0}, ld = cur;
    load_unit(F[0], ld.g, ld.it);
#pragma unroll
    for (int d = 1; d < DEPTH - 1; ++d) {
        const Cur n = adv(ld);
        if (n.g < n_groups) ld = n;
        load_unit(F[d], ld.g, ld.it);
    }
    lds_barrier();                                 // chunk 0 is in slot 0
    constexpr int L = DEPTH * 2 / (DEPTH % 2 == 0 ? 2 : 1);   // lcm(DEPTH, 2): sets and slots constant
    auto step = [&](auto k_c) __attribute__((always_inline)) -> bool {   // true: that was this workgroup's last unit
        constexpr int K = decltype(k_c)::value;
        {
            const Cur n = adv(ld);
            if (n.g < n_groups) ld = n;
        }
        load_unit(F[(K + DEPTH - 1) % DEPTH], ld.g, ld.it);
        __builtin_amdgcn_sched_barrier(0);
        compute_unit(F[K % DEPTH], cur.g, cur.it, std::integral_constant<int, K % 2>{});
        const Cur n = adv(cur);
        if (n.g >= n_groups) return true;
        lds_barrier();                             // the next chunk is in the other slot; this one is free
        cur = n;
        return false;
    };
    for (;;) {
        if (step(std::integral_constant<int, 0>{})) break;
        if (step(std::integral_constant<int, 1>{})) break;
        if constexpr (L > 2) {
            if (step(std::integral_constant<int, 2 % L>{})) break;
            if (step(std::integral_constant<int, 3 % L>{})) break;
            if (step(std::integral_constant<int, 4 % L>{})) break;
            if (step(std::integral_constant<int, 5 % L>{})) break;
        }
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
size_t mmvq_ring_lds_bytes(int nc) { return 2 * (size_t)ring_slot_bytes(nc); }

template <int T, int NC, int RPW>
constexpr int pre_depth() {
    return RPW == 2 && (T == T_Q8_0 || T == T_Q5_K || T == T_Q6_K || (T == T_Q4_K && NC == 8)) ? 2 : 3;
}

template <int T, int NC, int RPW, bool RAG, bool XA, bool PRE>
static hipError_t ring_one(const MmArgs &a0, uint8_t *img, hipStream_t st) {
    constexpr int WAVES = (NC >= 8 && !PRE) ? 16 : 8;   // PRE: 8 compute waves + the loader
    constexpr int THREADS = PRE ? (WAVES + 1) * WAVE : WAVES * WAVE;
    const size_t lds = mmvq_ring_lds_bytes(NC);
    // PRE: weight sets in flight per wave (mmvq_ring_pre_kernel): 3 where they fit the registers
    // without spills (two rows of Q8_0 / Q5_K, or of Q4_K at 8 columns, do not: 2 there), unless
    // GGML_MI355X_RING_DEPTH=2
    constexpr int D = pre_depth<T, NC, RPW>();
    const bool d3 = D == 3 && settings().ring_depth != 2;
    const void *kern;
    if constexpr (PRE)
        kern = d3 ? reinterpret_cast<const void *>(mmvq_ring_pre_kernel<T, NC, RPW, RAG, WAVES, D>)
                  : reinterpret_cast<const void *>(mmvq_ring_pre_kernel<T, NC, RPW, RAG, WAVES, 2>);
    else kern = reinterpret_cast<const void *>(mmvq_ring_kernel<T, NC, RPW, RAG, XA, WAVES>);
    static LdsAttr attr[2];   // per instantiation, depth and device; set once the call succeeded
    if (lds > 64 * 1024)
        if (const hipError_t e = lds_attr_once(kern, attr[d3]); e != hipSuccess) return e;
    MmArgs a = a0;
    const int nslots = ((a.K + 63) & ~63) / 64;
    a.n_it = (nslots + 63) / 64;
    const int rows_per_group = WAVES * RPW;
    const int n_groups = (a.N + rows_per_group - 1) / rows_per_group;
    const int grid_y = a.ne12 * a.ne13, grid_z = (a.M + NC - 1) / NC;
    // one round of resident workgroups (LDS-bound: 160 KiB / ring; at most 32 waves per CU);
    // more workgroups would re-quantize (or re-copy) the same chunks for fewer rows each
    const int per_cu = std::max(1, std::min(32 / (THREADS / WAVE), (int)(160 * 1024 / (lds + 1024))));
    const int64_t target_env = settings().ring_wgs;
    const int64_t target = target_env > 0 ? target_env : 256 * per_cu;
    const int want = (int)std::max<int64_t>(1, target / ((int64_t)grid_y * grid_z));
    const dim3 grid(std::min(n_groups, want), grid_y, grid_z);
    if constexpr (PRE) {   // one column group per launch (grid_z == 1): quantized once, then the mat-vec
        if (!(settings().diag & 256)) hipLaunchKernelGGL((mmvq_prequant<T, XA, NC>), dim3(a.n_it, NC, grid_y), dim3(512), 0, st, a, img);
        if (d3) hipLaunchKernelGGL((mmvq_ring_pre_kernel<T, NC, RPW, RAG, WAVES, D>), grid, dim3(THREADS), lds, st, a, (const uint8_t *)img);
        else hipLaunchKernelGGL((mmvq_ring_pre_kernel<T, NC, RPW, RAG, WAVES, 2>), grid, dim3(THREADS), lds, st, a, (const uint8_t *)img);
    } else {
        hipLaunchKernelGGL((mmvq_ring_kernel<T, NC, RPW, RAG, XA, WAVES>), grid, dim3(THREADS), lds, st, a);
    }
    return hipGetLastError();
}

template <int T, int NC, int RPW, bool PRE>
static hipError_t ring_flags(const MmArgs &a, uint8_t *img, hipStream_t st) {
    if constexpr (T == T_Q4_0 || T == T_Q8_0) {
        if (a.K % 64 != 0)
            return a.x_aligned16 ? ring_one<T, NC, RPW, true, true, PRE>(a, img, st) : ring_one<T, NC, RPW, true, false, PRE>(a, img, st);
    }
    return a.x_aligned16 ? ring_one<T, NC, RPW, false, true, PRE>(a, img, st) : ring_one<T, NC, RPW, false, false, PRE>(a, img, st);
}

template <int T>
static hipError_t ring_type(const MmArgs &a, int nc, int rpw, uint8_t *img, hipStream_t st) {
    if (img != nullptr) {   // pre-quantized column groups of 2, 4 and 8 (8 compute waves)
        // two rows per wave where the fragments fit (Q5_K / Q6_K spill with two at 4 columns)
        if constexpr (T != T_Q5_K && T != T_Q6_K) {
            if (rpw > 1) {
                if (nc == 2) return ring_flags<T, 2, 2, true>(a, img, st);
                if (nc == 4) return ring_flags<T, 4, 2, true>(a, img, st);
                if (nc == 8) return ring_flags<T, 8, 2, true>(a, img, st);
                return hipErrorInvalidValue;
            }
        }
        if (nc == 2) return ring_flags<T, 2, 1, true>(a, img, st);
        if (nc == 4) return ring_flags<T, 4, 1, true>(a, img, st);
        if (nc == 8) return ring_flags<T, 8, 1, true>(a, img, st);
        return hipErrorInvalidValue;
    }
    // 8 columns: 16 waves of one row each (see the kernel); Q6_K one row per wave throughout
    if (nc == 8) return ring_flags<T, 8, 1, false>(a, nullptr, st);
    if (rpw <= 1 || T == T_Q6_K) {
        switch (nc) {
            case 1: return ring_flags<T, 1, 1, false>(a, nullptr, st);
            case 2: return ring_flags<T, 2, 1, false>(a, nullptr, st);
            case 4: return ring_flags<T, 4, 1, false>(a, nullptr, st);
            default: return hipErrorInvalidValue;
        }
    }
    switch (nc) {
        case 1: return ring_flags<T, 1, 2, false>(a, nullptr, st);
        case 2: return ring_flags<T, 2, 2, false>(a, nullptr, st);
        case 4: return ring_flags<T, 4, 2, false>(a, nullptr, st);
        default: return hipErrorInvalidValue;
    }
}

// the kernel ring_type picks (the dispatch description, ggml_mi355x_mul_mat_plan)
std::string mmvq_ring_plan_text(int type, const MmArgs &a, int nc, int rpw, bool pre) {
    int r;
    if (pre) r = (type != T_Q5_K && type != T_Q6_K && rpw > 1) ? 2 : 1;
    else r = (nc == 8 || rpw <= 1 || type == T_Q6_K) ? 1 : 2;
    return std::string(pre ? "ring-pre" : "ring") + " nc=" + std::to_string(nc) + " rpw=" + std::to_string(r) +
           " cols=" + std::to_string(a.M);
}

// bytes of the pre-quantized image of one nc-column group (prequant path)
size_t mmvq_ring_img_bytes(const MmArgs &a, int nc) {
    const int nslots = ((a.K + 63) & ~63) / 64;
    return (size_t)((nslots + 63) / 64) * ring_slot_bytes(nc) * a.ne12 * a.ne13;
}

// plain MUL_MAT, a.M columns (1..8 per column group of nc in {1, 2, 4, 8}; the last group may be
// partial): grid.z = ceil(M / nc). img != nullptr (nc 4 / 8, one group, mmvq_ring_img_bytes of
// scratch): the column group is quantized once by mmvq_prequant
hipError_t mmvq_ring_launch(int type, const MmArgs &a, int nc, int rpw, uint8_t *img, hipStream_t st) {
    if (a.K < 8) return hipErrorInvalidValue;   // (the activation loads read 8 floats)
    if (img != nullptr && a.M > nc) return hipErrorInvalidValue;
    switch (type) {
        case T_Q4_0: return ring_type<T_Q4_0>(a, nc, rpw, img, st);
        case T_Q8_0: return ring_type<T_Q8_0>(a, nc, rpw, img, st);
        case T_Q4_K: return ring_type<T_Q4_K>(a, nc, rpw, img, st);
        case T_Q5_K: return ring_type<T_Q5_K>(a, nc, rpw, img, st);
        case T_Q6_K: return ring_type<T_Q6_K>(a, nc, rpw, img, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mi355x
