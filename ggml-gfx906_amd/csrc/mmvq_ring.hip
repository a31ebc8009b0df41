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

namespace mi355x {

constexpr int RING_K = 4096;                   // K per chunk
constexpr int RING_XBLK = RING_K / 32;         // 32-blocks per chunk (= XR_STRIDE: one per lane quad)
static_assert(RING_XBLK == XR_STRIDE, "one 32-block per lane quad and chunk");

__host__ __device__ constexpr int ring_slot_bytes(int nc) { return nc * RING_K + 4 * nc * (RING_K / 32) * 4; }

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

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
size_t mmvq_ring_lds_bytes(int nc) { return 2 * (size_t)ring_slot_bytes(nc); }

template <int T, int NC, int RPW, bool RAG, bool XA>
static hipError_t ring_one(const MmArgs &a0, hipStream_t st) {
    constexpr int WAVES = NC >= 8 ? 16 : 8;
    const size_t lds = mmvq_ring_lds_bytes(NC);
    auto kern = mmvq_ring_kernel<T, NC, RPW, RAG, XA, WAVES>;
    static bool attr_set = false;   // per instantiation; set only once the call succeeded
    if (lds > 64 * 1024 && !attr_set) {
        hipFuncAttributes fa{};
        hipError_t e = hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(kern));
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)(160 * 1024 - fa.sharedSizeBytes));
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return e;
        }
        attr_set = true;
    }
    MmArgs a = a0;
    const int nslots = ((a.K + 63) & ~63) / 64;
    a.n_it = (nslots + 63) / 64;
    const int rows_per_group = WAVES * RPW;
    const int n_groups = (a.N + rows_per_group - 1) / rows_per_group;
    const int grid_y = a.ne12 * a.ne13, grid_z = (a.M + NC - 1) / NC;
    // one round of resident workgroups (LDS-bound: 160 KiB / ring; at most 32 waves per CU);
    // more workgroups would re-quantize the same chunks for fewer rows each
    const int per_cu = std::max(1, std::min(32 / WAVES, (int)(160 * 1024 / (lds + 1024))));
    static const int64_t target_env = getenv("GGML_MI355X_RING_WGS") ? atoll(getenv("GGML_MI355X_RING_WGS")) : 0;
    const int64_t target = target_env > 0 ? target_env : 256 * per_cu;
    const int want = (int)std::max<int64_t>(1, target / ((int64_t)grid_y * grid_z));
    hipLaunchKernelGGL(kern, dim3(std::min(n_groups, want), grid_y, grid_z), dim3(WAVES * WAVE), lds, st, a);
    return hipGetLastError();
}

template <int T, int NC, int RPW>
static hipError_t ring_flags(const MmArgs &a, hipStream_t st) {
    if constexpr (T == T_Q4_0 || T == T_Q8_0) {
        if (a.K % 64 != 0)
            return a.x_aligned16 ? ring_one<T, NC, RPW, true, true>(a, st) : ring_one<T, NC, RPW, true, false>(a, st);
    }
    return a.x_aligned16 ? ring_one<T, NC, RPW, false, true>(a, st) : ring_one<T, NC, RPW, false, false>(a, st);
}

template <int T>
static hipError_t ring_type(const MmArgs &a, int nc, int rpw, hipStream_t st) {
    // 8 columns: 16 waves of one row each (see the kernel); Q6_K one row per wave throughout
    if (nc == 8) return ring_flags<T, 8, 1>(a, st);
    if (rpw <= 1 || T == T_Q6_K) {
        switch (nc) {
            case 1: return ring_flags<T, 1, 1>(a, st);
            case 2: return ring_flags<T, 2, 1>(a, st);
            case 4: return ring_flags<T, 4, 1>(a, st);
            default: return hipErrorInvalidValue;
        }
    }
    switch (nc) {
        case 1: return ring_flags<T, 1, 2>(a, st);
        case 2: return ring_flags<T, 2, 2>(a, st);
        case 4: return ring_flags<T, 4, 2>(a, st);
        default: return hipErrorInvalidValue;
    }
}

// plain MUL_MAT, a.M columns (1..8 per column group of nc in {1, 2, 4, 8}; the last group may be
// partial): grid.z = ceil(M / nc)
hipError_t mmvq_ring_launch(int type, const MmArgs &a, int nc, int rpw, hipStream_t st) {
    if (a.K < 8) return hipErrorInvalidValue;   // (the activation loads read 8 floats)
    switch (type) {
        case T_Q4_0: return ring_type<T_Q4_0>(a, nc, rpw, st);
        case T_Q8_0: return ring_type<T_Q8_0>(a, nc, rpw, st);
        case T_Q4_K: return ring_type<T_Q4_K>(a, nc, rpw, st);
        case T_Q5_K: return ring_type<T_Q5_K>(a, nc, rpw, st);
        case T_Q6_K: return ring_type<T_Q6_K>(a, nc, rpw, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mi355x
