// mmvq_fused.hip — the quantized mat-vec (mmvq_impl.h) with the decode-layer fusions of the
// GPT-2 engine (gpt2.cpp): a layer-norm prologue on the activations and a bias / GELU /
// residual epilogue on the outputs. One launch then replaces the reference graph's
// NORM -> MUL -> ADD -> MUL_MAT -> ADD [-> GELU] [-> ADD] chain
// (examples/gpt-2/main-sched.cpp:603-618, 620-634, 706-730, 760-808), i.e. five to seven ggml
// nodes and their HBM round trips become one weight stream.
//
// Instantiated for contiguous, 16-byte-aligned activations with K % 64 == 0 and K <= 8192
// (the GPT-2 shapes: K = n_embd or 4 n_embd); the host checks this before launching.
#include "mmvq_impl.h"

namespace mi355x {

size_t mmvq_lds_bytes(int K, int nc);

namespace {

// prepare_only: just raise the instantiation's dynamic-LDS limit. That is not a stream
// operation and fails inside a hipGraph capture, so mmvq_fused_prepare() runs it for every
// instantiation before the engine captures a decode step.
template <int T, int NC, int RPW>
hipError_t fused_one(const MmArgs &a, int grid_z, hipStream_t st, bool prepare_only = false) {
    auto kern = mmvq_kernel<T, NC, RPW, false, false, true, false, true>;
    static bool attr_set = false;   // per-instantiation
    if (!attr_set) {
        // 160 KB of LDS per CU minus the prologue's static reduction array
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 156 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    if (prepare_only) return hipSuccess;
    const int rows_per_group = MMVQ_WAVES * RPW;
    const int n_groups = (a.N + rows_per_group - 1) / rows_per_group;
    const int want = std::max(1, 2048 / grid_z);
    dim3 grid(std::min(n_groups, want), 1, grid_z);
    hipLaunchKernelGGL(kern, grid, dim3(MMVQ_THREADS), mmvq_lds_bytes(a.K, NC), st, a);
    return hipGetLastError();
}

template <int T, int RPW>
hipError_t fused_nc(const MmArgs &a, int nc, int grid_z, hipStream_t st) {
    switch (nc) {
        case 1: return fused_one<T, 1, RPW>(a, grid_z, st);
        case 2: return fused_one<T, 2, RPW>(a, grid_z, st);
        case 3: return fused_one<T, 3, RPW>(a, grid_z, st);
        case 4: return fused_one<T, 4, RPW>(a, grid_z, st);
        case 8: return fused_one<T, 8, RPW>(a, grid_z, st);
        default: return hipErrorInvalidValue;
    }
}

template <int T>
hipError_t fused_type(const MmArgs &a, int nc, int rpw, int grid_z, hipStream_t st) {
    return rpw <= 1 ? fused_nc<T, 1>(a, nc, grid_z, st) : fused_nc<T, 2>(a, nc, grid_z, st);
}

template <int T, int RPW>
hipError_t prepare_nc() {
    MmArgs a{};
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = fused_one<T, 1, RPW>(a, 1, nullptr, true);
    if (e == hipSuccess) e = fused_one<T, 2, RPW>(a, 1, nullptr, true);
    if (e == hipSuccess) e = fused_one<T, 3, RPW>(a, 1, nullptr, true);
    if (e == hipSuccess) e = fused_one<T, 4, RPW>(a, 1, nullptr, true);
    if (e == hipSuccess) e = fused_one<T, 8, RPW>(a, 1, nullptr, true);
    return e;
}

template <int T>
hipError_t prepare_type() {
    const hipError_t e = prepare_nc<T, 1>();
    return e != hipSuccess ? e : prepare_nc<T, 2>();
}

}  // namespace

// raise the LDS limit of every fused instantiation of `type` (outside any graph capture)
hipError_t mmvq_fused_prepare(int type) {
    switch (type) {
        case T_Q4_0: return prepare_type<T_Q4_0>();
        case T_Q8_0: return prepare_type<T_Q8_0>();
        case T_Q4_K: return prepare_type<T_Q4_K>();
        case T_Q5_K: return prepare_type<T_Q5_K>();
        case T_Q6_K: return prepare_type<T_Q6_K>();
        default: return hipErrorInvalidValue;
    }
}

// a.M columns in groups of nc (a.M % nc == 0); a.ne12 == a.ne13 == 1
hipError_t mmvq_fused_launch(int type, const MmArgs &a, int nc, int rpw, hipStream_t st) {
    if (a.K % 64 != 0 || a.K > 8192 || !a.x_aligned16 || a.ne12 != 1 || a.ne13 != 1 || nc <= 0 || a.M % nc != 0)
        return hipErrorInvalidValue;
    const int grid_z = a.M / nc;
    switch (type) {
        case T_Q4_0: return fused_type<T_Q4_0>(a, nc, rpw, grid_z, st);
        case T_Q8_0: return fused_type<T_Q8_0>(a, nc, rpw, grid_z, st);
        case T_Q4_K: return fused_type<T_Q4_K>(a, nc, rpw, grid_z, st);
        case T_Q5_K: return fused_type<T_Q5_K>(a, nc, rpw, grid_z, st);
        case T_Q6_K: return fused_type<T_Q6_K>(a, nc, rpw, grid_z, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mi355x
