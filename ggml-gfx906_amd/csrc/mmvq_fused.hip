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
#include "settings.h"

namespace mi355x {

size_t mmvq_lds_bytes(int K, int nc);
int mmvq_pick_lpr(int K);

namespace {

// prepare_only: just raise the instantiation's dynamic-LDS limit. That is not a stream
// operation and fails inside a hipGraph capture, so mmvq_fused_prepare() runs it for every
// instantiation before the engine captures a decode step.
template <int T, int NC, int LPR, int RPW, bool ATTN = false>
hipError_t fused_one(const MmArgs &a0, int grid_z, hipStream_t st, bool prepare_only = false) {
    auto kern = mmvq_kernel<T, NC, LPR, RPW, false, false, true, false, true, ATTN>;
    // 160 KB of LDS per CU minus the static arrays (layer-norm and argmax reductions), per device
    static LdsAttr attr;   // per instantiation
    if (const hipError_t e = lds_attr_once(reinterpret_cast<const void *>(kern), attr); e != hipSuccess) return e;
    if (prepare_only) return hipSuccess;
    MmArgs a = a0;
    a.n_it = ((a.K + 63) / 64 + LPR - 1) / LPR;
    const int rows_per_group = MMVQ_WAVES * (WAVE / LPR) * RPW;
    const int n_groups = (a.N + rows_per_group - 1) / rows_per_group;
    // resident-capacity grid (2 workgroups of 8 waves per CU at <= 128 VGPRs): tall matrices
    // (lm_head) walk their row groups with the prefetch pipeline instead of queueing rounds of
    // workgroups; EPI_ARGMAX needs one partial slot per workgroup (ARGMAX_SLOTS)
    const int target = settings().fused_wgs, tall = settings().fused_tall;
    const int want = std::max(1, std::min(ARGMAX_SLOTS, (n_groups > 4 * target ? tall : target) / grid_z));
    dim3 grid(std::min(n_groups, want), 1, grid_z);
    hipLaunchKernelGGL(kern, grid, dim3(MMVQ_THREADS), mmvq_lds_bytes(a.K, NC), st, a);
    return hipGetLastError();
}

template <int T, int LPR, int RPW, bool ATTN = false>
hipError_t fused_nc(const MmArgs &a, int nc, int grid_z, hipStream_t st) {
    switch (nc) {
        case 1: return fused_one<T, 1, LPR, RPW, ATTN>(a, grid_z, st);
        case 2: return fused_one<T, 2, LPR, RPW, ATTN>(a, grid_z, st);
        case 3: return fused_one<T, 3, LPR, RPW, ATTN>(a, grid_z, st);
        case 4: return fused_one<T, 4, LPR, RPW, ATTN>(a, grid_z, st);
        case 8: return fused_one<T, 8, LPR, RPW, ATTN>(a, grid_z, st);
        default: return hipErrorInvalidValue;
    }
}

template <int T, int LPR>
hipError_t fused_nc_attn(const MmArgs &a, int nc, int grid_z, hipStream_t st) {
    switch (nc) {
        case 1: return fused_one<T, 1, LPR, 1, true>(a, grid_z, st);
        case 2: return fused_one<T, 2, LPR, 1, true>(a, grid_z, st);
        case 3: return fused_one<T, 3, LPR, 1, true>(a, grid_z, st);
        default: return hipErrorInvalidValue;
    }
}

// lanes per row of a fused mat-vec: as mmvq_pick_lpr, but short matrices (N <= 1024, e.g. GPT-2
// 117M's 768-row projections) take 64 lanes (8 rows per workgroup instead of 32) so that they
// spread over 4x the CUs: 4.9 -> 4.0-4.4 us per launch in the drop-in decode (scripts/
// prof_plugin_shapes.sh), ~2% on the whole token
static int fused_lpr(const MmArgs &a) {
    return a.N <= settings().fused_lpr64_maxn ? 64 : mmvq_pick_lpr(a.K);
}

template <int T>
hipError_t fused_type(const MmArgs &a, int nc, int rpw, int grid_z, hipStream_t st) {
    if (a.attn_part != nullptr) {   // c_proj with the attention merge prologue (K = n_embd)
        if (a.K > 4096) return hipErrorInvalidValue;
        if (nc > 3) return hipErrorInvalidValue;   // (the merge partials of >3 columns would spill)
        return fused_lpr(a) == 16 ? fused_nc_attn<T, 16>(a, nc, grid_z, st) : fused_nc_attn<T, 64>(a, nc, grid_z, st);
    }
    if (fused_lpr(a) == 16) return fused_nc<T, 16, 1>(a, nc, grid_z, st);
    return rpw <= 1 ? fused_nc<T, 64, 1>(a, nc, grid_z, st) : fused_nc<T, 64, 2>(a, nc, grid_z, st);
}

template <int T, int LPR, int RPW>
hipError_t prepare_nc() {
    MmArgs a{};
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = fused_one<T, 1, LPR, RPW>(a, 1, nullptr, true);
    if (e == hipSuccess) e = fused_one<T, 2, LPR, RPW>(a, 1, nullptr, true);
    if (e == hipSuccess) e = fused_one<T, 3, LPR, RPW>(a, 1, nullptr, true);
    if (e == hipSuccess) e = fused_one<T, 4, LPR, RPW>(a, 1, nullptr, true);
    if (e == hipSuccess) e = fused_one<T, 8, LPR, RPW>(a, 1, nullptr, true);
    return e;
}

template <int T, int LPR>
hipError_t prepare_attn() {
    MmArgs a{};
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = fused_one<T, 1, LPR, 1, true>(a, 1, nullptr, true);
    if (e == hipSuccess) e = fused_one<T, 2, LPR, 1, true>(a, 1, nullptr, true);
    if (e == hipSuccess) e = fused_one<T, 3, LPR, 1, true>(a, 1, nullptr, true);
    return e;
}

template <int T>
hipError_t prepare_type() {
    hipError_t e = prepare_nc<T, 64, 1>();
    if (e == hipSuccess) e = prepare_nc<T, 64, 2>();
    if (e == hipSuccess) e = prepare_nc<T, 16, 1>();
    if (e == hipSuccess) e = prepare_attn<T, 16>();
    if (e == hipSuccess) e = prepare_attn<T, 64>();
    return e;
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

// widest column group with a kernel that divides M (groups of 4 / 8 serve K <= 4096)
int mmvq_fused_pick_nc(int M, int K) {
    for (int nc : {8, 4, 3, 2, 1})
        if (M % nc == 0 && (nc < 4 || K <= 4096)) return nc;
    return 1;
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
