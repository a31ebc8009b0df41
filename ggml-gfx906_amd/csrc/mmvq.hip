// mmvq.hip — launchers of the quantized mat-vec kernel (mmvq_impl.h) for plain MUL_MAT and
// MUL_MAT_ID. The fused decode-layer instantiations live in mmvq_fused.hip.
#include "mmvq_impl.h"
#include "settings.h"

#include <string>

namespace mi355x {

// ------------------------------------------------------------------------------------------
// host-side launch helpers (called from dispatch.cpp)
// ------------------------------------------------------------------------------------------
size_t mmvq_lds_bytes(int K, int nc) {
    const int Kpad = (K + 63) & ~63;
    return (size_t)nc * Kpad + sizeof(float) * (size_t)nc * (Kpad / 32) * 4;   // xq + xd + xs + x16
}

// lanes per weight row: the width (16 or 64) that leaves the fewest idle slot lanes for this K;
// ties go to 64 (fewer K iterations per row)
int mmvq_pick_lpr(int K) {
    const int force = settings().lpr;   // diagnostics
    if (force == 16 || force == 64) return force;
    const int nslots = (K + 63) / 64;
    const int u16 = 16 * ((nslots + 15) / 16), u64 = 64 * ((nslots + 63) / 64);
    return u16 < u64 ? 16 : 64;
}

int mmvq_rows_per_group(int lpr, int rpw) { return MMVQ_WAVES * (WAVE / lpr) * rpw; }

// workgroups a launch aims at (beyond that each walks more row groups): 2048 (scripts/mmvq_sweep.sh,
// round 2), 4096 for Q4_0 / Q4_K, whose kernels keep more waves resident (7 / 5 per SIMD against
// 3-4): on the bench's stacked launches Q4_0 4096^2 x 64 101.4-101.9 vs 103.7-104.2 us, Q4_K 103.8
// vs 106.8, Q4_K 4096 x 11008 x 24 103.6 vs 105.6, while Q5_K x 24 takes 143 vs 131 and Q6_K 171
// vs 165 (profiles/r06_mmvq_wgs_ab.txt, three interleaved rounds)
static int64_t mmvq_target_wgs(int type) {
    if (settings().mmvq_wgs > 0) return settings().mmvq_wgs;
    return type == T_Q4_0 || type == T_Q4_K ? 4096 : 2048;
}

template <int T, int NC, int LPR, int RPW, bool IDS, bool RAG, bool XA, bool BIGK>
static hipError_t launch_one(const MmArgs &a0, int grid_y, int grid_z, hipStream_t st) {
    const size_t lds = mmvq_lds_bytes(a0.K, NC);
    auto kern = mmvq_kernel<T, NC, LPR, RPW, IDS, RAG, XA, BIGK>;
    MmArgs a = a0;
    a.n_it = ((a.K + 63) / 64 + LPR - 1) / LPR;
    // more than 64 KB of dynamic LDS needs the attribute, once per instantiation and device. The
    // call fails inside a stream capture: the error is returned (the capture then fails and the
    // caller runs the graph eagerly once, which sets it).
    static LdsAttr attr;   // per instantiation
    if (lds > 64 * 1024)
        if (const hipError_t e = lds_attr_once(reinterpret_cast<const void *>(kern), attr); e != hipSuccess) return e;
    const int rows_per_group = MMVQ_WAVES * (WAVE / LPR) * RPW;
    const int n_groups = (a.N + rows_per_group - 1) / rows_per_group;
    // enough workgroups to fill 256 CUs ~4 deep; beyond that each workgroup walks more groups
    const int64_t others = (int64_t)grid_y * grid_z;
    const int64_t target = mmvq_target_wgs(T);
    // floor, not ceil: a launch just above a multiple of the resident capacity (4 workgroups of
    // 8 waves per CU = 1024) leaves a tail of workgroups that start only when others finish
    const int want = (int)std::max<int64_t>(1, target / others);
    dim3 grid(std::min(n_groups, want), grid_y, grid_z);
    hipLaunchKernelGGL(kern, grid, dim3(MMVQ_THREADS), lds, st, a);
    return hipGetLastError();
}

// K > 8192 (activations need more than two preloaded quantization rounds)
static bool is_bigk(const MmArgs &a) { return ((a.K + 63) & ~63) / 32 > 2 * XR_STRIDE; }

template <int T, int NC, int LPR, int RPW, bool IDS>
static hipError_t launch_flags(const MmArgs &a, int grid_y, int grid_z, hipStream_t st) {
    const bool rag = (a.K % 64) != 0;
    if (is_bigk(a)) {
        if constexpr (NC == 1 && LPR == 64) {
            if constexpr (T == T_Q4_0 || T == T_Q8_0) {
                if (rag) return launch_one<T, 1, 64, RPW, IDS, true, false, true>(a, grid_y, grid_z, st);
            }
            return a.x_aligned16 ? launch_one<T, 1, 64, RPW, IDS, false, true, true>(a, grid_y, grid_z, st)
                                 : launch_one<T, 1, 64, RPW, IDS, false, false, true>(a, grid_y, grid_z, st);
        }
        return hipErrorInvalidValue;   // host splits big-K launches into single columns of 64-lane rows
    }
    if constexpr (T == T_Q4_0 || T == T_Q8_0) {
        if (rag) {
            return a.x_aligned16 ? launch_one<T, NC, LPR, RPW, IDS, true, true, false>(a, grid_y, grid_z, st)
                                 : launch_one<T, NC, LPR, RPW, IDS, true, false, false>(a, grid_y, grid_z, st);
        }
    }
    return a.x_aligned16 ? launch_one<T, NC, LPR, RPW, IDS, false, true, false>(a, grid_y, grid_z, st)
                         : launch_one<T, NC, LPR, RPW, IDS, false, false, false>(a, grid_y, grid_z, st);
}

template <int T, int LPR, int RPW>
static hipError_t launch_nc(const MmArgs &a, int nc, int grid_y, int grid_z, hipStream_t st) {
    switch (nc) {
        case 1: return launch_flags<T, 1, LPR, RPW, false>(a, grid_y, grid_z, st);
        case 2: return launch_flags<T, 2, LPR, RPW, false>(a, grid_y, grid_z, st);
        case 3: return launch_flags<T, 3, LPR, RPW, false>(a, grid_y, grid_z, st);
        case 4: return launch_flags<T, 4, LPR, RPW, false>(a, grid_y, grid_z, st);
        case 8: return launch_flags<T, 8, LPR, RPW, false>(a, grid_y, grid_z, st);
        default: return hipErrorInvalidValue;
    }
}

// lanes per row of a launch, from hipGraph periods of back-to-back calls
// (profiles/r06_valu_plan_sweep.txt; mmvq_pick_lpr alone chose by idle slot lanes):
//  * below 6144 rows 64 from K = 1088 on, even where that leaves slot lanes idle: an 8-wave
//    workgroup then covers 8 or 16 rows instead of 32, and short matrices get the workgroups to
//    fill the chip (Q4_0 3072 x 768 3.2 vs 4.3 us, Q6_K 3072 x 768 at 4 columns 5.4 vs 8.2);
//  * from 6144 rows 16 for groups of 2..8 columns, also where both widths use every slot lane
//    (K = 4096): four rows per wave share each activation read and a workgroup serves twice the
//    rows, so its staging of the columns (load and quantization of nc x K values) is spread over
//    twice the weight bytes (Q6_K 4096 x 14336 at 8 columns 25.4 vs 43.8 us, Q5_K at 3 13.7 vs
//    19.2); single columns keep mmvq_pick_lpr's width there (Q4_0 2048 x 14336 5.8 vs 7.5 us
//    with 16, 4096 x 11008 7.6 vs 8.2 with 64);
//  * K <= 1024: mmvq_pick_lpr's width.
static int lanes_per_row(const MmArgs &a, int nc) {
    if (is_bigk(a)) return 64;
    const int l = mmvq_pick_lpr(a.K);
    if (settings().lpr == 16 || settings().lpr == 64 || a.K <= 1024) return l;
    if (a.N >= 6144) return nc >= 2 ? 16 : l;
    return 64;
}

// 16-lane rows only with one row per lane group
template <int T>
static hipError_t launch_type(const MmArgs &a, int nc, int grid_y, int grid_z, int rpw, hipStream_t st) {
    if (lanes_per_row(a, nc) == 16) return launch_nc<T, 16, 1>(a, nc, grid_y, grid_z, st);
    if (rpw <= 1) return launch_nc<T, 64, 1>(a, nc, grid_y, grid_z, st);
    return launch_nc<T, 64, 2>(a, nc, grid_y, grid_z, st);
}

// the launch launch_type / launch_one make (the dispatch description, ggml_mi355x_mul_mat_plan)
std::string mmvq_plan_text(int type, const MmArgs &a, int nc, int rpw) {
    const bool bigk = is_bigk(a);
    const int lpr = lanes_per_row(a, nc);
    const int r = lpr == 16 || rpw <= 1 ? 1 : 2;
    const int rows_per_group = MMVQ_WAVES * (WAVE / lpr) * r;
    const int n_groups = (a.N + rows_per_group - 1) / rows_per_group;
    const int64_t others = (int64_t)a.ne12 * a.ne13 * (a.M / nc);
    const int64_t target = mmvq_target_wgs(type);
    const int gx = (int)std::min<int64_t>(n_groups, std::max<int64_t>(1, target / others));
    return "mmvq nc=" + std::to_string(nc) + " lpr=" + std::to_string(lpr) + " rpw=" + std::to_string(r) +
           (bigk ? " bigk" : "") + " grid=" + std::to_string(gx) + "x" + std::to_string(a.ne12 * a.ne13) + "x" +
           std::to_string(a.M / nc);
}

// column-group widths that have kernels (dispatch.cpp splits M into these); groups of 4 and 8
// columns hold one activation round in registers, so they serve K <= 4096 only
bool mmvq_has_nc(int nc) { return nc == 1 || nc == 2 || nc == 3 || nc == 4 || nc == 8; }
int mmvq_max_k_for_nc(int nc) { return nc >= 4 ? 32 * XR_STRIDE : 64 * XR_STRIDE; }
bool mmvq_bigk(int K) { MmArgs a{}; a.K = K; return is_bigk(a); }

// plain MUL_MAT: a.M columns in groups of nc (a.M % nc == 0)
hipError_t mmvq_launch(int type, const MmArgs &a, int nc, int rpw, hipStream_t st) {
    const int grid_y = a.ne12 * a.ne13;
    const int grid_z = a.M / nc;
    switch (type) {
        case T_Q4_0: return launch_type<T_Q4_0>(a, nc, grid_y, grid_z, rpw, st);
        case T_Q8_0: return launch_type<T_Q8_0>(a, nc, grid_y, grid_z, rpw, st);
        case T_Q4_K: return launch_type<T_Q4_K>(a, nc, grid_y, grid_z, rpw, st);
        case T_Q5_K: return launch_type<T_Q5_K>(a, nc, grid_y, grid_z, rpw, st);
        case T_Q6_K: return launch_type<T_Q6_K>(a, nc, grid_y, grid_z, rpw, st);
        default: return hipErrorInvalidValue;
    }
}

// MUL_MAT_ID: one (expert slot, token) GEMV per grid.y
hipError_t mmvq_id_launch(int type, const MmArgs &a, int rpw, hipStream_t st) {
    const int grid_y = a.n_used * a.n_tok;
    (void)rpw;
    const bool l16 = mmvq_pick_lpr(a.K) == 16 && !is_bigk(a);
    switch (type) {
        case T_Q4_0: return l16 ? launch_flags<T_Q4_0, 1, 16, 1, true>(a, grid_y, 1, st) : launch_flags<T_Q4_0, 1, 64, 1, true>(a, grid_y, 1, st);
        case T_Q8_0: return l16 ? launch_flags<T_Q8_0, 1, 16, 1, true>(a, grid_y, 1, st) : launch_flags<T_Q8_0, 1, 64, 1, true>(a, grid_y, 1, st);
        case T_Q4_K: return l16 ? launch_flags<T_Q4_K, 1, 16, 1, true>(a, grid_y, 1, st) : launch_flags<T_Q4_K, 1, 64, 1, true>(a, grid_y, 1, st);
        case T_Q5_K: return l16 ? launch_flags<T_Q5_K, 1, 16, 1, true>(a, grid_y, 1, st) : launch_flags<T_Q5_K, 1, 64, 1, true>(a, grid_y, 1, st);
        case T_Q6_K: return l16 ? launch_flags<T_Q6_K, 1, 16, 1, true>(a, grid_y, 1, st) : launch_flags<T_Q6_K, 1, 64, 1, true>(a, grid_y, 1, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mi355x
