// dispatch.cpp — host-side dispatch of GGML_OP_MUL_MAT / GGML_OP_MUL_MAT_ID onto the gfx950
// kernels, plus the direct C API of include/ggml-mi355x.h.
//
// Behavioural reference: ggml_cuda_mul_mat (src/ggml-cuda/ggml-cuda.cu:2007-2090) picks the
// mat-vec kernel for ne11 <= 8 (MMVQ_MAX_BATCH_SIZE) and the tiled matrix kernel otherwise;
// this file keeps that split but routes to our own kernels.
#include "dispatch.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <memory>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/ggml-mi355x.h"
#include "qcommon.h"
#include "settings.h"

namespace mi355x {

hipError_t mmvq_launch(int type, const MmArgs &a, int nc, int rpw, hipStream_t st);
hipError_t mmvq_id_launch(int type, const MmArgs &a, int rpw, hipStream_t st);
size_t mmvq_lds_bytes(int K, int nc);
bool mmvq_has_nc(int nc);
int mmvq_max_k_for_nc(int nc);
bool mmvq_bigk(int K);
hipError_t mmvq_ring_launch(int type, const MmArgs &a, int nc, int rpw, uint8_t *img, hipStream_t st);
hipError_t mmvq_mma_launch(int type, const MmArgs &a, uint8_t *img, hipStream_t st);
size_t mmvq_mma_img_bytes(int type, const MmArgs &a);
bool mmvq_mma_supported(int type, const MmArgs &a);
bool mmvq_mma_one_part(int type, const MmArgs &a);
bool mmvq_mma_paired(int type, const MmArgs &a);
size_t mmvq_ring_img_bytes(const MmArgs &a, int nc);
hipError_t dequant_launch(int type, const void *src, float *dst, int64_t n, hipStream_t st);
struct RowsArgs {
    const uint8_t *src; int64_t nb01, nb02, nb03, ne01;
    const uint8_t *idx; int64_t nb10, nb11, nb12, ne10, ne11;
    uint8_t *dst; int64_t nb1, nb2, nb3;
    int64_t ne00;
    int *err;
};
hipError_t get_rows_launch(int type, const RowsArgs &a, int64_t nrows, hipStream_t st);
hipError_t get_rows_add_launch(int type, const RowsArgs &a, const RowsArgs &b, int64_t nrows, hipStream_t st);
struct QuantArgs {
    const uint8_t *src; int64_t nb01, nb02, nb03;
    uint8_t *dst; int64_t nb1, nb2, nb3;
    int64_t ne0, ne1, ne2, ne3;
};
hipError_t quantize_launch(int type, const QuantArgs &a, hipStream_t st);
struct CpyQArgs {
    const uint8_t *src; int64_t ne00, ne01, ne02; int64_t nb00, nb01, nb02, nb03;
    uint8_t *dst; int64_t ne0, ne1, ne2; int64_t nb0, nb1, nb2, nb3;
    int64_t n;
};
hipError_t cpy_q_launch(int type, bool to_f32, const CpyQArgs &a, hipStream_t st);
bool mmq8_supported(int type, const MmArgs &a);
bool mmq8_images_fit(int type, const MmArgs &a);
hipError_t mmq8_launch(int type, const MmArgs &a, hipStream_t st, Scratch &scratch);
int mmq8_tile_tokens(const MmArgs &a);
int64_t mmq8_tiles128(const MmArgs &a);
hipError_t mmq8r_launch(int type, const MmArgs &a, const void *rp, int ne02, int n_mat, hipStream_t st, Scratch &scratch);
bool mmq8_id_supported(int type, const MmArgs &a);
hipError_t mmq8_id_launch(int type, const MmArgs &a, hipStream_t st, Scratch &scratch);
std::string mmvq_plan_text(int type, const MmArgs &a, int nc, int rpw);
std::string mmvq_ring_plan_text(int type, const MmArgs &a, int nc, int rpw, bool pre);
std::string mmvq_mma_plan_text(int type, const MmArgs &a);
std::string mmq8_plan_text(const MmArgs &a);
bool mmvq_solo_default(int type, const MmArgs &a);
hipError_t mmvq_solo_launch(int type, const MmArgs &a, hipStream_t st);
std::string mmvq_solo_plan_text(int type, const MmArgs &a);

// mat-mat kernel family: the int8 MFMA tile (csrc/mmq8.hip). It takes every K and every
// 2-byte-aligned Q4_0 / Q8_0 / Q6_K layout (16-B aligned Q4_K / Q5_K) and is exact in the block
// scales. What it refuses (a K-quant view at an offset finer than 16 B, > 4 GiB spans) takes the
// mat-vec, which is exact too. (Rounds 1-4 also shipped f16 MFMA tiles, behind
// GGML_MI355X_MMQ=f16 for A/B only; with a known f16 range hole past d > 511 and no default
// shape using them they were removed in round 5)

static constexpr size_t LDS_LIMIT = 159 * 1024;   // 160 KB per CU, less the kernels' static arrays

int type_blck(int t) {
    switch (t) {
        case T_Q4_0: case T_Q8_0: return 32;
        case T_Q4_K: case T_Q5_K: case T_Q6_K: return 256;
        default: return 0;
    }
}

int type_bytes(int t) {
    switch (t) {
        case T_Q4_0: return 18;
        case T_Q8_0: return 34;
        case T_Q4_K: return 144;
        case T_Q5_K: return 176;
        case T_Q6_K: return 210;
        case T_F32: case T_I32: return 4;
        default: return 0;
    }
}

bool is_hot_quant(int t) { return type_blck(t) != 0; }

// rows per wave for the mat-vec. Every workgroup quantizes its column(s) of src1 once, so
// more rows per workgroup amortize that (the activation loads and their quantization are the
// critical path of a single-matrix launch, profiles/r06_single_launch_decomposition.txt); fewer
// rows give more workgroups. Two rows per wave from 4096 rows (x batch) on, i.e. from one
// 16-row workgroup per CU: single 4096 x 4096 Q4_0 4.91 vs 5.06-5.51 us, 4096 x 11008 Q4_K
// 8.7 vs 9.5, Q5_K 10.5-11.1 vs 11.6-11.8 (profiles/r06_singles_ab.txt, rocprof means, two
// interleaved rounds; round 5's rule switched at 16384).
// Q6_K keeps one row per wave: its two-row kernel needs 133 VGPRs, which leaves one 8-wave
// workgroup per CU instead of two (Q6_K 4096x11008 x24: 169 vs 178 us, profiles/r03_q6k_rpw.txt;
// single 4096 x 11008: 13.5-13.8 vs 12.6-12.8 us, profiles/r06_singles_ab.txt).
// Round 6, from hipGraph periods of back-to-back calls (profiles/r06_valu_plan_sweep.txt; the
// rule above came from rocprof kernel durations): two rows from 4096 rows also for the whole-K
// kernel's groups of 2..4 columns (Q4_0 4096^2 at 4 columns 5.7 vs 7.0 us, Q4_K 4096 x 11008 at 3
// 12.9 vs 14.4) and for the chunked-K kernel's column pairs (Q4_K 14336 x 4096 at 2 columns 11.5
// vs 12.9, Q4_0 4096 x 11008 9.5 vs 10.8); its single columns only for Q4_K / Q5_K (Q4_K 14336 x
// 4096 9.4 vs 10.1; Q8_0 there 14.2 vs 13.6 with one row); its groups of 4 / 8 columns keep the
// switch at 16384 rows (Q6_K 4096 x 14336 at 3 columns 22.9 vs 20.5 with two); Q8_0 / Q5_K groups
// of 3..4 columns keep one row from 12288 rows (Q5_K 4096 x 14336 at 3 columns 20.2 vs 18.9).
static int pick_rpw(int type, int64_t rows_total, int nc, bool ring) {
    if (settings().rpw > 0) return settings().rpw;
    if (type == T_Q6_K) return 1;
    if (ring) {
        if (nc == 1) return (type == T_Q4_K || type == T_Q5_K) && rows_total >= 4096 ? 2 : 1;
        return rows_total >= (nc == 2 ? 4096 : 16384) ? 2 : 1;
    }
    if (nc >= 3 && nc <= 4 && (type == T_Q8_0 || type == T_Q5_K) && rows_total >= 12288) return 1;
    return rows_total >= (nc <= 4 ? 4096 : 16384) ? 2 : 1;
}

// ------------------------------------------------------------------------------------------
// diagnostics: GGML_MI355X_STAMPS=1 makes every mat-vec launch record per-workgroup
// s_memrealtime stamps (start / activations in LDS / dots done / end) into a device buffer that
// ggml_mi355x_debug_stamps() copies out. Off by default: kernels test one null pointer.
// ------------------------------------------------------------------------------------------
static unsigned long long *g_stamps = nullptr;
static const size_t STAMP_SLOTS = 8 * 65536;

unsigned long long *stamps_buffer();
unsigned long long *stamps_buffer() {
    if (!settings().stamps) return nullptr;
    if (!g_stamps && hipMalloc(&g_stamps, STAMP_SLOTS * sizeof(unsigned long long)) != hipSuccess) g_stamps = nullptr;
    return g_stamps;
}

static bool aligned16(const void *p, int64_t s1, int64_t s2, int64_t s3) {
    return ((uintptr_t)p % 16) == 0 && s1 % 16 == 0 && s2 % 16 == 0 && s3 % 16 == 0;
}

int check_mul_mat(const TensorView &a, const TensorView &b, const TensorView &d) {
    if (!is_hot_quant(a.type) || b.type != T_F32 || d.type != T_F32) return GGML_MI355X_EINVAL;
    if (a.ne[0] != b.ne[0] || a.ne[0] % type_blck(a.type) != 0) return GGML_MI355X_EINVAL;
    if (a.ne[2] <= 0 || a.ne[3] <= 0 || b.ne[2] % a.ne[2] != 0 || b.ne[3] % a.ne[3] != 0) return GGML_MI355X_EINVAL;
    if (d.ne[0] != a.ne[1] || d.ne[1] != b.ne[1] || d.ne[2] != b.ne[2] || d.ne[3] != b.ne[3]) return GGML_MI355X_EINVAL;
    if ((int64_t)a.nb[0] != type_bytes(a.type) || b.nb[0] != 4 || d.nb[0] != 4) return GGML_MI355X_EINVAL;
    if (a.ne[0] > (1 << 24) || a.ne[1] > (1LL << 31) - 1 || b.ne[1] > (1LL << 31) - 1) return GGML_MI355X_EINVAL;
    return GGML_MI355X_OK;   // (any K: past the whole-K kernel's LDS the chunked one runs, use_ring)
}

static MmArgs base_args(const TensorView &a, const TensorView &b, const TensorView &d) {
    MmArgs m{};
    m.w = static_cast<const uint8_t *>(a.data);
    m.nb01 = (int64_t)a.nb[1]; m.nb02 = (int64_t)a.nb[2]; m.nb03 = (int64_t)a.nb[3];
    m.x = static_cast<const uint8_t *>(b.data);
    m.nb11 = (int64_t)b.nb[1]; m.nb12 = (int64_t)b.nb[2]; m.nb13 = (int64_t)b.nb[3];
    m.dst = static_cast<uint8_t *>(d.data);
    m.nb1 = (int64_t)d.nb[1]; m.nb2 = (int64_t)d.nb[2]; m.nb3 = (int64_t)d.nb[3];
    m.K = (int)a.ne[0];
    m.N = (int)a.ne[1];
    m.M = (int)b.ne[1];
    m.ne12 = (int)b.ne[2];
    m.ne13 = (int)b.ne[3];
    m.r2 = (int)(b.ne[2] / a.ne[2]);
    m.r3 = (int)(b.ne[3] / a.ne[3]);
    m.x_aligned16 = aligned16(b.data, m.nb11, m.nb12, m.nb13);
    m.stamps = stamps_buffer();
    m.diag = settings().diag;
    return m;
}

// the chunked-K mat-vec (mmvq_ring.hip) takes a column group when K > 4096 and either several
// columns share the pass (one pass over the weights for up to 8 columns at any K, where the
// whole-K kernel would split them into passes of 1..3 columns) or the group's whole-K image would
// not fit LDS. GGML_MI355X_RING: 0 = never (the whole-K kernel's column splits, measurements),
// 2 = also single columns at K > 4096.
static int ring_policy() { return settings().ring; }

static bool use_ring(int K, int ncols) {
    if (K <= 4096 || ring_policy() == 0) return mmvq_lds_bytes(K, 1) > LDS_LIMIT;
    return ncols >= 2 || ring_policy() == 2 || mmvq_bigk(K);
}

// column groups of at least ring_pre_min() columns at K > 4096 are quantized once per call into
// scratch (mmvq_prequant) instead of by every workgroup; GGML_MI355X_RING_PRE=0: in the
// workgroups (A/B), =2: from 2 columns on (default 4)
static int ring_pre_min() {
    const int v = settings().ring_pre;
    return v == 0 ? 1 << 30 : v == 2 ? 2 : 4;
}

// the int8 MFMA mat-vec (mmvq_mma.hip: the weights read once, the columns packed
// block-diagonally into the MFMA's 16 columns, flat in the column count) against the per-column
// VALU kernels, from hipGraph periods of back-to-back calls (profiles/r06_mma_plan_sweep.txt:
// 4 types x 10 shapes K x N from 4096 to 28672 x 3..8 columns, Infinity-Cache-cold weights; the
// round-5 rule came from eager launches, host-bound at these sizes). Used from
//   Q4_0  K < 8192: 5; else 3 at K >= 11008 or N >= 8192, else 4
//   Q8_0  3 columns at K >= 11008; else 5
//   Q4_K  3 at K >= 8192; else 5
// (below K = 8192 the whole-K VALU kernel with 16-lane rows, mmvq.hip lanes_per_row, takes 3..4
// columns: Q4_0 4096 x 14336 at 3 10.6 vs 14.7 us, Q4_K at 4 12.5 vs 17.2)
//   Q5_K  K < 8192: 5; to K = 16384 3 where the plan keeps one K part (its image fits the LDS;
//         elsewhere the unpaired form loses to the VALU kernels up to 7 columns: 27.4 vs 28.8 us
//         at 28672 x 4096), 3 at any K where the plan takes paired steps (28672 x 4096 at 3
//         columns 23.4 vs 27.4, profiles/r06_q5k_pairs.txt), and 8
//   Q6_K  K < 8192: 5; 3 from K = 12288, or from 8192 at N >= 8192; else 8 (profiles/r06_q6k_mma.txt:
//         14336 x 4096 at 3..8 columns 18.0-18.4 vs 21.3-27.3 us, 4096 x 4096 at 5..8 9.7-9.9 vs
//         13.2-14.2; at 11008 x 4096 the VALU kernels stay ahead to 5 columns)
// e.g. Q4_0 4096 x 4096 at 5..8 columns 8.4 vs 10.1-12.0 us, Q8_0 14336 x 4096 at 3..8 18.5 vs
// 20.3-23.0, Q5_K 14336 x 4096 at 3..8 17.5 vs 18.5-22.3 (the plan's one-K-part forms,
// profiles/r06_mma_plan_sweep.txt); everywhere else the VALU kernels are as fast or within 3 %. GGML_MI355X_MMA=N: from N columns on for every type it
// takes; 0: never.
static bool use_mma(int type, const MmArgs &g) {
    const int K = g.K, N = g.N, cols = g.M;
    const int v = settings().mma;
    if (v >= 0) return v != 0 && cols >= v;
    if (g.ne12 * g.ne13 > 1) return false;   // (8 batch slices: 2-4 % slower than the VALU kernels)
    if (K < 4096) return false;     // (outside the swept range; below 32 steps most of a workgroup's
                                    // 16 waves would idle, e.g. GPT-2's lm_head at K = 768)
    switch (type) {
        case T_Q4_0:
            if (K < 8192) return cols >= 5;
            return cols >= (K >= 11008 || N >= 8192 ? 3 : 4);
        case T_Q8_0: return cols >= (K >= 11008 ? 3 : 5);
        case T_Q4_K: return cols >= (K >= 8192 ? 3 : 5);
        case T_Q5_K:
            return K < 8192 ? cols >= 5 : cols >= 8 || (cols >= 3 && ((K <= 16384 && mmvq_mma_one_part(type, g)) || mmvq_mma_paired(type, g)));
        case T_Q6_K: return cols >= (K >= 12288 || (K >= 8192 && N >= 8192) ? 3 : K >= 8192 ? 8 : 5);
        default: return false;
    }
}

// mat-vec over columns [c0, c0 + ncols) in groups of at most 8 (scratch: the caller holds its
// mutex; nullptr = no pre-quantized images). plan != nullptr: launch nothing, append the launches
// that would run (ggml_mi355x_mul_mat_plan; scratch then counts as available)
static hipError_t run_mmvq(int type, MmArgs m, int c0, int ncols, hipStream_t st, Scratch *scratch = nullptr,
                           std::string *plan = nullptr) {
    const int64_t rows_total = (int64_t)m.N * m.ne12 * m.ne13;
    const bool have_scratch = scratch != nullptr || plan != nullptr;
    auto note = [&](const std::string &s) {
        if (!plan->empty()) *plan += "; ";
        *plan += s;
    };
    MmArgs gm = m;
    gm.x = m.x + (int64_t)c0 * m.nb11;
    gm.dst = m.dst + (int64_t)c0 * m.nb1;
    gm.M = ncols;
    if (have_scratch && ncols >= 1 && ncols <= 8 && use_mma(type, gm)) {
        const MmArgs &g = gm;
        // (nullptr inside a capture that would grow the scratch: the kernels below take it)
        if (mmvq_mma_supported(type, g)) {
            if (plan) {
                note(mmvq_mma_plan_text(type, g));
                return hipSuccess;
            }
            if (uint8_t *img = static_cast<uint8_t *>(scratch->get(mmvq_mma_img_bytes(type, g), st))) {
                const hipError_t e = mmvq_mma_launch(type, g, img, st);
                if (e != hipErrorInvalidValue) return e;   // (a shape the launcher refuses: the kernels below)
            }
        }
    }
    while (ncols > 0) {
        MmArgs g = m;
        g.x = m.x + (int64_t)c0 * m.nb11;
        g.dst = m.dst + (int64_t)c0 * m.nb1;
        int nc;
        hipError_t e;
        if (use_ring(m.K, ncols)) {
            const int take = std::min(ncols, 8);   // one launch: the last column group may be partial
            nc = take <= 1 ? 1 : take <= 2 ? 2 : take <= 4 ? 4 : 8;
            g.M = take;
            uint8_t *img = nullptr;
            if (plan) {
                note(mmvq_ring_plan_text(type, g, nc, pick_rpw(type, rows_total, nc, true), nc >= ring_pre_min()));
                e = hipSuccess;
            } else {
                if (nc >= ring_pre_min() && scratch != nullptr)   // (nullptr inside a capture that would grow it)
                    img = static_cast<uint8_t *>(scratch->get(mmvq_ring_img_bytes(g, nc), st));
                e = mmvq_ring_launch(type, g, nc, pick_rpw(type, rows_total, nc, true), img, st);
            }
            nc = take;
        } else {
            nc = mmvq_bigk(m.K) ? 1 : std::min(ncols, 8);
            while (nc > 1 && (!mmvq_has_nc(nc) || mmvq_lds_bytes(m.K, nc) > LDS_LIMIT || m.K > mmvq_max_k_for_nc(nc))) --nc;
            g.M = nc;
            const bool solo = nc == 1 && mmvq_solo_default(type, g);
            if (plan) {
                note(solo ? mmvq_solo_plan_text(type, g) : mmvq_plan_text(type, g, nc, pick_rpw(type, rows_total, nc, false)));
                e = hipSuccess;
            } else if (solo) {
                e = mmvq_solo_launch(type, g, st);
            } else {
                e = mmvq_launch(type, g, nc, pick_rpw(type, rows_total, nc, false), st);
            }
        }
        if (e != hipSuccess) return e;
        c0 += nc;
        ncols -= nc;
    }
    return hipSuccess;
}

static RpSrcView rp_view(const TensorView &w) {
    return RpSrcView{w.data, (int64_t)w.nb[1], (int64_t)w.nb[2], (int64_t)w.nb[3], (int)w.ne[0], (int)w.ne[1], (int)w.ne[2],
                     (int)(w.ne[2] * w.ne[3])};
}

size_t repack_size(const TensorView &w) {
    if (!is_hot_quant(w.type) || (int64_t)w.nb[0] != type_bytes(w.type) || w.ne[0] <= 0 || w.ne[1] <= 0) return 0;
    if (w.ne[0] > (1 << 24) || w.ne[1] > (1LL << 31) - 1 || w.ne[2] * w.ne[3] > (1LL << 31) - 1) return 0;
    const RpSrcView v = rp_view(w);
    return repack_supported(w.type, v) ? rp_layout(w.type, v.K, v.N, v.n_mat).bytes : 0;
}

int repack(const TensorView &w, void *dst, size_t bytes, hipStream_t st) {
    const size_t need = repack_size(w);
    if (need == 0) return GGML_MI355X_EINVAL;
    if (bytes < need || dst == nullptr) return GGML_MI355X_EINVAL;
    return repack_launch(w.type, rp_view(w), dst, st) == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
}

// mat-mat on repacked weights, per call: from this many tokens the int8 tile reads a repacked
// copy of src0 (made in scratch by one extra launch when the caller has none); below it, and for
// layouts the repack does not take, the in-place int8 tile. GGML_MI355X_MMQ_REPACK_MIN overrides
// (measurements: 0 = never repack per call).
static int repack_min_tokens() { return settings().mmq_repack_min; }

int mul_mat(const TensorView &a, const TensorView &b, const TensorView &d, hipStream_t st, Scratch &scratch) {
    return mul_mat_rp(a, nullptr, b, d, st, scratch);
}

// the kernel choice of mul_mat_rp, shared with ggml_mi355x_mul_mat_plan (plan != nullptr:
// describe, launch nothing)
static hipError_t mul_mat_route(const TensorView &a, const void *rp, const MmArgs &m, hipStream_t st, Scratch *scratch,
                                std::string *plan) {
    hipError_t e;
    const int n_mat = (int)(a.ne[2] * a.ne[3]);
    const int rmin = repack_min_tokens();
    // a caller's repacked copy (a 64-token tile) against the in-place tile: the copy wins while the
    // in-place tile runs 64-token tiles (Q8_0 4096 x 4096 x 512 36 vs 41.5 us) and at 512 tokens
    // over >= 256 128-token tiles (N = 11008: Q8_0 85 vs 95 us, Q6_K 124 vs 140; Q4_K 99 vs 95);
    // the in-place 128-token tile wins below 256 such tiles (4096 x 4096 x 768 Q8_0 54 vs 59, Q4_K
    // 55 vs 67) and from 1024 tokens on (x 2048 Q8_0 110 vs 116, Q4_K 109 vs 130, Q6_K 152 vs
    // 164) (profiles/r04_mmq_m_sweep.txt, r04_rp_shape_sweep.txt, r04_mmq8_tt_sweep2.txt). Both
    // are exact: only the fp32 order of the scale sums differs.
    // GGML_MI355X_MMQ_RP_ALL=1: always read the copy (measurements)
    const bool rp_all = settings().mmq_rp_all;
    const bool wide = !rp_all && mmq8_supported(a.type, m) && mmq8_tile_tokens(m) == 128 &&
                      (m.M >= 1024 || mmq8_tiles128(m) < 256);
    const bool use_rp = m.M > 8 && ((rp != nullptr && !wide) || (rmin > 0 && m.M >= rmin)) &&
                        repack_size(a) != 0 && mmq8_images_fit(a.type, m);
    if (plan) {
        if (use_rp) *plan = std::string(rp ? "mmq8r" : "repack+mmq8r") + " tile=128x64";
        else if (m.M > 8 && mmq8_supported(a.type, m)) *plan = mmq8_plan_text(m);
        else (void)run_mmvq(a.type, m, 0, m.M, st, nullptr, plan);
        return hipSuccess;
    }
    if (use_rp) e = mmq8r_launch(a.type, m, rp, (int)a.ne[2], n_mat, st, *scratch);
    else if (m.M > 8 && mmq8_supported(a.type, m)) e = mmq8_launch(a.type, m, st, *scratch);
    else e = run_mmvq(a.type, m, 0, m.M, st, scratch);
    return e;
}

int mul_mat_rp(const TensorView &a, const void *rp, const TensorView &b, const TensorView &d, hipStream_t st,
               Scratch &scratch) {
    const int rc = check_mul_mat(a, b, d);
    if (rc != GGML_MI355X_OK) return rc;
    if (a.ne[1] == 0 || b.ne[1] == 0 || b.ne[2] == 0 || b.ne[3] == 0) return GGML_MI355X_OK;
    const MmArgs m = base_args(a, b, d);
    std::lock_guard<std::mutex> hold(scratch.mu);   // until the scratch users are queued
    const hipError_t e = mul_mat_route(a, rp, m, st, &scratch, nullptr);
    if (e == hipErrorOutOfMemory) return GGML_MI355X_ENOMEM;
    return e == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
}

int check_mul_mat_id(const TensorView &as, const TensorView &b, const TensorView &ids, const TensorView &d) {
    if (!is_hot_quant(as.type) || b.type != T_F32 || ids.type != T_I32 || d.type != T_F32) return GGML_MI355X_EINVAL;
    if (as.ne[0] != b.ne[0] || as.ne[0] % type_blck(as.type) != 0 || as.ne[3] != 1 || b.ne[3] != 1) return GGML_MI355X_EINVAL;
    if (ids.ne[1] != b.ne[2] || b.ne[1] <= 0 || ids.ne[0] % b.ne[1] != 0) return GGML_MI355X_EINVAL;
    if (d.ne[0] != as.ne[1] || d.ne[1] != ids.ne[0] || d.ne[2] != ids.ne[1]) return GGML_MI355X_EINVAL;
    if ((int64_t)as.nb[0] != type_bytes(as.type) || b.nb[0] != 4 || d.nb[0] != 4 || ids.nb[0] != 4) return GGML_MI355X_EINVAL;
    if (mmvq_lds_bytes((int)as.ne[0], 1) > LDS_LIMIT) return GGML_MI355X_EINVAL;
    if (ids.ne[0] * ids.ne[1] > 65535) return GGML_MI355X_EINVAL;
    return GGML_MI355X_OK;
}

// (slot, token) pairs from which the grouped MFMA path beats one mat-vec per pair:
// settings().mmq_id_min, 64 by default

int mul_mat_id(const TensorView &as, const TensorView &b, const TensorView &ids, const TensorView &d, hipStream_t st,
               Scratch &scratch) {
    const int rc = check_mul_mat_id(as, b, ids, d);
    if (rc != GGML_MI355X_OK) return rc;
    if (ids.ne[0] == 0 || ids.ne[1] == 0 || as.ne[1] == 0) return GGML_MI355X_OK;
    MmArgs m{};
    m.w = static_cast<const uint8_t *>(as.data);
    m.nb01 = (int64_t)as.nb[1]; m.nb02 = (int64_t)as.nb[2]; m.nb03 = (int64_t)as.nb[3];
    m.x = static_cast<const uint8_t *>(b.data);
    m.nb11 = (int64_t)b.nb[1]; m.nb12 = (int64_t)b.nb[2]; m.nb13 = (int64_t)b.nb[3];
    m.dst = static_cast<uint8_t *>(d.data);
    m.nb1 = (int64_t)d.nb[1]; m.nb2 = (int64_t)d.nb[2]; m.nb3 = (int64_t)d.nb[3];
    m.K = (int)as.ne[0];
    m.N = (int)as.ne[1];
    m.M = 1;
    m.ne12 = 1; m.ne13 = 1; m.r2 = 1; m.r3 = 1;
    m.ids = static_cast<const int32_t *>(ids.data);
    m.ids_nb0 = (int64_t)ids.nb[0];
    m.ids_nb1 = (int64_t)ids.nb[1];
    m.n_used = (int)ids.ne[0];
    m.n_tok = (int)ids.ne[1];
    m.ne11_b = (int)b.ne[1];
    m.n_expert = (int)as.ne[2];
    m.x_aligned16 = aligned16(b.data, m.nb11, m.nb12, m.nb13);
    const bool grouped = m.n_used * m.n_tok >= settings().mmq_id_min;
    const bool i8 = grouped && mmq8_id_supported(as.type, m);
    std::lock_guard<std::mutex> hold(scratch.mu);
    const hipError_t e = i8 ? mmq8_id_launch(as.type, m, st, scratch) : mmvq_id_launch(as.type, m, 1, st);
    if (e == hipErrorOutOfMemory) return GGML_MI355X_ENOMEM;
    return e == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
}

// ------------------------------------------------------------------------------------------
// device error word: one int in host-mapped pinned memory that kernels raise on a failed
// precondition they can only see on the device (a GET_ROWS index out of range; the reference
// GGML_ASSERTs, src/ggml-cpu/ops.cpp:5157). Read after the stream has synchronized.
// ------------------------------------------------------------------------------------------
// One word per device, made on first use (the backend makes its device's at init, outside any
// stream capture). A failed allocation is not remembered: the next call tries again.
// hipHostMallocPortable: the word is valid whichever device is current when it is read.
static constexpr int ERR_DEVS = 64;
static int *g_err_host[ERR_DEVS], *g_err_dev[ERR_DEVS];
static std::mutex g_err_mu;

int *device_error_word() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= ERR_DEVS) {
        (void)hipGetLastError();
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_err_mu);
    if (g_err_dev[dev]) return g_err_dev[dev];
    void *h = nullptr;
    if (hipHostMalloc(&h, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(h);
        return nullptr;
    }
    *static_cast<int *>(h) = 0;
    g_err_host[dev] = static_cast<int *>(h);
    g_err_dev[dev] = static_cast<int *>(d);
    return g_err_dev[dev];
}

// device < 0: every device's word
int take_device_error(int device) {
    int v = 0;
    for (int i = 0; i < ERR_DEVS; ++i) {
        if (device >= 0 && i != device) continue;
        int *h;
        {
            std::lock_guard<std::mutex> lk(g_err_mu);
            h = g_err_host[i];
        }
        if (h) v |= __atomic_exchange_n(h, 0, __ATOMIC_ACQ_REL);
    }
    return v;
}

int dequantize(int type, const void *src, float *dst, int64_t n, hipStream_t st) {
    if (!is_hot_quant(type) || n < 0 || n % type_blck(type) != 0) return GGML_MI355X_EINVAL;
    if (n == 0) return GGML_MI355X_OK;
    return dequant_launch(type, src, dst, n, st) == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
}

// GET_ROWS (ggml_get_rows, reference src/ggml.c:3617-3637): a [ne00, ne01, ne02, ne03] hot type
// or f32, rows [r, ne02, ne03] i32, dst [ne00, r, ne02, ne03] f32
int check_get_rows(const TensorView &a, const TensorView &r, const TensorView &d) {
    if (!(is_hot_quant(a.type) || a.type == T_F32) || r.type != T_I32 || d.type != T_F32) return GGML_MI355X_EINVAL;
    const int blck = a.type == T_F32 ? 1 : type_blck(a.type);
    if (a.ne[0] % blck != 0 || (int64_t)a.nb[0] != type_bytes(a.type) || r.nb[0] != 4 || d.nb[0] != 4) return GGML_MI355X_EINVAL;
    if (a.ne[2] != r.ne[1] || a.ne[3] != r.ne[2] || r.ne[3] != 1) return GGML_MI355X_EINVAL;
    if (d.ne[0] != a.ne[0] || d.ne[1] != r.ne[0] || d.ne[2] != r.ne[1] || d.ne[3] != r.ne[2]) return GGML_MI355X_EINVAL;
    if (a.ne[1] <= 0 && r.ne[0] > 0) return GGML_MI355X_EINVAL;
    if (r.ne[0] * r.ne[1] * r.ne[2] > 65535) return GGML_MI355X_EINVAL;   // grid.y
    return GGML_MI355X_OK;
}

int get_rows(const TensorView &a, const TensorView &r, const TensorView &d, hipStream_t st) {
    const int rc = check_get_rows(a, r, d);
    if (rc != GGML_MI355X_OK) return rc;
    const int64_t nrows = r.ne[0] * r.ne[1] * r.ne[2];
    if (nrows == 0 || a.ne[0] == 0) return GGML_MI355X_OK;
    RowsArgs g{};
    g.src = static_cast<const uint8_t *>(a.data);
    g.nb01 = (int64_t)a.nb[1]; g.nb02 = (int64_t)a.nb[2]; g.nb03 = (int64_t)a.nb[3]; g.ne01 = a.ne[1];
    g.idx = static_cast<const uint8_t *>(r.data);
    g.nb10 = (int64_t)r.nb[0]; g.nb11 = (int64_t)r.nb[1]; g.nb12 = (int64_t)r.nb[2];
    g.ne10 = r.ne[0]; g.ne11 = r.ne[1];
    g.dst = static_cast<uint8_t *>(d.data);
    g.nb1 = (int64_t)d.nb[1]; g.nb2 = (int64_t)d.nb[2]; g.nb3 = (int64_t)d.nb[3];
    g.ne00 = a.ne[0];
    g.err = device_error_word();
    if (!g.err) return GGML_MI355X_EHIP;
    return get_rows_launch(a.type, g, nrows, st) == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
}

// GET_ROWS(a, ra) + GET_ROWS(b, rb) -> d in one launch (graph fusion of the GPT-2 embedding):
// a hot type or f32, b f32, both 2-D with a 1-D row list of the same length, d [ne00, rows] f32
int get_rows_add(const TensorView &a, const TensorView &ra, const TensorView &b, const TensorView &rb, const TensorView &d,
                 hipStream_t st) {
    int rc = check_get_rows(a, ra, d);
    if (rc == GGML_MI355X_OK) rc = check_get_rows(b, rb, d);
    if (rc != GGML_MI355X_OK) return rc;
    if (b.type != T_F32 || a.ne[2] != 1 || a.ne[3] != 1 || b.ne[2] != 1 || b.ne[3] != 1) return GGML_MI355X_EINVAL;
    if (ra.ne[1] != 1 || ra.ne[2] != 1 || rb.ne[0] != ra.ne[0] || rb.ne[1] != 1 || rb.ne[2] != 1) return GGML_MI355X_EINVAL;
    const int64_t nrows = ra.ne[0];
    if (nrows == 0 || a.ne[0] == 0) return GGML_MI355X_OK;
    auto args = [&](const TensorView &s, const TensorView &r) {
        RowsArgs g{};
        g.src = static_cast<const uint8_t *>(s.data);
        g.nb01 = (int64_t)s.nb[1]; g.nb02 = (int64_t)s.nb[2]; g.nb03 = (int64_t)s.nb[3]; g.ne01 = s.ne[1];
        g.idx = static_cast<const uint8_t *>(r.data);
        g.nb10 = (int64_t)r.nb[0]; g.nb11 = (int64_t)r.nb[1]; g.nb12 = (int64_t)r.nb[2];
        g.ne10 = r.ne[0]; g.ne11 = r.ne[1];
        g.dst = static_cast<uint8_t *>(d.data);
        g.nb1 = (int64_t)d.nb[1]; g.nb2 = (int64_t)d.nb[2]; g.nb3 = (int64_t)d.nb[3];
        g.ne00 = s.ne[0];
        g.err = device_error_word();
        return g;
    };
    if (!device_error_word()) return GGML_MI355X_EHIP;
    return get_rows_add_launch(a.type, args(a, ra), args(b, rb), nrows, st) == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
}

// f32 -> Q4_0 / Q8_0 (GGML_OP_CPY into a quantized tensor)
int check_quantize(const TensorView &s, const TensorView &d) {
    if (s.type != T_F32 || !(d.type == T_Q4_0 || d.type == T_Q8_0)) return GGML_MI355X_EINVAL;
    for (int i = 0; i < 4; ++i)
        if (s.ne[i] != d.ne[i]) return GGML_MI355X_EINVAL;
    if (s.ne[0] % 32 != 0 || s.nb[0] != 4 || (int64_t)d.nb[0] != type_bytes(d.type)) return GGML_MI355X_EINVAL;
    return GGML_MI355X_OK;
}

static int64_t nelements(const TensorView &t) { return t.ne[0] * t.ne[1] * t.ne[2] * t.ne[3]; }

static bool is_contiguous(const TensorView &t) {
    const int blck = t.type == T_F32 ? 1 : type_blck(t.type);
    if ((int64_t)t.nb[0] != type_bytes(t.type) || t.ne[0] % blck != 0) return false;
    const int64_t nb1 = (int64_t)t.nb[0] * (t.ne[0] / blck);
    return (t.ne[1] <= 1 || (int64_t)t.nb[1] == nb1) && (t.ne[2] <= 1 || (int64_t)t.nb[2] == nb1 * t.ne[1]) &&
           (t.ne[3] <= 1 || (int64_t)t.nb[3] == nb1 * t.ne[1] * t.ne[2]);
}

// GGML_OP_CPY (ggml_cpy, reference src/ggml.c; ggml_cuda_cpy src/ggml-cuda/cpy.cu) between the
// types of this path:
//   f32 -> Q4_0 / Q8_0   quantize_row_*_ref (check_quantize: same shape)
//   hot -> f32           dup_q (src/ggml-cpu/ops.cpp:1105-1154): same element count, src blocks
//                        along dim 0, dst rows holding whole blocks or dst contiguous (:1121-1123)
//   hot -> same hot      dup_bytes (ops.cpp:956-1103): same element count, whole blocks per row
int check_cpy(const TensorView &s, const TensorView &d) {
    if (s.type == T_F32 && is_hot_quant(d.type)) return check_quantize(s, d);
    if (!is_hot_quant(s.type) || !(d.type == T_F32 || d.type == s.type)) return GGML_MI355X_EINVAL;
    const int blck = type_blck(s.type);
    for (int i = 0; i < 4; ++i)
        if (s.ne[i] < 0 || d.ne[i] < 0) return GGML_MI355X_EINVAL;
    if (nelements(s) != nelements(d) || s.ne[0] % blck != 0 || (int64_t)s.nb[0] != type_bytes(s.type)) return GGML_MI355X_EINVAL;
    if (d.type == T_F32) {
        if (d.nb[0] != 4 || !(d.ne[0] % blck == 0 || is_contiguous(d))) return GGML_MI355X_EINVAL;
    } else if (d.ne[0] % blck != 0 || (int64_t)d.nb[0] != type_bytes(d.type)) {
        return GGML_MI355X_EINVAL;
    }
    if (nelements(s) > (1LL << 40)) return GGML_MI355X_EINVAL;   // 1-D grid
    return GGML_MI355X_OK;
}

int cpy(const TensorView &s, const TensorView &d, hipStream_t st) {
    if (s.type == T_F32) return quantize(s, d, st);
    const int rc = check_cpy(s, d);
    if (rc != GGML_MI355X_OK) return rc;
    if (nelements(s) == 0) return GGML_MI355X_OK;
    CpyQArgs q{};
    q.src = static_cast<const uint8_t *>(s.data);
    q.ne00 = s.ne[0]; q.ne01 = s.ne[1]; q.ne02 = s.ne[2];
    q.nb00 = (int64_t)s.nb[0]; q.nb01 = (int64_t)s.nb[1]; q.nb02 = (int64_t)s.nb[2]; q.nb03 = (int64_t)s.nb[3];
    q.dst = static_cast<uint8_t *>(d.data);
    q.ne0 = d.ne[0]; q.ne1 = d.ne[1]; q.ne2 = d.ne[2];
    q.nb0 = (int64_t)d.nb[0]; q.nb1 = (int64_t)d.nb[1]; q.nb2 = (int64_t)d.nb[2]; q.nb3 = (int64_t)d.nb[3];
    const bool to_f32 = d.type == T_F32;
    q.n = to_f32 ? nelements(s) : nelements(s) / type_blck(s.type);
    return cpy_q_launch(s.type, to_f32, q, st) == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
}

int quantize(const TensorView &s, const TensorView &d, hipStream_t st) {
    const int rc = check_quantize(s, d);
    if (rc != GGML_MI355X_OK) return rc;
    if (s.ne[0] * s.ne[1] * s.ne[2] * s.ne[3] == 0) return GGML_MI355X_OK;
    QuantArgs q{};
    q.src = static_cast<const uint8_t *>(s.data);
    q.nb01 = (int64_t)s.nb[1]; q.nb02 = (int64_t)s.nb[2]; q.nb03 = (int64_t)s.nb[3];
    q.dst = static_cast<uint8_t *>(d.data);
    q.nb1 = (int64_t)d.nb[1]; q.nb2 = (int64_t)d.nb[2]; q.nb3 = (int64_t)d.nb[3];
    q.ne0 = s.ne[0]; q.ne1 = s.ne[1]; q.ne2 = s.ne[2]; q.ne3 = s.ne[3];
    return quantize_launch(d.type, q, st) == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
}

// ------------------------------------------------------------------------------------------
// scratch: grow-only device buffer, one per (device, stream) user
// ------------------------------------------------------------------------------------------
void *Scratch::get(size_t bytes, hipStream_t st) {
    if (bytes <= cap) return ptr;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess) {
        (void)hipGetLastError();
        cs = hipStreamCaptureStatusNone;
    }
    if (cs != hipStreamCaptureStatusNone) {
        if (!short_in_capture)
            fprintf(stderr, "[ggml-mi355x] scratch of %zu bytes needed inside a hipGraph capture: run the launch once "
                            "eagerly on this stream before capturing it\n", bytes);
        short_in_capture = true;
        return nullptr;
    }
    if (ptr) {
        (void)hipStreamSynchronize(st);    // the only users of the old buffer are on this stream
        (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
    size_t want = std::max(bytes, (size_t)1 << 20);
    want = (want + 0xFFFFF) & ~(size_t)0xFFFFF;
    if (hipMalloc(&ptr, want) != hipSuccess) {
        (void)hipGetLastError();
        ptr = nullptr;
        return nullptr;
    }
    (void)hipGetDevice(&device);
    cap = want;
    ++gen;
    return ptr;
}

int *Scratch::counters(hipStream_t st) {
    if (cnt) return cnt;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess) {
        (void)hipGetLastError();
        cs = hipStreamCaptureStatusNone;
    }
    if (cs != hipStreamCaptureStatusNone) return nullptr;   // (the caller takes its other path)
    void *p = nullptr;
    if (hipMalloc(&p, COUNTERS * sizeof(int)) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (hipMemset(p, 0, COUNTERS * sizeof(int)) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFree(p);
        return nullptr;
    }
    cnt = static_cast<int *>(p);
    return cnt;
}

void Scratch::release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
    ++gen;
    if (cnt) (void)hipFree(cnt);
    cnt = nullptr;
}

Scratch::~Scratch() { release(); }

Scratch &scratch_for(hipStream_t st) {
    static std::mutex mu;
    static auto *reg = new std::map<std::pair<int, hipStream_t>, std::unique_ptr<Scratch>>();   // never destroyed: outlives HIP teardown
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lock(mu);
    auto &p = (*reg)[{dev, st}];
    if (!p) p = std::make_unique<Scratch>();
    return *p;
}

}  // namespace mi355x

// ==========================================================================================
// direct C API (include/ggml-mi355x.h)
// ==========================================================================================
using namespace mi355x;

static TensorView view_of(const ggml_mi355x_tensor *t) {
    TensorView v;
    v.type = t->type;
    v.data = t->data;
    for (int i = 0; i < 4; ++i) {
        v.ne[i] = t->ne[i];
        v.nb[i] = t->nb[i];
    }
    return v;
}


extern "C" {

int ggml_mi355x_mul_mat(const ggml_mi355x_tensor *src0, const ggml_mi355x_tensor *src1, ggml_mi355x_tensor *dst,
                        void *stream) {
    if (!src0 || !src1 || !dst) return GGML_MI355X_EINVAL;
    return mul_mat(view_of(src0), view_of(src1), view_of(dst), static_cast<hipStream_t>(stream),
                  scratch_for(static_cast<hipStream_t>(stream)));
}

int ggml_mi355x_repack_size(const ggml_mi355x_tensor *src0, size_t *bytes) {
    if (!src0 || !bytes) return GGML_MI355X_EINVAL;
    *bytes = repack_size(view_of(src0));
    return *bytes ? GGML_MI355X_OK : GGML_MI355X_EINVAL;
}

int ggml_mi355x_repack(const ggml_mi355x_tensor *src0, void *dst, size_t bytes, void *stream) {
    if (!src0) return GGML_MI355X_EINVAL;
    return repack(view_of(src0), dst, bytes, static_cast<hipStream_t>(stream));
}

int ggml_mi355x_mul_mat_repacked(const ggml_mi355x_tensor *src0, const void *repacked, const ggml_mi355x_tensor *src1,
                                 ggml_mi355x_tensor *dst, void *stream) {
    if (!src0 || !src1 || !dst || !repacked) return GGML_MI355X_EINVAL;
    if (repack_size(view_of(src0)) == 0) return GGML_MI355X_EINVAL;
    return mul_mat_rp(view_of(src0), repacked, view_of(src1), view_of(dst), static_cast<hipStream_t>(stream),
                      scratch_for(static_cast<hipStream_t>(stream)));
}

int ggml_mi355x_mul_mat_id(const ggml_mi355x_tensor *as, const ggml_mi355x_tensor *b, const ggml_mi355x_tensor *ids,
                           ggml_mi355x_tensor *dst, void *stream) {
    if (!as || !b || !ids || !dst) return GGML_MI355X_EINVAL;
    return mul_mat_id(view_of(as), view_of(b), view_of(ids), view_of(dst), static_cast<hipStream_t>(stream),
                      scratch_for(static_cast<hipStream_t>(stream)));
}

int ggml_mi355x_dequantize(int32_t type, const void *src, float *dst, int64_t n, void *stream) {
    return dequantize(type, src, dst, n, static_cast<hipStream_t>(stream));
}

int ggml_mi355x_get_rows(const ggml_mi355x_tensor *src0, const ggml_mi355x_tensor *rows, ggml_mi355x_tensor *dst,
                         void *stream) {
    if (!src0 || !rows || !dst) return GGML_MI355X_EINVAL;
    return get_rows(view_of(src0), view_of(rows), view_of(dst), static_cast<hipStream_t>(stream));
}

int ggml_mi355x_device_error(void) { return take_device_error(-1); }

int ggml_mi355x_cpy(const ggml_mi355x_tensor *src, ggml_mi355x_tensor *dst, void *stream) {
    if (!src || !dst) return GGML_MI355X_EINVAL;
    return cpy(view_of(src), view_of(dst), static_cast<hipStream_t>(stream));
}

int ggml_mi355x_quantize(const ggml_mi355x_tensor *src, ggml_mi355x_tensor *dst, void *stream) {
    if (!src || !dst) return GGML_MI355X_EINVAL;
    return quantize(view_of(src), view_of(dst), static_cast<hipStream_t>(stream));
}

int ggml_mi355x_supports_mul_mat(const ggml_mi355x_tensor *src0, const ggml_mi355x_tensor *src1) {
    if (!src0 || !src1) return 0;
    return is_hot_quant(src0->type) && src1->type == T_F32 && src0->ne[0] % type_blck(src0->type) == 0 &&
           src0->ne[0] <= (1 << 24);
}

// the MUL_MAT_ID geometry mul_mat_id accepts (check_mul_mat_id on the dst ggml_mul_mat_id makes:
// [N, n_used, T] f32), so that supports_op never claims what compute would refuse (whole-K
// activations in LDS: K up to ~108K)
int ggml_mi355x_supports_mul_mat_id(const ggml_mi355x_tensor *as, const ggml_mi355x_tensor *b, const ggml_mi355x_tensor *ids) {
    if (!as || !b || !ids) return 0;
    TensorView d{};
    d.type = T_F32;
    d.ne[0] = as->ne[1]; d.ne[1] = ids->ne[0]; d.ne[2] = ids->ne[1]; d.ne[3] = 1;
    d.nb[0] = 4; d.nb[1] = 4 * d.ne[0]; d.nb[2] = d.nb[1] * d.ne[1]; d.nb[3] = d.nb[2] * d.ne[2];
    return check_mul_mat_id(view_of(as), view_of(b), view_of(ids), d) == GGML_MI355X_OK;
}

int ggml_mi355x_reload_settings(void) {
    reload_settings();
    return GGML_MI355X_OK;
}

int ggml_mi355x_mul_mat_plan(const ggml_mi355x_tensor *src0, const ggml_mi355x_tensor *src1, int repacked, char *buf,
                             size_t len) {
    if (!src0 || !src1 || !buf || len == 0) return GGML_MI355X_EINVAL;
    const TensorView a = view_of(src0), b = view_of(src1);
    TensorView d{};
    d.type = T_F32;
    d.ne[0] = a.ne[1]; d.ne[1] = b.ne[1]; d.ne[2] = b.ne[2]; d.ne[3] = b.ne[3];
    d.nb[0] = 4; d.nb[1] = 4 * d.ne[0]; d.nb[2] = d.nb[1] * d.ne[1]; d.nb[3] = d.nb[2] * d.ne[2];
    const int rc = check_mul_mat(a, b, d);
    if (rc != GGML_MI355X_OK) return rc;
    std::string plan;
    if (a.ne[1] == 0 || b.ne[1] == 0 || b.ne[2] == 0 || b.ne[3] == 0) {
        plan = "none";
    } else {
        MmArgs m = base_args(a, b, d);
        static const uint8_t rp_token = 0;   // any non-null copy: only its presence routes
        (void)mul_mat_route(a, repacked ? &rp_token : nullptr, m, nullptr, nullptr, &plan);
    }
    snprintf(buf, len, "%s", plan.c_str());
    return GGML_MI355X_OK;
}

int ggml_mi355x_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int good = 0;
    for (int i = 0; i < n; ++i) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, i) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0) ++good;
    }
    return good;
}

// diagnostics only (not in the public header): copy the last launch's workgroup stamps
__attribute__((visibility("default"))) int ggml_mi355x_debug_stamps(unsigned long long *host, size_t n) {
    if (!g_stamps) return -1;
    if (n > STAMP_SLOTS) n = STAMP_SLOTS;
    return hipMemcpy(host, g_stamps, n * sizeof(unsigned long long), hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}

const char *ggml_mi355x_strerror(int status) {
    switch (status) {
        case GGML_MI355X_OK: return "ok";
        case GGML_MI355X_EINVAL: return "unsupported type or inconsistent shapes/strides";
        case GGML_MI355X_ENOMEM: return "device scratch allocation failed (or needed growth inside a hipGraph capture)";
        case GGML_MI355X_EHIP: return "HIP runtime error";
        case GGML_MI355X_ENODEV: return "no gfx950 device";
        default: return "unknown status";
    }
}

}  // extern "C"
