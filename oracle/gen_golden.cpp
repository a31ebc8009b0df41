// oracle/gen_golden.cpp — golden-vector generator (TEST INFRASTRUCTURE, run in the build
// container only). Linked against the REFERENCE ggml (oracle/_ref/libggml-ref.so, built from
// /root/reference sources in place by oracle/ref.mk). Writes small fixtures under
// tests/golden/ (+ manifest.json) that pin oracle/qref.c and, through it, the GPU kernels.
//
//   ./oracle/_ref/gen_golden tests/golden
//
// Inputs are produced by the portable splitmix64 generator (qref_fill_uniform, restated
// identically in numpy) so tests can regenerate them without storing megabytes; each record
// stores the seeds plus the reference's outputs (and sha256-free byte sizes for the big cases).
//
// Reference entry points exercised:
//   ggml_quantize_chunk (src/ggml.c:6989), ggml_get_type_traits()->to_float,
//   ggml_get_type_traits_cpu()->{from_float, vec_dot} (src/ggml-cpu/ggml-cpu.c:209-357),
//   ggml_vec_dot_*_generic (src/ggml-cpu/quants.c), quantize_row_q8_0_ref / q8_1_ref / q8_K_ref,
//   and full MUL_MAT / MUL_MAT_ID graphs on the CPU backend (src/ggml-cpu/ggml-cpu.c:1202,1476).
#include "ggml.h"
#include "ggml-alloc.h"
#include "ggml-backend.h"
#include "ggml-cpu.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
void quantize_row_q8_0_ref(const float *x, void *y, int64_t k);
void quantize_row_q8_1_ref(const float *x, void *y, int64_t k);
void quantize_row_q8_K_ref(const float *x, void *y, int64_t k);
void ggml_vec_dot_q4_0_q8_0_generic(int, float *, size_t, const void *, size_t, const void *, size_t, int);
void ggml_vec_dot_q8_0_q8_0_generic(int, float *, size_t, const void *, size_t, const void *, size_t, int);
void ggml_vec_dot_q4_K_q8_K_generic(int, float *, size_t, const void *, size_t, const void *, size_t, int);
void ggml_vec_dot_q5_K_q8_K_generic(int, float *, size_t, const void *, size_t, const void *, size_t, int);
void ggml_vec_dot_q6_K_q8_K_generic(int, float *, size_t, const void *, size_t, const void *, size_t, int);
}

static void fill_uniform(float *dst, int64_t n, uint64_t seed, float lo, float hi) {
    for (int64_t i = 0; i < n; ++i) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const float u = (float)(z >> 40) * 0x1.0p-24f;
        dst[i] = lo + (hi - lo) * u;
    }
}

static std::string g_dir;
static std::string g_manifest;
static bool g_first = true;

static void write_bin(const std::string &name, const void *p, size_t n) {
    std::string path = g_dir + "/" + name;
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) { perror(path.c_str()); exit(1); }
    fwrite(p, 1, n, f);
    fclose(f);
}

static void record(const std::string &json) {
    g_manifest += g_first ? "  " : ",\n  ";
    g_manifest += json;
    g_first = false;
}

static const ggml_type HOT[] = {GGML_TYPE_Q4_0, GGML_TYPE_Q8_0, GGML_TYPE_Q4_K, GGML_TYPE_Q5_K, GGML_TYPE_Q6_K};

// ---------------------------------------------------------------------------------------
// (i) weight quantization + dequantization, (ii) activation quantization, (iii) vec_dot
// ---------------------------------------------------------------------------------------
static void gen_quant() {
    const int64_t n = 4096;
    std::vector<float> cosx(n), unif(n), ones(n, 1.0f);
    for (int64_t i = 0; i < n; ++i) cosx[i] = 0.1f + 2 * cosf(i + 0.0f);   // test-quantize-fns.cpp:31-35
    fill_uniform(unif.data(), n, 1234, -1.0f, 1.0f);
    write_bin("input_cos.f32", cosx.data(), n * 4);
    write_bin("input_unif1234.f32", unif.data(), n * 4);

    struct { const char *tag; const float *x; } inputs[] = {{"cos", cosx.data()}, {"unif1234", unif.data()}};
    for (ggml_type t : HOT) {
        const char *tn = ggml_type_name(t);
        const size_t rs = ggml_row_size(t, n);
        for (auto &in : inputs) {
            // imx: 0 = no imatrix (_ref), 1 = ones with n_per_row = 4096, 2 = ones with n_per_row = block
            for (int imx = 0; imx < 3; ++imx) {
                std::vector<uint8_t> q(rs, 0);
                std::vector<float> dq(n);
                const int64_t npr = imx == 2 ? ggml_blck_size(t) : n;
                ggml_quantize_chunk(t, in.x, q.data(), 0, n / npr, npr, imx ? ones.data() : nullptr);
                ggml_get_type_traits(t)->to_float(q.data(), dq.data(), n);
                char name[128];
                snprintf(name, sizeof name, "quant_%s_%s_imx%d", tn, in.tag, imx);
                write_bin(std::string(name) + ".q", q.data(), q.size());
                write_bin(std::string(name) + ".deq.f32", dq.data(), n * 4);
                char js[512];
                snprintf(js, sizeof js,
                         "{\"kind\": \"quant\", \"name\": \"%s\", \"type\": \"%s\", \"type_id\": %d, \"input\": \"input_%s.f32\", "
                         "\"n\": %lld, \"imatrix\": %d, \"n_per_row\": %lld}",
                         name, tn, (int)t, in.tag, (long long)n, imx, (long long)npr);
                record(js);
            }
        }
    }

    // activation quantization: reference _ref quantizers and the x86 SIMD from_float actually used
    for (auto &in : inputs) {
        std::vector<uint8_t> a(ggml_row_size(GGML_TYPE_Q8_K, n) + 64, 0);
        quantize_row_q8_0_ref(in.x, a.data(), n);
        write_bin(std::string("act_q8_0_ref_") + in.tag + ".q", a.data(), ggml_row_size(GGML_TYPE_Q8_0, n));
        std::fill(a.begin(), a.end(), 0);
        ggml_get_type_traits_cpu(GGML_TYPE_Q8_0)->from_float(in.x, a.data(), n);
        write_bin(std::string("act_q8_0_x86_") + in.tag + ".q", a.data(), ggml_row_size(GGML_TYPE_Q8_0, n));
        std::fill(a.begin(), a.end(), 0);
        quantize_row_q8_1_ref(in.x, a.data(), n);
        write_bin(std::string("act_q8_1_ref_") + in.tag + ".q", a.data(), ggml_row_size(GGML_TYPE_Q8_1, n));
        std::fill(a.begin(), a.end(), 0);
        ggml_get_type_traits_cpu(GGML_TYPE_Q8_K)->from_float(in.x, a.data(), n);
        write_bin(std::string("act_q8_K_") + in.tag + ".q", a.data(), ggml_row_size(GGML_TYPE_Q8_K, n));
        char js[256];
        snprintf(js, sizeof js, "{\"kind\": \"act\", \"input\": \"input_%s.f32\", \"tag\": \"%s\", \"n\": %lld}", in.tag, in.tag, (long long)n);
        record(js);
    }

    // vec_dot: weights = _ref-quantized seed 1234, activations = from_float(vec_dot_type) of seed 5678
    std::vector<float> act(n);
    fill_uniform(act.data(), n, 5678, -1.0f, 1.0f);
    write_bin("input_unif5678.f32", act.data(), n * 4);
    typedef void (*dotfn)(int, float *, size_t, const void *, size_t, const void *, size_t, int);
    const dotfn generic[] = {ggml_vec_dot_q4_0_q8_0_generic, ggml_vec_dot_q8_0_q8_0_generic,
                             ggml_vec_dot_q4_K_q8_K_generic, ggml_vec_dot_q5_K_q8_K_generic,
                             ggml_vec_dot_q6_K_q8_K_generic};
    for (int ti = 0; ti < 5; ++ti) {
        const ggml_type t = HOT[ti];
        const auto *tr = ggml_get_type_traits_cpu(t);
        for (int64_t k : {256, 1024, 4096}) {
            std::vector<uint8_t> w(ggml_row_size(t, k)), a(ggml_row_size(tr->vec_dot_type, k));
            ggml_quantize_chunk(t, unif.data(), w.data(), 0, 1, k, nullptr);
            ggml_get_type_traits_cpu(tr->vec_dot_type)->from_float(act.data(), a.data(), k);
            float s_gen = 0, s_simd = 0;
            generic[ti]((int)k, &s_gen, 0, w.data(), 0, a.data(), 0, 1);
            tr->vec_dot((int)k, &s_simd, 0, w.data(), 0, a.data(), 0, 1);
            uint32_t bg, bs;
            memcpy(&bg, &s_gen, 4);
            memcpy(&bs, &s_simd, 4);
            char js[384];
            snprintf(js, sizeof js,
                     "{\"kind\": \"vec_dot\", \"type\": \"%s\", \"type_id\": %d, \"k\": %lld, \"w_seed\": 1234, \"a_seed\": 5678, "
                     "\"generic_bits\": %u, \"simd_bits\": %u, \"generic\": %.9g, \"simd\": %.9g}",
                     ggml_type_name(t), (int)t, (long long)k, bg, bs, s_gen, s_simd);
            record(js);
        }
    }
}

// ---------------------------------------------------------------------------------------
// (iv) MUL_MAT / (v) MUL_MAT_ID on the CPU backend
// ---------------------------------------------------------------------------------------
struct Graph {
    ggml_context *ctx = nullptr;
    ggml_backend_t be = nullptr;
    ggml_backend_buffer_t buf = nullptr;
    ~Graph() {
        if (buf) ggml_backend_buffer_free(buf);
        if (ctx) ggml_free(ctx);
    }
};

static ggml_backend_t cpu_backend() {
    static ggml_backend_t be = nullptr;
    if (!be) {
        be = ggml_backend_cpu_init();
        ggml_backend_cpu_set_n_threads(be, 8);
    }
    return be;
}

// quantize an f32 tensor's physical contents (all rows of ne0) with the _ref quantizer
static void set_weights(ggml_tensor *t, uint64_t seed) {
    const int64_t nel = ggml_nelements(t);
    std::vector<float> f(nel);
    fill_uniform(f.data(), nel, seed, -1.0f, 1.0f);
    if (t->type == GGML_TYPE_F32) {
        ggml_backend_tensor_set(t, f.data(), 0, nel * 4);
        return;
    }
    std::vector<uint8_t> q(ggml_nbytes(t));
    ggml_quantize_chunk(t->type, f.data(), q.data(), 0, nel / t->ne[0], t->ne[0], nullptr);
    ggml_backend_tensor_set(t, q.data(), 0, q.size());
}

static void set_f32(ggml_tensor *t, uint64_t seed) {
    const int64_t nel = ggml_nelements(t);
    std::vector<float> f(nel);
    fill_uniform(f.data(), nel, seed, -1.0f, 1.0f);
    ggml_backend_tensor_set(t, f.data(), 0, nel * 4);
}

static int g_mm_id = 0;

// mirrors test_mul_mat::build_graph (tests/test-backend-ops.cpp:3127-3191)
static void gen_mul_mat(ggml_type ta, int64_t m, int64_t n, int64_t k, int bs0, int bs1, int nr0, int nr1,
                        const int per[4], bool view, int64_t store_cols = -1) {
    Graph g;
    ggml_init_params ip = {64 * ggml_tensor_overhead() + ggml_graph_overhead(), nullptr, true};
    g.ctx = ggml_init(ip);
    const bool permuted = per[0] != 0 || per[1] != 1 || per[2] != 2 || per[3] != 3;
    ggml_tensor *a, *b, *a_phys, *b_phys;
    const int64_t ne_a[4] = {k, m, bs0, bs1};
    const int64_t ne_b[4] = {k, n, (int64_t)bs0 * nr0, (int64_t)bs1 * nr1};
    if (permuted) {
        a_phys = ggml_new_tensor_4d(g.ctx, ta, ne_a[per[0]], ne_a[per[1]], ne_a[per[2]], ne_a[per[3]]);
        b_phys = ggml_new_tensor_4d(g.ctx, GGML_TYPE_F32, ne_b[per[0]], ne_b[per[1]], ne_b[per[2]], ne_b[per[3]]);
        a = ggml_permute(g.ctx, a_phys, per[0], per[1], per[2], per[3]);
        b = ggml_permute(g.ctx, b_phys, per[0], per[1], per[2], per[3]);
    } else if (view) {
        a_phys = ggml_new_tensor_4d(g.ctx, ta, k * 2, m, bs0, bs1);
        b_phys = ggml_new_tensor_4d(g.ctx, GGML_TYPE_F32, k * 2, n, (int64_t)bs0 * nr0, (int64_t)bs1 * nr1);
        a = ggml_view_4d(g.ctx, a_phys, k, m, bs0, bs1, a_phys->nb[1], a_phys->nb[2], a_phys->nb[3], 0);
        b = ggml_view_4d(g.ctx, b_phys, k, n, (int64_t)bs0 * nr0, (int64_t)bs1 * nr1, b_phys->nb[1], b_phys->nb[2], b_phys->nb[3], 0);
    } else {
        a = a_phys = ggml_new_tensor_4d(g.ctx, ta, k, m, bs0, bs1);
        b = b_phys = ggml_new_tensor_4d(g.ctx, GGML_TYPE_F32, k, n, (int64_t)bs0 * nr0, (int64_t)bs1 * nr1);
    }
    ggml_tensor *out = ggml_mul_mat(g.ctx, a, b);
    ggml_cgraph *gf = ggml_new_graph(g.ctx);
    ggml_build_forward_expand(gf, out);
    g.buf = ggml_backend_alloc_ctx_tensors(g.ctx, cpu_backend());
    const uint64_t sa = 1000 + 2 * g_mm_id, sb = 1001 + 2 * g_mm_id;
    set_weights(a_phys, sa);
    set_f32(b_phys, sb);
    ggml_backend_graph_compute(cpu_backend(), gf);
    const int64_t cols = out->ne[1] * out->ne[2] * out->ne[3];
    std::vector<float> res(ggml_nelements(out));
    ggml_backend_tensor_get(out, res.data(), 0, res.size() * 4);
    char name[160];
    snprintf(name, sizeof name, "mm_%03d_%s_m%lld_n%lld_k%lld", g_mm_id, ggml_type_name(ta), (long long)m, (long long)n, (long long)k);
    size_t nstore = res.size();
    std::string sample_js, colsum_js;
    if (store_cols > 0 && store_cols < cols) {
        // big case: the reference's output is stored for a strided sample of columns that
        // touches every 128-column tile (its first 8 columns, every 16th, the tile edges), and
        // every column is pinned by its (sum, sum of squares) in f64
        std::vector<int64_t> pick;
        for (int64_t c = 0; c < cols; ++c)
            if (c < store_cols || c % 16 == 15 || c % 128 == 0 || c % 128 == 127 || c == cols - 1) pick.push_back(c);
        std::vector<float> sub;
        for (int64_t c : pick) sub.insert(sub.end(), res.begin() + c * out->ne[0], res.begin() + (c + 1) * out->ne[0]);
        write_bin(std::string(name) + ".out.f32", sub.data(), sub.size() * 4);
        nstore = sub.size();
        sample_js = ", \"sample_cols\": [";
        for (size_t i = 0; i < pick.size(); ++i) sample_js += (i ? ", " : "") + std::to_string(pick[i]);
        sample_js += "]";
        std::vector<double> cs(2 * cols);
        for (int64_t c = 0; c < cols; ++c) {
            double s1 = 0, s2 = 0;
            for (int64_t i = 0; i < out->ne[0]; ++i) {
                const double v = res[c * out->ne[0] + i];
                s1 += v;
                s2 += v * v;
            }
            cs[2 * c] = s1;
            cs[2 * c + 1] = s2;
        }
        write_bin(std::string(name) + ".colsums.f64", cs.data(), cs.size() * 8);
        colsum_js = ", \"colsums\": \"" + std::string(name) + ".colsums.f64\"";
    } else {
        write_bin(std::string(name) + ".out.f32", res.data(), nstore * 4);
    }
    char js[4096];
    snprintf(js, sizeof js,
             "{\"kind\": \"mul_mat\", \"name\": \"%s\", \"type\": \"%s\", \"type_id\": %d, \"m\": %lld, \"n\": %lld, \"k\": %lld, "
             "\"bs\": [%d, %d], \"nr\": [%d, %d], \"per\": [%d, %d, %d, %d], \"view\": %s, "
             "\"a_ne\": [%lld, %lld, %lld, %lld], \"b_ne\": [%lld, %lld, %lld, %lld], \"seed_a\": %llu, \"seed_b\": %llu, "
             "\"out_ne\": [%lld, %lld, %lld, %lld], \"stored_floats\": %zu%s%s}",
             name, ggml_type_name(ta), (int)ta, (long long)m, (long long)n, (long long)k, bs0, bs1, nr0, nr1,
             per[0], per[1], per[2], per[3], view ? "true" : "false",
             (long long)a_phys->ne[0], (long long)a_phys->ne[1], (long long)a_phys->ne[2], (long long)a_phys->ne[3],
             (long long)b_phys->ne[0], (long long)b_phys->ne[1], (long long)b_phys->ne[2], (long long)b_phys->ne[3],
             (unsigned long long)sa, (unsigned long long)sb,
             (long long)out->ne[0], (long long)out->ne[1], (long long)out->ne[2], (long long)out->ne[3], nstore,
             sample_js.c_str(), colsum_js.c_str());
    record(js);
    ++g_mm_id;
}

// deterministic expert routing: row t holds (i % n_mats) shuffled by splitmix (Fisher-Yates)
static void make_ids(std::vector<int32_t> &ids, int n_mats, int64_t n, uint64_t seed) {
    ids.resize((size_t)n_mats * n);
    std::vector<float> r((size_t)n_mats * n);
    fill_uniform(r.data(), (int64_t)r.size(), seed, 0.0f, 1.0f);
    for (int64_t t = 0; t < n; ++t) {
        int32_t *row = ids.data() + t * n_mats;
        for (int i = 0; i < n_mats; ++i) row[i] = i % n_mats;
        for (int i = n_mats - 1; i > 0; --i) {
            int j = (int)(r[t * n_mats + i] * (i + 1));
            if (j > i) j = i;
            std::swap(row[i], row[j]);
        }
    }
}

// mirrors test_mul_mat_id::build_graph (tests/test-backend-ops.cpp:3226-3246)
static void gen_mul_mat_id(ggml_type ta, int n_mats, int n_used, bool bcast, int64_t m, int64_t n, int64_t k) {
    Graph g;
    ggml_init_params ip = {64 * ggml_tensor_overhead() + ggml_graph_overhead(), nullptr, true};
    g.ctx = ggml_init(ip);
    ggml_tensor *as = ggml_new_tensor_3d(g.ctx, ta, k, m, n_mats);
    ggml_tensor *ids_full = ggml_new_tensor_2d(g.ctx, GGML_TYPE_I32, n_mats, n);
    ggml_tensor *ids = n_used != n_mats ? ggml_view_2d(g.ctx, ids_full, n_used, n, ids_full->nb[1], 0) : ids_full;
    ggml_tensor *b = ggml_new_tensor_3d(g.ctx, GGML_TYPE_F32, k, bcast ? 1 : n_used, n);
    ggml_tensor *out = ggml_mul_mat_id(g.ctx, as, b, ids);
    ggml_cgraph *gf = ggml_new_graph(g.ctx);
    ggml_build_forward_expand(gf, out);
    g.buf = ggml_backend_alloc_ctx_tensors(g.ctx, cpu_backend());
    const uint64_t sa = 1000 + 2 * g_mm_id, sb = 1001 + 2 * g_mm_id, si = 7000 + g_mm_id;
    set_weights(as, sa);
    set_f32(b, sb);
    std::vector<int32_t> idv;
    make_ids(idv, n_mats, n, si);
    ggml_backend_tensor_set(ids_full, idv.data(), 0, idv.size() * 4);
    ggml_backend_graph_compute(cpu_backend(), gf);
    std::vector<float> res(ggml_nelements(out));
    ggml_backend_tensor_get(out, res.data(), 0, res.size() * 4);
    char name[160];
    snprintf(name, sizeof name, "mmid_%03d_%s_e%d_u%d_b%d_n%lld", g_mm_id, ggml_type_name(ta), n_mats, n_used, (int)bcast, (long long)n);
    write_bin(std::string(name) + ".out.f32", res.data(), res.size() * 4);
    write_bin(std::string(name) + ".ids.i32", idv.data(), idv.size() * 4);
    char js[768];
    snprintf(js, sizeof js,
             "{\"kind\": \"mul_mat_id\", \"name\": \"%s\", \"type\": \"%s\", \"type_id\": %d, \"n_mats\": %d, \"n_used\": %d, "
             "\"b\": %s, \"m\": %lld, \"n\": %lld, \"k\": %lld, \"seed_a\": %llu, \"seed_b\": %llu, "
             "\"out_ne\": [%lld, %lld, %lld, %lld]}",
             name, ggml_type_name(ta), (int)ta, n_mats, n_used, bcast ? "true" : "false", (long long)m, (long long)n, (long long)k,
             (unsigned long long)sa, (unsigned long long)sb,
             (long long)out->ne[0], (long long)out->ne[1], (long long)out->ne[2], (long long)out->ne[3]);
    record(js);
    ++g_mm_id;
}

int main(int argc, char **argv) {
    g_dir = argc > 1 ? argv[1] : "tests/golden";
    ggml_cpu_init();
    gen_quant();

    const int id4[4] = {0, 1, 2, 3};
    for (ggml_type t : HOT) {
        for (int n = 1; n <= 9; ++n) gen_mul_mat(t, 16, n, 256, 1, 1, 1, 1, id4, false);
        gen_mul_mat(t, 16, 16, 256, 1, 1, 1, 1, id4, false);
    }
    const ggml_type base[] = {GGML_TYPE_Q4_0, GGML_TYPE_Q8_0, GGML_TYPE_Q4_K};
    const int pers[3][4] = {{0, 2, 1, 3}, {0, 1, 3, 2}, {0, 3, 2, 1}};
    for (ggml_type t : base) {
        for (int n : {1, 16}) {
            gen_mul_mat(t, 16, n, 256, 3, 2, 2, 2, id4, false);
            gen_mul_mat(t, 16, n, 256, 3, 1, 2, 1, id4, false);
            gen_mul_mat(t, 16, n, 256, 1, 1, 1, 2, id4, false);
        }
        for (int p = 0; p < 3; ++p) gen_mul_mat(t, 16, 8, 256, 2, 3, 1, 1, pers[p], false);
        gen_mul_mat(t, 16, 4, 256, 1, 1, 1, 1, id4, true);
        gen_mul_mat(t, 16, 16, 256, 2, 1, 1, 1, id4, true);
        gen_mul_mat(t, 16, 8, 1024, 3, 2, 1, 1, id4, false);
        gen_mul_mat(t, 33, 64, 1024, 1, 1, 1, 1, id4, false);    // ragged MFMA tiles
    }
    gen_mul_mat(GGML_TYPE_Q8_0, 16, 1, 32, 1, 1, 1, 1, id4, false);   // other_types k = blck
    for (ggml_type t : HOT) gen_mul_mat(t, 256, 129, 512, 1, 1, 1, 1, id4, false);
    // BASELINE.json configs (K = 4096)
    gen_mul_mat(GGML_TYPE_Q4_0, 4096, 1, 4096, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_K, 4096, 1, 4096, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_K, 11008, 1, 4096, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q5_K, 11008, 1, 4096, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q6_K, 11008, 1, 4096, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q8_0, 4096, 512, 4096, 1, 1, 1, 1, id4, false, 8);

    for (ggml_type t : HOT) {
        for (int n : {1, 32}) gen_mul_mat_id(t, 4, 2, false, 512, n, 256);
        gen_mul_mat_id(t, 8, 4, true, 64, 129, 256);
    }
    gen_mul_mat_id(GGML_TYPE_Q4_0, 8, 1, false, 128, 129, 256);

    // round 5: the chunked-K mat-vec (mmvq_ring.hip) — K past one 4096 chunk at 1..8 columns,
    // the reference's perf shapes' K (test-backend-ops.cpp:6195-6201, K = 14336) and LLaMA's
    // FFN-down K = 11008; ragged K (K % 64 == 32), a partial last chunk, broadcast batches, one
    // full-size 4096 x 14336 x 8 and K = 131072 (past the whole-K kernel's LDS)
    for (ggml_type t : HOT)
        for (int64_t k : {11008, 14336})
            for (int n : {1, 2, 5, 8}) gen_mul_mat(t, 256, n, k, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_0, 200, 3, 14368, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q8_0, 200, 7, 14368, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_K, 333, 7, 12288, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q6_K, 96, 4, 9216, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q8_0, 64, 4, 8192, 2, 1, 2, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q5_K, 48, 3, 8192, 1, 1, 1, 1, id4, true);
    gen_mul_mat(GGML_TYPE_Q4_0, 4096, 8, 14336, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_0, 16, 1, 131072, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q6_K, 16, 2, 131072, 1, 1, 1, 1, id4, false);

    // round 5, later: the int8-MFMA mat-vec's default forms (dispatch.cpp mma_min_cols) — paired
    // steps at 4 tokens (Q4_0 from 4 columns, Q8_0 from 3 at K = 14336), the K-quants' 8-token
    // form (Q4_K at K = 11008, Q5_K at K = 4096) and the wide-N rule (N = 8192 at K = 4096)
    gen_mul_mat(GGML_TYPE_Q4_0, 256, 4, 14336, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q8_0, 256, 3, 14336, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q8_0, 256, 4, 14336, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_K, 256, 6, 11008, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q5_K, 256, 6, 4096, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_0, 8192, 5, 4096, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_K, 8192, 8, 4096, 1, 1, 1, 1, id4, false);

    // round 6: the MFMA mat-vec's forms at K = 8192 / 28672 (one and two K parts, paired and
    // unpaired steps, 4- and 8-token column packing), the shapes whose MFMA run would not fit the
    // launcher's image (paired Q4_0 K = 25600 at 5..8 columns, Q4_K K = 49408 at 3: the VALU kernels
    // take them) and Q6_K at the reference perf harness's 8-column shape in full
    // (test-backend-ops.cpp:6195-6202, N = 4096, K = 14336)
    gen_mul_mat(GGML_TYPE_Q4_0, 256, 5, 8192, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_K, 256, 3, 8192, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q8_0, 256, 8, 8192, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_0, 256, 8, 28672, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q8_0, 256, 5, 28672, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_K, 256, 8, 28672, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q5_K, 256, 8, 28672, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_0, 64, 5, 25600, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q4_K, 64, 3, 49408, 1, 1, 1, 1, id4, false);
    gen_mul_mat(GGML_TYPE_Q6_K, 4096, 8, 14336, 1, 1, 1, 1, id4, false);

    std::string path = g_dir + "/manifest.json";
    FILE *f = fopen(path.c_str(), "w");
    fprintf(f, "{\n\"generator\": \"oracle/gen_golden.cpp linked to oracle/_ref/libggml-ref.so (reference sources, oracle/ref.mk)\",\n"
               "\"prng\": \"splitmix64 counter mode, see oracle/qref.c qref_fill_uniform\",\n\"records\": [\n%s\n]\n}\n",
            g_manifest.c_str());
    fclose(f);
    printf("wrote %s\n", path.c_str());
    return 0;
}
