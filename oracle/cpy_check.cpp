// oracle/cpy_check.cpp — TEST INFRASTRUCTURE ONLY (never part of the product path).
//
// A seeded sweep of the GGML_OP_CPY cases the reference's test-backend-ops runs
// (tests/test-backend-ops.cpp:5574-5602, struct test_cpy :2383-2435), on our plugin against
// ggml-cpu, through the reference's graph API. test-backend-ops seeds its inputs from
// std::random_device (:50-56), so one of its runs sees one draw per case; this draws `seeds`
// inputs per case from fixed seeds, so a rare input-dependent mismatch shows up and can be
// replayed. Per case and seed:
//   * src and dst are filled as init_tensor_uniform fills them (:42-120): uniform [-1, 1],
//     quantized types through ggml_quantize_chunk, with or without the dummy importance matrix
//     by the same first-value rule;
//   * the CPY graph is built as test_cpy builds it (src permuted, dst permuted, ggml_cpy);
//   * both dst tensors are read back whole and converted to f32 (the type's to_float), and the
//     NMSE is test-backend-ops' (:180-193) against the CPY bound 1e-6 (:2396-2398); the number of
//     differing dst bytes is reported too.
// usage: cpy_check PLUGIN [seeds]   (exit 0 = every case within the bound on every seed)
#include "ggml-alloc.h"
#include "ggml-backend.h"
#include "ggml-cpu.h"
#include "ggml.h"

#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

struct Case {
    ggml_type ts, td;
    std::array<int64_t, 4> ne, ps, pd;
};

static bool any(const std::array<int64_t, 4> &p) { return p[0] + p[1] + p[2] + p[3] > 0; }

struct Graph {
    ggml_context *ctx;
    ggml_tensor *src, *dst, *out;
    ggml_cgraph *gf;
    ggml_backend_buffer_t buf;
};

static Graph build(const Case &c, ggml_backend_t be) {
    ggml_init_params ip = {ggml_tensor_overhead() * 16 + ggml_graph_overhead(), nullptr, true};
    Graph g{};
    g.ctx = ggml_init(ip);
    g.src = ggml_new_tensor(g.ctx, c.ts, 4, c.ne.data());
    ggml_tensor *s = g.src;
    if (any(c.ps)) s = ggml_permute(g.ctx, s, (int)c.ps[0], (int)c.ps[1], (int)c.ps[2], (int)c.ps[3]);
    g.dst = ggml_new_tensor(g.ctx, c.td, 4, s->ne);
    ggml_tensor *d = g.dst;
    if (any(c.pd)) d = ggml_permute(g.ctx, d, (int)c.pd[0], (int)c.pd[1], (int)c.pd[2], (int)c.pd[3]);
    g.out = ggml_cpy(g.ctx, s, d);
    g.gf = ggml_new_graph(g.ctx);
    ggml_build_forward_expand(g.gf, g.out);
    g.buf = ggml_backend_alloc_ctx_tensors(g.ctx, be);
    if (!g.buf) { fprintf(stderr, "allocation failed\n"); exit(2); }
    return g;
}

static void release(Graph &g) {
    ggml_backend_buffer_free(g.buf);
    ggml_free(g.ctx);
}

// init_tensor_uniform's bytes for tensor type t (test-backend-ops.cpp:42-120)
static std::vector<uint8_t> fill(ggml_type t, int64_t n, int64_t ne0, std::mt19937 &rng) {
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    std::vector<float> x((size_t)n);
    for (auto &v : x) v = u(rng);
    std::vector<uint8_t> out;
    if (t == GGML_TYPE_F32) {
        out.resize(n * 4);
        memcpy(out.data(), x.data(), out.size());
    } else if (t == GGML_TYPE_F16) {
        out.resize(n * 2);
        ggml_fp32_to_fp16_row(x.data(), reinterpret_cast<ggml_fp16_t *>(out.data()), n);
    } else {
        std::vector<float> im((size_t)ne0, 1.0f);
        const float *imp = (!ggml_quantize_requires_imatrix(t) && x[0] > 0.f) ? nullptr : im.data();
        out.resize(ggml_row_size(t, n));
        ggml_quantize_chunk(t, x.data(), out.data(), 0, n / ne0, ne0, imp);
    }
    return out;
}

static std::vector<float> to_f32(ggml_type t, const std::vector<uint8_t> &b, int64_t n) {
    std::vector<float> f((size_t)n);
    if (t == GGML_TYPE_F32) memcpy(f.data(), b.data(), n * 4);
    else ggml_get_type_traits(t)->to_float(b.data(), f.data(), n);
    return f;
}

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: cpy_check PLUGIN [seeds]\n"); return 2; }
    const int seeds = argc > 2 ? atoi(argv[2]) : 100;
    ggml_backend_reg_t reg = ggml_backend_load(argv[1]);
    if (!reg || ggml_backend_reg_dev_count(reg) == 0) { fprintf(stderr, "plugin has no devices\n"); return 2; }
    ggml_backend_t gpu = ggml_backend_dev_init(ggml_backend_reg_dev_get(reg, 0), nullptr);
    ggml_backend_t cpu = ggml_backend_cpu_init();
    ggml_backend_cpu_set_n_threads(cpu, 8);

    const ggml_type types[] = {GGML_TYPE_F32, GGML_TYPE_F16, GGML_TYPE_Q4_0, GGML_TYPE_Q8_0,
                               GGML_TYPE_Q4_K, GGML_TYPE_Q5_K, GGML_TYPE_Q6_K};
    std::vector<Case> cases;
    for (ggml_type t : types) {   // same-type copies (:5575-5583)
        const int64_t nk = ggml_blck_size(t);
        for (int k = 1; k < 4; ++k) {
            cases.push_back({t, t, {k * nk, 2, 3, 4}, {0, 0, 0, 0}, {0, 0, 0, 0}});
            cases.push_back({t, t, {k * nk, 2, 3, 4}, {0, 2, 1, 3}, {0, 0, 0, 0}});
            cases.push_back({t, t, {k * nk, 2, 3, 4}, {0, 3, 1, 2}, {0, 2, 1, 3}});
        }
    }
    for (ggml_type ts : types)   // into / out of every type (:5585-5597)
        for (ggml_type td : types) {
            if (ts == td || (ts != GGML_TYPE_F32 && ts != GGML_TYPE_F16 && td != GGML_TYPE_F32)) continue;
            cases.push_back({ts, td, {256, 4, 4, 4}, {0, 0, 0, 0}, {0, 0, 0, 0}});
            cases.push_back({ts, td, {256, 2, 3, 4}, {0, 2, 1, 3}, {0, 0, 0, 0}});
        }
    for (ggml_type ts : {GGML_TYPE_F16, GGML_TYPE_F32})   // not contiguous (:5598-5602)
        for (ggml_type td : {GGML_TYPE_F16, GGML_TYPE_F32})
            cases.push_back({ts, td, {256, 2, 3, 4}, {1, 0, 2, 3}, {0, 0, 0, 0}});

    int n_run = 0, n_fail = 0;
    for (size_t ci = 0; ci < cases.size(); ++ci) {
        const Case &c = cases[ci];
        Graph gg = build(c, gpu), gc = build(c, cpu);
        if (!ggml_backend_supports_op(gpu, gg.out)) {
            release(gg);
            release(gc);
            continue;
        }
        ++n_run;
        const int64_t ns = ggml_nelements(gg.src), nd = ggml_nelements(gg.dst);
        double worst = 0;
        int worst_seed = -1;
        size_t worst_bytes = 0;
        for (int seed = 0; seed < seeds; ++seed) {
            std::mt19937 rng((uint32_t)(ci * 100003u + (uint32_t)seed));
            const std::vector<uint8_t> sb = fill(c.ts, ns, gg.src->ne[0], rng), db = fill(c.td, nd, gg.dst->ne[0], rng);
            for (Graph *g : {&gg, &gc}) {
                ggml_backend_tensor_set(g->src, sb.data(), 0, sb.size());
                ggml_backend_tensor_set(g->dst, db.data(), 0, db.size());
            }
            if (ggml_backend_graph_compute(gpu, gg.gf) != GGML_STATUS_SUCCESS ||
                ggml_backend_graph_compute(cpu, gc.gf) != GGML_STATUS_SUCCESS) {
                fprintf(stderr, "graph_compute failed\n");
                return 2;
            }
            std::vector<uint8_t> rg(ggml_nbytes(gg.dst)), rc(ggml_nbytes(gc.dst));
            ggml_backend_tensor_get(gg.dst, rg.data(), 0, rg.size());
            ggml_backend_tensor_get(gc.dst, rc.data(), 0, rc.size());
            size_t nbytes_diff = 0;
            for (size_t i = 0; i < rg.size(); ++i) nbytes_diff += rg[i] != rc[i];
            const std::vector<float> fg = to_f32(c.td, rg, nd), fc = to_f32(c.td, rc, nd);
            double num = 0, den = 0;
            bool finite = true;
            for (int64_t i = 0; i < nd; ++i) {
                finite = finite && std::isfinite(fg[i]);
                num += (fg[i] - (double)fc[i]) * (fg[i] - (double)fc[i]);
                den += (double)fc[i] * fc[i];
            }
            const double e = finite ? num / den : INFINITY;
            if (e > worst || worst_seed < 0) {
                worst = e;
                worst_seed = seed;
                worst_bytes = nbytes_diff;
            }
            if (!(e <= 1e-6)) {
                int shown = 0;
                printf("  FAIL seed %d nmse %.3e, %zu dst bytes differ; first elements:", seed, e, nbytes_diff);
                for (int64_t i = 0; i < nd && shown < 6; ++i)
                    if (fg[i] != fc[i]) {
                        printf(" [%lld] %.9g vs %.9g", (long long)i, fg[i], fc[i]);
                        ++shown;
                    }
                printf("\n");
            }
        }
        const bool ok = worst <= 1e-6;
        n_fail += !ok;
        printf("%s CPY %s -> %s ne=[%lld,%lld,%lld,%lld] permute_src=[%lld,%lld,%lld,%lld] permute_dst=[%lld,%lld,%lld,%lld]: "
               "%d seeds, worst nmse %.3e (seed %d, %zu dst bytes differ)\n",
               ok ? "OK  " : "FAIL", ggml_type_name(c.ts), ggml_type_name(c.td), (long long)c.ne[0], (long long)c.ne[1],
               (long long)c.ne[2], (long long)c.ne[3], (long long)c.ps[0], (long long)c.ps[1], (long long)c.ps[2],
               (long long)c.ps[3], (long long)c.pd[0], (long long)c.pd[1], (long long)c.pd[2], (long long)c.pd[3], seeds, worst,
               worst_seed, worst_bytes);
        release(gg);
        release(gc);
    }
    ggml_backend_free(gpu);
    ggml_backend_free(cpu);
    printf("%d cases run on the plugin, %d over the bound\n%s\n", n_run, n_fail, n_fail ? "CPY_CHECK_FAIL" : "CPY_CHECK_OK");
    return n_fail ? 1 : 0;
}
