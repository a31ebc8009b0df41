// oracle/repack_check.cpp — TEST INFRASTRUCTURE ONLY (never part of the product path).
//
// Drives our plugin's repacked-weight buffer type through the REFERENCE ggml backend API, the
// way a llama.cpp-style host uses extra buffer types: load the plugin with ggml_backend_load,
// fetch "ggml_backend_dev_get_extra_bufts" from its registry (reference ggml-backend.h:192;
// the CPU backend's own is ggml-cpu.cpp:619), allocate quantized weights in the first extra
// buffer type, and run GGML_OP_MUL_MAT on the plugin's backend against the same graph on
// ggml-cpu:
//   * the weight reads back byte-identical (the ggml bytes stay at tensor->data);
//   * supports_op claims the node;
//   * NMSE(plugin, ggml-cpu) <= 5e-4 (test-backend-ops' MUL_MAT bar, tests/test-backend-ops.cpp:3106),
//     at mat-vec sizes (ne11 <= 8, which read the ggml bytes) and mat-mat sizes (the repacked copy);
//   * after a second ggml_backend_tensor_set with other weights the result follows the new
//     weights (every write remakes the copy);
//   * the same after an asynchronous write (ggml_backend_tensor_set_async on the plugin's backend,
//     reference ggml-backend.cpp:234), after an upload in three chunks, and while an upload is
//     incomplete (the first chunk only: MUL_MAT must then read the ggml bytes, not the stale copy).
// usage: repack_check PLUGIN   (exit 0 = all cases pass)
#include "ggml-alloc.h"
#include "ggml-backend.h"
#include "ggml-cpu.h"
#include "ggml.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef ggml_backend_buffer_type_t *(*extra_bufts_fn)(ggml_backend_dev_t);

struct Weight {
    ggml_context *ctx;
    ggml_tensor *a;
    ggml_backend_buffer_t buf;
};

static Weight make_weight(ggml_backend_buffer_type_t bt, ggml_type t, int K, int N) {
    ggml_init_params pw = {ggml_tensor_overhead() * 4, nullptr, true};
    Weight w{};
    w.ctx = ggml_init(pw);
    w.a = ggml_new_tensor_2d(w.ctx, t, K, N);
    w.buf = ggml_backend_alloc_ctx_tensors_from_buft(w.ctx, bt);
    if (!w.buf) { fprintf(stderr, "weight allocation failed\n"); exit(2); }
    return w;
}

static std::vector<float> mul_mat(ggml_backend_t be, ggml_tensor *a, int M, const std::vector<float> &x, bool *supported) {
    const int K = (int)a->ne[0], N = (int)a->ne[1];
    ggml_init_params pc = {ggml_tensor_overhead() * 8 + ggml_graph_overhead(), nullptr, true};
    ggml_context *cc = ggml_init(pc);
    ggml_tensor *b = ggml_new_tensor_2d(cc, GGML_TYPE_F32, K, M);
    ggml_tensor *c = ggml_mul_mat(cc, a, b);
    ggml_cgraph *gf = ggml_new_graph(cc);
    ggml_build_forward_expand(gf, c);
    if (supported) *supported = ggml_backend_supports_op(be, c);
    ggml_gallocr_t ga = ggml_gallocr_new(ggml_backend_get_default_buffer_type(be));
    if (!ggml_gallocr_alloc_graph(ga, gf)) { fprintf(stderr, "graph allocation failed\n"); exit(2); }
    ggml_backend_tensor_set(b, x.data(), 0, x.size() * sizeof(float));
    if (ggml_backend_graph_compute(be, gf) != GGML_STATUS_SUCCESS) { fprintf(stderr, "graph_compute failed\n"); exit(2); }
    std::vector<float> out((size_t)N * M);
    ggml_backend_tensor_get(c, out.data(), 0, out.size() * sizeof(float));
    ggml_gallocr_free(ga);
    ggml_free(cc);
    return out;
}

static double nmse(const std::vector<float> &got, const std::vector<float> &want, bool *finite) {
    double num = 0, den = 0;
    *finite = true;
    for (size_t i = 0; i < got.size(); ++i) {
        *finite = *finite && std::isfinite(got[i]);
        num += (got[i] - want[i]) * (double)(got[i] - want[i]);
        den += want[i] * (double)want[i];
    }
    return num / (den > 0 ? den : 1);
}

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: repack_check PLUGIN\n"); return 2; }
    ggml_backend_reg_t reg = ggml_backend_load(argv[1]);
    if (!reg || ggml_backend_reg_dev_count(reg) == 0) { fprintf(stderr, "plugin has no devices\n"); return 2; }
    ggml_backend_dev_t dev = ggml_backend_reg_dev_get(reg, 0);
    auto extra = (extra_bufts_fn)ggml_backend_reg_get_proc_address(reg, "ggml_backend_dev_get_extra_bufts");
    if (!extra || !extra(dev) || !extra(dev)[0]) { fprintf(stderr, "no extra buffer types\n"); return 1; }
    ggml_backend_buffer_type_t rbt = extra(dev)[0];
    printf("extra buffer type: %s (supported by the device: %d)\n", ggml_backend_buft_name(rbt), ggml_backend_dev_supports_buft(dev, rbt));
    ggml_backend_t gpu = ggml_backend_dev_init(dev, nullptr);
    ggml_backend_t cpu = ggml_backend_cpu_init();
    ggml_backend_cpu_set_n_threads(cpu, 16);

    struct Case { ggml_type t; int K, N, M; } cases[] = {
        {GGML_TYPE_Q8_0, 4096, 4096, 512}, {GGML_TYPE_Q4_0, 2048, 1000, 64}, {GGML_TYPE_Q4_K, 1024, 333, 100},
        {GGML_TYPE_Q5_K, 512, 256, 16},    {GGML_TYPE_Q6_K, 1024, 777, 200}, {GGML_TYPE_Q8_0, 288, 100, 40},
        {GGML_TYPE_Q4_0, 4096, 512, 1},    {GGML_TYPE_Q6_K, 2048, 96, 5},
    };
    int fails = 0;
    std::mt19937 rng(4321);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    for (const Case &cs : cases) {
        std::vector<float> x((size_t)cs.K * cs.M);
        for (auto &v : x) v = u(rng);
        Weight wg = make_weight(rbt, cs.t, cs.K, cs.N), wc = make_weight(ggml_backend_cpu_buffer_type(), cs.t, cs.K, cs.N);
        bool ok_all = true;
        for (int pass = 0; pass < 5; ++pass) {   // 1: rewrite, 2: async, 3: in chunks, 4: first chunk only
            std::vector<float> w((size_t)cs.N * cs.K);
            for (auto &v : w) v = u(rng);
            std::vector<uint8_t> q(ggml_row_size(cs.t, cs.K) * cs.N);
            ggml_quantize_chunk(cs.t, w.data(), q.data(), 0, cs.N, cs.K, nullptr);
            const size_t rb = ggml_row_size(cs.t, cs.K), c1 = rb * (cs.N / 3), c2 = rb * (2 * cs.N / 3);
            if (pass == 2) {
                ggml_backend_tensor_set_async(gpu, wg.a, q.data(), 0, q.size());
                ggml_backend_synchronize(gpu);
            } else if (pass == 3) {
                ggml_backend_tensor_set(wg.a, q.data(), 0, c1);
                ggml_backend_tensor_set(wg.a, q.data() + c1, c1, c2 - c1);
                ggml_backend_tensor_set(wg.a, q.data() + c2, c2, q.size() - c2);
            } else if (pass == 4) {   // only the first rows change: the rest keep pass 3's bytes
                std::vector<uint8_t> prev(q.size());
                ggml_backend_tensor_get(wg.a, prev.data(), 0, prev.size());
                ggml_backend_tensor_set(wg.a, q.data(), 0, c1);
                memcpy(q.data() + c1, prev.data() + c1, q.size() - c1);
            } else {
                ggml_backend_tensor_set(wg.a, q.data(), 0, q.size());
            }
            ggml_backend_tensor_set(wc.a, q.data(), 0, q.size());
            std::vector<uint8_t> back(q.size());
            ggml_backend_tensor_get(wg.a, back.data(), 0, back.size());
            const bool rt = memcmp(back.data(), q.data(), q.size()) == 0;
            bool sup = false, finite = false;
            const std::vector<float> got = mul_mat(gpu, wg.a, cs.M, x, &sup);
            const std::vector<float> want = mul_mat(cpu, wc.a, cs.M, x, nullptr);
            const double e = nmse(got, want, &finite);
            const bool ok = rt && sup && finite && e <= 5e-4 && wg.a->extra != nullptr;
            ok_all = ok_all && ok;
            printf("%s %-5s K=%d N=%d M=%d pass=%d repacked=%d roundtrip=%d supports_op=%d nmse=%.3e\n", ok ? "OK  " : "FAIL",
                   ggml_type_name(cs.t), cs.K, cs.N, cs.M, pass, wg.a->extra != nullptr, rt, sup, e);
        }
        fails += !ok_all;
        ggml_backend_buffer_free(wg.buf);
        ggml_free(wg.ctx);
        ggml_backend_buffer_free(wc.buf);
        ggml_free(wc.ctx);
    }
    ggml_backend_free(gpu);
    ggml_backend_free(cpu);
    printf("%s\n", fails ? "REPACK_CHECK_FAIL" : "REPACK_CHECK_OK");
    return fails ? 1 : 0;
}
