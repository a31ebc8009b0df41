// oracle/split_check.cpp — TEST INFRASTRUCTURE ONLY (never part of the product path).
//
// Drives our plugin's row-split buffer type through the REFERENCE ggml backend API (the way a
// llama.cpp-style host does for tensor parallelism): load the plugin with ggml_backend_load,
// fetch "ggml_backend_split_buffer_type" from its registry (reference ggml-backend.h:187-200,
// ggml-cuda.cu:3733), allocate a quantized weight in it, run GGML_OP_MUL_MAT on the plugin's
// backend and compare with the same graph on ggml-cpu:
//   * the split weight reads back byte-identical (set_tensor / get_tensor over the shards);
//   * supports_op claims the node (so a scheduler would place it on the GPU);
//   * NMSE(plugin, ggml-cpu) <= 5e-4 (test-backend-ops' MUL_MAT bar, tests/test-backend-ops.cpp:3106).
// On a one-GPU box GGML_MI355X_SPLIT_SHARDS=k splits the weight into k shards on that GPU.
//
// usage: split_check PLUGIN [tensor_split fractions, e.g. 1,3]   (exit 0 = all cases pass)
#include "ggml-alloc.h"
#include "ggml-backend.h"
#include "ggml-cpu.h"
#include "ggml.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

typedef ggml_backend_buffer_type_t (*split_buft_fn)(int main_device, const float *tensor_split);

static std::vector<float> run(ggml_backend_t be, ggml_backend_buffer_type_t wbuft, ggml_type t, int K, int N, int M,
                              const std::vector<uint8_t> &q, const std::vector<float> &x, bool *roundtrip, bool *supported) {
    ggml_init_params pw = {ggml_tensor_overhead() * 4, nullptr, true};
    ggml_context *cw = ggml_init(pw);
    ggml_tensor *a = ggml_new_tensor_2d(cw, t, K, N);
    ggml_backend_buffer_t wb = ggml_backend_alloc_ctx_tensors_from_buft(cw, wbuft);
    if (!wb) { fprintf(stderr, "weight allocation failed\n"); exit(2); }
    ggml_backend_tensor_set(a, q.data(), 0, q.size());
    if (roundtrip) {
        std::vector<uint8_t> back(q.size());
        ggml_backend_tensor_get(a, back.data(), 0, back.size());
        *roundtrip = memcmp(back.data(), q.data(), q.size()) == 0;
    }
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
    ggml_backend_buffer_free(wb);
    ggml_free(cw);
    return out;
}

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: split_check PLUGIN [fractions]\n"); return 2; }
    std::vector<float> fr(16, 0.f);
    if (argc > 2) {
        int i = 0;
        for (char *tok = strtok(argv[2], ","); tok && i < 16; tok = strtok(nullptr, ",")) fr[i++] = (float)atof(tok);
    }
    ggml_backend_reg_t reg = ggml_backend_load(argv[1]);
    if (!reg || ggml_backend_reg_dev_count(reg) == 0) { fprintf(stderr, "plugin has no devices\n"); return 2; }
    auto split = (split_buft_fn)ggml_backend_reg_get_proc_address(reg, "ggml_backend_split_buffer_type");
    if (!split) { fprintf(stderr, "no ggml_backend_split_buffer_type\n"); return 1; }
    ggml_backend_t gpu = ggml_backend_dev_init(ggml_backend_reg_dev_get(reg, 0), nullptr);
    ggml_backend_t cpu = ggml_backend_cpu_init();
    ggml_backend_buffer_type_t sbt = split(0, fr.data());
    printf("split buffer type: %s\n", ggml_backend_buft_name(sbt));

    struct Case { ggml_type t; int K, N, M; } cases[] = {
        {GGML_TYPE_Q4_0, 4096, 1000, 1}, {GGML_TYPE_Q4_K, 2048, 4096, 3}, {GGML_TYPE_Q5_K, 1024, 333, 8},
        {GGML_TYPE_Q6_K, 1024, 777, 16}, {GGML_TYPE_Q8_0, 4096, 4096, 64}, {GGML_TYPE_Q4_0, 768, 50, 2},
    };
    int fails = 0;
    std::mt19937 rng(1234);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    for (const Case &cs : cases) {
        std::vector<float> w((size_t)cs.N * cs.K), x((size_t)cs.K * cs.M);
        for (auto &v : w) v = u(rng);
        for (auto &v : x) v = u(rng);
        std::vector<uint8_t> q(ggml_row_size(cs.t, cs.K) * cs.N);
        ggml_quantize_chunk(cs.t, w.data(), q.data(), 0, cs.N, cs.K, nullptr);
        bool rt = false, sup = false;
        const std::vector<float> got = run(gpu, sbt, cs.t, cs.K, cs.N, cs.M, q, x, &rt, &sup);
        const std::vector<float> want = run(cpu, ggml_backend_cpu_buffer_type(), cs.t, cs.K, cs.N, cs.M, q, x, nullptr, nullptr);
        double num = 0, den = 0;
        bool finite = true;
        for (size_t i = 0; i < got.size(); ++i) {
            finite = finite && std::isfinite(got[i]);
            num += (got[i] - want[i]) * (double)(got[i] - want[i]);
            den += want[i] * (double)want[i];
        }
        const double nmse = num / (den > 0 ? den : 1);
        const bool ok = rt && sup && finite && nmse <= 5e-4;
        fails += !ok;
        printf("%s %-5s K=%d N=%d M=%d roundtrip=%d supports_op=%d nmse=%.3e\n", ok ? "OK  " : "FAIL", ggml_type_name(cs.t), cs.K, cs.N,
               cs.M, rt, sup, nmse);
    }
    // an F32 matrix is refused at allocation (init_tensor fails, ggml-alloc returns NULL), not
    // accepted into shards that no backend could run
    {
        ggml_init_params pw = {ggml_tensor_overhead() * 2, nullptr, true};
        ggml_context *cw = ggml_init(pw);
        ggml_new_tensor_2d(cw, GGML_TYPE_F32, 256, 64);
        ggml_backend_buffer_t wb = ggml_backend_alloc_ctx_tensors_from_buft(cw, sbt);
        const bool refused = wb == nullptr;
        if (wb) ggml_backend_buffer_free(wb);
        ggml_free(cw);
        fails += !refused;
        printf("%s f32 weight in the split buffer refused=%d\n", refused ? "OK  " : "FAIL", refused);
    }
    ggml_backend_free(gpu);
    ggml_backend_free(cpu);
    printf("%s\n", fails ? "SPLIT_CHECK_FAIL" : "SPLIT_CHECK_OK");
    return fails ? 1 : 0;
}
