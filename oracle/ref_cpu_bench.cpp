// oracle/ref_cpu_bench.cpp — times the REFERENCE ggml-cpu MUL_MAT (test infrastructure; the
// `cpu_baseline` leg of bench.py). Linked against oracle/_ref/libggml-ref.so built from the
// reference sources by oracle/ref.mk. Never part of the product.
//
//   ref_cpu_bench <type> <K> <N> <M> <threads> <seconds> [copies]
//
// `copies` distinct weight matrices are cycled so the working set exceeds the LLC (HBM/DRAM-
// cold timing); prints one JSON line with the mean time per MUL_MAT.
#include "ggml.h"
#include "ggml-alloc.h"
#include "ggml-backend.h"
#include "ggml-cpu.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static void fill_uniform(float *dst, int64_t n, uint64_t seed) {
    for (int64_t i = 0; i < n; ++i) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        dst[i] = -1.0f + 2.0f * ((float)(z >> 40) * 0x1.0p-24f);
    }
}

int main(int argc, char **argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: %s <type> <K> <N> <M> <threads> <seconds> [copies]\n", argv[0]);
        return 2;
    }
    ggml_type t = GGML_TYPE_COUNT;
    for (int i = 0; i < GGML_TYPE_COUNT; ++i)
        if (ggml_type_name((ggml_type)i) && strcmp(ggml_type_name((ggml_type)i), argv[1]) == 0) t = (ggml_type)i;
    if (t == GGML_TYPE_COUNT) { fprintf(stderr, "unknown type %s\n", argv[1]); return 2; }
    const int64_t K = atoll(argv[2]), N = atoll(argv[3]), M = atoll(argv[4]);
    const int threads = atoi(argv[5]);
    const double seconds = atof(argv[6]);
    const int copies = argc > 7 ? atoi(argv[7]) : 1;

    ggml_cpu_init();
    ggml_backend_t be = ggml_backend_cpu_init();
    ggml_backend_cpu_set_n_threads(be, threads);

    ggml_init_params ip = {(size_t)(4 * copies + 8) * ggml_tensor_overhead() + (size_t)copies * ggml_graph_overhead(), nullptr, true};
    ggml_context *ctx = ggml_init(ip);
    std::vector<ggml_tensor *> W(copies), Y(copies);
    ggml_tensor *X = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, K, M);
    std::vector<ggml_cgraph *> G(copies);
    for (int c = 0; c < copies; ++c) {
        W[c] = ggml_new_tensor_2d(ctx, t, K, N);
        Y[c] = ggml_mul_mat(ctx, W[c], X);
        G[c] = ggml_new_graph(ctx);
        ggml_build_forward_expand(G[c], Y[c]);
    }
    ggml_backend_buffer_t buf = ggml_backend_alloc_ctx_tensors(ctx, be);
    {
        std::vector<float> f(K * N);
        std::vector<uint8_t> q(ggml_row_size(t, K) * N);
        fill_uniform(f.data(), (int64_t)f.size(), 1234);
        ggml_quantize_chunk(t, f.data(), q.data(), 0, N, K, nullptr);
        for (int c = 0; c < copies; ++c) ggml_backend_tensor_set(W[c], q.data(), 0, q.size());
        std::vector<float> x(K * M);
        fill_uniform(x.data(), (int64_t)x.size(), 5678);
        ggml_backend_tensor_set(X, x.data(), 0, x.size() * 4);
    }
    for (int c = 0; c < copies; ++c) ggml_backend_graph_compute(be, G[c]);   // warm-up
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    int64_t runs = 0;
    double el = 0;
    do {
        ggml_backend_graph_compute(be, G[runs % copies]);
        ++runs;
        el = std::chrono::duration<double>(clk::now() - t0).count();
    } while (el < seconds);
    const double per = el / runs;
    const double bytes = (double)ggml_row_size(t, K) * N + 4.0 * K * M + 4.0 * N * M;
    printf("{\"type\": \"%s\", \"K\": %lld, \"N\": %lld, \"M\": %lld, \"threads\": %d, \"copies\": %d, \"runs\": %lld, "
           "\"sec_per_mul_mat\": %.9g, \"GBps\": %.6g, \"GOPs\": %.6g}\n",
           argv[1], (long long)K, (long long)N, (long long)M, threads, copies, (long long)runs, per,
           bytes / per * 1e-9, 2.0 * K * N * M / per * 1e-9);
    ggml_backend_buffer_free(buf);
    ggml_free(ctx);
    ggml_backend_free(be);
    return 0;
}
