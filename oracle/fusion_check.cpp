// oracle/fusion_check.cpp — TEST INFRASTRUCTURE ONLY (never part of the product path).
//
// Drives the plugin's graph fusion (backend.cpp fuse_matvec / fuse_softmax) through the
// REFERENCE ggml API: every case builds one ggml graph with the chains GPT-2 emits
// (examples/gpt-2/main-sched.cpp:603-637, 690-706, 744-757, 765-822, 826-847), allocates it
// with ggml-alloc (so in-place reuse and aliasing happen as in a real run), computes it on the
// plugin's backend and on ggml-cpu, and compares every tensor the case reads back:
//   * the run's result, NMSE <= 5e-4 (test-backend-ops' MUL_MAT bar, tests/test-backend-ops.cpp:3106);
//   * in the negative cases, the intermediates that must NOT be skipped (an OUTPUT flag, a second
//     consumer) read back equal to ggml-cpu too.
// tests/test_graph_fusion.py runs it with fusion on (GGML_MI355X_DEBUG lists the fused runs) and
// with GGML_MI355X_FUSION=0, and asserts which cases fused.
//
// usage: fusion_check PLUGIN   (exit 0 = every case within the bar)
#include "ggml-alloc.h"
#include "ggml-backend.h"
#include "ggml-cpu.h"
#include "ggml.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <random>
#include <string>
#include <vector>

namespace {

struct Inputs {
    std::map<std::string, std::vector<uint8_t>> bytes;   // by tensor name
};

// builds the case's graph in ctx; returns the tensors to read back (first = the result)
using Builder = std::function<std::vector<ggml_tensor *>(ggml_context *, ggml_cgraph *)>;

std::vector<std::vector<float>> run(ggml_backend_t be, const Builder &build, const Inputs &in) {
    ggml_init_params p = {ggml_tensor_overhead() * 256 + ggml_graph_overhead(), nullptr, true};
    ggml_context *ctx = ggml_init(p);
    ggml_cgraph *gf = ggml_new_graph(ctx);
    std::vector<ggml_tensor *> outs = build(ctx, gf);
    for (ggml_tensor *t : outs) ggml_build_forward_expand(gf, t);
    ggml_gallocr_t ga = ggml_gallocr_new(ggml_backend_get_default_buffer_type(be));
    if (!ggml_gallocr_alloc_graph(ga, gf)) { fprintf(stderr, "graph allocation failed\n"); exit(2); }
    for (const auto &kv : in.bytes) {
        ggml_tensor *t = ggml_get_tensor(ctx, kv.first.c_str());
        if (!t) continue;   // an input this case does not use
        if (ggml_nbytes(t) != kv.second.size()) { fprintf(stderr, "size mismatch %s\n", kv.first.c_str()); exit(2); }
        ggml_backend_tensor_set(t, kv.second.data(), 0, kv.second.size());
    }
    if (ggml_backend_graph_compute(be, gf) != GGML_STATUS_SUCCESS) { fprintf(stderr, "graph_compute failed\n"); exit(2); }
    std::vector<std::vector<float>> res;
    for (ggml_tensor *t : outs) {
        std::vector<float> v(ggml_nelements(t));
        ggml_backend_tensor_get(t, v.data(), 0, v.size() * sizeof(float));
        res.push_back(std::move(v));
    }
    ggml_gallocr_free(ga);
    ggml_free(ctx);
    return res;
}

// the same allocated graph computed once per step; a step sets only the tensors it names (a
// later step that names nothing but x leaves the plugin's captured hipGraph valid: a replay)
std::vector<std::vector<std::vector<float>>> run_steps(ggml_backend_t be, const Builder &build, const std::vector<Inputs> &steps) {
    ggml_init_params p = {ggml_tensor_overhead() * 256 + ggml_graph_overhead(), nullptr, true};
    ggml_context *ctx = ggml_init(p);
    ggml_cgraph *gf = ggml_new_graph(ctx);
    std::vector<ggml_tensor *> outs = build(ctx, gf);
    for (ggml_tensor *t : outs) ggml_build_forward_expand(gf, t);
    ggml_gallocr_t ga = ggml_gallocr_new(ggml_backend_get_default_buffer_type(be));
    if (!ggml_gallocr_alloc_graph(ga, gf)) { fprintf(stderr, "graph allocation failed\n"); exit(2); }
    std::vector<std::vector<std::vector<float>>> res;
    for (const Inputs &in : steps) {
        for (const auto &kv : in.bytes) {
            ggml_tensor *t = ggml_get_tensor(ctx, kv.first.c_str());
            if (!t) continue;
            if (ggml_nbytes(t) != kv.second.size()) { fprintf(stderr, "size mismatch %s\n", kv.first.c_str()); exit(2); }
            ggml_backend_tensor_set(t, kv.second.data(), 0, kv.second.size());
        }
        if (ggml_backend_graph_compute(be, gf) != GGML_STATUS_SUCCESS) { fprintf(stderr, "graph_compute failed\n"); exit(2); }
        std::vector<std::vector<float>> r;
        for (ggml_tensor *t : outs) {
            std::vector<float> v(ggml_nelements(t));
            ggml_backend_tensor_get(t, v.data(), 0, v.size() * sizeof(float));
            r.push_back(std::move(v));
        }
        res.push_back(std::move(r));
    }
    ggml_gallocr_free(ga);
    ggml_free(ctx);
    return res;
}

ggml_tensor *input(ggml_context *ctx, const char *name, ggml_type t, int64_t n0, int64_t n1 = 1, int64_t n2 = 1) {
    ggml_tensor *x = ggml_new_tensor_3d(ctx, t, n0, n1, n2);
    ggml_set_name(x, name);
    ggml_set_input(x);
    return x;
}

// the layer input stays allocated after the norm read it, as GPT-2's residual stream does (its
// residual add reads it later). Without that, ggml-alloc may place the chain's result over the
// freed input, and the plugin then declines the fusion (every workgroup of the fused launch reads
// the whole input while others already store results) — the "freed_input" case covers that.
ggml_tensor *resident(ggml_tensor *x) {
    ggml_set_output(x);
    return x;
}

std::mt19937 rng(4321);

std::vector<uint8_t> f32_bytes(size_t n, float lo, float hi) {
    std::uniform_real_distribution<float> u(lo, hi);
    std::vector<uint8_t> b(n * 4);
    for (size_t i = 0; i < n; ++i) {
        const float v = u(rng);
        memcpy(&b[i * 4], &v, 4);
    }
    return b;
}

std::vector<uint8_t> f16_bytes(size_t n) {
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    std::vector<uint8_t> b(n * 2);
    for (size_t i = 0; i < n; ++i) {
        const ggml_fp16_t h = ggml_fp32_to_fp16(u(rng));
        memcpy(&b[i * 2], &h, 2);
    }
    return b;
}

std::vector<uint8_t> q_bytes(ggml_type t, int64_t K, int64_t N) {
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    std::vector<float> w((size_t)K * N);
    for (auto &v : w) v = u(rng);
    std::vector<uint8_t> q(ggml_row_size(t, K) * N);
    ggml_quantize_chunk(t, w.data(), q.data(), 0, N, K, nullptr);
    return q;
}

double nmse(const std::vector<float> &got, const std::vector<float> &want, bool *finite) {
    double num = 0, den = 0;
    for (size_t i = 0; i < got.size(); ++i) {
        if (!std::isfinite(got[i]) && !(std::isinf(got[i]) && got[i] == want[i])) *finite = false;
        if (std::isfinite(want[i])) {
            num += (got[i] - want[i]) * (double)(got[i] - want[i]);
            den += want[i] * (double)want[i];
        }
    }
    return num / (den > 0 ? den : 1);
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: fusion_check PLUGIN\n"); return 2; }
    ggml_backend_reg_t reg = ggml_backend_load(argv[1]);
    if (!reg || ggml_backend_reg_dev_count(reg) == 0) { fprintf(stderr, "plugin has no devices\n"); return 2; }
    ggml_backend_t gpu = ggml_backend_dev_init(ggml_backend_reg_dev_get(reg, 0), nullptr);
    ggml_backend_t cpu = ggml_backend_cpu_init();
    const float eps = 1e-5f;
    int fails = 0;

    auto check = [&](const std::string &name, const Builder &b, const Inputs &in, bool exact = false) {
        fprintf(stderr, "CASE %s\n", name.c_str());   // the plugin's debug log follows on stderr
        const auto got = run(gpu, b, in);
        const auto want = run(cpu, b, in);
        bool ok = true;
        std::string detail;
        for (size_t j = 0; j < got.size(); ++j) {
            bool finite = true;
            const double e = nmse(got[j], want[j], &finite);
            ok = ok && finite && e <= 5e-4;
            if (exact) ok = ok && got[j].size() == want[j].size() && memcmp(got[j].data(), want[j].data(), 4 * got[j].size()) == 0;
            char buf[64];
            snprintf(buf, sizeof buf, " out%zu=%.3e%s", j, e, finite ? "" : "(nonfinite)");
            detail += buf;
        }
        fails += !ok;
        printf("%s %s%s\n", ok ? "OK  " : "FAIL", name.c_str(), detail.c_str());
        fflush(stdout);
    };

    const ggml_type types[] = {GGML_TYPE_Q4_0, GGML_TYPE_Q8_0, GGML_TYPE_Q4_K, GGML_TYPE_Q5_K, GGML_TYPE_Q6_K};
    for (ggml_type t : types) {
        for (int M : {1, 3, 8}) {
            const int E = 768, F = 4 * E;
            Inputs in;
            in.bytes["x"] = f32_bytes((size_t)E * M, -2.f, 2.f);
            in.bytes["g"] = f32_bytes(E, 0.5f, 1.5f);
            in.bytes["b"] = f32_bytes(E, -0.2f, 0.2f);
            in.bytes["w_qkv"] = q_bytes(t, E, 3 * E);
            in.bytes["b_qkv"] = f32_bytes(3 * E, -0.5f, 0.5f);
            in.bytes["w_fc"] = q_bytes(t, E, F);
            in.bytes["b_fc"] = f32_bytes(F, -0.5f, 0.5f);
            in.bytes["w_mp"] = q_bytes(t, F, E);
            in.bytes["b_mp"] = f32_bytes(E, -0.5f, 0.5f);
            in.bytes["memk"] = f32_bytes((size_t)2 * 32 * E, -1.f, 1.f);
            in.bytes["memv"] = f32_bytes((size_t)2 * 32 * E, -1.f, 1.f);
            const std::string tag = std::string(ggml_type_name(t)) + " M=" + std::to_string(M);

            // layer-norm -> c_attn + bias (main-sched.cpp:603-637)
            check("ln_matvec_bias " + tag, [&](ggml_context *c, ggml_cgraph *) {
                ggml_tensor *x = resident(input(c, "x", GGML_TYPE_F32, E, M));
                ggml_tensor *h = ggml_add(c, ggml_mul(c, ggml_norm(c, x, eps), input(c, "g", GGML_TYPE_F32, E)), input(c, "b", GGML_TYPE_F32, E));
                ggml_tensor *y = ggml_add(c, ggml_mul_mat(c, input(c, "w_qkv", t, E, 3 * E), h), input(c, "b_qkv", GGML_TYPE_F32, 3 * E));
                return std::vector<ggml_tensor *>{y};
            }, in);

            // layer-norm -> fc + bias -> gelu -> proj + bias -> + residual (main-sched.cpp:765-822)
            check("mlp " + tag, [&](ggml_context *c, ggml_cgraph *) {
                ggml_tensor *x = resident(input(c, "x", GGML_TYPE_F32, E, M));
                ggml_tensor *h = ggml_add(c, ggml_mul(c, ggml_norm(c, x, eps), input(c, "g", GGML_TYPE_F32, E)), input(c, "b", GGML_TYPE_F32, E));
                h = ggml_gelu(c, ggml_add(c, ggml_mul_mat(c, input(c, "w_fc", t, E, F), h), input(c, "b_fc", GGML_TYPE_F32, F)));
                ggml_tensor *y = ggml_add(c, ggml_add(c, ggml_mul_mat(c, input(c, "w_mp", t, F, E), h), input(c, "b_mp", GGML_TYPE_F32, E)), x);
                return std::vector<ggml_tensor *>{y};
            }, in);

            // c_attn + bias, then the K / V cache writes of the new token(s) (main-sched.cpp:620-655,
            // layer 1 of 2 at n_past = 5): the plugin folds both copies into the mat-vec's epilogue
            check("qkv_cache " + tag, [&](ggml_context *c, ggml_cgraph *gf) {
                const int n_ctx = 32, il = 1, n_past = 5;
                ggml_tensor *x = resident(input(c, "x", GGML_TYPE_F32, E, M));
                ggml_tensor *memk = resident(input(c, "memk", GGML_TYPE_F32, 2 * n_ctx * E));
                ggml_tensor *memv = resident(input(c, "memv", GGML_TYPE_F32, 2 * n_ctx * E));
                // an unfused node first, so the fused run does not start at node 0
                ggml_tensor *xs = resident(ggml_scale(c, x, 0.5f));
                ggml_tensor *cur = ggml_add(c, ggml_mul_mat(c, input(c, "w_qkv", t, E, 3 * E), xs), input(c, "b_qkv", GGML_TYPE_F32, 3 * E));
                ggml_tensor *Kcur = ggml_view_2d(c, cur, E, M, cur->nb[1], 1 * sizeof(float) * E);
                ggml_tensor *Vcur = ggml_view_2d(c, cur, E, M, cur->nb[1], 2 * sizeof(float) * E);
                ggml_tensor *k = ggml_view_1d(c, memk, M * E, (ggml_element_size(memk) * E) * (il * n_ctx + n_past));
                ggml_tensor *v = ggml_view_1d(c, memv, M * E, (ggml_element_size(memv) * E) * (il * n_ctx + n_past));
                ggml_build_forward_expand(gf, ggml_cpy(c, Kcur, k));
                ggml_build_forward_expand(gf, ggml_cpy(c, Vcur, v));
                return std::vector<ggml_tensor *>{cur, memk, memv};
            }, in);

            // token + position embedding (main-sched.cpp:589-595): GET_ROWS(wte) + GET_ROWS(wpe)
            if (M > 1) {
                const int V = 64, n_ctx = 32;
                in.bytes["wte"] = q_bytes(t, E, V);
                in.bytes["wpe"] = f32_bytes((size_t)E * n_ctx, -1.f, 1.f);
                std::vector<uint8_t> tok(4 * M), pos(4 * M);
                for (int j = 0; j < M; ++j) {
                    const int32_t tv = (int32_t)(rng() % V), pv = 3 + j;
                    memcpy(&tok[4 * j], &tv, 4);
                    memcpy(&pos[4 * j], &pv, 4);
                }
                in.bytes["tok"] = tok;
                in.bytes["pos"] = pos;
                check("embed " + tag, [&](ggml_context *c, ggml_cgraph *) {
                    ggml_tensor *wte = input(c, "wte", t, E, V), *wpe = input(c, "wpe", GGML_TYPE_F32, E, n_ctx);
                    ggml_tensor *y = ggml_add(c, ggml_get_rows(c, wte, input(c, "tok", GGML_TYPE_I32, M)),
                                              ggml_get_rows(c, wpe, input(c, "pos", GGML_TYPE_I32, M)));
                    return std::vector<ggml_tensor *>{y};
                }, in, true);
            }

            // final layer-norm -> lm_head without bias (main-sched.cpp:826-847)
            check("ln_matvec " + tag, [&](ggml_context *c, ggml_cgraph *) {
                ggml_tensor *x = resident(input(c, "x", GGML_TYPE_F32, E, M));
                ggml_tensor *h = ggml_add(c, ggml_mul(c, ggml_norm(c, x, eps), input(c, "g", GGML_TYPE_F32, E)), input(c, "b", GGML_TYPE_F32, E));
                return std::vector<ggml_tensor *>{ggml_mul_mat(c, input(c, "w_fc", t, E, F), h)};
            }, in);
        }
    }

    // negative cases (Q4_0, M = 2): the skipped intermediates are needed elsewhere
    {
        const int E = 768, M = 2;
        Inputs in;
        in.bytes["x"] = f32_bytes((size_t)E * M, -2.f, 2.f);
        in.bytes["g"] = f32_bytes(E, 0.5f, 1.5f);
        in.bytes["b"] = f32_bytes(E, -0.2f, 0.2f);
        in.bytes["w"] = q_bytes(GGML_TYPE_Q4_0, E, E);
        in.bytes["bias"] = f32_bytes(E, -0.5f, 0.5f);
        // the norm is a requested output: the chain must not fuse, and the norm reads back
        check("neg_output_flag", [&](ggml_context *c, ggml_cgraph *) {
            ggml_tensor *x = input(c, "x", GGML_TYPE_F32, E, M);
            ggml_tensor *nrm = ggml_norm(c, x, eps);
            ggml_set_output(nrm);
            ggml_tensor *h = ggml_add(c, ggml_mul(c, nrm, input(c, "g", GGML_TYPE_F32, E)), input(c, "b", GGML_TYPE_F32, E));
            ggml_tensor *y = ggml_add(c, ggml_mul_mat(c, input(c, "w", GGML_TYPE_Q4_0, E, E), h), input(c, "bias", GGML_TYPE_F32, E));
            return std::vector<ggml_tensor *>{y, nrm};
        }, in);
        // the mat-vec result has a second consumer: the bias add may not swallow it
        check("neg_second_use", [&](ggml_context *c, ggml_cgraph *) {
            ggml_tensor *x = input(c, "x", GGML_TYPE_F32, E, M);
            ggml_tensor *mm = ggml_mul_mat(c, input(c, "w", GGML_TYPE_Q4_0, E, E), x);
            ggml_tensor *y = ggml_add(c, mm, input(c, "bias", GGML_TYPE_F32, E));
            ggml_tensor *z = ggml_scale(c, mm, 0.5f);
            return std::vector<ggml_tensor *>{y, z};
        }, in);
        // the chain's input is freed after the norm: correct whether or not the plugin fuses
        check("freed_input", [&](ggml_context *c, ggml_cgraph *) {
            ggml_tensor *x = input(c, "x", GGML_TYPE_F32, E, M);
            ggml_tensor *h = ggml_add(c, ggml_mul(c, ggml_norm(c, x, eps), input(c, "g", GGML_TYPE_F32, E)), input(c, "b", GGML_TYPE_F32, E));
            ggml_tensor *y = ggml_add(c, ggml_mul_mat(c, input(c, "w", GGML_TYPE_Q4_0, E, E), h), input(c, "bias", GGML_TYPE_F32, E));
            return std::vector<ggml_tensor *>{y};
        }, in);
        // mat-vec + bias + residual with the residual as the FIRST operand of the add
        check("resid_first_operand", [&](ggml_context *c, ggml_cgraph *) {
            ggml_tensor *x = input(c, "x", GGML_TYPE_F32, E, M);
            ggml_tensor *mm = ggml_add(c, ggml_mul_mat(c, input(c, "w", GGML_TYPE_Q4_0, E, E), x), input(c, "bias", GGML_TYPE_F32, E));
            return std::vector<ggml_tensor *>{ggml_add(c, x, mm)};
        }, in);
    }

    // attention weights: KQ -> scale -> causal mask -> soft_max (main-sched.cpp:690-706)
    for (int n_past : {0, 5, 63}) {
        for (int N : {1, 4}) {
            const int H = 12, n_kv = n_past + N;
            Inputs in;
            in.bytes["kq"] = f32_bytes((size_t)n_kv * N * H, -8.f, 8.f);
            const std::string tag = "n_past=" + std::to_string(n_past) + " N=" + std::to_string(N);
            check("softmax_chain " + tag, [&](ggml_context *c, ggml_cgraph *) {
                ggml_tensor *kq = input(c, "kq", GGML_TYPE_F32, n_kv, N, H);
                ggml_tensor *kq2 = ggml_scale(c, ggml_add(c, kq, kq), 0.125f);   // a producer node, as KQ is
                return std::vector<ggml_tensor *>{ggml_soft_max(c, ggml_diag_mask_inf(c, kq2, n_past))};
            }, in);
            check("softmax_mask_only " + tag, [&](ggml_context *c, ggml_cgraph *) {
                ggml_tensor *kq = input(c, "kq", GGML_TYPE_F32, n_kv, N, H);
                return std::vector<ggml_tensor *>{ggml_soft_max(c, ggml_diag_mask_inf(c, ggml_add(c, kq, kq), n_past))};
            }, in);
        }
    }

    // GPT-2's attention block as main-sched.cpp:641-732 builds it (layer 1 of 2, so every cache
    // view has an offset): the K / V cache writes, then Q . K^T -> scale -> causal mask ->
    // soft_max -> V^T . -> merged heads. The plugin runs the whole read side as one launch.
    for (int n_past : {0, 7, 100}) {
        for (int N : {1, 4}) {
            for (int variant : {0, 1, 2}) {   // 1: soft_max is an output, 2: f16 caches
                const int sm_out = variant == 1;
                const ggml_type ct = variant == 2 ? GGML_TYPE_F16 : GGML_TYPE_F32;
                if (variant != 0 && n_past != 7) continue;
                const int E = 768, H = 12, Dh = E / H, n_ctx = 128, n_layer = 2, il = 1;
                const float kq_scale = 1.0f / sqrtf((float)Dh);
                Inputs in;
                in.bytes["cur"] = f32_bytes((size_t)3 * E * N, -1.f, 1.f);
                const size_t n_cache = (size_t)n_layer * n_ctx * E;
                in.bytes["memk"] = ct == GGML_TYPE_F16 ? f16_bytes(n_cache) : f32_bytes(n_cache, -1.f, 1.f);
                in.bytes["memv"] = ct == GGML_TYPE_F16 ? f16_bytes(n_cache) : f32_bytes(n_cache, -1.f, 1.f);
                const std::string tag = "n_past=" + std::to_string(n_past) + " N=" + std::to_string(N);
                const char *kind = variant == 1 ? "attention_sm_output " : variant == 2 ? "attention_f16 " : "attention ";
                check(std::string(kind) + tag, [&](ggml_context *c, ggml_cgraph *gf) {
                    ggml_tensor *cur = resident(input(c, "cur", GGML_TYPE_F32, 3 * E, N));
                    ggml_tensor *memk = resident(input(c, "memk", ct, (int64_t)n_layer * n_ctx * E));
                    ggml_tensor *memv = resident(input(c, "memv", ct, (int64_t)n_layer * n_ctx * E));
                    ggml_tensor *Qcur = ggml_view_2d(c, cur, E, N, cur->nb[1], 0 * sizeof(float) * E);
                    ggml_tensor *Kcur = ggml_view_2d(c, cur, E, N, cur->nb[1], 1 * sizeof(float) * E);
                    ggml_tensor *Vcur = ggml_view_2d(c, cur, E, N, cur->nb[1], 2 * sizeof(float) * E);
                    ggml_tensor *k = ggml_view_1d(c, memk, N * E, (ggml_element_size(memk) * E) * (il * n_ctx + n_past));
                    ggml_tensor *v = ggml_view_1d(c, memv, N * E, (ggml_element_size(memv) * E) * (il * n_ctx + n_past));
                    ggml_build_forward_expand(gf, ggml_cpy(c, Kcur, k));
                    ggml_build_forward_expand(gf, ggml_cpy(c, Vcur, v));
                    ggml_tensor *Q = ggml_permute(c, ggml_cont_3d(c, Qcur, Dh, H, N), 0, 2, 1, 3);
                    ggml_tensor *K = ggml_permute(c,
                        ggml_reshape_3d(c, ggml_view_1d(c, memk, (n_past + N) * E, il * n_ctx * ggml_element_size(memk) * E), Dh, H, n_past + N),
                        0, 2, 1, 3);
                    ggml_tensor *KQ = ggml_mul_mat(c, K, Q);
                    ggml_tensor *sm = ggml_soft_max(c, ggml_diag_mask_inf(c, ggml_scale(c, KQ, kq_scale), n_past));
                    if (sm_out) ggml_set_output(sm);
                    ggml_tensor *Vt = ggml_cont_3d(c,
                        ggml_permute(c,
                            ggml_reshape_3d(c, ggml_view_1d(c, memv, (n_past + N) * E, il * n_ctx * ggml_element_size(memv) * E), Dh, H, n_past + N),
                            1, 2, 0, 3),
                        n_past + N, Dh, H);
                    ggml_tensor *KQV = ggml_mul_mat(c, Vt, sm);
                    ggml_tensor *out = ggml_cont_2d(c, ggml_permute(c, KQV, 0, 2, 1, 3), E, N);
                    return std::vector<ggml_tensor *>{out};
                }, in);
            }
        }
    }

    // a whole GPT-2 decode layer (main-sched.cpp:600-812 at N = 1, n_past = 5 of n_ctx = 16): the
    // plugin runs it as the engine's two launches (backend.cpp plan_layers). The same allocated
    // graph is computed four times: new x (capture), new x (a hipGraph replay), new x again, then
    // new c_proj / MLP-projection weights (for Q4_0 / Q8_0 that frees the plugin's copies of
    // them: the captured graph must not be replayed). Each step against a fresh ggml-cpu run on the
    // same inputs, the layer output and both caches (row n_past written by the layer).
    for (ggml_type t : types) {
        const int E = 256, H = E / 64, F = 4 * E, n_ctx = 16, n_past = 5;
        std::vector<Inputs> steps(4);
        Inputs &in = steps[0];
        in.bytes["x"] = f32_bytes(E, -2.f, 2.f);
        in.bytes["g1"] = f32_bytes(E, 0.5f, 1.5f);
        in.bytes["b1"] = f32_bytes(E, -0.2f, 0.2f);
        in.bytes["g2"] = f32_bytes(E, 0.5f, 1.5f);
        in.bytes["b2"] = f32_bytes(E, -0.2f, 0.2f);
        in.bytes["w_qkv"] = q_bytes(t, E, 3 * E);
        in.bytes["b_qkv"] = f32_bytes(3 * E, -0.5f, 0.5f);
        in.bytes["w_o"] = q_bytes(t, E, E);
        in.bytes["b_o"] = f32_bytes(E, -0.5f, 0.5f);
        in.bytes["w_fc"] = q_bytes(t, E, F);
        in.bytes["b_fc"] = f32_bytes(F, -0.5f, 0.5f);
        in.bytes["w_mp"] = q_bytes(t, F, E);
        in.bytes["b_mp"] = f32_bytes(E, -0.5f, 0.5f);
        in.bytes["memk"] = f32_bytes((size_t)n_ctx * E, -1.f, 1.f);
        in.bytes["memv"] = f32_bytes((size_t)n_ctx * E, -1.f, 1.f);
        for (int k = 1; k < 4; ++k) steps[k].bytes["x"] = f32_bytes(E, -2.f, 2.f);
        steps[3].bytes["w_o"] = q_bytes(t, E, E);
        steps[3].bytes["w_mp"] = q_bytes(t, F, E);
        const std::string name = std::string("gpt2_layer ") + ggml_type_name(t);
        fprintf(stderr, "CASE %s\n", name.c_str());
        // weights stay allocated (as in a weight buffer): later steps compute without re-setting
        // them, so ggml-alloc must not hand their memory to an intermediate after their last use
        auto W = [&](ggml_context *c, const char *nm, ggml_type ty, int64_t n0, int64_t n1 = 1) {
            return resident(input(c, nm, ty, n0, n1));
        };
        const Builder layer = [&](ggml_context *c, ggml_cgraph *gf) {
            ggml_tensor *x = input(c, "x", GGML_TYPE_F32, E);
            ggml_tensor *memk = resident(input(c, "memk", GGML_TYPE_F32, n_ctx * E));
            ggml_tensor *memv = resident(input(c, "memv", GGML_TYPE_F32, n_ctx * E));
            ggml_tensor *cur = ggml_add(c, ggml_mul(c, ggml_norm(c, x, eps), W(c, "g1", GGML_TYPE_F32, E)), W(c, "b1", GGML_TYPE_F32, E));
            cur = ggml_add(c, ggml_mul_mat(c, W(c, "w_qkv", t, E, 3 * E), cur), W(c, "b_qkv", GGML_TYPE_F32, 3 * E));
            ggml_tensor *Qcur = ggml_view_2d(c, cur, E, 1, cur->nb[1], 0);
            ggml_tensor *Kcur = ggml_view_2d(c, cur, E, 1, cur->nb[1], 1 * sizeof(float) * E);
            ggml_tensor *Vcur = ggml_view_2d(c, cur, E, 1, cur->nb[1], 2 * sizeof(float) * E);
            ggml_build_forward_expand(gf, ggml_cpy(c, Kcur, ggml_view_1d(c, memk, E, ggml_element_size(memk) * E * n_past)));
            ggml_build_forward_expand(gf, ggml_cpy(c, Vcur, ggml_view_1d(c, memv, E, ggml_element_size(memv) * E * n_past)));
            ggml_tensor *Q = ggml_permute(c, ggml_cont_3d(c, Qcur, 64, H, 1), 0, 2, 1, 3);
            ggml_tensor *K = ggml_permute(c, ggml_reshape_3d(c, ggml_view_1d(c, memk, (n_past + 1) * E, 0), 64, H, n_past + 1), 0, 2, 1, 3);
            ggml_tensor *sm = ggml_soft_max(c, ggml_diag_mask_inf(c, ggml_scale(c, ggml_mul_mat(c, K, Q), 0.125f), n_past));
            ggml_tensor *Vt = ggml_cont_3d(c, ggml_permute(c, ggml_reshape_3d(c, ggml_view_1d(c, memv, (n_past + 1) * E, 0), 64, H, n_past + 1), 1, 2, 0, 3),
                                           n_past + 1, 64, H);
            cur = ggml_cont_2d(c, ggml_permute(c, ggml_mul_mat(c, Vt, sm), 0, 2, 1, 3), E, 1);
            cur = ggml_add(c, ggml_mul_mat(c, W(c, "w_o", t, E, E), cur), W(c, "b_o", GGML_TYPE_F32, E));
            ggml_tensor *r1 = ggml_add(c, cur, x);
            cur = ggml_add(c, ggml_mul(c, ggml_norm(c, r1, eps), W(c, "g2", GGML_TYPE_F32, E)), W(c, "b2", GGML_TYPE_F32, E));
            cur = ggml_gelu(c, ggml_add(c, ggml_mul_mat(c, W(c, "w_fc", t, E, F), cur), W(c, "b_fc", GGML_TYPE_F32, F)));
            cur = ggml_add(c, ggml_mul_mat(c, W(c, "w_mp", t, F, E), cur), W(c, "b_mp", GGML_TYPE_F32, E));
            ggml_tensor *r2 = ggml_add(c, cur, r1);
            return std::vector<ggml_tensor *>{r2, memk, memv};
        };
        const auto got = run_steps(gpu, layer, steps);
        Inputs merged;
        for (int k = 0; k < 4; ++k) {
            for (const auto &kv : steps[k].bytes) merged.bytes[kv.first] = kv.second;
            const auto want = run(cpu, layer, merged);
            bool ok = true;
            std::string detail;
            for (size_t j = 0; j < want.size(); ++j) {
                bool finite = true;
                const double e = nmse(got[k][j], want[j], &finite);
                ok = ok && finite && e <= 5e-4;
                char buf[64];
                snprintf(buf, sizeof buf, " out%zu=%.3e%s", j, e, finite ? "" : "(nonfinite)");
                detail += buf;
            }
            fails += !ok;
            printf("%s %s step %d%s\n", ok ? "OK  " : "FAIL", name.c_str(), k, detail.c_str());
            fflush(stdout);
        }
    }

    ggml_backend_free(gpu);
    ggml_backend_free(cpu);
    printf("%s\n", fails ? "FUSION_CHECK_FAIL" : "FUSION_CHECK_OK");
    return fails ? 1 : 0;
}
