// gpt2.cpp — GPT-2 decode engine on gfx950 (C-ABI: include/ggml-mi355x-gpt2.h).
//
// Same model and arithmetic as the reference's examples/gpt-2/main-sched.cpp (graph
// :553-858, loader :155-546), restructured for MI355X:
//   * per layer, five launches instead of ~25 ggml nodes:
//       qkv  = mmvq_fused(attn_w, LN1(x)) + attn_b
//       attn = attn_decode(qkv, KV cache)            (stores K/V of the new token)
//       x   += mmvq_fused(proj_w, attn) + proj_b
//       h    = gelu(mmvq_fused(fc_w, LN2(x)) + fc_b)
//       x   += mmvq_fused(mlp_proj_w, h) + mlp_proj_b
//     so each weight matrix is streamed once and no normalized / biased intermediate makes an
//     HBM round trip;
//   * positions and next tokens live in device memory, so one step is a fixed launch sequence
//     captured once into a hipGraph and replayed;
//   * a model object is one pipeline stage (a layer range on one GPU); stages exchange the
//     n_seq x n_embd residual stream (3 KB per sequence) through the host driver (gpt2.py).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <string>
#include <vector>

#include "../../include/ggml-mi355x-gpt2.h"
#include "dispatch.h"
#include "qcommon.h"
#include "settings.h"

namespace mi355x {
hipError_t mmvq_fused_launch(int type, const MmArgs &a, int nc, int rpw, hipStream_t st);
hipError_t mmvq_fused_prepare(int type);
int mmvq_fused_pick_nc(int M, int K);
unsigned long long *stamps_buffer();
hipError_t gpt2_embed_launch(int wtype, const void *wte, int64_t wte_nb1, const float *wpe, const int32_t *tokens,
                             const int32_t *pos, float *x, int n_seq, int n_embd, int n_vocab, int n_ctx, hipStream_t st);
hipError_t gpt2_attn_launch(const float *qkv, float *kc, float *vc, const int32_t *pos, float *part, int n_seq, int n_head,
                            int n_embd, int n_ctx, float scale, hipStream_t st);
hipError_t gpt2_argmax_launch(const float *pv, const int32_t *pi, int n_seq, int32_t *tokens, int32_t *pos, hipStream_t st);
hipError_t gpt2_argmax_reset(float *pv, int32_t *pi, int n_seq, hipStream_t st);
hipError_t gpt2_advance_launch(int32_t *pos, int n_seq, hipStream_t st);
}  // namespace mi355x

using namespace mi355x;

namespace {

constexpr uint32_t FILE_MAGIC = 0x67676d6c;   // GGML_FILE_MAGIC, include/ggml.h:212
constexpr int QNT_VERSION_FACTOR = 1000;      // include/ggml.h:216

// ggml_ftype_to_ggml_type (src/ggml.c:1312-1342) restricted to what the fused mat-vec runs
int ftype_to_type(int ftype) {
    switch (ftype) {
        case 0: return T_F32;
        case 2: return T_Q4_0;
        case 7: return T_Q8_0;
        case 12: return T_Q4_K;
        case 13: return T_Q5_K;
        case 14: return T_Q6_K;
        default: return -1;
    }
}

int64_t row_bytes(int type, int64_t ne0) {
    if (type == T_F32) return ne0 * 4;
    return ne0 / type_blck(type) * type_bytes(type);
}

struct Tensor {
    uint8_t *data = nullptr;
    int type = T_F32;
    int64_t ne0 = 0, ne1 = 1;
    int64_t nbytes() const { return row_bytes(type, ne0) * ne1; }
};

struct Layer {
    Tensor ln1_g, ln1_b, ln2_g, ln2_b, attn_w, attn_b, proj_w, proj_b, fc_w, fc_b, mproj_w, mproj_b;
};

}  // namespace

struct ggml_mi355x_gpt2_model {
    ggml_mi355x_gpt2_hparams hp{};
    int wtype = -1;
    int l0 = 0, l1 = 0;
    bool first = false, last = false;
    int device = 0;
    uint8_t *arena = nullptr;
    int64_t arena_bytes = 0;
    Tensor wte, wpe, ln_f_g, ln_f_b, lm_head;
    std::vector<Layer> layers;                 // layers[l - l0]
    std::map<std::string, Tensor *> by_name;   // legacy names of the tensors this stage owns
    // 32-block types, two-launch layer: per layer, head-major c_proj and slice-major MLP
    // projection copies (gpt2_block_repack). One set per model, shared by its contexts;
    // (re)made from the weights by every ctx_init, so a context created after weights were
    // written through ggml_mi355x_gpt2_model_tensor sees them (the buffer never moves, so
    // captured decode graphs of earlier contexts stay valid and see the same bytes).
    uint8_t *rep = nullptr;
    std::vector<const uint8_t *> rep_o, rep_mp;
};

struct ggml_mi355x_gpt2_ctx {
    ggml_mi355x_gpt2_model *m = nullptr;
    int n_seq = 0;
    uint8_t *arena = nullptr;
    int32_t *tokens = nullptr, *pos = nullptr;
    float *x = nullptr, *qkv = nullptr, *attn = nullptr, *h = nullptr, *logits = nullptr;
    float *kc = nullptr, *vc = nullptr;        // [layer][seq][n_ctx][n_embd]
    float *part = nullptr;                     // attention partials [seq][head][ATTN_SPLITS][ATTN_PART_STRIDE]
    float *amax_v = nullptr;                   // lm_head per-workgroup argmax partials [seq][ARGMAX_SLOTS]
    int32_t *amax_i = nullptr;
    // two-launch layer (gpt2_block.hip): materialized residuals after attention / after the MLP
    // and the K-split partial slabs [split][seq][n_embd] of c_proj (per head) and the MLP proj
    bool block = false, rep = false;           // rep: the layers read the model's repacked copies
    float *xr = nullptr, *xm = nullptr, *p_attn = nullptr, *p_mlp = nullptr;
    std::map<hipStream_t, hipGraphExec_t> graphs;
};

namespace {

int hip_status_at(hipError_t e, const char *where) {
    if (e == hipSuccess) return GGML_MI355X_OK;
    fprintf(stderr, "gpt2: %s: %s\n", where, hipGetErrorString(e));
    return GGML_MI355X_EHIP;
}
#define hip_status(e) hip_status_at((e), #e)

int pick_nc(int n, int K) { return mmvq_fused_pick_nc(n, K); }

// y[n_seq][N] (+)= W[N][K] . x[n_seq][K] with the fused prologue / epilogue
int fused_matvec(const ggml_mi355x_gpt2_ctx *c, const Tensor &w, const float *x, float *y, const Tensor *ln_g, const Tensor *ln_b,
                 const Tensor *bias, int epi, hipStream_t st, const float *attn_part = nullptr) {
    // EPI_ARGMAX writes one partial per workgroup: ARGMAX_SLOTS bounds the grid (mmvq_fused.hip)
    MmArgs a{};
    const int K = (int)w.ne0, N = (int)w.ne1, M = c->n_seq;
    a.w = w.data;
    a.nb01 = row_bytes(w.type, K);
    a.nb02 = a.nb03 = a.nb01 * N;
    a.x = reinterpret_cast<const uint8_t *>(x);
    a.nb11 = (int64_t)K * 4;
    a.nb12 = a.nb13 = a.nb11 * M;
    a.dst = reinterpret_cast<uint8_t *>(y);
    a.nb1 = (int64_t)N * 4;
    a.nb2 = a.nb3 = a.nb1 * M;
    a.K = K;
    a.N = N;
    a.M = M;
    a.ne12 = a.ne13 = a.r2 = a.r3 = 1;
    a.x_aligned16 = 1;
    a.ln_g = ln_g ? reinterpret_cast<const float *>(ln_g->data) : nullptr;
    a.ln_b = ln_b ? reinterpret_cast<const float *>(ln_b->data) : nullptr;
    a.ln_eps = 1e-5f;   // gpt2_hparams::eps, main-sched.cpp:51
    a.bias = bias ? reinterpret_cast<const float *>(bias->data) : nullptr;
    a.epi = epi;
    a.amax_v = c->amax_v;
    a.amax_i = c->amax_i;
    a.attn_part = attn_part;                   // c_proj: activations = merged attention partials
    a.n_head = c->m->hp.n_head;
    // diagnostics: GGML_MI355X_STAMPS=1 + GGML_MI355X_STAMP_MV=i stamps the i-th fused mat-vec of
    // a decode step (0 = first layer's c_attn); scripts/gpt2_stamps.py reads them
    const int stamp_mv = settings().stamp_mv;
    static thread_local int mv_counter = 0;
    if (mv_counter++ == stamp_mv) a.stamps = stamps_buffer();
    if (epi & EPI_ARGMAX) mv_counter = 0;      // the last mat-vec of a step
    a.fused = 1;
    // the attention-merge prologue (c_proj) keeps its partials in registers: groups of <= 3 columns
    const int nc = attn_part ? (M % 3 == 0 ? 3 : M % 2 == 0 ? 2 : 1) : pick_nc(M, K);
    return hip_status(mmvq_fused_launch(w.type, a, nc, N >= 16384 ? 2 : 1, st));
}

int run_step(ggml_mi355x_gpt2_ctx *c, hipStream_t st) {
    const ggml_mi355x_gpt2_model *m = c->m;
    const auto &hp = m->hp;
    const int E = hp.n_embd;
    int rc;
    // the two-launch layer takes the embedding in layer 0's prologue (32-block types)
    const bool emb_fused = c->block && m->first && gpt2_block_embeds(m->wtype) && !settings().gpt2_embed_kernel;
    if (m->first && !emb_fused) {
        rc = hip_status(gpt2_embed_launch(m->wte.type, m->wte.data, row_bytes(m->wte.type, E), reinterpret_cast<const float *>(m->wpe.data),
                                          c->tokens, c->pos, c->x, c->n_seq, E, hp.n_vocab, hp.n_ctx, st));
        if (rc) return rc;
    }
    const float kq_scale = 1.0f / sqrtf(float(E) / hp.n_head);   // main-sched.cpp:587
    const size_t cache_layer = (size_t)c->n_seq * hp.n_ctx * E;
    if (c->block) {
        // two launches per layer; the residual travels as (base, bias, partial slabs) and is
        // summed by the next launch's prologue, then materialized into c->x for the stage
        // boundary / lm_head
        const float *base = c->x, *bias = nullptr, *parts = nullptr;
        int np = 0;
        const int n_sl = gpt2_block_mlp_slices(E);
        for (int l = m->l0; l < m->l1; ++l) {
            const Layer &L = m->layers[l - m->l0];
            float *kc = c->kc + (size_t)(l - m->l0) * cache_layer;
            float *vc = c->vc + (size_t)(l - m->l0) * cache_layer;
            auto f = [](const Tensor &t) { return reinterpret_cast<const float *>(t.data); };
            const bool rp = c->rep;
            rc = hip_status(gpt2_attn_block_launch(l - m->l0, m->wtype, base, bias, parts, np, c->xr, f(L.ln1_g), f(L.ln1_b), 1e-5f, L.attn_w.data,
                                                   row_bytes(m->wtype, E), f(L.attn_b), kc, vc, c->pos, kq_scale, hp.n_ctx,
                                                   rp ? m->rep_o[l - m->l0] : L.proj_w.data, row_bytes(m->wtype, E), c->p_attn, E,
                                                   hp.n_head, c->n_seq, emb_fused && l == 0 ? m->wte.data : nullptr,
                                                   row_bytes(m->wtype, E), reinterpret_cast<const float *>(m->wpe.data), c->tokens,
                                                   hp.n_vocab, st));
            if (rc) return rc;
            rc = hip_status(gpt2_mlp_block_launch(l - m->l0, m->wtype, c->xr, f(L.proj_b), c->p_attn, hp.n_head, c->xm, f(L.ln2_g), f(L.ln2_b),
                                                  1e-5f, L.fc_w.data, row_bytes(m->wtype, E), f(L.fc_b),
                                                  rp ? m->rep_mp[l - m->l0] : L.mproj_w.data, row_bytes(m->wtype, 4 * E), c->p_mlp, E,
                                                  hp.n_head, c->n_seq, st));
            if (rc) return rc;
            base = c->xm;
            bias = f(L.mproj_b);
            parts = c->p_mlp;
            np = n_sl;
        }
        if ((rc = hip_status(gpt2_resid_launch(base, bias, parts, np, c->x, E, c->n_seq, st)))) return rc;
        if (m->last) {
            if ((rc = fused_matvec(c, m->lm_head, c->x, c->logits, &m->ln_f_g, &m->ln_f_b, nullptr, EPI_ARGMAX, st))) return rc;
            return hip_status(gpt2_argmax_launch(c->amax_v, c->amax_i, c->n_seq, c->tokens, c->pos, st));
        }
        return hip_status(gpt2_advance_launch(c->pos, c->n_seq, st));
    }
    for (int l = m->l0; l < m->l1; ++l) {
        const Layer &L = m->layers[l - m->l0];
        float *kc = c->kc + (size_t)(l - m->l0) * cache_layer;
        float *vc = c->vc + (size_t)(l - m->l0) * cache_layer;
        if ((rc = fused_matvec(c, L.attn_w, c->x, c->qkv, &L.ln1_g, &L.ln1_b, &L.attn_b, 0, st))) return rc;
        if ((rc = hip_status(gpt2_attn_launch(c->qkv, kc, vc, c->pos, c->part, c->n_seq, hp.n_head, E, hp.n_ctx, kq_scale, st)))) return rc;
        if ((rc = fused_matvec(c, L.proj_w, c->attn, c->x, nullptr, nullptr, &L.proj_b, EPI_RESID, st, c->part))) return rc;
        if ((rc = fused_matvec(c, L.fc_w, c->x, c->h, &L.ln2_g, &L.ln2_b, &L.fc_b, EPI_GELU, st))) return rc;
        if ((rc = fused_matvec(c, L.mproj_w, c->h, c->x, nullptr, nullptr, &L.mproj_b, EPI_RESID, st))) return rc;
    }
    if (m->last) {
        // lm_head with the per-workgroup argmax epilogue, then one small launch that picks the
        // token and advances the positions
        if ((rc = fused_matvec(c, m->lm_head, c->x, c->logits, &m->ln_f_g, &m->ln_f_b, nullptr, EPI_ARGMAX, st))) return rc;
        return hip_status(gpt2_argmax_launch(c->amax_v, c->amax_i, c->n_seq, c->tokens, c->pos, st));
    }
    return hip_status(gpt2_advance_launch(c->pos, c->n_seq, st));
}

std::string layer_name(int i, const char *suffix) { return "model/h" + std::to_string(i) + "/" + suffix; }

}  // namespace

extern "C" {

int ggml_mi355x_gpt2_read_hparams(const char *fname, ggml_mi355x_gpt2_hparams *hp) {
    std::ifstream f(fname, std::ios::binary);
    if (!f || !hp) return GGML_MI355X_EINVAL;
    uint32_t magic = 0;
    f.read(reinterpret_cast<char *>(&magic), 4);
    if (!f || magic != FILE_MAGIC) return GGML_MI355X_EINVAL;
    int32_t v[6];
    f.read(reinterpret_cast<char *>(v), sizeof(v));
    if (!f) return GGML_MI355X_EINVAL;
    hp->n_vocab = v[0];
    hp->n_ctx = v[1];
    hp->n_embd = v[2];
    hp->n_head = v[3];
    hp->n_layer = v[4];
    hp->ftype = v[5] % QNT_VERSION_FACTOR;
    return GGML_MI355X_OK;
}

int ggml_mi355x_gpt2_model_init(const ggml_mi355x_gpt2_hparams *hp, int32_t layer_begin, int32_t layer_end,
                                ggml_mi355x_gpt2_model **out) {
    if (!hp || !out) return GGML_MI355X_EINVAL;
    *out = nullptr;
    const int wtype = ftype_to_type(hp->ftype);
    if (wtype < 0 || hp->n_embd <= 0 || hp->n_head <= 0 || hp->n_embd != 64 * hp->n_head || hp->n_vocab <= 0 || hp->n_ctx <= 0 ||
        hp->n_layer <= 0 || layer_begin < 0 || layer_end > hp->n_layer || layer_begin >= layer_end)
        return GGML_MI355X_EINVAL;
    // fused mat-vec: K % 64 == 0 and K <= 8192 for K = n_embd and 4 n_embd; K-quants need
    // whole 256-blocks
    const int blck = wtype == T_F32 ? 1 : type_blck(wtype);
    if (wtype == T_F32 || hp->n_embd % 64 != 0 || 4 * hp->n_embd > 8192 || hp->n_embd % blck != 0) return GGML_MI355X_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GGML_MI355X_ENODEV;

    auto *m = new ggml_mi355x_gpt2_model();
    m->hp = *hp;
    m->wtype = wtype;
    m->l0 = layer_begin;
    m->l1 = layer_end;
    m->first = layer_begin == 0;
    m->last = layer_end == hp->n_layer;
    (void)hipGetDevice(&m->device);
    const int64_t E = hp->n_embd;
    auto def = [&](Tensor &t, const std::string &name, int type, int64_t ne0, int64_t ne1) {
        t.type = type;
        t.ne0 = ne0;
        t.ne1 = ne1;
        m->by_name[name] = &t;
    };
    // shapes and types: main-sched.cpp:256-297
    if (m->first) {
        def(m->wte, "model/wte", wtype, E, hp->n_vocab);
        def(m->wpe, "model/wpe", T_F32, E, hp->n_ctx);
    }
    if (m->last) {
        def(m->ln_f_g, "model/ln_f/g", T_F32, E, 1);
        def(m->ln_f_b, "model/ln_f/b", T_F32, E, 1);
        def(m->lm_head, "model/lm_head", wtype, E, hp->n_vocab);
    }
    m->layers.resize(layer_end - layer_begin);
    for (int i = layer_begin; i < layer_end; ++i) {
        Layer &L = m->layers[i - layer_begin];
        def(L.ln1_g, layer_name(i, "ln_1/g"), T_F32, E, 1);
        def(L.ln1_b, layer_name(i, "ln_1/b"), T_F32, E, 1);
        def(L.ln2_g, layer_name(i, "ln_2/g"), T_F32, E, 1);
        def(L.ln2_b, layer_name(i, "ln_2/b"), T_F32, E, 1);
        def(L.attn_w, layer_name(i, "attn/c_attn/w"), wtype, E, 3 * E);
        def(L.attn_b, layer_name(i, "attn/c_attn/b"), T_F32, 3 * E, 1);
        def(L.proj_w, layer_name(i, "attn/c_proj/w"), wtype, E, E);
        def(L.proj_b, layer_name(i, "attn/c_proj/b"), T_F32, E, 1);
        def(L.fc_w, layer_name(i, "mlp/c_fc/w"), wtype, E, 4 * E);
        def(L.fc_b, layer_name(i, "mlp/c_fc/b"), T_F32, 4 * E, 1);
        def(L.mproj_w, layer_name(i, "mlp/c_proj/w"), wtype, 4 * E, E);
        def(L.mproj_b, layer_name(i, "mlp/c_proj/b"), T_F32, E, 1);
    }
    int64_t total = 0;
    for (auto &kv : m->by_name) total += (kv.second->nbytes() + 255) & ~int64_t(255);
    if (hipMalloc(&m->arena, (size_t)total) != hipSuccess) {
        delete m;
        return GGML_MI355X_ENOMEM;
    }
    m->arena_bytes = total;
    int64_t off = 0;
    for (auto &kv : m->by_name) {
        kv.second->data = m->arena + off;
        off += (kv.second->nbytes() + 255) & ~int64_t(255);
    }
    *out = m;
    return GGML_MI355X_OK;
}

int ggml_mi355x_gpt2_model_load(ggml_mi355x_gpt2_model *m, const char *fname) {
    if (!m || !fname) return GGML_MI355X_EINVAL;
    ggml_mi355x_gpt2_hparams hp{};
    if (ggml_mi355x_gpt2_read_hparams(fname, &hp) != 0) return GGML_MI355X_EINVAL;
    if (memcmp(&hp, &m->hp, sizeof(hp)) != 0) {
        fprintf(stderr, "gpt2: '%s' hparams differ from the model's\n", fname);
        return GGML_MI355X_EINVAL;
    }
    std::ifstream f(fname, std::ios::binary);
    f.seekg(4 + 6 * 4);
    int32_t n_vocab = 0;
    f.read(reinterpret_cast<char *>(&n_vocab), 4);
    if (!f || n_vocab != hp.n_vocab) return GGML_MI355X_EINVAL;   // main-sched.cpp:200-207
    for (int i = 0; i < n_vocab; ++i) {   // vocab words are skipped (:210-222)
        uint32_t len = 0;
        f.read(reinterpret_cast<char *>(&len), 4);
        f.seekg(len, std::ios::cur);
        if (!f) return GGML_MI355X_EINVAL;
    }
    std::vector<char> buf;
    bool has_lm_head = false;
    std::map<std::string, bool> seen;
    for (;;) {   // tensor records until EOF (:433-517)
        int32_t hdr[3];
        f.read(reinterpret_cast<char *>(hdr), sizeof(hdr));
        if (f.eof()) break;
        if (!f) return GGML_MI355X_EINVAL;
        const int n_dims = hdr[0], len = hdr[1], ttype = hdr[2];
        if (n_dims < 1 || n_dims > 2 || len <= 0 || len > 256) return GGML_MI355X_EINVAL;
        int32_t ne[2] = {1, 1};
        f.read(reinterpret_cast<char *>(ne), 4 * n_dims);
        std::string name(len, '\0');
        f.read(&name[0], len);
        if (!f) return GGML_MI355X_EINVAL;
        // every name must be a GPT-2 tensor (:453-456); shapes are checked for the ones kept
        const bool known = name == "model/wte" || name == "model/wpe" || name == "model/lm_head" || name == "model/ln_f/g" ||
                           name == "model/ln_f/b" || name.rfind("model/h", 0) == 0;
        if (!known) {
            fprintf(stderr, "gpt2: unknown tensor '%s' in model file\n", name.c_str());
            return GGML_MI355X_EINVAL;
        }
        const int64_t nel = (int64_t)ne[0] * ne[1];
        const int64_t nbytes = ttype == T_F32 ? nel * 4 : (type_blck(ttype) ? nel / type_blck(ttype) * type_bytes(ttype) : -1);
        if (nbytes < 0) {
            fprintf(stderr, "gpt2: tensor '%s' has unsupported type %d\n", name.c_str(), ttype);
            return GGML_MI355X_EINVAL;
        }
        std::vector<Tensor *> dst;
        auto it = m->by_name.find(name);
        if (it != m->by_name.end()) dst.push_back(it->second);
        if (name == "model/wte" && m->last && !has_lm_head) dst.push_back(&m->lm_head);   // tied head (:503-510)
        if (name == "model/lm_head") has_lm_head = true;
        if (dst.empty()) {
            f.seekg(nbytes, std::ios::cur);
            continue;
        }
        buf.resize((size_t)nbytes);
        f.read(buf.data(), nbytes);
        if (!f) return GGML_MI355X_EINVAL;
        for (Tensor *t : dst) {
            if (t->ne0 != ne[0] || t->ne1 != ne[1] || t->type != ttype || t->nbytes() != nbytes) {
                fprintf(stderr, "gpt2: tensor '%s' has wrong shape/type in model file: got [%d, %d] type %d, expected [%lld, %lld] type %d\n",
                        name.c_str(), ne[0], ne[1], ttype, (long long)t->ne0, (long long)t->ne1, t->type);
                return GGML_MI355X_EINVAL;
            }
            if (hipMemcpy(t->data, buf.data(), (size_t)nbytes, hipMemcpyHostToDevice) != hipSuccess) return GGML_MI355X_EHIP;
        }
        seen[name] = true;
        if (name == "model/wte" && m->last) seen["model/lm_head"] = true;
    }
    for (auto &kv : m->by_name) {
        if (!seen.count(kv.first)) {
            fprintf(stderr, "gpt2: tensor '%s' missing from model file\n", kv.first.c_str());
            return GGML_MI355X_EINVAL;
        }
    }
    return GGML_MI355X_OK;
}

int ggml_mi355x_gpt2_model_tensor(ggml_mi355x_gpt2_model *m, const char *name, void **data, int32_t *type, int64_t ne[2]) {
    if (!m || !name) return GGML_MI355X_EINVAL;
    auto it = m->by_name.find(name);
    if (it == m->by_name.end()) return GGML_MI355X_EINVAL;
    if (data) *data = it->second->data;
    if (type) *type = it->second->type;
    if (ne) {
        ne[0] = it->second->ne0;
        ne[1] = it->second->ne1;
    }
    return GGML_MI355X_OK;
}

int64_t ggml_mi355x_gpt2_model_bytes(const ggml_mi355x_gpt2_model *m) { return m ? m->arena_bytes : 0; }

void ggml_mi355x_gpt2_model_free(ggml_mi355x_gpt2_model *m) {
    if (!m) return;
    if (m->arena) (void)hipFree(m->arena);
    if (m->rep) (void)hipFree(m->rep);
    delete m;
}

}  // extern "C"

namespace {
// (re)make the model's repacked c_proj / MLP-projection copies from its current weights
int model_repack(ggml_mi355x_gpt2_model *m) {
    const size_t n_layers = m->l1 - m->l0;
    size_t ob = 0, mb = 0;
    (void)gpt2_block_repack(m->wtype, m->hp.n_embd, nullptr, nullptr, nullptr, nullptr, &ob, &mb, nullptr);
    if (!m->rep) {
        if (hipMalloc(&m->rep, (ob + mb) * n_layers) != hipSuccess) {
            m->rep = nullptr;
            return GGML_MI355X_ENOMEM;
        }
        for (size_t l = 0; l < n_layers; ++l) {
            m->rep_o.push_back(m->rep + l * (ob + mb));
            m->rep_mp.push_back(m->rep + l * (ob + mb) + ob);
        }
    }
    // other contexts of this model may have decode work queued on their own streams that reads
    // these copies: let it finish before rewriting them (a ctx_init must not run concurrently with
    // another thread's decode calls on the same model; include/ggml-mi355x-gpt2.h)
    if (hipDeviceSynchronize() != hipSuccess) return GGML_MI355X_EHIP;
    for (size_t l = 0; l < n_layers; ++l) {
        const Layer &L = m->layers[l];
        if (gpt2_block_repack(m->wtype, m->hp.n_embd, L.proj_w.data, const_cast<uint8_t *>(m->rep_o[l]), L.mproj_w.data,
                              const_cast<uint8_t *>(m->rep_mp[l]), nullptr, nullptr, nullptr) != hipSuccess)
            return GGML_MI355X_EHIP;
    }
    return hipDeviceSynchronize() == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
}
}  // namespace

extern "C" {

int ggml_mi355x_gpt2_ctx_init(ggml_mi355x_gpt2_model *m, int32_t n_seq, ggml_mi355x_gpt2_ctx **out) {
    if (!m || !out || n_seq < 1 || n_seq > 64) return GGML_MI355X_EINVAL;
    *out = nullptr;
    const auto &hp = m->hp;
    const size_t E = hp.n_embd, S = n_seq;
    const size_t n_layers = m->l1 - m->l0;
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t b_tok = al(4 * S), b_x = al(4 * S * E), b_qkv = al(12 * S * E), b_h = al(16 * S * E);
    const size_t b_logits = m->last ? al(4 * S * hp.n_vocab) : 0;
    const size_t b_cache = al(4 * n_layers * S * hp.n_ctx * E);
    const size_t b_amax = m->last ? al(4 * S * ARGMAX_SLOTS) : 0;
    const size_t b_part = al(4 * S * hp.n_head * ATTN_SPLITS * ATTN_PART_STRIDE);
    // GGML_MI355X_GPT2_BLOCK=0 selects the five-launch layer (A/B and fallback)
    const bool block = gpt2_block_supported(hp.n_embd, hp.n_head) && settings().gpt2_block != 0;
    const size_t b_pa = block ? al(4 * S * E * hp.n_head) : 0, b_pm = block ? al(4 * S * E * gpt2_block_mlp_slices(hp.n_embd)) : 0;
    const size_t b_xb = block ? b_x : 0;
    const size_t total = 2 * b_tok + 2 * b_x + b_qkv + b_h + b_logits + 2 * b_cache + 2 * b_amax + b_part + 2 * b_xb + b_pa + b_pm;
    if (mmvq_fused_prepare(m->wtype) != hipSuccess) return GGML_MI355X_EHIP;   // before any capture
    auto *c = new ggml_mi355x_gpt2_ctx();
    c->m = m;
    c->n_seq = n_seq;
    if (hipMalloc(&c->arena, total) != hipSuccess) {
        delete c;
        return GGML_MI355X_ENOMEM;
    }
    uint8_t *p = c->arena;
    auto take = [&](size_t b) { uint8_t *r = p; p += b; return r; };
    c->tokens = reinterpret_cast<int32_t *>(take(b_tok));
    c->pos = reinterpret_cast<int32_t *>(take(b_tok));
    c->x = reinterpret_cast<float *>(take(b_x));
    c->attn = reinterpret_cast<float *>(take(b_x));
    c->qkv = reinterpret_cast<float *>(take(b_qkv));
    c->h = reinterpret_cast<float *>(take(b_h));
    c->logits = m->last ? reinterpret_cast<float *>(take(b_logits)) : nullptr;
    c->kc = reinterpret_cast<float *>(take(b_cache));
    c->vc = reinterpret_cast<float *>(take(b_cache));
    c->part = reinterpret_cast<float *>(take(b_part));
    c->block = block;
    if (block) {
        c->xr = reinterpret_cast<float *>(take(b_xb));
        c->xm = reinterpret_cast<float *>(take(b_xb));
        c->p_attn = reinterpret_cast<float *>(take(b_pa));
        c->p_mlp = reinterpret_cast<float *>(take(b_pm));
    }
    if (m->last) {
        c->amax_v = reinterpret_cast<float *>(take(b_amax));
        c->amax_i = reinterpret_cast<int32_t *>(take(b_amax));
    }
    if (hipMemset(c->arena, 0, total) != hipSuccess ||
        (m->last && (gpt2_argmax_reset(c->amax_v, c->amax_i, n_seq, nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess))) {
        (void)hipFree(c->arena);
        delete c;
        return GGML_MI355X_EHIP;
    }
    if (block && gpt2_block_repacks(m->wtype)) {
        if (int rc = model_repack(m)) {
            ggml_mi355x_gpt2_ctx_free(c);
            return rc;
        }
        c->rep = true;
    }
    *out = c;
    return GGML_MI355X_OK;
}

int ggml_mi355x_gpt2_ctx_buffers(ggml_mi355x_gpt2_ctx *c, int32_t **tokens, int32_t **pos, float **hidden, float **logits) {
    if (!c) return GGML_MI355X_EINVAL;
    if (tokens) *tokens = c->tokens;
    if (pos) *pos = c->pos;
    if (hidden) *hidden = c->x;
    if (logits) *logits = c->logits;
    return GGML_MI355X_OK;
}

int ggml_mi355x_gpt2_decode(ggml_mi355x_gpt2_ctx *c, void *stream, int32_t use_graph) {
    if (!c) return GGML_MI355X_EINVAL;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (!use_graph) return run_step(c, st);
    auto it = c->graphs.find(st);
    if (it == c->graphs.end()) {
        if (st == nullptr) return GGML_MI355X_EINVAL;   // the legacy default stream cannot be captured
        hipGraph_t g = nullptr;
        if (int rc = hip_status(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed))) return rc;
        const int rc = run_step(c, st);
        const hipError_t e = hipStreamEndCapture(st, &g);
        if (rc != 0 || e != hipSuccess) {
            if (g) (void)hipGraphDestroy(g);
            return rc != 0 ? rc : hip_status(e);
        }
        hipGraphExec_t ex = nullptr;
        const hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (ei != hipSuccess) return hip_status(ei);
        it = c->graphs.emplace(st, ex).first;
    }
    return hip_status(hipGraphLaunch(it->second, st));
}

void ggml_mi355x_gpt2_ctx_free(ggml_mi355x_gpt2_ctx *c) {
    if (!c) return;
    for (auto &kv : c->graphs) (void)hipGraphExecDestroy(kv.second);
    if (c->arena) (void)hipFree(c->arena);
    delete c;
}

int ggml_mi355x_memcpy(void *dst, const void *src, size_t bytes, void *stream) {
    if (bytes == 0) return GGML_MI355X_OK;
    if (!dst || !src) return GGML_MI355X_EINVAL;
    return hip_status(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, static_cast<hipStream_t>(stream)));
}

}  // extern "C"
