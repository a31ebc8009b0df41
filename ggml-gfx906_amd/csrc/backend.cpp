// backend.cpp — the ggml dynamic backend ("MI355X") wrapping the gfx950 quantized MUL_MAT path.
//
// Fills the vtables of the reference's backend ABI (src/ggml-backend-impl.h:17-207; restated in
// ggml_abi.h) so an unmodified ggml loads this library with GGML_BACKEND_PATH /
// ggml_backend_load() and routes GGML_OP_MUL_MAT / GGML_OP_MUL_MAT_ID here:
//
//   reg     "MI355X"                     (cf. ggml_backend_cuda_reg, ggml-cuda.cu:3756-3819)
//   device  "MI355X<i>", one per gfx950  (cf. ggml-cuda.cu:3580-3755)
//   buft    device memory, 128-B aligned (cf. ggml-cuda.cu:700-760)
//   backend one HIP stream per instance  (cf. ggml_backend_cuda_i, ggml-cuda.cu:2990-3010)
//
// Design notes (MI355X-first, not a port):
//   * weights stay in the ggml block layout in HBM (no repack), so get/set_tensor are plain
//     copies and bit-exactness of round trips is trivial;
//   * the kernels never read past a row's last block, so no 512-element padding is added to
//     quantized allocations (the reference pads because its MMQ over-reads, ggml-cuda.cu:711-724);
//   * cross-device copies (the scheduler's pipeline hand-off, ggml-backend.cpp:1361-1393) are
//     hipMemcpyPeerAsync on the source stream + event wait on the destination stream — direct
//     xGMI DMA between the two GPUs with no host round trip.
//   * libggml-base symbols (buffer_init, graph accessors, nbytes) are resolved at load time with
//     dlsym(RTLD_DEFAULT): the library has no link-time dependency on ggml.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <array>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../../include/ggml-mi355x.h"
#include "dispatch.h"
#include "ggml_abi.h"
#include "settings.h"

using namespace mi355x;

namespace {

// ------------------------------------------------------------------------------------------
// libggml-base entry points (resolved lazily from the host process)
// ------------------------------------------------------------------------------------------
struct GgmlBase {
    ggml_backend_buffer_t (*buffer_init)(ggml_backend_buffer_type_t, struct ggml_backend_buffer_i, void *, size_t) = nullptr;
    int (*graph_n_nodes)(struct ggml_cgraph *) = nullptr;
    struct ggml_tensor *(*graph_node)(struct ggml_cgraph *, int) = nullptr;
    size_t (*nbytes)(const struct ggml_tensor *) = nullptr;
    ggml_backend_buffer_t (*cpu_buffer_from_ptr)(void *, size_t) = nullptr;
    ggml_backend_buffer_type_t (*cpu_buffer_type)(void) = nullptr;
    bool ok = false;
};

const GgmlBase &ggml_base() {
    static GgmlBase b = [] {
        GgmlBase g;
        g.buffer_init = reinterpret_cast<decltype(g.buffer_init)>(dlsym(RTLD_DEFAULT, "ggml_backend_buffer_init"));
        g.graph_n_nodes = reinterpret_cast<decltype(g.graph_n_nodes)>(dlsym(RTLD_DEFAULT, "ggml_graph_n_nodes"));
        g.graph_node = reinterpret_cast<decltype(g.graph_node)>(dlsym(RTLD_DEFAULT, "ggml_graph_node"));
        g.nbytes = reinterpret_cast<decltype(g.nbytes)>(dlsym(RTLD_DEFAULT, "ggml_nbytes"));
        g.cpu_buffer_from_ptr = reinterpret_cast<decltype(g.cpu_buffer_from_ptr)>(dlsym(RTLD_DEFAULT, "ggml_backend_cpu_buffer_from_ptr"));
        g.cpu_buffer_type = reinterpret_cast<decltype(g.cpu_buffer_type)>(dlsym(RTLD_DEFAULT, "ggml_backend_cpu_buffer_type"));
        g.ok = g.buffer_init && g.graph_n_nodes && g.graph_node && g.nbytes;
        return g;
    }();
    return b;
}

bool debug_on() {
    return settings().debug;
}

void logf(const char *fmt, ...) {
    if (!debug_on()) return;
    va_list ap;
    va_start(ap, fmt);
    fprintf(stderr, "[ggml-mi355x] ");
    vfprintf(stderr, fmt, ap);
    va_end(ap);
}

[[noreturn]] void fatal(const char *what, hipError_t e) {
    fprintf(stderr, "[ggml-mi355x] fatal: %s: %s\n", what, hipGetErrorString(e));
    abort();   // same policy as the reference's CUDA_CHECK (ggml-cuda.cu:94-98)
}

#define HIP_OK(call)                                 \
    do {                                             \
        const hipError_t e_ = (call);                \
        if (e_ != hipSuccess) fatal(#call, e_);      \
    } while (0)

// ------------------------------------------------------------------------------------------
// contexts
// ------------------------------------------------------------------------------------------
struct DeviceCtx {
    int device = 0;
    std::vector<int> peers;          // devices this one reaches by peer access (enabled at init)
    std::string name, desc;
    struct ggml_backend_buffer_type buft {};
    std::string buft_name;
    // repacked-weight buffer type (an "extra" buffer type, ggml_backend_dev_get_extra_bufts)
    struct ggml_backend_buffer_type rp_buft {};
    std::string rp_buft_name;
    ggml_backend_buffer_type_t extra_bufts[2] = {nullptr, nullptr};
};

struct BufferCtx {
    int device;
    void *base;
    // repacked-weight buffers: tensors written in part since their last repack (their copy is
    // stale until a write reaches the tensor's end; MUL_MAT reads src0 in place meanwhile)
    std::mutex rp_mu;
    std::set<const struct ggml_tensor *> rp_partial;
};

// per-shard state of one backend for split (row-sharded) mat-muls
struct ShardLane {
    int device = -1;
    hipStream_t stream = nullptr;     // on `device`
    hipEvent_t done = nullptr;        // recorded on `stream` after the shard's result landed in dst
    Scratch src1, dst, mm;            // src1 copy, the shard's [rows x cols] result, mat-mat scratch; on `device`
};

// graph fusion plan of one graph_compute (be_graph_compute): nodes skipped because a later fused
// launch computes them, and the fused attention launches by node index
// a whole GPT-2 decode layer (main-sched.cpp:600-812, one token) run as the engine's two launches
// (gpt2_block.hip); see plan_layers
struct LayerRun {
    int last = 0;                              // graph index of the layer's output node
    int type = 0, E = 0, n_head = 0, n_past = 0;
    const float *x = nullptr;                  // layer input (its first NORM's source)
    float *out = nullptr;                      // layer output (the last ADD)
    const float *ln1_g = nullptr, *ln1_b = nullptr, *ln2_g = nullptr, *ln2_b = nullptr;
    float eps1 = 0.f, eps2 = 0.f, scale = 0.f;
    const uint8_t *w_qkv = nullptr, *w_o = nullptr, *w_fc = nullptr, *w_mp = nullptr;
    int64_t nb_qkv = 0, nb_o = 0, nb_fc = 0, nb_mp = 0;
    const float *b_qkv = nullptr, *b_o = nullptr, *b_fc = nullptr, *b_mp = nullptr;
    float *kc = nullptr, *vc = nullptr;        // this layer's key / value rows (row p at p * E)
    int64_t cap = 0;                           // rows from kc / vc to the end of their cache buffers
    const struct ggml_tensor *out_t = nullptr;
    bool chain_in = false, chain_out = false;  // residual from / to the neighbouring fused layer
    const float *b_in = nullptr;               // chain_in: the previous layer's MLP-projection bias
};
struct FusePlan {
    std::vector<int8_t> skip;
    std::map<int, AttnView> attn;
    std::map<int, LayerRun> layers;   // by the graph index of the layer's first node
    // every fused layer at one position (a decode step): the layer launches read it from the
    // backend's device word (lf_pos, set before each run) instead of a kernel argument, so the
    // launch sequence, and a hipGraph of it, is the same for every token
    bool pos_word = false;
    int n_past = 0;
};

// hipGraph of the last graph_compute (cf. the reference's CUDA graphs, ggml-cuda.cu:2757-2998):
// the node properties it was captured from, and how many calls in a row needed a new capture
// (the sources' types and layouts are part of it: weights are leafs, not nodes, and the kernel a
// node launches depends on its weight's type and strides)
struct NodeProps {
    const void *node, *data;
    int32_t op, flags, type;
    int64_t ne[4];
    size_t nb[4];
    int32_t op_params[16];
    const void *src[GGMLABI_MAX_SRC], *src_data[GGMLABI_MAX_SRC];
    int32_t src_type[GGMLABI_MAX_SRC];
    int64_t src_ne[GGMLABI_MAX_SRC][4];
    size_t src_nb[GGMLABI_MAX_SRC][4];
};
// scratch_gen: the backend scratch's generation when `exec` was captured; a later eager run that
// grew (reallocated) the scratch invalidates the executable, whose mat-mat launches hold the old
// buffer's address
struct GraphCache {
    hipGraphExec_t exec = nullptr;
    std::vector<NodeProps> props;
    uint64_t scratch_gen = 0;
    uint64_t lr_gen = 0;              // fused-layer weight copies' generation at capture (g_lr_gen)
    int updates = 0;
    bool disabled = false;
};

struct BackendCtx {
    int device;
    hipStream_t stream = nullptr;
    std::string name;
    Scratch scratch;
    hipEvent_t src1_ready = nullptr;  // recorded on `stream` before shards start (split mat-mul)
    // recorded on `stream` after a scheduler hand-off copy (be_cpy_async); the destination
    // backend's stream waits on it. One event serves every copy: hipStreamWaitEvent waits for the
    // record that precedes the call, so re-recording it for the next copy is safe
    hipEvent_t copy_done = nullptr;
    std::vector<std::unique_ptr<ShardLane>> shards;
    FusePlan plan;                    // reused across graph_compute calls (no per-call allocation)
    GraphCache hg;
    // fused GPT-2 layers (plan_layers): partial slabs, the materialized residuals and the
    // position, allocated with the backend (a graph_compute may run inside a stream capture)
    float *lf_attn = nullptr, *lf_mlp = nullptr, *lf_x = nullptr, *lf_y = nullptr;
    int32_t *lf_pos = nullptr;
    void *lf_mem = nullptr;
    hipStream_t aux = nullptr;        // weight copies made for fused layers (not captured)
    hipEvent_t aux_ready = nullptr;   // recorded on `stream` before aux starts a copy
};

const char *BUFT_TAG = "MI355X";

DeviceCtx *dev_ctx(ggml_backend_dev_t d) { return static_cast<DeviceCtx *>(d->context); }

bool is_our_buft(ggml_backend_buffer_type_t buft);
void lr_invalidate(int device, const void *p, size_t n);   // fused-layer weight copies (plan_layers)

bool is_view_op(int op) {
    return op == GGMLABI_OP_NONE || op == GGMLABI_OP_RESHAPE || op == GGMLABI_OP_VIEW || op == GGMLABI_OP_PERMUTE ||
           op == GGMLABI_OP_TRANSPOSE;
}

// ggml node -> the graph_ops.hip description (ops around the matmuls);
// false for an op that is not one of them
bool graph_op_of(const struct ggml_tensor *node, GraphOp &g);

bool is_empty(const struct ggml_tensor *t) {
    for (int i = 0; i < 4; ++i)
        if (t->ne[i] == 0) return true;
    return false;
}

TensorView tv(const struct ggml_tensor *t) {
    TensorView v;
    v.type = t->type;
    v.data = t->data;
    for (int i = 0; i < 4; ++i) {
        v.ne[i] = t->ne[i];
        v.nb[i] = t->nb[i];
    }
    return v;
}

bool is_copy_op(int op) { return op == GGMLABI_OP_CPY || op == GGMLABI_OP_CONT || op == GGMLABI_OP_DUP; }

// a copy into or out of a quantized tensor (mi355x::cpy: quantize, dequantize, block copy)
bool is_quant_copy(const struct ggml_tensor *t) {
    return is_copy_op(t->op) && (is_hot_quant(t->type) || is_hot_quant(t->src[0]->type));
}

bool graph_op_of(const struct ggml_tensor *node, GraphOp &g) {
    g = GraphOp{};
    switch (node->op) {
        case GGMLABI_OP_ADD: g.op = GOP_ADD; break;
        case GGMLABI_OP_SUB: g.op = GOP_SUB; break;
        case GGMLABI_OP_MUL: g.op = GOP_MUL; break;
        case GGMLABI_OP_DIV: g.op = GOP_DIV; break;
        case GGMLABI_OP_NORM: g.op = GOP_NORM; break;
        case GGMLABI_OP_SCALE: g.op = GOP_SCALE; break;
        case GGMLABI_OP_DIAG_MASK_INF: g.op = GOP_DIAG_MASK_INF; break;
        case GGMLABI_OP_DIAG_MASK_ZERO: g.op = GOP_DIAG_MASK_ZERO; break;
        case GGMLABI_OP_SOFT_MAX: g.op = GOP_SOFT_MAX; break;
        case GGMLABI_OP_CPY:
        case GGMLABI_OP_CONT:
        case GGMLABI_OP_DUP: g.op = GOP_CPY; break;
        case GGMLABI_OP_MUL_MAT: g.op = GOP_MUL_MAT; break;
        case GGMLABI_OP_UNARY:
            if (node->op_params[0] != GGMLABI_UNARY_OP_GELU) return false;
            g.op = GOP_GELU;
            break;
        default: return false;
    }
    for (int i = 0; i < 4; ++i) g.params[i] = node->op_params[i];
    g.dst = tv(node);
    // CPY's second source is its destination (node is a view of it); it is not an input
    const int nsrc = node->op == GGMLABI_OP_CPY ? 1 : 3;
    for (int i = 0; i < nsrc; ++i) {
        g.has_src[i] = node->src[i] != nullptr;
        if (g.has_src[i]) g.src[i] = tv(node->src[i]);
    }
    return true;
}

// ------------------------------------------------------------------------------------------
// buffer
// ------------------------------------------------------------------------------------------
void buf_free(ggml_backend_buffer_t b) {
    auto *c = static_cast<BufferCtx *>(b->context);
    lr_invalidate(c->device, c->base, b->size);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipFree(c->base));
    delete c;
}

void *buf_base(ggml_backend_buffer_t b) { return static_cast<BufferCtx *>(b->context)->base; }

enum ggml_status buf_init_tensor(ggml_backend_buffer_t, struct ggml_tensor *) { return GGML_STATUS_SUCCESS; }

void buf_memset(ggml_backend_buffer_t b, struct ggml_tensor *t, uint8_t v, size_t off, size_t n) {
    auto *c = static_cast<BufferCtx *>(b->context);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipMemsetAsync(static_cast<uint8_t *>(t->data) + off, v, n, nullptr));
    HIP_OK(hipStreamSynchronize(nullptr));
    lr_invalidate(c->device, static_cast<uint8_t *>(t->data) + off, n);
}

// small host <-> device copies (a decode step's token id and position, and its logits row read
// back: three per token under the reference scheduler) go through a pinned bounce buffer on a stream of their own: a DMA from
// pinned memory, instead of the staged copy a pageable source takes. Same contract as the
// reference's set_tensor (cudaMemcpyAsync on its own stream + synchronize, ggml-cuda.cu:614-620):
// the bytes are on the device when the call returns; not ordered with the backend streams.
struct Bounce {
    std::mutex mu;
    void *host = nullptr;
    hipStream_t st = nullptr;
};
constexpr size_t BOUNCE_BYTES = 256 * 1024;   // (a GPT-2 logits row is 201 KB)
Bounce &bounce_of(int device) {
    static Bounce b[64];
    return b[device & 63];
}

void buf_set(ggml_backend_buffer_t b, struct ggml_tensor *t, const void *data, size_t off, size_t n) {
    auto *c = static_cast<BufferCtx *>(b->context);
    HIP_OK(hipSetDevice(c->device));
    uint8_t *dst = static_cast<uint8_t *>(t->data) + off;
    if (n <= BOUNCE_BYTES) {
        Bounce &bb = bounce_of(c->device);
        std::lock_guard<std::mutex> lk(bb.mu);
        if (bb.host == nullptr) {
            HIP_OK(hipHostMalloc(&bb.host, BOUNCE_BYTES, hipHostMallocDefault));
            HIP_OK(hipStreamCreateWithFlags(&bb.st, hipStreamNonBlocking));
        }
        std::memcpy(bb.host, data, n);
        HIP_OK(hipMemcpyAsync(dst, bb.host, n, hipMemcpyHostToDevice, bb.st));
        HIP_OK(hipStreamSynchronize(bb.st));
    } else {
        HIP_OK(hipMemcpyAsync(dst, data, n, hipMemcpyHostToDevice, nullptr));
        HIP_OK(hipStreamSynchronize(nullptr));
    }
    lr_invalidate(c->device, static_cast<uint8_t *>(t->data) + off, n);
}

void buf_get(ggml_backend_buffer_t b, const struct ggml_tensor *t, void *data, size_t off, size_t n) {
    auto *c = static_cast<BufferCtx *>(b->context);
    HIP_OK(hipSetDevice(c->device));
    const uint8_t *src = static_cast<const uint8_t *>(t->data) + off;
    if (n <= BOUNCE_BYTES) {
        Bounce &bb = bounce_of(c->device);
        std::lock_guard<std::mutex> lk(bb.mu);
        if (bb.host == nullptr) {
            HIP_OK(hipHostMalloc(&bb.host, BOUNCE_BYTES, hipHostMallocDefault));
            HIP_OK(hipStreamCreateWithFlags(&bb.st, hipStreamNonBlocking));
        }
        HIP_OK(hipMemcpyAsync(bb.host, src, n, hipMemcpyDeviceToHost, bb.st));
        HIP_OK(hipStreamSynchronize(bb.st));
        std::memcpy(data, bb.host, n);
        return;
    }
    HIP_OK(hipMemcpyAsync(data, src, n, hipMemcpyDeviceToHost, nullptr));
    HIP_OK(hipStreamSynchronize(nullptr));
}

bool buf_cpy(ggml_backend_buffer_t b, const struct ggml_tensor *src, struct ggml_tensor *dst) {
    if (!src->buffer || !is_our_buft(src->buffer->buft)) return false;
    auto *sc = static_cast<BufferCtx *>(src->buffer->context);
    auto *dc = static_cast<BufferCtx *>(b->context);
    const size_t n = ggml_base().nbytes(src);
    if (sc->device == dc->device) {
        HIP_OK(hipSetDevice(dc->device));
        HIP_OK(hipMemcpyAsync(dst->data, src->data, n, hipMemcpyDeviceToDevice, nullptr));
    } else {
        HIP_OK(hipSetDevice(sc->device));
        HIP_OK(hipMemcpyPeerAsync(dst->data, dc->device, src->data, sc->device, n, nullptr));
    }
    HIP_OK(hipStreamSynchronize(nullptr));
    lr_invalidate(dc->device, dst->data, n);
    return true;
}

void buf_clear(ggml_backend_buffer_t b, uint8_t v) {
    auto *c = static_cast<BufferCtx *>(b->context);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipMemsetAsync(c->base, v, b->size, nullptr));
    HIP_OK(hipStreamSynchronize(nullptr));
    lr_invalidate(c->device, c->base, b->size);
}

const struct ggml_backend_buffer_i BUFFER_IFACE = {
    buf_free, buf_base, buf_init_tensor, buf_memset, buf_set, buf_get, buf_cpy, buf_clear, nullptr,
};

// ------------------------------------------------------------------------------------------
// repacked-weight buffer ("MI355X<i>_Repack", offered through ggml_backend_dev_get_extra_bufts as
// the reference CPU backend offers its repack buffer, src/ggml-cpu/repack.cpp:1967 and
// ggml-cpu.cpp:619): a quantized tensor keeps its ggml bytes at `data` (so GET_ROWS, CPY, the
// mat-vec and get_tensor read it as usual) and gets, right behind them, the int8 tile's repacked
// copy (mmq8.hip: int8 codes in MFMA-fragment order + f32 block scales), pointed to by
// tensor->extra and remade by every write to the tensor. MUL_MAT with more than 8 tokens on such
// a weight runs the tile on the copy: no per-call weight decode.
// ------------------------------------------------------------------------------------------
size_t rp_extra_bytes(const struct ggml_tensor *t) {
    if (t->view_src != nullptr) return 0;
    TensorView v = tv(t);
    v.data = nullptr;
    const size_t n = repack_size(v);
    return n ? n + 256 : 0;   // + alignment slack of the copy
}

uint8_t *rp_extra_ptr(const struct ggml_tensor *t) {
    const uintptr_t end = reinterpret_cast<uintptr_t>(t->data) + ggml_base().nbytes(t);
    return reinterpret_cast<uint8_t *>((end + 255) & ~(uintptr_t)255);
}

std::atomic<uint64_t> g_lr_gen{0};   // (below: fused-layer copies; also bumped when a repacked copy goes stale / fresh)

// after a write of [off, off + n) into t: remake t's repacked copy on `st` once the write reaches
// the tensor's end (a whole-tensor write, or the last chunk of an upload in order, as the
// reference's CPU repack buffer takes only whole-tensor writes, repack.cpp:1879-1889); until then
// the copy is marked stale and MUL_MAT reads the ggml bytes in place (repacked_of). A change of
// staleness bumps g_lr_gen, so a hipGraph captured with the other choice is not replayed.
void rp_written(BufferCtx *c, struct ggml_tensor *t, size_t off, size_t n, hipStream_t st) {
    if (t->extra == nullptr) return;
    const size_t nbytes = ggml_base().nbytes(t);
    const bool complete = off + n >= nbytes;
    {
        std::lock_guard<std::mutex> lk(c->rp_mu);
        const bool was = c->rp_partial.count(t) != 0;
        if (complete) c->rp_partial.erase(t);
        else c->rp_partial.insert(t);
        if (was != !complete) g_lr_gen.fetch_add(1);
    }
    if (!complete) return;
    HIP_OK(hipSetDevice(c->device));
    if (repack(tv(t), t->extra, rp_extra_bytes(t) - 256, st) != GGML_MI355X_OK) fatal("repack", hipErrorInvalidValue);
}

void rp_refresh(BufferCtx *c, struct ggml_tensor *t, size_t off, size_t n) {
    if (t->extra == nullptr) return;
    rp_written(c, t, off, n, nullptr);
    HIP_OK(hipStreamSynchronize(nullptr));
}

enum ggml_status rp_init_tensor(ggml_backend_buffer_t, struct ggml_tensor *t) {
    t->extra = rp_extra_bytes(t) ? rp_extra_ptr(t) : nullptr;
    return GGML_STATUS_SUCCESS;
}

void rp_memset(ggml_backend_buffer_t b, struct ggml_tensor *t, uint8_t v, size_t off, size_t n) {
    buf_memset(b, t, v, off, n);
    rp_refresh(static_cast<BufferCtx *>(b->context), t, off, n);
}

void rp_set(ggml_backend_buffer_t b, struct ggml_tensor *t, const void *data, size_t off, size_t n) {
    buf_set(b, t, data, off, n);
    rp_refresh(static_cast<BufferCtx *>(b->context), t, off, n);
}

bool rp_cpy(ggml_backend_buffer_t b, const struct ggml_tensor *src, struct ggml_tensor *dst) {
    if (!buf_cpy(b, src, dst)) return false;
    rp_refresh(static_cast<BufferCtx *>(b->context), dst, 0, ggml_base().nbytes(dst));
    return true;
}

const struct ggml_backend_buffer_i RP_BUFFER_IFACE = {
    buf_free, buf_base, rp_init_tensor, rp_memset, rp_set, buf_get, rp_cpy, buf_clear, nullptr,
};

// ------------------------------------------------------------------------------------------
// buffer type
// ------------------------------------------------------------------------------------------
const char *buft_name(ggml_backend_buffer_type_t bt) { return static_cast<DeviceCtx *>(bt->context)->buft_name.c_str(); }

ggml_backend_buffer_t buft_alloc(ggml_backend_buffer_type_t bt, size_t size) {
    auto *d = static_cast<DeviceCtx *>(bt->context);
    if (!ggml_base().ok) {
        fprintf(stderr, "[ggml-mi355x] libggml-base symbols not found in the host process\n");
        return nullptr;
    }
    HIP_OK(hipSetDevice(d->device));
    void *p = nullptr;
    const size_t sz = size ? size : 1;
    if (hipMalloc(&p, sz) != hipSuccess) {
        (void)hipGetLastError();
        fprintf(stderr, "[ggml-mi355x] hipMalloc of %zu bytes on device %d failed\n", size, d->device);
        return nullptr;
    }
    logf("alloc %zu bytes on device %d -> %p\n", size, d->device, p);
    const bool rp = bt == &d->rp_buft;
    return ggml_base().buffer_init(bt, rp ? RP_BUFFER_IFACE : BUFFER_IFACE, new BufferCtx{d->device, p}, size);
}

size_t buft_align(ggml_backend_buffer_type_t) { return 128; }
size_t buft_max(ggml_backend_buffer_type_t) { return SIZE_MAX; }
size_t buft_alloc_size(ggml_backend_buffer_type_t, const struct ggml_tensor *t) { return ggml_base().nbytes(t); }
bool buft_is_host(ggml_backend_buffer_type_t) { return false; }

const struct ggml_backend_buffer_type_i BUFT_IFACE = {
    buft_name, buft_alloc, buft_align, buft_max, buft_alloc_size, buft_is_host,
};

const char *rp_buft_name(ggml_backend_buffer_type_t bt) { return static_cast<DeviceCtx *>(bt->context)->rp_buft_name.c_str(); }
size_t rp_buft_alloc_size(ggml_backend_buffer_type_t, const struct ggml_tensor *t) {
    return ggml_base().nbytes(t) + rp_extra_bytes(t);
}

const struct ggml_backend_buffer_type_i RP_BUFT_IFACE = {
    rp_buft_name, buft_alloc, buft_align, buft_max, rp_buft_alloc_size, buft_is_host,
};

bool is_rp_buft(ggml_backend_buffer_type_t buft) { return buft && buft->iface.get_name == rp_buft_name; }
// device memory of one of our devices (plain or repacked-weight buffer: both hold BufferCtx)
bool is_our_buft(ggml_backend_buffer_type_t buft) { return buft && (buft->iface.get_name == buft_name || is_rp_buft(buft)); }

// src0's repacked copy, when it lives in a repacked-weight buffer (else nullptr)
// (nullptr too while the copy is stale: the tensor was written in part since its last repack)
const void *repacked_of(const struct ggml_tensor *a) {
    if (!a->buffer || !is_rp_buft(a->buffer->buft) || a->view_src != nullptr || a->extra == nullptr) return nullptr;
    auto *c = static_cast<BufferCtx *>(a->buffer->context);
    std::lock_guard<std::mutex> lk(c->rp_mu);
    return c->rp_partial.count(a) ? nullptr : a->extra;
}

// ------------------------------------------------------------------------------------------
// row-split ("tensor parallel") buffer type: ggml_backend_split_buffer_type(main, tensor_split)
// (reference ggml-cuda.cu:763-1094). A weight matrix in such a buffer is cut by rows into one
// shard per device; MUL_MAT on it runs each shard's rows on that shard's device against a copy
// of src1 and writes the shard's rows of dst on the main device (be_split_mul_mat). Same
// partition rule as the reference's get_row_split (cumulative fractions, rows rounded down to
// a multiple of SPLIT_ROW_ROUND except at the end), no padding (our kernels never over-read).
//
// GGML_MI355X_SPLIT_SHARDS=k sets the number of shards (default: one per device). With more
// shards than devices, shard i lives on device i % n_devices: on a one-GPU box that runs the
// whole multi-shard path (separate allocations, stream / event hand-offs, src1 copies, strided
// gathers of dst) against one GPU, which is how the 1-GPU test box exercises it.
// ------------------------------------------------------------------------------------------
constexpr int SPLIT_MAX = 16;            // the reference's GGML_CUDA_MAX_DEVICES
constexpr int64_t SPLIT_ROW_ROUND = 16;  // one 16-lane mat-vec row group

int n_devices();
int device_of(int idx);
ggml_backend_dev_t dev_handle(int idx);

int n_shards() {
    const int forced = settings().split_shards;
    const int n = forced > 0 ? forced : n_devices();
    return std::max(1, std::min(n, SPLIT_MAX));
}
int shard_device(int i) { return device_of(i % std::max(1, n_devices())); }

struct SplitBuftCtx {
    int main_device;                   // our device index
    std::array<float, SPLIT_MAX> split;   // cumulative start fraction of each shard
    std::string name;
};

struct SplitExtra {
    std::array<void *, SPLIT_MAX> data{};
    std::array<int64_t, SPLIT_MAX> lo{}, hi{};
    int device[SPLIT_MAX] = {};
};

struct SplitBufCtx {
    std::vector<SplitExtra *> extras;
};

// rows [lo, hi) of shard id (get_row_split, ggml-cuda.cu:778-791)
void split_rows(int64_t nrows, const SplitBuftCtx &bc, int id, int64_t &lo, int64_t &hi) {
    const int n = n_shards();
    lo = id == 0 ? 0 : (int64_t)(nrows * bc.split[id]);
    lo -= lo % SPLIT_ROW_ROUND;
    if (id == n - 1) {
        hi = nrows;
    } else {
        hi = (int64_t)(nrows * bc.split[id + 1]);
        hi -= hi % SPLIT_ROW_ROUND;
    }
    hi = std::max(hi, lo);
}

int64_t nrows_of(const struct ggml_tensor *t) { return t->ne[1] * t->ne[2] * t->ne[3]; }

bool is_contiguous_rows(const struct ggml_tensor *t) {
    return (int64_t)t->nb[2] == (int64_t)t->nb[1] * t->ne[1] && (int64_t)t->nb[3] == (int64_t)t->nb[2] * t->ne[2];
}

const char *split_buft_name(ggml_backend_buffer_type_t bt) { return static_cast<SplitBuftCtx *>(bt->context)->name.c_str(); }
bool is_split_buft(ggml_backend_buffer_type_t bt) { return bt && bt->iface.get_name == split_buft_name; }

void split_buf_free(ggml_backend_buffer_t b) {
    auto *c = static_cast<SplitBufCtx *>(b->context);
    for (SplitExtra *e : c->extras) {
        for (int i = 0; i < SPLIT_MAX; ++i) {
            if (e->data[i]) {
                HIP_OK(hipSetDevice(e->device[i]));
                HIP_OK(hipFree(e->data[i]));
            }
        }
        delete e;
    }
    delete c;
}

void *split_buf_base(ggml_backend_buffer_t) { return reinterpret_cast<void *>(0x1000); }   // never dereferenced

enum ggml_status split_buf_init_tensor(ggml_backend_buffer_t b, struct ggml_tensor *t) {
    if (t->view_src != nullptr || !is_contiguous_rows(t)) {
        fprintf(stderr, "[ggml-mi355x] split buffers hold whole contiguous tensors only (%s)\n", t->name);
        return GGML_STATUS_FAILED;
    }
    // only the quantized MUL_MAT weights this backend runs row-split; an F16 / F32 matrix placed
    // here could be run by no backend (the CPU one cannot read split shards), so refuse it now
    // rather than fail late in the scheduler (the reference's split buffer also serves F16/F32)
    if (!is_hot_quant(t->type)) {
        fprintf(stderr, "[ggml-mi355x] split buffers hold Q4_0/Q8_0/Q4_K/Q5_K/Q6_K weights only (%s has type %d)\n", t->name,
                (int)t->type);
        return GGML_STATUS_FAILED;
    }
    const auto &bc = *static_cast<SplitBuftCtx *>(b->buft->context);
    auto *e = new SplitExtra();
    static_cast<SplitBufCtx *>(b->context)->extras.push_back(e);
    const int64_t nrows = nrows_of(t);
    for (int i = 0; i < n_shards(); ++i) {
        split_rows(nrows, bc, i, e->lo[i], e->hi[i]);
        e->device[i] = shard_device(i);
        if (e->hi[i] <= e->lo[i]) continue;
        HIP_OK(hipSetDevice(e->device[i]));
        if (hipMalloc(&e->data[i], (size_t)(e->hi[i] - e->lo[i]) * t->nb[1]) != hipSuccess) {
            (void)hipGetLastError();
            e->data[i] = nullptr;
            return GGML_STATUS_ALLOC_FAILED;
        }
    }
    t->extra = e;
    return GGML_STATUS_SUCCESS;
}

// whole-tensor set / get only, like the reference (ggml-cuda.cu:888-964)
void split_buf_set(ggml_backend_buffer_t, struct ggml_tensor *t, const void *data, size_t off, size_t n) {
    auto *e = static_cast<SplitExtra *>(t->extra);
    if (off != 0 || n != ggml_base().nbytes(t)) {
        fprintf(stderr, "[ggml-mi355x] split tensors must be set in their entirety\n");
        abort();
    }
    for (int i = 0; i < n_shards(); ++i) {
        if (!e->data[i]) continue;
        HIP_OK(hipSetDevice(e->device[i]));
        HIP_OK(hipMemcpy(e->data[i], static_cast<const uint8_t *>(data) + e->lo[i] * t->nb[1], (size_t)(e->hi[i] - e->lo[i]) * t->nb[1],
                         hipMemcpyHostToDevice));
    }
}

void split_buf_get(ggml_backend_buffer_t, const struct ggml_tensor *t, void *data, size_t off, size_t n) {
    auto *e = static_cast<SplitExtra *>(t->extra);
    if (off != 0 || n != ggml_base().nbytes(t)) {
        fprintf(stderr, "[ggml-mi355x] split tensors must be read in their entirety\n");
        abort();
    }
    for (int i = 0; i < n_shards(); ++i) {
        if (!e->data[i]) continue;
        HIP_OK(hipSetDevice(e->device[i]));
        HIP_OK(hipMemcpy(static_cast<uint8_t *>(data) + e->lo[i] * t->nb[1], e->data[i], (size_t)(e->hi[i] - e->lo[i]) * t->nb[1],
                         hipMemcpyDeviceToHost));
    }
}

void split_buf_clear(ggml_backend_buffer_t, uint8_t) {}

const struct ggml_backend_buffer_i SPLIT_BUFFER_IFACE = {
    split_buf_free, split_buf_base, split_buf_init_tensor, nullptr, split_buf_set, split_buf_get, nullptr, split_buf_clear, nullptr,
};

ggml_backend_buffer_t split_buft_alloc(ggml_backend_buffer_type_t bt, size_t size) {
    // the shards are allocated per tensor in init_tensor; `size` is the ggml-alloc bound
    return ggml_base().buffer_init(bt, SPLIT_BUFFER_IFACE, new SplitBufCtx(), size);
}

size_t split_buft_align(ggml_backend_buffer_type_t) { return 128; }

size_t split_buft_alloc_size(ggml_backend_buffer_type_t bt, const struct ggml_tensor *t) {
    const auto &bc = *static_cast<SplitBuftCtx *>(bt->context);
    size_t total = 0;
    for (int i = 0; i < n_shards(); ++i) {
        int64_t lo, hi;
        split_rows(nrows_of(t), bc, i, lo, hi);
        total += (size_t)(hi - lo) * t->nb[1];
    }
    return total;
}

bool split_buft_is_host(ggml_backend_buffer_type_t) { return false; }

const struct ggml_backend_buffer_type_i SPLIT_BUFT_IFACE = {
    split_buft_name, split_buft_alloc, split_buft_align, nullptr, split_buft_alloc_size, split_buft_is_host,
};

// the proc-address entry point (reference ggml_backend_cuda_split_buffer_type, ggml-cuda.cu:1054)
extern "C" ggml_backend_buffer_type_t mi355x_split_buffer_type(int main_device, const float *tensor_split) {
    static std::mutex mu;
    static std::map<std::pair<int, std::array<float, SPLIT_MAX>>, std::unique_ptr<ggml_backend_buffer_type>> types;
    std::lock_guard<std::mutex> lock(mu);
    if (main_device < 0 || main_device >= n_devices()) return nullptr;
    const int n = n_shards();
    std::array<float, SPLIT_MAX> cum{};
    bool all_zero = tensor_split == nullptr;
    if (!all_zero) {
        all_zero = true;
        for (int i = 0; i < n; ++i) all_zero = all_zero && tensor_split[i] == 0.f;
    }
    float sum = 0.f;
    for (int i = 0; i < n; ++i) {
        cum[i] = sum;
        sum += all_zero ? 1.f : tensor_split[i];   // default: equal shares (identical devices)
    }
    for (int i = 0; i < n; ++i) cum[i] /= sum;
    auto &slot = types[{main_device, cum}];
    if (!slot) {
        auto *ctx = new SplitBuftCtx{main_device, cum, "MI355X" + std::to_string(main_device) + "_Split"};
        slot.reset(new ggml_backend_buffer_type{SPLIT_BUFT_IFACE, dev_handle(main_device), ctx});
    }
    return slot.get();
}

// ------------------------------------------------------------------------------------------
// pinned host buffer type (reference ggml_backend_cuda_host_buffer_type, ggml-cuda.cu:1096-1160):
// page-locked memory behind ggml's own CPU buffer interface, so the CPU backend computes on
// it and set/get_tensor_async become real DMA. Falls back to a plain CPU buffer when pinning
// fails (GGML_MI355X_NO_PINNED disables it, like GGML_CUDA_NO_PINNED).
// ------------------------------------------------------------------------------------------
const char *host_buft_name(ggml_backend_buffer_type_t) { return "MI355X_Host"; }

void host_buf_free(ggml_backend_buffer_t b) { HIP_OK(hipHostFree(b->context)); }

ggml_backend_buffer_t host_buft_alloc(ggml_backend_buffer_type_t bt, size_t size) {
    const GgmlBase &gb = ggml_base();
    if (!gb.cpu_buffer_from_ptr || !gb.cpu_buffer_type) return nullptr;
    void *p = nullptr;
    if (!settings().no_pinned && hipHostMalloc(&p, size ? size : 1, hipHostMallocPortable) != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
    }
    if (!p) {
        ggml_backend_buffer_type_t cpu = gb.cpu_buffer_type();
        return cpu->iface.alloc_buffer(cpu, size);
    }
    ggml_backend_buffer_t b = gb.cpu_buffer_from_ptr(p, size);
    b->buft = bt;
    b->context = p;                       // the CPU buffer keeps its base pointer in context
    b->iface.free_buffer = host_buf_free;
    return b;
}

size_t host_buft_align(ggml_backend_buffer_type_t) { return 64; }   // TENSOR_ALIGNMENT of the CPU buffer
size_t host_buft_alloc_size(ggml_backend_buffer_type_t, const struct ggml_tensor *t) { return ggml_base().nbytes(t); }
bool host_buft_is_host(ggml_backend_buffer_type_t) { return true; }

ggml_backend_buffer_type_t host_buft() {
    static struct ggml_backend_buffer_type bt = {
        {host_buft_name, host_buft_alloc, host_buft_align, nullptr, host_buft_alloc_size, host_buft_is_host},
        nullptr,
        nullptr,
    };
    if (!bt.device) bt.device = dev_handle(0);
    return &bt;
}

// ggml_backend_register_host_buffer / unregister (reference ggml-cuda.cu:3733-3740): pin
// caller-owned memory for fast transfers
extern "C" bool mi355x_register_host_buffer(void *buffer, size_t size) {
    if (settings().no_pinned) return false;
    const hipError_t e = hipHostRegister(buffer, size, hipHostRegisterPortable | hipHostRegisterReadOnly);
    if (e != hipSuccess) (void)hipGetLastError();
    return e == hipSuccess;
}

extern "C" void mi355x_unregister_host_buffer(void *buffer) {
    if (hipHostUnregister(buffer) != hipSuccess) (void)hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// backend (stream)
// ------------------------------------------------------------------------------------------
ggml_guid BACKEND_GUID = {0x6d, 0x69, 0x33, 0x35, 0x35, 0x78, 0x2d, 0x67, 0x66, 0x78, 0x39, 0x35, 0x30, 0x2d, 0x71, 0x6d};

BackendCtx *be_ctx(ggml_backend_t b) { return static_cast<BackendCtx *>(b->context); }

const char *be_name(ggml_backend_t b) { return be_ctx(b)->name.c_str(); }

void be_free(ggml_backend_t b) {
    BackendCtx *c = be_ctx(b);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipStreamSynchronize(c->stream));
    if (c->hg.exec) HIP_OK(hipGraphExecDestroy(c->hg.exec));
    HIP_OK(hipStreamDestroy(c->stream));
    HIP_OK(hipStreamDestroy(c->aux));
    HIP_OK(hipEventDestroy(c->aux_ready));
    if (c->lf_mem) HIP_OK(hipFree(c->lf_mem));
    if (c->src1_ready) HIP_OK(hipEventDestroy(c->src1_ready));
    if (c->copy_done) HIP_OK(hipEventDestroy(c->copy_done));
    for (auto &L : c->shards) {
        if (!L || L->device < 0) continue;
        HIP_OK(hipSetDevice(L->device));
        HIP_OK(hipStreamSynchronize(L->stream));
        HIP_OK(hipStreamDestroy(L->stream));
        HIP_OK(hipEventDestroy(L->done));
        L->src1.release();   // on the shard's device
        L->dst.release();
        L->mm.release();
    }
    delete c;
    delete b;
}

// an asynchronous write into one of our buffers, queued on `st`: the same bookkeeping as the
// buffer's synchronous writes (buf_set / rp_set) — the fused-layer weight copies of the range
// are dropped, and a repacked-weight tensor's copy is remade on `st` behind the write
void written_async(struct ggml_tensor *t, size_t off, size_t n, hipStream_t st) {
    if (!t->buffer || !is_our_buft(t->buffer->buft)) return;
    auto *bc = static_cast<BufferCtx *>(t->buffer->context);
    if (is_rp_buft(t->buffer->buft)) rp_written(bc, t, off, n, st);
}

void be_set_async(ggml_backend_t b, struct ggml_tensor *t, const void *data, size_t off, size_t n) {
    BackendCtx *c = be_ctx(b);
    HIP_OK(hipSetDevice(c->device));
    lr_invalidate(c->device, static_cast<uint8_t *>(t->data) + off, n);
    HIP_OK(hipMemcpyAsync(static_cast<uint8_t *>(t->data) + off, data, n, hipMemcpyHostToDevice, c->stream));
    written_async(t, off, n, c->stream);
}

void be_get_async(ggml_backend_t b, const struct ggml_tensor *t, void *data, size_t off, size_t n) {
    BackendCtx *c = be_ctx(b);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipMemcpyAsync(data, static_cast<const uint8_t *>(t->data) + off, n, hipMemcpyDeviceToHost, c->stream));
}

bool is_our_backend(ggml_backend_t b);

// scheduler hand-off between two MI355X backends (pipeline split, ggml-backend.cpp:1383)
bool be_cpy_async(ggml_backend_t bsrc, ggml_backend_t bdst, const struct ggml_tensor *src, struct ggml_tensor *dst) {
    if (!is_our_backend(bsrc) || !is_our_backend(bdst)) return false;
    if (!src->buffer || !dst->buffer || !is_our_buft(src->buffer->buft) || !is_our_buft(dst->buffer->buft)) return false;
    BackendCtx *cs = be_ctx(bsrc), *cd = be_ctx(bdst);
    const size_t n = ggml_base().nbytes(src);
    lr_invalidate(cd->device, dst->data, n);
    HIP_OK(hipSetDevice(cs->device));
    if (cs->device == cd->device) {
        HIP_OK(hipMemcpyAsync(dst->data, src->data, n, hipMemcpyDeviceToDevice, cs->stream));
    } else {
        HIP_OK(hipMemcpyPeerAsync(dst->data, cd->device, src->data, cs->device, n, cs->stream));
    }
    if (cs != cd) {
        if (!cs->copy_done) HIP_OK(hipEventCreateWithFlags(&cs->copy_done, hipEventDisableTiming));
        HIP_OK(hipEventRecord(cs->copy_done, cs->stream));
        HIP_OK(hipSetDevice(cd->device));
        HIP_OK(hipStreamWaitEvent(cd->stream, cs->copy_done, 0));
    }
    written_async(dst, 0, n, cd->stream);   // (a repacked destination is remade on its own device)
    return true;
}

void be_sync(ggml_backend_t b) {
    BackendCtx *c = be_ctx(b);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipStreamSynchronize(c->stream));
    if (take_device_error(c->device)) {   // as the reference's GGML_ASSERT in get_rows (src/ggml-cpu/ops.cpp:5157)
        fprintf(stderr, "[ggml-mi355x] %s: GET_ROWS row index out of range\n", c->name.c_str());
        abort();
    }
}

// MUL_MAT whose src0 lives in a split buffer (reference ggml_cuda_op_mul_mat's split branch,
// ggml-cuda.cu:1441-1700, restructured): the shard on the main device computes its rows of
// dst in place on the backend stream; every other shard, on its own device and stream, waits
// for src1, copies it over xGMI (peer DMA), runs its rows into a local [rows x cols] block and
// writes that block into its rows of dst on the main device with one strided peer copy. The
// backend stream then waits for every shard. src1 / dst must be contiguous (checked by
// supports_op); src0 is 2-D.
int be_split_mul_mat(BackendCtx *c, struct ggml_tensor *node) {
    const struct ggml_tensor *a = node->src[0], *b = node->src[1];
    auto *e = static_cast<const SplitExtra *>(a->extra);
    const size_t row_b = a->nb[1];
    const int64_t cols = node->ne[1] * node->ne[2] * node->ne[3];   // dst rows of ne0 floats
    const size_t src1_bytes = ggml_base().nbytes(b);
    if (!c->src1_ready) HIP_OK(hipEventCreateWithFlags(&c->src1_ready, hipEventDisableTiming));
    HIP_OK(hipEventRecord(c->src1_ready, c->stream));
    int main_shard = -1;
    for (int i = 0; i < n_shards(); ++i)
        if (e->data[i] && e->device[i] == c->device) { main_shard = i; break; }
    int rc = GGML_MI355X_OK;
    for (int i = 0; i < n_shards() && rc == GGML_MI355X_OK; ++i) {
        if (!e->data[i]) continue;
        const int64_t rows = e->hi[i] - e->lo[i];
        TensorView wa = tv(a);
        wa.data = e->data[i];
        wa.ne[1] = rows;
        wa.nb[2] = wa.nb[3] = row_b * rows;
        if (i == main_shard) {
            TensorView d = tv(node);
            d.data = static_cast<uint8_t *>(node->data) + e->lo[i] * sizeof(float);
            d.ne[0] = rows;
            rc = mul_mat(wa, tv(b), d, c->stream, c->scratch);
            continue;
        }
        if ((int)c->shards.size() <= i) c->shards.resize(i + 1);
        if (!c->shards[i]) c->shards[i] = std::make_unique<ShardLane>();
        ShardLane &L = *c->shards[i];
        HIP_OK(hipSetDevice(e->device[i]));
        if (L.device != e->device[i]) {
            L.device = e->device[i];
            HIP_OK(hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking));
            HIP_OK(hipEventCreateWithFlags(&L.done, hipEventDisableTiming));
        }
        HIP_OK(hipStreamWaitEvent(L.stream, c->src1_ready, 0));
        void *x = L.src1.get(src1_bytes, L.stream);
        void *y = L.dst.get((size_t)rows * cols * sizeof(float), L.stream);
        if (!x || !y) { rc = GGML_MI355X_ENOMEM; break; }
        HIP_OK(hipMemcpyPeerAsync(x, e->device[i], b->data, c->device, src1_bytes, L.stream));
        TensorView xb = tv(b);
        xb.data = x;
        TensorView d = tv(node);
        d.data = y;
        d.ne[0] = rows;
        d.nb[1] = rows * sizeof(float);
        d.nb[2] = d.nb[1] * node->ne[1];
        d.nb[3] = d.nb[2] * node->ne[2];
        rc = mul_mat(wa, xb, d, L.stream, L.mm);
        if (rc != GGML_MI355X_OK) break;
        HIP_OK(hipMemcpy2DAsync(static_cast<uint8_t *>(node->data) + e->lo[i] * sizeof(float), node->nb[1], y, rows * sizeof(float),
                                rows * sizeof(float), cols, hipMemcpyDefault, L.stream));
        HIP_OK(hipEventRecord(L.done, L.stream));
        HIP_OK(hipSetDevice(c->device));
        HIP_OK(hipStreamWaitEvent(c->stream, L.done, 0));
    }
    HIP_OK(hipSetDevice(c->device));
    return rc;
}

// ------------------------------------------------------------------------------------------
// graph fusion. The reference fuses runs of nodes whose intermediates nobody else reads
// (ggml_can_fuse, src/ggml-impl.h:548-603; ggml_cuda_can_fuse, ggml-cuda.cu:2813-2870). The same
// rule decides here, on the whole graph's use counts, and a fused run is executed by ONE launch
// that writes only the run's last node:
//   [NORM, MUL, ADD,] MUL_MAT(hot quant, <= 8 columns) [, ADD bias [, GELU | ADD residual]]
//       -> the layer-norm-prologue / bias-GELU-residual-epilogue mat-vec (mmvq_fused.hip)
//   [SCALE,] [DIAG_MASK_INF,] SOFT_MAX  -> one soft_max launch applying its producers on load
// A plain MUL_MAT (nothing around it to fuse) keeps the generic dispatch. GGML_MI355X_FUSION=0
// turns fusion off.
// ------------------------------------------------------------------------------------------
bool fusion_on() {
    return settings().fusion;
}

// the graph's use count of t (ggml_node_has_n_uses, ggml-impl.h:550-557), -1 when t is unknown
int use_count(const struct ggml_cgraph *g, const struct ggml_tensor *t) {
    const struct ggml_hash_set &h = g->visited_hash_set;
    if (!g->use_counts || !h.used || !h.keys || h.size == 0) return -1;
    const size_t h0 = ((size_t)(uintptr_t)t >> 4) % h.size;
    size_t i = h0;
    while (h.used[i >> 5] & (1u << (i & 31))) {
        if (h.keys[i] == t) return g->use_counts[i];
        i = (i + 1) % h.size;
        if (i == h0) break;
    }
    return -1;
}

// an intermediate the fused launch may skip: one use in the whole graph, not a view (others may
// read it through the view source), not a requested output
bool skippable(const struct ggml_cgraph *g, const struct ggml_tensor *t) {
    return use_count(g, t) == 1 && t->view_src == nullptr && !(t->flags & GGMLABI_TENSOR_FLAG_OUTPUT);
}

bool same_shape_t(const struct ggml_tensor *a, const struct ggml_tensor *b) {
    for (int i = 0; i < 4; ++i)
        if (a->ne[i] != b->ne[i]) return false;
    return true;
}

// f32 vector of n elements, contiguous (the ln gamma / beta and bias operands)
bool f32_vec(const struct ggml_tensor *t, int64_t n) {
    return t->type == GGMLABI_TYPE_F32 && t->ne[0] == n && t->ne[1] == 1 && t->ne[2] == 1 && t->ne[3] == 1 && t->nb[0] == 4;
}

// f32 2-D [ne0, ne1] with unit element stride
bool f32_2d(const struct ggml_tensor *t) {
    return t->type == GGMLABI_TYPE_F32 && t->nb[0] == 4 && t->ne[2] == 1 && t->ne[3] == 1;
}

bool disjoint(const struct ggml_tensor *a, const struct ggml_tensor *b) {
    const uintptr_t a0 = (uintptr_t)a->data, a1 = a0 + ggml_base().nbytes(a);
    const uintptr_t b0 = (uintptr_t)b->data, b1 = b0 + ggml_base().nbytes(b);
    return a1 <= b0 || b1 <= a0;
}

// the same bytes with the same layout (an in-place result): element-wise kernels read and write
// each element in the same thread, so this aliasing is safe
bool identical(const struct ggml_tensor *a, const struct ggml_tensor *b) {
    if (a->data != b->data || a->type != b->type) return false;
    for (int i = 0; i < 4; ++i)
        if (a->ne[i] != b->ne[i] || a->nb[i] != b->nb[i]) return false;
    return true;
}

int next_compute(const struct ggml_cgraph *g, int i, int n);
bool is_plain_copy(const struct ggml_tensor *t);

// f32 elements stored densely in row-major order (what a flat copy writes)
bool f32_dense(const struct ggml_tensor *t) {
    if (t->type != GGMLABI_TYPE_F32 || t->nb[0] != 4) return false;
    int64_t expect = 4;
    for (int d = 0; d < 4; ++d) {
        if (t->ne[d] > 1 && (int64_t)t->nb[d] != expect) return false;
        expect *= t->ne[d];
    }
    return true;
}

// the copies right after a fused run whose source is a row range of its output `out` (GPT-2's
// K / V cache writes after the qkv mat-vec + bias, main-sched.cpp:648-655): at most two, only
// view nodes between. The fused launch stores those rows to the copy destinations as well, and
// the copy nodes are marked done in the plan. `last`: graph index of the run's last node.
// Returns how many were taken.
int absorb_copies(BackendCtx *c, const struct ggml_cgraph *g, int last, int n, const struct ggml_tensor *out,
                  const struct ggml_tensor *x, MmArgs &a) {
    int taken = 0, j = last, j_first = -1;
#define NOFOLD(why)                                                                 \
    {                                                                               \
        logf("copy %s not folded into the mat-vec: %s\n", g->nodes[j]->name, why); \
        break;                                                                      \
    }
    while (taken < 2) {
        j = next_compute(g, j, n);
        if (j >= n) break;
        const struct ggml_tensor *cp = g->nodes[j];
        const struct ggml_tensor *src = cp->src[0];
        if (!is_plain_copy(cp) || !src) break;   // not a copy: nothing to fold (quiet)
        if (c->plan.skip[j] || c->plan.attn.count(j)) NOFOLD("planned elsewhere");
        if (src->view_src != out) NOFOLD("source is not a view of the mat-vec's output");
        if (src->type != GGMLABI_TYPE_F32 || src->nb[0] != 4 || src->nb[1] != out->nb[1] || src->ne[1] != out->ne[1] ||
            src->ne[2] != 1 || src->ne[3] != 1)
            NOFOLD("source layout");
        const int64_t off = (int64_t)((const uint8_t *)src->data - (const uint8_t *)out->data);
        if (off < 0 || off % 4 != 0 || off / 4 + src->ne[0] > out->ne[0]) NOFOLD("source rows");
        if (!f32_dense(cp) || ggml_base().nbytes(cp) != (size_t)(4 * src->ne[0] * src->ne[1])) NOFOLD("destination layout");
        // the destination (the copy node's own data, a view of its src[1]) must not be read or
        // written by the fused launch otherwise, nor overlap the other folded copy
        if (!disjoint(cp, out) || !disjoint(cp, x)) NOFOLD("destination overlaps the mat-vec's input or output");
        if (taken == 1 && !disjoint(cp, g->nodes[j_first])) NOFOLD("destinations overlap");
        a.cp_dst[taken] = static_cast<float *>(cp->data);
        a.cp_r0[taken] = (int)(off / 4);
        a.cp_n[taken] = (int)src->ne[0];
        a.cp_nb1[taken] = 4 * src->ne[0];
        c->plan.skip[j] = 1;
        if (taken == 0) j_first = j;
        logf("copy %s folded into the mat-vec's epilogue\n", cp->name);
        ++taken;
    }
#undef NOFOLD
    return taken;
}

// nodes consumed by a fused mat-vec run at node i (0: no fusion); rc receives the launch status
// GET_ROWS(a), GET_ROWS(b), ADD(first, second) with both row results used only by the ADD ->
// one launch (the GPT-2 embedding, main-sched.cpp:589-595); returns the nodes consumed
int fuse_embed(BackendCtx *c, const struct ggml_cgraph *g, int i, int n, int &rc) {
    if (i + 2 >= n) return 0;
    struct ggml_tensor *ga = g->nodes[i], *gb2 = g->nodes[i + 1], *add = g->nodes[i + 2];
    if (ga->op != GGMLABI_OP_GET_ROWS || gb2->op != GGMLABI_OP_GET_ROWS || add->op != GGMLABI_OP_ADD) return 0;
    if (add->src[0] != ga || add->src[1] != gb2 || !skippable(g, ga) || !skippable(g, gb2)) return 0;
    if (ga->type != GGMLABI_TYPE_F32 || gb2->type != GGMLABI_TYPE_F32 || add->type != GGMLABI_TYPE_F32) return 0;
    if (!same_shape_t(ga, gb2) || !same_shape_t(ga, add) || ga->ne[2] != 1 || ga->ne[3] != 1) return 0;
    if (gb2->src[0]->type != GGMLABI_TYPE_F32) return 0;
    rc = get_rows_add(tv(ga->src[0]), tv(ga->src[1]), tv(gb2->src[0]), tv(gb2->src[1]), tv(add), c->stream);
    if (rc == GGML_MI355X_EINVAL) { rc = GGML_MI355X_OK; return 0; }   // shapes the fused kernel does not take
    logf("fused embedding (3 nodes) at %s\n", add->name);
    return 3;
}

int fuse_matvec(BackendCtx *c, const struct ggml_cgraph *g, int i, int n, int &rc) {
    auto at = [&](int k) -> struct ggml_tensor * { return i + k < n ? g->nodes[i + k] : nullptr; };
    const struct ggml_tensor *x = nullptr, *ln_g = nullptr, *ln_b = nullptr;
    float eps = 0.f;
    int k = 0;
    struct ggml_tensor *t0 = at(0);
    if (t0->op == GGMLABI_OP_NORM) {
        struct ggml_tensor *mul = at(1), *add = at(2);
        if (!mul || !add || mul->op != GGMLABI_OP_MUL || add->op != GGMLABI_OP_ADD) return 0;
        if (mul->src[0] != t0 || add->src[0] != mul) return 0;
        if (!skippable(g, t0) || !skippable(g, mul) || !skippable(g, add)) return 0;
        x = t0->src[0];
        if (!f32_2d(x) || !f32_2d(t0) || !same_shape_t(x, t0) || !same_shape_t(mul, t0) || !same_shape_t(add, t0)) return 0;
        if (!f32_vec(mul->src[1], x->ne[0]) || !f32_vec(add->src[1], x->ne[0])) return 0;
        ln_g = mul->src[1];
        ln_b = add->src[1];
        std::memcpy(&eps, &t0->op_params[0], sizeof eps);
        k = 3;
    }
    struct ggml_tensor *mm = at(k);
    if (!mm || mm->op != GGMLABI_OP_MUL_MAT) return 0;
    const struct ggml_tensor *w = mm->src[0];
    if (x != nullptr) {
        if (mm->src[1] != at(k - 1)) return 0;
    } else {
        x = mm->src[1];
    }
    if (!is_hot_quant(w->type) || (w->buffer && is_split_buft(w->buffer->buft))) return 0;
    if (w->ne[2] != 1 || w->ne[3] != 1 || (int64_t)w->nb[0] != type_bytes(w->type)) return 0;
    const int64_t K = w->ne[0], N = w->ne[1], M = mm->ne[1];
    if (K != x->ne[0] || K % 64 != 0 || K > 8192 || K % type_blck(w->type) != 0) return 0;
    if (!f32_2d(x) || x->ne[1] != M || M < 1 || M > 8 || !f32_2d(mm) || mm->ne[0] != N || N > (1LL << 31) - 1) return 0;
    if ((uintptr_t)x->data % 16 != 0 || x->nb[1] % 16 != 0) return 0;
    int last = k, epi = 0;
    const struct ggml_tensor *bias = nullptr, *resid = nullptr;
    struct ggml_tensor *b1 = at(k + 1);
    if (b1 && b1->op == GGMLABI_OP_ADD && b1->src[0] == mm && f32_vec(b1->src[1], N) && same_shape_t(b1, mm) && skippable(g, mm)) {
        bias = b1->src[1];
        last = k + 1;
        struct ggml_tensor *b2 = at(k + 2);
        if (b2 && skippable(g, b1) && same_shape_t(b2, b1)) {
            if (b2->op == GGMLABI_OP_UNARY && b2->op_params[0] == GGMLABI_UNARY_OP_GELU && b2->src[0] == b1) {
                epi |= EPI_GELU;
                last = k + 2;
            } else if (b2->op == GGMLABI_OP_ADD && (b2->src[0] == b1) != (b2->src[1] == b1)) {
                const struct ggml_tensor *r = b2->src[0] == b1 ? b2->src[1] : b2->src[0];
                if (f32_2d(r) && same_shape_t(r, b1)) {
                    resid = r;
                    epi |= EPI_RESID;
                    last = k + 2;
                }
            }
        }
    }
    // every workgroup reads all of x while others already store rows of out, so out must not
    // overlap x (ggml-alloc may have placed it there once x's last reader was done); the residual
    // is read element by element where it is written, so it may be out itself. When the whole run
    // fails that, retry without its last node.
    const struct ggml_tensor *out = nullptr;
    for (;; --last) {
        if (last < k) return 0;   // not even the MUL_MAT's own result can take it
        if (last < k + 2) { resid = nullptr; epi = 0; }
        if (last < k + 1) bias = nullptr;
        if (ln_g == nullptr && bias == nullptr) return 0;   // a lone MUL_MAT: generic dispatch
        out = at(last);
        if (!f32_2d(out) || !same_shape_t(out, mm)) return 0;
        if (!disjoint(x, out)) continue;
        if (resid && !disjoint(resid, out) && !(resid->data == out->data && resid->nb[1] == out->nb[1])) continue;
        break;
    }
    MmArgs a{};
    a.w = static_cast<const uint8_t *>(w->data);
    a.nb01 = (int64_t)w->nb[1];
    a.nb02 = a.nb03 = a.nb01 * N;
    a.x = static_cast<const uint8_t *>(x->data);
    a.nb11 = (int64_t)x->nb[1];
    a.nb12 = a.nb13 = a.nb11 * M;
    a.dst = static_cast<uint8_t *>(out->data);
    a.nb1 = (int64_t)out->nb[1];
    a.nb2 = a.nb3 = a.nb1 * M;
    a.K = (int)K;
    a.N = (int)N;
    a.M = (int)M;
    a.ne12 = a.ne13 = a.r2 = a.r3 = 1;
    a.x_aligned16 = 1;
    a.ln_g = ln_g ? static_cast<const float *>(ln_g->data) : nullptr;
    a.ln_b = ln_b ? static_cast<const float *>(ln_b->data) : nullptr;
    a.ln_eps = eps;
    a.bias = bias ? static_cast<const float *>(bias->data) : nullptr;
    a.epi = epi;
    if (resid) {
        a.resid = static_cast<const uint8_t *>(resid->data);
        a.resid_nb1 = (int64_t)resid->nb[1];
    }
    a.fused = 1;
    if (bias != nullptr && !(epi & EPI_ARGMAX)) absorb_copies(c, g, i + last, n, out, x, a);   // (last: offset from i)
    const hipError_t e = mmvq_fused_launch(w->type, a, mmvq_fused_pick_nc((int)M, (int)K), N >= 16384 ? 2 : 1, c->stream);
    rc = e == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP;
    logf("fused %d nodes at %s (mat-vec %s, M=%d)\n", last + 1, t0->name, w->name, (int)M);
    return last + 1;
}

// nodes consumed by a fused [SCALE,] [DIAG_MASK_INF,] SOFT_MAX run at node i (0: no fusion)
int fuse_softmax(BackendCtx *c, const struct ggml_cgraph *g, int i, int n, int &rc) {
    auto at = [&](int k) -> struct ggml_tensor * { return i + k < n ? g->nodes[i + k] : nullptr; };
    SoftmaxPre pre{1.0f, 0.0f, -1};
    int k = 0;
    const struct ggml_tensor *in = at(0)->src[0];
    if (at(0)->op == GGMLABI_OP_SCALE) {
        std::memcpy(&pre.scale, &at(0)->op_params[0], sizeof(float));
        std::memcpy(&pre.bias, &at(0)->op_params[1], sizeof(float));
        k = 1;
    }
    if (at(k) && at(k)->op == GGMLABI_OP_DIAG_MASK_INF && (k == 0 || at(k)->src[0] == at(k - 1))) {
        pre.n_past = at(k)->op_params[0];
        ++k;
    }
    struct ggml_tensor *sm = at(k);
    if (k == 0 || !sm || sm->op != GGMLABI_OP_SOFT_MAX || sm->src[0] != at(k - 1)) return 0;
    for (int j = 0; j < k; ++j)
        if (!skippable(g, at(j)) || !same_shape_t(at(j), sm) || at(j)->type != GGMLABI_TYPE_F32) return 0;
    if (!disjoint(in, sm) && !identical(in, sm)) return 0;
    GraphOp gop;
    if (!graph_op_of(sm, gop)) return 0;
    gop.src[0] = tv(in);
    rc = run_soft_max_pre(gop, pre, c->stream);
    logf("fused %d nodes at %s (soft_max)\n", k + 1, at(0)->name);
    return k + 1;
}

// ------------------------------------------------------------------------------------------
// attention fusion (a graph pre-pass; its nodes are not adjacent in the node order):
//   [CONT Q] .. MUL_MAT(K, Q) [SCALE] [DIAG_MASK_INF] SOFT_MAX, MUL_MAT(V^T, .) [PERMUTE, CONT]
// with [CONT V^T] earlier, is GPT-2's attention (main-sched.cpp:658-732). One run_attention
// launch at the last node replaces them: K is read through its view of the cache, Q and V^T
// through the sources of their CONT nodes when those are skippable, and the result is written
// straight into the final CONT's layout. Every intermediate must be skippable, and every compute
// node between the first skipped node and the launch must belong to the pattern (a skipped
// node's memory may be handed to a later node by ggml-alloc, so nothing else may run between).
// ------------------------------------------------------------------------------------------
// dims (ne[k], flat element stride fs[k]) at flat element offset f0 of a contiguous tensor whose
// flat element order is S's (what CONT makes) -> byte strides / offset into S. False when a dim
// would carry across S's dimensions (then no strided view exists).
bool flat_to_strided(int nd, const int64_t *ne, const int64_t *fs, int64_t f0, const struct ggml_tensor *S, int64_t *nb,
                     int64_t &off) {
    int64_t pre[5] = {1, 0, 0, 0, 0};
    for (int m = 0; m < 4; ++m) pre[m + 1] = pre[m] * S->ne[m];
    int64_t ext[4];
    off = 0;
    for (int m = 0; m < 4; ++m) {
        ext[m] = (f0 / pre[m]) % S->ne[m];
        off += ext[m] * (int64_t)S->nb[m];
    }
    if (f0 >= pre[4]) return false;
    for (int k = 0; k < nd; ++k) {
        nb[k] = 0;
        if (ne[k] <= 1) continue;
        int m = 3;
        while (m > 0 && (pre[m] > fs[k] || fs[k] % pre[m] != 0)) --m;
        const int64_t q = fs[k] / pre[m];
        ext[m] += q * (ne[k] - 1);
        nb[k] = q * (int64_t)S->nb[m];
    }
    for (int m = 0; m < 4; ++m)
        if (ext[m] >= S->ne[m]) return false;
    return true;
}

int next_compute(const struct ggml_cgraph *g, int i, int n) {
    for (int j = i + 1; j < n; ++j)
        if (!is_view_op(g->nodes[j]->op) && !is_empty(g->nodes[j])) return j;
    return n;
}

bool is_plain_copy(const struct ggml_tensor *t) {
    return is_copy_op(t->op) && !is_hot_quant(t->type) && !is_hot_quant(t->src[0]->type);
}

// two independent copies with only view nodes between them (GPT-2's K and V cache writes,
// main-sched.cpp:654-655) as one launch; returns the nodes consumed (0: no pair)
int pair_copies(BackendCtx *c, const struct ggml_cgraph *g, int i, int n, int &rc) {
    const struct ggml_tensor *a = g->nodes[i];
    const int j = next_compute(g, i, n);
    if (j >= n || c->plan.skip[j] || c->plan.attn.count(j)) return 0;
    const struct ggml_tensor *b = g->nodes[j];
    if (!is_plain_copy(b) || b->src[0] == a || !disjoint(a, b->src[0]) || !disjoint(b, a->src[0]) || !disjoint(a, b)) return 0;
    GraphOp ga, gb;
    if (!graph_op_of(a, ga) || !graph_op_of(b, gb) || !cpy_pairable(ga, gb)) return 0;
    rc = run_cpy_pair(ga, &gb, c->stream);
    logf("fused 2 copies at %s and %s\n", a->name, b->name);
    return j - i + 1;
}

bool attn_type(const struct ggml_tensor *t) { return t->type == GGMLABI_TYPE_F32 || t->type == GGMLABI_TYPE_F16; }

void match_attention(const struct ggml_cgraph *g, int n, int ism, FusePlan &plan) {
    struct ggml_tensor *sm = g->nodes[ism];
    if (sm->src[1] || sm->src[2] || sm->type != GGMLABI_TYPE_F32 || !skippable(g, sm)) return;
    AttnView a{};
    float max_bias;
    std::memcpy(&a.sm_scale, &sm->op_params[0], sizeof(float));
    std::memcpy(&max_bias, &sm->op_params[1], sizeof(float));
    if (max_bias != 0.0f) return;
    a.pre_s = 1.0f;
    a.n_past = -1;
    std::vector<const struct ggml_tensor *> skip = {sm};
    struct ggml_tensor *t = sm->src[0];
    if (t->op == GGMLABI_OP_DIAG_MASK_INF) {
        a.n_past = t->op_params[0];
        skip.push_back(t);
        t = t->src[0];
    }
    if (t->op == GGMLABI_OP_SCALE) {
        std::memcpy(&a.pre_s, &t->op_params[0], sizeof(float));
        std::memcpy(&a.pre_b, &t->op_params[1], sizeof(float));
        skip.push_back(t);
        t = t->src[0];
    }
    const struct ggml_tensor *kq = t;
    if (kq->op != GGMLABI_OP_MUL_MAT) return;
    skip.push_back(kq);
    for (const struct ggml_tensor *c : skip)
        if (!skippable(g, c) || !same_shape_t(c, sm) || c->type != GGMLABI_TYPE_F32) return;
    const struct ggml_tensor *K = kq->src[0], *Q = kq->src[1];
    const int ikqv = next_compute(g, ism, n);
    if (ikqv >= n) return;
    struct ggml_tensor *kqv = g->nodes[ikqv];
    if (kqv->op != GGMLABI_OP_MUL_MAT || kqv->src[1] != sm || kqv->type != GGMLABI_TYPE_F32) return;
    const struct ggml_tensor *Vt = kqv->src[0];
    const int64_t D = K->ne[0], n_kv = K->ne[1], Hk = K->ne[2], n_q = Q->ne[1], H = Q->ne[2];
    if (!attn_type(K) || Q->type != GGMLABI_TYPE_F32 || !attn_type(Vt)) return;
    if (K->ne[3] != 1 || Q->ne[3] != 1 || Q->ne[0] != D || Hk < 1 || H % Hk != 0) return;
    if (kq->ne[0] != n_kv || kq->ne[1] != n_q || kq->ne[2] != H || kq->ne[3] != 1) return;
    if (Vt->ne[0] != n_kv || Vt->ne[1] != D || Vt->ne[2] != Hk || Vt->ne[3] != 1) return;
    if (kqv->ne[0] != D || kqv->ne[1] != n_q || kqv->ne[2] != H || kqv->ne[3] != 1) return;
    if (D > ATTN_MAX_D || n_kv > ATTN_MAX_KV || n_q > 65535 || H > 65535) return;

    // output: through PERMUTE + CONT when that is what follows, else kqv itself
    int ianchor = ikqv;
    const struct ggml_tensor *out = kqv;
    int64_t onb[3] = {(int64_t)kqv->nb[0], (int64_t)kqv->nb[1], (int64_t)kqv->nb[2]};
    const int io = next_compute(g, ikqv, n);
    if (io < n) {
        const struct ggml_tensor *o = g->nodes[io], *p = o->src[0];
        if (o->op == GGMLABI_OP_CONT && o->type == GGMLABI_TYPE_F32 && p && p->op == GGMLABI_OP_PERMUTE && p->src[0] == kqv &&
            p->view_src == kqv && p->view_offs == 0 && use_count(g, kqv) == 1 && use_count(g, p) == 1 &&
            !(kqv->flags & GGMLABI_TENSOR_FLAG_OUTPUT) && !(p->flags & GGMLABI_TENSOR_FLAG_OUTPUT) && kqv->view_src == nullptr) {
            int64_t P[5] = {1, 0, 0, 0, 0};
            for (int j = 0; j < 4; ++j) P[j + 1] = P[j] * p->ne[j];
            const int64_t ne[3] = {D, n_q, H};
            int64_t fs[3] = {0, 0, 0}, nb[3], off;
            bool ok = true;
            for (int k = 0; k < 3 && ok; ++k) {
                if (ne[k] <= 1) continue;
                int jm = -1;
                for (int j = 0; j < 4; ++j)
                    if (p->nb[j] == kqv->nb[k] && p->ne[j] == kqv->ne[k]) jm = j;
                if (jm < 0) ok = false;
                else fs[k] = P[jm];
            }
            if (ok && flat_to_strided(3, ne, fs, 0, o, nb, off) && off == 0) {
                out = o;
                ianchor = io;
                for (int k = 0; k < 3; ++k) onb[k] = nb[k];
                skip.push_back(kqv);
            }
        }
    }
    a.o = out->data;
    a.o_d = onb[0]; a.o_i = onb[1]; a.o_h = onb[2];

    // Q: through its CONT when Q is a direct, single-use view of a skippable f32 CONT
    const struct ggml_tensor *qsrc = Q;
    a.q = Q->data;
    a.q_d = Q->nb[0]; a.q_i = Q->nb[1]; a.q_h = Q->nb[2];
    {
        const struct ggml_tensor *c = Q->view_src;
        if (is_view_op(Q->op) && c && Q->src[0] == c && c->op == GGMLABI_OP_CONT && c->type == GGMLABI_TYPE_F32 &&
            use_count(g, Q) == 1 && skippable(g, c) && c->src[0]->type == GGMLABI_TYPE_F32 && Q->nb[0] % 4 == 0 &&
            Q->nb[1] % 4 == 0 && Q->nb[2] % 4 == 0 && Q->view_offs % 4 == 0) {
            const int64_t ne[3] = {Q->ne[0], Q->ne[1], Q->ne[2]};
            const int64_t fs[3] = {(int64_t)Q->nb[0] / 4, (int64_t)Q->nb[1] / 4, (int64_t)Q->nb[2] / 4};
            int64_t nb[3], off;
            if (flat_to_strided(3, ne, fs, (int64_t)Q->view_offs / 4, c->src[0], nb, off)) {
                qsrc = c->src[0];
                a.q = static_cast<const char *>(qsrc->data) + off;
                a.q_d = nb[0]; a.q_i = nb[1]; a.q_h = nb[2];
                skip.push_back(c);
            }
        }
    }
    // V^T: through its CONT when that is skippable
    const struct ggml_tensor *vsrc = Vt;
    a.v = Vt->data;
    a.v_f16 = Vt->type == GGMLABI_TYPE_F16;
    a.v_j = Vt->nb[0]; a.v_d = Vt->nb[1]; a.v_h = Vt->nb[2];
    if (Vt->op == GGMLABI_OP_CONT && skippable(g, Vt) && Vt->src[0]->type == Vt->type) {
        const int64_t ne[3] = {Vt->ne[0], Vt->ne[1], Vt->ne[2]};
        const int64_t fs[3] = {1, Vt->ne[0], Vt->ne[0] * Vt->ne[1]};
        int64_t nb[3], off;
        if (flat_to_strided(3, ne, fs, 0, Vt->src[0], nb, off)) {
            vsrc = Vt->src[0];
            a.v = static_cast<const char *>(vsrc->data) + off;
            a.v_j = nb[0]; a.v_d = nb[1]; a.v_h = nb[2];
            skip.push_back(Vt);
        }
    }
    a.k = K->data;
    a.k_f16 = K->type == GGMLABI_TYPE_F16;
    a.k_d = K->nb[0]; a.k_j = K->nb[1]; a.k_h = K->nb[2];
#define NOFUSE(why)                                                                  \
    do {                                                                             \
        logf("attention at %s not fused: %s\n", sm->name, why);                      \
        return;                                                                      \
    } while (0)
    // the launch writes `out` while reading these. ggml-alloc may hand Q's source (freed once its
    // CONT ran) to the output: that is safe only when every (query, head) reads its Q row exactly
    // where it writes its result (a workgroup reads q before it writes o)
    const bool q_exact = a.o == a.q && (D <= 1 || a.o_d == a.q_d) && (n_q <= 1 || a.o_i == a.q_i) && (H <= 1 || a.o_h == a.q_h);
    if (!disjoint(out, qsrc) && !q_exact) NOFUSE("output overlaps Q");
    if (!disjoint(out, K) || !disjoint(out, vsrc)) NOFUSE("output overlaps K or V");
    int first = ianchor;
    std::vector<int> sidx;
    for (const struct ggml_tensor *x : skip) {   // the pattern's nodes sit shortly before the launch
        int j = ianchor;
        while (j >= 0 && ianchor - j < 256 && g->nodes[j] != x) --j;
        if (j < 0 || ianchor - j >= 256 || plan.skip[j] || plan.attn.count(j)) NOFUSE("pattern nodes not found");
        sidx.push_back(j);
        first = std::min(first, j);
    }
    // a node outside the pattern that runs between its first skipped node and the launch may write
    // what the launch reads only if it did so before the skipped node that read it (a cache write
    // ahead of the attention); its own inputs are never skipped nodes (those have one use each)
    auto pos = [&](const struct ggml_tensor *x) {
        for (size_t u = 0; u < skip.size(); ++u)
            if (skip[u] == x) return sidx[u];
        return ianchor;
    };
    const int rd_k = pos(kq);
    const int rd_q = qsrc == Q ? pos(kq) : pos(Q->view_src);
    const int rd_v = vsrc == Vt ? ianchor : pos(Vt);
    for (int j = first; j < ianchor; ++j) {
        const struct ggml_tensor *x = g->nodes[j];
        if (is_view_op(x->op) || is_empty(x) || std::find(sidx.begin(), sidx.end(), j) != sidx.end()) continue;
        if ((!disjoint(x, qsrc) && j > rd_q) || (!disjoint(x, K) && j > rd_k) || (!disjoint(x, vsrc) && j > rd_v))
            NOFUSE("an interleaved node overwrites an input");
    }
#undef NOFUSE
    a.D = (int)D; a.n_q = (int)n_q; a.n_kv = (int)n_kv; a.H = (int)H; a.Hk = (int)Hk;
    for (int j : sidx) plan.skip[j] = 1;
    plan.attn[ianchor] = a;
}

// ------------------------------------------------------------------------------------------
// GPT-2 layer fusion (a graph pre-pass, like the attention fusion below it in the plan). One
// decode layer of the reference example (main-sched.cpp:600-812 at N = 1: norm -> qkv -> K / V
// cache copies -> attention -> c_proj + residual -> norm -> fc + GELU -> proj + residual, ~28
// compute nodes) whose intermediates nobody outside the layer reads runs as the decode engine's
// two launches (gpt2_block.hip: the attention block and the MLP block, K-split c_proj and MLP
// projection as f32 partial slabs). Consecutive fused layers pass the residual as (base, bias,
// partials), summed by the next launch's prologue, exactly as the engine does; the last one of
// a run materializes its output node with one resid launch. Same arithmetic as the node-by-node
// path (int8 activations per 32-block, f32 scales), only the fp32 order of the K-split sums
// differs. GGML_MI355X_LAYER_FUSION=0 turns it off.
// ------------------------------------------------------------------------------------------
bool layer_fusion_on() {
    return settings().layer_fusion;
}

// head-major c_proj and slice-major MLP-projection copies of a fused layer's weights (Q4_0 /
// Q8_0: the block kernels stream those K-splits contiguously, gpt2_block_repack). Made on first
// use and kept while the weights' bytes are unchanged: every write into one of our buffers drops
// the copies whose source bytes it overlaps (lr_invalidate).
struct LayerCopies {
    int device;
    uintptr_t o0, o1, m0, m1;   // source byte ranges (c_proj, MLP projection)
    uint8_t *o, *mp;            // one allocation: c_proj copy, then the projection copy
};
std::mutex g_lr_mu;
std::vector<LayerCopies> g_lr;
// g_lr_gen (declared with the repacked buffer above) is bumped whenever copies are freed: a
// hipGraph captured before must not be replayed (its launches hold the freed copies' addresses),
// as the scratch generation guards the scratch

void lr_invalidate(int device, const void *p, size_t n) {
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(p), a1 = a0 + n;
    std::lock_guard<std::mutex> lk(g_lr_mu);
    for (size_t i = 0; i < g_lr.size();) {
        const LayerCopies &L = g_lr[i];
        if (L.device == device && ((a0 < L.o1 && L.o0 < a1) || (a0 < L.m1 && L.m0 < a1))) {
            HIP_OK(hipSetDevice(device));
            HIP_OK(hipFree(L.o));   // (hipFree waits for the kernels still reading it)
            g_lr_gen.fetch_add(1);
            g_lr[i] = g_lr.back();
            g_lr.pop_back();
        } else {
            ++i;
        }
    }
}

// the copies of (w_o, w_mp) on c's device; nullptr when they would have to be made inside a
// stream capture (the caller then fails the capture and the eager run makes them)
bool layer_copies(BackendCtx *c, int type, int E, const uint8_t *w_o, size_t o_bytes, const uint8_t *w_mp, size_t mp_bytes,
                  const uint8_t *&o, const uint8_t *&mp) {
    const uintptr_t o0 = reinterpret_cast<uintptr_t>(w_o), m0 = reinterpret_cast<uintptr_t>(w_mp);
    {
        std::lock_guard<std::mutex> lk(g_lr_mu);
        for (const LayerCopies &L : g_lr)
            if (L.device == c->device && L.o0 == o0 && L.m0 == m0) {
                o = L.o;
                mp = L.mp;
                return true;
            }
    }
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(c->stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
    size_t ob = 0, mb = 0;
    (void)gpt2_block_repack(type, E, nullptr, nullptr, nullptr, nullptr, &ob, &mb, nullptr);
    LayerCopies L{c->device, o0, o0 + o_bytes, m0, m0 + mp_bytes, nullptr, nullptr};
    HIP_OK(hipMalloc(&L.o, ob + mb));
    L.mp = L.o + ob;
    // the copies are made on the side stream behind everything queued on the backend stream so
    // far (an asynchronous write of the weights, ggml_backend_tensor_set_async, may still be in
    // flight there)
    HIP_OK(hipEventRecord(c->aux_ready, c->stream));
    HIP_OK(hipStreamWaitEvent(c->aux, c->aux_ready, 0));
    HIP_OK(gpt2_block_repack(type, E, w_o, L.o, w_mp, L.mp, nullptr, nullptr, c->aux));
    HIP_OK(hipStreamSynchronize(c->aux));
    std::lock_guard<std::mutex> lk(g_lr_mu);
    g_lr.push_back(L);
    o = L.o;
    mp = L.mp;
    return true;
}

// a hot-quant 2-D weight with packed rows (the weight copies of gpt2_block_repack take the ggml
// row pitch), not row-split
bool quant_2d(const struct ggml_tensor *w, int64_t ne0, int64_t ne1) {
    return is_hot_quant(w->type) && w->ne[0] == ne0 && w->ne[1] == ne1 && w->ne[2] == 1 && w->ne[3] == 1 &&
           ne0 % type_blck(w->type) == 0 && (int64_t)w->nb[0] == type_bytes(w->type) &&
           (int64_t)w->nb[1] == ne0 / type_blck(w->type) * type_bytes(w->type) && !(w->buffer && is_split_buft(w->buffer->buft));
}

// one layer starting at the NORM node i; the run's nodes are consecutive in the node order (the
// example's graph builds them so: the cache copies are expanded first, then the rest of the
// layer, main-sched.cpp:650-655). True and r filled when every check passes.
bool match_layer(const struct ggml_cgraph *g, int n, int i, LayerRun &r) {
    struct ggml_tensor *nodes[24];
    int idx[24], k = 0;
    for (int j = i; j < n && k < 24; j = next_compute(g, j, n)) {
        idx[k] = j;
        nodes[k++] = g->nodes[j];
        if (j == n - 1) break;
    }
    if (k < 24) return false;
#define NOLAYER(why)                                                      \
    do {                                                                  \
        logf("layer at %s not fused: %s\n", g->nodes[i]->name, why);      \
        return false;                                                     \
    } while (0)
    auto op_is = [](const struct ggml_tensor *t, int op) { return t->op == op; };
    struct ggml_tensor *n0 = nodes[0], *mul1 = nodes[1], *add1 = nodes[2], *mq = nodes[3], *qb = nodes[4];
    const struct ggml_tensor *X = n0->src[0];
    if (!op_is(n0, GGMLABI_OP_NORM) || !f32_2d(X) || X->ne[1] != 1 || !f32_2d(n0) || !same_shape_t(X, n0)) return false;
    const int64_t E = X->ne[0];
    if (E % 64 != 0 || !gpt2_block_supported((int)E, (int)(E / 64))) return false;
    if (!op_is(mul1, GGMLABI_OP_MUL) || mul1->src[0] != n0 || !f32_vec(mul1->src[1], E)) return false;
    if (!op_is(add1, GGMLABI_OP_ADD) || add1->src[0] != mul1 || !f32_vec(add1->src[1], E)) return false;
    if (!op_is(mq, GGMLABI_OP_MUL_MAT) || mq->src[1] != add1 || !quant_2d(mq->src[0], E, 3 * E)) return false;
    if (!op_is(qb, GGMLABI_OP_ADD) || qb->src[0] != mq || !f32_vec(qb->src[1], 3 * E) || !f32_2d(qb)) return false;
    const int T = mq->src[0]->type;
    // K / V cache copies: rows E.. and 2E.. of qkv into views of the caches
    struct ggml_tensor *ck = nodes[5], *cv = nodes[6];
    auto qkv_view = [&](const struct ggml_tensor *v, size_t off) {
        return v && v->view_src == qb && v->view_offs == off && v->ne[0] == E && v->ne[1] == 1 && v->type == GGMLABI_TYPE_F32 &&
               v->nb[0] == 4;
    };
    if (!op_is(ck, GGMLABI_OP_CPY) || !op_is(cv, GGMLABI_OP_CPY) || !qkv_view(ck->src[0], 4 * E) || !qkv_view(cv->src[0], 8 * E))
        NOLAYER("K / V cache copies");
    if (ck->type != GGMLABI_TYPE_F32 || cv->type != GGMLABI_TYPE_F32 || !f32_dense(ck) || !f32_dense(cv)) NOLAYER("cache type");
    // Q contiguous and V^T (either order), then KQ, scale, mask, soft_max, KQV, merge
    struct ggml_tensor *qc = nodes[7], *vt = nodes[8];
    if (qc->src[0] && qc->src[0]->view_src != qb) std::swap(qc, vt);
    if (!op_is(qc, GGMLABI_OP_CONT) || !qkv_view(qc->src[0], 0) || qc->ne[0] != 64 || qc->ne[1] != E / 64 || qc->ne[2] != 1)
        NOLAYER("Q");
    const int H = (int)(E / 64);
    struct ggml_tensor *kq = nodes[9], *sc = nodes[10], *dm = nodes[11], *sm = nodes[12], *kqv = nodes[13], *cur = nodes[14];
    if (!op_is(kq, GGMLABI_OP_MUL_MAT) || !op_is(sc, GGMLABI_OP_SCALE) || !op_is(dm, GGMLABI_OP_DIAG_MASK_INF) ||
        !op_is(sm, GGMLABI_OP_SOFT_MAX) || !op_is(kqv, GGMLABI_OP_MUL_MAT) || !op_is(cur, GGMLABI_OP_CONT))
        NOLAYER("attention ops");
    const struct ggml_tensor *K = kq->src[0], *Q = kq->src[1];
    if (!Q || Q->view_src != qc || Q->ne[0] != 64 || Q->ne[1] != 1 || Q->ne[2] != H) NOLAYER("Q permute");
    const int n_past = dm->op_params[0];
    const int64_t n_kv = n_past + 1;
    if (n_past < 0 || K->type != GGMLABI_TYPE_F32 || K->ne[0] != 64 || K->ne[1] != n_kv || K->ne[2] != H || K->nb[0] != 4 ||
        (int64_t)K->nb[1] != 4 * E || K->nb[2] != 256 || !K->view_src)
        NOLAYER("K view");
    if (sc->src[0] != kq || dm->src[0] != sc || sm->src[0] != dm || sm->src[1] || sm->src[2]) NOLAYER("score chain");
    float s_scale, s_bias, sm_scale, max_bias;
    std::memcpy(&s_scale, &sc->op_params[0], 4);
    std::memcpy(&s_bias, &sc->op_params[1], 4);
    std::memcpy(&sm_scale, &sm->op_params[0], 4);
    std::memcpy(&max_bias, &sm->op_params[1], 4);
    if (s_bias != 0.f || sm_scale != 1.f || max_bias != 0.f) NOLAYER("score parameters");
    const struct ggml_tensor *P = vt->src[0];
    if (!op_is(vt, GGMLABI_OP_CONT) || kqv->src[0] != vt || kqv->src[1] != sm || !P || !P->view_src || P->type != GGMLABI_TYPE_F32 ||
        P->ne[0] != n_kv || P->ne[1] != 64 || P->ne[2] != H || (int64_t)P->nb[0] != 4 * E || P->nb[1] != 4 || P->nb[2] != 256 ||
        vt->ne[0] != n_kv || vt->ne[1] != 64 || vt->ne[2] != H)
        NOLAYER("V^T");
    float *kc = static_cast<float *>(K->data), *vc = static_cast<float *>(P->data);
    if (ck->data != kc + n_past * E || cv->data != vc + n_past * E) NOLAYER("cache copies are not row n_past of the caches read");
    const struct ggml_tensor *mg = cur->src[0];
    if (!mg || mg->view_src != kqv || kqv->ne[0] != 64 || kqv->ne[1] != 1 || kqv->ne[2] != H || cur->ne[0] != E || cur->ne[1] != 1)
        NOLAYER("attention output");
    // c_proj + bias + residual, then the MLP
    struct ggml_tensor *mo = nodes[15], *ob = nodes[16], *r1 = nodes[17], *n1 = nodes[18], *mul2 = nodes[19], *add2 = nodes[20];
    struct ggml_tensor *mf = nodes[21], *fb = nodes[22], *ge = nodes[23];
    if (!op_is(mo, GGMLABI_OP_MUL_MAT) || mo->src[1] != cur || !quant_2d(mo->src[0], E, E) || mo->src[0]->type != T) NOLAYER("c_proj");
    if (!op_is(ob, GGMLABI_OP_ADD) || ob->src[0] != mo || !f32_vec(ob->src[1], E)) NOLAYER("c_proj bias");
    if (!op_is(r1, GGMLABI_OP_ADD) || !((r1->src[0] == ob && r1->src[1] == X) || (r1->src[0] == X && r1->src[1] == ob)))
        NOLAYER("attention residual");
    if (!op_is(n1, GGMLABI_OP_NORM) || n1->src[0] != r1) NOLAYER("ln_2");
    if (!op_is(mul2, GGMLABI_OP_MUL) || mul2->src[0] != n1 || !f32_vec(mul2->src[1], E)) NOLAYER("ln_2 gain");
    if (!op_is(add2, GGMLABI_OP_ADD) || add2->src[0] != mul2 || !f32_vec(add2->src[1], E)) NOLAYER("ln_2 bias");
    if (!op_is(mf, GGMLABI_OP_MUL_MAT) || mf->src[1] != add2 || !quant_2d(mf->src[0], E, 4 * E) || mf->src[0]->type != T)
        NOLAYER("fc");
    if (!op_is(fb, GGMLABI_OP_ADD) || fb->src[0] != mf || !f32_vec(fb->src[1], 4 * E)) NOLAYER("fc bias");
    if (!op_is(ge, GGMLABI_OP_UNARY) || ge->op_params[0] != GGMLABI_UNARY_OP_GELU || ge->src[0] != fb) NOLAYER("gelu");
    const int j24 = next_compute(g, idx[23], n), j25 = j24 < n ? next_compute(g, j24, n) : n, j26 = j25 < n ? next_compute(g, j25, n) : n;
    if (j26 >= n) NOLAYER("graph ends inside the layer");
    struct ggml_tensor *mp = g->nodes[j24], *pb = g->nodes[j25], *r2 = g->nodes[j26];
    if (!op_is(mp, GGMLABI_OP_MUL_MAT) || mp->src[1] != ge || !quant_2d(mp->src[0], 4 * E, E) || mp->src[0]->type != T) NOLAYER("mlp proj");
    if (!op_is(pb, GGMLABI_OP_ADD) || pb->src[0] != mp || !f32_vec(pb->src[1], E)) NOLAYER("mlp proj bias");
    if (!op_is(r2, GGMLABI_OP_ADD) || !((r2->src[0] == pb && r2->src[1] == r1) || (r2->src[0] == r1 && r2->src[1] == pb)) ||
        !f32_2d(r2) || !same_shape_t(r2, X))
        NOLAYER("mlp residual");
    // every tensor the layer produces (views included) is read only inside the layer and is not
    // a requested output, except the layer's output
    // (a sorted source list, not a map: this runs for every layer of every decode graph)
    thread_local std::vector<const struct ggml_tensor *> srcs;
    srcs.clear();
    for (int j = i; j <= j26; ++j)
        for (int s = 0; s < GGMLABI_MAX_SRC; ++s)
            if (g->nodes[j]->src[s]) srcs.push_back(g->nodes[j]->src[s]);
    std::sort(srcs.begin(), srcs.end());
    for (int j = i; j < j26; ++j) {
        const struct ggml_tensor *t = g->nodes[j];
        if (t->flags & GGMLABI_TENSOR_FLAG_OUTPUT) NOLAYER("an intermediate is a requested output");
        const int u = use_count(g, t);
        const auto rg = std::equal_range(srcs.begin(), srcs.end(), t);
        if (u < 0 || u != (int)(rg.second - rg.first)) NOLAYER("an intermediate is read outside the layer");
    }
    // (the output may sit on the input's memory: the input is read by the first launch only, the
    // output written by the last)
    if (!disjoint(r2, K) || !disjoint(r2, P)) NOLAYER("output overlaps the caches");
#undef NOLAYER
    r = LayerRun{};
    r.last = j26;
    r.type = T;
    r.E = (int)E;
    r.n_head = H;
    r.n_past = n_past;
    r.x = static_cast<const float *>(X->data);
    r.out = static_cast<float *>(r2->data);
    r.out_t = r2;
    r.ln1_g = static_cast<const float *>(mul1->src[1]->data);
    r.ln1_b = static_cast<const float *>(add1->src[1]->data);
    r.ln2_g = static_cast<const float *>(mul2->src[1]->data);
    r.ln2_b = static_cast<const float *>(add2->src[1]->data);
    std::memcpy(&r.eps1, &n0->op_params[0], 4);
    std::memcpy(&r.eps2, &n1->op_params[0], 4);
    r.scale = s_scale;
    r.w_qkv = static_cast<const uint8_t *>(mq->src[0]->data);
    r.nb_qkv = (int64_t)mq->src[0]->nb[1];
    r.w_o = static_cast<const uint8_t *>(mo->src[0]->data);
    r.nb_o = (int64_t)mo->src[0]->nb[1];
    r.w_fc = static_cast<const uint8_t *>(mf->src[0]->data);
    r.nb_fc = (int64_t)mf->src[0]->nb[1];
    r.w_mp = static_cast<const uint8_t *>(mp->src[0]->data);
    r.nb_mp = (int64_t)mp->src[0]->nb[1];
    r.b_qkv = static_cast<const float *>(qb->src[1]->data);
    r.b_o = static_cast<const float *>(ob->src[1]->data);
    r.b_fc = static_cast<const float *>(fb->src[1]->data);
    r.b_mp = static_cast<const float *>(pb->src[1]->data);
    r.kc = kc;
    r.vc = vc;
    {   // rows of K / V storage from the layer's first row to the end of the cache tensors
        const struct ggml_tensor *kb = K->view_src, *vb = P->view_src;
        const int64_t ck = ((const uint8_t *)kb->data + ggml_base().nbytes(kb) - (const uint8_t *)kc) / (4 * E);
        const int64_t cv2 = ((const uint8_t *)vb->data + ggml_base().nbytes(vb) - (const uint8_t *)vc) / (4 * E);
        r.cap = std::min(ck, cv2);
        if (r.cap <= n_past) return false;
    }
    return true;
}

void plan_layers(BackendCtx *c, const struct ggml_cgraph *g, int n, FusePlan &plan) {
    plan.layers.clear();
    if (!layer_fusion_on() || c->lf_mem == nullptr) return;
    LayerRun *prev = nullptr;
    for (int i = 0; i < n; ++i) {
        if (g->nodes[i]->op != GGMLABI_OP_NORM || plan.skip[i]) continue;
        LayerRun r;
        if (!match_layer(g, n, i, r)) continue;
        // chained: this layer's input is the previous fused layer's output, read by nothing else
        if (prev && prev->out == r.x && prev->E == r.E && next_compute(g, prev->last, n) == i && use_count(g, prev->out_t) == 2 &&
            !(prev->out_t->flags & GGMLABI_TENSOR_FLAG_OUTPUT)) {
            prev->chain_out = true;
            r.chain_in = true;
            r.b_in = prev->b_mp;
        }
        for (int j = i + 1; j <= r.last; ++j) plan.skip[j] = 1;
        auto it = plan.layers.emplace(i, r).first;
        prev = &it->second;
        logf("layer fused: %s .. %s (n_past %d%s)\n", g->nodes[i]->name, g->nodes[r.last]->name, r.n_past,
             r.chain_in ? ", residual from the previous layer" : "");
        i = r.last;
    }
    plan.pos_word = !plan.layers.empty();
    plan.n_past = plan.pos_word ? plan.layers.begin()->second.n_past : 0;
    for (const auto &kv : plan.layers) plan.pos_word = plan.pos_word && kv.second.n_past == plan.n_past;
}

int run_layer(BackendCtx *c, const LayerRun &r) {
    const uint8_t *w_o = r.w_o, *w_mp = r.w_mp;
    if (gpt2_block_repacks(r.type) &&
        !layer_copies(c, r.type, r.E, r.w_o, (size_t)r.nb_o * r.E, r.w_mp, (size_t)r.nb_mp * r.E, w_o, w_mp))
        return GGML_MI355X_EHIP;   // inside a capture: the eager run makes the copies
    const int n_sl = gpt2_block_mlp_slices(r.E);
    auto ok = [](hipError_t e) { return e == hipSuccess ? GGML_MI355X_OK : GGML_MI355X_EHIP; };
    int rc;
    const float *base = r.chain_in ? c->lf_y : r.x;
    // the kernels take the position as min(pos, n_ctx - 1): with the position word set to n_past
    // (plan.pos_word) n_ctx is the cache capacity, a bound only; otherwise the word holds
    // INT32_MAX and n_ctx = n_past + 1 carries the position
    const int n_ctx = c->plan.pos_word ? (int)std::min<int64_t>(r.cap, INT32_MAX) : r.n_past + 1;
    rc = ok(gpt2_attn_block_launch(0, r.type, base, r.b_in, r.chain_in ? c->lf_mlp : nullptr,
                                   r.chain_in ? n_sl : 0, c->lf_x, r.ln1_g, r.ln1_b, r.eps1, r.w_qkv, r.nb_qkv, r.b_qkv, r.kc,
                                   r.vc, c->lf_pos, r.scale, n_ctx, w_o, r.nb_o, c->lf_attn, r.E, r.n_head, 1, nullptr, 0,
                                   nullptr, nullptr, 0, c->stream));
    if (rc) return rc;
    rc = ok(gpt2_mlp_block_launch(0, r.type, c->lf_x, r.b_o, c->lf_attn, r.n_head, c->lf_y, r.ln2_g, r.ln2_b, r.eps2, r.w_fc, r.nb_fc,
                                  r.b_fc, w_mp, r.nb_mp, c->lf_mlp, r.E, r.n_head, 1, c->stream));
    if (rc) return rc;
    if (!r.chain_out) rc = ok(gpt2_resid_launch(c->lf_y, r.b_mp, c->lf_mlp, n_sl, r.out, r.E, 1, c->stream));
    return rc;
}

void plan_fusion(BackendCtx *c, const struct ggml_cgraph *g, int n, FusePlan &plan) {
    plan.skip.assign(n, 0);
    plan.attn.clear();
    plan.layers.clear();
    if (!fusion_on()) return;
    plan_layers(c, g, n, plan);
    for (int i = 0; i < n; ++i)
        if (g->nodes[i]->op == GGMLABI_OP_SOFT_MAX && !plan.skip[i]) match_attention(g, n, i, plan);
}

// queue every node of g on the backend stream (fused runs as planned); quiet: a failure is
// expected to be retried (inside a hipGraph capture) and is only logged in debug mode
// (planned: c->plan already holds this graph's plan and its position word is set)
void set_pos_word(BackendCtx *c) {
    if (c->lf_pos == nullptr) return;
    const int v = c->plan.pos_word ? c->plan.n_past : 0x7fffffff;
    HIP_OK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(c->lf_pos), v, 1, c->stream));
}

enum ggml_status run_nodes(BackendCtx *c, struct ggml_cgraph *g, bool quiet, bool planned = false) {
    const GgmlBase &gb = ggml_base();
    const int n = gb.graph_n_nodes(g);
    FusePlan &plan = c->plan;
    if (!planned) {
        plan_fusion(c, g, n, plan);
        if (!plan.layers.empty()) set_pos_word(c);
    }
    for (int i = 0; i < n; ++i) {
        struct ggml_tensor *node = gb.graph_node(g, i);
        if (is_empty(node) || is_view_op(node->op) || plan.skip[i]) continue;
        int rc = GGML_MI355X_OK;
        GraphOp gop;
        int fused = 0;
        auto at = plan.attn.find(i);
        auto lr = plan.layers.find(i);
        if (lr != plan.layers.end()) {
            rc = run_layer(c, lr->second);
            fused = lr->second.last - i + 1;
        } else if (at != plan.attn.end()) {
            rc = run_attention(at->second, c->stream);
            logf("fused attention at %s (n_kv=%d, n_q=%d, H=%d)\n", node->name, at->second.n_kv, at->second.n_q, at->second.H);
            fused = 1;
        } else if (fusion_on()) {
            if (node->op == GGMLABI_OP_NORM || node->op == GGMLABI_OP_MUL_MAT) fused = fuse_matvec(c, g, i, n, rc);
            else if (node->op == GGMLABI_OP_SCALE || node->op == GGMLABI_OP_DIAG_MASK_INF) fused = fuse_softmax(c, g, i, n, rc);
            else if (is_plain_copy(node)) fused = pair_copies(c, g, i, n, rc);
            else if (node->op == GGMLABI_OP_GET_ROWS) fused = fuse_embed(c, g, i, n, rc);
        }
        if (fused > 0) {
            i += fused - 1;
        } else if (node->op == GGMLABI_OP_MUL_MAT && node->src[0]->buffer && is_split_buft(node->src[0]->buffer->buft)) {
            rc = be_split_mul_mat(c, node);
        } else if (node->op == GGMLABI_OP_MUL_MAT && is_hot_quant(node->src[0]->type)) {
            rc = mul_mat_rp(tv(node->src[0]), repacked_of(node->src[0]), tv(node->src[1]), tv(node), c->stream, c->scratch);
        } else if (node->op == GGMLABI_OP_MUL_MAT_ID) {
            rc = mul_mat_id(tv(node->src[0]), tv(node->src[1]), tv(node->src[2]), tv(node), c->stream, c->scratch);
        } else if (node->op == GGMLABI_OP_GET_ROWS) {
            rc = get_rows(tv(node->src[0]), tv(node->src[1]), tv(node), c->stream);
        } else if (is_quant_copy(node)) {
            rc = cpy(tv(node->src[0]), tv(node), c->stream);   // for CPY node is the view of src[1]
        } else if (graph_op_of(node, gop)) {
            rc = run_graph_op(gop, c->stream);
        } else {
            fprintf(stderr, "[ggml-mi355x] unsupported op %d in graph (node %s)\n", node->op, node->name);
            return GGML_STATUS_FAILED;
        }
        if (rc != GGML_MI355X_OK) {
            if (quiet) logf("node %s (op %d) failed during capture: %s\n", node->name, node->op, ggml_mi355x_strerror(rc));
            else fprintf(stderr, "[ggml-mi355x] node %s (op %d) failed: %s\n", node->name, node->op, ggml_mi355x_strerror(rc));
            return GGML_STATUS_FAILED;
        }
    }
    return GGML_STATUS_SUCCESS;
}

// hipGraph use, as the reference decides for CUDA graphs (ggml-cuda.cu:2890-2998): on unless
// GGML_MI355X_GRAPHS=0; never for graphs with row-split weights (their shards run on other
// devices' streams); a graph whose nodes changed is re-captured and the executable updated in
// place, and after GGML_MI355X_GRAPH_MAX_UPDATES (default 4) such calls in a row the backend
// stops capturing (the graph changes every call, so capturing only adds host work).
bool graphs_on() {
    return settings().graphs;
}
int graph_max_updates() {
    return settings().graph_max_updates;
}

void node_props(const struct ggml_tensor *t, NodeProps &p) {
    std::memset(&p, 0, sizeof p);
    p.node = t;
    p.data = t->data;
    p.op = t->op;
    p.flags = t->flags;
    p.type = t->type;
    for (int i = 0; i < 4; ++i) {
        p.ne[i] = t->ne[i];
        p.nb[i] = t->nb[i];
    }
    std::memcpy(p.op_params, t->op_params, sizeof p.op_params);
    for (int i = 0; i < GGMLABI_MAX_SRC; ++i) {
        p.src[i] = t->src[i];
        p.src_data[i] = t->src[i] ? t->src[i]->data : nullptr;
        if (t->src[i]) {
            p.src_type[i] = t->src[i]->type;
            for (int d = 0; d < 4; ++d) {
                p.src_ne[i][d] = t->src[i]->ne[d];
                p.src_nb[i][d] = t->src[i]->nb[d];
            }
        }
    }
}

// a fused decode layer as one record of what its launches read (run_layer): everything but the
// position, which moves every token (the cache views, the mask's n_past, the score shapes) and
// reaches the kernels through the backend's position word instead (FusePlan::pos_word)
void layer_props(const struct ggml_tensor *first, const LayerRun &r, NodeProps &p) {
    std::memset(&p, 0, sizeof p);
    p.node = first;
    p.data = r.out;
    p.op = -1;                                   // (no ggml op has this id)
    p.type = r.type;
    p.ne[0] = r.E; p.ne[1] = r.n_head; p.ne[2] = r.last; p.ne[3] = (r.chain_in ? 1 : 0) | (r.chain_out ? 2 : 0);
    p.nb[0] = (size_t)r.nb_qkv; p.nb[1] = (size_t)r.nb_o; p.nb[2] = (size_t)r.nb_fc; p.nb[3] = (size_t)r.nb_mp;
    std::memcpy(&p.op_params[0], &r.eps1, 4);
    std::memcpy(&p.op_params[1], &r.eps2, 4);
    std::memcpy(&p.op_params[2], &r.scale, 4);
    std::memcpy(&p.op_params[3], &r.cap, 8);
    const void *ptrs[] = {r.x, r.ln1_g, r.ln1_b, r.ln2_g, r.ln2_b, r.w_qkv, r.w_o, r.w_fc, r.w_mp, r.b_qkv,
                          r.b_o, r.b_fc, r.b_mp, r.kc, r.vc, r.b_in};
    static_assert(sizeof ptrs / sizeof ptrs[0] <= 2 * GGMLABI_MAX_SRC, "room for the layer's pointers");
    for (size_t i = 0; i < sizeof ptrs / sizeof ptrs[0]; ++i) (i < GGMLABI_MAX_SRC ? p.src[i] : p.src_data[i - GGMLABI_MAX_SRC]) = ptrs[i];
}

// true when g (as planned) queues the launches the cached graph was captured from; refreshes the
// cache either way. Nodes compare by their properties; a fused decode layer by layer_props when
// its position comes from the position word, so a decode graph that differs from the last one
// only in its position is replayed, not re-captured.
bool graph_unchanged(GraphCache &hg, struct ggml_cgraph *g, const FusePlan &plan) {
    const GgmlBase &gb = ggml_base();
    const int n = gb.graph_n_nodes(g);
    thread_local std::vector<NodeProps> cur;
    cur.clear();
    for (int i = 0; i < n; ++i) {
        NodeProps p;
        const auto lr = plan.pos_word ? plan.layers.find(i) : plan.layers.end();
        if (lr != plan.layers.end()) {
            layer_props(gb.graph_node(g, i), lr->second, p);
            i = lr->second.last;
        } else {
            node_props(gb.graph_node(g, i), p);
        }
        cur.push_back(p);
    }
    const bool same = cur.size() == hg.props.size() && std::memcmp(cur.data(), hg.props.data(), cur.size() * sizeof(NodeProps)) == 0;
    hg.props.swap(cur);
    return same;
}

bool has_split_weights(struct ggml_cgraph *g) {
    const GgmlBase &gb = ggml_base();
    const int n = gb.graph_n_nodes(g);
    for (int i = 0; i < n; ++i) {
        const struct ggml_tensor *t = gb.graph_node(g, i);
        if (t->op == GGMLABI_OP_MUL_MAT && t->src[0]->buffer && is_split_buft(t->src[0]->buffer->buft)) return true;
    }
    return false;
}

enum ggml_status be_graph_compute(ggml_backend_t b, struct ggml_cgraph *g) {
    BackendCtx *c = be_ctx(b);
    if (!ggml_base().ok) return GGML_STATUS_FAILED;
    HIP_OK(hipSetDevice(c->device));
    GraphCache &hg = c->hg;
    if (!graphs_on() || hg.disabled || has_split_weights(g)) {
        // an eager run may grow (reallocate) the scratch a cached executable points into; the
        // generation check below then refuses to replay it
        return run_nodes(c, g, false);
    }
    plan_fusion(c, g, ggml_base().graph_n_nodes(g), c->plan);
    // the position word is written outside the captured launches, before every run of them
    if (!c->plan.layers.empty()) set_pos_word(c);
    const bool same = graph_unchanged(hg, g, c->plan) && hg.scratch_gen == c->scratch.gen && hg.lr_gen == g_lr_gen.load();
    if (same && hg.exec) {
        hg.updates = 0;
        logf("hipGraph replayed on %s (%d nodes%s)\n", c->name.c_str(), ggml_base().graph_n_nodes(g),
             c->plan.pos_word ? ", position word" : "");
        HIP_OK(hipGraphLaunch(hg.exec, c->stream));
        return GGML_STATUS_SUCCESS;
    }
    if (hg.exec && ++hg.updates >= graph_max_updates() && graph_max_updates() > 0) {
        logf("graph changed on %d calls in a row: no more hipGraph capture on %s\n", hg.updates, c->name.c_str());
        hg.disabled = true;
        HIP_OK(hipGraphExecDestroy(hg.exec));
        hg.exec = nullptr;
        return run_nodes(c, g, false);
    }
    c->scratch.short_in_capture = false;
    HIP_OK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed));
    const enum ggml_status st = run_nodes(c, g, true, true);
    hipGraph_t graph = nullptr;
    const hipError_t ec = hipStreamEndCapture(c->stream, &graph);
    if (st != GGML_STATUS_SUCCESS || ec != hipSuccess || graph == nullptr || c->scratch.short_in_capture) {
        // a launch that cannot be captured yet (first use of a scratch size, whether it failed or
        // took a scratch-free slower path): run eagerly once, which grows the scratch, and capture
        // on the next call
        (void)hipGetLastError();
        if (graph) (void)hipGraphDestroy(graph);
        hg.props.clear();
        return run_nodes(c, g, false, true);   // (planned, position word set above)
    }
    if (hg.exec) {
        hipGraphNode_t err_node = nullptr;
        hipGraphExecUpdateResult res;
        if (hipGraphExecUpdate(hg.exec, graph, &err_node, &res) != hipSuccess || res != hipGraphExecUpdateSuccess) {
            (void)hipGetLastError();
            HIP_OK(hipGraphExecDestroy(hg.exec));
            hg.exec = nullptr;
        }
    }
    if (!hg.exec) HIP_OK(hipGraphInstantiate(&hg.exec, graph, nullptr, nullptr, 0));
    hg.scratch_gen = c->scratch.gen;
    hg.lr_gen = g_lr_gen.load();
    HIP_OK(hipGraphDestroy(graph));
    HIP_OK(hipGraphLaunch(hg.exec, c->stream));
    return GGML_STATUS_SUCCESS;
}

void be_event_record(ggml_backend_t b, ggml_backend_event_t ev) {
    BackendCtx *c = be_ctx(b);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipEventRecord(static_cast<hipEvent_t>(ev->context), c->stream));
}

void be_event_wait(ggml_backend_t b, ggml_backend_event_t ev) {
    BackendCtx *c = be_ctx(b);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipStreamWaitEvent(c->stream, static_cast<hipEvent_t>(ev->context), 0));
}

const struct ggml_backend_i BACKEND_IFACE = {
    be_name, be_free, be_set_async, be_get_async, be_cpy_async, be_sync,
    nullptr, nullptr, nullptr, nullptr,
    be_graph_compute, be_event_record, be_event_wait,
};

bool is_our_backend(ggml_backend_t b) { return b && b->iface.graph_compute == be_graph_compute; }

// ------------------------------------------------------------------------------------------
// device
// ------------------------------------------------------------------------------------------
const char *dv_name(ggml_backend_dev_t d) { return dev_ctx(d)->name.c_str(); }
const char *dv_desc(ggml_backend_dev_t d) { return dev_ctx(d)->desc.c_str(); }

void dv_memory(ggml_backend_dev_t d, size_t *free_b, size_t *total_b) {
    HIP_OK(hipSetDevice(dev_ctx(d)->device));
    HIP_OK(hipMemGetInfo(free_b, total_b));
}

enum ggml_backend_dev_type dv_type(ggml_backend_dev_t) { return GGML_BACKEND_DEVICE_TYPE_GPU; }

void dv_props(ggml_backend_dev_t d, struct ggml_backend_dev_props *p) {
    p->name = dv_name(d);
    p->description = dv_desc(d);
    p->type = GGML_BACKEND_DEVICE_TYPE_GPU;
    dv_memory(d, &p->memory_free, &p->memory_total);
    p->caps.async = true;
    p->caps.host_buffer = true;
    p->caps.buffer_from_host_ptr = false;
    p->caps.events = true;
}

ggml_backend_t dv_init_backend(ggml_backend_dev_t d, const char *) {
    DeviceCtx *dc = dev_ctx(d);
    auto *c = new BackendCtx();
    c->device = dc->device;
    c->name = dc->name;
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&c->aux_ready, hipEventDisableTiming));
    (void)device_error_word();   // this device's GET_ROWS error word, made outside any capture
    {   // fused GPT-2 layers (plan_layers): n_embd <= 1024, <= 16 heads, <= 32 MLP slices, one sequence
        constexpr size_t E = 1024;
        HIP_OK(hipMalloc(&c->lf_mem, (16 + 32 + 2) * E * sizeof(float) + 256));
        c->lf_attn = static_cast<float *>(c->lf_mem);
        c->lf_mlp = c->lf_attn + 16 * E;
        c->lf_x = c->lf_mlp + 32 * E;
        c->lf_y = c->lf_x + E;
        // the block kernels take the position as min(pos[s], n_ctx - 1): pos holds INT32_MAX and
        // each launch passes n_ctx = n_past + 1, so no per-token write of the position
        c->lf_pos = reinterpret_cast<int32_t *>(c->lf_y + E);
        HIP_OK(hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(c->lf_pos), 0x7fffffff, 1));
    }
    // raise the fused mat-vec LDS limits now: that is not a stream operation, so it must not
    // first happen inside a hipGraph capture of be_graph_compute
    for (int t : {2, 8, 12, 13, 14}) HIP_OK(mmvq_fused_prepare(t));   // Q4_0 Q8_0 Q4_K Q5_K Q6_K
    auto *b = new ggml_backend();
    b->guid = &BACKEND_GUID;
    b->iface = BACKEND_IFACE;
    b->device = d;
    b->context = c;
    return b;
}

ggml_backend_buffer_type_t dv_buft(ggml_backend_dev_t d) { return &dev_ctx(d)->buft; }

ggml_backend_buffer_type_t dv_host_buft(ggml_backend_dev_t) { return host_buft(); }

bool supports_mm_operands(const struct ggml_tensor *a, const struct ggml_tensor *b) {
    if (!is_hot_quant(a->type) || b->type != GGMLABI_TYPE_F32) return false;
    if (a->ne[0] % type_blck(a->type) != 0 || (int64_t)a->nb[0] != type_bytes(a->type) || b->nb[0] != 4) return false;
    ggml_mi355x_tensor ta{}, tb{};
    ta.type = a->type;
    tb.type = b->type;
    for (int i = 0; i < 4; ++i) {
        ta.ne[i] = a->ne[i];
        tb.ne[i] = b->ne[i];
    }
    return ggml_mi355x_supports_mul_mat(&ta, &tb) != 0;
}

// mirrors the MUL_MAT arm of ggml_backend_cuda_device_supports_op (ggml-cuda.cu:3270-3330):
// only the quantized hot path is claimed; everything else stays on the CPU backend.
bool dv_supports_op(ggml_backend_dev_t d, const struct ggml_tensor *op) {
    // split buffers only feed MUL_MAT (reference ggml-cuda.cu:3215-3222), as a 2-D src0 against
    // contiguous f32 src1 / dst, with this device as the main device
    for (int i = 0; i < GGMLABI_MAX_SRC; ++i) {
        const struct ggml_tensor *t = op->src[i];
        if (!t || !t->buffer || !is_split_buft(t->buffer->buft)) continue;
        if (op->op != GGMLABI_OP_MUL_MAT || i != 0) return false;
        if (t->buffer->buft->device != d || t->ne[2] != 1 || t->ne[3] != 1) return false;
        if (!is_contiguous_rows(op->src[1]) || op->src[1]->nb[1] != op->src[1]->nb[0] * op->src[1]->ne[0]) return false;
        if (!is_contiguous_rows(op) || op->nb[1] != op->nb[0] * op->ne[0]) return false;
    }
    switch (op->op) {
        case GGMLABI_OP_NONE:
        case GGMLABI_OP_RESHAPE:
        case GGMLABI_OP_VIEW:
        case GGMLABI_OP_PERMUTE:
        case GGMLABI_OP_TRANSPOSE:
            return true;
        case GGMLABI_OP_MUL_MAT:
            if (!is_hot_quant(op->src[0]->type)) break;   // f32 / f16 weights: graph_ops (below)
            return op->type == GGMLABI_TYPE_F32 && supports_mm_operands(op->src[0], op->src[1]) &&
                   op->src[1]->ne[2] % op->src[0]->ne[2] == 0 && op->src[1]->ne[3] % op->src[0]->ne[3] == 0;
        case GGMLABI_OP_MUL_MAT_ID: {
            // exactly what mul_mat_id accepts (whole-K activations in LDS, <= 65535 pairs)
            if (op->type != GGMLABI_TYPE_F32 || !supports_mm_operands(op->src[0], op->src[1])) return false;
            const TensorView as = tv(op->src[0]), b = tv(op->src[1]), ids = tv(op->src[2]);
            return check_mul_mat_id(as, b, ids, tv(op)) == GGML_MI355X_OK;
        }
        // GET_ROWS of the hot quant types / f32 (dequantized rows, bit-exact), like get_rows_cuda
        case GGMLABI_OP_GET_ROWS:
            return check_get_rows(tv(op->src[0]), tv(op->src[1]), tv(op)) == GGML_MI355X_OK;
        // copies into / out of the hot types: f32 -> Q4_0 / Q8_0 (cpy_f32_q), Q* -> f32 (cpy_q_f32,
        // cpy.cu:94) and same-type block copies
        case GGMLABI_OP_CPY:
        case GGMLABI_OP_CONT:
        case GGMLABI_OP_DUP:
            if (is_quant_copy(op)) return check_cpy(tv(op->src[0]), tv(op)) == GGML_MI355X_OK;
            break;
        default:
            break;
    }
    // the f32 ops of the GPT-2 graph around the matmuls (graph_ops.hip)
    GraphOp g;
    return graph_op_of(op, g) && check_graph_op(g) == GGML_MI355X_OK;
}

bool dv_supports_buft(ggml_backend_dev_t d, ggml_backend_buffer_type_t bt) {
    if (is_split_buft(bt)) return bt->device == d;
    // a device's own buffer type only (as ggml_backend_cuda_device_supports_buft): with virtual
    // devices two plugin devices share one GPU, and the scheduler must still see two places
    return is_our_buft(bt) && static_cast<DeviceCtx *>(bt->context) == dev_ctx(d);
}

// like the CUDA backend: batched matmuls are worth moving weights across for
bool dv_offload_op(ggml_backend_dev_t, const struct ggml_tensor *op) {
    return (op->op == GGMLABI_OP_MUL_MAT || op->op == GGMLABI_OP_MUL_MAT_ID) && op->ne[1] >= 32;
}

ggml_backend_event_t dv_event_new(ggml_backend_dev_t d) {
    HIP_OK(hipSetDevice(dev_ctx(d)->device));
    hipEvent_t e;
    HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    auto *ev = new ggml_backend_event();
    ev->device = d;
    ev->context = e;
    return ev;
}

void dv_event_free(ggml_backend_dev_t d, ggml_backend_event_t ev) {
    HIP_OK(hipSetDevice(dev_ctx(d)->device));
    HIP_OK(hipEventDestroy(static_cast<hipEvent_t>(ev->context)));
    delete ev;
}

void dv_event_sync(ggml_backend_dev_t d, ggml_backend_event_t ev) {
    HIP_OK(hipSetDevice(dev_ctx(d)->device));
    HIP_OK(hipEventSynchronize(static_cast<hipEvent_t>(ev->context)));
}

const struct ggml_backend_device_i DEVICE_IFACE = {
    dv_name, dv_desc, dv_memory, dv_type, dv_props, dv_init_backend, dv_buft,
    dv_host_buft, nullptr,
    dv_supports_op, dv_supports_buft, dv_offload_op,
    dv_event_new, dv_event_free, dv_event_sync,
};

// ------------------------------------------------------------------------------------------
// registry
// ------------------------------------------------------------------------------------------
struct Registry {
    std::vector<std::unique_ptr<DeviceCtx>> ctxs;
    std::vector<std::unique_ptr<ggml_backend_device>> devs;
    struct ggml_backend_reg reg {};
};

const char *rg_name(ggml_backend_reg_t) { return "MI355X"; }

Registry &registry();

size_t rg_count(ggml_backend_reg_t) { return registry().devs.size(); }

ggml_backend_dev_t rg_dev(ggml_backend_reg_t, size_t i) {
    Registry &r = registry();
    return i < r.devs.size() ? r.devs[i].get() : nullptr;
}

struct ggml_backend_feature FEATURES[] = {
    {"ARCH", "gfx950"},
    {"MUL_MAT", "q4_0,q8_0,q4_K,q5_K,q6_K"},
    {"MMVQ", "wave64 dot4 + butterfly reduce"},
    {nullptr, nullptr},
};

struct ggml_backend_feature *rg_features(ggml_backend_reg_t) { return FEATURES; }

// ggml_backend_dev_get_extra_bufts (reference include/ggml-backend.h:192): NULL-terminated
ggml_backend_buffer_type_t *dv_extra_bufts(ggml_backend_dev_t d) { return dev_ctx(d)->extra_bufts; }

void *rg_proc(ggml_backend_reg_t, const char *name) {
    if (strcmp(name, "ggml_backend_get_features") == 0) return reinterpret_cast<void *>(rg_features);
    if (strcmp(name, "ggml_backend_split_buffer_type") == 0) return reinterpret_cast<void *>(mi355x_split_buffer_type);
    if (strcmp(name, "ggml_backend_dev_get_extra_bufts") == 0) return reinterpret_cast<void *>(dv_extra_bufts);
    if (strcmp(name, "ggml_backend_register_host_buffer") == 0) return reinterpret_cast<void *>(mi355x_register_host_buffer);
    if (strcmp(name, "ggml_backend_unregister_host_buffer") == 0) return reinterpret_cast<void *>(mi355x_unregister_host_buffer);
    if (strcmp(name, "ggml_mi355x_mul_mat") == 0) return reinterpret_cast<void *>(ggml_mi355x_mul_mat);
    if (strcmp(name, "ggml_mi355x_mul_mat_id") == 0) return reinterpret_cast<void *>(ggml_mi355x_mul_mat_id);
    if (strcmp(name, "ggml_mi355x_dequantize") == 0) return reinterpret_cast<void *>(ggml_mi355x_dequantize);
    return nullptr;
}

Registry &registry() {
    static Registry *r = [] {
        auto *R = new Registry();
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) {
            (void)hipGetLastError();
            n = 0;
        }
        auto add = [&](int hip_dev, const char *desc) {
            auto dc = std::make_unique<DeviceCtx>();
            dc->device = hip_dev;
            dc->name = std::string("MI355X") + std::to_string(R->ctxs.size());
            dc->desc = desc;
            dc->buft_name = std::string(BUFT_TAG) + std::to_string(R->ctxs.size());
            auto dev = std::make_unique<ggml_backend_device>();
            dev->iface = DEVICE_IFACE;
            dev->reg = &R->reg;
            dev->context = dc.get();
            dc->buft.iface = BUFT_IFACE;
            dc->buft.device = dev.get();
            dc->buft.context = dc.get();
            dc->rp_buft_name = dc->buft_name + "_Repack";
            dc->rp_buft.iface = RP_BUFT_IFACE;
            dc->rp_buft.device = dev.get();
            dc->rp_buft.context = dc.get();
            dc->extra_bufts[0] = &dc->rp_buft;
            R->ctxs.push_back(std::move(dc));
            R->devs.push_back(std::move(dev));
        };
        for (int i = 0; i < n; ++i) {
            hipDeviceProp_t p;
            if (hipGetDeviceProperties(&p, i) != hipSuccess || strncmp(p.gcnArchName, "gfx950", 6) != 0) continue;
            add(i, p.name);
        }
        // GGML_MI355X_VIRTUAL_DEVICES=k (testing): k plugin devices over the GPUs present, device
        // i on GPU i % n — on a one-GPU box the scheduler's multi-device split (graph splits,
        // cross-device tensor copies, stream / event hand-offs) runs with every device on GPU 0
        // (same-GPU copies instead of peer copies)
        const int n_real = (int)R->ctxs.size();
        for (int i = n_real; n_real > 0 && i < settings().virtual_devices; ++i) {
            const DeviceCtx &src = *R->ctxs[i % n_real];
            add(src.device, (src.desc + " (virtual)").c_str());
        }
        // peer access between every pair of our devices, once, at registry init: the scheduler's
        // cross-device hand-off (be_cpy_async) and the split buffer's row shards then move over
        // xGMI by direct DMA / direct loads. The reference enables it lazily around multi-device
        // mat-muls (ggml_cuda_set_peer_access, ggml-cuda.cu:1363-1393); an MI355X node is a full
        // xGMI mesh, so there is nothing to toggle per batch size.
        int prev = 0;
        (void)hipGetDevice(&prev);
        for (auto &a : R->ctxs) {
            for (auto &b : R->ctxs) {
                if (a->device == b->device) continue;
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, a->device, b->device) != hipSuccess || !can) {
                    (void)hipGetLastError();
                    continue;
                }
                (void)hipSetDevice(a->device);
                const hipError_t e = hipDeviceEnablePeerAccess(b->device, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    fprintf(stderr, "[ggml-mi355x] peer access %d -> %d: %s\n", a->device, b->device, hipGetErrorString(e));
                (void)hipGetLastError();
                a->peers.push_back(b->device);
            }
        }
        (void)hipSetDevice(prev);
        R->reg.api_version = GGMLABI_API_VERSION;
        R->reg.iface = {rg_name, rg_count, rg_dev, rg_proc};
        R->reg.context = nullptr;
        return R;
    }();
    return *r;
}

int n_devices() { return (int)registry().devs.size(); }
int device_of(int idx) { return registry().ctxs[idx]->device; }
ggml_backend_dev_t dev_handle(int idx) { return registry().devs[idx].get(); }

}  // namespace

extern "C" {

GGML_MI355X_API struct ggml_backend_reg *ggml_backend_mi355x_reg(void) { return &registry().reg; }

GGML_MI355X_API struct ggml_backend_reg *ggml_backend_init(void) { return ggml_backend_mi355x_reg(); }

GGML_MI355X_API int ggml_backend_score(void) { return ggml_mi355x_device_count() > 0 ? 100 : 0; }

}  // extern "C"
