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
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ggml-mi355x.h"
#include "dispatch.h"
#include "ggml_abi.h"

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
    bool ok = false;
};

const GgmlBase &ggml_base() {
    static GgmlBase b = [] {
        GgmlBase g;
        g.buffer_init = reinterpret_cast<decltype(g.buffer_init)>(dlsym(RTLD_DEFAULT, "ggml_backend_buffer_init"));
        g.graph_n_nodes = reinterpret_cast<decltype(g.graph_n_nodes)>(dlsym(RTLD_DEFAULT, "ggml_graph_n_nodes"));
        g.graph_node = reinterpret_cast<decltype(g.graph_node)>(dlsym(RTLD_DEFAULT, "ggml_graph_node"));
        g.nbytes = reinterpret_cast<decltype(g.nbytes)>(dlsym(RTLD_DEFAULT, "ggml_nbytes"));
        g.ok = g.buffer_init && g.graph_n_nodes && g.graph_node && g.nbytes;
        return g;
    }();
    return b;
}

bool debug_on() {
    static const bool on = getenv("GGML_MI355X_DEBUG") != nullptr;
    return on;
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
    std::string name, desc;
    struct ggml_backend_buffer_type buft {};
    std::string buft_name;
};

struct BufferCtx {
    int device;
    void *base;
};

struct BackendCtx {
    int device;
    hipStream_t stream = nullptr;
    std::string name;
    Scratch scratch;
};

const char *BUFT_TAG = "MI355X";

DeviceCtx *dev_ctx(ggml_backend_dev_t d) { return static_cast<DeviceCtx *>(d->context); }

bool is_our_buft(ggml_backend_buffer_type_t buft);

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
}

void buf_set(ggml_backend_buffer_t b, struct ggml_tensor *t, const void *data, size_t off, size_t n) {
    auto *c = static_cast<BufferCtx *>(b->context);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipMemcpyAsync(static_cast<uint8_t *>(t->data) + off, data, n, hipMemcpyHostToDevice, nullptr));
    HIP_OK(hipStreamSynchronize(nullptr));
}

void buf_get(ggml_backend_buffer_t b, const struct ggml_tensor *t, void *data, size_t off, size_t n) {
    auto *c = static_cast<BufferCtx *>(b->context);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipMemcpyAsync(data, static_cast<const uint8_t *>(t->data) + off, n, hipMemcpyDeviceToHost, nullptr));
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
    return true;
}

void buf_clear(ggml_backend_buffer_t b, uint8_t v) {
    auto *c = static_cast<BufferCtx *>(b->context);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipMemsetAsync(c->base, v, b->size, nullptr));
    HIP_OK(hipStreamSynchronize(nullptr));
}

const struct ggml_backend_buffer_i BUFFER_IFACE = {
    buf_free, buf_base, buf_init_tensor, buf_memset, buf_set, buf_get, buf_cpy, buf_clear, nullptr,
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
    return ggml_base().buffer_init(bt, BUFFER_IFACE, new BufferCtx{d->device, p}, size);
}

size_t buft_align(ggml_backend_buffer_type_t) { return 128; }
size_t buft_max(ggml_backend_buffer_type_t) { return SIZE_MAX; }
size_t buft_alloc_size(ggml_backend_buffer_type_t, const struct ggml_tensor *t) { return ggml_base().nbytes(t); }
bool buft_is_host(ggml_backend_buffer_type_t) { return false; }

const struct ggml_backend_buffer_type_i BUFT_IFACE = {
    buft_name, buft_alloc, buft_align, buft_max, buft_alloc_size, buft_is_host,
};

bool is_our_buft(ggml_backend_buffer_type_t buft) { return buft && buft->iface.get_name == buft_name; }

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
    HIP_OK(hipStreamDestroy(c->stream));
    delete c;
    delete b;
}

void be_set_async(ggml_backend_t b, struct ggml_tensor *t, const void *data, size_t off, size_t n) {
    BackendCtx *c = be_ctx(b);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipMemcpyAsync(static_cast<uint8_t *>(t->data) + off, data, n, hipMemcpyHostToDevice, c->stream));
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
    HIP_OK(hipSetDevice(cs->device));
    if (cs->device == cd->device) {
        HIP_OK(hipMemcpyAsync(dst->data, src->data, n, hipMemcpyDeviceToDevice, cs->stream));
    } else {
        HIP_OK(hipMemcpyPeerAsync(dst->data, cd->device, src->data, cs->device, n, cs->stream));
    }
    if (cs != cd) {
        hipEvent_t ev;
        HIP_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIP_OK(hipEventRecord(ev, cs->stream));
        HIP_OK(hipSetDevice(cd->device));
        HIP_OK(hipStreamWaitEvent(cd->stream, ev, 0));
        HIP_OK(hipEventDestroy(ev));   // destruction is deferred by the runtime until completion
    }
    return true;
}

void be_sync(ggml_backend_t b) {
    BackendCtx *c = be_ctx(b);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipStreamSynchronize(c->stream));
}

enum ggml_status be_graph_compute(ggml_backend_t b, struct ggml_cgraph *g) {
    BackendCtx *c = be_ctx(b);
    const GgmlBase &gb = ggml_base();
    if (!gb.ok) return GGML_STATUS_FAILED;
    HIP_OK(hipSetDevice(c->device));
    const int n = gb.graph_n_nodes(g);
    for (int i = 0; i < n; ++i) {
        struct ggml_tensor *node = gb.graph_node(g, i);
        if (is_empty(node) || is_view_op(node->op)) continue;
        int rc;
        GraphOp gop;
        if (node->op == GGMLABI_OP_MUL_MAT && is_hot_quant(node->src[0]->type)) {
            rc = mul_mat(tv(node->src[0]), tv(node->src[1]), tv(node), c->stream, c->scratch);
        } else if (node->op == GGMLABI_OP_MUL_MAT_ID) {
            rc = mul_mat_id(tv(node->src[0]), tv(node->src[1]), tv(node->src[2]), tv(node), c->stream, c->scratch);
        } else if (node->op == GGMLABI_OP_GET_ROWS) {
            rc = get_rows(tv(node->src[0]), tv(node->src[1]), tv(node), c->stream);
        } else if (node->op == GGMLABI_OP_CPY && is_hot_quant(node->type)) {
            rc = quantize(tv(node->src[0]), tv(node), c->stream);   // node is the view of src[1]
        } else if (graph_op_of(node, gop)) {
            rc = run_graph_op(gop, c->stream);
        } else {
            fprintf(stderr, "[ggml-mi355x] unsupported op %d in graph (node %s)\n", node->op, node->name);
            return GGML_STATUS_FAILED;
        }
        if (rc != GGML_MI355X_OK) {
            fprintf(stderr, "[ggml-mi355x] node %s (op %d) failed: %s\n", node->name, node->op, ggml_mi355x_strerror(rc));
            return GGML_STATUS_FAILED;
        }
    }
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
    p->caps.host_buffer = false;
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
    auto *b = new ggml_backend();
    b->guid = &BACKEND_GUID;
    b->iface = BACKEND_IFACE;
    b->device = d;
    b->context = c;
    return b;
}

ggml_backend_buffer_type_t dv_buft(ggml_backend_dev_t d) { return &dev_ctx(d)->buft; }

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
bool dv_supports_op(ggml_backend_dev_t, const struct ggml_tensor *op) {
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
        case GGMLABI_OP_MUL_MAT_ID:
            return op->type == GGMLABI_TYPE_F32 && supports_mm_operands(op->src[0], op->src[1]) &&
                   op->src[2]->type == GGMLABI_TYPE_I32 && op->src[2]->ne[0] * op->src[2]->ne[1] <= 65535;
        // GET_ROWS of the hot quant types / f32 (dequantized rows, bit-exact), like get_rows_cuda
        case GGMLABI_OP_GET_ROWS:
            return check_get_rows(tv(op->src[0]), tv(op->src[1]), tv(op)) == GGML_MI355X_OK;
        // f32 -> Q4_0 / Q8_0 copies (the reference GPU's cpy_f32_q subset of these types)
        case GGMLABI_OP_CPY:
            if (is_hot_quant(op->type)) return check_quantize(tv(op->src[0]), tv(op)) == GGML_MI355X_OK;
            break;
        default:
            break;
    }
    // the f32 ops of the GPT-2 graph around the matmuls (graph_ops.hip)
    GraphOp g;
    return graph_op_of(op, g) && check_graph_op(g) == GGML_MI355X_OK;
}

bool dv_supports_buft(ggml_backend_dev_t d, ggml_backend_buffer_type_t bt) {
    return is_our_buft(bt) && static_cast<DeviceCtx *>(bt->context)->device == dev_ctx(d)->device;
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
    nullptr, nullptr,
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

void *rg_proc(ggml_backend_reg_t, const char *name) {
    if (strcmp(name, "ggml_backend_get_features") == 0) return reinterpret_cast<void *>(rg_features);
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
        for (int i = 0; i < n; ++i) {
            hipDeviceProp_t p;
            if (hipGetDeviceProperties(&p, i) != hipSuccess || strncmp(p.gcnArchName, "gfx950", 6) != 0) continue;
            auto dc = std::make_unique<DeviceCtx>();
            dc->device = i;
            dc->name = std::string("MI355X") + std::to_string(R->ctxs.size());
            dc->desc = p.name;
            dc->buft_name = std::string(BUFT_TAG) + std::to_string(R->ctxs.size());
            auto dev = std::make_unique<ggml_backend_device>();
            dev->iface = DEVICE_IFACE;
            dev->reg = &R->reg;
            dev->context = dc.get();
            dc->buft.iface = BUFT_IFACE;
            dc->buft.device = dev.get();
            dc->buft.context = dc.get();
            R->ctxs.push_back(std::move(dc));
            R->devs.push_back(std::move(dev));
        }
        R->reg.api_version = GGMLABI_API_VERSION;
        R->reg.iface = {rg_name, rg_count, rg_dev, rg_proc};
        R->reg.context = nullptr;
        return R;
    }();
    return *r;
}

}  // namespace

extern "C" {

GGML_MI355X_API struct ggml_backend_reg *ggml_backend_mi355x_reg(void) { return &registry().reg; }

GGML_MI355X_API struct ggml_backend_reg *ggml_backend_init(void) { return ggml_backend_mi355x_reg(); }

GGML_MI355X_API int ggml_backend_score(void) { return ggml_mi355x_device_count() > 0 ? 100 : 0; }

}  // extern "C"
