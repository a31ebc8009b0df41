// ggml_abi.h — the subset of the ggml backend ABI (API version 1) this plugin implements.
//
// The plugin is loaded by an unmodified ggml (src/ggml-backend-reg.cpp:239-283), so these
// declarations must match the reference layouts field for field:
//   struct ggml_tensor ............... include/ggml.h:614-646
//   enum ggml_op / ggml_type / status  include/ggml.h:339-347, 372-412, 460-560
//   ggml_backend_dev_props / caps .... include/ggml-backend.h:140-159
//   buffer type / buffer / backend /
//   event / device / reg vtables ..... src/ggml-backend-impl.h:17-207
//   struct ggml_hash_set / ggml_cgraph  src/ggml-impl.h:181-212, 311-325 (read for use counts)
// tests/test_abi_layout.py compiles oracle/abi_check.cpp against the reference headers and
// this file side by side and asserts every offset, size and enum value used here agrees.
#pragma once

#include <stddef.h>
#include <stdint.h>

extern "C" {

#define GGMLABI_API_VERSION 1
#define GGMLABI_MAX_DIMS 4
#define GGMLABI_MAX_SRC 10
#define GGMLABI_MAX_OP_PARAMS 64
#define GGMLABI_MAX_NAME 64

enum ggml_status { GGML_STATUS_ALLOC_FAILED = -2, GGML_STATUS_FAILED = -1, GGML_STATUS_SUCCESS = 0, GGML_STATUS_ABORTED = 1 };

// only the op codes this backend inspects (values from include/ggml.h's enum ggml_op)
enum {
    GGMLABI_OP_NONE = 0,
    GGMLABI_OP_DUP = 1,
    GGMLABI_OP_ADD = 2,
    GGMLABI_OP_SUB = 6,
    GGMLABI_OP_MUL = 7,
    GGMLABI_OP_DIV = 8,
    GGMLABI_OP_NORM = 23,
    GGMLABI_OP_MUL_MAT = 28,
    GGMLABI_OP_MUL_MAT_ID = 29,
    GGMLABI_OP_SCALE = 31,
    GGMLABI_OP_CPY = 33,
    GGMLABI_OP_CONT = 34,
    GGMLABI_OP_RESHAPE = 35,
    GGMLABI_OP_VIEW = 36,
    GGMLABI_OP_PERMUTE = 37,
    GGMLABI_OP_TRANSPOSE = 38,
    GGMLABI_OP_GET_ROWS = 39,
    GGMLABI_OP_DIAG_MASK_INF = 43,
    GGMLABI_OP_DIAG_MASK_ZERO = 44,
    GGMLABI_OP_SOFT_MAX = 45,
    GGMLABI_OP_UNARY = 78,
};

// enum ggml_unary_op (include/ggml.h), the value in op_params[0] of a GGML_OP_UNARY node
enum { GGMLABI_UNARY_OP_GELU = 8 };

enum { GGMLABI_TYPE_F32 = 0, GGMLABI_TYPE_F16 = 1, GGMLABI_TYPE_I32 = 26 };

struct ggml_backend_buffer;
struct ggml_backend_buffer_type;
struct ggml_backend_device;
struct ggml_backend_reg;
struct ggml_backend;
struct ggml_backend_event;
struct ggml_cgraph;

struct ggml_tensor {
    int32_t type;
    struct ggml_backend_buffer *buffer;
    int64_t ne[GGMLABI_MAX_DIMS];
    size_t nb[GGMLABI_MAX_DIMS];
    int32_t op;
    int32_t op_params[GGMLABI_MAX_OP_PARAMS / sizeof(int32_t)];
    int32_t flags;
    struct ggml_tensor *src[GGMLABI_MAX_SRC];
    struct ggml_tensor *view_src;
    size_t view_offs;
    void *data;
    char name[GGMLABI_MAX_NAME];
    void *extra;
    char padding[8];
};

// include/ggml.h enum ggml_tensor_flag
enum { GGMLABI_TENSOR_FLAG_OUTPUT = 2 };

// the graph internals the fusion rules read (src/ggml-impl.h:181-212, 311-325): a graph's use
// counts are indexed by the slot of the tensor in visited_hash_set (linear probing from
// ((uintptr_t)t >> 4) % size, occupancy in the `used` bitset of 32-bit words). The scheduler's
// split graphs are views (ggml_graph_view, src/ggml.c:6545-6560) that share the whole graph's
// counts, so a use in another split is still counted.
struct ggml_hash_set {
    size_t size;
    uint32_t *used;
    struct ggml_tensor **keys;
};
struct ggml_cgraph {
    int size;
    int n_nodes;
    int n_leafs;
    struct ggml_tensor **nodes;
    struct ggml_tensor **grads;
    struct ggml_tensor **grad_accs;
    struct ggml_tensor **leafs;
    int32_t *use_counts;
    struct ggml_hash_set visited_hash_set;
    int32_t order;
};

typedef struct ggml_backend_buffer_type *ggml_backend_buffer_type_t;
typedef struct ggml_backend_buffer *ggml_backend_buffer_t;
typedef struct ggml_backend_event *ggml_backend_event_t;
typedef struct ggml_backend *ggml_backend_t;
typedef void *ggml_backend_graph_plan_t;
typedef struct ggml_backend_reg *ggml_backend_reg_t;
typedef struct ggml_backend_device *ggml_backend_dev_t;
typedef uint8_t ggml_guid[16];
typedef ggml_guid *ggml_guid_t;

enum ggml_backend_buffer_usage { GGML_BACKEND_BUFFER_USAGE_ANY = 0, GGML_BACKEND_BUFFER_USAGE_WEIGHTS = 1, GGML_BACKEND_BUFFER_USAGE_COMPUTE = 2 };
enum ggml_backend_dev_type { GGML_BACKEND_DEVICE_TYPE_CPU, GGML_BACKEND_DEVICE_TYPE_GPU, GGML_BACKEND_DEVICE_TYPE_ACCEL };

struct ggml_backend_dev_caps {
    bool async;
    bool host_buffer;
    bool buffer_from_host_ptr;
    bool events;
};

struct ggml_backend_dev_props {
    const char *name;
    const char *description;
    size_t memory_free;
    size_t memory_total;
    enum ggml_backend_dev_type type;
    struct ggml_backend_dev_caps caps;
};

struct ggml_backend_buffer_type_i {
    const char *(*get_name)(ggml_backend_buffer_type_t buft);
    ggml_backend_buffer_t (*alloc_buffer)(ggml_backend_buffer_type_t buft, size_t size);
    size_t (*get_alignment)(ggml_backend_buffer_type_t buft);
    size_t (*get_max_size)(ggml_backend_buffer_type_t buft);
    size_t (*get_alloc_size)(ggml_backend_buffer_type_t buft, const struct ggml_tensor *tensor);
    bool (*is_host)(ggml_backend_buffer_type_t buft);
};

struct ggml_backend_buffer_type {
    struct ggml_backend_buffer_type_i iface;
    ggml_backend_dev_t device;
    void *context;
};

struct ggml_backend_buffer_i {
    void (*free_buffer)(ggml_backend_buffer_t buffer);
    void *(*get_base)(ggml_backend_buffer_t buffer);
    enum ggml_status (*init_tensor)(ggml_backend_buffer_t buffer, struct ggml_tensor *tensor);
    void (*memset_tensor)(ggml_backend_buffer_t buffer, struct ggml_tensor *tensor, uint8_t value, size_t offset, size_t size);
    void (*set_tensor)(ggml_backend_buffer_t buffer, struct ggml_tensor *tensor, const void *data, size_t offset, size_t size);
    void (*get_tensor)(ggml_backend_buffer_t buffer, const struct ggml_tensor *tensor, void *data, size_t offset, size_t size);
    bool (*cpy_tensor)(ggml_backend_buffer_t buffer, const struct ggml_tensor *src, struct ggml_tensor *dst);
    void (*clear)(ggml_backend_buffer_t buffer, uint8_t value);
    void (*reset)(ggml_backend_buffer_t buffer);
};

struct ggml_backend_buffer {
    struct ggml_backend_buffer_i iface;
    ggml_backend_buffer_type_t buft;
    void *context;
    size_t size;
    enum ggml_backend_buffer_usage usage;
};

struct ggml_backend_i {
    const char *(*get_name)(ggml_backend_t backend);
    void (*free)(ggml_backend_t backend);
    void (*set_tensor_async)(ggml_backend_t backend, struct ggml_tensor *tensor, const void *data, size_t offset, size_t size);
    void (*get_tensor_async)(ggml_backend_t backend, const struct ggml_tensor *tensor, void *data, size_t offset, size_t size);
    bool (*cpy_tensor_async)(ggml_backend_t backend_src, ggml_backend_t backend_dst, const struct ggml_tensor *src, struct ggml_tensor *dst);
    void (*synchronize)(ggml_backend_t backend);
    ggml_backend_graph_plan_t (*graph_plan_create)(ggml_backend_t backend, const struct ggml_cgraph *cgraph);
    void (*graph_plan_free)(ggml_backend_t backend, ggml_backend_graph_plan_t plan);
    void (*graph_plan_update)(ggml_backend_t backend, ggml_backend_graph_plan_t plan, const struct ggml_cgraph *cgraph);
    enum ggml_status (*graph_plan_compute)(ggml_backend_t backend, ggml_backend_graph_plan_t plan);
    enum ggml_status (*graph_compute)(ggml_backend_t backend, struct ggml_cgraph *cgraph);
    void (*event_record)(ggml_backend_t backend, ggml_backend_event_t event);
    void (*event_wait)(ggml_backend_t backend, ggml_backend_event_t event);
};

struct ggml_backend {
    ggml_guid_t guid;
    struct ggml_backend_i iface;
    ggml_backend_dev_t device;
    void *context;
};

struct ggml_backend_event {
    struct ggml_backend_device *device;
    void *context;
};

struct ggml_backend_device_i {
    const char *(*get_name)(ggml_backend_dev_t dev);
    const char *(*get_description)(ggml_backend_dev_t dev);
    void (*get_memory)(ggml_backend_dev_t dev, size_t *free, size_t *total);
    enum ggml_backend_dev_type (*get_type)(ggml_backend_dev_t dev);
    void (*get_props)(ggml_backend_dev_t dev, struct ggml_backend_dev_props *props);
    ggml_backend_t (*init_backend)(ggml_backend_dev_t dev, const char *params);
    ggml_backend_buffer_type_t (*get_buffer_type)(ggml_backend_dev_t dev);
    ggml_backend_buffer_type_t (*get_host_buffer_type)(ggml_backend_dev_t dev);
    ggml_backend_buffer_t (*buffer_from_host_ptr)(ggml_backend_dev_t dev, void *ptr, size_t size, size_t max_tensor_size);
    bool (*supports_op)(ggml_backend_dev_t dev, const struct ggml_tensor *op);
    bool (*supports_buft)(ggml_backend_dev_t dev, ggml_backend_buffer_type_t buft);
    bool (*offload_op)(ggml_backend_dev_t dev, const struct ggml_tensor *op);
    ggml_backend_event_t (*event_new)(ggml_backend_dev_t dev);
    void (*event_free)(ggml_backend_dev_t dev, ggml_backend_event_t event);
    void (*event_synchronize)(ggml_backend_dev_t dev, ggml_backend_event_t event);
};

struct ggml_backend_device {
    struct ggml_backend_device_i iface;
    ggml_backend_reg_t reg;
    void *context;
};

struct ggml_backend_reg_i {
    const char *(*get_name)(ggml_backend_reg_t reg);
    size_t (*get_device_count)(ggml_backend_reg_t reg);
    ggml_backend_dev_t (*get_device)(ggml_backend_reg_t reg, size_t index);
    void *(*get_proc_address)(ggml_backend_reg_t reg, const char *name);
};

struct ggml_backend_reg {
    int api_version;
    struct ggml_backend_reg_i iface;
    void *context;
};

struct ggml_backend_feature {
    const char *name;
    const char *value;
};

}  // extern "C"
