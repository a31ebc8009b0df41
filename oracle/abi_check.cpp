// oracle/abi_check.cpp — TEST INFRASTRUCTURE (never linked into the product).
//
// Compiled twice by tests/test_abi_layout.py:
//   -DSIDE_REF  against the reference's own headers (include/ggml.h, include/ggml-backend.h,
//               src/ggml-backend-impl.h, src/ggml-impl.h)
//   -DSIDE_OURS against ggml-gfx906_amd/csrc/ggml_abi.h, the plugin's restatement
// Both print "name value" lines for every struct size, field offset and enum value the plugin
// relies on; the test requires the two listings to be identical, so the plugin's view of the
// ggml backend ABI (version 1) is pinned to the reference's, field for field.
#include <cstddef>
#include <cstdio>

#if defined(SIDE_REF)
#include "ggml.h"
#include "ggml-backend.h"
#include "ggml-backend-impl.h"
#include "ggml-impl.h"
#define E(ours, ref) std::printf("enum %s %d\n", #ours, (int)(ref));
#define API_VERSION GGML_BACKEND_API_VERSION
#include <cstdlib>
// ggml-impl.h's static inline hash helpers reference ggml_abort; this listing never calls them
extern "C" void ggml_abort(const char *, int, const char *, ...) { std::abort(); }
#elif defined(SIDE_OURS)
#include "ggml_abi.h"
#define E(ours, ref) std::printf("enum %s %d\n", #ours, (int)(ours));
#define API_VERSION GGMLABI_API_VERSION
#else
#error "define SIDE_REF or SIDE_OURS"
#endif

#define S(t) std::printf("sizeof %s %zu\n", #t, sizeof(struct t));
#define F(t, f) std::printf("offsetof %s.%s %zu\n", #t, #f, offsetof(struct t, f));

int main() {
    std::printf("api_version %d\n", (int)API_VERSION);
    E(GGMLABI_OP_NONE, GGML_OP_NONE)
    E(GGMLABI_OP_DUP, GGML_OP_DUP)
    E(GGMLABI_OP_ADD, GGML_OP_ADD)
    E(GGMLABI_OP_SUB, GGML_OP_SUB)
    E(GGMLABI_OP_MUL, GGML_OP_MUL)
    E(GGMLABI_OP_DIV, GGML_OP_DIV)
    E(GGMLABI_OP_NORM, GGML_OP_NORM)
    E(GGMLABI_OP_SCALE, GGML_OP_SCALE)
    E(GGMLABI_OP_CONT, GGML_OP_CONT)
    E(GGMLABI_OP_DIAG_MASK_INF, GGML_OP_DIAG_MASK_INF)
    E(GGMLABI_OP_DIAG_MASK_ZERO, GGML_OP_DIAG_MASK_ZERO)
    E(GGMLABI_OP_SOFT_MAX, GGML_OP_SOFT_MAX)
    E(GGMLABI_OP_UNARY, GGML_OP_UNARY)
    E(GGMLABI_UNARY_OP_GELU, GGML_UNARY_OP_GELU)
    E(GGMLABI_OP_MUL_MAT, GGML_OP_MUL_MAT)
    E(GGMLABI_OP_MUL_MAT_ID, GGML_OP_MUL_MAT_ID)
    E(GGMLABI_OP_CPY, GGML_OP_CPY)
    E(GGMLABI_OP_RESHAPE, GGML_OP_RESHAPE)
    E(GGMLABI_OP_VIEW, GGML_OP_VIEW)
    E(GGMLABI_OP_PERMUTE, GGML_OP_PERMUTE)
    E(GGMLABI_OP_TRANSPOSE, GGML_OP_TRANSPOSE)
    E(GGMLABI_OP_GET_ROWS, GGML_OP_GET_ROWS)
    E(GGMLABI_TENSOR_FLAG_OUTPUT, GGML_TENSOR_FLAG_OUTPUT)
    E(GGMLABI_TYPE_F32, GGML_TYPE_F32)
    E(GGMLABI_TYPE_F16, GGML_TYPE_F16)
    E(GGMLABI_TYPE_I32, GGML_TYPE_I32)
    E(GGML_STATUS_ALLOC_FAILED, GGML_STATUS_ALLOC_FAILED)
    E(GGML_STATUS_FAILED, GGML_STATUS_FAILED)
    E(GGML_STATUS_SUCCESS, GGML_STATUS_SUCCESS)
    E(GGML_STATUS_ABORTED, GGML_STATUS_ABORTED)
    E(GGML_BACKEND_BUFFER_USAGE_WEIGHTS, GGML_BACKEND_BUFFER_USAGE_WEIGHTS)
    E(GGML_BACKEND_BUFFER_USAGE_COMPUTE, GGML_BACKEND_BUFFER_USAGE_COMPUTE)
    E(GGML_BACKEND_DEVICE_TYPE_CPU, GGML_BACKEND_DEVICE_TYPE_CPU)
    E(GGML_BACKEND_DEVICE_TYPE_GPU, GGML_BACKEND_DEVICE_TYPE_GPU)

    S(ggml_tensor)
    F(ggml_tensor, type) F(ggml_tensor, buffer) F(ggml_tensor, ne) F(ggml_tensor, nb) F(ggml_tensor, op)
    F(ggml_tensor, op_params) F(ggml_tensor, flags) F(ggml_tensor, src) F(ggml_tensor, view_src)
    F(ggml_tensor, view_offs) F(ggml_tensor, data) F(ggml_tensor, name) F(ggml_tensor, extra)

    S(ggml_hash_set)
    F(ggml_hash_set, size) F(ggml_hash_set, used) F(ggml_hash_set, keys)
    S(ggml_cgraph)
    F(ggml_cgraph, size) F(ggml_cgraph, n_nodes) F(ggml_cgraph, n_leafs) F(ggml_cgraph, nodes) F(ggml_cgraph, grads)
    F(ggml_cgraph, grad_accs) F(ggml_cgraph, leafs) F(ggml_cgraph, use_counts) F(ggml_cgraph, visited_hash_set)
    F(ggml_cgraph, order)

    S(ggml_backend_dev_caps)
    F(ggml_backend_dev_caps, async) F(ggml_backend_dev_caps, host_buffer)
    F(ggml_backend_dev_caps, buffer_from_host_ptr) F(ggml_backend_dev_caps, events)
    S(ggml_backend_dev_props)
    F(ggml_backend_dev_props, name) F(ggml_backend_dev_props, description) F(ggml_backend_dev_props, memory_free)
    F(ggml_backend_dev_props, memory_total) F(ggml_backend_dev_props, type) F(ggml_backend_dev_props, caps)

    S(ggml_backend_buffer_type_i)
    F(ggml_backend_buffer_type_i, get_name) F(ggml_backend_buffer_type_i, alloc_buffer)
    F(ggml_backend_buffer_type_i, get_alignment) F(ggml_backend_buffer_type_i, get_max_size)
    F(ggml_backend_buffer_type_i, get_alloc_size) F(ggml_backend_buffer_type_i, is_host)
    S(ggml_backend_buffer_type)
    F(ggml_backend_buffer_type, iface) F(ggml_backend_buffer_type, device) F(ggml_backend_buffer_type, context)

    S(ggml_backend_buffer_i)
    F(ggml_backend_buffer_i, free_buffer) F(ggml_backend_buffer_i, get_base) F(ggml_backend_buffer_i, init_tensor)
    F(ggml_backend_buffer_i, memset_tensor) F(ggml_backend_buffer_i, set_tensor) F(ggml_backend_buffer_i, get_tensor)
    F(ggml_backend_buffer_i, cpy_tensor) F(ggml_backend_buffer_i, clear) F(ggml_backend_buffer_i, reset)
    S(ggml_backend_buffer)
    F(ggml_backend_buffer, iface) F(ggml_backend_buffer, buft) F(ggml_backend_buffer, context)
    F(ggml_backend_buffer, size) F(ggml_backend_buffer, usage)

    S(ggml_backend_i)
    F(ggml_backend_i, get_name) F(ggml_backend_i, free) F(ggml_backend_i, set_tensor_async)
    F(ggml_backend_i, get_tensor_async) F(ggml_backend_i, cpy_tensor_async) F(ggml_backend_i, synchronize)
    F(ggml_backend_i, graph_plan_create) F(ggml_backend_i, graph_plan_free) F(ggml_backend_i, graph_plan_update)
    F(ggml_backend_i, graph_plan_compute) F(ggml_backend_i, graph_compute) F(ggml_backend_i, event_record)
    F(ggml_backend_i, event_wait)
    S(ggml_backend)
    F(ggml_backend, guid) F(ggml_backend, iface) F(ggml_backend, device) F(ggml_backend, context)
    S(ggml_backend_event)
    F(ggml_backend_event, device) F(ggml_backend_event, context)

    S(ggml_backend_device_i)
    F(ggml_backend_device_i, get_name) F(ggml_backend_device_i, get_description) F(ggml_backend_device_i, get_memory)
    F(ggml_backend_device_i, get_type) F(ggml_backend_device_i, get_props) F(ggml_backend_device_i, init_backend)
    F(ggml_backend_device_i, get_buffer_type) F(ggml_backend_device_i, get_host_buffer_type)
    F(ggml_backend_device_i, buffer_from_host_ptr) F(ggml_backend_device_i, supports_op)
    F(ggml_backend_device_i, supports_buft) F(ggml_backend_device_i, offload_op) F(ggml_backend_device_i, event_new)
    F(ggml_backend_device_i, event_free) F(ggml_backend_device_i, event_synchronize)
    S(ggml_backend_device)
    F(ggml_backend_device, iface) F(ggml_backend_device, reg) F(ggml_backend_device, context)

    S(ggml_backend_reg_i)
    F(ggml_backend_reg_i, get_name) F(ggml_backend_reg_i, get_device_count) F(ggml_backend_reg_i, get_device)
    F(ggml_backend_reg_i, get_proc_address)
    S(ggml_backend_reg)
    F(ggml_backend_reg, api_version) F(ggml_backend_reg, iface) F(ggml_backend_reg, context)
    S(ggml_backend_feature)
    F(ggml_backend_feature, name) F(ggml_backend_feature, value)
    return 0;
}
