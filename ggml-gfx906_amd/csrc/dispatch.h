// dispatch.h — internal host interface between the ggml backend glue (backend.cpp), the
// direct C API and the kernel launchers.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "qmm_args.h"

namespace mi355x {

struct TensorView {
    int type;
    void *data;
    int64_t ne[4];
    size_t nb[4];
};

// grow-only device scratch owned by one stream user
struct Scratch {
    void *ptr = nullptr;
    size_t cap = 0;
    void *get(size_t bytes, hipStream_t st);
    ~Scratch();
};

int type_blck(int t);
int type_bytes(int t);
bool is_hot_quant(int t);

int check_mul_mat(const TensorView &a, const TensorView &b, const TensorView &d);
int check_mul_mat_id(const TensorView &as, const TensorView &b, const TensorView &ids, const TensorView &d);

int mul_mat(const TensorView &a, const TensorView &b, const TensorView &d, hipStream_t st, Scratch &scratch);
int mul_mat_id(const TensorView &as, const TensorView &b, const TensorView &ids, const TensorView &d, hipStream_t st,
               Scratch &scratch);
int dequantize(int type, const void *src, float *dst, int64_t n, hipStream_t st);
int check_get_rows(const TensorView &a, const TensorView &rows, const TensorView &d);
int get_rows(const TensorView &a, const TensorView &rows, const TensorView &d, hipStream_t st);
int check_quantize(const TensorView &src, const TensorView &d);
int quantize(const TensorView &src, const TensorView &d, hipStream_t st);

}  // namespace mi355x
