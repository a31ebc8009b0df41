// scripts/pkfma_mfma_repro.hip — minimal reproducer (measurement, not product code) for the
// packed-f32 fault of DESIGN.md §4.2: does a v_pk_fma_f32 lose its write on some lanes when it
// executes while v_mfma_i32_32x32x32_i8 instructions on OTHER registers are in flight?
//
// Every wave runs ITER rounds of: one MFMA (a dependent accumulator chain on registers the
// VALU never touches) followed by PK packed fmas on an independent register pair, inside one asm
// statement so the compiler neither reorders nor pads it. The packed chain p = p * 1 + 1 counts
// rounds exactly in f32; at the end every lane must hold ITER * PK (+ start). Lanes that do not
// are counted per 16-lane quarter. The same kernel with v_fma_f32 (two scalar fmas per packed
// one) is the control. No data dependence exists between the MFMAs and the fmas, so the
// compiler's gfx950 hazard model (scripts/mfma_hazard_scan.py) asks for no wait states.
//   hipcc --offload-arch=gfx950 -O3 scripts/pkfma_mfma_repro.hip -o scripts/pkfma_mfma_repro && scripts/pkfma_mfma_repro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); }     \
    } while (0)

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int ITER = 4096;

template <bool PACKED, int PK>
__global__ __launch_bounds__(256) void repro(float *out, int *mf) {
    i32x4 a = {(int)threadIdx.x, 1, 2, 3}, b = {1, 1, 1, 1};
    i32x16 acc = {};
    f32x2 p = {0.f, 0.f};
    const f32x2 one = {1.f, 1.f};
    for (int it = 0; it < ITER; ++it) {
        if constexpr (PACKED) {
            if constexpr (PK == 4)
                asm volatile(
                    "v_mfma_i32_32x32x32_i8 %0, %2, %3, %0\n\t"
                    "v_pk_fma_f32 %1, %1, %4, %4\n\tv_pk_fma_f32 %1, %1, %4, %4\n\t"
                    "v_pk_fma_f32 %1, %1, %4, %4\n\tv_pk_fma_f32 %1, %1, %4, %4"
                    : "+v"(acc), "+v"(p) : "v"(a), "v"(b), "v"(one));
            else
                asm volatile(
                    "v_mfma_i32_32x32x32_i8 %0, %2, %3, %0\n\t"
                    "v_pk_fma_f32 %1, %1, %4, %4\n\tv_pk_fma_f32 %1, %1, %4, %4\n\t"
                    "v_pk_fma_f32 %1, %1, %4, %4\n\tv_pk_fma_f32 %1, %1, %4, %4\n\t"
                    "v_pk_fma_f32 %1, %1, %4, %4\n\tv_pk_fma_f32 %1, %1, %4, %4\n\t"
                    "v_pk_fma_f32 %1, %1, %4, %4\n\tv_pk_fma_f32 %1, %1, %4, %4"
                    : "+v"(acc), "+v"(p) : "v"(a), "v"(b), "v"(one));
        } else {
            float x = p.x, y = p.y;
            if constexpr (PK == 4)
                asm volatile(
                    "v_mfma_i32_32x32x32_i8 %0, %3, %4, %0\n\t"
                    "v_fma_f32 %1, %1, 1.0, 1.0\n\tv_fma_f32 %2, %2, 1.0, 1.0\n\t"
                    "v_fma_f32 %1, %1, 1.0, 1.0\n\tv_fma_f32 %2, %2, 1.0, 1.0\n\t"
                    "v_fma_f32 %1, %1, 1.0, 1.0\n\tv_fma_f32 %2, %2, 1.0, 1.0\n\t"
                    "v_fma_f32 %1, %1, 1.0, 1.0\n\tv_fma_f32 %2, %2, 1.0, 1.0"
                    : "+v"(acc), "+v"(x), "+v"(y) : "v"(a), "v"(b));
            else
                asm volatile(
                    "v_mfma_i32_32x32x32_i8 %0, %3, %4, %0\n\t"
                    "v_fma_f32 %1, %1, 1.0, 1.0\n\tv_fma_f32 %2, %2, 1.0, 1.0\n\t"
                    "v_fma_f32 %1, %1, 1.0, 1.0\n\tv_fma_f32 %2, %2, 1.0, 1.0\n\t"
                    "v_fma_f32 %1, %1, 1.0, 1.0\n\tv_fma_f32 %2, %2, 1.0, 1.0\n\t"
                    "v_fma_f32 %1, %1, 1.0, 1.0\n\tv_fma_f32 %2, %2, 1.0, 1.0\n\t"
                    "v_fma_f32 %1, %1, 1.0, 1.0\n\tv_fma_f32 %2, %2, 1.0, 1.0\n\t"
                    "v_fma_f32 %1, %1, 1.0, 1.0\n\tv_fma_f32 %2, %2, 1.0, 1.0\n\t"
                    "v_fma_f32 %1, %1, 1.0, 1.0\n\tv_fma_f32 %2, %2, 1.0, 1.0\n\t"
                    "v_fma_f32 %1, %1, 1.0, 1.0\n\tv_fma_f32 %2, %2, 1.0, 1.0"
                    : "+v"(acc), "+v"(x), "+v"(y) : "v"(a), "v"(b));
            p.x = x;
            p.y = y;
        }
    }
    asm volatile("s_nop 15\n\ts_nop 15" :::);   // (the last MFMA's results are read below)
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    out[2 * g] = p.x;
    out[2 * g + 1] = p.y;
    int s = 0;
    for (int i = 0; i < 16; ++i) s += acc[i];
    mf[g] = s;   // keeps the MFMA chain live
}

template <bool PACKED, int PK>
static void run(const char *name, int blocks) {
    const int n = blocks * 256;
    float *d;
    int *m;
    CK(hipMalloc(&d, 2 * n * sizeof(float)));
    CK(hipMalloc(&m, n * sizeof(int)));
    float *h = (float *)malloc(2 * n * sizeof(float));
    long bad[4] = {0, 0, 0, 0}, runs = 0;
    for (int r = 0; r < 20; ++r) {
        hipLaunchKernelGGL((repro<PACKED, PK>), dim3(blocks), dim3(256), 0, 0, d, m);
        CK(hipGetLastError());
        CK(hipMemcpy(h, d, 2 * n * sizeof(float), hipMemcpyDeviceToHost));
        const float want = (float)ITER * PK;
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < 2; ++j)
                if (h[2 * i + j] != want) ++bad[(i & 63) >> 4];
        ++runs;
    }
    printf("%-28s %d waves x %d rounds x %d runs: wrong lanes by quarter 0-15 %ld  16-31 %ld  32-47 %ld  48-63 %ld\n", name,
           n / 64, ITER, (int)runs, bad[0], bad[1], bad[2], bad[3]);
    CK(hipFree(d));
    CK(hipFree(m));
    free(h);
}

int main() {
    const int blocks = 256 * 4;   // 4 workgroups of 4 waves per CU
    run<true, 4>("packed, 4 per MFMA", blocks);
    run<true, 8>("packed, 8 per MFMA", blocks);
    run<false, 4>("scalar pairs, 4 per MFMA", blocks);
    run<false, 8>("scalar pairs, 8 per MFMA", blocks);
    return 0;
}
