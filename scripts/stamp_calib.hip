// scripts/stamp_calib.hip — calibrates the s_memrealtime workgroup stamps used by
// GGML_MI355X_STAMPS: how long do an empty barrier phase, 256 dependent VALU ops and an LDS
// round trip take when 512 x 256-thread workgroups run at once? (probe, not product code)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void calib(unsigned long long *st, float *out, int n) {
    __shared__ float lds[256];
    const bool s = threadIdx.x == 0;
    if (s) st[blockIdx.x * 8 + 0] = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (s) st[blockIdx.x * 8 + 1] = __builtin_amdgcn_s_memrealtime();
    float v = lds[(threadIdx.x + 1) & 255];
    for (int i = 0; i < n; ++i) v = v * 1.0001f + 0.5f;
    if (s) st[blockIdx.x * 8 + 2] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (s) st[blockIdx.x * 8 + 3] = __builtin_amdgcn_s_memrealtime();
    if (v == 12345.f) out[blockIdx.x] = v;
}

int main() {
    unsigned long long *st;
    float *out;
    hipMalloc(&st, 8 * 4096 * 8);
    hipMalloc(&out, 4096 * 4);
    for (int n : {0, 256, 1024}) {
        for (int rep = 0; rep < 20; ++rep) hipLaunchKernelGGL(calib, dim3(512), dim3(256), 0, 0, st, out, n);
        hipDeviceSynchronize();
        std::vector<unsigned long long> h(512 * 8);
        hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
        std::vector<double> a, b, c;
        for (int w = 0; w < 512; ++w) {
            a.push_back((double)(h[w * 8 + 1] - h[w * 8 + 0]) * 10);
            b.push_back((double)(h[w * 8 + 2] - h[w * 8 + 1]) * 10);
            c.push_back((double)(h[w * 8 + 3] - h[w * 8 + 2]) * 10);
        }
        std::sort(a.begin(), a.end());
        std::sort(b.begin(), b.end());
        std::sort(c.begin(), c.end());
        printf("n=%4d  median ns: lds+barrier %.0f   %d dependent fma %.0f   barrier %.0f\n", n, a[256], n, b[256], c[256]);
    }
    return 0;
}
