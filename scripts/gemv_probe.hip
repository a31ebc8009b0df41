// scripts/gemv_probe.hip — measurement probe (not product code): which part of a single
// 9.47 MB mat-vec launch costs the time? Variants over the same bytes (Q4_0 4096x4096 weight
// bytes, 512 workgroups x 512 threads, 64 rotated buffers => HBM-cold), run under
// rocprofv3 --kernel-trace:
//   A  coalesced stream: lane i loads 16 B at 16 i (the hbm_probe floor)
//   B  mat-vec access pattern: one 2304-B row per wave, lane l loads 36 B at 36 l
//      (dwordx4 + dwordx4 + dword)
//   C  B + activation prologue: every workgroup loads a 16 KB vector, writes it to LDS,
//      barrier, then consumes the weights against LDS
//   D  C + wave reduction and one store per row
//   E  coalesced loads into LDS by row (lane i -> 16 B at 16 i of its wave's row), barrier-free
//      per wave, then lanes read their 36-B blocks back from LDS
//   hipcc --offload-arch=gfx950 -O3 scripts/gemv_probe.hip -o scripts/gemv_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); }    \
    } while (0)

constexpr int ROW = 2304;   // Q4_0 row of 4096 values
constexpr int NROWS = 4096;

__global__ __launch_bounds__(512) void k_stream(const uint4 *__restrict__ p, uint32_t *out) {
    const size_t per_wg = (size_t)ROW * NROWS / 16 / gridDim.x;
    const uint4 *b = p + blockIdx.x * per_wg;
    uint32_t acc = 0;
    for (size_t i = threadIdx.x; i < per_wg; i += blockDim.x) {
        const uint4 v = b[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

struct __attribute__((packed, aligned(4))) u4a4 { uint32_t v[4]; };

template <int V>
__global__ __launch_bounds__(512) void k_gemv(const uint8_t *__restrict__ w, const float *__restrict__ x, float *__restrict__ y,
                                              int xrep = 0, int xdiv = 1) {
    x += (size_t)(blockIdx.x % (xrep ? xrep : 1)) * 4096;
    __shared__ float xs[4096];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 8 + wave;
    float4 xa, xb;
    if constexpr (V >= 2 && V != 5 && V != 6) {
        xa = reinterpret_cast<const float4 *>(x)[(threadIdx.x / xdiv) * 2];
        xb = reinterpret_cast<const float4 *>(x)[(threadIdx.x / xdiv) * 2 + 1];
    }
    uint32_t D[9];
    if constexpr (V == 4) {
        __shared__ uint4 wl[8][ROW / 16 + 4];
        const uint4 *src = reinterpret_cast<const uint4 *>(w + (size_t)row * ROW);
        for (int i = lane; i < ROW / 16; i += 64) wl[wave][i] = src[i];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0);
        const uint8_t *p = reinterpret_cast<const uint8_t *>(&wl[wave][0]) + lane * 36;
        for (int i = 0; i < 9; ++i) D[i] = reinterpret_cast<const uint32_t *>(p)[i];
    } else {
        const uint8_t *p = w + (size_t)row * ROW + lane * 36;
        const u4a4 a = *reinterpret_cast<const u4a4 *>(p);
        const u4a4 b = *reinterpret_cast<const u4a4 *>(p + 16);
        D[8] = *reinterpret_cast<const uint32_t *>(p + 32);
        for (int i = 0; i < 4; ++i) { D[i] = a.v[i]; D[4 + i] = b.v[i]; }
    }
    float acc = 0.f;
    if constexpr (V == 5) {           // F: 16 KB of LDS written, no barrier, no x
        xs[threadIdx.x] = (float)D[0];
        for (int i = 0; i < 9; ++i) acc += (float)(D[i] & 0xff) * xs[(threadIdx.x + i) & 4095];
    } else if constexpr (V == 6) {    // G: barrier only
        __syncthreads();
        for (int i = 0; i < 9; ++i) acc += (float)(D[i] & 0xff);
    } else if constexpr (V == 7) {    // H: x in registers, barrier, no LDS
        __syncthreads();
        for (int i = 0; i < 9; ++i) acc += (float)(D[i] & 0xff) * xa.x * xb.y;
    } else if constexpr (V == 8) {    // I: x in registers, no barrier, no LDS
        for (int i = 0; i < 9; ++i) acc += (float)(D[i] & 0xff) * xa.x * xb.y;
    } else if constexpr (V >= 2) {
        reinterpret_cast<float4 *>(xs)[threadIdx.x * 2] = xa;
        reinterpret_cast<float4 *>(xs)[threadIdx.x * 2 + 1] = xb;
        __syncthreads();
        for (int i = 0; i < 9; ++i) acc += (float)(D[i] & 0xff) * xs[lane + 64 * i];
    } else {
        for (int i = 0; i < 9; ++i) acc += (float)(D[i] & 0xff);
    }
    if constexpr (V >= 3 && V != 4) {
        for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d);
        if (lane == 0) y[row] = acc;
    } else {
        if (acc == 1234.5f) y[row] = acc;
    }
}

int main() {
    const size_t bytes = (size_t)ROW * NROWS;
    const int copies = 64;
    std::vector<uint8_t *> bufs(copies);
    for (auto &b : bufs) {
        CK(hipMalloc(&b, bytes));
        CK(hipMemset(b, 1, bytes));
    }
    float *x, *y;
    uint32_t *o;
    CK(hipMalloc(&x, 512 * 4096 * 4));
    CK(hipMemset(x, 0, 512 * 4096 * 4));
    CK(hipMalloc(&y, NROWS * 4));
    CK(hipMalloc(&o, 1 << 16));
    auto run = [&](const char *name, auto launch) {
        for (int i = 0; i < copies; ++i) launch(i);
        CK(hipDeviceSynchronize());
        for (int i = 0; i < 256; ++i) launch(i);
        CK(hipDeviceSynchronize());
        printf("%s done\n", name);
    };
    run("A stream", [&](int i) { hipLaunchKernelGGL(k_stream, dim3(512), dim3(512), 0, 0, reinterpret_cast<const uint4 *>(bufs[i % copies]), o); });
    run("B pattern", [&](int i) { hipLaunchKernelGGL(k_gemv<1>, dim3(512), dim3(512), 0, 0, bufs[i % copies], x, y); });
    run("C prologue", [&](int i) { hipLaunchKernelGGL(k_gemv<2>, dim3(512), dim3(512), 0, 0, bufs[i % copies], x, y); });
    run("D reduce", [&](int i) { hipLaunchKernelGGL(k_gemv<3>, dim3(512), dim3(512), 0, 0, bufs[i % copies], x, y); });
    run("C rep512 (own x copy per WG)", [&](int i) { hipLaunchKernelGGL(k_gemv<2>, dim3(512), dim3(512), 0, 0, bufs[i % copies], x, y, 512, 1); });
    run("C rep8 (one x copy per XCD)", [&](int i) { hipLaunchKernelGGL(k_gemv<2>, dim3(512), dim3(512), 0, 0, bufs[i % copies], x, y, 8, 1); });
    run("C div8 (2 KB of x per WG)", [&](int i) { hipLaunchKernelGGL(k_gemv<2>, dim3(512), dim3(512), 0, 0, bufs[i % copies], x, y, 0, 8); });
    run("F lds only", [&](int i) { hipLaunchKernelGGL(k_gemv<5>, dim3(512), dim3(512), 0, 0, bufs[i % copies], x, y, 0, 1); });
    run("G barrier only", [&](int i) { hipLaunchKernelGGL(k_gemv<6>, dim3(512), dim3(512), 0, 0, bufs[i % copies], x, y, 0, 1); });
    run("H x regs + barrier", [&](int i) { hipLaunchKernelGGL(k_gemv<7>, dim3(512), dim3(512), 0, 0, bufs[i % copies], x, y, 0, 1); });
    run("I x regs", [&](int i) { hipLaunchKernelGGL(k_gemv<8>, dim3(512), dim3(512), 0, 0, bufs[i % copies], x, y, 0, 1); });
    run("E coalesced+lds", [&](int i) { hipLaunchKernelGGL(k_gemv<4>, dim3(512), dim3(512), 0, 0, bufs[i % copies], x, y); });
    return 0;
}
