// scripts/hbm_probe.hip — measurement probe (not product code): how fast can one launch
// stream B bytes from HBM on MI355X, as a function of B and the grid shape? Gives the floor
// a GEMV of the same byte count can reach. Rotates over enough buffers to stay HBM-cold.
//   hipcc --offload-arch=gfx950 -O3 scripts/hbm_probe.hip -o scripts/hbm_probe && scripts/hbm_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

// each workgroup streams `per_wg` bytes with dwordx4 loads, UNROLL loads in flight per lane
template <int UNROLL>
__global__ void stream_read(const uint4 *__restrict__ p, size_t per_wg_vec, uint32_t *out) {
    const uint4 *base = p + (size_t)blockIdx.x * per_wg_vec;
    uint32_t acc = 0;
    for (size_t i = threadIdx.x; i < per_wg_vec; i += (size_t)blockDim.x * UNROLL) {
        uint4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const size_t j = i + (size_t)u * blockDim.x;
            v[u] = j < per_wg_vec ? base[j] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;   // keep the loads alive
}

// the same stream with the non-temporal policy (global_load_dwordx4 ... nt): whole lines per
// wave instruction
template <int UNROLL>
__global__ void stream_read_nt(const uint4 *__restrict__ p, size_t per_wg_vec, uint32_t *out) {
    const uint4 *base = p + (size_t)blockIdx.x * per_wg_vec;
    uint32_t acc = 0;
    for (size_t i = threadIdx.x; i < per_wg_vec; i += (size_t)blockDim.x * UNROLL) {
        uint4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const size_t j = i + (size_t)u * blockDim.x;
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(base + (j < per_wg_vec ? j : 0)));
            v[u] = make_uint4(t[0], t[1], t[2], t[3]);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// LDS-DMA stream: every wave moves 1-KiB pieces (16 B per lane) into its own LDS ring of RING
// pieces, keeping RING - 1 in flight, and touches one dword of each landed piece. AUX: cache
// policy of the DMA (0 default, 2 nt).
typedef __attribute__((address_space(3))) void *lds_ptr_t;
template <int RING, int AUX>
__global__ __launch_bounds__(256) void stream_lds_dma(const uint8_t *__restrict__ p, size_t per_wg, uint32_t *out) {
    __shared__ __align__(16) uint8_t ring[4][RING][1024];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint8_t *base = p + (size_t)blockIdx.x * per_wg;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, (uint32_t)per_wg, 0x00020000);
    const int n_pieces = (int)(per_wg / 1024);
    uint32_t acc = 0;
    int issued = 0;
    for (int k = wave; k < n_pieces && issued < RING - 1; k += 4, ++issued)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)ring[wave][issued % RING], 16, (uint32_t)(k * 1024 + lane * 16), 0, 0, AUX);
    int done = 0;
    for (int k = wave; k < n_pieces; k += 4, ++done) {
        const int kn = k + 4 * (RING - 1);
        if (kn < n_pieces) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)ring[wave][(done + RING - 1) % RING], 16, (uint32_t)(kn * 1024 + lane * 16), 0, 0, AUX);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RING - 1) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        acc ^= reinterpret_cast<const uint32_t *>(ring[wave][done % RING])[lane];
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

struct __attribute__((packed, aligned(2))) u4a2 { uint32_t v[4]; };

// same stream, but every 16-byte load is shifted by `off` bytes (2 = Q6_K-like misalignment)
__global__ void stream_read_off(const uint8_t *__restrict__ p, size_t per_wg_vec, int off, uint32_t *out) {
    const uint8_t *base = p + (size_t)blockIdx.x * per_wg_vec * 16 + off;
    uint32_t acc = 0;
    for (size_t i = threadIdx.x; i < per_wg_vec - 1; i += (size_t)blockDim.x * 4) {
        u4a2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t j = i + (size_t)u * blockDim.x;
            if (j < per_wg_vec - 1) v[u] = *reinterpret_cast<const u4a2 *>(base + j * 16);
            else v[u] = u4a2{{0, 0, 0, 0}};
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc ^= v[u].v[0] ^ v[u].v[1] ^ v[u].v[2] ^ v[u].v[3];
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ void empty_kernel(uint32_t *out) {
    if (threadIdx.x == 12345) out[0] = 1;
}

// the bare stream under a per-grid kernel name, so a rocprofv3 kernel trace separates the grids
template <int TAG>
__global__ void stream_read_tag(const uint4 *__restrict__ p, size_t per_wg_vec, uint32_t *out) {
    const uint4 *base = p + (size_t)blockIdx.x * per_wg_vec;
    uint32_t acc = 0;
    for (size_t i = threadIdx.x; i < per_wg_vec; i += (size_t)blockDim.x * 4) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t j = i + (size_t)u * blockDim.x;
            v[u] = j < per_wg_vec ? base[j] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main(int argc, char **argv) {
    if (argc > 1 && argv[1][0] == 's') {
        // single launches of a bare 9,469,952-B stream (one Q4_K 4096 x 4096 matrix), 64 rotated
        // copies (HBM-cold, > the 256 MiB Infinity Cache), 128 launches per grid, one sync each:
        // for rocprofv3 --kernel-trace --stats, the floor beside the mat-vec's single launches
        // (scripts/prof_singles.py) on the same basis
        const size_t bytes = 9469952 / 16 * 16;
        const int copies = 64;
        std::vector<uint4 *> bufs(copies);
        for (auto &b : bufs) { CK(hipMalloc(&b, bytes)); CK(hipMemset(b, 1, bytes)); }
        uint32_t *o;
        CK(hipMalloc(&o, 1 << 20));
        auto go = [&](auto kern, int wgs) {
            const size_t per = bytes / 16 / wgs;
            for (int i = 0; i < 128 + copies; ++i) {
                hipLaunchKernelGGL(kern, dim3(wgs), dim3(512), 0, 0, bufs[i % copies], per, o);
                CK(hipDeviceSynchronize());
            }
        };
        go(stream_read_tag<256>, 256);
        go(stream_read_tag<512>, 512);
        go(stream_read_tag<1024>, 1024);
        go(stream_read_tag<2048>, 2048);
        printf("done\n");
        return 0;
    }
    {
        uint32_t *o;
        CK(hipMalloc(&o, 64));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        for (int th : {64, 256, 512, 1024}) {
            for (int wgs : {256, 512, 1024, 2048, 4096}) {
                for (int i = 0; i < 64; ++i) hipLaunchKernelGGL(empty_kernel, dim3(wgs), dim3(th), 0, 0, o);
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(a, 0));
                for (int i = 0; i < 512; ++i) hipLaunchKernelGGL(empty_kernel, dim3(wgs), dim3(th), 0, 0, o);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                printf("empty kernel threads=%4d wgs=%5d waves=%6d  back-to-back %6.2f us/launch\n", th, wgs, wgs * th / 64, ms * 1e3 / 512);
            }
        }
        if (argc > 1 && argv[1][0] == 'e') return 0;
    }
    if (argc > 1 && argv[1][0] == 'n') {   // 576 MiB, two buffers alternating: plain vs nt vs LDS-DMA
        const size_t bytes = 603979776;
        uint8_t *bufs[2];
        uint32_t *o;
        for (auto &b : bufs) { CK(hipMalloc(&b, bytes)); CK(hipMemset(b, 1, bytes)); }
        CK(hipMalloc(&o, 1 << 20));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        auto run = [&](const char *name, auto launch) {
            for (int i = 0; i < 4; ++i) launch(bufs[i & 1]);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a, 0));
            for (int i = 0; i < 20; ++i) launch(bufs[i & 1]);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("%-40s %7.0f GB/s\n", name, bytes * 20 / (ms * 1e-3) / 1e9);
        };
        for (int rep = 0; rep < 2; ++rep) {
            for (int wgs : {2048, 4096}) {
                const size_t per = bytes / 16 / wgs;
                char nm[64];
                snprintf(nm, sizeof nm, "plain dwordx4 x4, 512 thr, %d wgs", wgs);
                run(nm, [&](uint8_t *p) { hipLaunchKernelGGL(stream_read<4>, dim3(wgs), dim3(512), 0, 0, (const uint4 *)p, per, o); });
                snprintf(nm, sizeof nm, "nt    dwordx4 x4, 512 thr, %d wgs", wgs);
                run(nm, [&](uint8_t *p) { hipLaunchKernelGGL(stream_read_nt<4>, dim3(wgs), dim3(512), 0, 0, (const uint4 *)p, per, o); });
            }
            for (int wgs : {512, 1024, 2048}) {
                const size_t per = bytes / wgs;
                char nm[64];
                snprintf(nm, sizeof nm, "lds-dma ring 8 default, %d wgs", wgs);
                run(nm, [&](uint8_t *p) { hipLaunchKernelGGL((stream_lds_dma<8, 0>), dim3(wgs), dim3(256), 0, 0, p, per, o); });
                snprintf(nm, sizeof nm, "lds-dma ring 8 nt, %d wgs", wgs);
                run(nm, [&](uint8_t *p) { hipLaunchKernelGGL((stream_lds_dma<8, 2>), dim3(wgs), dim3(256), 0, 0, p, per, o); });
                snprintf(nm, sizeof nm, "lds-dma ring 16 nt, %d wgs", wgs);
                run(nm, [&](uint8_t *p) { hipLaunchKernelGGL((stream_lds_dma<16, 2>), dim3(wgs), dim3(256), 0, 0, p, per, o); });
            }
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'a') {
        const size_t bytes = 603979776;   // 576 MiB
        uint8_t *buf;
        uint32_t *o;
        CK(hipMalloc(&buf, bytes + 64));
        CK(hipMalloc(&o, 1 << 20));
        CK(hipMemset(buf, 1, bytes + 64));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        for (int off : {0, 2, 4, 8, 0}) {
            const int wgs = 4096;
            const size_t per = bytes / 16 / wgs;
            hipLaunchKernelGGL(stream_read_off, dim3(wgs), dim3(256), 0, 0, buf, per, off, o);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a, 0));
            for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(stream_read_off, dim3(wgs), dim3(256), 0, 0, buf, per, off, o);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("576 MiB stream, 16-B loads at offset %d: %.0f GB/s\n", off, bytes * 10 / (ms * 1e-3) / 1e9);
        }
        return 0;
    }
    const size_t sizes[] = {9469952 / 16 * 16, 25362432, 37748736, 100663296};
    const int threads_opts[] = {256, 512};
    const int wg_opts[] = {256, 512, 1024, 2048};
    uint32_t *out;
    CK(hipMalloc(&out, 1 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (size_t bytes : sizes) {
        const int copies = (int)std::max<size_t>(4, (size_t)(700ull << 20) / bytes);
        std::vector<uint4 *> bufs(copies);
        for (auto &b : bufs) {
            CK(hipMalloc(&b, bytes));
            CK(hipMemset(b, 1, bytes));
        }
        for (int th : threads_opts) {
            for (int wgs : wg_opts) {
                const size_t per_wg_vec = bytes / 16 / wgs;
                auto launch = [&](int i) {
                    hipLaunchKernelGGL(stream_read<4>, dim3(wgs), dim3(th), 0, 0, bufs[i % copies], per_wg_vec, out);
                };
                for (int i = 0; i < copies; ++i) launch(i);
                CK(hipDeviceSynchronize());
                // per-launch duration with events around single launches (median of 64)
                std::vector<float> ts;
                for (int i = 0; i < 64; ++i) {
                    CK(hipEventRecord(e0, 0));
                    launch(i);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    ts.push_back(ms * 1e3f);
                }
                std::sort(ts.begin(), ts.end());
                // back-to-back throughput over 256 launches
                CK(hipEventRecord(e0, 0));
                for (int i = 0; i < 256; ++i) launch(i);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double b2b_us = ms * 1e3 / 256;
                printf("bytes=%10zu threads=%d wgs=%5d  single median %7.2f us (%6.0f GB/s)   back-to-back %7.2f us/launch (%6.0f GB/s)\n",
                       bytes, th, wgs, ts[32], bytes / (ts[32] * 1e-6) / 1e9, b2b_us, bytes / (b2b_us * 1e-6) / 1e9);
            }
        }
        for (auto &b : bufs) CK(hipFree(b));
    }
    return 0;
}
