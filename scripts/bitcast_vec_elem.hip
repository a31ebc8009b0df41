// Minimal reproducer: ROCm 7.2 clang (AMD clang 22.0.0git, roc-7.2.0 26014) miscompiles
// __builtin_bit_cast of an ext_vector_type element. Both kernels below load ONE dword and store
// it (or undefined registers) for every element:
//   hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S scripts/bitcast_vec_elem.hip -o - | grep global_
// Found in round 5: the stream-K partial stores of mmq8.hip wrote acc0[0] sixteen times.
// The fix there is to store the float values themselves (no bit_cast).
#include <hip/hip_runtime.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void loop_index(const float *in, unsigned *out) {   // stores in[0]*3 sixteen times
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = in[i * 64 + threadIdx.x] * 3.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i * 64 + threadIdx.x] = __builtin_bit_cast(unsigned, acc[i]);
}

__global__ void const_index(const f32x4 *in, unsigned *out) {   // loads a[0] only, stores v[0:3]
    f32x4 a = in[threadIdx.x];
    out[threadIdx.x * 4 + 0] = __builtin_bit_cast(unsigned, a[0]);
    out[threadIdx.x * 4 + 1] = __builtin_bit_cast(unsigned, a[1]);
    out[threadIdx.x * 4 + 2] = __builtin_bit_cast(unsigned, a[2]);
    out[threadIdx.x * 4 + 3] = __builtin_bit_cast(unsigned, a[3]);
}
