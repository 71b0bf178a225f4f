// A one-kernel code object for scripts/parent_probe.py (mode torchinit-tiny):
// does launching ANY kernel outside torch's own code objects, in a process
// where torch initialised the device, set off the multi-process stalls?
// Build (in-tree, tools/ is git-ignored but travels with gpurun):
//   hipcc --offload-arch=gfx950 -O2 -shared -fPIC -o tools/libtiny_kernel.so scripts/tiny_kernel.hip
#include <hip/hip_runtime.h>

__global__ void k_tiny_add(float *d, const float *s, unsigned long n)
{
    const unsigned long i = (unsigned long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        d[i] += s[i];
    }
}

extern "C" int tiny_add(float *d, const float *s, unsigned long n)
{
    hipLaunchKernelGGL(k_tiny_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, d, s, n);
    return (int)hipDeviceSynchronize();
}

// the same with this build's access pattern: one wave per workgroup, one
// 16-B non-temporal load of each operand and one non-temporal store per lane
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(64) k_tiny_add_nt(u32x4 *d, const u32x4 *s, unsigned long n)
{
    const unsigned long i = (unsigned long)blockIdx.x * 64 + threadIdx.x;
    if (i < n) {
        u32x4 a = __builtin_nontemporal_load(s + i), b = __builtin_nontemporal_load(d + i);
        float fa[4], fb[4];
        __builtin_memcpy(fa, &a, 16);
        __builtin_memcpy(fb, &b, 16);
        for (int k = 0; k < 4; k++) {
            fb[k] += fa[k];
        }
        __builtin_memcpy(&b, fb, 16);
        __builtin_nontemporal_store(b, d + i);
    }
}

extern "C" int tiny_add_nt(float *d, const float *s, unsigned long n)
{
    const unsigned long nv = n / 4;
    hipLaunchKernelGGL(k_tiny_add_nt, dim3((unsigned)((nv + 63) / 64)), dim3(64), 0, 0,
                       (u32x4*)d, (const u32x4*)s, nv);
    return (int)hipDeviceSynchronize();
}
