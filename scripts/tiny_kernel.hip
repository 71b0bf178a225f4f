// A one-kernel code object for scripts/parent_probe.py (mode torchinit-tiny):
// does launching ANY kernel outside torch's own code objects, in a process
// where torch initialised the device, set off the multi-process stalls?
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
