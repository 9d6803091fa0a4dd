// Start-up costs the `blt` CLI pays before its first window (tools/cli_phases.sh): process start to
// main, HIP runtime init (first API call), device context (hipSetDevice + hipFree(0)), first
// allocation, the library's code object load (first launch of a trivial kernel), each in seconds.
//   hipcc -O2 --offload-arch=gfx950 tools/hip_init_probe.cpp -o build/hip_init_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <time.h>

static double now() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

__global__ void nop_kernel(int* p) {
    if (p && threadIdx.x == 0) p[0] = 1;
}

int main() {
    const double t0 = now();
    int n = 0;
    (void)hipGetDeviceCount(&n);
    const double t1 = now();
    (void)hipSetDevice(0);
    (void)hipFree(nullptr);
    const double t2 = now();
    int* d = nullptr;
    (void)hipMalloc(&d, 1 << 20);
    const double t3 = now();
    hipLaunchKernelGGL(nop_kernel, dim3(1), dim3(64), 0, 0, d);
    (void)hipDeviceSynchronize();
    const double t4 = now();
    void* h = nullptr;
    (void)hipHostMalloc(&h, 64 << 20, 0);
    const double t5 = now();
    printf("{\"devices\": %d, \"runtime_init_s\": %.4f, \"context_s\": %.4f, \"malloc_s\": %.4f, "
           "\"first_launch_s\": %.4f, \"pinned_64mib_s\": %.4f}\n", n, t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4);
    return 0;
}
