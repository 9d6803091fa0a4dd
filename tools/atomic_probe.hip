// Throughput of device-scope atomics on one address (the tickets and list counters of the
// kernels), against the same grids without them and with the atomics spread over 64 lines.
//   hipcc -O3 --offload-arch=gfx950 tools/atomic_probe.hip -o build/atomic_probe && build/atomic_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

// mode 0: no atomic (tile = blockIdx); 1: one ticket per workgroup on one word; 2: on one of 64 words
__global__ void grid_kernel(uint32_t* ctr, uint32_t* out, int mode) {
    __shared__ uint32_t s;
    if (threadIdx.x == 0) {
        uint32_t t = blockIdx.x;
        if (mode == 1) t = atomicAdd(ctr, 1u);
        else if (mode == 2) t = atomicAdd(ctr + 32u * (blockIdx.x & 63u), 1u);
        s = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// persistent: 256 workgroups claim tickets until `total` are gone, one at a time
__global__ void persist_kernel(uint32_t* ctr, uint32_t* out, uint32_t total) {
    __shared__ uint32_t s;
    for (;;) {
        if (threadIdx.x == 0) s = atomicAdd(ctr, 1u);
        __syncthreads();
        const uint32_t t = s;
        __syncthreads();
        if (t >= total) break;
        if (threadIdx.x == 0) out[t] = blockIdx.x;
    }
}

int main() {
    uint32_t *ctr, *out;
    CK(hipMalloc(&ctr, 64 * 32 * 4));
    CK(hipMalloc(&out, 4u << 20));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const unsigned grids[] = {2048, 8192, 32768, 131072};
    for (int mode = 0; mode < 3; ++mode) {
        for (unsigned g : grids) {
            float best = 1e9f;
            for (int r = 0; r < 5; ++r) {
                CK(hipMemset(ctr, 0, 64 * 32 * 4));
                CK(hipEventRecord(a));
                hipLaunchKernelGGL(grid_kernel, dim3(g), dim3(256), 0, 0, ctr, out, mode);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (ms < best) best = ms;
            }
            printf("{\"probe\": \"grid\", \"mode\": %d, \"workgroups\": %u, \"us\": %.1f, \"ns_per_wg\": %.2f}\n", mode, g,
                   best * 1e3f, best * 1e6f / g);
        }
    }
    for (unsigned total : {32768u, 131072u}) {
        float best = 1e9f;
        for (int r = 0; r < 5; ++r) {
            CK(hipMemset(ctr, 0, 64 * 32 * 4));
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(persist_kernel, dim3(256), dim3(1024), 0, 0, ctr, out, total);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (ms < best) best = ms;
        }
        printf("{\"probe\": \"persist\", \"tickets\": %u, \"us\": %.1f, \"ns_per_ticket\": %.2f}\n", total, best * 1e3f,
               best * 1e6f / total);
    }
    return 0;
}
