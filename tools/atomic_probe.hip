// Same-address returning atomics from many waves (diagnostic): is one global counter the cost of a
// kernel in which every wave appends its result with atomicAdd(counter, 1)?  Launches N one-wave blocks
// whose lane 0 does one returning atomicAdd on a single counter (and, "spread", on one of 64 counters
// 256 B apart), timed with HIP events; a no-atomic launch of the same grid is the floor.
// hipcc --offload-arch=gfx950 -O3 tools/atomic_probe.hip -o tools/atomic_probe && ./tools/atomic_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void append_kernel(int* ctr, int* out, int mode) {
    if (threadIdx.x != 0) return;
    int v = blockIdx.x;
    if (mode == 1) v = atomicAdd(ctr, 1);
    if (mode == 2) v = atomicAdd(ctr + 64 * (blockIdx.x & 63), 1);
    out[blockIdx.x] = v;
}

int main() {
    int *ctr, *out;
    const int nmax = 1 << 18;
    if (hipMalloc(&ctr, 64 * 64 * sizeof(int)) || hipMalloc(&out, nmax * sizeof(int))) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[3] = {"none", "single", "spread64"};
    for (int n = 1024; n <= nmax; n *= 4)
        for (int mode = 0; mode < 3; ++mode) {
            float best = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                hipMemset(ctr, 0, 64 * 64 * sizeof(int));
                hipEventRecord(e0);
                append_kernel<<<n, 64>>>(ctr, out, mode);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            printf("waves %7d  %-9s %8.1f us  (%.1f ns per wave)\n", n, names[mode], best * 1e3, best * 1e6 / n);
        }
    return 0;
}
