// Back-to-back launch cost on this MI355X: what a gated no-op launch of the selection
// chain pays. 200 launches per variant, HIP events around them, average per launch:
// "host" = enqueued back to back from an idle stream (the host's launch rate can
// bound it), "gpu" = enqueued behind a 3 ms spin kernel, so the queue is full when
// they run and only the GPU side is timed.
// Build: hipcc --offload-arch=gfx950 -O3 tools/launchbench.hip -o /tmp/launchbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Big {   // a SelWS-sized argument block
    void* p[48];
    long long n[8];
};

__global__ void k_empty() {}
__global__ void k_empty_big(Big b) {
    if (b.n[0] == 12345) b.n[1] = 0;   // keep the argument alive
}
__global__ void k_one_load(int* flag) {
    if (*flag) flag[1] = 1;   // the flag is 0: every block exits after one load
}
// the shape of a gated selection kernel: every field of a large argument block read
// (scalar loads), a flag behind a pointer from it, 1024 threads, 12 KB of LDS
__global__ void __launch_bounds__(1024) k_gate_like(Big b) {
    __shared__ int lds[3072];
    long long acc = 0;
#pragma unroll
    for (int i = 0; i < 48; ++i) acc += reinterpret_cast<long long>(b.p[i]);
    const int* flag = reinterpret_cast<const int*>(b.p[0]);
    if (*flag) {
        lds[threadIdx.x] = (int)acc;
        __syncthreads();
        reinterpret_cast<int*>(b.p[1])[threadIdx.x] = lds[(threadIdx.x + 1) & 1023];
    }
}
__global__ void k_two_loads(const int* table, int* flag) {
    const int t = table[blockIdx.x & 63] & 63;
    if (flag[t]) flag[100] = 1;
}

__global__ void k_spin(long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
}

template <class F>
static float timeit(F launch, int reps, hipStream_t s, bool behind_spin = false) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 20; ++i) launch();
    CK(hipStreamSynchronize(s));
    if (behind_spin) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 300000000LL);   // ~3 ms at 100 MHz clock64
    CK(hipEventRecord(a, s));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / reps;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    int* flag;
    CK(hipMalloc(&flag, 4096 * sizeof(int)));
    CK(hipMemset(flag, 0, 4096 * sizeof(int)));
    Big big{};
    for (int i = 0; i < 48; ++i) big.p[i] = flag + 2048;   // a zero flag; p[1] is never written
    const int reps = 200;
    for (int spin = 0; spin < 2; ++spin)
        for (int grid : {1, 256, 4096}) {
            printf("{\"mode\": \"%s\", \"grid\": %d, \"empty_us\": %.2f, \"empty_bigarg_us\": %.2f, "
                   "\"one_load_us\": %.2f, \"two_loads_us\": %.2f, \"gate_like_us\": %.2f}\n", spin ? "gpu" : "host",
                   grid,
                   timeit([&] { hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s); }, reps, s, spin),
                   timeit([&] { hipLaunchKernelGGL(k_empty_big, dim3(grid), dim3(256), 0, s, big); }, reps, s, spin),
                   timeit([&] { hipLaunchKernelGGL(k_one_load, dim3(grid), dim3(256), 0, s, flag); }, reps, s, spin),
                   timeit([&] { hipLaunchKernelGGL(k_two_loads, dim3(grid), dim3(256), 0, s, flag, flag + 64); }, reps,
                          s, spin),
                   timeit([&] { hipLaunchKernelGGL(k_gate_like, dim3(grid), dim3(1024), 0, s, big); }, reps, s, spin));
        }
    CK(hipFree(flag));
    return 0;
}
