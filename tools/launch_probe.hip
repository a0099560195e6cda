// Launch cost of a no-op workgroup set by its resources: what k_nth_select costs when
// no tensor needs the replay (54 workgroups of 512 threads, 151 KB LDS, 384 B/lane
// scratch). Each variant runs after a plain kernel, 400 times, timed with events.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/_launch_probe tools/launch_probe.hip
//   tools/_launch_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_prev(int* flag) {
    if (threadIdx.x == 0 && flag[blockIdx.x] == 12345) flag[blockIdx.x] = 1;
}

// variants: LDS on/off, scratch on/off; the work is never taken (flag is 0)
template <bool kLds, bool kScratch>
__global__ void __launch_bounds__(512) k_var(int* flag, int idx) {
    if (flag[blockIdx.x] != 7) return;
    if constexpr (kLds) {
        __shared__ unsigned long long big[150 * 1024 / 8];
        big[threadIdx.x * 37 % (150 * 128)] = idx;
        __syncthreads();
        flag[blockIdx.x + 1000] = (int)big[(threadIdx.x + idx) % (150 * 128)];
    }
    if constexpr (kScratch) {
        volatile int a[96];
        for (int i = 0; i < 96; ++i) a[i] = i * idx;
        flag[blockIdx.x + 2000] = a[(threadIdx.x + idx) % 96];
    }
}

template <typename F>
static float timed(F launch, hipStream_t s, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 20; ++i) launch();
    (void)hipEventRecord(a, s);
    for (int i = 0; i < reps; ++i) launch();
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms * 1000.f / reps;
}

int main() {
    int* flag = nullptr;
    CK(hipMalloc(&flag, 4096 * sizeof(int)));
    CK(hipMemset(flag, 0, 4096 * sizeof(int)));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const int reps = 400;
    const dim3 g(54), b(512);
    const float base = timed([&] { hipLaunchKernelGGL(k_prev, g, dim3(64), 0, s, flag); }, s, reps);
    auto pair = [&](auto kern, const char* name) {
        const float us = timed([&] {
            hipLaunchKernelGGL(k_prev, g, dim3(64), 0, s, flag);
            hipLaunchKernelGGL(kern, g, b, 0, s, flag, 3);
        }, s, reps);
        std::printf("%-22s %7.2f us per pair, %7.2f us over the plain kernel alone\n", name, us, us - base);
    };
    std::printf("plain kernel alone     %7.2f us\n", base);
    pair(k_var<false, false>, "no-op");
    pair(k_var<true, false>, "no-op + 150 KB LDS");
    pair(k_var<false, true>, "no-op + scratch");
    pair(k_var<true, true>, "no-op + LDS + scratch");
    CK(hipStreamSynchronize(s));
    CK(hipFree(flag));
    return 0;
}
