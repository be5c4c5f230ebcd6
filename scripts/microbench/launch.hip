// Launch-to-launch time of back-to-back kernels in a captured HIP graph
// (157 blocks x 64 lanes, like the round kernel), against a persistent
// kernel that separates its rounds with a device-wide barrier.
//   hipcc --offload-arch=gfx950 -O3 launch.hip -o launch && ./launch
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kGrid = 157, kRounds = 64;

// empty round
__global__ void k_empty(int i) {}

// one dependent load and one store per lane (the round's first and last memory ops)
__global__ void k_touch(const unsigned* __restrict__ a, unsigned* __restrict__ b, int i) {
    const int t = blockIdx.x * 64 + threadIdx.x;
    b[t] = a[t] + (unsigned)i;
}

// every block reads all blocks' shares of the previous round (the ticketless fold)
__global__ void k_fold(const unsigned long long* __restrict__ parts, unsigned long long* __restrict__ mine, int i) {
    unsigned long long m = ~0ull;
    if (i > 0)
        for (int j = threadIdx.x; j < kGrid; j += 64) {
            const unsigned long long v = parts[((i - 1) & 1) * kGrid + j];
            m = v < m ? v : m;
        }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(m, off, 64);
        m = o < m ? o : m;
    }
    if (threadIdx.x == 0) mine[(i & 1) * kGrid + blockIdx.x] = m + blockIdx.x;
}

// kRounds rounds in one launch: a device-wide barrier between rounds
// (arrive: one atomic per block; wait: poll the counter)
__global__ void k_persistent(unsigned* __restrict__ count, unsigned long long* __restrict__ stamps) {
    for (int r = 0; r < kRounds; r++) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __atomic_fetch_add(count, 1u, __ATOMIC_RELEASE);
            const unsigned target = (unsigned)(r + 1) * gridDim.x;
            while (__hip_atomic_load(count, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            }
            if (blockIdx.x == 0) stamps[r] = wall_clock64();
        }
        __syncthreads();
    }
}

template <class F>
static double graph_us(hipStream_t s, F enqueue) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    enqueue();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 3; w++) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e0, s));
    const int reps = 20;
    for (int w = 0; w < reps; w++) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return ms * 1e3 / (reps * kRounds);
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    unsigned *a, *b, *count;
    unsigned long long *parts, *stamps;
    CK(hipMalloc(&a, kGrid * 64 * 4));
    CK(hipMalloc(&b, kGrid * 64 * 4));
    CK(hipMalloc(&count, 4));
    CK(hipMalloc(&parts, 2 * kGrid * 8));
    CK(hipMalloc(&stamps, kRounds * 8));
    CK(hipMemset(a, 0, kGrid * 64 * 4));
    CK(hipMemset(parts, 0, 2 * kGrid * 8));
    printf("graph of %d empty kernels:        %6.2f us per kernel\n", kRounds,
           graph_us(s, [&] { for (int i = 0; i < kRounds; i++) hipLaunchKernelGGL(k_empty, dim3(kGrid), dim3(64), 0, s, i); }));
    printf("graph of %d load+store kernels:   %6.2f us per kernel\n", kRounds,
           graph_us(s, [&] { for (int i = 0; i < kRounds; i++) hipLaunchKernelGGL(k_touch, dim3(kGrid), dim3(64), 0, s, a, b, i); }));
    printf("graph of %d share-fold kernels:   %6.2f us per kernel\n", kRounds,
           graph_us(s, [&] { for (int i = 0; i < kRounds; i++) hipLaunchKernelGGL(k_fold, dim3(kGrid), dim3(64), 0, s, parts, parts, i); }));
    // persistent kernel with a grid barrier per round
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    double best = 1e9;
    for (int rep = 0; rep < 5; rep++) {
        CK(hipMemset(count, 0, 4));
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(k_persistent, dim3(kGrid), dim3(64), 0, s, count, stamps);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned long long h[kRounds];
        CK(hipMemcpy(h, stamps, sizeof(h), hipMemcpyDeviceToHost));
        const double per = (h[kRounds - 1] - h[0]) * 10.0 / 1e3 / (kRounds - 1);   // 100 MHz wall clock -> us
        if (per < best) best = per;
        if (rep == 4) printf("persistent kernel, grid barrier:   %6.2f us per round (launch incl. %.1f us total)\n", best, ms * 1e3);
    }
    return 0;
}
