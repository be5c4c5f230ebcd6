// Dependent-load latency on MI355X: pointer chase over working sets of
// different sizes, repeated across kernel launches (does the L2 keep lines
// across a kernel boundary?), plus a returning-atomic chain.
//   hipcc --offload-arch=gfx950 -O3 latency.hip -o latency && ./latency
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void chase(const uint32_t* __restrict__ next, int hops, uint32_t start, unsigned long long* out) {
    uint32_t i = start;
    const unsigned long long t0 = clock64();
    for (int k = 0; k < hops; k++) i = __builtin_nontemporal_load(&next[i]) , i = next[i];
    const unsigned long long t1 = clock64();
    out[0] = t1 - t0;
    out[1] = i;
}

__global__ void chase_plain(const uint32_t* __restrict__ next, int hops, uint32_t start, unsigned long long* out) {
    uint32_t i = start;
    const unsigned long long t0 = clock64();
    for (int k = 0; k < hops; k++) i = next[i];
    const unsigned long long t1 = clock64();
    out[0] = t1 - t0;
    out[1] = i;
}

__global__ void atomic_chain(uint32_t* ctr, int n, unsigned long long* out) {
    uint32_t v = 0;
    const unsigned long long t0 = clock64();
    for (int k = 0; k < n; k++) v = atomicAdd(&ctr[(v & 0) * 32], 1u + (v & 0));
    const unsigned long long t1 = clock64();
    out[0] = t1 - t0;
    out[1] = v;
}

int main() {
    const size_t line = 128 / 4;   // u32 per 128-B line
    std::vector<size_t> sizes = {16u << 10, 256u << 10, 2u << 20, 16u << 20, 128u << 20, 1024u << 20};
    unsigned long long* d_out;
    CK(hipMalloc(&d_out, 16));
    const int hops = 2000;
    for (size_t S : sizes) {
        const size_t nl = S / 128;
        std::vector<uint32_t> perm(nl);
        for (size_t i = 0; i < nl; i++) perm[i] = (uint32_t)i;
        std::mt19937 rng(1);
        std::shuffle(perm.begin() + 1, perm.end(), rng);
        std::vector<uint32_t> h(nl * line, 0);
        for (size_t i = 0; i < nl; i++) h[perm[i] * line] = perm[(i + 1) % nl] * line;
        uint32_t* d;
        CK(hipMalloc(&d, S));
        CK(hipMemcpy(d, h.data(), S, hipMemcpyHostToDevice));
        unsigned long long r[2];
        printf("S=%8zu KB:", S >> 10);
        for (int rep = 0; rep < 3; rep++) {
            hipLaunchKernelGGL(chase_plain, dim3(1), dim3(1), 0, 0, d, hops, 0u, d_out);
            CK(hipMemcpy(r, d_out, 16, hipMemcpyDeviceToHost));
            printf("  launch%d %6.0f cyc/hop", rep, (double)r[0] / hops);
        }
        printf("\n");
        CK(hipFree(d));
    }
    uint32_t* ctr;
    CK(hipMalloc(&ctr, 4096));
    CK(hipMemset(ctr, 0, 4096));
    unsigned long long r[2];
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(atomic_chain, dim3(1), dim3(1), 0, 0, ctr, 1000, d_out);
        CK(hipMemcpy(r, d_out, 16, hipMemcpyDeviceToHost));
        printf("returning atomicAdd chain: %.0f cyc/op\n", (double)r[0] / 1000);
    }
    return 0;
}
