// Cost model of the round kernel's primitives on MI355X (one wave per SIMD,
// 157-1250 waves like the round kernel).  Cycles are clock64 (s_memtime)
// ticks, converted with the wall clock (100 MHz) measured alongside.
//   hipcc --offload-arch=gfx950 -O3 costs.hip -o costs && ./costs
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

struct Out {
    unsigned long long cyc, wall, sink;
};

__device__ __forceinline__ void put(Out* o, unsigned long long c, unsigned long long w, unsigned long long s) {
    if (threadIdx.x == 0) o[blockIdx.x] = Out{c, w, s};
}

// dependent integer chain (the rand_r LCG step): 2 VALU per step
__global__ void k_int_chain(int n, Out* o) {
    uint32_t x = threadIdx.x * 7919u + blockIdx.x;
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
#pragma unroll 8
    for (int i = 0; i < n; i++) x = x * 1103515245u + 12345u;
    put(o, clock64() - c0, wall_clock64() - w0, x);
}

// 8 independent integer chains: issue rate
__global__ void k_int_ilp(int n, Out* o) {
    uint32_t x[8];
    for (int j = 0; j < 8; j++) x[j] = threadIdx.x * 7919u + blockIdx.x + j;
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
    for (int i = 0; i < n; i++)
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = x[j] * 1103515245u + 12345u;
    uint32_t s = 0;
    for (int j = 0; j < 8; j++) s ^= x[j];
    put(o, clock64() - c0, wall_clock64() - w0, s);
}

// dependent 64-bit compare-select chain (event-key style)
__global__ void k_u64_chain(int n, Out* o) {
    uint64_t a = threadIdx.x, b = blockIdx.x * 3ull;
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
    for (int i = 0; i < n; i++) {
        const uint64_t m = a < b ? a : b;
        a = m + 0x9E3779B97F4A7C15ull;
        b ^= m;
    }
    put(o, clock64() - c0, wall_clock64() - w0, a ^ b);
}

// dependent f64 division by the RAND_MAX constant (next_double)
__global__ void k_fdiv(int n, Out* o) {
    double x = 1.0 + threadIdx.x;
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
    for (int i = 0; i < n; i++) x = (x + 12345.0) / 2147483647.0;
    put(o, clock64() - c0, wall_clock64() - w0, (unsigned long long)(x * 1e18));
}

// divergent branches: lane-dependent switch, 6 arms of a few instructions
__global__ void k_diverge(int n, Out* o) {
    uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
    for (int i = 0; i < n; i++) {
        switch ((x >> 7) % 6) {
        case 0: x = x * 3u + 1u; break;
        case 1: x = (x ^ 0x5bd1e995u) + 7u; break;
        case 2: x = (x << 3) ^ (x >> 2); break;
        case 3: x = x * 0x27d4eb2du; break;
        case 4: x = ~x + 0x165667b1u; break;
        default: x = (x >> 1) * 5u; break;
        }
    }
    put(o, clock64() - c0, wall_clock64() - w0, x);
}

// clock64 read cost
__global__ void k_clock(int n, Out* o) {
    unsigned long long acc = 0;
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
    for (int i = 0; i < n; i++) acc += clock64();
    put(o, clock64() - c0, wall_clock64() - w0, acc);
}

// LDS dependent chain (per-lane slots, stride 64 like the due list)
__global__ void k_lds_chain(int n, Out* o) {
    __shared__ uint32_t s[64 * 16];
    for (int j = 0; j < 16; j++) s[j * 64 + threadIdx.x] = (j * 5 + 3) & 15;
    __syncthreads();
    uint32_t i = 0;
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
    for (int k = 0; k < n; k++) i = s[i * 64 + threadIdx.x];
    put(o, clock64() - c0, wall_clock64() - w0, i);
}

// dependent random 16-B loads, one chain per lane, over a table of `nel` entries
__global__ void k_chase(const uint4* __restrict__ t, uint64_t nel, int n, Out* o) {
    uint64_t i = ((uint64_t)blockIdx.x * 64 + threadIdx.x) * 2654435761ull % nel;
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
    for (int k = 0; k < n; k++) {
        const uint4 v = t[i];
        i = (((uint64_t)v.y << 32) | v.x) % nel;
    }
    put(o, clock64() - c0, wall_clock64() - w0, i);
}

// dependent returning atomics at random addresses of a `nel`-word table
__global__ void k_atomic(uint32_t* t, uint64_t nel, int n, Out* o) {
    uint64_t i = ((uint64_t)blockIdx.x * 64 + threadIdx.x) * 2654435761ull % nel;
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
    for (int k = 0; k < n; k++) {
        const uint32_t v = atomicAdd(&t[i], 1u);
        i = (i * 6364136223846793005ull + v + 1442695040888963407ull) % nel;
    }
    put(o, clock64() - c0, wall_clock64() - w0, i);
}

static void report(const char* name, const std::vector<Out>& h, int n, double per) {
    double c = 0, w = 0, cm = 0, wm = 0;
    for (const Out& x : h) {
        c += x.cyc; w += x.wall;
        cm = std::max(cm, (double)x.cyc); wm = std::max(wm, (double)x.wall);
    }
    c /= h.size(); w /= h.size();
    const double ghz = c / (w * 10.0);
    printf("%-34s %8.1f cyc/op  %7.1f ns/op (max wave %7.1f ns/op)  [clock64 %.2f GHz]\n", name, c / (n * per),
           w * 10.0 / (n * per), wm * 10.0 / (n * per), ghz);
}

int main() {
    int grids[] = {157, 1250};
    Out* d_o;
    CK(hipMalloc(&d_o, sizeof(Out) * 4096));
    const uint64_t big = (1ull << 30) / 16 * 2;   // 2 GB of 16-B entries (path-table scale)
    const uint64_t mid = (16ull << 20) / 16;      // 16 MB
    uint4* d_t;
    CK(hipMalloc(&d_t, big * 16));
    {
        std::vector<uint4> h(1 << 20);
        std::mt19937_64 rng(7);
        for (uint64_t off = 0; off < big; off += h.size()) {
            for (auto& v : h) {
                const uint64_t r = rng();
                v = make_uint4((uint32_t)r, (uint32_t)(r >> 32), 0, 0);
            }
            CK(hipMemcpy(d_t + off, h.data(), h.size() * 16, hipMemcpyHostToDevice));
        }
    }
    uint32_t* d_a;
    CK(hipMalloc(&d_a, (16ull << 20)));
    CK(hipMemset(d_a, 0, 16ull << 20));
    for (int g : grids) {
        printf("== grid %d blocks x 64 lanes\n", g);
        std::vector<Out> h(g);
        auto run = [&](const char* nm, int n, double per, auto launch) {
            launch();
            CK(hipDeviceSynchronize());
            launch();
            CK(hipMemcpy(h.data(), d_o, sizeof(Out) * g, hipMemcpyDeviceToHost));
            report(nm, h, n, per);
        };
        const int n = 4096;
        run("int LCG step (dependent, 2 VALU)", n, 1, [&] { hipLaunchKernelGGL(k_int_chain, dim3(g), dim3(64), 0, 0, n, d_o); });
        run("int LCG step (8 independent)", n, 8, [&] { hipLaunchKernelGGL(k_int_ilp, dim3(g), dim3(64), 0, 0, n, d_o); });
        run("u64 min/add/xor (dependent)", n, 1, [&] { hipLaunchKernelGGL(k_u64_chain, dim3(g), dim3(64), 0, 0, n, d_o); });
        run("f64 div by RAND_MAX (dependent)", 1024, 1, [&] { hipLaunchKernelGGL(k_fdiv, dim3(g), dim3(64), 0, 0, 1024, d_o); });
        run("6-way divergent switch step", n, 1, [&] { hipLaunchKernelGGL(k_diverge, dim3(g), dim3(64), 0, 0, n, d_o); });
        run("clock64 read", n, 1, [&] { hipLaunchKernelGGL(k_clock, dim3(g), dim3(64), 0, 0, n, d_o); });
        run("LDS dependent load", n, 1, [&] { hipLaunchKernelGGL(k_lds_chain, dim3(g), dim3(64), 0, 0, n, d_o); });
        run("16-B load chain, 16 MB table", 256, 1, [&] { hipLaunchKernelGGL(k_chase, dim3(g), dim3(64), 0, 0, d_t, mid, 256, d_o); });
        run("16-B load chain, 2 GB table", 256, 1, [&] { hipLaunchKernelGGL(k_chase, dim3(g), dim3(64), 0, 0, d_t, big, 256, d_o); });
        run("returning atomicAdd chain, 16 MB", 256, 1, [&] { hipLaunchKernelGGL(k_atomic, dim3(g), dim3(64), 0, 0, d_a, (16ull << 20) / 4, 256, d_o); });
    }
    return 0;
}
