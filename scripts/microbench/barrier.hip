// Per-round cost of the seam a persistent round kernel needs, against the
// kernel boundary it would replace (157 blocks x 64 lanes, like the round
// kernel at 10 k hosts).  Rounds are chained: every block's round r+1 starts
// only once every block's round r share is visible.
//   P1 tagged shares: lane 0 of each block stores {value, tag} as one 16-B
//      write-through (sc1) store, drains it; every block polls all shares
//      (lane k: shares k, k+64, k+128, 16-B sc1 loads) until every tag is r.
//   P2 P1 + a dependent hand-off: before its share each lane stores a 16-B
//      record (sc1) into another block's slot; after the poll each lane loads
//      its own slot (sc1), as the round's calendar reads would.
//   P3 P2, with a skew: block b spins b % 8 * 0.25 us before publishing.
//   hipcc --offload-arch=gfx950 -O3 barrier.hip -o barrier && ./barrier
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kGrid = 157, kRounds = 256;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st16_sc1(void* p, uint4 v) {
    const u32x4 x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
}
__device__ __forceinline__ uint4 ld16_sc1(const void* p) {
    u32x4 x;
    asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(p) : "memory");
    return make_uint4(x[0], x[1], x[2], x[3]);
}

template <int MODE>
__global__ __launch_bounds__(64) void k_pers(uint4* __restrict__ shares, uint4* __restrict__ slots,
                                             unsigned long long* __restrict__ stamps, unsigned tag0,
                                             unsigned* __restrict__ bad) {
    const unsigned lane = threadIdx.x, b = blockIdx.x;
    unsigned acc = 0;
    for (int r = 0; r < kRounds; r++) {
        const unsigned tag = tag0 + (unsigned)r;
        if (MODE >= 2) {
            // hand-off: this lane's record for lane `lane` of block (b + 37) % grid
            const unsigned d = (b + 37u) % kGrid;
            st16_sc1(&slots[((size_t)(r & 1) * kGrid + d) * 64 + lane], make_uint4(tag, b, lane, acc));
        }
        if (MODE >= 3) {
            const unsigned long long t0 = wall_clock64();
            while (wall_clock64() - t0 < (unsigned long long)(b % 8) * 25) {}
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // parity slots: a block can run one round ahead of a slow poller, never two
        uint4* sh = shares + (size_t)(r & 1) * kGrid;
        if (lane == 0) st16_sc1(&sh[b], make_uint4(b, r, acc, tag));
        // poll every block's share of round r
        const unsigned long long t0 = wall_clock64();
        for (;;) {
            bool ok = true;
            for (unsigned j = lane; j < (unsigned)kGrid; j += 64) {
                const uint4 s = ld16_sc1(&sh[j]);
                ok = ok && s.w == tag;
                acc += s.z;
            }
            if (__ballot(!ok) == 0) break;
            if (wall_clock64() - t0 > 200000000ull) { atomicOr(bad, 1u); return; }   // 2 s
        }
        if (MODE >= 2) {
            const uint4 v = ld16_sc1(&slots[((size_t)(r & 1) * kGrid + b) * 64 + lane]);
            if (v.x != tag) atomicOr(bad, 2u);
            acc += v.y;
        }
        if (b == 0 && lane == 0) stamps[r] = wall_clock64();
    }
    if (acc == 0xFFFFFFFFu) slots[0] = make_uint4(acc, 0, 0, 0);
}

template <int MODE>
static void run(hipStream_t s, uint4* shares, uint4* slots, unsigned long long* stamps, unsigned* bad,
                unsigned& tag0, const char* name) {
    double best = 1e9;
    for (int rep = 0; rep < 5; rep++) {
        hipLaunchKernelGGL(k_pers<MODE>, dim3(kGrid), dim3(64), 0, s, shares, slots, stamps, tag0, bad);
        CK(hipStreamSynchronize(s));
        tag0 += kRounds + 1;
        unsigned long long h[kRounds];
        CK(hipMemcpy(h, stamps, sizeof(h), hipMemcpyDeviceToHost));
        const double per = (h[kRounds - 1] - h[8]) * 10.0 / 1e3 / (kRounds - 9);   // 100 MHz wall clock
        if (per < best) best = per;
    }
    unsigned hb = 0;
    CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
    printf("%-52s %6.2f us per round%s\n", name, best, hb ? "  (FAILED: stale or timeout)" : "");
    CK(hipMemset(bad, 0, 4));
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    uint4 *shares, *slots;
    unsigned long long* stamps;
    unsigned* bad;
    CK(hipMalloc(&shares, 2 * kGrid * 16));
    CK(hipMalloc(&slots, 2 * kGrid * 64 * 16));
    CK(hipMalloc(&stamps, kRounds * 8));
    CK(hipMalloc(&bad, 4));
    CK(hipMemset(shares, 0, 2 * kGrid * 16));
    CK(hipMemset(slots, 0, 2 * kGrid * 64 * 16));
    CK(hipMemset(bad, 0, 4));
    unsigned tag0 = 1;
    run<1>(s, shares, slots, stamps, bad, tag0, "P1 tagged-share poll (sc1)");
    run<2>(s, shares, slots, stamps, bad, tag0, "P2 + one 16-B hand-off per lane (sc1 store/load)");
    run<3>(s, shares, slots, stamps, bad, tag0, "P3 = P2 + skew 0..1.75 us by block");
    return 0;
}
