// Known-byte kernels in the round kernel's access patterns, to calibrate
// rocprofv3's FETCH_SIZE / WRITE_SIZE (MI355X_MICROARCH.md: FETCH_SIZE reports
// half the bytes of a wide coalesced 16-B-per-lane read; other widths are
// uncalibrated).  Each kernel runs once over 64 MiB-scale buffers (past the
// L2s); this program prints one JSON line naming each kernel's algorithmic
// read and write bytes, and scripts/pmc_calib.py divides the counters of a
// `rocprofv3 --pmc FETCH_SIZE` (and a separate WRITE_SIZE) run by them.
//   hipcc --offload-arch=gfx950 -O3 pmc_calib.hip -o pmc_calib
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kLanes = 1 << 19;   // 512 Ki lanes: 64 MiB of 128-B records

// (1) the host record: one 128-B line per lane, read as 8 x 16 B by its lane
__global__ void k_rec_read(const uint4* __restrict__ rec, uint32_t* __restrict__ out) {
    const size_t l = (size_t)blockIdx.x * 64 + threadIdx.x;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) { const uint4 v = rec[l * 8 + k]; s += v.x ^ v.y ^ v.z ^ v.w; }
    out[l] = s;
}
// (2) the same record written back whole (store_ctx)
__global__ void k_rec_write(uint4* __restrict__ rec) {
    const size_t l = (size_t)blockIdx.x * 64 + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 8; k++) rec[l * 8 + k] = make_uint4((uint32_t)l, k, 1, 2);
}
// (3) a 32-B event per lane from a line of its own, scattered (calendar slots)
__device__ __forceinline__ size_t scat(size_t l) { return (l * 2654435761ull) & (kLanes - 1); }
__global__ void k_ev_read(const uint4* __restrict__ ev, uint32_t* __restrict__ out) {
    const size_t l = (size_t)blockIdx.x * 64 + threadIdx.x;
    const size_t i = scat(l) * 8;   // slot 0 of line scat(l) (128-B lines of 4 events)
    const uint4 a = ev[i], b = ev[i + 1];
    out[l] = a.x ^ b.w;
}
// (4) the same slots written with four 8-B write-through stores (ev_st_sc1)
__global__ void k_ev_write_sc1(uint64_t* __restrict__ ev) {
    const size_t l = (size_t)blockIdx.x * 64 + threadIdx.x;
    uint64_t* d = ev + scat(l) * 16;
#pragma unroll
    for (int k = 0; k < 4; k++) __hip_atomic_store(d + k, (uint64_t)l + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// (5) a 16-B path entry per lane from a line of its own, scattered
__global__ void k_pv_read(const uint4* __restrict__ pv, uint32_t* __restrict__ out) {
    const size_t l = (size_t)blockIdx.x * 64 + threadIdx.x;
    const uint4 a = pv[scat(l) * 8];
    out[l] = a.x ^ a.z;
}
// (6) 16-B sc1 buffer loads, coalesced (the persistent rounds' bitmap words)
__global__ void k_sc1_read(const uint4* __restrict__ p, uint32_t* __restrict__ out) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const size_t l = (size_t)blockIdx.x * 64 + threadIdx.x;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(p + (size_t)blockIdx.x * 64 * 2), (short)0,
                                                                 64 * 32, 0x00020000);
    const v4u a = __builtin_amdgcn_raw_buffer_load_b128(r, threadIdx.x * 32, 0, 16);
    const v4u b = __builtin_amdgcn_raw_buffer_load_b128(r, threadIdx.x * 32 + 16, 0, 16);
    out[l] = a[0] ^ b[3];
}

int main() {
    uint4* big;
    uint32_t* out;
    CK(hipMalloc(&big, (size_t)kLanes * 128));
    CK(hipMalloc(&out, (size_t)kLanes * 4));
    CK(hipMemset(big, 1, (size_t)kLanes * 128));
    CK(hipMemset(out, 0, (size_t)kLanes * 4));
    const dim3 g(kLanes / 64), b(64);
    const unsigned long long L = kLanes;
    hipLaunchKernelGGL(k_rec_read, g, b, 0, 0, big, out);
    hipLaunchKernelGGL(k_rec_write, g, b, 0, 0, big);
    hipLaunchKernelGGL(k_ev_read, g, b, 0, 0, big, out);
    hipLaunchKernelGGL(k_ev_write_sc1, g, b, 0, 0, (uint64_t*)big);
    hipLaunchKernelGGL(k_pv_read, g, b, 0, 0, big, out);
    hipLaunchKernelGGL(k_sc1_read, dim3(kLanes / 64 / 4), b, 0, 0, big, out);
    CK(hipDeviceSynchronize());
    printf("{\"k_rec_read\": {\"read\": %llu, \"write\": %llu}, \"k_rec_write\": {\"read\": 0, \"write\": %llu}, "
           "\"k_ev_read\": {\"read\": %llu, \"write\": %llu}, \"k_ev_write_sc1\": {\"read\": 0, \"write\": %llu}, "
           "\"k_pv_read\": {\"read\": %llu, \"write\": %llu}, \"k_sc1_read\": {\"read\": %llu, \"write\": %llu}}\n",
           L * 128, L * 4, L * 128, L * 32, L * 4, L * 32, L * 16, L * 4, (L / 4) * 32, (L / 4) * 4);
    return 0;
}
