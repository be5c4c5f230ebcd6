// Feasibility: two processes on one GPU; process 0 allocates uncached device
// memory and exports an IPC handle; process 1 maps it, and the two exchange
// tagged blocks with in-kernel polling (bounded), 1000 times.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>
#include <sys/wait.h>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("rank %d: %s failed: %s\n", rank, #x, hipGetErrorString(e_)); exit(1); } } while (0)

// write n words + tag to dst (peer), then wait for my own buffer's tag == seq
__global__ void k_put_wait(unsigned* dst, const unsigned* mine, unsigned n, unsigned seq, unsigned* err) {
    for (unsigned i = threadIdx.x; i < n; i += blockDim.x) __hip_atomic_store(dst + 1 + i, seq * 1000u + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __atomic_thread_fence(__ATOMIC_RELEASE);
        __hip_atomic_store(dst, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        unsigned long long t0 = wall_clock64();
        while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
            __builtin_amdgcn_s_sleep(2);
            if (wall_clock64() - t0 > 100000000ull) { atomicOr(err, 1u); break; }   // 1 s
        }
    }
    __syncthreads();
    for (unsigned i = threadIdx.x; i < n; i += blockDim.x)
        if (__hip_atomic_load(mine + 1 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != seq * 1000u + i) atomicOr(err, 2u);
}

int main() {
    int fd01[2], fd10[2];
    if (pipe(fd01) || pipe(fd10)) return 1;
    int rank = 0;
    pid_t pid = fork();
    if (pid == 0) rank = 1;
    const unsigned n = 2048;
    unsigned* mine = nullptr;
    int rank_ = rank; (void)rank_;
    CK(hipSetDevice(0));
    CK(hipExtMallocWithFlags((void**)&mine, 4 * (n + 1), hipDeviceMallocUncached));
    CK(hipMemset(mine, 0, 4 * (n + 1)));
    hipIpcMemHandle_t h, ph;
    CK(hipIpcGetMemHandle(&h, mine));
    int wfd = rank == 0 ? fd01[1] : fd10[1], rfd = rank == 0 ? fd10[0] : fd01[0];
    if (write(wfd, &h, sizeof h) != sizeof h || read(rfd, &ph, sizeof ph) != sizeof ph) { printf("pipe\n"); return 1; }
    unsigned* peer = nullptr;
    CK(hipIpcOpenMemHandle((void**)&peer, ph, hipIpcMemLazyEnablePeerAccess));
    unsigned* err;
    CK(hipMalloc(&err, 4));
    CK(hipMemset(err, 0, 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (unsigned s = 1; s <= 1000; s++) hipLaunchKernelGGL(k_put_wait, dim3(1), dim3(256), 0, 0, peer, mine, n, s, err);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    unsigned e = 0;
    CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    printf("rank %d: 1000 tagged exchanges of %u words, err %u, %.2f us each\n", rank, n, e, ms * 1000 / 1000);
    CK(hipIpcCloseMemHandle(peer));
    if (pid > 0) { int st; waitpid(pid, &st, 0); }
    return e ? 3 : 0;
}
