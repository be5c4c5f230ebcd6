// comm.hip -- communicators of an engine group (include/shdgpu.h shd_comm_*):
// the per-round exchange of slave.c:437-462's rounds across GPUs.
//
//   RCCL   one process per GPU; ncclAllToAll / ncclAllGather enqueued on the
//          caller's stream (capturable in the engine's batch graphs) over xGMI.
//   host   processes of one machine meeting in shared memory (shd_xhost.c):
//          device buffers are staged through pinned host memory.  It runs the
//          group protocol where RCCL cannot (several ranks on one GPU), so the
//          multi-process path is testable on a one-GPU box.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "shd_device.h"

static_assert(sizeof(ncclUniqueId) == SHD_XID_BYTES, "RCCL unique id size");

static int stage(shd_comm* c, size_t bytes) {
    if (c->h_stage_bytes >= bytes) return SHD_OK;
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    c->h_stage = nullptr;
    c->h_stage_bytes = 0;
    SHD_HIP(hipHostMalloc(&c->h_stage, bytes ? bytes : 64));
    c->h_stage_bytes = bytes;
    return SHD_OK;
}

extern "C" int shd_comm_create_rccl(const uint8_t id[SHD_XID_BYTES], int world, int rank, int device,
                                    shd_comm** out) {
    if (!id || world <= 0 || world > 64 || rank < 0 || rank >= world || !out) return SHD_EINVAL;
    SHD_HIP(hipSetDevice(device));
    shd_comm* c = new shd_comm();
    c->kind = SHD_COMM_RCCL;
    c->world = world; c->rank = rank; c->device = device;
    ncclUniqueId u;
    memcpy(&u, id, SHD_XID_BYTES);
    if (hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking) != hipSuccess ||
        ncclCommInitRank(&c->nccl, world, u, rank) != ncclSuccess) {
        c->nccl = nullptr;
        shd_comm_destroy(c);
        return SHD_ENODEV;
    }
    *out = c;
    return SHD_OK;
}

extern "C" int shd_comm_create_host(const char* name, int world, int rank, int device, shd_comm** out) {
    if (!name || world <= 0 || world > 64 || rank < 0 || rank >= world || !out) return SHD_EINVAL;
    SHD_HIP(hipSetDevice(device));
    shd_comm* c = new shd_comm();
    c->kind = SHD_COMM_HOST;
    c->world = world; c->rank = rank; c->device = device;
    int rc = hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking) == hipSuccess ? SHD_OK : SHD_ENODEV;
    if (!rc) rc = shd_xhost_open(name, world, rank, (size_t)8 << 20, &c->hx);
    if (rc) { shd_comm_destroy(c); return rc; }
    *out = c;
    return SHD_OK;
}

extern "C" int shd_comm_rank(const shd_comm* c, int* rank, int* world) {
    if (!c || !rank || !world) return SHD_EINVAL;
    *rank = c->rank;
    *world = c->world;
    return SHD_OK;
}

extern "C" void shd_comm_destroy(shd_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    if (c->hx) shd_xhost_close(c->hx);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->s) (void)hipStreamDestroy(c->s);
    delete c;
}

int shd_comm_alltoall_dev(shd_comm* c, const void* d_send, void* d_recv, size_t bytes, hipStream_t s) {
    if (c->kind == SHD_COMM_RCCL) {
        if (ncclAllToAll(d_send, d_recv, bytes, ncclUint8, c->nccl, s) != ncclSuccess) return SHD_ENODEV;
        return SHD_OK;
    }
    const size_t all = bytes * (size_t)c->world;
    int rc = stage(c, 2 * all);
    if (rc) return rc;
    char* hs = (char*)c->h_stage;
    SHD_HIP(hipMemcpyAsync(hs, d_send, all, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    if ((rc = shd_xhost_alltoall(c->hx, hs, bytes, hs + all))) return rc;
    SHD_HIP(hipMemcpyAsync(d_recv, hs + all, all, hipMemcpyHostToDevice, s));
    SHD_HIP(hipStreamSynchronize(s));
    return SHD_OK;
}

// (declared where it is used: csrc/tcp.hip)
__attribute__((visibility("hidden"))) int shd_comm_alltoallv_dev(shd_comm* c, const char* d_send, const size_t* send_off, const size_t* send_bytes,
                           char* d_recv, const size_t* recv_off, const size_t* recv_bytes, hipStream_t s) {
    const int W = c->world;
    if (c->kind == SHD_COMM_RCCL) {
        if (ncclGroupStart() != ncclSuccess) return SHD_ENODEV;
        int rc = SHD_OK;
        for (int p = 0; p < W && !rc; p++) {
            if (send_bytes[p] &&
                ncclSend(d_send + send_off[p], send_bytes[p], ncclUint8, p, c->nccl, s) != ncclSuccess)
                rc = SHD_ENODEV;
            if (!rc && recv_bytes[p] &&
                ncclRecv(d_recv + recv_off[p], recv_bytes[p], ncclUint8, p, c->nccl, s) != ncclSuccess)
                rc = SHD_ENODEV;
        }
        if (ncclGroupEnd() != ncclSuccess) rc = SHD_ENODEV;
        return rc;
    }
    size_t blk = 0;   // every rank's largest block (each rank passes the same sizes' maximum: both directions)
    for (int p = 0; p < W; p++) blk = std::max(blk, std::max(send_bytes[p], recv_bytes[p]));
    unsigned long long mine = blk;
    std::vector<unsigned long long> all(W);
    int rc = shd_xhost_allgather(c->hx, &mine, sizeof(mine), all.data());
    if (rc) return rc;
    blk = 0;
    for (unsigned long long v : all) blk = std::max(blk, (size_t)v);
    if (blk == 0) return SHD_OK;
    const size_t tot = blk * (size_t)W;
    if ((rc = stage(c, 2 * tot))) return rc;
    char* hs = (char*)c->h_stage;
    for (int p = 0; p < W; p++)
        if (send_bytes[p]) SHD_HIP(hipMemcpyAsync(hs + (size_t)p * blk, d_send + send_off[p], send_bytes[p],
                                                  hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    if ((rc = shd_xhost_alltoall(c->hx, hs, blk, hs + tot))) return rc;
    for (int p = 0; p < W; p++)
        if (recv_bytes[p]) SHD_HIP(hipMemcpyAsync(d_recv + recv_off[p], hs + tot + (size_t)p * blk, recv_bytes[p],
                                                  hipMemcpyHostToDevice, s));
    SHD_HIP(hipStreamSynchronize(s));
    return SHD_OK;
}

int shd_comm_allgather_dev(shd_comm* c, const void* d_send, void* d_recv, size_t bytes, hipStream_t s) {
    if (c->kind == SHD_COMM_RCCL) {
        if (ncclAllGather(d_send, d_recv, bytes, ncclUint8, c->nccl, s) != ncclSuccess) return SHD_ENODEV;
        return SHD_OK;
    }
    std::vector<char> mine(bytes), all(bytes * (size_t)c->world);
    SHD_HIP(hipMemcpyAsync(mine.data(), d_send, bytes, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    int rc = shd_xhost_allgather(c->hx, mine.data(), bytes, all.data());
    if (rc) return rc;
    SHD_HIP(hipMemcpyAsync(d_recv, all.data(), all.size(), hipMemcpyHostToDevice, s));
    SHD_HIP(hipStreamSynchronize(s));
    return SHD_OK;
}

int shd_comm_allgather_host(shd_comm* c, const void* mine, size_t bytes, void* out) {
    if (c->kind == SHD_COMM_HOST) return shd_xhost_allgather(c->hx, mine, bytes, out);
    SHD_HIP(hipSetDevice(c->device));
    char* d = nullptr;
    const size_t all = bytes * (size_t)c->world;
    SHD_HIP(hipMalloc((void**)&d, all ? all : 64));
    int rc = SHD_OK;
    if (bytes && hipMemcpyAsync(d + (size_t)c->rank * bytes, mine, bytes, hipMemcpyHostToDevice, c->s) != hipSuccess)
        rc = SHD_ENODEV;
    if (!rc && bytes && ncclAllGather(d + (size_t)c->rank * bytes, d, bytes, ncclUint8, c->nccl, c->s) != ncclSuccess)
        rc = SHD_ENODEV;
    if (!rc && bytes && hipMemcpyAsync(out, d, all, hipMemcpyDeviceToHost, c->s) != hipSuccess) rc = SHD_ENODEV;
    if (!rc && hipStreamSynchronize(c->s) != hipSuccess) rc = SHD_ENODEV;
    (void)hipFree(d);
    return rc;
}
