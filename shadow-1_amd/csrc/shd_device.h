// shd_device.h -- internal declarations shared by the libshdgpu HIP sources.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shdgpu.h"
#include "../host/shd_host.h"

#define SHD_HIP(x)                                                      \
    do {                                                                \
        hipError_t e_ = (x);                                            \
        if (e_ != hipSuccess) {                                         \
            shd_set_hip_error(e_, #x, __FILE__, __LINE__);              \
            return SHD_ENODEV;                                          \
        }                                                               \
    } while (0)

void shd_set_hip_error(hipError_t e, const char* what, const char* file, int line);

static constexpr uint64_t kDistInf = 0x7FF0000000000000ull;   // +inf as u64
static constexpr int32_t kNoRank = 0x7FFFFFFF;

// Path-cache device state (owned by shd_pc, consumed by the engine).
// path value as stored: latency (ms) and reliability, interleaved
struct shd_pv {
    double lat, rel;
};

struct shd_pc {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t flags = 0;
    shd_csr csr{};
    shd_graph_props props{};
    int32_t V = 0, E = 0, T = 0;
    int directed = 0, complete = 0, prefer_direct = 0, rows_mode = 0, has_vloss = 0;
    // host copies
    int32_t* h_attached = nullptr;      // [T]
    int32_t* h_att_index = nullptr;     // [V] -> attached index or -1
    double* h_w = nullptr;              // [E]
    double* h_eloss = nullptr;          // [E]
    double* h_vloss = nullptr;          // [V] NaN = absent
    int32_t* h_self_eid = nullptr;      // [T] self-loop eid or -1
    // device graph
    int32_t *d_arc_off = nullptr, *d_arc_dst = nullptr;
    double* d_arc_w = nullptr;
    int32_t *d_rin_off = nullptr, *d_rin_src = nullptr, *d_rin_eid = nullptr;
    double* d_rin_w = nullptr;
    int32_t* d_arc_src = nullptr;   // forward arc -> tail vertex
    int32_t* d_arc_rin = nullptr;   // forward arc -> its index among the head's in-arcs
    double* d_rin_r = nullptr;      // in-arc -> its edge's 1 - loss
    int32_t *d_inc_off = nullptr, *d_inc_eid = nullptr;
    int32_t *d_nbr_off = nullptr, *d_nbr_v = nullptr, *d_nbr_eid = nullptr;
    double *d_w = nullptr, *d_eloss = nullptr, *d_vloss = nullptr;
    int32_t *d_attached = nullptr, *d_self_eid = nullptr;
    // device tables [T][T] and [T] of (latency, reliability) pairs: one 16-B
    // load per lookup in the event loop
    shd_pv* d_row = nullptr;
    size_t rows_alloc = 0;              // rows allocated in d_row beyond T (sharded builds pad to world blocks)
    shd_pv* d_dir = nullptr;
    shd_pv* d_self = nullptr;
    uint8_t* d_adj = nullptr;           // [T][T] 1 = adjacent (direct path exists)
    void* d_scratch = nullptr;          // global-memory SSSP scratch (large V)
    size_t scratch_bytes = 0;
    bool lds_off_ok = false;            // the row kernel may keep the CSR's arc offsets in LDS
    int32_t* d_tie_rows = nullptr;      // [T] rows with equal-cost predecessors (first pass)
    void* d_tie_scratch = nullptr;      // tied rows' parents (k_sssp_tie_lds / k_sssp_tie_parents)
    size_t tie_scratch_bytes = 0;
    void* d_tie_lane = nullptr;         // k_sssp_tie_parents' lane heaps (rows whose heap outgrew LDS)
    size_t tie_lane_bytes = 0;
    bool w_int = false;                 // whole-number arc weights, V x the largest < 2^30 (4-B tie heap values)
    int64_t* d_stats = nullptr;         // ties, max hops, max iters, unroutable, lat mismatch, minlat bits, tie rows
    bool built = false;
    shd_pc_info info{};
    // host lazy-cache adapter state (shd_pc_lookup)
    int32_t* h_rank = nullptr;          // [T] row run order, kNoRank if never
    int32_t* h_self_rank = nullptr;     // [T] self-path store order
    uint8_t* h_direct_stored = nullptr; // lazily allocated [T*T] bits for direct/adjacent stores
    int32_t next_rank = 0;
    double min_stored_latency = 0.0;
    void* counts = nullptr;             // std::unordered_map<uint64_t,uint64_t>*
    void* touches = nullptr;            // PcTouches* (shd_pc_defer_touches), or null
};

// resolved value for a (src attached idx, dst attached idx) pair given ranks
// (device + host): see DESIGN.md "First-touch rule".

// ---- group communicators (comm.hip): RCCL or the host-memory transport ----
#include <rccl/rccl.h>
enum { SHD_COMM_RCCL = 1, SHD_COMM_HOST = 2 };
struct shd_comm {
    int kind = 0;
    int world = 1, rank = 0, device = 0;
    ncclComm_t nccl = nullptr;
    shd_xhost* hx = nullptr;
    hipStream_t s = nullptr;            // the communicator's own stream
    void* h_stage = nullptr;            // pinned staging (host transport)
    size_t h_stage_bytes = 0;
};
// device buffers, enqueued on `s` (RCCL) or staged through host memory
// (host transport: synchronizes `s`); recv holds world blocks
__attribute__((visibility("hidden"))) int shd_comm_alltoall_dev(shd_comm* c, const void* d_send, void* d_recv,
                                                                size_t bytes_per_peer, hipStream_t s);
__attribute__((visibility("hidden"))) int shd_comm_allgather_dev(shd_comm* c, const void* d_send, void* d_recv,
                                                                 size_t bytes, hipStream_t s);
// host buffers, blocking: out[r * bytes ...] = rank r's `bytes`
__attribute__((visibility("hidden"))) int shd_comm_allgather_host(shd_comm* c, const void* mine, size_t bytes,
                                                                  void* out);
