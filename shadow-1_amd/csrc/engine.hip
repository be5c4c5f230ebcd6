// engine.hip -- the conservative round/window packet event loop on MI355X.
//
// One GPU thread owns one simulated host.  Per round [ws, we) each host pops
// its events in (time, src, seq) order (event_compare, event.c:110-153; the
// dst key is the host itself) and executes them with the reference semantics
// of the PHOLD-UDP model (DESIGN.md "Model"):
//
//   worker_sendPacket      worker.c:260-321   path value, one RNG draw per send,
//                                              drop unless chance <= reliability,
//                                              delivery at now + ceil(lat * 1e6)
//   router_enqueue/CoDel   router.c:104-133, router_queue_codel.c:113-267
//   token buckets + refill network_interface.c:102-226, 421-455, 519-579
//   PHOLD application      test_phold.c (chooseNode, implicit-bind port, one
//                                        message per received message)
//
// W = min over attached pairs of ceil(lat*1e6) ns (every inter-host event
// lands at or after the window end), so a host never receives an event for
// the round it is executing: rounds are serial-equivalent and the result is
// the reference's serial (--workers 0) run bit for bit.  Self events that fall
// inside the window (refills, +1 ns loopback / epoll notifications) are
// processed in the same round by the owning thread.
//
// Device layout (HBM): one 128-B record per host; per
// host a calendar of time bins (the common path for inter-host events), a
// 4-ary heap of 32-B events fed by double-buffered inboxes (the rest), CoDel
// and send FIFOs.  The first-touch path-cache rule is
// applied from per-vertex row ranks; the rare sends whose pair was unranked at
// round start are logged, resolved in serial order, and finalised.
//
// One translation unit, in parts: eng_device.h (types, per-host event code),
// eng_round.h (one engine's round kernels), eng_exchange.h (engine-group
// exchange kernels), this file (the single-engine host driver and C-ABI) and
// eng_group.h (the engine-group host driver and C-ABI).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "shd_device.h"

namespace {

#include "eng_device.h"
#include "eng_round.h"
#include "eng_exchange.h"

}  // namespace

// ------------------------------------------------------------------ host driver
// Test hooks that change the engine's semantics (forced first-touch ambiguity,
// every round protected, a failing peer mapping) exist only in the test build
// (make testhooks -> libshdgpu_th.so, -DSHD_TEST_HOOKS), which the tests that
// need them load in a child process; the product library ignores these names.
#ifdef SHD_NO_LEAN   // A/B build: the general instantiations for every model
static constexpr bool kNoLean = true;
#else
static constexpr bool kNoLean = false;
#endif
// the lean round kernels (LEAN: no optional feature, no bootstrap period --
// every bench model): their feature word and bootstrap end are constants
template <class PT>
static bool lean_model(const PT& P) { return !kNoLean && P.feat == 0 && P.bootstrap_end == 0; }
#ifdef SHD_TEST_HOOKS
static bool test_hook(const char* name) { return getenv(name) != nullptr; }
#else
static bool test_hook(const char*) { return false; }
#endif

struct shd_eng {
    int device = 0;
    hipStream_t stream = nullptr;
    shd_pc* pc = nullptr;
    Params P{};
    int32_t H = 0, h0 = 0, nloc = 0;
    uint64_t window = 0;
    int parity = 0;
    bool booted = false;
    bool heartbeats = false;    // SHD_QF_HEARTBEATS: snapshots in P.hb
    std::vector<uint64_t> host_hb;   // <host heartbeatfrequency> per host (empty: P.heartbeat)
    std::vector<int32_t> app_peer_dev;   // per host: the SHD_DEST_PEER host (device copy), else -1
    std::vector<int32_t> app_peer;   // per host: >= 0 where it reads on the socket it sends from
                                     // (SHD_SEND_ONCE; the status writer's port rule), empty: PHOLD
    std::vector<void*> allocs;
    std::vector<size_t> alloc_bytes;
    // protected rounds (DESIGN.md "First-touch rule"): device state copied
    // before a round that may log many first touches, restored when one of its
    // drop decisions turns out ambiguous, then the round reruns with the ranks
    std::vector<void*> snap;
    std::vector<uint8_t> snap_kind;   // per entry: 0 device, 1 pinned host, 2 pageable host
    bool snap_failed = false;
    // the copy as a restore point (shd_eng_run_until): `snap` holds the state
    // at the start of round snap_round, window start snap_next, and nothing
    // outside the rounds has changed the state since (push_events, ingest and
    // the host-driven co-simulation rounds clear snap_valid)
    bool snap_valid = false;
    bool in_replay = false;
    int snap_parity = 0;
    uint64_t snap_round = 0, snap_next = 0;
    DevSummary snap_sum{};
    // the stops of the run_until calls since the copy: a round's window ends at
    // min(start + W, stop), so a replay stops at each of them again to run the
    // same windows (the same rounds resolve the same first-touch logs)
    std::vector<uint64_t> snap_stops;
    // shd_eng_round_begin's state copy, for shd_eng_round_retry
    bool rb_snap = false;
    int rb_parity = 0;
    uint64_t rb_round = 0, rb_ws = 0, rb_we = 0;
    DevSummary rb_sum{};
    bool logged_any = false;                // a round has logged a first touch
    uint64_t last_logged = 0;               // first touches logged by the last round
    // inputs kept on device
    uint32_t* d_rng0 = nullptr;
    uint64_t* d_bwd = nullptr;
    uint64_t* d_bwu = nullptr;
    int32_t* d_host_att = nullptr;
    double* d_cum = nullptr;
    DestGuide* d_guide = nullptr;
    int4* d_self_thr = nullptr;
    uint64_t* d_host_hb = nullptr;
    int32_t* d_app_peer = nullptr;
    uint8_t* d_app_mode = nullptr;
    uint32_t* d_app_nstart = nullptr;
    int32_t n_cls = 1;
    uint64_t t_done = 0;                    // end of the last executed round's window (push_events floor)
    int32_t* d_rank = nullptr;
    int32_t* d_self_rank = nullptr;
    DevSummary* d_sum = nullptr;
    DevSummary* h_sum = nullptr;   // pinned
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_kernel_ms = 0;
    double kernel_ms_total = 0;
    // host mirrors for the first-touch resolution
    std::vector<int32_t> h_rank, h_self_rank;
    int32_t next_rank = 0;
    uint64_t pending_resolved = 0;
    uint64_t round_ws = 0, round_we = 0, round_pending = 0, round_events = 0, round_pkt = 0, round_active = 0;
    uint64_t round = 0;                     // rounds executed (parity = round & 1)
    // device-driven pipeline
    static constexpr int kBatch = 64;
    static constexpr int kPsBatch = 128;      // rounds of a persistent launch (k_round_ps)
    static constexpr int kRing = 2 * kBatch + 2;
    static_assert(kPsBatch + 2 <= kRing, "a persistent batch's summaries fit the ring");
    DevSummary* d_ring = nullptr;
    DevSummary* h_ring = nullptr;           // pinned
    uint32_t* d_halt = nullptr;
    int32_t* d_next_rank = nullptr;
    unsigned long long* d_trace_n = nullptr;
    hipEvent_t bev[2 * kBatch] = {};
    DevCtl* d_ctl = nullptr;                // per-batch inputs (device) and their pinned staging
    DevCtl* h_ctl = nullptr;
    DevSummary* h_seed = nullptr;           // pinned: ring slots 0 and 1 at a batch start
    hipGraphExec_t batch_graph = nullptr;   // captured batch of kBatch device-driven rounds
    hipGraphExec_t batch_graph_tl = nullptr;   // the same, ticketless (k_round_tl)
    TlPart* d_tpart = nullptr;              // [2][grid] ticketless round shares
    bool tl_ready = false;                  // the last batch logged no first touch: run ticketless
    Params* d_pr = nullptr;                 // device copies of P, one per summary-ring slot (sum = &d_ring[i])
    // persistent rounds (k_round_ps): one launch per batch when the round grid
    // fits the GPU one block per CU and the engine holds every host
    bool ps_ok = false;
    bool sp_ok = false;                     // the sparse persistent kernel (k_round_sp) instead
    bool sp_lrec = false;                   // its hosts' records resident in LDS for a batch
    size_t sp_dyn = 0;                      // its dynamic LDS bytes
    bool sp_dense = false;                  // the last batch had many active hosts: launch-per-round batches
    bool sp_forced = false;                 // SHD_SP_HOSTS: the sparse kernel whatever the density
    uint32_t sp_hosts = 0;                  // ... its hosts per block
    uint32_t sp_grid = 0;
    PsShare* d_pshare = nullptr;            // [2][grid] tagged round shares
    uint32_t ps_epoch = 1;                  // share tags issued (never 0, never reused)
    double wall_khz = 100000.0;             // device wall clock (wall_clock64) rate
    uint64_t trace_cap = 0;
};

// the largest rand_r value x with (double)x / RAND_MAX <= c (-1 if none):
// the quotient is correctly rounded on host and device alike and monotone in
// x, so the device compares integers instead of dividing
static int32_t draw_threshold(double c) {
    int64_t lo = -1, hi = 2147483647;   // invariant: ok(lo) (or lo == -1), !ok(hi + 1)
    auto ok = [c](int64_t x) { return (double)x / 2147483647.0 <= c; };
    if (ok(hi)) return (int32_t)hi;
    while (hi - lo > 1) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (ok(mid)) lo = mid; else hi = mid;
    }
    return (int32_t)lo;
}

template <typename T>
static int ealloc(shd_eng* e, T** p, size_t n, bool zero = true) {
    void* q = nullptr;
    SHD_HIP(hipMalloc(&q, sizeof(T) * (n ? n : 1)));
    e->allocs.push_back(q);
    e->alloc_bytes.push_back(sizeof(T) * (n ? n : 1));
    if (zero) SHD_HIP(hipMemsetAsync(q, 0, sizeof(T) * (n ? n : 1), e->stream));
    *p = (T*)q;
    return SHD_OK;
}

#define EALLOC(ptr, n)                          \
    do {                                        \
        int rc_ = ealloc(e, &(ptr), (size_t)(n)); \
        if (rc_) { shd_eng_destroy(e); return rc_; } \
    } while (0)

// The datagram application of every host (shd_model::app other than PHOLD),
// checked so that no datagram can reach a port nobody listens on (the device
// hands every datagram that reaches a started host to its application):
// mode[h] = send | dest << 2 | per_read << 4, nstart[h] its start count,
// peer[h] its SHD_DEST_PEER host (else -1).  *rq_cap: the per-host ring of
// the sources of unread datagrams (replying hosts only; 0: none), bounded by
// the datagrams that can be in flight at once.
static int resolve_apps(const shd_model* m, int32_t n_cls, std::vector<uint8_t>& mode, std::vector<uint32_t>& nstart,
                        std::vector<int32_t>& peer, uint32_t* rq_cap, uint64_t* max_start) {
    const int32_t H = m->n_hosts;
    mode.assign(H, 0);
    nstart.assign(H, 0);
    peer.assign(H, -1);
    *rq_cap = 0;
    *max_start = 0;
    if (m->app == SHD_APP_UDP_ECHO) {
        // the UDP echo's roles: every client's server is a server host; a
        // socket holds at most the requests in flight to it (its clients' loads)
        if (!m->app_peer) return SHD_EINVAL;
        std::vector<uint64_t> held(H, m->load);
        for (int32_t h = 0; h < H; h++) {
            const int32_t s = m->app_peer[h];
            if (s < -1 || s >= H || s == h || (s >= 0 && m->app_peer[s] != -1)) return SHD_EINVAL;
            if (s >= 0) held[s] += m->load;
            mode[h] = s < 0 ? (uint8_t)(SHD_SEND_LISTENER | SHD_DEST_REPLY << 2 | 1u << 4)
                            : (uint8_t)(SHD_SEND_ONCE | SHD_DEST_PEER << 2 | 1u << 4);
            nstart[h] = s < 0 ? 0u : m->load;
            peer[h] = s;
        }
        uint64_t cap = 16;
        for (int32_t h = 0; h < H; h++) cap = std::max<uint64_t>(cap, held[h]);
        if (cap > 65535) return SHD_ERANGE;   // (a 16-bit ring head in the record)
        *rq_cap = (uint32_t)cap;
        *max_start = m->load;
        return SHD_OK;
    }
    // SHD_APP_UDP
    auto refuse = [](const char* why, long a, long b) {
        fprintf(stderr, "shd_eng_create: SHD_APP_UDP: %s (%ld, %ld)\n", why, a, b);
        return SHD_EINVAL;
    };
    if (!m->app_spec || !m->host_app || m->n_app_specs == 0 || m->n_app_specs > 256)
        return refuse("no specs, or more than 256", (long)m->n_app_specs, 0);
    for (uint32_t k = 0; k < m->n_app_specs; k++) {
        const shd_udp_app& a = m->app_spec[k];
        if (a.send > SHD_SEND_LISTENER || a.dest > SHD_DEST_REPLY || a.per_read > 1)
            return refuse("spec out of range", (long)k, 0);
        if (a.dest == SHD_DEST_REPLY && (a.n_start || a.send == SHD_SEND_EACH))
            return refuse("a replying spec that starts or sends from new sockets", (long)k, 0);
    }
    bool any_reply = false;
    uint64_t total = 0;
    for (int32_t h = 0; h < H; h++) {
        if (m->host_app[h] >= m->n_app_specs) return refuse("host_app out of range", (long)h, m->host_app[h]);
        const shd_udp_app& a = m->app_spec[m->host_app[h]];
        mode[h] = (uint8_t)(a.send | a.dest << 2 | a.per_read << 4);
        nstart[h] = a.n_start;
        total += a.n_start;
        *max_start = std::max<uint64_t>(*max_start, a.n_start);
        any_reply |= a.dest == SHD_DEST_REPLY;
    }
    auto listens = [&](int32_t x) { return (mode[x] & 3u) != SHD_SEND_ONCE; };
    auto replies = [&](int32_t x) { return ((mode[x] >> 2) & 3u) == SHD_DEST_REPLY; };
    // the weighted rows: a host with positive weight is a destination of the
    // row's hosts, so it must listen; and, if any of them sends from a new
    // socket each time, must not reply (the reply would go to a closed port)
    std::vector<uint8_t> row_used(n_cls, 0), row_each(n_cls, 0);
    for (int32_t h = 0; h < H; h++) {
        if (((mode[h] >> 2) & 3u) != SHD_DEST_WEIGHTED) continue;
        const int32_t cl = m->host_class ? m->host_class[h] : 0;
        row_used[cl] = 1;
        if ((mode[h] & 3u) == SHD_SEND_EACH) row_each[cl] = 1;
    }
    for (int32_t cl = 0; cl < n_cls; cl++) {
        if (!row_used[cl]) continue;
        const double* cum = m->dest_cum + (size_t)cl * H;
        for (int32_t i = 0; i < H; i++) {
            const bool pos = i == 0 ? cum[0] > 0.0 : cum[i] > cum[i - 1];
            if (!pos) continue;
            if (!listens(i)) return refuse("a weighted destination does not listen (class, host)", cl, i);
            if (row_each[cl] && replies(i))
                return refuse("a replying host is a weighted destination of new-socket senders (class, host)", cl, i);
        }
    }
    for (int32_t h = 0; h < H; h++) {
        if (((mode[h] >> 2) & 3u) != SHD_DEST_PEER) continue;
        const int32_t s = m->app_peer ? m->app_peer[h] : -1;
        if (s < 0 || s >= H || s == h || !listens(s)) return refuse("a peer that does not listen (host, peer)", h, s);
        if ((mode[h] & 3u) == SHD_SEND_EACH && replies(s))
            return refuse("a replying peer of a new-socket sender (host, peer)", h, s);
        peer[h] = s;
    }
    if (any_reply) {
        // every datagram in flight started as some host's start datagram
        // (one read answers with at most one): a socket holds at most them all
        const uint64_t cap = std::max<uint64_t>(16, total);
        if (cap > 65535) return SHD_ERANGE;   // (a 16-bit ring head in the record)
        *rq_cap = (uint32_t)cap;
    }
    return SHD_OK;
}

extern "C" int shd_eng_create(const shd_model* m, shd_pc* pc, int32_t host_begin, int32_t host_end, int device,
                              shd_eng** out) {
    if (!m || !pc || !out || !pc->built || m->n_hosts <= 0) return SHD_EINVAL;
    if (host_begin < 0 || host_end > m->n_hosts || host_begin >= host_end) return SHD_EINVAL;
    if (!m->host_vertex || !m->host_rng || !m->bw_down_kibps || !m->bw_up_kibps || !m->dest_cum) return SHD_EINVAL;
    if (m->heartbeat_interval == 0) return SHD_EINVAL;
    const int32_t H = m->n_hosts;
    // destination-weight classes: dest_cum is [n_cls][H], host_class picks the row
    const int32_t n_cls = m->n_classes > 1 ? m->n_classes : 1;
    if (n_cls > 1 && !m->host_class) return SHD_EINVAL;
    if (n_cls > 256) return SHD_EINVAL;
    if (m->host_class)
        for (int32_t h = 0; h < H; h++)
            if ((int32_t)m->host_class[h] >= n_cls) return SHD_EINVAL;
    uint64_t hb_min = m->heartbeat_interval;
    if (m->host_heartbeat)
        for (int32_t h = 0; h < H; h++) {
            if (m->host_heartbeat[h] == 0) return SHD_EINVAL;
            hb_min = std::min<uint64_t>(hb_min, m->host_heartbeat[h]);
        }
    // every host must sit on an attached vertex of the path cache
    std::vector<int32_t> host_att(H);
    std::vector<int32_t> hosts_on(pc->T, 0);
    for (int32_t h = 0; h < H; h++) {
        const int32_t v = m->host_vertex[h];
        if (v < 0 || v >= pc->V || pc->h_att_index[v] < 0) return SHD_EINVAL;
        host_att[h] = pc->h_att_index[v];
        hosts_on[host_att[h]]++;
    }
    // row mode needs a self-loop on every attached vertex (a row without one
    // fails as a whole in the reference, topology.c:1490-1495)
    if (pc->rows_mode && pc->info.n_unroutable != 0) return SHD_EINVAL;
    shd_eng* e = new shd_eng();
    e->device = device;
    e->pc = pc;
    e->H = H; e->h0 = host_begin; e->nloc = host_end - host_begin;
    if (hipSetDevice(device) != hipSuccess) { delete e; return SHD_ENODEV; }
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) { delete e; return SHD_ENODEV; }
    (void)hipEventCreate(&e->ev0);
    (void)hipEventCreate(&e->ev1);
    Params& P = e->P;
    P.H = H; P.h0 = host_begin; P.nloc = e->nloc;
    P.hpw = 64;
    if (const char* s = getenv("SHD_HPW")) P.hpw = std::min(64, std::max(1, atoi(s)));
    // default capacities: packets in flight TO a host are ~ load x (mean latency
    // of its inbound paths / global mean latency), up to ~10x load on the
    // bundled topology (5 - 2294 ms edges); one round's arrivals peak at the
    // application start (every host sends `load` messages at once)
    P.evq_cap = m->evq_cap ? m->evq_cap : std::max<uint32_t>(64, 16 * m->load + 64);
    P.inbox_cap = m->inbox_cap ? m->inbox_cap : std::max<uint32_t>(64, 4 * m->load + 32);
    P.cq_cap = m->codelq_cap ? m->codelq_cap : 64;
    P.tq_cap = m->txq_cap ? m->txq_cap : 64;
    // the host record keeps FIFO positions in 16 bits and CoDel's queued bytes in 32
    if (P.cq_cap > 65535 || P.tq_cap > 65535 ||
        (uint64_t)P.cq_cap * ((uint64_t)m->payload + SHD_HEADER_UDP) >> 32) {
        shd_eng_destroy(e);
        return SHD_EINVAL;
    }
    if (m->host_heartbeat) e->host_hb.assign(m->host_heartbeat, m->host_heartbeat + H);
    // the applications other than PHOLD: every host's datagram application as
    // a mode byte (send | dest << 2 | per_read << 4) and its start count
    std::vector<uint8_t> app_mode;
    std::vector<uint32_t> app_nstart;
    uint64_t max_start = m->load;
    if (m->app == SHD_APP_UDP_ECHO || m->app == SHD_APP_UDP) {
        std::vector<int32_t> peer(H, -1);
        const int rc0 = resolve_apps(m, n_cls, app_mode, app_nstart, peer, &P.rq_cap, &max_start);
        if (rc0) { shd_eng_destroy(e); return rc0; }
        e->app_peer.assign(H, -1);   // the status writer: hosts that read on their sending socket
        for (int32_t h = 0; h < H; h++)
            if ((app_mode[h] & 3u) == SHD_SEND_ONCE) e->app_peer[h] = 0;
        e->app_peer_dev = peer;
    } else if (m->app != SHD_APP_PHOLD) {
        shd_eng_destroy(e);
        return SHD_EINVAL;
    }
    P.app = m->app;
    P.end_time = m->end_time; P.bootstrap_end = m->bootstrap_end; P.heartbeat = m->heartbeat_interval;
    P.app_start = m->app_start; P.load = m->load; P.payload = m->payload;
    P.pkt_len = m->payload + SHD_HEADER_UDP;
    P.force_ambig = test_hook("SHD_FORCE_AMBIG");
    const size_t n = (size_t)e->nloc;
    EALLOC(P.hs, n);
    EALLOC(P.hc, n);
    EALLOC(P.part, n);
    EALLOC(e->d_tpart, 2 * n);
    EALLOC(P.gpart, n / kTickGroup + 2);
    EALLOC(P.tick, n / kTickGroup + 3);
    {
        int rc;
        P.evq_stride = ((P.evq_cap + 3) & ~3u) + 4;   // heap root at +3: child groups 128-B aligned
        if ((rc = ealloc(e, &P.evq, n * P.evq_stride, false)) || (rc = ealloc(e, &P.hnext, n)) ||
            (rc = ealloc(e, &P.inbox[0], n * P.inbox_cap, false)) ||
            (rc = ealloc(e, &P.inbox[1], n * P.inbox_cap, false)) || (rc = ealloc(e, &P.inbox_n[0], n)) ||
            (rc = ealloc(e, &P.inbox_n[1], n)) || (rc = ealloc(e, &P.cq, n * P.cq_cap, false)) ||
            (rc = ealloc(e, &P.tq, n * P.tq_cap, false))) {
            shd_eng_destroy(e);
            return rc;
        }
    }
    e->n_cls = n_cls;
    const size_t HC = (size_t)H * (size_t)n_cls;
    EALLOC(e->d_rng0, H); EALLOC(e->d_bwd, H); EALLOC(e->d_bwu, H); EALLOC(e->d_host_att, H); EALLOC(e->d_cum, HC);
    EALLOC(e->d_guide, HC);
    EALLOC(e->d_self_thr, H);
    if (m->host_heartbeat) EALLOC(e->d_host_hb, H);
    if (!app_mode.empty()) {
        EALLOC(e->d_app_peer, H);
        EALLOC(e->d_app_mode, H);
        EALLOC(e->d_app_nstart, H);
        if (P.rq_cap) EALLOC(P.rq, n * P.rq_cap);
    }
    // destination guide table per class: guide[k] = first i with cum[i] >= k / H (H if none)
    std::vector<DestGuide> guide(HC);
    for (int32_t cl = 0; cl < n_cls; cl++) {
        const double* cum = m->dest_cum + (size_t)cl * H;
        DestGuide* gd = guide.data() + (size_t)cl * H;
        for (int32_t k = 0, i = 0; k < H; k++) {
            const double t = (double)k / (double)H;
            while (i < H && !(cum[i] >= t)) i++;
            gd[k].i = i;
            gd[k].pad = 0;
            for (int j = 0; j < 3; j++) {
                gd[k].cum[j] = i + j < H ? cum[i + j] : 2.0;
                gd[k].att[j] = i + j < H ? host_att[i + j] : -1;
            }
        }
        for (int32_t i = 1; i < H; i++)
            if (!(cum[i] >= cum[i - 1])) { shd_eng_destroy(e); return SHD_EINVAL; }
    }
    EALLOC(e->d_rank, pc->T); EALLOC(e->d_self_rank, pc->T);
    EALLOC(e->d_sum, 1);
    if (hipHostMalloc((void**)&e->h_sum, sizeof(DevSummary)) != hipSuccess) { shd_eng_destroy(e); return SHD_ENOMEM; }
    memset(e->h_sum, 0, sizeof(DevSummary));
    EALLOC(e->d_ring, shd_eng::kRing);
    if (hipHostMalloc((void**)&e->h_ring, sizeof(DevSummary) * shd_eng::kRing) != hipSuccess) {
        shd_eng_destroy(e);
        return SHD_ENOMEM;
    }
    EALLOC(e->d_halt, 1); EALLOC(e->d_next_rank, 1); EALLOC(e->d_trace_n, 1); EALLOC(e->d_ctl, 1);
    if (hipHostMalloc((void**)&e->h_ctl, sizeof(DevCtl)) != hipSuccess ||
        hipHostMalloc((void**)&e->h_seed, 2 * sizeof(DevSummary)) != hipSuccess) {
        shd_eng_destroy(e);
        return SHD_ENOMEM;
    }
    {
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
            e->wall_khz = khz;
    }
    for (auto& ev : e->bev) (void)hipEventCreate(&ev);
    P.halt = e->d_halt; P.next_rank = e->d_next_rank; P.trace_n = e->d_trace_n;
    P.pend_cap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(1u << 16, (uint64_t)n * (max_start + 4)), 1u << 30);
    P.remote_cap = (uint32_t)std::min<uint64_t>((uint64_t)n * P.inbox_cap, 1u << 30);
    {
        int rc;
        if ((rc = ealloc(e, &P.pend, P.pend_cap, false))) { shd_eng_destroy(e); return rc; }
        const bool multi = !(host_begin == 0 && host_end == H);
        if ((rc = ealloc(e, &P.remote, multi ? P.remote_cap : 1, false))) { shd_eng_destroy(e); return rc; }
        if (!multi) P.remote_cap = 0;
        e->trace_cap = m->trace ? std::max<uint64_t>(1u << 20, (uint64_t)n * 4096) : 1;
        if (m->trace) e->trace_cap = std::min<uint64_t>(e->trace_cap, 1ull << 27);
        if ((rc = ealloc(e, &P.trace_buf, e->trace_cap, false))) { shd_eng_destroy(e); return rc; }
        P.trace_cap = e->trace_cap;
    }
    hipStream_t s = e->stream;
    if (hipMemcpyAsync(e->d_rng0, m->host_rng, 4 * (size_t)H, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(e->d_bwd, m->bw_down_kibps, 8 * (size_t)H, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(e->d_bwu, m->bw_up_kibps, 8 * (size_t)H, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(e->d_host_att, host_att.data(), 4 * (size_t)H, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(e->d_cum, m->dest_cum, 8 * HC, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(e->d_guide, guide.data(), sizeof(DestGuide) * HC, hipMemcpyHostToDevice, s) != hipSuccess ||
        (m->host_heartbeat &&
         hipMemcpyAsync(e->d_host_hb, m->host_heartbeat, 8 * (size_t)H, hipMemcpyHostToDevice, s) != hipSuccess) ||
        (e->d_app_peer &&
         (hipMemcpyAsync(e->d_app_peer, e->app_peer_dev.data(), 4 * (size_t)H, hipMemcpyHostToDevice, s) != hipSuccess ||
          hipMemcpyAsync(e->d_app_mode, app_mode.data(), (size_t)H, hipMemcpyHostToDevice, s) != hipSuccess ||
          hipMemcpyAsync(e->d_app_nstart, app_nstart.data(), 4 * (size_t)H, hipMemcpyHostToDevice, s) != hipSuccess))) {
        shd_eng_destroy(e);
        return SHD_ENODEV;
    }
    e->h_rank.assign(pc->T, kNoRank);
    e->h_self_rank.assign(pc->T, kNoRank);
    if (hipMemcpyAsync(e->d_rank, e->h_rank.data(), 4 * (size_t)pc->T, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(e->d_self_rank, e->h_self_rank.data(), 4 * (size_t)pc->T, hipMemcpyHostToDevice, s) !=
            hipSuccess) {
        shd_eng_destroy(e);
        return SHD_ENODEV;
    }
    P.host_att = e->d_host_att;
    P.dest_cum = e->d_cum;
    P.dest_guide = e->d_guide;
    P.host_hb = e->d_host_hb;
    P.app_peer = e->d_app_peer;
    P.app_mode = e->d_app_mode;
    P.app_nstart = e->d_app_nstart;
    P.no_app_start = (m->queue_flags & SHD_QF_NO_APP_START) ? 1 : 0;
    // draw thresholds: x / RAND_MAX <= c  <=>  x <= draw_threshold(c)
    {
        // per host, from its own class's cumulative weights
        std::vector<int4> thr(H);
        std::vector<int32_t> cls_dst_thr(n_cls);
        for (int32_t cl = 0; cl < n_cls; cl++) cls_dst_thr[cl] = draw_threshold(m->dest_cum[(size_t)cl * H + H - 1]);
        for (int32_t h = 0; h < H; h++) {
            const int32_t cl = m->host_class ? (int32_t)m->host_class[h] : 0;
            const double* cum = m->dest_cum + (size_t)cl * H;
            // (a host after every draw -- its predecessor's cumulative weight
            // already 1: no draw of its own; the empty range, not INT32_MAX + 1)
            const int64_t lo = h ? (int64_t)draw_threshold(cum[h - 1]) + 1 : 0;
            thr[h].x = lo > INT32_MAX ? 1 : (int32_t)lo;
            thr[h].y = lo > INT32_MAX ? 0 : draw_threshold(cum[h]);
            thr[h].z = cls_dst_thr[cl];
            thr[h].w = cl;
        }
        const int32_t dst_thr0 = cls_dst_thr[0];
        // closed-form destinations: host h at attached index h, thresholds
        // thr[i] = floor((i+1) R / H) but for a few i (the exceptions).  Both
        // pick functions are step functions of x changing only at thr[i]+1
        // and f(i)+1, so checking every such x (and 0) checks them all.
        {
            constexpr uint64_t R = 2147483647ull;
            bool ok = getenv("SHD_NO_DEST_CLOSED") == nullptr && n_cls == 1;
            for (int32_t h = 0; h < H && ok; h++) ok = host_att[h] == h;
            std::vector<int32_t> ty(H);
            for (int32_t i = 0; i < H && ok; i++) ty[i] = draw_threshold(m->dest_cum[i]);   // (monotone; thr.y may be emptied)
            auto f = [&](int32_t i) { return (int64_t)(((uint64_t)(i + 1) * R) / (uint64_t)H); };
            auto pick_true = [&](int64_t x) {   // first i with thr[i] >= x
                return (int32_t)(std::lower_bound(ty.begin(), ty.end(), (int32_t)x) - ty.begin());
            };
            auto pick_closed = [&](int64_t x) {
                const uint64_t c = ((uint64_t)x * (uint64_t)H + (R - 1)) / R;
                return c ? (int32_t)c - 1 : 0;
            };
            std::vector<std::pair<int32_t, int32_t>> exc;
            for (int32_t i = 0; i < H && ok; i++) {
                if (f(i) == ty[i]) continue;
                const int64_t lo = std::min<int64_t>(f(i), ty[i]) + 1, hi = std::max<int64_t>(f(i), ty[i]);
                for (int64_t x = lo; x <= hi && ok; x++) {
                    if (x > dst_thr0) break;
                    const int32_t t = pick_true(x);
                    if (t != pick_closed(x)) {
                        if (exc.size() == (size_t)kDestExc) ok = false;
                        else exc.push_back({(int32_t)x, t});
                    }
                }
            }
            auto pick_exc = [&](int64_t x) {
                int32_t d = pick_closed(x);
                for (auto& p : exc) if (p.first == x) d = p.second;
                return d;
            };
            for (int32_t i = 0; i < H && ok; i++)
                for (int64_t x : {(int64_t)0, (int64_t)ty[i] + 1, f(i) + 1})
                    if (x <= dst_thr0 && pick_exc(x) != pick_true(x)) ok = false;
            P.dest_closed = ok ? 1 : 0;
            P.n_exc = ok ? (int32_t)exc.size() : 0;
            for (size_t j = 0; j < exc.size() && ok; j++) { P.exc_x[j] = exc[j].first; P.exc_d[j] = exc[j].second; }
        }
        if (hipMemcpyAsync(e->d_self_thr, thr.data(), sizeof(int4) * (size_t)H, hipMemcpyHostToDevice, e->stream) !=
                hipSuccess ||
            hipStreamSynchronize(e->stream) != hipSuccess) {
            shd_eng_destroy(e);
            return SHD_ENODEV;
        }
        P.self_thr = e->d_self_thr;
    }
    P.T = pc->T;
    P.complete = pc->complete; P.prefer_direct = pc->prefer_direct; P.directed = pc->directed;
    P.row = pc->d_row; P.dir = pc->d_dir; P.self = pc->d_self;
    P.adj = pc->d_adj;
    P.rank = e->d_rank; P.self_rank = e->d_self_rank;
    if (m->queue_flags & SHD_QF_COUNT_PATHS) {
        int rc;
        if ((rc = ealloc(e, &P.pcount, (size_t)pc->T * pc->T))) { shd_eng_destroy(e); return rc; }
    }
    if (m->queue_flags & SHD_QF_HEARTBEATS) {
        // heartbeats at k * interval < end_time, k >= 1 (none when end_time is 0)
        const uint64_t k = m->end_time > 0 ? (m->end_time - 1) / hb_min : 0;
        if (k > (1u << 20)) { shd_eng_destroy(e); return SHD_ERANGE; }
        P.hb_k = (uint32_t)k;
        e->heartbeats = true;
        int rc;
        if (k && (rc = ealloc(e, &P.hb, (size_t)n * k))) { shd_eng_destroy(e); return rc; }
    }
    P.feat = (m->trace ? F_TRACE : 0u) | (P.hb ? F_HB : 0u) | (P.pcount ? F_PCOUNT : 0u) |
             (P.host_hb ? F_HOSTHB : 0u) | (P.force_ambig ? F_AMBIG : 0u) |
             ((m->trace && (m->queue_flags & SHD_QF_TRACE_STATUS)) ? F_STATUS : 0u) |
             (P.app != SHD_APP_PHOLD ? F_APP : 0u);
    P.sum = e->d_sum;
    // the serial-equivalent window W: min over every latency a send can be
    // served (rows, direct values, self values) -> ceil(lat * 1e6) ns
    {
        unsigned long long* d_min = nullptr;
        if (hipMalloc((void**)&d_min, 8) != hipSuccess) { shd_eng_destroy(e); return SHD_ENOMEM; }
        unsigned long long init = kDistInf;
        (void)hipMemcpyAsync(d_min, &init, 8, hipMemcpyHostToDevice, s);
        const size_t TT = (size_t)pc->T * pc->T;
        const int blocks = (int)std::min<size_t>((TT + 255) / 256, 4096);
        if (pc->rows_mode) {
            hipLaunchKernelGGL(k_min_valid, dim3(blocks), dim3(256), 0, s, pc->d_row, TT, d_min);
            hipLaunchKernelGGL(k_min_valid, dim3((pc->T + 255) / 256), dim3(256), 0, s, pc->d_self,
                               (size_t)pc->T, d_min);
        }
        if (pc->complete || pc->prefer_direct)
            hipLaunchKernelGGL(k_min_valid, dim3(blocks), dim3(256), 0, s, pc->d_dir, TT, d_min);
        unsigned long long bits = 0;
        (void)hipMemcpyAsync(&bits, d_min, 8, hipMemcpyDeviceToHost, s);
        if (hipStreamSynchronize(s) != hipSuccess) { (void)hipFree(d_min); shd_eng_destroy(e); return SHD_ENODEV; }
        (void)hipFree(d_min);
        double ml;
        memcpy(&ml, &bits, 8);
        if (!(ml > 0.0) || bits == kDistInf) { shd_eng_destroy(e); return SHD_EINVAL; }
        e->window = (uint64_t)ceil(ml * (double)SHD_MS);
        if (e->window == 0) e->window = 1;
    }
    // calendar: bin width = the largest power of two <= W (Params complete below)
    if (!(m->queue_flags & SHD_QF_NO_CALENDAR)) {
        P.bin_shift = 63u - (uint32_t)__builtin_clzll(e->window);
        int rc;
        if ((rc = ealloc(e, &P.bins, n * kNB * kBinCap, false)) || (rc = ealloc(e, &P.bin_n, n * kNB)) ||
            (rc = ealloc(e, &P.bin_bits, n * kNBW))) {
            shd_eng_destroy(e);
            return rc;
        }
    }
    {   // the per-slot device copies of P
        int rc;
        if ((rc = ealloc(e, &e->d_pr, shd_eng::kRing, false))) { shd_eng_destroy(e); return rc; }
        std::vector<Params> pr(shd_eng::kRing, P);
        for (int i = 0; i < shd_eng::kRing; i++) pr[i].sum = &e->d_ring[i];
        if (hipMemcpyAsync(e->d_pr, pr.data(), sizeof(Params) * pr.size(), hipMemcpyHostToDevice, e->stream) !=
                hipSuccess ||
            hipStreamSynchronize(e->stream) != hipSuccess) {
            shd_eng_destroy(e);
            return SHD_ENODEV;
        }
    }
    {   // persistent rounds: every block resident (one per CU), one engine for all hosts
        const int grid = (e->nloc + P.hpw - 1) / P.hpw;
        int ncu = 0, per_cu = 0;
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
        const bool lean = lean_model(P);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lean ? reinterpret_cast<const void*>(&k_round_ps<true>)
                                                                       : reinterpret_cast<const void*>(&k_round_ps<false>),
                                                         kBlock, 0) != hipSuccess)
            per_cu = 0;
        (void)hipGetLastError();
        // (blocks of one wave: up to two per CU, below what LDS and registers admit)
        // SHD_SP_HOSTS=<n>: the sparse kernel with n hosts per block whatever the size
        // (it selects between exact paths: a knob for tests and measurements)
        const char* sp_env = getenv("SHD_SP_HOSTS");
        const uint32_t sp_force = sp_env ? (uint32_t)strtoul(sp_env, nullptr, 10) : 0u;
        e->ps_ok = e->h0 == 0 && e->nloc == H && ncu > 0 && per_cu >= 2 && grid <= 2 * ncu && !sp_force;
        size_t nshare = e->ps_ok ? (size_t)grid : 0;
        if (!e->ps_ok && e->h0 == 0 && e->nloc == H && ncu > 0) {
            // too many hosts for a resident wave each: blocks of sph hosts, about two per CU
            int per_cu_sp = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_sp,
                                                             lean ? reinterpret_cast<const void*>(&k_round_sp<true>)
                                                                  : reinterpret_cast<const void*>(&k_round_sp<false>),
                                                             kBlock, sp_dyn_bytes(kSpMaxHosts, false)) != hipSuccess)
                per_cu_sp = 0;
            (void)hipGetLastError();
            // about two blocks per CU (where occupancy admits two): at the C5 shard 256 hosts a
            // block ran 23.6 ms a step against 26.2 ms at one block of 512 per CU, and 250 k hosts
            // 28.5 ms at 512 against 38.7 ms at 1024 (profiles/r05/sph); three per CU lost again
            const uint64_t bpc = per_cu_sp >= 2 ? 2 : 1;
            const uint64_t per = ((uint64_t)e->nloc + bpc * ncu - 1) / (bpc * ncu);
            const uint32_t sph = sp_force ? (sp_force + 63) / 64 * 64
                                          : (uint32_t)std::max<uint64_t>(256, (per + 63) / 64 * 64);
            const uint32_t g = (uint32_t)(((uint64_t)e->nloc + sph - 1) / sph);
            const bool no_sp = getenv("SHD_NO_SP") != nullptr;   // perf knob: k_round_tl batches instead
            if (getenv("SHD_SP_VERBOSE"))
                fprintf(stderr, "shd: sparse rounds: %d CUs, %d blocks per CU resident, %u hosts per block, %u blocks\n",
                        ncu, per_cu_sp, sph, g);
            // the block's records resident in LDS for the batch where the grid still fits resident
            // with them (SHD_SP_NO_LREC: records in HBM, the A/B knob)
            int per_cu_lrec = 0;
            if (!getenv("SHD_SP_NO_LREC") && sph <= kSpMaxHosts &&
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_lrec,
                                                             lean ? reinterpret_cast<const void*>(&k_round_sp<true>)
                                                                  : reinterpret_cast<const void*>(&k_round_sp<false>),
                                                             kBlock, sp_dyn_bytes(sph, true)) != hipSuccess)
                per_cu_lrec = 0;
            (void)hipGetLastError();
            const bool lrec = per_cu_lrec >= 1 && g <= (uint32_t)(ncu * per_cu_lrec);
            if (getenv("SHD_SP_VERBOSE"))
                fprintf(stderr, "shd: sparse rounds: records in %s (%d blocks per CU with them)\n",
                        lrec ? "LDS" : "HBM", per_cu_lrec);
            if (!no_sp && per_cu_sp >= 1 && sph <= kSpMaxHosts && g <= (uint32_t)(ncu * per_cu_sp)) {
                e->sp_ok = true;
                e->sp_lrec = lrec;
                e->sp_dyn = sp_dyn_bytes(lrec ? sph : kSpMaxHosts, lrec);
                e->sp_forced = sp_force != 0;
                e->sp_hosts = sph;
                e->sp_grid = g;
                nshare = g;
            }
        }
        if (nshare) {
            int rc;
            if ((rc = ealloc(e, &e->d_pshare, 2 * nshare))) { shd_eng_destroy(e); return rc; }
        }
    }
    *out = e;
    return SHD_OK;
}

extern "C" int shd_eng_window(shd_eng* e, uint64_t* w) {
    if (!e || !w) return SHD_EINVAL;
    *w = e->window;
    return SHD_OK;
}

static DevSummary host_fresh_summary() {
    DevSummary z{};
    z.next_time = kInf;
    z.t_first = kInf;
    return z;
}

// device time of a round kernel from its summary's wall-clock stamps
static double round_kernel_ms(const shd_eng* e, const DevSummary& r) {
    if (r.t_first == kInf || r.t_last < r.t_first) return 0.0;
    return (double)(r.t_last - r.t_first) / e->wall_khz;
}

static int reset_summary(shd_eng* e) {
    DevSummary z = host_fresh_summary();
    SHD_HIP(hipMemcpyAsync(e->d_sum, &z, sizeof(z), hipMemcpyHostToDevice, e->stream));
    SHD_HIP(hipStreamSynchronize(e->stream));
    return SHD_OK;
}

static int read_summary(shd_eng* e) {
    SHD_HIP(hipMemcpyAsync(e->h_sum, e->d_sum, sizeof(DevSummary), hipMemcpyDeviceToHost, e->stream));
    SHD_HIP(hipStreamSynchronize(e->stream));
    return SHD_OK;
}

extern "C" int shd_eng_boot(shd_eng* e) {
    if (!e) return SHD_EINVAL;
    SHD_HIP(hipSetDevice(e->device));
    memset(e->h_sum, 0, sizeof(DevSummary));
    int rc = reset_summary(e);
    if (rc) return rc;
    if (e->P.bins) {   // empty calendar; every slot's time = kInf (never in a window)
        const size_t n = (size_t)e->nloc;
        SHD_HIP(hipMemsetAsync(e->P.bins, 0xFF, sizeof(shd_event) * n * kNB * kBinCap, e->stream));
        SHD_HIP(hipMemsetAsync(e->P.bin_n, 0, 4 * n * kNB, e->stream));
        SHD_HIP(hipMemsetAsync(e->P.bin_bits, 0, 4 * n * kNBW, e->stream));
    }
    const int grid = (e->nloc + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_boot, dim3(grid), dim3(kBlock), 0, e->stream, dp(e->P), e->d_rng0, e->d_bwd, e->d_bwu);
    SHD_HIP(hipGetLastError());
    if ((rc = read_summary(e))) return rc;
    e->parity = 0;
    e->booted = true;
    e->snap_valid = false;
    if (e->h_sum->error) return SHD_EOVERFLOW;
    return SHD_OK;
}

extern "C" int shd_eng_push_events(shd_eng* e, const shd_event* ev, uint64_t n) {
    if (!e || (n && !ev)) return SHD_EINVAL;
    if (!e->booted) return SHD_EINVAL;
    if (!n) return SHD_OK;
    e->snap_valid = false;   // a replay from the copy would miss these events
    if (n > (1u << 30)) return SHD_ERANGE;
    // two kinds: application starts of this engine's hosts (each consumes its
    // host's next event ID here), and packet deliveries from hosts outside this
    // engine (their sender's ID and packet id come with them)
    std::vector<shd_event> starts, pkts;
    for (uint64_t i = 0; i < n; i++) {
        const shd_event& x = ev[i];
        const bool local_dst = (int64_t)x.dst >= e->h0 && (int64_t)x.dst < (int64_t)e->h0 + e->nloc;
        const bool local_src = (int64_t)x.src >= e->h0 && (int64_t)x.src < (int64_t)e->h0 + e->nloc;
        if (!local_dst || x.time < e->t_done) return SHD_EINVAL;
        if (x.kind == SHD_EV_APP_START && x.src == x.dst) {
            starts.push_back(x);
            starts.back().pkt = 0;
        } else if (x.kind == SHD_EV_PACKET && !local_src && (int64_t)x.src < (int64_t)e->H) {
            pkts.push_back(x);
        } else {
            return SHD_EINVAL;
        }
    }
    // stable grouping of the starts by host: a host's starts keep their array order (its IDs)
    std::stable_sort(starts.begin(), starts.end(), [](const shd_event& a, const shd_event& b) { return a.dst < b.dst; });
    std::vector<uint32_t> off;
    for (size_t i = 0; i < starts.size(); i++)
        if (i == 0 || starts[i].dst != starts[i - 1].dst) off.push_back((uint32_t)i);
    off.push_back((uint32_t)starts.size());
    const uint32_t ngrp = (uint32_t)off.size() - 1;
    SHD_HIP(hipSetDevice(e->device));
    shd_event* d_ev = nullptr;
    uint32_t* d_off = nullptr;
    SHD_HIP(hipMalloc((void**)&d_ev, sizeof(shd_event) * n));
    if (hipMalloc((void**)&d_off, 4 * off.size()) != hipSuccess) { (void)hipFree(d_ev); return SHD_ENOMEM; }
    int rc = SHD_OK;
    e->P.sum = e->d_sum;
    if ((!starts.empty() && hipMemcpyAsync(d_ev, starts.data(), sizeof(shd_event) * starts.size(),
                                           hipMemcpyHostToDevice, e->stream) != hipSuccess) ||
        (!pkts.empty() && hipMemcpyAsync(d_ev + starts.size(), pkts.data(), sizeof(shd_event) * pkts.size(),
                                         hipMemcpyHostToDevice, e->stream) != hipSuccess) ||
        hipMemcpyAsync(d_off, off.data(), 4 * off.size(), hipMemcpyHostToDevice, e->stream) != hipSuccess)
        rc = SHD_ENODEV;
    if (!rc) {
        // the summary's next time is the loop's window start: seed it with the
        // host view, the kernels lower it to the earliest pushed time
        e->h_sum->error = 0;
        if (hipMemcpyAsync(e->d_sum, e->h_sum, sizeof(DevSummary), hipMemcpyHostToDevice, e->stream) != hipSuccess)
            rc = SHD_ENODEV;
    }
    const int parity = (int)(e->round & 1);
    if (!rc && ngrp) {
        hipLaunchKernelGGL(k_push, dim3((ngrp + 255) / 256), dim3(256), 0, e->stream, dp(e->P), (const shd_event*)d_ev,
                           (const uint32_t*)d_off, ngrp, parity);
        if (hipGetLastError() != hipSuccess) rc = SHD_ENODEV;
    }
    if (!rc && !pkts.empty()) {
        const uint32_t np = (uint32_t)pkts.size();
        hipLaunchKernelGGL(k_push_packets, dim3((np + 255) / 256), dim3(256), 0, e->stream, dp(e->P),
                           (const shd_event*)(d_ev + starts.size()), np, parity);
        if (hipGetLastError() != hipSuccess) rc = SHD_ENODEV;
    }
    if (!rc) rc = read_summary(e);
    (void)hipFree(d_ev);
    (void)hipFree(d_off);
    if (!rc && e->h_sum->error) rc = SHD_EOVERFLOW;
    return rc;
}

// the outbox of the last round (events for hosts of other engines or of the
// CPU side), copied to the caller's host array
extern "C" int shd_eng_take_remote(shd_eng* e, shd_event* out, uint64_t cap, uint64_t* n) {
    if (!e || !n) return SHD_EINVAL;
    const uint64_t cnt = std::min<uint64_t>(e->h_sum->n_remote, e->P.remote_cap);
    if (e->h_sum->n_remote > e->P.remote_cap) return SHD_EOVERFLOW;
    if (cnt > cap) { *n = cnt; return SHD_ERANGE; }
    SHD_HIP(hipSetDevice(e->device));
    if (cnt) {
        if (!out) return SHD_EINVAL;
        SHD_HIP(hipMemcpyAsync(out, e->P.remote, sizeof(shd_event) * cnt, hipMemcpyDeviceToHost, e->stream));
        SHD_HIP(hipStreamSynchronize(e->stream));
    }
    *n = cnt;
    return SHD_OK;
}

// first-touch resolution in serial order (DESIGN.md "First-touch rule"): sort
// the logged queries of ALL engines by the executing event's key, assign row
// ranks (identically on every engine), then finalize this engine's sends
static void sort_pending(std::vector<shd_pending>& recs) {
    std::sort(recs.begin(), recs.end(), [](const shd_pending& x, const shd_pending& y) {
        if (x.qtime != y.qtime) return x.qtime < y.qtime;
        if (x.qhost != y.qhost) return x.qhost < y.qhost;
        if (x.qsrc != y.qsrc) return x.qsrc < y.qsrc;
        if (x.qseq != y.qseq) return x.qseq < y.qseq;
        return x.qsub < y.qsub;
    });
}

extern "C" int shd_eng_round_kernel(shd_eng* e, uint64_t ws, uint64_t we, shd_round_summary* out) {
    if (!e || !e->booted || we <= ws || we - ws > e->window) return SHD_EINVAL;
    SHD_HIP(hipSetDevice(e->device));
    int rc = reset_summary(e);
    if (rc) return rc;
    const int grid = (e->nloc + e->P.hpw - 1) / e->P.hpw;
    e->P.sum = e->d_sum;
    SHD_HIP(hipEventRecord(e->ev0, e->stream));
    hipLaunchKernelGGL(k_round, dim3(grid), dim3(kBlock), 0, e->stream, dp(e->P), ws, we, e->parity);
    SHD_HIP(hipGetLastError());
    SHD_HIP(hipEventRecord(e->ev1, e->stream));
    if ((rc = read_summary(e))) return rc;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e->ev0, e->ev1);
    e->last_kernel_ms = ms;
    e->kernel_ms_total += ms;
    e->round_ws = ws;
    e->round_we = we;
    e->round_pending = e->h_sum->n_pending;
    e->round_events = e->h_sum->n_events;
    e->round_pkt = e->h_sum->n_pkt_events;
    e->round_active = e->h_sum->n_active;
    if (out) {
        out->window_start = ws; out->window_end = we;
        out->next_time = e->h_sum->next_time;
        out->n_events = e->h_sum->n_events; out->n_pkt_events = e->h_sum->n_pkt_events;
        out->n_pending = e->h_sum->n_pending; out->n_remote = e->h_sum->n_remote; out->error = e->h_sum->error;
    }
    return SHD_OK;
}

extern "C" int shd_eng_pending_copy(shd_eng* e, shd_pending* out, uint64_t cap, uint64_t* n) {
    if (!e || !n || (cap && !out)) return SHD_EINVAL;
    const uint64_t cnt = e->round_pending;
    if (cnt > e->P.pend_cap) return SHD_EOVERFLOW;
    if (cnt > cap) { *n = cnt; return SHD_ERANGE; }
    SHD_HIP(hipSetDevice(e->device));
    if (cnt) {
        SHD_HIP(hipMemcpyAsync(out, e->P.pend, sizeof(shd_pending) * cnt, hipMemcpyDeviceToHost, e->stream));
        SHD_HIP(hipStreamSynchronize(e->stream));
    }
    *n = cnt;
    return SHD_OK;
}

// row ranks for a round's first-touch log, in serial order (the device holds
// the ranks; they are read, extended and written back)
static int assign_ranks(shd_eng* e, const shd_pending* all, uint64_t n_all) {
    SHD_HIP(hipMemcpyAsync(e->h_rank.data(), e->d_rank, 4 * (size_t)e->pc->T, hipMemcpyDeviceToHost, e->stream));
    SHD_HIP(hipMemcpyAsync(e->h_self_rank.data(), e->d_self_rank, 4 * (size_t)e->pc->T, hipMemcpyDeviceToHost,
                           e->stream));
    SHD_HIP(hipMemcpyAsync(&e->next_rank, e->d_next_rank, 4, hipMemcpyDeviceToHost, e->stream));
    SHD_HIP(hipStreamSynchronize(e->stream));
    std::vector<shd_pending> recs(all, all + n_all);
    sort_pending(recs);
    const bool directed = e->pc->directed;
    for (const shd_pending& r : recs) {
        const int32_t a = (int32_t)r.a, b = (int32_t)r.b;
        if (a < 0 || b < 0 || a >= e->pc->T || b >= e->pc->T) return SHD_EINVAL;
        if (a == b) {
            if (e->h_rank[a] == kNoRank && e->h_self_rank[a] == kNoRank) e->h_self_rank[a] = e->next_rank++;
        } else if (directed) {
            if (e->h_rank[a] == kNoRank) e->h_rank[a] = e->next_rank++;
        } else {
            if (e->h_rank[a] == kNoRank && e->h_rank[b] == kNoRank) e->h_rank[a] = e->next_rank++;
        }
    }
    const int32_t T = e->pc->T;
    SHD_HIP(hipMemcpyAsync(e->d_rank, e->h_rank.data(), 4 * (size_t)T, hipMemcpyHostToDevice, e->stream));
    SHD_HIP(hipMemcpyAsync(e->d_self_rank, e->h_self_rank.data(), 4 * (size_t)T, hipMemcpyHostToDevice, e->stream));
    SHD_HIP(hipMemcpyAsync(e->d_next_rank, &e->next_rank, 4, hipMemcpyHostToDevice, e->stream));
    SHD_HIP(hipStreamSynchronize(e->stream));
    return SHD_OK;
}

extern "C" int shd_eng_resolve(shd_eng* e, const shd_pending* all, uint64_t n_all) {
    if (!e || (n_all && !all)) return SHD_EINVAL;
    if (!n_all) return SHD_OK;
    SHD_HIP(hipSetDevice(e->device));
    int rc = assign_ranks(e, all, n_all);
    if (rc) return rc;
    const uint32_t n = (uint32_t)e->round_pending;
    if (n) {
        hipLaunchKernelGGL(k_finalize, dim3((n + 255) / 256), dim3(256), 0, e->stream, dp(e->P),
                           (const Pending*)e->P.pend, n, e->parity ^ 1);
        SHD_HIP(hipGetLastError());
    }
    e->pending_resolved += n;
    return SHD_OK;
}

extern "C" int shd_eng_end_round(shd_eng* e, shd_round_summary* out) {
    if (!e) return SHD_EINVAL;
    int rc = read_summary(e);
    if (rc) return rc;
    e->parity ^= 1;
    e->round++;
    e->t_done = std::max<uint64_t>(e->t_done, e->round_we);
    if (out) {
        out->window_start = e->round_ws; out->window_end = e->round_we;
        out->next_time = e->h_sum->next_time;
        out->n_events = e->round_events; out->n_pkt_events = e->round_pkt;
        out->n_pending = e->round_pending; out->n_remote = e->h_sum->n_remote; out->error = e->h_sum->error;
    }
    // finalized: a later shd_eng_resolve without a round (first touches of
    // another side only) assigns ranks and finalizes nothing
    e->round_pending = 0;
    if (e->h_sum->error & SHD_ERR_AMBIGUOUS) return SHD_EAMBIG;
    if (e->h_sum->error) return SHD_EOVERFLOW;
    return SHD_OK;
}

extern "C" int shd_eng_run_round(shd_eng* e, uint64_t ws, uint64_t we, shd_round_summary* out) {
    int rc = shd_eng_round_kernel(e, ws, we, out);
    if (rc) return rc;
    if (e->round_pending) {
        std::vector<shd_pending> recs(e->round_pending);
        uint64_t n = 0;
        if ((rc = shd_eng_pending_copy(e, recs.data(), recs.size(), &n))) return rc;
        if ((rc = shd_eng_resolve(e, recs.data(), n))) return rc;
    }
    return shd_eng_end_round(e, out);
}

// Device-driven rounds (single engine): a batch of kBatch rounds is one
// captured graph of k_round_dev launches, each reading its window start from
// the previous round's summary on the device, its stop time and parity from
// the batch control block, and resolving small first-touch logs in its last
// block.  The host reads the batch's summaries once per batch.  A round whose
// first-touch log is too large for the device path halts the batch; the host
// resolves it (shd_eng_resolve) and resumes after it.
static int enqueue_batch(shd_eng* e) {
    constexpr int B = shd_eng::kBatch;
    const int grid = (e->nloc + e->P.hpw - 1) / e->P.hpw;
    for (int i = 0; i < B; i++) {
        hipLaunchKernelGGL(k_round_dev, dim3(grid), dim3(kBlock), 0, e->stream, round_args(e->P),
                           (const DevSummary*)&e->d_ring[i], (const DevCtl*)e->d_ctl,
                           (const DParams*)(e->d_pr + i + 1), &e->d_ring[i + 2], i, e->window);
    }
    SHD_HIP(hipGetLastError());
    return SHD_OK;
}

static int enqueue_batch_tl(shd_eng* e) {
    constexpr int B = shd_eng::kBatch;
    const int grid = (e->nloc + e->P.hpw - 1) / e->P.hpw;
    for (int i = 0; i < B; i++) {
        // (the lean instantiation for models with no optional feature: ParamsT::feat == 0)
        if (lean_model(e->P))
            hipLaunchKernelGGL(k_round_tl<true>, dim3(grid), dim3(kBlock), 0, e->stream, e->window, i, &e->d_ring[i],
                               (const DevCtl*)e->d_ctl, e->d_tpart, (const DParams*)(e->d_pr + i + 1),
                               &e->d_ring[i + 2], round_args(e->P));
        else
            hipLaunchKernelGGL(k_round_tl<false>, dim3(grid), dim3(kBlock), 0, e->stream, e->window, i, &e->d_ring[i],
                               (const DevCtl*)e->d_ctl, e->d_tpart, (const DParams*)(e->d_pr + i + 1),
                               &e->d_ring[i + 2], round_args(e->P));
    }
    hipLaunchKernelGGL(k_fold_tl, dim3(1), dim3(64), 0, e->stream, (const TlPart*)e->d_tpart, (uint32_t)grid, B - 1,
                       &e->d_ring[B], e->d_halt);
    SHD_HIP(hipGetLastError());
    return SHD_OK;
}

static int launch_batch(shd_eng* e, bool tl) {
    static const bool no_graph = getenv("SHD_NO_GRAPH") != nullptr;
    if (no_graph) return tl ? enqueue_batch_tl(e) : enqueue_batch(e);
    hipGraphExec_t& ge = tl ? e->batch_graph_tl : e->batch_graph;
    if (!ge) {
        hipGraph_t gr = nullptr;
        SHD_HIP(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
        const int rc = tl ? enqueue_batch_tl(e) : enqueue_batch(e);
        const hipError_t ec = hipStreamEndCapture(e->stream, &gr);
        if (rc) return rc;
        SHD_HIP(ec);
        const hipError_t ei = hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
        (void)hipGraphDestroy(gr);
        SHD_HIP(ei);
    }
    SHD_HIP(hipGraphLaunch(ge, e->stream));
    return SHD_OK;
}

// a persistent batch: nb rounds in one launch (k_round_ps); the shares' tags
// advance past the batch whatever it ran
// when launch-per-round batches beat k_round_sp: the last batch's packet events per host-round
// above 0.08, or its active hosts above 30 % of the hosts (several passes a block).  Measured
// per batch kind over whole runs (profiles/r05/sph/spverb/): C5's shard decays from 90 % active
// hosts at 0.35 events per active host, where the sparse round loses up to 46 % (0.67: 82 against
// 60 µs a round), through a tie at 0.09 events per host-round (46 against 47 µs) to 4 % active,
// where it wins by a third (23 against 33 µs); C4 at 14 % active hosts but 1.4 events each
// (0.2 per host-round) runs 226 µs sparse against 128 µs; C3 at 100 k hosts (0.3 per host-round)
// 45 against 43 µs.  (SHD_SP_DENSE_FRAC / SHD_SP_DENSE_PKT: other thresholds, for measurements)
static double env_or(const char* name, double dflt) {
    const char* v = getenv(name);
    return v ? strtod(v, nullptr) : dflt;
}
static bool sp_dense_batch(uint64_t rounds, uint64_t active, uint64_t pkt, uint64_t nloc) {
    static const double f_act = env_or("SHD_SP_DENSE_FRAC", 0.3), f_pkt = env_or("SHD_SP_DENSE_PKT", 0.08);
    const double hr = (double)rounds * (double)nloc;
    return (double)active > f_act * hr || (double)pkt > f_pkt * hr;
}

static int launch_batch_ps(shd_eng* e, int nb) {
    const uint64_t ticks = (uint64_t)(2.0 * e->wall_khz * 1000.0);   // 2 s: a block that never comes
    const bool lean = lean_model(e->P);   // (the lean instantiations)
    if (e->sp_ok) {
        hipLaunchKernelGGL(lean ? k_round_sp<true> : k_round_sp<false>, dim3(e->sp_grid), dim3(kBlock), e->sp_dyn,
                           e->stream, e->window, nb, e->d_ring, (const DevCtl*)e->d_ctl, e->d_pshare,
                           (const DParams*)e->d_pr, ticks, e->sp_hosts, (int)e->sp_lrec);
    } else {
        const int grid = (e->nloc + e->P.hpw - 1) / e->P.hpw;
        hipLaunchKernelGGL(lean ? k_round_ps<true> : k_round_ps<false>, dim3(grid), dim3(kBlock), 0, e->stream,
                           e->window, nb, e->d_ring, (const DevCtl*)e->d_ctl, e->d_pshare, (const DParams*)e->d_pr,
                           ticks);
    }
    SHD_HIP(hipGetLastError());
    e->ps_epoch += (uint32_t)nb;
    if (e->ps_epoch < (uint32_t)nb + 1u) e->ps_epoch = 1;   // (wrapped: restart past 0)
    return SHD_OK;
}

// ---- protected rounds.  A first-touch send whose drop decision differs
// under the two candidate rows cannot be decided before the round's log is
// ranked (probability ~3.5e-7 per logged send on the bench graph: it fired
// at 1M hosts, 16M sends logged at the application start).  Rounds that may
// log many first touches -- every round until one has logged, and the round
// after one that logged kProtectMin or more -- run one at a time behind a
// copy of the engine's device state; an ambiguous round is rolled back,
// ranked from its own log (the log does not depend on the decisions: queries
// come from the RNG stream, and the drop decision only moves event IDs), and
// rerun, now with no undecided send.
static constexpr uint64_t kProtectMin = 64;

static bool protect_all() { return test_hook("SHD_PROTECT_ALL"); }
static bool protect_off() { return getenv("SHD_NO_PROTECT") != nullptr; }

// the state copy's memory: device memory, or where that is exhausted (round 6:
// a 1 M-host engine beside its state copy on a full device) pinned host memory,
// else pageable host memory -- the copy then crosses PCIe and a protected round
// costs more, but the rounds stay protected and ambiguous first touches stay
// recoverable instead of failing the run
static void snap_free(shd_eng* e) {
    for (size_t i = 0; i < e->snap.size(); i++) {
        if (!e->snap[i]) continue;
        const uint8_t k = i < e->snap_kind.size() ? e->snap_kind[i] : 0;
        if (k == 0) (void)hipFree(e->snap[i]);
        else if (k == 1) (void)hipHostFree(e->snap[i]);
        else free(e->snap[i]);
    }
    e->snap.clear();
    e->snap_kind.clear();
}
static int snapshot_state(shd_eng* e, bool restore) {
    if (!restore && e->snap.size() != e->allocs.size()) {
        bool warned = false;
        for (size_t i = e->snap.size(); i < e->allocs.size(); i++) {
            const size_t bytes = e->alloc_bytes[i];
            void* q = nullptr;
            uint8_t kind = 0;
            if (test_hook("SHD_SNAP_NO_DEVICE") || hipMalloc(&q, bytes) != hipSuccess) {
                (void)hipGetLastError();
                q = nullptr;
                kind = 1;
                if (hipHostMalloc(&q, bytes, hipHostMallocDefault) != hipSuccess) {
                    (void)hipGetLastError();
                    kind = 2;
                    q = malloc(bytes);
                }
                if (!q) {
                    snap_free(e);
                    e->snap_failed = true;
                    fprintf(stderr, "libshdgpu: no memory for the protected-round state copy; "
                                    "rounds run unprotected (an ambiguous first touch fails the run)\n");
                    return SHD_ENOMEM;
                }
                if (!warned && getenv("SHD_VERBOSE"))
                    fprintf(stderr, "libshdgpu: the protected-round state copy in host memory (%s)\n",
                            kind == 1 ? "pinned" : "pageable");
                warned = true;
            }
            e->snap.push_back(q);
            e->snap_kind.push_back(kind);
        }
    }
    for (size_t i = 0; i < e->allocs.size(); i++) {
        void* dst = restore ? e->allocs[i] : e->snap[i];
        const void* src = restore ? e->snap[i] : e->allocs[i];
        const hipMemcpyKind k = e->snap_kind[i] == 0 ? hipMemcpyDeviceToDevice
                                : restore ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
        SHD_HIP(hipMemcpyAsync(dst, src, e->alloc_bytes[i], k, e->stream));
    }
    if (std::any_of(e->snap_kind.begin(), e->snap_kind.end(), [](uint8_t k) { return k == 2; }))
        SHD_HIP(hipStreamSynchronize(e->stream));   // (pageable copies: done before the host moves on)
    return SHD_OK;
}

// a state copy at the start of the round about to run from window start `next`
static int take_restore_point(shd_eng* e, uint64_t next) {
    const int rc = snapshot_state(e, false);
    if (rc) { e->snap_valid = false; return rc; }
    e->snap_valid = true;
    e->snap_round = e->round;
    e->snap_parity = e->parity;
    e->snap_sum = *e->h_sum;
    e->snap_next = next;
    e->snap_stops.clear();
    return SHD_OK;
}

static bool replay_off() { return getenv("SHD_NO_REPLAY") != nullptr; }
// rounds after which a restore point is renewed (the test build: SHD_RESTORE_EVERY)
static uint64_t restore_every() {
#ifdef SHD_TEST_HOOKS
    if (const char* v = getenv("SHD_RESTORE_EVERY")) return strtoull(v, nullptr, 10);
#endif
    return 1ull << 16;
}

static bool want_protect(const shd_eng* e) {
    if (protect_off() || e->snap_failed) return false;
    // complete graphs serve the direct value, which does not depend on which
    // endpoint came first: nothing is ever logged, nothing can be ambiguous
    if (e->P.complete && !protect_all()) return false;
    return protect_all() || !e->logged_any || e->last_logged >= kProtectMin;
}

// one protected round [ws, we) (host-driven, k_round); returns its summary
static int protected_round(shd_eng* e, uint64_t ws, uint64_t we, shd_round_summary* out, uint32_t* reruns) {
    int rc = take_restore_point(e, ws);
    if (rc == SHD_ENOMEM) return shd_eng_run_round(e, ws, we, out);
    if (rc) return rc;
    const int parity0 = e->parity;
    const uint64_t round0 = e->round;
    const DevSummary sum0 = *e->h_sum;
    if ((rc = shd_eng_round_kernel(e, ws, we, nullptr))) return rc;
    if ((e->h_sum->error & SHD_ERR_AMBIGUOUS) && !(e->h_sum->error & ~(uint32_t)SHD_ERR_AMBIGUOUS) &&
        e->round_pending && e->round_pending <= e->P.pend_cap) {
        std::vector<shd_pending> recs(e->round_pending);
        uint64_t n = 0;
        if ((rc = shd_eng_pending_copy(e, recs.data(), recs.size(), &n))) return rc;
        // roll back, keep nothing of the round but the ranks of its log
        if ((rc = snapshot_state(e, true))) return rc;
        e->parity = parity0;
        e->round = round0;
        *e->h_sum = sum0;
        if ((rc = assign_ranks(e, recs.data(), n))) return rc;
        (*reruns)++;
        if ((rc = shd_eng_round_kernel(e, ws, we, nullptr))) return rc;
        if (e->round_pending) {   // every pair of the log is ranked now
            e->h_sum->error |= SHD_ERR_INTERNAL;
            return shd_eng_end_round(e, out);
        }
    }
    if (e->round_pending) {
        std::vector<shd_pending> recs(e->round_pending);
        uint64_t n = 0;
        if ((rc = shd_eng_pending_copy(e, recs.data(), recs.size(), &n))) return rc;
        if ((rc = shd_eng_resolve(e, recs.data(), n))) return rc;
    }
    return shd_eng_end_round(e, out);
}

// A round whose first touches are ranked with another side's (one lazy path
// cache across a co-simulation, INTEGRATION.md "Mixed CPU/GPU hosts"): the
// kernel behind a state copy when first touches may still come (want_protect);
// shd_eng_round_retry rolls back to it, ranks `all` in serial order and runs
// the window again (an ambiguous first-touch drop decision: the other side's
// first touches of the window may rank rows before the engine's)
extern "C" int shd_eng_round_begin(shd_eng* e, uint64_t ws, uint64_t we, shd_round_summary* out) {
    if (!e || !e->booted || we <= ws || we - ws > e->window) return SHD_EINVAL;
    SHD_HIP(hipSetDevice(e->device));
    e->rb_snap = false;
    e->snap_valid = false;   // the co-simulation's rounds: the copy is the retry's only
    if (want_protect(e)) {
        const int rc = snapshot_state(e, false);
        if (rc == SHD_OK) {
            e->rb_snap = true;
            e->rb_parity = e->parity;
            e->rb_round = e->round;
            e->rb_sum = *e->h_sum;
            e->rb_ws = ws;
            e->rb_we = we;
        } else if (rc != SHD_ENOMEM) {
            return rc;
        }
    }
    const int rc = shd_eng_round_kernel(e, ws, we, out);
    if (rc) return rc;
    e->last_logged = e->round_pending;
    if (e->round_pending) e->logged_any = true;
    return SHD_OK;
}

extern "C" int shd_eng_round_retry(shd_eng* e, const shd_pending* all, uint64_t n_all, shd_round_summary* out) {
    if (!e || (n_all && !all)) return SHD_EINVAL;
    if (!e->rb_snap) return SHD_EAMBIG;   // not protected: the ambiguity stands
    SHD_HIP(hipSetDevice(e->device));
    e->rb_snap = false;
    int rc = snapshot_state(e, true);
    if (rc) return rc;
    e->parity = e->rb_parity;
    e->round = e->rb_round;
    *e->h_sum = e->rb_sum;
    if ((rc = assign_ranks(e, all, n_all))) return rc;
    if ((rc = shd_eng_round_kernel(e, e->rb_ws, e->rb_we, out))) return rc;
    // every first touch of the window is ranked now: the engine's (its queries
    // after an ambiguous one share their source with it) and the other side's
    if (e->round_pending) {
        e->h_sum->error |= SHD_ERR_INTERNAL;
        if (out) out->error = e->h_sum->error;
    }
    return SHD_OK;
}

// An unprotected round (a batch round) logged a first touch whose drop
// decision differs under the two candidate rows: nothing of it can be kept.
// Go back to the last restore point, run the rounds from there to the
// ambiguous round's start again, and run that round protected (rolled back to
// its own copy, its log ranked, run again).  None of the replayed rounds can
// be ambiguous: they make the same sends with the same draws, and every
// vertex ranked in the first run is ranked now (the ranks assigned since the
// copy are restored with it and assigned again in the same serial order), so
// a send is undecided in the replay only if it was undecided and decidable
// the first time.  No snapshot of the round itself is needed.
static int replay_ambiguous(shd_eng* e, uint64_t ws, uint64_t stop, shd_round_summary* r, shd_run_stats* s) {
    if (!e->snap_valid || e->in_replay) return SHD_EAMBIG;
    int rc = snapshot_state(e, true);
    if (rc) return rc;
    e->round = e->snap_round;
    e->parity = e->snap_parity;
    *e->h_sum = e->snap_sum;
    e->h_sum->next_time = e->snap_next;
    e->tl_ready = false;
    SHD_HIP(hipStreamSynchronize(e->stream));
    const uint64_t round0 = e->round;
    const double kms = e->kernel_ms_total;
    std::vector<uint64_t> stops = e->snap_stops;   // (a protected round of the replay takes a new copy)
    // the restore point's own round runs protected again: it may be the
    // protected round that took the copy and was ambiguous itself (rolled back
    // and rerun from its log), which unprotected would be ambiguous again
    if (e->snap_next < ws) {
        uint64_t we0 = e->snap_next + e->window;
        const uint64_t stop0 = stops.empty() ? stop : stops.front();
        if (we0 > stop0 || we0 < e->snap_next) we0 = stop0;
        shd_round_summary r0{};
        e->in_replay = true;
        rc = protected_round(e, e->snap_next, we0, &r0, &s->n_rounds_rerun);
        e->in_replay = false;
        if (rc) return rc;
        e->h_sum->next_time = r0.next_time;
    }
    stops.push_back(ws);
    e->in_replay = true;
    double sub_ms = 0;
    for (const uint64_t b : stops) {
        if (b <= e->h_sum->next_time || b > ws) continue;
        shd_run_stats sub{};
        rc = shd_eng_run_until(e, b, &sub);
        sub_ms += sub.device_ms_round_kernel;
        s->n_rounds_rerun += sub.n_rounds_rerun;
        if (rc) break;
    }
    e->in_replay = false;
    e->kernel_ms_total = kms + sub_ms;
    if (rc) return rc;
    if (e->h_sum->next_time != ws) return SHD_EAMBIG;   // (the replay did not reach the round: cannot happen)
    s->n_rounds_replayed += e->round - round0;
    uint64_t we = ws + e->window;
    if (we > stop || we < ws) we = stop;
    rc = protected_round(e, ws, we, r, &s->n_rounds_rerun);
    s->n_rounds_protected++;
    return rc;
}

extern "C" int shd_eng_run_until(shd_eng* e, uint64_t t_stop, shd_run_stats* st) {
    if (!e) return SHD_EINVAL;
    // a partial engine's sends to hosts outside it leave by rounds
    // (shd_eng_run_round + shd_eng_take_remote) or a group, never a batch
    if (e->h0 != 0 || e->nloc != e->H) return SHD_EINVAL;
    auto t0 = std::chrono::steady_clock::now();
    int rc = SHD_OK;
    if (!e->booted && (rc = shd_eng_boot(e))) return rc;
    SHD_HIP(hipSetDevice(e->device));
    shd_run_stats s{};
    s.window_ns = e->window;
    const uint64_t stop = std::min<uint64_t>(t_stop, e->P.end_time);
    uint64_t next = e->h_sum->next_time;
    if (!e->in_replay) e->kernel_ms_total = 0;
    const uint64_t pend0 = e->pending_resolved;
    // a restore point for an ambiguous unprotected round (replay_ambiguous);
    // complete graphs never log a first touch.  A point more than
    // restore_every() rounds old is renewed -- here and between the batches of
    // this call, after a batch that ended cleanly -- so that a replay never
    // reruns more than that plus one batch (a copy of the state every 2^16
    // rounds: 0.01 % of C3's run, 0.6 % of the 1 M-host shard's)
    const uint64_t every = restore_every();
    const bool stale = e->snap_valid && e->round - e->snap_round > every;
    if ((!e->snap_valid || stale) && !e->snap_failed && !e->P.complete && !replay_off() && next < stop &&
        !want_protect(e)) {
        const int rc0 = take_restore_point(e, next);
        if (rc0 && rc0 != SHD_ENOMEM) return rc0;
    }
    constexpr int B = shd_eng::kBatch, R = shd_eng::kRing;
    static_assert(R >= B + 2, "summary ring");
    while (next < stop && rc == SHD_OK) {
        if (want_protect(e)) {
            uint64_t we = next + e->window;
            if (we > stop || we < next) we = stop;
            shd_round_summary r{};
            const uint64_t pend_before = e->pending_resolved;
            rc = protected_round(e, next, we, &r, &s.n_rounds_rerun);
            s.n_rounds_protected++;
            if (rc && rc != SHD_EAMBIG && rc != SHD_EOVERFLOW) break;
            s.n_rounds++;
            s.n_events += r.n_events;
            s.n_pkt_events += r.n_pkt_events;
            s.n_host_rounds += e->round_active;   // the kept run of the round
            s.final_time = we;
            if (r.error) { s.error = r.error; break; }
            e->last_logged = e->pending_resolved - pend_before;
            if (e->last_logged) e->logged_any = true;
            e->tl_ready = e->last_logged == 0;
            next = r.next_time;
            continue;
        }
        // a stale restore point renewed between batches (the state is at a
        // round start, window start `next`, as at a call's entry), so that the
        // rounds a replay reruns stay bounded within one long call too
        if (e->snap_valid && !e->in_replay && e->round - e->snap_round > every && !e->snap_failed &&
            !replay_off()) {
            e->h_sum->next_time = next;
            const int rc0 = take_restore_point(e, next);
            if (rc0 && rc0 != SHD_ENOMEM) { rc = rc0; break; }
            s.n_restore_points++;
        }
        // slot 0 carries the window start; rounds use slots 1..B
        e->h_seed[0] = host_fresh_summary();
        e->h_seed[0].next_time = next;
        e->h_seed[1] = host_fresh_summary();
        e->h_ctl->stop = stop;
        e->h_ctl->round_base = e->round;
        e->h_ctl->xtag = e->ps_epoch;   // persistent rounds: round i's shares are tagged ps_epoch + i
        SHD_HIP(hipMemcpyAsync(e->d_ring, e->h_seed, 2 * sizeof(DevSummary), hipMemcpyHostToDevice, e->stream));
        SHD_HIP(hipMemcpyAsync(e->d_ctl, e->h_ctl, sizeof(DevCtl), hipMemcpyHostToDevice, e->stream));
        SHD_HIP(hipMemsetAsync(e->d_halt, 0, 4, e->stream));
        SHD_HIP(hipEventRecord(e->bev[0], e->stream));
        static const bool no_tl = getenv("SHD_NO_TL") != nullptr;
        static const bool no_ps = getenv("SHD_NO_PS") != nullptr;   // perf knob: launch-per-round batches only
        const bool tl = e->tl_ready && !no_tl;
        // the sparse kernel scans and compacts its blocks' active hosts every
        // round: it wins while few hosts are active (C5 at 125 k hosts: 4 % of
        // the hosts per round, 25.3 against 30.8 us per round), launch-per-round
        // batches when many are (C4: 14 %, 146 against 211 us; C3 at 100 k: 37 %,
        // 43 against 63 us).  Both are exact: the choice follows the last batch.
        const bool ps = tl && (e->ps_ok || (e->sp_ok && !e->sp_dense)) && !no_ps;
        const int nb = ps ? shd_eng::kPsBatch : B;
        if (ps) {
            if ((rc = launch_batch_ps(e, nb))) break;
            s.n_batches_persistent++;
            if (e->sp_ok) s.n_batches_sparse++;
        } else if ((rc = launch_batch(e, tl))) {
            break;
        }
        s.n_batches++;
        if (tl) s.n_batches_ticketless++;
        SHD_HIP(hipEventRecord(e->bev[1], e->stream));
        uint32_t halt = 0;
        SHD_HIP(hipMemcpyAsync(e->h_ring, e->d_ring, sizeof(DevSummary) * (nb + 1), hipMemcpyDeviceToHost, e->stream));
        SHD_HIP(hipMemcpyAsync(&halt, e->d_halt, 4, hipMemcpyDeviceToHost, e->stream));
        SHD_HIP(hipStreamSynchronize(e->stream));
        {
            float ms = 0;
            if (hipEventElapsedTime(&ms, e->bev[0], e->bev[1]) == hipSuccess) s.device_ms_launches += ms;
        }
        // ticketless batches unless first touches come thick: a ticketless
        // round that logs halts its batch for the host's resolution, a
        // ticketed one resolves a small log on the device.  After a batch
        // with at most one logging round the next batch is ticketless (the
        // late, rare logs cost one halt each); after more, it is ticketed.
        uint32_t n_logs = 0;
        uint64_t b_rounds = 0, b_active = 0, b_pkt = 0;
        double b_ms = 0;
        bool amb = false;
        uint64_t amb_ws = 0;
        for (int i = 0; i < nb; i++) {
            const DevSummary& r = e->h_ring[i + 1];
            const uint64_t ws = e->h_ring[i].next_time;
            if (ws >= stop) { next = ws; break; }   // the rest only forwarded the time
            const double ms = round_kernel_ms(e, r);
            e->kernel_ms_total += ms;
            e->last_kernel_ms = ms;
            if ((r.error & SHD_ERR_AMBIGUOUS) && !(r.error & ~(uint32_t)SHD_ERR_AMBIGUOUS) && e->snap_valid &&
                !e->in_replay && !replay_off()) {
                amb = true;   // this round and the batch's later ones are dropped: replay_ambiguous
                amb_ws = ws;
                break;
            }
            if (r.n_pending) n_logs++;
            const bool halted_here = halt && r.n_pending > (tl ? 0ull : (unsigned long long)kResolveMax);
            s.n_rounds++;
            s.n_events += r.n_events;
            s.n_pkt_events += r.n_pkt_events;
            s.n_host_rounds += r.n_active;
            b_rounds++;
            b_active += r.n_active;
            b_pkt += r.n_pkt_events;
            b_ms += ms;
            uint64_t we = ws + e->window;
            if (we > stop || we < ws) we = stop;
            s.final_time = we;
            e->round++;
            e->parity = (int)(e->round & 1);
            if (halted_here) {
                // host resolution of this round's log, then resume after it
                e->round_pending = r.n_pending;
                *e->h_sum = r;
                SHD_HIP(hipMemcpyAsync(e->d_sum, &r, sizeof(r), hipMemcpyHostToDevice, e->stream));
                std::vector<shd_pending> recs(r.n_pending);
                uint64_t n = 0;
                const int saved_parity = e->parity;
                e->parity = (int)((e->round - 1) & 1);   // the halted round's parity
                e->P.sum = e->d_sum;
                if ((rc = shd_eng_pending_copy(e, recs.data(), recs.size(), &n)) ||
                    (rc = shd_eng_resolve(e, recs.data(), n)) || (rc = read_summary(e))) {
                    e->parity = saved_parity;
                    break;
                }
                e->parity = saved_parity;
                e->last_logged = r.n_pending;
                e->logged_any = true;
                next = e->h_sum->next_time;
                if (e->h_sum->error) {
                    s.error = e->h_sum->error;
                    rc = (e->h_sum->error & SHD_ERR_AMBIGUOUS) ? SHD_EAMBIG : SHD_EOVERFLOW;
                }
                break;
            }
            if (r.n_pending) e->pending_resolved += r.n_pending;
            e->last_logged = r.n_pending;
            if (r.n_pending) e->logged_any = true;
            if (r.error) {
                s.error = r.error;
                rc = (r.error & SHD_ERR_AMBIGUOUS) ? SHD_EAMBIG : SHD_EOVERFLOW;
                break;
            }
            next = r.next_time;
        }
        e->tl_ready = n_logs <= 1;
        if (b_rounds && tl && getenv("SHD_SP_VERBOSE"))
            fprintf(stderr, "shd: batch %s rounds %llu active/round %.4f pkt/round %.1f us/round %.2f\n",
                    e->sp_ok && !e->sp_dense ? "sp" : "tl", (unsigned long long)b_rounds,
                    (double)b_active / ((double)b_rounds * (double)e->nloc), (double)b_pkt / (double)b_rounds,
                    b_ms * 1e3 / (double)b_rounds);
        if (b_rounds && tl && !e->sp_forced) e->sp_dense = sp_dense_batch(b_rounds, b_active, b_pkt, (uint64_t)e->nloc);
        if (amb) {
            uint64_t we = amb_ws + e->window;
            if (we > stop || we < amb_ws) we = stop;
            shd_round_summary r{};
            const uint64_t pend_before = e->pending_resolved;
            rc = replay_ambiguous(e, amb_ws, stop, &r, &s);
            if (rc && !(rc == SHD_EOVERFLOW && r.error)) break;
            s.n_rounds++;
            s.n_events += r.n_events;
            s.n_pkt_events += r.n_pkt_events;
            s.n_host_rounds += e->round_active;
            s.final_time = we;
            if (r.error) { s.error = r.error; rc = rc ? rc : SHD_EOVERFLOW; break; }
            e->last_logged = e->pending_resolved - pend_before;
            if (e->last_logged) e->logged_any = true;
            e->tl_ready = e->last_logged == 0;
            next = r.next_time;
        }
    }
    e->h_sum->next_time = next;
    // every event before `stop` has run: the engine's clock stands at stop
    if (rc == SHD_OK) e->t_done = std::max<uint64_t>(e->t_done, std::min<uint64_t>(stop, next));
    if (rc == SHD_OK && e->snap_valid && !e->in_replay && stop > e->snap_next &&
        (e->snap_stops.empty() || e->snap_stops.back() != stop))
        e->snap_stops.push_back(stop);
    s.n_pending_resolved = e->pending_resolved - pend0;
    s.device_ms_round_kernel = e->kernel_ms_total;
    s.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (st) *st = s;
    return rc;
}

#ifdef SHD_TIMING
extern "C" int shd_debug_timing(uint64_t* out) {   // 64 x 2048 x 24
    SHD_HIP(hipDeviceSynchronize());
    SHD_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tim), sizeof(g_tim)));
    return SHD_OK;
}
extern "C" int shd_debug_counts(uint64_t* out, int reset) {   // 8
    SHD_HIP(hipDeviceSynchronize());
    SHD_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cnt), sizeof(g_cnt)));
    if (reset) {
        static const unsigned long long z[8] = {};
        SHD_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_cnt), z, sizeof(g_cnt)));
    }
    return SHD_OK;
}
extern "C" int shd_debug_kind_costs(uint64_t* out, int reset) {   // 10 x 4
    SHD_HIP(hipDeviceSynchronize());
    SHD_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kc), sizeof(g_kc)));
    if (reset) {
        static const unsigned long long z[10][4] = {};
        SHD_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_kc), z, sizeof(g_kc)));
    }
    return SHD_OK;
}
#endif
#ifdef SHD_PROF
// profiling build only: read (and clear) the per-phase clock totals
extern "C" int shd_debug_waves(uint64_t* out) {   // 128 x 8, then reset
    SHD_HIP(hipDeviceSynchronize());
    SHD_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave), sizeof(g_wave)));
    static unsigned long long z[128][8];
    for (int i = 0; i < 128; i++) {
        for (int k = 0; k < 8; k++) z[i][k] = 0;
        z[i][0] = ~0ull;
    }
    SHD_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_wave), z, sizeof(z)));
    return SHD_OK;
}

extern "C" int shd_debug_prof(uint64_t* out, int n) {
    if (n < 2 * PR_N + 2) return SHD_EINVAL;
    SHD_HIP(hipDeviceSynchronize());
    SHD_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * (2 * PR_N + 2)));
    unsigned long long z[2 * PR_N + 2] = {};
    SHD_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)));
    return SHD_OK;
}
#endif

extern "C" int shd_eng_run(shd_eng* e, shd_run_stats* st) {
    if (!e) return SHD_EINVAL;
    return shd_eng_run_until(e, e->P.end_time, st);
}

extern "C" int shd_eng_remote_copy(shd_eng* e, void* dev_dst, uint64_t cap, uint64_t* n) {
    if (!e || !n) return SHD_EINVAL;
    const uint64_t cnt = std::min<uint64_t>(e->h_sum->n_remote, e->P.remote_cap);
    if (cnt > cap) { *n = cnt; return SHD_ERANGE; }
    SHD_HIP(hipSetDevice(e->device));
    if (cnt) {
        if (!dev_dst) return SHD_EINVAL;
        SHD_HIP(hipMemcpyAsync(dev_dst, e->P.remote, sizeof(shd_event) * cnt, hipMemcpyDeviceToDevice, e->stream));
        SHD_HIP(hipStreamSynchronize(e->stream));
    }
    *n = cnt;
    return SHD_OK;
}

extern "C" int shd_eng_ingest(shd_eng* e, const void* ev, uint64_t n) {
    if (!e || (n && !ev)) return SHD_EINVAL;
    if (!n) return SHD_OK;
    e->snap_valid = false;
    SHD_HIP(hipSetDevice(e->device));
    hipLaunchKernelGGL(k_ingest, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream, dp(e->P),
                       (const shd_event*)ev, n, e->parity);
    SHD_HIP(hipGetLastError());
    SHD_HIP(hipStreamSynchronize(e->stream));
    return SHD_OK;
}

extern "C" int shd_eng_next_time(shd_eng* e, uint64_t* t) {
    if (!e || !t) return SHD_EINVAL;
    *t = e->h_sum->next_time;
    return SHD_OK;
}

static uint64_t trace_total(shd_eng* e) {
    unsigned long long t = 0;
    if (hipMemcpy(&t, e->d_trace_n, 8, hipMemcpyDeviceToHost) != hipSuccess) return 0;
    return t;
}

extern "C" int shd_eng_trace_count(shd_eng* e, uint64_t* n) {
    if (!e || !n) return SHD_EINVAL;
    SHD_HIP(hipSetDevice(e->device));
    *n = std::min<uint64_t>(trace_total(e), e->trace_cap);
    return SHD_OK;
}

extern "C" int shd_eng_trace_copy(shd_eng* e, shd_trace_rec* out, uint64_t cap, uint64_t* n) {
    if (!e || !out || !n) return SHD_EINVAL;
    SHD_HIP(hipSetDevice(e->device));
    const uint64_t cnt = std::min<uint64_t>(std::min<uint64_t>(trace_total(e), e->trace_cap), cap);
    if (cnt) SHD_HIP(hipMemcpy(out, e->P.trace_buf, sizeof(shd_trace_rec) * cnt, hipMemcpyDeviceToHost));
    *n = cnt;
    return SHD_OK;
}

extern "C" int shd_eng_digest(shd_eng* e, shd_host_digest* out) {
    if (!e || !out) return SHD_EINVAL;
    SHD_HIP(hipSetDevice(e->device));
    shd_host_digest* d = nullptr;
    SHD_HIP(hipMalloc((void**)&d, sizeof(shd_host_digest) * (size_t)e->nloc));
    hipLaunchKernelGGL(k_digest, dim3((e->nloc + 255) / 256), dim3(256), 0, e->stream, dp(e->P), d);
    hipError_t err = hipMemcpyAsync(out, d, sizeof(shd_host_digest) * (size_t)e->nloc, hipMemcpyDeviceToHost, e->stream);
    hipError_t err2 = hipStreamSynchronize(e->stream);
    (void)hipFree(d);
    if (err != hipSuccess || err2 != hipSuccess) return SHD_ENODEV;
    return SHD_OK;
}

extern "C" int shd_eng_path_counts(shd_eng* e, uint64_t* out, uint64_t cap, uint64_t* n) {
    if (!e || !n || (cap && !out)) return SHD_EINVAL;
    if (!e->P.pcount) return SHD_EINVAL;   // SHD_QF_COUNT_PATHS was not set
    const uint64_t cnt = (uint64_t)e->pc->T * e->pc->T;
    *n = cnt;
    if (cap < cnt) return SHD_ERANGE;
    SHD_HIP(hipSetDevice(e->device));
    std::vector<uint32_t> h(cnt);
    SHD_HIP(hipMemcpyAsync(h.data(), (const uint32_t*)e->P.pcount, 4 * cnt, hipMemcpyDeviceToHost, e->stream));
    SHD_HIP(hipStreamSynchronize(e->stream));
    for (uint64_t i = 0; i < cnt; i++) out[i] = h[i];
    return SHD_OK;
}

extern "C" int shd_eng_heartbeats(shd_eng* e, uint32_t* out, uint64_t cap, uint64_t* n) {
    if (!e || !n || (cap && !out)) return SHD_EINVAL;
    if (!e->heartbeats) return SHD_EINVAL;   // not requested at creation
    const uint64_t cnt = (uint64_t)e->nloc * e->P.hb_k * 2;
    *n = cnt;
    if (cap < cnt) return SHD_ERANGE;
    if (!cnt) return SHD_OK;
    SHD_HIP(hipSetDevice(e->device));
    SHD_HIP(hipMemcpyAsync(out, (const uint2*)e->P.hb, 4 * cnt, hipMemcpyDeviceToHost, e->stream));
    SHD_HIP(hipStreamSynchronize(e->stream));
    return SHD_OK;
}

extern "C" int shd_eng_status_lines(shd_eng* e, const uint32_t* ips, const uint32_t* host_ids, uint32_t listen_port,
                                    shd_lines** out) {
    if (!e || !ips || !out) return SHD_EINVAL;
    uint64_t n = 0, got = 0;
    int rc = shd_eng_trace_count(e, &n);
    if (rc) return rc;
    std::vector<shd_trace_rec> tr(n ? n : 1);
    if (n && (rc = shd_eng_trace_copy(e, tr.data(), n, &got))) return rc;
    return shd_status_lines(tr.data(), got, ips, host_ids, (uint32_t)e->H, e->P.payload, listen_port,
                            e->app_peer.empty() ? nullptr : e->app_peer.data(), out);
}

extern "C" int shd_eng_node_lines(shd_eng* e, uint32_t local_host, shd_lines** out) {
    if (!e || !out || local_host >= (uint32_t)e->nloc || !e->heartbeats) return SHD_EINVAL;
    const uint32_t h = (uint32_t)e->h0 + local_host;
    const uint64_t iv = e->host_hb.empty() ? e->P.heartbeat : e->host_hb[h];
    // this host's heartbeats at k * iv < end_time, k >= 1 (P.hb holds hb_k per host)
    uint64_t k = e->P.end_time > 0 && iv ? (e->P.end_time - 1) / iv : 0;
    if (k > e->P.hb_k) k = e->P.hb_k;
    std::vector<uint32_t> snap(2 * (k ? k : 1));
    if (k) {
        SHD_HIP(hipSetDevice(e->device));
        SHD_HIP(hipMemcpyAsync(snap.data(), (const uint2*)e->P.hb + (size_t)local_host * e->P.hb_k, 8 * k,
                               hipMemcpyDeviceToHost, e->stream));
        SHD_HIP(hipStreamSynchronize(e->stream));
    }
    return shd_node_lines(snap.data(), k, iv, e->P.payload, h, out);
}

extern "C" int shd_eng_stream(shd_eng* e, void** s) {
    if (!e || !s) return SHD_EINVAL;
    *s = (void*)e->stream;
    return SHD_OK;
}

extern "C" int shd_eng_last_kernel_ms(shd_eng* e, double* ms) {
    if (!e || !ms) return SHD_EINVAL;
    *ms = e->last_kernel_ms;
    return SHD_OK;
}

extern "C" void shd_eng_destroy(shd_eng* e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    for (void* p : e->allocs) (void)hipFree(p);
    snap_free(e);   // the protected rounds' / restore point's state copy
    if (e->h_sum) (void)hipHostFree(e->h_sum);
    if (e->h_ring) (void)hipHostFree(e->h_ring);
    if (e->h_ctl) (void)hipHostFree(e->h_ctl);
    if (e->h_seed) (void)hipHostFree(e->h_seed);
    if (e->batch_graph) (void)hipGraphExecDestroy(e->batch_graph);
    if (e->batch_graph_tl) (void)hipGraphExecDestroy(e->batch_graph_tl);
    for (auto& ev : e->bev)
        if (ev) (void)hipEventDestroy(ev);
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

#include "eng_group.h"
