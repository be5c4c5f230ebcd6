// eng_group.h -- host driver of the engine groups (shd_xgroup, include/shdgpu.h):
// rounds across engines with one exchange per round.  Part of libshdgpu's
// engine translation unit (csrc/engine.hip includes it after the single-engine
// driver); not a standalone header.
#pragma once

// ===================================================================== engine groups
// shd_xgroup (include/shdgpu.h): rounds across engines with one fixed-size
// all-to-all per round.  DESIGN.md "Multi-GPU" describes the protocol.
#define SHD_NCCL(x)                                                                                  \
    do {                                                                                             \
        ncclResult_t r_ = (x);                                                                       \
        if (r_ != ncclSuccess) {                                                                     \
            fprintf(stderr, "libshdgpu: %s: %s (%s:%d)\n", #x, ncclGetErrorString(r_), __FILE__, __LINE__); \
            return SHD_ENODEV;                                                                       \
        }                                                                                            \
    } while (0)

struct shd_xgroup {
    shd_comm* comm = nullptr;          // null: the local transport (engines of one process)
    bool own_comm = false;             // created by shd_xgroup_create_rccl
    int world = 1;                     // engines in the group
    int rank0 = 0;                     // group rank of local engine 0
    std::vector<shd_eng*> engs;        // this process's engines, rank order
    uint32_t xcap = 0;                 // events per peer block
    size_t stride = 0;                 // event slots per peer block (header + xcap)
    uint64_t window = 0, end_time = 0;
    struct Loc {
        shd_event* xsend = nullptr;
        shd_event* xrecv[2] = {nullptr, nullptr};
        uint32_t* xcount = nullptr;
        XHeader* halt_hdr = nullptr;
        Params* d_xpr = nullptr;   // device copies of the exchange-mode P, one per summary-ring slot
        TlPart* parts = nullptr;   // [2][grid] ticketless round shares (k_round_xtl -> k_xfold)
        uint32_t* xcnt = nullptr;  // fused peer-to-peer rounds: region slot counters [2][world][xnbx]
    };
    std::vector<Loc> loc;
    uint64_t xseq = 0;                 // exchanges done: the latest headers are in xrecv[(xseq - 1) & 1]
    bool started = false;
    hipStream_t xs = nullptr;          // local transport: the copy stream
    hipEvent_t xev = nullptr;
    std::vector<hipEvent_t> eev;
    uint64_t next = kInf;              // group next event time (host view)
    bool fixed_cap = false;            // block size given by the caller
    uint64_t last_spill_batch = ~0ull; // batch index of the last spill halt
    uint64_t batches = 0;
    int last_nb = shd_eng::kBatch;     // rounds in the last batch (its last summary is d_ring[last_nb])
    // full batches captured as HIP graphs (RCCL transport, one engine per
    // process), one per exchange parity at the batch start
    hipGraphExec_t graph[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};   // [sparse][parity]
    bool graph_failed = false;
    // fused rounds over engines with more 64-host blocks than resident waves
    // (the north star's 125 k-host shard): k_round_spx, blocks of sp_hosts
    // hosts, while few hosts are active per round (sp_dense: the last batch
    // had many, k_round_px instead -- the exchange is the same either way)
    uint32_t sp_hosts = 0, sp_grid = 0;
    bool sp_dense = false, sp_forced = false;
    // protected rounds (as for one engine): group-wide, so every rank decides alike
    bool logged_any = false;
    uint64_t last_logged = 0;          // first touches gathered from the whole group at the last log
    // peer-to-peer transport (shd_xgroup_create_p2p; one engine per process)
    bool p2p = false;
    shd_event* p2p_base = nullptr;     // own receive blocks [2][world][stride], uncached, IPC-exported
    std::vector<shd_event*> p2p_peer;  // every rank's receive blocks as mapped here (own: p2p_base)
    shd_event** d_peers = nullptr;     // the same on the device
    uint32_t* d_xerr = nullptr;        // set by a wait that timed out
    uint64_t xepoch = 0;               // exchange tags issued (never rolled back)
    bool fused = false;                // peer-to-peer rounds fused with their exchange (k_round_px)
    uint32_t xnbx = 0;                 // fused: region blocks per rank
    // one engine per process: the last exchange's headers and the wait-error word,
    // copied back with the batch's summaries (one stream synchronisation per batch)
    XHeader* h_hdr = nullptr;          // pinned, [64]
    uint32_t* h_xerr = nullptr;        // pinned
};

// peer-to-peer rounds complete the previous round's exchange in their own
// launch (k_round_px); SHD_X_UNFUSED=1 keeps the separate k_xchg launch (A/B)
static bool x_fuse_env() {
    static const bool unfused = getenv("SHD_X_UNFUSED") != nullptr;
    return !unfused;
}

// the fused schedule's regions: own base of parity w
static shd_event* x_rgn(const shd_xgroup* g, int w) {
    return g->p2p_base + 2 * (size_t)g->world * g->stride + (size_t)w * g->world * g->xnbx * kXSlots;
}

// header granule replicas (fused schedule): [2][kXReplMax - 1][world] 32-B
// slots after the regions, all kXReplMax copies in use
static uint64_t x_hoff(const shd_xgroup* g) {
    return 2 * (uint64_t)g->world * g->stride + 2 * (uint64_t)g->world * g->xnbx * kXSlots;
}
static const shd_event* x_rep(const shd_xgroup* g, int w) {
    return g->p2p_base + x_hoff(g) + (size_t)w * (kXReplMax - 1) * g->world;
}

static bool x_want_protect(const shd_xgroup* g) {
    if (protect_off()) return false;
    if (g->engs[0]->P.complete && !protect_all()) return false;   // nothing is ever logged (want_protect)
    for (const shd_eng* e : g->engs)
        if (e->snap_failed) return false;
    return protect_all() || !g->logged_any || g->last_logged >= kProtectMin;
}

static Params xparams(const shd_xgroup* g, int k, DevSummary* sum) {
    Params P = g->engs[k]->P;
    P.xsend = g->loc[k].xsend;
    P.xcount = g->loc[k].xcount;
    P.xcap = g->xcap;
    P.xworld = g->world;
    P.xpeer = g->p2p ? (shd_event* const*)g->d_peers : nullptr;   // sends stored straight into the peers' blocks
    P.xme = g->rank0;
    P.sum = sum;
    if (g->fused) {
        P.xcnt = g->loc[k].xcnt;
        P.xnbx = g->xnbx;
        P.xrcap = std::min<uint32_t>(kXSlots, g->xcap);
        P.xroff = 2 * (uint64_t)g->world * g->stride;
    }
    return P;
}

// the fixed-size all-to-all: block d of every sender's xsend -> block s of
// receiver d's xrecv[xseq & 1]
// a peer-to-peer exchange: every engine's blocks put into the peers' receive
// blocks of parity wi under tag (ctl->xtag + tag_add, or tag_add), then the
// wait for every peer's (and, for a round, the ingest of what came)
static void x_p2p_launch(shd_xgroup* g, int wi, uint32_t tag_add, int use_ctl, const Params& P, int ri, int ingest) {
    shd_eng* e = g->engs[0];
    hipLaunchKernelGGL(k_xput, dim3(g->world), dim3(256), 0, e->stream, (const shd_event*)g->loc[0].xsend,
                       (shd_event* const*)g->d_peers, (uint32_t)g->stride, g->xcap, g->world, g->rank0, wi,
                       (const DevCtl*)e->d_ctl, tag_add, use_ctl);
    const uint64_t nthr = ingest ? (uint64_t)g->world * g->xcap : 1;
    hipLaunchKernelGGL(k_xwait_ingest, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, e->stream, dp(P),
                       (const shd_event*)g->loc[0].xrecv[wi], (const DevCtl*)e->d_ctl, tag_add, use_ctl, ri, ingest,
                       g->d_xerr);
}

static int x_p2p_check(shd_xgroup* g) {
    if (!g->p2p) return SHD_OK;
    uint32_t bad = 0;
    SHD_HIP(hipMemcpy(&bad, g->d_xerr, 4, hipMemcpyDeviceToHost));
    if (bad) {
        fprintf(stderr, "libshdgpu: peer-to-peer exchange: a peer's block did not come within %llu s\n",
                kXWaitTicks / 100000000ull);
        return SHD_ENODEV;
    }
    return SHD_OK;
}

static int x_exchange(shd_xgroup* g) {
    const size_t bytes = g->stride * sizeof(shd_event);
    const int wi = (int)(g->xseq & 1);
    if (g->p2p) {
        const uint32_t tag = (uint32_t)(++g->xepoch);
        x_p2p_launch(g, wi, tag, 0, xparams(g, 0, g->engs[0]->d_sum), 0, 0);
        SHD_HIP(hipGetLastError());
    } else if (g->comm) {
        shd_eng* e = g->engs[0];
        const int rc = shd_comm_alltoall_dev(g->comm, g->loc[0].xsend, g->loc[0].xrecv[wi], bytes, e->stream);
        if (rc) return rc;
    } else {
        const int n = g->world;
        for (int k = 0; k < n; k++) {
            SHD_HIP(hipEventRecord(g->eev[k], g->engs[k]->stream));
            SHD_HIP(hipStreamWaitEvent(g->xs, g->eev[k], 0));
        }
        XPtrs X;
        for (int k = 0; k < n; k++) {
            X.send[k] = g->loc[k].xsend;
            X.recv[k] = g->loc[k].xrecv[wi];
        }
        hipLaunchKernelGGL(k_xcopy_local, dim3(8, n, n), dim3(256), 0, g->xs, X, (uint64_t)g->stride);
        SHD_HIP(hipGetLastError());
        SHD_HIP(hipEventRecord(g->xev, g->xs));
        for (int k = 0; k < n; k++) SHD_HIP(hipStreamWaitEvent(g->engs[k]->stream, g->xev, 0));
    }
    g->xseq++;
    return SHD_OK;
}

// headers of the latest exchange as seen by local engine 0
static int x_headers(shd_xgroup* g, std::vector<XHeader>& h) {
    shd_eng* e = g->engs[0];
    h.resize(g->world);
    const shd_event* src = g->loc[0].xrecv[(g->xseq - 1) & 1];
    SHD_HIP(hipMemcpy2DAsync(h.data(), sizeof(XHeader), src, g->stride * sizeof(shd_event), sizeof(XHeader),
                             g->world, hipMemcpyDeviceToHost, e->stream));
    SHD_HIP(hipStreamSynchronize(e->stream));
    return x_p2p_check(g);
}

static void x_next_from(shd_xgroup* g, const XHeader* h, int n);
static int x_read_next(shd_xgroup* g) {
    std::vector<XHeader> h;
    int rc = x_headers(g, h);
    if (rc) return rc;
    x_next_from(g, h.data(), (int)h.size());
    return SHD_OK;
}
static void x_next_from(shd_xgroup* g, const XHeader* h, int n) {
    uint64_t t = kInf;
    uint32_t fl = 0;
    for (int i = 0; i < n; i++) {
        const XHeader& x = h[i];
        t = std::min<uint64_t>(t, x.next_time);
        fl |= x.flags;
    }
    // a flagged last round (first-touch log, spill, error) is recovered at the
    // next batch's first round; its headers' times leave out what the
    // recovery delivers, so the loop must run on whatever they say
    g->next = fl ? 0 : t;
}

// every engine's first-touch records of the flagged round, in any order
static int x_gather_pending(shd_xgroup* g, std::vector<shd_pending>& all) {
    std::vector<shd_pending> mine;
    for (shd_eng* e : g->engs) {
        const uint64_t n = e->round_pending;
        if (n > e->P.pend_cap) return SHD_EOVERFLOW;
        const size_t at = mine.size();
        mine.resize(at + n);
        if (n) SHD_HIP(hipMemcpy(mine.data() + at, e->P.pend, sizeof(shd_pending) * n, hipMemcpyDeviceToHost));
    }
    if (!g->comm) {
        all.swap(mine);
        return SHD_OK;
    }
    // every rank's count, then every rank's records (padded to the largest)
    const int W = g->world;
    const unsigned long long my = mine.size();
    std::vector<unsigned long long> cnt(W);
    int rc = shd_comm_allgather_host(g->comm, &my, 8, cnt.data());
    if (rc) return rc;
    const unsigned long long mx = *std::max_element(cnt.begin(), cnt.end());
    all.clear();
    if (mx == 0) return SHD_OK;
    std::vector<shd_pending> pad(mx), got((size_t)mx * W);
    std::copy(mine.begin(), mine.end(), pad.begin());
    if ((rc = shd_comm_allgather_host(g->comm, pad.data(), sizeof(shd_pending) * mx, got.data()))) return rc;
    for (int r = 0; r < W; r++) all.insert(all.end(), got.begin() + (size_t)r * mx, got.begin() + (size_t)r * mx + cnt[r]);
    return SHD_OK;
}

static int x_ingest(shd_eng* e, const Params& P, const shd_event* d_ev, uint64_t n, int parity) {
    if (!n) return SHD_OK;
    hipLaunchKernelGGL(k_ingest, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream, dp(P), d_ev, n, parity);
    SHD_HIP(hipGetLastError());
    return SHD_OK;
}

// deliver the remote buffers (block spills and finalized first-touch sends of
// the flagged round, whose summary is ring slot `slot`) with a variable-size
// exchange; the receivers' next round merges them (inbox[round & 1])
static int x_exchange_remote(shd_xgroup* g, int slot) {
    const int nl = (int)g->engs.size();
    std::vector<std::vector<std::vector<shd_event>>> out(nl);   // [local sender][peer]
    for (int k = 0; k < nl; k++) {
        shd_eng* e = g->engs[k];
        DevSummary r;
        SHD_HIP(hipMemcpy(&r, &e->d_ring[slot], sizeof(r), hipMemcpyDeviceToHost));
        const uint64_t n = std::min<uint64_t>(r.n_remote, e->P.remote_cap);
        std::vector<shd_event> ev(n);
        if (n) SHD_HIP(hipMemcpy(ev.data(), e->P.remote, sizeof(shd_event) * n, hipMemcpyDeviceToHost));
        out[k].assign(g->world, {});
        const uint64_t H = (uint64_t)e->P.H, N = (uint64_t)g->world;
        for (const shd_event& x : ev) {
            int64_t p = (int64_t)(((uint64_t)x.dst * N) / H);
            while (p + 1 < (int64_t)N && (H * (uint64_t)(p + 1)) / N <= x.dst) p++;
            while (p > 0 && (H * (uint64_t)p) / N > x.dst) p--;
            out[k][p].push_back(x);
        }
        const unsigned long long z = 0;   // the spill is consumed
        SHD_HIP(hipMemcpy(&e->d_ring[slot].n_remote, &z, 8, hipMemcpyHostToDevice));
    }
    if (!g->comm) {
        for (int d = 0; d < nl; d++) {
            std::vector<shd_event> in;
            for (int s = 0; s < nl; s++) in.insert(in.end(), out[s][d].begin(), out[s][d].end());
            if (in.empty()) continue;
            shd_eng* e = g->engs[d];
            shd_event* d_ev = nullptr;
            SHD_HIP(hipMalloc((void**)&d_ev, sizeof(shd_event) * in.size()));
            int rc = SHD_OK;
            if (hipMemcpy(d_ev, in.data(), sizeof(shd_event) * in.size(), hipMemcpyHostToDevice) != hipSuccess)
                rc = SHD_ENODEV;
            if (!rc) rc = x_ingest(e, xparams(g, d, &e->d_ring[slot]), d_ev, in.size(), (int)(e->round & 1));
            if (!rc && hipStreamSynchronize(e->stream) != hipSuccess) rc = SHD_ENODEV;
            (void)hipFree(d_ev);
            if (rc) return rc;
        }
        return SHD_OK;
    }
    // a communicator (one engine per process): every rank's per-peer counts,
    // then every rank's bucketed events (an all-to-all-v through an
    // all-gather: spills are rare and small)
    shd_eng* e = g->engs[0];
    const int W = g->world, me = g->rank0;
    std::vector<unsigned long long> sc(W), allc((size_t)W * W);
    for (int p = 0; p < W; p++) sc[p] = out[0][p].size();
    int rc = shd_comm_allgather_host(g->comm, sc.data(), 8 * (size_t)W, allc.data());
    if (rc) return rc;
    unsigned long long mx = 0;
    for (int r = 0; r < W; r++) {
        unsigned long long t = 0;
        for (int p = 0; p < W; p++) t += allc[(size_t)r * W + p];
        mx = std::max(mx, t);
    }
    if (mx == 0) return SHD_OK;
    std::vector<shd_event> flat(mx), got((size_t)mx * W);
    size_t k = 0;
    for (int p = 0; p < W; p++)
        for (const shd_event& x : out[0][p]) flat[k++] = x;
    if ((rc = shd_comm_allgather_host(g->comm, flat.data(), sizeof(shd_event) * mx, got.data()))) return rc;
    std::vector<shd_event> in;
    for (int r = 0; r < W; r++) {
        size_t off = (size_t)r * mx;
        for (int p = 0; p < me; p++) off += allc[(size_t)r * W + p];
        in.insert(in.end(), got.begin() + off, got.begin() + off + allc[(size_t)r * W + me]);
    }
    if (in.empty()) return SHD_OK;
    shd_event* d_ev = nullptr;
    SHD_HIP(hipMalloc((void**)&d_ev, sizeof(shd_event) * in.size()));
    if (hipMemcpy(d_ev, in.data(), sizeof(shd_event) * in.size(), hipMemcpyHostToDevice) != hipSuccess) rc = SHD_ENODEV;
    if (!rc) rc = x_ingest(e, xparams(g, 0, &e->d_ring[slot]), d_ev, in.size(), (int)(e->round & 1));
    if (!rc && hipStreamSynchronize(e->stream) != hipSuccess) rc = SHD_ENODEV;
    (void)hipFree(d_ev);
    return rc;
}

static void x_p2p_unmap(shd_xgroup* g) {
    for (size_t p = 0; p < g->p2p_peer.size(); p++)
        if (g->p2p_peer[p] && g->p2p_peer[p] != g->p2p_base) (void)hipIpcCloseMemHandle(g->p2p_peer[p]);
    g->p2p_peer.clear();
    if (g->p2p_base) (void)hipFree(g->p2p_base);
    g->p2p_base = nullptr;
}

// x_p2p_map's self-check (k_p2p_probe_put / _check); every step collective
static int x_p2p_probe(shd_xgroup* g) {
    shd_eng* e = g->engs[0];
    const int W = g->world, me = g->rank0;
    if (W > 64) return SHD_EINVAL;
    // a generation all ranks agree on (rank 0's clock), so that a granule left
    // by an earlier mapping at the same address never passes
    uint32_t gen = (uint32_t)std::chrono::steady_clock::now().time_since_epoch().count() | 1u;
    std::vector<uint32_t> gens(W);
    int rc = shd_comm_allgather_host(g->comm, &gen, 4, gens.data());
    if (rc) return rc;
    gen = gens[0];
    int corrupt = 0;
#ifdef SHD_TEST_HOOKS   // test build: exchanged events this rank loses on taking them
    if (const char* f = getenv("SHD_TEST_XDROP")) {
        const int n = atoi(f);
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_test_xdrop), &n, sizeof(n));
    }
#endif
#ifdef SHD_TEST_HOOKS   // test build: this rank puts a wrong granule (every rank must then fail alike)
    if (const char* f = getenv("SHD_P2P_PROBE_CORRUPT"))
        if (atoi(f) == me) corrupt = 1;
#endif
    uint32_t ok = 1;
    unsigned long long* d_bad = nullptr;
    unsigned long long bad = ~0ull;
    if (hipMalloc((void**)&d_bad, sizeof(*d_bad)) != hipSuccess) ok = 0;
    if (ok) {
        hipLaunchKernelGGL(k_p2p_probe_put, dim3(1), dim3(64), 0, e->stream, g->d_peers, W, me, g->stride, gen, corrupt);
        if (hipStreamSynchronize(e->stream) != hipSuccess) ok = 0;
    }
    std::vector<uint32_t> oks(W);
    if ((rc = shd_comm_allgather_host(g->comm, &ok, 4, oks.data()))) { (void)hipFree(d_bad); return rc; }
    for (uint32_t x : oks) ok &= x;
    if (ok) {   // every rank's puts have drained
        hipLaunchKernelGGL(k_p2p_probe_check, dim3(1), dim3(64), 0, e->stream, g->p2p_base, W, me, g->stride, gen,
                           d_bad);
        if (hipMemcpyAsync(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
            hipStreamSynchronize(e->stream) != hipSuccess)
            ok = 0;
        if (bad) {
            fprintf(stderr, "shd_xgroup: peer-to-peer self-check failed on rank %d: granules from senders %#llx "
                            "missing or wrong\n", me, bad);
            ok = 0;
        }
        // the probe's slots back to "no exchange yet" before any rank's first put
        for (int p = 0; p < W && ok; p++)
            if (hipMemsetAsync(g->p2p_base + (size_t)p * g->stride, 0, sizeof(shd_event), e->stream) != hipSuccess)
                ok = 0;
        if (hipStreamSynchronize(e->stream) != hipSuccess) ok = 0;
    }
    (void)hipGetLastError();
    (void)hipFree(d_bad);
    if ((rc = shd_comm_allgather_host(g->comm, &ok, 4, oks.data()))) return rc;
    for (uint32_t x : oks) ok &= x;
    return ok ? SHD_OK : SHD_ENODEV;
}

// the peer-to-peer receive blocks: allocated uncached (a peer's stores land
// in memory, no L2 of this GPU holds a stale copy), exported by IPC handle,
// every rank's handle all-gathered and mapped.  The handle exchange is also
// the barrier that makes the old blocks (a regrowth) free to release: every
// rank is between batches, all puts into them done
static int x_p2p_map(shd_xgroup* g) {
    shd_eng* e = g->engs[0];
    const int W = g->world;
    x_p2p_unmap(g);
    // every step is collective: a rank that fails still takes part in both
    // all-gathers, so that every rank learns it and all fail alike
    struct Share {
        hipIpcMemHandle_t h;
        uint32_t ok;
        uint32_t pad[15];
    };
    Share mine{};
    const size_t bytes = (2 * (size_t)W * g->stride +
                          (g->fused ? 2 * (size_t)W * g->xnbx * kXSlots + 2 * (size_t)(kXReplMax - 1) * W : 0)) *
                         sizeof(shd_event);
    if (hipExtMallocWithFlags((void**)&g->p2p_base, bytes, hipDeviceMallocUncached) == hipSuccess &&
        hipMemset(g->p2p_base, 0, bytes) == hipSuccess &&   // tag 0: no exchange yet (tags start at 1)
        hipDeviceSynchronize() == hipSuccess && hipIpcGetMemHandle(&mine.h, g->p2p_base) == hipSuccess)
        mine.ok = 1;
    (void)hipGetLastError();
    std::vector<Share> all(W);
    int rc = shd_comm_allgather_host(g->comm, &mine, sizeof(Share), all.data());
    if (rc) return rc;
    uint32_t ok = 1;
    for (const Share& x : all) ok &= x.ok;
    g->p2p_peer.assign(W, nullptr);
#ifdef SHD_TEST_HOOKS   // test build: this rank fails to map its peers (every rank must then fail alike)
    if (const char* f = getenv("SHD_P2P_FAIL_RANK"))
        if (atoi(f) == g->rank0) ok = 0;
#endif
    for (int p = 0; p < W && ok; p++) {
        if (p == g->rank0) {
            g->p2p_peer[p] = g->p2p_base;
            continue;
        }
        void* q = nullptr;
        if (hipIpcOpenMemHandle(&q, all[p].h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
            (void)hipGetLastError();
            ok = 0;
            break;
        }
        g->p2p_peer[p] = (shd_event*)q;
    }
    if (ok && !g->d_peers && ealloc(e, &g->d_peers, (size_t)64)) ok = 0;
    if (ok && !g->d_xerr && ealloc(e, &g->d_xerr, 1)) ok = 0;
    if (ok && hipMemcpy(g->d_peers, g->p2p_peer.data(), sizeof(shd_event*) * W, hipMemcpyHostToDevice) != hipSuccess)
        ok = 0;
    // the second all-gather: every rank mapped every block (and a barrier: no
    // rank puts into the new blocks before every rank has them)
    std::vector<uint32_t> oks(W);
    if ((rc = shd_comm_allgather_host(g->comm, &ok, 4, oks.data()))) return rc;
    for (uint32_t x : oks) ok &= x;
    if (!ok) {
        x_p2p_unmap(g);
        return SHD_ENODEV;
    }
    // the self-check: one known granule from every rank into every peer's
    // block over the mapping, read back by the receiver; a transport that
    // loses or garbles it fails the group's creation on every rank alike
    // (SHD_ENODEV, the caller falls back to the all-to-all) instead of
    // silently wrong rounds
    if ((rc = x_p2p_probe(g))) {
        x_p2p_unmap(g);
        return rc;
    }
    g->loc[0].xrecv[0] = g->p2p_base;
    g->loc[0].xrecv[1] = g->p2p_base + (size_t)W * g->stride;
    return SHD_OK;
}

static int x_alloc(shd_xgroup* g) {
    g->stride = (size_t)g->xcap + 1;
    g->loc.resize(g->engs.size());
    if (g->fused) {
        const shd_eng* e = g->engs[0];
        const int64_t per = (e->P.H + g->world - 1) / g->world;
        g->xnbx = (uint32_t)((per + e->P.hpw - 1) / e->P.hpw);
    }
    for (size_t k = 0; k < g->engs.size(); k++) {
        shd_eng* e = g->engs[k];
        shd_xgroup::Loc& L = g->loc[k];
        SHD_HIP(hipSetDevice(e->device));
        const size_t n = g->stride * (size_t)g->world;
        int rc;
        if (g->p2p) {
            if ((rc = ealloc(e, &L.xsend, n)) || (rc = x_p2p_map(g))) return rc;
        } else if ((rc = ealloc(e, &L.xsend, n)) || (rc = ealloc(e, &L.xrecv[0], n)) ||
                   (rc = ealloc(e, &L.xrecv[1], n))) {
            return rc;
        }
        if ((rc = ealloc(e, &L.xcount, g->world)) || (rc = ealloc(e, &L.halt_hdr, g->world)) ||
            (rc = ealloc(e, &L.d_xpr, shd_eng::kRing, false)) ||
            (rc = ealloc(e, &L.parts, 2 * (size_t)((e->nloc + e->P.hpw - 1) / e->P.hpw))))
            return rc;
        if (g->fused && (rc = ealloc(e, &L.xcnt, 2 * (size_t)g->world * g->xnbx))) return rc;
        std::vector<Params> pr(shd_eng::kRing);
        for (int i = 0; i < shd_eng::kRing; i++) pr[i] = xparams(g, (int)k, &e->d_ring[i]);
        SHD_HIP(hipMemcpyAsync(L.d_xpr, pr.data(), sizeof(Params) * pr.size(), hipMemcpyHostToDevice, e->stream));
        SHD_HIP(hipStreamSynchronize(e->stream));
    }
    return SHD_OK;
}

static uint32_t x_default_cap(const shd_eng* e, int world) {
    // a round's sends to one peer are ~ nloc / world x (sends per host per
    // window, well below 1 at W = the minimum path latency): two sends per
    // host of headroom; bursts beyond the block spill to the host path, and
    // spills in consecutive batches grow the block (x_grow)
    return (uint32_t)std::max<int64_t>(256, 2 * (int64_t)e->nloc / world);
}

extern "C" int shd_xgroup_unique_id(uint8_t id[SHD_XID_BYTES]) {
    if (!id) return SHD_EINVAL;
    ncclUniqueId u;
    SHD_NCCL(ncclGetUniqueId(&u));
    memcpy(id, &u, SHD_XID_BYTES);
    return SHD_OK;
}

static void x_drop_graphs(shd_xgroup* g) {
    for (auto& gk : g->graph)
        for (auto& ge : gk)
            if (ge) {
                (void)hipGraphExecDestroy(ge);
                ge = nullptr;
            }
}

static void x_free(shd_xgroup* g) {
    if (!g) return;
    if (g->h_hdr) (void)hipHostFree(g->h_hdr);
    if (g->h_xerr) (void)hipHostFree(g->h_xerr);
    x_drop_graphs(g);
    x_p2p_unmap(g);
    if (g->comm && g->own_comm) shd_comm_destroy(g->comm);
    for (auto& ev : g->eev)
        if (ev) (void)hipEventDestroy(ev);
    if (g->xev) (void)hipEventDestroy(g->xev);
    if (g->xs) (void)hipStreamDestroy(g->xs);
    delete g;   // buffers belong to the engines' allocation lists
}

extern "C" int shd_xgroup_create_local(shd_eng* const* engines, int n, uint32_t block_events, shd_xgroup** out) {
    if (!engines || n <= 0 || n > 64 || !out) return SHD_EINVAL;
    shd_xgroup* g = new shd_xgroup();
    g->world = n;
    g->rank0 = 0;
    for (int k = 0; k < n; k++) {
        shd_eng* e = engines[k];
        if (!e || e->device != engines[0]->device || e->P.H != engines[0]->P.H) { x_free(g); return SHD_EINVAL; }
        const int64_t H = e->P.H;
        if (e->h0 != (int32_t)((H * k) / n) || e->h0 + e->nloc != (int32_t)((H * (k + 1)) / n)) {
            x_free(g);
            return SHD_EINVAL;   // the group partition is (H*p)/N
        }
        g->engs.push_back(e);
    }
    g->window = kInf;
    for (shd_eng* e : g->engs) g->window = std::min<uint64_t>(g->window, e->window);
    g->end_time = engines[0]->P.end_time;
    g->xcap = block_events ? block_events : x_default_cap(engines[0], n);
    g->fixed_cap = block_events != 0;
    if (hipSetDevice(engines[0]->device) != hipSuccess ||
        hipStreamCreateWithFlags(&g->xs, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&g->xev, hipEventDisableTiming) != hipSuccess) {
        x_free(g);
        return SHD_ENODEV;
    }
    g->eev.assign(n, nullptr);
    for (auto& ev : g->eev)
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) { x_free(g); return SHD_ENODEV; }
    int rc = x_alloc(g);
    if (rc) { x_free(g); return rc; }
    *out = g;
    return SHD_OK;
}

static int x_create(shd_eng* e, shd_comm* comm, uint32_t block_events, bool p2p, shd_xgroup** out) {
    if (!e || !comm || !out) return SHD_EINVAL;
    const int world = comm->world, rank = comm->rank;
    if (world > 64) return SHD_EINVAL;   // the round kernel folds the peers' headers in one wave
    const int64_t H = e->P.H;
    if (e->h0 != (int32_t)((H * rank) / world) || e->h0 + e->nloc != (int32_t)((H * (rank + 1)) / world))
        return SHD_EINVAL;
    SHD_HIP(hipSetDevice(e->device));
    shd_xgroup* g = new shd_xgroup();
    g->comm = comm;
    g->world = world;
    g->rank0 = rank;
    g->p2p = p2p;
    g->engs.push_back(e);
    // the group agrees on W (min) and checks the model: H and end time equal everywhere
    // (and the hosts per wave: the fused schedule's regions are per block of hpw hosts;
    // the device and round-kernel grid: see below)
    hipDeviceProp_t prop{};
    int ncu = 256;
    unsigned long long dev_id = (unsigned long long)e->device;
    if (hipGetDeviceProperties(&prop, e->device) == hipSuccess) {
        ncu = prop.multiProcessorCount;
        dev_id = ((unsigned long long)prop.pciDomainID << 32) | ((unsigned long long)prop.pciBusID << 8) |
                 (unsigned long long)prop.pciDeviceID;
    }
    const unsigned long long nblk = (unsigned long long)((e->nloc + e->P.hpw - 1) / e->P.hpw);
    const unsigned long long mine[6] = {(unsigned long long)e->window, (unsigned long long)H,
                                        (unsigned long long)e->P.end_time, (unsigned long long)e->P.hpw,
                                        dev_id, nblk};
    std::vector<unsigned long long> all(6 * (size_t)world);
    int rc = shd_comm_allgather_host(comm, mine, sizeof(mine), all.data());
    if (rc) { x_free(g); return rc; }
    g->window = kInf;
    unsigned long long shared_blocks = 0;
    int sharers = 0;
    for (int r = 0; r < world; r++) {
        if (all[6 * r + 1] != (unsigned long long)H || all[6 * r + 2] != e->P.end_time ||
            all[6 * r + 3] != (unsigned long long)e->P.hpw) {
            x_free(g);
            return SHD_EINVAL;
        }
        g->window = std::min<uint64_t>(g->window, all[6 * r]);
        if (all[6 * r + 4] == dev_id) {
            sharers++;
            shared_blocks += all[6 * r + 5];
        }
    }
    // Every block of a fused round waits for the peers' headers, so the peers'
    // launches must run beside it.  With one rank per GPU they do; ranks that
    // share a GPU (tests, rehearsals) are fused only while all their blocks fit
    // the GPU's compute units one each (three ranks of 157 blocks on one GPU
    // waited out their 30 s: the device did not run the three launches at once)
    g->fused = p2p && x_fuse_env() && (sharers <= 1 || shared_blocks <= (unsigned long long)ncu);
    g->end_time = e->P.end_time;
    if (g->fused && !getenv("SHD_X_NO_SP")) {
        // the sparse fused round (k_round_spx): blocks of sph hosts, about two
        // per CU, when the engine has more 64-host blocks than two per CU
        // (SHD_SP_HOSTS=<n>: n hosts per block whatever the size, as for one engine)
        const char* sp_env = getenv("SHD_SP_HOSTS");
        const uint32_t sp_force = sp_env ? (uint32_t)strtoul(sp_env, nullptr, 10) : 0u;
        // (about two blocks per CU with one rank per GPU, as for one engine; one per CU when
        // ranks share the GPU)
        const uint64_t bpc = sharers <= 1 ? 2 : 1;
        const uint64_t per = ((uint64_t)e->nloc + bpc * ncu - 1) / (bpc * ncu);
        const uint32_t sph = sp_force ? (sp_force + 63) / 64 * 64
                                      : (uint32_t)std::max<uint64_t>(256, (per + 63) / 64 * 64);
        const uint32_t grid = (uint32_t)(((uint64_t)e->nloc + sph - 1) / sph);
        // (ranks sharing a GPU: every block of every sharer resident at once,
        // one per CU, as for the fused schedule itself)
        if ((sp_force || nblk > 2ull * (unsigned long long)ncu) && sph <= kSpMaxHosts && e->P.hpw == 64 &&
            (sharers <= 1 || (uint64_t)sharers * std::max<uint32_t>(grid, (uint32_t)world) <= (uint64_t)ncu)) {
            g->sp_hosts = sph;
            g->sp_grid = grid;
            g->sp_forced = sp_force != 0;
        }
    }
    g->xcap = block_events ? block_events : x_default_cap(e, world);
    g->fixed_cap = block_events != 0;
    if ((rc = x_alloc(g))) { x_free(g); return rc; }
    if (hipHostMalloc((void**)&g->h_hdr, sizeof(XHeader) * 64, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&g->h_xerr, sizeof(uint32_t), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        x_free(g);
        return SHD_ENOMEM;
    }
    *g->h_xerr = 0;
    *out = g;
    return SHD_OK;
}

extern "C" int shd_xgroup_create(shd_eng* e, shd_comm* comm, uint32_t block_events, shd_xgroup** out) {
    return x_create(e, comm, block_events, false, out);
}

extern "C" int shd_xgroup_create_p2p(shd_eng* e, shd_comm* comm, uint32_t block_events, shd_xgroup** out) {
    if (comm && comm->world > 64) return SHD_EINVAL;   // d_peers holds 64 pointers
    return x_create(e, comm, block_events, true, out);
}

extern "C" int shd_xgroup_create_rccl(shd_eng* e, const uint8_t id[SHD_XID_BYTES], int world, int rank,
                                      uint32_t block_events, shd_xgroup** out) {
    if (!e || !id || world <= 0 || world > 64 || rank < 0 || rank >= world || !out) return SHD_EINVAL;
    const int64_t H = e->P.H;
    if (e->h0 != (int32_t)((H * rank) / world) || e->h0 + e->nloc != (int32_t)((H * (rank + 1)) / world))
        return SHD_EINVAL;
    shd_comm* c = nullptr;
    int rc = shd_comm_create_rccl(id, world, rank, e->device, &c);
    if (rc) return rc;
    if ((rc = shd_xgroup_create(e, c, block_events, out))) { shd_comm_destroy(c); return rc; }
    (*out)->own_comm = true;
    return SHD_OK;
}

extern "C" int shd_xgroup_next_time(shd_xgroup* g, uint64_t* t) {
    if (!g || !t) return SHD_EINVAL;
    *t = g->next;
    return SHD_OK;
}

extern "C" void shd_xgroup_destroy(shd_xgroup* g) { x_free(g); }

// nb rounds of the engine group: per round, every engine's k_round_x, the
// all-to-all, every engine's k_ingest_x
static bool x_sparse(const shd_xgroup* g) { return g->sp_grid && !g->sp_dense; }

static int x_enqueue_fused(shd_xgroup* g, int nb) {
    shd_eng* e = g->engs[0];
    shd_xgroup::Loc& L = g->loc[0];
    const uint32_t nblk = (uint32_t)((e->nloc + e->P.hpw - 1) / e->P.hpw);
    const bool sp = x_sparse(g);
    const bool lean = lean_model(e->P);   // (the lean instantiations)
    for (int i = 0; i < nb; i++) {
        const int wp = (int)((g->xseq - 1) & 1);   // exchange i - 1 (for round 0: the one before the batch)
        if (sp) {
            const uint32_t grid = std::max<uint32_t>(g->sp_grid, (uint32_t)g->world);
            hipLaunchKernelGGL(lean ? k_round_spx<true> : k_round_spx<false>, dim3(grid), dim3(kBlock), 0, e->stream,
                               g->window, i, &e->d_ring[i],
                               (const DevCtl*)e->d_ctl, L.parts, (const DParams*)(L.d_xpr + i + 1), &e->d_ring[i + 2],
                               (const shd_event*)L.xrecv[wp], x_rgn(g, wp), (shd_event* const*)g->d_peers,
                               L.halt_hdr, g->d_xerr, g->world, g->rank0, wp, x_rep(g, wp), x_hoff(g), kXReplMax,
                               g->sp_hosts, g->sp_grid, i == 0 ? 1 : 0);
        } else if (i == 0) {
            hipLaunchKernelGGL(k_round_xtl, dim3(nblk), dim3(kBlock), 0, e->stream, round_args(e->P),
                               (const DParams*)(L.d_xpr + 1), (const shd_event*)L.xrecv[wp], L.halt_hdr,
                               &e->d_ring[2], (const DevCtl*)e->d_ctl, 0, g->window, L.parts);
        } else {
            // every peer's header needs its put block, also when the engine has fewer blocks of hosts
            const uint32_t grid = std::max<uint32_t>(nblk, (uint32_t)g->world);
            hipLaunchKernelGGL(lean ? k_round_px<true> : k_round_px<false>, dim3(grid), dim3(kBlock), 0, e->stream,
                               g->window, i, &e->d_ring[i],
                               (const DevCtl*)e->d_ctl, L.parts, (const DParams*)(L.d_xpr + i + 1), &e->d_ring[i + 2],
                               round_args(e->P), (const shd_event*)L.xrecv[wp], x_rgn(g, wp),
                               (shd_event* const*)g->d_peers, L.halt_hdr, g->d_xerr, g->world, g->rank0, wp,
                               x_rep(g, wp), x_hoff(g), kXReplMax);
        }
        g->xseq++;   // exchange i: completed by round i + 1's launch, or k_xchg_px below
    }
    const int wl = (int)((g->xseq - 1) & 1);
    const Params P = xparams(g, 0, &e->d_ring[nb]);
    hipLaunchKernelGGL(k_xchg_px, dim3((unsigned)g->world + nblk), dim3(kBlock), 0, e->stream, dp(P),
                       (const TlPart*)L.parts, sp ? g->sp_grid : nblk, nblk, nb - 1, (const DevCtl*)e->d_ctl,
                       (shd_event* const*)g->d_peers,
                       g->world, g->rank0, wl, (const shd_event*)L.xrecv[wl], x_rgn(g, wl), g->d_xerr, x_rep(g, wl),
                       x_hoff(g), kXReplMax);
    return SHD_OK;
}

static int x_enqueue_rounds(shd_xgroup* g, int nb) {
    if (g->fused) return x_enqueue_fused(g, nb);
    const int nl = (int)g->engs.size();
    int rc = SHD_OK;
    for (int i = 0; i < nb; i++) {
        const int ri = (int)((g->xseq - 1) & 1);
        for (int k = 0; k < nl; k++) {
            shd_eng* e = g->engs[k];
            const int grid = (e->nloc + e->P.hpw - 1) / e->P.hpw;
            hipLaunchKernelGGL(k_round_xtl, dim3(grid), dim3(kBlock), 0, e->stream, round_args(e->P),
                               (const DParams*)(g->loc[k].d_xpr + i + 1), (const shd_event*)g->loc[k].xrecv[ri],
                               g->loc[k].halt_hdr, &e->d_ring[i + 2], (const DevCtl*)e->d_ctl, i, g->window,
                               g->loc[k].parts);
            if (g->p2p) continue;   // k_xchg below folds the shares
            hipLaunchKernelGGL(k_xfold, dim3(1), dim3(64), 0, e->stream, dp(xparams(g, k, &e->d_ring[i + 1])),
                               (const TlPart*)g->loc[k].parts, (uint32_t)grid, i, (const DevCtl*)e->d_ctl);
        }
        if (g->p2p) {   // fold + put, then wait and ingest; the tag is ctl->xtag + i
            const int wi = (int)(g->xseq & 1);
            shd_eng* e = g->engs[0];
            const Params P = xparams(g, 0, &e->d_ring[i + 1]);
            const uint32_t nblk = (uint32_t)((e->nloc + e->P.hpw - 1) / e->P.hpw);
            const uint64_t nthr = (uint64_t)g->world * g->xcap;
            hipLaunchKernelGGL(k_xchg, dim3((unsigned)(g->world + (nthr + 255) / 256)), dim3(256), 0, e->stream,
                               dp(P), (const TlPart*)g->loc[0].parts, nblk, i, (const DevCtl*)e->d_ctl,
                               (shd_event* const*)g->d_peers, g->rank0, wi, (uint32_t)i,
                               (const shd_event*)g->loc[0].xrecv[wi], g->d_xerr);
            g->xseq++;
            continue;
        }
        if ((rc = x_exchange(g))) return rc;
        const int wi = (int)((g->xseq - 1) & 1);
        for (int k = 0; k < nl; k++) {
            shd_eng* e = g->engs[k];
            const Params P = xparams(g, k, &e->d_ring[i + 1]);
            const uint64_t nthr = (uint64_t)g->world * g->xcap;
            hipLaunchKernelGGL(k_ingest_x, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, e->stream, dp(P),
                               (const shd_event*)g->loc[k].xrecv[wi], (const DevCtl*)e->d_ctl, i);
        }
    }
    return SHD_OK;
}

// a full batch replays a captured graph when the transport allows it (RCCL,
// one engine per process); a capture that fails is not tried again
static int x_launch_rounds(shd_xgroup* g, int nb) {
    static const bool no_graph = getenv("SHD_NO_GRAPH") != nullptr;
    if (nb != shd_eng::kBatch || !g->comm || (g->comm->kind != SHD_COMM_RCCL && !g->p2p) || g->engs.size() != 1 ||
        g->graph_failed || no_graph)
        return x_enqueue_rounds(g, nb);
    shd_eng* e = g->engs[0];
    const int par = (int)(g->xseq & 1);
    hipGraphExec_t& ge = g->graph[g->fused && x_sparse(g) ? 1 : 0][par];
    if (!ge) {
        const uint64_t xseq0 = g->xseq;
        hipGraph_t gr = nullptr;
        SHD_HIP(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
        const int rc = x_enqueue_rounds(g, nb);
        const hipError_t ec = hipStreamEndCapture(e->stream, &gr);
        g->xseq = xseq0;
        hipError_t ei = hipErrorUnknown;
        if (rc == SHD_OK && ec == hipSuccess && gr) ei = hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
        if (gr) (void)hipGraphDestroy(gr);
        if (ei != hipSuccess) {
            ge = nullptr;
            (void)hipGetLastError();
            g->graph_failed = true;
            fprintf(stderr, "libshdgpu: engine-group batch capture failed (rc %d, %s); launching directly\n", rc,
                    hipGetErrorString(ec != hipSuccess ? ec : ei));
            return x_enqueue_rounds(g, nb);
        }
    }
    SHD_HIP(hipGraphLaunch(ge, e->stream));
    g->xseq += (uint64_t)nb;   // one exchange per round, as the direct launch counts them
    return SHD_OK;
}

extern "C" int shd_xgroup_run_until(shd_xgroup* g, uint64_t t_stop, shd_run_stats* st) {
    if (!g) return SHD_EINVAL;
    auto t0 = std::chrono::steady_clock::now();
    const int nl = (int)g->engs.size();
    int rc = SHD_OK;
    shd_run_stats s{};
    s.window_ns = g->window;
    for (shd_eng* e : g->engs) {
        SHD_HIP(hipSetDevice(e->device));
        if (!e->booted && (rc = shd_eng_boot(e))) return rc;
    }
    if (!g->started) {
        // the first headers: every engine's next event time after boot
        for (int k = 0; k < nl; k++) {
            shd_eng* e = g->engs[k];
            SHD_HIP(hipMemsetAsync(e->d_halt, 0, 4, e->stream));
            hipLaunchKernelGGL(k_xpack, dim3(1), dim3(64), 0, e->stream, dp(xparams(g, k, e->d_sum)), e->d_sum, 1);
        }
        if ((rc = x_exchange(g))) return rc;
        g->started = true;
    }
    if ((rc = x_read_next(g))) return rc;
    const uint64_t stop = std::min<uint64_t>(t_stop, g->end_time);
    constexpr int B = shd_eng::kBatch;
    std::vector<uint64_t> pend0(nl);
    for (int k = 0; k < nl; k++) pend0[k] = g->engs[k]->pending_resolved;
    double kms = 0;
    while (g->next < stop && rc == SHD_OK) {
        g->batches++;
        // a protected batch is one round behind a copy of every engine's device
        // state (the exchange buffers are engine allocations too)
        const bool prot = x_want_protect(g);
        const int nb = prot ? 1 : B;
        const uint64_t xseq0 = g->xseq, next0 = g->next;
        const int last_nb0 = g->last_nb;
        std::vector<uint64_t> round0(nl);
        if (prot) {
            for (int k = 0; k < nl && !rc; k++) {
                round0[k] = g->engs[k]->round;
                SHD_HIP(hipSetDevice(g->engs[k]->device));
                g->engs[k]->snap_valid = false;   // the group's copy, not a run_until restore point
                rc = snapshot_state(g->engs[k], false);
            }
            if (rc) break;
            s.n_rounds_protected++;
        }
        for (int k = 0; k < nl; k++) {
            shd_eng* e = g->engs[k];
            // slot 0 keeps the previous batch's last round: a flag in its
            // headers halts this batch's first round, and the recovery needs it
            SHD_HIP(hipMemcpyAsync(&e->d_ring[0], &e->d_ring[g->last_nb], sizeof(DevSummary), hipMemcpyDeviceToDevice,
                                   e->stream));
            e->h_seed[1] = host_fresh_summary();
            e->h_ctl->stop = stop;
            e->h_ctl->round_base = e->round;
            e->h_ctl->xtag = g->xepoch + 1;   // peer-to-peer: round i's exchange is tagged xtag + i
            e->h_ctl->xpar = g->xseq & 1;     // peer-to-peer: round i's receive blocks have parity xpar + i
            SHD_HIP(hipMemcpyAsync(&e->d_ring[1], &e->h_seed[1], sizeof(DevSummary), hipMemcpyHostToDevice,
                                   e->stream));
            SHD_HIP(hipMemcpyAsync(e->d_ctl, e->h_ctl, sizeof(DevCtl), hipMemcpyHostToDevice, e->stream));
            SHD_HIP(hipMemsetAsync(e->d_halt, 0, 4, e->stream));
        }
        SHD_HIP(hipEventRecord(g->engs[0]->bev[0], g->engs[0]->stream));
        const bool sparse_batch = g->fused && x_sparse(g);
        if ((rc = x_launch_rounds(g, nb))) break;
        s.n_batches++;
        if (sparse_batch) s.n_batches_sparse++;
        g->xepoch += (uint64_t)nb;
        SHD_HIP(hipGetLastError());
        SHD_HIP(hipEventRecord(g->engs[0]->bev[1], g->engs[0]->stream));
        for (int k = 0; k < nl; k++) {
            shd_eng* e = g->engs[k];
            SHD_HIP(hipMemcpyAsync(e->h_ring, e->d_ring, sizeof(DevSummary) * (B + 1), hipMemcpyDeviceToHost,
                                   e->stream));
        }
        // one engine per process: the last exchange's headers and the wait-error word
        // come back with the summaries (no synchronous copy of its own for each)
        const bool prefetched = g->h_hdr && nl == 1;
        if (prefetched) {
            shd_eng* e = g->engs[0];
            SHD_HIP(hipMemcpy2DAsync(g->h_hdr, sizeof(XHeader), g->loc[0].xrecv[(g->xseq - 1) & 1],
                                     g->stride * sizeof(shd_event), sizeof(XHeader), g->world,
                                     hipMemcpyDeviceToHost, e->stream));
            if (g->p2p) SHD_HIP(hipMemcpyAsync(g->h_xerr, g->d_xerr, 4, hipMemcpyDeviceToHost, e->stream));
        }
        for (int k = 0; k < nl; k++) SHD_HIP(hipStreamSynchronize(g->engs[k]->stream));
        if (prefetched && g->p2p ? *g->h_xerr != 0 : false) {
            fprintf(stderr, "libshdgpu: peer-to-peer exchange: a peer's block did not come within %llu s\n",
                    kXWaitTicks / 100000000ull);
            rc = SHD_ENODEV;
            break;
        }
        if (!prefetched && (rc = x_p2p_check(g))) break;
        {
            float ms = 0;   // the batch on engine 0's stream: rounds + exchanges
            if (hipEventElapsedTime(&ms, g->engs[0]->bev[0], g->engs[0]->bev[1]) == hipSuccess)
                s.device_ms_launches += ms;
        }
        g->last_nb = nb;
        if (prot && g->engs[0]->h_ring[1].flags == 0u && g->engs[0]->h_ring[1].ws < stop) {
            // the round ran; its flags came back with its own exchange
            std::vector<XHeader> hh;
            if ((rc = x_headers(g, hh))) break;
            uint32_t fl = 0, errs = 0;
            for (const XHeader& x : hh) {
                fl |= x.flags;
                errs |= x.error;
            }
            if ((fl & XF_ERROR) && errs == (uint32_t)SHD_ERR_AMBIGUOUS) {
                std::vector<shd_pending> all;
                for (int k = 0; k < nl; k++) g->engs[k]->round_pending = g->engs[k]->h_ring[1].n_pending;
                if ((rc = x_gather_pending(g, all))) break;
                for (int k = 0; k < nl && !rc; k++) {
                    shd_eng* e = g->engs[k];
                    SHD_HIP(hipSetDevice(e->device));
                    if ((rc = snapshot_state(e, true))) break;
                    e->round = round0[k];
                    e->parity = (int)(e->round & 1);
                    rc = assign_ranks(e, all.data(), all.size());
                }
                if (rc) break;
                g->xseq = xseq0;
                g->next = next0;
                g->last_nb = last_nb0;
                s.n_rounds_rerun++;
                continue;   // the same round again, protected again, every pair of its log ranked
            }
        }
        int halted_at = -1;
        bool done = false;
        for (int i = 0; i < nb; i++) {
            const DevSummary& r0 = g->engs[0]->h_ring[i + 1];
            if (r0.flags == 1u) { halted_at = i; break; }
            if (r0.flags != 0u) break;   // skipped: cannot precede a halt
            if (r0.ws >= stop) {
                g->next = r0.ws;
                done = true;
                break;
            }
            s.n_rounds++;
            uint64_t we = r0.ws + g->window;
            if (we > stop || we < r0.ws) we = stop;
            s.final_time = we;
            for (int k = 0; k < nl; k++) {
                shd_eng* e = g->engs[k];
                const DevSummary& r = e->h_ring[i + 1];
                s.n_events += r.n_events;
                s.n_pkt_events += r.n_pkt_events;
                s.n_host_rounds += r.n_active;
                const double ms = round_kernel_ms(e, r);
                kms += ms;
                e->last_kernel_ms = ms;
                e->round++;
                e->parity = (int)(e->round & 1);
            }
        }
        if (g->sp_grid && !g->sp_forced && nl == 1) {   // the next batch's kernel, from this batch's activity
            uint64_t br = 0, ba = 0, bp = 0;
            const int upto = halted_at >= 0 ? halted_at : nb;
            for (int i = 0; i < upto; i++) {
                const DevSummary& r0 = g->engs[0]->h_ring[i + 1];
                if (r0.flags != 0u || r0.ws >= stop) break;
                br++;
                ba += r0.n_active;
                bp += r0.n_pkt_events;
            }
            if (br) g->sp_dense = sp_dense_batch(br, ba, bp, (uint64_t)g->engs[0]->nloc);
        }
        if (done) break;
        if (halted_at < 0) {
            g->last_logged = 0;
            if (prefetched) x_next_from(g, g->h_hdr, g->world);
            else if ((rc = x_read_next(g))) break;
            continue;
        }
        g->last_logged = 0;
        // the round before halted_at (ring slot halted_at) was flagged somewhere in the group
        const int slot = halted_at;
        std::vector<XHeader> hh(g->world);
        SHD_HIP(hipMemcpy(hh.data(), g->loc[0].halt_hdr, sizeof(XHeader) * g->world, hipMemcpyDeviceToHost));
        uint32_t fl = 0;
        uint32_t errs = 0;
        for (const XHeader& x : hh) {
            fl |= x.flags;
            errs |= x.error;
        }
        if (fl & XF_ERROR) {
            s.error = errs;
            rc = (errs & SHD_ERR_AMBIGUOUS) ? SHD_EAMBIG : SHD_EOVERFLOW;
            break;
        }
        if (fl & XF_PENDING) {
            std::vector<shd_pending> all;
            for (int k = 0; k < nl; k++) g->engs[k]->round_pending = g->engs[k]->h_ring[slot].n_pending;
            if ((rc = x_gather_pending(g, all))) break;
            g->last_logged = all.size();
            if (!all.empty()) g->logged_any = true;
            for (int k = 0; k < nl && !rc; k++) {
                shd_eng* e = g->engs[k];
                DevSummary* const keep = e->P.sum;
                e->P.sum = &e->d_ring[slot];           // the flagged round's summary; remote -> e->P.remote
                e->parity = (int)((e->round - 1) & 1);  // the flagged round's parity
                rc = shd_eng_resolve(e, all.data(), all.size());
                e->P.sum = keep;
                e->parity = (int)(e->round & 1);
            }
            if (rc) break;
            for (int k = 0; k < nl; k++) SHD_HIP(hipStreamSynchronize(g->engs[k]->stream));
        }
        if ((rc = x_exchange_remote(g, slot))) break;
        if ((fl & XF_OVERFLOW) && !g->fixed_cap) {
            // spills in two consecutive batches: the blocks are too small for
            // this traffic, not just for a burst.  Every rank sees the same
            // flags in the same batch, so all grow alike.
            if (g->last_spill_batch != ~0ull && g->batches - g->last_spill_batch <= 1) {
                if (g->fused && g->xcap >= kXSlots) {
                    // fused rounds spill from a full region (kXSlots events per
                    // peer and destination block, whatever xcap): when it
                    // persists past single protected rounds (the application
                    // start's burst), a hot block outruns its regions, and the
                    // two-launch schedule takes over, whose per-peer blocks of
                    // xcap events do not spill
                    if (nb > 1) {
                        g->fused = false;
                        x_drop_graphs(g);
                        if ((rc = x_alloc(g))) break;
                    }
                } else if (g->xcap < (1u << 22)) {
                    g->xcap *= 2;
                    x_drop_graphs(g);   // the graphs point at the old blocks
                    if ((rc = x_alloc(g))) break;
                }
            }
            g->last_spill_batch = g->batches;
        }
        // fresh headers: next event times after the recovery, no flags
        for (int k = 0; k < nl; k++) {
            shd_eng* e = g->engs[k];
            SHD_HIP(hipMemsetAsync(e->d_halt, 0, 4, e->stream));
            hipLaunchKernelGGL(k_xpack, dim3(1), dim3(64), 0, e->stream, dp(xparams(g, k, &e->d_ring[slot])),
                               (const DevSummary*)&e->d_ring[slot], 1);
        }
        if ((rc = x_exchange(g))) break;
        for (int k = 0; k < nl; k++) {
            DevSummary r;
            shd_eng* e = g->engs[k];
            SHD_HIP(hipMemcpyAsync(&r, &e->d_ring[slot], sizeof(r), hipMemcpyDeviceToHost, e->stream));
            SHD_HIP(hipStreamSynchronize(e->stream));
            if (r.error) {
                s.error |= r.error;
                rc = (r.error & SHD_ERR_AMBIGUOUS) ? SHD_EAMBIG : SHD_EOVERFLOW;
            }
        }
        if (rc) break;
        if ((rc = x_read_next(g))) break;
    }
    for (int k = 0; k < nl; k++) {
        shd_eng* e = g->engs[k];
        e->h_sum->next_time = g->next;
        if (rc == SHD_OK) e->t_done = std::max<uint64_t>(e->t_done, std::min<uint64_t>(stop, g->next));
        s.n_pending_resolved += e->pending_resolved - pend0[k];
    }
    s.device_ms_round_kernel = kms;
    s.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (st) *st = s;
    return rc;
}
