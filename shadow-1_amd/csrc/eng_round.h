// eng_round.h -- the round kernels of one engine: boot, the round body (idle
// test, calendar merge, event loop, flush, close), round completion, the
// ticketed (k_round_dev) and ticketless (k_round_tl) batches, first-touch
// finalization, pushed events, digests.
// Part of libshdgpu's engine translation unit (csrc/engine.hip includes it
// inside its anonymous namespace); not a standalone header.
#pragma once

// ------------------------------------------------------------------ kernels

// host_boot for every local host at t = 0 (host.c:372-390)
__global__ __launch_bounds__(kBlock) void k_boot(DParams P, const uint32_t* __restrict__ rng0,
                                                  const uint64_t* __restrict__ bw_down,
                                                  const uint64_t* __restrict__ bw_up) {
    const int32_t l = blockIdx.x * kBlock + threadIdx.x;
    uint64_t next = kInf;
    uint32_t err = 0;
    if (l < P.nloc) {
        const uint32_t h = (uint32_t)(P.h0 + l);
        // _networkinterface_setupTokenBuckets (network_interface.c:192-226)
        const uint64_t rxr = bw_down[h] * 1024 / 1000, txr = bw_up[h] * 1024 / 1000;
        // bucket capacity refill + MTU within the record's 32 bits
        if (((rxr + SHD_MTU) | (txr + SHD_MTU)) >> 32) err |= SHD_ERR_INTERNAL;
        HostRec r;
        r.ev_seq = 0; r.cq_total = 0; r.cq_iexp = 0; r.cq_ndrop = 0; r.rx_rem = 0; r.tx_rem = 0;
        for (int k = 0; k < 3; k++) { r.tt[k] = kInf; r.ts_back[k] = 0; }
        P.hc[l] = HostCnt{0, 0, 0, 0, 0, 0};
        r.rng = rng0[h]; r.pkt_seq = 0; r.rx_refill = (uint32_t)rxr; r.tx_refill = (uint32_t)txr;
        r.flags = P.app_mode ? (uint32_t)P.app_mode[h] << kAppShift : 0u;   // (F_APP: the host's application)
        r.unread = 0; r.cq_dc = 0; r.cq_dcl = 0; r.cq_head = 0; r.cq_count = 0;
        r.tq_head = 0; r.tq_count = 0; r.evq_n = 0; r.if_in = 0; r.if_out = 0; r.rq_head = 0; r.port = 0;
        P.hs[l] = r;
        P.inbox_n[0][l] = 0; P.inbox_n[1][l] = 0;
        HostCtx c;
        hot_load(P, c);
        load_ctx(P, c, l, r, P.host_att[h], P.self_thr[h]);
        c.now = 0;
        c.q_seq = 0; c.q_src = c.h; c.q_sub = 0;
        schedule_self(P, c, SHD_EV_HEARTBEAT, hb_interval(P, c.k.feat, h), 0);   // tracker_new, tracker.c:141,607-610
        refill_cb(P, c);                                               // ethernet startRefilling
        schedule_self(P, c, SHD_EV_REFILL_LO, SHD_MS, 0);              // loopback refill at +1 ms
        if (!P.no_app_start) schedule_self(P, c, SHD_EV_APP_START, P.app_start, 0);   // process_schedule
        store_ctx(P, c);
        next = host_next(c);
        err |= c.err;
    }
    block_reduce_publish<kBlock>(P, next, 0, 0, err);
}

// a calendar slot's event, if it is one of the window's: onto the due list
// (unsorted; sorted once all bins are read).  `nw` counts the window's
// events; those past kDueCap go to the heap afterwards (due_overflow)
__device__ __forceinline__ void due_add(const EvV& x, uint32_t& nw, uint64_t ws, uint64_t we) {
    const uint64_t t = evv_time(x);
    if (t < ws || t >= we) return;
    if (nw < (uint32_t)kDueCap) ev_st(s_due + nw * kBlock + threadIdx.x, x);
    nw++;
}

// rare: more than kDueCap window events.  The bins are read again in the
// same order (the window's events in them cannot change during the round)
// and the events past the first kDueCap go to the heap
__device__ __forceinline__ void due_overflow(const DParams& P, HostCtx& c, uint64_t b0, uint32_t wbits, uint64_t ws,
                                          uint64_t we, uint32_t nrx = 0) {
    uint32_t k = 0;
    for (uint32_t j = 0; j < 3; j++) {
        if (((wbits >> j) & 1u) == 0) continue;
        const size_t bi = (size_t)c.l * kNB + ((uint32_t)(b0 + j) & (kNB - 1));
        for (uint32_t s = 0; s < kBinCap; s++) {
            const shd_event& x = P.bins[bi * kBinCap + s];
            if (x.time < ws || x.time >= we) continue;
            if (k >= (uint32_t)kDueCap) heap_push(P, c, x);
            k++;
        }
    }
    for (uint32_t r = 0; r < nrx; r++) {   // then the received ones, in the order due_add took them
        const shd_event& x = s_rx[r * kBlock + threadIdx.x];
        if (x.time < ws || x.time >= we) continue;
        if (k >= (uint32_t)kDueCap) heap_push(P, c, x);
        k++;
    }
}

// bit p of a bitmap held in registers (static word indices only)
__device__ __forceinline__ uint32_t bit_at(const uint32_t (&w)[kNBW], uint32_t p) {
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < (int)kNBW; j++) v |= (p >> 5) == (uint32_t)j ? w[j] : 0u;
    return (v >> (p & 31)) & 1u;
}

// the lane's host (P.nloc: none)
__device__ __forceinline__ int32_t lane_host(const DParams& P) {
    return (int32_t)threadIdx.x < P.hpw ? (int32_t)blockIdx.x * P.hpw + (int32_t)threadIdx.x : P.nloc;
}

// One scalar load per 64-B line of the Params copy, issued at kernel entry
// with the other first loads; consumed (params_warm_done) where the kernel
// waits for its window start anyway.  The round's later scalar loads of
// Params fields then hit the scalar cache instead of each paying an L2 trip.
__device__ __forceinline__ uint32_t params_warm(const DParams* Pp) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(Pp);
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < (int)((sizeof(DParams) + 63) / 64); k++) acc ^= w[k * 16];
    return acc;
}
__device__ __forceinline__ void params_warm_done(uint32_t acc) { asm volatile("" ::"s"(acc)); }

// what a round reads of a host before it knows the window: both inbox
// counts, the earliest timer/heap time, the calendar bitmap, the host record,
// its attached vertex and loopback thresholds.  None of it depends on the
// window start, so the round kernels issue these loads together with the
// loads of the window start and control words (one memory round trip).  The
// pointers come by value in the kernel arguments (RoundArgs), not through the
// Params pointer: one scalar load level instead of two before the first
// vector load.
template <template <class> class Ptr>
struct RoundArgsT {
    Ptr<const HostRec> hs;
    Ptr<const uint64_t> hnext;
    Ptr<const uint32_t> nin0, nin1;
    Ptr<const uint32_t> bits;   // null: no calendar
    Ptr<const int32_t> att;     // host_att + h0
    Ptr<const int4> st;         // self_thr + h0
    Ptr<const uint32_t> halt;
    int32_t nloc, hpw;
    uint32_t nblk;   // grid size (blocks of hpw hosts)
    uint32_t pad;
};
using DRoundArgs = RoundArgsT<GlobalPtr>;
static DRoundArgs round_args(const Params& P) {
    const DParams& d = dp(P);
    DRoundArgs a;
    a.hs = d.hs; a.hnext = d.hnext; a.nin0 = d.inbox_n[0]; a.nin1 = d.inbox_n[1];
    a.bits = d.bins ? d.bin_bits : nullptr;
    a.att = d.host_att + P.h0; a.st = d.self_thr + P.h0;
    a.halt = d.halt; a.nloc = P.nloc; a.hpw = P.hpw;
    a.nblk = (uint32_t)((P.nloc + P.hpw - 1) / P.hpw); a.pad = 0;
    return a;
}
__device__ __forceinline__ DRoundArgs round_args_dev(const DParams& P) {
    DRoundArgs a;
    a.hs = P.hs; a.hnext = P.hnext; a.nin0 = P.inbox_n[0]; a.nin1 = P.inbox_n[1];
    a.bits = P.bins ? P.bin_bits : nullptr;
    a.att = P.host_att + P.h0; a.st = P.self_thr + P.h0;
    a.halt = P.halt; a.nloc = P.nloc; a.hpw = P.hpw;
    a.nblk = (uint32_t)((P.nloc + P.hpw - 1) / P.hpw); a.pad = 0;
    return a;
}
struct HostIn {
    uint32_t nin[2];
    uint64_t t0;
    uint32_t w[kNBW];
    HostRec rec;
    int32_t att;
    int4 st;
};
// every lane loads (lanes past the last host read the last host's entries
// and ignore them): no branch, so no wait at a join before other loads issue
__device__ __forceinline__ void host_in_load(const DRoundArgs& a, HostIn& in) {
    const int32_t l0 = (int32_t)threadIdx.x < a.hpw ? (int32_t)blockIdx.x * a.hpw + (int32_t)threadIdx.x : a.nloc;
    const int32_t l = l0 < a.nloc ? l0 : a.nloc - 1;
    // the idle test's words first: the idle test and the window's bin loads
    // wait for them only, not for the 160-B record behind them
    in.nin[0] = a.nin0[l];
    in.nin[1] = a.nin1[l];
    in.t0 = a.hnext[l];
    if (a.bits) {
        const uint4* bp = (const uint4*)(a.bits + (size_t)l * kNBW);
        const uint4 x = bp[0], y = bp[1];
        in.w[0] = x.x; in.w[1] = x.y; in.w[2] = x.z; in.w[3] = x.w;
        in.w[4] = y.x; in.w[5] = y.y; in.w[6] = y.z; in.w[7] = y.w;
    } else {
#pragma unroll
        for (int j = 0; j < (int)kNBW; j++) in.w[j] = 0;
    }
}

// one round [ws, we): merge inbox[parity] and the calendar bins of the
// window, run events < we
// RX: the fused peer-to-peer round's received window events (s_rx).  LEAN
// (round 6): the model uses none of the optional features (ParamsT::feat == 0)
// and has no bootstrap period -- the bench's models: the context's feature
// word and bootstrap end are the constant 0, so the trace, status, heartbeat,
// path-counter and datagram-application paths and the bootstrapping tests fold
// away (registers and issue the PHOLD path does not need)
template <bool RX = false, bool LEAN = false>
__device__ __forceinline__ void round_body(const DParams& P, const HostIn& in, uint64_t ws, uint64_t we, int parity,
                                           uint64_t& next_out, uint64_t& nev_out, uint64_t& npkt_out,
                                           uint32_t& err_out, uint32_t xwi = 0) {
    const int32_t l = lane_host(P);
#ifdef SHD_PROF
    const unsigned long long w0 = wall_clock64();
#endif
    TIM(1);
#ifdef SHD_TIMING
    if (threadIdx.x == 0)
        for (int i = 0; i < 10; i++)
            for (int j = 0; j < 4; j++) s_kc[i][j] = 0;
#endif
    uint64_t next = kInf, nev = 0, npkt = 0;
    uint32_t err = 0;
    // the window's calendar bins: b0 .. b0 + nbin - 1 (nbin <= 3: bin width <= W)
    const uint64_t b0 = ws >> P.bin_shift;
    const uint32_t nbin = P.bins ? (uint32_t)(((we - 1) >> P.bin_shift) - b0) + 1u : 0u;
    uint32_t w[kNBW];
    // hosts with nothing due this round touch 3 words and their bitmap, not their whole state
    bool idle = false;
    uint32_t wbits = 0;   // bit j: window bin j is non-empty
    HostRec rec;
    int32_t rec_att;
    int4 rec_st;
    uint32_t nin0 = 0;
    if (l < P.nloc) {
        nin0 = parity ? in.nin[1] : in.nin[0];
        const uint64_t t0 = in.t0;
#pragma unroll
        for (int j = 0; j < (int)kNBW; j++) w[j] = in.w[j];
        if (P.bins) {
#pragma unroll
            for (uint32_t j = 0; j < 3; j++)
                if (j < nbin) wbits |= bit_at(w, (uint32_t)(b0 + j) & (kNB - 1)) << j;
        } else {
#pragma unroll
            for (int j = 0; j < (int)kNBW; j++) w[j] = 0;
        }
        if (nbin > 3) err |= SHD_ERR_INTERNAL;   // window wider than W
        if (nin0 == 0 && t0 >= we && wbits == 0 && (!RX || s_rxn[threadIdx.x] == 0)) {
            idle = true;
            next = t0;
            if (P.bins) {
                // the window's bins hold nothing: their counts are zero (a
                // count is nonzero only behind a set bit, cal_push), no reset
                const uint64_t cb = cal_lower_bound(P, w, we);
                next = cb < next ? cb : next;
            }
        }
    }
    TIM(2);
    const bool active = l < P.nloc && !idle;
#ifdef SHD_TIMING
    uint64_t n_it = 0, k_tk = 0, k_be = 0, k_rw = 0, k_fl = 0, k_in = 0;
    uint64_t k_l0 = 0, n_kinds = 0, n_lanes = 0;
#ifdef SHD_TIMING_LIGHT   // phase stamps only: no clock reads inside the event loop
#define KT0(v)
#define KTA(acc, v)
#else
#define KT0(v) const uint64_t v = clock64();
#define KTA(acc, v) acc += clock64() - v;
#endif
#else
#define KT0(v)
#define KTA(acc, v)
#endif
    HostCtx c;   // idle lanes take part in the wave's flushes with no sends
    hot_load(P, c);
    if (LEAN) { c.k.feat = 0; c.k.boot_end = 0; }
    PendDel pd;
    send_pool_reset(c); c.att = 0; c.cls = 0; c.err = 0;
    c.ws = ws; c.ws_mod = (uint32_t)(ws % SHD_MS); c.np = parity ^ 1; c.xwi = xwi; c.xput = 0; c.pf_lim = 0;
    // the window's non-empty bins, all slots loaded before the host record is
    // consumed (one round trip, overlapping the record's)
    EvV bx[3][kBinCap];
    if (active && P.bins) {
#pragma unroll
        for (uint32_t j = 0; j < 3; j++) {
            if (((wbits >> j) & 1u) == 0) continue;
            const size_t bi = (size_t)l * kNB + ((uint32_t)(b0 + j) & (kNB - 1));
            static_assert(kBinCap == 4, "the slots are read as four named events");
            const auto bp = P.bins + bi * kBinCap;
#pragma unroll
            for (uint32_t k = 0; k < kBinCap; k++) bx[j][k] = ev_ld(bp + k);
        }
    }
    // the host record behind the bins, in the same round trip, for the
    // hosts with something due only (idle hosts' records are never read)
    if (active) {
        rec = P.hs[l];
        rec_att = P.host_att[P.h0 + l];
        rec_st = P.self_thr[P.h0 + l];
    }
    PROF_T0(t_all)
    if (active) {
        load_ctx(P, c, l, rec, rec_att, rec_st);
        TIMA(7);
        c.ws = ws;
        c.ws_mod = (uint32_t)(ws % SHD_MS);
        c.np = parity ^ 1;
#ifdef SHD_PROF
        c.prof = ProfAcc{};
#endif
        PROF_ADD(c, PR_LOAD, t_all)
        // merge inbound events of the previous round
        PROF_T0(t_m)
        const uint32_t nin = nin0;
        if (nin) {
            const shd_event* ib = P.inbox[parity] + (size_t)l * P.inbox_cap;
            const uint32_t n = nin < P.inbox_cap ? nin : P.inbox_cap;
            for (uint32_t i = 0; i < n; i++) { TCNT(4); heap_push(P, c, ib[i]); }
            P.inbox_n[parity][l] = 0;
        }
        // the window's calendar events, sorted into the due list.  The slots
        // of a non-empty bin are filtered by time alone: a slot never written
        // in the bin's current use holds kInf or an older use's event (before
        // ws), a slot being written by this round's appends holds a time >= we
        // (or still the old one), so the bin's count is not needed here
        if (P.bins) {
            uint32_t nw = 0;
#pragma unroll
            for (uint32_t j = 0; j < 3; j++) {
                if (((wbits >> j) & 1u) == 0) continue;
#pragma unroll
                for (uint32_t k = 0; k < kBinCap; k++) due_add(bx[j][k], nw, ws, we);
            }
            uint32_t nrx = 0;
            if (RX) {
                nrx = s_rxn[threadIdx.x];
                nrx = nrx < (uint32_t)kRxCap ? nrx : (uint32_t)kRxCap;
                for (uint32_t r = 0; r < nrx; r++) due_add(ev_ld(s_rx + r * kBlock + threadIdx.x), nw, ws, we);
            }
            c.nd = nw < (uint32_t)kDueCap ? nw : (uint32_t)kDueCap;
            if (nw > (uint32_t)kDueCap) due_overflow(P, c, b0, wbits, ws, we, nrx);
            // insertion sort of the due list (LDS only)
            for (uint32_t i = 1; i < c.nd; i++) {
                const EvV x = ev_ld(s_due + i * kBlock + threadIdx.x);
                uint32_t k = i;
                for (; k > 0; k--) {
                    const EvV y = ev_ld(s_due + (k - 1) * kBlock + threadIdx.x);
                    if (!evv_less(x, y)) break;
                    ev_st(s_due + k * kBlock + threadIdx.x, y);
                }
                ev_st(s_due + k * kBlock + threadIdx.x, x);
            }
            c.dt = c.nd ? s_due[threadIdx.x].time : kInf;
        }
        PROF_ADD(c, PR_MERGE, t_m)
        TIMA(8);
#ifdef SHD_TIMING
        k_l0 = clock64();
#endif
    }
    // the event loop.  An event's shared steps run in the same iteration as
    // its start.  A lane whose deferred sends need a flush before it can go
    // on (its send buffer is full, or a loopback send needs the exact event
    // ID) leaves the inner loop with its event suspended; the wave's flush
    // (all lanes, outside the inner loop) runs, and the suspended lanes
    // resume.  Normally the outer loop runs once: one flush per round.
    {
        // per-lane state: 0 needs its next event, 1 is running one, 2 waits
        // for a flush, 3 is done.  Both loops exit on wave-uniform tests only
        // (no divergent breaks: the exec-mask bookkeeping stays small).
        uint32_t st = active ? 0u : 3u;
        pd.kind = 0;
        for (;;) {
            KT0(q4)
            for (;;) {
#ifdef SHD_TIMING
                n_it++;
#endif
#if defined(SHD_TIMING) && !defined(SHD_TIMING_LIGHT)
                const uint64_t i_t0 = clock64();
                uint64_t i_tk = 0, i_be = 0;
                uint32_t i_cls = 0;
#endif
                if (st == 0u) {
                    PROF_T0(t_p)
                    shd_event e;
                    KT0(q0)
                    const bool more = take_next(P, c, we, e);
                    KTA(k_tk, q0)
#if defined(SHD_TIMING) && !defined(SHD_TIMING_LIGHT)
                    i_tk = clock64();
                    if (more) {
                        i_cls = e.kind & 7;
                        if (e.kind == SHD_EV_PACKET && !(c.cq_count == 0 && c.rx_rem >= SHD_MTU && !bootstrapping(P, c)))
                            i_cls = 8;
                    }
#endif
                    PROF_ADD(c, PR_POP, t_p)
#if defined(SHD_TIMING) && !defined(SHD_TIMING_LIGHT)
                    {   // divergence census: distinct event kinds started in this iteration
                        const uint32_t ks = more ? 1u << (e.kind & 31) : 0u;
                        for (uint32_t b = 1; b < 8; b++) n_kinds += __ballot((ks >> b) & 1u) != 0;
                        n_lanes += __popcll(__ballot(ks != 0));
                    }
#endif
                    if (more) {
                        c.now = e.time;
                        KT0(q1)
                        begin_event(P, c, e);
                        KTA(k_be, q1)
#if defined(SHD_TIMING) && !defined(SHD_TIMING_LIGHT)
                        i_be = clock64();
#endif
                        st = ((c.w_fl & ~W_READ) | c.w_msgs) ? 1u : 0u;   // the shared steps, if any are left
#ifndef SHD_NO_FUSE
                        // An arrival schedules its notification at +1 ns, and
                        // that is almost always the host's next event: when the
                        // notification timer is strictly the earliest candidate
                        // (so take_next would return it next) and in the window,
                        // it runs now, in the same iteration (the wave's lanes
                        // then run arrival + notification together instead of
                        // spreading them over two iterations)
                        if (st == 0u && c.tt2 < we) {
                            const uint64_t t = c.tt2, ht = c.evq_n ? c.top_time : kInf;
                            if (t < c.tt0 && t < c.tt1 && t < c.dt && t < ht && notify_fast_ok(P, c)) {
                                TCNT(5);
                                c.tt2 = kInf;
                                c.now = t;
                                c.c_events++;
                                c.q_seq = c.ts2; c.q_src = c.h; c.q_sub = 0;
                                c.w_msgs = 0; c.w_fl = 0;
                                notify_fast(P, c);
                                st = c.w_fl ? 1u : 0u;
                            }
                        }
                        // the same for the periodic refill (at the next 1 ms
                        // boundary) with both queues empty
                        if (st == 0u && c.tt1 < we) {
                            const uint64_t t = c.tt1, ht = c.evq_n ? c.top_time : kInf;
                            if (t < c.tt0 && t < c.tt2 && t < c.dt && t < ht && c.cq_count == 0 && c.tq_count == 0) {
                                TCNT(5);
                                c.tt1 = kInf;
                                c.now = t;
                                c.c_events++;
                                c.q_seq = c.ts1; c.q_src = c.h; c.q_sub = 0;
                                c.w_msgs = 0; c.w_fl = 0;
                                refill_fast(P, c);
                            }
                        }
#endif
                    } else {
                        st = 3u;
                    }
                }
                if (st == 1u) {
                    KT0(q2)
                    st = run_work(P, c) ? 0u : 2u;
                    KTA(k_rw, q2)
                }
#if defined(SHD_TIMING) && !defined(SHD_TIMING_LIGHT)
                {
                    const uint64_t i_t1 = clock64();
                    const uint64_t m = __ballot(i_cls != 0);
                    if (m) {
                        const int f = __ffsll((unsigned long long)m) - 1;
                        const uint32_t u = __shfl(i_cls, f, 64);
                        const uint64_t tk = __shfl(i_tk, f, 64), be = __shfl(i_be, f, 64);
                        if (__ballot(i_cls != 0 && i_cls != u) == 0 && threadIdx.x == 0) {
                            s_kc[u][0] += 1;
                            s_kc[u][1] += i_t1 - i_t0;
                            s_kc[u][2] += tk - i_t0;
                            s_kc[u][3] += be - tk;
                        }
                    }
                }
#endif
                if (__ballot(st <= 1u) == 0) break;
            }
            KTA(k_in, q4)
            KT0(q3)
            if (threadIdx.x == 0) TCNT(6);
            if (st == 2u) TCNT(7);
#ifdef SHD_TIMING_LIGHT
            TIM(11);   // the (last) flush starts
#endif
            const bool last = __ballot(st == 2u) == 0;   // no lane waits to resume: the round's last flush
            flush_wave(P, c, last, pd);
            KTA(k_fl, q3)
            if (last) break;
            if (st == 2u) st = 1u;
        }
    }
    TIM(9);
    if (active) {
#if defined(SHD_TIMING) && !defined(SHD_TIMING_LIGHT)
        {
            uint64_t v[7] = {n_it, k_tk, k_be, k_rw, clock64() - k_l0, k_fl, k_in};
#pragma unroll
            for (int j = 0; j < 7; j++)
                for (int off = 32; off > 0; off >>= 1) {
                    const uint64_t o = __shfl_xor(v[j], off, 64);
                    v[j] = o > v[j] ? o : v[j];
                }
            TIMV(11, v[0]);
            TIMV(12, v[1]);
            TIMV(13, v[2]);
            TIMV(14, v[3]);
            TIMV(15, v[4]);
            TIMV(16, v[5]);
            TIMV(17, v[6]);
            TIMV(18, n_kinds);
            TIMV(19, n_lanes);
        }
#endif
        next = host_next(c);
        if (c.min_emit < next) next = c.min_emit;
        if (P.bins) {
            // bins wholly before we are consumed: reset them (no append of
            // this round can target them: appends are >= we and within the
            // horizon).  Only a bin with its bit set has a nonzero count: an
            // append that claims a slot sets the bit once its event is stored,
            // and one past the capacity follows the claims below it (cal_push,
            // flush), so the empty bins' counts are left alone -- a store per
            // host and bin, most of the round's write traffic otherwise.
#pragma unroll
            for (uint32_t j = 0; j < 3; j++) {
                const uint64_t b = b0 + j;
                if (j < nbin && ((b + 1) << P.bin_shift) <= we && ((wbits >> j) & 1u)) {
                    const uint32_t p = (uint32_t)b & (kNB - 1);
                    P.bin_n[(size_t)l * kNB + p] = 0;
                    const uint32_t m = 1u << (p & 31);
                    atomicAnd(&P.bin_bits[(size_t)l * kNBW + (p >> 5)], ~m);
#pragma unroll
                    for (int k = 0; k < (int)kNBW; k++)
                        if ((p >> 5) == (uint32_t)k) w[k] &= ~m;
                }
            }
            const uint64_t cb = cal_lower_bound(P, w, we);
            next = cb < next ? cb : next;
        }
        nev = c.c_events;
        npkt = c.c_pkt;
        err |= c.err;
        PROF_T0(t_s)
        TIMA(10);
        store_ctx(P, c);
        PROF_ADD(c, PR_STORE, t_s)
        PROF_ADD(c, PR_TOTAL, t_all)
#ifdef SHD_PROF
        c.prof.v[PR_NEV] = nev;
        for (int i = 0; i < PR_N; i++) {
            atomicAdd(&g_prof[i], c.prof.v[i]);
            atomicMax(&g_prof[PR_N + i], c.prof.v[i]);
        }
        atomicAdd(&g_prof[2 * PR_N], 1ull);
#endif
    }
#ifdef SHD_PROF
    {
        uint64_t mx = nev;
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t o = __shfl_xor(mx, off, 64);
            mx = o > mx ? o : mx;
        }
        const unsigned long long w1 = wall_clock64();
        if (threadIdx.x == 0) {
            unsigned long long* g = g_wave[((uintptr_t)P.sum / sizeof(DevSummary)) & 127];
            atomicMin(&g[0], w0);
            atomicMax(&g[1], w1);
            atomicMax(&g[2], w1 - w0);
            atomicAdd(&g[3], w1 - w0);
            atomicAdd(&g[4], 1ull);
            atomicMax(&g[5], (unsigned long long)mx);
            atomicAdd(&g[6], (unsigned long long)mx);
        }
    }
#endif
#ifdef SHD_TIMING
    if (threadIdx.x == 0)
        for (int i = 0; i < 10; i++)
            if (s_kc[i][0])
                for (int j = 0; j < 4; j++) atomicAdd(&g_kc[i][j], s_kc[i][j]);
#endif
    flush_finish(P, c, pd);
    err |= c.err;
    // peer-to-peer: a wave that stored into a peer's receive block drains
    // those stores before the round ends (k_xchg tags the blocks next)
    if (P.xpeer && __ballot(c.xput != 0)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    TIM(3);
    next_out = next; nev_out = nev; npkt_out = npkt; err_out = err;
}

__global__ __launch_bounds__(kBlock) void k_round(DParams P, uint64_t ws, uint64_t we, int parity) {
    uint64_t next, nev, npkt;
    uint32_t err;
    HostIn in;
    host_in_load(round_args_dev(P), in);
    round_body(P, in, ws, we, parity, next, nev, npkt, err);
    (void)round_complete(P, next, nev, npkt, err);
}

// finalize resolved pending sends: value from the min-rank row, then deliver
__device__ void finalize_one(const DParams& P, const Pending& r, int next_parity, uint64_t& next, uint32_t& err) {
    if (r.delivered != 1u) return;
    const PathVal pv = path_value(P, (int32_t)r.a, (int32_t)r.b);
    if (!pv.resolved) err |= SHD_ERR_AMBIGUOUS;
    if (P.pcount) {   // counted once the pair has its rank (incrementPathPacketCounter, worker.c:296)
        const int32_t a = (int32_t)r.a, b = (int32_t)r.b;
        const int32_t ra = P.complete ? kNoRank : P.rank[a], rb = a == b ? kNoRank : P.rank[b];
        const uint32_t adj = P.prefer_direct ? P.adj[(size_t)a * P.T + b] : 0u;
        atomicAdd(&P.pcount[path_key(P, a, b, ra, rb, adj)], 1u);
    }
    shd_event e;
    e.time = r.qtime + (uint64_t)ceil(pv.lat * (double)SHD_MS);
    e.seq = r.seq; e.src = r.qhost; e.dst = r.dst; e.pkt = r.pkt; e.kind = SHD_EV_PACKET;
    if (e.time >= P.end_time) return;
    if (e.time < next) next = e.time;
    const int32_t dl = (int32_t)e.dst - P.h0;
    if (dl >= 0 && dl < P.nloc) {
        uint32_t slot = atomicAdd(&P.inbox_n[next_parity][dl], 1u);
        if (slot >= P.inbox_cap) err |= SHD_ERR_INBOX_OVERFLOW;
        else P.inbox[next_parity][(size_t)dl * P.inbox_cap + slot] = e;
    } else {
        unsigned long long slot = atomicAdd(&P.sum->n_remote, 1ull);
        if (slot >= P.remote_cap) err |= SHD_ERR_REMOTE_OVERFLOW;
        else P.remote[slot] = e;
    }
}

__global__ void k_finalize(DParams P, const Pending* __restrict__ pend, uint32_t n, int next_parity) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t next = kInf;
    uint32_t err = 0;
    if (i < n) finalize_one(P, pend[i], next_parity, next, err);
    if (next != kInf) atomicMin(&P.sum->next_time, (unsigned long long)next);
    if (err) atomicOr(&P.sum->error, err);
}

// device-side first-touch resolution for rounds with few logged queries (the
// common case after warm-up), run by the last block of the round: rank the
// records by serial key (counting sort: keys are unique), one lane assigns
// row ranks in that order, every lane finalizes its records.  Larger rounds
// halt the batch for the host path (shd_eng_resolve).
constexpr int kResolveMax = 256;
__device__ __forceinline__ bool pend_less(const Pending& x, const Pending& y) {
    if (x.qtime != y.qtime) return x.qtime < y.qtime;
    if (x.qhost != y.qhost) return x.qhost < y.qhost;
    if (x.qsrc != y.qsrc) return x.qsrc < y.qsrc;
    if (x.qseq != y.qseq) return x.qseq < y.qseq;
    return x.qsub < y.qsub;
}

__device__ void resolve_block(const DParams& P, int next_parity) {
    __shared__ Pending recs[kResolveMax];
    __shared__ int16_t order[kResolveMax];
    const unsigned long long n = P.sum->n_pending;
    if (n == 0) return;
    if (n > (unsigned long long)kResolveMax) {
        if (threadIdx.x == 0) *P.halt = 1u;
        return;
    }
    const int cnt = (int)n;
    for (int i = threadIdx.x; i < cnt; i += blockDim.x) recs[i] = P.pend[i];
    __syncthreads();
    for (int i = threadIdx.x; i < cnt; i += blockDim.x) {
        int pos = 0;
        for (int j = 0; j < cnt; j++) pos += pend_less(recs[j], recs[i]) ? 1 : 0;
        order[pos] = (int16_t)i;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t nr = *P.next_rank;
        int32_t* rank = (int32_t*)P.rank;
        int32_t* srank = (int32_t*)P.self_rank;
        for (int k = 0; k < cnt; k++) {
            const Pending& r = recs[order[k]];
            const int32_t a = (int32_t)r.a, b = (int32_t)r.b;
            if (a == b) {
                if (rank[a] == kNoRank && srank[a] == kNoRank) srank[a] = nr++;
            } else if (P.directed) {
                if (rank[a] == kNoRank) rank[a] = nr++;
            } else {
                if (rank[a] == kNoRank && rank[b] == kNoRank) rank[a] = nr++;
            }
        }
        *P.next_rank = nr;
        __threadfence();
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // drop L1 lines of the rank arrays
    uint64_t next = kInf;
    uint32_t err = 0;
    for (int i = threadIdx.x; i < cnt; i += blockDim.x) finalize_one(P, recs[i], next_parity, next, err);
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(next, off, 64);
        next = o < next ? o : next;
        err |= __shfl_xor(err, off, 64);
    }
    if (threadIdx.x == 0) {
        if (next != kInf) atomicMin(&P.sum->next_time, (unsigned long long)next);
        if (err) atomicOr(&P.sum->error, err);
    }
}

// device-driven round i of a batch (single engine): the window start is the
// previous round's next event time (read on the device), so rounds run back
// to back from one batch launch (or graph) with no host round trip; the last
// block resolves the round's first-touch log.  A round past `stop` only
// forwards the time.  `init` is the next round's summary, initialised here.
// The hot kernels take Params through a pointer to a device copy (one per
// summary-ring slot): fields are scalar-loaded where used instead of all held
// in SGPRs, which otherwise spill to VGPR lanes around every branch.
__global__ __launch_bounds__(kBlock) void k_round_dev(DRoundArgs a, const DevSummary* __restrict__ prev,
                                                       const DevCtl* __restrict__ ctl, const DParams* __restrict__ Pp,
                                                       DevSummary* __restrict__ init, int i, uint64_t window) {
    const DParams& P = *Pp;
#ifdef SHD_TIMING
    if (threadIdx.x == 0 && blockIdx.x < 2048) g_tim[((uintptr_t)P.sum / sizeof(DevSummary)) & 63][blockIdx.x][0] = wall_clock64();
#endif
    // the round's inputs and the hosts' state, loaded together (one round trip)
    HostIn in;
    host_in_load(a, in);
    const uint32_t halt = *a.halt;
    const uint64_t stop = ctl->stop, rbase = ctl->round_base, ws = prev->next_time;
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    // one test of all three loads, so that they issue together (no wait
    // between the halt flag and the window start)
    if ((halt != 0) | (ws >= stop)) {
        if (halt == 0 && lead) {   // only forwards the time
            atomicMin(&P.sum->t_first, (unsigned long long)wall_clock64());
            *init = fresh_summary();
            atomicMin(&P.sum->next_time, (unsigned long long)ws);
        }
        return;
    }
    if (lead) {
        atomicMin(&P.sum->t_first, (unsigned long long)wall_clock64());
        *init = fresh_summary();
    }
    const int parity = (int)((rbase + (uint64_t)i) & 1);
    uint64_t we = ws + window;
    if (we > stop || we < ws) we = stop;
    uint64_t next, nev, npkt;
    uint32_t err;
    round_body(P, in, ws, we, parity, next, nev, npkt, err);
    TIM(4);
    if (!round_complete(P, next, nev, npkt, err)) {
        TIM(5);
        return;
    }
    TIM(5);
    if (threadIdx.x == 0) P.sum->ws = ws;
    resolve_block(P, parity ^ 1);
    TIM(6);
    if (threadIdx.x == 0) atomicMax(&P.sum->t_last, (unsigned long long)wall_clock64());
}

// Ticketless rounds.  Every block writes its share of the round's summary
// (TlPart) and ends; there is no completion ticket.  The next round's blocks
// each fold all the shares of this one (one load per lane, issued with the
// host-state loads) to get their window start, and its block 0 publishes the
// fold as this round's summary; k_fold_tl publishes the batch's last round.
// Without a ticket no block sees the whole round's first-touch log, so a
// round that logged is resolved by the host: the next round halts the batch.
// The host runs these batches once a batch has logged nothing.
struct TlPart {
    unsigned long long next, t_end;
    unsigned int nev, npkt, err, nact;   // nact: hosts with at least one event
};
__device__ __forceinline__ void tl_fold(TlPart& a, const TlPart& b) {
    a.next = b.next < a.next ? b.next : a.next;
    a.t_end = b.t_end > a.t_end ? b.t_end : a.t_end;
    a.nev += b.nev;
    a.npkt += b.npkt;
    a.err |= b.err;
    a.nact += b.nact;
}
// the wave's fold of the shares [0, n) (one wave per block)
__device__ __forceinline__ TlPart tl_gather(const TlPart* __restrict__ parts, uint32_t n) {
    TlPart f{kInf, 0, 0, 0, 0, 0};
    for (uint32_t j = threadIdx.x; j < n; j += 64) tl_fold(f, parts[j]);
    for (int off = 32; off > 0; off >>= 1) {
        TlPart o;
        o.next = __shfl_xor(f.next, off, 64);
        o.t_end = __shfl_xor(f.t_end, off, 64);
        o.nev = __shfl_xor(f.nev, off, 64);
        o.npkt = __shfl_xor(f.npkt, off, 64);
        o.err = __shfl_xor(f.err, off, 64);
        o.nact = __shfl_xor(f.nact, off, 64);
        tl_fold(f, o);
    }
    return f;
}
// The shares in two phases, so that their loads go out first and the
// host-state loads behind them (the window start waits only for these):
// tl_issue loads shares [base, base + 256) as four independent loads per lane
// (indices past the end read the last share and are not folded), tl_fold4
// folds them in
__device__ __forceinline__ void tl_issue(const TlPart* __restrict__ parts, uint32_t n, uint32_t base, TlPart (&v)[4]) {
    const uint32_t last = n - 1;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t j = base + 64u * k + threadIdx.x;
        v[k] = parts[j < n ? j : last];
    }
}
__device__ __forceinline__ void tl_fold4(TlPart& f, const TlPart (&v)[4], uint32_t n, uint32_t base) {
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (base + 64u * k + threadIdx.x < n) tl_fold(f, v[k]);
}
__device__ __forceinline__ void tl_reduce(TlPart& f, bool full) {
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(f.next, off, 64);
        f.next = o < f.next ? o : f.next;
        if (full) {
            const uint64_t te = __shfl_xor(f.t_end, off, 64);
            f.t_end = te > f.t_end ? te : f.t_end;
            f.nev += __shfl_xor(f.nev, off, 64);
            f.npkt += __shfl_xor(f.npkt, off, 64);
            f.err |= __shfl_xor(f.err, off, 64);
            f.nact += __shfl_xor(f.nact, off, 64);
        }
    }
}

// publish a round's fold into its summary; a round that logged first touches
// halts the batch (the host resolves its log)
__device__ __forceinline__ void tl_publish(DevSummary* s, const TlPart& f, uint32_t* halt) {
    if (f.next != kInf) atomicMin(&s->next_time, f.next);
    if (f.nev) atomicAdd(&s->n_events, (unsigned long long)f.nev);
    if (f.npkt) atomicAdd(&s->n_pkt_events, (unsigned long long)f.npkt);
    if (f.err) atomicOr(&s->error, f.err);
    if (f.nact) atomicAdd(&s->n_active, f.nact);
    atomicMax(&s->t_last, f.t_end);
    if (s->n_pending) *halt = 1u;
}

// round i of a ticketless batch: shares of round i go to parts[i & 1]
// (argument order: what the first memory round trip needs comes first, so
// that one scalar load batch brings all of it)
template <bool LEAN>
__global__ __launch_bounds__(kBlock) void k_round_tl(uint64_t window, int i, DevSummary* __restrict__ prev,
                                                      const DevCtl* __restrict__ ctl, TlPart* __restrict__ parts,
                                                      const DParams* __restrict__ Pp, DevSummary* __restrict__ init,
                                                      DRoundArgs a) {
    const DParams& P = *Pp;
#ifdef SHD_TIMING
    if (threadIdx.x == 0 && blockIdx.x < 2048) g_tim[((uintptr_t)P.sum / sizeof(DevSummary)) & 63][blockIdx.x][0] = wall_clock64();
#endif
    const unsigned long long t_entry = wall_clock64();   // the round's start on the device clock (t_first)
    const uint32_t nblk = a.nblk;   // == gridDim.x, without the dispatch-packet load
    // all scalar arguments in the first load batch (the compiler otherwise
    // fetches some after the first vector loads are issued, one level later)
    asm volatile("" ::"s"(i), "s"(prev), "s"(ctl), "s"(parts), "s"(nblk), "s"(a.nloc), "s"(a.hpw), "s"(window));
    // the window start's inputs go out first: halt, the control words, the
    // previous round's summary and its shares (round 0 of the batch starts at
    // the seeded time; later rounds fold the previous round's shares, whose
    // first-touch log count halts).  The host-state loads follow; the window
    // start then waits for its own loads only (vmcnt counts in issue order)
    uint32_t halt = *a.halt;
    uint64_t stop = ctl->stop, rbase = ctl->round_base, ws0 = prev->next_time, npend = prev->n_pending;
    const TlPart* pp = parts + (size_t)((i - 1) & 1) * nblk;
    TlPart pv[4];
    if (i > 0) tl_issue(pp, nblk, 0, pv);
    const uint32_t warm = params_warm(Pp);
    HostIn in;
    host_in_load(a, in);
    // consumed only here, once every load is out (the compiler would
    // otherwise move their scalar copies, and the waits, above the rest)
    asm volatile("" : "+v"(halt), "+v"(stop), "+v"(rbase), "+v"(ws0), "+v"(npend));
    // every block needs the shares' min next time; block 0 folds the rest
    // of them too, for the summary
    TlPart f{kInf, 0, 0, 0, 0, 0};
    if (i > 0) {
        tl_fold4(f, pv, nblk, 0);
        for (uint32_t base = 256; base < nblk; base += 256) {   // grids above 256 blocks
            tl_issue(pp, nblk, base, pv);
            tl_fold4(f, pv, nblk, base);
        }
        tl_reduce(f, blockIdx.x == 0);
    }
    const uint64_t ws = f.next < ws0 ? f.next : ws0;
    params_warm_done(warm);
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    if (lead && i > 0) tl_publish(prev, f, (uint32_t*)a.halt);
    TlPart* mine = parts + (size_t)(i & 1) * nblk + blockIdx.x;
    if ((halt != 0) | (i > 0 && npend != 0) | (ws >= stop)) {
        if (halt == 0 && !(i > 0 && npend != 0)) {   // only forwards the time
            if (lead) {
                atomicMin(&P.sum->t_first, t_entry);
                *init = fresh_summary();
                P.sum->ws = ws;
            }
            if (threadIdx.x == 0) *mine = TlPart{ws, (unsigned long long)wall_clock64(), 0, 0, 0, 0};
        }
        return;
    }
    if (lead) {
        atomicMin(&P.sum->t_first, t_entry);
        *init = fresh_summary();
        P.sum->ws = ws;
    }
    const int parity = (int)((rbase + (uint64_t)i) & 1);
    uint64_t we = ws + window;
    if (we > stop || we < ws) we = stop;
    uint64_t next, nev, npkt;
    uint32_t err;
    round_body<false, LEAN>(P, in, ws, we, parity, next, nev, npkt, err);
    TIM(4);
    const uint32_t nact = (uint32_t)__popcll(__ballot(nev != 0));   // hosts that executed an event
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(next, off, 64);
        next = o < next ? o : next;
        nev += __shfl_xor(nev, off, 64);
        npkt += __shfl_xor(npkt, off, 64);
        err |= __shfl_xor(err, off, 64);
    }
    if (threadIdx.x == 0)
        *mine = TlPart{next, (unsigned long long)wall_clock64(), (unsigned)nev, (unsigned)npkt, err, nact};
    TIM(5);
}

// after a ticketless batch: publish its last round (shares in parts[(n-1) & 1])
__global__ __launch_bounds__(64) void k_fold_tl(const TlPart* __restrict__ parts, uint32_t nblk, int last,
                                                DevSummary* __restrict__ s, uint32_t* __restrict__ halt) {
    const TlPart f = tl_gather(parts + (size_t)(last & 1) * nblk, nblk);
    if (threadIdx.x == 0 && *halt == 0u) tl_publish(s, f, halt);
}

// ------------------------------------------------------------- persistent rounds
// k_round_ps: a batch of rounds in ONE launch, for a single engine whose round
// grid fits the GPU one block per CU (10 k hosts: 157 blocks).  Every block
// keeps its 64 hosts' state (HostCtx) in registers, and their heap roots and
// FIFO heads in LDS, from the first round of the batch to the last; the
// records, next times and counters are stored once, at the end.  Between
// rounds there is no kernel boundary: each block publishes its share of the
// round (next time, flags; counts) as two tagged 16-B write-through granules
// into a parity slot, after its wave drained every hand-off store, and every
// block polls all shares of the round before it starts the next one -- the
// window start is their min (slave.c:437-462 / master.c:450-480's round step,
// as k_round_tl's fold).  Hand-offs between blocks within the launch follow
// the sc1-store / sc1-load form of MI355X_MICROARCH.md (inter-workgroup
// visibility): calendar and inbox events are stored with ev_st_sc1, the
// counts reset with agent-scope stores, claimed with atomics; the owner reads
// its bitmap, inbox counts, bins and inbox events with sc1 buffer loads.
// A round that logged a first touch, or an error, ends the launch after its
// summary is published (the host resolves it, as for k_round_tl); so does a
// window start at or past the stop time.
struct PsShare {
    uint4 a;   // next time lo, hi, flags (SHD_ERR_* | kPsPend), tag
    uint4 b;   // events, packet events, active hosts, tag
    uint4 c;   // k_round_ps: the noted destinations (note_dirty: local host, kDirtyNone, kDirtyAll) x 3, tag
};
static_assert(sizeof(PsShare) == 48, "three 16-B granules");
constexpr uint32_t kPsPend = 0x40000000u;   // share flag: the block's hosts logged a first touch
constexpr uint32_t kBufWord3 = 0x00020000u;  // raw buffer descriptor word 3 (gfx9)
constexpr int kAuxSc1 = 16;                   // buffer op cache policy: sc1 (agent scope)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint64_t bytes) {
    const uint32_t n = bytes > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)bytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)n, (int)kBufWord3);
}
__device__ __forceinline__ uint4 ld16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const v4u x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, kAuxSc1);
    return make_uint4(x[0], x[1], x[2], x[3]);
}
__device__ __forceinline__ uint32_t ld4_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, kAuxSc1);
}
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off, uint4 v) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const v4u x = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(x, r, (int)off, 0, kAuxSc1);
}
__device__ __forceinline__ shd_event evv_event(const EvV& x) {
    shd_event e;
    e.time = evv_time(x); e.seq = evv_seq(x);
    e.src = x.b.x; e.dst = x.b.y; e.pkt = x.b.z; e.kind = x.b.w;
    return e;
}

// this block's windows onto the hand-off arrays (the block's hosts only);
// nin / inbox: the round's parity (chosen per round by scalar selects: an
// array indexed by the parity would be kept in scratch)
struct PsRsrc {
    __amdgpu_buffer_rsrc_t bits, bins, nin, inbox;
};

// the rare overflow of the due list, as due_overflow, reading the bins again
// with sc1 loads (they may hold other blocks' appends of this launch)
__device__ __forceinline__ void ps_due_overflow(const DParams& P, HostCtx& c, const PsRsrc& R, uint32_t lb, uint64_t b0,
                                uint32_t wbits, uint64_t ws, uint64_t we) {
    uint32_t k = 0;
    for (uint32_t j = 0; j < 3; j++) {
        if (((wbits >> j) & 1u) == 0) continue;
        const uint32_t bi = lb * kNB + ((uint32_t)(b0 + j) & (kNB - 1));
        for (uint32_t s = 0; s < kBinCap; s++) {
            const uint32_t off = (bi * kBinCap + s) * 32u;
            const EvV x{ld16_sc1(R.bins, off), ld16_sc1(R.bins, off + 16)};
            const uint64_t t = evv_time(x);
            if (t < ws || t >= we) continue;
            if (k >= (uint32_t)kDueCap) heap_push(P, c, evv_event(x));
            k++;
        }
    }
}

// per-round fields of a persistent host context.  pf (k_round_ps with a
// calendar): the receivers load the next window's first kPfBins bins before
// the round's barrier, so appends to earlier bins are noted (HostCtx::pf_lim)
constexpr uint32_t kPfBins = 3;
__device__ __forceinline__ void ps_round_reset(const DParams& P, HostCtx& c, uint64_t ws, uint64_t we, int parity,
                                               bool pf) {
    c.ws = ws; c.ws_mod = (uint32_t)(ws % SHD_MS); c.np = parity ^ 1; c.xwi = 0; c.xput = 0;
    c.c_events = c.c_pkt = c.c_sent = c.c_idrop = c.c_cdrop = c.c_recv = 0;
    c.min_emit = kInf; c.err = 0; c.n_pend = 0;
    c.dh = 0; c.nd = 0; c.dt = kInf; send_pool_reset(c); c.seq_base = c.ev_seq;
    c.w_msgs = 0; c.w_fl = 0;
    c.pf_lim = pf ? (we >> P.bin_shift) + kPfBins : 0;
    if (pf && threadIdx.x == 0) s_dn = 0;
}

// The round of a lane's host once its hand-off words are read (nin: this
// parity's inbox count; w: the calendar bitmap, wbits its window bins), up to
// its event loop: bins and inbox merged into the due list and the heap, the
// window's wholly consumed bins reset.  `active` lanes run; the others take
// part in the wave's flushes only.  As round_body, with the hand-off arrays
// read by sc1 loads (other blocks of the launch wrote them).
// SP (k_round_sp): the context is loaded here, from the record the caller
// issued the loads of, once the bins' loads are out too (one round trip)
struct SpIn {
    HostRec rec;
    int32_t att;
    int4 st;
    int32_t l;
    uint32_t xwi;   // the engine group's exchange parity of the round (k_round_spx), else 0
};
template <bool SP>
__device__ __forceinline__ void ps_prologue(const DParams& P, HostCtx& c, bool active, uint32_t lb, const PsRsrc& R,
                                            uint64_t ws, uint64_t we, int parity, uint32_t nin, uint32_t (&w)[kNBW],
                                            uint32_t wbits, const SpIn* sp = nullptr) {
    const uint64_t b0 = ws >> P.bin_shift;
    const uint32_t nbin = P.bins ? (uint32_t)(((we - 1) >> P.bin_shift) - b0) + 1u : 0u;
    // the window's bins, every slot of a non-empty one in one round trip
    EvV bx[3][kBinCap];
    if (active && P.bins) {
#pragma unroll
        for (uint32_t j = 0; j < 3; j++) {
            if (((wbits >> j) & 1u) == 0) continue;
            const uint32_t bi = lb * kNB + ((uint32_t)(b0 + j) & (kNB - 1));
#pragma unroll
            for (uint32_t k = 0; k < kBinCap; k++) {
                const uint32_t off = (bi * kBinCap + k) * 32u;
                bx[j][k] = EvV{ld16_sc1(R.bins, off), ld16_sc1(R.bins, off + 16)};
            }
        }
    }
    if (SP) {
        if (active) load_ctx(P, c, sp->l, sp->rec, sp->att, sp->st);
        ps_round_reset(P, c, ws, we, parity, false);
        c.xwi = sp->xwi;
    }
    if (active) {
        if (nin) {   // inbound events of the previous round -> heap
            const uint32_t n = nin < P.inbox_cap ? nin : P.inbox_cap;
            for (uint32_t i = 0; i < n; i++) {
                const uint32_t off = (lb * P.inbox_cap + i) * 32u;
                TCNT(4);
                heap_push(P, c, evv_event(EvV{ld16_sc1(R.inbox, off), ld16_sc1(R.inbox, off + 16)}));
            }
            __hip_atomic_store(&P.inbox_n[parity][c.l], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (P.bins) {
            uint32_t nw = 0;
#pragma unroll
            for (uint32_t j = 0; j < 3; j++) {
                if (((wbits >> j) & 1u) == 0) continue;
#pragma unroll
                for (uint32_t k = 0; k < kBinCap; k++) due_add(bx[j][k], nw, ws, we);
            }
            c.nd = nw < (uint32_t)kDueCap ? nw : (uint32_t)kDueCap;
            if (nw > (uint32_t)kDueCap) ps_due_overflow(P, c, R, lb, b0, wbits, ws, we);
            for (uint32_t i = 1; i < c.nd; i++) {   // insertion sort of the due list (LDS)
                const EvV x = ev_ld(s_due + i * kBlock + threadIdx.x);
                uint32_t k = i;
                for (; k > 0; k--) {
                    const EvV y = ev_ld(s_due + (k - 1) * kBlock + threadIdx.x);
                    if (!evv_less(x, y)) break;
                    ev_st(s_due + k * kBlock + threadIdx.x, y);
                }
                ev_st(s_due + k * kBlock + threadIdx.x, x);
            }
            c.dt = c.nd ? s_due[threadIdx.x].time : kInf;
            // the window's wholly consumed bins: counts reset (write-through) and
            // bits cleared now, so that these stores land during the event loop
            // rather than in front of the round's share (no append of this round
            // can target them: appends are >= we and within the horizon)
#pragma unroll
            for (uint32_t j = 0; j < 3; j++) {
                const uint64_t b = b0 + j;
                if (j < nbin && ((b + 1) << P.bin_shift) <= we && ((wbits >> j) & 1u)) {
                    const uint32_t p = (uint32_t)b & (kNB - 1);
                    __hip_atomic_store(&P.bin_n[(size_t)c.l * kNB + p], 0u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    const uint32_t m = 1u << (p & 31);
                    atomicAnd(&P.bin_bits[(size_t)c.l * kNBW + (p >> 5)], ~m);
#pragma unroll
                    for (int k = 0; k < (int)kNBW; k++)
                        if ((p >> 5) == (uint32_t)k) w[k] &= ~m;
                }
            }
        }
    }
    TIMP(2);
}

// k_round_ps, a round whose window the previous round loaded ahead (every
// host of the wave unnoted): the due list is in s_due already -- pnd sorted
// events of the bins from the previous window's end on, of which those before
// `we` are this round's -- and the bitmap of the previous round's close (pw)
// names the window's non-empty bins.  The bins wholly consumed are reset as
// in ps_prologue; their bits go to cm, cleared from the bitmap loaded at this
// round's start once it has landed (ps_loop_close).
__device__ __forceinline__ void ps_prologue_pf(const DParams& P, HostCtx& c, bool active, uint64_t ws, uint64_t we,
                                               uint32_t pnd, uint32_t wbits, uint32_t (&cm)[kNBW]) {
    const uint64_t b0 = ws >> P.bin_shift;
    const uint32_t nbin = (uint32_t)(((we - 1) >> P.bin_shift) - b0) + 1u;
    if (active) {
        uint32_t nd = 0;
        for (; nd < pnd; nd++)
            if (s_due[nd * kBlock + threadIdx.x].time >= we) break;
        c.nd = nd;
        c.dt = nd ? s_due[threadIdx.x].time : kInf;
#pragma unroll
        for (uint32_t j = 0; j < 3; j++) {
            const uint64_t b = b0 + j;
            if (j < nbin && ((b + 1) << P.bin_shift) <= we && ((wbits >> j) & 1u)) {
                const uint32_t p = (uint32_t)b & (kNB - 1);
                __hip_atomic_store(&P.bin_n[(size_t)c.l * kNB + p], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t m = 1u << (p & 31);
                atomicAnd(&P.bin_bits[(size_t)c.l * kNBW + (p >> 5)], ~m);
#pragma unroll
                for (int k = 0; k < (int)kNBW; k++)
                    if ((p >> 5) == (uint32_t)k) cm[k] |= m;
            }
        }
    }
    TIMP(2);
}

// the next window's first kPfBins bins (from bin b on), loaded before the
// round's barrier: the slots of each non-empty one (bit set in w) in registers
struct PfBins {
    EvV x[kPfBins][kBinCap];
    uint32_t m;   // bit j: bin b + j was loaded
};
__device__ __forceinline__ void pf_issue(const PsRsrc& R, uint32_t lb, uint64_t b, const uint32_t (&w)[kNBW],
                                         bool has, PfBins& pb) {
    pb.m = 0;
    if (!has) return;
#pragma unroll
    for (uint32_t j = 0; j < kPfBins; j++) {
        const uint32_t p = (uint32_t)(b + j) & (kNB - 1);
        if (!bit_at(w, p)) continue;
        pb.m |= 1u << j;
        const uint32_t bi = lb * kNB + p;
#pragma unroll
        for (uint32_t k = 0; k < kBinCap; k++) {
            const uint32_t off = (bi * kBinCap + k) * 32u;
            pb.x[j][k] = EvV{ld16_sc1(R.bins, off), ld16_sc1(R.bins, off + 16)};
        }
    }
}
// the loaded bins' events in [lo, hi) into s_due, sorted (the round's due
// list is spent); their count, or kDueCap + 1 when they do not fit (the next
// round then reads its window as without prefetch)
__device__ __forceinline__ uint32_t pf_stage(const PfBins& pb, uint64_t lo, uint64_t hi) {
    uint32_t nw = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPfBins; j++) {
        if (((pb.m >> j) & 1u) == 0) continue;
#pragma unroll
        for (uint32_t k = 0; k < kBinCap; k++) due_add(pb.x[j][k], nw, lo, hi);
    }
    if (nw > (uint32_t)kDueCap) return (uint32_t)kDueCap + 1u;
    for (uint32_t i = 1; i < nw; i++) {
        const EvV x = ev_ld(s_due + i * kBlock + threadIdx.x);
        uint32_t k = i;
        for (; k > 0; k--) {
            const EvV y = ev_ld(s_due + (k - 1) * kBlock + threadIdx.x);
            if (!evv_less(x, y)) break;
            ev_st(s_due + k * kBlock + threadIdx.x, y);
        }
        ev_st(s_due + k * kBlock + threadIdx.x, x);
    }
    return nw;
}

// the window bins of a bitmap (bit j: bin b0 + j is non-empty); an idle
// host's next time from its own next event and its bitmap
__device__ __forceinline__ uint32_t ps_window_bits(const DParams& P, HostCtx& c, const uint32_t (&w)[kNBW],
                                                   uint64_t ws, uint64_t we) {
    const uint64_t b0 = ws >> P.bin_shift;
    const uint32_t nbin = P.bins ? (uint32_t)(((we - 1) >> P.bin_shift) - b0) + 1u : 0u;
    uint32_t wbits = 0;
    if (P.bins) {
#pragma unroll
        for (uint32_t j = 0; j < 3; j++)
            if (j < nbin) wbits |= bit_at(w, (uint32_t)(b0 + j) & (kNB - 1)) << j;
    }
    if (nbin > 3) c.err |= SHD_ERR_INTERNAL;
    return wbits;
}
__device__ __forceinline__ uint64_t ps_idle_next(const DParams& P, const uint32_t (&w)[kNBW], uint64_t t0,
                                                 uint64_t we) {
    uint64_t next = t0;
    if (P.bins) {
        const uint64_t cb = cal_lower_bound(P, w, we);
        next = cb < next ? cb : next;
    }
    return next;
}

// The round's event loop (as round_body's: per-lane state 0 needs its next
// event, 1 runs one, 2 waits for a flush, 3 done; wave-uniform exits only)
// and its close: the lane's next time (an idle lane's from its timers and
// bitmap), the last flush's stores.  cm: bits to clear from w first (bins the
// prologue reset, when w was loaded in parallel).  PF: the next window's bins
// are loaded between the loop and the close, into *pb.
template <bool PF>
__device__ __forceinline__ void ps_loop_close(const DParams& P, HostCtx& c, bool active, bool has, const PsRsrc& R,
                                              uint32_t lb, uint64_t we, uint32_t (&w)[kNBW],
                                              const uint32_t (&cm)[kNBW], uint64_t& next, PfBins* pb) {
    PendDel pd;
    pd.kind = 0;
#ifdef SHD_TIMING_LIGHT
    uint32_t n_it = 0, n_fl = 0;
    unsigned long long t_take = 0, t_work = 0, t_fl = 0, ta = 0, t_q[3] = {0, 0, 0};
#endif
    {
        uint32_t st = active ? 0u : 3u;
        for (;;) {
            for (;;) {
#ifdef SHD_TIMING_LIGHT
                n_it++;
                ta = wall_clock64();
#endif
                if (st == 0u) {
                    shd_event e;
#ifdef SHD_TIMING_LIGHT
                    const unsigned long long q0 = wall_clock64();
#endif
                    const bool got = take_next(P, c, we, e);
#ifdef SHD_TIMING_LIGHT
                    const unsigned long long q1 = wall_clock64();
                    t_q[0] += q1 - q0;
#endif
                    if (got) {
                        c.now = e.time;
                        begin_event(P, c, e);
#ifdef SHD_TIMING_LIGHT
                        t_q[1] += wall_clock64() - q1;
#endif
                        st = ((c.w_fl & ~W_READ) | c.w_msgs) ? 1u : 0u;
#ifndef SHD_NO_FUSE
#ifdef SHD_TIMING_LIGHT
                        const unsigned long long q2 = wall_clock64();
#endif
                        if (st == 0u && c.tt2 < we) {   // the notification, when it is next (round_body)
                            const uint64_t t = c.tt2, ht = c.evq_n ? c.top_time : kInf;
                            if (t < c.tt0 && t < c.tt1 && t < c.dt && t < ht && notify_fast_ok(P, c)) {
                                c.tt2 = kInf; c.now = t; c.c_events++;
                                c.q_seq = c.ts2; c.q_src = c.h; c.q_sub = 0;
                                c.w_msgs = 0; c.w_fl = 0;
                                notify_fast(P, c);
                                st = c.w_fl ? 1u : 0u;
                            }
                        }
#ifdef SHD_TIMING_LIGHT
                        t_q[2] += wall_clock64() - q2;
#endif
                        if (st == 0u && c.tt1 < we) {   // the periodic refill, when it is next
                            const uint64_t t = c.tt1, ht = c.evq_n ? c.top_time : kInf;
                            if (t < c.tt0 && t < c.tt2 && t < c.dt && t < ht && c.cq_count == 0 && c.tq_count == 0) {
                                c.tt1 = kInf; c.now = t; c.c_events++;
                                c.q_seq = c.ts1; c.q_src = c.h; c.q_sub = 0;
                                c.w_msgs = 0; c.w_fl = 0;
                                refill_fast(P, c);
                            }
                        }
#endif
                    } else {
                        st = 3u;
                    }
                }
#ifdef SHD_TIMING_LIGHT
                {
                    const unsigned long long tb = wall_clock64();
                    t_take += tb - ta;
                    ta = tb;
                }
#endif
                if (st == 1u) st = run_work(P, c) ? 0u : 2u;
#ifdef SHD_TIMING_LIGHT
                t_work += wall_clock64() - ta;
#endif
                if (__ballot(st <= 1u) == 0) break;
            }
            const bool last = __ballot(st == 2u) == 0;
#ifdef SHD_TIMING
            if (last) TIMP(3);   // the round's last flush starts
#endif
#ifdef SHD_TIMING_LIGHT
            n_fl++;
            ta = wall_clock64();
#endif
            flush_wave<true>(P, c, last, pd);
#ifdef SHD_TIMING_LIGHT
            if (!last) t_fl += wall_clock64() - ta;
#endif
            if (last) break;
            if (st == 2u) st = 1u;
        }
    }
    TIMP(4);
#ifdef SHD_TIMING_LIGHT
    TIMVP(16, (uint64_t)n_it);   // loop iterations of the wave
    TIMVP(17, (uint64_t)n_fl);   // flushes
    TIMVP(18, (uint64_t)__popcll(__ballot(active)));
    TIMVP(8, t_take);    // in take_next + begin_event (+ the fused notification / refill)
    TIMVP(9, t_work);    // in run_work
    TIMVP(10, t_fl);     // in the flushes before the last
    TIMVP(11, t_q[0]);   // of 8: take_next
    TIMVP(15, t_q[1]);   //       begin_event
    TIMVP(19, t_q[2]);   //       the fused notification (the rest: the fused refill, the loop's own)
#endif
#pragma unroll
    for (int k = 0; k < (int)kNBW; k++) w[k] &= ~cm[k];
    if (PF) pf_issue(R, lb, we >> P.bin_shift, w, has, *pb);
    if (active) {
        next = host_next(c);
        if (c.min_emit < next) next = c.min_emit;
        if (P.bins) {   // (the consumed bins were cleared in w)
            const uint64_t cb = cal_lower_bound(P, w, we);
            next = cb < next ? cb : next;
        }
    } else if (has) {
        next = ps_idle_next(P, w, host_next(c), we);
    }
    flush_finish(P, c, pd);
    TIMP(5);
}

// k_round_sp's round of an active host (ps_prologue + ps_loop_close)
template <bool SP>
__device__ __forceinline__ void ps_round_body(const DParams& P, HostCtx& c, bool active, uint32_t lb, const PsRsrc& R,
                                              uint64_t ws, uint64_t we, int parity, uint32_t nin,
                                              uint32_t (&w)[kNBW], uint32_t wbits, uint64_t& next,
                                              const SpIn* sp = nullptr) {
    ps_prologue<SP>(P, c, active, lb, R, ws, we, parity, nin, w, wbits, sp);
    uint32_t cm[kNBW];
#pragma unroll
    for (int k = 0; k < (int)kNBW; k++) cm[k] = 0;
    ps_loop_close<false>(P, c, active, active, R, lb, we, w, cm, next, nullptr);
}

// The shares' granules are stored in three planes (round 6): granule g of slot
// s at (g * nsl + s) * 16, nsl = the slots of both parities -- so a wave's poll
// of 64 blocks' first granules reads 1 KB of consecutive lines instead of 64
// sectors 48 B apart (every block polls every share every round: at the C5
// shard 489 x 489 of them); SHD_PS_AOS keeps the 48-B records for an A/B
#ifdef SHD_PS_AOS
__device__ __forceinline__ uint32_t ps_goff(uint32_t nsl, uint32_t slot, uint32_t g) { return slot * 48u + g * 16u; }
#else
__device__ __forceinline__ uint32_t ps_goff(uint32_t nsl, uint32_t slot, uint32_t g) { return (g * nsl + slot) * 16u; }
#endif
// the share of round i: its three granules tagged, stored write-through after
// the wave's hand-off stores drained; d: the noted destinations
__device__ __forceinline__ void ps_publish(__amdgpu_buffer_rsrc_t rs, uint32_t nsl, uint32_t slot, uint64_t next,
                                           uint32_t flags, uint32_t nev, uint32_t npkt, uint32_t nact, uint32_t tag,
                                           uint4 d) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every store of this wave has landed
    if (threadIdx.x == 0) {
        st16_sc1(rs, ps_goff(nsl, slot, 0), make_uint4((uint32_t)next, (uint32_t)(next >> 32), flags, tag));
        st16_sc1(rs, ps_goff(nsl, slot, 1), make_uint4(nev, npkt, nact, tag));
        st16_sc1(rs, ps_goff(nsl, slot, 2), make_uint4(d.x, d.y, d.z, tag));
    }
}
// the block's noted destinations for its share (after its last flush)
__device__ __forceinline__ uint4 ps_noted(bool pf) {
    uint4 d = make_uint4(kDirtyNone, kDirtyNone, kDirtyNone, 0);
    if (!pf) return d;
    const uint32_t n = s_dn;
    if (n > kDirtyMax) return make_uint4(kDirtyAll, kDirtyAll, kDirtyAll, 0);
    if (n > 0) d.x = s_dl[0];
    if (n > 1) d.y = s_dl[1];
    if (n > 2) d.z = s_dl[2];
    return d;
}

// every block's share of round i (slots [base, base + nblk)), K per lane per
// poll (64 K blocks a chunk, the chunks one after the other): poll until all
// carry `tag`, folding them; block 0 also folds the counts.  DIRTY: the noted
// destinations too -- bit k of `dmask`: host hb + k of this block was named,
// `dall`: some block noted more than it could name.  False on timeout
template <bool DIRTY, int K = 4>
__device__ __forceinline__ bool ps_gather(__amdgpu_buffer_rsrc_t rs, uint32_t nsl, uint32_t base, uint32_t nblk, uint32_t tag,
                                          bool counts,
                          uint64_t ticks, uint64_t& next, uint32_t& flags, uint32_t& nev, uint32_t& npkt,
                          uint32_t& nact, uint32_t hb = 0, uint32_t hpw = 0, uint64_t* dmask = nullptr,
                          bool* dall = nullptr) {
    next = kInf; flags = 0; nev = 0; npkt = 0; nact = 0;
    uint64_t dm = 0;
    uint32_t da = 0;
    const unsigned long long t0 = wall_clock64();
    for (uint32_t c0 = 0; c0 < nblk; c0 += 64u * K) {
        uint32_t need = 0;
#pragma unroll
        for (int k = 0; k < K; k++)
            if (c0 + 64u * k + threadIdx.x < nblk) need |= 1u << k;
        while (__ballot(need != 0)) {
            uint4 a[K], b[K], d[K];
#pragma unroll
            for (int k = 0; k < K; k++) {
                const uint32_t sl = base + c0 + 64u * k + threadIdx.x;
                a[k] = make_uint4(0, 0, 0, 0);
                b[k] = a[k];
                d[k] = a[k];
                if ((need >> k) & 1u) {
                    a[k] = ld16_sc1(rs, ps_goff(nsl, sl, 0));
                    if (counts) b[k] = ld16_sc1(rs, ps_goff(nsl, sl, 1));
                    if (DIRTY) d[k] = ld16_sc1(rs, ps_goff(nsl, sl, 2));
                }
            }
#pragma unroll
            for (int k = 0; k < K; k++) {
                if (!((need >> k) & 1u) || a[k].w != tag || (counts && b[k].w != tag) || (DIRTY && d[k].w != tag))
                    continue;
                const uint64_t t = ((uint64_t)a[k].y << 32) | a[k].x;
                next = t < next ? t : next;
                flags |= a[k].z;
                nev += b[k].x; npkt += b[k].y; nact += b[k].z;
                if (DIRTY) {
                    const uint32_t v[3] = {d[k].x, d[k].y, d[k].z};
#pragma unroll
                    for (int q = 0; q < 3; q++) {
                        if (v[q] == kDirtyAll) da = 1;
                        else if (v[q] - hb < hpw) dm |= 1ull << (v[q] - hb);
                    }
                }
                need &= ~(1u << k);
            }
            if (__ballot(need != 0) == 0) break;
            if (wall_clock64() - t0 > ticks) return false;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(next, off, 64);
        next = o < next ? o : next;
        flags |= __shfl_xor(flags, off, 64);
        nev += __shfl_xor(nev, off, 64);
        npkt += __shfl_xor(npkt, off, 64);
        nact += __shfl_xor(nact, off, 64);
        if (DIRTY) {
            dm |= __shfl_xor(dm, off, 64);
            da |= __shfl_xor(da, off, 64);
        }
    }
    if (DIRTY) {
        *dmask = dm;
        *dall = da != 0;
    }
    return true;
}

// a summary slot set fresh, written through (other blocks' atomics go to it)
__device__ __forceinline__ void ps_fresh(DevSummary* s) {
    uint64_t* d = (uint64_t*)s;
    static_assert(sizeof(DevSummary) % 8 == 0, "8-B words");
    const DevSummary z = fresh_summary();
    const uint64_t* q = (const uint64_t*)&z;
#pragma unroll
    for (int k = 0; k < (int)(sizeof(DevSummary) / 8); k++)
        __hip_atomic_store(d + k, q[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Cross-barrier prefetch (round 4).  A round's critical path starts with two
// dependent memory round trips per host -- the hand-off words (inbox count,
// calendar bitmap), then the window's bins -- behind the barrier.  But the
// next window's events are, but for a few, in the calendar before the round
// ends: a delivery made in round i lands at or after we_i + W, so only the
// sends with a latency below ~3 W can reach the bins [b(we_i), b(we_i) + 3)
// after the receiver has read them.  So each block loads those bins of its
// hosts between its last flush and its close (the loads overlap the flush's
// claims and the close's stores, and land before the share's drain), stages
// their events in the due list after publishing, and the next round starts
// its event loop right after the barrier.  Every append to a bin before
// pf_lim, and every inbox append, is noted by its sender (note_dirty) and
// named in the sender's share; a wave with a named host (or whose window
// reaches past the loaded bins, or whose prefetch overflowed the due list)
// reads its hand-off words after the barrier as before.  The bitmap each round
// uses for its close and for the next prefetch is loaded at its start and
// consumed after its loop; it holds every append of the rounds before (an
// append of this round is covered by its sender's own next time, min_emit).
// The persistent kernels' parameters: one copy for the whole batch (P0 =
// Pr[1]), whose fields stay in the scalar cache across rounds -- the copies
// Pr[i + 1] differ in `sum` only, and a copy per round made every round's
// first read of each field a scalar-cache miss; the round's summary is
// s_rsum.  (Timing builds keep the copy per round: the stamps' slot follows
// P.sum.  SHD_PS_PR: the same, for an A/B.)
#if defined(SHD_TIMING_P0)
#define PS_PARAMS(i)                                                                          \
    const DParams& P = P0;                                                                    \
    if (threadIdx.x == 0) {                                                                   \
        s_rsum = &ring[(i) + 1];                                                              \
        s_tslot = (uint32_t)(((uintptr_t)&ring[(i) + 1] / sizeof(DevSummary)) & 63);          \
    }
#elif defined(SHD_TIMING) || defined(SHD_PS_PR)
#define PS_PARAMS(i)                                    \
    const DParams& P = Pr[(i) + 1];                     \
    if (threadIdx.x == 0) s_rsum = &ring[(i) + 1]
#else
#define PS_PARAMS(i)                                    \
    const DParams& P = P0;                              \
    if (threadIdx.x == 0) s_rsum = &ring[(i) + 1]
#endif


#ifndef SHD_NO_PF
constexpr bool kPsPf = true;
#else
constexpr bool kPsPf = false;
#endif

template <bool LEAN>
__global__ __launch_bounds__(kBlock) void k_round_ps(uint64_t window, int nb, DevSummary* __restrict__ ring,
                                                      const DevCtl* __restrict__ ctl, PsShare* __restrict__ shares,
                                                      const DParams* __restrict__ Pr, uint64_t ticks) {
    const DParams& P0 = Pr[1];
    const uint32_t nblk = (uint32_t)((P0.nloc + P0.hpw - 1) / P0.hpw);
    const int32_t l = lane_host(P0);
    const bool has = l < P0.nloc;
    const uint32_t lb = threadIdx.x;
    const uint32_t hb = blockIdx.x * (uint32_t)P0.hpw;   // the block's first host
    PsRsrc R0, R1;   // parity 0 and 1
    {
        const uint32_t hpw = (uint32_t)P0.hpw;
        R0.bits = buf_rsrc(P0.bin_bits ? P0.bin_bits + (size_t)hb * kNBW : nullptr, (uint64_t)hpw * kNBW * 4);
        R0.bins = buf_rsrc(P0.bins ? P0.bins + (size_t)hb * kNB * kBinCap : nullptr,
                           (uint64_t)hpw * kNB * kBinCap * sizeof(shd_event));
        R1.bits = R0.bits;
        R1.bins = R0.bins;
        R0.nin = buf_rsrc(P0.inbox_n[0] + hb, (uint64_t)hpw * 4);
        R1.nin = buf_rsrc(P0.inbox_n[1] + hb, (uint64_t)hpw * 4);
        R0.inbox = buf_rsrc(P0.inbox[0] + (size_t)hb * P0.inbox_cap, (uint64_t)hpw * P0.inbox_cap * sizeof(shd_event));
        R1.inbox = buf_rsrc(P0.inbox[1] + (size_t)hb * P0.inbox_cap, (uint64_t)hpw * P0.inbox_cap * sizeof(shd_event));
    }
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(shares, (uint64_t)2 * nblk * sizeof(PsShare));
    HostCtx c;
    hot_load(P0, c);
    if (LEAN) { c.k.feat = 0; c.k.boot_end = 0; }
    if (has) {
        load_ctx(P0, c, l, P0.hs[l], P0.host_att[P0.h0 + l], P0.self_thr[P0.h0 + l]);
    } else {
        c.l = P0.nloc; c.h = 0; c.att = 0; c.cls = 0; c.evq_n = 0; c.top_time = kInf; c.peer = -1; c.rq_head = 0;
        c.tt0 = c.tt1 = c.tt2 = kInf; c.ev_seq = 0; c.cq_hv = false; c.tq_hv = false; c.pf_lim = 0;
    }
    uint32_t acc[6] = {0, 0, 0, 0, 0, 0};
    uint64_t ws = ring[0].next_time;
    const uint64_t stop = ctl->stop, rbase = ctl->round_base;
    const uint32_t tag0 = (uint32_t)ctl->xtag;
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    // the prefetch carried from a round to the next (wave-uniform but pnd,
    // dirty): valid, its first bin, the due events staged (kDueCap + 1:
    // overflow), the bitmap of that round's close, named by a share
    const bool pfm = kPsPf && P0.bins != nullptr;
    bool pf = false;
    uint64_t pf_b0 = 0;
    uint32_t pnd = 0, dirty = 0;
    uint32_t pw[kNBW];
#pragma unroll
    for (int k = 0; k < (int)kNBW; k++) pw[k] = 0;
    for (int i = 0; i < nb; i++) {
        PS_PARAMS(i);
        const unsigned long long t_start = wall_clock64();
#ifdef SHD_TIMING
        if (threadIdx.x == 0 && blockIdx.x < 2048) g_tim[PS_TIM_SLOT()][blockIdx.x][0] = t_start;
#endif
        if (lead) ps_fresh(&ring[i + 2]);   // the next round's summary (this round's: ring[i + 1])
        const int parity = (int)((rbase + (uint64_t)i) & 1);
        uint64_t we = ws + window;
        if (we > stop || we < ws) we = stop;
        PsRsrc R = R0;
        R.nin = parity ? R1.nin : R0.nin;
        R.inbox = parity ? R1.inbox : R0.inbox;
        const bool fast = pf && ((we - 1) >> P.bin_shift) <= pf_b0 + (kPfBins - 1) &&
                          __ballot(has && (dirty != 0 || pnd > (uint32_t)kDueCap)) == 0;
        ps_round_reset(P, c, ws, we, parity, pfm);
        uint32_t w[kNBW], cm[kNBW];
#pragma unroll
        for (int k = 0; k < (int)kNBW; k++) { w[k] = 0; cm[k] = 0; }
        bool active = false;
        if (fast) {
            // the bitmap for the close and the next prefetch goes out now and is
            // consumed after the loop; the window's events are staged already
            if (has) {
                const uint4 x = ld16_sc1(R.bits, lb * 32u), y = ld16_sc1(R.bits, lb * 32u + 16u);
                w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w; w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
            }
            const uint32_t wbits = ps_window_bits(P, c, pw, ws, we);
            TIMP(1);
            active = has && !(host_next(c) >= we && wbits == 0);   // (no inbox: it would have been named)
            ps_prologue_pf(P, c, active, ws, we, pnd, wbits, cm);
        } else {
            // the round's hand-off words: this parity's inbox count, the calendar bitmap
            uint32_t nin = 0;
            if (has) {
                nin = ld4_sc1(R.nin, lb * 4u);
                if (P.bins) {
                    const uint4 x = ld16_sc1(R.bits, lb * 32u), y = ld16_sc1(R.bits, lb * 32u + 16u);
                    w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w; w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
                }
            }
            const uint32_t wbits = ps_window_bits(P, c, w, ws, we);
            TIMP(1);
            active = has && !(nin == 0 && host_next(c) >= we && wbits == 0);
            ps_prologue<false>(P, c, active, lb, R, ws, we, parity, nin, w, wbits);
        }
        uint64_t next = kInf;
        PfBins pb;
        ps_loop_close<kPsPf>(P, c, active, has, R, lb, we, w, cm, next, &pb);
        acc[0] += c.c_events; acc[1] += c.c_pkt; acc[2] += c.c_sent;
        acc[3] += c.c_idrop; acc[4] += c.c_cdrop; acc[5] += c.c_recv;
        uint32_t nev = c.c_events, npkt = c.c_pkt, err = c.err;
        const uint32_t pend = c.n_pend ? kPsPend : 0u;
        const uint32_t nact = (uint32_t)__popcll(__ballot(nev != 0));
        uint32_t fl = err | pend;
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t o = __shfl_xor(next, off, 64);
            next = o < next ? o : next;
            nev += __shfl_xor(nev, off, 64);
            npkt += __shfl_xor(npkt, off, 64);
            fl |= __shfl_xor(fl, off, 64);
        }
        const uint32_t tag = tag0 + (uint32_t)i;
        const uint32_t base = (uint32_t)(i & 1) * nblk;
        ps_publish(rs, 2 * nblk, base + blockIdx.x, next, fl, nev, npkt, nact, tag, ps_noted(pfm));
        TIMP(6);
        if (pfm) {   // the next window's events, staged while the other blocks finish
            const uint64_t b1 = we >> P.bin_shift;
            pnd = pf_stage(pb, we, (b1 + kPfBins) << P.bin_shift);
            pf_b0 = b1;
#pragma unroll
            for (int k = 0; k < (int)kNBW; k++) pw[k] = w[k];
        }
        uint64_t f_next, dm = 0;
        uint32_t f_fl, f_nev, f_npkt, f_nact;
        bool dall = false;
        const bool ok_v = ps_gather<kPsPf>(rs, 2 * nblk, base, nblk, tag, blockIdx.x == 0, ticks, f_next, f_fl, f_nev, f_npkt,
                                           f_nact, hb, (uint32_t)P.hpw, &dm, &dall);
        TIMP(7);
        // the folds are wave-uniform: said so to the compiler, so that the
        // round loop and the parity branch stay scalar (with a vector exit
        // condition the host context would be merged through divergent flow)
        const bool ok = __builtin_amdgcn_readfirstlane((int)ok_v) != 0;
        f_fl = __builtin_amdgcn_readfirstlane(f_fl);
        f_next = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(f_next >> 32)) << 32) |
                 (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)f_next);
        if (!ok) {   // a block never came: the launch is not resident (or a block faulted)
            if (threadIdx.x == 0) {
                atomicOr(&ring[i + 1].error, SHD_ERR_INTERNAL);
                *P.halt = 1u;
            }
            break;
        }
        if (lead) {   // round i's summary (its log count came by atomics during the round)
            DevSummary* s = &ring[i + 1];
            atomicMin(&s->next_time, f_next);
            if (f_nev) atomicAdd(&s->n_events, (unsigned long long)f_nev);
            if (f_npkt) atomicAdd(&s->n_pkt_events, (unsigned long long)f_npkt);
            if (f_nact) atomicAdd(&s->n_active, f_nact);
            if (f_fl & ~kPsPend) atomicOr(&s->error, f_fl & ~kPsPend);
            atomicMin(&s->t_first, t_start);
            atomicMax(&s->t_last, (unsigned long long)wall_clock64());
            __hip_atomic_store(&s->ws, (unsigned long long)ws, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (f_fl & kPsPend) *P.halt = 1u;
        }
        if (f_fl) break;            // a first touch to resolve, or an error: the host takes over
        ws = f_next;
        if (ws >= stop) break;      // the rest only forwards the time (ring[i + 1].next_time says so)
        pf = pfm;
        dirty = (dall || ((dm >> lb) & 1ull)) ? 1u : 0u;
    }
    // the hosts' state, once for the whole batch
    if (has) {
        c.c_events = acc[0]; c.c_pkt = acc[1]; c.c_sent = acc[2];
        c.c_idrop = acc[3]; c.c_cdrop = acc[4]; c.c_recv = acc[5];
        store_ctx(P0, c);
    }
}

// ------------------------------------------------------ sparse persistent rounds
// k_round_sp: k_round_ps for engines whose hosts outnumber what one resident
// wave per 64 hosts can hold (the per-GPU shard of the north-star model:
// 125 k hosts = 1954 waves of ~256 VGPRs and 40 KB of LDS, against 1024 such
// waves resident; k_round_tl then runs every round in two passes of blocks).
// Here a block owns `sph` hosts (a multiple of 64; one block per CU) and, per
// round, scans their hand-off words and own next times (hnext), compacts the
// hosts with something due into a list in LDS, and runs them 64 at a time:
// each pass loads its hosts' records (load_ctx), runs ps_round_body, and
// stores them (store_ctx, with hnext).  In the models this is for, a few
// percent of the hosts have an event in a given window, so a round is one
// pass of a few active lanes per block instead of every host's lane.  The
// hosts' records, heaps and queues are read and written by their own block
// only (plain accesses, one CU); the hand-off arrays by sc1 loads, as in
// k_round_ps, whose share protocol and ring summaries this kernel shares.
constexpr uint32_t kSpMaxHosts = 4096;   // hosts per block at most (64 groups of 64)
// groups of 64 hosts whose hand-off words one scan batch loads together (one
// memory round trip each batch; 8: the 125 k-host shard's ~490 hosts per block
// in one)
#ifndef SHD_SP_SCAN
#define SHD_SP_SCAN 8
#endif
constexpr int kSpScan = SHD_SP_SCAN;
// shares per lane per poll of the sparse round's barrier: 4 (chunks of 256
// blocks, one after the other) measured faster than 8 at the C5 shard's 489
// blocks, 76.7 against 75.6 M (round 6, profiles/r06/sp3)
#ifndef SHD_SP_GATHER_K
#define SHD_SP_GATHER_K 4
#endif
constexpr int kSpGatherK = SHD_SP_GATHER_K;
__shared__ uint16_t s_act[kSpMaxHosts];  // the round's active hosts (index in the block)
__shared__ uint32_t s_aw[(kNBW + 1) * kBlock];   // the first pass's hand-off words: bitmap, inbox count

// k_round_sp / k_round_spx: the round's scan of a block's hosts [hb, hb + nh)
// (ngrp groups of 64): the hosts with something due in [ws, we) go to s_act
// (their words to s_aw for the first pass), nact counts them; next: the least
// next time of the lane's idle hosts
// (alist: the list's LDS array; lhn: the block's hosts' next times in LDS, or
// null: the global hnext)
__device__ __forceinline__ void sp_scan(const DParams& P, const PsRsrc& R, uint32_t hb, uint32_t nh, uint32_t ngrp,
                                        uint64_t ws, uint64_t we, uint64_t& next, uint32_t& nact, uint16_t* alist,
                                        const uint64_t* lhn) {
    const uint32_t lane = threadIdx.x;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    next = kInf;
    nact = 0;
    // the scan: every host's words and own next time, kSpScan groups per
    // round trip.  The window's bins sit at the same ring positions for
    // every host (b0 is the round's), so each host's window bits are two
    // words picked by a uniform index and one shift; and an idle host's
    // calendar bound is not worked out per host: the first non-empty bin
    // from we's on, in ring order, of the OR of the idle hosts' bitmaps is
    // the least of theirs (bits_first_from is a min over set bits), so the
    // block ORs them and takes one bound for the lot (round 6: the per-host
    // bound was 3/4 of the scan, ~3.5 us a round at the C5 shard); each
    // lane ORs its own groups' idle hosts, and the fold of the lanes' next
    // times takes the least
    uint32_t orw[kNBW];
#pragma unroll
    for (int j = 0; j < (int)kNBW; j++) orw[j] = 0;
    const uint32_t p0 = (uint32_t)(ws >> P.bin_shift) & (kNB - 1);
    const uint32_t nbin = P.bins ? (uint32_t)(((we - 1) >> P.bin_shift) - (ws >> P.bin_shift)) + 1u : 0u;
    const uint32_t wi0 = p0 >> 5, wi1 = (wi0 + 1u) & (kNBW - 1), wsh = p0 & 31u;
    const uint32_t wmask = nbin >= 3 ? 7u : (1u << nbin) - 1u;
    for (uint32_t g0 = 0; g0 < ngrp; g0 += kSpScan) {
        uint32_t nin4[kSpScan], w4[kSpScan][kNBW];
        uint64_t t4[kSpScan];
#pragma unroll
        for (int q = 0; q < kSpScan; q++) {
            const uint32_t lb = (g0 + q) * 64u + lane;
            nin4[q] = 0; t4[q] = kInf;
#pragma unroll
            for (int j = 0; j < (int)kNBW; j++) w4[q][j] = 0;
            if (g0 + q < ngrp && lb < nh) {
                nin4[q] = ld4_sc1(R.nin, lb * 4u);
                if (P.bins) {
                    const uint4 x = ld16_sc1(R.bits, lb * 32u), y = ld16_sc1(R.bits, lb * 32u + 16u);
                    w4[q][0] = x.x; w4[q][1] = x.y; w4[q][2] = x.z; w4[q][3] = x.w;
                    w4[q][4] = y.x; w4[q][5] = y.y; w4[q][6] = y.z; w4[q][7] = y.w;
                }
                t4[q] = lhn ? lhn[lb] : P.hnext[hb + lb];
            }
        }
#ifdef SHD_TIMING
        if (g0 == 0) {   // the first scan batch's words have landed
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            TIMVP(22, wall_clock64());
        }
#endif
#pragma unroll
        for (int q = 0; q < kSpScan; q++) {
            if (g0 + q >= ngrp) break;   // (uniform)
            const uint32_t lb = (g0 + q) * 64u + lane;
            const bool has = lb < nh;
            uint32_t lo = w4[q][0], hi = w4[q][1];
#pragma unroll
            for (int j = 1; j < (int)kNBW; j++) {   // uniform picks: v_cndmask on a scalar condition
                lo = wi0 == (uint32_t)j ? w4[q][j] : lo;
                hi = wi1 == (uint32_t)j ? w4[q][j] : hi;
            }
            hi = wi1 == 0u ? w4[q][0] : hi;
            const uint32_t wbits = (uint32_t)(((((uint64_t)hi) << 32) | lo) >> wsh) & wmask;
            const bool act = has && !(nin4[q] == 0 && t4[q] >= we && wbits == 0);
            if (has && !act) {
                next = t4[q] < next ? t4[q] : next;
#pragma unroll
                for (int j = 0; j < (int)kNBW; j++) orw[j] |= w4[q][j];
            }
            const uint64_t m = __ballot(act);
            if (act) {
                const uint32_t k = nact + (uint32_t)__popcll(m & lt_mask);
                alist[k] = (uint16_t)lb;
                if (k < (uint32_t)kBlock) {
#pragma unroll
                    for (int j = 0; j < (int)kNBW; j++) s_aw[j * kBlock + k] = w4[q][j];
                    s_aw[kNBW * kBlock + k] = nin4[q];
                }
            }
            nact += (uint32_t)__popcll(m);
        }
    }
    if (P.bins) {   // the lane's idle hosts' calendar bound: one, from their bitmaps' OR (the
                    // block's min over the lanes comes with the round's fold below)
        const uint64_t cb = cal_lower_bound(P, orw, we);
        next = cb < next ? cb : next;
    }
#ifdef SHD_TIMING
    TIMVP(23, wall_clock64());   // the compaction done (before the barrier)
#endif
}

// k_round_sp / k_round_spx: the scan's active hosts, 64 at a time: each pass
// loads its hosts' records (with the bins' loads, ps_round_body<true>), runs
// their round and stores them; next / nev / npkt / fl / nhost accumulate the
// lane's share (PEND: a logged first touch flags kPsPend)
// (alist: the scan's list; lrec / lhn: the block's hosts' records and next
// times in LDS, or null: the global ones)
template <bool PEND>
__device__ __forceinline__ void sp_passes(const DParams& P, HostCtx& c, const PsRsrc& R, uint32_t hb, uint32_t nact,
                                          uint64_t ws, uint64_t we, int parity, uint32_t xwi, uint64_t& next,
                                          uint32_t& nev, uint32_t& npkt, uint32_t& fl, uint32_t& nhost,
                                          const uint16_t* alist, HostRec* lrec, uint64_t* lhn) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t base = 0; base < nact; base += kBlock) {
        const uint32_t k = base + lane;
        const bool act = k < nact;
        const uint32_t lb = act ? (uint32_t)alist[k] : 0u;
        const int32_t l = (int32_t)(hb + lb);
        uint32_t nin = 0, w[kNBW];
#pragma unroll
        for (int j = 0; j < (int)kNBW; j++) w[j] = 0;
        if (act) {
            if (base == 0) {
#pragma unroll
                for (int j = 0; j < (int)kNBW; j++) w[j] = s_aw[j * kBlock + k];
                nin = s_aw[kNBW * kBlock + k];
            } else {   // later passes (more than 64 active hosts): the words again
                nin = ld4_sc1(R.nin, lb * 4u);
                if (P.bins) {
                    const uint4 x = ld16_sc1(R.bits, lb * 32u), y = ld16_sc1(R.bits, lb * 32u + 16u);
                    w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w; w[4] = y.x; w[5] = y.y; w[6] = y.z; w[7] = y.w;
                }
            }
        }
        SpIn in;   // the record's loads go out with the bins' (ps_round_body<true>)
        in.l = l;
        in.xwi = xwi;
        if (act) {
            in.rec = lrec ? lrec[lb] : P.hs[l];
            in.att = P.host_att[P.h0 + l];
            in.st = P.self_thr[P.h0 + l];
        }
        const uint32_t wbits = ps_window_bits(P, c, w, ws, we);
        uint64_t hn = kInf;
        ps_round_body<true>(P, c, act, lb, R, ws, we, parity, nin, w, wbits, hn, &in);
        if (act) {
            if (lrec) store_ctx(P, c, &lrec[lb], &lhn[lb]);
            else store_ctx(P, c);
        }
        next = hn < next ? hn : next;
        nev += c.c_events; npkt += c.c_pkt;
        fl |= c.err | (PEND && c.n_pend ? kPsPend : 0u);
        nhost += (uint32_t)__popcll(__ballot(act && c.c_events != 0));
        __syncthreads();   // (the next pass reuses the lanes' LDS slots)
    }
}

// k_round_sp's dynamic LDS: the scan's list (sph 2-B entries), then, with lrec
// (round 6: where two blocks per CU still fit), the block's hosts' records and
// next times for the whole batch -- loaded at its start, stored at its end, so
// a pass neither loads a record from HBM nor stores one before the share's drain
extern __shared__ __align__(16) char s_spdyn[];
__host__ __device__ constexpr size_t sp_dyn_bytes(uint32_t sph, bool lrec) {
    return (((size_t)2 * sph + 127) & ~(size_t)127) + (lrec ? (size_t)sph * (sizeof(HostRec) + 8) : 0);
}
template <bool LEAN>
__global__ __launch_bounds__(kBlock) void k_round_sp(uint64_t window, int nb, DevSummary* __restrict__ ring,
                                                      const DevCtl* __restrict__ ctl, PsShare* __restrict__ shares,
                                                      const DParams* __restrict__ Pr, uint64_t ticks, uint32_t sph,
                                                      int lrec_on) {
    const DParams& P0 = Pr[1];
    const uint32_t nblk = gridDim.x;
    const uint32_t lane = threadIdx.x;
    const uint32_t hb = blockIdx.x * sph;   // the block's first host
    const uint32_t nh = (uint32_t)P0.nloc - hb < sph ? (uint32_t)P0.nloc - hb : sph;
    const uint32_t ngrp = (nh + 63u) >> 6;
    PsRsrc R0, R1;   // parity 0 and 1, over the block's hosts
    {
        R0.bits = buf_rsrc(P0.bin_bits ? P0.bin_bits + (size_t)hb * kNBW : nullptr, (uint64_t)nh * kNBW * 4);
        R0.bins = buf_rsrc(P0.bins ? P0.bins + (size_t)hb * kNB * kBinCap : nullptr,
                           (uint64_t)nh * kNB * kBinCap * sizeof(shd_event));
        R1.bits = R0.bits;
        R1.bins = R0.bins;
        R0.nin = buf_rsrc(P0.inbox_n[0] + hb, (uint64_t)nh * 4);
        R1.nin = buf_rsrc(P0.inbox_n[1] + hb, (uint64_t)nh * 4);
        R0.inbox = buf_rsrc(P0.inbox[0] + (size_t)hb * P0.inbox_cap, (uint64_t)nh * P0.inbox_cap * sizeof(shd_event));
        R1.inbox = buf_rsrc(P0.inbox[1] + (size_t)hb * P0.inbox_cap, (uint64_t)nh * P0.inbox_cap * sizeof(shd_event));
    }
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(shares, (uint64_t)2 * nblk * sizeof(PsShare));
    HostCtx c;
    hot_load(P0, c);
    if (LEAN) { c.k.feat = 0; c.k.boot_end = 0; }
    c.l = P0.nloc; c.h = 0; c.att = 0; c.cls = 0; c.evq_n = 0; c.top_time = kInf; c.peer = -1; c.rq_head = 0;
    c.tt0 = c.tt1 = c.tt2 = kInf; c.ev_seq = 0; c.cq_hv = false; c.tq_hv = false;
    uint64_t ws = ring[0].next_time;
    const uint64_t stop = ctl->stop, rbase = ctl->round_base;
    const uint32_t tag0 = (uint32_t)ctl->xtag;
    const bool lead = blockIdx.x == 0 && lane == 0;
    uint16_t* alist = (uint16_t*)s_spdyn;
    HostRec* lrec = lrec_on ? (HostRec*)(s_spdyn + sp_dyn_bytes(sph, false)) : nullptr;
    uint64_t* lhn = lrec_on ? (uint64_t*)(lrec + sph) : nullptr;
    if (lrec) {   // the block's hosts' records and next times, for the batch
        for (uint32_t j = lane; j < nh; j += kBlock) {
            lrec[j] = P0.hs[hb + j];
            lhn[j] = P0.hnext[hb + j];
        }
        __syncthreads();
    }
    for (int i = 0; i < nb; i++) {
        PS_PARAMS(i);
        const unsigned long long t_start = wall_clock64();
#ifdef SHD_TIMING
        if (lane == 0 && blockIdx.x < 2048) g_tim[PS_TIM_SLOT()][blockIdx.x][0] = t_start;
#endif
        if (lead) ps_fresh(&ring[i + 2]);
        const int parity = (int)((rbase + (uint64_t)i) & 1);
        uint64_t we = ws + window;
        if (we > stop || we < ws) we = stop;
        PsRsrc R = R0;
        R.nin = parity ? R1.nin : R0.nin;
        R.inbox = parity ? R1.inbox : R0.inbox;
        ps_round_reset(P, c, ws, we, parity, false);
        uint64_t next;
        uint32_t nact;
        sp_scan(P, R, hb, nh, ngrp, ws, we, next, nact, alist, lhn);
        __syncthreads();
        TIMP(1);
        TIMVP(20, (uint64_t)nact);   // the block's active hosts this round
        TIMVP(21, (uint64_t)((nact + kBlock - 1) / kBlock));   // passes
        // the active hosts, 64 at a time
        uint32_t nev = 0, npkt = 0, fl = 0, nhost = 0;
        sp_passes<true>(P, c, R, hb, nact, ws, we, parity, 0u, next, nev, npkt, fl, nhost, alist, lrec, lhn);
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t o = __shfl_xor(next, off, 64);
            next = o < next ? o : next;
            nev += __shfl_xor(nev, off, 64);
            npkt += __shfl_xor(npkt, off, 64);
            fl |= __shfl_xor(fl, off, 64);
        }
        const uint32_t tag = tag0 + (uint32_t)i;
        const uint32_t sbase = (uint32_t)(i & 1) * nblk;
        ps_publish(rs, 2 * nblk, sbase + blockIdx.x, next, fl, nev, npkt, nhost, tag, ps_noted(false));
        TIMP(6);
        uint64_t f_next;
        uint32_t f_fl, f_nev, f_npkt, f_nact;
        const bool ok_v = ps_gather<false, kSpGatherK>(rs, 2 * nblk, sbase, nblk, tag, blockIdx.x == 0, ticks, f_next, f_fl,
                                                       f_nev, f_npkt, f_nact);
        TIMP(7);
        const bool ok = __builtin_amdgcn_readfirstlane((int)ok_v) != 0;
        f_fl = __builtin_amdgcn_readfirstlane(f_fl);
        f_next = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(f_next >> 32)) << 32) |
                 (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)f_next);
        if (!ok) {
            if (lane == 0) {
                atomicOr(&ring[i + 1].error, SHD_ERR_INTERNAL);
                *P.halt = 1u;
            }
            break;
        }
        if (lead) {
            DevSummary* sm = &ring[i + 1];
            atomicMin(&sm->next_time, f_next);
            if (f_nev) atomicAdd(&sm->n_events, (unsigned long long)f_nev);
            if (f_npkt) atomicAdd(&sm->n_pkt_events, (unsigned long long)f_npkt);
            if (f_nact) atomicAdd(&sm->n_active, f_nact);
            if (f_fl & ~kPsPend) atomicOr(&sm->error, f_fl & ~kPsPend);
            atomicMin(&sm->t_first, t_start);
            atomicMax(&sm->t_last, (unsigned long long)wall_clock64());
            __hip_atomic_store(&sm->ws, (unsigned long long)ws, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (f_fl & kPsPend) *P.halt = 1u;
        }
        if (f_fl) break;
        ws = f_next;
        if (ws >= stop) break;
    }
    if (lrec) {   // the records and next times back, once for the batch
        __syncthreads();
        for (uint32_t j = lane; j < nh; j += kBlock) {
            P0.hs[hb + j] = lrec[j];
            P0.hnext[hb + j] = lhn[j];
        }
    }
}

// ingest events from other engines into inbox[parity]
__global__ void k_ingest(DParams P, const shd_event* __restrict__ ev, uint64_t n, int parity) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const shd_event e = ev[i];
    const int32_t dl = (int32_t)e.dst - P.h0;
    if (dl < 0 || dl >= P.nloc) { atomicOr(&P.sum->error, SHD_ERR_REMOTE_OVERFLOW); return; }
    uint32_t slot = atomicAdd(&P.inbox_n[parity][dl], 1u);
    if (slot >= P.inbox_cap) { atomicOr(&P.sum->error, SHD_ERR_INBOX_OVERFLOW); return; }
    P.inbox[parity][(size_t)dl * P.inbox_cap + slot] = e;
}

// caller-pushed self events (shd_eng_push_events): one thread per host with
// pushed events, in array order.  event_new_ consumes the host's next event ID
// (event.c:38); scheduler_push drops a time >= end (scheduler.c:346-349); the
// rest go to the inbox the next round merges into the host's heap
__global__ void k_push(DParams P, const shd_event* __restrict__ ev, const uint32_t* __restrict__ grp_off,
                       uint32_t ngrp, int parity) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ngrp) return;
    const uint32_t b = grp_off[g], en = grp_off[g + 1];
    const int32_t dl = (int32_t)ev[b].dst - P.h0;
    const uint64_t seq0 = P.hs[dl].ev_seq;
    uint64_t seq = seq0;
    uint64_t next = kInf;
    uint32_t err = 0;
    for (uint32_t i = b; i < en; i++) {
        shd_event e = ev[i];
        e.seq = seq++;
        if (e.time >= P.end_time) continue;
        const uint32_t slot = atomicAdd(&P.inbox_n[parity][dl], 1u);
        if (slot >= P.inbox_cap) { err |= SHD_ERR_INBOX_OVERFLOW; continue; }
        P.inbox[parity][(size_t)dl * P.inbox_cap + slot] = e;
        next = e.time < next ? e.time : next;
    }
    // the record keeps a live timer's ID as its distance back from ev_seq
    // (store_ctx): the IDs consumed here move ev_seq, not the timers' IDs
    HostRec& r = P.hs[dl];
    for (int k = 0; k < 3; k++) {
        if (r.tt[k] == kInf) continue;
        const uint64_t back = (uint64_t)r.ts_back[k] + (seq - seq0);
        if (back >> 32) err |= SHD_ERR_INTERNAL;
        r.ts_back[k] = (uint32_t)back;
    }
    r.ev_seq = seq;
    if (next != kInf) atomicMin(&P.sum->next_time, (unsigned long long)next);
    if (err) atomicOr(&P.sum->error, err);
}

// packets from hosts outside this engine (shd_eng_push_events: the delivery
// events a CPU-side host's worker_sendPacket made, worker.c:260-321): the
// sender's event ID and packet id come with them; scheduler_push drops a time
// >= end (scheduler.c:346-349); the rest go to the inbox the next round
// merges into the destination's heap.  One thread per event.
__global__ void k_push_packets(DParams P, const shd_event* __restrict__ ev, uint32_t n, int parity) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const shd_event e = ev[i];
    if (e.time >= P.end_time) return;
    const int32_t dl = (int32_t)e.dst - P.h0;
    const uint32_t slot = atomicAdd(&P.inbox_n[parity][dl], 1u);
    if (slot >= P.inbox_cap) { atomicOr(&P.sum->error, SHD_ERR_INBOX_OVERFLOW); return; }
    P.inbox[parity][(size_t)dl * P.inbox_cap + slot] = e;
    atomicMin(&P.sum->next_time, (unsigned long long)e.time);
}
