// eng_exchange.h -- the engine group's exchange kernels: the all-to-all
// transport (k_round_xtl, k_xfold, k_ingest_x), the peer-to-peer transport
// (k_xput, k_xwait_ingest, k_xchg) and the fused peer-to-peer rounds
// (k_round_px, k_xchg_px).
// Part of libshdgpu's engine translation unit (csrc/engine.hip includes it
// inside its anonymous namespace); not a standalone header.
#pragma once

// ---- exchange mode kernels (shd_xgroup) ----
// local transport: block d of sender s -> block s of receiver d, header plus
// the counted events only; grid (slots, receiver, sender)
struct XPtrs {
    const shd_event* send[64];
    shd_event* recv[64];
};
__global__ void k_xcopy_local(XPtrs X, uint64_t stride) {
    const int s = blockIdx.z, d = blockIdx.y;
    const shd_event* src = X.send[s] + (size_t)d * stride;
    shd_event* dst = X.recv[d] + (size_t)s * stride;
    const uint32_t n = ((const XHeader*)src)->count;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// headers of this engine's blocks, one lane per peer: the engine's next event
// time and the round's flags; `clean` after a host recovery (the recovered
// round's flags are not repeated).  Resets the per-peer counters.
__device__ void xpack_block(const DParams& P, const DevSummary* sum, int clean, uint64_t next_time) {
    const int32_t p = threadIdx.x;
    if (p >= P.xworld) return;
    const uint32_t cnt = P.xcount[p];
    XHeader h;
    h.next_time = next_time;
    h.count = cnt < P.xcap ? cnt : P.xcap;
    uint32_t fl = 0;
    if (!clean) {
        if (sum->n_pending) fl |= XF_PENDING;
        if (sum->n_remote) fl |= XF_OVERFLOW;
        if (sum->error) fl |= XF_ERROR;
    }
    h.flags = fl;
    h.n_pending = clean ? 0 : sum->n_pending;
    h.error = sum->error;
    h.tag = 0;
    *(XHeader*)(P.xsend + (size_t)p * (P.xcap + 1)) = h;
    P.xcount[p] = 0;
}

__global__ void k_xpack(DParams P, const DevSummary* __restrict__ sum, int clean) {
    if (*P.halt) return;
    xpack_block(P, sum, clean, sum->next_time);
}

// The same round without the completion ticket: every block writes its share
// of the summary and ends; k_xfold (one wave, launched next on the stream)
// folds the shares and packs this engine's headers for the exchange.
__global__ __launch_bounds__(kBlock) void k_round_xtl(DRoundArgs a, const DParams* __restrict__ Pp,
                                                      const shd_event* __restrict__ xrecv,
                                                      XHeader* __restrict__ halt_hdr, DevSummary* __restrict__ init,
                                                      const DevCtl* __restrict__ ctl, int i, uint64_t window,
                                                      TlPart* __restrict__ parts) {
    const DParams& P = *Pp;
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    const unsigned long long t_entry = wall_clock64();
    const int32_t xworld = P.xworld;
    const size_t stride = (size_t)P.xcap + 1;
    // as k_round_tl: the window start's loads first (halt, control words,
    // every peer's header: lane p loads header p), the host state behind them
    uint32_t halt = *a.halt;
    uint64_t stop = ctl->stop, rbase = ctl->round_base;
    const XHeader hx = *(const XHeader*)(xrecv + (size_t)((int32_t)threadIdx.x < xworld ? threadIdx.x : 0) * stride);
    uint64_t ws = (int32_t)threadIdx.x < xworld ? hx.next_time : kInf;
    uint32_t fl = (int32_t)threadIdx.x < xworld ? hx.flags : 0u;
    HostIn in;
    host_in_load(a, in);
    asm volatile("" : "+v"(halt), "+v"(stop), "+v"(rbase), "+v"(ws), "+v"(fl));
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(ws, off, 64);
        ws = o < ws ? o : ws;
        fl |= __shfl_xor(fl, off, 64);
    }
    if (halt) {
        if (lead) P.sum->flags = 2u;
        return;
    }
    const int parity = (int)((rbase + (uint64_t)i) & 1);
    if (fl) {
        if (blockIdx.x == 0) {
            if ((int32_t)threadIdx.x < P.xworld) halt_hdr[threadIdx.x] = *(const XHeader*)(xrecv + threadIdx.x * stride);
            if (threadIdx.x == 0) {
                *P.halt = 1u;
                P.sum->flags = 1u;
            }
        }
        return;
    }
    if (lead) {
        atomicMin(&P.sum->t_first, t_entry);
        *init = fresh_summary();
        P.sum->ws = ws;
    }
    if (ws >= stop) return;   // only forwards the time (k_xfold packs it)
    uint64_t we = ws + window;
    if (we > stop || we < ws) we = stop;
    uint64_t next, nev, npkt;
    uint32_t err;
    round_body(P, in, ws, we, parity, next, nev, npkt, err, (uint32_t)((ctl->xpar + (uint64_t)i) & 1));
    const uint32_t nact = (uint32_t)__popcll(__ballot(nev != 0));   // hosts that executed an event
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(next, off, 64);
        next = o < next ? o : next;
        nev += __shfl_xor(nev, off, 64);
        npkt += __shfl_xor(npkt, off, 64);
        err |= __shfl_xor(err, off, 64);
    }
    if (threadIdx.x == 0)
        parts[(size_t)(i & 1) * gridDim.x + blockIdx.x] =
            TlPart{next, (unsigned long long)wall_clock64(), (unsigned)nev, (unsigned)npkt, err, nact};
}

__global__ __launch_bounds__(64) void k_xfold(DParams P, const TlPart* __restrict__ parts, uint32_t nblk, int i,
                                              const DevCtl* __restrict__ ctl) {
    // one load batch: halt, the summary fields the round accumulated (log
    // count, spills, errors), the window start, the stop time and the shares;
    // the summary is this kernel's alone to complete (fresh from the previous
    // round but for those fields), so it is written with plain stores and the
    // headers are packed from registers
    DevSummary* sum = P.sum;
    const uint32_t halt = *P.halt;
    const uint64_t ws = sum->ws, stop = ctl->stop, npend = sum->n_pending, nrem = sum->n_remote;
    const uint64_t next0 = sum->next_time;
    const uint32_t err0 = sum->error;
    TlPart f{kInf, 0, 0, 0, 0, 0};
    const bool fwd = ws >= stop;
    const TlPart* pp = parts + (size_t)(i & 1) * nblk;
    for (uint32_t j = threadIdx.x; j < nblk; j += 64) {
        const TlPart x = pp[j];
        if (!fwd) tl_fold(f, x);
    }
    if (halt) return;
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
    uint64_t next = fwd ? ws : f.next;
    next = next0 < next ? next0 : next;
    const uint32_t err = err0 | f.err;
    if (threadIdx.x == 0) {
        sum->next_time = next;
        if (!fwd) {
            sum->n_events = f.nev;
            sum->n_pkt_events = f.npkt;
            sum->n_active = f.nact;
            sum->error = err;
            sum->t_last = f.t_end;
        }
    }
    // this engine's headers (xpack_block with the values in registers)
    const int32_t p = threadIdx.x;
    if (p >= P.xworld) return;
    const uint32_t cnt = P.xcount[p];
    XHeader h;
    h.next_time = next;
    h.count = cnt < P.xcap ? cnt : P.xcap;
    uint32_t fl = 0;
    if (!fwd) {
        if (npend) fl |= XF_PENDING;
        if (nrem) fl |= XF_OVERFLOW;
        if (err) fl |= XF_ERROR;
    }
    h.flags = fl;
    h.n_pending = fwd ? 0 : npend;
    h.error = fwd ? err0 : err;
    h.tag = 0;
    *(XHeader*)(P.xsend + (size_t)p * (P.xcap + 1)) = h;
    P.xcount[p] = 0;
}

// events received in the exchange -> inbox[parity] of the next round
__global__ void k_ingest_x(DParams P, const shd_event* __restrict__ xrecv, const DevCtl* __restrict__ ctl, int ri) {
    if (*P.halt) return;
    const int parity = (int)((ctl->round_base + (uint64_t)ri + 1) & 1);   // the next round's inbox
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t p = t / P.xcap, s = t % P.xcap;
    if (p >= (uint64_t)P.xworld) return;
    const shd_event* blk = xrecv + p * ((uint64_t)P.xcap + 1);
    if (s >= ((const XHeader*)blk)->count) return;
    const shd_event e = blk[1 + s];
    const int32_t dl = (int32_t)e.dst - P.h0;
    if (dl < 0 || dl >= P.nloc) { atomicOr(&P.sum->error, SHD_ERR_REMOTE_OVERFLOW); return; }
    if (cal_push(P, dl, e, P.sum->ws)) return;   // the horizon of the round that sent it
    const uint32_t slot = atomicAdd(&P.inbox_n[parity][dl], 1u);
    if (slot >= P.inbox_cap) { atomicOr(&P.sum->error, SHD_ERR_INBOX_OVERFLOW); return; }
    P.inbox[parity][(size_t)dl * P.inbox_cap + slot] = e;
}

// ---- peer-to-peer exchange (shd_xgroup_create_p2p) ----
// Every engine's receive blocks ([2][world][stride] events) live in uncached
// device memory exported by IPC handle and mapped by every peer; a sender
// writes its block for peer p straight into p's receive blocks (over xGMI
// between GPUs), header last, tagged with the exchange's number; the
// receiver's next kernel waits for every peer's tag, then ingests.  Tags are
// never reused (a rerun round takes new ones), so a stale block cannot match.
constexpr unsigned long long kXWaitTicks = 3000000000ull;   // 30 s at the 100 MHz wall clock

__device__ __forceinline__ uint32_t x_tag(const DevCtl* ctl, uint32_t add, int use_ctl) {
    return use_ctl ? (uint32_t)ctl->xtag + add : add;
}

// block p: this engine's block for peer p -> p's receive block `me` of parity wi
// The block's events and header go out as write-through system-scope stores
// (the receive blocks are uncached: no L2 on either side keeps them); every
// storing wave drains them (vmcnt(0)) before the barrier, then one lane
// stores the header body, drains it, and stores the tag
__device__ __forceinline__ void x_put(const shd_event* __restrict__ src, shd_event* __restrict__ dst, uint32_t n,
                                      XHeader h, uint32_t tag) {
    const uint4* s16 = (const uint4*)(src + 1);
    for (uint32_t k = threadIdx.x; k < 2 * n; k += blockDim.x) st16_sys((uint4*)(dst + 1) + k, s16[k]);
    // the header's second 16 B ride with the events; its first 16 B (which
    // hold the tag) go alone, after every storing wave drained (one 16-B
    // store is not torn: a reader that sees the tag sees all of the header)
    const uint4 g0 = make_uint4((uint32_t)h.next_time, (uint32_t)(h.next_time >> 32), h.flags, tag);
    const uint4 g1 = make_uint4((uint32_t)h.n_pending, (uint32_t)(h.n_pending >> 32), h.error, h.count);
    if (threadIdx.x == 0) st16_sys((uint4*)dst + 1, g1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave, before the barrier
    __syncthreads();
    if (threadIdx.x == 0) {
        st16_sys(dst, g0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

__global__ __launch_bounds__(256) void k_xput(const shd_event* __restrict__ xsend, shd_event* const* __restrict__ peers,
                                               uint32_t stride, uint32_t xcap, int world, int me, int wi,
                                               const DevCtl* __restrict__ ctl, uint32_t tag_add, int use_ctl) {
    const int p = blockIdx.x;
    const shd_event* src = xsend + (size_t)p * stride;
    shd_event* dst = peers[p] + ((size_t)wi * world + me) * stride;
    XHeader h = *(const XHeader*)src;
    const uint32_t n = h.count < xcap ? h.count : xcap;
    x_put(src, dst, n, h, x_tag(ctl, tag_add, use_ctl));
}

// k_xfold and k_xput in one launch (peer-to-peer rounds): block p folds the
// round's shares (every block alike), packs this engine's header for peer p
// (block 0 also completes the summary), then puts the block into p's receive
// blocks.  A halted round re-sends the last header under the new tag, as the
// all-to-all re-sends the unchanged send blocks.
__device__ __forceinline__ void xfold_put(const DParams& P, const TlPart* __restrict__ parts, uint32_t nblk, int i,
                                          const DevCtl* __restrict__ ctl, shd_event* const* __restrict__ peers, int me,
                                          int wi, uint32_t tag_add, int use_ctl, int p) {
    __shared__ TlPart s_f[4];
    DevSummary* sum = P.sum;
    const uint32_t halt = *P.halt;
    const uint64_t ws = sum->ws, stop = ctl->stop, npend = sum->n_pending, nrem = sum->n_remote;
    const uint64_t next0 = sum->next_time;
    const uint32_t err0 = sum->error;
    const size_t stride = (size_t)P.xcap + 1;
    shd_event* src = P.xsend + (size_t)p * stride;
    if (!halt) {
        const bool fwd = ws >= stop;
        TlPart f{kInf, 0, 0, 0, 0, 0};
        const TlPart* pp = parts + (size_t)(i & 1) * nblk;
        for (uint32_t j = threadIdx.x; j < nblk; j += blockDim.x)
            if (!fwd) tl_fold(f, pp[j]);
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
        if ((threadIdx.x & 63) == 0) s_f[threadIdx.x >> 6] = f;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (uint32_t w = 1; w < blockDim.x / 64; w++) tl_fold(f, s_f[w]);
            uint64_t next = fwd ? ws : f.next;
            next = next0 < next ? next0 : next;
            const uint32_t err = err0 | f.err;
            if (p == 0) {
                sum->next_time = next;
                if (!fwd) {
                    sum->n_events = f.nev;
                    sum->n_pkt_events = f.npkt;
                    sum->n_active = f.nact;
                    atomicOr(&sum->error, err);   // the ingest of the same launch may add bits
                    sum->t_last = f.t_end;
                }
            }
            const uint32_t cnt = P.xcount[p];
            XHeader h;
            h.next_time = next;
            h.count = cnt < P.xcap ? cnt : P.xcap;
            uint32_t fl = 0;
            if (!fwd) {
                if (npend) fl |= XF_PENDING;
                if (nrem) fl |= XF_OVERFLOW;
                if (err) fl |= XF_ERROR;
            }
            h.flags = fl;
            h.n_pending = fwd ? 0 : npend;
            h.error = fwd ? err0 : err;
            h.tag = 0;
            *(XHeader*)src = h;
            P.xcount[p] = 0;
        }
    }
    __syncthreads();
    // the put (as k_xput); the round stored its events into the peer's block
    // already (P.xpeer): then only the header goes
    shd_event* dst = peers[p] + ((size_t)wi * P.xworld + me) * stride;
    XHeader h = *(const XHeader*)src;
    const uint32_t n = P.xpeer ? 0u : (h.count < P.xcap ? h.count : P.xcap);
    x_put(src, dst, n, h, x_tag(ctl, tag_add, use_ctl));
}

// wait for every peer's block of this exchange (bounded: a peer that never
// comes sets *xerr, and later waits of the batch return at once), then, for a
// round's exchange, the received events -> the next round's calendar / inbox
__device__ __forceinline__ void xwait_ingest(const DParams& P, const shd_event* __restrict__ xrecv,
                                             const DevCtl* __restrict__ ctl, uint32_t tag_add, int use_ctl, int ri,
                                             int ingest, uint32_t* __restrict__ xerr, uint32_t blk) {
    __shared__ uint32_t s_bad;
    const uint32_t tag = x_tag(ctl, tag_add, use_ctl);
    const size_t stride = (size_t)P.xcap + 1;
    if (threadIdx.x == 0) s_bad = __hip_atomic_load(xerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (s_bad) return;
    if ((int32_t)threadIdx.x < P.xworld) {
        const uint32_t* tw = (const uint32_t*)(xrecv + threadIdx.x * stride) + 3;   // XHeader::tag
        const unsigned long long t0 = wall_clock64();
        // relaxed polls (an acquire per poll would invalidate this CU's caches
        // each time), one acquire once the tag is there
        while (__hip_atomic_load(tw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != tag) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > kXWaitTicks) {
                atomicOr(&s_bad, 1u);
                __hip_atomic_fetch_or(xerr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    // no acquire fence: the receive blocks are uncached device memory (no L2
    // line of them on any XCD) and this CU holds no L1 line of them (the
    // kernel started with an invalidated L1, and the polls bypass it), so
    // the loads behind the barrier read what the peers' drained
    // write-through stores left in memory
    __syncthreads();
    if (s_bad) {
        if (threadIdx.x == 0) *P.halt = 1u;
        return;
    }
    if (!ingest) return;
    const uint64_t t = (uint64_t)blk * blockDim.x + threadIdx.x;
    const uint64_t p = t / P.xcap, s = t % P.xcap;
    if (p >= (uint64_t)P.xworld) return;
    // halt, the round base, the block's count and the slot's event in one
    // round trip (the slot is inside the block whatever the count); each is
    // consumed only once all are out, or the compiler would issue them one
    // behind the other's branch
    const shd_event* b = xrecv + p * stride;
    uint32_t halt = *P.halt;
    uint64_t rbase = ctl->round_base, ws = P.sum->ws;
    uint32_t cnt = ((const XHeader*)b)->count;
    uint4 e0 = ((const uint4*)(b + 1 + s))[0], e1 = ((const uint4*)(b + 1 + s))[1];
    asm volatile("" : "+v"(halt), "+v"(rbase), "+v"(ws), "+v"(cnt), "+v"(e0.x), "+v"(e0.y), "+v"(e0.z), "+v"(e0.w), "+v"(e1.x),
                 "+v"(e1.y), "+v"(e1.z), "+v"(e1.w));
    if (halt || s >= cnt) return;
    const int parity = (int)((rbase + (uint64_t)ri + 1) & 1);   // the next round's inbox
    shd_event e;
    {
        const uint4 ev[2] = {e0, e1};
        static_assert(sizeof(ev) == sizeof(e), "two 16-B halves");
        __builtin_memcpy(&e, ev, sizeof(e));
    }
    const int32_t dl = (int32_t)e.dst - P.h0;
    if (dl < 0 || dl >= P.nloc) { atomicOr(&P.sum->error, SHD_ERR_REMOTE_OVERFLOW); return; }
    if (cal_push(P, dl, e, ws)) return;
    const uint32_t slot = atomicAdd(&P.inbox_n[parity][dl], 1u);
    if (slot >= P.inbox_cap) { atomicOr(&P.sum->error, SHD_ERR_INBOX_OVERFLOW); return; }
    P.inbox[parity][(size_t)dl * P.inbox_cap + slot] = e;
}

__global__ __launch_bounds__(256) void k_xwait_ingest(DParams P, const shd_event* __restrict__ xrecv,
                                                       const DevCtl* __restrict__ ctl, uint32_t tag_add,
                                                       int use_ctl, int ri, int ingest, uint32_t* __restrict__ xerr) {
    xwait_ingest(P, xrecv, ctl, tag_add, use_ctl, ri, ingest, xerr, blockIdx.x);
}

// a round's whole exchange in one launch: blocks [0, world) fold and put
// (k_xfold_put), the rest wait for every peer's block and ingest.  The put
// blocks never wait, so the launch completes whatever the placement
__global__ __launch_bounds__(256) void k_xchg(DParams P, const TlPart* __restrict__ parts, uint32_t nblk, int i,
                                               const DevCtl* __restrict__ ctl, shd_event* const* __restrict__ peers,
                                               int me, int wi, uint32_t tag_add, const shd_event* __restrict__ xrecv,
                                               uint32_t* __restrict__ xerr) {
    if ((int)blockIdx.x < P.xworld)
        xfold_put(P, parts, nblk, i, ctl, peers, me, wi, tag_add, 1, (int)blockIdx.x);
    else
        xwait_ingest(P, xrecv, ctl, tag_add, 1, i, 1, xerr, blockIdx.x - (uint32_t)P.xworld);
}

// ---- fused peer-to-peer rounds (the default peer-to-peer schedule) ----
// Round i's launch (k_round_px) also completes exchange i - 1, so a round is
// one launch: blocks [0, world) fold round i - 1's shares and put this
// engine's header for peer p (granule 0 -- next time, flags, tag -- in one
// 16-B store; a flagged header's granule 1 first, drained); every block then
// waits for every peer's header of exchange i - 1 (lane p polls peer p's
// granule 0), takes the window start as their min, and ingests what the
// peers stored for its own hosts during round i - 1: region [wi][p][block]
// of kXSlots events, lane k reading slot k of every peer's region.  An event
// goes to its host's calendar (or inbox), and the lane that owns the host
// learns it through LDS, so the host state loaded at entry stays valid
// without a second round trip.  A batch: k_round_xtl (round 0: the exchange
// before it is done), k_round_px (rounds 1 ..), k_xchg_px (the last round's
// exchange).  Region slots hold an event iff its time is nonzero; the
// receiver zeroes a slot's time once it took the event (the sender stores
// into that region again two exchanges later, after it saw this engine's
// next header, which follows the end of this launch).
static_assert(kXSlots == (uint32_t)kBlock, "one region slot per lane");
constexpr int kXDefCap = 2;   // received events per lane whose calendar store waits for the round's end

__device__ __forceinline__ uint4 ld16_sys(const void* p) {
    u32x4 x;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(p) : "memory");
    return make_uint4(x[0], x[1], x[2], x[3]);
}

// The mapping's self-check (round 6: the transport had never crossed a
// device when the group was created).  Lane p < W stores a known 16-B granule
// into peer p's receive block, at this rank's header slot of parity 0, with the
// same system-scope store the exchange uses, and drains it; after a barrier
// over the communicator each rank reads every sender's granule from its own
// block with the exchange's system-scope load and checks it (bad: the senders
// whose granule was missing or wrong, one bit each).  The slots are zeroed
// again before the group's first exchange.
constexpr uint32_t kProbeMagic = 0x5ad0c0deu;
__global__ void k_p2p_probe_put(shd_event* const* __restrict__ peers, int world, int me, size_t stride, uint32_t gen,
                                int corrupt) {
    const int p = (int)threadIdx.x;
    if (p < world) {
        const uint4 v = make_uint4(kProbeMagic, (uint32_t)me, (uint32_t)p, gen + (uint32_t)corrupt);
        st16_sys(peers[p] + (size_t)me * stride, v);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__global__ void k_p2p_probe_check(const shd_event* __restrict__ mine, int world, int me, size_t stride, uint32_t gen,
                                  unsigned long long* __restrict__ bad) {
    const int p = (int)threadIdx.x;
    const bool ok = p >= world || [&] {
        const uint4 v = ld16_sys(mine + (size_t)p * stride);
        return v.x == kProbeMagic && v.y == (uint32_t)p && v.z == (uint32_t)me && v.w == gen;
    }();
    const unsigned long long m = __ballot(!ok);
    if (p == 0) *bad = m;
}

#ifdef SHD_TEST_HOOKS
// test build: exchanged events to lose on taking them (SHD_TEST_XDROP), so
// that a check of a group's end state against one engine can be seen to fail
__device__ int g_test_xdrop;
__device__ __forceinline__ bool test_xdrop() { return g_test_xdrop > 0 && atomicSub(&g_test_xdrop, 1) > 0; }
#define TEST_XDROP() if (test_xdrop()) continue
#else
#define TEST_XDROP()
#endif

// the events of the regions [p][blk] (p != xme) of one parity -> calendar /
// inbox[parity] of the block's hosts; s_n / s_w (or null): what each lane's
// host received, for the lane (inbox count, calendar bins).  Returns error bits.
__device__ uint32_t xrgn_ingest_from(const DParams& P, shd_event* __restrict__ rgn, uint32_t blk, uint64_t ws_send,
                                     int parity, uint32_t* s_n, uint32_t (*s_w)[kBlock], int32_t first) {
    uint32_t err = 0;
    const int32_t W = P.xworld;
    for (int32_t p0 = first; p0 < W; p0 += 8) {
        uint4 ea[8], eb[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {   // every slot's load out before any is consumed
            const int32_t p = p0 + k;
            ea[k] = make_uint4(0, 0, 0, 0);
            eb[k] = ea[k];
            if (p < W && p != P.xme) {
                const uint4* q = (const uint4*)(rgn + ((size_t)p * P.xnbx + blk) * kXSlots + threadIdx.x);
                ea[k] = q[0];
                eb[k] = q[1];
            }
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if ((ea[k].x | ea[k].y) == 0) continue;   // time 0: an empty slot
            shd_event e;
            {
                const uint4 ev[2] = {ea[k], eb[k]};
                __builtin_memcpy(&e, ev, sizeof(e));
            }
            // taken: a system-scope store, so that it has landed (not just left
            // this CU) before this block's next share lets the peer store there again
            __hip_atomic_store((unsigned long long*)(rgn + ((size_t)(p0 + k) * P.xnbx + blk) * kXSlots + threadIdx.x),
                               0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            TEST_XDROP();
            const int32_t dl = (int32_t)e.dst - P.h0;
            const int32_t j = dl - (int32_t)blk * P.hpw;
            if (dl < 0 || dl >= P.nloc || j < 0 || j >= P.hpw) {
                err |= SHD_ERR_REMOTE_OVERFLOW;
                continue;
            }
            if (P.bins) {   // cal_push, the bin noted for the owner lane
                const uint64_t bb = e.time >> P.bin_shift;
                if (bb - (ws_send >> P.bin_shift) <= kHorizon) {
                    const uint32_t pb = (uint32_t)bb & (kNB - 1);
                    const size_t bi = (size_t)dl * kNB + pb;
                    const uint32_t s = atomicAdd(&P.bin_n[bi], 1u);
                    if (s < kBinCap) {
                        ev_st_sc1(&P.bins[bi * kBinCap + s], e);   // write-through: the hand-off reaches other XCDs without a kernel boundary
                        atomicOr(&P.bin_bits[(size_t)dl * kNBW + (pb >> 5)], 1u << (pb & 31));
                        if (s_w) atomicOr(&s_w[pb >> 5][j], 1u << (pb & 31));
                        continue;
                    }
                }
            }
            const uint32_t slot = atomicAdd(&P.inbox_n[parity][dl], 1u);
            if (slot >= P.inbox_cap) {
                err |= SHD_ERR_INBOX_OVERFLOW;
                continue;
            }
            ev_st_sc1(&P.inbox[parity][(size_t)dl * P.inbox_cap + slot], e);
            if (s_n) atomicAdd(&s_n[j], 1u);
        }
    }
    return err;
}
__device__ __forceinline__ uint32_t xrgn_ingest(const DParams& P, shd_event* __restrict__ rgn, uint32_t blk,
                                                uint64_t ws_send, int parity, uint32_t* s_n, uint32_t (*s_w)[kBlock]) {
    return xrgn_ingest_from(P, rgn, blk, ws_send, parity, s_n, s_w, 0);
}

// the fused round's ingest (its window [ws, we) known, the round to run):
// peers [0, 8) of the regions only (the rest through xrgn_ingest).  An event
// of the window joins its host's due list (s_rx); a later one within the
// horizon claims its calendar slot now and is stored after the round
// (xrgn_store: the claims' round trip overlaps the round's), parked in
// s_def (at most kXDefCap per lane, in arrival order), its bin noted in s_w
// for the owner lane's next time; the rest
// (a full s_rx, beyond the horizon) go to the calendar / inbox at once,
// noted in s_n / s_w.  dm bit k: slot k's claim is in sl[k].
__device__ __forceinline__ uint32_t xrgn_take(const DParams& P, shd_event* __restrict__ rgn, uint32_t blk,
                                              uint64_t ws, uint64_t we, int parity, uint32_t* s_n,
                                              uint32_t (*s_w)[kBlock], shd_event* s_def, uint32_t (&sl)[8],
                                              uint32_t& dm) {
    uint32_t err = 0;
    const int32_t W = P.xworld;
    uint4 ea[8], eb[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        ea[k] = make_uint4(0, 0, 0, 0);
        eb[k] = ea[k];
        if (k < W && k != P.xme) {
            const uint4* q = (const uint4*)(rgn + ((size_t)k * P.xnbx + blk) * kXSlots + threadIdx.x);
            ea[k] = q[0];
            eb[k] = q[1];
        }
    }
    dm = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if ((ea[k].x | ea[k].y) == 0) continue;
        shd_event e;
        {
            const uint4 ev[2] = {ea[k], eb[k]};
            __builtin_memcpy(&e, ev, sizeof(e));
        }
        __hip_atomic_store((unsigned long long*)(rgn + ((size_t)k * P.xnbx + blk) * kXSlots + threadIdx.x), 0ull,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);   // taken (system scope: as above)
        TEST_XDROP();
        const int32_t dl = (int32_t)e.dst - P.h0;
        const int32_t j = dl - (int32_t)blk * P.hpw;
        if (dl < 0 || dl >= P.nloc || j < 0 || j >= P.hpw) {
            err |= SHD_ERR_REMOTE_OVERFLOW;
            continue;
        }
        const uint64_t bb = e.time >> P.bin_shift;
        if (e.time < ws) {   // cannot be: the sender's next time counts it
            err |= SHD_ERR_INTERNAL;
            continue;
        }
        if (e.time < we) {   // the window's
            const uint32_t r = atomicAdd(&s_rxn[j], 1u);
            if (r < (uint32_t)kRxCap) {
                s_rx[r * kBlock + j] = e;
                continue;
            }
        } else if (bb - (ws >> P.bin_shift) <= kHorizon && __popc(dm) < kXDefCap) {
            const uint32_t pb = (uint32_t)bb & (kNB - 1);
            sl[k] = atomicAdd(&P.bin_n[(size_t)dl * kNB + pb], 1u);   // consumed after the round
            s_def[__popc(dm) * kBlock + threadIdx.x] = e;                // parked in arrival order
            dm |= 1u << k;
            atomicOr(&s_w[pb >> 5][j], 1u << (pb & 31));
            continue;
        }
        // at once: the inbox of this round (merged at its start)
        const uint32_t slot = atomicAdd(&P.inbox_n[parity][dl], 1u);
        if (slot >= P.inbox_cap) {
            err |= SHD_ERR_INBOX_OVERFLOW;
            continue;
        }
        ev_st_sc1(&P.inbox[parity][(size_t)dl * P.inbox_cap + slot], e);
        atomicAdd(&s_n[j], 1u);
    }
    return err;
}

// after the round: the parked events into the slots claimed for them (a full
// bin: the next round's inbox)
__device__ __forceinline__ uint32_t xrgn_store(const DParams& P, const shd_event* s_def, const uint32_t (&sl)[8],
                                               uint32_t dm, int next_parity) {
    uint32_t err = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (!((dm >> k) & 1u)) continue;
        const shd_event e = s_def[__popc(dm & ((1u << k) - 1u)) * kBlock + threadIdx.x];
        const int32_t dl = (int32_t)e.dst - P.h0;
        const uint32_t pb = (uint32_t)(e.time >> P.bin_shift) & (kNB - 1);
        const size_t bi = (size_t)dl * kNB + pb;
        if (sl[k] < kBinCap) {
            ev_st_sc1(&P.bins[bi * kBinCap + sl[k]], e);
            atomicOr(&P.bin_bits[(size_t)dl * kNBW + (pb >> 5)], 1u << (pb & 31));
            continue;
        }
        const uint32_t slot = atomicAdd(&P.inbox_n[next_parity][dl], 1u);
        if (slot >= P.inbox_cap) {
            err |= SHD_ERR_INBOX_OVERFLOW;
            continue;
        }
        ev_st_sc1(&P.inbox[next_parity][(size_t)dl * P.inbox_cap + slot], e);
    }
    return err;
}

// block p (< world) of an exchange: fold the round's shares (loaded into pv
// by the caller; more past 256 blocks), complete its summary (block 0), pack
// this engine's header for peer p and put it into p's header block (wi, me).
// A halted round re-sends the last header under the new tag.
__device__ __forceinline__ void px_fold_put(const DParams& P, DevSummary* sum, const TlPart (&pv)[4],
                                            const TlPart* __restrict__ pp, uint32_t nblk, uint64_t pws,
                                            uint64_t npend, uint64_t nrem, uint64_t pnext, uint32_t perr,
                                            uint64_t stop, uint32_t halt, uint32_t bad,
                                            shd_event* const* __restrict__ peers,
                                            int world, int me, int wi, uint32_t tag, uint64_t xhoff, int nrep) {
    const int p = (int)blockIdx.x;
    const size_t stride = (size_t)P.xcap + 1;
    shd_event* src = P.xsend + (size_t)p * stride;
    TlPart f{kInf, 0, 0, 0, 0, 0};
    tl_fold4(f, pv, nblk, 0);
    for (uint32_t base = 256; base < nblk; base += 256) {
        TlPart v[4];
        tl_issue(pp, nblk, base, v);
        tl_fold4(f, v, nblk, base);
    }
    tl_reduce(f, true);
    XHeader h;
    if (!halt) {
        const bool fwd = pws >= stop;
        uint64_t next = fwd ? pws : f.next;
        next = pnext < next ? pnext : next;
        const uint32_t err = perr | f.err;
        h.next_time = next;
        uint32_t fl = 0;
        if (!fwd) {
            if (npend) fl |= XF_PENDING;
            if (nrem) fl |= XF_OVERFLOW;
            if (err) fl |= XF_ERROR;
        }
        h.flags = fl;
        h.tag = 0;
        h.n_pending = fwd ? 0 : npend;
        h.error = fwd ? perr : err;
        h.count = 0;
        if (threadIdx.x == 0) {
            if (p == 0) {
                sum->next_time = next;
                if (!fwd) {
                    sum->n_events = f.nev;
                    sum->n_pkt_events = f.npkt;
                    sum->n_active = f.nact;
                    atomicOr(&sum->error, err);
                    sum->t_last = f.t_end;
                }
            }
            *(XHeader*)src = h;   // the last header (a halted round re-sends it)
        }
    } else {
        h = *(const XHeader*)src;
        // this engine's wait for a peer timed out: the re-sent header carries
        // an error, so that every peer halts at the same exchange and fails
        // alike (no rank runs on, or enters a recovery collective, alone)
        if (bad) {
            h.flags |= XF_ERROR;
            h.error |= SHD_ERR_INTERNAL;
        }
    }
    // granule 0 also into the nrep - 1 replicas (the pollers of the peer's
    // blocks spread over them: fewer reads of one address per round trip)
    if ((int)threadIdx.x < nrep) {
        shd_event* dst = peers[p] + ((size_t)wi * world + me) * stride;
        const uint4 g0 = make_uint4((uint32_t)h.next_time, (uint32_t)(h.next_time >> 32), h.flags, tag);
        if (threadIdx.x == 0) {
            const uint4 g1 = make_uint4((uint32_t)h.n_pending, (uint32_t)(h.n_pending >> 32), h.error, h.count);
            st16_sys((uint4*)dst + 1, g1);
        }
        if (h.flags) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // a flagged header's body before its tag
        if (threadIdx.x > 0)
            dst = peers[p] + xhoff + ((size_t)wi * (kXReplMax - 1) + (threadIdx.x - 1)) * world + me;
        st16_sys(dst, g0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// wait for every peer's header of an exchange (lane p polls peer p's granule
// 0, bounded: a peer that never comes sets *xerr, and later waits return at
// once); the min next time and the flags over the group.  Wave-uniform.
__device__ __forceinline__ bool px_wait(const shd_event* __restrict__ xhdr, size_t stride, int world, uint32_t tag,
                                        uint32_t bad, uint32_t* __restrict__ xerr, uint64_t& ws, uint32_t& fl,
                                        const shd_event* __restrict__ xrep, int nrep, uint32_t blk) {
    ws = kInf;
    fl = 0;
    if (!bad && (int)threadIdx.x < world) {
        // replica blk % nrep of granule 0 (replica 0: the header block itself)
        const uint32_t r = blk % (uint32_t)nrep;
        const void* hp = r == 0 ? (const void*)(xhdr + (size_t)threadIdx.x * stride)
                                : (const void*)(xrep + (size_t)(r - 1) * world + threadIdx.x);
        const unsigned long long t0 = wall_clock64();
        for (;;) {
            const uint4 hx = ld16_sys(hp);
            if (hx.w == tag) {
                ws = ((uint64_t)hx.y << 32) | hx.x;
                fl = hx.z;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > kXWaitTicks) {
                bad = 1;
                __hip_atomic_fetch_or(xerr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(ws, off, 64);
        ws = o < ws ? o : ws;
        fl |= __shfl_xor(fl, off, 64);
    }
    return __ballot(bad != 0) != 0;
}

// zero this block's stripe of the region counters of parity wi (their sends
// were made in the previous round of that parity; the next use is two rounds on)
__device__ __forceinline__ void px_reset_counts(const DParams& P, int wi, uint32_t blk, uint32_t nblk) {
    const size_t n = (size_t)P.xworld * P.xnbx;
    uint32_t* c = P.xcnt + (size_t)wi * n;
    // agent-scope stores: the counters take other XCDs' atomics (a plain store
    // could sit in this XCD's L2 until a kernel boundary writes it back)
    for (size_t j = (size_t)blk * kBlock + threadIdx.x; j < n; j += (size_t)nblk * kBlock)
        __hip_atomic_store(&c[j], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool LEAN>   // LEAN: ParamsT::feat == 0 (round_body)
__global__ __launch_bounds__(kBlock) void k_round_px(uint64_t window, int i, DevSummary* __restrict__ prev,
                                                      const DevCtl* __restrict__ ctl, TlPart* __restrict__ parts,
                                                      const DParams* __restrict__ Pp, DevSummary* __restrict__ init,
                                                      DRoundArgs a, const shd_event* __restrict__ xhdr,
                                                      shd_event* __restrict__ rgn, shd_event* const* __restrict__ peers,
                                                      XHeader* __restrict__ halt_hdr, uint32_t* __restrict__ xerr,
                                                      int world, int me, int wprev, const shd_event* __restrict__ xrep,
                                                      uint64_t xhoff, int nrep) {
    __shared__ uint32_t s_xn[kBlock];
    __shared__ uint32_t s_xw[kNBW][kBlock];
    __shared__ shd_event s_def[kXDefCap * kBlock];
    const DParams& P = *Pp;
    const unsigned long long t_entry = wall_clock64();
    const uint32_t nblk = a.nblk;
    const bool putter = (int)blockIdx.x < world;
    asm volatile("" ::"s"(i), "s"(prev), "s"(ctl), "s"(parts), "s"(nblk), "s"(a.nloc), "s"(a.hpw), "s"(window));
    // the loads of the exchange go out first (halt, control words, round
    // i - 1's summary, its shares for the put blocks), the host state behind
    uint32_t halt = *a.halt, bad = *xerr;
    uint64_t stop = ctl->stop, rbase = ctl->round_base, xtag = ctl->xtag, xpar = ctl->xpar, pws = prev->ws;
    uint64_t npend = 0, nrem = 0, pnext = 0;
    uint32_t perr = 0;
    const TlPart* pp = parts + (size_t)((i - 1) & 1) * nblk;
    TlPart pv[4];
    if (putter) {
        tl_issue(pp, nblk, 0, pv);
        npend = prev->n_pending;
        nrem = prev->n_remote;
        pnext = prev->next_time;
        perr = prev->error;
    }
    const uint32_t warm = params_warm(Pp);
    HostIn in;
    host_in_load(a, in);
    s_xn[threadIdx.x] = 0;
    s_rxn[threadIdx.x] = 0;
#pragma unroll
    for (int k = 0; k < (int)kNBW; k++) s_xw[k][threadIdx.x] = 0;
    asm volatile("" : "+v"(halt), "+v"(bad), "+v"(stop), "+v"(rbase), "+v"(xtag), "+v"(xpar), "+v"(pws));
    const uint32_t tag = (uint32_t)(xtag + (uint64_t)(i - 1));
    const size_t stride = (size_t)P.xcap + 1;
    if (putter)
        px_fold_put(P, prev, pv, pp, nblk, pws, npend, nrem, pnext, perr, stop, halt, bad, peers, world, me, wprev, tag,
                    xhoff, nrep);
    if (blockIdx.x >= nblk) return;   // a put block past the engine's hosts (grid = max(nblk, world))
    uint64_t ws;
    uint32_t fl;
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    if (px_wait(xhdr, stride, world, tag, bad, xerr, ws, fl, xrep, nrep, blockIdx.x)) {
        if (threadIdx.x == 0) *P.halt = 1u;
        if (lead) P.sum->flags = 2u;
        return;
    }
    const int parity = (int)((rbase + (uint64_t)i) & 1);
    __syncthreads();   // s_xn / s_xw / s_rxn zeroed
    uint32_t ierr = 0;
    uint64_t we = ws + window;
    if (we > stop || we < ws) we = stop;
    // a round that runs takes the window's events onto the due lists and
    // defers the calendar stores of the rest; otherwise all go in at once
    const bool runs = !halt && !fl && ws < stop && P.bins;
    uint32_t sl[8], dm = 0;
    if (runs) {
        ierr = xrgn_take(P, rgn, blockIdx.x, ws, we, parity, s_xn, s_xw, s_def, sl, dm);
        if (world > 8) {   // peers past the first eight
            ierr |= xrgn_ingest_from(P, rgn, blockIdx.x, pws, parity, s_xn, s_xw, 8);
        }
    } else if (!halt) {
        ierr = xrgn_ingest(P, rgn, blockIdx.x, pws, parity, s_xn, s_xw);
    }
    px_reset_counts(P, wprev, blockIdx.x, nblk);
    __syncthreads();
    if (halt) {
        if (lead) P.sum->flags = 2u;
        return;
    }
    if (fl) {   // flagged somewhere in the group: every engine halts here alike
        if (blockIdx.x == 0) {
            if ((int)threadIdx.x < world) {
                const void* hp = xhdr + (size_t)threadIdx.x * stride;
                const uint4 g0 = ld16_sys(hp), g1 = ld16_sys((const uint4*)hp + 1);
                XHeader h;
                h.next_time = ((uint64_t)g0.y << 32) | g0.x;
                h.flags = g0.z;
                h.tag = g0.w;
                h.n_pending = ((uint64_t)g1.y << 32) | g1.x;
                h.error = g1.z;
                h.count = g1.w;
                halt_hdr[threadIdx.x] = h;
            }
            if (threadIdx.x == 0) {
                *P.halt = 1u;
                P.sum->flags = 1u;
            }
        }
        return;
    }
    if (lead) {
        atomicMin(&P.sum->t_first, t_entry);
        *init = fresh_summary();
        P.sum->ws = ws;
    }
    if (ws >= stop) return;   // only forwards the time (the next exchange packs it)
    params_warm_done(warm);
    // (the window end: computed above)
    {   // what this lane's host received in the exchange
        const uint32_t n = s_xn[threadIdx.x];
        if (parity) in.nin[1] += n;
        else in.nin[0] += n;
#pragma unroll
        for (int k = 0; k < (int)kNBW; k++) in.w[k] |= s_xw[k][threadIdx.x];
    }
    uint64_t next, nev, npkt;
    uint32_t err;
    round_body<true, LEAN>(P, in, ws, we, parity, next, nev, npkt, err, (uint32_t)((xpar + (uint64_t)i) & 1));
    if (dm) ierr |= xrgn_store(P, s_def, sl, dm, parity ^ 1);
    err |= ierr;
    const uint32_t nact = (uint32_t)__popcll(__ballot(nev != 0));
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(next, off, 64);
        next = o < next ? o : next;
        nev += __shfl_xor(nev, off, 64);
        npkt += __shfl_xor(npkt, off, 64);
        err |= __shfl_xor(err, off, 64);
    }
    if (threadIdx.x == 0)
        parts[(size_t)(i & 1) * nblk + blockIdx.x] =
            TlPart{next, (unsigned long long)wall_clock64(), (unsigned)nev, (unsigned)npkt, err, nact};
}

// ---- sparse fused rounds (k_round_spx): the engine group at the north
// star's shard (125 k hosts per GPU, a few percent of them with something due
// in a window).  k_round_px gives every 64-host block a wave per round (1954
// waves at 125 k hosts, against ~768 resident: three passes of blocks, each
// taking the exchange's wait); here, as in the single engine's k_round_sp, a
// block owns sph hosts (a multiple of 64, so its region blocks are whole),
// takes what the peers stored for them into their calendars / inboxes, scans
// their hand-off words, compacts the hosts with something due and runs them
// 64 at a time.  Still one launch per round (the region take reads slots a
// peer stored into over xGMI: a launch boundary between the peer's stores and
// the take keeps every load of a slot off a stale line), with
// k_round_px's fold / put / wait in front: blocks [0, world) fold round i - 1's
// shares and put the headers, every block waits for every peer's header.
// first: the batch's round 0 (the exchange before it is complete: its headers
// read from xhdr, its regions taken by the last batch's k_xchg_px).
template <bool LEAN>   // LEAN: ParamsT::feat == 0 (round_body)
__global__ __launch_bounds__(kBlock) void k_round_spx(uint64_t window, int i, DevSummary* __restrict__ prev,
                                                       const DevCtl* __restrict__ ctl, TlPart* __restrict__ parts,
                                                       const DParams* __restrict__ Pp, DevSummary* __restrict__ init,
                                                       const shd_event* __restrict__ xhdr, shd_event* __restrict__ rgn,
                                                       shd_event* const* __restrict__ peers,
                                                       XHeader* __restrict__ halt_hdr, uint32_t* __restrict__ xerr,
                                                       int world, int me, int wprev, const shd_event* __restrict__ xrep,
                                                       uint64_t xhoff, int nrep, uint32_t sph, uint32_t nsp, int first) {
    const DParams& P = *Pp;
    const unsigned long long t_entry = wall_clock64();
    const bool putter = !first && (int)blockIdx.x < world;
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    uint32_t halt = *P.halt, bad = *xerr;
    const uint64_t stop = ctl->stop, rbase = ctl->round_base, xtag = ctl->xtag, xpar = ctl->xpar;
    const size_t stride = (size_t)P.xcap + 1;
    uint64_t ws = kInf, pws = 0;
    uint32_t fl = 0;
    if (first) {   // as k_round_xtl: lane p reads peer p's header of the completed exchange
        const XHeader hx = *(const XHeader*)(xhdr + (size_t)((int)threadIdx.x < world ? threadIdx.x : 0) * stride);
        ws = (int)threadIdx.x < world ? hx.next_time : kInf;
        fl = (int)threadIdx.x < world ? hx.flags : 0u;
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t o = __shfl_xor(ws, off, 64);
            ws = o < ws ? o : ws;
            fl |= __shfl_xor(fl, off, 64);
        }
        if (blockIdx.x >= nsp) return;
    } else {
        pws = prev->ws;
        const TlPart* pp = parts + (size_t)((i - 1) & 1) * nsp;
        const uint32_t tag = (uint32_t)(xtag + (uint64_t)(i - 1));
        if (putter) {
            TlPart pv[4];
            tl_issue(pp, nsp, 0, pv);
            px_fold_put(P, prev, pv, pp, nsp, pws, prev->n_pending, prev->n_remote, prev->next_time, prev->error, stop,
                        halt, bad, peers, world, me, wprev, tag, xhoff, nrep);
        }
        if (blockIdx.x >= nsp) return;   // a put block past the engine's blocks (grid = max(nsp, world))
        if (px_wait(xhdr, stride, world, tag, bad, xerr, ws, fl, xrep, nrep, blockIdx.x)) {
            if (threadIdx.x == 0) *P.halt = 1u;
            if (lead) P.sum->flags = 2u;
            return;
        }
    }
    const int parity = (int)((rbase + (uint64_t)i) & 1);
    const uint32_t hb = blockIdx.x * sph;   // the block's first host
    const uint32_t nh = (uint32_t)P.nloc - hb < sph ? (uint32_t)P.nloc - hb : sph;
    const uint32_t ngrp = (nh + 63u) >> 6;
    uint32_t ierr = 0;
    if (!first) {
        // the peers' stores for this block's hosts (region blocks hb / 64 ...),
        // into their calendars / inboxes, before the scan reads them
        if (!halt && world > 1)
            for (uint32_t gq = 0; gq < ngrp; gq++)
                ierr |= xrgn_ingest_from(P, rgn, hb / 64u + gq, pws, parity, nullptr, nullptr, 0);
        px_reset_counts(P, wprev, blockIdx.x, nsp);
    }
    if (halt) {
        if (lead) P.sum->flags = 2u;
        return;
    }
    if (fl) {   // flagged somewhere in the group: every engine halts here alike
        if (blockIdx.x == 0) {
            if ((int)threadIdx.x < world) {
                const void* hp = xhdr + (size_t)threadIdx.x * stride;
                XHeader h;
                if (first) {
                    h = *(const XHeader*)hp;
                } else {
                    const uint4 g0 = ld16_sys(hp), g1 = ld16_sys((const uint4*)hp + 1);
                    h.next_time = ((uint64_t)g0.y << 32) | g0.x;
                    h.flags = g0.z;
                    h.tag = g0.w;
                    h.n_pending = ((uint64_t)g1.y << 32) | g1.x;
                    h.error = g1.z;
                    h.count = g1.w;
                }
                halt_hdr[threadIdx.x] = h;
            }
            if (threadIdx.x == 0) {
                *P.halt = 1u;
                P.sum->flags = 1u;
            }
        }
        return;
    }
    if (lead) {
        atomicMin(&P.sum->t_first, t_entry);
        *init = fresh_summary();
        P.sum->ws = ws;
    }
    if (ws >= stop) return;   // only forwards the time (the next exchange packs it)
    uint64_t we = ws + window;
    if (we > stop || we < ws) we = stop;
    if (threadIdx.x == 0) s_rsum = P.sum;
#ifdef SHD_TIMING_P0
    if (threadIdx.x == 0) s_tslot = TIM_SLOT();
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the take's stores, before the scan's loads
    __syncthreads();
    // ---- k_round_sp's round over this block's hosts
    PsRsrc R;
    R.bits = buf_rsrc(P.bin_bits ? P.bin_bits + (size_t)hb * kNBW : nullptr, (uint64_t)nh * kNBW * 4);
    R.bins = buf_rsrc(P.bins ? P.bins + (size_t)hb * kNB * kBinCap : nullptr,
                      (uint64_t)nh * kNB * kBinCap * sizeof(shd_event));
    R.nin = buf_rsrc(P.inbox_n[parity] + hb, (uint64_t)nh * 4);
    R.inbox = buf_rsrc(P.inbox[parity] + (size_t)hb * P.inbox_cap, (uint64_t)nh * P.inbox_cap * sizeof(shd_event));
    HostCtx c;
    hot_load(P, c);
    if (LEAN) { c.k.feat = 0; c.k.boot_end = 0; }
    c.l = P.nloc; c.h = 0; c.att = 0; c.cls = 0; c.evq_n = 0; c.top_time = kInf; c.peer = -1; c.rq_head = 0;
    c.tt0 = c.tt1 = c.tt2 = kInf; c.ev_seq = 0; c.cq_hv = false; c.tq_hv = false;
    const uint32_t xwi = (uint32_t)((xpar + (uint64_t)i) & 1);
    ps_round_reset(P, c, ws, we, parity, false);
    c.xwi = xwi;
    uint64_t next;
    uint32_t nact;
    sp_scan(P, R, hb, nh, ngrp, ws, we, next, nact, s_act, nullptr);
    __syncthreads();
    uint32_t nev = 0, npkt = 0, err = c.err | ierr, nhost = 0;
    sp_passes<false>(P, c, R, hb, nact, ws, we, parity, xwi, next, nev, npkt, err, nhost, s_act, nullptr, nullptr);
    // peer-to-peer: this block's stores into the peers' regions land before the
    // round ends (the next launch's put block announces them)
    if (P.xpeer) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(next, off, 64);
        next = o < next ? o : next;
        nev += __shfl_xor(nev, off, 64);
        npkt += __shfl_xor(npkt, off, 64);
        err |= __shfl_xor(err, off, 64);
    }
    if (threadIdx.x == 0)
        parts[(size_t)(i & 1) * nsp + blockIdx.x] =
            TlPart{next, (unsigned long long)wall_clock64(), (unsigned)nev, (unsigned)npkt, err, nhost};
}

// the exchange of a batch's last round i (P.sum: its summary): blocks
// [0, world) fold the round's nparts shares and put, blocks [world, world +
// nblk) wait and ingest their 64-host block's regions into the next round's
// calendar / inbox
__global__ __launch_bounds__(kBlock) void k_xchg_px(DParams P, const TlPart* __restrict__ parts, uint32_t nparts,
                                                     uint32_t nblk, int i,
                                                     const DevCtl* __restrict__ ctl, shd_event* const* __restrict__ peers,
                                                     int world, int me, int wi, const shd_event* __restrict__ xhdr,
                                                     shd_event* __restrict__ rgn, uint32_t* __restrict__ xerr,
                                                     const shd_event* __restrict__ xrep, uint64_t xhoff, int nrep) {
    DevSummary* sum = P.sum;
    uint32_t halt = *P.halt, bad = *xerr;
    uint64_t stop = ctl->stop, rbase = ctl->round_base, xtag = ctl->xtag, pws = sum->ws;
    const uint32_t tag = (uint32_t)(xtag + (uint64_t)i);
    const TlPart* pp = parts + (size_t)(i & 1) * nparts;
    if ((int)blockIdx.x < world) {
        TlPart pv[4];
        tl_issue(pp, nparts, 0, pv);
        const uint64_t npend = sum->n_pending, nrem = sum->n_remote, pnext = sum->next_time;
        const uint32_t perr = sum->error;
        px_fold_put(P, sum, pv, pp, nparts, pws, npend, nrem, pnext, perr, stop, halt, bad, peers, world, me, wi, tag,
                    xhoff, nrep);
        return;
    }
    const uint32_t blk = blockIdx.x - (uint32_t)world;
    uint64_t ws;
    uint32_t fl;
    if (px_wait(xhdr, (size_t)P.xcap + 1, world, tag, bad, xerr, ws, fl, xrep, nrep, blk)) {
        if (threadIdx.x == 0) *P.halt = 1u;
        return;
    }
    if (!halt) {
        const uint32_t err = xrgn_ingest(P, rgn, blk, pws, (int)((rbase + (uint64_t)i + 1) & 1), nullptr, nullptr);
        if (err) atomicOr(&sum->error, err);
    }
    px_reset_counts(P, wi, blk, nblk);
}

__global__ void k_digest(DParams P, shd_host_digest* __restrict__ out) {
    const int32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= P.nloc) return;
    shd_host_digest d;
    const HostRec r = P.hs[l];
    d.ev_seq = r.ev_seq; d.rx_remaining = r.rx_rem; d.tx_remaining = r.tx_rem;
    d.codel_total = r.cq_total; d.codel_interval_expire = r.cq_iexp; d.codel_next_drop = r.cq_ndrop;
    const HostCnt k = P.hc[l];
    d.n_events = k.events; d.n_pkt_events = k.pkt; d.n_sent = k.sent;
    d.n_inet_drop = k.idrop; d.n_codel_drop = k.cdrop; d.n_recv = k.recv;
    d.rng = r.rng; d.pkt_seq = r.pkt_seq;
    const uint32_t f = r.flags;
    d.codel_mode = (f & F_CODEL_DROP_MODE) ? 1u : 0u;
    d.codel_count = r.cq_count; d.codel_drop_count = r.cq_dc; d.codel_drop_count_last = r.cq_dcl;
    d.unread = r.unread;
    d.flags = (f & F_REFILL_PENDING ? 1u : 0u) | (f & F_NOTIFY_PENDING ? 2u : 0u) | (f & F_LISTENING ? 4u : 0u) |
              (r.tq_count ? 8u : 0u);
    out[l] = d;
}

// min over valid latencies of a table -> *out (u64 bits)
__global__ void k_min_valid(const shd_pv* __restrict__ a, size_t n, unsigned long long* __restrict__ out) {
    __shared__ unsigned long long sm[256];
    unsigned long long m = kDistInf;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double v = a[i].lat;
        if (v >= 0.0) {
            const unsigned long long b = (unsigned long long)__double_as_longlong(v);
            if (b < m) m = b;
        }
    }
    sm[threadIdx.x] = m;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s && sm[threadIdx.x + s] < sm[threadIdx.x]) sm[threadIdx.x] = sm[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMin(out, sm[0]);
}
