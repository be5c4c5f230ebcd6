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
// Device layout (HBM): struct-of-arrays host state; a per-host binary heap of
// 32-B events; double-buffered per-host inboxes filled with one atomicAdd per
// event on the destination's counter; per-host CoDel and send FIFOs.  The
// first-touch path-cache rule is applied from per-vertex row ranks;
// the rare sends whose pair was unranked at round start are logged, resolved
// in serial order on the host after the round, and finalised by k_finalize.
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

constexpr uint64_t kInf = 0xFFFFFFFFFFFFFFFFull;
constexpr uint32_t F_REFILL_PENDING = 1u, F_NOTIFY_PENDING = 2u, F_LISTENING = 4u, F_CODEL_DROP_MODE = 8u;
constexpr double kRandMax = 2147483647.0;
constexpr uint64_t kCodelTarget = 10ull * SHD_MS;      // router_queue_codel.c:42
constexpr uint64_t kCodelInterval = 100ull * SHD_MS;   // router_queue_codel.c:48
// calendar geometry: bins per host (a ring), event slots per bin, bitmap
// words, and the append horizon in bins ahead of the round's first bin.  The
// horizon stops short of the ring by 4 so that no append in round r can land
// in a slot the owner reads or clears in round r or r+1.
constexpr uint32_t kNB = 256, kBinCap = 4, kNBW = kNB / 32, kHorizon = kNB - 4;
constexpr int kDueCap = 6;             // due-list slots per host (more due events take the heap)
constexpr int kSendCap = 5;            // deferred sends per host between flushes (<= 16; with the
                                       // due list and the flush's arrays, 40 KB of LDS per block:
                                       // four blocks per CU once hosts fill the machine)
constexpr int kBlock = 64;             // round-kernel workgroup: one wave, one host per lane

struct CodelEnt {
    uint64_t ts;
    uint32_t src;
    uint32_t pkt;
};
// send-FIFO entry: the destination draw (rand_r value; the destination itself
// is resolved when the send is flushed) and the packet id
struct TxEnt {
    uint32_t r;
    uint32_t pkt;
};

// A send whose destination, path lookup and drop decision are deferred to the
// host's next flush (flush_sends).  The host's own control flow never depends
// on them: the RNG draws are made at send time, loopback is decided from the
// host's own cumulative-weight interval, and the event ID a passing send
// consumes is handled with provisional IDs fixed up at the flush.
struct SendRec {
    uint64_t now;      // send time
    uint64_t q_seq;    // the executing event's seq (first-touch log key)
    uint32_t q_src;    // the executing event's src
    uint32_t pseq;     // provisional event ID - seq_base
    uint32_t r;        // destination draw (rand_r value)
    uint32_t chance;   // reliability draw (rand_r value)
    uint32_t pkt;
    uint32_t q_sub;    // send index within the executing event; bit 31: bootstrapping
};
static_assert(sizeof(SendRec) == 40, "send record layout");

// Per-host state record in HBM (local host index), one 128-B line: the round
// kernel reads and writes it whole, as 8 16-B accesses; it holds every field
// the host's event handling mutates except the queues' contents and the
// counters.  Narrowed where the range allows (HostCtx holds the full widths):
// a live timer's event ID as its distance back from ev_seq (a timer is armed
// at most a heartbeat interval's events ago; an empty slot's ID is never
// read), the token buckets and CoDel's byte count in 32 bits (checked at
// create: refill + MTU and capacity x packet length below 2^32), the FIFO
// heads and lengths in 16 bits (capacities <= 65535).
struct alignas(128) HostRec {
    uint64_t ev_seq;                       // host_getNewEventID counter (host.c:397)
    uint64_t cq_iexp, cq_ndrop;            // CoDel: interval expiry, next drop
    uint64_t tt[3];                        // timer slots (heartbeat, refill, notify): time (kInf: empty)
    uint32_t ts_back[3];                   // ... their event IDs: ev_seq - ID (0 for an empty slot)
    uint32_t rx_rem, tx_rem;               // token buckets: bytes remaining
    uint32_t cq_total;                     // CoDel: bytes queued
    uint32_t rng, pkt_seq;                 // rand_r state, packet counter
    uint32_t rx_refill, tx_refill;         // token-bucket refill per 1 ms (bytes)
    uint32_t flags, unread;
    uint32_t cq_dc, cq_dcl;                // CoDel drop counts
    uint16_t cq_head, cq_count, tq_head, tq_count;   // FIFO heads / lengths
    uint32_t evq_n;
    uint32_t if_in, if_out;                // tracker node counters: interface packets in / out (cumulative)
    uint32_t pad;
};
static_assert(sizeof(HostRec) == 128, "host record: one 128-B line, 8 x 16 B");

// per-host counters; a round adds its deltas with fire-and-forget atomics
struct HostCnt {
    unsigned long long events, pkt, sent, idrop, cdrop, recv;
};

// a block's share of the round summary (round_complete)
struct BlockPart {
    unsigned long long next, nev, npkt;
    unsigned int err, nact;   // nact: hosts with at least one event
};
constexpr uint32_t kTickGroup = 64;   // blocks per first-level completion ticket

// a send whose (src,dst) pair was unranked at round start (include/shdgpu.h)
using Pending = shd_pending;
static_assert(sizeof(Pending) == 56, "pending record layout");

// engine-wide counters / summary on the device
struct DevSummary {
    unsigned long long next_time;
    unsigned long long n_events;
    unsigned long long n_pkt_events;
    unsigned long long n_pending;
    unsigned long long n_remote;
    unsigned int error;
    unsigned int flags;            // exchange mode: 1 = this round halted the batch, 2 = skipped
    unsigned long long ws;         // the round's window start (device-driven rounds)
    unsigned long long t_first;    // device wall clock: first block start, last block end
    unsigned long long t_last;
    unsigned int done;             // blocks finished (last-block ticket)
    unsigned int n_active;         // hosts that executed at least one event (ticketless rounds)
};

__device__ __forceinline__ DevSummary fresh_summary() {
    DevSummary z{};
    z.next_time = ~0ull;
    z.t_first = ~0ull;
    return z;
}

// per-batch inputs of the device-driven rounds (device memory, so that a
// captured batch graph is replayed unchanged): round i of the batch has
// parity (round_base + i) & 1
struct DevCtl {
    unsigned long long stop;
    unsigned long long round_base;
    unsigned long long xtag;   // peer-to-peer exchanges: the tag of the batch's first round (round i: + i)
    unsigned long long xpar;   // peer-to-peer: the receive-block parity of the batch's first round (round i: + i)
};

// Exchange mode (shd_xgroup): the per-peer blocks of the fixed-size
// all-to-all buffers start with one header slot, then `xcap` events.
// Granule 0 (the first 16 B) holds what a round needs to start -- the next
// time, the flags and, peer-to-peer, the exchange's tag -- so that one 16-B
// store publishes it and one 16-B load reads it; granule 1 what a flagged
// round's recovery needs.
struct XHeader {
    unsigned long long next_time;  // sender's earliest pending event (its hosts + its sends in flight)
    uint32_t flags;                // XF_* of the sender's round
    uint32_t tag;                  // peer-to-peer: the exchange's number (0 on the other transports)
    unsigned long long n_pending;  // sender's first-touch log of the round
    uint32_t error;
    uint32_t count;                // events in this block (<= xcap)
};
static_assert(sizeof(XHeader) == sizeof(shd_event), "header fills one event slot");
constexpr uint32_t XF_PENDING = 1u, XF_OVERFLOW = 2u, XF_ERROR = 4u;
// fused peer-to-peer rounds: event slots per (sender, destination block) region
// and round; one lane of the receiving block reads one slot
constexpr uint32_t kXSlots = 64;
constexpr int kXReplMax = 8;   // fused peer-to-peer rounds: copies of a header's granule 0 (x_nrep)

// destination-pick guide: for bucket k, i = the first index with
// dest_cum[i] >= k / H, and the next three cumulative weights inline, so an
// even-weight pick resolves in one 32-B load
struct DestGuide {
    int32_t i;
    int32_t att[3];  // attached-vertex index of hosts i .. i+2 (-1 past the end)
    double cum[3];   // dest_cum[i .. i+2], 2.0 past the end
    double pad;
};
static_assert(sizeof(DestGuide) == 48, "guide entry: three 16-B loads");

constexpr int kDestExc = 16;   // closed-form destination exceptions (ParamsT::exc_x)
// ParamsT::feat: the model's optional features (all off on the bench's models)
constexpr uint32_t F_TRACE = 1u, F_HB = 2u, F_PCOUNT = 4u, F_HOSTHB = 8u, F_AMBIG = 16u, F_STATUS = 64u;

template <template <class> class Ptr>
struct ParamsT {
    // hosts
    int32_t H;                  // total hosts of the model
    int32_t h0, nloc;           // this engine's hosts [h0, h0+nloc)
    int32_t hpw;                // hosts per wave in the round kernel (lanes >= hpw idle)
    uint32_t evq_cap, inbox_cap, cq_cap, tq_cap;
    uint64_t end_time, bootstrap_end, heartbeat, app_start;
    uint32_t load, payload, feat, pkt_len;   // feat: F_* optional features of the model
    // per-host state records (local index), and the earliest pending event
    // of each host's timers and heap (read alone by the idle test)
    Ptr<HostRec> hs;
    Ptr<HostCnt> hc;
    Ptr<uint64_t> hnext;
    // queues: per-host 4-ary heap of the other events (packets, loopback, boot one-shots)
    Ptr<shd_event> evq;              // slab of evq_stride entries per host, heap at +3
    uint32_t evq_stride;
    Ptr<shd_event> inbox[2];
    Ptr<uint32_t> inbox_n[2];
    // round completion (round_complete): per-block and per-group summary
    // shares, and the two-level tickets (reset by the blocks that win them)
    Ptr<BlockPart> part;
    Ptr<BlockPart> gpart;
    Ptr<uint32_t> tick;
    // calendar (null = off): per host a ring of kNB time bins of width
    // 2^bin_shift <= W ns with kBinCap event slots each.  Senders append with
    // one atomic on the bin's count; the owner reads the <= 3 bins of its
    // window in one pass.  Far-future events and full bins take the inbox.
    Ptr<shd_event> bins;             // [nloc][kNB][kBinCap]
    Ptr<uint32_t> bin_n;             // [nloc][kNB] appends (may exceed kBinCap: those went to the inbox)
    Ptr<uint32_t> bin_bits;          // [nloc][kNBW] non-empty bins
    uint32_t bin_shift;
    Ptr<CodelEnt> cq;
    Ptr<TxEnt> tq;
    // global host tables (all H hosts)
    Ptr<const int32_t> host_att;     // attached index of every host
    // destination weights per class (each PHOLD process reads its own weights
    // file): row c of dest_cum / dest_guide is class c's, [n_cls][H]
    Ptr<const double> dest_cum;
    Ptr<const DestGuide> dest_guide;   // [n_cls][H]: bucket k -> first i with dest_cum[i] >= k / H
    // destination draws as rand_r values x (r = x / RAND_MAX), per host h:
    // there is a destination iff x <= self_thr[h].z; its own draws (loopback)
    // are self_thr[h].x <= x <= self_thr[h].y (precomputed, exact); .w = class
    Ptr<const int4> self_thr;
    Ptr<const uint64_t> host_hb;     // per-host heartbeat interval [H] (null: `heartbeat`)
    int32_t no_app_start;            // SHD_QF_NO_APP_START: boot schedules no application start
    // closed-form destinations (dest_closed): even weights, host h attached
    // at index h.  The draw x picks host max(ceil(x*H/RAND_MAX) - 1, 0),
    // except at the listed draws (where the f64 cumulative sums round across
    // a threshold); verified on the host at every step of both functions
    int32_t dest_closed, n_exc;
    int32_t force_ambig;        // test hook (SHD_FORCE_AMBIG): every undecided first-touch send is ambiguous
    Ptr<uint32_t> pcount;       // per-path packet counters [T][T] (SHD_QF_COUNT_PATHS), else null
    Ptr<uint2> hb;              // heartbeat snapshots [nloc][hb_k] (SHD_QF_HEARTBEATS), else null
    uint32_t hb_k;
    int32_t exc_x[kDestExc], exc_d[kDestExc];
    // path cache
    int32_t T;
    int32_t complete, prefer_direct, directed;
    Ptr<const shd_pv> row;           // [T][T] (lat, rel)
    Ptr<const shd_pv> dir;           // [T][T] direct-edge values
    Ptr<const shd_pv> self;          // [T] self-path values
    Ptr<const uint8_t> adj;
    Ptr<const int32_t> rank;
    Ptr<const int32_t> self_rank;
    // outputs
    Ptr<Pending> pend;
    uint32_t pend_cap;
    Ptr<shd_event> remote;
    uint32_t remote_cap;
    Ptr<shd_trace_rec> trace_buf;
    uint64_t trace_cap;
    unsigned long long* trace_n;   // cumulative trace records
    Ptr<DevSummary> sum;               // this round's summary
    Ptr<int32_t> next_rank;            // row-rank counter (device is the source of truth)
    Ptr<uint32_t> halt;                // set when a round needs host-side resolution
    // exchange mode (null xsend: remote events go to `remote`)
    Ptr<shd_event> xsend;              // [xworld][xcap + 1]
    Ptr<uint32_t> xcount;              // [xworld] events queued per peer this round
    uint32_t xcap;
    int32_t xworld;                // engines of the group; host partition (H*p)/xworld
    // peer-to-peer transport: every rank's receive blocks ([2][xworld][xcap+1]
    // events, mapped here); a round stores its sends to peer p straight into
    // block (wi, xme) of xpeer[p] (null: the send blocks xsend)
    shd_event* const* xpeer;
    int32_t xme, xpad;
    // fused peer-to-peer rounds: a send for host d of peer p goes to p's
    // region [wi][xme][(d - h0(p)) / hpw] (xpeer[p] + xroff, kXSlots events
    // per region; slot from xcnt[wi][p][block]); null xcnt: the blocks above
    Ptr<uint32_t> xcnt;                // [2][xworld][xnbx]
    uint32_t xnbx;                     // region blocks per rank: ceil(ceil(H / xworld) / hpw)
    uint32_t xrcap;                    // region slots used: min(kXSlots, xcap) (small blocks force spills)
    uint64_t xroff;                    // events from a rank's receive base to its regions
};
// The host fills Params (plain pointers); device code reads the same bytes
// as DParams, whose pointers carry the global address space, so that loads
// and stores through a Params read via a pointer stay global_* instructions
// (generic pointers would make every access a flat_* one).
template <class T> using HostPtr = T*;
#ifdef __HIP_DEVICE_COMPILE__
template <class T> using GlobalPtr = T __attribute__((address_space(1)))*;
#else   // the host pass only type-checks device code: no address spaces there
template <class T> using GlobalPtr = T*;
#endif
using Params = ParamsT<HostPtr>;
using DParams = ParamsT<GlobalPtr>;
static_assert(sizeof(Params) == sizeof(DParams), "one layout");
static inline const DParams& dp(const Params& P) { return *reinterpret_cast<const DParams*>(&P); }


// engine of the group that owns host h: the partition is b[p] = (H*p)/N
__device__ __forceinline__ int32_t owner_of(const DParams& P, uint32_t h) {
    const uint64_t H = (uint64_t)P.H, N = (uint64_t)P.xworld;
    int64_t p = (int64_t)(((uint64_t)h * N) / H);
    while (p + 1 < (int64_t)N && (H * (uint64_t)(p + 1)) / N <= h) p++;
    while (p > 0 && (H * (uint64_t)p) / N > h) p--;
    return (int32_t)p;
}

// --------------------------------------------------------------- profiling
// Built with -DSHD_PROF (make prof -> libshdgpu_prof.so, scripts/prof_round.py):
// per-thread shader-clock totals per phase, summed and max-reduced into g_prof.
enum {
    PR_TOTAL, PR_LOAD, PR_MERGE, PR_POP, PR_EXEC_PKT, PR_EXEC_NOTIFY, PR_EXEC_REFILL, PR_EXEC_OTHER, PR_PICK,
    PR_SEND, PR_STORE, PR_NEV, PR_N
};
#ifdef SHD_TIMING
// -DSHD_TIMING (make timing -> libshdgpu_tim.so, scripts/round_timing.py):
// wall-clock stamps per block at the round's phase boundaries, 64 round slots
// keyed by the summary address x 2048 blocks x 8 stamps
__device__ unsigned long long g_tim[64][2048][20];
// per event class, over iterations in which every lane that starts an event
// starts one of that class: {iterations, cycles, of which take_next, of which
// begin_event}.  Class = kind (1..7), 8 = a packet on the general path
__device__ unsigned long long g_kc[10][4];
// event-path counters (timing build): cq / tq entries loaded from HBM, heap
// pushes / pops, inbox events merged, events, flushes, suspended lanes
__device__ unsigned long long g_cnt[8];
#ifdef SHD_TIMING_LIGHT   // phase stamps only: no per-event counters either
#define TCNT(i)
#else
#define TCNT(i) atomicAdd(&g_cnt[i], 1ull)
#endif
__shared__ unsigned long long s_kc[10][4];
#ifdef SHD_TIMING_NOWAIT   // stamps when the wave gets there, without draining its memory ops
#define TIM_WAIT()
#else
#define TIM_WAIT() asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory")
#endif
#define TIM(k)                                                                                         \
    do {                                                                                               \
        TIM_WAIT();                                                                                    \
        if (threadIdx.x == 0 && blockIdx.x < 2048)                                                     \
            g_tim[((uintptr_t)P.sum / sizeof(DevSummary)) & 63][blockIdx.x][k] = wall_clock64();       \
    } while (0)
// inside a divergent region: the first active lane stamps
#define TIMA(k)                                                                                        \
    do {                                                                                               \
        TIM_WAIT();                                                                                    \
        if ((int)threadIdx.x == __ffsll((unsigned long long)__ballot(1)) - 1 && blockIdx.x < 2048)     \
            g_tim[((uintptr_t)P.sum / sizeof(DevSummary)) & 63][blockIdx.x][k] = wall_clock64();       \
    } while (0)
#define TIMV(k, v)                                                                                     \
    do {                                                                                               \
        if ((int)threadIdx.x == __ffsll((unsigned long long)__ballot(1)) - 1 && blockIdx.x < 2048)     \
            g_tim[((uintptr_t)P.sum / sizeof(DevSummary)) & 63][blockIdx.x][k] = (v);                  \
    } while (0)
#else
#define TIM(k)
#define TIMA(k)
#define TIMV(k, v)
#define TCNT(i)
#endif
#ifdef SHD_PROF
__device__ unsigned long long g_prof[2 * PR_N + 2];
// per-round wave timing (100 MHz wall clock), 128 round slots keyed by the
// summary address: min start, max end, max wave duration, sum of durations,
// waves, max events of a lane, sum over waves of the wave's max lane events
__device__ unsigned long long g_wave[128][8];
struct ProfAcc {
    unsigned long long v[PR_N] = {};
};
#define PROF_T0(name) const unsigned long long name = clock64();
#define PROF_ADD(c, i, t0) (c).prof.v[i] += clock64() - (t0);
#else
#define PROF_T0(name)
#define PROF_ADD(c, i, t0)
#endif

// --------------------------------------------------------------- RNG
__device__ __forceinline__ int32_t rand_r_dev(uint32_t& x) {
    uint32_t r;
    x = x * 1103515245u + 12345u;
    r = (x >> 16) & 2047u;
    x = x * 1103515245u + 12345u;
    r = (r << 10) ^ ((x >> 16) & 1023u);
    x = x * 1103515245u + 12345u;
    r = (r << 10) ^ ((x >> 16) & 1023u);
    return (int32_t)r;
}

// --------------------------------------------------------------- per-host context
// Params fields the event code reads on every event, held in registers.
// Read through the Params pointer, they are invariant loads, which the
// compiler re-issues (a scalar load and its wait) at each use rather than
// keep; launder() makes each a VGPR value it must keep.
struct HotK {
    uint64_t end_time, boot_end;
    uint32_t pkt_len, cq_cap, tq_cap, evq_cap;
    uint32_t feat;   // F_* (wave-uniform, held in an SGPR)
};
template <class T>
__device__ __forceinline__ T launder(T x) {
#ifndef SHD_NO_LAUNDER
    asm volatile("" : "+v"(x));
#endif
    return x;
}
// the same for a wave-uniform value, kept in an SGPR: branches on it are
// scalar branches, so a feature that is off costs a compare and a jump, and
// the loads behind it are skipped rather than issued under an empty exec mask
__device__ __forceinline__ uint32_t launder_s(uint32_t x) {
    asm volatile("" : "+s"(x));
    return x;
}

struct HostCtx {
    HotK k;
    int32_t l;       // local index
    uint32_t h;      // global host id
    uint64_t now;
    uint32_t rng;
    uint64_t ev_seq;
    uint32_t pkt_seq;
    uint64_t rx_rem, tx_rem;
    uint32_t rx_refill, tx_refill;
    uint32_t flags;
    uint32_t unread;
    uint64_t cq_total, cq_iexp, cq_ndrop;
    uint32_t cq_dc, cq_dcl, cq_head, cq_count;
    uint32_t tq_head, tq_count;
    uint32_t evq_n;
    uint64_t top_time;          // heap root's time (the root itself: s_top; valid when evq_n > 0)
    uint32_t dh, nd;            // next / count of the window's calendar events (s_due)
    uint64_t dt;                // time of the due list's head (kInf: none left)
    uint32_t ns;                // deferred sends (s_send)
    uint64_t seq_base;          // ev_seq at the last flush: IDs >= it are provisional
    int32_t self_lo, self_hi;   // loopback draws (Params::self_thr)
    int32_t dst_thr;            // draws with a destination: x <= dst_thr (this host's weights)
    uint32_t cls;               // destination-weight class
    uint32_t w_msgs;            // the executing event's remaining work (run_work): messages, W_* steps
    uint32_t w_fl;
    uint64_t tt0, tt1, tt2;     // timer times (kInf = empty): heartbeat, refill, notify
    uint64_t ts0, ts1, ts2;     // timer event IDs
    bool cq_hv, tq_hv;          // FIFO head entries held in LDS (s_cqh, s_tqh), not yet stored
    int32_t att;                // this host's attached-vertex index
    uint32_t c_events, c_pkt, c_sent, c_idrop, c_cdrop, c_recv;   // this round's counter deltas
    uint32_t if_in, if_out;     // HostRec::if_in / if_out
    // current executing event key (for first-touch logging)
    uint64_t q_seq;
    uint32_t q_src;
    uint32_t q_sub;
    uint64_t min_emit;   // min time of events sent to other hosts
    uint64_t ws;         // the round's window start (calendar append horizon)
    uint32_t ws_mod;     // ws % 1 ms (refill alignment)
    int np;              // the next round's inbox parity
    uint32_t xwi;        // peer-to-peer: this round's receive-block parity
    uint32_t xput;       // peer-to-peer: this lane stored into a peer's receive block
    uint32_t err;
    uint32_t n_pend;
#ifdef SHD_PROF
    ProfAcc prof;
#endif
};

constexpr uint32_t W_RX = 1u, W_TX = 2u, W_REFILL = 4u, W_SENDING = 8u, W_READ = 16u;   // HostCtx::w_fl (W_READ: the messages answer reads)

// per-lane LDS of the round kernel (one wave per block; [slot][lane] layouts)
__shared__ shd_event s_top[kBlock];              // heap root
__shared__ shd_event s_due[kDueCap * kBlock];    // the window's calendar events, sorted
// fused peer-to-peer rounds: events received for the window itself, per host
// (they join the due list after the calendar's; round_body<true>)
constexpr int kRxCap = 2;
__shared__ shd_event s_rx[kRxCap * kBlock];
__shared__ uint32_t s_rxn[kBlock];
__shared__ CodelEnt s_cqh[kBlock];               // CoDel FIFO head
__shared__ TxEnt s_tqh[kBlock];                  // send FIFO head

__device__ __forceinline__ bool ev_less(const shd_event& a, const shd_event& b) {
    if (a.time != b.time) return a.time < b.time;
    if (a.src != b.src) return a.src < b.src;
    return a.seq < b.seq;
}

// An event held as two 16-B vectors.  Choosing between events held as
// structs lets the compiler select between their addresses, which puts
// them in scratch; selects between vector values stay in registers.
// a = {time lo, time hi, seq lo, seq hi}, b = {src, dst, pkt, kind}.
struct EvV {
    uint4 a, b;
};
static_assert(sizeof(shd_event) == 32, "EvV mirrors shd_event");
template <class T>
__device__ __forceinline__ EvV ev_ld(T* p) {
    const uint4* q = (const uint4*)p;
    return EvV{q[0], q[1]};
}
template <class T>
__device__ __forceinline__ void ev_st(T* p, const EvV& x) {
    uint4* q = (uint4*)p;
    q[0] = x.a;
    q[1] = x.b;
}
__device__ __forceinline__ uint64_t evv_time(const EvV& x) { return ((uint64_t)x.a.y << 32) | x.a.x; }
__device__ __forceinline__ uint64_t evv_seq(const EvV& x) { return ((uint64_t)x.a.w << 32) | x.a.z; }
__device__ __forceinline__ bool evv_less(const EvV& x, const EvV& y) {
    const uint64_t tx = evv_time(x), ty = evv_time(y);
    if (tx != ty) return tx < ty;
    if (x.b.x != y.b.x) return x.b.x < y.b.x;
    return evv_seq(x) < evv_seq(y);
}
__device__ __forceinline__ EvV evv_sel(bool c, const EvV& x, const EvV& y) {
    EvV r;
    r.a.x = c ? x.a.x : y.a.x; r.a.y = c ? x.a.y : y.a.y; r.a.z = c ? x.a.z : y.a.z; r.a.w = c ? x.a.w : y.a.w;
    r.b.x = c ? x.b.x : y.b.x; r.b.y = c ? x.b.y : y.b.y; r.b.z = c ? x.b.z : y.b.z; r.b.w = c ? x.b.w : y.b.w;
    return r;
}

// 4-ary min-heap; the slab's entry 3 is the root, so the four children of
// node i (4i+1 .. 4i+4) fill one aligned 128-B line.  The root is cached in
// LDS (s_top) and its time in a register: peeking never touches HBM.
__device__ __forceinline__ shd_event* heap_base(const DParams& P, const HostCtx& c) {
    return P.evq + (size_t)c.l * P.evq_stride + 3;
}

// (e by value: an event passed by reference into global memory is loaded
// once, and its time is consumed here, not left pending into the event loop)
__device__ void heap_push(const DParams& P, HostCtx& c, const shd_event e_in) {
    TCNT(2);
    shd_event e = e_in;
    e.time = launder(e.time);
    shd_event* hp = heap_base(P, c);
    if (c.evq_n >= c.k.evq_cap) { c.err |= SHD_ERR_EVQ_OVERFLOW; return; }
    uint32_t i = c.evq_n++;
    if (i == 0) {
        hp[0] = e;
        s_top[threadIdx.x] = e;
        c.top_time = e.time;
        return;
    }
    if (e.time <= c.top_time && ev_less(e, s_top[threadIdx.x])) {   // it will end at the root
        s_top[threadIdx.x] = e;
        c.top_time = e.time;
    }
    while (i > 0) {
        const uint32_t p = (i - 1) >> 2;
        const shd_event pe = hp[p];
        if (!ev_less(e, pe)) break;
        hp[i] = pe;
        i = p;
    }
    hp[i] = e;
}

// remove the root; the new root is re-cached.  The four children are read
// whole (an index past the end rereads the last entry and never wins)
__device__ void heap_pop(const DParams& P, HostCtx& c) {
    TCNT(3);
    shd_event* hp = heap_base(P, c);
    const uint32_t n = --c.evq_n;
    if (n == 0) return;
    const EvV last = ev_ld(hp + n);
    uint32_t i = 0;
    for (;;) {
        const uint32_t c1 = 4 * i + 1;
        if (c1 >= n) break;
        uint32_t m = c1;
        EvV me = ev_ld(hp + c1);
#pragma unroll
        for (int k = 1; k < 4; k++) {
            const uint32_t ck = c1 + k < n ? c1 + k : n - 1;
            const EvV x = ev_ld(hp + ck);
            const bool lt = c1 + k < n && evv_less(x, me);
            me = evv_sel(lt, x, me);
            m = lt ? ck : m;
        }
        if (!evv_less(me, last)) break;
        ev_st(hp + i, me);
        if (i == 0) { ev_st(s_top + threadIdx.x, me); c.top_time = evv_time(me); }
        i = m;
    }
    ev_st(hp + i, last);
    if (i == 0) { ev_st(s_top + threadIdx.x, last); c.top_time = evv_time(last); }
}

__device__ __forceinline__ void trace(const DParams& P, HostCtx& c, uint64_t t, uint64_t seq, uint32_t host,
                                      uint32_t peer, uint32_t pkt, uint32_t kind) {
    if (!(c.k.feat & F_TRACE)) return;
    unsigned long long i = atomicAdd(P.trace_n, 1ull);
    if (i >= P.trace_cap) { c.err |= SHD_ERR_TRACE_OVERFLOW; return; }
    shd_trace_rec r;
    r.time = t; r.seq = seq; r.host = host; r.peer = peer; r.pkt = pkt; r.kind = kind;
    P.trace_buf[i] = r;
}

__device__ __forceinline__ bool bootstrapping(const DParams& P, const HostCtx& c) { return c.now < c.k.boot_end; }

// the tracker interval of host h (<host heartbeatfrequency>, host.c:240; the
// option default otherwise)
__device__ __forceinline__ uint64_t hb_interval(const DParams& P, uint32_t feat, uint32_t h) {
    return (feat & F_HOSTHB) ? P.host_hb[h] : P.heartbeat;
}

__device__ __forceinline__ void hot_load(const DParams& P, HostCtx& c) {
    c.k.end_time = launder(P.end_time);
    c.k.boot_end = launder(P.bootstrap_end);
    c.k.pkt_len = launder(P.pkt_len);
    c.k.cq_cap = launder(P.cq_cap);
    c.k.tq_cap = launder(P.tq_cap);
    c.k.evq_cap = launder(P.evq_cap);
    c.k.feat = launder_s(P.feat);
}

// event_new_ (consumes the source's event ID, event.c:38) + scheduler_push
// (discards time >= end, scheduler.c:346-349) for a self event
__device__ void schedule_self(const DParams& P, HostCtx& c, uint32_t kind, uint64_t delay, uint32_t pkt) {
    // heap events carry exact IDs: the send loop flushes the deferred sends
    // before a loopback send (timer slots may hold provisional IDs, fixed up
    // by the flush)
    if (kind != SHD_EV_HEARTBEAT && kind != SHD_EV_REFILL && kind != SHD_EV_NOTIFY && c.ns) c.err |= SHD_ERR_INTERNAL;
    shd_event e;
    e.time = c.now + delay;
    e.seq = c.ev_seq++;
    e.src = c.h;
    e.dst = c.h;
    e.pkt = pkt;
    e.kind = kind;
    if (e.time >= c.k.end_time) return;
    switch (kind) {   // at most one pending instance each (flags / self-rescheduling)
    case SHD_EV_HEARTBEAT:
        if (c.tt0 != kInf) c.err |= SHD_ERR_INTERNAL;
        c.tt0 = e.time; c.ts0 = e.seq;
        break;
    case SHD_EV_REFILL:
        if (c.tt1 != kInf) c.err |= SHD_ERR_INTERNAL;
        c.tt1 = e.time; c.ts1 = e.seq;
        break;
    case SHD_EV_NOTIFY:
        if (c.tt2 != kInf) c.err |= SHD_ERR_INTERNAL;
        c.tt2 = e.time; c.ts2 = e.seq;
        break;
    default:
        heap_push(P, c, e);
    }
}

// append an event of a later round to local host dl's calendar; false when it
// is beyond the horizon of the round starting at `ws` or the bin is full (the
// caller then takes the inbox).  The event is stored before the bin's bit is
// set; readers filter slots by time, so a slot claimed but not yet written
// (time still that of an older, processed event, or kInf) is never taken.
__device__ __forceinline__ bool cal_push(const DParams& P, int32_t dl, const shd_event& e, uint64_t ws) {
    if (!P.bins) return false;
    const uint64_t b = e.time >> P.bin_shift;
    if (b - (ws >> P.bin_shift) > kHorizon) return false;
    const uint32_t p = (uint32_t)b & (kNB - 1);
    const size_t bi = (size_t)dl * kNB + p;
    const uint32_t s = atomicAdd(&P.bin_n[bi], 1u);
    if (s >= kBinCap) return false;
    P.bins[bi * kBinCap + s] = e;
    atomicOr(&P.bin_bits[(size_t)dl * kNBW + (p >> 5)], 1u << (p & 31));
    return true;
}

// a 16-B write-through (system-scope) store: the line leaves every cache on
// the way (peer-to-peer receive blocks).  hipcc does not count it: its
// writers drain with an explicit s_waitcnt vmcnt(0); the s_nop keeps the
// data registers intact until the store has read them
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_sys(void* p, uint4 v) {
    const u32x4 x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
}

// deliver an inter-host event: to the destination's calendar (or inbox) for a
// later round, or to the remote outbox when it lives on another engine
// the calendar-less part of a delivery: the inbox of a local destination
// (merged into its heap next round), else the peer's all-to-all block or the
// remote outbox
__device__ void emit_nocal(const DParams& P, HostCtx& c, const shd_event& e) {
    const int32_t dl = (int32_t)e.dst - P.h0;
    if (dl >= 0 && dl < P.nloc) {
        uint32_t slot = atomicAdd(&P.inbox_n[c.np][dl], 1u);
        if (slot >= P.inbox_cap) { c.err |= SHD_ERR_INBOX_OVERFLOW; return; }
        P.inbox[c.np][(size_t)dl * P.inbox_cap + slot] = e;
    } else {
        if (P.xcnt) {   // fused peer-to-peer rounds: into the region of the destination's block
            const int32_t peer = owner_of(P, e.dst);
            const uint32_t hp0 = (uint32_t)(((uint64_t)P.H * (uint64_t)peer) / (uint64_t)P.xworld);
            const uint32_t blk = (e.dst - hp0) / (uint32_t)P.hpw;
            const size_t r = ((size_t)c.xwi * P.xworld + peer) * P.xnbx + blk;
            const uint32_t s = blk < P.xnbx ? atomicAdd(&P.xcnt[r], 1u) : kXSlots;
            if (s < P.xrcap) {
                shd_event* d = P.xpeer[peer] + P.xroff +
                               (((size_t)c.xwi * P.xworld + P.xme) * P.xnbx + blk) * kXSlots + s;
                const EvV x = ev_ld(&e);
                st16_sys(d, x.a);
                st16_sys((char*)d + 16, x.b);
                c.xput = 1;
                return;
            }
            // region full: spill (as a full block below)
        } else if (P.xsend) {   // exchange mode: straight into the peer's all-to-all block
            const int32_t peer = owner_of(P, e.dst);
            const uint32_t s = atomicAdd(&P.xcount[peer], 1u);
            if (s < P.xcap) {
                if (P.xpeer) {   // peer-to-peer: into the peer's receive block, write-through
                    shd_event* d = P.xpeer[peer] + ((size_t)c.xwi * P.xworld + P.xme) * (P.xcap + 1) + 1 + s;
                    const EvV x = ev_ld(&e);
                    st16_sys(d, x.a);
                    st16_sys((char*)d + 16, x.b);
                    c.xput = 1;
                } else {
                    P.xsend[(size_t)peer * (P.xcap + 1) + 1 + s] = e;
                }
                return;
            }
            // block full: spill to the remote buffer (the header says so, the
            // group halts after the exchange and the host delivers the spill)
        }
        unsigned long long slot = atomicAdd(&P.sum->n_remote, 1ull);
        if (slot >= P.remote_cap) { c.err |= SHD_ERR_REMOTE_OVERFLOW; return; }
        P.remote[slot] = e;
    }
}

// _networkinterface_scheduleNextRefillIfNeeded (network_interface.c:130-161),
// timeStartedRefillingBuckets = 0
__device__ void refill_if_needed(const DParams& P, HostCtx& c) {
    const bool need = (c.tx_rem < c.tx_refill + SHD_MTU) || (c.rx_rem < c.rx_refill + SHD_MTU);
    if (need && !(c.flags & F_REFILL_PENDING)) {
        // now % 1 ms from the round's ws % 1 ms and the 32-bit offset into the round
        const uint32_t off = (uint32_t)(c.now - c.ws) + c.ws_mod;
        const uint64_t until = SHD_MS - (off % (uint32_t)SHD_MS);
        schedule_self(P, c, SHD_EV_REFILL, until, 0);
        c.flags |= F_REFILL_PENDING;
    }
}
__device__ __forceinline__ void consume(uint64_t& rem, uint64_t n) { rem = (n >= rem) ? 0 : rem - n; }

// _networkinterface_receivePacket (network_interface.c:375-419)
__device__ void if_receive_packet(const DParams& P, HostCtx& c, uint32_t src, uint32_t pkt) {
    c.if_in++;   // tracker_addInputBytes (network_interface.c:415)
    if (c.flags & F_LISTENING) {
        trace(P, c, c.now, 0, c.h, src, pkt, SHD_TR_RECV);
        c.c_recv++;
        c.unread++;
        if (!(c.flags & F_NOTIFY_PENDING)) {   // epoll.c:345-365, +1 ns
            schedule_self(P, c, SHD_EV_NOTIFY, 1, 0);
            c.flags |= F_NOTIFY_PENDING;
        }
    } else {
        trace(P, c, c.now, 0, c.h, src, pkt, SHD_TR_IF_DROP);
    }
}

// ---- CoDel (router_queue_codel.c) on the per-host FIFO ----
__device__ __forceinline__ uint64_t codel_control_law(uint32_t count, uint64_t ts) {
    const uint64_t newTS = ts + kCodelInterval;
    const double result = ((double)newTS) / sqrt((double)count);
    return (uint64_t)round(result);
}

__device__ bool codel_helper(const DParams& P, HostCtx& c, bool& okToDrop, CodelEnt& out) {
    okToDrop = false;
    if (c.cq_count == 0) { c.cq_iexp = 0; return false; }
    if (c.cq_hv) {
        out = s_cqh[threadIdx.x];
        c.cq_hv = false;
    } else {
        out = P.cq[(size_t)c.l * c.k.cq_cap + c.cq_head];
        TCNT(0);
    }
    c.cq_head = (c.cq_head + 1 == c.k.cq_cap) ? 0 : c.cq_head + 1;
    c.cq_count--;
    c.cq_total -= c.k.pkt_len;
    const uint64_t sojourn = c.now - out.ts;
    if (sojourn < kCodelTarget || c.cq_total < SHD_MTU) {
        c.cq_iexp = 0;
    } else {
        if (c.cq_iexp == 0) c.cq_iexp = c.now + kCodelInterval;
        else if (c.now >= c.cq_iexp) okToDrop = true;
    }
    return true;
}

__device__ __forceinline__ void codel_drop(const DParams& P, HostCtx& c, const CodelEnt& e) {
    trace(P, c, c.now, 0, c.h, e.src, e.pkt, SHD_TR_CODEL_DROP);
    c.c_cdrop++;
}

__device__ bool codel_dequeue(const DParams& P, HostCtx& c, CodelEnt& out) {
    bool okToDrop = false;
    CodelEnt pkt;
    bool have = codel_helper(P, c, okToDrop, pkt);
    if (!have) { c.flags &= ~F_CODEL_DROP_MODE; return false; }
    if (c.flags & F_CODEL_DROP_MODE) {
        if (!okToDrop) c.flags &= ~F_CODEL_DROP_MODE;
        while (c.now >= c.cq_ndrop && (c.flags & F_CODEL_DROP_MODE)) {
            codel_drop(P, c, pkt);
            c.cq_dc++;
            have = codel_helper(P, c, okToDrop, pkt);
            if (okToDrop) c.cq_ndrop = codel_control_law(c.cq_dc, c.cq_ndrop);
            else c.flags &= ~F_CODEL_DROP_MODE;
        }
    } else if (okToDrop) {
        codel_drop(P, c, pkt);
        have = codel_helper(P, c, okToDrop, pkt);
        c.flags |= F_CODEL_DROP_MODE;
        const uint32_t delta = c.cq_dc - c.cq_dcl;
        c.cq_dc = 1;
        const bool recently = c.now < c.cq_ndrop + 16 * kCodelInterval;
        if (recently && delta > 1) c.cq_dc = delta;
        c.cq_ndrop = codel_control_law(c.cq_dc, c.now);
        c.cq_dcl = c.cq_dc;
    }
    if (!have) return false;
    out = pkt;
    return true;
}

// networkinterface_receivePackets (network_interface.c:421-455)
__device__ void if_receive_packets(const DParams& P, HostCtx& c) {
    const bool boot = bootstrapping(P, c);
    while (boot || c.rx_rem >= SHD_MTU) {
        CodelEnt p;
        if (!codel_dequeue(P, c, p)) break;
        if_receive_packet(P, c, p.src, p.pkt);
        if (!boot) {
            consume(c.rx_rem, c.k.pkt_len);
            refill_if_needed(P, c);
        }
    }
}

// ---- path value with the first-touch rule ----
struct PathVal {
    double lat, rel;
    double lat2, rel2;   // second candidate when unresolved
    bool resolved;
    bool log;            // the query must be logged for rank assignment
};

// the raw candidates of a path value, loaded in one round trip (the mode
// branches are uniform: kernel parameters); path_select applies the rank rule
struct PathRaw {
    shd_pv d, v1, v2;   // direct; row[a][b] (a == b: row[a][a]); row[b][a] (a == b: self[a])
    int32_t rb, rs;     // rank[b], self_rank[a] (a == b)
    uint32_t adj;
};

__device__ __forceinline__ void path_load(const DParams& P, int32_t a, int32_t b, PathRaw& x) {
    const size_t ab = (size_t)a * P.T + b, ba = (size_t)b * P.T + a;
    x.adj = 0; x.rb = kNoRank; x.rs = kNoRank;
    if (P.complete) { x.d = P.dir[ab]; return; }
    if (P.prefer_direct) { x.adj = P.adj[ab]; x.d = P.dir[ab]; }
    x.v1 = P.row[ab];
    if (a == b) {
        x.rs = P.self_rank[a];
        x.v2 = P.self[a];
    } else {
        x.rb = P.rank[b];
        x.v2 = P.row[ba];
    }
}

// the same candidates for the flush, every load unconditional (indices of
// tables the mode does not use point at entry 0): no branch between loads,
// so all of them are in flight together (one memory round trip).  The
// direct-edge table and the rank arrays are always allocated; row falls
// back to dir when there are no rows (complete graphs, which never use it)
__device__ __forceinline__ void path_load_flat(const DParams& P, int32_t a, int32_t b, PathRaw& x) {
    const size_t ab = (size_t)a * P.T + b, ba = (size_t)b * P.T + a;
    const bool use_dir = P.complete || P.prefer_direct, use_rows = !P.complete;
    const size_t i_d = use_dir ? ab : 0, i_ab = use_rows ? ab : 0, i_ba = use_rows ? ba : 0;
    const shd_pv* rowp = P.row ? (const shd_pv*)P.row : (const shd_pv*)P.dir;
    shd_pv d = P.dir[i_d];
    uint32_t adj = P.adj[i_d];
    shd_pv v1 = rowp[i_ab], v2 = rowp[i_ba], vs = P.self[a];
    int32_t rb = P.rank[b], rs = P.self_rank[a];
    // consumed here, all together: left to the compiler, each load would be
    // sunk into the branch of path_select that uses it, one round trip each
    d.lat = launder(d.lat); d.rel = launder(d.rel); adj = launder(adj);
    v1.lat = launder(v1.lat); v1.rel = launder(v1.rel); v2.lat = launder(v2.lat); v2.rel = launder(v2.rel);
    vs.lat = launder(vs.lat); vs.rel = launder(vs.rel); rb = launder(rb); rs = launder(rs);
    x.d = d;
    x.adj = P.prefer_direct ? adj : 0u;
    x.v1 = v1;
    x.v2 = a == b ? vs : v2;
    x.rb = a == b ? kNoRank : rb;
    x.rs = a == b ? rs : kNoRank;
}

__device__ __forceinline__ PathVal path_select(const DParams& P, int32_t a, int32_t b, int32_t ra, const PathRaw& x) {
    PathVal v;
    v.resolved = true;
    v.log = false;
    if (P.complete || (P.prefer_direct && x.adj)) {
        v.lat = x.d.lat; v.rel = x.d.rel;
        return v;
    }
    if (a == b) {
        const shd_pv& sp = x.v2;   // self[a]
        const shd_pv& r = x.v1;    // row[a][a]
        if (ra == kNoRank && x.rs == kNoRank) {
            v.resolved = false; v.log = true;
            v.lat = sp.lat; v.rel = sp.rel;
            v.lat2 = r.lat; v.rel2 = r.rel;
        } else if (x.rs < ra) {
            v.lat = sp.lat; v.rel = sp.rel;
        } else {
            v.lat = r.lat; v.rel = r.rel;
        }
        return v;
    }
    if (ra == kNoRank && x.rb == kNoRank) {
        v.resolved = false; v.log = true;
        v.lat = x.v1.lat; v.rel = x.v1.rel;
        v.lat2 = x.v2.lat; v.rel2 = x.v2.rel;
        return v;
    }
    if (P.directed && ra == kNoRank) v.log = true;   // row a still runs (directed rerun rule)
    const shd_pv& w = ra < x.rb ? x.v1 : x.v2;
    v.lat = w.lat; v.rel = w.rel;
    return v;
}

// the cached entry a served send counted against (topology.c:2053-2063): the
// row of the lower rank (the entry stored first, write-once per pair), the
// pair's direct entry (one per unordered pair), or the vertex's own entry
__device__ __forceinline__ size_t path_key(const DParams& P, int32_t a, int32_t b, int32_t ra, int32_t rb, uint32_t adj) {
    const int32_t lo = a < b ? a : b, hi = a < b ? b : a;
    if (P.complete || (P.prefer_direct && adj) || a == b) return (size_t)lo * P.T + hi;
    return ra < rb ? (size_t)a * P.T + b : (size_t)b * P.T + a;
}

__device__ PathVal path_value(const DParams& P, int32_t a, int32_t b) {
    PathRaw x;
    const int32_t ra = P.complete ? kNoRank : P.rank[a];
    path_load(P, a, b, x);
    return path_select(P, a, b, ra, x);
}

__device__ void log_pending(const DParams& P, HostCtx& c, const SendRec& q, int32_t a, int32_t b, uint32_t delivered,
                            uint32_t dst, uint64_t seq) {
    unsigned long long i = atomicAdd(&P.sum->n_pending, 1ull);
    c.n_pend++;
    if (i >= P.pend_cap) { c.err |= SHD_ERR_PENDING_OVERFLOW; return; }
    Pending r;
    r.qtime = q.now; r.qseq = q.q_seq; r.qhost = c.h; r.qsrc = q.q_src; r.qsub = q.q_sub & 0x7FFFFFFFu;
    r.a = (uint32_t)a; r.b = (uint32_t)b; r.delivered = delivered; r.dst = dst; r.pkt = q.pkt; r.seq = seq;
    P.pend[i] = r;
}

// LDS of the round kernel (one wave per block; [slot][lane] layouts)
__shared__ SendRec s_send[kSendCap * kBlock];    // deferred sends
__shared__ shd_event s_res[kSendCap * kBlock];   // flush: resolved sends, then the events to deliver
__shared__ uint16_t s_idx[kSendCap * kBlock];    // flush: record -> (lane << 4) | slot
__shared__ int32_t s_att[kBlock];                // flush: each lane's attached vertex
__shared__ uint32_t s_cls[kBlock];               // flush: each lane's destination-weight class

// loopback test of a destination draw (network_interface.c:548-555): the
// first i with dest_cum[i] >= r = x / RAND_MAX is this host, i.e.
// dest_cum[h-1] < r <= dest_cum[h]; r is monotone in x, so that is an
// interval of x, precomputed on the host with the same division
__device__ __forceinline__ bool is_self_draw(const HostCtx& c, uint32_t rv) {
    return (int32_t)rv >= c.self_lo && (int32_t)rv <= c.self_hi;
}

// _phold_chooseNode (test_phold.c:160-178): the first i with dest_cum[i] >= r.
// guide[k] is a lower bound of it for any k <= r*H - 1; for even weights the
// answer is one of the next three entries (their attached index inline), else
// a binary search finishes the job.  Only called for draws r <= dest_cum[H-1].
__device__ __forceinline__ uint32_t guide_index(const DParams& P, double r) {
    int32_t k = (int32_t)(r * (double)P.H) - 1;
    return (uint32_t)(k < 0 ? 0 : (k > P.H - 1 ? P.H - 1 : k));
}
__device__ __forceinline__ double u2d(uint32_t lo, uint32_t hi) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// the guide entry is passed as its three 16-B vectors (a struct chosen from
// by index would be put in scratch): g0 = {i, att[0..2]}, g1 = {cum[0], cum[1]},
// g2 = {cum[2], pad}
template <class CumPtr>
__device__ __forceinline__ void guide_pick(const DParams& P, CumPtr cum, uint4 g0, uint4 g1, uint4 g2, double r,
                                           int32_t& dst, int32_t& att) {
    const bool f0 = u2d(g1.x, g1.y) >= r, f1 = u2d(g1.z, g1.w) >= r, f2 = u2d(g2.x, g2.y) >= r;
    if (f0 || f1 || f2) {
        dst = (int32_t)g0.x + (f0 ? 0 : f1 ? 1 : 2);
        att = (int32_t)(f0 ? g0.y : f1 ? g0.z : g0.w);
        return;
    }
    int32_t lo = (int32_t)g0.x + 3, hi = P.H;
    while (lo < hi) {
        const int32_t mid = lo + ((hi - lo) >> 1);
        if (cum[mid] >= r) hi = mid; else lo = mid + 1;
    }
    dst = lo;
    att = P.host_att[lo];
}

// worker_sendPacket (worker.c:260-321), deferred: the reliability draw is
// made now (it is drawn for every non-loopback send, worker.c:286); the
// path lookup, the drop decision and the delivery happen at the next flush
__device__ void worker_send_deferred(const DParams& P, HostCtx& c, uint32_t rv, uint32_t pkt) {
    const uint32_t chance = (uint32_t)rand_r_dev(c.rng);
    SendRec q;
    q.now = c.now; q.q_seq = c.q_seq; q.q_src = c.q_src;
    q.pseq = (uint32_t)(c.ev_seq - c.seq_base);
    q.r = rv; q.chance = chance; q.pkt = pkt;
    q.q_sub = (c.q_sub++ & 0x7FFFFFFFu) | (bootstrapping(P, c) ? 0x80000000u : 0u);
    s_send[c.ns * kBlock + threadIdx.x] = q;
    c.ns++;
    c.ev_seq++;   // provisional: a dropped send gives its ID back at the flush
    c.if_out++;   // tracker_addOutputBytes (network_interface.c:571)
}

// Resolve every lane's deferred sends together.  Called by all lanes of the
// wave (convergent; lanes with no host have ns = 0).  Record-parallel: each
// lane picks the destination and looks up the path of one send (one memory
// round trip each per 64 sends of the wave); then each host walks its own
// sends in order (event IDs, counters, traces, first-touch logs, LDS only);
// then record-parallel deliveries (one round trip for the calendar claims).
// a delivery of the round's last flush whose calendar claim is in flight:
// its store waits until the round's closing work is issued (flush_finish)
struct PendDel {
    uint64_t bi;     // bin index
    uint32_t slot;   // claimed slot (kind 1)
    uint32_t kind;   // 0 none, 1 calendar claim issued, 2 inbox / remote
};

__device__ __forceinline__ void flush_wave(const DParams& P, HostCtx& c, bool defer, PendDel& pd) {
    pd.kind = 0;
    const uint32_t lane = threadIdx.x;
    const uint32_t n = c.ns;
    uint32_t pre = n;   // inclusive, then exclusive prefix of the lanes' counts
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(pre, off, 64);
        if ((int)lane >= off) pre += o;
    }
    const uint32_t total = __shfl(pre, 63, 64);
    pre -= n;
    if (total == 0) return;
    const bool one = defer && total <= (uint32_t)kBlock;   // the round's last flush, one batch
    for (uint32_t i = 0; i < n; i++) s_idx[pre + i] = (uint16_t)((lane << 4) | i);
    s_att[lane] = c.att;
    s_cls[lane] = c.cls;
    __syncthreads();
#ifdef SHD_TIMING_LIGHT
    TIM(12);
#endif
    uint32_t err = 0;
    for (uint32_t base = 0; base < total; base += kBlock) {
        const uint32_t r = base + lane;
        if (r >= total) continue;
        const uint32_t id = s_idx[r];
        const uint32_t hl = id >> 4, i = id & 15u;
        const SendRec q = s_send[i * kBlock + hl];
        const int32_t a = s_att[hl];
        int32_t dst, b;
        if (P.dest_closed) {   // no table: one memory round trip fewer
            const uint64_t nx = (uint64_t)q.r * (uint64_t)(uint32_t)P.H;
            const uint64_t cx = (nx + 2147483646ull) / 2147483647ull;
            int32_t d = cx ? (int32_t)cx - 1 : 0;
#pragma unroll
            for (int j = 0; j < kDestExc; j++)   // unrolled: the list is read in one scalar batch
                d = (j < P.n_exc && (int32_t)q.r == P.exc_x[j]) ? P.exc_d[j] : d;
            dst = d;
            b = d;
        } else {
            const double rr = (double)q.r / kRandMax;
            const size_t row = (size_t)s_cls[hl] * (size_t)P.H;
            const uint4* gq = (const uint4*)(P.dest_guide + row + guide_index(P, rr));
            const uint4 g0 = gq[0], g1 = gq[1], g2 = gq[2];
            guide_pick(P, P.dest_cum + row, g0, g1, g2, rr, dst, b);
        }
        PathRaw x;
        int32_t ra_l = P.rank[a];
        path_load_flat(P, a, b, x);
        ra_l = launder(ra_l);
        const int32_t ra = P.complete ? kNoRank : ra_l;
        const PathVal pv = path_select(P, a, b, ra, x);
        const double chance = (double)q.chance / kRandMax;
        const bool boot = (q.q_sub >> 31) != 0;
        const bool pass = boot || chance <= pv.rel || P.payload == 0;
        if (!pv.resolved) {
            const bool pass2 = boot || chance <= pv.rel2 || P.payload == 0;
            if (pass != pass2 || (c.k.feat & F_AMBIG)) err |= SHD_ERR_AMBIGUOUS;
        }
        if ((c.k.feat & F_PCOUNT) && pass && pv.resolved) atomicAdd(&P.pcount[path_key(P, a, b, ra, x.rb, x.adj)], 1u);
        shd_event e;
        e.time = q.now + (uint64_t)ceil(pv.lat * (double)SHD_MS);
        e.seq = 0;
        e.src = (uint32_t)b;   // the destination's attached index, for the first-touch log
        e.dst = (uint32_t)dst;
        e.pkt = 0;
        e.kind = (pass ? 1u : 0u) | (pv.log ? 2u : 0u) | (pv.resolved ? 4u : 0u);
        s_res[r] = e;
        // the round's last flush (one batch: record r is lane r's): the
        // calendar claim goes out now, under the per-host walk and the
        // round's closing work; the store follows in flush_finish
        if (one && pass && pv.resolved && e.time < c.k.end_time) {
            const int32_t dl = (int32_t)dst - P.h0;
            const uint64_t bb = e.time >> P.bin_shift;
            pd.kind = 2;
            if (P.bins && dl >= 0 && dl < P.nloc && bb - (c.ws >> P.bin_shift) <= kHorizon) {
                pd.bi = (size_t)dl * kNB + ((uint32_t)bb & (kNB - 1));
                pd.slot = atomicAdd(&P.bin_n[pd.bi], 1u);
                pd.kind = 1;
            }
        }
    }
    __syncthreads();
#ifdef SHD_TIMING_LIGHT
    TIM(13);
#endif
    // per host, in send order (worker.c:286-320)
    uint32_t failmask = 0, nfail = 0;
    for (uint32_t i = 0; i < n; i++) {
        shd_event e = s_res[pre + i];
        const SendRec q = s_send[i * kBlock + lane];
        const bool pass = e.kind & 1u, log = (e.kind & 2u) != 0, resolved = (e.kind & 4u) != 0;
        const int32_t b = (int32_t)e.src;
        uint32_t emit = 0;
        if (pass) {
            const uint64_t seq = c.seq_base + q.pseq - nfail;
            trace(P, c, q.now, seq, c.h, e.dst, q.pkt, SHD_TR_SENT);
            c.c_sent++;
            // 1 = delivery waits for the resolution, 2 = already delivered
            if (log) log_pending(P, c, q, c.att, b, resolved ? 2u : 1u, e.dst, seq);
            if (resolved && e.time < c.k.end_time) {   // scheduler_push drops time >= end
                emit = SHD_EV_PACKET;
                if (e.time < c.min_emit) c.min_emit = e.time;
            }
            e.seq = seq;
        } else {
            trace(P, c, q.now, 0, c.h, e.dst, q.pkt, SHD_TR_INET_DROP);
            c.c_idrop++;
            if (log) log_pending(P, c, q, c.att, b, 0u, e.dst, 0);
            failmask |= 1u << i;
            nfail++;
        }
        e.src = c.h;
        e.pkt = q.pkt;
        e.kind = emit;
        s_res[pre + i] = e;
    }
    if (nfail) {
        // timers scheduled since the last flush hold provisional IDs: an ID
        // x loses the dropped sends issued before it
        uint64_t f0 = 0, f1 = 0, f2 = 0;
        const bool p0 = c.tt0 != kInf && c.ts0 >= c.seq_base, p1 = c.tt1 != kInf && c.ts1 >= c.seq_base,
                   p2 = c.tt2 != kInf && c.ts2 >= c.seq_base;
        if (p0 || p1 || p2) {
            for (uint32_t i = 0; i < n; i++) {
                if (!((failmask >> i) & 1u)) continue;
                const uint64_t xi = c.seq_base + s_send[i * kBlock + lane].pseq;
                f0 += xi < c.ts0; f1 += xi < c.ts1; f2 += xi < c.ts2;
            }
            if (p0) c.ts0 -= f0;
            if (p1) c.ts1 -= f1;
            if (p2) c.ts2 -= f2;
        }
        c.ev_seq -= nfail;
    }
    c.seq_base = c.ev_seq;
    c.ns = 0;
    __syncthreads();
#ifdef SHD_TIMING_LIGHT
    TIM(14);
#endif
    // deliveries: calendar claims for 64 events at a time, then the stores.
    // The round's last flush (one batch) only issues the claims; the stores
    // follow the round's closing work, which hides the claims' round trip.
    if (one) {   // claims already issued in the resolve loop
        c.err |= err;
        return;   // s_res[lane] stays for flush_finish
    }
    for (uint32_t base = 0; base < total; base += kBlock) {
        const uint32_t r = base + lane;
        if (r >= total) continue;
        const shd_event e = s_res[r];
        if (!e.kind) continue;
        const int32_t dl = (int32_t)e.dst - P.h0;
        const uint64_t bb = e.time >> P.bin_shift;
        if (P.bins && dl >= 0 && dl < P.nloc && bb - (c.ws >> P.bin_shift) <= kHorizon) {
            const size_t bi = (size_t)dl * kNB + ((uint32_t)bb & (kNB - 1));
            const uint32_t slot = atomicAdd(&P.bin_n[bi], 1u);
            if (slot < kBinCap) {
                P.bins[bi * kBinCap + slot] = e;
                const uint32_t p = (uint32_t)bb & (kNB - 1);
                atomicOr(&P.bin_bits[(size_t)dl * kNBW + (p >> 5)], 1u << (p & 31));
                continue;
            }
        }
        emit_nocal(P, c, e);
    }
    c.err |= err;
    __syncthreads();   // s_res / s_idx are reused by the next flush
}

// the stores of the round's last flush (after its claims returned)
__device__ __forceinline__ void flush_finish(const DParams& P, HostCtx& c, const PendDel& pd) {
    if (pd.kind == 0) return;
    const shd_event e = s_res[threadIdx.x];
    if (pd.kind == 1 && pd.slot < kBinCap) {
        P.bins[pd.bi * kBinCap + pd.slot] = e;
        const uint32_t p = (uint32_t)(pd.bi & (kNB - 1));
        const int32_t dl = (int32_t)e.dst - P.h0;
        atomicOr(&P.bin_bits[(size_t)dl * kNBW + (p >> 5)], 1u << (p & 31));
        return;
    }
    emit_nocal(P, c, e);
}

// _networkinterface_sendPackets (network_interface.c:519-579), FIFO qdisc.
// Returns true when it stopped early for a flush of the deferred sends (the
// buffer is full, or the next send is a loopback, whose trace and event take
// the exact event ID); the caller flushes and calls it again.
__device__ bool if_send_step(const DParams& P, HostCtx& c) {
    const bool boot = bootstrapping(P, c);
    while (c.tx_rem >= SHD_MTU) {
        if (c.tq_count == 0) break;
        TxEnt p;
        if (c.tq_hv) {
            p = s_tqh[threadIdx.x];
        } else {
            p = P.tq[(size_t)c.l * c.k.tq_cap + c.tq_head];
            TCNT(1);
            s_tqh[threadIdx.x] = p;   // keep the peeked head: a flush may come first
            c.tq_hv = true;
        }
        const bool self = is_self_draw(c, p.r);
        if (c.ns && (self || c.ns == (uint32_t)kSendCap)) return true;
        c.tq_hv = false;
        c.tq_head = (c.tq_head + 1 == c.k.tq_cap) ? 0 : c.tq_head + 1;
        c.tq_count--;
        if (self) {
            trace(P, c, c.now, c.ev_seq, c.h, c.h, p.pkt, SHD_TR_LOCAL);
            c.if_out++;
            schedule_self(P, c, SHD_EV_LOCAL, 1, p.pkt);
        } else {
            PROF_T0(ts)
            worker_send_deferred(P, c, p.r, p.pkt);
            PROF_ADD(c, PR_SEND, ts)
        }
        if (!boot) {
            consume(c.tx_rem, c.k.pkt_len);
            refill_if_needed(P, c);
        }
    }
    return false;
}

// _host_getRandomPort / _host_getRandomFreePort (host.c:1058-1110).
// The draw lands in [MIN_RANDOM_PORT, 65535], never on the listener, so
// exactly one rand_r step triple is consumed and its value is not needed.
static_assert(SHD_PHOLD_LISTEN_PORT < SHD_MIN_RANDOM_PORT, "a random port never hits the listener");
__device__ __forceinline__ void random_free_port(HostCtx& c) { (void)rand_r_dev(c.rng); }
// the same draw, with the port it makes (the status trace records it):
// round(nextDouble * (65535 - MIN_RANDOM_PORT)) + MIN_RANDOM_PORT
__device__ __forceinline__ uint32_t random_free_port_value(HostCtx& c) {
    const int32_t v = rand_r_dev(c.rng);
    const double pick = rint((double)v / 2147483647.0 * (double)(65535u - SHD_MIN_RANDOM_PORT));
    return (uint32_t)(uint16_t)((uint16_t)pick + (uint16_t)SHD_MIN_RANDOM_PORT);
}
// the application's side of a datagram (SHD_QF_TRACE_STATUS): the bind's port
// draw and the SND_CREATED record, or the plain draw
__device__ __forceinline__ void bind_and_create(const DParams& P, HostCtx& c, uint32_t pkt) {
    if (c.k.feat & F_STATUS) {
        const uint32_t port = random_free_port_value(c);
        trace(P, c, c.now, port, c.h, ~0u, pkt, SHD_TR_CREATED);
    } else {
        random_free_port(c);
    }
}
__device__ __forceinline__ void app_read(const DParams& P, HostCtx& c) {
    if ((c.k.feat & F_STATUS) && (c.w_fl & W_READ)) trace(P, c, c.now, 0, c.h, ~0u, ~0u, SHD_TR_READ);
}

// _phold_sendNewMessage (test_phold.c:218-230) up to the socket send: draw
// the destination (resolved at the flush; only whether one exists matters
// here), bind, queue the datagram; false when nothing was queued
__device__ bool enqueue_new_message(const DParams& P, HostCtx& c) {
    PROF_T0(tp)
    const uint32_t rv = (uint32_t)rand_r_dev(c.rng);
    PROF_ADD(c, PR_PICK, tp)
    if ((int32_t)rv > c.dst_thr) return false;   // no i with dest_cum[i] >= r
    bind_and_create(P, c, c.pkt_seq);
    const uint32_t pkt = c.pkt_seq++;
    if (c.tq_count >= c.k.tq_cap) { c.err |= SHD_ERR_TXQ_OVERFLOW; return false; }
    if (c.tq_count == 0) {
        s_tqh[threadIdx.x] = TxEnt{rv, pkt};
        c.tq_hv = true;
    } else {
        uint32_t tail = c.tq_head + c.tq_count;
        if (tail >= c.k.tq_cap) tail -= c.k.tq_cap;
        P.tq[(size_t)c.l * c.k.tq_cap + tail] = TxEnt{rv, pkt};
    }
    c.tq_count++;
    return true;
}

// _networkinterface_refillTokenBucketsCB (network_interface.c:163-183)
__device__ void refill_cb(const DParams& P, HostCtx& c) {
    c.flags &= ~F_REFILL_PENDING;
    c.rx_rem += c.rx_refill;
    if (c.rx_rem > c.rx_refill + SHD_MTU) c.rx_rem = c.rx_refill + SHD_MTU;
    c.tx_rem += c.tx_refill;
    if (c.tx_rem > c.tx_refill + SHD_MTU) c.tx_rem = c.tx_refill + SHD_MTU;
    if_receive_packets(P, c);
    if (if_send_step(P, c)) c.err |= SHD_ERR_INTERNAL;   // boot: nothing queued, nothing deferred
    refill_if_needed(P, c);
}

// One event, in two parts.  begin_event does the kind-specific part and
// leaves the shared steps (CoDel dequeue + receive, message generation, the
// send loop) as work in the context; run_work runs them, so the lanes of a
// wave that execute different kinds in the same iteration converge on them.
// run_work returns early when the deferred sends need a flush (the round loop
// flushes and resumes it).  Per kind, the steps and their order are the
// reference's:
//   REFILL    refill_cb: top up, receive, send, schedule next refill
//   PACKET    router_enqueue, receive if the queue was empty
//   NOTIFY    one new message per unread datagram, each sent right away
//   APP_START `load` new messages
// The steady-state notification, straight-line: one unread datagram, an
// empty send queue with room in the send bucket and in the deferred-send
// buffer, past the bootstrap period: one new message, sent at once unless it
// draws this host (then the general send loop takes it).  The same draws and
// steps, in the same order, as the general NOTIFY path of begin_event.
__device__ __forceinline__ bool notify_fast_ok(const DParams& P, const HostCtx& c) {
    return c.unread == 1u && c.tq_count == 0 && c.tx_rem >= SHD_MTU && c.ns < (uint32_t)kSendCap &&
           !(c.k.feat & F_TRACE) && !bootstrapping(P, c);
}
__device__ __forceinline__ void notify_fast(const DParams& P, HostCtx& c) {
    c.flags &= ~F_NOTIFY_PENDING;
    c.unread = 0;
    const uint32_t rv = (uint32_t)rand_r_dev(c.rng);
    if ((int32_t)rv <= c.dst_thr) {   // else no destination: nothing queued
        random_free_port(c);
        const uint32_t pkt = c.pkt_seq++;
        if (is_self_draw(c, rv)) {   // loopback: queued; run_work sends it (after a flush)
            s_tqh[threadIdx.x] = TxEnt{rv, pkt};
            c.tq_hv = true;
            c.tq_count = 1;
            c.w_fl = W_SENDING;
        } else {
            worker_send_deferred(P, c, rv, pkt);
            consume(c.tx_rem, c.k.pkt_len);
            refill_if_needed(P, c);
        }
    }
}

// the periodic refill with both queues empty: top up; the receive loop's
// one dequeue attempt only resets CoDel's interval and drop mode, the send
// loop does nothing (as the general REFILL case of begin_event)
__device__ __forceinline__ void refill_fast(const DParams& P, HostCtx& c) {
    c.flags &= ~F_REFILL_PENDING;
    c.rx_rem += c.rx_refill;
    if (c.rx_rem > c.rx_refill + SHD_MTU) c.rx_rem = c.rx_refill + SHD_MTU;
    c.tx_rem += c.tx_refill;
    if (c.tx_rem > c.tx_refill + SHD_MTU) c.tx_rem = c.tx_refill + SHD_MTU;
    if (bootstrapping(P, c) || c.rx_rem >= SHD_MTU) {
        c.cq_iexp = 0;
        c.flags &= ~F_CODEL_DROP_MODE;
    }
    refill_if_needed(P, c);
}

__device__ void begin_event(const DParams& P, HostCtx& c, const shd_event& e) {
    TCNT(5);
    c.c_events++;
    c.q_seq = e.seq;
    c.q_src = e.src;
    c.q_sub = 0;
    c.w_msgs = 0;
    c.w_fl = 0;
#ifndef SHD_NO_EVFAST
    // The steady-state arrival, straight-line: a packet that meets an empty
    // router queue with room in the receive bucket at a listening host (no
    // tracing, past the bootstrap period) is enqueued, dequeued at once
    // (sojourn 0: CoDel's interval and drop mode reset) and received; the
    // epoll notification is scheduled at +1 ns unless one is pending (its ID
    // is consumed even when it falls past the end).  The same steps as the
    // general path below, in the same order.
    if (e.kind == SHD_EV_PACKET && c.cq_count == 0 && c.rx_rem >= SHD_MTU && (c.flags & F_LISTENING) &&
        !(c.k.feat & F_TRACE) && !bootstrapping(P, c)) {
        c.c_pkt++;
        c.c_recv++;
        c.if_in++;
        c.unread++;
        c.cq_head = (c.cq_head + 1 == c.k.cq_cap) ? 0 : c.cq_head + 1;
        c.cq_iexp = 0;
        const bool nt = !(c.flags & F_NOTIFY_PENDING);
        if (nt && c.tt2 != kInf) c.err |= SHD_ERR_INTERNAL;
        const uint64_t id = c.ev_seq, tn = c.now + 1;
        c.ev_seq += nt ? 1u : 0u;
        const bool set = nt && tn < c.k.end_time;
        c.tt2 = set ? tn : c.tt2;
        c.ts2 = set ? id : c.ts2;
        c.flags = (c.flags & ~F_CODEL_DROP_MODE) | F_NOTIFY_PENDING;
        consume(c.rx_rem, c.k.pkt_len);
        refill_if_needed(P, c);
        return;
    }
    if (e.kind == SHD_EV_NOTIFY && notify_fast_ok(P, c)) {
        notify_fast(P, c);
        return;
    }
    if (e.kind == SHD_EV_REFILL && c.cq_count == 0 && c.tq_count == 0) {
        refill_fast(P, c);
        return;
    }
#endif
    switch (e.kind) {
    case SHD_EV_HEARTBEAT:
        // tracker_heartbeat (tracker.c:566-611): the node counters at the k-th
        // heartbeat, cumulative (the reader takes the per-interval differences)
        if (c.k.feat & F_HB) {
            const uint64_t k = c.now / hb_interval(P, c.k.feat, c.h);
            if (k >= 1 && k <= P.hb_k) P.hb[(size_t)c.l * P.hb_k + (k - 1)] = make_uint2(c.if_in, c.if_out);
        }
        schedule_self(P, c, SHD_EV_HEARTBEAT, hb_interval(P, c.k.feat, c.h), 0);
        break;
    case SHD_EV_REFILL:
        // _networkinterface_refillTokenBucketsCB (network_interface.c:163-183)
        c.flags &= ~F_REFILL_PENDING;
        c.rx_rem += c.rx_refill;
        if (c.rx_rem > c.rx_refill + SHD_MTU) c.rx_rem = c.rx_refill + SHD_MTU;
        c.tx_rem += c.tx_refill;
        if (c.tx_rem > c.tx_refill + SHD_MTU) c.tx_rem = c.tx_refill + SHD_MTU;
        if (c.cq_count == 0 && c.tq_count == 0) {
            // both queues empty: the receive loop's one dequeue attempt only
            // resets CoDel's interval and drop mode; the send loop does nothing
            if (bootstrapping(P, c) || c.rx_rem >= SHD_MTU) {
                c.cq_iexp = 0;
                c.flags &= ~F_CODEL_DROP_MODE;
            }
            refill_if_needed(P, c);
        } else {
            c.w_fl = W_RX | W_TX | W_REFILL;
        }
        break;
    case SHD_EV_REFILL_LO:
        break;
    case SHD_EV_APP_START:
        c.flags |= F_LISTENING;
        c.w_msgs = P.load;
        break;
    case SHD_EV_PACKET: {
        // _worker_runDeliverPacketTask -> router_enqueue (router.c:104-122)
        c.c_pkt++;
        trace(P, c, c.now, e.seq, c.h, e.src, e.pkt, SHD_TR_ARRIVE);
        if (c.cq_count == 0 && c.rx_rem >= SHD_MTU && !bootstrapping(P, c)) {
            // an empty router queue and room in the receive bucket: the packet
            // is enqueued and dequeued at once (sojourn 0: CoDel's interval
            // and drop mode reset; the second dequeue attempt finds nothing)
            c.cq_head = (c.cq_head + 1 == c.k.cq_cap) ? 0 : c.cq_head + 1;
            c.cq_iexp = 0;
            c.flags &= ~F_CODEL_DROP_MODE;
            if_receive_packet(P, c, e.src, e.pkt);
            consume(c.rx_rem, c.k.pkt_len);
            refill_if_needed(P, c);
            break;
        }
        const bool was_empty = c.cq_count == 0;
        if (c.cq_count >= c.k.cq_cap) { c.err |= SHD_ERR_CODELQ_OVERFLOW; break; }
        const CodelEnt ent{c.now, e.src, e.pkt};
        if (was_empty) {   // the head stays in LDS; stored only if still queued at round end
            s_cqh[threadIdx.x] = ent;
            c.cq_hv = true;
        } else {
            uint32_t tail = c.cq_head + c.cq_count;
            if (tail >= c.k.cq_cap) tail -= c.k.cq_cap;
            P.cq[(size_t)c.l * c.k.cq_cap + tail] = ent;
        }
        c.cq_count++;
        c.cq_total += c.k.pkt_len;
        c.w_fl = was_empty ? W_RX : 0u;
        break;
    }
    case SHD_EV_LOCAL:
        if_receive_packet(P, c, c.h, e.pkt);
        break;
    case SHD_EV_NOTIFY:
        c.flags &= ~F_NOTIFY_PENDING;
        c.w_msgs = c.unread;
        c.w_fl |= W_READ;
        c.unread = 0;
        break;
    default:
        c.err |= SHD_ERR_INTERNAL;
        break;
    }
    if (c.w_fl & W_RX) {
        if_receive_packets(P, c);
        c.w_fl &= ~W_RX;
    }
    // new messages while the send queue is empty and the bucket has room go
    // straight to the wire (enqueue, then the send loop pops it at once);
    // anything else -- a loopback, a full send buffer, a backlog, the
    // bootstrap period -- is left to run_work's general loop, in order
    const bool boot = bootstrapping(P, c);
    // (one exit: a loopback ends the loop through tq_count)
    while (c.w_msgs && c.tq_count == 0 && c.tx_rem >= SHD_MTU && c.ns < (uint32_t)kSendCap && !boot) {
        app_read(P, c);
        const uint32_t rv = (uint32_t)rand_r_dev(c.rng);
        c.w_msgs--;
        if ((int32_t)rv <= c.dst_thr) {   // else no destination: nothing queued
            bind_and_create(P, c, c.pkt_seq);
            const uint32_t pkt = c.pkt_seq++;
            if (is_self_draw(c, rv)) {   // loopback: queued; run_work sends it (after a flush)
                s_tqh[threadIdx.x] = TxEnt{rv, pkt};
                c.tq_hv = true;
                c.tq_count = 1;
                c.w_fl |= W_SENDING;
            } else {
                worker_send_deferred(P, c, rv, pkt);
                consume(c.tx_rem, c.k.pkt_len);
                refill_if_needed(P, c);
            }
        }
    }
}

// the event's shared steps: while (msgs || tx) { a new message if any;
// the send loop }; then the refill check.  False when it stopped for a flush.
__device__ bool run_work(const DParams& P, HostCtx& c) {
    for (;;) {
        if (c.w_fl & W_SENDING) {
            if (if_send_step(P, c)) return false;
            c.w_fl &= ~W_SENDING;
        }
        if (c.w_msgs) {
            app_read(P, c);
            const bool go = enqueue_new_message(P, c);
            c.w_msgs--;
            if (go) c.w_fl |= W_SENDING;
            continue;
        }
        if (c.w_fl & W_TX) {
            c.w_fl = (c.w_fl & ~W_TX) | W_SENDING;
            continue;
        }
        break;
    }
    if (c.w_fl & W_REFILL) {
        refill_if_needed(P, c);
        c.w_fl &= ~W_REFILL;
    }
    return true;
}

// the host's state from its record (loaded by the caller, with the idle
// test: one memory round trip for both) and the heap root
__device__ __forceinline__ void load_ctx(const DParams& P, HostCtx& c, int32_t l, const HostRec& r, int32_t att,
                                         int4 st) {
    // every field taken from the record is consumed here (launder): a load
    // still pending at the event loop would make each iteration, and the
    // code after the loop, wait for all the wave's outstanding stores (one
    // vmcnt counter, in order)
    c.l = l;
    c.h = (uint32_t)(P.h0 + l);
    c.rng = launder(r.rng); c.ev_seq = launder(r.ev_seq); c.pkt_seq = launder(r.pkt_seq);
    c.rx_rem = launder(r.rx_rem); c.tx_rem = launder(r.tx_rem); c.rx_refill = launder(r.rx_refill); c.tx_refill = launder(r.tx_refill);
    c.flags = launder(r.flags); c.unread = launder(r.unread);
    c.cq_total = launder(r.cq_total); c.cq_iexp = launder(r.cq_iexp); c.cq_ndrop = launder(r.cq_ndrop);
    c.cq_dc = launder(r.cq_dc); c.cq_dcl = launder(r.cq_dcl); c.cq_head = launder(r.cq_head); c.cq_count = launder(r.cq_count);
    c.tq_head = launder(r.tq_head); c.tq_count = launder(r.tq_count);
    c.if_in = launder(r.if_in); c.if_out = launder(r.if_out);
    c.evq_n = launder(r.evq_n);
    if (r.evq_n) {
        const shd_event t = P.evq[(size_t)l * P.evq_stride + 3];
        s_top[threadIdx.x] = t;
        c.top_time = launder(t.time);
    } else {
        c.top_time = kInf;
    }
    c.tt0 = launder(r.tt[0]); c.tt1 = launder(r.tt[1]); c.tt2 = launder(r.tt[2]);
    c.ts0 = c.ev_seq - launder(r.ts_back[0]); c.ts1 = c.ev_seq - launder(r.ts_back[1]);
    c.ts2 = c.ev_seq - launder(r.ts_back[2]);
    c.c_events = c.c_pkt = c.c_sent = c.c_idrop = c.c_cdrop = c.c_recv = 0;
    c.cq_hv = false; c.tq_hv = false;
    c.att = launder(att);
    c.min_emit = kInf; c.err = 0; c.n_pend = 0;
    c.ws = 0; c.ws_mod = 0; c.dh = 0; c.nd = 0; c.dt = kInf;
    c.ns = 0; c.seq_base = c.ev_seq; c.np = 0;
    c.w_msgs = 0; c.w_fl = 0;
    c.self_lo = launder(st.x);
    c.self_hi = launder(st.y);
    c.dst_thr = launder(st.z);
    c.cls = launder((uint32_t)st.w);
}

// earliest pending event of the host (timers and heap)
__device__ __forceinline__ uint64_t host_next(const HostCtx& c) {
    uint64_t t = c.evq_n ? c.top_time : kInf;
    t = c.tt0 < t ? c.tt0 : t;
    t = c.tt1 < t ? c.tt1 : t;
    return c.tt2 < t ? c.tt2 : t;
}

// the due list's next head time, after a take
__device__ __forceinline__ void due_advance(HostCtx& c) {
    c.dh++;
    const uint32_t k = c.dh < c.nd ? c.dh : 0u;
    const uint64_t t = s_due[k * kBlock + threadIdx.x].time;
    c.dt = c.dh < c.nd ? t : kInf;
}

// the host's next event in (time, src, seq) order if it is before `we`:
// the earliest timer (src = the host) against the heap root and the head
// of the window's calendar events (general case: equal times)
__device__ __forceinline__ bool take_next_full(const DParams& P, HostCtx& c, uint64_t we, shd_event& e) {
    uint64_t bt = c.tt0, bs = c.ts0;
    uint32_t kind = SHD_EV_HEARTBEAT;
    int slot = 0;
    if (c.tt1 < bt || (c.tt1 == bt && c.tt1 != kInf && c.ts1 < bs)) { bt = c.tt1; bs = c.ts1; kind = SHD_EV_REFILL; slot = 1; }
    if (c.tt2 < bt || (c.tt2 == bt && c.tt2 != kInf && c.ts2 < bs)) { bt = c.tt2; bs = c.ts2; kind = SHD_EV_NOTIFY; slot = 2; }
    bool timer = bt != kInf;
    // the queued candidate: heap root against the head of the due list
    const bool hq = c.evq_n != 0 && c.top_time < we, dq = c.dh < c.nd;   // due events are all < we
    bool use_due = false;
    if (hq || dq) {
        shd_event t;
        if (hq && dq) {
            const shd_event d = s_due[c.dh * kBlock + threadIdx.x], h = s_top[threadIdx.x];
            use_due = ev_less(d, h);
            t = use_due ? d : h;
        } else if (dq) {
            t = s_due[c.dh * kBlock + threadIdx.x];
            use_due = true;
        } else {
            t = s_top[threadIdx.x];
        }
        if (!timer || t.time < bt || (t.time == bt && (t.src < c.h || (t.src == c.h && t.seq < bs)))) {
            timer = false;
            e = t;
        }
    }
    if (timer) {
        if (bt >= we) return false;
        e.time = bt; e.seq = bs; e.src = c.h; e.dst = c.h; e.pkt = 0; e.kind = kind;
        if (slot == 0) c.tt0 = kInf;
        else if (slot == 1) c.tt1 = kInf;
        else c.tt2 = kInf;
        return true;
    }
    if (use_due) {
        due_advance(c);
        return true;
    }
    if (!hq) return false;
    heap_pop(P, c);
    return true;
}

// Common case: the earliest of the five candidate times (three timers, the
// due head, the heap root) is unique, so it alone decides (a tie needs the
// (src, seq) order: take_next_full).  Times only, all in registers.
__device__ __forceinline__ bool take_next(const DParams& P, HostCtx& c, uint64_t we, shd_event& e) {
    const uint64_t ht = c.evq_n ? c.top_time : kInf;
    const uint64_t m01 = c.tt0 < c.tt1 ? c.tt0 : c.tt1;
    const uint64_t bt = m01 < c.tt2 ? m01 : c.tt2;
    const uint64_t qt = c.dt < ht ? c.dt : ht;
    const uint64_t t = bt < qt ? bt : qt;
    if (t >= we) return false;
    const uint32_t neq = (uint32_t)(c.tt0 == t) + (uint32_t)(c.tt1 == t) + (uint32_t)(c.tt2 == t) +
                         (uint32_t)(c.dt == t) + (uint32_t)(ht == t);
    if (neq != 1u) return take_next_full(P, c, we, e);
    if (c.dt == t) {
        e = s_due[c.dh * kBlock + threadIdx.x];
        due_advance(c);
        return true;
    }
    if (ht == t) {
        e = s_top[threadIdx.x];
        heap_pop(P, c);
        return true;
    }
    e.time = t; e.src = c.h; e.dst = c.h; e.pkt = 0;
    if (c.tt0 == t) { e.seq = c.ts0; e.kind = SHD_EV_HEARTBEAT; c.tt0 = kInf; }
    else if (c.tt1 == t) { e.seq = c.ts1; e.kind = SHD_EV_REFILL; c.tt1 = kInf; }
    else { e.seq = c.ts2; e.kind = SHD_EV_NOTIFY; c.tt2 = kInf; }
    return true;
}

// circular distance from bin position q to the first set bit of the bitmap
// (kNB if none); static word indices only (no scratch)
__device__ __forceinline__ uint32_t bits_first_from(const uint32_t (&w)[kNBW], uint32_t q) {
    uint32_t best = kNB;
#pragma unroll
    for (int j = 0; j < (int)kNBW; j++) {
        const uint32_t m = w[j];
        const uint32_t base = 32u * j;
        uint32_t hi, lo;   // bits at positions >= q, < q
        if (base + 31 < q) { hi = 0; lo = m; }
        else if (base >= q) { hi = m; lo = 0; }
        else { const uint32_t k = q - base; hi = m & (~0u << k); lo = m & ((1u << k) - 1u); }
        if (hi) { const uint32_t d = base + __builtin_ctz(hi) - q; best = d < best ? d : best; }
        if (lo) { const uint32_t d = base + __builtin_ctz(lo) + kNB - q; best = d < best ? d : best; }
    }
    return best;
}

// lower bound of the earliest calendar event at or after `we`: the start of
// the first non-empty bin from we's bin on (stale bits only lower it)
__device__ __forceinline__ uint64_t cal_lower_bound(const DParams& P, const uint32_t (&w)[kNBW], uint64_t we) {
    const uint64_t bwe = we >> P.bin_shift;
    const uint32_t d = bits_first_from(w, (uint32_t)bwe & (kNB - 1));
    if (d >= kNB) return kInf;
    const uint64_t t = (bwe + d) << P.bin_shift;
    return t > we ? t : we;
}

__device__ void store_ctx(const DParams& P, const HostCtx& c) {
    const int32_t l = c.l;
    HostRec r;
    r.ev_seq = c.ev_seq; r.cq_total = (uint32_t)c.cq_total; r.cq_iexp = c.cq_iexp; r.cq_ndrop = c.cq_ndrop;
    r.rx_rem = (uint32_t)c.rx_rem; r.tx_rem = (uint32_t)c.tx_rem;
    r.tt[0] = c.tt0; r.tt[1] = c.tt1; r.tt[2] = c.tt2;
    r.ts_back[0] = c.tt0 != kInf ? (uint32_t)(c.ev_seq - c.ts0) : 0u;
    r.ts_back[1] = c.tt1 != kInf ? (uint32_t)(c.ev_seq - c.ts1) : 0u;
    r.ts_back[2] = c.tt2 != kInf ? (uint32_t)(c.ev_seq - c.ts2) : 0u;
    r.rng = c.rng; r.pkt_seq = c.pkt_seq; r.rx_refill = c.rx_refill; r.tx_refill = c.tx_refill;
    r.flags = c.flags; r.unread = c.unread;
    r.cq_dc = c.cq_dc; r.cq_dcl = c.cq_dcl;
    r.cq_head = (uint16_t)c.cq_head; r.cq_count = (uint16_t)c.cq_count;
    r.tq_head = (uint16_t)c.tq_head; r.tq_count = (uint16_t)c.tq_count; r.evq_n = c.evq_n;
    r.if_in = c.if_in; r.if_out = c.if_out; r.pad = 0;
    P.hs[l] = r;
    if (c.cq_hv) P.cq[(size_t)l * c.k.cq_cap + c.cq_head] = s_cqh[threadIdx.x];
    if (c.tq_hv) P.tq[(size_t)l * c.k.tq_cap + c.tq_head] = s_tqh[threadIdx.x];
    HostCnt* hc = P.hc + l;   // counter deltas: fire-and-forget atomics
    if (c.c_events) atomicAdd(&hc->events, (unsigned long long)c.c_events);
    if (c.c_pkt) atomicAdd(&hc->pkt, (unsigned long long)c.c_pkt);
    if (c.c_sent) atomicAdd(&hc->sent, (unsigned long long)c.c_sent);
    if (c.c_idrop) atomicAdd(&hc->idrop, (unsigned long long)c.c_idrop);
    if (c.c_cdrop) atomicAdd(&hc->cdrop, (unsigned long long)c.c_cdrop);
    if (c.c_recv) atomicAdd(&hc->recv, (unsigned long long)c.c_recv);
    P.hnext[l] = host_next(c);
}

template <int BLOCK>
__device__ void block_reduce_publish(const DParams& P, uint64_t next, uint64_t nev, uint64_t npkt, uint32_t err) {
    __shared__ unsigned long long s_next[BLOCK / 64], s_ev[BLOCK / 64], s_pkt[BLOCK / 64];
    __shared__ unsigned int s_err[BLOCK / 64];
    // wave reductions (64 lanes)
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(next, off, 64);
        next = o < next ? o : next;
        nev += __shfl_xor(nev, off, 64);
        npkt += __shfl_xor(npkt, off, 64);
        err |= __shfl_xor(err, off, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { s_next[w] = next; s_ev[w] = nev; s_pkt[w] = npkt; s_err[w] = err; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < BLOCK / 64; i++) {
            if (s_next[i] < s_next[0]) s_next[0] = s_next[i];
            s_ev[0] += s_ev[i]; s_pkt[0] += s_pkt[i]; s_err[0] |= s_err[i];
        }
        if (s_next[0] != kInf) atomicMin(&P.sum->next_time, s_next[0]);
        if (s_ev[0]) atomicAdd(&P.sum->n_events, s_ev[0]);
        if (s_pkt[0]) atomicAdd(&P.sum->n_pkt_events, s_pkt[0]);
        if (s_err[0]) atomicOr(&P.sum->error, s_err[0]);
    }
}

// The round's summary without a same-address atomic per block: every block
// writes its share; a two-level ticket (groups of kTickGroup blocks) elects
// the last block of each group to fold the group, and the last of those to
// fold the groups into P.sum.  True in that one block, which then sees every
// block's stores (pending records, inbox and calendar appends).  One wave per
// block (kBlock == 64).
__device__ __forceinline__ void part_fold(BlockPart& a, const BlockPart& b) {
    a.next = b.next < a.next ? b.next : a.next;
    a.nev += b.nev;
    a.npkt += b.npkt;
    a.err |= b.err;
    a.nact += b.nact;
}
__device__ __forceinline__ void part_wave_reduce(BlockPart& q) {
    for (int off = 32; off > 0; off >>= 1) {
        BlockPart o;
        o.next = __shfl_xor(q.next, off, 64);
        o.nev = __shfl_xor(q.nev, off, 64);
        o.npkt = __shfl_xor(q.npkt, off, 64);
        o.err = __shfl_xor(q.err, off, 64);
        o.nact = __shfl_xor(q.nact, off, 64);
        part_fold(q, o);
    }
}
__device__ bool round_complete(const DParams& P, uint64_t next, uint64_t nev, uint64_t npkt, uint32_t err) {
    static_assert(kBlock == 64 && kTickGroup <= 64, "one wave per block; a group folds in one pass");
    __shared__ int s_last;
    BlockPart q{next, nev, npkt, err, nev != 0 ? 1u : 0u};   // summed over the lanes below
    part_wave_reduce(q);
    const uint32_t nblk = gridDim.x, g = blockIdx.x / kTickGroup;
    const uint32_t ngrp = (nblk + kTickGroup - 1) / kTickGroup;
    if (threadIdx.x == 0) {
        P.part[blockIdx.x] = q;
        __threadfence();
        const uint32_t gsize = nblk - g * kTickGroup < kTickGroup ? nblk - g * kTickGroup : kTickGroup;
        s_last = atomicAdd(&P.tick[g], 1u) == gsize - 1;
    }
    __syncthreads();
    if (!s_last) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    {
        const uint32_t i = g * kTickGroup + threadIdx.x;
        BlockPart x{kInf, 0, 0, 0, 0};
        if (threadIdx.x < kTickGroup && i < nblk) x = P.part[i];
        part_wave_reduce(x);
        if (threadIdx.x == 0) {
            P.gpart[g] = x;
            P.tick[g] = 0;   // every block of the group has taken its ticket
            __threadfence();
            s_last = atomicAdd(&P.tick[ngrp], 1u) == ngrp - 1;
        }
    }
    __syncthreads();
    if (!s_last) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    BlockPart x{kInf, 0, 0, 0, 0};
    for (uint32_t i = threadIdx.x; i < ngrp; i += 64) part_fold(x, P.gpart[i]);
    part_wave_reduce(x);
    if (threadIdx.x == 0) {
        P.tick[ngrp] = 0;
        if (x.next != kInf) atomicMin(&P.sum->next_time, x.next);
        if (x.nev) atomicAdd(&P.sum->n_events, x.nev);
        if (x.npkt) atomicAdd(&P.sum->n_pkt_events, x.npkt);
        if (x.err) atomicOr(&P.sum->error, x.err);
        if (x.nact) atomicAdd(&P.sum->n_active, x.nact);
        __threadfence();
    }
    __syncthreads();
    return true;
}

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
        r.flags = 0; r.unread = 0; r.cq_dc = 0; r.cq_dcl = 0; r.cq_head = 0; r.cq_count = 0;
        r.tq_head = 0; r.tq_count = 0; r.evq_n = 0; r.if_in = 0; r.if_out = 0; r.pad = 0;
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
#ifdef SHD_REC_EARLY   // A/B: every lane's record in the first round trip
    in.rec = a.hs[l];
    in.att = a.att[l];
    in.st = a.st[l];
#endif
}

// one round [ws, we): merge inbox[parity] and the calendar bins of the
// window, run events < we
template <bool RX = false>   // RX: the fused peer-to-peer round's received window events (s_rx)
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
#ifdef SHD_REC_EARLY
    const HostRec& rec = in.rec;
    const int32_t rec_att = in.att;
    const int4 rec_st = in.st;
#else
    HostRec rec;
    int32_t rec_att;
    int4 rec_st;
#endif
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
#elif defined(SHD_MARK)   // asm listing markers (static code-size census)
#define KT0(v) asm volatile("; MARK " #v " begin" ::: "memory");
#define KTA(acc, v) asm volatile("; MARK " #v " end" ::: "memory");
#else
#define KT0(v)
#define KTA(acc, v)
#endif
    HostCtx c;   // idle lanes take part in the wave's flushes with no sends
    hot_load(P, c);
    PendDel pd;
    c.ns = 0; c.att = 0; c.cls = 0; c.err = 0;
    c.ws = ws; c.ws_mod = (uint32_t)(ws % SHD_MS); c.np = parity ^ 1; c.xwi = xwi; c.xput = 0;
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
#ifndef SHD_REC_EARLY
    // the host record behind the bins, in the same round trip, for the
    // hosts with something due only (idle hosts' records are never read)
    if (active) {
        rec = P.hs[l];
        rec_att = P.host_att[P.h0 + l];
        rec_st = P.self_thr[P.h0 + l];
    }
#endif
    if (active) {
        PROF_T0(t_all)
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
    round_body(P, in, ws, we, parity, next, nev, npkt, err);
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
    uint64_t seq = P.hs[dl].ev_seq;
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
    P.hs[dl].ev_seq = seq;
    if (next != kInf) atomicMin(&P.sum->next_time, (unsigned long long)next);
    if (err) atomicOr(&P.sum->error, err);
}

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

// one round of an engine group: the window start is the min over the
// headers of the last exchange; any flagged header (a first-touch log, a
// spill or an error anywhere in the group) halts the batch on every engine
// alike.  The last block writes this engine's headers for the next exchange.
__global__ __launch_bounds__(kBlock) void k_round_x(DRoundArgs a, const DParams* __restrict__ Pp,
                                                    const shd_event* __restrict__ xrecv,
                                                    XHeader* __restrict__ halt_hdr, DevSummary* __restrict__ init,
                                                    const DevCtl* __restrict__ ctl, int i, uint64_t window) {
    const DParams& P = *Pp;
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    HostIn in;
    host_in_load(a, in);
    if (*a.halt) {
        if (lead) P.sum->flags = 2u;
        return;
    }
    if (lead) {
        atomicMin(&P.sum->t_first, (unsigned long long)wall_clock64());
        *init = fresh_summary();
    }
    const uint64_t stop = ctl->stop;
    const int parity = (int)((ctl->round_base + (uint64_t)i) & 1);
    const size_t stride = (size_t)P.xcap + 1;
    uint64_t ws = kInf;
    uint32_t fl = 0;
    for (int32_t p = 0; p < P.xworld; p++) {
        const XHeader h = *(const XHeader*)(xrecv + (size_t)p * stride);
        ws = h.next_time < ws ? h.next_time : ws;
        fl |= h.flags;
    }
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
    if (ws >= stop) {   // only forwards the time
        if (blockIdx.x == 0) {
            if (threadIdx.x == 0) {
                P.sum->ws = ws;
                atomicMin(&P.sum->next_time, (unsigned long long)ws);
            }
            xpack_block(P, P.sum, 1, ws);
        }
        return;
    }
    uint64_t we = ws + window;
    if (we > stop || we < ws) we = stop;
    uint64_t next, nev, npkt;
    uint32_t err;
    round_body(P, in, ws, we, parity, next, nev, npkt, err);
    if (!round_complete(P, next, nev, npkt, err)) return;
    if (threadIdx.x == 0) P.sum->ws = ws;
    xpack_block(P, P.sum, 0, P.sum->next_time);
    if (threadIdx.x == 0) atomicMax(&P.sum->t_last, (unsigned long long)wall_clock64());
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
// stores the header body, drains it, and stores the tag.  fence: a release
// fence (an L2 write-back) before the tag as well (A/B, SHD_X_FENCE)
__device__ __forceinline__ void x_put(const shd_event* __restrict__ src, shd_event* __restrict__ dst, uint32_t n,
                                      XHeader h, uint32_t tag, int fence) {
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
        if (fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        st16_sys(dst, g0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

__global__ __launch_bounds__(256) void k_xput(const shd_event* __restrict__ xsend, shd_event* const* __restrict__ peers,
                                               uint32_t stride, uint32_t xcap, int world, int me, int wi,
                                               const DevCtl* __restrict__ ctl, uint32_t tag_add, int use_ctl,
                                               int fence) {
    const int p = blockIdx.x;
    const shd_event* src = xsend + (size_t)p * stride;
    shd_event* dst = peers[p] + ((size_t)wi * world + me) * stride;
    XHeader h = *(const XHeader*)src;
    const uint32_t n = h.count < xcap ? h.count : xcap;
    x_put(src, dst, n, h, x_tag(ctl, tag_add, use_ctl), fence);
}

// k_xfold and k_xput in one launch (peer-to-peer rounds): block p folds the
// round's shares (every block alike), packs this engine's header for peer p
// (block 0 also completes the summary), then puts the block into p's receive
// blocks.  A halted round re-sends the last header under the new tag, as the
// all-to-all re-sends the unchanged send blocks.
__device__ __forceinline__ void xfold_put(const DParams& P, const TlPart* __restrict__ parts, uint32_t nblk, int i,
                                          const DevCtl* __restrict__ ctl, shd_event* const* __restrict__ peers, int me,
                                          int wi, uint32_t tag_add, int use_ctl, int p, int fence) {
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
    x_put(src, dst, n, h, x_tag(ctl, tag_add, use_ctl), fence);
}

__global__ __launch_bounds__(256) void k_xfold_put(DParams P, const TlPart* __restrict__ parts, uint32_t nblk, int i,
                                                    const DevCtl* __restrict__ ctl, shd_event* const* __restrict__ peers,
                                                    int me, int wi, uint32_t tag_add, int use_ctl, int fence) {
    xfold_put(P, parts, nblk, i, ctl, peers, me, wi, tag_add, use_ctl, (int)blockIdx.x, fence);
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
#ifdef SHD_X_ACQUIRE   // A/B: an acquire fence (this CU's L1 invalidated) after the polls
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
#endif
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
                                               uint32_t* __restrict__ xerr, int fence) {
    if ((int)blockIdx.x < P.xworld)
        xfold_put(P, parts, nblk, i, ctl, peers, me, wi, tag_add, 1, (int)blockIdx.x, fence);
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
            *(uint64_t*)(rgn + ((size_t)(p0 + k) * P.xnbx + blk) * kXSlots + threadIdx.x) = 0;   // taken
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
                        P.bins[bi * kBinCap + s] = e;
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
            P.inbox[parity][(size_t)dl * P.inbox_cap + slot] = e;
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
        *(uint64_t*)(rgn + ((size_t)k * P.xnbx + blk) * kXSlots + threadIdx.x) = 0;   // taken
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
        P.inbox[parity][(size_t)dl * P.inbox_cap + slot] = e;
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
            P.bins[bi * kBinCap + sl[k]] = e;
            atomicOr(&P.bin_bits[(size_t)dl * kNBW + (pb >> 5)], 1u << (pb & 31));
            continue;
        }
        const uint32_t slot = atomicAdd(&P.inbox_n[next_parity][dl], 1u);
        if (slot >= P.inbox_cap) {
            err |= SHD_ERR_INBOX_OVERFLOW;
            continue;
        }
        P.inbox[next_parity][(size_t)dl * P.inbox_cap + slot] = e;
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
                                            uint64_t stop, uint32_t halt, shd_event* const* __restrict__ peers,
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
    for (size_t j = (size_t)blk * kBlock + threadIdx.x; j < n; j += (size_t)nblk * kBlock) c[j] = 0;
}

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
        px_fold_put(P, prev, pv, pp, nblk, pws, npend, nrem, pnext, perr, stop, halt, peers, world, me, wprev, tag,
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
    round_body<true>(P, in, ws, we, parity, next, nev, npkt, err, (uint32_t)((xpar + (uint64_t)i) & 1));
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

// the exchange of a batch's last round i (P.sum: its summary): blocks
// [0, world) fold and put, blocks [world, world + nblk) wait and ingest their
// block's regions into the next round's calendar / inbox
__global__ __launch_bounds__(kBlock) void k_xchg_px(DParams P, const TlPart* __restrict__ parts, uint32_t nblk, int i,
                                                     const DevCtl* __restrict__ ctl, shd_event* const* __restrict__ peers,
                                                     int world, int me, int wi, const shd_event* __restrict__ xhdr,
                                                     shd_event* __restrict__ rgn, uint32_t* __restrict__ xerr,
                                                     const shd_event* __restrict__ xrep, uint64_t xhoff, int nrep) {
    DevSummary* sum = P.sum;
    uint32_t halt = *P.halt, bad = *xerr;
    uint64_t stop = ctl->stop, rbase = ctl->round_base, xtag = ctl->xtag, pws = sum->ws;
    const uint32_t tag = (uint32_t)(xtag + (uint64_t)i);
    const TlPart* pp = parts + (size_t)(i & 1) * nblk;
    if ((int)blockIdx.x < world) {
        TlPart pv[4];
        tl_issue(pp, nblk, 0, pv);
        const uint64_t npend = sum->n_pending, nrem = sum->n_remote, pnext = sum->next_time;
        const uint32_t perr = sum->error;
        px_fold_put(P, sum, pv, pp, nblk, pws, npend, nrem, pnext, perr, stop, halt, peers, world, me, wi, tag, xhoff,
                    nrep);
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

}  // namespace

// ------------------------------------------------------------------ host driver
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
    std::vector<void*> allocs;
    std::vector<size_t> alloc_bytes;
    // protected rounds (DESIGN.md "First-touch rule"): device state copied
    // before a round that may log many first touches, restored when one of its
    // drop decisions turns out ambiguous, then the round reruns with the ranks
    std::vector<void*> snap;
    bool snap_failed = false;
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
    static constexpr int kRing = 2 * kBatch + 2;
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
    P.end_time = m->end_time; P.bootstrap_end = m->bootstrap_end; P.heartbeat = m->heartbeat_interval;
    P.app_start = m->app_start; P.load = m->load; P.payload = m->payload;
    P.pkt_len = m->payload + SHD_HEADER_UDP;
    P.force_ambig = getenv("SHD_FORCE_AMBIG") != nullptr;
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
    P.pend_cap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(1u << 16, (uint64_t)n * (m->load + 4)), 1u << 30);
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
         hipMemcpyAsync(e->d_host_hb, m->host_heartbeat, 8 * (size_t)H, hipMemcpyHostToDevice, s) != hipSuccess)) {
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
            thr[h].x = h ? draw_threshold(cum[h - 1]) + 1 : 0;
            thr[h].y = draw_threshold(cum[h]);
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
            for (int32_t i = 0; i < H; i++) ty[i] = thr[i].y;
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
             ((m->trace && (m->queue_flags & SHD_QF_TRACE_STATUS)) ? F_STATUS : 0u);
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
    if (e->h_sum->error) return SHD_EOVERFLOW;
    return SHD_OK;
}

extern "C" int shd_eng_push_events(shd_eng* e, const shd_event* ev, uint64_t n) {
    if (!e || (n && !ev)) return SHD_EINVAL;
    if (!e->booted) return SHD_EINVAL;
    if (!n) return SHD_OK;
    if (n > (1u << 30)) return SHD_ERANGE;
    for (uint64_t i = 0; i < n; i++) {
        const shd_event& x = ev[i];
        if (x.kind != SHD_EV_APP_START || x.src != x.dst || (int64_t)x.dst < e->h0 ||
            (int64_t)x.dst >= (int64_t)e->h0 + e->nloc || x.time < e->t_done)
            return SHD_EINVAL;
    }
    // stable grouping by host: a host's events keep their array order (its IDs)
    std::vector<uint32_t> idx(n);
    for (uint64_t i = 0; i < n; i++) idx[i] = (uint32_t)i;
    std::stable_sort(idx.begin(), idx.end(), [ev](uint32_t a, uint32_t b) { return ev[a].dst < ev[b].dst; });
    std::vector<shd_event> sorted(n);
    std::vector<uint32_t> off;
    for (uint64_t i = 0; i < n; i++) {
        sorted[i] = ev[idx[i]];
        sorted[i].pkt = 0;
        if (i == 0 || sorted[i].dst != sorted[i - 1].dst) off.push_back((uint32_t)i);
    }
    off.push_back((uint32_t)n);
    const uint32_t ngrp = (uint32_t)off.size() - 1;
    SHD_HIP(hipSetDevice(e->device));
    shd_event* d_ev = nullptr;
    uint32_t* d_off = nullptr;
    SHD_HIP(hipMalloc((void**)&d_ev, sizeof(shd_event) * n));
    if (hipMalloc((void**)&d_off, 4 * off.size()) != hipSuccess) { (void)hipFree(d_ev); return SHD_ENOMEM; }
    int rc = SHD_OK;
    e->P.sum = e->d_sum;
    if (hipMemcpyAsync(d_ev, sorted.data(), sizeof(shd_event) * n, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
        hipMemcpyAsync(d_off, off.data(), 4 * off.size(), hipMemcpyHostToDevice, e->stream) != hipSuccess)
        rc = SHD_ENODEV;
    if (!rc) {
        // the summary's next time is the loop's window start: seed it with the
        // host view, the kernel lowers it to the earliest pushed time
        e->h_sum->error = 0;
        if (hipMemcpyAsync(e->d_sum, e->h_sum, sizeof(DevSummary), hipMemcpyHostToDevice, e->stream) != hipSuccess)
            rc = SHD_ENODEV;
    }
    if (!rc) {
        hipLaunchKernelGGL(k_push, dim3((ngrp + 255) / 256), dim3(256), 0, e->stream, dp(e->P), (const shd_event*)d_ev,
                           (const uint32_t*)d_off, ngrp, (int)(e->round & 1));
        if (hipGetLastError() != hipSuccess) rc = SHD_ENODEV;
    }
    if (!rc) rc = read_summary(e);
    (void)hipFree(d_ev);
    (void)hipFree(d_off);
    if (!rc && e->h_sum->error) rc = SHD_EOVERFLOW;
    return rc;
}

// first-touch resolution in serial order: sort the logged queries
// by the executing event's key, assign row ranks, finalize delivered sends
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
        hipLaunchKernelGGL(k_round_tl, dim3(grid), dim3(kBlock), 0, e->stream, e->window, i, &e->d_ring[i],
                           (const DevCtl*)e->d_ctl, e->d_tpart, (const DParams*)(e->d_pr + i + 1), &e->d_ring[i + 2],
                           round_args(e->P));
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

static bool protect_all() { return getenv("SHD_PROTECT_ALL") != nullptr; }
static bool protect_off() { return getenv("SHD_NO_PROTECT") != nullptr; }

static int snapshot_state(shd_eng* e, bool restore) {
    if (!restore && e->snap.size() != e->allocs.size()) {
        for (size_t i = e->snap.size(); i < e->allocs.size(); i++) {
            void* q = nullptr;
            if (hipMalloc(&q, e->alloc_bytes[i]) != hipSuccess) {
                (void)hipGetLastError();
                for (void* p : e->snap) (void)hipFree(p);
                e->snap.clear();
                e->snap_failed = true;
                fprintf(stderr, "libshdgpu: no memory for the protected-round state copy; "
                                "rounds run unprotected (an ambiguous first touch fails the run)\n");
                return SHD_ENOMEM;
            }
            e->snap.push_back(q);
        }
    }
    for (size_t i = 0; i < e->allocs.size(); i++) {
        void* dst = restore ? e->allocs[i] : e->snap[i];
        const void* src = restore ? e->snap[i] : e->allocs[i];
        SHD_HIP(hipMemcpyAsync(dst, src, e->alloc_bytes[i], hipMemcpyDeviceToDevice, e->stream));
    }
    return SHD_OK;
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
    int rc = snapshot_state(e, false);
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

extern "C" int shd_eng_run_until(shd_eng* e, uint64_t t_stop, shd_run_stats* st) {
    if (!e) return SHD_EINVAL;
    auto t0 = std::chrono::steady_clock::now();
    int rc = SHD_OK;
    if (!e->booted && (rc = shd_eng_boot(e))) return rc;
    SHD_HIP(hipSetDevice(e->device));
    shd_run_stats s{};
    s.window_ns = e->window;
    const uint64_t stop = std::min<uint64_t>(t_stop, e->P.end_time);
    uint64_t next = e->h_sum->next_time;
    e->kernel_ms_total = 0;
    const uint64_t pend0 = e->pending_resolved;
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
        // slot 0 carries the window start; rounds use slots 1..B
        e->h_seed[0] = host_fresh_summary();
        e->h_seed[0].next_time = next;
        e->h_seed[1] = host_fresh_summary();
        e->h_ctl->stop = stop;
        e->h_ctl->round_base = e->round;
        SHD_HIP(hipMemcpyAsync(e->d_ring, e->h_seed, 2 * sizeof(DevSummary), hipMemcpyHostToDevice, e->stream));
        SHD_HIP(hipMemcpyAsync(e->d_ctl, e->h_ctl, sizeof(DevCtl), hipMemcpyHostToDevice, e->stream));
        SHD_HIP(hipMemsetAsync(e->d_halt, 0, 4, e->stream));
        SHD_HIP(hipEventRecord(e->bev[0], e->stream));
        static const bool no_tl = getenv("SHD_NO_TL") != nullptr;
        const bool tl = e->tl_ready && !no_tl;
        if ((rc = launch_batch(e, tl))) break;
        s.n_batches++;
        if (tl) s.n_batches_ticketless++;
        SHD_HIP(hipEventRecord(e->bev[1], e->stream));
        uint32_t halt = 0;
        SHD_HIP(hipMemcpyAsync(e->h_ring, e->d_ring, sizeof(DevSummary) * (B + 1), hipMemcpyDeviceToHost, e->stream));
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
        for (int i = 0; i < B; i++) {
            const DevSummary& r = e->h_ring[i + 1];
            const uint64_t ws = e->h_ring[i].next_time;
            if (ws >= stop) { next = ws; break; }   // the rest only forwarded the time
            const double ms = round_kernel_ms(e, r);
            e->kernel_ms_total += ms;
            e->last_kernel_ms = ms;
            if (r.n_pending) n_logs++;
            const bool halted_here = halt && r.n_pending > (tl ? 0ull : (unsigned long long)kResolveMax);
            s.n_rounds++;
            s.n_events += r.n_events;
            s.n_pkt_events += r.n_pkt_events;
            s.n_host_rounds += r.n_active;
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
                if (e->h_sum->error) { s.error = e->h_sum->error; rc = SHD_EOVERFLOW; }
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
        static const bool tl_strict = getenv("SHD_TL_STRICT") != nullptr;   // A/B: ticketless only after a quiet batch
        e->tl_ready = tl_strict ? (n_logs == 0 && !halt) : n_logs <= 1;
    }
    e->h_sum->next_time = next;
    // every event before `stop` has run: the engine's clock stands at stop
    if (rc == SHD_OK) e->t_done = std::max<uint64_t>(e->t_done, std::min<uint64_t>(stop, next));
    s.n_pending_resolved = e->pending_resolved - pend0;
    s.device_ms_round_kernel = e->kernel_ms_total;
    s.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (st) *st = s;
    return rc;
}

#ifdef SHD_TIMING
extern "C" int shd_debug_timing(uint64_t* out) {   // 64 x 2048 x 20
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
    hipGraphExec_t graph[2] = {nullptr, nullptr};
    bool graph_failed = false;
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

// peer-to-peer: the round stores its sends straight into the peers' receive
// blocks (A/B: SHD_X_STAGED copies them from the send blocks in k_xchg)
static bool x_direct() {
    static const bool staged = getenv("SHD_X_STAGED") != nullptr;
    return !staged;
}

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
// slots after the regions; SHD_X_REPL (1 .. 8, default 8) copies in use
static int x_nrep() {
    static const int n = [] {
        const char* v = getenv("SHD_X_REPL");
        const int k = v ? atoi(v) : kXReplMax;
        return k < 1 ? 1 : (k > kXReplMax ? kXReplMax : k);
    }();
    return n;
}
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
    P.xpeer = (g->p2p && x_direct()) ? (shd_event* const*)g->d_peers : nullptr;
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
static int x_fence() {
    static const int f = getenv("SHD_X_FENCE") != nullptr;
    return f;
}

static void x_p2p_launch(shd_xgroup* g, int wi, uint32_t tag_add, int use_ctl, const Params& P, int ri, int ingest) {
    shd_eng* e = g->engs[0];
    hipLaunchKernelGGL(k_xput, dim3(g->world), dim3(256), 0, e->stream, (const shd_event*)g->loc[0].xsend,
                       (shd_event* const*)g->d_peers, (uint32_t)g->stride, g->xcap, g->world, g->rank0, wi,
                       (const DevCtl*)e->d_ctl, tag_add, use_ctl, x_fence());
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
    // test hook: this rank fails to map its peers (every rank must then fail alike)
    if (const char* f = getenv("SHD_P2P_FAIL_RANK"))
        if (atoi(f) == g->rank0) ok = 0;
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
    for (auto& ge : g->graph)
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
    g->fused = p2p && x_direct() && x_fuse_env() && (sharers <= 1 || shared_blocks <= (unsigned long long)ncu);
    g->end_time = e->P.end_time;
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
static int x_enqueue_fused(shd_xgroup* g, int nb) {
    shd_eng* e = g->engs[0];
    shd_xgroup::Loc& L = g->loc[0];
    const uint32_t nblk = (uint32_t)((e->nloc + e->P.hpw - 1) / e->P.hpw);
    for (int i = 0; i < nb; i++) {
        const int wp = (int)((g->xseq - 1) & 1);   // exchange i - 1 (for round 0: the one before the batch)
        if (i == 0) {
            hipLaunchKernelGGL(k_round_xtl, dim3(nblk), dim3(kBlock), 0, e->stream, round_args(e->P),
                               (const DParams*)(L.d_xpr + 1), (const shd_event*)L.xrecv[wp], L.halt_hdr,
                               &e->d_ring[2], (const DevCtl*)e->d_ctl, 0, g->window, L.parts);
        } else {
            // every peer's header needs its put block, also when the engine has fewer blocks of hosts
            const uint32_t grid = std::max<uint32_t>(nblk, (uint32_t)g->world);
            hipLaunchKernelGGL(k_round_px, dim3(grid), dim3(kBlock), 0, e->stream, g->window, i, &e->d_ring[i],
                               (const DevCtl*)e->d_ctl, L.parts, (const DParams*)(L.d_xpr + i + 1), &e->d_ring[i + 2],
                               round_args(e->P), (const shd_event*)L.xrecv[wp], x_rgn(g, wp),
                               (shd_event* const*)g->d_peers, L.halt_hdr, g->d_xerr, g->world, g->rank0, wp,
                               x_rep(g, wp), x_hoff(g), x_nrep());
        }
        g->xseq++;   // exchange i: completed by round i + 1's launch, or k_xchg_px below
    }
    const int wl = (int)((g->xseq - 1) & 1);
    const Params P = xparams(g, 0, &e->d_ring[nb]);
    hipLaunchKernelGGL(k_xchg_px, dim3((unsigned)g->world + nblk), dim3(kBlock), 0, e->stream, dp(P),
                       (const TlPart*)L.parts, nblk, nb - 1, (const DevCtl*)e->d_ctl, (shd_event* const*)g->d_peers,
                       g->world, g->rank0, wl, (const shd_event*)L.xrecv[wl], x_rgn(g, wl), g->d_xerr, x_rep(g, wl),
                       x_hoff(g), x_nrep());
    return SHD_OK;
}

static int x_enqueue_rounds(shd_xgroup* g, int nb) {
    if (g->fused) return x_enqueue_fused(g, nb);
    const int nl = (int)g->engs.size();
    int rc = SHD_OK;
    for (int i = 0; i < nb; i++) {
        const int ri = (int)((g->xseq - 1) & 1);
        static const bool ticket_env = getenv("SHD_X_TICKET") != nullptr;   // A/B: the ticketed round
        const bool ticket = ticket_env && !g->p2p;   // (the peer-to-peer exchange folds the ticketless shares)
        for (int k = 0; k < nl; k++) {
            shd_eng* e = g->engs[k];
            const int grid = (e->nloc + e->P.hpw - 1) / e->P.hpw;
            if (ticket) {
                hipLaunchKernelGGL(k_round_x, dim3(grid), dim3(kBlock), 0, e->stream, round_args(e->P),
                                   (const DParams*)(g->loc[k].d_xpr + i + 1),
                                   (const shd_event*)g->loc[k].xrecv[ri], g->loc[k].halt_hdr, &e->d_ring[i + 2],
                                   (const DevCtl*)e->d_ctl, i, g->window);
            } else {
                hipLaunchKernelGGL(k_round_xtl, dim3(grid), dim3(kBlock), 0, e->stream, round_args(e->P),
                                   (const DParams*)(g->loc[k].d_xpr + i + 1),
                                   (const shd_event*)g->loc[k].xrecv[ri], g->loc[k].halt_hdr, &e->d_ring[i + 2],
                                   (const DevCtl*)e->d_ctl, i, g->window, g->loc[k].parts);
                if (g->p2p) continue;   // k_xfold_put below
                hipLaunchKernelGGL(k_xfold, dim3(1), dim3(64), 0, e->stream, dp(xparams(g, k, &e->d_ring[i + 1])),
                                   (const TlPart*)g->loc[k].parts, (uint32_t)grid, i, (const DevCtl*)e->d_ctl);
            }
        }
        if (g->p2p) {   // fold + put, then wait and ingest; the tag is ctl->xtag + i
            const int wi = (int)(g->xseq & 1);
            shd_eng* e = g->engs[0];
            const Params P = xparams(g, 0, &e->d_ring[i + 1]);
            const uint32_t nblk = (uint32_t)((e->nloc + e->P.hpw - 1) / e->P.hpw);
            static const bool split = getenv("SHD_X_SPLIT_PUT") != nullptr;   // A/B: k_xfold, then k_xput
            static const bool two = getenv("SHD_X_TWO_LAUNCH") != nullptr;    // A/B: k_xfold_put, k_xwait_ingest
            if (!split && !two) {
                const uint64_t nthr = (uint64_t)g->world * g->xcap;
                hipLaunchKernelGGL(k_xchg, dim3((unsigned)(g->world + (nthr + 255) / 256)), dim3(256), 0, e->stream,
                                   dp(P), (const TlPart*)g->loc[0].parts, nblk, i, (const DevCtl*)e->d_ctl,
                                   (shd_event* const*)g->d_peers, g->rank0, wi, (uint32_t)i,
                                   (const shd_event*)g->loc[0].xrecv[wi], g->d_xerr, x_fence());
            } else if (split) {
                hipLaunchKernelGGL(k_xfold, dim3(1), dim3(64), 0, e->stream, dp(P), (const TlPart*)g->loc[0].parts,
                                   nblk, i, (const DevCtl*)e->d_ctl);
                x_p2p_launch(g, wi, (uint32_t)i, 1, P, i, 1);
            } else {
                hipLaunchKernelGGL(k_xfold_put, dim3(g->world), dim3(256), 0, e->stream, dp(P),
                                   (const TlPart*)g->loc[0].parts, nblk, i, (const DevCtl*)e->d_ctl,
                                   (shd_event* const*)g->d_peers, g->rank0, wi, (uint32_t)i, 1, x_fence());
                const uint64_t nthr = (uint64_t)g->world * g->xcap;
                hipLaunchKernelGGL(k_xwait_ingest, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, e->stream,
                                   dp(P), (const shd_event*)g->loc[0].xrecv[wi], (const DevCtl*)e->d_ctl, (uint32_t)i,
                                   1, i, 1, g->d_xerr);
            }
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
    hipGraphExec_t& ge = g->graph[par];
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
        if ((rc = x_launch_rounds(g, nb))) break;
        s.n_batches++;
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
            if (g->last_spill_batch != ~0ull && g->batches - g->last_spill_batch <= 1 && g->xcap < (1u << 22)) {
                g->xcap *= 2;
                x_drop_graphs(g);   // the graphs point at the old blocks
                if ((rc = x_alloc(g))) break;
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
