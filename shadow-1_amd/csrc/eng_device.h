// eng_device.h -- the engine's device types and per-host event code: host
// record, parameters, RNG, queues (heap, calendar), CoDel, token buckets, path
// values with the first-touch rule, deferred sends and their wave flush, event
// dispatch (begin_event / run_work / take_next), host context load/store.
// Part of libshdgpu's engine translation unit (csrc/engine.hip includes it
// inside its anonymous namespace); not a standalone header.
#pragma once

constexpr uint64_t kInf = 0xFFFFFFFFFFFFFFFFull;
constexpr uint32_t F_REFILL_PENDING = 1u, F_NOTIFY_PENDING = 2u, F_LISTENING = 4u, F_CODEL_DROP_MODE = 8u,
                   F_BOUND = 16u;   // an SHD_SEND_ONCE socket is bound (its first sendto drew the port)
// the host's datagram application (F_APP: not PHOLD), in the flags word from
// boot on: bits 8-9 shd_udp_app::send, 10-11 dest, 12 per_read
constexpr uint32_t kAppShift = 8u;
__device__ __forceinline__ uint32_t app_send(uint32_t flags) { return (flags >> kAppShift) & 3u; }
__device__ __forceinline__ uint32_t app_dest(uint32_t flags) { return (flags >> (kAppShift + 2)) & 3u; }
__device__ __forceinline__ bool app_per_read(uint32_t flags) { return ((flags >> (kAppShift + 4)) & 1u) != 0; }
// a send's destination draw (TxEnt::r, SendRec::r): a rand_r value (PHOLD's
// destination pick, resolved at the flush), or a host named by the
// application (the UDP echo's server or the sender being answered)
constexpr uint32_t kDstHost = 0x80000000u;
constexpr double kRandMax = 2147483647.0;
constexpr uint64_t kCodelTarget = 10ull * SHD_MS;      // router_queue_codel.c:42
constexpr uint64_t kCodelInterval = 100ull * SHD_MS;   // router_queue_codel.c:48
// calendar geometry: bins per host (a ring), event slots per bin, bitmap
// words, and the append horizon in bins ahead of the round's first bin.  The
// horizon stops short of the ring by 4 so that no append in round r can land
// in a slot the owner reads or clears in round r or r+1.
constexpr uint32_t kNB = 256, kBinCap = 4, kNBW = kNB / 32, kHorizon = kNB - 4;
constexpr int kDueCap = 6;             // due-list slots per host (more due events take the heap)
constexpr int kPool = 288;             // deferred sends of the wave between flushes, in one pool
                                       // shared by its hosts (a busy host may take most of it);
                                       // with the due list and the flush's arrays, < 40 KB of LDS
                                       // per block: four blocks per CU once hosts fill the machine
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
    uint16_t lane;     // the sending host's lane
    uint16_t next;     // the host's next record in the pool (in send order)
    uint32_t _pad;
};
static_assert(sizeof(SendRec) == 48, "send record layout");

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
    uint16_t rq_head;                      // SHD_DEST_REPLY: the head of the socket's source ring (its length is unread)
    uint16_t port;                         // SHD_SEND_ONCE: its socket's port (F_BOUND)
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
constexpr uint32_t F_TRACE = 1u, F_HB = 2u, F_PCOUNT = 4u, F_HOSTHB = 8u, F_AMBIG = 16u, F_STATUS = 64u,
                   F_APP = 128u;    // the application is not PHOLD: per-host modes (app_send / app_dest)

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
    // the application (shd_model::app): SHD_APP_PHOLD, or a datagram
    // application per host (SHD_APP_UDP_ECHO / SHD_APP_UDP): app_mode[h]
    // (send | dest << 2 | per_read << 4, copied into the flags word at boot),
    // app_nstart[h] its start datagrams, app_peer[h] its SHD_DEST_PEER host; a
    // replying host keeps a ring of the sources of the datagrams its socket
    // holds ([nloc][rq_cap], recvfrom's address)
    uint32_t app, rq_cap;
    Ptr<const int32_t> app_peer;
    Ptr<const uint8_t> app_mode;
    Ptr<const uint32_t> app_nstart;
    Ptr<uint32_t> rq;
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
__device__ unsigned long long g_tim[64][2048][24];
// per event class, over iterations in which every lane that starts an event
// starts one of that class: {iterations, cycles, of which take_next, of which
// begin_event}.  Class = kind (1..7), 8 = a packet on the general path
__device__ unsigned long long g_kc[10][4];
// event-path counters (timing build): cq / tq entries loaded from HBM, heap
// pushes / pops, inbox events merged, events, flushes, suspended lanes
__device__ unsigned long long g_cnt[8];
#if defined(SHD_TIMING_LIGHT) && !defined(SHD_TCNT)   // phase stamps only: no per-event counters either
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
// SHD_TIMING_P0: the persistent kernels keep their one parameter copy (as the
// product does; a copy per round costs scalar-cache misses every round and
// doubled the sparse round's time in round 5's stamps) and name the round's
// slot in LDS instead (s_tslot, valid while s_tslot_key holds the key; the
// persistent kernels clear it on exit)
#define TIM_SLOT() (uint32_t)(((uintptr_t)P.sum / sizeof(DevSummary)) & 63)
#ifdef SHD_TIMING_P0
__shared__ uint32_t s_tslot;
#define PS_TIM_SLOT() (s_tslot & 63u)
#else
#define PS_TIM_SLOT() TIM_SLOT()
#endif
#define TIM(k)                                                                                         \
    do {                                                                                               \
        TIM_WAIT();                                                                                    \
        if (threadIdx.x == 0 && blockIdx.x < 2048)                                                     \
            g_tim[TIM_SLOT()][blockIdx.x][k] = wall_clock64();                                         \
    } while (0)
// in the persistent rounds' code (k_round_ps / _sp / _spx): the slot from LDS
// under SHD_TIMING_P0
#define TIMP(k)                                                                                        \
    do {                                                                                               \
        TIM_WAIT();                                                                                    \
        if (threadIdx.x == 0 && blockIdx.x < 2048)                                                     \
            g_tim[PS_TIM_SLOT()][blockIdx.x][k] = wall_clock64();                                      \
    } while (0)
#define TIMVP(k, v)                                                                                    \
    do {                                                                                               \
        if ((int)threadIdx.x == __ffsll((unsigned long long)__ballot(1)) - 1 && blockIdx.x < 2048)     \
            g_tim[PS_TIM_SLOT()][blockIdx.x][k] = (v);                                                 \
    } while (0)
// inside a divergent region: the first active lane stamps
#define TIMA(k)                                                                                        \
    do {                                                                                               \
        TIM_WAIT();                                                                                    \
        if ((int)threadIdx.x == __ffsll((unsigned long long)__ballot(1)) - 1 && blockIdx.x < 2048)     \
            g_tim[TIM_SLOT()][blockIdx.x][k] = wall_clock64();                                         \
    } while (0)
#define TIMV(k, v)                                                                                     \
    do {                                                                                               \
        if ((int)threadIdx.x == __ffsll((unsigned long long)__ballot(1)) - 1 && blockIdx.x < 2048)     \
            g_tim[TIM_SLOT()][blockIdx.x][k] = (v);                                                    \
    } while (0)
#else
#define TIM(k)
#define TIMP(k)
#define TIMA(k)
#define TIMV(k, v)
#define TIMVP(k, v)
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
// glibc rand_r: three steps of x <- a x + c (mod 2^32), 11 + 10 + 10 bits of
// their states.  The three states are taken from x directly (x_k = a^k x +
// c (a^(k-1) + ... + 1)): three independent multiplies instead of a chain
// of three, the same values
constexpr uint32_t kLcgA = 1103515245u, kLcgC = 12345u;
constexpr uint32_t kLcgA2 = kLcgA * kLcgA, kLcgC2 = kLcgA * kLcgC + kLcgC;
constexpr uint32_t kLcgA3 = kLcgA * kLcgA2, kLcgC3 = kLcgA * kLcgC2 + kLcgC;
__device__ __forceinline__ int32_t rand_r_dev(uint32_t& x) {
    const uint32_t x1 = x * kLcgA + kLcgC, x2 = x * kLcgA2 + kLcgC2, x3 = x * kLcgA3 + kLcgC3;
    uint32_t r = (x1 >> 16) & 2047u;
    r = (r << 10) ^ ((x2 >> 16) & 1023u);
    r = (r << 10) ^ ((x3 >> 16) & 1023u);
    x = x3;
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
    asm volatile("" : "+v"(x));
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
    int32_t peer;               // UDP echo: -1 a server, else the client's server host (PHOLD: -1)
    uint32_t rq_head, port;     // HostRec::rq_head / port
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
    // k_round_ps: the first calendar bin the receivers did NOT load ahead for
    // the next round (0 elsewhere): an append to an earlier bin, and every
    // inbox append, is noted for the share (note_dirty)
    uint64_t pf_lim;
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

// k_round_ps's cross-barrier prefetch (eng_round.h): the blocks load the next
// window's calendar bins before the round's barrier, so an append that lands
// in a bin a receiver may already have read (before HostCtx::pf_lim), or in an
// inbox, is noted here and published with the round's share; the receiving
// host then reads its hand-off words after the barrier, as without prefetch
constexpr uint32_t kDirtyMax = 3;                 // destinations one share names
constexpr uint32_t kDirtyNone = 0xFFFFFFFFu, kDirtyAll = 0xFFFFFFFEu;
__shared__ uint32_t s_dn;                          // appends noted this round
__shared__ uint32_t s_dl[kDirtyMax];              // ... their local destinations (the first kDirtyMax)
__device__ __forceinline__ void note_dirty(int32_t dl) {
    const uint32_t k = atomicAdd(&s_dn, 1u);
    if (k < kDirtyMax) s_dl[k] = (uint32_t)dl;
}

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

// An event handed to another host's calendar or inbox: two 16-B agent-scope
// write-through stores (global_store_dwordx4 sc1: written through to memory,
// the line dropped from the writer's L2).  The persistent rounds (k_round_ps)
// read such events in a later round of the same launch, on another CU and
// possibly another XCD, with sc1 loads after every writer drained
// (MI355X_MICROARCH.md, inter-workgroup visibility: sc1 stores + sc1 loads);
// the launch-per-round kernels read them after a kernel boundary.  hipcc does
// not count an asm store: the writers drain with an explicit
// s_waitcnt vmcnt(0) (vmcnt is in issue order, so the compiler's own waits
// stay conservative); the s_nop keeps the data registers intact until the
// store has read them.  (Four 8-B atomic stores would write 4x the bytes:
// rocprofv3 WRITE_SIZE counts 32 B per 8-B sc1 store, profiles/r03.)
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ev_st_sc1(shd_event* p, const shd_event& e) {
    const u32x4_t a = {(uint32_t)e.time, (uint32_t)(e.time >> 32), (uint32_t)e.seq, (uint32_t)(e.seq >> 32)};
    const u32x4_t b = {e.src, e.dst, e.pkt, e.kind};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\tglobal_store_dwordx4 %0, %2, off offset:16 sc1\n\ts_nop 1"
                 ::"v"(p), "v"(a), "v"(b) : "memory");
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
        if (c.pf_lim) note_dirty(dl);
        uint32_t slot = atomicAdd(&P.inbox_n[c.np][dl], 1u);
        if (slot >= P.inbox_cap) { c.err |= SHD_ERR_INBOX_OVERFLOW; return; }
        ev_st_sc1(&P.inbox[c.np][(size_t)dl * P.inbox_cap + slot], e);
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

// UDP echo: the socket keeps each datagram's source (recvfrom's address), in
// arrival order, in a ring of rq_cap behind rq_head; its length is `unread`
// (called after unread counted the datagram)
__device__ __forceinline__ void rq_push(const DParams& P, HostCtx& c, uint32_t src) {
    if (c.unread > P.rq_cap) { c.err |= SHD_ERR_INTERNAL; return; }
    uint32_t t = c.rq_head + c.unread - 1;
    if (t >= P.rq_cap) t -= P.rq_cap;
    P.rq[(size_t)c.l * P.rq_cap + t] = src;
}

// _networkinterface_receivePacket (network_interface.c:375-419)
__device__ void if_receive_packet(const DParams& P, HostCtx& c, uint32_t src, uint32_t pkt) {
    c.if_in++;   // tracker_addInputBytes (network_interface.c:415)
    if (c.flags & F_LISTENING) {
        trace(P, c, c.now, 0, c.h, src, pkt, SHD_TR_RECV);
        c.c_recv++;
        c.unread++;
        if ((c.k.feat & F_APP) && app_dest(c.flags) == SHD_DEST_REPLY) rq_push(P, c, src);
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

// the persistent kernels' summary of the running round (they read one copy
// of the parameters for the whole batch, whose `sum` is the batch's first)
__shared__ DevSummary* s_rsum;

__device__ void log_pending(const DParams& P, HostCtx& c, const SendRec& q, int32_t a, int32_t b, uint32_t delivered,
                            uint32_t dst, uint64_t seq, DevSummary* sum) {
    unsigned long long i = atomicAdd(&sum->n_pending, 1ull);
    c.n_pend++;
    if (i >= P.pend_cap) { c.err |= SHD_ERR_PENDING_OVERFLOW; return; }
    Pending r;
    r.qtime = q.now; r.qseq = q.q_seq; r.qhost = c.h; r.qsrc = q.q_src; r.qsub = q.q_sub & 0x7FFFFFFFu;
    r.a = (uint32_t)a; r.b = (uint32_t)b; r.delivered = delivered; r.dst = dst; r.pkt = q.pkt; r.seq = seq;
    P.pend[i] = r;
}

// LDS of the round kernel (one wave per block).  The deferred sends of the
// wave's hosts share one pool: a record is claimed with an LDS atomic and
// linked into its host's list (head / tail per lane), so that one busy host
// (a popular relay) can defer hundreds of sends between flushes while the
// others defer a few.  A send may be deferred only while the pool has room
// for one more record per lane (send_room): every code path defers at most
// one send per lane between two such checks.
__shared__ SendRec s_send[kPool];               // deferred sends
__shared__ shd_event s_res[kPool];              // flush: resolved sends, then the events to deliver
__shared__ uint32_t s_pool_n;                   // records claimed (may pass kPool: then unclaimed)
__shared__ uint16_t s_shd[kBlock], s_stl[kBlock];   // each lane's first and last record
__shared__ int32_t s_att[kBlock];                // flush: each lane's attached vertex
__shared__ uint32_t s_cls[kBlock];               // flush: each lane's destination-weight class

__device__ __forceinline__ bool send_room() {
    const uint32_t n = __hip_atomic_load(&s_pool_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return n + (uint32_t)kBlock <= (uint32_t)kPool;
}
// no deferred sends (round start; every lane of the wave)
__device__ __forceinline__ void send_pool_reset(HostCtx& c) {
    c.ns = 0;
    s_pool_n = 0;
}

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
    q.lane = (uint16_t)threadIdx.x;
    q.next = 0xFFFFu;
    q._pad = 0;
    const uint32_t k = atomicAdd(&s_pool_n, 1u);   // < kPool: the caller saw send_room()
    s_send[k] = q;
    if (c.ns) s_send[s_stl[threadIdx.x]].next = (uint16_t)k;
    else s_shd[threadIdx.x] = (uint16_t)k;
    s_stl[threadIdx.x] = (uint16_t)k;
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
    uint16_t kind;   // 0 none, 1 calendar claim issued, 2 inbox / remote
    uint16_t near;   // kind 1: the bin is before HostCtx::pf_lim (note_dirty)
};

// the destination of a draw with closed-form destinations (dest_closed):
// _phold_chooseNode's first i with dest_cum[i] >= x / RAND_MAX, from the
// even cumulative weights' formula and the host-made exception list
__device__ __forceinline__ int32_t closed_dest(const DParams& P, uint32_t r) {
    const uint64_t nx = (uint64_t)r * (uint64_t)(uint32_t)P.H;
    const uint64_t cx = (nx + 2147483646ull) / 2147483647ull;
    int32_t d = cx ? (int32_t)cx - 1 : 0;
#pragma unroll
    for (int j = 0; j < kDestExc; j++)   // unrolled: the list is read in one scalar batch
        d = (j < P.n_exc && (int32_t)r == P.exc_x[j]) ? P.exc_d[j] : d;
    return d;
}

template <bool PS = false>
__device__ __forceinline__ void flush_wave(const DParams& P, HostCtx& c, bool defer, PendDel& pd) {
    pd.kind = 0;
    const uint32_t lane = threadIdx.x;
    const uint32_t n = c.ns;
    const uint32_t claimed = __hip_atomic_load(&s_pool_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t total = __builtin_amdgcn_readfirstlane(claimed < (uint32_t)kPool ? claimed : (uint32_t)kPool);
    if (total == 0) return;
    const bool one = defer && total <= (uint32_t)kBlock;   // the round's last flush, one batch
    s_att[lane] = c.att;
    s_cls[lane] = c.cls;
    __syncthreads();
#ifdef SHD_TIMING_LIGHT
    TIMP(12);
#endif
    uint32_t err = 0;
    for (uint32_t base = 0; base < total; base += kBlock) {
        const uint32_t r = base + lane;
        if (r >= total) continue;
        const SendRec q = s_send[r];
        const uint32_t hl = q.lane;
        const int32_t a = s_att[hl];
        int32_t dst, b;
        if (q.r & kDstHost) {   // a destination the application named (UDP echo)
            dst = (int32_t)(q.r & ~kDstHost);
            b = P.host_att[dst];
        } else if (P.dest_closed) {   // no table: one memory round trip fewer
            dst = closed_dest(P, q.r);
            b = dst;
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
                pd.near = bb < c.pf_lim ? 1u : 0u;
            }
        }
    }
    __syncthreads();
#ifdef SHD_TIMING_LIGHT
    TIMP(13);
#endif
    // per host, in send order (worker.c:286-320).  Timers scheduled since the
    // last flush hold provisional IDs: an ID x loses the dropped sends issued
    // before it
    uint32_t nfail = 0;
    uint64_t f0 = 0, f1 = 0, f2 = 0;
    const bool p0 = c.tt0 != kInf && c.ts0 >= c.seq_base, p1 = c.tt1 != kInf && c.ts1 >= c.seq_base,
               p2 = c.tt2 != kInf && c.ts2 >= c.seq_base;
    uint32_t k = n ? s_shd[lane] : 0u;
    for (uint32_t i = 0; i < n; i++) {
        shd_event e = s_res[k];
        const SendRec q = s_send[k];
        const bool pass = e.kind & 1u, log = (e.kind & 2u) != 0, resolved = (e.kind & 4u) != 0;
        const int32_t b = (int32_t)e.src;
        uint32_t emit = 0;
        if (pass) {
            const uint64_t seq = c.seq_base + q.pseq - nfail;
            trace(P, c, q.now, seq, c.h, e.dst, q.pkt, SHD_TR_SENT);
            c.c_sent++;
            // 1 = delivery waits for the resolution, 2 = already delivered
            if (log) log_pending(P, c, q, c.att, b, resolved ? 2u : 1u, e.dst, seq, PS ? s_rsum : P.sum);
            if (resolved && e.time < c.k.end_time) {   // scheduler_push drops time >= end
                emit = SHD_EV_PACKET;
                if (e.time < c.min_emit) c.min_emit = e.time;
            }
            e.seq = seq;
        } else {
            trace(P, c, q.now, 0, c.h, e.dst, q.pkt, SHD_TR_INET_DROP);
            c.c_idrop++;
            if (log) log_pending(P, c, q, c.att, b, 0u, e.dst, 0, PS ? s_rsum : P.sum);
            const uint64_t xi = c.seq_base + q.pseq;
            f0 += xi < c.ts0; f1 += xi < c.ts1; f2 += xi < c.ts2;
            nfail++;
        }
        e.src = c.h;
        e.pkt = q.pkt;
        e.kind = emit;
        s_res[k] = e;
        k = q.next;
    }
    if (nfail) {
        if (p0) c.ts0 -= f0;
        if (p1) c.ts1 -= f1;
        if (p2) c.ts2 -= f2;
        c.ev_seq -= nfail;
    }
    c.seq_base = c.ev_seq;
    c.ns = 0;
    __syncthreads();
    if (lane == 0) s_pool_n = 0;   // (every lane read it above, before the barrier)
#ifdef SHD_TIMING_LIGHT
    TIMP(14);
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
                ev_st_sc1(&P.bins[bi * kBinCap + slot], e);
                const uint32_t p = (uint32_t)bb & (kNB - 1);
                atomicOr(&P.bin_bits[(size_t)dl * kNBW + (p >> 5)], 1u << (p & 31));
                if (bb < c.pf_lim) note_dirty(dl);
                continue;
            }
        }
        emit_nocal(P, c, e);
    }
    c.err |= err;
    __syncthreads();   // s_res is reused by the next flush
}

// the stores of the round's last flush (after its claims returned)
__device__ __forceinline__ void flush_finish(const DParams& P, HostCtx& c, const PendDel& pd) {
    if (pd.kind == 0) return;
    const shd_event e = s_res[threadIdx.x];
    if (pd.kind == 1 && pd.slot < kBinCap) {
        ev_st_sc1(&P.bins[pd.bi * kBinCap + pd.slot], e);
        const uint32_t p = (uint32_t)(pd.bi & (kNB - 1));
        const int32_t dl = (int32_t)e.dst - P.h0;
        atomicOr(&P.bin_bits[(size_t)dl * kNBW + (p >> 5)], 1u << (p & 31));
        if (pd.near) note_dirty(dl);
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
        if ((c.ns && self) || !send_room()) return true;
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

// The device application hook: the draws and records of one new datagram
// before it is queued on the interface; rv: its destination draw (kDstHost |
// host: a named destination), false when nothing is sent.  `reading`: the
// message answers a datagram the application just read (NOTIFY's messages).
//   PHOLD (_phold_sendNewMessage, test_phold.c:218-230): the destination draw,
//     resolved at the flush (no destination: nothing sent), the implicit
//     bind's port draw, SND_CREATED;
//   a datagram application (F_APP: SHD_APP_UDP, SHD_APP_UDP_ECHO, shdgpu.h
//     shd_udp_app; oracle/ref_harness/ref_loop.c apps 2 and 3): a replying
//     host takes the read datagram's source off its ring; a read-only host
//     sends nothing for it; the destination is the weighted draw (as PHOLD's),
//     the peer or that source; the source port is a new socket's (a port draw
//     per datagram), the one socket's (bound by its first sendto: one draw,
//     host.c:1514-1525) or the listener's.
__device__ __forceinline__ bool app_message(const DParams& P, HostCtx& c, bool reading, uint32_t& rv,
                                            uint32_t& pkt) {
    if (!(c.k.feat & F_APP)) {
        rv = (uint32_t)rand_r_dev(c.rng);
        if ((int32_t)rv > c.dst_thr) return false;   // no i with dest_cum[i] >= r
        bind_and_create(P, c, c.pkt_seq);
        pkt = c.pkt_seq++;
        return true;
    }
    const uint32_t send = app_send(c.flags), dest = app_dest(c.flags);
    uint32_t src = 0;
    if (reading && dest == SHD_DEST_REPLY) {   // the datagram read leaves the socket (its source: the ring)
        src = P.rq[(size_t)c.l * P.rq_cap + c.rq_head];
        c.rq_head = c.rq_head + 1 == P.rq_cap ? 0u : c.rq_head + 1;
    }
    if (reading && !app_per_read(c.flags)) return false;
    if (dest == SHD_DEST_WEIGHTED) {
        rv = (uint32_t)rand_r_dev(c.rng);
        if ((int32_t)rv > c.dst_thr) return false;
    } else {
        rv = (dest == SHD_DEST_REPLY ? src : (uint32_t)c.peer) | kDstHost;
    }
    if (send == SHD_SEND_EACH) {
        bind_and_create(P, c, c.pkt_seq);
        pkt = c.pkt_seq++;
        return true;
    }
    uint32_t sport = SHD_PHOLD_LISTEN_PORT;
    if (send == SHD_SEND_ONCE) {
        if (!(c.flags & F_BOUND)) {
            c.port = random_free_port_value(c);
            c.flags |= F_BOUND;
        }
        sport = c.port;
    }
    if (c.k.feat & F_STATUS) trace(P, c, c.now, sport, c.h, ~0u, c.pkt_seq, SHD_TR_CREATED);
    pkt = c.pkt_seq++;
    return true;
}

// _phold_sendNewMessage (test_phold.c:218-230) up to the socket send: draw
// the destination (resolved at the flush; only whether one exists matters
// here), bind, queue the datagram; false when nothing was queued
__device__ bool enqueue_new_message(const DParams& P, HostCtx& c) {
    PROF_T0(tp)
    uint32_t rv, pkt;
    const bool go = app_message(P, c, (c.w_fl & W_READ) != 0, rv, pkt);
    PROF_ADD(c, PR_PICK, tp)
    if (!go) return false;
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
    return c.unread == 1u && c.tq_count == 0 && c.tx_rem >= SHD_MTU && send_room() &&
           !(c.k.feat & F_TRACE) && !bootstrapping(P, c);
}
__device__ __forceinline__ void notify_fast(const DParams& P, HostCtx& c) {
    c.flags &= ~F_NOTIFY_PENDING;
    c.unread = 0;
    uint32_t rv, pkt;
    if (app_message(P, c, true, rv, pkt)) {   // else no destination: nothing queued
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
        if ((c.k.feat & F_APP) && app_dest(c.flags) == SHD_DEST_REPLY) rq_push(P, c, e.src);
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
        c.w_msgs = (c.k.feat & F_APP) ? P.app_nstart[c.h] : P.load;   // (a replying host: 0)
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
    while (c.w_msgs && c.tq_count == 0 && c.tx_rem >= SHD_MTU && send_room() && !boot) {
        app_read(P, c);
        uint32_t rv, pkt;
        const bool go = app_message(P, c, (c.w_fl & W_READ) != 0, rv, pkt);
        c.w_msgs--;
        if (go) {   // else no destination: nothing queued
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
    c.rq_head = launder((uint32_t)r.rq_head); c.port = launder((uint32_t)r.port);
    c.peer = (c.k.feat & F_APP) ? launder(P.app_peer[P.h0 + l]) : -1;
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
    c.min_emit = kInf; c.err = 0; c.n_pend = 0; c.pf_lim = 0;
    c.ws = 0; c.ws_mod = 0; c.dh = 0; c.nd = 0; c.dt = kInf;
    send_pool_reset(c); c.seq_base = c.ev_seq; c.np = 0;
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

// rec / hn: where the record and the next time go (default: the host's
// global ones; k_round_sp with LDS-resident records: the block's LDS copies)
__device__ __forceinline__ void store_ctx(const DParams& P, HostCtx& c, HostRec* rec = nullptr,
                                          uint64_t* hn = nullptr) {
    const int32_t l = c.l;
    HostRec r;
    r.ev_seq = c.ev_seq; r.cq_total = (uint32_t)c.cq_total; r.cq_iexp = c.cq_iexp; r.cq_ndrop = c.cq_ndrop;
    r.rx_rem = (uint32_t)c.rx_rem; r.tx_rem = (uint32_t)c.tx_rem;
    r.tt[0] = c.tt0; r.tt[1] = c.tt1; r.tt[2] = c.tt2;
    // a live timer's ID as its distance back from ev_seq, in 32 bits: a
    // distance of 2^32 or more (a long heartbeat interval on a busy host) is
    // an error, never a silent wrap
    const uint64_t b0 = c.tt0 != kInf ? c.ev_seq - c.ts0 : 0u, b1 = c.tt1 != kInf ? c.ev_seq - c.ts1 : 0u,
                   b2 = c.tt2 != kInf ? c.ev_seq - c.ts2 : 0u;
    if ((b0 | b1 | b2) >> 32) c.err |= SHD_ERR_INTERNAL;
    r.ts_back[0] = (uint32_t)b0;
    r.ts_back[1] = (uint32_t)b1;
    r.ts_back[2] = (uint32_t)b2;
    r.rng = c.rng; r.pkt_seq = c.pkt_seq; r.rx_refill = c.rx_refill; r.tx_refill = c.tx_refill;
    r.flags = c.flags; r.unread = c.unread;
    r.cq_dc = c.cq_dc; r.cq_dcl = c.cq_dcl;
    r.cq_head = (uint16_t)c.cq_head; r.cq_count = (uint16_t)c.cq_count;
    r.tq_head = (uint16_t)c.tq_head; r.tq_count = (uint16_t)c.tq_count; r.evq_n = c.evq_n;
    r.if_in = c.if_in; r.if_out = c.if_out;
    r.rq_head = (uint16_t)c.rq_head; r.port = (uint16_t)c.port;
    if (rec) *rec = r;
    else P.hs[l] = r;
    if (c.cq_hv) P.cq[(size_t)l * c.k.cq_cap + c.cq_head] = s_cqh[threadIdx.x];
    if (c.tq_hv) P.tq[(size_t)l * c.k.tq_cap + c.tq_head] = s_tqh[threadIdx.x];
    HostCnt* hc = P.hc + l;   // counter deltas: fire-and-forget atomics
    if (c.c_events) atomicAdd(&hc->events, (unsigned long long)c.c_events);
    if (c.c_pkt) atomicAdd(&hc->pkt, (unsigned long long)c.c_pkt);
    if (c.c_sent) atomicAdd(&hc->sent, (unsigned long long)c.c_sent);
    if (c.c_idrop) atomicAdd(&hc->idrop, (unsigned long long)c.c_idrop);
    if (c.c_cdrop) atomicAdd(&hc->cdrop, (unsigned long long)c.c_cdrop);
    if (c.c_recv) atomicAdd(&hc->recv, (unsigned long long)c.c_recv);
    if (hn) *hn = host_next(c);
    else P.hnext[l] = host_next(c);
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
