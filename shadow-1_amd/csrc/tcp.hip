// tcp.hip -- the TCP path on the GPU (include/shdtcp.h).
//
// The reference's TCP, run for the processes of the reference's own TCP test
// (src/test/tcp/test_tcp.c, nonblocking-epoll) on every host of a model:
//
//   connection state machine   host/descriptor/tcp.c:607-698, 1777-2099
//   segments, windows, flush   tcp.c:729-852, 1090-1278
//   retransmission, RTO        tcp.c:854-1065, 1280-1333 (RFC 6298)
//   SACK / lost ranges         tcp_retransmit_tally.cc
//   Reno                       tcp_cong_reno.c
//   buffer autotuning          tcp.c:363-591
//   user send / receive        tcp.c:2126-2327, host.c:1466-1604
//   connect / listen / accept  tcp.c:1462-1558, host.c:1111-1358
//   close                      tcp.c:2363-2408
//   socket buffers             socket.c:284-455
//   interface, FIFO qdisc      network_interface.c:87-226, 375-605
//   worker_sendPacket          worker.c:260-321
//   router + CoDel             router.c:104-140, router_queue_codel.c
//   epoll notification         epoll.c:252-395, 411-615, 638-683
//   binary heaps               utility/priority_queue.c
//
// Execution: conservative rounds of width W = the smallest path latency
// between hosts (ceil(ms * 1e6)); one lane per host runs every event of its
// own heap before the round's end in event order (time, src, seq; event.c:
// 110-153), exactly as the serial loop would, because nothing another host
// does inside the round can reach it before the round ends.  A delivery to
// another host goes into the round's mailbox with its packet copy and is
// taken by the receiver's lane at the start of the next round.  Every piece
// of state lives in HBM in fixed-capacity per-host / per-socket arrays; an
// overflow sets an error bit instead of corrupting anything.
//
// The work is branchy per-host control flow with a few events per host and
// round: latency-bound by design ("TCP"); it shares nothing with
// the UDP engine's LDS-resident round kernels.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/shdtcp.h"
#include "shd_device.h"   // struct shd_pc: the path cache's device tables (shd_tcp_model.path_cache)
// comm.hip: device buffers of per-peer sizes -- peer p gets send_bytes[p] from d_send +
// send_off[p], this rank recv_bytes[p] from peer p into d_recv + recv_off[p] (the sizes
// agreed beforehand); RCCL: grouped send / receive on `s`; the host transport: fixed
// blocks of the largest size through host memory (synchronizes `s`)
__attribute__((visibility("hidden"))) int shd_pc_fold_ranked(shd_pc* pc, const int32_t* old_rank,
                                                             const int32_t* old_self);
__attribute__((visibility("hidden"))) int shd_comm_alltoallv_dev(shd_comm* c, const char* d_send,
                                                                 const size_t* send_off, const size_t* send_bytes,
                                                                 char* d_recv, const size_t* recv_off,
                                                                 const size_t* recv_bytes, hipStream_t s);

namespace {

constexpr uint64_t kMs = 1000000ull;
constexpr uint64_t kSec = 1000000000ull;
constexpr uint32_t kMTU = 1500, kHdr = 66, kMSS = kMTU - kHdr;
constexpr uint32_t kHdrUdp = 42;    // CONFIG_HEADER_SIZE_UDPIPETH (definitions.h:176)
constexpr uint16_t kUdpPort = 8998; // the datagram applications' port (test_phold.c's PHOLD_LISTEN_PORT)
constexpr uint32_t kDgramMax = 65507;   // CONFIG_DATAGRAM_MAX_SIZE (definitions.h:193)
constexpr int kSock = 8;            // sockets per host (a listener, its children, clients); a model with
                                    // datagram processes gets 2 * kSock (their per-datagram sockets wait at the
                                    // interface): Glob::spk, never more than the qdisc queues hold
constexpr int kProcs = 8;           // processes per host
constexpr uint32_t kQ = 4096;       // per-socket packet queues
constexpr uint32_t kQc = 256;       // control-packet queue
constexpr uint32_t kTimers = 256;   // pending RTO timer expirations
constexpr uint32_t kSacks = 512;    // the receiver's SACK list
constexpr uint32_t kRanges = 64;    // tally ranges per set
constexpr uint32_t kKids = 8;
constexpr uint32_t kPoolDefault = 8192;   // packets per host (buffered, in flight, queued for retransmission)
constexpr uint32_t kPktSack = 128;  // SACK entries carried by one segment (the receive window's holes)
constexpr uint32_t kSt = 96;        // delivery statuses a packet's line lists (each loss retransmission adds 6)
constexpr uint32_t kEv = 8192;      // events per host
constexpr uint32_t kCq = 4096;      // CoDel queue per host
constexpr uint32_t kTr = 1u << 16;  // trace records per host
constexpr uint32_t kTrSack = 1u << 20;
#ifdef SHD_TCP_PROF
constexpr uint32_t kProf = 20, kProfRounds = 4096;   // steps timed per lane, rounds kept
#endif
constexpr uint32_t kMailMin = 1u << 16;   // mailbox slots per round: max(this, 16 per host)
// the mailbox in 64 parts with a fill counter each (host h claims in part h % 64,
// 32 slots per host), each lane folding the earliest delivery it sent into its
// own next time (measured against one counter and one atomicMin in round 4:
// profiles/r04/tcp); a full part spills into a shared overflow range (half the
// parts' size, its own counter), so one host with a wide window can send far
// more than its part in a round (a few hosts at ~1 Gbit/s and 50 ms latency)
constexpr uint32_t kMailSub = 64;
constexpr uint32_t kMailSack = 8;   // SACK entries per mailbox slot on average (their own arena)
constexpr uint32_t kPq = 8;         // vertex pairs a host remembers having queried (first-query log)
constexpr uint32_t kTrk = 10;       // tracker counters per direction (DHost::trk)
constexpr uint32_t kXRetx = 1;      // DPkt::xflags: the packet was retransmitted (PDS_SND_TCP_RETRANSMITTED)
constexpr uint32_t kXUdp = 2;       // DPkt::xflags: a datagram (PUDP, packet.c:320-321)
constexpr uint32_t kTrUdp = 1u << 31;   // TRec::flags: the record is a datagram's (packet_toString's PUDP form)
constexpr uint32_t kLocalRanks = 6;  // path_cache mode: rows a lane can run in one round (more: fall back)
constexpr int32_t kLocalRank0 = 0x7FFF0000;   // pseudo-ranks of a lane's in-round rows: past every real rank
enum : uint32_t { kFtRowA = 0, kFtRowB = 1, kFtSelf = 2 };

// ProtocolTCPFlags (protocol.h:23-31)
enum : uint32_t { F_RST = 1 << 1, F_SYN = 1 << 2, F_ACK = 1 << 3, F_SACK = 1 << 4, F_FIN = 1 << 5, F_DUPACK = 1 << 6 };
enum : uint8_t {
    S_SND_CREATED, S_SND_TCP_ENQUEUE_THROTTLED, S_SND_TCP_ENQUEUE_RETRANSMIT, S_SND_TCP_DEQUEUE_RETRANSMIT,
    S_SND_TCP_RETRANSMITTED, S_SND_SOCKET_BUFFERED, S_SND_INTERFACE_SENT, S_INET_SENT, S_INET_DROPPED,
    S_ROUTER_ENQUEUED, S_ROUTER_DEQUEUED, S_ROUTER_DROPPED, S_RCV_INTERFACE_RECEIVED, S_RCV_INTERFACE_DROPPED,
    S_RCV_SOCKET_PROCESSED, S_RCV_SOCKET_DROPPED, S_RCV_TCP_ENQUEUE_UNORDERED, S_RCV_SOCKET_BUFFERED,
    S_RCV_SOCKET_DELIVERED, S_DESTROYED
};
const char* const kStatusName[] = {
    "SND_CREATED", "SND_TCP_ENQUEUE_THROTTLED", "SND_TCP_ENQUEUE_RETRANSMIT", "SND_TCP_DEQUEUE_RETRANSMIT",
    "SND_TCP_RETRANSMITTED", "SND_SOCKET_BUFFERED", "SND_INTERFACE_SENT", "INET_SENT", "INET_DROPPED",
    "ROUTER_ENQUEUED", "ROUTER_DEQUEUED", "ROUTER_DROPPED", "RCV_INTERFACE_RECEIVED", "RCV_INTERFACE_DROPPED",
    "RCV_SOCKET_PROCESSED", "RCV_SOCKET_DROPPED", "RCV_TCP_ENQUEUE_UNORDERED", "RCV_SOCKET_BUFFERED",
    "RCV_SOCKET_DELIVERED", "PDS_DESTROYED"};
enum : uint32_t { Q_THROTTLED = 1, Q_UNORDERED = 2 };
enum : uint32_t { DS_ACTIVE = 1, DS_READABLE = 2, DS_WRITABLE = 4, DS_CLOSED = 8 };
enum { TS_CLOSED, TS_LISTEN, TS_SYNSENT, TS_SYNRECEIVED, TS_ESTABLISHED, TS_FINWAIT1, TS_FINWAIT2, TS_CLOSING,
       TS_TIMEWAIT, TS_CLOSEWAIT, TS_LASTACK };
enum : uint32_t { TF_LOCAL_CLOSED_RD = 1, TF_LOCAL_CLOSED_WR = 2, TF_REMOTE_CLOSED = 4, TF_EOF_RD_SIGNALED = 8,
                  TF_EOF_WR_SIGNALED = 16, TF_RESET_SIGNALED = 32, TF_WAS_ESTABLISHED = 64,
                  TF_CONNECT_SIGNALED = 128, TF_SHOULD_SEND_WR_FIN = 256 };
enum : uint32_t { TE_CONNECTION_RESET = 1, TE_SEND_EOF = 2, TE_RECEIVE_EOF = 4 };
enum : uint32_t { PF_PROCESSED = 1, PF_DATA_RECEIVED = 2, PF_DATA_ACKED = 4, PF_DATA_LOST = 16, PF_RWND_UPDATED = 32 };
enum { E_WOULDBLOCK = 11, E_INPROGRESS = 115, E_ALREADY = 114, E_ISCONN = 106, E_NOTCONN = 107, E_PIPE = 32,
       E_CONNRESET = 104, E_CONNREFUSED = 111 };
enum : uint32_t { K_HEARTBEAT, K_REFILL, K_REFILL_LO, K_PSTART, K_NOTIFY, K_DELIVER, K_DELACK, K_RTO, K_CLOSE,
                  K_WINUPD, K_LOCAL };
enum { T_SRV_START, T_SRV_ACCEPT, T_SRV_RECV, T_SRV_SEND, T_CLI_START, T_CLI_CONNECT, T_CLI_SEND, T_CLI_RECV,
       T_DONE };

struct DPkt {
    uint32_t host_id; int32_t refs;
    uint64_t pid;
    uint32_t flags, sip, dip;
    uint16_t sport, dport;
    uint32_t seq, ack, win, len;
    uint64_t tsval, tsecho;
    double prio;
    uint32_t nsack, nst;
    uint32_t inq, xflags;   // Q_THROTTLED / Q_UNORDERED: in its socket's heap (the reference's
                            // priority_queue membership lookup, O(1) instead of a scan)
    uint8_t st[kSt];
    // its SACK list (nsack entries) is out of line: Glob::psack at its pool slot,
    // Glob::msack while it travels (a copy moves this record only)
};
struct DEv { uint64_t time, seq; uint32_t src, kind; int32_t obj, pkt; };
struct Mail { uint32_t dst, src; uint64_t time, seq; uint32_t sack_off, _pad; DPkt pkt; };
static_assert(sizeof(DEv) == 32 && sizeof(Mail) == 216, "bench.py's algorithmic bytes of the TCP rounds");
struct TRec {
    uint64_t time; int32_t host; uint32_t status;
    uint32_t host_id, flags, sip, dip;
    uint64_t pid;
    uint16_t sport, dport; uint32_t seq, ack, win, len;
    uint64_t tsval, tsecho;
    uint32_t sack_off, nsack, nst;
    uint8_t st[kSt];
};
template <uint32_t N> struct Ring {   // GQueue
    uint32_t head, n;
    int32_t a[N];
};
template <uint32_t N> struct IHeap { uint32_t n; int32_t a[N]; };   // priority_queue.c over indices
// the same heap over packets ordered by TCP sequence, each entry carrying its
// key ((seq << 32) | pool index): a level is one load, not an index then the
// packet's sequence (a packet's sequence does not change while it is queued)
template <uint32_t N> struct KHeap { uint32_t n, kmax; uint64_t a[N]; };   // kmax >= every key held
template <uint32_t N> struct THeap { uint32_t n; uint64_t a[N]; };  // timer expirations
struct Rng64 { int64_t a, b; };
struct RVec { uint32_t n; Rng64 r[kRanges]; };
struct Tally { int64_t last_ack; uint64_t ndup; RVec marked, sacked, retx, lost, tmp; };

struct DSock {   // every scalar first (a few lines per socket), then the containers
    int16_t used, udp;      // udp: a datagram socket (udp.c), else TCP (the scalars' layout as before it)
    int32_t host, proc;
    uint32_t status;
    int32_t bound; uint32_t bound_ip; uint16_t bound_port, peer_port;
    uint32_t peer_ip;
    int32_t assoc, assoc_general;
    uint64_t in_len, in_size, in_pending, out_len, out_size, out_pending;
    int32_t state, state_last;
    uint32_t flags, error;
    uint32_t r_start, r_next, r_window, r_end, r_last_window, r_last_ack, r_last_seq;
    uint64_t r_last_ts; int32_t r_winupd;
    uint32_t s_unacked, s_next, s_window, s_end, s_last_ack, s_last_window, s_highest, s_packets_sent,
        s_quick_acks, s_delack_counter;
    int32_t s_delack_sched;
    uint32_t nsack;
    // the retransmit queue (tcp.c's GHashTable by sequence) as a sequence-sorted
    // window [rh, rh + nrtx) of rtx (packets) and rtxs (their sequences)
    uint32_t nrtx, rh; uint64_t rtx_len; int32_t rto; uint64_t desired;
    uint32_t backoff;
    int32_t at_did_init; uint64_t at_bytes, at_last_adjust, at_space;
    uint32_t cwnd; int32_t reno_state; uint64_t reno_ndup; uint32_t reno_nacked, reno_ssthresh;
    int32_t srtt, rttvar;
    uint64_t retx_count; uint32_t info_rtt;
    uint64_t throttled_len, unordered_len;
    int32_t partial; uint32_t partial_off;
    int32_t server; uint32_t nkids, npending;
    uint32_t last_peer_ip, last_ip; uint16_t last_peer_port;
    int32_t child, parent, child_state;
    // the path of this socket's last sent packet (host, vertex pair, latency,
    // reliability: constant over a run), keyed by its destination address
    uint32_t pc_ip; int32_t pc_host, pc_va, pc_vb; double pc_lat, pc_rel;
    int32_t kids[kKids], pending[kKids];
    Ring<kQc> outctl;
    THeap<kTimers> timers;
    Tally tally;
    KHeap<kQ> throttled;
    KHeap<kQ> unordered;
    Ring<kQ> in, out;
    int32_t sacks[kSacks];
    int32_t rtx[kQ]; uint32_t rtxs[kQ];
};
struct DProc {
    int32_t host, index, peer, running, step, fd, listenfd, wait_fd;
    int32_t app, _pad;   // >= 0: the datagram application app_spec[4 * app ..] (else the TCP echo)
    uint32_t wait_events, done;
    int32_t ep_ready, ep_scheduled, ep_notifying;
    uint64_t start;
};
struct DHost {
    uint32_t ip, rng, pkt_seq, err;
    uint64_t ev_seq, events, deliveries;
    double prio;
    uint64_t rx_rem, rx_cap, rx_refill, tx_rem, tx_cap, tx_refill;
    uint64_t bw_down, bw_up;   // configured KiB/s (worker_getNodeBandwidth{Down,Up})
    int32_t refill_pending, nsock, next_handle;
    IHeap<2 * kSock> fifo;
    Ring<2 * kSock> rrq;    // the RR qdisc's sockets wanting to send (rrQueue, network_interface.c:58)
    // CoDel (router_queue_codel.c)
    uint32_t cq_head, cq_n; uint64_t cq_total, cq_iexp, cq_next_drop; uint32_t cq_dc, cq_dc_last; int32_t cq_mode;
    uint32_t nfree, ntr, ntrs, nev;
    // the vertex pairs this host has queried (unordered, (min << 32) | max):
    // its first query of each goes to the run's first-query log (touch_log)
    uint32_t npq, nhb;
    uint64_t pq[kPq];
    // the tracker's interface counters of the running heartbeat interval
    // (tracker.c:183-214; the loopback task's packets included), inbound then
    // outbound, each in the counter string's order (tracker.c:391-417 without
    // the two totals): packets-control, bytes-control-header,
    // packets-control-retrans, bytes-control-header-retrans, packets-data,
    // bytes-data-header, bytes-data-payload, packets-data-retrans,
    // bytes-data-header-retrans, bytes-data-payload-retrans
    uint64_t trk[2 * kTrk];
};
struct CqEnt { uint64_t ts; uint32_t len; int32_t pkt; };

// the round driver's device-side state (the host only reads it between batches)
struct TCtl {
    uint64_t wend;       // the running round's window end
    uint64_t rounds;     // rounds started; round k reads mailbox k & 1 and writes the other
    uint32_t halted, sched_i;   // sched_i: the next entry of the first-touch schedule (Glob::sched_*)
    uint64_t max_mail;   // the most deliveries one round's mailbox took (shd_tcp_result)
    uint64_t max_ovf;    // ... and the most of them in its shared overflow range
    uint32_t ft_bad, ft_nr0;   // path_cache mode: a round's first-touch choice the serial order contradicts;
                               // next_rank before that round's replay
    uint64_t tmin;       // a group's round: this engine's earliest pending event (k_tcp_window, local)
    uint32_t xerr, _pad3;   // a group's exchange failed: SHD_TCP_ERR_MAILBOX / _INTERNAL bits
};

struct Glob {
    int32_t H, P;
    const double *lat, *rel;
    uint64_t end_time, hb, W, now_dummy;
    uint32_t tcp_bytes, trace, recv_buf, send_buf, tcp_window, _pad;
    DHost* host;
    DSock* sock;            // [H][spk]
    DProc* proc;            // [P]
    int32_t* host_procs;    // [H][kProcs]
    DPkt* pool;             // [H][pool_cap]
    int32_t* psack;         // [H][pool_cap][kPktSack] each pool slot's SACK list
    int32_t* freel;         // [H][pool_cap]
    const int32_t* hv;      // [H] host -> vertex (the path tables' index)
    int32_t V; uint32_t pool_cap;
    DEv* ev;                // [H][kEv] each host's event heap
    CqEnt* cq;              // [H][kCq]
    Mail* mail;             // [2][mail_cap] the two mailboxes (a round's input, its output)
    uint32_t* nmail;        // [2][kMailSub + 1] their fill counts (the parts', then the overflow's)
    int32_t* msack;         // [2][msack_cap] the SACK lists of the mails that carry one
    uint32_t* nmsack;       // [2] their fill counts
    uint32_t msack_cap, _pad4;
    int32_t* mhead;         // [2][H] each destination's list of mails (-1: none)
    int32_t* mnext;         // [2][mail_cap] the next mail of the same destination
    uint32_t mail_cap, mail_part;   // slots in all; slots per part (the overflow: the rest)
    uint32_t mail_stride, _pad8;    // a mailbox's slots: mail_cap, then a group's world * xcap from the others
    TCtl* ctl;
    const uint64_t* ip_key; // [ip_mask + 1] (ip << 32 | host), open addressing: host_of_ip's table
    uint32_t ip_mask, _pad5;
    Mail* mail_in; int32_t* mhead_in; int32_t* mnext_in;     // a lane's view of the round
    Mail* mail_out; uint32_t* n_out; int32_t* mhead_out; int32_t* mnext_out;
    const int32_t* msack_in; int32_t* msack_out; uint32_t* nmsack_out;
    TRec* tr;               // [H][kTr]
    int32_t* trs;           // [H][kTrSack]
    uint64_t* next_time;    // [H]
    shd_tcp_query* qlog;    // [qlog_cap] each host's first query of each vertex pair (touch_log)
    uint32_t* nqlog;
    uint32_t qlog_cap, _pad3;
    uint64_t* node;         // [H][node_k][2 * kTrk] tracker counters per heartbeat, or null
    uint32_t node_k, qdisc_rr;
    uint64_t* prof;         // SHD_TCP_PROF builds: [H][2 * kProf] cycles and counts per step
    uint32_t* prof_round;   // [2][kProfRounds] per round: the most events and cycles of a lane
    // path_cache mode (shd_tcp_model.path_cache): the cache's device tables
    // ([T][T] rows and direct values, [T] self values), the ranks as of the
    // round's start (kNoRank: never), and the round's log of queries whose
    // row depended on the order within the round (pc_query, k_tcp_window)
    const shd_pv *prow, *pself, *pdir;
    const uint8_t* padj;
    const int32_t* pself_eid;
    int32_t* rank;          // [T] row run order
    int32_t* srank;         // [T] self-path store order
    int32_t* next_rank;     // [1]
    shd_tcp_query* ft;      // [ft_cap] (_pad: the choice, kFtRowA / kFtRowB / kFtSelf)
    uint32_t* nft;
    int32_t* ftord;         // [ft_cap] the log in serial order (scratch of k_tcp_window)
    uint32_t ft_cap; int32_t pT;
    uint32_t pcm, pc_complete, pc_prefer_direct, sched_n;
    // the first-touch schedule (one engine): entry i ranks sched_v[sched_off[i],
    // sched_off[i + 1]) (v: a row, ~v: a self path) in that order when round
    // sched_round[i] opens, before it runs (tcp_run_impl's reruns)
    const uint32_t* sched_round;
    const uint32_t* sched_off;
    const int32_t* sched_v;
    // the datagram processes (shd_tcp_model.proc_app): their applications
    // {send, dest, n_start, per_read}, each host's SHD_DEST_PEER host, the
    // SHD_DEST_WEIGHTED rows ([n_classes][H] cumulative) and class per host
    const uint32_t* app_spec;
    const int32_t* app_peer;
    const double* dest_cum;
    const uint8_t* host_class;
    int32_t n_classes; uint32_t udp_payload;
    int32_t spk, _pad7;     // sockets per host
    // a run sharded over a group (shd_tcp_run_group): this engine's hosts
    // [h0, h0 + nloc) of the model's H (the per-host arrays hold these; one
    // engine: h0 = 0, nloc = H), every host's address and bandwidths, each
    // process's listening port (its owner publishes it: port_new), and the
    // round's deliveries for the other engines (per engine a segment: XSegHead,
    // xcap mails, xsack_cap SACK words)
    int32_t h0, nloc;
    const uint32_t* ip_all;
    const uint64_t* bwu_all;
    const uint64_t* bwd_all;
    uint32_t* proc_port;    // [P] 0: not listening (yet)
    uint32_t* nport_new;    // [1] this round's publications ...
    uint64_t* port_new;     // [pcap] ... (process << 32 | port)
    uint32_t pcap, _pad9;   // publications per engine and round at most: the most processes one engine has
    char* xsend;            // [world] segments
    int32_t world, me;
    uint32_t xcap, xsack_cap;
    size_t xseg;            // bytes per segment
};
struct XSegHead { uint32_t n, nsack, err, _pad[13]; };   // 64 B, then xcap Mails, then xsack_cap SACK words
static_assert(sizeof(XSegHead) == 64, "segment header");

// ------------------------------------------------------------ per-lane context
struct L {
    const Glob* g;
    int32_t h;              // the lane's host: its index in this engine's per-host arrays
    int32_t gh;             // ... and in the model (h0 + h): event keys, packet IDs, paths, logs
    DHost* H;
    uint64_t now;
    int32_t active;
    // the executing event's key (event_compare: time, this host, src, seq) and
    // the index of the next path query within it (first-query log)
    uint32_t ksrc, kq;
    uint64_t kseq;
    uint64_t mail_min;      // the earliest delivery this lane sent this round (part counters)
    // path_cache mode: the rows / self paths this lane's own queries ran in the
    // round so far (vertex * 2 + kind), in order: its pseudo-ranks
    uint32_t nlr;
    int32_t lr[kLocalRanks];
};
__device__ __forceinline__ DPkt* PK(const L& c, int32_t i) { return &c.g->pool[(size_t)c.h * c.g->pool_cap + i]; }
__device__ __forceinline__ int32_t* PSK(const L& c, int32_t i) {
    return c.g->psack + ((size_t)c.h * c.g->pool_cap + i) * kPktSack;
}
__device__ __forceinline__ int32_t sidx(const L& c, const DSock* k) { return (int32_t)(k - c.g->sock); }
__device__ __forceinline__ DSock* SK(const L& c, int32_t j) { return &c.g->sock[(size_t)c.h * c.g->spk + j]; }
// packet_getHeaderSize (packet.c:318-323)
__device__ __forceinline__ uint32_t hdr_of(const DPkt* p) { return (p->xflags & kXUdp) ? kHdrUdp : kHdr; }

__device__ int32_t rand_r_dev(uint32_t* state) {   // glibc rand_r (random.c's source)
    uint32_t next = *state;
    int32_t result;
    next *= 1103515245u; next += 12345u;
    result = (int32_t)((next / 65536u) % 2048u);
    next *= 1103515245u; next += 12345u;
    result <<= 10; result ^= (int32_t)((next / 65536u) % 1024u);
    next *= 1103515245u; next += 12345u;
    result <<= 10; result ^= (int32_t)((next / 65536u) % 1024u);
    *state = next;
    return result;
}
// the state after n steps of rand_r's LCG (x -> 1103515245 x + 12345 mod 2^32)
// in O(log n): powers of one affine map compose in any order
__device__ uint32_t lcg_jump(uint32_t x, uint64_t n) {
    uint32_t a = 1103515245u, b = 12345u, ra = 1u, rb = 0u;
    for (; n; n >>= 1) {
        if (n & 1) { ra = a * ra; rb = a * rb + b; }
        b = a * b + b;
        a = a * a;
    }
    return ra * x + rb;
}
__device__ double next_double(uint32_t* s) { return (double)(((double)rand_r_dev(s)) / ((double)2147483647)); }

// ------------------------------------------------------------ heaps (priority_queue.c)
template <uint32_t N, class Less> __device__ uint32_t ih_up(IHeap<N>& q, uint32_t i, Less lt) {
    while (i > 0 && lt(q.a[i], q.a[(i - 1) / 2])) { int32_t t = q.a[i]; q.a[i] = q.a[(i - 1) / 2]; q.a[(i - 1) / 2] = t; i = (i - 1) / 2; }
    return i;
}
template <uint32_t N, class Less> __device__ uint32_t ih_down(IHeap<N>& q, uint32_t i, Less lt) {
    uint32_t ch;
    while ((ch = 2 * i + 1) < q.n) {
        if (ch + 1 < q.n && lt(q.a[ch + 1], q.a[ch])) ch = ch + 1;
        if (lt(q.a[ch], q.a[i])) { int32_t t = q.a[i]; q.a[i] = q.a[ch]; q.a[ch] = t; i = ch; } else break;
    }
    return i;
}
template <uint32_t N> __device__ int ih_find(const IHeap<N>& q, int32_t x) {
    for (uint32_t i = 0; i < q.n; i++) if (q.a[i] == x) return (int)i;
    return -1;
}
template <uint32_t N, class Less> __device__ bool ih_push(IHeap<N>& q, int32_t x, Less lt, uint32_t& err) {
    const int old = ih_find(q, x);
    if (old >= 0) { ih_up(q, ih_down(q, (uint32_t)old, lt), lt); return false; }
    if (q.n >= N) { err |= SHD_TCP_ERR_QUEUE; return false; }
    q.a[q.n++] = x;
    ih_up(q, q.n - 1, lt);
    return true;
}
// push of an element known to be absent (its membership is tracked outside)
template <uint32_t N, class Less> __device__ bool ih_push_new(IHeap<N>& q, int32_t x, Less lt, uint32_t& err) {
    if (q.n >= N) { err |= SHD_TCP_ERR_QUEUE; return false; }
    q.a[q.n++] = x;
    ih_up(q, q.n - 1, lt);
    return true;
}
template <uint32_t N, class Less> __device__ int32_t ih_pop(IHeap<N>& q, Less lt) {
    if (!q.n) return -1;
    const int32_t x = q.a[0];
    q.a[0] = q.a[q.n - 1];
    q.a[q.n - 1] = x;
    q.n--;
    ih_down(q, 0, lt);
    return x;
}
// packet_compareTCPSequence (packet.c:207-221) on the entries' keys; the
// swaps are ih_up's / ih_down's, so ties resolve as the reference heap's do
__device__ __forceinline__ bool kh_less(uint64_t x, uint64_t y) { return (uint32_t)(x >> 32) < (uint32_t)(y >> 32); }
template <uint32_t N> __device__ void kh_up(KHeap<N>& q, uint32_t i) {
    while (i > 0 && kh_less(q.a[i], q.a[(i - 1) / 2])) {
        const uint64_t t = q.a[i]; q.a[i] = q.a[(i - 1) / 2]; q.a[(i - 1) / 2] = t; i = (i - 1) / 2;
    }
}
template <uint32_t N> __device__ void kh_down(KHeap<N>& q, uint32_t i) {
    uint32_t ch;
    while ((ch = 2 * i + 1) < q.n) {
        if (ch + 1 < q.n && kh_less(q.a[ch + 1], q.a[ch])) ch = ch + 1;
        if (kh_less(q.a[ch], q.a[i])) { const uint64_t t = q.a[i]; q.a[i] = q.a[ch]; q.a[ch] = t; i = ch; } else break;
    }
}
template <uint32_t N> __device__ bool kh_push_new(KHeap<N>& q, int32_t x, uint32_t seq, uint32_t& err) {
    if (q.n >= N) { err |= SHD_TCP_ERR_QUEUE; return false; }
    const bool last = q.n == 0 || seq >= q.kmax;   // not below any key: no parent is greater (no swap)
    q.a[q.n++] = ((uint64_t)seq << 32) | (uint32_t)x;
    if (!last) kh_up(q, q.n - 1);
    if (q.n == 1 || seq > q.kmax) q.kmax = seq;
    return true;
}
template <uint32_t N> __device__ __forceinline__ int32_t kh_top(const KHeap<N>& q) { return (int32_t)(uint32_t)q.a[0]; }
template <uint32_t N> __device__ void kh_pop(KHeap<N>& q) {
    if (!q.n) return;
    const uint64_t x = q.a[0];
    q.a[0] = q.a[q.n - 1];
    q.a[q.n - 1] = x;
    q.n--;
    kh_down(q, 0);
}
template <uint32_t N> __device__ void th_push(THeap<N>& q, uint64_t x, uint32_t& err) {
    if (q.n >= N) { err |= SHD_TCP_ERR_QUEUE; return; }
    uint32_t i = q.n++;
    q.a[i] = x;
    while (i > 0 && q.a[i] < q.a[(i - 1) / 2]) { uint64_t t = q.a[i]; q.a[i] = q.a[(i - 1) / 2]; q.a[(i - 1) / 2] = t; i = (i - 1) / 2; }
}
template <uint32_t N> __device__ void th_pop(THeap<N>& q) {
    if (!q.n) return;
    uint64_t x = q.a[0];
    q.a[0] = q.a[q.n - 1];
    q.a[q.n - 1] = x;
    q.n--;
    uint32_t i = 0, ch;
    while ((ch = 2 * i + 1) < q.n) {
        if (ch + 1 < q.n && q.a[ch + 1] < q.a[ch]) ch = ch + 1;
        if (q.a[ch] < q.a[i]) { uint64_t t = q.a[i]; q.a[i] = q.a[ch]; q.a[ch] = t; i = ch; } else break;
    }
}
template <uint32_t N> __device__ void rg_push(Ring<N>& r, int32_t x, uint32_t& err) {
    if (r.n >= N) { err |= SHD_TCP_ERR_QUEUE; return; }
    r.a[(r.head + r.n) % N] = x;
    r.n++;
}
template <uint32_t N> __device__ int32_t rg_peek(const Ring<N>& r) { return r.n ? r.a[r.head] : -1; }
template <uint32_t N> __device__ int32_t rg_pop(Ring<N>& r) {
    if (!r.n) return -1;
    const int32_t x = r.a[r.head];
    r.head = (r.head + 1) % N;
    r.n--;
    return x;
}

// ------------------------------------------------------------ event heap (event.c:110-153)
__device__ __forceinline__ bool ev_less(const DEv& a, const DEv& b) {
    if (a.time != b.time) return a.time < b.time;
    if (a.src != b.src) return a.src < b.src;
    return a.seq < b.seq;
}
// A binary heap per host (a 4-ary heap with a node's four children on one
// 128-B line was measured: 19.85 against 19.88 M TCP events/s, not kept).
// Keys (time, src, seq) are unique, so any heap pops in the same order.
__device__ __forceinline__ DEv* evq_base(const Glob* g, int32_t h) { return g->ev + (size_t)h * kEv; }
__device__ void evq_push(const L& c, const DEv& e) {
    DEv* q = evq_base(c.g, c.h);
    uint32_t& n = c.H->nev;
    if (n >= kEv) { c.H->err |= SHD_TCP_ERR_EVQ; return; }
    uint32_t i = n++;
    while (i > 0) {
        const uint32_t p = (i - 1) / 2;
        if (!ev_less(e, q[p])) break;
        q[i] = q[p];
        i = p;
    }
    q[i] = e;
}
__device__ DEv evq_pop(const L& c) {
    DEv* q = evq_base(c.g, c.h);
    uint32_t& n = c.H->nev;
    const DEv top = q[0], last = q[--n];
    uint32_t i = 0;
    for (;;) {
        const uint32_t l = 2 * i + 1, r = l + 1;
        uint32_t m = i;
        const DEv* best = &last;
        if (l < n && ev_less(q[l], *best)) { m = l; best = &q[l]; }
        if (r < n && ev_less(q[r], *best)) { m = r; best = &q[r]; }
        if (m == i) break;
        q[i] = q[m];
        i = m;
    }
    if (n) q[i] = last;
    return top;
}
// event_new_ consumes the source's ID; scheduler_push drops past the end (scheduler.c:342-357)
__device__ bool sched_task(L& c, uint64_t delay, uint32_t kind, int32_t obj) {
    DEv e;
    e.time = c.now + delay; e.seq = c.H->ev_seq++; e.src = (uint32_t)c.gh; e.kind = kind; e.obj = obj; e.pkt = -1;
    if (e.time >= c.g->end_time) return false;
    evq_push(c, e);
    return true;
}

// ------------------------------------------------------------ packets and their lines
__device__ void pkt_status(L& c, int32_t pi, uint8_t st) {   // packet_addDeliveryStatus (packet.c:647-659)
    DPkt* p = PK(c, pi);
    DHost* H = c.H;
    if (st == S_SND_TCP_RETRANSMITTED) p->xflags |= kXRetx;   // packet_getDeliveryStatus's OR of every status
    if (!c.g->trace) return;   // the list is read by the lines only
    if (p->nst < kSt) p->st[p->nst++] = st;
    else H->err |= SHD_TCP_ERR_TRACE;   // a line would lose statuses: fail, never truncate
    if (H->ntr >= kTr) { H->err |= SHD_TCP_ERR_TRACE; return; }
    TRec* r = &c.g->tr[(size_t)c.h * kTr + H->ntr++];
    r->time = c.now; r->host = c.active; r->status = st;
    r->host_id = p->host_id; r->pid = p->pid; r->flags = p->flags | ((p->xflags & kXUdp) ? kTrUdp : 0u);
    r->sip = p->sip; r->dip = p->dip;
    r->sport = p->sport; r->dport = p->dport; r->seq = p->seq; r->ack = p->ack; r->win = p->win; r->len = p->len;
    r->tsval = p->tsval; r->tsecho = p->tsecho; r->nst = p->nst;
    for (uint32_t i = 0; i < p->nst; i++) r->st[i] = p->st[i];
    r->sack_off = H->ntrs; r->nsack = p->nsack;
    if (H->ntrs + p->nsack > kTrSack) { H->err |= SHD_TCP_ERR_TRACE; r->nsack = 0; return; }
    const int32_t* sk = PSK(c, pi);
    for (uint32_t i = 0; i < p->nsack; i++) c.g->trs[(size_t)c.h * kTrSack + H->ntrs + i] = sk[i];
    H->ntrs += p->nsack;
}
__device__ int32_t pkt_alloc(L& c) {
    DHost* H = c.H;
    if (!H->nfree) { H->err |= SHD_TCP_ERR_POOL; return -1; }
    return c.g->freel[(size_t)c.h * c.g->pool_cap + --H->nfree];
}
__device__ int32_t pkt_new(L& c, uint32_t len) {   // packet_new (packet.c:74-95)
    const int32_t i = pkt_alloc(c);
    if (i < 0) return -1;
    DPkt* p = PK(c, i);
    memset(p, 0, c.g->trace ? sizeof(DPkt) : offsetof(DPkt, st));
    p->refs = 1;
    p->host_id = (uint32_t)c.gh + 1;
    p->pid = c.H->pkt_seq++;
    p->len = len;
    if (len > 0) p->prio = ++c.H->prio;   // host_getNextPacketPriority (host.c:1663-1666)
    return i;
}
__device__ void pkt_ref(L& c, int32_t i) { PK(c, i)->refs++; }
// a packet record copied: its status list only when lines are written (no
// other reader)
__device__ __forceinline__ void pkt_copy_rec(DPkt* d, const DPkt* p, bool st) {
    if (st) { *d = *p; return; }
    static_assert(offsetof(DPkt, st) % 8 == 0, "the record's head in 8-B words");
    const uint64_t* a = (const uint64_t*)p;
    uint64_t* b = (uint64_t*)d;
#pragma unroll
    for (uint32_t i = 0; i < offsetof(DPkt, st) / 8; i++) b[i] = a[i];
}
__device__ void pkt_unref(L& c, int32_t i) {   // packet.c:194-201
    DPkt* p = PK(c, i);
    if (--p->refs == 0) {
        pkt_status(c, i, S_DESTROYED);
        c.g->freel[(size_t)c.h * c.g->pool_cap + c.H->nfree++] = i;
    }
}

// ------------------------------------------------------------ epoll (one watch per process)
__device__ bool watch_ready(const L& c, const DProc* pr) {
    if (pr->wait_fd < 0) return false;
    const DSock* k = &c.g->sock[pr->wait_fd];
    if ((k->status & DS_CLOSED) || !(k->status & DS_ACTIVE)) return false;
    return ((k->status & DS_READABLE) && (pr->wait_events & 1)) || ((k->status & DS_WRITABLE) && (pr->wait_events & 4));
}
__device__ void ep_schedule(L& c, DProc* pr) {   // _epoll_scheduleNotification (epoll.c:345-366)
    if (pr->ep_notifying) return;
    if (!pr->ep_scheduled && pr->running)
        if (sched_task(c, 1, K_NOTIFY, pr->index)) pr->ep_scheduled = 1;
}
__device__ void ep_status_changed(L& c, DProc* pr) {   // epoll_descriptorStatusChanged (epoll.c:585-615)
    pr->ep_ready = watch_ready(c, pr);
    if (pr->ep_ready) ep_schedule(c, pr);
}
__device__ void sock_status(L& c, DSock* k, uint32_t bits, bool set) {   // descriptor_adjustStatus
    if (set) k->status |= bits; else k->status &= ~bits;
    if (k->proc >= 0) {
        DProc* pr = &c.g->proc[k->proc];
        if (pr->wait_fd == sidx(c, k)) ep_status_changed(c, pr);
    }
}

// ------------------------------------------------------------ socket buffers (socket.c)
__device__ __forceinline__ uint64_t in_size(const DSock* k) { return k->in_pending ? k->in_pending : k->in_size; }
__device__ __forceinline__ uint64_t out_size(const DSock* k) { return k->out_pending ? k->out_pending : k->out_size; }
__device__ __forceinline__ uint64_t in_space(const DSock* k) { const uint64_t s = in_size(k); return s < k->in_len ? 0 : s - k->in_len; }
__device__ __forceinline__ uint64_t out_space(const DSock* k) { const uint64_t s = out_size(k); return s < k->out_len ? 0 : s - k->out_len; }
__device__ void set_in_size(DSock* k, uint64_t n) {
    if (n >= k->in_len) { k->in_size = n; k->in_pending = 0; } else { k->in_size = k->in_len; k->in_pending = n; }
}
__device__ void set_out_size(DSock* k, uint64_t n) {
    if (n >= k->out_len) { k->out_size = n; k->out_pending = 0; } else { k->out_size = k->out_len; k->out_pending = n; }
}
__device__ __forceinline__ uint64_t tcp_out_len(const DSock* k) { return k->throttled_len + k->rtx_len; }
__device__ uint64_t space_out(const DSock* k) {
    const int64_t s = (int64_t)out_space(k) - (int64_t)tcp_out_len(k);
    return s > 0 ? (uint64_t)s : 0;
}
__device__ uint64_t space_in(const DSock* k) {
    const int64_t s = (int64_t)in_space(k) - (int64_t)k->unordered_len;
    return s > 0 ? (uint64_t)s : 0;
}
__device__ uint64_t space_out_incl_tcp(const DSock* k) {
    const uint64_t sp = out_space(k), tl = tcp_out_len(k);
    return tl < sp ? sp - tl : 0;
}
__device__ int32_t sock_peek_out(const L& c, const DSock* k) { return k->outctl.n ? rg_peek(k->outctl) : rg_peek(k->out); }
struct SockLess {   // _networkinterface_compareSocket: never equal
    const L* c;
    __device__ bool operator()(int32_t a, int32_t b) const {
        const DPkt* pa = PK(*c, sock_peek_out(*c, &c->g->sock[a]));
        const DPkt* pb = PK(*c, sock_peek_out(*c, &c->g->sock[b]));
        return !(pa->prio > pb->prio);
    }
};

__device__ void if_send_packets(L& c);
__device__ void udp_release(L& c, DSock* k);
__device__ bool sock_add_input(L& c, DSock* k, int32_t pi) {   // socket.c:319-343
    DPkt* p = PK(c, pi);
    if (p->len > in_space(k)) return false;
    rg_push(k->in, pi, c.H->err);
    pkt_ref(c, pi);
    k->in_len += p->len;
    pkt_status(c, pi, S_RCV_SOCKET_BUFFERED);
    if (k->in_len > 0) sock_status(c, k, DS_READABLE, true);
    return true;
}
__device__ int32_t sock_remove_input(L& c, DSock* k) {   // socket.c:345-372
    const int32_t pi = rg_pop(k->in);
    if (pi >= 0) {
        k->in_len -= PK(c, pi)->len;
        if (k->in_pending > 0) set_in_size(k, k->in_pending);
        if (k->in_len <= 0) sock_status(c, k, DS_READABLE, false);
    }
    return pi;
}
__device__ bool sock_add_output(L& c, DSock* k, int32_t pi) {   // socket.c:385-424
    DPkt* p = PK(c, pi);
    if (p->len > out_space(k)) return false;
    if (p->prio == 0.0) rg_push(k->outctl, pi, c.H->err); else rg_push(k->out, pi, c.H->err);
    k->out_len += p->len;
    pkt_status(c, pi, S_SND_SOCKET_BUFFERED);
    if (space_out_incl_tcp(k) <= 0) sock_status(c, k, DS_WRITABLE, false);
    // networkinterface_wantsSend (network_interface.c:581-605): tracked once
    if (c.g->qdisc_rr) {
        bool found = false;   // g_queue_find
        for (uint32_t i = 0; i < c.H->rrq.n; i++)
            found |= c.H->rrq.a[(c.H->rrq.head + i) % (2 * kSock)] == sidx(c, k);
        if (!found) rg_push(c.H->rrq, sidx(c, k), c.H->err);
    } else if (ih_find(c.H->fifo, sidx(c, k)) < 0) {
        ih_push(c.H->fifo, sidx(c, k), SockLess{&c}, c.H->err);
    }
    if_send_packets(c);
    return true;
}
__device__ int32_t sock_remove_output(L& c, DSock* k) {   // socket.c:426-451
    const int32_t pi = k->outctl.n ? rg_pop(k->outctl) : rg_pop(k->out);
    if (pi >= 0) {
        k->out_len -= PK(c, pi)->len;
        if (k->out_pending > 0) set_out_size(k, k->out_pending);
        if (space_out_incl_tcp(k) > 0) sock_status(c, k, DS_WRITABLE, true);
    }
    return pi;
}

// ------------------------------------------------------------ paths
// the first host holding ip (dns.c: one address per host), by binary search
// over the sorted (ip, host) keys
// the host of an address: a hash table with linear probing, a lookup one
// line in the common case (a binary search over the sorted addresses was 17
// dependent loads at 65 536 hosts, on every packet sent)
__host__ __device__ __forceinline__ uint32_t ip_slot(uint32_t ip, uint32_t mask) { return (ip * 0x9E3779B1u) >> 7 & mask; }
__device__ int32_t host_of_ip(const L& c, uint32_t ip) {
    const uint64_t* k = c.g->ip_key;
    const uint32_t mask = c.g->ip_mask;
    for (uint32_t i = ip_slot(ip, mask), n = 0; n <= mask; i = (i + 1) & mask, n++) {
        const uint64_t v = k[i];
        if (v == ~0ull) return -1;
        if ((uint32_t)(v >> 32) == ip) return (int32_t)(uint32_t)v;
    }
    return -1;
}
// A path query of the executing event (topology_isRoutable / getLatency /
// getReliability, topology.c:2053-2092).  Which endpoint's Dijkstra row serves
// a pair depends on the serial order of every pair's FIRST query
// (_topology_getPathEntry, topology.c:1969-2051): the host's
// first query of each vertex pair is logged with the event's key, so the
// caller can rank the run's first touches in serial order afterwards and
// check the tables it passed against them (shadow-1_amd/tcp.py)
__device__ void touch_log(L& c, int32_t va, int32_t vb) {
    const uint32_t q = c.kq++;
    const uint64_t key = va < vb ? ((uint64_t)(uint32_t)va << 32) | (uint32_t)vb
                                 : ((uint64_t)(uint32_t)vb << 32) | (uint32_t)va;
    DHost* H = c.H;
    const uint32_t n = H->npq < kPq ? H->npq : kPq;
    for (uint32_t i = 0; i < n; i++)
        if (H->pq[i] == key) return;
    if (H->npq < kPq) H->pq[H->npq] = key;
    H->npq++;   // past kPq every unremembered pair's query is logged (a superset: harmless)
    const uint32_t slot = atomicAdd(c.g->nqlog, 1u);
    if (slot >= c.g->qlog_cap) { H->err |= SHD_TCP_ERR_QLOG; return; }
    shd_tcp_query r;
    r.time = c.now; r.seq = c.kseq; r.host = (uint32_t)c.gh; r.src = c.ksrc; r.index = q;
    r.v_src = va; r.v_dst = vb; r._pad = 0;
    c.g->qlog[slot] = r;
}

// the path entry of hosts a -> b; an unknown host or a pair with no route
// (latency < 0: shd_tcp_run refuses models whose connections have one, so
// this is an internal error) fails the run instead of scheduling a delivery
// at a negative delay
// path_cache mode: the lazy cache's rule (pathcache.hip pc_lookup_at,
// topology.c:1969-2051) on the device.  A pair with a ranked endpoint at the
// round's start is decided: the lower-ranked endpoint's row (self pairs: the
// self path or the row, by the same rule).  A pair with none depends on the
// order of the round's first touches: the lane decides it as the serial loop
// would if no other lane touched these vertices earlier in the window -- the
// round-start ranks plus its own earlier rows of the round (pseudo-ranks) --
// and logs the query with its key and choice; k_tcp_window replays the log in
// serial order, ranks the rows that ran and checks every choice.
__device__ int32_t eff_rank(const L& c, int32_t v, uint32_t kind) {
    const int32_t r = kind ? c.g->srank[v] : c.g->rank[v];
    if (r != kNoRank) return r;
    const int32_t key = v * 2 + (int32_t)kind;
    for (uint32_t p = 0; p < c.nlr && p < kLocalRanks; p++)
        if (c.lr[p] == key) return kLocalRank0 + (int32_t)p;
    return kNoRank;
}
__device__ void ft_log(L& c, int32_t va, int32_t vb, uint32_t choice) {
    const uint32_t slot = atomicAdd(c.g->nft, 1u);
    if (slot >= c.g->ft_cap) { c.H->err |= SHD_TCP_ERR_FIRST_TOUCH; return; }
    shd_tcp_query r;
    r.time = c.now; r.seq = c.kseq; r.host = (uint32_t)c.gh; r.src = c.ksrc; r.index = c.kq - 1;
    r.v_src = va; r.v_dst = vb; r._pad = choice;
    c.g->ft[slot] = r;
}
__device__ void ft_run_local(L& c, int32_t v, uint32_t kind) {
    if (c.nlr >= kLocalRanks) { c.H->err |= SHD_TCP_ERR_FIRST_TOUCH; return; }
    c.lr[c.nlr++] = v * 2 + (int32_t)kind;
}
// the query of vertex pair (va, vb); want: the value is used (not only the
// first touch of topology_isRoutable)
__device__ void pc_query(L& c, int32_t va, int32_t vb, double& lat, double& rel) {
    const Glob& g = *c.g;
    const size_t T = (size_t)g.pT;
    c.kq++;
    shd_pv v{-1.0, -1.0};
    if (g.pc_complete || (g.pc_prefer_direct && g.padj[(size_t)va * T + vb])) {
        v = g.pdir[(size_t)va * T + vb];
        if (isnan(v.lat)) v = shd_pv{-1.0, -1.0};
    } else if (va == vb) {
        const int32_t ra0 = g.rank[va], rs0 = g.srank[va];
        bool self;
        if (ra0 == kNoRank && rs0 == kNoRank) {
            const int32_t ra = eff_rank(c, va, 0), rs = eff_rank(c, va, 1);
            if (ra == kNoRank && rs == kNoRank) { ft_run_local(c, va, 1); self = true; }
            else self = rs < ra;
            ft_log(c, va, vb, self ? kFtSelf : kFtRowA);
        } else {
            self = rs0 < ra0;
        }
        v = self ? g.pself[va] : g.prow[(size_t)va * T + va];
    } else {
        const int32_t ra0 = g.rank[va], rb0 = g.rank[vb];
        bool own;
        bool fail = false;
        if (ra0 == kNoRank && rb0 == kNoRank) {
            const int32_t ra = eff_rank(c, va, 0), rb = eff_rank(c, vb, 0);
            if (ra == kNoRank && rb == kNoRank) {   // a miss: va's row runs (and fails without a self-loop)
                ft_run_local(c, va, 0);
                own = true;
                fail = g.pself_eid[va] < 0;
            } else {
                own = ra != kNoRank && (rb == kNoRank || ra < rb);
            }
            ft_log(c, va, vb, own ? kFtRowA : kFtRowB);
        } else {
            own = ra0 != kNoRank && (rb0 == kNoRank || ra0 < rb0);
        }
        if (!fail) v = own ? g.prow[(size_t)va * T + vb] : g.prow[(size_t)vb * T + va];
    }
    lat = v.lat;
    rel = v.rel;
}

__device__ void path(L& c, int32_t a, int32_t b, double& lat, double& rel) {
    if (a < 0 || b < 0) {
        c.H->err |= SHD_TCP_ERR_INTERNAL;
        lat = 1.0; rel = 0.0;
        return;
    }
    if (c.g->pcm) {
        pc_query(c, c.g->hv[a], c.g->hv[b], lat, rel);
    } else {
        touch_log(c, c.g->hv[a], c.g->hv[b]);
        const size_t i = (size_t)c.g->hv[a] * (size_t)c.g->V + (size_t)c.g->hv[b];
        lat = c.g->lat[i];
        rel = c.g->rel[i];
    }
    if (!(lat >= 0.0)) {
        c.H->err |= SHD_TCP_ERR_INTERNAL;
        lat = 1.0; rel = 0.0;
    }
}

// ------------------------------------------------------------ retransmit queue
// logical index i of the window is physical rh + i; sequences are unique
__device__ uint32_t rtx_lower(const DSock* k, uint32_t seq) {   // first i with seq_i >= seq
    uint32_t lo = 0, hi = k->nrtx;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (k->rtxs[k->rh + mid] < seq) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ int rtx_find(const L& c, const DSock* k, uint32_t seq) {
    const uint32_t i = rtx_lower(k, seq);
    return (i < k->nrtx && k->rtxs[k->rh + i] == seq) ? (int)i : -1;
}
__device__ __forceinline__ int32_t rtx_at(const DSock* k, uint32_t i) { return k->rtx[k->rh + i]; }
__device__ void rtx_remove_at(DSock* k, uint32_t i) {   // shifts the shorter side
    if (i < k->nrtx - 1 - i) {
        for (uint32_t j = i; j > 0; j--) {
            k->rtx[k->rh + j] = k->rtx[k->rh + j - 1];
            k->rtxs[k->rh + j] = k->rtxs[k->rh + j - 1];
        }
        k->rh++;
    } else {
        for (uint32_t j = i; j + 1 < k->nrtx; j++) {
            k->rtx[k->rh + j] = k->rtx[k->rh + j + 1];
            k->rtxs[k->rh + j] = k->rtxs[k->rh + j + 1];
        }
    }
    if (--k->nrtx == 0) k->rh = 0;
}
__device__ bool rtx_insert(DSock* k, int32_t pi, uint32_t seq, uint32_t& err) {
    if (k->nrtx >= kQ) { err |= SHD_TCP_ERR_QUEUE; return false; }
    if (k->rh + k->nrtx == kQ) {   // the window reached the end: move it to the front
        for (uint32_t j = 0; j < k->nrtx; j++) { k->rtx[j] = k->rtx[k->rh + j]; k->rtxs[j] = k->rtxs[k->rh + j]; }
        k->rh = 0;
    }
    uint32_t i = k->nrtx;
    while (i > 0 && k->rtxs[k->rh + i - 1] > seq) {   // from the end: sends append in order
        k->rtx[k->rh + i] = k->rtx[k->rh + i - 1];
        k->rtxs[k->rh + i] = k->rtxs[k->rh + i - 1];
        i--;
    }
    k->rtx[k->rh + i] = pi;
    k->rtxs[k->rh + i] = seq;
    k->nrtx++;
    return true;
}
__device__ void tcp_add_retransmit(L& c, DSock* k, int32_t pi) {   // tcp.c:854-873
    DPkt* p = PK(c, pi);
    if (rtx_find(c, k, p->seq) >= 0) return;
    if (!rtx_insert(k, pi, p->seq, c.H->err)) return;
    pkt_ref(c, pi);
    pkt_status(c, pi, S_SND_TCP_ENQUEUE_RETRANSMIT);
    k->rtx_len += p->len;
    if (space_out(k) == 0) sock_status(c, k, DS_WRITABLE, false);
}
__device__ void tcp_clear_retransmit(L& c, DSock* k, uint32_t seq) {   // tcp.c:876-897 (sequence order)
    while (k->nrtx && k->rtxs[k->rh] < seq) {   // the lowest sequence below `seq` first
        const int32_t pi = rtx_at(k, 0);
        k->rtx_len -= PK(c, pi)->len;
        pkt_status(c, pi, S_SND_TCP_DEQUEUE_RETRANSMIT);
        rtx_remove_at(k, 0);
        pkt_unref(c, pi);
    }
    if (space_out(k) > 0) sock_status(c, k, DS_WRITABLE, true);
}
__device__ void tcp_clear_retransmit_range(L& c, DSock* k, uint32_t begin, uint32_t end) {   // tcp.c:900-920
    // the sequences in [begin, end) present, ascending (a run of the window)
    const uint32_t at = rtx_lower(k, begin);
    while (at < k->nrtx && k->rtxs[k->rh + at] < end) {
        const int32_t pi = rtx_at(k, at);
        k->rtx_len -= PK(c, pi)->len;
        pkt_status(c, pi, S_SND_TCP_DEQUEUE_RETRANSMIT);
        rtx_remove_at(k, at);
        pkt_unref(c, pi);
    }
    if (space_out(k) > 0) sock_status(c, k, DS_WRITABLE, true);
}

// ------------------------------------------------------------ the retransmit tally (tcp_retransmit_tally.cc)
__device__ void rv_insert_at(RVec& v, uint32_t at, int64_t a, int64_t b, uint32_t& err) {
    if (v.n >= kRanges) { err |= SHD_TCP_ERR_QUEUE; return; }
    for (uint32_t j = v.n; j > at; j--) v.r[j] = v.r[j - 1];
    v.r[at].a = a; v.r[at].b = b; v.n++;
}
__device__ void rv_push(RVec& v, int64_t a, int64_t b, uint32_t& err) { rv_insert_at(v, v.n, a, b, err); }
__device__ __forceinline__ bool r_overlap(Rng64 x, Rng64 y) { return x.a < y.b && y.a < x.b; }
__device__ __forceinline__ bool r_adj(Rng64 x, Rng64 y) { return x.b == y.a || y.b == x.a; }
__device__ void ranges_insert(RVec& v, int64_t a, int64_t b, uint32_t& err) {   // cc:57-102
    const Rng64 val = {a, b};
    uint32_t first = v.n, it = 0;
    for (; it < v.n && val.b >= v.r[it].a; ++it)
        if (first == v.n && (r_overlap(v.r[it], val) || r_adj(v.r[it], val))) first = it;
    const uint32_t second = it;
    if (first == v.n) { rv_insert_at(v, second, a, b, err); return; }
    Rng64& x = v.r[first];
    if (val.a < x.a) x.a = val.a;
    if (val.b > x.b) x.b = val.b;
    for (uint32_t j = first + 1; j < second; j++) {
        if (v.r[j].a < x.a) x.a = v.r[j].a;
        if (v.r[j].b > x.b) x.b = v.r[j].b;
    }
    const uint32_t ne = second - (first + 1);
    for (uint32_t j = second; j < v.n; j++) v.r[j - ne] = v.r[j];
    v.n -= ne;
}
__device__ void ranges_subtract(const RVec& lhs, const RVec& rhs, RVec& out, uint32_t& err) {   // cc:104-175
    out.n = 0;
    if (rhs.n == 0) { for (uint32_t i = 0; i < lhs.n; i++) rv_push(out, lhs.r[i].a, lhs.r[i].b, err); return; }
    if (lhs.n == 0) return;
    uint32_t idx = 0, j = 0;
    Rng64 cur = lhs.r[0];
    while (idx < lhs.n && j < rhs.n) {
        const Rng64 rj = rhs.r[j];
        if (rj.b <= cur.a) {
            ++j;
        } else if (cur.b <= rj.a) {
            rv_push(out, cur.a, cur.b, err);
            ++idx;
            if (idx < lhs.n) cur = lhs.r[idx];
        } else {
            Rng64 sub[2]; int ns = 0;
            if (r_overlap(cur, rj)) {
                if (cur.a < rj.a) { sub[ns].a = cur.a; sub[ns].b = rj.a; ns++; }
                if (rj.b < cur.b) { sub[ns].a = rj.b; sub[ns].b = cur.b; ns++; }
            } else {
                sub[ns++] = cur;
            }
            if (ns == 2) rv_push(out, sub[0].a, sub[0].b, err);
            if (ns >= 1) cur = sub[ns - 1];
            else { ++idx; if (idx < lhs.n) cur = lhs.r[idx]; }
        }
    }
    if (j == rhs.n) {
        rv_push(out, cur.a, cur.b, err);
        ++idx;
        while (idx < lhs.n) { rv_push(out, lhs.r[idx].a, lhs.r[idx].b, err); idx++; }
    }
}
__device__ void tally_compute_lost(Tally& t, uint32_t& err) {
    ranges_subtract(t.marked, t.sacked, t.tmp, err);
    ranges_subtract(t.tmp, t.retx, t.lost, err);
}
__device__ void tally_tidy(const Tally& t, RVec& v) {   // cc:316-335
    if (v.n > 0 && t.last_ack >= v.r[0].a && t.last_ack < v.r[0].b - 1) {
        v.r[0].a = t.last_ack;
    } else if (v.n > 0 && t.last_ack >= v.r[0].b - 1) {
        uint32_t k = 0;
        for (uint32_t i = 0; i < v.n; i++) if (!(t.last_ack >= v.r[i].b)) v.r[k++] = v.r[i];
        v.n = k;
    }
}
__device__ uint32_t tally_update(Tally& t, uint32_t last_ack, bool is_dup, uint32_t& err) {   // cc:192-220
    uint32_t ret = 0;
    if (is_dup && (int64_t)last_ack == t.last_ack) {
        ++t.ndup;
    } else if ((int64_t)last_ack > t.last_ack) {
        t.last_ack = last_ack;
        t.ndup = 0;
        tally_tidy(t, t.marked);
        tally_tidy(t, t.sacked);
        tally_tidy(t, t.retx);
    }
    bool contains = false;
    for (uint32_t i = 0; i < t.retx.n; i++)
        if (t.last_ack >= t.retx.r[i].a && t.last_ack < t.retx.r[i].b) contains = true;
    if (t.ndup >= 3 && !contains) {
        ranges_insert(t.marked, t.last_ack, t.last_ack + 1, err);
        tally_compute_lost(t, err);
        if (t.lost.n > 0) ret |= PF_DATA_LOST;
    }
    return ret;
}
__device__ void tally_mark_sacked(Tally& t, const int32_t* s, uint32_t n, uint32_t& err) {   // cc:224-245
    int64_t first = -1;
    for (uint32_t i = 0; i < n; i++) {
        if (first == -1) first = s[i];
        if (i + 1 == n || s[i + 1] != s[i] + 1) { ranges_insert(t.sacked, first, (int64_t)s[i] + 1, err); first = -1; }
    }
}

// ------------------------------------------------------------ timers
__device__ void tcp_schedule_rto(L& c, DSock* k, uint64_t now, uint64_t delay) {   // tcp.c:925-946
    th_push(k->timers, now + delay, c.H->err);
    sched_task(c, delay, K_RTO, sidx(c, k));
}
__device__ void tcp_schedule_rto_if_needed(L& c, DSock* k, uint64_t now) {   // tcp.c:948-960
    if (k->timers.n && k->timers.a[0] <= k->desired) return;
    tcp_schedule_rto(c, k, now, k->desired - now);
}
__device__ void tcp_set_rto_timer(L& c, DSock* k, uint64_t now) {   // tcp.c:962-971
    k->desired = now + (uint64_t)k->rto * kMs;
    tcp_schedule_rto_if_needed(c, k, now);
}
__device__ void tcp_set_rto(DSock* k, int v) {   // tcp.c:982-989
    k->rto = v;
    if (k->rto > 120000) k->rto = 120000;
    if (k->rto < 200) k->rto = 200;
}

// ------------------------------------------------------------ Reno (tcp_cong_reno.c)
__device__ void reno_new_ack(DSock* k, uint32_t n) {
    if (k->reno_state == 0) {   // slow start (:65-89), into congestion avoidance with the leftover
        k->reno_ndup = 0;
        const uint32_t nc = k->cwnd + n;
        if (nc < k->reno_ssthresh) { k->cwnd = nc; return; }
        n = nc - k->reno_ssthresh;
        k->cwnd = k->reno_ssthresh;
        k->reno_nacked = 0;
        k->reno_state = 2;
    } else if (k->reno_state == 1) {   // fast recovery (:97-104)
        k->reno_ndup = 0;
        k->cwnd = k->reno_ssthresh;
        k->reno_nacked = 0;
        k->reno_state = 2;
    }
    k->reno_nacked += n;   // congestion avoidance (:108-118)
    while (k->reno_nacked >= k->cwnd) { k->reno_nacked -= k->cwnd; k->cwnd += 1; }
}
__device__ void reno_dup_ack(DSock* k) {
    if (k->reno_state == 1) { k->cwnd += 1; return; }
    k->reno_ndup++;
    if (k->reno_ndup == 3) { k->reno_ssthresh = (k->cwnd / 2) + 1; k->cwnd = k->reno_ssthresh + 3; k->reno_state = 1; }
}
__device__ void reno_timeout(DSock* k) {
    k->reno_ndup = 0;
    k->reno_ssthresh = (k->cwnd / 2) + 1;
    k->cwnd = 10;
    k->reno_state = 0;
}

// ------------------------------------------------------------ TCP
__device__ int32_t sock_new(L& c) {   // host_createDescriptor + tcp_new (tcp.c:2452-2512)
    DHost* H = c.H;
    int32_t j = 0;   // a released datagram socket's slot first (udp_release)
    while (j < H->nsock && SK(c, j)->used) j++;
    if (j == H->nsock) {
        if (H->nsock >= c.g->spk) { H->err |= SHD_TCP_ERR_SOCKETS; return -1; }
        H->nsock++;
    }
    DSock* k = SK(c, j);
    const int32_t si = sidx(c, k);
    memset(k, 0, offsetof(DSock, outctl));   // the scalars
    k->used = 1; k->host = c.h; k->proc = -1; k->parent = -1; k->partial = -1;
    k->in.head = k->in.n = 0; k->out.head = k->out.n = 0; k->outctl.head = k->outctl.n = 0;
    k->state = TS_CLOSED; k->state_last = 0; k->flags = 0; k->error = 0;
    return si;
}
__device__ void sock_init_tcp(DSock* k, uint32_t recv_buf, uint32_t send_buf, uint32_t iw) {
    k->in_size = recv_buf; k->out_size = send_buf;
    k->r_winupd = 0; k->r_last_ts = 0; k->r_last_seq = 0; k->r_start = 1; k->r_next = 1; k->r_end = 1;
    k->r_window = iw; k->r_last_window = iw; k->r_last_ack = 1;
    k->s_unacked = 1; k->s_next = 1; k->s_end = 1; k->s_last_ack = 1; k->s_window = iw; k->s_last_window = iw;
    k->s_highest = 0; k->s_packets_sent = 0; k->s_quick_acks = 0; k->s_delack_counter = 0; k->s_delack_sched = 0;
    k->nsack = 0; k->nrtx = 0; k->rh = 0; k->rtx_len = 0; k->timers.n = 0; k->desired = 0; k->backoff = 0;
    k->tally.last_ack = -1; k->tally.ndup = 0;
    k->tally.marked.n = k->tally.sacked.n = k->tally.retx.n = k->tally.lost.n = k->tally.tmp.n = 0;
    k->at_did_init = 0; k->at_bytes = 0; k->at_last_adjust = 0; k->at_space = 0;
    k->cwnd = 1; k->reno_state = 0; k->reno_ndup = 0; k->reno_nacked = 0; k->reno_ssthresh = 0x7fffffffu;
    k->srtt = 0; k->rttvar = 0; k->retx_count = 0; k->info_rtt = 0;
    k->throttled.n = 0; k->throttled_len = 0; k->unordered.n = 0; k->unordered_len = 0;
    k->partial = -1; k->partial_off = 0;
    k->server = 0; k->nkids = 0; k->npending = 0; k->last_peer_ip = 0; k->last_ip = 0; k->last_peer_port = 0;
    k->child = 0; k->parent = -1; k->child_state = 0;
    tcp_set_rto(k, 1000);
}
__device__ uint32_t tcp_get_ip(const L& c, const DSock* k) {   // tcp.c:335-353
    if (k->server) return k->bound ? k->bound_ip : k->last_ip;
    if (k->child) { const DSock* pa = &c.g->sock[k->parent]; return pa->bound ? pa->bound_ip : pa->last_ip; }
    return k->bound_ip;
}
__device__ uint32_t tcp_get_peer_ip(const DSock* k) {
    uint32_t ip = k->peer_ip;
    if (k->server && ip == 0) ip = k->last_peer_ip;
    return ip;
}
__device__ uint32_t src_ip_for(const L& c, const DSock* k, uint32_t dst) {
    uint32_t ip = tcp_get_ip(c, k);
    if (ip == 0) ip = (dst == 0x7f000001u) ? 0x7f000001u : c.g->ip_all[c.gh];
    return ip;
}
__device__ void tcp_update_rcv_window(DSock* k) { k->r_window = (uint32_t)(in_space(k) / kMSS); }   // tcp.c:762-782
__device__ void tcp_update_snd_window(DSock* k) {   // tcp.c:784-789
    const int lw = (int)k->r_last_window;
    k->s_window = (uint32_t)((int)k->cwnd < lw ? (int)k->cwnd : lw);
}
__device__ void tcp_set_state(L& c, DSock* k, int st);
__device__ void tcp_tune_initial_buffers(L& c, DSock* k) {   // tcp.c:441-533
    k->at_did_init = 1;
    const uint32_t dip = tcp_get_peer_ip(k);
    const uint32_t sip = src_ip_for(c, k, dip);
    if (sip == dip) { set_in_size(k, 6291456); set_out_size(k, 4194304); k->info_rtt = 0xffffffffu; return; }
    const int32_t a = host_of_ip(c, sip), b = host_of_ip(c, dip);
    double l1, l2, r;
    path(c, a, b, l1, r);   // _tcp_calculateRTT (tcp.c:363-405)
    path(c, b, a, l2, r);
    const uint32_t rtt = (uint32_t)ceil(l1) + (uint32_t)ceil(l2);
    const uint32_t au = (uint32_t)c.g->bwu_all[a], ad = (uint32_t)c.g->bwd_all[a];
    const uint32_t bu = (uint32_t)c.g->bwu_all[b], bd = (uint32_t)c.g->bwd_all[b];
    const uint32_t sbw = au < bd ? au : bd;
    const uint32_t rbw = ad < bu ? ad : bu;
    // float arithmetic as the reference writes it (tcp.c:504, 514)
    uint64_t sendbuf = (uint64_t)(((float)(rtt * sbw) * 1024.0f * 1.25f) / 1000.0f);
    uint64_t recvbuf = (uint64_t)(((float)(rtt * rbw) * 1024.0f * 1.25f) / 1000.0f);
    sendbuf = sendbuf < 16384 ? 16384 : sendbuf > 4194304 ? 4194304 : sendbuf;
    recvbuf = recvbuf < 87380 ? 87380 : recvbuf > 6291456 ? 6291456 : recvbuf;
    set_in_size(k, recvbuf);
    set_out_size(k, sendbuf);
}
__device__ uint64_t rtt_mem(const L& c, const DSock* k, bool rmem) {   // tcp.c:407-427
    const DHost* H = &c.g->host[k->host];
    const uint64_t refill = rmem ? H->rx_refill : H->tx_refill;
    const uint64_t kib = (uint64_t)(uint32_t)((refill * 1000u) / 1024u);
    const double rtt_s = ((double)k->srtt) / ((double)1000);
    return (uint64_t)((double)(kib * 1024) * rtt_s);
}
__device__ __forceinline__ uint64_t clamp_u(uint64_t v, uint64_t lo, uint64_t hi) { return v < lo ? lo : v > hi ? hi : v; }
__device__ void tcp_autotune_rcv(L& c, DSock* k, uint32_t copied) {   // tcp.c:535-564
    k->at_bytes += copied;
    uint64_t space = 2 * k->at_bytes;
    if (k->at_space > space) space = k->at_space;
    const uint64_t cur = in_size(k);
    if (space > cur) {
        k->at_space = space;
        const uint64_t mx = clamp_u(rtt_mem(c, k, true), 6291456, 62914560);
        const uint64_t nsz = space < mx ? space : mx;
        if (nsz > cur) set_in_size(k, nsz);
    }
    if (k->at_last_adjust == 0) {
        k->at_last_adjust = c.now;
    } else if (k->srtt > 0) {
        if (c.now - k->at_last_adjust > (uint64_t)k->srtt * kMs) { k->at_last_adjust = c.now; k->at_bytes = 0; }
    }
}
__device__ void tcp_autotune_snd(L& c, DSock* k) {   // tcp.c:566-591
    const uint64_t mx = clamp_u(rtt_mem(c, k, false), 4194304, 41943040);
    uint64_t nsz = (uint64_t)2404 * 2 * (uint64_t)k->cwnd;
    if (nsz > mx) nsz = mx;
    if (nsz > out_size(k)) set_out_size(k, nsz);
}
__device__ void tcp_buffer_out(L& c, DSock* k, int32_t pi) {   // tcp.c:729-745
    DPkt* p = PK(c, pi);
    if (p->inq & Q_THROTTLED) return;   // already queued (priority_queue_push's lookup)
    if (!kh_push_new(k->throttled, pi, p->seq, c.H->err)) return;
    p->inq |= Q_THROTTLED;
    pkt_ref(c, pi);
    k->throttled_len += PK(c, pi)->len;
    if (space_out(k) == 0) sock_status(c, k, DS_WRITABLE, false);
    pkt_status(c, pi, S_SND_TCP_ENQUEUE_THROTTLED);
}
__device__ void tcp_buffer_in(L& c, DSock* k, int32_t pi) {   // tcp.c:747-760
    DPkt* p = PK(c, pi);
    if (p->inq & Q_UNORDERED) return;
    if (!kh_push_new(k->unordered, pi, p->seq, c.H->err)) return;
    p->inq |= Q_UNORDERED;
    pkt_ref(c, pi);
    k->unordered_len += PK(c, pi)->len;
    pkt_status(c, pi, S_RCV_TCP_ENQUEUE_UNORDERED);
}
__device__ int32_t tcp_create_packet(L& c, DSock* k, uint32_t flags, uint32_t len) {   // tcp.c:791-835
    const uint32_t dip = tcp_get_peer_ip(k);
    const uint16_t sport = k->child ? c.g->sock[k->parent].bound_port : k->bound_port;
    const uint16_t dport = k->server ? k->last_peer_port : k->peer_port;
    const uint32_t sip = src_ip_for(c, k, dip);
    tcp_update_rcv_window(k);
    const bool fin_not_ack = (flags & F_FIN) && !(flags & F_ACK);
    const uint32_t seq = (len > 0 || fin_not_ack) ? k->s_next : 0;
    const int32_t pi = pkt_new(c, len);
    if (pi < 0) return -1;
    DPkt* p = PK(c, pi);
    p->flags = flags; p->sip = sip; p->sport = sport; p->dip = dip; p->dport = dport; p->seq = seq;
    pkt_status(c, pi, S_SND_CREATED);
    if (seq > 0) k->s_next++;
    return pi;
}
__device__ void tcp_retransmit_packet(L& c, DSock* k, uint32_t seq) {   // tcp.c:1027-1065
    const int at = rtx_find(c, k, seq);
    if (at < 0) return;
    const int32_t pi = rtx_at(k, (uint32_t)at);
    rtx_remove_at(k, (uint32_t)at);
    k->rtx_len -= PK(c, pi)->len;
    pkt_status(c, pi, S_SND_TCP_DEQUEUE_RETRANSMIT);
    if (space_out(k) > 0) sock_status(c, k, DS_WRITABLE, true);
    tcp_set_rto_timer(c, k, c.now);
    tcp_buffer_out(c, k, pi);
    pkt_status(c, pi, S_SND_TCP_RETRANSMITTED);
    k->retx_count++;
    pkt_unref(c, pi);
}
// tcp_networkInterfaceIsAboutToSendPacket (tcp.c:1090-1119)
__device__ void tcp_about_to_send(L& c, DSock* k, int32_t pi) {
    DPkt* p = PK(c, pi);
    if (k->nsack > 0) {
        if (k->nsack > kPktSack) c.H->err |= SHD_TCP_ERR_SACK;
        p->flags |= F_SACK;
        p->nsack = k->nsack < kPktSack ? k->nsack : kPktSack;
        int32_t* sk = PSK(c, pi);
        for (uint32_t i = 0; i < p->nsack; i++) sk[i] = k->sacks[i];
    }
    p->ack = k->r_next;
    p->win = k->r_window;
    p->tsval = c.now;
    p->tsecho = k->r_last_ts;
    k->s_last_ack = k->r_next;
    k->s_last_window = k->r_window;
    if (p->flags & F_ACK) k->s_delack_counter = 0;
    if (p->seq > 0 || (p->flags & F_SYN)) {
        tcp_add_retransmit(c, k, pi);
        if (!k->desired) tcp_set_rto_timer(c, k, c.now);
    }
}
// _tcp_flush (tcp.c:1121-1278).  The FIN it may send flushes again; that
// inner flush reaches its own FIN step in FINWAIT1 / LASTACK, where
// _tcp_sendShutdownFin sends nothing, so the inner pass only clears the flag.
// Outer and inner flush are separate instantiations: the call graph has no
// cycle, so the compiler sizes every lane's stack exactly (no dynamic stack).
template <bool kOuter> __device__ void tcp_flush_body(L& c, DSock* k);
__device__ void tcp_send_shutdown_fin(L& c, DSock* k, bool from_flush) {   // tcp.c:1067-1088
    bool send = false;
    if (k->state == TS_ESTABLISHED || k->state == TS_SYNRECEIVED) { tcp_set_state(c, k, TS_FINWAIT1); send = true; }
    else if (k->state == TS_CLOSEWAIT) { tcp_set_state(c, k, TS_LASTACK); send = true; }
    if (send) {
        const int32_t fin = tcp_create_packet(c, k, F_FIN, 0);
        if (fin < 0) return;
        tcp_buffer_out(c, k, fin);
        tcp_flush_body<false>(c, k);
        pkt_unref(c, fin);
    }
}
template <bool kOuter> __device__ void tcp_flush_body(L& c, DSock* k) {
    tcp_update_rcv_window(k);
    tcp_update_snd_window(k);
    const uint32_t nl = k->tally.lost.n;
    if (nl > 0) {
        Rng64 lr[kRanges];
        for (uint32_t i = 0; i < nl; i++) lr[i] = k->tally.lost.r[i];
        for (uint32_t i = 0; i < nl; i++) {
            for (uint32_t j = (uint32_t)lr[i].a; j < (uint32_t)lr[i].b; ++j) tcp_retransmit_packet(c, k, j);
            ranges_insert(k->tally.retx, lr[i].a, lr[i].b, c.H->err);   // mark_retransmitted (cc:257-263)
            tally_compute_lost(k->tally, c.H->err);
        }
    }
    while (k->throttled.n) {
        const int32_t pi = kh_top(k->throttled);
        DPkt* p = PK(c, pi);
        const uint32_t len = p->len;
        if (len > 0) {
            const bool in_window = p->seq < (uint32_t)(k->s_unacked + k->s_window);
            const bool in_buffer = len <= out_space(k);
            if (!in_buffer || !in_window) break;
        }
        kh_pop(k->throttled);
        p->inq &= ~Q_THROTTLED;
        k->throttled_len -= len;
        sock_add_output(c, k, pi);
        k->s_packets_sent++;
        if (p->seq > k->s_highest) k->s_highest = p->seq;
    }
    while (k->unordered.n) {
        const int32_t pi = kh_top(k->unordered);
        DPkt* p = PK(c, pi);
        if (p->seq == k->r_next && sock_add_input(c, k, pi)) {
            k->r_last_seq = p->seq;
            kh_pop(k->unordered);
            p->inq &= ~Q_UNORDERED;
            const uint32_t len = p->len;
            pkt_unref(c, pi);
            k->unordered_len -= len;
            k->r_next++;
            continue;
        }
        break;
    }
    if ((k->flags & TF_SHOULD_SEND_WR_FIN) && tcp_out_len(k) == 0) {
        if (kOuter) tcp_send_shutdown_fin(c, k, true);
        k->flags &= ~TF_SHOULD_SEND_WR_FIN;
    }
    if ((k->flags & TF_LOCAL_CLOSED_WR) || (k->error & TE_CONNECTION_RESET)) k->error |= TE_SEND_EOF;
    if ((k->flags & TF_LOCAL_CLOSED_RD) || (k->flags & TF_REMOTE_CLOSED) || (k->error & TE_CONNECTION_RESET)) {
        if (k->r_next >= k->r_end && !(k->flags & TF_EOF_RD_SIGNALED)) {
            k->error |= TE_RECEIVE_EOF;
            sock_status(c, k, DS_READABLE, true);
        }
    }
    if ((k->error & TE_CONNECTION_RESET) && (k->flags & TF_RESET_SIGNALED)) sock_status(c, k, DS_WRITABLE, false);
    else if ((k->error & TE_SEND_EOF) && (k->flags & TF_EOF_WR_SIGNALED)) sock_status(c, k, DS_WRITABLE, false);
    else if (space_out(k) <= 0) sock_status(c, k, DS_WRITABLE, false);
    else sock_status(c, k, DS_WRITABLE, true);
}
__device__ __forceinline__ void tcp_flush(L& c, DSock* k) { tcp_flush_body<true>(c, k); }
__device__ void tcp_send_control(L& c, DSock* k, uint32_t flags) {   // tcp.c:837-852
    const int32_t ci = tcp_create_packet(c, k, flags, 0);
    if (ci < 0) return;
    PK(c, ci)->prio = 0.0;
    tcp_buffer_out(c, k, ci);
    tcp_flush(c, k);
    pkt_unref(c, ci);
}
__device__ void tcp_set_state(L& c, DSock* k, int st) {   // tcp.c:607-693
    k->state_last = k->state;
    k->state = st;
    if (st == TS_LISTEN) {
        sock_status(c, k, DS_ACTIVE, true);
    } else if (st == TS_ESTABLISHED) {
        k->flags |= TF_WAS_ESTABLISHED;
        sock_status(c, k, DS_ACTIVE | DS_WRITABLE, true);
    } else if (st == TS_CLOSED) {
        tcp_clear_retransmit(c, k, 0xffffffffu);
        sock_status(c, k, DS_ACTIVE, false);
        if (!k->server || k->nkids == 0) {
            if (k->child && k->parent >= 0) {
                DSock* pa = &c.g->sock[k->parent];
                for (uint32_t i = 0; i < pa->nkids; i++)
                    if (pa->kids[i] == sidx(c, k)) { pa->kids[i] = pa->kids[--pa->nkids]; break; }
                if (pa->state == TS_CLOSED && pa->nkids == 0) { pa->assoc = 0; pa->assoc_general = 0; }
            }
            k->assoc = 0;   // host_closeDescriptor: _host_disassociateInterface
            k->assoc_general = 0;
        }
    } else if (st == TS_TIMEWAIT) {
        const uint64_t delay = (k->child && k->parent >= 0) ? kSec : 60 * kSec;   // CONFIG_TCPCLOSETIMER_DELAY
        sched_task(c, delay, K_CLOSE, sidx(c, k));
    }
}
__device__ void tcp_update_rtt(L& c, DSock* k, uint64_t ts) {   // tcp.c:991-1025
    int rtt = (int)((c.now - ts) / kMs);
    if (rtt <= 0) rtt = 1;
    if (!k->srtt) {
        k->srtt = rtt;
        k->rttvar = rtt / 2;
        if (!k->at_did_init) tcp_tune_initial_buffers(c, k);
    } else {
        k->rttvar = (3 * k->rttvar / 4) + (abs(k->srtt - rtt) / 4);
        k->srtt = (7 * k->srtt / 8) + (rtt / 8);
    }
    tcp_set_rto(k, k->srtt + 4 * k->rttvar);
}
__device__ uint32_t tcp_data_processing(L& c, DSock* k, int32_t pi) {   // tcp.c:1597-1660
    DPkt* p = PK(c, pi);
    uint32_t fl = 0;
    if (p->seq >= k->r_next + k->r_window) {
        fl |= PF_PROCESSED;
        pkt_status(c, pi, S_RCV_SOCKET_DROPPED);
    } else if (p->seq >= k->r_next) {
        fl |= PF_PROCESSED;
        const bool is_next = p->seq == k->r_next;
        const bool fits = p->len <= space_in(k);
        if (!is_next && fits) {
            if (k->nsack >= kSacks) c.H->err |= SHD_TCP_ERR_SACK;
            else k->sacks[k->nsack++] = (int32_t)p->seq;
        } else if (k->nsack > 0) {
            uint32_t it = 0;
            if (k->sacks[0] <= (int32_t)p->seq + 1) {
                uint32_t nx = 1;
                while (nx < k->nsack) {
                    const int32_t cur = k->sacks[it], nxt = k->sacks[nx];
                    if (cur + 1 < nxt && cur > (int32_t)p->seq) break;
                    it = nx;
                    nx = it + 1;
                }
                const int32_t cut = k->sacks[it];   // _tcp_removeSacks (tcp.c:1579-1595)
                uint32_t w = 0;
                for (uint32_t i = 0; i < k->nsack; i++) if (k->sacks[i] > cut) k->sacks[w++] = k->sacks[i];
                k->nsack = w;
            }
        }
        const bool waiting_read = (k->status & DS_READABLE) != 0;
        if ((is_next && !waiting_read) || fits) {
            tcp_buffer_in(c, k, pi);
            fl |= PF_DATA_RECEIVED;
        } else {
            pkt_status(c, pi, S_RCV_SOCKET_DROPPED);
        }
    }
    return fl;
}
__device__ uint32_t tcp_ack_processing(L& c, DSock* k, int32_t pi) {   // tcp.c:1662-1750
    DPkt* p = PK(c, pi);
    uint32_t fl = PF_PROCESSED;
    const uint32_t prev_win = k->r_last_window;
    const bool valid_ack = p->ack > k->s_unacked && p->ack <= k->s_next;
    const bool valid_win = (p->ack == k->r_last_ack && p->win > prev_win) || (p->ack > k->r_last_ack && p->win != prev_win);
    if (p->win != prev_win) fl |= PF_RWND_UPDATED;
    const bool is_dup = (p->flags & F_DUPACK) != 0;
    fl |= tally_update(k->tally, p->ack, is_dup, c.H->err);
    if (is_dup) reno_dup_ack(k);
    int n_acked = 0;
    if (valid_ack) {
        tcp_clear_retransmit_range(c, k, k->r_last_ack, p->ack);
        k->r_last_ack = p->ack;
        n_acked = (int)(p->ack - k->s_unacked);
        k->s_unacked = p->ack;
        if (n_acked > 0) {
            fl |= PF_DATA_ACKED;
            reno_new_ack(k, (uint32_t)n_acked);
            tcp_autotune_snd(c, k);
        }
        if (k->backoff > 2) { k->srtt = 0; k->rttvar = 0; tcp_set_rto(k, 1000); }
        k->backoff = 0;
    }
    if (valid_win) k->r_last_window = p->win;
    if (k->rtx_len == 0) k->desired = 0;
    else if (n_acked > 0) tcp_set_rto_timer(c, k, c.now);
    return fl;
}
__device__ void tcp_process(L& c, DSock* k, int32_t pi) {   // tcp.c:1777-2099
    DPkt* p = PK(c, pi);
    if (k->server) {   // _tcp_getSourceTCP: a child keyed by the peer's ip:port
        for (uint32_t i = 0; i < k->nkids; i++) {
            DSock* ch = &c.g->sock[k->kids[i]];
            if (ch->peer_ip == p->sip && ch->peer_port == p->sport) { k = ch; break; }
        }
    }
    if (p->flags & F_RST) {
        if (k->state != TS_LISTEN && !(k->error & TE_CONNECTION_RESET)) {   // TCPS_LISTEN is a bit there, a state here
            k->error |= TE_CONNECTION_RESET;
            k->flags |= TF_REMOTE_CLOSED;
            tcp_set_state(c, k, TS_TIMEWAIT);
            k->r_end = k->r_next;
        }
        return;
    }
    if (k->server) { k->last_peer_ip = p->sip; k->last_peer_port = p->sport; k->last_ip = p->dip; }
    uint32_t fl = 0, resp = 0;
    switch (k->state) {
    case TS_LISTEN:
        if (p->flags & F_SYN) {
            fl |= PF_PROCESSED;
            const int32_t ci = sock_new(c);   // a multiplexed child (tcp.c:1824-1853)
            if (ci < 0) return;
            DSock* ch = &c.g->sock[ci];
            sock_init_tcp(ch, c.g->recv_buf, c.g->send_buf, c.g->tcp_window);
            ch->child = 1;
            ch->parent = sidx(c, k);
            ch->child_state = 1;
            ch->peer_ip = p->sip; ch->peer_port = p->sport;
            ch->bound = 1; ch->bound_ip = k->bound_ip; ch->bound_port = k->bound_port;
            if (k->nkids >= kKids) { c.H->err |= SHD_TCP_ERR_SOCKETS; return; }
            k->kids[k->nkids++] = ci;
            ch->r_start = p->seq;
            ch->r_next = ch->r_start + 1;
            tcp_set_state(c, ch, TS_SYNRECEIVED);
            k = ch;
            resp = F_SYN | F_ACK;
        }
        break;
    case TS_SYNSENT:
        if ((p->flags & F_SYN) && (p->flags & F_ACK)) {
            fl |= PF_PROCESSED;
            k->r_start = p->seq;
            k->r_next = k->r_start + 1;
            resp |= F_ACK;
            tcp_set_state(c, k, TS_ESTABLISHED);
            tcp_clear_retransmit(c, k, 1);
        } else if (p->flags & F_SYN) {
            fl |= PF_PROCESSED;
            k->r_start = p->seq;
            k->r_next = k->r_start + 1;
            resp |= F_ACK;
            tcp_set_state(c, k, TS_SYNRECEIVED);
        }
        break;
    case TS_SYNRECEIVED:
        if (p->flags & F_ACK) {
            fl |= PF_PROCESSED;
            tcp_set_state(c, k, TS_ESTABLISHED);
            tcp_clear_retransmit(c, k, 1);
            if (k->child) {
                k->child_state = 2;
                DSock* pa = &c.g->sock[k->parent];
                if (pa->npending >= kKids) { c.H->err |= SHD_TCP_ERR_SOCKETS; return; }
                pa->pending[pa->npending++] = sidx(c, k);
                sock_status(c, pa, DS_READABLE, true);
            }
        }
        break;
    case TS_ESTABLISHED:
        if (p->flags & F_FIN) {
            fl |= PF_PROCESSED;
            k->flags |= TF_REMOTE_CLOSED;
            resp |= F_FIN | F_ACK;
            tcp_set_state(c, k, TS_CLOSEWAIT);
            k->r_end = p->seq;
        }
        break;
    case TS_FINWAIT1:
        if ((p->flags & F_FIN) && (p->flags & F_ACK)) {
            fl |= PF_PROCESSED;
            tcp_set_state(c, k, TS_FINWAIT2);
        } else if (p->flags & F_FIN) {
            fl |= PF_PROCESSED;
            resp |= F_FIN | F_ACK;
            k->flags |= TF_REMOTE_CLOSED;
            tcp_set_state(c, k, TS_CLOSING);
            k->r_end = p->seq;
        }
        break;
    case TS_FINWAIT2:
        if (p->flags & F_FIN) {
            fl |= PF_PROCESSED;
            resp |= F_FIN | F_ACK;
            k->flags |= TF_REMOTE_CLOSED;
            tcp_set_state(c, k, TS_TIMEWAIT);
            k->r_end = p->seq;
        }
        break;
    case TS_CLOSING:
        if ((p->flags & F_FIN) && (p->flags & F_ACK)) { fl |= PF_PROCESSED; tcp_set_state(c, k, TS_TIMEWAIT); }
        break;
    case TS_TIMEWAIT:
    case TS_CLOSEWAIT:
        break;
    case TS_LASTACK:
        if ((p->flags & F_FIN) && (p->flags & F_ACK)) { fl |= PF_PROCESSED; tcp_set_state(c, k, TS_CLOSED); return; }
        break;
    default:
        pkt_status(c, pi, S_RCV_SOCKET_DROPPED);
        return;
    }
    if (k->state == TS_LISTEN) {
        if (!(fl & PF_PROCESSED)) pkt_status(c, pi, S_RCV_SOCKET_DROPPED);
        return;
    }
    if (p->len > 0 && !(k->error & TE_RECEIVE_EOF)) fl |= tcp_data_processing(c, k, pi);
    if (p->flags & F_ACK) fl |= tcp_ack_processing(c, k, pi);
    if (!(fl & PF_PROCESSED)) { pkt_status(c, pi, S_RCV_SOCKET_DROPPED); return; }
    if (p->nsack) tally_mark_sacked(k->tally, PSK(c, pi), p->nsack, c.H->err);
    k->r_last_ts = p->tsval;
    if (p->tsecho && k->backoff == 0) tcp_update_rtt(c, k, p->tsecho);
    if (p->seq > k->r_next && p->seq < k->r_next + k->r_window) resp |= (F_ACK | F_DUPACK);
    else if (fl & PF_DATA_RECEIVED) resp |= F_ACK;
    if (resp != 0 && (!(k->error & TE_RECEIVE_EOF) || (resp & F_FIN))) {
        if (resp != F_ACK) {
            tcp_send_control(c, k, resp);
        } else {
            if (!k->s_delack_sched) {   // a delayed ACK task (tcp.c:2066-2089)
                uint64_t delay;
                if (k->s_quick_acks < 1000) { delay = kMs; k->s_quick_acks++; } else delay = 5 * kMs;
                sched_task(c, delay, K_DELACK, sidx(c, k));
                k->s_delack_sched = 1;
            }
            k->s_delack_counter++;
        }
    }
    tcp_flush(c, k);
    k->r_last_ts = 0;
}

// ------------------------------------------------------------ the interface (network_interface.c)
__device__ void refill_if_needed(L& c) {   // :130-161, started at t = 0
    DHost* H = c.H;
    if (((H->tx_rem < H->tx_cap) || (H->rx_rem < H->rx_cap)) && !H->refill_pending) {
        sched_task(c, kMs - (c.now % kMs), K_REFILL, -1);
        H->refill_pending = 1;
    }
}
__device__ __forceinline__ void consume(uint64_t& rem, uint64_t n) { rem = (n >= rem) ? 0 : rem - n; }
// the association keys are (protocol, port, peer); general: peer 0:0
__device__ DSock* lookup_socket(L& c, int32_t udp, uint16_t port, uint32_t peer_ip, uint16_t peer_port) {   // :385-403
    for (int32_t j = 0; j < c.H->nsock; j++) {
        DSock* k = SK(c, j);
        if (k->assoc && k->assoc_general && k->udp == udp && k->bound_port == port) return k;
    }
    for (int32_t j = 0; j < c.H->nsock; j++) {
        DSock* k = SK(c, j);
        if (k->assoc && !k->assoc_general && k->udp == udp && k->bound_port == port && k->peer_ip == peer_ip &&
            k->peer_port == peer_port)
            return k;
    }
    return nullptr;
}
// CoDel (router_queue_codel.c:148-267)
constexpr uint64_t kCodelTarget = 10 * kMs, kCodelInterval = 100 * kMs;
__device__ bool cq_helper(L& c, bool& ok, CqEnt& out) {
    DHost* H = c.H;
    ok = false;
    if (H->cq_n == 0) { H->cq_iexp = 0; return false; }
    out = c.g->cq[(size_t)c.h * kCq + H->cq_head];
    H->cq_head = (H->cq_head + 1) % kCq;
    H->cq_n--;
    H->cq_total -= out.len;
    const uint64_t sojourn = c.now - out.ts;
    if (sojourn < kCodelTarget || H->cq_total < kMTU) {
        H->cq_iexp = 0;
    } else {
        if (H->cq_iexp == 0) H->cq_iexp = c.now + kCodelInterval;
        else if (c.now >= H->cq_iexp) ok = true;
    }
    return true;
}
__device__ uint64_t cq_law(uint32_t count, uint64_t ts) {
    return (uint64_t)round(((double)(ts + kCodelInterval)) / sqrt((double)count));
}
__device__ void cq_drop(L& c, const CqEnt& e) {
    pkt_status(c, e.pkt, S_ROUTER_DROPPED);
    pkt_unref(c, e.pkt);
}
__device__ bool cq_dequeue(L& c, CqEnt& out) {
    DHost* H = c.H;
    bool ok = false;
    CqEnt e;
    bool have = cq_helper(c, ok, e);
    if (!have) { H->cq_mode = 0; return false; }
    if (H->cq_mode) {
        if (!ok) H->cq_mode = 0;
        while (c.now >= H->cq_next_drop && H->cq_mode) {
            cq_drop(c, e);
            H->cq_dc++;
            have = cq_helper(c, ok, e);
            if (ok) H->cq_next_drop = cq_law(H->cq_dc, H->cq_next_drop);
            else H->cq_mode = 0;
        }
    } else if (ok) {
        cq_drop(c, e);
        have = cq_helper(c, ok, e);
        H->cq_mode = 1;
        const uint32_t delta = H->cq_dc - H->cq_dc_last;
        H->cq_dc = 1;
        const bool recent = c.now < H->cq_next_drop + 16 * kCodelInterval;
        if (recent && delta > 1) H->cq_dc = delta;
        H->cq_next_drop = cq_law(H->cq_dc, c.now);
        H->cq_dc_last = H->cq_dc;
    }
    if (!have) return false;
    out = e;
    return true;
}
// tracker_addInputBytes / tracker_addOutputBytes (tracker.c:216-276), the
// node counters only (LOG_INFO_FLAGS_NODE); dir 0 in, 1 out
__device__ void tracker_add(L& c, int32_t pi, int dir) {
    if (!c.g->node) return;
    const DPkt* p = PK(c, pi);
    uint64_t* t = c.H->trk + kTrk * dir;
    const uint64_t hdr = hdr_of(p), pay = p->len;
    const bool rx = (p->xflags & kXRetx) != 0;
    if (pay > 0) {
        if (rx) { t[7]++; t[8] += hdr; t[9] += pay; }
        else { t[4]++; t[5] += hdr; t[6] += pay; }
    } else {
        if (rx) { t[2]++; t[3] += hdr; }
        else { t[0]++; t[1] += hdr; }
    }
}
__device__ void if_receive_packet(L& c, int32_t pi) {   // _networkinterface_receivePacket (:375-419)
    const DPkt* p = PK(c, pi);
    pkt_status(c, pi, S_RCV_INTERFACE_RECEIVED);
    DSock* k = lookup_socket(c, (p->xflags & kXUdp) ? 1 : 0, p->dport, p->sip, p->sport);
    if (k) {
        pkt_status(c, pi, S_RCV_SOCKET_PROCESSED);   // socket_pushInPacket
        if (k->udp) {   // udp_processPacket (udp.c:52-61)
            if (p->len > 0 && !sock_add_input(c, k, pi)) pkt_status(c, pi, S_RCV_SOCKET_DROPPED);
        } else {
            tcp_process(c, k, pi);
        }
    } else {
        pkt_status(c, pi, S_RCV_INTERFACE_DROPPED);
    }
    tracker_add(c, pi, 0);   // :415
}
__device__ void if_receive_packets(L& c) {   // :421-455
    DHost* H = c.H;
    while (H->rx_rem >= kMTU) {
        CqEnt e;
        if (!cq_dequeue(c, e)) break;
        pkt_status(c, e.pkt, S_ROUTER_DEQUEUED);
        const uint64_t len = (uint64_t)PK(c, e.pkt)->len + hdr_of(PK(c, e.pkt));
        if_receive_packet(c, e.pkt);
        pkt_unref(c, e.pkt);
        consume(H->rx_rem, len);
        refill_if_needed(c);
    }
}
// a delivery for another engine's host: its record (and SACK list) into that
// engine's segment of the round's exchange (shd_tcp_run_group), taken by the
// receiver before the next round (k_tcp_xingest)
__device__ void xsend_mail(L& c, int32_t pi, int32_t d, uint64_t t, uint64_t seq) {
    const Glob& g = *c.g;
    const DPkt* p = PK(c, pi);
    int32_t r = 0;   // the engine of host d: the contiguous split of shd_tcp_run_group
    while (r + 1 < g.world && (int64_t)d >= ((int64_t)(r + 1) * g.H) / g.world) r++;
    char* seg = g.xsend + (size_t)r * g.xseg;
    XSegHead* hd = (XSegHead*)seg;
    uint32_t off = 0;
    if (p->nsack) {   // the SACK list's space first: a claimed mail slot is always written whole
        off = atomicAdd(&hd->nsack, p->nsack);
        if (off + p->nsack > g.xsack_cap) { c.H->err |= SHD_TCP_ERR_MAILBOX; return; }
        int32_t* dst = (int32_t*)(seg + sizeof(XSegHead) + (size_t)g.xcap * sizeof(Mail)) + off;
        const int32_t* sk = PSK(c, pi);
        for (uint32_t i = 0; i < p->nsack; i++) dst[i] = sk[i];
    }
    const uint32_t k = atomicAdd(&hd->n, 1u);
    if (k >= g.xcap) { c.H->err |= SHD_TCP_ERR_MAILBOX; return; }
    Mail* m = (Mail*)(seg + sizeof(XSegHead)) + k;
    m->dst = (uint32_t)d; m->src = (uint32_t)c.gh; m->time = t; m->seq = seq;
    m->sack_off = off;
    pkt_copy_rec(&m->pkt, p, g.trace);
    m->pkt.refs = 1;
    m->pkt.inq = 0;
}
// a server's listening port, for its clients (DProc::peer) on any engine
__device__ void publish_port(L& c, int32_t proc, uint16_t port) {
    c.g->proc_port[proc] = port;
    if (c.g->world > 1) {
        const uint32_t k = atomicAdd(c.g->nport_new, 1u);
        if (k >= c.g->pcap) { c.H->err |= SHD_TCP_ERR_INTERNAL; return; }
        c.g->port_new[k] = ((uint64_t)(uint32_t)proc << 32) | port;
    }
}
__device__ void worker_send_packet(L& c, int32_t pi, DSock* ks) {   // worker.c:260-321
    DPkt* p = PK(c, pi);
    int32_t d;
    double lat, rel;
    if (ks->pc_ip != 0 && ks->pc_ip == p->dip) {   // the sending socket's path: no dependent loads
        d = ks->pc_host;
        if (c.g->pcm) c.kq++;   // the pair's value is stored: a repeat query changes nothing
        else touch_log(c, ks->pc_va, ks->pc_vb);
        lat = ks->pc_lat; rel = ks->pc_rel;
    } else {
        d = host_of_ip(c, p->dip);
        path(c, c.gh, d, lat, rel);
        if (d >= 0 && lat >= 0.0 && !c.H->err) {
            ks->pc_ip = p->dip; ks->pc_host = d; ks->pc_va = c.g->hv[c.gh]; ks->pc_vb = c.g->hv[d];
            ks->pc_lat = lat; ks->pc_rel = rel;
        }
    }
    const double chance = next_double(&c.H->rng);
    if (chance <= rel || p->len == 0) {
        const uint64_t t = c.now + (uint64_t)ceil(lat * (double)kMs);
        pkt_status(c, pi, S_INET_SENT);
        const uint64_t seq = c.H->ev_seq++;   // event_new_ (the delivery's ID)
        if (t >= c.g->end_time) return;
        if (d == c.gh) { c.H->err |= SHD_TCP_ERR_INTERNAL; return; }
        if (t < c.mail_min) c.mail_min = t;   // folded into next_time[h] at the round's end
        const int32_t dl = d - c.g->h0;
        if (dl < 0 || dl >= c.g->nloc) {   // another engine's host: its segment of the round's exchange
            xsend_mail(c, pi, d, t, seq);
            return;
        }
        const uint32_t part = (uint32_t)c.h % kMailSub, per = c.g->mail_part;
        const uint32_t kk = atomicAdd(c.g->n_out + part, 1u);
        uint32_t slot = part * per + kk;
        if (kk >= per) {   // the part is full: the shared overflow range
            const uint32_t ko = atomicAdd(c.g->n_out + kMailSub, 1u);
            if (ko >= c.g->mail_cap - per * kMailSub) { c.H->err |= SHD_TCP_ERR_MAILBOX; return; }
            slot = per * kMailSub + ko;
        }
        Mail* m = &c.g->mail_out[slot];
        m->dst = (uint32_t)dl; m->src = (uint32_t)c.gh; m->time = t; m->seq = seq;
        m->sack_off = 0;
        if (p->nsack) {   // the SACK list travels in the mailbox's arena
            const uint32_t off = atomicAdd(c.g->nmsack_out, p->nsack);
            if (off + p->nsack > c.g->msack_cap) { c.H->err |= SHD_TCP_ERR_MAILBOX; return; }
            const int32_t* sk = PSK(c, pi);
            for (uint32_t i = 0; i < p->nsack; i++) c.g->msack_out[off + i] = sk[i];
            m->sack_off = off;
        }
        pkt_copy_rec(&m->pkt, p, c.g->trace);   // packet_copy: the copy starts with one reference (the task's)
        m->pkt.refs = 1;
        m->pkt.inq = 0;   // the copy is in no queue of the receiver
        c.g->mnext_out[slot] = atomicExch(&c.g->mhead_out[dl], (int32_t)slot);   // the receiver's list
    } else {
        pkt_status(c, pi, S_INET_DROPPED);
    }
}
__device__ void if_send_packets(L& c) {   // :519-579, FIFO qdisc
    DHost* H = c.H;
    const SockLess lt{&c};
    while (H->tx_rem >= kMTU) {
        int32_t pi = -1;
        DSock* ks = nullptr;   // the socket the packet came from
        DSock* drained = nullptr;   // ... left the sendable queue (a closed datagram socket is released after)
        while (c.g->qdisc_rr && pi < 0 && H->rrq.n) {   // _networkinterface_selectRoundRobin (:466-490)
            const int32_t si = rg_pop(H->rrq);
            DSock* k = &c.g->sock[si];
            ks = k;
            pi = sock_remove_output(c, k);
            if (pi >= 0 && !k->udp) tcp_about_to_send(c, k, pi);   // _networkinterface_updatePacketHeader (:457-463)
            if (sock_peek_out(c, k) >= 0) rg_push(H->rrq, si, H->err);
            else drained = k;
        }
        while (pi < 0 && H->fifo.n) {   // _networkinterface_selectFirstInFirstOut (:492-517)
            const int32_t si = ih_pop(H->fifo, lt);
            DSock* k = &c.g->sock[si];
            ks = k;
            pi = sock_remove_output(c, k);
            if (pi >= 0 && !k->udp) tcp_about_to_send(c, k, pi);
            if (sock_peek_out(c, k) >= 0) ih_push(H->fifo, si, lt, H->err);
            else drained = k;
        }
        if (pi < 0) {
            if (drained) udp_release(c, drained);
            break;
        }
        pkt_status(c, pi, S_SND_INTERFACE_SENT);
        if (PK(c, pi)->dip == H->ip) {   // our own interface (:548-555): a +1 ns task, no router, no mailbox
            pkt_ref(c, pi);
            DEv e;
            e.time = c.now + 1; e.seq = H->ev_seq++; e.src = (uint32_t)c.gh; e.kind = K_LOCAL; e.obj = -1; e.pkt = pi;
            if (e.time < c.g->end_time) evq_push(c, e);
            else pkt_unref(c, pi);   // scheduler_push refused it: the task's reference goes now
        } else {
            worker_send_packet(c, pi, ks);
        }
        consume(H->tx_rem, (uint64_t)PK(c, pi)->len + hdr_of(PK(c, pi)));
        refill_if_needed(c);
        tracker_add(c, pi, 1);   // :571
        pkt_unref(c, pi);
        if (drained) udp_release(c, drained);
    }
}
__device__ void refill_cb(L& c) {   // :163-183
    DHost* H = c.H;
    H->refill_pending = 0;
    H->rx_rem += H->rx_refill; if (H->rx_rem > H->rx_cap) H->rx_rem = H->rx_cap;
    H->tx_rem += H->tx_refill; if (H->tx_rem > H->tx_cap) H->tx_rem = H->tx_cap;
    if_receive_packets(c);
    if_send_packets(c);
    refill_if_needed(c);
}

// ------------------------------------------------------------ host calls (host.c)
__device__ uint16_t random_port(L& c) {   // :1058-1070
    const double f = next_double(&c.H->rng);
    const double pick = round(f * (double)(65535 - 10000));
    return (uint16_t)((uint16_t)pick + 10000);
}
// _host_isInterfaceAvailable (host.c:1029-1056) -> networkinterface_isAssociated
// (network_interface.c:279-301): the protocol's port is taken by a socket
// associated with no peer (the general key) or with this peer
__device__ bool port_free(L& c, int32_t udp, uint16_t port, uint32_t peer_ip, uint16_t peer_port) {
    for (int32_t j = 0; j < c.H->nsock; j++) {
        const DSock* k = SK(c, j);
        if (!k->assoc || k->udp != udp || k->bound_port != port) continue;
        if (k->assoc_general || (k->peer_ip == peer_ip && k->peer_port == peer_port)) return false;
    }
    return true;
}
__device__ uint16_t random_free_port(L& c, int32_t udp, uint32_t pip, uint16_t pport) {   // :1072-1110
    for (int i = 0; i < 10; i++) { const uint16_t p = random_port(c); if (port_free(c, udp, p, pip, pport)) return p; }
    const uint16_t start = random_port(c);
    uint16_t next = start == 65535 ? 10000 : (uint16_t)(start + 1);
    while (next != start) {
        if (port_free(c, udp, next, pip, pport)) return next;
        next = next == 65535 ? 10000 : (uint16_t)(next + 1);
    }
    return 0;
}
__device__ int tcp_connect_error(DSock* k) {   // tcp.c:1367-1390
    if (k->error & TE_CONNECTION_RESET) {
        k->flags |= TF_RESET_SIGNALED;
        return (k->flags & TF_WAS_ESTABLISHED) ? E_CONNRESET : E_CONNREFUSED;
    }
    if (k->state == TS_SYNSENT || k->state == TS_SYNRECEIVED) return E_ALREADY;
    if ((k->flags & TF_EOF_RD_SIGNALED) && (k->flags & TF_EOF_WR_SIGNALED)) return E_NOTCONN;
    if (k->state != TS_CLOSED) return E_ISCONN;
    return 0;
}
__device__ void tcp_eof_signalled(L& c, DSock* k, uint32_t f) {   // tcp.c:2113-2124
    k->flags |= f;
    if ((k->flags & TF_EOF_RD_SIGNALED) && (k->flags & TF_EOF_WR_SIGNALED)) {
        sock_status(c, k, DS_CLOSED, true);
        sock_status(c, k, DS_ACTIVE, false);
    }
}
__device__ int host_send(L& c, DSock* k, uint64_t n, uint64_t& copied) {   // host.c:1466-1555, tcp.c:2126-2178
    if (k->status & DS_CLOSED) return 9;
    const int err = tcp_connect_error(k);
    if (err != E_ISCONN) {
        if (err == E_ALREADY) { sock_status(c, k, DS_WRITABLE, false); return E_WOULDBLOCK; }
        return err;
    }
    if (k->error & TE_SEND_EOF) {
        if (k->flags & TF_EOF_WR_SIGNALED) return E_NOTCONN;
        tcp_eof_signalled(c, k, TF_EOF_WR_SIGNALED);
        return E_PIPE;
    }
    const uint64_t acceptable = n < 65535 ? n : 65535;
    const uint64_t space = space_out(k);
    uint64_t remaining = acceptable < space ? acceptable : space, done = 0;
    while (remaining > 0) {
        const uint64_t cl = remaining < kMSS ? remaining : kMSS;
        const int32_t pi = tcp_create_packet(c, k, F_ACK, (uint32_t)cl);
        if (pi < 0) return E_WOULDBLOCK;
        if (cl > 0) k->s_end++;
        tcp_buffer_out(c, k, pi);
        pkt_unref(c, pi);
        remaining -= cl;
        done += cl;
    }
    tcp_flush(c, k);
    if (done == 0) return E_WOULDBLOCK;
    copied = done;
    return 0;
}
__device__ int host_receive(L& c, DSock* k, uint64_t n, uint64_t& copied) {   // host.c:1557-1604, tcp.c:2192-2327
    tcp_flush(c, k);
    uint64_t remaining = n, total = 0;
    if (remaining > 0 && k->partial >= 0) {
        const uint32_t pb = PK(c, k->partial)->len - k->partial_off;
        const uint64_t cl = pb < remaining ? pb : remaining;
        total += cl; remaining -= cl;
        if (cl >= pb) {
            pkt_status(c, k->partial, S_RCV_SOCKET_DELIVERED);
            pkt_unref(c, k->partial);
            k->partial = -1;
            k->partial_off = 0;
        } else {
            k->partial_off += (uint32_t)cl;
        }
    }
    while (remaining > 0) {
        const int32_t pi = sock_remove_input(c, k);
        if (pi < 0) break;
        const uint32_t plen = PK(c, pi)->len;
        const uint64_t cl = plen < remaining ? plen : remaining;
        total += cl; remaining -= cl;
        if (cl < plen) { k->partial = pi; k->partial_off = (uint32_t)cl; break; }
        pkt_status(c, pi, S_RCV_SOCKET_DELIVERED);
        pkt_unref(c, pi);
    }
    if (k->in_len > 0 || k->partial >= 0) {
        sock_status(c, k, DS_READABLE, true);
    } else if (k->unordered_len == 0 && (k->error & TE_RECEIVE_EOF)) {
        if (total > 0) {
            sock_status(c, k, DS_READABLE, true);
        } else {
            if (k->flags & TF_EOF_RD_SIGNALED) return E_NOTCONN;
            tcp_eof_signalled(c, k, TF_EOF_RD_SIGNALED);
            copied = 0;
            return 0;
        }
    } else {
        sock_status(c, k, DS_READABLE, false);
    }
    tcp_autotune_rcv(c, k, (uint32_t)total);
    tcp_update_rcv_window(k);
    if (k->r_window > k->s_last_window && !k->r_winupd) {
        sched_task(c, 1, K_WINUPD, sidx(c, k));
        k->r_winupd = 1;
    }
    if (total == 0) return E_WOULDBLOCK;
    copied = total;
    return 0;
}
__device__ void tcp_close(L& c, DSock* k) {   // descriptor_close + tcp_close (tcp.c:2363-2408)
    sock_status(c, k, DS_CLOSED, true);
    k->flags |= TF_LOCAL_CLOSED_WR | TF_LOCAL_CLOSED_RD;
    sock_status(c, k, DS_ACTIVE, false);
    switch (k->state) {
    case TS_LISTEN:
    case TS_SYNSENT: tcp_set_state(c, k, TS_CLOSED); return;
    case TS_SYNRECEIVED:
    case TS_ESTABLISHED:
    case TS_CLOSEWAIT:
        if (tcp_out_len(k) == 0) tcp_send_shutdown_fin(c, k, false);
        else k->flags |= TF_SHOULD_SEND_WR_FIN;
        return;
    case TS_FINWAIT1: case TS_FINWAIT2: case TS_CLOSING: case TS_TIMEWAIT: case TS_LASTACK: return;
    default: tcp_set_state(c, k, TS_CLOSED); return;
    }
}

// ------------------------------------------------------------ datagram sockets (udp.c, host.c)
// host_createDescriptor(DT_UDPSOCKET) -> udp_new (udp.c:211-223): active and
// writable at once, the host's socket buffer sizes
__device__ int32_t udp_sock_new(L& c) {
    const int32_t si = sock_new(c);
    if (si < 0) return -1;
    DSock* k = &c.g->sock[si];
    k->udp = 1;
    k->in_size = c.g->recv_buf;
    k->out_size = c.g->send_buf;
    k->status = DS_ACTIVE | DS_WRITABLE;
    return si;
}
// host_sendUserData (host.c:1466-1555) for a datagram socket: the implicit
// bind of an unbound socket (a random free port on the default interface,
// no peer: :1514-1525), then udp_sendUserData (udp.c:75-142): one packet of
// n <= CONFIG_DATAGRAM_MAX_SIZE bytes into the socket's output buffer
__device__ int udp_send_user(L& c, DSock* k, uint32_t n, uint32_t ip, uint16_t port) {
    if (k->status & DS_CLOSED) return 9;   // EBADF
    if (!k->bound) {
        const uint16_t bp = random_free_port(c, 1, 0, 0);
        if (!bp) return 99;   // EADDRNOTAVAIL
        k->bound = 1; k->bound_ip = c.H->ip; k->bound_port = bp;
        k->peer_ip = 0; k->peer_port = 0;
        k->assoc = 1; k->assoc_general = 1;
    }
    if (out_space(k) < n) return E_WOULDBLOCK;
    const int32_t pi = pkt_new(c, n);
    if (pi < 0) return E_WOULDBLOCK;
    DPkt* p = PK(c, pi);
    p->xflags |= kXUdp;   // packet_setUDP (PUDP_NONE)
    p->sip = k->bound_ip ? k->bound_ip : c.H->ip;   // INADDR_ANY: the default address
    p->sport = k->bound_port; p->dip = ip; p->dport = port;
    pkt_status(c, pi, S_SND_CREATED);
    sock_add_output(c, k, pi);   // the buffer holds the packet's reference (space checked above)
    return 0;
}
// host_receiveUserData -> udp_receiveUserData (udp.c:144-178): the next
// datagram, its source address
__device__ int udp_recv_user(L& c, DSock* k, uint32_t& sip, uint16_t& sport, uint32_t& n) {
    const int32_t pi = sock_remove_input(c, k);
    if (pi < 0) return E_WOULDBLOCK;
    const DPkt* p = PK(c, pi);
    n = p->len < 65536u ? p->len : 65536u;
    pkt_status(c, pi, S_RCV_SOCKET_DELIVERED);
    sip = p->sip; sport = p->sport;
    pkt_unref(c, pi);
    return 0;
}
// a closed datagram socket's last reference goes when it is neither in the
// host's descriptors nor in the interface's sendable queue: its slot is
// released (socket_free drops what its buffers still hold, socket.c:36-56)
__device__ void udp_release(L& c, DSock* k) {
    if (!k->udp || !(k->status & DS_CLOSED) || k->out.n || k->outctl.n) return;
    while (k->in.n) pkt_unref(c, rg_pop(k->in));
    k->used = 0;
}
// host_closeUser -> descriptor_close -> udp_close -> host_closeDescriptor
// (host.c:768-771, 571-583): closed, no longer associated
__device__ void udp_close(L& c, DSock* k) {
    sock_status(c, k, DS_CLOSED, true);
    k->assoc = 0; k->assoc_general = 0;
    udp_release(c, k);
}

// ------------------------------------------------------------ the echo application (test_tcp.c:713-810)
__device__ void app_wait(L& c, DProc* pr, int32_t fd, uint32_t events) {   // epoll_ctl ADD (epoll.c:411-433)
    pr->wait_fd = fd;
    pr->wait_events = events;
    c.g->sock[fd].proc = pr->index;
    ep_status_changed(c, pr);
}

// ------------------------------------------------------------ the datagram application
// shd_udp_app (shdgpu.h) in a process, as the reference's loop runs it
// (oracle/ref_harness/ref_loop.c udp_start / udp_send / udp_continue, over
// test_phold.c's calls): a socket listening on PHOLD's port (SHD_SEND_EACH,
// SHD_SEND_LISTENER) or bound by its first sendto (SHD_SEND_ONCE), one epoll
// watch for reading it for the process's life; n_start datagrams at start,
// one per datagram read when per_read
__device__ void udp_app_send(L& c, DProc* pr, uint32_t rip, uint16_t rport) {
    const uint32_t* a = c.g->app_spec + 4u * (uint32_t)pr->app;
    uint32_t ip;
    uint16_t port = kUdpPort;
    if (a[1] == 0) {   // SHD_DEST_WEIGHTED: _phold_chooseNode (test_phold.c:160-178), the first
                       // host whose cumulative weight reaches the draw (a lower bound: the rows ascend)
        const double r = next_double(&c.H->rng);
        const double* cum = c.g->dest_cum;
        if (c.g->host_class && c.g->n_classes > 1) cum += (size_t)c.g->host_class[c.gh] * (size_t)c.g->H;
        int32_t lo = 0, hi = c.g->H;
        while (lo < hi) {
            const int32_t mid = (lo + hi) >> 1;
            if (cum[mid] >= r) hi = mid; else lo = mid + 1;
        }
        if (lo >= c.g->H) return;   // none: _phold_sendToNode sends nothing
        ip = c.g->ip_all[lo];
    } else if (a[1] == 1) {   // SHD_DEST_PEER
        ip = c.g->ip_all[c.g->app_peer[c.gh]];
    } else {                  // SHD_DEST_REPLY: recvfrom's address
        ip = rip;
        port = rport;
    }
    if (a[0] == 0) {   // SHD_SEND_EACH: socket, sendto (its implicit bind draws a port), close
        const int32_t si = udp_sock_new(c);
        if (si < 0) return;
        DSock* k = &c.g->sock[si];
        (void)udp_send_user(c, k, c.g->udp_payload, ip, port);
        udp_close(c, k);
    } else {
        (void)udp_send_user(c, &c.g->sock[pr->listenfd], c.g->udp_payload, ip, port);
    }
}
__device__ void udp_app_start(L& c, DProc* pr) {
    const uint32_t* a = c.g->app_spec + 4u * (uint32_t)pr->app;
    const int32_t li = udp_sock_new(c);
    if (li < 0) { pr->step = T_DONE; return; }
    pr->listenfd = li;
    DSock* l = &c.g->sock[li];
    if (a[0] != 1 && port_free(c, 1, kUdpPort, 0, 0)) {   // bind INADDR_ANY:8998 (host.c:1111-1189)
        l->bound = 1; l->bound_ip = 0; l->bound_port = kUdpPort;
        l->assoc = 1; l->assoc_general = 1;
    }
    app_wait(c, pr, li, 1);   // epoll_ctl ADD, EPOLLIN
    for (uint32_t i = 0; i < a[2]; i++) udp_app_send(c, pr, 0, 0);
}
// every datagram the socket holds, while epoll_wait reports it readable
__device__ void udp_app_continue(L& c, DProc* pr) {
    const uint32_t* a = c.g->app_spec + 4u * (uint32_t)pr->app;
    DSock* k = &c.g->sock[pr->listenfd];
    for (int guard = 0; watch_ready(c, pr) && guard < (1 << 20); guard++) {
        for (;;) {
            uint32_t ip = 0, n = 0;
            uint16_t port = 0;
            if (udp_recv_user(c, k, ip, port, n) != 0 || n == 0) break;
            if (a[3]) udp_app_send(c, pr, ip, port);
        }
    }
}
__device__ void app_run(L& c, DProc* pr) {
    const uint32_t N = c.g->tcp_bytes;
    for (int guard = 0; guard < 64; guard++) {
        switch (pr->step) {
        case T_SRV_START: {
            const int32_t li = sock_new(c);
            if (li < 0) { pr->step = T_DONE; return; }
            DSock* l = &c.g->sock[li];
            sock_init_tcp(l, c.g->recv_buf, c.g->send_buf, c.g->tcp_window);
            pr->listenfd = li;
            l->bound = 1; l->bound_ip = 0; l->bound_port = random_free_port(c, 0, 0, 0);   // bind INADDR_ANY:0
            publish_port(c, pr->index, l->bound_port);
            l->assoc = 1; l->assoc_general = 1;
            l->server = 1;   // listen (tcp.c:1486-1494)
            tcp_set_state(c, l, TS_LISTEN);
            pr->step = T_SRV_ACCEPT;
            break;
        }
        case T_SRV_ACCEPT: {   // tcp_acceptServerPeer (tcp.c:1496-1558)
            DSock* l = &c.g->sock[pr->listenfd];
            if (l->npending == 0) {
                sock_status(c, l, DS_READABLE, false);
                app_wait(c, pr, pr->listenfd, 1);
                return;
            }
            const int32_t ci = l->pending[0];
            for (uint32_t i = 1; i < l->npending; i++) l->pending[i - 1] = l->pending[i];
            l->npending--;
            DSock* ch = &c.g->sock[ci];
            ch->child_state = 3;
            sock_status(c, ch, DS_ACTIVE | DS_WRITABLE, true);
            sock_status(c, l, DS_READABLE, l->npending > 0);
            pr->fd = ci;
            pr->done = 0;
            pr->step = T_SRV_RECV;
            break;
        }
        case T_SRV_RECV:
        case T_CLI_RECV: {
            while (pr->done < N) {
                uint64_t n = 0;
                const int rc = host_receive(c, &c.g->sock[pr->fd], N - pr->done, n);
                if (rc == E_WOULDBLOCK) { app_wait(c, pr, pr->fd, 1); return; }
                if (rc != 0 || n == 0) break;
                pr->done += (uint32_t)n;
            }
            if (pr->step == T_SRV_RECV) { pr->done = 0; pr->step = T_SRV_SEND; }
            else { tcp_close(c, &c.g->sock[pr->fd]); pr->step = T_DONE; }
            break;
        }
        case T_SRV_SEND:
        case T_CLI_SEND: {
            while (pr->done < N) {
                uint64_t n = 0;
                const int rc = host_send(c, &c.g->sock[pr->fd], N - pr->done, n);
                if (rc == E_WOULDBLOCK) { app_wait(c, pr, pr->fd, 4); return; }
                if (rc != 0 || n == 0) break;
                pr->done += (uint32_t)n;
            }
            if (pr->step == T_SRV_SEND) {
                tcp_close(c, &c.g->sock[pr->fd]);
                tcp_close(c, &c.g->sock[pr->listenfd]);
                pr->step = T_DONE;
            } else {
                pr->done = 0;
                pr->step = T_CLI_RECV;
            }
            break;
        }
        case T_CLI_START: {
            // _fillcharbuf: N rand() calls whose values nothing reads -- the
            // state they leave, by a jump of 3N LCG steps (rand_r takes three)
            c.H->rng = lcg_jump(c.H->rng, 3ull * N);
            const int32_t si = sock_new(c);
            if (si < 0) { pr->step = T_DONE; return; }
            sock_init_tcp(&c.g->sock[si], c.g->recv_buf, c.g->send_buf, c.g->tcp_window);
            pr->fd = si;
            pr->step = T_CLI_CONNECT;
            break;
        }
        case T_CLI_CONNECT: {   // host_connectToPeer (host.c:1191-1282), tcp_connectToPeer (tcp.c:1462-1484)
            // the server's port as test_tcp.c's message queue hands it over (its
            // owner publishes it when it binds; none yet: the client gives up)
            const uint32_t port = c.g->proc_port[pr->peer];
            if (port == 0) { pr->step = T_DONE; return; }
            const int32_t sh = c.g->proc[pr->peer].host;
            const uint32_t ip = c.g->ip_all[sh];
            if (ip != c.H->ip) {   // topology_isRoutable (host.c:1224-1234): a first touch, value unused
                if (c.g->pcm) {
                    double l_, r_;
                    pc_query(c, c.g->hv[c.gh], c.g->hv[sh], l_, r_);
                } else {
                    touch_log(c, c.g->hv[c.gh], c.g->hv[sh]);
                }
            }
            DSock* k = &c.g->sock[pr->fd];
            if (!k->bound) {   // implicit bind to the default interface, peer-specific
                const uint16_t bp = random_free_port(c, 0, ip, port);
                k->bound = 1; k->bound_ip = c.H->ip; k->bound_port = bp;
                k->peer_ip = ip; k->peer_port = port;
                k->assoc = 1; k->assoc_general = 0;
            }
            int rc = tcp_connect_error(k);
            if (rc == E_ISCONN && !(k->flags & TF_CONNECT_SIGNALED)) {
                k->flags |= TF_CONNECT_SIGNALED;
                rc = 0;
            } else if (rc == 0) {
                tcp_send_control(c, k, F_SYN);
                tcp_set_state(c, k, TS_SYNSENT);
                rc = E_INPROGRESS;
            }
            if (rc == E_INPROGRESS || rc == E_ALREADY) { app_wait(c, pr, pr->fd, 4); return; }
            if (rc != 0 && rc != E_ISCONN) { pr->step = T_DONE; return; }
            pr->done = 0;
            pr->step = T_CLI_SEND;
            break;
        }
        default:
            return;
        }
    }
}

// ------------------------------------------------------------ events
__device__ void execute(L& c, const DEv& e) {
    switch (e.kind) {
    case K_HEARTBEAT:   // tracker_heartbeat (tracker.c:566-611): the interval's counters, cleared
        if (c.g->node) {
            DHost* H = c.H;
            if (H->nhb < c.g->node_k) {
                uint64_t* o = c.g->node + ((size_t)c.h * c.g->node_k + H->nhb) * (2 * kTrk);
                for (uint32_t j = 0; j < 2 * kTrk; j++) o[j] = H->trk[j];
            } else {
                H->err |= SHD_TCP_ERR_INTERNAL;
            }
            H->nhb++;
            for (uint32_t j = 0; j < 2 * kTrk; j++) H->trk[j] = 0;
        }
        sched_task(c, c.g->hb, K_HEARTBEAT, -1);
        break;
    case K_REFILL: refill_cb(c); break;
    case K_REFILL_LO: break;
    case K_PSTART: {   // the process's start task (process.c:1334-1357)
        DProc* pr = &c.g->proc[e.obj];
        if (pr->running) break;
        pr->running = 1;
        if (pr->app >= 0) { udp_app_start(c, pr); break; }
        pr->step = pr->peer < 0 ? T_SRV_START : T_CLI_START;
        app_run(c, pr);
        break;
    }
    case K_NOTIFY: {   // _epoll_tryNotify (epoll.c:638-683)
        DProc* pr = &c.g->proc[e.obj];
        pr->ep_scheduled = 0;
        if (!pr->running || !pr->ep_ready) break;
        pr->ep_notifying = 1;
        if (watch_ready(c, pr)) {
            if (pr->app >= 0) {   // the datagram application keeps its watch
                pr->ep_ready = 0;
                udp_app_continue(c, pr);
            } else {   // epoll_wait collects the event, then EPOLL_CTL_DEL
                if (pr->wait_fd >= 0) c.g->sock[pr->wait_fd].proc = -1;
                pr->wait_fd = -1;
                pr->ep_ready = 0;
                app_run(c, pr);
            }
        }
        pr->ep_notifying = 0;
        pr->ep_ready = watch_ready(c, pr);
        if (pr->ep_ready) ep_schedule(c, pr);
        break;
    }
    case K_LOCAL: {   // the loopback task (network_interface.c:551-554)
        if_receive_packet(c, e.pkt);
        c.active = -1;   // the task's reference goes after event_execute cleared the host, as K_DELIVER's
        pkt_unref(c, e.pkt);
        break;
    }
    case K_DELIVER: {   // _worker_runDeliverPacketTask -> router_enqueue (router.c:104-122)
        DHost* H = c.H;
        const bool was_empty = H->cq_n == 0;
        if (H->cq_n >= kCq) { H->err |= SHD_TCP_ERR_QUEUE; break; }
        CqEnt* q = &c.g->cq[(size_t)c.h * kCq + (H->cq_head + H->cq_n) % kCq];
        q->ts = c.now; q->len = PK(c, e.pkt)->len + hdr_of(PK(c, e.pkt)); q->pkt = e.pkt;
        H->cq_n++;
        H->cq_total += q->len;
        pkt_ref(c, e.pkt);
        pkt_status(c, e.pkt, S_ROUTER_ENQUEUED);
        if (was_empty) if_receive_packets(c);
        c.active = -1;   // the task's reference goes after event_execute cleared the host
        pkt_unref(c, e.pkt);
        break;
    }
    case K_DELACK: {   // tcp.c:1767-1774
        DSock* k = &c.g->sock[e.obj];
        k->s_delack_sched = 0;
        if (k->s_delack_counter > 0) { tcp_send_control(c, k, F_ACK); k->s_delack_counter = 0; }
        break;
    }
    case K_RTO: {   // tcp.c:1280-1333
        DSock* k = &c.g->sock[e.obj];
        th_pop(k->timers);
        if (k->state == TS_CLOSED) { k->desired = 0; tcp_clear_retransmit(c, k, 0xffffffffu); break; }
        if (k->nrtx == 0) { k->desired = 0; break; }
        if (k->desired == 0) break;
        if (k->desired > c.now) { tcp_schedule_rto_if_needed(c, k, c.now); break; }
        k->backoff++;
        tcp_set_rto(k, k->rto * 2);
        tcp_set_rto_timer(c, k, c.now);
        reno_timeout(k);
        k->tally.retx.n = 0;   // retransmit_tally_clear_retransmitted
        uint32_t b = k->r_last_ack, en = k->s_highest + 1;   // retransmit_tally_mark_lost (cc:247-255)
        if (b != en + 1) {
            if (b == en) en += 1;
            ranges_insert(k->tally.marked, b, en, c.H->err);
            tally_compute_lost(k->tally, c.H->err);
        }
        tcp_flush(c, k);
        break;
    }
    case K_CLOSE: tcp_set_state(c, &c.g->sock[e.obj], TS_CLOSED); break;   // tcp.c:695-698
    case K_WINUPD: {   // tcp.c:2180-2190
        DSock* k = &c.g->sock[e.obj];
        tcp_send_control(c, k, F_ACK);
        k->r_winupd = 0;
        break;
    }
    default: c.H->err |= SHD_TCP_ERR_INTERNAL; break;
    }
}

// every host's packet free list: pops 0, 1, 2, ...
__global__ void k_tcp_free_init(int32_t* freel, size_t n, uint32_t cap) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) freel[i] = (int32_t)(cap - 1 - (uint32_t)(i % cap));
}

// host_boot at t = 0 (host.c:372-390): heartbeat, the ethernet refill inline,
// the loopback refill at +1 ms, then each process's start task
__global__ void __launch_bounds__(64) k_tcp_boot(Glob g) {
    const int32_t h = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (h >= g.nloc) return;
    Glob gl = g;
    L c{&gl, h, gl.h0 + h, &gl.host[h], 0, h, 0, 0, 0, ~0ull};
    sched_task(c, gl.hb, K_HEARTBEAT, -1);
    refill_cb(c);
    sched_task(c, kMs, K_REFILL_LO, -1);
    for (int j = 0; j < kProcs; j++) {
        const int32_t pi = gl.host_procs[h * kProcs + j];
        if (pi < 0) break;
        const uint64_t st = gl.proc[pi].start;
        sched_task(c, st > 0 ? st : 1, K_PSTART, pi);
    }
    const uint32_t n = c.H->nev;
    gl.next_time[h] = n ? evq_base(&gl, h)[0].time : ~0ull;
}

// the next round's window (worker.c:293's conservative width W past the
// earliest pending event of any host or mailbox); ends the run at end_time.
// One block; launched before every round, so a batch of rounds runs without
// the host.
// path_cache mode: the last round's first-touch log in serial order
// (event_compare's key, then the query's index in its event), replayed
// against the ranks: each logged choice checked, the rows and self paths that
// ran ranked (pc_lookup_at's rule).  One block; the log is small (a vertex is
// first touched once per run).
struct FtKey {
    uint64_t time, seq;
    uint32_t host, src, index, pad;
};
__device__ __forceinline__ bool ft_less(const FtKey& x, const FtKey& y) {
    if (x.time != y.time) return x.time < y.time;
    if (x.host != y.host) return x.host < y.host;
    if (x.src != y.src) return x.src < y.src;
    if (x.seq != y.seq) return x.seq < y.seq;
    return x.index < y.index;
}
// a logged choice the serial order contradicts is harmless when both
// candidates give the pair the same bits (latency and reliability): the lane
// computed exactly what the serial loop computes, and the replay ranks the
// rows as the serial order does (every later choice of that lane that its
// in-round pseudo-ranks decided is logged and checked on its own).  Not
// where a row's run can fail (a vertex without a self-loop: pc_query's miss)
__device__ __forceinline__ bool pv_same(const shd_pv& x, const shd_pv& y) {
    return __double_as_longlong(x.lat) == __double_as_longlong(y.lat) &&
           __double_as_longlong(x.rel) == __double_as_longlong(y.rel);
}
__device__ bool ft_same_value(const Glob& g, int32_t a, int32_t b) {
    if (g.pself_eid[a] < 0 || g.pself_eid[b] < 0) return false;
    const size_t T = (size_t)g.pT;
    if (a == b) return pv_same(g.pself[a], g.prow[(size_t)a * T + a]);
    return pv_same(g.prow[(size_t)a * T + b], g.prow[(size_t)b * T + a]);
}
constexpr uint32_t kFtTile = 512;
constexpr int32_t kFtLdsRanks = 4096;   // vertices whose ranks the replay keeps in LDS
__device__ bool ft_replay(const Glob& g, uint32_t n) {
    __shared__ FtKey tile[kFtTile];
    __shared__ int32_t s_rank[kFtLdsRanks], s_srank[kFtLdsRanks];
    __shared__ uint32_t s_bad;
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    // positions: the entries with a smaller key (the keys are distinct)
    for (uint32_t base = 0; base < n; base += nt) {
        const uint32_t i = base + tid;
        const bool own = i < n;
        FtKey a{};
        if (own) { const shd_tcp_query& q = g.ft[i]; a = FtKey{q.time, q.seq, q.host, q.src, q.index, 0}; }
        uint32_t pos = 0;
        for (uint32_t t0 = 0; t0 < n; t0 += kFtTile) {
            __syncthreads();
            for (uint32_t j = tid; j < kFtTile && t0 + j < n; j += nt) {
                const shd_tcp_query& q = g.ft[t0 + j];
                tile[j] = FtKey{q.time, q.seq, q.host, q.src, q.index, 0};
            }
            __syncthreads();
            const uint32_t m = n - t0 < kFtTile ? n - t0 : kFtTile;
            if (own)
                for (uint32_t j = 0; j < m; j++) pos += ft_less(tile[j], a) ? 1u : 0u;
        }
        if (own) g.ftord[pos] = (int32_t)i;
    }
    const bool lds = g.pT <= kFtLdsRanks;
    if (lds)
        for (int32_t v = (int32_t)tid; v < g.pT; v += (int32_t)nt) { s_rank[v] = g.rank[v]; s_srank[v] = g.srank[v]; }
    if (tid == 0) s_bad = 0;
    __syncthreads();
    int32_t* rk = lds ? s_rank : g.rank;
    int32_t* sk = lds ? s_srank : g.srank;
    // the replay, in chunks of the sorted (source, destination, choice) staged in LDS
    int32_t nr = *g.next_rank;
    uint32_t* chunk = (uint32_t*)tile;   // 3 words an entry
    constexpr uint32_t kChunk = sizeof(tile) / 12;
    for (uint32_t c0 = 0; c0 < n; c0 += kChunk) {
        const uint32_t m = n - c0 < kChunk ? n - c0 : kChunk;
        __syncthreads();
        for (uint32_t j = tid; j < m; j += nt) {
            const shd_tcp_query& q = g.ft[g.ftord[c0 + j]];
            chunk[3 * j] = (uint32_t)q.v_src; chunk[3 * j + 1] = (uint32_t)q.v_dst; chunk[3 * j + 2] = q._pad;
        }
        __syncthreads();
        if (tid == 0) {
            for (uint32_t j = 0; j < m; j++) {
                const int32_t a = (int32_t)chunk[3 * j], b = (int32_t)chunk[3 * j + 1];
                const uint32_t choice = chunk[3 * j + 2];
                uint32_t truth;
                if (a == b) {
                    const int32_t ra = rk[a], rs = sk[a];
                    if (ra == kNoRank && rs == kNoRank) { sk[a] = nr++; truth = kFtSelf; }
                    else truth = rs < ra ? kFtSelf : kFtRowA;
                } else {
                    const int32_t ra = rk[a], rb = rk[b];
                    if (ra == kNoRank && rb == kNoRank) { rk[a] = nr++; truth = kFtRowA; }
                    else truth = (ra != kNoRank && (rb == kNoRank || ra < rb)) ? kFtRowA : kFtRowB;
                }
                if (truth != choice && !ft_same_value(g, a, b)) s_bad = 1;
            }
        }
    }
    __syncthreads();
    if (lds)
        for (int32_t v = (int32_t)tid; v < g.pT; v += (int32_t)nt) { g.rank[v] = s_rank[v]; g.srank[v] = s_srank[v]; }
    if (tid == 0) { *g.next_rank = nr; *g.nft = 0; }
    __syncthreads();
    return s_bad != 0;
}

// local: a group's round -- this engine's earliest pending event goes to
// ctl->tmin and the host decides the window over the group (k_tcp_decide)
__global__ void k_tcp_window(Glob g, int local) {
    __shared__ uint64_t red[16];
    TCtl* ctl = g.ctl;
    if (ctl->halted) return;
    if (g.pcm) {
        const uint32_t n = *g.nft;   // the last round's log (uniform)
        if (n) {
            const int32_t nr0 = *g.next_rank;
            const bool bad = n > g.ft_cap || ft_replay(g, n);
            if (bad) {
                if (threadIdx.x == 0) { ctl->ft_bad = 1; ctl->ft_nr0 = (uint32_t)nr0; ctl->halted = 1; }
                return;
            }
        }
        // the schedule's entry for the round this window opens: its first
        // touches ranked, in the serial order an earlier run of the same
        // model found for them, before any lane queries (one engine)
        if (!local && threadIdx.x == 0 && ctl->sched_i < g.sched_n &&
            g.sched_round[ctl->sched_i] == (uint32_t)(ctl->rounds + 1)) {
            const uint32_t i = ctl->sched_i;
            int32_t nr = *g.next_rank;
            for (uint32_t j = g.sched_off[i]; j < g.sched_off[i + 1]; j++) {
                const int32_t v = g.sched_v[j];
                if (v >= 0) g.rank[v] = nr++;
                else g.srank[~v] = nr++;
            }
            *g.next_rank = nr;
            ctl->sched_i = i + 1;
        }
    }
    __shared__ uint32_t s_mail;
    if (threadIdx.x == 0) s_mail = 0;
    __syncthreads();
    {   // the next round's output mailbox starts empty (read before thread 0 moves
        // rounds on); what it took two rounds ago is counted first
        const uint64_t k = ctl->rounds;
        if (threadIdx.x <= kMailSub) {
            uint32_t* n = &g.nmail[((k + 1) & 1) * (kMailSub + 1) + threadIdx.x];
            const uint32_t cap = threadIdx.x < kMailSub ? g.mail_part : g.mail_cap - g.mail_part * kMailSub;
            const uint32_t v = *n;
            if (v) atomicAdd(&s_mail, v < cap ? v : cap);
            if (threadIdx.x == kMailSub && v > ctl->max_ovf) ctl->max_ovf = v < cap ? v : cap;
            *n = 0;
        }
        if (threadIdx.x == kMailSub + 1) g.nmsack[(k + 1) & 1] = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0 && s_mail > ctl->max_mail) ctl->max_mail = s_mail;
    uint64_t t = ~0ull;
    for (int32_t i = (int32_t)threadIdx.x; i <= g.nloc; i += (int32_t)blockDim.x) {
        const uint64_t x = g.next_time[i];
        t = x < t ? x : t;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t y = __shfl_xor(t, o);
        t = y < t ? y : t;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t w = 1; w < blockDim.x / 64; w++) t = red[w] < t ? red[w] : t;
        if (local) {
            ctl->tmin = t;
            g.next_time[g.nloc] = ~0ull;
        } else if (t == ~0ull || t >= g.end_time) {
            ctl->halted = 1;
        } else {
            const uint64_t k = ctl->rounds;
            ctl->wend = t + g.W;
            ctl->rounds = k + 1;
            g.next_time[g.nloc] = ~0ull;  // ... and so does its earliest delivery
        }
    }
}

// ---- a group's exchange (shd_tcp_run_group)
// the window over the group: t (the min of the engines' ctl->tmin); the
// segments and publications of the round start empty
__global__ void k_tcp_decide(Glob g, uint64_t t) {
    TCtl* ctl = g.ctl;
    if (threadIdx.x == 0) {
        if (ctl->halted) return;
        if (t == ~0ull || t >= g.end_time) {
            ctl->halted = 1;
        } else {
            ctl->wend = t + g.W;
            ctl->rounds++;
        }
        *g.nport_new = 0;
    }
    if ((int)threadIdx.x < g.world) {
        XSegHead* hd = (XSegHead*)(g.xsend + (size_t)threadIdx.x * g.xseg);
        hd->n = 0; hd->nsack = 0; hd->err = 0;
    }
}
// the deliveries the other engines sent this engine in the round just run:
// into the round's output mailbox after its own slots (slot mail_cap + r *
// xcap + i), each linked into its host's list, its SACK list into the arena
// cnt: [world][2] the mails and SACK words each engine sent this one
__global__ void k_tcp_xingest(Glob g, const char* __restrict__ xrecv, const uint32_t* __restrict__ cnt) {
    const int32_t r = (int32_t)blockIdx.x;
    if (r == g.me) return;
    const TCtl* ctl = g.ctl;
    const uint64_t k = ctl->rounds - 1;
    const uint32_t out = (uint32_t)(k & 1) ^ 1u;
    const char* seg = xrecv + (size_t)r * g.xseg;
    const uint32_t n = cnt[2 * r] < g.xcap ? cnt[2 * r] : g.xcap;
    const Mail* src = (const Mail*)(seg + sizeof(XSegHead));
    const int32_t* sks = (const int32_t*)(seg + sizeof(XSegHead) + (size_t)g.xcap * sizeof(Mail));
    Mail* mail = g.mail + (size_t)out * g.mail_stride;
    int32_t* mhead = g.mhead + (size_t)out * g.nloc;
    int32_t* mnext = g.mnext + (size_t)out * g.mail_stride;
    int32_t* msack = g.msack + (size_t)out * g.msack_cap;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        Mail m = src[i];
        const int32_t dl = (int32_t)m.dst - g.h0;
        if (dl < 0 || dl >= g.nloc) { atomicOr(&g.ctl->xerr, (uint32_t)SHD_TCP_ERR_INTERNAL); continue; }
        if (m.pkt.nsack) {
            if (m.pkt.nsack > kPktSack || m.sack_off + m.pkt.nsack > g.xsack_cap) {
                atomicOr(&g.ctl->xerr, (uint32_t)SHD_TCP_ERR_INTERNAL);
                continue;
            }
            const uint32_t off = atomicAdd(g.nmsack + out, m.pkt.nsack);
            if (off + m.pkt.nsack > g.msack_cap) { atomicOr(&g.ctl->xerr, (uint32_t)SHD_TCP_ERR_MAILBOX); continue; }
            for (uint32_t j = 0; j < m.pkt.nsack; j++) msack[off + j] = sks[m.sack_off + j];
            m.sack_off = off;
        }
        m.dst = (uint32_t)dl;
        const uint32_t slot = g.mail_cap + (uint32_t)r * g.xcap + i;
        mail[slot] = m;
        mnext[slot] = atomicExch(&mhead[dl], (int32_t)slot);
    }
}
// what this engine's segments hold after the round ([world][2]: mails, SACK
// words), then the round's first-touch log entries (path_cache mode)
__global__ void k_tcp_xheads(Glob g, uint32_t* __restrict__ heads) {
    const int32_t p = (int32_t)threadIdx.x;
    if (p == 0) heads[2 * g.world] = g.pcm ? *g.nft : 0u;
    if (p >= g.world) return;
    const XSegHead* hd = (const XSegHead*)(g.xsend + (size_t)p * g.xseg);
    heads[2 * p] = hd->n < g.xcap ? hd->n : g.xcap;
    heads[2 * p + 1] = hd->nsack < g.xsack_cap ? hd->nsack : g.xsack_cap;
}
// the listening ports the group's engines published in the last round
// ([world][1 + pcap]: the count, then process << 32 | port)
__global__ void k_tcp_ports(Glob g, const uint64_t* __restrict__ all) {
    const int32_t r = (int32_t)blockIdx.x;
    const uint64_t* a = all + (size_t)r * (1 + g.pcap);
    const uint32_t n = (uint32_t)a[0] < g.pcap ? (uint32_t)a[0] : g.pcap;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint64_t v = a[1 + i];
        g.proc_port[(uint32_t)(v >> 32)] = (uint32_t)v;
    }
}
// this engine's publications of the round, packed for the all-gather
__global__ void k_tcp_ports_pack(Glob g, uint64_t* __restrict__ mine) {
    const uint32_t n = *g.nport_new;
    if (threadIdx.x == 0) mine[0] = n;
    for (uint32_t i = threadIdx.x; i < n && i < g.pcap; i += blockDim.x) mine[1 + i] = g.port_new[i];
}

// a delivery from the round's input mailbox onto the host's heap (its packet
// copied into the pool, its SACK list from the mailbox's arena)
__device__ bool ingest_mail(L& c, int32_t s) {
    const Glob& gl = *c.g;
    const Mail* m = &gl.mail_in[s];
    const int32_t pi = pkt_alloc(c);
    if (pi < 0) return false;
    pkt_copy_rec(PK(c, pi), &m->pkt, gl.trace);
    if (m->pkt.nsack) {
        int32_t* sk = PSK(c, pi);
        for (uint32_t i = 0; i < m->pkt.nsack; i++) sk[i] = gl.msack_in[m->sack_off + i];
    }
    DEv e;
    e.time = m->time; e.seq = m->seq; e.src = m->src; e.kind = K_DELIVER; e.obj = -1; e.pkt = pi;
    evq_push(c, e);
    c.H->deliveries++;
    return true;
}

// one conservative round: the mailbox's deliveries for this host, then every
// event before the window's end
__global__ void __launch_bounds__(64) k_tcp_round(Glob g) {
    // the round's view of the globals is uniform: one copy in LDS that every
    // lane's c.g reads by broadcast (a per-lane copy would live in scratch)
    __shared__ Glob gl;
    const int32_t h = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (g.ctl->halted) return;   // uniform: read before any lane diverges
    const uint64_t k = g.ctl->rounds - 1, wend = g.ctl->wend;
    const uint32_t in = (uint32_t)(k & 1), out = in ^ 1u;
    if (threadIdx.x == 0) {
        gl = g;
        gl.mail_in = g.mail + (size_t)in * g.mail_stride; gl.mhead_in = g.mhead + (size_t)in * g.nloc;
        gl.mnext_in = g.mnext + (size_t)in * g.mail_stride;
        gl.mail_out = g.mail + (size_t)out * g.mail_stride; gl.n_out = g.nmail + (size_t)out * (kMailSub + 1);
        gl.mhead_out = g.mhead + (size_t)out * g.nloc; gl.mnext_out = g.mnext + (size_t)out * g.mail_stride;
        gl.msack_in = g.msack + (size_t)in * g.msack_cap; gl.msack_out = g.msack + (size_t)out * g.msack_cap;
        gl.nmsack_out = g.nmsack + out;
    }
    __syncthreads();
    if (h >= g.nloc) return;
#ifndef SHD_TCP_GLOBAL_HOST
    // the host's record lives in LDS for the round (every H-> access of its
    // events at LDS latency instead of a cache's): other lanes read only its
    // fixed fields (ip, bandwidths, refills) from the global copy
    __shared__ DHost s_host[64];
    s_host[threadIdx.x] = gl.host[h];
    L c{&gl, h, gl.h0 + h, &s_host[threadIdx.x], 0, h, 0, 0, 0, ~0ull};
#else
    L c{&gl, h, gl.h0 + h, &gl.host[h], 0, h, 0, 0, 0, ~0ull};
#endif
#ifdef SHD_TCP_PROF
    uint64_t* pf = gl.prof + (size_t)h * 2 * kProf;
    const uint64_t t_lane = clock64();
    uint64_t t_p = t_lane;
#define TCP_PROF(slot) do { const uint64_t t_ = clock64(); pf[(slot)] += t_ - t_p; pf[kProf + (slot)]++; t_p = t_; } while (0)
#else
#define TCP_PROF(slot) do { } while (0)
#endif
    // this host's deliveries (any order: the heap's key (time, src, seq) is
    // unique; the chain measured faster than an index per destination, 20.14
    // against 19.69 M TCP events/s, profiles/r04/tcpab4)
    int32_t s = gl.mhead_in[h];
    gl.mhead_in[h] = -1;   // the list is empty again when this mailbox is next written
    for (; s >= 0; s = gl.mnext_in[s])
        if (!ingest_mail(c, s)) break;
    TCP_PROF(0);
    uint64_t nev = 0;
    while (c.H->nev && evq_base(&gl, h)[0].time < wend && !c.H->err) {
        const DEv e = evq_pop(c);
        TCP_PROF(1);
        c.now = e.time;
        c.active = h;
        c.ksrc = e.src; c.kseq = e.seq; c.kq = 0;
        execute(c, e);
        TCP_PROF(2 + (e.kind < 12 ? e.kind : 12));
        if (++nev > (1u << 24)) c.H->err |= SHD_TCP_ERR_INTERNAL;   // a runaway round: stop, report
    }
#ifdef SHD_TCP_PROF
    {
        const uint64_t cyc = clock64() - t_lane;
        pf[14] += cyc; pf[kProf + 14]++;
        if (nev > pf[15]) pf[15] = nev;
        if (k < kProfRounds) {
            atomicMax(gl.prof_round + k, (uint32_t)nev);
            atomicMax(gl.prof_round + kProfRounds + k, (uint32_t)(cyc >> 10));
        }
    }
#endif
    c.H->events += nev;
    // a host that stopped on an error leaves the run (the caller sees the bit)
    gl.next_time[h] = (c.H->nev && !c.H->err) ? evq_base(&gl, h)[0].time : ~0ull;
    if (c.mail_min < gl.next_time[h]) gl.next_time[h] = c.mail_min;   // its deliveries count either way
#ifndef SHD_TCP_GLOBAL_HOST
    gl.host[h] = *c.H;
#endif
}

#define HCHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "shd_tcp: %s: %s\n", #x, hipGetErrorString(e_)); rc = -5; goto done; } } while (0)

void ip_str(uint32_t ip, char* b) { snprintf(b, 20, "%u.%u.%u.%u", (ip >> 24) & 255, (ip >> 16) & 255, (ip >> 8) & 255, ip & 255); }

// packet_toString (packet.c:518-641) from a device record
void format_line(std::string& o, const TRec& r, const int32_t* sacks, int32_t host) {
    char buf[512], s[20], d[20];
    ip_str(r.sip, s);
    ip_str(r.dip, d);
    if (r.flags & kTrUdp) {   // PUDP (packet.c:535-548)
        snprintf(buf, sizeof(buf), "%llu\t%d\t[%s] packetID=%u:%llu %s:%u -> %s:%u bytes=%u", (unsigned long long)r.time,
                 host, kStatusName[r.status], r.host_id, (unsigned long long)r.pid, s, r.sport, d, r.dport, r.len);
        o += buf;
        if (r.nst) {
            o += " status=";
            for (uint32_t i = 0; i < r.nst && i < kSt; i++) {
                o += kStatusName[r.st[i]];
                if (i + 1 < r.nst) o += ",";
            }
        }
        o += "\n";
        return;
    }
    snprintf(buf, sizeof(buf), "%llu\t%d\t[%s] packetID=%u:%llu %s:%u -> %s:%u seq=%u ack=%u sack=",
             (unsigned long long)r.time, host, kStatusName[r.status], r.host_id, (unsigned long long)r.pid, s, r.sport, d,
             r.dport, r.seq, r.ack);
    o += buf;
    int32_t first = -1, last = -1;
    for (uint32_t i = 0; i < r.nsack; i++) {
        const int32_t sq = sacks[i];
        if (first == -1) first = sq;
        else if (last == -1 || sq == last + 1) last = sq;
        else { snprintf(buf, sizeof(buf), "%d-%d ", first, last); o += buf; first = sq; last = -1; }
    }
    if (first != -1) {
        snprintf(buf, sizeof(buf), "%d", first); o += buf;
        if (last != -1) { snprintf(buf, sizeof(buf), "-%d", last); o += buf; }
    } else {
        o += "NA";
    }
    snprintf(buf, sizeof(buf), " window=%u bytes=%u header=", r.win, r.len);
    o += buf;
    if (r.flags & F_RST) o += "RST";
    if (r.flags & F_SYN) o += "SYN";
    if (r.flags & F_FIN) o += "FIN";
    if (r.flags & F_ACK) o += "ACK";
    if (r.flags & F_DUPACK) o += "DUPACK";
    snprintf(buf, sizeof(buf), " tsval=%llu tsechoreply=%llu", (unsigned long long)r.tsval, (unsigned long long)r.tsecho);
    o += buf;
    if (r.nst) {
        o += " status=";
        for (uint32_t i = 0; i < r.nst && i < kSt; i++) {
            o += kStatusName[r.st[i]];
            if (i + 1 < r.nst) o += ",";
        }
    }
    o += "\n";
}

int32_t rand_r_host(uint32_t* state) {
    uint32_t next = *state;
    int32_t result;
    next *= 1103515245u; next += 12345u;
    result = (int32_t)((next / 65536u) % 2048u);
    next *= 1103515245u; next += 12345u;
    result <<= 10; result ^= (int32_t)((next / 65536u) % 1024u);
    next *= 1103515245u; next += 12345u;
    result <<= 10; result ^= (int32_t)((next / 65536u) % 1024u);
    *state = next;
    return result;
}

}  // namespace

// path_cache mode's window and route check, from the cache's device tables:
// the smallest ceil(latency) in ns over the connections' vertex pairs (hosts
// that talk only to their peers: the same pairs the table path fills), in
// both orientations' rows (either endpoint's may serve the pair; the window
// only bounds the rounds), and whether some connection's pair has no route.
// conn: (client vertex, server vertex, same host, route required) quads.
__global__ void k_tcp_pc_prep(const shd_pv* __restrict__ row, const shd_pv* __restrict__ self,
                              const shd_pv* __restrict__ dir, const uint8_t* __restrict__ adj, int complete,
                              int prefer_direct, int32_t T, const int32_t* __restrict__ conn, int32_t nconn,
                              unsigned long long* __restrict__ out) {
    auto lat_of = [&](int32_t u, int32_t v, double& l) {
        if (complete || (prefer_direct && adj[(size_t)u * T + v])) { l = dir[(size_t)u * T + v].lat; return; }
        if (u == v) {
            const double a = self[u].lat, b = row[(size_t)u * T + u].lat;
            l = (a >= 0 && (b < 0 || a < b)) ? a : b;
            return;
        }
        const double a = row[(size_t)u * T + v].lat, b = row[(size_t)v * T + u].lat;
        l = (a >= 0 && b >= 0) ? (a < b ? a : b) : -1.0;
    };
    unsigned long long w = ~0ull;
    for (int32_t k = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x); k < nconn; k += (int32_t)(gridDim.x * blockDim.x)) {
        const int32_t u = conn[4 * k], v = conn[4 * k + 1];
        double l1, l2;
        lat_of(u, v, l1);
        lat_of(v, u, l2);
        if (!(l1 >= 0) || !(l2 >= 0)) {
            if (conn[4 * k + 3]) atomicOr(out + 1, 1ull);   // a connection's pair without a route
            continue;
        }
        if (conn[4 * k + 2]) continue;   // a host's connection to itself: the loopback, no path
        const double l = l1 < l2 ? l1 : l2;
        const unsigned long long x = (unsigned long long)ceil(l * (double)kMs);
        w = x < w ? x : w;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(w, o);
        w = y < w ? y : w;
    }
    if ((threadIdx.x & 63) == 0 && w != ~0ull) atomicMin(out, w);
}

// the datagram processes' share of the window (any two hosts may exchange a
// datagram): the least latency over every pair of vertices hosts occupy (occ:
// 0 none, 1 one host, 2 several; a vertex with itself only when two hosts
// share it), straight from the occupancy on the device -- no host-side list of
// pairs (O(V^2) of them once hosts sit on ~10 k vertices)
__global__ void k_tcp_pc_prep_occ(const shd_pv* __restrict__ row, const shd_pv* __restrict__ self,
                                  const shd_pv* __restrict__ dir, const uint8_t* __restrict__ adj, int complete,
                                  int prefer_direct, int32_t T, const uint8_t* __restrict__ occ,
                                  unsigned long long* __restrict__ out) {
    auto lat_of = [&](int32_t u, int32_t v, double& l) {
        if (complete || (prefer_direct && adj[(size_t)u * T + v])) { l = dir[(size_t)u * T + v].lat; return; }
        if (u == v) {
            const double a = self[u].lat, b = row[(size_t)u * T + u].lat;
            l = (a >= 0 && (b < 0 || a < b)) ? a : b;
            return;
        }
        const double a = row[(size_t)u * T + v].lat, b = row[(size_t)v * T + u].lat;
        l = (a >= 0 && b >= 0) ? (a < b ? a : b) : -1.0;
    };
    unsigned long long w = ~0ull;
    const uint64_t n = (uint64_t)T * (uint64_t)T;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
        const int32_t u = (int32_t)(k / (uint64_t)T), v = (int32_t)(k % (uint64_t)T);
        if (v < u || !occ[u] || !occ[v] || (u == v && occ[u] < 2)) continue;
        double l1, l2;
        lat_of(u, v, l1);
        lat_of(v, u, l2);
        if (!(l1 >= 0) || !(l2 >= 0)) continue;   // (no route: the datagram is never sent)
        const double l = l1 < l2 ? l1 : l2;
        const unsigned long long x = (unsigned long long)ceil(l * (double)kMs);
        w = x < w ? x : w;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(w, o);
        w = y < w ? y : w;
    }
    if ((threadIdx.x & 63) == 0 && w != ~0ull) atomicMin(out, w);
}

static int tcp_pc_prep(shd_pc* pc, const std::vector<int32_t>& conn, const std::vector<uint8_t>& occ, uint64_t* W) {
    int32_t* d_conn = nullptr;
    unsigned long long* d_out = nullptr;
    unsigned long long h_out[2] = {~0ull, 0ull};
    int rc = 0;
    const int32_t T = pc->T;
    const int32_t nconn = (int32_t)(conn.size() / 4);
    if (hipSetDevice(pc->device) != hipSuccess || hipMalloc(&d_conn, sizeof(int32_t) * (conn.size() + 4)) != hipSuccess ||
        hipMalloc(&d_out, 16) != hipSuccess ||
        (nconn && hipMemcpy(d_conn, conn.data(), sizeof(int32_t) * conn.size(), hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(d_out, h_out, 16, hipMemcpyHostToDevice) != hipSuccess) {
        rc = -5;
    } else {
        k_tcp_pc_prep<<<(unsigned)std::min<int32_t>((nconn + 255) / 256 + 1, 1024), 256>>>(
            pc->d_row, pc->d_self, pc->d_dir, pc->d_adj, pc->complete, pc->prefer_direct, T, d_conn, nconn, d_out);
        if (!occ.empty()) {
            uint8_t* d_occ = nullptr;
            if (hipMalloc(&d_occ, occ.size()) != hipSuccess ||
                hipMemcpy(d_occ, occ.data(), occ.size(), hipMemcpyHostToDevice) != hipSuccess) {
                rc = -5;
            } else {
                const uint64_t n = (uint64_t)T * (uint64_t)T;
                k_tcp_pc_prep_occ<<<(unsigned)std::min<uint64_t>((n + 255) / 256, 4096), 256>>>(
                    pc->d_row, pc->d_self, pc->d_dir, pc->d_adj, pc->complete, pc->prefer_direct, T, d_occ, d_out);
            }
            (void)hipFree(d_occ);   // (hipFree waits for the kernel)
        }
        if (rc || hipGetLastError() != hipSuccess || hipMemcpy(h_out, d_out, 16, hipMemcpyDeviceToHost) != hipSuccess)
            rc = -5;
    }
    (void)hipFree(d_conn); (void)hipFree(d_out);
    if (rc) return rc;
    if (h_out[1]) return -113;   // EHOSTUNREACH, as the table path
    *W = h_out[0];
    return 0;
}

// a group's small all-gather of host words through two kept device buffers (one
// RCCL all-gather on the run's stream, or the host transport's): shd_comm_
// allgather_host would allocate and free device memory every call, twice a round
static int group_allgather(shd_comm* comm, char* d_mine, char* d_all, const void* mine, void* all, size_t bytes,
                           hipStream_t st) {
    if (comm->kind == SHD_COMM_HOST) return shd_comm_allgather_host(comm, mine, bytes, all) ? -5 : 0;
    if (hipMemcpyAsync(d_mine, mine, bytes, hipMemcpyHostToDevice, st) != hipSuccess) return -5;
    if (shd_comm_allgather_dev(comm, d_mine, d_all, bytes, st)) return -5;
    if (hipMemcpyAsync(all, d_all, bytes * (size_t)comm->world, hipMemcpyDeviceToHost, st) != hipSuccess) return -5;
    return hipStreamSynchronize(st) == hipSuccess ? 0 : -5;
}

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

// The run's device buffers come from a per-device workspace.  By default it
// is released at the end of each call; after shd_tcp_keep_workspace(1) it
// outlasts the call (grown when a run needs more) until
// shd_tcp_keep_workspace(0): the per-host arenas of a large model are tens of
// GB, and allocating and freeing them every call costs more wall time than
// the rounds themselves.  One run at a time uses a device's
// workspace (its lock is held for the call).
enum WsSlot {
    kWsLat, kWsRel, kWsRank, kWsSrank, kWsNextRank, kWsFt, kWsFtord, kWsNft, kWsHv, kWsHost, kWsSock, kWsProc,
    kWsHostProcs, kWsPool, kWsPsack, kWsFreel, kWsEv, kWsCq, kWsMsack, kWsNmsack, kWsMail, kWsNmail, kWsMhead,
    kWsMnext, kWsCtl, kWsIpk, kWsNode, kWsTr, kWsTrs, kWsNextTime, kWsQlog, kWsNqlog, kWsProf, kWsProfRound,
    kWsAppSpec, kWsAppPeer, kWsDestCum, kWsHostClass, kWsIpAll, kWsBwu, kWsBwd, kWsProcPort, kWsPortNew, kWsXsend,
    kWsXrecv, kWsPmine, kWsPall, kWsXcnt, kWsGmine, kWsGall, kWsSlots
};
struct TcpWs {
    std::mutex mu;
    void* p[kWsSlots] = {};
    size_t n[kWsSlots] = {};
};
constexpr int kWsDevices = 64;
static TcpWs g_ws[kWsDevices];

static void ws_free_all(TcpWs& w) {
    for (int i = 0; i < kWsSlots; i++) {
        if (w.p[i]) (void)hipFree(w.p[i]);
        w.p[i] = nullptr;
        w.n[i] = 0;
    }
}

template <class T>
static hipError_t ws_alloc(TcpWs& w, int slot, T** out, size_t bytes) {
    if (bytes == 0) bytes = 1;
    if (w.n[slot] < bytes) {
        if (w.p[slot]) (void)hipFree(w.p[slot]);
        w.p[slot] = nullptr;
        w.n[slot] = 0;
        const hipError_t e = hipMalloc(&w.p[slot], bytes);
        if (e != hipSuccess) return e;
        w.n[slot] = bytes;
    }
    *out = (T*)w.p[slot];
    return hipSuccess;
}

static bool g_ws_keep = false;

extern "C" void shd_tcp_keep_workspace(int32_t keep) {
    g_ws_keep = keep != 0;
    if (keep) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (int d = 0; d < kWsDevices; d++) {
        std::lock_guard<std::mutex> lk(g_ws[d].mu);
        bool any = false;
        for (int i = 0; i < kWsSlots; i++) any |= g_ws[d].p[i] != nullptr;
        if (!any) continue;
        (void)hipSetDevice(d);
        ws_free_all(g_ws[d]);
    }
    (void)hipSetDevice(cur);
}

// shd_tcp_run on one engine (comm null) or on this engine's share of a group
// (shd_tcp_run_group: hosts [h0, h0 + nloc), the round's window agreed over
// the group, deliveries between engines exchanged after every round)
// one engine's first-touch schedule across the reruns of one shd_tcp_run call
// (Glob::sched_*): a run whose round R contradicts a device choice that changes
// a value stops there; the ranks that round's replay assigned, in serial order,
// are added for round R and the model runs again from the start -- the rounds
// before R are the same rounds, and in round R every such pair then has a
// ranked endpoint at the round's start, which is the serial loop's value
constexpr size_t kFtReruns = 256;   // schedule entries (reruns) one call makes at most
struct TcpSched {
    std::vector<uint32_t> round, off{0};
    std::vector<int32_t> v;
    bool extended = false;
};
static int tcp_run_impl(const shd_tcp_model* m, shd_comm* comm, int32_t trace, shd_tcp_result** out,
                        TcpSched* sch = nullptr) {
    const auto t_call = std::chrono::steady_clock::now();
    auto t_results = t_call;
    shd_pc* pc = m ? m->path_cache : nullptr;
    const int32_t world = comm ? comm->world : 1, me = comm ? comm->rank : 0;
    if (!m || !out || m->n_hosts <= 0 || m->n_hosts > (1 << 26) || m->n_procs < 0 || !m->host_ip || !m->host_seed || !m->bw_down_kibps ||
        !m->bw_up_kibps || (!pc && (!m->path_lat_ms || !m->path_rel || m->n_vertices <= 0)) || !m->host_vertex ||
        (m->n_procs && (!m->proc_host || !m->proc_start || !m->proc_peer)))
        return -22;
    // path_cache mode: a built cache of an undirected graph (the directed
    // lookup reruns rows, topology.c:1987-1990: not restated on the device)
    if (pc && (!pc->built || pc->directed || (!pc->complete && !pc->d_row))) return -22;
    const int32_t H = m->n_hosts, P = m->n_procs;
    if (world > H || world > 64) return -22;   // (the group's per-engine tables below hold 64)
    const int32_t h0 = (int32_t)(((int64_t)me * H) / world);
    const int32_t nloc = (int32_t)(((int64_t)(me + 1) * H) / world) - h0;
    auto app_of = [&](int32_t k) { return m->proc_app ? m->proc_app[k] : -1; };
    bool any_udp = false;
    for (int32_t k = 0; k < P; k++) {
        if (m->proc_host[k] < 0 || m->proc_host[k] >= H) return -22;
        if (m->proc_peer[k] >= P || (m->proc_peer[k] >= 0 && m->proc_peer[m->proc_peer[k]] >= 0)) return -22;
        // a client's server runs the echo; a datagram process has no echo peer
        if (m->proc_peer[k] >= 0 && app_of(m->proc_peer[k]) >= 0) return -22;
        if (app_of(k) >= 0 && m->proc_peer[k] >= 0) return -22;
        any_udp |= app_of(k) >= 0;
    }
    if (any_udp) {   // the datagram processes' applications (shd_tcp_model's comment)
        if (!m->app_spec || m->n_app_specs <= 0 || m->udp_payload < 1 || m->udp_payload > kDgramMax) return -22;
        std::vector<uint8_t> seen(H, 0);
        for (int32_t k = 0; k < P; k++) {
            const int32_t a = app_of(k);
            if (a < 0) continue;
            if (a >= m->n_app_specs || seen[m->proc_host[k]]++) return -22;
            const uint32_t* s = m->app_spec + 4 * (size_t)a;
            if (s[0] > 2 || s[1] > 2 || s[3] > 1) return -22;
            if (s[1] == 0 && !m->dest_cum) return -22;
            if (s[1] == 1 && (!m->app_peer || m->app_peer[m->proc_host[k]] < 0 || m->app_peer[m->proc_host[k]] >= H))
                return -22;
        }
        if (m->host_class && m->n_classes > 1)
            for (int32_t a = 0; a < H; a++) if (m->host_class[a] >= m->n_classes) return -22;
    }
    const int32_t V = pc ? pc->T : m->n_vertices;
    std::vector<int32_t> hvi(H);   // each host's table index: the given one, or its attached index in the cache
    for (int32_t a = 0; a < H; a++) {
        if (pc) {
            if (m->host_vertex[a] < 0 || m->host_vertex[a] >= pc->V || pc->h_att_index[m->host_vertex[a]] < 0) return -22;
            hvi[a] = pc->h_att_index[m->host_vertex[a]];
        } else {
            if (m->host_vertex[a] < 0 || m->host_vertex[a] >= V) return -22;
            hvi[a] = m->host_vertex[a];
        }
    }
    const uint32_t pool_cap = m->packets_per_host ? m->packets_per_host : kPoolDefault;
    if (pool_cap > (1u << 24)) return -22;
    std::vector<int32_t> per_vertex(V, 0);
    for (int32_t a = 0; a < H; a++) per_vertex[hvi[a]]++;
    uint64_t W = ~0ull;
    if (!pc) {
        // a client whose server is unreachable: the reference's connect fails with
        // ECONNREFUSED (host.c:1224-1234, topology_isRoutable); the device
        // application has no such branch, so the model is refused here
        for (int32_t k = 0; k < P; k++) {
            if (m->proc_peer[k] < 0) continue;
            const size_t u = (size_t)hvi[m->proc_host[k]], v = (size_t)hvi[m->proc_host[m->proc_peer[k]]];
            if (!(m->path_lat_ms[u * V + v] >= 0.0) || !(m->path_lat_ms[v * V + u] >= 0.0)) return -113;   // EHOSTUNREACH
        }
        // the window: the smallest latency between two different hosts, in ns
        // (ceil, worker.c:293), over the vertex pairs some pair of distinct hosts
        // realizes (a vertex with itself only when two hosts share it)
        for (int32_t u = 0; u < V; u++) {
            if (!per_vertex[u]) continue;
            for (int32_t v = 0; v < V; v++) {
                if (!per_vertex[v] || (u == v && per_vertex[u] < 2)) continue;
                const double l = m->path_lat_ms[(size_t)u * V + v];
                if (l < 0) continue;
                const uint64_t w = (uint64_t)ceil(l * (double)kMs);
                if (w < W) W = w;
            }
        }
    } else {
        // the same from the cache's device tables: either endpoint's row may
        // serve a pair, so both count (the window only bounds the rounds)
        std::vector<int32_t> conn;   // (client vertex, server vertex, same host, route required)
        for (int32_t k = 0; k < P; k++)
            if (m->proc_peer[k] >= 0) {
                const int32_t hc = m->proc_host[k], hs = m->proc_host[m->proc_peer[k]];
                conn.push_back(hvi[hc]); conn.push_back(hvi[hs]); conn.push_back(hc == hs ? 1 : 0); conn.push_back(1);
            }
        std::vector<uint8_t> occ;   // datagrams may go between any two hosts: every pair of their vertices bounds it
        if (any_udp) {
            occ.resize(V);
            for (int32_t u = 0; u < V; u++) occ[u] = (uint8_t)std::min<int32_t>(per_vertex[u], 2);
        }
        const int rr = tcp_pc_prep(pc, conn, occ, &W);
        if (rr) return rr;
    }
    if (W == 0) return -22;
    if (W == ~0ull) W = m->end_time ? m->end_time : 1;
    // test_tcp.c's client takes its server's listening port when it connects
    // (its message queue); the device publishes a port where the server's bind
    // runs, and another lane -- or, on a group, another engine -- sees it from
    // the next round on.  A client on another host that starts within
    // [server start, server start + W) could connect in the server's own round,
    // and what it read would depend on the lanes' timing (one engine) or
    // differ from the one-engine run (a group): such a model is refused, on
    // one engine and on a group alike.  W later the port is always there; a
    // client that starts before its server finds none on every path, as in
    // the serial loop
    for (int32_t k = 0; k < P; k++) {
        const int32_t s = m->proc_peer[k];
        if (s < 0 || m->proc_host[k] == m->proc_host[s]) continue;
        if (m->proc_start[k] >= m->proc_start[s] && m->proc_start[k] - m->proc_start[s] < W) return -22;
    }

    int rc = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kWsDevices) return -5;
    TcpWs& ws = g_ws[dev];
    std::unique_lock<std::mutex> ws_lock(ws.mu);
    const bool ws_keep = g_ws_keep;
    Glob g;
    memset(&g, 0, sizeof(g));
    std::vector<DHost> hh(nloc);
    std::vector<DProc> pp(P > 0 ? P : 1);
    std::vector<int32_t> hp((size_t)nloc * kProcs, -1);
    shd_tcp_result* res = (shd_tcp_result*)calloc(1, sizeof(shd_tcp_result));
    double* d_lat = nullptr; double* d_rel = nullptr;
    uint32_t* d_spec = nullptr; int32_t* d_apeer = nullptr; double* d_cum = nullptr; uint8_t* d_cls = nullptr;
    int32_t* d_hv = nullptr;
    uint64_t* d_ipk = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipStream_t st = nullptr;
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
    TCtl hctl;
    std::vector<uint64_t> ipk;
    uint64_t rounds = 0;
    std::vector<DHost> hout(nloc);
    uint32_t* d_ipall = nullptr; uint64_t* d_bwu = nullptr; uint64_t* d_bwd = nullptr;
    uint32_t* d_sched = nullptr;   // the first-touch schedule (TcpSched), when it has entries
    char* d_xrecv = nullptr; uint64_t* d_pmine = nullptr; uint64_t* d_pall = nullptr; uint32_t* d_xcnt = nullptr;
    char* d_gmine = nullptr; char* d_gall = nullptr;
    constexpr size_t kGatherMax = 1024;   // bytes one rank contributes to a control all-gather (<= 64 engines)
    for (int32_t i = 0; i < nloc; i++) {
        DHost& x = hh[i];
        const int32_t gi = h0 + i;
        memset(&x, 0, sizeof(x));
        x.ip = m->host_ip[gi];
        x.rng = m->host_seed[gi];
        x.bw_down = m->bw_down_kibps[gi];
        x.bw_up = m->bw_up_kibps[gi];
        x.tx_refill = m->bw_up_kibps[gi] * 1024 / 1000;   // _networkinterface_setupTokenBuckets (:192-226)
        x.rx_refill = m->bw_down_kibps[gi] * 1024 / 1000;
        x.tx_cap = x.tx_refill + kMTU;
        x.rx_cap = x.rx_refill + kMTU;
        x.nfree = pool_cap;
        x.next_handle = 3;
    }
    for (int32_t k = 0; k < P; k++) {
        DProc& pr = pp[k];
        memset(&pr, 0, sizeof(pr));
        pr.host = m->proc_host[k]; pr.index = k; pr.peer = m->proc_peer[k]; pr.start = m->proc_start[k];
        pr.fd = pr.listenfd = pr.wait_fd = -1;
        pr.app = app_of(k);
        if (pr.host < h0 || pr.host >= h0 + nloc) continue;   // another engine's
        int32_t* slot = &hp[(size_t)(pr.host - h0) * kProcs];
        int j = 0;
        while (j < kProcs && slot[j] >= 0) j++;
        if (j == kProcs) { free(res); return -22; }
        slot[j] = k;
    }

    {   // host_of_ip's table: at most half full; an address's first host wins (host order)
        uint32_t cap = 64;
        while (cap < 2u * (uint32_t)H) cap <<= 1;
        ipk.assign(cap, ~0ull);
        g.ip_mask = cap - 1;
        for (int32_t i = 0; i < H; i++) {
            const uint32_t ip = m->host_ip[i];
            uint32_t k = ip_slot(ip, g.ip_mask);
            while (ipk[k] != ~0ull && (uint32_t)(ipk[k] >> 32) != ip) k = (k + 1) & g.ip_mask;
            if (ipk[k] == ~0ull) ipk[k] = ((uint64_t)ip << 32) | (uint32_t)i;
        }
    }
    g.H = H; g.P = P; g.W = W;
    g.h0 = h0; g.nloc = nloc; g.world = world; g.me = me;
    g.end_time = m->end_time; g.hb = m->heartbeat_interval ? m->heartbeat_interval : kSec;
    g.tcp_bytes = m->tcp_bytes; g.trace = (trace & SHD_TCP_TRACE_STATUS) ? 1 : 0;
    g.recv_buf = m->recv_buf; g.send_buf = m->send_buf; g.tcp_window = m->tcp_window;
    if (m->qdisc > 1) { free(res); return -22; }
    g.qdisc_rr = m->qdisc;
    g.spk = any_udp ? 2 * kSock : kSock;   // (the qdisc queues hold 2 * kSock sockets)
    if (any_udp) {
        g.udp_payload = m->udp_payload;
        g.n_classes = m->n_classes;
        const size_t ncum = (size_t)(m->host_class && m->n_classes > 1 ? m->n_classes : 1) * (size_t)H;
        HCHECK(ws_alloc(ws, kWsAppSpec, &d_spec, sizeof(uint32_t) * 4 * (size_t)m->n_app_specs));
        HCHECK(hipMemcpy(d_spec, m->app_spec, sizeof(uint32_t) * 4 * (size_t)m->n_app_specs, hipMemcpyHostToDevice));
        g.app_spec = d_spec;
        if (m->app_peer) {
            HCHECK(ws_alloc(ws, kWsAppPeer, &d_apeer, sizeof(int32_t) * (size_t)H));
            HCHECK(hipMemcpy(d_apeer, m->app_peer, sizeof(int32_t) * (size_t)H, hipMemcpyHostToDevice));
            g.app_peer = d_apeer;
        }
        if (m->dest_cum) {
            HCHECK(ws_alloc(ws, kWsDestCum, &d_cum, sizeof(double) * ncum));
            HCHECK(hipMemcpy(d_cum, m->dest_cum, sizeof(double) * ncum, hipMemcpyHostToDevice));
            g.dest_cum = d_cum;
        }
        if (m->host_class && m->n_classes > 1) {
            HCHECK(ws_alloc(ws, kWsHostClass, &d_cls, (size_t)H));
            HCHECK(hipMemcpy(d_cls, m->host_class, (size_t)H, hipMemcpyHostToDevice));
            g.host_class = d_cls;
        }
    }
    if (!pc) {
        HCHECK(ws_alloc(ws, kWsLat, &d_lat, sizeof(double) * (size_t)V * V));
        HCHECK(ws_alloc(ws, kWsRel, &d_rel, sizeof(double) * (size_t)V * V));
        HCHECK(hipMemcpy(d_lat, m->path_lat_ms, sizeof(double) * (size_t)V * V, hipMemcpyHostToDevice));
        HCHECK(hipMemcpy(d_rel, m->path_rel, sizeof(double) * (size_t)V * V, hipMemcpyHostToDevice));
    } else {   // the cache's tables and ranks (copied back at the end)
        g.pcm = 1;
        g.pT = V;
        g.pc_complete = pc->complete ? 1u : 0u;
        g.pc_prefer_direct = pc->prefer_direct ? 1u : 0u;
        g.prow = pc->d_row; g.pself = pc->d_self; g.pdir = pc->d_dir; g.padj = pc->d_adj; g.pself_eid = pc->d_self_eid;
        HCHECK(ws_alloc(ws, kWsRank, &g.rank, sizeof(int32_t) * (size_t)V));
        HCHECK(ws_alloc(ws, kWsSrank, &g.srank, sizeof(int32_t) * (size_t)V));
        HCHECK(ws_alloc(ws, kWsNextRank, &g.next_rank, sizeof(int32_t)));
        HCHECK(hipMemcpy(g.rank, pc->h_rank, sizeof(int32_t) * (size_t)V, hipMemcpyHostToDevice));
        HCHECK(hipMemcpy(g.srank, pc->h_self_rank, sizeof(int32_t) * (size_t)V, hipMemcpyHostToDevice));
        HCHECK(hipMemcpy(g.next_rank, &pc->next_rank, sizeof(int32_t), hipMemcpyHostToDevice));
        g.ft_cap = (uint32_t)H * 4u > (1u << 16) ? (uint32_t)H * 4u : (1u << 16);   // (a group's: every engine's log)
        HCHECK(ws_alloc(ws, kWsFt, &g.ft, sizeof(shd_tcp_query) * (size_t)g.ft_cap));
        HCHECK(ws_alloc(ws, kWsFtord, &g.ftord, sizeof(int32_t) * (size_t)g.ft_cap));
        HCHECK(ws_alloc(ws, kWsNft, &g.nft, sizeof(uint32_t)));
        HCHECK(hipMemset(g.nft, 0, sizeof(uint32_t)));
        if (sch && !sch->round.empty() && world == 1) {
            const size_t nr = sch->round.size(), nv = sch->v.size();
            HCHECK(hipMalloc((void**)&d_sched, sizeof(uint32_t) * (2 * nr + 1) + sizeof(int32_t) * (nv ? nv : 1)));
            HCHECK(hipMemcpy(d_sched, sch->round.data(), sizeof(uint32_t) * nr, hipMemcpyHostToDevice));
            HCHECK(hipMemcpy(d_sched + nr, sch->off.data(), sizeof(uint32_t) * (nr + 1), hipMemcpyHostToDevice));
            if (nv) HCHECK(hipMemcpy(d_sched + 2 * nr + 1, sch->v.data(), sizeof(int32_t) * nv, hipMemcpyHostToDevice));
            g.sched_round = d_sched;
            g.sched_off = d_sched + nr;
            g.sched_v = (const int32_t*)(d_sched + 2 * nr + 1);
            g.sched_n = (uint32_t)nr;
        }
    }
    HCHECK(ws_alloc(ws, kWsIpAll, &d_ipall, sizeof(uint32_t) * (size_t)H));
    HCHECK(hipMemcpy(d_ipall, m->host_ip, sizeof(uint32_t) * (size_t)H, hipMemcpyHostToDevice));
    HCHECK(ws_alloc(ws, kWsBwu, &d_bwu, sizeof(uint64_t) * (size_t)H));
    HCHECK(hipMemcpy(d_bwu, m->bw_up_kibps, sizeof(uint64_t) * (size_t)H, hipMemcpyHostToDevice));
    HCHECK(ws_alloc(ws, kWsBwd, &d_bwd, sizeof(uint64_t) * (size_t)H));
    HCHECK(hipMemcpy(d_bwd, m->bw_down_kibps, sizeof(uint64_t) * (size_t)H, hipMemcpyHostToDevice));
    g.ip_all = d_ipall; g.bwu_all = d_bwu; g.bwd_all = d_bwd;
    HCHECK(ws_alloc(ws, kWsProcPort, &g.proc_port, sizeof(uint32_t) * pp.size()));
    HCHECK(hipMemset(g.proc_port, 0, sizeof(uint32_t) * pp.size()));
    {   // every engine sizes the publications alike: the most processes any engine's hosts run
        std::vector<uint32_t> per(world, 0);
        for (int32_t k = 0; k < P; k++) {
            int32_t r = 0;
            while (r + 1 < world && (int64_t)m->proc_host[k] >= ((int64_t)(r + 1) * H) / world) r++;
            per[r]++;
        }
        g.pcap = 1;
        for (uint32_t v : per) g.pcap = v > g.pcap ? v : g.pcap;
    }
    HCHECK(ws_alloc(ws, kWsPortNew, &g.port_new, sizeof(uint64_t) * (g.pcap + 1)));
    g.nport_new = (uint32_t*)(g.port_new + g.pcap);
    HCHECK(hipMemset(g.port_new, 0, sizeof(uint64_t) * (g.pcap + 1)));
    if (world > 1) {   // the exchange's segments (SHD_TCP_XCAP: deliveries per engine pair and round)
        g.xcap = (uint32_t)std::max<int64_t>(16384, 8 * (int64_t)nloc);
        if (const char* e = getenv("SHD_TCP_XCAP")) {
            const long v = strtol(e, nullptr, 10);
            if (v >= 16 && v <= (1l << 22)) g.xcap = (uint32_t)v;
        }
        g.xsack_cap = g.xcap * kMailSack;
        g.xseg = sizeof(XSegHead) + (size_t)g.xcap * sizeof(Mail) + (size_t)g.xsack_cap * sizeof(int32_t);
        g.xseg = (g.xseg + 255) & ~(size_t)255;
        HCHECK(ws_alloc(ws, kWsXsend, &g.xsend, g.xseg * (size_t)world));
        HCHECK(ws_alloc(ws, kWsXrecv, &d_xrecv, g.xseg * (size_t)world));
        HCHECK(hipMemset(g.xsend, 0, g.xseg * (size_t)world));
        HCHECK(ws_alloc(ws, kWsPmine, &d_pmine, sizeof(uint64_t) * (1 + g.pcap)));
        HCHECK(ws_alloc(ws, kWsPall, &d_pall, sizeof(uint64_t) * (1 + g.pcap) * (size_t)world));
        HCHECK(ws_alloc(ws, kWsXcnt, &d_xcnt, sizeof(uint32_t) * (4 * (size_t)world + 2)));
        HCHECK(ws_alloc(ws, kWsGmine, &d_gmine, kGatherMax));
        HCHECK(ws_alloc(ws, kWsGall, &d_gall, kGatherMax * (size_t)world));
    }
    HCHECK(ws_alloc(ws, kWsHv, &d_hv, sizeof(int32_t) * (size_t)H));
    HCHECK(hipMemcpy(d_hv, hvi.data(), sizeof(int32_t) * (size_t)H, hipMemcpyHostToDevice));
    g.lat = d_lat; g.rel = d_rel; g.hv = d_hv; g.V = V; g.pool_cap = pool_cap;
    HCHECK(ws_alloc(ws, kWsHost, &g.host, sizeof(DHost) * nloc));
    HCHECK(hipMemcpy(g.host, hh.data(), sizeof(DHost) * nloc, hipMemcpyHostToDevice));
    HCHECK(ws_alloc(ws, kWsSock, &g.sock, sizeof(DSock) * (size_t)nloc * g.spk));
    HCHECK(hipMemset(g.sock, 0, sizeof(DSock) * (size_t)nloc * g.spk));
    HCHECK(ws_alloc(ws, kWsProc, &g.proc, sizeof(DProc) * pp.size()));
    HCHECK(hipMemcpy(g.proc, pp.data(), sizeof(DProc) * pp.size(), hipMemcpyHostToDevice));
    HCHECK(ws_alloc(ws, kWsHostProcs, &g.host_procs, sizeof(int32_t) * hp.size()));
    HCHECK(hipMemcpy(g.host_procs, hp.data(), sizeof(int32_t) * hp.size(), hipMemcpyHostToDevice));
    HCHECK(ws_alloc(ws, kWsPool, &g.pool, sizeof(DPkt) * (size_t)nloc * pool_cap));
    HCHECK(ws_alloc(ws, kWsPsack, &g.psack, sizeof(int32_t) * kPktSack * (size_t)nloc * pool_cap));
    HCHECK(ws_alloc(ws, kWsFreel, &g.freel, sizeof(int32_t) * (size_t)nloc * pool_cap));
    k_tcp_free_init<<<(unsigned)(((size_t)nloc * pool_cap + 255) / 256), 256>>>(g.freel, (size_t)nloc * pool_cap, pool_cap);
    HCHECK(hipGetLastError());
    HCHECK(ws_alloc(ws, kWsEv, &g.ev, sizeof(DEv) * (size_t)nloc * kEv));
    HCHECK(ws_alloc(ws, kWsCq, &g.cq, sizeof(CqEnt) * (size_t)nloc * kCq));
    {
        const uint32_t parts = (uint32_t)nloc * 32u > kMailMin ? (uint32_t)nloc * 32u : kMailMin;
        g.mail_part = parts / kMailSub;
        uint32_t ovf = g.mail_part * kMailSub / 2;
        // SHD_TCP_MAIL_PART: smaller parts (the same overflow range), so that a
        // test's model of a few hundred hosts exercises the overflow path
        if (const char* e = getenv("SHD_TCP_MAIL_PART")) {
            const long v = strtol(e, nullptr, 10);
            if (v >= 1 && v < (long)g.mail_part) g.mail_part = (uint32_t)v;
        }
        g.mail_cap = g.mail_part * kMailSub + ovf;
        g.mail_stride = g.mail_cap + (world > 1 ? (uint32_t)world * g.xcap : 0u);
    }
    g.msack_cap = g.mail_cap * kMailSack;
    HCHECK(ws_alloc(ws, kWsMsack, &g.msack, sizeof(int32_t) * 2 * (size_t)g.msack_cap));
    HCHECK(ws_alloc(ws, kWsNmsack, &g.nmsack, sizeof(uint32_t) * 2));
    HCHECK(hipMemset(g.nmsack, 0, sizeof(uint32_t) * 2));
    HCHECK(ws_alloc(ws, kWsMail, &g.mail, sizeof(Mail) * 2 * (size_t)g.mail_stride));
    HCHECK(ws_alloc(ws, kWsNmail, &g.nmail, sizeof(uint32_t) * 2 * (kMailSub + 1)));
    HCHECK(hipMemset(g.nmail, 0, sizeof(uint32_t) * 2 * (kMailSub + 1)));
    HCHECK(ws_alloc(ws, kWsMhead, &g.mhead, sizeof(int32_t) * 2 * (size_t)nloc));
    HCHECK(hipMemset(g.mhead, 0xff, sizeof(int32_t) * 2 * (size_t)nloc));
    HCHECK(ws_alloc(ws, kWsMnext, &g.mnext, sizeof(int32_t) * 2 * (size_t)g.mail_stride));
    HCHECK(ws_alloc(ws, kWsCtl, &g.ctl, sizeof(TCtl)));
    HCHECK(hipMemset(g.ctl, 0, sizeof(TCtl)));
    HCHECK(ws_alloc(ws, kWsIpk, &d_ipk, sizeof(uint64_t) * ipk.size()));
    HCHECK(hipMemcpy(d_ipk, ipk.data(), sizeof(uint64_t) * ipk.size(), hipMemcpyHostToDevice));
    g.ip_key = d_ipk;
    if (trace & SHD_TCP_TRACE_NODE) {   // every heartbeat before the end, per host
        g.node_k = (uint32_t)((m->end_time - 1) / g.hb) + 1;
        if (ws_alloc(ws, kWsNode, &g.node, sizeof(uint64_t) * 2 * kTrk * (size_t)nloc * g.node_k) != hipSuccess) {
            (void)hipGetLastError();
            fprintf(stderr, "shd_tcp_run: no device memory for the tracker counters\n");
            rc = -12;
            goto done;
        }
    }
    if (g.trace) {
        // kTr records and kTrSack SACK words per host (about 16 MB): a traced
        // run of many hosts may not fit; say so instead of a bare -ENOMEM
        const size_t need = (sizeof(TRec) * (size_t)kTr + sizeof(int32_t) * (size_t)kTrSack) * (size_t)nloc;
        if (ws_alloc(ws, kWsTr, &g.tr, sizeof(TRec) * (size_t)nloc * kTr) != hipSuccess ||
            ws_alloc(ws, kWsTrs, &g.trs, sizeof(int32_t) * (size_t)nloc * kTrSack) != hipSuccess) {
            (void)hipGetLastError();
            fprintf(stderr, "shd_tcp_run: no device memory for the status trace of %d hosts (%.1f GB); "
                            "run without trace\n", nloc, need / 1e9);
            rc = -12;
            goto done;
        }
    }
    HCHECK(ws_alloc(ws, kWsNextTime, &g.next_time, sizeof(uint64_t) * (nloc + 1)));
    HCHECK(hipMemset(g.next_time, 0xff, sizeof(uint64_t) * (nloc + 1)));
    // every host can log kPq first queries (touch_log)
    g.qlog_cap = (uint32_t)nloc * kPq > (1u << 16) ? (uint32_t)nloc * kPq : (1u << 16);
    HCHECK(ws_alloc(ws, kWsQlog, &g.qlog, sizeof(shd_tcp_query) * (size_t)g.qlog_cap));
    HCHECK(ws_alloc(ws, kWsNqlog, &g.nqlog, sizeof(uint32_t)));
#ifdef SHD_TCP_PROF
    HCHECK(ws_alloc(ws, kWsProf, &g.prof, sizeof(uint64_t) * 2 * kProf * (size_t)nloc));
    HCHECK(hipMemset(g.prof, 0, sizeof(uint64_t) * 2 * kProf * (size_t)nloc));
    HCHECK(ws_alloc(ws, kWsProfRound, &g.prof_round, sizeof(uint32_t) * 2 * kProfRounds));
    HCHECK(hipMemset(g.prof_round, 0, sizeof(uint32_t) * 2 * kProfRounds));
#endif
    HCHECK(hipMemset(g.nqlog, 0, sizeof(uint32_t)));
    HCHECK(hipEventCreate(&e0));
    HCHECK(hipEventCreate(&e1));
    HCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    // the initialisation above (k_tcp_free_init, the memsets) ran on the null
    // stream, which a non-blocking stream does not wait for: finish it first
    HCHECK(hipDeviceSynchronize());
    res->setup_ms = ms_since(t_call);
    {
        // rounds run in batches of kBatch (window kernel, round kernel) pairs
        // captured once as a graph: no host round trip inside a batch; a
        // halted run turns the batch's remaining kernels into no-ops
        // one host per lane, 64 per wave (16 per wave measured +4 % at 16 k
        // hosts, DESIGN.md §6: not kept)
        const int threads = 64, blocks = (nloc + threads - 1) / threads;
        constexpr int kBatch = 64;
        if (world == 1) {
            HCHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
            for (int i = 0; i < kBatch; i++) {
                k_tcp_window<<<1, 1024, 0, st>>>(g, 0);
                k_tcp_round<<<blocks, threads, 0, st>>>(g);
            }
            HCHECK(hipStreamEndCapture(st, &graph));
            HCHECK(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));
        }
        HCHECK(hipEventRecord(e0, st));
        k_tcp_boot<<<blocks, threads, 0, st>>>(g);
        HCHECK(hipGetLastError());
        for (;;) {
            if (world == 1) {
                HCHECK(hipGraphLaunch(gexec, st));
                HCHECK(hipMemcpyAsync(&hctl, g.ctl, sizeof(TCtl), hipMemcpyDeviceToHost, st));
                HCHECK(hipStreamSynchronize(st));
            } else {
                // a group's round (slave.c:437-462 across engines): the earliest
                // event over the group opens the window; the round's ports and
                // deliveries for the other engines are exchanged after it
                k_tcp_window<<<1, 1024, 0, st>>>(g, 1);
                k_tcp_ports_pack<<<1, 256, 0, st>>>(g, d_pmine);
                HCHECK(hipMemcpyAsync(&hctl, g.ctl, sizeof(TCtl), hipMemcpyDeviceToHost, st));
                HCHECK(hipStreamSynchronize(st));
                struct { uint64_t tmin; uint32_t nport, halted; } mine{hctl.tmin, 0, hctl.halted}, all[64];
                {
                    uint64_t np = 0;
                    HCHECK(hipMemcpy(&np, d_pmine, sizeof(uint64_t), hipMemcpyDeviceToHost));
                    mine.nport = (uint32_t)np;
                }
                static_assert(sizeof(mine) <= 1024, "control word");
                if (group_allgather(comm, d_gmine, d_gall, &mine, all, sizeof(mine), st)) { rc = -5; goto done; }
                uint64_t t = ~0ull;
                uint32_t anyport = 0, halted = 0;
                for (int r = 0; r < world; r++) {
                    t = all[r].tmin < t ? all[r].tmin : t;
                    anyport |= all[r].nport;
                    halted |= all[r].halted;
                }
                if (anyport) {
                    if (shd_comm_allgather_dev(comm, d_pmine, d_pall, sizeof(uint64_t) * (1 + g.pcap), st)) {
                        rc = -5;
                        goto done;
                    }
                    k_tcp_ports<<<world, 256, 0, st>>>(g, d_pall);
                }
                if (halted) t = ~0ull;   // an engine stopped: every engine ends at the same round
                k_tcp_decide<<<1, 64, 0, st>>>(g, t);
                if (t == ~0ull || t >= g.end_time) {
                    HCHECK(hipMemcpyAsync(&hctl, g.ctl, sizeof(TCtl), hipMemcpyDeviceToHost, st));
                    HCHECK(hipStreamSynchronize(st));
                    break;
                }
                k_tcp_round<<<blocks, threads, 0, st>>>(g);
                HCHECK(hipGetLastError());
                {   // the segments' used parts only: the counts first (one all-gather), then an all-to-all-v
                    uint32_t heads[129], allh[64 * 129];
                    const size_t hs = 2 * (size_t)world + 1;   // per engine: its segments' counts, its log entries
                    k_tcp_xheads<<<1, 64, 0, st>>>(g, d_xcnt);
                    HCHECK(hipMemcpyAsync(heads, d_xcnt, sizeof(uint32_t) * hs, hipMemcpyDeviceToHost, st));
                    HCHECK(hipStreamSynchronize(st));
                    if (group_allgather(comm, d_gmine, d_gall, heads, allh, sizeof(uint32_t) * hs, st)) {
                        rc = -5;
                        goto done;
                    }
                    if (g.pcm) {   // the round's first touches: every engine's log replayed alike (k_tcp_window)
                        uint32_t mx = 0, tot = 0;
                        for (int r = 0; r < world; r++) {
                            const uint32_t n = allh[(size_t)r * hs + 2 * world];
                            mx = n > mx ? n : mx;
                            tot += n;
                        }
                        if (mx) {
                            if (mx > g.ft_cap || tot > g.ft_cap) { res->error |= SHD_TCP_ERR_FIRST_TOUCH; break; }
                            std::vector<shd_tcp_query> mine_q(mx), all_q((size_t)mx * world);
                            const uint32_t nme = allh[(size_t)me * hs + 2 * world];
                            if (nme) HCHECK(hipMemcpy(mine_q.data(), g.ft, sizeof(shd_tcp_query) * nme, hipMemcpyDeviceToHost));
                            if (shd_comm_allgather_host(comm, mine_q.data(), sizeof(shd_tcp_query) * mx, all_q.data())) {
                                rc = -5;
                                goto done;
                            }
                            std::vector<shd_tcp_query> uni;
                            uni.reserve(tot);
                            for (int r = 0; r < world; r++)
                                for (uint32_t j = 0; j < allh[(size_t)r * hs + 2 * world]; j++)
                                    uni.push_back(all_q[(size_t)r * mx + j]);
                            HCHECK(hipMemcpy(g.ft, uni.data(), sizeof(shd_tcp_query) * tot, hipMemcpyHostToDevice));
                            HCHECK(hipMemcpy(g.nft, &tot, sizeof(uint32_t), hipMemcpyHostToDevice));
                        }
                    }
                    size_t so[64], sb[64], ro[64], rb[64], so2[64], sb2[64], ro2[64], rb2[64];
                    uint32_t mine_in[128];
                    const size_t sack_at = sizeof(XSegHead) + (size_t)g.xcap * sizeof(Mail);
                    for (int p = 0; p < world; p++) {
                        const bool self = p == me;
                        so[p] = ro[p] = (size_t)p * g.xseg + sizeof(XSegHead);
                        so2[p] = ro2[p] = (size_t)p * g.xseg + sack_at;
                        sb[p] = self ? 0 : (size_t)heads[2 * p] * sizeof(Mail);
                        sb2[p] = self ? 0 : (size_t)heads[2 * p + 1] * sizeof(int32_t);
                        const uint32_t* from = allh + (size_t)p * hs + 2 * me;   // what p sent this engine
                        mine_in[2 * p] = self ? 0 : from[0];
                        mine_in[2 * p + 1] = self ? 0 : from[1];
                        rb[p] = (size_t)mine_in[2 * p] * sizeof(Mail);
                        rb2[p] = (size_t)mine_in[2 * p + 1] * sizeof(int32_t);
                    }
                    if (shd_comm_alltoallv_dev(comm, g.xsend, so, sb, d_xrecv, ro, rb, st) ||
                        shd_comm_alltoallv_dev(comm, g.xsend, so2, sb2, d_xrecv, ro2, rb2, st)) {
                        rc = -5;
                        goto done;
                    }
                    // (blocking: the counts leave this stack frame; the last round's ingest has finished)
                    HCHECK(hipMemcpy(d_xcnt + hs, mine_in, sizeof(uint32_t) * 2 * world, hipMemcpyHostToDevice));
                    k_tcp_xingest<<<world, 256, 0, st>>>(g, d_xrecv, d_xcnt + hs);
                }
                HCHECK(hipGetLastError());
                HCHECK(hipMemcpyAsync(&hctl, g.ctl, sizeof(TCtl), hipMemcpyDeviceToHost, st));
                HCHECK(hipStreamSynchronize(st));
            }
            if (hctl.halted) break;
            if (hctl.rounds > (1ull << 26)) { res->error |= SHD_TCP_ERR_INTERNAL; break; }
        }
        rounds = hctl.rounds;
        HCHECK(hipEventRecord(e1, st));
        HCHECK(hipEventSynchronize(e1));
        float ms = 0;
        HCHECK(hipEventElapsedTime(&ms, e0, e1));
        res->device_ms = ms;
    }
    t_results = std::chrono::steady_clock::now();
    HCHECK(hipMemcpy(hout.data(), g.host, sizeof(DHost) * nloc, hipMemcpyDeviceToHost));
    {   // the first-query log (a group's: every engine's, so that each ranks the run's first touches alike)
        uint32_t nq = 0;
        HCHECK(hipMemcpy(&nq, g.nqlog, sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (nq > g.qlog_cap) nq = g.qlog_cap;   // (the run's error bits say so)
        std::vector<shd_tcp_query> mine(nq ? nq : 1);
        if (nq) HCHECK(hipMemcpy(mine.data(), g.qlog, sizeof(shd_tcp_query) * nq, hipMemcpyDeviceToHost));
        if (world == 1) {
            res->queries = (shd_tcp_query*)malloc(sizeof(shd_tcp_query) * (nq ? nq : 1));
            memcpy(res->queries, mine.data(), sizeof(shd_tcp_query) * (nq ? nq : 1));
            res->n_queries = nq;
        } else {
            std::vector<uint32_t> counts(world);
            if (shd_comm_allgather_host(comm, &nq, sizeof(nq), counts.data())) { rc = -5; goto done; }
            uint32_t mx = 1, tot = 0;
            for (uint32_t c : counts) { mx = c > mx ? c : mx; tot += c; }
            mine.resize(mx);
            std::vector<shd_tcp_query> all((size_t)mx * world);
            if (shd_comm_allgather_host(comm, mine.data(), sizeof(shd_tcp_query) * mx, all.data())) { rc = -5; goto done; }
            res->queries = (shd_tcp_query*)malloc(sizeof(shd_tcp_query) * (tot ? tot : 1));
            res->n_queries = tot;
            size_t o = 0;
            for (int r = 0; r < world; r++)
                for (uint32_t j = 0; j < counts[r]; j++) res->queries[o++] = all[(size_t)r * mx + j];
        }
    }
    res->first_host = h0;
    res->n_local_hosts = nloc;
    res->next_event_id = (uint64_t*)calloc(nloc, sizeof(uint64_t));
    res->next_packet_id = (uint64_t*)calloc(nloc, sizeof(uint64_t));
    res->rng_probe = (uint32_t*)calloc(nloc, sizeof(uint32_t));
    res->rounds = rounds;
    {   // the last two rounds' mailboxes were never counted by k_tcp_window
        std::vector<uint32_t> nm(2 * (kMailSub + 1));
        HCHECK(hipMemcpy(nm.data(), g.nmail, sizeof(uint32_t) * nm.size(), hipMemcpyDeviceToHost));
        TCtl cx;
        HCHECK(hipMemcpy(&cx, g.ctl, sizeof(TCtl), hipMemcpyDeviceToHost));
        res->max_round_deliveries = cx.max_mail;
        res->max_round_overflow = cx.max_ovf;
        if (cx.ft_bad) res->error |= SHD_TCP_ERR_FIRST_TOUCH;
        if (cx.ft_bad && sch && pc && world == 1 && sch->round.size() < kFtReruns) {
            // the contradicted round's first touches in serial order: the
            // ranks its replay assigned, [ft_nr0, next_rank)
            std::vector<int32_t> rk(V), sk(V);
            int32_t nr1 = 0;
            HCHECK(hipMemcpy(rk.data(), g.rank, sizeof(int32_t) * (size_t)V, hipMemcpyDeviceToHost));
            HCHECK(hipMemcpy(sk.data(), g.srank, sizeof(int32_t) * (size_t)V, hipMemcpyDeviceToHost));
            HCHECK(hipMemcpy(&nr1, g.next_rank, sizeof(int32_t), hipMemcpyDeviceToHost));
            const int32_t nr0 = (int32_t)cx.ft_nr0;
            std::vector<int32_t> ord(nr1 > nr0 ? nr1 - nr0 : 0, INT32_MIN);
            for (int32_t v = 0; v < V; v++) {
                if (rk[v] != kNoRank && rk[v] >= nr0 && rk[v] < nr1) ord[rk[v] - nr0] = v;
                if (sk[v] != kNoRank && sk[v] >= nr0 && sk[v] < nr1) ord[sk[v] - nr0] = ~v;
            }
            bool ok = !ord.empty();
            for (int32_t x : ord) ok &= x != INT32_MIN;
            if (ok) {
                sch->round.push_back((uint32_t)cx.rounds);
                sch->v.insert(sch->v.end(), ord.begin(), ord.end());
                sch->off.push_back((uint32_t)sch->v.size());
                sch->extended = true;
            }
        }
        res->error |= cx.xerr;
        if (pc && !cx.ft_bad) {   // the cache's ranks as the serial run leaves them
            std::vector<int32_t> old_rank(pc->h_rank, pc->h_rank + V), old_self(pc->h_self_rank, pc->h_self_rank + V);
            HCHECK(hipMemcpy(pc->h_rank, g.rank, sizeof(int32_t) * (size_t)V, hipMemcpyDeviceToHost));
            HCHECK(hipMemcpy(pc->h_self_rank, g.srank, sizeof(int32_t) * (size_t)V, hipMemcpyDeviceToHost));
            HCHECK(hipMemcpy(&pc->next_rank, g.next_rank, sizeof(int32_t), hipMemcpyDeviceToHost));
            // and minimumPathLatency with the entries those rows stored
            if (const int fr = shd_pc_fold_ranked(pc, old_rank.data(), old_self.data())) { rc = fr; goto done; }
        }
        for (int b = 0; b < 2; b++) {
            uint64_t sum = 0;
            for (uint32_t j = 0; j <= kMailSub; j++) {
                const uint32_t cap = j < kMailSub ? g.mail_part : g.mail_cap - g.mail_part * kMailSub;
                const uint32_t v = nm[b * (kMailSub + 1) + j];
                sum += v < cap ? v : cap;
                if (j == kMailSub && (v < cap ? v : cap) > res->max_round_overflow) res->max_round_overflow = v < cap ? v : cap;
            }
            if (sum > res->max_round_deliveries) res->max_round_deliveries = sum;
        }
    }
    for (int32_t i = 0; i < nloc; i++) {
        res->next_event_id[i] = hout[i].ev_seq;
        res->next_packet_id[i] = hout[i].pkt_seq;
        uint32_t st = hout[i].rng;
        res->rng_probe[i] = (uint32_t)rand_r_host(&st);
        res->events += hout[i].events;
        res->deliveries += hout[i].deliveries;
        res->error |= hout[i].err;
    }
    if (g.node) {
        res->node_k = g.node_k;
        res->n_heartbeats = (uint32_t*)calloc(nloc, sizeof(uint32_t));
        res->node_counters = (uint64_t*)malloc(sizeof(uint64_t) * 2 * kTrk * (size_t)nloc * g.node_k);
        HCHECK(hipMemcpy(res->node_counters, g.node, sizeof(uint64_t) * 2 * kTrk * (size_t)nloc * g.node_k,
                         hipMemcpyDeviceToHost));
        for (int32_t i = 0; i < nloc; i++) res->n_heartbeats[i] = hout[i].nhb < g.node_k ? hout[i].nhb : g.node_k;
    }
    if (g.trace) {
        std::string text;
        std::vector<TRec> recs;
        std::vector<int32_t> sk;
        for (int32_t i = 0; i < nloc; i++) {
            recs.resize(hout[i].ntr);
            sk.resize(hout[i].ntrs + 1);
            if (hout[i].ntr)
                HCHECK(hipMemcpy(recs.data(), g.tr + (size_t)i * kTr, sizeof(TRec) * hout[i].ntr, hipMemcpyDeviceToHost));
            if (hout[i].ntrs)
                HCHECK(hipMemcpy(sk.data(), g.trs + (size_t)i * kTrSack, sizeof(int32_t) * hout[i].ntrs, hipMemcpyDeviceToHost));
            for (const TRec& r : recs) format_line(text, r, sk.data() + r.sack_off, h0 + i);
            res->n_lines += hout[i].ntr;
        }
        res->lines = (char*)malloc(text.size() + 1);
        memcpy(res->lines, text.data(), text.size());
        res->lines[text.size()] = 0;
        res->len = text.size();
    }
#ifdef SHD_TCP_PROF
    {   // the steps' cycles summed over hosts, and per round the busiest lane
        std::vector<uint64_t> pf(2 * kProf * (size_t)nloc);
        std::vector<uint32_t> pr(2 * kProfRounds);
        HCHECK(hipMemcpy(pf.data(), g.prof, sizeof(uint64_t) * pf.size(), hipMemcpyDeviceToHost));
        HCHECK(hipMemcpy(pr.data(), g.prof_round, sizeof(uint32_t) * pr.size(), hipMemcpyDeviceToHost));
        static const char* kName[kProf] = {"ingest", "evq_pop", "HEARTBEAT", "REFILL", "REFILL_LO", "PSTART",
                                           "NOTIFY", "DELIVER", "DELACK", "RTO", "CLOSE", "WINUPD", "LOCAL",
                                           "-", "lane_round", "max_ev", "-", "-", "-", "-"};
        fprintf(stderr, "tcp_prof: step cycles_total count cycles_per\n");
        for (uint32_t j = 0; j < kProf; j++) {
            uint64_t cy = 0, n = 0;
            for (int32_t i = 0; i < nloc; i++) {
                const uint64_t* q = pf.data() + (size_t)i * 2 * kProf;
                if (j == 15) { cy = std::max(cy, q[j]); continue; }
                cy += q[j]; n += q[kProf + j];
            }
            if (cy || n) fprintf(stderr, "tcp_prof: %s %llu %llu %.1f\n", kName[j], (unsigned long long)cy,
                                 (unsigned long long)n, n ? (double)cy / (double)n : 0.0);
        }
        const uint64_t nr = std::min<uint64_t>(hctl.rounds, kProfRounds);
        for (uint64_t r = 0; r < nr; r++)
            fprintf(stderr, "tcp_round: %llu max_ev %u max_kcyc %u\n", (unsigned long long)r, pr[r], pr[kProfRounds + r]);
    }
#endif
    res->results_ms = ms_since(t_results);
done:
    const auto t_free = std::chrono::steady_clock::now();
    if (d_sched) (void)hipFree(d_sched);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (gexec) (void)hipGraphExecDestroy(gexec);
    if (graph) (void)hipGraphDestroy(graph);
    if (st) (void)hipStreamDestroy(st);
    if (!ws_keep || rc) ws_free_all(ws);   // a failed run leaves no workspace behind
    ws_lock.unlock();
    if (rc) { shd_tcp_result_free(res); return rc; }
    res->teardown_ms = ms_since(t_free);
    *out = res;
    return 0;
}

extern "C" int shd_tcp_run(const shd_tcp_model* m, int32_t trace, shd_tcp_result** out) {
    // path_cache mode: a contradicted round makes the next run rank that
    // round's first touches before it runs (TcpSched); every round before it
    // runs again the same, so the reruns cost the rounds up to each
    // contradiction.  Past kFtReruns the contradiction stands
    // (SHD_TCP_ERR_FIRST_TOUCH: the caller's tables)
    TcpSched sch;
    for (uint32_t k = 0;; k++) {
        sch.extended = false;
        const int rc = tcp_run_impl(m, nullptr, trace, out, &sch);
        if (rc || !sch.extended) {
            if (!rc && *out) (*out)->first_touch_reruns = k;
            return rc;
        }
        shd_tcp_result_free(*out);
        *out = nullptr;
    }
}

extern "C" int shd_tcp_run_group(const shd_tcp_model* m, shd_comm* comm, int32_t trace, shd_tcp_result** out) {
    if (!comm) return -22;
    if (hipSetDevice(comm->device) != hipSuccess) return -5;
    return tcp_run_impl(m, comm, trace, out);
}

extern "C" void shd_tcp_result_free(shd_tcp_result* r) {
    if (!r) return;
    free(r->lines);
    free(r->next_event_id);
    free(r->next_packet_id);
    free(r->rng_probe);
    free(r->queries);
    free(r->node_counters);
    free(r->n_heartbeats);
    free(r);
}
