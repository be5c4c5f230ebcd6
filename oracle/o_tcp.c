/*
 * o_tcp.c -- TEST INFRASTRUCTURE (oracle).  A CPU restatement of the
 * reference's TCP path, run on the serial event loop (--workers 0) with the
 * echo application of src/test/tcp/test_tcp.c (nonblocking-epoll mode).  It
 * writes the [STATUS] lines of packet_addDeliveryStatus (packet.c:647-659)
 * so a run can be compared line for line with the reference's own loop
 * (oracle/ref_harness/ref_loop.c, app 1).  Nothing here is shipped: the
 * engine never links it.
 *
 *   connection state machine   host/descriptor/tcp.c:607-698, 1777-2099
 *   segments, windows, flush   tcp.c:729-852, 1090-1278
 *   retransmission, RTO        tcp.c:854-1065, 1280-1333 (RFC 6298)
 *   SACK / lost ranges         tcp_retransmit_tally.cc (all of it)
 *   Reno                       tcp_cong_reno.c (all of it)
 *   buffer autotuning          tcp.c:363-591
 *   user send / receive        tcp.c:2126-2327, host.c:1466-1604
 *   connect / listen / accept  tcp.c:1462-1558, host.c:1111-1358
 *   close / shutdown           tcp.c:2363-2437
 *   socket buffers             host/descriptor/socket.c:284-455
 *   interface FIFO qdisc       host/network_interface.c:87-91, 375-605
 *   worker_sendPacket          core/worker.c:260-321 (copy per delivery)
 *   router + CoDel             routing/router.c:104-140, o_codel.c
 *   epoll notification         host/descriptor/epoll.c:252-395, 411-615, 638-683
 *   priority queue             utility/priority_queue.c (binary heap)
 *   packet strings             routing/packet.c:518-641
 *
 * Scope: one TCP socket per client process, a listener and its children per
 * server process, IPv4 over each host's default interface (no loopback
 * traffic), the default FIFO qdisc, CPU delay off.  Descriptor reference
 * counts are not restated: sockets are never freed, so packets left in a
 * closed socket's buffers never print PDS_DESTROYED (the echo model leaves
 * none).  The retransmit queue's full clear (_tcp_clearRetransmit with -1)
 * walks sequence order, not GHashTable order.
 */
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define MS 1000000ull
#define SEC 1000000000ull
#define MTU 1500u
#define HDR_TCP 66u
#define HDR_UDP 42u          /* CONFIG_HEADER_SIZE_UDPIPETH (definitions.h:176) */
#define UDP_PORT 8998        /* the datagram applications' port (test_phold.c's) */
#define MSS (MTU - HDR_TCP)

/* ProtocolTCPFlags (protocol.h:23-31) */
enum { F_RST = 1 << 1, F_SYN = 1 << 2, F_ACK = 1 << 3, F_SACK = 1 << 4, F_FIN = 1 << 5, F_DUPACK = 1 << 6 };
/* PacketDeliveryStatusFlags, in packet.c:491-516's names */
enum {
    S_SND_CREATED, S_SND_TCP_ENQUEUE_THROTTLED, S_SND_TCP_ENQUEUE_RETRANSMIT, S_SND_TCP_DEQUEUE_RETRANSMIT,
    S_SND_TCP_RETRANSMITTED, S_SND_SOCKET_BUFFERED, S_SND_INTERFACE_SENT, S_INET_SENT, S_INET_DROPPED,
    S_ROUTER_ENQUEUED, S_ROUTER_DEQUEUED, S_ROUTER_DROPPED, S_RCV_INTERFACE_RECEIVED, S_RCV_INTERFACE_DROPPED,
    S_RCV_SOCKET_PROCESSED, S_RCV_SOCKET_DROPPED, S_RCV_TCP_ENQUEUE_UNORDERED, S_RCV_SOCKET_BUFFERED,
    S_RCV_SOCKET_DELIVERED, S_DESTROYED
};
static const char* const k_status_name[] = {
    "SND_CREATED", "SND_TCP_ENQUEUE_THROTTLED", "SND_TCP_ENQUEUE_RETRANSMIT", "SND_TCP_DEQUEUE_RETRANSMIT",
    "SND_TCP_RETRANSMITTED", "SND_SOCKET_BUFFERED", "SND_INTERFACE_SENT", "INET_SENT", "INET_DROPPED",
    "ROUTER_ENQUEUED", "ROUTER_DEQUEUED", "ROUTER_DROPPED", "RCV_INTERFACE_RECEIVED", "RCV_INTERFACE_DROPPED",
    "RCV_SOCKET_PROCESSED", "RCV_SOCKET_DROPPED", "RCV_TCP_ENQUEUE_UNORDERED", "RCV_SOCKET_BUFFERED",
    "RCV_SOCKET_DELIVERED", "PDS_DESTROYED"
};
/* DescriptorStatus (descriptor_types.h) */
enum { DS_ACTIVE = 1 << 0, DS_READABLE = 1 << 1, DS_WRITABLE = 1 << 2, DS_CLOSED = 1 << 3 };
/* TCPState / flags / errors / process flags (tcp.c:42-89) */
enum { TS_CLOSED, TS_LISTEN, TS_SYNSENT, TS_SYNRECEIVED, TS_ESTABLISHED, TS_FINWAIT1, TS_FINWAIT2, TS_CLOSING,
       TS_TIMEWAIT, TS_CLOSEWAIT, TS_LASTACK };
enum { TF_LOCAL_CLOSED_RD = 1 << 0, TF_LOCAL_CLOSED_WR = 1 << 1, TF_REMOTE_CLOSED = 1 << 2,
       TF_EOF_RD_SIGNALED = 1 << 3, TF_EOF_WR_SIGNALED = 1 << 4, TF_RESET_SIGNALED = 1 << 5,
       TF_WAS_ESTABLISHED = 1 << 6, TF_CONNECT_SIGNALED = 1 << 7, TF_SHOULD_SEND_WR_FIN = 1 << 8 };
enum { TE_CONNECTION_RESET = 1 << 0, TE_SEND_EOF = 1 << 1, TE_RECEIVE_EOF = 1 << 2 };
enum { PF_PROCESSED = 1 << 0, PF_DATA_RECEIVED = 1 << 1, PF_DATA_ACKED = 1 << 2, PF_DATA_SACKED = 1 << 3,
       PF_DATA_LOST = 1 << 4, PF_RWND_UPDATED = 1 << 5 };
enum { ERR_EWOULDBLOCK = 11, ERR_EINPROGRESS = 115, ERR_EALREADY = 114, ERR_EISCONN = 106, ERR_ENOTCONN = 107,
       ERR_EPIPE = 32, ERR_ECONNRESET = 104, ERR_ECONNREFUSED = 111 };

/* ------------------------------------------------------------ packets */
typedef struct opkt {
    uint32_t host_id;            /* packet_new's hostID (host_getID: index + 1) */
    uint64_t pid;
    int refs;
    uint32_t flags, sip, dip;    /* IPs in host byte order */
    uint16_t sport, dport;       /* host byte order */
    uint32_t seq, ack, win;
    uint64_t tsval, tsecho;
    int32_t* sacks; uint32_t nsack;
    uint32_t len;
    double prio;
    uint8_t st[128]; uint32_t nst;
    int32_t owner;               /* host whose active events print its lines (-2: none) */
    int udp;                     /* a datagram (PUDP) */
} opkt;
static uint32_t hdr_of(const opkt* p) { return p->udp ? HDR_UDP : HDR_TCP; }   /* packet.c:318-323 */

typedef struct { char* s; size_t len, cap; uint64_t n; } obuf;
static void ob_put(obuf* b, const char* s, size_t n) {
    if (b->len + n + 1 > b->cap) {
        size_t nc = b->cap ? b->cap : (1u << 20);
        while (b->len + n + 1 > nc) nc *= 2;
        b->s = realloc(b->s, nc);
        b->cap = nc;
    }
    memcpy(b->s + b->len, s, n);
    b->len += n;
    b->s[b->len] = 0;
}
static void ob_printf(obuf* b, const char* fmt, ...) {
    char tmp[8192];
    va_list ap;
    va_start(ap, fmt);
    int n = vsnprintf(tmp, sizeof(tmp), fmt, ap);
    va_end(ap);
    if (n > 0) ob_put(b, tmp, (size_t)(n < (int)sizeof(tmp) ? n : (int)sizeof(tmp) - 1));
}

/* ------------------------------------------------------------ binary heap
 * (utility/priority_queue.c): push re-heapifies an element already present,
 * pop swaps the last element to the root and sifts it down */
typedef int (*pq_cmp)(const void* a, const void* b);
typedef struct { void** a; uint32_t n, cap; pq_cmp cmp; } opq;
static int pq_smaller(opq* q, uint32_t i, uint32_t j) { return q->cmp(q->a[i], q->a[j]) < 0; }
static void pq_swap(opq* q, uint32_t i, uint32_t j) { void* t = q->a[i]; q->a[i] = q->a[j]; q->a[j] = t; }
static uint32_t pq_up(opq* q, uint32_t i) {
    while (i > 0 && pq_smaller(q, i, (i - 1) / 2)) { pq_swap(q, i, (i - 1) / 2); i = (i - 1) / 2; }
    return i;
}
static uint32_t pq_down(opq* q, uint32_t i) {
    uint32_t c;
    while ((c = 2 * i + 1) < q->n) {
        if (c + 1 < q->n && pq_smaller(q, c + 1, c)) c = c + 1;
        if (pq_smaller(q, c, i)) { pq_swap(q, i, c); i = c; } else break;
    }
    return i;
}
static int pq_index(opq* q, const void* x) {
    for (uint32_t i = 0; i < q->n; i++) if (q->a[i] == x) return (int)i;
    return -1;
}
static int pq_push(opq* q, void* x) {
    int old = pq_index(q, x);
    if (old >= 0) { pq_up(q, pq_down(q, (uint32_t)old)); return 0; }
    if (q->n == q->cap) { q->cap = q->cap ? 2 * q->cap : 16; q->a = realloc(q->a, q->cap * sizeof(void*)); }
    q->a[q->n] = x;
    q->n++;
    pq_up(q, q->n - 1);
    return 1;
}
static void* pq_peek(opq* q) { return q->n ? q->a[0] : NULL; }
static void* pq_pop(opq* q) {
    if (!q->n) return NULL;
    void* x = q->a[0];
    pq_swap(q, 0, q->n - 1);
    q->n--;
    pq_down(q, 0);
    return x;
}
/* packet_compareTCPSequence (packet.c:207-221) */
static int cmp_seq(const void* a, const void* b) {
    const uint32_t x = ((const opkt*)a)->seq, y = ((const opkt*)b)->seq;
    return x < y ? -1 : x > y ? 1 : 0;
}
/* utility_simulationTimeCompare */
static int cmp_time(const void* a, const void* b) {
    const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y ? 1 : 0;
}

/* ------------------------------------------------------------ retransmit tally
 * (tcp_retransmit_tally.cc): sorted half-open ranges of int64 */
typedef struct { int64_t a, b; } rng_t;
typedef struct { rng_t* r; uint32_t n, cap; } rvec;
static void rv_push(rvec* v, int64_t a, int64_t b) {
    if (v->n == v->cap) { v->cap = v->cap ? 2 * v->cap : 8; v->r = realloc(v->r, v->cap * sizeof(rng_t)); }
    v->r[v->n].a = a; v->r[v->n].b = b; v->n++;
}
static void rv_insert_at(rvec* v, uint32_t at, int64_t a, int64_t b) {
    rv_push(v, 0, 0);
    memmove(&v->r[at + 1], &v->r[at], (v->n - 1 - at) * sizeof(rng_t));
    v->r[at].a = a; v->r[at].b = b;
}
static int r_overlap(rng_t x, rng_t y) { return x.a < y.b && y.a < x.b; }
static int r_adj(rng_t x, rng_t y) { return x.b == y.a || y.b == x.a; }
/* ranges_insert (cc:85-102) with ranges_mergable (cc:57-78) */
static void ranges_insert(rvec* v, int64_t a, int64_t b) {
    const rng_t val = {a, b};
    uint32_t first = v->n, it = 0;
    for (; it < v->n && val.b >= v->r[it].a; ++it)
        if (first == v->n && (r_overlap(v->r[it], val) || r_adj(v->r[it], val))) first = it;
    const uint32_t second = it;
    if (first == v->n) {
        rv_insert_at(v, second, a, b);
    } else {
        rng_t* x = &v->r[first];
        if (val.a < x->a) x->a = val.a;
        if (val.b > x->b) x->b = val.b;
        for (uint32_t j = first + 1; j < second; j++) {
            if (v->r[j].a < x->a) x->a = v->r[j].a;
            if (v->r[j].b > x->b) x->b = v->r[j].b;
        }
        const uint32_t nerase = second - (first + 1);
        memmove(&v->r[first + 1], &v->r[second], (v->n - second) * sizeof(rng_t));
        v->n -= nerase;
    }
}
/* ranges_subtract (cc:104-175) */
static void ranges_subtract(const rvec* lhs, const rvec* rhs, rvec* out) {
    out->n = 0;
    if (rhs->n == 0) {
        for (uint32_t i = 0; i < lhs->n; i++) rv_push(out, lhs->r[i].a, lhs->r[i].b);
        return;
    }
    if (lhs->n == 0) return;
    uint32_t idx = 0, j = 0;
    rng_t cur = lhs->r[0];
    while (idx < lhs->n && j < rhs->n) {
        const rng_t rj = rhs->r[j];
        if (rj.b <= cur.a) {
            ++j;
        } else if (cur.b <= rj.a) {
            rv_push(out, cur.a, cur.b);
            ++idx;
            if (idx < lhs->n) cur = lhs->r[idx];
        } else {
            rng_t sub[2]; int ns = 0;
            if (r_overlap(cur, rj)) {
                if (cur.a < rj.a) { sub[ns].a = cur.a; sub[ns].b = rj.a; ns++; }
                if (rj.b < cur.b) { sub[ns].a = rj.b; sub[ns].b = cur.b; ns++; }
            } else {
                sub[ns++] = cur;
            }
            if (ns == 2) rv_push(out, sub[0].a, sub[0].b);
            if (ns >= 1) cur = sub[ns - 1];
            else { ++idx; if (idx < lhs->n) cur = lhs->r[idx]; }
        }
    }
    if (j == rhs->n) {
        rv_push(out, cur.a, cur.b);
        ++idx;
        while (idx < lhs->n) { rv_push(out, lhs->r[idx].a, lhs->r[idx].b); idx++; }
    }
}
typedef struct { int64_t last_ack; uint64_t ndup; rvec marked, sacked, retx, lost, tmp; } tally_t;
static void tally_compute_lost(tally_t* t) {   /* cc:311-314 */
    ranges_subtract(&t->marked, &t->sacked, &t->tmp);
    ranges_subtract(&t->tmp, &t->retx, &t->lost);
}
static void tally_tidy(tally_t* t, rvec* v) {   /* cc:316-335 */
    if (v->n > 0 && t->last_ack >= v->r[0].a && t->last_ack < v->r[0].b - 1) {
        v->r[0].a = t->last_ack;
    } else if (v->n > 0 && t->last_ack >= v->r[0].b - 1) {
        uint32_t k = 0;
        for (uint32_t i = 0; i < v->n; i++) if (!(t->last_ack >= v->r[i].b)) v->r[k++] = v->r[i];
        v->n = k;
    }
}
static uint32_t tally_update(tally_t* t, uint32_t last_ack, int is_dup) {   /* cc:192-220 */
    uint32_t ret = 0;
    if (is_dup && (int64_t)last_ack == t->last_ack) {
        ++t->ndup;
    } else if ((int64_t)last_ack > t->last_ack) {
        t->last_ack = last_ack;
        t->ndup = 0;
        tally_tidy(t, &t->marked);
        tally_tidy(t, &t->sacked);
        tally_tidy(t, &t->retx);
    }
    int contains = 0;
    for (uint32_t i = 0; i < t->retx.n; i++)
        if (t->last_ack >= t->retx.r[i].a && t->last_ack < t->retx.r[i].b) contains = 1;
    if (t->ndup >= 3 && !contains) {
        ranges_insert(&t->marked, t->last_ack, t->last_ack + 1);
        tally_compute_lost(t);
        if (t->lost.n > 0) ret |= PF_DATA_LOST;
    }
    return ret;
}
static void tally_mark_sacked(tally_t* t, const int32_t* s, uint32_t n) {   /* cc:224-245 */
    int64_t first = -1;
    for (uint32_t i = 0; i < n; i++) {
        if (first == -1) first = s[i];
        if (i + 1 == n || s[i + 1] != s[i] + 1) {
            ranges_insert(&t->sacked, first, (int64_t)s[i] + 1);
            first = -1;
        }
    }
}
static void tally_mark_lost(tally_t* t, uint32_t begin, uint32_t end) {   /* cc:247-255 */
    if (begin == end + 1) return;
    if (begin == end) end += 1;
    ranges_insert(&t->marked, begin, end);
    tally_compute_lost(t);
}
static void tally_mark_retransmitted(tally_t* t, uint32_t begin, uint32_t end) {   /* cc:257-263 */
    ranges_insert(&t->retx, begin, end);
    tally_compute_lost(t);
}

/* ------------------------------------------------------------ model state */
typedef struct { int32_t* v; uint32_t n, cap; } ivec;
static void iv_push(ivec* v, int32_t x) {
    if (v->n == v->cap) { v->cap = v->cap ? 2 * v->cap : 16; v->v = realloc(v->v, v->cap * sizeof(int32_t)); }
    v->v[v->n++] = x;
}
typedef struct { opkt** p; uint32_t head, n, cap; } pqueue;   /* GQueue of packets */
static void fq_push(pqueue* q, opkt* p) {
    if (q->n == q->cap) {
        uint32_t nc = q->cap ? 2 * q->cap : 16;
        opkt** a = malloc(nc * sizeof(opkt*));
        for (uint32_t i = 0; i < q->n; i++) a[i] = q->p[(q->head + i) % q->cap];
        free(q->p); q->p = a; q->cap = nc; q->head = 0;
    }
    q->p[(q->head + q->n) % q->cap] = p;
    q->n++;
}
static opkt* fq_peek(pqueue* q) { return q->n ? q->p[q->head] : NULL; }
static opkt* fq_pop(pqueue* q) {
    if (!q->n) return NULL;
    opkt* p = q->p[q->head];
    q->head = (q->head + 1) % q->cap;
    q->n--;
    return p;
}

typedef struct osock {
    int32_t host, handle, proc;          /* proc: the process whose epoll watches it (-1) */
    int udp, used;                       /* a datagram socket (udp.c); used: not released */
    uint32_t status;
    int bound; uint32_t bound_ip; uint16_t bound_port;
    uint32_t peer_ip; uint16_t peer_port;
    pqueue in, out, outctl;
    uint64_t in_len, in_size, in_pending, out_len, out_size, out_pending;
    int assoc;                           /* associated with the host's interfaces */
    int assoc_general;                   /* INADDR_ANY / listener key (peer 0:0) */
    /* tcp.c:117-243 */
    int state, state_last;
    uint32_t flags, error;
    struct { int state; uint32_t start, next, window, end, recovery; uint64_t last_ts;
             uint32_t last_window, last_ack, last_seq; int winupd_pending; } rcv;
    struct { uint32_t unacked, next, window, end, last_ack, last_window, highest, packets_sent, quick_acks;
             int delack_sched; uint32_t delack_counter; ivec sacks; } snd;
    struct { opkt** q; uint32_t nq, capq; uint64_t qlen; int timeout; opq timers;
             uint64_t desired; uint32_t backoff; tally_t tally; } rtx;
    struct { int enabled, did_init; uint64_t bytes_copied, last_adjust, space; } at;
    uint32_t cwnd;
    struct { int state; uint64_t ndup; uint32_t ca_nacked, ssthresh; } reno;   /* 0 SS, 1 FR, 2 CA */
    struct { int srtt, rttvar; } timing;
    struct { uint64_t last_data_sent, last_ack_sent, last_data_recv, last_ack_recv, retx_count; uint32_t rtt; } info;
    opq throttled; uint64_t throttled_len;
    opq unordered; uint64_t unordered_len;
    opkt* partial; uint32_t partial_off;
    /* server / child (tcp.c:91-113) */
    int server; ivec children; ivec pending; uint32_t last_peer_ip, last_ip; uint16_t last_peer_port;
    int child; int32_t parent; int child_state;
} osock;

typedef struct oproc {
    int32_t host, index, peer;           /* peer: -1 server, else the server process */
    uint64_t start;
    int running, step;
    int32_t fd, listenfd, wait_fd;       /* socket indices */
    uint32_t wait_events, done;
    /* the process's epoll (epoll.c): one watch at a time */
    int ep_ready, ep_readable, ep_scheduled, ep_notifying;
    int32_t app;                         /* >= 0: the datagram application cfg->app_spec[4 * app ..] */
} oproc;

typedef struct ohost_t {
    uint32_t ip, rng, pkt_seq;
    uint64_t ev_seq;
    double prio;
    int32_t vertex;
    uint64_t rx_rem, rx_cap, rx_refill, tx_rem, tx_cap, tx_refill;
    int refill_pending;
    opq fifo;                            /* sockets wanting to send (network_interface.c:87-91) */
    osock** rr; uint32_t rr_head, rr_n, rr_cap;   /* the same for the RR qdisc: a FIFO of sockets (rrQueue) */
    o_codel codel;
    int32_t next_handle;
} ohost_t;

typedef struct tev { uint64_t time, seq; uint32_t dst, src, kind; int32_t obj; opkt* pkt; } tev;
enum { K_HEARTBEAT, K_REFILL, K_REFILL_LO, K_PSTART, K_NOTIFY, K_DELIVER, K_DELACK, K_RTO, K_CLOSE, K_WINUPD, K_LOCAL };

typedef struct {
    const o_tcp_cfg* cfg;
    o_topo* topo;
    ohost_t* h;
    osock* s; uint32_t ns, caps;
    oproc* p;
    tev* q; uint64_t nq, capq;
    uint64_t now;
    int32_t active;                      /* the executing event's host (-1 after a deliver task) */
    opkt** pool; uint32_t npool, cappool; /* packets by CoDel id */
    obuf out;
} T;

static T* G;

static int ev_less(const tev* a, const tev* b) {   /* event.c:110-153 */
    if (a->time != b->time) return a->time < b->time;
    if (a->dst != b->dst) return a->dst < b->dst;
    if (a->src != b->src) return a->src < b->src;
    return a->seq < b->seq;
}
static void q_push(T* t, const tev* e) {
    if (t->nq == t->capq) { t->capq = t->capq ? 2 * t->capq : 1024; t->q = realloc(t->q, t->capq * sizeof(tev)); }
    uint64_t i = t->nq++;
    while (i > 0) {
        uint64_t par = (i - 1) / 2;
        if (!ev_less(e, &t->q[par])) break;
        t->q[i] = t->q[par]; i = par;
    }
    t->q[i] = *e;
}
static tev q_pop(T* t) {
    tev top = t->q[0], last = t->q[--t->nq];
    uint64_t i = 0;
    for (;;) {
        uint64_t l = 2 * i + 1, r = l + 1, m = i;
        const tev* best = &last;
        if (l < t->nq && ev_less(&t->q[l], best)) { m = l; best = &t->q[l]; }
        if (r < t->nq && ev_less(&t->q[r], best)) { m = r; best = &t->q[r]; }
        if (m == i) break;
        t->q[i] = t->q[m]; i = m;
    }
    if (t->nq) t->q[i] = last;
    return top;
}
/* event_new_ consumes the source host's event ID; scheduler_push drops
 * events at or past the end time (scheduler.c:342-357) */
static int push_ev(T* t, uint32_t src, uint32_t dst, uint64_t time, uint32_t kind, int32_t obj, opkt* pkt) {
    tev e;
    e.time = time; e.seq = t->h[src].ev_seq++; e.src = src; e.dst = dst; e.kind = kind; e.obj = obj; e.pkt = pkt;
    if (time >= t->cfg->end_time) return 0;
    q_push(t, &e);
    return 1;
}
static int sched_task(T* t, uint32_t h, uint64_t delay, uint32_t kind, int32_t obj) {
    return push_ev(t, h, h, t->now + delay, kind, obj, NULL);
}

/* ------------------------------------------------------------ packet lines */
static void ip_str(uint32_t ip, char* buf) {
    sprintf(buf, "%u.%u.%u.%u", (ip >> 24) & 255, (ip >> 16) & 255, (ip >> 8) & 255, ip & 255);
}
/* packet_toString (packet.c:518-641) */
static void pkt_string(const opkt* p, obuf* b) {
    char s[20], d[20];
    ip_str(p->sip, s); ip_str(p->dip, d);
    if (p->udp) {   /* PUDP (packet.c:535-548) */
        ob_printf(b, "packetID=%u:%llu %s:%u -> %s:%u bytes=%u", p->host_id, (unsigned long long)p->pid, s, p->sport,
                  d, p->dport, p->len);
        if (p->nst) {
            ob_printf(b, " status=");
            for (uint32_t i = 0; i < p->nst; i++) ob_printf(b, i + 1 < p->nst ? "%s," : "%s", k_status_name[p->st[i]]);
        }
        return;
    }
    ob_printf(b, "packetID=%u:%llu %s:%u -> %s:%u seq=%u ack=%u sack=", p->host_id, (unsigned long long)p->pid, s,
              p->sport, d, p->dport, p->seq, p->ack);
    int32_t first = -1, last = -1;
    for (uint32_t i = 0; i < p->nsack; i++) {
        int32_t sq = p->sacks[i];
        if (first == -1) first = sq;
        else if (last == -1 || sq == last + 1) last = sq;
        else { ob_printf(b, "%d-%d ", first, last); first = sq; last = -1; }
    }
    if (first != -1) { ob_printf(b, "%d", first); if (last != -1) ob_printf(b, "-%d", last); }
    else ob_printf(b, "NA");
    ob_printf(b, " window=%u bytes=%u", p->win, p->len);
    ob_printf(b, " header=");
    if (p->flags & F_RST) ob_printf(b, "RST");
    if (p->flags & F_SYN) ob_printf(b, "SYN");
    if (p->flags & F_FIN) ob_printf(b, "FIN");
    if (p->flags & F_ACK) ob_printf(b, "ACK");
    if (p->flags & F_DUPACK) ob_printf(b, "DUPACK");
    ob_printf(b, " tsval=%llu tsechoreply=%llu", (unsigned long long)p->tsval, (unsigned long long)p->tsecho);
    if (p->nst) {
        ob_printf(b, " status=");
        for (uint32_t i = 0; i < p->nst; i++) ob_printf(b, i + 1 < p->nst ? "%s," : "%s", k_status_name[p->st[i]]);
    }
}
/* packet_addDeliveryStatus (packet.c:647-659) at debug level: one line, at
 * the simulated time, on the active host */
static void pkt_status(opkt* p, int st) {
    if (p->nst < sizeof(p->st)) p->st[p->nst++] = (uint8_t)st;
    if (G->cfg->no_lines) return;
    obuf* b = &G->out;
    ob_printf(b, "%llu\t%d\t[%s] ", (unsigned long long)G->now, G->active, k_status_name[st]);
    pkt_string(p, b);
    ob_put(b, "\n", 1);
    b->n++;
}
static opkt* pkt_new(uint32_t h, uint32_t len) {   /* packet_new (packet.c:74-95) */
    opkt* p = calloc(1, sizeof(opkt));
    p->refs = 1;
    p->host_id = h + 1;
    p->pid = G->h[h].pkt_seq++;
    p->len = len;
    if (len > 0) p->prio = ++G->h[h].prio;   /* host_getNextPacketPriority (host.c:1663-1666) */
    return p;
}
static void pkt_ref(opkt* p) { p->refs++; }
static void pkt_unref(opkt* p) {   /* packet.c:194-201 */
    if (--p->refs == 0) {
        pkt_status(p, S_DESTROYED);
        free(p->sacks);
        free(p);
    }
}
static opkt* pkt_copy(const opkt* p) {   /* packet_copy (packet.c:100-161) */
    opkt* c = malloc(sizeof(opkt));
    *c = *p;
    c->refs = 1;
    if (p->nsack) { c->sacks = malloc(p->nsack * sizeof(int32_t)); memcpy(c->sacks, p->sacks, p->nsack * sizeof(int32_t)); }
    return c;
}

/* ------------------------------------------------------------ forward decls */
static void tcp_flush(osock* k);
static void if_send_packets(int32_t h);
static void sock_status(osock* k, uint32_t bits, int set);
static void tcp_process(osock* k, opkt* p);
static void udp_release(osock* k);

static int32_t sidx(const osock* k) { return (int32_t)(k - G->s); }

/* ------------------------------------------------------------ epoll (epoll.c)
 * The process's one watch: its readiness (_epollwatch_isReady: not closed,
 * active, read/write interest met), the epoll's readability
 * (_epoll_adjustStatus) and the notification task (+1 ns,
 * _epoll_scheduleNotification) while the process runs */
static int watch_ready(oproc* pr) {
    if (pr->wait_fd < 0) return 0;
    const osock* k = &G->s[pr->wait_fd];
    if ((k->status & DS_CLOSED) || !(k->status & DS_ACTIVE)) return 0;
    return ((k->status & DS_READABLE) && (pr->wait_events & 1)) || ((k->status & DS_WRITABLE) && (pr->wait_events & 4));
}
static void ep_schedule(oproc* pr) {
    if (pr->ep_notifying) return;
    if (!pr->ep_scheduled && pr->running) {
        if (sched_task(G, (uint32_t)pr->host, 1, K_NOTIFY, pr->index)) pr->ep_scheduled = 1;
    }
}
static void ep_status_changed(oproc* pr) {   /* epoll_descriptorStatusChanged (epoll.c:585-615) */
    pr->ep_ready = watch_ready(pr);
    pr->ep_readable = pr->ep_ready;
    if (pr->ep_readable) ep_schedule(pr);
}
static void sock_status(osock* k, uint32_t bits, int set) {   /* descriptor_adjustStatus (descriptor.c:95-137) */
    if (set) k->status |= bits; else k->status &= ~bits;
    if (k->proc >= 0) {
        oproc* pr = &G->p[k->proc];
        if (pr->wait_fd == sidx(k)) ep_status_changed(pr);
    }
}

/* ------------------------------------------------------------ sockets */
static uint64_t in_space(const osock* k) {
    const uint64_t sz = k->in_pending ? k->in_pending : k->in_size;
    return sz < k->in_len ? 0 : sz - k->in_len;
}
static uint64_t out_space(const osock* k) {
    const uint64_t sz = k->out_pending ? k->out_pending : k->out_size;
    return sz < k->out_len ? 0 : sz - k->out_len;
}
static uint64_t in_size(const osock* k) { return k->in_pending ? k->in_pending : k->in_size; }
static uint64_t out_size(const osock* k) { return k->out_pending ? k->out_pending : k->out_size; }
static void set_in_size(osock* k, uint64_t n) {   /* socket.c:294-304 */
    if (n >= k->in_len) { k->in_size = n; k->in_pending = 0; } else { k->in_size = k->in_len; k->in_pending = n; }
}
static void set_out_size(osock* k, uint64_t n) {
    if (n >= k->out_len) { k->out_size = n; k->out_pending = 0; } else { k->out_size = k->out_len; k->out_pending = n; }
}
static uint64_t tcp_out_len(const osock* k) { return k->throttled_len + k->rtx.qlen; }   /* tcp.c:701-706 */
static uint64_t space_out(const osock* k) {   /* _tcp_getBufferSpaceOut (tcp.c:714-720) */
    const int64_t s = (int64_t)out_space(k) - (int64_t)tcp_out_len(k);
    return s > 0 ? (uint64_t)s : 0;
}
static uint64_t space_in(const osock* k) {   /* _tcp_getBufferSpaceIn */
    const int64_t s = (int64_t)in_space(k) - (int64_t)k->unordered_len;
    return s > 0 ? (uint64_t)s : 0;
}
static uint64_t space_out_incl_tcp(const osock* k) {   /* socket.c:373-383 */
    const uint64_t sp = out_space(k), tl = tcp_out_len(k);
    return tl < sp ? sp - tl : 0;
}
static int sock_add_input(osock* k, opkt* p) {   /* socket_addToInputBuffer (socket.c:319-343) */
    if (p->len > in_space(k)) return 0;
    fq_push(&k->in, p);
    pkt_ref(p);
    k->in_len += p->len;
    pkt_status(p, S_RCV_SOCKET_BUFFERED);
    if (k->in_len > 0) sock_status(k, DS_READABLE, 1);
    return 1;
}
static opkt* sock_remove_input(osock* k) {   /* socket.c:345-372 */
    opkt* p = fq_pop(&k->in);
    if (p) {
        k->in_len -= p->len;
        if (k->in_pending > 0) set_in_size(k, k->in_pending);
        if (k->in_len <= 0) sock_status(k, DS_READABLE, 0);
    }
    return p;
}
/* the RR qdisc's GQueue of sockets (network_interface.c:58, 466-490, 586-591) */
static void rr_push(ohost_t* H, osock* k) {
    if (H->rr_n == H->rr_cap) {
        const uint32_t nc = H->rr_cap ? 2 * H->rr_cap : 8;
        osock** a = malloc(sizeof(osock*) * nc);
        for (uint32_t i = 0; i < H->rr_n; i++) a[i] = H->rr[(H->rr_head + i) % H->rr_cap];
        free(H->rr);
        H->rr = a; H->rr_head = 0; H->rr_cap = nc;
    }
    H->rr[(H->rr_head + H->rr_n++) % H->rr_cap] = k;
}
static void rr_push_once(ohost_t* H, osock* k) {   /* g_queue_find, then push_tail */
    for (uint32_t i = 0; i < H->rr_n; i++)
        if (H->rr[(H->rr_head + i) % H->rr_cap] == k) return;
    rr_push(H, k);
}
static osock* rr_pop(ohost_t* H) {
    osock* k = H->rr[H->rr_head];
    H->rr_head = (H->rr_head + 1) % H->rr_cap;
    H->rr_n--;
    return k;
}
static int sock_add_output(osock* k, opkt* p) {   /* socket_addToOutputBuffer (socket.c:385-424) */
    if (p->len > out_space(k)) return 0;
    if (p->prio == 0.0) fq_push(&k->outctl, p); else fq_push(&k->out, p);
    k->out_len += p->len;
    pkt_status(p, S_SND_SOCKET_BUFFERED);
    if (space_out_incl_tcp(k) <= 0) sock_status(k, DS_WRITABLE, 0);
    /* networkinterface_wantsSend (network_interface.c:581-605): tracked once */
    if (G->cfg->qdisc_rr) rr_push_once(&G->h[k->host], k);
    else if (pq_index(&G->h[k->host].fifo, k) < 0) pq_push(&G->h[k->host].fifo, k);
    if_send_packets(k->host);
    return 1;
}
static opkt* sock_peek_out(osock* k) { return k->outctl.n ? fq_peek(&k->outctl) : fq_peek(&k->out); }
static opkt* sock_remove_output(osock* k) {   /* socket.c:426-451 */
    opkt* p = k->outctl.n ? fq_pop(&k->outctl) : fq_pop(&k->out);
    if (p) {
        k->out_len -= p->len;
        if (k->out_pending > 0) set_out_size(k, k->out_pending);
        if (space_out_incl_tcp(k) > 0) sock_status(k, DS_WRITABLE, 1);
    }
    return p;
}
/* _networkinterface_compareSocket: the next packets' priorities, never equal */
static int cmp_sock(const void* a, const void* b) {
    const opkt* pa = sock_peek_out((osock*)a);
    const opkt* pb = sock_peek_out((osock*)b);
    return pa->prio > pb->prio ? 1 : -1;
}

/* ------------------------------------------------------------ paths */
static void path(int32_t a, int32_t b, double* lat, double* rel) {
    o_topo_get(G->topo, G->h[a].vertex, G->h[b].vertex, lat, rel);
}
static int32_t host_of_ip(uint32_t ip) {
    for (int32_t i = 0; i < G->cfg->n_hosts; i++) if (G->h[i].ip == ip) return i;
    return -1;
}

/* ------------------------------------------------------------ retransmit queue */
static opkt* rtx_find(osock* k, uint32_t seq, uint32_t* at) {
    for (uint32_t i = 0; i < k->rtx.nq; i++) if (k->rtx.q[i]->seq == seq) { if (at) *at = i; return k->rtx.q[i]; }
    return NULL;
}
static void rtx_remove_at(osock* k, uint32_t i) {
    memmove(&k->rtx.q[i], &k->rtx.q[i + 1], (k->rtx.nq - i - 1) * sizeof(opkt*));
    k->rtx.nq--;
}
static void tcp_add_retransmit(osock* k, opkt* p) {   /* tcp.c:854-873 */
    if (rtx_find(k, p->seq, NULL)) return;
    if (k->rtx.nq == k->rtx.capq) { k->rtx.capq = k->rtx.capq ? 2 * k->rtx.capq : 16; k->rtx.q = realloc(k->rtx.q, k->rtx.capq * sizeof(opkt*)); }
    k->rtx.q[k->rtx.nq++] = p;
    pkt_ref(p);
    pkt_status(p, S_SND_TCP_ENQUEUE_RETRANSMIT);
    k->rtx.qlen += p->len;
    if (space_out(k) == 0) sock_status(k, DS_WRITABLE, 0);
}
static int cmp_rtx(const void* a, const void* b) {
    const uint32_t x = (*(opkt* const*)a)->seq, y = (*(opkt* const*)b)->seq;
    return x < y ? -1 : x > y ? 1 : 0;
}
static void tcp_clear_retransmit(osock* k, uint32_t seq) {   /* tcp.c:876-897 (walked in sequence order) */
    qsort(k->rtx.q, k->rtx.nq, sizeof(opkt*), cmp_rtx);
    uint32_t w = 0;
    opkt** gone = malloc((k->rtx.nq + 1) * sizeof(opkt*));
    uint32_t ng = 0;
    for (uint32_t i = 0; i < k->rtx.nq; i++) {
        opkt* p = k->rtx.q[i];
        if (p->seq < seq) {
            k->rtx.qlen -= p->len;
            pkt_status(p, S_SND_TCP_DEQUEUE_RETRANSMIT);
            gone[ng++] = p;
        } else {
            k->rtx.q[w++] = p;
        }
    }
    k->rtx.nq = w;
    for (uint32_t i = 0; i < ng; i++) pkt_unref(gone[i]);
    free(gone);
    if (space_out(k) > 0) sock_status(k, DS_WRITABLE, 1);
}
static void tcp_clear_retransmit_range(osock* k, uint32_t begin, uint32_t end) {   /* tcp.c:900-920 */
    for (uint32_t sq = begin; sq < end; ++sq) {
        uint32_t at;
        opkt* p = rtx_find(k, sq, &at);
        if (p) {
            k->rtx.qlen -= p->len;
            pkt_status(p, S_SND_TCP_DEQUEUE_RETRANSMIT);
            rtx_remove_at(k, at);
            pkt_unref(p);
        }
    }
    if (space_out(k) > 0) sock_status(k, DS_WRITABLE, 1);
}

/* ------------------------------------------------------------ timers */
static void tcp_schedule_rto(osock* k, uint64_t now, uint64_t delay) {   /* tcp.c:925-946 */
    uint64_t* x = malloc(sizeof(uint64_t));
    *x = now + delay;
    pq_push(&k->rtx.timers, x);
    sched_task(G, (uint32_t)k->host, delay, K_RTO, sidx(k));
}
static void tcp_schedule_rto_if_needed(osock* k, uint64_t now) {   /* tcp.c:948-960 */
    uint64_t* nx = pq_peek(&k->rtx.timers);
    if (nx && *nx <= k->rtx.desired) return;
    tcp_schedule_rto(k, now, k->rtx.desired - now);
}
static void tcp_set_rto_timer(osock* k, uint64_t now) {   /* tcp.c:962-971 */
    k->rtx.desired = now + (uint64_t)k->rtx.timeout * MS;
    tcp_schedule_rto_if_needed(k, now);
}
static void tcp_set_rto(osock* k, int v) {   /* tcp.c:982-989: [200 ms, 120 s] */
    k->rtx.timeout = v;
    if (k->rtx.timeout > 120000) k->rtx.timeout = 120000;
    if (k->rtx.timeout < 200) k->rtx.timeout = 200;
}

/* ------------------------------------------------------------ Reno (tcp_cong_reno.c) */
static void reno_new_ack(osock* k, uint32_t n);
static void reno_to_cong_avoid(osock* k, uint32_t n) {   /* :40-45 */
    k->reno.ca_nacked = 0;
    k->reno.state = 2;
    reno_new_ack(k, n);
}
static void reno_new_ack(osock* k, uint32_t n) {
    if (k->reno.state == 0) {   /* slow start (:65-89) */
        k->reno.ndup = 0;
        uint32_t nc = k->cwnd + n;
        if (nc >= k->reno.ssthresh) {
            const uint32_t left = nc - k->reno.ssthresh;
            k->cwnd = k->reno.ssthresh;
            reno_to_cong_avoid(k, left);
        } else {
            k->cwnd = nc;
        }
    } else if (k->reno.state == 1) {   /* fast recovery (:97-104) */
        k->reno.ndup = 0;
        k->cwnd = k->reno.ssthresh;
        reno_to_cong_avoid(k, n);
    } else {   /* congestion avoidance (:108-118) */
        k->reno.ca_nacked += n;
        while (k->reno.ca_nacked >= k->cwnd) { k->reno.ca_nacked -= k->cwnd; k->cwnd += 1; }
    }
}
static void reno_dup_ack(osock* k) {
    if (k->reno.state == 1) { k->cwnd += 1; return; }   /* :93-95 */
    k->reno.ndup++;                                      /* :49-63 */
    if (k->reno.ndup == 3) {
        k->reno.ssthresh = (k->cwnd / 2) + 1;
        k->cwnd = k->reno.ssthresh + 3;
        k->reno.state = 1;
    }
}
static void reno_timeout(osock* k) {   /* :150-161 */
    k->reno.ndup = 0;
    k->reno.ssthresh = (k->cwnd / 2) + 1;
    k->cwnd = 10;
    k->reno.state = 0;
}

/* ------------------------------------------------------------ the TCP socket */
static int32_t sock_new(int32_t h) {   /* tcp_new (tcp.c:2452-2512) */
    uint32_t si = 0;   /* a released datagram socket's slot first */
    while (si < G->ns && G->s[si].used) si++;
    if (si == G->ns) {
        if (G->ns == G->caps) { fprintf(stderr, "o_tcp: socket table full\n"); abort(); }   /* never moves */
        G->ns++;
    }
    osock* k = &G->s[si];
    memset(k, 0, sizeof(*k));
    k->used = 1;
    k->host = h;
    k->handle = G->h[h].next_handle++;
    k->proc = -1;
    k->parent = -1;
    k->in_size = G->cfg->recv_buf;
    k->out_size = G->cfg->send_buf;
    /* tcp_cong_reno_init: ca init sets 10, then cwnd = 1 (tcp_cong_reno.c:122-184) */
    k->cwnd = 1;
    k->reno.ssthresh = 0x7fffffff;
    const uint32_t iw = G->cfg->tcp_window;
    k->snd.window = iw; k->snd.last_window = iw; k->rcv.window = iw; k->rcv.last_window = iw;
    k->snd.unacked = 1; k->snd.next = 1; k->snd.end = 1; k->snd.last_ack = 1;
    k->rcv.end = 1; k->rcv.next = 1; k->rcv.start = 1; k->rcv.last_ack = 1;
    k->at.enabled = 1;
    k->throttled.cmp = cmp_seq;
    k->unordered.cmp = cmp_seq;
    k->rtx.timers.cmp = cmp_time;
    k->rtx.tally.last_ack = -1;
    tcp_set_rto(k, 1000);
    return (int32_t)si;
}
static uint32_t tcp_get_ip(osock* k) {   /* tcp.c:335-353 */
    if (k->server) return k->bound ? k->bound_ip : k->last_ip;
    if (k->child) { osock* pa = &G->s[k->parent]; return pa->bound ? pa->bound_ip : pa->last_ip; }
    return k->bound_ip;
}
static uint32_t tcp_get_peer_ip(osock* k) {   /* tcp.c:355-361 */
    uint32_t ip = k->peer_ip;
    if (k->server && ip == 0) ip = k->last_peer_ip;
    return ip;
}
static uint32_t src_ip_for(osock* k, uint32_t dst) {
    uint32_t ip = tcp_get_ip(k);
    if (ip == 0) ip = (dst == 0x7f000001u) ? 0x7f000001u : G->h[k->host].ip;
    return ip;
}
static void tcp_update_rcv_window(osock* k) {   /* tcp.c:762-782 */
    k->rcv.window = (uint32_t)(in_space(k) / MSS);
}
static void tcp_update_snd_window(osock* k) {   /* tcp.c:784-789 */
    const int lw = (int)k->rcv.last_window;
    k->snd.window = (uint32_t)((int)k->cwnd < lw ? (int)k->cwnd : lw);
}
static void tcp_set_state(osock* k, int st);
static void tcp_tune_initial_buffers(osock* k) {   /* tcp.c:441-533 */
    k->at.did_init = 1;
    const uint32_t sip = src_ip_for(k, tcp_get_peer_ip(k));
    const uint32_t dip = tcp_get_peer_ip(k);
    if (sip == dip) {
        set_in_size(k, 6291456);
        set_out_size(k, 4194304);
        k->info.rtt = 0xffffffffu;
        return;
    }
    const int32_t a = host_of_ip(sip), b = host_of_ip(dip);
    /* _tcp_calculateRTT (tcp.c:363-405): ceil of both one-way latencies */
    double l1, l2, r;
    path(a, b, &l1, &r);
    path(b, a, &l2, &r);
    const uint32_t rtt = (uint32_t)ceil(l1) + (uint32_t)ceil(l2);
    const uint32_t my_up = (uint32_t)G->cfg->bw_up_kibps[a], their_down = (uint32_t)G->cfg->bw_down_kibps[b];
    const uint32_t sbw = my_up < their_down ? my_up : their_down;
    uint64_t sendbuf = (uint64_t)(((float)(rtt * sbw) * 1024.0f * 1.25f) / 1000.0f);
    const uint32_t my_down = (uint32_t)G->cfg->bw_down_kibps[a], their_up = (uint32_t)G->cfg->bw_up_kibps[b];
    const uint32_t rbw = my_down < their_up ? my_down : their_up;
    uint64_t recvbuf = (uint64_t)(((float)(rtt * rbw) * 1024.0f * 1.25f) / 1000.0f);
    if (sendbuf < 16384) sendbuf = 16384;
    if (sendbuf > 4194304) sendbuf = 4194304;
    if (recvbuf < 87380) recvbuf = 87380;
    if (recvbuf > 6291456) recvbuf = 6291456;
    set_in_size(k, recvbuf);
    set_out_size(k, sendbuf);
}
static uint64_t rtt_mem(osock* k, int rmem) {   /* tcp.c:407-427 */
    const ohost_t* H = &G->h[k->host];
    const uint64_t refill = rmem ? H->rx_refill : H->tx_refill;
    const uint64_t kib = (uint64_t)((uint32_t)((refill * 1000u) / 1024u));   /* getSpeed{Down,Up}KiBps */
    const uint64_t bw = kib * 1024;
    const double rtt_s = ((double)k->timing.srtt) / ((double)1000);
    return (uint64_t)((double)bw * rtt_s);
}
static uint64_t clamp_u(uint64_t v, uint64_t lo, uint64_t hi) { return v < lo ? lo : v > hi ? hi : v; }
static void tcp_autotune_rcv(osock* k, uint32_t copied) {   /* tcp.c:535-564 */
    k->at.bytes_copied += copied;
    uint64_t space = 2 * k->at.bytes_copied;
    if (k->at.space > space) space = k->at.space;
    const uint64_t cur = in_size(k);
    if (space > cur) {
        k->at.space = space;
        const uint64_t mx = clamp_u(rtt_mem(k, 1), 6291456, 62914560);
        const uint64_t nsz = space < mx ? space : mx;
        if (nsz > cur) set_in_size(k, nsz);
    }
    if (k->at.last_adjust == 0) {
        k->at.last_adjust = G->now;
    } else if (k->timing.srtt > 0) {
        const uint64_t thr = (uint64_t)k->timing.srtt * MS;
        if (G->now - k->at.last_adjust > thr) { k->at.last_adjust = G->now; k->at.bytes_copied = 0; }
    }
}
static void tcp_autotune_snd(osock* k) {   /* tcp.c:566-591 */
    const uint64_t mx = clamp_u(rtt_mem(k, 0), 4194304, 41943040);
    uint64_t nsz = (uint64_t)2404 * 2 * (uint64_t)k->cwnd;
    if (nsz > mx) nsz = mx;
    if (nsz > out_size(k)) set_out_size(k, nsz);
}
static void tcp_buffer_out(osock* k, opkt* p) {   /* tcp.c:729-745 */
    if (pq_index(&k->throttled, p) >= 0) return;
    pq_push(&k->throttled, p);
    pkt_ref(p);
    k->throttled_len += p->len;
    if (space_out(k) == 0) sock_status(k, DS_WRITABLE, 0);
    pkt_status(p, S_SND_TCP_ENQUEUE_THROTTLED);
}
static void tcp_buffer_in(osock* k, opkt* p) {   /* tcp.c:747-760 */
    if (pq_index(&k->unordered, p) >= 0) return;
    pq_push(&k->unordered, p);
    pkt_ref(p);
    k->unordered_len += p->len;
    pkt_status(p, S_RCV_TCP_ENQUEUE_UNORDERED);
}
static opkt* tcp_create_packet(osock* k, uint32_t flags, uint32_t len) {   /* tcp.c:791-835 */
    const uint32_t dip = tcp_get_peer_ip(k);
    const uint16_t sport = k->child ? G->s[k->parent].bound_port : k->bound_port;
    const uint16_t dport = k->server ? k->last_peer_port : k->peer_port;
    const uint32_t sip = src_ip_for(k, dip);
    tcp_update_rcv_window(k);
    const int fin_not_ack = (flags & F_FIN) && !(flags & F_ACK);
    const uint32_t seq = (len > 0 || fin_not_ack) ? k->snd.next : 0;
    opkt* p = pkt_new((uint32_t)k->host, len);
    p->flags = flags; p->sip = sip; p->sport = sport; p->dip = dip; p->dport = dport; p->seq = seq;
    pkt_status(p, S_SND_CREATED);
    if (seq > 0) k->snd.next++;
    return p;
}
static void tcp_send_control(osock* k, uint32_t flags) {   /* tcp.c:837-852 */
    opkt* c = tcp_create_packet(k, flags, 0);
    c->prio = 0.0;
    tcp_buffer_out(k, c);
    tcp_flush(k);
    pkt_unref(c);
}
static void tcp_retransmit_packet(osock* k, uint32_t seq) {   /* tcp.c:1027-1065 */
    uint32_t at;
    opkt* p = rtx_find(k, seq, &at);
    if (!p) return;
    rtx_remove_at(k, at);
    k->rtx.qlen -= p->len;
    pkt_status(p, S_SND_TCP_DEQUEUE_RETRANSMIT);
    if (space_out(k) > 0) sock_status(k, DS_WRITABLE, 1);
    tcp_set_rto_timer(k, G->now);
    tcp_buffer_out(k, p);
    pkt_status(p, S_SND_TCP_RETRANSMITTED);
    k->info.retx_count++;
    pkt_unref(p);
}
static void tcp_send_shutdown_fin(osock* k) {   /* tcp.c:1067-1088 */
    int send = 0;
    if (k->state == TS_ESTABLISHED || k->state == TS_SYNRECEIVED) { tcp_set_state(k, TS_FINWAIT1); send = 1; }
    else if (k->state == TS_CLOSEWAIT) { tcp_set_state(k, TS_LASTACK); send = 1; }
    if (send) {
        opkt* fin = tcp_create_packet(k, F_FIN, 0);
        tcp_buffer_out(k, fin);
        tcp_flush(k);
        pkt_unref(fin);
    }
}
/* tcp_networkInterfaceIsAboutToSendPacket (tcp.c:1090-1119) */
static void tcp_about_to_send(osock* k, opkt* p) {
    if (k->snd.sacks.n > 0) {
        free(p->sacks);
        p->flags |= F_SACK;
        p->nsack = k->snd.sacks.n;
        p->sacks = malloc(p->nsack * sizeof(int32_t));
        memcpy(p->sacks, k->snd.sacks.v, p->nsack * sizeof(int32_t));
    }
    p->ack = k->rcv.next;
    p->win = k->rcv.window;
    p->tsval = G->now;
    p->tsecho = k->rcv.last_ts;
    k->snd.last_ack = k->rcv.next;
    k->snd.last_window = k->rcv.window;
    k->info.last_ack_sent = G->now;
    if (p->flags & F_ACK) k->snd.delack_counter = 0;
    if (p->seq > 0 || (p->flags & F_SYN)) {
        tcp_add_retransmit(k, p);
        if (!k->rtx.desired) tcp_set_rto_timer(k, G->now);
    }
}
static void tcp_flush(osock* k) {   /* tcp.c:1121-1278 */
    tcp_update_rcv_window(k);
    tcp_update_snd_window(k);
    if (k->rtx.tally.lost.n > 0) {
        const uint32_t nl = k->rtx.tally.lost.n;
        uint32_t* lr = malloc(2 * nl * sizeof(uint32_t));
        for (uint32_t i = 0; i < nl; i++) { lr[2 * i] = (uint32_t)k->rtx.tally.lost.r[i].a; lr[2 * i + 1] = (uint32_t)k->rtx.tally.lost.r[i].b; }
        for (uint32_t i = 0; i < nl; i++) {
            for (uint32_t j = lr[2 * i]; j < lr[2 * i + 1]; ++j) tcp_retransmit_packet(k, j);
            tally_mark_retransmitted(&k->rtx.tally, lr[2 * i], lr[2 * i + 1]);
        }
        free(lr);
    }
    while (k->throttled.n) {
        opkt* p = pq_peek(&k->throttled);
        if (!p) break;
        const uint32_t len = p->len;
        if (len > 0) {
            const int in_window = p->seq < (uint32_t)(k->snd.unacked + k->snd.window);
            const int in_buffer = len <= out_space(k);
            if (!in_buffer || !in_window) break;
            k->info.last_data_sent = G->now;
        }
        pq_pop(&k->throttled);
        k->throttled_len -= len;
        sock_add_output(k, p);
        k->snd.packets_sent++;
        if (p->seq > k->snd.highest) k->snd.highest = p->seq;
    }
    while (k->unordered.n) {
        opkt* p = pq_peek(&k->unordered);
        if (p->seq == k->rcv.next) {
            if (sock_add_input(k, p)) {
                k->rcv.last_seq = p->seq;
                pq_pop(&k->unordered);
                const uint32_t len = p->len;
                pkt_unref(p);
                k->unordered_len -= len;
                k->rcv.next++;
                continue;
            }
        }
        break;
    }
    if ((k->flags & TF_SHOULD_SEND_WR_FIN) && tcp_out_len(k) == 0) {
        tcp_send_shutdown_fin(k);
        k->flags &= ~TF_SHOULD_SEND_WR_FIN;
    }
    if ((k->flags & TF_LOCAL_CLOSED_WR) || (k->error & TE_CONNECTION_RESET)) k->error |= TE_SEND_EOF;
    if ((k->flags & TF_LOCAL_CLOSED_RD) || (k->flags & TF_REMOTE_CLOSED) || (k->error & TE_CONNECTION_RESET)) {
        if (k->rcv.next >= k->rcv.end && !(k->flags & TF_EOF_RD_SIGNALED)) {
            k->error |= TE_RECEIVE_EOF;
            sock_status(k, DS_READABLE, 1);
        }
    }
    if ((k->error & TE_CONNECTION_RESET) && (k->flags & TF_RESET_SIGNALED)) sock_status(k, DS_WRITABLE, 0);
    else if ((k->error & TE_SEND_EOF) && (k->flags & TF_EOF_WR_SIGNALED)) sock_status(k, DS_WRITABLE, 0);
    else if (space_out(k) <= 0) sock_status(k, DS_WRITABLE, 0);
    else sock_status(k, DS_WRITABLE, 1);
}

/* _host_disassociateInterface via host_closeDescriptor */
static void host_close_descriptor(osock* k) { k->assoc = 0; k->assoc_general = 0; }

static void tcp_set_state(osock* k, int st) {   /* tcp.c:607-693 */
    k->state_last = k->state;
    k->state = st;
    switch (st) {
    case TS_LISTEN: sock_status(k, DS_ACTIVE, 1); break;
    case TS_ESTABLISHED: k->flags |= TF_WAS_ESTABLISHED; sock_status(k, DS_ACTIVE | DS_WRITABLE, 1); break;
    case TS_CLOSED: {
        tcp_clear_retransmit(k, 0xffffffffu);
        sock_status(k, DS_ACTIVE, 0);
        if (!k->server || k->children.n == 0) {
            if (k->child && k->parent >= 0) {
                osock* pa = &G->s[k->parent];
                for (uint32_t i = 0; i < pa->children.n; i++)
                    if (pa->children.v[i] == sidx(k)) { pa->children.v[i] = pa->children.v[--pa->children.n]; break; }
                if (pa->state == TS_CLOSED && pa->children.n == 0) host_close_descriptor(pa);
            }
            host_close_descriptor(k);
        }
        break;
    }
    case TS_TIMEWAIT: {
        uint64_t delay = 60 * SEC;   /* CONFIG_TCPCLOSETIMER_DELAY */
        if (k->child && k->parent >= 0) delay = SEC;
        sched_task(G, (uint32_t)k->host, delay, K_CLOSE, sidx(k));
        break;
    }
    default: break;
    }
}
static void tcp_update_rtt(osock* k, uint64_t ts) {   /* tcp.c:991-1025 */
    int rtt = (int)((G->now - ts) / MS);
    if (rtt <= 0) rtt = 1;
    if (!k->timing.srtt) {
        k->timing.srtt = rtt;
        k->timing.rttvar = rtt / 2;
        if (k->at.enabled && !k->at.did_init) tcp_tune_initial_buffers(k);
    } else {
        k->timing.rttvar = (3 * k->timing.rttvar / 4) + (abs(k->timing.srtt - rtt) / 4);
        k->timing.srtt = (7 * k->timing.srtt / 8) + (rtt / 8);
    }
    tcp_set_rto(k, k->timing.srtt + 4 * k->timing.rttvar);
}
static void tcp_remove_sacks(osock* k, int32_t seq) {   /* tcp.c:1579-1595 */
    uint32_t w = 0;
    for (uint32_t i = 0; i < k->snd.sacks.n; i++) if (k->snd.sacks.v[i] > seq) k->snd.sacks.v[w++] = k->snd.sacks.v[i];
    k->snd.sacks.n = w;
}
static uint32_t tcp_data_processing(osock* k, opkt* p) {   /* tcp.c:1597-1660 */
    uint32_t fl = 0;
    if (p->seq >= k->rcv.next + k->rcv.window) {
        fl |= PF_PROCESSED;
        pkt_status(p, S_RCV_SOCKET_DROPPED);
    } else if (p->seq >= k->rcv.next) {
        fl |= PF_PROCESSED;
        const int is_next = p->seq == k->rcv.next;
        const int fits = p->len <= space_in(k);
        if (!is_next && fits) {
            iv_push(&k->snd.sacks, (int32_t)p->seq);
        } else if (k->snd.sacks.n > 0) {
            uint32_t it = 0;
            const int32_t first = k->snd.sacks.v[0];
            if (first <= (int32_t)p->seq + 1) {
                uint32_t nx = 1;
                while (nx < k->snd.sacks.n) {
                    const int32_t cur = k->snd.sacks.v[it], nxt = k->snd.sacks.v[nx];
                    if (cur + 1 < nxt && cur > (int32_t)p->seq) break;
                    it = nx;
                    nx = it + 1;
                }
                tcp_remove_sacks(k, k->snd.sacks.v[it]);
            }
        }
        const int waiting_read = (k->status & DS_READABLE) != 0;
        if ((is_next && !waiting_read) || fits) {
            tcp_buffer_in(k, p);
            k->info.last_data_recv = G->now;
            fl |= PF_DATA_RECEIVED;
        } else {
            pkt_status(p, S_RCV_SOCKET_DROPPED);
        }
    }
    return fl;
}
static uint32_t tcp_ack_processing(osock* k, opkt* p) {   /* tcp.c:1662-1750 */
    uint32_t fl = PF_PROCESSED;
    const uint32_t prev_win = k->rcv.last_window;
    const int valid_ack = p->ack > k->snd.unacked && p->ack <= k->snd.next;
    const int valid_win = (p->ack == k->rcv.last_ack && p->win > prev_win) ||
                          (p->ack > k->rcv.last_ack && p->win != prev_win);
    if (p->win != prev_win) fl |= PF_RWND_UPDATED;
    const int is_dup = (p->flags & F_DUPACK) != 0;
    fl |= tally_update(&k->rtx.tally, p->ack, is_dup);
    if (is_dup) reno_dup_ack(k);
    int n_acked = 0;
    if (valid_ack) {
        tcp_clear_retransmit_range(k, k->rcv.last_ack, p->ack);
        k->rcv.last_ack = p->ack;
        n_acked = (int)(p->ack - k->snd.unacked);
        k->snd.unacked = p->ack;
        if (n_acked > 0) {
            fl |= PF_DATA_ACKED;
            reno_new_ack(k, (uint32_t)n_acked);
            if (k->at.enabled) tcp_autotune_snd(k);
        }
        if (k->rtx.backoff > 2) {
            k->timing.srtt = 0;
            k->timing.rttvar = 0;
            tcp_set_rto(k, 1000);
        }
        k->rtx.backoff = 0;
    }
    if (valid_win) k->rcv.last_window = p->win;
    if (k->rtx.qlen == 0) k->rtx.desired = 0;
    else if (n_acked > 0) tcp_set_rto_timer(k, G->now);
    k->info.last_ack_recv = G->now;
    return fl;
}
static void tcp_process(osock* k, opkt* p) {   /* tcp.c:1777-2099 */
    /* _tcp_getSourceTCP: a server's child keyed by the peer's ip:port */
    if (k->server) {
        for (uint32_t i = 0; i < k->children.n; i++) {
            osock* c = &G->s[k->children.v[i]];
            if (c->peer_ip == p->sip && c->peer_port == p->sport) { k = c; break; }
        }
    }
    if (p->flags & F_RST) {
        if (k->state != TS_LISTEN && !(k->error & TE_CONNECTION_RESET)) {   /* TCPS_LISTEN is a bit there; a state here */
            k->error |= TE_CONNECTION_RESET;
            k->flags |= TF_REMOTE_CLOSED;
            tcp_set_state(k, TS_TIMEWAIT);
            k->rcv.end = k->rcv.next;
        }
        return;
    }
    if (k->server) { k->last_peer_ip = p->sip; k->last_peer_port = p->sport; k->last_ip = p->dip; }
    uint32_t fl = 0, resp = 0;
    switch (k->state) {
    case TS_LISTEN:
        if (p->flags & F_SYN) {
            fl |= PF_PROCESSED;
            const int32_t li = sidx(k);
            const int32_t ci = sock_new(k->host);   /* host_createDescriptor: a new TCP socket */
            osock* l = &G->s[li];
            osock* c = &G->s[ci];
            c->child = 1;
            c->parent = li;
            c->child_state = 1;
            c->peer_ip = p->sip; c->peer_port = p->sport;
            c->bound = 1; c->bound_ip = l->bound_ip; c->bound_port = l->bound_port;
            iv_push(&l->children, ci);
            c->rcv.start = p->seq;
            c->rcv.next = c->rcv.start + 1;
            tcp_set_state(c, TS_SYNRECEIVED);
            k = c;
            resp = F_SYN | F_ACK;
        }
        break;
    case TS_SYNSENT:
        if ((p->flags & F_SYN) && (p->flags & F_ACK)) {
            fl |= PF_PROCESSED;
            k->rcv.start = p->seq;
            k->rcv.next = k->rcv.start + 1;
            resp |= F_ACK;
            tcp_set_state(k, TS_ESTABLISHED);
            tcp_clear_retransmit(k, 1);
        } else if (p->flags & F_SYN) {
            fl |= PF_PROCESSED;
            k->rcv.start = p->seq;
            k->rcv.next = k->rcv.start + 1;
            resp |= F_ACK;
            tcp_set_state(k, TS_SYNRECEIVED);
        }
        break;
    case TS_SYNRECEIVED:
        if (p->flags & F_ACK) {
            fl |= PF_PROCESSED;
            tcp_set_state(k, TS_ESTABLISHED);
            tcp_clear_retransmit(k, 1);
            if (k->child) {
                k->child_state = 2;
                osock* pa = &G->s[k->parent];
                iv_push(&pa->pending, sidx(k));
                sock_status(pa, DS_READABLE, 1);
            }
        }
        break;
    case TS_ESTABLISHED:
        if (p->flags & F_FIN) {
            fl |= PF_PROCESSED;
            k->flags |= TF_REMOTE_CLOSED;
            resp |= F_FIN | F_ACK;
            tcp_set_state(k, TS_CLOSEWAIT);
            k->rcv.end = p->seq;
        }
        break;
    case TS_FINWAIT1:
        if ((p->flags & F_FIN) && (p->flags & F_ACK)) {
            fl |= PF_PROCESSED;
            tcp_set_state(k, TS_FINWAIT2);
        } else if (p->flags & F_FIN) {
            fl |= PF_PROCESSED;
            resp |= F_FIN | F_ACK;
            k->flags |= TF_REMOTE_CLOSED;
            tcp_set_state(k, TS_CLOSING);
            k->rcv.end = p->seq;
        }
        break;
    case TS_FINWAIT2:
        if (p->flags & F_FIN) {
            fl |= PF_PROCESSED;
            resp |= F_FIN | F_ACK;
            k->flags |= TF_REMOTE_CLOSED;
            tcp_set_state(k, TS_TIMEWAIT);
            k->rcv.end = p->seq;
        }
        break;
    case TS_CLOSING:
        if ((p->flags & F_FIN) && (p->flags & F_ACK)) { fl |= PF_PROCESSED; tcp_set_state(k, TS_TIMEWAIT); }
        break;
    case TS_TIMEWAIT:
    case TS_CLOSEWAIT:
        break;
    case TS_LASTACK:
        if ((p->flags & F_FIN) && (p->flags & F_ACK)) { fl |= PF_PROCESSED; tcp_set_state(k, TS_CLOSED); return; }
        break;
    default:
        pkt_status(p, S_RCV_SOCKET_DROPPED);
        return;
    }
    if (k->state == TS_LISTEN) {
        if (!(fl & PF_PROCESSED)) pkt_status(p, S_RCV_SOCKET_DROPPED);
        return;
    }
    if (p->len > 0 && !(k->error & TE_RECEIVE_EOF)) fl |= tcp_data_processing(k, p);
    if (p->flags & F_ACK) fl |= tcp_ack_processing(k, p);
    if (!(fl & PF_PROCESSED)) {
        pkt_status(p, S_RCV_SOCKET_DROPPED);
        return;
    }
    if (p->nsack) tally_mark_sacked(&k->rtx.tally, p->sacks, p->nsack);
    k->rcv.last_ts = p->tsval;
    if (p->tsecho && k->rtx.backoff == 0) tcp_update_rtt(k, p->tsecho);
    if (p->seq > k->rcv.next && p->seq < k->rcv.next + k->rcv.window) resp |= (F_ACK | F_DUPACK);
    else if (fl & PF_DATA_RECEIVED) resp |= F_ACK;
    if (resp != 0 && (!(k->error & TE_RECEIVE_EOF) || (resp & F_FIN))) {
        if (resp != F_ACK) {
            tcp_send_control(k, resp);
        } else {
            if (!k->snd.delack_sched) {
                uint64_t delay;
                if (k->snd.quick_acks < 1000) { delay = MS; k->snd.quick_acks++; } else delay = 5 * MS;
                sched_task(G, (uint32_t)k->host, delay, K_DELACK, sidx(k));
                k->snd.delack_sched = 1;
            }
            k->snd.delack_counter++;
        }
    }
    tcp_flush(k);
    k->rcv.last_ts = 0;
}

/* ------------------------------------------------------------ the interface */
static void refill_if_needed(int32_t h) {   /* network_interface.c:130-161 (started at t = 0) */
    ohost_t* H = &G->h[h];
    if (((H->tx_rem < H->tx_cap) || (H->rx_rem < H->rx_cap)) && !H->refill_pending) {
        sched_task(G, (uint32_t)h, MS - (G->now % MS), K_REFILL, -1);
        H->refill_pending = 1;
    }
}
static void consume(uint64_t* rem, uint64_t n) { *rem = (n >= *rem) ? 0 : *rem - n; }
static osock* lookup_socket(int32_t h, int udp, uint16_t port, uint32_t peer_ip, uint16_t peer_port) {
    /* the general key (listeners) first, then the destination-specific one
     * (network_interface.c:385-403); keys are per protocol */
    for (uint32_t i = 0; i < G->ns; i++) {
        osock* k = &G->s[i];
        if (k->used && k->host == h && k->assoc && k->assoc_general && k->udp == udp && k->bound_port == port) return k;
    }
    for (uint32_t i = 0; i < G->ns; i++) {
        osock* k = &G->s[i];
        if (k->used && k->host == h && k->assoc && !k->assoc_general && k->udp == udp && k->bound_port == port &&
            k->peer_ip == peer_ip && k->peer_port == peer_port)
            return k;
    }
    return NULL;
}
static void if_receive_packet(int32_t h, opkt* p) {   /* network_interface.c:375-419 */
    pkt_status(p, S_RCV_INTERFACE_RECEIVED);
    osock* k = lookup_socket(h, p->udp, p->dport, p->sip, p->sport);
    if (k) {
        pkt_status(p, S_RCV_SOCKET_PROCESSED);   /* socket_pushInPacket (socket.c:140-145) */
        if (k->udp) {   /* udp_processPacket (udp.c:52-61) */
            if (p->len > 0 && !sock_add_input(k, p)) pkt_status(p, S_RCV_SOCKET_DROPPED);
        } else {
            tcp_process(k, p);
        }
    } else {
        pkt_status(p, S_RCV_INTERFACE_DROPPED);
    }
}
static void if_receive_packets(int32_t h) {   /* network_interface.c:421-455 */
    ohost_t* H = &G->h[h];
    o_codel_entry drops[64];
    while (H->rx_rem >= MTU) {
        o_codel_entry e;
        uint32_t nd = 0;
        const int have = o_codel_dequeue(&H->codel, G->now, &e, drops, 64, &nd);
        for (uint32_t i = 0; i < nd && i < 64; i++) {   /* CoDel drops (router_queue_codel.c:135-146) */
            opkt* dp = G->pool[drops[i].id];
            pkt_status(dp, S_ROUTER_DROPPED);
            pkt_unref(dp);
        }
        if (!have) break;
        opkt* p = G->pool[e.id];
        pkt_status(p, S_ROUTER_DEQUEUED);   /* router_dequeue (router.c:125-133) */
        const uint64_t len = (uint64_t)p->len + hdr_of(p);
        if_receive_packet(h, p);
        pkt_unref(p);
        consume(&H->rx_rem, len);
        refill_if_needed(h);
    }
}
static void worker_send_packet(int32_t h, opkt* p) {   /* worker.c:260-321 */
    const int32_t d = host_of_ip(p->dip);
    double lat, rel;
    path(h, d, &lat, &rel);   /* topology_getReliability */
    const double chance = o_next_double(&G->h[h].rng);
    if (chance <= rel || p->len == 0) {
        path(h, d, &lat, &rel);   /* topology_getLatency */
        const uint64_t t = G->now + (uint64_t)ceil(lat * (double)MS);
        o_topo_count_packet(G->topo, G->h[h].vertex, G->h[d].vertex);
        pkt_status(p, S_INET_SENT);
        opkt* c = pkt_copy(p);
        push_ev(G, (uint32_t)h, (uint32_t)d, t, K_DELIVER, -1, c);
    } else {
        pkt_status(p, S_INET_DROPPED);
    }
}
static void if_send_packets(int32_t h) {   /* network_interface.c:519-579 */
    ohost_t* H = &G->h[h];
    while (H->tx_rem >= MTU) {
        opkt* p = NULL;
        osock* drained = NULL;   /* left the sendable queue: a closed datagram socket is released after */
        if (G->cfg->qdisc_rr) {
            while (!p && H->rr_n) {   /* _networkinterface_selectRoundRobin (:466-490) */
                osock* k = rr_pop(H);
                p = sock_remove_output(k);
                if (p && !k->udp) tcp_about_to_send(k, p);   /* _networkinterface_updatePacketHeader */
                if (sock_peek_out(k)) rr_push(H, k);
                else drained = k;
            }
        }
        while (!p && H->fifo.n) {   /* _networkinterface_selectFirstInFirstOut (:492-517) */
            osock* k = pq_pop(&H->fifo);
            p = sock_remove_output(k);
            if (p && !k->udp) tcp_about_to_send(k, p);
            if (sock_peek_out(k)) pq_push(&H->fifo, k);
            else drained = k;
        }
        if (!p) {
            if (drained) udp_release(drained);
            break;
        }
        pkt_status(p, S_SND_INTERFACE_SENT);
        if (p->dip == H->ip) {   /* our own interface (:548-555): a +1 ns task, no router, no bandwidth */
            pkt_ref(p);
            if (!push_ev(G, (uint32_t)h, (uint32_t)h, G->now + 1, K_LOCAL, -1, p)) pkt_unref(p);
        } else {
            worker_send_packet(h, p);
        }
        consume(&H->tx_rem, (uint64_t)p->len + hdr_of(p));
        refill_if_needed(h);
        pkt_unref(p);
        if (drained) udp_release(drained);
    }
}
static void refill_cb(int32_t h) {   /* network_interface.c:163-183 */
    ohost_t* H = &G->h[h];
    H->refill_pending = 0;
    H->rx_rem += H->rx_refill; if (H->rx_rem > H->rx_cap) H->rx_rem = H->rx_cap;
    H->tx_rem += H->tx_refill; if (H->tx_rem > H->tx_cap) H->tx_rem = H->tx_cap;
    if_receive_packets(h);
    if_send_packets(h);
    refill_if_needed(h);
}

/* ------------------------------------------------------------ host calls */
static uint16_t random_port(ohost_t* H) {   /* host.c:1058-1070 */
    const double f = o_next_double(&H->rng);
    const double pick = round(f * (double)(65535 - 10000));
    uint16_t p = (uint16_t)pick;
    return (uint16_t)(p + 10000);
}
/* _host_isInterfaceAvailable (host.c:1029-1056) -> networkinterface_isAssociated
 * (network_interface.c:279-301): the port is taken by a socket associated with
 * no peer (the general key) or with this peer */
static int port_free(int32_t h, int udp, uint16_t port, uint32_t pip, uint16_t pport) {
    for (uint32_t i = 0; i < G->ns; i++) {
        const osock* k = &G->s[i];
        if (!k->used || k->host != h || !k->assoc || k->udp != udp || k->bound_port != port) continue;
        if (k->assoc_general || (k->peer_ip == pip && k->peer_port == pport)) return 0;
    }
    return 1;
}
static uint16_t random_free_port(int32_t h, int udp, uint32_t pip, uint16_t pport) {   /* host.c:1072-1110 */
    ohost_t* H = &G->h[h];
    for (int i = 0; i < 10; i++) { uint16_t p = random_port(H); if (port_free(h, udp, p, pip, pport)) return p; }
    const uint16_t start = random_port(H);
    uint16_t next = start == 65535 ? 10000 : (uint16_t)(start + 1);
    while (next != start) {
        if (port_free(h, udp, next, pip, pport)) return next;
        next = next == 65535 ? 10000 : (uint16_t)(next + 1);
    }
    return 0;
}
static int tcp_connect_error(osock* k) {   /* tcp.c:1367-1390 */
    if (k->error & TE_CONNECTION_RESET) {
        k->flags |= TF_RESET_SIGNALED;
        return (k->flags & TF_WAS_ESTABLISHED) ? ERR_ECONNRESET : ERR_ECONNREFUSED;
    } else if (k->state == TS_SYNSENT || k->state == TS_SYNRECEIVED) {
        return ERR_EALREADY;
    } else if ((k->flags & TF_EOF_RD_SIGNALED) && (k->flags & TF_EOF_WR_SIGNALED)) {
        return ERR_ENOTCONN;
    } else if (k->state != TS_CLOSED) {
        return ERR_EISCONN;
    }
    return 0;
}
static int host_connect(int32_t h, osock* k, uint32_t ip, uint16_t port) {   /* host.c:1191-1282 */
    double lat, rel;
    path(h, host_of_ip(ip), &lat, &rel);   /* topology_isRoutable */
    if (!k->bound) {
        const uint16_t bp = random_free_port(h, 0, ip, port);
        k->bound = 1; k->bound_ip = G->h[h].ip; k->bound_port = bp;
        k->peer_ip = ip; k->peer_port = port;
        k->assoc = 1; k->assoc_general = 0;
    }
    /* tcp_connectToPeer (tcp.c:1462-1484) */
    const int err = tcp_connect_error(k);
    if (err == ERR_EISCONN && !(k->flags & TF_CONNECT_SIGNALED)) { k->flags |= TF_CONNECT_SIGNALED; return 0; }
    else if (err) return err;
    tcp_send_control(k, F_SYN);
    tcp_set_state(k, TS_SYNSENT);
    return ERR_EINPROGRESS;
}
static void tcp_eof_signalled(osock* k, uint32_t f) {   /* tcp.c:2113-2124 */
    k->flags |= f;
    if ((k->flags & TF_EOF_RD_SIGNALED) && (k->flags & TF_EOF_WR_SIGNALED)) {
        sock_status(k, DS_CLOSED, 1);
        sock_status(k, DS_ACTIVE, 0);
    }
}
static int64_t tcp_send_user(osock* k, uint64_t n) {   /* tcp.c:2126-2178 */
    if (k->error & TE_SEND_EOF) {
        if (k->flags & TF_EOF_WR_SIGNALED) return -2;
        tcp_eof_signalled(k, TF_EOF_WR_SIGNALED);
        return -3;
    }
    const uint64_t acceptable = n < 65535 ? n : 65535;
    const uint64_t space = space_out(k);
    uint64_t remaining = acceptable < space ? acceptable : space;
    uint64_t copied = 0;
    while (remaining > 0) {
        const uint64_t cl = remaining < MSS ? remaining : MSS;
        opkt* p = tcp_create_packet(k, F_ACK, (uint32_t)cl);
        if (cl > 0) k->snd.end++;
        tcp_buffer_out(k, p);
        pkt_unref(p);
        remaining -= cl;
        copied += cl;
    }
    tcp_flush(k);
    return copied == 0 ? -1 : (int64_t)copied;
}
static int host_send(int32_t h, osock* k, uint64_t n, uint64_t* copied) {   /* host.c:1466-1555 */
    (void)h;
    if (k->status & DS_CLOSED) return 9;
    const int err = tcp_connect_error(k);
    if (err != ERR_EISCONN) {
        if (err == ERR_EALREADY) { sock_status(k, DS_WRITABLE, 0); return ERR_EWOULDBLOCK; }
        return err;
    }
    const int64_t r = tcp_send_user(k, n);
    if (r > 0) *copied = (uint64_t)r;
    else if (r == -2) return ERR_ENOTCONN;
    else if (r == -3) return ERR_EPIPE;
    else if (r < 0) return ERR_EWOULDBLOCK;
    return 0;
}
static int64_t tcp_receive_user(osock* k, uint64_t n) {   /* tcp.c:2192-2327 */
    tcp_flush(k);
    uint64_t remaining = n, total = 0;
    if (remaining > 0 && k->partial) {
        const uint32_t pb = k->partial->len - k->partial_off;
        const uint64_t cl = pb < remaining ? pb : remaining;
        total += cl; remaining -= cl;
        if (cl >= pb) {
            pkt_status(k->partial, S_RCV_SOCKET_DELIVERED);
            pkt_unref(k->partial);
            k->partial = NULL;
            k->partial_off = 0;
        } else {
            k->partial_off += (uint32_t)cl;
        }
    }
    while (remaining > 0) {
        opkt* p = sock_remove_input(k);
        if (!p) break;
        const uint64_t cl = p->len < remaining ? p->len : remaining;
        total += cl; remaining -= cl;
        if (cl < p->len) { k->partial = p; k->partial_off = (uint32_t)cl; break; }
        pkt_status(p, S_RCV_SOCKET_DELIVERED);
        pkt_unref(p);
    }
    if (k->in_len > 0 || k->partial) {
        sock_status(k, DS_READABLE, 1);
    } else if (k->unordered_len == 0 && (k->error & TE_RECEIVE_EOF)) {
        if (total > 0) {
            sock_status(k, DS_READABLE, 1);
        } else {
            if (k->flags & TF_EOF_RD_SIGNALED) return -2;
            tcp_eof_signalled(k, TF_EOF_RD_SIGNALED);
            return 0;
        }
    } else {
        sock_status(k, DS_READABLE, 0);
    }
    if (k->at.enabled) tcp_autotune_rcv(k, (uint32_t)total);
    tcp_update_rcv_window(k);
    if (k->rcv.window > k->snd.last_window && !k->rcv.winupd_pending) {
        sched_task(G, (uint32_t)k->host, 1, K_WINUPD, sidx(k));
        k->rcv.winupd_pending = 1;
    }
    return total == 0 ? -1 : (int64_t)total;
}
static int host_receive(osock* k, uint64_t n, uint64_t* copied) {   /* host.c:1557-1604 */
    const int64_t r = tcp_receive_user(k, n);
    if (r > 0) *copied = (uint64_t)r;
    else if (r == -2) return ERR_ENOTCONN;
    else if (r < 0) return ERR_EWOULDBLOCK;
    return 0;
}
static void tcp_close(osock* k) {   /* descriptor_close + tcp_close (tcp.c:2363-2408) */
    sock_status(k, DS_CLOSED, 1);
    k->flags |= TF_LOCAL_CLOSED_WR | TF_LOCAL_CLOSED_RD;
    sock_status(k, DS_ACTIVE, 0);
    switch (k->state) {
    case TS_LISTEN:
    case TS_SYNSENT: tcp_set_state(k, TS_CLOSED); return;
    case TS_SYNRECEIVED:
    case TS_ESTABLISHED:
    case TS_CLOSEWAIT:
        if (tcp_out_len(k) == 0) tcp_send_shutdown_fin(k);
        else k->flags |= TF_SHOULD_SEND_WR_FIN;
        break;
    case TS_FINWAIT1: case TS_FINWAIT2: case TS_CLOSING: case TS_TIMEWAIT: case TS_LASTACK: return;
    default: tcp_set_state(k, TS_CLOSED); return;
    }
}

/* ------------------------------------------------------------ the echo application
 * (test_tcp.c:713-810, ref_loop.c app 1) */
enum { T_SRV_START, T_SRV_ACCEPT, T_SRV_RECV, T_SRV_SEND, T_CLI_START, T_CLI_CONNECT, T_CLI_SEND, T_CLI_RECV,
       T_DONE };
static void app_wait(oproc* pr, int32_t fd, uint32_t events) {   /* epoll_ctl ADD (epoll.c:411-433) */
    pr->wait_fd = fd;
    pr->wait_events = events;
    G->s[fd].proc = pr->index;
    ep_status_changed(pr);
}
static void app_run(oproc* pr) {
    const int32_t h = pr->host;
    const uint32_t N = G->cfg->tcp_bytes;
    for (;;) {
        switch (pr->step) {
        case T_SRV_START: {
            const int32_t li = sock_new(h);
            osock* l = &G->s[li];
            pr->listenfd = li;
            /* bind INADDR_ANY:0 (host.c:1111-1189): a random free port */
            l->bound = 1; l->bound_ip = 0; l->bound_port = random_free_port(h, 0, 0, 0);
            l->assoc = 1; l->assoc_general = 1;
            /* listen (host.c:1284-1335, tcp.c:1486-1494) */
            l->server = 1;
            tcp_set_state(l, TS_LISTEN);
            pr->step = T_SRV_ACCEPT;
            break;
        }
        case T_SRV_ACCEPT: {   /* tcp_acceptServerPeer (tcp.c:1496-1558) */
            osock* l = &G->s[pr->listenfd];
            if (l->pending.n == 0) {
                sock_status(l, DS_READABLE, 0);
                app_wait(pr, pr->listenfd, 1);
                return;
            }
            const int32_t ci = l->pending.v[0];
            memmove(l->pending.v, l->pending.v + 1, (l->pending.n - 1) * sizeof(int32_t));
            l->pending.n--;
            osock* c = &G->s[ci];
            c->child_state = 3;
            sock_status(c, DS_ACTIVE | DS_WRITABLE, 1);
            sock_status(l, DS_READABLE, l->pending.n > 0);
            pr->fd = ci;
            pr->done = 0;
            pr->step = T_SRV_RECV;
            break;
        }
        case T_SRV_RECV:
        case T_CLI_RECV: {
            while (pr->done < N) {
                uint64_t n = 0;
                const int rc = host_receive(&G->s[pr->fd], N - pr->done, &n);
                if (rc == ERR_EWOULDBLOCK) { app_wait(pr, pr->fd, 1); return; }
                if (rc != 0 || n == 0) break;
                pr->done += (uint32_t)n;
            }
            if (pr->step == T_SRV_RECV) { pr->done = 0; pr->step = T_SRV_SEND; }
            else { tcp_close(&G->s[pr->fd]); pr->step = T_DONE; }
            break;
        }
        case T_SRV_SEND:
        case T_CLI_SEND: {
            while (pr->done < N) {
                uint64_t n = 0;
                const int rc = host_send(h, &G->s[pr->fd], N - pr->done, &n);
                if (rc == ERR_EWOULDBLOCK) { app_wait(pr, pr->fd, 4); return; }
                if (rc != 0 || n == 0) break;
                pr->done += (uint32_t)n;
            }
            if (pr->step == T_SRV_SEND) {
                tcp_close(&G->s[pr->fd]);
                tcp_close(&G->s[pr->listenfd]);
                pr->step = T_DONE;
            } else {
                pr->done = 0;
                pr->step = T_CLI_RECV;
            }
            break;
        }
        case T_CLI_START: {
            for (uint32_t i = 0; i < N; i++) (void)o_rand_r(&G->h[h].rng);   /* _fillcharbuf: rand() */
            pr->fd = sock_new(h);
            pr->step = T_CLI_CONNECT;
            break;
        }
        case T_CLI_CONNECT: {
            const oproc* sp = &G->p[pr->peer];
            if (sp->listenfd < 0) { pr->step = T_DONE; return; }
            const uint32_t ip = G->h[sp->host].ip;
            const uint16_t port = G->s[sp->listenfd].bound_port;
            const int rc = host_connect(h, &G->s[pr->fd], ip, port);
            if (rc == ERR_EINPROGRESS || rc == ERR_EALREADY) { app_wait(pr, pr->fd, 4); return; }
            if (rc != 0 && rc != ERR_EISCONN) { pr->step = T_DONE; return; }
            pr->done = 0;
            pr->step = T_CLI_SEND;
            break;
        }
        default:
            return;
        }
    }
}
static void app_continue(oproc* pr) {   /* process_continue on an epoll notification */
    if (!watch_ready(pr)) return;   /* epoll_wait collects nothing */
    /* the events are collected (epoll_getEvents), then the watch is removed
     * (EPOLL_CTL_DEL) */
    if (pr->wait_fd >= 0) G->s[pr->wait_fd].proc = -1;
    pr->wait_fd = -1;
    pr->ep_ready = 0;
    pr->ep_readable = 0;
    app_run(pr);
}

/* ------------------------------------------------------------ datagram sockets (udp.c, host.c) */
static int32_t udp_sock_new(int32_t h) {   /* host_createDescriptor(DT_UDPSOCKET) -> udp_new (udp.c:211-223) */
    const int32_t si = sock_new(h);
    osock* k = &G->s[si];
    k->udp = 1;
    k->status = DS_ACTIVE | DS_WRITABLE;
    return si;
}
/* host_sendUserData (host.c:1466-1555): the implicit bind (:1514-1525), then
 * udp_sendUserData (udp.c:75-142): one packet into the output buffer */
static int udp_send_user(int32_t h, int32_t si, uint32_t n, uint32_t ip, uint16_t port) {
    osock* k = &G->s[si];
    if (k->status & DS_CLOSED) return 9;
    if (!k->bound) {
        const uint16_t bp = random_free_port(h, 1, 0, 0);
        k->bound = 1; k->bound_ip = G->h[h].ip; k->bound_port = bp;
        k->peer_ip = 0; k->peer_port = 0;
        k->assoc = 1; k->assoc_general = 1;
    }
    if (out_space(k) < n) return ERR_EWOULDBLOCK;
    opkt* p = pkt_new((uint32_t)h, n);
    p->udp = 1;
    p->sip = k->bound_ip ? k->bound_ip : G->h[h].ip;
    p->sport = k->bound_port; p->dip = ip; p->dport = port;
    pkt_status(p, S_SND_CREATED);
    sock_add_output(k, p);
    return 0;
}
/* a closed datagram socket with nothing left to send: released */
static void udp_release(osock* k) {
    if (!k->udp || !(k->status & DS_CLOSED) || k->out.n || k->outctl.n) return;
    while (k->in.n) pkt_unref(fq_pop(&k->in));
    free(k->in.p); free(k->out.p); free(k->outctl.p);
    memset(k, 0, sizeof(*k));   /* used = 0 */
}
static void udp_close(int32_t si) {   /* descriptor_close -> udp_close -> host_closeDescriptor (host.c:768-771) */
    osock* k = &G->s[si];
    sock_status(k, DS_CLOSED, 1);
    k->assoc = 0; k->assoc_general = 0;
    udp_release(k);
}
/* the datagram application (oracle/ref_harness/ref_loop.c udp_send / udp_start /
 * udp_continue, over test_phold.c's calls) */
static void udp_app_send(oproc* pr, uint32_t rip, uint16_t rport) {
    const int32_t h = pr->host;
    const uint32_t* a = G->cfg->app_spec + 4u * (uint32_t)pr->app;
    uint32_t ip;
    uint16_t port = UDP_PORT;
    if (a[1] == 0) {   /* _phold_chooseNode (test_phold.c:160-178): the first host whose weight reaches the draw */
        const double r = o_next_double(&G->h[h].rng);
        const double* cum = G->cfg->dest_cum;
        if (G->cfg->host_class && G->cfg->n_classes > 1) cum += (size_t)G->cfg->host_class[h] * (size_t)G->cfg->n_hosts;
        int32_t chosen = -1;
        for (int32_t i = 0; i < G->cfg->n_hosts; i++)
            if (cum[i] >= r) { chosen = i; break; }
        if (chosen < 0) return;
        ip = G->h[chosen].ip;
    } else if (a[1] == 1) {
        ip = G->h[G->cfg->app_peer[h]].ip;
    } else {
        ip = rip;
        port = rport;
    }
    if (a[0] == 0) {   /* a socket per datagram: socket, sendto, close */
        const int32_t si = udp_sock_new(h);
        (void)udp_send_user(h, si, G->cfg->udp_payload, ip, port);
        udp_close(si);
    } else {
        (void)udp_send_user(h, pr->listenfd, G->cfg->udp_payload, ip, port);
    }
}
static void udp_app_start(oproc* pr) {
    const int32_t h = pr->host;
    const uint32_t* a = G->cfg->app_spec + 4u * (uint32_t)pr->app;
    const int32_t li = udp_sock_new(h);
    pr->listenfd = li;
    if (a[0] != 1 && port_free(h, 1, UDP_PORT, 0, 0)) {   /* bind INADDR_ANY:8998 */
        osock* l = &G->s[li];
        l->bound = 1; l->bound_ip = 0; l->bound_port = UDP_PORT;
        l->assoc = 1; l->assoc_general = 1;
    }
    app_wait(pr, li, 1);   /* epoll_ctl ADD, EPOLLIN: kept for the process's life */
    for (uint32_t i = 0; i < a[2]; i++) udp_app_send(pr, 0, 0);
}
static void udp_app_continue(oproc* pr) {   /* every datagram, while epoll_wait reports the socket readable */
    const uint32_t* a = G->cfg->app_spec + 4u * (uint32_t)pr->app;
    while (watch_ready(pr)) {
        for (;;) {
            opkt* p = sock_remove_input(&G->s[pr->listenfd]);   /* udp_receiveUserData (udp.c:144-178) */
            if (!p) break;
            pkt_status(p, S_RCV_SOCKET_DELIVERED);
            const uint32_t ip = p->sip;
            const uint16_t port = p->sport;
            pkt_unref(p);
            if (a[3]) udp_app_send(pr, ip, port);
        }
    }
}

/* ------------------------------------------------------------ events */
static void execute(const tev* e) {
    const int32_t h = (int32_t)e->dst;
    G->active = h;
    switch (e->kind) {
    case K_HEARTBEAT: {
        const uint64_t hb = G->cfg->heartbeat_interval;
        sched_task(G, (uint32_t)h, hb, K_HEARTBEAT, -1);
        break;
    }
    case K_REFILL: refill_cb(h); break;
    case K_REFILL_LO: break;
    case K_PSTART: {   /* process start task (process.c:1055-1195) */
        oproc* pr = &G->p[e->obj];
        if (pr->running) break;
        pr->running = 1;
        if (pr->app >= 0) { udp_app_start(pr); break; }
        pr->step = pr->peer < 0 ? T_SRV_START : T_CLI_START;
        app_run(pr);
        break;
    }
    case K_NOTIFY: {   /* _epoll_tryNotify (epoll.c:638-683) */
        oproc* pr = &G->p[e->obj];
        pr->ep_scheduled = 0;
        if (!pr->running) break;
        if (pr->ep_ready) {
            pr->ep_notifying = 1;
            if (pr->app >= 0) {   /* the datagram application keeps its watch */
                if (watch_ready(pr)) { pr->ep_ready = 0; pr->ep_readable = 0; udp_app_continue(pr); }
            } else {
                app_continue(pr);
            }
            pr->ep_notifying = 0;
            pr->ep_ready = watch_ready(pr);
            pr->ep_readable = pr->ep_ready;
            if (pr->ep_readable) ep_schedule(pr);
        }
        break;
    }
    case K_DELIVER: {   /* _worker_runDeliverPacketTask -> router_enqueue (router.c:104-122) */
        opkt* p = e->pkt;
        ohost_t* H = &G->h[h];
        const int was_empty = H->codel.count == 0;
        if (G->npool == G->cappool) { G->cappool = G->cappool ? 2 * G->cappool : 1024; G->pool = realloc(G->pool, G->cappool * sizeof(opkt*)); }
        const uint32_t id = G->npool++;
        G->pool[id] = p;
        o_codel_enqueue(&H->codel, G->now, p->len + hdr_of(p), id, e->src);
        pkt_ref(p);
        pkt_status(p, S_ROUTER_ENQUEUED);
        if (was_empty) if_receive_packets(h);
        /* the task's reference goes after the event (host -1: no active host) */
        G->active = -1;
        pkt_unref(p);
        break;
    }
    case K_LOCAL: {   /* _networkinterface_receivePacket as the loopback task (network_interface.c:551-554) */
        if_receive_packet(h, e->pkt);
        G->active = -1;   /* the task's reference goes after the event, as K_DELIVER's */
        pkt_unref(e->pkt);
        break;
    }
    case K_DELACK: {   /* _tcp_sendACKTaskCallback (tcp.c:1767-1774) */
        osock* k = &G->s[e->obj];
        k->snd.delack_sched = 0;
        if (k->snd.delack_counter > 0) { tcp_send_control(k, F_ACK); k->snd.delack_counter = 0; }
        break;
    }
    case K_RTO: {   /* _tcp_runRetransmitTimerExpiredTask (tcp.c:1280-1333) */
        osock* k = &G->s[e->obj];
        uint64_t* x = pq_pop(&k->rtx.timers);
        free(x);
        if (k->state == TS_CLOSED) { k->rtx.desired = 0; tcp_clear_retransmit(k, 0xffffffffu); break; }
        if (k->rtx.nq == 0) { k->rtx.desired = 0; break; }
        if (k->rtx.desired == 0) break;
        if (k->rtx.desired > G->now) { tcp_schedule_rto_if_needed(k, G->now); break; }
        k->rtx.backoff++;
        tcp_set_rto(k, k->rtx.timeout * 2);
        tcp_set_rto_timer(k, G->now);
        reno_timeout(k);
        k->rtx.tally.retx.n = 0;
        tally_mark_lost(&k->rtx.tally, k->rcv.last_ack, k->snd.highest + 1);
        tcp_flush(k);
        break;
    }
    case K_CLOSE: tcp_set_state(&G->s[e->obj], TS_CLOSED); break;   /* tcp.c:695-698 */
    case K_WINUPD: {   /* _tcp_sendWindowUpdate (tcp.c:2180-2190) */
        osock* k = &G->s[e->obj];
        tcp_send_control(k, F_ACK);
        k->rcv.winupd_pending = 0;
        break;
    }
    default: break;
    }
}

int o_tcp_run(const o_tcp_cfg* cfg, o_topo* topo, o_tcp_out* out) {
    if (!cfg || !out || cfg->n_hosts <= 0) return -1;
    T t;
    memset(&t, 0, sizeof(t));
    out->events = 0;
    G = &t;
    t.cfg = cfg;
    t.topo = topo;
    const int32_t H = cfg->n_hosts;
    t.h = calloc((size_t)H, sizeof(ohost_t));
    t.p = calloc((size_t)(cfg->n_procs > 0 ? cfg->n_procs : 1), sizeof(oproc));
    t.caps = (uint32_t)(4 * (cfg->n_procs > 0 ? cfg->n_procs : 1) + 16 + (cfg->proc_app ? 32 * H : 0));
    t.s = calloc(t.caps, sizeof(osock));
    for (int32_t i = 0; i < H; i++) {
        ohost_t* h = &t.h[i];
        h->ip = cfg->host_ip[i];
        h->rng = cfg->host_seed[i];
        h->vertex = cfg->host_vertex[i];
        h->fifo.cmp = cmp_sock;
        h->next_handle = 3;
        /* _networkinterface_setupTokenBuckets (network_interface.c:192-226) */
        h->tx_refill = cfg->bw_up_kibps[i] * 1024 / 1000;
        h->rx_refill = cfg->bw_down_kibps[i] * 1024 / 1000;
        h->tx_cap = h->tx_refill + MTU;
        h->rx_cap = h->rx_refill + MTU;
        o_codel_init(&h->codel, 64);
    }
    for (int32_t k = 0; k < cfg->n_procs; k++) {
        oproc* pr = &t.p[k];
        pr->host = cfg->proc_host[k]; pr->index = k; pr->peer = cfg->proc_peer[k]; pr->start = cfg->proc_start[k];
        pr->fd = pr->listenfd = pr->wait_fd = -1;
        pr->app = cfg->proc_app ? cfg->proc_app[k] : -1;
    }
    /* host_boot (host.c:372-390), every host at t = 0 in order */
    for (int32_t i = 0; i < H; i++) {
        t.now = 0;
        t.active = i;
        sched_task(&t, (uint32_t)i, cfg->heartbeat_interval, K_HEARTBEAT, -1);
        refill_cb(i);
        sched_task(&t, (uint32_t)i, MS, K_REFILL_LO, -1);
        for (int32_t k = 0; k < cfg->n_procs; k++)
            if (cfg->proc_host[k] == i) sched_task(&t, (uint32_t)i, cfg->proc_start[k] > 0 ? cfg->proc_start[k] : 1, K_PSTART, k);
    }
    while (t.nq) {
        tev e = q_pop(&t);
        t.now = e.time;
        execute(&e);
        out->events++;
    }
    out->lines = t.out.s;
    out->len = t.out.len;
    out->n_lines = t.out.n;
    out->next_event_id = calloc((size_t)H, sizeof(uint64_t));
    out->next_packet_id = calloc((size_t)H, sizeof(uint64_t));
    out->rng_probe = calloc((size_t)H, sizeof(uint32_t));
    for (int32_t i = 0; i < H; i++) {
        out->next_event_id[i] = t.h[i].ev_seq;
        out->next_packet_id[i] = t.h[i].pkt_seq;
        out->rng_probe[i] = (uint32_t)o_rand_r(&t.h[i].rng);
        o_codel_free(&t.h[i].codel);
    }
    /* the model's own allocations (packets still referenced are left) */
    for (uint32_t i = 0; i < t.ns; i++) {
        osock* k = &t.s[i];
        free(k->in.p); free(k->out.p); free(k->outctl.p); free(k->rtx.q);
        for (uint32_t j = 0; j < k->rtx.timers.n; j++) free(k->rtx.timers.a[j]);
        free(k->rtx.timers.a); free(k->throttled.a); free(k->unordered.a);
        free(k->snd.sacks.v); free(k->children.v); free(k->pending.v);
        free(k->rtx.tally.marked.r); free(k->rtx.tally.sacked.r); free(k->rtx.tally.retx.r);
        free(k->rtx.tally.lost.r); free(k->rtx.tally.tmp.r);
    }
    for (int32_t i = 0; i < H; i++) { free(t.h[i].fifo.a); free(t.h[i].rr); }
    free(t.s); free(t.p); free(t.h); free(t.q); free(t.pool);
    G = NULL;
    return 0;
}

void o_tcp_free(o_tcp_out* out) {
    if (!out) return;
    free(out->lines);
    free(out->next_event_id);
    free(out->next_packet_id);
    free(out->rng_probe);
    memset(out, 0, sizeof(*out));
}
