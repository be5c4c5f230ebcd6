/*
 * shd_status.c -- the reference's observability lines, made by libshdgpu from
 * what the engine records, so that a Shadow build linking the C-ABI logs what
 * the reference logs:
 *
 *   [STATUS] lines   packet_addDeliveryStatus (packet.c:647-659): every status a
 *                    UDP datagram passes through, logged as "[<STATUS>] " +
 *                    packet_toString (packet.c:518-547 header, 616-633 the
 *                    ordered status list so far), from an engine trace recorded
 *                    with SHD_QF_TRACE_STATUS;
 *   [node] lines     _tracker_logNode (tracker.c:419-465) of one host, from its
 *                    cumulative interface counters at each heartbeat
 *                    (SHD_QF_HEARTBEATS).
 *
 * Each trace kind stands for the reference calls it summarises:
 *   CREATED     udp.c:116 SND_CREATED, socket.c:405 SND_SOCKET_BUFFERED
 *   SENT        network_interface.c:545 SND_INTERFACE_SENT, worker.c:306 INET_SENT
 *   INET_DROP   network_interface.c:545, worker.c:319 INET_DROPPED
 *   LOCAL       network_interface.c:545 (the loopback shortcut, own address)
 *   ARRIVE      router.c:113 ROUTER_ENQUEUED
 *   CODEL_DROP  router_queue_codel.c:139 ROUTER_DROPPED
 *   RECV        router.c:129, network_interface.c:382, socket.c:143, socket.c:330
 *   IF_DROP     router.c:129, network_interface.c:382, network_interface.c:411
 *   READ        udp.c:158 RCV_SOCKET_DELIVERED
 * and a packet object's last reference logs PDS_DESTROYED with its list
 * (packet.c:194-201).  The Python harness (shdgpu.status_lines) is the same
 * algorithm; tests/test_status_cpu.py checks the two against each other and
 * tests/test_ref_loop_*.py this writer against the reference's own lines.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "shd_host.h"

enum {
    ST_SND_CREATED, ST_SND_SOCKET_BUFFERED, ST_SND_INTERFACE_SENT, ST_INET_SENT, ST_INET_DROPPED,
    ST_ROUTER_ENQUEUED, ST_ROUTER_DEQUEUED, ST_ROUTER_DROPPED, ST_RCV_INTERFACE_RECEIVED,
    ST_RCV_INTERFACE_DROPPED, ST_RCV_SOCKET_PROCESSED, ST_RCV_SOCKET_BUFFERED, ST_RCV_SOCKET_DELIVERED,
    ST_PDS_DESTROYED, ST_N
};
static const char* const kStName[ST_N] = {
    "SND_CREATED", "SND_SOCKET_BUFFERED", "SND_INTERFACE_SENT", "INET_SENT", "INET_DROPPED",
    "ROUTER_ENQUEUED", "ROUTER_DEQUEUED", "ROUTER_DROPPED", "RCV_INTERFACE_RECEIVED",
    "RCV_INTERFACE_DROPPED", "RCV_SOCKET_PROCESSED", "RCV_SOCKET_BUFFERED", "RCV_SOCKET_DELIVERED",
    "PDS_DESTROYED"};

/* the statuses of each trace kind (index SHD_TR_*), -1 terminated */
static const int8_t kStOf[SHD_TR_READ + 1][5] = {
    [SHD_TR_CREATED] = {ST_SND_CREATED, ST_SND_SOCKET_BUFFERED, -1},
    [SHD_TR_SENT] = {ST_SND_INTERFACE_SENT, ST_INET_SENT, -1},
    [SHD_TR_INET_DROP] = {ST_SND_INTERFACE_SENT, ST_INET_DROPPED, -1},
    [SHD_TR_LOCAL] = {ST_SND_INTERFACE_SENT, -1},
    [SHD_TR_ARRIVE] = {ST_ROUTER_ENQUEUED, -1},
    [SHD_TR_CODEL_DROP] = {ST_ROUTER_DROPPED, -1},
    [SHD_TR_RECV] = {ST_ROUTER_DEQUEUED, ST_RCV_INTERFACE_RECEIVED, ST_RCV_SOCKET_PROCESSED, ST_RCV_SOCKET_BUFFERED,
                     -1},
    [SHD_TR_IF_DROP] = {ST_ROUTER_DEQUEUED, ST_RCV_INTERFACE_RECEIVED, ST_RCV_INTERFACE_DROPPED, -1},
    [SHD_TR_READ] = {ST_RCV_SOCKET_DELIVERED, -1},
};

/* ---- growable line set ---- */
typedef struct {
    shd_lines* l;
    uint64_t cap, tcap;
    int oom;
} lbuf;

static void lb_add(lbuf* b, uint64_t t, uint32_t host, const char* s, size_t len) {
    shd_lines* l = b->l;
    if (b->oom) return;
    if (l->n + 1 >= b->cap) {
        const uint64_t c = b->cap ? 2 * b->cap : 1024;
        uint64_t* nt = realloc(l->time, c * sizeof(uint64_t));
        if (nt) l->time = nt;
        uint32_t* nh = realloc(l->host, c * sizeof(uint32_t));
        if (nh) l->host = nh;
        uint64_t* no = realloc(l->off, (c + 1) * sizeof(uint64_t));
        if (no) l->off = no;
        if (!nt || !nh || !no) { b->oom = 1; return; }
        b->cap = c;
    }
    const uint64_t at = l->off[l->n];
    if (at + len + 1 > b->tcap) {
        uint64_t c = b->tcap ? 2 * b->tcap : 65536;
        while (at + len + 1 > c) c *= 2;
        char* nx = realloc(l->text, c);
        if (!nx) { b->oom = 1; return; }
        l->text = nx;
        b->tcap = c;
    }
    memcpy(l->text + at, s, len);
    l->text[at + len] = 0;   /* kept terminated; the next line overwrites it */
    l->time[l->n] = t;
    l->host[l->n] = host;
    l->off[l->n + 1] = at + len;
    l->n++;
}

static int lb_init(lbuf* b, shd_lines** out) {
    memset(b, 0, sizeof(*b));
    b->l = calloc(1, sizeof(shd_lines));
    if (!b->l) return SHD_ENOMEM;
    b->l->off = calloc(1, sizeof(uint64_t));
    if (!b->l->off) { free(b->l); return SHD_ENOMEM; }
    *out = NULL;
    return SHD_OK;
}

static int lb_done(lbuf* b, shd_lines** out) {
    if (b->oom) { shd_lines_free(b->l); return SHD_ENOMEM; }
    if (!b->l->text) {
        b->l->text = calloc(1, 1);
        if (!b->l->text) { shd_lines_free(b->l); return SHD_ENOMEM; }
    }
    *out = b->l;
    return SHD_OK;
}

void shd_lines_free(shd_lines* l) {
    if (!l) return;
    free(l->time);
    free(l->host);
    free(l->off);
    free(l->text);
    free(l);
}

/* ---- per-datagram records, keyed by (source host, packet id) ---- */
#define HIST_MAX 24
typedef struct {
    uint64_t key;         /* (host << 32) | pkt; ~0: empty slot */
    uint64_t created_at;  /* CREATED time, ~0 if none */
    int64_t send_i;       /* the sender record (SENT / INET_DROP / LOCAL) following its creation, or -1 */
    uint32_t port, dst;   /* the bind's port draw; the destination host (~0: none) */
    uint8_t local, arrived, nh, pad;
    uint8_t hist[HIST_MAX];
} dgram;

typedef struct {
    dgram* t;
    uint64_t mask;
} dmap;

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
static dgram* dm_get(dmap* m, uint64_t key, int create) {
    uint64_t i = mix64(key) & m->mask;
    for (;;) {
        dgram* d = &m->t[i];
        if (d->key == key) return d;
        if (d->key == ~0ull) {
            if (!create) return NULL;
            memset(d, 0, sizeof(*d));
            d->key = key;
            d->created_at = ~0ull;
            d->send_i = -1;
            d->dst = 0xFFFFFFFFu;
            return d;
        }
        i = (i + 1) & m->mask;
    }
}
static uint64_t dkey(uint32_t h, uint32_t pkt) { return ((uint64_t)h << 32) | pkt; }

/* per-host FIFO of datagrams buffered in the socket (their keys) */
typedef struct {
    uint64_t* q;
    uint32_t head, n, cap;
} fifo;

static int fifo_push(fifo* f, uint64_t k) {
    if (f->head + f->n == f->cap) {
        if (f->head) {
            memmove(f->q, f->q + f->head, f->n * sizeof(uint64_t));
            f->head = 0;
        } else {
            const uint32_t c = f->cap ? 2 * f->cap : 8;
            uint64_t* q = realloc(f->q, c * sizeof(uint64_t));
            if (!q) return SHD_ENOMEM;
            f->q = q;
            f->cap = c;
        }
    }
    f->q[f->head + f->n++] = k;
    return SHD_OK;
}

typedef struct {
    const shd_trace_rec* r;
    uint64_t i;
} srec;
static int srec_cmp(const void* a, const void* b) {
    const srec* x = a;
    const srec* y = b;
    if (x->r->time != y->r->time) return x->r->time < y->r->time ? -1 : 1;
    if (x->r->host != y->r->host) return x->r->host < y->r->host ? -1 : 1;
    return x->i < y->i ? -1 : x->i > y->i;
}

static int ip_str(char* o, uint32_t ip) {
    return sprintf(o, "%u.%u.%u.%u", (ip >> 24) & 255u, (ip >> 16) & 255u, (ip >> 8) & 255u, ip & 255u);
}

typedef struct {
    lbuf* b;
    dmap* m;
    const uint32_t* ips;
    const uint32_t* ids;
    uint32_t nh, payload, lport;
    const uint32_t* dport;   /* [nh] the port a datagram to host h is addressed to */
    char* line;
} wctx;

/* "[<name>] packetID=<id>:<pkt> <src>:<port> -> <dst>:<lport> bytes=<n> status=<list>" */
static void put_line(wctx* w, uint64_t t, uint32_t at, const dgram* d, int name) {
    const uint32_t src = (uint32_t)(d->key >> 32), pkt = (uint32_t)d->key;
    char* o = w->line;
    o += sprintf(o, "[%s] packetID=%u:%u ", kStName[name], w->ids ? w->ids[src] : src + 1, pkt);
    o += ip_str(o, w->ips[src]);
    o += sprintf(o, ":%u -> ", d->port);
    const int known = d->dst != 0xFFFFFFFFu && d->dst < w->nh;
    if (known) o += ip_str(o, w->ips[d->dst]);
    else *o++ = '?';
    o += sprintf(o, ":%u bytes=%u status=", known ? w->dport[d->dst] : w->lport, w->payload);
    for (int k = 0; k < d->nh; k++) {
        if (k) *o++ = ',';
        const char* s = kStName[d->hist[k]];
        const size_t n = strlen(s);
        memcpy(o, s, n);
        o += n;
    }
    lb_add(w->b, t, at, w->line, (size_t)(o - w->line));
}

static void emit(wctx* w, uint64_t t, uint32_t at, dgram* d, const int8_t* names) {
    for (; *names >= 0; names++) {
        if (d->nh < HIST_MAX) d->hist[d->nh++] = (uint8_t)*names;
        else w->b->oom = 1;
        put_line(w, t, at, d, *names);
    }
}
/* the last reference of a packet object; a sent datagram's original is
 * released after its copy when scheduler_push dropped the copy's event
 * (worker.c:306-313, network_interface.c:577, scheduler.c:346-349) */
static void destroyed(wctx* w, uint64_t t, uint32_t at, dgram* d, int copy_dropped) {
    if (d->nh < HIST_MAX) d->hist[d->nh] = ST_PDS_DESTROYED;
    else { w->b->oom = 1; return; }
    d->nh++;
    for (int k = 0; k < (copy_dropped ? 2 : 1); k++) put_line(w, t, at, d, ST_PDS_DESTROYED);
    d->nh--;
}
static void send_side(wctx* w, uint64_t t, uint32_t h, dgram* d, uint32_t kind) {
    emit(w, t, h, d, kStOf[kind]);
    if (kind == SHD_TR_SENT) destroyed(w, t, h, d, !d->arrived);
    else if (kind == SHD_TR_INET_DROP) destroyed(w, t, h, d, 0);
}

int shd_status_lines(const shd_trace_rec* tr, uint64_t n, const uint32_t* ips, const uint32_t* host_ids,
                     uint32_t n_hosts, uint32_t payload, uint32_t listen_port, const int32_t* app_peer,
                     shd_lines** out) {
    if (!out || (n && !tr) || !ips || !n_hosts) return SHD_EINVAL;
    for (uint64_t i = 0; i < n; i++) {
        if (tr[i].host >= n_hosts || tr[i].kind < SHD_TR_SENT || tr[i].kind > SHD_TR_READ) return SHD_EINVAL;
        /* every kind but the application's two names the other host in `peer`
         * (the destination, or the datagram's source), which indexes ips[] */
        if (tr[i].kind <= SHD_TR_LOCAL && tr[i].peer >= n_hosts) return SHD_EINVAL;
    }
    lbuf b;
    int rc = lb_init(&b, out);
    if (rc) return rc;
    srec* s = malloc((n ? n : 1) * sizeof(srec));
    dmap m = {0};
    uint64_t cap = 64;
    while (cap < 2 * n + 64) cap *= 2;
    m.t = malloc(cap * sizeof(dgram));
    m.mask = cap - 1;
    fifo* inbox = calloc(n_hosts, sizeof(fifo));
    char* line = malloc(512 + HIST_MAX * 32);
    uint32_t* dport = malloc(n_hosts * sizeof(uint32_t));   /* the port datagrams to host h go to */
    if (!s || !m.t || !inbox || !line || !dport) { rc = SHD_ENOMEM; goto out; }
    for (uint32_t h = 0; h < n_hosts; h++) dport[h] = listen_port;
    if (app_peer)   /* UDP echo: a client's socket port, from its own datagrams' source port */
        for (uint64_t i = 0; i < n; i++)
            if (tr[i].kind == SHD_TR_CREATED && app_peer[tr[i].host] >= 0) dport[tr[i].host] = (uint32_t)(tr[i].seq & 0xFFFF);
    for (uint64_t i = 0; i < cap; i++) m.t[i].key = ~0ull;
    for (uint64_t i = 0; i < n; i++) { s[i].r = &tr[i]; s[i].i = i; }
    qsort(s, n, sizeof(srec), srec_cmp);   /* by (time, host), records of one host in trace order */
    /* what the sender's records say of each datagram */
    for (uint64_t i = 0; i < n; i++) {
        const shd_trace_rec* r = s[i].r;
        if (r->kind == SHD_TR_CREATED) {
            dgram* d = dm_get(&m, dkey(r->host, r->pkt), 1);
            d->port = (uint32_t)r->seq;
            d->created_at = r->time;
        } else if (r->kind == SHD_TR_SENT || r->kind == SHD_TR_INET_DROP || r->kind == SHD_TR_LOCAL) {
            dgram* d = dm_get(&m, dkey(r->host, r->pkt), 1);
            d->dst = r->peer;
            if (r->kind == SHD_TR_LOCAL) d->local = 1;
        } else if (r->kind == SHD_TR_ARRIVE) {
            dm_get(&m, dkey(r->peer, r->pkt), 1)->arrived = 1;
        }
    }
    /* a datagram sent in the instant it was created follows its creation at
     * once (sendto -> networkinterface_wantsSend -> _networkinterface_sendPackets) */
    for (uint64_t i = 0; i < n; i++) {
        const shd_trace_rec* r = s[i].r;
        if (r->kind == SHD_TR_SENT || r->kind == SHD_TR_INET_DROP || r->kind == SHD_TR_LOCAL) {
            dgram* d = dm_get(&m, dkey(r->host, r->pkt), 0);
            if (d->created_at == r->time) d->send_i = (int64_t)i;
        }
    }
    wctx w = {&b, &m, ips, host_ids, n_hosts, payload, listen_port, dport, line};
    for (uint64_t i = 0; i < n && !b.oom; i++) {
        const shd_trace_rec* r = s[i].r;
        const uint32_t k = r->kind, h = r->host;
        const uint64_t t = r->time;
        if (k == SHD_TR_SENT || k == SHD_TR_INET_DROP || k == SHD_TR_LOCAL) {
            dgram* d = dm_get(&m, dkey(h, r->pkt), 0);
            if (d->send_i == (int64_t)i) continue;   /* emitted with its creation */
            send_side(&w, t, h, d, k);
        } else if (k == SHD_TR_CREATED) {
            dgram* d = dm_get(&m, dkey(h, r->pkt), 0);
            emit(&w, t, h, d, kStOf[k]);
            if (d->send_i >= 0) send_side(&w, t, h, d, s[d->send_i].r->kind);
        } else if (k == SHD_TR_READ) {
            fifo* f = &inbox[h];
            if (f->n) {
                dgram* d = dm_get(&m, f->q[f->head], 0);
                f->head++;
                f->n--;
                emit(&w, t, h, d, kStOf[k]);
                destroyed(&w, t, h, d, 0);   /* the socket's reference, udp.c:169 */
            }
        } else {   /* the receiver's records name the datagram by (source, pkt) */
            const uint64_t key = dkey(r->peer, r->pkt);
            dgram* d = dm_get(&m, key, 1);
            const int8_t* names = kStOf[k];
            if ((k == SHD_TR_RECV || k == SHD_TR_IF_DROP) && d->local) names++;   /* no router on the loopback */
            emit(&w, t, h, d, names);
            if (k == SHD_TR_RECV) {
                if (fifo_push(&inbox[h], key)) b.oom = 1;
            } else if (k == SHD_TR_CODEL_DROP || k == SHD_TR_IF_DROP) {
                /* the queue's reference (router_queue_codel.c), or the
                 * interface's (network_interface.c:446) / the local task's (:553) */
                destroyed(&w, t, h, d, 0);
            }
        }
    }
out:
    if (inbox)
        for (uint32_t h = 0; h < n_hosts; h++) free(inbox[h].q);
    free(inbox);
    free(line);
    free(dport);
    free(m.t);
    free(s);
    if (rc) { shd_lines_free(b.l); return rc; }
    return lb_done(&b, out);
}

/* ---- [shadow-heartbeat] [node] lines (tracker.c:419-465) ---- */
#define SHD_HEADER_UDP 42u   /* definitions.h:176-183 */

/* _tracker_getCounterString (tracker.c:399-417) for `packets` first-sent UDP
 * datagrams of `payload` bytes (_tracker_updateCounters, tracker.c:183-214:
 * payload > 0 is data, 0 control); no retransmissions */
static int counter_str(char* o, uint64_t packets, uint32_t payload) {
    const uint64_t h = packets * SHD_HEADER_UDP, p = packets * payload;
    if (payload > 0)
        return sprintf(o, "%llu,%llu,0,0,0,0,%llu,%llu,%llu,0,0,0", (unsigned long long)packets,
                       (unsigned long long)(h + p), (unsigned long long)packets, (unsigned long long)h,
                       (unsigned long long)p);
    return sprintf(o, "%llu,%llu,%llu,%llu,0,0,0,0,0,0,0,0", (unsigned long long)packets, (unsigned long long)h,
                   (unsigned long long)packets, (unsigned long long)h);
}

static const char kNodeHeader[] =
    "[shadow-heartbeat] [node-header] interval-seconds,recv-bytes,send-bytes,cpu-percent,"
    "delayed-count,avgdelay-milliseconds;inbound-localhost-counters;outbound-localhost-counters;"
    "inbound-remote-counters;outbound-remote-counters where counters are: "
    "packets-total,bytes-total,packets-control,bytes-control-header,"
    "packets-control-retrans,bytes-control-header-retrans,"
    "packets-data,bytes-data-header,bytes-data-payload,"
    "packets-data-retrans,bytes-data-header-retrans,bytes-data-payload-retrans";

int shd_node_lines(const uint32_t* snaps, uint64_t k, uint64_t interval_ns, uint32_t payload, uint32_t host,
                   shd_lines** out) {
    if (!out || (k && !snaps) || !interval_ns) return SHD_EINVAL;
    lbuf b;
    int rc = lb_init(&b, out);
    if (rc) return rc;
    const unsigned secs = (unsigned)(interval_ns / 1000000000ull);
    char zero[128], ci[128], co[128], line[1024];
    counter_str(zero, 0, payload);
    /* tracker_new runs the first heartbeat inline at boot (tracker.c:141): the
     * header, then an all-zero line, before the K periodic ones */
    lb_add(&b, 0, host, kNodeHeader, sizeof(kNodeHeader) - 1);
    int len = sprintf(line, "[shadow-heartbeat] [node] %u,%d,%d,%f,%d,%f;%s;%s;%s;%s", secs, 0, 0, 0.0, 0, 0.0, zero,
                      zero, zero, zero);
    lb_add(&b, 0, host, line, (size_t)len);
    uint32_t pin = 0, pout = 0;
    for (uint64_t j = 0; j < k; j++) {
        /* cumulative uint32 device counters (wrap after 2^32 packets); the
         * reference's are per interval, cleared at every heartbeat (tracker.c:584-593) */
        const uint32_t din = snaps[2 * j] - pin, dout = snaps[2 * j + 1] - pout;
        pin = snaps[2 * j];
        pout = snaps[2 * j + 1];
        const uint64_t rb = (uint64_t)din * (SHD_HEADER_UDP + payload), sb = (uint64_t)dout * (SHD_HEADER_UDP + payload);
        counter_str(ci, din, payload);
        counter_str(co, dout, payload);
        /* the loopback shortcut keeps the host's own address
         * (network_interface.c:548-555): every packet counts as remote; the
         * CPU model is off (cpu-percent 0, no delays) */
        len = sprintf(line, "[shadow-heartbeat] [node] %u,%llu,%llu,%f,%d,%f;%s;%s;%s;%s", secs,
                      (unsigned long long)rb, (unsigned long long)sb, 0.0, 0, 0.0, zero, zero, ci, co);
        lb_add(&b, (j + 1) * interval_ns, host, line, (size_t)len);
    }
    return lb_done(&b, out);
}

/* _tracker_getCounterString (tracker.c:399-417) from the ten counters of one
 * direction (shdtcp.h's order): the totals, then the ten */
static int counters_str(char* o, const uint64_t* t) {
    const unsigned long long pk = t[0] + t[2] + t[4] + t[7], by = t[1] + t[3] + t[5] + t[6] + t[8] + t[9];
    return sprintf(o, "%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu", pk, by,
                   (unsigned long long)t[0], (unsigned long long)t[1], (unsigned long long)t[2],
                   (unsigned long long)t[3], (unsigned long long)t[4], (unsigned long long)t[5],
                   (unsigned long long)t[6], (unsigned long long)t[7], (unsigned long long)t[8],
                   (unsigned long long)t[9]);
}

int shd_tracker_node_lines(const uint64_t* counters, uint64_t k, uint64_t interval_ns, uint32_t host,
                           shd_lines** out) {
    if (!out || (k && !counters) || !interval_ns) return SHD_EINVAL;
    lbuf b;
    int rc = lb_init(&b, out);
    if (rc) return rc;
    const unsigned secs = (unsigned)(interval_ns / 1000000000ull);
    static const uint64_t kZero[10] = {0};
    char zero[256], ci[256], co[256], line[1400];
    counters_str(zero, kZero);
    lb_add(&b, 0, host, kNodeHeader, sizeof(kNodeHeader) - 1);
    int len = sprintf(line, "[shadow-heartbeat] [node] %u,%d,%d,%f,%d,%f;%s;%s;%s;%s", secs, 0, 0, 0.0, 0, 0.0, zero,
                      zero, zero, zero);
    lb_add(&b, 0, host, line, (size_t)len);
    for (uint64_t j = 0; j < k; j++) {
        const uint64_t* in = counters + 20 * j;
        const uint64_t* ou = in + 10;
        const unsigned long long rb = in[1] + in[3] + in[5] + in[6] + in[8] + in[9];
        const unsigned long long sb = ou[1] + ou[3] + ou[5] + ou[6] + ou[8] + ou[9];
        counters_str(ci, in);
        counters_str(co, ou);
        /* the CPU model is off (cpu-percent 0, no delays); no loopback TCP */
        len = sprintf(line, "[shadow-heartbeat] [node] %u,%llu,%llu,%f,%d,%f;%s;%s;%s;%s", secs, rb, sb, 0.0, 0, 0.0,
                      zero, zero, ci, co);
        lb_add(&b, (j + 1) * interval_ns, host, line, (size_t)len);
    }
    return lb_done(&b, out);
}
