/*
 * o_engine.c -- TEST INFRASTRUCTURE (oracle).  The serial reference event loop
 * (--workers 0: one global queue, one round to end_time; slave.c:415-428,
 * scheduler_policy_global_single.c:40-71) running the PHOLD-UDP model of
 * DESIGN.md on the reference's own per-host mechanisms:
 *
 *   event order           core/work/event.c:110-153
 *   push / end-time drop  core/scheduler/scheduler.c:342-357 (ID consumed first:
 *                         event_new_ assigns it, event.c:38)
 *   worker_sendPacket     core/worker.c:260-321
 *   deliver -> router     core/worker.c:253-258, routing/router.c:104-133
 *   CoDel                 routing/router_queue_codel.c (o_codel.c)
 *   token buckets         host/network_interface.c:102-226
 *   receive loop          host/network_interface.c:421-455
 *   send loop             host/network_interface.c:519-579 (loopback shortcut 548-555)
 *   epoll notify (+1 ns)  host/descriptor/epoll.c:345-365
 *   heartbeat             host/tracker.c:566-611
 *   boot                  host/host.c:372-390 (tracker, refill start per interface,
 *                         process_schedule)
 *   PHOLD application     src/test/phold/test_phold.c:107-110, 160-178, 180-240, 280-315
 *   implicit bind port    host/host.c:1058-1110, 1514-1525
 * Path latency / reliability come from the lazy path cache restatement
 * (o_pathcache.c), queried in serial event order exactly as worker.c does.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"

#define RAND_MAX_D ((double)2147483647)

/* ---- event_compare (event.c:110-153) ---- */
int o_event_compare(const shd_event* a, const shd_event* b) {
    if (a->time != b->time) return a->time > b->time ? 1 : -1;
    if (a->dst != b->dst) return a->dst > b->dst ? 1 : -1;
    if (a->src != b->src) return a->src > b->src ? 1 : -1;
    if (a->seq != b->seq) return a->seq > b->seq ? 1 : -1;
    return 0;
}

/* ---- global binary heap (pop order = total order of event_compare) ---- */
typedef struct { shd_event* a; uint64_t n, cap; } eheap;
static void eh_push(eheap* h, const shd_event* e) {
    if (h->n == h->cap) { h->cap = h->cap ? h->cap * 2 : 1024; h->a = realloc(h->a, h->cap * sizeof(shd_event)); }
    uint64_t i = h->n++;
    while (i > 0) {
        uint64_t p = (i - 1) / 2;
        if (o_event_compare(&h->a[p], e) <= 0) break;
        h->a[i] = h->a[p]; i = p;
    }
    h->a[i] = *e;
}
static shd_event eh_pop(eheap* h) {
    shd_event top = h->a[0];
    shd_event last = h->a[--h->n];
    uint64_t i = 0;
    for (;;) {
        uint64_t l = 2 * i + 1, r = l + 1, m = i;
        const shd_event* best = &last;
        if (l < h->n && o_event_compare(&h->a[l], best) < 0) { m = l; best = &h->a[l]; }
        if (r < h->n && o_event_compare(&h->a[r], best) < 0) { m = r; best = &h->a[r]; }
        if (m == i) break;
        h->a[i] = h->a[m]; i = m;
    }
    if (h->n) h->a[i] = last;
    return top;
}

typedef struct { uint32_t dst, pkt; } txent;
typedef struct {
    uint32_t rng; uint64_t ev_seq; uint32_t pkt_seq;
    uint64_t rx_rem, rx_cap, rx_refill, tx_rem, tx_cap, tx_refill;
    int refill_pending, notify_pending, listening;
    uint32_t unread;
    o_codel codel;
    txent* txq; uint32_t txq_head, txq_count, txq_cap;
    uint64_t n_events, n_pkt_events, n_sent, n_inet_drop, n_codel_drop, n_recv;
    /* tracker node counters (tracker.c:216-275): packets through the interface,
     * in (_networkinterface_receivePacket) and out (_networkinterface_sendPackets);
     * cumulative here, differenced per heartbeat by the reader */
    uint32_t if_in, if_out;
} ohost;

typedef struct {
    const shd_model* m;
    o_topo* topo;
    ohost* hosts;
    eheap q;
    uint64_t now;
    o_run* out;
} ctx_t;

static void trace(ctx_t* c, uint64_t t, uint64_t seq, uint32_t host, uint32_t peer, uint32_t pkt, uint32_t kind) {
    if (!c->m->trace) return;
    o_run* r = c->out;
    if (r->n_trace == r->cap_trace) {
        r->cap_trace = r->cap_trace ? r->cap_trace * 2 : 4096;
        r->trace = realloc(r->trace, r->cap_trace * sizeof(shd_trace_rec));
    }
    shd_trace_rec* x = &r->trace[r->n_trace++];
    x->time = t; x->seq = seq; x->host = host; x->peer = peer; x->pkt = pkt; x->kind = kind;
}

static inline int bootstrapping(ctx_t* c) { return c->now < c->m->bootstrap_end; }

/* event_new_ (consumes the source host's event ID, event.c:38) + scheduler_push
 * (discards time >= endTime, scheduler.c:346-349) */
static void push_event(ctx_t* c, uint32_t src, uint32_t dst, uint64_t t, uint32_t kind, uint32_t pkt) {
    shd_event e;
    e.time = t; e.seq = c->hosts[src].ev_seq++; e.src = src; e.dst = dst; e.pkt = pkt; e.kind = kind;
    if (t >= c->m->end_time) return;
    eh_push(&c->q, &e);
}
/* worker_scheduleTask (worker.c:235-251): self event at now + delay */
static void schedule_task(ctx_t* c, uint32_t h, uint32_t kind, uint64_t delay, uint32_t pkt) {
    push_event(c, h, h, c->now + delay, kind, pkt);
}

/* _networkinterface_scheduleNextRefillIfNeeded (network_interface.c:130-161);
 * timeStartedRefillingBuckets = 0 (all hosts boot at t = 0) */
static void refill_if_needed(ctx_t* c, uint32_t h) {
    ohost* H = &c->hosts[h];
    int need = (H->tx_rem < H->tx_cap) || (H->rx_rem < H->rx_cap);
    if (need && !H->refill_pending) {
        uint64_t interval = SHD_MS;
        uint64_t offset = c->now - 0;
        uint64_t until = interval - (offset % interval);
        schedule_task(c, h, SHD_EV_REFILL, until, 0);
        H->refill_pending = 1;
    }
}
static inline void consume(uint64_t* rem, uint64_t n) { *rem = (n >= *rem) ? 0 : *rem - n; }

/* _networkinterface_receivePacket (network_interface.c:375-419): hand the
 * datagram to the bound UDP socket (PHOLD listener on 8998) or drop it */
static void if_receive_packet(ctx_t* c, uint32_t h, uint32_t src, uint32_t pkt) {
    ohost* H = &c->hosts[h];
    H->if_in++;                        /* tracker_addInputBytes, n_i.c:415 */
    if (H->listening) {
        trace(c, c->now, 0, h, src, pkt, SHD_TR_RECV);
        H->n_recv++;
        H->unread++;
        /* socket readable -> epoll schedules one notification at +1 ns */
        if (!H->notify_pending) {
            schedule_task(c, h, SHD_EV_NOTIFY, 1, 0);
            H->notify_pending = 1;
        }
    } else {
        trace(c, c->now, 0, h, src, pkt, SHD_TR_IF_DROP);
    }
}

/* networkinterface_receivePackets (network_interface.c:421-455) */
static void if_receive_packets(ctx_t* c, uint32_t h) {
    ohost* H = &c->hosts[h];
    int boot = bootstrapping(c);
    o_codel_entry drops[64];
    while (boot || H->rx_rem >= SHD_MTU) {
        o_codel_entry p; uint32_t nd = 0;
        int have = o_codel_dequeue(&H->codel, c->now, &p, drops, 64, &nd);
        for (uint32_t i = 0; i < nd && i < 64; i++) {
            trace(c, c->now, 0, h, drops[i].src, drops[i].id, SHD_TR_CODEL_DROP);
            H->n_codel_drop++;
        }
        if (nd > 64) { fprintf(stderr, "oracle: codel drop burst > 64\n"); abort(); }
        if (!have) break;
        if_receive_packet(c, h, p.src, p.id);
        if (!boot) {
            consume(&H->rx_rem, p.len);
            refill_if_needed(c, h);
        }
    }
}

/* worker_sendPacket (worker.c:260-321) */
static void worker_send_packet(ctx_t* c, uint32_t h, uint32_t dst, uint32_t pkt) {
    ohost* H = &c->hosts[h];
    int32_t sv = c->m->host_vertex[h], dv = c->m->host_vertex[dst];
    double lat, rel;
    o_topo_get(c->topo, sv, dv, &lat, &rel);          /* topology_getReliability */
    double reliability = rel;
    double chance = o_next_double(&H->rng);
    if (bootstrapping(c) || chance <= reliability || c->m->payload == 0) {
        o_topo_get(c->topo, sv, dv, &lat, &rel);      /* topology_getLatency */
        uint64_t delay = (uint64_t)ceil(lat * (double)SHD_MS);
        uint64_t t = c->now + delay;
        o_topo_count_packet(c->topo, sv, dv);         /* incrementPathPacketCounter */
        trace(c, c->now, H->ev_seq, h, dst, pkt, SHD_TR_SENT);
        H->n_sent++;
        push_event(c, h, dst, t, SHD_EV_PACKET, pkt);
    } else {
        trace(c, c->now, 0, h, dst, pkt, SHD_TR_INET_DROP);
        H->n_inet_drop++;
    }
}

/* _networkinterface_sendPackets (network_interface.c:519-579), FIFO qdisc */
static void if_send_packets(ctx_t* c, uint32_t h) {
    ohost* H = &c->hosts[h];
    int boot = bootstrapping(c);
    uint32_t len = c->m->payload + SHD_HEADER_UDP;
    while (H->tx_rem >= SHD_MTU) {
        if (H->txq_count == 0) break;
        txent p = H->txq[H->txq_head];
        H->txq_head = (H->txq_head + 1) % H->txq_cap;
        H->txq_count--;
        H->if_out++;                   /* tracker_addOutputBytes, n_i.c:571 */
        if (p.dst == h) {
            /* packet to our own address: +1 ns local task, no router / RNG */
            trace(c, c->now, H->ev_seq, h, h, p.pkt, SHD_TR_LOCAL);
            schedule_task(c, h, SHD_EV_LOCAL, 1, p.pkt);
        } else {
            worker_send_packet(c, h, p.dst, p.pkt);
        }
        if (!boot) {
            consume(&H->tx_rem, len);
            refill_if_needed(c, h);
        }
    }
}

/* _host_getRandomPort (host.c:1058-1070) */
static uint16_t random_port(ohost* H) {
    double randomFraction = o_next_double(&H->rng);
    double numPotentialPorts = (double)(65535 - SHD_MIN_RANDOM_PORT);
    double randomPick = round(randomFraction * numPotentialPorts);
    uint16_t p = (uint16_t)randomPick;
    p = (uint16_t)(p + (uint16_t)SHD_MIN_RANDOM_PORT);
    return p;
}
/* _host_getRandomFreePort (host.c:1072-1110); the only port taken on the
 * default interface in this model is the PHOLD listener */
static uint16_t random_free_port(ohost* H) {
    for (int i = 0; i < 10; i++) {
        uint16_t p = random_port(H);
        if (p != SHD_PHOLD_LISTEN_PORT) return p;
    }
    uint16_t start = random_port(H);
    uint16_t next = (start == 65535) ? (uint16_t)SHD_MIN_RANDOM_PORT : (uint16_t)(start + 1);
    while (next != start) {
        if (next != SHD_PHOLD_LISTEN_PORT) return next;
        next = (next == 65535) ? (uint16_t)SHD_MIN_RANDOM_PORT : (uint16_t)(next + 1);
    }
    return 0;
}

/* _phold_sendNewMessage (test_phold.c:218-230): chooseNode with random()
 * (process_emu_random -> host RNG, process.c:4790-4795), then socket +
 * sendto (implicit bind: one random port, host.c:1514-1525), UDP packet,
 * networkinterface_wantsSend -> sendPackets */
static void send_new_message(ctx_t* c, uint32_t h) {
    ohost* H = &c->hosts[h];
    double r = ((double)o_rand_r(&H->rng)) / RAND_MAX_D;
    /* first i with cumulative >= r (test_phold.c:165-176) */
    const double* cum = c->m->dest_cum;
    int32_t lo = 0, hi = c->m->n_hosts;   /* search [lo,hi) */
    while (lo < hi) { int32_t mid = lo + (hi - lo) / 2; if (cum[mid] >= r) hi = mid; else lo = mid + 1; }
    if (lo >= c->m->n_hosts) return;      /* NULL node: nothing sent */
    uint32_t dst = (uint32_t)lo;
    (void)random_free_port(H);
    uint32_t pkt = H->pkt_seq++;
    if (H->txq_count == H->txq_cap) {
        uint32_t ncap = H->txq_cap * 2;
        txent* nq = malloc(sizeof(txent) * ncap);
        for (uint32_t i = 0; i < H->txq_count; i++) nq[i] = H->txq[(H->txq_head + i) % H->txq_cap];
        free(H->txq); H->txq = nq; H->txq_cap = ncap; H->txq_head = 0;
    }
    H->txq[(H->txq_head + H->txq_count) % H->txq_cap] = (txent){dst, pkt};
    H->txq_count++;
    if_send_packets(c, h);
}

/* _networkinterface_refillTokenBucketsCB (network_interface.c:163-183) */
static void refill_cb(ctx_t* c, uint32_t h) {
    ohost* H = &c->hosts[h];
    H->refill_pending = 0;
    H->rx_rem += H->rx_refill; if (H->rx_rem > H->rx_cap) H->rx_rem = H->rx_cap;
    H->tx_rem += H->tx_refill; if (H->tx_rem > H->tx_cap) H->tx_rem = H->tx_cap;
    if_receive_packets(c, h);
    if_send_packets(c, h);
    refill_if_needed(c, h);
}

/* heartbeat snapshots (tracker_heartbeat, tracker.c:566-611): at the k-th
 * heartbeat (time k*interval, k >= 1) host h stores its cumulative interface
 * counters at g_hb[(h*g_hb_k + k-1)*2 + {0: in, 1: out}] */
static uint32_t* g_hb = NULL;
static uint32_t g_hb_k = 0;
void o_engine_set_heartbeats_out(uint32_t* hb, uint32_t k_max) { g_hb = hb; g_hb_k = k_max; }
static void execute(ctx_t* c, const shd_event* e) {
    uint32_t h = e->dst;
    ohost* H = &c->hosts[h];
    H->n_events++;
    switch (e->kind) {
    case SHD_EV_HEARTBEAT:
        if (g_hb) {
            uint64_t k = c->now / c->m->heartbeat_interval;
            if (k >= 1 && k <= g_hb_k) {
                g_hb[((uint64_t)h * g_hb_k + k - 1) * 2] = H->if_in;
                g_hb[((uint64_t)h * g_hb_k + k - 1) * 2 + 1] = H->if_out;
            }
        }
        schedule_task(c, h, SHD_EV_HEARTBEAT, c->m->heartbeat_interval, 0);
        break;
    case SHD_EV_REFILL:
        refill_cb(c, h);
        break;
    case SHD_EV_REFILL_LO:
        /* loopback interface: buckets reach capacity, nothing to send or receive */
        break;
    case SHD_EV_APP_START:
        H->listening = 1;
        for (uint32_t i = 0; i < c->m->load; i++) send_new_message(c, h);
        break;
    case SHD_EV_PACKET: {
        /* _worker_runDeliverPacketTask -> router_enqueue (router.c:104-122) */
        H->n_pkt_events++;
        trace(c, c->now, e->seq, h, e->src, e->pkt, SHD_TR_ARRIVE);
        int was_empty = H->codel.count == 0;
        o_codel_enqueue(&H->codel, c->now, c->m->payload + SHD_HEADER_UDP, e->pkt, e->src);
        if (was_empty) if_receive_packets(c, h);
        break;
    }
    case SHD_EV_LOCAL:
        if_receive_packet(c, h, h, e->pkt);
        break;
    case SHD_EV_NOTIFY: {
        H->notify_pending = 0;
        uint32_t n = H->unread;
        H->unread = 0;
        for (uint32_t i = 0; i < n; i++) send_new_message(c, h);
        break;
    }
    default:
        fprintf(stderr, "oracle: bad event kind %u\n", e->kind);
        abort();
    }
}

/* host_boot at t = 0 (host.c:372-390) */
static void boot(ctx_t* c, uint32_t h) {
    ohost* H = &c->hosts[h];
    c->now = 0;
    /* tracker_new -> tracker_heartbeat inline -> next heartbeat (tracker.c:141, 607-610) */
    schedule_task(c, h, SHD_EV_HEARTBEAT, c->m->heartbeat_interval, 0);
    /* ethernet interface: timeStarted = 0, refill inline (network_interface.c:185-190) */
    refill_cb(c, h);
    /* loopback interface: G_MAXUINT32 KiB/s buckets; one refill at +1 ms */
    schedule_task(c, h, SHD_EV_REFILL_LO, SHD_MS, 0);
    /* process_schedule: start task at starttime (process.c:1344) */
    schedule_task(c, h, SHD_EV_APP_START, c->m->app_start, 0);
    (void)H;
}

static uint64_t g_mark = UINT64_MAX;
void o_engine_set_mark(uint64_t t) { g_mark = t; }
/* per-path packet counts at the end of a run (topology.c:2053-2063, logged by
 * _topology_logAllCachedPaths at teardown, 1929-1965): counts[s*V + d] = the
 * packet count of the cached entry stored as (s, d), 0 where none is stored */
static uint64_t* g_counts = NULL;
static int32_t g_counts_v = 0;
void o_engine_set_counts_out(uint64_t* counts, int32_t n_vertices) { g_counts = counts; g_counts_v = n_vertices; }

int o_engine_run(const shd_model* m, const shd_graph* gin, int32_t force_rows, o_run* out) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    memset(out, 0, sizeof(*out));
    ctx_t c;
    memset(&c, 0, sizeof(c));
    c.m = m; c.out = out;
    o_graph* g = o_graph_new(gin);
    /* attached vertices = verticesWithAttachedHosts */
    char* att = calloc(g->V, 1);
    int32_t na = 0;
    for (int32_t h = 0; h < m->n_hosts; h++) att[m->host_vertex[h]] = 1;
    int32_t* attached = malloc(sizeof(int32_t) * g->V);
    for (int32_t v = 0; v < g->V; v++) if (att[v]) attached[na++] = v;
    c.topo = o_topo_new(g, attached, na, force_rows);
    c.hosts = calloc(m->n_hosts, sizeof(ohost));
    for (int32_t h = 0; h < m->n_hosts; h++) {
        ohost* H = &c.hosts[h];
        H->rng = m->host_rng[h];
        /* _networkinterface_setupTokenBuckets (network_interface.c:192-226) */
        H->rx_refill = m->bw_down_kibps[h] * 1024 / 1000;
        H->tx_refill = m->bw_up_kibps[h] * 1024 / 1000;
        H->rx_cap = H->rx_refill + SHD_MTU;
        H->tx_cap = H->tx_refill + SHD_MTU;
        o_codel_init(&H->codel, 16);
        H->txq_cap = 16; H->txq = malloc(sizeof(txent) * 16);
    }
    for (int32_t h = 0; h < m->n_hosts; h++) boot(&c, (uint32_t)h);
    int marked = 0;
    while (c.q.n) {
        shd_event e = eh_pop(&c.q);
        c.now = e.time;
        if (!marked && c.now >= g_mark) {
            struct timespec tm;
            clock_gettime(CLOCK_MONOTONIC, &tm);
            out->mark_events = out->n_events; out->mark_pkt_events = out->n_pkt_events;
            out->mark_wall_ms = (tm.tv_sec - t0.tv_sec) * 1e3 + (tm.tv_nsec - t0.tv_nsec) * 1e-6;
            marked = 1;
        }
        execute(&c, &e);
        out->n_events++;
        if (e.kind == SHD_EV_PACKET) out->n_pkt_events++;
    }
    out->digest = calloc(m->n_hosts, sizeof(shd_host_digest));
    for (int32_t h = 0; h < m->n_hosts; h++) {
        ohost* H = &c.hosts[h];
        shd_host_digest* d = &out->digest[h];
        d->ev_seq = H->ev_seq; d->rng = H->rng; d->pkt_seq = H->pkt_seq;
        d->rx_remaining = H->rx_rem; d->tx_remaining = H->tx_rem;
        d->codel_total = H->codel.total; d->codel_interval_expire = H->codel.interval_expire;
        d->codel_next_drop = H->codel.next_drop; d->codel_mode = H->codel.mode;
        d->codel_count = H->codel.count; d->codel_drop_count = H->codel.drop_count;
        d->codel_drop_count_last = H->codel.drop_count_last;
        d->unread = H->unread;
        d->flags = (H->refill_pending ? 1u : 0u) | (H->notify_pending ? 2u : 0u) | (H->listening ? 4u : 0u)
                 | (H->txq_count ? 8u : 0u);
        d->n_events = H->n_events; d->n_pkt_events = H->n_pkt_events; d->n_sent = H->n_sent;
        d->n_inet_drop = H->n_inet_drop; d->n_codel_drop = H->n_codel_drop; d->n_recv = H->n_recv;
        o_codel_free(&H->codel); free(H->txq);
    }
    out->rows_run = o_topo_rows_run(c.topo);
    out->self_run = o_topo_self_run(c.topo);
    free(c.hosts); free(c.q.a); free(att); free(attached);
    if (g_counts)
        for (int32_t a = 0; a < g_counts_v; a++)
            for (int32_t b = 0; b < g_counts_v; b++) g_counts[(size_t)a * g_counts_v + b] = o_topo_stored_count(c.topo, a, b);
    o_topo_free(c.topo); o_graph_free(g);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    out->wall_ms = (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) * 1e-6;
    return 0;
}

void o_run_free(o_run* r) {
    free(r->trace); free(r->digest);
    memset(r, 0, sizeof(*r));
}
