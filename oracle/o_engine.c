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
#include <pthread.h>
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
    /* a replying host (SHD_DEST_REPLY): the sources of the datagrams its
     * socket holds, in arrival order (recvfrom's address); an SHD_SEND_ONCE
     * host's implicitly bound port */
    uint32_t* rxq; uint32_t rxq_head, rxq_count, rxq_cap;
    int bound; uint16_t port;
} ohost;

/* a send whose pair had no cache entry at round start (parallel mode): its
 * drop decision was the same under both candidate rows, its delivery time
 * waits for the round's first touches to run in serial order */
typedef struct {
    uint64_t qtime, qseq;            /* executing event: time, seq */
    uint32_t qhost, qsrc, qsub;      /*   its host, its src, the query's position */
    int32_t s, d;                    /* vertices queried */
    uint32_t pass, dst, pkt;
    uint64_t seq;                    /* the delivery's event ID (pass) */
} opend;
typedef struct { shd_event* a; uint64_t n, cap; } evvec;
typedef struct { opend* a; uint64_t n, cap; } pendvec;

typedef struct {
    const shd_model* m;
    o_topo* topo;
    ohost* hosts;
    eheap q;            /* serial mode: the one global queue */
    uint64_t now;
    o_run* out;
    /* parallel mode (o_state_run_parallel), per worker thread */
    eheap* hq;          /* per-host queues (NULL: serial mode) */
    const o_graph* g;
    const int32_t* att_index;   /* vertex -> position in the row-cache targets */
    double** row_lat;
    double** row_rel;
    evvec mbox;         /* this round's events for other hosts */
    pendvec pend;       /* this round's first-touch sends */
    uint64_t q_time, q_seq;
    uint32_t q_host, q_src, q_sub;
    uint64_t n_ambig, n_events, n_pkt;
    /* one side of a co-simulation (o_state_new_part): only the hosts
     * [h_lo, h_hi) live here; events for the others leave by `egress`
     * (part = 0: every host is here) */
    int32_t part, h_lo, h_hi;
    evvec egress;
    /* one lazy cache across the sides (o_state_defer_touches): the other
     * side's first touches of the window, sorted, the next to apply; this
     * side's own; the attached vertices by index */
    shd_pending* ftd; uint64_t nftd, iftd;
    shd_pending* ftown; uint64_t nftown, capftown;
    int32_t ft_on;
    const int32_t* attached;
} ctx_t;

static void evvec_push(evvec* v, const shd_event* e) {
    if (v->n == v->cap) { v->cap = v->cap ? 2 * v->cap : 1024; v->a = realloc(v->a, v->cap * sizeof(shd_event)); }
    v->a[v->n++] = *e;
}
static void pendvec_push(pendvec* v, const opend* p) {
    if (v->n == v->cap) { v->cap = v->cap ? 2 * v->cap : 64; v->a = realloc(v->a, v->cap * sizeof(opend)); }
    v->a[v->n++] = *p;
}

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
    if (c->part && (dst < (uint32_t)c->h_lo || dst >= (uint32_t)c->h_hi)) {   /* the other side's host */
        evvec_push(&c->egress, &e);
        return;
    }
    if (!c->hq) eh_push(&c->q, &e);
    else if (dst == src) eh_push(&c->hq[dst], &e);    /* the executing host's own queue */
    else evvec_push(&c->mbox, &e);                    /* delivered at the round's end */
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

/* the datagram application host h runs (shdgpu.h shd_udp_app): PHOLD's
 * (test_phold.c), the UDP echo's server or client (ref_loop.c app 2), or the
 * model's own per-host spec (SHD_APP_UDP, ref_loop.c app 3); *peer: the
 * SHD_DEST_PEER host */
static shd_udp_app app_of(const ctx_t* c, uint32_t h, int32_t* peer) {
    shd_udp_app a = {SHD_SEND_EACH, SHD_DEST_WEIGHTED, c->m->load, 1};
    *peer = -1;
    if (c->m->app == SHD_APP_UDP_ECHO) {
        *peer = c->m->app_peer[h];
        if (*peer < 0) a = (shd_udp_app){SHD_SEND_LISTENER, SHD_DEST_REPLY, 0, 1};
        else a = (shd_udp_app){SHD_SEND_ONCE, SHD_DEST_PEER, c->m->load, 1};
    } else if (c->m->app == SHD_APP_UDP) {
        a = c->m->app_spec[c->m->host_app[h]];
        if (a.dest == SHD_DEST_PEER) *peer = c->m->app_peer[h];
    }
    return a;
}

/* _networkinterface_receivePacket (network_interface.c:375-419): hand the
 * datagram to the bound UDP socket (PHOLD listener on 8998) or drop it */
static void if_receive_packet(ctx_t* c, uint32_t h, uint32_t src, uint32_t pkt) {
    ohost* H = &c->hosts[h];
    H->if_in++;                        /* tracker_addInputBytes, n_i.c:415 */
    if (H->listening) {
        trace(c, c->now, 0, h, src, pkt, SHD_TR_RECV);
        H->n_recv++;
        H->unread++;
        int32_t pr;
        if (app_of(c, h, &pr).dest == SHD_DEST_REPLY) {   /* the socket keeps the datagram's source */
            if (H->rxq_count == H->rxq_cap) {
                uint32_t ncap = H->rxq_cap ? 2 * H->rxq_cap : 16;
                uint32_t* nq = malloc(sizeof(uint32_t) * ncap);
                for (uint32_t i = 0; i < H->rxq_count; i++) nq[i] = H->rxq[(H->rxq_head + i) % H->rxq_cap];
                free(H->rxq); H->rxq = nq; H->rxq_cap = ncap; H->rxq_head = 0;
            }
            H->rxq[(H->rxq_head + H->rxq_count) % H->rxq_cap] = src;
            H->rxq_count++;
        }
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

/* the two values a pair without a cache entry can be served, by which
 * endpoint runs its source row first (DESIGN.md "First-touch rule"): the
 * direct value twice; for s == d the "2 x min edge" self value or row s's own
 * entry; else row s's or row d's entry */
static void first_touch_candidates(ctx_t* c, int32_t s, int32_t d, double* l1, double* r1, double* l2, double* r2) {
    if (o_topo_is_complete(c->topo) || (c->g->prefer_direct && o_get_eid(c->g, s, d) >= 0)) {
        o_direct_path(c->g, s, d, l1, r1);
        *l2 = *l1; *r2 = *r1;
        return;
    }
    const int32_t js = c->att_index[s], jd = c->att_index[d];
    if (s == d) {
        o_self_path(c->g, s, l1, r1);
        *l2 = c->row_lat[s][js]; *r2 = c->row_rel[s][js];
        return;
    }
    *l1 = c->row_lat[s][jd]; *r1 = c->row_rel[s][jd];
    *l2 = c->row_lat[d][js]; *r2 = c->row_rel[d][js];
}

/* worker_sendPacket in parallel mode: the path cache is read-only during the
 * round; a pair with no entry logs the send for the round-end resolution */
static void worker_send_packet_par(ctx_t* c, uint32_t h, uint32_t dst, uint32_t pkt) {
    ohost* H = &c->hosts[h];
    int32_t sv = c->m->host_vertex[h], dv = c->m->host_vertex[dst];
    double lat, rel;
    const int stored = o_topo_peek(c->topo, sv, dv, &lat, &rel);
    double chance = o_next_double(&H->rng);
    int pass;
    if (stored) {
        pass = bootstrapping(c) || chance <= rel || c->m->payload == 0;
    } else {
        double l1, r1, l2, r2;
        first_touch_candidates(c, sv, dv, &l1, &r1, &l2, &r2);
        pass = bootstrapping(c) || chance <= r1 || c->m->payload == 0;
        const int pass2 = bootstrapping(c) || chance <= r2 || c->m->payload == 0;
        if (pass != pass2) c->n_ambig++;
        opend p;
        p.qtime = c->q_time; p.qseq = c->q_seq; p.qhost = c->q_host; p.qsrc = c->q_src; p.qsub = c->q_sub++;
        p.s = sv; p.d = dv; p.pass = (uint32_t)pass; p.dst = dst; p.pkt = pkt; p.seq = pass ? H->ev_seq : 0;
        pendvec_push(&c->pend, &p);
    }
    if (pass) {
        H->n_sent++;
        if (stored) {
            uint64_t t = c->now + (uint64_t)ceil(lat * (double)SHD_MS);
            push_event(c, h, dst, t, SHD_EV_PACKET, pkt);
        } else {
            H->ev_seq++;   /* event_new_ consumes the ID now; the time comes at the round's end */
        }
    } else {
        H->n_inet_drop++;
    }
}

/* event_compare's order of two queries' executing events (time, host, src,
 * seq), then their position in the event */
static int pend_key_less(const shd_pending* x, const shd_pending* y) {
    if (x->qtime != y->qtime) return x->qtime < y->qtime;
    if (x->qhost != y->qhost) return x->qhost < y->qhost;
    if (x->qsrc != y->qsrc) return x->qsrc < y->qsrc;
    if (x->qseq != y->qseq) return x->qseq < y->qseq;
    return x->qsub < y->qsub;
}
static int pend_key_cmp(const void* a, const void* b) {
    const shd_pending* x = a; const shd_pending* y = b;
    return pend_key_less(x, y) ? -1 : pend_key_less(y, x) ? 1 : 0;
}
/* the one-cache protocol at a query of this side (serial mode): the other
 * side's first touches before it in event order go to the cache first; a
 * query that runs a row or a self path is logged as this side's first touch */
static void first_touch_sync(ctx_t* c, int32_t sv, int32_t dv) {
    shd_pending k;
    memset(&k, 0, sizeof(k));
    k.qtime = c->q_time; k.qseq = c->q_seq; k.qhost = c->q_host; k.qsrc = c->q_src; k.qsub = c->q_sub++;
    while (c->iftd < c->nftd && pend_key_less(&c->ftd[c->iftd], &k)) {
        const shd_pending* r = &c->ftd[c->iftd++];
        o_topo_touch(c->topo, c->attached[r->a], c->attached[r->b]);
    }
    if (!o_topo_would_run(c->topo, sv, dv)) return;
    if (c->nftown == c->capftown) {
        c->capftown = c->capftown ? 2 * c->capftown : 64;
        c->ftown = realloc(c->ftown, c->capftown * sizeof(shd_pending));
    }
    k.a = (uint32_t)c->att_index[sv]; k.b = (uint32_t)c->att_index[dv];
    c->ftown[c->nftown++] = k;
}

/* worker_sendPacket (worker.c:260-321) */
static void worker_send_packet(ctx_t* c, uint32_t h, uint32_t dst, uint32_t pkt) {
    if (c->hq) { worker_send_packet_par(c, h, dst, pkt); return; }
    ohost* H = &c->hosts[h];
    int32_t sv = c->m->host_vertex[h], dv = c->m->host_vertex[dst];
    double lat, rel;
    if (c->ft_on) first_touch_sync(c, sv, dv);
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

/* one datagram of host h's application (app_of), `payload` bytes:
 *   the destination: SHD_DEST_WEIGHTED _phold_sendNewMessage's chooseNode
 *     (test_phold.c:160-178, 218-230) with random() (process_emu_random -> host
 *     RNG, process.c:4790-4795) over the host's own weights (each process reads
 *     its weights file, test_phold.c:341-356), no host drawn: nothing sent;
 *     SHD_DEST_PEER the peer; SHD_DEST_REPLY `src`, the datagram just read;
 *   the source port: SHD_SEND_EACH a new socket whose sendto binds it
 *     implicitly (one random port, host.c:1514-1525), closed after;
 *     SHD_SEND_ONCE the host's one socket, bound by its first sendto;
 *     SHD_SEND_LISTENER the listener (PHOLD's port, no draw);
 * then the UDP packet, networkinterface_wantsSend -> sendPackets */
static void app_send(ctx_t* c, uint32_t h, const shd_udp_app* a, int32_t peer, uint32_t src) {
    ohost* H = &c->hosts[h];
    uint32_t dst;
    if (a->dest == SHD_DEST_WEIGHTED) {
        double r = ((double)o_rand_r(&H->rng)) / RAND_MAX_D;
        const double* cum = c->m->dest_cum;
        if (c->m->host_class && c->m->n_classes > 1)
            cum += (size_t)c->m->host_class[h] * (size_t)c->m->n_hosts;
        int32_t lo = 0, hi = c->m->n_hosts;   /* first i with cumulative >= r, in [lo,hi) */
        while (lo < hi) { int32_t mid = lo + (hi - lo) / 2; if (cum[mid] >= r) hi = mid; else lo = mid + 1; }
        if (lo >= c->m->n_hosts) return;      /* NULL node: nothing sent */
        dst = (uint32_t)lo;
    } else {
        dst = a->dest == SHD_DEST_REPLY ? src : (uint32_t)peer;
    }
    uint16_t port = SHD_PHOLD_LISTEN_PORT;
    if (a->send == SHD_SEND_EACH) {
        port = random_free_port(H);
    } else if (a->send == SHD_SEND_ONCE) {
        if (!H->bound) { H->port = random_free_port(H); H->bound = 1; }
        port = H->port;
    }
    uint32_t pkt = H->pkt_seq++;
    /* packet_new + PDS_SND_CREATED (udp.c:116), PDS_SND_SOCKET_BUFFERED (socket.c:405) */
    if (c->m->queue_flags & SHD_QF_TRACE_STATUS) trace(c, c->now, port, h, ~0u, pkt, SHD_TR_CREATED);
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
/* the tracker interval of host h (<host heartbeatfrequency>, host.c:240) */
static uint64_t hb_interval(const ctx_t* c, uint32_t h) {
    return c->m->host_heartbeat ? c->m->host_heartbeat[h] : c->m->heartbeat_interval;
}
static uint32_t* g_hb = NULL;
static uint32_t g_hb_k = 0;
void o_engine_set_heartbeats_out(uint32_t* hb, uint32_t k_max) { g_hb = hb; g_hb_k = k_max; }
static void execute(ctx_t* c, const shd_event* e) {
    uint32_t h = e->dst;
    ohost* H = &c->hosts[h];
    H->n_events++;
    c->q_time = e->time; c->q_seq = e->seq; c->q_host = e->dst; c->q_src = e->src; c->q_sub = 0;
    switch (e->kind) {
    case SHD_EV_HEARTBEAT:
        if (g_hb) {
            uint64_t k = c->now / hb_interval(c, h);
            if (k >= 1 && k <= g_hb_k) {
                g_hb[((uint64_t)h * g_hb_k + k - 1) * 2] = H->if_in;
                g_hb[((uint64_t)h * g_hb_k + k - 1) * 2 + 1] = H->if_out;
            }
        }
        schedule_task(c, h, SHD_EV_HEARTBEAT, hb_interval(c, h), 0);
        break;
    case SHD_EV_REFILL:
        refill_cb(c, h);
        break;
    case SHD_EV_REFILL_LO:
        /* loopback interface: buckets reach capacity, nothing to send or receive */
        break;
    case SHD_EV_APP_START: {
        H->listening = 1;
        int32_t peer;
        const shd_udp_app a = app_of(c, h, &peer);
        for (uint32_t i = 0; i < a.n_start; i++) app_send(c, h, &a, peer, 0);   /* _phold_bootstrapMessages */
        break;
    }
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
        /* _phold_wait_and_process_events (test_phold.c:287-315): each recvfrom
         * (PDS_RCV_SOCKET_DELIVERED, udp.c:158) answered by one new message */
        int32_t peer;
        const shd_udp_app a = app_of(c, h, &peer);
        for (uint32_t i = 0; i < n; i++) {
            if (c->m->queue_flags & SHD_QF_TRACE_STATUS) trace(c, c->now, 0, h, ~0u, ~0u, SHD_TR_READ);
            uint32_t src = 0;
            if (a.dest == SHD_DEST_REPLY) {   /* recvfrom's address: the datagram's source */
                src = H->rxq[H->rxq_head];
                H->rxq_head = (H->rxq_head + 1) % H->rxq_cap;
                H->rxq_count--;
            }
            if (a.per_read) app_send(c, h, &a, peer, src);
        }
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
    schedule_task(c, h, SHD_EV_HEARTBEAT, hb_interval(c, h), 0);
    /* ethernet interface: timeStarted = 0, refill inline (network_interface.c:185-190) */
    refill_cb(c, h);
    /* loopback interface: G_MAXUINT32 KiB/s buckets; one refill at +1 ms */
    schedule_task(c, h, SHD_EV_REFILL_LO, SHD_MS, 0);
    /* process_schedule: start task at starttime (process.c:1344); with
     * SHD_QF_NO_APP_START the caller's pushed start events take its place */
    if (!(c->m->queue_flags & SHD_QF_NO_APP_START)) schedule_task(c, h, SHD_EV_APP_START, c->m->app_start, 0);
    (void)H;
}

/* caller-pushed events (shd_eng_push_events): self application starts, each
 * consuming its host's next event ID in array order, after every host booted */
static const shd_event* g_push = NULL;
static uint64_t g_npush = 0;
void o_engine_set_pushes(const shd_event* ev, uint64_t n) { g_push = ev; g_npush = n; }

/* ======================================================================
 * Engine state: boot, serial rounds, parallel rounds, clone, digest.
 * ====================================================================== */
struct o_state {
    ctx_t c;
    o_graph* g;
    int32_t* attached; int32_t na;
    int32_t* att_index;           /* [V] position in attached, -1 */
    double** row_lat; double** row_rel;   /* [V] precomputed rows (NULL until o_state_rows) */
    o_run run;                    /* counts (+ trace in serial mode) */
    int shared;                   /* a clone: graph, attached list and row cache belong to the original */
};

static double now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

static o_state* state_new(const shd_model* m, const shd_graph* gin, int32_t force_rows, int32_t h_lo,
                          int32_t h_hi) {
    o_state* S = calloc(1, sizeof(*S));
    ctx_t* c = &S->c;
    c->m = m; c->out = &S->run;
    c->part = !(h_lo == 0 && h_hi == m->n_hosts);
    c->h_lo = h_lo; c->h_hi = h_hi;   /* the hosts that boot here */
    S->g = o_graph_new(gin);
    c->g = S->g;
    /* attached vertices = verticesWithAttachedHosts */
    char* att = calloc(S->g->V, 1);
    for (int32_t h = 0; h < m->n_hosts; h++) att[m->host_vertex[h]] = 1;
    S->attached = malloc(sizeof(int32_t) * (S->g->V + 1));
    S->att_index = malloc(sizeof(int32_t) * S->g->V);
    for (int32_t v = 0; v < S->g->V; v++) {
        S->att_index[v] = att[v] ? S->na : -1;
        if (att[v]) S->attached[S->na++] = v;
    }
    free(att);
    c->att_index = S->att_index;
    c->attached = S->attached;
    c->topo = o_topo_new(S->g, S->attached, S->na, force_rows);
    c->hosts = calloc(m->n_hosts, sizeof(ohost));
    for (int32_t h = 0; h < m->n_hosts; h++) {
        ohost* H = &c->hosts[h];
        H->rng = m->host_rng[h];
        /* _networkinterface_setupTokenBuckets (network_interface.c:192-226) */
        H->rx_refill = m->bw_down_kibps[h] * 1024 / 1000;
        H->tx_refill = m->bw_up_kibps[h] * 1024 / 1000;
        H->rx_cap = H->rx_refill + SHD_MTU;
        H->tx_cap = H->tx_refill + SHD_MTU;
        o_codel_init(&H->codel, 16);
        H->txq_cap = 16; H->txq = malloc(sizeof(txent) * 16);
    }
    for (int32_t h = h_lo; h < h_hi; h++) boot(c, (uint32_t)h);
    for (uint64_t i = 0; i < g_npush; i++) {
        const shd_event* p = &g_push[i];
        if (p->kind != SHD_EV_APP_START || p->src != p->dst || p->dst >= (uint32_t)m->n_hosts) {
            fprintf(stderr, "oracle: bad pushed event\n");
            abort();
        }
        if (p->dst >= (uint32_t)h_lo && p->dst < (uint32_t)h_hi) push_event(c, p->src, p->dst, p->time, p->kind, 0);
    }
    return S;
}
o_state* o_state_new(const shd_model* m, const shd_graph* gin, int32_t force_rows) {
    return state_new(m, gin, force_rows, 0, m->n_hosts);
}

/* ---- co-simulation: one side of packet ingress/egress at the boundary.
 * Hosts [h_lo, h_hi) run here in the serial loop; the others are simulated
 * elsewhere (the GPU engine, or another part).  worker_sendPacket's scheduler_push
 * of a packet for a host of another worker (worker.c:541-571) becomes an
 * egress event; the other side's packets for hosts here arrive by
 * o_state_inject, between windows of W (every cross-host event of a window
 * lands at or after its end, so the union is the serial run). ---- */
o_state* o_state_new_part(const shd_model* m, const shd_graph* gin, int32_t h_lo, int32_t h_hi) {
    if (h_lo < 0 || h_hi > m->n_hosts || h_lo >= h_hi) return NULL;
    return state_new(m, gin, 0, h_lo, h_hi);
}
int o_state_inject(o_state* S, const shd_event* ev, uint64_t n) {
    ctx_t* c = &S->c;
    for (uint64_t i = 0; i < n; i++) {
        const shd_event* e = &ev[i];
        if (e->kind != SHD_EV_PACKET || e->dst < (uint32_t)c->h_lo || e->dst >= (uint32_t)c->h_hi ||
            (e->src >= (uint32_t)c->h_lo && e->src < (uint32_t)c->h_hi))
            return -1;
        if (e->time >= c->m->end_time) continue;   /* scheduler_push drops it (scheduler.c:346-349) */
        if (c->hq) eh_push(&c->hq[e->dst], e);
        else eh_push(&c->q, e);
    }
    return 0;
}
/* the events for the other side's hosts since the last call: *n = the count;
 * copied when out != NULL and cap covers it (then the list empties) */
int o_state_take_egress(o_state* S, shd_event* out, uint64_t cap, uint64_t* n) {
    evvec* v = &S->c.egress;
    *n = v->n;
    if (!out) return 0;
    if (cap < v->n) return -1;
    memcpy(out, v->a, sizeof(shd_event) * v->n);
    v->n = 0;
    return 0;
}
int o_state_defer_touches(o_state* S, const shd_pending* recs, uint64_t n) {
    ctx_t* c = &S->c;
    if (c->hq || c->iftd < c->nftd) return -1;   /* serial mode; the last window's all applied */
    for (uint64_t i = 0; i < n; i++)
        if (recs[i].a >= (uint32_t)S->na || recs[i].b >= (uint32_t)S->na) return -1;
    c->ft_on = 1;
    c->ftd = realloc(c->ftd, (n + 1) * sizeof(shd_pending));
    if (n) memcpy(c->ftd, recs, n * sizeof(shd_pending));
    qsort(c->ftd, n, sizeof(shd_pending), pend_key_cmp);
    c->nftd = n; c->iftd = 0;
    return 0;
}
int o_state_take_touches(o_state* S, shd_pending* out, uint64_t cap, uint64_t* n) {
    ctx_t* c = &S->c;
    while (c->iftd < c->nftd) {
        const shd_pending* r = &c->ftd[c->iftd++];
        o_topo_touch(c->topo, c->attached[r->a], c->attached[r->b]);
    }
    *n = c->nftown;
    if (!out) return 0;
    if (cap < c->nftown) return -1;
    if (c->nftown) memcpy(out, c->ftown, c->nftown * sizeof(shd_pending));
    c->nftown = 0;
    return 0;
}

/* time of the next event here (UINT64_MAX when none) */
uint64_t o_state_next_time(const o_state* S) { return S->c.q.n ? S->c.q.a[0].time : UINT64_MAX; }
/* the trace so far: *n = its length; copied when out != NULL and cap covers it */
int o_state_trace(const o_state* S, shd_trace_rec* out, uint64_t cap, uint64_t* n) {
    *n = S->run.n_trace;
    if (!out) return 0;
    if (cap < S->run.n_trace) return -1;
    memcpy(out, S->run.trace, sizeof(shd_trace_rec) * S->run.n_trace);
    return 0;
}

/* every attached vertex's source row, `threads` rows at a time (the values
 * _topology_computeSourcePaths computes do not depend on when it runs; the
 * lazy cache then takes them from here instead of running Dijkstra) */
typedef struct { o_state* S; int32_t next; pthread_mutex_t mu; } rowjob;
static void* row_worker(void* arg) {
    rowjob* J = arg;
    o_state* S = J->S;
    int32_t* ok = malloc(sizeof(int32_t) * (S->na + 1));
    for (;;) {
        pthread_mutex_lock(&J->mu);
        int32_t j = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (j >= S->na) break;
        int32_t v = S->attached[j];
        double* lat = malloc(sizeof(double) * S->na);
        double* rel = malloc(sizeof(double) * S->na);
        o_sssp_row(S->g, v, S->attached, S->na, lat, rel, ok, NULL, NULL);
        for (int32_t k = 0; k < S->na; k++) if (!ok[k]) lat[k] = NAN;
        S->row_lat[v] = lat; S->row_rel[v] = rel;
    }
    free(ok);
    return NULL;
}
void o_state_rows(o_state* S, int threads) {
    if (S->row_lat) return;
    S->row_lat = calloc(S->g->V, sizeof(double*));
    S->row_rel = calloc(S->g->V, sizeof(double*));
    if (!o_topo_is_complete(S->c.topo) || S->g->prefer_direct) {
        rowjob J = {S, 0, PTHREAD_MUTEX_INITIALIZER};
        if (threads < 1) threads = 1;
        pthread_t* th = malloc(sizeof(pthread_t) * threads);
        for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, row_worker, &J);
        for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
        free(th);
    }
    o_topo_set_row_cache(S->c.topo, S->row_lat, S->row_rel);
    S->c.row_lat = S->row_lat; S->c.row_rel = S->row_rel;
}

static uint64_t g_mark = UINT64_MAX;
void o_engine_set_mark(uint64_t t) { g_mark = t; }

/* serial mode (--workers 0): pop in event_compare order while time < t_until */
void o_state_run_serial(o_state* S, uint64_t t_until) {
    ctx_t* c = &S->c;
    o_run* out = &S->run;
    const double t0 = now_ms();
    int marked = out->mark_wall_ms != 0;
    while (c->q.n && c->q.a[0].time < t_until) {
        shd_event e = eh_pop(&c->q);
        c->now = e.time;
        if (!marked && c->now >= g_mark) {
            out->mark_events = out->n_events; out->mark_pkt_events = out->n_pkt_events;
            out->mark_wall_ms = out->wall_ms + now_ms() - t0;
            marked = 1;
        }
        execute(c, &e);
        out->n_events++;
        if (e.kind == SHD_EV_PACKET) out->n_pkt_events++;
    }
    out->wall_ms += now_ms() - t0;
}

/* ---- parallel rounds (a host-steal-equivalent scheduler, serial-equivalent
 * windows: scheduler_policy_host_steal.c:227-431 with W <= every path delay,
 * so no clamp ever applies and the result is the serial run's) ---- */
typedef struct {
    o_state* S;
    int T;
    ctx_t* tc;                 /* per-thread contexts */
    pthread_barrier_t bar;
    uint64_t we;               /* this round's window end */
    int stop;
    int32_t next_chunk;        /* work queue: host chunks of kChunk */
    pthread_mutex_t mu;
    uint64_t* tmin;            /* per thread: min next time over the hosts it ran */
} parjob;
enum { kChunk = 64 };

static int pend_cmp(const void* x, const void* y) {
    const opend* a = x; const opend* b = y;
    if (a->qtime != b->qtime) return a->qtime < b->qtime ? -1 : 1;
    if (a->qhost != b->qhost) return a->qhost < b->qhost ? -1 : 1;
    if (a->qsrc != b->qsrc) return a->qsrc < b->qsrc ? -1 : 1;
    if (a->qseq != b->qseq) return a->qseq < b->qseq ? -1 : 1;
    return a->qsub < b->qsub ? -1 : (a->qsub > b->qsub);
}

static void par_round_work(parjob* J, int k) {
    ctx_t* c = &J->tc[k];
    const int32_t H = J->S->c.m->n_hosts;
    const uint64_t we = J->we;
    uint64_t mn = UINT64_MAX;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        int32_t ch = J->next_chunk++;
        pthread_mutex_unlock(&J->mu);
        int32_t h0 = ch * kChunk;
        if (h0 >= H) break;
        int32_t h1 = h0 + kChunk < H ? h0 + kChunk : H;
        for (int32_t h = h0; h < h1; h++) {
            eheap* q = &c->hq[h];
            while (q->n && q->a[0].time < we) {
                shd_event e = eh_pop(q);
                c->now = e.time;
                execute(c, &e);
                c->n_events++;
                if (e.kind == SHD_EV_PACKET) c->n_pkt++;
            }
            if (q->n && q->a[0].time < mn) mn = q->a[0].time;
        }
    }
    J->tmin[k] = mn;
}

static void* par_thread(void* arg) {
    parjob** pj = arg;
    parjob* J = pj[0];
    int k = (int)(pj[1] - pj[0]);   /* thread index smuggled as an offset */
    for (;;) {
        pthread_barrier_wait(&J->bar);
        if (J->stop) break;
        par_round_work(J, k);
        pthread_barrier_wait(&J->bar);
    }
    return NULL;
}

int o_state_run_parallel(o_state* S, uint64_t t_until, int threads, o_par_stats* st) {
    ctx_t* base = &S->c;
    const shd_model* m = base->m;
    const int32_t H = m->n_hosts;
    memset(st, 0, sizeof(*st));
    if (S->g->directed || m->trace || S->c.part) return -1;   /* the bench graphs: undirected, no trace, whole */
    o_state_rows(S, threads);
    /* per-host queues from the global one */
    eheap* hq = calloc(H, sizeof(eheap));
    while (base->q.n) { shd_event e = eh_pop(&base->q); eh_push(&hq[e.dst], &e); }
    /* W: every path latency is at least the smallest edge latency */
    double wmin = INFINITY;
    for (int32_t i = 0; i < S->g->E; i++) if (S->g->w[i] < wmin) wmin = S->g->w[i];
    uint64_t W = (uint64_t)ceil(wmin * (double)SHD_MS);
    if (W == 0) W = 1;
    parjob J;
    memset(&J, 0, sizeof(J));
    J.S = S; J.T = threads < 1 ? 1 : threads;
    pthread_mutex_init(&J.mu, NULL);
    pthread_barrier_init(&J.bar, NULL, (unsigned)J.T);
    J.tc = calloc(J.T, sizeof(ctx_t));
    J.tmin = calloc(J.T, sizeof(uint64_t));
    for (int k = 0; k < J.T; k++) {
        J.tc[k] = *base;
        J.tc[k].hq = hq;
        memset(&J.tc[k].mbox, 0, sizeof(evvec));
        memset(&J.tc[k].pend, 0, sizeof(pendvec));
        J.tc[k].n_ambig = J.tc[k].n_events = J.tc[k].n_pkt = 0;
    }
    parjob** args = malloc(sizeof(parjob*) * 2 * J.T);
    pthread_t* th = malloc(sizeof(pthread_t) * J.T);
    for (int k = 1; k < J.T; k++) {
        args[2 * k] = &J;
        args[2 * k + 1] = &J + k;
        pthread_create(&th[k], NULL, par_thread, &args[2 * k]);
    }
    const double t0 = now_ms();
    uint64_t ws = UINT64_MAX;
    for (int32_t h = 0; h < H; h++) if (hq[h].n && hq[h].a[0].time < ws) ws = hq[h].a[0].time;
    pendvec all = {0};
    while (ws < t_until) {
        uint64_t we = ws + W;
        if (we > t_until || we < ws) we = t_until;
        J.we = we; J.next_chunk = 0;
        pthread_barrier_wait(&J.bar);            /* round start */
        par_round_work(&J, 0);
        pthread_barrier_wait(&J.bar);            /* every host ran its events < we */
        st->rounds++;
        /* round end (one thread): deliveries, then the first touches in serial order */
        uint64_t nx = UINT64_MAX;
        all.n = 0;
        for (int k = 0; k < J.T; k++) {
            ctx_t* c = &J.tc[k];
            if (J.tmin[k] < nx) nx = J.tmin[k];
            for (uint64_t i = 0; i < c->mbox.n; i++) {
                eh_push(&hq[c->mbox.a[i].dst], &c->mbox.a[i]);
                if (c->mbox.a[i].time < nx) nx = c->mbox.a[i].time;
            }
            c->mbox.n = 0;
            for (uint64_t i = 0; i < c->pend.n; i++) pendvec_push(&all, &c->pend.a[i]);
            c->pend.n = 0;
        }
        if (all.n) {
            qsort(all.a, all.n, sizeof(opend), pend_cmp);
            for (uint64_t i = 0; i < all.n; i++) {
                const opend* p = &all.a[i];
                double lat, rel;
                o_topo_get(base->topo, p->s, p->d, &lat, &rel);   /* runs the row, stores */
                if (!p->pass) continue;
                shd_event e;
                e.time = p->qtime + (uint64_t)ceil(lat * (double)SHD_MS);
                e.seq = p->seq; e.src = p->qhost; e.dst = p->dst; e.pkt = p->pkt; e.kind = SHD_EV_PACKET;
                if (e.time >= m->end_time) continue;
                eh_push(&hq[e.dst], &e);
                if (e.time < nx) nx = e.time;
            }
            st->first_touch_sends += all.n;
        }
        ws = nx;
    }
    J.stop = 1;
    pthread_barrier_wait(&J.bar);
    for (int k = 1; k < J.T; k++) pthread_join(th[k], NULL);
    st->wall_ms = now_ms() - t0;
    for (int k = 0; k < J.T; k++) {
        st->n_events += J.tc[k].n_events;
        st->n_pkt_events += J.tc[k].n_pkt;
        st->ambiguous += J.tc[k].n_ambig;
        free(J.tc[k].mbox.a); free(J.tc[k].pend.a);
    }
    st->window_ns = W;
    st->threads = J.T;
    S->run.n_events += st->n_events;
    S->run.n_pkt_events += st->n_pkt_events;
    /* back to one global queue (the serial loop can continue) */
    for (int32_t h = 0; h < H; h++) {
        while (hq[h].n) { shd_event e = eh_pop(&hq[h]); eh_push(&base->q, &e); }
        free(hq[h].a);
    }
    free(hq); free(all.a); free(args); free(th); free(J.tc); free(J.tmin);
    pthread_barrier_destroy(&J.bar);
    pthread_mutex_destroy(&J.mu);
    return 0;
}

static void ohost_clone(ohost* dst, const ohost* src) {
    *dst = *src;
    dst->codel.q = malloc(sizeof(o_codel_entry) * src->codel.cap);
    memcpy(dst->codel.q, src->codel.q, sizeof(o_codel_entry) * src->codel.cap);
    dst->txq = malloc(sizeof(txent) * src->txq_cap);
    memcpy(dst->txq, src->txq, sizeof(txent) * src->txq_cap);
}

/* a deep copy (the row cache is shared, read-only) */
o_state* o_state_clone(const o_state* S) {
    o_state* C = calloc(1, sizeof(*C));
    *C = *S;
    C->c.out = &C->run;
    C->run.trace = NULL; C->run.n_trace = C->run.cap_trace = 0; C->run.digest = NULL;
    const int32_t H = S->c.m->n_hosts;
    /* the graph, attached list and row cache are read-only: shared with S */
    C->c.topo = o_topo_clone(S->c.topo);
    C->c.hosts = malloc(sizeof(ohost) * H);
    for (int32_t h = 0; h < H; h++) ohost_clone(&C->c.hosts[h], &S->c.hosts[h]);
    C->c.q.a = malloc(sizeof(shd_event) * (S->c.q.cap ? S->c.q.cap : 1));
    memcpy(C->c.q.a, S->c.q.a, sizeof(shd_event) * S->c.q.n);
    C->c.egress.a = malloc(sizeof(shd_event) * (S->c.egress.cap ? S->c.egress.cap : 1));
    memcpy(C->c.egress.a, S->c.egress.a, sizeof(shd_event) * S->c.egress.n);
    C->c.ftd = NULL; C->c.nftd = C->c.iftd = 0;   /* the one-cache protocol starts afresh */
    C->c.ftown = NULL; C->c.nftown = C->c.capftown = 0; C->c.ft_on = 0;
    C->shared = 1;
    return C;
}

void o_state_digest(const o_state* S, shd_host_digest* out) {
    const shd_model* m = S->c.m;
    for (int32_t h = 0; h < m->n_hosts; h++) {
        const ohost* H = &S->c.hosts[h];
        shd_host_digest* d = &out[h];
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
    }
}

const o_run* o_state_stats(const o_state* S) { return &S->run; }

void o_state_free(o_state* S) {
    if (!S) return;
    for (int32_t h = 0; h < S->c.m->n_hosts; h++) { o_codel_free(&S->c.hosts[h].codel); free(S->c.hosts[h].txq); }
    free(S->c.hosts); free(S->c.q.a); free(S->c.egress.a); free(S->c.ftd); free(S->c.ftown);
    o_topo_free(S->c.topo);
    if (!S->shared) {
        if (S->row_lat) {
            for (int32_t v = 0; v < S->g->V; v++) { free(S->row_lat[v]); free(S->row_rel[v]); }
            free(S->row_lat); free(S->row_rel);
        }
        o_graph_free(S->g);
        free(S->attached); free(S->att_index);
    }
    free(S->run.trace); free(S->run.digest);
    free(S);
}

/* the bench's CPU baseline: the same workload warmed up once (rows computed
 * on `threads` cores, then the serial loop to t_mark), then the window
 * [t_mark, t_end) timed twice from that state -- serial on one core, and in
 * parallel rounds on `threads` cores -- and the two end states compared */
int o_baseline(const shd_model* m, const shd_graph* g, uint64_t t_mark, uint64_t t_end, int threads,
               o_baseline_out* out) {
    memset(out, 0, sizeof(*out));
    double t0 = now_ms();
    o_state* A = o_state_new(m, g, 0);
    o_state_rows(A, threads);
    out->rows_ms = now_ms() - t0;
    t0 = now_ms();
    o_state_run_serial(A, t_mark);
    out->warmup_ms = now_ms() - t0;
    o_state* B = o_state_clone(A);
    const uint64_t e0 = A->run.n_events, p0 = A->run.n_pkt_events;
    t0 = now_ms();
    o_state_run_serial(A, t_end);
    out->serial_ms = now_ms() - t0;
    out->serial_events = A->run.n_events - e0;
    out->serial_pkt_events = A->run.n_pkt_events - p0;
    o_par_stats ps;
    int rc = o_state_run_parallel(B, t_end, threads, &ps);
    out->parallel_ms = ps.wall_ms;
    out->parallel_events = ps.n_events;
    out->parallel_pkt_events = ps.n_pkt_events;
    out->parallel_rounds = ps.rounds;
    out->parallel_first_touch = ps.first_touch_sends;
    out->ambiguous = ps.ambiguous;
    out->threads = ps.threads;
    out->window_ns = ps.window_ns;
    if (rc == 0) {
        const int32_t H = m->n_hosts;
        shd_host_digest* da = malloc(sizeof(shd_host_digest) * H);
        shd_host_digest* db = malloc(sizeof(shd_host_digest) * H);
        o_state_digest(A, da);
        o_state_digest(B, db);
        out->same_end_state = memcmp(da, db, sizeof(shd_host_digest) * H) == 0;
        free(da); free(db);
    }
    o_state_free(B);
    o_state_free(A);
    return rc;
}

/* per-path packet counts at the end of a run (topology.c:2053-2063, logged by
 * _topology_logAllCachedPaths at teardown, 1929-1965): counts[s*V + d] = the
 * packet count of the cached entry stored as (s, d), 0 where none is stored */
static uint64_t* g_counts = NULL;
static int32_t g_counts_v = 0;
void o_engine_set_counts_out(uint64_t* counts, int32_t n_vertices) { g_counts = counts; g_counts_v = n_vertices; }

int o_engine_run(const shd_model* m, const shd_graph* gin, int32_t force_rows, o_run* out) {
    const double t0 = now_ms();
    o_state* S = o_state_new(m, gin, force_rows);
    S->run.wall_ms = now_ms() - t0;
    o_state_run_serial(S, UINT64_MAX);
    *out = S->run;
    S->run.trace = NULL;   /* handed over */
    out->digest = calloc(m->n_hosts, sizeof(shd_host_digest));
    o_state_digest(S, out->digest);
    out->rows_run = o_topo_rows_run(S->c.topo);
    out->self_run = o_topo_self_run(S->c.topo);
    if (g_counts)
        for (int32_t a = 0; a < g_counts_v; a++)
            for (int32_t b = 0; b < g_counts_v; b++)
                g_counts[(size_t)a * g_counts_v + b] = o_topo_stored_count(S->c.topo, a, b);
    o_state_free(S);
    out->wall_ms = now_ms() - t0;
    return 0;
}

void o_run_free(o_run* r) {
    free(r->trace); free(r->digest);
    memset(r, 0, sizeof(*r));
}
