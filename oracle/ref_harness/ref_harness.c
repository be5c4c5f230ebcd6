/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Links the reference's OWN sources, compiled unmodified from /root/reference
 * by oracle/Makefile into oracle/_ref/libshdref.so:
 *   src/main/utility/random.c           (rand_r RNG)
 *   src/main/utility/priority_queue.c   (the scheduler's binary heap)
 *   src/main/routing/router_queue_codel.c (CoDel)
 * and exposes a flat API to tests/test_oracle_ref.py, which checks the oracle
 * restatement (oracle/o_rng.c, o_codel.c) against them.  The six functions
 * below are the collaborators router_queue_codel.c calls (its packet and
 * worker), implemented here as a test double: a packet with an id and a
 * length, and a settable clock.
 */
#include <glib.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "main/routing/packet.h"
#include "main/routing/router.h"
#include "main/routing/router_queue_codel.h"
#include "main/utility/priority_queue.h"
#include "main/utility/random.h"

struct _Packet {
    uint32_t id, payload, header, status;
    int refs;
};

static SimulationTime g_now;
static uint32_t g_drops[1 << 16];
static uint32_t g_ndrops;

SimulationTime worker_getCurrentTime(void) { return g_now; }
void packet_ref(Packet* p) { p->refs++; }
void packet_unref(Packet* p) {
    if (--p->refs <= 0) free(p);
}
guint packet_getPayloadLength(Packet* p) { return p->payload; }
guint packet_getHeaderSize(Packet* p) { return p->header; }
void packet_addDeliveryStatus(Packet* p, PacketDeliveryStatusFlags status) {
    p->status |= (uint32_t)status;
    if (status == PDS_ROUTER_DROPPED && g_ndrops < (1u << 16)) g_drops[g_ndrops++] = p->id;
}

/* ---- CoDel ---- */
void* ref_codel_new(void) { return routerqueuecodel_getHooks()->new(); }
void ref_codel_free(void* q) { routerqueuecodel_getHooks()->free(q); }
int ref_codel_enqueue(void* q, uint64_t now, uint32_t id, uint32_t payload) {
    g_now = now;
    Packet* p = calloc(1, sizeof(Packet));
    p->id = id; p->payload = payload; p->header = 42; p->refs = 1;
    gboolean ok = routerqueuecodel_getHooks()->enqueue(q, p);
    packet_unref(p);   /* the queue holds its own reference */
    return ok ? 1 : 0;
}
/* returns 1 and *id when a packet comes out; dropped ids via ref_codel_drops */
int ref_codel_dequeue(void* q, uint64_t now, uint32_t* id) {
    g_now = now;
    Packet* p = routerqueuecodel_getHooks()->dequeue(q);
    if (!p) return 0;
    *id = p->id;
    packet_unref(p);
    return 1;
}
uint32_t ref_codel_drops(uint32_t* out, uint32_t cap) {
    uint32_t n = g_ndrops < cap ? g_ndrops : cap;
    memcpy(out, g_drops, n * sizeof(uint32_t));
    g_ndrops = 0;
    return n;
}

/* ---- RNG ---- */
void* ref_random_new(uint32_t seed) { return random_new(seed); }
void ref_random_free(void* r) { random_free(r); }
int32_t ref_random_rand(void* r) { return random_rand(r); }
double ref_random_next_double(void* r) { return random_nextDouble(r); }
uint32_t ref_random_next_uint(void* r) { return random_nextUInt(r); }

/* ---- priority queue over 4-tuple keys (event_compare order) ---- */
typedef struct { uint64_t time; uint32_t dst, src; uint64_t seq; } key4;
static gint key4_compare(gconstpointer pa, gconstpointer pb, gpointer ud) {
    const key4* a = pa; const key4* b = pb;
    if (a->time != b->time) return a->time > b->time ? 1 : -1;
    if (a->dst != b->dst) return a->dst > b->dst ? 1 : -1;
    if (a->src != b->src) return a->src > b->src ? 1 : -1;
    if (a->seq != b->seq) return a->seq > b->seq ? 1 : -1;
    return 0;
}
/* push n keys in the given order, pop them all: out[i] = index popped i-th */
int ref_pq_order(const uint64_t* time, const uint32_t* dst, const uint32_t* src, const uint64_t* seq,
                 uint32_t n, uint32_t* out) {
    PriorityQueue* q = priorityqueue_new(key4_compare, NULL, NULL);
    key4* ks = calloc(n ? n : 1, sizeof(key4));
    for (uint32_t i = 0; i < n; i++) {
        ks[i].time = time[i]; ks[i].dst = dst[i]; ks[i].src = src[i]; ks[i].seq = seq[i];
        priorityqueue_push(q, &ks[i]);
    }
    for (uint32_t i = 0; i < n; i++) {
        key4* k = priorityqueue_pop(q);
        out[i] = (uint32_t)(k - ks);
    }
    priorityqueue_free(q);
    free(ks);
    return 0;
}
