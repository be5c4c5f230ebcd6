/*
 * topo_harness.c -- TEST INFRASTRUCTURE.  Stands in for the Shadow functions
 * libshdshadow.so (shadow-1_amd/host/topology_shd.c, sched_policy_shd.c) calls,
 * so the reference Topology API and the SchedulerPolicy can be driven from the
 * tests without Shadow:
 *   address_toHostIP          address.c (an Address holds a host-order IP here)
 *   random_nextDouble         random.c:39-43: rand_r(&seedState) / RAND_MAX
 *   worker_updateMinTimeJump  worker.c:429-432 (records the values it gets)
 */
#include <stdint.h>
#include <stdlib.h>

struct _Address { uint32_t ip; };
struct _Random { unsigned int seedState; unsigned int initialSeed; };

struct _Address* harness_address_new(uint32_t host_ip) {
    struct _Address* a = malloc(sizeof(*a));
    a->ip = host_ip;
    return a;
}
void harness_address_free(struct _Address* a) { free(a); }
unsigned int address_toHostIP(struct _Address* a) { return a->ip; }

struct _Random* harness_random_new(unsigned int seed) {
    struct _Random* r = malloc(sizeof(*r));
    r->seedState = seed;
    r->initialSeed = seed;
    return r;
}
void harness_random_free(struct _Random* r) { free(r); }
unsigned int harness_random_state(struct _Random* r) { return r->seedState; }
double random_nextDouble(struct _Random* r) { return ((double)rand_r(&r->seedState)) / ((double)RAND_MAX); }

static double g_min_jumps[1 << 16];
static int g_n_min_jumps = 0;
void worker_updateMinTimeJump(double minPathLatency) {
    if (g_n_min_jumps < (1 << 16)) g_min_jumps[g_n_min_jumps] = minPathLatency;
    g_n_min_jumps++;
}
int harness_min_jumps(double* out, int cap) {
    for (int i = 0; i < g_n_min_jumps && i < cap; i++) out[i] = g_min_jumps[i];
    return g_n_min_jumps;
}

/* ---- Shadow's Event (event.c:18-43, event_compare 110-153) and glib's GQueue,
 * as much of them as sched_policy_shd.c calls ---- */
struct _Event { uint64_t time; uint32_t dst, src; uint64_t seq; int refs; uint32_t pkt; };
struct _Event* harness_event_new(uint64_t time, uint32_t src, uint32_t dst, uint64_t seq) {
    struct _Event* e = malloc(sizeof(*e));
    e->time = time; e->src = src; e->dst = dst; e->seq = seq; e->refs = 1; e->pkt = ~0u;
    return e;
}
/* a deliver-packet task: the event's packet ID */
struct _Event* harness_packet_event_new(uint64_t time, uint32_t src, uint32_t dst, uint64_t seq, uint32_t pkt) {
    struct _Event* e = harness_event_new(time, src, dst, seq);
    e->pkt = pkt;
    return e;
}
uint64_t event_getTime(struct _Event* e) { return e->time; }
uint64_t harness_event_seq(struct _Event* e) { return e->seq; }
uint32_t harness_event_dst(struct _Event* e) { return e->dst; }
uint32_t harness_event_src(struct _Event* e) { return e->src; }
uint32_t harness_event_pkt(struct _Event* e) { return e->pkt; }
static int g_unrefs = 0;
void event_unref(struct _Event* e) { if (--e->refs == 0) { free(e); g_unrefs++; } }
int harness_unrefs(void) { return g_unrefs; }
int event_compare(const struct _Event* a, const struct _Event* b, void* userData) {
    (void)userData;
    if (a->time != b->time) return a->time > b->time ? 1 : -1;
    if (a->dst != b->dst) return a->dst > b->dst ? 1 : -1;   /* host IDs in registration order */
    if (a->src != b->src) return a->src > b->src ? 1 : -1;
    if (a->seq != b->seq) return a->seq > b->seq ? 1 : -1;
    return 0;
}
struct _GQueue { void** v; unsigned int n, cap; };
struct _GQueue* g_queue_new(void) { return calloc(1, sizeof(struct _GQueue)); }
void g_queue_push_tail(struct _GQueue* q, void* data) {
    if (q->n == q->cap) { q->cap = q->cap ? 2 * q->cap : 16; q->v = realloc(q->v, sizeof(void*) * q->cap); }
    q->v[q->n++] = data;
}
void g_queue_free(struct _GQueue* q) { free(q->v); free(q); }
unsigned int g_queue_get_length(struct _GQueue* q) { return q->n; }
