/*
 * sched_policy_shd.c -- a Shadow SchedulerPolicy (src/main/core/scheduler/
 * scheduler_policy.h:31-51) whose offloaded hosts run on libshdgpu's engine.
 *
 * Shadow's scheduler (scheduler.c:116-176) picks a policy by type and drives
 * it through the vtable: addHost at registration (scheduler.c:419), push from
 * scheduler_push (scheduler.c:342-357), pop and getNextTime from the worker
 * round loop (scheduler.c:362-417, worker.c:182-193).  This policy, meant to
 * be added as SP_GPU_ROUNDS, serves two kinds of work in the
 * same conservative windows:
 *
 *   - the offloaded hosts' packet event loop, on the GPU: the first pop of a
 *     round advances the engine (or engine group) to that round's barrier
 *     with shd_eng_run_until / shd_xgroup_run_until, i.e. every device round
 *     of W inside [window start, barrier);
 *   - the events Shadow's CPU side still creates (hosts that are not
 *     offloaded, control tasks): one heap in event_compare order (event.c:
 *     110-153), the global_single policy's (scheduler_policy_global_single.c:
 *     40-71): push keeps the caller's reference, pop hands it back, events
 *     at or past the barrier wait.
 *
 * getNextTime is the minimum of the heap's head and the engine's next event.
 *
 * With a bridge (schedulerpolicygpurounds_new_bridged) the engine holds only
 * some hosts of the model (a partial engine) and the two sides exchange
 * packets, the way two of Shadow's workers do (worker_sendPacket's
 * scheduler_push of a deliver-packet task for another worker's host,
 * worker.c:541-571):
 *   - ingress: a push whose event the bridge claims (a packet for an
 *     offloaded host) becomes an shd_event; the policy keeps it until the
 *     engine's next round (shd_eng_push_events) and drops the Shadow event;
 *   - egress: after each engine round, the deliveries its hosts sent to
 *     CPU-side hosts (shd_eng_take_remote) become Shadow events through the
 *     bridge and join the heap; every one is due at or after the barrier.
 * The engine then runs one device round per Shadow round, [its next event,
 * barrier): the bridge needs Shadow's window (the runahead) to be at most the
 * engine's W, so that nothing either side sends lands inside the round.
 *
 * Shadow's own functions (event.c, glib) are resolved when Shadow links this
 * file; with -DSHD_CHECK_AGAINST_REFERENCE and the reference header included
 * (tests/test_boundary_cpu.py) the struct layout and every vtable signature
 * are checked against scheduler_policy.h at compile time.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/shdgpu.h"

#ifndef SHD_CHECK_AGAINST_REFERENCE
typedef struct _Event Event;
typedef struct _Host Host;
typedef struct _GQueue GQueue;
typedef uint64_t SimulationTime;   /* core/support/definitions.h:18 (guint64) */
typedef struct _SchedulerPolicy SchedulerPolicy;
/* scheduler_policy.h:40-51 (MAGIC_DECLARE adds a guint only in DEBUG builds) */
struct _SchedulerPolicy {
    int type;
    void* data;
    int referenceCount;
    void (*addHost)(SchedulerPolicy*, Host*, pthread_t);
    GQueue* (*getAssignedHosts)(SchedulerPolicy*);
    void (*push)(SchedulerPolicy*, Event*, Host*, Host*, SimulationTime);
    Event* (*pop)(SchedulerPolicy*, SimulationTime);
    SimulationTime (*getNextTime)(SchedulerPolicy*);
    void (*free)(SchedulerPolicy*);
#ifdef SHD_SHADOW_DEBUG
    unsigned int magic;
#endif
};
/* Shadow's (event.c) and glib's */
extern int event_compare(const Event* a, const Event* b, void* userData);
extern SimulationTime event_getTime(Event* event);
extern void event_unref(Event* event);
extern GQueue* g_queue_new(void);
extern void g_queue_push_tail(GQueue* queue, void* data);
extern void g_queue_free(GQueue* queue);
#endif

#define SHD_SP_GPU_ROUNDS 6   /* the SchedulerPolicyType value it would take */
#define SHD_SIMTIME_MAX_ (UINT64_MAX - 1)

/* packet ingress / egress between Shadow's CPU-side hosts and a partial
 * engine's offloaded hosts (the integrator's conversions of Shadow's Event
 * and Packet objects; INTEGRATION.md "Mixed CPU/GPU hosts") */
typedef struct shd_policy_bridge {
    /* a push of `event` (srcHost -> dstHost): return 1 and fill *out (kind
     * SHD_EV_PACKET, time, model host IDs src/dst, seq = the event's ID, pkt =
     * the packet's ID) when it is a packet for an offloaded host; 0 keeps the
     * event on the CPU side */
    int (*ingress)(void* user, Event* event, Host* srcHost, Host* dstHost, shd_event* out);
    /* the Shadow deliver-packet event for a delivery from an offloaded host to a
     * CPU-side host (NULL: dropped, and counted as an error) */
    Event* (*egress)(void* user, const shd_event* delivery);
    void* user;
    /* optional (both or neither): one lazy path cache across the sides
     * (topology.c:1969-2051 is one global cache).  touches_in hands the CPU
     * side the engine's first touches of the round before the round's CPU
     * events pop (the CPU side's cache applies each just before its first
     * later query, in event_compare order); touches_out, after them, returns
     * the CPU side's own first touches of the round (its queries that ran a
     * source row or a self path), which the engine's resolution ranks with its
     * own.  NULL: the two sides' first touches of a round are not ordered with
     * each other, exact on complete and prefer-direct graphs only. */
    void (*touches_in)(void* user, const shd_pending* engine_touches, uint64_t n);
    uint64_t (*touches_out)(void* user, const shd_pending** cpu_touches);
} shd_policy_bridge;

typedef struct {
    Event** heap;              /* binary min-heap in event_compare order */
    size_t n, cap;
    GQueue* hosts;             /* every registered host: one driving thread */
    shd_eng* eng;              /* the offloaded hosts' engine, or NULL */
    shd_xgroup* grp;           /* or the engine group this process drives */
    SimulationTime advanced;   /* the engine has run every round below this barrier */
    int error;                 /* the engine's last error status */
    int bridged;               /* a partial engine exchanging packets through `bridge` */
    shd_policy_bridge bridge;
    shd_event* ingress;        /* packets for offloaded hosts, until the engine's next round */
    size_t n_in, cap_in;
    shd_event* egress;         /* a round's deliveries to CPU-side hosts */
    size_t cap_out;
    int open;                  /* touches bridge: 1 a round ran whose resolution waits for the CPU side's
                                  first touches, 2 a window with no device round (ranks only) */
    int open_ambiguous;        /* its kernel flagged an ambiguous first-touch drop decision */
    shd_pending* touch;        /* its first touches: the engine's, then the CPU side's */
    size_t n_touch, cap_touch;
} gpu_policy;

static int ev_lt(Event* a, Event* b) { return event_compare(a, b, NULL) < 0; }

static void _gpurounds_addHost(SchedulerPolicy* policy, Host* host, pthread_t assignedThread) {
    gpu_policy* d = policy->data;
    (void)assignedThread;
    if (!d->hosts) d->hosts = g_queue_new();
    g_queue_push_tail(d->hosts, host);
}

static GQueue* _gpurounds_getHosts(SchedulerPolicy* policy) {
    gpu_policy* d = policy->data;
    return d->hosts;
}

static void heap_push(gpu_policy* d, Event* event);

static void _gpurounds_push(SchedulerPolicy* policy, Event* event, Host* srcHost, Host* dstHost,
                            SimulationTime barrier) {
    gpu_policy* d = policy->data;
    (void)barrier;   /* global order: no clamp (global_single.c:40-55) */
    if (d->bridged) {
        shd_event x;
        if (d->bridge.ingress(d->bridge.user, event, srcHost, dstHost, &x)) {
            if (d->n_in == d->cap_in) {
                size_t nc = d->cap_in ? 2 * d->cap_in : 1024;
                shd_event* ni = realloc(d->ingress, sizeof(shd_event) * nc);
                if (!ni) { d->error = SHD_ENOMEM; event_unref(event); return; }
                d->ingress = ni;
                d->cap_in = nc;
            }
            d->ingress[d->n_in++] = x;
            event_unref(event);   /* the packet lives on the device now */
            return;
        }
    }
    heap_push(d, event);
}

static void heap_push(gpu_policy* d, Event* event) {
    if (d->n == d->cap) {
        size_t nc = d->cap ? 2 * d->cap : 1024;
        Event** nh = realloc(d->heap, sizeof(Event*) * nc);
        if (!nh) return;
        d->heap = nh;
        d->cap = nc;
    }
    size_t i = d->n++;
    while (i > 0) {
        size_t p = (i - 1) / 2;
        if (!ev_lt(event, d->heap[p])) break;
        d->heap[i] = d->heap[p];
        i = p;
    }
    d->heap[i] = event;
}

static Event* heap_pop(gpu_policy* d) {
    Event* top = d->heap[0];
    Event* last = d->heap[--d->n];
    size_t i = 0;
    for (;;) {
        size_t l = 2 * i + 1, r = l + 1, m = i;
        Event* best = last;
        if (l < d->n && ev_lt(d->heap[l], best)) { m = l; best = d->heap[l]; }
        if (r < d->n && ev_lt(d->heap[r], best)) { m = r; best = d->heap[r]; }
        if (m == i) break;
        d->heap[i] = d->heap[m];
        i = m;
    }
    if (d->n) d->heap[i] = last;
    return top;
}

/* the buffered ingress into the engine (one push per flush) */
static void flush_ingress(gpu_policy* d) {
    if (!d->n_in) return;
    const int rc = shd_eng_push_events(d->eng, d->ingress, d->n_in);
    if (rc != SHD_OK) d->error = rc;
    d->n_in = 0;
}

static int touch_room(gpu_policy* d, size_t n) {
    if (d->n_touch + n <= d->cap_touch) return 1;
    size_t nc = d->cap_touch ? d->cap_touch : 256;
    while (nc < d->n_touch + n) nc *= 2;
    shd_pending* nt = realloc(d->touch, sizeof(shd_pending) * nc);
    if (!nt) { d->error = SHD_ENOMEM; return 0; }
    d->touch = nt;
    d->cap_touch = nc;
    return 1;
}

static void take_egress(gpu_policy* d);

/* touches bridge: the open round's resolution, over both sides' first touches
 * (after the round's CPU events), then its end and egress */
static void finish_open(gpu_policy* d) {
    if (!d->open) return;
    const int open = d->open;
    d->open = 0;
    const shd_pending* cp = NULL;
    const uint64_t nc = d->bridge.touches_out(d->bridge.user, &cp);
    if (nc && (!cp || !touch_room(d, nc))) { if (!cp) d->error = SHD_EINVAL; return; }
    if (nc) memcpy(d->touch + d->n_touch, cp, sizeof(shd_pending) * nc);
    d->n_touch += nc;
    const int ran = open == 1;   /* 2: no device round this window, ranks only */
    shd_round_summary r;
    int rc;
    if (ran && d->open_ambiguous)   /* the drop decision waited for the ranking: the window again */
        rc = shd_eng_round_retry(d->eng, d->touch, d->n_touch, &r);
    else
        rc = shd_eng_resolve(d->eng, d->touch, d->n_touch);
    d->n_touch = 0;
    if (rc != SHD_OK) { d->error = rc; return; }
    if (!ran) return;
    if ((rc = shd_eng_end_round(d->eng, &r)) != SHD_OK) { d->error = rc; return; }
    take_egress(d);
}

/* bridged: the engine's one round of this Shadow round, then its egress
 * (touches bridge: the round's kernel and its first touches to the CPU side;
 * the rest in finish_open) */
static void advance_bridged(gpu_policy* d, SimulationTime barrier) {
    finish_open(d);
    flush_ingress(d);
    uint64_t g = UINT64_MAX, W = 0;
    shd_eng_next_time(d->eng, &g);
    shd_eng_window(d->eng, &W);
    const SimulationTime ws = g > d->advanced ? g : d->advanced;
    d->advanced = barrier;
    if (ws >= barrier) {                           /* nothing on the device before the barrier */
        if (d->bridge.touches_in) {   /* the CPU side's first touches still go to the engine's ranks */
            d->bridge.touches_in(d->bridge.user, NULL, 0);
            d->open = 2;
        }
        return;
    }
    if (barrier - ws > W) { d->error = SHD_EINVAL; return; }   /* Shadow's window is wider than W */
    shd_round_summary r;
    int rc;
    if (d->bridge.touches_in) {
        if ((rc = shd_eng_round_begin(d->eng, ws, barrier, &r)) != SHD_OK) { d->error = rc; return; }
        d->open_ambiguous = (r.error & SHD_ERR_AMBIGUOUS) != 0;
        uint64_t n = 0;
        rc = shd_eng_pending_copy(d->eng, NULL, 0, &n);
        if (rc != SHD_OK && rc != SHD_ERANGE) { d->error = rc; return; }
        if (!touch_room(d, n)) return;
        if (n && (rc = shd_eng_pending_copy(d->eng, d->touch, d->cap_touch, &n)) != SHD_OK) { d->error = rc; return; }
        d->n_touch = n;
        d->bridge.touches_in(d->bridge.user, d->touch, n);
        d->open = 1;
        return;
    }
    rc = shd_eng_run_round(d->eng, ws, barrier, &r);
    if (rc != SHD_OK) { d->error = rc; return; }
    take_egress(d);
}

/* the round's deliveries to CPU-side hosts, as Shadow events in the heap */
static void take_egress(gpu_policy* d) {
    int rc;
    uint64_t n = 0;
    rc = shd_eng_take_remote(d->eng, d->egress, d->cap_out, &n);
    if (rc == SHD_ERANGE) {
        shd_event* no = realloc(d->egress, sizeof(shd_event) * n);
        if (!no) { d->error = SHD_ENOMEM; return; }
        d->egress = no;
        d->cap_out = n;
        rc = shd_eng_take_remote(d->eng, d->egress, d->cap_out, &n);
    }
    if (rc != SHD_OK) { d->error = rc; return; }
    for (uint64_t i = 0; i < n; i++) {
        Event* ev = d->bridge.egress(d->bridge.user, &d->egress[i]);
        if (ev) heap_push(d, ev);
        else d->error = SHD_EINVAL;
    }
}

/* run the engine's rounds below the barrier once per barrier */
static void advance(gpu_policy* d, SimulationTime barrier) {
    if (barrier <= d->advanced || (!d->eng && !d->grp)) return;
    if (d->bridged) { advance_bridged(d, barrier); return; }
    shd_run_stats st;
    const int rc = d->grp ? shd_xgroup_run_until(d->grp, barrier, &st) : shd_eng_run_until(d->eng, barrier, &st);
    if (rc != SHD_OK) d->error = rc;
    d->advanced = barrier;
}

static Event* _gpurounds_pop(SchedulerPolicy* policy, SimulationTime barrier) {
    gpu_policy* d = policy->data;
    advance(d, barrier);
    if (d->n == 0 || event_getTime(d->heap[0]) >= barrier) return NULL;
    return heap_pop(d);
}

static SimulationTime _gpurounds_getNextTime(SchedulerPolicy* policy) {
    gpu_policy* d = policy->data;
    if (d->bridged) {
        finish_open(d);     /* the round's CPU events have run: its egress joins the heap */
        flush_ingress(d);   /* the engine's next time covers what it was sent */
    }
    SimulationTime t = d->n ? event_getTime(d->heap[0]) : (SimulationTime)SHD_SIMTIME_MAX_;
    uint64_t g = UINT64_MAX;
    if (d->grp) shd_xgroup_next_time(d->grp, &g);
    else if (d->eng) shd_eng_next_time(d->eng, &g);
    return g < t ? g : t;
}

static void _gpurounds_free(SchedulerPolicy* policy) {
    gpu_policy* d = policy->data;
    while (d->n) event_unref(heap_pop(d));
    free(d->heap);
    free(d->ingress);
    free(d->egress);
    free(d->touch);
    if (d->hosts) g_queue_free(d->hosts);
    free(d);
    free(policy);
}

/* the policy over an engine (or, with grp != NULL, over an engine group this
 * process drives); eng and grp may both be NULL (CPU events only).  The
 * caller keeps ownership of the engine / group. */
SchedulerPolicy* schedulerpolicygpurounds_new(shd_eng* eng, shd_xgroup* grp) {
    SchedulerPolicy* p = calloc(1, sizeof(SchedulerPolicy));
    gpu_policy* d = calloc(1, sizeof(gpu_policy));
    if (!p || !d) { free(p); free(d); return NULL; }
    d->eng = eng;
    d->grp = grp;
    p->type = SHD_SP_GPU_ROUNDS;
    p->data = d;
    p->referenceCount = 1;
    p->addHost = _gpurounds_addHost;
    p->getAssignedHosts = _gpurounds_getHosts;
    p->push = _gpurounds_push;
    p->pop = _gpurounds_pop;
    p->getNextTime = _gpurounds_getNextTime;
    p->free = _gpurounds_free;
    return p;
}

/* the policy over a partial engine whose hosts exchange packets with Shadow's
 * CPU-side hosts through `bridge` (copied); NULL for an incomplete bridge */
SchedulerPolicy* schedulerpolicygpurounds_new_bridged(shd_eng* eng, const shd_policy_bridge* bridge) {
    if (!eng || !bridge || !bridge->ingress || !bridge->egress || !bridge->touches_in != !bridge->touches_out)
        return NULL;
    SchedulerPolicy* p = schedulerpolicygpurounds_new(eng, NULL);
    if (!p) return NULL;
    gpu_policy* d = p->data;
    d->bridged = 1;
    d->bridge = *bridge;
    return p;
}

/* the engine's last error status seen by the policy (0 = none) */
int schedulerpolicygpurounds_error(SchedulerPolicy* policy) { return ((gpu_policy*)policy->data)->error; }

#ifdef SHD_CHECK_AGAINST_REFERENCE
/* every vtable entry has the reference's function type */
static const SchedulerPolicyAddHostFunc chk_add = _gpurounds_addHost;
static const SchedulerPolicyGetHostsFunc chk_hosts = _gpurounds_getHosts;
static const SchedulerPolicyPushFunc chk_push = _gpurounds_push;
static const SchedulerPolicyPopFunc chk_pop = _gpurounds_pop;
static const SchedulerPolicyGetNextTimeFunc chk_next = _gpurounds_getNextTime;
static const SchedulerPolicyFreeFunc chk_free = _gpurounds_free;
/* and the layout this file assumes without the header is the reference's
 * (release build: MAGIC_DECLARE is empty) */
_Static_assert(offsetof(struct _SchedulerPolicy, data) == sizeof(void*), "data");
_Static_assert(offsetof(struct _SchedulerPolicy, referenceCount) == 2 * sizeof(void*), "referenceCount");
_Static_assert(offsetof(struct _SchedulerPolicy, addHost) == 3 * sizeof(void*), "addHost");
_Static_assert(offsetof(struct _SchedulerPolicy, free) == 8 * sizeof(void*), "free");
_Static_assert(sizeof(struct _SchedulerPolicy) == 9 * sizeof(void*), "size");
#endif
