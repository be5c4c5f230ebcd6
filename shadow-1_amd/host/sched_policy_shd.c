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
 * The two kinds do not exchange packets (an offloaded host's traffic stays on
 * the device); that is the partition INTEGRATION.md describes.
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

typedef struct {
    Event** heap;              /* binary min-heap in event_compare order */
    size_t n, cap;
    GQueue* hosts;             /* every registered host: one driving thread */
    shd_eng* eng;              /* the offloaded hosts' engine, or NULL */
    shd_xgroup* grp;           /* or the engine group this process drives */
    SimulationTime advanced;   /* the engine has run every round below this barrier */
    int error;                 /* the engine's last error status */
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

static void _gpurounds_push(SchedulerPolicy* policy, Event* event, Host* srcHost, Host* dstHost,
                            SimulationTime barrier) {
    gpu_policy* d = policy->data;
    (void)srcHost; (void)dstHost; (void)barrier;   /* global order: no clamp (global_single.c:40-55) */
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

/* run the engine's rounds below the barrier once per barrier */
static void advance(gpu_policy* d, SimulationTime barrier) {
    if (barrier <= d->advanced || (!d->eng && !d->grp)) return;
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
