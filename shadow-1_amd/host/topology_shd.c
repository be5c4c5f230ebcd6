/*
 * topology_shd.c -- Shadow's Topology API (src/main/routing/topology.h:17-28)
 * implemented over libshdgpu.  Linking this file into Shadow in place of
 * src/main/routing/topology.c moves the path cache to the GPU without touching
 * its callers (master.c:224/115, host.c:181/243/1227, worker.c:284-296,
 * master.c:484 via tcp.c:388-389).
 *
 * The signatures are the reference's, with glib's types spelled as their C
 * equivalents on x86-64 Linux (gchar = char, gdouble = double, gboolean = int,
 * guint64 = unsigned long); tests/test_boundary_cpu.py compiles this file with
 * the reference header force-included, so any drift is a compile error.
 * Address and Random stay opaque: the three functions below are Shadow's own
 * (address.c, random.c, worker.c) and are resolved when Shadow links this.
 *
 *   topology_new          topology.c:2486-2510  graphml load + validation
 *                                               (shd_graphml_load_file, shd_graph_check)
 *   topology_attach       topology.c:2371-2430  shd_topology_attach_cb with the host's Random
 *   topology_detach       topology.c:2432-2443
 *   topology_getLatency / getReliability / isRoutable / incrementPathPacketCounter
 *                         topology.c:2053-2092  shd_pc_lookup / shd_pc_count_packet (the
 *                                               lazy first-touch semantics)
 *   worker_updateMinTimeJump upcall             topology.c:1374-1385 (on every decrease)
 *
 * The path cache is built on the GPU at the first lookup after the hosts
 * attached (Shadow registers every host before the first event runs,
 * master.c:394-397); an attach after that rebuilds it, which drops the
 * first-touch history, as a second topology_new would.  Errors follow the
 * reference: NULL from topology_new, -1 latency / reliability, FALSE.
 * Threading: one lock serializes the calls, as the reference's graphLock does
 * for its cache misses (topology.c:1747).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/shdgpu.h"

typedef struct _Topology Topology;
typedef struct _Address Address;
typedef struct _Random Random;

/* Shadow's own functions (address.c, random.c:39-43, worker.c:429-432) */
extern unsigned int address_toHostIP(Address* address);
extern double random_nextDouble(Random* random);
extern void worker_updateMinTimeJump(double minPathLatency);

struct _Topology {
    shd_graphml* gm;
    shd_pc* pc;
    int device;
    int dirty;                    /* attachments changed since the cache was built */
    int32_t* hosts_on;            /* [V] hosts attached per vertex */
    uint32_t* ip_key;             /* open addressing: host-order IP -> vertex */
    int32_t* ip_vert;
    size_t cap, n;
    double reported_min;          /* last minimum latency sent to the worker */
    pthread_mutex_t lock;
};

static size_t ip_slot(const Topology* t, uint32_t ip) {
    size_t i = (ip * 2654435761u) & (t->cap - 1);
    while (t->ip_vert[i] != -1 && t->ip_key[i] != ip) i = (i + 1) & (t->cap - 1);
    return i;
}

static int ip_put(Topology* t, uint32_t ip, int32_t v) {
    if (2 * (t->n + 1) > t->cap) {
        size_t oc = t->cap, nc = oc ? 2 * oc : 1024;
        uint32_t* ok = t->ip_key;
        int32_t* ov = t->ip_vert;
        t->ip_key = malloc(sizeof(uint32_t) * nc);
        t->ip_vert = malloc(sizeof(int32_t) * nc);
        if (!t->ip_key || !t->ip_vert) return -1;
        for (size_t i = 0; i < nc; i++) t->ip_vert[i] = -1;
        t->cap = nc;
        t->n = 0;
        for (size_t i = 0; i < oc; i++)
            if (ov[i] >= 0) {
                size_t j = ip_slot(t, ok[i]);
                t->ip_key[j] = ok[i];
                t->ip_vert[j] = ov[i];
                t->n++;
            }
        free(ok);
        free(ov);
    }
    size_t i = ip_slot(t, ip);
    if (t->ip_vert[i] < 0) t->n++;
    t->ip_key[i] = ip;
    t->ip_vert[i] = v;
    return 0;
}

static int32_t ip_get(const Topology* t, uint32_t ip) {
    if (!t->cap) return -1;
    return t->ip_vert[ip_slot(t, ip)];
}

/* a removal keeps the probe chains intact: the slots after it are re-put */
static void ip_del(Topology* t, uint32_t ip) {
    if (!t->cap) return;
    size_t i = ip_slot(t, ip);
    if (t->ip_vert[i] < 0) return;
    t->ip_vert[i] = -1;
    t->n--;
    for (size_t j = (i + 1) & (t->cap - 1); t->ip_vert[j] >= 0; j = (j + 1) & (t->cap - 1)) {
        uint32_t k = t->ip_key[j];
        int32_t v = t->ip_vert[j];
        t->ip_vert[j] = -1;
        t->n--;
        ip_put(t, k, v);
    }
}

Topology* topology_new(const char* graphPath) {
    shd_graphml* gm = NULL;
    if (!graphPath || shd_graphml_load_file(graphPath, &gm) != SHD_OK) return NULL;
    shd_graph_props props;
    /* _topology_checkGraph (topology.c:1187-1210): invalid graphs give NULL */
    if (shd_graph_check(&gm->g, &props) != SHD_OK || !props.is_connected) {
        shd_graphml_free(gm);
        return NULL;
    }
    Topology* t = calloc(1, sizeof(*t));
    if (!t) { shd_graphml_free(gm); return NULL; }
    t->gm = gm;
    t->hosts_on = calloc((size_t)gm->g.n_vertices, sizeof(int32_t));
    const char* dev = getenv("SHD_DEVICE");
    t->device = dev ? atoi(dev) : 0;
    t->dirty = 1;
    pthread_mutex_init(&t->lock, NULL);
    return t;
}

void topology_free(Topology* t) {
    if (!t) return;
    if (t->pc) shd_pc_destroy(t->pc);
    shd_graphml_free(t->gm);
    free(t->hosts_on);
    free(t->ip_key);
    free(t->ip_vert);
    pthread_mutex_destroy(&t->lock);
    free(t);
}

static double draw(void* r) { return random_nextDouble((Random*)r); }

void topology_attach(Topology* t, Address* address, Random* randomSourcePool, char* ipHint, char* citycodeHint,
                     char* countrycodeHint, char* geocodeHint, char* typeHint, unsigned long* bwDownOut,
                     unsigned long* bwUpOut) {
    if (!t || !address || !randomSourcePool) return;
    int32_t v = -1;
    uint64_t down = 0, up = 0;
    if (shd_topology_attach_cb(t->gm, draw, randomSourcePool, ipHint, citycodeHint, countrycodeHint, geocodeHint,
                               typeHint, &v, &down, &up) != SHD_OK)
        return;
    pthread_mutex_lock(&t->lock);
    if (ip_put(t, address_toHostIP(address), v) == 0) {
        if (t->hosts_on[v]++ == 0) t->dirty = 1;   /* a new attached vertex: new rows */
    }
    pthread_mutex_unlock(&t->lock);
    if (bwDownOut) *bwDownOut = (unsigned long)down;
    if (bwUpOut) *bwUpOut = (unsigned long)up;
}

void topology_detach(Topology* t, Address* address) {
    if (!t || !address) return;
    pthread_mutex_lock(&t->lock);
    ip_del(t, address_toHostIP(address));   /* the virtualIP entry goes; cached paths stay */
    pthread_mutex_unlock(&t->lock);
}

/* (re)build the cache over the vertices with attached hosts (topology.c:2393) */
static int ensure_built(Topology* t) {
    if (!t->dirty && t->pc) return 0;
    const int32_t V = t->gm->g.n_vertices;
    int32_t* att = malloc(sizeof(int32_t) * (size_t)(V + 1));
    int32_t na = 0;
    for (int32_t v = 0; v < V; v++) if (t->hosts_on[v] > 0) att[na++] = v;
    if (t->pc) { shd_pc_destroy(t->pc); t->pc = NULL; }
    int rc = na ? shd_pc_create(&t->gm->g, att, na, 0, t->device, &t->pc) : SHD_EINVAL;
    free(att);
    if (rc == SHD_OK) rc = shd_pc_build(t->pc);
    if (rc != SHD_OK) {
        if (t->pc) shd_pc_destroy(t->pc);
        t->pc = NULL;
        return -1;
    }
    t->dirty = 0;
    t->reported_min = 0;
    return 0;
}

/* the cache entry of the pair (0) or -1 (unknown address, no path) */
static int lookup_locked(Topology* t, Address* src, Address* dst, double* lat, double* rel) {
    if (!src || !dst || ensure_built(t)) return -1;
    const int32_t s = ip_get(t, address_toHostIP(src)), d = ip_get(t, address_toHostIP(dst));
    if (s < 0 || d < 0) return -1;
    if (shd_pc_lookup(t->pc, s, d, lat, rel) != SHD_OK || *lat < 0) return -1;
    double mn = 0;
    shd_pc_min_stored_latency(t->pc, &mn);
    if (mn > 0 && (t->reported_min == 0 || mn < t->reported_min)) {
        t->reported_min = mn;
        worker_updateMinTimeJump(mn);   /* topology.c:1383-1385 */
    }
    return 0;
}

int topology_isRoutable(Topology* t, Address* srcAddress, Address* dstAddress) {
    if (!t) return 0;
    double lat, rel;
    pthread_mutex_lock(&t->lock);
    const int ok = lookup_locked(t, srcAddress, dstAddress, &lat, &rel) == 0;
    pthread_mutex_unlock(&t->lock);
    return ok;
}

double topology_getLatency(Topology* t, Address* srcAddress, Address* dstAddress) {
    if (!t) return -1;
    double lat = -1, rel = -1;
    pthread_mutex_lock(&t->lock);
    if (lookup_locked(t, srcAddress, dstAddress, &lat, &rel)) lat = -1;
    pthread_mutex_unlock(&t->lock);
    return lat;
}

double topology_getReliability(Topology* t, Address* srcAddress, Address* dstAddress) {
    if (!t) return -1;
    double lat = -1, rel = -1;
    pthread_mutex_lock(&t->lock);
    if (lookup_locked(t, srcAddress, dstAddress, &lat, &rel)) rel = -1;
    pthread_mutex_unlock(&t->lock);
    return rel;
}

void topology_incrementPathPacketCounter(Topology* t, Address* srcAddress, Address* dstAddress) {
    if (!t || !srcAddress || !dstAddress) return;
    pthread_mutex_lock(&t->lock);
    if (ensure_built(t) == 0) {
        const int32_t s = ip_get(t, address_toHostIP(srcAddress)), d = ip_get(t, address_toHostIP(dstAddress));
        if (s >= 0 && d >= 0) shd_pc_count_packet(t->pc, s, d);
    }
    pthread_mutex_unlock(&t->lock);
}

/* not in topology.h: read back a path's packet count (what topology_free logs,
 * _topology_logAllCachedPaths, topology.c:1929-1965) */
unsigned long topology_shd_getPathPacketCount(Topology* t, Address* srcAddress, Address* dstAddress) {
    uint64_t n = 0;
    if (!t || !srcAddress || !dstAddress) return 0;
    pthread_mutex_lock(&t->lock);
    const int32_t s = ip_get(t, address_toHostIP(srcAddress)), d = ip_get(t, address_toHostIP(dstAddress));
    if (t->pc && s >= 0 && d >= 0) shd_pc_packet_count(t->pc, s, d, &n);
    pthread_mutex_unlock(&t->lock);
    return (unsigned long)n;
}
