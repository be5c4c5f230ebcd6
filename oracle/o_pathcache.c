/*
 * o_pathcache.c -- TEST INFRASTRUCTURE (oracle).  Restates the path cache of
 * src/main/routing/topology.c:
 *   _topology_getEdgeHelper            402-444
 *   _topology_computePathProperties    1407-1523
 *   _topology_computeShortestPathToSelf 1545-1653
 *   _topology_computeSourcePaths       1655-1875
 *   _topology_lookupDirectPath         1877-1927
 *   _topology_shouldStorePath / storePathInCache 1307-1386
 *   _topology_getPathEntry             1969-2051
 * and igraph 0.7.1 igraph_get_shortest_paths_dijkstra as published
 * (structural_properties.c: 2-way indexed max-heap on -distance, relax in
 * igraph_incident order, first finite distance or strictly shorter wins,
 * early exit once every target is popped, path to the source = [source]).
 * igraph is absent from the image: its tie-breaking is restated, not pinned.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ---------------- igraph_2wheap_t (published igraph heap.c) ---------------- */
typedef struct { double* data; int32_t* index; int32_t* index2; int32_t size; } wheap;
#define PARENT(x) (((x) + 1) / 2 - 1)
#define LEFTCHILD(x) (((x) + 1) * 2 - 1)
#define RIGHTCHILD(x) (((x) + 1) * 2)

static void wh_switch(wheap* h, int32_t e1, int32_t e2) {
    if (e1 == e2) return;
    int32_t tmp1 = h->index[e1], tmp2 = h->index[e2];
    h->index2[tmp1] = e2 + 2;
    h->index2[tmp2] = e1 + 2;
    h->index[e1] = tmp2; h->index[e2] = tmp1;
    double t = h->data[e1]; h->data[e1] = h->data[e2]; h->data[e2] = t;
}
static void wh_shift_up(wheap* h, int32_t elem) {
    while (!(elem == 0 || h->data[elem] < h->data[PARENT(elem)])) {
        wh_switch(h, elem, PARENT(elem));
        elem = PARENT(elem);
    }
}
static void wh_sink(wheap* h, int32_t head) {
    for (;;) {
        int32_t size = h->size;
        if (LEFTCHILD(head) >= size) return;
        if (RIGHTCHILD(head) == size || h->data[LEFTCHILD(head)] >= h->data[RIGHTCHILD(head)]) {
            if (h->data[head] < h->data[LEFTCHILD(head)]) {
                wh_switch(h, head, LEFTCHILD(head)); head = LEFTCHILD(head);
            } else return;
        } else {
            if (h->data[head] < h->data[RIGHTCHILD(head)]) {
                wh_switch(h, head, RIGHTCHILD(head)); head = RIGHTCHILD(head);
            } else return;
        }
    }
}
static void wh_push(wheap* h, int32_t idx, double elem) {
    int32_t size = h->size++;
    h->data[size] = elem; h->index[size] = idx; h->index2[idx] = size + 2;
    wh_shift_up(h, size);
}
static int32_t wh_max_index(wheap* h) { return h->index[0]; }
static double wh_delete_max(wheap* h) {
    double tmp = h->data[0];
    int32_t tmpidx = h->index[0];
    wh_switch(h, 0, h->size - 1);
    h->size--;
    h->index2[tmpidx] = 0;
    wh_sink(h, 0);
    return tmp;
}
static void wh_modify(wheap* h, int32_t idx, double elem) {
    int32_t pos = h->index2[idx] - 2;
    h->data[pos] = elem;
    wh_sink(h, pos);
    wh_shift_up(h, pos);
}

static inline int32_t other_end(const o_graph* g, int32_t e, int32_t v) {
    return g->from[e] == v ? g->to[e] : g->from[e];
}
/* only OUT-mode neighbours of a directed graph: the head of the edge */
static inline int32_t out_head(const o_graph* g, int32_t e, int32_t v) {
    return g->directed ? g->to[e] : other_end(g, e, v);
}

/* vertex reliability factor present? (_topology_findVertexAttributeDouble) */
static inline int vrel(const o_graph* g, int32_t v, double* r) {
    if (!g->vloss) return 0;
    double l = g->vloss[v];
    if (isnan(l)) return 0;
    *r = (1.0f - l);
    return 1;
}

/* _topology_lookupDirectPath, topology.c:1877-1927 */
int o_direct_path(const o_graph* g, int32_t s, int32_t d, double* lat, double* rel) {
    double totalLatency = 0.0, totalReliability = 1.0, r;
    if (vrel(g, s, &r)) totalReliability *= r;
    if (vrel(g, d, &r)) totalReliability *= r;
    int32_t e = o_get_eid(g, s, d);
    if (e < 0) { *lat = -1; *rel = -1; return -1; }
    totalLatency += g->w[e];
    totalReliability *= (1.0f - g->eloss[e]);
    *lat = totalLatency; *rel = totalReliability;
    return 0;
}

/* _topology_computeShortestPathToSelf, topology.c:1545-1653: min latency over
 * incident OUT edges (first strict minimum, 1592), latency 2*min, reliability
 * r(e)^2; no vertex loss factor */
int o_self_path(const o_graph* g, int32_t s, double* lat, double* rel) {
    double minLatency = 0.0f, relMin = 0.0f;
    int32_t n = o_incident_count(g, s);
    int32_t* eids = malloc(sizeof(int32_t) * (n + 1));
    o_incident(g, s, eids, n);
    for (int32_t i = 0; i < n; i++) {
        int32_t e = eids[i];
        double el = g->w[e];
        if (minLatency == 0 || el < minLatency) {
            minLatency = el;
            relMin = 1.0f - g->eloss[e];
        }
    }
    free(eids);
    if (n == 0) { *lat = -1; *rel = -1; return -1; }
    *lat = 2.0f * minLatency;
    *rel = relMin * relMin;
    return 0;
}

/* _topology_computePathProperties, topology.c:1407-1523 over a vertex path */
static int path_properties(const o_graph* g, int32_t src, const int32_t* pv, int32_t nV,
                           double* lat, double* rel) {
    double totalLatency = 0.0, totalReliability = (double)1, r;
    if (vrel(g, src, &r)) totalReliability *= r;
    int32_t target = pv[nV - 1];
    if ((src != target) || (src == target && nV > 2)) {
        if (vrel(g, target, &r)) totalReliability *= r;
    }
    int32_t start = nV == 1 ? 0 : 1;
    int32_t fromV = src;
    for (int32_t i = start; i < nV; i++) {
        int32_t toV = pv[i];
        int32_t e = o_get_eid(g, fromV, toV);
        if (e < 0) return -1;
        totalLatency += g->w[e];
        totalReliability *= (1.0f - g->eloss[e]);
        fromV = toV;
    }
    *lat = totalLatency; *rel = totalReliability;
    return 0;
}

int o_sssp_row(const o_graph* g, int32_t src, const int32_t* targets, int32_t nt,
               double* lat, double* rel, int32_t* ok, int32_t* hops, int64_t* ties) {
    int32_t V = g->V;
    double* dists = malloc(sizeof(double) * V);
    int32_t* parent = calloc(V, sizeof(int32_t));   /* eid+1, 0 = none */
    char* is_target = calloc(V, 1);
    wheap h;
    h.data = malloc(sizeof(double) * (V + 1));
    h.index = malloc(sizeof(int32_t) * (V + 1));
    h.index2 = calloc(V + 1, sizeof(int32_t));
    h.size = 0;
    for (int32_t v = 0; v < V; v++) dists[v] = -1.0;
    int32_t to_reach = nt;
    for (int32_t j = 0; j < nt; j++) {
        if (!is_target[targets[j]]) is_target[targets[j]] = 1; else to_reach--;
    }
    dists[src] = 0.0;
    parent[src] = 0;
    wh_push(&h, src, 0);
    int32_t maxdeg = 0;
    for (int32_t v = 0; v < V; v++) { int32_t c = o_incident_count(g, v); if (c > maxdeg) maxdeg = c; }
    int32_t* neis = malloc(sizeof(int32_t) * (maxdeg + 1));
    while (h.size > 0 && to_reach > 0) {
        int32_t minnei = wh_max_index(&h);
        double mindist = -wh_delete_max(&h);
        if (is_target[minnei]) { is_target[minnei] = 0; to_reach--; }
        int32_t nlen;
        if (g->directed) {   /* lazy inclist, mode OUT on a directed graph */
            nlen = 0;
            for (int32_t i = g->os[minnei]; i < g->os[minnei + 1]; i++) neis[nlen++] = g->oi[i];
        } else {
            nlen = o_incident(g, minnei, neis, maxdeg + 1);
        }
        for (int32_t i = 0; i < nlen; i++) {
            int32_t edge = neis[i];
            int32_t tto = out_head(g, edge, minnei);
            double altdist = mindist + g->w[edge];
            double curdist = dists[tto];
            if (curdist < 0) {
                dists[tto] = altdist; parent[tto] = edge + 1;
                wh_push(&h, tto, -altdist);
            } else if (altdist < curdist) {
                dists[tto] = altdist; parent[tto] = edge + 1;
                wh_modify(&h, tto, -altdist);
            }
        }
    }
    /* count vertices whose final distance is reached by more than one
     * predecessor with the minimal predecessor distance (unpinned ties) */
    int64_t nties = 0;
    int32_t* inc = ties ? malloc(sizeof(int32_t) * (2 * (size_t)(maxdeg + 1) + 1)) : NULL;
    for (int32_t v = 0; v < V && ties; v++) {
        if (v == src || dists[v] < 0) continue;
        double bestd = -1; int32_t nbest = 0;
        /* scan in-arcs: the incident list for undirected graphs */
        int32_t m = 0;
        if (g->directed) {
            for (int32_t i = g->is[v]; i < g->is[v + 1] && m < 2 * (maxdeg + 1); i++) inc[m++] = g->ii[i];
        } else {
            m = o_incident(g, v, inc, 2 * (maxdeg + 1));
        }
        for (int32_t i = 0; i < m; i++) {
            int32_t e = inc[i];
            int32_t u = g->directed ? g->from[e] : other_end(g, e, v);
            if (u == v || dists[u] < 0) continue;
            if (dists[u] + g->w[e] == dists[v]) {
                if (nbest == 0 || dists[u] < bestd) { bestd = dists[u]; nbest = 1; }
                else if (dists[u] == bestd) nbest++;
            }
        }
        if (nbest > 1) nties++;
    }
    free(inc);
    if (ties) *ties = nties;
    /* paths (igraph 0.7.1: walk parent eids; path to the source = [source]) */
    int32_t* pv = malloc(sizeof(int32_t) * (V + 1));
    for (int32_t j = 0; j < nt; j++) {
        int32_t node = targets[j];
        int32_t size = 0, act = node;
        while (parent[act]) { size++; act = other_end(g, parent[act] - 1, act); }
        pv[size] = node;
        act = node;
        int32_t k = size;
        while (parent[act]) { act = other_end(g, parent[act] - 1, act); pv[--k] = act; }
        int32_t nV = size + 1;
        if (hops) hops[j] = size;
        double l = -1, r = -1;
        int rc = path_properties(g, src, pv, nV, &l, &r);
        if (rc == 0 && l == 0) l = 1;   /* topology.c:1848-1852 */
        lat[j] = l; rel[j] = r;
        if (ok) ok[j] = (rc == 0);
    }
    free(pv); free(neis); free(dists); free(parent); free(is_target);
    free(h.data); free(h.index); free(h.index2);
    return 0;
}

/* ------------------------ lazy cache (topology.c:1284-2051) ------------------------ */
typedef struct { uint64_t key; double lat, rel; uint64_t count; int32_t used, direct; } slot_t;
struct o_topo {
    const o_graph* g;
    shd_graph_props props;
    int32_t* targets; int32_t nt;
    slot_t* tab; uint64_t cap, n;
    double min_latency;
    int32_t rows_run, self_run;
    int32_t force_rows;
    /* optional precomputed source rows by vertex (o_topo_set_row_cache): the
     * values _topology_computeSourcePaths would compute (order-independent),
     * NaN latency where computePathProperties fails; [V] pointers or NULL */
    double** row_lat;
    double** row_rel;
    uint8_t* ran;   /* [V] a source row of this vertex has run */
    int owns_rows;  /* row_lat / row_rel from o_topo_precompute_rows */
};

static uint64_t hkey(int32_t s, int32_t d) { return ((uint64_t)(uint32_t)s << 32) | (uint32_t)d; }
static uint64_t hmix(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
    return k;
}
static slot_t* tab_find(o_topo* t, int32_t s, int32_t d) {
    uint64_t k = hkey(s, d), i = hmix(k) & (t->cap - 1);
    while (t->tab[i].used) {
        if (t->tab[i].key == k) return &t->tab[i];
        i = (i + 1) & (t->cap - 1);
    }
    return NULL;
}
static void tab_insert(o_topo* t, int32_t s, int32_t d, double lat, double rel, int direct) {
    if ((t->n + 1) * 2 > t->cap) {
        uint64_t oc = t->cap; slot_t* old = t->tab;
        t->cap = oc * 2; t->tab = calloc(t->cap, sizeof(slot_t)); t->n = 0;
        for (uint64_t i = 0; i < oc; i++)
            if (old[i].used) {
                uint64_t j = hmix(old[i].key) & (t->cap - 1);
                while (t->tab[j].used) j = (j + 1) & (t->cap - 1);
                t->tab[j] = old[i]; t->n++;
            }
        free(old);
    }
    uint64_t k = hkey(s, d), i = hmix(k) & (t->cap - 1);
    while (t->tab[i].used) i = (i + 1) & (t->cap - 1);
    t->tab[i].used = 1; t->tab[i].key = k; t->tab[i].lat = lat; t->tab[i].rel = rel;
    t->tab[i].count = 0; t->tab[i].direct = direct;
    t->n++;
}

o_topo* o_topo_new(const o_graph* g, const int32_t* attached, int32_t n_attached, int32_t force_rows) {
    o_topo* t = calloc(1, sizeof(*t));
    t->g = g;
    o_graph_props(g, &t->props);
    t->force_rows = force_rows;
    if (force_rows) t->props.is_complete = 0;
    t->nt = n_attached;
    t->targets = malloc(sizeof(int32_t) * (n_attached + 1));
    memcpy(t->targets, attached, sizeof(int32_t) * n_attached);
    t->cap = 1024; t->tab = calloc(t->cap, sizeof(slot_t));
    t->ran = calloc(g->V > 0 ? g->V : 1, 1);
    return t;
}
void o_topo_free(o_topo* t) {
    if (!t) return;
    if (t->owns_rows) {
        for (int32_t v = 0; v < t->g->V; v++) { free(t->row_lat[v]); free(t->row_rel[v]); }
        free(t->row_lat); free(t->row_rel);
    }
    free(t->targets); free(t->tab); free(t->ran); free(t);
}

static slot_t* from_cache(o_topo* t, int32_t s, int32_t d) { return tab_find(t, s, d); }

/* _topology_shouldStorePath + _topology_storePathInCache (1307-1386) */
static void store(o_topo* t, int direct, int32_t s, int32_t d, double lat, double rel) {
    if (from_cache(t, s, d) || from_cache(t, d, s)) return;
    if (t->props.is_complete && !direct) return;
    if (t->g->prefer_direct && !direct && o_get_eid(t->g, s, d) >= 0) return;
    tab_insert(t, s, d, lat, rel, direct);
    if (t->min_latency == 0 || lat < t->min_latency) t->min_latency = lat;
}

static int compute_source_paths(o_topo* t, int32_t s, int32_t d) {
    if (s == d) {
        double lat, rel;
        if (o_self_path(t->g, s, &lat, &rel) != 0) return 0;
        t->self_run++;
        store(t, 0, s, s, lat, rel);
        return 1;
    }
    double* lat = malloc(sizeof(double) * t->nt);
    double* rel = malloc(sizeof(double) * t->nt);
    int32_t* ok = malloc(sizeof(int32_t) * t->nt);
    if (t->row_lat && t->row_lat[s]) {
        for (int32_t j = 0; j < t->nt; j++) {
            lat[j] = t->row_lat[s][j]; rel[j] = t->row_rel[s][j]; ok[j] = !isnan(lat[j]);
        }
    } else {
        o_sssp_row(t->g, s, t->targets, t->nt, lat, rel, ok, NULL, NULL);
    }
    t->rows_run++;
    t->ran[s] = 1;
    int all = 1;
    for (int32_t j = 0; j < t->nt; j++) {
        if (ok[j]) store(t, 0, s, t->targets[j], lat[j], rel[j]);
        else all = 0;
    }
    free(lat); free(rel); free(ok);
    return all;
}

static slot_t* get_path_entry(o_topo* t, int32_t s, int32_t d) {
    slot_t* p = from_cache(t, s, d);
    if (!p && !t->g->directed) p = from_cache(t, d, s);
    if (!p) {
        int success;
        int adjacent = o_get_eid(t->g, s, d) >= 0;
        if (t->props.is_complete || (t->g->prefer_direct && adjacent)) {
            double lat, rel;
            success = o_direct_path(t->g, s, d, &lat, &rel) == 0;
            if (success) store(t, 1, s, d, lat, rel);
        } else {
            success = compute_source_paths(t, s, d);
        }
        if (success) {
            p = from_cache(t, s, d);
            if (!p) p = from_cache(t, d, s);
        }
    }
    return p;
}

int o_topo_get(o_topo* t, int32_t s, int32_t d, double* lat, double* rel) {
    slot_t* p = get_path_entry(t, s, d);
    if (!p) { *lat = -1; *rel = -1; return -1; }
    *lat = p->lat; *rel = p->rel;
    return 0;
}
void o_topo_count_packet(o_topo* t, int32_t s, int32_t d) {
    slot_t* p = get_path_entry(t, s, d);
    if (p) p->count++;
}
uint64_t o_topo_packet_count(o_topo* t, int32_t s, int32_t d) {
    slot_t* p = from_cache(t, s, d);
    if (!p && !t->g->directed) p = from_cache(t, d, s);
    return p ? p->count : 0;
}
uint64_t o_topo_stored_count(o_topo* t, int32_t s, int32_t d) {
    slot_t* p = from_cache(t, s, d);
    return p ? p->count : 0;
}
double o_topo_min_latency(o_topo* t) { return t->min_latency; }
int32_t o_topo_rows_run(o_topo* t) { return t->rows_run; }
int32_t o_topo_self_run(o_topo* t) { return t->self_run; }

/* every attached vertex's source row on `threads` cores, kept by the cache
 * (the values _topology_computeSourcePaths computes do not depend on when it
 * runs): bench.py times the reference's own loop over this cache with the rows
 * already there, as it times the port (o_state_rows) */
#include <pthread.h>
typedef struct { o_topo* t; int32_t next; pthread_mutex_t mu; } prow_job;
static void* prow_worker(void* arg) {
    prow_job* J = arg;
    o_topo* t = J->t;
    int32_t* ok = malloc(sizeof(int32_t) * (t->nt + 1));
    for (;;) {
        pthread_mutex_lock(&J->mu);
        int32_t j = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (j >= t->nt) break;
        int32_t v = t->targets[j];
        double* lat = malloc(sizeof(double) * t->nt);
        double* rel = malloc(sizeof(double) * t->nt);
        o_sssp_row(t->g, v, t->targets, t->nt, lat, rel, ok, NULL, NULL);
        for (int32_t k = 0; k < t->nt; k++) if (!ok[k]) lat[k] = NAN;
        t->row_lat[v] = lat; t->row_rel[v] = rel;
    }
    free(ok);
    return NULL;
}
void o_topo_precompute_rows(o_topo* t, int threads) {
    if (t->row_lat) return;
    t->row_lat = calloc(t->g->V, sizeof(double*));
    t->row_rel = calloc(t->g->V, sizeof(double*));
    t->owns_rows = 1;
    prow_job J = {t, 0, PTHREAD_MUTEX_INITIALIZER};
    if (threads < 1) threads = 1;
    pthread_t* th = malloc(sizeof(pthread_t) * threads);
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, prow_worker, &J);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    free(th);
}

/* ---------------- support for the parallel baseline (o_baseline.c) ---------------- */
void o_topo_set_row_cache(o_topo* t, double** row_lat, double** row_rel) { t->row_lat = row_lat; t->row_rel = row_rel; }
int32_t o_topo_n_targets(const o_topo* t) { return t->nt; }
const int32_t* o_topo_targets(const o_topo* t) { return t->targets; }
int o_topo_is_complete(const o_topo* t) { return t->props.is_complete; }

/* read-only lookup (no row runs, no stores; safe for concurrent readers): 1
 * and the stored value when the pair has an entry in either orientation */
int o_topo_peek(const o_topo* t, int32_t s, int32_t d, double* lat, double* rel) {
    slot_t* p = tab_find((o_topo*)t, s, d);
    if (!p && !t->g->directed) p = tab_find((o_topo*)t, d, s);
    if (!p) return 0;
    *lat = p->lat; *rel = p->rel;
    return 1;
}

int o_topo_would_run(const o_topo* t, int32_t s, int32_t d) {
    if (tab_find((o_topo*)t, s, d)) return 0;
    if (!t->g->directed && tab_find((o_topo*)t, d, s)) return 0;
    if (t->props.is_complete || (t->g->prefer_direct && o_get_eid(t->g, s, d) >= 0)) return 0;
    /* a directed rerun of a row that ran already (its reverse entry was stored
     * first, topology.c:1987-1990) stores nothing new: not a first touch */
    if (s != d && t->ran[s]) return 0;
    return 1;
}
void o_topo_touch(o_topo* t, int32_t s, int32_t d) { (void)get_path_entry(t, s, d); }

o_topo* o_topo_clone(const o_topo* t) {
    o_topo* c = malloc(sizeof(*c));
    *c = *t;
    c->owns_rows = 0;   /* the rows stay the original's */
    c->ran = malloc(t->g->V > 0 ? t->g->V : 1);
    memcpy(c->ran, t->ran, t->g->V > 0 ? t->g->V : 1);
    c->targets = malloc(sizeof(int32_t) * (t->nt + 1));
    memcpy(c->targets, t->targets, sizeof(int32_t) * t->nt);
    c->tab = malloc(sizeof(slot_t) * t->cap);
    memcpy(c->tab, t->tab, sizeof(slot_t) * t->cap);
    return c;
}
