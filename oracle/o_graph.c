/*
 * o_graph.c -- TEST INFRASTRUCTURE (oracle).  An igraph-0.7.1-shaped indexed
 * edge list (igraph's published type_indexededgelist.c: undirected edges are
 * stored with from = max(a,b), to = min(a,b); `oi` orders edges by (from,to),
 * `ii` by (to,from); igraph_incident(OUT) lists out-edges then, for undirected
 * graphs, in-edges, so a self-loop appears twice) plus the graph checks of
 * topology.c:450-552 and 724-809.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static const int32_t* g_sort_k1;
static const int32_t* g_sort_k2;
static int cmp_k12(const void* pa, const void* pb) {
    int32_t a = *(const int32_t*)pa, b = *(const int32_t*)pb;
    if (g_sort_k1[a] != g_sort_k1[b]) return g_sort_k1[a] < g_sort_k1[b] ? -1 : 1;
    if (g_sort_k2[a] != g_sort_k2[b]) return g_sort_k2[a] < g_sort_k2[b] ? -1 : 1;
    return a < b ? -1 : (a > b);
}

o_graph* o_graph_new(const shd_graph* in) {
    o_graph* g = calloc(1, sizeof(*g));
    int32_t V = in->n_vertices, E = in->n_edges;
    g->V = V; g->E = E; g->directed = in->directed; g->prefer_direct = in->prefer_direct;
    g->from = malloc(sizeof(int32_t) * (E + 1));
    g->to = malloc(sizeof(int32_t) * (E + 1));
    g->w = malloc(sizeof(double) * (E + 1));
    g->eloss = malloc(sizeof(double) * (E + 1));
    g->vloss = NULL;
    if (in->vertex_loss) {
        g->vloss = malloc(sizeof(double) * (V + 1));
        memcpy(g->vloss, in->vertex_loss, sizeof(double) * V);
    }
    for (int32_t e = 0; e < E; e++) {
        int32_t a = in->edge_src[e], b = in->edge_dst[e];
        if (in->directed || a > b) { g->from[e] = a; g->to[e] = b; }
        else { g->from[e] = b; g->to[e] = a; }
        g->w[e] = in->edge_latency[e];
        g->eloss[e] = in->edge_loss[e];
    }
    g->oi = malloc(sizeof(int32_t) * (E + 1));
    g->ii = malloc(sizeof(int32_t) * (E + 1));
    for (int32_t e = 0; e < E; e++) g->oi[e] = g->ii[e] = e;
    g_sort_k1 = g->from; g_sort_k2 = g->to;
    qsort(g->oi, E, sizeof(int32_t), cmp_k12);
    g_sort_k1 = g->to; g_sort_k2 = g->from;
    qsort(g->ii, E, sizeof(int32_t), cmp_k12);
    g->os = calloc(V + 1, sizeof(int32_t));
    g->is = calloc(V + 1, sizeof(int32_t));
    for (int32_t e = 0; e < E; e++) { g->os[g->from[e] + 1]++; g->is[g->to[e] + 1]++; }
    for (int32_t v = 0; v < V; v++) { g->os[v + 1] += g->os[v]; g->is[v + 1] += g->is[v]; }
    return g;
}

void o_graph_free(o_graph* g) {
    if (!g) return;
    free(g->from); free(g->to); free(g->w); free(g->eloss); free(g->vloss);
    free(g->oi); free(g->ii); free(g->os); free(g->is); free(g);
}

int32_t o_incident_count(const o_graph* g, int32_t v) {
    int32_t n = g->os[v + 1] - g->os[v];
    if (!g->directed) n += g->is[v + 1] - g->is[v];
    return n;
}

int32_t o_incident(const o_graph* g, int32_t v, int32_t* eids, int32_t cap) {
    int32_t n = 0;
    for (int32_t i = g->os[v]; i < g->os[v + 1]; i++) { if (n < cap) eids[n] = g->oi[i]; n++; }
    if (!g->directed)
        for (int32_t i = g->is[v]; i < g->is[v + 1]; i++) { if (n < cap) eids[n] = g->ii[i]; n++; }
    return n;
}

int32_t o_get_eid(const o_graph* g, int32_t a, int32_t b) {
    /* binary search in the (from,to,eid)-sorted index, as igraph_get_eid does;
     * the first match is the lowest eid among parallel edges */
    int32_t from = a, to = b;
    if (!g->directed && a < b) { from = b; to = a; }
    int32_t lo = g->os[from], hi = g->os[from + 1];
    while (lo < hi) {
        int32_t mid = lo + (hi - lo) / 2;
        if (g->to[g->oi[mid]] < to) lo = mid + 1; else hi = mid;
    }
    if (lo < g->os[from + 1] && g->to[g->oi[lo]] == to) return g->oi[lo];
    return -1;
}

/* strongly connected with one cluster (topology.c:738-806) and the
 * completeness test of _topology_isComplete (topology.c:450-552) */
int o_graph_props(const o_graph* g, shd_graph_props* out) {
    memset(out, 0, sizeof(*out));
    int32_t V = g->V;
    out->is_directed = g->directed;
    out->prefer_direct = g->prefer_direct;
    int32_t* stack = malloc(sizeof(int32_t) * (V + 1));
    char* seen = calloc(V + 1, 1);
    int connected = 1;
    for (int pass = 0; pass < (g->directed ? 2 : 1) && V > 0; pass++) {
        memset(seen, 0, V);
        int32_t sp = 0, nseen = 1;
        stack[sp++] = 0; seen[0] = 1;
        while (sp) {
            int32_t v = stack[--sp];
            /* pass 0: follow out-edges (from==v -> to); pass 1: reversed */
            for (int32_t i = g->os[v]; i < g->os[v + 1]; i++) {
                int32_t e = g->oi[i];
                int32_t u = g->to[e];
                if (pass == 1) break;
                if (!seen[u]) { seen[u] = 1; nseen++; stack[sp++] = u; }
            }
            for (int32_t i = g->is[v]; i < g->is[v + 1]; i++) {
                int32_t e = g->ii[i];
                int32_t u = g->from[e];
                if (g->directed && pass == 0) break;
                if (!seen[u]) { seen[u] = 1; nseen++; stack[sp++] = u; }
            }
        }
        if (nseen != V) connected = 0;
    }
    out->is_connected = connected;
    int complete = 1;
    int32_t maxdeg = 0;
    for (int32_t v = 0; v < V; v++) {
        int32_t ecount = o_incident_count(g, v);
        if (ecount > maxdeg) maxdeg = ecount;
        if (o_get_eid(g, v, v) >= 0) {
            out->n_self_loops++;
            if (!g->directed) ecount -= 1;
        }
        if (ecount < V) complete = 0;
    }
    out->is_complete = complete;
    out->max_out_degree = maxdeg;
    free(stack); free(seen);
    return 0;
}
