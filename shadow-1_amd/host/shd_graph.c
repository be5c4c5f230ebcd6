/*
 * shd_graph.c -- host side of libshdgpu: graph indexing and validation,
 * the rand_r RNG and the seed chain, and host attach.
 *
 *   shd_graph_check      topology.c:450-552 (_topology_isComplete),
 *                        724-809 (_topology_checkGraphProperties),
 *                        1041-1124 (edge latency > 0, loss in [0,1])
 *   shd_csr_build        device layout of the graph (see shd_host.h)
 *   shd_rand_r ...       utility/random.c:32-51 (glibc rand_r)
 *   shd_seed_chain       master.c:95,417; slave.c:182,198,301
 *   shd_topology_attach  topology.c:2094-2369 (_topology_findAttachmentVertex)
 */
#include <arpa/inet.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include "shd_host.h"

/* ------------------------------------------------------------------ RNG */
int32_t shd_rand_r(uint32_t* state) {
    uint32_t x = *state;
    uint32_t r;
    x = x * 1103515245u + 12345u;
    r = (x >> 16) & 2047u;
    x = x * 1103515245u + 12345u;
    r = (r << 10) ^ ((x >> 16) & 1023u);
    x = x * 1103515245u + 12345u;
    r = (r << 10) ^ ((x >> 16) & 1023u);
    *state = x;
    return (int32_t)r;
}

double shd_next_double(uint32_t* state) {
    return (double)shd_rand_r(state) / 2147483647.0;
}

uint32_t shd_next_uint(uint32_t* state) {
    double f = shd_next_double(state);
    return (uint32_t)(f * 4294967295.0);
}

int shd_seed_chain(uint32_t options_seed, int32_t n_hosts, uint32_t* host_seeds) {
    if (n_hosts < 0 || (n_hosts > 0 && !host_seeds)) return SHD_EINVAL;
    uint32_t master = options_seed;
    uint32_t slave = shd_next_uint(&master);
    (void)shd_next_uint(&slave);
    for (int32_t i = 0; i < n_hosts; i++) host_seeds[i] = shd_next_uint(&slave);
    return SHD_OK;
}

/* ------------------------------------------------------------------ CSR */
typedef struct { int32_t k1, k2, eid; } key3;
static int cmp_key3(const void* a, const void* b) {
    const key3* x = a; const key3* y = b;
    if (x->k1 != y->k1) return x->k1 < y->k1 ? -1 : 1;
    if (x->k2 != y->k2) return x->k2 < y->k2 ? -1 : 1;
    return x->eid < y->eid ? -1 : (x->eid > y->eid);
}

int shd_csr_build(const shd_graph* g, shd_csr* c) {
    memset(c, 0, sizeof(*c));
    if (!g || g->n_vertices <= 0 || g->n_edges < 0) return SHD_EINVAL;
    int32_t V = g->n_vertices, E = g->n_edges;
    c->V = V; c->E = E; c->directed = g->directed;
    for (int32_t e = 0; e < E; e++) {
        if (g->edge_src[e] < 0 || g->edge_src[e] >= V || g->edge_dst[e] < 0 || g->edge_dst[e] >= V)
            return SHD_EINVAL;
    }
    /* igraph storage: undirected edges with from = max, to = min */
    key3* by_from = malloc(sizeof(key3) * (E + 1));
    key3* by_to = malloc(sizeof(key3) * (E + 1));
    for (int32_t e = 0; e < E; e++) {
        int32_t a = g->edge_src[e], b = g->edge_dst[e];
        int32_t fr = a, to = b;
        if (!g->directed && a < b) { fr = b; to = a; }
        by_from[e] = (key3){fr, to, e};
        by_to[e] = (key3){to, fr, e};
    }
    qsort(by_from, E, sizeof(key3), cmp_key3);
    qsort(by_to, E, sizeof(key3), cmp_key3);
    int32_t* os = calloc(V + 1, sizeof(int32_t));
    int32_t* is = calloc(V + 1, sizeof(int32_t));
    for (int32_t i = 0; i < E; i++) { os[by_from[i].k1 + 1]++; is[by_to[i].k1 + 1]++; }
    for (int32_t v = 0; v < V; v++) { os[v + 1] += os[v]; is[v + 1] += is[v]; }

    /* incidence lists in igraph_incident(OUT) order */
    c->inc_off = calloc(V + 1, sizeof(int32_t));
    for (int32_t v = 0; v < V; v++) {
        int32_t n = os[v + 1] - os[v];
        if (!g->directed) n += is[v + 1] - is[v];
        c->inc_off[v + 1] = c->inc_off[v] + n;
    }
    c->inc_eid = malloc(sizeof(int32_t) * (c->inc_off[V] + 1));
    for (int32_t v = 0; v < V; v++) {
        int32_t k = c->inc_off[v];
        for (int32_t i = os[v]; i < os[v + 1]; i++) c->inc_eid[k++] = by_from[i].eid;
        if (!g->directed)
            for (int32_t i = is[v]; i < is[v + 1]; i++) c->inc_eid[k++] = by_to[i].eid;
    }

    /* relaxation arcs (OUT mode), self-loops dropped */
    c->arc_off = calloc(V + 1, sizeof(int32_t));
    c->rin_off = calloc(V + 1, sizeof(int32_t));
    for (int32_t e = 0; e < E; e++) {
        int32_t a = g->edge_src[e], b = g->edge_dst[e];
        if (a == b) continue;
        c->arc_off[a + 1]++;
        c->rin_off[b + 1]++;
        if (!g->directed) { c->arc_off[b + 1]++; c->rin_off[a + 1]++; }
    }
    for (int32_t v = 0; v < V; v++) { c->arc_off[v + 1] += c->arc_off[v]; c->rin_off[v + 1] += c->rin_off[v]; }
    int32_t na = c->arc_off[V];
    c->arc_dst = malloc(sizeof(int32_t) * (na + 1));
    c->arc_eid = malloc(sizeof(int32_t) * (na + 1));
    c->arc_w = malloc(sizeof(double) * (na + 1));
    c->rin_src = malloc(sizeof(int32_t) * (na + 1));
    c->rin_eid = malloc(sizeof(int32_t) * (na + 1));
    c->rin_w = malloc(sizeof(double) * (na + 1));
    /* order arcs of each vertex by the igraph incidence order (ties only) */
    int32_t* fill = malloc(sizeof(int32_t) * (V + 1));
    memcpy(fill, c->arc_off, sizeof(int32_t) * (V + 1));
    for (int32_t v = 0; v < V; v++) {
        for (int32_t k = c->inc_off[v]; k < c->inc_off[v + 1]; k++) {
            int32_t e = c->inc_eid[k];
            int32_t a = g->edge_src[e], b = g->edge_dst[e];
            if (a == b) continue;
            int32_t head;
            if (g->directed) { if (a != v) continue; head = b; }
            else head = (a == v) ? b : a;
            int32_t p = fill[v]++;
            c->arc_dst[p] = head; c->arc_eid[p] = e; c->arc_w[p] = g->edge_latency[e];
        }
    }
    memcpy(fill, c->rin_off, sizeof(int32_t) * (V + 1));
    for (int32_t v = 0; v < V; v++) {
        for (int32_t p = c->arc_off[v]; p < c->arc_off[v + 1]; p++) {
            int32_t x = c->arc_dst[p];
            int32_t q = fill[x]++;
            c->rin_src[q] = v; c->rin_eid[q] = c->arc_eid[p]; c->rin_w[q] = c->arc_w[p];
        }
    }
    free(fill);

    /* neighbour lists sorted by (neighbour, eid) for get_eid */
    c->nbr_off = calloc(V + 1, sizeof(int32_t));
    for (int32_t e = 0; e < E; e++) {
        int32_t a = g->edge_src[e], b = g->edge_dst[e];
        c->nbr_off[a + 1]++;
        if (!g->directed && a != b) c->nbr_off[b + 1]++;
    }
    for (int32_t v = 0; v < V; v++) c->nbr_off[v + 1] += c->nbr_off[v];
    int32_t nn = c->nbr_off[V];
    key3* nb = malloc(sizeof(key3) * (nn + 1));
    int32_t* f2 = malloc(sizeof(int32_t) * (V + 1));
    memcpy(f2, c->nbr_off, sizeof(int32_t) * (V + 1));
    for (int32_t e = 0; e < E; e++) {
        int32_t a = g->edge_src[e], b = g->edge_dst[e];
        nb[f2[a]++] = (key3){a, b, e};
        if (!g->directed && a != b) nb[f2[b]++] = (key3){b, a, e};
    }
    qsort(nb, nn, sizeof(key3), cmp_key3);
    c->nbr_v = malloc(sizeof(int32_t) * (nn + 1));
    c->nbr_eid = malloc(sizeof(int32_t) * (nn + 1));
    for (int32_t i = 0; i < nn; i++) { c->nbr_v[i] = nb[i].k2; c->nbr_eid[i] = nb[i].eid; }
    free(nb); free(f2);

    c->max_degree = 0;
    for (int32_t v = 0; v < V; v++) {
        int32_t d = c->arc_off[v + 1] - c->arc_off[v];
        if (d > c->max_degree) c->max_degree = d;
    }
    free(by_from); free(by_to); free(os); free(is);
    return SHD_OK;
}

void shd_csr_free(shd_csr* c) {
    if (!c) return;
    free(c->inc_off); free(c->inc_eid);
    free(c->arc_off); free(c->arc_dst); free(c->arc_eid); free(c->arc_w);
    free(c->rin_off); free(c->rin_src); free(c->rin_eid); free(c->rin_w);
    free(c->nbr_off); free(c->nbr_v); free(c->nbr_eid);
    memset(c, 0, sizeof(*c));
}

int32_t shd_csr_get_eid(const shd_csr* c, int32_t a, int32_t b) {
    int32_t lo = c->nbr_off[a], hi = c->nbr_off[a + 1];
    while (lo < hi) {
        int32_t mid = lo + (hi - lo) / 2;
        if (c->nbr_v[mid] < b) lo = mid + 1; else hi = mid;
    }
    if (lo < c->nbr_off[a + 1] && c->nbr_v[lo] == b) return c->nbr_eid[lo];
    return -1;
}

/* ------------------------------------------------------------ graph check */
int shd_graph_check(const shd_graph* g, shd_graph_props* out) {
    if (!g || !out) return SHD_EINVAL;
    memset(out, 0, sizeof(*out));
    shd_csr c;
    int rc = shd_csr_build(g, &c);
    if (rc) return rc;
    int32_t V = c.V;
    out->is_directed = g->directed;
    out->prefer_direct = g->prefer_direct;
    /* per-edge validation (topology.c:1068-1102) */
    int valid = 1;
    for (int32_t e = 0; e < g->n_edges; e++) {
        double l = g->edge_latency[e], p = g->edge_loss[e];
        if (isnan(l) || !(l > 0.0f)) valid = 0;
        if (isnan(p) || !(p >= 0.0f && p <= 1.0f)) valid = 0;
    }
    if (g->vertex_loss)
        for (int32_t v = 0; v < V; v++) {
            double p = g->vertex_loss[v];
            if (!isnan(p) && !(p >= 0.0f && p <= 1.0f)) valid = 0;
        }
    /* strong connectivity: forward and reverse reachability from vertex 0 */
    int32_t* stack = malloc(sizeof(int32_t) * (V + 1));
    char* seen = malloc(V + 1);
    int connected = 1;
    for (int pass = 0; pass < 2; pass++) {
        const int32_t* off = pass ? c.rin_off : c.arc_off;
        const int32_t* nx = pass ? c.rin_src : c.arc_dst;
        memset(seen, 0, V);
        int32_t sp = 0, n = 1;
        stack[sp++] = 0; seen[0] = 1;
        while (sp) {
            int32_t v = stack[--sp];
            for (int32_t k = off[v]; k < off[v + 1]; k++) {
                int32_t u = nx[k];
                if (!seen[u]) { seen[u] = 1; n++; stack[sp++] = u; }
            }
        }
        if (n != V) connected = 0;
    }
    out->is_connected = connected;
    /* _topology_isComplete: every vertex has >= V incident OUT edges, an
     * undirected self-loop counted once (topology.c:488-541) */
    int complete = 1;
    for (int32_t v = 0; v < V; v++) {
        int32_t ecount = c.inc_off[v + 1] - c.inc_off[v];
        if (ecount > out->max_out_degree) out->max_out_degree = ecount;
        if (shd_csr_get_eid(&c, v, v) >= 0) {
            out->n_self_loops++;
            if (!g->directed) ecount -= 1;
        }
        if (ecount < V) complete = 0;
    }
    out->is_complete = complete;
    free(stack); free(seen);
    shd_csr_free(&c);
    if (!valid) return SHD_EINVAL;
    if (!connected) return SHD_ENOTCONN;
    return SHD_OK;
}

/* ------------------------------------------------------------------ attach */
/* address_stringToIP (address.c:145-152): inet_pton, the network-order s_addr,
 * INADDR_NONE when the string does not parse (strictly dotted-quad decimal:
 * no "10.1", no octal or hex parts) */
static uint32_t string_to_ip(const char* s) {
    struct in_addr a;
    if (s && inet_pton(AF_INET, s, &a) == 1) return a.s_addr;
    return INADDR_NONE;
}
/* a usable IP (topology.c:2123-2128, 2261-2267): the network-order value is
 * compared with the HOST-order constants as the reference does, so on x86-64
 * "127.0.0.1" is usable and "1.0.0.127" (s_addr == INADDR_LOOPBACK) is not */
static int ip_usable(const char* s, uint32_t* ip) {
    if (!s) return 0;
    const uint32_t v = string_to_ip(s);
    if (v == INADDR_NONE || v == INADDR_ANY || v == INADDR_LOOPBACK) return 0;
    *ip = v;
    return 1;
}
static int str_eq(const char* a, const char* b) { return a && b && strcasecmp(a, b) == 0; }

static double draw_state(void* st) { return shd_next_double((uint32_t*)st); }

int shd_topology_attach(const shd_graphml* gm, uint32_t* rng, const char* ip_hint,
                        const char* city, const char* country, const char* geo, const char* type,
                        int32_t* vertex_out, uint64_t* bw_down_out, uint64_t* bw_up_out) {
    if (!rng) return SHD_EINVAL;
    return shd_topology_attach_cb(gm, draw_state, rng, ip_hint, city, country, geo, type, vertex_out,
                                  bw_down_out, bw_up_out);
}

int shd_topology_attach_cb(const shd_graphml* gm, double (*next_double)(void*), void* rng, const char* ip_hint,
                           const char* city, const char* country, const char* geo, const char* type,
                           int32_t* vertex_out, uint64_t* bw_down_out, uint64_t* bw_up_out) {
    if (!gm || !next_double || !vertex_out) return SHD_EINVAL;
    int32_t V = gm->g.n_vertices;
    enum { CITY_TYPE, CITY, COUNTRY_TYPE, COUNTRY, GEO_TYPE, GEO, TYPE, ALL, NQ };
    int32_t* q[NQ]; int32_t qn[NQ]; int32_t nip[NQ];
    for (int i = 0; i < NQ; i++) { q[i] = malloc(sizeof(int32_t) * (V + 1)); qn[i] = 0; nip[i] = 0; }
    uint32_t req_ip = 0;
    int req_usable = ip_usable(ip_hint, &req_ip);
    int exact = 0;
    for (int32_t v = 0; v < V; v++) {
        uint32_t vip = 0;
        int has_ip = ip_usable(gm->vertex_ip ? gm->vertex_ip[v] : NULL, &vip);
        if (req_usable && has_ip && vip == req_ip) {
            if (!exact) for (int i = 0; i < NQ; i++) { qn[i] = 0; nip[i] = 0; }
            exact = 1;
            q[ALL][qn[ALL]++] = v; nip[ALL]++;
        }
        if (exact) continue;
        q[ALL][qn[ALL]++] = v; if (has_ip) nip[ALL]++;
        int cm = str_eq(gm->vertex_citycode ? gm->vertex_citycode[v] : NULL, city);
        int om = str_eq(gm->vertex_countrycode ? gm->vertex_countrycode[v] : NULL, country);
        int gmm = str_eq(gm->vertex_geocode ? gm->vertex_geocode[v] : NULL, geo);
        int tm = str_eq(gm->vertex_type ? gm->vertex_type[v] : NULL, type);
        if (cm && tm) { q[CITY_TYPE][qn[CITY_TYPE]++] = v; if (has_ip) nip[CITY_TYPE]++; }
        if (cm) { q[CITY][qn[CITY]++] = v; if (has_ip) nip[CITY]++; }
        if (om && tm) { q[COUNTRY_TYPE][qn[COUNTRY_TYPE]++] = v; if (has_ip) nip[COUNTRY_TYPE]++; }
        if (om) { q[COUNTRY][qn[COUNTRY]++] = v; if (has_ip) nip[COUNTRY]++; }
        if (gmm && tm) { q[GEO_TYPE][qn[GEO_TYPE]++] = v; if (has_ip) nip[GEO_TYPE]++; }
        if (gmm) { q[GEO][qn[GEO]++] = v; if (has_ip) nip[GEO]++; }
        if (tm) { q[TYPE][qn[TYPE]++] = v; if (has_ip) nip[TYPE]++; }
    }
    int pick = ALL, lpm;
    for (int i = 0; i < ALL; i++) if (qn[i] > 0) { pick = i; break; }
    if (pick == ALL) lpm = (ip_hint && nip[ALL] > 0);
    else lpm = (req_usable && nip[pick] > 0);
    int32_t n = qn[pick];
    int32_t vertex = -1;
    if (n <= 0) goto out;
    if (lpm && !exact) {
        /* _topology_getLongestPrefixMatch (topology.c:2219-2246) */
        uint32_t best = 0;
        for (int32_t i = 0; i < n; i++) {
            int32_t v = q[pick][i];
            /* every candidate's IP as parsed, usable or not (topology.c:2232-2236) */
            const uint32_t vip = string_to_ip(gm->vertex_ip ? gm->vertex_ip[v] : NULL);
            uint32_t match = ~(vip ^ req_ip);
            if (match > best || best == 0) { best = match; vertex = v; }
        }
    } else {
        double r = next_double(rng);
        int32_t range = n - 1;
        int32_t chosen = (int32_t)round((double)(range * r));
        vertex = q[pick][chosen];
    }
out:
    for (int i = 0; i < NQ; i++) free(q[i]);
    if (vertex < 0) return SHD_EINVAL;
    *vertex_out = vertex;
    if (bw_down_out) *bw_down_out = (uint64_t)gm->bw_down[vertex];
    if (bw_up_out) *bw_up_out = (uint64_t)gm->bw_up[vertex];
    return SHD_OK;
}
