/*
 * shd_graphml.c -- graphml topology loader for libshdgpu.
 *
 * Replaces igraph_read_graph_graphml as called by _topology_loadGraph
 * (topology.c:371-399) plus the attribute reads of topology.c:565-722 and the
 * latency weight extraction of topology.c:1212-1246.  Uses libxml2, the parser
 * igraph 0.7.1 itself uses.  Vertex and edge ids are document order of <node>
 * and <edge> elements; <key> defaults apply to elements without <data>;
 * attributes are looked up by attr.name and domain (for="node"/"edge"/"graph").
 */
#include <libxml/parser.h>
#include <libxml/tree.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include "shd_host.h"

typedef struct { char* id; char* name; int domain; char* def; } gkey; /* domain 0 node 1 edge 2 graph */

static int is_el(xmlNode* n, const char* name) {
    return n->type == XML_ELEMENT_NODE && strcmp((const char*)n->name, name) == 0;
}
static char* prop(xmlNode* n, const char* name) {
    xmlChar* v = xmlGetProp(n, (const xmlChar*)name);
    if (!v) return NULL;
    char* s = strdup((const char*)v);
    xmlFree(v);
    return s;
}
static char* text(xmlNode* n) {
    xmlChar* v = xmlNodeGetContent(n);
    if (!v) return strdup("");
    char* s = strdup((const char*)v);
    xmlFree(v);
    return s;
}
static double num(const char* s) {
    if (!s) return NAN;
    while (*s == ' ' || *s == '\t' || *s == '\n' || *s == '\r') s++;
    if (!*s) return NAN;
    char* end = NULL;
    double v = strtod(s, &end);
    if (end == s) return NAN;
    return v;
}
static char* trimdup(const char* s) {
    if (!s) return NULL;
    while (*s == ' ' || *s == '\t' || *s == '\n' || *s == '\r') s++;
    size_t n = strlen(s);
    while (n > 0 && (s[n - 1] == ' ' || s[n - 1] == '\t' || s[n - 1] == '\n' || s[n - 1] == '\r')) n--;
    char* r = malloc(n + 1);
    memcpy(r, s, n); r[n] = 0;
    return r;
}

static uint64_t str_hash(const char* s) {
    uint64_t h = 1469598103934665603ULL;
    while (*s) { h ^= (unsigned char)*s++; h *= 1099511628211ULL; }
    return h;
}
static int32_t id_find(const int32_t* htab, uint64_t hcap, char** ids, const char* s) {
    if (!s) return -1;
    uint64_t h = str_hash(s) & (hcap - 1);
    while (htab[h] >= 0) {
        if (!strcmp(ids[htab[h]], s)) return htab[h];
        h = (h + 1) & (hcap - 1);
    }
    return -1;
}

static int load_doc(xmlDoc* doc, shd_graphml** out) {
    xmlNode* root = xmlDocGetRootElement(doc);
    if (!root || !is_el(root, "graphml")) return SHD_EINVAL;
    gkey* keys = NULL; int nkeys = 0;
    xmlNode* graph = NULL;
    for (xmlNode* n = root->children; n; n = n->next) {
        if (is_el(n, "key")) {
            keys = realloc(keys, sizeof(gkey) * (nkeys + 1));
            gkey* k = &keys[nkeys++];
            k->id = prop(n, "id");
            k->name = prop(n, "attr.name");
            if (!k->name) k->name = k->id ? strdup(k->id) : strdup("");
            char* f = prop(n, "for");
            k->domain = (f && !strcmp(f, "edge")) ? 1 : (f && !strcmp(f, "graph")) ? 2 : 0;
            free(f);
            k->def = NULL;
            for (xmlNode* d = n->children; d; d = d->next)
                if (is_el(d, "default")) k->def = text(d);
        } else if (is_el(n, "graph") && !graph) {
            graph = n;
        }
    }
    int rc = SHD_EINVAL;
    if (!graph) goto done;
    char* ed = prop(graph, "edgedefault");
    int directed = ed && !strcmp(ed, "directed");
    free(ed);
    /* count nodes / edges (document order) */
    int32_t V = 0, E = 0;
    for (xmlNode* n = graph->children; n; n = n->next) {
        if (is_el(n, "node")) V++;
        else if (is_el(n, "edge")) E++;
    }
    if (V <= 0) goto done;
    shd_graphml* gm = calloc(1, sizeof(*gm));
    int32_t* esrc = malloc(sizeof(int32_t) * (E + 1));
    int32_t* edst = malloc(sizeof(int32_t) * (E + 1));
    double* elat = malloc(sizeof(double) * (E + 1));
    double* eloss = malloc(sizeof(double) * (E + 1));
    double* vloss = malloc(sizeof(double) * (V + 1));
    gm->bw_down = malloc(sizeof(double) * (V + 1));
    gm->bw_up = malloc(sizeof(double) * (V + 1));
    gm->edge_jitter = malloc(sizeof(double) * (E + 1));
    gm->vertex_id = calloc(V + 1, sizeof(char*));
    gm->vertex_ip = calloc(V + 1, sizeof(char*));
    gm->vertex_citycode = calloc(V + 1, sizeof(char*));
    gm->vertex_countrycode = calloc(V + 1, sizeof(char*));
    gm->vertex_geocode = calloc(V + 1, sizeof(char*));
    gm->vertex_type = calloc(V + 1, sizeof(char*));
    int has_vloss = 0, prefer_direct = 0;
    /* graph-level attributes: preferdirectpaths (string) */
    for (xmlNode* n = graph->children; n; n = n->next) {
        if (!is_el(n, "data")) continue;
        char* k = prop(n, "key");
        for (int i = 0; i < nkeys; i++)
            if (keys[i].domain == 2 && k && keys[i].id && !strcmp(keys[i].id, k) &&
                !strncasecmp(keys[i].name, "preferdirectpaths", 17)) {
                char* v = trimdup(text(n));
                if (v && (!strncasecmp(v, "true", 4) || !strncasecmp(v, "yes", 3) || !strncasecmp(v, "1", 1)))
                    prefer_direct = 1;
                free(v);
            }
        free(k);
    }
    for (int i = 0; i < nkeys; i++)
        if (keys[i].domain == 2 && !strncasecmp(keys[i].name, "preferdirectpaths", 17) && keys[i].def) {
            /* a default with no <data> also counts */
            int found_data = 0;
            for (xmlNode* n = graph->children; n; n = n->next) if (is_el(n, "data")) {
                char* k = prop(n, "key"); if (k && keys[i].id && !strcmp(k, keys[i].id)) found_data = 1; free(k);
            }
            if (!found_data && (!strncasecmp(keys[i].def, "true", 4) || !strncasecmp(keys[i].def, "yes", 3) ||
                                !strncasecmp(keys[i].def, "1", 1)))
                prefer_direct = 1;
        }
    /* nodes */
    char** node_ids = calloc(V + 1, sizeof(char*));
    int32_t v = 0;
    for (xmlNode* n = graph->children; n; n = n->next) {
        if (!is_el(n, "node")) continue;
        node_ids[v] = prop(n, "id");
        gm->vertex_id[v] = node_ids[v] ? strdup(node_ids[v]) : strdup("");
        double bwd = NAN, bwu = NAN, pl = NAN;
        char* sv[5] = {NULL, NULL, NULL, NULL, NULL};  /* ip city country geo type */
        const char* names[5] = {"ip", "citycode", "countrycode", "geocode", "type"};
        for (int i = 0; i < nkeys; i++) {
            if (keys[i].domain != 0) continue;
            char* val = NULL;
            for (xmlNode* d = n->children; d; d = d->next) {
                if (!is_el(d, "data")) continue;
                char* k = prop(d, "key");
                if (k && keys[i].id && !strcmp(k, keys[i].id)) { free(val); val = text(d); }
                free(k);
            }
            if (!val && keys[i].def) val = strdup(keys[i].def);
            if (!val) continue;
            const char* nm = keys[i].name;
            if (!strcasecmp(nm, "bandwidthdown")) bwd = num(val);
            else if (!strcasecmp(nm, "bandwidthup")) bwu = num(val);
            else if (!strcasecmp(nm, "packetloss")) { pl = num(val); has_vloss = 1; }
            else {
                for (int j = 0; j < 5; j++)
                    if (!strcasecmp(nm, names[j])) { free(sv[j]); sv[j] = trimdup(val); }
            }
            free(val);
        }
        gm->bw_down[v] = bwd; gm->bw_up[v] = bwu; vloss[v] = pl;
        /* empty strings count as absent (_topology_findVertexAttributeString) */
        for (int j = 0; j < 5; j++) if (sv[j] && !sv[j][0]) { free(sv[j]); sv[j] = NULL; }
        gm->vertex_ip[v] = sv[0]; gm->vertex_citycode[v] = sv[1]; gm->vertex_countrycode[v] = sv[2];
        gm->vertex_geocode[v] = sv[3]; gm->vertex_type[v] = sv[4];
        v++;
    }
    /* edges: node id -> document index through an open-addressing table */
    uint64_t hcap = 16;
    while (hcap < (uint64_t)V * 2) hcap <<= 1;
    int32_t* htab = malloc(sizeof(int32_t) * hcap);
    for (uint64_t i = 0; i < hcap; i++) htab[i] = -1;
    for (int32_t i = 0; i < V; i++) {
        if (!node_ids[i]) continue;
        uint64_t hsh = str_hash(node_ids[i]) & (hcap - 1);
        while (htab[hsh] >= 0) hsh = (hsh + 1) & (hcap - 1);
        htab[hsh] = i;   /* duplicates: first in document order wins on lookup */
    }
    int32_t e = 0;
    int bad = 0;
    for (xmlNode* n = graph->children; n; n = n->next) {
        if (!is_el(n, "edge")) continue;
        char* s = prop(n, "source");
        char* t = prop(n, "target");
        int32_t si = id_find(htab, hcap, node_ids, s), ti = id_find(htab, hcap, node_ids, t);
        free(s); free(t);
        if (si < 0 || ti < 0) bad = 1;
        esrc[e] = si; edst[e] = ti;
        double lat = NAN, pl = NAN, jit = NAN;
        for (int i = 0; i < nkeys; i++) {
            if (keys[i].domain != 1) continue;
            char* val = NULL;
            for (xmlNode* d = n->children; d; d = d->next) {
                if (!is_el(d, "data")) continue;
                char* k = prop(d, "key");
                if (k && keys[i].id && !strcmp(k, keys[i].id)) { free(val); val = text(d); }
                free(k);
            }
            if (!val && keys[i].def) val = strdup(keys[i].def);
            if (!val) continue;
            if (!strcasecmp(keys[i].name, "latency")) lat = num(val);
            else if (!strcasecmp(keys[i].name, "packetloss")) pl = num(val);
            else if (!strcasecmp(keys[i].name, "jitter")) jit = num(val);
            free(val);
        }
        elat[e] = lat; eloss[e] = pl; gm->edge_jitter[e] = jit;
        e++;
    }
    for (int32_t i = 0; i < V; i++) free(node_ids[i]);
    free(node_ids); free(htab);
    gm->g.n_vertices = V; gm->g.n_edges = E; gm->g.directed = directed;
    gm->g.prefer_direct = prefer_direct;
    gm->g.edge_src = esrc; gm->g.edge_dst = edst; gm->g.edge_latency = elat; gm->g.edge_loss = eloss;
    if (has_vloss) gm->g.vertex_loss = vloss; else { free(vloss); gm->g.vertex_loss = NULL; }
    if (bad) { shd_graphml_free(gm); rc = SHD_EINVAL; goto done; }
    *out = gm;
    rc = SHD_OK;
done:
    for (int i = 0; i < nkeys; i++) { free(keys[i].id); free(keys[i].name); free(keys[i].def); }
    free(keys);
    return rc;
}

int shd_graphml_load_string(const char* xml, size_t len, shd_graphml** out) {
    if (!xml || !out) return SHD_EINVAL;
    xmlDoc* doc = xmlReadMemory(xml, (int)len, "topology.graphml", NULL, XML_PARSE_NONET | XML_PARSE_HUGE);
    if (!doc) return SHD_EINVAL;
    int rc = load_doc(doc, out);
    xmlFreeDoc(doc);
    return rc;
}

int shd_graphml_load_file(const char* path, shd_graphml** out) {
    if (!path || !out) return SHD_EINVAL;
    xmlDoc* doc = xmlReadFile(path, NULL, XML_PARSE_NONET | XML_PARSE_HUGE);
    if (!doc) return SHD_EINVAL;
    int rc = load_doc(doc, out);
    xmlFreeDoc(doc);
    return rc;
}

void shd_graphml_free(shd_graphml* gm) {
    if (!gm) return;
    int32_t V = gm->g.n_vertices;
    free((void*)gm->g.edge_src); free((void*)gm->g.edge_dst);
    free((void*)gm->g.edge_latency); free((void*)gm->g.edge_loss); free((void*)gm->g.vertex_loss);
    free(gm->bw_down); free(gm->bw_up); free(gm->edge_jitter);
    char** lists[6] = {gm->vertex_id, gm->vertex_ip, gm->vertex_citycode, gm->vertex_countrycode,
                       gm->vertex_geocode, gm->vertex_type};
    for (int j = 0; j < 6; j++) {
        if (!lists[j]) continue;
        for (int32_t i = 0; i < V; i++) free(lists[j][i]);
        free(lists[j]);
    }
    free(gm);
}
