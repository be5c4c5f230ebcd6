/* shd_config.c -- the shadow.config.xml front-end of the path:
 * host registration order, `quantity` naming and DNS IP assignment, so that a
 * reference config yields the same host list, names and addresses that the
 * reference registers before attach (shd_topology_attach) and the engine.
 *
 *   element/attribute names     core/support/configuration.c:262-300 (topology),
 *                               404-480 (host), 560-600 (process)
 *   host expansion and naming   core/master.c:304-320, 397 (document order;
 *                               "<id><i+1>" when quantity > 1)
 *   addresses                   host/host.c:166-167 (loopback registered first,
 *                               then the ethernet address with the IP hint),
 *                               routing/dns.c:40-134, 183-196 (counter from
 *                               11.0.0.0, reserved ranges skipped, unique IPs)
 *
 * Attribute names are matched case-insensitively, the first occurrence wins
 * (configuration.c's "!isSet &&" tests).  Unknown attributes of the elements
 * read here are ignored rather than rejected: the plugin/process layer they
 * belong to is outside this path. */
#include <ctype.h>
#include <stdint.h>
#include <arpa/inet.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include <libxml/parser.h>
#include <libxml/tree.h>

#include "shd_host.h"

static char* dup_str(const char* s) {
    if (!s) return NULL;
    size_t n = strlen(s);
    char* d = (char*)malloc(n + 1);
    if (d) memcpy(d, s, n + 1);
    return d;
}

/* the first attribute of `node` named `name` (ASCII case-insensitive) */
static char* attr_ci(xmlNodePtr node, const char* name) {
    for (xmlAttrPtr a = node->properties; a; a = a->next) {
        if (!a->name || strcasecmp((const char*)a->name, name)) continue;
        xmlChar* v = xmlNodeListGetString(node->doc, a->children, 1);
        char* r = dup_str(v ? (const char*)v : "");
        if (v) xmlFree(v);
        return r;
    }
    return NULL;
}

/* g_ascii_strtoull(value, NULL, 10): leading digits, 0 if none */
static uint64_t to_u64(const char* s) {
    if (!s) return 0;
    while (isspace((unsigned char)*s)) s++;
    return strtoull(s, NULL, 10);
}

void shd_config_free(shd_config* c) {
    if (!c) return;
    for (int32_t i = 0; i < c->n_hosts; i++) {
        shd_config_host* h = &c->hosts[i];
        free(h->name); free(h->ip_hint); free(h->citycode_hint); free(h->countrycode_hint);
        free(h->geocode_hint); free(h->type_hint); free(h->process_start_s);
    }
    free(c->hosts);
    free(c->topology_path);
    free(c->topology_text);
    free(c);
}

static int add_host(shd_config* c, int32_t* cap, const shd_config_host* h) {
    if (c->n_hosts == *cap) {
        int32_t nc = *cap ? 2 * *cap : 16;
        shd_config_host* p = (shd_config_host*)realloc(c->hosts, sizeof(shd_config_host) * (size_t)nc);
        if (!p) return SHD_ENOMEM;
        c->hosts = p;
        *cap = nc;
    }
    c->hosts[c->n_hosts++] = *h;
    return SHD_OK;
}

static int parse_doc(xmlDocPtr doc, shd_config** out) {
    xmlNodePtr root = xmlDocGetRootElement(doc);
    if (!root || strcasecmp((const char*)root->name, "shadow")) return SHD_EINVAL;
    shd_config* c = (shd_config*)calloc(1, sizeof(shd_config));
    if (!c) return SHD_ENOMEM;
    int32_t cap = 0;
    int rc = SHD_OK;
    char* v;
    if ((v = attr_ci(root, "stoptime"))) { c->stop_time_s = to_u64(v); free(v); }
    if ((v = attr_ci(root, "bootstraptime"))) { c->bootstrap_time_s = to_u64(v); free(v); }
    for (xmlNodePtr n = root->children; n && rc == SHD_OK; n = n->next) {
        if (n->type != XML_ELEMENT_NODE) continue;
        const char* tag = (const char*)n->name;
        if (!strcasecmp(tag, "kill")) {   /* legacy <kill time=.../> */
            if ((v = attr_ci(n, "time"))) { c->stop_time_s = to_u64(v); free(v); }
        } else if (!strcasecmp(tag, "topology")) {
            if ((v = attr_ci(n, "path"))) {
                free(c->topology_path);
                c->topology_path = v;
            }
            xmlChar* txt = xmlNodeGetContent(n);   /* inline graphml (CDATA) */
            if (txt) {
                const char* t = (const char*)txt;
                while (isspace((unsigned char)*t)) t++;
                if (*t) {
                    free(c->topology_text);
                    c->topology_text = dup_str(t);
                }
                xmlFree(txt);
            }
        } else if (!strcasecmp(tag, "host") || !strcasecmp(tag, "node")) {
            char* id = attr_ci(n, "id");
            if (!id || !*id) { free(id); rc = SHD_EINVAL; break; }
            char* q = attr_ci(n, "quantity");
            const uint64_t quantity = q ? to_u64(q) : 1;
            free(q);
            char* iph = attr_ci(n, "iphint");
            char* cch = attr_ci(n, "citycodehint");
            char* coh = attr_ci(n, "countrycodehint");
            char* geh = attr_ci(n, "geocodehint");
            char* tyh = attr_ci(n, "typehint");
            char* bd = attr_ci(n, "bandwidthdown");
            char* bu = attr_ci(n, "bandwidthup");
            char* hb = attr_ci(n, "heartbeatfrequency");
            /* the host's processes in document order: their start times */
            int32_t np = 0;
            uint64_t* starts = NULL;
            for (xmlNodePtr k = n->children; k && rc == SHD_OK; k = k->next) {
                if (k->type != XML_ELEMENT_NODE) continue;
                if (strcasecmp((const char*)k->name, "process") && strcasecmp((const char*)k->name, "application"))
                    continue;
                char* st = attr_ci(k, "starttime");
                if (!st) st = attr_ci(k, "time");   /* deprecated alias, configuration.c:576-577 */
                if (!st) { rc = SHD_EINVAL; break; }  /* starttime is required (configuration.c:596-598) */
                uint64_t* ns = (uint64_t*)realloc(starts, sizeof(uint64_t) * (size_t)(np + 1));
                if (!ns) { free(st); rc = SHD_ENOMEM; break; }
                starts = ns;
                starts[np++] = to_u64(st);
                free(st);
            }
            for (uint64_t i = 0; i < quantity && rc == SHD_OK; i++) {
                shd_config_host h;
                memset(&h, 0, sizeof(h));
                size_t len = strlen(id) + 24;
                h.name = (char*)malloc(len);
                if (!h.name) { rc = SHD_ENOMEM; break; }
                if (quantity > 1) snprintf(h.name, len, "%s%llu", id, (unsigned long long)(i + 1));
                else snprintf(h.name, len, "%s", id);
                h.ip_hint = dup_str(iph);
                h.citycode_hint = dup_str(cch);
                h.countrycode_hint = dup_str(coh);
                h.geocode_hint = dup_str(geh);
                h.type_hint = dup_str(tyh);
                h.bw_down_kibps = to_u64(bd);
                h.bw_up_kibps = to_u64(bu);
                h.heartbeat_s = to_u64(hb);
                h.n_processes = np;
                if (np) {
                    h.process_start_s = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)np);
                    if (!h.process_start_s) { free(h.name); rc = SHD_ENOMEM; break; }
                    memcpy(h.process_start_s, starts, sizeof(uint64_t) * (size_t)np);
                }
                rc = add_host(c, &cap, &h);
            }
            free(starts);
            free(id); free(iph); free(cch); free(coh); free(geh); free(tyh); free(bd); free(bu); free(hb);
        }
    }
    if (rc != SHD_OK) {
        shd_config_free(c);
        return rc;
    }
    *out = c;
    return SHD_OK;
}

int shd_config_load_buffer(const char* xml, size_t n, shd_config** out) {
    if (!xml || !out) return SHD_EINVAL;
    xmlDocPtr doc = xmlReadMemory(xml, (int)n, "shadow.config.xml", NULL, XML_PARSE_NONET | XML_PARSE_HUGE);
    if (!doc) return SHD_EINVAL;
    int rc = parse_doc(doc, out);
    xmlFreeDoc(doc);
    return rc;
}

int shd_config_load_file(const char* path, shd_config** out) {
    if (!path || !out) return SHD_EINVAL;
    xmlDocPtr doc = xmlReadFile(path, NULL, XML_PARSE_NONET | XML_PARSE_HUGE);
    if (!doc) return SHD_EINVAL;
    int rc = parse_doc(doc, out);
    xmlFreeDoc(doc);
    return rc;
}

/* ---------------------------------------------------------------- DNS */
/* dotted quad -> host-order u32 as address_stringToIP does it (inet_pton,
 * address.c:145-152, then ntohl): no whitespace, signs or leading-zero
 * octets; 0 with *ok = 0 when malformed */
static uint32_t ip_parse(const char* s, int* ok) {
    struct in_addr a;
    *ok = 0;
    if (!s || inet_pton(AF_INET, s, &a) != 1) return 0;
    *ok = 1;
    return ntohl(a.s_addr);
}

/* _dns_isRestricted (dns.c:74-95), on host-order addresses */
static int ip_restricted(uint32_t ip) {
    static const struct { uint32_t net; int bits; } r[] = {
        {0x00000000u, 8},  {0x0A000000u, 8},  {0x64400000u, 10}, {0x7F000000u, 8},
        {0xA9FE0000u, 16}, {0xAC100000u, 12}, {0xC0000000u, 29}, {0xC0000200u, 24},
        {0xC0586300u, 24}, {0xC0A80000u, 16}, {0xC6120000u, 15}, {0xC6336400u, 24},
        {0xCB007100u, 24}, {0xE0000000u, 4},  {0xF0000000u, 4},  {0xFFFFFFFFu, 32},
    };
    for (size_t i = 0; i < sizeof(r) / sizeof(r[0]); i++) {
        const uint32_t mask = r[i].bits ? 0xFFFFFFFFu << (32 - r[i].bits) : 0;
        if ((ip & mask) == (r[i].net & mask)) return 1;
    }
    return 0;
}

typedef struct { uint32_t* v; size_t n, cap; } ipset;   /* open addressing, 0 = empty */
static int ipset_has(const ipset* s, uint32_t ip) {
    if (!s->cap) return 0;
    for (size_t i = (ip * 2654435761u) & (s->cap - 1);; i = (i + 1) & (s->cap - 1)) {
        if (s->v[i] == 0) return 0;
        if (s->v[i] == ip) return 1;
    }
}
static int ipset_add(ipset* s, uint32_t ip) {
    if (2 * (s->n + 1) > s->cap) {
        size_t nc = s->cap ? 2 * s->cap : 1024;
        uint32_t* nv = (uint32_t*)calloc(nc, 4);
        if (!nv) return SHD_ENOMEM;
        for (size_t i = 0; i < s->cap; i++)
            if (s->v[i])
                for (size_t j = (s->v[i] * 2654435761u) & (nc - 1);; j = (j + 1) & (nc - 1))
                    if (!nv[j]) { nv[j] = s->v[i]; break; }
        free(s->v);
        s->v = nv;
        s->cap = nc;
    }
    for (size_t i = (ip * 2654435761u) & (s->cap - 1);; i = (i + 1) & (s->cap - 1)) {
        if (s->v[i] == ip) return SHD_OK;
        if (!s->v[i]) { s->v[i] = ip; s->n++; return SHD_OK; }
    }
}

/* dns_register for every host in registration order (host.c:166-167): the
 * loopback registration takes a MAC only; the ethernet address keeps its
 * hint when the hint is unrestricted and unused, else takes the next counter
 * address that is neither (dns.c:102-134).  ip_out: host-order IPv4. */
int shd_dns_assign(const shd_config* c, uint32_t* ip_out) {
    if (!c || (c->n_hosts && !ip_out)) return SHD_EINVAL;
    ipset used = {0};
    uint32_t counter = 0x0B000000u;   /* ntohl(11.0.0.0), dns.c:193 */
    int rc = SHD_OK;
    for (int32_t i = 0; i < c->n_hosts && rc == SHD_OK; i++) {
        uint32_t ip = 0;
        int ok = 0, have = 0;
        if (c->hosts[i].ip_hint) {
            ip = ip_parse(c->hosts[i].ip_hint, &ok);
            /* a hint of 127.0.0.1 is the local address (dns.c:121-123) */
            if (ok && ip == 0x7F000001u) have = 1;
            else if (ok && !ip_restricted(ip) && !ipset_has(&used, ip)) have = 1;
        }
        if (!have) {
            do ip = ++counter; while (ip_restricted(ip) || ipset_has(&used, ip));
        }
        if (ip != 0x7F000001u) rc = ipset_add(&used, ip);
        ip_out[i] = ip;
    }
    free(used.v);
    return rc;
}
