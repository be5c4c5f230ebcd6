/*
 * ref_net.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Links four more of the reference's OWN sources, compiled unmodified from
 * /root/reference by oracle/Makefile into oracle/_ref/libshdref_net.so:
 *   src/main/routing/dns.c      (address assignment: dns_register)
 *   src/main/routing/address.c  (Address, address_stringToIP / ipToNewString)
 *   src/main/routing/packet.c   (packet_addDeliveryStatus / packet_toString)
 *   src/main/routing/payload.c  (the packet's payload)
 * and exposes a flat API to tests/golden/make_ref_net.py (fixtures) and
 * tests/test_oracle_ref.py (live checks), which pin the product's DNS
 * (host/shd_config.c shd_dns_assign) and [STATUS] writer (shdgpu.status_lines)
 * to them.  The functions below stand in for the collaborators those files
 * call: the worker (debug level on, no active host), the host's packet
 * priority, the object counter, and the logger, which here captures each
 * message() line instead of printing it.
 */
#include <arpa/inet.h>
#include <glib.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "main/core/support/object_counter.h"
#include "main/routing/address.h"
#include "main/routing/dns.h"
#include "main/routing/packet.h"
#include "support/logger/log_level.h"
#include "support/logger/logger.h"

/* ---- collaborators (test doubles) ---- */
typedef struct _Host Host;
gboolean worker_isFiltered(LogLevel level) { return FALSE; }   /* debug level: every status is logged */
Host* worker_getActiveHost(void) { return NULL; }
gdouble host_getNextPacketPriority(Host* host) { return 0.0; }
void worker_countObject(ObjectType otype, CounterType ctype) {}
Logger* logger_getDefault(void) { return NULL; }

static char* g_cap;         /* capture buffer for message() lines */
static size_t g_cap_len, g_cap_size;

void logger_log(Logger* logger, LogLevel level, const gchar* fileName, const gchar* functionName,
                const gint lineNumber, const gchar* format, ...) {
    if (!g_cap || level != LOGLEVEL_MESSAGE) return;
    va_list ap;
    va_start(ap, format);
    int n = vsnprintf(g_cap + g_cap_len, g_cap_size > g_cap_len ? g_cap_size - g_cap_len : 0, format, ap);
    va_end(ap);
    if (n < 0) return;
    g_cap_len += (size_t)n;
    if (g_cap_len + 1 < g_cap_size) {
        g_cap[g_cap_len++] = '\n';
        g_cap[g_cap_len] = 0;
    }
}

/* ---- DNS: host_setup's two registrations per host (host.c:166-167) ----
 * hints[i] may be NULL; ip_out[i] = the ethernet address, host order */
int ref_dns_assign(int n, const char* const* hints, uint32_t* ip_out) {
    DNS* dns = dns_new();
    for (int i = 0; i < n; i++) {
        char name[32];
        snprintf(name, sizeof(name), "host%d", i);
        Address* lo = dns_register(dns, (GQuark)(i + 1), name, "127.0.0.1");
        Address* eth = dns_register(dns, (GQuark)(i + 1), name, (gchar*)hints[i]);
        ip_out[i] = address_toHostIP(eth);
        address_unref(lo);
        address_unref(eth);
    }
    dns_free(dns);
    return 0;
}

/* ---- [STATUS] lines: one UDP datagram through a scripted status list ----
 * IPs in host order, ports as numbers; out receives one line per status,
 * "[<STATUS>] <packet_toString>" as message() formats it (packet.c:657) */
int ref_status_story(uint32_t host_id, uint64_t pkt_id, uint32_t src_ip, uint32_t sport, uint32_t dst_ip,
                     uint32_t dport, uint32_t payload_len, const uint32_t* statuses, int n, char* out,
                     size_t cap) {
    static char zeros[65536];
    if (payload_len > sizeof(zeros)) return -1;
    g_cap = out;
    g_cap_len = 0;
    g_cap_size = cap;
    if (cap) out[0] = 0;
    Packet* p = packet_new(payload_len ? zeros : NULL, payload_len, host_id, pkt_id);
    packet_setUDP(p, PUDP_NONE, htonl(src_ip), htons((in_port_t)sport), htonl(dst_ip), htons((in_port_t)dport));
    for (int i = 0; i < n; i++) packet_addDeliveryStatus(p, (PacketDeliveryStatusFlags)statuses[i]);
    packet_unref(p);
    g_cap = NULL;
    return g_cap_len + 1 < cap ? 0 : -1;
}
