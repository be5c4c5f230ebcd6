/*
 * ref_loop.c -- TEST INFRASTRUCTURE ONLY.
 *
 * The reference's own serial event loop, compiled unmodified from
 * /root/reference by oracle/Makefile into oracle/_ref/libshdref_loop.so:
 *   core/worker.c (worker_run, worker_sendPacket, worker_scheduleTask),
 *   core/work/event.c + task.c, core/scheduler/scheduler.c + its policies
 *   (SP_SERIAL_GLOBAL: scheduler_policy_global_single.c), core/support/options.c
 *   (the CLI defaults), host/host.c (boot, descriptors, implicit bind,
 *   sendUserData / receiveUserData), host/network_interface.c (token buckets,
 *   refill, FIFO qdisc, loopback), host/tracker.c (heartbeat), host/cpu.c,
 *   host/descriptor/{descriptor,transport,socket,udp,tcp,tcp_cong,tcp_cong_reno,
 *   tcp_retransmit_tally,epoll,channel,timer}.c, routing/{router,
 *   router_queue_codel,router_queue_single,router_queue_static,packet,payload,
 *   address,dns}.c, utility/{random,priority_queue,utility,byte_queue,
 *   count_down_latch,pcap_writer}.c, core/support/object_counter.c,
 *   support/logger/log_level.c.
 *
 * Nothing here restates any of that.  This file is the collaborators the build
 * cannot compile, as test doubles:
 *   - slave_* (core/slave.c needs the whole master/config stack): DNS,
 *     topology, options, bootstrap end, "scheduler is running";
 *   - topology_* (routing/topology.c needs igraph, absent from the image): the
 *     caller's path-cache lookup (the oracle's lazy cache, o_topo_get, which
 *     reproduces the first-touch rule), host -> vertex from the caller;
 *   - process_* (host/process.c needs the generated rpth.h): process_schedule
 *     as process.c:1334-1357 schedules it; the "plugin" is the application
 *     the caller names, run on the process's start task and on each epoll
 *     notification (process_continue), issuing the same host_* calls the
 *     process_emu_* syscall handlers make (process.c:1412-1530, 2005-2130,
 *     2946-2990, 4790-4795);
 *   - the loggers: message-level lines (the [STATUS] packet lines of
 *     packet.c:647-659 at debug filter level, the tracker's heartbeat lines)
 *     captured with their simulated time and active host.
 *
 * The application is src/test/phold/test_phold.c's logic (start listening,
 * bootstrap `load` messages, on every readable notification read every
 * datagram and answer each byte with a new message), restated over the
 * syscalls above; its destination choice uses the caller's cumulative weights
 * (the model's, test_phold.c:160-178).  The run is the reference's serial
 * mode (--workers 0, slave.c:415-428): one scheduler, one worker, one round
 * to the end time.
 */
#include <arpa/inet.h>
#include <glib.h>
#include <glib/gstdio.h>
#include <netinet/in.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <fcntl.h>
#include <sys/epoll.h>
#include <time.h>

#include "main/core/logger/shadow_logger.h"
#include "main/core/scheduler/scheduler.h"
#include "main/core/slave.h"
#include "main/core/support/definitions.h"
#include "main/core/support/object_counter.h"
#include "main/core/support/options.h"
#include "main/core/work/task.h"
#include "main/core/worker.h"
#include "main/host/descriptor/descriptor.h"
#include "main/host/descriptor/socket.h"
#include "main/host/host.h"
#include "main/host/process.h"
#include "main/routing/address.h"
#include "main/routing/dns.h"
#include "main/routing/topology.h"
#include "main/utility/random.h"
#include "support/logger/log_level.h"
#include "support/logger/logger.h"

/* ------------------------------------------------------------ the run's config */
typedef int (*ref_path_fn)(void* ctx, int32_t src_vertex, int32_t dst_vertex, double* lat_ms, double* rel);

typedef struct ref_loop_cfg {
    int32_t n_hosts;
    int32_t app;                  /* 0 = PHOLD-UDP (test_phold.c), 1 = TCP echo, 2 = UDP echo,
                                     3 = a datagram application per host (app_spec below) */
    const uint32_t* host_seed;    /* [H] host RNG state after attach (the model's host_rng) */
    const int32_t* host_vertex;   /* [H] */
    const uint64_t* bw_down_kibps, *bw_up_kibps;   /* [H] */
    const double* dest_cum;       /* [n_classes][H] PHOLD cumulative weights */
    const uint8_t* host_class;    /* [H] or NULL */
    int32_t n_classes, _pad;
    const uint64_t* host_heartbeat;   /* [H] ns or NULL */
    const uint64_t* host_start;       /* [H] process start (ns) or NULL: app_start */
    int32_t n_procs, _pad2;           /* > 0: these processes instead of one per host */
    const int32_t* proc_host;         /* [n_procs] in each host's <process> order */
    const uint64_t* proc_start;       /* [n_procs] */
    uint64_t end_time, bootstrap_end, heartbeat_interval, app_start;
    uint32_t load, payload;
    ref_path_fn path;
    void* path_ctx;
    const char* root_dir;         /* host data directories (host_setup mkdirs them) */
    /* app 1 (TCP echo): proc_peer[k] = -1 for a server, else the server process
     * the client k connects to; each client sends tcp_bytes, the server echoes */
    const int32_t* proc_peer;
    uint32_t tcp_bytes, _pad3;
    /* 1: the default log level's work only -- debug records filtered (the
     * [STATUS] lines are not even formatted) and no line kept: for timing the
     * reference's loop (scripts/r04/ref_loop_timing.py) */
    int32_t quiet;
    /* 1: --interface-qdisc=rr (options.c:162; round-robin over the sockets
     * that want to send, network_interface.c:466-490) instead of fifo */
    int32_t qdisc_rr;
    /* wall-clock marks (bench.py's reference CPU baseline): the monotonic clock
     * at the first path lookup (a send) at simulated time >= mark_time[k]; 0 = off */
    uint64_t mark_time[2];
    /* app 3 (shdgpu.h shd_udp_app): host h runs app_spec[4 * host_app[h] ..]
     * = {send, dest, n_start, per_read}; app_peer[h]: its SHD_DEST_PEER host */
    const uint32_t* app_spec;
    const uint8_t* host_app;
    const int32_t* app_peer;
    /* app 1 with datagram processes beside the TCP echo ones (one model, both
     * transports on each host's interface): proc_app[k] >= 0 runs
     * app_spec[4 * proc_app[k] ..] in process k instead of the echo (at most
     * one such process per host: they share PHOLD's port); NULL: all echo */
    const int32_t* proc_app;
} ref_loop_cfg;

typedef struct ref_loop_out {
    char* lines;                  /* "<time>\t<host index>\t<line>\n" per message-level line */
    size_t len, cap;
    uint64_t n_lines;
    uint32_t* ip;                 /* [H] host byte order */
    uint64_t* next_event_id;      /* [H] host_getNewEventID at the end */
    uint64_t* next_packet_id;     /* [H] */
    uint32_t* rng_probe;          /* [H] random_rand of the host RNG at the end */
    double mark_wall_s[2];        /* monotonic seconds at mark_time[k] (0 if never reached) */
} ref_loop_out;

static const ref_loop_cfg* g_cfg;
static ref_loop_out* g_out;
static DNS* g_dns;
static Options* g_options;
static Scheduler* g_sched;
static Host** g_hosts;

/* ------------------------------------------------------------ slave doubles */
struct _Slave { int dummy; };
static struct _Slave g_slave;
static struct _Topology { int dummy; } g_topology;

DNS* slave_getDNS(Slave* slave) { return g_dns; }
Topology* slave_getTopology(Slave* slave) { return (Topology*)&g_topology; }
Options* slave_getOptions(Slave* slave) { return g_options; }
SimulationTime slave_getBootstrapEndTime(Slave* slave) { return g_cfg->bootstrap_end; }
gboolean slave_schedulerIsRunning(Slave* slave) { return g_sched && scheduler_isRunning(g_sched); }
void slave_countObject(ObjectType otype, CounterType ctype) {}
void slave_storeCounts(Slave* slave, ObjectCounter* objectCounter) {}
void slave_updateMinTimeJump(Slave* slave, gdouble minPathLatency) {}
void slave_incrementPluginError(Slave* slave) {}

static int32_t host_index_of(GQuark id) { return (int32_t)id - 1; }

static void note_marks(void) {
    for (int k = 0; k < 2; k++) {
        if (!g_out || !g_cfg->mark_time[k] || g_out->mark_wall_s[k] != 0) continue;
        if (worker_getCurrentTime() < g_cfg->mark_time[k]) continue;
        struct timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        g_out->mark_wall_s[k] = (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
    }
}

static int path_of(Address* a, Address* b, double* lat, double* rel) {
    note_marks();
    const int32_t ha = host_index_of((GQuark)address_getID(a)), hb = host_index_of((GQuark)address_getID(b));
    if (ha < 0 || hb < 0 || ha >= g_cfg->n_hosts || hb >= g_cfg->n_hosts) { *lat = -1; *rel = -1; return -1; }
    return g_cfg->path(g_cfg->path_ctx, g_cfg->host_vertex[ha], g_cfg->host_vertex[hb], lat, rel);
}
gdouble slave_getLatency(Slave* slave, GQuark sourceNodeID, GQuark destinationNodeID) {
    double lat, rel;
    const int32_t a = host_index_of(sourceNodeID), b = host_index_of(destinationNodeID);
    g_cfg->path(g_cfg->path_ctx, g_cfg->host_vertex[a], g_cfg->host_vertex[b], &lat, &rel);
    return lat;
}
guint32 slave_getNodeBandwidthUp(Slave* slave, GQuark nodeID, in_addr_t ip) {
    return (guint32)g_cfg->bw_up_kibps[host_index_of(nodeID)];
}
guint32 slave_getNodeBandwidthDown(Slave* slave, GQuark nodeID, in_addr_t ip) {
    return (guint32)g_cfg->bw_down_kibps[host_index_of(nodeID)];
}

/* ------------------------------------------------------------ topology doubles */
void topology_attach(Topology* top, Address* address, Random* randomSourcePool, gchar* ipHint,
                     gchar* citycodeHint, gchar* countrycodeHint, gchar* geocodeHint, gchar* typeHint,
                     guint64* bwDownOut, guint64* bwUpOut) {
    /* the caller's attachment (host_vertex; the seed is the RNG state after
     * the attach draw) */
    const int32_t h = host_index_of((GQuark)address_getID(address));
    *bwDownOut = g_cfg->bw_down_kibps[h];
    *bwUpOut = g_cfg->bw_up_kibps[h];
}
/* host_shutdown's first step after the run (host.c:318-321): the host's end
 * state, read while its RNG and counters still exist */
void topology_detach(Topology* top, Address* address) {
    const int32_t h = host_index_of((GQuark)address_getID(address));
    if (!g_out || h < 0 || h >= g_cfg->n_hosts) return;
    g_out->next_event_id[h] = host_getNewEventID(g_hosts[h]);
    g_out->next_packet_id[h] = host_getNewPacketID(g_hosts[h]);
    g_out->rng_probe[h] = (uint32_t)random_rand(host_getRandom(g_hosts[h]));
}
gboolean topology_isRoutable(Topology* top, Address* srcAddress, Address* dstAddress) {
    double lat, rel;
    path_of(srcAddress, dstAddress, &lat, &rel);
    return lat >= 0;
}
gdouble topology_getLatency(Topology* top, Address* srcAddress, Address* dstAddress) {
    double lat, rel;
    path_of(srcAddress, dstAddress, &lat, &rel);
    return lat;
}
gdouble topology_getReliability(Topology* top, Address* srcAddress, Address* dstAddress) {
    double lat, rel;
    path_of(srcAddress, dstAddress, &lat, &rel);
    return rel;
}
void topology_incrementPathPacketCounter(Topology* top, Address* srcAddress, Address* dstAddress) {}

/* ------------------------------------------------------------ logger doubles */
struct _ShadowLogger { int dummy; };
static struct _ShadowLogger g_slogger;
ShadowLogger* shadow_logger_getDefault() { return &g_slogger; }
/* debug filter level: packet_addDeliveryStatus logs every status (packet.c:652) */
gboolean shadow_logger_shouldFilter(ShadowLogger* logger, LogLevel level) {
    return g_cfg && g_cfg->quiet && level > LOGLEVEL_MESSAGE;
}
void shadow_logger_flushRecords(ShadowLogger* logger, pthread_t callerThread) {}
void shadow_logger_register(ShadowLogger* logger, pthread_t callerThread) {}
Logger* logger_getDefault(void) { return NULL; }

static void out_append(const char* s, size_t n) {
    if (g_out->len + n + 1 > g_out->cap) {
        size_t nc = g_out->cap ? g_out->cap : (1u << 20);
        while (g_out->len + n + 1 > nc) nc *= 2;
        g_out->lines = realloc(g_out->lines, nc);
        g_out->cap = nc;
    }
    memcpy(g_out->lines + g_out->len, s, n);
    g_out->len += n;
    g_out->lines[g_out->len] = 0;
}

void logger_log(Logger* logger, LogLevel level, const gchar* fileName, const gchar* functionName,
                const gint lineNumber, const gchar* format, ...) {
    if (!g_out || level != LOGLEVEL_MESSAGE || !g_sched || !scheduler_isRunning(g_sched) || !worker_isAlive() ||
        g_cfg->quiet)
        return;
    /* a packet whose last reference goes with its deliver task is released
     * after event_execute cleared the active host (event.c:86, worker.c:187):
     * host -1, the line still at the event's time */
    Host* h = worker_getActiveHost();
    const SimulationTime now = worker_getCurrentTime();
    char buf[4096];
    int n = snprintf(buf, sizeof(buf), "%llu\t%d\t", (unsigned long long)now, h ? host_index_of(host_getID(h)) : -1);
    va_list ap;
    va_start(ap, format);
    int m = vsnprintf(buf + n, sizeof(buf) - (size_t)n - 2, format, ap);
    va_end(ap);
    if (m < 0) return;
    size_t len = (size_t)n + (size_t)(m < (int)(sizeof(buf) - (size_t)n - 2) ? m : (int)(sizeof(buf) - (size_t)n - 3));
    buf[len++] = '\n';
    out_append(buf, len);
    g_out->n_lines++;
}

/* ------------------------------------------------------------ process doubles */
struct _Process {
    Host* host;
    SimulationTime startTime, stopTime;
    gint refcount;
    gboolean running;
    gint epollfd;     /* the descriptor whose readiness continues the process */
    gint listenfd;
    /* app 1 (TCP echo) */
    gint index, step, fd, wait_fd;
    /* apps 3 and 1's datagram processes: {send, dest, n_start, per_read} */
    const uint32_t* spec;
    guint32 done;
    gchar* buf;
};
static Process** g_procs;

Process* process_new(gpointer host, guint processID, SimulationTime startTime, SimulationTime stopTime,
                     const gchar* pluginName, const gchar* pluginPath, const gchar* pluginSymbol,
                     const gchar* preloadName, const gchar* preloadPath, gchar* arguments) {
    Process* p = g_new0(Process, 1);
    p->host = host;
    p->startTime = startTime;
    p->stopTime = stopTime;
    p->refcount = 1;
    p->epollfd = -1;
    p->listenfd = -1;
    p->fd = -1;
    p->wait_fd = -1;
    p->index = arguments ? atoi(arguments) : -1;
    if (g_cfg->app == 1 && g_procs && p->index >= 0 && p->index < g_cfg->n_procs) g_procs[p->index] = p;
    return p;
}
void process_ref(Process* proc) { proc->refcount++; }
void process_unref(Process* proc) {
    if (--proc->refcount == 0) {
        if (g_procs && proc->index >= 0 && proc->index < g_cfg->n_procs && g_procs[proc->index] == proc)
            g_procs[proc->index] = NULL;
        g_free(proc->buf);
        g_free(proc);
    }
}
gboolean process_isRunning(Process* proc) { return proc->running; }
gboolean process_wantsNotify(Process* proc, gint epollfd) {
    return proc->running && epollfd == proc->epollfd;
}
void process_migrate(Process* proc, gpointer threads) {}
void process_stop(Process* proc) { proc->running = FALSE; }

/* ---- the application: test_phold.c over the syscall handlers' host_* calls */
#define PHOLD_LISTEN_PORT 8998

static void phold_send_new_message(Process* proc) {
    Host* host = proc->host;
    const int32_t h = host_index_of(host_getID(host));
    /* _phold_chooseNode (test_phold.c:160-178): random() = process_emu_random
     * = random_rand(host RNG) (process.c:4790-4795) */
    const double r = ((double)random_rand(host_getRandom(host))) / ((double)RAND_MAX);
    const double* cum = g_cfg->dest_cum;
    if (g_cfg->host_class && g_cfg->n_classes > 1) cum += (size_t)g_cfg->host_class[h] * (size_t)g_cfg->n_hosts;
    int32_t chosen = -1;
    for (int32_t i = 0; i < g_cfg->n_hosts; i++)
        if (cum[i] >= r) { chosen = i; break; }
    if (chosen < 0) return;   /* NULL node name: _phold_sendToNode warns, nothing sent */
    /* _phold_sendToNode (test_phold.c:180-216): socket, sendto, close */
    const in_addr_t ip = host_getDefaultIP(g_hosts[chosen]);
    gint fd = host_createDescriptor(host, DT_UDPSOCKET);           /* process_emu_socket (process.c:2080-2129) */
    Descriptor* desc = host_lookupDescriptor(host, fd);
    descriptor_setFlags(desc, descriptor_getFlags(desc) | O_NONBLOCK);
    gint8 msg = 64;
    gsize bytes = 0;
    (void)host_sendUserData(host, fd, &msg, g_cfg->payload ? g_cfg->payload : 1, ip,
                            (in_addr_t)htons(PHOLD_LISTEN_PORT), &bytes);   /* _process_emu_sendHelper */
    (void)host_closeUser(host, fd);                                 /* process_emu_close (process.c:2946-2990) */
}

static void phold_start(Process* proc) {
    Host* host = proc->host;
    /* _phold_startListening (test_phold.c:232-268) */
    proc->listenfd = host_createDescriptor(host, DT_UDPSOCKET);
    Descriptor* desc = host_lookupDescriptor(host, proc->listenfd);
    descriptor_setFlags(desc, descriptor_getFlags(desc) | O_NONBLOCK);
    struct sockaddr_in bindAddr;
    memset(&bindAddr, 0, sizeof(bindAddr));
    bindAddr.sin_family = AF_INET;
    bindAddr.sin_addr.s_addr = htonl(INADDR_ANY);
    bindAddr.sin_port = htons(PHOLD_LISTEN_PORT);
    (void)host_bindToInterface(host, proc->listenfd, (struct sockaddr*)&bindAddr);
    /* epoll_create -> host_createDescriptor(DT_EPOLL) (process.c:1975-2003) */
    proc->epollfd = host_createDescriptor(host, DT_EPOLL);
    struct epoll_event ev;
    memset(&ev, 0, sizeof(ev));
    ev.events = EPOLLIN;
    ev.data.fd = proc->listenfd;
    (void)host_epollControl(host, proc->epollfd, EPOLL_CTL_ADD, proc->listenfd, &ev);
    /* _phold_bootstrapMessages (test_phold.c:225-230) */
    for (uint32_t i = 0; i < g_cfg->load; i++) phold_send_new_message(proc);
}

/* _phold_wait_and_process_events (test_phold.c:270-315), repeated while
 * epoll_wait would return at once (the main loop, 317-330) */
static void phold_continue(Process* proc) {
    Host* host = proc->host;
    for (;;) {
        struct epoll_event evs[10];
        gint nfds = 0;
        if (host_epollGetEvents(host, proc->epollfd, evs, 10, &nfds) != 0 || nfds <= 0) break;
        for (gint i = 0; i < nfds; i++) {
            for (;;) {
                gchar buffer[2048];
                in_addr_t ip = 0;
                in_port_t port = 0;
                gsize nBytes = 0;
                gint rc = host_receiveUserData(host, proc->listenfd, buffer, sizeof(buffer), &ip, &port, &nBytes);
                if (rc != 0 || nBytes == 0) break;
                /* one new message per byte read (test_phold.c:305-307); PHOLD's
                 * messages are 1 byte, the model's larger payloads (C5) keep
                 * one answer per datagram */
                const gsize nmsg = g_cfg->payload <= 1 ? nBytes : 1;
                for (gsize b = 0; b < nmsg; b++) phold_send_new_message(proc);
            }
        }
    }
}

/* ---- app 2: a UDP request/response echo over the same host_* calls (the
 * device application hook's second application, shdgpu.h SHD_APP_UDP_ECHO).
 * A server (peer -1) binds PHOLD_LISTEN_PORT and answers every datagram it
 * reads with one of `payload` bytes to the sender's address and port, from
 * its bound socket; a client opens one socket, sends `load` requests to its
 * server's listener (the first sendto binds the socket implicitly: one
 * random port, host.c:1514-1525) and answers every reply it reads with a new
 * request on the same socket -- a closed loop of `load` requests in flight.
 * cfg->proc_peer is indexed by host here: the server host of each client. */
static const gchar g_echo_buf[65536];

static void echo_send(Process* proc, in_addr_t ip, in_port_t port) {
    gsize bytes = 0;
    (void)host_sendUserData(proc->host, proc->listenfd, (gpointer)g_echo_buf, g_cfg->payload ? g_cfg->payload : 1,
                            ip, (in_addr_t)port, &bytes);
}

static void echo_start(Process* proc) {
    Host* host = proc->host;
    const int32_t h = host_index_of(host_getID(host));
    const int32_t peer = g_cfg->proc_peer[h];
    proc->listenfd = host_createDescriptor(host, DT_UDPSOCKET);
    Descriptor* desc = host_lookupDescriptor(host, proc->listenfd);
    descriptor_setFlags(desc, descriptor_getFlags(desc) | O_NONBLOCK);
    if (peer < 0) {
        struct sockaddr_in bindAddr;
        memset(&bindAddr, 0, sizeof(bindAddr));
        bindAddr.sin_family = AF_INET;
        bindAddr.sin_addr.s_addr = htonl(INADDR_ANY);
        bindAddr.sin_port = htons(PHOLD_LISTEN_PORT);
        (void)host_bindToInterface(host, proc->listenfd, (struct sockaddr*)&bindAddr);
    }
    proc->epollfd = host_createDescriptor(host, DT_EPOLL);
    struct epoll_event ev;
    memset(&ev, 0, sizeof(ev));
    ev.events = EPOLLIN;
    ev.data.fd = proc->listenfd;
    (void)host_epollControl(host, proc->epollfd, EPOLL_CTL_ADD, proc->listenfd, &ev);
    if (peer >= 0)
        for (uint32_t i = 0; i < g_cfg->load; i++)
            echo_send(proc, host_getDefaultIP(g_hosts[peer]), htons(PHOLD_LISTEN_PORT));
}

/* every readable datagram answered (as phold_continue's loop) */
static void echo_continue(Process* proc) {
    Host* host = proc->host;
    const int32_t peer = g_cfg->proc_peer[host_index_of(host_getID(host))];
    for (;;) {
        struct epoll_event evs[10];
        gint nfds = 0;
        if (host_epollGetEvents(host, proc->epollfd, evs, 10, &nfds) != 0 || nfds <= 0) break;
        for (gint i = 0; i < nfds; i++) {
            for (;;) {
                gchar buffer[65536];
                in_addr_t ip = 0;
                in_port_t port = 0;
                gsize nBytes = 0;
                gint rc = host_receiveUserData(host, proc->listenfd, buffer, sizeof(buffer), &ip, &port, &nBytes);
                if (rc != 0 || nBytes == 0) break;
                if (peer < 0) echo_send(proc, ip, port);
                else echo_send(proc, host_getDefaultIP(g_hosts[peer]), htons(PHOLD_LISTEN_PORT));
            }
        }
    }
}

/* ---- app 3: a datagram application per host (shdgpu.h shd_udp_app, the
 * device application hook's general form) over the same host_* calls as
 * test_phold.c.  send: 0 (EACH) listen on PHOLD's port, each datagram from a
 * new socket (socket, sendto -- its implicit bind draws a port --, close), as
 * _phold_sendToNode; 1 (ONCE) no listener, one socket whose first sendto binds
 * it, replies read on it; 2 (LISTENER) listen on PHOLD's port and send from it.
 * dest: 0 (WEIGHTED) _phold_chooseNode over the host's weights row, to PHOLD's
 * port (none drawn: nothing sent); 1 (PEER) app_peer[h]'s PHOLD port; 2 (REPLY)
 * the address and port recvfrom gave.  n_start datagrams when the process
 * starts; per_read: one datagram per datagram read, else none. */
static const uint32_t* udp_spec(int32_t h) { return g_cfg->app_spec + 4u * g_cfg->host_app[h]; }

static void udp_send(Process* proc, in_addr_t rip, in_port_t rport) {
    Host* host = proc->host;
    const int32_t h = host_index_of(host_getID(host));
    const uint32_t* a = proc->spec;
    in_addr_t ip;
    in_port_t port = htons(PHOLD_LISTEN_PORT);
    if (a[1] == 0) {
        const double r = ((double)random_rand(host_getRandom(host))) / ((double)RAND_MAX);
        const double* cum = g_cfg->dest_cum;
        if (g_cfg->host_class && g_cfg->n_classes > 1) cum += (size_t)g_cfg->host_class[h] * (size_t)g_cfg->n_hosts;
        int32_t chosen = -1;
        for (int32_t i = 0; i < g_cfg->n_hosts; i++)
            if (cum[i] >= r) { chosen = i; break; }
        if (chosen < 0) return;
        ip = host_getDefaultIP(g_hosts[chosen]);
    } else if (a[1] == 1) {
        ip = host_getDefaultIP(g_hosts[g_cfg->app_peer[h]]);
    } else {
        ip = rip;
        port = rport;
    }
    gsize bytes = 0;
    const gsize n = g_cfg->payload ? g_cfg->payload : 1;
    if (a[0] == 0) {
        gint fd = host_createDescriptor(host, DT_UDPSOCKET);
        Descriptor* desc = host_lookupDescriptor(host, fd);
        descriptor_setFlags(desc, descriptor_getFlags(desc) | O_NONBLOCK);
        (void)host_sendUserData(host, fd, (gpointer)g_echo_buf, n, ip, (in_addr_t)port, &bytes);
        (void)host_closeUser(host, fd);
    } else {
        (void)host_sendUserData(host, proc->listenfd, (gpointer)g_echo_buf, n, ip, (in_addr_t)port, &bytes);
    }
}

static void udp_start(Process* proc) {
    Host* host = proc->host;
    const uint32_t* a = proc->spec;
    proc->listenfd = host_createDescriptor(host, DT_UDPSOCKET);
    Descriptor* desc = host_lookupDescriptor(host, proc->listenfd);
    descriptor_setFlags(desc, descriptor_getFlags(desc) | O_NONBLOCK);
    if (a[0] != 1) {
        struct sockaddr_in bindAddr;
        memset(&bindAddr, 0, sizeof(bindAddr));
        bindAddr.sin_family = AF_INET;
        bindAddr.sin_addr.s_addr = htonl(INADDR_ANY);
        bindAddr.sin_port = htons(PHOLD_LISTEN_PORT);
        (void)host_bindToInterface(host, proc->listenfd, (struct sockaddr*)&bindAddr);
    }
    proc->epollfd = host_createDescriptor(host, DT_EPOLL);
    struct epoll_event ev;
    memset(&ev, 0, sizeof(ev));
    ev.events = EPOLLIN;
    ev.data.fd = proc->listenfd;
    (void)host_epollControl(host, proc->epollfd, EPOLL_CTL_ADD, proc->listenfd, &ev);
    for (uint32_t i = 0; i < a[2]; i++) udp_send(proc, 0, 0);
}

static void udp_continue(Process* proc) {
    Host* host = proc->host;
    const uint32_t* a = proc->spec;
    for (;;) {
        struct epoll_event evs[10];
        gint nfds = 0;
        if (host_epollGetEvents(host, proc->epollfd, evs, 10, &nfds) != 0 || nfds <= 0) break;
        for (gint i = 0; i < nfds; i++) {
            for (;;) {
                gchar buffer[65536];
                in_addr_t ip = 0;
                in_port_t port = 0;
                gsize nBytes = 0;
                gint rc = host_receiveUserData(host, proc->listenfd, buffer, sizeof(buffer), &ip, &port, &nBytes);
                if (rc != 0 || nBytes == 0) break;
                if (a[3]) udp_send(proc, ip, port);
            }
        }
    }
}

/* ---- app 1: src/test/tcp/test_tcp.c's echo test in its nonblocking-epoll
 * mode (_run_server / _run_client, test_tcp.c:713-810), restated over the
 * host_* calls the syscall handlers make.  The client fills its buffer with
 * rand() (_fillcharbuf, test_tcp.c:103-108: process_emu_rand draws the host
 * RNG, process.c:4772-4777), connects, sends tcp_bytes, reads them back and
 * closes; the server binds port 0 (a random port, host.c:1165-1170), listens,
 * accepts one peer, reads tcp_bytes, echoes them and closes both sockets.
 * The port reaches the client as the test's message queue hands it over
 * (test_tcp.c:268-273, 204-205).  A wait (_wait_epoll, test_tcp.c:132-174)
 * watches the descriptor for EPOLLIN / EPOLLOUT on the process's epoll and
 * removes the watch when the process continues. */
enum { T_SRV_START, T_SRV_ACCEPT, T_SRV_RECV, T_SRV_SEND, T_CLI_START, T_CLI_CONNECT, T_CLI_SEND,
       T_CLI_RECV, T_DONE };

static void tcp_wait(Process* proc, gint fd, uint32_t events) {
    Host* host = proc->host;
    struct epoll_event ev;
    memset(&ev, 0, sizeof(ev));
    ev.events = events;
    ev.data.fd = fd;
    proc->wait_fd = fd;
    (void)host_epollControl(host, proc->epollfd, EPOLL_CTL_ADD, fd, &ev);
}

static int tcp_server_port(int32_t spi, in_addr_t* ip, in_port_t* port) {
    Process* s = (spi >= 0 && spi < g_cfg->n_procs) ? g_procs[spi] : NULL;
    if (!s || s->listenfd < 0) return -1;
    Descriptor* d = host_lookupDescriptor(s->host, s->listenfd);
    if (!d) return -1;
    in_addr_t bip = 0;
    socket_getSocketName((Socket*)d, &bip, port);
    *ip = host_getDefaultIP(s->host);
    return 0;
}

static void tcp_run(Process* proc) {
    Host* host = proc->host;
    const uint32_t N = g_cfg->tcp_bytes;
    for (;;) {
        switch (proc->step) {
        case T_SRV_START: {
            proc->listenfd = host_createDescriptor(host, DT_TCPSOCKET);
            Descriptor* d = host_lookupDescriptor(host, proc->listenfd);
            descriptor_setFlags(d, descriptor_getFlags(d) | O_NONBLOCK);
            struct sockaddr_in a;
            memset(&a, 0, sizeof(a));
            a.sin_family = AF_INET;
            a.sin_addr.s_addr = htonl(INADDR_ANY);
            a.sin_port = 0;
            (void)host_bindToInterface(host, proc->listenfd, (struct sockaddr*)&a);
            (void)host_listenForPeer(host, proc->listenfd, 100);
            proc->step = T_SRV_ACCEPT;
            break;
        }
        case T_SRV_ACCEPT: {
            in_addr_t ip = 0;
            in_port_t port = 0;
            gint child = -1;
            gint rc = host_acceptNewPeer(host, proc->listenfd, &ip, &port, &child);
            if (rc == EWOULDBLOCK || rc == EAGAIN) { tcp_wait(proc, proc->listenfd, EPOLLIN); return; }
            if (rc != 0) { proc->step = T_DONE; return; }
            proc->fd = child;
            proc->done = 0;
            proc->step = T_SRV_RECV;
            break;
        }
        case T_SRV_RECV:
        case T_CLI_RECV: {
            while (proc->done < N) {
                in_addr_t ip = 0;
                in_port_t port = 0;
                gsize n = 0;
                gint rc = host_receiveUserData(host, proc->fd, proc->buf + proc->done, N - proc->done, &ip, &port, &n);
                if (rc == EWOULDBLOCK || rc == EAGAIN) { tcp_wait(proc, proc->fd, EPOLLIN); return; }
                if (rc != 0 || n == 0) break;   /* error or EOF */
                proc->done += (guint32)n;
            }
            if (proc->step == T_SRV_RECV) {
                proc->done = 0;
                proc->step = T_SRV_SEND;
            } else {
                (void)host_closeUser(host, proc->fd);
                proc->step = T_DONE;
            }
            break;
        }
        case T_SRV_SEND:
        case T_CLI_SEND: {
            while (proc->done < N) {
                gsize n = 0;
                gint rc = host_sendUserData(host, proc->fd, proc->buf + proc->done, N - proc->done, 0, 0, &n);
                if (rc == EWOULDBLOCK || rc == EAGAIN) { tcp_wait(proc, proc->fd, EPOLLOUT); return; }
                if (rc != 0 || n == 0) break;
                proc->done += (guint32)n;
            }
            if (proc->step == T_SRV_SEND) {
                (void)host_closeUser(host, proc->fd);
                (void)host_closeUser(host, proc->listenfd);
                proc->step = T_DONE;
            } else {
                proc->done = 0;
                proc->step = T_CLI_RECV;
            }
            break;
        }
        case T_CLI_START: {
            for (uint32_t i = 0; i < N; i++)
                proc->buf[i] = (gchar)('a' + random_rand(host_getRandom(host)) % 26);
            proc->fd = host_createDescriptor(host, DT_TCPSOCKET);
            Descriptor* d = host_lookupDescriptor(host, proc->fd);
            descriptor_setFlags(d, descriptor_getFlags(d) | O_NONBLOCK);
            proc->step = T_CLI_CONNECT;
            break;
        }
        case T_CLI_CONNECT: {
            struct sockaddr_in a;
            memset(&a, 0, sizeof(a));
            a.sin_family = AF_INET;
            if (tcp_server_port(g_cfg->proc_peer[proc->index], &a.sin_addr.s_addr, &a.sin_port) != 0) {
                proc->step = T_DONE;
                return;
            }
            gint rc = host_connectToPeer(host, proc->fd, (struct sockaddr*)&a);
            if (rc == EINPROGRESS || rc == EALREADY) { tcp_wait(proc, proc->fd, EPOLLOUT); return; }
            if (rc != 0 && rc != EISCONN) { proc->step = T_DONE; return; }
            proc->done = 0;
            proc->step = T_CLI_SEND;
            break;
        }
        default:
            return;
        }
    }
}

static void tcp_start(Process* proc) {
    proc->buf = g_malloc0(g_cfg->tcp_bytes ? g_cfg->tcp_bytes : 1);
    proc->epollfd = host_createDescriptor(proc->host, DT_EPOLL);
    proc->step = g_cfg->proc_peer[proc->index] < 0 ? T_SRV_START : T_CLI_START;
    tcp_run(proc);
}

static void tcp_continue(Process* proc) {
    Host* host = proc->host;
    struct epoll_event evs[4];
    gint nfds = 0;
    if (host_epollGetEvents(host, proc->epollfd, evs, 4, &nfds) != 0 || nfds <= 0) return;
    (void)host_epollControl(host, proc->epollfd, EPOLL_CTL_DEL, proc->wait_fd, NULL);
    proc->wait_fd = -1;
    tcp_run(proc);
}

static void process_start_task(Process* proc, gpointer nothing) {
    /* _process_start (process.c:1055-1195): the process runs its main until it
     * blocks */
    if (proc->running) return;
    worker_setActiveProcess(proc);
    proc->running = TRUE;
    if (g_cfg->app == 1 && g_cfg->proc_app && proc->index >= 0 && g_cfg->proc_app[proc->index] >= 0)
        proc->spec = g_cfg->app_spec + 4u * (uint32_t)g_cfg->proc_app[proc->index];
    else if (g_cfg->app == 3)
        proc->spec = udp_spec(host_index_of(host_getID(proc->host)));
    if (g_cfg->app == 0) phold_start(proc);
    else if (proc->spec) udp_start(proc);
    else if (g_cfg->app == 1) tcp_start(proc);
    else if (g_cfg->app == 2) echo_start(proc);
    worker_setActiveProcess(NULL);
}
static void process_stop_task(Process* proc, gpointer nothing) { process_stop(proc); }

void process_schedule(Process* proc, gpointer nothing) {
    /* process.c:1334-1357 */
    SimulationTime now = worker_getCurrentTime();
    if (proc->stopTime == 0 || proc->startTime < proc->stopTime) {
        SimulationTime startDelay = proc->startTime <= now ? 1 : proc->startTime - now;
        process_ref(proc);
        Task* t = task_new((TaskCallbackFunc)process_start_task, proc, NULL, (TaskObjectFreeFunc)process_unref, NULL);
        worker_scheduleTask(t, startDelay);
        task_unref(t);
    }
    if (proc->stopTime > 0 && proc->stopTime > proc->startTime) {
        SimulationTime stopDelay = proc->stopTime <= now ? 1 : proc->stopTime - now;
        process_ref(proc);
        Task* t = task_new((TaskCallbackFunc)process_stop_task, proc, NULL, (TaskObjectFreeFunc)process_unref, NULL);
        worker_scheduleTask(t, stopDelay);
        task_unref(t);
    }
}

void process_continue(Process* proc) {
    if (!process_isRunning(proc)) return;
    worker_setActiveProcess(proc);
    if (g_cfg->app == 0) phold_continue(proc);
    else if (proc->spec) udp_continue(proc);
    else if (g_cfg->app == 1) tcp_continue(proc);
    else if (g_cfg->app == 2) echo_continue(proc);
    worker_setActiveProcess(NULL);
}

/* ------------------------------------------------------------ the run */
int ref_loop_run(const ref_loop_cfg* cfg, ref_loop_out* out) {
    if (!cfg || !out || cfg->n_hosts <= 0 || !cfg->path) return -1;
    g_cfg = cfg;
    g_out = out;
    memset(out, 0, sizeof(*out));
    const int32_t H = cfg->n_hosts;
    out->ip = calloc((size_t)H, sizeof(uint32_t));
    out->next_event_id = calloc((size_t)H, sizeof(uint64_t));
    out->next_packet_id = calloc((size_t)H, sizeof(uint64_t));
    out->rng_probe = calloc((size_t)H, sizeof(uint32_t));

    /* the CLI defaults (options.c:60-240) with one config file argument */
    gchar* argv[] = {"shadow", "shadow.config.xml", NULL};
    gchar* argv_rr[] = {"shadow", "--interface-qdisc=rr", "shadow.config.xml", NULL};
    g_options = cfg->qdisc_rr ? options_new(3, argv_rr) : options_new(2, argv);
    if (!g_options) return -2;
    g_dns = dns_new();
    Scheduler* sched = scheduler_new(SP_SERIAL_GLOBAL, 0, &g_slave, 1, cfg->end_time);
    g_sched = sched;
    g_hosts = calloc((size_t)H, sizeof(Host*));
    if (cfg->app == 1) {
        if (cfg->n_procs <= 0 || !cfg->proc_peer) return -3;
        g_procs = calloc((size_t)cfg->n_procs, sizeof(Process*));
    }
    for (int32_t i = 0; i < H; i++) {
        /* master.c:300-380 (host parameters), slave_addNewVirtualHost (host_new +
         * host_setup + scheduler_addHost) */
        HostParameters p;
        memset(&p, 0, sizeof(p));
        char name[32];
        snprintf(name, sizeof(name), "peer%d", i + 1);
        p.id = (GQuark)(i + 1);
        p.nodeSeed = cfg->host_seed[i];
        p.hostname = name;
        p.cpuFrequency = 2500000;
        p.cpuThreshold = 0;
        p.cpuPrecision = 200;
        p.logLevel = options_getLogLevel(g_options);
        p.heartbeatLogLevel = options_getHeartbeatLogLevel(g_options);
        p.heartbeatInterval = cfg->host_heartbeat ? cfg->host_heartbeat[i] : cfg->heartbeat_interval;
        p.heartbeatLogInfo = options_getHeartbeatLogInfo(g_options);
        p.recvBufSize = options_getSocketReceiveBufferSize(g_options);
        p.autotuneRecvBuf = options_doAutotuneReceiveBuffer(g_options);
        p.sendBufSize = options_getSocketSendBufferSize(g_options);
        p.autotuneSendBuf = options_doAutotuneSendBuffer(g_options);
        p.interfaceBufSize = options_getInterfaceBufferSize(g_options);
        p.qdisc = options_getQueuingDiscipline(g_options);
        Host* host = host_new(&p);
        host_setup(host, g_dns, (Topology*)&g_topology, 0, cfg->root_dir);
        if (cfg->app == 1) {
            for (int32_t k = 0; k < cfg->n_procs; k++)
                if (cfg->proc_host[k] == i) {
                    char arg[16];
                    snprintf(arg, sizeof(arg), "%d", k);
                    host_addApplication(host, cfg->proc_start[k], 0, "testtcp", "testtcp.so", NULL, NULL, NULL, arg);
                }
        } else if (cfg->n_procs > 0) {
            for (int32_t k = 0; k < cfg->n_procs; k++)
                if (cfg->proc_host[k] == i)
                    host_addApplication(host, cfg->proc_start[k], 0, "phold", "phold.so", NULL, NULL, NULL, "");
        } else {
            const uint64_t st = cfg->host_start ? cfg->host_start[i] : cfg->app_start;
            host_addApplication(host, st, 0, "phold", "phold.so", NULL, NULL, NULL, "");
        }
        scheduler_addHost(sched, host);
        g_hosts[i] = host;
        out->ip[i] = ntohl(host_getDefaultIP(host));
    }
    scheduler_start(sched);
    WorkerRunData* data = g_new0(WorkerRunData, 1);
    data->threadID = 0;
    data->scheduler = sched;
    data->userData = &g_slave;
    /* boots the hosts, pops every event before the end time, then shuts the
     * hosts down (scheduler_awaitFinish; the end state is read in
     * topology_detach) */
    worker_run(data);
    g_out = NULL;
    g_sched = NULL;
    return 0;
}

void ref_loop_free(ref_loop_out* out) {
    if (!out) return;
    free(out->lines);
    free(out->ip);
    free(out->next_event_id);
    free(out->next_packet_id);
    free(out->rng_probe);
    memset(out, 0, sizeof(*out));
}
