/*
 * shdgpu.h -- C-ABI of libshdgpu, the MI355X-native simulated-network core.
 *
 * libshdgpu replaces two pieces of Shadow 1.14 (joskid/shadow-1):
 *
 *   1. the topology PATH CACHE (src/main/routing/topology.c), which maps a
 *      (source vertex, destination vertex) pair to a latency (ms) and a
 *      reliability, built lazily with igraph Dijkstra;
 *   2. the conservative round/window PACKET EVENT LOOP (src/main/core/scheduler/,
 *      master.c, slave.c, worker.c) that delivers packets between hosts through
 *      the path cache, the reliability drop, the per-host RNG, the CoDel router
 *      queue and the receive token bucket.
 *
 * Conventions: plain C types only, opaque handles, every call returns 0 or a
 * negative errno-style status (SHD_E*).  No exceptions cross the ABI.  The
 * library owns device buffers; callers own host buffers (copied in).  An engine
 * handle is driven by ONE host thread and is not re-entrant.
 *
 * Reference interfaces each entry point replaces are cited per declaration
 * (paths relative to the reference repository root).  The ctypes / C binding a
 * Shadow maintainer would add is shown in INTEGRATION.md.
 */
#ifndef SHDGPU_H
#define SHDGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- status */
#define SHD_OK 0
#define SHD_EINVAL (-22)     /* bad argument / invalid graph                 */
#define SHD_ENOMEM (-12)     /* host or device allocation failed             */
#define SHD_ENODEV (-19)     /* no HIP device / HIP runtime error            */
#define SHD_EOVERFLOW (-75)  /* a fixed-capacity device queue overflowed     */
#define SHD_ERANGE (-34)     /* path longer than supported / bad index       */
#define SHD_EAMBIG (-125)    /* first-touch drop decision ambiguous */
#define SHD_ENOTCONN (-107)  /* topology not strongly connected (topology.c:800-806) */

/* time: unsigned nanoseconds, SimulationTime (core/support/definitions.h:18-64) */
#define SHD_SIMTIME_INVALID UINT64_MAX
#define SHD_SIMTIME_MAX (UINT64_MAX - 1)
#define SHD_MS 1000000ULL
#define SHD_SEC 1000000000ULL
#define SHD_MTU 1500u                 /* CONFIG_MTU, definitions.h:188            */
#define SHD_HEADER_UDP 42u            /* CONFIG_HEADER_SIZE_UDPIPETH, definitions.h:176 */
#define SHD_MIN_RANDOM_PORT 10000u    /* MIN_RANDOM_PORT, definitions.h:94        */
#define SHD_PHOLD_LISTEN_PORT 8998u   /* PHOLD_LISTEN_PORT, src/test/phold/test_phold.c:34 */

/* ------------------------------------------------------------ graph input */
/*
 * A topology graph as read from graphml (topology.c:371-399, igraph document
 * order): vertex ids and edge ids are document order.  For undirected graphs an
 * edge (a,b) is stored once.  Absent numeric attributes are NaN
 * (_topology_findVertexAttributeDouble treats NaN as absent, topology.c:330-347).
 */
typedef struct shd_graph {
    int32_t n_vertices;
    int32_t n_edges;
    int32_t directed;               /* graphml edgedefault="directed"          */
    int32_t prefer_direct;          /* graph attr preferdirectpaths true/yes/1 (topology.c:760-790) */
    const int32_t* edge_src;        /* [E] document order                      */
    const int32_t* edge_dst;        /* [E]                                     */
    const double* edge_latency;     /* [E] ms, > 0 (topology.c:1070)          */
    const double* edge_loss;        /* [E] in [0,1] (topology.c:1090)         */
    const double* vertex_loss;      /* [V] or NULL; NaN = attribute absent    */
} shd_graph;

/* Validation of topology_new (topology.c:1187-1210): strongly connected, one
 * cluster, latency > 0, loss in [0,1].  Also reports the completeness test of
 * _topology_isComplete (topology.c:450-552). */
typedef struct shd_graph_props {
    int32_t is_connected;
    int32_t is_complete;
    int32_t is_directed;
    int32_t prefer_direct;
    int32_t n_self_loops;
    int32_t max_out_degree;
} shd_graph_props;
int shd_graph_check(const shd_graph* g, shd_graph_props* out);

/* graphml loader (libxml2, the parser igraph 0.7.1 uses).  Replaces
 * igraph_read_graph_graphml + the attribute extraction of topology.c:371-399,
 * 565-722, 1212-1246.  Arrays are allocated by the library; free with
 * shd_graphml_free.  Vertex string attributes are returned for attach. */
typedef struct shd_graphml {
    shd_graph g;
    double* bw_down;                /* [V] vertex bandwidthdown (KiB/s), NaN if absent */
    double* bw_up;                  /* [V] vertex bandwidthup                  */
    char** vertex_id;               /* [V] "id" attribute (graphml node id)    */
    char** vertex_ip;               /* [V] "ip" or NULL                        */
    char** vertex_citycode;         /* [V] or NULL                             */
    char** vertex_countrycode;      /* [V] or NULL                             */
    char** vertex_geocode;          /* [V] or NULL                             */
    char** vertex_type;             /* [V] or NULL                             */
    double* edge_jitter;            /* [E] NaN if absent                       */
} shd_graphml;
int shd_graphml_load_file(const char* path, shd_graphml** out);
int shd_graphml_load_string(const char* xml, size_t len, shd_graphml** out);

/* ------------------------------------------------------------ config front-end */
/*
 * shadow.config.xml -> the registered host list (core/support/configuration.c,
 * core/master.c:304-320,397): hosts in document order, `quantity` copies named
 * "<id><i>" (i from 1) when quantity > 1, their hints and bandwidth overrides;
 * the topology as a path or inline graphml (CDATA).  Units as in the file:
 * seconds, KiB/s.
 */
typedef struct shd_config_host {
    char* name;
    char* ip_hint;          /* NULL when absent, as are the other hints */
    char* citycode_hint;
    char* countrycode_hint;
    char* geocode_hint;
    char* type_hint;
    uint64_t bw_down_kibps; /* 0 = take the attached vertex's bandwidth (host.c:183-189) */
    uint64_t bw_up_kibps;
    uint64_t heartbeat_s;   /* 0 = the option default */
    int32_t n_processes;    /* <process> / <application> children, document order */
    int32_t _pad;
    uint64_t* process_start_s;   /* [n_processes] starttime (or legacy time), seconds
                                  * (configuration.c:576-579; master.c:299 scales by 1 s) */
} shd_config_host;
typedef struct shd_config {
    int32_t n_hosts;
    shd_config_host* hosts;
    uint64_t stop_time_s;       /* <shadow stoptime> (or legacy <kill time>) */
    uint64_t bootstrap_time_s;  /* <shadow bootstraptime> */
    char* topology_path;        /* <topology path>, NULL if inline */
    char* topology_text;        /* inline graphml, NULL if by path */
} shd_config;
int shd_config_load_file(const char* path, shd_config** out);
int shd_config_load_buffer(const char* xml, size_t len, shd_config** out);
void shd_config_free(shd_config* c);
/* dns_register in registration order (dns.c:102-134, host.c:166-167): each
 * host's ethernet IPv4 (host byte order) -- the hint when it is unrestricted and
 * not taken (127.0.0.1 stays local), else the next address after 11.0.0.0 that
 * is neither reserved nor taken.  ip_out has n_hosts entries. */
int shd_dns_assign(const shd_config* c, uint32_t* ip_out);
void shd_graphml_free(shd_graphml* gm);

/* ------------------------------------------------------------ path cache */
/*
 * Path-cache build.  Replaces the lazy cache of _topology_getPathEntry
 * (topology.c:1969-2051) and everything it calls:
 *   direct paths  _topology_lookupDirectPath        topology.c:1877-1927
 *   source rows   _topology_computeSourcePaths      topology.c:1655-1875
 *                 (igraph_get_shortest_paths_dijkstra, topology.c:1756)
 *   properties    _topology_computePathProperties   topology.c:1407-1523
 *   self paths    _topology_computeShortestPathToSelf topology.c:1545-1653
 *
 * The device computes, for every attached source vertex, its full row to every
 * attached target (the values _topology_computeSourcePaths would store), the
 * direct-path value of every adjacent attached pair and the "2 x min incident
 * edge" self value.  The reference's write-once / first-touch selection rules
 * (topology.c:1307-1336, 1988-1990, 2034-2037) are applied on top by
 * shd_pc_lookup (host, low rate) and by the engine (device, per packet).
 *
 * Tables are [n_attached][n_attached] row-major f64 in HBM, indexed by the
 * position of a vertex in the `attached` array given at creation.
 */
typedef struct shd_pc shd_pc;

#define SHD_PC_FORCE_ROWS 0x1u   /* compute SSSP rows even on complete graphs (C2 forced mode) */
#define SHD_PC_NO_TABLES_ON_HOST 0x2u

typedef struct shd_pc_info {
    int32_t n_vertices;
    int32_t n_attached;
    int32_t is_complete;
    int32_t is_directed;
    int32_t prefer_direct;
    int32_t rows_computed;          /* rows built (0 in pure direct mode)      */
    int64_t n_ties;                 /* vertices whose shortest-path parent was not unique */
    int32_t max_hops;               /* longest shortest path (edges)           */
    int32_t sssp_iterations_max;    /* deepest frontier iteration count        */
    int32_t n_unroutable;           /* row entries with no path (self without self-loop) */
    double min_latency_ms;          /* min over all table latencies (topology.c:1374-1378) */
    double build_ms_device;         /* device time of the table build (HIP events) */
    double build_ms_sssp;           /* device time of the SSSP-row kernel alone */
    double build_ms_props;          /* device time of the path-properties kernel */
    double build_ms_direct;         /* device time of the direct-table kernel   */
    int32_t n_tie_rows;             /* rows whose parents came from the restated igraph heap
                                       (k_sssp_tie_g / k_sssp_tie_parents: equal-cost
                                       predecessors) */
    int32_t n_tie_rows_global;      /* ... of them run again through lane heaps in global
                                       scratch (k_sssp_tie_parents: a heap past the LDS one) */
    int32_t n_tie_rows_predicted;   /* ... of them listed without a first pass: a build on
                                       whole-number weights whose probe rows (2 x CUs) were
                                       90 % tied (round 6; their ties counted in the second
                                       pass, sssp_iterations_max over the probe only) */
    int32_t _pad0;
} shd_pc_info;

/* attached: vertex ids with >=1 attached host (topology.c:2393, verticesWithAttachedHosts) */
int shd_pc_create(const shd_graph* g, const int32_t* attached, int32_t n_attached,
                  uint32_t flags, int device, shd_pc** out);
int shd_pc_build(shd_pc* pc);
int shd_pc_get_info(const shd_pc* pc, shd_pc_info* out);
/* D2H copy of source rows [row0, row0+nrows) of the row tables (lat ms, rel) */
int shd_pc_copy_rows(shd_pc* pc, int32_t row0, int32_t nrows, double* lat, double* rel);
/* D2H copy of the direct tables (only adjacent pairs valid; NaN elsewhere) */
int shd_pc_copy_direct(shd_pc* pc, int32_t row0, int32_t nrows, double* lat, double* rel);
/* D2H copy of the per-attached-vertex self values (2*min incident edge) */
int shd_pc_copy_self(shd_pc* pc, double* lat, double* rel);
/* Lazy lookup with the reference's first-touch semantics (serial order of the
 * calls = the reference's serial event order).  Replaces topology_getLatency /
 * topology_getReliability (topology.c:2065-2087).  Returns latency -1 and
 * reliability -1 when the reference would (error path, topology.c:2040-2046). */
int shd_pc_lookup(shd_pc* pc, int32_t src_vertex, int32_t dst_vertex, double* lat, double* rel);
/* n shd_pc_lookup calls in array order (the same first-touch semantics, ranks
 * and minimumPathLatency), in one device round trip: the driver of the TCP
 * path resolves its [V, V] path tables with it (shadow-1_amd/tcp.py).  Under
 * shd_pc_defer_touches' protocol the queries run one by one. */
int shd_pc_lookup_batch(shd_pc* pc, const int32_t* src_vertex, const int32_t* dst_vertex, uint64_t n,
                        double* lat, double* rel);
/* topology_incrementPathPacketCounter (topology.c:2053-2063) + read back */
int shd_pc_count_packet(shd_pc* pc, int32_t src_vertex, int32_t dst_vertex);
int shd_pc_packet_count(shd_pc* pc, int32_t src_vertex, int32_t dst_vertex, uint64_t* count);
/* master_updateMinTimeJump / _master_getMinTimeJump (master.c:133-159):
 * (u64)floor(min stored latency ms) * 1e6 ns, 10 ms default if 0, >= runahead */
int shd_pc_min_time_jump(shd_pc* pc, uint64_t runahead_ns, uint64_t* jump_ns);
/* the topology's minimumPathLatency (ms) over the entries stored so far
 * (topology.c:1374-1378); 0 before any (the value worker_updateMinTimeJump gets) */
int shd_pc_min_stored_latency(shd_pc* pc, double* ms);
void shd_pc_destroy(shd_pc* pc);

/* ------------------------------------------------------------ RNG / seeds */
/* glibc rand_r as used by utility/random.c:32-51 */
int32_t shd_rand_r(uint32_t* state);
double shd_next_double(uint32_t* state);          /* random.c:39-43 */
uint32_t shd_next_uint(uint32_t* state);          /* random.c:45-51 */
/* seed chain master.c:95,417 -> slave.c:182,198 -> slave.c:301 (registration order) */
int shd_seed_chain(uint32_t options_seed, int32_t n_hosts, uint32_t* host_seeds);

/* ------------------------------------------------------------ attach */
/* _topology_findAttachmentVertex (topology.c:2248-2369): hint filtering, exact
 * IP match, longest-prefix match, else random pick with the host RNG
 * (one nextDouble draw, topology.c:2326-2334).  Hints may be NULL. */
int shd_topology_attach(const shd_graphml* gm, uint32_t* host_rng_state, const char* ip_hint,
                        const char* citycode_hint, const char* countrycode_hint,
                        const char* geocode_hint, const char* type_hint,
                        int32_t* vertex_out, uint64_t* bw_down_out, uint64_t* bw_up_out);
/* the same with the caller's RNG: next_double(rng) is the host's
 * random_nextDouble (random.c:39-43), drawn once when the pick is random */
int shd_topology_attach_cb(const shd_graphml* gm, double (*next_double)(void*), void* rng,
                           const char* ip_hint, const char* citycode_hint, const char* countrycode_hint,
                           const char* geocode_hint, const char* type_hint,
                           int32_t* vertex_out, uint64_t* bw_down_out, uint64_t* bw_up_out);

/* ------------------------------------------------------------ engine */
/*
 * The packet event loop for the PHOLD-UDP model (DESIGN.md section "Model"):
 * per-host application from src/test/phold/test_phold.c on the reference's own
 * socket / interface / router / worker path:
 *   worker_sendPacket            core/worker.c:260-321
 *   _worker_runDeliverPacketTask core/worker.c:253-258, routing/router.c:104-133
 *   CoDel                        routing/router_queue_codel.c:113-267
 *   token buckets + refill       host/network_interface.c:102-226, 421-455, 519-579
 *   event order                  core/work/event.c:110-153
 *   window / rounds              core/master.c:450-480, core/slave.c:413-466
 * Hosts [host_begin, host_end) of the model live on this engine's device
 * (one engine per GPU; see DESIGN.md "Multi-GPU").
 */
typedef struct shd_model {
    int32_t n_hosts;
    int32_t _pad0;
    const int32_t* host_vertex;     /* [H] graph vertex id                     */
    const uint32_t* host_rng;       /* [H] RNG state at boot (after attach draw) */
    const uint64_t* bw_down_kibps;  /* [H]                                     */
    const uint64_t* bw_up_kibps;    /* [H]                                     */
    const double* dest_cum;         /* [H] PHOLD cumulative weights (test_phold.c:160-178) */
    uint64_t end_time;              /* <shadow stoptime> / kill time (ns)      */
    uint64_t bootstrap_end;         /* <shadow bootstraptime> (ns)             */
    uint64_t heartbeat_interval;    /* --heartbeat-frequency (ns), options.c:85 */
    uint64_t app_start;             /* <application starttime> (ns)            */
    uint32_t load;                  /* PHOLD load=                             */
    uint32_t payload;               /* message bytes (PHOLD sends 1)           */
    uint32_t trace;                 /* record delivered-packet trace           */
    uint32_t evq_cap;               /* per-host event heap capacity (0=default) */
    uint32_t inbox_cap;             /* per-host per-round inbound capacity     */
    uint32_t codelq_cap;            /* per-host router queue capacity (<= 65535, and
                                       x (payload + 42) below 2^32; 0 = 64)    */
    uint32_t txq_cap;               /* per-host interface send queue capacity (<= 65535; 0 = 64) */
    uint32_t queue_flags;           /* SHD_QF_*: 0 = default (calendar + heap) */
    /* Per-host variants (NULL / 0 = the scalar above for every host).  Each PHOLD
     * process reads its own weights file (test_phold.c:341-356, per-process
     * arguments), so hosts of different classes draw destinations from
     * different cumulative weights: dest_cum is then [n_classes][H] and
     * host_class[h] picks the row (the Tor-scale model: relays and clients). */
    const uint8_t* host_class;      /* [H] or NULL (every host class 0)        */
    int32_t n_classes;              /* rows of dest_cum (0 = 1)                */
    int32_t _pad1;
    /* <host heartbeatfrequency> per host (ns), tracker interval (host.c:240) */
    const uint64_t* host_heartbeat; /* [H] or NULL                             */
    /* The application every host runs (the device application hook):
     *   SHD_APP_PHOLD     test_phold.c (load, dest_cum, host_class above);
     *   SHD_APP_UDP_ECHO  a UDP request/response echo: app_peer[h] = -1 makes h a
     *                     server on PHOLD's port answering every datagram it reads
     *                     with `payload` bytes to the sender's address and port;
     *                     app_peer[h] = s makes h a client of server host s that
     *                     keeps `load` requests in flight on one socket (the
     *                     first sendto binds it: one random port). */
    uint32_t app;                   /* SHD_APP_*                               */
    int32_t _pad2;
    const int32_t* app_peer;        /* [H] (SHD_APP_UDP_ECHO; SHD_APP_UDP's SHD_DEST_PEER
                                       hosts: the host sent to) or NULL          */
    /*   SHD_APP_UDP       a datagram application per host: host h runs
     *                     app_spec[host_app[h]] (shd_udp_app below); PHOLD is
     *                     {SHD_SEND_EACH, SHD_DEST_WEIGHTED, load, 1}, the echo's
     *                     server {SHD_SEND_LISTENER, SHD_DEST_REPLY, 0, 1} and
     *                     client {SHD_SEND_ONCE, SHD_DEST_PEER, load, 1}. */
    const struct shd_udp_app* app_spec;   /* [n_app_specs] (SHD_APP_UDP) or NULL */
    const uint8_t* host_app;        /* [H] (SHD_APP_UDP) or NULL               */
    uint32_t n_app_specs;           /* <= 256                                  */
    uint32_t _pad3;
} shd_model;

enum { SHD_APP_PHOLD = 0, SHD_APP_UDP_ECHO = 1, SHD_APP_UDP = 2 };

/* SHD_APP_UDP: what a host's process does at its start and with each datagram
 * it reads, over the calls test_phold.c makes (socket, bind, sendto, recvfrom,
 * close; udp.c:75-142).  Every datagram carries the model's `payload` bytes.
 *   send  SHD_SEND_EACH      listen on PHOLD's port; each datagram from a new
 *                            socket (an implicit bind: one port draw each,
 *                            host.c:1514-1525), closed after the sendto;
 *         SHD_SEND_LISTENER  listen on PHOLD's port and send from that socket;
 *         SHD_SEND_ONCE      no listener: one socket, bound by its first sendto
 *                            (one port draw); replies are read on it.
 *   dest  SHD_DEST_WEIGHTED  _phold_chooseNode over the host's dest_cum row (no
 *                            host drawn: nothing sent), to PHOLD's port;
 *         SHD_DEST_PEER      app_peer[h], to PHOLD's port;
 *         SHD_DEST_REPLY     the source address and port of the datagram just
 *                            read (n_start must be 0).
 *   n_start   datagrams sent when the process starts;
 *   per_read  1: one datagram per datagram read (PHOLD's rule); 0: read only.
 * shd_eng_create refuses (SHD_EINVAL) a model whose datagrams could reach a
 * port no socket listens on: a weighted or peer destination that does not
 * listen (SHD_SEND_ONCE), a replying host that an SHD_SEND_EACH host can send
 * to, or SHD_SEND_EACH with SHD_DEST_REPLY. */
typedef struct shd_udp_app {
    uint32_t send, dest, n_start, per_read;
} shd_udp_app;
enum { SHD_SEND_EACH = 0, SHD_SEND_ONCE = 1, SHD_SEND_LISTENER = 2 };
enum { SHD_DEST_WEIGHTED = 0, SHD_DEST_PEER = 1, SHD_DEST_REPLY = 2 };

/* queue_flags: SHD_QF_NO_CALENDAR routes every inter-host event through the
 * per-host inbox and heap (the calendar's fallback path), for testing */
enum { SHD_QF_NO_CALENDAR = 1,
       /* count packets per cached path entry on the device (incrementPathPacketCounter,
        * topology.c:2053-2063 / worker.c:296; read with shd_eng_path_counts) */
       SHD_QF_COUNT_PATHS = 2,
       /* keep every host's tracker node counters at each heartbeat (tracker_heartbeat,
        * tracker.c:566-611; read with shd_eng_heartbeats) */
       SHD_QF_HEARTBEATS = 4,
       /* boot schedules no application start: the caller pushes each host's
        * process start events (<process starttime>, process_schedule,
        * process.c:1344) with shd_eng_push_events */
       SHD_QF_NO_APP_START = 8,
       /* with `trace`: also the application's side of each datagram
        * (SHD_TR_CREATED, SHD_TR_READ), for the [STATUS] packet lines
        * (packet_addDeliveryStatus, packet.c:647-659; shdgpu.status_lines) */
       SHD_QF_TRACE_STATUS = 16 };

/* one event (32 B): key (time, dst, src, seq) = event_compare, event.c:110-153 */
typedef struct shd_event {
    uint64_t time;
    uint64_t seq;                   /* srcHostEventID (host_getNewEventID, host.c:397) */
    uint32_t src;
    uint32_t dst;
    uint32_t pkt;                   /* packet id on src (host_getNewPacketID) */
    uint32_t kind;                  /* SHD_EV_*                                */
} shd_event;

enum {
    SHD_EV_HEARTBEAT = 1,   /* tracker_heartbeat, host/tracker.c:566-611            */
    SHD_EV_REFILL = 2,      /* _networkinterface_refillTokenBucketsCB, n_i.c:163-183 */
    SHD_EV_REFILL_LO = 3,   /* loopback interface refill (one at boot)               */
    SHD_EV_APP_START = 4,   /* process start task, host/process.c:1344               */
    SHD_EV_PACKET = 5,      /* _worker_runDeliverPacketTask, worker.c:253            */
    SHD_EV_LOCAL = 6,       /* loopback shortcut +1 ns, network_interface.c:548-555 */
    SHD_EV_NOTIFY = 7       /* epoll notification +1 ns, descriptor/epoll.c:345-365 */
};

/* trace record (32 B): one per packet state change, compared as a multiset */
typedef struct shd_trace_rec {
    uint64_t time;
    uint64_t seq;                   /* event seq for ARRIVE, else 0            */
    uint32_t host;                  /* host where it happened                  */
    uint32_t peer;                  /* the other host of the packet            */
    uint32_t pkt;                   /* packet id on its source host            */
    uint32_t kind;                  /* SHD_TR_*                                */
} shd_trace_rec;

enum {
    SHD_TR_SENT = 1,        /* PDS_INET_SENT at the sender (worker.c:300)            */
    SHD_TR_INET_DROP = 2,   /* PDS_INET_DROPPED (worker.c:319)                       */
    SHD_TR_ARRIVE = 3,      /* deliver event executed = PDS_ROUTER_ENQUEUED          */
    SHD_TR_CODEL_DROP = 4,  /* PDS_ROUTER_DROPPED in CoDel (router_queue_codel.c:135) */
    SHD_TR_RECV = 5,        /* PDS_RCV_INTERFACE_RECEIVED (network_interface.c:380)  */
    SHD_TR_IF_DROP = 6,     /* PDS_RCV_INTERFACE_DROPPED (no bound socket)           */
    SHD_TR_LOCAL = 7,       /* loopback shortcut delivery                            */
    /* SHD_QF_TRACE_STATUS only: */
    SHD_TR_CREATED = 8,     /* the application's sendto: PDS_SND_CREATED (udp.c:116) and
                               PDS_SND_SOCKET_BUFFERED (socket.c:405); seq = the source
                               port drawn by the implicit bind (host.c:1058-1110), peer =
                               ~0 (the destination is in the packet's SENT / INET_DROP /
                               LOCAL record)                                             */
    SHD_TR_READ = 9         /* the application's recvfrom of the socket's oldest datagram:
                               PDS_RCV_SOCKET_DELIVERED (udp.c:158); peer = pkt = ~0     */
};

/* per-host end state, compared bit for bit against the oracle */
typedef struct shd_host_digest {
    uint64_t ev_seq;
    uint64_t rx_remaining;
    uint64_t tx_remaining;
    uint64_t codel_total;
    uint64_t codel_interval_expire;
    uint64_t codel_next_drop;
    uint64_t n_events;
    uint64_t n_pkt_events;
    uint64_t n_sent;
    uint64_t n_inet_drop;
    uint64_t n_codel_drop;
    uint64_t n_recv;
    uint32_t rng;
    uint32_t pkt_seq;
    uint32_t codel_mode;
    uint32_t codel_count;
    uint32_t codel_drop_count;
    uint32_t codel_drop_count_last;
    uint32_t unread;
    uint32_t flags;
} shd_host_digest;

typedef struct shd_round_summary {
    uint64_t window_start;
    uint64_t window_end;
    uint64_t next_time;             /* min next event time on this engine      */
    uint64_t n_events;              /* events executed this round              */
    uint64_t n_pkt_events;          /* packet-deliver events executed          */
    uint64_t n_pending;             /* sends awaiting first-touch resolution   */
    uint64_t n_remote;              /* events for hosts of other engines       */
    uint32_t error;                 /* SHD_ERR_* bits                          */
    uint32_t _pad;
} shd_round_summary;

enum {
    SHD_ERR_EVQ_OVERFLOW = 1, SHD_ERR_INBOX_OVERFLOW = 2, SHD_ERR_CODELQ_OVERFLOW = 4,
    SHD_ERR_TXQ_OVERFLOW = 8, SHD_ERR_AMBIGUOUS = 16, SHD_ERR_PENDING_OVERFLOW = 32,
    SHD_ERR_TRACE_OVERFLOW = 64, SHD_ERR_REMOTE_OVERFLOW = 128,
    SHD_ERR_INTERNAL = 0x80000000u  /* engine invariant broken (bad event kind, timer slot reuse) */
};

typedef struct shd_run_stats {
    uint64_t n_rounds;
    uint64_t n_events;
    uint64_t n_pkt_events;
    uint64_t n_pending_resolved;
    uint64_t window_ns;             /* the serial-equivalent window W          */
    uint64_t final_time;
    double device_ms_round_kernel;  /* round-kernel time, device wall clock (first block start
                                       to last block end, summed over rounds) */
    double wall_ms;
    double device_ms_launches;      /* HIP-event time of the round launches on the engine's
                                       stream (batches; includes the gaps between launches) */
    uint32_t error;
    uint32_t n_batches_ticketless;  /* device batches run without the completion ticket
                                       (no first touch logged in the batch before) */
    uint32_t n_rounds_protected;    /* rounds run one at a time behind a state copy (they
                                       could log many first touches) */
    uint32_t n_rounds_rerun;        /* protected rounds rolled back and rerun after an
                                       ambiguous first-touch drop decision */
    uint64_t n_host_rounds;         /* (host, round) pairs in which the host executed at least
                                       one event: the host-state reads of SURVEY.md 8(d) */
    uint64_t n_batches;             /* device batches launched (shd_eng: 64 round launches
                                       each, or one persistent launch of 128 rounds;
                                       shd_xgroup: up to 64 rounds each) */
    uint64_t n_batches_persistent;  /* shd_eng batches run as one persistent launch
                                       (k_round_ps: the round grid fits the GPU;
                                       k_round_sp: more hosts, blocks of many) */
    uint64_t n_batches_sparse;      /* ... of them, sparse (k_round_sp)           */
    uint64_t n_rounds_replayed;     /* rounds run again from the last state copy to recover
                                       an unprotected round whose first-touch drop decision
                                       was ambiguous (shd_eng_run_until) */
    uint64_t n_restore_points;      /* restore points renewed between the batches of this call
                                       (a point older than 2^16 rounds) */
} shd_run_stats;

typedef struct shd_eng shd_eng;
int shd_eng_create(const shd_model* m, shd_pc* pc, int32_t host_begin, int32_t host_end,
                   int device, shd_eng** out);
/* the serial-equivalent window: min over attached pairs of ceil(lat*1e6) ns */
int shd_eng_window(shd_eng* e, uint64_t* window_ns);
/* host_boot for every local host (host.c:372-390) at t=0 */
int shd_eng_boot(shd_eng* e);
/* Events from the caller (event_new_ + scheduler_push, event.c:28-43,
 * scheduler.c:342-357): after shd_eng_boot and before the rounds reach their
 * times (time >= the end of the last round run).  Two kinds are accepted:
 *  - SHD_EV_APP_START self events (src == dst, a host of this engine): each
 *    consumes its host's next event ID on the device (the `seq` field is
 *    ignored), in array order per host -- the order process_schedule runs a
 *    host's processes at boot (host.c:372-390);
 *  - SHD_EV_PACKET deliveries from a host outside this engine (src in
 *    [0, n_hosts) but not in [host_begin, host_end); dst a host of this
 *    engine): packet ingress from hosts the caller simulates itself
 *    (worker_sendPacket's scheduler_push of the packet event for a host of
 *    another worker, worker.c:541-571).  `seq` is the sender's event ID and
 *    `pkt` its packet ID, both kept; the event merges into its host's queue
 *    by (time, src, seq) like any other.
 * Either is dropped when its time is >= end_time.  SHD_EINVAL for anything
 * else, or for a time before the engine's current simulated time. */
int shd_eng_push_events(shd_eng* e, const shd_event* ev, uint64_t n);
/* one round [window_start, window_end) on this engine; remote-bound events are
 * kept in the outbox until shd_eng_take_remote */
int shd_eng_run_round(shd_eng* e, uint64_t window_start, uint64_t window_end,
                      shd_round_summary* out);
/* whole single-engine run to end_time (rounds of W) */
int shd_eng_run(shd_eng* e, shd_run_stats* out);
/* per-path packet counters (model queue_flags & SHD_QF_COUNT_PATHS): out[a*T + b] =
 * packets this engine sent over the cached entry stored as (a, b), a and b attached
 * indices; a direct entry (complete graphs, prefer-direct adjacent pairs) and a
 * vertex's own entry are keyed (min, max).  *n = T*T; SHD_ERANGE if cap < T*T.
 * Replaces the Path.packetCount logged by _topology_logAllCachedPaths
 * (topology.c:1929-1965); engines of a group each count their own sends. */
int shd_eng_path_counts(shd_eng* e, uint64_t* out, uint64_t cap, uint64_t* n);
/* rounds while the next event time is below t_stop (rounds never cross t_stop);
 * stats cover this call only.  A whole-model engine only (host_begin 0,
 * host_end n_hosts; SHD_EINVAL otherwise): a partial engine runs rounds
 * (shd_eng_run_round) or joins a group. */
int shd_eng_run_until(shd_eng* e, uint64_t t_stop, shd_run_stats* out);
/* A round split into its phases, for drivers that own several engines (one
 * per GPU, DESIGN.md "Multi-GPU").  shd_eng_run_round = round_kernel, then,
 * if the round logged first-touch queries, pending_copy + resolve with this
 * engine's records, then end_round. */
typedef struct shd_pending {
    uint64_t qtime;                 /* key of the executing event: time, seq */
    uint64_t qseq;
    uint32_t qhost;                 /*   its destination host (the sender)   */
    uint32_t qsrc;                  /*   its source host                     */
    uint32_t qsub;                  /*   position of the query in the event  */
    uint32_t a, b;                  /* attached indices (src, dst) queried   */
    uint32_t delivered;             /* 0 dropped, 1 awaiting resolution, 2 sent */
    uint32_t dst;                   /* destination host of the packet        */
    uint32_t pkt;
    uint64_t seq;                   /* packet event seq                      */
} shd_pending;
int shd_eng_round_kernel(shd_eng* e, uint64_t window_start, uint64_t window_end,
                         shd_round_summary* out);
int shd_eng_pending_copy(shd_eng* e, shd_pending* out, uint64_t cap, uint64_t* n);
/* `all` = the pending records of EVERY engine this round (any order): row
 * ranks are assigned in serial event order, then this engine's sends are
 * finalized (delivery time from the min-rank row) */
int shd_eng_resolve(shd_eng* e, const shd_pending* all, uint64_t n_all);
int shd_eng_end_round(shd_eng* e, shd_round_summary* out);
/* One lazy path cache across a co-simulation (INTEGRATION.md "Mixed CPU/GPU
 * hosts"): shd_eng_round_begin = shd_eng_round_kernel behind a device state
 * copy while first touches may still come.  When its summary carries
 * SHD_ERR_AMBIGUOUS (a first-touch drop decision that depends on which row
 * ranks first), shd_eng_round_retry rolls the engine back to the copy, ranks
 * `all` (this round's pending records and the other side's first touches of
 * the window) in serial event order and runs the window again (then
 * end_round; nothing is left to resolve).  SHD_EAMBIG from the retry when the
 * round ran without a copy (out of device memory for it). */
int shd_eng_round_begin(shd_eng* e, uint64_t window_start, uint64_t window_end, shd_round_summary* out);
int shd_eng_round_retry(shd_eng* e, const shd_pending* all, uint64_t n_all, shd_round_summary* out);
/* The CPU side of that protocol on a path cache its lookups go through (the
 * topology adapter's, topology_shd.c): shd_pc_defer_touches takes the engine's
 * first touches of the window (shd_pending, attached indices, any order;
 * SHD_EINVAL while the last window's are not all applied); shd_pc_query_key
 * names the executing event (event_compare's key: time, host = its
 * destination, src, seq) before its lookups, which count from 0 within it;
 * shd_pc_lookup then applies every deferred touch before the query's key
 * first, and logs the query when it ranks a row or a self path;
 * shd_pc_take_touches applies the rest and returns the logged queries in
 * event order (*n = the count; copied when out != NULL and cap covers it,
 * SHD_ERANGE otherwise; then the log empties).  The pc and the engine must
 * start with the same ranks (both fresh). */
int shd_pc_defer_touches(shd_pc* pc, const shd_pending* recs, uint64_t n);
int shd_pc_query_key(shd_pc* pc, uint64_t time, uint32_t host, uint32_t src, uint64_t seq);
int shd_pc_take_touches(shd_pc* pc, shd_pending* out, uint64_t cap, uint64_t* n);
/* events this engine produced for hosts of other engines (device to device
 * copy into dev_dst, capacity cap events) and ingest of received events */
int shd_eng_remote_copy(shd_eng* e, void* dev_dst, uint64_t cap, uint64_t* n);
/* packet egress: the events the last round (shd_eng_run_round) produced for
 * hosts outside this engine -- the deliveries offloaded hosts send to hosts
 * the caller simulates -- copied to a host array of capacity cap (SHD_ERANGE
 * with *n = the count when cap is short).  The round's outbox holds them until
 * the next round starts; the caller owes them to their destination hosts
 * (worker_sendPacket, worker.c:541-571). */
int shd_eng_take_remote(shd_eng* e, shd_event* out, uint64_t cap, uint64_t* n);
int shd_eng_ingest(shd_eng* e, const void* dev_events, uint64_t n_events);
int shd_eng_next_time(shd_eng* e, uint64_t* next_time);
int shd_eng_trace_count(shd_eng* e, uint64_t* n);
int shd_eng_trace_copy(shd_eng* e, shd_trace_rec* out, uint64_t cap, uint64_t* n);
int shd_eng_digest(shd_eng* e, shd_host_digest* out);   /* [host_end-host_begin] */
int shd_eng_stream(shd_eng* e, void** hip_stream);
/* tracker node counters (model queue_flags & SHD_QF_HEARTBEATS): out[(l*K + k)*2 + j]
 * = local host l's cumulative interface packet count, j = 0 in
 * (_networkinterface_receivePacket, network_interface.c:415) / 1 out
 * (_networkinterface_sendPackets, network_interface.c:571), taken at its heartbeat
 * at (k+1)*heartbeat_interval; K = (end_time-1)/heartbeat_interval.  Each counted
 * packet is a data packet of payload + 42 header bytes, so the per-interval
 * differences give the [shadow-heartbeat] [node] line (tracker.c:419-465).
 * *n = nloc*K*2; SHD_ERANGE if cap < *n. */
int shd_eng_heartbeats(shd_eng* e, uint32_t* out, uint64_t cap, uint64_t* n);

/* ---- the reference's log lines, made by the library ----
 * A set of lines: line i is text[off[i] .. off[i+1]) (no newline; text is
 * NUL-terminated after the last line), logged at simulated time time[i] (ns)
 * by host index host[i].  Released with shd_lines_free. */
typedef struct shd_lines {
    uint64_t n;
    uint64_t* time;
    uint32_t* host;
    uint64_t* off;                  /* [n + 1] */
    char* text;
} shd_lines;
/* The [STATUS] lines of packet_addDeliveryStatus (packet.c:647-659) from a
 * trace recorded with SHD_QF_TRACE_STATUS: every status each UDP datagram
 * passes through, "[<STATUS>] packetID=<hostID>:<pkt> <srcIP>:<srcPort> ->
 * <dstIP>:<dstPort> bytes=<payload> status=<S1>,...,<Sk>" (packet_toString,
 * packet.c:518-547, 616-633), and PDS_DESTROYED where a packet object's last
 * reference goes (packet.c:194-201; not the frees at teardown).  ips[h]: host
 * h's address (host order), host_ids[h] its host_getID (NULL: h + 1),
 * listen_port the destination port; app_peer: NULL (PHOLD) or the model's
 * SHD_APP_UDP_ECHO roles -- a datagram to a client goes to the port its socket
 * was bound to (its own datagrams' source port).  Ordered by (time, host),
 * each host's lines in the reference's call-chain order. */
int shd_status_lines(const shd_trace_rec* tr, uint64_t n, const uint32_t* ips, const uint32_t* host_ids,
                     uint32_t n_hosts, uint32_t payload, uint32_t listen_port, const int32_t* app_peer,
                     shd_lines** out);
/* The [shadow-heartbeat] lines of _tracker_logNode (tracker.c:419-465) of one
 * host: the header and the all-zero boot line at t = 0 (tracker_new's inline
 * heartbeat, tracker.c:141), then one line per snapshot k at (k+1)*interval
 * from the cumulative interface counters snapshots[2k] (in), [2k+1] (out). */
int shd_node_lines(const uint32_t* snapshots, uint64_t k, uint64_t interval_ns, uint32_t payload, uint32_t host,
                   shd_lines** out);
/* The same lines from full tracker counters of each interval, [k][20]: the
 * ten remote inbound counters then the ten remote outbound ones, in the
 * counter string's order without its two totals (shdtcp.h's node_counters:
 * control / data packets, first sent and retransmitted, and their header and
 * payload bytes); the localhost counters are zero */
int shd_tracker_node_lines(const uint64_t* counters, uint64_t k, uint64_t interval_ns, uint32_t host,
                           shd_lines** out);
/* The same from an engine: the [STATUS] lines of its whole trace (the model's
 * payload; ips / host_ids over all H hosts), and local host l's [node] lines
 * (its own heartbeat interval; heartbeats before end_time). */
int shd_eng_status_lines(shd_eng* e, const uint32_t* ips, const uint32_t* host_ids, uint32_t listen_port,
                         shd_lines** out);
int shd_eng_node_lines(shd_eng* e, uint32_t local_host, shd_lines** out);
void shd_lines_free(shd_lines* l);
/* HIP-event device time of the last round kernel launch (ms) */
int shd_eng_last_kernel_ms(shd_eng* e, double* ms);
void shd_eng_destroy(shd_eng* e);

/* ---- engine groups (DESIGN.md "Multi-GPU") ----
 * One engine per rank; rank p owns hosts [(H*p)/N, (H*(p+1))/N).  Every round
 * is one fixed-size all-to-all whose per-peer blocks carry a header (the
 * sender's next event time and flags) and the events for that peer, so the
 * next window start (the min over the headers), the halt decision and the
 * delivery need no host round trip: the round loop of slave.c:413-466 /
 * master.c:148-192 across GPUs.  Rounds run in device-driven batches; a
 * round with first-touch queries, a block overflow or an error anywhere in
 * the group halts the batch on every rank alike, the host resolves it and
 * the batch resumes.  Transports: RCCL (one engine per process; the
 * multi-GPU path) or local (several engines driven by one host thread,
 * device-to-device copies). */
#define SHD_XID_BYTES 128
typedef struct shd_xgroup shd_xgroup;
/* RCCL unique id: rank 0 makes it, every rank passes the same bytes */
int shd_xgroup_unique_id(uint8_t id[SHD_XID_BYTES]);
/* Communicators of a group, one per process:
 *   rccl  one process per GPU, RCCL over xGMI (id from shd_xgroup_unique_id);
 *   host  processes of one machine meeting in a POSIX shared-memory segment
 *         named `name` (unique per group), device buffers staged through host
 *         memory: several ranks may share one GPU, which RCCL refuses.
 * A communicator serves the sharded path-cache build and an engine group. */
typedef struct shd_comm shd_comm;
int shd_comm_create_rccl(const uint8_t id[SHD_XID_BYTES], int world, int rank, int device, shd_comm** out);
int shd_comm_create_host(const char* name, int world, int rank, int device, shd_comm** out);
int shd_comm_rank(const shd_comm* c, int* rank, int* world);
void shd_comm_destroy(shd_comm* c);
/* The path cache's source rows sharded over the communicator's ranks: rank r
 * computes rows [r*R, (r+1)*R) with R = ceil(T / world), then every rank
 * all-gathers the row blocks into its full table (north_star: APSP sharded by
 * source rows).  Same tables as shd_pc_build; build_ms_* time this rank's
 * kernels, shd_pc_info.build_ms_device the whole call (exchange included). */
int shd_pc_build_sharded(shd_pc* pc, shd_comm* comm);
/* an engine group over a communicator (not owned: destroy it after the group) */
int shd_xgroup_create(shd_eng* e, shd_comm* comm, uint32_t block_events, shd_xgroup** out);
/* the same group with the peer-to-peer transport: every engine's receive
 * blocks in uncached device memory exported by IPC handle and mapped by every
 * rank; a round's blocks are stored straight into the peers' receive blocks
 * (xGMI between GPUs), header last under a tag that is never reused, and each
 * receiver's next kernel waits for every peer's tag (bounded: 30 s, then
 * SHD_ENODEV).  No collective launch per round; the communicator carries the
 * handle exchange and the host-side recovery.  The ranks' processes must be
 * able to map each other's memory (one node); all ranks fail alike if not. */
int shd_xgroup_create_p2p(shd_eng* e, shd_comm* comm, uint32_t block_events, shd_xgroup** out);
/* block_events: events per peer block per round (0 = default) */
int shd_xgroup_create_rccl(shd_eng* e, const uint8_t id[SHD_XID_BYTES], int world, int rank,
                           uint32_t block_events, shd_xgroup** out);
int shd_xgroup_create_local(shd_eng* const* engines, int n, uint32_t block_events, shd_xgroup** out);
/* boots the engines if needed, then rounds while the group's next event time
 * is below t_stop; stats: this process's engines, this call */
int shd_xgroup_run_until(shd_xgroup* g, uint64_t t_stop, shd_run_stats* out);
int shd_xgroup_next_time(shd_xgroup* g, uint64_t* next_time);
void shd_xgroup_destroy(shd_xgroup* g);

/* library */
const char* shd_version(void);
int shd_device_count(int* n);

#ifdef __cplusplus
}
#endif
#endif /* SHDGPU_H */
