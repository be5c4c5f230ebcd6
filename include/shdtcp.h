/*
 * shdtcp.h -- the TCP path on the GPU, C ABI.
 *
 * Runs the reference's TCP (host/descriptor/tcp.c, tcp_cong_reno.c,
 * tcp_retransmit_tally.cc, the socket buffers of socket.c and the interface of
 * network_interface.c) for client/server processes running the reference's own
 * TCP test application (src/test/tcp/test_tcp.c, nonblocking-epoll: connect,
 * send N bytes, read them echoed back, close) on every host of a model, in
 * conservative rounds on one GPU: one lane per host, a round is every event
 * before the window's end (the smallest path latency), deliveries cross hosts
 * through a mailbox between rounds.  Results equal the reference's serial loop
 * (tests/test_tcp_gpu.py against tests/golden/ref_tcp.json).
 *
 * The boundary is the same one shdgpu.h draws for the UDP path: plain
 * pointers and sizes, no torch types.  Path latency and reliability per host
 * pair come either from libshdgpu's path cache itself (path_cache set: the
 * lazy cache's first-touch rule applied on the device, round by round, as the
 * UDP engine does -- DESIGN.md §4), or from caller tables (Shadow's
 * topology_getLatency / topology_getReliability, topology.c:2053-2092, or
 * shd_pc_lookup), resolved in the order the serial loop touches them.
 */
#ifndef SHD_TCP_H
#define SHD_TCP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct shd_tcp_model {
    int32_t n_hosts, n_procs;
    const uint32_t* host_ip;          /* [H] host byte order (dns.c's addresses)        */
    const uint32_t* host_seed;        /* [H] host RNG state after attach                */
    const uint64_t* bw_down_kibps;    /* [H]                                            */
    const uint64_t* bw_up_kibps;      /* [H]                                            */
    int32_t n_vertices;               /* V: the attached vertices the tables index      */
    const int32_t* host_vertex;       /* [H] each host's vertex index in [0, V)         */
    const double* path_lat_ms;        /* [V*V] src_vertex*V + dst_vertex; < 0: no route
                                         (pairs no host pair uses may be left < 0)       */
    const double* path_rel;           /* [V*V]                                          */
    const int32_t* proc_host;         /* [P] the host of each process, <process> order  */
    const uint64_t* proc_start;       /* [P] start time (ns)                            */
    const int32_t* proc_peer;         /* [P] -1: server; else the server process index  */
    uint64_t end_time;                /* ns; events at or past it are never run         */
    uint64_t heartbeat_interval;      /* ns (tracker heartbeats consume event IDs)      */
    uint32_t tcp_bytes;               /* bytes each client sends (test_tcp.c BUFFERSIZE) */
    uint32_t recv_buf, send_buf;      /* initial socket buffers (CONFIG_*_BUFFER_SIZE)   */
    uint32_t tcp_window;              /* --tcp-windows (options.c:79)                    */
    uint32_t packets_per_host;        /* packet pool per host (0: 8192); more live packets
                                         set SHD_TCP_ERR_POOL                             */
    uint32_t qdisc;                   /* --interface-qdisc (options.c:162): 0 fifo, 1 rr
                                         (network_interface.c:466-517)                    */
    uint32_t _pad;
    /* A built path cache of this model's graph (shdgpu.h shd_pc_create: an
     * undirected graph, the hosts' vertices attached), or NULL.  Set: every
     * path query of the run goes to the cache's device tables under the lazy
     * cache's first-touch rule (topology.c:1969-2051): a pair with a ranked
     * endpoint at the round's start takes the lower-ranked endpoint's row; a
     * pair with none takes the querying source's row, the query logged with
     * its event key, and between rounds the log is ranked in serial order
     * (event_compare's key, then the query's index within its event), which
     * both checks every such choice and ranks the rows that ran.  A choice the
     * serial order contradicts (two unranked endpoints first touched from both
     * sides within one window) ends the run with SHD_TCP_ERR_FIRST_TOUCH; the
     * caller then runs the model on tables (the fields above).  The cache's
     * ranks are left as the serial run leaves them.  host_vertex then holds
     * graph vertex ids, and n_vertices / path_lat_ms / path_rel are unused. */
    struct shd_pc* path_cache;
    /* Datagram processes beside the echo ones: both transports in one model,
     * on each host's one interface (qdisc, token buckets, CoDel queue) --
     * network_interface.c:519-579 serves TCP and UDP sockets alike.
     * proc_app[k] >= 0: process k runs the datagram application
     * app_spec[4 * proc_app[k] ..] = shd_udp_app's {send, dest, n_start,
     * per_read} (shdgpu.h; PHOLD's port 8998) instead of the echo, with
     * proc_peer[k] = -1; at most one such process per host.  NULL proc_app:
     * every process runs the echo.  udp_payload: bytes per datagram (1 ..
     * 65507); app_peer [H]: the SHD_DEST_PEER host of each host; dest_cum
     * [n_classes][H] / host_class [H]: SHD_DEST_WEIGHTED's cumulative weights
     * (host_class NULL: row 0).  A host then holds up to 16 sockets at once
     * (8 otherwise): more set SHD_TCP_ERR_SOCKETS. */
    const int32_t* proc_app;
    const uint32_t* app_spec;
    int32_t n_app_specs;
    uint32_t udp_payload;
    const int32_t* app_peer;
    const double* dest_cum;
    const uint8_t* host_class;
    int32_t n_classes, _pad2;
} shd_tcp_model;

/* the first path query a host made of a vertex pair (topology_isRoutable /
 * getLatency / getReliability): the executing event's key (event_compare:
 * time, host, src, seq) and the query's index within that event; the caller
 * ranks the run's first touches in this order (shadow-1_amd/tcp.py) */
typedef struct shd_tcp_query {
    uint64_t time, seq;
    uint32_t host, src, index;
    int32_t v_src, v_dst;             /* vertex indices (path table) of the query       */
    uint32_t _pad;
} shd_tcp_query;

typedef struct shd_tcp_result {
    char* lines;                      /* "<time>\t<host>\t[STATUS] ...\n", each host's lines in
                                         its execution order, hosts in index order           */
    size_t len;
    uint64_t n_lines;
    uint64_t* next_event_id;          /* [H] host event counter at the end                */
    uint64_t* next_packet_id;         /* [H]                                              */
    uint32_t* rng_probe;              /* [H] the next rand_r value of each host RNG       */
    uint64_t rounds;                  /* conservative rounds run                          */
    uint64_t events;                  /* events executed                                  */
    double device_ms;                 /* GPU time of the rounds (HIP events)              */
    uint32_t error;                   /* SHD_TCP_ERR_* bits; nonzero: results invalid     */
    uint64_t deliveries;              /* packets handed to a receiving host (worker.c:260-321's
                                         delivery events executed)                           */
    shd_tcp_query* queries;           /* each host's first query of each vertex pair      */
    uint64_t n_queries;
    /* with SHD_TCP_TRACE_NODE: the tracker's node counters of every heartbeat
     * interval (tracker.c:183-214, 566-611), [H][node_k][20]: inbound remote
     * then outbound remote, each packets-control, bytes-control-header,
     * packets-control-retrans, bytes-control-header-retrans, packets-data,
     * bytes-data-header, bytes-data-payload, packets-data-retrans,
     * bytes-data-header-retrans, bytes-data-payload-retrans; a host's packets
     * to its own address (the loopback task, network_interface.c:548-555) are
     * counted here as the reference counts them: remote, since tracker.c:223
     * and :255 call a packet local only when its address is 127.0.0.1, which
     * no model's sockets use, so the localhost counters are zero.
     * n_heartbeats[h] of them are host h's.
     * shd_tracker_node_lines (shdgpu.h) makes the [node] lines of a host. */
    uint64_t* node_counters;
    uint32_t* n_heartbeats;
    uint32_t node_k;
    uint32_t first_touch_reruns;      /* path_cache mode: runs this call made again from the start,
                                         each with one more round's first touches ranked in
                                         serial order before it runs (a contradicted device
                                         choice that changed a value) */
    uint64_t max_round_deliveries;    /* the most deliveries one round's mailbox took */
    uint64_t max_round_overflow;      /* ... and the most of them in its shared overflow range */
    double setup_ms, results_ms, teardown_ms;   /* the call's host wall time around the rounds:
                                                   allocation and upload, copies back and
                                                   formatting, release */
    /* the hosts this result covers: [first_host, first_host + n_local_hosts)
     * (shd_tcp_run: all of them; shd_tcp_run_group: this engine's share) --
     * the per-host arrays above (next_event_id, next_packet_id, rng_probe,
     * node_counters, n_heartbeats) and the lines are these hosts'; the lines
     * carry the model's host index.  queries: every engine's. */
    int32_t first_host, n_local_hosts;
} shd_tcp_result;

/* shd_tcp_run's `trace` bits */
enum { SHD_TCP_TRACE_STATUS = 1, SHD_TCP_TRACE_NODE = 2 };

enum {
    SHD_TCP_ERR_EVQ = 1, SHD_TCP_ERR_POOL = 2, SHD_TCP_ERR_QUEUE = 4, SHD_TCP_ERR_SOCKETS = 8,
    SHD_TCP_ERR_MAILBOX = 16, SHD_TCP_ERR_TRACE = 32, SHD_TCP_ERR_SACK = 64, SHD_TCP_ERR_INTERNAL = 128,
    SHD_TCP_ERR_QLOG = 256, SHD_TCP_ERR_FIRST_TOUCH = 512
};

/* Run the model to end_time on the current HIP device (the reference's
 * src/main/core/worker.c loop for these processes; see the file comment).  trace & 1 writes the
 * [STATUS] lines (packet.c:647-659); trace & 2 keeps the tracker's node
 * counters per heartbeat (the [node] lines, tracker.c:419-465).  Returns 0 or a negative errno-style code:
 * -22 an invalid model, -113 a client whose server has no route in either
 * direction (the reference's connect fails with ECONNREFUSED there,
 * host.c:1224-1234; the device application has no such branch), -12 no device
 * memory for the trace buffers, -5 a HIP error.  A client on another host than
 * its server that starts less than one window W (the smallest path latency)
 * after it is refused (-22): it could connect in the round its server binds,
 * and the port it reads would depend on the lanes' timing.  *out is allocated by the call
 * and released by shd_tcp_result_free. */
int shd_tcp_run(const shd_tcp_model* m, int32_t trace, shd_tcp_result** out);
void shd_tcp_result_free(shd_tcp_result* r);

/* The same model on a group of engines, one per process and GPU (shdgpu.h
 * shd_comm: RCCL, or the host-memory transport for several processes on one
 * GPU), every rank calling with the same model: rank r runs hosts
 * [r * H / world, (r + 1) * H / world) -- the reference's rounds across
 * workers (slave.c:437-462) with its hosts' events, both transports, the
 * qdisc, buckets and CoDel queue on the engine that owns the host.  Each
 * round's window starts at the earliest pending event over the group (an
 * all-gather of a few words per engine); after the round the deliveries for
 * other engines' hosts go to them: every engine writes them into one segment
 * per destination engine (SHD_TCP_XCAP deliveries per engine pair and round,
 * max(16384, 8 x the engine's hosts) by default; more set
 * SHD_TCP_ERR_MAILBOX), the segments' counts go round in one all-gather and
 * only their used parts in an all-to-all-v (grouped send / receive on RCCL),
 * and the servers' listening ports their clients connect to are published to
 * every engine.  Results equal shd_tcp_run's on the same model, host by host
 * (a client on another host than its server must start at least one window
 * after it, or the model is refused with -22, as on one engine).  Paths: with path_cache (every rank's own
 * cache of the same graph, built alike) each round's first-touch log of every
 * engine is gathered and replayed alike on every rank, so the ranks stay
 * equal and a contradicted choice stops every rank at the same round
 * (SHD_TCP_ERR_FIRST_TOUCH); with tables the queries every engine logged come
 * back in each rank's result, for the caller's ranking as on one engine.
 * Returns as shd_tcp_run, -5 also when the group's communication fails.
 * Failure is collective only where every rank sees it: an error bit of the
 * run, a halted engine (every engine ends at that round) and a first-touch
 * log too long for the device end every rank at the same round; a HIP error
 * local to one rank ends that rank's call, and the others stay in their next
 * collective until the transport gives up (the host transport after its
 * 300-s barrier timeout; RCCL does not time out). */
struct shd_comm;
int shd_tcp_run_group(const shd_tcp_model* m, struct shd_comm* comm, int32_t trace, shd_tcp_result** out);

/* keep != 0: shd_tcp_run keeps its device buffers (the per-host event queues,
 * packet pools, sockets and mailboxes: tens of GB at 64 k hosts) for the next
 * call on the same device instead of allocating and freeing them each call;
 * 0 (the default): release them now and after every call.  A caller that runs
 * many models in one process (a parameter sweep, the bench) sets 1. */
void shd_tcp_keep_workspace(int32_t keep);

#ifdef __cplusplus
}
#endif
#endif
