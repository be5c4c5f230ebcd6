/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference (Shadow 1.14, joskid/shadow-1)
 * algorithms on the accelerated path.  It is the parity checker for libshdgpu:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it, and never as the thing measured or shipped.  The product path
 * (shadow-1_amd/) does not link, include or call anything under oracle/.
 *
 * Every function cites the reference file:line it restates.  Pinning status:
 *  - RNG, priority-queue order, CoDel: pinned against the reference's own
 *    random.c / priority_queue.c / router_queue_codel.c compiled into
 *    oracle/_ref (tests/test_oracle_ref.py).
 *  - Path cache: distances/paths pinned against networkx 3.4.2 Dijkstra on
 *    tie-free graphs (tests/golden/make_pathcache_golden.py); the igraph 0.7.1
 *    Dijkstra itself is absent from the image (not vendored, not installed), so
 *    its TIE-BREAKING is restated from its published algorithm and is
 *    "parity unpinned" ("Oracle").
 *  - Event loop: restated from worker.c / event.c / scheduler.c /
 *    network_interface.c / router.c / tracker.c.  Pinned as a whole to the
 *    reference's OWN serial loop: worker.c, scheduler.c, host.c,
 *    network_interface.c, router*.c, descriptor/ (all), tracker.c, packet.c ...
 *    compiled unmodified into oracle/_ref/libshdref_loop.so, with test doubles
 *    only for what the image cannot build (slave.c, the igraph topology --
 *    served by this oracle's lazy path cache --, the rpth process layer, the
 *    loggers; oracle/ref_harness/ref_loop.c).  Every [STATUS] and [node] line,
 *    event-ID and packet counter and RNG state of eight models (lossy, CoDel,
 *    loopback, per-host heartbeats, pushed multi-process starts, bootstrap,
 *    the Tor-scale classes, C1) equals the reference's
 *    (tests/golden/ref_loop.json, tests/test_ref_loop_cpu.py).
 */
#ifndef SHD_ORACLE_H
#define SHD_ORACLE_H

#include <stdint.h>
#include "../include/shdgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- RNG (utility/random.c:32-51 over glibc rand_r) ---- */
int32_t o_rand_r(uint32_t* state);
double o_next_double(uint32_t* state);
uint32_t o_next_uint(uint32_t* state);
int o_seed_chain(uint32_t options_seed, int32_t n_hosts, uint32_t* host_seeds);

/* ---- igraph-0.7.1-shaped graph (type_indexededgelist.c as published) ---- */
typedef struct o_graph {
    int32_t V, E, directed;
    int32_t* from;   /* undirected: max(a,b); directed: a */
    int32_t* to;     /* undirected: min(a,b); directed: b */
    double* w;       /* latency */
    double* eloss;
    double* vloss;   /* NULL or [V] with NaN = absent */
    int32_t* oi;     /* edge ids sorted by (from,to,eid) */
    int32_t* ii;     /* edge ids sorted by (to,from,eid) */
    int32_t* os;     /* [V+1] */
    int32_t* is;     /* [V+1] */
    int32_t prefer_direct;
} o_graph;

o_graph* o_graph_new(const shd_graph* g);
void o_graph_free(o_graph* g);
/* igraph_incident(graph, v, IGRAPH_OUT) order; returns count, fills eids (cap) */
int32_t o_incident(const o_graph* g, int32_t v, int32_t* eids, int32_t cap);
int32_t o_incident_count(const o_graph* g, int32_t v);
/* igraph_get_eid(from,to,directedness,error=false): -1 if none (lowest eid) */
int32_t o_get_eid(const o_graph* g, int32_t a, int32_t b);
int o_graph_props(const o_graph* g, shd_graph_props* out);

/* ---- path cache primitives ---- */
/* _topology_lookupDirectPath (topology.c:1877-1927) */
int o_direct_path(const o_graph* g, int32_t s, int32_t d, double* lat, double* rel);
/* _topology_computeShortestPathToSelf (topology.c:1545-1653) */
int o_self_path(const o_graph* g, int32_t s, double* lat, double* rel);
/* one Dijkstra row (topology.c:1655-1875 with igraph 0.7.1 Dijkstra):
 * lat/rel per target; ok[j]=0 when computePathProperties fails (no edge);
 * hops[j] = path edge count; ties (out) = #vertices with a non-unique parent */
int o_sssp_row(const o_graph* g, int32_t src, const int32_t* targets, int32_t nt,
               double* lat, double* rel, int32_t* ok, int32_t* hops, int64_t* ties);

/* ---- lazy path cache with the reference's semantics ---- */
typedef struct o_topo o_topo;
o_topo* o_topo_new(const o_graph* g, const int32_t* attached, int32_t n_attached,
                   int32_t force_rows);
void o_topo_free(o_topo* t);
/* precomputed rows by vertex ([V] pointers, NaN latency = no path) */
void o_topo_set_row_cache(o_topo* t, double** row_lat, double** row_rel);
/* every attached vertex's row on `threads` cores, owned by the cache */
void o_topo_precompute_rows(o_topo* t, int threads);
int32_t o_topo_n_targets(const o_topo* t);
const int32_t* o_topo_targets(const o_topo* t);
int o_topo_is_complete(const o_topo* t);
/* read-only: 1 and the value when the pair has an entry in either orientation */
int o_topo_peek(const o_topo* t, int32_t s, int32_t d, double* lat, double* rel);
o_topo* o_topo_clone(const o_topo* t);
/* 1 when _topology_getPathEntry(s, d) would run a source row or a self path
 * now (no entry to serve it, not a direct-path pair): a first touch */
int o_topo_would_run(const o_topo* t, int32_t s, int32_t d);
/* _topology_getPathEntry(s, d) for its effect on the cache only */
void o_topo_touch(o_topo* t, int32_t s, int32_t d);
/* _topology_getPathEntry (topology.c:1969-2051) -> path latency/reliability;
 * returns 0 and -1/-1 when the reference returns NULL */
int o_topo_get(o_topo* t, int32_t s, int32_t d, double* lat, double* rel);
void o_topo_count_packet(o_topo* t, int32_t s, int32_t d);
uint64_t o_topo_packet_count(o_topo* t, int32_t s, int32_t d);
/* the count of the entry stored as (s, d) only (no orientation fallback) */
uint64_t o_topo_stored_count(o_topo* t, int32_t s, int32_t d);
/* o_engine_run fills counts[s*V + d] = o_topo_stored_count at the end of the run */
void o_engine_set_counts_out(uint64_t* counts, int32_t n_vertices);
double o_topo_min_latency(o_topo* t);
int32_t o_topo_rows_run(o_topo* t);
int32_t o_topo_self_run(o_topo* t);

/* ---- CoDel (routing/router_queue_codel.c) ---- */
typedef struct o_codel_entry { uint64_t ts; uint32_t len; uint32_t id; uint32_t src; uint32_t _pad; } o_codel_entry;
typedef struct o_codel {
    o_codel_entry* q; uint32_t cap, head, count;
    uint64_t total;
    uint32_t mode;                 /* 0 store, 1 drop */
    uint64_t interval_expire;
    uint64_t next_drop;
    uint32_t drop_count, drop_count_last;
} o_codel;
void o_codel_init(o_codel* c, uint32_t cap);
void o_codel_free(o_codel* c);
int o_codel_enqueue(o_codel* c, uint64_t now, uint32_t len, uint32_t id, uint32_t src);
/* returns 1 and fills *out when a packet is dequeued; dropped entries are
 * appended to drops (cap ndrops_cap) */
int o_codel_dequeue(o_codel* c, uint64_t now, o_codel_entry* out, o_codel_entry* drops,
                    uint32_t ndrops_cap, uint32_t* ndrops);
uint64_t o_codel_control_law(uint32_t count, uint64_t ts);

/* ---- serial event loop for the PHOLD-UDP model ---- */
typedef struct o_run {
    shd_trace_rec* trace; uint64_t n_trace, cap_trace;
    shd_host_digest* digest;   /* [H] */
    uint64_t n_events, n_pkt_events;
    uint64_t window_ns;        /* min ceil(lat*1e6) over attached pairs (for info) */
    int32_t rows_run, self_run;
    double wall_ms;
    /* state when simulated time first reached the mark (o_engine_set_mark) */
    uint64_t mark_events, mark_pkt_events;
    double mark_wall_ms;
} o_run;
/* events pushed by the caller after boot (shd_eng_push_events semantics) */
void o_engine_set_pushes(const shd_event* ev, uint64_t n);
/* steady-state timing: record counters/wall time when sim time reaches t */
void o_engine_set_mark(uint64_t t);
/* serial mode (--workers 0): one global queue ordered by event_compare,
 * one round to end_time (slave.c:415-428) */
int o_engine_run(const shd_model* m, const shd_graph* g, int32_t force_rows, o_run* out);
void o_run_free(o_run* r);

/* ---- engine state: the serial loop in steps, parallel rounds, clones ---- */
typedef struct o_state o_state;
typedef struct o_par_stats {
    uint64_t rounds, n_events, n_pkt_events, first_touch_sends, ambiguous, window_ns;
    double wall_ms;
    int32_t threads, _pad;
} o_par_stats;
o_state* o_state_new(const shd_model* m, const shd_graph* g, int32_t force_rows);
/* precompute every attached vertex's source row on `threads` cores */
void o_state_rows(o_state* s, int threads);
/* the serial loop (one global queue) while the next event is before t_until */
void o_state_run_serial(o_state* s, uint64_t t_until);
/* the same window in parallel rounds of W (W <= every path latency, so the
 * result is the serial run's): hosts in chunks over `threads` cores, each host
 * its own queue (scheduler_policy_host_steal.c:227-431 without the clamp);
 * first touches of a round resolved at its end in serial order.  -1 for
 * directed graphs or a traced model. */
int o_state_run_parallel(o_state* s, uint64_t t_until, int threads, o_par_stats* st);
o_state* o_state_clone(const o_state* s);
void o_state_digest(const o_state* s, shd_host_digest* out);   /* [H] */
const o_run* o_state_stats(const o_state* s);
/* co-simulation (packet ingress/egress at the boundary, shd_eng_push_events /
 * shd_eng_take_remote): a state of the hosts [h_lo, h_hi) only; sends to
 * other hosts leave by o_state_take_egress, the other side's packets for hosts
 * here come in by o_state_inject; o_state_run_serial runs the windows */
o_state* o_state_new_part(const shd_model* m, const shd_graph* g, int32_t h_lo, int32_t h_hi);
int o_state_inject(o_state* s, const shd_event* ev, uint64_t n);
int o_state_take_egress(o_state* s, shd_event* out, uint64_t cap, uint64_t* n);
uint64_t o_state_next_time(const o_state* s);
/* one lazy path cache across the sides (round 4): before a window, the other
 * side's first touches of that window (shd_pending records, attached indices,
 * any order) -- each is applied to this side's cache just before the first
 * query of this side that comes after it in event order; after the window,
 * o_state_take_touches applies the rest and returns this side's own first
 * touches of the window (o_topo_would_run at the query) as shd_pending
 * records, in event order: *n = the count, copied when out != NULL and cap
 * covers it (then the list empties) */
int o_state_defer_touches(o_state* s, const shd_pending* recs, uint64_t n);
int o_state_take_touches(o_state* s, shd_pending* out, uint64_t cap, uint64_t* n);
int o_state_trace(const o_state* s, shd_trace_rec* out, uint64_t cap, uint64_t* n);
void o_state_free(o_state* s);

/* the bench's CPU baseline (bench.py cpu_baseline): warm up to t_mark, then
 * time [t_mark, t_end) serially on one core and in parallel rounds on
 * `threads` cores from the same state; same_end_state = 1 when both end
 * states are equal bit for bit */
typedef struct o_baseline_out {
    double rows_ms, warmup_ms, serial_ms, parallel_ms;
    uint64_t serial_events, serial_pkt_events, parallel_events, parallel_pkt_events;
    uint64_t parallel_rounds, parallel_first_touch, ambiguous, window_ns;
    int32_t threads, same_end_state;
} o_baseline_out;
int o_baseline(const shd_model* m, const shd_graph* g, uint64_t t_mark, uint64_t t_end, int threads,
               o_baseline_out* out);

/* ---- reference priority order (event.c:110-153) as a checker ---- */
int o_event_compare(const shd_event* a, const shd_event* b);

/* ---- the TCP path (o_tcp.c): the echo test of src/test/tcp/test_tcp.c on the
 * serial loop, writing packet.c's [STATUS] lines ("<time>\t<host>\t<line>\n";
 * host -1: a delivery's copy released after its task) ---- */
typedef struct o_tcp_cfg {
    int32_t n_hosts, n_procs;
    const uint32_t* host_ip;          /* [H] host byte order (the DNS's) */
    const uint32_t* host_seed;        /* [H] host RNG state after attach */
    const int32_t* host_vertex;       /* [H] */
    const uint64_t* bw_down_kibps, *bw_up_kibps;   /* [H] */
    const int32_t* proc_host;         /* [P] */
    const uint64_t* proc_start;       /* [P] */
    const int32_t* proc_peer;         /* [P] -1 server, else the server process */
    uint64_t end_time, heartbeat_interval;
    uint32_t tcp_bytes, recv_buf, send_buf, tcp_window;
    uint32_t no_lines;                /* 1: keep the statuses, write no lines (bench.py's CPU baseline) */
    uint32_t qdisc_rr;                /* 1: the round-robin qdisc (network_interface.c:466-490) */
    /* datagram processes beside the echo ones (shdtcp.h's shd_tcp_model fields) */
    const int32_t* proc_app;          /* [P] -1 echo, else the application's index; NULL: none */
    const uint32_t* app_spec;         /* [n][4] {send, dest, n_start, per_read} */
    uint32_t udp_payload, _pad;
    const int32_t* app_peer;          /* [H] */
    const double* dest_cum;           /* [n_classes][H] */
    const uint8_t* host_class;        /* [H] or NULL */
    int32_t n_classes, _pad2;
} o_tcp_cfg;
typedef struct o_tcp_out {
    char* lines; size_t len; uint64_t n_lines;
    uint64_t* next_event_id; uint64_t* next_packet_id; uint32_t* rng_probe;
    uint64_t events;                  /* events executed */
} o_tcp_out;
int o_tcp_run(const o_tcp_cfg* cfg, o_topo* topo, o_tcp_out* out);
void o_tcp_free(o_tcp_out* out);

#ifdef __cplusplus
}

#endif
#endif
