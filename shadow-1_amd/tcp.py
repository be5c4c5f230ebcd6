"""Host driver of the TCP path on the GPU (include/shdtcp.h, csrc/tcp.hip).

Mirrors what a Shadow build would do around shd_tcp_run: the hosts' addresses
and RNG states come from the config front-end (dns.c's addresses, the seed
chain after attach), and the path latency / reliability of every host pair
comes from the product's lazy path cache (topology.c:2053-2092).

Which endpoint's Dijkstra row serves a pair depends on the serial order of
every pair's FIRST query (_topology_getPathEntry, topology.c:1969-2051).  By
default (mode "device") the run takes the cache itself (shd_tcp_model.
path_cache): the device applies the first-touch rule round by round -- pairs
with a ranked endpoint at a round's start decided, the others decided by the
querying lane and logged, the log ranked in serial order between rounds
(k_tcp_window) -- so one run, with no first-touch guess on the host.  A round
whose lanes touched the same unranked vertices from both sides in a way the
serial order contradicts ends the run with SHD_TCP_ERR_FIRST_TOUCH; the
driver then takes the table path below.

The table path (mode "tables", and the fallback): the tables passed to
shd_tcp_run are resolved in a first-touch order (one shd_pc_lookup_batch call),
and the run logs each host's first query of each vertex pair with its event
key (shd_tcp_result.queries).  The driver ranks the logged queries in serial
order (time, host, src, seq, index within the event), replays them through a
fresh lazy cache and compares the values every logged pair gets with the ones
the run used: equal, the run's order of first touches IS the serial one (the
run is a deterministic function of the values, so the serial loop with these
values makes the same queries in the same order); otherwise the run is
repeated with the new tables, until they agree (first_touch_runs in the
result).  The first guess is a client's connect touching (client, server)
first (topology_isRoutable, host.c:1224-1234), clients by start time.
"""
from __future__ import annotations

import ctypes as C

import time

import numpy as np

import shdgpu as S
import sim

RECV_BUF = 174760   # CONFIG_RECV_BUFFER_SIZE (definitions.h:159)
SEND_BUF = 131072   # CONFIG_SEND_BUFFER_SIZE (definitions.h:153)
TCP_WINDOW = 10     # --tcp-windows default (options.c:79)


def resolve(g: S.GraphArrays, att, first_queries, pairs, V):
    """[V, V] latency / reliability tables from a fresh lazy path cache whose
    first touches are `first_queries` [(s, d)] in that order (vertex indices);
    then both orientations of every pair in `pairs` (cache hits: their rows
    have run).  Pairs not listed stay -1."""
    lat = np.full((V, V), -1.0)
    rel = np.full((V, V), -1.0)
    fq = np.asarray(first_queries, dtype=np.int64).reshape(-1, 2)
    pq = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
    both = np.stack([pq, pq[:, ::-1]], axis=1).reshape(-1, 2)   # each pair, then its reverse, after the first touches
    q = np.concatenate([fq, both])
    pc = sim.PathCache(g, att)
    try:
        # one shd_pc_lookup_batch call: the queries in order, one device round trip
        lq, rq = pc.lookup_batch(att[q[:, 0]], att[q[:, 1]]) if len(q) else (np.zeros(0), np.zeros(0))
    finally:
        pc.close()
    k = len(fq)
    lat[both[:, 0], both[:, 1]] = lq[k:]
    rel[both[:, 0], both[:, 1]] = rq[k:]
    return lat, rel


def path_table(model: S.ModelArrays, g: S.GraphArrays, procs, peers, reverse=False, all_pairs=False):
    """Latency (ms) and reliability per pair of attached vertices ([V, V],
    V = the distinct vertices the hosts sit on) from the path cache, pairs
    resolved in the first guess of the first-touch order (clients by start
    time, each touching (client, server) first); pairs no connection uses stay
    -1 (all_pairs: every pair is filled, for datagrams that may go anywhere);
    reverse: the clients in reverse order (a wrong guess, for tests).
    Returns (lat, rel, host -> vertex index, attached vertices)."""
    m = model.struct
    H = int(m.n_hosts)
    hv = np.ctypeslib.as_array(m.host_vertex, shape=(H,)).copy()
    att, hvi = np.unique(hv, return_inverse=True)
    order = sorted(((p[1], k) for k, p in enumerate(procs) if peers[k] >= 0), reverse=reverse)
    q = [(hvi[procs[k][0]], hvi[procs[peers[k]][0]]) for _, k in order]
    V = len(att)
    pairs = q + [(a, b) for a in range(V) for b in range(a, V)] if all_pairs else q
    lat, rel = resolve(g, att, q, pairs, V)
    return lat, rel, hvi.astype(np.int32), att


def serial_first_queries(queries: np.ndarray):
    """The logged first queries in serial order (event_compare's key, then the
    query's index within the event): [(s, d)] vertex pairs, and the distinct
    unordered pairs"""
    q = queries[np.lexsort((queries["index"], queries["seq"], queries["src"], queries["host"], queries["time"]))]
    order = [(int(a), int(b)) for a, b in zip(q["v_src"], q["v_dst"])]
    pairs = sorted({(min(a, b), max(a, b)) for a, b in order})
    return order, pairs


def run(model: S.ModelArrays, g: S.GraphArrays, ips, procs, peers, nbytes=20000, trace=True,
        recv_buf=RECV_BUF, send_buf=SEND_BUF, tcp_window=TCP_WINDOW, packets_per_host=0, guess_reversed=False,
        node=False, qdisc=0, mode="device", udp=None, comm=None):
    """Run the TCP echo model on the GPU: procs = [(host, start ns)], peers =
    [-1 | server process]; ips: host-order uint32 per host.  Returns
    dict(lines=[(t, h, line)] in each host's order, next_event_id,
    next_packet_id, rng_probe, rounds, events, device_ms, first_touch
    ("device", or "tables" with first_touch_runs); with node:
    node_lines=[(t, h, line)], every host's tracker [node] lines by (time,
    host), from the library's writer).
    mode "device": the path cache's first-touch rule on the device (falls back
    to "tables" when a round's choice is contradicted, or on a directed graph);
    guess_reversed: the table path from a wrong first-touch guess (tests).
    udp: dict(apps=[-1 | spec index per process], specs=[(send, dest,
    n_start, per_read)], app_peer=[H], payload=bytes) -- the processes with
    an index run that datagram application (shd_tcp_model.proc_app) instead
    of the echo; the model's dest_cum / host_class give SHD_DEST_WEIGHTED's
    weights.
    comm (sim.Comm): this rank's share of a group run (shd_tcp_run_group: every
    rank calls with the same model; the result covers hosts [first_host,
    first_host + n_local_hosts), the lines carry the model's host index); every
    rank's first touches are ranked together, on the device (each round's logs
    gathered) or over the tables' query logs."""
    if mode == "device" and not guess_reversed and not g.directed:
        m = model.struct
        H = int(m.n_hosts)
        hv = np.ctypeslib.as_array(m.host_vertex, shape=(H,)).copy()
        t_pc = time.perf_counter()
        pc = sim.PathCache(g, np.unique(hv))
        pc_ms = (time.perf_counter() - t_pc) * 1e3
        try:
            out = _run_once(model, ips, procs, peers, None, None, hv.astype(np.int32), nbytes, trace, recv_buf,
                            send_buf, tcp_window, packets_per_host, node, qdisc, pc=pc, udp=udp, comm=comm)
        finally:
            pc.close()
        if out is not None:
            out.pop("queries")
            out["first_touch"] = "device"
            out["host_ms"]["path_cache"] = pc_ms
            return out
    lat, rel, hvi, att = path_table(model, g, procs, peers, reverse=guess_reversed, all_pairs=udp is not None)
    V = lat.shape[0]
    for runs in range(1, 9):
        out = _run_once(model, ips, procs, peers, lat, rel, hvi, nbytes, trace, recv_buf, send_buf, tcp_window,
                        packets_per_host, node, qdisc, udp=udp, comm=comm)
        order, pairs = serial_first_queries(out.pop("queries"))
        lat2, rel2 = resolve(g, att, order, pairs, V)
        ij = tuple(np.array([(a, b) for a, b in pairs] + [(b, a) for a, b in pairs], dtype=np.int64).T) \
            if pairs else (np.zeros(0, np.int64), np.zeros(0, np.int64))
        same = np.array_equal(lat[ij].view(np.uint64), lat2[ij].view(np.uint64)) and \
            np.array_equal(rel[ij].view(np.uint64), rel2[ij].view(np.uint64))
        if same:
            out["first_touch"] = "tables"
            out["first_touch_runs"] = runs
            out["first_touch_pairs"] = len(pairs)
            out["first_touch_order"] = [(int(att[a]), int(att[b])) for a, b in order]   # graph vertices
            return out
        # the serial order of this run's first touches: run again on it
        lat, rel = lat.copy(), rel.copy()
        lat[ij], rel[ij] = lat2[ij], rel2[ij]
    raise S.ShdError("shd_tcp_run: the first-touch order did not settle in 8 runs")


def _run_once(model, ips, procs, peers, lat, rel, hvi, nbytes, trace, recv_buf, send_buf, tcp_window,
              packets_per_host, node=False, qdisc=0, pc=None, udp=None, comm=None):
    """one shd_tcp_run on the given path tables, or with pc (sim.PathCache) on
    the cache itself (hvi: graph vertices then); None when that run's
    first-touch choices were contradicted (SHD_TCP_ERR_FIRST_TOUCH)"""
    m = model.struct
    H = int(m.n_hosts)
    keep = dict(ip=np.ascontiguousarray(ips, dtype=np.uint32), hv=np.ascontiguousarray(hvi, dtype=np.int32),
                lat=np.ascontiguousarray(lat if lat is not None else np.zeros((1, 1))),
                rel=np.ascontiguousarray(rel if rel is not None else np.zeros((1, 1))),
                ph=np.ascontiguousarray([p[0] for p in procs], dtype=np.int32),
                ps=np.ascontiguousarray([p[1] for p in procs], dtype=np.uint64),
                pp=np.ascontiguousarray(peers, dtype=np.int32))
    tm = S.TcpModel()
    tm.n_hosts = H
    tm.n_procs = len(procs)
    tm.host_ip = S.as_ptr(keep["ip"], C.c_uint32)
    tm.host_seed = m.host_rng
    tm.bw_down_kibps = m.bw_down_kibps
    tm.bw_up_kibps = m.bw_up_kibps
    tm.n_vertices = lat.shape[0] if lat is not None else 0
    tm.host_vertex = S.as_ptr(keep["hv"], C.c_int32)
    tm.path_lat_ms = S.as_ptr(keep["lat"], C.c_double)
    tm.path_rel = S.as_ptr(keep["rel"], C.c_double)
    tm.proc_host = S.as_ptr(keep["ph"], C.c_int32)
    tm.proc_start = S.as_ptr(keep["ps"], C.c_uint64)
    tm.proc_peer = S.as_ptr(keep["pp"], C.c_int32)
    tm.end_time = m.end_time
    tm.heartbeat_interval = m.heartbeat_interval
    tm.tcp_bytes = nbytes
    tm.recv_buf = recv_buf
    tm.send_buf = send_buf
    tm.tcp_window = tcp_window
    tm.packets_per_host = packets_per_host
    tm.qdisc = int(qdisc)   # --interface-qdisc: 0 fifo, 1 rr
    if pc is not None:
        tm.path_cache = pc.ptr.value
    if udp is not None:
        keep["pa"] = np.ascontiguousarray(udp["apps"], dtype=np.int32)
        keep["sp"] = np.ascontiguousarray([[int(x) for x in a] for a in udp["specs"]], dtype=np.uint32).ravel()
        keep["ap"] = np.ascontiguousarray(udp.get("app_peer", [-1] * H), dtype=np.int32)
        tm.proc_app = S.as_ptr(keep["pa"], C.c_int32)
        tm.app_spec = S.as_ptr(keep["sp"], C.c_uint32)
        tm.n_app_specs = len(udp["specs"])
        tm.udp_payload = int(udp.get("payload", m.payload or 1))
        tm.app_peer = S.as_ptr(keep["ap"], C.c_int32)
        tm.dest_cum = m.dest_cum
        tm.host_class = m.host_class
        tm.n_classes = m.n_classes
    res = C.POINTER(S.TcpResult)()
    bits = (S.TCP_TRACE_STATUS if trace else 0) | (S.TCP_TRACE_NODE if node else 0)
    if comm is not None:
        S.check(S.lib().shd_tcp_run_group(C.byref(tm), comm.ptr, bits, C.byref(res)), "shd_tcp_run_group")
    else:
        S.check(S.lib().shd_tcp_run(C.byref(tm), bits, C.byref(res)), "shd_tcp_run")
    try:
        r = res.contents
        h0, HL = int(r.first_host), int(r.n_local_hosts)
        if pc is not None and r.error == S.TCP_ERR_FIRST_TOUCH:
            return None
        if r.error:
            raise S.ShdError(f"shd_tcp_run: error bits {r.error:#x}")
        text = C.string_at(r.lines, r.len).decode() if r.len else ""
        lines = []
        for ln in text.splitlines():
            t, h, body = ln.split("\t", 2)
            lines.append((int(t), int(h), body))
        out = dict(lines=lines, first_host=h0, n_local_hosts=HL,
                   next_event_id=np.ctypeslib.as_array(r.next_event_id, shape=(HL,)).copy(),
                   next_packet_id=np.ctypeslib.as_array(r.next_packet_id, shape=(HL,)).copy(),
                   rng_probe=np.ctypeslib.as_array(r.rng_probe, shape=(HL,)).copy(),
                   rounds=int(r.rounds), events=int(r.events), deliveries=int(r.deliveries),
                   max_round_deliveries=int(r.max_round_deliveries), max_round_overflow=int(r.max_round_overflow),
                   host_ms=dict(setup=float(r.setup_ms), results=float(r.results_ms), teardown=float(r.teardown_ms)),
                   first_touch_reruns=int(r.first_touch_reruns),
                   device_ms=float(r.device_ms),
                   queries=np.frombuffer(C.string_at(r.queries, int(r.n_queries) * S.TCP_QUERY_DTYPE.itemsize),
                                         dtype=S.TCP_QUERY_DTYPE).copy() if r.n_queries else
                   np.zeros(0, dtype=S.TCP_QUERY_DTYPE))
        if node:
            k = int(r.node_k)
            cnt = np.ctypeslib.as_array(r.node_counters, shape=(HL * k * 20,)).reshape(HL, k, 20)
            nhb = np.ctypeslib.as_array(r.n_heartbeats, shape=(HL,))
            hb = int(tm.heartbeat_interval) or S.SHD_SEC
            nl = []
            for i in range(HL):
                c = np.ascontiguousarray(cnt[i, :int(nhb[i])])
                lp = C.POINTER(S.Lines)()
                S.check(S.lib().shd_tracker_node_lines(c.ctypes.data_as(C.POINTER(C.c_uint64)), len(c), hb, h0 + i,
                                                       C.byref(lp)), "shd_tracker_node_lines")
                nl += S.take_lines(lp)
            out["node_lines"] = sorted(nl, key=lambda x: (x[0], x[1]))
    finally:
        S.lib().shd_tcp_result_free(res)
    return out
