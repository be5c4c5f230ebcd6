"""Host driver of the TCP path on the GPU (include/shdtcp.h, csrc/tcp.hip).

Mirrors what a Shadow build would do around shd_tcp_run: the hosts' addresses
and RNG states come from the config front-end (dns.c's addresses, the seed
chain after attach), and the path latency / reliability of every host pair is
read from the product's lazy path cache (shd_pc_lookup, topology.c:2053-2092)
in the order the serial loop first touches the pairs: a client's connect
(host_connectToPeer's topology_isRoutable, host.c:1224-1234) touches
(client, server) before anything travels back.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

import shdgpu as S
import sim

RECV_BUF = 174760   # CONFIG_RECV_BUFFER_SIZE (definitions.h:159)
SEND_BUF = 131072   # CONFIG_SEND_BUFFER_SIZE (definitions.h:153)
TCP_WINDOW = 10     # --tcp-windows default (options.c:79)


def path_table(model: S.ModelArrays, g: S.GraphArrays, procs, peers):
    """Latency (ms) and reliability per pair of attached vertices ([V, V],
    V = the distinct vertices the hosts sit on) from the path cache, pairs
    resolved in first-touch order (clients by start time); pairs no
    connection uses stay -1.  Returns (lat, rel, host -> vertex index)."""
    m = model.struct
    H = int(m.n_hosts)
    hv = np.ctypeslib.as_array(m.host_vertex, shape=(H,)).copy()
    att, hvi = np.unique(hv, return_inverse=True)
    V = len(att)
    pc = sim.PathCache(g, att)
    lat = np.full((V, V), -1.0)
    rel = np.full((V, V), -1.0)
    order = sorted((p[1], k) for k, p in enumerate(procs) if peers[k] >= 0)
    try:
        for _, k in order:
            a, b = hvi[procs[k][0]], hvi[procs[peers[k]][0]]
            for s, d in ((a, b), (b, a)):
                if lat[s, d] < 0:
                    lat[s, d], rel[s, d] = pc.lookup(att[s], att[d])
    finally:
        pc.close()
    return lat, rel, hvi.astype(np.int32)


def run(model: S.ModelArrays, g: S.GraphArrays, ips, procs, peers, nbytes=20000, trace=True,
        recv_buf=RECV_BUF, send_buf=SEND_BUF, tcp_window=TCP_WINDOW, packets_per_host=0):
    """Run the TCP echo model on the GPU: procs = [(host, start ns)], peers =
    [-1 | server process]; ips: host-order uint32 per host.  Returns
    dict(lines=[(t, h, line)] in each host's order, next_event_id,
    next_packet_id, rng_probe, rounds, events, device_ms)."""
    m = model.struct
    H = int(m.n_hosts)
    lat, rel, hvi = path_table(model, g, procs, peers)
    keep = dict(ip=np.ascontiguousarray(ips, dtype=np.uint32), hv=np.ascontiguousarray(hvi),
                lat=np.ascontiguousarray(lat), rel=np.ascontiguousarray(rel),
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
    tm.n_vertices = lat.shape[0]
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
    res = C.POINTER(S.TcpResult)()
    S.check(S.lib().shd_tcp_run(C.byref(tm), 1 if trace else 0, C.byref(res)), "shd_tcp_run")
    try:
        r = res.contents
        if r.error:
            raise S.ShdError(f"shd_tcp_run: error bits {r.error:#x}")
        text = C.string_at(r.lines, r.len).decode() if r.len else ""
        lines = []
        for ln in text.splitlines():
            t, h, body = ln.split("\t", 2)
            lines.append((int(t), int(h), body))
        out = dict(lines=lines,
                   next_event_id=np.ctypeslib.as_array(r.next_event_id, shape=(H,)).copy(),
                   next_packet_id=np.ctypeslib.as_array(r.next_packet_id, shape=(H,)).copy(),
                   rng_probe=np.ctypeslib.as_array(r.rng_probe, shape=(H,)).copy(),
                   rounds=int(r.rounds), events=int(r.events), deliveries=int(r.deliveries),
                   device_ms=float(r.device_ms))
    finally:
        S.lib().shd_tcp_result_free(res)
    return out
