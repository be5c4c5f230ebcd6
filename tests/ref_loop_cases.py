"""The models run through the reference's own compiled event loop
(oracle/_ref/libshdref_loop.so, tests/ref_loop_ffi.py) -- TEST INFRASTRUCTURE.

Each case builds the same model for three runs: the reference loop (fixtures,
tests/golden/make_ref_loop.py), the oracle (tests/test_ref_loop_cpu.py) and the
HIP engine (tests/test_ref_loop_gpu.py).  Every case traces the application's
side too (SHD_QF_TRACE_STATUS), so the [STATUS] lines of packet.c:647-659 can
be made from any of the three and compared line for line.
"""
import hashlib
import os

import numpy as np

import shdgpu as S
import workloads as W

# every case records the application's side of each datagram (the [STATUS]
# lines) and the tracker counters (the [node] lines)
TS = S.SHD_QF_TRACE_STATUS | S.SHD_QF_HEARTBEATS
HERE = os.path.dirname(os.path.abspath(__file__))


def _phold_v100():
    """PHOLD-UDP, 100 hosts on a 100-vertex geometric graph, edge loss U[0, 0.01]
    (INET drops), loopback sends included."""
    g = W.geometric_graph(100, seed=9)
    m = W.phold_model(W.hosts_on_vertices(100, 1), end_time=3 * S.SHD_SEC, trace=True, load=8, queue_flags=TS)
    return dict(model=m, graph=g)


def _codel():
    """1500-B messages into 512 KiB/s receive buckets: CoDel queues build and drop."""
    g = W.geometric_graph(60, seed=9)
    m = W.phold_model(W.hosts_on_vertices(60, 1), end_time=3 * S.SHD_SEC, trace=True, payload=1500, bw_down=512,
                      codelq_cap=256, load=32, queue_flags=TS)
    return dict(model=m, graph=g)


def _two_per_vertex_lossy():
    """Two hosts per vertex (paths between hosts of one vertex are the vertex's
    self path), edge loss U[0, 0.05]."""
    g = W.geometric_graph(60, seed=5, loss_max=0.05)
    m = W.phold_model(W.hosts_on_vertices(60, 2), end_time=3 * S.SHD_SEC, trace=True, load=4, queue_flags=TS)
    return dict(model=m, graph=g)


def _heartbeats():
    """Per-host heartbeat intervals 0.5 / 1 / 2 s (<host heartbeatfrequency>):
    the tracker's [node] lines."""
    V, end = 60, int(4.5 * S.SHD_SEC)
    g = W.geometric_graph(V, seed=3)
    hbi = np.array([S.SHD_SEC // 2, S.SHD_SEC, 2 * S.SHD_SEC], dtype=np.uint64)[np.arange(V) % 3]
    m0 = W.phold_model(W.hosts_on_vertices(V, 1), end_time=end, trace=True)
    m = S.ModelArrays(m0.host_vertex, m0.host_rng, m0.bw_down, m0.bw_up, m0.dest_cum, end_time=end, trace=True,
                      queue_flags=TS, host_heartbeat=hbi)
    return dict(model=m, graph=g, hb_k=(end - 1) // (S.SHD_SEC // 2))


def _pushed_starts():
    """0-6 processes per host (several at the first heartbeat, one past the
    end time): the caller's pushed application starts, in <process> order."""
    V = 60
    g = W.geometric_graph(V, seed=13)
    m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=3 * S.SHD_SEC, trace=True, load=3,
                      queue_flags=S.SHD_QF_NO_APP_START | TS)
    rng = np.random.default_rng(2)
    ev = []
    for h in range(V):
        for k in range(int(rng.integers(0, 3)) + (4 if h % 5 == 0 else 0)):
            t = S.SHD_SEC if (h % 5 == 0 and k < 4) else \
                int(rng.integers(1, 4)) * S.SHD_SEC // 2 + int(rng.integers(0, 1000))
            ev.append((t, 0, h, h, 0, S.EV_APP_START))
    ev.append((5 * S.SHD_SEC, 0, 3, 3, 0, S.EV_APP_START))
    return dict(model=m, graph=g, pushes=np.array(ev, dtype=S.EVENT_DTYPE), hb_k=2)


def _tor():
    """BASELINE C4's relay/client model at 340 hosts on the bundled (complete)
    topology: per-class destination weights, random attachment."""
    g, m = W.tor_model(40, 300, end_time=3 * S.SHD_SEC, trace=True, queue_flags=TS)
    return dict(model=m, graph=g)


def _bootstrap():
    """<shadow bootstraptime> 1.5 s: no drops and unlimited receive while it lasts."""
    g = W.geometric_graph(40, seed=21, loss_max=0.05)
    m = W.phold_model(W.hosts_on_vertices(40, 1), end_time=3 * S.SHD_SEC, trace=True, load=6,
                      bootstrap_end=int(1.5 * S.SHD_SEC), payload=1500, bw_down=512, codelq_cap=512, queue_flags=TS)
    return dict(model=m, graph=g)


def _c1():
    """BASELINE C1: the bundled example config (2 hosts on the 1-vertex "isp"
    topology, starts at 1 s / 2 s) through the config front-end, PHOLD-UDP in
    place of tgen, to 60 s."""
    with open(os.path.join(HERE, "golden", "example_shadow.config.xml"), "rb") as f:
        xml = f.read()
    g, m, pushes, names, ips = W.config_model(xml, trace=True, queue_flags=TS)
    m = S.ModelArrays(m.host_vertex, m.host_rng, m.bw_down, m.bw_up, m.dest_cum, end_time=60 * S.SHD_SEC,
                      load=m.struct.load, payload=m.struct.payload, trace=True, host_heartbeat=m.host_heartbeat,
                      queue_flags=int(m.struct.queue_flags))
    return dict(model=m, graph=g, pushes=pushes)


def _udp_echo():
    """The second device application (SHD_APP_UDP_ECHO, ref_loop.c app 2): 20
    servers and 40 clients, two or three clients per server, 4 requests in
    flight each, edge loss U[0, 0.02] (lost requests and replies shrink the
    loops)."""
    V = 60
    g = W.geometric_graph(V, seed=17, loss_max=0.02)
    peer = np.array([-1] * 20 + [(h * 7) % 20 for h in range(20, V)], dtype=np.int32)
    m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=3 * S.SHD_SEC, trace=True, load=4, queue_flags=TS,
                      app_peer=peer)
    return dict(model=m, graph=g)


def _udp_echo_codel():
    """UDP echo with 1500-B datagrams into 512 KiB/s receive buckets at the
    servers: 8 servers, 32 clients with 8 requests in flight each -- CoDel
    queues build and drop at the servers."""
    V = 40
    g = W.geometric_graph(V, seed=29)
    peer = np.array([-1] * 8 + [h % 8 for h in range(8, V)], dtype=np.int32)
    bw = np.where(peer < 0, 512, 10240).astype(np.uint64)
    m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=3 * S.SHD_SEC, trace=True, load=8, payload=1500,
                      bw_down=bw, codelq_cap=512, queue_flags=TS, app_peer=peer)
    return dict(model=m, graph=g)


def _udp_mix(payload=1, bw_server=10240, client_load=2):
    """The general datagram application (SHD_APP_UDP, ref_loop.c app 3): five
    kinds of host on one 60-vertex geometric graph, edge loss U[0, 0.02]:
    20 PHOLD hosts (new socket per datagram, weighted destinations over
    themselves and the sinks, 3 each at the start, one per read), 10 servers
    (reply from the listener to whatever they read), 15 clients (one socket,
    weighted over the servers, 2 requests in flight each), 5 one-way senders
    (4 datagrams from the listener to one sink each, nothing per read) and 10
    sinks (read only)."""
    V = 60
    g = W.geometric_graph(V, seed=31, loss_max=0.02)
    m0 = W.phold_model(W.hosts_on_vertices(V, 1), end_time=3 * S.SHD_SEC, trace=True)
    kind = np.array([0] * 20 + [1] * 10 + [2] * 15 + [3] * 5 + [4] * 10, dtype=np.uint8)
    specs = [(S.SHD_SEND_EACH, S.SHD_DEST_WEIGHTED, 3, 1),      # PHOLD
             (S.SHD_SEND_LISTENER, S.SHD_DEST_REPLY, 0, 1),     # server
             (S.SHD_SEND_ONCE, S.SHD_DEST_WEIGHTED, client_load, 1),   # client
             (S.SHD_SEND_LISTENER, S.SHD_DEST_PEER, 4, 0),      # one-way sender
             (S.SHD_SEND_LISTENER, S.SHD_DEST_WEIGHTED, 0, 0)]  # sink
    w = np.zeros((2, V))
    w[0, (kind == 0) | (kind == 4)] = 1.0      # class 0: PHOLD hosts and sinks
    w[1, kind == 1] = 1.0                      # class 1 (clients): the servers
    cum = np.cumsum(w / w.sum(axis=1, keepdims=True), axis=1)
    for r in range(2):   # exactly 1 from each row's last weighted host on (the rest stay unweighted)
        cum[r, np.flatnonzero(w[r])[-1]:] = 1.0
    cls = (kind == 2).astype(np.uint8)
    peer = np.full(V, -1, dtype=np.int32)
    peer[kind == 3] = np.flatnonzero(kind == 4)[:5]
    bw = np.where(kind == 1, bw_server, 10240).astype(np.uint64)
    m = S.ModelArrays(m0.host_vertex, m0.host_rng, bw, m0.bw_up, cum, end_time=3 * S.SHD_SEC, trace=True,
                      payload=payload, codelq_cap=512, queue_flags=TS, host_class=cls, app_peer=peer,
                      app_specs=specs, host_app=kind)
    return dict(model=m, graph=g)


CASES = {
    "phold_v100": _phold_v100,
    "codel": _codel,
    "two_per_vertex_lossy": _two_per_vertex_lossy,
    "heartbeats": _heartbeats,
    "pushed_starts": _pushed_starts,
    "tor": _tor,
    "bootstrap": _bootstrap,
    "c1": _c1,
    "udp_echo": _udp_echo,
    "udp_echo_codel": _udp_echo_codel,
    "udp_mix": _udp_mix,
    # 1500-B datagrams into 256 KiB/s receive buckets at the servers, 24
    # requests in flight per client: the servers' CoDel queues build and drop
    "udp_mix_codel": lambda: _udp_mix(payload=1500, bw_server=256, client_load=24),
}


def procs_of(case):
    p = case.get("pushes")
    return None if p is None else [(int(e["dst"]), int(e["time"])) for e in p]


def split_lines(lines):
    """(status lines, heartbeat lines) of a run, each ordered by (time, host),
    every host's lines in their own order"""
    key = lambda x: (x[0], x[1])   # noqa: E731  (a stable sort)
    st = sorted((x for x in lines if not x[2].startswith("[shadow-heartbeat]")), key=key)
    hb = sorted((x for x in lines if x[2].startswith("[shadow-heartbeat]")), key=key)
    return st, hb


def digest_lines(lines) -> str:
    h = hashlib.sha256()
    for t, host, body in lines:
        h.update(b"%d\t%d\t%s\n" % (t, host, body.encode()))
    return h.hexdigest()


def heartbeat_lines(model, hb, K):
    """The [node] lines every host logs (tracker.c:419-465), from [H, K, 2]
    interface counters (the oracle's or the engine's), with the times they are
    logged at (boot, then every interval)."""
    m = model.struct
    H = int(m.n_hosts)
    hbi = np.ctypeslib.as_array(m.host_heartbeat, shape=(H,)) if m.host_heartbeat else \
        np.full(H, int(m.heartbeat_interval), dtype=np.uint64)
    end = int(m.end_time)
    out = []
    for h in range(H):
        k = (end - 1) // int(hbi[h])
        ls = S.tracker_node_lines(hb[h, :k], int(hbi[h]), int(m.payload))
        times = [0, 0] + [int(hbi[h]) * (i + 1) for i in range(k)]
        out += [(t, h, x) for t, x in zip(times, ls)]
    return sorted(out, key=lambda x: (x[0], x[1]))
