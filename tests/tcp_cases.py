"""TCP echo models (src/test/tcp/test_tcp.c in its nonblocking-epoll mode) run
through the reference's own loop (oracle/_ref/libshdref_loop.so, app 1) and
the oracle's restatement (oracle/o_tcp.c) -- TEST INFRASTRUCTURE.

The first two cases are the reference's own TCP tests
(src/test/tcp/tcp-nonblocking-epoll-{lossless,lossy}.test.shadow.config.xml):
one vertex with a 50 ms self-loop, loss 0 / 0.25, 10240 KiB/s, the server at
1 s, the client at 2 s, 20000 bytes each way, kill at 300 s.  The others widen
them: a 2 MB transfer (slow start into congestion avoidance, buffer
autotuning), 2 % loss on 500 kB (fast retransmit, SACK ranges), slow links
(CoDel queues at the receiver), heavy loss (RTO backoff), ten pairs on a lossy
geometric graph, hosts running several servers and clients at once, and a
pair whose first touch comes from the server's side.

The mixed_* cases put both transports in one model: besides the echo
processes, processes running a datagram application (shdgpu.h shd_udp_app:
send socket, destination rule, datagrams at start, one answer per datagram
read) share the hosts' interfaces, qdiscs, buckets and CoDel queues with the
TCP sockets (network_interface.c:519-579) -- run by the reference's loop with
the same per-process applications (oracle/ref_harness/ref_loop.c, app 1 with
proc_app).
"""
import hashlib

import numpy as np

import shdgpu as S
import workloads as W

SEC = S.SHD_SEC


def _one_vertex(lat, loss):
    return S.GraphArrays(1, [0], [0], [lat], [loss])


def _pair(lat, loss, nbytes, end_s, **bw):
    g = _one_vertex(lat, loss)
    return dict(graph=g, hv=[0, 0], procs=[(0, SEC), (1, 2 * SEC)], peers=[-1, 0], nbytes=nbytes, end=end_s, bw=bw)


def _geo_pairs():
    g = W.geometric_graph(30, seed=4, loss_max=0.05)
    H = 20
    procs = [(2 * i, SEC) for i in range(H // 2)] + [(2 * i + 1, 2 * SEC + i * 1000) for i in range(H // 2)]
    peers = [-1] * (H // 2) + list(range(H // 2))
    return dict(graph=g, hv=list(np.arange(H) % 30), procs=procs, peers=peers, nbytes=100000, end=60, bw={})


def _shared_hosts():
    g = W.geometric_graph(10, seed=2, loss_max=0.02)
    procs = [(0, SEC), (1, SEC), (2, SEC), (0, 2 * SEC), (1, 2 * SEC), (2, 2 * SEC), (0, 2 * SEC + 5)]
    return dict(graph=g, hv=[0, 3, 7], procs=procs, peers=[-1, -1, -1, 1, 2, 0, 2], nbytes=200000, end=60, bw={})


def _server_first():
    """the server side touches first: host 1 runs two servers and, at 2 s, a
    client of host 0's server, so vertex 17's row runs first; at 3 s host 2
    connects to one of host 1's servers and at 4 s host 0 to the other -- (0, 17)
    is then served by the row of 17, the server's vertex, not the connecting
    client's (a 40-vertex geometric graph: multi-hop paths whose two
    orientations differ in the last bits).  (test_tcp.c's server serves one
    peer and closes its listener: one server per client.)"""
    g = W.geometric_graph(40, seed=24, loss_max=0.01)
    procs = [(0, SEC), (1, SEC), (1, SEC), (1, 2 * SEC), (2, 3 * SEC), (0, 4 * SEC)]
    return dict(graph=g, hv=[0, 17, 33], procs=procs, peers=[-1, -1, -1, 0, 1, 2], nbytes=50000, end=30, bw={})


def _shared_hosts_rr():
    """shared_hosts under --interface-qdisc=rr: a host's client sockets and its
    server's child take turns at the interface (network_interface.c:466-490)"""
    c = _shared_hosts()
    c["qdisc"] = 1
    return c


def _loopback_pair():
    """a client of its own host's server: every packet goes out and comes back
    through the host's own interface as a +1 ns task (network_interface.c:548-555)"""
    return dict(graph=_one_vertex(50.0, 0.0), hv=[0], procs=[(0, SEC), (0, 2 * SEC)], peers=[-1, 0],
                nbytes=300000, end=60, bw={})


def _loopback_mixed():
    """host 0 serves a local client and a remote one while its own client talks
    to host 1: loopback and routed packets share host 0's interface and buckets"""
    g = W.geometric_graph(10, seed=2, loss_max=0.02)
    procs = [(0, SEC), (0, SEC), (1, SEC), (0, 2 * SEC), (1, 2 * SEC), (0, 2 * SEC + 7)]
    return dict(graph=g, hv=[0, 3], procs=procs, peers=[-1, -1, -1, 0, 1, 2], nbytes=200000, end=60, bw={})


EACH, ONCE, LISTENER = S.SHD_SEND_EACH, S.SHD_SEND_ONCE, S.SHD_SEND_LISTENER
WEIGHTED, PEER, REPLY = S.SHD_DEST_WEIGHTED, S.SHD_DEST_PEER, S.SHD_DEST_REPLY


def _mixed_hosts():
    """five hosts on a lossy geometric graph: an echo pair (server on host 0,
    client on host 1) and datagram processes -- host 0 PHOLD-like (a socket per
    datagram to a weighted host's listener, one per datagram read: it shares
    host 0's interface with the TCP server's child), hosts 2 and 3 a
    listener pair (2 sends to its peer 3, 3 answers each datagram to its
    sender), host 1 a connected-style client (one implicitly bound socket,
    beside its TCP client: both draw ports from host 1's RNG), host 4 no
    listener (datagrams for it are dropped at its interface)"""
    g = W.geometric_graph(12, seed=5, loss_max=0.02)
    procs = [(0, SEC), (1, 2 * SEC), (0, SEC + 500), (2, SEC), (3, SEC), (1, SEC + 300)]
    peers = [-1, 0, -1, -1, -1, -1]
    apps = [-1, -1, 0, 1, 2, 3]
    specs = [(EACH, WEIGHTED, 3, 1), (LISTENER, PEER, 4, 1), (LISTENER, REPLY, 0, 1), (ONCE, PEER, 2, 1)]
    return dict(graph=g, hv=[0, 4, 8, 11, 2], procs=procs, peers=peers, nbytes=300000, end=40, bw={},
                apps=apps, specs=specs, app_peer=[-1, 0, 3, -1, -1], payload=700)


def _mixed_slow_rr():
    """mixed_hosts on slow links (256 KiB/s down, 512 up: the receivers' CoDel
    queues fill) under the round-robin qdisc: the datagram sockets and the
    TCP sockets take turns at each interface"""
    c = _mixed_hosts()
    c["bw"] = dict(bw_down=256, bw_up=512)
    c["qdisc"] = 1
    c["payload"] = 1200
    return c


def _mixed_loopback():
    """one host with a loopback echo pair and a datagram listener sending to
    its own address (the +1 ns loopback task for UDP too), a second host
    PHOLD-like to both"""
    procs = [(0, SEC), (0, 2 * SEC), (0, SEC + 10), (1, SEC)]
    return dict(graph=_one_vertex(25.0, 0.0), hv=[0, 0], procs=procs, peers=[-1, 0, -1, -1], nbytes=100000, end=30,
                bw={}, apps=[-1, -1, 0, 1], specs=[(LISTENER, PEER, 3, 0), (EACH, WEIGHTED, 2, 1)], app_peer=[0, -1],
                payload=300)


CASES = {
    "ref_epoll_lossless": lambda: _pair(50.0, 0.0, 20000, 300),
    "ref_epoll_lossy": lambda: _pair(50.0, 0.25, 20000, 300),
    "bulk_2mb": lambda: _pair(50.0, 0.0, 2000000, 60),
    "lossy_2pct": lambda: _pair(50.0, 0.02, 500000, 60),
    "slow_links": lambda: _pair(20.0, 0.0, 300000, 60, bw_down=256, bw_up=512),
    "heavy_loss": lambda: _pair(30.0, 0.25, 200000, 200),
    "geo_pairs": _geo_pairs,
    "shared_hosts": _shared_hosts,
    "server_first": _server_first,
    "shared_hosts_rr": _shared_hosts_rr,
    "loopback_pair": _loopback_pair,
    "loopback_mixed": _loopback_mixed,
    "mixed_hosts": _mixed_hosts,
    "mixed_slow_rr": _mixed_slow_rr,
    "mixed_loopback": _mixed_loopback,
}

# the cases with echo processes only (oracle/o_tcp.c restates TCP alone)
ECHO_CASES = [n for n in CASES if not n.startswith("mixed_")]


def build(name):
    c = CASES[name]()
    m = W.phold_model(np.asarray(c["hv"], dtype=np.int32), end_time=c["end"] * SEC, trace=True,
                      queue_flags=S.SHD_QF_TRACE_STATUS, load=0, payload=c.get("payload", 1), **c["bw"])
    return c, m


def udp_arg(c):
    """tcp.run's udp argument of a case (None: echo processes only)"""
    if "apps" not in c:
        return None
    return dict(apps=c["apps"], specs=c["specs"], app_peer=c["app_peer"], payload=c.get("payload", 1))


def tcp_arg(c):
    """ref_loop_ffi.run's tcp argument of a case"""
    t = dict(peers=c["peers"], nbytes=c["nbytes"], qdisc=c.get("qdisc", 0))
    if "apps" in c:
        t.update(apps=c["apps"], specs=c["specs"], app_peer=c["app_peer"])
    return t


def status_lines(lines):
    """The [STATUS] lines (the tracker's heartbeat lines are not part of the TCP restatement)."""
    return [ln for ln in lines if not ln[2].startswith("[shadow-heartbeat]")]


def node_lines(lines):
    """The tracker's [shadow-heartbeat] lines (header, boot line, one per
    heartbeat), by (time, host), each host's in its own order."""
    return sorted((ln for ln in lines if ln[2].startswith("[shadow-heartbeat]")), key=lambda x: (x[0], x[1]))


def digest(lines):
    h = hashlib.sha256()
    for t, host, body in lines:
        h.update(f"{t}\t{host}\t{body}\n".encode())
    return h.hexdigest()


def ip_ints(ips):
    return [int.from_bytes(bytes(int(x) for x in ip.split(".")), "big") for ip in ips]


def by_host(lines):
    """Each host's lines in its own order (the GPU runs hosts in parallel; a
    host's own sequence is the serial loop's)."""
    return sorted(lines, key=lambda x: x[1])   # stable: keeps each host's order
