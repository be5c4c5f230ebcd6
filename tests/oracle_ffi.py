"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference (see oracle/oracle.h); it is
the checker for libshdgpu and is never on the product path.
"""
import ctypes as C
import os

import numpy as np

import shdgpu as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "oracle", "liboracle.so")
P = C.POINTER


class ORun(C.Structure):
    _fields_ = [("trace", P(S.TraceRec)), ("n_trace", C.c_uint64), ("cap_trace", C.c_uint64),
                ("digest", P(S.HostDigest)), ("n_events", C.c_uint64), ("n_pkt_events", C.c_uint64),
                ("window_ns", C.c_uint64), ("rows_run", C.c_int32), ("self_run", C.c_int32),
                ("wall_ms", C.c_double), ("mark_events", C.c_uint64),
                ("mark_pkt_events", C.c_uint64), ("mark_wall_ms", C.c_double)]


class OCodelEntry(C.Structure):
    _fields_ = [("ts", C.c_uint64), ("len", C.c_uint32), ("id", C.c_uint32), ("src", C.c_uint32),
                ("_pad", C.c_uint32)]


class OCodel(C.Structure):
    _fields_ = [("q", P(OCodelEntry)), ("cap", C.c_uint32), ("head", C.c_uint32),
                ("count", C.c_uint32), ("total", C.c_uint64), ("mode", C.c_uint32),
                ("interval_expire", C.c_uint64), ("next_drop", C.c_uint64),
                ("drop_count", C.c_uint32), ("drop_count_last", C.c_uint32)]


class OBaseline(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("rows_ms", "warmup_ms", "serial_ms", "parallel_ms")] + \
               [(n, C.c_uint64) for n in ("serial_events", "serial_pkt_events", "parallel_events",
                                          "parallel_pkt_events", "parallel_rounds", "parallel_first_touch",
                                          "ambiguous", "window_ns")] + \
               [("threads", C.c_int32), ("same_end_state", C.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run `make -C oracle` (or __graft_entry__.build())")
        l = C.CDLL(LIB)
        l.o_rand_r.restype = C.c_int32; l.o_rand_r.argtypes = [P(C.c_uint32)]
        l.o_next_double.restype = C.c_double; l.o_next_double.argtypes = [P(C.c_uint32)]
        l.o_next_uint.restype = C.c_uint32; l.o_next_uint.argtypes = [P(C.c_uint32)]
        l.o_seed_chain.argtypes = [C.c_uint32, C.c_int32, P(C.c_uint32)]
        l.o_graph_new.restype = C.c_void_p; l.o_graph_new.argtypes = [P(S.Graph)]
        l.o_graph_free.argtypes = [C.c_void_p]
        l.o_graph_props.argtypes = [C.c_void_p, P(S.GraphProps)]
        l.o_direct_path.argtypes = [C.c_void_p, C.c_int32, C.c_int32, P(C.c_double), P(C.c_double)]
        l.o_self_path.argtypes = [C.c_void_p, C.c_int32, P(C.c_double), P(C.c_double)]
        l.o_sssp_row.argtypes = [C.c_void_p, C.c_int32, P(C.c_int32), C.c_int32, P(C.c_double),
                                 P(C.c_double), P(C.c_int32), P(C.c_int32), P(C.c_int64)]
        l.o_topo_new.restype = C.c_void_p
        l.o_topo_new.argtypes = [C.c_void_p, P(C.c_int32), C.c_int32, C.c_int32]
        l.o_topo_free.argtypes = [C.c_void_p]
        l.o_topo_precompute_rows.argtypes = [C.c_void_p, C.c_int]
        l.o_topo_get.argtypes = [C.c_void_p, C.c_int32, C.c_int32, P(C.c_double), P(C.c_double)]
        l.o_topo_would_run.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
        l.o_topo_touch.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
        l.o_topo_count_packet.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
        l.o_topo_packet_count.restype = C.c_uint64
        l.o_topo_packet_count.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
        l.o_topo_min_latency.restype = C.c_double; l.o_topo_min_latency.argtypes = [C.c_void_p]
        l.o_topo_rows_run.restype = C.c_int32; l.o_topo_rows_run.argtypes = [C.c_void_p]
        l.o_codel_init.argtypes = [P(OCodel), C.c_uint32]
        l.o_codel_free.argtypes = [P(OCodel)]
        l.o_codel_enqueue.argtypes = [P(OCodel), C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
        l.o_codel_dequeue.argtypes = [P(OCodel), C.c_uint64, P(OCodelEntry), P(OCodelEntry),
                                      C.c_uint32, P(C.c_uint32)]
        l.o_codel_control_law.restype = C.c_uint64
        l.o_codel_control_law.argtypes = [C.c_uint32, C.c_uint64]
        l.o_engine_run.argtypes = [P(S.Model), P(S.Graph), C.c_int32, P(ORun)]
        l.o_run_free.argtypes = [P(ORun)]
        l.o_event_compare.argtypes = [P(S.Event), P(S.Event)]
        l.o_engine_set_mark.argtypes = [C.c_uint64]
        l.o_engine_set_counts_out.argtypes = [C.c_void_p, C.c_int32]
        l.o_engine_set_heartbeats_out.argtypes = [C.c_void_p, C.c_uint32]
        l.o_engine_set_pushes.argtypes = [C.c_void_p, C.c_uint64]
        l.o_baseline.argtypes = [P(S.Model), P(S.Graph), C.c_uint64, C.c_uint64, C.c_int, P(OBaseline)]
        l.o_state_new.restype = C.c_void_p
        l.o_state_new.argtypes = [P(S.Model), P(S.Graph), C.c_int32]
        l.o_state_new_part.restype = C.c_void_p
        l.o_state_new_part.argtypes = [P(S.Model), P(S.Graph), C.c_int32, C.c_int32]
        l.o_state_run_serial.argtypes = [C.c_void_p, C.c_uint64]
        l.o_state_inject.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        l.o_state_take_egress.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, P(C.c_uint64)]
        l.o_state_defer_touches.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        l.o_state_take_touches.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, P(C.c_uint64)]
        l.o_state_next_time.restype = C.c_uint64
        l.o_state_next_time.argtypes = [C.c_void_p]
        l.o_state_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, P(C.c_uint64)]
        l.o_state_digest.argtypes = [C.c_void_p, C.c_void_p]
        l.o_state_stats.restype = P(ORun)
        l.o_state_stats.argtypes = [C.c_void_p]
        l.o_state_free.argtypes = [C.c_void_p]
        _lib = l
    return _lib


class OGraph:
    def __init__(self, g: S.GraphArrays):
        self.g = g
        self.ptr = lib().o_graph_new(C.byref(g.struct))

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().o_graph_free(self.ptr)
            self.ptr = None

    def props(self):
        p = S.GraphProps()
        lib().o_graph_props(self.ptr, C.byref(p))
        return p

    def row(self, src, targets, count_ties=True):
        t = np.ascontiguousarray(targets, dtype=np.int32)
        n = len(t)
        lat = np.empty(n); rel = np.empty(n)
        ok = np.empty(n, np.int32); hops = np.empty(n, np.int32)
        ties = C.c_int64(0)
        lib().o_sssp_row(self.ptr, int(src), S.as_ptr(t, C.c_int32), n, S.as_ptr(lat, C.c_double),
                         S.as_ptr(rel, C.c_double), S.as_ptr(ok, C.c_int32),
                         S.as_ptr(hops, C.c_int32), C.byref(ties) if count_ties else None)
        return lat, rel, ok, hops, ties.value

    def direct(self, s, d):
        a, b = C.c_double(), C.c_double()
        rc = lib().o_direct_path(self.ptr, int(s), int(d), C.byref(a), C.byref(b))
        return (a.value, b.value) if rc == 0 else (float("nan"), float("nan"))

    def self_path(self, s):
        a, b = C.c_double(), C.c_double()
        lib().o_self_path(self.ptr, int(s), C.byref(a), C.byref(b))
        return a.value, b.value


class OTopo:
    def __init__(self, og: OGraph, attached, force_rows=False):
        self.og = og
        self.att = np.ascontiguousarray(attached, dtype=np.int32)
        self.ptr = lib().o_topo_new(og.ptr, S.as_ptr(self.att, C.c_int32), len(self.att),
                                    int(force_rows))

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().o_topo_free(self.ptr)
            self.ptr = None

    def get(self, s, d):
        a, b = C.c_double(), C.c_double()
        lib().o_topo_get(self.ptr, int(s), int(d), C.byref(a), C.byref(b))
        return a.value, b.value

    def rows_run(self):
        return lib().o_topo_rows_run(self.ptr)

    def would_run(self, s, d) -> bool:
        return bool(lib().o_topo_would_run(self.ptr, int(s), int(d)))

    def touch(self, s, d):
        lib().o_topo_touch(self.ptr, int(s), int(d))


def engine_run(model: S.ModelArrays, g: S.GraphArrays, force_rows=False, mark=None, path_counts=None,
               heartbeats=None, pushes=None):
    """Serial reference loop; returns (trace ndarray, digest ndarray, ORun stats dict).
    path_counts: a uint64 [V, V] array filled with the packet count of every
    cached path entry, by the orientation it is stored under.
    heartbeats: a uint32 [H, K, 2] array filled with each host's cumulative
    interface (in, out) packet counts at its k-th heartbeat (tracker.c:566-611)."""
    if heartbeats is not None:
        assert heartbeats.dtype == np.uint32 and heartbeats.ndim == 3 and heartbeats.flags.c_contiguous
        lib().o_engine_set_heartbeats_out(heartbeats.ctypes.data, heartbeats.shape[1])
    else:
        lib().o_engine_set_heartbeats_out(None, 0)
    push = None if pushes is None else np.ascontiguousarray(pushes, dtype=S.EVENT_DTYPE)
    lib().o_engine_set_pushes(None if push is None or not len(push) else push.ctypes.data,
                              0 if push is None else len(push))
    lib().o_engine_set_mark((1 << 64) - 1 if mark is None else int(mark))
    if path_counts is not None:
        assert path_counts.dtype == np.uint64 and path_counts.shape == (g.n_vertices, g.n_vertices)
        assert path_counts.flags.c_contiguous
        lib().o_engine_set_counts_out(path_counts.ctypes.data, g.n_vertices)
    else:
        lib().o_engine_set_counts_out(None, 0)
    r = ORun()
    rc = lib().o_engine_run(C.byref(model.struct), C.byref(g.struct), int(force_rows), C.byref(r))
    assert rc == 0
    n = r.n_trace
    tr = np.empty(n, dtype=S.TRACE_DTYPE)
    if n:
        C.memmove(tr.ctypes.data, r.trace, n * 32)
    H = model.n_hosts
    dg = np.empty(H, dtype=S.DIGEST_DTYPE)
    C.memmove(dg.ctypes.data, r.digest, H * S.DIGEST_DTYPE.itemsize)
    stats = dict(n_events=r.n_events, n_pkt_events=r.n_pkt_events, rows_run=r.rows_run,
                 self_run=r.self_run, wall_ms=r.wall_ms, mark_events=r.mark_events,
                 mark_pkt_events=r.mark_pkt_events, mark_wall_ms=r.mark_wall_ms)
    lib().o_run_free(C.byref(r))
    reset_outputs()
    return tr, dg, stats


class OState:
    """An oracle engine state (oracle.h o_state_*).  With `hosts=(lo, hi)` it is
    one side of a co-simulation: only those hosts run here, their sends to the
    others leave by take_egress(), the others' packets come in by inject()."""

    def __init__(self, model: S.ModelArrays, g: S.GraphArrays, hosts=None, pushes=None):
        self.model, self.g = model, g   # the state points into both
        push = None if pushes is None else np.ascontiguousarray(pushes, dtype=S.EVENT_DTYPE)
        lib().o_engine_set_pushes(None if push is None or not len(push) else push.ctypes.data,
                                  0 if push is None else len(push))
        if hosts is None:
            self.ptr = lib().o_state_new(C.byref(model.struct), C.byref(g.struct), 0)
        else:
            self.ptr = lib().o_state_new_part(C.byref(model.struct), C.byref(g.struct), int(hosts[0]),
                                              int(hosts[1]))
        reset_outputs()
        assert self.ptr, "o_state_new_part: bad host range"

    def run_serial(self, t_until):
        lib().o_state_run_serial(self.ptr, int(t_until))

    def inject(self, events):
        ev = np.ascontiguousarray(events, dtype=S.EVENT_DTYPE)
        assert lib().o_state_inject(self.ptr, ev.ctypes.data if len(ev) else None, len(ev)) == 0

    def take_egress(self) -> np.ndarray:
        n = C.c_uint64()
        lib().o_state_take_egress(self.ptr, None, 0, C.byref(n))
        out = np.empty(n.value, dtype=S.EVENT_DTYPE)
        assert lib().o_state_take_egress(self.ptr, out.ctypes.data if n.value else None, n.value,
                                         C.byref(n)) == 0
        return out

    def defer_touches(self, recs):
        """the other side's first touches of the coming window (one lazy cache
        across the sides, oracle.h o_state_defer_touches)"""
        r = np.ascontiguousarray(recs, dtype=S.PENDING_DTYPE)
        assert lib().o_state_defer_touches(self.ptr, r.ctypes.data if len(r) else None, len(r)) == 0

    def take_touches(self) -> np.ndarray:
        """this side's first touches of the window just run (the other side's
        deferred ones applied first)"""
        n = C.c_uint64()
        lib().o_state_take_touches(self.ptr, None, 0, C.byref(n))
        out = np.empty(n.value, dtype=S.PENDING_DTYPE)
        assert lib().o_state_take_touches(self.ptr, out.ctypes.data if n.value else None, n.value,
                                          C.byref(n)) == 0
        return out

    def next_time(self) -> int:
        return lib().o_state_next_time(self.ptr)

    def trace(self) -> np.ndarray:
        n = C.c_uint64()
        lib().o_state_trace(self.ptr, None, 0, C.byref(n))
        out = np.empty(n.value, dtype=S.TRACE_DTYPE)
        if n.value:
            assert lib().o_state_trace(self.ptr, out.ctypes.data, n.value, C.byref(n)) == 0
        return out

    def digest(self) -> np.ndarray:
        out = np.empty(self.model.n_hosts, dtype=S.DIGEST_DTYPE)
        lib().o_state_digest(self.ptr, out.ctypes.data)
        return out

    def counts(self):
        r = lib().o_state_stats(self.ptr).contents
        return r.n_events, r.n_pkt_events

    def close(self):
        if getattr(self, "ptr", None):
            lib().o_state_free(self.ptr)
            self.ptr = None

    __del__ = close


def rand_r(state: int):
    s = C.c_uint32(state)
    v = lib().o_rand_r(C.byref(s))
    return v, s.value


def reset_outputs():
    """Clear the oracle's optional output / input hooks (heartbeat snapshots,
    path counts, pushed events, the mark): they point at caller arrays."""
    lib().o_engine_set_heartbeats_out(None, 0)
    lib().o_engine_set_counts_out(None, 0)
    lib().o_engine_set_pushes(None, 0)
    lib().o_engine_set_mark((1 << 64) - 1)


def baseline(model: S.ModelArrays, g: S.GraphArrays, t_mark: int, t_end: int, threads: int) -> dict:
    """The bench's CPU baseline (oracle.h o_baseline): warm up to t_mark, then
    the window [t_mark, t_end) serially on one core and in parallel rounds on
    `threads` cores from the same state; returns the timings, the counts and
    whether both end states are equal."""
    reset_outputs()
    o = OBaseline()
    rc = lib().o_baseline(C.byref(model.struct), C.byref(g.struct), int(t_mark), int(t_end), int(threads),
                          C.byref(o))
    out = {f: getattr(o, f) for f, _ in OBaseline._fields_}
    out["rc"] = rc
    return out


# ---- the TCP path (o_tcp.c) ----
class TcpCfg(C.Structure):
    _fields_ = [("n_hosts", C.c_int32), ("n_procs", C.c_int32),
                ("host_ip", C.POINTER(C.c_uint32)), ("host_seed", C.POINTER(C.c_uint32)),
                ("host_vertex", C.POINTER(C.c_int32)),
                ("bw_down_kibps", C.POINTER(C.c_uint64)), ("bw_up_kibps", C.POINTER(C.c_uint64)),
                ("proc_host", C.POINTER(C.c_int32)), ("proc_start", C.POINTER(C.c_uint64)),
                ("proc_peer", C.POINTER(C.c_int32)),
                ("end_time", C.c_uint64), ("heartbeat_interval", C.c_uint64),
                ("tcp_bytes", C.c_uint32), ("recv_buf", C.c_uint32), ("send_buf", C.c_uint32),
                ("tcp_window", C.c_uint32), ("no_lines", C.c_uint32), ("qdisc_rr", C.c_uint32),
                ("proc_app", C.POINTER(C.c_int32)), ("app_spec", C.POINTER(C.c_uint32)),
                ("udp_payload", C.c_uint32), ("_pad", C.c_uint32), ("app_peer", C.POINTER(C.c_int32)),
                ("dest_cum", C.POINTER(C.c_double)), ("host_class", C.POINTER(C.c_uint8)),
                ("n_classes", C.c_int32), ("_pad2", C.c_int32)]


class TcpOut(C.Structure):
    _fields_ = [("lines", C.c_char_p), ("len", C.c_size_t), ("n_lines", C.c_uint64),
                ("next_event_id", C.POINTER(C.c_uint64)), ("next_packet_id", C.POINTER(C.c_uint64)),
                ("rng_probe", C.POINTER(C.c_uint32)), ("events", C.c_uint64)]


def tcp_run(model, g, ips, procs, peers, nbytes=20000, recv_buf=174760, send_buf=131072, tcp_window=10,
            lines=True, qdisc=0, udp=None):
    """The oracle's TCP echo run (o_tcp.c) on the model's hosts: procs = [(host,
    start)], peers = [-1 | server process]; ips: host-order uint32 per host.
    Returns dict(lines=[(t, h, line)], next_event_id, next_packet_id, rng_probe)
    with a delivery copy's release (host -1) put on its receiver, as the
    reference-loop binding does.  udp: as shadow-1_amd/tcp.py's (datagram
    processes beside the echo ones)."""
    import numpy as np
    m = model.struct
    H = int(m.n_hosts)
    og = lib().o_graph_new(C.byref(g.struct))
    hv = np.ctypeslib.as_array(m.host_vertex, shape=(H,)).copy()
    att = np.ascontiguousarray(np.unique(hv).astype(np.int32))
    topo = lib().o_topo_new(og, att.ctypes.data_as(C.POINTER(C.c_int32)), len(att), 0)
    ipa = np.ascontiguousarray(ips, dtype=np.uint32)
    ph = np.ascontiguousarray([p[0] for p in procs], dtype=np.int32)
    ps = np.ascontiguousarray([p[1] for p in procs], dtype=np.uint64)
    pp = np.ascontiguousarray(peers, dtype=np.int32)
    cfg = TcpCfg()
    cfg.n_hosts = H
    cfg.n_procs = len(ph)
    cfg.host_ip = ipa.ctypes.data_as(C.POINTER(C.c_uint32))
    cfg.host_seed = m.host_rng
    cfg.host_vertex = m.host_vertex
    cfg.bw_down_kibps = m.bw_down_kibps
    cfg.bw_up_kibps = m.bw_up_kibps
    cfg.proc_host = ph.ctypes.data_as(C.POINTER(C.c_int32))
    cfg.proc_start = ps.ctypes.data_as(C.POINTER(C.c_uint64))
    cfg.proc_peer = pp.ctypes.data_as(C.POINTER(C.c_int32))
    cfg.end_time = m.end_time
    cfg.heartbeat_interval = m.heartbeat_interval
    cfg.tcp_bytes = nbytes
    cfg.recv_buf = recv_buf
    cfg.send_buf = send_buf
    cfg.tcp_window = tcp_window
    cfg.no_lines = 0 if lines else 1
    cfg.qdisc_rr = int(qdisc)
    if udp is not None:
        pa = np.ascontiguousarray(udp["apps"], dtype=np.int32)
        sp = np.ascontiguousarray([[int(x) for x in a] for a in udp["specs"]], dtype=np.uint32).ravel()
        ap = np.ascontiguousarray(udp.get("app_peer", [-1] * H), dtype=np.int32)
        cfg.proc_app = pa.ctypes.data_as(C.POINTER(C.c_int32))
        cfg.app_spec = sp.ctypes.data_as(C.POINTER(C.c_uint32))
        cfg.app_peer = ap.ctypes.data_as(C.POINTER(C.c_int32))
        cfg.udp_payload = int(udp.get("payload", m.payload or 1))
        cfg.dest_cum = m.dest_cum
        cfg.host_class = m.host_class
        cfg.n_classes = m.n_classes
    out = TcpOut()
    l = lib()
    l.o_tcp_run.argtypes = [C.POINTER(TcpCfg), C.c_void_p, C.POINTER(TcpOut)]
    l.o_tcp_free.argtypes = [C.POINTER(TcpOut)]
    try:
        rc = l.o_tcp_run(C.byref(cfg), topo, C.byref(out))
        assert rc == 0, rc
        text = C.string_at(out.lines, out.len).decode() if out.len else ""
        ipstr = [".".join(str((int(x) >> s) & 255) for s in (24, 16, 8, 0)) for x in ipa]
        by_ip = {ip: h for h, ip in enumerate(ipstr)}
        lines = []
        for ln in text.splitlines():
            t, h, body = ln.split("\t", 2)
            h = int(h)
            if h < 0 and " -> " in body:
                h = by_ip[body.split(" -> ")[1].split(":")[0]]
            lines.append((int(t), h, body))
        res = dict(lines=lines,
                   next_event_id=np.ctypeslib.as_array(out.next_event_id, shape=(H,)).copy(),
                   next_packet_id=np.ctypeslib.as_array(out.next_packet_id, shape=(H,)).copy(),
                   rng_probe=np.ctypeslib.as_array(out.rng_probe, shape=(H,)).copy(),
                   events=int(out.events))
        l.o_tcp_free(C.byref(out))
    finally:
        lib().o_topo_free(topo)
        lib().o_graph_free(og)
    return res
