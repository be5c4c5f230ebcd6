"""ctypes binding of oracle/_ref/libshdref_loop.so -- TEST INFRASTRUCTURE ONLY.

The reference's own serial event loop (worker.c, scheduler.c, host.c,
network_interface.c, router*.c, descriptor/*.c, tracker.c, packet.c, ...)
compiled unmodified from /root/reference (oracle/Makefile `ref`), with the
collaborators the image cannot build as test doubles (oracle/ref_harness/
ref_loop.c).  It only exists in the build container: the tests that use it
skip where it was not built, and the fixtures it makes are committed under
tests/golden/ (tests/golden/make_ref_loop.py) for everywhere else.
"""
import ctypes as C
import os
import shutil
import tempfile

import numpy as np

import oracle_ffi as O
import shdgpu as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "oracle", "_ref", "libshdref_loop.so")
P = C.POINTER

class Cfg(C.Structure):
    _fields_ = [("n_hosts", C.c_int32), ("app", C.c_int32),
                ("host_seed", P(C.c_uint32)), ("host_vertex", P(C.c_int32)),
                ("bw_down_kibps", P(C.c_uint64)), ("bw_up_kibps", P(C.c_uint64)),
                ("dest_cum", P(C.c_double)), ("host_class", P(C.c_uint8)),
                ("n_classes", C.c_int32), ("_pad", C.c_int32),
                ("host_heartbeat", P(C.c_uint64)), ("host_start", P(C.c_uint64)),
                ("n_procs", C.c_int32), ("_pad2", C.c_int32), ("proc_host", P(C.c_int32)),
                ("proc_start", P(C.c_uint64)),
                ("end_time", C.c_uint64), ("bootstrap_end", C.c_uint64),
                ("heartbeat_interval", C.c_uint64), ("app_start", C.c_uint64),
                ("load", C.c_uint32), ("payload", C.c_uint32),
                ("path", C.c_void_p), ("path_ctx", C.c_void_p), ("root_dir", C.c_char_p),
                ("proc_peer", P(C.c_int32)), ("tcp_bytes", C.c_uint32), ("_pad3", C.c_uint32),
                ("quiet", C.c_int32), ("qdisc_rr", C.c_int32), ("mark_time", C.c_uint64 * 2),
                ("app_spec", P(C.c_uint32)), ("host_app", P(C.c_uint8)), ("app_peer", P(C.c_int32)),
                ("proc_app", P(C.c_int32))]


class Out(C.Structure):
    _fields_ = [("lines", C.c_char_p), ("len", C.c_size_t), ("cap", C.c_size_t), ("n_lines", C.c_uint64),
                ("ip", P(C.c_uint32)), ("next_event_id", P(C.c_uint64)), ("next_packet_id", P(C.c_uint64)),
                ("rng_probe", P(C.c_uint32)), ("mark_wall_s", C.c_double * 2)]


_lib = None


def available() -> bool:
    return os.path.exists(LIB)


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(LIB)
        _lib.ref_loop_run.argtypes = [P(Cfg), P(Out)]
        _lib.ref_loop_free.argtypes = [P(Out)]
    return _lib


def _ptr(a, ct):
    return None if a is None else a.ctypes.data_as(P(ct))


def run(model: S.ModelArrays, g: S.GraphArrays, host_start=None, procs=None, tcp=None, quiet=False, echo=None,
        marks=None, row_threads=0):
    """run_inproc in a forked child: the reference keeps process-wide state
    (the worker's thread-private object, glib quarks), so one run per process."""
    import multiprocessing as mp
    ctx = mp.get_context("fork")
    rd, wr = ctx.Pipe(duplex=False)

    def child():
        try:
            wr.send(("ok", run_inproc(model, g, host_start, procs, tcp, quiet, echo, marks, row_threads)))
        except BaseException as ex:   # noqa: BLE001 -- reported to the parent
            wr.send(("err", repr(ex)))
        wr.close()

    p = ctx.Process(target=child)
    p.start()
    wr.close()
    try:
        status, res = rd.recv()
    except EOFError:
        status, res = "err", "the reference loop's process died"
    p.join()
    if status != "ok":
        raise RuntimeError(res)
    return res


def run_inproc(model: S.ModelArrays, g: S.GraphArrays, host_start=None, procs=None, tcp=None, quiet=False,
               echo=None, marks=None, row_threads=0):
    """Run the model through the reference's loop; returns dict(lines=[(t, h, line)],
    ip=[str], next_event_id, next_packet_id, rng_probe (uint arrays)).
    host_start: [H] process start times (default: the model's app_start);
    procs: [(host, start)] processes in <process> order instead (the oracle's
    and the engine's pushed SHD_EV_APP_START events, in push order);
    tcp: dict(peers=[-1 | server process index per process], nbytes=N) runs
    the TCP echo test (test_tcp.c) in those processes instead of PHOLD; with
    apps=[-1 | index into specs per process], specs=[shd_udp_app-like
    (send, dest, n_start, per_read)] and app_peer=[H] the processes with an
    index run that datagram application instead (both transports in one model);
    echo: [H] -1 | server host runs the UDP request/response echo instead;
    marks: (t0, t1) simulated ns -> res["mark_wall_s"], the monotonic clock at
    the first send at or after each (the reference's own loop timed over a
    window); row_threads > 0: the path cache's rows computed on that many cores
    before the run (o_topo_precompute_rows), so the loop's time is the loop's."""
    m = model.struct
    H = int(m.n_hosts)
    og = O.lib().o_graph_new(C.byref(g.struct))
    hv = np.ctypeslib.as_array(m.host_vertex, shape=(H,)).copy()
    att = np.ascontiguousarray(np.unique(hv).astype(np.int32))
    topo = O.lib().o_topo_new(og, att.ctypes.data_as(P(C.c_int32)), len(att), 0)
    rows_s = 0.0
    if row_threads > 0:
        import time
        t0 = time.perf_counter()
        O.lib().o_topo_precompute_rows(topo, int(row_threads))
        rows_s = time.perf_counter() - t0
    keep = []
    cfg = Cfg()
    cfg.n_hosts = H
    cfg.quiet = 1 if quiet else 0
    cfg.app = 0 if tcp is None else 1
    if getattr(model, "app_specs", None) is not None:   # app 3: the model's per-host datagram applications
        cfg.app = 3
        sp = np.ascontiguousarray([[a.send, a.dest, a.n_start, a.per_read] for a in model.app_specs],
                                  dtype=np.uint32).ravel()
        keep.append(sp)
        cfg.app_spec = _ptr(sp, C.c_uint32)
        cfg.host_app = _ptr(model.host_app, C.c_uint8)
        if model.app_peer is not None:
            cfg.app_peer = _ptr(model.app_peer, C.c_int32)
    elif echo is not None:   # the UDP echo application: echo[h] = -1 (server) or h's server host
        cfg.app = 2
        ep = np.ascontiguousarray(echo, dtype=np.int32)
        keep.append(ep)
        cfg.proc_peer = _ptr(ep, C.c_int32)
    if tcp is not None:
        pp = np.ascontiguousarray(tcp["peers"], dtype=np.int32)
        keep.append(pp)
        cfg.proc_peer = _ptr(pp, C.c_int32)
        cfg.tcp_bytes = int(tcp.get("nbytes", 20000))
        cfg.qdisc_rr = int(tcp.get("qdisc", 0))
        if tcp.get("apps") is not None:
            pa = np.ascontiguousarray(tcp["apps"], dtype=np.int32)
            sp = np.ascontiguousarray([[int(x) for x in a] for a in tcp["specs"]], dtype=np.uint32).ravel()
            ap = np.ascontiguousarray(tcp["app_peer"], dtype=np.int32)
            keep += [pa, sp, ap]
            cfg.proc_app = _ptr(pa, C.c_int32)
            cfg.app_spec = _ptr(sp, C.c_uint32)
            cfg.app_peer = _ptr(ap, C.c_int32)
    cfg.host_seed = m.host_rng
    cfg.host_vertex = m.host_vertex
    cfg.bw_down_kibps = m.bw_down_kibps
    cfg.bw_up_kibps = m.bw_up_kibps
    cfg.dest_cum = m.dest_cum
    cfg.host_class = m.host_class
    cfg.n_classes = m.n_classes
    cfg.host_heartbeat = m.host_heartbeat
    if host_start is not None:
        hs = np.ascontiguousarray(host_start, dtype=np.uint64)
        keep.append(hs)
        cfg.host_start = _ptr(hs, C.c_uint64)
    if procs is not None:
        ph = np.ascontiguousarray([p[0] for p in procs], dtype=np.int32)
        ps = np.ascontiguousarray([p[1] for p in procs], dtype=np.uint64)
        keep += [ph, ps]
        cfg.n_procs = len(ph)
        cfg.proc_host = _ptr(ph, C.c_int32)
        cfg.proc_start = _ptr(ps, C.c_uint64)
    cfg.end_time = m.end_time
    cfg.bootstrap_end = m.bootstrap_end
    cfg.heartbeat_interval = m.heartbeat_interval
    cfg.app_start = m.app_start
    cfg.load = m.load
    cfg.payload = m.payload
    cfg.path = C.cast(O.lib().o_topo_get, C.c_void_p).value
    cfg.path_ctx = topo
    tmp = tempfile.mkdtemp(prefix="shd_ref_loop_")
    cfg.root_dir = tmp.encode()
    if marks is not None:
        cfg.mark_time[0], cfg.mark_time[1] = int(marks[0]), int(marks[1])
    out = Out()
    try:
        import time
        t0 = time.perf_counter()
        rc = lib().ref_loop_run(C.byref(cfg), C.byref(out))
        run_s = time.perf_counter() - t0
        assert rc == 0, rc
        text = C.string_at(out.lines, out.len).decode() if out.len else ""
        ips = [".".join(str((x >> s) & 255) for s in (24, 16, 8, 0))
               for x in np.ctypeslib.as_array(out.ip, shape=(H,))]
        by_ip = {ip: h for h, ip in enumerate(ips)}
        lines = []
        for ln in text.splitlines():
            t, h, body = ln.split("\t", 2)
            h = int(h)
            if h < 0 and " -> " in body:   # released outside any host's event: the deliver task's
                # packet, on its receiver (the host after "->")
                h = by_ip[body.split(" -> ")[1].split(":")[0]]
            if h >= 0:   # (the scheduler's own boot messages have no host)
                lines.append((int(t), h, body))
        res = dict(lines=lines, ip=ips,
                   next_event_id=np.ctypeslib.as_array(out.next_event_id, shape=(H,)).copy(),
                   next_packet_id=np.ctypeslib.as_array(out.next_packet_id, shape=(H,)).copy(),
                   rng_probe=np.ctypeslib.as_array(out.rng_probe, shape=(H,)).copy(), run_s=run_s,
                   mark_wall_s=(out.mark_wall_s[0], out.mark_wall_s[1]), rows_s=rows_s)
        lib().ref_loop_free(C.byref(out))
    finally:
        O.lib().o_topo_free(topo)
        O.lib().o_graph_free(og)
        shutil.rmtree(tmp, ignore_errors=True)
    return res
