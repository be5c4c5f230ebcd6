"""Python host driver over libshdgpu: path cache + engine handles.

This mirrors how Shadow's C host side would drive the C-ABI:
master/slave create the path cache from the topology (topology_new), hosts are
registered (seeds, attach, bandwidth), and the scheduler loop advances rounds.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

import shdgpu as S

SHD_PC_FORCE_ROWS = 1


class PathCache:
    def __init__(self, g: S.GraphArrays, attached, flags=0, device=0, build=True):
        self.g = g
        self.att = np.ascontiguousarray(attached, dtype=np.int32)
        self.ptr = C.c_void_p()
        S.check(S.lib().shd_pc_create(C.byref(g.struct), S.as_ptr(self.att, C.c_int32), len(self.att),
                                      flags, device, C.byref(self.ptr)), "shd_pc_create")
        if build:
            self.build()

    def build(self):
        S.check(S.lib().shd_pc_build(self.ptr), "shd_pc_build")

    def build_sharded(self, comm: "Comm"):
        """Source rows sharded over the communicator's ranks, then all-gathered."""
        S.check(S.lib().shd_pc_build_sharded(self.ptr, comm.ptr), "shd_pc_build_sharded")

    def info(self) -> S.PcInfo:
        i = S.PcInfo()
        S.check(S.lib().shd_pc_get_info(self.ptr, C.byref(i)), "shd_pc_get_info")
        return i

    def _table(self, fn, row0, nrows):
        T = len(self.att)
        lat = np.empty((nrows, T)); rel = np.empty((nrows, T))
        S.check(fn(self.ptr, row0, nrows, S.as_ptr(lat, C.c_double), S.as_ptr(rel, C.c_double)),
                "copy table")
        return lat, rel

    def rows(self, row0=0, nrows=None):
        n = len(self.att) - row0 if nrows is None else nrows
        return self._table(S.lib().shd_pc_copy_rows, row0, n)

    def direct(self, row0=0, nrows=None):
        n = len(self.att) - row0 if nrows is None else nrows
        return self._table(S.lib().shd_pc_copy_direct, row0, n)

    def self_values(self):
        T = len(self.att)
        lat = np.empty(T); rel = np.empty(T)
        S.check(S.lib().shd_pc_copy_self(self.ptr, S.as_ptr(lat, C.c_double), S.as_ptr(rel, C.c_double)),
                "copy self")
        return lat, rel

    def lookup(self, s, d):
        a, b = C.c_double(), C.c_double()
        S.check(S.lib().shd_pc_lookup(self.ptr, int(s), int(d), C.byref(a), C.byref(b)), "lookup")
        return a.value, b.value

    def lookup_batch(self, src, dst):
        """shd_pc_lookup of every (src[i], dst[i]) in order, in one call
        (shd_pc_lookup_batch): (lat, rel) arrays"""
        s = np.ascontiguousarray(src, dtype=np.int32)
        d = np.ascontiguousarray(dst, dtype=np.int32)
        lat = np.empty(len(s)); rel = np.empty(len(s))
        S.check(S.lib().shd_pc_lookup_batch(self.ptr, S.as_ptr(s, C.c_int32), S.as_ptr(d, C.c_int32), len(s),
                                            S.as_ptr(lat, C.c_double), S.as_ptr(rel, C.c_double)), "lookup_batch")
        return lat, rel

    def close(self):
        if self.ptr:
            S.lib().shd_pc_destroy(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Engine:
    """One engine = the hosts [host_begin, host_end) of a model on one GPU."""

    def __init__(self, model: S.ModelArrays, pc: PathCache, host_begin=0, host_end=None, device=0):
        self.model = model
        self.pc = pc
        self.h0 = int(host_begin)
        self.h1 = int(model.n_hosts if host_end is None else host_end)
        self.ptr = C.c_void_p()
        S.check(S.lib().shd_eng_create(C.byref(model.struct), pc.ptr, self.h0, self.h1, device,
                                       C.byref(self.ptr)), "shd_eng_create")

    @property
    def window(self) -> int:
        w = C.c_uint64()
        S.check(S.lib().shd_eng_window(self.ptr, C.byref(w)), "shd_eng_window")
        return w.value

    def boot(self):
        S.check(S.lib().shd_eng_boot(self.ptr), "shd_eng_boot")

    def push_events(self, events: np.ndarray):
        """shd_eng_push_events: caller-scheduled application starts, and packet
        deliveries from hosts the caller simulates (ingress), after boot."""
        ev = np.ascontiguousarray(events, dtype=S.EVENT_DTYPE)
        S.check(S.lib().shd_eng_push_events(self.ptr, ev.ctypes.data if len(ev) else None, len(ev)),
                "shd_eng_push_events")

    def run(self) -> S.RunStats:
        st = S.RunStats()
        rc = S.lib().shd_eng_run(self.ptr, C.byref(st))
        S.check(rc, f"shd_eng_run (error bits {st.error:#x})")
        return st

    def run_until(self, t_stop) -> S.RunStats:
        st = S.RunStats()
        rc = S.lib().shd_eng_run_until(self.ptr, int(t_stop), C.byref(st))
        S.check(rc, f"shd_eng_run_until (error bits {st.error:#x})")
        return st

    def run_round(self, ws, we) -> S.RoundSummary:
        r = S.RoundSummary()
        rc = S.lib().shd_eng_run_round(self.ptr, int(ws), int(we), C.byref(r))
        S.check(rc, f"shd_eng_run_round (error bits {r.error:#x})")
        return r

    # ---- phases of a round for multi-engine drivers (driver.py) ----
    def round_kernel(self, ws, we) -> S.RoundSummary:
        r = S.RoundSummary()
        S.check(S.lib().shd_eng_round_kernel(self.ptr, int(ws), int(we), C.byref(r)), "round_kernel")
        return r

    def round_begin(self, ws, we) -> S.RoundSummary:
        """round_kernel behind a state copy (shd_eng_round_begin)"""
        r = S.RoundSummary()
        S.check(S.lib().shd_eng_round_begin(self.ptr, int(ws), int(we), C.byref(r)), "shd_eng_round_begin")
        return r

    def round_retry(self, recs: np.ndarray) -> S.RoundSummary:
        """roll back to round_begin's copy, rank `recs`, run the window again"""
        recs = np.ascontiguousarray(recs, dtype=S.PENDING_DTYPE)
        r = S.RoundSummary()
        S.check(S.lib().shd_eng_round_retry(self.ptr, recs.ctypes.data if len(recs) else None, len(recs),
                                            C.byref(r)), "shd_eng_round_retry")
        return r

    def pending_records(self) -> np.ndarray:
        n = C.c_uint64()
        cap = 4096
        buf = np.empty(cap, dtype=S.PENDING_DTYPE)
        rc = S.lib().shd_eng_pending_copy(self.ptr, buf.ctypes.data, cap, C.byref(n))
        if rc == -34:   # ERANGE: more than cap
            buf = np.empty(n.value, dtype=S.PENDING_DTYPE)
            rc = S.lib().shd_eng_pending_copy(self.ptr, buf.ctypes.data, n.value, C.byref(n))
        S.check(rc, "shd_eng_pending_copy")
        return buf[:n.value]

    def resolve(self, recs: np.ndarray):
        recs = np.ascontiguousarray(recs, dtype=S.PENDING_DTYPE)
        S.check(S.lib().shd_eng_resolve(self.ptr, recs.ctypes.data if len(recs) else None, len(recs)),
                "shd_eng_resolve")

    def end_round(self) -> S.RoundSummary:
        r = S.RoundSummary()
        rc = S.lib().shd_eng_end_round(self.ptr, C.byref(r))
        S.check(rc, f"shd_eng_end_round (error bits {r.error:#x})")
        return r

    def remote_copy(self, dev_ptr: int, cap_events: int) -> int:
        n = C.c_uint64()
        S.check(S.lib().shd_eng_remote_copy(self.ptr, C.c_void_p(dev_ptr), int(cap_events), C.byref(n)),
                "shd_eng_remote_copy")
        return n.value

    def take_remote(self) -> np.ndarray:
        """shd_eng_take_remote: the last round's deliveries to hosts outside
        this engine (egress), as an EVENT_DTYPE array."""
        n = C.c_uint64()
        rc = S.lib().shd_eng_take_remote(self.ptr, None, 0, C.byref(n))
        if rc == -34:   # ERANGE: n holds the count
            out = np.empty(n.value, dtype=S.EVENT_DTYPE)
            rc = S.lib().shd_eng_take_remote(self.ptr, out.ctypes.data, n.value, C.byref(n))
            S.check(rc, "shd_eng_take_remote")
            return out[:n.value]
        S.check(rc, "shd_eng_take_remote")
        return np.empty(0, dtype=S.EVENT_DTYPE)

    def next_time(self) -> int:
        t = C.c_uint64()
        S.check(S.lib().shd_eng_next_time(self.ptr, C.byref(t)), "next_time")
        return t.value

    def trace(self) -> np.ndarray:
        n = C.c_uint64()
        S.check(S.lib().shd_eng_trace_count(self.ptr, C.byref(n)), "trace_count")
        out = np.empty(n.value, dtype=S.TRACE_DTYPE)
        got = C.c_uint64()
        if n.value:
            S.check(S.lib().shd_eng_trace_copy(self.ptr, out.ctypes.data, n.value, C.byref(got)),
                    "trace_copy")
        return out[:got.value] if n.value else out

    def digest(self) -> np.ndarray:
        out = np.empty(self.h1 - self.h0, dtype=S.DIGEST_DTYPE)
        S.check(S.lib().shd_eng_digest(self.ptr, out.ctypes.data), "digest")
        return out

    def remote(self):
        p = C.c_void_p(); n = C.c_uint64()
        S.check(S.lib().shd_eng_remote_buffer(self.ptr, C.byref(p), C.byref(n)), "remote_buffer")
        return p.value, n.value

    def heartbeats(self) -> np.ndarray:
        """[nloc, K, 2] uint32 cumulative interface packets (in, out) of each local host
        at its k-th heartbeat (SHD_QF_HEARTBEATS); S.tracker_node_lines formats them."""
        n = C.c_uint64()
        rc = S.lib().shd_eng_heartbeats(self.ptr, None, 0, C.byref(n))
        if rc not in (0, -34):
            S.check(rc, "shd_eng_heartbeats")
        out = np.zeros(n.value, dtype=np.uint32)
        if n.value:
            S.check(S.lib().shd_eng_heartbeats(self.ptr, out.ctypes.data_as(C.POINTER(C.c_uint32)), n.value,
                                               C.byref(n)), "shd_eng_heartbeats")
        nloc = self.h1 - self.h0
        return out.reshape(nloc, (n.value // (2 * nloc)) if nloc else 0, 2)

    def status_lines(self, ips, host_ids=None, listen_port=S.SHD_PHOLD_LISTEN_PORT) -> list:
        """[(time_ns, host, line)]: the [STATUS] lines of the engine's trace, made
        by the library (shd_eng_status_lines, packet.c:647-659)"""
        ip = S._ips_u32(ips)
        ids = None if host_ids is None else np.ascontiguousarray(np.asarray(host_ids, dtype=np.uint32))
        out = C.POINTER(S.Lines)()
        S.check(S.lib().shd_eng_status_lines(self.ptr, ip.ctypes.data_as(C.POINTER(C.c_uint32)),
                                             None if ids is None else ids.ctypes.data_as(C.POINTER(C.c_uint32)),
                                             int(listen_port), C.byref(out)), "shd_eng_status_lines")
        return S.take_lines(out)

    def node_lines(self, local_host: int) -> list:
        """[(time_ns, host, line)]: local host l's [shadow-heartbeat] lines, made by
        the library from its heartbeat counters (shd_eng_node_lines, tracker.c:419-465)"""
        out = C.POINTER(S.Lines)()
        S.check(S.lib().shd_eng_node_lines(self.ptr, int(local_host), C.byref(out)), "shd_eng_node_lines")
        return S.take_lines(out)

    def path_counts(self) -> np.ndarray:
        """[T, T] uint64 packet counts per cached path entry (SHD_QF_COUNT_PATHS)."""
        n = C.c_uint64()
        rc = S.lib().shd_eng_path_counts(self.ptr, None, 0, C.byref(n))
        if rc not in (0, -34):
            S.check(rc, "shd_eng_path_counts")
        out = np.zeros(n.value, dtype=np.uint64)
        S.check(S.lib().shd_eng_path_counts(self.ptr, out.ctypes.data_as(C.POINTER(C.c_uint64)), n.value,
                                            C.byref(n)), "shd_eng_path_counts")
        T = int(round(np.sqrt(n.value)))
        return out.reshape(T, T)

    def ingest(self, dev_ptr, n):
        S.check(S.lib().shd_eng_ingest(self.ptr, C.c_void_p(dev_ptr), int(n)), "ingest")

    def last_kernel_ms(self) -> float:
        v = C.c_double()
        S.check(S.lib().shd_eng_last_kernel_ms(self.ptr, C.byref(v)), "last_kernel_ms")
        return v.value

    def close(self):
        if self.ptr:
            S.lib().shd_eng_destroy(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Comm:
    """A group communicator (shd_comm): `rccl(uid, world, rank, device)` or
    `host(name, world, rank, device)` (processes of one machine, shared memory)."""

    def __init__(self, ptr):
        self.ptr = ptr

    @classmethod
    def rccl(cls, uid: bytes, world, rank, device=0):
        buf = (C.c_uint8 * S.SHD_XID_BYTES).from_buffer_copy(uid)
        ptr = C.c_void_p()
        S.check(S.lib().shd_comm_create_rccl(buf, int(world), int(rank), int(device), C.byref(ptr)),
                "shd_comm_create_rccl")
        return cls(ptr)

    @classmethod
    def host(cls, name: str, world, rank, device=0):
        ptr = C.c_void_p()
        S.check(S.lib().shd_comm_create_host(name.encode(), int(world), int(rank), int(device), C.byref(ptr)),
                "shd_comm_create_host")
        return cls(ptr)

    def close(self):
        if self.ptr:
            S.lib().shd_comm_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class XGroup:
    """Engines stepping rounds together with one fixed-size all-to-all per
    round (shd_xgroup, DESIGN.md "Multi-GPU").  `local(engines)`: all engines
    in this process (device-to-device copies); `rccl(engine, uid, world,
    rank)`: one engine per process over RCCL (uid from `unique_id()` on rank 0,
    shared by every rank)."""

    def __init__(self, ptr, engines):
        self.ptr = ptr
        self.engines = engines

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * S.SHD_XID_BYTES)()
        S.check(S.lib().shd_xgroup_unique_id(buf), "shd_xgroup_unique_id")
        return bytes(buf)

    @classmethod
    def local(cls, engines, block_events=0):
        arr = (C.c_void_p * len(engines))(*[e.ptr.value for e in engines])
        ptr = C.c_void_p()
        S.check(S.lib().shd_xgroup_create_local(arr, len(engines), int(block_events), C.byref(ptr)),
                "shd_xgroup_create_local")
        return cls(ptr, list(engines))

    @classmethod
    def rccl(cls, engine, uid: bytes, world, rank, block_events=0):
        buf = (C.c_uint8 * S.SHD_XID_BYTES).from_buffer_copy(uid)
        ptr = C.c_void_p()
        S.check(S.lib().shd_xgroup_create_rccl(engine.ptr, buf, int(world), int(rank), int(block_events),
                                               C.byref(ptr)), "shd_xgroup_create_rccl")
        return cls(ptr, [engine])

    @classmethod
    def over(cls, engine, comm: Comm, block_events=0, p2p=False):
        """One engine of this process in a group over a communicator; p2p: the
        peer-to-peer transport (receive blocks mapped by IPC handle, stored
        into directly), else the communicator's all-to-all."""
        ptr = C.c_void_p()
        fn = "shd_xgroup_create_p2p" if p2p else "shd_xgroup_create"
        S.check(getattr(S.lib(), fn)(engine.ptr, comm.ptr, int(block_events), C.byref(ptr)), fn)
        g = cls(ptr, [engine])
        g.p2p = p2p
        return g

    def run_until(self, t_stop) -> S.RunStats:
        st = S.RunStats()
        rc = S.lib().shd_xgroup_run_until(self.ptr, int(t_stop), C.byref(st))
        S.check(rc, f"shd_xgroup_run_until (error bits {st.error:#x})")
        return st

    def run(self) -> S.RunStats:
        return self.run_until(self.engines[0].model.params["end_time"])

    def next_time(self) -> int:
        t = C.c_uint64()
        S.check(S.lib().shd_xgroup_next_time(self.ptr, C.byref(t)), "shd_xgroup_next_time")
        return t.value

    def close(self):
        if self.ptr:
            S.lib().shd_xgroup_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def sort_trace(tr: np.ndarray) -> np.ndarray:
    """Canonical order for multiset comparison of traces."""
    return np.sort(tr, order=["time", "host", "kind", "peer", "pkt", "seq"])
