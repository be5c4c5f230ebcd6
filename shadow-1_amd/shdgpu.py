"""ctypes binding of libshdgpu (include/shdgpu.h).

This is the Python mirror of the C-ABI a Shadow maintainer would bind (see
INTEGRATION.md).  It loads the in-tree ``libshdgpu.so`` built by
``__graft_entry__.build()`` and fails loudly when it is missing: there is no
CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SHDGPU_LIB") or os.path.join(HERE, "libshdgpu.so")   # override: profiling build

SHD_XID_BYTES = 128
SHD_MS = 1_000_000
SHD_SEC = 1_000_000_000
SHD_MTU = 1500
SHD_HEADER_UDP = 42
SHD_QF_NO_CALENDAR = 1      # queue_flags: every inter-host event through inbox + heap
SHD_QF_COUNT_PATHS = 2      # queue_flags: per-path packet counters on the device
SHD_QF_HEARTBEATS = 4       # queue_flags: tracker node counters at every heartbeat
SHD_QF_NO_APP_START = 8     # queue_flags: the caller pushes the application starts (shd_eng_push_events)
SHD_QF_TRACE_STATUS = 16    # queue_flags: with trace, the application's records too (status_lines)
ERR_AMBIGUOUS = 16          # shd_round_summary.error: an ambiguous first-touch drop decision (SHD_ERR_AMBIGUOUS)
SHD_PHOLD_LISTEN_PORT = 8998   # PHOLD_LISTEN_PORT, test_phold.c:34
SHD_MIN_RANDOM_PORT = 10000    # MIN_RANDOM_PORT, definitions.h:94

EV_HEARTBEAT, EV_REFILL, EV_REFILL_LO, EV_APP_START, EV_PACKET, EV_LOCAL, EV_NOTIFY = range(1, 8)
TR_SENT, TR_INET_DROP, TR_ARRIVE, TR_CODEL_DROP, TR_RECV, TR_IF_DROP, TR_LOCAL, TR_CREATED, TR_READ = range(1, 10)

ERRORS = {
    0: "ok", -22: "EINVAL", -12: "ENOMEM", -19: "ENODEV", -75: "EOVERFLOW",
    -34: "ERANGE", -125: "EAMBIG", -107: "ENOTCONN",
}


class ShdError(RuntimeError):
    pass


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        raise ShdError(f"{what} failed: {rc} ({ERRORS.get(rc, '?')})")


P = C.POINTER


class Graph(C.Structure):
    _fields_ = [
        ("n_vertices", C.c_int32), ("n_edges", C.c_int32),
        ("directed", C.c_int32), ("prefer_direct", C.c_int32),
        ("edge_src", P(C.c_int32)), ("edge_dst", P(C.c_int32)),
        ("edge_latency", P(C.c_double)), ("edge_loss", P(C.c_double)),
        ("vertex_loss", P(C.c_double)),
    ]


class GraphProps(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "is_connected", "is_complete", "is_directed", "prefer_direct", "n_self_loops",
        "max_out_degree")]


class ConfigHost(C.Structure):
    _fields_ = [("name", C.c_char_p), ("ip_hint", C.c_char_p), ("citycode_hint", C.c_char_p),
                ("countrycode_hint", C.c_char_p), ("geocode_hint", C.c_char_p), ("type_hint", C.c_char_p),
                ("bw_down_kibps", C.c_uint64), ("bw_up_kibps", C.c_uint64), ("heartbeat_s", C.c_uint64),
                ("n_processes", C.c_int32), ("_pad", C.c_int32), ("process_start_s", C.POINTER(C.c_uint64))]


class Config(C.Structure):
    _fields_ = [("n_hosts", C.c_int32), ("hosts", C.POINTER(ConfigHost)), ("stop_time_s", C.c_uint64),
                ("bootstrap_time_s", C.c_uint64), ("topology_path", C.c_char_p), ("topology_text", C.c_char_p)]


class GraphML(C.Structure):
    _fields_ = [
        ("g", Graph), ("bw_down", P(C.c_double)), ("bw_up", P(C.c_double)),
        ("vertex_id", P(C.c_char_p)), ("vertex_ip", P(C.c_char_p)),
        ("vertex_citycode", P(C.c_char_p)), ("vertex_countrycode", P(C.c_char_p)),
        ("vertex_geocode", P(C.c_char_p)), ("vertex_type", P(C.c_char_p)),
        ("edge_jitter", P(C.c_double)),
    ]


class PcInfo(C.Structure):
    _fields_ = [
        ("n_vertices", C.c_int32), ("n_attached", C.c_int32), ("is_complete", C.c_int32),
        ("is_directed", C.c_int32), ("prefer_direct", C.c_int32), ("rows_computed", C.c_int32),
        ("n_ties", C.c_int64), ("max_hops", C.c_int32), ("sssp_iterations_max", C.c_int32),
        ("n_unroutable", C.c_int32), ("min_latency_ms", C.c_double),
        ("build_ms_device", C.c_double), ("build_ms_sssp", C.c_double),
        ("build_ms_props", C.c_double), ("build_ms_direct", C.c_double),
        ("n_tie_rows", C.c_int32), ("n_tie_rows_global", C.c_int32),
        ("n_tie_rows_predicted", C.c_int32), ("_pad0", C.c_int32),
    ]


class UdpApp(C.Structure):
    """shd_udp_app (include/shdgpu.h): one host's datagram application."""
    _fields_ = [("send", C.c_uint32), ("dest", C.c_uint32), ("n_start", C.c_uint32), ("per_read", C.c_uint32)]


class Model(C.Structure):
    _fields_ = [
        ("n_hosts", C.c_int32), ("_pad0", C.c_int32),
        ("host_vertex", P(C.c_int32)), ("host_rng", P(C.c_uint32)),
        ("bw_down_kibps", P(C.c_uint64)), ("bw_up_kibps", P(C.c_uint64)),
        ("dest_cum", P(C.c_double)),
        ("end_time", C.c_uint64), ("bootstrap_end", C.c_uint64),
        ("heartbeat_interval", C.c_uint64), ("app_start", C.c_uint64),
        ("load", C.c_uint32), ("payload", C.c_uint32), ("trace", C.c_uint32),
        ("evq_cap", C.c_uint32), ("inbox_cap", C.c_uint32), ("codelq_cap", C.c_uint32),
        ("txq_cap", C.c_uint32), ("queue_flags", C.c_uint32),
        ("host_class", P(C.c_uint8)), ("n_classes", C.c_int32), ("_pad1", C.c_int32),
        ("host_heartbeat", P(C.c_uint64)),
        ("app", C.c_uint32), ("_pad2", C.c_int32), ("app_peer", P(C.c_int32)),
        ("app_spec", P(UdpApp)), ("host_app", P(C.c_uint8)), ("n_app_specs", C.c_uint32), ("_pad3", C.c_uint32),
    ]


SHD_APP_PHOLD, SHD_APP_UDP_ECHO, SHD_APP_UDP = 0, 1, 2
SHD_SEND_EACH, SHD_SEND_ONCE, SHD_SEND_LISTENER = 0, 1, 2
SHD_DEST_WEIGHTED, SHD_DEST_PEER, SHD_DEST_REPLY = 0, 1, 2


class Event(C.Structure):
    _fields_ = [("time", C.c_uint64), ("seq", C.c_uint64), ("src", C.c_uint32),
                ("dst", C.c_uint32), ("pkt", C.c_uint32), ("kind", C.c_uint32)]


class TraceRec(C.Structure):
    _fields_ = [("time", C.c_uint64), ("seq", C.c_uint64), ("host", C.c_uint32),
                ("peer", C.c_uint32), ("pkt", C.c_uint32), ("kind", C.c_uint32)]


TRACE_DTYPE = np.dtype([("time", "<u8"), ("seq", "<u8"), ("host", "<u4"), ("peer", "<u4"),
                        ("pkt", "<u4"), ("kind", "<u4")])


class HostDigest(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "ev_seq", "rx_remaining", "tx_remaining", "codel_total", "codel_interval_expire",
        "codel_next_drop", "n_events", "n_pkt_events", "n_sent", "n_inet_drop",
        "n_codel_drop", "n_recv")] + [(n, C.c_uint32) for n in (
            "rng", "pkt_seq", "codel_mode", "codel_count", "codel_drop_count",
            "codel_drop_count_last", "unread", "flags")]


DIGEST_DTYPE = np.dtype([(n, "<u8") for n in (
    "ev_seq", "rx_remaining", "tx_remaining", "codel_total", "codel_interval_expire",
    "codel_next_drop", "n_events", "n_pkt_events", "n_sent", "n_inet_drop", "n_codel_drop",
    "n_recv")] + [(n, "<u4") for n in ("rng", "pkt_seq", "codel_mode", "codel_count",
                                      "codel_drop_count", "codel_drop_count_last", "unread",
                                      "flags")])
assert DIGEST_DTYPE.itemsize == C.sizeof(HostDigest)
assert TRACE_DTYPE.itemsize == C.sizeof(TraceRec) == 32
assert C.sizeof(Event) == 32


PENDING_DTYPE = np.dtype([("qtime", "<u8"), ("qseq", "<u8"), ("qhost", "<u4"), ("qsrc", "<u4"),
                          ("qsub", "<u4"), ("a", "<u4"), ("b", "<u4"), ("delivered", "<u4"),
                          ("dst", "<u4"), ("pkt", "<u4"), ("seq", "<u8")])
assert PENDING_DTYPE.itemsize == 56
EVENT_DTYPE = np.dtype([("time", "<u8"), ("seq", "<u8"), ("src", "<u4"), ("dst", "<u4"),
                        ("pkt", "<u4"), ("kind", "<u4")])


class RoundSummary(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "window_start", "window_end", "next_time", "n_events", "n_pkt_events", "n_pending",
        "n_remote")] + [("error", C.c_uint32), ("_pad", C.c_uint32)]


class RunStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "n_rounds", "n_events", "n_pkt_events", "n_pending_resolved", "window_ns",
        "final_time")] + [("device_ms_round_kernel", C.c_double), ("wall_ms", C.c_double),
                          ("device_ms_launches", C.c_double), ("error", C.c_uint32),
                          ("n_batches_ticketless", C.c_uint32), ("n_rounds_protected", C.c_uint32),
                          ("n_rounds_rerun", C.c_uint32), ("n_host_rounds", C.c_uint64),
                          ("n_batches", C.c_uint64), ("n_batches_persistent", C.c_uint64),
                          ("n_batches_sparse", C.c_uint64), ("n_rounds_replayed", C.c_uint64),
                         ("n_restore_points", C.c_uint64)]


# exported symbols (checked by tests/test_abi.py against include/shdgpu.h)
class TcpModel(C.Structure):
    """shd_tcp_model (include/shdtcp.h)"""
    _fields_ = [("n_hosts", C.c_int32), ("n_procs", C.c_int32),
                ("host_ip", P(C.c_uint32)), ("host_seed", P(C.c_uint32)),
                ("bw_down_kibps", P(C.c_uint64)), ("bw_up_kibps", P(C.c_uint64)),
                ("n_vertices", C.c_int32), ("host_vertex", P(C.c_int32)),
                ("path_lat_ms", P(C.c_double)), ("path_rel", P(C.c_double)),
                ("proc_host", P(C.c_int32)), ("proc_start", P(C.c_uint64)), ("proc_peer", P(C.c_int32)),
                ("end_time", C.c_uint64), ("heartbeat_interval", C.c_uint64),
                ("tcp_bytes", C.c_uint32), ("recv_buf", C.c_uint32), ("send_buf", C.c_uint32),
                ("tcp_window", C.c_uint32), ("packets_per_host", C.c_uint32), ("qdisc", C.c_uint32),
                ("_pad", C.c_uint32), ("path_cache", C.c_void_p),
                ("proc_app", P(C.c_int32)), ("app_spec", P(C.c_uint32)), ("n_app_specs", C.c_int32),
                ("udp_payload", C.c_uint32), ("app_peer", P(C.c_int32)), ("dest_cum", P(C.c_double)),
                ("host_class", P(C.c_uint8)), ("n_classes", C.c_int32), ("_pad2", C.c_int32)]


class TcpResult(C.Structure):
    """shd_tcp_result (include/shdtcp.h)"""
    _fields_ = [("lines", C.c_void_p), ("len", C.c_size_t), ("n_lines", C.c_uint64),
                ("next_event_id", P(C.c_uint64)), ("next_packet_id", P(C.c_uint64)),
                ("rng_probe", P(C.c_uint32)), ("rounds", C.c_uint64), ("events", C.c_uint64),
                ("device_ms", C.c_double), ("error", C.c_uint32), ("deliveries", C.c_uint64),
                ("queries", C.c_void_p), ("n_queries", C.c_uint64),
                ("node_counters", P(C.c_uint64)), ("n_heartbeats", P(C.c_uint32)), ("node_k", C.c_uint32),
                ("first_touch_reruns", C.c_uint32), ("max_round_deliveries", C.c_uint64), ("max_round_overflow", C.c_uint64),
                ("setup_ms", C.c_double), ("results_ms", C.c_double), ("teardown_ms", C.c_double),
                ("first_host", C.c_int32), ("n_local_hosts", C.c_int32)]


TCP_TRACE_STATUS, TCP_TRACE_NODE = 1, 2   # shd_tcp_run's trace bits
TCP_ERR_FIRST_TOUCH = 512                  # SHD_TCP_ERR_FIRST_TOUCH (include/shdtcp.h)


TCP_QUERY_DTYPE = np.dtype([("time", "<u8"), ("seq", "<u8"), ("host", "<u4"), ("src", "<u4"), ("index", "<u4"),
                            ("v_src", "<i4"), ("v_dst", "<i4"), ("_pad", "<u4")])   # shd_tcp_query


class Lines(C.Structure):
    """shd_lines (include/shdgpu.h): line i is text[off[i]:off[i+1]], logged at
    time[i] by host[i]"""
    _fields_ = [("n", C.c_uint64), ("time", C.POINTER(C.c_uint64)), ("host", C.POINTER(C.c_uint32)),
                ("off", C.POINTER(C.c_uint64)), ("text", C.c_void_p)]


_SIGS = {
    "shd_tcp_run": (C.c_int, [P(TcpModel), C.c_int32, P(P(TcpResult))]),
    "shd_tcp_run_group": (C.c_int, [P(TcpModel), C.c_void_p, C.c_int32, P(P(TcpResult))]),
    "shd_tcp_result_free": (None, [P(TcpResult)]),
    "shd_tcp_keep_workspace": (None, [C.c_int32]),
    "shd_tracker_node_lines": (C.c_int, [P(C.c_uint64), C.c_uint64, C.c_uint64, C.c_uint32, P(P(Lines))]),
    "shd_graph_check": (C.c_int, [P(Graph), P(GraphProps)]),
    "shd_graphml_load_file": (C.c_int, [C.c_char_p, P(P(GraphML))]),
    "shd_graphml_load_string": (C.c_int, [C.c_char_p, C.c_size_t, P(P(GraphML))]),
    "shd_config_load_file": (C.c_int, [C.c_char_p, P(P(Config))]),
    "shd_config_load_buffer": (C.c_int, [C.c_char_p, C.c_size_t, P(P(Config))]),
    "shd_config_free": (None, [P(Config)]),
    "shd_dns_assign": (C.c_int, [P(Config), P(C.c_uint32)]),
    "shd_graphml_free": (None, [P(GraphML)]),
    "shd_pc_create": (C.c_int, [P(Graph), P(C.c_int32), C.c_int32, C.c_uint32, C.c_int,
                                P(C.c_void_p)]),
    "shd_pc_build": (C.c_int, [C.c_void_p]),
    "shd_pc_get_info": (C.c_int, [C.c_void_p, P(PcInfo)]),
    "shd_pc_copy_rows": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, P(C.c_double),
                                   P(C.c_double)]),
    "shd_pc_copy_direct": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, P(C.c_double),
                                     P(C.c_double)]),
    "shd_pc_copy_self": (C.c_int, [C.c_void_p, P(C.c_double), P(C.c_double)]),
    "shd_pc_lookup": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, P(C.c_double),
                                P(C.c_double)]),
    "shd_pc_lookup_batch": (C.c_int, [C.c_void_p, P(C.c_int32), P(C.c_int32), C.c_uint64, P(C.c_double),
                                      P(C.c_double)]),
    "shd_pc_count_packet": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    "shd_pc_packet_count": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, P(C.c_uint64)]),
    "shd_pc_min_time_jump": (C.c_int, [C.c_void_p, C.c_uint64, P(C.c_uint64)]),
    "shd_pc_min_stored_latency": (C.c_int, [C.c_void_p, P(C.c_double)]),
    "shd_pc_destroy": (None, [C.c_void_p]),
    "shd_rand_r": (C.c_int32, [P(C.c_uint32)]),
    "shd_next_double": (C.c_double, [P(C.c_uint32)]),
    "shd_next_uint": (C.c_uint32, [P(C.c_uint32)]),
    "shd_seed_chain": (C.c_int, [C.c_uint32, C.c_int32, P(C.c_uint32)]),
    "shd_topology_attach": (C.c_int, [P(GraphML), P(C.c_uint32), C.c_char_p, C.c_char_p,
                                      C.c_char_p, C.c_char_p, C.c_char_p, P(C.c_int32),
                                      P(C.c_uint64), P(C.c_uint64)]),
    "shd_topology_attach_cb": (C.c_int, [P(GraphML), C.c_void_p, C.c_void_p, C.c_char_p, C.c_char_p,
                                         C.c_char_p, C.c_char_p, C.c_char_p, P(C.c_int32),
                                         P(C.c_uint64), P(C.c_uint64)]),
    "shd_eng_create": (C.c_int, [P(Model), C.c_void_p, C.c_int32, C.c_int32, C.c_int,
                                 P(C.c_void_p)]),
    "shd_eng_window": (C.c_int, [C.c_void_p, P(C.c_uint64)]),
    "shd_eng_boot": (C.c_int, [C.c_void_p]),
    "shd_eng_push_events": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "shd_eng_run_round": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, P(RoundSummary)]),
    "shd_eng_run": (C.c_int, [C.c_void_p, P(RunStats)]),
    "shd_eng_run_until": (C.c_int, [C.c_void_p, C.c_uint64, P(RunStats)]),
    "shd_eng_round_kernel": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, P(RoundSummary)]),
    "shd_eng_pending_copy": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, P(C.c_uint64)]),
    "shd_eng_resolve": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "shd_eng_round_begin": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p]),
    "shd_pc_defer_touches": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "shd_pc_query_key": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64]),
    "shd_pc_take_touches": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, P(C.c_uint64)]),
    "shd_eng_round_retry": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    "shd_eng_end_round": (C.c_int, [C.c_void_p, P(RoundSummary)]),
    "shd_eng_remote_copy": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, P(C.c_uint64)]),
    "shd_eng_take_remote": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, P(C.c_uint64)]),
    "shd_eng_ingest": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "shd_eng_next_time": (C.c_int, [C.c_void_p, P(C.c_uint64)]),
    "shd_eng_trace_count": (C.c_int, [C.c_void_p, P(C.c_uint64)]),
    "shd_eng_trace_copy": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, P(C.c_uint64)]),
    "shd_eng_digest": (C.c_int, [C.c_void_p, C.c_void_p]),
    "shd_eng_path_counts": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_uint64, P(C.c_uint64)]),
    "shd_eng_heartbeats": (C.c_int, [C.c_void_p, P(C.c_uint32), C.c_uint64, P(C.c_uint64)]),
    "shd_eng_stream": (C.c_int, [C.c_void_p, P(C.c_void_p)]),
    "shd_status_lines": (C.c_int, [C.c_void_p, C.c_uint64, P(C.c_uint32), P(C.c_uint32), C.c_uint32, C.c_uint32,
                                   C.c_uint32, P(C.c_int32), P(P(Lines))]),
    "shd_node_lines": (C.c_int, [P(C.c_uint32), C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, P(P(Lines))]),
    "shd_eng_status_lines": (C.c_int, [C.c_void_p, P(C.c_uint32), P(C.c_uint32), C.c_uint32, P(P(Lines))]),
    "shd_eng_node_lines": (C.c_int, [C.c_void_p, C.c_uint32, P(P(Lines))]),
    "shd_lines_free": (None, [P(Lines)]),
    "shd_eng_last_kernel_ms": (C.c_int, [C.c_void_p, P(C.c_double)]),
    "shd_eng_destroy": (None, [C.c_void_p]),
    "shd_version": (C.c_char_p, []),
    "shd_device_count": (C.c_int, [P(C.c_int)]),
    "shd_xgroup_unique_id": (C.c_int, [P(C.c_uint8)]),
    "shd_xgroup_create_rccl": (C.c_int, [C.c_void_p, P(C.c_uint8), C.c_int, C.c_int, C.c_uint32,
                                         P(C.c_void_p)]),
    "shd_xgroup_create_local": (C.c_int, [P(C.c_void_p), C.c_int, C.c_uint32, P(C.c_void_p)]),
    "shd_xgroup_run_until": (C.c_int, [C.c_void_p, C.c_uint64, P(RunStats)]),
    "shd_xgroup_create": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, P(C.c_void_p)]),
    "shd_xgroup_create_p2p": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, P(C.c_void_p)]),
    "shd_comm_create_rccl": (C.c_int, [P(C.c_uint8), C.c_int, C.c_int, C.c_int, P(C.c_void_p)]),
    "shd_comm_create_host": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, P(C.c_void_p)]),
    "shd_comm_rank": (C.c_int, [C.c_void_p, P(C.c_int), P(C.c_int)]),
    "shd_comm_destroy": (None, [C.c_void_p]),
    "shd_pc_build_sharded": (C.c_int, [C.c_void_p, C.c_void_p]),
    "shd_xgroup_next_time": (C.c_int, [C.c_void_p, P(C.c_uint64)]),
    "shd_xgroup_destroy": (None, [C.c_void_p]),
}

_lib = None


def engine_source_sha1() -> str:
    """SHA-1 over the engine's translation unit (csrc/engine.hip and its parts):
    the key under which profiles (PMC traffic) of this source are recorded."""
    import hashlib
    h = hashlib.sha1()
    d = os.path.join(HERE, "csrc")
    for f in ("engine.hip", "eng_device.h", "eng_round.h", "eng_exchange.h", "eng_group.h", "shd_device.h"):
        h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()


def lib() -> C.CDLL:
    """Load libshdgpu.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ShdError(f"{LIB_PATH} missing: run __graft_entry__.build() first "
                           "(there is no CPU fallback)")
        # One HIP runtime per process: the torch wheel bundles its own
        # libamdhip64.so.7.  Loading torch first makes libshdgpu's NEEDED
        # libamdhip64.so.7 resolve to that same copy (same SONAME), so device
        # pointers can flow between torch tensors (RCCL exchange) and libshdgpu.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        l = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def exported_symbols() -> list[str]:
    return sorted(_SIGS)


def as_ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(P(ctype))


# ----------------------------------------------------------------- helpers
class GraphArrays:
    """Owns the numpy arrays behind a ``Graph`` struct (document order)."""

    def __init__(self, n_vertices, src, dst, latency, loss, vertex_loss=None,
                 directed=False, prefer_direct=False):
        self.n_vertices = int(n_vertices)
        self.src = np.ascontiguousarray(src, dtype=np.int32)
        self.dst = np.ascontiguousarray(dst, dtype=np.int32)
        self.latency = np.ascontiguousarray(latency, dtype=np.float64)
        self.loss = np.ascontiguousarray(loss, dtype=np.float64)
        self.vertex_loss = (None if vertex_loss is None else
                            np.ascontiguousarray(vertex_loss, dtype=np.float64))
        self.directed = bool(directed)
        self.prefer_direct = bool(prefer_direct)
        self.struct = Graph(
            self.n_vertices, len(self.src), int(self.directed), int(self.prefer_direct),
            as_ptr(self.src, C.c_int32), as_ptr(self.dst, C.c_int32),
            as_ptr(self.latency, C.c_double), as_ptr(self.loss, C.c_double),
            None if self.vertex_loss is None else as_ptr(self.vertex_loss, C.c_double))

    @property
    def n_edges(self):
        return len(self.src)


def load_config(xml: bytes):
    """shadow.config.xml -> (hosts: list of dicts in registration order,
    ips: host-order uint32 array from shd_dns_assign, stop_time_s, topology text or path)."""
    ptr = P(Config)()
    check(lib().shd_config_load_buffer(xml, len(xml), C.byref(ptr)), "shd_config_load_buffer")
    try:
        c = ptr.contents
        dec = lambda b: None if b is None else b.decode()  # noqa: E731
        hosts = [dict(name=dec(h.name), ip_hint=dec(h.ip_hint), citycode_hint=dec(h.citycode_hint),
                      countrycode_hint=dec(h.countrycode_hint), geocode_hint=dec(h.geocode_hint),
                      type_hint=dec(h.type_hint), bw_down_kibps=h.bw_down_kibps, bw_up_kibps=h.bw_up_kibps,
                      heartbeat_s=h.heartbeat_s,
                      process_start_s=[h.process_start_s[k] for k in range(h.n_processes)])
                 for h in (c.hosts[i] for i in range(c.n_hosts))]
        ips = np.zeros(max(c.n_hosts, 1), dtype=np.uint32)
        check(lib().shd_dns_assign(ptr, ips.ctypes.data_as(P(C.c_uint32))), "shd_dns_assign")
        topo = dec(c.topology_text) if c.topology_text else dec(c.topology_path)
        return hosts, ips[:c.n_hosts], c.stop_time_s, topo
    finally:
        lib().shd_config_free(ptr)


def ip_str(ip: int) -> str:
    ip = int(ip)
    return "%d.%d.%d.%d" % (ip >> 24, (ip >> 16) & 255, (ip >> 8) & 255, ip & 255)


def graph_from_graphml(gm_ptr) -> GraphArrays:
    gm = gm_ptr.contents
    g = gm.g
    V, E = g.n_vertices, g.n_edges
    src = np.ctypeslib.as_array(g.edge_src, (E,)).copy()
    dst = np.ctypeslib.as_array(g.edge_dst, (E,)).copy()
    lat = np.ctypeslib.as_array(g.edge_latency, (E,)).copy()
    loss = np.ctypeslib.as_array(g.edge_loss, (E,)).copy()
    vl = np.ctypeslib.as_array(g.vertex_loss, (V,)).copy() if g.vertex_loss else None
    return GraphArrays(V, src, dst, lat, loss, vl, bool(g.directed), bool(g.prefer_direct))


class ModelArrays:
    """Owns the numpy arrays behind a ``Model`` struct."""

    def __init__(self, host_vertex, host_rng, bw_down, bw_up, dest_cum, *, end_time,
                 app_start=1 * SHD_SEC, load=16, payload=1, heartbeat_interval=SHD_SEC,
                 bootstrap_end=0, trace=False, evq_cap=0, inbox_cap=0, codelq_cap=0,
                 txq_cap=0, queue_flags=0, host_class=None, host_heartbeat=None, app_peer=None,
                 app_specs=None, host_app=None):
        """dest_cum: [H] (one weights row for every host) or [n_classes, H] with
        host_class [H] picking each host's row; host_heartbeat: [H] ns or None;
        app_peer: None (every host runs PHOLD) or [H] -1 | server host (every
        host runs the UDP request/response echo, SHD_APP_UDP_ECHO);
        app_specs: [(send, dest, n_start, per_read)] with host_app [H] picking
        each host's (SHD_APP_UDP, include/shdgpu.h shd_udp_app; app_peer then
        names the SHD_DEST_PEER hosts' peers)."""
        self.host_vertex = np.ascontiguousarray(host_vertex, dtype=np.int32)
        self.host_rng = np.ascontiguousarray(host_rng, dtype=np.uint32)
        self.bw_down = np.ascontiguousarray(bw_down, dtype=np.uint64)
        self.bw_up = np.ascontiguousarray(bw_up, dtype=np.uint64)
        self.dest_cum = np.ascontiguousarray(dest_cum, dtype=np.float64)
        H = len(self.host_vertex)
        n_classes = 1 if self.dest_cum.ndim == 1 else self.dest_cum.shape[0]
        assert all(len(a) == H for a in (self.host_rng, self.bw_down, self.bw_up))
        assert self.dest_cum.shape[-1] == H
        self.host_class = None if host_class is None else np.ascontiguousarray(host_class, dtype=np.uint8)
        assert n_classes == 1 or (self.host_class is not None and len(self.host_class) == H)
        self.n_classes = n_classes
        self.host_heartbeat = None if host_heartbeat is None else \
            np.ascontiguousarray(host_heartbeat, dtype=np.uint64)
        self.app_peer = None if app_peer is None else np.ascontiguousarray(app_peer, dtype=np.int32)
        assert self.app_peer is None or len(self.app_peer) == H
        self.app = SHD_APP_PHOLD if self.app_peer is None else SHD_APP_UDP_ECHO
        self.app_specs = None
        self.host_app = None
        # the status writer's port rule: >= 0 for a host that reads on the
        # socket it sends from (the echo's clients, SHD_SEND_ONCE), else -1
        self.status_peer = self.app_peer
        if app_specs is not None:
            assert host_app is not None and len(host_app) == H and 0 < len(app_specs) <= 256
            self.app = SHD_APP_UDP
            self.app_specs = (UdpApp * len(app_specs))(*[UdpApp(*map(int, a)) for a in app_specs])
            self.host_app = np.ascontiguousarray(host_app, dtype=np.uint8)
            once = np.array([int(a[0]) == SHD_SEND_ONCE for a in app_specs], dtype=bool)
            self.status_peer = np.where(once[self.host_app], 0, -1).astype(np.int32)
        self.params = dict(end_time=int(end_time), app_start=int(app_start), load=int(load),
                           payload=int(payload), heartbeat_interval=int(heartbeat_interval),
                           bootstrap_end=int(bootstrap_end), trace=int(bool(trace)),
                           queue_flags=int(queue_flags))
        self.struct = Model(
            H, 0, as_ptr(self.host_vertex, C.c_int32), as_ptr(self.host_rng, C.c_uint32),
            as_ptr(self.bw_down, C.c_uint64), as_ptr(self.bw_up, C.c_uint64),
            as_ptr(self.dest_cum, C.c_double), int(end_time), int(bootstrap_end),
            int(heartbeat_interval), int(app_start), int(load), int(payload), int(bool(trace)),
            int(evq_cap), int(inbox_cap), int(codelq_cap), int(txq_cap), int(queue_flags),
            None if self.host_class is None else as_ptr(self.host_class, C.c_uint8), int(n_classes), 0,
            None if self.host_heartbeat is None else as_ptr(self.host_heartbeat, C.c_uint64),
            self.app, 0, None if self.app_peer is None else as_ptr(self.app_peer, C.c_int32),
            None if self.app_specs is None else C.cast(self.app_specs, P(UdpApp)),
            None if self.host_app is None else as_ptr(self.host_app, C.c_uint8),
            0 if self.app_specs is None else len(self.app_specs), 0)

    @property
    def n_hosts(self):
        return len(self.host_vertex)


# ---- tracker heartbeat lines (host/tracker.c) ----
SHD_HEADER_UDP = 42          # definitions.h:176-183

TRACKER_COUNTER_HEADER = (   # _tracker_getCounterHeaderString, tracker.c:391-397
    "packets-total,bytes-total,packets-control,bytes-control-header,"
    "packets-control-retrans,bytes-control-header-retrans,"
    "packets-data,bytes-data-header,bytes-data-payload,"
    "packets-data-retrans,bytes-data-header-retrans,bytes-data-payload-retrans")

NODE_HEADER_LINE = (         # _tracker_logNode's header, tracker.c:429-441
    "[shadow-heartbeat] [node-header] interval-seconds,recv-bytes,send-bytes,cpu-percent,"
    "delayed-count,avgdelay-milliseconds;inbound-localhost-counters;outbound-localhost-counters;"
    "inbound-remote-counters;outbound-remote-counters where counters are: " + TRACKER_COUNTER_HEADER)


def _counter_string(packets: int, payload: int) -> str:
    """_tracker_getCounterString (tracker.c:399-417) for `packets` first-sent UDP
    datagrams (_tracker_updateCounters, tracker.c:183-214: payload > 0 is 'data',
    payload 0 is 'control'); PHOLD-UDP has no retransmissions."""
    h, p = packets * SHD_HEADER_UDP, packets * payload
    if payload > 0:
        f = (packets, h + p, 0, 0, 0, 0, packets, h, p, 0, 0, 0)
    else:
        f = (packets, h, packets, h, 0, 0, 0, 0, 0, 0, 0, 0)
    return ",".join(str(x) for x in f)


def take_lines(ptr) -> list:
    """[(time_ns, host, line)] of a shd_lines* made by the library, which is freed"""
    try:
        L = ptr.contents
        n = int(L.n)
        if n == 0:
            return []
        off = np.ctypeslib.as_array(L.off, shape=(n + 1,)).copy()
        t = np.ctypeslib.as_array(L.time, shape=(n,)).tolist()
        h = np.ctypeslib.as_array(L.host, shape=(n,)).tolist()
        text = C.string_at(L.text, int(off[-1])).decode()
        return [(t[i], h[i], text[off[i]:off[i + 1]]) for i in range(n)]
    finally:
        lib().shd_lines_free(ptr)


def _ips_u32(ips) -> np.ndarray:
    out = np.empty(len(ips), dtype=np.uint32)
    for i, ip in enumerate(ips):
        if isinstance(ip, str):
            a = [int(x) for x in ip.split(".")]
            out[i] = (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]
        else:
            out[i] = int(ip)
    return out


def tracker_node_lines(snapshots, interval_ns: int, payload: int) -> list:
    """The [shadow-heartbeat] [node] lines of one host (tracker.c:419-465), made
    by the library's writer (shd_node_lines) from the host's cumulative
    interface counters at each heartbeat ([K, 2] uint32 in/out)."""
    snap = np.ascontiguousarray(np.asarray(snapshots, dtype=np.uint32).reshape(-1, 2))
    out = C.POINTER(Lines)()
    check(lib().shd_node_lines(snap.ctypes.data_as(C.POINTER(C.c_uint32)), len(snap), int(interval_ns),
                               int(payload), 0, C.byref(out)), "shd_node_lines")
    return [x[2] for x in take_lines(out)]


def tracker_node_lines_py(snapshots, interval_ns: int, payload: int) -> list:
    """The [shadow-heartbeat] [node] lines of one host (tracker.c:419-465) from its
    cumulative interface counters at each heartbeat (shd_eng_heartbeats: [K, 2]
    uint32 in/out).  Every counter is cleared at each heartbeat (tracker.c:584-593),
    so a line holds the differences to the previous heartbeat.  The loopback
    shortcut keeps the host's own address (network_interface.c:548-555), so all
    packets count as remote; the CPU model is off (cpu-percent 0, no delays)."""
    secs = int(interval_ns // SHD_SEC)
    zero = _counter_string(0, payload)
    # tracker_new runs the first heartbeat inline at boot (tracker.c:141): the
    # header, then an all-zero line, before the K periodic ones
    lines = [NODE_HEADER_LINE, "[shadow-heartbeat] [node] %u,%d,%d,%f,%d,%f;%s;%s;%s;%s" % (
        secs, 0, 0, 0.0, 0, 0.0, zero, zero, zero, zero)]
    prev = (0, 0)
    for cin, cout in np.asarray(snapshots, dtype=np.int64).tolist():
        # the device counters are cumulative uint32 (wrap after 2^32 packets);
        # the reference's are per-interval gsize, cleared at every heartbeat
        din, dout = (cin - prev[0]) & 0xFFFFFFFF, (cout - prev[1]) & 0xFFFFFFFF
        prev = (cin, cout)
        rb, sb = din * (SHD_HEADER_UDP + payload), dout * (SHD_HEADER_UDP + payload)
        lines.append("[shadow-heartbeat] [node] %u,%d,%d,%f,%d,%f;%s;%s;%s;%s" % (
            secs, rb, sb, 0.0, 0, 0.0, zero, zero, _counter_string(din, payload), _counter_string(dout, payload)))
    return lines


# ---- [STATUS] packet lines (packet_addDeliveryStatus, packet.c:647-659) ----
# Every status a packet passes through is logged as `[<STATUS>] <packet_toString>`
# (packet.c:518-641), the string ending in the packet's whole status list so far.
# The lines come from an engine (or oracle) trace recorded with
# SHD_QF_TRACE_STATUS; each trace kind stands for the reference's calls:
_STATUS_OF = {
    TR_CREATED: ("SND_CREATED", "SND_SOCKET_BUFFERED"),          # udp.c:116, socket.c:405
    TR_SENT: ("SND_INTERFACE_SENT", "INET_SENT"),                # network_interface.c:545, worker.c:306
    TR_INET_DROP: ("SND_INTERFACE_SENT", "INET_DROPPED"),        # network_interface.c:545, worker.c:319
    TR_LOCAL: ("SND_INTERFACE_SENT",),                           # network_interface.c:545 (own address)
    TR_ARRIVE: ("ROUTER_ENQUEUED",),                             # router.c:113
    TR_CODEL_DROP: ("ROUTER_DROPPED",),                          # router_queue_codel.c:139
    # router.c:129 (not for the loopback shortcut), network_interface.c:382,
    # socket.c:143, socket.c:330
    TR_RECV: ("ROUTER_DEQUEUED", "RCV_INTERFACE_RECEIVED", "RCV_SOCKET_PROCESSED", "RCV_SOCKET_BUFFERED"),
    TR_IF_DROP: ("ROUTER_DEQUEUED", "RCV_INTERFACE_RECEIVED", "RCV_INTERFACE_DROPPED"),   # n_i.c:382, 411
    TR_READ: ("RCV_SOCKET_DELIVERED",),                          # udp.c:158
}


# the delivery-status flags (packet.h:19-41), by the names packet_toString prints
STATUS_FLAG = {
    "SND_CREATED": 1 << 1, "SND_TCP_ENQUEUE_THROTTLED": 1 << 2, "SND_TCP_ENQUEUE_RETRANSMIT": 1 << 3,
    "SND_TCP_DEQUEUE_RETRANSMIT": 1 << 4, "SND_TCP_RETRANSMITTED": 1 << 5, "SND_SOCKET_BUFFERED": 1 << 6,
    "SND_INTERFACE_SENT": 1 << 7, "INET_SENT": 1 << 8, "INET_DROPPED": 1 << 9, "ROUTER_ENQUEUED": 1 << 10,
    "ROUTER_DEQUEUED": 1 << 11, "ROUTER_DROPPED": 1 << 12, "RCV_INTERFACE_RECEIVED": 1 << 13,
    "RCV_INTERFACE_DROPPED": 1 << 14, "RCV_SOCKET_PROCESSED": 1 << 15, "RCV_SOCKET_DROPPED": 1 << 16,
    "RCV_TCP_ENQUEUE_UNORDERED": 1 << 17, "RCV_SOCKET_BUFFERED": 1 << 18, "RCV_SOCKET_DELIVERED": 1 << 19,
}


def status_line(name: str, host_id: int, pkt: int, src_ip, sport: int, dst_ip, dport: int, payload: int,
                history) -> str:
    """One [STATUS] line of a UDP datagram: `[<name>] ` + packet_toString
    (packet.c:518-547 UDP header part, 616-633 the ordered status list), as
    packet_addDeliveryStatus logs it (packet.c:647-659); `history` is the
    datagram's status list including `name`."""
    return "[%s] packetID=%u:%u %s:%u -> %s:%u bytes=%u status=%s" % (
        name, host_id, pkt, ip_string(src_ip), sport, ip_string(dst_ip) if dst_ip is not None else "?", dport,
        payload, ",".join(history))


def ip_string(ip) -> str:
    """A host address as address_ipToNewString prints it (dotted quad); `ip` is
    a dotted string or a host-order integer."""
    if isinstance(ip, str):
        return ip
    ip = int(ip)
    return "%d.%d.%d.%d" % ((ip >> 24) & 255, (ip >> 16) & 255, (ip >> 8) & 255, ip & 255)


def status_lines(trace, ips, host_ids=None, payload: int = 1, listen_port: int = SHD_PHOLD_LISTEN_PORT,
                 app_peer=None) -> list:
    """[STATUS] lines of a run traced with SHD_QF_TRACE_STATUS, made by the
    library's writer (shd_status_lines, include/shdgpu.h): a list of
    (time_ns, host index, line).  app_peer: the UDP echo model's roles (None:
    PHOLD).  status_lines_py is the same algorithm in Python
    (tests/test_status_cpu.py checks the two against each other)."""
    tr = np.ascontiguousarray(np.asarray(trace, dtype=TRACE_DTYPE))
    ip = _ips_u32(ips)
    ids = None if host_ids is None else np.ascontiguousarray(np.asarray(host_ids, dtype=np.uint32))
    out = C.POINTER(Lines)()
    check(lib().shd_status_lines(tr.ctypes.data if len(tr) else None, len(tr),
                                 ip.ctypes.data_as(C.POINTER(C.c_uint32)),
                                 None if ids is None else ids.ctypes.data_as(C.POINTER(C.c_uint32)),
                                 len(ip), int(payload), int(listen_port),
                                 None if app_peer is None else
                                 np.ascontiguousarray(app_peer, dtype=np.int32).ctypes.data_as(C.POINTER(C.c_int32)),
                                 C.byref(out)), "shd_status_lines")
    return take_lines(out)


def status_lines_py(trace, ips, host_ids=None, payload: int = 1, listen_port: int = SHD_PHOLD_LISTEN_PORT,
                    app_peer=None) -> list:
    """[STATUS] lines of a run traced with SHD_QF_TRACE_STATUS: a list of
    (time_ns, host index, line), line = "[<STATUS>] packetID=<hostID>:<pkt>
    <srcIP>:<srcPort> -> <dstIP>:<dstPort> bytes=<n> status=<S1>,...,<Sk>"
    (packet.c:522-547, 616-633, 657).  `ips[h]` is host h's address,
    `host_ids[h]` its host_getID (default h + 1); the destination port is the
    PHOLD listener (test_phold.c:223), the source port the implicit bind's
    draw (the CREATED record).  Order: by (time, host), records of one host in
    the engine's order, except that a datagram sent in the instant it was
    created follows its creation at once, as in the reference's call chain
    (sendto -> networkinterface_wantsSend -> _networkinterface_sendPackets).
    Each packet object's release logs a PDS_DESTROYED line (packet.c:198) where
    its last reference goes during the run; the frees at the simulation's
    teardown (datagrams still queued or unread at the end) are not included."""
    tr = np.asarray(trace, dtype=TRACE_DTYPE)
    if host_ids is None:
        host_ids = [h + 1 for h in range(len(ips))]
    order = np.lexsort((np.arange(len(tr)), tr["host"], tr["time"]))
    tr = tr[order]
    NONE = 0xFFFFFFFF
    dport = [listen_port] * len(ips)   # a UDP echo client's socket port: its own datagrams' source port
    if app_peer is not None:
        for r in tr:
            if int(r["kind"]) == TR_CREATED and app_peer[int(r["host"])] >= 0:
                dport[int(r["host"])] = int(r["seq"]) & 0xFFFF
    port, dst, created_at, local = {}, {}, {}, set()
    for r in tr:
        k, h, p = int(r["kind"]), int(r["host"]), int(r["pkt"])
        if k == TR_CREATED:
            port[(h, p)] = int(r["seq"])
            created_at[(h, p)] = int(r["time"])
        elif k in (TR_SENT, TR_INET_DROP, TR_LOCAL):
            dst[(h, p)] = int(r["peer"])
            if k == TR_LOCAL:
                local.add((h, p))
    sends = {}   # sender records that follow their creation
    for i, r in enumerate(tr):
        k, h, p = int(r["kind"]), int(r["host"]), int(r["pkt"])
        if k in (TR_SENT, TR_INET_DROP, TR_LOCAL) and created_at.get((h, p)) == int(r["time"]):
            sends[(h, p)] = i
    hist = {}
    inbox = {}   # per host: datagrams buffered in the socket, oldest first
    out = []

    def emit(t, at, key, statuses):
        src, pkt = key
        st = hist.setdefault(key, [])
        d = dst.get(key, NONE)
        for name in statuses:
            st.append(name)
            out.append((t, at, status_line(name, host_ids[src], pkt, ips[src], port.get(key, 0),
                                           ips[d] if d != NONE else None, dport[d] if d != NONE else listen_port,
                                           payload, st)))

    arrived = {(int(r["peer"]), int(r["pkt"])) for r in tr if int(r["kind"]) == TR_ARRIVE}

    def destroyed(t, at, key, copy_dropped=False):
        # packet_unref's last reference (packet.c:194-201) logs PDS_DESTROYED with
        # the object's list.  A sent datagram is two objects from INET_SENT on
        # (worker.c:306-313 copies it for the receiver): the sender's original
        # is released at once (network_interface.c:577), after the copy when
        # scheduler_push dropped the copy's event past the end (scheduler.c:346-349)
        d = dst.get(key, NONE)
        st = hist[key] + ["PDS_DESTROYED"]
        line = status_line("PDS_DESTROYED", host_ids[key[0]], key[1], ips[key[0]], port.get(key, 0),
                           ips[d] if d != NONE else None, dport[d] if d != NONE else listen_port, payload, st)
        for _ in range(2 if copy_dropped else 1):
            out.append((t, at, line))

    def send_side(t, h, key, k):
        emit(t, h, key, _STATUS_OF[k])
        if k == TR_SENT:
            destroyed(t, h, key, copy_dropped=key not in arrived)
        elif k == TR_INET_DROP:
            destroyed(t, h, key)

    for i, r in enumerate(tr):
        k, h, p, t = int(r["kind"]), int(r["host"]), int(r["pkt"]), int(r["time"])
        if k in (TR_SENT, TR_INET_DROP, TR_LOCAL) and sends.get((h, p)) == i:
            continue   # emitted with its creation
        if k == TR_CREATED:
            emit(t, h, (h, p), _STATUS_OF[k])
            j = sends.get((h, p))
            if j is not None:
                send_side(t, h, (h, p), int(tr[j]["kind"]))
        elif k in (TR_SENT, TR_INET_DROP, TR_LOCAL):
            send_side(t, h, (h, p), k)
        elif k == TR_READ:
            q = inbox.get(h)
            if q:
                key = q.pop(0)
                emit(t, h, key, _STATUS_OF[k])
                destroyed(t, h, key)   # the socket's reference, udp.c:169
        else:   # the receiver's records name the packet by (source, pkt)
            key = (int(r["peer"]), p)
            names = _STATUS_OF[k]
            if k in (TR_RECV, TR_IF_DROP) and key in local:
                names = names[1:]   # the loopback shortcut skips the router
            emit(t, h, key, names)
            if k == TR_RECV:
                inbox.setdefault(h, []).append(key)
            elif k in (TR_CODEL_DROP, TR_IF_DROP):
                # the queue's reference (router_queue_codel.c), or the interface's
                # (network_interface.c:446) / the local task's (:553): the last one
                destroyed(t, h, key)
    return out
