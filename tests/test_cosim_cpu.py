"""Packet ingress / egress between two sides of one model, on the oracle
(CPU; the checker for the GPU co-simulation tests).

Two oracle states each hold part of the hosts (oracle.h o_state_new_part);
they run the same windows of W and, between windows, exchange the packet
deliveries their hosts sent to the other side -- worker_sendPacket's
scheduler_push of a deliver-packet task for another worker's host
(worker.c:541-571), every one due at or after the window's end because W is
at most every path latency.  The union of their traces and end states must be
the whole serial run's, bit for bit.  On the bundled topology (complete: every
pair's path is its direct edge) the value of a path does not depend on which
side's cache touched it first.
"""
import math

import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S
import workloads as W
from sim import sort_trace

U64_MAX = (1 << 64) - 1


def min_window(g: S.GraphArrays) -> int:
    """A window no path is shorter than: the smallest edge latency, in ns."""
    return max(1, int(math.ceil(float(np.min(g.latency)) * S.SHD_MS)))


def cosim(m, g, cuts, W_ns):
    """The oracle split at `cuts`, windows of W_ns; returns (trace, digest,
    events, packets exchanged)."""
    H = m.n_hosts
    bounds = [0] + list(cuts) + [H]
    parts = [O.OState(m, g, hosts=(bounds[i], bounds[i + 1])) for i in range(len(bounds) - 1)]
    end = m.params["end_time"]
    exchanged = 0
    while True:
        ws = min(p.next_time() for p in parts)
        if ws >= end or ws == U64_MAX:
            break
        we = ws + W_ns
        for p in parts:
            p.run_serial(we)
        out = [p.take_egress() for p in parts]
        allev = np.concatenate(out)
        assert np.all(allev["time"] >= we)                       # nothing lands inside the window
        assert np.all(allev["kind"] == S.EV_PACKET)
        for i, p in enumerate(parts):
            mine = allev[(allev["dst"] >= bounds[i]) & (allev["dst"] < bounds[i + 1])]
            assert np.all((mine["src"] < bounds[i]) | (mine["src"] >= bounds[i + 1]))
            p.inject(mine)
        exchanged += len(allev)
    tr = sort_trace(np.concatenate([p.trace() for p in parts]))
    dg = np.concatenate([parts[i].digest()[bounds[i]:bounds[i + 1]] for i in range(len(parts))])
    ev = sum(p.counts()[0] for p in parts)
    for p in parts:
        p.close()
    return tr, dg, ev, exchanged


@pytest.mark.parametrize("cuts", [(150,), (1,), (60, 199)])
def test_oracle_sides_exchanging_packets_equal_the_serial_run(cuts):
    g = W.bundled_graph()
    hv = np.sort(np.random.default_rng(3).integers(0, g.n_vertices, 240)).astype(np.int32)
    m = W.phold_model(hv, end_time=int(2.5 * S.SHD_SEC), trace=True, load=6)
    tr, dg, ev, exchanged = cosim(m, g, cuts, min_window(g))
    otr, odg, ost = O.engine_run(m, g)
    assert exchanged > 100
    assert ev == ost["n_events"]
    assert len(tr) == len(otr) and np.array_equal(tr, sort_trace(otr))
    assert np.array_equal(dg, odg)


def test_oracle_sides_with_status_records_and_codel_drops():
    # the application's side of each datagram (SHD_QF_TRACE_STATUS) and router
    # drops on a slow receiver cross the boundary the same way
    g = W.bundled_graph()
    hv = np.sort(np.random.default_rng(5).integers(0, g.n_vertices, 120)).astype(np.int32)
    m = W.phold_model(hv, end_time=3 * S.SHD_SEC, trace=True, load=24, payload=1000, bw_down=200,
                      bw_up=100000, codelq_cap=256, queue_flags=S.SHD_QF_TRACE_STATUS)
    tr, dg, _, _ = cosim(m, g, (70,), min_window(g))
    otr, odg, _ = O.engine_run(m, g)
    assert np.count_nonzero(tr["kind"] == S.TR_CODEL_DROP) > 0
    assert np.array_equal(tr, sort_trace(otr))
    assert np.array_equal(dg, odg)


def test_inject_rejects_events_for_the_other_side():
    g = W.bundled_graph()
    hv = np.arange(10, dtype=np.int32)
    m = W.phold_model(hv, end_time=S.SHD_SEC)
    st = O.OState(m, g, hosts=(0, 5))
    bad = np.zeros(1, dtype=S.EVENT_DTYPE)
    bad["kind"] = S.EV_PACKET
    bad["src"], bad["dst"] = 1, 7                          # for a host of the other side
    assert O.lib().o_state_inject(st.ptr, bad.ctypes.data, 1) == -1
    bad["src"], bad["dst"] = 2, 3                          # from a host of this side
    assert O.lib().o_state_inject(st.ptr, bad.ctypes.data, 1) == -1
    st.close()
