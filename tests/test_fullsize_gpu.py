"""Event-loop parity at BASELINE's full sizes (C3: 10 k hosts on the 10 k-vertex
geometric graph; the N = 2 bench workload: 20 k hosts on the same graph).

The serial oracle needs about a minute for the 10 k Dijkstra rows alone, so at
these sizes parity is checked through properties that do not depend on size:
the run is the same, bit for bit, whether the hosts run on one engine or are
sharded over an engine group exactly as bench.py --gpus N shards them
(contiguous registration-order blocks, one all-to-all per round), and the same
from one run to the next (the reference's determinism tests,
src/test/determinism).  The small-size tests in test_engine_gpu.py tie both
sides to the oracle.
"""
import numpy as np
import pytest

import shdgpu as S
import workloads as W
from sim import Engine, PathCache

pytestmark = pytest.mark.gpu

V = 10000
END = 3 * S.SHD_SEC          # boot, application start at 1 s, two seconds of traffic


def bench_workload(hosts):
    """The host placement and PHOLD model bench.py builds (seed 1, load 16,
    1-byte payloads, edge loss U[0, 0.0005])."""
    g = W.geometric_graph(V, seed=1, loss_max=0.0005)
    hpv = max(1, hosts // V)
    hv = (np.arange(hosts, dtype=np.int64) * V // hosts).astype(np.int32) if hosts != V * hpv else \
        W.hosts_on_vertices(V, hpv)
    m = W.phold_model(hv, end_time=END, seed=1, load=16, payload=1)
    return g, m


def single(m, pc):
    e = Engine(m, pc)
    st = e.run()
    dg = e.digest()
    e.close()
    return st, dg


@pytest.fixture(scope="module")
def c3():
    g, m = bench_workload(V)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    yield g, m, pc
    pc.close()


def test_c3_full_size_deterministic(c3):
    _, m, pc = c3
    st1, d1 = single(m, pc)
    st2, d2 = single(m, pc)
    assert st1.n_pkt_events > 1_000_000 and st1.error == 0
    assert (st1.n_events, st1.n_pkt_events, st1.n_rounds) == (st2.n_events, st2.n_pkt_events, st2.n_rounds)
    assert np.array_equal(d1, d2)
    # per-host counters add up to the run's totals
    assert int(d1["n_pkt_events"].sum()) == st1.n_pkt_events
    assert int(d1["n_events"].sum()) == st1.n_events


@pytest.mark.parametrize("hosts,parts", [(V, 2), (2 * V, 2), (V, 4), (4 * V, 4), (8 * V, 8)])
def test_bench_workload_sharded_group_equals_single_engine(hosts, parts):
    """(N V, N) is bench.py --gpus N's workload (weak scaling: N x 10 k hosts on the
    same graph), sharded as its N ranks shard it."""
    from driver import partition
    from sim import XGroup
    g, m = bench_workload(hosts)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    st, d1 = single(m, pc)
    pb = partition(m.n_hosts, parts)
    engines = [Engine(m, pc, pb[i], pb[i + 1]) for i in range(parts)]
    grp = XGroup.local(engines)
    gst = grp.run()
    dg = np.concatenate([e.digest() for e in engines])
    assert gst.error == 0
    assert gst.n_pkt_events == st.n_pkt_events and gst.n_events == st.n_events
    assert np.array_equal(dg, d1)
    grp.close()
    for e in engines:
        e.close()
    pc.close()


def test_c5_million_hosts_group_equals_single_engine():
    """BASELINE C5's scale on one GPU: 1 M hosts, 100 per vertex of the 10 k-vertex
    graph (the scripts/c5_single.sh workload).  The application start logs
    ~16 M first touches, so the protected rounds run here; two engines of a
    group must end where one engine ends."""
    from driver import partition
    from sim import XGroup
    g = W.geometric_graph(V, seed=1, loss_max=0.0005)
    m = W.phold_model(W.hosts_on_vertices(V, 100), end_time=int(1.5 * S.SHD_SEC), seed=1, load=16,
                      payload=1)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    st, d1 = single(m, pc)
    assert st.error == 0 and st.n_rounds_protected > 0 and st.n_pkt_events > 10_000_000
    pb = partition(m.n_hosts, 2)
    engines = [Engine(m, pc, pb[i], pb[i + 1]) for i in range(2)]
    grp = XGroup.local(engines)
    gst = grp.run()
    assert gst.error == 0
    assert gst.n_pkt_events == st.n_pkt_events and gst.n_events == st.n_events
    assert np.array_equal(np.concatenate([e.digest() for e in engines]), d1)
    grp.close()
    for e in engines:
        e.close()
    pc.close()
