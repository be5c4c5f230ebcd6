"""The oracle's path cache and serial loop against independent fixtures
(networkx Dijkstra golden vectors, the bundled topology's known shape) and the
reference's selection rules (topology.c)."""
import os

import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S
import workloads as W

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_geo300():
    z = np.load(os.path.join(GOLD, "pathcache_geo300.npz"))
    g = S.GraphArrays(300, z["src"], z["dst"], z["latency"], z["loss"], z["vertex_loss"])
    return g, z


def bits(x):
    return np.ascontiguousarray(x, dtype=np.float64).view(np.uint64)


def test_oracle_rows_match_networkx_golden():
    g, z = golden_geo300()
    og = O.OGraph(g)
    targets = np.arange(300, dtype=np.int32)
    for i, s in enumerate(z["sources"]):
        lat, rel, ok, hops, ties = og.row(int(s), targets)
        assert ties == 0 and ok.all()
        m = np.arange(300) != s
        assert np.array_equal(bits(lat[m]), bits(z["lat"][i][m]))
        assert np.array_equal(bits(rel[m]), bits(z["rel"][i][m]))
        assert np.array_equal(hops[m], z["hops"][i][m])


def test_bundled_topology_shape_and_completeness():
    g = W.bundled_graph()
    og = O.OGraph(g)
    p = og.props()
    assert (g.n_vertices, g.n_edges) == (183, 16836)
    assert p.is_complete == 1 and p.is_connected == 1 and p.n_self_loops == 183
    pp = S.GraphProps()
    assert S.lib().shd_graph_check(S.C.byref(g.struct), S.C.byref(pp)) == 0
    assert (pp.is_complete, pp.is_connected, pp.n_self_loops) == (1, 1, 183)


def test_direct_path_reliability_order():
    # ((1 * r(s)) * r(d)) * r(e) with r = 1.0f - loss (topology.c:1900-1921)
    g = W.bundled_graph()
    og = O.OGraph(g)
    e = 100
    s, d = int(g.src[e]), int(g.dst[e])
    lat, rel = og.direct(s, d)
    assert lat == 0.0 + g.latency[e]
    vl = g.vertex_loss
    assert rel == ((1.0 * (1.0 - vl[s])) * (1.0 - vl[d])) * (1.0 - g.loss[e])


def test_lazy_cache_complete_graph_serves_direct_paths():
    g = W.bundled_graph()
    att = np.arange(183, dtype=np.int32)
    ot = O.OTopo(O.OGraph(g), att)
    og = O.OGraph(g)
    for s, d in [(1, 2), (2, 1), (50, 50), (7, 180)]:
        assert ot.get(s, d) == og.direct(s, d)
    assert ot.rows_run() == 0


def path_graph_asym():
    """0-1-2-3 chain plus a long direct 0-3 edge: the left fold from either end
    differs in the last bit ((0.1+0.2)+0.3 != (0.3+0.2)+0.1)."""
    src = [0, 1, 2, 0, 0, 1, 2, 3]
    dst = [1, 2, 3, 3, 0, 1, 2, 3]
    lat = [0.1, 0.2, 0.3, 50.0, 1.0, 1.0, 1.0, 1.0]
    loss = [0.001, 0.002, 0.003, 0.0, 0, 0, 0, 0]
    return S.GraphArrays(4, src, dst, lat, loss)


def test_first_touch_orientation_rule():
    g = path_graph_asym()
    og = O.OGraph(g)
    att = np.arange(4, dtype=np.int32)
    l03 = og.row(0, att)[0][3]
    l30 = og.row(3, att)[0][0]
    assert l03 == (0.1 + 0.2) + 0.3 and l30 == (0.3 + 0.2) + 0.1
    assert l03 != l30   # the folds differ: orientation is observable
    # row 0 runs first: every later lookup of {0,3} serves row 0's value
    ot = O.OTopo(og, att)
    assert ot.get(0, 3)[0] == l03 and ot.get(3, 0)[0] == l03
    ot2 = O.OTopo(og, att)
    assert ot2.get(3, 0)[0] == l30 and ot2.get(0, 3)[0] == l30


def test_self_path_before_row_gives_twice_min_edge():
    g = path_graph_asym()
    og = O.OGraph(g)
    att = np.arange(4, dtype=np.int32)
    ot = O.OTopo(og, att)
    lat, rel = ot.get(2, 2)                  # before row 2 ran: 2 x min incident edge
    assert (lat, rel) == (2.0 * 0.2, (1.0 - 0.002) * (1.0 - 0.002))
    assert (lat, rel) == og.self_path(2)
    ot2 = O.OTopo(og, att)
    ot2.get(2, 3)                            # row 2 runs first ...
    assert ot2.get(2, 2) == (1.0, 1.0)       # ... and stores [2] = the self-loop


def test_oracle_engine_is_deterministic_and_consistent():
    g = W.geometric_graph(80, seed=5)
    m = W.phold_model(W.hosts_on_vertices(80, 1), end_time=int(2.5 * S.SHD_SEC), trace=True)
    tr1, dg1, st1 = O.engine_run(m, g)
    tr2, dg2, st2 = O.engine_run(m, g)
    assert np.array_equal(tr1, tr2) and np.array_equal(dg1, dg2)
    kinds = np.bincount(tr1["kind"], minlength=8)
    # every delivered packet that arrived was sent; arrivals are packet events
    assert kinds[S.TR_ARRIVE] == st1["n_pkt_events"] <= kinds[S.TR_SENT]
    assert dg1["n_pkt_events"].sum() == st1["n_pkt_events"]
    # each arrival carries the seq its sender assigned (event_new_, event.c:38)
    sent = {(int(r["host"]), int(r["seq"])) for r in tr1[tr1["kind"] == S.TR_SENT]}
    arr = tr1[tr1["kind"] == S.TR_ARRIVE]
    assert all((int(r["peer"]), int(r["seq"])) in sent for r in arr[:2000])
    # heartbeats, refills and app start consumed ids first (boot order, host.c:372-390)
    assert (dg1["ev_seq"] >= 4).all()


def test_serial_trace_is_time_ordered():
    g = W.bundled_graph()
    hv = np.arange(0, 183, 3, dtype=np.int32)
    m = W.phold_model(hv, end_time=2 * S.SHD_SEC, trace=True, load=4)
    tr, dg, st = O.engine_run(m, g)
    assert np.all(np.diff(tr["time"].astype(np.int64)) >= 0)
    assert st["rows_run"] == 0


def test_oracle_heartbeat_counters_follow_the_trace():
    """tracker node counters at each heartbeat (tracker.c:566-611): away from the
    heartbeat instants themselves, the cumulative in / out counts equal the
    interface receptions (RECV, IF_DROP) and departures (SENT, INET_DROP, LOCAL)
    traced before them; the [node] lines carry the per-interval differences."""
    end = int(3.5 * S.SHD_SEC)
    g = W.geometric_graph(120, seed=5)
    m = W.phold_model(W.hosts_on_vertices(120, 1), end_time=end, trace=True,
                      queue_flags=S.SHD_QF_HEARTBEATS)
    hb = np.zeros((m.n_hosts, 3, 2), dtype=np.uint32)
    tr, _, _ = O.engine_run(m, g, heartbeats=hb)
    inn = np.isin(tr["kind"], [S.TR_RECV, S.TR_IF_DROP])
    out = np.isin(tr["kind"], [S.TR_SENT, S.TR_INET_DROP, S.TR_LOCAL])
    checked = 0
    for h in range(m.n_hosts):
        mine = tr["host"] == h
        for k in range(1, 4):
            T = k * S.SHD_SEC
            if np.any(mine & (tr["time"] == T)):
                continue          # the order against the heartbeat needs the event key
            assert hb[h, k - 1, 0] == np.count_nonzero(mine & inn & (tr["time"] < T))
            assert hb[h, k - 1, 1] == np.count_nonzero(mine & out & (tr["time"] < T))
            checked += 1
    assert checked > 200 and int(hb[:, -1].sum()) > 1000
    lines = S.tracker_node_lines(hb[3], S.SHD_SEC, 1)
    assert lines[0].startswith("[shadow-heartbeat] [node-header] interval-seconds,")
    # the boot heartbeat (tracker_new -> tracker_heartbeat inline, tracker.c:141)
    # logs an all-zero line, then one line per periodic heartbeat: K + 1 lines
    assert len(lines) == 1 + 1 + 3
    assert lines[1] == lines[1].split("] [node] ")[0] + "] [node] 1,0,0,0.000000,0,0.000000;" + ";".join(
        [",".join(["0"] * 12)] * 4)
    d = np.diff(np.vstack([[0, 0], hb[3].astype(np.int64)]), axis=0)
    for line, (din, dout) in zip(lines[2:], d):
        head, loc_in, loc_out, rem_in, rem_out = line.split("] [node] ")[1].split(";")
        f = head.split(",")
        assert f[0] == "1" and int(f[1]) == din * 43 and int(f[2]) == dout * 43
        assert loc_in == loc_out == ",".join(["0"] * 12)
        assert rem_in.split(",")[:2] == [str(din), str(din * 43)]
        assert rem_out.split(",")[6:9] == [str(dout), str(dout * 42), str(dout)]


@pytest.mark.parametrize("kind", ["rows", "rows_lossy", "complete"])
def test_parallel_rounds_equal_the_serial_loop(kind):
    """The CPU baseline's parallel variant (host-partitioned rounds of W <=
    every path latency, per-host queues, first touches resolved at the round's
    end in serial order) ends in the serial loop's state, bit for bit, from a
    state warmed up serially; several first-touch rounds fall in the window."""
    if kind == "complete":
        g = W.bundled_graph()
        hv = np.sort(np.random.default_rng(3).integers(0, g.n_vertices, 600)).astype(np.int32)
    else:
        g = W.geometric_graph(400, seed=9, loss_max=0.01 if kind == "rows_lossy" else 0.0)
        hv = W.hosts_on_vertices(400, 1)
    m = W.phold_model(hv, end_time=4 * S.SHD_SEC, load=8)
    out = O.baseline(m, g, int(1.3 * S.SHD_SEC), 4 * S.SHD_SEC, 4)
    assert out["rc"] == 0 and out["same_end_state"] == 1, out
    assert out["serial_pkt_events"] == out["parallel_pkt_events"] > 10000
    assert out["ambiguous"] == 0
    if kind != "complete":
        assert out["parallel_first_touch"] > 0
