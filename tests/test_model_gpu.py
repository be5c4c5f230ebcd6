"""Model-level features on the GPU engine, each against the serial oracle:

* destination-weight classes (each PHOLD process reads its own weights file,
  test_phold.c:341-356): the Tor-scale relay / client model (BASELINE C4) at
  small size, and a three-class model on a geometric graph;
* per-host heartbeat intervals (<host heartbeatfrequency>, tracker interval,
  host.c:240; tracker.c:566-611);
* caller-pushed application starts (shd_eng_push_events: process_schedule per
  <process starttime>, host.c:372-390, process.c:1344).
"""
import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S
import workloads as W
from sim import Engine, PathCache, XGroup, sort_trace

pytestmark = pytest.mark.gpu


def assert_same_run(eng_or_engines, st_pkt, m, g, **okw):
    engines = eng_or_engines if isinstance(eng_or_engines, list) else [eng_or_engines]
    otr, odg, ost = O.engine_run(m, g, **okw)
    tr = sort_trace(np.concatenate([e.trace() for e in engines]))
    dg = np.concatenate([e.digest() for e in engines])
    assert st_pkt == ost["n_pkt_events"] > 0
    assert np.array_equal(tr, sort_trace(otr))
    assert np.array_equal(dg, odg)
    return otr


def test_tor_model_relays_and_clients_match_oracle():
    g, m = W.tor_model(60, 540, end_time=3 * S.SHD_SEC, trace=True, load=4)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc)
    st = eng.run()
    otr = assert_same_run(eng, st.n_pkt_events, m, g)
    recv = otr[otr["kind"] == S.TR_RECV]
    # clients only send to relays: every client-to-client delivery is impossible
    sent = otr[otr["kind"] == S.TR_SENT]
    assert not np.any((sent["host"] >= 60) & (sent["peer"] >= 60))
    assert np.count_nonzero(recv["host"] >= 60) > 100       # relays forward to clients


@pytest.mark.parametrize("parts", [1, 3])
def test_three_weight_classes_on_geometric_graph(parts):
    from driver import partition
    V = 240
    g = W.geometric_graph(V, seed=11)
    hv = W.hosts_on_vertices(V, 1)
    rng = np.random.default_rng(5)
    rows = []
    for k in range(3):   # class 0 uniform, class 1 skewed, class 2 only the first half
        w = np.ones(V) if k == 0 else rng.pareto(1.5, V) + 0.1
        if k == 2:
            w[V // 2:] = 0.0
        rows.append(W.phold_cum(w))
    cls = (np.arange(V) % 3).astype(np.uint8)
    # skewed weights: the heaviest hosts receive many times the mean (capacities sized for them)
    m = W.phold_model(hv, end_time=3 * S.SHD_SEC, trace=True, dest_cum=np.stack(rows), host_class=cls,
                      inbox_cap=1024, evq_cap=4096, codelq_cap=1024)
    pc = PathCache(g, W.attached_vertices(hv))
    if parts == 1:
        eng = Engine(m, pc)
        st = eng.run()
        assert_same_run(eng, st.n_pkt_events, m, g)
    else:
        pb = partition(m.n_hosts, parts)
        engines = [Engine(m, pc, pb[i], pb[i + 1]) for i in range(parts)]
        grp = XGroup.local(engines)
        st = grp.run()
        assert_same_run(engines, st.n_pkt_events, m, g)
        grp.close()


def test_per_host_heartbeat_intervals_match_oracle():
    V = 150
    end = int(4.5 * S.SHD_SEC)
    g = W.geometric_graph(V, seed=3)
    hbi = np.array([S.SHD_SEC // 2, S.SHD_SEC, 2 * S.SHD_SEC], dtype=np.uint64)[np.arange(V) % 3]
    m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=end, queue_flags=S.SHD_QF_HEARTBEATS,
                      trace=True)
    m = S.ModelArrays(m.host_vertex, m.host_rng, m.bw_down, m.bw_up, m.dest_cum, end_time=end,
                      trace=True, queue_flags=S.SHD_QF_HEARTBEATS, host_heartbeat=hbi)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc)
    st = eng.run()
    hb = eng.heartbeats()
    K = (end - 1) // (S.SHD_SEC // 2)
    assert hb.shape == (V, K, 2)
    ohb = np.zeros((V, K, 2), dtype=np.uint32)
    assert_same_run(eng, st.n_pkt_events, m, g, heartbeats=ohb)
    assert np.array_equal(hb, ohb)
    # a 2 s host has two snapshots, the rest of its row stays zero
    assert np.all(hb[2::3, 2:] == 0) and np.any(hb[2::3, :2] != 0)


def test_pushed_application_starts_match_oracle():
    V = 200
    g = W.geometric_graph(V, seed=7)
    m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=3 * S.SHD_SEC, trace=True, load=6,
                      queue_flags=S.SHD_QF_NO_APP_START)
    rng = np.random.default_rng(2)
    ev = []
    for h in range(V):
        for _ in range(int(rng.integers(0, 3))):   # 0, 1 or 2 processes per host
            t = int(rng.integers(1, 4)) * S.SHD_SEC // 2 + int(rng.integers(0, 1000))
            ev.append((t, 0, h, h, 0, S.EV_APP_START))
    ev.append((5 * S.SHD_SEC, 0, 3, 3, 0, S.EV_APP_START))   # past the end: dropped, ID consumed
    pushes = np.array(ev, dtype=S.EVENT_DTYPE)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc)
    eng.boot()
    eng.push_events(pushes)
    st = eng.run()
    assert_same_run(eng, st.n_pkt_events, m, g, pushes=pushes)


def test_pushed_starts_at_the_first_heartbeat_keep_timer_ids():
    """Several processes per host starting exactly at the first heartbeat
    (1 s): the pushes consume event IDs after the boot timers were armed, so
    the heartbeat (ID 0) and the pending refill keep their IDs and run before
    the starts in (time, src, seq) order (event.c:110-153).  A shift of the
    timers' IDs by the pushed count would put the starts first and change the
    heartbeat counters and every later ID (advisor finding, round 2)."""
    V = 80
    g = W.geometric_graph(V, seed=13)
    m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=3 * S.SHD_SEC, trace=True, load=3,
                      queue_flags=S.SHD_QF_NO_APP_START | S.SHD_QF_HEARTBEATS)
    ev = []
    for h in range(V):
        for _ in range(4 + h % 3):   # 4..6 processes per host, all at 1 s
            ev.append((S.SHD_SEC, 0, h, h, 0, S.EV_APP_START))
    pushes = np.array(ev, dtype=S.EVENT_DTYPE)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc)
    eng.boot()
    eng.push_events(pushes)
    st = eng.run()
    K = (3 * S.SHD_SEC - 1) // S.SHD_SEC
    ohb = np.zeros((V, K, 2), dtype=np.uint32)
    assert_same_run(eng, st.n_pkt_events, m, g, pushes=pushes, heartbeats=ohb)
    assert np.array_equal(eng.heartbeats(), ohb)


def test_push_events_rejects_what_it_cannot_take():
    V = 60
    g = W.geometric_graph(V, seed=7)
    m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=2 * S.SHD_SEC,
                      queue_flags=S.SHD_QF_NO_APP_START)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc)
    bad_kind = np.array([(S.SHD_SEC, 0, 1, 1, 0, S.EV_PACKET)], dtype=S.EVENT_DTYPE)
    with pytest.raises(S.ShdError):
        eng.push_events(bad_kind)            # not booted yet
    eng.boot()
    with pytest.raises(S.ShdError):
        eng.push_events(bad_kind)
    with pytest.raises(S.ShdError):
        eng.push_events(np.array([(S.SHD_SEC, 0, 1, 2, 0, S.EV_APP_START)], dtype=S.EVENT_DTYPE))
    eng.run_until(S.SHD_SEC)
    with pytest.raises(S.ShdError):          # before the engine's current time
        eng.push_events(np.array([(S.SHD_SEC // 2, 0, 1, 1, 0, S.EV_APP_START)], dtype=S.EVENT_DTYPE))
    eng.push_events(np.array([(S.SHD_SEC + 5, 0, 1, 1, 0, S.EV_APP_START)], dtype=S.EVENT_DTYPE))
    st = eng.run()
    assert st.n_pkt_events > 0


@pytest.mark.parametrize("codel", [False, True], ids=["plain", "codel"])
def test_status_trace_matches_oracle(codel):
    """SHD_QF_TRACE_STATUS: the application's records (CREATED with the bind's
    port draw, READ) on the device equal the oracle's, and so do the [STATUS]
    lines made from them (packet.c:518-659).  codel: 1500-B payloads into a
    512 KiB/s receive bucket, so packets queue and CoDel drops some."""
    V = 120
    g = W.geometric_graph(V, seed=9)
    kw = dict(payload=1500, bw_down=512, codelq_cap=256, load=32) if codel else dict(load=4)
    m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=3 * S.SHD_SEC, trace=True,
                      queue_flags=S.SHD_QF_TRACE_STATUS, **kw)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc)
    st = eng.run()
    otr = assert_same_run(eng, st.n_pkt_events, m, g)
    kinds = np.bincount(otr["kind"], minlength=10)
    assert kinds[S.TR_CREATED] > 0 and kinds[S.TR_READ] > 0
    if codel:
        assert kinds[S.TR_CODEL_DROP] > 0
    ips = ["11.0.0.%d" % (h + 1) for h in range(V)]
    payload = kw.get("payload", 1)
    assert S.status_lines(eng.trace(), ips, payload=payload) == S.status_lines(otr, ips, payload=payload)
