"""Event-loop parity on the GPU: libshdgpu engine vs the serial oracle.

The oracle runs the reference's serial mode (--workers 0, one global queue in
event_compare order, slave.c:415-428); the engine runs serial-equivalent
rounds of width W on the GPU.  Traces (every packet state change) must be the
same multiset and every host's end state must match bit for bit.
"""
import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S
import workloads as W
from sim import Engine, PathCache, sort_trace

pytestmark = pytest.mark.gpu


def run_both(g, model, force_rows=False):
    att = W.attached_vertices(model.host_vertex)
    pc = PathCache(g, att, flags=1 if force_rows else 0)
    eng = Engine(model, pc)
    st = eng.run()
    gtr = sort_trace(eng.trace())
    gdg = eng.digest()
    otr, odg, ost = O.engine_run(model, g, force_rows=force_rows)
    otr = sort_trace(otr)
    return (gtr, gdg, st), (otr, odg, ost), eng, pc


def assert_same(gpu, ora):
    (gtr, gdg, st), (otr, odg, ost) = gpu, ora
    assert st.n_events == ost["n_events"]
    assert st.n_pkt_events == ost["n_pkt_events"]
    assert len(gtr) == len(otr)
    assert np.array_equal(gtr, otr)
    assert np.array_equal(gdg, odg)


@pytest.mark.parametrize("queue_flags,closed", [(0, True), (S.SHD_QF_NO_CALENDAR, True), (0, False)])
def test_geometric_one_host_per_vertex(queue_flags, closed, monkeypatch):
    # one host per vertex, even weights: destinations in closed form (the
    # table-free pick), or through the guide table (SHD_NO_DEST_CLOSED)
    if not closed:
        monkeypatch.setenv("SHD_NO_DEST_CLOSED", "1")
    # queue_flags=NO_CALENDAR: every inter-host event takes the inbox + heap path
    g = W.geometric_graph(300, seed=2)
    m = W.phold_model(W.hosts_on_vertices(300, 1), end_time=3 * S.SHD_SEC, trace=True,
                      queue_flags=queue_flags)
    gpu, ora, eng, _ = run_both(g, m)
    assert_same(gpu, ora)
    assert gpu[2].n_rounds > 100
    assert gpu[2].n_batches_ticketless > 0                         # ticketless batches exercised
    assert gpu[2].n_batches_persistent > 0                         # ... as persistent launches (k_round_ps)
    assert np.count_nonzero(gpu[0]["kind"] == S.TR_LOCAL) > 0     # self-sends exercised
    assert np.count_nonzero(gpu[0]["kind"] == S.TR_INET_DROP) > 0  # reliability drops


def run_hooked(scenario, arg, timeout=300, **env_over):
    """A scenario of tests/hook_worker.py in a child process on the test build
    (libshdgpu_th.so: the semantics-changing hooks exist only there), with
    SHD_FORCE_AMBIG and SHD_PROTECT_ALL set; the child checks the run against
    the oracle and returns its statistics."""
    import json
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, SHD_FORCE_AMBIG="1", SHD_PROTECT_ALL="1",
               SHDGPU_LIB=os.path.join(os.path.dirname(here), "shadow-1_amd", "libshdgpu_th.so"))
    for k, v in env_over.items():
        if v is None:
            env.pop(k, None)
        else:
            env[k] = v
    p = subprocess.run([sys.executable, "-u", os.path.join(here, "hook_worker.py"), scenario, str(arg)],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=timeout)
    out = p.stdout.decode(errors="replace")
    assert p.returncode == 0, out[-3000:]
    return json.loads(out.strip().splitlines()[-1])


@pytest.mark.parametrize("hpv", [1, 3])
def test_ambiguous_first_touch_rounds_roll_back(hpv):
    # SHD_FORCE_AMBIG: every undecided first-touch send counts as ambiguous, so
    # every round that logs one is rolled back to its state copy, ranked from
    # its own log and rerun (SHD_PROTECT_ALL: every round behind a copy); the
    # run must still be the serial oracle's, bit for bit (checked in the child)
    st = run_hooked("engine_rollback", hpv)
    assert st["rerun"] > 0 and st["protected"] == st["rounds"]


@pytest.mark.parametrize("steps", [1, 3])
def test_ambiguous_unprotected_rounds_replay(steps):
    # protection off (SHD_NO_PROTECT) with every undecided first-touch send
    # forced ambiguous: an unprotected batch round that logs one cannot be
    # kept, so shd_eng_run_until goes back to its last restore point, runs to
    # the round's start again and runs the round protected; the run is the
    # serial oracle's, bit for bit (checked in the child)
    st = run_hooked("engine_replay", steps, SHD_PROTECT_ALL=None, SHD_NO_PROTECT="1")
    assert st["replayed"] > 0 and st["rerun"] > 0 and st["protected"] < st["rounds"], st


def test_restore_point_renewed_between_batches():
    # a restore point older than the renewal interval is renewed
    # between the batches of one call too (not only at a call's entry), so an
    # ambiguous round late in a long call replays a bounded number of rounds.
    # With the interval at 8 rounds (test build) the one-call run renews it,
    # stays the oracle's bit for bit, and replays fewer rounds than with the
    # default interval
    far = run_hooked("engine_replay", 1, SHD_PROTECT_ALL=None, SHD_NO_PROTECT="1")
    near = run_hooked("engine_replay", 1, SHD_PROTECT_ALL=None, SHD_NO_PROTECT="1", SHD_RESTORE_EVERY="8")
    assert far["renewed"] == 0 and near["renewed"] > 0, (far, near)
    assert near["rerun"] > 0 and near["replayed"] <= far["replayed"], (far, near)


def test_product_library_ignores_the_test_hooks(monkeypatch):
    # the product build has no hooks: with the variables set, nothing is forced
    monkeypatch.setenv("SHD_FORCE_AMBIG", "1")
    monkeypatch.setenv("SHD_PROTECT_ALL", "1")
    g = W.geometric_graph(200, seed=4)
    m = W.phold_model(W.hosts_on_vertices(200, 1), end_time=2 * S.SHD_SEC, trace=True)
    gpu, ora, eng, _ = run_both(g, m)
    assert_same(gpu, ora)
    st = gpu[2]
    assert st.n_rounds_rerun == 0 and st.n_rounds_protected < st.n_rounds


def test_default_protection_covers_the_application_start():
    # without the hook: the rounds up to the first logging one, and those after
    # a round that logged >= 64 first touches, run behind a state copy
    g = W.geometric_graph(300, seed=2)
    m = W.phold_model(W.hosts_on_vertices(300, 1), end_time=3 * S.SHD_SEC, trace=True)
    gpu, ora, eng, _ = run_both(g, m)
    assert_same(gpu, ora)
    st = gpu[2]
    assert 0 < st.n_rounds_protected < st.n_rounds and st.n_rounds_rerun == 0
    assert st.n_batches_ticketless > 0


@pytest.mark.parametrize("kind", ["rows", "rows_shared_vertices", "complete"])
def test_per_path_packet_counters_match_oracle(kind):
    # incrementPathPacketCounter (topology.c:2053-2063, worker.c:296): every
    # passing send counts against the cached entry it was served from; the
    # counts of each unordered pair (both orientations summed: a direct entry
    # is keyed (min, max) here, by its first query in the reference) and of
    # each vertex's own entry must match the serial oracle
    if kind == "complete":
        g = W.bundled_graph()
        hv = np.random.default_rng(1).integers(0, g.n_vertices, 400).astype(np.int32)
        hv = np.sort(hv)
    else:
        g = W.geometric_graph(250, seed=8)
        hv = W.hosts_on_vertices(250, 2 if kind == "rows_shared_vertices" else 1)
    m = W.phold_model(hv, end_time=3 * S.SHD_SEC, queue_flags=S.SHD_QF_COUNT_PATHS)
    att = W.attached_vertices(m.host_vertex)
    pc = PathCache(g, att)
    eng = Engine(m, pc)
    st = eng.run()
    cnt = eng.path_counts()
    V = g.n_vertices
    ocnt = np.zeros((V, V), dtype=np.uint64)
    _, _, ost = O.engine_run(m, g, path_counts=ocnt)
    assert st.n_pkt_events == ost["n_pkt_events"]
    o = ocnt[np.ix_(att, att)]                       # attached indices
    sym = lambda c: np.triu(c + c.T, 1) + np.diag(np.diag(c))   # noqa: E731
    assert int(o.sum()) > 1000
    assert int(cnt.sum()) == int(o.sum())
    assert np.array_equal(sym(cnt), sym(o))


def test_bundled_complete_graph_many_hosts_per_vertex():
    g = W.bundled_graph()
    rng = np.random.default_rng(0)
    hv = np.sort(rng.integers(0, g.n_vertices, 400)).astype(np.int32)
    m = W.phold_model(hv, end_time=3 * S.SHD_SEC, trace=True, load=8)
    gpu, ora, _, _ = run_both(g, m)
    assert_same(gpu, ora)


def test_geometric_shared_vertices_rows_and_self_paths():
    g = W.geometric_graph(120, seed=4, vertex_loss=True)
    m = W.phold_model(W.hosts_on_vertices(120, 3), end_time=int(2.5 * S.SHD_SEC), trace=True)
    gpu, ora, _, _ = run_both(g, m)
    assert_same(gpu, ora)


def test_codel_drops_under_low_receive_bandwidth():
    g = W.geometric_graph(150, seed=8)
    m = W.phold_model(W.hosts_on_vertices(150, 1), end_time=4 * S.SHD_SEC, trace=True, load=24,
                      payload=1000, bw_down=600, bw_up=100000, codelq_cap=256)
    gpu, ora, _, _ = run_both(g, m)
    assert_same(gpu, ora)
    assert np.count_nonzero(gpu[0]["kind"] == S.TR_CODEL_DROP) > 0


def test_bootstrap_period_and_forced_rows_on_complete_graph():
    g = W.bundled_graph()
    hv = np.arange(0, g.n_vertices, 2, dtype=np.int32)
    m = W.phold_model(hv, end_time=3 * S.SHD_SEC, trace=True, bootstrap_end=2 * S.SHD_SEC, bw_down=100)
    gpu, ora, _, _ = run_both(g, m, force_rows=True)
    assert_same(gpu, ora)


def test_prefer_direct_paths():
    g = W.geometric_graph(200, seed=12)
    g2 = S.GraphArrays(g.n_vertices, g.src, g.dst, g.latency, g.loss, None, prefer_direct=True)
    m = W.phold_model(W.hosts_on_vertices(200, 1), end_time=3 * S.SHD_SEC, trace=True)
    gpu, ora, _, _ = run_both(g2, m)
    assert_same(gpu, ora)


def test_run_to_run_determinism():
    # reference determinism1/2 tests (src/test/determinism) compare two runs
    g = W.geometric_graph(500, seed=3)
    m = W.phold_model(W.hosts_on_vertices(500, 1), end_time=3 * S.SHD_SEC, trace=True)
    att = W.attached_vertices(m.host_vertex)
    pc = PathCache(g, att)
    outs = []
    for _ in range(2):
        e = Engine(m, pc)
        e.run()
        outs.append((sort_trace(e.trace()), e.digest()))
        e.close()
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("sph,kind", [(256, "geo"), (64, "geo"), (1024, "codel"), (192, "complete"), (64, "wide")])
def test_sparse_persistent_rounds_match_oracle(sph, kind, monkeypatch):
    """k_round_sp (the engines with more hosts than resident waves: the C5
    shard) forced on small models with SHD_SP_HOSTS: blocks of `sph` hosts scan
    their hosts, compact the active ones and run them 64 at a time (several
    passes a round at 1024 hosts per block); the result is the serial run's.
    "wide": 33 600 hosts in 525 blocks, more shares than one round trip of the
    gather polls (512)."""
    monkeypatch.setenv("SHD_SP_HOSTS", str(sph))
    if kind == "wide":
        g = W.geometric_graph(400, seed=2)
        m = W.phold_model(W.hosts_on_vertices(400, 84), end_time=int(1.3 * S.SHD_SEC), trace=True, load=2)
    elif kind == "complete":
        g = W.bundled_graph()
        hv = np.sort(np.random.default_rng(2).integers(0, g.n_vertices, 700)).astype(np.int32)
        m = W.phold_model(hv, end_time=3 * S.SHD_SEC, trace=True, load=8)
    elif kind == "codel":
        g = W.geometric_graph(300, seed=8)
        m = W.phold_model(W.hosts_on_vertices(300, 4), end_time=3 * S.SHD_SEC, trace=True, load=24,
                          payload=1000, bw_down=600, bw_up=100000, codelq_cap=256)
    else:
        g = W.geometric_graph(400, seed=2)
        m = W.phold_model(W.hosts_on_vertices(400, 2), end_time=3 * S.SHD_SEC, trace=True)
    gpu, ora, eng, _ = run_both(g, m)
    assert_same(gpu, ora)
    st = gpu[2]
    assert st.n_batches_sparse > 0 and st.n_batches_sparse == st.n_batches_persistent
    if kind == "codel":
        assert np.count_nonzero(gpu[0]["kind"] == S.TR_CODEL_DROP) > 0


@pytest.mark.parametrize("parts", [2, 3])
def test_sharded_engines_match_oracle(parts):
    """Hosts partitioned over several engines (DESIGN.md "Multi-GPU"): the
    exchanged events and the global first-touch resolution reproduce the
    serial run exactly."""
    from driver import LocalCluster, partition
    g = W.geometric_graph(240, seed=6)
    m = W.phold_model(W.hosts_on_vertices(240, 1), end_time=3 * S.SHD_SEC, trace=True)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    pb = partition(m.n_hosts, parts)
    engines = [Engine(m, pc, pb[i], pb[i + 1]) for i in range(parts)]
    cl = LocalCluster(engines, pb)
    cl.boot()
    res = cl.run_until(m.params["end_time"])
    assert res.exchanged > 0 and res.pending > 0
    tr = sort_trace(np.concatenate([e.trace() for e in engines]))
    dg = np.concatenate([e.digest() for e in engines])
    otr, odg, ost = O.engine_run(m, g)
    assert res.pkt_events == ost["n_pkt_events"]
    assert np.array_equal(tr, sort_trace(otr))
    assert np.array_equal(dg, odg)


@pytest.mark.parametrize("parts,block", [(2, 0), (3, 0), (4, 6), (2, 1)])
def test_engine_group_local_matches_oracle(parts, block):
    """shd_xgroup (one fixed-size all-to-all per round, device-driven batches)
    with the in-process transport: several engines on one GPU.  Small blocks
    force spills, so the halt + host delivery path runs too; stopping and
    resuming at arbitrary times must not change anything."""
    from driver import partition
    from sim import XGroup
    g = W.geometric_graph(240, seed=6)
    m = W.phold_model(W.hosts_on_vertices(240, 1), end_time=3 * S.SHD_SEC, trace=True)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    pb = partition(m.n_hosts, parts)
    engines = [Engine(m, pc, pb[i], pb[i + 1]) for i in range(parts)]
    grp = XGroup.local(engines, block_events=block)
    pkt = pend = 0
    for t in (int(0.7 * S.SHD_SEC), int(1.0 * S.SHD_SEC) + 3, 2 * S.SHD_SEC, m.params["end_time"]):
        st = grp.run_until(t)
        pkt += st.n_pkt_events
        pend += st.n_pending_resolved
    assert pend > 0
    tr = sort_trace(np.concatenate([e.trace() for e in engines]))
    dg = np.concatenate([e.digest() for e in engines])
    otr, odg, ost = O.engine_run(m, g)
    assert pkt == ost["n_pkt_events"]
    assert np.array_equal(tr, sort_trace(otr))
    assert np.array_equal(dg, odg)
    grp.close()


@pytest.mark.parametrize("parts", [2, 3])
def test_engine_group_ambiguous_rounds_roll_back(parts):
    """Protected rounds in the engine group: with every undecided first-touch
    send forced ambiguous and every round protected, each logging round is
    rolled back on every engine (exchange buffers included), ranked from the
    logs of all engines and rerun; the result is still the oracle's (checked
    in the child, tests/hook_worker.py)."""
    st = run_hooked("group_rollback", parts)
    assert st["rerun"] > 0 and st["protected"] >= st["rounds"]


def test_engine_group_rccl_single_rank():
    """The RCCL transport end to end with one rank (the multi-rank case needs
    one GPU per rank: RCCL refuses two ranks on one device)."""
    from sim import XGroup
    g = W.geometric_graph(200, seed=9)
    m = W.phold_model(W.hosts_on_vertices(200, 1), end_time=2 * S.SHD_SEC, trace=True)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc)
    grp = XGroup.rccl(eng, XGroup.unique_id(), 1, 0)
    st = grp.run()
    otr, odg, ost = O.engine_run(m, g)
    assert st.n_pkt_events == ost["n_pkt_events"]
    assert np.array_equal(sort_trace(eng.trace()), sort_trace(otr))
    assert np.array_equal(eng.digest(), odg)
    grp.close()


@pytest.mark.parametrize("kind", ["plain", "codel", "sharded"])
def test_heartbeat_node_counters_match_oracle(kind):
    """tracker_heartbeat (tracker.c:566-611): every host's interface counters at
    each heartbeat (in: network_interface.c:415, out: 571), trace off so the
    straight-line event paths run; the [node] lines follow from them."""
    from driver import partition
    from sim import XGroup
    end = int(4.5 * S.SHD_SEC)
    g = W.geometric_graph(200, seed=3)
    kw = dict(load=24, payload=1000, bw_down=600, bw_up=100000, codelq_cap=256) if kind == "codel" else {}
    m = W.phold_model(W.hosts_on_vertices(200, 1), end_time=end, queue_flags=S.SHD_QF_HEARTBEATS, **kw)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    if kind == "sharded":
        pb = partition(m.n_hosts, 3)
        engines = [Engine(m, pc, pb[i], pb[i + 1]) for i in range(3)]
        grp = XGroup.local(engines)
        grp.run()
        hb = np.concatenate([e.heartbeats() for e in engines])
        grp.close()
    else:
        eng = Engine(m, pc)
        eng.run()
        hb = eng.heartbeats()
    K = (end - 1) // S.SHD_SEC
    ohb = np.zeros((m.n_hosts, K, 2), dtype=np.uint32)
    O.engine_run(m, g, heartbeats=ohb)
    assert hb.shape == ohb.shape == (m.n_hosts, 4, 2)
    assert int(ohb[:, -1].sum()) > 1000
    assert np.array_equal(hb, ohb)
    lines = S.tracker_node_lines(hb[7], S.SHD_SEC, int(m.params["payload"]))
    assert lines == S.tracker_node_lines(ohb[7], S.SHD_SEC, int(m.params["payload"]))
