"""Event-loop parity at BASELINE's full sizes against oracle fixtures.

tests/golden/make_fullsize.py ran the serial oracle (the reference's
--workers 0 loop restated) on each configuration of tests/fullsize_configs.py
and committed what the HIP engine must reproduce bit for bit:

* C1  the bundled example config (2 hosts, 1-vertex topology) through the
      config front-end: the full trace and both host digests;
* C3  the bench's headline (10 k hosts on the 10 k-vertex graph, lossless) and
      its lossy run (edge loss U[0, 0.0005]), 3 simulated seconds: every host's
      digest and trace multiset hash, on one engine and on groups of 2 and 4
      engines sharded as bench.py --gpus N shards them;
* C5  1 M hosts with CoDel queues building (1500-B payloads, rx 512 KiB/s):
      digest hashes per 1024-host block and the counter sums, on one engine and
      on a 2-engine group.

Beyond the fixtures, the bench workloads at N = 1..8 (N x 10 k hosts) sharded
over N engines must equal one engine running all the hosts (the reference's
determinism tests compare runs the same way, src/test/determinism).
"""
import os

import numpy as np
import pytest

import fixture_hash as FH
import shdgpu as S
import workloads as W
from fullsize_configs import CONFIGS, V, build, c3_hosts
from sim import Engine, PathCache, XGroup, sort_trace

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture(key):
    return np.load(os.path.join(GOLDEN, CONFIGS[key]["file"]))


def run_engines(m, pc, parts, pushes=None):
    """One engine (parts = 1) or a local group of `parts` engines; returns
    (stats, engines, group or None)."""
    from driver import partition
    if parts == 1:
        e = Engine(m, pc)
        if pushes is not None:
            e.boot()
            e.push_events(pushes)
        return e.run(), [e], None
    pb = partition(m.n_hosts, parts)
    engines = [Engine(m, pc, pb[i], pb[i + 1]) for i in range(parts)]
    if pushes is not None:
        for e in engines:
            e.boot()
            mine = pushes[(pushes["dst"] >= e.h0) & (pushes["dst"] < e.h1)]
            e.push_events(mine)
    grp = XGroup.local(engines)
    return grp.run(), engines, grp


def close_all(engines, grp):
    if grp is not None:
        grp.close()
    for e in engines:
        e.close()


@pytest.mark.parametrize("parts", [1, 2])
def test_c1_example_config_matches_oracle_fixture(parts):
    fx = fixture("c1")
    g, m, pushes = build("c1")
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    st, engines, grp = run_engines(m, pc, parts, pushes)
    assert st.error == 0
    tr = sort_trace(np.concatenate([e.trace() for e in engines]))
    dg = np.concatenate([e.digest() for e in engines])
    assert (st.n_events, st.n_pkt_events) == tuple(int(x) for x in fx["totals"][:2])
    assert np.array_equal(tr, sort_trace(fx["trace"]))
    assert np.array_equal(dg, fx["digest"])
    close_all(engines, grp)
    pc.close()


@pytest.fixture(scope="module", params=["c3", "c3_lossy"])
def c3(request):
    g, m, _ = build(request.param)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    yield request.param, m, pc
    pc.close()


@pytest.mark.parametrize("parts", [1, 2, 4])
def test_c3_full_size_matches_oracle_fixture(c3, parts):
    key, m, pc = c3
    fx = fixture(key)
    st, engines, grp = run_engines(m, pc, parts)
    assert st.error == 0
    tr = np.concatenate([e.trace() for e in engines])
    dg = np.concatenate([e.digest() for e in engines])
    n_ev, n_pkt, n_tr = (int(x) for x in fx["totals"])
    assert (st.n_events, st.n_pkt_events, len(tr)) == (n_ev, n_pkt, n_tr)
    assert n_pkt > 1_000_000
    assert np.array_equal(dg, fx["digest"])
    th = FH.trace_host_hashes(tr, m.n_hosts)
    bad = np.nonzero(th != fx["trace_hash"])[0]
    assert len(bad) == 0, f"{len(bad)} hosts' traces differ, first {bad[:8]}"
    close_all(engines, grp)


@pytest.mark.parametrize("parts", [1, 2])
def test_c5_codel_million_hosts_matches_oracle_fixture(parts):
    cfg = CONFIGS["c5"]
    fx = fixture("c5")
    g, m, _ = build("c5")
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    st, engines, grp = run_engines(m, pc, parts)
    assert st.error == 0
    dg = np.concatenate([e.digest() for e in engines])
    close_all(engines, grp)
    pc.close()
    n_ev, n_pkt, _ = (int(x) for x in fx["totals"])
    assert (st.n_events, st.n_pkt_events) == (n_ev, n_pkt)
    sums = [int(dg[f].sum()) for f in ("n_events", "n_pkt_events", "n_sent", "n_inet_drop", "n_codel_drop",
                                       "n_recv")]
    assert sums == [int(x) for x in fx["sums"]]
    assert sums[4] > 100_000                   # CoDel dropped: the queues built
    bh = FH.digest_block_hashes(dg, cfg["block"])
    bad = np.nonzero(bh != fx["block_hash"])[0]
    assert len(bad) == 0, f"{len(bad)} host blocks differ, first {bad[:8]}"


def test_bench_headline_run_to_run_deterministic():
    g = W.geometric_graph(V, seed=1, loss_max=0.0)
    m = W.phold_model(c3_hosts(V), end_time=3 * S.SHD_SEC, seed=1, load=16, payload=1)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    outs = []
    for _ in range(2):
        e = Engine(m, pc)
        st = e.run()
        outs.append(((st.n_events, st.n_pkt_events, st.n_rounds, st.n_host_rounds), e.digest()))
        e.close()
    assert outs[0][0] == outs[1][0] and np.array_equal(outs[0][1], outs[1][1])
    d1 = outs[0][1]
    assert int(d1["n_pkt_events"].sum()) == outs[0][0][1]
    # active host-rounds (bench.py's roofline bytes): at most one per host per
    # round, at most one per event
    n_ev, _, n_rounds, n_hr = outs[0][0]
    assert 0 < n_hr <= min(n_ev, n_rounds * m.n_hosts)
    pc.close()


@pytest.mark.parametrize("hosts,parts", [(2 * V, 2), (4 * V, 4), (8 * V, 8)])
def test_bench_workload_sharded_group_equals_single_engine(hosts, parts):
    """(N V, N) is bench.py --gpus N's workload (weak scaling: N x 10 k hosts on the
    same graph), sharded as its N ranks shard it."""
    from driver import partition
    g = W.geometric_graph(V, seed=1, loss_max=0.0)
    m = W.phold_model(c3_hosts(hosts), end_time=3 * S.SHD_SEC, seed=1, load=16, payload=1)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    e = Engine(m, pc)
    st = e.run()
    d1 = e.digest()
    e.close()
    pb = partition(m.n_hosts, parts)
    engines = [Engine(m, pc, pb[i], pb[i + 1]) for i in range(parts)]
    grp = XGroup.local(engines)
    gst = grp.run()
    dg = np.concatenate([x.digest() for x in engines])
    assert gst.error == 0
    assert gst.n_pkt_events == st.n_pkt_events and gst.n_events == st.n_events
    assert gst.n_host_rounds == st.n_host_rounds   # the same rounds, the same active hosts
    assert np.array_equal(dg, d1)
    close_all(engines, grp)
    pc.close()


def run_one_rank_p2p(m, pc):
    """the engine group's fused peer-to-peer schedule with one rank (bench.py
    --group): an RCCL communicator of one, the whole model on its engine"""
    from sim import Comm
    e = Engine(m, pc)
    comm = Comm.rccl(XGroup.unique_id(), 1, 0, 0)
    grp = XGroup.over(e, comm, p2p=True)
    st = grp.run()
    return st, e, grp, comm


@pytest.mark.parametrize("sp", ["auto", "forced"])
def test_c3_full_size_sparse_group_rounds_match_fixture(c3, sp, monkeypatch):
    """k_round_spx (the sparse fused group round): C3 through a one-rank
    peer-to-peer group with the sparse kernel forced (SHD_SP_HOSTS: blocks of
    256 hosts) or as the group picks it (auto: 157 blocks of 64 hosts fit the
    GPU, so k_round_px) -- the fixture's digests and traces either way"""
    key, m, pc = c3
    if sp == "forced":
        monkeypatch.setenv("SHD_SP_HOSTS", "256")
    fx = fixture(key)
    st, e, grp, comm = run_one_rank_p2p(m, pc)
    assert st.error == 0
    tr = e.trace()
    dg = e.digest()
    n_ev, n_pkt, n_tr = (int(x) for x in fx["totals"])
    assert (st.n_events, st.n_pkt_events, len(tr)) == (n_ev, n_pkt, n_tr)
    assert np.array_equal(dg, fx["digest"])
    th = FH.trace_host_hashes(tr, m.n_hosts)
    assert np.array_equal(th, fx["trace_hash"])
    grp.close(); e.close(); comm.close()


def test_c5_codel_million_hosts_sparse_group_rounds_match_fixture():
    """The north star's model through the one-rank fused group: 15 625 blocks
    of 64 hosts, so k_round_spx runs the sparse rounds (blocks of ~4 k hosts,
    one per CU) -- bit-exact against the full-size oracle fixture"""
    cfg = CONFIGS["c5"]
    fx = fixture("c5")
    g, m, _ = build("c5")
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    st, e, grp, comm = run_one_rank_p2p(m, pc)
    assert st.error == 0
    dg = e.digest()
    grp.close(); e.close(); comm.close()
    pc.close()
    n_ev, n_pkt, _ = (int(x) for x in fx["totals"])
    assert (st.n_events, st.n_pkt_events) == (n_ev, n_pkt)
    bh = FH.digest_block_hashes(dg, cfg["block"])
    assert np.array_equal(bh, fx["block_hash"])


def test_c5_protected_rounds_with_the_state_copy_in_host_memory():
    """The protected rounds' state copy falls back to host memory when device
    memory is exhausted (test build: SHD_SNAP_NO_DEVICE makes every device
    allocation of the copy fail): the 1 M-host C5 run keeps its protected
    rounds and still equals the oracle fixture bit for bit (checked in the
    child, tests/hook_worker.py c5_snap_host)."""
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, SHD_SNAP_NO_DEVICE="1", SHD_VERBOSE="1",
               SHDGPU_LIB=os.path.join(os.path.dirname(here), "shadow-1_amd", "libshdgpu_th.so"))
    p = subprocess.run([sys.executable, "-u", os.path.join(here, "hook_worker.py"), "c5_snap_host", "0"], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=900)
    out = p.stdout.decode(errors="replace")
    assert p.returncode == 0, out[-3000:]
    assert "state copy in host memory" in out, out[-2000:]
    st = json.loads(out.strip().splitlines()[-1])
    assert st["protected"] > 0, st
