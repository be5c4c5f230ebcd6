#!/usr/bin/env python3
"""Scenarios that need a semantics-changing test hook -- TEST INFRASTRUCTURE.

The hooks (SHD_FORCE_AMBIG: every undecided first-touch send counts as
ambiguous; SHD_PROTECT_ALL: every round behind a state copy) exist only in the
test build libshdgpu_th.so (-DSHD_TEST_HOOKS).  tests/test_engine_gpu.py runs
each scenario here in a child process with SHDGPU_LIB pointing at that build,
so the pytest process itself only ever loads the product library.  The child
checks the run against the serial oracle bit for bit and prints one JSON line
of run statistics; any mismatch is an assertion (non-zero exit).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(HERE), "shadow-1_amd"), HERE]

import numpy as np  # noqa: E402


def engine_rollback(hpv):
    import oracle_ffi as O
    import workloads as W
    import shdgpu as S
    from sim import Engine, PathCache, sort_trace
    g = W.geometric_graph(200, seed=4)
    m = W.phold_model(W.hosts_on_vertices(200, hpv), end_time=3 * S.SHD_SEC, trace=True)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc)
    st = eng.run()
    otr, odg, ost = O.engine_run(m, g)
    assert st.n_events == ost["n_events"] and st.n_pkt_events == ost["n_pkt_events"]
    assert np.array_equal(sort_trace(eng.trace()), sort_trace(otr))
    assert np.array_equal(eng.digest(), odg)
    return dict(rerun=st.n_rounds_rerun, protected=st.n_rounds_protected, rounds=st.n_rounds)


def group_rollback(parts):
    import oracle_ffi as O
    import workloads as W
    import shdgpu as S
    from driver import partition
    from sim import Engine, PathCache, XGroup, sort_trace
    g = W.geometric_graph(200, seed=5)
    m = W.phold_model(W.hosts_on_vertices(200, 2), end_time=3 * S.SHD_SEC, trace=True)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    pb = partition(m.n_hosts, parts)
    engines = [Engine(m, pc, pb[i], pb[i + 1]) for i in range(parts)]
    grp = XGroup.local(engines)
    pkt = rerun = prot = rounds = 0
    for t in (int(1.0 * S.SHD_SEC) + 3, m.params["end_time"]):
        st = grp.run_until(t)
        pkt += st.n_pkt_events
        rerun += st.n_rounds_rerun
        prot += st.n_rounds_protected
        rounds += st.n_rounds
    tr = sort_trace(np.concatenate([e.trace() for e in engines]))
    dg = np.concatenate([e.digest() for e in engines])
    otr, odg, ost = O.engine_run(m, g)
    assert pkt == ost["n_pkt_events"]
    assert np.array_equal(tr, sort_trace(otr))
    assert np.array_equal(dg, odg)
    grp.close()
    return dict(rerun=rerun, protected=prot, rounds=rounds)


def engine_replay(steps):
    """SHD_FORCE_AMBIG with SHD_NO_PROTECT: no round runs behind a copy of its
    own, so every round that logs an undecided first-touch send is an
    ambiguous unprotected round; each is recovered by replaying from the last
    restore point (shd_eng_run_until) and must leave the run the oracle's.
    steps > 1: the run is split into that many run_until calls."""
    import oracle_ffi as O
    import workloads as W
    import shdgpu as S
    from sim import Engine, PathCache, sort_trace
    g = W.geometric_graph(200, seed=4)
    m = W.phold_model(W.hosts_on_vertices(200, 2), end_time=3 * S.SHD_SEC, trace=True)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc)
    end = m.params["end_time"]
    tot = dict(replayed=0, rerun=0, protected=0, rounds=0, pkt=0, events=0, renewed=0, max_replay=0)
    for k in range(1, steps + 1):
        st = eng.run_until(end * k // steps)
        tot["replayed"] += st.n_rounds_replayed
        tot["renewed"] += st.n_restore_points
        tot["rerun"] += st.n_rounds_rerun
        tot["protected"] += st.n_rounds_protected
        tot["rounds"] += st.n_rounds
        tot["pkt"] += st.n_pkt_events
        tot["events"] += st.n_events
    otr, odg, ost = O.engine_run(m, g)
    assert tot["events"] == ost["n_events"] and tot["pkt"] == ost["n_pkt_events"], (tot, ost)
    assert np.array_equal(sort_trace(eng.trace()), sort_trace(otr))
    assert np.array_equal(eng.digest(), odg)
    return tot


def c5_snap_host(_):
    """SHD_SNAP_NO_DEVICE: the protected-round state copy cannot take device
    memory (as on a full device), so it goes to host memory; the 1 M-host C5
    model with CoDel queues building, its first-touch rounds protected behind
    that copy, must still equal the committed oracle fixture."""
    import fixture_hash as FH
    import workloads as W
    from fullsize_configs import CONFIGS, build
    from sim import Engine, PathCache
    cfg = CONFIGS["c5"]
    fx = np.load(os.path.join(HERE, "golden", cfg["file"]))
    g, m, _ = build("c5")
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc)
    st = eng.run()
    assert st.error == 0
    dg = eng.digest()
    n_ev, n_pkt, _ = (int(x) for x in fx["totals"])
    assert (st.n_events, st.n_pkt_events) == (n_ev, n_pkt), (st.n_events, st.n_pkt_events, n_ev, n_pkt)
    bh = FH.digest_block_hashes(dg, cfg["block"])
    bad = np.nonzero(bh != fx["block_hash"])[0]
    assert len(bad) == 0, f"{len(bad)} host blocks differ, first {bad[:8]}"
    return dict(protected=int(st.n_rounds_protected), rerun=int(st.n_rounds_rerun), rounds=int(st.n_rounds))


SCENARIOS = {"engine_rollback": engine_rollback, "group_rollback": group_rollback, "engine_replay": engine_replay,
             "c5_snap_host": c5_snap_host}


def main():
    import shdgpu as S
    assert os.path.basename(S.LIB_PATH) == "libshdgpu_th.so", S.LIB_PATH
    name, arg = sys.argv[1], int(sys.argv[2])
    print(json.dumps(SCENARIOS[name](arg)))


if __name__ == "__main__":
    main()
