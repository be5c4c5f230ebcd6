"""The engine group across PROCESSES: `world` child processes, one engine
each, over the host-memory communicator (shd_comm_create_host; RCCL refuses
two ranks on one GPU, so this is how the multi-process group protocol runs on
a one-GPU box).  Every rank builds its share of the path cache's source rows
and all-gathers them (shd_pc_build_sharded, APSP sharded by source rows); the
group then runs the round protocol of shd_xgroup -- per-round all-to-all of
blocks with headers, halts, first-touch logs gathered from every rank, spills
delivered with the all-to-all-v, protected rounds -- with stops and resumes.
The union of the ranks' traces and host states must be the serial oracle's,
bit for bit, and every rank's table the single-process build's.
"""
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S
import workloads as W
from sim import PathCache, sort_trace

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


# the test build with the semantics-changing hooks (-DSHD_TEST_HOOKS), for the ranks that need one
TH_LIB = os.path.join(os.path.dirname(HERE), "shadow-1_amd", "libshdgpu_th.so")


def run_ranks(world, tmp_path, extra=(), env_extra=None, timeout=240):
    name = "shdtest_" + uuid.uuid4().hex[:16]
    env = dict(os.environ)
    env.update(env_extra or {})
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "xgroup_worker.py"), "--rank", str(r),
                               "--world", str(world), "--name", name, "--out", str(tmp_path)] + list(extra),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env)
             for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{outs[r][-3000:]}"
    return [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(world)]


def check_against_oracle(res, V, hpv, end_s, loss, load):
    g = W.geometric_graph(V, seed=6, loss_max=loss)
    m = W.phold_model(W.hosts_on_vertices(V, hpv), end_time=int(end_s * S.SHD_SEC), trace=True, load=load)
    otr, odg, ost = O.engine_run(m, g)
    tr = sort_trace(np.concatenate([r["trace"] for r in res]))
    dg = np.concatenate([r["digest"] for r in res])
    pkt = sum(int(r["stats"][0]) for r in res)
    assert pkt == ost["n_pkt_events"] > 0
    assert np.array_equal(tr, sort_trace(otr))
    assert np.array_equal(dg, odg)
    # the sharded tables are the one-process build's, on every rank
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    lat, rel = pc.rows()
    info = pc.info()
    for r in res:
        assert np.array_equal(r["lat"].view(np.uint64), lat.view(np.uint64))
        assert np.array_equal(r["rel"].view(np.uint64), rel.view(np.uint64))
        assert tuple(r["ties"].tolist()) == (info.n_ties, info.max_hops, info.sssp_iterations_max)
    pc.close()
    return res


@pytest.mark.parametrize("p2p", [False, True], ids=["alltoall", "p2p"])
@pytest.mark.parametrize("world,block", [(2, 0), (3, 0), (2, 4)])
def test_multiprocess_group_matches_oracle(world, block, p2p, tmp_path):
    """block 4: tiny per-peer blocks force spills (halts + the all-to-all-v,
    and regrown blocks: the peer-to-peer receive blocks are remapped).  p2p:
    each rank's receive blocks mapped by every rank and stored into directly,
    with tagged headers and in-kernel waits (on this box the ranks share one
    GPU: the protocol, not xGMI)."""
    res = run_ranks(world, tmp_path, extra=["--block", str(block)] + (["--p2p"] if p2p else []))
    check_against_oracle(res, 240, 1, 3.0, 0.01, 16)
    assert sum(int(r["stats"][2]) for r in res) > 0          # first-touch logs resolved across ranks
    rounds = {int(r["stats"][3]) for r in res}
    assert len(rounds) == 1                                    # every rank ran the same rounds


@pytest.mark.parametrize("world,hpv", [(4, 1), (3, 3), (9, 1)])
def test_multiprocess_p2p_fused_rounds(world, hpv, tmp_path):
    """The fused peer-to-peer schedule with more ranks than round-kernel blocks
    (4 ranks of 60 hosts: one block each, the launch padded to a put block per
    peer), with several blocks per rank (3 x 240 hosts: 4 blocks, events
    sorted into per-destination-block regions of every peer), and with more
    than eight peers (9 ranks: the regions of peers past the eighth are taken
    by the round's second ingest pass)."""
    res = run_ranks(world, tmp_path, extra=["--p2p", "--hpv", str(hpv)])
    check_against_oracle(res, 240, hpv, 3.0, 0.01, 16)
    assert len({int(r["stats"][3]) for r in res}) == 1


@pytest.mark.parametrize("world,hpv", [(2, 1), (3, 3)])
def test_multiprocess_p2p_sparse_rounds(world, hpv, tmp_path):
    """k_round_spx, the sparse fused round, forced (SHD_SP_HOSTS=64: blocks of
    64 hosts scanned and compacted): each round takes the peers' stores for its
    blocks' hosts into their calendars / inboxes before the scan, and its own
    sends for other ranks go into their regions as k_round_px's do"""
    res = run_ranks(world, tmp_path, extra=["--p2p", "--hpv", str(hpv)], env_extra={"SHD_SP_HOSTS": "64"})
    check_against_oracle(res, 240, hpv, 3.0, 0.01, 16)
    assert len({int(r["stats"][3]) for r in res}) == 1


@pytest.mark.parametrize("p2p", [False, True], ids=["alltoall", "p2p"])
def test_multiprocess_group_tor_model(p2p, tmp_path):
    """BASELINE C4's relay/client model over 3 processes: per-class destination
    weights (each PHOLD process's weights file), hosts attached at random on
    the bundled (complete) topology, the relays -- most of the traffic -- all
    on rank 0, so the exchange is lopsided.  Bit-exact vs the serial oracle."""
    R, C, load = 40, 200, 4
    res = run_ranks(3, tmp_path, extra=["--tor", f"{R},{C}", "--load", str(load), "--end-s", "2.5"] +
                    (["--p2p"] if p2p else []))
    g, m = W.tor_model(R, C, end_time=int(2.5 * S.SHD_SEC), trace=True, load=load)
    otr, odg, ost = O.engine_run(m, g)
    tr = sort_trace(np.concatenate([r["trace"] for r in res]))
    dg = np.concatenate([r["digest"] for r in res])
    assert sum(int(r["stats"][0]) for r in res) == ost["n_pkt_events"] > 0
    assert np.array_equal(tr, sort_trace(otr))
    assert np.array_equal(dg, odg)
    assert len({int(r["stats"][3]) for r in res}) == 1


@pytest.mark.parametrize("p2p", [False, True], ids=["alltoall", "p2p"])
def test_multiprocess_group_rolls_back_ambiguous_rounds(p2p, tmp_path):
    """Every undecided first-touch send forced ambiguous and every round
    protected: each logging round is rolled back on every process from its
    state copy, ranked from the logs all-gathered from every rank, rerun
    (p2p: the rerun's exchanges take new tags)."""
    res = run_ranks(2, tmp_path, extra=["--vertices", "160", "--hpv", "2"] + (["--p2p"] if p2p else []),
                    env_extra={"SHD_FORCE_AMBIG": "1", "SHD_PROTECT_ALL": "1", "SHDGPU_LIB": TH_LIB})
    check_against_oracle(res, 160, 2, 3.0, 0.01, 16)
    assert all(int(r["stats"][5]) > 0 for r in res)            # reruns happened on every rank


def test_p2p_self_check_failure_fails_every_rank_alike(tmp_path):
    """The peer-to-peer mapping's self-check (round 6): every rank puts a known
    granule into every peer's receive block over the mapping and each receiver
    checks what came.  A rank that puts a wrong one (test hook) fails the
    check at its peers: every rank gets SHD_ENODEV from
    shd_xgroup_create_p2p alike, falls back to the all-to-all transport, and
    the run still matches the oracle."""
    res = run_ranks(2, tmp_path, extra=["--p2p"], env_extra={"SHD_P2P_PROBE_CORRUPT": "1", "SHDGPU_LIB": TH_LIB})
    check_against_oracle(res, 240, 1, 3.0, 0.01, 16)
    assert all(int(r["stats"][6]) == 1 for r in res)


def test_p2p_mapping_failure_on_one_rank_fails_every_rank_alike(tmp_path):
    """A rank that cannot map its peers' receive blocks (test hook) takes part
    in both all-gathers of the mapping: every rank gets SHD_ENODEV from
    shd_xgroup_create_p2p, none waits forever, and all fall back to the
    all-to-all transport (as bench.py does) and still match the oracle."""
    res = run_ranks(2, tmp_path, extra=["--p2p"], env_extra={"SHD_P2P_FAIL_RANK": "1", "SHDGPU_LIB": TH_LIB})
    check_against_oracle(res, 240, 1, 3.0, 0.01, 16)
    assert all(int(r["stats"][6]) == 1 for r in res)
