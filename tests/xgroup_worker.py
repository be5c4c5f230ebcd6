#!/usr/bin/env python3
"""One rank of a multi-process engine group -- TEST INFRASTRUCTURE
(tests/test_xgroup_procs_gpu.py starts `world` of these as child processes).

Each rank builds the same model, creates a host-memory communicator
(shd_comm_create_host), builds the path cache with its source rows sharded
over the ranks and all-gathered (shd_pc_build_sharded), runs its engine in a
group over that communicator (shd_xgroup_create, or shd_xgroup_create_p2p:
receive blocks mapped by IPC handle) with stops and resumes, and
writes its trace, host digests and the full row table to <out>/rank<r>.npz.
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(HERE), "shadow-1_amd"), HERE]

import numpy as np  # noqa: E402


def model(V, hpv, end, loss, load, tor=None):
    import shdgpu as S
    import workloads as W
    if tor:   # the Tor-scale relay/client model (per-class destination weights) on the bundled topology
        return W.tor_model(tor[0], tor[1], end_time=end, trace=True, load=load)
    g = W.geometric_graph(V, seed=6, loss_max=loss)
    m = W.phold_model(W.hosts_on_vertices(V, hpv), end_time=end, trace=True, load=load)
    return g, m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--name", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--vertices", type=int, default=240)
    ap.add_argument("--hpv", type=int, default=1)
    ap.add_argument("--end-s", type=float, default=3.0)
    ap.add_argument("--loss", type=float, default=0.01)
    ap.add_argument("--load", type=int, default=16)
    ap.add_argument("--block", type=int, default=0)
    ap.add_argument("--p2p", action="store_true", help="the peer-to-peer transport (shd_xgroup_create_p2p)")
    ap.add_argument("--tor", default="", help="R,C: the Tor-scale model with R relays and C clients")
    a = ap.parse_args()
    import shdgpu as S
    import workloads as W
    from driver import partition
    from sim import Comm, Engine, PathCache, XGroup
    end = int(a.end_s * S.SHD_SEC)
    tor = tuple(int(x) for x in a.tor.split(",")) if a.tor else None
    g, m = model(a.vertices, a.hpv, end, a.loss, a.load, tor)
    comm = Comm.host(a.name, a.world, a.rank, device=0)
    pc = PathCache(g, W.attached_vertices(m.host_vertex), build=False)
    pc.build_sharded(comm)
    info = pc.info()
    # (a complete graph keeps only the direct table: no rows to compare)
    lat, rel = pc.rows() if not info.is_complete else (np.zeros(0), np.zeros(0))
    pb = partition(m.n_hosts, a.world)
    eng = Engine(m, pc, pb[a.rank], pb[a.rank + 1])
    fallback = 0
    try:
        grp = XGroup.over(eng, comm, block_events=a.block, p2p=a.p2p)
    except S.ShdError:   # the peer-to-peer mapping failed on some rank: every rank falls back alike
        if not a.p2p:
            raise
        fallback = 1
        grp = XGroup.over(eng, comm, block_events=a.block)
    pkt = ev = pend = rounds = prot = rerun = 0
    for t in (int(0.7 * S.SHD_SEC), S.SHD_SEC + 3, 2 * S.SHD_SEC, end):
        st = grp.run_until(min(t, end))
        pkt += st.n_pkt_events
        ev += st.n_events
        pend += st.n_pending_resolved
        rounds += st.n_rounds
        prot += st.n_rounds_protected
        rerun += st.n_rounds_rerun
    np.savez(os.path.join(a.out, f"rank{a.rank}.npz"), trace=eng.trace(), digest=eng.digest(), lat=lat, rel=rel,
             stats=np.array([pkt, ev, pend, rounds, prot, rerun, fallback], dtype=np.uint64),
             ties=np.array([info.n_ties, info.max_hops, info.sssp_iterations_max], dtype=np.int64))
    grp.close()
    eng.close()
    pc.close()
    comm.close()
    print(f"rank {a.rank}: {pkt} packet events, {rounds} rounds", flush=True)


if __name__ == "__main__":
    main()
