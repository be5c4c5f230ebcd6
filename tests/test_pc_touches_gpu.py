"""The CPU side's half of the one-cache protocol on the product's path cache
(include/shdgpu.h shd_pc_defer_touches / shd_pc_query_key / shd_pc_take_touches:
the calls a topology adapter makes when its host's lookups share one lazy
cache with an engine, INTEGRATION.md "Mixed CPU/GPU hosts").

The oracle's lazy cache (oracle/o_pathcache.c, the restatement of
topology.c:1969-2051) is fed the same engine first touches and CPU-side
queries in ONE serial order (event_compare's key); the product cache gets the
engine's touches of each window up front and the CPU side's queries one event
at a time.  The CPU side's values must be the oracle's bit for bit, and the
first touches it reports must be exactly the queries that ran a row in the
oracle.  On the directed graph (tests/test_ingress_gpu.py) and on the grid
(equal-cost paths: each endpoint's row takes its own, with its own
reliability) which endpoint ranks first decides a pair's value.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S
import workloads as W
from sim import PathCache
from test_ingress_gpu import directed_graph

pytestmark = pytest.mark.gpu


def _key(r):
    return (int(r["qtime"]), int(r["qhost"]), int(r["qsrc"]), int(r["qseq"]), int(r["qsub"]))


def _records(rng, n, t0, hosts, T):
    r = np.zeros(n, S.PENDING_DTYPE)
    r["qtime"] = t0 + rng.integers(0, 1000, n)
    r["qhost"] = rng.integers(hosts[0], hosts[1], n)
    r["qsrc"] = rng.integers(0, 40, n)
    r["qseq"] = rng.integers(0, 1 << 20, n)
    r["a"] = rng.integers(0, T, n)
    r["b"] = rng.integers(0, T, n)
    return r


@pytest.mark.parametrize("graph", ["directed", "grid"])
@pytest.mark.parametrize("seed", [11, 12])
def test_pc_touch_protocol_is_one_serial_cache(seed, graph):
    g = directed_graph() if graph == "directed" else W.grid_graph()
    rng = np.random.default_rng(seed)
    hv = np.sort(rng.integers(0, g.n_vertices, 40)).astype(np.int32)
    att = W.attached_vertices(hv)
    T = len(att)
    pc = PathCache(g, att)
    ot = O.OTopo(O.OGraph(g), att)
    n_logged = n_diff = 0
    for w in range(40):
        t0 = w * 1000
        eng = _records(rng, int(rng.integers(0, 8)), t0, (20, 40), T)    # the engine's first touches
        cpu = _records(rng, int(rng.integers(1, 12)), t0, (0, 20), T)    # CPU-side queries, one per event
        cpu = cpu[sorted(range(len(cpu)), key=lambda i: _key(cpu[i]))]
        # the oracle: both sides in one serial order
        o_vals, o_log = [], []
        items = sorted([(_key(r), 0, r) for r in eng] + [(_key(r), 1, r) for r in cpu], key=lambda x: x[:2])
        for _, side, r in items:
            s, d = att[r["a"]], att[r["b"]]
            if side == 0:
                ot.touch(s, d)
                continue
            if ot.would_run(s, d):
                o_log.append((_key(r), int(r["a"]), int(r["b"])))
            o_vals.append(ot.get(s, d))
        # the product cache: the engine's touches first, the CPU side's queries event by event
        e = np.ascontiguousarray(eng)
        S.check(S.lib().shd_pc_defer_touches(pc.ptr, e.ctypes.data if len(e) else None, len(e)), "defer")
        vals = []
        for r in cpu:
            S.check(S.lib().shd_pc_query_key(pc.ptr, int(r["qtime"]), int(r["qhost"]), int(r["qsrc"]),
                                             int(r["qseq"])), "query_key")
            vals.append(pc.lookup(att[r["a"]], att[r["b"]]))
        n = C.c_uint64()
        S.check(S.lib().shd_pc_take_touches(pc.ptr, None, 0, C.byref(n)), "take")
        out = np.zeros(n.value, S.PENDING_DTYPE)
        S.check(S.lib().shd_pc_take_touches(pc.ptr, out.ctypes.data if n.value else None, n.value, C.byref(n)),
                "take")
        assert [(_key(r), int(r["a"]), int(r["b"])) for r in out] == o_log
        assert np.array_equal(np.array(vals).view(np.uint64), np.array(o_vals).view(np.uint64))
        n_logged += len(o_log)
        # where the orientations differ, the order decided the value
        n_diff += sum(1 for r in cpu if pc_rows_differ(pc, att, r))
    assert n_logged > 5
    assert n_diff > 0
    pc.close()


def pc_rows_differ(pc, att, r):
    """row a's and row b's values of the pair differ (the pair's two orientations)"""
    a, b = int(r["a"]), int(r["b"])
    if a == b:
        return False
    la, ra = pc.rows(a, 1)
    lb, rb = pc.rows(b, 1)
    return la[0, b] != lb[0, a] or ra[0, b] != rb[0, a]
