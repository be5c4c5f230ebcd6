"""Path-cache parity on the GPU: libshdgpu tables vs the oracle, bit for bit.

Reference: src/main/routing/topology.c (rows 1655-1875 + 1407-1523, direct
1877-1927, self 1545-1653, lazy selection 1969-2051).
"""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S
import workloads as W
from pc_helpers import PathCache, same_bits

pytestmark = pytest.mark.gpu

SHD_PC_FORCE_ROWS = 1


def oracle_rows(g, attached, rows):
    og = O.OGraph(g)
    lat = np.empty((len(rows), len(attached))); rel = np.empty_like(lat)
    ties = 0
    for k, r in enumerate(rows):
        l, rr, ok, hops, t = og.row(attached[r], attached)
        l[ok == 0] = -1.0; rr[ok == 0] = -1.0
        lat[k], rel[k] = l, rr
        ties += t
    return lat, rel, ties


def test_bundled_direct_mode_bit_exact():
    g = W.bundled_graph()
    att = np.arange(g.n_vertices, dtype=np.int32)
    pc = PathCache(g, att)
    info = pc.info()
    assert info.is_complete == 1 and info.rows_computed == 0
    lat, rel = pc.direct()
    og = O.OGraph(g)
    olat = np.empty_like(lat); orel = np.empty_like(rel)
    for i, s in enumerate(att):
        for j, d in enumerate(att):
            olat[i, j], orel[i, j] = og.direct(s, d)
    assert same_bits(lat, olat) and same_bits(rel, orel)
    # reference mode: the lazy lookup serves direct paths
    for s, d in [(0, 5), (5, 0), (17, 17), (182, 3)]:
        assert pc.lookup(s, d) == (olat[s, d], orel[s, d])


def test_bundled_forced_rows_bit_exact():
    g = W.bundled_graph()
    att = np.arange(g.n_vertices, dtype=np.int32)
    pc = PathCache(g, att, flags=SHD_PC_FORCE_ROWS)
    info = pc.info()
    assert info.rows_computed == g.n_vertices
    lat, rel = pc.rows()
    olat, orel, ties = oracle_rows(g, att, range(len(att)))
    assert info.n_ties == ties
    assert same_bits(lat, olat) and same_bits(rel, orel)
    # the 737 off-diagonal pairs where the shortest path is not the direct edge
    dl, _ = pc.direct()
    off = ~np.eye(len(att), dtype=bool)
    assert int(np.sum(np.triu(lat < dl, 1))) == 737


@pytest.mark.parametrize("V,seed,vloss", [(2000, 11, "all"), (3000, 5, "all"), (3000, 5, "none"),
                                           (2500, 3, "mixed"), (10000, 1, "none")])
def test_geometric_rows_bit_exact(V, seed, vloss):
    # "none": every target takes the tree-prefix reliability; "all": every
    # target has a vertex factor and walks its chain; "mixed": both in one row
    g = W.geometric_graph(V, seed=seed, vertex_loss=vloss != "none")
    if vloss == "mixed":
        vl = g.vertex_loss.copy()
        vl[::2] = np.nan          # attribute absent on even vertices
        g = S.GraphArrays(V, g.src, g.dst, g.latency, g.loss, vl)
    att = np.arange(V, dtype=np.int32)
    pc = PathCache(g, att)
    info = pc.info()
    assert info.is_complete == 0 and info.rows_computed == V
    assert info.n_ties == 0 and info.n_tie_rows == 0   # tie-free: one pass, no heap rerun
    rows = list(range(0, V, max(1, V // 64))) + [V - 1]
    lat, rel = pc.rows()
    olat, orel, ties = oracle_rows(g, att, rows)
    assert same_bits(lat[rows], olat) and same_bits(rel[rows], orel)
    slat, srel = pc.self_values()
    og = O.OGraph(g)
    ref = np.array([og.self_path(v) for v in att])
    assert same_bits(slat, ref[:, 0]) and same_bits(srel, ref[:, 1])


def test_geometric_subset_attached_and_global_scratch_path():
    # V above the LDS capacity (14 B/vertex > 160 KiB) -> global-memory kernel
    V = 12500
    g = W.geometric_graph(V, seed=7)
    rng = np.random.default_rng(0)
    att = np.sort(rng.choice(V, 300, replace=False)).astype(np.int32)
    pc = PathCache(g, att)
    lat, rel = pc.rows()
    rows = list(range(0, len(att), 10))
    olat, orel, _ = oracle_rows(g, att, rows)
    assert same_bits(lat[rows], olat) and same_bits(rel[rows], orel)


def test_lazy_lookup_first_touch_matches_reference_cache():
    g = W.geometric_graph(400, seed=9, vertex_loss=True)
    att = np.arange(400, dtype=np.int32)
    pc = PathCache(g, att)
    ot = O.OTopo(O.OGraph(g), att)
    rng = np.random.default_rng(1)
    for _ in range(3000):
        s, d = (int(x) for x in rng.integers(0, 400, 2))
        a = pc.lookup(s, d)
        b = ot.get(s, d)
        assert np.array(a).view(np.uint64).tolist() == np.array(b).view(np.uint64).tolist(), (s, d)


# Graphs with equal-cost paths (integer latencies, grids, parallel edges): a
# vertex's parent is its first exact predecessor in the igraph heap's pop
# order, which the row kernel's rule (smallest d[u], then lowest edge id) does
# not see; such rows are rerun through k_sssp_tie_parents (the restated
# igraph_2wheap Dijkstra) and must equal the oracle bit for bit.
def _half_ms(g):
    # the same graph at half the latencies: ties kept (k / 2 is exact), the weights no
    # longer whole numbers -- the tie kernel's 8-B heap values, no predicted build
    return S.GraphArrays(g.n_vertices, g.src, g.dst, g.latency * 0.5, g.loss, g.vertex_loss, directed=g.directed)


TIE_GRAPHS = {
    "grid6": lambda: W.grid_graph(6),
    "grid6_half_ms": lambda: _half_ms(W.grid_graph(6)),
    "geo_half_ms_300": lambda: _half_ms(W.geometric_graph(300, seed=3, integer_latency=True)),
    "grid6_directed": lambda: W.grid_graph(6, directed=True),
    "grid6_parallel": lambda: W.grid_graph(6, parallel=True),
    "grid30": lambda: W.grid_graph(30, seed=2),
    "geo_int_300": lambda: W.geometric_graph(300, seed=3, integer_latency=True),
    "geo_int_2000_vloss": lambda: W.geometric_graph(2000, seed=4, integer_latency=True, vertex_loss=True),
    "geo_int_5000": lambda: W.geometric_graph(5000, seed=6, integer_latency=True),
}


@pytest.mark.parametrize("name", sorted(TIE_GRAPHS))
def test_tie_rows_bit_exact(name):
    g = TIE_GRAPHS[name]()
    V = g.n_vertices
    att = np.arange(V, dtype=np.int32)
    pc = PathCache(g, att)
    info = pc.info()
    assert info.rows_computed == V and info.n_ties > 0 and info.n_tie_rows > 0
    rows = list(range(V)) if V <= 1000 else list(range(0, V, max(1, V // 97))) + [V - 1]
    lat, rel = pc.rows()
    olat, orel, ties = oracle_rows(g, att, rows)
    if len(rows) == V:
        assert info.n_ties == ties
    assert same_bits(lat[rows], olat) and same_bits(rel[rows], orel)


@pytest.mark.parametrize("name", ["grid30", "geo_int_2000_vloss"])
def test_tie_rows_bit_exact_on_the_lane_heap_kernel(name, monkeypatch):
    # round 6 moved tied rows to k_sssp_tie_lds (one row per wave, its heap in
    # LDS); SHD_PC_TIE_GLOBAL keeps k_sssp_tie_parents (lane heaps in global
    # scratch), which the LDS kernel still falls back to: both stay exact
    monkeypatch.setenv("SHD_PC_TIE_GLOBAL", "1")
    test_tie_rows_bit_exact(name)


def test_predicted_all_tied_build_equals_the_first_pass_over_every_row(monkeypatch):
    # round 6: on whole-number weights a probe of 2 x CUs rows runs the first
    # pass; when 90 % tie, the other rows go to the tie kernel without one and
    # the second pass counts their ties.  Same table, same tie count as the
    # first pass over every row (SHD_PC_NO_TIE_PREDICT)
    g = W.geometric_graph(5000, seed=6, integer_latency=True)
    att = np.arange(g.n_vertices, dtype=np.int32)
    pc = PathCache(g, att)
    a = pc.info()
    lat, rel = pc.rows()
    monkeypatch.setenv("SHD_PC_NO_TIE_PREDICT", "1")
    pc2 = PathCache(g, att)
    b = pc2.info()
    lat2, rel2 = pc2.rows()
    assert a.n_tie_rows_predicted > 0 and b.n_tie_rows_predicted == 0
    assert a.n_ties == b.n_ties and a.max_hops == b.max_hops and a.n_unroutable == b.n_unroutable
    assert same_bits(lat, lat2) and same_bits(rel, rel2)


def test_tie_rows_heap_past_lds_falls_back_bit_exact():
    # two hubs joined to every leaf at one whole millisecond: from a leaf, the
    # other leaves tie (both hubs are exact predecessors) and the heap holds
    # every leaf at once -- past the LDS heap at 5000 vertices, so each row is
    # run again through the lane heaps in global scratch; still the oracle's
    V = 5000
    leaves = np.arange(2, V, dtype=np.int64)
    src = np.concatenate([np.zeros(V - 2, np.int64), np.ones(V - 2, np.int64), [0]])
    dst = np.concatenate([leaves, leaves, [1]])
    rng = np.random.default_rng(3)
    g = S.GraphArrays(V, src, dst, np.full(len(src), 1.0), rng.uniform(0.0, 0.01, len(src)))
    att = np.arange(V, dtype=np.int32)
    pc = PathCache(g, att)
    info = pc.info()
    assert info.n_tie_rows > 0 and info.n_tie_rows_global > 0, (info.n_tie_rows, info.n_tie_rows_global)
    lat, rel = pc.rows()
    rows = [0, 1, 2, 3, 777, V - 1]
    olat, orel, _ = oracle_rows(g, att, rows)
    assert same_bits(lat[rows], olat) and same_bits(rel[rows], orel)


def test_tie_rows_global_scratch_path_and_subset():
    # V above the LDS capacity: both passes on the global-memory row kernel
    V = 12500
    g = W.geometric_graph(V, seed=8, integer_latency=True)
    rng = np.random.default_rng(2)
    att = np.sort(rng.choice(V, 240, replace=False)).astype(np.int32)
    pc = PathCache(g, att)
    info = pc.info()
    assert info.n_tie_rows > 0
    lat, rel = pc.rows()
    rows = list(range(0, len(att), 7))
    olat, orel, _ = oracle_rows(g, att, rows)
    assert same_bits(lat[rows], olat) and same_bits(rel[rows], orel)


def test_tie_graph_lazy_lookup_matches_reference_cache():
    g = W.grid_graph(12, seed=4)
    V = g.n_vertices
    att = np.arange(V, dtype=np.int32)
    pc = PathCache(g, att)
    ot = O.OTopo(O.OGraph(g), att)
    rng = np.random.default_rng(5)
    for _ in range(2000):
        s, d = (int(x) for x in rng.integers(0, V, 2))
        a = pc.lookup(s, d)
        b = ot.get(s, d)
        assert np.array(a).view(np.uint64).tolist() == np.array(b).view(np.uint64).tolist(), (s, d)


def _directed_geo(V, seed):
    g0 = W.geometric_graph(V, seed=seed, loss_max=0.01)
    src, dst = g0.src.astype(np.int64), g0.dst.astype(np.int64)
    nsl = src != dst
    rng = np.random.default_rng(seed)
    return S.GraphArrays(V, np.concatenate([src, dst[nsl]]), np.concatenate([dst, src[nsl]]),
                         np.concatenate([g0.latency, g0.latency[nsl] * (1.0 + rng.random(int(nsl.sum())))]),
                         np.concatenate([g0.loss, g0.loss[nsl]]), directed=True)


@pytest.mark.parametrize("name", ["geo", "grid", "directed", "bundled", "prefer_direct"])
def test_lookup_batch_equals_sequential_lookups(name):
    """shd_pc_lookup_batch: the same values, ranks and minimumPathLatency as
    the same queries through shd_pc_lookup one by one (one device round trip
    instead of one per query: the TCP driver's path tables)"""
    if name == "geo":
        g = W.geometric_graph(500, seed=4, vertex_loss=True)
    elif name == "grid":
        g = W.grid_graph(10, seed=3)
    elif name == "directed":
        g = _directed_geo(300, 6)
    elif name == "bundled":
        g = W.bundled_graph()
    else:
        g0 = W.geometric_graph(400, seed=8)
        g = S.GraphArrays(g0.n_vertices, g0.src, g0.dst, g0.latency, g0.loss, prefer_direct=True)
    rng = np.random.default_rng(11)
    att = np.sort(rng.choice(g.n_vertices, min(g.n_vertices, 250), replace=False)).astype(np.int32)
    q = att[rng.integers(0, len(att), (4000, 2))]
    q[::37, 1] = q[::37, 0]   # self pairs among them
    a = PathCache(g, att)
    b = PathCache(g, att)
    for part in (q[:1500], q[1500:]):   # two batches: the second starts from the first's ranks
        lat, rel = a.lookup_batch(part[:, 0], part[:, 1])
        want = np.array([b.lookup(int(s), int(d)) for s, d in part])
        assert same_bits(lat, want[:, 0]) and same_bits(rel, want[:, 1])
        ma, mb = C.c_double(), C.c_double()
        S.check(S.lib().shd_pc_min_stored_latency(a.ptr, C.byref(ma)), "min")
        S.check(S.lib().shd_pc_min_stored_latency(b.ptr, C.byref(mb)), "min")
        assert ma.value == mb.value
    a.close()
    b.close()
