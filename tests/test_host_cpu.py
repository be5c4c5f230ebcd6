"""libshdgpu host side (no GPU needed): RNG, seed chain, graphml loader,
graph validation, attach."""
import ctypes as C
import json
import lzma
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S
import workloads as W

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NS = "{http://graphml.graphdrawing.org/xmlns}"


def test_product_rng_matches_golden():
    k = json.load(open(os.path.join(GOLD, "rng_kats.json")))
    l = S.lib()
    for seed, vals in k["rand_r"].items():
        s = C.c_uint32(int(seed))
        assert [l.shd_rand_r(C.byref(s)) for _ in range(8)] + [s.value] == vals
    for seed, vals in k["next_double"].items():
        s = C.c_uint32(int(seed))
        assert [l.shd_next_double(C.byref(s)).hex() for _ in range(8)] == vals
    assert list(W.seed_chain(64)) == k["seed_chain_1"]["hosts"]


def test_graphml_loader_matches_elementtree_on_bundled():
    xml = lzma.open(os.path.join(GOLD, "topology.graphml.xml.xz")).read()
    g, gm = W.load_graphml_bytes(xml)
    root = ET.fromstring(xml)
    keys = {k.get("id"): (k.get("attr.name"), k.get("for")) for k in root.iter(NS + "key")}
    graph = root.find(NS + "graph")
    nodes = graph.findall(NS + "node")
    ids = [n.get("id") for n in nodes]
    idx = {v: i for i, v in enumerate(ids)}
    edges = graph.findall(NS + "edge")
    assert g.n_vertices == len(nodes) and g.n_edges == len(edges)
    assert [gm.contents.vertex_id[i].decode() for i in range(len(ids))] == ids
    for e, ed in enumerate(edges):
        assert g.src[e] == idx[ed.get("source")] and g.dst[e] == idx[ed.get("target")]
        d = {keys[x.get("key")][0]: x.text for x in ed.findall(NS + "data")}
        assert g.latency[e] == float(d["latency"]) and g.loss[e] == float(d["packetloss"])
    for i, n in enumerate(nodes[:50]):
        d = {keys[x.get("key")][0]: x.text for x in n.findall(NS + "data")}
        assert gm.contents.bw_up[i] == float(d["bandwidthup"])
        ip = gm.contents.vertex_ip[i]
        assert (ip.decode() if ip else None) == d.get("ip")
    S.lib().shd_graphml_free(gm)


def test_example_topology_c1():
    # resource/examples/shadow.config.xml: one vertex "isp", self-loop 50 ms, loss 0.01
    xml = open(os.path.join(GOLD, "example_topology.graphml"), "rb").read()
    g, gm = W.load_graphml_bytes(xml)
    assert (g.n_vertices, g.n_edges) == (1, 1)
    assert g.latency[0] == 50.0 and g.loss[0] == 0.01
    p = S.GraphProps()
    assert S.lib().shd_graph_check(C.byref(g.struct), C.byref(p)) == 0
    assert p.is_complete == 1   # 1 vertex with its self-loop is complete
    og = O.OGraph(g)
    assert og.direct(0, 0) == (50.0, ((1.0 * 1.0) * 1.0) * (1.0 - 0.01))
    # two hosts attach to the only vertex; each attach draws once (topology.c:2326)
    seeds = W.seed_chain(2)
    for h in range(2):
        st = C.c_uint32(int(seeds[h]))
        v = C.c_int32(); bd = C.c_uint64(); bu = C.c_uint64()
        assert S.lib().shd_topology_attach(gm, C.byref(st), None, None, None, None, None, C.byref(v),
                                           C.byref(bd), C.byref(bu)) == 0
        s2 = C.c_uint32(int(seeds[h])); S.lib().shd_rand_r(C.byref(s2))
        assert v.value == 0 and st.value == s2.value and (bd.value, bu.value) == (17038, 2251)
    S.lib().shd_graphml_free(gm)


def test_graph_check_rejects_invalid_graphs():
    l = S.lib()
    p = S.GraphProps()
    disc = S.GraphArrays(4, [0, 2], [1, 3], [1.0, 1.0], [0.0, 0.0])
    assert l.shd_graph_check(C.byref(disc.struct), C.byref(p)) == -107   # ENOTCONN
    bad = S.GraphArrays(2, [0], [1], [0.0], [0.0])                      # latency must be > 0
    assert l.shd_graph_check(C.byref(bad.struct), C.byref(p)) == -22
    bad2 = S.GraphArrays(2, [0], [1], [1.0], [1.5])                     # loss in [0,1]
    assert l.shd_graph_check(C.byref(bad2.struct), C.byref(p)) == -22
    d = S.GraphArrays(3, [0, 1, 2], [1, 2, 0], [1.0, 1.0, 1.0], [0, 0, 0], directed=True)
    assert l.shd_graph_check(C.byref(d.struct), C.byref(p)) == 0
    d2 = S.GraphArrays(3, [0, 1], [1, 2], [1.0, 1.0], [0, 0], directed=True)  # not strongly connected
    assert l.shd_graph_check(C.byref(d2.struct), C.byref(p)) == -107


def test_completeness_rule_counts_incident_edges():
    # _topology_isComplete counts incident edges per vertex, self-loop once
    l = S.lib()
    p = S.GraphProps()
    full = S.GraphArrays(3, [0, 0, 1, 0, 1, 2], [1, 2, 2, 0, 1, 2], [1.0] * 6, [0.0] * 6)
    assert l.shd_graph_check(C.byref(full.struct), C.byref(p)) == 0 and p.is_complete == 1
    noloop = S.GraphArrays(3, [0, 0, 1], [1, 2, 2], [1.0] * 3, [0.0] * 3)
    assert l.shd_graph_check(C.byref(noloop.struct), C.byref(p)) == 0 and p.is_complete == 0
    og = O.OGraph(noloop)
    assert og.props().is_complete == 0


def test_attach_exact_ip_and_filters_on_bundled():
    xml = lzma.open(os.path.join(GOLD, "topology.graphml.xml.xz")).read()
    g, gm = W.load_graphml_bytes(xml)
    ips = [gm.contents.vertex_ip[i] for i in range(g.n_vertices)]
    usable = [i for i, ip in enumerate(ips) if ip and ip != b"0.0.0.0"]
    assert usable
    vi = usable[3]
    st = C.c_uint32(5); v = C.c_int32()
    assert S.lib().shd_topology_attach(gm, C.byref(st), ips[vi], None, None, None, None, C.byref(v),
                                       None, None) == 0
    assert v.value == vi
    s2 = C.c_uint32(5); S.lib().shd_rand_r(C.byref(s2))
    assert st.value == s2.value   # the exact match still consumes one draw
    # country hint narrows the candidates
    cc = gm.contents.vertex_countrycode[10]
    st = C.c_uint32(9)
    assert S.lib().shd_topology_attach(gm, C.byref(st), None, None, cc, None, None, C.byref(v), None,
                                       None) == 0
    assert gm.contents.vertex_countrycode[v.value] == cc
    S.lib().shd_graphml_free(gm)


def test_uniform_cum_is_the_phold_left_fold():
    cum = W.uniform_cum(1000)
    c = 0.0
    for i in range(1000):
        c += 1.0 / 1000.0
        assert cum[i] == c
