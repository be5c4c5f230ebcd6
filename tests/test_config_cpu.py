"""Config front-end on the CPU: shadow.config.xml host
registration order, `quantity` naming (master.c:304-320), hints and overrides
(configuration.c:404-480), DNS addresses (dns.c:40-134, 183-196; host.c:166-167),
and the inline-graphml topology through the product loader.

The expected addresses below (the counter starts at 11.0.0.0 and is
pre-incremented, reserved ranges and taken addresses are skipped, a hint is
kept when it is unrestricted and not taken, and 127.0.0.1 stays local) are
the reference's own: this CONFIG's hosts are case 0 of tests/golden/ref_net.json,
which the reference's dns.c compiled unmodified produced
(tests/golden/make_ref_net.py); test_ref_net_cpu.py checks them and two more
cases against that fixture.
"""
import os

import numpy as np
import pytest

import shdgpu as S

CONFIG = b"""<shadow stoptime="1800" bootstraptime="60">
  <topology path="~/topology.graphml.xml"/>
  <plugin id="phold" path="libphold.so"/>
  <host id="relay" quantity="3" bandwidthdown="10240" BandwidthUp="5120" iphint="11.0.0.3">
    <process plugin="phold" starttime="1" arguments="x"/>
  </host>
  <host id="client" countrycodehint="US" typehint="client" heartbeatfrequency="60">
    <process plugin="phold" starttime="2" arguments="y"/>
  </host>
  <host id="private" iphint="10.1.2.3"/>
  <host id="localhost" iphint="127.0.0.1"/>
  <host id="bad" iphint="not-an-ip"/>
  <host id="exact" iphint="52.0.0.7" quantity="1"/>
  <host id="dup" iphint="52.0.0.7"/>
  <host id="none" quantity="0"/>
</shadow>
"""


def test_hosts_in_registration_order_with_quantity_names():
    hosts, ips, stop, topo = S.load_config(CONFIG)
    names = [h["name"] for h in hosts]
    assert names == ["relay1", "relay2", "relay3", "client", "private", "localhost", "bad", "exact", "dup"]
    assert stop == 1800
    assert topo == "~/topology.graphml.xml"
    r = hosts[0]
    assert (r["bw_down_kibps"], r["bw_up_kibps"]) == (10240, 5120)   # attribute names are case-insensitive
    assert hosts[3]["countrycode_hint"] == "US" and hosts[3]["type_hint"] == "client"
    assert hosts[3]["heartbeat_s"] == 60 and hosts[3]["bw_down_kibps"] == 0
    assert all(h["ip_hint"] == "11.0.0.3" for h in hosts[:3])


def test_dns_addresses_follow_the_reference_counter():
    hosts, ips, _, _ = S.load_config(CONFIG)
    got = [S.ip_str(x) for x in ips]
    assert got == [
        "11.0.0.3",    # relay1 keeps its hint
        "11.0.0.1",    # relay2: hint taken -> counter 11.0.0.1
        "11.0.0.2",    # relay3
        "11.0.0.4",    # client: 11.0.0.3 is taken
        "11.0.0.5",    # private: 10/8 is reserved
        "127.0.0.1",   # localhost stays local
        "11.0.0.6",    # bad: not an address
        "52.0.0.7",    # exact keeps its hint
        "11.0.0.7",    # dup: hint taken
    ]
    assert len(set(got)) == len(got)


@pytest.mark.parametrize("hint,kept", [
    ("172.16.5.5", False), ("172.32.0.1", True), ("192.168.1.1", False), ("198.19.255.255", False),
    ("198.20.0.1", True), ("224.0.0.1", False), ("255.255.255.255", False), ("0.1.2.3", False),
    ("100.127.255.255", False), ("100.128.0.0", True), ("169.254.9.9", False), ("192.0.0.7", False),
    ("192.0.0.8", True), ("203.0.113.9", False), ("240.1.1.1", False), ("127.0.0.2", False),
])
def test_reserved_ranges(hint, kept):
    # _dns_isRestricted (dns.c:74-95): a reserved hint is replaced by the counter
    hosts, ips, _, _ = S.load_config(b'<shadow><host id="h" iphint="%s"/></shadow>' % hint.encode())
    assert S.ip_str(ips[0]) == (hint if kept else "11.0.0.1")


def test_rejects_non_shadow_root_and_missing_host_id():
    with pytest.raises(S.ShdError):
        S.load_config(b"<graphml/>")
    with pytest.raises(S.ShdError):
        S.load_config(b'<shadow><host quantity="2"/></shadow>')


def test_inline_topology_loads_through_the_graphml_loader():
    ref = "/root/reference/resource/examples/shadow.config.xml"
    if os.path.exists(ref):
        xml = open(ref, "rb").read()
    else:   # the same shape: one vertex, one self-loop, hosts without hints
        xml = (b'<shadow stoptime="3600"><topology><![CDATA[<?xml version="1.0" encoding="utf-8"?>'
               b'<graphml xmlns="http://graphml.graphdrawing.org/xmlns">'
               b'<key attr.name="packetloss" attr.type="double" for="edge" id="d6" />'
               b'<key attr.name="latency" attr.type="double" for="edge" id="d5" />'
               b'<graph edgedefault="undirected"><node id="isp"/>'
               b'<edge source="isp" target="isp"><data key="d5">50.0</data><data key="d6">0.01</data></edge>'
               b'</graph></graphml>]]></topology>'
               b'<host id="server"/><host id="client"/></shadow>')
    hosts, ips, stop, topo = S.load_config(xml)
    assert [h["name"] for h in hosts] == ["server", "client"]
    assert stop == 3600
    assert [S.ip_str(x) for x in ips] == ["11.0.0.1", "11.0.0.2"]
    assert topo.lstrip().startswith("<?xml")
    gm = C_load_graphml(topo.encode())
    g = gm.contents.g
    assert g.n_vertices == 1 and g.n_edges == 1


def C_load_graphml(xml: bytes):
    import ctypes as C
    ptr = C.POINTER(S.GraphML)()
    S.check(S.lib().shd_graphml_load_string(xml, len(xml), C.byref(ptr)), "shd_graphml_load_string")
    return ptr


def test_large_quantity_addresses_are_unique():
    hosts, ips, _, _ = S.load_config(b'<shadow><host id="n" quantity="70000"/></shadow>')
    assert len(hosts) == 70000 and hosts[-1]["name"] == "n70000"
    assert len(np.unique(ips)) == 70000
    assert S.ip_str(ips[-1]) == "11.1.17.112"   # 11.0.0.0 + 70000, nothing reserved in between
