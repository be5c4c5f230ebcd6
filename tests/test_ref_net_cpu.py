"""The product's DNS and [STATUS] writer against the reference's own dns.c and
packet.c (tests/golden/ref_net.json, made by tests/golden/make_ref_net.py from
those files compiled unmodified into oracle/_ref/libshdref_net.so):

* shd_dns_assign (host/shd_config.c), driven through the config front-end,
  gives every host the ethernet address dns_register gives it (host.c:166-167,
  dns.c:102-134);
* shdgpu.status_line formats each line exactly as packet_addDeliveryStatus
  logs it (packet.c:518-659), PDS_DESTROYED included;
* shdgpu.status_lines, on traces of each datagram fate (delivered and read,
  dropped on the path, dropped by CoDel, dropped at a non-listening
  interface, loopback, dropped at push past the end), produces per packet
  exactly the reference's lines of its objects: the copy's, with the sender's
  original released right after INET_SENT (worker.c:306-313,
  network_interface.c:577).

Where the reference library was built here (the build container), the same
checks also run live against it on random inputs.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

import shdgpu as S

HERE = os.path.dirname(os.path.abspath(__file__))
FX = json.load(open(os.path.join(HERE, "golden", "ref_net.json")))
REF_LIB = os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libshdref_net.so")
NONE = 0xFFFFFFFF


def config_with_hints(hints):
    hs = "".join('<host id="h%d"%s/>' % (i, "" if h is None else ' iphint="%s"' % h) for i, h in enumerate(hints))
    return ('<shadow stoptime="10"><topology path="t.graphml"/>%s</shadow>' % hs).encode()


@pytest.mark.parametrize("case", range(len(FX["dns"])))
def test_dns_matches_reference(case):
    c = FX["dns"][case]
    hosts, ips, _, _ = S.load_config(config_with_hints(c["hints"]))
    assert [S.ip_str(x) for x in ips] == c["ips"]


def test_status_line_format_matches_reference():
    for item in FX["status"]:
        st, want = item["story"], item["lines"]
        names = st["statuses"] + ["PDS_DESTROYED"]
        got = [S.status_line(n, st["host_id"], st["pkt"], st["src"], st["sport"], st["dst"], st["dport"],
                             st["payload"], names[:k + 1]) for k, n in enumerate(names)]
        assert got == want, st


def story_lines(hid, pkt, role):
    for item in FX["status"]:
        s = item["story"]
        if s["host_id"] == hid and s["pkt"] == pkt and s["role"] == role:
            return item["lines"]
    raise KeyError((hid, pkt, role))


def lines_of(out, hid, pkt):
    tag = "packetID=%u:%u " % (hid, pkt)
    return [l for t, h, l in out if tag in l]


def R(t, seq, host, peer, pkt, kind):
    return (t, seq, host, peer, pkt, kind)


def sent_datagram_lines(hid, pkt):
    """the reference's lines of a sent datagram: the copy's up to INET_SENT,
    the original's release, then the rest of the copy's life"""
    copy, orig = story_lines(hid, pkt, "copy"), story_lines(hid, pkt, "orig")
    k = next(i for i, l in enumerate(copy) if l.startswith("[INET_SENT]")) + 1
    return copy[:k] + [orig[-1]] + copy[k:]


def test_status_lines_delivered_and_read():
    tr = np.array([R(1000, 12345, 0, NONE, 5, S.TR_CREATED), R(1000, 3, 0, 1, 5, S.TR_SENT),
                   R(2000, 0, 1, 0, 5, S.TR_ARRIVE), R(2000, 0, 1, 0, 5, S.TR_RECV),
                   R(2001, 0, 1, NONE, NONE, S.TR_READ)], dtype=S.TRACE_DTYPE)
    out = S.status_lines(tr, ["11.0.0.1", "11.0.0.2"], host_ids=[7, 8], payload=1)
    assert lines_of(out, 7, 5) == sent_datagram_lines(7, 5)


def test_status_lines_dropped_on_the_path():
    tr = np.array([R(50, 10000, 0, NONE, 0, S.TR_CREATED), R(50, 0, 0, 1, 0, S.TR_INET_DROP)],
                  dtype=S.TRACE_DTYPE)
    out = S.status_lines(tr, ["11.0.0.9", "11.0.3.7"], host_ids=[3, 4], payload=1)
    assert lines_of(out, 3, 0) == story_lines(3, 0, "orig")


def test_status_lines_codel_drop_and_interface_drop():
    hid, pkt = 4294967295, 4294967294
    tr = np.array([R(10, 65535, 0, NONE, pkt, S.TR_CREATED), R(10, 0, 0, 1, pkt, S.TR_SENT),
                   R(90, 0, 1, 0, pkt, S.TR_ARRIVE), R(95, 0, 1, 0, pkt, S.TR_CODEL_DROP)], dtype=S.TRACE_DTYPE)
    out = S.status_lines(tr, ["52.0.0.7", "11.0.0.1"], host_ids=[hid, 9], payload=1500)
    assert lines_of(out, hid, pkt) == sent_datagram_lines(hid, pkt)
    tr = np.array([R(10, 40000, 0, NONE, 99, S.TR_CREATED), R(10, 0, 0, 1, 99, S.TR_SENT),
                   R(90, 0, 1, 0, 99, S.TR_ARRIVE), R(90, 0, 1, 0, 99, S.TR_IF_DROP)], dtype=S.TRACE_DTYPE)
    out = S.status_lines(tr, ["11.0.0.2", "11.0.0.3"], host_ids=[12, 13], payload=1500)
    assert lines_of(out, 12, 99) == sent_datagram_lines(12, 99)


def test_status_lines_loopback_and_push_drop():
    tr = np.array([R(7, 10001, 0, NONE, 0, S.TR_CREATED), R(7, 1, 0, 0, 0, S.TR_LOCAL),
                   R(8, 0, 0, 0, 0, S.TR_RECV), R(9, 0, 0, NONE, NONE, S.TR_READ)], dtype=S.TRACE_DTYPE)
    out = S.status_lines(tr, ["11.0.0.2"], host_ids=[8], payload=1)
    assert lines_of(out, 8, 0) == story_lines(8, 0, "loop")
    # sent, and its delivery past the end: scheduler_push drops the copy's
    # event, releasing the copy before the sender releases the original
    tr = np.array([R(5, 1, 0, NONE, 1, S.TR_CREATED), R(5, 0, 0, 1, 1, S.TR_SENT)], dtype=S.TRACE_DTYPE)
    out = S.status_lines(tr, ["100.0.0.1", "11.0.0.1"], host_ids=[1, 2], payload=0)
    copy, orig = story_lines(1, 1, "copy"), story_lines(1, 1, "orig")
    assert lines_of(out, 1, 1) == copy + [orig[-1]]


# ---- live against the reference build (build container only) ----
needs_ref = pytest.mark.skipif(not os.path.exists(REF_LIB), reason="oracle/_ref not built (GPU box / no reference)")


@needs_ref
def test_dns_live_random_hints():
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_ref_net as M
    l = M.lib()
    rng = np.random.default_rng(3)
    pool = ["11.0.0.%d" % k for k in range(1, 40)] + ["10.0.0.1", "127.0.0.1", "100.64.1.1", "8.8.8.8",
                                                      "11.0.0.0", "255.255.255.255", "x", "11.0.0.07"]
    for _ in range(20):
        hints = [None if rng.random() < 0.4 else pool[int(rng.integers(len(pool)))] for _ in range(60)]
        _, ips, _, _ = S.load_config(config_with_hints(hints))
        assert [S.ip_str(x) for x in ips] == M.ref_dns(l, hints)


@needs_ref
def test_status_line_live_random_stories():
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_ref_net as M
    l = M.lib()
    rng = np.random.default_rng(4)
    names = [n for n in S.STATUS_FLAG]
    for _ in range(50):
        st = dict(host_id=int(rng.integers(0, 2**32)), pkt=int(rng.integers(0, 2**63)),
                  src="%d.%d.%d.%d" % tuple(rng.integers(0, 256, 4)), sport=int(rng.integers(0, 65536)),
                  dst="%d.%d.%d.%d" % tuple(rng.integers(0, 256, 4)), dport=int(rng.integers(0, 65536)),
                  payload=int(rng.integers(0, 3000)),
                  statuses=[names[int(i)] for i in rng.integers(0, len(names), int(rng.integers(1, 12)))])
        seq = st["statuses"] + ["PDS_DESTROYED"]
        got = [S.status_line(n, st["host_id"], st["pkt"], st["src"], st["sport"], st["dst"], st["dport"],
                             st["payload"], seq[:k + 1]) for k, n in enumerate(seq)]
        assert got == M.ref_story(l, st)
