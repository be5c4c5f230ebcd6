"""The oracle's TCP restatement (oracle/o_tcp.c) against the reference's own
TCP (tcp.c, tcp_cong_reno.c, tcp_retransmit_tally.cc and the loop around them,
compiled unmodified into oracle/_ref/libshdref_loop.so) -- the parity pin of
SURVEY §8 (f)4.

Every case of tests/tcp_cases.py: the oracle's [STATUS] lines (packet.c:647-659:
every delivery status of every segment with its sequence, ACK, SACK ranges,
window, flags and timestamps) hash to the fixture the reference loop made
(tests/golden/ref_tcp.json, tests/golden/make_ref_tcp.py), and every host's
event-ID counter, packet-ID counter and RNG state end where the reference's do.
Where the reference loop is built here, a live run is compared line for line.
"""
import json
import os

import numpy as np
import pytest

import oracle_ffi as O
import ref_loop_ffi as R
import tcp_cases as TC

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "ref_tcp.json")))


def _oracle(name):
    c, m = TC.build(name)
    return O.tcp_run(m, c["graph"], TC.ip_ints(FIX[name]["ips"]), c["procs"], c["peers"], nbytes=c["nbytes"],
                     qdisc=c.get("qdisc", 0), udp=TC.udp_arg(c))


@pytest.mark.parametrize("name", list(TC.CASES))
def test_tcp_oracle_equals_reference_fixture(name):
    f = FIX[name]
    o = _oracle(name)
    assert len(o["lines"]) == f["n_status"]
    assert TC.digest(o["lines"]) == f["status_sha256"]
    assert TC.digest(TC.by_host(o["lines"])) == f["status_by_host_sha256"]
    assert o["next_event_id"].tolist() == f["next_event_id"]
    assert o["next_packet_id"].tolist() == f["next_packet_id"]
    assert o["rng_probe"].tolist() == f["rng_probe"]


def test_tcp_fixture_cases_exercise_the_machinery():
    """The fixtures cover what the restatement claims: handshakes, data,
    retransmissions (RTO and SACK-driven), drops in the network and at the
    receiver's queue, and the close sequence."""
    seen = set()
    for name in ("ref_epoll_lossy", "lossy_2pct", "slow_links", "heavy_loss"):
        for _, _, body in _oracle(name)["lines"]:
            seen.add(body[1:body.index("]")])
            for tag in ("header=SYN ", "header=SYNACK", "header=FIN ", "header=FINACK", "DUPACK", "sack=NA"):
                if tag in body:
                    seen.add(tag)
            if " sack=" in body and " sack=NA" not in body:
                seen.add("sack-ranges")
    for need in ("SND_TCP_RETRANSMITTED", "INET_DROPPED", "RCV_TCP_ENQUEUE_UNORDERED", "RCV_SOCKET_DELIVERED",
                 "header=SYN ", "header=SYNACK", "header=FIN ", "header=FINACK", "DUPACK", "sack-ranges"):
        assert need in seen, need


def test_rr_qdisc_changes_the_run():
    """the round-robin fixture is not the FIFO one: its hosts' sockets take
    turns at the interface in another order (network_interface.c:466-517)"""
    assert FIX["shared_hosts_rr"]["status_sha256"] != FIX["shared_hosts"]["status_sha256"]


@pytest.mark.skipif(not R.available(), reason="reference loop not built here (oracle/Makefile ref)")
@pytest.mark.parametrize("name", ["ref_epoll_lossless", "ref_epoll_lossy", "lossy_2pct"])
def test_tcp_oracle_equals_live_reference(name):
    c, m = TC.build(name)
    r = R.run(m, c["graph"], procs=c["procs"], tcp=dict(peers=c["peers"], nbytes=c["nbytes"]))
    o = O.tcp_run(m, c["graph"], TC.ip_ints(r["ip"]), c["procs"], c["peers"], nbytes=c["nbytes"])
    a = TC.status_lines(r["lines"])
    b = o["lines"]
    for i, (x, y) in enumerate(zip(a, b)):
        assert x == y, (i, x, y)
    assert len(a) == len(b)
    assert np.array_equal(r["next_event_id"], o["next_event_id"])
    assert np.array_equal(r["rng_probe"], o["rng_probe"])
