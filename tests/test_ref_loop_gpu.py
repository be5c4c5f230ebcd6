"""The HIP engine against the reference's OWN event loop.

tests/golden/ref_loop.json holds what Shadow's serial loop -- worker.c,
scheduler.c, host.c, network_interface.c, router*.c, descriptor/*.c,
tracker.c, packet.c compiled unmodified from /root/reference
(tests/golden/make_ref_loop.py) -- logged and ended in for the models of
tests/ref_loop_cases.py.  The engine runs the same models through
libshdgpu.so; the library's writers make the [STATUS] lines from its trace
(shd_eng_status_lines) and the [node] lines from its tracker counters
(shd_eng_node_lines), and both, with every host's event-ID and packet counters
and RNG state, must be the reference's.
"""
import json
import os

import numpy as np
import pytest

import oracle_ffi as O
import ref_loop_cases as RC
import shdgpu as S
import workloads as W
from sim import Engine, PathCache

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "ref_loop.json")) as f:
    FIX = json.load(f)


@pytest.mark.parametrize("name", sorted(RC.CASES))
def test_engine_equals_reference_loop(name):
    fx = FIX[name]
    case = RC.CASES[name]()
    m, g = case["model"], case["graph"]
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc)
    if case.get("pushes") is not None:
        eng.boot()
        eng.push_events(case["pushes"])
    eng.run()
    # the library's own writers (shd_eng_status_lines / shd_eng_node_lines: what a
    # Shadow build linking the C-ABI logs), from the device trace and counters
    st = sorted(eng.status_lines(fx["ips"]), key=lambda x: (x[0], x[1]))
    assert len(st) == fx["n_status"]
    assert RC.digest_lines(st) == fx["status_sha256"]
    hbl = sorted((x for h in range(m.n_hosts) for x in eng.node_lines(h)), key=lambda x: (x[0], x[1]))
    assert len(hbl) == fx["n_heartbeat"]
    assert RC.digest_lines(hbl) == fx["heartbeat_sha256"]
    hb = eng.heartbeats()
    assert RC.digest_lines(RC.heartbeat_lines(m, hb, hb.shape[1])) == fx["heartbeat_sha256"]
    dg = eng.digest()
    assert dg["ev_seq"].tolist() == fx["next_event_id"]
    assert dg["pkt_seq"].tolist() == fx["next_packet_id"]
    probe = []
    for s in dg["rng"]:
        c = O.C.c_uint32(int(s))
        probe.append(int(O.lib().o_rand_r(O.C.byref(c))))
    assert probe == fx["rng_probe"]
