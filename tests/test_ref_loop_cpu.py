"""The oracle's composed event loop against the reference's OWN loop.

tests/golden/ref_loop.json comes from Shadow's worker.c / scheduler.c / host.c
/ network_interface.c / router*.c / descriptor/*.c / tracker.c / packet.c
compiled unmodified from /root/reference and run in serial mode
(tests/golden/make_ref_loop.py, oracle/ref_harness/ref_loop.c).  Here the
oracle (oracle/o_engine.c, the restatement the HIP engine is checked against)
runs the same models, and every [STATUS] line, every tracker [node] line and
every host's event-ID counter, packet counter and RNG state must be the
reference's.  tests/test_ref_loop_gpu.py holds the HIP engine to the same
fixtures.
"""
import json
import os

import numpy as np
import pytest

import oracle_ffi as O
import ref_loop_cases as RC
import ref_loop_ffi as R
import shdgpu as S

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "ref_loop.json")) as f:
    FIX = json.load(f)


def hb_k(case):
    m = case["model"].struct
    H = int(m.n_hosts)
    hbi = np.ctypeslib.as_array(m.host_heartbeat, shape=(H,)) if m.host_heartbeat else [int(m.heartbeat_interval)]
    return max(1, (int(m.end_time) - 1) // int(min(hbi)))


def oracle_lines(case, fx):
    m, g = case["model"], case["graph"]
    K = hb_k(case)
    hb = np.zeros((m.n_hosts, K, 2), dtype=np.uint32)
    tr, dg, _ = O.engine_run(m, g, pushes=case.get("pushes"), heartbeats=hb)
    st = S.status_lines(tr, fx["ips"], payload=int(m.struct.payload), app_peer=m.status_peer)
    st = sorted(st, key=lambda x: (x[0], x[1]))
    return st, RC.heartbeat_lines(m, hb, K), dg


@pytest.mark.parametrize("name", sorted(RC.CASES))
def test_oracle_equals_reference_loop(name):
    fx = FIX[name]
    case = RC.CASES[name]()
    st, hb, dg = oracle_lines(case, fx)
    assert len(st) == fx["n_status"]
    assert RC.digest_lines(st) == fx["status_sha256"]
    assert len(hb) == fx["n_heartbeat"]
    assert RC.digest_lines(hb) == fx["heartbeat_sha256"]
    assert dg["ev_seq"].tolist() == fx["next_event_id"]
    assert dg["pkt_seq"].tolist() == fx["next_packet_id"]
    probe = []
    for s in dg["rng"]:
        st_ = O.C.c_uint32(int(s))
        probe.append(int(O.lib().o_rand_r(O.C.byref(st_))))
    assert probe == fx["rng_probe"]


@pytest.mark.skipif(not R.available(), reason="oracle/_ref/libshdref_loop.so not built (needs /root/reference)")
@pytest.mark.parametrize("name", ["pushed_starts", "bootstrap", "c1"])
def test_reference_loop_reproduces_its_fixture(name):
    fx = FIX[name]
    case = RC.CASES[name]()
    r = R.run(case["model"], case["graph"], procs=RC.procs_of(case))
    st, hb = RC.split_lines(r["lines"])
    assert r["ip"] == fx["ips"]
    assert RC.digest_lines(st) == fx["status_sha256"]
    assert RC.digest_lines(hb) == fx["heartbeat_sha256"]
    assert r["next_event_id"].tolist() == fx["next_event_id"]
