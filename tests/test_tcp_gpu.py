"""The TCP path on the GPU (csrc/tcp.hip through include/shdtcp.h) against the
reference's own TCP loop: every case of tests/tcp_cases.py, each host's
[STATUS] lines in its own order equal to the reference's
(tests/golden/ref_tcp.json: count and SHA-256 grouped by host), every host's
event-ID counter, packet counter and RNG state equal at the end.  The oracle's
lines (oracle/o_tcp.c, pinned to the same fixtures on the CPU) locate the first
difference when there is one."""
import json
import os

import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S
import tcp as TCPGPU
import tcp_cases as TC

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "ref_tcp.json")))


# cases whose first touches contradict a lane's choice within one window in a
# way that changes a value, so that the device run stops with
# SHD_TCP_ERR_FIRST_TOUCH and the driver runs the tables: none of the fixtures
# since round 5 (the replay accepts a contradicted choice whose two candidate
# rows give the pair the same bits).  shared_hosts(_rr) (0->1, 1->2, 2->0 at the
# same instant: host 2's lane chose vertex 7's row where the serial order
# takes vertex 0's) and loopback_mixed (a self path ranked in the round in
# which host 1 first queries (3, 0)) contradict only such choices;
# test_tcp_gpu_device_first_touch_contradiction_reruns_on_the_device keeps one that
# does not (since round 6 one engine reruns it on the device, ranked)
DEVICE_FALLS_BACK = set()


@pytest.mark.parametrize("mode", ["device", "tables"])
@pytest.mark.parametrize("name", list(TC.CASES))
def test_tcp_gpu_equals_reference(name, mode):
    """mode "device": the path cache's first-touch rule applied on the device
    (shd_tcp_model.path_cache); "tables": path tables resolved by the driver"""
    f = FIX[name]
    c, m = TC.build(name)
    ips = TC.ip_ints(f["ips"])
    r = TCPGPU.run(m, c["graph"], ips, c["procs"], c["peers"], nbytes=c["nbytes"], node=True, qdisc=c.get("qdisc", 0),
                   mode=mode, udp=TC.udp_arg(c))
    got = r["lines"]
    if "apps" in c and TC.digest(got) != f["status_by_host_sha256"]:
        # both transports: the reference's loop itself locates the first difference where it was built
        import ref_loop_ffi as R
        if R.available():
            want = TC.by_host(TC.status_lines(R.run(m, c["graph"], procs=c["procs"], tcp=TC.tcp_arg(c))["lines"]))
            for i, (x, y) in enumerate(zip(got, want)):
                assert x == y, (i, x, y)
        assert len(got) == f["n_status"], (len(got), f["n_status"])
        assert TC.digest(got) == f["status_by_host_sha256"]
    # the tracker's [node] lines: the library's writer over the device's counters
    assert len(r["node_lines"]) == f["n_heartbeat"]
    assert TC.digest(r["node_lines"]) == f["heartbeat_sha256"]
    if TC.digest(got) != f["status_by_host_sha256"]:
        want = TC.by_host(O.tcp_run(m, c["graph"], ips, c["procs"], c["peers"], nbytes=c["nbytes"],
                                    qdisc=c.get("qdisc", 0))["lines"])
        for i, (x, y) in enumerate(zip(got, want)):
            assert x == y, (i, x, y)
        assert len(got) == len(want), (len(got), len(want))
    assert len(got) == f["n_status"]
    assert r["next_event_id"].tolist() == f["next_event_id"]
    assert r["next_packet_id"].tolist() == f["next_packet_id"]
    assert r["rng_probe"].tolist() == f["rng_probe"]
    assert r["rounds"] > 0 and r["events"] > 0
    assert r["first_touch"] == ("tables" if mode == "device" and name in DEVICE_FALLS_BACK else mode)


@pytest.mark.parametrize("hosts,loss", [(64, 0.0), (96, 0.02)])
def test_tcp_gpu_scaled_model_equals_oracle(hosts, loss):
    """bench.py --workload tcp's model (workloads.tcp_echo_model) at a size the
    oracle runs in a second: every host's [STATUS] lines and end state equal
    the oracle's (oracle/o_tcp.c, pinned above to the reference's tcp.c loop)."""
    import workloads as W
    g, m, ips, procs, peers, nb = W.tcp_echo_model(hosts, 40, end_s=12, nbytes=60000, loss_max=loss)
    r = TCPGPU.run(m, g, ips, procs, peers, nbytes=nb)
    o = O.tcp_run(m, g, ips, procs, peers, nbytes=nb)
    want = TC.by_host(o["lines"])
    assert len(r["lines"]) == len(want) and r["lines"] == want
    assert r["next_event_id"].tolist() == o["next_event_id"].tolist()
    assert r["next_packet_id"].tolist() == o["next_packet_id"].tolist()
    assert r["rng_probe"].tolist() == o["rng_probe"].tolist()
    assert r["events"] == o["events"] and r["deliveries"] > 0


@pytest.mark.parametrize("hosts,loss,qdisc", [(96, 0.02, 0), (128, 0.01, 1)])
def test_tcp_gpu_mixed_transports_equal_oracle(hosts, loss, qdisc):
    """Both transports at a few hundred processes (workloads.
    mixed_transport_model: the echo pairs plus a datagram process on every
    host, four kinds of application): every host's [STATUS] lines and end
    state equal the oracle's (oracle/o_tcp.c, pinned to the reference's loop
    on the mixed_* fixtures), with the path cache on the device and on
    tables."""
    import workloads as W
    g, m, ips, procs, peers, nb, udp = W.mixed_transport_model(hosts, 40, end_s=10, nbytes=60000, loss_max=loss)
    o = O.tcp_run(m, g, ips, procs, peers, nbytes=nb, qdisc=qdisc, udp=udp)
    want = TC.by_host(o["lines"])
    assert sum(" bytes=" in ln[2] and " seq=" not in ln[2] for ln in want) > 1000   # datagrams' lines
    for mode in ("device", "tables"):
        r = TCPGPU.run(m, g, ips, procs, peers, nbytes=nb, qdisc=qdisc, udp=udp, mode=mode)
        assert len(r["lines"]) == len(want) and r["lines"] == want, mode
        assert r["next_event_id"].tolist() == o["next_event_id"].tolist()
        assert r["next_packet_id"].tolist() == o["next_packet_id"].tolist()
        assert r["rng_probe"].tolist() == o["rng_probe"].tolist()
        assert r["events"] == o["events"]


@pytest.mark.parametrize("hosts,loss", [(96, 0.02)])
def test_tcp_gpu_untraced_run_equals_oracle(hosts, loss):
    """The bench's mode: no lines written, so the device keeps no status list
    and copies packet records without it -- the run's end state and event
    count are still the oracle's, and the tracker's node lines the traced
    run's."""
    import workloads as W
    g, m, ips, procs, peers, nb = W.tcp_echo_model(hosts, 40, end_s=12, nbytes=60000, loss_max=loss)
    r = TCPGPU.run(m, g, ips, procs, peers, nbytes=nb, trace=False, node=True)
    t = TCPGPU.run(m, g, ips, procs, peers, nbytes=nb, trace=True, node=True)
    o = O.tcp_run(m, g, ips, procs, peers, nbytes=nb)
    assert r["lines"] == [] or all(ln[2].startswith("[shadow-heartbeat]") for ln in r["lines"])
    assert r["next_event_id"].tolist() == o["next_event_id"].tolist()
    assert r["next_packet_id"].tolist() == o["next_packet_id"].tolist()
    assert r["rng_probe"].tolist() == o["rng_probe"].tolist()
    assert r["events"] == o["events"]
    assert TC.node_lines(r["node_lines"]) == TC.node_lines(t["node_lines"]) and len(r["node_lines"]) > 0


@pytest.mark.parametrize("name", ["geo_pairs", "shared_hosts", "server_first"])
def test_tcp_gpu_first_touch_order_settles(name):
    """The path tables start from a wrong first-touch order (the clients
    reversed): the run's first-query log ranks the touches in serial order and
    the driver reruns until the tables agree (shadow-1_amd/tcp.py) -- the end
    result is the reference's, whatever the first guess."""
    f = FIX[name]
    c, m = TC.build(name)
    ips = TC.ip_ints(f["ips"])
    r = TCPGPU.run(m, c["graph"], ips, c["procs"], c["peers"], nbytes=c["nbytes"], guess_reversed=True)
    assert TC.digest(r["lines"]) == f["status_by_host_sha256"]
    assert r["next_event_id"].tolist() == f["next_event_id"]
    assert r["rng_probe"].tolist() == f["rng_probe"]
    assert r["first_touch_pairs"] > 0
    # where the reversed guess serves some pair from the other endpoint's row
    # (and the two orientations differ in their bits), a second run settles it
    lat_r, rel_r, _, _ = TCPGPU.path_table(m, c["graph"], c["procs"], c["peers"], reverse=True)
    lat_c, rel_c, _, _ = TCPGPU.path_table(m, c["graph"], c["procs"], c["peers"])
    wrong = not (np.array_equal(lat_r.view(np.uint64), lat_c.view(np.uint64)) and
                 np.array_equal(rel_r.view(np.uint64), rel_c.view(np.uint64)))
    assert r["first_touch_runs"] == (2 if wrong else 1)
    if name == "server_first":
        assert wrong   # the case is built so that the order matters


def test_tcp_gpu_wide_window_uses_the_mailbox_overflow(monkeypatch):
    """Fast, long connections (about 1 Gbit/s links, 8 MB each way) whose
    hosts share mailbox parts (the mailbox is split into 64 parts by host
    index: hosts 1, 65 and 129 are clients in part 1, hosts 0, 64 and 128
    servers in part 0).  The model's busiest round takes a few thousand
    deliveries, tens per part; with the parts cut to 8 slots
    (SHD_TCP_MAIL_PART, the overflow range left at its size) the sends spill
    into the shared overflow range -- the run must neither fail with
    SHD_TCP_ERR_MAILBOX nor differ from the oracle."""
    import workloads as W
    g, m, ips, procs, peers, nb = W.tcp_echo_model(130, 40, end_s=8, nbytes=8_000_000, bw_down=122070,
                                                   bw_up=122070)
    monkeypatch.setenv("SHD_TCP_MAIL_PART", "8")
    r = TCPGPU.run(m, g, ips, procs, peers, nbytes=nb, trace=False)
    monkeypatch.delenv("SHD_TCP_MAIL_PART")
    o = O.tcp_run(m, g, ips, procs, peers, nbytes=nb, lines=False)
    assert r["next_event_id"].tolist() == o["next_event_id"].tolist()
    assert r["next_packet_id"].tolist() == o["next_packet_id"].tolist()
    assert r["rng_probe"].tolist() == o["rng_probe"].tolist()
    assert r["events"] == o["events"]
    assert r["max_round_overflow"] > 0, (r["max_round_deliveries"], r["max_round_overflow"])


def test_tcp_gpu_device_first_touch_contradiction_reruns_on_the_device():
    """Two hosts each run a server and a client of the other's server, the
    clients' connects (topology_isRoutable: a first touch) 10 us apart in one
    window: each lane, seeing both vertices unranked, decides its own
    vertex's row; in serial order host 1's touch comes first, so host 0's
    query hits host 1's row.  The replay between rounds finds the
    contradiction; since round 6 shd_tcp_run runs the model again with that
    round's first touches ranked in serial order before it runs (no table
    fallback) -- the result is the oracle's."""
    import workloads as W
    g, m, ips, _, _, nb = W.tcp_echo_model(2, 30, end_s=6, nbytes=30000)
    if g.n_vertices and m.host_vertex[0] == m.host_vertex[1]:
        pytest.skip("the two hosts share a vertex")
    procs = [(0, S.SHD_SEC), (1, S.SHD_SEC), (0, 2 * S.SHD_SEC + 10000), (1, 2 * S.SHD_SEC)]
    peers = [-1, -1, 1, 0]
    r = TCPGPU.run(m, g, ips, procs, peers, nbytes=nb)
    o = O.tcp_run(m, g, ips, procs, peers, nbytes=nb)
    assert r["first_touch"] == "device" and r["first_touch_reruns"] >= 1, (r["first_touch"], r["first_touch_reruns"])
    assert r["lines"] == TC.by_host(o["lines"])
    assert r["next_event_id"].tolist() == o["next_event_id"].tolist()
    assert r["rng_probe"].tolist() == o["rng_probe"].tolist()
    # the same connects a window apart: no contradiction, the device decides
    procs2 = [(0, S.SHD_SEC), (1, S.SHD_SEC), (0, 2 * S.SHD_SEC + 200 * S.SHD_MS), (1, 2 * S.SHD_SEC)]
    r2 = TCPGPU.run(m, g, ips, procs2, peers, nbytes=nb)
    o2 = O.tcp_run(m, g, ips, procs2, peers, nbytes=nb)
    assert r2["first_touch"] == "device"
    assert r2["lines"] == TC.by_host(o2["lines"])
    assert r2["next_event_id"].tolist() == o2["next_event_id"].tolist()


def test_tcp_gpu_refuses_a_connect_in_its_servers_window():
    """a client reads its server's listening port when it
    connects, and the device publishes that port in the round the server
    binds; a client on another host starting less than one window W after its
    server could connect in that same round and read the port or not by the
    lanes' timing (on a group: differently from one engine).  Such a model is
    refused; the same client a window later runs and equals the oracle."""
    import workloads as W
    g, m, ips, _, _, nb = W.tcp_echo_model(2, 30, end_s=4, nbytes=20000)
    procs = [(0, S.SHD_SEC), (1, S.SHD_SEC + 1000)]
    peers = [-1, 0]
    with pytest.raises(S.ShdError):
        TCPGPU.run(m, g, ips, procs, peers, nbytes=nb)
    procs2 = [(0, S.SHD_SEC), (1, S.SHD_SEC + 300 * S.SHD_MS)]
    r = TCPGPU.run(m, g, ips, procs2, peers, nbytes=nb)
    o = O.tcp_run(m, g, ips, procs2, peers, nbytes=nb)
    assert r["lines"] == TC.by_host(o["lines"])
    assert r["next_event_id"].tolist() == o["next_event_id"].tolist()


def test_tcp_gpu_path_cache_min_latency_follows_the_run():
    """after a run on the path cache itself, the cache's
    minimumPathLatency (shd_pc_min_stored_latency, which topology_shd.c reads
    for the min time jump) includes the entries of the rows the run ranked, as
    if the run's first touches had gone through shd_pc_lookup in serial order:
    a fresh cache replaying the settled first-touch order of the tables path
    ends with the same value."""
    import ctypes as C
    import sim
    import workloads as W
    g, m, ips, procs, peers, nb = W.tcp_echo_model(24, 30, end_s=4, nbytes=20000)
    hv = np.asarray(m.host_vertex, dtype=np.int32)
    pc = sim.PathCache(g, np.unique(hv))
    out = TCPGPU._run_once(m, ips, procs, peers, None, None, hv, nb, False, TCPGPU.RECV_BUF, TCPGPU.SEND_BUF,
                           TCPGPU.TCP_WINDOW, 0, pc=pc)
    assert out is not None   # the device's first touches held
    r = TCPGPU.run(m, g, ips, procs, peers, nbytes=nb, trace=False, mode="tables")
    pc2 = sim.PathCache(g, np.unique(hv))
    for a, b in r["first_touch_order"]:
        pc2.lookup(a, b)
    m1, m2 = C.c_double(), C.c_double()
    S.check(S.lib().shd_pc_min_stored_latency(pc.ptr, C.byref(m1)), "min")
    S.check(S.lib().shd_pc_min_stored_latency(pc2.ptr, C.byref(m2)), "min")
    assert m1.value == m2.value > 0, (m1.value, m2.value)
