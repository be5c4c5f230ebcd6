"""The [STATUS] packet lines (packet_addDeliveryStatus / packet_toString,
packet.c:518-659) from a status trace (SHD_QF_TRACE_STATUS), on a hand-built
trace whose expected lines follow the reference's call chain, and on an
oracle run (every datagram's statuses well formed).  The line format and each
fate's lines are pinned to the reference's packet.c in test_ref_net_cpu.py."""
import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S
import workloads as W

NONE = 0xFFFFFFFF


def rec(t, seq, host, peer, pkt, kind):
    return (t, seq, host, peer, pkt, kind)


def test_status_lines_follow_the_reference_call_chain():
    # host 0 creates packet 5 (port 12345) to host 1 and sends it at once; it
    # arrives at t=2000, is dequeued, read at t=2001; host 1 answers with
    # packet 0 to itself (loopback: no router), received at +1 ns
    tr = np.array([
        rec(1000, 12345, 0, NONE, 5, S.TR_CREATED),
        rec(2000, 7, 1, 0, 5, S.TR_ARRIVE),
        rec(2000, 0, 1, 0, 5, S.TR_RECV),
        rec(2001, 0, 1, NONE, NONE, S.TR_READ),
        rec(2001, 10001, 1, NONE, 0, S.TR_CREATED),
        rec(2002, 0, 1, 1, 0, S.TR_RECV),
        rec(1000, 3, 0, 1, 5, S.TR_SENT),          # out of order, as a flush writes it
        rec(2001, 9, 1, 1, 0, S.TR_LOCAL),
    ], dtype=S.TRACE_DTYPE)
    lines = S.status_lines(tr, ["11.0.0.1", "11.0.0.2"], host_ids=[7, 8])
    a = "packetID=7:5 11.0.0.1:12345 -> 11.0.0.2:8998 bytes=1 status="
    b = "packetID=8:0 11.0.0.2:10001 -> 11.0.0.2:8998 bytes=1 status="
    want = [
        (1000, 0, "[SND_CREATED] " + a + "SND_CREATED"),
        (1000, 0, "[SND_SOCKET_BUFFERED] " + a + "SND_CREATED,SND_SOCKET_BUFFERED"),
        (1000, 0, "[SND_INTERFACE_SENT] " + a + "SND_CREATED,SND_SOCKET_BUFFERED,SND_INTERFACE_SENT"),
        (1000, 0, "[INET_SENT] " + a + "SND_CREATED,SND_SOCKET_BUFFERED,SND_INTERFACE_SENT,INET_SENT"),
        # the sender releases its original at once; the copy travels on
        (1000, 0, "[PDS_DESTROYED] " + a + "SND_CREATED,SND_SOCKET_BUFFERED,SND_INTERFACE_SENT,INET_SENT,"
                                           "PDS_DESTROYED"),
        (2000, 1, "[ROUTER_ENQUEUED] " + a + "SND_CREATED,SND_SOCKET_BUFFERED,SND_INTERFACE_SENT,INET_SENT,"
                                             "ROUTER_ENQUEUED"),
    ]
    assert lines[:6] == want
    seq_a = [l for t, h, l in lines if "packetID=7:5" in l]
    assert seq_a[-2].startswith("[RCV_SOCKET_DELIVERED] ")
    assert seq_a[-1].endswith("ROUTER_ENQUEUED,ROUTER_DEQUEUED,RCV_INTERFACE_RECEIVED,RCV_SOCKET_PROCESSED,"
                              "RCV_SOCKET_BUFFERED,RCV_SOCKET_DELIVERED,PDS_DESTROYED")   # the read releases it
    assert [t for t, h, l in lines if "packetID=7:5" in l][-1] == 2001
    seq_b = [l for t, h, l in lines if "packetID=8:0" in l]
    assert seq_b[-1].endswith("status=SND_CREATED,SND_SOCKET_BUFFERED,SND_INTERFACE_SENT,RCV_INTERFACE_RECEIVED,"
                              "RCV_SOCKET_PROCESSED,RCV_SOCKET_BUFFERED")   # loopback: no router, not read yet
    assert [x[0] for x in lines] == sorted(x[0] for x in lines)


def test_oracle_status_trace_is_well_formed():
    V = 40
    g = W.geometric_graph(V, seed=3)
    m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=2 * S.SHD_SEC, trace=True, load=3,
                      queue_flags=S.SHD_QF_TRACE_STATUS)
    otr, odg, ost = O.engine_run(m, g)
    kinds = np.bincount(otr["kind"], minlength=10)
    assert kinds[S.TR_CREATED] == kinds[S.TR_SENT] + kinds[S.TR_INET_DROP] + kinds[S.TR_LOCAL] > 0
    assert kinds[S.TR_READ] > 0
    assert np.all((otr["seq"][otr["kind"] == S.TR_CREATED] >= S.SHD_MIN_RANDOM_PORT))
    lines = S.status_lines(otr, ["11.0.0.%d" % (h + 1) for h in range(V)])
    by_pkt = {}
    for t, h, l in lines:
        by_pkt.setdefault(l.split()[1], []).append(l.split("status=")[1].split(","))
    for key, sts in by_pkt.items():
        live = [x for x in sts if x[-1] != "PDS_DESTROYED"]
        last = live[-1]
        assert last[:2] == ["SND_CREATED", "SND_SOCKET_BUFFERED"], key
        assert all(x == last[:len(x)] for x in live)          # each line's list extends the previous
        # a release closes one object's list: the list it ends is one of the packet's lists
        for x in sts:
            if x[-1] == "PDS_DESTROYED":
                assert x[:-1] in live, key
    # without the flag the trace has no application records
    m2 = W.phold_model(W.hosts_on_vertices(V, 1), end_time=2 * S.SHD_SEC, trace=True, load=3)
    otr2, _, _ = O.engine_run(m2, g)
    assert not np.any(otr2["kind"] >= S.TR_CREATED)
    assert len(otr2) == len(otr) - kinds[S.TR_CREATED] - kinds[S.TR_READ]


def test_c_writer_equals_the_python_restatement():
    """libshdgpu's writers (shd_status_lines, shd_node_lines: the C-ABI a Shadow
    build links) against the Python restatement of the same algorithm, line for
    line and in the same order: an oracle status trace with CoDel drops,
    interface drops past the end and loopback sends, and heartbeat snapshots
    with a 32-bit wrap.  (test_ref_loop_cpu.py pins the writer to the
    reference's own lines.)"""
    V = 30
    g = W.geometric_graph(V, seed=5)
    for kw in ({}, {"payload": 1500, "bw_down": 512, "load": 6}):
        m = W.phold_model(W.hosts_on_vertices(V, 2), end_time=2 * S.SHD_SEC, trace=True,
                          queue_flags=S.SHD_QF_TRACE_STATUS, **({"load": 3} | kw))
        otr, _, _ = O.engine_run(m, g)
        ips = ["10.%d.%d.%d" % (h >> 16, (h >> 8) & 255, h & 255) for h in range(2 * V)]
        ids = [3 * h + 2 for h in range(2 * V)]
        for pl in (1, 1500):
            c = S.status_lines(otr, ips, host_ids=ids, payload=pl)
            assert c == S.status_lines_py(otr, ips, host_ids=ids, payload=pl)
            assert len(c) > len(otr)
    # the UDP echo application: replies go to each client's bound port
    peer = np.array([-1] * 6 + [h % 6 for h in range(6, V)], dtype=np.int32)
    m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=2 * S.SHD_SEC, trace=True, load=3,
                      queue_flags=S.SHD_QF_TRACE_STATUS, app_peer=peer)
    otr, _, _ = O.engine_run(m, g)
    ips = ["11.0.%d.%d" % (h >> 8, h & 255) for h in range(V)]
    c = S.status_lines(otr, ips, payload=1, app_peer=peer)
    assert c == S.status_lines_py(otr, ips, payload=1, app_peer=peer)
    assert any(":8998 -> " in x[2] for x in c) and any(" -> 11.0.0.%d:8998 " % (k + 1) in x[2] for k in range(6) for x in c[:50])
    snaps = np.array([[5, 7], [9, 9], [0xFFFFFFF0, 20], [3, 25]], dtype=np.uint32)
    for pl in (0, 1, 1500):
        assert S.tracker_node_lines(snaps, S.SHD_SEC, pl) == S.tracker_node_lines_py(snaps, S.SHD_SEC, pl)
        assert S.tracker_node_lines(snaps[:0], 2 * S.SHD_SEC, pl) == S.tracker_node_lines_py(snaps[:0], 2 * S.SHD_SEC, pl)


def test_tracker_node_lines_from_full_counters():
    """shd_tracker_node_lines (the TCP path's [node] lines): the header and the
    boot line at t = 0, then per interval _tracker_logNode's line
    (tracker.c:419-465) with _tracker_getCounterString's twelve fields
    (tracker.c:399-417) for the remote counters, localhost all zero.  Checked
    against the format written out here from those lines of the reference."""
    import ctypes as C
    cnt = np.zeros((2, 20), dtype=np.uint64)
    # interval 1: in 3 control (66 B each), 2 data (66 + 1000), 1 data retransmit (66 + 500);
    #             out 4 control, 1 control retransmit
    cnt[0, :10] = [3, 198, 0, 0, 2, 132, 2000, 1, 66, 500]
    cnt[0, 10:] = [4, 264, 1, 66, 0, 0, 0, 0, 0, 0]
    lp = C.POINTER(S.Lines)()
    S.check(S.lib().shd_tracker_node_lines(cnt.ctypes.data_as(C.POINTER(C.c_uint64)), 2, 2 * S.SHD_SEC, 7,
                                           C.byref(lp)), "shd_tracker_node_lines")
    lines = S.take_lines(lp)
    assert [(t, h) for t, h, _ in lines] == [(0, 7), (0, 7), (2 * S.SHD_SEC, 7), (4 * S.SHD_SEC, 7)]
    assert lines[0][2].startswith("[shadow-heartbeat] [node-header] interval-seconds,recv-bytes,")
    z = ",".join(["0"] * 12)
    assert lines[1][2] == f"[shadow-heartbeat] [node] 2,0,0,0.000000,0,0.000000;{z};{z};{z};{z}"
    rin = 198 + 132 + 2000 + 66 + 500
    rout = 264 + 66
    assert lines[2][2] == (f"[shadow-heartbeat] [node] 2,{rin},{rout},0.000000,0,0.000000;{z};{z};"
                           f"6,{rin},3,198,0,0,2,132,2000,1,66,500;5,{rout},4,264,1,66,0,0,0,0,0,0")
    assert lines[3][2] == f"[shadow-heartbeat] [node] 2,0,0,0.000000,0,0.000000;{z};{z};{z};{z}"


def test_status_writer_refuses_out_of_range_peers():
    """shd_status_lines indexes ips[] with every record's peer (the sender's
    destination, the receiver's source): a record naming a host past n_hosts
    (or ~0) is refused with -EINVAL instead of read out of bounds."""
    V = 12
    g = W.geometric_graph(V, seed=3)
    m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=2 * S.SHD_SEC, trace=True, load=2,
                      queue_flags=S.SHD_QF_TRACE_STATUS)
    otr, _, _ = O.engine_run(m, g)
    ips = ["10.0.0.%d" % (h + 1) for h in range(V)]
    assert len(S.status_lines(otr, ips)) > 0
    for kind in (S.TR_SENT, S.TR_ARRIVE, S.TR_RECV):
        bad = otr.copy()
        k = int(np.nonzero(bad["kind"] == kind)[0][0])
        for peer in (V, 0xFFFFFFFF):
            bad["peer"][k] = peer
            with pytest.raises(S.ShdError):
                S.status_lines(bad, ips)
