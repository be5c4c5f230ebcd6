"""The device application hook at sizes beyond the
reference-loop fixtures: the UDP request/response echo (SHD_APP_UDP_ECHO,
oracle/ref_harness/ref_loop.c app 2; tests/test_ref_loop_gpu.py holds the
engine to the reference's own loop on the small cases) against the oracle's
serial loop -- every trace record (a multiset: the engine runs hosts in
parallel) and every host's end state, on the kernels the engine picks for
thousands of hosts (persistent rounds) and with CoDel queues at the servers."""
import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S
import workloads as W
from sim import Engine, PathCache, sort_trace

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("hosts,servers,payload,bw", [(4096, 1024, 1, 10240), (2000, 200, 1500, 512)])
def test_udp_echo_engine_equals_oracle(hosts, servers, payload, bw):
    V = 1000
    g = W.geometric_graph(V, seed=41, loss_max=0.01)
    hv = (np.arange(hosts, dtype=np.int64) * V // hosts).astype(np.int32)
    peer = np.array([-1] * servers + [(h * 13) % servers for h in range(servers, hosts)], dtype=np.int32)
    bwd = np.where(peer < 0, bw, 10240).astype(np.uint64)
    m = W.phold_model(hv, end_time=3 * S.SHD_SEC, trace=True, load=4, payload=payload, bw_down=bwd,
                      codelq_cap=1024, app_peer=peer)
    pc = PathCache(g, W.attached_vertices(hv))
    eng = Engine(m, pc)
    st = eng.run()
    otr, odg, ost = O.engine_run(m, g)
    assert st.n_pkt_events == ost["n_pkt_events"] > 0
    assert np.array_equal(sort_trace(eng.trace()), sort_trace(otr))
    assert np.array_equal(eng.digest(), odg)
    if payload > 1:   # the servers' queues built and dropped
        assert (otr["kind"] == S.TR_CODEL_DROP).sum() > 0


def _mix(hosts, V=1000, payload=1, bw_server=10240, client_load=4, seed=43):
    """SHD_APP_UDP at scale: the five kinds of tests/ref_loop_cases.py's
    udp_mix in the same proportions (PHOLD hosts over themselves and the
    sinks; servers replying from the listener; clients on one socket over
    the servers; one-way senders to a sink each; sinks)."""
    g = W.geometric_graph(V, seed=seed, loss_max=0.01)
    hv = (np.arange(hosts, dtype=np.int64) * V // hosts).astype(np.int32)
    kind = (np.arange(hosts) * 7 % 12)
    kind = np.select([kind < 4, kind < 6, kind < 9, kind < 10], [0, 1, 2, 3], 4).astype(np.uint8)
    specs = [(S.SHD_SEND_EACH, S.SHD_DEST_WEIGHTED, 3, 1), (S.SHD_SEND_LISTENER, S.SHD_DEST_REPLY, 0, 1),
             (S.SHD_SEND_ONCE, S.SHD_DEST_WEIGHTED, client_load, 1), (S.SHD_SEND_LISTENER, S.SHD_DEST_PEER, 4, 0),
             (S.SHD_SEND_LISTENER, S.SHD_DEST_WEIGHTED, 0, 0)]
    w = np.zeros((2, hosts))
    w[0, (kind == 0) | (kind == 4)] = 1.0
    w[1, kind == 1] = 1.0
    cum = np.cumsum(w / w.sum(axis=1, keepdims=True), axis=1)
    for r in range(2):   # exactly 1 from each row's last weighted host on (the rest stay unweighted)
        cum[r, np.flatnonzero(w[r])[-1]:] = 1.0
    sinks = np.flatnonzero(kind == 4)
    peer = np.full(hosts, -1, dtype=np.int32)
    one = np.flatnonzero(kind == 3)
    peer[one] = sinks[np.arange(len(one)) % len(sinks)]
    m0 = W.phold_model(hv, end_time=3 * S.SHD_SEC, trace=True)
    bw = np.where(kind == 1, bw_server, 10240).astype(np.uint64)
    m = S.ModelArrays(hv, m0.host_rng, bw, m0.bw_up, cum, end_time=3 * S.SHD_SEC, trace=True, payload=payload,
                      codelq_cap=1024, host_class=(kind == 2).astype(np.uint8), app_peer=peer, app_specs=specs,
                      host_app=kind)
    return g, m, specs, kind, peer, cum


@pytest.mark.parametrize("hosts,payload,bw,load", [(4096, 1, 10240, 4), (2000, 1500, 256, 24)])
def test_udp_app_mix_engine_equals_oracle(hosts, payload, bw, load):
    # SHD_APP_UDP (shd_udp_app per host) on the persistent kernels the engine
    # picks for thousands of hosts: the oracle's serial loop (pinned to the
    # reference loop by tests/test_ref_loop_cpu.py's udp_mix cases) record for
    # record, every host's end state; with CoDel drops at the servers
    g, m, *_ = _mix(hosts, payload=payload, bw_server=bw, client_load=load)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc)
    st = eng.run()
    otr, odg, ost = O.engine_run(m, g)
    assert st.n_pkt_events == ost["n_pkt_events"] > 0
    assert np.array_equal(sort_trace(eng.trace()), sort_trace(otr))
    assert np.array_equal(eng.digest(), odg)
    if payload > 1:
        assert (otr["kind"] == S.TR_CODEL_DROP).sum() > 0


def test_udp_app_models_that_could_reach_a_closed_port_are_refused():
    # shd_eng_create: a weighted destination that does not listen, a replying
    # host a new-socket-per-datagram host can reach, SHD_SEND_EACH with
    # SHD_DEST_REPLY -- each SHD_EINVAL (the device hands every datagram to the
    # application; such a datagram would be dropped at a closed port instead)
    hosts = 240
    g, m, specs, kind, peer, cum = _mix(hosts, V=200)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    bad = []
    cum2 = cum.copy()   # the PHOLD row onto a client too (clients do not listen)
    w = np.diff(np.concatenate([[0.0], cum[0]]))
    w[np.flatnonzero(kind == 2)[0]] = w.max()
    cum2[0] = np.cumsum(w / w.sum())
    cum2[0, -1] = 1.0
    bad.append(dict(dest_cum=cum2))
    cum3 = cum.copy()   # the PHOLD row onto a server (it would reply to a closed socket)
    w = np.diff(np.concatenate([[0.0], cum[0]]))
    w[np.flatnonzero(kind == 1)[0]] = w.max()
    cum3[0] = np.cumsum(w / w.sum())
    cum3[0, -1] = 1.0
    bad.append(dict(dest_cum=cum3))
    sp = list(specs)
    sp[1] = (S.SHD_SEND_EACH, S.SHD_DEST_REPLY, 0, 1)
    bad.append(dict(app_specs=sp))
    for kw in bad:
        args = dict(dest_cum=cum, app_specs=specs)
        args.update(kw)
        mb = S.ModelArrays(m.host_vertex, m.host_rng, m.bw_down, m.bw_up, args["dest_cum"], end_time=S.SHD_SEC,
                           host_class=(kind == 2).astype(np.uint8), app_peer=peer, app_specs=args["app_specs"],
                           host_app=kind)
        with pytest.raises(S.ShdError, match="EINVAL"):
            Engine(mb, pc)
