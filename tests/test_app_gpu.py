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
