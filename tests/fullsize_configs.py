"""The full-size parity configurations (tests/golden/make_fullsize.py makes
their fixtures with the oracle; tests/test_fullsize_gpu.py checks the HIP
engine against them).  One definition for both sides."""
import os

import shdgpu as S
import workloads as W

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C1_CONFIG = os.path.join(REPO, "tests", "golden", "example_shadow.config.xml")

V = 10000

CONFIGS = {
    "c1": dict(file="c1_example.npz", fixture="full_trace"),
    "c3": dict(file="c3_full.npz", fixture="trace_hash", loss=0.0, end=3 * S.SHD_SEC),
    "c3_lossy": dict(file="c3_lossy_full.npz", fixture="trace_hash", loss=0.0005, end=3 * S.SHD_SEC),
    "c5": dict(file="c5_codel_full.npz", fixture="block_hash", block=1024, loss=0.01,
               end=int(1.25 * S.SHD_SEC)),
}


def c3_hosts(hosts):
    """bench.py's host placement for N x 10 k hosts on the 10 k-vertex graph."""
    import numpy as np
    hpv = max(1, hosts // V)
    return (np.arange(hosts, dtype=np.int64) * V // hosts).astype(np.int32) if hosts != V * hpv else \
        W.hosts_on_vertices(V, hpv)


def build(key, trace=None):
    """(graph, model, pushed events or None) of a configuration."""
    cfg = CONFIGS[key]
    if key == "c1":
        xml = open(C1_CONFIG, "rb").read()
        g, m, pushes, _, _ = W.config_model(xml, load=16, payload=1, trace=True if trace is None else trace)
        return g, m, pushes
    g = W.geometric_graph(V, seed=1, loss_max=cfg["loss"])
    if key.startswith("c3"):
        m = W.phold_model(c3_hosts(V), end_time=cfg["end"], seed=1, load=16, payload=1,
                          trace=True if trace is None else trace)
        return g, m, None
    # c5: CoDel queues building at 1 M hosts
    m = W.phold_model(W.hosts_on_vertices(V, 100), end_time=cfg["end"], seed=1, load=32, payload=1500,
                      bw_down=512, bw_up=10240, codelq_cap=256, trace=bool(trace))
    return g, m, None
