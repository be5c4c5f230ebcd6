"""SHD_APP_UDP mix at scale: where the engine and the oracle first differ
(debugging aid for tests/test_app_gpu.py)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402

import oracle_ffi as O  # noqa: E402
import test_app_gpu as T  # noqa: E402
import workloads as W  # noqa: E402
from sim import Engine, PathCache, sort_trace  # noqa: E402

for hosts, payload, bw, load in [(4096, 1, 10240, 4), (2000, 1500, 256, 24), (600, 1, 10240, 4)]:
    g, m, specs, kind, peer, cum = T._mix(hosts, payload=payload, bw_server=bw, client_load=load)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    try:
        eng = Engine(m, pc)
    except Exception as ex:   # noqa: BLE001
        print(hosts, "create:", ex, flush=True)
        continue
    st = eng.run()
    otr, odg, ost = O.engine_run(m, g)
    print(hosts, "pkt events", st.n_pkt_events, ost["n_pkt_events"], flush=True)
    a, b = sort_trace(eng.trace()), sort_trace(otr)
    dg = eng.digest()
    bad = np.flatnonzero(np.any(np.stack([dg[f] != odg[f] for f in dg.dtype.names]), axis=0))
    print("hosts with a different end state:", len(bad), bad[:10], "kinds", kind[bad[:10]], flush=True)
    for h in bad[:3]:
        ea, ob = a[a["host"] == h], b[b["host"] == h]
        n = min(len(ea), len(ob))
        d = np.flatnonzero(ea[:n] != ob[:n])
        i = d[0] if len(d) else n
        print(" host", h, "kind", kind[h], "records", len(ea), len(ob), "first diff", i, flush=True)
        for k in range(max(0, i - 2), min(n, i + 3)):
            print("   eng", ea[k], "\n   ora", ob[k], flush=True)
