import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd"), os.path.join(REPO, "tests")]
import numpy as np
import shdgpu as S, workloads as W, oracle_ffi as O
from sim import Engine, PathCache, sort_trace
g = W.bundled_graph()
rng = np.random.default_rng(0)
hv = np.sort(rng.integers(0, g.n_vertices, 400)).astype(np.int32)
for cap in (64, 256, 2048):
    m = W.phold_model(hv, end_time=3 * S.SHD_SEC, trace=True, load=8, evq_cap=cap, inbox_cap=cap)
    pc = PathCache(g, W.attached_vertices(hv))
    e = Engine(m, pc)
    print("window", e.window, flush=True)
    e.boot()
    nxt = e.next_time(); rounds = 0
    try:
        while nxt < m.params["end_time"]:
            r = e.run_round(nxt, min(nxt + e.window, m.params["end_time"]))
            rounds += 1
            nxt = r.next_time
        tr = sort_trace(e.trace()); dg = e.digest()
        otr, odg, ost = O.engine_run(m, g)
        otr = sort_trace(otr)
        print(cap, "rounds", rounds, "same trace", np.array_equal(tr, otr), "same digest", np.array_equal(dg, odg), len(tr), len(otr))
        if not np.array_equal(dg, odg):
            bad = np.nonzero(dg != odg)[0][:5]; print(dg[bad]); print(odg[bad])
    except Exception as ex:
        print(cap, "failed at round", rounds, "time", nxt, ex)
