"""APSP build time (10 k x 10 k) on the tie-free headline graph and on the same
geometry with whole-millisecond latencies (every row has equal-cost paths)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "shadow-1_amd"))
import numpy as np  # noqa: E402

import workloads as W  # noqa: E402
from sim import PathCache  # noqa: E402

out = {}
for name, kw in (("float", {}), ("integer", dict(integer_latency=True))):
    g = W.geometric_graph(10000, seed=1, **kw)
    att = np.arange(10000, dtype=np.int32)
    best = None
    for rep in range(3):
        pc = PathCache(g, att)
        i = pc.info()
        best = i if best is None or i.build_ms_device < best.build_ms_device else best
        pc.close()
    out[name] = dict(build_ms=round(best.build_ms_device, 3), sssp_ms=round(best.build_ms_sssp, 3),
                     n_ties=int(best.n_ties), n_tie_rows=int(best.n_tie_rows),
                     n_tie_rows_global=int(best.n_tie_rows_global))
    print(name, out[name], flush=True)
print(json.dumps(out))
