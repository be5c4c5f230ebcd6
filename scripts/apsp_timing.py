"""Time the path-cache build (APSP rows) on the GPU for the BASELINE configs."""
import os, sys, time, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd"), os.path.join(REPO, "tests")]
import numpy as np
import workloads as W
from pc_helpers import PathCache

out = {}
g = W.bundled_graph()
att = np.arange(g.n_vertices, dtype=np.int32)
for name, flags in (("bundled_direct", 0), ("bundled_forced_rows", 1)):
    pc = PathCache(g, att, flags=flags)
    t = []
    for _ in range(5):
        pc.build(); t.append(pc.info().build_ms_device)
    i = pc.info()
    out[name] = dict(ms=min(t), sssp_ms=i.build_ms_sssp, iters=i.sssp_iterations_max, hops=i.max_hops)
    pc.close()
for V in (10000,):
    t0 = time.time(); g = W.geometric_graph(V, seed=1); tg = time.time() - t0
    att = np.arange(V, dtype=np.int32)
    pc = PathCache(g, att)
    t = []
    for _ in range(3):
        pc.build(); i = pc.info(); t.append((i.build_ms_device, i.build_ms_sssp))
    out[f"geometric_{V}"] = dict(E=g.n_edges, gen_s=tg, ms=min(x[0] for x in t), sssp_ms=min(x[1] for x in t),
                                 iters=i.sssp_iterations_max, hops=i.max_hops, ties=i.n_ties,
                                 minlat=i.min_latency_ms)
    pc.close()
print(json.dumps(out, indent=1))
