"""First-touch logs over simulated time on the bench model (10 k hosts): rounds
that log, records per logging round, distinct vertices involved, and the
ranks assigned (host-driven rounds, so every log is seen)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402

import shdgpu as S  # noqa: E402
import workloads as W  # noqa: E402
from sim import Engine, PathCache  # noqa: E402

V = 10000
g = W.geometric_graph(V, seed=1, loss_max=0.0005)
m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=6 * S.SHD_SEC, seed=1, load=16, payload=1)
pc = PathCache(g, W.attached_vertices(m.host_vertex))
e = Engine(m, pc)
e.boot()
win = e.window
t = e.next_time()
per_sec = {}
verts = {}
while t < m.params["end_time"]:
    r = e.round_kernel(t, min(t + win, m.params["end_time"]))
    if r.n_pending:
        recs = e.pending_records()
        e.resolve(recs)
        sec = int(t // S.SHD_SEC)
        c = per_sec.setdefault(sec, [0, 0])
        c[0] += 1
        c[1] += len(recs)
        verts.setdefault(sec, set()).update(np.unique(np.concatenate([recs["a"], recs["b"]])).tolist())
        if sec >= 2 and c[0] <= 3:
            print("sec", sec, "t", t, "recs (a, b, qhost, dst):",
                  [(int(x["a"]), int(x["b"]), int(x["qhost"]), int(x["dst"])) for x in recs[:4]])
    s = e.end_round()
    t = s.next_time
for sec in sorted(per_sec):
    print(f"second {sec}: logging rounds {per_sec[sec][0]}, records {per_sec[sec][1]}, "
          f"vertices {len(verts[sec])}")
