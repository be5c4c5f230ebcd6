#!/usr/bin/env python3
"""Hosts per wave of the round kernel (SHD_HPW) against the rate, on the bench
headline workload; per-step times show where the first-touch warm-up ends."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import shdgpu as S  # noqa: E402
import workloads as W  # noqa: E402
from sim import Engine, PathCache  # noqa: E402

V = 10000
hpws = [int(x) for x in (sys.argv[1:] or ["64", "32", "16"])]
g = W.geometric_graph(V, seed=1, loss_max=0.0)
hv = W.hosts_on_vertices(V, 1)
m = W.phold_model(hv, end_time=12 * S.SHD_SEC, seed=1, load=16, payload=1)
pc = PathCache(g, W.attached_vertices(hv))
for hpw in hpws:
    os.environ["SHD_HPW"] = str(hpw)
    e = Engine(m, pc)
    e.boot()
    e.run_until(2 * S.SHD_SEC)
    per = []
    tot_pkt = tot_s = 0
    for k in range(3, 11):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = e.run_until(k * S.SHD_SEC)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        per.append((round(dt * 1e3, 2), st.n_rounds, st.n_batches_ticketless, round(st.device_ms_launches / max(st.n_rounds, 1) * 1e3, 2)))
        tot_pkt += st.n_pkt_events
        tot_s += dt
    print(f"hpw {hpw}: {tot_pkt / tot_s / 1e6:.1f} M packet events/s; per step (ms, rounds, tl batches, us/launch): {per}",
          flush=True)
    e.close()
