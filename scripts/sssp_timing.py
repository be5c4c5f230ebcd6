"""Cycle accounting of the SSSP row kernel's Bellman-Ford (measurement build:
make -C shadow-1_amd pcvariant PC_FLAGS=-DSHD_SSSP_TIMING PCV=t; run with
SHDGPU_LIB=shadow-1_amd/libshdgpu_pcvt.so).  Per block (one row at a time per
CU): cycles summed over its waves' lane 0 for the BF total (per wave), the scan
of the chunk loop (frontier work included), the frontier work, the barrier wait;
iterations, frontier vertices, rows."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd"), os.path.join(REPO, "tests")]
import shdgpu as S          # noqa: E402
import workloads as W       # noqa: E402
from pc_helpers import PathCache   # noqa: E402

V = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
g = W.geometric_graph(V, seed=1)
pc = PathCache(g, np.arange(V, dtype=np.int32))
pc.build()
i = pc.info()
out = np.zeros((1024, 16), dtype=np.uint64)
f = S.lib().shd_debug_sssp_timing
f.argtypes = [C.c_void_p]
assert f(out.ctypes.data) == 0
used = out[:, 7] > 0
o = out[used].astype(np.float64)
waves = 16
print(f"V={V} build {i.build_ms_sssp:.2f} ms, blocks {used.sum()}, rows {int(o[:, 7].sum())}")
print(f"per row: iterations {o[:, 4].sum() / o[:, 7].sum():.1f}, frontier vertices {o[:, 5].sum() / o[:, 7].sum():.0f}")
tot = o[:, 0].sum() / waves
for k, name in ((1, "iteration loop (scan + frontier)"), (2, "frontier work"), (3, "barrier wait")):
    print(f"{name:36s} {o[:, k].sum() / waves / tot * 100:5.1f} % of BF cycles (per-wave mean)")
print(f"BF cycles per row per wave {tot / o[:, 7].sum():.0f}; per iteration {tot / o[:, 4].sum():.0f}")
rows = o[:, 7].sum()
for k, name in ((0, "Bellman-Ford"), (8, "parents"), (9, "targets, first pass"), (10, "tree arrays"),
                (11, "tree prefix sweeps"), (12, "reliability pass")):
    print(f"{name:36s} {o[:, k].sum() / waves / rows:10.0f} cycles per row per wave")
