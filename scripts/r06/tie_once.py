"""One path-cache build of the 10 k whole-millisecond geometric graph (every row ties): the
tie kernel's profiling target (rocprofv3 --pmc / --kernel-trace); --float: the tie-free graph."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "shadow-1_amd"))
import numpy as np  # noqa: E402

import workloads as W  # noqa: E402
from sim import PathCache  # noqa: E402

# (--float: the headline's tie-free graph instead)
g = W.geometric_graph(10000, seed=1, integer_latency="--float" not in sys.argv)
pc = PathCache(g, np.arange(10000, dtype=np.int32))
i = pc.info()
print("build_ms", round(i.build_ms_device, 3), "tie_rows", i.n_tie_rows, flush=True)
pc.close()
