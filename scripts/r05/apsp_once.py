"""One 10 k x 10 k APSP build (the PMC passes' workload)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "shadow-1_amd"))
import numpy as np  # noqa: E402

import workloads as W  # noqa: E402
from sim import PathCache  # noqa: E402

g = W.geometric_graph(10000, seed=1)
pc = PathCache(g, np.arange(10000, dtype=np.int32))
print("build_ms", round(pc.info().build_ms_device, 3), flush=True)
pc.close()
