#!/usr/bin/env python3
"""Per-dispatch distribution of FETCH_SIZE / WRITE_SIZE (KB) of k_round_tl:
deciles over the last 2048 dispatches (diagnostic)."""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_bytes import per_dispatch  # noqa: E402

for d, c in ((sys.argv[1], "FETCH_SIZE"), (sys.argv[2], "WRITE_SIZE")):
    v = np.array(per_dispatch(d, c, "k_round_tl"))
    t = v[-2048:]
    print(c, "all", len(v), "mean %.1f" % v.mean(), "| last 2048 mean %.1f" % t.mean(),
          "deciles", np.percentile(t, [0, 10, 25, 50, 75, 90, 100]).round(1).tolist())
