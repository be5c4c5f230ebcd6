#!/usr/bin/env python3
"""Full-size parity fixtures from the oracle -- TEST INFRASTRUCTURE.

Runs the serial oracle (oracle/liboracle.so: the reference's --workers 0 loop
restated) on the BASELINE configurations at the sizes the
bench runs them, and commits what the HIP engine must reproduce bit for bit:

  c1_example.npz      C1: resource/examples/shadow.config.xml (2 hosts, the
                      1-vertex "isp" topology, process starts at 1 s / 2 s,
                      stoptime 3600 s) through the config front-end, PHOLD-UDP
                      in place of tgen: the full trace and every host digest.
  c3_full.npz         C3 exactly as bench.py builds its headline (10 k hosts on
                      the 10 k-vertex geometric graph, seed 1, load 16, 1-byte
                      messages, lossless paths), 3 simulated seconds: every host
                      digest, each host's trace multiset hash, totals.
  c3_lossy_full.npz   the same with edge loss U[0, 0.0005] (bench's lossy run).
  c5_codel_full.npz   C5 at full size with CoDel queues building: 1 M hosts,
                      100 per vertex of the 10 k-vertex graph, edge loss
                      U[0, 0.01], 1500-B payloads, rx 512 KiB/s, load 32,
                      to 1.25 s (the application starts at 1 s): digest hashes
                      per 1024-host block, the CoDel drop total, totals.

The reference event loop itself cannot be built here, so
these pin the HIP engine to the restatement at full size; the restatement's
pieces are pinned to the reference's own C (tests/test_oracle_ref.py).

usage: python tests/golden/make_fullsize.py [c1 c3 c3_lossy c5]
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd"), os.path.join(REPO, "tests")]

import fixture_hash as FH   # noqa: E402
import oracle_ffi as O      # noqa: E402
import shdgpu as S          # noqa: E402
import workloads as W       # noqa: E402
from fullsize_configs import CONFIGS, build   # noqa: E402


def dump(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path)} B)", flush=True)


def main(which):
    for key in which:
        cfg = CONFIGS[key]
        t0 = time.time()
        g, m, pushes = build(key)
        trace = cfg["fixture"] in ("full_trace", "trace_hash")
        tr, dg, st = O.engine_run(m, g, pushes=pushes)
        print(f"{key}: oracle {time.time() - t0:.1f}s  events {st['n_events']}  packet events "
              f"{st['n_pkt_events']}  trace {len(tr)}", flush=True)
        tot = np.array([st["n_events"], st["n_pkt_events"], len(tr)], dtype=np.uint64)
        if cfg["fixture"] == "full_trace":
            dump(cfg["file"], trace=tr, digest=dg, totals=tot)
        elif cfg["fixture"] == "trace_hash":
            assert trace
            dump(cfg["file"], digest=dg, trace_hash=FH.trace_host_hashes(tr, m.n_hosts), totals=tot)
        else:
            sums = np.array([int(dg[f].sum()) for f in ("n_events", "n_pkt_events", "n_sent", "n_inet_drop",
                                                          "n_codel_drop", "n_recv")], dtype=np.uint64)
            dump(cfg["file"], block_hash=FH.digest_block_hashes(dg, cfg["block"]), sums=sums, totals=tot,
                 codel_max_queue=np.array([int(dg["codel_count"].max())]))


if __name__ == "__main__":
    main(sys.argv[1:] or list(CONFIGS))
