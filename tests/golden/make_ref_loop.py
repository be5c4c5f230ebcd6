#!/usr/bin/env python3
"""Fixtures from the reference's own event loop -- TEST INFRASTRUCTURE.

Runs every model of tests/ref_loop_cases.py through oracle/_ref/
libshdref_loop.so: Shadow's worker.c / scheduler.c / host.c /
network_interface.c / router*.c / descriptor/*.c / tracker.c / packet.c ...
compiled unmodified from /root/reference (oracle/Makefile `ref`), in serial
mode, with the collaborators the image cannot build (slave, the igraph
topology, the rpth process layer, the loggers) as the test doubles of
oracle/ref_harness/ref_loop.c.  The topology double serves the oracle's lazy
path cache (o_topo_get), the one piece of the composition that stays a
restatement (igraph is absent).

Written to tests/golden/ref_loop.json, per case:
  ips             the addresses the reference's DNS gave the hosts
  n_status, status_sha256
                  every [STATUS] line (packet.c:647-659) the run logged, with
                  its simulated time and host, ordered by (time, host), each
                  host's lines in the order they were logged
  n_heartbeat, heartbeat_sha256
                  the same for the tracker's [shadow-heartbeat] lines
  next_event_id, next_packet_id, rng_probe
                  per host at the end: the event and packet ID counters and
                  the next rand_r of the host RNG

usage: python tests/golden/make_ref_loop.py [case ...]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd"), os.path.join(REPO, "tests")]

import ref_loop_cases as RC   # noqa: E402
import ref_loop_ffi as R      # noqa: E402

OUT = os.path.join(HERE, "ref_loop.json")


def main(names):
    data = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            data = json.load(f)
    for name in names or list(RC.CASES):
        case = RC.CASES[name]()
        t0 = time.time()
        r = R.run(case["model"], case["graph"], procs=RC.procs_of(case), echo=case["model"].app_peer)
        st, hb = RC.split_lines(r["lines"])
        data[name] = dict(ips=r["ip"], n_status=len(st), status_sha256=RC.digest_lines(st),
                          n_heartbeat=len(hb), heartbeat_sha256=RC.digest_lines(hb),
                          next_event_id=[int(x) for x in r["next_event_id"]],
                          next_packet_id=[int(x) for x in r["next_packet_id"]],
                          rng_probe=[int(x) for x in r["rng_probe"]])
        print(f"{name}: {len(st)} status lines, {len(hb)} heartbeat lines, {time.time() - t0:.1f} s")
    with open(OUT, "w") as f:
        json.dump(data, f, indent=0, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main(sys.argv[1:])
