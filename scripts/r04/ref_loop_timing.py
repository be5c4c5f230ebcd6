"""The reference's OWN serial loop timed beside the port.

oracle/_ref/libshdref_loop.so is Shadow's worker.c / scheduler.c / host.c /
network_interface.c / router*.c / descriptor/*.c / tracker.c / packet.c
compiled unmodified (oracle/Makefile `ref`), run in serial mode (--workers 0)
with the harness's doubles for what the image cannot build (ref_loop.c), here
at the default log level's work (cfg.quiet: debug records filtered, so the
[STATUS] lines are not formatted).  The port is oracle/o_engine.c (bench.py's
cpu_baseline) and oracle/o_tcp.c.  Both run on this container's cores, one
thread each, on:

  C3   bench.py's headline workload (10 k hosts, 10 k-vertex geometric graph,
       load 16, lossless) -- the simulated second [2 s, 3 s): each loop is run
       to 2 s and to 3 s and the difference of the two wall times is divided
       into the packet events of [2 s, 3 s) (boot, application start and the
       lazy path cache's rows cancel);
  TCP  bench.py --workload tcp's model (echo pairs, 500 kB each way) at a
       bounded host count, whole runs.

Run in the build container only (it needs /root/reference's build):
  python scripts/r04/ref_loop_timing.py > profiles/r04/ref_loop_timing.json
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "shadow-1_amd")]

import numpy as np  # noqa: E402

import oracle_ffi as O  # noqa: E402
import ref_loop_ffi as R  # noqa: E402
import shdgpu as S  # noqa: E402
import workloads as W  # noqa: E402


def c3(end_s):
    V = 10000
    g = W.geometric_graph(V, seed=1, loss_max=0.0)
    m = W.phold_model(W.hosts_on_vertices(V, 1), end_time=int(end_s * S.SHD_SEC), seed=1, load=16, payload=1)
    return m, g


def port_run(m, g):
    t0 = time.perf_counter()
    _, dg, st = O.engine_run(m, g)
    return time.perf_counter() - t0, st, dg


def main():
    out = {"host_cpu": os.popen("grep -m1 'model name' /proc/cpuinfo").read().split(":")[-1].strip(),
           "threads": 1}
    # ---- C3, the simulated second [2 s, 3 s)
    res = {}
    for end in (2, 3):
        m, g = c3(end)
        r = R.run(m, g, quiet=True)
        pw, st, dg = port_run(m, g)
        assert r["next_event_id"].tolist() == dg["ev_seq"].tolist(), "reference and port end states differ"
        res[end] = dict(ref_s=r["run_s"], port_s=pw, pkt=int(st["n_pkt_events"]), ev=int(st["n_events"]))
    pkt = res[3]["pkt"] - res[2]["pkt"]
    ref_s = res[3]["ref_s"] - res[2]["ref_s"]
    port_s = res[3]["port_s"] - res[2]["port_s"]
    out["c3"] = {"window": "simulated [2 s, 3 s)", "packet_events": pkt,
                 "events": res[3]["ev"] - res[2]["ev"],
                 "reference_s": round(ref_s, 3), "reference_pkt_events_per_s": round(pkt / ref_s, 1),
                 "port_s": round(port_s, 3), "port_pkt_events_per_s": round(pkt / port_s, 1),
                 "reference_over_port": round(port_s / ref_s, 3),
                 "runs": {str(k): v for k, v in res.items()},
                 "same_end_state": True}
    # ---- TCP echo, whole runs
    H = int(os.environ.get("TCP_HOSTS", "1024"))
    g, m, ips, procs, peers, nb = W.tcp_echo_model(H, 1000, seed=1, end_s=20, nbytes=500000)
    ipa = np.asarray(ips, dtype=np.uint32)
    r = R.run(m, g, procs=procs, tcp=dict(peers=peers, nbytes=nb), quiet=True)
    t0 = time.perf_counter()
    o = O.tcp_run(m, g, ipa, procs, peers, nbytes=nb, lines=False)
    ps = time.perf_counter() - t0
    same = r["next_event_id"].tolist() == o["next_event_id"].tolist() and \
        r["rng_probe"].tolist() == o["rng_probe"].tolist()
    out["tcp"] = {"hosts": H, "events": int(o["events"]), "reference_s": round(r["run_s"], 3),
                  "reference_events_per_s": round(o["events"] / r["run_s"], 1),
                  "port_s": round(ps, 3), "port_events_per_s": round(o["events"] / ps, 1),
                  "reference_over_port": round(ps / r["run_s"], 3), "same_end_state": bool(same)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
