#!/usr/bin/env python3
"""One rank of a TCP-path group run -- TEST INFRASTRUCTURE (tests/
test_tcp_group_gpu.py starts `world` of these as child processes).

Each rank builds the same model (a case of tests/tcp_cases.py, or
workloads.mixed_transport_model / tcp_echo_model at a given size), creates a
host-memory communicator (shd_comm_create_host: several ranks on one GPU),
runs its share of the hosts through shd_tcp_run_group (shadow-1_amd/tcp.py
with comm) and writes its hosts' lines and end state to <out>/rank<r>.npz.
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(HERE), "shadow-1_amd"), HERE]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--name", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--case", required=True, help="a tcp_cases name, or mixed:H:loss:qdisc, or echo:H:loss")
    ap.add_argument("--mode", default="tables", choices=["tables", "device"])
    a = ap.parse_args()
    import sim
    import tcp as TCPGPU
    import tcp_cases as TC
    import workloads as W
    udp, qdisc = None, 0
    if a.case.startswith(("mixed:", "echo:")):
        kind, h, loss, *rest = a.case.split(":")
        if kind == "mixed":
            g, m, ips, procs, peers, nb, udp = W.mixed_transport_model(int(h), 40, end_s=10, nbytes=60000,
                                                                        loss_max=float(loss))
            qdisc = int(rest[0]) if rest else 0
        else:
            g, m, ips, procs, peers, nb = W.tcp_echo_model(int(h), 40, end_s=12, nbytes=60000, loss_max=float(loss))
    else:
        fix = json.load(open(os.path.join(HERE, "golden", "ref_tcp.json")))[a.case]
        c, m = TC.build(a.case)
        g, ips, procs, peers, nb = c["graph"], TC.ip_ints(fix["ips"]), c["procs"], c["peers"], c["nbytes"]
        udp, qdisc = TC.udp_arg(c), c.get("qdisc", 0)
    comm = sim.Comm.host(a.name, a.world, a.rank, 0)
    r = TCPGPU.run(m, g, ips, procs, peers, nbytes=nb, node=True, qdisc=qdisc, udp=udp, comm=comm, mode=a.mode)
    comm.close()
    np.savez(os.path.join(a.out, f"rank{a.rank}.npz"), lines=json.dumps(r["lines"]),
             node_lines=json.dumps(r["node_lines"]), next_event_id=r["next_event_id"],
             next_packet_id=r["next_packet_id"], rng_probe=r["rng_probe"], first_host=r["first_host"],
             n_local_hosts=r["n_local_hosts"], rounds=r["rounds"], events=r["events"],
             first_touch_runs=r.get("first_touch_runs", 0), first_touch=r["first_touch"])
    print(f"rank {a.rank}: hosts [{r['first_host']}, {r['first_host'] + r['n_local_hosts']}) rounds {r['rounds']} "
          f"events {r['events']}", flush=True)


if __name__ == "__main__":
    main()
