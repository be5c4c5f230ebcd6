"""Fixtures of the TCP echo models from the reference's own loop -- TEST
INFRASTRUCTURE.  Runs each case of tests/tcp_cases.py through
oracle/_ref/libshdref_loop.so (the reference's tcp.c, tcp_cong_reno.c,
tcp_retransmit_tally.cc, socket.c, network_interface.c, worker.c ... compiled
unmodified; oracle/Makefile `ref`) and stores what a run must reproduce:
the host IPs, the number and SHA-256 of the [STATUS] lines (in the serial
order, and grouped by host in each host's order) and of the tracker's [node]
lines (by time and host), and every host's
next event ID, next packet ID and RNG draw at the end.

    python tests/golden/make_ref_tcp.py        # -> tests/golden/ref_tcp.json
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(os.path.dirname(HERE)), "shadow-1_amd")]

import ref_loop_ffi as R  # noqa: E402
import tcp_cases as TC  # noqa: E402


def main():
    path = os.path.join(HERE, "ref_tcp.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    names = sys.argv[1:] or list(TC.CASES)
    for name in names:
        c, m = TC.build(name)
        r = R.run(m, c["graph"], procs=c["procs"], tcp=TC.tcp_arg(c))
        st = TC.status_lines(r["lines"])
        hb = TC.node_lines(r["lines"])
        out[name] = dict(ips=r["ip"], n_status=len(st), status_sha256=TC.digest(st),
                         n_heartbeat=len(hb), heartbeat_sha256=TC.digest(hb),
                         status_by_host_sha256=TC.digest(TC.by_host(st)),
                         next_event_id=[int(x) for x in r["next_event_id"]],
                         next_packet_id=[int(x) for x in r["next_packet_id"]],
                         rng_probe=[int(x) for x in r["rng_probe"]])
        print(name, len(st), flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
