"""max deliveries per round of the TCP path for a few wide-window models"""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd"), os.path.join(REPO, "tests")]
import tcp as T  # noqa: E402
import workloads as W  # noqa: E402
for bw, nb, V, hosts in [(122070, 20_000_000, 40, 2), (122070, 8_000_000, 40, 130)]:
    g, m, ips, procs, peers, _ = W.tcp_echo_model(hosts, V, end_s=8, nbytes=nb, bw_down=bw, bw_up=bw)
    r = T.run(m, g, ips, procs, peers, nbytes=nb, trace=False)
    print(bw, nb, V, hosts, "rounds", r["rounds"], "events", r["events"], "max/round", r["max_round_deliveries"], "overflow", r["max_round_overflow"], r["first_touch"],
          "err", r.get("error"), flush=True)
