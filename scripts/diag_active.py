"""Active host-round counts: single engine vs engine group (diagnostic)."""
import os
import sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "shadow-1_amd"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests")]
import shdgpu as S  # noqa: E402
import workloads as W  # noqa: E402
from driver import partition  # noqa: E402
from fullsize_configs import V, c3_hosts  # noqa: E402
from sim import Engine, PathCache, XGroup  # noqa: E402

hosts, parts = int(sys.argv[1]), int(sys.argv[2])
v = int(sys.argv[3]) if len(sys.argv) > 3 else V
g = W.geometric_graph(v, seed=1, loss_max=0.0)
m = W.phold_model(c3_hosts(hosts) if v == V else W.hosts_on_vertices(v, hosts // v),
                  end_time=3 * S.SHD_SEC, seed=1, load=16, payload=1)
pc = PathCache(g, W.attached_vertices(m.host_vertex))
e = Engine(m, pc)
st = e.run()
print("single", st.n_rounds, st.n_events, st.n_pkt_events, st.n_host_rounds, st.n_batches_ticketless,
      st.n_rounds_protected, flush=True)
e.close()
pb = partition(m.n_hosts, parts)
engines = [Engine(m, pc, pb[i], pb[i + 1]) for i in range(parts)]
grp = XGroup.local(engines)
gst = grp.run()
print("group", gst.n_rounds, gst.n_events, gst.n_pkt_events, gst.n_host_rounds, gst.n_batches_ticketless,
      gst.n_rounds_protected, flush=True)
