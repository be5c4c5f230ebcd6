"""Debug: the RCCL engine group at one rank, with and without protected rounds."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd"), os.path.join(REPO, "tests")]
import shdgpu as S, workloads as W
from sim import Engine, PathCache, XGroup
g = W.geometric_graph(200, seed=9)
m = W.phold_model(W.hosts_on_vertices(200, 1), end_time=2 * S.SHD_SEC, trace=True)
pc = PathCache(g, W.attached_vertices(m.host_vertex))
for mode in sys.argv[1:]:
    if mode == "noprot":
        os.environ["SHD_NO_PROTECT"] = "1"
    else:
        os.environ.pop("SHD_NO_PROTECT", None)
    for tr in ("local", "rccl"):
        eng = Engine(m, pc)
        grp = XGroup.rccl(eng, XGroup.unique_id(), 1, 0) if tr == "rccl" else XGroup.local([eng])
        try:
            st = grp.run()
            print(mode, tr, "rounds", st.n_rounds, "pkt", st.n_pkt_events, "prot", st.n_rounds_protected,
                  "rerun", st.n_rounds_rerun, "final", st.final_time, "err", st.error, flush=True)
        except Exception as ex:
            print(mode, tr, "EXC", ex, flush=True)
        grp.close(); eng.close()
