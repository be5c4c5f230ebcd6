#!/usr/bin/env python3
"""Per-round cost of the round drivers on one GPU (C3 workload, 10k hosts):
single engine (shd_eng_run_until), a one-rank RCCL engine group, and local
groups of 2 / 4 engines sharing the GPU (device-to-device exchange)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd")]


def main():
    import torch
    torch.cuda.set_device(0)
    import shdgpu as S
    import workloads as W
    from driver import partition
    from sim import Engine, PathCache, XGroup
    V = H = 10000
    g = W.geometric_graph(V, seed=1, loss_max=0.0005)
    hv = W.hosts_on_vertices(V, 1)
    m = W.phold_model(hv, end_time=4 * S.SHD_SEC, seed=1, load=16, payload=1)
    pc = PathCache(g, W.attached_vertices(hv), device=0)
    modes = sys.argv[1:] or ["single", "rccl1", "local2", "local4"]
    for mode in modes:
        if mode == "single":
            e = Engine(m, pc)
            e.boot()
            runner, engines = e.run_until, [e]
        elif mode == "rccl1":
            e = Engine(m, pc)
            grp = XGroup.rccl(e, XGroup.unique_id(), 1, 0)
            runner, engines = grp.run_until, [e]
        else:
            n = int(mode[-1])
            pb = partition(H, n)
            engines = [Engine(m, pc, pb[i], pb[i + 1]) for i in range(n)]
            grp = XGroup.local(engines)
            runner = grp.run_until
        runner(2 * S.SHD_SEC)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = runner(3 * S.SHD_SEC)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"{mode:7s} rounds {st.n_rounds}  {dt * 1e6 / max(st.n_rounds, 1):7.1f} us/round  "
              f"kernel {st.device_ms_round_kernel * 1e3 / max(st.n_rounds, 1) / len(engines):6.1f} us/engine-round  "
              f"pkt events/s {st.n_pkt_events / dt / 1e6:.2f} M", flush=True)
        if mode != "single":
            grp.close()
        for x in engines:
            x.close()


if __name__ == "__main__":
    main()
