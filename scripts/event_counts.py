#!/usr/bin/env python3
"""Per-round event-path counters of the round kernels (full timing build):

    make -C shadow-1_amd timing && cp shadow-1_amd/libshdgpu_tim.so shadow-1_amd/libshdgpu_cnt.so
    SHDGPU_LIB=shadow-1_amd/libshdgpu_cnt.so python3 scripts/event_counts.py --workload c5 --hosts 125000

Counts (TCNT in eng_device.h) over one simulated 0.2 s after a 2 s warm-up:
CoDel / send-FIFO entries loaded from HBM, heap pushes and pops, inbox
events merged, events, wave flushes, lanes suspended for a flush.
"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd")]

import numpy as np  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["c3", "c4", "c5"], default="c3")
    ap.add_argument("--hosts", type=int, default=10000)
    ap.add_argument("--vertices", type=int, default=10000)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import shdgpu as S
    import workloads as W
    from sim import Engine, PathCache
    lib = S.lib()
    if a.workload == "c4":
        g, m = W.tor_model(6500, 50000, end_time=4 * S.SHD_SEC, seed=1, load=4, payload=1)
        hv = m.host_vertex
    else:
        hv = (np.arange(a.hosts, dtype=np.int64) * a.vertices // a.hosts).astype(np.int32)
        if a.workload == "c5":
            g = W.geometric_graph(a.vertices, seed=1, loss_max=0.01)
            m = W.phold_model(hv, end_time=4 * S.SHD_SEC, seed=1, load=32, payload=1500, bw_down=512,
                              bw_up=10240, codelq_cap=256)
        else:
            g = W.geometric_graph(a.vertices, seed=1, loss_max=0.0)
            m = W.phold_model(hv, end_time=4 * S.SHD_SEC, seed=1, load=16, payload=1)
    pc = PathCache(g, W.attached_vertices(hv), device=0)
    pc.build()
    eng = Engine(m, pc, device=0)
    eng.boot()
    eng.run_until(2 * S.SHD_SEC)
    cn = np.zeros(8, dtype=np.uint64)
    fc = lib.shd_debug_counts
    fc.restype = C.c_int
    fc.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    fc(cn.ctypes.data_as(C.POINTER(C.c_uint64)), 1)
    st = eng.run_until(int(2.2 * S.SHD_SEC))
    fc(cn.ctypes.data_as(C.POINTER(C.c_uint64)), 1)
    nr = max(st.n_rounds, 1)
    names = ["cq HBM loads", "tq HBM loads", "heap pushes", "heap pops", "inbox merged", "events",
             "flushes (waves)", "suspended lanes"]
    print(f"{a.workload} {m.n_hosts} hosts, W {eng.window} ns: {st.n_rounds} rounds, "
          f"{st.n_pkt_events / nr:.0f} packet events, {st.n_events / nr:.0f} events, "
          f"{st.n_host_rounds / nr:.0f} active hosts per round; persistent {st.n_batches_persistent} "
          f"(sparse {st.n_batches_sparse}) of {st.n_batches} batches")
    print("per round: " + ", ".join(f"{names[i]} {cn[i] / nr:.1f}" for i in range(8)))


if __name__ == "__main__":
    main()
