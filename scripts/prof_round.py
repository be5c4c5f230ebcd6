#!/usr/bin/env python3
"""Per-phase clock breakdown of the round kernel (instrumented build).

    make -C shadow-1_amd prof
    SHDGPU_LIB=shadow-1_amd/libshdgpu_prof.so python scripts/prof_round.py

Runs the bench workload (C3: 10k hosts on a 10k-vertex geometric graph, load
16), warms up, then reports, over one simulated second, the per-phase shader
clock totals of the non-idle host threads: the mean per thread-round and the
max over thread-rounds (the max bounds the kernel's critical path).
"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd")]

import numpy as np  # noqa: E402

NAMES = ["total", "load_ctx", "merge", "pop", "exec_pkt", "exec_notify", "exec_refill", "exec_other",
         "pick_dest", "send_packet", "store_ctx", "events"]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--vertices", type=int, default=10000)
    ap.add_argument("--hosts", type=int, default=10000)
    ap.add_argument("--load", type=int, default=None)
    ap.add_argument("--workload", choices=["c3", "c4", "c5"], default="c3",
                    help="c4: bench.py's Tor-scale model (6.5 k relays + 50 k clients); c5: bench.py's C5 "
                         "model at --hosts hosts (the per-GPU shard: 125000)")
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import shdgpu as S
    import workloads as W
    from sim import Engine, PathCache
    lib = S.lib()
    n = 2 * len(NAMES) + 2
    try:
        f = lib.shd_debug_prof
        f.restype = C.c_int
        f.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    except AttributeError:   # plain build: kernel time only
        f = lambda b, k: None  # noqa: E731
    buf = (C.c_uint64 * n)()
    if a.workload == "c4":   # as bench.py --workload c4 (lossless edges: --lossy-edge-loss-max 0)
        g, m = W.tor_model(6500, 50000, end_time=4 * S.SHD_SEC, seed=1, load=a.load or 4, payload=1)
        hv = m.host_vertex
        a.hosts = m.n_hosts
    elif a.workload == "c5":
        g = W.geometric_graph(a.vertices, seed=1, loss_max=0.01)
        hv = (np.arange(a.hosts, dtype=np.int64) * a.vertices // a.hosts).astype(np.int32)
        m = W.phold_model(hv, end_time=4 * S.SHD_SEC, seed=1, load=a.load or 32, payload=1500, bw_down=512,
                          bw_up=10240, codelq_cap=256)
    else:
        g = W.geometric_graph(a.vertices, seed=1, loss_max=0.0005)
        hv = (np.arange(a.hosts, dtype=np.int64) * a.vertices // a.hosts).astype(np.int32)
        m = W.phold_model(hv, end_time=4 * S.SHD_SEC, seed=1, load=a.load or 16, payload=1)
    pc = PathCache(g, W.attached_vertices(hv), device=0)
    pc.build()
    eng = Engine(m, pc, 0, a.hosts, device=0)
    eng.boot()
    eng.run_until(2 * S.SHD_SEC)
    f(buf, n)
    try:
        fw = lib.shd_debug_waves
        fw.restype = C.c_int
        fw.argtypes = [C.POINTER(C.c_uint64)]
    except AttributeError:
        fw = None
    wbuf = (C.c_uint64 * (128 * 8))()
    if fw:
        fw(wbuf)
    st = eng.run_until(3 * S.SHD_SEC)
    f(buf, n)
    v = np.array(buf[:], dtype=np.float64)
    k = len(NAMES)
    cnt = v[2 * k]
    rounds = st.n_rounds
    print(f"[{os.path.basename(S.LIB_PATH)} hpw={os.environ.get('SHD_HPW', '64')}] rounds {rounds}  kernel {st.device_ms_round_kernel / max(rounds, 1) * 1e3:.1f} us/round  "
          f"active thread-rounds {cnt:.0f} ({cnt / max(rounds, 1):.0f}/round)")
    for i, nm in enumerate(NAMES if cnt else []):
        print(f"  {nm:12s} mean {v[i] / max(cnt, 1):10.1f}   max {v[k + i]:10.0f}")
    if fw:
        # one more simulated 100 ms: per-round wave statistics (last <= 128 rounds)
        fw(wbuf)
        eng.run_until(int(3.1 * S.SHD_SEC))
        fw(wbuf)
        w = np.array(wbuf[:], dtype=np.float64).reshape(128, 8)
        w = w[w[:, 4] > 0]
        span = (w[:, 1] - w[:, 0]) / 100.0   # us (100 MHz)
        print(f"wave timing over {len(w)} rounds (us): span mean {span.mean():.1f} max {span.max():.1f}; "
              f"longest wave mean {w[:, 2].mean() / 100:.1f}; mean wave {(w[:, 3] / w[:, 4]).mean() / 100:.1f}; "
              f"waves/round {w[:, 4].mean():.0f}; max lane events/round mean {w[:, 5].mean():.1f} "
              f"max {w[:, 5].max():.0f}; mean over waves of max-lane events {(w[:, 6] / w[:, 4]).mean():.2f}")
    eng.close()
    pc.close()


if __name__ == "__main__":
    main()
