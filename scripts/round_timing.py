#!/usr/bin/env python3
"""Per-block phase stamps of the round kernel (timing build).

    make -C shadow-1_amd timing
    SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so python scripts/round_timing.py

Stamps (100 MHz wall clock, relative to the round's first kernel entry):
0 kernel entry, 1 round body (after halt/ctl/prev loads), 2 after the idle
check, 3 after the active hosts' processing, 4 after the block reduction,
5 after the last-block ticket, 6 last block after the first-touch resolve.
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
    ap.add_argument("--vertices", type=int, default=10000)
    ap.add_argument("--hosts", type=int, default=10000)
    ap.add_argument("--load", type=int, default=16)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import shdgpu as S
    import workloads as W
    from sim import Engine, PathCache
    lib = S.lib()
    f = lib.shd_debug_timing
    f.restype = C.c_int
    f.argtypes = [C.POINTER(C.c_uint64)]
    g = W.geometric_graph(a.vertices, seed=1, loss_max=0.0)   # the bench headline (lossless)
    hv = (np.arange(a.hosts, dtype=np.int64) * a.vertices // a.hosts).astype(np.int32)
    m = W.phold_model(hv, end_time=4 * S.SHD_SEC, seed=1, load=a.load, payload=1)
    pc = PathCache(g, W.attached_vertices(hv), device=0)
    pc.build()
    eng = Engine(m, pc, 0, a.hosts, device=0)
    eng.boot()
    eng.run_until(2 * S.SHD_SEC)
    eng.run_until(int(2.2 * S.SHD_SEC))   # ticketless batches from here on
    kc = np.zeros(40, dtype=np.uint64)
    fk = lib.shd_debug_kind_costs
    fk.restype = C.c_int
    fk.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    fk(kc.ctypes.data_as(C.POINTER(C.c_uint64)), 1)
    cn = np.zeros(8, dtype=np.uint64)
    fc = lib.shd_debug_counts
    fc.restype = C.c_int
    fc.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    fc(cn.ctypes.data_as(C.POINTER(C.c_uint64)), 1)
    st = eng.run_until(int(2.5 * S.SHD_SEC))
    fk(kc.ctypes.data_as(C.POINTER(C.c_uint64)), 1)
    fc(cn.ctypes.data_as(C.POINTER(C.c_uint64)), 1)
    nr = max(st.n_rounds, 1)
    names = ["cq HBM loads", "tq HBM loads", "heap pushes", "heap pops", "inbox merged", "events", "flushes (waves)",
             "suspended lanes"]
    print("per round: " + ", ".join(f"{names[i]} {cn[i] / nr:.1f}" for i in range(8)))
    buf = np.zeros(64 * 2048 * 24, dtype=np.uint64)
    f(buf.ctypes.data_as(C.POINTER(C.c_uint64)))
    t = buf.reshape(64, 2048, 24).astype(np.int64)
    hpw = int(os.environ.get("SHD_HPW", "64"))
    grid = (a.hosts + hpw - 1) // hpw
    t = t[:, :grid, :]
    print(f"ticketless batches {st.n_batches_ticketless}")
    print(f"kernel {st.device_ms_round_kernel / max(st.n_rounds, 1) * 1e3:.1f} us/round (in-kernel stamps), "
          f"wall {st.wall_ms / max(st.n_rounds, 1) * 1e3:.1f} us/round, grid {grid}")
    names = ["entry", "body", "idle-chk", "active", "reduce", "ticket", "resolve"]
    rows = []
    keep = []
    for r in range(64):
        x = t[r]
        if (x[:, 0] == 0).any() or (x[:, 1:6] < x[:, :1]).any():
            continue   # a forward-only round (stamp 0 only) or stale stamps
        t0 = x[:, 0].min()
        rel = (x[:, :11] - t0) / 100.0   # us
        fresh = (x[:, 7:11] >= t0).all(axis=1, keepdims=True)   # stale stamps: no active host this round
        rel[:, 7:11] = np.where(fresh, rel[:, 7:11], 0)
        rows.append(rel)
        keep.append(r)
    rows = np.array(rows)   # rounds x blocks x 8
    print(f"{len(rows)} rounds; us from the round's first kernel entry: mean over rounds of (mean, max over blocks)")
    for k in range(6):
        v = rows[:, :, k]
        print(f"  {names[k]:9s} mean {v.mean():6.2f}  max {v.max(axis=1).mean():6.2f}")
    last = rows[:, :, 6].max(axis=1)
    print(f"  {names[6]:9s} (last block) {last.mean():6.2f}")
    # inside the active section (first active lane's stamps; blocks with an active host)
    act = rows[:, :, 9] > 0
    for k0, k1, nm in ((2, 7, "load_ctx"), (7, 8, "bins+merge"), (8, 9, "event loop"), (9, 10, "cal clear+next"),
                       (10, 3, "store ctx")):
        d = (rows[:, :, k1] - rows[:, :, k0])
        print(f"  {nm:15s} per block: mean {d[act].mean():7.2f} max {np.where(act, d, 0).max(axis=1).mean():7.2f} us")
    if os.environ.get("SHD_TIMING_LIGHT"):
        fl = (t[keep][:, :, 11] - t[keep][:, :, 0].min(axis=1, keepdims=True)) / 100.0
        ok = (t[keep][:, :, 11] >= t[keep][:, :, 0].min(axis=1, keepdims=True)) & (rows[:, :, 9] > 0)
        d = rows[:, :, 9] - fl
        print(f"  flush (light stamps) per block: mean {d[ok].mean():.2f} max {np.where(ok, d, 0).max(axis=1).mean():.2f} us; "
              f"flush start mean {fl[ok].mean():.2f}")
        t0 = t[keep][:, :, 0].min(axis=1, keepdims=True)
        prev = fl
        for k, nm in ((12, "prefix + index"), (13, "resolve (path loads)"), (14, "per-host walk")):
            x = (t[keep][:, :, k] - t0) / 100.0
            okk = ok & (t[keep][:, :, k] >= t0)
            dd = x - prev
            print(f"    {nm:22s} mean {dd[okk].mean():.2f} max {np.where(okk, dd, 0).max(axis=1).mean():.2f} us")
            prev = x
        dd = rows[:, :, 9] - prev
        print(f"    {'claims issue':22s} mean {dd[ok].mean():.2f} us")
        return
    raw = t[keep][:, :, 11:18].astype(np.float64)
    ok = raw[:, :, 4] > 0
    loopw = rows[:, :, 9] - rows[:, :, 8]   # us (wall) of the event loop
    ghz = raw[:, :, 4][ok & act].sum() / (loopw[ok & act].sum() * 1e3) if (ok & act).any() else 0
    print(f"  loop iterations/wave (max lane) mean {raw[:, :, 0][ok].mean():.1f} max {raw[:, :, 0].max():.0f}; "
          f"clock64 rate {ghz:.2f} GHz")
    tot = raw[:, :, 4][ok].mean()
    for j, nm in ((1, "take_next"), (2, "begin_event"), (3, "run_work"), (5, "flush_wave"), (6, "inner loops")):
        print(f"    {nm:12s} {raw[:, :, j][ok].mean():9.0f} cyc/wave ({100 * raw[:, :, j][ok].mean() / tot:4.1f}% of loop "
              f"{tot:.0f}); per iteration {raw[:, :, j][ok].sum() / raw[:, :, 0][ok].sum():7.0f}")
    kd = t[keep][:, :, 18:20].astype(np.float64)
    it = raw[:, :, 0][ok].sum()
    print(f"  divergence: {kd[:, :, 0][ok].sum() / it:.2f} distinct event kinds and "
          f"{kd[:, :, 1][ok].sum() / it:.1f} lanes starting an event per iteration")
    kc = kc.reshape(10, 4).astype(np.float64)
    kn = {1: "HEARTBEAT", 2: "REFILL", 3: "REFILL_LO", 4: "APP_START", 5: "PACKET fast", 6: "LOCAL", 7: "NOTIFY",
          8: "PACKET general"}
    print("  single-class iterations: class, iterations, cycles per iteration (take_next / begin_event / rest)")
    for k in range(1, 9):
        if kc[k, 0]:
            n = kc[k, 0]
            print(f"    {kn[k]:15s} {n:10.0f} {kc[k, 1] / n:7.0f} ({kc[k, 2] / n:5.0f} / {kc[k, 3] / n:5.0f} / "
                  f"{(kc[k, 1] - kc[k, 2] - kc[k, 3]) / n:5.0f})")
    d = rows[:, :, 3] - rows[:, :, 2]
    print(f"  active-phase duration per block: mean {d.mean():.2f} max {d.max(axis=1).mean():.2f} us")
    d = rows[:, :, 5] - rows[:, :, 3]
    print(f"  reduce+ticket per block: mean {d.mean():.2f} max {d.max(axis=1).mean():.2f} us")
    eng.close()
    pc.close()


if __name__ == "__main__":
    main()
