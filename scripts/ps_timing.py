#!/usr/bin/env python3
"""Per-block phase stamps of the persistent round kernel (k_round_ps), from
the timing build:

    make -C shadow-1_amd timing TIMING_FLAGS=-DSHD_TIMING_LIGHT
    SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so python3 scripts/ps_timing.py

Stamps (100 MHz wall clock; every stamp first drains the wave's memory ops):
0 round start, 1 hand-off words read (idle test; k_round_sp: the scan and compaction), 2 bins + inbox merged and
sorted, 3 last flush starts, 4 event loop + flushes done, 5 close done
(bin resets, last deliveries), 6 share published (drained), 7 every share of
the round seen.  Printed relative to the round's earliest start: mean over
rounds of the mean and the max over blocks; and the phase durations.
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
    ap.add_argument("--load", type=int, default=None)
    ap.add_argument("--at", type=float, default=2.0, help="simulated seconds before the measured rounds")
    ap.add_argument("--workload", choices=["c3", "c5"], default="c3",
                    help="c5: bench.py's C5 model at --hosts hosts (the per-GPU shard: 125000; k_round_sp)")
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
    hv = (np.arange(a.hosts, dtype=np.int64) * a.vertices // a.hosts).astype(np.int32)
    if a.workload == "c5":
        g = W.geometric_graph(a.vertices, seed=1, loss_max=0.01)
        m = W.phold_model(hv, end_time=int((a.at + 2) * S.SHD_SEC), seed=1, load=a.load or 32, payload=1500, bw_down=512,
                          bw_up=10240, codelq_cap=256)
    else:
        g = W.geometric_graph(a.vertices, seed=1, loss_max=0.0)
        m = W.phold_model(hv, end_time=int((a.at + 2) * S.SHD_SEC), seed=1, load=a.load or 16, payload=1)
    pc = PathCache(g, W.attached_vertices(hv), device=0)
    pc.build()
    eng = Engine(m, pc, 0, a.hosts, device=0)
    eng.boot()
    eng.run_until(int(a.at * S.SHD_SEC))
    buf0 = np.zeros(64 * 2048 * 24, dtype=np.uint64)
    f(buf0.ctypes.data_as(C.POINTER(C.c_uint64)))   # the stamps before the measured rounds
    fc = lib.shd_debug_counts
    fc.restype = C.c_int
    fc.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    cn = np.zeros(8, dtype=np.uint64)
    fc(cn.ctypes.data_as(C.POINTER(C.c_uint64)), 1)
    st = eng.run_until(int(a.at * S.SHD_SEC) + 60 * eng.window)   # under one persistent batch: its rounds leave their stamps
    print(f"persistent batches {st.n_batches_persistent} of {st.n_batches}, rounds {st.n_rounds}, "
          f"{st.device_ms_launches / max(st.n_rounds, 1) * 1e3:.2f} us/round (HIP events)")
    fc(cn.ctypes.data_as(C.POINTER(C.c_uint64)), 1)
    if cn.any():   # a -DSHD_TCNT build: event-path counters over the measured rounds
        nr = max(st.n_rounds, 1)
        names_c = ["cq loads", "tq loads", "heap pushes", "heap pops", "inbox merged", "events", "flushes",
                   "suspended lanes"]
        print("counters per round: " + ", ".join(f"{n} {int(v) / nr:.1f}" for n, v in zip(names_c, cn)) +
              f"; packet events {st.n_pkt_events / nr:.1f}, events {st.n_events / nr:.1f}")
    buf = np.zeros(64 * 2048 * 24, dtype=np.uint64)
    f(buf.ctypes.data_as(C.POINTER(C.c_uint64)))
    t = buf.reshape(64, 2048, 24).astype(np.int64)
    t_before = buf0.reshape(64, 2048, 24).astype(np.int64)
    # the measured launch's blocks (k_round_ps: one per 64 hosts; k_round_sp: fewer) and its rounds' slots
    fresh = t[:, :, 0] != t_before[:, :, 0]
    grid = int(np.count_nonzero(fresh.any(axis=0)))
    t_all = np.where(fresh[:, :, None], t, 0)[:, :grid, :]
    t = t_all[:, :, :8]
    rows = []
    skipped = [0, 0]
    for r in range(64):
        x = t[r]
        t0 = x[:, 0].min()
        if t0 == 0 or (x[:, 6:8] < t0).any():
            skipped[0 if t0 == 0 else 1] += 1
            continue
        rel = (x - t0) / 100.0
        rel[x < t0] = np.nan    # a phase no lane of the block reached this round (no active host)
        rows.append(rel)
    rows = np.array(rows)
    if not len(rows):
        print(f"no complete round among the 64 slots (no start stamp: {skipped[0]}, older stamps: {skipped[1]}; "
              f"{grid} blocks)")
        return
    names = ["start", "words read", "bins merged", "last flush", "loop done", "close done", "published", "all seen"]
    print(f"{len(rows)} rounds; us from the round's earliest block start: mean over rounds of (mean, max over blocks)")
    for k in range(8):
        v = rows[:, :, k]
        print(f"  {k} {names[k]:12s} mean {np.nanmean(v):6.2f}  max {np.nanmean(np.nanmax(v, axis=1)):6.2f}")
    # the last flush's resolve loop (stamps 12, 13), in blocks that flushed
    fl = []
    for r in range(64):
        x = t_all[r]
        t0 = x[:, 0].min()
        ok = (x[:, 12] >= t0) & (x[:, 13] >= x[:, 12]) & (t0 > 0)
        if ok.any():
            fl.append(((x[ok, 12] - t0) / 100.0, (x[ok, 13] - x[ok, 12]) / 100.0))
    if fl:
        print(f"  last flush resolve: starts mean {np.mean([a.mean() for a, _ in fl]):.2f} us, lasts mean "
              f"{np.mean([b.mean() for _, b in fl]):.2f} / max {np.mean([b.max() for _, b in fl]):.2f} us")
    # the event loop: iterations (16), flushes (17), active lanes (18) per block and round, and
    # how the loop's length (stamp 2 -> 4) follows them
    it, nfl, nact, dur, seg = [], [], [], [], []
    for r in range(64):
        x = t_all[r]
        t0 = x[:, 0].min()
        ok = (t0 > 0) & (x[:, 4] >= x[:, 2]) & (x[:, 2] >= t0) & (x[:, 16] < 10000)
        it += list(x[ok, 16]); nfl += list(x[ok, 17]); nact += list(x[ok, 18])
        seg += [list(v) for v in x[ok][:, [8, 9, 10, 11, 15, 19]] / 100.0]
        dur += list((x[ok, 4] - x[ok, 2]) / 100.0)
    if it:
        it, nfl, nact, dur, seg = map(np.array, (it, nfl, nact, dur, seg))
        print(f"  loop: iterations mean {it.mean():.2f} max {it.max()}; flushes mean {nfl.mean():.2f}; "
              f"active lanes mean {nact.mean():.1f}; loop us mean {dur.mean():.2f}")
        for k in sorted(set(it.tolist()))[:12]:
            sel = it == k
            print(f"    {k:3d} iterations: {sel.sum():5d} block-rounds, loop {dur[sel].mean():.2f} us "
                  f"(take+begin {seg[sel, 0].mean():.2f} = take_next {seg[sel, 3].mean():.2f} + begin_event "
                  f"{seg[sel, 4].mean():.2f} + notify {seg[sel, 5].mean():.2f} + rest; run_work "
                  f"{seg[sel, 1].mean():.2f}, early flushes {seg[sel, 2].mean():.2f}), flushes {nfl[sel].mean():.2f}")
    # k_round_sp: active hosts (20) and passes (21) per block and round
    na, npas = [], []
    for r in range(64):
        x = t_all[r]
        t0 = x[:, 0].min()
        ok = (t0 > 0) & (x[:, 1] >= t0) & (x[:, 20] < 100000)
        na += list(x[ok, 20]); npas += list(x[ok, 21])
    if na and max(npas) > 0:
        na, npas = np.array(na), np.array(npas)
        print(f"  sparse: active hosts per block-round mean {na.mean():.2f} max {na.max()}; passes mean "
              f"{npas.mean():.2f} max {npas.max()}; blocks with none {np.mean(na == 0) * 100:.1f} %")
    # k_round_sp's scan: its first batch's words landed (22), the compaction done (23), from the round start
    sl, sc = [], []
    for r in range(64):
        x = t_all[r]
        t0 = x[:, 0].min()
        ok = (t0 > 0) & (x[:, 22] >= x[:, 0]) & (x[:, 23] >= x[:, 22]) & (x[:, 0] > 0)
        sl += list((x[ok, 22] - x[ok, 0]) / 100.0); sc += list((x[ok, 23] - x[ok, 22]) / 100.0)
    if sl:
        print(f"  sparse scan: block start -> words landed {np.mean(sl):.2f} us (max {np.max(sl):.2f}), "
              f"-> compaction done {np.mean(sc):.2f} us (max {np.max(sc):.2f})")
    # phase durations (mean over rounds of the mean over blocks)
    d = np.diff(rows, axis=2)
    print("  phase durations, mean over blocks: " + ", ".join(
        f"{names[k]}<-{names[k - 1]} {np.nanmean(d[:, :, k - 1]):.2f}" for k in range(1, 8)))
    per = np.diff(np.nanmax(rows[:, :, 7], axis=1))
    print(f"  round period (max 'all seen' to the next) {np.mean(per[per > 0]):.2f} us")


if __name__ == "__main__":
    main()
