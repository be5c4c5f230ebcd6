#!/usr/bin/env python3
"""bench.py -- simulated packet events/s of libshdgpu (BASELINE.json metric).

Workload (N = --gpus, weak scaling): PHOLD-UDP on a V-vertex random geometric
topology (BASELINE.md C3 at N = 1: 10k hosts, one per vertex, load 16, 1-byte
messages; N x 10k hosts, N per vertex, at N > 1, toward C5).  One "step" is one
second of simulated time on the loaded model; W warmup steps (boot, the
application start at t = 1 s and the lazy path-cache warm-up) are untimed, then
K steps are timed between a barrier + synchronize on both sides; the reported
time is the max over ranks.  value = packet events (executed deliver-packet
events, worker.c:253) of all ranks / time.

Also reported: the APSP path-cache build time for the same 10k-vertex topology
(BASELINE metric 2), a roofline object for the round kernel (HIP-event device
time on the engine's stream; algorithmic bytes defined in DESIGN.md), and the
oracle's serial CPU loop as cpu_baseline (rank 0, N = 1 only).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd")]

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8 TB/s HBM3E (spec)
# algorithmic bytes = 80 per packet event (event read 32 +
# new event written 32 + path entry 16) + 136 per active host-round (host
# state read + written once per round in which the host executes anything)
BYTES_PER_PKT_EVENT = 80
BYTES_PER_HOST_ROUND = 136


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--vertices", type=int, default=10000)
    ap.add_argument("--hosts-per-gpu", type=int, default=None,
                    help="c3: hosts per GPU (default 10000, weak scaling); c5: given, the C5 model with this many "
                         "hosts per GPU (weak scaling: 125000 is the per-GPU shard of the north star's 1 M hosts "
                         "over 8 GPUs), absent, 1 M hosts split over the GPUs (strong scaling)")
    ap.add_argument("--load", type=int, default=None,
                    help="PHOLD messages per host at the application start (default 16; 4 for c4)")
    ap.add_argument("--payload", type=int, default=1)
    ap.add_argument("--step-ms", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--edge-loss-max", type=float, default=0.0,
                    help="edge loss ~ U[0, x] of the headline run.  PHOLD never regenerates a lost "
                         "message, so any loss makes the population (and the rate) decay with "
                         "simulated time; the default 0 keeps it stationary, so the value does not "
                         "depend on --steps / --warmup")
    ap.add_argument("--lossy-edge-loss-max", type=float, default=0.0005,
                    help="edge loss ~ U[0, x] of the lossy C3 run reported beside the headline "
                         "(its packet events per step show the decay); 0 skips it")
    ap.add_argument("--workload", choices=["c3", "c4", "c5", "tcp"], default="c3",
                    help="c3: PHOLD-UDP on the geometric topology (the headline, weak scaling); c4: the "
                         "Tor-scale relay/client model on the bundled topology (hosts fixed, strong scaling); "
                         "c5: 1 M hosts (100 per vertex of the geometric topology), 1500-B messages, 512 KiB/s "
                         "downlinks so CoDel queues build, edge loss U[0, 0.01] (hosts fixed, strong scaling; "
                         "lost messages are not regenerated, so the rate depends on the window); tcp: the "
                         "TCP path (include/shdtcp.h) on workloads.tcp_echo_model, one run per step")
    ap.add_argument("--tcp-bytes", type=int, default=500000, help="tcp: bytes each client echoes")
    ap.add_argument("--tcp-end-s", type=int, default=20, help="tcp: simulated seconds")
    ap.add_argument("--tcp-udp", action="store_true",
                    help="tcp: both transports -- workloads.mixed_transport_model (a datagram process on every "
                         "host beside the echo pairs)")
    ap.add_argument("--tcp-pool", type=int, default=2048,
                    help="tcp: packet pool per host (shd_tcp_model.packets_per_host; overflow fails the run)")
    ap.add_argument("--relays", type=int, default=6500)
    ap.add_argument("--clients", type=int, default=50000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true",
                    help="N > 1: skip the end-state check against one engine over all hosts on rank 0")
    ap.add_argument("--no-reference-cpu", action="store_true",
                    help="skip timing the reference's own serial loop (oracle/_ref/libshdref_loop.so)")
    ap.add_argument("--reference-window-ms", type=int, nargs=2, default=[1100, 1200],
                    help="the simulated window [t0, t1) over which the reference's own loop is timed")
    ap.add_argument("--cpu-sample-steps", type=int, default=0,
                    help="timed steps the CPU baseline runs (0 = all of them: the same window as value)")
    ap.add_argument("--exchange", choices=["p2p", "rccl", "torch"], default="p2p",
                    help="N > 1: p2p = shd_xgroup with the peer-to-peer transport (each rank's receive blocks "
                         "IPC-mapped by every rank and stored into over xGMI, tagged headers, in-kernel waits; "
                         "falls back to rccl if the mapping fails); rccl = shd_xgroup with one fixed-size RCCL "
                         "all-to-all per round; torch = driver.DistCluster (host-driven, torch.distributed)")
    ap.add_argument("--comm", choices=["rccl", "host"], default="rccl",
                    help="the engine group's communicator: rccl (one process per GPU), or host (processes of one "
                         "machine over shared memory, torch.distributed over gloo, every rank on GPU 0): a "
                         "rehearsal of the N > 1 path on a one-GPU machine, not a measurement")
    ap.add_argument("--group", action="store_true",
                    help="run the shd_xgroup path even at N = 1 (a one-rank RCCL group)")
    ap.add_argument("--quiet", action="store_true")
    return ap.parse_args()


class Roctx:
    """roctx ranges around the timed region, so that a
    `rocprofv3 --marker-trace --kernel-trace` run of this script can restrict
    its kernel statistics to the timed region (scripts/rocprof_timed.py);
    without the profiler they cost nothing.  Absent library: no markers."""
    def __init__(self):
        import ctypes
        self.lib = None
        # rocprofv3 (rocprofiler-sdk) traces the markers of its own roctx library
        for name in ("librocprofiler-sdk-roctx.so", "libroctx64.so"):
            try:
                self.lib = ctypes.CDLL(name)
                self.lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                break
            except OSError:
                self.lib = None

    def push(self, name):
        if self.lib is not None:
            self.lib.roctxRangePushA(name.encode())

    def pop(self):
        if self.lib is not None:
            self.lib.roctxRangePop()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


# RCCL writes its version banner to stdout when a communicator is created:
# everything but the JSON line goes to stderr
_STDOUT_FD = os.dup(1)
os.dup2(2, 1)


def main():
    args = parse()
    if args.workload == "tcp":
        return tcp_main(args)
    if args.load is None:
        args.load = {"c4": 4, "c5": 32}.get(args.workload, 16)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = args.gpus
    import torch
    dist = None
    rehearsal = args.comm == "host" and world > 1
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(0 if rehearsal else local_rank)
        dist.init_process_group("gloo" if rehearsal else "nccl")
    else:
        torch.cuda.set_device(0)
    dev = local_rank if world > 1 and not rehearsal else 0
    tdev = "cpu" if rehearsal else "cuda"   # the torch.distributed tensors' device

    import shdgpu as S
    import workloads as W
    from sim import Engine, PathCache
    from driver import DistCluster, partition

    t_setup = time.perf_counter()
    step = args.step_ms * S.SHD_MS
    end_time = (args.warmup + args.steps) * step
    if args.workload == "c4":
        # BASELINE C4: Tor-scale relays + clients on the bundled topology,
        # the hosts split over the ranks (strong scaling: the total is fixed)
        g, model = W.tor_model(args.relays, args.clients, end_time=end_time, seed=args.seed, load=args.load,
                               payload=args.payload)
        host_vertex = model.host_vertex
        V, H = g.n_vertices, model.n_hosts
    elif args.workload == "c5":
        # BASELINE C5 exactly as tests/fullsize_configs.py builds its fixture, the
        # 1 M hosts split over the ranks (the total is fixed); or with
        # --hosts-per-gpu, the same model at that many hosts per GPU
        V, hpv = args.vertices, 100
        g = W.geometric_graph(V, seed=args.seed, loss_max=0.01)
        if args.hosts_per_gpu:
            H = args.hosts_per_gpu * max(world, 1)
            host_vertex = (np.arange(H, dtype=np.int64) * V // H).astype(np.int32)
        else:
            host_vertex = W.hosts_on_vertices(V, hpv)
            H = len(host_vertex)
        model = W.phold_model(host_vertex, end_time=end_time, seed=args.seed, load=args.load, payload=1500,
                              bw_down=512, bw_up=10240, codelq_cap=256)
    else:
        V = args.vertices
        H = (args.hosts_per_gpu or 10000) * max(world, 1)
        g = W.geometric_graph(V, seed=args.seed, loss_max=args.edge_loss_max)
        hpv = max(1, H // V)
        host_vertex = (np.arange(H, dtype=np.int64) * V // H).astype(np.int32) if H != V * hpv else \
            W.hosts_on_vertices(V, hpv)
        model = W.phold_model(host_vertex, end_time=end_time, seed=args.seed, load=args.load,
                              payload=args.payload)
    att = W.attached_vertices(host_vertex)
    use_group = args.group or (world > 1 and args.exchange in ("p2p", "rccl"))
    comm = None
    if use_group:
        # one communicator per process: the sharded path-cache build and the
        # engine group's per-round exchange both run over it
        from sim import Comm, XGroup
        uid = torch.zeros(S.SHD_XID_BYTES, dtype=torch.uint8, device=tdev)
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(XGroup.unique_id() if not rehearsal else os.urandom(S.SHD_XID_BYTES)),
                                       dtype=torch.uint8))
        if world > 1:
            dist.broadcast(uid, 0)
        if rehearsal:   # the shared-memory segment's name from the broadcast token
            comm = Comm.host("shdbench_" + bytes(uid.cpu().numpy().tobytes())[:8].hex(), world, rank, dev)
        else:
            comm = Comm.rccl(bytes(uid.cpu().numpy().tobytes()), max(world, 1), rank, dev)
    # host buffers handed over at the boundary (graph CSR, model tables): their
    # upload is timed apart and reported as the PCIe-inclusive rate, never `value`
    torch.cuda.synchronize()
    t_up = time.perf_counter()
    pc = PathCache(g, att, device=dev, build=False)
    torch.cuda.synchronize()
    upload_s = time.perf_counter() - t_up
    # APSP (BASELINE metric 2): every rank builds every row (replicated), and
    # with a communicator each rank builds its block of rows and all-gathers
    # them (sharded by source rows); both timed, the engine runs on the last
    builds, sharded = [], []
    for _ in range(2):
        pc.build()
        builds.append(pc.info().build_ms_device)
    info = pc.info()
    if comm is not None and world > 1:
        for _ in range(2):
            if world > 1:
                dist.barrier()
            pc.build_sharded(comm)
            sharded.append(pc.info().build_ms_device)
    pb = partition(H, max(world, 1))
    t_up = time.perf_counter()
    eng = Engine(model, pc, pb[rank], pb[rank + 1], device=dev)
    torch.cuda.synchronize()
    upload_s += time.perf_counter() - t_up
    log(rank, f"setup {time.perf_counter() - t_setup:.1f}s  V={V} E={g.n_edges} H={H} W={eng.window}ns "
              f"apsp={min(builds):.1f}ms iters={info.sssp_iterations_max} hops={info.max_hops}")

    exchange = "none (single engine)"
    transport = "none" if world <= 1 and not use_group else "torch.distributed"
    if use_group:
        transport = "host-memory all-to-all" if args.comm == "host" else "rccl"
        exchange = "shd_xgroup/%s all-to-all" % ("host-memory" if args.comm == "host" else "RCCL")
        grp = None
        if args.exchange == "p2p":
            try:   # every rank fails alike (the mapping is checked collectively)
                grp = XGroup.over(eng, comm, p2p=True)
                # (ranks sharing a GPU are fused only while all their blocks fit its CUs one each)
                two_launch = os.environ.get("SHD_X_UNFUSED") or (
                    rehearsal and world * -(-(pb[rank + 1] - pb[rank]) // 64) >
                    torch.cuda.get_device_properties(dev).multi_processor_count)
                transport = "p2p"
                exchange = ("shd_xgroup/peer-to-peer (IPC-mapped receive blocks, xGMI stores, "
                            + ("a separate exchange launch per round)" if two_launch else
                               "each round's launch completes the previous round's exchange)"))
            except S.ShdError as ex:
                log(rank, f"peer-to-peer transport unavailable ({ex}); RCCL all-to-all instead")
                transport += "-after-p2p-map-or-self-check-failed"
        if grp is None:
            grp = XGroup.over(eng, comm)
        run = lambda t: grp.run_until(t)  # noqa: E731
    elif world > 1:
        cl = DistCluster(eng, pb, rank, world, dist, torch)
        cl.boot()
        run = lambda t: cl.run_until(t)  # noqa: E731
    else:
        eng.boot()
        run = lambda t: eng.run_until(t)  # noqa: E731

    # warmup
    tw = time.perf_counter()
    failed = None
    try:
        wst = run(args.warmup * step)
    except S.ShdError as ex:
        if not (use_group and getattr(grp, "p2p", False)):
            raise
        failed = ex
    if use_group and getattr(grp, "p2p", False):
        # a peer-to-peer exchange that never completes (its waits end after
        # 30 s with ENODEV) fails the warm-up on every rank; then all of them
        # rebuild the engine and run over the RCCL all-to-all instead
        bad = torch.tensor([1.0 if failed is not None else 0.0], device=tdev)
        if world > 1:
            dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        if bad.item() > 0:
            log(rank, f"peer-to-peer warm-up failed ({failed or 'on another rank'}); RCCL all-to-all instead")
            grp.close()
            eng.close()
            eng = Engine(model, pc, pb[rank], pb[rank + 1], device=dev)
            grp = XGroup.over(eng, comm)
            exchange = ("shd_xgroup/%s all-to-all (peer-to-peer warm-up failed)"
                        % ("host-memory" if args.comm == "host" else "RCCL"))
            transport = ("host-memory all-to-all" if args.comm == "host" else "rccl") + "-after-p2p-timeout"
            run = lambda t: grp.run_until(t)  # noqa: E731
            wst = run(args.warmup * step)
    torch.cuda.synchronize()
    log(rank, f"warmup {time.perf_counter() - tw:.1f}s")

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    mark = Roctx()
    barrier()
    mark.push("shd_timed_region")
    t0 = time.perf_counter()
    st = run(end_time)
    barrier()
    t1 = time.perf_counter()
    mark.pop()
    elapsed = t1 - t0
    if world > 1 and not use_group:
        pkt, evs, rounds, kms, ems = st.pkt_events, st.events, st.rounds, st.kernel_ms, st.kernel_ms
        hr = getattr(st, "host_rounds", 0)
    else:
        pkt, evs, rounds = st.n_pkt_events, st.n_events, st.n_rounds
        kms, ems = st.device_ms_round_kernel, st.device_ms_launches
        hr = st.n_host_rounds
    tot = torch.tensor([float(pkt), float(evs), float(kms), float(ems), float(hr)], dtype=torch.float64,
                       device=tdev)
    mx = torch.tensor([elapsed, upload_s], dtype=torch.float64, device=tdev)
    if world > 1:
        dist.all_reduce(tot)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    pkt_all, ev_all, kms_all, ems_all, hr_all = tot.tolist()
    elapsed, upload_max = mx.tolist()
    value = pkt_all / elapsed
    # rounds run behind a state copy (they could log many first touches) and
    # those rolled back on an ambiguous drop decision, warm-up + timed region
    protected = {k: int(getattr(wst, k, 0)) + int(getattr(st, k, 0))
                 for k in ("n_rounds_protected", "n_rounds_rerun")}

    # roofline of the round kernel, per round (per rank-round).  The round's
    # duration is the HIP-event time of the batches on the engine's stream over
    # the timed region divided by their rounds (a batch is one persistent
    # launch of up to 128 rounds, k_round_ps, or 64 graph-launched round
    # kernels; either way the gaps between launches are included); the
    # device-clock time of the rounds themselves is reported beside it.
    launches = rounds * max(world, 1)
    alg_bytes = BYTES_PER_PKT_EVENT * pkt_all + BYTES_PER_HOST_ROUND * hr_all
    avg_launch_ms = (ems_all if ems_all > 0 else kms_all) / max(launches, 1)
    achieved = (alg_bytes / max(launches, 1)) / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
    # the dominant kernel: ticketless device rounds on one engine (k_round_tl,
    # once no first touch is logged), the engine group's k_round_x across GPUs
    # (peer-to-peer rounds after a batch's first are k_round_px, which also completes the exchange)
    fused = use_group and exchange.startswith("shd_xgroup/peer-to-peer") and "completes the previous" in exchange
    n_ps = 0 if (world > 1 and not use_group) else int(getattr(st, "n_batches_persistent", 0))
    n_bat = 0 if (world > 1 and not use_group) else int(getattr(st, "n_batches", 0))
    n_sp = 0 if (world > 1 and not use_group) else int(getattr(st, "n_batches_sparse", 0))
    kname = (("k_round_spx" if n_bat and 2 * n_sp >= n_bat else "k_round_px") if fused else "k_round_xtl") \
        if use_group else \
        ("k_round" if world > 1 else (("k_round_sp" if 2 * n_sp >= n_ps else "k_round_ps")
                                       if n_ps and 2 * n_ps >= n_bat else "k_round_tl"))
    wkey = "%s-%dh" % (args.workload, H // max(world, 1))
    roofline = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": pmc_traffic(wkey, kname),
                "traffic_key": wkey + "/" + kname,
                "kernel": kname, "batches": {"all": n_bat, "persistent": n_ps, "sparse": n_sp},
                "avg_launch_us": round(avg_launch_ms * 1e3, 3),
                "avg_round_us": round(avg_launch_ms * 1e3, 3),
                "rounds_per_launch": round(rounds / max(n_bat, 1), 1) if n_bat else None,
                "avg_in_kernel_us": round(kms_all / max(launches, 1) * 1e3, 3),
                "launches": int(launches), "bytes_per_launch": round(alg_bytes / max(launches, 1), 1),
                "alg_bytes": "SURVEY.md 8(d): 80 B x packet events + 136 B x active host-rounds",
                "packet_events_per_launch": round(pkt_all / max(launches, 1), 1),
                "active_hosts_per_launch": round(hr_all / max(launches, 1), 1)}

    parity = None
    if world > 1 and not args.no_parity:
        parity = parity_leg(args, S, g, att, model, eng, pb, rank, world, dev, end_time, dist, torch, tdev,
                            int(getattr(wst, "n_pkt_events", getattr(wst, "pkt_events", 0))) + int(pkt))

    lossy = None
    if world == 1 and args.lossy_edge_loss_max > 0 and not use_group and args.workload == "c3":
        lossy = lossy_leg(args, S, W, Engine, PathCache, host_vertex, step, end_time, dev, torch)

    cpu_baseline = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_baseline = cpu_leg(args, S, W, g, model, step, value)
        if args.workload == "c3" and not args.no_reference_cpu:
            cpu_baseline["reference"] = reference_leg(args, S, W, g, host_vertex)

    if rank == 0:
        out = {
            "metric": "simulated packet events/sec",
            "value": round(value, 1),
            "unit": "packet events/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong" if args.workload == "c4" or (args.workload == "c5" and not args.hosts_per_gpu)
                       else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (bundled topology, Tor-scale relay/client PHOLD-UDP traffic, seed %d)"
                     if args.workload == "c4" else
                     "synthetic (random geometric topology + PHOLD-UDP traffic, seed %d)") % args.seed,
            "config": {"workload": ("C4 Tor-scale (%d relays + %d clients, bundled %d-vertex topology; edge loss "
                                    "0.005: the population decays, the rate depends on the window)"
                                    % (args.relays, args.clients, V)) if args.workload == "c4" else
                                   ("C5 model, %d hosts (%s, %d-vertex geometric topology), 1500-B messages, "
                                    "512 KiB/s downlinks (CoDel queues build), edge loss U[0,0.01]: the population "
                                    "decays, the rate depends on the window"
                                    % (H, "%d per GPU" % args.hosts_per_gpu if args.hosts_per_gpu else "100 per vertex",
                                       V)) if args.workload == "c5" else
                                   ("C3 PHOLD-UDP, stationary population (N x %d hosts, %d-vertex geometric topology)"
                                    % (args.hosts_per_gpu or 10000, V)),
                       "edge_loss": ("bundled (0.005)" if args.workload == "c4" else
                                     "U[0,0.01]" if args.workload == "c5" else "U[0,%g]" % args.edge_loss_max),
                       "hosts": H, "vertices": V, "edges": int(g.n_edges), "load": args.load,
                       "payload_bytes": 1500 if args.workload == "c5" else args.payload, "sim_seconds_per_step": args.step_ms / 1000.0,
                       "window_ns": int(eng.window),
                       "parallelism": ("REHEARSAL (not a measurement): hosts sharded over %d processes sharing "
                                       "GPU 0, host-memory communicator" % world) if rehearsal else
                                      "hosts sharded over %d GPU" % max(world, 1),
                       "exchange": (exchange if use_group else
                                    "torch.distributed" if world > 1 else "none (single engine)")},
            "transport": transport,
            "parity": parity,
            "all_events_per_s": round(ev_all / elapsed, 1),
            # the same events over the timed region plus the one-time host->device
            # upload of the boundary's host buffers (engine + path-cache creation)
            "pcie_inclusive": {"value": round(pkt_all / (elapsed + upload_max), 1),
                               "upload_ms": round(upload_max * 1e3, 3)},
            "rounds": int(rounds),
            "timed_batches": None if (world > 1 and not use_group) else int(getattr(st, "n_batches", 0)),
            "timed_batches_ticketless": None if (world > 1 and not use_group) else int(st.n_batches_ticketless),
            "timed_batches_persistent": None if (world > 1 and not use_group) else n_ps,
            "first_touch": protected,
            "apsp": {"rows": int(info.rows_computed), "vertices": V, "build_ms": round(min(builds), 3),
                     "sssp_kernel_ms": round(info.build_ms_sssp, 3), "iterations": int(info.sssp_iterations_max),
                     "max_hops": int(info.max_hops), "ties": int(info.n_ties),
                     "replicated_build_ms": round(min(builds), 3),
                     "sharded_build_ms": round(min(sharded), 3) if sharded else None,
                     "sharded_note": "rows [r*T/N, (r+1)*T/N) per rank + RCCL all-gather (wall time of the call)"
                                     if sharded else "N = 1: no sharding"},
            "roofline": roofline,
            "cpu_baseline": cpu_baseline,
            "lossy_c3": lossy,
        }
        sys.stdout.flush()
        os.dup2(_STDOUT_FD, 1)   # the JSON line is the only thing on stdout
        print(json.dumps(out), flush=True)
    if use_group:
        grp.close()
    eng.close()
    pc.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


def tcp_main(args):
    """The TCP path measured like the headline: a step is one
    whole shd_tcp_run of workloads.tcp_echo_model (hosts resident in HBM from
    the call's upload on; the value is device time of the rounds, HIP events on
    the run's stream).  At N > 1 (torch.distributed.run) the hosts are
    --hosts-per-gpu per GPU, sharded over the ranks by shd_tcp_run_group
    (weak scaling; RCCL, or --comm host: every rank on one GPU over the
    host-memory transport, a rehearsal); the value is every rank's events over
    the slowest rank's device time."""
    import torch
    import shdgpu as S
    import workloads as W
    import tcp as T
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    rehearsal = args.comm == "host" and world > 1
    dist = comm = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(0 if rehearsal else local_rank)
        dist.init_process_group("gloo" if rehearsal else "nccl")
        from sim import Comm, XGroup
        tdev = "cpu" if rehearsal else "cuda"
        uid = torch.zeros(S.SHD_XID_BYTES, dtype=torch.uint8, device=tdev)
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(XGroup.unique_id() if not rehearsal else os.urandom(S.SHD_XID_BYTES)),
                                       dtype=torch.uint8))
        dist.broadcast(uid, 0)
        dev = 0 if rehearsal else local_rank
        if rehearsal:
            comm = Comm.host("shdtcp_" + bytes(uid.cpu().numpy().tobytes())[:8].hex(), world, rank, dev)
        else:
            comm = Comm.rccl(bytes(uid.cpu().numpy().tobytes()), world, rank, dev)
    else:
        torch.cuda.set_device(0)
    H = (args.hosts_per_gpu or 65536) * max(world, 1)
    pool = args.tcp_pool
    V = min(args.vertices, 1000)
    def mk(n):
        if args.tcp_udp:
            return W.mixed_transport_model(n, V, seed=args.seed, end_s=args.tcp_end_s, nbytes=args.tcp_bytes,
                                           loss_max=args.edge_loss_max)
        return W.tcp_echo_model(n, V, seed=args.seed, end_s=args.tcp_end_s, nbytes=args.tcp_bytes,
                                loss_max=args.edge_loss_max) + (None,)
    g, m, ips, procs, peers, nb, udp = mk(H)
    # a caller running many models keeps the run's device buffers between
    # calls (shdtcp.h shd_tcp_keep_workspace); the first call allocates them
    S.lib().shd_tcp_keep_workspace(1)
    run1 = lambda: T.run(m, g, ips, procs, peers, nbytes=nb, trace=False, packets_per_host=pool,  # noqa: E731
                         comm=comm, udp=udp)
    for _ in range(args.warmup):
        run1()
    mark = Roctx()
    runs = []
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    mark.push("shd_timed_region")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runs.append(run1())
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    mark.pop()
    r = runs[-1]
    assert all(x["events"] == r["events"] and x["rounds"] == r["rounds"] for x in runs), "runs differ"
    dev_s = sum(x["device_ms"] for x in runs) / 1e3
    events = r["events"] * len(runs)
    deliv = r["deliveries"] * len(runs)
    if dist is not None:   # every rank's events over the slowest rank's time
        red = torch.tensor([float(events), float(deliv)], dtype=torch.float64, device="cpu" if rehearsal else "cuda")
        dist.all_reduce(red)
        mx = torch.tensor([dev_s, wall], dtype=torch.float64, device=red.device)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        events, deliv = int(red[0].item()), int(red[1].item())
        dev_s, wall = float(mx[0].item()), float(mx[1].item())
        comm.close()
        if rank != 0:
            dist.destroy_process_group()
            return
    # algorithmic bytes per executed event: its 32-B record pushed and popped
    # once (64 B); per delivery the mailbox record written and read once
    mail_b = 216   # sizeof(Mail) in csrc/tcp.hip (static_assert there; SACK lists travel apart)
    alg = 64 * r["events"] + 2 * mail_b * r["deliveries"]
    per_round_us = r["device_ms"] * 1e3 / max(r["rounds"], 1)
    achieved = alg / (r["device_ms"] / 1e3) / 1e9
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        # bounded sample: the same model at min(H, 4096) hosts (the same
        # per-pair work); the GPU runs that sample too, and the end states of
        # every host must agree
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests"))
        import oracle_ffi as O
        hs = min(H, 4096)
        gs, ms, ipss, pss, prs, _, us = mk(hs) if hs != H else (g, m, ips, procs, peers, nb, udp)
        rs = T.run(ms, gs, ipss, pss, prs, nbytes=nb, trace=False, packets_per_host=pool, udp=us) if hs != H else r
        tc = time.perf_counter()
        o = O.tcp_run(ms, gs, ipss, pss, prs, nbytes=nb, lines=False, udp=us)
        cs = time.perf_counter() - tc
        same = (o["events"] == rs["events"] and o["next_event_id"].tolist() == rs["next_event_id"].tolist()
                and o["next_packet_id"].tolist() == rs["next_packet_id"].tolist()
                and o["rng_probe"].tolist() == rs["rng_probe"].tolist())
        cpu = {"value": round(o["events"] / cs, 1), "unit": "TCP events/s", "cores": 1, "kind": "port",
               "sample": "oracle/o_tcp.c serial loop (pinned to the reference's tcp.c loop), [STATUS] lines off, "
                         "on the same model at %d hosts: %d events in %.2f s" % (hs, o["events"], cs),
               "gpu_sample_value": round(rs["events"] / (rs["device_ms"] / 1e3), 1),
               "same_end_state_as_gpu": bool(same)}
    out = {
        "metric": "simulated TCP events/sec", "value": round(events / dev_s, 1), "unit": "events/s",
        "n_gpus": max(world, 1), "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dev_s * 1e3 / len(runs), 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (random geometric topology + TCP echo pairs, seed %d)"
        % args.seed,
        "config": {"workload": "TCP echo (src/test/tcp/test_tcp.c, nonblocking-epoll), %d hosts / %d pairs, "
                               "%d-vertex geometric topology, %d B each way, %d s simulated%s"
                               % (H, H // 2, V, nb, args.tcp_end_s,
                                  "; and a datagram process per host (workloads.mixed_transport_model)"
                                  if args.tcp_udp else ""),
                   "hosts": H, "vertices": V, "packets_per_host": pool,
                   "parallelism": "one lane per host, %s" % (
                       "1 GPU" if world <= 1 else "hosts sharded over %d ranks (shd_tcp_run_group, %s)"
                       % (world, "host-memory transport, one GPU: rehearsal" if rehearsal else "RCCL"))},
        "packet_deliveries_per_s": round(deliv / dev_s, 1), "wall_s": round(wall, 3),
        # the same events over the whole calls' wall time (the model's upload,
        # the per-host allocations and setup, the rounds, the copies back): the
        # rate a caller of shd_tcp_run sees end to end; `value` is device time
        "wall_inclusive": {"value": round(events / wall, 1), "unit": "events/s",
                           "device_share": round(dev_s / wall, 3),
                           "host_ms_last_run": {k: round(v, 1) for k, v in r.get("host_ms", {}).items()}},
        "first_touch": r.get("first_touch"), "first_touch_reruns": r.get("first_touch_reruns"),
        "rounds": r["rounds"], "events_per_run": r["events"], "deliveries_per_run": r["deliveries"],
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(achieved / 8000.0, 6), "traffic": None, "kernel": "k_tcp_round",
                     "avg_round_us": round(per_round_us, 3),
                     "alg_bytes": "64 B x events + 2 x %d B x deliveries" % mail_b},
        "cpu_baseline": cpu,
    }
    os.dup2(_STDOUT_FD, 1)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def lossy_leg(args, S, W, Engine, PathCache, host_vertex, step, end_time, dev, torch):
    """The same C3 workload with edge loss U[0, --lossy-edge-loss-max], timed
    step by step: PHOLD never regenerates a lost message, so the population
    and the rate decay with simulated time (reported per step, never `value`)."""
    g = W.geometric_graph(args.vertices, seed=args.seed, loss_max=args.lossy_edge_loss_max)
    model = W.phold_model(host_vertex, end_time=end_time, seed=args.seed, load=args.load,
                          payload=args.payload)
    pc = PathCache(g, W.attached_vertices(host_vertex), device=dev)
    eng = Engine(model, pc, device=dev)
    eng.boot()
    eng.run_until(args.warmup * step)
    per_step, tot_pkt, tot_s = [], 0, 0.0
    for k in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = eng.run_until((args.warmup + k + 1) * step)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        per_step.append(int(st.n_pkt_events))
        tot_pkt += st.n_pkt_events
        tot_s += dt
    eng.close()
    pc.close()
    return {"edge_loss": "U[0,%g]" % args.lossy_edge_loss_max, "value": round(tot_pkt / tot_s, 1),
            "unit": "packet events/s", "packet_events_per_step": per_step,
            "note": "lost messages are never regenerated: the rate depends on the simulated window"}


def pmc_traffic(workload, kernel):
    """HBM bytes per round of the round kernel from the committed rocprofv3
    PMC passes of THIS workload and kernel (profiles/r06, r05 or r04/pmc_traffic.json,
    scripts/pmc_traffic.py: FETCH_SIZE x the calibrated read correction +
    WRITE_SIZE, over the timed region's dispatches), used only when they were
    taken of the engine source being run; else None (no inherited numbers)."""
    try:
        import shdgpu as S
        sha = S.engine_source_sha1()
    except (OSError, ValueError):
        return None
    prof = {}
    for rnd in ("r06", "r05", "r04"):   # the newest round's passes of this source
        try:
            prof = json.load(open(os.path.join(REPO, "profiles", rnd, "pmc_traffic.json")))
        except (OSError, ValueError):
            continue
        if prof.get("engine_source_sha1") == sha:
            break
    if prof.get("engine_source_sha1") != sha:
        return None
    ent = prof.get("entries", {}).get(workload + "/" + kernel)
    return None if ent is None else ent.get("hbm_bytes_per_round")


def cpu_threads():
    """Host cores to use: the box's CPU share (OMP_NUM_THREADS is set to it on
    the GPU box), else the affinity mask."""
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    return max(1, n or min(len(os.sched_getaffinity(0)), 16))


def parity_leg(args, S, g, att, model, eng, pb, rank, world, dev, end_time, dist, torch, tdev, pkt_local):
    """N > 1: the run checked against the same model on ONE engine.  After the
    timed region every rank hashes its hosts' end states (shd_eng_digest:
    event-ID counter, RNG, queues, CoDel state and counters of each host,
    SHA-256 over the rank's slice) and its packet-event count; rank 0 runs the
    whole model, all H hosts, on one engine of its own GPU over the same
    [0, end) on a path cache built afresh, and compares slice by slice.  The
    line says whether the transport that ran (`transport`) left every rank's
    hosts exactly where the single engine leaves them.  Untimed."""
    import hashlib
    from sim import Engine, PathCache
    t0 = time.perf_counter()
    mine = np.frombuffer(hashlib.sha256(eng.digest().tobytes()).digest(), dtype=np.uint8).astype(np.int64)
    mine = np.concatenate([mine, [pkt_local]])
    t = torch.tensor(mine, dtype=torch.int64, device=tdev)
    got = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(got, t)
    got = [x.cpu().numpy() for x in got]
    res = torch.zeros(2 + world, dtype=torch.int64, device=tdev)
    if rank == 0:
        pc1 = PathCache(g, att, device=dev)
        ref = Engine(model, pc1, 0, model.n_hosts, device=dev)
        ref.boot()
        rst = ref.run_until(end_time)
        dg = ref.digest()
        ref.close()
        pc1.close()
        ok = []
        for r in range(world):
            h = hashlib.sha256(dg[pb[r]:pb[r + 1]].tobytes()).digest()
            ok.append(int(bytes(got[r][:32].astype(np.uint8).tobytes()) == h))
        pkt_group = int(sum(int(x[32]) for x in got))
        res[0] = int(all(ok) and pkt_group == int(rst.n_pkt_events))
        res[1] = int(rst.n_pkt_events)
        res[2:] = torch.tensor(ok, dtype=torch.int64)
    dist.broadcast(res, 0)
    r = res.cpu().numpy()
    return {"ok": bool(r[0]), "ranks_ok": [bool(x) for x in r[2:]],
            "pkt_events_single_engine": int(r[1]),
            "pkt_events_group": int(sum(int(x[32]) for x in got)),
            "reference": "one engine over all %d hosts on rank 0's GPU, same model, [0, %.3f s), fresh path cache; "
                         "per-rank SHA-256 of the hosts' end-state digests (shd_eng_digest)" %
                         (model.n_hosts, end_time / 1e9),
            "ms": round((time.perf_counter() - t0) * 1e3, 1)}


def cpu_leg(args, S, W, g, model, step, value):
    """The reference's scheduler semantics on the host cores, on the SAME
    workload and simulated window as `value` (oracle.h o_baseline): one
    warm-up to t = warmup steps (Dijkstra rows on all cores, then the serial
    loop: boot, application start, lazy path cache), then the timed window
    [warmup, warmup + steps) run twice from that state --
      * serially on 1 core (--workers 0: one global queue, slave.c:415-428);
      * in parallel rounds on `cores` threads, host-steal style
        (scheduler_policy_host_steal.c:227-431; per-host queues, hosts pulled
        in chunks, windows W <= every path latency so nothing is clamped and
        the result is the serial one; first touches resolved at each round's
        end in serial order) --
    and both end states compared bit for bit.  --cpu-sample-steps bounds the
    window (default: all timed steps)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    try:
        import oracle_ffi as O
        O.lib()
    except Exception as ex:   # the checker is absent: report it, never substitute
        return {"value": None, "unit": "packet events/s", "cores": 1, "kind": "port",
                "sample": f"oracle unavailable: {ex}"}
    n_steps = args.steps if args.cpu_sample_steps <= 0 else min(args.steps, args.cpu_sample_steps)
    t_mark = args.warmup * step
    t_end = t_mark + n_steps * step
    m = model
    host_vertex = model.host_vertex
    thr = cpu_threads()
    b = O.baseline(m, g, t_mark, t_end, thr)
    ser = b["serial_pkt_events"] / (b["serial_ms"] * 1e-3) if b["serial_ms"] > 0 else None
    par = b["parallel_pkt_events"] / (b["parallel_ms"] * 1e-3) if b["parallel_ms"] > 0 else None
    win = "simulated [%g s, %g s)" % (t_mark / 1e9, t_end / 1e9)
    return {"value": round(ser, 1) if ser else None, "unit": "packet events/s", "cores": 1, "kind": "port",
            "sample": "oracle serial loop (reference --workers 0 semantics) on the bench's own workload "
                      "(%d hosts, %d-vertex graph, load %d) over %s: %d packet events in %.2f s"
                      % (len(host_vertex), g.n_vertices, args.load, win, b["serial_pkt_events"],
                         b["serial_ms"] * 1e-3),
            "parallel": {"value": round(par, 1) if par else None, "cores": int(b["threads"]),
                         "kind": "port",
                         "sample": "same state, same window, parallel rounds (host-steal equivalent, W = %d ns, "
                                   "%d rounds, %d first-touch sends resolved at round ends): %d packet events "
                                   "in %.2f s" % (b["window_ns"], b["parallel_rounds"], b["parallel_first_touch"],
                                                   b["parallel_pkt_events"], b["parallel_ms"] * 1e-3),
                         "same_end_state_as_serial": bool(b["same_end_state"]),
                         "ambiguous_first_touches": int(b["ambiguous"])},
            "gpu_over_cpu_1core": round(value / ser, 1) if ser else None,
            "gpu_over_cpu_parallel": round(value / par, 1) if par else None,
            "warmup_s": round((b["rows_ms"] + b["warmup_ms"]) * 1e-3, 2),
            "apsp_rows_all_cores_s": round(b["rows_ms"] * 1e-3, 2)}


def reference_leg(args, S, W, g, host_vertex):
    """The reference's OWN serial scheduler loop timed on this box's host cores
    (BASELINE north_star: "the reference Shadow CPU scheduler timed on the box's
    own host cores"): oracle/_ref/libshdref_loop.so is Shadow's worker.c,
    scheduler.c (SP_SERIAL_GLOBAL, --workers 0, slave.c:415-428), host.c,
    network_interface.c, router*.c, tracker.c, packet.c and the descriptors
    compiled unmodified from the reference tree in the build container (it
    travels prebuilt; test doubles only for what the image cannot compile,
    oracle/ref_harness/ref_loop.c).  A bounded sample of the headline workload:
    the same C3 model, its loop timed over the simulated window
    --reference-window-ms (wall clock between the first sends at or after each
    end), the path cache's rows computed on all cores beforehand (the lazy
    cache's double serves them; Dijkstra is the APSP metric, timed apart).  The
    port (oracle/o_engine.c) is timed on the same window beside it; the packet
    events of the window are the port's count (the two loops' end states are
    equal, tests/test_ref_loop_cpu.py and ref_loop.json)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    t0_ms, t1_ms = args.reference_window_ms
    t0, t1 = t0_ms * S.SHD_MS, t1_ms * S.SHD_MS
    res = {"value": None, "unit": "packet events/s", "cores": 1, "kind": "reference"}
    try:
        import oracle_ffi as O
        import ref_loop_ffi as R
        if not R.available():
            res["sample"] = "oracle/_ref/libshdref_loop.so not built"
            return res
        m = W.phold_model(host_vertex, end_time=t1 + S.SHD_MS, seed=args.seed, load=args.load, payload=args.payload)
        thr = cpu_threads()
        tw = time.perf_counter()
        r = R.run(m, g, quiet=True, marks=(t0, t1), row_threads=thr)
        wall = time.perf_counter() - tw
        ref_s = r["mark_wall_s"][1] - r["mark_wall_s"][0]
        b = O.baseline(m, g, t0, t1, thr)
    except Exception as ex:   # noqa: BLE001 -- reported, never substituted
        res["sample"] = f"reference loop unavailable: {ex}"
        return res
    pkt = int(b["serial_pkt_events"])
    port = pkt / (b["serial_ms"] * 1e-3) if b["serial_ms"] > 0 else None
    res.update({
        "value": round(pkt / ref_s, 1) if ref_s > 0 else None,
        "sample": "the reference's own serial loop (oracle/_ref/libshdref_loop.so: worker.c, scheduler.c "
                  "SP_SERIAL_GLOBAL, host.c, network_interface.c, router*.c, tracker.c, packet.c compiled "
                  "unmodified; debug records filtered as at the default log level) on the bench's C3 model "
                  "(%d hosts, %d-vertex graph, load %d), timed over simulated [%g s, %g s): %d packet events "
                  "in %.2f s; path-cache rows precomputed on %d cores (%.1f s, not in the window)"
                  % (len(host_vertex), g.n_vertices, args.load, t0 / 1e9, t1 / 1e9, pkt, ref_s, thr, r["rows_s"]),
        "port_same_window": {"value": round(port, 1) if port else None, "cores": 1, "kind": "port"},
        "reference_over_port": round((pkt / ref_s) / port, 4) if port and ref_s > 0 else None,
        "run_s": round(wall, 1)})
    return res


if __name__ == "__main__":
    main()
