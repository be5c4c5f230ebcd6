"""Packet ingress / egress at the boundary: the
GPU engine holds some of a model's hosts and exchanges datagrams with hosts
simulated on the CPU side -- here the oracle's hosts, split the same way
(oracle.h o_state_new_part; tests/test_cosim_cpu.py pins that split against
the whole serial run).

* shd_eng_push_events accepts SHD_EV_PACKET deliveries from hosts outside the
  engine (worker_sendPacket's scheduler_push for another worker's host,
  worker.c:541-571) and shd_eng_take_remote returns the engine's deliveries to
  them, one window of W at a time;
* the SP_GPU_ROUNDS policy with a bridge (sched_policy_shd.c
  schedulerpolicygpurounds_new_bridged) does the same inside Shadow's round
  loop: CPU-side sends pushed through the policy reach the engine, the
  engine's sends come back as Shadow events popped in their round.
The union of both sides' traces and end states must equal the whole model's
serial oracle run bit for bit.

One lazy path cache across the sides (topology.c:1969-2051 is one global
cache): on a graph that is not complete, a pair's value depends on which
endpoint's row ran first, so the two sides' first touches of a window are put
in one serial order.  The engine runs its window first (its first touches are
pending, their deliveries wait); the CPU side gets them (o_state_defer_touches)
and applies each to its cache just before its first later query, in event
order; its own first touches come back (o_state_take_touches), and the
engine's resolution ranks both (shd_eng_resolve over the union).  On the
directed graph below a pair's orientations are different paths with different
latencies: without the protocol the co-simulation diverges from the serial run
(checked).  The grid (workloads.grid_graph: every edge 1 ms) has equal-cost
paths between almost every pair, so each endpoint's Dijkstra takes its own
path, with its own reliability: there the path cache's tie rows
(k_sssp_tie_parents, igraph's heap order) and the one-cache protocol are both
on the line.  (On an undirected tie-free graph the two rows of a pair differ in
the last bits of their folds only, which a PHOLD delivery almost never sees.)
"""
import ctypes as C

import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S
import workloads as W
from sim import Engine, PathCache, sort_trace

pytestmark = pytest.mark.gpu
U64_MAX = (1 << 64) - 1
EINVAL = -22


def directed_graph(V=36, seed=5, loss_max=0.01):
    """a geometric graph with every edge both ways, the reverse with its own
    latency and loss: a pair's two orientations are different paths, and the
    directed lookup serves (a, b) from whichever endpoint's row ran first (the
    reverse path when it was b's, topology.c:2034-2037)"""
    g0 = W.geometric_graph(V, seed=seed, loss_max=loss_max)
    src, dst, lat, loss = g0.src.astype(np.int64), g0.dst.astype(np.int64), g0.latency, g0.loss
    rng = np.random.default_rng(seed + 1000)
    nsl = src != dst
    k = int(nsl.sum())
    return S.GraphArrays(V, np.concatenate([src, dst[nsl]]), np.concatenate([dst, src[nsl]]),
                         np.concatenate([lat, lat[nsl] * (1.0 + rng.random(k))]),
                         np.concatenate([loss, rng.random(k) * loss_max]), directed=True)


def model(n_hosts=300, seed=3, graph="bundled", **kw):
    g = {"bundled": W.bundled_graph, "directed": directed_graph, "grid": W.grid_graph}[graph]()
    hv = np.sort(np.random.default_rng(seed).integers(0, g.n_vertices, n_hosts)).astype(np.int32)
    kw.setdefault("load", 8)
    m = W.phold_model(hv, end_time=3 * S.SHD_SEC, trace=True, **kw)
    return g, m


def union_equal(m, g, cut, gtr, gdg, ctr, cdg):
    otr, odg, _ = O.engine_run(m, g)
    tr = sort_trace(np.concatenate([ctr, gtr]))
    return (len(tr) == len(otr) and np.array_equal(tr, sort_trace(otr)) and np.array_equal(cdg[:cut], odg[:cut])
            and np.array_equal(gdg, odg[cut:]))


def cosim(m, g, cut, one_cache=True):
    """the engine over hosts [cut, H), the oracle over [0, cut), window by
    window; one_cache: the first touches of both sides in one serial order"""
    H = m.n_hosts
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc, cut, H)
    eng.boot()
    cpu = O.OState(m, g, hosts=(0, cut))
    Wn = eng.window
    end = m.params["end_time"]
    n = dict(ingress=0, egress=0, rounds=0, engine_touches=0, cpu_touches=0, retries=0)
    while True:
        ws = min(cpu.next_time(), eng.next_time())
        if ws >= end:
            break
        we = ws + Wn
        if one_cache:
            r = eng.round_begin(ws, we)                # the engine's window first: its first touches pend
            pe = eng.pending_records()
            cpu.defer_touches(pe)                      # applied at their place in the CPU side's order
            cpu.run_serial(we)
            pcpu = cpu.take_touches()
            both = np.concatenate([pe, pcpu])
            if r.error & S.ERR_AMBIGUOUS:              # a drop decision the ranking decides: run it again
                assert eng.round_retry(both).error == 0
                n["retries"] += 1
            else:
                eng.resolve(both)                      # one ranking of both sides' first touches
            eng.end_round()
            n["engine_touches"] += len(pe)
            n["cpu_touches"] += len(pcpu)
        else:
            cpu.run_serial(we)
            eng.run_round(ws, we)
        out = eng.take_remote()                    # engine -> CPU side (egress)
        inc = cpu.take_egress()                    # CPU side -> engine (ingress)
        assert np.all(out["time"] >= we) and np.all(out["dst"] < cut) and np.all(out["src"] >= cut)
        assert np.all(out["kind"] == S.EV_PACKET)
        if len(inc):
            eng.push_events(inc)
        cpu.inject(out)
        n["ingress"] += len(inc)
        n["egress"] += len(out)
        n["rounds"] += 1
    res = (eng.trace(), eng.digest(), cpu.trace(), cpu.digest())
    cpu.close()
    eng.close()
    pc.close()
    return res, n


@pytest.mark.parametrize("graph,cut,kw", [("bundled", 120, {}), ("bundled", 1, {}), ("bundled", 299, {}),
                                          ("bundled", 70, dict(load=24, payload=1000, bw_down=200, bw_up=100000,
                                                               codelq_cap=256, queue_flags=S.SHD_QF_TRACE_STATUS)),
                                          ("directed", 120, {}), ("directed", 1, {}), ("directed", 299, {}),
                                          ("grid", 120, {}), ("grid", 1, {}), ("grid", 299, {})])
def test_engine_exchanges_packets_with_cpu_side_hosts(graph, cut, kw):
    g, m = model(graph=graph, **kw)
    (gtr, gdg, ctr, cdg), n = cosim(m, g, cut)
    assert n["ingress"] > 50 and n["egress"] > 50 and n["rounds"] > 100
    if graph != "bundled":   # both sides touch first, on a graph where it matters
        assert n["engine_touches"] > 0 and n["cpu_touches"] > 0
    assert union_equal(m, g, cut, gtr, gdg, ctr, cdg)
    if kw:
        assert np.count_nonzero(gtr["kind"] == S.TR_CODEL_DROP) > 0


def test_orientations_matter_without_one_cache():
    """the directed model is one where the first-touch order decides values:
    the two sides' first touches left unordered, the union is not the serial
    run (or an engine round's drop decision is left ambiguous)"""
    g, m = model(graph="directed")
    try:
        (gtr, gdg, ctr, cdg), _ = cosim(m, g, 120, one_cache=False)
    except S.ShdError as e:
        assert "EAMBIG" in str(e)
        return
    assert not union_equal(m, g, 120, gtr, gdg, ctr, cdg)


def test_push_events_validates_packet_ingress():
    g, m = model(n_hosts=40)
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc, 20, 40)
    eng.boot()
    ev = np.zeros(1, dtype=S.EVENT_DTYPE)
    ev["kind"], ev["time"], ev["seq"], ev["pkt"] = S.EV_PACKET, S.SHD_SEC, 7, 3

    def rc(src, dst, time=S.SHD_SEC, kind=S.EV_PACKET):
        x = ev.copy()
        x["src"], x["dst"], x["time"], x["kind"] = src, dst, time, kind
        return S.lib().shd_eng_push_events(eng.ptr, x.ctypes.data, 1)

    assert rc(25, 30) == EINVAL   # from a host of this engine
    assert rc(3, 5) == EINVAL   # for a host outside it
    assert rc(3, 45) == EINVAL   # no such host
    assert rc(40, 30) == EINVAL   # no such sender
    assert rc(3, 30, kind=S.EV_NOTIFY) == EINVAL
    assert rc(3, 30) == 0        # a delivery from a CPU-side host
    assert eng.next_time() <= S.SHD_SEC
    assert rc(3, 30, time=m.params["end_time"]) == 0   # dropped at the end (scheduler.c:346-349)
    # a whole-model run_until is refused on a partial engine (its sends would have nowhere to go)
    st = S.RunStats()
    assert S.lib().shd_eng_run_until(eng.ptr, 2 * S.SHD_SEC, C.byref(st)) == EINVAL
    eng.close()


# ---- through the scheduler policy (sched_policy_shd.c) ----
ING = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(S.Event))
EGR = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.POINTER(S.Event))
TIN = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_uint64)
TOUT = C.CFUNCTYPE(C.c_uint64, C.c_void_p, C.POINTER(C.c_void_p))


class Bridge(C.Structure):
    _fields_ = [("ingress", ING), ("egress", EGR), ("user", C.c_void_p), ("touches_in", TIN),
                ("touches_out", TOUT)]


@pytest.mark.parametrize("graph,one_cache", [("bundled", False), ("directed", True), ("grid", True)])
def test_bridged_policy_exchanges_packets_in_shadows_round_loop(graph, one_cache):
    import test_boundary_gpu as B
    h, t = B.libs()
    for f, res, args in (("harness_packet_event_new", C.c_void_p,
                          [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32]),
                         ("harness_event_src", C.c_uint32, [C.c_void_p]),
                         ("harness_event_dst", C.c_uint32, [C.c_void_p]),
                         ("harness_event_pkt", C.c_uint32, [C.c_void_p]),
                         ("event_unref", None, [C.c_void_p])):
        getattr(h, f).restype = res
        getattr(h, f).argtypes = args
    t.schedulerpolicygpurounds_new_bridged.restype = C.c_void_p
    t.schedulerpolicygpurounds_new_bridged.argtypes = [C.c_void_p, C.POINTER(Bridge)]

    g, m = model(seed=9, graph=graph)
    H, cut = m.n_hosts, 140
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc, cut, H)
    eng.boot()
    cpu = O.OState(m, g, hosts=(0, cut))
    counts = dict(ingress=0, egress=0, kept=0)

    def ingress(user, ev, src, dst, out):
        d = h.harness_event_dst(ev)
        if d < cut:
            counts["kept"] += 1
            return 0
        out[0] = S.Event(h.event_getTime(ev), h.harness_event_seq(ev), h.harness_event_src(ev), d,
                         h.harness_event_pkt(ev), S.EV_PACKET)
        counts["ingress"] += 1
        return 1

    def egress(user, x):
        e = x.contents
        counts["egress"] += 1
        return h.harness_packet_event_new(e.time, e.src, e.dst, e.seq, e.pkt)

    keep = {}

    def touches_in(user, recs, n):   # the engine's first touches of the round -> the CPU side's cache
        counts["engine_touches"] += n
        cpu.defer_touches(np.ctypeslib.as_array(C.cast(recs, C.POINTER(C.c_uint8)), shape=(n * 56,))
                          .view(S.PENDING_DTYPE).copy() if n else np.zeros(0, S.PENDING_DTYPE))

    def touches_out(user, out):      # the CPU side's own, after the round's CPU events
        keep["t"] = cpu.take_touches()
        counts["cpu_touches"] += len(keep["t"])
        out[0] = keep["t"].ctypes.data if len(keep["t"]) else None
        return len(keep["t"])

    counts.update(engine_touches=0, cpu_touches=0)
    br = Bridge(ING(ingress), EGR(egress), None, TIN(touches_in) if one_cache else TIN(),
                TOUT(touches_out) if one_cache else TOUT())
    pp = t.schedulerpolicygpurounds_new_bridged(eng.ptr.value, C.byref(br))
    assert pp
    pol = C.cast(pp, C.POINTER(B.Policy)).contents
    Wn = eng.window
    end = m.params["end_time"]
    nxt = min(pol.getNextTime(pp), cpu.next_time())
    rounds = 0
    while nxt < end:
        barrier = nxt + Wn                          # slave.c:437-462, runahead = W
        due = []
        while True:                                 # the round's pops: deliveries from offloaded hosts
            ev = pol.pop(pp, barrier)
            if not ev:
                break
            assert nxt <= h.event_getTime(ev) < barrier
            due.append((h.event_getTime(ev), h.harness_event_seq(ev), h.harness_event_src(ev),
                        h.harness_event_dst(ev), h.harness_event_pkt(ev), S.EV_PACKET))
            h.event_unref(ev)
        cpu.inject(np.array(due, dtype=S.EVENT_DTYPE))
        cpu.run_serial(barrier)                     # the CPU-side hosts' events of the round
        for e in cpu.take_egress():                 # their sends to offloaded hosts: scheduler_push
            pol.push(pp, h.harness_packet_event_new(int(e["time"]), int(e["src"]), int(e["dst"]),
                                                    int(e["seq"]), int(e["pkt"])), None, None, barrier)
        assert t.schedulerpolicygpurounds_error(pp) == 0
        rounds += 1
        nxt = min(pol.getNextTime(pp), cpu.next_time())
    assert counts["ingress"] > 50 and counts["egress"] > 50 and counts["kept"] == 0
    assert rounds > 100
    if one_cache:
        assert counts["engine_touches"] > 0 and counts["cpu_touches"] > 0
    assert union_equal(m, g, cut, eng.trace(), eng.digest(), cpu.trace(), cpu.digest())
    pol.free(pp)
    cpu.close()
    eng.close()
