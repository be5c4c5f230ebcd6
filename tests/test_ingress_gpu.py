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
serial oracle run bit for bit.  The bundled topology is complete, so a path's
value does not depend on which side touched it first (on other graphs the two
sides' first touches within a window are not interleaved: DESIGN.md).
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


def model(n_hosts=300, seed=3, **kw):
    g = W.bundled_graph()
    hv = np.sort(np.random.default_rng(seed).integers(0, g.n_vertices, n_hosts)).astype(np.int32)
    kw.setdefault("load", 8)
    m = W.phold_model(hv, end_time=3 * S.SHD_SEC, trace=True, **kw)
    return g, m


def check_union(m, g, cut, gtr, gdg, ctr, cdg):
    otr, odg, _ = O.engine_run(m, g)
    tr = sort_trace(np.concatenate([ctr, gtr]))
    assert len(tr) == len(otr)
    assert np.array_equal(tr, sort_trace(otr))
    assert np.array_equal(cdg[:cut], odg[:cut])
    assert np.array_equal(gdg, odg[cut:])


@pytest.mark.parametrize("cut,kw", [(120, {}), (1, {}), (299, {}),
                                    (70, dict(load=24, payload=1000, bw_down=200, bw_up=100000,
                                              codelq_cap=256, queue_flags=S.SHD_QF_TRACE_STATUS))])
def test_engine_exchanges_packets_with_cpu_side_hosts(cut, kw):
    g, m = model(**kw)
    H = m.n_hosts
    pc = PathCache(g, W.attached_vertices(m.host_vertex))
    eng = Engine(m, pc, cut, H)
    eng.boot()
    cpu = O.OState(m, g, hosts=(0, cut))
    Wn = eng.window
    end = m.params["end_time"]
    n_in = n_out = rounds = 0
    while True:
        ws = min(cpu.next_time(), eng.next_time())
        if ws >= end:
            break
        we = ws + Wn
        cpu.run_serial(we)
        eng.run_round(ws, we)
        out = eng.take_remote()                    # engine -> CPU side (egress)
        inc = cpu.take_egress()                    # CPU side -> engine (ingress)
        assert np.all(out["time"] >= we) and np.all(out["dst"] < cut) and np.all(out["src"] >= cut)
        assert np.all(out["kind"] == S.EV_PACKET)
        if len(inc):
            eng.push_events(inc)
        cpu.inject(out)
        n_in += len(inc)
        n_out += len(out)
        rounds += 1
    assert n_in > 50 and n_out > 50 and rounds > 100
    check_union(m, g, cut, eng.trace(), eng.digest(), cpu.trace(), cpu.digest())
    if kw:
        assert np.count_nonzero(eng.trace()["kind"] == S.TR_CODEL_DROP) > 0
    cpu.close()
    eng.close()


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


class Bridge(C.Structure):
    _fields_ = [("ingress", ING), ("egress", EGR), ("user", C.c_void_p)]


def test_bridged_policy_exchanges_packets_in_shadows_round_loop():
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

    g, m = model(seed=9)
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

    br = Bridge(ING(ingress), EGR(egress), None)
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
    check_union(m, g, cut, eng.trace(), eng.digest(), cpu.trace(), cpu.digest())
    pol.free(pp)
    cpu.close()
    eng.close()
