"""Pin the oracle against the reference: glibc rand_r, the reference's own
random.c / router_queue_codel.c / priority_queue.c (compiled into oracle/_ref
from /root/reference; golden fixtures generated from them are committed), and
the seed chain of master.c / slave.c."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import oracle_ffi as O
import shdgpu as S

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
REF_SO = os.path.join(os.path.dirname(HERE), "oracle", "_ref", "libshdref.so")


@pytest.fixture(scope="module")
def kats():
    return json.load(open(os.path.join(GOLD, "rng_kats.json")))


def test_rand_r_kats(kats):
    for seed, vals in kats["rand_r"].items():
        s = int(seed)
        got = []
        for _ in range(8):
            v, s = O.rand_r(s)
            got.append(v)
        assert got + [s] == vals
    # survey section A.5 values
    assert kats["rand_r"]["1"][:5] == [476707713, 1186278907, 505671508, 2137716191, 936145377]


def test_next_double_and_uint_kats(kats):
    l = O.lib()
    for seed, vals in kats["next_double"].items():
        s = C.c_uint32(int(seed))
        assert [l.o_next_double(C.byref(s)).hex() for _ in range(8)] == vals
    for seed, vals in kats["next_uint"].items():
        s = C.c_uint32(int(seed))
        assert [l.o_next_uint(C.byref(s)) for _ in range(8)] == vals


def test_seed_chain(kats):
    ch = kats["seed_chain_1"]
    assert (ch["slave"], ch["scheduler"]) == (953415426, 2714057858)
    seeds = (C.c_uint32 * 64)()
    O.lib().o_seed_chain(1, 64, seeds)
    assert list(seeds) == ch["hosts"]


def replay_oracle_codel(ops):
    l = O.lib()
    q = O.OCodel()
    l.o_codel_init(C.byref(q), 16)
    drops = (O.OCodelEntry * 4096)()
    outs = []
    for op in ops:
        if op[0] == "enq":
            l.o_codel_enqueue(C.byref(q), op[1], op[3] + 42, op[2], 0)
            outs.append(["enq"])
        else:
            e = O.OCodelEntry()
            nd = C.c_uint32()
            ok = l.o_codel_dequeue(C.byref(q), op[1], C.byref(e), drops, 4096, C.byref(nd))
            outs.append(["deq", int(ok), int(e.id) if ok else -1, [int(drops[i].id) for i in range(nd.value)]])
    l.o_codel_free(C.byref(q))
    return outs


def test_codel_matches_reference_timelines():
    scripts = json.load(open(os.path.join(GOLD, "codel_trace.json")))
    total_drops = 0
    for s in scripts:
        assert replay_oracle_codel(s["ops"]) == s["outs"]
        total_drops += sum(len(o[3]) for o in s["outs"] if o[0] == "deq")
    assert total_drops > 1000   # drop mode and the control law are exercised


def test_codel_control_law_quirk():
    # controlLaw divides the ABSOLUTE timestamp + interval by sqrt(count)
    # (router_queue_codel.c:198-205)
    l = O.lib()
    for count, ts in [(1, 0), (2, 5_000_000_000), (7, 123_456_789), (100, 3_000_000_000_000)]:
        assert l.o_codel_control_law(count, ts) == int(round((ts + 100_000_000) / np.sqrt(count)))


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (no /root/reference)")
def test_priority_queue_pops_in_event_compare_order():
    l = C.CDLL(REF_SO)
    l.ref_pq_order.argtypes = [C.c_void_p] * 4 + [C.c_uint32, C.c_void_p]
    rng = np.random.default_rng(3)
    n = 5000
    time = rng.integers(0, 50, n).astype(np.uint64)
    dst = rng.integers(0, 5, n).astype(np.uint32)
    src = rng.integers(0, 5, n).astype(np.uint32)
    seq = rng.permutation(n).astype(np.uint64)
    out = np.empty(n, np.uint32)
    l.ref_pq_order(time.ctypes.data, dst.ctypes.data, src.ctypes.data, seq.ctypes.data, n, out.ctypes.data)
    keys = np.zeros(n, dtype=S.EVENT_DTYPE)
    keys["time"], keys["dst"], keys["src"], keys["seq"] = time, dst, src, seq
    order = np.lexsort((seq, src, dst, time))
    assert np.array_equal(out, order)
    # the oracle's comparator agrees pairwise
    ev = (S.Event * 2)()
    for i in range(200):
        a, b = int(out[i]), int(out[i + 1])
        ev[0] = S.Event(int(time[a]), int(seq[a]), int(src[a]), int(dst[a]), 0, 0)
        ev[1] = S.Event(int(time[b]), int(seq[b]), int(src[b]), int(dst[b]), 0, 0)
        assert O.lib().o_event_compare(C.byref(ev[0]), C.byref(ev[1])) < 0


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (no /root/reference)")
def test_codel_fixture_reproduces_from_reference_build():
    import importlib.util
    spec = importlib.util.spec_from_file_location("mg", os.path.join(GOLD, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    got = mg.codel_trace(mg.ref_lib())
    assert got == json.load(open(os.path.join(GOLD, "codel_trace.json")))
