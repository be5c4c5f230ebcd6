"""The N>1 round protocol of driver.DistCluster over torch.distributed "gloo",
world_size 2, on the CPU (DESIGN.md "Multi-GPU").

The engines here are a host-side stand-in (no GPU in this container) with the
same duck interface as sim.Engine: round_kernel / pending_records / resolve /
end_round / remote_copy / ingest.  The stand-in model keeps the properties
the protocol relies on (slave.c:415-428 conservative windows, worker.c:253
sends at least one window ahead):

  * every host executes its events in (time, src, seq) order;
  * an executed event sends one event to a host picked from a per-host
    counter, `lat(src, dst) >= window` ahead, so it never lands in the
    window that produced it;
  * the first send over a (src, dst) pair is a "first touch": the send is
    held, a pending record is logged, and the pair's latency is set only when
    the records of ALL ranks have been gathered (the rank of the pair in the
    serial order of the gathered records shifts its latency), exactly the
    global resolution the real engine does for path-cache rows.

The run over two ranks must produce the same per-host execution logs as one
engine owning every host, which is the serial-equivalence the real engine is
tested for on the GPU (tests/test_engine_gpu.py).
"""
import ctypes as C
import heapq
import os
import socket

import numpy as np
import pytest

import shdgpu as S
from driver import EV_WORDS, INF, DistCluster, partition

WINDOW = 1000
END = 60 * WINDOW
N_HOSTS = 24


class _Summary:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class _Model:
    params = {"end_time": END}


class ToyEngine:
    """Host-side stand-in for sim.Engine over hosts [h0, h1)."""

    def __init__(self, h0, h1, n_hosts=N_HOSTS):
        self.h0, self.h1, self.n = h0, h1, n_hosts
        self.window = WINDOW
        self.model = _Model()
        self.q = {h: [] for h in range(h0, h1)}          # per-host heap of (time, src, seq)
        self.ids = {h: 0 for h in range(h0, h1)}
        self.count = {h: 0 for h in range(h0, h1)}
        self.log = {h: [] for h in range(h0, h1)}
        self.lat = {}                                   # resolved (src, dst) -> latency
        self.held = []                                  # sends waiting for their pair
        self.pending = []
        self.outbox = []
        self.min_sent = INF

    def _push(self, h, t, src, seq):
        heapq.heappush(self.q[h], (t, src, seq))

    def boot(self):
        for h in self.q:
            for k in range(2):
                self._push(h, WINDOW + 37 * ((h * 5 + k * 3) % 11), h, self.ids[h])
                self.ids[h] += 1

    def next_time(self):
        return min([q[0][0] for q in self.q.values() if q] + [INF])

    def _send(self, src, t, dst):
        seq = self.ids[src]
        self.ids[src] += 1
        if (src, dst) not in self.lat:
            self.held.append((src, t, dst, seq))
            self.pending.append((t, seq, src, dst))
            return
        self._emit(src, t, dst, seq)

    def _emit(self, src, t, dst, seq):
        ta = t + self.lat[(src, dst)]
        if ta >= END:
            return
        if self.h0 <= dst < self.h1:
            self._push(dst, ta, src, seq)
        else:
            self.outbox.append((ta, seq, src, dst))
        self.min_sent = min(self.min_sent, ta)

    def round_kernel(self, ws, we):
        n = 0
        for h, q in self.q.items():
            while q and q[0][0] < we:
                t, src, seq = heapq.heappop(q)
                self.log[h].append((t, src, seq))
                self.count[h] += 1
                dst = (h * 7 + self.count[h] * 13) % self.n
                self._send(h, t, dst)
                n += 1
        return _Summary(n_pending=len(self.pending), n_events=n, n_pkt_events=n)

    def pending_records(self):
        recs = np.zeros(len(self.pending), dtype=S.PENDING_DTYPE)
        for i, (t, seq, src, dst) in enumerate(self.pending):
            recs[i]["qtime"], recs[i]["qseq"], recs[i]["qhost"], recs[i]["dst"] = t, seq, src, dst
        return recs

    def resolve(self, recs):
        order = np.lexsort((recs["qseq"], recs["qhost"], recs["qtime"]))
        for r, i in enumerate(order):
            key = (int(recs[i]["qhost"]), int(recs[i]["dst"]))
            if key not in self.lat:   # every rank sees the same records in the same order
                self.lat[key] = WINDOW + 101 * ((key[0] + 3 * key[1]) % 9) + r % 3
        self.pending = []
        held, self.held = self.held, []
        for src, t, dst, seq in held:
            self._emit(src, t, dst, seq)

    def end_round(self):
        nt = min(self.next_time(), self.min_sent)
        self.min_sent = INF
        return _Summary(next_time=nt)

    def remote_copy(self, ptr, cap):
        ev = np.zeros((len(self.outbox), EV_WORDS), dtype=np.int32)
        for i, (t, seq, src, dst) in enumerate(self.outbox):
            ev[i, 0:2] = np.array([t], dtype=np.uint64).view(np.int32)
            ev[i, 2:4] = np.array([seq], dtype=np.uint64).view(np.int32)
            ev[i, 4], ev[i, 5] = src, dst
        assert len(self.outbox) <= cap
        C.memmove(ptr, ev.ctypes.data, ev.nbytes)
        self.outbox = []
        return ev.shape[0]

    def ingest(self, ptr, n):
        ev = np.frombuffer((C.c_int32 * (n * EV_WORDS)).from_address(ptr), dtype=np.int32).reshape(n, EV_WORDS)
        for row in ev:
            t = int(row[0:2].copy().view(np.uint64)[0])
            seq = int(row[2:4].copy().view(np.uint64)[0])
            src, dst = int(row[4]), int(row[5])
            assert self.h0 <= dst < self.h1
            self._push(dst, t, src, seq)

    def last_kernel_ms(self):
        return 0.0


def _serial():
    e = ToyEngine(0, N_HOSTS)
    e.boot()
    nxt = e.next_time()
    rounds = 0
    while nxt < END:
        e.round_kernel(nxt, min(nxt + WINDOW, END))
        if e.pending:
            e.resolve(e.pending_records())
        nxt = e.end_round().next_time
        rounds += 1
    return e.log, rounds


def _rank_main(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pb = partition(N_HOSTS, world)
    eng = ToyEngine(pb[rank], pb[rank + 1])
    cl = DistCluster(eng, pb, rank, world, dist, torch, device="cpu")
    cl.boot()
    res = cl.run_until(INF)
    np.save(os.path.join(out_dir, f"log{rank}.npy"),
            np.array([(h, t, s, q) for h, L in eng.log.items() for (t, s, q) in L], dtype=np.int64))
    np.save(os.path.join(out_dir, f"res{rank}.npy"), np.array([res.rounds, res.exchanged, res.pending]))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_partition_blocks_cover_hosts():
    for n, p in [(10, 3), (10000, 8), (7, 7), (5, 2)]:
        b = partition(n, p)
        assert b[0] == 0 and b[-1] == n and all(b[i] <= b[i + 1] for i in range(p))


@pytest.mark.parametrize("world", [2])
def test_dist_cluster_gloo_matches_single_engine(world, tmp_path):
    import torch.multiprocessing as mp
    ref_log, ref_rounds = _serial()
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = np.concatenate([np.load(tmp_path / f"log{r}.npy") for r in range(world)])
    want = np.array([(h, t, s, q) for h, L in ref_log.items() for (t, s, q) in L], dtype=np.int64)
    assert len(want) > 500
    got = got[np.lexsort(got.T[::-1])]
    want = want[np.lexsort(want.T[::-1])]
    np.testing.assert_array_equal(got, want)
    res = [np.load(tmp_path / f"res{r}.npy") for r in range(world)]
    assert res[0][0] == res[1][0] == ref_rounds           # same windows on every rank
    assert sum(r[1] for r in res) > 0                       # cross-rank events were exchanged
    assert res[0][2] == res[1][2] > 0                       # first touches gathered globally
