"""Round drivers: the conservative window loop of master.c / slave.c over one or
more engines (DESIGN.md "Multi-GPU").

Each engine owns a contiguous block of hosts.  One round is:

  1. every engine runs its round kernel on [ws, we)                 (device)
  2. first-touch queries logged this round (rare after warm-up) are gathered
     from ALL engines and resolved identically everywhere            (host)
  3. events bound for hosts of other engines are exchanged          (xGMI)
  4. next window start = min over engines of their next event time

`LocalCluster` drives several engines inside one process (tests; one GPU or
several); `DistCluster` drives one engine per rank with torch.distributed:
backend "nccl" is RCCL on ROCm (device tensors over xGMI), "gloo" is the CPU
transport used by the CPU tests.  Per round: one all_gather of a small int64
control vector and, when any rank has events for another, one
all_to_all_single of 32-B event records.  Engines are duck-typed (sim.Engine
on the GPU; tests/test_driver_cpu.py uses a host-side stand-in).
"""
from __future__ import annotations

import time

import numpy as np

import shdgpu as S

EV_BYTES = 32
EV_WORDS = 8          # int32 words per event
DST_WORD = 5          # shd_event.dst
INF = (1 << 64) - 1


def partition(n_hosts: int, n_parts: int) -> list[int]:
    """Contiguous host blocks (registration order): part p owns [b[p], b[p+1])."""
    return [(n_hosts * p) // n_parts for p in range(n_parts + 1)]


class RunResult:
    def __init__(self):
        self.rounds = 0
        self.events = 0
        self.pkt_events = 0
        self.pending = 0
        self.exchanged = 0
        self.kernel_ms = 0.0
        self.wall_s = 0.0


def _u64(x) -> int:
    return int(np.int64(x).view(np.uint64))


def _i64(x) -> int:
    return int(np.uint64(x).view(np.int64))


class LocalCluster:
    """Several engines in one process; exchange through device tensors."""

    def __init__(self, engines, part_begin, device="cuda"):
        import torch
        self.torch = torch
        self.engines = engines
        self.part_begin = list(part_begin)
        self.window = min(e.window for e in engines)
        self.end_time = engines[0].model.params["end_time"]
        self.next = INF
        self.dev = device
        self.bufs = [torch.empty(max(1, e.h1 - e.h0) * 256 * EV_BYTES, dtype=torch.uint8, device=device)
                     for e in engines]
        self.pb = torch.tensor(self.part_begin[1:-1], device=device, dtype=torch.int64)

    def boot(self):
        for e in self.engines:
            e.boot()
        self.next = min(e.next_time() for e in self.engines)

    def _exchange(self) -> int:
        torch = self.torch
        outs = []
        for e, b in zip(self.engines, self.bufs):
            n = e.remote_copy(b.data_ptr(), b.numel() // EV_BYTES)
            outs.append(b[: n * EV_BYTES].view(torch.int32).view(-1, EV_WORDS))
        if not any(o.shape[0] for o in outs):
            return 0
        allev = torch.cat(outs)
        part = torch.bucketize(allev[:, DST_WORD].to(torch.int64), self.pb, right=True)
        sels = [allev[part == p].contiguous() for p in range(len(self.engines))]
        # torch kernels run on torch's stream, the engines on their own streams
        torch.cuda.current_stream().synchronize()
        total = 0
        for sel, e in zip(sels, self.engines):
            if sel.shape[0]:
                e.ingest(sel.data_ptr(), sel.shape[0])
                total += sel.shape[0]
        return total

    def run_until(self, t_stop) -> RunResult:
        res = RunResult()
        t0 = time.perf_counter()
        stop = min(t_stop, self.end_time)
        while self.next < stop:
            ws = self.next
            we = min(ws + self.window, stop)
            sums = [e.round_kernel(ws, we) for e in self.engines]
            npend = sum(s.n_pending for s in sums)
            if npend:
                recs = np.concatenate([e.pending_records() for e in self.engines])
                for e in self.engines:
                    e.resolve(recs)
                res.pending += npend
            ends = [e.end_round() for e in self.engines]
            res.exchanged += self._exchange()
            self.next = min(s.next_time for s in ends)
            res.rounds += 1
            res.events += sum(s.n_events for s in sums)
            res.pkt_events += sum(s.n_pkt_events for s in sums)
            res.kernel_ms += sum(e.last_kernel_ms() for e in self.engines)
        res.wall_s = time.perf_counter() - t0
        return res


class DistCluster:
    """One engine per rank; collectives through torch.distributed."""

    def __init__(self, engine, part_begin, rank, world, dist, torch_mod, device="cuda"):
        self.eng = engine
        self.part_begin = list(part_begin)
        self.rank, self.world = rank, world
        self.dist, self.torch = dist, torch_mod
        self.dev = device
        self.end_time = engine.model.params["end_time"]
        torch = torch_mod
        w = torch.tensor([engine.window], dtype=torch.int64, device=device)
        dist.all_reduce(w, op=dist.ReduceOp.MIN)
        self.window = int(w.item())
        cap = max(1, engine.h1 - engine.h0) * 256
        self.sendbuf = torch.empty(cap * EV_BYTES, dtype=torch.uint8, device=device)
        self.pb = torch.tensor(self.part_begin[1:-1], device=device, dtype=torch.int64)
        self.next = INF

    def _allgather_i64(self, vec):
        torch = self.torch
        t = torch.tensor([int(v) for v in vec], dtype=torch.int64, device=self.dev)
        out = torch.empty(self.world * len(vec), dtype=torch.int64, device=self.dev)
        self.dist.all_gather_into_tensor(out, t)
        return out.view(self.world, len(vec)).cpu().numpy()

    def boot(self):
        self.eng.boot()
        g = self._allgather_i64([_i64(self.eng.next_time())])
        self.next = min(_u64(x) for x in g[:, 0])

    def _gather_pending(self, local: np.ndarray) -> np.ndarray:
        torch = self.torch
        isz = S.PENDING_DTYPE.itemsize
        counts = self._allgather_i64([len(local)])[:, 0]
        mx = int(counts.max())
        raw = np.zeros(mx * isz, dtype=np.uint8)
        raw[: local.nbytes] = np.ascontiguousarray(local).view(np.uint8)
        t = torch.from_numpy(raw).to(self.dev)
        out = torch.empty(self.world * raw.size, dtype=torch.uint8, device=self.dev)
        self.dist.all_gather_into_tensor(out, t)
        allb = out.view(self.world, -1).cpu().numpy()
        parts = [allb[r, : int(counts[r]) * isz].copy().view(S.PENDING_DTYPE) for r in range(self.world)]
        return np.concatenate(parts)

    def run_until(self, t_stop) -> RunResult:
        torch = self.torch
        res = RunResult()
        t0 = time.perf_counter()
        stop = min(t_stop, self.end_time)
        while self.next < stop:
            ws = self.next
            we = min(ws + self.window, stop)
            s = self.eng.round_kernel(ws, we)
            npend = self._allgather_i64([s.n_pending])[:, 0]
            if npend.sum():
                self.eng.resolve(self._gather_pending(self.eng.pending_records()))
                res.pending += int(npend.sum())
            e = self.eng.end_round()
            n = self.eng.remote_copy(self.sendbuf.data_ptr(), self.sendbuf.numel() // EV_BYTES)
            ev = self.sendbuf[: n * EV_BYTES].view(torch.int32).view(-1, EV_WORDS)
            if n:
                part = torch.bucketize(ev[:, DST_WORD].to(torch.int64), self.pb, right=True)
                order = torch.argsort(part, stable=True)
                ev = ev[order].contiguous()
                send_counts = torch.bincount(part, minlength=self.world).cpu().tolist()
            else:
                send_counts = [0] * self.world
            ctl = self._allgather_i64([_i64(e.next_time)] + send_counts)
            recv_counts = [int(x) for x in ctl[:, 1 + self.rank]]
            if ctl[:, 1:].sum():
                recv = torch.empty(sum(recv_counts) * EV_WORDS, dtype=torch.int32, device=self.dev)
                self.dist.all_to_all_single(recv, ev.reshape(-1), [c * EV_WORDS for c in recv_counts],
                                            [c * EV_WORDS for c in send_counts])
                if self.dev != "cpu":
                    torch.cuda.current_stream().synchronize()
                if sum(recv_counts):
                    self.eng.ingest(recv.data_ptr(), sum(recv_counts))
                res.exchanged += sum(recv_counts)
            self.next = min(_u64(x) for x in ctl[:, 0])
            res.rounds += 1
            res.events += s.n_events
            res.pkt_events += s.n_pkt_events
            res.kernel_ms += self.eng.last_kernel_ms()
        res.wall_s = time.perf_counter() - t0
        return res
