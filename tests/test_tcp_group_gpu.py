"""The TCP path (both transports) on a group of engines, one process each
(shd_tcp_run_group over the host-memory communicator: the ranks share one GPU
here, each running its contiguous share of the hosts): the union of the ranks'
lines, tracker lines and end states equals the reference's own loop on the
fixtures (tests/golden/ref_tcp.json) and the oracle (oracle/o_tcp.c) on the
scaled models -- deliveries between engines exchanged after every round,
the servers' listening ports published across engines, the window agreed
over the group."""
import json
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

import oracle_ffi as O
import tcp_cases as TC

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "ref_tcp.json")))
DEVICE_FALLS_BACK = set()   # (test_tcp_gpu.py's: the cases whose device choices the serial order contradicts)


def run_ranks(world, case, tmp_path, timeout=240, mode="tables"):
    name = "shdtcp_" + uuid.uuid4().hex[:16]
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "tcp_group_worker.py"), "--rank", str(r),
                               "--world", str(world), "--name", name, "--out", str(tmp_path), "--case", case,
                               "--mode", mode],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{outs[r][-3000:]}"
    res = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(world)]
    # the ranks' hosts tile the model in rank order
    assert [int(x["first_host"]) for x in res] == sorted(int(x["first_host"]) for x in res)
    lines = [tuple(x) for r in res for x in json.loads(str(r["lines"]))]
    node = sorted((tuple(x) for r in res for x in json.loads(str(r["node_lines"]))), key=lambda x: (x[0], x[1]))
    cat = {k: np.concatenate([r[k] for r in res]).tolist() for k in ("next_event_id", "next_packet_id", "rng_probe")}
    return lines, node, cat, res


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["mixed_hosts", "mixed_slow_rr", "geo_pairs", "shared_hosts"])
@pytest.mark.parametrize("mode", ["tables", "device"])
def test_tcp_group_equals_reference(name, world, mode, tmp_path):
    """mode "device": the path cache's first-touch rule on the device, every
    engine's log of a round gathered and replayed alike (a contradicted choice:
    every rank falls back to tables together, as shared_hosts does on one engine)"""
    f = FIX[name]
    lines, node, cat, res = run_ranks(world, name, tmp_path, mode=mode)
    assert len(lines) == f["n_status"]
    assert TC.digest(lines) == f["status_by_host_sha256"]
    assert len(node) == f["n_heartbeat"] and TC.digest(node) == f["heartbeat_sha256"]
    assert cat["next_event_id"] == f["next_event_id"]
    assert cat["next_packet_id"] == f["next_packet_id"]
    assert cat["rng_probe"] == f["rng_probe"]
    modes = {str(r["first_touch"]) for r in res}
    assert len(modes) == 1   # every rank alike
    if mode == "device" and name in ("geo_pairs", "mixed_hosts"):
        assert modes == {"device"}
    if mode == "device" and name in DEVICE_FALLS_BACK:
        assert modes == {"tables"}


@pytest.mark.parametrize("case,world", [("mixed:96:0.02:0", 3), ("mixed:128:0.01:1", 4), ("echo:96:0.02", 2)])
def test_tcp_group_scaled_equals_oracle(case, world, tmp_path):
    import workloads as W
    kind, h, loss, *rest = case.split(":")
    if kind == "mixed":
        g, m, ips, procs, peers, nb, udp = W.mixed_transport_model(int(h), 40, end_s=10, nbytes=60000,
                                                                    loss_max=float(loss))
        qdisc = int(rest[0]) if rest else 0
    else:
        g, m, ips, procs, peers, nb = W.tcp_echo_model(int(h), 40, end_s=12, nbytes=60000, loss_max=float(loss))
        udp, qdisc = None, 0
    o = O.tcp_run(m, g, ips, procs, peers, nbytes=nb, qdisc=qdisc, udp=udp)
    lines, _, cat, res = run_ranks(world, case, tmp_path)
    want = TC.by_host(o["lines"])
    assert len(lines) == len(want)
    assert lines == want
    assert cat["next_event_id"] == o["next_event_id"].tolist()
    assert cat["next_packet_id"] == o["next_packet_id"].tolist()
    assert cat["rng_probe"] == o["rng_probe"].tolist()
    assert sum(int(r["events"]) for r in res) == o["events"]


def test_tcp_group_rccl_one_rank_equals_one_engine():
    """The RCCL communicator's calls of the group run (all-gathers, the grouped
    send / receive of the all-to-all-v) on a one-rank group: RCCL refuses two
    ranks on one GPU, so the multi-rank path is tested over the host-memory
    transport above and this runs RCCL's side alone -- equal to shd_tcp_run."""
    import sim
    import tcp as TCPGPU
    f = FIX["mixed_hosts"]
    c, m = TC.build("mixed_hosts")
    ips = TC.ip_ints(f["ips"])
    comm = sim.Comm.rccl(sim.XGroup.unique_id(), 1, 0, 0)
    try:
        r = TCPGPU.run(m, c["graph"], ips, c["procs"], c["peers"], nbytes=c["nbytes"], node=True,
                       udp=TC.udp_arg(c), comm=comm, mode="tables")
    finally:
        comm.close()
    assert r["first_host"] == 0 and r["n_local_hosts"] == len(ips)
    assert TC.digest(r["lines"]) == f["status_by_host_sha256"]
    assert r["next_event_id"].tolist() == f["next_event_id"]
    assert r["rng_probe"].tolist() == f["rng_probe"]
