"""bench.py at N > 1 checks its own end state (round 6): after the timed
region every rank hashes its hosts' end states and rank 0 runs the whole model
on one engine of its own GPU over the same [0, end); the line carries
"parity" and the transport that actually ran.  Rehearsed here with two ranks
sharing the one GPU over the host-memory communicator (the peer-to-peer
transport runs as on a node, IPC-mapped receive blocks included); with the
test build's hook that loses exchanged events on taking them
(SHD_TEST_XDROP) the same run must report parity false."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TH_LIB = os.path.join(REPO, "shadow-1_amd", "libshdgpu_th.so")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("drop", [0, 50])
def test_bench_rehearsal_checks_the_group_against_one_engine(drop):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    if drop:
        env.update(SHDGPU_LIB=TH_LIB, SHD_TEST_XDROP=str(drop))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--comm", "host", "--steps", "1", "--warmup", "1",
           "--hosts-per-gpu", "2000", "--vertices", "2000", "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=env, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-3000:]
    line = json.loads(p.stdout.decode().strip().splitlines()[-1])
    par = line["parity"]
    assert line["transport"] == "p2p", line["transport"]
    assert par["ok"] == (drop == 0), par
    assert par["ranks_ok"] == [drop == 0] * 2 or drop, par
    if drop == 0:
        assert par["pkt_events_group"] == par["pkt_events_single_engine"] > 0, par
