"""Debug: the persistent group rounds (k_round_pg) against the oracle on the
multi-process tests' models; prints the first trace records that differ."""
import os
import sys
import tempfile
from pathlib import Path

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd"), os.path.join(REPO, "tests")]
import numpy as np   # noqa: E402
import oracle_ffi as O   # noqa: E402
import shdgpu as S   # noqa: E402
import workloads as W   # noqa: E402
from sim import sort_trace   # noqa: E402
import subprocess   # noqa: E402
import uuid   # noqa: E402


def run_ranks(world, tmp_path, extra=(), env_extra=None, timeout=240):
    name = "shdtest_" + uuid.uuid4().hex[:16]
    env = dict(os.environ)
    env.update(env_extra or {})
    w = os.path.join(REPO, "tests", "xgroup_worker.py")
    procs = [subprocess.Popen([sys.executable, "-u", w, "--rank", str(r), "--world", str(world), "--name", name,
                               "--out", str(tmp_path)] + list(extra),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env) for r in range(world)]
    for r, p in enumerate(procs):
        out, _ = p.communicate(timeout=timeout)
        print(f"--- rank {r} output (tail)")
        print("\n".join(out.decode(errors="replace").splitlines()[-400:]))
    return [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(world)]

R, C = 40, 200
for world, env, load in ((3, {"SHDGPU_LIB": "shadow-1_amd/libshdgpu_var.so"}, 4),):
    with tempfile.TemporaryDirectory() as td:
        res = run_ranks(world, Path(td), extra=["--tor", f"{R},{C}", "--load", str(load), "--end-s", "2.5", "--p2p"],
                        env_extra=env)
    g, m = W.tor_model(R, C, end_time=int(2.5 * S.SHD_SEC), trace=True, load=load)
    otr, odg, ost = O.engine_run(m, g)
    tr = sort_trace(np.concatenate([r["trace"] for r in res]))
    pkt = sum(int(r["stats"][0]) for r in res)
    otr = sort_trace(otr)
    print(f"tor world {world} load {load} env {env}: pkt {pkt} oracle {ost['n_pkt_events']}, trace {len(tr)} oracle {len(otr)}")
    for r in res:
        print("   stats [pkt, ev, pend, rounds, prot, rerun, fallback]", r["stats"].tolist())
    n = min(len(tr), len(otr))
    d = np.nonzero(tr[:n] != otr[:n])[0]
    if len(d) or len(tr) != len(otr):
        i = int(d[0]) if len(d) else n
        print("  first difference at", i)
        for k in range(max(0, i - 2), min(n, i + 6)):
            print("   dev", tr[k], "  orc", otr[k])
        # the missing record's send
        o = otr[i]
        snd = tr[(tr["kind"] == 1) & (tr["host"] == o["peer"]) & (tr["pkt"] == o["pkt"])]
        print("  device's SENT for the first oracle-only record:", snd)
    sys.stdout.flush()
