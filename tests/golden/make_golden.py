"""Generate the committed golden fixtures for the oracle (run in the build
container; the outputs are small data files, never reference source).

Sources of truth, per fixture:
  rng_kats.json          glibc rand_r through ctypes (libc.so.6) and the
                         reference's own random.c compiled into oracle/_ref
                         (random_new / random_nextDouble / random_nextUInt),
                         plus the seed chain master.c:95,417 -> slave.c:182,198,301
                         computed with the reference random.c.
  codel_trace.json       scripted enqueue/dequeue timelines driven through the
                         reference's own router_queue_codel.c (oracle/_ref).
  pathcache_geo300.npz   networkx 3.4.2 single_source_dijkstra distances and
                         paths on a tie-free 300-vertex geometric graph, with
                         latency / reliability folded along networkx's path in
                         the order of _topology_computePathProperties
                         (topology.c:1407-1523).  Independent of igraph.
  bundled_summary.json   counts of the bundled topology (topology.graphml.xml.xz,
                         itself a data file of the reference, resource/).

Usage: python tests/golden/make_golden.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "shadow-1_amd"), os.path.join(REPO, "tests")]

import workloads as W  # noqa: E402

REF_SO = os.path.join(REPO, "oracle", "_ref", "libshdref.so")


def ref_lib():
    l = C.CDLL(REF_SO)
    l.ref_random_new.restype = C.c_void_p; l.ref_random_new.argtypes = [C.c_uint32]
    l.ref_random_rand.restype = C.c_int32; l.ref_random_rand.argtypes = [C.c_void_p]
    l.ref_random_next_double.restype = C.c_double; l.ref_random_next_double.argtypes = [C.c_void_p]
    l.ref_random_next_uint.restype = C.c_uint32; l.ref_random_next_uint.argtypes = [C.c_void_p]
    l.ref_random_free.argtypes = [C.c_void_p]
    l.ref_codel_new.restype = C.c_void_p
    l.ref_codel_free.argtypes = [C.c_void_p]
    l.ref_codel_enqueue.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32]
    l.ref_codel_dequeue.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint32)]
    l.ref_codel_drops.restype = C.c_uint32
    l.ref_codel_drops.argtypes = [C.POINTER(C.c_uint32), C.c_uint32]
    l.ref_pq_order.argtypes = [C.c_void_p] * 4 + [C.c_uint32, C.c_void_p]
    return l


def rng_kats(l):
    libc = C.CDLL("libc.so.6")
    libc.rand_r.restype = C.c_int
    libc.rand_r.argtypes = [C.POINTER(C.c_uint)]
    out = {"rand_r": {}, "next_double": {}, "next_uint": {}}
    for seed in (1, 2, 12345, 953415426, 2714057858, 0xFFFFFFFF):
        s = C.c_uint(seed)
        out["rand_r"][str(seed)] = [libc.rand_r(C.byref(s)) for _ in range(8)] + [s.value]
        r = l.ref_random_new(seed)
        out["next_double"][str(seed)] = [l.ref_random_next_double(r).hex() for _ in range(8)]
        l.ref_random_free(r)
        r = l.ref_random_new(seed)
        out["next_uint"][str(seed)] = [l.ref_random_next_uint(r) for _ in range(8)]
        l.ref_random_free(r)
    # seed chain for --seed 1 (reference random.c objects chained as master/slave do)
    master = l.ref_random_new(1)
    slave_seed = l.ref_random_next_uint(master)
    slave = l.ref_random_new(slave_seed)
    sched = l.ref_random_next_uint(slave)
    hosts = [l.ref_random_next_uint(slave) for _ in range(64)]
    out["seed_chain_1"] = {"slave": slave_seed, "scheduler": sched, "hosts": hosts}
    return out


def codel_scripts():
    """Deterministic timelines that drive CoDel through store/drop modes."""
    rng = np.random.default_rng(7)
    scripts = []
    for k in range(6):
        ops = []
        t = 0
        pid = 0
        burst = [5, 20, 60, 150, 300, 40][k]
        for step in range(400):
            t += int(rng.integers(100_000, 3_000_000))
            for _ in range(int(rng.integers(0, burst // 10 + 2))):
                ops.append(["enq", t, pid, int(rng.choice([1, 500, 1458]))])
                pid += 1
            if rng.random() < 0.6:
                ops.append(["deq", t + int(rng.integers(0, 50_000_000))])
                t = ops[-1][1]
        scripts.append(ops)
    return scripts


def codel_trace(l):
    res = []
    for ops in codel_scripts():
        q = l.ref_codel_new()
        outs = []
        buf = (C.c_uint32 * 65536)()
        for op in ops:
            if op[0] == "enq":
                l.ref_codel_enqueue(q, op[1], op[2], op[3])
                outs.append(["enq"])
            else:
                pid = C.c_uint32()
                ok = l.ref_codel_dequeue(q, op[1], C.byref(pid))
                n = l.ref_codel_drops(buf, 65536)
                outs.append(["deq", int(ok), int(pid.value) if ok else -1, list(buf[:n])])
        l.ref_codel_free(q)
        res.append({"ops": ops, "outs": outs})
    return res


def fold_path(g, path):
    """latency/reliability folded along a vertex path (topology.c:1428-1508)."""
    lat = 0.0
    rel = 1.0
    src, dst = path[0], path[-1]
    if g.vertex_loss is not None and not np.isnan(g.vertex_loss[src]):
        rel *= (1.0 - g.vertex_loss[src])
    if g.vertex_loss is not None and not np.isnan(g.vertex_loss[dst]) and src != dst:
        rel *= (1.0 - g.vertex_loss[dst])
    eid = {}
    for e, (a, b) in enumerate(zip(g.src.tolist(), g.dst.tolist())):
        eid.setdefault((min(a, b), max(a, b)), e)
    for a, b in zip(path[:-1], path[1:]):
        e = eid[(min(a, b), max(a, b))]
        lat += float(g.latency[e])
        rel *= (1.0 - float(g.loss[e]))
    return lat, rel


def pathcache_geo300():
    import networkx as nx
    g = W.geometric_graph(300, seed=21, vertex_loss=True)
    G = nx.Graph()
    G.add_nodes_from(range(g.n_vertices))
    for a, b, w in zip(g.src.tolist(), g.dst.tolist(), g.latency.tolist()):
        if a != b:
            G.add_edge(a, b, weight=w)
    srcs = list(range(0, 300, 7))
    lat = np.zeros((len(srcs), 300)); rel = np.zeros_like(lat); hops = np.zeros(lat.shape, np.int32)
    for i, s in enumerate(srcs):
        dist, paths = nx.single_source_dijkstra(G, s, weight="weight")
        for t in range(300):
            if t == s:
                lat[i, t] = np.nan; rel[i, t] = np.nan
                continue
            p = paths[t]
            l_, r_ = fold_path(g, p)
            assert l_ == dist[t]
            lat[i, t], rel[i, t], hops[i, t] = l_, r_, len(p) - 1
    np.savez_compressed(os.path.join(HERE, "pathcache_geo300.npz"), src=g.src, dst=g.dst,
                        latency=g.latency, loss=g.loss, vertex_loss=g.vertex_loss,
                        sources=np.array(srcs), lat=lat, rel=rel, hops=hops)


def bundled_summary():
    g = W.bundled_graph()
    d = {"V": g.n_vertices, "E": g.n_edges,
         "self_loops": int(np.sum(g.src == g.dst)),
         "latency_min": float(g.latency.min()), "latency_max": float(g.latency.max()),
         "distinct_latency": int(len(np.unique(g.latency))),
         "edge_loss_unique": sorted(set(g.loss.tolist())),
         "vertex_loss_unique": sorted(set(np.nan_to_num(g.vertex_loss, nan=-1).tolist()))}
    return d


if __name__ == "__main__":
    l = ref_lib()
    with open(os.path.join(HERE, "rng_kats.json"), "w") as f:
        json.dump(rng_kats(l), f, indent=1)
    with open(os.path.join(HERE, "codel_trace.json"), "w") as f:
        json.dump(codel_trace(l), f)
    pathcache_geo300()
    with open(os.path.join(HERE, "bundled_summary.json"), "w") as f:
        json.dump(bundled_summary(), f, indent=1)
    print("golden fixtures written")
