"""Synthetic workloads for the BASELINE configs (host side, numpy).

The reference has no generators for these configs; they are defined in
SURVEY.md section 8(d) / BASELINE.md section 2.2:

* C2  the bundled topology (resource/topology.graphml.xml.xz, 183 vertices,
      complete) -- a committed data fixture under tests/golden/.
* C3  PHOLD-UDP, 10k hosts, one per vertex of a 10k-vertex random geometric
      graph (unit square, radius 1.5x the connectivity threshold, latency
      1 + 50*distance ms, edge loss U[0, 0.01], a self-loop on every vertex).
* C5  the same graph family with 100 hosts per vertex (1M hosts at V = 10k).

Host ids are dense registration order; host seeds follow the reference seed
chain (master.c:95,417 -> slave.c:182,198,301) and each host's RNG then
consumes the one nextDouble draw of topology_attach (topology.c:2326-2334),
which the reference makes even on an exact-IP match.
"""
from __future__ import annotations

import lzma
import math
import os

import numpy as np

import shdgpu as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUNDLED_XZ = os.path.join(REPO, "tests", "golden", "topology.graphml.xml.xz")


def bundled_graphml_bytes() -> bytes:
    with lzma.open(BUNDLED_XZ) as f:
        return f.read()


def load_graphml_bytes(xml: bytes):
    """Parse graphml with libshdgpu's loader; returns (GraphArrays, GraphML*)."""
    lib = S.lib()
    gm = S.P(S.GraphML)()
    S.check(lib.shd_graphml_load_string(xml, len(xml), S.C.byref(gm)), "shd_graphml_load_string")
    return S.graph_from_graphml(gm), gm


def bundled_graph():
    g, gm = load_graphml_bytes(bundled_graphml_bytes())
    S.lib().shd_graphml_free(gm)
    return g


def geometric_graph(n_vertices: int, seed: int = 1, radius_factor: float = 1.5,
                    loss_max: float = 0.01, self_loops: bool = True,
                    vertex_loss: bool = False, max_tries: int = 20,
                    integer_latency: bool = False) -> S.GraphArrays:
    """Random geometric graph in the unit square; connected (retries seeds).
    integer_latency: whole milliseconds (ceil), as Shadow topologies usually
    have them -- equal-cost paths everywhere."""
    rng = np.random.default_rng(seed)
    V = int(n_vertices)
    r = radius_factor * math.sqrt(math.log(max(V, 2)) / (math.pi * max(V, 2)))
    for _ in range(max_tries):
        pts = rng.random((V, 2))
        # grid bucketing: O(V * degree)
        cell = max(r, 1e-9)
        ncell = max(1, int(1.0 / cell))
        cx = np.minimum((pts[:, 0] * ncell).astype(np.int64), ncell - 1)
        cy = np.minimum((pts[:, 1] * ncell).astype(np.int64), ncell - 1)
        cid = cx * ncell + cy
        order = np.argsort(cid, kind="stable")
        cs = cid[order]
        starts = np.searchsorted(cs, np.arange(ncell * ncell))
        ends = np.searchsorted(cs, np.arange(ncell * ncell), side="right")
        src, dst = [], []
        for dx in (-1, 0, 1):
            for dy in (-1, 0, 1):
                nx, ny = cx + dx, cy + dy
                ok = (nx >= 0) & (nx < ncell) & (ny >= 0) & (ny < ncell)
                for i in np.nonzero(ok)[0]:
                    c = nx[i] * ncell + ny[i]
                    js = order[starts[c]:ends[c]]
                    js = js[js > i]
                    if len(js) == 0:
                        continue
                    d = np.hypot(pts[js, 0] - pts[i, 0], pts[js, 1] - pts[i, 1])
                    js = js[d <= r]
                    src.append(np.full(len(js), i, dtype=np.int64))
                    dst.append(js)
        src = np.concatenate(src) if src else np.zeros(0, np.int64)
        dst = np.concatenate(dst) if dst else np.zeros(0, np.int64)
        # connectivity check (union-find)
        parent = np.arange(V)

        def find(x):
            while parent[x] != x:
                parent[x] = parent[parent[x]]
                x = parent[x]
            return x
        for a, b in zip(src.tolist(), dst.tolist()):
            ra, rb = find(a), find(b)
            if ra != rb:
                parent[ra] = rb
        roots = {find(i) for i in range(V)}
        if len(roots) == 1:
            break
        r *= 1.1
    else:
        raise RuntimeError("could not generate a connected geometric graph")
    dist = np.hypot(pts[src, 0] - pts[dst, 0], pts[src, 1] - pts[dst, 1])
    lat = 1.0 + 50.0 * dist
    if integer_latency:
        lat = np.ceil(lat)
    loss = rng.random(len(src)) * loss_max
    # document order: shuffle edges so ids are not sorted by endpoint
    perm = rng.permutation(len(src))
    src, dst, lat, loss = src[perm], dst[perm], lat[perm], loss[perm]
    if self_loops:
        sl_lat = 1.0 + 50.0 * r * rng.random(V) + 0.5
        if integer_latency:
            sl_lat = np.ceil(sl_lat)
        sl_loss = rng.random(V) * loss_max
        src = np.concatenate([src, np.arange(V)])
        dst = np.concatenate([dst, np.arange(V)])
        lat = np.concatenate([lat, sl_lat])
        loss = np.concatenate([loss, sl_loss])
    vl = rng.random(V) * 0.001 if vertex_loss else None
    return S.GraphArrays(V, src, dst, lat, loss, vl)


def grid_graph(side: int = 6, seed: int = 5, loss_max: float = 0.05, directed: bool = False,
               parallel: bool = False) -> S.GraphArrays:
    """side x side grid, every edge (and self-loop) 1 ms: equal-cost paths
    between almost every pair, edge loss U[0, loss_max], edges in a shuffled
    document order.  directed: every edge both ways, each with its own loss;
    parallel: a second copy of every tenth edge (equal latency, its own loss)."""
    rng = np.random.default_rng(seed)
    src, dst = [], []
    for y in range(side):
        for x in range(side):
            v = y * side + x
            if x + 1 < side:
                src.append(v); dst.append(v + 1)
            if y + 1 < side:
                src.append(v); dst.append(v + side)
    if directed:
        src, dst = src + dst, dst + src
    if parallel:
        src += src[::10]; dst += dst[::10]
    V = side * side
    src += list(range(V))
    dst += list(range(V))
    perm = rng.permutation(len(src))
    src, dst = np.array(src)[perm], np.array(dst)[perm]
    return S.GraphArrays(V, src, dst, np.ones(len(src)), rng.random(len(src)) * loss_max, directed=directed)


def seed_chain(n_hosts: int, options_seed: int = 1) -> np.ndarray:
    seeds = np.zeros(n_hosts, dtype=np.uint32)
    S.check(S.lib().shd_seed_chain(options_seed, n_hosts, S.as_ptr(seeds, S.C.c_uint32)),
            "shd_seed_chain")
    return seeds


def after_attach_draw(seeds: np.ndarray) -> np.ndarray:
    """Advance each host RNG by the one attach draw (topology.c:2326-2334)."""
    out = seeds.copy()
    # rand_r = 3 LCG steps; vectorised
    x = out.astype(np.uint64)
    for _ in range(3):
        x = (x * np.uint64(1103515245) + np.uint64(12345)) & np.uint64(0xFFFFFFFF)
    return x.astype(np.uint32)


def uniform_cum(n_hosts: int) -> np.ndarray:
    """PHOLD cumulative weights for equal weights (test_phold.c:160-178):
    cumulative += w_i / total, accumulated in order in f64."""
    w = 1.0
    total = 0.0
    for _ in range(1):  # total = sum of n ones, exact
        total = float(n_hosts) * w
    norm = w / total
    cum = np.empty(n_hosts, dtype=np.float64)
    c = 0.0
    # sequential f64 accumulation (np.cumsum is sequential for 1-D float64)
    cum[:] = np.cumsum(np.full(n_hosts, norm, dtype=np.float64))
    # guard: np.cumsum must equal the scalar left fold
    if n_hosts <= 4096:
        for i in range(n_hosts):
            c += norm
            assert cum[i] == c
    return cum


def phold_cum(weights) -> np.ndarray:
    """_phold_chooseNode's cumulative weights (test_phold.c:160-178) from a
    weights file's values (test_phold.c:341-356): totalWeight is the sequential
    sum of the weights, and cumulative += weights[i] / totalWeight, in order."""
    w = np.ascontiguousarray(weights, dtype=np.float64)
    total = np.add.accumulate(w)[-1] if len(w) else 0.0       # sequential left fold
    return np.add.accumulate(w / total)                       # per-element division, then the fold


def phold_model(host_vertex, *, end_time, seed=1, bw_down=10240, bw_up=10240, load=16,
                payload=1, app_start=S.SHD_SEC, heartbeat=S.SHD_SEC, bootstrap_end=0,
                trace=False, dest_cum=None, host_class=None, host_rng=None, **caps) -> S.ModelArrays:
    """PHOLD-UDP hosts; dest_cum None = uniform weights over all hosts, else
    [H] or [n_classes, H] (then host_class [H]); host_rng None = the seed
    chain after the attach draw (one random pick per host)."""
    H = len(host_vertex)
    seeds = after_attach_draw(seed_chain(H, seed)) if host_rng is None else host_rng
    bd = np.broadcast_to(np.asarray(bw_down, dtype=np.uint64), (H,)).copy()
    bu = np.broadcast_to(np.asarray(bw_up, dtype=np.uint64), (H,)).copy()
    cum = uniform_cum(H) if dest_cum is None else dest_cum
    return S.ModelArrays(host_vertex, seeds, bd, bu, cum, end_time=end_time,
                         app_start=app_start, load=load, payload=payload,
                         heartbeat_interval=heartbeat, bootstrap_end=bootstrap_end, trace=trace,
                         host_class=host_class, **caps)


def attach_random(gm_ptr, seeds: np.ndarray):
    """topology_attach for hosts with no hints (topology.c:2326-2334): one
    host-RNG draw picks the vertex.  Returns (vertex [H], rng after [H],
    bw_down [H], bw_up [H]) with the vertex bandwidths (host.c:183-189)."""
    lib = S.lib()
    H = len(seeds)
    vert = np.empty(H, np.int32)
    rng = np.ascontiguousarray(seeds, dtype=np.uint32).copy()
    bd = np.empty(H, np.uint64)
    bu = np.empty(H, np.uint64)
    st = S.C.c_uint32()
    v = S.C.c_int32()
    d = S.C.c_uint64()
    u = S.C.c_uint64()
    for h in range(H):
        st.value = int(rng[h])
        S.check(lib.shd_topology_attach(gm_ptr, S.C.byref(st), None, None, None, None, None,
                                        S.C.byref(v), S.C.byref(d), S.C.byref(u)), "shd_topology_attach")
        vert[h], rng[h], bd[h], bu[h] = v.value, st.value, d.value, u.value
    return vert, rng, bd, bu


def tor_model(n_relays: int, n_clients: int, *, end_time, seed=1, load=4, payload=1,
              app_start=S.SHD_SEC, client_share=0.5, sigma=1.0, trace=False, **caps):
    """BASELINE C4, synthetic Tor-scale traffic on the bundled topology (the
    ccs-2018 traffic model is a placeholder in the reference,
    docs/2018-ccs-tmodel.md:1).  Hosts 0..R-1 are relays, R..R+C-1 clients,
    each a PHOLD-UDP process with its own weights file (test_phold.c:341-356):
      - a client sends to relays only, by relay weight (log-normal, seeded);
      - a relay forwards to relays by the same weights and to clients
        (uniformly) with total share `client_share`.
    Hosts attach at random with their RNG (topology.c:2326-2334) and take the
    vertex bandwidths.  Returns (graph, model, graphml pointer to free)."""
    xml = bundled_graphml_bytes()
    g, gm = load_graphml_bytes(xml)
    H = n_relays + n_clients
    seeds = seed_chain(H, seed)
    vert, rng, bd, bu = attach_random(gm, seeds)
    S.lib().shd_graphml_free(gm)
    wr = np.random.default_rng(seed + 7).lognormal(0.0, sigma, n_relays)
    w_client_row = np.concatenate([wr, np.zeros(n_clients)])
    cw = float(np.add.accumulate(wr)[-1]) * client_share / (1.0 - client_share) / max(n_clients, 1)
    w_relay_row = np.concatenate([wr, np.full(n_clients, cw)])
    cum = np.stack([phold_cum(w_relay_row), phold_cum(w_client_row)])
    cls = np.concatenate([np.zeros(n_relays, np.uint8), np.ones(n_clients, np.uint8)])
    # the popular relays take far more than a uniform share of the traffic:
    # per-host queue capacities sized for the heaviest relay, not the mean
    # (an overflow is reported as SHD_EOVERFLOW, never silent)
    p_client = wr.max() / float(np.add.accumulate(wr)[-1])
    p_relay = wr.max() / float(np.add.accumulate(w_relay_row)[-1])
    burst = load * (n_clients * p_client + n_relays * p_relay)   # the start's sends to the heaviest relay
    pow2 = lambda x: 1 << int(math.ceil(math.log2(max(x, 1))))  # noqa: E731
    caps.setdefault("inbox_cap", max(1024, pow2(2 * burst)))
    caps.setdefault("evq_cap", max(2048, pow2(4 * burst)))
    caps.setdefault("codelq_cap", max(1024, pow2(2 * burst)))
    m = phold_model(vert, end_time=end_time, seed=seed, bw_down=bd, bw_up=bu, load=load, payload=payload,
                    app_start=app_start, trace=trace, dest_cum=cum, host_class=cls, host_rng=rng, **caps)
    return g, m


def hosts_on_vertices(n_vertices: int, hosts_per_vertex: int) -> np.ndarray:
    """Registration order: host i on vertex i // hosts_per_vertex."""
    return np.repeat(np.arange(n_vertices, dtype=np.int32), hosts_per_vertex)


def attached_vertices(host_vertex) -> np.ndarray:
    return np.unique(np.asarray(host_vertex, dtype=np.int32))


def config_model(xml: bytes, *, load=16, payload=1, seed=1, trace=False, topology_bytes=None, **caps):
    """A shadow.config.xml through the reference's set-up path, with PHOLD-UDP
    in place of the configured plugins (the tgen binary of the bundled example
    is not in the reference tree):
      configuration_new -> hosts in document order, `quantity` names, hints,
        bandwidth overrides, <process starttime> (shd_config_load_buffer);
      dns_register (shd_dns_assign); seed chain (master.c:95,417 -> slave.c:301);
      topology_new on the inline or referenced graphml;
      topology_attach per host (hints, one RNG draw) with the vertex bandwidth
        unless the host sets its own (host.c:176-192);
      process_schedule per process at boot (host.c:372-390): pushed starts.
    Returns (graph, model, pushed start events, host names, ips)."""
    hosts, ips, stop_s, topo = S.load_config(xml)
    if topology_bytes is not None:
        gxml = topology_bytes
    elif topo and topo.lstrip().startswith("<"):
        gxml = topo.encode()
    else:
        raise ValueError("config_model: the topology is a path; pass its bytes as topology_bytes")
    lib = S.lib()
    gm = S.P(S.GraphML)()
    S.check(lib.shd_graphml_load_string(gxml, len(gxml), S.C.byref(gm)), "shd_graphml_load_string")
    g = S.graph_from_graphml(gm)
    H = len(hosts)
    seeds = seed_chain(H, seed)
    vert = np.empty(H, np.int32)
    rng = seeds.copy()
    bd = np.empty(H, np.uint64)
    bu = np.empty(H, np.uint64)
    st, v, d, u = S.C.c_uint32(), S.C.c_int32(), S.C.c_uint64(), S.C.c_uint64()
    enc = lambda x: None if x is None else x.encode()  # noqa: E731
    for i, h in enumerate(hosts):
        st.value = int(rng[i])
        S.check(lib.shd_topology_attach(gm, S.C.byref(st), enc(h["ip_hint"]), enc(h["citycode_hint"]),
                                        enc(h["countrycode_hint"]), enc(h["geocode_hint"]), enc(h["type_hint"]),
                                        S.C.byref(v), S.C.byref(d), S.C.byref(u)), "shd_topology_attach")
        vert[i], rng[i] = v.value, st.value
        bd[i] = h["bw_down_kibps"] or d.value
        bu[i] = h["bw_up_kibps"] or u.value
    lib.shd_graphml_free(gm)
    hb = np.array([(h["heartbeat_s"] or 1) * S.SHD_SEC for h in hosts], dtype=np.uint64)
    pushes = np.array([(t * S.SHD_SEC, 0, i, i, 0, S.EV_APP_START)
                       for i, h in enumerate(hosts) for t in h["process_start_s"]], dtype=S.EVENT_DTYPE)
    m = S.ModelArrays(vert, rng, bd, bu, uniform_cum(H), end_time=stop_s * S.SHD_SEC, load=load,
                      payload=payload, trace=trace, host_heartbeat=hb,
                      queue_flags=S.SHD_QF_NO_APP_START | caps.pop("queue_flags", 0), **caps)
    return g, m, pushes, [h["name"] for h in hosts], ips


def tcp_echo_model(n_hosts: int, n_vertices: int, *, seed: int = 1, end_s: int = 20, nbytes: int = 100000,
                   loss_max: float = 0.0, bw_down=10240, bw_up=10240):
    """The TCP path's scaled model (include/shdtcp.h): the reference's TCP echo
    test (src/test/tcp/test_tcp.c, nonblocking-epoll) run by n_hosts / 2
    client/server pairs on a random geometric topology.  Host h sits on vertex
    h * V // H; even hosts run a server from 1 s; the client on host 2i + 1
    starts at 2 s + i us and connects to the server of pair (i + n/2) mod n,
    so connections cross the graph.  Addresses are 11.0.0.1 upwards (no .0 /
    .255 octet, as dns.c hands them out).  Returns (graph, model, ips, procs,
    peers, nbytes)."""
    H = int(n_hosts) & ~1
    n = H // 2
    g = geometric_graph(n_vertices, seed=seed, loss_max=loss_max)
    hv = (np.arange(H, dtype=np.int64) * n_vertices // H).astype(np.int32)
    m = phold_model(hv, end_time=end_s * S.SHD_SEC, seed=seed, load=0, bw_down=bw_down, bw_up=bw_up)
    ips, ip = [], (11 << 24) + 1
    while len(ips) < H:
        if (ip & 255) not in (0, 255):
            ips.append(ip)
        ip += 1
    procs = [(2 * i, S.SHD_SEC) for i in range(n)] + [(2 * i + 1, 2 * S.SHD_SEC + i * 1000) for i in range(n)]
    peers = [-1] * n + [(i + n // 2) % n for i in range(n)]
    return g, m, ips, procs, peers, nbytes


def mixed_transport_model(n_hosts: int, n_vertices: int, *, seed: int = 1, end_s: int = 12, nbytes: int = 60000,
                          loss_max: float = 0.0, payload: int = 512, bw_down=10240, bw_up=10240):
    """tcp_echo_model's echo pairs plus one datagram process per host
    (shd_tcp_model.proc_app, shdgpu.h shd_udp_app), from 1 s + h us, by h % 4:
    0 PHOLD-like (a socket per datagram to a weighted host's listener, 2 at
    start, one per datagram read), 1 a listener sending to its peer h + 1 (2 at
    start, one per read), 2 a listener answering each datagram to its sender,
    3 a connected-style client (one implicitly bound socket) of host h - 1's
    listener.  Both transports share each host's interface.  Returns (graph,
    model, ips, procs, peers, nbytes, udp) with udp as shadow-1_amd/tcp.py's
    run() takes it."""
    g, _, ips, procs, peers, nb = tcp_echo_model(n_hosts, n_vertices, seed=seed, end_s=end_s, nbytes=nbytes,
                                                 loss_max=loss_max, bw_down=bw_down, bw_up=bw_up)
    H = len(ips)
    hv = (np.arange(H, dtype=np.int64) * n_vertices // H).astype(np.int32)
    m = phold_model(hv, end_time=end_s * S.SHD_SEC, seed=seed, load=0, payload=payload, bw_down=bw_down, bw_up=bw_up)
    specs = [(S.SHD_SEND_EACH, S.SHD_DEST_WEIGHTED, 2, 1), (S.SHD_SEND_LISTENER, S.SHD_DEST_PEER, 2, 1),
             (S.SHD_SEND_LISTENER, S.SHD_DEST_REPLY, 0, 1), (S.SHD_SEND_ONCE, S.SHD_DEST_PEER, 1, 1)]
    app_peer = [-1] * H
    apps = [-1] * len(procs)
    for h in range(H):
        k = h % 4
        if k == 1 and h + 1 < H:
            app_peer[h] = h + 1
        elif k == 3:
            app_peer[h] = h - 1
        elif k == 1:
            k = 2   # the last host has no peer after it: it answers instead
        procs = procs + [(h, S.SHD_SEC + h * 1000)]
        peers = peers + [-1]
        apps.append(k)
    udp = dict(apps=apps, specs=specs, app_peer=app_peer, payload=payload)
    return g, m, ips, procs, peers, nb, udp
