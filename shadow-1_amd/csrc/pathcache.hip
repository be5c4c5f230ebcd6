// pathcache.hip -- the topology path cache on MI355X (gfx950).
//
// Replaces the lazy igraph-Dijkstra cache of src/main/routing/topology.c with
// three device kernels that fill [T][T] f64 tables in HBM (T = attached
// vertices):
//
//   k_sssp_rows    one workgroup per source row (persistent over rows):
//                  frontier Bellman-Ford in LDS (distances as u64 bit patterns
//                  of non-negative doubles, ds_min_u64), then each vertex picks
//                  its shortest-path parent (the in-arc with d[u]+w == d[v] and
//                  the smallest d[u], the arc Dijkstra relaxes first), then every
//                  target walks its parent chain and folds latency and
//                  reliability FORWARD from the source exactly as
//                  _topology_computePathProperties does (topology.c:1407-1523):
//                  lat = ((0+w1)+w2)+..., rel = ((1*r(src))*r(dst))*r(e1)*r(e2)...
//                  Relaxation d[x] = d[u] + w(u,x) is the same left fold, so the
//                  converged distance equals igraph's on tie-free graphs.
//   k_direct       direct-path values of adjacent pairs (topology.c:1877-1927).
//   k_self         "2 x min incident edge" self values (topology.c:1545-1653).
//
// No MFMA: min-plus relaxation is not a multiply-add contraction.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>
#include <unordered_map>

#include "shd_device.h"

static char g_last_error[512];
void shd_set_hip_error(hipError_t e, const char* what, const char* file, int line) {
    snprintf(g_last_error, sizeof(g_last_error), "%s:%d %s -> %s", file, line, what,
             hipGetErrorString(e));
    fprintf(stderr, "libshdgpu: %s\n", g_last_error);
}

extern "C" const char* shd_version(void) { return "libshdgpu 0.1 (gfx950)"; }

extern "C" int shd_device_count(int* n) {
    if (!n) return SHD_EINVAL;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return SHD_OK;
}

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ double u2d(uint64_t u) { return __longlong_as_double((long long)u); }
__device__ __forceinline__ uint64_t d2u(double d) { return (uint64_t)__double_as_longlong(d); }
// k_sssp_tie_g's per-vertex entry of a row (there: why no heap position)
template <typename HV>
struct TieG {
    HV negd;       // the heap value (-distance) at its last push / decrease
    uint32_t st;   // 0 unreached, 2 reached
};

// reliability factor of a vertex whose packetloss attribute is present
// (_topology_findVertexAttributeDouble: NaN means absent, topology.c:330-347)
__device__ __forceinline__ bool vrel(const double* vloss, int32_t v, double* r) {
    if (!vloss) return false;
    double l = vloss[v];
    if (isnan(l)) return false;
    *r = (double)1.0f - l;
    return true;
}

#ifdef SHD_SSSP_TIMING   // measurement build (scripts/sssp_timing.py): cycles per phase per block
__device__ unsigned long long g_sssp_tim[1024][16];
extern "C" int shd_debug_sssp_timing(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return SHD_ENODEV;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sssp_tim), sizeof(g_sssp_tim)) == hipSuccess ? SHD_OK : SHD_ENODEV;
}
#define SST_T0(v) const unsigned long long v = clock64();
#define SST_ADD(k, v) if (threadIdx.x % 64 == 0 && blockIdx.x < 1024) atomicAdd(&g_sssp_tim[blockIdx.x][k], clock64() - v);
#define SST_CNT(k, n) if (blockIdx.x < 1024) atomicAdd(&g_sssp_tim[blockIdx.x][k], (unsigned long long)(n));
#else
#define SST_T0(v)
#define SST_ADD(k, v)
#define SST_CNT(k, n)
#endif

// ------------------------------------------------------------------ SSSP rows
// Per-row working set: dist u64[V], parent i32[V] (index into the rin_* arcs),
// upd u16[V] (iteration at which the vertex last improved = frontier stamp).
constexpr int kChunk = 32;   // edges folded per pass of the forward chain walk
#ifndef SHD_SSSP_BFQ
#define SHD_SSSP_BFQ 2   // queued frontier: vertices per half-wave relaxed together
#endif
#ifndef SHD_SSSP_MIXQ
#define SHD_SSSP_MIXQ 0  // 1: the two-row kernel's rows share one queue (21.35 against 20.28 ms: not kept)
#endif
#ifndef SHD_SSSP_BALLOT
#define SHD_SSSP_BALLOT 0  // 1: the two-row kernel walks only its non-empty bit words (a ballot, one readlane
                           // each) instead of every chunk's four shuffles: 22.1-22.4 against 21.4 ms on the
                           // 10 k table (scripts/r05/gpu_apsp_ballot.sh, profiles/r05/apsp_ballot/): not kept
#endif
#ifndef SHD_SSSP_BFQ2
#define SHD_SSSP_BFQ2 2  // ... in the two-row kernel (1: 21.6 ms, 2: 20.3 ms on the 10 k table)
#endif

template <int BLOCK>
__device__ void sssp_one_row(int32_t row, int32_t src, int32_t V, int32_t T,
                             const int32_t* __restrict__ arc_off, const int32_t* __restrict__ arc_dst,
                             const double* __restrict__ arc_w, const int32_t* __restrict__ arc_src,
                             const int32_t* __restrict__ arc_rin, const int32_t* __restrict__ rin_off,
                             const int32_t* __restrict__ rin_src, const int32_t* __restrict__ rin_eid,
                             const double* __restrict__ rin_w, const double* __restrict__ rin_r,
                             const double* __restrict__ w_e,
                             const double* __restrict__ eloss, const double* __restrict__ vloss,
                             const int32_t* __restrict__ attached, const int32_t* __restrict__ self_eid,
                             shd_pv* __restrict__ out,
                             int64_t* __restrict__ stats, uint64_t* dist, int32_t* parent,
                             uint16_t* upd, int* flags /* LDS int[4] */,
                             const int32_t* __restrict__ fpar, int32_t* __restrict__ tie_rows,
                             int32_t* fl_pre, int32_t* fl_beg, uint64_t* fl_dv /* LDS [BLOCK] each */,
                             const uint16_t* off16, const int32_t* cbase /* LDS arc offsets, or null */,
                             bool bfq /* queued frontier: four vertices a wave in flight */,
                             int bf_it = -1 /* >= 0: dist holds the row's converged distances (sssp_bf2) */,
                             bool count_ties = false /* with fpar: count the row's ties all the same */) {
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6, hl = lane & 31;
    const bool upper = lane >= 32;
    int it = 0;
    if (bf_it >= 0) {   // the distances came from the two-row Bellman-Ford
        for (int32_t v = tid; v < V; v += BLOCK) parent[v] = -1;
        if (tid < 4) flags[tid] = 0;
        it = bf_it;
        __syncthreads();
    } else {
    for (int32_t v = tid; v < V; v += BLOCK) {
        dist[v] = kDistInf;
        parent[v] = -1;
        upd[v] = 0xFFFF;
    }
    if (tid < 4) flags[tid] = 0;
    __syncthreads();
    if (tid == 0) { dist[src] = 0; upd[src] = 0; }
    __syncthreads();

    // ---- frontier Bellman-Ford: vertices improved in iteration `it` relax in it+1.
    // Wave-cooperative: a wave ballots a 64-vertex chunk for frontier vertices
    // (their arc ranges loaded by their own lanes in one batch), then each
    // half-wave relaxes one frontier vertex's out-arcs, 32 arcs per load round,
    // instead of one lane walking ~20 arcs with a dependent L2 load per arc.
    // Any relaxation order reaches the same fixpoint: d[x] = min over paths of
    // the left-folded sum (fl(a + w) is monotone in a).
    SST_T0(t_bf)
    for (;;) {
        if (tid == 0) flags[(it + 1) % 3] = 0;
        const uint16_t stamp = (uint16_t)it;
        SST_T0(t_it)
        if (bfq) {
            // queued frontier: the wave's chunks are balloted as before, but
            // frontier vertices go to a four-entry queue (uniform registers)
            // and are relaxed four at a time -- each half-wave takes two, the
            // first arc load of both issued before either relaxes -- so a wave
            // keeps two vertices' loads in flight where the pairs below keep
            // one (a chunk holds ~1.3 frontier vertices: the pairs mostly ran
            // one half-wave on one vertex)
            constexpr int Q = SHD_SSSP_BFQ;   // vertices per half-wave in flight
            int32_t q[2 * Q];
#pragma unroll
            for (int j = 0; j < 2 * Q; j++) q[j] = -1;
            int nq = 0;
            auto arc_range = [&](int32_t v, int32_t& b, int32_t& e) {
                if (off16) {
                    b = cbase[v >> 6] + off16[v];
                    e = v + 1 < V ? cbase[(v + 1) >> 6] + off16[v + 1] : cbase[(V + 63) >> 6];
                } else {
                    b = arc_off[v];
                    e = arc_off[v + 1];
                }
            };
            auto relax = [&](int32_t x, double cand) {
                const uint64_t nb = d2u(cand);
                if (nb < dist[x]) {
                    const uint64_t old = atomicMin((unsigned long long*)&dist[x], (unsigned long long)nb);
                    if (nb < old) {
                        upd[x] = (uint16_t)(it + 1);
                        flags[it % 3] = 1;
                    }
                }
            };
            auto run_q = [&]() {
                int32_t bq[Q], eq[Q], xq[Q];
                double dq[Q], wq[Q];
#pragma unroll
                for (int j = 0; j < Q; j++) {
                    const int32_t v = upper ? q[2 * j + 1] : q[2 * j];
                    bq[j] = 0; eq[j] = 0; dq[j] = 0.0;
                    if (v >= 0) { arc_range(v, bq[j], eq[j]); dq[j] = u2d(dist[v]); }
                }
#pragma unroll
                for (int j = 0; j < Q; j++) {
                    const int32_t k = bq[j] + hl;
                    xq[j] = -1; wq[j] = 0.0;
                    if (k < eq[j]) { xq[j] = arc_dst[k]; wq[j] = arc_w[k]; }
                }
#pragma unroll
                for (int j = 0; j < Q; j++)
                    if (xq[j] >= 0) relax(xq[j], dq[j] + wq[j]);
#pragma unroll
                for (int j = 0; j < Q; j++)
                    for (int32_t k = bq[j] + hl + 32; k < eq[j]; k += 32) relax(arc_dst[k], dq[j] + arc_w[k]);
            };
            auto push = [&](int32_t fv) {
#pragma unroll
                for (int j = 0; j < 2 * Q - 1; j++) q[j] = q[j + 1];
                q[2 * Q - 1] = fv;
            };
            for (int32_t c0 = wv * 64; c0 < V; c0 += BLOCK) {
                const int32_t v = c0 + lane;
                uint64_t mask = __ballot(v < V && upd[v] == stamp);
                while (mask) {
                    const int32_t fv = c0 + __ffsll((unsigned long long)mask) - 1;
                    mask &= mask - 1;
                    push(fv);
                    if (++nq == 2 * Q) {
                        run_q();
                        nq = 0;
                    }
                }
            }
            if (nq) {
                while (nq < 2 * Q) { push(-1); nq++; }
                run_q();
            }
        } else
        for (int32_t c0 = wv * 64; c0 < V; c0 += BLOCK) {
            const int32_t v = c0 + lane;
#ifdef SHD_SSSP_GS   // A/B: a vertex improved earlier in this sweep relaxes now too (and again next sweep)
            const uint16_t uv = v < V ? upd[v] : 0xFFFF;
            const bool fr = v < V && (uv == stamp || uv == (uint16_t)(stamp + 1));
#else
            const bool fr = v < V && upd[v] == stamp;
#endif
            uint64_t mask = __ballot(fr);
            if (!mask) continue;
            SST_T0(t_rx)
            if (lane == 0) { SST_CNT(5, __popcll(mask)); }
            int32_t beg = 0, end = 0;
            uint64_t dvb = 0;
            if (fr) {
                if (off16) {   // the arc offsets from LDS: no L2 round trip before the arcs' loads
                    beg = cbase[v >> 6] + off16[v];
                    end = v + 1 < V ? cbase[(v + 1) >> 6] + off16[v + 1] : cbase[(V + 63) >> 6];
                } else {
                    beg = arc_off[v];
                    end = arc_off[v + 1];
                }
                dvb = dist[v];
            }
#ifdef SHD_SSSP_FLAT
            // A/B (measured and rejected): the chunk's frontier
            // arcs flattened over the wave -- an exclusive scan of the frontier
            // lanes' degrees in LDS, each lane up to four arcs per step (owner
            // by binary search over the scan), every arc's loads out before any
            // is consumed: one L2 round trip for a chunk's arcs however many
            // frontier vertices it holds.  37.1 ms for the 10 k table against
            // 24.5 ms with the half-wave pairs below (a chunk holds ~1.3
            // frontier vertices in the graph's own order: the scan is overhead)
            {
                const int32_t deg = fr ? end - beg : 0;
                int32_t inc = deg;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const int32_t y = __shfl_up(inc, off, 64);
                    if (lane >= off) inc += y;
                }
                const int32_t total = __shfl(inc, 63, 64);
                int32_t* pre = fl_pre + wv * 64;
                fl_pre[wv * 64 + lane] = inc - deg;
                fl_beg[wv * 64 + lane] = beg;
                fl_dv[wv * 64 + lane] = dvb;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                for (int32_t k0 = 0; k0 < total; k0 += 256) {
                    int32_t xs[4];
                    double ws[4], dv4[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int32_t k = k0 + j * 64 + lane;
                        xs[j] = -1;
                        if (k < total) {
                            int32_t lo = 0, hi = 64;   // the last lane whose exclusive prefix is <= k
                            while (hi - lo > 1) {
                                const int32_t mid = (lo + hi) >> 1;
                                if (pre[mid] <= k) lo = mid; else hi = mid;
                            }
                            const int32_t a = fl_beg[wv * 64 + lo] + (k - pre[lo]);
                            xs[j] = arc_dst[a];
                            ws[j] = arc_w[a];
                            dv4[j] = u2d(fl_dv[wv * 64 + lo]);
                        }
                    }
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        if (xs[j] < 0) continue;
                        const int32_t x = xs[j];
                        const uint64_t nb = d2u(dv4[j] + ws[j]);
                        if (nb < dist[x]) {
                            const uint64_t old = atomicMin((unsigned long long*)&dist[x], (unsigned long long)nb);
                            if (nb < old) {
                                upd[x] = (uint16_t)(it + 1);
                                flags[it % 3] = 1;
                            }
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();   // (the scan slots are rewritten by the wave's next chunk)
                mask = 0;
            }
#endif
            while (mask) {
                const int l0 = __ffsll((unsigned long long)mask) - 1;
                mask &= mask - 1;
                const int l1 = mask ? __ffsll((unsigned long long)mask) - 1 : l0;
                if (mask) mask &= mask - 1;
                const int src_lane = upper ? l1 : l0;
                // every lane takes part in every shuffle (an inactive source lane reads as 0)
                const int32_t b = __shfl(beg, src_lane), e_all = __shfl(end, src_lane);
                const int32_t e = (upper && l1 == l0) ? b : e_all;
                const double dv = u2d((uint64_t)__shfl((long long)dvb, src_lane));
                for (int32_t k = b + hl; k < e; k += 32) {
                    const int32_t x = arc_dst[k];
                    const uint64_t nb = d2u(dv + arc_w[k]);
                    if (nb < dist[x]) {
                        const uint64_t old = atomicMin((unsigned long long*)&dist[x], (unsigned long long)nb);
                        if (nb < old) {
                            upd[x] = (uint16_t)(it + 1);
                            flags[it % 3] = 1;
                        }
                    }
                }
            }
            SST_ADD(2, t_rx)
        }
        SST_ADD(1, t_it)
        SST_T0(t_bar)
        __syncthreads();
        SST_ADD(3, t_bar)
        const bool more = flags[it % 3] != 0;
        it++;
        if (!more || it >= 0xFFFE) break;
    }
    SST_ADD(0, t_bf)
    if (tid == 0) { SST_CNT(4, it); SST_CNT(7, 1); }
    }   // (bf_it < 0)

#if defined(SHD_SSSP_STOP_AFTER) && SHD_SSSP_STOP_AFTER == 1   // phase ablation (scripts/apsp_phases.sh)
    __syncthreads();
    return;
#endif
    // ---- parent per vertex: smallest d[u] among exact predecessors (d[u] + w
    // == d[v]; every such u is final: a later decrease of d[u] would undercut
    // d[v]), equal d[u] (a tie Dijkstra breaks by heap order, unpinned) ->
    // lowest edge id.  One streaming pass over the forward arcs in CSR order
    // (coalesced: lane per arc, four arcs per lane in flight) counts each
    // vertex's exact predecessors and records one; the few vertices with more
    // than one (ties, equal-cost paths) take the exact rule over their in-arcs.
    // (Round 1 scanned every vertex's in-arcs, lane per vertex: uncoalesced,
    // 9.7 of the 29 ms of the 10 k-row table.)
    int64_t my_ties = 0;
    SST_T0(t_par)
    if (fpar && !count_ties) {
        // the row's parents given (k_sssp_tie_parents: igraph's first relaxer
        // in its heap's pop order, for a row with equal-cost predecessors)
        for (int32_t v = tid; v < V; v += BLOCK) parent[v] = fpar[v];
    } else if (fpar) {
        // count_ties: a row sent to the tie kernel without a first pass (a
        // predicted all-tied build, on whole-number weights: every distance an
        // exact integer below 2^30) -- its ties counted, its parents the given
        // ones.  A tie: two or more exact predecessors at the least exact
        // predecessor distance; per vertex that least distance (32-bit atomicMin
        // in parent[]), then the exact predecessors at it (16-bit counts in upd):
        // two streaming passes over the arcs instead of an in-arc walk per vertex
        uint32_t* mind = (uint32_t*)parent;
        uint32_t* cnt2 = (uint32_t*)upd;
        for (int32_t v = tid; v < V; v += BLOCK) mind[v] = 0xFFFFFFFFu;
        for (int32_t w = tid; w < (V + 1) / 2; w += BLOCK) cnt2[w] = 0;
        __syncthreads();
        const int32_t na = arc_off[V];
        for (int pass = 0; pass < 2; pass++) {
            for (int32_t k0 = tid; k0 < na; k0 += 4 * BLOCK) {
                int32_t uu[4], xx[4];
                double ww[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int32_t k = min(k0 + j * BLOCK, na - 1);
                    uu[j] = arc_src[k];
                    xx[j] = arc_dst[k];
                    ww[j] = arc_w[k];
                }
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int32_t k = k0 + j * BLOCK;
                    if (k >= na) break;
                    const int32_t x = xx[j];
                    if (x == src) continue;
                    const uint64_t dub = dist[uu[j]];
                    if (dub == kDistInf) continue;
                    if (u2d(dub) + ww[j] != u2d(dist[x])) continue;
                    const uint32_t du = (uint32_t)u2d(dub);
                    if (pass == 0) atomicMin(&mind[x], du);
                    else if (du == mind[x]) atomicAdd(&cnt2[x >> 1], 1u << ((x & 1) * 16));
                }
            }
            __syncthreads();
        }
        for (int32_t v = tid; v < V; v += BLOCK)
            if (upd[v] > 1) my_ties++;
        __syncthreads();
        for (int32_t v = tid; v < V; v += BLOCK) parent[v] = fpar[v];
    } else {
        uint32_t* cnt2 = (uint32_t*)upd;   // two 16-bit counts per word (the BF stamps are done with)
        for (int32_t w = tid; w < (V + 1) / 2; w += BLOCK) cnt2[w] = 0;
        __syncthreads();
        const int32_t na = arc_off[V];
        for (int32_t k0 = tid; k0 < na; k0 += 4 * BLOCK) {
            int32_t uu[4], xx[4];
            double ww[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {   // the four arcs' loads go out together
                const int32_t k = min(k0 + j * BLOCK, na - 1);
                uu[j] = arc_src[k];
                xx[j] = arc_dst[k];
                ww[j] = arc_w[k];
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int32_t k = k0 + j * BLOCK;
                if (k >= na) break;
                const int32_t x = xx[j];
                if (x == src) continue;
                const uint64_t dub = dist[uu[j]];
                if (dub == kDistInf) continue;
                if (u2d(dub) + ww[j] == u2d(dist[x])) {
                    atomicAdd(&cnt2[x >> 1], 1u << ((x & 1) * 16));
                    parent[x] = arc_rin[k];
                }
            }
        }
        __syncthreads();
        for (int32_t v = tid; v < V; v += BLOCK) {
            if (upd[v] <= 1) continue;
            const double dv = u2d(dist[v]);
            int32_t best = -1;
            uint64_t bestd = kDistInf;
            int nbest = 0;
            const int32_t kb = rin_off[v], ke = rin_off[v + 1];
            for (int32_t k = kb; k < ke; k++) {
                const uint64_t dub = dist[rin_src[k]];
                if (dub == kDistInf) continue;
                if (u2d(dub) + rin_w[k] == dv) {
                    if (best < 0 || dub < bestd) { best = k; bestd = dub; nbest = 1; }
                    else if (dub == bestd) {
                        nbest++;
                        if (rin_eid[k] < rin_eid[best]) best = k;
                    }
                }
            }
            parent[v] = best;
            if (nbest > 1) my_ties++;
        }
    }
    if (my_ties) {
        atomicAdd((unsigned long long*)&stats[0], (unsigned long long)my_ties);
        flags[3] = 1;
    }
    SST_ADD(8, t_par)
    if (tid == 0 && !fpar) atomicMax((unsigned long long*)&stats[2], (unsigned long long)it);
    __syncthreads();
    // A vertex with several exact predecessors at the same smallest d[u] (equal-
    // cost paths, or parallel edges) takes its parent from the heap's pop order
    // in igraph's Dijkstra, which the rule above does not see: the row is listed
    // for k_sssp_tie_parents and finished by a second pass with those parents.
    if (tie_rows) {
        const bool tie_row = flags[3] != 0;
        __syncthreads();
        if (tie_row) {
            if (tid == 0) tie_rows[atomicAdd((unsigned long long*)&stats[6], 1ull)] = row;
            return;
        }
    }

#if defined(SHD_SSSP_STOP_AFTER) && SHD_SSSP_STOP_AFTER == 2
    return;
#endif
    // ---- properties per target (topology.c:1407-1523).
    // lat: the forward fold w1 + w2 + ... along the parent chain is the very
    // relaxation that set dist[t] (the parent satisfies d[u] + w == d[t] with
    // final values), so lat == dist[t] bit for bit.
    // rel: ((1 * r(src)) * r(dst)) * r(e1) * r(e2) ...; for a target without a
    // vertex factor that is the prefix P[t] = P[u] * r(e) over the tree,
    // P[src] = 1 * r(src), computed level by level in LDS.  Targets with a
    // vertex loss factor walk their chain (the factor enters second).
    double rsrc = 1.0;
    const bool has_rsrc = vrel(vloss, src, &rsrc);
    int32_t my_maxhops = 0;
    int64_t my_unroutable = 0, my_mismatch = 0;
    SST_T0(t_p1)
    // (1) special targets in full, lat half of the others
    for (int32_t j = tid; j < T; j += BLOCK) {
        const int32_t t = attached[j];
        double lat, rel, rt;
        if (t == src) {
            // igraph 0.7.1 returns the path [src]: the self-loop edge alone, no
            // destination factor (topology.c:1456-1508)
            const int32_t e = self_eid[row];
            if (e < 0) {
                lat = -1.0; rel = -1.0; my_unroutable++;
            } else {
                lat = 0.0 + w_e[e];
                rel = 1.0;
                if (has_rsrc) rel *= rsrc;
                rel *= ((double)1.0f - eloss[e]);
            }
        } else if (dist[t] == kDistInf) {
            lat = -1.0; rel = -1.0; my_unroutable++;
        } else if (vrel(vloss, t, &rt)) {
            rel = 1.0;
            if (has_rsrc) rel *= rsrc;
            rel *= rt;
            int32_t k = 0;
            bool broken = false;   // (a parent chain that does not reach the source: counted, never followed)
            for (int32_t v = t; v != src; v = rin_src[parent[v]]) {
                if (parent[v] < 0 || k >= V) { broken = true; break; }
                k++;
            }
            if (broken) {
                my_mismatch++;
                out[(size_t)row * T + j] = shd_pv{-1.0, -1.0};
                continue;
            }
            if (k > my_maxhops) my_maxhops = k;
            lat = 0.0;
            int32_t eid_buf[kChunk];
            for (int32_t done = 0; done < k; done += kChunk) {
                const int32_t cnt = min(kChunk, k - done);
                int32_t v = t;
                for (int32_t s = 0; s < k - done - cnt; s++) v = rin_src[parent[v]];
                for (int32_t s = cnt - 1; s >= 0; s--) {
                    const int32_t a = parent[v];
                    eid_buf[s] = rin_eid[a];
                    v = rin_src[a];
                }
                for (int32_t s = 0; s < cnt; s++) {
                    const int32_t e = eid_buf[s];
                    lat += w_e[e];
                    rel *= ((double)1.0f - eloss[e]);
                }
            }
            if (d2u(lat) != dist[t]) my_mismatch++;
            if (lat == 0) lat = 1;   // topology.c:1848-1852
        } else {
            lat = u2d(dist[t]);
            if (lat == 0) lat = 1;
            // the whole pair (rel filled in by (4)): a wave's stores then cover
            // whole lines, where 8-B stores at a 16-B stride leave every line
            // (and ECC word) half written, for a read-modify-write in memory
            out[(size_t)row * T + j] = shd_pv{lat, 0.0};
            continue;
        }
        out[(size_t)row * T + j] = shd_pv{lat, rel};
    }
    __syncthreads();
    SST_ADD(9, t_p1)
    SST_T0(t_p2)
#if defined(SHD_SSSP_STOP_AFTER) && SHD_SSSP_STOP_AFTER == 4   // phase ablation: targets' first pass only
    return;
#endif
    // (2) tree arrays: parent[v] <- parent vertex, dist[v] <- edge factor r(e)
    // (rin_r: the in-arc's 1 - loss, precomputed), four vertices per thread
    // with their loads out together
    constexpr uint16_t kTodo = 0xFFFF, kNever = 0xFFFE;
    for (int32_t v0 = tid; v0 < V; v0 += 4 * BLOCK) {
        int32_t pa[4], pu[4];
        double pr[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int32_t v = v0 + j * BLOCK;
            pa[j] = (v < V && v != src && dist[v] != kDistInf) ? parent[v] : -1;
            pu[j] = pa[j] >= 0 ? rin_src[pa[j]] : -1;
            pr[j] = pa[j] >= 0 ? rin_r[pa[j]] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int32_t v = v0 + j * BLOCK;
            if (v >= V) break;
            if (v == src) {
                dist[v] = d2u(has_rsrc ? 1.0 * rsrc : 1.0);
                upd[v] = 0;
            } else if (pa[j] >= 0) {
                parent[v] = pu[j];
                dist[v] = d2u(pr[j]);
                upd[v] = kTodo;
            } else {
                upd[v] = kNever;
            }
        }
    }
    __syncthreads();
    SST_ADD(10, t_p2)
    SST_T0(t_p3)
#if defined(SHD_SSSP_STOP_AFTER) && SHD_SSSP_STOP_AFTER == 3   // phase ablation: no level passes
    return;
#endif
    // (3) the tree prefix, without a barrier per level: every thread sweeps
    // its own vertices until each is done; a vertex finishes once its parent
    // has (P[v] = P[u] * r(e), the order of the reference's forward fold),
    // taking the parent's depth + 1 (the level the per-level passes of round 1
    // gave it).  Its product is written before its depth (a workgroup release
    // between them), and readers read the depth first, through volatile LDS
    // accesses, so a done parent's product is its final one.  A chain of L
    // hops needs at most L sweeps of its vertices' threads; threads never
    // wait on each other, so some vertex finishes in every round of sweeps.
    {
        volatile uint16_t* vupd = upd;
        volatile uint64_t* vdist = dist;
        bool left = true;
        for (int32_t sweep = 0; left; sweep++) {
            left = false;
            for (int32_t v = tid; v < V; v += BLOCK) {
                if (vupd[v] != kTodo) continue;
                const int32_t u = parent[v];
                const uint16_t du = vupd[u];
                if (du >= kNever) {   // the parent is not done yet
                    left = true;
                    continue;
                }
                vdist[v] = d2u(u2d(vdist[u]) * u2d(vdist[v]));
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                vupd[v] = (uint16_t)(du + 1);
            }
            if (sweep > V) {   // cannot be: a parent chain longer than the graph
                atomicAdd((unsigned long long*)&stats[4], 1ull);
                break;
            }
        }
    }
    __syncthreads();
    SST_ADD(11, t_p3)
    SST_T0(t_p4)
    // (4) rel half of the prefix targets
    for (int32_t j = tid; j < T; j += BLOCK) {
        const int32_t t = attached[j];
        if (t == src || upd[t] >= kNever) continue;
        double rt;
        if (vrel(vloss, t, &rt)) continue;
        shd_pv* o = &out[(size_t)row * T + j];
        *o = shd_pv{o->lat, u2d(dist[t])};   // the pair whole again (see (1))
        if ((int32_t)upd[t] > my_maxhops) my_maxhops = upd[t];
    }
    if (my_maxhops) atomicMax((unsigned long long*)&stats[1], (unsigned long long)my_maxhops);
    if (my_unroutable) atomicAdd((unsigned long long*)&stats[3], (unsigned long long)my_unroutable);
    if (my_mismatch) atomicAdd((unsigned long long*)&stats[4], (unsigned long long)my_mismatch);
    __syncthreads();
    SST_ADD(12, t_p4)
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_sssp_rows_lds(
    int32_t V, int32_t T, const int32_t* __restrict__ arc_off, const int32_t* __restrict__ arc_dst,
    const double* __restrict__ arc_w, const int32_t* __restrict__ arc_src, const int32_t* __restrict__ arc_rin,
    const int32_t* __restrict__ rin_off,
    const int32_t* __restrict__ rin_src, const int32_t* __restrict__ rin_eid,
    const double* __restrict__ rin_w, const double* __restrict__ rin_r, const double* __restrict__ w_e,
    const double* __restrict__ eloss,
    const double* __restrict__ vloss, const int32_t* __restrict__ attached,
    const int32_t* __restrict__ self_eid, shd_pv* __restrict__ out,
    int64_t* __restrict__ stats, int32_t row0, int32_t row1, const int32_t* __restrict__ row_list,
    const int32_t* __restrict__ fpar, int32_t* __restrict__ tie_rows, int mode /* bit 0 LDS offsets, 1 queued */,
    const char* __restrict__ gdist, int gkind, const uint8_t* __restrict__ gok, int32_t cnt_from) {
    // gdist (round 6): the tied rows' distances from k_sssp_tie_g's per-row entries
    // (gkind 4: TieG<int32_t>, 8: TieG<double>), for the rows gok marks complete --
    // no Bellman-Ford again for them, only the properties over the given parents
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int ldsoff = mode & 1;
    uint64_t* dist = (uint64_t*)smem;
    int32_t* parent = (int32_t*)(smem + (size_t)8 * V);
    uint16_t* upd = (uint16_t*)(smem + (size_t)12 * V);
    int* flags = (int*)(smem + (((size_t)14 * V + 15) & ~(size_t)15));
    // ldsoff: the forward CSR's offsets kept in LDS for every row of the block
    // (a 32-bit base per 64-vertex chunk, a 16-bit offset per vertex; the host
    // checked that a chunk's arcs number below 65 536)
    uint16_t* off16 = nullptr;
    int32_t* cbase = nullptr;
    if (ldsoff) {
        off16 = (uint16_t*)(smem + (((size_t)14 * V + 15) & ~(size_t)15) + 16);
        cbase = (int32_t*)(smem + (((size_t)14 * V + 15) & ~(size_t)15) + 16 + (((size_t)2 * V + 15) & ~(size_t)15));
        const int32_t nch = (V + 63) >> 6;
        for (int32_t v = (int32_t)threadIdx.x; v < V; v += BLOCK) off16[v] = (uint16_t)(arc_off[v] - arc_off[v & ~63]);
        for (int32_t cix = (int32_t)threadIdx.x; cix <= nch; cix += BLOCK) cbase[cix] = arc_off[cix < nch ? cix << 6 : V];
        __syncthreads();
    }
#ifdef SHD_SSSP_FLAT
    __shared__ int32_t fl_pre[BLOCK], fl_beg[BLOCK];
    __shared__ uint64_t fl_dv[BLOCK];
#else
    int32_t *fl_pre = nullptr, *fl_beg = nullptr;
    uint64_t* fl_dv = nullptr;
#endif
    // row_list: the second pass over listed rows [row0, row1) of it, parents from fpar
    for (int32_t i = row0 + (int32_t)blockIdx.x; i < row1; i += gridDim.x) {
        const int32_t row = row_list ? row_list[i] : i;
        int bf_it = -1;
        if (gdist && gok[i - row0]) {   // (0.0 - value: +0.0 at the source, as the Bellman-Ford's)
            const size_t r = (size_t)(i - row0) * V;
            for (int32_t v = (int32_t)threadIdx.x; v < V; v += BLOCK) {
                uint64_t d = kDistInf;
                if (gkind == 4) {
                    const TieG<int32_t> e = ((const TieG<int32_t>*)gdist)[r + v];
                    if (e.st == 2u) d = d2u(0.0 - (double)e.negd);
                } else {
                    const TieG<double> e = ((const TieG<double>*)gdist)[r + v];
                    if (e.st == 2u) d = d2u(0.0 - e.negd);
                }
                dist[v] = d;
            }
            bf_it = 0;
            __syncthreads();
        }
        sssp_one_row<BLOCK>(row, attached[row], V, T, arc_off, arc_dst, arc_w, arc_src, arc_rin, rin_off, rin_src,
                            rin_eid,
                            rin_w, rin_r, w_e, eloss, vloss, attached, self_eid, out, stats, dist,
                            parent, upd, flags, fpar ? fpar + (size_t)(i - row0) * V : nullptr, tie_rows, fl_pre,
                            fl_beg, fl_dv, off16, cbase, (mode & 2) != 0, bf_it, fpar && i - row0 >= cnt_from);
    }
}

// ---- two rows per workgroup (k_sssp_rows2_lds, the default where both
// rows' distances fit the LDS: 10 080 vertices).  A row's Bellman-Ford is a
// chain of ~50 dependent frontier iterations, each the slowest wave's chunk
// scan and relaxations and a workgroup barrier: latency, not throughput.  Two
// rows in one loop give every wave two independent chains between the same
// barriers.  Their distances fill the LDS (8 B a vertex each), so the 16-bit
// stamps give way to one bit a vertex per row: a relaxation that improves x
// sets x's bit (an LDS atomic or); right after the barrier each wave takes
// (atomic exchange with 0) the bit words of its own chunks, one word per lane,
// and relaxes the vertices they name.  A bit set in an iteration after its
// word was taken waits for the next one (as the stamps did); one set before
// (a faster wave's relaxation) is taken at once -- any order reaches the same
// fixpoint (fl(a + w) is monotone), and a vertex still relaxes once per
// improvement.  The rows' properties then run one at a time through
// sssp_one_row's phases (bf_it), row B's distances parked in global scratch.
template <int BLOCK, int NCH>
__device__ void sssp_bf2(int32_t srcA, int32_t srcB /* -1: none */, int32_t V, const int32_t* __restrict__ arc_off,
                         const int32_t* __restrict__ arc_dst, const double* __restrict__ arc_w, uint64_t* dA,
                         uint64_t* dB, uint32_t* bA, uint32_t* bB /* [ceil(V / 32)] each */,
                         int* flags /* LDS int[8]: A's at 0..2, B's at 4..6 */, int* itA, int* itB) {
    constexpr int NW = BLOCK / 64;
    static_assert(2 * NCH <= 32, "a wave's bit words of both rows in one lane each");
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hl = lane & 31;
    const bool upper = lane >= 32;
    const int32_t nw32 = (V + 31) >> 5;
    for (int32_t v = tid; v < V; v += BLOCK) { dA[v] = kDistInf; dB[v] = kDistInf; }
    for (int32_t k = tid; k < nw32; k += BLOCK) { bA[k] = 0; bB[k] = 0; }
    if (tid < 8) flags[tid] = 0;
    __syncthreads();
    if (tid == 0) {
        dA[srcA] = 0;
        bA[srcA >> 5] = 1u << (srcA & 31);
        if (srcB >= 0) {
            dB[srcB] = 0;
            bB[srcB >> 5] = 1u << (srcB & 31);
        }
    }
    __syncthreads();
    bool liveA = true, liveB = srcB >= 0;
    int it = 0;
    *itA = 0;
    *itB = 0;
    for (;;) {
        if (tid == 0) { flags[(it + 1) % 3] = 0; flags[4 + (it + 1) % 3] = 0; }
        // the wave's bit words: lane 2c + h holds row A's word h of chunk c,
        // lane 32 + 2c + h row B's
        uint32_t wbits = 0;
        {
            const int r = lane >> 5, j = lane & 31, c = j >> 1;
            const int32_t k = (wv + c * NW) * 2 + (j & 1);   // word index: chunk (wv + c NW), half j & 1
            if (j < 2 * NCH && k < nw32 && (r == 0 ? liveA : liveB)) wbits = atomicExch(r == 0 ? &bA[k] : &bB[k], 0u);
        }
        constexpr int Q = SHD_SSSP_BFQ2;
        int32_t qa[2 * Q], qb[2 * Q];
#pragma unroll
        for (int j = 0; j < 2 * Q; j++) { qa[j] = -1; qb[j] = -1; }
        int na = 0, nb = 0;
        auto relax = [&](uint64_t* d, uint32_t* b, int* fl, int32_t x, double cand) {
            const uint64_t nbv = d2u(cand);
            if (nbv < d[x]) {
                const uint64_t old = atomicMin((unsigned long long*)&d[x], (unsigned long long)nbv);
                if (nbv < old) {
                    atomicOr(&b[x >> 5], 1u << (x & 31));
                    fl[it % 3] = 1;
                }
            }
        };
        auto run_q = [&](uint64_t* d, uint32_t* b, int* fl, int32_t (&q)[2 * Q]) {
            int32_t bq[Q], eq[Q], xq[Q];
            double dq[Q], wq[Q];
#pragma unroll
            for (int j = 0; j < Q; j++) {
                const int32_t v = upper ? q[2 * j + 1] : q[2 * j];
                bq[j] = 0; eq[j] = 0; dq[j] = 0.0;
                if (v >= 0 && v < V) { bq[j] = arc_off[v]; eq[j] = arc_off[v + 1]; dq[j] = u2d(d[v]); }
            }
#pragma unroll
            for (int j = 0; j < Q; j++) {
                const int32_t k = bq[j] + hl;
                xq[j] = -1; wq[j] = 0.0;
                if (k < eq[j]) { xq[j] = arc_dst[k]; wq[j] = arc_w[k]; }
            }
#pragma unroll
            for (int j = 0; j < Q; j++)
                if (xq[j] >= 0) relax(d, b, fl, xq[j], dq[j] + wq[j]);
#pragma unroll
            for (int j = 0; j < Q; j++)
                for (int32_t k = bq[j] + hl + 32; k < eq[j]; k += 32) relax(d, b, fl, arc_dst[k], dq[j] + arc_w[k]);
        };
        auto push = [&](int32_t (&q)[2 * Q], int32_t fv) {
#pragma unroll
            for (int j = 0; j < 2 * Q - 1; j++) q[j] = q[j + 1];
            q[2 * Q - 1] = fv;
        };
#if SHD_SSSP_MIXQ
        // one queue for both rows (an entry: the vertex | row << 30): a
        // half-wave's vertex of row A and the other's of row B relax together,
        // both rows' loads in flight at once
        int32_t qm[2 * Q];
#pragma unroll
        for (int j = 0; j < 2 * Q; j++) qm[j] = -1;
        int nm = 0;
        auto run_qm = [&]() {
            int32_t bq[Q], eq[Q], xq[Q], rq[Q];
            double dq[Q], wq[Q];
#pragma unroll
            for (int j = 0; j < Q; j++) {
                const int32_t e = upper ? qm[2 * j + 1] : qm[2 * j];
                const int32_t v = e & 0x3FFFFFFF;
                rq[j] = e >= 0 ? (e >> 30) : 0;
                bq[j] = 0; eq[j] = 0; dq[j] = 0.0;
                if (e >= 0 && v < V) {
                    bq[j] = arc_off[v]; eq[j] = arc_off[v + 1];
                    dq[j] = u2d(rq[j] ? dB[v] : dA[v]);
                }
            }
#pragma unroll
            for (int j = 0; j < Q; j++) {
                const int32_t k = bq[j] + hl;
                xq[j] = -1; wq[j] = 0.0;
                if (k < eq[j]) { xq[j] = arc_dst[k]; wq[j] = arc_w[k]; }
            }
#pragma unroll
            for (int j = 0; j < Q; j++)
                if (xq[j] >= 0) relax(rq[j] ? dB : dA, rq[j] ? bB : bA, rq[j] ? flags + 4 : flags, xq[j], dq[j] + wq[j]);
#pragma unroll
            for (int j = 0; j < Q; j++)
                for (int32_t k = bq[j] + hl + 32; k < eq[j]; k += 32)
                    relax(rq[j] ? dB : dA, rq[j] ? bB : bA, rq[j] ? flags + 4 : flags, arc_dst[k], dq[j] + arc_w[k]);
        };
        (void)na; (void)nb; (void)run_q;
#endif
#if SHD_SSSP_BALLOT && !SHD_SSSP_MIXQ
        {   // the wave's non-empty words, lane by lane: row A's (lanes 0-19) then row B's (32-51);
            // any order reaches the same fixpoint (as the bits taken early above)
            uint64_t nz = __ballot(wbits != 0u);
            while (nz) {
                const int ln = __ffsll((unsigned long long)nz) - 1;
                nz &= nz - 1;
                uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)wbits, ln);
                const int j = ln & 31;
                const int32_t base = (wv + (j >> 1) * NW) * 64 + (j & 1) * 32;
                if (ln < 32) {
                    while (m) {
                        push(qa, base + __builtin_ctz(m));
                        m &= m - 1;
                        if (++na == 2 * Q) { run_q(dA, bA, flags, qa); na = 0; }
                    }
                } else {
                    while (m) {
                        push(qb, base + __builtin_ctz(m));
                        m &= m - 1;
                        if (++nb == 2 * Q) { run_q(dB, bB, flags + 4, qb); nb = 0; }
                    }
                }
            }
        }
#else
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            const int32_t c0 = (wv + c * NW) * 64;
            uint64_t mA = (uint64_t)(uint32_t)__shfl((int)wbits, 2 * c) |
                          ((uint64_t)(uint32_t)__shfl((int)wbits, 2 * c + 1) << 32);
            uint64_t mB = (uint64_t)(uint32_t)__shfl((int)wbits, 32 + 2 * c) |
                          ((uint64_t)(uint32_t)__shfl((int)wbits, 32 + 2 * c + 1) << 32);
            // (uniform; each half widened from uint32_t: an int would sign-extend)
            mA = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)mA) |
                 ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(mA >> 32)) << 32);
            mB = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)mB) |
                 ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(mB >> 32)) << 32);
#if SHD_SSSP_MIXQ
            while (mA | mB) {
                int32_t fv;
                if (mA) {
                    fv = c0 + __ffsll((unsigned long long)mA) - 1;
                    mA &= mA - 1;
                } else {
                    fv = (c0 + __ffsll((unsigned long long)mB) - 1) | (1 << 30);
                    mB &= mB - 1;
                }
                push(qm, fv);
                if (++nm == 2 * Q) { run_qm(); nm = 0; }
            }
        }
        if (nm) {
            while (nm < 2 * Q) { push(qm, -1); nm++; }
            run_qm();
        }
#else
            while (mA) {
                const int32_t fv = c0 + __ffsll((unsigned long long)mA) - 1;
                mA &= mA - 1;
                push(qa, fv);
                if (++na == 2 * Q) { run_q(dA, bA, flags, qa); na = 0; }
            }
            while (mB) {
                const int32_t fv = c0 + __ffsll((unsigned long long)mB) - 1;
                mB &= mB - 1;
                push(qb, fv);
                if (++nb == 2 * Q) { run_q(dB, bB, flags + 4, qb); nb = 0; }
            }
        }
#endif
#endif
#if !SHD_SSSP_MIXQ
        if (na) {
            while (na < 2 * Q) { push(qa, -1); na++; }
            run_q(dA, bA, flags, qa);
        }
        if (nb) {
            while (nb < 2 * Q) { push(qb, -1); nb++; }
            run_q(dB, bB, flags + 4, qb);
        }
#endif
        __syncthreads();
        const bool moreA = liveA && flags[it % 3] != 0, moreB = liveB && flags[4 + it % 3] != 0;
        it++;
        if (liveA && !moreA) *itA = it;
        if (liveB && !moreB) *itB = it;
        liveA = moreA;
        liveB = moreB;
        if ((!liveA && !liveB) || it >= 0xFFFE) break;
    }
}

// a row's properties after sssp_bf2 (sssp_one_row's phases from its parents on)
template <int BLOCK>
__device__ __forceinline__ void sssp_post_row(
    int32_t row, int32_t V, int32_t T, const int32_t* __restrict__ arc_off, const int32_t* __restrict__ arc_dst,
    const double* __restrict__ arc_w, const int32_t* __restrict__ arc_src, const int32_t* __restrict__ arc_rin,
    const int32_t* __restrict__ rin_off, const int32_t* __restrict__ rin_src, const int32_t* __restrict__ rin_eid,
    const double* __restrict__ rin_w, const double* __restrict__ rin_r, const double* __restrict__ w_e,
    const double* __restrict__ eloss, const double* __restrict__ vloss, const int32_t* __restrict__ attached,
    const int32_t* __restrict__ self_eid, shd_pv* __restrict__ out, int64_t* __restrict__ stats, uint64_t* dist,
    int32_t* parent, uint16_t* upd, int* flags, int32_t* __restrict__ tie_rows, int bf_it) {
    sssp_one_row<BLOCK>(row, attached[row], V, T, arc_off, arc_dst, arc_w, arc_src, arc_rin, rin_off, rin_src, rin_eid,
                        rin_w, rin_r, w_e, eloss, vloss, attached, self_eid, out, stats, dist, parent, upd, flags,
                        nullptr, tie_rows, nullptr, nullptr, nullptr, nullptr, nullptr, false, bf_it);
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_sssp_rows2_lds(
    int32_t V, int32_t T, const int32_t* __restrict__ arc_off, const int32_t* __restrict__ arc_dst,
    const double* __restrict__ arc_w, const int32_t* __restrict__ arc_src, const int32_t* __restrict__ arc_rin,
    const int32_t* __restrict__ rin_off,
    const int32_t* __restrict__ rin_src, const int32_t* __restrict__ rin_eid,
    const double* __restrict__ rin_w, const double* __restrict__ rin_r, const double* __restrict__ w_e,
    const double* __restrict__ eloss,
    const double* __restrict__ vloss, const int32_t* __restrict__ attached,
    const int32_t* __restrict__ self_eid, shd_pv* __restrict__ out,
    int64_t* __restrict__ stats, int32_t row0, int32_t row1, int32_t* __restrict__ tie_rows,
    uint64_t* __restrict__ park /* [grid][V]: row B's distances while row A's properties run */) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint64_t* rA = (uint64_t*)smem;
    uint64_t* rB = (uint64_t*)(smem + (size_t)8 * V);
    const size_t nbw = (size_t)((V + 31) >> 5);
    uint32_t* bA = (uint32_t*)(smem + (size_t)16 * V);
    uint32_t* bB = bA + nbw;
    int* flags = (int*)(bB + nbw);
    uint64_t* pk = park + (size_t)blockIdx.x * V;
    const int tid = threadIdx.x;
    for (int32_t p = row0 + 2 * (int32_t)blockIdx.x; p < row1; p += 2 * (int32_t)gridDim.x) {
        const int32_t ra = p, rb = p + 1 < row1 ? p + 1 : -1;
        int itA = 0, itB = 0;
        sssp_bf2<BLOCK, 10>(attached[ra], rb >= 0 ? attached[rb] : -1, V, arc_off, arc_dst, arc_w, rA, rB, bA, bB,
                            flags, &itA, &itB);
        if (rb >= 0)
            for (int32_t v = tid; v < V; v += BLOCK) pk[v] = rB[v];
        __syncthreads();
        // row A: its distances in rA, parents and stamps in rB's space
        sssp_post_row<BLOCK>(ra, V, T, arc_off, arc_dst, arc_w, arc_src, arc_rin, rin_off, rin_src, rin_eid, rin_w,
                             rin_r, w_e, eloss, vloss, attached, self_eid, out, stats, rA, (int32_t*)rB,
                             (uint16_t*)(smem + (size_t)12 * V), flags, tie_rows, itA);
        __syncthreads();
        if (rb < 0) continue;
        for (int32_t v = tid; v < V; v += BLOCK) rA[v] = pk[v];
        __syncthreads();
        sssp_post_row<BLOCK>(rb, V, T, arc_off, arc_dst, arc_w, arc_src, arc_rin, rin_off, rin_src, rin_eid, rin_w,
                             rin_r, w_e, eloss, vloss, attached, self_eid, out, stats, rA, (int32_t*)rB,
                             (uint16_t*)(smem + (size_t)12 * V), flags, tie_rows, itB);
        __syncthreads();
    }
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_sssp_rows_global(
    int32_t V, int32_t T, const int32_t* __restrict__ arc_off, const int32_t* __restrict__ arc_dst,
    const double* __restrict__ arc_w, const int32_t* __restrict__ arc_src, const int32_t* __restrict__ arc_rin,
    const int32_t* __restrict__ rin_off,
    const int32_t* __restrict__ rin_src, const int32_t* __restrict__ rin_eid,
    const double* __restrict__ rin_w, const double* __restrict__ rin_r, const double* __restrict__ w_e,
    const double* __restrict__ eloss,
    const double* __restrict__ vloss, const int32_t* __restrict__ attached,
    const int32_t* __restrict__ self_eid, shd_pv* __restrict__ out,
    int64_t* __restrict__ stats, char* __restrict__ scratch, size_t per_block, int32_t row0, int32_t row1,
    const int32_t* __restrict__ row_list, const int32_t* __restrict__ fpar, int32_t* __restrict__ tie_rows,
    int mode /* bit 1 queued */) {
    __shared__ int flags[4];
#ifdef SHD_SSSP_FLAT
    __shared__ int32_t fl_pre[BLOCK], fl_beg[BLOCK];
    __shared__ uint64_t fl_dv[BLOCK];
#else
    int32_t *fl_pre = nullptr, *fl_beg = nullptr;
    uint64_t* fl_dv = nullptr;
#endif
    char* base = scratch + per_block * blockIdx.x;
    uint64_t* dist = (uint64_t*)base;
    int32_t* parent = (int32_t*)(base + (size_t)8 * V);
    uint16_t* upd = (uint16_t*)(base + (size_t)12 * V);
    for (int32_t i = row0 + (int32_t)blockIdx.x; i < row1; i += gridDim.x) {
        const int32_t row = row_list ? row_list[i] : i;
        sssp_one_row<BLOCK>(row, attached[row], V, T, arc_off, arc_dst, arc_w, arc_src, arc_rin, rin_off, rin_src,
                            rin_eid,
                            rin_w, rin_r, w_e, eloss, vloss, attached, self_eid, out, stats, dist,
                            parent, upd, flags, fpar ? fpar + (size_t)(i - row0) * V : nullptr, tie_rows, fl_pre,
                            fl_beg, fl_dv, nullptr, nullptr, (mode & 2) != 0);
    }
}

// ------------------------------------------------------------------ tie rows
// igraph 0.7.1's igraph_get_shortest_paths_dijkstra, restated for the rows that
// have equal-cost predecessors (o_pathcache.c:156-202 is the oracle's copy):
// an indexed binary max-heap on -distance (igraph_2wheap_t), arcs relaxed in
// igraph_incident(OUT) order (the CSR keeps it; self-loops, which never
// improve a distance, are dropped), the first finite distance or a strictly
// shorter one setting the parent.  So a vertex's parent is its first exact
// predecessor in relaxation order, and among predecessors at one distance that
// order is the heap's.  Every row runs to an empty heap (igraph stops once
// every target is popped; the parents on a target's path are final by then
// either way).  One lane per row, kTieLanes rows per wave (a wave per 16 rows:
// more waves in flight for a latency-bound walk, less divergence per wave);
// the lane's dist and heap live in global scratch with the lane as the
// fastest index, so the heap's top levels, which every lane walks, share lines.  Sifts move a hole instead
// of swapping: the same final arrangement as igraph_2wheap_switch steps.
struct TieLane {
    double* dist;      // [V] lane-strided, -1 = unreached
    double* hdat;      // [V] heap values (-distance)
    int32_t* hidx;     // [V] heap position -> vertex
    int32_t* hidx2;    // [V] vertex -> heap position + 2
};
constexpr int kTieLanes = 16;
#define TL(p, i) (p)[(size_t)(i) * kTieLanes]

__device__ __forceinline__ void tie_shift_up(TieLane& h, int32_t elem, double val, int32_t id) {
    while (elem != 0) {
        const int32_t par = (elem + 1) / 2 - 1;
        const double pv = TL(h.hdat, par);
        if (val < pv) break;   // igraph_2wheap_shift_up: stop at the top or below a larger parent
        const int32_t pid = TL(h.hidx, par);
        TL(h.hdat, elem) = pv;
        TL(h.hidx, elem) = pid;
        TL(h.hidx2, pid) = elem + 2;
        elem = par;
    }
    TL(h.hdat, elem) = val;
    TL(h.hidx, elem) = id;
    TL(h.hidx2, id) = elem + 2;
}

// igraph_2wheap_sink from `head` holding (val, id); returns its final position
__device__ __forceinline__ int32_t tie_sink(TieLane& h, int32_t size, int32_t head, double val, int32_t id) {
    for (;;) {
        const int32_t l = 2 * head + 1, r = 2 * head + 2;
        if (l >= size) break;
        const double dl = TL(h.hdat, l);
        int32_t c = l;
        double dc = dl;
        if (r != size) {
            const double dr = TL(h.hdat, r);
            if (!(dl >= dr)) { c = r; dc = dr; }
        }
        if (!(val < dc)) break;
        const int32_t cid = TL(h.hidx, c);
        TL(h.hdat, head) = dc;
        TL(h.hidx, head) = cid;
        TL(h.hidx2, cid) = head + 2;
        head = c;
    }
    TL(h.hdat, head) = val;
    TL(h.hidx, head) = id;
    TL(h.hidx2, id) = head + 2;
    return head;
}

__global__ __launch_bounds__(kTieLanes) void k_sssp_tie_parents(
    int32_t V, int32_t n, const int32_t* __restrict__ rows, const int32_t* __restrict__ attached,
    const int32_t* __restrict__ arc_off, const int32_t* __restrict__ arc_dst, const double* __restrict__ arc_w,
    const int32_t* __restrict__ arc_rin, int32_t* __restrict__ fpar, char* __restrict__ scratch,
    const int32_t* __restrict__ slots) {   // slots: the chunk's slots to run (null: [0, n))
    const int32_t i = (int32_t)blockIdx.x * kTieLanes + (int32_t)threadIdx.x;
    if (i >= n) return;
    const int32_t slot = slots ? slots[i] : i;
    char* wbase = scratch + (size_t)blockIdx.x * kTieLanes * (size_t)V * 24;
    TieLane h;
    h.dist = (double*)wbase + threadIdx.x;
    h.hdat = (double*)(wbase + (size_t)kTieLanes * V * 8) + threadIdx.x;
    h.hidx = (int32_t*)(wbase + (size_t)kTieLanes * V * 16) + threadIdx.x;
    h.hidx2 = (int32_t*)(wbase + (size_t)kTieLanes * V * 20) + threadIdx.x;
    int32_t* par = fpar + (size_t)slot * V;
    for (int32_t v = 0; v < V; v++) {
        TL(h.dist, v) = -1.0;
        par[v] = -1;
    }
    const int32_t src = attached[rows[slot]];
    TL(h.dist, src) = 0.0;
    int32_t size = 1;
    TL(h.hdat, 0) = 0.0;
    TL(h.hidx, 0) = src;
    TL(h.hidx2, src) = 2;
    while (size > 0) {
        // igraph_2wheap_max_index + igraph_2wheap_delete_max
        const int32_t u = TL(h.hidx, 0);
        const double mindist = -TL(h.hdat, 0);
        size--;
        if (size > 0) (void)tie_sink(h, size, 0, TL(h.hdat, size), TL(h.hidx, size));
        const int32_t kb = arc_off[u], ke = arc_off[u + 1];
        for (int32_t k = kb; k < ke; k++) {
            const int32_t x = arc_dst[k];
            const double alt = mindist + arc_w[k];
            const double cur = TL(h.dist, x);
            if (cur < 0) {                 // the first finite distance: push
                TL(h.dist, x) = alt;
                par[x] = arc_rin[k];
                tie_shift_up(h, size, -alt, x);
                size++;
            } else if (alt < cur) {        // strictly shorter: igraph_2wheap_modify
                TL(h.dist, x) = alt;
                par[x] = arc_rin[k];
                // data[pos] = -alt; sink(pos); shift_up(pos) -- the shift starts at
                // pos again, with whatever the sink left there (the element itself:
                // a larger value never sinks)
                const int32_t pos = TL(h.hidx2, x) - 2;
                (void)tie_sink(h, size, pos, -alt, x);
                tie_shift_up(h, pos, TL(h.hdat, pos), TL(h.hidx, pos));
            }
        }
    }
}
#undef TL

// The same Dijkstra, one row per one-wave block with the row's state in LDS
// (round 6: k_sssp_tie_parents' lane heaps in global scratch -- 240 KB a row at
// 10 k vertices, every tied row in flight at once -- made each of a row's ~35
// dependent heap steps per pop an HBM round trip: 490 ms for the 10 k
// all-tied build).  Here the row keeps
//   st[V]   uint16: 0 unreached, 1 popped, heap position + 2 (igraph's index2)
//   hv[hc]  the heap's values (-distance), hi[hc] its vertices (uint16)
// in LDS, and no distance array: an unreached vertex's is none, a heap
// member's is -hv[pos] (exact), and a popped vertex is never relaxed (alt =
// d(u) + w >= d(u) >= its distance: igraph's "strictly shorter" never holds).
// A pop's arcs are loaded by the wave's lanes at once, each with its target's
// state and value (only a target that an earlier arc of the same pop touched
// can have changed since -- the same vertex again, a parallel edge: re-read),
// and lane 0 runs the heap steps igraph takes, in arc order, only for the
// arcs that push or decrease.  A row whose heap outgrows hc is left to
// k_sssp_tie_parents (listed in ovf).  Same parents as k_sssp_tie_parents.
template <typename HV>
__device__ __forceinline__ void tlds_shift_up(HV* hv, uint16_t* hi, uint16_t* st, int32_t elem, HV val,
                                              int32_t id) {
    while (elem != 0) {
        const int32_t par = (elem + 1) / 2 - 1;
        const HV pv = hv[par];
        if (val < pv) break;
        const int32_t pid = hi[par];
        hv[elem] = pv;
        hi[elem] = (uint16_t)pid;
        st[pid] = (uint16_t)(elem + 2);
        elem = par;
    }
    hv[elem] = val;
    hi[elem] = (uint16_t)id;
    st[id] = (uint16_t)(elem + 2);
}
template <typename HV>
__device__ __forceinline__ void tlds_sink(HV* hv, uint16_t* hi, uint16_t* st, int32_t size, int32_t head, HV val,
                                          int32_t id) {
    for (;;) {
        const int32_t l = 2 * head + 1, r = 2 * head + 2;
        if (l >= size) break;
        const HV dl = hv[l];
        const HV dr = r != size ? hv[r] : (HV)0;
        const int32_t il = hi[l], ir = r != size ? hi[r] : 0;
        int32_t c = l, cid = il;
        HV dc = dl;
        if (r != size && !(dl >= dr)) { c = r; dc = dr; cid = ir; }
        if (!(val < dc)) break;
        hv[head] = dc;
        hi[head] = (uint16_t)cid;
        st[cid] = (uint16_t)(head + 2);
        head = c;
    }
    hv[head] = val;
    hi[head] = (uint16_t)id;
    st[id] = (uint16_t)(head + 2);
}
__device__ __forceinline__ double bcast_d(double v, int lane) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// (one wave per block: the lanes' LDS accesses are ordered by the wave's own
// instruction order, so no __syncthreads -- whose workgroup fence would drain
// every outstanding global store and load, the parents' stores and the next
// pop's arc loads, twice a pop -- only a compiler fence)
// STG (round 6): the vertex states in the block's slice of global scratch
// (L2-resident) instead of LDS, so LDS holds the heap only -- 10 KB a row at
// 1024 entries, 16 rows per CU against 5 with 20 KB of states beside it (10 k
// vertices).  Every state store is lane 0's; the other lanes read states only
// in the arcs' parallel loads, behind a workgroup-scope fence (a wait for lane
// 0's stores); lane 0 re-reads a state only for a decrease (its heap position
// moves with other vertices' steps) or a repeated target.
#define TIE_WAVE_SYNC()                                              \
    do {                                                             \
        if (STG) {                                                   \
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   \
            __builtin_amdgcn_wave_barrier();                         \
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   \
        } else {                                                     \
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
            __builtin_amdgcn_wave_barrier();                         \
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
        }                                                            \
    } while (0)
// HV: the heap's values (-distance): double, or int32_t where every arc weight
// is a whole number and V x the largest stays below 2^30 (shd_pc::w_int) --
// then every distance igraph's doubles hold is an exact integer of that range,
// the same order and ties, and a heap entry takes 6 B instead of 10
template <bool STG, typename HV>
__global__ __launch_bounds__(64) void k_sssp_tie_lds(
    int32_t V, int32_t n, const int32_t* __restrict__ rows, const int32_t* __restrict__ attached,
    const int32_t* __restrict__ arc_off, const int32_t* __restrict__ arc_dst, const double* __restrict__ arc_w,
    const int32_t* __restrict__ arc_rin, int32_t* __restrict__ fpar, int32_t hc, int32_t* __restrict__ ovf,
    uint16_t* __restrict__ stg) {
    extern __shared__ __align__(16) char tsm[];
    uint16_t* st = STG ? stg + (size_t)blockIdx.x * V : (uint16_t*)tsm;
    HV* hv = (HV*)(tsm + (STG ? 0 : (((size_t)2 * V + 15) & ~(size_t)15)));
    uint16_t* hi = (uint16_t*)(hv + hc);
    const int lane = (int)threadIdx.x;
    for (int32_t slot = (int32_t)blockIdx.x; slot < n; slot += (int32_t)gridDim.x) {
        int32_t* par = fpar + (size_t)slot * V;
        for (int32_t v = lane; v < V; v += 64) {
            st[v] = 0;
            par[v] = -1;
        }
        TIE_WAVE_SYNC();
        const int32_t src = attached[rows[slot]];
        int32_t size = 1;
        if (lane == 0) {
            hv[0] = (HV)0;
            hi[0] = (uint16_t)src;
            st[src] = 2;
        }
        int ovfl = 0;
        // the next pop's first chunk of arcs, loaded while lane 0 sinks: the
        // heap top after a pop's relaxations is the next pop's vertex
        int32_t pkb = arc_off[src], pke = arc_off[src + 1];
        int32_t px = -1, prin = 0;
        double pw = 0.0;
        if (pkb + lane < pke) {
            px = arc_dst[pkb + lane];
            pw = arc_w[pkb + lane];
            prin = arc_rin[pkb + lane];
        }
        while (size > 0 && !ovfl) {
            // the pop (igraph_2wheap_max_index + delete_max), by lane 0
            int32_t u0 = 0;
            double md0 = 0.0;
            if (lane == 0) {
                u0 = hi[0];
                md0 = -(double)hv[0];
                size--;
                if (size > 0) tlds_sink(hv, hi, st, size, 0, hv[size], hi[size]);
                st[u0] = 1;
            }
            const double md = bcast_d(md0, 0);
            size = __builtin_amdgcn_readfirstlane(size);
            TIE_WAVE_SYNC();
            const int32_t kb = pkb, ke = pke;
            int32_t top = -1;
            for (int32_t c0 = kb; c0 < ke && !ovfl; c0 += 64) {
                const int32_t k = c0 + lane;
                const bool valid = k < ke;
                int32_t x = -1, rin = 0;
                double w = 0.0;
                if (c0 == kb) { x = px; w = pw; rin = prin; }
                else if (valid) { x = arc_dst[k]; w = arc_w[k]; rin = arc_rin[k]; }
                const double alt = md + w;
                double cur = 0.0;
                uint32_t sx = 1;
                if (valid) {
                    sx = st[x];
                    if (sx >= 2) cur = -(double)hv[sx - 2];
                }
                const int32_t cnt = ke - c0 < 64 ? ke - c0 : 64;
                bool dup = false;   // an earlier arc of this chunk to the same vertex
                for (int32_t i = 0; i < cnt; i++) dup |= i < lane && __builtin_amdgcn_readlane(x, i) == x;
                uint64_t m = __ballot(valid && (dup || sx == 0 || (sx >= 2 && alt < cur)));
                const uint64_t mdup = STG ? __ballot(dup) : 0ull;
                if (lane == 0) {
                    while (m) {
                        const int j = __builtin_ctzll(m);
                        m &= m - 1;
                        const int32_t xj = __builtin_amdgcn_readlane(x, j);
                        const double aj = bcast_d(alt, j);
                        const int32_t rj = __builtin_amdgcn_readlane(rin, j);
                        // (STG: an unreached target of a first visit is still
                        // unreached -- no other arc of the chunk reaches it)
                        const uint32_t s0 = STG ? (uint32_t)__builtin_amdgcn_readlane((int)sx, j) : 1u;
                        const uint32_t sj = (STG && s0 == 0u && !((mdup >> j) & 1ull)) ? 0u : (uint32_t)st[xj];
                        if (sj == 0) {   // the first finite distance: push
                            if (size >= hc) { ovfl = 1; break; }
                            par[xj] = rj;
                            tlds_shift_up(hv, hi, st, size, (HV)(-aj), xj);
                            size++;
                        } else if (sj >= 2) {   // strictly shorter: igraph_2wheap_modify
                            const int32_t pos = (int32_t)sj - 2;
                            if (aj < -(double)hv[pos]) {
                                par[xj] = rj;
                                tlds_sink(hv, hi, st, size, pos, (HV)(-aj), xj);
                                tlds_shift_up(hv, hi, st, pos, hv[pos], hi[pos]);
                            }
                        }
                    }
                }
                size = __builtin_amdgcn_readfirstlane(size);
                ovfl = __builtin_amdgcn_readfirstlane(ovfl);
                TIE_WAVE_SYNC();
            }
            // the next pop's vertex (the top now) and its first chunk of arcs,
            // issued before its sink
            int32_t t0 = -1;
            if (lane == 0 && size > 0) t0 = hi[0];
            top = __builtin_amdgcn_readfirstlane(t0);
            if (top >= 0 && !ovfl) {
                pkb = arc_off[top];
                pke = arc_off[top + 1];
                px = -1;
                if (pkb + lane < pke) {
                    px = arc_dst[pkb + lane];
                    pw = arc_w[pkb + lane];
                    prin = arc_rin[pkb + lane];
                }
            }
        }
        if (ovfl && lane == 0) ovf[1 + atomicAdd(ovf, 1)] = slot;
        TIE_WAVE_SYNC();
    }
}
#undef TIE_WAVE_SYNC

// The same Dijkstra with no vertex -> heap position map at all (round 6,
// SHD_PC_TIE_KIND=g; k_sssp_tie_lds<true> kept that map in global scratch and
// stored a vertex's new position at every step of every sift, then waited for
// those stores before the next pop's arcs could read it).  Per vertex, in the
// block's slice of global scratch, only what changes at a push or a decrease:
// its state (0 unreached, 2 reached) and its heap value (-distance).  A popped
// vertex keeps state 2 and its final value: an arc from the popped vertex u
// (d(u) >= every popped distance) gives alt = d(u) + w >= that value, never
// igraph's "strictly shorter", exactly as the popped state did.  So the sifts
// touch LDS only, a pop's arcs and their targets' entries are loaded before
// the pop's sink (nothing in them changes at a pop), and a decrease finds its
// vertex's heap position by a search of the heap's vertex array by the whole
// wave (<= hc / 64 LDS reads a lane).  Same parents as k_sssp_tie_lds.
// (a level's reads go out together -- both children's values and vertices,
// the right child's even where it is past the end: k_sssp_tie_g holds at most
// hc - 1 entries, so that slot is still the heap's -- so a level costs one LDS
// round trip, not three)
// (dz: a zero the compiler cannot see through -- a VGPR from inline asm -- so
// that the index arithmetic of lane 0's sifts stays in VALU instead of being
// scalarized: the one scalar unit of a CU serialised the sifts of all 26
// rows on it (SQ_ACTIVE_INST_SCA ~ 68 % of the CU's cycles, profiles/r06/tiepmc))
__device__ __forceinline__ int32_t tg_vzero() {
    int32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}
template <typename HV>
__device__ __forceinline__ void tg_shift_up(HV* hv, uint16_t* hi, int32_t elem, HV val, int32_t id) {
    while (elem != 0) {
        const int32_t par = (elem + 1) / 2 - 1;
        const HV pv = hv[par];
        const uint16_t pid = hi[par];
        if (val < pv) break;
        hv[elem] = pv;
        hi[elem] = pid;
        elem = par;
    }
    hv[elem] = val;
    hi[elem] = (uint16_t)id;
}
template <typename HV>
__device__ __forceinline__ void tg_sink(HV* hv, uint16_t* hi, int32_t size, int32_t head, HV val, int32_t id) {
    for (;;) {
        const int32_t l = 2 * head + 1, r = 2 * head + 2;
        if (l >= size) break;
        const HV dl = hv[l], dr = hv[r];
        const uint16_t il = hi[l], ir = hi[r];
        const bool right = r != size && !(dl >= dr);
        const int32_t c = right ? r : l;
        const HV dc = right ? dr : dl;
        if (!(val < dc)) break;
        hv[head] = dc;
        hi[head] = right ? ir : il;
        head = c;
    }
    hv[head] = val;
    hi[head] = (uint16_t)id;
}
// The same sifts for VH: the index arithmetic in VALU (the positions come in
// derived from tg_vzero), and every exit test made uniform by reading lane 0's
// outcome into a scalar (readfirstlane) -- a divergent loop would spend as
// many scalar instructions on its exec masks as the scalarized one spends on
// the arithmetic
template <typename HV>
__device__ __forceinline__ void tg_shift_up_v(HV* hv, uint16_t* hi, int32_t elem, HV val, int32_t id) {
    for (;;) {
        if (!__builtin_amdgcn_readfirstlane((int)(elem != 0))) break;
        const int32_t par = (elem + 1) / 2 - 1;
        const HV pv = hv[par];
        const uint16_t pid = hi[par];
        if (__builtin_amdgcn_readfirstlane((int)(val < pv))) break;
        hv[elem] = pv;
        hi[elem] = pid;
        elem = par;
    }
    hv[elem] = val;
    hi[elem] = (uint16_t)id;
}
template <typename HV>
__device__ __forceinline__ void tg_sink_v(HV* hv, uint16_t* hi, int32_t size, int32_t head, HV val, int32_t id) {
    for (;;) {
        const int32_t l = 2 * head + 1, r = 2 * head + 2;
        if (!__builtin_amdgcn_readfirstlane((int)(l < size))) break;
        const HV dl = hv[l], dr = hv[r];
        const uint16_t il = hi[l], ir = hi[r];
        const bool right = r != size && !(dl >= dr);
        const HV dc = right ? dr : dl;
        if (!__builtin_amdgcn_readfirstlane((int)(val < dc))) break;
        hv[head] = dc;
        hi[head] = right ? ir : il;
        head = right ? r : l;
    }
    hv[head] = val;
    hi[head] = (uint16_t)id;
}
template <typename HV>
__device__ __forceinline__ TieG<HV> tg_load(const TieG<HV>* g, int32_t x) {
    return g[x];
}
#define TG_WG_SYNC()                                             \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   \
        __builtin_amdgcn_wave_barrier();                         \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   \
    } while (0)
#define TG_WAVE_SYNC()                                           \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
    } while (0)
__global__ void k_iota(int32_t* __restrict__ out, int32_t n, int32_t base) {
    const int32_t k = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k < n) out[k] = base + k;
}
// per arc: does an earlier arc of its source's list, in the same 64-arc chunk
// (chunks from the list's start), go to the same vertex (a parallel edge the
// tie kernel's chunk must take in order); computed once per tied build
__global__ void k_arc_dup(int32_t na, const int32_t* __restrict__ arc_off, const int32_t* __restrict__ arc_src,
                          const int32_t* __restrict__ arc_dst, uint8_t* __restrict__ dup) {
    const int32_t k = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (k >= na) return;
    const int32_t kb = arc_off[arc_src[k]];
    const int32_t c0 = kb + ((k - kb) & ~63);
    const int32_t x = arc_dst[k];
    uint8_t d = 0;
    for (int32_t j = c0; j < k; j++) d |= arc_dst[j] == x ? 1 : 0;
    dup[k] = d;
}
template <typename HV, bool VH>
__global__ __launch_bounds__(64) void k_sssp_tie_g(
    int32_t V, int32_t n, const int32_t* __restrict__ rows, const int32_t* __restrict__ attached,
    const int32_t* __restrict__ arc_off, const int32_t* __restrict__ arc_dst, const double* __restrict__ arc_w,
    const int32_t* __restrict__ arc_rin, int32_t* __restrict__ fpar, int32_t hc, int32_t* __restrict__ ovf,
    TieG<HV>* __restrict__ gsc, const uint8_t* __restrict__ arc_dup, uint8_t* __restrict__ gok) {
    // gsc: V entries per ROW of the chunk (they are the row's distances for the
    // second pass, k_sssp_rows_lds's gdist); gok[slot]: the row ran to its end
    extern __shared__ __align__(16) char tsm[];
    HV* hv = (HV*)tsm;
    uint16_t* hi = (uint16_t*)(hv + hc);
    const int lane = (int)threadIdx.x;
    for (int32_t slot = (int32_t)blockIdx.x; slot < n; slot += (int32_t)gridDim.x) {
        int32_t* par = fpar + (size_t)slot * V;
        TieG<HV>* g = gsc + (size_t)slot * V;
        for (int32_t v = lane; v < V; v += 64) {
            g[v].st = 0u;
            par[v] = -1;
        }
        const int32_t src = attached[rows[slot]];
        int32_t size = 1;
        if (lane == 0) {
            hv[0] = (HV)0;
            hi[0] = (uint16_t)src;
        }
        TG_WG_SYNC();
        if (lane == 0) g[src] = TieG<HV>{(HV)0, 2u};
        TG_WG_SYNC();
        int ovfl = 0;
        // the next pop's first chunk of arcs and their targets' entries
        int32_t pkb = arc_off[src], pke = arc_off[src + 1];
        int32_t px = -1, prin = 0, pdup = 0;
        double pw = 0.0;
        TieG<HV> pg{(HV)0, 1u};
        if (pkb + lane < pke) {
            px = arc_dst[pkb + lane];
            pw = arc_w[pkb + lane];
            prin = arc_rin[pkb + lane];
            pdup = arc_dup[pkb + lane];
            pg = tg_load(g, px);
        }
        while (size > 0 && !ovfl) {
            // the pop (igraph_2wheap_max_index + delete_max), by lane 0
            double md0 = 0.0;
            if (lane == 0) {
                md0 = -(double)hv[0];
                size--;
                const int32_t dz = VH ? tg_vzero() : 0;
                if (size > 0) {
                    if (VH) tg_sink_v(hv, hi, size, dz, hv[size + dz], (int32_t)hi[size + dz]);
                    else tg_sink(hv, hi, size, 0, hv[size], (int32_t)hi[size]);
                }
            }
            const double md = bcast_d(md0, 0);
            size = __builtin_amdgcn_readfirstlane(size);
            TG_WAVE_SYNC();
            const int32_t kb = pkb, ke = pke;
            // (every chunk's arcs and entries come through the same registers, p*: a
            // later chunk's are loaded after the previous chunk's stores, as the next
            // pop's are -- one set of load targets, so no wait for them lands in the
            // sifts)
            for (int32_t c0 = kb; c0 < ke && !ovfl; c0 += 64) {
                if (c0 != kb && c0 + lane < ke) {   // a later chunk's, after the previous chunk's stores
                    const int32_t k = c0 + lane;
                    px = arc_dst[k];
                    pw = arc_w[k];
                    prin = arc_rin[k];
                    pdup = arc_dup[k];
                    pg = tg_load(g, px);
                }
                const bool valid = c0 + lane < ke;
                const int32_t x = px, rin = prin, xd = pdup;
                const double w = pw;
                const TieG<HV> gx = pg;
                const double alt = md + w;
                const bool dup = valid && xd != 0;   // an earlier arc of this chunk to the same vertex (k_arc_dup)
                uint64_t m = __ballot(valid && (dup || gx.st == 0u || (gx.st == 2u && alt < -(double)gx.negd)));
                const uint64_t mdup = __ballot(dup);
                // the entry's words copied out of the load's target registers (an asm
                // move), so that reading them in the loop below waits for nothing --
                // a wait there would also wait for the loop's own stores
                uint32_t gst, gng;
                {
                    const uint32_t s0 = gx.st;
                    uint32_t n0;
                    if (sizeof(HV) == 4) n0 = (uint32_t)(int32_t)gx.negd; else n0 = 0u;
                    asm volatile("v_mov_b32 %0, %1" : "=v"(gst) : "v"(s0));
                    asm volatile("v_mov_b32 %0, %1" : "=v"(gng) : "v"(n0));
                }
                // every lane runs the candidates (uniform: m), lane 0 the heap steps
                while (m) {
                    const int j = __builtin_ctzll(m);
                    m &= m - 1;
                    const int32_t xj = __builtin_amdgcn_readlane(x, j);
                    const double aj = bcast_d(alt, j);
                    const int32_t rj = __builtin_amdgcn_readlane(rin, j);
                    uint32_t sj = (uint32_t)__builtin_amdgcn_readlane((int)gst, j);
                    double cj = -(double)(HV)0;
                    {
                        HV nj;
                        if (sizeof(HV) == 4) {
                            nj = (HV)(int32_t)__builtin_amdgcn_readlane((int)gng, j);
                        } else {
                            nj = (HV)bcast_d((double)gx.negd, j);
                        }
                        cj = -(double)nj;
                    }
                    if ((mdup >> j) & 1ull) {   // a target an earlier arc of this chunk changed: lane 0's own stores
                        uint32_t s0 = 0u;
                        double c0v = 0.0;
                        if (lane == 0) {
                            const TieG<HV> e = g[xj];
                            s0 = e.st;
                            c0v = -(double)e.negd;
                        }
                        sj = (uint32_t)__builtin_amdgcn_readfirstlane((int)s0);
                        cj = bcast_d(c0v, 0);
                    }
                    if (sj == 0u) {   // the first finite distance: push
                        if (size >= hc - 1) { ovfl = 1; break; }   // (hc - 1: tg_sink's read of a right child)
                        if (lane == 0) {
                            par[xj] = rj;
                            const int32_t dz = VH ? tg_vzero() : 0;
                            if (VH) tg_shift_up_v(hv, hi, size + dz, (HV)(-aj), xj);
                            else tg_shift_up(hv, hi, size, (HV)(-aj), xj);
                            g[xj] = TieG<HV>{(HV)(-aj), 2u};
                        }
                        size++;
                        TG_WAVE_SYNC();
                    } else if (aj < cj) {   // strictly shorter: igraph_2wheap_modify
                        // its heap position: the wave searches the heap's vertices
                        int32_t f = -1;
                        for (int32_t i = lane; i < size; i += 64)
                            if ((int32_t)hi[i] == xj) f = i;
                        const uint64_t fm = __ballot(f >= 0);
                        const int32_t pos = fm ? __builtin_amdgcn_readlane(f, __builtin_ctzll(fm)) : -1;
                        if (lane == 0 && pos >= 0) {
                            par[xj] = rj;
                            const int32_t dz = VH ? tg_vzero() : 0;
                            if (VH) {
                                tg_sink_v(hv, hi, size, pos + dz, (HV)(-aj), xj);
                                tg_shift_up_v(hv, hi, pos + dz, hv[pos + dz], (int32_t)hi[pos + dz]);
                            } else {
                                tg_sink(hv, hi, size, pos, (HV)(-aj), xj);
                                tg_shift_up(hv, hi, pos, hv[pos], (int32_t)hi[pos]);
                            }
                            g[xj].negd = (HV)(-aj);
                        }
                        if (pos < 0) ovfl = 2;   // (never: a reached vertex with a larger value is in the heap)
                        TG_WAVE_SYNC();
                    }
                }
                ovfl = __builtin_amdgcn_readfirstlane(ovfl);
                TG_WG_SYNC();   // the chunk's stores before the next loads of the entries
            }
            // the next pop's vertex (the top now), its first chunk of arcs and their
            // entries, issued before its sink
            int32_t t0 = -1;
            if (lane == 0 && size > 0) t0 = hi[0];
            const int32_t top = __builtin_amdgcn_readfirstlane(t0);
            if (top >= 0 && !ovfl) {
                pkb = arc_off[top];
                pke = arc_off[top + 1];
                // (no defaults for the lanes past the list: `valid` masks them, and a
                // register reset here would wait for every store of the pop first)
                if (pkb + lane < pke) {
                    px = arc_dst[pkb + lane];
                    pw = arc_w[pkb + lane];
                    prin = arc_rin[pkb + lane];
                    pdup = arc_dup[pkb + lane];
                    pg = tg_load(g, px);
                }
            }
        }
        if (ovfl && lane == 0) ovf[1 + atomicAdd(ovf, 1)] = slot;
        if (lane == 0) gok[slot] = ovfl ? 0 : 1;
        TG_WG_SYNC();
    }
}
#undef TG_WG_SYNC
#undef TG_WAVE_SYNC

// ------------------------------------------------------------------ direct
// _topology_lookupDirectPath (topology.c:1877-1927) for every attached pair;
// igraph_get_eid through the (neighbour, eid)-sorted lists (lowest parallel eid)
__device__ __forceinline__ int32_t dev_get_eid(const int32_t* nbr_off, const int32_t* nbr_v,
                                               const int32_t* nbr_eid, int32_t a, int32_t b) {
    int32_t lo = nbr_off[a], hi = nbr_off[a + 1];
    const int32_t end = hi;
    while (lo < hi) {
        int32_t mid = lo + ((hi - lo) >> 1);
        if (nbr_v[mid] < b) lo = mid + 1; else hi = mid;
    }
    return (lo < end && nbr_v[lo] == b) ? nbr_eid[lo] : -1;
}

__global__ void k_direct(int32_t T, const int32_t* __restrict__ attached, const int32_t* __restrict__ nbr_off,
                         const int32_t* __restrict__ nbr_v, const int32_t* __restrict__ nbr_eid,
                         const double* __restrict__ w_e, const double* __restrict__ eloss,
                         const double* __restrict__ vloss, shd_pv* __restrict__ out,
                         uint8_t* __restrict__ adj_out) {
    const size_t n = (size_t)T * T;
    for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n;
         idx += (size_t)gridDim.x * blockDim.x) {
        const int32_t i = (int32_t)(idx / T), j = (int32_t)(idx % T);
        const int32_t s = attached[i], d = attached[j];
        const int32_t e = dev_get_eid(nbr_off, nbr_v, nbr_eid, s, d);
        double lat = __longlong_as_double(0x7FF8000000000000ll), rel = lat;
        if (e >= 0) {
            double tl = 0.0, tr = 1.0, r;
            if (vrel(vloss, s, &r)) tr *= r;
            if (vrel(vloss, d, &r)) tr *= r;
            tl += w_e[e];
            tr *= ((double)1.0f - eloss[e]);
            lat = tl; rel = tr;
        }
        out[idx] = shd_pv{lat, rel};
        adj_out[idx] = e >= 0;
    }
}

// ------------------------------------------------------------------ self
// _topology_computeShortestPathToSelf (topology.c:1545-1653): first strict
// minimum over the igraph_incident(OUT) list; latency 2*min, reliability r^2
__global__ void k_self(int32_t T, const int32_t* __restrict__ attached, const int32_t* __restrict__ inc_off,
                       const int32_t* __restrict__ inc_eid, const double* __restrict__ w_e,
                       const double* __restrict__ eloss, shd_pv* __restrict__ out) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= T) return;
    const int32_t v = attached[i];
    double minLatency = 0.0f, relMin = 0.0f;
    const int32_t k0 = inc_off[v], k1 = inc_off[v + 1];
    for (int32_t k = k0; k < k1; k++) {
        const int32_t e = inc_eid[k];
        const double el = w_e[e];
        if (minLatency == 0 || el < minLatency) {
            minLatency = el;
            relMin = (double)1.0f - eloss[e];
        }
    }
    if (k1 == k0) { out[i] = shd_pv{-1.0, -1.0}; return; }
    out[i] = shd_pv{(double)2.0f * minLatency, relMin * relMin};
}

// min over valid (>= 0, non-NaN) latencies of a table -> stats[5] as u64 bits
__global__ void k_min_latency(const shd_pv* __restrict__ a, size_t n, int64_t* __restrict__ stats) {
    __shared__ unsigned long long smin[256];
    unsigned long long m = kDistInf;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double v = a[i].lat;
        if (v >= 0.0) { unsigned long long b = (unsigned long long)__double_as_longlong(v); if (b < m) m = b; }
    }
    smin[threadIdx.x] = m;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s && smin[threadIdx.x + s] < smin[threadIdx.x]) smin[threadIdx.x] = smin[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMin((unsigned long long*)&stats[5], smin[0]);
}

// ------------------------------------------------------------------ host API
template <typename T>
static int dalloc_copy(T** d, const T* h, size_t n) {
    SHD_HIP(hipMalloc((void**)d, sizeof(T) * (n ? n : 1)));
    if (n) SHD_HIP(hipMemcpy(*d, h, sizeof(T) * n, hipMemcpyHostToDevice));
    return SHD_OK;
}

static void pc_free_device(shd_pc* pc) {
    void* ptrs[] = {pc->d_arc_off, pc->d_arc_dst, pc->d_arc_w, pc->d_arc_src, pc->d_arc_rin, pc->d_rin_off,
                    pc->d_rin_src, pc->d_rin_eid,
                    pc->d_rin_w, pc->d_rin_r, pc->d_inc_off, pc->d_inc_eid, pc->d_nbr_off, pc->d_nbr_v, pc->d_nbr_eid,
                    pc->d_w, pc->d_eloss, pc->d_vloss, pc->d_attached, pc->d_self_eid, pc->d_row,
                    pc->d_dir, pc->d_self, pc->d_adj,
                    pc->d_scratch, pc->d_stats, pc->d_tie_rows, pc->d_tie_scratch, pc->d_tie_lane};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
}

// ------------------------------------------------------------------ spatial relabelling
// A/B, off unless SHD_PC_RELABEL is set (measured and rejected, DESIGN.md §6:
// 27.7 ms for the 10 k table against 24.5 ms; a compact frontier lands in the
// chunks of a few waves, which then hold the barrier for the rest).  A vertex
// order from the graph alone (graphml topologies carry no coordinates):
// recursive bisection by hop distance -- the subset's BFS distances from a far
// vertex (the farthest from an arbitrary one), split at the median, until 64
// vertices -- so that a chunk of 64 consecutive labels is a compact region and
// a Bellman-Ford frontier (a shell around its source) meets few chunks.
// perm[old] = new.
struct PermCsr {
    std::vector<int32_t> perm, inv;
    std::vector<int32_t> inc_off, inc_eid, arc_off, arc_dst, arc_eid, rin_off, rin_src, rin_eid, nbr_off, nbr_v, nbr_eid;
    std::vector<double> arc_w, rin_w;
    shd_csr view{};
};

static void spatial_order(const shd_csr& c, std::vector<int32_t>& perm) {
    const int32_t V = c.V;
    perm.assign(V, 0);
    if (!getenv("SHD_PC_RELABEL") || V <= 64) {
        for (int32_t v = 0; v < V; v++) perm[v] = v;
        return;
    }
    // undirected neighbour lists (both arc directions)
    std::vector<int32_t> off(V + 1, 0), nb;
    for (int32_t v = 0; v < V; v++) off[v + 1] = (c.arc_off[v + 1] - c.arc_off[v]) + (c.rin_off[v + 1] - c.rin_off[v]);
    for (int32_t v = 0; v < V; v++) off[v + 1] += off[v];
    nb.resize(off[V]);
    for (int32_t v = 0; v < V; v++) {
        int32_t k = off[v];
        for (int32_t a = c.arc_off[v]; a < c.arc_off[v + 1]; a++) nb[k++] = c.arc_dst[a];
        for (int32_t a = c.rin_off[v]; a < c.rin_off[v + 1]; a++) nb[k++] = c.rin_src[a];
    }
    std::vector<int32_t> order(V), dist(V, -1), mark(V, 0), q(V);
    for (int32_t v = 0; v < V; v++) order[v] = v;
    int32_t stamp = 0;
    // BFS within order[lo, hi) (vertices marked `stamp`) from s: dist, the last vertex reached
    auto bfs = [&](int32_t lo, int32_t hi, int32_t s) {
        for (int32_t i = lo; i < hi; i++) dist[order[i]] = -1;
        int32_t qh = 0, qt = 0, last = s;
        dist[s] = 0;
        q[qt++] = s;
        while (qh < qt) {
            const int32_t u = q[qh++];
            last = u;
            for (int32_t k = off[u]; k < off[u + 1]; k++) {
                const int32_t x = nb[k];
                if (mark[x] == stamp && dist[x] < 0) { dist[x] = dist[u] + 1; q[qt++] = x; }
            }
        }
        return last;
    };
    struct Range { int32_t lo, hi; };
    std::vector<Range> st{{0, V}};
    while (!st.empty()) {
        const Range r = st.back();
        st.pop_back();
        if (r.hi - r.lo <= 64) continue;
        stamp++;
        for (int32_t i = r.lo; i < r.hi; i++) mark[order[i]] = stamp;
        const int32_t far = bfs(r.lo, r.hi, bfs(r.lo, r.hi, order[r.lo]));
        (void)far;
        // (the second BFS ran from the far vertex: dist holds its distances;
        // vertices it did not reach sort last, in their current order)
        std::stable_sort(order.begin() + r.lo, order.begin() + r.hi, [&](int32_t a, int32_t b) {
            const uint32_t da = (uint32_t)dist[a], db = (uint32_t)dist[b];
            return da < db;
        });
        const int32_t mid = r.lo + (((r.hi - r.lo) / 2 + 63) / 64) * 64;   // chunk-aligned halves
        st.push_back({mid < r.hi ? mid : r.hi, r.hi});
        st.push_back({r.lo, mid < r.hi ? mid : r.hi});
    }
    for (int32_t i = 0; i < V; i++) perm[order[i]] = i;
}

static void pc_relabel(const shd_csr& c, PermCsr& p) {
    const int32_t V = c.V;
    spatial_order(c, p.perm);
    p.inv.assign(V, 0);
    for (int32_t v = 0; v < V; v++) p.inv[p.perm[v]] = v;
    const auto& perm = p.perm;
    const auto& inv = p.inv;
    auto lists = [&](const int32_t* off, std::vector<int32_t>& noff) {
        noff.assign(V + 1, 0);
        for (int32_t n = 0; n < V; n++) noff[n + 1] = noff[n] + (off[inv[n] + 1] - off[inv[n]]);
    };
    lists(c.inc_off, p.inc_off);
    lists(c.arc_off, p.arc_off);
    lists(c.rin_off, p.rin_off);
    lists(c.nbr_off, p.nbr_off);
    p.inc_eid.resize(p.inc_off[V] + 1);
    p.arc_dst.resize(p.arc_off[V] + 1); p.arc_eid.resize(p.arc_off[V] + 1); p.arc_w.resize(p.arc_off[V] + 1);
    p.rin_src.resize(p.rin_off[V] + 1); p.rin_eid.resize(p.rin_off[V] + 1); p.rin_w.resize(p.rin_off[V] + 1);
    p.nbr_v.resize(p.nbr_off[V] + 1); p.nbr_eid.resize(p.nbr_off[V] + 1);
    std::vector<std::pair<int32_t, int32_t>> tmp;
    for (int32_t n = 0; n < V; n++) {
        const int32_t o = inv[n];
        for (int32_t k = c.inc_off[o], j = p.inc_off[n]; k < c.inc_off[o + 1]; k++, j++) p.inc_eid[j] = c.inc_eid[k];
        for (int32_t k = c.arc_off[o], j = p.arc_off[n]; k < c.arc_off[o + 1]; k++, j++) {   // incidence order kept
            p.arc_dst[j] = perm[c.arc_dst[k]]; p.arc_eid[j] = c.arc_eid[k]; p.arc_w[j] = c.arc_w[k];
        }
        for (int32_t k = c.rin_off[o], j = p.rin_off[n]; k < c.rin_off[o + 1]; k++, j++) {
            p.rin_src[j] = perm[c.rin_src[k]]; p.rin_eid[j] = c.rin_eid[k]; p.rin_w[j] = c.rin_w[k];
        }
        // neighbour lists sorted again by (new neighbour label, eid): the lowest
        // parallel eid stays first for get_eid
        tmp.clear();
        for (int32_t k = c.nbr_off[o]; k < c.nbr_off[o + 1]; k++) tmp.push_back({perm[c.nbr_v[k]], c.nbr_eid[k]});
        std::sort(tmp.begin(), tmp.end());
        for (size_t k = 0; k < tmp.size(); k++) { p.nbr_v[p.nbr_off[n] + k] = tmp[k].first; p.nbr_eid[p.nbr_off[n] + k] = tmp[k].second; }
    }
    shd_csr& w = p.view;
    w.V = V; w.E = c.E; w.directed = c.directed; w.max_degree = c.max_degree;
    w.inc_off = p.inc_off.data(); w.inc_eid = p.inc_eid.data();
    w.arc_off = p.arc_off.data(); w.arc_dst = p.arc_dst.data(); w.arc_eid = p.arc_eid.data(); w.arc_w = p.arc_w.data();
    w.rin_off = p.rin_off.data(); w.rin_src = p.rin_src.data(); w.rin_eid = p.rin_eid.data(); w.rin_w = p.rin_w.data();
    w.nbr_off = p.nbr_off.data(); w.nbr_v = p.nbr_v.data(); w.nbr_eid = p.nbr_eid.data();
}

extern "C" int shd_pc_create(const shd_graph* g, const int32_t* attached, int32_t n_attached, uint32_t flags,
                             int device, shd_pc** out) {
    if (!g || !attached || n_attached <= 0 || !out) return SHD_EINVAL;
    shd_graph_props props;
    int rc = shd_graph_check(g, &props);
    if (rc) return rc;
    for (int32_t i = 0; i < n_attached; i++)
        if (attached[i] < 0 || attached[i] >= g->n_vertices) return SHD_EINVAL;
    shd_pc* pc = new shd_pc();
    pc->device = device;
    pc->flags = flags;
    pc->props = props;
    pc->V = g->n_vertices;
    pc->E = g->n_edges;
    pc->T = n_attached;
    pc->directed = g->directed;
    pc->prefer_direct = g->prefer_direct;
    pc->complete = props.is_complete && !(flags & SHD_PC_FORCE_ROWS);
    pc->rows_mode = !pc->complete;
    if ((rc = shd_csr_build(g, &pc->csr))) { delete pc; return rc; }
    const int32_t V = pc->V, E = pc->E, T = pc->T;
    pc->h_attached = (int32_t*)malloc(sizeof(int32_t) * T);
    memcpy(pc->h_attached, attached, sizeof(int32_t) * T);
    pc->h_att_index = (int32_t*)malloc(sizeof(int32_t) * V);
    for (int32_t v = 0; v < V; v++) pc->h_att_index[v] = -1;
    for (int32_t i = 0; i < T; i++) {
        if (pc->h_att_index[attached[i]] >= 0) { shd_pc_destroy(pc); return SHD_EINVAL; }  // duplicate
        pc->h_att_index[attached[i]] = i;
    }
    pc->h_w = (double*)malloc(sizeof(double) * (E + 1));
    pc->h_eloss = (double*)malloc(sizeof(double) * (E + 1));
    memcpy(pc->h_w, g->edge_latency, sizeof(double) * E);
    memcpy(pc->h_eloss, g->edge_loss, sizeof(double) * E);
    pc->h_vloss = (double*)malloc(sizeof(double) * V);
    pc->has_vloss = g->vertex_loss != nullptr;
    for (int32_t v = 0; v < V; v++) pc->h_vloss[v] = g->vertex_loss ? g->vertex_loss[v] : NAN;
    pc->h_self_eid = (int32_t*)malloc(sizeof(int32_t) * T);
    for (int32_t i = 0; i < T; i++) pc->h_self_eid[i] = shd_csr_get_eid(&pc->csr, attached[i], attached[i]);
    pc->h_rank = (int32_t*)malloc(sizeof(int32_t) * T);
    pc->h_self_rank = (int32_t*)malloc(sizeof(int32_t) * T);
    for (int32_t i = 0; i < T; i++) pc->h_rank[i] = pc->h_self_rank[i] = kNoRank;
    pc->counts = new std::unordered_map<uint64_t, uint64_t>();

    if (hipSetDevice(device) != hipSuccess) { shd_pc_destroy(pc); return SHD_ENODEV; }
    if (hipStreamCreateWithFlags(&pc->stream, hipStreamNonBlocking) != hipSuccess) {
        shd_pc_destroy(pc);
        return SHD_ENODEV;
    }
    // the device's copy of the graph, relabelled in a spatial order when
    // SHD_PC_RELABEL is set (pc_relabel; the identity otherwise).  Every rule
    // that depends on order keeps the original one: each vertex's arcs stay in
    // igraph incidence order (the tie rows' heap Dijkstra relaxes in it),
    // parents break ties by original edge ids, and the neighbour lists keep the
    // lowest parallel edge id first.
    PermCsr pcsr;
    pc_relabel(pc->csr, pcsr);
    const shd_csr& c = pcsr.view;
    const int32_t na = c.arc_off[V];
    // the row kernel may keep the arc offsets in LDS (16 bits within a 64-vertex chunk)
    pc->lds_off_ok = getenv("SHD_PC_LDS_OFF") != nullptr;   // opt-in: neutral to slower
    for (int32_t v0 = 0; v0 < V && pc->lds_off_ok; v0 += 64)
        if (c.arc_off[std::min(V, v0 + 64)] - c.arc_off[v0] >= 65536) pc->lds_off_ok = false;
    // per forward arc: its tail vertex and the index of the same arc among its
    // head's in-arcs (the parent pass streams the forward arcs, the tree walks
    // use the in-arc indices)
    std::vector<int32_t> arc_src((size_t)na + 1), arc_rin((size_t)na + 1);
    for (int32_t u = 0; u < V; u++)
        for (int32_t k = c.arc_off[u]; k < c.arc_off[u + 1]; k++) {
            arc_src[k] = u;
            const int32_t x = c.arc_dst[k];
            int32_t a = -1;
            for (int32_t j = c.rin_off[x]; j < c.rin_off[x + 1]; j++)
                if (c.rin_src[j] == u && c.rin_eid[j] == c.arc_eid[k]) { a = j; break; }
            if (a < 0) { shd_pc_destroy(pc); return SHD_EINVAL; }   // the two CSRs disagree
            arc_rin[k] = a;
        }
    // per in-arc: the edge's reliability factor 1 - loss ((double)1.0f - loss, topology.c:437)
    std::vector<double> rin_r((size_t)na + 1);
    for (int32_t a = 0; a < na; a++) rin_r[a] = (double)1.0f - g->edge_loss[c.rin_eid[a]];
    {   // whole-number weights with V x the largest below 2^30: the tie kernel's 4-B heap values
        double wmax = 0.0;
        bool wi = true;
        for (int32_t k = 0; k < na && wi; k++) {
            const double w = c.arc_w[k];
            wi = std::isfinite(w) && w >= 0.0 && w == std::floor(w);
            wmax = w > wmax ? w : wmax;
        }
        pc->w_int = wi && wmax * (double)V < (double)(1 << 30);
    }
    if ((rc = dalloc_copy(&pc->d_arc_off, c.arc_off, V + 1)) || (rc = dalloc_copy(&pc->d_arc_dst, c.arc_dst, na)) ||
        (rc = dalloc_copy(&pc->d_arc_w, c.arc_w, na)) || (rc = dalloc_copy(&pc->d_rin_off, c.rin_off, V + 1)) ||
        (rc = dalloc_copy(&pc->d_rin_src, c.rin_src, na)) || (rc = dalloc_copy(&pc->d_rin_eid, c.rin_eid, na)) ||
        (rc = dalloc_copy(&pc->d_rin_w, c.rin_w, na)) || (rc = dalloc_copy(&pc->d_inc_off, c.inc_off, V + 1)) ||
        (rc = dalloc_copy(&pc->d_arc_src, arc_src.data(), na)) || (rc = dalloc_copy(&pc->d_arc_rin, arc_rin.data(), na)) ||
        (rc = dalloc_copy(&pc->d_rin_r, rin_r.data(), na)) ||
        (rc = dalloc_copy(&pc->d_inc_eid, c.inc_eid, c.inc_off[V])) ||
        (rc = dalloc_copy(&pc->d_nbr_off, c.nbr_off, V + 1)) || (rc = dalloc_copy(&pc->d_nbr_v, c.nbr_v, c.nbr_off[V])) ||
        (rc = dalloc_copy(&pc->d_nbr_eid, c.nbr_eid, c.nbr_off[V])) || (rc = dalloc_copy(&pc->d_w, pc->h_w, E)) ||
        (rc = dalloc_copy(&pc->d_eloss, pc->h_eloss, E)) || (rc = dalloc_copy(&pc->d_self_eid, pc->h_self_eid, T))) {
        shd_pc_destroy(pc);
        return rc;
    }
    {   // attached vertices and vertex loss factors in the device's labels
        std::vector<int32_t> att_d(T);
        for (int32_t i = 0; i < T; i++) att_d[i] = pcsr.perm[attached[i]];
        std::vector<double> vl_d(V);
        for (int32_t v = 0; v < V; v++) vl_d[pcsr.perm[v]] = pc->h_vloss[v];
        if ((rc = dalloc_copy(&pc->d_attached, att_d.data(), T)) ||
            (pc->has_vloss && (rc = dalloc_copy(&pc->d_vloss, vl_d.data(), V)))) {
            shd_pc_destroy(pc);
            return rc;
        }
    }
    const size_t TT = (size_t)T * T;
    if (hipMalloc((void**)&pc->d_dir, sizeof(shd_pv) * TT) != hipSuccess ||
        hipMalloc((void**)&pc->d_adj, TT) != hipSuccess || hipMalloc((void**)&pc->d_self, sizeof(shd_pv) * T) != hipSuccess ||
        hipMalloc((void**)&pc->d_stats, 8 * 8) != hipSuccess) {
        shd_pc_destroy(pc);
        return SHD_ENOMEM;
    }
    if (pc->rows_mode) {
        if (hipMalloc((void**)&pc->d_row, sizeof(shd_pv) * TT) != hipSuccess ||
            hipMalloc((void**)&pc->d_tie_rows, sizeof(int32_t) * T) != hipSuccess) {
            shd_pc_destroy(pc);
            return SHD_ENOMEM;
        }
    }
    pc->info.n_vertices = V;
    pc->info.n_attached = T;
    pc->info.is_complete = pc->complete;
    pc->info.is_directed = pc->directed;
    pc->info.prefer_direct = pc->prefer_direct;
    *out = pc;
    return SHD_OK;
}

#ifndef SHD_ROW_BLOCK
#define SHD_ROW_BLOCK 1024
#endif
constexpr int kRowBlock = SHD_ROW_BLOCK;   // workgroup of the LDS row kernel past 2 k vertices
// the dynamic row arrays' budget: 160 KiB less the kernels' static LDS (the
// SHD_SSSP_FLAT A/B's scan slots, 16 B a thread of the 1024-thread block)
#ifdef SHD_SSSP_FLAT
static constexpr size_t kLdsMax = 160 * 1024 - 16 * 1024 - 64;
#else
static constexpr size_t kLdsMax = 160 * 1024;
#endif
static size_t lds_bytes_for(int32_t V) { return (((size_t)14 * V + 15) & ~(size_t)15) + 16; }
// the arc offsets in LDS (ldsoff): 16-bit per vertex, a 32-bit base per 64-vertex chunk
// the row kernels' frontier: queued (default) or the half-wave pairs
// (SHD_PC_BF_PAIRS, the A/B of DESIGN.md §6)
static int bf_queue_bit() {
    static const int b = getenv("SHD_PC_BF_PAIRS") ? 0 : 2;
    return b;
}
// the two-row kernel: both rows' distances (16 B a vertex), their frontier
// bits and the flags; its
// waves scan ten 64-vertex chunks each at most (sssp_bf2<1024, 10>)
static size_t two_row_lds(int32_t V) { return (size_t)16 * V + (size_t)8 * ((V + 31) / 32) + 32; }
static bool two_row_ok(const shd_pc* pc) {
    static const bool off = getenv("SHD_PC_ONE_ROW") != nullptr;   // A/B: one row per workgroup
    return !off && kRowBlock == 1024 && pc->V <= 10 * 1024 && two_row_lds(pc->V) <= kLdsMax;
}
static size_t lds_off_bytes(int32_t V) {
    return (((size_t)2 * V + 15) & ~(size_t)15) + ((((size_t)(V + 63) / 64 + 1) * 4 + 15) & ~(size_t)15);
}
// the LDS layout of a row kernel launch: the row arrays, then (when they fit
// and the graph allows, shd_pc::lds_off_ok) the arc offsets
static size_t lds_launch_bytes(const shd_pc* pc, bool* ldsoff) {
    const size_t rows = lds_bytes_for(pc->V);
    *ldsoff = pc->lds_off_ok && rows + lds_off_bytes(pc->V) <= kLdsMax;
    return rows + (*ldsoff ? lds_off_bytes(pc->V) : 0);
}

// The rows the first pass listed (equal-cost predecessors somewhere in the
// row): their parents from k_sssp_tie_parents, in chunks of rows whose heaps
// fit a bounded scratch, then the row kernel again with those parents.
// cnt_from: tie-list entries from this index on were listed without a first
// pass (a predicted all-tied build): the second pass counts their ties
static int finish_tie_rows(shd_pc* pc, int ncu, int64_t cnt_from) {
    hipStream_t s = pc->stream;
    const int32_t V = pc->V, T = pc->T;
    int64_t n = 0;
    SHD_HIP(hipMemcpyAsync(&n, pc->d_stats + 6, sizeof(n), hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    pc->info.n_tie_rows = (int32_t)n;
    pc->info.n_tie_rows_global = 0;
    if (n <= 0) return SHD_OK;
    if (n > T) return SHD_ERANGE;
    // k_sssp_tie_lds where a row's state fits LDS beside a heap of >= 256
    // entries (as many blocks per CU as fit, up to 4); else, and for its rows
    // whose heap outgrows that, k_sssp_tie_parents (SHD_PC_TIE_GLOBAL: always)
    const size_t st_bytes = ((size_t)2 * V + 15) & ~(size_t)15;
    // A heap of 1024 entries (the rows of the 10 k whole-millisecond graph peak
    // between 600 and 1024: at 600, 503 of 10 000 rows outgrew it) beside the
    // row's 2-B vertex states, as many blocks per CU as LDS holds: the build
    // ran 439 ms at the largest heap that fits four per CU, 365 ms at 1024
    // (five per CU), 534 / 642 ms at 600 / 400 (rows falling back); round 5's
    // lane heaps 480-490 ms (profiles/r06/tiehc).  SHD_PC_TIE_HC: another
    // capacity (measurements)
    // STG: the states in global scratch and LDS for the heap only, where that
    // puts more rows on a CU (SHD_PC_TIE_STG=0 / 1 forces either)
    int hc = 0, bpc = 0;
    bool stg = false, hv4 = false;
    if (V <= 65533 && !getenv("SHD_PC_TIE_GLOBAL")) {
        const char* hc_env = getenv("SHD_PC_TIE_HC");
        const char* stg_env = getenv("SHD_PC_TIE_STG");
        hc = std::max(64, std::min(hc_env ? atoi(hc_env) : 1024, std::min(V, 65533)));
        hv4 = pc->w_int && !getenv("SHD_PC_TIE_HV8");   // (4-B heap values with STG only)
        const int bpc_g = (int)std::min<size_t>(32, std::max<size_t>(1, kLdsMax / ((size_t)hc * (hv4 ? 6 : 10))));
        int hc_l = hc;
        if (st_bytes + (size_t)hc_l * 10 > kLdsMax)
            hc_l = (int)std::min<size_t>(std::min(V, 65533), (kLdsMax - std::min(kLdsMax, st_bytes)) / 10);
        const int bpc_l = hc_l >= 64 ? (int)std::min<size_t>(8, std::max<size_t>(1, kLdsMax / (st_bytes + (size_t)hc_l * 10))) : 0;
        stg = stg_env ? atoi(stg_env) != 0 : (bpc_g > bpc_l || hc_l < hc);
        if (stg) {
            bpc = bpc_g;
        } else {
            hc = hc_l;
            bpc = bpc_l;
            hv4 = false;
        }
        if (!bpc) hc = 0;
    }
    const size_t tl_lds = (stg ? 0 : st_bytes) + (size_t)hc * (hv4 ? 6 : 10);
    // with the states out of LDS: k_sssp_tie_g (no position map) unless
    // SHD_PC_TIE_KIND=st (k_sssp_tie_lds<true>: the position map in global scratch)
    const char* kind_env = getenv("SHD_PC_TIE_KIND");
    const bool tg = stg && !(kind_env && strcmp(kind_env, "st") == 0);
    const bool vh = !getenv("SHD_PC_TIE_SHEAP");   // (the sifts in VALU; SHD_PC_TIE_SHEAP: scalarized)
    const void* tie_fn = tg ? (hv4 ? (vh ? (const void*)k_sssp_tie_g<int32_t, true> : (const void*)k_sssp_tie_g<int32_t, false>)
                                   : (vh ? (const void*)k_sssp_tie_g<double, true> : (const void*)k_sssp_tie_g<double, false>))
                       : stg ? (hv4 ? (const void*)k_sssp_tie_lds<true, int32_t> : (const void*)k_sssp_tie_lds<true, double>)
                             : (const void*)k_sssp_tie_lds<false, double>;
    // parents (4 B per vertex and row), and for k_sssp_tie_parents 24 B of lane
    // scratch per vertex and row; <= 4 GiB a chunk (every row of a 10 k-vertex
    // graph at once)
    const size_t g_entry = tg ? (hv4 ? sizeof(TieG<int32_t>) : sizeof(TieG<double>)) : 0;
    const size_t per_row = (size_t)V * (28 + g_entry);   // (+ k_sssp_tie_g's per-row entries)
    int64_t chunk = std::max<int64_t>(kTieLanes, (int64_t)(((size_t)4 << 30) / per_row) / kTieLanes * kTieLanes);
    chunk = std::min<int64_t>(chunk, (n + kTieLanes - 1) / kTieLanes * kTieLanes);
    const size_t need_p = (size_t)chunk * V * 4;
    const size_t need = need_p;
    if (!pc->d_tie_scratch || pc->tie_scratch_bytes < need) {
        if (pc->d_tie_scratch) (void)hipFree(pc->d_tie_scratch);
        pc->d_tie_scratch = nullptr;
        pc->tie_scratch_bytes = 0;
        SHD_HIP(hipMalloc(&pc->d_tie_scratch, need));
        pc->tie_scratch_bytes = need;
    }
    // the call's temporary device buffers, freed on every return (an error return
    // too; hipFree waits for the device, so no kernel of the call still uses them)
    struct TmpBufs {
        void* p[4] = {nullptr, nullptr, nullptr, nullptr};
        ~TmpBufs() {
            for (void* q : p)
                if (q) (void)hipFree(q);
        }
    } tmp;
    int32_t* d_ovf = nullptr;
    if (hc) {   // [0]: the count, then the slots of the rows whose heap outgrew hc
        SHD_HIP(hipMalloc(&d_ovf, sizeof(int32_t) * (1 + (size_t)chunk)));
        tmp.p[0] = d_ovf;
        SHD_HIP(hipFuncSetAttribute(tie_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tl_lds));
    }
    // STG: V states per block of the grid; k_sssp_tie_g: V entries per row of a
    // chunk, which the second pass reads as the rows' distances (d_gd; its
    // Bellman-Ford again was 22 of the 10 k all-tied build's 105 ms;
    // SHD_PC_TIE_NOGD: the Bellman-Ford again)
    uint16_t* d_stg = nullptr;
    uint8_t* d_gok = nullptr;
    if (hc && stg) {
        const size_t g = tg ? (size_t)std::min<int64_t>(chunk, n)
                            : (size_t)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(chunk, n), (int64_t)ncu * bpc));
        SHD_HIP(hipMalloc(&d_stg, g * (size_t)V * (tg ? g_entry : sizeof(uint16_t))));
        tmp.p[1] = d_stg;
        if (tg) {
            SHD_HIP(hipMalloc(&d_gok, g));
            tmp.p[2] = d_gok;
        }
    }
    const char* d_gd = (tg && !getenv("SHD_PC_TIE_NOGD")) ? (const char*)d_stg : nullptr;
    const int gkind = d_gd ? (hv4 ? 4 : 8) : 0;
    uint8_t* d_dup = nullptr;   // (k_sssp_tie_g: the arcs' repeated-target flags)
    if (hc && tg) {
        int32_t na = 0;
        SHD_HIP(hipMemcpyAsync(&na, pc->d_arc_off + V, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        SHD_HIP(hipStreamSynchronize(s));
        SHD_HIP(hipMalloc(&d_dup, (size_t)na + 1));
        tmp.p[3] = d_dup;
        if (na > 0) {
            hipLaunchKernelGGL(k_arc_dup, dim3((na + 255) / 256), dim3(256), 0, s, na, pc->d_arc_off, pc->d_arc_src,
                               pc->d_arc_dst, d_dup);
            SHD_HIP(hipGetLastError());
        }
    }
    int32_t* fpar = (int32_t*)pc->d_tie_scratch;
    bool lo = false;
    const size_t lds_rows = lds_bytes_for(V), lds = lds_launch_bytes(pc, &lo);
    for (int64_t c0 = 0; c0 < n; c0 += chunk) {
        const int32_t cn = (int32_t)std::min<int64_t>(chunk, n - c0);
        const int32_t* rows = pc->d_tie_rows + c0;
        int32_t nov = hc ? 0 : cn;   // rows for the lane heaps (all of them without k_sssp_tie_lds)
        if (hc) {
            SHD_HIP(hipMemsetAsync(d_ovf, 0, sizeof(int32_t), s));
            // every slot filled (the grid strides over the rows): as many rows for every
            // block instead (10 000 rows on 5 000 blocks, not 6 656) ran 186 against 168 ms
            // -- a row's time grows little with the rows beside it on the CU
            // (profiles/r06/tiefill)
            const int grid = std::max(1, std::min(cn, ncu * bpc));
            if (tg && hv4 && vh)
                hipLaunchKernelGGL((k_sssp_tie_g<int32_t, true>), dim3(grid), dim3(64), tl_lds, s, V, cn, rows,
                                   pc->d_attached, pc->d_arc_off, pc->d_arc_dst, pc->d_arc_w, pc->d_arc_rin, fpar,
                                   (int32_t)hc, d_ovf, (TieG<int32_t>*)d_stg, d_dup, d_gok);
            else if (tg && hv4)
                hipLaunchKernelGGL((k_sssp_tie_g<int32_t, false>), dim3(grid), dim3(64), tl_lds, s, V, cn, rows,
                                   pc->d_attached, pc->d_arc_off, pc->d_arc_dst, pc->d_arc_w, pc->d_arc_rin, fpar,
                                   (int32_t)hc, d_ovf, (TieG<int32_t>*)d_stg, d_dup, d_gok);
            else if (tg && vh)
                hipLaunchKernelGGL((k_sssp_tie_g<double, true>), dim3(grid), dim3(64), tl_lds, s, V, cn, rows,
                                   pc->d_attached, pc->d_arc_off, pc->d_arc_dst, pc->d_arc_w, pc->d_arc_rin, fpar,
                                   (int32_t)hc, d_ovf, (TieG<double>*)d_stg, d_dup, d_gok);
            else if (tg)
                hipLaunchKernelGGL((k_sssp_tie_g<double, false>), dim3(grid), dim3(64), tl_lds, s, V, cn, rows,
                                   pc->d_attached, pc->d_arc_off, pc->d_arc_dst, pc->d_arc_w, pc->d_arc_rin, fpar,
                                   (int32_t)hc, d_ovf, (TieG<double>*)d_stg, d_dup, d_gok);
            else if (stg && hv4)
                hipLaunchKernelGGL((k_sssp_tie_lds<true, int32_t>), dim3(grid), dim3(64), tl_lds, s, V, cn, rows,
                                   pc->d_attached, pc->d_arc_off, pc->d_arc_dst, pc->d_arc_w, pc->d_arc_rin, fpar,
                                   (int32_t)hc, d_ovf, d_stg);
            else if (stg)
                hipLaunchKernelGGL((k_sssp_tie_lds<true, double>), dim3(grid), dim3(64), tl_lds, s, V, cn, rows,
                                   pc->d_attached, pc->d_arc_off, pc->d_arc_dst, pc->d_arc_w, pc->d_arc_rin, fpar,
                                   (int32_t)hc, d_ovf, d_stg);
            else
                hipLaunchKernelGGL((k_sssp_tie_lds<false, double>), dim3(grid), dim3(64), tl_lds, s, V, cn, rows,
                                   pc->d_attached, pc->d_arc_off, pc->d_arc_dst, pc->d_arc_w, pc->d_arc_rin, fpar,
                                   (int32_t)hc, d_ovf, d_stg);
            SHD_HIP(hipGetLastError());
            SHD_HIP(hipMemcpyAsync(&nov, d_ovf, sizeof(int32_t), hipMemcpyDeviceToHost, s));
            SHD_HIP(hipStreamSynchronize(s));
            pc->info.n_tie_rows_global += nov;
        }
        if (nov) {   // (a heap past hc: those rows again through lane heaps in global scratch)
            const size_t ns = (size_t)((nov + kTieLanes - 1) / kTieLanes) * kTieLanes * V * 24;
            if (!pc->d_tie_lane || pc->tie_lane_bytes < ns) {
                if (pc->d_tie_lane) (void)hipFree(pc->d_tie_lane);
                pc->d_tie_lane = nullptr;
                pc->tie_lane_bytes = 0;
                SHD_HIP(hipMalloc(&pc->d_tie_lane, ns));
                pc->tie_lane_bytes = ns;
            }
            hipLaunchKernelGGL(k_sssp_tie_parents, dim3((nov + kTieLanes - 1) / kTieLanes), dim3(kTieLanes), 0, s, V,
                               nov, rows, pc->d_attached, pc->d_arc_off, pc->d_arc_dst, pc->d_arc_w, pc->d_arc_rin,
                               fpar, (char*)pc->d_tie_lane, hc ? (const int32_t*)(d_ovf + 1) : nullptr);
            SHD_HIP(hipGetLastError());
        }
        if (lds_rows <= kLdsMax && V <= 2048) {
            const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(8, kLdsMax / lds));
            const int grid = std::max(1, std::min(cn, ncu * per_cu));
            hipLaunchKernelGGL(k_sssp_rows_lds<256>, dim3(grid), dim3(256), lds, s, V, T, pc->d_arc_off,
                               pc->d_arc_dst, pc->d_arc_w, pc->d_arc_src, pc->d_arc_rin, pc->d_rin_off, pc->d_rin_src,
                               pc->d_rin_eid, pc->d_rin_w, pc->d_rin_r, pc->d_w, pc->d_eloss, pc->d_vloss,
                               pc->d_attached, pc->d_self_eid, pc->d_row, pc->d_stats, 0, cn, rows, fpar, nullptr,
                               (lo ? 1 : 0) | bf_queue_bit(),
                               (const char*)d_gd, gkind, d_gok,
                               (int32_t)std::min<int64_t>(INT32_MAX, std::max<int64_t>(-1, cnt_from - c0)));
        } else if (lds_rows <= kLdsMax) {
            const int grid = std::max(1, std::min(cn, ncu));
            hipLaunchKernelGGL(k_sssp_rows_lds<kRowBlock>, dim3(grid), dim3(kRowBlock), lds, s, V, T, pc->d_arc_off,
                               pc->d_arc_dst, pc->d_arc_w, pc->d_arc_src, pc->d_arc_rin, pc->d_rin_off, pc->d_rin_src,
                               pc->d_rin_eid, pc->d_rin_w, pc->d_rin_r, pc->d_w, pc->d_eloss, pc->d_vloss,
                               pc->d_attached, pc->d_self_eid, pc->d_row, pc->d_stats, 0, cn, rows, fpar, nullptr,
                               (lo ? 1 : 0) | bf_queue_bit(),
                               (const char*)d_gd, gkind, d_gok,
                               (int32_t)std::min<int64_t>(INT32_MAX, std::max<int64_t>(-1, cnt_from - c0)));
        } else {
            // the first pass sized d_scratch for ncu * 4 blocks
            const size_t per_block = ((size_t)14 * V + 255) & ~(size_t)255;
            const int grid = (int)std::max<size_t>(1, std::min<size_t>((size_t)cn, pc->scratch_bytes / per_block));
            hipLaunchKernelGGL(k_sssp_rows_global<512>, dim3(grid), dim3(512), 0, s, V, T, pc->d_arc_off,
                               pc->d_arc_dst, pc->d_arc_w, pc->d_arc_src, pc->d_arc_rin, pc->d_rin_off, pc->d_rin_src,
                               pc->d_rin_eid, pc->d_rin_w, pc->d_rin_r, pc->d_w, pc->d_eloss, pc->d_vloss,
                               pc->d_attached, pc->d_self_eid, pc->d_row, pc->d_stats, (char*)pc->d_scratch, per_block,
                               0, cn, rows, fpar, nullptr, bf_queue_bit());
        }
        SHD_HIP(hipGetLastError());
    }
    return SHD_OK;
}

// the build; with a communicator this rank computes its block of source
// rows and the blocks are all-gathered (shd_pc_build_sharded)
static int pc_build(shd_pc* pc, shd_comm* comm) {
    if (!pc) return SHD_EINVAL;
    SHD_HIP(hipSetDevice(pc->device));
    const int32_t V = pc->V, T = pc->T;
    hipStream_t s = pc->stream;
    const int W = comm ? comm->world : 1, me = comm ? comm->rank : 0;
    const int32_t R = (int32_t)((T + W - 1) / W);              // rows per rank
    const int32_t row0 = std::min<int32_t>(T, me * R), row1 = std::min<int32_t>(T, row0 + R);
    if (pc->rows_mode && (size_t)R * W > (size_t)T && pc->rows_alloc < (size_t)R * W) {
        // the all-gather takes equal blocks: pad the table to W * R rows
        shd_pv* nr = nullptr;
        SHD_HIP(hipMalloc((void**)&nr, sizeof(shd_pv) * (size_t)R * W * T));
        (void)hipFree(pc->d_row);
        pc->d_row = nr;
        pc->rows_alloc = (size_t)R * W;
    }
    const auto t_call = std::chrono::steady_clock::now();
    int64_t init_stats[8] = {0, 0, 0, 0, 0, (int64_t)kDistInf, 0, 0};
    SHD_HIP(hipMemcpyAsync(pc->d_stats, init_stats, sizeof(init_stats), hipMemcpyHostToDevice, s));
    hipEvent_t ev[4];
    for (auto& e : ev) SHD_HIP(hipEventCreate(&e));
    SHD_HIP(hipEventRecord(ev[0], s));
    // direct values + adjacency for every attached pair (used in complete and
    // prefer-direct modes; cheap otherwise)
    {
        const size_t TT = (size_t)T * T;
        int blocks = (int)std::min<size_t>((TT + 255) / 256, 8192);
        hipLaunchKernelGGL(k_direct, dim3(blocks), dim3(256), 0, s, T, pc->d_attached, pc->d_nbr_off, pc->d_nbr_v,
                           pc->d_nbr_eid, pc->d_w, pc->d_eloss, pc->d_vloss, pc->d_dir, pc->d_adj);
        hipLaunchKernelGGL(k_self, dim3((T + 255) / 256), dim3(256), 0, s, T, pc->d_attached, pc->d_inc_off,
                           pc->d_inc_eid, pc->d_w, pc->d_eloss, pc->d_self);
        SHD_HIP(hipGetLastError());
    }
    SHD_HIP(hipEventRecord(ev[1], s));
    if (pc->rows_mode) {
        bool lo = false;
        int64_t cnt_from = INT64_MAX;   // (a predicted all-tied build: the tie list's unprobed rows)
        pc->info.n_tie_rows_predicted = 0;
        const size_t lds_rows = lds_bytes_for(V), lds = lds_launch_bytes(pc, &lo);
        int ncu = 256;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, pc->device) == hipSuccess) ncu = prop.multiProcessorCount;
        if (lds_rows <= kLdsMax) {
            if (V <= 2048) {
                int per_cu = (int)std::max<size_t>(1, std::min<size_t>(8, kLdsMax / lds));
                int grid = std::max(1, std::min(row1 - row0, ncu * per_cu));
                SHD_HIP(hipFuncSetAttribute((const void*)k_sssp_rows_lds<256>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                hipLaunchKernelGGL(k_sssp_rows_lds<256>, dim3(grid), dim3(256), lds, s, V, T, pc->d_arc_off,
                                   pc->d_arc_dst, pc->d_arc_w, pc->d_arc_src, pc->d_arc_rin, pc->d_rin_off, pc->d_rin_src, pc->d_rin_eid,
                                   pc->d_rin_w, pc->d_rin_r, pc->d_w, pc->d_eloss, pc->d_vloss, pc->d_attached,
                                   pc->d_self_eid,
                                   pc->d_row, pc->d_stats, row0, row1, nullptr, nullptr, pc->d_tie_rows,
                                   (lo ? 1 : 0) | bf_queue_bit(),
                               (const char*)nullptr, 0, (const uint8_t*)nullptr, 0);
            } else if (two_row_ok(pc)) {
                // two rows per workgroup (sssp_bf2), row B parked in d_scratch
                const size_t lds2 = two_row_lds(V);
                const int grid = std::max(1, std::min((row1 - row0 + 1) / 2, ncu));
                const size_t park = (size_t)grid * V * sizeof(uint64_t);
                // A predicted all-tied build (round 6): on whole-number weights the first
                // pass runs one probe of 2 x CUs rows; when 90 % of them tie, the other
                // rows go to the tie kernel without a first pass (whose Bellman-Ford a
                // tied row only used to be listed), and the second pass counts their
                // ties (SHD_PC_NO_TIE_PREDICT: the first pass over every row)
                const bool predict = pc->w_int && W == 1 && !getenv("SHD_PC_NO_TIE_PREDICT") &&
                                     row1 - row0 > 8 * grid;
                const int32_t prow1 = predict ? row0 + 2 * grid : row1;
                if (!pc->d_scratch || pc->scratch_bytes < park) {
                    if (pc->d_scratch) (void)hipFree(pc->d_scratch);
                    pc->d_scratch = nullptr;
                    pc->scratch_bytes = 0;
                    SHD_HIP(hipMalloc(&pc->d_scratch, park));
                    pc->scratch_bytes = park;
                }
                SHD_HIP(hipFuncSetAttribute((const void*)k_sssp_rows2_lds<kRowBlock>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2));
                hipLaunchKernelGGL(k_sssp_rows2_lds<kRowBlock>, dim3(grid), dim3(kRowBlock), lds2, s, V, T,
                                   pc->d_arc_off, pc->d_arc_dst, pc->d_arc_w, pc->d_arc_src, pc->d_arc_rin,
                                   pc->d_rin_off, pc->d_rin_src, pc->d_rin_eid, pc->d_rin_w, pc->d_rin_r, pc->d_w,
                                   pc->d_eloss, pc->d_vloss, pc->d_attached, pc->d_self_eid, pc->d_row, pc->d_stats,
                                   row0, prow1, pc->d_tie_rows, (uint64_t*)pc->d_scratch);
                if (predict) {
                    SHD_HIP(hipGetLastError());
                    int64_t nt = 0;
                    SHD_HIP(hipMemcpyAsync(&nt, pc->d_stats + 6, sizeof(nt), hipMemcpyDeviceToHost, s));
                    SHD_HIP(hipStreamSynchronize(s));
                    if (nt * 10 >= (int64_t)(prow1 - row0) * 9) {
                        const int32_t nr = row1 - prow1;
                        hipLaunchKernelGGL(k_iota, dim3((nr + 255) / 256), dim3(256), 0, s, pc->d_tie_rows + nt, nr,
                                           prow1);
                        const int64_t tot = nt + nr;
                        SHD_HIP(hipMemcpyAsync(pc->d_stats + 6, &tot, sizeof(tot), hipMemcpyHostToDevice, s));
                        cnt_from = nt;
                        pc->info.n_tie_rows_predicted = nr;
                    } else {
                        hipLaunchKernelGGL(k_sssp_rows2_lds<kRowBlock>, dim3(grid), dim3(kRowBlock), lds2, s, V, T,
                                           pc->d_arc_off, pc->d_arc_dst, pc->d_arc_w, pc->d_arc_src, pc->d_arc_rin,
                                           pc->d_rin_off, pc->d_rin_src, pc->d_rin_eid, pc->d_rin_w, pc->d_rin_r,
                                           pc->d_w, pc->d_eloss, pc->d_vloss, pc->d_attached, pc->d_self_eid,
                                           pc->d_row, pc->d_stats, prow1, row1, pc->d_tie_rows,
                                           (uint64_t*)pc->d_scratch);
                    }
                }
            } else {
                int grid = std::max(1, std::min(row1 - row0, ncu));
                SHD_HIP(hipFuncSetAttribute((const void*)k_sssp_rows_lds<kRowBlock>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                hipLaunchKernelGGL(k_sssp_rows_lds<kRowBlock>, dim3(grid), dim3(kRowBlock), lds, s, V, T, pc->d_arc_off,
                                   pc->d_arc_dst, pc->d_arc_w, pc->d_arc_src, pc->d_arc_rin, pc->d_rin_off, pc->d_rin_src, pc->d_rin_eid,
                                   pc->d_rin_w, pc->d_rin_r, pc->d_w, pc->d_eloss, pc->d_vloss, pc->d_attached,
                                   pc->d_self_eid,
                                   pc->d_row, pc->d_stats, row0, row1, nullptr, nullptr, pc->d_tie_rows,
                                   (lo ? 1 : 0) | bf_queue_bit(),
                               (const char*)nullptr, 0, (const uint8_t*)nullptr, 0);
            }
        } else {
            const size_t per_block = ((size_t)14 * V + 255) & ~(size_t)255;
            int grid = std::max(1, std::min(row1 - row0, ncu * 4));
            if (!pc->d_scratch || pc->scratch_bytes < per_block * grid) {
                if (pc->d_scratch) (void)hipFree(pc->d_scratch);
                pc->scratch_bytes = per_block * grid;
                SHD_HIP(hipMalloc(&pc->d_scratch, pc->scratch_bytes));
            }
            hipLaunchKernelGGL(k_sssp_rows_global<512>, dim3(grid), dim3(512), 0, s, V, T, pc->d_arc_off,
                               pc->d_arc_dst, pc->d_arc_w, pc->d_arc_src, pc->d_arc_rin, pc->d_rin_off, pc->d_rin_src, pc->d_rin_eid, pc->d_rin_w,
                               pc->d_rin_r, pc->d_w, pc->d_eloss, pc->d_vloss, pc->d_attached, pc->d_self_eid, pc->d_row,
                               pc->d_stats, (char*)pc->d_scratch, per_block, row0, row1, nullptr, nullptr,
                               pc->d_tie_rows, bf_queue_bit());
        }
        SHD_HIP(hipGetLastError());
        const int rc = finish_tie_rows(pc, ncu, cnt_from);
        if (rc) { for (auto& e : ev) (void)hipEventDestroy(e); return rc; }
    }
    SHD_HIP(hipEventRecord(ev[2], s));
    if (comm && pc->rows_mode && W > 1) {
        // the row blocks, all-gathered in place (block r starts at row r * R)
        const size_t blk = sizeof(shd_pv) * (size_t)R * T;
        const int rc = shd_comm_allgather_dev(comm, (const char*)pc->d_row + blk * me, pc->d_row, blk, s);
        if (rc) { for (auto& e : ev) (void)hipEventDestroy(e); return rc; }
    }
    {
        const size_t TT = (size_t)T * T;
        int blocks = (int)std::min<size_t>((TT + 255) / 256, 4096);
        const shd_pv* tab = pc->rows_mode ? pc->d_row : pc->d_dir;
        hipLaunchKernelGGL(k_min_latency, dim3(blocks), dim3(256), 0, s, tab, TT, pc->d_stats);
        SHD_HIP(hipGetLastError());
    }
    SHD_HIP(hipEventRecord(ev[3], s));
    SHD_HIP(hipStreamSynchronize(s));
    float ms_dir = 0, ms_rows = 0, ms_all = 0;
    SHD_HIP(hipEventElapsedTime(&ms_dir, ev[0], ev[1]));
    SHD_HIP(hipEventElapsedTime(&ms_rows, ev[1], ev[2]));
    SHD_HIP(hipEventElapsedTime(&ms_all, ev[0], ev[3]));
    for (auto& e : ev) (void)hipEventDestroy(e);
    int64_t st[8];
    SHD_HIP(hipMemcpy(st, pc->d_stats, sizeof(st), hipMemcpyDeviceToHost));
    if (comm && W > 1) {   // this rank's row statistics -> the group's
        std::vector<int64_t> all((size_t)8 * W);
        const int rc = shd_comm_allgather_host(comm, st, sizeof(st), all.data());
        if (rc) return rc;
        for (int r = 0; r < W; r++) {
            if (r == me) continue;
            const int64_t* o = &all[(size_t)8 * r];
            st[0] += o[0];
            st[1] = std::max(st[1], o[1]);
            st[2] = std::max(st[2], o[2]);
            st[3] += o[3];
            st[4] += o[4];
            st[6] += o[6];
        }
    }
    pc->info.n_tie_rows = (int32_t)st[6];
    pc->info.rows_computed = pc->rows_mode ? T : 0;
    pc->info.n_ties = st[0];
    pc->info.max_hops = (int32_t)st[1];
    pc->info.sssp_iterations_max = (int32_t)st[2];
    pc->info.n_unroutable = (int32_t)st[3];
    uint64_t mb = (uint64_t)st[5];
    double ml;
    memcpy(&ml, &mb, 8);
    pc->info.min_latency_ms = ml;
    pc->info.build_ms_direct = ms_dir;
    pc->info.build_ms_sssp = ms_rows;
    pc->info.build_ms_props = 0.0;   // fused into the SSSP kernel
    pc->info.build_ms_device = comm ? std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() -
                                                                                 t_call).count()
                                    : ms_all;
    if (st[4] != 0) {
        fprintf(stderr, "libshdgpu: %lld latency folds differ from converged distances\n", (long long)st[4]);
        return SHD_ERANGE;
    }
    pc->built = true;
    return SHD_OK;
}

extern "C" int shd_pc_build(shd_pc* pc) { return pc_build(pc, nullptr); }

extern "C" int shd_pc_build_sharded(shd_pc* pc, shd_comm* comm) {
    if (!pc || !comm) return SHD_EINVAL;
    return pc_build(pc, comm);
}

extern "C" int shd_pc_get_info(const shd_pc* pc, shd_pc_info* out) {
    if (!pc || !out) return SHD_EINVAL;
    *out = pc->info;
    return SHD_OK;
}

// device (lat, rel) pairs -> the caller's two arrays, in bounded chunks
static int split_copy(const shd_pv* src, size_t n, double* lat, double* rel) {
    constexpr size_t kChunk = 1u << 20;
    std::vector<shd_pv> buf(std::min(n, kChunk));
    for (size_t i = 0; i < n; i += kChunk) {
        const size_t m = std::min(kChunk, n - i);
        SHD_HIP(hipMemcpy(buf.data(), src + i, sizeof(shd_pv) * m, hipMemcpyDeviceToHost));
        for (size_t k = 0; k < m; k++) {
            if (lat) lat[i + k] = buf[k].lat;
            if (rel) rel[i + k] = buf[k].rel;
        }
    }
    return SHD_OK;
}

static int copy_table(shd_pc* pc, const shd_pv* d, int32_t row0, int32_t nrows, double* lat, double* rel) {
    if (!pc || !pc->built || row0 < 0 || nrows < 0 || row0 + nrows > pc->T) return SHD_EINVAL;
    if (!d) return SHD_EINVAL;
    SHD_HIP(hipSetDevice(pc->device));
    const size_t off = (size_t)row0 * pc->T, n = (size_t)nrows * pc->T;
    return split_copy(d + off, n, lat, rel);
}

extern "C" int shd_pc_copy_rows(shd_pc* pc, int32_t row0, int32_t nrows, double* lat, double* rel) {
    if (!pc) return SHD_EINVAL;
    return copy_table(pc, pc->d_row, row0, nrows, lat, rel);
}
extern "C" int shd_pc_copy_direct(shd_pc* pc, int32_t row0, int32_t nrows, double* lat, double* rel) {
    if (!pc) return SHD_EINVAL;
    return copy_table(pc, pc->d_dir, row0, nrows, lat, rel);
}
extern "C" int shd_pc_copy_self(shd_pc* pc, double* lat, double* rel) {
    if (!pc || !pc->built) return SHD_EINVAL;
    SHD_HIP(hipSetDevice(pc->device));
    return split_copy(pc->d_self, (size_t)pc->T, lat, rel);
}

// ------------------------------------------------------------------ lazy lookup (host adapter)
// The reference stores each unordered pair once, from whichever row ran first
// (topology.c:1307-1336), and a row for source s runs on the first query
// (s,d) that misses in both orientations (1987-1990, 2030).  Direct paths
// are stored by the first query of an adjacent pair (2019-2021).
static int fetch2(shd_pc* pc, const shd_pv* d, size_t idx, double* lat, double* rel) {
    shd_pv v;
    SHD_HIP(hipMemcpy(&v, d + idx, sizeof(v), hipMemcpyDeviceToHost));
    *lat = v.lat;
    *rel = v.rel;
    return SHD_OK;
}

static void note_min(shd_pc* pc, double lat) {
    if (pc->min_stored_latency == 0 || lat < pc->min_stored_latency) pc->min_stored_latency = lat;
}

static int run_row_for_min(shd_pc* pc, int32_t a) {
    // the row stores every {a,t} not yet stored: track minimumPathLatency
    const int32_t T = pc->T;
    double* buf = (double*)malloc(8 * (size_t)T);
    if (!buf) return SHD_ENOMEM;
    if (split_copy(pc->d_row + (size_t)a * T, (size_t)T, buf, nullptr) != SHD_OK) {
        free(buf);
        return SHD_ENODEV;
    }
    for (int32_t t = 0; t < T; t++) {
        const bool stored = (t == a) ? (pc->h_self_rank[a] != kNoRank) : (pc->h_rank[t] != kNoRank);
        if (stored || buf[t] < 0) continue;
        if (pc->prefer_direct) {
            uint8_t adj = 0;
            if (hipMemcpy(&adj, pc->d_adj + (size_t)a * T + t, 1, hipMemcpyDeviceToHost) != hipSuccess) {
                free(buf);
                return SHD_ENODEV;
            }
            if (adj) continue;
        }
        note_min(pc, buf[t]);
    }
    free(buf);
    return SHD_OK;
}

// One lazy cache across a co-simulation, this cache being the CPU side's
// (INTEGRATION.md "Mixed CPU/GPU hosts"): the other side's first touches of
// the window, in event order, applied just before this side's first later
// query; this side's own first touches (lookups that rank a row), logged
struct PcTouches {
    std::vector<shd_pending> defer;
    size_t next = 0;
    std::vector<shd_pending> own;
    shd_pending key{};
    bool on = false;
};
static bool pend_key_less(const shd_pending& x, const shd_pending& y) {
    if (x.qtime != y.qtime) return x.qtime < y.qtime;
    if (x.qhost != y.qhost) return x.qhost < y.qhost;
    if (x.qsrc != y.qsrc) return x.qsrc < y.qsrc;
    if (x.qseq != y.qseq) return x.qseq < y.qseq;
    return x.qsub < y.qsub;
}
static int pc_lookup_at(shd_pc* pc, int32_t a, int32_t b, double* lat, double* rel);

// the deferred touches before `k` (or all: k null) to the cache
static int pc_apply_deferred(shd_pc* pc, const shd_pending* k) {
    PcTouches* t = (PcTouches*)pc->touches;
    while (t->next < t->defer.size() && (!k || pend_key_less(t->defer[t->next], *k))) {
        const shd_pending& r = t->defer[t->next++];
        double l, q;
        const int rc = pc_lookup_at(pc, (int32_t)r.a, (int32_t)r.b, &l, &q);
        if (rc) return rc;
    }
    return SHD_OK;
}

extern "C" int shd_pc_defer_touches(shd_pc* pc, const shd_pending* recs, uint64_t n) {
    if (!pc || (n && !recs)) return SHD_EINVAL;
    if (!pc->touches) pc->touches = new PcTouches();
    PcTouches* t = (PcTouches*)pc->touches;
    if (t->next < t->defer.size()) return SHD_EINVAL;   // the last window's not all applied
    for (uint64_t i = 0; i < n; i++)
        if (recs[i].a >= (uint32_t)pc->T || recs[i].b >= (uint32_t)pc->T) return SHD_EINVAL;
    t->defer.assign(recs, recs + n);
    std::sort(t->defer.begin(), t->defer.end(), pend_key_less);
    t->next = 0;
    t->on = true;
    return SHD_OK;
}

extern "C" int shd_pc_query_key(shd_pc* pc, uint64_t time, uint32_t host, uint32_t src, uint64_t seq) {
    if (!pc) return SHD_EINVAL;
    if (!pc->touches) pc->touches = new PcTouches();
    PcTouches* t = (PcTouches*)pc->touches;
    t->key = shd_pending{};
    t->key.qtime = time; t->key.qhost = host; t->key.qsrc = src; t->key.qseq = seq; t->key.qsub = 0;
    return SHD_OK;
}

extern "C" int shd_pc_take_touches(shd_pc* pc, shd_pending* out, uint64_t cap, uint64_t* n) {
    if (!pc || !n) return SHD_EINVAL;
    PcTouches* t = (PcTouches*)pc->touches;
    if (!t) { *n = 0; return SHD_OK; }
    if (pc->built) {
        const int rc = pc_apply_deferred(pc, nullptr);
        if (rc) return rc;
    }
    *n = t->own.size();
    if (!out) return SHD_OK;
    if (cap < t->own.size()) return SHD_ERANGE;
    if (!t->own.empty()) memcpy(out, t->own.data(), sizeof(shd_pending) * t->own.size());
    t->own.clear();
    return SHD_OK;
}

extern "C" int shd_pc_lookup(shd_pc* pc, int32_t sv, int32_t dv, double* lat, double* rel) {
    if (!pc || !pc->built || !lat || !rel || sv < 0 || dv < 0 || sv >= pc->V || dv >= pc->V) return SHD_EINVAL;
    const int32_t a = pc->h_att_index[sv], b = pc->h_att_index[dv];
    if (a < 0 || b < 0) { *lat = -1; *rel = -1; return SHD_EINVAL; }
    PcTouches* t = (PcTouches*)pc->touches;
    if (!t || !t->on) return pc_lookup_at(pc, a, b, lat, rel);
    shd_pending k = t->key;
    k.qsub = t->key.qsub++;
    int rc = pc_apply_deferred(pc, &k);
    if (rc) return rc;
    const int32_t nr0 = pc->next_rank;
    if ((rc = pc_lookup_at(pc, a, b, lat, rel))) return rc;
    if (pc->next_rank != nr0) {   // this lookup ranked a row (or a self path): a first touch
        k.a = (uint32_t)a;
        k.b = (uint32_t)b;
        t->own.push_back(k);
    }
    return SHD_OK;
}

// shd_pc_lookup by attached indices (the rank rule, then the value)
static int pc_lookup_at(shd_pc* pc, int32_t a, int32_t b, double* lat, double* rel) {
    SHD_HIP(hipSetDevice(pc->device));
    const int32_t T = pc->T;
    uint8_t adj = 0;
    if (pc->prefer_direct && !pc->complete)
        SHD_HIP(hipMemcpy(&adj, pc->d_adj + (size_t)a * T + b, 1, hipMemcpyDeviceToHost));
    if (pc->complete || adj) {
        int rc = fetch2(pc, pc->d_dir, (size_t)a * T + b, lat, rel);
        if (rc) return rc;
        if (isnan(*lat)) { *lat = -1; *rel = -1; return SHD_OK; }
        note_min(pc, *lat);
        return SHD_OK;
    }
    if (a == b) {
        // self pair: stored by row a ([a] with the self-loop) or by the
        // self-path computation, whichever came first
        int32_t ra = pc->h_rank[a], rs = pc->h_self_rank[a];
        if (ra == kNoRank && rs == kNoRank) {
            pc->h_self_rank[a] = rs = pc->next_rank++;
            int rc = fetch2(pc, pc->d_self, (size_t)a, lat, rel);
            if (rc) return rc;
            if (*lat < 0) return SHD_OK;
            note_min(pc, *lat);
            return SHD_OK;
        }
        if (rs < ra) return fetch2(pc, pc->d_self, (size_t)a, lat, rel);
        return fetch2(pc, pc->d_row, (size_t)a * T + a, lat, rel);
    }
    int32_t ra = pc->h_rank[a], rb = pc->h_rank[b];
    // undirected: a miss needs both orientations missing (1987-1990);
    // directed: only (a,b) is checked, so a row reruns when b stored {a,b}
    const bool hit = pc->directed ? (ra != kNoRank && ra < rb) : (ra != kNoRank || rb != kNoRank);
    bool failed = false;
    if (!hit) {
        if (pc->h_rank[a] == kNoRank) {
            int rc = run_row_for_min(pc, a);
            if (rc) return rc;
            pc->h_rank[a] = pc->next_rank++;
        }
        // the row fails as a whole when its [a] entry has no self-loop
        // (computePathProperties returns FALSE, topology.c:1490-1495, 1857)
        if (pc->h_self_eid[a] < 0) failed = true;
        ra = pc->h_rank[a];
    }
    if (failed) { *lat = -1; *rel = -1; return SHD_OK; }
    // value from whichever endpoint's row ran first; on directed graphs this can
    // be the reverse path (topology.c:2034-2037)
    if (ra != kNoRank && (rb == kNoRank || ra < rb))
        return fetch2(pc, pc->d_row, (size_t)a * T + b, lat, rel);
    return fetch2(pc, pc->d_row, (size_t)b * T + a, lat, rel);
}

// ------------------------------------------------------------------ batched lazy lookup
// shd_pc_lookup over a list of queries in their order, with one upload, one
// gather kernel and one download instead of a device round trip per query:
// the rank rule (pc_lookup_at) runs on the host to name each query's table
// entry, the entries are gathered on the device, and the rows the batch ranks
// fold their newly stored entries into minimumPathLatency on the device
// (run_row_for_min's rule, with "stored when the row ran" read off the final
// ranks: a target stored before row a ran has a smaller rank than a's).
enum : uint8_t { kPvDir = 0, kPvSelf = 1, kPvRow = 2, kPvFail = 3 };

__global__ void k_pc_gather(const uint8_t* __restrict__ kind, const uint64_t* __restrict__ idx, uint64_t n,
                            const shd_pv* __restrict__ dir, const shd_pv* __restrict__ self,
                            const shd_pv* __restrict__ row, shd_pv* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t k = kind[i];
        shd_pv v{-1.0, -1.0};
        if (k == kPvDir) v = dir[idx[i]];
        else if (k == kPvSelf) v = self[idx[i]];
        else if (k == kPvRow) v = row[idx[i]];
        out[i] = v;
    }
}

// min over the entries each newly ranked row stored (rows[j] ranked rrank[j])
__global__ void k_pc_newrow_min(const int32_t* __restrict__ rows, const int32_t* __restrict__ rrank, int32_t nr,
                                int32_t T, const int32_t* __restrict__ rank, const int32_t* __restrict__ self_rank,
                                const shd_pv* __restrict__ row, const uint8_t* __restrict__ adj, int prefer_direct,
                                unsigned long long* __restrict__ out) {
    __shared__ unsigned long long sm[256];
    unsigned long long m = kDistInf;
    const size_t n = (size_t)nr * T;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int32_t j = (int32_t)(i / T), t = (int32_t)(i % T), a = rows[j], R = rrank[j];
        const bool stored = t == a ? self_rank[a] < R : rank[t] < R;
        if (stored) continue;
        if (prefer_direct && adj[(size_t)a * T + t]) continue;
        const double lat = row[(size_t)a * T + t].lat;
        if (!(lat >= 0.0)) continue;
        const unsigned long long b = (unsigned long long)__double_as_longlong(lat);
        m = b < m ? b : m;
    }
    sm[threadIdx.x] = m;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k && sm[threadIdx.x + k] < sm[threadIdx.x]) sm[threadIdx.x] = sm[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMin(out, sm[0]);
}

extern "C" int shd_pc_lookup_batch(shd_pc* pc, const int32_t* src_vertex, const int32_t* dst_vertex, uint64_t n,
                                   double* lat, double* rel) {
    if (!pc || !pc->built || (n && (!src_vertex || !dst_vertex || !lat || !rel))) return SHD_EINVAL;
    for (uint64_t i = 0; i < n; i++)
        if (src_vertex[i] < 0 || dst_vertex[i] < 0 || src_vertex[i] >= pc->V || dst_vertex[i] >= pc->V ||
            pc->h_att_index[src_vertex[i]] < 0 || pc->h_att_index[dst_vertex[i]] < 0)
            return SHD_EINVAL;
    PcTouches* tch = (PcTouches*)pc->touches;
    if ((tch && tch->on) || (!pc->complete && !pc->rows_mode)) {   // the co-simulation's protocol: query by query
        for (uint64_t i = 0; i < n; i++) {
            const int rc = shd_pc_lookup(pc, src_vertex[i], dst_vertex[i], &lat[i], &rel[i]);
            if (rc) return rc;
        }
        return SHD_OK;
    }
    if (!n) return SHD_OK;
    const int32_t T = pc->T;
    std::vector<uint8_t> kind(n);
    std::vector<uint64_t> idx(n);
    std::vector<int32_t> nrow, nrank;
    for (uint64_t i = 0; i < n; i++) {   // pc_lookup_at's rule, deciding the entry only
        const int32_t a = pc->h_att_index[src_vertex[i]], b = pc->h_att_index[dst_vertex[i]];
        const bool adj = pc->prefer_direct && !pc->complete &&
                         shd_csr_get_eid(&pc->csr, pc->h_attached[a], pc->h_attached[b]) >= 0;
        if (pc->complete || adj) { kind[i] = kPvDir; idx[i] = (uint64_t)a * T + b; continue; }
        if (a == b) {
            int32_t ra = pc->h_rank[a], rs = pc->h_self_rank[a];
            if (ra == kNoRank && rs == kNoRank) pc->h_self_rank[a] = rs = pc->next_rank++;
            if (rs < ra) { kind[i] = kPvSelf; idx[i] = (uint64_t)a; }
            else { kind[i] = kPvRow; idx[i] = (uint64_t)a * T + a; }
            continue;
        }
        int32_t ra = pc->h_rank[a], rb = pc->h_rank[b];
        const bool hit = pc->directed ? (ra != kNoRank && ra < rb) : (ra != kNoRank || rb != kNoRank);
        if (!hit) {
            if (pc->h_rank[a] == kNoRank) {
                pc->h_rank[a] = pc->next_rank++;
                nrow.push_back(a);
                nrank.push_back(pc->h_rank[a]);
            }
            ra = pc->h_rank[a];
            if (pc->h_self_eid[a] < 0) { kind[i] = kPvFail; idx[i] = 0; continue; }
        }
        kind[i] = kPvRow;
        idx[i] = (ra != kNoRank && (rb == kNoRank || ra < rb)) ? (uint64_t)a * T + b : (uint64_t)b * T + a;
    }
    SHD_HIP(hipSetDevice(pc->device));
    hipStream_t s = pc->stream;
    uint8_t* d_kind = nullptr;
    uint64_t* d_idx = nullptr;
    shd_pv* d_out = nullptr;
    int32_t *d_rows = nullptr, *d_rrank = nullptr, *d_rank = nullptr, *d_srank = nullptr;
    unsigned long long* d_min = nullptr;
    std::vector<shd_pv> out(n);
    unsigned long long mn = kDistInf;
    int rc = SHD_OK;
    const size_t nr = nrow.size();
    if (hipMalloc(&d_kind, n) != hipSuccess || hipMalloc(&d_idx, 8 * n) != hipSuccess ||
        hipMalloc(&d_out, sizeof(shd_pv) * n) != hipSuccess || hipMalloc(&d_min, 8) != hipSuccess ||
        (nr && (hipMalloc(&d_rows, 4 * nr) != hipSuccess || hipMalloc(&d_rrank, 4 * nr) != hipSuccess ||
                hipMalloc(&d_rank, 4 * (size_t)T) != hipSuccess || hipMalloc(&d_srank, 4 * (size_t)T) != hipSuccess))) {
        rc = SHD_ENOMEM;
        goto done;
    }
    if (hipMemcpyAsync(d_kind, kind.data(), n, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_idx, idx.data(), 8 * n, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_min, &mn, 8, hipMemcpyHostToDevice, s) != hipSuccess) { rc = SHD_ENODEV; goto done; }
    hipLaunchKernelGGL(k_pc_gather, dim3((unsigned)std::min<uint64_t>((n + 255) / 256, 4096)), dim3(256), 0, s,
                       d_kind, d_idx, n, pc->d_dir, pc->d_self, pc->d_row, d_out);
    if (nr) {
        if (hipMemcpyAsync(d_rows, nrow.data(), 4 * nr, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemcpyAsync(d_rrank, nrank.data(), 4 * nr, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemcpyAsync(d_rank, pc->h_rank, 4 * (size_t)T, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemcpyAsync(d_srank, pc->h_self_rank, 4 * (size_t)T, hipMemcpyHostToDevice, s) != hipSuccess) {
            rc = SHD_ENODEV;
            goto done;
        }
        const size_t tot = nr * (size_t)T;
        hipLaunchKernelGGL(k_pc_newrow_min, dim3((unsigned)std::min<size_t>((tot + 255) / 256, 2048)), dim3(256), 0, s,
                           d_rows, d_rrank, (int32_t)nr, T, d_rank, d_srank, pc->d_row, pc->d_adj,
                           pc->prefer_direct, d_min);
    }
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(out.data(), d_out, sizeof(shd_pv) * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(&mn, d_min, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
        rc = SHD_ENODEV;
        goto done;
    }
    // minimumPathLatency: the new rows' stored entries (in rank order, min is
    // order-free), then the direct and self values as pc_lookup_at notes them
    if (nr && mn != kDistInf) {
        double m;
        memcpy(&m, &mn, 8);
        note_min(pc, m);
    }
    for (uint64_t i = 0; i < n; i++) {
        double l = out[i].lat, r = out[i].rel;
        if (kind[i] == kPvDir) {
            if (isnan(l)) { l = -1; r = -1; }
            else note_min(pc, l);
        } else if (kind[i] == kPvSelf) {
            if (l >= 0) note_min(pc, l);
        }
        lat[i] = l;
        rel[i] = r;
    }
done:
    for (void* q : {(void*)d_kind, (void*)d_idx, (void*)d_out, (void*)d_rows, (void*)d_rrank, (void*)d_rank,
                    (void*)d_srank, (void*)d_min})
        if (q) (void)hipFree(q);
    return rc;
}

extern "C" int shd_pc_count_packet(shd_pc* pc, int32_t sv, int32_t dv) {
    double lat, rel;
    int rc = shd_pc_lookup(pc, sv, dv, &lat, &rel);
    if (rc) return rc;
    if (lat < 0) return SHD_OK;
    auto* m = (std::unordered_map<uint64_t, uint64_t>*)pc->counts;
    int32_t a = pc->h_att_index[sv], b = pc->h_att_index[dv];
    uint64_t key = ((uint64_t)(uint32_t)std::min(a, b) << 32) | (uint32_t)std::max(a, b);
    (*m)[key]++;
    return SHD_OK;
}

extern "C" int shd_pc_packet_count(shd_pc* pc, int32_t sv, int32_t dv, uint64_t* count) {
    if (!pc || !count || sv < 0 || dv < 0 || sv >= pc->V || dv >= pc->V) return SHD_EINVAL;
    int32_t a = pc->h_att_index[sv], b = pc->h_att_index[dv];
    if (a < 0 || b < 0) return SHD_EINVAL;
    auto* m = (std::unordered_map<uint64_t, uint64_t>*)pc->counts;
    uint64_t key = ((uint64_t)(uint32_t)std::min(a, b) << 32) | (uint32_t)std::max(a, b);
    auto it = m->find(key);
    *count = it == m->end() ? 0 : it->second;
    return SHD_OK;
}

extern "C" int shd_pc_min_time_jump(shd_pc* pc, uint64_t runahead_ns, uint64_t* jump_ns) {
    if (!pc || !jump_ns) return SHD_EINVAL;
    // master_updateMinTimeJump (master.c:148-159): floor(ms) * 1e6 ns;
    // _master_getMinTimeJump (133-146): 10 ms default if 0, >= runahead
    uint64_t j = (uint64_t)floor(pc->min_stored_latency) * SHD_MS;
    if (j == 0) j = 10 * SHD_MS;
    if (runahead_ns > j) j = runahead_ns;
    *jump_ns = j;
    return SHD_OK;
}

// minimumPathLatency after a run that ranked rows on the device (shd_tcp_run's
// path_cache mode, pc->h_rank / h_self_rank holding the run's final ranks,
// old_rank / old_self the ranks before it): the entries each newly ranked row
// stored (k_pc_newrow_min, run_row_for_min's rule) and each newly stored self
// path (pc_lookup_at's self branch) are folded in.  The direct entries of a
// complete graph, which pc_lookup_at notes on every lookup, are not: the
// device path keeps no list of the pairs it queried
__attribute__((visibility("hidden"))) int shd_pc_fold_ranked(shd_pc* pc, const int32_t* old_rank,
                                                             const int32_t* old_self) {
    if (!pc || pc->complete || !pc->d_row) return SHD_OK;
    const int32_t T = pc->T;
    std::vector<int32_t> nrow, nrank;
    bool new_self = false;
    for (int32_t a = 0; a < T; a++) {
        if (old_rank[a] == kNoRank && pc->h_rank[a] != kNoRank) { nrow.push_back(a); nrank.push_back(pc->h_rank[a]); }
        new_self |= old_self[a] == kNoRank && pc->h_self_rank[a] != kNoRank;
    }
    SHD_HIP(hipSetDevice(pc->device));
    if (new_self) {
        std::vector<shd_pv> sv(T);
        SHD_HIP(hipMemcpy(sv.data(), pc->d_self, sizeof(shd_pv) * (size_t)T, hipMemcpyDeviceToHost));
        for (int32_t a = 0; a < T; a++)
            if (old_self[a] == kNoRank && pc->h_self_rank[a] != kNoRank && pc->h_self_rank[a] < pc->h_rank[a] &&
                sv[a].lat >= 0)
                note_min(pc, sv[a].lat);
    }
    if (nrow.empty()) return SHD_OK;
    const size_t nr = nrow.size();
    int32_t *d_rows = nullptr, *d_rrank = nullptr, *d_rank = nullptr, *d_srank = nullptr;
    unsigned long long* d_min = nullptr;
    unsigned long long mn = kDistInf;
    int rc = SHD_OK;
    hipStream_t s = pc->stream;
    if (hipMalloc(&d_rows, 4 * nr) != hipSuccess || hipMalloc(&d_rrank, 4 * nr) != hipSuccess ||
        hipMalloc(&d_rank, 4 * (size_t)T) != hipSuccess || hipMalloc(&d_srank, 4 * (size_t)T) != hipSuccess ||
        hipMalloc(&d_min, 8) != hipSuccess) {
        rc = SHD_ENOMEM;
    } else if (hipMemcpyAsync(d_rows, nrow.data(), 4 * nr, hipMemcpyHostToDevice, s) != hipSuccess ||
               hipMemcpyAsync(d_rrank, nrank.data(), 4 * nr, hipMemcpyHostToDevice, s) != hipSuccess ||
               hipMemcpyAsync(d_rank, pc->h_rank, 4 * (size_t)T, hipMemcpyHostToDevice, s) != hipSuccess ||
               hipMemcpyAsync(d_srank, pc->h_self_rank, 4 * (size_t)T, hipMemcpyHostToDevice, s) != hipSuccess ||
               hipMemcpyAsync(d_min, &mn, 8, hipMemcpyHostToDevice, s) != hipSuccess) {
        rc = SHD_ENODEV;
    } else {
        const size_t tot = nr * (size_t)T;
        hipLaunchKernelGGL(k_pc_newrow_min, dim3((unsigned)std::min<size_t>((tot + 255) / 256, 2048)), dim3(256), 0, s,
                           d_rows, d_rrank, (int32_t)nr, T, d_rank, d_srank, pc->d_row, pc->d_adj, pc->prefer_direct,
                           d_min);
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(&mn, d_min, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            rc = SHD_ENODEV;
        else if (mn != kDistInf) {
            double m;
            memcpy(&m, &mn, 8);
            note_min(pc, m);
        }
    }
    for (void* q : {(void*)d_rows, (void*)d_rrank, (void*)d_rank, (void*)d_srank, (void*)d_min})
        if (q) (void)hipFree(q);
    return rc;
}

extern "C" int shd_pc_min_stored_latency(shd_pc* pc, double* ms) {
    if (!pc || !ms) return SHD_EINVAL;
    *ms = pc->min_stored_latency;
    return SHD_OK;
}

extern "C" void shd_pc_destroy(shd_pc* pc) {
    if (!pc) return;
    (void)hipSetDevice(pc->device);
    pc_free_device(pc);
    if (pc->stream) (void)hipStreamDestroy(pc->stream);
    shd_csr_free(&pc->csr);
    free(pc->h_attached); free(pc->h_att_index); free(pc->h_w); free(pc->h_eloss); free(pc->h_vloss);
    free(pc->h_self_eid); free(pc->h_rank); free(pc->h_self_rank); free(pc->h_direct_stored);
    delete (std::unordered_map<uint64_t, uint64_t>*)pc->counts;
    delete (PcTouches*)pc->touches;
    delete pc;
}
