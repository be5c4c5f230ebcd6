/*
 * shd_host.h -- internal host-side structures of libshdgpu (not part of the
 * C-ABI).  The CSR built here is the device layout of the topology graph.
 */
#ifndef SHD_HOST_H
#define SHD_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "../../include/shdgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/*
 * Graph index in the orders the reference depends on:
 *  - inc_*: igraph_incident(v, IGRAPH_OUT) order (undirected: edges stored with
 *    from=max, to=min; out-list sorted by (to,eid) then in-list sorted by
 *    (from,eid); a self-loop appears in both).  Used by the self-path scan
 *    (topology.c:1559-1603, first strict minimum).
 *  - arc_*: relaxation arcs v -> x for SSSP (self-loops dropped; they never
 *    improve a distance), with the arc weight copied next to the head so one
 *    relaxation reads 12 contiguous bytes.
 *  - rin_*: reverse arcs x <- v (for undirected graphs identical to arc_*),
 *    used to pick each vertex's shortest-path parent after convergence.
 *  - nbr_*: per-vertex neighbour list sorted by (neighbour, eid) for
 *    igraph_get_eid (lowest eid among parallel edges).
 */
typedef struct shd_csr {
    int32_t V, E, directed;
    int32_t* inc_off; int32_t* inc_eid;
    int32_t* arc_off; int32_t* arc_dst; int32_t* arc_eid; double* arc_w;
    int32_t* rin_off; int32_t* rin_src; int32_t* rin_eid; double* rin_w;
    int32_t* nbr_off; int32_t* nbr_v; int32_t* nbr_eid;
    int32_t max_degree;
} shd_csr;

__attribute__((visibility("hidden"))) int shd_csr_build(const shd_graph* g, shd_csr* out);
__attribute__((visibility("hidden"))) void shd_csr_free(shd_csr* c);
__attribute__((visibility("hidden"))) int32_t shd_csr_get_eid(const shd_csr* c, int32_t a, int32_t b);

/* host-memory transport of an engine group (shd_xhost.c): processes of one
 * machine meeting in a POSIX shared-memory segment */
typedef struct shd_xhost shd_xhost;
__attribute__((visibility("hidden"))) int shd_xhost_open(const char* name, int world, int rank, size_t slot_bytes,
                                                         shd_xhost** out);
__attribute__((visibility("hidden"))) int shd_xhost_barrier(shd_xhost* x);
__attribute__((visibility("hidden"))) int shd_xhost_allgather(shd_xhost* x, const void* mine, size_t bytes,
                                                              void* out);
__attribute__((visibility("hidden"))) int shd_xhost_alltoall(shd_xhost* x, const void* send, size_t bytes,
                                                             void* recv);
__attribute__((visibility("hidden"))) void shd_xhost_close(shd_xhost* x);

#ifdef __cplusplus
}
#endif
#endif
