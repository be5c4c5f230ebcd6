/*
 * shd_xhost.c -- the host-memory transport of the engine group (shd_comm of
 * kind "host"): ranks are processes on one machine (any GPUs, or one GPU
 * shared), meeting in a POSIX shared-memory segment.  It carries the same
 * collectives the RCCL transport does (all-to-all of the per-round blocks,
 * all-gather of first-touch logs and row shards, the spill exchange), staged
 * through host memory: the per-round exchange of slave.c:437-462's rounds
 * without a GPU interconnect, so the group protocol can run with several
 * processes where RCCL cannot (RCCL refuses two ranks on one device).
 *
 * Segment: a header (barrier count and generation), then `world` scratch
 * slots of `slot` bytes.  A collective writes the caller's part into its
 * slot, meets at the barrier, reads what it needs, meets again; larger
 * payloads go in pieces of the slot size.  Rank 0 creates the segment
 * (exclusively: a segment of that name left by an earlier group -- one whose
 * rank 0 died before unlinking it, or whose barrier broke -- is marked
 * superseded, unlinked and created afresh) and unlinks it at close; the other
 * ranks wait for rank 0's `ready` word, and drop a segment that is broken or
 * superseded and open the name again.  Callers still derive the name from a
 * random token, as RCCL's unique id.  Joining is a handshake with a live rank
 * 0: a joiner posts a fresh token of its own in its arrival slot and waits for
 * rank 0 to echo it back, so a stale segment (whose rank 0 is gone, but which
 * still reads ready and may hold a leftover barrier count) never lets a joiner
 * through; it waits there until the new rank 0 marks that segment superseded,
 * then opens the name again.
 */
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "shd_host.h"

struct shd_xhost_hdr {
    uint32_t count;       /* arrivals at the current barrier */
    uint32_t gen;         /* barrier generation */
    uint32_t world;
    uint32_t broken;      /* set by a rank whose barrier timed out: every barrier fails */
    uint32_t ready;       /* kReady once rank 0 has initialised the segment */
    uint32_t superseded;  /* set by a rank 0 that replaced this (stale) segment */
    uint32_t _pad[2];
    uint64_t arrived[64]; /* joiner r's token (0: not yet), rank 0 echoes it in ack[r] */
    uint64_t ack[64];
};
enum { kReady = 0x58484F53u };
enum { kHdrBytes = (sizeof(struct shd_xhost_hdr) + 63) & ~63 };

struct shd_xhost {
    char name[128];
    int world, rank, fd;
    size_t slot;          /* scratch bytes per rank */
    size_t map_bytes;
    char* base;           /* mapping: header, then world slots */
    double timeout_s;
};

static char* slot_ptr(shd_xhost* x, int r) { return x->base + kHdrBytes + (size_t)r * x->slot; }

static double mono_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

/* rank 0: a fresh zero-filled segment under the name, replacing a stale one */
static int xhost_create(shd_xhost* x) {
    for (int tries = 0; tries < 4; tries++) {
        x->fd = shm_open(x->name, O_RDWR | O_CREAT | O_EXCL, 0600);
        if (x->fd >= 0) break;
        if (errno != EEXIST) return SHD_ENODEV;
        const int old = shm_open(x->name, O_RDWR, 0600);
        if (old >= 0) {
            struct stat so;
            if (fstat(old, &so) == 0 && (size_t)so.st_size >= sizeof(struct shd_xhost_hdr)) {
                void* m = mmap(NULL, sizeof(struct shd_xhost_hdr), PROT_READ | PROT_WRITE, MAP_SHARED, old, 0);
                if (m != MAP_FAILED) {
                    __atomic_store_n(&((struct shd_xhost_hdr*)m)->superseded, 1u, __ATOMIC_RELEASE);
                    munmap(m, sizeof(struct shd_xhost_hdr));
                }
            }
            close(old);
        }
        fprintf(stderr, "libshdgpu: host transport %s: replacing a stale segment of that name\n", x->name);
        shm_unlink(x->name);
    }
    if (x->fd < 0) return SHD_ENODEV;
    if (ftruncate(x->fd, (off_t)x->map_bytes) != 0) { close(x->fd); shm_unlink(x->name); return SHD_ENOMEM; }
    x->base = mmap(NULL, x->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, x->fd, 0);
    if (x->base == MAP_FAILED) { close(x->fd); shm_unlink(x->name); return SHD_ENOMEM; }
    struct shd_xhost_hdr* h = (struct shd_xhost_hdr*)x->base;
    h->world = (uint32_t)x->world;
    __atomic_store_n(&h->ready, (uint32_t)kReady, __ATOMIC_RELEASE);
    /* echo every joiner's token (this segment is fresh: only live joiners post) */
    const double t0 = mono_s();
    for (int r = 1; r < x->world; r++) {
        uint64_t tok;
        while ((tok = __atomic_load_n(&h->arrived[r], __ATOMIC_ACQUIRE)) == 0) {
            if (mono_s() - t0 > x->timeout_s) {
                fprintf(stderr, "libshdgpu: host transport %s: rank %d never joined in %.0f s\n", x->name, r,
                        x->timeout_s);
                __atomic_store_n(&h->broken, 1u, __ATOMIC_RELEASE);
                munmap(x->base, x->map_bytes);
                close(x->fd);
                shm_unlink(x->name);
                return SHD_ENODEV;
            }
            usleep(100);
        }
        __atomic_store_n(&h->ack[r], tok, __ATOMIC_RELEASE);
    }
    return SHD_OK;
}

/* the other ranks: rank 0's segment once it is ready (a broken or superseded
 * one is dropped and the name opened again), within the barrier timeout */
static int xhost_join(shd_xhost* x) {
    const double t0 = mono_s();
    for (;;) {
        if (mono_s() - t0 > x->timeout_s) {
            fprintf(stderr, "libshdgpu: host transport %s: rank %d found no ready segment in %.0f s\n", x->name,
                    x->rank, x->timeout_s);
            return SHD_ENODEV;
        }
        x->fd = shm_open(x->name, O_RDWR, 0600);
        if (x->fd < 0) {
            if (errno != ENOENT) return SHD_ENODEV;
            usleep(200);
            continue;
        }
        struct stat st;
        if (fstat(x->fd, &st) != 0 || (size_t)st.st_size < x->map_bytes) {   /* not sized yet (or stale) */
            close(x->fd);
            usleep(200);
            continue;
        }
        x->base = mmap(NULL, x->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, x->fd, 0);
        if (x->base == MAP_FAILED) { close(x->fd); return SHD_ENOMEM; }
        struct shd_xhost_hdr* h = (struct shd_xhost_hdr*)x->base;
        for (;;) {
            const int bad = __atomic_load_n(&h->superseded, __ATOMIC_ACQUIRE) ||
                            __atomic_load_n(&h->broken, __ATOMIC_ACQUIRE);
            if (!bad && __atomic_load_n(&h->ready, __ATOMIC_ACQUIRE) == (uint32_t)kReady) {
                if (h->world != (uint32_t)x->world) { munmap(x->base, x->map_bytes); close(x->fd); return SHD_EINVAL; }
                /* the handshake: a token only this call knows, echoed by a live rank 0 */
                struct timespec ts;
                clock_gettime(CLOCK_MONOTONIC, &ts);
                uint64_t tok = ((uint64_t)getpid() << 32) ^ (uint64_t)ts.tv_nsec ^ ((uint64_t)ts.tv_sec << 20) ^
                               ((uint64_t)x->rank << 56);
                if (!tok) tok = 1;
                __atomic_store_n(&h->arrived[x->rank], tok, __ATOMIC_RELEASE);
                for (;;) {
                    if (__atomic_load_n(&h->ack[x->rank], __ATOMIC_ACQUIRE) == tok) return SHD_OK;
                    if (__atomic_load_n(&h->superseded, __ATOMIC_ACQUIRE) ||
                        __atomic_load_n(&h->broken, __ATOMIC_ACQUIRE) || mono_s() - t0 > x->timeout_s)
                        break;
                    usleep(100);
                }
                break;
            }
            if (bad || mono_s() - t0 > x->timeout_s) break;
            usleep(100);
        }
        munmap(x->base, x->map_bytes);
        close(x->fd);
        usleep(200);
    }
}

int shd_xhost_open(const char* name, int world, int rank, size_t slot_bytes, shd_xhost** out) {
    if (!name || !*name || strlen(name) > 100 || world <= 0 || world > 64 || rank < 0 || rank >= world ||
        !slot_bytes || !out)
        return SHD_EINVAL;
    shd_xhost* x = calloc(1, sizeof(*x));
    if (!x) return SHD_ENOMEM;
    snprintf(x->name, sizeof(x->name), "/%s", name[0] == '/' ? name + 1 : name);
    x->world = world;
    x->rank = rank;
    x->slot = (slot_bytes + 63) & ~(size_t)63;
    x->map_bytes = kHdrBytes + (size_t)world * x->slot;
    const char* to = getenv("SHD_XHOST_TIMEOUT");
    x->timeout_s = to ? atof(to) : 300.0;
    const int rc = rank == 0 ? xhost_create(x) : xhost_join(x);
    if (rc) { free(x); return rc; }
    *out = x;
    return shd_xhost_barrier(x);
}

/* a generation barrier; SHD_ENODEV if the others do not arrive in time.  A
 * timeout breaks the group for good (its arrival count can no longer be
 * trusted): the ranks waiting, and every later barrier, fail at once. */
int shd_xhost_barrier(shd_xhost* x) {
    struct shd_xhost_hdr* h = (struct shd_xhost_hdr*)x->base;
    if (__atomic_load_n(&h->broken, __ATOMIC_ACQUIRE) || __atomic_load_n(&h->superseded, __ATOMIC_ACQUIRE))
        return SHD_ENODEV;
    const uint32_t g = __atomic_load_n(&h->gen, __ATOMIC_ACQUIRE);
    if (__atomic_add_fetch(&h->count, 1, __ATOMIC_ACQ_REL) == (uint32_t)x->world) {
        __atomic_store_n(&h->count, 0, __ATOMIC_RELAXED);
        __atomic_store_n(&h->gen, g + 1, __ATOMIC_RELEASE);
        return SHD_OK;
    }
    const double t0 = mono_s();
    unsigned spins = 0;
    while (__atomic_load_n(&h->gen, __ATOMIC_ACQUIRE) == g) {
        if (++spins > 1000) sched_yield();
        if (__atomic_load_n(&h->broken, __ATOMIC_ACQUIRE) || __atomic_load_n(&h->superseded, __ATOMIC_ACQUIRE))
            return SHD_ENODEV;
        if ((spins & 0xFFF) == 0 && mono_s() - t0 > x->timeout_s) {
            fprintf(stderr, "libshdgpu: host transport %s: rank %d waited %.0f s at a barrier\n", x->name, x->rank,
                    x->timeout_s);
            __atomic_store_n(&h->broken, 1u, __ATOMIC_RELEASE);
            return SHD_ENODEV;
        }
    }
    return SHD_OK;
}

/* out[r] = the `bytes` each rank r passed (out: world * bytes) */
int shd_xhost_allgather(shd_xhost* x, const void* mine, size_t bytes, void* out) {
    const size_t piece = x->slot;
    for (size_t off = 0; off < bytes || (bytes == 0 && off == 0); off += piece) {
        const size_t n = bytes - off < piece ? bytes - off : piece;
        if (n) memcpy(slot_ptr(x, x->rank), (const char*)mine + off, n);
        int rc = shd_xhost_barrier(x);
        if (rc) return rc;
        for (int r = 0; r < x->world && n; r++) memcpy((char*)out + (size_t)r * bytes + off, slot_ptr(x, r), n);
        if ((rc = shd_xhost_barrier(x))) return rc;
        if (bytes == 0) break;
    }
    return SHD_OK;
}

/* send: world blocks of `bytes` (block p for rank p); recv: world blocks
 * (block p from rank p) */
int shd_xhost_alltoall(shd_xhost* x, const void* send, size_t bytes, void* recv) {
    const int W = x->world;
    const size_t piece = x->slot / (size_t)W;
    if (!piece) return SHD_ERANGE;
    for (size_t off = 0; off < bytes; off += piece) {
        const size_t n = bytes - off < piece ? bytes - off : piece;
        char* mine = slot_ptr(x, x->rank);
        for (int p = 0; p < W; p++) memcpy(mine + (size_t)p * piece, (const char*)send + (size_t)p * bytes + off, n);
        int rc = shd_xhost_barrier(x);
        if (rc) return rc;
        for (int p = 0; p < W; p++)
            memcpy((char*)recv + (size_t)p * bytes + off, slot_ptr(x, p) + (size_t)x->rank * piece, n);
        if ((rc = shd_xhost_barrier(x))) return rc;
    }
    return SHD_OK;
}

void shd_xhost_close(shd_xhost* x) {
    if (!x) return;
    (void)shd_xhost_barrier(x);   /* nobody is inside a collective any more */
    munmap(x->base, x->map_bytes);
    close(x->fd);
    if (x->rank == 0) shm_unlink(x->name);
    free(x);
}
