/*
 * o_rng.c -- TEST INFRASTRUCTURE (oracle).  Restates utility/random.c over the
 * glibc rand_r algorithm, and the seed chain of master.c / slave.c.
 */
#include <math.h>
#include <stdint.h>

#include "oracle.h"

/* glibc stdlib/rand_r.c: three LCG steps, 11 + 10 + 10 output bits. */
int32_t o_rand_r(uint32_t* state) {
    uint32_t next = *state;
    int32_t result;
    next *= 1103515245u;
    next += 12345u;
    result = (int32_t)((next / 65536u) % 2048u);
    next *= 1103515245u;
    next += 12345u;
    result <<= 10;
    result ^= (int32_t)((next / 65536u) % 1024u);
    next *= 1103515245u;
    next += 12345u;
    result <<= 10;
    result ^= (int32_t)((next / 65536u) % 1024u);
    *state = next;
    return result;
}

/* random_nextDouble, random.c:39-43 (RAND_MAX = 2147483647) */
double o_next_double(uint32_t* state) {
    int32_t v = o_rand_r(state);
    return (double)(((double)v) / ((double)2147483647));
}

/* random_nextUInt, random.c:45-51 */
uint32_t o_next_uint(uint32_t* state) {
    double f = o_next_double(state);
    double maxUint = (double)UINT32_MAX;
    return (uint32_t)(f * maxUint);
}

/* master_new: random_new(options seed) (master.c:95); master_run:
 * slaveSeed = random_nextUInt(master) (master.c:417); slave_new: random_new
 * (slaveSeed) (slave.c:182), schedulerSeed = nextUInt (slave.c:198);
 * slave_addNewVirtualHost: nodeSeed = nextUInt per host in registration order
 * (slave.c:301). */
int o_seed_chain(uint32_t options_seed, int32_t n_hosts, uint32_t* host_seeds) {
    uint32_t master = options_seed;
    uint32_t slave = o_next_uint(&master);
    (void)o_next_uint(&slave); /* scheduler seed */
    for (int32_t i = 0; i < n_hosts; i++) host_seeds[i] = o_next_uint(&slave);
    return 0;
}
