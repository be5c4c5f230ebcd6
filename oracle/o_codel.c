/*
 * o_codel.c -- TEST INFRASTRUCTURE (oracle).  Restates the CoDel router queue
 * of src/main/routing/router_queue_codel.c (enqueue 113-137, dequeue helper
 * 148-196, control law 198-205, dequeue 207-267).  Pinned against the
 * reference file itself compiled into oracle/_ref (tests/test_oracle_ref.py).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define TARGET (10ULL * SHD_MS)     /* CODEL_PARAM_TARGET_DELAY_SIMTIME, :42 */
#define INTERVAL (100ULL * SHD_MS)  /* CODEL_PARAM_INTERVAL_SIMTIME, :48     */

void o_codel_init(o_codel* c, uint32_t cap) {
    memset(c, 0, sizeof(*c));
    c->cap = cap;
    c->q = calloc(cap, sizeof(o_codel_entry));
}
void o_codel_free(o_codel* c) { free(c->q); c->q = NULL; }

int o_codel_enqueue(o_codel* c, uint64_t now, uint32_t len, uint32_t id, uint32_t src) {
    if (c->count >= c->cap) {   /* grow: the reference limit is G_MAXUINT */
        uint32_t ncap = c->cap ? c->cap * 2 : 16;
        o_codel_entry* nq = calloc(ncap, sizeof(o_codel_entry));
        for (uint32_t i = 0; i < c->count; i++) nq[i] = c->q[(c->head + i) % c->cap];
        free(c->q); c->q = nq; c->cap = ncap; c->head = 0;
    }
    o_codel_entry* e = &c->q[(c->head + c->count) % c->cap];
    e->ts = now; e->len = len; e->id = id; e->src = src; e->_pad = 0;
    c->count++;
    c->total += len;
    return 1;
}

static int dequeue_helper(o_codel* c, uint64_t now, int* okToDrop, o_codel_entry* out) {
    *okToDrop = 0;
    if (c->count == 0) { c->interval_expire = 0; return 0; }
    *out = c->q[c->head];
    c->head = (c->head + 1) % c->cap;
    c->count--;
    c->total -= out->len;
    uint64_t sojourn = now - out->ts;
    if (sojourn < TARGET || c->total < SHD_MTU) {
        c->interval_expire = 0;
    } else {
        if (c->interval_expire == 0) c->interval_expire = now + INTERVAL;
        else if (now >= c->interval_expire) *okToDrop = 1;
    }
    return 1;
}

uint64_t o_codel_control_law(uint32_t count, uint64_t ts) {
    uint64_t newTS = ts + INTERVAL;
    double result = ((double)newTS) / sqrt((double)count);
    double rounded = round(result);
    return (uint64_t)rounded;
}

int o_codel_dequeue(o_codel* c, uint64_t now, o_codel_entry* out, o_codel_entry* drops,
                    uint32_t ndrops_cap, uint32_t* ndrops) {
    int okToDrop = 0;
    *ndrops = 0;
    o_codel_entry pkt;
    int have = dequeue_helper(c, now, &okToDrop, &pkt);
    if (!have) { c->mode = 0; return 0; }
    if (c->mode == 1) {
        if (!okToDrop) c->mode = 0;
        while (now >= c->next_drop && c->mode == 1) {
            if (*ndrops < ndrops_cap) drops[*ndrops] = pkt;
            (*ndrops)++;
            c->drop_count++;
            have = dequeue_helper(c, now, &okToDrop, &pkt);
            if (okToDrop) c->next_drop = o_codel_control_law(c->drop_count, c->next_drop);
            else c->mode = 0;
        }
    } else if (okToDrop) {
        if (*ndrops < ndrops_cap) drops[*ndrops] = pkt;
        (*ndrops)++;
        have = dequeue_helper(c, now, &okToDrop, &pkt);
        c->mode = 1;
        uint32_t delta = c->drop_count - c->drop_count_last;
        c->drop_count = 1;
        int droppingRecently = (now < c->next_drop + (16 * INTERVAL)) ? 1 : 0;
        if (droppingRecently && delta > 1) c->drop_count = delta;
        c->next_drop = o_codel_control_law(c->drop_count, now);
        c->drop_count_last = c->drop_count;
    }
    if (!have) return 0;
    *out = pkt;
    return 1;
}
