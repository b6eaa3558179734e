/*
 * msa_ranks_test -- CPU test of the C host's rank layer (msa_ranks.c): the
 * launcher, the shm transport's all-gather and all-to-all-v, and the shard
 * routing, with N forked ranks and no GPU.  Exit 0 = every check passed.
 *
 *   msa_ranks_test routing
 *   msa_ranks_test exchange N     (N ranks: all-gather, all-to-all-v, barrier)
 *   msa_ranks_test fail N         (rank N-1 fails: the launcher must return its
 *                                  code without hanging the others)
 *   mpirun -np N msa_ranks_test launched [fail]
 *                                 (the same checks with N processes an external
 *                                  launcher started: they join as one job)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "msa_ranks.h"

#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            fprintf(stderr, "check failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                       \
        }                                                                   \
    } while (0)

static int routing(void) {
    /* mirrors tests/test_dist.py::test_head_owners / test_tail_plan */
    int owner[4];
    const uint64_t h1[4] = {0, 5, 0, 3}, s1[4] = {10, 10, 10, 10};
    msa_head_owners(h1, s1, 4, owner);
    CHECK(owner[0] == -1 && owner[1] == 0 && owner[2] == -1 && owner[3] == 2);
    const uint64_t h2[3] = {0, 10, 4}, s2[3] = {10, 10, 10};
    msa_head_owners(h2, s2, 3, owner);
    CHECK(owner[0] == -1 && owner[1] == 0 && owner[2] == 0);
    const uint64_t h3[4] = {0, 10, 10, 0};
    msa_head_owners(h3, s1, 4, owner);
    CHECK(owner[0] == -1 && owner[1] == 0 && owner[2] == 0 && owner[3] == -1);
    uint64_t send[3], recv[3];
    msa_tail_plan(0, h2, s2, 3, send, recv);
    CHECK(send[0] == 0 && send[1] == 0 && send[2] == 0 && recv[0] == 0 && recv[1] == 10 && recv[2] == 4);
    msa_tail_plan(1, h2, s2, 3, send, recv);
    CHECK(send[0] == 10 && send[1] == 0 && send[2] == 0 && recv[0] + recv[1] + recv[2] == 0);
    msa_tail_plan(2, h2, s2, 3, send, recv);
    CHECK(send[0] == 4 && send[1] == 0 && send[2] == 0);
    return 0;
}

/* rank r sends (r + 1) * (p + 1) * 1000 + 7 bytes of value (r * 16 + p) to rank p */
static uint64_t blk(int r, int p) { return (uint64_t)(r + 1) * (uint64_t)(p + 1) * 1000u + 7u; }

static int exchange_rank(int rank, int world, msa_shared *sh, void *arg) {
    (void)arg;
    msa_tr *t = msa_tr_shm(sh, rank, world);
    CHECK(t != NULL);
    for (int round = 0; round < 3; ++round) {
        uint64_t mine[2] = {(uint64_t)rank * 3 + round, ~(uint64_t)rank}, all[2 * MSA_MAX_RANKS];
        CHECK(t->allgather(t, mine, sizeof mine, all) == 0);
        for (int r = 0; r < world; ++r) CHECK(all[2 * r] == (uint64_t)r * 3 + round && all[2 * r + 1] == ~(uint64_t)r);
        uint64_t sc[MSA_MAX_RANKS], rc[MSA_MAX_RANKS], ns = 0, nr = 0;
        for (int p = 0; p < world; ++p) {
            sc[p] = blk(rank, p);
            rc[p] = blk(p, rank);
            ns += sc[p];
            nr += rc[p];
        }
        unsigned char *sb = t->alloc(t, ns), *rb = t->alloc(t, nr);
        CHECK(sb && rb);
        uint64_t o = 0;
        for (int p = 0; p < world; ++p) {
            memset(sb + o, rank * 16 + p + round, sc[p]);
            o += sc[p];
        }
        CHECK(t->alltoallv(t, sb, sc, rb, rc) == 0);
        o = 0;
        for (int p = 0; p < world; ++p) {
            for (uint64_t i = 0; i < rc[p]; ++i) CHECK(rb[o + i] == (unsigned char)(p * 16 + rank + round));
            o += rc[p];
        }
        t->release(t, sb);
        t->release(t, rb);
        uint64_t sum = 0;
        CHECK(msa_allreduce_sum_u64(t, (uint64_t)rank + 1, &sum) == 0);
        CHECK(sum == (uint64_t)world * (world + 1) / 2);
        CHECK(msa_barrier(t) == 0);
    }
    t->destroy(t);
    return 0;
}

static int fail_rank(int rank, int world, msa_shared *sh, void *arg) {
    (void)arg;
    msa_tr *t = msa_tr_shm(sh, rank, world);
    if (rank == world - 1) return 3;  /* dies before the collective */
    unsigned char z = 0, all[MSA_MAX_RANKS];
    /* must not block forever: the job is flagged as failed (or the forking
     * launcher ends this rank) */
    if (t->allgather(t, &z, 1, all)) return 4;
    return 0;
}

int main(int argc, char **argv) {
    msa_launch L;
    const int launched = msa_launcher_detect(&L);
    if (argc >= 2 && !strcmp(argv[1], "launched")) {  /* under mpirun (or a launcher's environment) */
        if (launched != 1) { fprintf(stderr, "not started by a launcher (%d)\n", launched); return 1; }
        if (argc >= 3 && !strcmp(argv[2], "fail")) return msa_launcher_run(&L, fail_rank, NULL);
        return msa_launcher_run(&L, exchange_rank, NULL);
    }
    if (argc >= 2 && !strcmp(argv[1], "routing")) return routing();
    if (argc >= 3 && !strcmp(argv[1], "exchange")) return msa_spawn_ranks(atoi(argv[2]), exchange_rank, NULL);
    if (argc >= 3 && !strcmp(argv[1], "fail")) {
        const int rc = msa_spawn_ranks(atoi(argv[2]), fail_rank, NULL);
        return rc == 3 ? 0 : 1;
    }
    fprintf(stderr, "usage: msa_ranks_test routing | exchange N | fail N\n");
    return 2;
}
