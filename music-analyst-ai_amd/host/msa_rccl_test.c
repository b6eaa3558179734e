/*
 * msa_rccl_test -- CPU test of the RCCL transport (host/msa_rccl.c) against
 * the in-process HIP / RCCL stand-ins of host/test_stub (host memory, a
 * thread per rank, RCCL's send/recv matching): the transport's own logic --
 * all-gather staging, all-to-all-v offsets with zero-size peers (no empty
 * operation may be posted), the device buffer pool (reuse, the POOL_N limit,
 * eviction), set_stream (no host wait once on the library's stream), and the
 * clean failure of msa_tr_rccl.  RCCL itself runs on the GPU tests.
 *
 *   msa_rccl_test exchange N | pool | initfail | mallocfail
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "msa_ranks.h"
#include "test_stub/stub_rt.h"

#define CHECK(c)                                                                   \
    do {                                                                           \
        if (!(c)) {                                                                \
            fprintf(stderr, "check failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

/* rank r sends blk(r, p) bytes to rank p; some pairs exchange nothing */
static uint64_t blk(int r, int p, int round) {
    if ((r + 2 * p + round) % 3 == 0) return 0;
    return (uint64_t)(r + 1) * (uint64_t)(p + 1) * 1000u + 7u;
}

typedef struct {
    int rank, world, rc;
    msa_shared *sh;
} Arg;

static int exchange_body(int rank, int world, msa_shared *sh) {
    msa_tr *t = msa_tr_rccl(sh, rank, world, rank);
    CHECK(t != NULL);
    CHECK(!strcmp(t->kind, "rccl"));
    for (int round = 0; round < 4; ++round) {
        uint64_t mine[2] = {(uint64_t)rank * 3 + round, ~(uint64_t)rank}, all[2 * MSA_MAX_RANKS];
        CHECK(t->allgather(t, mine, sizeof mine, all) == 0);
        for (int r = 0; r < world; ++r) CHECK(all[2 * r] == (uint64_t)r * 3 + round && all[2 * r + 1] == ~(uint64_t)r);
        uint64_t sc[MSA_MAX_RANKS], rc[MSA_MAX_RANKS], ns = 0, nr = 0;
        for (int p = 0; p < world; ++p) {
            sc[p] = blk(rank, p, round);
            rc[p] = blk(p, rank, round);
            ns += sc[p];
            nr += rc[p];
        }
        unsigned char *sb = t->alloc(t, ns), *rb = t->alloc(t, nr);  /* "device" buffers of the pool */
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
    }
    /* on an external stream (the library's): exchanges return without a host wait */
    hipStream_t ext;
    CHECK(hipStreamCreateWithFlags(&ext, hipStreamNonBlocking) == hipSuccess);
    t->set_stream(t, ext);
    stub_stats a, b;
    uint64_t sc[MSA_MAX_RANKS], rc[MSA_MAX_RANKS];
    for (int p = 0; p < world; ++p) sc[p] = rc[p] = 64;
    unsigned char *sb = t->alloc(t, 64 * (size_t)world), *rb = t->alloc(t, 64 * (size_t)world);
    CHECK(sb && rb);
    memset(sb, rank, 64 * (size_t)world);
    stub_get_stats(&a);
    CHECK(t->alltoallv(t, sb, sc, rb, rc) == 0);
    stub_get_stats(&b);
    if (world == 1) CHECK(b.syncs == a.syncs);  /* no stream sync inside the exchange */
    for (int p = 0; p < world; ++p) CHECK(rb[64 * p] == (unsigned char)p);
    t->release(t, sb);
    t->release(t, rb);
    t->set_stream(t, NULL);
    t->destroy(t);
    (void)hipStreamDestroy(ext);
    return 0;
}
static void *exchange_thread(void *p) {
    Arg *a = (Arg *)p;
    a->rc = exchange_body(a->rank, a->world, a->sh);
    if (a->rc) msa_shared_fail(a->sh);
    return NULL;
}
static int exchange(int world) {
    msa_shared *sh = msa_shared_create(world);
    CHECK(sh != NULL);
    pthread_t th[MSA_MAX_RANKS];
    Arg args[MSA_MAX_RANKS];
    for (int r = 0; r < world; ++r) {
        args[r] = (Arg){r, world, 0, sh};
        CHECK(pthread_create(&th[r], NULL, exchange_thread, &args[r]) == 0);
    }
    int bad = 0;
    for (int r = 0; r < world; ++r) {
        pthread_join(th[r], NULL);
        bad |= args[r].rc;
    }
    msa_shared_destroy(sh, world);
    stub_stats s;
    stub_get_stats(&s);
    CHECK(!bad);
    CHECK(s.live_allocs == 0 && s.streams_live == 0);  /* every pool buffer and stream released */
    return 0;
}

/* the pool: reuse of a free buffer that fits, POOL_N (16) buffers at most in
 * use, eviction of the smallest free buffer when all slots hold buffers */
static int pool(void) {
    msa_shared *sh = msa_shared_create(1);
    msa_tr *t = msa_tr_rccl(sh, 0, 1, 0);
    CHECK(t != NULL);
    stub_stats a, b;
    void *p[17];
    for (int i = 0; i < 16; ++i) CHECK((p[i] = t->alloc(t, 1000)) != NULL);
    stub_get_stats(&a);
    CHECK(t->alloc(t, 1000) == NULL);  /* a 17th buffer in use: refused */
    t->release(t, p[3]);
    CHECK(t->alloc(t, 500) == p[3]);   /* a free buffer that fits is reused */
    stub_get_stats(&b);
    CHECK(b.mallocs == a.mallocs);
    for (int i = 0; i < 16; ++i) t->release(t, p[i]);
    stub_get_stats(&a);
    void *big = t->alloc(t, (size_t)8 << 20);  /* fits none: the smallest free buffer makes room */
    CHECK(big != NULL);
    stub_get_stats(&b);
    CHECK(b.frees == a.frees + 1 && b.mallocs == a.mallocs + 1);
    t->release(t, big);
    CHECK(t->alloc(t, (size_t)4 << 20) == big);  /* rounded capacities: the big one serves smaller requests */
    t->destroy(t);
    msa_shared_destroy(sh, 1);
    stub_get_stats(&b);
    CHECK(b.live_allocs == 0 && b.streams_live == 0);
    return 0;
}

/* the communicator cannot be set up: NULL, nothing left allocated */
static int initfail(void) {
    stub_fail_init(1);
    msa_shared *sh = msa_shared_create(1);
    msa_tr *t = msa_tr_rccl(sh, 0, 1, 0);
    CHECK(t == NULL);
    msa_shared_destroy(sh, 1);
    stub_stats s;
    stub_get_stats(&s);
    CHECK(s.live_allocs == 0 && s.streams_live == 0);
    stub_fail_init(0);
    return 0;
}

/* device memory runs out: the exchange buffer request fails cleanly */
static int mallocfail(void) {
    msa_shared *sh = msa_shared_create(1);
    msa_tr *t = msa_tr_rccl(sh, 0, 1, 0);
    CHECK(t != NULL);
    stub_fail_malloc_at(1);
    CHECK(t->alloc(t, 100) == NULL);
    stub_fail_malloc_at(0);
    void *p = t->alloc(t, 100);
    CHECK(p != NULL);
    t->release(t, p);
    t->destroy(t);
    msa_shared_destroy(sh, 1);
    stub_stats s;
    stub_get_stats(&s);
    CHECK(s.live_allocs == 0 && s.streams_live == 0);
    return 0;
}

int main(int argc, char **argv) {
    stub_reset();
    if (argc >= 3 && !strcmp(argv[1], "exchange")) return exchange(atoi(argv[2]));
    if (argc >= 2 && !strcmp(argv[1], "pool")) return pool();
    if (argc >= 2 && !strcmp(argv[1], "initfail")) return initfail();
    if (argc >= 2 && !strcmp(argv[1], "mallocfail")) return mallocfail();
    fprintf(stderr, "usage: msa_rccl_test exchange N | pool | initfail | mallocfail\n");
    return 2;
}
