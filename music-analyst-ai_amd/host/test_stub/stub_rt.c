/* HIP / RCCL test stand-ins over host memory (see test_stub/hip, test_stub/rccl). */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "stub_rt.h"

static _Atomic long g_mallocs, g_frees, g_streams, g_syncs, g_sends, g_recvs, g_malloc_calls;
static _Atomic int g_fail_init;
static _Atomic long g_fail_malloc_at;

void stub_get_stats(stub_stats *s) {
    s->mallocs = g_mallocs;
    s->frees = g_frees;
    s->live_allocs = g_mallocs - g_frees;
    s->streams_live = g_streams;
    s->syncs = g_syncs;
    s->sends = g_sends;
    s->recvs = g_recvs;
}
void stub_reset(void) {
    g_mallocs = g_frees = g_streams = g_syncs = g_sends = g_recvs = g_malloc_calls = 0;
    g_fail_init = 0;
    g_fail_malloc_at = 0;
}
void stub_fail_init(int on) { g_fail_init = on; }
void stub_fail_malloc_at(long k) { g_fail_malloc_at = k; g_malloc_calls = 0; }

struct stub_stream { int dummy; };
hipError_t hipSetDevice(int device) { return device >= 0 ? hipSuccess : hipErrorInvalidDevice; }
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned flags) {
    (void)flags;
    *s = calloc(1, sizeof(struct stub_stream));
    ++g_streams;
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
    free(s);
    --g_streams;
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t s) {
    (void)s;
    ++g_syncs;
    return hipSuccess;
}
hipError_t hipMalloc(void **p, size_t n) {
    const long k = ++g_malloc_calls;
    if (g_fail_malloc_at && k == g_fail_malloc_at) return hipErrorOutOfMemory;
    *p = malloc(n ? n : 1);
    if (!*p) return hipErrorOutOfMemory;
    ++g_mallocs;
    return hipSuccess;
}
hipError_t hipFree(void *p) {
    if (p) {
        free(p);
        ++g_frees;
    }
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void *dst, const void *src, size_t n, hipMemcpyKind k, hipStream_t s) {
    (void)k;
    (void)s;
    memmove(dst, src, n);
    return hipSuccess;
}
const char *hipGetErrorString(hipError_t e) { return e == hipSuccess ? "hipSuccess" : "stub HIP error"; }

/* ---------------------------------------------------------------- fabric */
#define MAXR 64
typedef struct Msg {
    struct Msg *next;
    size_t n;
    unsigned char data[];
} Msg;
typedef struct {
    char key[128];
    int world, joined;
    pthread_barrier_t bar;
    const void *ag_src[MAXR];  /* all-gather: each rank's contribution */
    pthread_mutex_t mu;        /* point-to-point: FIFO mailboxes src -> dst */
    pthread_cond_t cv;
    Msg *head[MAXR][MAXR], *tail[MAXR][MAXR];
} Fabric;
struct stub_comm {
    Fabric *f;
    int rank;
};
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static Fabric *g_fab[16];
static _Atomic long g_idc;

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    memset(id, 0, sizeof *id);
    snprintf(id->internal, sizeof id->internal, "stub-%ld-%ld", (long)getpid(), (long)++g_idc);
    return ncclSuccess;
}
ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank) {
    *comm = NULL;
    if (g_fail_init) return ncclSystemError;
    if (nranks < 1 || nranks > MAXR || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    pthread_mutex_lock(&g_mu);
    Fabric *f = NULL;
    int free_slot = -1;
    for (int i = 0; i < 16; ++i) {
        if (g_fab[i] && !strcmp(g_fab[i]->key, id.internal)) f = g_fab[i];
        if (!g_fab[i] && free_slot < 0) free_slot = i;
    }
    if (!f) {
        if (free_slot < 0) { pthread_mutex_unlock(&g_mu); return ncclSystemError; }
        f = calloc(1, sizeof *f);
        memcpy(f->key, id.internal, sizeof f->key);
        f->world = nranks;
        pthread_barrier_init(&f->bar, NULL, (unsigned)nranks);
        pthread_mutex_init(&f->mu, NULL);
        pthread_cond_init(&f->cv, NULL);
        g_fab[free_slot] = f;
    }
    ++f->joined;
    pthread_mutex_unlock(&g_mu);
    struct stub_comm *c = calloc(1, sizeof *c);
    c->f = f;
    c->rank = rank;
    pthread_barrier_wait(&f->bar);
    *comm = c;
    return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return ncclInvalidArgument;
    pthread_mutex_lock(&g_mu);
    Fabric *f = comm->f;
    if (--f->joined == 0) {
        for (int i = 0; i < 16; ++i)
            if (g_fab[i] == f) g_fab[i] = NULL;
        pthread_barrier_destroy(&f->bar);
        pthread_mutex_destroy(&f->mu);
        pthread_cond_destroy(&f->cv);
        for (int a = 0; a < MAXR; ++a)
            for (int b = 0; b < MAXR; ++b)
                for (Msg *m = f->head[a][b]; m;) {
                    Msg *nx = m->next;
                    free(m);
                    m = nx;
                }
        free(f);
    }
    pthread_mutex_unlock(&g_mu);
    free(comm);
    return ncclSuccess;
}
ncclResult_t ncclAllGather(const void *send, void *recv, size_t count, ncclDataType_t t, ncclComm_t c, hipStream_t s) {
    (void)t;
    (void)s;
    Fabric *f = c->f;
    /* a private copy first: in place, recv + rank * count is the send buffer */
    void *mine = malloc(count ? count : 1);
    memcpy(mine, send, count);
    f->ag_src[c->rank] = mine;
    pthread_barrier_wait(&f->bar);
    for (int r = 0; r < f->world; ++r) memcpy((char *)recv + (size_t)r * count, f->ag_src[r], count);
    pthread_barrier_wait(&f->bar);
    free(mine);
    return ncclSuccess;
}

/* grouped point-to-point: recorded per thread, executed at ncclGroupEnd */
typedef struct {
    int send;  /* 1 send, 0 recv */
    void *buf;
    size_t n;
    int peer;
    ncclComm_t comm;
} Op;
static __thread Op t_ops[4 * MAXR];
static __thread int t_nops, t_depth;

ncclResult_t ncclGroupStart(void) {
    if (t_depth++ == 0) t_nops = 0;
    return ncclSuccess;
}
static ncclResult_t record(int send, void *buf, size_t n, int peer, ncclComm_t c) {
    if (!c || peer < 0 || peer >= c->f->world || t_nops >= 4 * MAXR) return ncclInvalidArgument;
    if (n == 0) return ncclInvalidUsage;  /* the transport must not post empty operations */
    t_ops[t_nops++] = (Op){send, buf, n, peer, c};
    if (send) ++g_sends;
    else ++g_recvs;
    return ncclSuccess;
}
ncclResult_t ncclSend(const void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
    (void)t;
    (void)s;
    return record(1, (void *)buf, count, peer, c);
}
ncclResult_t ncclRecv(void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
    (void)t;
    (void)s;
    return record(0, buf, count, peer, c);
}
/* sends are buffered (copied into the peer's mailbox), receives wait for
 * the matching send: no synchronisation between ranks that exchange nothing */
ncclResult_t ncclGroupEnd(void) {
    if (--t_depth > 0) return ncclSuccess;
    ncclResult_t rc = ncclSuccess;
    for (int i = 0; i < t_nops; ++i) {
        if (!t_ops[i].send) continue;
        Fabric *f = t_ops[i].comm->f;
        const int me = t_ops[i].comm->rank, p = t_ops[i].peer;
        Msg *m = malloc(sizeof(Msg) + t_ops[i].n);
        m->next = NULL;
        m->n = t_ops[i].n;
        memcpy(m->data, t_ops[i].buf, t_ops[i].n);
        pthread_mutex_lock(&f->mu);
        if (f->tail[me][p]) f->tail[me][p]->next = m;
        else f->head[me][p] = m;
        f->tail[me][p] = m;
        pthread_cond_broadcast(&f->cv);
        pthread_mutex_unlock(&f->mu);
    }
    for (int i = 0; i < t_nops; ++i) {
        if (t_ops[i].send) continue;
        Fabric *f = t_ops[i].comm->f;
        const int me = t_ops[i].comm->rank, p = t_ops[i].peer;
        pthread_mutex_lock(&f->mu);
        while (!f->head[p][me]) pthread_cond_wait(&f->cv, &f->mu);
        Msg *m = f->head[p][me];
        f->head[p][me] = m->next;
        if (!m->next) f->tail[p][me] = NULL;
        pthread_mutex_unlock(&f->mu);
        if (m->n != t_ops[i].n) rc = ncclInvalidUsage;  /* RCCL requires matching sizes */
        else memcpy(t_ops[i].buf, m->data, m->n);
        free(m);
    }
    t_nops = 0;
    return rc;
}
const char *ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "no error" : "stub RCCL error"; }
