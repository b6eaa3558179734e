/*
 * msa_rccl.c -- the RCCL transport of the C host's rank layer (msa_ranks.h):
 * one rank per GPU, device buffers, RCCL over xGMI.
 *
 *   all-gather   ncclAllGather of the (small) control data -- shard transfer
 *                functions, piece sizes, heads, partition sizes, timings;
 *   all-to-all-v one ncclGroupStart/End of ncclSend + ncclRecv per peer:
 *                the head bytes of records cut by a shard boundary, the
 *                key-hash partitions of the count tables, the ranked blocks
 *                gathered to rank 0 (replacing send_hash_table /
 *                receive_hash_table, parallel_spotify.c:397-432).
 * The communicator is set up with the ncclUniqueId rank 0 publishes in the
 * launcher's shared block.  Once the rank's libmsa_hip context exists, the
 * collectives are enqueued on the library's own stream (set_stream): the
 * export kernels, the exchange and the import kernels are stream-ordered, so
 * an all-to-all returns without a host wait, and transport buffers come from
 * a pool of device buffers kept for the job (a released buffer is reused by a
 * later exchange on the same stream: no hipMalloc / hipFree per collective).
 * The all-gather of control data ends with a copy to the host and one wait.
 */
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "msa_ranks.h"

#define POOL_N 16
typedef struct {
    void *p;
    size_t cap;
    int used;
} PoolBuf;
typedef struct {
    ncclComm_t comm;
    hipStream_t own;     /* until set_stream */
    hipStream_t stream;  /* where every collective is enqueued */
    void *scratch;
    size_t scratch_bytes;
    PoolBuf pool[POOL_N]; /* every transport buffer of the job, in use or free */
} RcclImpl;

#define NCCL_OK(x, what)                                                                          \
    do {                                                                                          \
        ncclResult_t r_ = (x);                                                                    \
        if (r_ != ncclSuccess) {                                                                  \
            fprintf(stderr, "rank %d: %s: %s\n", t->rank, what, ncclGetErrorString(r_));          \
            return -1;                                                                            \
        }                                                                                         \
    } while (0)
#define HIP_OK(x, what)                                                                           \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "rank %d: %s: %s\n", t->rank, what, hipGetErrorString(e_));           \
            return -1;                                                                            \
        }                                                                                         \
    } while (0)

static int rc_allgather(msa_tr *t, const void *in, size_t bytes, void *out) {
    RcclImpl *im = (RcclImpl *)t->impl;
    const size_t need = bytes * (size_t)t->world;
    if (need > im->scratch_bytes) {
        if (im->scratch) (void)hipFree(im->scratch);
        im->scratch = NULL;
        HIP_OK(hipMalloc(&im->scratch, need), "hipMalloc");
        im->scratch_bytes = need;
    }
    char *sc = (char *)im->scratch;
    HIP_OK(hipMemcpyAsync(sc + bytes * (size_t)t->rank, in, bytes, hipMemcpyHostToDevice, im->stream), "copy in");
    NCCL_OK(ncclAllGather(sc + bytes * (size_t)t->rank, sc, bytes, ncclUint8, im->comm, im->stream), "ncclAllGather");
    HIP_OK(hipMemcpyAsync(out, sc, need, hipMemcpyDeviceToHost, im->stream), "copy out");
    HIP_OK(hipStreamSynchronize(im->stream), "sync");
    return 0;
}

/* A rank's block for itself is a device copy on the exchange stream, not an
 * RCCL message to itself (a world of one sent a 1.8 GB self-message through
 * ncclSend / ncclRecv and received corrupt bytes: the configs[4] merge failed);
 * messages to other ranks go in pieces of at most RC_PIECE bytes, the sender
 * and the receiver cutting the same byte count the same way. */
#define RC_PIECE ((uint64_t)256 << 20)
static int rc_alltoallv(msa_tr *t, const void *send, const uint64_t *sc, void *recv, const uint64_t *rc) {
    RcclImpl *im = (RcclImpl *)t->impl;
    uint64_t so = 0, ro = 0, sself = 0, rself = 0;
    for (int p = 0; p < t->rank; ++p) {
        sself += sc[p];
        rself += rc[p];
    }
    if (sc[t->rank] != rc[t->rank]) {
        fprintf(stderr, "rank %d: all-to-all: %llu bytes sent to itself, %llu expected\n", t->rank,
                (unsigned long long)sc[t->rank], (unsigned long long)rc[t->rank]);
        return -1;
    }
    if (sc[t->rank])
        HIP_OK(hipMemcpyAsync((char *)recv + rself, (const char *)send + sself, sc[t->rank], hipMemcpyDeviceToDevice,
                              im->stream), "self copy");
    NCCL_OK(ncclGroupStart(), "ncclGroupStart");
    for (int p = 0; p < t->world; ++p) {
        if (p != t->rank) {
            for (uint64_t k = 0; k < sc[p]; k += RC_PIECE) {
                const uint64_t n = sc[p] - k < RC_PIECE ? sc[p] - k : RC_PIECE;
                NCCL_OK(ncclSend((const char *)send + so + k, n, ncclUint8, p, im->comm, im->stream), "ncclSend");
            }
            for (uint64_t k = 0; k < rc[p]; k += RC_PIECE) {
                const uint64_t n = rc[p] - k < RC_PIECE ? rc[p] - k : RC_PIECE;
                NCCL_OK(ncclRecv((char *)recv + ro + k, n, ncclUint8, p, im->comm, im->stream), "ncclRecv");
            }
        }
        so += sc[p];
        ro += rc[p];
    }
    NCCL_OK(ncclGroupEnd(), "ncclGroupEnd");
    /* on the library's stream the consumers are ordered after the exchange */
    if (im->stream == im->own) HIP_OK(hipStreamSynchronize(im->stream), "sync");
    return 0;
}

/* Transport buffers: every device buffer the job allocated stays in the pool
 * (in use or free); an exchange takes the smallest free one that fits, else
 * a new one rounded up to 2 MiB so that growing exchanges reuse it.  A free
 * buffer's last readers were enqueued on the same stream as its next writer. */
static void *rc_alloc(msa_tr *t, size_t n) {
    RcclImpl *im = (RcclImpl *)t->impl;
    int best = -1, empty = -1, spare = -1;
    for (int i = 0; i < POOL_N; ++i) {
        PoolBuf *b = &im->pool[i];
        if (!b->p) { if (empty < 0) empty = i; continue; }
        if (b->used) continue;
        if (b->cap >= n && (best < 0 || b->cap < im->pool[best].cap)) best = i;
        if (spare < 0 || b->cap < im->pool[spare].cap) spare = i;
    }
    if (best >= 0) {
        im->pool[best].used = 1;
        return im->pool[best].p;
    }
    if (empty < 0) {  /* pool full: the smallest free buffer makes room */
        if (spare < 0) {
            fprintf(stderr, "rank %d: more than %d transport buffers in use\n", t->rank, POOL_N);
            return NULL;
        }
        (void)hipStreamSynchronize(im->stream);
        (void)hipFree(im->pool[spare].p);
        im->pool[spare].p = NULL;
        empty = spare;
    }
    const size_t cap = ((n ? n : 1) + ((size_t)2 << 20) - 1) & ~(((size_t)2 << 20) - 1);
    void *p = NULL;
    if (hipMalloc(&p, cap) != hipSuccess) {
        fprintf(stderr, "rank %d: hipMalloc(%zu) failed\n", t->rank, cap);
        return NULL;
    }
    im->pool[empty].p = p;
    im->pool[empty].cap = cap;
    im->pool[empty].used = 1;
    return p;
}
static void rc_release(msa_tr *t, void *p) {
    RcclImpl *im = (RcclImpl *)t->impl;
    for (int i = 0; p && i < POOL_N; ++i)
        if (im->pool[i].p == p) im->pool[i].used = 0;
}
static void rc_set_stream(msa_tr *t, void *stream) {
    RcclImpl *im = (RcclImpl *)t->impl;
    (void)hipStreamSynchronize(im->stream);
    im->stream = stream ? (hipStream_t)stream : im->own;
}
static void rc_destroy(msa_tr *t) {
    RcclImpl *im = (RcclImpl *)t->impl;
    if (im) {
        if (im->stream) (void)hipStreamSynchronize(im->stream);
        if (im->comm) ncclCommDestroy(im->comm);
        if (im->scratch) (void)hipFree(im->scratch);
        for (int i = 0; i < POOL_N; ++i)
            if (im->pool[i].p) (void)hipFree(im->pool[i].p);
        if (im->own) (void)hipStreamDestroy(im->own);
        free(im);
    }
    free(t);
}

/* RCCL prints its version banner on stdout at initialisation; the CLI's
 * stdout is the reference's summary, byte for byte, so the banner goes to
 * stderr instead. */
static int stdout_to_stderr(void) {
    fflush(stdout);
    const int saved = dup(1);
    if (saved >= 0) dup2(2, 1);
    return saved;
}
static void stdout_restore(int saved) {
    fflush(stdout);
    if (saved >= 0) {
        dup2(saved, 1);
        close(saved);
    }
}

msa_tr *msa_tr_rccl(msa_shared *sh, int rank, int world, int device) {
    msa_tr *t = calloc(1, sizeof *t);
    RcclImpl *im = calloc(1, sizeof *im);
    if (!t || !im) { free(t); free(im); return NULL; }
    t->rank = rank;
    t->world = world;
    t->kind = "rccl";
    t->allgather = rc_allgather;
    t->alltoallv = rc_alltoallv;
    t->alloc = rc_alloc;
    t->release = rc_release;
    t->destroy = rc_destroy;
    t->set_stream = rc_set_stream;
    t->sh = sh;
    t->impl = im;
    ncclUniqueId id;
    _Static_assert(sizeof(ncclUniqueId) <= 128, "ncclUniqueId fits the shared blob");
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&im->own, hipStreamNonBlocking) != hipSuccess) {
        fprintf(stderr, "rank %d: cannot use GPU %d\n", rank, device);
        rc_destroy(t);
        return NULL;
    }
    im->stream = im->own;
    const int saved = stdout_to_stderr();
    msa_tr *res = t;
    if (rank == 0) {
        if (ncclGetUniqueId(&id) != ncclSuccess) {
            fprintf(stderr, "rank 0: ncclGetUniqueId failed\n");
            rc_destroy(t);
            stdout_restore(saved);
            return NULL;
        }
        memcpy(msa_shared_blob(sh), &id, sizeof id);
    }
    if (msa_shared_barrier(sh)) {  /* the id is published */
        rc_destroy(t);
        stdout_restore(saved);
        return NULL;
    }
    memcpy(&id, msa_shared_blob(sh), sizeof id);
    const ncclResult_t r = ncclCommInitRank(&im->comm, world, id, rank);
    if (r != ncclSuccess) {
        fprintf(stderr, "rank %d: ncclCommInitRank: %s\n", rank, ncclGetErrorString(r));
        im->comm = NULL;
        rc_destroy(t);
        res = NULL;
    }
    stdout_restore(saved);
    return res;
}
