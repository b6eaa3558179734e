/*
 * msa_ranks.h -- rank layer of the C host (bin/parallel_spotify --processes N):
 * one process per GPU, the shard routing and the byte exchanges of the
 * multi-GPU pipeline.  Replaces the reference's MPI usage
 * (/root/reference/src/parallel_spotify.c: MPI_Init / rank split 866-916, the
 * hash-table send/receive 397-432 driven at 1011-1025, the timing reductions
 * 1040-1066).
 *
 * Two transports behind one interface:
 *   rccl  one rank per GPU: RCCL (librccl) on device buffers -- all-gather for
 *         the small control data, grouped ncclSend/ncclRecv for the
 *         all-to-all-v of head bytes, table partitions and ranked blocks
 *         (xGMI peer-to-peer on an MI355X node);
 *   shm   host buffers through the node's shared memory: several ranks per
 *         GPU (rehearsal on a one-GPU box) and the CPU tests of this layer.
 * Transport buffers (msa_tr_alloc) are device memory for rccl and host memory
 * for shm; libmsa_hip accepts either wherever this layer hands it one.
 */
#ifndef MSA_RANKS_H
#define MSA_RANKS_H

#include <stddef.h>
#include <stdint.h>

#define MSA_MAX_RANKS 64

/* Shared by the launcher and every rank: created (MAP_SHARED) before fork. */
typedef struct msa_shared msa_shared;
msa_shared *msa_shared_create(int world);
void msa_shared_destroy(msa_shared *s, int world);
/* all ranks of the job (process-shared barrier); 0 on success, -1 once any
 * rank has flagged a failure */
int msa_shared_barrier(msa_shared *s);
/* flag this job as failed: every rank's current and later barriers return -1 */
void msa_shared_fail(msa_shared *s);
/* 128 bytes the ranks share (the rccl transport's ncclUniqueId) */
unsigned char *msa_shared_blob(msa_shared *s);

typedef struct msa_tr msa_tr;
struct msa_tr {
    int rank, world;
    const char *kind; /* "rccl" | "shm" */
    /* host in[bytes] from every rank -> host out[world * bytes] (rank order) */
    int (*allgather)(msa_tr *t, const void *in, size_t bytes, void *out);
    /* send = blocks for ranks 0..world-1 (send_counts bytes each, back to back)
     * -> recv = blocks from ranks 0..world-1 (recv_counts bytes each) */
    int (*alltoallv)(msa_tr *t, const void *send, const uint64_t *send_counts, void *recv,
                     const uint64_t *recv_counts);
    void *(*alloc)(msa_tr *t, size_t bytes);
    void (*release)(msa_tr *t, void *p);
    void (*destroy)(msa_tr *t);
    /* optional (rccl): enqueue the exchanges on this HIP stream -- the rank's
     * libmsa_hip stream (msa_stream), so that exports, exchanges and imports
     * are stream-ordered and released buffers are reused without a wait */
    void (*set_stream)(msa_tr *t, void *stream);
    msa_shared *sh;
    void *impl;
};

msa_tr *msa_tr_shm(msa_shared *sh, int rank, int world);
/* RCCL on `device`; rank 0 publishes the ncclUniqueId through sh.  NULL on
 * failure (message on stderr).  Defined in msa_rccl.c. */
msa_tr *msa_tr_rccl(msa_shared *sh, int rank, int world, int device);

int msa_barrier(msa_tr *t);
/* sum over ranks of one value per rank */
int msa_allreduce_sum_u64(msa_tr *t, uint64_t v, uint64_t *sum);

/* --------------------------------------------------------------- routing
 * A shard's "head" = its leading bytes that belong to a record begun on an
 * earlier shard.  owner[r] = the nearest earlier rank holding a record start
 * (head < size), -1 for rank 0 and for empty heads: rank r's head goes there
 * (mirrors msa/dist.py head_owners / tail_plan). */
void msa_head_owners(const uint64_t *heads, const uint64_t *sizes, int world, int *owner);
void msa_tail_plan(int rank, const uint64_t *heads, const uint64_t *sizes, int world, uint64_t *send,
                   uint64_t *recv);

/* Launcher: fork `world` rank processes (before anything touches the GPU),
 * run fn(rank, world, sh, arg) in each, wait; if a rank fails, the others are
 * terminated (they may be blocked in a collective).  Returns the first
 * failing rank's exit code, else 0. */
int msa_spawn_ranks(int world, int (*fn)(int rank, int world, msa_shared *sh, void *arg), void *arg);

/* External launchers: `mpirun -np N prog ...` (MPICH Hydra: PMI_RANK /
 * PMI_SIZE / PMI_FD; Open MPI: OMPI_COMM_WORLD_RANK / _SIZE) start N unrelated
 * processes that join as the N ranks of this layer (msa_ranks.c). */
typedef struct {
    int rank, world;
    int local_world;   /* ranks on this node as the launcher states it, -1 if it does not */
    const char *kind;  /* "hydra" | "openmpi" */
    int pmi_fd;        /* Hydra's PMI-1 descriptor, -1 without one */
    char key[160];     /* job key: names the shared block */
} msa_launch;
/* 1: started by a launcher (any world size, L filled); 0: not; -1: the
 * launcher's variables are malformed */
int msa_launcher_detect(msa_launch *L);
/* Join the launcher's job (rendezvous in a /dev/shm block keyed by the job;
 * the PMI handshake under Hydra) and run fn(rank, world, sh, arg) as this
 * process's rank; a failing rank flags the job so that the others' barriers
 * return instead of waiting.  Returns fn's exit code (2 if joining failed).
 * Call before anything touches the GPU. */
int msa_launcher_run(msa_launch *L, int (*fn)(int rank, int world, msa_shared *sh, void *arg), void *arg);

#endif
