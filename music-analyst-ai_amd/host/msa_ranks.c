/*
 * msa_ranks.c -- launcher, routing and the shared-memory transport of the C
 * host's rank layer (msa_ranks.h).  Host C only: no HIP here (the RCCL
 * transport lives in msa_rccl.c), so this part is tested on the CPU.
 */
#define _GNU_SOURCE
#include "msa_ranks.h"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#define SH_SLOT 65536 /* bytes per rank of one small all-gather */

struct msa_shared {
    pthread_barrier_t bar;
    long tag;                  /* launcher pid: names this job's /dev/shm files */
    unsigned char nccl_id[128]; /* ncclUniqueId of the rccl transport          */
    unsigned char slots[];     /* world * SH_SLOT                              */
};

static size_t shared_bytes(int world) { return sizeof(msa_shared) + (size_t)world * SH_SLOT; }

msa_shared *msa_shared_create(int world) {
    if (world < 1 || world > MSA_MAX_RANKS) return NULL;
    msa_shared *s = mmap(NULL, shared_bytes(world), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (s == MAP_FAILED) return NULL;
    pthread_barrierattr_t a;
    pthread_barrierattr_init(&a);
    pthread_barrierattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
    if (pthread_barrier_init(&s->bar, &a, (unsigned)world) != 0) {
        munmap(s, shared_bytes(world));
        return NULL;
    }
    pthread_barrierattr_destroy(&a);
    s->tag = (long)getpid();
    return s;
}

void msa_shared_destroy(msa_shared *s, int world) {
    if (!s) return;
    /* files of this job a failed rank may have left behind */
    char pre[64];
    int pl = snprintf(pre, sizeof pre, "msa_%ld_", s->tag);
    DIR *d = opendir("/dev/shm");
    if (d) {
        struct dirent *e;
        char path[512];
        while ((e = readdir(d)))
            if (!strncmp(e->d_name, pre, (size_t)pl)) {
                snprintf(path, sizeof path, "/dev/shm/%s", e->d_name);
                unlink(path);
            }
        closedir(d);
    }
    /* no pthread_barrier_destroy: after a failed rank the barrier may still
     * count killed waiters, and glibc's destroy waits for them forever */
    munmap(s, shared_bytes(world));
}

static int sh_barrier(msa_shared *s) {
    const int rc = pthread_barrier_wait(&s->bar);
    return (rc == 0 || rc == PTHREAD_BARRIER_SERIAL_THREAD) ? 0 : -1;
}
int msa_shared_barrier(msa_shared *s) { return sh_barrier(s); }
unsigned char *msa_shared_blob(msa_shared *s) { return s->nccl_id; }

int msa_barrier(msa_tr *t) {
    unsigned char z = 0, all[MSA_MAX_RANKS];
    return t->allgather(t, &z, 1, all);
}

int msa_allreduce_sum_u64(msa_tr *t, uint64_t v, uint64_t *sum) {
    uint64_t all[MSA_MAX_RANKS];
    if (t->allgather(t, &v, sizeof v, all)) return -1;
    uint64_t s = 0;
    for (int r = 0; r < t->world; ++r) s += all[r];
    *sum = s;
    return 0;
}

/* ------------------------------------------------------------ shm transport */
typedef struct {
    uint64_t seq;
} ShmImpl;

static int shm_allgather(msa_tr *t, const void *in, size_t bytes, void *out) {
    if (bytes > SH_SLOT) {
        fprintf(stderr, "rank %d: shm all-gather of %zu bytes exceeds its %d-byte slot\n", t->rank, bytes, SH_SLOT);
        return -1;
    }
    memcpy(t->sh->slots + (size_t)t->rank * SH_SLOT, in, bytes);
    if (sh_barrier(t->sh)) return -1;
    for (int r = 0; r < t->world; ++r) memcpy((char *)out + (size_t)r * bytes, t->sh->slots + (size_t)r * SH_SLOT, bytes);
    return sh_barrier(t->sh);
}

static void shm_name(char *b, size_t n, long tag, uint64_t seq, int src, int dst) {
    snprintf(b, n, "/dev/shm/msa_%ld_%llu_%d_%d", tag, (unsigned long long)seq, src, dst);
}

static int write_file(const char *path, const char *p, uint64_t n) {
    int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0600);
    if (fd < 0) return -1;
    while (n) {
        ssize_t w = write(fd, p, n > (1u << 30) ? (1u << 30) : n);
        if (w <= 0) { close(fd); return -1; }
        p += w;
        n -= (uint64_t)w;
    }
    return close(fd);
}

static int read_file(const char *path, char *p, uint64_t n) {
    int fd = open(path, O_RDONLY);
    if (fd < 0) return -1;
    while (n) {
        ssize_t r = read(fd, p, n > (1u << 30) ? (1u << 30) : n);
        if (r <= 0) { close(fd); return -1; }
        p += r;
        n -= (uint64_t)r;
    }
    return close(fd);
}

static int shm_alltoallv(msa_tr *t, const void *send, const uint64_t *sc, void *recv, const uint64_t *rc) {
    ShmImpl *im = (ShmImpl *)t->impl;
    const uint64_t seq = im->seq++;
    char path[256];
    uint64_t so = 0, ro = 0;
    int err = 0;
    for (int p = 0; p < t->world; ++p) {
        if (sc[p] && p != t->rank) {
            shm_name(path, sizeof path, t->sh->tag, seq, t->rank, p);
            if (write_file(path, (const char *)send + so, sc[p])) err = 1;
        }
        so += sc[p];
    }
    if (sh_barrier(t->sh)) return -1;
    so = 0;
    for (int p = 0; p < t->rank; ++p) so += sc[p];
    for (int p = 0; p < t->world; ++p) {
        if (rc[p]) {
            if (p == t->rank) {
                if (rc[p] != sc[p]) err = 1;
                else memcpy((char *)recv + ro, (const char *)send + so, rc[p]);
            } else {
                shm_name(path, sizeof path, t->sh->tag, seq, p, t->rank);
                if (read_file(path, (char *)recv + ro, rc[p])) err = 1;
                unlink(path);
            }
        }
        ro += rc[p];
    }
    if (sh_barrier(t->sh)) return -1;
    if (err) fprintf(stderr, "rank %d: shm all-to-all failed\n", t->rank);
    return err ? -1 : 0;
}

static void *shm_alloc(msa_tr *t, size_t n) {
    (void)t;
    return malloc(n ? n : 1);
}
static void shm_release(msa_tr *t, void *p) {
    (void)t;
    free(p);
}
static void shm_destroy(msa_tr *t) {
    free(t->impl);
    free(t);
}

msa_tr *msa_tr_shm(msa_shared *sh, int rank, int world) {
    msa_tr *t = calloc(1, sizeof *t);
    ShmImpl *im = calloc(1, sizeof *im);
    if (!t || !im) { free(t); free(im); return NULL; }
    t->rank = rank;
    t->world = world;
    t->kind = "shm";
    t->allgather = shm_allgather;
    t->alltoallv = shm_alltoallv;
    t->alloc = shm_alloc;
    t->release = shm_release;
    t->destroy = shm_destroy;
    t->sh = sh;
    t->impl = im;
    return t;
}

/* ------------------------------------------------------------------ routing */
void msa_head_owners(const uint64_t *heads, const uint64_t *sizes, int world, int *owner) {
    int last_start = -1;
    for (int r = 0; r < world; ++r) {
        owner[r] = (r > 0 && heads[r] > 0) ? last_start : -1;
        if (r == 0 || heads[r] < sizes[r]) last_start = r;
    }
}

void msa_tail_plan(int rank, const uint64_t *heads, const uint64_t *sizes, int world, uint64_t *send, uint64_t *recv) {
    int owner[MSA_MAX_RANKS];
    msa_head_owners(heads, sizes, world, owner);
    for (int r = 0; r < world; ++r) send[r] = recv[r] = 0;
    if (owner[rank] >= 0) send[owner[rank]] = heads[rank];
    for (int r = 0; r < world; ++r)
        if (owner[r] == rank) recv[r] = heads[r];
}

/* ----------------------------------------------------------------- launcher */
int msa_spawn_ranks(int world, int (*fn)(int, int, msa_shared *, void *), void *arg) {
    msa_shared *sh = msa_shared_create(world);
    if (!sh) {
        fprintf(stderr, "cannot create the shared rank block for %d ranks\n", world);
        return 2;
    }
    pid_t pid[MSA_MAX_RANKS];
    int alive[MSA_MAX_RANKS];
    fflush(stdout);
    fflush(stderr);
    int started = 0, first_fail = 0;
    for (int r = 0; r < world; ++r) {
        pid_t p = fork();
        if (p == 0) {
            const int rc = fn(r, world, sh, arg);
            fflush(stdout);
            fflush(stderr);
            _exit(rc & 0xFF);
        }
        if (p < 0) {
            fprintf(stderr, "fork failed: %s\n", strerror(errno));
            first_fail = 2;
            break;
        }
        pid[r] = p;
        alive[r] = 1;
        ++started;
    }
    int left = started;
    if (first_fail)
        for (int r = 0; r < started; ++r) kill(pid[r], SIGTERM);
    while (left > 0) {
        int st = 0;
        pid_t p = waitpid(-1, &st, 0);
        if (p < 0) {
            if (errno == EINTR) continue;
            break;
        }
        int r = -1;
        for (int i = 0; i < started; ++i)
            if (alive[i] && pid[i] == p) r = i;
        if (r < 0) continue;
        alive[r] = 0;
        --left;
        const int code = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
        if (code && !first_fail) {
            first_fail = code;
            /* the other ranks may wait in a collective for this one forever */
            for (int i = 0; i < started; ++i)
                if (alive[i]) kill(pid[i], SIGTERM);
        }
    }
    msa_shared_destroy(sh, world);
    return first_fail;
}
