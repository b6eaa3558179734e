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
#include <sched.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#define SH_SLOT 65536 /* bytes per rank of one small all-gather */
#define SH_READY 0x6d73615f6a6f6221ull /* "msa_job!": a launcher rank's block is initialised */

struct msa_shared {
    _Atomic unsigned count;    /* ranks arrived at the current barrier          */
    _Atomic unsigned gen;      /* barrier generation                            */
    _Atomic int failed;        /* a rank failed: every barrier returns -1       */
    _Atomic unsigned joined;   /* launcher mode: ranks that mapped the block    */
    _Atomic unsigned long long ready; /* launcher mode: SH_READY once initialised */
    int world;
    long tag;                  /* creator's pid: names this job's /dev/shm files */
    unsigned char nccl_id[128]; /* ncclUniqueId of the rccl transport          */
    unsigned char slots[];     /* world * SH_SLOT                              */
};

static size_t shared_bytes(int world) { return sizeof(msa_shared) + (size_t)world * SH_SLOT; }

static void shared_init(msa_shared *s, int world) {
    atomic_store(&s->count, 0);
    atomic_store(&s->gen, 0);
    atomic_store(&s->failed, 0);
    atomic_store(&s->joined, 0);
    s->world = world;
    s->tag = (long)getpid();
}

msa_shared *msa_shared_create(int world) {
    if (world < 1 || world > MSA_MAX_RANKS) return NULL;
    msa_shared *s = mmap(NULL, shared_bytes(world), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (s == MAP_FAILED) return NULL;
    shared_init(s, world);
    return s;
}

/* the /dev/shm files of this job's shm exchanges (a failed rank may have left
 * some behind) */
static void shared_unlink_files(const msa_shared *s) {
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
}

void msa_shared_destroy(msa_shared *s, int world) {
    if (!s) return;
    shared_unlink_files(s);
    munmap(s, shared_bytes(world));
}

void msa_shared_fail(msa_shared *s) {
    if (s) atomic_store(&s->failed, 1);
}

/* Generation barrier on the shared block.  A waiter spins briefly, then
 * yields, then sleeps in 20 us steps; it gives up when any rank has flagged a
 * failure (msa_shared_fail), so that a rank dying outside a forking launcher
 * (mpirun does not end the job's other processes) cannot leave the others
 * waiting forever. */
static int sh_barrier(msa_shared *s) {
    const unsigned g = atomic_load(&s->gen);
    if (atomic_fetch_add(&s->count, 1) == (unsigned)s->world - 1) {
        atomic_store(&s->count, 0);
        atomic_fetch_add(&s->gen, 1);
        return 0;
    }
    /* a completed barrier returns 0 even if a rank failed right after it (its
     * failure shows at the next barrier) */
    for (unsigned spin = 0; atomic_load(&s->gen) == g; ++spin) {
        if (atomic_load(&s->failed)) return atomic_load(&s->gen) == g ? -1 : 0;
        if (spin < 256) continue;
        if (spin < 4096) sched_yield();
        else {
            const struct timespec ts = {0, 20000};
            nanosleep(&ts, NULL);
        }
    }
    return 0;
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
            msa_shared_fail(sh);
            /* the other ranks may wait in a collective for this one forever */
            for (int i = 0; i < started; ++i)
                if (alive[i]) kill(pid[i], SIGTERM);
        }
    }
    msa_shared_destroy(sh, world);
    return first_fail;
}

/* -------------------------------------------------------- external launchers
 * `mpirun -np N bin/parallel_spotify ...` -- the reference's own launch
 * (/root/reference/scripts/run_performance.sh:23; MPI_Init / MPI_Comm_rank /
 * MPI_Comm_size at parallel_spotify.c:725-730) -- starts N unrelated processes.
 * They join as the N ranks of this layer: rank and size from the launcher's
 * environment, a job key, and a shared block in /dev/shm named by that key
 * (created by rank 0, mapped by the others, unlinked once all have mapped it).
 *
 *   MPICH Hydra  PMI_RANK / PMI_SIZE; the job key is the PMI key-value space
 *                name, asked over the PMI-1 wire protocol on the descriptor
 *                Hydra passes in PMI_FD, whose barrier also orders the block's
 *                creation before the other ranks open it;
 *   Open MPI     OMPI_COMM_WORLD_RANK / _SIZE; the job key is PMIX_NAMESPACE
 *                (or OMPI_MCA_ess_base_jobid); the other ranks poll for the
 *                block rank 0 publishes.
 * One node only: the block is node-local shared memory. */

static int pmi_send(int fd, const char *cmd) {
    size_t len = strlen(cmd), done = 0;
    while (done < len) {
        const ssize_t w = write(fd, cmd + done, len - done);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) return -1;
        done += (size_t)w;
    }
    return 0;
}

/* one request, one response line (without its '\n') */
static int pmi_call(int fd, const char *cmd, char *resp, size_t n) {
    if (pmi_send(fd, cmd)) return -1;
    size_t k = 0;
    for (;;) {
        char c;
        const ssize_t r = read(fd, &c, 1);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return -1;
        if (c == '\n') break;
        if (k + 1 < n) resp[k++] = c;
    }
    resp[k] = 0;
    return 0;
}

/* value of `key=` in a PMI response line (space-separated key=value words) */
static int pmi_field(const char *resp, const char *key, char *out, size_t n) {
    const size_t kl = strlen(key);
    for (const char *p = resp; (p = strstr(p, key)); p += kl)
        if ((p == resp || p[-1] == ' ') && p[kl] == '=') {
            const char *v = p + kl + 1;
            const size_t m = strcspn(v, " ");
            if (m >= n) return -1;
            memcpy(out, v, m);
            out[m] = 0;
            return 0;
        }
    return -1;
}

/* rc=0, or no rc at all (Hydra's my_kvsname response carries none) */
static int pmi_rc_ok(const char *resp) {
    char v[16];
    return pmi_field(resp, "rc", v, sizeof v) != 0 || !strcmp(v, "0");
}

static int pmi_init(msa_launch *L) {
    char resp[512];
    if (pmi_call(L->pmi_fd, "cmd=init pmi_version=1 pmi_subversion=1\n", resp, sizeof resp) ||
        strncmp(resp, "cmd=response_to_init", 20) || !pmi_rc_ok(resp))
        return -1;
    if (pmi_call(L->pmi_fd, "cmd=get_my_kvsname\n", resp, sizeof resp) || strncmp(resp, "cmd=my_kvsname", 14) ||
        !pmi_rc_ok(resp) ||
        pmi_field(resp, "kvsname", L->key, sizeof L->key))
        return -1;
    return 0;
}

static int pmi_barrier(msa_launch *L) {
    char resp[128];
    return pmi_call(L->pmi_fd, "cmd=barrier_in\n", resp, sizeof resp) || strncmp(resp, "cmd=barrier_out", 15) ? -1 : 0;
}

static void pmi_finalize(msa_launch *L) {
    char resp[128];
    (void)pmi_call(L->pmi_fd, "cmd=finalize\n", resp, sizeof resp);
}

static int env_int(const char *name, int *v) {
    const char *s = getenv(name);
    if (!s || !*s) return 0;
    char *end = NULL;
    const long x = strtol(s, &end, 10);
    if (*end || x < 0 || x > 1 << 20) return -1;
    *v = (int)x;
    return 1;
}

int msa_launcher_detect(msa_launch *L) {
    memset(L, 0, sizeof *L);
    L->pmi_fd = -1;
    L->local_world = -1;
    int r = 0, w = 0, fd = -1, a, b;
    if ((a = env_int("PMI_RANK", &r)) && (b = env_int("PMI_SIZE", &w))) {
        if (a < 0 || b < 0) return -1;
        L->kind = "hydra";
        if (env_int("PMI_FD", &fd) == 1) L->pmi_fd = fd;
        else snprintf(L->key, sizeof L->key, "ppid%ld", (long)getppid());
        if (env_int("MPI_LOCALNRANKS", &L->local_world) < 0) return -1;
    } else if ((a = env_int("OMPI_COMM_WORLD_RANK", &r)) && (b = env_int("OMPI_COMM_WORLD_SIZE", &w))) {
        if (a < 0 || b < 0) return -1;
        L->kind = "openmpi";
        const char *ns = getenv("PMIX_NAMESPACE");
        if (!ns || !*ns) ns = getenv("OMPI_MCA_ess_base_jobid");
        if (ns && *ns) snprintf(L->key, sizeof L->key, "%s", ns);
        else snprintf(L->key, sizeof L->key, "ppid%ld", (long)getppid());
        if (env_int("OMPI_COMM_WORLD_LOCAL_SIZE", &L->local_world) < 0) return -1;
    } else {
        return 0;
    }
    if (w < 1 || r >= w) return -1;
    L->rank = r;
    L->world = w;
    return 1;
}

/* /dev/shm/msa_job_<key>, the key reduced to [A-Za-z0-9_.-] */
static void job_path(const msa_launch *L, char *path, size_t n) {
    char k[sizeof L->key];
    size_t i = 0;
    for (; L->key[i] && i + 1 < sizeof k; ++i) {
        const char c = L->key[i];
        k[i] = ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_' || c == '.' ||
                c == '-')
                   ? c
                   : '_';
    }
    k[i] = 0;
    snprintf(path, n, "/dev/shm/msa_job_%s_%d", k, L->world);
}

static msa_shared *job_create(const char *path, int world) {
    unlink(path); /* a block a crashed job of the same key left behind */
    const int fd = open(path, O_RDWR | O_CREAT | O_EXCL, 0600);
    if (fd < 0) return NULL;
    msa_shared *s = NULL;
    if (ftruncate(fd, (off_t)shared_bytes(world)) == 0) {
        s = mmap(NULL, shared_bytes(world), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (s == MAP_FAILED) s = NULL;
    }
    close(fd);
    if (!s) {
        unlink(path);
        return NULL;
    }
    shared_init(s, world);
    atomic_store(&s->ready, SH_READY);
    return s;
}

static int creator_alive(const msa_shared *s) {
    return s->tag > 0 && (kill((pid_t)s->tag, 0) == 0 || errno == EPERM);
}

/* the block rank 0 published; without PMI, poll for it (up to `wait_s`) */
static msa_shared *job_open(const char *path, int world, double wait_s) {
    struct timespec t0, t;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (;;) {
        const int fd = open(path, O_RDWR);
        if (fd >= 0) {
            struct stat st;
            msa_shared *s = NULL;
            if (fstat(fd, &st) == 0 && (size_t)st.st_size == shared_bytes(world)) {
                s = mmap(NULL, shared_bytes(world), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
                if (s == MAP_FAILED) s = NULL;
            }
            close(fd);
            /* a block whose creator is gone was left by a crashed job of the
             * same key: keep polling for rank 0's fresh one (job_create
             * unlinks the stale file before creating its own) */
            if (s && atomic_load(&s->ready) == SH_READY && s->world == world && creator_alive(s)) return s;
            if (s) munmap(s, shared_bytes(world));
        }
        clock_gettime(CLOCK_MONOTONIC, &t);
        if ((double)(t.tv_sec - t0.tv_sec) + 1e-9 * (double)(t.tv_nsec - t0.tv_nsec) > wait_s) return NULL;
        const struct timespec ts = {0, 2000000};
        nanosleep(&ts, NULL);
    }
}

int msa_launcher_run(msa_launch *L, int (*fn)(int, int, msa_shared *, void *), void *arg) {
    const int rank = L->rank, world = L->world;
    if (world > MSA_MAX_RANKS) {
        if (rank == 0) fprintf(stderr, "%d processes: at most %d are supported\n", world, MSA_MAX_RANKS);
        return 2;
    }
    if (L->local_world >= 0 && L->local_world != world) {
        if (rank == 0)
            fprintf(stderr, "the %d launched processes span more than one node (%d on this one): one node only\n",
                    world, L->local_world);
        return 2;
    }
    if (L->pmi_fd >= 0 && pmi_init(L)) {
        fprintf(stderr, "rank %d: PMI handshake with the launcher failed\n", rank);
        return 2;
    }
    char path[320];
    job_path(L, path, sizeof path);
    msa_shared *sh = NULL;
    int ok = 1;
    if (rank == 0) {
        sh = job_create(path, world);
        if (!sh) {
            fprintf(stderr, "rank 0: cannot create the shared rank block %s: %s\n", path, strerror(errno));
            ok = 0;
        }
    }
    if (L->pmi_fd >= 0 && pmi_barrier(L)) ok = 0; /* rank 0's block exists (or never will) */
    if (rank != 0 && ok) {
        sh = job_open(path, world, L->pmi_fd >= 0 ? 10.0 : 120.0);
        if (!sh) fprintf(stderr, "rank %d: no shared rank block %s from rank 0\n", rank, path);
    }
    if (!sh) {
        if (L->pmi_fd >= 0) pmi_finalize(L);
        return 2;
    }
    atomic_fetch_add(&sh->joined, 1);
    const int joined = sh_barrier(sh) == 0; /* every rank has mapped the block: its name can go */
    if (rank == 0) unlink(path);
    if (!joined) {
        munmap(sh, shared_bytes(world));
        if (L->pmi_fd >= 0) pmi_finalize(L);
        return 2;
    }
    fflush(stdout);
    const int rc = fn(rank, world, sh, arg);
    fflush(stdout);
    fflush(stderr);
    if (rc) {
        msa_shared_fail(sh);
        shared_unlink_files(sh);
    }
    munmap(sh, shared_bytes(world));
    if (L->pmi_fd >= 0) pmi_finalize(L);
    return rc;
}
