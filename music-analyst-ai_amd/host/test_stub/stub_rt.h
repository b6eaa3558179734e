/* Counters and failure switches of the HIP / RCCL test stand-ins (stub_rt.c). */
#ifndef MSA_STUB_RT_H
#define MSA_STUB_RT_H
#include <stddef.h>
typedef struct {
    long mallocs, frees, live_allocs, streams_live, syncs, sends, recvs;
} stub_stats;
void stub_get_stats(stub_stats *s);
void stub_reset(void);
/* fail every ncclCommInitRank / the k-th hipMalloc (1-based; 0: never) */
void stub_fail_init(int on);
void stub_fail_malloc_at(long k);
#endif
