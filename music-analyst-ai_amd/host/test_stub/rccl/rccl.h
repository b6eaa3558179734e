/* Test stand-in for RCCL (host/test_stub: CPU tests of host/msa_rccl.c only).
 * A communicator is one rank of an in-process "fabric" shared by the threads
 * that called ncclCommInitRank with the same id: all-gather and grouped
 * send/recv copy host memory between them, with the matching RCCL enforces
 * (a recv must meet a send of the same size from that peer). */
#ifndef MSA_STUB_RCCL_H
#define MSA_STUB_RCCL_H
#include <stddef.h>
#include <hip/hip_runtime_api.h>

typedef enum { ncclSuccess = 0, ncclUnhandledCudaError = 1, ncclSystemError = 2, ncclInternalError = 3,
               ncclInvalidArgument = 4, ncclInvalidUsage = 5 } ncclResult_t;
typedef enum { ncclUint8 = 1 } ncclDataType_t;
typedef struct { char internal[128]; } ncclUniqueId;
typedef struct stub_comm *ncclComm_t;

ncclResult_t ncclGetUniqueId(ncclUniqueId *id);
ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank);
ncclResult_t ncclCommDestroy(ncclComm_t comm);
ncclResult_t ncclAllGather(const void *send, void *recv, size_t count, ncclDataType_t t, ncclComm_t comm,
                           hipStream_t s);
ncclResult_t ncclGroupStart(void);
ncclResult_t ncclGroupEnd(void);
ncclResult_t ncclSend(const void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s);
ncclResult_t ncclRecv(void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s);
const char *ncclGetErrorString(ncclResult_t r);
#endif
