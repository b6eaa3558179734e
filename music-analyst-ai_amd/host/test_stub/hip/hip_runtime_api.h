/* Test stand-in for the HIP runtime API (host/test_stub: CPU tests of
 * host/msa_rccl.c only, never linked into the product).  "Device" memory is
 * host memory; streams are bookkeeping; allocations and syncs are counted and
 * can be made to fail (stub_rt.h). */
#ifndef MSA_STUB_HIP_RUNTIME_API_H
#define MSA_STUB_HIP_RUNTIME_API_H
#include <stddef.h>

typedef int hipError_t;
#define hipSuccess 0
#define hipErrorOutOfMemory 2
#define hipErrorInvalidDevice 101
typedef struct stub_stream *hipStream_t;
#define hipStreamNonBlocking 1u
typedef enum { hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2, hipMemcpyDeviceToDevice = 3 } hipMemcpyKind;

hipError_t hipSetDevice(int device);
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned flags);
hipError_t hipStreamDestroy(hipStream_t s);
hipError_t hipStreamSynchronize(hipStream_t s);
hipError_t hipMalloc(void **p, size_t n);
hipError_t hipFree(void *p);
hipError_t hipMemcpyAsync(void *dst, const void *src, size_t n, hipMemcpyKind k, hipStream_t s);
const char *hipGetErrorString(hipError_t e);
#endif
