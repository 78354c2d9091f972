// RCCL API subset used by csrc/hip/comm.cpp, implemented by selftest_comm.cpp as a
// deterministic fake communicator (non-blocking semantics: calls may return ncclInProgress;
// ncclCommGetAsyncError reports progress; ncclCommAbort frees the communicator).
#pragma once
#include <cstddef>
#include "../hip/hip_runtime_api.h"

typedef enum { ncclSuccess = 0, ncclUnhandledCudaError = 1, ncclSystemError = 2, ncclInternalError = 3,
               ncclInvalidArgument = 4, ncclInvalidUsage = 5, ncclRemoteError = 6, ncclInProgress = 7 } ncclResult_t;
typedef enum { ncclInt8 = 0, ncclUint8 = 1, ncclInt32 = 2, ncclInt64 = 4, ncclFloat16 = 6, ncclFloat32 = 7,
               ncclBfloat16 = 9 } ncclDataType_t;
typedef enum { ncclSum = 0, ncclProd = 1, ncclMax = 2, ncclMin = 3, ncclAvg = 4 } ncclRedOp_t;
struct ncclComm;
typedef struct ncclComm* ncclComm_t;
typedef struct { char internal[128]; } ncclUniqueId;
typedef struct { int blocking; } ncclConfig_t;
#define NCCL_CONFIG_INITIALIZER {1}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id);
ncclResult_t ncclGetVersion(int* v);
const char* ncclGetErrorString(ncclResult_t r);
const char* ncclGetLastError(ncclComm_t c);
ncclResult_t ncclCommInitRankConfig(ncclComm_t* c, int n, ncclUniqueId id, int rank, ncclConfig_t* cfg);
ncclResult_t ncclCommGetAsyncError(ncclComm_t c, ncclResult_t* st);
ncclResult_t ncclCommAbort(ncclComm_t c);
ncclResult_t ncclCommFinalize(ncclComm_t c);
ncclResult_t ncclCommDestroy(ncclComm_t c);
ncclResult_t ncclAllReduce(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
ncclResult_t ncclBroadcast(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
ncclResult_t ncclAllGather(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
ncclResult_t ncclReduceScatter(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
ncclResult_t ncclAllToAll(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
ncclResult_t ncclGroupStart();
ncclResult_t ncclGroupEnd();
