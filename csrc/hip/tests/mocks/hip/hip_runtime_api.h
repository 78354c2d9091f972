// Minimal host-API stand-in for the RCCL-engine sanitizer self-test (no GPU, plain g++).
#pragma once
typedef int hipError_t;
enum { hipSuccess = 0 };
typedef struct ihipStream_t* hipStream_t;
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline const char* hipGetErrorString(hipError_t) { return "mock"; }
inline hipError_t hipGetLastError() { return hipSuccess; }
