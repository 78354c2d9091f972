// Host-only helpers shared by the kernels' launch code and the RCCL engine: error checks and
// the raw-stream conversion.  Needs only the HIP host API, so comm.cpp (and its sanitizer
// self-test with mocked HIP / RCCL headers, tests/test_native_sanitize.py) builds without
// the device toolchain.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace voda {

#define VODA_HIP_CHECK(expr)                                                              \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +       \
                               " at " __FILE__ ":" + std::to_string(__LINE__));         \
  } while (0)

#define VODA_CHECK(cond, msg)                                                            \
  do {                                                                                   \
    if (!(cond)) throw std::invalid_argument(std::string("vodascheduler_amd: ") + (msg)); \
  } while (0)

enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

inline hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace voda
