// Shared helpers of libgnnrec: error reporting across the C ABI and launch checks.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "../../include/gnnrec.h"

namespace gnnrec {

// Thread-local message of the last failure (gnnrec_last_error()).
void set_error(const char* fmt, ...);

// Converts the launch status of the last kernel into a gnnrec_status.
int check_launch(const char* what);

inline hipStream_t as_hip(gnnrec_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

#define GNNREC_REQUIRE(cond, ...)          \
  do {                                     \
    if (!(cond)) {                         \
      ::gnnrec::set_error(__VA_ARGS__);    \
      return GNNREC_EINVAL;                \
    }                                      \
  } while (0)

// CSR operand as the kernels see it (row_ptr has n_rows+1 absolute offsets).
struct Csr {
  const int64_t* row_ptr;
  const int32_t* col;
  const float* val;
  int64_t n_rows;
};

}  // namespace gnnrec
