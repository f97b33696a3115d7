// Internal helpers shared by the libfsmi translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/fsmi.h"

namespace fsmi {

constexpr int kWave = 64;  // CDNA wavefront

void set_error(const char* fmt, ...);
void clear_error();

// Kernel-duration instrumentation (runtime.hip).  Construct before the
// launch, destroy after: records a start/stop hipEvent pair on `stream`
// when timing is enabled and the stream is not being captured.
class LaunchTimer {
 public:
  LaunchTimer(int kernel, hipStream_t stream);
  ~LaunchTimer();

 private:
  hipStream_t stream_;
  void* stop_ = nullptr;
};

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int finish_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return static_cast<int>(e);
  }
  return FSMI_OK;
}

inline unsigned ceil_div(long long a, long long b) { return static_cast<unsigned>((a + b - 1) / b); }

// XCD-aware block remap: the dispatcher deals blocks round-robin over the 8
// XCDs (MI355X_MICROARCH.md, workgroup dispatch), so block b and b+8 share an
// L2.  This bijection gives each XCD a contiguous range of logical work items
// so neighbouring items (which re-read the same rows) hit the same L2.
__device__ __forceinline__ unsigned xcd_remap(unsigned bid, unsigned nblocks) {
  const unsigned per = nblocks / 8u, rem = nblocks % 8u;
  const unsigned xcd = bid % 8u, slot = bid / 8u;
  // first `rem` XCDs own per+1 items, the rest own per
  const unsigned base = xcd < rem ? xcd * (per + 1u) : rem * (per + 1u) + (xcd - rem) * per;
  return base + slot;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

}  // namespace fsmi

#define FSMI_CHECK_ARG(cond, ...)          \
  do {                                     \
    if (!(cond)) {                         \
      ::fsmi::set_error(__VA_ARGS__);      \
      return FSMI_ERR_ARG;                 \
    }                                      \
  } while (0)
