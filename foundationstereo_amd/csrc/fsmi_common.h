// Internal helpers shared by the libfsmi translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <functional>
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

// In-kernel launch clock (runtime.hip): while timing is on and the stream is not being captured,
// an instrumented launch gets a zeroed device array of 2 x nwaves stamps (s_memrealtime, 100 MHz):
// every wave stores its start at the top and its end after its stores are acknowledged -- plain
// stores to its own slot, no atomics (same-address atomics from ~10k waves cost the lookup 3x).
// The host takes max(end) - min(start) per launch; waves that exit early leave a 0 end.
// nullptr otherwise (graph replays carry no clock).  bench.py divides the roofline bytes by this
// duration: the kernel's execution time, without the event-record latency around a launch.
// timeline = true: the launch takes a slot only in timer mode 3 (a whole forward's timeline,
// fsmi_timer_dump_captured); the geometry kernels (false) take one in modes 1 / 2 as well
unsigned long long* clock_slot(int kernel, hipStream_t stream, long long nwaves, const char* tag = nullptr,
                               bool timeline = false);


// Replay hook for fsmi_timer_replay: while timing is on (and not capturing), an instrumented
// entry point registers a closure that re-issues its last launch with identical arguments on the
// same stream (the kernels are pure functions of their inputs, so re-running them rewrites the
// same outputs).  bench.py times a back-to-back batch of replays between two hipEvents, which
// amortises the event-record latency a single bracketed launch carries.
void set_replay(int kernel, hipStream_t stream, std::function<void()> fn);

// Range flag of the split-precision convs (runtime.hip): one host-mapped int (pinned host memory
// the GPU writes through its device alias), allocated on first use; kernels store 1 into it when
// a scaled activation left fp16's range.  Read / reset by fsmi_range_status.  nullptr if the
// allocation failed (the kernels then skip the flag).
int* range_flag_device();
// Safe range mode (fsmi_set_range_safe): 2D convs take a per-chunk exponent (mode 1) instead of
// one fixed from the first nonzero chunk; read when a launch's arguments are built.
int range_safe();

// the wave's slot index, wave-uniform (readfirstlane: SGPRs, so a value the compiler keeps from the
// begin stamp to the end stamp costs the main loop no VGPR -- the per-lane form cost the conv tiles
// 5-20 VGPRs and the cfg2 step 5 %, round 5)
__device__ __forceinline__ unsigned clock_wave_id() {
  const unsigned blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const unsigned wpb = (blockDim.x * blockDim.y * blockDim.z + 63) / 64;
  const unsigned w = __builtin_amdgcn_readfirstlane((threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z)) / 64);
  return __builtin_amdgcn_readfirstlane(blk * wpb + w);
}
// every lane of the wave stores the same stamp to the same slot (one vector store, no lane predicate)
__device__ __forceinline__ void clock_begin(unsigned long long* slot) {
  if (slot) slot[2 * static_cast<size_t>(clock_wave_id())] = wall_clock64();
}
__device__ __forceinline__ void clock_end(unsigned long long* slot) {
  if (slot) {
    __builtin_amdgcn_s_waitcnt(0);
    slot[2 * static_cast<size_t>(clock_wave_id()) + 1] = wall_clock64();
  }
}

// Clock of a kernel whose waves may leave early: the end stamp from the scope's exit (destructor).
struct ClockScope {
  unsigned long long* slot;
  __device__ __forceinline__ explicit ClockScope(unsigned long long* s) : slot(s) { clock_begin(s); }
  __device__ __forceinline__ ~ClockScope() { clock_end(slot); }
};

// The conv / pointwise / MLP / aux kernels stamp their clocks only in the timeline build
// (FSMI_TIMELINE=1, _lib/libfsmi_timeline.so for tools/replay_timeline.py): even a disabled stamp kept
// the slot pointer and the wave id live through the main loops and cost the cfg2 step 5 % (round 5).
// The geometry kernels (build, all-pairs, pyramid, lookup) stamp in every build (bench.py's roofline).
#ifndef FSMI_TIMELINE
#define FSMI_TIMELINE 0
#endif
#if FSMI_TIMELINE
#define FSMI_TIMELINE_CLOCK(slot) ClockScope fsmi_clock_scope_(slot)
#else
#define FSMI_TIMELINE_CLOCK(slot) (void)(slot)
#endif

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
