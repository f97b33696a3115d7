// Library plumbing: thread-local error text, version, live launch timing.
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "fsmi_common.h"

namespace fsmi {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

void clear_error() { g_err.clear(); }

// --------------------------------------------------------------------------
// Launch timing.  Each launch of an instrumented kernel takes a (start, stop)
// event pair from a per-kernel pool; queries synchronise the recorded stops.
// --------------------------------------------------------------------------
namespace {
struct Pool {
  std::vector<hipEvent_t> start, stop;
  size_t used = 0;
};
std::mutex g_mu;
bool g_enabled = false;
bool g_clock_in_capture = false;   // fsmi_timer_enable(2 / 3): clock slots also inside stream capture
bool g_timeline = false;           // fsmi_timer_enable(3): every instrumented kernel takes a slot
Pool g_pool[FSMI_K_COUNT];

bool take(int k, hipEvent_t* s, hipEvent_t* e) {
  Pool& p = g_pool[k];
  if (p.used == p.start.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess) return false;
    if (hipEventCreate(&b) != hipSuccess) { (void)hipEventDestroy(a); return false; }
    p.start.push_back(a);
    p.stop.push_back(b);
  }
  *s = p.start[p.used];
  *e = p.stop[p.used];
  ++p.used;
  return true;
}
}  // namespace

// in-kernel clock: a device arena of per-wave (start, end) stamps, bump-allocated per launch and
// zeroed at enable / reset; per kernel the host keeps (offset, nwaves) of each launch.  16M stamps (128 MB)
// serve timer modes 1 / 2 (bench.py: only the geometry kernels stamp -- the hierarchical cfg5 step's
// captured lookups alone take ~6M, reserved for the process, plus as many for the eager pass after it;
// 4M stamps failed cfg3's and cfg5's lines); timer mode 3 (the timeline build's whole forward) grows it
// to 64M (512 MB) when no captured graph holds slots in it
constexpr size_t kClockArenaSmall = size_t(1) << 24;
constexpr size_t kClockArenaBig = size_t(1) << 26;
size_t g_clock_cap = 0;                                // stamps allocated
unsigned long long* g_clock = nullptr;
size_t g_clock_top = 0;
// slots handed to launches captured into a hipGraph (timer mode 2) stay reserved for the life of the
// process: the graph keeps writing them on every replay, so a later session (clock_init) must never
// hand the same addresses to new launches.  Sessions bump-allocate above this floor.
size_t g_clock_floor = 0;
// (offset, nwaves) per instrumented launch: eager launches of the current session (cleared by
// clock_init), and launches baked into captured graphs (kept across sessions, like their slots, until
// fsmi_timer_release_captured -- the graphs keep rewriting them on every replay)
std::vector<std::pair<size_t, long long>> g_clock_launch[FSMI_K_COUNT];
std::vector<std::pair<size_t, long long>> g_clock_captured[FSMI_K_COUNT];
// every captured launch in capture order, for fsmi_timer_dump_captured (the replay's timeline)
struct CapRecord {
  int kernel;
  size_t off;
  long long nwaves;
  const void* stream;
  std::string tag;
};
std::vector<CapRecord> g_clock_caplog;
// launches that found the arena full, eager (this session) and captured (reported by the queries)
long long g_clock_dropped[FSMI_K_COUNT], g_clock_dropped_cap[FSMI_K_COUNT];

static int clock_init(bool big = false) {
  const size_t want = big ? kClockArenaBig : kClockArenaSmall;
  if (g_clock && g_clock_cap < want && g_clock_floor == 0) {   // grow: no graph holds a slot in it
    if (hipDeviceSynchronize() != hipSuccess || hipFree(g_clock) != hipSuccess) return FSMI_ERR_ARG;
    g_clock = nullptr;
  }
  if (!g_clock) {
    if (hipMalloc(&g_clock, sizeof(unsigned long long) * want) != hipSuccess) {
      g_clock = nullptr;
      g_clock_cap = 0;
      return FSMI_ERR_ARG;
    }
    g_clock_cap = want;
  }
  if (hipMemset(g_clock + g_clock_floor, 0, sizeof(unsigned long long) * (g_clock_cap - g_clock_floor)) !=
      hipSuccess)
    return FSMI_ERR_ARG;
  g_clock_top = g_clock_floor;
  for (auto& v : g_clock_launch) v.clear();
  for (auto& d : g_clock_dropped) d = 0;
  return FSMI_OK;
}

unsigned long long* clock_slot(int kernel, hipStream_t stream, long long nwaves, const char* tag, bool timeline) {
  if (!g_enabled || !g_clock || nwaves <= 0 || (timeline && !g_timeline)) return nullptr;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &st) != hipSuccess) return nullptr;
  // inside a capture the slot pointer is baked into the graph node: every replay overwrites the same
  // stamps, so a query after replaying reads the last replay's launches (timer mode 2 only)
  if (st != hipStreamCaptureStatusNone && !g_clock_in_capture) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  const size_t need = 2 * static_cast<size_t>(nwaves);
  const bool captured = st != hipStreamCaptureStatusNone;
  if (g_clock_top + need > g_clock_cap) {
    // the query of this kernel fails instead of silently under-counting
    ++(captured ? g_clock_dropped_cap : g_clock_dropped)[kernel];
    return nullptr;
  }
  (captured ? g_clock_captured : g_clock_launch)[kernel].emplace_back(g_clock_top, nwaves);
  if (captured) g_clock_caplog.push_back({kernel, g_clock_top, nwaves, stream, tag ? tag : ""});
  unsigned long long* p = g_clock + g_clock_top;
  g_clock_top += need;
  if (captured) g_clock_floor = g_clock_top;   // baked into a graph: reserved
  return p;
}

std::function<void()> g_replay[FSMI_K_COUNT];
hipStream_t g_replay_stream[FSMI_K_COUNT];

void set_replay(int kernel, hipStream_t stream, std::function<void()> fn) {
  if (!g_enabled) return;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return;
  std::lock_guard<std::mutex> lk(g_mu);
  g_replay[kernel] = std::move(fn);
  g_replay_stream[kernel] = stream;
}

namespace {
std::mutex g_range_mu;
int* g_range_host = nullptr;
int* g_range_dev = nullptr;
int g_range_safe = 0;
}  // namespace

int range_safe() { return __atomic_load_n(&g_range_safe, __ATOMIC_RELAXED); }

// NaN-fill `out` when the range flag is set (one flag read per block): the last node of a captured
// forward, so a replay that overflowed never returns a finite disparity (fsmi_range_poison)
__global__ __launch_bounds__(256) void range_poison_kernel(const int* flag, float* out, long long n) {
  __shared__ int f;
  // a system-scope atomic load of the host-mapped flag (global_load ... sc0 sc1; a volatile load
  // became a flat load)
  if (threadIdx.x == 0) f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  if (!f) return;
  for (long long i = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * 256)
    out[i] = __builtin_nanf("");
}

int* range_flag_device() {
  std::lock_guard<std::mutex> lk(g_range_mu);
  if (!g_range_dev) {
    void* h = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&h, sizeof(int), hipHostMallocMapped) != hipSuccess) return nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipHostFree(h);
      return nullptr;
    }
    g_range_host = static_cast<int*>(h);
    *g_range_host = 0;
    g_range_dev = static_cast<int*>(d);
  }
  return g_range_dev;
}

LaunchTimer::LaunchTimer(int kernel, hipStream_t stream) : stream_(stream) {
  if (!g_enabled) return;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return;
  std::lock_guard<std::mutex> lk(g_mu);
  hipEvent_t s, e;
  if (!take(kernel, &s, &e)) return;
  (void)hipEventRecord(s, stream);
  stop_ = e;
}

LaunchTimer::~LaunchTimer() {
  if (stop_) (void)hipEventRecord(reinterpret_cast<hipEvent_t>(stop_), stream_);
}

}  // namespace fsmi

extern "C" {


}  // extern "C"

extern "C" {

int fsmi_version(void) { return 100; }

const char* fsmi_last_error(void) { return fsmi::g_err.c_str(); }

const char* fsmi_arch(void) { return "gfx950"; }

int fsmi_timer_enable(int on) {
  std::lock_guard<std::mutex> lk(fsmi::g_mu);
  fsmi::g_enabled = on != 0;
  fsmi::g_clock_in_capture = on >= 2;
  fsmi::g_timeline = on == 3;
  for (auto& f : fsmi::g_replay) f = nullptr;      // a replay only targets buffers of the current session
  if (fsmi::g_enabled) {
    if (fsmi::clock_init(fsmi::g_timeline) != FSMI_OK) {
      fsmi::set_error("fsmi_timer_enable: clock slots");
      return FSMI_ERR_ARG;
    }
    for (auto& p : fsmi::g_pool) {  // pre-create so the timed region does not pay for it
      while (p.start.size() < 64) {
        hipEvent_t a, b;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
          fsmi::set_error("fsmi_timer_enable: hipEventCreate failed");
          return FSMI_ERR_ARG;
        }
        p.start.push_back(a);
        p.stop.push_back(b);
      }
    }
  }
  return FSMI_OK;
}

int fsmi_timer_reset(void) {
  std::lock_guard<std::mutex> lk(fsmi::g_mu);
  for (auto& p : fsmi::g_pool) p.used = 0;
  for (auto& f : fsmi::g_replay) f = nullptr;
  if (fsmi::g_enabled) {
    if (hipDeviceSynchronize() != hipSuccess || fsmi::clock_init(fsmi::g_timeline) != FSMI_OK) {
      fsmi::set_error("fsmi_timer_reset: clock slots");
      return FSMI_ERR_ARG;
    }
  }
  return FSMI_OK;
}

int fsmi_timer_replay(int kernel, int reps, double* avg_ms) {
  FSMI_CHECK_ARG(kernel >= 0 && kernel < FSMI_K_COUNT && reps > 0, "fsmi_timer_replay: kernel %d reps %d", kernel,
                 reps);
  std::function<void()> fn;
  hipStream_t s;
  {
    std::lock_guard<std::mutex> lk(fsmi::g_mu);
    fn = fsmi::g_replay[kernel];
    s = fsmi::g_replay_stream[kernel];
  }
  FSMI_CHECK_ARG(static_cast<bool>(fn), "fsmi_timer_replay: no recorded launch of kernel %d", kernel);
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
    fsmi::set_error("fsmi_timer_replay: hipEventCreate failed");
    return FSMI_ERR_ARG;
  }
  hipError_t e = hipStreamSynchronize(s);
  fn();                                          // one untimed replay
  if (e == hipSuccess) e = hipEventRecord(e0, s);
  for (int i = 0; i < reps && e == hipSuccess; ++i) fn();
  if (e == hipSuccess) e = hipEventRecord(e1, s);
  if (e == hipSuccess) e = hipEventSynchronize(e1);
  float ms = 0.f;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (e != hipSuccess) {
    fsmi::set_error("fsmi_timer_replay: %s", hipGetErrorString(e));
    return static_cast<int>(e);
  }
  if (avg_ms) *avg_ms = static_cast<double>(ms) / reps;
  return FSMI_OK;
}

int fsmi_range_status(int reset, int* overflowed) {
  FSMI_CHECK_ARG(overflowed, "fsmi_range_status: null pointer");
  if (!fsmi::range_flag_device()) {
    fsmi::set_error("fsmi_range_status: host-mapped flag unavailable");
    return FSMI_ERR_ARG;
  }
  std::lock_guard<std::mutex> lk(fsmi::g_range_mu);
  *overflowed = __atomic_load_n(fsmi::g_range_host, __ATOMIC_ACQUIRE);
  if (reset) __atomic_store_n(fsmi::g_range_host, 0, __ATOMIC_RELEASE);
  return FSMI_OK;
}

int fsmi_range_poison(float* out, long long n, void* stream) {
  FSMI_CHECK_ARG(out && n >= 0, "fsmi_range_poison: bad output");
  int* flag = fsmi::range_flag_device();
  FSMI_CHECK_ARG(flag, "fsmi_range_poison: host-mapped flag unavailable");
  if (n == 0) return FSMI_OK;
  hipStream_t s = fsmi::as_stream(stream);
  hipLaunchKernelGGL(fsmi::range_poison_kernel, dim3(static_cast<unsigned>((n + 255) / 256 < 64 ? (n + 255) / 256 : 64)), dim3(256),
                     0, s, flag, out, n);
  return fsmi::finish_launch("fsmi_range_poison");
}

int fsmi_set_range_safe(int safe) {
  __atomic_store_n(&fsmi::g_range_safe, safe ? 1 : 0, __ATOMIC_RELAXED);
  return FSMI_OK;
}

int fsmi_get_range_safe(int* safe) {
  FSMI_CHECK_ARG(safe, "fsmi_get_range_safe: null pointer");
  *safe = fsmi::range_safe();
  return FSMI_OK;
}

static int query_clock(const std::vector<std::pair<size_t, long long>>& launches, double* total_ms,
                       long long* count) {
  double tot = 0.0;
  long long n = 0;
  if (!launches.empty()) {
    hipError_t e = hipDeviceSynchronize();
    std::vector<unsigned long long> v;
    for (const auto& l : launches) {
      v.resize(2 * static_cast<size_t>(l.second));
      if (e == hipSuccess)
        e = hipMemcpy(v.data(), fsmi::g_clock + l.first, v.size() * sizeof(unsigned long long),
                      hipMemcpyDeviceToHost);
      if (e != hipSuccess) {
        fsmi::set_error("fsmi_timer_query_clock: %s", hipGetErrorString(e));
        return static_cast<int>(e);
      }
      unsigned long long t0 = ~0ULL, t1 = 0;
      for (size_t i = 0; i < v.size(); i += 2) {
        if (v[i]) t0 = std::min(t0, v[i]);
        t1 = std::max(t1, v[i + 1]);
      }
      if (t1 > t0) {
        tot += static_cast<double>(t1 - t0) * 1e-5;   // 100 MHz ticks -> ms
        ++n;
      }
    }
  }
  if (total_ms) *total_ms = tot;
  if (count) *count = n;
  return FSMI_OK;
}

int fsmi_timer_query_clock(int kernel, double* total_ms, long long* count) {
  FSMI_CHECK_ARG(kernel >= 0 && kernel < FSMI_K_COUNT, "fsmi_timer_query_clock: bad kernel id %d", kernel);
  std::lock_guard<std::mutex> lk(fsmi::g_mu);
  FSMI_CHECK_ARG(fsmi::g_clock_dropped[kernel] == 0, "fsmi_timer_query_clock: %lld launches of kernel %d found the "
                 "clock arena full", fsmi::g_clock_dropped[kernel], kernel);
  return query_clock(fsmi::g_clock_launch[kernel], total_ms, count);
}

int fsmi_timer_query_clock_captured(int kernel, double* total_ms, long long* count) {
  FSMI_CHECK_ARG(kernel >= 0 && kernel < FSMI_K_COUNT, "fsmi_timer_query_clock_captured: bad kernel id %d", kernel);
  std::lock_guard<std::mutex> lk(fsmi::g_mu);
  FSMI_CHECK_ARG(fsmi::g_clock_dropped_cap[kernel] == 0, "fsmi_timer_query_clock_captured: %lld captured launches "
                 "of kernel %d found the clock arena full", fsmi::g_clock_dropped_cap[kernel], kernel);
  return query_clock(fsmi::g_clock_captured[kernel], total_ms, count);
}

int fsmi_timer_dump_captured(char* buf, long long size, long long* needed) {
  std::lock_guard<std::mutex> lk(fsmi::g_mu);
  std::string text;
  if (!fsmi::g_clock_caplog.empty()) {
    hipError_t e = hipDeviceSynchronize();
    std::vector<unsigned long long> v;
    char line[96];
    for (const auto& r : fsmi::g_clock_caplog) {
      v.resize(2 * static_cast<size_t>(r.nwaves));
      if (e == hipSuccess)
        e = hipMemcpy(v.data(), fsmi::g_clock + r.off, v.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
      if (e != hipSuccess) {
        fsmi::set_error("fsmi_timer_dump_captured: %s", hipGetErrorString(e));
        return static_cast<int>(e);
      }
      unsigned long long t0 = ~0ULL, t1 = 0;
      for (size_t i = 0; i < v.size(); i += 2) {
        if (v[i]) t0 = std::min(t0, v[i]);
        t1 = std::max(t1, v[i + 1]);
      }
      if (t0 == ~0ULL) t0 = 0;
      snprintf(line, sizeof(line), "%d %p %llu %llu ", r.kernel, r.stream, t0, t1);
      text += line;
      text += r.tag;
      text += "\n";
    }
  }
  if (needed) *needed = static_cast<long long>(text.size()) + 1;
  if (buf && size > 0) {
    const size_t n = std::min(text.size(), static_cast<size_t>(size - 1));
    memcpy(buf, text.data(), n);
    buf[n] = 0;
  }
  return FSMI_OK;
}

int fsmi_timer_captured_count(long long* n) {
  FSMI_CHECK_ARG(n, "fsmi_timer_captured_count: null pointer");
  std::lock_guard<std::mutex> lk(fsmi::g_mu);
  *n = static_cast<long long>(fsmi::g_clock_caplog.size());
  return FSMI_OK;
}

int fsmi_timer_release_captured(void) {
  std::lock_guard<std::mutex> lk(fsmi::g_mu);
  for (auto& v : fsmi::g_clock_captured) v.clear();
  fsmi::g_clock_caplog.clear();
  for (auto& d : fsmi::g_clock_dropped_cap) d = 0;
  fsmi::g_clock_floor = 0;
  fsmi::g_clock_top = 0;
  // the slots are handed out again from 0: start a clean session (the arena zeroed, this session's eager
  // records -- which point into slots about to be reused -- and their drop counts cleared), so a later
  // launch never reads another launch's stale stamps
  if (fsmi::g_clock) {
    if (hipDeviceSynchronize() != hipSuccess || fsmi::clock_init(fsmi::g_timeline) != FSMI_OK) {
      fsmi::set_error("fsmi_timer_release_captured: clock slots");
      return FSMI_ERR_ARG;
    }
  }
  return FSMI_OK;
}

int fsmi_timer_query(int kernel, double* total_ms, long long* count) {
  FSMI_CHECK_ARG(kernel >= 0 && kernel < FSMI_K_COUNT, "fsmi_timer_query: bad kernel id %d", kernel);
  std::lock_guard<std::mutex> lk(fsmi::g_mu);
  fsmi::Pool& p = fsmi::g_pool[kernel];
  double tot = 0.0;
  for (size_t i = 0; i < p.used; ++i) {
    hipError_t e = hipEventSynchronize(p.stop[i]);
    if (e != hipSuccess) {
      fsmi::set_error("fsmi_timer_query: %s", hipGetErrorString(e));
      return static_cast<int>(e);
    }
    float ms = 0.f;
    e = hipEventElapsedTime(&ms, p.start[i], p.stop[i]);
    if (e != hipSuccess) {
      fsmi::set_error("fsmi_timer_query: %s", hipGetErrorString(e));
      return static_cast<int>(e);
    }
    tot += ms;
  }
  if (total_ms) *total_ms = tot;
  if (count) *count = static_cast<long long>(p.used);
  return FSMI_OK;
}

}  // extern "C"
