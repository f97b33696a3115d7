// Library plumbing: thread-local error text, version, live launch timing.
#include <mutex>
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

int fsmi_version(void) { return 100; }

const char* fsmi_last_error(void) { return fsmi::g_err.c_str(); }

const char* fsmi_arch(void) { return "gfx950"; }

int fsmi_timer_enable(int on) {
  std::lock_guard<std::mutex> lk(fsmi::g_mu);
  fsmi::g_enabled = on != 0;
  if (fsmi::g_enabled) {
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
