// Error channel, version and tuning table of the pis_* C-ABI (include/pis_capi.h).
#include <atomic>
#include <cstdarg>

#include "common.h"

namespace pis {
static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

// kernel-variant knobs (defaults = the measured best on MI355X)
static std::atomic<int> g_tune[PIS_TUNE_NKEYS] = {0, 16, 0, 1, 0, 1, 512, 0, 1, 1024, 4, 1, 0, 4, 3, 1, 1, 2,
                                                   1, 1, 1, 0, 1, 0, 0, 0, 2, 1, 0, 1, 0, 1, 1, 0, 0, 512, 0, 0, 1, 2, 2, 0, 1, 1, 0, 0, 1,
                                                   0, 1, 2};

int tune_get(int key) { return (key > 0 && key < PIS_TUNE_NKEYS) ? g_tune[key].load() : 0; }

static std::atomic<pis_launch_hook_t> g_hook{nullptr};
static std::atomic<void*> g_hook_user{nullptr};

void launch_hook(const char* kernel, int phase, hipStream_t s, double flop) {
  const pis_launch_hook_t fn = g_hook.load(std::memory_order_relaxed);
  if (fn) fn(kernel, phase, (pis_stream_t)s, flop, g_hook_user.load(std::memory_order_relaxed));
}

// pis_arm_gemm_event: an event the NEXT F(4x4) contraction launched by this thread records on its
// stream right after the GEMM (before the output transform), then the slot is disarmed
static thread_local hipEvent_t g_gemm_event = nullptr;

void gemm_done(hipStream_t s) {
  if (g_gemm_event) {
    (void)hipEventRecord(g_gemm_event, s);
    g_gemm_event = nullptr;
  }
}
}  // namespace pis

extern "C" const char* pis_last_error(void) { return pis::g_last_error; }
extern "C" int pis_version(void) { return 1; }

extern "C" int pis_arm_gemm_event(void* event) {
  const int pending = pis::g_gemm_event != nullptr;
  pis::g_gemm_event = (hipEvent_t)event;
  return pending;
}

extern "C" int pis_stream_create(int priority, pis_stream_t* out) {
  PIS_CHECK_ARG(out != nullptr, "pis_stream_create: out is NULL");
  hipStream_t s = nullptr;
  const hipError_t e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority);
  if (e != hipSuccess) {
    pis::set_error("pis_stream_create: %s", hipGetErrorString(e));
    return PIS_ERR_LAUNCH;
  }
  *out = (pis_stream_t)s;
  return PIS_OK;
}

extern "C" int pis_stream_destroy(pis_stream_t stream) {
  PIS_CHECK_ARG(stream != nullptr, "pis_stream_destroy: NULL stream");
  const hipError_t e = hipStreamDestroy((hipStream_t)stream);
  if (e != hipSuccess) {
    pis::set_error("pis_stream_destroy: %s", hipGetErrorString(e));
    return PIS_ERR_LAUNCH;
  }
  return PIS_OK;
}

extern "C" int pis_stream_capture_status(pis_stream_t stream) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  const hipError_t e = hipStreamIsCapturing((hipStream_t)stream, &st);
  if (e != hipSuccess) {
    pis::set_error("pis_stream_capture_status: %s", hipGetErrorString(e));
    return PIS_ERR_LAUNCH;
  }
  return (int)st;
}

extern "C" void pis_set_launch_hook(pis_launch_hook_t fn, void* user) {
  pis::g_hook_user.store(user);
  pis::g_hook.store(fn);
}

extern "C" int pis_tune(int key, int value) {
  if (key <= 0 || key >= PIS_TUNE_NKEYS) {
    pis::set_error("pis_tune: unknown key %d", key);
    return PIS_ERR_ARG;
  }
  if (key == PIS_TUNE_IGEMM_BK && value >= 0 && value != 16 && value != 32) {
    pis::set_error("pis_tune: igemm K-step must be 16 or 32");
    return PIS_ERR_ARG;
  }
  const int prev = pis::g_tune[key].load();
  if (value >= 0) pis::g_tune[key].store(value);
  return prev;
}
