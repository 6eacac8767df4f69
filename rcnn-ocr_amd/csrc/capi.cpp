// Library-level entry points: version + thread-local error string.
#include <string.h>
#include <hip/hip_runtime.h>
#include "crnn_internal.hpp"

static thread_local char g_err[512] = "";

int crnn_set_error(int code, const char* msg) {
  strncpy(g_err, msg, sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = 0;
  return code ? code : (int)hipErrorInvalidValue;
}

extern "C" int crnn_version(void) { return 100; }

// tuning switches (A/B in one process); defaults are the measured-best settings
static int g_opts[CRNN_OPT_COUNT] = {1, 0, 1, 0, 0, 1, 3, 1, 1, 1, 1, 1, 0, 1, 2, 0, 2, 0, 1, 0, 1, 1, 1, 1};

int crnn_cu_count() {
  static int n = -1;
  if (n < 0) {
    int dev = 0;
    hipDeviceProp_t p;
    n = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) ? p.multiProcessorCount : 256;
    if (n < 1) n = 256;
  }
  return n;
}

int crnn_option(int key) { return (key >= 0 && key < CRNN_OPT_COUNT) ? g_opts[key] : 0; }

extern "C" int crnn_get_option(int key) { return crnn_option(key); }

extern "C" int crnn_set_option(int key, int value) {
  if (key < 0 || key >= CRNN_OPT_COUNT) return crnn_set_error((int)hipErrorInvalidValue, "crnn_set_option: bad key");
  g_opts[key] = value;
  return 0;
}

extern "C" const char* crnn_last_error_string(void) {
  if (g_err[0]) return g_err;
  return hipGetErrorString(hipGetLastError());
}
