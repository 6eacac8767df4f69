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

extern "C" const char* crnn_last_error_string(void) {
  if (g_err[0]) return g_err;
  return hipGetErrorString(hipGetLastError());
}
