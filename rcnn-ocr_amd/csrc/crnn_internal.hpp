// Internal helpers shared by the .hip translation units of libcrnn_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include "crnn_hip.h"

// records a message for crnn_last_error_string() and returns `code`
int crnn_set_error(int code, const char* msg);
// crnn_set_option() values (capi.cpp)
int crnn_option(int key);
// compute units of the current device (capi.cpp, cached)
int crnn_cu_count();

inline int grid_for(long n, int block = 256, int cap = 8192) {
  long g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}
