// Common host-side declarations for the MI355X hot-path library (libuvio_hp.so).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <stdexcept>
#include <string>

#include "../../include/uvio_hp.h"
#include "hp_math.h"

namespace uvhp {

void options_default(uvio_hp_options_t *o);
int options_load(const char *path, uvio_hp_options_t *o, std::string *err);

struct HpError : std::runtime_error {
  int code;
  HpError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define HP_HIP(call)                                                                                     \
  do {                                                                                                   \
    hipError_t e_ = (call);                                                                              \
    if (e_ != hipSuccess)                                                                                \
      throw ::uvhp::HpError(UVIO_HP_E_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_));     \
  } while (0)

}  // namespace uvhp
