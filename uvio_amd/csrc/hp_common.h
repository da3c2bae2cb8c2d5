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

// Wait for a stream by polling it from this thread instead of hipStreamSynchronize: the calling thread stays
// on its core (a blocking wait lets the core idle and clock down, and the host work right after the wait -- the
// feature-database walks, the next batch -- then runs measurably slower).  Every host wait of the library is
// latency-critical and short (< a few ms).
inline void spin_sync(hipStream_t s) {
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady)
      throw HpError(UVIO_HP_E_DEVICE, std::string("hipStreamQuery: ") + hipGetErrorString(e));
    __builtin_ia32_pause();
  }
}

}  // namespace uvhp
