// ORACLE — test infrastructure only (see la.h header).  The C-ABI handle of the restatement (capi.cpp, probe.cpp).
#pragma once
#include <string>

#include "manager.h"

struct orc_handle {
  orc::Manager m;
  std::string err;
  explicit orc_handle(const uvio_hp_options_t &o) : m(o) {}
};
