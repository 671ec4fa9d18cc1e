// Environment-driven fault injection. The reference has none;
// the resume / degradation / temporary-exit paths it relies on
// (erp_boinc_wrapper.cpp:560-570, demod_binary.c:546-652,
// cuda/app/demod_binary_hs_cuda.cu:207-219) are exercised here by setting
//
//   BRP_FAULT=<fault>[,<fault>...]     fault = name | name:param
//
//   kill_after_template:N  request a BOINC quit once N templates are done
//   hip_oom[:N]            every device allocation (after the first N) fails
//                          (-> temporary exit)
//   pinned_fail            every pinned host allocation fails (-> pageable)
//   hs_cap_raw             BRP_HS_CAP is taken as is, below the bounded output's size
//                          (the bounded output overflows: tie-storm re-run)
//   segv_after_template:N  invalid store once N templates are done (crash report)
//   slow_template:MS       sleep MS ms per applied template (paces client tests)
//   resource_error         the search returns a host allocation failure
//                          (-> BOINC temporary exit)
//   slow_exit:MS           finish() sleeps MS ms after reporting its status to the
//                          supervising parent (stands in for the GPU context's
//                          teardown in CPU tests of boinc::supervise)
//   collective_timeout[:R] rank R (default 1) stalls before the all-gather
//                          (Python side, parallel/dist.py)
#pragma once

#include <cstdlib>
#include <cstring>
#include <string>

namespace brp {

// Returns true if `name` is listed in BRP_FAULT; *param receives the text after
// "name:" (empty if none).
inline bool fault_enabled(const char* name, std::string* param = nullptr) {
  const char* env = std::getenv("BRP_FAULT");
  if (!env || !*env) return false;
  const size_t len = std::strlen(name);
  const char* p = env;
  while (*p) {
    const char* end = std::strchr(p, ',');
    const size_t tok = end ? static_cast<size_t>(end - p) : std::strlen(p);
    if (tok >= len && std::strncmp(p, name, len) == 0 && (tok == len || p[len] == ':')) {
      if (param) param->assign(tok > len ? p + len + 1 : p + tok, tok > len ? tok - len - 1 : 0);
      return true;
    }
    if (!end) break;
    p = end + 1;
  }
  return false;
}

}  // namespace brp
