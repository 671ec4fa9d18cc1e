// Error-code space. The RADPUL_* values are the reference's (demod_binary.h:25-73)
// so BOINC-side tooling that interprets exit codes keeps working. The HIP
// backend gets its own 3001+ block; allocation failures map to a BOINC
// temporary exit exactly like the CUDA/OpenCL ones (erp_boinc_wrapper.cpp:560-570).
#pragma once

namespace brp {

enum ErrorCode : int {
  RADPUL_OK = 0,
  RADPUL_EMEM = 1,
  RADPUL_EFILE = 2,
  RADPUL_EIO = 3,
  RADPUL_EVAL = 4,
  RADPUL_EMISC = 5,

  // MI355X/HIP backend
  RADPUL_HIP_DEVICE_FIND = 3001,
  RADPUL_HIP_DEVICE_SET = 3002,
  RADPUL_HIP_DEVICE_PROP = 3003,
  RADPUL_HIP_MEM_ALLOC_HOST = 3005,
  RADPUL_HIP_MEM_ALLOC_DEVICE = 3006,
  RADPUL_HIP_MEM_COPY_HOST_DEVICE = 3007,
  RADPUL_HIP_MEM_COPY_DEVICE_HOST = 3008,
  RADPUL_HIP_FFT_PLAN = 3011,
  RADPUL_HIP_KERNEL_INVOKE = 3015,
  RADPUL_HIP_GRAPH = 3016,
  RADPUL_HIP_CAND_OVERFLOW = 3017,
  RADPUL_HIP_COLLECTIVE = 3018,

  // wrapper (reference erp_boinc_wrapper.h option errors)
  EINSTEINRADIO_EXIT = 0,
  EINSTEINRADIO_EMEM = 10,
  EINSTEINRADIO_EOPT = 11,
};

// Errors for which the BOINC wrapper requests a temporary exit (retry later).
inline bool is_transient_resource_error(int code) {
  return code == RADPUL_HIP_MEM_ALLOC_HOST || code == RADPUL_HIP_MEM_ALLOC_DEVICE ||
         code == RADPUL_HIP_FFT_PLAN;
}

const char* error_string(int code);

}  // namespace brp
