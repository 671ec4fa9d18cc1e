#include "log.hpp"
#include "errors.hpp"
#include "formats.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <mutex>
#include <unistd.h>

namespace brp {

namespace {
int g_level = -1;
std::mutex g_log_mutex;

int init_level() {
  const char* env = std::getenv("BRP_LOGLEVEL");
  if (env) {
    int v = std::atoi(env);
    if (v >= LOG_ERROR && v <= LOG_DEBUG) return v;
  }
  return LOG_INFO;
}
}  // namespace

void set_log_level(int level) { g_level = level; }
int log_level() {
  if (g_level < 0) g_level = init_level();
  return g_level;
}

void log_vmessage(LogLevel level, bool show_level, const char* fmt, va_list ap) {
  if (level > log_level()) return;
  std::lock_guard<std::mutex> lock(g_log_mutex);
  FILE* out = (level == LOG_DEBUG) ? stdout : stderr;
  const char* tag = "UNKWN";
  switch (level) {
    case LOG_ERROR: tag = "ERROR"; break;
    case LOG_WARN: tag = "WARN "; break;
    case LOG_INFO: tag = "INFO "; break;
    case LOG_DEBUG: tag = "DEBUG"; break;
  }
  // a leading newline in the message is printed before the prefix
  if (fmt[0] == '\n') {
    std::fputc('\n', out);
    if (fmt[1] != '\0') ++fmt;
  }
  if (show_level) {
    char tbuf[16] = {0};
    std::time_t now = std::time(nullptr);
    std::tm tm_local;
    localtime_r(&now, &tm_local);
    std::strftime(tbuf, sizeof(tbuf), "%H:%M:%S", &tm_local);
    std::fprintf(out, "[%s][%d][%s] ", tbuf, static_cast<int>(getpid()), tag);
  } else {
    std::fputs("------> ", out);
  }
  std::vfprintf(out, fmt, ap);
  std::fflush(out);
}

void log_message(LogLevel level, bool show_level, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  log_vmessage(level, show_level, fmt, ap);
  va_end(ap);
}

const char* error_string(int code) {
  switch (code) {
    case RADPUL_OK: return "success";
    case RADPUL_EMEM: return "out of memory";
    case RADPUL_EFILE: return "file error";
    case RADPUL_EIO: return "I/O error";
    case RADPUL_EVAL: return "invalid value";
    case RADPUL_EMISC: return "miscellaneous error";
    case RADPUL_HIP_DEVICE_FIND: return "no usable HIP device";
    case RADPUL_HIP_DEVICE_SET: return "cannot select HIP device";
    case RADPUL_HIP_DEVICE_PROP: return "cannot query HIP device";
    case RADPUL_HIP_MEM_ALLOC_HOST: return "host (pinned) allocation failed";
    case RADPUL_HIP_MEM_ALLOC_DEVICE: return "device allocation failed";
    case RADPUL_HIP_MEM_COPY_HOST_DEVICE: return "host->device copy failed";
    case RADPUL_HIP_MEM_COPY_DEVICE_HOST: return "device->host copy failed";
    case RADPUL_HIP_FFT_PLAN: return "unsupported FFT length";
    case RADPUL_HIP_KERNEL_INVOKE: return "kernel launch failed";
    case RADPUL_HIP_GRAPH: return "HIP graph error";
    case RADPUL_HIP_CAND_OVERFLOW: return "candidate buffer overflow";
    case RADPUL_HIP_COLLECTIVE: return "collective communication failed";
    case EINSTEINRADIO_EMEM: return "wrapper out of memory";
    case EINSTEINRADIO_EOPT: return "invalid option";
    default: return "unknown error";
  }
}

bool host_is_big_endian() {
  const uint16_t word = 0x0001;
  return reinterpret_cast<const uint8_t*>(&word)[0] == 0;
}

void endian_swap(uint8_t* data, size_t elem_size, size_t n) {
  if (elem_size <= 1) return;
  for (size_t e = 0; e < n; ++e, data += elem_size) {
    for (size_t a = 0, b = elem_size - 1; a < b; ++a, --b) {
      uint8_t t = data[a];
      data[a] = data[b];
      data[b] = t;
    }
  }
}

void swap_header(DDHeader& h) {
  double* d = &h.tsample;  // 15 leading doubles
  endian_swap(reinterpret_cast<uint8_t*>(d), sizeof(double), 15);
  endian_swap(reinterpret_cast<uint8_t*>(&h.filesize), sizeof(uint32_t), 3);
  endian_swap(reinterpret_cast<uint8_t*>(&h.smprec), sizeof(uint16_t), 6);
}

}  // namespace brp
