#include "ipc.hpp"

#include <cstdio>
#include <cstring>
#include <iomanip>
#include <sstream>

#include "runtime.hpp"

namespace brp {
namespace ipc {

namespace {
char* g_shmem = nullptr;
double g_last_update = 0.0;

std::string fixed3(double v) {
  std::ostringstream o;
  o << std::fixed << std::setprecision(3) << v;
  return o.str();
}
std::string general3(double v) {
  std::ostringstream o;
  o << std::setprecision(3) << v;
  return o.str();
}
}  // namespace

std::string render_xml(const SearchInfo& info) {
  std::ostringstream ps;
  for (int i = 0; i < kBinsScreensaver; ++i)
    ps << std::setw(2) << std::setfill('0') << std::hex << static_cast<int>(info.power_spectrum[i]);
  const boinc::Status st = boinc::get_status();
  std::ostringstream x;
  x << "<?xml version=\"1.0\" encoding=\"UTF-8\"?>\n";
  x << "<graphics_info>\n";
  x << "  <skypos_rac>" << fixed3(info.skypos_rac) << "</skypos_rac>\n";
  x << "  <skypos_dec>" << fixed3(info.skypos_dec) << "</skypos_dec>\n";
  x << "  <dispersion>" << fixed3(info.dispersion_measure) << "</dispersion>\n";
  x << "  <orb_radius>" << fixed3(info.orbital_radius) << "</orb_radius>\n";
  x << "  <orb_period>" << fixed3(info.orbital_period) << "</orb_period>\n";
  x << "  <orb_phase>" << fixed3(info.orbital_phase) << "</orb_phase>\n";
  x << "  <power_spectrum>" << ps.str() << "</power_spectrum>\n";
  x << "  <fraction_done>" << fixed3(boinc::get_fraction_done()) << "</fraction_done>\n";
  x << "  <cpu_time>" << fixed3(boinc::worker_thread_cpu_time()) << "</cpu_time>\n";
  x << "  <update_time>" << fixed3(boinc::dtime()) << "</update_time>\n";
  x << "  <boinc_status>\n";
  x << "    <no_heartbeat>" << st.no_heartbeat << "</no_heartbeat>\n";
  x << "    <suspended>" << st.suspended << "</suspended>\n";
  x << "    <quit_request>" << st.quit_request << "</quit_request>\n";
  x << "    <reread_init_data_file>" << st.reread_init_data_file << "</reread_init_data_file>\n";
  x << "    <abort_request>" << st.abort_request << "</abort_request>\n";
  x << "    <working_set_size>" << general3(st.working_set_size) << "</working_set_size>\n";
  x << "    <max_working_set_size>" << general3(st.max_working_set_size) << "</max_working_set_size>\n";
  x << "  </boinc_status>\n";
  x << "</graphics_info>\n";
  return x.str();
}

int setup_shmem() {
  g_shmem = boinc::graphics_make_shmem(kShmemAppName, kShmemSize);
  if (!g_shmem) {
    std::fprintf(stderr, "Failed to create shared memory area!\n");
    return -1;
  }
  update_shmem(SearchInfo());
  return 0;
}

bool update_due() { return boinc::dtime() - g_last_update >= 1.0; }

void update_shmem(const SearchInfo& info) {
  if (!g_shmem) return;
  g_last_update = boinc::dtime();
  const std::string doc = render_xml(info);
  std::memset(g_shmem, 0, kShmemSize);
  if (!doc.empty() && doc.size() < static_cast<size_t>(kShmemSize)) {
    std::memcpy(g_shmem, doc.data(), doc.size());  // NUL-terminated by the memset
  } else {
    std::fprintf(stderr, "Error writing shared memory data (size limit exceeded)!\n");
  }
}

}  // namespace ipc
}  // namespace brp
