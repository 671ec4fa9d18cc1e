#include "boinc_shim.hpp"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fcntl.h>
#include <fstream>
#include <sstream>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../core/log.hpp"

namespace brp {
namespace boinc {

namespace {
InitData g_init;
std::atomic<int> g_quit{0};
double g_fraction = 0.0;
double g_last_checkpoint = 0.0;
bool g_standalone = true;

std::string xml_tag(const std::string& doc, const char* tag) {
  const std::string open = std::string("<") + tag + ">";
  const std::string close = std::string("</") + tag + ">";
  const size_t a = doc.find(open);
  if (a == std::string::npos) return {};
  const size_t b = doc.find(close, a + open.size());
  if (b == std::string::npos) return {};
  return doc.substr(a + open.size(), b - a - open.size());
}

void parse_init_data() {
  std::ifstream f("init_data.xml");
  if (!f) return;
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string doc = ss.str();
  g_init.valid = true;
  g_standalone = false;
  std::string v;
  if (!(v = xml_tag(doc, "userid")).empty()) g_init.userid = std::atoi(v.c_str());
  g_init.user_name = xml_tag(doc, "user_name");
  if (!(v = xml_tag(doc, "hostid")).empty()) g_init.hostid = std::atoi(v.c_str());
  g_init.host_cpid = xml_tag(doc, "host_cpid");
  if (!(v = xml_tag(doc, "gpu_device_num")).empty()) g_init.gpu_device_num = std::atoi(v.c_str());
  if (!(v = xml_tag(doc, "checkpoint_period")).empty()) g_init.checkpoint_period = std::atof(v.c_str());
}

void write_progress_file() {
  // boinc_fraction_done: the client reads it from shared memory; standalone we
  // keep a small text file so harnesses (cf. debian runall.sh) can poll it
  const char* path = std::getenv("BRP_PROGRESS_FILE");
  if (!path) return;
  FILE* f = std::fopen(path, "w");
  if (!f) return;
  std::fprintf(f, "%.6f\n", g_fraction);
  std::fclose(f);
}
}  // namespace

int init(int, char**) {
  parse_init_data();
  const char* cp = std::getenv("BRP_CHECKPOINT_PERIOD");
  if (cp) g_init.checkpoint_period = std::atof(cp);
  g_last_checkpoint = dtime();
  return 0;
}

bool is_standalone() { return g_standalone; }
const InitData& init_data() { return g_init; }

int resolve_filename(const std::string& logical, std::string& physical) {
  physical = logical;
  // BOINC slot directories hold "soft link" files: <soft_link>../../projects/x</soft_link>
  FILE* f = std::fopen(logical.c_str(), "r");
  if (!f) return 0;
  char buf[512] = {0};
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* a = std::strstr(buf, "<soft_link>");
  if (a) {
    a += std::strlen("<soft_link>");
    const char* b = std::strstr(a, "</soft_link>");
    if (b) physical.assign(a, b - a);
  }
  return 0;
}

void fraction_done(double f) {
  g_fraction = f;
  write_progress_file();
}
double get_fraction_done() { return g_fraction; }

bool time_to_checkpoint() { return dtime() - g_last_checkpoint >= g_init.checkpoint_period; }
void checkpoint_completed() { g_last_checkpoint = dtime(); }
void begin_critical_section() {}
void end_critical_section() {}

Status get_status() {
  Status s;
  s.quit_request = g_quit.load() ? 1 : 0;
  struct rusage ru;
  if (getrusage(RUSAGE_SELF, &ru) == 0) s.working_set_size = ru.ru_maxrss * 1024.0;
  s.max_working_set_size = s.working_set_size;
  return s;
}

void request_quit() { g_quit.store(1); }
void clear_quit() { g_quit.store(0); }

double worker_thread_cpu_time() {
  struct rusage ru;
  if (getrusage(RUSAGE_SELF, &ru) != 0) return 0.0;
  return ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6 + ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6;
}

double dtime() {
  using namespace std::chrono;
  return duration<double>(system_clock::now().time_since_epoch()).count();
}

char* graphics_make_shmem(const char* app_name, int size) {
  const std::string path = std::string("boinc_") + app_name + "_0";
  const int fd = ::open(path.c_str(), O_RDWR | O_CREAT, 0666);
  if (fd < 0) return nullptr;
  if (ftruncate(fd, size) != 0) {
    ::close(fd);
    return nullptr;
  }
  void* p = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) return nullptr;
  std::memset(p, 0, size);
  return static_cast<char*>(p);
}

void finish(int status) {
  std::fflush(stdout);
  std::fflush(stderr);
  std::exit(status);
}

void temporary_exit(int delay_s, const char* reason) {
  log_message(LOG_WARN, true, "Temporary exit (%d s): %s\n", delay_s, reason ? reason : "");
  std::fflush(stderr);
  std::exit(0);
}

}  // namespace boinc
}  // namespace brp
