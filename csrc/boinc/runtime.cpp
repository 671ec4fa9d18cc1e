#include "runtime.hpp"

#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <thread>

#include "../core/fault.hpp"
#include "../core/log.hpp"
#include "../core/trace.hpp"
#include "client_shm.hpp"

namespace brp {
namespace boinc {

namespace {

constexpr double kTimerPeriod = 0.1;     // s between services of the channels
constexpr double kStatusPeriod = 1.0;    // s between app status messages
constexpr double kHeartbeatGiveup = 30;  // s without a heartbeat before leaving

InitData g_init;
bool g_standalone = true;
SharedMem* g_shm = nullptr;
int g_lock_fd = -1;

std::atomic<int> g_quit{0}, g_abort{0}, g_no_heartbeat{0}, g_suspended{0}, g_reread{0};
std::atomic<int> g_critical{0};
std::atomic<double> g_fraction{0.0};
std::atomic<int> g_pass{0}, g_passes{1};
std::atomic<double> g_last_checkpoint{0.0};
std::atomic<double> g_checkpoint_cpu{0.0};
std::atomic<double> g_wss{0.0}, g_max_wss{0.0};
std::atomic<int> g_status_sent{0};

// supervise(): the child's end of the status pipe (-1: not supervised)
int g_report_fd = -1;
pid_t g_child = -1;

// the exit status to the supervising parent (async-signal-safe; once)
void report_status(int status) {
  const int fd = g_report_fd;
  if (fd < 0) return;
  g_report_fd = -1;
  const int32_t v = status;
  ssize_t w;
  do {
    w = ::write(fd, &v, sizeof(v));
  } while (w < 0 && errno == EINTR);
  (void)w;
}

// a signal sent to the parent's PID goes on to the child; one the terminal
// sent to the whole foreground process group (Ctrl-C: SI_KERNEL) reached the
// child already and is not doubled (the crash handler counts kill signals)
void forward_signal(int sig, siginfo_t* info, void*) {
  if (g_child > 0 && (info == nullptr || info->si_code != SI_KERNEL)) ::kill(g_child, sig);
}

std::mutex g_suspend_mu;
std::condition_variable g_suspend_cv;
std::thread g_timer;
std::atomic<bool> g_timer_stop{false};
std::thread::id g_timer_id;

std::string xml_tag(const std::string& doc, const char* tag) {
  const std::string open = std::string("<") + tag + ">";
  const std::string close = std::string("</") + tag + ">";
  const size_t a = doc.find(open);
  if (a == std::string::npos) return {};
  const size_t b = doc.find(close, a + open.size());
  if (b == std::string::npos) return {};
  return doc.substr(a + open.size(), b - a - open.size());
}

bool has_tag(const char* doc, const char* tag) { return std::strstr(doc, tag) != nullptr; }

double env_double(const char* name, double dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atof(v) : dflt;
}

void parse_init_data() {
  std::ifstream f("init_data.xml");
  if (!f) return;
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string doc = ss.str();
  g_init.valid = true;
  std::string v;
  if (!(v = xml_tag(doc, "userid")).empty()) g_init.userid = std::atoi(v.c_str());
  g_init.user_name = xml_tag(doc, "user_name");
  if (!(v = xml_tag(doc, "hostid")).empty()) g_init.hostid = std::atoi(v.c_str());
  g_init.host_cpid = xml_tag(doc, "host_cpid");
  g_init.wu_name = xml_tag(doc, "wu_name");
  if (!(v = xml_tag(doc, "slot")).empty()) g_init.slot = std::atoi(v.c_str());
  if (!(v = xml_tag(doc, "gpu_device_num")).empty()) g_init.gpu_device_num = std::atoi(v.c_str());
  if (!(v = xml_tag(doc, "checkpoint_period")).empty()) g_init.checkpoint_period = std::atof(v.c_str());
  if (!(v = xml_tag(doc, "fraction_done_start")).empty()) g_init.fraction_done_start = std::atof(v.c_str());
  if (!(v = xml_tag(doc, "fraction_done_end")).empty()) g_init.fraction_done_end = std::atof(v.c_str());
}

bool attach_shmem() {
  const int fd = ::open(kMmapFileName, O_RDWR);
  if (fd < 0) return false;
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < static_cast<off_t>(sizeof(SharedMem))) {
    ::close(fd);
    return false;
  }
  void* p = mmap(nullptr, sizeof(SharedMem), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) return false;
  g_shm = static_cast<SharedMem*>(p);
  return true;
}

// one instance per slot (libboinc's boinc_lockfile)
bool acquire_lockfile() {
  g_lock_fd = ::open(kLockFile, O_WRONLY | O_CREAT, 0644);
  if (g_lock_fd < 0) return false;
  const double wait = env_double("BRP_LOCK_WAIT", 35.0);
  const double t0 = dtime();
  for (;;) {
    struct flock fl;
    std::memset(&fl, 0, sizeof(fl));
    fl.l_type = F_WRLCK;
    fl.l_whence = SEEK_SET;
    if (fcntl(g_lock_fd, F_SETLK, &fl) == 0) return true;
    if (dtime() - t0 >= wait) return false;
    std::this_thread::sleep_for(std::chrono::milliseconds(250));
  }
}

double process_cpu_time() {
  struct rusage ru;
  if (getrusage(RUSAGE_SELF, &ru) != 0) return 0.0;
  return ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6 + ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6;
}

double reported_fraction() {
  const int passes = std::max(1, g_passes.load());
  const double f = (g_fraction.load() + g_pass.load()) / passes;
  return g_init.fraction_done_start + f * (g_init.fraction_done_end - g_init.fraction_done_start);
}

bool send_status(double fraction) {
  if (!g_shm) return false;
  char msg[kMsgChannelSize];
  std::snprintf(msg, sizeof(msg),
                "<current_cpu_time>%e</current_cpu_time>\n"
                "<checkpoint_cpu_time>%e</checkpoint_cpu_time>\n"
                "<fraction_done>%e</fraction_done>\n",
                process_cpu_time(), g_checkpoint_cpu.load(), fraction);
  if (!g_shm->app_status.send_msg(msg)) return false;
  g_status_sent.fetch_add(1);
  return true;
}

void wake_suspended() {
  std::lock_guard<std::mutex> lk(g_suspend_mu);
  g_suspend_cv.notify_all();
}

// leave now, from whichever thread noticed (libboinc exits from its timer
// thread; _exit keeps static destructors away from the running workers)
[[noreturn]] void exit_now(int status) {
  std::fflush(nullptr);
  if (g_lock_fd >= 0) ::close(g_lock_fd);
  report_status(status);
  _exit(status);
}

void handle_heartbeat(double now, double& last_heartbeat) {
  char buf[kMsgChannelSize];
  if (!g_shm->heartbeat.get_msg(buf)) return;
  if (has_tag(buf, "<heartbeat/>")) last_heartbeat = now;
  std::string doc(buf);
  std::string v;
  if (!(v = xml_tag(doc, "wss")).empty()) g_wss.store(std::atof(v.c_str()));
  if (!(v = xml_tag(doc, "max_wss")).empty()) g_max_wss.store(std::atof(v.c_str()));
  if (has_tag(buf, "<reread_app_info/>") || has_tag(buf, "<reread_init_data_file/>")) g_reread.store(1);
}

void handle_process_control() {
  char buf[kMsgChannelSize];
  if (!g_shm->process_control_request.get_msg(buf)) return;
  if (has_tag(buf, "<suspend/>")) {
    log_message(LOG_INFO, true, "Received suspend message from the client.\n");
    g_suspended.store(1);
  }
  if (has_tag(buf, "<resume/>")) {
    log_message(LOG_INFO, true, "Received resume message from the client.\n");
    g_suspended.store(0);
    wake_suspended();
  }
  if (has_tag(buf, "<abort/>")) {
    log_message(LOG_WARN, true, "Received abort message from the client - exiting.\n");
    g_abort.store(1);
    exit_now(kExitAbortedByClient);
  }
  if (has_tag(buf, "<quit/>")) {
    log_message(LOG_INFO, true, "Received quit message from the client.\n");
    g_quit.store(1);
    wake_suspended();
    // inside a critical section the template loop sees quit_request at the
    // next template boundary and leaves without a final checkpoint
    if (g_critical.load() == 0) exit_now(0);
  }
}

void timer_loop() {
  const double giveup = env_double("BRP_HEARTBEAT_GIVEUP", kHeartbeatGiveup);
  double last_heartbeat = dtime();
  double last_status = 0.0;
  while (!g_timer_stop.load()) {
    std::this_thread::sleep_for(std::chrono::duration<double>(kTimerPeriod));
    const double now = dtime();
    handle_heartbeat(now, last_heartbeat);
    handle_process_control();
    if (now - last_heartbeat > giveup && !g_no_heartbeat.load()) {
      log_message(LOG_WARN, true, "No heartbeat from the client for %.0f s - exiting.\n", now - last_heartbeat);
      g_no_heartbeat.store(1);
      wake_suspended();
      if (g_critical.load() == 0) exit_now(0);
    }
    if (now - last_status >= kStatusPeriod && send_status(reported_fraction())) last_status = now;
  }
}

void stop_timer() {
  if (!g_timer.joinable()) return;
  if (std::this_thread::get_id() == g_timer_id) return;
  g_timer_stop.store(true);
  g_timer.join();
}

void write_progress_file() {
  // standalone harnesses (cf. debian runall.sh) poll this text file
  const char* path = std::getenv("BRP_PROGRESS_FILE");
  if (!path) return;
  FILE* f = std::fopen(path, "w");
  if (!f) return;
  std::fprintf(f, "%.6f\n", reported_fraction());
  std::fclose(f);
}

void write_marker(const char* path, const char* text) {
  FILE* f = std::fopen(path, "w");
  if (!f) return;
  std::fputs(text, f);
  std::fclose(f);
}

}  // namespace

int init(int, char**) {
  parse_init_data();
  const char* cp = std::getenv("BRP_CHECKPOINT_PERIOD");
  if (cp) g_init.checkpoint_period = std::atof(cp);
  g_last_checkpoint.store(dtime());
  g_standalone = !(g_init.valid && attach_shmem());
  if (g_standalone) return 0;
  if (!acquire_lockfile()) {
    log_message(LOG_ERROR, true, "Can't acquire lockfile %s - another instance is running in this slot.\n", kLockFile);
    exit_now(0);
  }
  g_timer_stop.store(false);
  g_timer = std::thread(timer_loop);
  g_timer_id = g_timer.get_id();
  return 0;
}

void shutdown() {
  stop_timer();
  if (g_shm) munmap(g_shm, sizeof(SharedMem));
  g_shm = nullptr;
  if (g_lock_fd >= 0) ::close(g_lock_fd);
  g_lock_fd = -1;
  g_standalone = true;
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
  g_fraction.store(f);
  write_progress_file();
}
double get_fraction_done() { return reported_fraction(); }
void set_pass(int pass, int passes) {
  g_pass.store(pass);
  g_passes.store(std::max(1, passes));
}

bool time_to_checkpoint() {
  if (dtime() - g_last_checkpoint.load() < g_init.checkpoint_period) return false;
  begin_critical_section();
  return true;
}
void checkpoint_completed() {
  g_last_checkpoint.store(dtime());
  g_checkpoint_cpu.store(process_cpu_time());
  end_critical_section();
}
void begin_critical_section() { g_critical.fetch_add(1); }
void end_critical_section() { g_critical.fetch_sub(1); }

void suspend_point() {
  if (!g_suspended.load(std::memory_order_relaxed)) return;
  std::unique_lock<std::mutex> lk(g_suspend_mu);
  g_suspend_cv.wait(lk, [] { return !g_suspended.load() || g_quit.load() || g_abort.load() || g_no_heartbeat.load(); });
}

Status get_status() {
  Status s;
  s.quit_request = g_quit.load(std::memory_order_relaxed);
  s.abort_request = g_abort.load(std::memory_order_relaxed);
  s.no_heartbeat = g_no_heartbeat.load(std::memory_order_relaxed);
  s.suspended = g_suspended.load(std::memory_order_relaxed);
  s.reread_init_data_file = g_reread.load(std::memory_order_relaxed);
  s.working_set_size = g_wss.load(std::memory_order_relaxed);
  s.max_working_set_size = g_max_wss.load(std::memory_order_relaxed);
  return s;
}

void request_quit() {
  g_quit.store(1);
  wake_suspended();
}
void clear_quit() { g_quit.store(0); }
double worker_thread_cpu_time() { return process_cpu_time(); }
int status_messages_sent() { return g_status_sent.load(); }

double dtime() {
  using namespace std::chrono;
  return duration<double>(system_clock::now().time_since_epoch()).count();
}

// libboinc names the graphics segment after the slot the client runs the task
// in ("boinc_<app>_<slot>", graphics2_util.cpp), so two tasks on one host do
// not share it; standalone runs (no init_data.xml slot) use slot 0, which the
// reference's runall.sh polls (debian/extra/einstein_bench/runall.sh)
char* graphics_make_shmem(const char* app_name, int size) {
  const int slot = g_init.slot >= 0 ? g_init.slot : 0;
  const std::string path = std::string("boinc_") + app_name + "_" + std::to_string(slot);
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

bool fast_exit_enabled() {
  const char* e = std::getenv("BRP_FAST_EXIT");
  return !(e && std::strcmp(e, "0") == 0);
}

void finish(int status) {
  std::fprintf(stderr, "called boinc_finish(%d)\n", status);
  if (!g_standalone && g_shm) {
    // final status with fraction_done 1, once the client took the last one
    stop_timer();
    for (int k = 0; k < 20 && !send_status(1.0); ++k) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
  char text[32];
  std::snprintf(text, sizeof(text), "%d\n", status);
  write_marker(kFinishCalledFile, text);
  trace::phase("finish");
  std::fflush(nullptr);
  if (g_lock_fd >= 0) ::close(g_lock_fd);
  // results, checkpoint removal and the finish marker are on disk: leave
  // without the HIP runtime's and the C++ statics' teardown (the kernel driver
  // reclaims device memory at process exit); BRP_FAST_EXIT=0 keeps exit()
  if (fast_exit_enabled()) {
    report_status(status);
    std::string ms;
    if (fault_enabled("slow_exit", &ms)) std::this_thread::sleep_for(std::chrono::milliseconds(std::atol(ms.c_str())));
    ::_exit(status);
  }
  std::exit(status);
}

void quit_exit(int status) {
  stop_timer();
  exit_now(status);
}

void temporary_exit(int delay_s, const char* reason) {
  log_message(LOG_WARN, true, "Temporary exit (%d s): %s\n", delay_s, reason ? reason : "");
  stop_timer();
  std::string text = std::to_string(delay_s) + "\n";
  if (reason) text += std::string(reason) + "\n";
  write_marker(kTemporaryExitFile, text.c_str());
  exit_now(0);
}

void finish_from_signal(int status) {
  char text[16];
  int n = 0;
  unsigned v = status < 0 ? static_cast<unsigned>(-status) : static_cast<unsigned>(status);
  char rev[12];
  int r = 0;
  do {
    rev[r++] = static_cast<char>('0' + v % 10);
    v /= 10;
  } while (v && r < 11);
  if (status < 0) text[n++] = '-';
  while (r) text[n++] = rev[--r];
  text[n++] = '\n';
  const int fd = ::open(kFinishCalledFile, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd >= 0) {
    ssize_t w = ::write(fd, text, n);
    (void)w;
    ::close(fd);
  }
  report_status(status);
  _exit(status);
}

void supervise() {
#if defined(__SANITIZE_ADDRESS__) || defined(__SANITIZE_THREAD__)
  return;
#elif defined(__has_feature)
#if __has_feature(address_sanitizer) || __has_feature(thread_sanitizer)
  return;
#endif
#endif
  const char* e = std::getenv("BRP_SUPERVISE");
  if (e && std::strcmp(e, "0") == 0) return;
  int fds[2];
  if (::pipe2(fds, O_CLOEXEC) != 0) return;  // run unsupervised
  std::fflush(nullptr);
  const pid_t parent = ::getpid();
  const pid_t pid = ::fork();
  if (pid < 0) {
    ::close(fds[0]);
    ::close(fds[1]);
    return;
  }
  if (pid == 0) {
    ::close(fds[0]);
    g_report_fd = fds[1];
    // the client's SIGKILL of the parent takes the child (and its GPU work) with it
    ::prctl(PR_SET_PDEATHSIG, SIGKILL);
    if (::getppid() != parent) _exit(kExitAbortedByClient);
    return;
  }
  ::close(fds[1]);
  g_child = pid;
  struct sigaction sa{};
  sa.sa_sigaction = forward_signal;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESTART | SA_SIGINFO;
  for (int sig : {SIGTERM, SIGINT, SIGHUP, SIGQUIT, SIGUSR1, SIGUSR2, SIGCONT}) ::sigaction(sig, &sa, nullptr);
  int32_t v = 0;
  size_t got = 0;
  while (got < sizeof(v)) {
    const ssize_t r = ::read(fds[0], reinterpret_cast<char*>(&v) + got, sizeof(v) - got);
    if (r > 0) got += static_cast<size_t>(r);
    else if (r < 0 && errno == EINTR) continue;
    else break;  // EOF: the child left without reporting
  }
  if (got == sizeof(v)) _exit(v);  // results on disk; the child's teardown goes on without us
  int st = 0;
  while (::waitpid(pid, &st, 0) < 0 && errno == EINTR) {
  }
  if (WIFEXITED(st)) _exit(WEXITSTATUS(st));
  if (WIFSIGNALED(st)) {
    const int sig = WTERMSIG(st);
    struct sigaction dfl{};
    dfl.sa_handler = SIG_DFL;
    sigemptyset(&dfl.sa_mask);
    ::sigaction(sig, &dfl, nullptr);
    ::raise(sig);
    _exit(128 + sig);
  }
  _exit(1);
}

}  // namespace boinc
}  // namespace brp
