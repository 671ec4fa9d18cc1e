// Minimal standalone implementation of the BOINC API subset the application
// uses (SURVEY.md 7.1 list; call sites erp_boinc_wrapper.cpp:147-573,
// erp_boinc_ipc.cpp:69-207, demod_binary.c:451-1605).
//
// Without a BOINC client ("standalone mode", boinc_is_standalone() in the
// reference) it behaves like libboinc_api does standalone: logical file names
// resolve to themselves (or follow a <soft_link>), checkpoints are allowed every
// checkpoint period, progress goes to a file, the graphics shared memory is an
// mmap'ed file "boinc_EinsteinRadio_0". init_data.xml in the working directory
// is parsed when present (user/host/gpu_device_num).
#pragma once

#include <string>

namespace brp {
namespace boinc {

struct Status {
  int no_heartbeat = 0;
  int suspended = 0;
  int quit_request = 0;
  int reread_init_data_file = 0;
  int abort_request = 0;
  double working_set_size = 0;
  double max_working_set_size = 0;
};

struct InitData {
  bool valid = false;
  int userid = 0;
  std::string user_name;
  int hostid = 0;
  std::string host_cpid;
  int gpu_device_num = -1;
  double checkpoint_period = 60.0;
};

int init(int argc, char** argv);
bool is_standalone();
const InitData& init_data();
int resolve_filename(const std::string& logical, std::string& physical);
void fraction_done(double f);
double get_fraction_done();
bool time_to_checkpoint();
void checkpoint_completed();
void begin_critical_section();
void end_critical_section();
Status get_status();
// request a clean stop (signal handler / tests)
void request_quit();
void clear_quit();
double worker_thread_cpu_time();
double dtime();
// graphics shared memory (mmap'ed file); returns nullptr on failure
char* graphics_make_shmem(const char* app_name, int size);
[[noreturn]] void finish(int status);
[[noreturn]] void temporary_exit(int delay_s, const char* reason);

}  // namespace boinc
}  // namespace brp
