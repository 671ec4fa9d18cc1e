// App-side BOINC runtime: the subset of libboinc_api the reference uses
// (SURVEY.md 7.1 list; call sites erp_boinc_wrapper.cpp:147-573,
// erp_boinc_ipc.cpp:69-207, demod_binary.c:451-1605), written for this app.
//
// Client mode (init_data.xml and boinc_mmap_file in the working directory,
// i.e. a BOINC slot): the slot lock file is held, a timer thread services the
// shared-memory channels (client_shm.hpp) every 0.1 s:
//   * <heartbeat/> resets the give-up clock; 30 s without one sets
//     no_heartbeat and the app leaves (exit 0, as after a quit);
//   * <suspend/> / <resume/>: suspend_point() blocks the calling thread while
//     suspended. Pipelines call it before every batch and the in-order applier
//     at every template boundary, so no GPU work starts while suspended;
//     batches already inside a critical section run to completion;
//   * <quit/>: outside a critical section the timer thread exits the process
//     at once (status 0, no boinc_finish_called marker); inside one, the
//     quit_request status ends the template loop at the next template and the
//     app exits without a final checkpoint (demod_binary.c:1436-1441, 1489-1492);
//   * <abort/>: exit 194 (EXIT_ABORTED_BY_CLIENT) at once;
//   * once a second the app status (current/checkpoint CPU time,
//     fraction_done scaled by the pass and the client's fraction range) is
//     posted when the client consumed the previous message.
// finish() / temporary_exit() write the boinc_finish_called /
// boinc_temporary_exit marker files before exiting; boinc_time_to_checkpoint
// enters a critical section that boinc_checkpoint_completed leaves.
//
// Standalone mode (no init_data.xml or no mmap file, boinc_is_standalone() in
// the reference): logical names resolve to themselves (or follow a
// <soft_link>), checkpoints are allowed every checkpoint period, progress goes
// to $BRP_PROGRESS_FILE when set, and nothing waits on a client.
//
// get_status() / suspend_point() / fraction_done() only touch atomics (no
// system calls), so the per-template hook of an 8-GPU process stays cheap.
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
  std::string wu_name;
  int slot = -1;
  int gpu_device_num = -1;
  double checkpoint_period = 60.0;
  double fraction_done_start = 0.0;
  double fraction_done_end = 1.0;
};

int init(int argc, char** argv);
// stop the timer thread and detach (tests and the Python bindings)
void shutdown();
bool is_standalone();
const InitData& init_data();
int resolve_filename(const std::string& logical, std::string& physical);

// fraction of the current pass; reported as (f + pass) / passes
// (erp_fraction_done, erp_boinc_wrapper.cpp:200-202)
void fraction_done(double f);
double get_fraction_done();
void set_pass(int pass, int passes);

// true when a checkpoint is due; enters a critical section that
// checkpoint_completed() leaves
bool time_to_checkpoint();
void checkpoint_completed();
void begin_critical_section();
void end_critical_section();
// block while the client has the task suspended (no-op otherwise)
void suspend_point();
Status get_status();

// request a clean stop (fault injection, tests)
void request_quit();
void clear_quit();
double worker_thread_cpu_time();
double dtime();
// graphics shared memory (mmap'ed file); returns nullptr on failure
char* graphics_make_shmem(const char* app_name, int size);
// status sent to the client so far (tests)
int status_messages_sent();

[[noreturn]] void finish(int status);
// finish() leaves with _exit() after flushing (default; BRP_FAST_EXIT=0: exit())
bool fast_exit_enabled();
// quit / abort / lost heartbeat: leave without the finish marker
[[noreturn]] void quit_exit(int status);
[[noreturn]] void temporary_exit(int delay_s, const char* reason);
// async-signal-safe finish for fatal signal handlers (open/write/_exit only)
[[noreturn]] void finish_from_signal(int status);

// Process supervision (the app binary's first call, before any thread or HIP
// call): the process forks; the child returns and runs the application, the
// parent -- the PID the BOINC client and /usr/bin/time wait for -- waits for
// it and never touches the GPU. Every exit path of the child reports its
// status once the results and markers are on disk (finish, quit, temporary
// exit, fatal signals), and the parent leaves with that status at once: the
// kernel driver's teardown of the child's GPU context (80-120 ms on MI355X,
// profiles/app_phases_r6.txt) no longer delays the client. A child that dies
// without reporting is waited for and its status or signal mirrored.
// Termination signals sent to the parent are forwarded to the child, and the
// child is killed if the parent dies (SIGKILL from the client). Off with
// BRP_SUPERVISE=0 and in sanitizer builds.
void supervise();

}  // namespace boinc
}  // namespace brp
