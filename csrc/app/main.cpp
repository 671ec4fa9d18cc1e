// Process entry of the BOINC application (reference erp_boinc_wrapper.cpp:487-584):
// signal handling and crash reports (csrc/boinc/crash.hpp), BOINC runtime
// init (client shared memory, heartbeat, process control; csrc/boinc/runtime.hpp),
// worker, and the mapping of transient resource errors to a BOINC temporary exit.
#include "../boinc/crash.hpp"
#include "../boinc/runtime.hpp"
#include "../core/errors.hpp"
#include "../core/log.hpp"
#include "../core/trace.hpp"
#include "search.hpp"

int main(int argc, char** argv) {
  // first: the parent (the PID the client waits for) leaves as soon as the
  // child's results are on disk, not after the GPU context's teardown
  brp::boinc::supervise();
  brp::trace::phase("main");
  brp::log_message(brp::LOG_INFO, true, "Application startup - thank you for supporting Einstein@Home!\n");
  brp::log_message(brp::LOG_DEBUG, true, "Setting up diagnotics and exception handling...\n");
  brp::crash::install();
  brp::trace::phase("crash handlers");
  brp::log_message(brp::LOG_DEBUG, true, "Initializing BOINC...\n");
  brp::boinc::init(argc, argv);
  brp::trace::phase("boinc runtime init");
  brp::log_message(brp::LOG_DEBUG, true, "Calling worker, let's get started...\n");
  const int result = brp::wrapper_main(argc, argv);
  if (brp::is_transient_resource_error(result)) {
    brp::log_message(brp::LOG_WARN, true,
                     "Sorry, at the moment your system doesn't have enough free CPU/GPU memory to run this task!\n");
    brp::log_message(brp::LOG_WARN, false, "Returning control to BOINC, delaying next attempt for at least 15 minutes...\n");
    brp::boinc::temporary_exit(900, "Not enough free CPU/GPU memory available! Delaying next attempt for at least 15 minutes...");
  }
  brp::trace::phase("worker returned");
  brp::log_message(brp::LOG_DEBUG, true, "Shutting down BOINC... Bye!\n");
  brp::boinc::finish(result);
}
