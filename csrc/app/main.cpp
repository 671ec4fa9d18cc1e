// Process entry of the BOINC application (reference erp_boinc_wrapper.cpp:487-584):
// diagnostics, signal handling (SIGTERM/SIGINT ignored three times, the 4th
// exits; fatal signals print a backtrace), BOINC init, worker, and the mapping
// of transient resource errors to a BOINC temporary exit.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../boinc/boinc_shim.hpp"
#include "../core/errors.hpp"
#include "../core/log.hpp"
#include "search.hpp"

namespace {

void sighandler(int sig, siginfo_t*, void*) {
  static int killcounter = 0;
  brp::log_message(brp::LOG_ERROR, true, "\nApplication caught signal %d.\n", sig);
  if (sig == SIGTERM || sig == SIGINT) {
    ++killcounter;
    if (killcounter >= 4) {
      brp::log_message(brp::LOG_WARN, true, "Got 4th kill-signal, guess you mean it. Exiting now!\n\n");
      brp::boinc::finish(brp::EINSTEINRADIO_EXIT);
    }
    // ask the search loop to stop at the next template boundary
    brp::boinc::request_quit();
    return;
  }
  void* frames[64];
  const int n = backtrace(frames, 64);
  brp::log_message(brp::LOG_ERROR, false, "\nObtained %d stack frames for this thread.\n", n);
  brp::log_message(brp::LOG_ERROR, false, "Backtrace:\n");
  backtrace_symbols_fd(frames, n, fileno(stderr));
  brp::log_message(brp::LOG_ERROR, false, "End of backtrace\n\n");
  std::_Exit(sig);
}

}  // namespace

int main(int argc, char** argv) {
  brp::log_message(brp::LOG_INFO, true, "Application startup - thank you for supporting Einstein@Home!\n");
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = sighandler;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESTART | SA_SIGINFO;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGSEGV, &sa, nullptr);
  sigaction(SIGFPE, &sa, nullptr);
  sigaction(SIGILL, &sa, nullptr);
  sigaction(SIGBUS, &sa, nullptr);
  sigaction(SIGABRT, &sa, nullptr);
  brp::boinc::init(argc, argv);
  const int result = brp::wrapper_main(argc, argv);
  if (brp::is_transient_resource_error(result)) {
    brp::log_message(brp::LOG_WARN, true,
                     "Sorry, at the moment your system doesn't have enough free CPU/GPU memory to run this task!\n");
    brp::boinc::temporary_exit(900, "Not enough free CPU/GPU memory available! Delaying next attempt for at least 15 minutes...");
  }
  brp::boinc::finish(result);
}
