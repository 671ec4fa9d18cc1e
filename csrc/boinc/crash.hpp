// Signal handling and crash reports of the application (reference
// erp_boinc_wrapper.cpp:123-192 with the libbfd symbolisation of
// erp_execinfo_plus.c:212-316).
//
// install() does everything that allocates or takes locks up front: it reads
// the function symbols of the executable (.symtab, demangled) and the list of
// loaded modules into static tables, loads the unwinder, and duplicates
// stderr. The handlers then only use write(2), backtrace(), table lookups,
// sleep(3) and _exit(2):
//   * SIGTERM / SIGINT are ignored three times; the 4th finishes the task
//     (a BOINC user pressing Ctrl-C must not kill the app; the client sends
//     <quit/> instead);
//   * SIGSEGV / SIGBUS / SIGILL / SIGFPE / SIGABRT print
//     "#k 0xADDR in function+0xOFF" for frames of the executable and
//     "module+0xOFF" for shared libraries, sleep ($BRP_CRASH_SLEEP, default
//     5 s as the reference) so other threads can report too, then finish with
//     the signal number as exit status (boinc_finish(sig)).
#pragma once

namespace brp {
namespace crash {

void install();
// symbolise one code address with the tables of install() (tests / debugging)
bool describe(const void* addr, char* out, int out_size);

}  // namespace crash
}  // namespace brp
