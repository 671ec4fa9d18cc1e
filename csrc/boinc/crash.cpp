#include "crash.hpp"

#include <cxxabi.h>
#include <elf.h>
#include <execinfo.h>
#include <fcntl.h>
#include <link.h>
#include <signal.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../core/errors.hpp"
#include "runtime.hpp"

namespace brp {
namespace crash {

namespace {

struct Sym {
  uintptr_t lo, hi;  // link-time addresses [lo, hi)
  uint32_t name;     // offset into g_names
};

struct Module {
  uintptr_t lo, hi;  // run-time extent of the PT_LOAD segments
  uintptr_t base;    // load bias
  char name[128];
};

// The executable's function symbols, read and demangled on a thread started
// by install() (16-20 ms for this binary, which would otherwise delay the HIP
// runtime start behind it) and published whole: a crash before then prints
// module offsets only. Never freed (the loader may still run at exit).
struct SymTable {
  std::vector<Sym> syms;
  std::string names;
};
std::atomic<const SymTable*> g_tab{nullptr};
uintptr_t g_exe_bias = 0;
uintptr_t g_exe_lo = 0, g_exe_hi = 0;
constexpr int kMaxModules = 128;
Module g_mods[kMaxModules];
int g_nmods = 0;
int g_fd = 2;
unsigned g_sleep_s = 5;
volatile sig_atomic_t g_kills = 0;

// ---- async-signal-safe output ------------------------------------------------
void put(const char* s) {
  size_t n = std::strlen(s);
  while (n) {
    const ssize_t w = ::write(g_fd, s, n);
    if (w <= 0) return;
    s += w;
    n -= static_cast<size_t>(w);
  }
}
void put_dec(long v) {
  char b[24];
  int i = 23;
  b[i] = 0;
  const bool neg = v < 0;
  unsigned long u = neg ? static_cast<unsigned long>(-v) : static_cast<unsigned long>(v);
  do {
    b[--i] = static_cast<char>('0' + u % 10);
    u /= 10;
  } while (u);
  if (neg) b[--i] = '-';
  put(b + i);
}
void put_hex(uintptr_t v) {
  char b[24];
  int i = 23;
  b[i] = 0;
  do {
    b[--i] = "0123456789abcdef"[v & 15];
    v >>= 4;
  } while (v);
  b[--i] = 'x';
  b[--i] = '0';
  put(b + i);
}

// ---- symbol tables (install time) --------------------------------------------
int collect_module(struct dl_phdr_info* info, size_t, void*) {
  uintptr_t lo = UINTPTR_MAX, hi = 0;
  for (int k = 0; k < info->dlpi_phnum; ++k) {
    const ElfW(Phdr)& ph = info->dlpi_phdr[k];
    if (ph.p_type != PT_LOAD) continue;
    lo = std::min<uintptr_t>(lo, info->dlpi_addr + ph.p_vaddr);
    hi = std::max<uintptr_t>(hi, info->dlpi_addr + ph.p_vaddr + ph.p_memsz);
  }
  const bool is_exe = g_nmods == 0;  // the first entry is the executable
  if (is_exe) {
    g_exe_bias = info->dlpi_addr;
    g_exe_lo = lo;
    g_exe_hi = hi;
  }
  if (g_nmods < kMaxModules && lo < hi) {
    Module& m = g_mods[g_nmods++];
    m.lo = lo;
    m.hi = hi;
    m.base = info->dlpi_addr;
    const char* nm = (info->dlpi_name && *info->dlpi_name) ? info->dlpi_name : "executable";
    const char* slash = std::strrchr(nm, '/');
    std::snprintf(m.name, sizeof(m.name), "%s", slash ? slash + 1 : nm);
  } else if (is_exe) {
    ++g_nmods;
  }
  return 0;
}

void load_symbols() {
  auto* tab = new SymTable;
  std::vector<Sym>& g_syms = tab->syms;
  std::string& g_names = tab->names;
  struct Publish {
    SymTable* t;
    ~Publish() { g_tab.store(t, std::memory_order_release); }  // an empty table too
  } publish{tab};
  FILE* f = std::fopen("/proc/self/exe", "rb");
  if (!f) return;
  std::vector<char> img;
  char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) img.insert(img.end(), buf, buf + n);
  std::fclose(f);
  if (img.size() < sizeof(ElfW(Ehdr))) return;
  const auto* eh = reinterpret_cast<const ElfW(Ehdr)*>(img.data());
  if (std::memcmp(eh->e_ident, ELFMAG, SELFMAG) != 0 || eh->e_shoff == 0) return;
  if (eh->e_shoff + static_cast<size_t>(eh->e_shnum) * sizeof(ElfW(Shdr)) > img.size()) return;
  const auto* sh = reinterpret_cast<const ElfW(Shdr)*>(img.data() + eh->e_shoff);
  // prefer the full .symtab; an unstripped build has it, .dynsym is the fallback
  int symsec = -1;
  for (int k = 0; k < eh->e_shnum; ++k)
    if (sh[k].sh_type == SHT_SYMTAB) symsec = k;
  if (symsec < 0)
    for (int k = 0; k < eh->e_shnum; ++k)
      if (sh[k].sh_type == SHT_DYNSYM) symsec = k;
  if (symsec < 0) return;
  const ElfW(Shdr)& ss = sh[symsec];
  const ElfW(Shdr)& st = sh[ss.sh_link];
  if (ss.sh_offset + ss.sh_size > img.size() || st.sh_offset + st.sh_size > img.size()) return;
  const auto* syms = reinterpret_cast<const ElfW(Sym)*>(img.data() + ss.sh_offset);
  const size_t count = ss.sh_size / sizeof(ElfW(Sym));
  const char* strtab = img.data() + st.sh_offset;
  for (size_t k = 0; k < count; ++k) {
    const ElfW(Sym)& s = syms[k];
    if (ELF64_ST_TYPE(s.st_info) != STT_FUNC || s.st_value == 0 || s.st_size == 0) continue;
    if (s.st_name >= st.sh_size) continue;
    const char* raw = strtab + s.st_name;
    int status = -1;
    char* dem = abi::__cxa_demangle(raw, nullptr, nullptr, &status);
    Sym e{static_cast<uintptr_t>(s.st_value), static_cast<uintptr_t>(s.st_value + s.st_size),
          static_cast<uint32_t>(g_names.size())};
    g_names += (status == 0 && dem) ? dem : raw;
    g_names.push_back('\0');
    std::free(dem);
    g_syms.push_back(e);
  }
  std::sort(g_syms.begin(), g_syms.end(), [](const Sym& a, const Sym& b) { return a.lo < b.lo; });
}

// lookup without allocation: binary search over the sorted table
const Sym* find_sym(const SymTable* tab, uintptr_t link_addr) {
  if (tab == nullptr) return nullptr;
  const std::vector<Sym>& g_syms = tab->syms;
  size_t lo = 0, hi = g_syms.size();
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (g_syms[mid].lo <= link_addr) lo = mid + 1;
    else hi = mid;
  }
  if (lo == 0) return nullptr;
  const Sym& s = g_syms[lo - 1];
  return link_addr < s.hi ? &s : nullptr;
}

void put_frame(int k, void* pc) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(pc);
  put("#");
  put_dec(k);
  put(" ");
  put_hex(a);
  const SymTable* tab = g_tab.load(std::memory_order_acquire);
  if (a >= g_exe_lo && a < g_exe_hi) {
    if (const Sym* s = find_sym(tab, a - g_exe_bias)) {
      put(" in ");
      put(tab->names.c_str() + s->name);
      put("+");
      put_hex(a - g_exe_bias - s->lo);
      put("\n");
      return;
    }
  }
  for (int m = 0; m < g_nmods && m < kMaxModules; ++m) {
    if (a >= g_mods[m].lo && a < g_mods[m].hi) {
      put(" in ");
      put(g_mods[m].name);
      put("+");
      put_hex(a - g_mods[m].base);
      put("\n");
      return;
    }
  }
  put(" in ??\n");
}

void handler(int sig, siginfo_t*, void*) {
  put("\n[");
  put_dec(static_cast<long>(getpid()));
  put("][ERROR] Application caught signal ");
  put_dec(sig);
  put(".\n");
  if (sig == SIGTERM || sig == SIGINT) {
    g_kills = g_kills + 1;
    if (g_kills >= 4) {
      put("Got 4th kill-signal, guess you mean it. Exiting now!\n\n");
      boinc::finish_from_signal(EINSTEINRADIO_EXIT);
    }
    return;
  }
  // a crash while the symbol loader still runs waits for it (up to 2 s;
  // nanosleep is async-signal-safe, the loader is another thread)
  for (int w = 0; w < 200 && g_tab.load(std::memory_order_acquire) == nullptr; ++w) {
    const struct timespec ts{0, 10 * 1000 * 1000};
    nanosleep(&ts, nullptr);
  }
  void* frames[64];
  const int n = backtrace(frames, 64);
  put("\nObtained ");
  put_dec(n);
  put(" stack frames for this thread.\nBacktrace:\n");
  for (int k = 0; k < n; ++k) put_frame(k, frames[k]);
  put("End of backtrace\n\n");
  // let the other threads catch the signal too (erp_boinc_wrapper.cpp:188-190)
  if (g_sleep_s) sleep(g_sleep_s);
  boinc::finish_from_signal(sig);
}

}  // namespace

void install() {
  void* warm[2];
  backtrace(warm, 2);  // loads the unwinder now, not inside the handler
  g_nmods = 0;
  dl_iterate_phdr(collect_module, nullptr);
  std::thread(load_symbols).detach();
  const int fd = dup(2);
  if (fd >= 0) g_fd = fd;
  if (const char* s = std::getenv("BRP_CRASH_SLEEP")) g_sleep_s = static_cast<unsigned>(std::atoi(s));
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = handler;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESTART | SA_SIGINFO;
  for (int sig : {SIGTERM, SIGINT, SIGSEGV, SIGFPE, SIGILL, SIGBUS, SIGABRT}) sigaction(sig, &sa, nullptr);
}

bool describe(const void* addr, char* out, int out_size) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(addr);
  const SymTable* tab = g_tab.load(std::memory_order_acquire);
  if (a >= g_exe_lo && a < g_exe_hi) {
    if (const Sym* s = find_sym(tab, a - g_exe_bias)) {
      std::snprintf(out, out_size, "%s", tab->names.c_str() + s->name);
      return true;
    }
  }
  return false;
}

}  // namespace crash
}  // namespace brp
