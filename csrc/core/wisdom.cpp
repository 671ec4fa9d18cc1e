#include "wisdom.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <fstream>
#include <sstream>

namespace brp {

namespace {

// value of "key": <number or "string"> inside one flat JSON object text
bool field(const std::string& obj, const std::string& key, std::string& out) {
  const std::string pat = "\"" + key + "\"";
  size_t p = obj.find(pat);
  if (p == std::string::npos) return false;
  p = obj.find(':', p + pat.size());
  if (p == std::string::npos) return false;
  ++p;
  while (p < obj.size() && (obj[p] == ' ' || obj[p] == '\t' || obj[p] == '\n' || obj[p] == '\r')) ++p;
  if (p >= obj.size()) return false;
  if (obj[p] == '"') {
    const size_t q = obj.find('"', p + 1);
    if (q == std::string::npos) return false;
    out = obj.substr(p + 1, q - p - 1);
    return true;
  }
  size_t q = p;
  while (q < obj.size() && obj[q] != ',' && obj[q] != '}' && obj[q] != '\n') ++q;
  out = obj.substr(p, q - p);
  while (!out.empty() && (out.back() == ' ' || out.back() == '\r' || out.back() == '\t')) out.pop_back();
  return !out.empty();
}

int int_field(const std::string& obj, const char* key) {
  std::string v;
  if (!field(obj, key, v)) return -1;
  char* end = nullptr;
  const long x = std::strtol(v.c_str(), &end, 10);
  return (end && *end == '\0') ? static_cast<int>(x) : -1;
}

std::string arch_base(const std::string& a) { return a.substr(0, a.find(':')); }

}  // namespace

std::string wisdom_path() {
  if (const char* e = std::getenv("BRP_WISDOM")) return e;
  Dl_info info;
  if (dladdr(reinterpret_cast<void*>(&wisdom_path), &info) == 0 || info.dli_fname == nullptr) return "";
  std::string p = info.dli_fname;         // .../bin/app or .../boinc_app_eah_brp_amd/_brp*.so
  size_t s = p.rfind('/');
  if (s == std::string::npos) return "";
  p = p.substr(0, s);                     // .../bin
  s = p.rfind('/');
  p = (s == std::string::npos) ? std::string(".") : p.substr(0, s);  // repository root
  return p + "/data/wisdom/mi355x.json";
}

PlanWisdom load_wisdom(const std::string& path, const std::string& arch, uint32_t M) {
  PlanWisdom w;
  if (path.empty()) return w;
  std::ifstream f(path);
  if (!f) return w;
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string doc = ss.str();
  // scan the flat entry objects {...} (no nesting inside an entry)
  size_t p = doc.find('[');
  while (p != std::string::npos) {
    const size_t a = doc.find('{', p);
    if (a == std::string::npos) break;
    const size_t b = doc.find('}', a);
    if (b == std::string::npos) break;
    const std::string obj = doc.substr(a, b - a + 1);
    std::string ea;
    if (field(obj, "arch", ea) && arch_base(ea) == arch_base(arch) && int_field(obj, "M") == static_cast<int>(M)) {
      w.found = true;
      w.persist_per_cu = int_field(obj, "persist_per_cu");
      w.batch = int_field(obj, "batch");
      w.pipelines = int_field(obj, "pipelines");
      return w;
    }
    p = b + 1;
  }
  return w;
}

}  // namespace brp
