#include "io.hpp"

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <zlib.h>

#include "errors.hpp"
#include "log.hpp"
#include "stats.hpp"

namespace brp {

int work_unit_format(const std::string& path, bool& four_bit) {
  if (path.find(".binary") != std::string::npos) {
    four_bit = false;
    return 0;
  }
  if (path.find(".bin4") != std::string::npos) {
    four_bit = true;
    return 0;
  }
  log_message(LOG_ERROR, true, "Unknown file format (extension) for input file: %s\n", path.c_str());
  return RADPUL_EFILE;
}

int read_work_unit(const std::string& path, WorkUnit& wu) {
  int rc = work_unit_format(path, wu.four_bit);
  if (rc) return rc;
  gzFile in = gzopen(path.c_str(), "rb");
  if (!in) {
    log_message(LOG_ERROR, true, "Couldn't open input file: %s (%s)\n", path.c_str(), std::strerror(errno));
    return RADPUL_EIO;
  }
  if (gzread(in, &wu.header, sizeof(DDHeader)) != static_cast<int>(sizeof(DDHeader))) {
    log_message(LOG_ERROR, true, "Premature end of data in file: %s\n", path.c_str());
    gzclose(in);
    return RADPUL_EIO;
  }
  if (host_is_big_endian()) swap_header(wu.header);
  const uint32_t n = wu.header.nsamples;
  const uint32_t n_packed = wu.four_bit ? static_cast<uint32_t>(n * 0.5) : n;
  std::vector<uint8_t> packed(n_packed);
  if (n_packed && gzread(in, packed.data(), n_packed) != static_cast<int>(n_packed)) {
    log_message(LOG_ERROR, true, "Premature end of data in file: %s\n", path.c_str());
    gzclose(in);
    return RADPUL_EIO;
  }
  if (gzclose(in) != Z_OK) {
    log_message(LOG_ERROR, true, "Couldn't close input file: %s\n", path.c_str());
    return RADPUL_EIO;
  }
  const double scale = wu.header.scale;
  wu.samples.assign(n, 0.0f);
  wu.packed = packed;
  if (wu.four_bit) {
    for (uint32_t i = 0; i < n_packed; ++i) {
      const uint8_t c = packed[i];
      wu.samples[2 * i + 1] = static_cast<float>(static_cast<float>(c % 16) / scale);
      wu.samples[2 * i] = static_cast<float>(static_cast<float>(c >> 4) / scale);
    }
  } else {
    for (uint32_t i = 0; i < n_packed; ++i) {
      wu.samples[i] = static_cast<float>(static_cast<int8_t>(packed[i]) / scale);
    }
  }
  return 0;
}

int write_work_unit(const std::string& path, const DDHeader& header,
                    const std::vector<uint8_t>& payload, bool gzip) {
  DDHeader h = header;
  if (host_is_big_endian()) swap_header(h);
  if (gzip) {
    gzFile out = gzopen(path.c_str(), "wb");
    if (!out) return RADPUL_EIO;
    bool ok = gzwrite(out, &h, sizeof(h)) == static_cast<int>(sizeof(h));
    if (!payload.empty())
      ok = ok && gzwrite(out, payload.data(), payload.size()) == static_cast<int>(payload.size());
    ok = (gzclose(out) == Z_OK) && ok;
    return ok ? 0 : RADPUL_EIO;
  }
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return RADPUL_EIO;
  bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1;
  if (!payload.empty()) ok = ok && std::fwrite(payload.data(), 1, payload.size(), f) == payload.size();
  ok = (std::fclose(f) == 0) && ok;
  return ok ? 0 : RADPUL_EIO;
}

namespace {
// fgets-based line iteration with the reference's `fgets(...) && !feof(...)`
// condition: a final line without newline is not delivered.
template <typename Fn>
int for_each_line(FILE* f, Fn&& fn) {
  char line[kFnLength];
  for (;;) {
    if (!std::ferror(f) && std::fgets(line, kFnLength, f) != nullptr && !std::feof(f)) {
      int rc = fn(line);
      if (rc) return rc;
    } else if (std::feof(f)) {
      return 0;
    } else {
      return -1;
    }
  }
}
}  // namespace

int read_template_bank(const std::string& path, TemplateBank& bank) {
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) {
    log_message(LOG_ERROR, true, "Couldn't open template bank file: %s (%s).\n", path.c_str(),
                std::strerror(errno));
    return RADPUL_EIO;
  }
  bank.P.clear();
  bank.tau.clear();
  bank.Psi0.clear();
  int rc = for_each_line(f, [&](const char* line) {
    double P, tau, psi;
    if (std::sscanf(line, "%lg %lg %lg\n", &P, &tau, &psi) != 3) {
      log_message(LOG_ERROR, true, "Line %zu in templatebank %s seems to be damaged.\n",
                  bank.P.size() + 1, path.c_str());
      return static_cast<int>(RADPUL_EVAL);
    }
    bank.P.push_back(P);
    bank.tau.push_back(tau);
    bank.Psi0.push_back(psi);
    return 0;
  });
  std::fclose(f);
  if (rc < 0) {
    log_message(LOG_ERROR, true, "Couldn't determine number of templates in %s.\n", path.c_str());
    return RADPUL_EIO;
  }
  return rc;
}

int read_zaplist(const std::string& path, std::vector<ZapRange>& ranges) {
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) {
    log_message(LOG_ERROR, true, "Couldn't open zaplist file: %s (%s)\n", path.c_str(), std::strerror(errno));
    return RADPUL_EFILE;
  }
  ranges.clear();
  int line_no = 0;
  int rc = for_each_line(f, [&](const char* line) {
    ++line_no;
    ZapRange r;
    if (std::sscanf(line, "%lg %lg", &r.fmin, &r.fmax) != 2) {
      log_message(LOG_ERROR, true, "Couldn't read complete line no. %d from zaplist file %s.\n", line_no,
                  path.c_str());
      return static_cast<int>(RADPUL_EIO);
    }
    ranges.push_back(r);
    return 0;
  });
  std::fclose(f);
  return rc < 0 ? RADPUL_EIO : rc;
}

int read_checkpoint(const std::string& path, Checkpoint& cp, bool& exists) {
  FILE* f = std::fopen(path.c_str(), "rb");
  exists = (f != nullptr);
  if (!f) return 0;
  if (std::fread(&cp.header, sizeof(CPHeader), 1, f) != 1) {
    log_message(LOG_ERROR, true, "Premature end of data header in file: %s\n", path.c_str());
    std::fclose(f);
    return RADPUL_EFILE;
  }
  if (std::fread(cp.cands, sizeof(CPCand), kCandTotal, f) != static_cast<size_t>(kCandTotal)) {
    log_message(LOG_ERROR, true, "Couldn't read all candidates from checkpoint!\n");
    std::fclose(f);
    return RADPUL_EIO;
  }
  if (std::fclose(f)) return RADPUL_EIO;
  if (host_is_big_endian()) {
    endian_swap(reinterpret_cast<uint8_t*>(&cp.header.n_template), 4, 1);
    for (auto& c : cp.cands) {
      endian_swap(reinterpret_cast<uint8_t*>(&c.power), 8, 5);
      endian_swap(reinterpret_cast<uint8_t*>(&c.n_harm), 4, 2);
    }
  }
  return 0;
}

int write_checkpoint(const std::string& path, const Checkpoint& cp) {
  const std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) {
    log_message(LOG_ERROR, true, "Couldn't open temporary checkpoint file: %s (%s).\n", tmp.c_str(),
                std::strerror(errno));
    return RADPUL_EIO;
  }
  Checkpoint out = cp;
  if (host_is_big_endian()) {
    endian_swap(reinterpret_cast<uint8_t*>(&out.header.n_template), 4, 1);
    for (auto& c : out.cands) {
      endian_swap(reinterpret_cast<uint8_t*>(&c.power), 8, 5);
      endian_swap(reinterpret_cast<uint8_t*>(&c.n_harm), 4, 2);
    }
  }
  bool ok = std::fwrite(&out.header, sizeof(CPHeader), 1, f) == 1 &&
            std::fwrite(out.cands, sizeof(CPCand), kCandTotal, f) == static_cast<size_t>(kCandTotal);
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) {
    log_message(LOG_ERROR, true, "Couldn't write temporary checkpoint file: %s\n", tmp.c_str());
    return RADPUL_EIO;
  }
  if (std::rename(tmp.c_str(), path.c_str())) {
    log_message(LOG_ERROR, true, "Couldn't rename temporary checkpoint file (%s) to %s (%s).\n", tmp.c_str(),
                path.c_str(), std::strerror(errno));
    return RADPUL_EFILE;
  }
  return 0;
}

namespace {
// compare_structs_by_ifa (demod_binary.c:1713-1740): fA desc, power desc, f0 desc
bool by_ifa(const CPCand& a, const CPCand& b) {
  if (a.fA != b.fA) return a.fA > b.fA;
  if (a.power != b.power) return a.power > b.power;
  return a.f0 > b.f0;
}
}  // namespace

int write_results(const std::string& path, CPCand* cands, double t_obs, const ResultHeaderInfo& info) {
  // significance and normalisation to units of sigma_N = sqrt(N_h)
  for (int i = 0; i < kCandTotal; ++i) {
    CPCand& c = cands[i];
    float sigma;
    switch (c.n_harm) {
      case 1: sigma = 1.0f; break;
      case 2: sigma = static_cast<float>(std::sqrt(2.0)); break;
      case 4: sigma = 2.0f; break;
      case 8: sigma = static_cast<float>(std::sqrt(8.0)); break;
      case 16: sigma = 4.0f; break;
      default: sigma = 0.0f; break;
    }
    if (sigma > 0.0f) {
      c.fA = candidate_significance(c.power, c.n_harm);
      c.power /= sigma;
    } else {
      c.fA = -10.0;
    }
  }
  std::stable_sort(cands, cands + kCandTotal, by_ifa);

  const std::string tmp = path + ".tmp";
  FILE* out = std::fopen(tmp.c_str(), "w");
  if (!out) {
    log_message(LOG_ERROR, true, "Couldn't open temporary output file: %s (%s)\n", tmp.c_str(),
                std::strerror(errno));
    return RADPUL_EIO;
  }
  if (info.write_header) {
    std::fprintf(out, "%% User: %i (%s)\n%% Host: %i (%s)\n%% Date: %s\n%% Exec: %s\n%% ERP git id: %s\n%% BOINC rev.: %s\n\n",
                 info.user_id, info.user_name.empty() ? "unknown" : info.user_name.c_str(), info.host_id,
                 info.host_cpid.empty() ? "unknown" : info.host_cpid.c_str(), [] {
                   static char buf[32];
                   std::time_t t = std::time(nullptr);
                   std::tm tm_utc;
                   gmtime_r(&t, &tm_utc);
                   std::strftime(buf, sizeof(buf), "%Y-%m-%dT%H:%M:%S+00:00", &tm_utc);
                   return static_cast<const char*>(buf);
                 }(),
                 info.exec_name.empty() ? "unknown" : info.exec_name.c_str(),
                 info.git_id.empty() ? "unknown" : info.git_id.c_str(),
                 info.boinc_rev.empty() ? "unknown" : info.boinc_rev.c_str());
  }
  const double res_factor = 1.0 / t_obs;
  int counter = 0;
  while (counter < kCandPerLevel && cands[0].fA > 0.0) {
    if (std::fprintf(out, "%6.12f %6.12f %6.12f %6.12f %g %g %d\n", cands[0].f0 * res_factor, cands[0].P_b,
                     cands[0].tau, cands[0].Psi, cands[0].power, cands[0].fA, cands[0].n_harm) < 0) {
      std::fclose(out);
      return RADPUL_EIO;
    }
    ++counter;
    const uint32_t f0 = cands[0].f0;
    for (int j = 0; j < kCandTotal; ++j)
      if (cands[j].f0 == f0) cands[j].fA = -10.0;
    std::stable_sort(cands, cands + kCandTotal, by_ifa);
  }
  if (std::fprintf(out, "%%DONE%%\n") < 7) {
    std::fclose(out);
    return RADPUL_EIO;
  }
  if (std::fclose(out)) return RADPUL_EIO;
  if (std::rename(tmp.c_str(), path.c_str())) {
    log_message(LOG_ERROR, true, "Couldn't rename temporary output file (%s) to final output file: %s (%s)\n",
                tmp.c_str(), path.c_str(), std::strerror(errno));
    return RADPUL_EFILE;
  }
  return 0;
}

int read_results(const std::string& path, std::vector<ResultLine>& lines, bool& done_marker) {
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) return RADPUL_EIO;
  lines.clear();
  done_marker = false;
  char buf[1024];
  while (std::fgets(buf, sizeof(buf), f)) {
    if (buf[0] == '%') {
      if (std::strncmp(buf, "%DONE%", 6) == 0) done_marker = true;
      continue;
    }
    ResultLine r;
    if (std::sscanf(buf, "%lf %lf %lf %lf %lf %lf %d", &r.f0_hz, &r.P_b, &r.tau, &r.Psi, &r.power, &r.fA,
                    &r.n_harm) == 7)
      lines.push_back(r);
  }
  std::fclose(f);
  return 0;
}

int dump_float_buffer(const float* buffer, size_t size, const std::string& path) {
  FILE* out = std::fopen(path.c_str(), "w");
  if (!out) {
    log_message(LOG_ERROR, true, "Error opening file \"%s\" for buffer dump!\n", path.c_str());
    return RADPUL_EFILE;
  }
  for (size_t i = 0; i < size; ++i) std::fprintf(out, "%e\n", buffer[i]);
  std::fclose(out);
  log_message(LOG_DEBUG, true, "Successfully wrote buffer to \"%s\"...\n", path.c_str());
  return 0;
}

}  // namespace brp
