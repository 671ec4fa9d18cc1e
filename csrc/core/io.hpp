// Host file I/O of the search: work units, template banks, zaplists,
// checkpoints and result files. File semantics follow the reference MAIN
// (demod_binary.c) including its parsing quirks, cited per function.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "formats.hpp"

namespace brp {

struct WorkUnit {
  DDHeader header{};           // byte-swapped to host order
  bool four_bit = true;        // .bin4 (4-bit) or .binary (8-bit)
  std::vector<float> samples;  // header.nsamples unpacked samples
  // the payload as stored (2 samples per byte for 4-bit): a device uploads
  // these n/2 (or n) bytes and unpacks them itself (hipk::launch_unpack)
  // instead of the 4n bytes of floats
  std::vector<uint8_t> packed;
};

// Format from the file name: ".binary" -> 8-bit, ".bin4" -> 4-bit, else
// RADPUL_EFILE (demod_binary.c:318-325). Returns 0 and sets four_bit.
int work_unit_format(const std::string& path, bool& four_bit);

// Read a (gzip'd or plain) work unit and unpack it to floats
// (demod_binary.c:655-850): 4-bit high nibble first, value/scale.
int read_work_unit(const std::string& path, WorkUnit& wu);

// Write a work unit (used by the synthetic-data generators and tests).
int write_work_unit(const std::string& path, const DDHeader& header,
                    const std::vector<uint8_t>& payload, bool gzip);

struct TemplateBank {
  std::vector<double> P, tau, Psi0;  // as parsed ("%lg %lg %lg")
  size_t size() const { return P.size(); }
};

// Parse a template bank. Lines are read with fgets(256) and a final line
// lacking '\n' is ignored (fgets && !feof, demod_binary.c:513); a line
// without three numbers is RADPUL_EVAL (:516-524).
int read_template_bank(const std::string& path, TemplateBank& bank);

struct ZapRange {
  double fmin, fmax;  // Hz
};
// Zaplist: "%lg %lg" lines, same fgets/feof quirk (demod_binary.c:993-1009).
int read_zaplist(const std::string& path, std::vector<ZapRange>& ranges);

struct Checkpoint {
  CPHeader header{};
  CPCand cands[kCandTotal]{};
};
// Returns RADPUL_EFILE/EIO on a damaged file, 0 on success; `exists` false if
// the file cannot be opened (fresh start).
int read_checkpoint(const std::string& path, Checkpoint& cp, bool& exists);
// Atomic write: <path>.tmp then rename (demod_binary.c:1743-1783).
int write_checkpoint(const std::string& path, const Checkpoint& cp);

struct ResultHeaderInfo {
  bool write_header = false;  // BOINC provenance header (demod_binary.c:1616-1622)
  int user_id = 0;
  std::string user_name;
  int host_id = 0;
  std::string host_cpid;
  std::string exec_name;
  std::string git_id;
  std::string boinc_rev;
};

// Final result file: significance, sort, per-f0 dedupe across harmonics,
// at most 100 lines, "%DONE%" marker, atomic rename (demod_binary.c:1501-1685).
// `cands` is modified (fA filled in, powers normalised, sorted).
// One "%e" value per line, the reference's debug buffer dump
// (dumpFloatBufferToTextFile, erp_utilities.cpp:216-233).
int dump_float_buffer(const float* buffer, size_t size, const std::string& path);

int write_results(const std::string& path, CPCand* cands, double t_obs,
                  const ResultHeaderInfo& info);

// Reads back candidate lines of a result file (for tests / validation).
struct ResultLine {
  double f0_hz, P_b, tau, Psi, power, fA;
  int n_harm;
};
int read_results(const std::string& path, std::vector<ResultLine>& lines, bool& done_marker);

}  // namespace brp
