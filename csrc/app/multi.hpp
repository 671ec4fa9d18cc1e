// Multi-work-unit batching (the reference processes several WUs of one BOINC
// task as sequential "passes", erp_boinc_wrapper.cpp:411-474). Here K work
// units of the same shape are resident in HBM at once: every device pipeline
// holds all K (whitened) series, and one batch mixes templates of different
// WUs, so the per-WU setup work (whitening, host I/O) and the per-batch host
// round trips are amortised over K × bank templates.
//
// Per WU the candidate table still evolves exactly as in the sequential
// reference: (template, WU) pairs are dealt in blocks of one batch of
// templates per WU and applied in that order, each to its own WU's table.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../core/search_core.hpp"
#include "search.hpp"

namespace brp {

struct MultiResult {
  uint32_t pairs_run = 0;    // (template, WU) pairs processed
  double t_prepare = 0;      // seconds: read + whiten + upload of all WUs
  double t_templates = 0;    // seconds: the template loop
  BackendStats stats;
};

class MultiSession {
 public:
  MultiSession();
  ~MultiSession();
  // `inputs`: K work units that must share the FFT geometry; opt supplies the
  // bank, zaplist and search flags (its inputfile/outputfile are ignored).
  // ctl.gpus pipelines on ctl.devices (HIP only).
  int open(const std::vector<std::string>& inputs, const SearchOptions& opt, const SearchControl& ctl);
  int prepare();
  // templates [begin, end) of every WU; tables[k] receives WU k's candidates
  int run(uint32_t begin, uint32_t end, std::vector<CandidateTable>& tables, MultiResult& res);
  // result files (and final checkpoints when opt.checkpointfile is set, suffixed
  // with the WU index) for every WU
  int finalize(const std::vector<std::string>& outputs, uint32_t n_done, std::vector<CandidateTable>& tables);
  size_t work_units() const;
  uint32_t total() const;
  const SearchGeometry& geometry() const;
  BackendStats stats() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

}  // namespace brp
