// Multi-work-unit batching (the reference processes several WUs of one BOINC
// task as sequential "passes", erp_boinc_wrapper.cpp:411-474). Here K work
// units of the same shape are resident in HBM at once: every device pipeline
// holds all K (whitened) series, and one batch mixes templates of different
// WUs, so the per-WU setup work (whitening, host I/O) and the per-batch host
// round trips are amortised over K × bank templates.
//
// Per WU the candidate table still evolves exactly as in the sequential
// reference: (template, WU) pairs are dealt WU-major in blocks of
// BRP_MULTI_BLOCK batches of templates (default 64, at most the bank): block
// [t0, t0 + TB) of WU 0, the same block of WU 1, ..., then the next block. A
// batch holds templates of one WU (except where per-WU resume points cut a
// block short), each WU sees its templates in increasing order, and pairs
// are applied in deal order, each to its own WU's table. After a whole block
// every WU has completed the same template prefix: the checkpoint points of
// the batched multi-pass task (csrc/app/passes.cpp).
#pragma once

#include <cstdint>
#include <functional>
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
  bool interrupted = false;  // the hook asked to stop (quit / abort / lost heartbeat)
  BackendStats stats;
};

// Called after every applied batch with the pairs applied so far in this run
// and, when the batch completed a deal block, the template prefix every WU
// has now completed (0 otherwise). Return false to stop after this batch.
using MultiHook = std::function<bool(uint64_t pairs_applied, uint32_t prefix_done)>;

// deal block in templates for batch size B and a bank of `total` templates:
// BRP_MULTI_BLOCK (default 64) batches, capped at the bank (no 32-bit wrap)
uint32_t multi_block_templates(int B, uint32_t total);

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
  // per-WU first templates (resumed WUs), optional hook (progress, checkpoints, quit)
  int run(const std::vector<uint32_t>& begins, uint32_t end, std::vector<CandidateTable>& tables, MultiResult& res,
          const MultiHook& hook);
  // block size override for tests (0: BRP_MULTI_BLOCK / default)
  void set_block_batches(uint32_t n);
  // open() failed because the work units differ in FFT geometry
  bool shape_mismatch() const;
  const SearchInfo& info() const;
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
