// The search driver (reference MAIN, demod_binary.c:117-1695).
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "../core/io.hpp"
#include "../core/search_core.hpp"
#include "../engine/backend.hpp"

namespace brp {

struct SearchResult {
  CandidateTable table;
  SearchGeometry geom;
  uint32_t templates_total = 0;
  uint32_t templates_done = 0;   // including those restored from a checkpoint
  uint32_t templates_run = 0;    // processed in this call
  bool interrupted = false;      // quit request: no final checkpoint/output
  double t_setup = 0, t_templates = 0, t_total = 0;  // seconds
  uint64_t dirty_pages = 0;
  BackendStats stats;
};

struct SearchControl {
  // restrict to templates [begin, end) of the bank (sharded runs); end=0: all
  uint32_t begin = 0, end = 0;
  bool write_output = true;       // result file + final checkpoint
  bool use_checkpoint = true;
  int gpus = 1;                   // devices driven by this process (in-order merge)
  int pipelines = 1;              // independent pipelines (stream + buffers) per device
  uint32_t progress_every = 1;    // fraction_done / screensaver every N templates
  std::vector<int> devices;       // explicit device ids (optional)
  // called after every template applied (progress hooks / fault injection)
  std::function<void(uint32_t done, uint32_t total)> on_template;
};

// The application's last pass leaves its device state (buffers, streams) to
// process exit instead of freeing it: the OS reclaims it faster than the
// teardown (whole-process wall time). Off by default (library use).
void set_keep_device_state_on_return(bool on);

// Per-template hook of SearchSession::run: return false to stop after this template.
using TemplateHook = std::function<bool(uint32_t done, const SearchInfo& info)>;

// One work unit held open: bank, series, geometry and the device backends.
// Reused across runs (benchmark steps, sharded ranges) without re-reading files.
class SearchSession {
 public:
  SearchSession();
  ~SearchSession();
  // read bank / WU / zaplist and create the backends (no device work yet)
  int open(const SearchOptions& opt, const SearchControl& ctl);
  // (re)upload the raw series and whiten it on the device(s); required before run()
  int prepare();
  // -z + dump directory: write the debug buffer dumps (called by prepare())
  int dump_debug_buffers();
  // process templates [begin, end) and apply them in template order to `table`
  int run(uint32_t begin, uint32_t end, CandidateTable& table, SearchResult& res, const TemplateHook& hook);
  const SearchGeometry& geometry() const;
  const TemplateBank& bank() const;
  const WorkUnit& work_unit() const;
  const SearchOptions& options() const;
  uint32_t total() const;
  BackendStats stats() const;
  // Global pruning across ranks (parallel/dist.py FloorSync): level floors
  // (100th power, 0 while a level is not full) of the table the running
  // run() applies to, and lower bounds of the *merged* table's floors that
  // other ranks reported. Device thresholds become max(chi2, own floor,
  // external floor); the table itself is applied with its own thresholds, so
  // only bins that can never reach the merged table are filtered out
  // (demod_binary.c:1268-1282 semantics). External floors only
  // rise; reset them before every independent search.
  void local_floors(float out[kNumHarmonicLevels]) const;
  void raise_external_floors(const float f[kNumHarmonicLevels]);
  void reset_external_floors();

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

// Screensaver sky position / DM of a WU header (demod_binary.c:745-771).
void sky_position(const DDHeader& h, SearchInfo& info);

// Full search of one WU with the options' files. Returns a RADPUL_* code.
int run_search(const SearchOptions& opt, const SearchControl& ctl, SearchResult& res);

// MAIN-compatible entry: parses the reference command line (short options and
// the --input_file style long names, demod_binary.c:217-445) plus MI355X
// extensions (--mi355x-batch N, --mi355x-gpus N, --mi355x-cpu).
int search_main(int argc, char** argv);

// Parse the MAIN command line (plus --mi355x-* extensions) into options.
int parse_search_args(int argc, char** argv, SearchOptions& opt, SearchControl& ctl, bool& spin);

// Batched multi-pass task: the pending passes (indices into in/out) run as one
// MultiSession with per-WU checkpoints "<cp>.<pass>", results and reference
// pass semantics. Sets `fallback` (and returns 0) when the WUs cannot be
// batched (different shapes, no HIP FFT plan); the caller then runs the passes
// sequentially.
int run_passes_batched(const std::vector<std::string>& in, const std::vector<std::string>& out,
                       const std::vector<size_t>& pending, const SearchOptions& opt, const SearchControl& ctl,
                       bool& fallback);

// BOINC wrapper entry (erp_boinc_wrapper.cpp:242-584): getopt_long with the
// dashed long names, several -i/-o pairs processed as sequential passes.
int wrapper_main(int argc, char** argv);

// Final stage shared by single and sharded runs: checkpoint + result file.
int finalize_output(const SearchOptions& opt, const SearchGeometry& g, uint32_t n_done, CandidateTable& table,
                    const std::string& exec_name);

}  // namespace brp
