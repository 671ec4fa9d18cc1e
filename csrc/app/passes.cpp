// Batched multi-pass BOINC task.
//
// The reference wrapper processes the -i/-o pairs of one task as sequential
// passes (erp_boinc_wrapper.cpp:411-474): skip a pass whose output exists, run
// MAIN on it, delete the checkpoint, report fraction_done = (frac + pass) /
// passes. Here every pending pass of the same shape is resident in HBM at once
// (MultiSession: one whitened series per WU, batches dealt WU-major in blocks)
// and the per-WU semantics are kept:
//   * each WU's candidate table evolves exactly as in its own sequential pass,
//     so the result files are byte-identical to the sequential ones;
//   * checkpoints are per WU, "<cp>.<pass index>" (the reference's layout and
//     atomic write), written at deal-block boundaries where every pending WU
//     has completed the same template prefix; a reference-style "<cp>" whose
//     header names one of the pending inputs is also accepted on resume;
//   * a WU resumes at its own checkpointed template;
//   * quit / abort / lost heartbeat leave without final checkpoints
//     (demod_binary.c:1489-1492); on success every pass gets its final
//     checkpoint and result file, then the checkpoints are deleted.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../boinc/ipc.hpp"
#include "../boinc/runtime.hpp"
#include "../core/errors.hpp"
#include "../core/fault.hpp"
#include "../core/io.hpp"
#include "../core/log.hpp"
#include "multi.hpp"
#include "search.hpp"

namespace brp {

namespace {

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

std::string pass_checkpoint(const std::string& cp, size_t pass) { return cp + "." + std::to_string(pass); }

// checkpoint of input `in` (n_template, table) from `path`; rc != 0 on a
// damaged or inconsistent file, `found` false when there is none for `in`
int restore(const std::string& path, const std::string& in, uint32_t total, CandidateTable& table, uint32_t& n,
            bool& found) {
  found = false;
  Checkpoint cp;
  bool exists = false;
  int rc = read_checkpoint(path, cp, exists);
  if (rc || !exists) return rc;
  cp.header.originalfile[kFnLength - 1] = 0;
  if (in != cp.header.originalfile) return 0;
  if (cp.header.n_template > total) {
    log_message(LOG_ERROR, true,
                "Header checkpoint file %s contains inconsistent information about number of templates done "
                "(%u > %u).\n",
                path.c_str(), cp.header.n_template, total);
    return RADPUL_EFILE;
  }
  std::memcpy(table.data(), cp.cands, sizeof(cp.cands));
  n = cp.header.n_template;
  found = true;
  return 0;
}

int write_cp(const std::string& path, const std::string& in, uint32_t n, CandidateTable& table) {
  Checkpoint cp;
  std::memset(&cp.header, 0, sizeof(cp.header));
  cp.header.n_template = n;
  std::snprintf(cp.header.originalfile, sizeof(cp.header.originalfile), "%s", in.c_str());
  std::memcpy(cp.cands, table.data(), sizeof(cp.cands));
  return write_checkpoint(path, cp);
}

}  // namespace

int run_passes_batched(const std::vector<std::string>& in, const std::vector<std::string>& out,
                       const std::vector<size_t>& pending, const SearchOptions& opt, const SearchControl& ctl,
                       bool& fallback) {
  fallback = false;
  const double t_start = now_s();
  const size_t passes = in.size();
  const size_t K = pending.size();
  std::vector<std::string> ins, outs;
  for (size_t p : pending) {
    ins.push_back(in[p]);
    outs.push_back(out[p]);
  }
  // every pipeline of every device is one engine of the session
  SearchControl mctl = ctl;
  const int ngpu = std::max(1, ctl.gpus), per_dev = std::max(1, ctl.pipelines);
  mctl.gpus = ngpu * per_dev;
  mctl.devices.clear();
  int dev0 = opt.device;
  if (dev0 < 0 && boinc::init_data().gpu_device_num >= 0) dev0 = boinc::init_data().gpu_device_num;
  if (dev0 < 0) dev0 = 0;
  for (int g = 0; g < ngpu; ++g)
    for (int k = 0; k < per_dev; ++k) mctl.devices.push_back(ngpu > 1 ? g : dev0);
  log_message(LOG_INFO, true, "Starting data processing of %zu work units in one batched pass...\n", K);
  if (fault_enabled("resource_error")) return RADPUL_HIP_MEM_ALLOC_HOST;

  MultiSession ms;
  boinc::begin_critical_section();
  int rc = ms.open(ins, opt, mctl);
  boinc::end_critical_section();
  if (rc) {
    if (ms.shape_mismatch() || rc == RADPUL_HIP_FFT_PLAN) {
      fallback = true;
      return 0;
    }
    return rc;
  }
  const uint32_t total = ms.total();

  // per-WU resume points
  std::vector<CandidateTable> tables(K);
  std::vector<uint32_t> begins(K, 0);
  const bool use_cp = ctl.use_checkpoint && !opt.checkpointfile.empty();
  if (use_cp) {
    for (size_t k = 0; k < K; ++k) {
      bool found = false;
      rc = restore(pass_checkpoint(opt.checkpointfile, pending[k]), ins[k], total, tables[k], begins[k], found);
      if (!rc && !found) rc = restore(opt.checkpointfile, ins[k], total, tables[k], begins[k], found);
      if (rc) return rc;
      if (found)
        log_message(LOG_INFO, true, "Continuing work on %s at template no. %u\n", ins[k].c_str(), begins[k]);
    }
  }
  const uint32_t first = *std::min_element(begins.begin(), begins.end());
  if (first < total) {
    boinc::begin_critical_section();
    rc = ms.prepare();
    boinc::end_critical_section();
    if (rc) return rc;
  }

  // progress: passes already complete + per-WU template fractions
  uint64_t restored = 0;
  for (uint32_t b : begins) restored += b;
  const double done_passes = static_cast<double>(passes - K);
  boinc::set_pass(0, 1);
  long kill_after = -1;
  std::string fault_arg;
  if (fault_enabled("kill_after_template", &fault_arg)) kill_after = std::atol(fault_arg.c_str());
  int cp_rc = 0;
  const double t_loop = now_s();
  auto hook = [&](uint64_t applied, uint32_t prefix) -> bool {
    const double frac = (done_passes + static_cast<double>(restored + applied) / total) / passes;
    boinc::fraction_done(frac);
    if (ipc::update_due()) ipc::update_shmem(ms.info());
    if (prefix > 0 && use_cp && boinc::time_to_checkpoint()) {
      for (size_t k = 0; k < K && !cp_rc; ++k)
        cp_rc = write_cp(pass_checkpoint(opt.checkpointfile, pending[k]), ins[k], std::max(begins[k], prefix),
                         tables[k]);
      if (cp_rc) {
        boinc::end_critical_section();
        return false;
      }
      log_message(LOG_INFO, true, "Checkpoint committed!\n");
      boinc::checkpoint_completed();
    }
    if (kill_after >= 0 && prefix >= static_cast<uint32_t>(kill_after)) boinc::request_quit();
    boinc::suspend_point();
    const boinc::Status st = boinc::get_status();
    return !(st.quit_request || st.abort_request || st.no_heartbeat);
  };
  MultiResult res;
  if (first < total) rc = ms.run(begins, total, tables, res, hook);
  if (rc) return rc;
  if (cp_rc) return cp_rc;
  if (res.interrupted) {
    log_message(LOG_WARN, true, "BOINC wants us to quit prematurely or we lost contact! Exiting...\n");
    boinc::quit_exit(0);
  }
  const double t_templates = now_s() - t_loop;
  for (size_t k = 0; k < K; ++k) {
    SearchOptions o = opt;
    o.inputfile = ins[k];
    o.outputfile = outs[k];
    o.checkpointfile = use_cp ? pass_checkpoint(opt.checkpointfile, pending[k]) : std::string();
    rc = finalize_output(o, ms.geometry(), total, tables[k], "einsteinbinary_mi355x");
    if (rc) {
      log_message(LOG_ERROR, true, "Demodulation failed (error: %i)!\n", rc);
      return rc;
    }
  }
  // the passes are done: remove their checkpoints (erp_boinc_wrapper.cpp:463-464)
  if (!opt.checkpointfile.empty()) {
    for (size_t k = 0; k < K; ++k) std::remove(pass_checkpoint(opt.checkpointfile, pending[k]).c_str());
    std::remove(opt.checkpointfile.c_str());
  }
  const uint64_t pairs = res.pairs_run;
  log_message(LOG_INFO, true, "Throughput: %llu (template, WU) pairs in %.3f s (%.1f pairs/s, %zu WUs, setup %.3f s)\n",
              static_cast<unsigned long long>(pairs), t_templates, pairs / std::max(t_templates, 1e-9), K,
              t_loop - t_start);
  log_message(LOG_INFO, true, "Data processing finished successfully!\n");
  return 0;
}

}  // namespace brp
