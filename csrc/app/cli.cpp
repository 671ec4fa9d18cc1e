// Command-line front ends: MAIN-compatible parser and the BOINC wrapper.
#include <getopt.h>

#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../boinc/runtime.hpp"
#include "../boinc/ipc.hpp"
#include "../core/errors.hpp"
#include "../core/log.hpp"
#include "../engine/backend.hpp"
#include "search.hpp"

#ifndef BRP_GIT_ID
#define BRP_GIT_ID "unknown"
#endif

namespace brp {

namespace {

void print_usage(const char* prog) {
  std::printf("\nUsage: %s [options], options are:\n\n", prog);
  std::printf(" -h, --help\t\t\tboolean\tPrint this message\n");
  std::printf(" -i, --input_file\t\tstring\tThe name of the input file.\n");
  std::printf(" -o, --output_file\t\tstring\tThe name of the candidate output file.\n");
  std::printf(" -t, --template_bank\t\tstring\tThe name of the random template bank.\n");
  std::printf(" -c, --checkpoint_file\t\tstring\tThe name of the checkpoint file.\n");
  std::printf(" -l, --zaplist_file\t\tstring\tThe name of the zaplist file.\n");
  std::printf(" -f, --f0\t\t\tfloat\tThe maximum signal frequency (in Hz)\n");
  std::printf(" -A, --false_alarm\t\tfloat\tFalse alarm probability.\n");
  std::printf(" -P, --padding\t\t\tfloat\tThe frequency over-resolution factor.\n");
  std::printf(" -W, --whitening\t\tboolean\tSwitch for power spectrum whitening and line zapping.\n");
  std::printf(" -B, --box\t\t\tint\tWindow width for the running median in frequeny bins.\n");
  std::printf(" -D, --device\t\tinteger\tThe GPU device ID to be used.\n");
  std::printf(" -z, --debug\t\t\tboolean\tRun program in debug mode.\n");
  std::printf(" --mi355x-batch\t\tinteger\tTemplates per device batch (default 1).\n");
  std::printf(" --mi355x-gpus\t\tinteger\tGPUs (or CPU worker threads with --mi355x-cpu) driven by this process (default 1).\n");
  std::printf(" --mi355x-cpu\t\t\tboolean\tUse the CPU golden backend.\n");
  std::printf(" --mi355x-ps-fp16\t\tboolean\tStore the power spectrum as fp16 (needs -W). Inexact: near-tie\n"
              "\t\t\t\t\ttable entries may differ from fp32 (experiment, not the product path).\n");
  std::printf(" --mi355x-spin\t\t\tboolean\tBusy-wait for the GPU instead of sleeping (default: blocking sync).\n");
  std::printf(" --mi355x-pipelines\t\tinteger\tIndependent pipelines per GPU (default 3, one template each).\n");
  std::printf(" --mi355x-no-checkpoint\t\tboolean\tNever read or write checkpoints (Debian NOCHECKPOINTING build).\n");
  std::printf(" --mi355x-progress-every\tinteger\tReport fraction done every N templates (Debian COMMUNICATIONREDUCTION).\n");
  std::printf(" --mi355x-sequential-passes\tboolean\tRun several -i/-o pairs one after another instead of batched.\n");
  std::printf(" --mi355x-dump-dir\t\tstring\tWith -z: write the whitened series and template 0's resampled series and\n"
              "\t\t\t\t\tpower spectrum as text (one value per line) into this directory.\n");
  std::printf("\n");
}

bool is(const char* a, const char* s, const char* l) { return std::strcmp(a, s) == 0 || std::strcmp(a, l) == 0; }

}  // namespace

int parse_search_args(int argc, char** argv, SearchOptions& opt, SearchControl& ctl, bool& spin) {
  opt = SearchOptions();
  ctl = SearchControl();
  spin = false;  // --mi355x-spin: busy-wait host synchronisation
  // measured best on one MI355X: 3 pipelines of one template each (the FFT
  // intermediates of every pipeline stay in the Infinity Cache)
  ctl.pipelines = 3;
  opt.batch = 1;
  int i = 1;
  auto need = [&](int k) -> const char* {
    if (k + 1 >= argc) return nullptr;
    return argv[k + 1];
  };
  while (i < argc) {
    const char* a = argv[i];
    const char* v = need(i);
    if (is(a, "-W", "--whitening")) {
      opt.white = true;
      i++;
    } else if (is(a, "-P", "--padding")) {
      if (!v) return RADPUL_EVAL;
      const double x = std::atof(v);
      if (x < 1.0) {
        log_message(LOG_ERROR, true, "Nonsense value: padding factor %g < 1.0.\n", x);
        return RADPUL_EVAL;
      }
      if (x > 10.0) {
        log_message(LOG_ERROR, true, "Nonsense value: padding factor %g > 10.0.\n", x);
        return RADPUL_EVAL;
      }
      opt.padding = static_cast<float>(x);
      i += 2;
    } else if (is(a, "-B", "--box")) {
      if (!v) return RADPUL_EVAL;
      const int x = std::atoi(v);
      if (x < 0) {
        log_message(LOG_ERROR, true, "Nonsense value: window size for running median %d is negative.\n", x);
        return RADPUL_EVAL;
      }
      if (x > 250000) {
        log_message(LOG_ERROR, true, "Nonsense value: window size for running median too large: %d.\n", x);
        return RADPUL_EVAL;
      }
      opt.window = static_cast<uint32_t>(x);
      i += 2;
    } else if (is(a, "-z", "--debug")) {
      opt.debug = true;
      log_message(LOG_DEBUG, true, "Running program in debugging mode.\n");
      i++;
    } else if (is(a, "-f", "--f0")) {
      if (!v) return RADPUL_EVAL;
      const double x = std::atof(v);
      if (x < 0.0) {
        log_message(LOG_ERROR, true, "Nonsense value: upper limit for search frequency %g is negative.\n", x);
        return RADPUL_EVAL;
      }
      if (x > 16.0e3) {
        log_message(LOG_ERROR, true, "Nonsense value: upper limit for search frequency %g > 16 kHz.\n", x);
        return RADPUL_EVAL;
      }
      opt.f0 = static_cast<float>(x);
      i += 2;
    } else if (is(a, "-A", "--false_alarm")) {
      if (!v) return RADPUL_EVAL;
      const double x = std::atof(v);
      if (x < 0.0) {
        log_message(LOG_ERROR, true, "Nonsense value: false alarm rate %g is negative.\n", x);
        return RADPUL_EVAL;
      }
      if (x > 1.0) {
        log_message(LOG_ERROR, true, "Nonsense value: false alarm rate %g > 1.0.\n", x);
        return RADPUL_EVAL;
      }
      opt.fA = static_cast<float>(x);
      i += 2;
    } else if (is(a, "-i", "--input_file")) {
      if (!v) return RADPUL_EFILE;
      opt.inputfile = v;
      bool four;
      if (work_unit_format(opt.inputfile, four)) return RADPUL_EFILE;
      i += 2;
    } else if (is(a, "-o", "--output_file")) {
      if (!v) return RADPUL_EFILE;
      opt.outputfile = v;
      if (opt.outputfile.size() + 4 >= static_cast<size_t>(kFnLength + 4)) {
        log_message(LOG_ERROR, true, "Couldn't prepare temporary output file name: %s\n", v);
        return RADPUL_EFILE;
      }
      i += 2;
    } else if (is(a, "-c", "--checkpoint_file")) {
      if (!v) return RADPUL_EFILE;
      opt.checkpointfile = v;
      if (opt.checkpointfile.size() + 4 >= static_cast<size_t>(kFnLength + 4)) {
        log_message(LOG_ERROR, true, "Couldn't prepare temporary checkpoint file name: %s\n", v);
        return RADPUL_EFILE;
      }
      i += 2;
    } else if (is(a, "-t", "--template_bank")) {
      if (!v) return RADPUL_EFILE;
      opt.templatebank = v;
      i += 2;
    } else if (is(a, "-l", "--zaplist_file")) {
      if (!v) return RADPUL_EFILE;
      opt.zaplistfile = v;
      i += 2;
    } else if (is(a, "-D", "--device")) {
      if (!v || !std::isdigit(static_cast<unsigned char>(*v))) {
        log_message(LOG_ERROR, true, "Invalid GPU device ID encountered: %s\n", v ? v : "");
        return RADPUL_EVAL;
      }
      errno = 0;
      const long d = std::strtol(v, nullptr, 10);
      if (errno != 0) return RADPUL_EVAL;
      opt.device = static_cast<int>(d);
      i += 2;
    } else if (std::strcmp(a, "--mi355x-batch") == 0) {
      if (!v) return RADPUL_EVAL;
      opt.batch = std::atoi(v);
      i += 2;
    } else if (std::strcmp(a, "--mi355x-gpus") == 0) {
      if (!v) return RADPUL_EVAL;
      ctl.gpus = std::max(1, std::atoi(v));
      i += 2;
    } else if (std::strcmp(a, "--mi355x-pipelines") == 0) {
      if (!v) return RADPUL_EVAL;
      ctl.pipelines = std::max(1, std::atoi(v));
      i += 2;
    } else if (std::strcmp(a, "--mi355x-no-checkpoint") == 0) {
      // runtime form of the Debian package's -DNOCHECKPOINTING
      // (debian/patches/disable_checkpointing.patch)
      ctl.use_checkpoint = false;
      i++;
    } else if (std::strcmp(a, "--mi355x-progress-every") == 0) {
      // runtime form of -DCOMMUNICATIONREDUCTION=N (debian/patches/progressfraction.patch)
      if (!v) return RADPUL_EVAL;
      ctl.progress_every = static_cast<uint32_t>(std::max(1, std::atoi(v)));
      i += 2;
    } else if (std::strcmp(a, "--mi355x-ps-fp16") == 0) {
      opt.ps_fp16 = true;
      i++;
    } else if (std::strcmp(a, "--mi355x-spin") == 0) {
      spin = true;
      i++;
    } else if (std::strcmp(a, "--mi355x-cpu") == 0) {
      opt.use_cpu = true;
      i++;
    } else if (std::strcmp(a, "--mi355x-dump-dir") == 0) {
      if (!v) return RADPUL_EFILE;
      opt.dump_dir = v;
      i += 2;
    } else if (is(a, "-h", "--help")) {
      print_usage(argv[0]);
      return RADPUL_EMISC;
    } else {
      log_message(LOG_ERROR, true, "\nUnknown option \"%s\". Use '%s --help'.\n\n", a, argv[0]);
      return RADPUL_EMISC;
    }
  }
  if (!ctl.use_checkpoint && !opt.checkpointfile.empty()) {
    log_message(LOG_ERROR, true, "Disabled checkpointing - '-c %s' option ignored\n", opt.checkpointfile.c_str());
    opt.checkpointfile.clear();
  }
  return 0;
}

int search_main(int argc, char** argv) {
  SearchOptions opt;
  SearchControl ctl;
  bool spin = false;
  int prc = parse_search_args(argc, argv, opt, ctl, spin);
  if (prc) return prc;
  // a BOINC app shares the host: wait for the GPU by sleeping, as the
  // reference's blocking-sync context does, unless --mi355x-spin
  hip_set_blocking_sync(!spin);
  SearchResult res;
  int rc = run_search(opt, ctl, res);
  if (rc == 0 && res.templates_run > 0) {
    log_message(LOG_INFO, true, "Throughput: %u templates in %.3f s (%.1f templates/s, setup %.3f s)\n",
                res.templates_run, res.t_templates, res.templates_run / std::max(res.t_templates, 1e-9), res.t_setup);
  }
  // quit / abort / lost heartbeat: leave without a final checkpoint and
  // without the finish marker (demod_binary.c:1489-1492 calls exit(0))
  if (rc == 0 && res.interrupted) boinc::quit_exit(0);
  return rc;
}

int wrapper_main(int argc, char** argv) {
  std::vector<std::string> fwd;       // forwarded options (short forms)
  std::vector<std::string> inputs, outputs;
  std::string checkpoint;
  bool sequential = false;  // --mi355x-sequential-passes
  fwd.push_back(argv[0]);
  static struct option long_options[] = {{"input-file", required_argument, 0, 'i'},
                                         {"template-bank-file", required_argument, 0, 't'},
                                         {"output-file", required_argument, 0, 'o'},
                                         {"checkpoint-file", required_argument, 0, 'c'},
                                         {"zaplist-file", required_argument, 0, 'l'},
                                         {"f0", required_argument, 0, 'f'},
                                         {"false-alarm", required_argument, 0, 'A'},
                                         {"kill-line", no_argument, 0, 'K'},
                                         {"padding", required_argument, 0, 'P'},
                                         {"whitening", no_argument, 0, 'W'},
                                         {"box", required_argument, 0, 'B'},
                                         {"device", required_argument, 0, 'D'},
                                         {"debug", no_argument, 0, 'z'},
                                         {"help", no_argument, 0, 'h'},
                                         {"version", no_argument, 0, 'v'},
                                         {"mi355x-batch", required_argument, 0, 1001},
                                         {"mi355x-gpus", required_argument, 0, 1002},
                                         {"mi355x-cpu", no_argument, 0, 1003},
                                         {"mi355x-ps-fp16", no_argument, 0, 1004},
                                         {"mi355x-spin", no_argument, 0, 1005},
                                         {"mi355x-pipelines", required_argument, 0, 1006},
                                         {"mi355x-no-checkpoint", no_argument, 0, 1007},
                                         {"mi355x-progress-every", required_argument, 0, 1008},
                                         {"mi355x-sequential-passes", no_argument, 0, 1009},
                                         {"mi355x-dump-dir", required_argument, 0, 1010},
                                         {0, 0, 0, 0}};
  optind = 1;
  auto file_arg = [&](const char* opt, const char* val) {
    std::string phys;
    boinc::resolve_filename(val, phys);
    fwd.push_back(opt);
    fwd.push_back(phys);
  };
  for (;;) {
    int idx = 0;
    const int r = getopt_long(argc, argv, "i:t:o:c:l:f:A:KP:WB:D:zhv", long_options, &idx);
    if (r == -1) break;
    switch (r) {
      case 'i': inputs.push_back(optarg); break;
      case 'o': outputs.push_back(optarg); break;
      case 't': file_arg("-t", optarg); break;
      case 'c':
        checkpoint = optarg;
        file_arg("-c", optarg);
        break;
      case 'l': file_arg("-l", optarg); break;
      case 'f': fwd.push_back("-f"); fwd.push_back(optarg); break;
      case 'A': fwd.push_back("-A"); fwd.push_back(optarg); break;
      case 'K': fwd.push_back("-K"); break;  // forwarded; MAIN rejects it (reference quirk)
      case 'P': fwd.push_back("-P"); fwd.push_back(optarg); break;
      case 'W': fwd.push_back("-W"); break;
      case 'B': fwd.push_back("-B"); fwd.push_back(optarg); break;
      case 'D': fwd.push_back("-D"); fwd.push_back(optarg); break;
      case 'z': fwd.push_back("-z"); break;
      case 'h': fwd.push_back("-h"); break;
      case 'v':
        log_message(LOG_INFO, true, "Version information:\n");
        log_message(LOG_INFO, false, "Binary Pulsar Search Revision: %s\n", BRP_GIT_ID);
        log_message(LOG_INFO, false, "BOINC Revision: %s\n", "brp-app-runtime (client shared memory protocol)");
        return 0;
      case 1001: fwd.push_back("--mi355x-batch"); fwd.push_back(optarg); break;
      case 1002: fwd.push_back("--mi355x-gpus"); fwd.push_back(optarg); break;
      case 1003: fwd.push_back("--mi355x-cpu"); break;
      case 1004: fwd.push_back("--mi355x-ps-fp16"); break;
      case 1005: fwd.push_back("--mi355x-spin"); break;
      case 1006: fwd.push_back("--mi355x-pipelines"); fwd.push_back(optarg); break;
      case 1007: fwd.push_back("--mi355x-no-checkpoint"); break;
      case 1008: fwd.push_back("--mi355x-progress-every"); fwd.push_back(optarg); break;
      case 1009: sequential = true; break;
      case 1010: fwd.push_back("--mi355x-dump-dir"); fwd.push_back(optarg); break;
      default: boinc::finish(EINSTEINRADIO_EOPT);
    }
  }
  if (optind < argc) {
    log_message(LOG_WARN, true, "Non-option arguments encountered:\n");
    while (optind < argc) log_message(LOG_WARN, false, "%s\n", argv[optind++]);
  }
  int result = 0;
  if (inputs.size() != outputs.size()) {
    log_message(LOG_ERROR, true, "number of input- and output files don't match\n");
    result = 1;
  }
  if (ipc::setup_shmem()) {
    log_message(LOG_WARN, true, "Shared memory setup failed!\n");
  }
  const size_t passes = inputs.size();
  // several pending same-shape passes on the HIP backend: one batched session
  // holds every pending WU in HBM (csrc/app/passes.cpp); otherwise, and for
  // passes it cannot batch, the reference's sequential loop below
  if (!result && passes >= 2 && !sequential) {
    std::vector<std::string> in_phys(passes), out_phys(passes);
    std::vector<size_t> pending;
    for (size_t p = 0; p < passes; ++p) {
      boinc::resolve_filename(inputs[p], in_phys[p]);
      boinc::resolve_filename(outputs[p], out_phys[p]);
      if (FILE* fp = std::fopen(out_phys[p].c_str(), "r")) {
        log_message(LOG_INFO, true, "Output file: '%s' already exists - skipping pass\n", out_phys[p].c_str());
        std::fclose(fp);
      } else {
        pending.push_back(p);
      }
    }
    std::vector<char*> av;
    for (auto& a : fwd) av.push_back(const_cast<char*>(a.c_str()));
    av.push_back(nullptr);
    SearchOptions opt;
    SearchControl ctl;
    bool spin = false;
    if (pending.size() >= 2 && parse_search_args(static_cast<int>(fwd.size()), av.data(), opt, ctl, spin) == 0 &&
        !opt.use_cpu) {
      hip_set_blocking_sync(!spin);
      bool fallback = false;
      result = run_passes_batched(in_phys, out_phys, pending, opt, ctl, fallback);
      if (!fallback) {
        if (result) log_message(LOG_ERROR, true, "Demodulation failed (error: %i)!\n", result);
        return result;
      }
      log_message(LOG_INFO, true, "Work units differ in shape: processing the passes one after another.\n");
    }
  }
  for (size_t pass = 0; pass < passes && !result; ++pass) {
    std::vector<std::string> args = fwd;
    std::string in_phys, out_phys;
    boinc::resolve_filename(inputs[pass], in_phys);
    boinc::resolve_filename(outputs[pass], out_phys);
    args.push_back("-i");
    args.push_back(in_phys);
    args.push_back("-o");
    args.push_back(out_phys);
    if (FILE* fp = std::fopen(out_phys.c_str(), "r")) {
      log_message(LOG_INFO, true, "Output file: '%s' already exists - skipping pass\n", out_phys.c_str());
      std::fclose(fp);
      continue;
    }
    std::vector<char*> av;
    for (auto& s : args) av.push_back(const_cast<char*>(s.c_str()));
    av.push_back(nullptr);
    boinc::set_pass(static_cast<int>(pass), static_cast<int>(passes));
    // the last pass's device state is left to process exit (BRP_FAST_EXIT=0: freed)
    set_keep_device_state_on_return(pass + 1 == passes && boinc::fast_exit_enabled());
    result = search_main(static_cast<int>(args.size()), av.data());
    set_keep_device_state_on_return(false);
    if (result) {
      log_message(LOG_ERROR, true, "Demodulation failed (error: %i)!\n", result);
      break;
    }
    log_message(LOG_DEBUG, true, "Demodulation successful!\n");
    if (!checkpoint.empty()) {
      std::string cp_phys;
      boinc::resolve_filename(checkpoint, cp_phys);
      std::remove(cp_phys.c_str());
    }
  }
  return result;
}

}  // namespace brp
