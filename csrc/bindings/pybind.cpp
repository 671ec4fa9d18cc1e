// Python bindings of the native BRP framework (module boinc_app_eah_brp_amd._brp).
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <stdexcept>

#include "../app/multi.hpp"
#include "../app/search.hpp"
#include "../boinc/runtime.hpp"
#include "../boinc/ipc.hpp"
#include "../core/cpu_backend.hpp"
#include "../core/cpu_fft.hpp"
#include "../core/errors.hpp"
#include "../core/gsl_compat.hpp"
#include "../core/io.hpp"
#include "../core/log.hpp"
#include "../core/resamp_math.hpp"
#include "../core/rngmed.hpp"
#include "../core/search_core.hpp"
#include "../core/stats.hpp"
#include "../core/wisdom.hpp"
#include "../engine/hip_engine.hpp"
#include "../hip/checked.hpp"

namespace py = pybind11;
using namespace brp;

namespace {

void check(int rc, const char* what) {
  if (rc) throw std::runtime_error(std::string(what) + " failed: " + error_string(rc) + " (" + std::to_string(rc) + ")");
}

py::dict header_to_dict(const DDHeader& h) {
  py::dict d;
  d["tsample"] = h.tsample;
  d["tobs"] = h.tobs;
  d["timestamp"] = h.timestamp;
  d["fcenter"] = h.fcenter;
  d["fchan"] = h.fchan;
  d["RA"] = h.RA;
  d["DEC"] = h.DEC;
  d["gal_l"] = h.gal_l;
  d["gal_b"] = h.gal_b;
  d["AZstart"] = h.AZstart;
  d["ZAstart"] = h.ZAstart;
  d["ASTstart"] = h.ASTstart;
  d["LSTstart"] = h.LSTstart;
  d["DM"] = h.DM;
  d["scale"] = h.scale;
  d["filesize"] = h.filesize;
  d["datasize"] = h.datasize;
  d["nsamples"] = h.nsamples;
  d["smprec"] = h.smprec;
  d["nchan"] = h.nchan;
  d["nifs"] = h.nifs;
  d["lagformat"] = h.lagformat;
  d["sum"] = h.sum;
  d["level"] = h.level;
  d["name"] = std::string(h.name, strnlen(h.name, kFnLength));
  d["originalfile"] = std::string(h.originalfile, strnlen(h.originalfile, kFnLength));
  d["proj_id"] = std::string(h.proj_id, strnlen(h.proj_id, kFnLength));
  d["observers"] = std::string(h.observers, strnlen(h.observers, kFnLength));
  return d;
}

DDHeader dict_to_header(const py::dict& d) {
  DDHeader h;
  std::memset(&h, 0, sizeof(h));
  auto getd = [&](const char* k, double def) { return d.contains(k) ? d[k].cast<double>() : def; };
  auto getu = [&](const char* k, unsigned def) { return d.contains(k) ? d[k].cast<unsigned>() : def; };
  h.tsample = getd("tsample", 64.0);
  h.tobs = getd("tobs", 0.0);
  h.timestamp = getd("timestamp", 0.0);
  h.fcenter = getd("fcenter", 0.0);
  h.fchan = getd("fchan", 0.0);
  h.RA = getd("RA", 0.0);
  h.DEC = getd("DEC", 0.0);
  h.gal_l = getd("gal_l", 0.0);
  h.gal_b = getd("gal_b", 0.0);
  h.DM = getd("DM", 0.0);
  h.scale = getd("scale", 1.0);
  h.nsamples = getu("nsamples", 0);
  h.filesize = getu("filesize", 0);
  h.datasize = getu("datasize", 0);
  h.nchan = static_cast<uint16_t>(getu("nchan", 0));
  h.nifs = static_cast<uint16_t>(getu("nifs", 1));
  auto sets = [&](const char* k, char* dst) {
    if (d.contains(k)) std::snprintf(dst, kFnLength, "%s", d[k].cast<std::string>().c_str());
  };
  sets("name", h.name);
  sets("originalfile", h.originalfile);
  sets("proj_id", h.proj_id);
  sets("observers", h.observers);
  return h;
}

SearchOptions dict_to_options(const py::dict& d) {
  SearchOptions o;
  if (d.contains("f0")) o.f0 = d["f0"].cast<float>();
  if (d.contains("padding")) o.padding = d["padding"].cast<float>();
  if (d.contains("fA")) o.fA = d["fA"].cast<float>();
  if (d.contains("window")) o.window = d["window"].cast<uint32_t>();
  if (d.contains("white")) o.white = d["white"].cast<bool>();
  if (d.contains("debug")) o.debug = d["debug"].cast<bool>();
  if (d.contains("device")) o.device = d["device"].cast<int>();
  if (d.contains("batch")) o.batch = d["batch"].cast<int>();
  if (d.contains("use_cpu")) o.use_cpu = d["use_cpu"].cast<bool>();
  if (d.contains("ps_fp16")) o.ps_fp16 = d["ps_fp16"].cast<bool>();
  if (d.contains("inputfile")) o.inputfile = d["inputfile"].cast<std::string>();
  if (d.contains("outputfile")) o.outputfile = d["outputfile"].cast<std::string>();
  if (d.contains("templatebank")) o.templatebank = d["templatebank"].cast<std::string>();
  if (d.contains("checkpointfile")) o.checkpointfile = d["checkpointfile"].cast<std::string>();
  if (d.contains("zaplistfile")) o.zaplistfile = d["zaplistfile"].cast<std::string>();
  if (d.contains("dump_dir")) o.dump_dir = d["dump_dir"].cast<std::string>();
  return o;
}

py::dict geometry_to_dict(const SearchGeometry& g) {
  py::dict d;
  d["n_unpadded"] = g.n_unpadded;
  d["nsamples"] = g.nsamples;
  d["fft_size"] = g.fft_size;
  d["window_2"] = g.window_2;
  d["fundamental_idx_hi"] = g.fundamental_idx_hi;
  d["harmonic_idx_hi"] = g.harmonic_idx_hi;
  d["nr_pages"] = g.nr_pages;
  d["t_obs"] = g.t_obs;
  d["t_obs_d"] = g.t_obs_d;
  d["dt"] = g.dt;
  d["step_inv"] = g.step_inv;
  d["prob"] = g.prob;
  d["chi2_thr"] = std::vector<float>(g.chi2_thr, g.chi2_thr + 5);
  return d;
}

SearchGeometry dict_to_geometry(const py::dict& d) {
  SearchGeometry g;
  g.n_unpadded = d["n_unpadded"].cast<uint32_t>();
  g.nsamples = d["nsamples"].cast<uint32_t>();
  g.fft_size = d["fft_size"].cast<uint32_t>();
  g.window_2 = d["window_2"].cast<uint32_t>();
  g.fundamental_idx_hi = d["fundamental_idx_hi"].cast<uint32_t>();
  g.harmonic_idx_hi = d["harmonic_idx_hi"].cast<uint32_t>();
  g.nr_pages = d["nr_pages"].cast<uint32_t>();
  g.t_obs = d["t_obs"].cast<float>();
  g.t_obs_d = d["t_obs_d"].cast<double>();
  g.dt = d["dt"].cast<float>();
  g.step_inv = d["step_inv"].cast<float>();
  g.prob = d["prob"].cast<float>();
  auto thr = d["chi2_thr"].cast<std::vector<float>>();
  for (int h = 0; h < 5; ++h) g.chi2_thr[h] = thr.at(h);
  return g;
}

py::array_t<uint8_t> table_bytes(const CandidateTable& t) {
  py::array_t<uint8_t> a(sizeof(CPCand) * kCandTotal);
  std::memcpy(a.mutable_data(), t.data(), sizeof(CPCand) * kCandTotal);
  return a;
}

void table_from_bytes(CandidateTable& t, py::array_t<uint8_t, py::array::c_style> a) {
  if (static_cast<size_t>(a.size()) != sizeof(CPCand) * kCandTotal) throw std::invalid_argument("need 24000 bytes");
  std::memcpy(t.data(), a.data(), sizeof(CPCand) * kCandTotal);
}

py::list cands_to_list(const std::vector<TemplateCands>& out) {
  py::list res;
  for (const auto& tc : out) {
    py::list lv;
    for (int h = 0; h < kNumHarmonicLevels; ++h) {
      py::array_t<uint32_t> bins(tc.level[h].size());
      py::array_t<float> pw(tc.level[h].size());
      for (size_t q = 0; q < tc.level[h].size(); ++q) {
        bins.mutable_at(q) = tc.level[h][q].bin;
        pw.mutable_at(q) = tc.level[h][q].power;
      }
      lv.append(py::make_tuple(bins, pw));
    }
    res.append(lv);
  }
  return res;
}

std::vector<TemplateInput> arrays_to_templates(py::array_t<float> P, py::array_t<float> tau, py::array_t<float> psi) {
  if (P.size() != tau.size() || P.size() != psi.size()) throw std::invalid_argument("template arrays differ in size");
  std::vector<TemplateInput> t(P.size());
  for (ssize_t k = 0; k < P.size(); ++k) t[k] = TemplateInput{P.at(k), tau.at(k), psi.at(k)};
  return t;
}

}  // namespace

// the checked build (_build.py --checked) is the module _brp_checked
#ifndef BRP_MODULE_NAME
#define BRP_MODULE_NAME _brp
#endif
PYBIND11_MODULE(BRP_MODULE_NAME, m) {
  m.doc() = "MI355X-native Einstein@Home binary radio pulsar search: native core";
  m.attr("DD_HEADER_SIZE") = sizeof(DDHeader);
  m.attr("CP_HEADER_SIZE") = sizeof(CPHeader);
  m.attr("CP_CAND_SIZE") = sizeof(CPCand);
  m.attr("N_CAND") = kCandTotal;
  m.attr("N_CAND_5") = kCandPerLevel;
  m.def("set_log_level", &set_log_level);
  m.def("error_string", &error_string);

  // ---------------------------------------------------------------- I/O
  m.def("read_work_unit", [](const std::string& path) {
    WorkUnit wu;
    check(read_work_unit(path, wu), "read_work_unit");
    py::array_t<float> s(wu.samples.size());
    std::memcpy(s.mutable_data(), wu.samples.data(), wu.samples.size() * sizeof(float));
    return py::make_tuple(header_to_dict(wu.header), s, wu.four_bit);
  });
  m.def("write_work_unit", [](const std::string& path, const py::dict& hdr, py::array_t<uint8_t> payload, bool gz) {
    std::vector<uint8_t> p(payload.data(), payload.data() + payload.size());
    check(write_work_unit(path, dict_to_header(hdr), p, gz), "write_work_unit");
  });
  m.def("read_template_bank", [](const std::string& path) {
    TemplateBank b;
    check(read_template_bank(path, b), "read_template_bank");
    return py::make_tuple(py::array_t<double>(b.P.size(), b.P.data()), py::array_t<double>(b.tau.size(), b.tau.data()),
                          py::array_t<double>(b.Psi0.size(), b.Psi0.data()));
  });
  m.def("read_zaplist", [](const std::string& path) {
    std::vector<ZapRange> z;
    check(read_zaplist(path, z), "read_zaplist");
    std::vector<std::pair<double, double>> out;
    for (auto& r : z) out.emplace_back(r.fmin, r.fmax);
    return out;
  });
  m.def("read_checkpoint", [](const std::string& path) -> py::object {
    Checkpoint cp;
    bool exists = false;
    check(read_checkpoint(path, cp, exists), "read_checkpoint");
    if (!exists) return py::none();
    CandidateTable t;
    std::memcpy(t.data(), cp.cands, sizeof(cp.cands));
    cp.header.originalfile[kFnLength - 1] = 0;
    return py::make_tuple(cp.header.n_template, std::string(cp.header.originalfile), t);
  });
  m.def("write_checkpoint", [](const std::string& path, uint32_t n, const std::string& orig, const CandidateTable& t) {
    Checkpoint cp;
    std::memset(&cp.header, 0, sizeof(cp.header));
    cp.header.n_template = n;
    std::snprintf(cp.header.originalfile, kFnLength, "%s", orig.c_str());
    std::memcpy(cp.cands, t.data(), sizeof(cp.cands));
    check(write_checkpoint(path, cp), "write_checkpoint");
  });
  m.def("read_results", [](const std::string& path) {
    std::vector<ResultLine> lines;
    bool done = false;
    check(read_results(path, lines, done), "read_results");
    py::list l;
    for (auto& r : lines) l.append(py::make_tuple(r.f0_hz, r.P_b, r.tau, r.Psi, r.power, r.fA, r.n_harm));
    return py::make_tuple(l, done);
  });

  // ---------------------------------------------------------------- numerics
  m.def("chisq_Q_even", &chisq_Q_even);
  m.def("chisq_Qinv_even", &chisq_Qinv_even);
  m.def("single_bin_probability", &single_bin_probability);
  m.def("power_thresholds", [](float prob) {
    float thr[5];
    power_thresholds(prob, thr);
    return std::vector<float>(thr, thr + 5);
  });
  m.def("candidate_significance", &candidate_significance);
  py::class_<Taus2>(m, "Taus2")
      .def(py::init<unsigned long>(), py::arg("seed") = 1)
      .def("set", &Taus2::set)
      .def("get", &Taus2::get)
      .def("uniform", &Taus2::uniform);
  m.def("gaussian_ziggurat", &gaussian_ziggurat);
  m.def("checked_build", &hipk::checked_build,
        "True in the device-side debug build (_brp_checked: bounds-checked kernel accesses, verified launches)");
  m.def(
      "device_check",
      []() {
        std::string rep;
        int rc;
        {
          py::gil_scoped_release rel;
          rc = hipk::device_check(&rep);
        }
        if (rc) throw std::runtime_error(rep);
      },
      "Synchronise the device and raise RuntimeError naming the fault if any work since the last check failed "
      "(checked build: the kernel, source line and address of an out-of-bounds access or guard-zone write)");
  m.def("hip_running_median", [](py::array_t<float, py::array::c_style> x, uint32_t w, int reps, int device) {
    std::vector<float> in(x.data(), x.data() + x.size()), out;
    double ms = 0;
    {
      py::gil_scoped_release rel;
      check(hip_running_median(device, in, w, out, reps, &ms), "hip_running_median");
    }
    return py::make_tuple(py::array_t<float>(out.size(), out.data()), ms);
  }, py::arg("x"), py::arg("w"), py::arg("reps") = 0, py::arg("device") = 0);
  m.def("running_median", [](py::array_t<float, py::array::c_style> x, size_t w) {
    if (static_cast<size_t>(x.size()) < w || w == 0) throw std::invalid_argument("window larger than input");
    py::array_t<float> out(x.size() - w + 1);
    running_median(x.data(), x.size(), w, out.mutable_data());
    return out;
  });
  m.def("lut_sin", [](float x) { return lut_sin(x, kSinLut, kCosLut); });
  m.def("lut_tables", []() {
    return py::make_tuple(std::vector<float>(kSinLut, kSinLut + kLutSize), std::vector<float>(kCosLut, kCosLut + kLutSize));
  });
  m.def("rfft", [](py::array_t<double, py::array::c_style> x) {
    std::vector<double> v(x.data(), x.data() + x.size());
    std::vector<cd> X;
    rfft_forward(v, X);
    py::array_t<std::complex<double>> out(X.size());
    std::memcpy(out.mutable_data(), X.data(), X.size() * sizeof(cd));
    return out;
  });
  m.def("irfft", [](py::array_t<std::complex<double>, py::array::c_style> X, size_t n) {
    std::vector<cd> v(X.data(), X.data() + X.size());
    std::vector<double> x;
    rfft_inverse(v, n, x);
    return py::array_t<double>(x.size(), x.data());
  });

  // ---------------------------------------------------------------- search core
  m.def("derive_geometry", [](const py::dict& hdr, const py::dict& opt) {
    SearchGeometry g;
    check(derive_geometry(dict_to_header(hdr), dict_to_options(opt), g), "derive_geometry");
    return geometry_to_dict(g);
  });
  py::class_<CandidateTable>(m, "CandidateTable")
      .def(py::init<>())
      .def("reset", &CandidateTable::reset)
      .def("floor_power", &CandidateTable::floor_power)
      .def("thresholds",
           [](const CandidateTable& t, std::vector<float> chi2) {
             float thr[5];
             t.thresholds(chi2.data(), thr);
             return std::vector<float>(thr, thr + 5);
           })
      .def("apply_level",
           [](CandidateTable& t, int h, py::array_t<uint32_t> bins, py::array_t<float> pw, float thr, float P, float tau,
              float psi) {
             std::vector<BinPower> v(bins.size());
             for (ssize_t q = 0; q < bins.size(); ++q) v[q] = BinPower{bins.at(q), pw.at(q)};
             return t.apply_level(h, v.data(), v.size(), thr, P, tau, psi);
           })
      .def("merge", &CandidateTable::merge)
      .def("to_bytes", &table_bytes)
      .def("from_bytes", &table_from_bytes)
      .def("entries", [](const CandidateTable& t) {
        py::list l;
        for (int i = 0; i < kCandTotal; ++i) {
          const CPCand& c = t.data()[i];
          l.append(py::make_tuple(c.f0, c.power, c.P_b, c.tau, c.Psi, c.n_harm));
        }
        return l;
      });
  m.def("write_results", [](const std::string& path, CandidateTable t, double t_obs, bool header) {
    ResultHeaderInfo info;
    info.write_header = header;
    CPCand c[kCandTotal];
    std::memcpy(c, t.data(), sizeof(c));
    check(write_results(path, c, t_obs, info), "write_results");
  });

  // ---------------------------------------------------------------- CPU golden model
  m.def("cpu_resample", [](py::array_t<float, py::array::c_style> series, const py::dict& gd, float P, float tau, float psi) {
    const SearchGeometry g = dict_to_geometry(gd);
    const ResampParams p = make_resamp_params(g.nsamples, g.n_unpadded, g.fft_size, g.dt, g.step_inv, P, tau, psi);
    std::vector<float> out;
    uint32_t n_steps = 0;
    float mean = 0;
    cpu_resample(series.data(), p, out, &n_steps, &mean);
    return py::make_tuple(py::array_t<float>(out.size(), out.data()), n_steps, mean);
  });
  m.def("wisdom_path", &wisdom_path);
  m.def("load_wisdom", [](const std::string& path, const std::string& arch, uint32_t M) {
    const PlanWisdom w = load_wisdom(path, arch, M);
    py::dict d;
    d["found"] = w.found;
    d["persist_per_cu"] = w.persist_per_cu;
    d["batch"] = w.batch;
    d["pipelines"] = w.pipelines;
    return d;
  });
  // n_steps of many templates: bracketed search (what the HIP engine uploads)
  // and the reference's descending scan
  m.def("n_steps", [](const py::dict& gd, py::array_t<float> P, py::array_t<float> tau, py::array_t<float> psi,
                      bool scan) {
    const SearchGeometry g = dict_to_geometry(gd);
    const size_t n = static_cast<size_t>(P.size());
    py::array_t<uint32_t> out(n);
    auto o = out.mutable_unchecked<1>();
    auto pp = P.unchecked<1>();
    auto tt = tau.unchecked<1>();
    auto ss = psi.unchecked<1>();
    for (size_t i = 0; i < n; ++i) {
      const ResampParams p = make_resamp_params(g.nsamples, g.n_unpadded, g.fft_size, g.dt, g.step_inv, pp(i), tt(i), ss(i));
      o(i) = scan ? resamp_n_steps_scan(p, kSinLut, kCosLut) : resamp_n_steps(p, kSinLut, kCosLut);
    }
    return out;
  }, py::arg("geometry"), py::arg("P"), py::arg("tau"), py::arg("psi"), py::arg("scan") = false);
  m.def("cpu_power_spectrum", [](py::array_t<float, py::array::c_style> x, uint32_t fft_size) {
    std::vector<float> v(x.data(), x.data() + x.size()), ps;
    cpu_power_spectrum(v, fft_size, ps);
    return py::array_t<float>(ps.size(), ps.data());
  });
  m.def("cpu_harmonic_sum", [](py::array_t<float, py::array::c_style> ps, const py::dict& gd, std::vector<float> thr) {
    const SearchGeometry g = dict_to_geometry(gd);
    std::vector<float> v(ps.data(), ps.data() + ps.size());
    std::vector<BinPower> out[5];
    std::vector<float> sumspec;
    cpu_harmonic_sum(v, g, thr.data(), out, &sumspec);
    TemplateCands tc;
    for (int h = 0; h < 5; ++h) tc.level[h] = out[h];
    py::array_t<float> ss({5, static_cast<int>(g.fundamental_idx_hi)});
    std::memcpy(ss.mutable_data(), sumspec.data(), sumspec.size() * sizeof(float));
    return py::make_tuple(cands_to_list({tc})[0], ss);
  });
  m.def("cpu_whiten", [](py::array_t<float, py::array::c_style> series, const py::dict& gd, const py::dict& od,
                         std::vector<std::pair<double, double>> zaps) {
    const SearchGeometry g = dict_to_geometry(gd);
    std::vector<float> v(series.data(), series.data() + series.size());
    std::vector<ZapRange> z;
    for (auto& p : zaps) z.push_back(ZapRange{p.first, p.second});
    check(cpu_whiten(v, g, dict_to_options(od), z), "cpu_whiten");
    return py::array_t<float>(v.size(), v.data());
  });
  m.def("zap_noise", [](int32_t seed, const py::dict& gd, const py::dict& od, std::vector<std::pair<double, double>> zaps) {
    std::vector<ZapRange> z;
    for (auto& p : zaps) z.push_back(ZapRange{p.first, p.second});
    ZapNoise n;
    make_zap_noise(seed, dict_to_geometry(gd), dict_to_options(od), z, n);
    return py::make_tuple(py::array_t<uint32_t>(n.bin.size(), n.bin.data()), py::array_t<float>(n.re.size(), n.re.data()),
                          py::array_t<float>(n.im.size(), n.im.data()));
  });

  // ---------------------------------------------------------------- HIP engine
  py::class_<HipEngine>(m, "HipEngine")
      .def(py::init<>())
      .def("init", [](HipEngine& e, int device, int batch) { check(e.init(device, batch), "HipEngine.init"); },
           py::arg("device") = -1, py::arg("batch") = 4)
      .def("setup",
           [](HipEngine& e, const py::dict& gd, py::array_t<float, py::array::c_style> series, float mu0) {
             std::vector<float> v(series.data(), series.data() + series.size());
             check(e.setup(dict_to_geometry(gd), v, mu0), "HipEngine.setup");
           })
      .def("setup_from_wu",
           [](HipEngine& e, const py::dict& gd, const std::string& path, float mu0) {
             WorkUnit wu;
             check(read_work_unit(path, wu), "read_work_unit");
             check(e.setup_packed(dict_to_geometry(gd), wu, mu0), "HipEngine.setup_packed");
             // the payload upload is queued from `wu`, which dies with this
             // scope: wait for it (the app pins and keeps its WU buffer instead)
             if (hipSetDevice(e.device()) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
               throw std::runtime_error("HipEngine.setup_from_wu: device synchronisation failed");
           })
      .def("download_series",
           [](HipEngine& e) {
             std::vector<float> v;
             check(e.download_series(v), "HipEngine.download_series");
             return py::array_t<float>(v.size(), v.data());
           })
      .def("whiten",
           [](HipEngine& e, const py::dict& od, std::vector<std::pair<double, double>> zaps,
              py::array_t<float, py::array::c_style> series) {
             std::vector<float> v(series.data(), series.data() + series.size());
             std::vector<ZapRange> z;
             for (auto& p : zaps) z.push_back(ZapRange{p.first, p.second});
             check(e.whiten(dict_to_options(od), z, v), "HipEngine.whiten");
             return py::array_t<float>(v.size(), v.data());
           })
      .def("process",
           [](HipEngine& e, py::array_t<float> P, py::array_t<float> tau, py::array_t<float> psi, std::vector<float> thr) {
             if (thr.size() < static_cast<size_t>(kNumHarmonicLevels))
               throw py::value_error("HipEngine.process: need one threshold per harmonic level (5)");
             auto t = arrays_to_templates(P, tau, psi);
             std::vector<TemplateCands> out;
             {
               py::gil_scoped_release rel;
               check(e.process(t.data(), static_cast<int>(t.size()), thr.data(), out), "HipEngine.process");
             }
             return cands_to_list(out);
           })
      .def("set_ps_fp16", [](HipEngine& e, bool on) { e.set_ps_fp16(on); })
      .def("submit",
           [](HipEngine& e, py::array_t<float> P, py::array_t<float> tau, py::array_t<float> psi, std::vector<float> thr) {
             if (thr.size() < static_cast<size_t>(kNumHarmonicLevels))
               throw py::value_error("HipEngine.submit: need one threshold per harmonic level (5)");
             auto t = arrays_to_templates(P, tau, psi);
             check(e.submit(t.data(), static_cast<int>(t.size()), thr.data(), 0), "HipEngine.submit");
           })
      .def("complete",
           [](HipEngine& e) {
             std::vector<TemplateCands> out;
             {
               py::gil_scoped_release rel;
               check(e.complete(out), "HipEngine.complete");
             }
             return cands_to_list(out);
           })
      .def("max_in_flight", &HipEngine::max_in_flight)
      .def("batch", &HipEngine::batch, "templates per submitted batch (launch-group size x BRP_SERIAL)")
      .def("adopt_series", [](HipEngine& e, const HipEngine& src) { check(e.adopt_series(src), "HipEngine.adopt_series"); })
      .def("power_spectrum",
           [](HipEngine& e, float P, float tau, float psi) {
             std::vector<float> ps;
             uint32_t n_steps = 0;
             check(e.power_spectrum(TemplateInput{P, tau, psi}, ps, &n_steps), "HipEngine.power_spectrum");
             return py::make_tuple(py::array_t<float>(ps.size(), ps.data()), n_steps);
           })
      .def("bound_cells",
           [](HipEngine& e, int k) {
             std::vector<float> c;
             check(e.bound_cells(k, c), "HipEngine.bound_cells");
             return py::array_t<float>(c.size(), c.data());
           })
      .def("benchmark_stages",
           [](HipEngine& e, py::array_t<float> P, py::array_t<float> tau, py::array_t<float> psi, int reps) {
             auto t = arrays_to_templates(P, tau, psi);
             std::vector<double> us;
             {
               py::gil_scoped_release rel;
               check(e.benchmark_stages(t.data(), static_cast<int>(t.size()), reps, us), "benchmark_stages");
             }
             py::dict d;
             const char* names[] = {"prologue", "pass1", "pass2", "pass3", "harmonic", "epilogue", "batch"};
             for (size_t i = 0; i < us.size(); ++i) d[names[i]] = us[i];
             return d;
           })
      .def("plan",
           [](HipEngine& e) {
             const FFTPlan3& p = e.plan();
             return py::make_tuple(p.M, p.L1, p.L2, p.L3);
           })
      .def("stats", [](HipEngine& e) {
        const BackendStats s = e.stats();
        py::dict d;
        d["busy_span_ms"] = s.busy_span_ms;
        d["whiten_ms"] = s.whiten_ms;
        d["templates"] = s.templates;
        d["batches"] = s.batches;
        d["overflow_reruns"] = s.overflow_reruns;
        d["tie_reruns"] = s.tie_reruns;
        d["select_batches"] = s.select_batches;
        d["list_dma_copies"] = s.list_dma_copies;
        d["shared_series_batches"] = s.shared_series_batches;
        d["peer_series_copies"] = s.peer_series_copies;
        return d;
      });
  m.def("fft_plan", [](uint32_t M) -> py::object {
    FFTPlan3 p;
    if (!make_fft_plan(M, p)) return py::none();
    return py::make_tuple(p.L1, p.L2, p.L3);
  });
  m.def("bluestein_plan", [](uint32_t Mb) -> py::object {
    FFTPlan3 p;
    if (!make_bluestein_plan(Mb, p)) return py::none();
    return py::make_tuple(p.M, p.L1, p.L2, p.L3);
  });

  // ---------------------------------------------------------------- driver
  m.def(
      "run_search",
      [](const py::dict& od, uint32_t begin, uint32_t end, bool write_output, bool use_checkpoint, int gpus,
         int pipelines, uint32_t progress_every) {
        SearchOptions opt = dict_to_options(od);
        SearchControl ctl;
        ctl.begin = begin;
        ctl.end = end;
        ctl.write_output = write_output;
        ctl.use_checkpoint = use_checkpoint;
        ctl.gpus = gpus;
        ctl.pipelines = std::max(1, pipelines);
        ctl.progress_every = std::max<uint32_t>(1, progress_every);
        SearchResult res;
        int rc;
        {
          py::gil_scoped_release rel;
          rc = run_search(opt, ctl, res);
        }
        check(rc, "run_search");
        py::dict d;
        d["table"] = res.table;
        d["geometry"] = geometry_to_dict(res.geom);
        d["templates_total"] = res.templates_total;
        d["templates_done"] = res.templates_done;
        d["templates_run"] = res.templates_run;
        d["interrupted"] = res.interrupted;
        d["t_setup"] = res.t_setup;
        d["t_templates"] = res.t_templates;
        d["t_total"] = res.t_total;
        d["busy_span_ms"] = res.stats.busy_span_ms;
        d["whiten_ms"] = res.stats.whiten_ms;
        d["overflow_reruns"] = res.stats.overflow_reruns;
        d["tie_reruns"] = res.stats.tie_reruns;
        d["select_batches"] = res.stats.select_batches;
        d["select_exits"] = res.stats.select_exits;
        return d;
      },
      py::arg("options"), py::arg("begin") = 0, py::arg("end") = 0, py::arg("write_output") = true,
      py::arg("use_checkpoint") = true, py::arg("gpus") = 1, py::arg("pipelines") = 1, py::arg("progress_every") = 1);
  py::class_<SearchSession>(m, "SearchSession")
      .def(py::init<>())
      .def(
          "open",
          [](SearchSession& s, const py::dict& od, int gpus, std::vector<int> devices) {
            SearchControl ctl;
            ctl.gpus = gpus;
            ctl.devices = devices;
            check(s.open(dict_to_options(od), ctl), "SearchSession.open");
          },
          py::arg("options"), py::arg("gpus") = 1, py::arg("devices") = std::vector<int>())
      .def("prepare",
           [](SearchSession& s) {
             int rc;
             {
               py::gil_scoped_release rel;
               rc = s.prepare();
             }
             check(rc, "SearchSession.prepare");
           })
      .def(
          "run",
          [](SearchSession& s, uint32_t begin, uint32_t end, CandidateTable table) {
            SearchResult res;
            int rc;
            {
              py::gil_scoped_release rel;
              rc = s.run(begin, end, table, res, nullptr);
            }
            check(rc, "SearchSession.run");
            py::dict d;
            d["templates_run"] = res.templates_run;
            d["dirty_pages"] = res.dirty_pages;
            return py::make_tuple(table, d);
          },
          py::arg("begin"), py::arg("end"), py::arg("table") = CandidateTable())
      .def("geometry", [](SearchSession& s) { return geometry_to_dict(s.geometry()); })
      .def("total", &SearchSession::total)
      .def("local_floors",
           [](const SearchSession& s) {
             float f[kNumHarmonicLevels];
             s.local_floors(f);
             return std::vector<float>(f, f + kNumHarmonicLevels);
           })
      .def("raise_external_floors",
           [](SearchSession& s, std::vector<float> f) {
             if (f.size() != static_cast<size_t>(kNumHarmonicLevels)) throw std::runtime_error("need 5 floors");
             s.raise_external_floors(f.data());
           })
      .def("reset_external_floors", &SearchSession::reset_external_floors)
      .def("stats", [](SearchSession& s) {
        const BackendStats st = s.stats();
        py::dict d;
        d["busy_span_ms"] = st.busy_span_ms;
        d["whiten_ms"] = st.whiten_ms;
        d["templates"] = st.templates;
        d["batches"] = st.batches;
        d["overflow_reruns"] = st.overflow_reruns;
        d["tie_reruns"] = st.tie_reruns;
        d["select_batches"] = st.select_batches;
        d["select_exits"] = st.select_exits;
        d["list_dma_copies"] = st.list_dma_copies;
        d["candidates"] = st.candidates;
        d["shared_series_batches"] = st.shared_series_batches;
        d["peer_series_copies"] = st.peer_series_copies;
        return d;
      });
  py::class_<MultiSession>(m, "MultiSession")
      .def(py::init<>())
      .def(
          "open",
          [](MultiSession& s, std::vector<std::string> inputs, const py::dict& od, int pipelines,
             std::vector<int> devices) {
            SearchControl ctl;
            ctl.gpus = pipelines;
            ctl.devices = devices;
            check(s.open(inputs, dict_to_options(od), ctl), "MultiSession.open");
          },
          py::arg("inputs"), py::arg("options"), py::arg("pipelines") = 1, py::arg("devices") = std::vector<int>())
      .def("prepare",
           [](MultiSession& s) {
             int rc;
             {
               py::gil_scoped_release rel;
               rc = s.prepare();
             }
             check(rc, "MultiSession.prepare");
           })
      .def(
          "run",
          [](MultiSession& s, uint32_t begin, uint32_t end, uint32_t block_batches) {
            std::vector<CandidateTable> tables;
            MultiResult res;
            int rc;
            {
              py::gil_scoped_release rel;
              s.set_block_batches(block_batches);
              rc = s.run(begin, end, tables, res);
            }
            check(rc, "MultiSession.run");
            py::dict d;
            d["pairs_run"] = res.pairs_run;
            d["t_templates"] = res.t_templates;
            return py::make_tuple(tables, d);
          },
          py::arg("begin") = 0, py::arg("end") = 0, py::arg("block_batches") = 0)
      .def("finalize",
           [](MultiSession& s, std::vector<std::string> outputs, uint32_t n_done, std::vector<CandidateTable> tables) {
             check(s.finalize(outputs, n_done, tables), "MultiSession.finalize");
           })
      .def("work_units", &MultiSession::work_units)
      .def("total", &MultiSession::total)
      .def("geometry", [](MultiSession& s) { return geometry_to_dict(s.geometry()); })
      .def("stats", [](MultiSession& s) {
        const BackendStats st = s.stats();
        py::dict d;
        d["busy_span_ms"] = st.busy_span_ms;
        d["whiten_ms"] = st.whiten_ms;
        d["templates"] = st.templates;
        d["batches"] = st.batches;
        d["candidates"] = st.candidates;
        d["overflow_reruns"] = st.overflow_reruns;
        d["tie_reruns"] = st.tie_reruns;
        d["select_batches"] = st.select_batches;
        d["shared_series_batches"] = st.shared_series_batches;
        return d;
      });
  m.def("finalize_output", [](const py::dict& od, const py::dict& gd, uint32_t n_done, CandidateTable t) {
    check(finalize_output(dict_to_options(od), dict_to_geometry(gd), n_done, t, "einsteinbinary_mi355x"),
          "finalize_output");
  });
  m.def("search_main", [](std::vector<std::string> args) {
    std::vector<char*> av;
    for (auto& s : args) av.push_back(const_cast<char*>(s.c_str()));
    av.push_back(nullptr);
    py::gil_scoped_release rel;
    return search_main(static_cast<int>(args.size()), av.data());
  });
  m.def("boinc_request_quit", &boinc::request_quit);
  m.def("boinc_clear_quit", &boinc::clear_quit);
  m.def("boinc_init", []() { return boinc::init(0, nullptr); });
  m.def("render_shmem_xml", []() { return ipc::render_xml(SearchInfo()); });
}
