// On-disk / shared-memory formats of the BRP search.
//
// Byte-compatible with the reference's packed structs (reference structs.h:40-161):
//   DD_Header  (work-unit header)      1168 B   structs.h:74-105
//   CP_Header  (checkpoint header)      260 B   structs.h:111-115
//   CP_Cand    (checkpoint candidate)    48 B   structs.h:121-130
// Everything is little-endian on disk; big-endian hosts swap on read
// (reference demod_binary.c:674-703).
#pragma once

#include <cstddef>
#include <cstdint>

namespace brp {

constexpr int kFnLength = 256;        // FN_LENGTH, structs.h:32
constexpr int kBinsScreensaver = 40;  // N_BINS_SS, structs.h:33
constexpr double kMicrosec = 1.0e-6;  // MICROSEC, structs.h:34
constexpr int kNumHarmonicLevels = 5; // 1,2,4,8,16 summed harmonics
constexpr int kCandPerLevel = 100;    // N_CAND_5, demod_binary.c:83
constexpr int kCandTotal = 500;       // N_CAND, demod_binary.c:84
constexpr int kLogPsPageSize = 10;    // LOG_PS_PAGE_SIZE, hs_common.h:36

#pragma pack(push, 1)
struct DDHeader {
  double tsample;     // sample time [us]
  double tobs;        // observation time [s]
  double timestamp;   // MJD
  double fcenter;     // MHz
  double fchan;       // kHz
  double RA;          // hhmmss.s (J2000)
  double DEC;         // ddmmss.s (J2000)
  double gal_l;
  double gal_b;
  double AZstart;
  double ZAstart;
  double ASTstart;
  double LSTstart;
  double DM;          // trial dispersion measure [pc cm^-3]
  double scale;       // packed value v represents v/scale
  uint32_t filesize;
  uint32_t datasize;
  uint32_t nsamples;  // number of (unpadded) samples
  uint16_t smprec;
  uint16_t nchan;
  uint16_t nifs;
  uint16_t lagformat;
  uint16_t sum;
  uint16_t level;
  char name[kFnLength];
  char originalfile[kFnLength];
  char proj_id[kFnLength];
  char observers[kFnLength];
};

struct CPHeader {
  uint32_t n_template;            // number of templates completed
  char originalfile[kFnLength];   // input file name the checkpoint belongs to
};

struct CPCand {
  double power;    // summed power (before the final /sqrt(N_h))
  double P_b;      // orbital period [s]
  double tau;      // projected orbital radius [lt-s]
  double Psi;      // initial orbital phase [rad]
  double fA;       // -log10 false alarm probability (final stage only)
  uint32_t n_harm; // number of summed harmonics (1,2,4,8,16), 0 = empty slot
  uint32_t f0;     // frequency bin
};
#pragma pack(pop)

static_assert(sizeof(DDHeader) == 1168, "DDHeader must be byte-compatible (1168 B)");
static_assert(sizeof(CPHeader) == 260, "CPHeader must be byte-compatible (260 B)");
static_assert(sizeof(CPCand) == 48, "CPCand must be byte-compatible (48 B)");
static_assert(offsetof(DDHeader, nsamples) == 128, "DDHeader layout");
static_assert(offsetof(CPCand, n_harm) == 40, "CPCand layout");

// Screensaver / progress telemetry (reference erp_boinc_ipc.h:36-44).
struct SearchInfo {
  double skypos_rac = 0;
  double skypos_dec = 0;
  double dispersion_measure = 0;
  double orbital_radius = 0;
  double orbital_period = 0;
  double orbital_phase = 0;
  unsigned char power_spectrum[kBinsScreensaver] = {0};
};

bool host_is_big_endian();
void endian_swap(uint8_t* data, size_t elem_size, size_t n);
void swap_header(DDHeader& h);

}  // namespace brp
