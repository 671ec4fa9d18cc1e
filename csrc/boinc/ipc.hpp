// Screensaver / progress telemetry in BOINC graphics shared memory
// (reference erp_boinc_ipc.{h,cpp}): 1024-byte area "EinsteinRadio" holding a
// <graphics_info> XML document, hand-formatted here (no libxml2).
#pragma once

#include <string>

#include "../core/formats.hpp"

namespace brp {
namespace ipc {

constexpr const char* kShmemAppName = "EinsteinRadio";
constexpr int kShmemSize = 1024;

int setup_shmem();
void update_shmem(const SearchInfo& info);
// XML document as it would be written (for tests)
std::string render_xml(const SearchInfo& info);
// rate limit for update_shmem (the reference updates every template)
bool update_due();

}  // namespace ipc
}  // namespace brp
