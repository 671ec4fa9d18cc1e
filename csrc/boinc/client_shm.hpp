// Layout of the app <-> BOINC client shared memory ("boinc_mmap_file" in the
// slot directory) and its message channels.
//
// The reference links libboinc_api, which attaches this segment in
// boinc_init_options() (called from erp_boinc_init, erp_boinc_ipc.cpp:206-208)
// and services it from a timer. The segment is eight fixed 1024-byte channels;
// byte 0 of a channel is the "full" flag and the NUL-terminated XML message
// follows it. A sender only writes into an empty channel; the receiver copies
// the text out and clears the flag. The client writes heartbeat and
// process-control requests, the app writes its status.
//
// No BOINC client or libboinc source is available here: the layout follows the
// documented channel protocol and its parity with a real client is unpinned
// (tests/test_boinc_client_cpu.py drives it with an in-repo fake client).
#pragma once

#include <cstddef>
#include <cstring>

namespace brp {
namespace boinc {

constexpr size_t kMsgChannelSize = 1024;
constexpr const char* kMmapFileName = "boinc_mmap_file";
constexpr const char* kFinishCalledFile = "boinc_finish_called";
constexpr const char* kTemporaryExitFile = "boinc_temporary_exit";
constexpr const char* kLockFile = "boinc_lockfile";
constexpr int kExitAbortedByClient = 194;

struct MsgChannel {
  char buf[kMsgChannelSize];

  bool has_msg() const { return buf[0] != 0; }
  // copy the pending message (if any) into msg and mark the channel empty
  bool get_msg(char* msg) {
    if (!buf[0]) return false;
    std::strncpy(msg, buf + 1, kMsgChannelSize - 1);
    msg[kMsgChannelSize - 1] = 0;
    __atomic_store_n(&buf[0], 0, __ATOMIC_RELEASE);
    return true;
  }
  // post msg if the channel is empty (the reader consumed the previous one)
  bool send_msg(const char* msg) {
    if (__atomic_load_n(&buf[0], __ATOMIC_ACQUIRE)) return false;
    std::strncpy(buf + 1, msg, kMsgChannelSize - 2);
    buf[kMsgChannelSize - 1] = 0;
    __atomic_store_n(&buf[0], 1, __ATOMIC_RELEASE);
    return true;
  }
};

// Channel order is part of the protocol.
struct SharedMem {
  MsgChannel process_control_request;  // client -> app: <quit/> <suspend/> <resume/> <abort/>
  MsgChannel process_control_reply;
  MsgChannel graphics_request;
  MsgChannel graphics_reply;
  MsgChannel heartbeat;                // client -> app: <heartbeat/> [<wss>..] every second
  MsgChannel app_status;               // app -> client: cpu times, fraction_done
  MsgChannel trickle_up;
  MsgChannel trickle_down;
};
static_assert(sizeof(SharedMem) == 8 * kMsgChannelSize, "eight 1 KB channels");
static_assert(offsetof(SharedMem, heartbeat) == 4 * kMsgChannelSize, "channel order");
static_assert(offsetof(SharedMem, app_status) == 5 * kMsgChannelSize, "channel order");

}  // namespace boinc
}  // namespace brp
