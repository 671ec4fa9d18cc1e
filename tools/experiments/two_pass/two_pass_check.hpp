// Host-side self-test of the two-pass plan's index algebra (fft_two_pass.hip):
// pass A's output positions form a permutation of a column and match tp_pos,
// the swizzled LDS block and the Stockham stages cover every element once,
// pass B's row tiles stay inside a column. Returns "" or what failed.
#pragma once

#include <string>

namespace brp {
namespace hipk {

std::string two_pass_selftest();

}  // namespace hipk
}  // namespace brp
