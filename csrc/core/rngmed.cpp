#include "rngmed.hpp"

#include <algorithm>
#include <cstring>
#include <vector>

namespace brp {

void running_median(const float* input, size_t length, size_t bsize, float* medians) {
  if (bsize == 0 || length < bsize) return;
  const bool odd = (bsize & 1) != 0;
  const size_t mid = (bsize + (bsize & 1)) / 2 - 1;
  std::vector<float> win(input, input + bsize);
  std::sort(win.begin(), win.end());
  auto median_of = [&]() -> float {
    if (odd) return win[mid];
    const float s = win[mid] + win[mid + 1];
    return static_cast<float>(static_cast<double>(s) / 2.0);
  };
  medians[0] = median_of();
  const size_t n_out = length - bsize + 1;
  for (size_t k = 1; k < n_out; ++k) {
    const float old_v = input[k - 1];
    const float new_v = input[k + bsize - 1];
    if (old_v == new_v) {
      medians[k] = medians[k - 1];
      continue;
    }
    // remove one instance of old_v
    auto it_old = std::lower_bound(win.begin(), win.end(), old_v);
    size_t pos_old = static_cast<size_t>(it_old - win.begin());
    // insertion point of new_v in the window without old_v
    auto it_new = std::upper_bound(win.begin(), win.end(), new_v);
    size_t pos_new = static_cast<size_t>(it_new - win.begin());
    if (pos_new > pos_old) {
      // shift (pos_old, pos_new) left by one, place new at pos_new-1
      std::memmove(&win[pos_old], &win[pos_old + 1], (pos_new - pos_old - 1) * sizeof(float));
      win[pos_new - 1] = new_v;
    } else {
      // shift [pos_new, pos_old) right by one, place new at pos_new
      std::memmove(&win[pos_new + 1], &win[pos_new], (pos_old - pos_new) * sizeof(float));
      win[pos_new] = new_v;
    }
    medians[k] = median_of();
  }
}

}  // namespace brp
