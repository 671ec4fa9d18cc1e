// Running median over a window of `bsize` samples (reference rngmed.c:48-341,
// Mohanty's algorithm). Output medians[k] = median(input[k .. k+bsize-1]) for
// k < length-bsize+1; for even bsize the two middle order statistics are
// averaged as (a+b)/2 with the sum rounded to float first, like the reference.
// Any exact order-statistic algorithm is bit-identical, so the CPU path uses
// a sorted window and the GPU path (csrc/hip/whiten.hip) a blocked LDS select.
#pragma once

#include <cstddef>

namespace brp {

void running_median(const float* input, size_t length, size_t bsize, float* medians);

}  // namespace brp
