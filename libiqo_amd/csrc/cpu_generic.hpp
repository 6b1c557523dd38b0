// cpu_generic.hpp -- the drop-in classes' CPU backend (cpu_generic.cpp): the host plan's records
// applied with the reference's Generic per-pixel formulas, output rows split over threads.
#pragma once

#include <cstddef>
#include <cstdint>

#include "plan.hpp"

namespace iqo_amd {

// One frame, host pointers, byte strides.  threads <= 0: std::thread::hardware_concurrency().
void cpu_resize(const Plan &p, size_t srcSt, const uint8_t *src, size_t dstSt, uint8_t *dst, int threads = 0);

} // namespace iqo_amd
