// tpe_device.hpp -- device helpers shared by the fit and scoring kernels.
#pragma once
#include <math.h>

#include "tpe_internal.hpp"

namespace tpe {

// numpy.maximum / numpy.minimum: NaN propagates from either side.
__device__ __forceinline__ double np_maximum(double a, double b) {
  if (a != a) return a;
  if (b != b) return b;
  return a >= b ? a : b;
}
__device__ __forceinline__ double np_minimum(double a, double b) {
  if (a != a) return a;
  if (b != b) return b;
  return a <= b ? a : b;
}

// normal_cdf, hyperopt/tpe.py:96-101 (no FMA contraction: bit-level parity).
__device__ __forceinline__ double normal_cdf(double x, double mu, double sigma) {
#pragma clang fp contract(off)
  const double bottom = np_maximum(1.4142135623730951 * sigma, kEPS);
  const double z = (x - mu) / bottom;
  return 0.5 * (1.0 + erf(z));
}

// Total order of numpy argsort on float64 as an unsigned key: ascending,
// -0.0 == +0.0, every NaN after +inf and equal to each other (ties are then
// broken by position by the callers, i.e. a stable sort).
__device__ __forceinline__ uint64_t sort_key(double v) {
  if (v != v) return ~0ull;
  if (v == 0.0) return 0x8000000000000000ull;
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

// (key, position) lexicographic order
__device__ __forceinline__ bool kp_less(uint64_t ka, uint32_t pa, uint64_t kb, uint32_t pb) {
  return ka < kb || (ka == kb && pa < pb);
}

}  // namespace tpe
