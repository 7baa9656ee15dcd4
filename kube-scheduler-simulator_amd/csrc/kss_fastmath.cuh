// kss_fastmath.cuh — exact integer and IEEE-double divisions for the scoring hot loop,
// without the general division sequences.
//
// The scores of the reference are Go int64 divisions (LeastAllocated / MostAllocated,
// DefaultNormalizeScore, the Fit weight average) and IEEE float64 divisions
// (BalancedAllocation, balanced_allocation.go balancedResourceScorer).  The divisors are
// either per node and constant for a launch (Allocatable) or per pod and uniform
// (normalisation maxima, the Fit weight sum), so a reciprocal is computed once and every
// division becomes a multiply plus an exact correction:
//
//   * integer quotients whose value is at most ~100: an estimate from the reciprocal is
//     within +-1 of floor(x / d) (its relative error is below 2^-20, the quotient below
//     2^7), and one integer compare in each direction makes it exact;
//   * float64 quotients: with y = RN(1/b) (correctly rounded, computed by an IEEE
//     division), q0 = RN(a*y) is within 1.5 ulp of a/b; one FMA residual step makes it
//     faithful, and a second is the correctly rounded quotient by Markstein's theorem
//     (y within 1/2 ulp of 1/b, q faithful => RN(q + (a - b q) y) = RN(a/b)).  Every
//     operand is an integer below 2^53, so a and b convert exactly.  explicit fma() is an
//     IEEE operation and is unaffected by -ffp-contract=off.
// tests/test_fastmath.py checks both identities on the host against the plain
// divisions over the value ranges the device path admits.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kss {

// floor(x / d) for 0 <= x, 0 < d, x / d <= ~2^7 and d, x < 2^31 (the estimate's
// error bound needs only the small quotient; x may exceed 2^24).  rd = rcp(d).
// Branch-free: with d > 0 at most one of the two corrections applies.
__device__ __forceinline__ int32_t small_div(int32_t x, int32_t d, float rd) {
  const int32_t q = (int32_t)((float)x * rd);
  const int64_t p = (int64_t)q * d;
  return q + (p + d <= (int64_t)x ? 1 : 0) - (p > (int64_t)x ? 1 : 0);
}

// floor(x / A) for 0 <= x < 2^53, 0 < A < 2^53, x / A <= ~2^7; invA = RN(1 / (double)A).
__device__ __forceinline__ int32_t quot_small_i64(int64_t x, int64_t A, double invA) {
  int32_t q = (int32_t)((double)x * invA);
  const int64_t r = x - (int64_t)q * A;
  if (r < 0) q--;
  else if (r >= A) q++;
  return q;
}

// RN(a / b) for integers 0 <= a, 0 < b < 2^53, y = RN(1 / (double)b).
__device__ __forceinline__ double div_rn(int64_t ai, int64_t bi, double y) {
  const double a = (double)ai, b = (double)bi;
  double q = a * y;
  double r = fma(-q, b, a);
  q = fma(r, y, q);
  r = fma(-q, b, a);
  return fma(r, y, q);
}

// The same on integers held in doubles (every value an integer below 2^53, so exact):
// the compact kernel keeps node state and pod requests as doubles, which removes the
// int64 <-> double conversions from the loop.
__device__ __forceinline__ int32_t quot_small_d(double x, double A, double invA) {
  int32_t q = (int32_t)(x * invA);
  const double r = fma(-(double)q, A, x);  // q * A and x are integers below 2^53: exact
  if (r < 0.0) q--;
  else if (r >= A) q++;
  return q;
}

__device__ __forceinline__ double div_rn_d(double a, double b, double y) {
  double q = a * y;
  double r = fma(-q, b, a);
  q = fma(r, y, q);
  r = fma(-q, b, a);
  return fma(r, y, q);
}

__device__ __forceinline__ int32_t alloc_score_d(int strategy, double requested, double capacity, double inv) {
  if (strategy == KSS_FIT_MOST_ALLOCATED) {
    if (requested > capacity) requested = capacity;
    return quot_small_d(requested * 100.0, capacity, inv);
  }
  if (requested > capacity) return 0;
  return quot_small_d((capacity - requested) * 100.0, capacity, inv);
}

// leastRequestedScore / mostRequestedScore (noderesources/least_allocated.go,
// most_allocated.go) for 0 < capacity < 2^46: quotient in [0, 100].
__device__ __forceinline__ int32_t alloc_score_fast(int strategy, int64_t requested, int64_t capacity, double inv) {
  if (strategy == KSS_FIT_MOST_ALLOCATED) {
    if (requested > capacity) requested = capacity;
    return quot_small_i64(requested * 100, capacity, inv);
  }
  if (requested > capacity) return 0;
  return quot_small_i64((capacity - requested) * 100, capacity, inv);
}

}  // namespace kss
