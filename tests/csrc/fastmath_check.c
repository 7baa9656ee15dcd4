/* Host check of the exact-division identities of kube-scheduler-simulator_amd/csrc/kss_fastmath.cuh
 * (TEST INFRASTRUCTURE).  Built and run by tests/test_fastmath.py with gcc -O2 -ffp-contract=off.
 * Each identity is evaluated with the same operation sequence the device uses and compared
 * with the plain division (integer floor / IEEE double division) over random and edge
 * operands; the float reciprocal of small_div is perturbed by +-1 ulp (v_rcp_f32 is not
 * correctly rounded).  Prints the number of mismatches per identity. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
  s += 0x9E3779B97F4A7C15ull;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static int32_t small_div(int32_t x, int32_t d, float rd) {  /* branch-free, as on the device */
  const int32_t q = (int32_t)((float)x * rd);
  const int64_t p = (int64_t)q * d;
  return q + (p + d <= (int64_t)x ? 1 : 0) - (p > (int64_t)x ? 1 : 0);
}

static int32_t quot_small_i64(int64_t x, int64_t A, double invA) {
  int32_t q = (int32_t)((double)x * invA);
  const int64_t r = x - (int64_t)q * A;
  if (r < 0) q--;
  else if (r >= A) q++;
  return q;
}

static double div_rn(int64_t ai, int64_t bi, double y) {
  const double a = (double)ai, b = (double)bi;
  double q = a * y;
  double r = fma(-q, b, a);
  q = fma(r, y, q);
  r = fma(-q, b, a);
  return fma(r, y, q);
}

static int32_t quot_small_d(double x, double A, double invA) {
  int32_t q = (int32_t)(x * invA);
  const double r = fma(-(double)q, A, x);
  if (r < 0.0) q--;
  else if (r >= A) q++;
  return q;
}

/* least_bf (kss_simple.cuh): leastRequestedScore, branch-free, capacity > 0 */
static int32_t least_bf(double requested, double capacity, double inv) {
  const int over = requested > capacity;
  const double x = (capacity - (over ? capacity : requested)) * 100.0;
  int32_t q = (int32_t)(x * inv);
  const double r = fma(-(double)q, capacity, x);
  q += (r >= capacity ? 1 : 0) - (r < 0.0 ? 1 : 0);
  return over ? 0 : q;
}

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 1000000;
  long bad_small = 0, bad_quot = 0, bad_div = 0;
  /* small_div: x = 100 * v, v <= d (normalisation), and x <= 100 * d (Fit weight average) */
  for (long i = 0; i < n; i++) {
    int32_t d = 1 + (int32_t)(rnd() % ((i & 1) ? 65535 : (4u << 20)));
    int32_t x = (int32_t)(rnd() % ((uint64_t)100 * d + 1));
    if (x < 0) continue;
    float r0 = 1.0f / (float)d;
    float rs[3] = {r0, nextafterf(r0, 0.0f), nextafterf(r0, 1.0f)};
    for (int k = 0; k < 3; k++)
      if (small_div(x, d, rs[k]) != x / d) bad_small++;
  }
  /* quot_small_i64: x = (A - R) * 100 or R * 100, 0 <= R <= A < 2^46 */
  for (long i = 0; i < n; i++) {
    int bits = 1 + (int)(rnd() % 46);
    int64_t A = 1 + (int64_t)(rnd() % ((1ull << bits) - 1));
    int64_t R = (int64_t)(rnd() % (uint64_t)(A + 1));
    int64_t x = (i & 1) ? (A - R) * 100 : R * 100;
    if (quot_small_i64(x, A, 1.0 / (double)A) != x / A) bad_quot++;
    if (quot_small_d((double)x, (double)A, 1.0 / (double)A) != x / A) bad_quot++;
    /* requested in [0, 2A]: over-capacity requests score 0 */
    int64_t Rq = (int64_t)(rnd() % (uint64_t)(2 * A + 1));
    int32_t want = Rq > A ? 0 : (int32_t)((A - Rq) * 100 / A);
    if (least_bf((double)Rq, (double)A, 1.0 / (double)A) != want) bad_quot++;
  }
  /* div_rn: 0 <= a < 2^53, 1 <= b < 2^46 (requested / allocatable, either order of size) */
  for (long i = 0; i < n; i++) {
    int bb = 1 + (int)(rnd() % 46), ab = 1 + (int)(rnd() % 53);
    int64_t b = 1 + (int64_t)(rnd() % ((1ull << bb) - 1));
    int64_t a = (int64_t)(rnd() % (1ull << ab));
    if ((i & 3) == 0) a = (int64_t)(rnd() % (uint64_t)(b + 1));          /* fraction <= 1 */
    if ((i & 7) == 1) b = (int64_t)((1ull << bb) - 1);                  /* all-ones mantissa divisors */
    double want = (double)a / (double)b;
    double got = div_rn(a, b, 1.0 / (double)b);
    if (got != want) bad_div++;
  }
  printf("%ld %ld %ld\n", bad_small, bad_quot, bad_div);
  return 0;
}
