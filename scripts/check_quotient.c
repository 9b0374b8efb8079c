/* The compact xT iteration (xt_iter_ell_kernel, SA_XE_QDIV) forms cnt / move as
 *   r = RN(1 / move), y = RN(cnt * r), T = RN(y + r * RN(cnt - y * move))  (two fmas)
 * and relies on T == RN(cnt / move), the IEEE quotient the reference's numpy division gives.
 * This checks it on the host: every cnt < 65536 against divisors 1..D and 2^40 - D/2 .. 2^40 +
 * D/2, then N random (cnt, move) pairs (cnt up to 2^31, move up to 2^53, all-ones divisors).
 * The xT binning (bin_quot, sa_common.h) forms x / 105 and y / 68 the same way with the constant
 * reciprocal: checked on N random doubles per divisor, over 2^-960..2^960 with random signs and
 * uniform in [0, 128).
 * Prints "n=<checked> bad=<mismatches>", exits 1 on a mismatch.
 *   gcc -O2 -mfma -ffp-contract=off scripts/check_quotient.c -lm && ./a.out [D] [N] */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t rs = 88172645463325252ull;
static uint64_t xr(void) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return rs;
}
static long long n_checked, n_bad;
static void check(double q, double m) {  /* q / m as the kernels form it == IEEE q / m */
  const double r = 1.0 / m, y = q * r, t = fma(fma(-y, m, q), r, y);
  ++n_checked;
  if (t != q / m && n_bad++ < 10) printf("mismatch q=%.17g m=%.17g got %.17g want %.17g\n", q, m, t, q / m);
}
int main(int argc, char** argv) {
  const long long D = argc > 1 ? atoll(argv[1]) : 6000, N = argc > 2 ? atoll(argv[2]) : 400000000LL;
  for (long long m = 1; m <= D; ++m)
    for (uint32_t q = 0; q < 65536; ++q) check(q, (double)m);
  for (long long m = (1ll << 40) - D / 2; m <= (1ll << 40) + D / 2; ++m)
    for (uint32_t q = 0; q < 65536; ++q) check(q, (double)m);
  for (long long it = 0; it < N; ++it) {
    uint64_t m;
    switch (it % 4) {
      case 0: m = 1 + xr() % 1000; break;
      case 1: m = 1 + xr() % 1000000; break;
      case 2: m = 1 + (xr() >> (11 + xr() % 40)); break;
      default: m = (1ull << (1 + xr() % 52)) - 1 - xr() % 3; if (!m) m = 1;
    }
    uint32_t q = 1 + (uint32_t)(xr() % ((it & 1) ? 65535u : 256u));
    if ((it & 7) == 3) q = 1 + (uint32_t)(xr() % 2147483647u);
    check(q, (double)m);
  }
  const double field[2] = {105.0, 68.0};
  for (int f = 0; f < 2; ++f)
    for (long long it = 0; it < N; ++it) {
      double x;
      if (it & 1) {
        x = (double)(xr() >> 11) * 0x1p-53 * 128.0;
      } else {
        const uint64_t u = (xr() & 0x000FFFFFFFFFFFFFull) | ((uint64_t)(63 + xr() % 1920) << 52);
        memcpy(&x, &u, 8);
        if (xr() & 1) x = -x;
      }
      check(x, field[f]);
    }
  printf("n=%lld bad=%lld\n", n_checked, n_bad);
  return n_bad != 0;
}
