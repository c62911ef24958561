// Exhaustive check: t / 0.001f == Markstein(t, y = RN(1/0.001f)) for every float t >= 0.5 with a
// finite quotient (mzh_signed_parabolic, csrc/mzh_device.h).  gcc -O2 -ffp-contract=off markstein_c.c -lm
#include <stdio.h>
#include <math.h>
#include <string.h>
#include <stdint.h>
int main(void) {
  const float b = 0.001000000047497451305389404296875f;
  const float y = 1.0f / b;
  uint32_t lo, hi; float f = 0.5f; memcpy(&lo, &f, 4); f = 3.4028234663852886e38f; memcpy(&hi, &f, 4);
  unsigned long long bad = 0, n = 0;
  for (uint32_t u = lo; u <= hi; ++u) {
    float t; memcpy(&t, &u, 4);
    float q = t * y;
    float r = fmaf(-q, b, t);
    float res = fmaf(r, y, q);
    float ref = t / b;
    if (memcmp(&res, &ref, 4) != 0 && !(isinf(ref))) { if (bad < 5) printf("mismatch t=%a res=%a ref=%a\n", t, res, ref); ++bad; }
    ++n;
  }
  printf("checked %llu, mismatches %llu, y=%a\n", n, bad, y);
  return 0;
}
