/* oracle/check_logf.c -- pins oc_logf to the host glibc (TEST INFRASTRUCTURE): every positive
 * float (and the special values) bit-exactly against libm logf. Exit status 0 iff no mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "orb_oracle.h"

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

int main(void) {
  long long bad = 0;
  unsigned long long sum = 0;
#pragma omp parallel for reduction(+ : bad, sum) schedule(static, 1 << 16)
  for (long long i = 0; i <= 0x7f800000LL; i++) {
    const float x = u2f((uint32_t)i);
    const uint32_t a = f2u(logf(x)), b = f2u(oc_logf(x));
    bad += a != b;
    sum += b;
  }
  printf("{\"n\": %lld, \"logf_mismatch\": %lld, \"checksum\": %llu}\n", 0x7f800001LL, bad, sum);
  return bad ? 1 : 0;
}
