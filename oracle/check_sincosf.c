/* oracle/check_sincosf.c -- pins oc_sinf/oc_cosf to the host glibc (TEST INFRASTRUCTURE).
 * Compares every float in [lo, hi) (default [0, 2pi): the range of ORB keypoint angles in
 * radians, orb_extractor.cpp:53) bit-exactly against libm sinf/cosf and prints the mismatch
 * counts and a checksum of all outputs. Exit status 0 iff no mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

int main(int argc, char** argv) {
  float lo = argc > 1 ? strtof(argv[1], NULL) : 0.0f;
  float hi = argc > 2 ? strtof(argv[2], NULL) : 6.28318548f;
  uint32_t a = f2u(lo), b = f2u(hi);
  long long bad_s = 0, bad_c = 0;
  unsigned long long sum = 0;
#pragma omp parallel for reduction(+ : bad_s, bad_c, sum) schedule(static, 1 << 16)
  for (long long i = (long long)a; i < (long long)b; i++) {
    float x = u2f((uint32_t)i);
    float s0 = sinf(x), c0 = cosf(x), s1 = oc_sinf(x), c1 = oc_cosf(x);
    bad_s += f2u(s0) != f2u(s1);
    bad_c += f2u(c0) != f2u(c1);
    sum += (unsigned long long)f2u(s1) * 3u + f2u(c1);
  }
  printf("{\"n\": %lld, \"sin_mismatch\": %lld, \"cos_mismatch\": %lld, \"checksum\": %llu}\n",
         (long long)b - (long long)a, bad_s, bad_c, sum);
  return (bad_s || bad_c) ? 1 : 0;
}
