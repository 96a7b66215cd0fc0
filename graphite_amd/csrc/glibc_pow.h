// glibc_pow.h -- pow(), bit-exact with the reference's pow on x86-64: glibc
// 2.35's __pow_fma (sysdeps/ieee754/dbl-64/e_pow.c, the ARM optimized-routines
// algorithm, compiled with -mfma -mavx2 and picked by the ifunc on any CPU with
// FMA + AVX2), and the x86-64 (uint64_t) conversion of a double.
//
// Why: MovingGeometricMean::compute (moving_average.h:119-135) keeps its mean as
// a chain of pow() results, and (T) _geometric_mean truncates it, so one last-bit
// difference of pow moves a queue's reference time.  ROCm's device pow differs
// from glibc's in the last bit on many operands, so the engine carries glibc's:
//   * the same algorithm: log_inline (a 128-entry table, a degree-7 polynomial in
//     double-double), y * log(x) split into hi + lo, exp_inline (128-entry 2^(i/N)
//     table, degree-5 polynomial), specialcase for results near the overflow /
//     subnormal ranges, and e_pow.c's special operands (zero, inf, nan, x < 0,
//     tiny or huge y);
//   * the same FMA contraction as __pow_fma: every fma below is one the x86 build
//     fuses (read off its disassembly), and nothing else is fused -- this header
//     is compiled with -ffp-contract=off (libgnoc.so and the host test alike);
//   * the same tables (pow_tables.h, generated from this image's libm by
//     tools/gen_pow_tables.py).
// tests/cpp/test_pow.cc checks pow() against glibc's on the host over random and
// special operands, and to_u64_x86 against gcc's cast.
//
// Upstream notice.  This header restates the algorithm, constants and operation
// order of glibc 2.35 sysdeps/ieee754/dbl-64/e_pow.c and e_exp_data.c /
// e_pow_log_data.c: "Copyright (C) 2018-2022 Free Software Foundation, Inc.
// This file is part of the GNU C Library", distributed under the GNU Lesser
// General Public License, version 2.1 or (at your option) any later version.
// glibc took the algorithm from Arm's optimized-routines (Copyright (c) 2018,
// Arm Limited; MIT OR Apache-2.0 WITH LLVM-exception).  Those terms apply to
// this restatement and to pow_tables.h.
//
// Exactness holds against THAT pow: the reference's std::pow on an x86-64 host
// whose glibc 2.35 ifunc picks __pow_fma (FMA + AVX2).  A host without FMA, or
// another libm, runs another last-bit-inexact routine; geometric-mean results
// computed there are not pinned by this header.
#pragma once

#include <cstdint>

#include "pow_tables.h"

namespace gnoc {
namespace gpow {

__host__ __device__ __forceinline__ uint64_t asu(double x) { return __builtin_bit_cast(uint64_t, x); }
__host__ __device__ __forceinline__ double asd(uint64_t x) { return __builtin_bit_cast(double, x); }
__host__ __device__ __forceinline__ uint32_t top12(double x) { return (uint32_t) (asu(x) >> 52); }

constexpr uint64_t OFF = 0x3fe6955500000000ull;   // log table: z in [0x1.69555p-1, 0x1.69555p0)
constexpr uint32_t SIGN_BIAS = 0x800u << 7;        // exp_inline: negative result
constexpr uint64_t INF_BITS = 0x7ff0000000000000ull;
constexpr uint64_t ONE_BITS = 0x3ff0000000000000ull;

__host__ __device__ __forceinline__ double oflow(uint32_t sign)
{
   const double y = sign ? -0x1p769 : 0x1p769;
   return y * 0x1p769;
}
__host__ __device__ __forceinline__ double uflow(uint32_t sign)
{
   const double y = sign ? -0x1p-767 : 0x1p-767;
   return y * 0x1p-767;
}
__host__ __device__ __forceinline__ double divzero(uint32_t sign)
{
   const double y = sign ? -1.0 : 1.0;
   return y / 0.0;
}
__host__ __device__ __forceinline__ double invalid(double x) { return (x - x) / (x - x); }
__host__ __device__ __forceinline__ bool zeroinfnan(uint64_t i) { return 2 * i - 1 >= 2 * INF_BITS - 1; }
__host__ __device__ __forceinline__ bool issignaling(double x)
{
   const uint64_t ix = asu(x);
   return 2 * (ix ^ 0x0008000000000000ull) > 2 * 0x7ff8000000000000ull;
}
// 0: not an integer, 1: odd integer, 2: even integer
__host__ __device__ __forceinline__ int checkint(uint64_t iy)
{
   const int e = (int) (iy >> 52 & 0x7ff);
   if (e < 0x3ff) return 0;
   if (e > 0x3ff + 52) return 2;
   if (iy & ((1ull << (0x3ff + 52 - e)) - 1)) return 0;
   if (iy & (1ull << (0x3ff + 52 - e))) return 1;
   return 2;
}

// log(x) = hi + tail for x = ix (positive, normal).
__host__ __device__ __forceinline__ double log_inline(uint64_t ix, double& tail)
{
   const uint64_t tmp = ix - OFF;
   const uint32_t i = (uint32_t) ((tmp >> 45) % 128u);
   const int k = (int) ((int64_t) tmp >> 52);
   const uint64_t iz = ix - (tmp & (0xfffull << 52));
   const double z = asd(iz);
   const double kd = (double) k;
   const double invc = LOG_TAB[3 * i], logc = LOG_TAB[3 * i + 1], logctail = LOG_TAB[3 * i + 2];
   const double r = __builtin_fma(z, invc, -1.0);
   const double t1 = __builtin_fma(kd, LN2HI, logc);
   const double t2 = t1 + r;
   const double lo1 = __builtin_fma(kd, LN2LO, logctail);
   const double lo2 = t1 - t2 + r;
   const double ar = LOG_POLY[0] * r;
   const double ar2 = r * ar;
   const double ar3 = r * ar2;
   const double hi = t2 + ar2;
   const double lo3 = __builtin_fma(ar, r, -ar2);
   const double lo4 = t2 - hi + ar2;
   // p = ar3 * (A1 + r A2 + ar2 (A3 + r A4 + ar2 (A5 + r A6))), fused into the sum
   const double q56 = __builtin_fma(r, LOG_POLY[6], LOG_POLY[5]);
   const double q36 = __builtin_fma(ar2, q56, __builtin_fma(r, LOG_POLY[4], LOG_POLY[3]));
   const double q16 = __builtin_fma(ar2, q36, __builtin_fma(r, LOG_POLY[2], LOG_POLY[1]));
   const double lo = __builtin_fma(ar3, q16, lo1 + lo2 + lo3 + lo4);
   const double y = hi + lo;
   tail = hi - y + lo;
   return y;
}

__host__ __device__ __forceinline__ double specialcase(double tmp, uint64_t sbits, uint64_t ki)
{
   if ((ki & 0x80000000u) == 0)
   {
      // k > 0: the exponent of scale may have overflowed by <= 460
      sbits -= 1009ull << 52;
      const double scale = asd(sbits);
      return 0x1p1009 * __builtin_fma(scale, tmp, scale);
   }
   // k < 0: rounded once before scaling into the subnormal range
   sbits += 1022ull << 52;
   const double scale = asd(sbits);
   const double st = scale * tmp;   // used twice: not fused
   double y = scale + st;
   if ((y < 0 ? -y : y) < 1.0)
   {
      const double one = y < 0.0 ? -1.0 : 1.0;
      double lo = scale - y + st;
      const double hi = one + y;
      lo = one - hi + y + lo;
      y = (hi + lo) - one;
      if (y == 0) y = asd(sbits & 0x8000000000000000ull);
   }
   return 0x1p-1022 * y;
}

// exp(x + xtail), negated when sign_bias is set.
__host__ __device__ __forceinline__ double exp_inline(double x, double xtail, uint32_t sign_bias)
{
   uint32_t abstop = top12(x) & 0x7ff;
   if (abstop - 0x3c9u >= 0x408u - 0x3c9u)
   {
      if (abstop - 0x3c9u >= 0x80000000u)
      {
         // tiny x (0 included)
         const double one = 1.0 + x;
         return sign_bias ? -one : one;
      }
      if (abstop >= 0x409u) return (asu(x) >> 63) ? uflow(sign_bias) : oflow(sign_bias);
      abstop = 0;   // large x: specialcase below
   }
   double kd = __builtin_fma(x, EXP_INVLN2N, EXP_SHIFT);
   const uint64_t ki = asu(kd);
   kd -= EXP_SHIFT;
   double r = __builtin_fma(kd, EXP_NEGLN2LON, __builtin_fma(kd, EXP_NEGLN2HIN, x));
   r = xtail + r;
   const uint32_t idx = 2u * (uint32_t) (ki % 128u);
   const uint64_t top = (ki + sign_bias) << 45;
   const double tail = asd(EXP_TAB[idx]);
   const uint64_t sbits = EXP_TAB[idx + 1] + top;
   const double r2 = r * r;
   const double tmp = __builtin_fma(r2 * r2, __builtin_fma(r, EXP_C[3], EXP_C[2]),
                                    __builtin_fma(r2, __builtin_fma(r, EXP_C[1], EXP_C[0]), tail + r));
   if (abstop == 0) return specialcase(tmp, sbits, ki);
   const double scale = asd(sbits);
   return __builtin_fma(scale, tmp, scale);
}

__host__ __device__ inline double pow(double x, double y)
{
   uint32_t sign_bias = 0;
   uint64_t ix = asu(x);
   const uint64_t iy = asu(y);
   uint32_t topx = top12(x);
   const uint32_t topy = top12(y);
   if (topx - 0x001u >= 0x7feu || (topy & 0x7ff) - 0x3beu >= 0x80u)
   {
      if (zeroinfnan(iy))
      {
         if (2 * iy == 0) return issignaling(x) ? x + y : 1.0;
         if (ix == ONE_BITS) return issignaling(y) ? x + y : 1.0;
         if (2 * ix > 2 * INF_BITS || 2 * iy > 2 * INF_BITS) return x + y;
         if (2 * ix == 2 * ONE_BITS) return 1.0;
         if ((2 * ix < 2 * ONE_BITS) == !(iy >> 63)) return 0.0;   // |x| < 1 and y = inf, or |x| > 1 and y = -inf
         return y * y;
      }
      if (zeroinfnan(ix))
      {
         double x2 = x * x;
         if ((ix >> 63) && checkint(iy) == 1)
         {
            x2 = -x2;
            sign_bias = 1;
         }
         if (2 * ix == 0 && (iy >> 63)) return divzero(sign_bias);
         return (iy >> 63) ? 1 / x2 : x2;
      }
      // x and y are finite and non-zero
      if (ix >> 63)
      {
         const int yint = checkint(iy);
         if (yint == 0) return invalid(x);
         if (yint == 1) sign_bias = SIGN_BIAS;
         ix &= 0x7fffffffffffffffull;
         topx &= 0x7ff;
      }
      if ((topy & 0x7ff) - 0x3beu >= 0x80u)
      {
         if (ix == ONE_BITS) return 1.0;
         if ((topy & 0x7ff) < 0x3beu) return ix > ONE_BITS ? 1.0 + y : 1.0 - y;   // |y| tiny
         return (ix > ONE_BITS) == (topy < 0x800u) ? oflow(0) : uflow(0);
      }
      if (topx == 0)
      {
         // subnormal x: normalise so the exponent becomes negative
         ix = asu(x * 0x1p52);
         ix &= 0x7fffffffffffffffull;
         ix -= 52ull << 52;
      }
   }
   double lo;
   const double hi = log_inline(ix, lo);
   const double ehi = y * hi;
   const double elo = __builtin_fma(y, lo, __builtin_fma(y, hi, -ehi));
   return exp_inline(ehi, elo, sign_bias);
}

// (uint64_t) v as gcc compiles it for x86-64: comisd 2^63, cvttsd2si of v or of
// v - 2^63 (then the top bit flipped); cvttsd2si gives 2^63 for NaN and for
// anything outside the int64 range.
__host__ __device__ __forceinline__ uint64_t cvtt_x86(double w)
{
   if (w >= -0x1p63 && w < 0x1p63) return (uint64_t) (int64_t) w;
   return 0x8000000000000000ull;
}
__host__ __device__ __forceinline__ uint64_t to_u64_x86(double v)
{
   if (v >= 0x1p63) return cvtt_x86(v - 0x1p63) ^ 0x8000000000000000ull;
   return cvtt_x86(v);
}

}  // namespace gpow
}  // namespace gnoc
