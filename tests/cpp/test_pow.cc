// Host check of graphite_amd/csrc/glibc_pow.h (the engine's device pow for the
// geometric moving average) against this image's glibc pow, bit for bit, and of
// its x86-64 double -> uint64 conversion against gcc's cast.  The header is
// product code written for HIP; plain g++ sees its __host__ __device__ marks as
// empty.  Built by __graft_entry__.build() with -ffp-contract=off (like
// libgnoc.so); run by tests/test_pow.py.
#define __host__
#define __device__
#define __forceinline__ inline
#include "glibc_pow.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

namespace {

uint64_t bits(double x)
{
   uint64_t u;
   std::memcpy(&u, &x, 8);
   return u;
}
double dbl(uint64_t u)
{
   double x;
   std::memcpy(&x, &u, 8);
   return x;
}
// NaNs compare equal whatever their payload (the engine only converts them)
bool same(double a, double b) { return bits(a) == bits(b) || (std::isnan(a) && std::isnan(b)); }

// not folded at compile time: the cast of NaN / out-of-range values is what the
// x86 instructions do, which is what the reference's (T) _geometric_mean does
__attribute__((noinline)) uint64_t cast_gcc(double v)
{
   volatile double w = v;
   return (uint64_t) w;
}

}  // namespace

int main(int argc, char** argv)
{
   const long n = argc > 1 ? std::atol(argv[1]) : 2000000;
   std::mt19937_64 rng(12345);
   long bad = 0, total = 0;
   auto check = [&](double x, double y) {
      const double want = ::pow(x, y), got = gnoc::gpow::pow(x, y);
      total++;
      if (!same(want, got))
      {
         if (bad < 10) std::printf("MISMATCH pow(%a, %a): glibc %a, gpow %a\n", x, y, want, got);
         bad++;
      }
   };
   // 1. the operands of MovingGeometricMean::compute: integer cycle counts x,
   //    exponents 1 / w and w, and products pow(g, w) * x
   std::uniform_int_distribution<uint64_t> cyc(0, (1ull << 40));
   std::uniform_int_distribution<uint32_t> win(1, 65536);
   for (long i = 0; i < n; i++)
   {
      const uint64_t xc = (i & 7) == 0 ? (cyc(rng) & 0xFFFFF) : cyc(rng) >> (rng() % 40);
      const uint32_t w = (i & 3) == 0 ? win(rng) : 1 + (uint32_t) (rng() % 128);
      const double x = (double) xc;
      check(x, 1.0 / (double) w);
      const double g = std::ldexp(1.0 + (double) (rng() >> 11) * 0x1p-53, (int) (rng() % 64));
      check(g, (double) (w - 1));
      check(::pow(g, (double) (w % 64)) * x, 1.0 / (double) (w % 64 + 1));
   }
   // 2. random finite doubles (every exponent range, both signs), random y
   for (long i = 0; i < n; i++)
   {
      const double x = dbl(rng() & ~(i & 1 ? 0ull : 0x8000000000000000ull));
      const double y = (i & 3) == 0 ? (double) (int64_t) (rng() % 2001 - 1000) : dbl((rng() & 0x800FFFFFFFFFFFFFull) | ((uint64_t) (0x3a0 + rng() % 0xA0) << 52));
      if (std::isfinite(x)) check(x, y);
   }
   // 3. results near the overflow / underflow / subnormal boundaries (specialcase)
   for (long i = 0; i < n / 4; i++)
   {
      const double x = 1.0 + (double) (rng() >> 11) * 0x1p-50;
      const double target = (i & 1 ? 1.0 : -1.0) * (700.0 + (double) (rng() % 50000) * 0.001);
      check(x, target / std::log(x));
      check(2.0, -1074.5 + (double) (rng() % 100000) * 1e-4);
   }
   // 4. special operands
   const double sp[] = { 0.0, -0.0, 1.0, -1.0, 2.0, -2.0, 0.5, 3.0, -3.0, 1e-310, -1e-310, 0x1p-1074, 1e300, -1e300,
                         INFINITY, -INFINITY, NAN, 0x1p-70, -0x1p-70, 0x1p70, 1.0 + 0x1p-52, 1.0 - 0x1p-53, 1e-20, 65536.0 };
   for (double x : sp)
      for (double y : sp) check(x, y);
   // 5. gcc's (uint64_t) cast
   long cbad = 0;
   const double cv[] = { 0.0, -0.0, 0.7, -0.7, -1.0, -5.5, 1e19, 0x1p63, 0x1p64, 1e30, -1e30, INFINITY, -INFINITY, NAN,
                         0x1.fffffffffffffp62, 0x1p63 + 2048.0, -0x1p63, 18446744073709549568.0 };
   for (double v : cv)
      if (cast_gcc(v) != gnoc::gpow::to_u64_x86(v))
      {
         std::printf("CAST MISMATCH %a: gcc %llx, ours %llx\n", v, (unsigned long long) cast_gcc(v),
                     (unsigned long long) gnoc::gpow::to_u64_x86(v));
         cbad++;
      }
   for (long i = 0; i < n; i++)
   {
      const double v = dbl(rng());
      if (cast_gcc(v) != gnoc::gpow::to_u64_x86(v)) cbad++;
   }
   std::printf("pow: %ld of %ld differ; cast: %ld differ\n", bad, total, cbad);
   return bad || cbad ? 1 : 0;
}
