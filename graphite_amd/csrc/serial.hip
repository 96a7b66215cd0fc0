// serial.hip -- QueueModelBasic with a moving average (engine path 3).
//
// queue_model_basic.cc:35-61 with queue_model/basic/moving_avg_enabled: the
// queue's reference time is not the packet time but a moving average over the
// window of packet times it has seen (common/misc/moving_average.h), and the
// FIFO recurrence runs on that reference time:
//   ref = MA.compute(t);  d = max(Q - ref, 0);  Q = max(Q, ref) + F.
// The arithmetic mean is a running FP64 sum whose rounding depends on every
// earlier request of the queue, so a queue is one serial walk over its requests
// in (time, packet id) order.  What stays parallel is the port DAG of XY routing
// (DESIGN.md 2): every port of a level gets its whole request stream from earlier
// levels.  Unlike the FIFO paths, a port's departures are NOT in arrival order
// here (ref < t lets a later packet wait less), so the streams are re-sorted:
//
//   per level:  k_ma_keys   key = (port index in level, t_ps), value = packet id,
//                           one entry per packet (non-visitors get the max key)
//               radix sort  stable, bits [0, 49 + level bits) (ties: packet id)
//               k_ma_bounds first / last entry of each port
//               k_ma_gather cycles and flits of each sorted request
//               k_ma_walk   one thread per port: the reference's arithmetic, in
//                           order -> queue delay per request, port counters
//               k_ma_apply  each packet's time / contention / zero-load
//
// The geometric mean is refused by gnoc_set_basic_moving_average: its pow()
// chain is not bit-reproducible against glibc.  Arithmetic mean and median are
// bit-exact against
// oracle/gnoc_oracle.c (orc_ma_compute, pinned against the
// reference's own moving_average.h compiled in oracle/_ref).  This TU is compiled
// with -ffp-contract=off (no FMA contraction), like the M/G/1 arithmetic.
#pragma once

#include "common.h"

namespace gnoc {

enum : int { MA_NONE = 0, MA_ARITHMETIC = 1, MA_GEOMETRIC = 2, MA_MEDIAN = 3 };   // include/gnoc.h

constexpr uint32_t MA_T_BITS = 49;   // packet times < 2^49 ps (checked per level)
constexpr uint64_t MA_T_MASK = (1ull << MA_T_BITS) - 1;

__device__ __forceinline__ uint32_t ma_flits(uint32_t bits, uint32_t fw)
{
   return (bits % fw) ? bits / fw + 1 : bits / fw;   // network_model.cc:202-212
}

// Packet state before the first level: unrouted packets (self-sends, unmodeled,
// network_model.cc:413-468) finish at their injection time with no delay.
__global__ void k_ma_init(uint64_t n, uint32_t W, const uint64_t* __restrict__ inj, const uint32_t* __restrict__ src,
                          const uint32_t* __restrict__ dst, const uint32_t* __restrict__ flags,
                          uint64_t* __restrict__ ptime, uint64_t* __restrict__ fin, uint64_t* __restrict__ zl,
                          uint64_t* __restrict__ cont, unsigned long long* __restrict__ counters)
{
   unsigned long long hops = 0, routed = 0;
   for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x)
   {
      ptime[i] = inj[i];
      fin[i] = inj[i];
      zl[i] = 0;
      cont[i] = 0;
      const uint32_t s = src[i], d = dst[i];
      if (s != d && !(flags && (flags[i] & 1u)))
      {
         const uint32_t sx = s % W, sy = s / W, dx = d % W, dy = d / W;
         routed++;
         hops += (sx > dx ? sx - dx : dx - sx) + (sy > dy ? sy - dy : dy - sy) + 1;   // H + 1 mesh routers
      }
   }
   if (hops) atomicAdd(&counters[0], hops);
   if (routed) atomicAdd(&counters[1], routed);
}

// The port a packet src s -> dst d requests at level lvl of the plan (engine.hip
// build_static_levels), or ~0u when its route has no port there.
__device__ __forceinline__ uint32_t ma_port_at(uint32_t W, uint32_t s, uint32_t d, uint32_t lvl, uint32_t nlvl)
{
   const uint32_t sx = s % W, sy = s / W, dx = d % W, dy = d / W;
   if (lvl == 0) return s * PORTS + P_INJ;
   if (lvl == nlvl - 1) return d * PORTS + P_SELF;
   if (lvl < W)
   {
      const uint32_t l = lvl;
      if (sx < dx && sx <= l - 1 && l - 1 < dx) return (sy * W + l - 1) * PORTS + P_RIGHT;
      if (sx > dx && dx < W - l && W - l <= sx) return (sy * W + W - l) * PORTS + P_LEFT;
      return ~0u;
   }
   const uint32_t k = lvl - W, H = nlvl - W;   // nlvl = W + H
   if (sy < dy && sy <= k && k < dy) return (k * W + dx) * PORTS + P_UP;
   if (sy > dy && dy < H - 1 - k && H - 1 - k <= sy) return ((H - 1 - k) * W + dx) * PORTS + P_DOWN;
   return ~0u;
}

__global__ void k_ma_keys(uint64_t n, uint32_t W, uint32_t lvl, uint32_t nlvl, uint32_t k0, uint64_t invalid,
                          const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                          const uint32_t* __restrict__ flags, const uint32_t* __restrict__ port_k,
                          const uint64_t* __restrict__ ptime, uint64_t* __restrict__ key, uint32_t* __restrict__ val,
                          unsigned* __restrict__ err)
{
   for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x)
   {
      uint64_t kv = invalid;
      const uint32_t s = src[i], d = dst[i];
      if (s != d && !(flags && (flags[i] & 1u)))
      {
         const uint32_t p = ma_port_at(W, s, d, lvl, nlvl);
         if (p != ~0u)
         {
            const uint64_t t = ptime[i];
            if (t > MA_T_MASK) atomicOr(err, 1u);
            kv = ((uint64_t) (port_k[p] - k0) << MA_T_BITS) | (t & MA_T_MASK);
         }
      }
      key[i] = kv;
      val[i] = (uint32_t) i;
   }
}

__global__ void k_ma_bounds(uint64_t n, uint64_t invalid, const uint64_t* __restrict__ key, uint32_t* __restrict__ lo,
                            uint32_t* __restrict__ hi)
{
   for (uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; j < n; j += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint64_t k = key[j];
      if (k == invalid) continue;
      const uint32_t p = (uint32_t) (k >> MA_T_BITS);
      if (j == 0 || (uint32_t) (key[j - 1] >> MA_T_BITS) != p) lo[p] = (uint32_t) j;
      if (j + 1 == n || key[j + 1] == invalid || (uint32_t) (key[j + 1] >> MA_T_BITS) != p) hi[p] = (uint32_t) (j + 1);
   }
}

// Per sorted request j: the queue's input in cycles and the packet's flit count
// (coalesced; takes every load off the serial walk's dependency chain).
// For the arithmetic mean with a full window, also the increment
// (x / w) - (old / w) of moving_average.h:97-98: it depends only on the request
// and the one w places earlier in the port's segment, so its two FP64 divisions
// leave the serial walk (which then adds it, in order, exactly as the reference).
__global__ void k_ma_gather(uint64_t n, uint64_t invalid, uint32_t flit_width, double f, int ma_type, uint32_t ma_max,
                            const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                            const uint32_t* __restrict__ bits, const uint32_t* __restrict__ lo,
                            uint64_t* __restrict__ tcs, uint32_t* __restrict__ Fs, double* __restrict__ delta)
{
   for (uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; j < n; j += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint64_t k = key[j];
      if (k == invalid) continue;
      const uint64_t tc = cyc_of<false>(k & MA_T_MASK, f);   // Time::toCycles, time_types.h:104-109
      tcs[j] = tc;
      Fs[j] = ma_flits(bits[val[j]], flit_width);
      if (ma_type == MA_ARITHMETIC && j - lo[(uint32_t) (k >> MA_T_BITS)] >= ma_max)
      {
         const uint64_t old = cyc_of<false>(key[j - ma_max] & MA_T_MASK, f);
         delta[j] = ((double) tc / (double) ma_max) - ((double) old / (double) ma_max);
      }
   }
}

// One queue: QueueModelBasic::computeQueueDelay (queue_model_basic.cc:35-61) with
// MovingAverage<UInt64>::compute (moving_average.h:90-110 arithmetic, 153-162
// median), one thread per port over its sorted requests.
// The window is the port's last `ma_max` inputs, i.e. the previous entries of
// the same sorted segment, so the ring buffer's reads become plain indexed
// loads: the arithmetic mean's increment uses entry j - max (k_ma_gather), the median the
// entry front + size / 2 of the window after the add.  Loads run one block of
// MA_B requests ahead of the FP64 chain (registers, double-buffered).
constexpr int MA_B = 32;

template <int ma_type>
__global__ void __launch_bounds__(64) k_ma_walk(uint32_t nloc, const uint32_t* __restrict__ ports,
                                                uint32_t ma_max, const uint64_t* __restrict__ tcs,
                                                const uint32_t* __restrict__ Fs, const uint32_t* __restrict__ lo,
                                                const uint32_t* __restrict__ hi, const double* delta, uint64_t* dout,
                                                uint64_t* __restrict__ port_sum, uint64_t* __restrict__ port_cnt,
                                                uint64_t* __restrict__ port_flit, uint64_t* __restrict__ port_last)
{
   const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
   if (p >= nloc) return;
   const uint32_t port = ports[p];
   const uint32_t j0 = lo[p], j1 = hi[p];
   double mean = 0.0;   // MovingArithmeticMean's _arithmetic_mean(0.0), moving_average.h:88
   uint64_t Q = 0, sum = 0, flits = 0;
   uint64_t cx[MA_B], co[MA_B], nx[MA_B], no[MA_B];
   uint32_t cf[MA_B], nf[MA_B];
   // entry j's window partner: the mean's gathered increment, or the median
   auto other = [&](uint32_t j) -> uint64_t {
      const uint32_t seen = j - j0;   // requests before j
      if (ma_type == MA_MEDIAN)
      {
         const uint32_t w = seen + 1 < ma_max ? seen + 1 : ma_max;
         return tcs[j + 1 - w + w / 2];
      }
      return seen >= ma_max ? __builtin_bit_cast(uint64_t, delta[j]) : 0ull;   // the gathered increment
   };
   auto load = [&](uint32_t base, uint64_t* X, uint64_t* O, uint32_t* F) {
#pragma unroll
      for (int i = 0; i < MA_B; i++)
      {
         const uint32_t j = base + (uint32_t) i;
         if (j < j1)
         {
            X[i] = tcs[j];
            F[i] = Fs[j];
            O[i] = other(j);
         }
      }
   };
   load(j0, cx, co, cf);
   for (uint32_t base = j0; base < j1; base += MA_B)
   {
      load(base + MA_B, nx, no, nf);
#pragma unroll
      for (int i = 0; i < MA_B; i++)
      {
         const uint32_t j = base + (uint32_t) i;
         if (j >= j1) continue;
         const uint64_t tc = cx[i];
         const uint32_t F = cf[i];
         const uint32_t seen = j - j0;
         const uint32_t cw = seen < ma_max ? seen : ma_max;   // window size before the add
         uint64_t ref;
         if constexpr (ma_type == MA_MEDIAN)
            ref = co[i];
         else
         {
            static_assert(ma_type == MA_ARITHMETIC, "the geometric mean is refused (gnoc_set_basic_moving_average)");
            if (cw == ma_max)
               mean += __builtin_bit_cast(double, co[i]);   // (tc / cw) - (old / cw), k_ma_gather
            else
               mean = (mean * (double) cw + (double) tc) / (double) (cw + 1);
            ref = (uint64_t) mean;
         }
         // d = max(Q - ref, 0); Q = max(Q, ref) + F.  QueueModel's
         // _last_request_time = max(ref + d + F) = max over requests of the new Q,
         // which never decreases: the final Q (queue_model.cc:48-53)
         const uint64_t top = Q > ref ? Q : ref;
         const uint64_t d = top - ref;
         Q = top + F;
         flits += F;
         sum += d;
         dout[j] = d;
      }
#pragma unroll
      for (int i = 0; i < MA_B; i++)
      {
         cx[i] = nx[i];
         co[i] = no[i];
         cf[i] = nf[i];
      }
   }
   port_sum[port] = sum;
   port_cnt[port] = j1 - j0;
   port_flit[port] = flits;
   port_last[port] = Q;
}

// Per request: RouterModel / Hop bookkeeping (router_model.cc:70-108,
// network_model.cc:556-563) and, at SELF, the receive serialization
// (network_model.cc:142-150).  Each packet has at most one request per level.
__global__ void k_ma_apply(uint64_t n, uint64_t invalid, const uint32_t* __restrict__ ports, double f, uint64_t rl_ps,
                           const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                           const uint32_t* __restrict__ Fs, const uint64_t* __restrict__ dout,
                           uint64_t* __restrict__ ptime, uint64_t* __restrict__ fin, uint64_t* __restrict__ zl,
                           uint64_t* __restrict__ cont)
{
   for (uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; j < n; j += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint64_t k = key[j];
      if (k == invalid) continue;
      const uint32_t dir = ports[(uint32_t) (k >> MA_T_BITS)] % PORTS;
      const uint32_t id = val[j];
      const uint64_t hop_ps = dir == P_INJ ? ps_of<false>(0, f) : rl_ps;   // injection router: delay 0
      const uint64_t cps = ps_of<false>(dout[j], f);
      uint64_t tn = (k & MA_T_MASK) + cps + hop_ps;
      uint64_t z = zl[id] + hop_ps;
      cont[id] += cps;
      if (dir == P_SELF)
      {
         const uint64_t fps = ps_of<false>(Fs[j], f);
         tn += fps;
         z += fps;
         fin[id] = tn;
      }
      zl[id] = z;
      ptime[id] = tn;
   }
}

}  // namespace gnoc
