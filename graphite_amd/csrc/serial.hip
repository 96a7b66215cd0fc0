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
//               k_ma_gather cycles and flits of each sorted request, and what the
//                           mean needs that depends on no state: the arithmetic
//                           mean's increment x/w - old/w, the geometric mean's
//                           factor pow(x, 1/w) / pow(old, 1/w), or the median itself
//               k_ma_chain  one lane per port: only the mean's FP64 chain, in order
//                           (one add / multiply per request once the window is full)
//               k_ma_scan1/2/3  the queue, QueueModelBasic's d = max(Q - ref, 0),
//                           Q = max(Q, ref) + F, as a segmented max-plus scan over the
//                           level's sorted requests (per 1024-entry block, a one-wave
//                           scan of the block aggregates, then the block again with
//                           its carry): delay per request, each port's last Q
//               k_ma_ports  per-port delay / flit sums (blocks of a port's segment)
//               k_ma_apply  each packet's time / contention / zero-load
//
// The geometric mean's pow is glibc's (glibc_pow.h, bit-exact with the x86-64
// FMA build the reference links), and ref = (T) mean is the x86-64 conversion
// (to_u64_x86: a NaN or inf mean -- a window holding a 0 -- converts as it does
// there).  Arithmetic mean, geometric mean and median are bit-exact against
// oracle/gnoc_oracle.c (orc_ma_compute, pinned against the reference's own
// moving_average.h compiled in oracle/_ref).  This TU is compiled with
// -ffp-contract=off (no FMA contraction), like the M/G/1 arithmetic.
#pragma once

#include "common.h"
#include "glibc_pow.h"

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

// Each port's segment [lo, hi) of the sorted entries, and the number of valid
// entries (requests of the level) in *mcount.
__global__ void k_ma_bounds(uint64_t n, uint64_t invalid, const uint64_t* __restrict__ key, uint32_t* __restrict__ lo,
                            uint32_t* __restrict__ hi, uint32_t* __restrict__ mcount)
{
   for (uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; j < n; j += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint64_t k = key[j];
      if (k == invalid) continue;
      const uint32_t p = (uint32_t) (k >> MA_T_BITS);
      const bool last = j + 1 == n || key[j + 1] == invalid;
      if (j == 0 || (uint32_t) (key[j - 1] >> MA_T_BITS) != p) lo[p] = (uint32_t) j;
      if (last || (uint32_t) (key[j + 1] >> MA_T_BITS) != p) hi[p] = (uint32_t) (j + 1);
      if (last) *mcount = (uint32_t) (j + 1);
   }
}

// Per sorted request j: the queue's input in cycles and the packet's flit count
// (coalesced; takes every load off the serial chain), and the part of the
// moving average that depends only on the request and the one w places earlier
// in the port's segment (the window's oldest entry once the window is full,
// moving_average.h:90-95, 121-126):
//   arithmetic  delta = (x / w) - (old / w)          (moving_average.h:93-94)
//   geometric   fac = pow(x, 1 / w) / pow(old, 1 / w)  (:125)
//   median      ref = the window's middle entry        (:149-153), final
// The chain adds / multiplies delta / fac in order, exactly as the reference.
template <int MT>
__global__ void k_ma_gather(uint64_t n, uint64_t invalid, uint32_t flit_width, double f, uint32_t ma_max,
                            const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                            const uint32_t* __restrict__ bits, const uint32_t* __restrict__ lo,
                            uint64_t* __restrict__ tcs, uint32_t* __restrict__ Fs, double* __restrict__ delta,
                            uint64_t* __restrict__ ref)
{
   for (uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; j < n; j += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint64_t k = key[j];
      if (k == invalid) continue;
      const uint64_t tc = cyc_of<false>(k & MA_T_MASK, f);   // Time::toCycles, time_types.h:104-109
      tcs[j] = tc;
      Fs[j] = ma_flits(bits[val[j]], flit_width);
      const uint32_t seen = (uint32_t) (j - lo[(uint32_t) (k >> MA_T_BITS)]);   // requests before j
      if (MT == MA_MEDIAN)
      {
         // after the add the window holds the last min(seen + 1, w) requests; the
         // median index is front + size / 2
         const uint32_t w = seen + 1 < ma_max ? seen + 1 : ma_max;
         ref[j] = cyc_of<false>(key[j + 1 - w + w / 2] & MA_T_MASK, f);
      }
      else if (seen >= ma_max)
      {
         const uint64_t old = cyc_of<false>(key[j - ma_max] & MA_T_MASK, f);
         if (MT == MA_ARITHMETIC)
            delta[j] = ((double) tc / (double) ma_max) - ((double) old / (double) ma_max);
         else
         {
            const double e = 1.0 / (double) ma_max;
            delta[j] = gpow::pow((double) tc, e) / gpow::pow((double) old, e);
         }
      }
   }
}

// The mean's serial chain, one lane per port over its sorted requests
// (MovingArithmeticMean / MovingGeometricMean::compute, moving_average.h:87-135):
// while the window fills, the reference's full formula; then one FP64 add or
// multiply per request with the gathered delta / factor.  Writes the mean of
// every request (the conversion to the reference time and the queue itself are
// parallel: k_ma_scan).  Loads run one block of MA_B requests ahead.
constexpr int MA_B = 32;

template <int MT>
__global__ void __launch_bounds__(64) k_ma_chain(uint32_t nloc, uint32_t ma_max, const uint64_t* __restrict__ tcs,
                                                 const uint32_t* __restrict__ lo, const uint32_t* __restrict__ hi,
                                                 const double* __restrict__ delta, double* __restrict__ mean_out)
{
   const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
   if (p >= nloc) return;
   const uint32_t j0 = lo[p], j1 = hi[p];
   // _arithmetic_mean(0.0) / _geometric_mean(1.0), moving_average.h:84, 116
   double m = MT == MA_ARITHMETIC ? 0.0 : 1.0;
   const uint32_t jf = j1 - j0 < ma_max ? j1 : j0 + ma_max;   // end of the filling requests
   for (uint32_t j = j0; j < jf; j++)
   {
      const uint32_t cw = j - j0;   // window size before the add
      const double x = (double) tcs[j];
      if (MT == MA_ARITHMETIC)
         m = (m * (double) cw + x) / (double) (cw + 1);
      else
         m = gpow::pow(gpow::pow(m, (double) cw) * x, 1.0 / (double) (cw + 1));
      mean_out[j] = m;
   }
   double cur[MA_B], nxt[MA_B];
   auto load = [&](uint32_t base, double* D) {
#pragma unroll
      for (int i = 0; i < MA_B; i++)
         if (base + (uint32_t) i < j1) D[i] = delta[base + i];
   };
   load(jf, cur);
   for (uint32_t base = jf; base < j1; base += MA_B)
   {
      load(base + MA_B, nxt);
#pragma unroll
      for (int i = 0; i < MA_B; i++)
      {
         if (base + (uint32_t) i >= j1) break;
         if (MT == MA_ARITHMETIC) m += cur[i];
         else m *= cur[i];
         mean_out[base + i] = m;
      }
#pragma unroll
      for (int i = 0; i < MA_B; i++) cur[i] = nxt[i];
   }
}

// ---- the queue as a segmented max-plus scan ----------------------------------
// QueueModelBasic::computeQueueDelay (queue_model_basic.cc:35-61) on ref:
//   d = max(Q - ref, 0);  Q = max(Q, ref) + F,  Q = 0 at a port's first request.
// Request j is the map Q -> max(Q + F, ref + F); a port's first request ignores Q
// (reset).  Maps compose: (A1, B1) then (A2, B2) = (A1 + A2, max(B1 + A2, B2)).
// _last_request_time (queue_model.cc:48-53) is the port's final Q (it never
// decreases).  u64 arithmetic as in the reference: ref may be 2^63 (a NaN mean).
constexpr uint32_t MS_T = 256, MS_PER = 4, MS_CH = MS_T * MS_PER;   // entries per scan block

struct MaAgg
{
   uint64_t A, B;
   uint32_t reset;
};
__device__ __forceinline__ MaAgg ma_op(const MaAgg& x, const MaAgg& y)   // x, then y
{
   if (y.reset) return y;
   MaAgg r;
   r.A = x.A + y.A;
   const uint64_t b = x.B + y.A;
   r.B = b > y.B ? b : y.B;
   r.reset = x.reset;
   return r;
}
template <int MT>
__device__ __forceinline__ uint64_t ma_ref(const uint64_t* ref, uint64_t j)
{
   if (MT == MA_MEDIAN) return ref[j];
   return gpow::to_u64_x86(__builtin_bit_cast(double, ref[j]));   // (T) _mean, moving_average.h:103, 134
}
__device__ __forceinline__ bool ma_first(const uint64_t* key, const uint32_t* lo, uint64_t j)
{
   return lo[(uint32_t) (key[j] >> MA_T_BITS)] == (uint32_t) j;
}

// Block-wide exclusive scan of one aggregate per thread (LDS, 256 threads); the
// block's total in `tot`.
__device__ MaAgg ma_block_scan(MaAgg v, MaAgg& tot)
{
   __shared__ uint64_t sA[MS_T], sB[MS_T];
   __shared__ uint32_t sR[MS_T];
   const uint32_t t = threadIdx.x;
   MaAgg inc = v;
   for (uint32_t off = 1; off < MS_T; off <<= 1)
   {
      sA[t] = inc.A;
      sB[t] = inc.B;
      sR[t] = inc.reset;
      __syncthreads();
      if (t >= off)
      {
         MaAgg prev;
         prev.A = sA[t - off];
         prev.B = sB[t - off];
         prev.reset = sR[t - off];
         inc = ma_op(prev, inc);
      }
      __syncthreads();
   }
   sA[t] = inc.A;
   sB[t] = inc.B;
   sR[t] = inc.reset;
   __syncthreads();
   tot.A = sA[MS_T - 1];
   tot.B = sB[MS_T - 1];
   tot.reset = sR[MS_T - 1];
   MaAgg ex;
   ex.A = t ? sA[t - 1] : 0;
   ex.B = t ? sB[t - 1] : 0;
   ex.reset = t ? sR[t - 1] : 0;
   __syncthreads();
   return ex;
}

template <int MT>
__device__ __forceinline__ MaAgg ma_thread_agg(uint64_t m, const uint64_t* key, const uint32_t* lo, const uint64_t* ref,
                                               const uint32_t* Fs, uint64_t j0)
{
   MaAgg g;
   g.A = 0;
   g.B = 0;
   g.reset = 0;
#pragma unroll
   for (uint32_t q = 0; q < MS_PER; q++)
   {
      const uint64_t j = j0 + q;
      if (j >= m) break;
      const uint64_t F = Fs[j], r = ma_ref<MT>(ref, j);
      MaAgg e;
      e.A = F;
      e.B = r + F;
      e.reset = ma_first(key, lo, j) ? 1u : 0u;
      g = ma_op(g, e);
   }
   return g;
}

// 1: the aggregate of each block of MS_CH requests
template <int MT>
__global__ __launch_bounds__(MS_T) void k_ma_scan1(const uint32_t* __restrict__ mcount, const uint64_t* __restrict__ key, const uint32_t* __restrict__ lo,
                                                   const uint64_t* __restrict__ ref, const uint32_t* __restrict__ Fs,
                                                   uint64_t* __restrict__ bA, uint64_t* __restrict__ bB, uint32_t* __restrict__ bR)
{
   const uint64_t m = *mcount;
   if ((uint64_t) blockIdx.x * MS_CH >= m) return;   // the grid covers every packet; the level has m requests
   const uint64_t j0 = (uint64_t) blockIdx.x * MS_CH + threadIdx.x * MS_PER;
   MaAgg tot;
   ma_block_scan(ma_thread_agg<MT>(m, key, lo, ref, Fs, j0), tot);
   if (threadIdx.x == 0)
   {
      bA[blockIdx.x] = tot.A;
      bB[blockIdx.x] = tot.B;
      bR[blockIdx.x] = tot.reset;
   }
}

// 2: one wave: the queue value entering each block (exclusive scan of the block
// aggregates applied to Q = 0; block 0 starts a port)
__global__ __launch_bounds__(64) void k_ma_scan2(const uint32_t* __restrict__ mcount, const uint64_t* __restrict__ bA, const uint64_t* __restrict__ bB,
                                                 const uint32_t* __restrict__ bR, uint64_t* __restrict__ qin)
{
   const uint32_t lane = threadIdx.x;
   const uint32_t nb = (*mcount + MS_CH - 1) / MS_CH;
   MaAgg carry;
   carry.A = 0;
   carry.B = 0;
   carry.reset = 1;
   for (uint32_t b0 = 0; b0 < nb; b0 += 64)
   {
      const uint32_t b = b0 + lane;
      MaAgg v;
      v.A = b < nb ? bA[b] : 0;
      v.B = b < nb ? bB[b] : 0;
      v.reset = b < nb ? bR[b] : 0;
      MaAgg inc = v;
      for (int off = 1; off < 64; off <<= 1)
      {
         MaAgg prev;
         prev.A = __shfl_up(inc.A, off);
         prev.B = __shfl_up(inc.B, off);
         prev.reset = __shfl_up(inc.reset, off);
         if ((int) lane >= off) inc = ma_op(prev, inc);
      }
      MaAgg ex;
      ex.A = __shfl_up(inc.A, 1);
      ex.B = __shfl_up(inc.B, 1);
      ex.reset = __shfl_up(inc.reset, 1);
      if (lane == 0)
      {
         ex.A = 0;
         ex.B = 0;
         ex.reset = 0;
      }
      const MaAgg before = ma_op(carry, ex);   // everything before block b (carry starts with a reset)
      if (b < nb) qin[b] = before.B > before.A ? before.B : before.A;   // max(0 + A, B)
      MaAgg last;
      last.A = __shfl(inc.A, 63);
      last.B = __shfl(inc.B, 63);
      last.reset = __shfl(inc.reset, 63);
      carry = ma_op(carry, last);
   }
}

// 3: each block again with its carry: delay per request, each port's final Q
template <int MT>
__global__ __launch_bounds__(MS_T) void k_ma_scan3(const uint32_t* __restrict__ mcount, const uint64_t* __restrict__ key, const uint32_t* __restrict__ lo,
                                                   const uint32_t* __restrict__ hi, const uint32_t* __restrict__ ports,
                                                   const uint64_t* __restrict__ ref, const uint32_t* __restrict__ Fs,
                                                   const uint64_t* __restrict__ qin, uint64_t* __restrict__ dout,
                                                   uint64_t* __restrict__ port_last)
{
   const uint64_t m = *mcount;
   if ((uint64_t) blockIdx.x * MS_CH >= m) return;
   const uint64_t j0 = (uint64_t) blockIdx.x * MS_CH + threadIdx.x * MS_PER;
   MaAgg tot;
   const MaAgg ex = ma_block_scan(ma_thread_agg<MT>(m, key, lo, ref, Fs, j0), tot);
   // Q before this thread's first request
   uint64_t Q = qin[blockIdx.x];
   if (ex.reset) Q = ex.B > ex.A ? ex.B : ex.A;
   else
   {
      const uint64_t b = Q + ex.A;
      Q = b > ex.B ? b : ex.B;
   }
#pragma unroll
   for (uint32_t q = 0; q < MS_PER; q++)
   {
      const uint64_t j = j0 + q;
      if (j >= m) break;
      const uint32_t pk = (uint32_t) (key[j] >> MA_T_BITS);
      if (lo[pk] == (uint32_t) j) Q = 0;
      const uint64_t r = ma_ref<MT>(ref, j);
      const uint64_t top = Q > r ? Q : r;
      dout[j] = top - r;
      Q = top + Fs[j];
      if (hi[pk] == (uint32_t) j + 1) port_last[ports[pk]] = Q;
   }
}

// Per-port delay and flit sums: grid (ports, blocks per port), integer atomics
// (deterministic); counts are the segment lengths.
__global__ __launch_bounds__(256) void k_ma_ports(const uint32_t* __restrict__ ports, const uint32_t* __restrict__ lo,
                                                  const uint32_t* __restrict__ hi, const uint64_t* __restrict__ dout,
                                                  const uint32_t* __restrict__ Fs, unsigned long long* __restrict__ port_sum,
                                                  unsigned long long* __restrict__ port_cnt,
                                                  unsigned long long* __restrict__ port_flit)
{
   const uint32_t p = blockIdx.x, j0 = lo[p], j1 = hi[p];
   unsigned long long s = 0, fl = 0;
   for (uint32_t j = j0 + blockIdx.y * blockDim.x + threadIdx.x; j < j1; j += gridDim.y * blockDim.x)
   {
      s += dout[j];
      fl += Fs[j];
   }
   for (int off = 32; off > 0; off >>= 1)
   {
      s += __shfl_down(s, off);
      fl += __shfl_down(fl, off);
   }
   if ((threadIdx.x & 63) == 0)
   {
      if (s) atomicAdd(&port_sum[ports[p]], s);
      if (fl) atomicAdd(&port_flit[ports[p]], fl);
   }
   if (blockIdx.y == 0 && threadIdx.x == 0) port_cnt[ports[p]] = j1 - j0;
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
