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

// Sort keys: (port index in level) << tb | t_ps.  tb = 32 while every request
// time of the batch is below 2^32 ps (5 radix passes on 32x32), else 49; a
// request at or beyond 2^tb ps sets a flag and the host reruns with tb = 49
// (the engine refuses times beyond 2^49 ps).
constexpr uint32_t MA_T_BITS = 49;
__device__ __forceinline__ uint32_t kport(uint64_t k, uint32_t tb) { return (uint32_t) (k >> tb); }
__device__ __forceinline__ uint64_t ktime(uint64_t k, uint32_t tb) { return k & ((1ull << tb) - 1); }

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

// ---- the level's requests in (port, time, packet id) order -----------------
// Compaction (packet order), then a stable LSD radix sort on 8-bit digits.
// Blocks of RS_CH entries; the ranking inside a block uses wave ballots (a
// wave's 64 entries matched on their digit by 8 ballots), so equal keys keep
// packet order: ties of (port, t) go by packet id as in the reference's event
// queue.
constexpr uint32_t RS_T = 256, RS_PER = 8, RS_CH = RS_T * RS_PER, RS_BINS = 256;

__device__ __forceinline__ uint64_t lanes_below() { return (1ull << (threadIdx.x & 63)) - 1; }

// The requests of level lvl: entry i of the compacted list is a (key, packet id)
// pair.  Pass 1 counts per block; the block offsets are an exclusive scan.
__device__ __forceinline__ bool ma_visit(uint32_t W, uint32_t lvl, uint32_t nlvl, const uint32_t* src, const uint32_t* dst,
                                         const uint32_t* flags, uint64_t i, uint32_t& p)
{
   const uint32_t s = src[i], d = dst[i];
   if (s == d || (flags && (flags[i] & 1u))) return false;
   p = ma_port_at(W, s, d, lvl, nlvl);
   return p != ~0u;
}

__global__ __launch_bounds__(RS_T) void k_ma_count(uint64_t n, uint32_t W, uint32_t lvl, uint32_t nlvl,
                                                   const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                                                   const uint32_t* __restrict__ flags, uint32_t* __restrict__ bcnt)
{
   __shared__ uint32_t wc[RS_T / 64];
   uint32_t c = 0;
   for (uint32_t q = 0; q < RS_PER; q++)
   {
      const uint64_t i = (uint64_t) blockIdx.x * RS_CH + q * RS_T + threadIdx.x;
      uint32_t p;
      if (i < n && ma_visit(W, lvl, nlvl, src, dst, flags, i, p)) c++;
   }
   for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off);
   if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
   __syncthreads();
   if (threadIdx.x == 0)
   {
      uint32_t t = 0;
      for (uint32_t w = 0; w < RS_T / 64; w++) t += wc[w];
      bcnt[blockIdx.x] = t;
   }
}

// Exclusive scan of nb counts in place (one block of 1024); the total in *total.
__global__ __launch_bounds__(1024) void k_ma_scan_counts(uint32_t nb, uint32_t* __restrict__ cnt, uint32_t* __restrict__ total)
{
   __shared__ uint32_t part[1024];
   const uint32_t t = threadIdx.x, per = (nb + 1023) / 1024, b0 = t * per, b1 = min(nb, b0 + per);
   uint32_t sum = 0;
   for (uint32_t b = b0; b < b1; b++) sum += cnt[b];
   part[t] = sum;
   __syncthreads();
   for (uint32_t off = 1; off < 1024; off <<= 1)
   {
      const uint32_t v = t >= off ? part[t - off] : 0u;
      __syncthreads();
      part[t] += v;
      __syncthreads();
   }
   uint32_t run = part[t] - sum;
   for (uint32_t b = b0; b < b1; b++)
   {
      const uint32_t c = cnt[b];
      cnt[b] = run;
      run += c;
   }
   if (t == 1023) *total = part[1023];
}

// Pass 2: the compacted (key, packet id) list, in packet order.
__global__ __launch_bounds__(RS_T) void k_ma_keys(uint64_t n, uint32_t W, uint32_t lvl, uint32_t nlvl, uint32_t k0, uint32_t tb,
                                                  const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                                                  const uint32_t* __restrict__ flags, const uint32_t* __restrict__ port_k,
                                                  const uint64_t* __restrict__ ptime, const uint32_t* __restrict__ boff,
                                                  uint64_t* __restrict__ key, uint32_t* __restrict__ val,
                                                  unsigned* __restrict__ err)
{
   __shared__ uint32_t wc[RS_T / 64];
   const uint32_t w = threadIdx.x >> 6;
   uint32_t run = boff[blockIdx.x];
   for (uint32_t q = 0; q < RS_PER; q++)
   {
      const uint64_t i = (uint64_t) blockIdx.x * RS_CH + q * RS_T + threadIdx.x;
      uint32_t p = 0;
      const bool v = i < n && ma_visit(W, lvl, nlvl, src, dst, flags, i, p);
      const uint64_t bal = __ballot(v);
      if ((threadIdx.x & 63) == 0) wc[w] = (uint32_t) __popcll(bal);
      __syncthreads();
      uint32_t before = run;
      for (uint32_t u = 0; u < w; u++) before += wc[u];
      if (v)
      {
         const uint64_t t = ptime[i];
         if (t >> tb) atomicOr(err, 1u);
         const uint32_t j = before + (uint32_t) __popcll(bal & lanes_below());
         key[j] = ((uint64_t) (port_k[p] - k0) << tb) | t;
         val[j] = (uint32_t) i;
      }
      for (uint32_t u = 0; u < RS_T / 64; u++) run += wc[u];
      __syncthreads();
   }
}

// Radix pass, 1: per-block digit histograms, digit-major hist[d * nbs + b]
// (nbs = the host's bound on the block count).
template <typename K>
__global__ __launch_bounds__(RS_T) void k_rs_hist(const uint32_t* __restrict__ mcount, uint32_t shift, uint32_t nbs,
                                                  const K* __restrict__ key, uint32_t* __restrict__ hist)
{
   __shared__ uint32_t h[RS_BINS];
   const uint32_t m = *mcount;
   if ((uint64_t) blockIdx.x * RS_CH >= m) return;
   h[threadIdx.x] = 0;
   __syncthreads();
   for (uint32_t q = 0; q < RS_PER; q++)
   {
      const uint32_t i = blockIdx.x * RS_CH + q * RS_T + threadIdx.x;
      if (i < m) atomicAdd(&h[(uint32_t) (key[i] >> shift) & 0xFFu], 1u);
   }
   __syncthreads();
   hist[(size_t) threadIdx.x * nbs + blockIdx.x] = h[threadIdx.x];
}

// Block-wide exclusive sum of one value per thread (RS_T threads); total in tot.
__device__ __forceinline__ uint32_t rs_block_exclusive(uint32_t v, uint32_t& tot)
{
   __shared__ uint32_t sc[RS_T];
   const uint32_t t = threadIdx.x;
   sc[t] = v;
   __syncthreads();
   for (uint32_t off = 1; off < RS_T; off <<= 1)
   {
      const uint32_t u = t >= off ? sc[t - off] : 0u;
      __syncthreads();
      sc[t] += u;
      __syncthreads();
   }
   const uint32_t inc = sc[t];
   tot = sc[RS_T - 1];
   __syncthreads();
   return inc - v;
}

// Radix pass, 2: one block per digit: the exclusive scan of its row over the
// blocks (in place) and the digit's total.
__global__ __launch_bounds__(RS_T) void k_rs_offsets(const uint32_t* __restrict__ mcount, uint32_t nbs,
                                                     uint32_t* __restrict__ hist, uint32_t* __restrict__ dtot)
{
   const uint32_t nb = (*mcount + RS_CH - 1) / RS_CH;
   uint32_t* row = hist + (size_t) blockIdx.x * nbs;
   uint32_t carry = 0;
   for (uint32_t c = 0; c < nb; c += RS_T)
   {
      const uint32_t b = c + threadIdx.x;
      const uint32_t v = b < nb ? row[b] : 0u;
      uint32_t tot;
      const uint32_t ex = rs_block_exclusive(v, tot);
      if (b < nb) row[b] = carry + ex;
      carry += tot;
   }
   if (threadIdx.x == 0) dtot[blockIdx.x] = carry;
}

// Radix pass, 3: stable scatter.  Wave w of the block takes the block's entries
// [w 512, (w + 1) 512) in 8 sub-rounds of 64: first its per-digit counts (LDS
// atomics), then, after one block-wide prefix of the counts over the waves, its
// placement with wave-local state only -- a lane's rank among the lanes of the
// same digit from 8 ballots, its position from the wave's running counter of
// that digit (read by every lane before the leader advances it: a wave's LDS
// operations execute in program order).  Two block barriers per 2,048 entries.
template <typename K, typename V>
__global__ __launch_bounds__(RS_T) void k_rs_scatter(const uint32_t* __restrict__ mcount, uint32_t shift, uint32_t nbs,
                                                     const K* __restrict__ kin, const V* __restrict__ vin,
                                                     const uint32_t* __restrict__ offs, const uint32_t* __restrict__ dtot,
                                                     K* __restrict__ kout, V* __restrict__ vout)
{
   constexpr uint32_t NW = RS_T / 64, WCH = RS_CH / NW;   // entries per wave
   __shared__ uint32_t wb[NW][RS_BINS];
   const uint32_t m = *mcount;
   if ((uint64_t) blockIdx.x * RS_CH >= m) return;
   const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
   for (uint32_t u = 0; u < NW; u++) wb[u][t] = 0;
   __syncthreads();
   const uint32_t i0 = blockIdx.x * RS_CH + w * WCH;
   K kr[RS_PER];
   V vr[RS_PER];
#pragma unroll
   for (uint32_t q = 0; q < RS_PER; q++)
   {
      const uint32_t i = i0 + q * 64 + lane;
      kr[q] = K(0);
      vr[q] = V{};
      if (i < m)
      {
         kr[q] = kin[i];
         vr[q] = vin[i];
         atomicAdd(&wb[w][(uint32_t) (kr[q] >> shift) & 0xFFu], 1u);
      }
   }
   __syncthreads();
   {
      // thread t = digit t: the block's base for it, then each wave's start
      uint32_t tot;
      uint32_t run = rs_block_exclusive(dtot[t], tot) + offs[(size_t) t * nbs + blockIdx.x];
#pragma unroll
      for (uint32_t u = 0; u < NW; u++)
      {
         const uint32_t c = wb[u][t];
         wb[u][t] = run;
         run += c;
      }
   }
   __syncthreads();
#pragma unroll
   for (uint32_t q = 0; q < RS_PER; q++)
   {
      const uint32_t i = i0 + q * 64 + lane;
      const bool v = i < m;
      const uint32_t dg = (uint32_t) (kr[q] >> shift) & 0xFFu;
      uint64_t peers = __ballot(v);
#pragma unroll
      for (int b = 0; b < 8; b++)
      {
         const uint64_t bb = __ballot((dg >> b) & 1u);
         peers &= ((dg >> b) & 1u) ? bb : ~bb;
      }
      const uint32_t rank = (uint32_t) __popcll(peers & lanes_below());
      const uint32_t pos = v ? wb[w][dg] + rank : 0u;
      __builtin_amdgcn_wave_barrier();
      if (v && rank == 0) wb[w][dg] += (uint32_t) __popcll(peers);
      __builtin_amdgcn_wave_barrier();
      if (v)
      {
         kout[pos] = kr[q];
         vout[pos] = vr[q];
      }
   }
}

// ---- injection slots of large meshes (N > 4096: sweeps) ----------------------
// The stable group-by-source of the trace as a 2-pass LSD radix sort of
// (source, record) pairs -- the per-chunk source counters of the scatter kernels
// need N words of LDS per wave, which a 16,384-tile sweep mesh cannot give them.
// Packets this rank does not place get the key N and sort last.
__global__ void k_set_u32(uint32_t* p, uint32_t v) { *p = v; }

__global__ void k_src_keys(uint64_t n, uint32_t N, const uint32_t* __restrict__ src, const uint8_t* __restrict__ routed,
                           const uint64_t* __restrict__ inj, const uint32_t* __restrict__ aux,
                           const uint32_t* __restrict__ gid, uint32_t* __restrict__ key, Rec* __restrict__ rec)
{
   for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x)
   {
      const bool placed = (routed[i] & 2) != 0;
      key[i] = placed ? src[i] : N;
      Rec r;
      r.t = inj[i];
      r.id = gid ? gid[i] : (uint32_t) i;
      r.aux = aux[i];
      rec[i] = r;
   }
}

// First sorted position of every present source.
__global__ void k_src_first(uint64_t m, uint32_t N, const uint32_t* __restrict__ key, uint32_t* __restrict__ first)
{
   for (uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; j < m; j += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint32_t s = key[j];
      if (s < N && (j == 0 || key[j - 1] != s)) first[s] = (uint32_t) j;
   }
}

// The sorted records into their injection slots (coalesced: a source's records
// are consecutive in both), with the 1-in-64 key samples.
__global__ void k_src_place(uint64_t m, uint32_t N, const uint32_t* __restrict__ key, const Rec* __restrict__ rec,
                            const uint32_t* __restrict__ first, const uint64_t* __restrict__ slot_base,
                            Rec* __restrict__ recs, uint64_t* __restrict__ samp_t, uint32_t* __restrict__ samp_id)
{
   for (uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; j < m; j += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint32_t s = key[j];
      if (s >= N) continue;
      const uint64_t pos = slot_base[slot_of(s, P_INJ, IN_LOCAL)] + (j - first[s]);
      const Rec r = rec[j];
      recs[pos] = r;
      if ((pos & 63) == 0)
      {
         samp_t[pos >> 6] = r.t;
         samp_id[pos >> 6] = r.id;
      }
   }
}

// Each port's segment [lo, hi) of the sorted requests.
__global__ void k_ma_bounds(const uint32_t* __restrict__ mcount, uint32_t tb, const uint64_t* __restrict__ key,
                            uint32_t* __restrict__ lo, uint32_t* __restrict__ hi)
{
   const uint64_t m = *mcount;
   for (uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; j < m; j += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint32_t p = kport(key[j], tb);
      if (j == 0 || kport(key[j - 1], tb) != p) lo[p] = (uint32_t) j;
      if (j + 1 == m || kport(key[j + 1], tb) != p) hi[p] = (uint32_t) (j + 1);
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
__global__ void k_ma_gather(const uint32_t* __restrict__ mcount, uint32_t tb, uint32_t flit_width, double f, uint32_t ma_max,
                            const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                            const uint32_t* __restrict__ bits, const uint32_t* __restrict__ lo,
                            uint64_t* __restrict__ tcs, uint32_t* __restrict__ Fs, double* __restrict__ delta,
                            uint64_t* __restrict__ ref)
{
   const uint64_t n = *mcount;
   for (uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; j < n; j += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint64_t k = key[j];
      const uint64_t tc = cyc_of<false>(ktime(k, tb), f);   // Time::toCycles, time_types.h:104-109
      tcs[j] = tc;
      Fs[j] = ma_flits(bits[val[j]], flit_width);
      const uint32_t seen = (uint32_t) (j - lo[kport(k, tb)]);   // requests before j
      if (MT == MA_MEDIAN)
      {
         // after the add the window holds the last min(seen + 1, w) requests; the
         // median index is front + size / 2
         const uint32_t w = seen + 1 < ma_max ? seen + 1 : ma_max;
         ref[j] = cyc_of<false>(ktime(key[j + 1 - w + w / 2], tb), f);
      }
      else if (seen >= ma_max)
      {
         const uint64_t old = cyc_of<false>(ktime(key[j - ma_max], tb), f);
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

// The mean's serial chain over one port's sorted requests
// (MovingArithmeticMean / MovingGeometricMean::compute, moving_average.h:87-135):
// while the window fills, the reference's full formula; then one FP64 add or
// multiply per request with the gathered delta / factor.  Writes the mean of
// every request (the conversion to the reference time and the queue itself are
// parallel: k_ma_scan).  One wave per port: the wave moves blocks of 64 deltas
// and means with coalesced loads / stores (the next block in flight) through
// LDS, and lane 0 runs only the FP64 chain out of LDS.  (A lane per port with a
// global store per request waited on its own stores -- gfx9's vmcnt counts
// stores too -- at ~60 ns per request.)
template <int MT>
__global__ void __launch_bounds__(64) k_ma_chain(uint32_t nloc, uint32_t ma_max, const uint64_t* __restrict__ tcs,
                                                 const uint32_t* __restrict__ lo, const uint32_t* __restrict__ hi,
                                                 const double* __restrict__ delta, double* __restrict__ mean_out)
{
   __shared__ double din[64], dres[64];
   const uint32_t p = blockIdx.x, lane = threadIdx.x;
   if (p >= nloc) return;
   const uint32_t j0 = lo[p], j1 = hi[p];
   // _arithmetic_mean(0.0) / _geometric_mean(1.0), moving_average.h:84, 116
   double m = MT == MA_ARITHMETIC ? 0.0 : 1.0;
   const uint32_t jf = j1 - j0 < ma_max ? j1 : j0 + ma_max;   // end of the filling requests
   if (lane == 0)
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
   double nxt = jf + lane < j1 ? delta[jf + lane] : 0.0;
   for (uint32_t base = jf; base < j1; base += 64)
   {
      const double cur = nxt;
      if (base + 64 + lane < j1) nxt = delta[base + 64 + lane];   // the next block in flight
      din[lane] = cur;
      __builtin_amdgcn_wave_barrier();
      if (lane == 0)
      {
         const uint32_t cnt = j1 - base < 64 ? j1 - base : 64;
         if (cnt == 64)
         {
            // full block: the LDS reads of a group issue ahead of its dependent chain
#pragma unroll
            for (int g = 0; g < 64; g += 16)
            {
               double v[16];
#pragma unroll
               for (int k = 0; k < 16; k++) v[k] = din[g + k];
#pragma unroll
               for (int k = 0; k < 16; k++)
               {
                  if (MT == MA_ARITHMETIC) m += v[k];
                  else m *= v[k];
                  dres[g + k] = m;
               }
            }
         }
         else
            for (uint32_t i = 0; i < cnt; i++)
            {
               if (MT == MA_ARITHMETIC) m += din[i];
               else m *= din[i];
               dres[i] = m;
            }
      }
      __builtin_amdgcn_wave_barrier();
      if (base + lane < j1) mean_out[base + lane] = dres[lane];
      __builtin_amdgcn_wave_barrier();
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
__device__ __forceinline__ bool ma_first(const uint64_t* key, const uint32_t* lo, uint64_t j, uint32_t tb)
{
   return lo[kport(key[j], tb)] == (uint32_t) j;
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
__device__ __forceinline__ MaAgg ma_thread_agg(uint64_t m, uint32_t tb, const uint64_t* key, const uint32_t* lo,
                                               const uint64_t* ref, const uint32_t* Fs, uint64_t j0)
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
      e.reset = ma_first(key, lo, j, tb) ? 1u : 0u;
      g = ma_op(g, e);
   }
   return g;
}

// 1: the aggregate of each block of MS_CH requests
template <int MT>
__global__ __launch_bounds__(MS_T) void k_ma_scan1(const uint32_t* __restrict__ mcount, uint32_t tb, const uint64_t* __restrict__ key, const uint32_t* __restrict__ lo,
                                                   const uint64_t* __restrict__ ref, const uint32_t* __restrict__ Fs,
                                                   uint64_t* __restrict__ bA, uint64_t* __restrict__ bB, uint32_t* __restrict__ bR)
{
   const uint64_t m = *mcount;
   if ((uint64_t) blockIdx.x * MS_CH >= m) return;   // the grid covers every packet; the level has m requests
   const uint64_t j0 = (uint64_t) blockIdx.x * MS_CH + threadIdx.x * MS_PER;
   MaAgg tot;
   ma_block_scan(ma_thread_agg<MT>(m, tb, key, lo, ref, Fs, j0), tot);
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
__global__ __launch_bounds__(MS_T) void k_ma_scan3(const uint32_t* __restrict__ mcount, uint32_t tb, const uint64_t* __restrict__ key, const uint32_t* __restrict__ lo,
                                                   const uint32_t* __restrict__ hi, const uint32_t* __restrict__ ports,
                                                   const uint64_t* __restrict__ ref, const uint32_t* __restrict__ Fs,
                                                   const uint64_t* __restrict__ qin, uint64_t* __restrict__ dout,
                                                   uint64_t* __restrict__ port_last)
{
   const uint64_t m = *mcount;
   if ((uint64_t) blockIdx.x * MS_CH >= m) return;
   const uint64_t j0 = (uint64_t) blockIdx.x * MS_CH + threadIdx.x * MS_PER;
   MaAgg tot;
   const MaAgg ex = ma_block_scan(ma_thread_agg<MT>(m, tb, key, lo, ref, Fs, j0), tot);
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
      const uint32_t pk = kport(key[j], tb);
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
// network_model.cc:556-563): the packet leaves the router at t + delay + hop
// delay (the injection router's is 0), plus, at SELF, the receive serialization
// (network_model.cc:142-150).  Only the packet's time is carried between levels;
// zero-load and contention follow in closed form (k_ma_final).
__global__ void k_ma_apply(const uint32_t* __restrict__ mcount, uint32_t tb, const uint32_t* __restrict__ ports, double f,
                           uint64_t rl_ps, const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                           const uint32_t* __restrict__ Fs, const uint64_t* __restrict__ dout, uint64_t* __restrict__ ptime,
                           uint64_t* __restrict__ fin)
{
   const uint64_t n = *mcount;   // the level's requests
   for (uint64_t j = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; j < n; j += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint64_t k = key[j];
      const uint32_t dir = ports[kport(k, tb)] % PORTS;
      const uint32_t id = val[j];
      const uint64_t hop_ps = dir == P_INJ ? ps_of<false>(0, f) : rl_ps;   // injection router: delay 0
      uint64_t tn = ktime(k, tb) + ps_of<false>(dout[j], f) + hop_ps;
      if (dir == P_SELF)
      {
         tn += ps_of<false>(Fs[j], f);
         fin[id] = tn;
      }
      else
         ptime[id] = tn;
   }
}

// After the last level: zero-load = the injection router's 0 + (H + 1) router and
// link delays + the serialization (the per-hop sums k_ma_apply's predecessor kept
// per packet), contention = final - inject - zero-load (= the sum of the queue
// delays in ps, exactly).
__global__ void k_ma_final(uint64_t n, uint32_t W, uint32_t flit_width, double f, uint64_t rl_ps,
                           const uint64_t* __restrict__ inj, const uint32_t* __restrict__ src,
                           const uint32_t* __restrict__ dst, const uint32_t* __restrict__ bits,
                           const uint32_t* __restrict__ flags, const uint64_t* __restrict__ fin, uint64_t* __restrict__ zl,
                           uint64_t* __restrict__ cont)
{
   for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint32_t s = src[i], d = dst[i];
      if (s == d || (flags && (flags[i] & 1u))) continue;   // k_ma_init's zeros stand
      const uint32_t sx = s % W, sy = s / W, dx = d % W, dy = d / W;
      const uint64_t hops = (sx > dx ? sx - dx : dx - sx) + (sy > dy ? sy - dy : dy - sy) + 1;
      const uint64_t z = ps_of<false>(0, f) + hops * rl_ps + ps_of<false>(ma_flits(bits[i], flit_width), f);
      zl[i] = z;
      cont[i] = fin[i] - inj[i] - z;
   }
}

}  // namespace gnoc
