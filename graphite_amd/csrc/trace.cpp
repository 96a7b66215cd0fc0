// trace.cpp -- synthetic packet traces (host side, not on the timed path).
//
// Restates the traffic of tests/benchmarks/synthetic_network/synthetic_network.cc
// so the engine and the oracle see the same deterministic, timestamp-ordered
// input the reference app would inject (with fixed seeds instead of time(NULL)).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "gnoc.h"

namespace {

// glibc drand48_r: x <- (0x5DEECE66D x + 0xB) mod 2^48, result x / 2^48;
// srand48_r(seed): x = (seed << 16) | 0x330E  (common/misc/random.h:15-28).
struct Drand48
{
   uint64_t x;
   explicit Drand48(long seed) { x = ((uint64_t) (uint32_t) seed << 16) | 0x330Eull; }
   double next()
   {
      x = (0x5DEECE66Dull * x + 0xBull) & ((1ull << 48) - 1);
      return (double) x / 281474976710656.0;   // exact: 48-bit mantissa
   }
};

// NetworkModelEMeshHopByHop::computeMemoryControllerPositions, emesh_hop_by_hop.cc:323-364
std::vector<uint32_t> mc_positions(int W, int H, int num)
{
   std::vector<uint32_t> out;
   const int mw = (int) std::floor(std::sqrt((double) num));
   const int mh = (int) std::ceil(1.0 * num / mw);
   int k = 0;
   for (int j = 0; j < mh && k < num; j++)
      for (int i = 0; i < mw && k < num; i++)
      {
         int sx = W / mw, sy = H / mh;
         const int bx = i * sx, by = j * sy;
         if (i == mw - 1) sx = W - (mw - 1) * sx;
         if (j == mh - 1) sy = H - (mh - 1) * sy;
         out.push_back((uint32_t) ((bx + sx / 2) + (by + sy / 2) * W));
         k++;
      }
   return out;
}

}  // namespace

extern "C" int gnoc_trace_synthetic(int32_t W, int32_t H, double f, double load, uint64_t ppt, uint32_t payload,
                                    uint64_t seed, double hot_frac, int32_t num_hot, uint64_t* inject_ps,
                                    uint32_t* src, uint32_t* dst, uint32_t* bits, size_t capacity, size_t* n_out)
{
   return gnoc_trace_synthetic_pattern(GNOC_TRAFFIC_UNIFORM_RANDOM, W, H, f, load, ppt, payload, seed, hot_frac,
                                       num_hot, inject_ps, src, dst, bits, capacity, n_out);
}

extern "C" int gnoc_trace_synthetic_pattern(int32_t pattern, int32_t W, int32_t H, double f, double load, uint64_t ppt,
                                            uint32_t payload, uint64_t seed, double hot_frac, int32_t num_hot,
                                            uint64_t* inject_ps, uint32_t* src, uint32_t* dst, uint32_t* bits,
                                            size_t capacity, size_t* n_out)
{
   if (W <= 0 || H <= 0 || !(f > 0) || !(load > 0) || load > 1.0 || !n_out) return GNOC_EINVAL;
   if (pattern < GNOC_TRAFFIC_UNIFORM_RANDOM || pattern > GNOC_TRAFFIC_NEAREST_NEIGHBOR) return GNOC_EINVAL;
   const int N = W * H;
   const bool pow2 = (N & (N - 1)) == 0;
   // bit complement and shuffle assert a power-of-two tile count (synthetic_network.cc:290, 299)
   if ((pattern == GNOC_TRAFFIC_BIT_COMPLEMENT || pattern == GNOC_TRAFFIC_SHUFFLE) && !pow2) return GNOC_EINVAL;
   const uint64_t total = (uint64_t) N * ppt;
   *n_out = (size_t) total;
   if (!inject_ps) return GNOC_OK;
   if (capacity < total || !src || !dst || !bits) return GNOC_EINVAL;
   if (hot_frac > 0 && num_hot <= 0) return GNOC_EINVAL;

   // A tile's destination schedule: send_vec[k % size] (synthetic_network.cc:183).
   // uniformRandomTrafficGenerator (:232-286): send_matrix[slot][sender], an LCG
   // schedule; the other patterns (:288-341) send every packet to one tile.
   std::vector<uint32_t> sendm;
   if (pattern == GNOC_TRAFFIC_UNIFORM_RANDOM)
   {
      sendm.resize((size_t) N * N);
      sendm[0] = (uint32_t) (N / 2);
      for (int i = 0; i < N; i++)
      {
         if (i) sendm[(size_t) i * N] = sendm[(size_t) (i - 1) * N + 1 % N];
         for (int j = 1; j < N; j++)
            sendm[(size_t) i * N + j] = (uint32_t) ((13ull * sendm[(size_t) i * N + j - 1] + 5) % (uint64_t) N);
      }
      // the reference asserts every slot row and sender column is a permutation (:254-279)
      std::vector<uint8_t> seen(N);
      for (int i = 0; i < N; i++)
      {
         std::fill(seen.begin(), seen.end(), 0);
         for (int j = 0; j < N; j++) seen[sendm[(size_t) i * N + j]] = 1;
         for (int j = 0; j < N; j++) if (!seen[j]) return GNOC_EINVAL;
      }
   }
   else
   {
      sendm.resize(N);
      int nbits = 0;
      while ((1 << (nbits + 1)) <= N) nbits++;   // floorLog2
      for (int t = 0; t < N; t++)
      {
         const int sx = t % W, sy = t / W;   // computeEMeshPosition (:350-354)
         int64_t d = 0;
         switch (pattern)
         {
            case GNOC_TRAFFIC_BIT_COMPLEMENT: d = (~t) & (N - 1); break;                              // :288-295
            case GNOC_TRAFFIC_SHUFFLE: d = ((t >> (nbits - 1)) & 1) | ((t << 1) & (N - 1)); break;     // :297-305
            case GNOC_TRAFFIC_TRANSPOSE: d = (int64_t) sx * W + sy; break;                            // :307-317
            case GNOC_TRAFFIC_TORNADO: d = (int64_t) ((sy + H / 2) % H) * W + (sx + W / 2) % W; break; // :319-329
            default: d = (int64_t) ((sy + 1) % H) * W + (sx + 1) % W; break;                          // :331-341
         }
         if (d < 0 || d >= N) return GNOC_EINVAL;   // transpose of a non-square mesh
         sendm[t] = (uint32_t) d;
      }
   }
   const bool fixed = pattern != GNOC_TRAFFIC_UNIFORM_RANDOM;
   const std::vector<uint32_t> hot = hot_frac > 0 ? mc_positions(W, H, num_hot) : std::vector<uint32_t>();

   // Per tile: the cycle of each send (Bernoulli per cycle while packets remain,
   // synthetic_network.cc:182-221, canSendPacket :230-233).
   std::vector<std::vector<uint64_t>> cyc(N);
   std::vector<std::vector<uint32_t>> dsts(N);
   auto work = [&](int t0, int t1) {
      for (int t = t0; t < t1; t++)
      {
         Drand48 r((long) (seed + (uint64_t) t));
         Drand48 rh((long) (seed + 0x5bd1e995ull + (uint64_t) t));
         auto& c = cyc[t];
         auto& d = dsts[t];
         c.resize(ppt);
         d.resize(ppt);
         uint64_t sent = 0;
         for (uint64_t cycle = 0; sent < ppt; cycle++)
         {
            if (r.next() * 1.0 < load)
            {
               uint32_t dd = fixed ? sendm[t] : sendm[(size_t) (sent % (uint64_t) N) * N + t];
               if (hot_frac > 0 && rh.next() < hot_frac)
                  dd = hot[(size_t) (rh.next() * (double) hot.size()) % hot.size()];
               c[sent] = cycle;
               d[sent] = dd;
               sent++;
            }
         }
      }
   };
   const int nth = (int) std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
   std::vector<std::thread> th;
   for (int k = 0; k < nth; k++) th.emplace_back(work, (int) ((int64_t) N * k / nth), (int) ((int64_t) N * (k + 1) / nth));
   for (auto& x : th) x.join();

   // global (cycle, src) order via counting sort on cycle; stable in src
   uint64_t maxc = 0;
   for (int t = 0; t < N; t++) if (ppt) maxc = std::max(maxc, cyc[t][ppt - 1]);
   std::vector<uint64_t> start(maxc + 2, 0);
   for (int t = 0; t < N; t++) for (uint64_t k = 0; k < ppt; k++) start[cyc[t][k] + 1]++;
   for (uint64_t k = 1; k < start.size(); k++) start[k] += start[k - 1];
   // ONE_CYCLE = Latency(1, f) in picoseconds (synthetic_network.cc:224)
   const uint64_t one = (uint64_t) std::ceil(((double) 1000 * 1.0) / f);
   const uint32_t nbits = (64u + payload) * 8u;   // NetPacket::bufferSize()*8, network.cc:705-708
   for (int t = 0; t < N; t++)
      for (uint64_t k = 0; k < ppt; k++)
      {
         const uint64_t pos = start[cyc[t][k]]++;
         inject_ps[pos] = cyc[t][k] * one;
         src[pos] = (uint32_t) t;
         dst[pos] = dsts[t][k];
         bits[pos] = nbits;
      }
   return GNOC_OK;
}

// ---------------------------------------------------------------------------
// on-disk trace format (include/gnoc.h, gnoc_trace_header)
// ---------------------------------------------------------------------------
static_assert(sizeof(gnoc_trace_header) == 128, "trace header is 128 bytes");

extern "C" int gnoc_trace_file_write(const char* path, const gnoc_config* cfg, const gnoc_packets* pk, size_t n)
{
   return gnoc_trace_file_write_q(path, cfg, nullptr, pk, n);
}

extern "C" int gnoc_trace_file_write_q(const char* path, const gnoc_config* cfg, const gnoc_trace_queue* q,
                                       const gnoc_packets* pk, size_t n)
{
   if (!path || !cfg || !pk) return GNOC_EINVAL;
   if (n && (!pk->inject_ps || !pk->src || !pk->dst || !pk->bits)) return GNOC_EINVAL;
   FILE* f = std::fopen(path, "wb");
   if (!f) return GNOC_EINVAL;
   gnoc_trace_header h;
   std::memset(&h, 0, sizeof(h));
   std::memcpy(h.magic, GNOC_TRACE_MAGIC, 8);
   h.version = 2;
   h.header_bytes = sizeof(h);
   h.num_packets = n;
   h.cfg = *cfg;
   h.ma_type = q ? q->ma_type : GNOC_MOVING_AVG_NONE;
   h.ma_window = q ? q->ma_window : 1u;
   bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1;
   ok = ok && (n == 0 || std::fwrite(pk->inject_ps, 8, n, f) == n);
   ok = ok && (n == 0 || std::fwrite(pk->src, 4, n, f) == n);
   ok = ok && (n == 0 || std::fwrite(pk->dst, 4, n, f) == n);
   ok = ok && (n == 0 || std::fwrite(pk->bits, 4, n, f) == n);
   if (pk->flags) ok = ok && (n == 0 || std::fwrite(pk->flags, 4, n, f) == n);
   else
   {
      std::vector<uint32_t> z(std::min<size_t>(n, 1 << 20), 0);
      for (size_t done = 0; ok && done < n; done += z.size())
      {
         const size_t k = std::min(z.size(), n - done);
         ok = std::fwrite(z.data(), 4, k, f) == k;
      }
   }
   ok = (std::fclose(f) == 0) && ok;
   return ok ? GNOC_OK : GNOC_EINVAL;
}

extern "C" int gnoc_trace_file_read(const char* path, gnoc_config* cfg_out, uint64_t* inject_ps, uint32_t* src,
                                    uint32_t* dst, uint32_t* bits, uint32_t* flags, size_t capacity, size_t* n_out)
{
   return gnoc_trace_file_read_q(path, cfg_out, nullptr, inject_ps, src, dst, bits, flags, capacity, n_out);
}

extern "C" int gnoc_trace_file_read_q(const char* path, gnoc_config* cfg_out, gnoc_trace_queue* q_out,
                                      uint64_t* inject_ps, uint32_t* src, uint32_t* dst, uint32_t* bits, uint32_t* flags,
                                      size_t capacity, size_t* n_out)
{
   if (!path || !n_out) return GNOC_EINVAL;
   FILE* f = std::fopen(path, "rb");
   if (!f) return GNOC_EINVAL;
   gnoc_trace_header h;
   bool ok = std::fread(&h, sizeof(h), 1, f) == 1;
   ok = ok && std::memcmp(h.magic, GNOC_TRACE_MAGIC, 8) == 0 && (h.version == 1 || h.version == 2) &&
        h.header_bytes == sizeof(h);
   if (!ok)
   {
      std::fclose(f);
      return GNOC_ETRACE;
   }
   const size_t n = (size_t) h.num_packets;
   *n_out = n;
   if (cfg_out) *cfg_out = h.cfg;
   if (q_out)
   {
      // version 1 carried no queue settings: the reference's defaults (no moving average)
      q_out->ma_type = h.version >= 2 ? h.ma_type : GNOC_MOVING_AVG_NONE;
      q_out->ma_window = h.version >= 2 ? h.ma_window : 1u;
   }
   if (!inject_ps)
   {
      std::fclose(f);
      return GNOC_OK;
   }
   if (capacity < n || !src || !dst || !bits)
   {
      std::fclose(f);
      return GNOC_EINVAL;
   }
   ok = n == 0 || std::fread(inject_ps, 8, n, f) == n;
   ok = ok && (n == 0 || std::fread(src, 4, n, f) == n);
   ok = ok && (n == 0 || std::fread(dst, 4, n, f) == n);
   ok = ok && (n == 0 || std::fread(bits, 4, n, f) == n);
   if (flags) ok = ok && (n == 0 || std::fread(flags, 4, n, f) == n);
   std::fclose(f);
   return ok ? GNOC_OK : GNOC_ETRACE;
}

// Run fn(k) for k in [0, nt): blocks 1.. on new threads where the host gives them,
// the rest (and block 0) on the calling thread -- a thread the system refuses
// (std::system_error) costs parallelism, not the call.
template <class F>
static void run_blocks(size_t nt, F&& fn)
{
   std::vector<std::thread> th;
   size_t k = 1;
   try
   {
      th.reserve(nt);
      for (; k < nt; k++) th.emplace_back(fn, k);
   }
   catch (...)
   {
   }
   for (size_t r = k; r < nt; r++) fn(r);
   fn(0);
   for (auto& x : th) x.join();
}

static int pack_trace(const gnoc_packets* pk, size_t n, uint16_t* dt, uint16_t* src, uint16_t* dst, uint16_t* bits,
                      uint8_t* flags, uint64_t* abs_ps, size_t abs_cap, gnoc_pack_info* info);

// The delta wire format's encoder (include/gnoc.h gnoc_pack_trace): blocks of the
// trace on the host's threads; pass 1 validates and counts each block's escapes,
// pass 2 writes, each block's escapes at its offset in abs_ps.  Never throws
// across the C boundary: an allocation failure is GNOC_ENOMEM.
extern "C" int gnoc_pack_trace(const gnoc_packets* pk, size_t n, uint16_t* dt, uint16_t* src, uint16_t* dst,
                               uint16_t* bits, uint8_t* flags, uint64_t* abs_ps, size_t abs_cap, gnoc_pack_info* info)
{
   try
   {
      return pack_trace(pk, n, dt, src, dst, bits, flags, abs_ps, abs_cap, info);
   }
   catch (...)
   {
      return GNOC_ENOMEM;
   }
}

static int pack_trace(const gnoc_packets* pk, size_t n, uint16_t* dt, uint16_t* src, uint16_t* dst, uint16_t* bits,
                      uint8_t* flags, uint64_t* abs_ps, size_t abs_cap, gnoc_pack_info* info)
{
   if (!pk || !info) return GNOC_EINVAL;
   if (n && (!pk->inject_ps || !pk->src || !pk->dst || !pk->bits || !dt || !src || !dst)) return GNOC_EINVAL;
   const uint64_t* t = pk->inject_ps;
   const uint64_t t0 = n ? t[0] : 0;
   const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
   const size_t nt = std::max<size_t>(1, std::min<size_t>({ (size_t) hw, (size_t) 16, n / 65536 + 1 }));
   const size_t blk = (n + nt - 1) / std::max<size_t>(nt, 1);
   struct Part
   {
      uint64_t esc = 0;
      uint32_t fl = 0;
      bool bad = false, one = true;
   };
   std::vector<Part> part(nt);
   const uint32_t b0 = n ? pk->bits[0] : 0u;
   auto count = [&](size_t k) {
      Part& q = part[k];
      const size_t lo = k * blk, hi = std::min(n, lo + blk);
      for (size_t i = lo; i < hi; i++)
      {
         const uint64_t d = t[i] - (i ? t[i - 1] : t0);
         q.esc += d >= 0xFFFFull;
         const uint32_t f = pk->flags ? pk->flags[i] : 0u;
         q.fl |= f;
         q.one &= pk->bits[i] == b0;
         q.bad |= pk->src[i] > 0xFFFFu || pk->dst[i] > 0xFFFFu || pk->bits[i] > 0xFFFFu || f > 0xFFu;
      }
   };
   run_blocks(nt, count);
   uint64_t nesc = 0;
   uint32_t fl = 0;
   bool bad = false, one = true;
   std::vector<uint64_t> eoff(nt);
   for (size_t k = 0; k < nt; k++)
   {
      eoff[k] = nesc;
      nesc += part[k].esc;
      fl |= part[k].fl;
      bad |= part[k].bad;
      one &= part[k].one;
   }
   info->t0 = t0;
   info->n_abs = nesc;
   info->bits_all = one ? b0 : 0xFFFFFFFFu;
   info->flags_any = fl;
   if (bad || nesc > abs_cap || (nesc && !abs_ps) || (!one && !bits) || (fl && !flags)) return GNOC_EINVAL;
   auto write = [&](size_t k) {
      const size_t lo = k * blk, hi = std::min(n, lo + blk);
      uint64_t e = eoff[k];
      for (size_t i = lo; i < hi; i++)
      {
         const uint64_t d = t[i] - (i ? t[i - 1] : t0);
         if (d >= 0xFFFFull)
         {
            dt[i] = 0xFFFFu;
            abs_ps[e++] = t[i];
         }
         else dt[i] = (uint16_t) d;
         src[i] = (uint16_t) pk->src[i];
         dst[i] = (uint16_t) pk->dst[i];
         if (bits) bits[i] = (uint16_t) pk->bits[i];
         if (flags) flags[i] = (uint8_t) (pk->flags ? pk->flags[i] : 0u);
      }
   };
   run_blocks(nt, write);
   return GNOC_OK;
}
