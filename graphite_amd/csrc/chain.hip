// chain.hip -- v4 engine: the X and Y phases of the port DAG as port CHAINS
// processed in time windows, records flowing from port to port through LDS.
//
// Under XY routing (network_model_emesh_hop_by_hop.cc:229-240) a row's RIGHT
// ports form a chain RIGHT(0,y) -> RIGHT(1,y) -> ... : every record a RIGHT
// port emits either continues to the next RIGHT port or turns (UP / DOWN / SELF
// of the next tile).  LEFT, UP and DOWN ports form chains the same way.  A
// chain port's arrival stream is the (t, id)-merge of the chain's own stream and
// a few "insert" slots written by earlier phases (IN_LOCAL for X ports; IN_LOCAL,
// IN_W, IN_E for Y ports).
//
// Time is cut into windows [w D, (w+1) D), D = 2^dshift ps, the last one
// unbounded.  One workgroup task = (chain, window): it walks the chain's ports
// in order, keeping the window's arrival stream in LDS:
//   port i:  stream (sorted)  --FIFO max-plus scan-->  departures
//            continuing departures with t' < window end stay in LDS and are
//            merged with port i+1's inserts of this window; the rest turn
//            (HBM stores into the next ports' slots, positions = route counts)
//            or spill (t' >= window end: HBM, taken by task (chain, w+1)).
// Hand-off, one per (port, window): task (chain, w) publishes port i's queue
// state after window w (tail X, route counts, history-tree "no gap yet" bit)
// and the port's still-unconsumed spill range; task (chain, w+1) polls it
// (8-byte epoch-tagged granules, sc1 stores and loads, MI355X_MICROARCH.md
// "Valid forms").  Tasks are handed out window-major, strictly in order to
// running workgroups, so a task's predecessor is always running or done.
//
// The history tree's serial state (queue_model_history_tree.cc:58-64) only
// matters while a queue has never idled; without the M/G/1 branch it is the
// FIFO recurrence, so the chain runs FIFO and checks, per record, the branch
// condition X > t + p while the port has had no gap.  If it would fire (or an
// earlier level wrote exception tails, or a window overflows LDS) the kernel
// raises a flag and the host reruns the batch (smaller windows / level engine).
#include "common.h"

namespace gnoc {
namespace ch {

#ifndef CH_T_V
#define CH_T_V 256
#endif
constexpr int T = CH_T_V;                 // threads per workgroup
constexpr int NWV = T / 64;
// threads that carry the descriptor (32) / insert-bounds (<= 6) prefetches: other
// waves than wave 0 (which polls) when there are some
constexpr uint32_t DESC_T0 = NWV >= 2 ? 64u : 0u;
constexpr uint32_t BND_T0 = NWV >= 3 ? 128u : 32u;
#ifndef CH_CAP_V
#define CH_CAP_V (8 * CH_T_V)
#endif
constexpr int CAP = CH_CAP_V;             // stream records per (port, window)
constexpr int PER = CAP / T;              // records per thread
#ifndef CH_ICAP_V
#define CH_ICAP_V (2 * CH_T_V)
#endif
constexpr int ICAP = CH_ICAP_V;           // inserts per (port, window), + spill-ins of the slow path
constexpr int IPER = ICAP / T;
#ifndef CH_MINW
#define CH_MINW 3                         // waves per SIMD the registers must leave room for (3 workgroups per CU)
#endif
constexpr int NLMAX = 3;                  // local insert lists (Y ports: LOCAL, W, E)
constexpr int SW = 8;                     // state words per (chain port, window)
constexpr uint32_t F_RETRY = 1u;          // a window overflowed LDS: rerun with smaller windows
constexpr uint32_t F_FALLBACK = 2u;       // M/G/1 would fire, exception tails, ...: rerun on the level engine
constexpr uint32_t F_ROUTE = 4u;          // route-count invariant broken (internal error)
constexpr uint32_t F_TIMEOUT = 8u;        // a hand-off wait timed out
constexpr uint32_t F_ANY = F_RETRY | F_FALLBACK | F_ROUTE | F_TIMEOUT;
constexpr uint64_t SPIN_CYCLES = 1ull << 31;
constexpr uint64_t M48 = (1ull << 48) - 1;
constexpr uint64_t OFF_LIM = (1ull << 32) - 4096;   // time offsets within a window (32-bit cycle math)
constexpr uint32_t NONE = 0xFFFFFFFFu;

// LDS index padding: one u64 per 32 entries, so a thread's contiguous segment
// (stride PER across lanes) hits distinct banks.
__host__ __device__ constexpr uint32_t pad(uint32_t r) { return r + (r >> 5); }
constexpr int CAPP = CAP + CAP / 32;

// Route-count fields of a chain port's outputs: SELF, the chain direction, UP,
// DOWN (an X port never sends the opposite X way; a Y port only SELF or on).
__host__ __device__ __forceinline__ uint32_t field_of(uint32_t nd, uint32_t cont)
{
   return nd == cont ? 1u : nd == P_SELF ? 0u : nd == P_UP ? 2u : 3u;
}

}  // namespace ch

// One port of a chain (k_chain_plan): output slots of the next tile per route
// field, insert slots of this port.  128 bytes: one wave copies it.
struct __attribute__((aligned(16))) ChainPort
{
   uint64_t obase[4];    // output slot base per field (SELF, cont, UP, DOWN)
   uint64_t ibase[3];    // insert slot bases (IN_LOCAL, IN_W, IN_E)
   uint32_t ocap[4];     // output slot capacities
   uint32_t icnt[3];     // insert slot record counts
   uint32_t port, tile, dir, cont;   // cont: the chain direction
   uint32_t nx, ny, rl, nl;          // next tile, R + Lk (ps), local insert lists
   uint32_t pad0[3];
};
static_assert(sizeof(ChainPort) == 128, "ChainPort is one 128-B line");

struct ChainArgs
{
   DevCfg c;
   const ChainPort* cp;           // [nch * len] (this phase)
   const uint32_t* bt;            // [(cpi * nl + j) * (nW + 1) + w] window bounds of insert slots
   Rec* recs;
   uint64_t* samp_t;
   uint32_t* samp_id;
   uint64_t* st;                  // [(cpi + cp0) * nW + w] * SW  hand-off state
   unsigned long long* port_sum;
   unsigned long long* port_cnt;
   unsigned long long* port_flit;
   unsigned long long* port_last;
   unsigned* errflag;             // [0] route invariant, [2] exception tails exist, [4] chain flags
   unsigned* ctr;                 // dequeue head
   uint32_t nch, len, nW, dshift;
   uint32_t cp0;                  // state index offset of this phase
   uint32_t pad0;
   uint64_t etag;                 // epoch << 48
   uint64_t* stamps;              // debug (GNOC_STAMPS=1): [(task * len + i) * 16 + k] phase stamps, else null
   uint32_t exp;                  // debug (GNOC_CHAIN_EXPERIMENT, timing only, results wrong): 1 no HBM
                                  // stores, 2 no hand-off waits, 4 no merge searches
   uint32_t pad1;
};

namespace ch {

struct Smem
{
   uint64_t key[CAPP];            // (t - wbase) << 32 | id, sorted
   uint32_t aux[CAPP];            // dx | dy << 10 | F << 20
   uint64_t ikey[ICAP];           // next port's inserts, one sorted list; the slow path's spill-ins behind them
   uint32_t iaux[ICAP];
   uint64_t rkey[ICAP];           // Y ports: the three insert slots' ranges as fetched (premerge -> ikey)
   uint32_t raux[ICAP];
   ChainPort cp[3];               // ports i, i+1, i+2 (ring)
   uint32_t blo[2][NLMAX], bhi[2][NLMAX];   // window bounds of ports i+1, i+2 (ring)
   uint32_t ioff[NLMAX + 1];      // insert list offsets (NL local lists, end)
   uint32_t ioff_next[NLMAX];
   uint64_t wA[NWV], wB[NWV], wC[NWV];
   uint64_t X_in, ssum;
   uint32_t cnt_in[4];
   uint32_t mode_in, n, n_inwin, first_gap, first_fire;
   uint32_t Kpp, Pep;             // predecessor's spill range of this port
   uint32_t Kout, Pend;           // this window's, after it
   uint32_t P0cur, nin_prev, ncont_prev;   // this port's chain input: records before / kept / all of this window
   uint32_t sp_skip, sp_take, abort_, next_task, published;
};

__device__ __forceinline__ uint64_t ld1(const uint64_t* p)
{
   return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st1(uint64_t* p, uint64_t v)
{
   __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// LDS-only workgroup barrier (no global store is read back by the workgroup).
__device__ __forceinline__ void bar()
{
   asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void mp(uint64_t& A, uint64_t& B, uint64_t a2, uint64_t b2)
{
   const uint64_t nb = B + a2;
   B = nb > b2 ? nb : b2;
   A += a2;
}
__device__ __forceinline__ uint32_t cf(uint64_t c, uint32_t f) { return (uint32_t) ((c >> (16 * f)) & 0xFFFFu); }

// Max-plus aggregate of a run of requests: X -> max(X + A, B); C = route counts
// (4 x 16-bit fields).  (A, B) of one request: (F, tc + F), cycles relative to
// the window's base cycle (32-bit).
struct Agg
{
   uint32_t A, B;
   uint64_t C;
};
__device__ __forceinline__ Agg agg_op(const Agg& x, const Agg& y)   // x, then y
{
   Agg r;
   r.A = x.A + y.A;
   const uint32_t nb = x.B + y.A;
   r.B = nb > y.B ? nb : y.B;
   r.C = x.C + y.C;
   return r;
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ uint32_t dpp32(uint32_t v)
{
   return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, CTRL, RM, BM, false);
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ uint64_t dpp64(uint64_t v)
{
   const uint32_t lo = dpp32<CTRL, RM, BM>((uint32_t) v), hi = dpp32<CTRL, RM, BM>((uint32_t) (v >> 32));
   return (uint64_t) lo | ((uint64_t) hi << 32);
}
// The identity (0, 0, 0) is what DPP leaves in lanes without a source (B >= 0).
template <int CTRL, int RM, int BM>
__device__ __forceinline__ Agg dpp_agg(const Agg& v)
{
   Agg r;
   r.A = dpp32<CTRL, RM, BM>(v.A);
   r.B = dpp32<CTRL, RM, BM>(v.B);
   r.C = dpp64<CTRL, RM, BM>(v.C);
   return r;
}
// Inclusive wave scan (GFX9 DPP: row_shr 1, 2, 4, 8; row_bcast 15, 31).
__device__ __forceinline__ Agg wave_scan(Agg v)
{
   v = agg_op(dpp_agg<0x111, 0xF, 0xF>(v), v);
   v = agg_op(dpp_agg<0x112, 0xF, 0xF>(v), v);
   v = agg_op(dpp_agg<0x114, 0xF, 0xF>(v), v);
   v = agg_op(dpp_agg<0x118, 0xF, 0xF>(v), v);
   v = agg_op(dpp_agg<0x142, 0xA, 0xF>(v), v);
   v = agg_op(dpp_agg<0x143, 0xC, 0xF>(v), v);
   return v;
}
// Wave sums (same DPP pattern); the total is in lane 63.
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v)
{
   v += dpp32<0x111, 0xF, 0xF>(v);
   v += dpp32<0x112, 0xF, 0xF>(v);
   v += dpp32<0x114, 0xF, 0xF>(v);
   v += dpp32<0x118, 0xF, 0xF>(v);
   v += dpp32<0x142, 0xA, 0xF>(v);
   v += dpp32<0x143, 0xC, 0xF>(v);
   return v;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v)
{
   v += dpp64<0x111, 0xF, 0xF>(v);
   v += dpp64<0x112, 0xF, 0xF>(v);
   v += dpp64<0x114, 0xF, 0xF>(v);
   v += dpp64<0x118, 0xF, 0xF>(v);
   v += dpp64<0x142, 0xA, 0xF>(v);
   v += dpp64<0x143, 0xC, 0xF>(v);
   return v;
}
__device__ __forceinline__ uint32_t sgpr(uint32_t v) { return (uint32_t) __builtin_amdgcn_readfirstlane((int) v); }
__device__ __forceinline__ uint64_t sgpr64(uint64_t v)
{
   return (uint64_t) sgpr((uint32_t) v) | ((uint64_t) sgpr((uint32_t) (v >> 32)) << 32);
}

// Lower bound (number of entries < k) in the sorted u64 array a[0, n), by
// binary lifting: n is block-uniform, so every lane runs floor(log2 n) + 1
// iterations with no divergence; one LDS read each.
__device__ __forceinline__ uint32_t lb(const uint64_t* a, uint32_t n, uint64_t k)
{
   uint32_t pos = 0;
   for (uint32_t step = n ? 1u << (31 - __builtin_clz(n)) : 0u; step; step >>= 1)
   {
      const uint32_t q = pos + step;
      const uint64_t v = a[(q <= n ? q : n) - 1];
      pos = (q <= n && v < k) ? q : pos;
   }
   return pos;
}
// same over the padded stream array
__device__ __forceinline__ uint32_t lbp(const uint64_t* a, uint32_t n, uint64_t k)
{
   uint32_t pos = 0;
   for (uint32_t step = n ? 1u << (31 - __builtin_clz(n)) : 0u; step; step >>= 1)
   {
      const uint32_t q = pos + step;
      const uint64_t v = a[pad((q <= n ? q : n) - 1)];
      pos = (q <= n && v < k) ? q : pos;
   }
   return pos;
}

__device__ __forceinline__ void flag(const ChainArgs& a, uint32_t f)
{
   if (!a.exp) atomicOr(a.errflag + 4, f);
}
__device__ __forceinline__ bool flagged(const ChainArgs& a)
{
   return (__hip_atomic_load(a.errflag + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & F_ANY) != 0;
}

// One wave copies a 128-B port descriptor.
__device__ __forceinline__ void load_cp(ChainPort* dst, const ChainPort* src, uint32_t lane)
{
   if (lane < 32) reinterpret_cast<uint32_t*>(dst)[lane] = reinterpret_cast<const uint32_t*>(src)[lane];
}
// The same in two halves: the load a step ahead into a register, the LDS store later
// (a store right behind its load would stall the wave for the whole round trip).
__device__ __forceinline__ uint32_t fetch_cp(const ChainPort* src, uint32_t lane)
{
   return lane < 32 ? reinterpret_cast<const uint32_t*>(src)[lane] : 0u;
}
__device__ __forceinline__ void put_cp(ChainPort* dst, uint32_t v, uint32_t lane)
{
   if (lane < 32) reinterpret_cast<uint32_t*>(dst)[lane] = v;
}
// Window bounds [lo, hi) of the insert slots of chain port cpi (lanes < 2 nl).
__device__ __forceinline__ void load_bounds(Smem& sm, const ChainArgs& a, uint32_t slot, uint32_t cpi, uint32_t nl,
                                            uint32_t w, uint32_t lane)
{
   if (lane < 2 * nl)
   {
      const uint32_t j = lane < nl ? lane : lane - nl;
      const uint32_t v = a.bt[((uint64_t) cpi * nl + j) * (a.nW + 1) + w + (lane < nl ? 0u : 1u)];
      if (lane < nl) sm.blo[slot][j] = v;
      else sm.bhi[slot][j] = v;
   }
}

__device__ __forceinline__ uint32_t fetch_bounds(const ChainArgs& a, uint32_t cpi, uint32_t nl, uint32_t w, uint32_t lane)
{
   if (lane >= 2 * nl) return 0u;
   const uint32_t j = lane < nl ? lane : lane - nl;
   return a.bt[((uint64_t) cpi * nl + j) * (a.nW + 1) + w + (lane < nl ? 0u : 1u)];
}
__device__ __forceinline__ void put_bounds(Smem& sm, uint32_t slot, uint32_t v, uint32_t nl, uint32_t lane)
{
   if (lane < 2 * nl)
   {
      if (lane < nl) sm.blo[slot][lane] = v;
      else sm.bhi[slot][lane - nl] = v;
   }
}

// Poll the state words [0, nw) of block s until all carry the epoch tag (lane
// q < nw holds word q).  Wave-wide; false on abort.
__device__ bool poll_words(const ChainArgs& a, const uint64_t* s, uint32_t nw, uint32_t lane, uint64_t& v)
{
   if (a.exp & 2u) return true;
   const uint64_t t0 = __builtin_amdgcn_s_memtime();
   for (;;)
   {
      bool ok = true;
      if (lane < nw) ok = (v & ~M48) == a.etag;
      if (__all(ok)) return true;
      if (__builtin_amdgcn_s_memtime() - t0 > SPIN_CYCLES)
      {
         if (lane == 0) flag(a, F_TIMEOUT);
         return false;
      }
      if (flagged(a)) return false;
      __builtin_amdgcn_s_sleep(1);
      if (lane < nw) v = ld1(s + lane);
   }
}

// Issue the loads of a port's local inserts of this window (registers).
template <int NL>
__device__ __forceinline__ uint32_t fetch_inserts(Smem& sm, const ChainArgs& a, uint32_t ring, uint32_t br,
                                                  Rec (&iv)[IPER])
{
   const uint32_t tid = threadIdx.x;
   const ChainPort& P = sm.cp[ring];
   uint32_t off[NL + 1], lo[NL];
   off[0] = 0;
#pragma unroll
   for (int j = 0; j < NL; j++)
   {
      // bounds come from sorted slots; clamped so that nothing can load out of range
      lo[j] = min(sm.blo[br][j], P.icnt[j]);
      const uint32_t hi = min(max(sm.bhi[br][j], lo[j]), P.icnt[j]);
      off[j + 1] = off[j] + (hi - lo[j]);
   }
   const uint32_t itot = off[NL];
   if (tid == 0)
      for (int j = 1; j < NL; j++) sm.ioff_next[j] = off[j];
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = tid + (uint32_t) q * T;
      iv[q].t = 0;
      iv[q].id = 0;
      iv[q].aux = 0;
      if (g < itot && g < (uint32_t) ICAP)
      {
         uint32_t j = 0;
#pragma unroll
         for (int l = 1; l < NL; l++)
            if (g >= off[l]) j = (uint32_t) l;
         iv[q] = a.recs[P.ibase[j] + lo[j] + (g - off[j])];
      }
   }
   return itot;
}

// Fetched inserts into LDS as keys relative to wbase: X ports (one slot)
// straight into the insert list, Y ports into the staging lists (premerge).
template <int NL>
__device__ __forceinline__ bool store_inserts(Smem& sm, const Rec (&iv)[IPER], uint32_t itot, uint64_t wbase)
{
   const uint32_t tid = threadIdx.x;
   bool bad = false;
   uint64_t* K = NL > 1 ? sm.rkey : sm.ikey;
   uint32_t* X = NL > 1 ? sm.raux : sm.iaux;
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = tid + (uint32_t) q * T;
      if (g < itot && g < (uint32_t) ICAP)
      {
         const uint64_t dt = iv[q].t - wbase;
         bad |= dt >= OFF_LIM;
         K[g] = (dt << 32) | iv[q].id;
         X[g] = iv[q].aux;
      }
   }
   if (tid == 0)
   {
      sm.ioff[0] = 0;
      for (int j = 1; j < NL; j++) sm.ioff[j] = sm.ioff_next[j];
      sm.ioff[NL] = itot;
   }
   return bad;
}

// Y ports: the staged slot ranges (each sorted) merged into one sorted insert
// list: own index + lower bounds in the other two ranges.  Reads the staging
// lists (written before the preceding barrier); ikey is read after the next.
template <int NL>
__device__ __forceinline__ void premerge(Smem& sm, uint32_t itot)
{
   if (NL == 1) return;
   const uint32_t tid = threadIdx.x;
   uint32_t o[NL + 1];
#pragma unroll
   for (int l = 0; l <= NL; l++) o[l] = sm.ioff[l];
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = tid + (uint32_t) q * T;
      if (g >= itot || g >= (uint32_t) ICAP) continue;
      const uint64_t k = sm.rkey[g];
      uint32_t own = 0;
#pragma unroll
      for (int l = 1; l < NL; l++)
         if (g >= o[l]) own = (uint32_t) l;
      uint32_t pos = g - o[own];
#pragma unroll
      for (int l = 0; l < NL; l++)
         if ((uint32_t) l != own) pos += lb(sm.rkey + o[l], o[l + 1] - o[l], k);
      sm.ikey[pos] = k;
      sm.iaux[pos] = sm.raux[g];
   }
}

// Merge the kept records (registers: keys rk, aux ra, index ci among the kept;
// bit j of km marks one) with the sorted insert list sm.ikey[0, itot) into the
// stream sm.key/aux.  Position = own index + entries of the other list below
// (keys are unique: one record per packet per port).  The kept keys sit at
// key[pad(ci)], written before the barrier preceding this call.
__device__ void merge(Smem& sm, uint32_t nkeep, uint32_t itot, const uint64_t (&rk)[PER], const uint32_t (&ra)[PER],
                      uint32_t (&ci)[PER], uint32_t km, uint32_t exp, uint64_t* stp = nullptr)
{
   const uint32_t tid = threadIdx.x;
   if (exp & 4u)
   {
      // timing experiment: kept records then inserts, unsorted
      bar();
#pragma unroll
      for (int j = 0; j < PER; j++)
         if ((km >> j) & 1u) { sm.key[pad(ci[j])] = rk[j]; sm.aux[pad(ci[j])] = ra[j]; }
      for (uint32_t g = tid; g < itot; g += T) { sm.key[pad(nkeep + g)] = sm.ikey[g]; sm.aux[pad(nkeep + g)] = sm.iaux[g]; }
      if (tid == 0) sm.n = nkeep + itot;
      bar();
      return;
   }
   // kept records: inserts below the first one by search, then by advancing
   uint32_t cur = 0;
   bool first = true;
#pragma unroll
   for (int j = 0; j < PER; j++)
   {
      if (!((km >> j) & 1u)) continue;
      if (first) cur = lb(sm.ikey, itot, rk[j]);
      else
         while (cur < itot && sm.ikey[cur] < rk[j]) cur++;
      first = false;
      ci[j] += cur;
   }
   // inserts: own index + kept below
   uint64_t ik[IPER];
   uint32_t ia[IPER], pi[IPER];
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = tid + (uint32_t) q * T;
      pi[q] = NONE;
      ik[q] = 0;
      ia[q] = 0;
      if (g >= itot) continue;
      ik[q] = sm.ikey[g];
      ia[q] = sm.iaux[g];
      pi[q] = g + lbp(sm.key, nkeep, ik[q]);
   }
   if (stp && tid == 0) stp[10] = __builtin_amdgcn_s_memtime();
   bar();
   if (stp && tid == 0) stp[11] = __builtin_amdgcn_s_memtime();
#pragma unroll
   for (int j = 0; j < PER; j++)
      if ((km >> j) & 1u)
      {
         sm.key[pad(ci[j])] = rk[j];
         sm.aux[pad(ci[j])] = ra[j];
      }
#pragma unroll
   for (int q = 0; q < IPER; q++)
      if (pi[q] != NONE)
      {
         sm.key[pad(pi[q])] = ik[q];
         sm.aux[pad(pi[q])] = ia[q];
      }
   if (tid == 0) sm.n = nkeep + itot;
   bar();
}

// Cycles of a stream record relative to the window base cycle wb = max(wq - 1, 0):
// Time::toCycles at 1 GHz, ceil((wbase + off) / 1000) - wb, with wbase = 1000 wq + wr
// (32-bit division; off + wr + 999 < 2^32 by the OFF_LIM check on every key).
__device__ __forceinline__ uint32_t rcyc(uint32_t off, uint32_t wr, uint32_t d0)
{
   return (wr + off + 999u) / 1000u + d0;
}

// This thread's segment of the stream into registers and its aggregate.
__device__ __forceinline__ Agg load_segment(const Smem& sm, uint32_t a0, uint32_t cnt, uint32_t wr, uint32_t d0,
                                            uint32_t nx, uint32_t ny, uint32_t cont, uint64_t (&rk)[PER],
                                            uint32_t (&ra)[PER])
{
   Agg g;
   g.A = 0;
   g.B = 0;
   g.C = 0;
#pragma unroll
   for (int j = 0; j < PER; j++)
   {
      rk[j] = 0;
      ra[j] = 0;
      if ((uint32_t) j < cnt)
      {
         rk[j] = sm.key[pad(a0 + j)];
         ra[j] = sm.aux[pad(a0 + j)];
         const uint32_t p = aux_F(ra[j]);
         const uint32_t nb = g.B + p, b2 = rcyc((uint32_t) (rk[j] >> 32), wr, d0) + p;
         g.B = nb > b2 ? nb : b2;
         g.A += p;
         g.C += 1ull << (16 * field_of(xy_dir(nx, ny, aux_dx(ra[j]), aux_dy(ra[j])), cont));
      }
   }
   return g;
}

// Block scan: exclusive prefix of this thread, block totals.  One barrier.
__device__ __forceinline__ void block_scan(Smem& sm, const Agg& g, Agg& ex, Agg& tot)
{
   const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
   const Agg inc = wave_scan(g);
   if (lane == 63) { sm.wA[wv] = inc.A; sm.wB[wv] = inc.B; sm.wC[wv] = inc.C; }
   Agg e;   // exclusive within the wave: the inclusive value of lane - 1 (wave_shr 1)
   e.A = dpp32<0x138, 0xF, 0xF>(inc.A);
   e.B = dpp32<0x138, 0xF, 0xF>(inc.B);
   e.C = dpp64<0x138, 0xF, 0xF>(inc.C);
   bar();
   Agg p;
   p.A = 0;
   p.B = 0;
   p.C = 0;
   Agg t = p;
#pragma unroll
   for (int v = 0; v < NWV; v++)
   {
      Agg q;
      q.A = (uint32_t) sm.wA[v];
      q.B = (uint32_t) sm.wB[v];
      q.C = sm.wC[v];
      if ((uint32_t) v < wv) p = agg_op(p, q);
      t = agg_op(t, q);
   }
   ex = agg_op(p, e);
   tot = t;
}

// Spill-ins of this port (slow path): [Kpp, Pep) of its chain slot, written by
// earlier windows at the previous port; those with t in this window are merged
// into the stream (rk/ra: this thread's current segment [a0, a0 + cnt)).
// Returns the records taken; sets sm.sp_skip (consumed by earlier windows).
__device__ uint32_t spill_in(Smem& sm, const ChainArgs& a, uint64_t sbase, uint32_t spn, uint32_t sbuf, uint32_t n,
                             uint64_t wbase, uint64_t wlen, const uint64_t (&rk)[PER], const uint32_t (&ra)[PER],
                             uint32_t a0, uint32_t cnt)
{
   const uint32_t tid = threadIdx.x;
   Rec sv[IPER];
   uint32_t nb = 0, nt = 0;
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = tid + (uint32_t) q * T;
      sv[q].t = 0;
      sv[q].id = 0;
      sv[q].aux = 0;
      if (g < spn)
      {
         const uint64_t* r = reinterpret_cast<const uint64_t*>(a.recs + sbase + g);
         sv[q].t = ld1(r);
         const uint64_t ia = ld1(r + 1);
         sv[q].id = (uint32_t) ia;
         sv[q].aux = (uint32_t) (ia >> 32);
         nb += sv[q].t < wbase ? 1u : 0u;
         nt += (sv[q].t >= wbase && sv[q].t - wbase < wlen) ? 1u : 0u;
      }
   }
   if (nb) atomicAdd(&sm.sp_skip, nb);
   if (nt) atomicAdd(&sm.sp_take, nt);
   bar();
   const uint32_t skip = sm.sp_skip, take = sm.sp_take;
   if (!take || n + take > (uint32_t) CAP) return take;
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = tid + (uint32_t) q * T;
      if (g < spn && sv[q].t >= wbase && sv[q].t - wbase < wlen)
      {
         const uint32_t o = sbuf + (g - skip);
         sm.ikey[o] = ((sv[q].t - wbase) << 32) | sv[q].id;
         sm.iaux[o] = sv[q].aux;
      }
   }
   bar();
   uint32_t ps[PER];
#pragma unroll
   for (int j = 0; j < PER; j++) ps[j] = (uint32_t) j < cnt ? a0 + j + lb(sm.ikey + sbuf, take, rk[j]) : NONE;
   uint32_t pq[IPER];
   uint64_t qk[IPER];
   uint32_t qa[IPER];
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = tid + (uint32_t) q * T;
      pq[q] = NONE;
      qk[q] = 0;
      qa[q] = 0;
      if (g < take)
      {
         qk[q] = sm.ikey[sbuf + g];
         qa[q] = sm.iaux[sbuf + g];
         pq[q] = g + lbp(sm.key, n, qk[q]);
      }
   }
   bar();
#pragma unroll
   for (int j = 0; j < PER; j++)
      if (ps[j] != NONE)
      {
         sm.key[pad(ps[j])] = rk[j];
         sm.aux[pad(ps[j])] = ra[j];
      }
#pragma unroll
   for (int q = 0; q < IPER; q++)
      if (pq[q] != NONE)
      {
         sm.key[pad(pq[q])] = qk[q];
         sm.aux[pad(pq[q])] = qa[q];
      }
   if (tid == 0) sm.n = n + take;
   bar();
   return take;
}

// ---------------------------------------------------------------------------
// one task: chain c, window w
// ---------------------------------------------------------------------------
#define CH_STAMP(k)                                                                                         \
   do                                                                                                      \
   {                                                                                                       \
      if (a.stamps && threadIdx.x == 0)                                                                     \
         a.stamps[((uint64_t) tk * len + i) * 16 + (k)] = __builtin_amdgcn_s_memtime();                     \
   } while (0)

template <int NL>
__device__ void task(Smem& sm, const ChainArgs& a, uint32_t c, uint32_t w, uint32_t tk)
{
   const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
   const uint64_t wbase = (uint64_t) w << a.dshift;
   const uint64_t wlen = (w + 1 < a.nW) ? (1ull << a.dshift) : OFF_LIM;   // kept offsets: t' - wbase < wlen
   const uint64_t wq = wbase / 1000ull;
   const uint32_t wr = (uint32_t) (wbase - wq * 1000ull);
   const uint64_t wb = wq ? wq - 1 : 0;          // base cycle: every request of the window has tc > wb (w > 0)
   const uint32_t d0 = (uint32_t) (wq - wb);
   const uint32_t len = a.len, nW = a.nW;
   const uint32_t cpb = c * len;
   const int analytical = a.c.analytical;

   // ---- prologue: descriptors and insert bounds of ports 0 and 1, port 0's stream;
   // then the pipeline's first prefetches (port 1's inserts, port 2's descriptor and bounds)
   for (uint32_t x = tid; x < 64u + 4u * NL; x += T)
   {
      if (x < 32) load_cp(&sm.cp[0], a.cp + cpb, x);
      else if (x < 64) { if (len > 1) load_cp(&sm.cp[1], a.cp + cpb + 1, x - 32); }
      else if (x < 64u + 2u * NL) load_bounds(sm, a, 0, cpb, NL, w, x - 64);
      else if (len > 1) load_bounds(sm, a, 1, cpb + 1, NL, w, x - 64 - 2 * NL);
   }
   if (tid == 0)
   {
      sm.abort_ = 0;
      sm.P0cur = 0;      // port 0 has no chain input
      sm.nin_prev = 0;
      sm.ncont_prev = 0;
   }
   bar();
   uint64_t rk[PER];
   uint32_t ra[PER], ci[PER];
   Rec iv[IPER];             // the next port's inserts in flight
   uint32_t itot_cur = 0;    // their count
   uint32_t cpv = 0, bv = 0; // descriptor / bounds of the port after next, in flight (waves 1 / 2)
   {
      const uint32_t itot = fetch_inserts<NL>(sm, a, 0, 0, iv);
      const bool bad = store_inserts<NL>(sm, iv, itot, wbase);
      if (itot > (uint32_t) ICAP || itot > (uint32_t) CAP)
      {
         if (tid == 0) flag(a, F_RETRY);
         return;
      }
      if (bad) flag(a, F_FALLBACK);
      bar();
      premerge<NL>(sm, itot);
      bar();
#pragma unroll
      for (int j = 0; j < PER; j++) { rk[j] = 0; ra[j] = 0; ci[j] = 0; }
      merge(sm, 0, itot, rk, ra, ci, 0u, a.exp);
      if (len > 1) itot_cur = fetch_inserts<NL>(sm, a, 1, 1, iv);
      if (tid - DESC_T0 < 32u && len > 2) cpv = fetch_cp(a.cp + cpb + 2, tid - DESC_T0);
      if (tid - BND_T0 < 32u && len > 2) bv = fetch_bounds(a, cpb + 2, NL, w, tid - BND_T0);
   }

   for (uint32_t i = 0; i < len; i++)
   {
      const uint32_t cpi = cpb + i;
      const ChainPort& P = sm.cp[i % 3];
      const bool has_next = i + 1 < len;
      uint64_t* const stw = a.st + ((uint64_t) (a.cp0 + cpi) * nW + w) * SW;          // this window's state
      const uint64_t* const stp = w ? a.st + ((uint64_t) (a.cp0 + cpi) * nW + w - 1) * SW : nullptr;   // predecessor's

      // ---- [A] land last step's prefetches: port i+1's inserts, port i+2's descriptor and
      // bounds; load the predecessor's state of this port
      CH_STAMP(0);
      const uint32_t itot = itot_cur;
      bool ibad = false;
      if (has_next) ibad = store_inserts<NL>(sm, iv, itot, wbase);
      if (tid - DESC_T0 < 32u && i + 2 < len) put_cp(&sm.cp[(i + 2) % 3], cpv, tid - DESC_T0);
      if (tid - BND_T0 < 32u && i + 2 < len) put_bounds(sm, (i + 2) & 1, bv, NL, tid - BND_T0);
      uint64_t pv = 0;
      if (wv == 0 && w && lane < (uint32_t) SW) pv = ld1(stp + lane);
      CH_STAMP(7);

      const uint32_t nx = sgpr(P.nx), ny = sgpr(P.ny), cont = sgpr(P.cont);
      uint32_t n = sgpr(sm.n), k = 0, a0 = 0, cnt = 0;
      Agg ex, tot;
      bool first = true;
      for (;;)
      {
         // ---- [B][C] the stream: segments, block scan (first pass: no spill-ins yet)
         k = (n + T - 1) / T;
         a0 = min(tid * k, n);
         cnt = min(k, n - a0);
         {
            const Agg g0 = load_segment(sm, a0, cnt, wr, d0, nx, ny, cont, rk, ra);
            if (first) CH_STAMP(8);
            block_scan(sm, g0, ex, tot);   // #1
         }
         if (!first) break;
         CH_STAMP(1);
         first = false;
         if (ibad) flag(a, F_FALLBACK);
         // Y ports: the three insert ranges into one sorted list (read after barrier #3)
         if (has_next) premerge<NL>(sm, itot);

         // ---- [D] predecessor's state (wave 0)
         if (wv == 0)
         {
            uint64_t X_in = 0;
            uint32_t cin[4] = { 0, 0, 0, 0 };
            uint32_t mode = analytical ? 1u : 0u, Kpp = 0, Pep = 0;
            bool ok = true;
            if (w)
            {
               ok = poll_words(a, stp, SW, lane, pv);
               if (ok)
               {
                  X_in = __shfl(pv, 0) & M48;
#pragma unroll
                  for (int f = 0; f < 4; f++) cin[f] = (uint32_t) (__shfl(pv, 1 + f) & M48);
                  mode = (uint32_t) (__shfl(pv, 5) & 1u);
                  Kpp = (uint32_t) (__shfl(pv, 6) & M48);
                  Pep = (uint32_t) (__shfl(pv, 7) & M48);
               }
            }
            CH_STAMP(2);
            // window-relative tail: an earlier tail behaves like the base cycle (every tc > wb)
            const uint64_t xr = X_in > wb ? X_in - wb : 0;
            if (xr >= (1ull << 31)) ok = false;
            const uint32_t Xr = (uint32_t) xr;
            const uint32_t Kout = sm.nin_prev ? sm.P0cur + sm.nin_prev : Kpp;
            const uint32_t Pend = sm.P0cur + sm.ncont_prev;
            if (lane == 0)
            {
               if (!ok)
               {
                  sm.abort_ = 1;
                  if (xr >= (1ull << 31)) flag(a, F_FALLBACK);
               }
               sm.X_in = Xr;
               for (int f = 0; f < 4; f++) sm.cnt_in[f] = cin[f];
               sm.mode_in = mode;
               sm.Kpp = Kpp;
               sm.Pep = Pep;
               sm.ssum = 0;
               sm.n_inwin = 0;
               sm.first_gap = NONE;
               sm.first_fire = NONE;
               sm.sp_skip = 0;
               sm.sp_take = 0;
               sm.Kout = Kout;   // this port's spill range after this window (no spill-ins)
               sm.Pend = Pend;
            }
            const bool early = ok && !mode && Pep == Kpp;
            if (lane == 0) sm.published = early ? 1u : 0u;
            if (early && lane < (uint32_t) SW)
            {
               // inclusive = carry x aggregate, published before the outputs
               const uint32_t nx0 = Xr + tot.A;
               uint64_t v = 0;
               if (lane == 0) v = wb + (nx0 > tot.B ? nx0 : tot.B);
               else if (lane < 5) v = (uint64_t) (cin[lane - 1] + cf(tot.C, lane - 1));
               else if (lane == 6) v = Kout;
               else if (lane == 7) v = Pend;
               st1(stw + lane, a.etag | v);
            }
         }
         bar();   // #2
         CH_STAMP(3);
         if (sm.abort_) return;
         // next prefetches (they land at the next step's [A]): port i+2's inserts (its
         // descriptor and bounds landed at this step's [A]), port i+3's descriptor and bounds
         if (i + 2 < len) itot_cur = fetch_inserts<NL>(sm, a, (i + 2) % 3, (i + 2) & 1, iv);
         if (tid - DESC_T0 < 32u && i + 3 < len) cpv = fetch_cp(a.cp + cpi + 3, tid - DESC_T0);
         if (tid - BND_T0 < 32u && i + 3 < len) bv = fetch_bounds(a, cpi + 3, NL, w, tid - BND_T0);
         if (sm.Pep == sm.Kpp) break;
         // ---- slow path: spill-ins (about one step in twenty)
         const uint32_t Kpp = sm.Kpp, spn = sm.Pep - sm.Kpp;
         const bool sok = i > 0 && spn + min(itot, (uint32_t) ICAP) <= (uint32_t) ICAP &&
                          (uint64_t) Kpp + spn <= a.cp[cpi - 1].ocap[1];
         if (!sok)
         {
            if (tid == 0) flag(a, F_FALLBACK);
            return;
         }
         const uint32_t take = spill_in(sm, a, a.cp[cpi - 1].obase[1] + Kpp, spn, itot, n, wbase, wlen, rk, ra, a0, cnt);
         if (n + take > (uint32_t) CAP)
         {
            if (tid == 0) flag(a, F_RETRY);
            return;
         }
         if (tid == 0 && !sm.nin_prev) sm.Kout = Kpp + sm.sp_skip + take;   // the consumed prefix of the old spills
         n += take;   // rescan (the stream changed)
         if (!take) first = true;   // nothing merged: the scan stands
         if (!take) break;
      }
      if (!sm.published)
      {
         bar();
         // publish now (unless the history tree still has no gap: after the outputs)
         if (wv == 0 && !sm.mode_in && lane < (uint32_t) SW)
         {
            const uint32_t nx0 = sm.X_in + tot.A;
            uint64_t v = 0;
            if (lane == 0) v = wb + (nx0 > tot.B ? nx0 : tot.B);
            else if (lane < 5) v = (uint64_t) (sm.cnt_in[lane - 1] + cf(tot.C, lane - 1));
            else if (lane == 6) v = sm.Kout;
            else if (lane == 7) v = sm.Pend;
            st1(stw + lane, a.etag | v);
         }
      }

      // ---- [E] recurrence, outputs; kept records overwrite rk (new key) in place
      const uint32_t Xin = sgpr(sm.X_in);
      const uint32_t mode_in = sgpr(sm.mode_in);
      uint32_t X = Xin + ex.A;
      X = X > ex.B ? X : ex.B;
      uint32_t run[4];
#pragma unroll
      for (int f = 0; f < 4; f++) run[f] = sgpr(sm.cnt_in[f]) + cf(ex.C, f);
      const uint32_t P0n = sgpr(sm.cnt_in[1]);   // chain-direction records before this window
      const uint32_t rl = sgpr(P.rl);
      uint32_t km = 0;
      uint64_t ssum = 0;
      uint32_t nkeep = 0, fgap = NONE, ffire = NONE;
      bool spilled = false, bad = false, route = false;
      CH_STAMP(12);
#pragma unroll
      for (int j = 0; j < PER; j++)
      {
         if ((uint32_t) j >= cnt) continue;
         const uint32_t off = (uint32_t) (rk[j] >> 32);
         const uint32_t id = (uint32_t) rk[j];
         const uint32_t ax = ra[j];
         const uint32_t tc = rcyc(off, wr, d0);
         const uint32_t p = aux_F(ax);
         const uint32_t Xb = X;
         const uint32_t cc = Xb > tc ? Xb - tc : 0;
         X = (Xb > tc ? Xb : tc) + p;
         if (mode_in)
         {
            // history tree with no gap yet: an idle period makes one (:79-86); the M/G/1
            // branch fires while there is none and the tail lies beyond t + p (:58-64)
            if (tc > Xb && fgap == NONE) fgap = a0 + j;
            if (Xb > tc + p && ffire == NONE) ffire = a0 + j;
         }
         ssum += cc;
         const uint64_t dn = (uint64_t) off + (uint64_t) cc * 1000ull + rl;   // t' - wbase
         const uint32_t f = field_of(xy_dir(nx, ny, aux_dx(ax), aux_dy(ax)), cont);
         uint32_t pos = 0;
#pragma unroll
         for (int q = 0; q < 4; q++)
            if (f == (uint32_t) q) pos = run[q]++;
         if (f == 1 && dn < wlen)
         {
            km |= 1u << j;
            rk[j] = (dn << 32) | id;
            ci[j] = pos - P0n;
            nkeep++;
            continue;
         }
         if (pos >= P.ocap[f]) { route = true; continue; }
         if (a.exp & 1u) continue;
         const uint64_t gp = P.obase[f] + pos;
         const uint64_t tn = wbase + dn;
         if (f == 1)
         {
            // spill: taken by task (chain, w+1) at the next port (sc1: read in-launch)
            bad |= w + 1 >= nW;   // the last window keeps everything (or its offsets overflowed)
            uint64_t* r = reinterpret_cast<uint64_t*>(a.recs + gp);
            st1(r, tn);
            st1(r + 1, (uint64_t) id | ((uint64_t) ax << 32));
            spilled = true;
         }
         else
         {
            Rec o;
            o.t = tn;
            o.id = id;
            o.aux = ax;
            a.recs[gp] = o;
            if ((gp & 63) == 0)
            {
               a.samp_t[gp >> 6] = tn;
               a.samp_id[gp >> 6] = id;
            }
         }
      }
      CH_STAMP(13);
      // kept keys at their index (the search array of the next merge: the stream's
      // own reads all happened before barrier #1)
#pragma unroll
      for (int j = 0; j < PER; j++)
         if ((km >> j) & 1u) sm.key[pad(ci[j])] = rk[j];
      if (route) flag(a, F_ROUTE);
      if (bad) flag(a, F_FALLBACK);
      // block reductions: queue delay sum, kept records, first gap / M/G/1 condition
      ssum = wave_sum64(ssum);
      nkeep = wave_sum32(nkeep);
      if (lane == 63)
      {
         if (ssum) atomicAdd((unsigned long long*) &sm.ssum, (unsigned long long) ssum);
         if (nkeep) atomicAdd(&sm.n_inwin, nkeep);
      }
      if (mode_in)
      {
         if (fgap != NONE) atomicMin(&sm.first_gap, fgap);
         if (ffire != NONE) atomicMin(&sm.first_fire, ffire);
      }
      if (__any(spilled)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drained before the next publish
      bar();   // #3
      CH_STAMP(4);

      // ---- [F] late publish (no gap yet), port counters, route check (wave 0)
      const uint32_t nin = sm.n_inwin;
      if (wv == 0)
      {
         const uint32_t nx0 = Xin + tot.A;
         const uint64_t Xo = wb + (nx0 > tot.B ? nx0 : tot.B);
         if (!sm.published && mode_in && lane < (uint32_t) SW)
         {
            const uint32_t fg = sm.first_gap, ff = sm.first_fire;
            // the M/G/1 branch would serve a request that arrives before the first gap
            if (lane == 0 && ff != NONE && (fg == NONE || ff < fg)) flag(a, F_FALLBACK);
            uint64_t v = 0;
            if (lane == 0) v = Xo;
            else if (lane < 5) v = (uint64_t) (sm.cnt_in[lane - 1] + cf(tot.C, lane - 1));
            else if (lane == 5) v = (fg == NONE) ? 1u : 0u;   // still no gap after this window
            else if (lane == 6) v = sm.Kout;
            else v = sm.Pend;
            st1(stw + lane, a.etag | v);
         }
         if (lane == 0)
         {
            if (w + 1 == nW)
            {
               // every record of the port has passed: the route counts fill every output slot
               bool full = true;
               for (uint32_t f = 0; f < 4; f++) full &= sm.cnt_in[f] + cf(tot.C, f) == P.ocap[f];
               if (!full) flag(a, F_ROUTE);
            }
            if (n)
            {
               const uint32_t port = P.port;
               atomicAdd(&a.port_sum[port], (unsigned long long) sm.ssum);
               atomicAdd(&a.port_cnt[port], (unsigned long long) n);
               atomicAdd(&a.port_flit[port], (unsigned long long) tot.A);
               atomicMax(&a.port_last[port], (unsigned long long) Xo);
            }
            // the next port's chain input: records before this window, kept, all of this window
            sm.P0cur = sm.cnt_in[1];
            sm.nin_prev = nin;
            sm.ncont_prev = cf(tot.C, 1);
         }
      }
      CH_STAMP(9);
      if (!has_next) break;
      if (itot > (uint32_t) ICAP || nin + itot > (uint32_t) CAP)   // (every thread knows both)
      {
         if (tid == 0) flag(a, F_RETRY);
         return;
      }
      // ---- [G] next port's stream: kept records + its inserts
      merge(sm, nin, itot, rk, ra, ci, km, a.exp,
            a.stamps ? a.stamps + ((uint64_t) tk * len + i) * 16 : nullptr);   // #4, #5
      CH_STAMP(5);
      if (a.stamps && tid == 0)
         a.stamps[((uint64_t) tk * len + i) * 16 + 6] = (uint64_t) n | ((uint64_t) itot << 16) |
                                                     ((uint64_t) nin << 32) | ((uint64_t) (sm.Pep != sm.Kpp) << 63);
   }
}

template <int NL>
__global__ __launch_bounds__(T, CH_MINW) void k_chain(ChainArgs a)
{
   __shared__ Smem sm;
   const uint32_t tid = threadIdx.x;
   const uint32_t ntasks = a.nch * a.nW;
   // an earlier level served a request by M/G/1 (exception tails): the chain's
   // inputs are not in FIFO order -> the level engine reruns the batch
   if (a.errflag[2] != 0)
   {
      if (tid == 0 && blockIdx.x == 0) flag(a, F_FALLBACK);
      return;
   }
   for (;;)
   {
      // window-major, strictly in order to running workgroups: a task's predecessor
      // (same chain, window - 1) is always held by a running workgroup or done
      if (tid == 0) sm.next_task = atomicAdd(a.ctr, 1u);
      bar();
      const uint32_t tk = sm.next_task;
      if (tk >= ntasks || flagged(a)) return;
      task<NL>(sm, a, tk % a.nch, tk / a.nch, tk);
      bar();
   }
}

// ---------------------------------------------------------------------------
// plan and window bounds
// ---------------------------------------------------------------------------
// One thread per chain port.  Chains of the X phase: rows [ry0, ry1), RIGHT
// (x = 0 .. W-2) then LEFT (x = W-1 .. 1); of the Y phase: columns [cx0, cx1),
// UP (y = 0 .. H-2) then DOWN (y = H-1 .. 1).
__global__ __launch_bounds__(256) void k_chain_plan(DevCfg c, uint32_t ncpx, uint32_t ncpy, uint32_t ry0, uint32_t cx0,
                                                    const uint32_t* __restrict__ slot_cnt,
                                                    const uint64_t* __restrict__ slot_base, ChainPort* __restrict__ out)
{
   const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
   if (k >= ncpx + ncpy) return;
   const uint32_t W = c.W, H = c.H;
   uint32_t x, y, dir, nl;
   if (k < ncpx)
   {
      const uint32_t len = W - 1, ch = k / len, i = k % len;
      y = ry0 + ch / 2;
      dir = (ch & 1) ? P_LEFT : P_RIGHT;
      x = dir == P_RIGHT ? i : W - 1 - i;
      nl = 1;
   }
   else
   {
      const uint32_t kk = k - ncpx, len = H - 1, ch = kk / len, i = kk % len;
      x = cx0 + ch / 2;
      dir = (ch & 1) ? P_DOWN : P_UP;
      y = dir == P_UP ? i : H - 1 - i;
      nl = 3;
   }
   const uint32_t tile = y * W + x;
   uint32_t ntile = tile;
   if (dir == P_RIGHT) ntile = tile + 1;
   else if (dir == P_LEFT) ntile = tile - 1;
   else if (dir == P_UP) ntile = tile + W;
   else ntile = tile - W;
   const uint32_t nside = in_side_after(dir);
   ChainPort p;
   const uint32_t fdir[4] = { P_SELF, dir, P_UP, P_DOWN };
   for (uint32_t f = 0; f < 4; f++)
   {
      // a Y port's UP / DOWN fields other than its own direction carry nothing
      const bool used = f < 2 || dir == P_LEFT || dir == P_RIGHT;
      const uint32_t os = slot_of(ntile, fdir[f], slot_side(fdir[f], nside));
      p.obase[f] = used ? slot_base[os] : 0;
      p.ocap[f] = used ? slot_cnt[os] : 0;
   }
   const uint32_t sides[3] = { IN_LOCAL, IN_W, IN_E };
   for (uint32_t j = 0; j < 3; j++)
   {
      const uint32_t s = slot_of(tile, dir, sides[j]);
      p.ibase[j] = j < nl ? slot_base[s] : 0;
      p.icnt[j] = j < nl ? slot_cnt[s] : 0;
   }
   p.port = tile * PORTS + dir;
   p.tile = tile;
   p.dir = dir;
   p.cont = dir;
   p.nx = ntile % W;
   p.ny = ntile / W;
   p.rl = (uint32_t) rl_of(c, tile);
   p.nl = nl;
   p.pad0[0] = p.pad0[1] = p.pad0[2] = 0;
   out[k] = p;
}

// One workgroup per (chain port, insert list): bt[w] = first record of the
// slot with t >= w D (w < nW), bt[nW] = record count.  Window of t:
// min(t >> dshift, nW - 1) (the last window is unbounded).
__global__ __launch_bounds__(256) void k_win_bounds(const ChainPort* __restrict__ cp, uint32_t nl, uint32_t nW,
                                                    uint32_t dshift, const Rec* __restrict__ recs,
                                                    uint32_t* __restrict__ bt)
{
   const uint32_t k = blockIdx.x / nl, j = blockIdx.x % nl;
   const uint64_t base = cp[k].ibase[j];
   const uint32_t n = cp[k].icnt[j];
   uint32_t* b = bt + (uint64_t) blockIdx.x * (nW + 1);
   const uint64_t wl = nW - 1;
   if (n == 0)
   {
      for (uint32_t v = threadIdx.x; v <= nW; v += blockDim.x) b[v] = 0;
      return;
   }
   for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
   {
      uint64_t wi = recs[base + i].t >> dshift;
      wi = wi < wl ? wi : wl;
      int64_t wp = -1;
      if (i)
      {
         uint64_t q = recs[base + i - 1].t >> dshift;
         wp = (int64_t) (q < wl ? q : wl);
      }
      for (int64_t v = wp + 1; v <= (int64_t) wi; v++) b[v] = i;
      if (i == n - 1)
         for (uint64_t v = wi + 1; v <= nW; v++) b[v] = n;
   }
}

// Zero the per-port counters of ports whose direction is in dmask (a phase
// that reruns on the level engine after the chain engine declined it).
__global__ __launch_bounds__(256) void k_zero_ports(uint32_t nports, uint32_t dmask, unsigned long long* __restrict__ s0,
                                                    unsigned long long* __restrict__ s1, unsigned long long* __restrict__ s2,
                                                    unsigned long long* __restrict__ s3, unsigned long long* __restrict__ s4)
{
   const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
   if (p >= nports || !((dmask >> (p % PORTS)) & 1u)) return;
   s0[p] = 0;
   s1[p] = 0;
   s2[p] = 0;
   s3[p] = 0;
   s4[p] = 0;
}

}  // namespace ch
}  // namespace gnoc
