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
//            or spill (t' >= window end: HBM, picked up by task (chain, w+1)).
// The queue state of port i at the start of window w is the inclusive state of
// task (chain, w-1) at port i: a chained hand-off per (port, window) (8-byte
// epoch-tagged granules, sc1 stores and loads, MI355X_MICROARCH.md "Valid
// forms").  Tasks are handed out window-major, so a task's predecessor is
// always running or done: no deadlock.
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

constexpr int T = 256;                    // threads per workgroup
#ifndef CH_CAP_V
#define CH_CAP_V 2048
#endif
constexpr int CAP = CH_CAP_V;             // stream records per (port, window)
constexpr int PER = CAP / T;              // records per thread
#ifndef CH_ICAP_V
#define CH_ICAP_V 768
#endif
constexpr int ICAP = CH_ICAP_V;           // inserts (+ spill-ins) per (port, window)
constexpr int IPER = ICAP / T;
constexpr int NLMAX = 3;                  // local insert lists (Y ports: LOCAL, W, E)
constexpr int SW = 16;                    // state words per (chain port, window)
constexpr uint32_t F_RETRY = 1u;          // a window overflowed LDS: rerun with smaller windows
constexpr uint32_t F_FALLBACK = 2u;       // M/G/1 would fire, exception tails, ...: rerun on the level engine
constexpr uint32_t F_ROUTE = 4u;          // route-count invariant broken (internal error)
constexpr uint32_t F_TIMEOUT = 8u;        // a hand-off wait timed out
constexpr uint32_t F_ANY = F_RETRY | F_FALLBACK | F_ROUTE | F_TIMEOUT;
constexpr uint64_t SPIN_CYCLES = 1ull << 31;
constexpr uint64_t M48 = (1ull << 48) - 1;

// LDS index padding: one u64 per 32 entries, so a thread's contiguous segment
// (stride PER across lanes) hits distinct banks.
__host__ __device__ constexpr uint32_t pad(uint32_t r) { return r + (r >> 5); }
constexpr int CAPP = CAP + CAP / 32;

}  // namespace ch

// One port of a chain (k_chain_plan): output slots of the next tile, insert
// slots of this port.  128 bytes: one wave copies it with one load per lane.
struct __attribute__((aligned(16))) ChainPort
{
   uint64_t obase[5];    // output slot base per next direction
   uint64_t ibase[3];    // insert slot bases (IN_LOCAL, IN_W, IN_E)
   uint32_t ocap[5];     // output slot capacities
   uint32_t icnt[3];     // insert slot record counts
   uint32_t port, tile, dir, cont;   // cont: the chain direction (continuing next dir)
   uint32_t nx, ny, rl, nl;          // next tile, R + Lk (ps), local insert lists
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
};

namespace ch {

struct Smem
{
   uint64_t key[CAPP];            // (t - wbase) << 32 | id, sorted
   uint32_t aux[CAPP];            // dx | dy << 10 | F << 20
   uint64_t ikey[ICAP];           // insert lists (local lists, then spill-ins)
   uint32_t iaux[ICAP];
   ChainPort cp[3];               // ports i, i+1, i+2 (ring)
   uint32_t blo[2][NLMAX], bhi[2][NLMAX];   // window bounds of ports i+1, i+2 (ring)
   uint32_t ioff[NLMAX + 2];      // insert list offsets (NL local lists, spill list, end)
   uint32_t ioff_next[NLMAX];     // local list offsets of the inserts in flight
   uint64_t wA[T / 64], wB[T / 64], wC[T / 64];
   uint64_t X_in;
   uint32_t cnt_in[5];
   uint32_t mode_in;
   uint64_t ssum;
   uint32_t n, n_inwin, first_gap, first_fire;
   uint32_t Kp_prev, sp_lo, sp_n, sp_skip, sp_take;
   uint32_t abort_, next_task, itot;
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
__device__ __forceinline__ uint32_t cf(uint64_t c, uint32_t d) { return (uint32_t) ((c >> (12 * d)) & 0xFFFu); }
__device__ __forceinline__ uint64_t cyc(uint64_t ps) { return (ps + 999ull) / 1000ull; }

// lower bound of k in the sorted u64 array a[0, n)
__device__ __forceinline__ uint32_t lb(const uint64_t* a, uint32_t n, uint64_t k)
{
   uint32_t lo = 0, hi = n;
   while (lo < hi)
   {
      const uint32_t m = (lo + hi) >> 1;
      if (a[m] < k) lo = m + 1;
      else hi = m;
   }
   return lo;
}
// same over the padded stream array
__device__ __forceinline__ uint32_t lbp(const uint64_t* a, uint32_t n, uint64_t k)
{
   uint32_t lo = 0, hi = n;
   while (lo < hi)
   {
      const uint32_t m = (lo + hi) >> 1;
      if (a[pad(m)] < k) lo = m + 1;
      else hi = m;
   }
   return lo;
}

__device__ __forceinline__ void flag(const ChainArgs& a, uint32_t f)
{
   atomicOr(a.errflag + 4, f);
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

// Poll the hand-off words [w0, w0 + nw) of state block s until all carry the
// epoch tag (lane q < nw holds word w0 + q).  Wave-wide; false on abort.
__device__ bool poll_words(const ChainArgs& a, const uint64_t* s, uint32_t w0, uint32_t nw, uint32_t lane, uint64_t& v)
{
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
      if (lane < nw) v = ld1(s + w0 + lane);
   }
}

// Merge the kept continuing records (registers: keys rk, aux ra, continuing
// index ci; bit j of km marks a kept record) with the insert lists in sm.ikey
// (offsets sm.ioff[0..NL+1]) into the stream sm.key/aux.  Positions = own index
// + lower bounds in every other list (keys are unique: one record per packet
// per port).  The kept keys sit at key[pad(ci)] (written by the caller before
// the barrier preceding this call).
template <int NL>
__device__ void merge(Smem& sm, uint32_t nkeep, const uint64_t (&rk)[PER], const uint32_t (&ra)[PER],
                      uint32_t (&ci)[PER], uint32_t km, uint32_t ntot)
{
   const uint32_t tid = threadIdx.x;
   constexpr int NLIST = NL + 1;   // local lists + spill-ins
   uint32_t lo_l[NLIST], n_l[NLIST];
#pragma unroll
   for (int l = 0; l < NLIST; l++)
   {
      lo_l[l] = sm.ioff[l];
      n_l[l] = sm.ioff[l + 1] - sm.ioff[l];
   }
   // kept records: own index + inserts below, per list (first by search, then advance)
   uint32_t cur[NLIST];
#pragma unroll
   for (int l = 0; l < NLIST; l++) cur[l] = 0;
   bool first = true;
#pragma unroll
   for (int j = 0; j < PER; j++)
   {
      if (!((km >> j) & 1u)) continue;
      uint32_t p = ci[j];
#pragma unroll
      for (int l = 0; l < NLIST; l++)
      {
         if (first) cur[l] = lb(sm.ikey + lo_l[l], n_l[l], rk[j]);
         else
            while (cur[l] < n_l[l] && sm.ikey[lo_l[l] + cur[l]] < rk[j]) cur[l]++;
         p += cur[l];
      }
      first = false;
      ci[j] = p;
   }
   // inserts: own index + kept below + other lists below
   const uint32_t itot = sm.ioff[NLIST];
   uint64_t ik[IPER];
   uint32_t ia[IPER], pi[IPER];
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = tid + (uint32_t) q * T;
      pi[q] = 0xFFFFFFFFu;
      ik[q] = 0;
      ia[q] = 0;
      if (g >= itot) continue;
      ik[q] = sm.ikey[g];
      ia[q] = sm.iaux[g];
      uint32_t own = 0;
#pragma unroll
      for (int l = 0; l < NLIST; l++)
         if (g >= lo_l[l] && g < lo_l[l] + n_l[l]) own = (uint32_t) l;
      uint32_t p = g - sm.ioff[own] + lbp(sm.key, nkeep, ik[q]);
#pragma unroll
      for (int l = 0; l < NLIST; l++)
         if ((uint32_t) l != own) p += lb(sm.ikey + lo_l[l], n_l[l], ik[q]);
      pi[q] = p;
   }
   bar();
#pragma unroll
   for (int j = 0; j < PER; j++)
      if ((km >> j) & 1u)
      {
         sm.key[pad(ci[j])] = rk[j];
         sm.aux[pad(ci[j])] = ra[j];
      }
#pragma unroll
   for (int q = 0; q < IPER; q++)
      if (pi[q] != 0xFFFFFFFFu)
      {
         sm.key[pad(pi[q])] = ik[q];
         sm.aux[pad(pi[q])] = ia[q];
      }
   if (tid == 0) sm.n = ntot;
   bar();
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
      // bounds come from sorted slots; clamped so that nothing else can load out of range
      lo[j] = min(sm.blo[br][j], P.icnt[j]);
      const uint32_t hi = min(max(sm.bhi[br][j], lo[j]), P.icnt[j]);
      off[j + 1] = off[j] + (hi - lo[j]);
   }
   const uint32_t itot = off[NL];
   // list offsets for store_inserts / merge (written before the barrier that precedes their use)
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

// Write fetched inserts into the insert buffer as keys relative to wbase, and
// the list offsets (local lists of bounds ring br; the spill list empty).
template <int NL>
__device__ __forceinline__ bool store_inserts(Smem& sm, const Rec (&iv)[IPER], uint32_t itot, uint64_t wbase,
                                              uint32_t br)
{
   const uint32_t tid = threadIdx.x;
   bool bad = false;
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = tid + (uint32_t) q * T;
      if (g < itot && g < (uint32_t) ICAP)
      {
         const uint64_t dt = iv[q].t - wbase;
         bad |= (dt >> 32) != 0;
         sm.ikey[g] = (dt << 32) | iv[q].id;
         sm.iaux[g] = iv[q].aux;
      }
   }
   if (tid == 0)
   {
      sm.ioff[0] = 0;
      for (int j = 1; j < NL; j++) sm.ioff[j] = sm.ioff_next[j];
      sm.ioff[NL] = itot;
      sm.ioff[NL + 1] = itot;
   }
   return bad;
}

// ---------------------------------------------------------------------------
// one task: chain c, window w
// ---------------------------------------------------------------------------
template <int NL>
__device__ void task(Smem& sm, const ChainArgs& a, uint32_t c, uint32_t w)
{
   const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
   const uint64_t wbase = (uint64_t) w << a.dshift;
   const uint64_t wend = (w + 1 < a.nW) ? (uint64_t) (w + 1) << a.dshift : ~0ull;
   const uint32_t len = a.len, nW = a.nW;
   const uint32_t cpb = c * len;
   const int analytical = a.c.analytical;

   // ---- prologue: ports 0 and 1, bounds of their inserts, port 0's stream
   if (wv == 0) load_cp(&sm.cp[0], a.cp + cpb, lane);
   if (wv == 1 && len > 1) load_cp(&sm.cp[1], a.cp + cpb + 1, lane);
   if (wv == 2) load_bounds(sm, a, 0, cpb, NL, w, lane);
   if (wv == 3 && len > 1) load_bounds(sm, a, 1, cpb + 1, NL, w, lane);
   if (tid == 0) sm.abort_ = 0;
   bar();
   uint64_t rk[PER];
   uint32_t ra[PER], ci[PER];
   {
      Rec iv[IPER];
      const uint32_t itot = fetch_inserts<NL>(sm, a, 0, 0, iv);
      const bool bad = store_inserts<NL>(sm, iv, itot, wbase, 0);
      if (tid == 0 && (itot > (uint32_t) ICAP || itot > (uint32_t) CAP)) { flag(a, F_RETRY); sm.abort_ = 1; }
      if (bad) { flag(a, F_FALLBACK); sm.abort_ = 1; }
      bar();
      if (sm.abort_) return;
#pragma unroll
      for (int j = 0; j < PER; j++) { rk[j] = 0; ra[j] = 0; ci[j] = 0; }
      merge<NL>(sm, 0, rk, ra, ci, 0u, itot);
   }

   for (uint32_t i = 0; i < len; i++)
   {
      const uint32_t cpi = cpb + i;
      const ChainPort& P = sm.cp[i % 3];
      const bool has_next = i + 1 < len;
      uint64_t* const stw = a.st + ((uint64_t) (a.cp0 + cpi) * nW + w) * SW;          // this window's state
      const uint64_t* const stp = w ? a.st + ((uint64_t) (a.cp0 + cpi) * nW + w - 1) * SW : nullptr;   // predecessor's

      // ---- [A] prefetch: next port's inserts; descriptor + bounds of port i+2; predecessor state
      uint32_t itot = 0;
      Rec iv[IPER];
      if (has_next) itot = fetch_inserts<NL>(sm, a, (i + 1) % 3, (i + 1) & 1, iv);
      if (wv == 1 && i + 2 < len) load_cp(&sm.cp[(i + 2) % 3], a.cp + cpi + 2, lane);
      if (wv == 2 && i + 2 < len) load_bounds(sm, a, i & 1, cpi + 2, NL, w, lane);
      uint64_t pv = 0;
      if (wv == 0 && w && lane < 7) pv = ld1(stp + lane);

      // ---- [B] this thread's segment of the stream -> registers, local aggregate
      const uint32_t n = sm.n;
      const uint32_t k = (n + T - 1) / T;
      const uint32_t a0 = min(tid * k, n);
      const uint32_t cnt = min(k, n - a0);
      const uint32_t nx = P.nx, ny = P.ny, cont = P.cont;
      uint64_t A = 0, B = 0, C = 0;
#pragma unroll
      for (int j = 0; j < PER; j++)
      {
         rk[j] = 0;
         ra[j] = 0;
         if ((uint32_t) j < cnt)
         {
            rk[j] = sm.key[pad(a0 + j)];
            ra[j] = sm.aux[pad(a0 + j)];
            const uint64_t tc = cyc(wbase + (rk[j] >> 32));
            const uint64_t p = aux_F(ra[j]);
            mp(A, B, p, tc + p);
            C += 1ull << (12 * xy_dir(nx, ny, aux_dx(ra[j]), aux_dy(ra[j])));
         }
      }
      // ---- [C] block scan
      uint64_t iA = A, iB = B, iC = C;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1)
      {
         const uint64_t pA = __shfl_up(iA, off), pB = __shfl_up(iB, off), pC = __shfl_up(iC, off);
         if ((int) lane >= off)
         {
            uint64_t x = pA, y = pB;
            mp(x, y, iA, iB);
            iA = x;
            iB = y;
            iC += pC;
         }
      }
      if (lane == 63) { sm.wA[wv] = iA; sm.wB[wv] = iB; sm.wC[wv] = iC; }
      bar();   // #1
      uint64_t eA = 0, eB = 0, eC = 0;
      for (uint32_t v = 0; v < wv; v++)
      {
         mp(eA, eB, sm.wA[v], sm.wB[v]);
         eC += sm.wC[v];
      }
      {
         uint64_t xA = __shfl_up(iA, 1), xB = __shfl_up(iB, 1), xC = __shfl_up(iC, 1);
         if (lane == 0) { xA = 0; xB = 0; xC = 0; }
         mp(eA, eB, xA, xB);
         eC += xC;
      }
      uint64_t TA = 0, TB = 0, TC = 0;
#pragma unroll
      for (int v = 0; v < T / 64; v++)
      {
         mp(TA, TB, sm.wA[v], sm.wB[v]);
         TC += sm.wC[v];
      }
      // the next port's local inserts into the (free) insert buffer
      bool ibad = false;
      if (has_next) ibad = store_inserts<NL>(sm, iv, itot, wbase, (i + 1) & 1);

      // ---- [D] predecessor's inclusive state (wave 0), early publish when FIFO
      if (wv == 0)
      {
         uint64_t X_in = 0;
         uint32_t cin[5] = { 0, 0, 0, 0, 0 };
         uint32_t mode = analytical ? 1u : 0u;
         bool ok = true;
         if (w)
         {
            ok = poll_words(a, stp, 0, 7, lane, pv);
            if (ok)
            {
               X_in = __shfl(pv, 0) & M48;
#pragma unroll
               for (int d = 0; d < 5; d++) cin[d] = (uint32_t) (__shfl(pv, 1 + d) & M48);
               mode = (uint32_t) (__shfl(pv, 6) & 1u);
            }
         }
         if (!ok)
         {
            if (lane == 0) sm.abort_ = 1;
         }
         else
         {
            if (lane == 0)
            {
               sm.X_in = X_in;
               for (int d = 0; d < 5; d++) sm.cnt_in[d] = cin[d];
               sm.mode_in = mode;
               sm.ssum = 0;
               sm.n_inwin = 0;
               sm.first_gap = 0xFFFFFFFFu;
               sm.first_fire = 0xFFFFFFFFu;
            }
            if (!mode && lane < 7)
            {
               // inclusive = carry x aggregate, published before the outputs
               const uint64_t nx0 = X_in + TA;
               const uint64_t Xo = nx0 > TB ? nx0 : TB;
               uint64_t v = 0;
               if (lane == 0) v = Xo;
               else if (lane < 6) v = (uint64_t) (cin[lane - 1] + cf(TC, lane - 1));
               st1(stw + lane, a.etag | v);
            }
         }
      }
      bar();   // #2
      if (sm.abort_) return;

      // ---- [E] recurrence, outputs; kept records overwrite rk (new key) in place
      const uint64_t X_in = sm.X_in;
      const uint32_t mode_in = sm.mode_in;
      uint64_t X = X_in + eA;
      X = X > eB ? X : eB;
      uint32_t run[5];
#pragma unroll
      for (int d = 0; d < 5; d++) run[d] = sm.cnt_in[d] + cf(eC, d);
      const uint32_t P0n = sm.cnt_in[cont];   // continuing records before this window
      const uint64_t rl = P.rl;
      uint32_t km = 0;
      uint64_t ssum = 0;
      uint32_t nkeep = 0, fgap = 0xFFFFFFFFu, ffire = 0xFFFFFFFFu;
      bool spilled = false, bad = false, route = false;
#pragma unroll
      for (int j = 0; j < PER; j++)
      {
         if ((uint32_t) j >= cnt) continue;
         const uint64_t t = wbase + (rk[j] >> 32);
         const uint32_t id = (uint32_t) rk[j];
         const uint32_t ax = ra[j];
         const uint64_t tc = cyc(t);
         const uint64_t p = aux_F(ax);
         const uint64_t Xb = X;
         const uint64_t cc = Xb > tc ? Xb - tc : 0;
         X = (Xb > tc ? Xb : tc) + p;
         if (mode_in)
         {
            // history tree with no gap yet: an idle period makes one (:79-86); the M/G/1
            // branch fires while there is none and the tail lies beyond t + p (:58-64)
            if (tc > Xb && fgap == 0xFFFFFFFFu) fgap = a0 + j;
            if (Xb > tc + p && ffire == 0xFFFFFFFFu) ffire = a0 + j;
         }
         ssum += cc;
         const uint64_t tn = t + cc * 1000ull + rl;
         const uint32_t nd = xy_dir(nx, ny, aux_dx(ax), aux_dy(ax));
         uint32_t pos = 0;
#pragma unroll
         for (int d = 0; d < 5; d++)
            if (nd == (uint32_t) d) pos = run[d]++;
         if (nd == cont && tn < wend)
         {
            const uint64_t dt = tn - wbase;
            bad |= (dt >> 32) != 0;
            km |= 1u << j;
            rk[j] = (dt << 32) | id;
            ci[j] = pos - P0n;
            nkeep++;
            continue;
         }
         if (pos >= P.ocap[nd]) { route = true; continue; }
         const uint64_t gp = P.obase[nd] + pos;
         if (nd == cont)
         {
            // spill: picked up by task (chain, w+1) at the next port (sc1: read in-launch)
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
      if (route) flag(a, F_ROUTE);
      if (bad || ibad) flag(a, F_FALLBACK);
      // block reductions: queue delay sum, kept records, first gap / M/G/1 condition
      for (int off = 32; off > 0; off >>= 1)
      {
         ssum += __shfl_down(ssum, off);
         nkeep += __shfl_down(nkeep, off);
      }
      if (lane == 0)
      {
         if (ssum) atomicAdd((unsigned long long*) &sm.ssum, (unsigned long long) ssum);
         if (nkeep) atomicAdd(&sm.n_inwin, nkeep);
      }
      if (mode_in)
      {
         if (fgap != 0xFFFFFFFFu) atomicMin(&sm.first_gap, fgap);
         if (ffire != 0xFFFFFFFFu) atomicMin(&sm.first_fire, ffire);
      }
      if (__any(spilled)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // spills drained before the spill word
      bar();   // #3

      // ---- [F] late publish (no gap yet), port counters, spill word
      if (wv == 0)
      {
         const uint32_t nin = sm.n_inwin;
         if (mode_in && lane < 7)
         {
            const uint32_t fg = sm.first_gap, ff = sm.first_fire;
            // the M/G/1 branch would serve a request that arrives before the first gap
            if (lane == 0 && ff != 0xFFFFFFFFu && (fg == 0xFFFFFFFFu || ff < fg)) flag(a, F_FALLBACK);
            const uint64_t nx0 = X_in + TA;
            const uint64_t Xo = nx0 > TB ? nx0 : TB;
            uint64_t v = 0;
            if (lane == 0) v = Xo;
            else if (lane < 6) v = (uint64_t) (sm.cnt_in[lane - 1] + cf(TC, lane - 1));
            else v = (fg == 0xFFFFFFFFu) ? 1u : 0u;   // still no gap after this window
            st1(stw + lane, a.etag | v);
         }
         if (lane == 0 && w + 1 == nW)
         {
            // every record of the port has passed: the route counts must fill every output slot
            bool full = true;
            for (uint32_t d = 0; d < 5; d++) full &= sm.cnt_in[d] + cf(TC, d) == P.ocap[d];
            if (!full) flag(a, F_ROUTE);
         }
         if (lane == 0 && n)
         {
            const uint32_t port = P.port;
            atomicAdd(&a.port_sum[port], (unsigned long long) sm.ssum);
            atomicAdd(&a.port_cnt[port], (unsigned long long) n);
            atomicAdd(&a.port_flit[port], (unsigned long long) TA);
            const uint64_t nx0 = X_in + TA;
            atomicMax(&a.port_last[port], (unsigned long long) (nx0 > TB ? nx0 : TB));
         }
         if (has_next)
         {
            // spill word of port i+1: [K', Pend) = its unconsumed spill range after this window
            uint64_t sv = 0;
            bool ok = true;
            const uint64_t* spw = w ? a.st + ((uint64_t) (a.cp0 + cpi + 1) * nW + w - 1) * SW : nullptr;
            if (w)
            {
               if (lane < 2) sv = ld1(spw + 8 + lane);
               ok = poll_words(a, spw, 8, 2, lane, sv);
            }
            if (!ok)
            {
               if (lane == 0) sm.abort_ = 1;
            }
            else
            {
               const uint32_t Kpp = w ? (uint32_t) (__shfl(sv, 0) & M48) : 0u;
               const uint32_t Pep = w ? (uint32_t) (__shfl(sv, 1) & M48) : 0u;
               const uint32_t Kp = nin ? P0n + nin : Kpp;
               const uint32_t Pe = P0n + cf(TC, cont);
               uint64_t* spo = a.st + ((uint64_t) (a.cp0 + cpi + 1) * nW + w) * SW;
               if (lane < 2) st1(spo + 8 + lane, a.etag | (uint64_t) (lane ? Pe : Kp));
               if (lane == 0)
               {
                  sm.sp_lo = Kpp;
                  sm.sp_n = Pep - Kpp;
                  sm.sp_skip = 0;
                  sm.sp_take = 0;
               }
            }
         }
      }
      bar();   // #4
      if (sm.abort_) return;
      if (!has_next) break;

      // ---- [G] next port's stream: kept records + its inserts (+ spill-ins)
      const uint32_t nin = sm.n_inwin;
      const uint32_t spn = sm.sp_n;
      uint32_t sp_take = 0;
      if (spn)
      {
         // spill-ins: [K', Pend) of the next port's chain slot, records with t in this window
         const uint64_t sbase = P.obase[cont] + sm.sp_lo;
         const bool sok = spn <= (uint32_t) ICAP && (uint64_t) sm.sp_lo + spn <= P.ocap[cont];
         if (!sok && tid == 0) { flag(a, F_FALLBACK); sm.abort_ = 1; }
         Rec sv[IPER];
         uint32_t nb = 0, nt = 0;
#pragma unroll
         for (int q = 0; q < IPER; q++)
         {
            const uint32_t g = tid + (uint32_t) q * T;
            sv[q].t = 0;
            sv[q].id = 0;
            sv[q].aux = 0;
            if (g < spn && sok)
            {
               const uint64_t* r = reinterpret_cast<const uint64_t*>(a.recs + sbase + g);
               sv[q].t = ld1(r);
               const uint64_t ia = ld1(r + 1);
               sv[q].id = (uint32_t) ia;
               sv[q].aux = (uint32_t) (ia >> 32);
               nb += sv[q].t < wbase ? 1u : 0u;
               nt += (sv[q].t >= wbase && sv[q].t < wend) ? 1u : 0u;
            }
         }
         if (nb) atomicAdd(&sm.sp_skip, nb);
         if (nt) atomicAdd(&sm.sp_take, nt);
         bar();
         if (sm.abort_) return;
         const uint32_t skip = sm.sp_skip;
         sp_take = sm.sp_take;
         bool sbad = false;
#pragma unroll
         for (int q = 0; q < IPER; q++)
         {
            const uint32_t g = tid + (uint32_t) q * T;
            if (g < spn && sok && sv[q].t >= wbase && sv[q].t < wend)
            {
               const uint32_t o = itot + (g - skip);
               if (o < (uint32_t) ICAP)
               {
                  const uint64_t dt = sv[q].t - wbase;
                  sbad |= (dt >> 32) != 0;
                  sm.ikey[o] = (dt << 32) | sv[q].id;
                  sm.iaux[o] = sv[q].aux;
               }
            }
         }
         if (sbad) flag(a, F_FALLBACK);
      }
      // kept keys at their continuing index (the search array for the inserts)
#pragma unroll
      for (int j = 0; j < PER; j++)
         if ((km >> j) & 1u) sm.key[pad(ci[j])] = rk[j];
      if (tid == 0)
      {
         sm.ioff[NL + 1] = sm.ioff[NL] + sp_take;
         if (itot + sp_take > (uint32_t) ICAP || nin + itot + sp_take > (uint32_t) CAP)
         {
            flag(a, F_RETRY);
            sm.abort_ = 1;
         }
      }
      bar();   // #5
      if (sm.abort_) return;
      merge<NL>(sm, nin, rk, ra, ci, km, nin + itot + sp_take);   // #6, #7
   }
}

template <int NL>
__global__ __launch_bounds__(T, 3) void k_chain(ChainArgs a)
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
      task<NL>(sm, a, tk % a.nch, tk / a.nch);
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
   for (uint32_t d = 0; d < 5; d++)
   {
      const uint32_t os = slot_of(ntile, d, slot_side(d, nside));
      p.obase[d] = slot_base[os];
      p.ocap[d] = slot_cnt[os];
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
