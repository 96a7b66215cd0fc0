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
// Time is cut into windows [w D, (w+1) D), the last one unbounded; D per phase,
// sized from the batch's busiest port and then from the fill the previous run
// measured (engine.hip choose_windows / adapt_windows).  One workgroup task = (chain, window): it walks the chain's ports
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

// One wave per task: the scan, the reductions and the hand-off state stay in
// registers, and LDS needs no barriers (a wave's LDS operations execute in
// program order).
constexpr int T = 64;
#ifndef CH_PER_V
#define CH_PER_V 11
#endif
constexpr int PER = CH_PER_V;             // stream records per lane
constexpr int CAP = PER * T;              // stream records per (port, window)
#ifndef CH_IPER_V
#define CH_IPER_V 2
#endif
constexpr int IPER = CH_IPER_V;
constexpr int ICAP = IPER * T;            // inserts per (port, window), + spill-ins of the slow path
#ifndef CH_MINW
#define CH_MINW 3                         // waves per SIMD the registers must leave room for
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

// LDS index padding of the kept list: one u64 per 32 entries, so the lanes'
// segments (stride about PER) hit distinct banks.
__host__ __device__ constexpr uint32_t pad(uint32_t r) { return r + (r >> 5); }
constexpr int CAPP = CAP + CAP / 32 + 1;   // + the ~0 behind a full list


// Route-count fields of a chain port's outputs: SELF, the chain direction, UP,
// DOWN (an X port never sends the opposite X way; a Y port only SELF or on).
__host__ __device__ __forceinline__ uint32_t field_of(uint32_t nd, uint32_t cont)
{
   return nd == cont ? 1u : nd == P_SELF ? 0u : nd == P_UP ? 2u : 3u;
}
// The same for a record of an X chain (XC) or a Y chain, from its destination and
// the next tile (nx, ny): under XY routing an X-chain record has dx at or beyond
// nx in the chain's direction, a Y-chain record dy at or beyond ny.
template <bool XC>
__device__ __forceinline__ uint32_t route_field(uint32_t nx, uint32_t ny, uint32_t aux)
{
   const uint32_t dx = aux & AUX_C_MASK, dy = (aux >> AUX_C_BITS) & AUX_C_MASK;
   if (!XC) return dy != ny ? 1u : 0u;
   return dx != nx ? 1u : dy > ny ? 2u : dy < ny ? 3u : 0u;
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

// One chain's windows: length D (ps), nW of them; its hand-off state block and
// window-bounds block (offsets into ChainArgs::st / bt).  Chains of a phase may
// have different windows (each is sized from its own measured fill).
struct ChainWin
{
   uint64_t D;
   uint64_t st_off;               // u64 words: state of (port i, window w) at st_off + (i nW + w) SW
   uint64_t bt_off;               // u32 words: bounds of (port i, list j) at bt_off + (i nl + j)(nW + 1)
   uint32_t nW;
   uint32_t pad;
};

struct ChainArgs
{
   DevCfg c;
   const ChainPort* cp;           // [nch * len] (this phase)
   const uint32_t* bt;            // window bounds of insert slots (per chain: ChainWin::bt_off)
   Rec* recs;
   uint64_t* samp_t;
   uint32_t* samp_id;
   uint64_t* st;                  // hand-off state (per chain: ChainWin::st_off)
   unsigned long long* port_sum;
   unsigned long long* port_cnt;
   unsigned long long* port_flit;
   unsigned long long* port_last;
   unsigned* errflag;             // [0] route invariant, [2] exception tails exist, [4] chain flags
   unsigned* ctr;                 // dequeue head
   uint32_t nch, len, ntasks, pad2;
   const ChainWin* cw;            // [nch] windows per chain: window w = [w D, (w + 1) D), the last one unbounded
   const uint32_t* tasks;         // [ntasks] c << 16 | w, ordered by the window's start time w D
   uint32_t cp0;                  // unused (0)
   uint32_t pad0;
   uint64_t etag;                 // epoch << 48
   unsigned* nmax;                // [2 c] the most stream records, [2 c + 1] the most inserts of chain c's steps
   uint64_t* stamps;              // debug (GNOC_STAMPS=1): [(task * len + i) * 16 + k] phase stamps, else null
   uint32_t exp;                  // unused
   uint32_t pad1;
};


namespace ch {

struct Smem
{
   // Port i's stream is the (t, id)-merge of two sorted lists, never materialised:
   // the records kept from port i-1 (rewritten in place by port i: every read of
   // the list precedes every write) and port i's inserts (double buffered by port
   // parity: port i+1's land while port i runs).  ~0 sits behind each list's end.
   uint64_t kkey[CAPP];           // kept: (t - wbase) << 32 | id
   uint32_t kaux[CAPP];           // dx | dy << 10 | F << 20
   uint64_t ikey[2][ICAP + 1];    // inserts
   uint32_t iaux[2][ICAP + 1];
   uint64_t rkey[ICAP + 1];       // Y ports' three fetched slot ranges (premerge -> ikey); the slow
   uint32_t raux[ICAP + 1];       // path's inserts + spill-ins
   ChainPort cp[3];               // ports i, i+1, i+2 (ring)
   uint32_t blo[2][NLMAX], bhi[2][NLMAX];   // window bounds of ports i+1, i+2 (ring)
   uint32_t ioffs[2][NLMAX + 1];  // offsets of a port's local insert lists (by port parity)
};

__device__ __forceinline__ uint64_t ld1(const uint64_t* p)
{
   return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st1(uint64_t* p, uint64_t v)
{
   __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Compiler-only ordering point between LDS phases of the one wave.
__device__ __forceinline__ void wsync() { asm volatile("" ::: "memory"); }
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
__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) { return (uint32_t) __builtin_amdgcn_readlane((int) v, l); }
__device__ __forceinline__ uint64_t rdl64(uint64_t v, int l)
{
   return (uint64_t) rdl((uint32_t) v, l) | ((uint64_t) rdl((uint32_t) (v >> 32), l) << 32);
}

// Lower bound (number of entries < k) in the sorted u64 array a[0, n), by
// binary lifting: n is wave-uniform, so every lane runs floor(log2 n) + 1
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

__device__ __forceinline__ void flag(const ChainArgs& a, uint32_t f) { atomicOr(a.errflag + 4, f); }
// A window of chain c overflowed LDS: the run retries, halving that chain's windows.
__device__ __forceinline__ void flag_overflow(const ChainArgs& a, uint32_t c)
{
   flag(a, F_RETRY);
   atomicMax(a.nmax + 2 * c, 0xFFFFFFFFu);
}
__device__ __forceinline__ bool flagged(const ChainArgs& a)
{
   return (__hip_atomic_load(a.errflag + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & F_ANY) != 0;
}

// A 128-B port descriptor: 32 lanes, one dword each.  The prefetch splits into
// the load a step ahead (register) and the LDS store at the next step.
__device__ __forceinline__ void load_cp(ChainPort* dst, const ChainPort* src, uint32_t l)
{
   reinterpret_cast<uint32_t*>(dst)[l] = reinterpret_cast<const uint32_t*>(src)[l];
}
__device__ __forceinline__ uint32_t fetch_cp(const ChainPort* src, uint32_t l)
{
   return reinterpret_cast<const uint32_t*>(src)[l];
}
__device__ __forceinline__ void put_cp(ChainPort* dst, uint32_t v, uint32_t l) { reinterpret_cast<uint32_t*>(dst)[l] = v; }
// Window bounds [lo, hi) of the insert slots of port i of a chain whose bounds
// block starts at bt_off (l < 2 nl).
__device__ __forceinline__ uint32_t fetch_bounds(const ChainArgs& a, uint64_t bt_off, uint32_t nW, uint32_t i, uint32_t nl,
                                                 uint32_t w, uint32_t l)
{
   if (l >= 2 * nl) return 0u;
   const uint32_t j = l < nl ? l : l - nl;
   return a.bt[bt_off + ((uint64_t) i * nl + j) * (nW + 1) + w + (l < nl ? 0u : 1u)];
}
__device__ __forceinline__ void put_bounds(Smem& sm, uint32_t slot, uint32_t v, uint32_t nl, uint32_t l)
{
   if (l < nl) sm.blo[slot][l] = v;
   else if (l < 2 * nl) sm.bhi[slot][l - nl] = v;
}

// Poll the state words [0, nw) of block s until all carry the epoch tag (lane
// q < nw holds word q).  Wave-wide; false on abort.
__device__ bool poll_words(const ChainArgs& a, const uint64_t* s, uint32_t nw, uint32_t lane, uint64_t& v)
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
      if (lane < nw) v = ld1(s + lane);
   }
}

// Issue the loads of a port's local inserts of this window (registers); off =
// the lists' offsets in the port's insert list (uniform).
template <int NL>
__device__ __forceinline__ uint32_t fetch_inserts(Smem& sm, const ChainArgs& a, uint32_t ring, uint32_t br,
                                                  Rec (&iv)[IPER], uint32_t parity)
{
   const uint32_t lane = threadIdx.x;
   const ChainPort& P = sm.cp[ring];
   uint32_t lo[NL], off[NL + 1];
   uint64_t base[NL];
   off[0] = 0;
#pragma unroll
   for (int j = 0; j < NL; j++)
   {
      // bounds come from sorted slots; clamped so that nothing can load out of range
      const uint32_t cnt = sgpr(P.icnt[j]);
      lo[j] = min(sgpr(sm.blo[br][j]), cnt);
      const uint32_t hi = min(max(sgpr(sm.bhi[br][j]), lo[j]), cnt);
      off[j + 1] = off[j] + (hi - lo[j]);
      base[j] = sgpr64(P.ibase[j]) + lo[j];
   }
   const uint32_t itot = off[NL];
   // the lists' offsets, for premerge (LDS: no scalar registers held across the step)
   if (NL > 1 && lane <= (uint32_t) NL) sm.ioffs[parity][lane] = off[lane < (uint32_t) NL ? lane : NL];
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = lane + (uint32_t) q * T;
      iv[q].t = 0;
      iv[q].id = 0;
      iv[q].aux = 0;
      if (g < itot && g < (uint32_t) ICAP)
      {
         uint32_t j = 0;
#pragma unroll
         for (int l = 1; l < NL; l++)
            if (g >= off[l]) j = (uint32_t) l;
         iv[q] = a.recs[base[j] + (g - off[j])];
      }
   }
   return itot;
}

// Fetched inserts into LDS as keys relative to wbase: X ports (one slot)
// straight into insert list `buf`, Y ports into the staging lists (premerge).
template <int NL>
__device__ __forceinline__ bool store_inserts(Smem& sm, const Rec (&iv)[IPER], uint32_t itot, uint64_t wbase, uint32_t buf)
{
   const uint32_t lane = threadIdx.x;
   bool bad = false;
   uint64_t* K = NL > 1 ? sm.rkey : sm.ikey[buf];
   uint32_t* X = NL > 1 ? sm.raux : sm.iaux[buf];
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = lane + (uint32_t) q * T;
      if (g < itot && g < (uint32_t) ICAP)
      {
         const uint64_t dt = iv[q].t - wbase;
         bad |= dt >= OFF_LIM;
         K[g] = (dt << 32) | iv[q].id;
         X[g] = iv[q].aux;
      }
   }
   if (NL == 1 && lane == 0 && itot <= (uint32_t) ICAP) K[itot] = ~0ull;
   return __any(bad);
}

// Y ports: the staged slot ranges (each sorted) merged into insert list `buf`:
// own index + lower bounds in the other two ranges.
template <int NL>
__device__ __forceinline__ void premerge(Smem& sm, uint32_t itot, uint32_t buf, uint32_t parity)
{
   if (NL == 1) return;
   const uint32_t lane = threadIdx.x;
   wsync();
   uint32_t o[NL + 1];
#pragma unroll
   for (int l = 0; l <= NL; l++) o[l] = sm.ioffs[parity][l];
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = lane + (uint32_t) q * T;
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
      sm.ikey[buf][pos] = k;
      sm.iaux[buf][pos] = sm.raux[g];
   }
   if (lane == 0 && itot <= (uint32_t) ICAP) sm.ikey[buf][itot] = ~0ull;
   wsync();
}

// Cycles of a stream record relative to the window base cycle wb = max(wq - 1, 0):
// Time::toCycles at 1 GHz, ceil((wbase + off) / 1000) - wb, with wbase = 1000 wq + wr
// (32-bit division; off + wr + 999 < 2^32 by the OFF_LIM check on every key).
__device__ __forceinline__ uint32_t rcyc(uint32_t off, uint32_t wr, uint32_t d0)
{
   return (wr + off + 999u) / 1000u + d0;
}

// Merge path: how many inserts are among the first d records of the merged
// (kept K[0, nK), inserts I[0, nI)) stream.  Binary lifting over the insert
// list (the short one), no divergence; keys are unique (one record per packet
// per port).
__device__ __forceinline__ uint32_t mp_split(const uint64_t* K, uint32_t nK, const uint64_t* I, uint32_t nI, uint32_t d)
{
   const uint32_t lo = d > nK ? d - nK : 0u, hi = d < nI ? d : nI;
   uint32_t pos = lo;
   for (uint32_t step = nI ? 1u << (31 - __builtin_clz(nI)) : 0u; step; step >>= 1)
   {
      const uint32_t q = pos + step;
      const bool in = q <= hi;
      // insert q-1 precedes kept record d-q: it is among the first d
      const uint64_t vi = I[in ? q - 1 : 0u], vk = K[pad(in ? d - q : 0u)];
      pos = (in && vi < vk) ? q : pos;
   }
   return pos;
}

// This lane's records of the merged stream (kept from x, inserts from y; cnt
// of them) into registers, and their aggregate.
template <bool XC>
__device__ __forceinline__ Agg walk(const uint64_t* K, const uint32_t* KA, const uint64_t* I, const uint32_t* IA,
                                   uint32_t x, uint32_t y, uint32_t cnt, uint32_t wr, uint32_t d0, uint32_t nx,
                                   uint32_t ny, uint32_t cont, uint64_t (&rk)[PER], uint32_t (&ra)[PER], uint32_t& yend)
{
   Agg g;
   g.A = 0;
   g.B = 0;
   g.C = 0;
   uint64_t kx = K[pad(x)], ky = I[y];   // the heads (~0 behind each list's end)
#pragma unroll
   for (int j = 0; j < PER; j++)
   {
      rk[j] = 0;
      ra[j] = 0;
      if ((uint32_t) j < cnt)
      {
         const bool tk = kx < ky;
         rk[j] = tk ? kx : ky;
         ra[j] = *(tk ? KA + pad(x) : IA + y);
         x += tk ? 1u : 0u;
         y += tk ? 0u : 1u;
         const uint64_t h = *(tk ? K + pad(x) : I + y);
         kx = tk ? h : kx;
         ky = tk ? ky : h;
         const uint32_t p = aux_F(ra[j]);
         const uint32_t nb = g.B + p, b2 = rcyc((uint32_t) (rk[j] >> 32), wr, d0) + p;
         g.B = nb > b2 ? nb : b2;
         g.A += p;
         g.C += 1ull << (16 * route_field<XC>(nx, ny, ra[j]));
      }
   }
   yend = y;
   return g;
}

// Spill-ins of this port (slow path): [Kpp, Pep) of its chain slot, written by
// earlier windows at the previous port (sorted: FIFO departure order).  Those
// with t in this window join the port's insert list: (I, nI) and they merge into
// the staging list.  Returns the records taken; skip = those consumed by
// earlier windows.
__device__ uint32_t spill_in(Smem& sm, const ChainArgs& a, uint64_t sbase, uint32_t spn, const uint64_t* I,
                             const uint32_t* IA, uint32_t nI, uint32_t nK, uint64_t wbase, uint64_t wlen, uint32_t& skip)
{
   const uint32_t lane = threadIdx.x;
   Rec sv[IPER];
   uint32_t nb = 0, nt = 0;
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = lane + (uint32_t) q * T;
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
   skip = rdl(wave_sum32(nb), 63);
   const uint32_t take = rdl(wave_sum32(nt), 63);
   if (!take) return 0;
   // staged right behind the kept list's end (the caller checked the room)
   uint64_t* const sk = sm.kkey + pad(nK) + 1;
   uint32_t* const sa = sm.kaux + pad(nK) + 1;
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = lane + (uint32_t) q * T;
      if (g < spn && sv[q].t >= wbase && sv[q].t - wbase < wlen)
      {
         sk[g - skip] = ((sv[q].t - wbase) << 32) | sv[q].id;
         sa[g - skip] = sv[q].aux;
      }
   }
   wsync();
#pragma unroll
   for (int q = 0; q < IPER; q++)
   {
      const uint32_t g = lane + (uint32_t) q * T;
      if (g < take)
      {
         const uint64_t k = sk[g];
         const uint32_t p = g + lb(I, nI, k);
         sm.rkey[p] = k;
         sm.raux[p] = sa[g];
      }
      if (g < nI)
      {
         const uint64_t k = I[g];
         const uint32_t p = g + lb(sk, take, k);
         sm.rkey[p] = k;
         sm.raux[p] = IA[g];
      }
   }
   if (lane == 0) sm.rkey[nI + take] = ~0ull;
   wsync();
   return take;
}

// State word `lane` (< SW) of a port after a window: tail X, route counts, "no
// gap yet", the port's unconsumed spill range.
__device__ __forceinline__ uint64_t state_word(uint32_t lane, uint64_t Xo, const uint32_t (&cin)[4], uint64_t C,
                                               uint32_t nogap, uint32_t Kout, uint32_t Pend)
{
   uint64_t v = Xo;
#pragma unroll
   for (int f = 0; f < 4; f++)
      if (lane == 1u + f) v = cin[f] + cf(C, f);
   if (lane == 5) v = nogap;
   if (lane == 6) v = Kout;
   if (lane == 7) v = Pend;
   return v;
}

// ---------------------------------------------------------------------------
// one task: chain c, window w (one wave)
// ---------------------------------------------------------------------------
// Phase stamps (tools/chain_stamps.py): a -DCH_STAMPS build with GNOC_STAMPS=1.
#ifdef CH_STAMPS
#define CH_STAMP(k)                                                                                         \
   do                                                                                                      \
   {                                                                                                       \
      if (a.stamps && lane == 0) a.stamps[((uint64_t) tk * len + i) * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
   } while (0)
#else
#define CH_STAMP(k) \
   do             \
   {              \
   } while (0)
#endif

template <int NL>
__device__ void task(Smem& sm, const ChainArgs& a, uint32_t c, uint32_t w, uint32_t tk)
{
   const uint32_t lane = threadIdx.x;
   const uint64_t D = a.cw[c].D, st_off = a.cw[c].st_off, bt_off = a.cw[c].bt_off;
   const uint32_t nW = a.cw[c].nW;
   const uint64_t wbase = (uint64_t) w * D;
   const uint64_t wlen = (w + 1 < nW) ? D : OFF_LIM;   // kept offsets: t' - wbase < wlen
   const uint64_t wq = wbase / 1000ull;
   const uint32_t wr = (uint32_t) (wbase - wq * 1000ull);
   const uint64_t wb = wq ? wq - 1 : 0;          // base cycle: every request of the window has tc > wb (w > 0)
   const uint32_t d0 = (uint32_t) (wq - wb);
   const uint32_t len = a.len;
   const uint32_t cpb = c * len;
   const uint32_t mode0 = a.c.analytical ? 1u : 0u;

   // ---- prologue: descriptors and insert bounds of ports 0 and 1, port 0's inserts;
   // then the pipeline's first prefetches (port 1's inserts, port 2's descriptor and bounds)
   if (lane < 32) load_cp(&sm.cp[0], a.cp + cpb, lane);
   else if (len > 1) load_cp(&sm.cp[1], a.cp + cpb + 1, lane - 32);
   if (lane < 2 * NL) put_bounds(sm, 0, fetch_bounds(a, bt_off, nW, 0, NL, w, lane), NL, lane);
   else if (lane < 4 * NL && len > 1) put_bounds(sm, 1, fetch_bounds(a, bt_off, nW, 1, NL, w, lane - 2 * NL), NL, lane - 2 * NL);
   if (lane == 0) sm.kkey[0] = ~0ull;
   wsync();
   uint64_t rk[PER];
   uint32_t ra[PER];
   Rec iv[IPER];                 // the next port's inserts in flight
   uint32_t itot_f = 0;          // their count
   uint32_t cpv = 0, bv = 0;     // descriptor / bounds of the port after next, in flight
   uint32_t nK = 0, nI = 0;      // this port's kept records and inserts
   uint32_t P0cur = 0, nin_prev = 0, ncont_prev = 0;   // this port's chain input: records before / kept / all of this window
   uint32_t nmax = 0, imax = 0;  // the fullest stream / insert list of this task (window sizing)
   {
      nI = fetch_inserts<NL>(sm, a, 0, 0, iv, 0);
      if (nI > (uint32_t) ICAP)
      {
         if (lane == 0) flag_overflow(a, c);
         return;
      }
      if (store_inserts<NL>(sm, iv, nI, wbase, 0) && lane == 0) flag(a, F_FALLBACK);
      premerge<NL>(sm, nI, 0, 0);
      if (len > 1) itot_f = fetch_inserts<NL>(sm, a, 1, 1, iv, 1);
      if (len > 2)
      {
         if (lane < 32) cpv = fetch_cp(a.cp + cpb + 2, lane);
         else bv = fetch_bounds(a, bt_off, nW, 2, NL, w, lane - 32);
      }
   }

   for (uint32_t i = 0; i < len; i++)
   {
      const uint32_t cpi = cpb + i;
      const uint32_t b = i & 1u, bn = b ^ 1u;
      const ChainPort& P = sm.cp[i % 3];
      const bool has_next = i + 1 < len;
      uint64_t* const stw = a.st + st_off + ((uint64_t) i * nW + w) * SW;          // this window's state
      const uint64_t* const stp = w ? stw - SW : nullptr;                           // predecessor's

      // ---- [A] land last step's prefetches: port i+1's inserts, port i+2's descriptor and
      // bounds; load the predecessor's state of this port
      CH_STAMP(0);
      const uint32_t itot = itot_f;
      bool ibad = false;
      if (has_next) ibad = store_inserts<NL>(sm, iv, itot, wbase, bn);
      if (i + 2 < len)
      {
         if (lane < 32) put_cp(&sm.cp[(i + 2) % 3], cpv, lane);
         else put_bounds(sm, (i + 2) & 1, bv, NL, lane - 32);
      }
      uint64_t pv = 0;
      if (w && lane < (uint32_t) SW) pv = ld1(stp + lane);
      const uint32_t nx = sgpr(P.nx), ny = sgpr(P.ny), cont = sgpr(P.cont), rl = sgpr(P.rl), port = sgpr(P.port);
      wsync();
      CH_STAMP(7);

      const uint64_t* Ic = sm.ikey[b];
      const uint32_t* IAc = sm.iaux[b];
      uint32_t n = nK + nI, a0 = 0, cnt = 0;
      Agg ex, tot;
      bool first = true, published = false;
      uint32_t Xr = 0, mode = mode0, Kpp = 0, Pep = 0, Kout = 0, Pend = 0;
      uint32_t cin[4] = { 0, 0, 0, 0 };
      for (;;)
      {
         // ---- [B][C] this lane's segment of the merged stream, wave scan (first pass: no
         // spill-ins yet)
         {
            const uint32_t k = (n + T - 1) / T;
            a0 = min(lane * k, n);
            cnt = min(k, n - a0);
            const uint32_t y = mp_split(sm.kkey, nK, Ic, nI, a0);
            uint32_t yend = 0;
            const Agg g0 = walk<NL == 1>(sm.kkey, sm.kaux, Ic, IAc, a0 - y, y, cnt, wr, d0, nx, ny, cont, rk, ra, yend);
#ifdef CH_DEBUG
            // the next lane's split must be where this one's walk ended
            const uint32_t ynext = (uint32_t) __shfl_down((int) y, 1);
            if ((lane < 63 && cnt && a0 + cnt < n && ynext != yend) || yend > nI || a0 + cnt - yend > nK)
               flag(a, F_ROUTE | 64u);
#endif
            if (first) CH_STAMP(8);
            const Agg inc = wave_scan(g0);
            ex.A = dpp32<0x138, 0xF, 0xF>(inc.A);   // exclusive: wave_shr 1
            ex.B = dpp32<0x138, 0xF, 0xF>(inc.B);
            ex.C = dpp64<0x138, 0xF, 0xF>(inc.C);
            tot.A = rdl(inc.A, 63);
            tot.B = rdl(inc.B, 63);
            tot.C = rdl64(inc.C, 63);
         }
         if (!first) break;
         CH_STAMP(1);
         first = false;
         if (ibad && lane == 0) flag(a, F_FALLBACK);
         // Y ports: the three insert ranges into one sorted list (read at the next step)
         if (has_next) premerge<NL>(sm, itot, bn, (i + 1) & 1);

         // ---- [D] predecessor's state
         bool ok = true;
         uint64_t X_in = 0;
         if (w)
         {
            ok = poll_words(a, stp, SW, lane, pv);
            X_in = rdl64(pv, 0) & M48;
#pragma unroll
            for (int f = 0; f < 4; f++) cin[f] = (uint32_t) (rdl64(pv, 1 + f) & M48);
            mode = (uint32_t) (rdl64(pv, 5) & 1u);
            Kpp = (uint32_t) (rdl64(pv, 6) & M48);
            Pep = (uint32_t) (rdl64(pv, 7) & M48);
         }
         CH_STAMP(2);
         if (!ok) return;
         // window-relative tail: an earlier tail behaves like the base cycle (every tc > wb)
         const uint64_t xr = X_in > wb ? X_in - wb : 0;
         if (xr >= (1ull << 31))
         {
            if (lane == 0) flag(a, F_FALLBACK);
            return;
         }
         Xr = (uint32_t) xr;
         Kout = nin_prev ? P0cur + nin_prev : Kpp;   // this port's spill range after this window
         Pend = P0cur + ncont_prev;
         // publish before the outputs unless spill-ins change the stream or the history
         // tree has had no gap yet (then the outputs decide)
         published = !mode && Pep == Kpp;
         if (published && lane < (uint32_t) SW)
         {
            const uint32_t nx0 = Xr + tot.A;
            st1(stw + lane, a.etag | state_word(lane, wb + (nx0 > tot.B ? nx0 : tot.B), cin, tot.C, 0u, Kout, Pend));
         }
         CH_STAMP(3);
         // next prefetches (they land at the next step's [A]): port i+2's inserts (its
         // descriptor and bounds landed at this step's [A]), port i+3's descriptor and bounds
         if (i + 2 < len) itot_f = fetch_inserts<NL>(sm, a, (i + 2) % 3, (i + 2) & 1, iv, (i + 2) & 1);
         if (i + 3 < len)
         {
            if (lane < 32) cpv = fetch_cp(a.cp + cpi + 3, lane);
            else bv = fetch_bounds(a, bt_off, nW, i + 3, NL, w, lane - 32);
         }
         if (Pep == Kpp) break;
         // ---- slow path: spill-ins join the insert list, then rescan
         const uint32_t spn = Pep - Kpp;
         const bool sok = i > 0 && spn + nI <= (uint32_t) ICAP && (uint64_t) Kpp + spn <= a.cp[cpi - 1].ocap[1] &&
                          pad(nK) + 1 + spn <= (uint32_t) CAPP;   // room to stage the spills behind the kept list
         if (!sok)
         {
            if (lane == 0) flag(a, F_FALLBACK);
            return;
         }
         uint32_t skip = 0;
         const uint32_t take = spill_in(sm, a, a.cp[cpi - 1].obase[1] + Kpp, spn, Ic, IAc, nI, nK, wbase, wlen, skip);
         if (n + take > (uint32_t) CAP)
         {
            if (lane == 0) flag_overflow(a, c);
            return;
         }
         if (!nin_prev) Kout = Kpp + skip + take;   // the consumed prefix of the old spills
         if (!take) break;   // nothing merged: the scan stands
         Ic = sm.rkey;
         IAc = sm.raux;
         nI += take;
         n += take;          // rescan (the stream changed)
      }
      // publish now (unless the history tree still has no gap: after the outputs)
      if (!published && !mode && lane < (uint32_t) SW)
      {
         const uint32_t nx0 = Xr + tot.A;
         st1(stw + lane, a.etag | state_word(lane, wb + (nx0 > tot.B ? nx0 : tot.B), cin, tot.C, 0u, Kout, Pend));
      }

      // ---- [E] recurrence, outputs: kept records in place into the kept list
      uint32_t X = Xr + ex.A;
      X = X > ex.B ? X : ex.B;
      uint32_t run[4];
#pragma unroll
      for (int f = 0; f < 4; f++) run[f] = cin[f] + cf(ex.C, f);
      const uint32_t P0n = cin[1];   // chain-direction records before this window
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
         if (mode)
         {
            // history tree with no gap yet: an idle period makes one (:79-86); the M/G/1
            // branch fires while there is none and the tail lies beyond t + p (:58-64)
            if (tc > Xb && fgap == NONE) fgap = a0 + j;
            if (Xb > tc + p && ffire == NONE) ffire = a0 + j;
         }
         ssum += cc;
         const uint64_t dn = (uint64_t) off + (uint64_t) cc * 1000ull + rl;   // t' - wbase
         const uint32_t f = route_field<NL == 1>(nx, ny, ax);
         uint32_t pos = 0;
#pragma unroll
         for (int q = 0; q < 4; q++)
            if (f == (uint32_t) q) pos = run[q]++;
         if (f == 1)
         {
            // continuing: kept (a prefix of the window's continuing records) or spilled;
            // a spill marks the kept list's end (~0 at its index, the first one counts)
            const uint32_t ci = pos - P0n;
            const bool keep = dn < wlen;
            sm.kkey[pad(ci)] = keep ? ((dn << 32) | id) : ~0ull;
            if (keep)
            {
               sm.kaux[pad(ci)] = ax;
               nkeep++;
               continue;
            }
         }
         // the output slot of field f: read per record from the descriptor (no scalar
         // registers held across the step; the next prefetch lands in another slot)
         if (pos >= P.ocap[f]) { route = true; continue; }
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
      // the kept list's end when nothing spilled
      if (lane == 0) sm.kkey[pad(cf(tot.C, 1))] = ~0ull;
      if (__any(route) && lane == 0) flag(a, F_ROUTE);
      if (__any(bad) && lane == 0) flag(a, F_FALLBACK);
      // wave reductions: queue delay sum, kept records, first gap / M/G/1 condition
      const uint64_t ssw = rdl64(wave_sum64(ssum), 63);
      const uint32_t nin = rdl(wave_sum32(nkeep), 63);
      if (__any(spilled)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drained before the next publish
      wsync();
      CH_STAMP(4);

      // ---- [F] late publish (no gap yet), port counters, route check
      const uint32_t nx0 = Xr + tot.A;
      const uint64_t Xo = wb + (nx0 > tot.B ? nx0 : tot.B);
      if (!published && mode)
      {
         // the records are in lane order: the first lane with a gap / firing holds the first
         const uint64_t mg = __ballot(fgap != NONE), mf = __ballot(ffire != NONE);
         const uint32_t fg = mg ? rdl(fgap, __builtin_ctzll(mg)) : NONE;
         const uint32_t ff = mf ? rdl(ffire, __builtin_ctzll(mf)) : NONE;
         // the M/G/1 branch would serve a request that arrives before the first gap
         if (lane == 0 && ff != NONE && (fg == NONE || ff < fg)) flag(a, F_FALLBACK);
         if (lane < (uint32_t) SW)
            st1(stw + lane, a.etag | state_word(lane, Xo, cin, tot.C, fg == NONE ? 1u : 0u, Kout, Pend));
      }
      if (lane == 0)
      {
         if (w + 1 == nW)
         {
            // every record of the port has passed: the route counts fill every output slot
            bool full = true;
            for (uint32_t f = 0; f < 4; f++) full &= cin[f] + cf(tot.C, f) == P.ocap[f];
            if (!full) flag(a, F_ROUTE);
         }
         if (n)
         {
            atomicAdd(&a.port_sum[port], (unsigned long long) ssw);
            atomicAdd(&a.port_cnt[port], (unsigned long long) n);
            atomicAdd(&a.port_flit[port], (unsigned long long) tot.A);
            atomicMax(&a.port_last[port], (unsigned long long) Xo);
         }
      }
      nmax = n > nmax ? n : nmax;
      imax = itot > imax ? itot : imax;   // the next port's inserts (checked against ICAP below)
      // the next port's chain input: records before this window, kept, all of this window
      P0cur = cin[1];
      nin_prev = nin;
      ncont_prev = cf(tot.C, 1);
      CH_STAMP(9);
#ifdef CH_STAMPS
      if (a.stamps && lane == 0)
         a.stamps[((uint64_t) tk * len + i) * 16 + 6] = (uint64_t) n | ((uint64_t) itot << 16) |
                                                     ((uint64_t) nin << 32) | ((uint64_t) (Pep != Kpp) << 63);
#endif
      if (!has_next) break;
      if (itot > (uint32_t) ICAP || nin + itot > (uint32_t) CAP)
      {
         if (lane == 0) flag_overflow(a, c);
         return;
      }
      nK = nin;
      nI = itot;
   }
   if (lane == 0)
   {
      atomicMax(a.nmax + 2 * c, nmax);
      atomicMax(a.nmax + 2 * c + 1, imax);
   }
}

template <int NL>
__global__ __launch_bounds__(T, CH_MINW) void k_chain(ChainArgs a)
{
   __shared__ Smem sm;
   const uint32_t ntasks = a.ntasks;
   // an earlier level served a request by M/G/1 (exception tails): the chain's
   // inputs are not in FIFO order -> the level engine reruns the batch
   if (a.errflag[2] != 0)
   {
      if (threadIdx.x == 0 && blockIdx.x == 0) flag(a, F_FALLBACK);
      return;
   }
   for (;;)
   {
      // in window start-time order, strictly in order to running workgroups: a task's
      // predecessor (same chain, window - 1) is always held by a running workgroup or done
      uint32_t tk = 0;
      if (threadIdx.x == 0) tk = atomicAdd(a.ctr, 1u);
      tk = rdl(tk, 0);
      if (tk >= ntasks || flagged(a)) return;
      const uint32_t cw = a.tasks[tk];
      task<NL>(sm, a, cw >> 16, cw & 0xFFFFu, tk);
      wsync();
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
// min(t / D, nW - 1) (the last window is unbounded).
__global__ __launch_bounds__(256) void k_win_bounds(const ChainPort* __restrict__ cp, uint32_t nl, uint32_t len,
                                                    const ChainWin* __restrict__ cw, const Rec* __restrict__ recs,
                                                    uint32_t* __restrict__ bt)
{
   const uint32_t k = blockIdx.x / nl, j = blockIdx.x % nl, c = k / len, i = k % len;
   const uint64_t D = cw[c].D;
   const uint32_t nW = cw[c].nW;
   const uint64_t base = cp[k].ibase[j];
   const uint32_t n = cp[k].icnt[j];
   uint32_t* b = bt + cw[c].bt_off + ((uint64_t) i * nl + j) * (nW + 1);
   const uint64_t wl = nW - 1;
   if (n == 0)
   {
      for (uint32_t v = threadIdx.x; v <= nW; v += blockDim.x) b[v] = 0;
      return;
   }
   // t / D by a double reciprocal and one correction step (t < 2^50, D >= 1024:
   // the estimate is off by at most one); the previous record's window comes from
   // the neighbouring lane
   const double inv = 1.0 / (double) D;
   auto win = [&](uint64_t t) -> uint64_t {
      uint64_t q = (uint64_t) ((double) t * inv);
      if (q * D > t) q--;
      else if ((q + 1) * D <= t) q++;
      return q < wl ? q : wl;
   };
   // BW_U rounds of the workgroup per step: their loads are in flight together
   constexpr uint32_t BW_U = 4;
   for (uint32_t i0 = 0; i0 < n; i0 += BW_U * blockDim.x)
   {
      uint64_t tt[BW_U], tp[BW_U];
#pragma unroll
      for (uint32_t q = 0; q < BW_U; q++)
      {
         const uint32_t i = i0 + q * blockDim.x + threadIdx.x;
         tt[q] = i < n ? recs[base + i].t : 0;
         tp[q] = (threadIdx.x & 63) == 0 && i && i < n ? recs[base + i - 1].t : 0;
      }
#pragma unroll
      for (uint32_t q = 0; q < BW_U; q++)
      {
         const uint32_t i = i0 + q * blockDim.x + threadIdx.x;
         const uint64_t wi = i < n ? win(tt[q]) : wl;
         uint64_t wprev = (uint64_t) __shfl_up((long long) wi, 1);
         if ((threadIdx.x & 63) == 0) wprev = i ? win(tp[q]) : 0;
         if (i >= n) continue;
         const int64_t wp = i ? (int64_t) wprev : -1;
         for (int64_t v = wp + 1; v <= (int64_t) wi; v++) b[v] = i;
         if (i == n - 1)
            for (uint64_t v = wi + 1; v <= nW; v++) b[v] = n;
      }
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
