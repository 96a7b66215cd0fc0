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
// Time is cut into windows [w D, (w+1) D), the last one unbounded; D per chain,
// sized from the batch's busiest port and then from the fill the previous run
// measured (engine.hip choose_windows / adapt_windows).  One task = (chain,
// window) = one wave: it walks the chain's ports in order, keeping the window's
// arrival stream in LDS:
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
// Two protocols (task_ser / task_lb), chosen per phase by the engine from their
// measured times: the serial one waits for window w-1's state of each port; the
// look-back one composes the nearest inclusive state with the aggregates the
// windows after it publish right after their scans (a hot chain's windows then
// stop queueing behind each other), waiting serially only where exactness needs
// it (a queue that may still have had no gap; pending spills).
//
// A step (one port of one task) works on ROWS: the merged stream in 64-record
// rows, record 64 r + lane in lane `lane` of row r.  The merge of the kept list
// and the inserts is a bitmap over merged positions (each insert's position =
// its rank in the kept list + its index), so every lane finds its record with
// one mbcnt and every row loads with independent LDS reads; a row is scanned
// with DPP (max-plus), route ranks come from ballots + mbcnt, so one row's
// turning records of one direction land on consecutive HBM addresses and the
// kept records on consecutive LDS entries.
//
// The history tree's serial state (queue_model_history_tree.cc:58-64) only
// matters while a queue has never idled; without the M/G/1 branch it is the
// FIFO recurrence, so the chain runs FIFO and checks, per record, the branch
// condition X > t + p while the port has had no gap.  If it would fire (or an
// earlier level wrote exception tails the engine has not merged, k_exc_merge, or
// a window overflows LDS) the kernel raises a flag and the host reruns the batch
// (merged tails / smaller windows / level engine).
#include "common.h"

namespace gnoc {
namespace ch {

// One wave per task: the scan, the reductions and the hand-off state stay in
// registers, and LDS needs no barriers (a wave's LDS operations execute in
// program order).
constexpr int T = 64;
#ifndef CH_ROWS_V
#define CH_ROWS_V 11
#endif
constexpr int ROWS = CH_ROWS_V;           // stream rows per (port, window)
constexpr int CAP = ROWS * T;             // stream records per (port, window)
constexpr int IROWS = 2;
constexpr int ICAP = IROWS * T;           // inserts per (port, window); spill-ins of the slow path
constexpr int SBN = CAP + ICAP;           // stream buffer: kept [0, CAP), inserts [CAP, CAP + ICAP)
constexpr int BMW = CAP / 32;             // insert bitmap words over merged positions
#ifndef CH_XCD_ONLY
#define CH_XCD_ONLY 0     // 1: hand-off stores always kept in the L2 (XCD-local queues only)
#endif
#ifndef CH_MINW
#define CH_MINW 4                         // waves per SIMD the registers must leave room for
#endif
constexpr int NLMAX = 3;                  // local insert lists (Y ports: LOCAL, W, E)
constexpr uint32_t IJ_NWB = 1025;         // window bounds / boundaries kept in LDS: chains of at most 1,024 windows
// State granules per (chain port, window), each an epoch-tagged u64 written by one
// sc1 store:
//   INC  (inclusive, after the look-back): tail X, the 4 cumulative route counts, "no gap yet"
//   AGG  (own aggregate, before the look-back): B (absolute cycles), A, the 4 window counts
//   KO   the port's consumed spill prefix after this window
//   POST (after the outputs, its spill stores drained): the chain outputs before this
//        window (low 32 bits) and its kept count (bits 32..47)
//   MG   (with INC while the queue has had no gap yet): the QueueModelMG1 sums narr, s1,
//        s2 (exact integers) and newest, lanes G_MG .. G_MG + 3
constexpr int SW = 16;
enum : int { G_X = 0, G_CNT = 1, G_MODE = 5, G_AB = 6, G_AA = 7, G_AC = 8, G_KO = 9, G_POST = 10, G_MG = 12 };
constexpr uint64_t INC_MASK = 0x3Full, AGG_MASK = 0x1C0ull;
constexpr int SW_SER = 8;                 // the serial protocol's state: X, 4 counts, "no gap yet", KO, spill end
constexpr int LB_POST = 2 * SW;           // the look-back prefetch's lane for POST of (w-1, i-1)
static_assert(LB_POST < 64, "look-back prefetch fits one wave");
constexpr uint32_t F_RETRY = 1u;          // a window overflowed LDS: rerun with smaller windows
constexpr uint32_t F_FALLBACK = 2u;       // M/G/1 would fire, exception tails, ...: rerun on the level engine
constexpr uint32_t F_ROUTE = 4u;          // route-count invariant broken (internal error)
constexpr uint32_t F_TIMEOUT = 8u;        // a hand-off wait timed out
constexpr uint32_t F_ANY = F_RETRY | F_FALLBACK | F_ROUTE | F_TIMEOUT;
// why a chain run declined (bits above F_ANY; reported with GNOC_CHAIN_DEBUG=1)
enum : uint32_t { R_OFFSET = 1u << 8, R_TAIL = 1u << 9, R_SPILLIN = 1u << 10, R_LASTSPILL = 1u << 11, R_MG1 = 1u << 12,
                  R_EXC = 1u << 13, R_OVF_INS = 1u << 14, R_OVF_STREAM = 1u << 15, R_XDONE = 1u << 17,
                  R_MGBAD = 1u << 18, R_MGB_KEPT = 1u << 19, R_MGB_SPILL = 1u << 20, R_MGB_OVF = 1u << 21,
                  R_XCD = 1u << 22 };
constexpr uint64_t SPIN_CYCLES = 1ull << 31;
constexpr uint64_t M48 = (1ull << 48) - 1;
constexpr uint64_t OFF_LIM = (1ull << 32) - 4096;   // time offsets within a window (32-bit cycle math)
constexpr uint32_t NONE = 0xFFFFFFFFu;
static_assert(BMW <= T && CAP % 64 == 0, "bitmap words: one per lane");

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
// field, insert slots of this port, as record indices (the chain engine runs only
// while the record buffer has fewer than 2^32 records).  128 bytes: a wave loads
// it as one dword per lane (lanes 0-31; lanes 32-37 load the insert bounds of the
// window, ch::load_pd).
struct __attribute__((aligned(16))) ChainPort
{
   uint32_t obase[4];    // [0-3]   output slot first record per field (SELF, cont, UP, DOWN)
   uint32_t ocap[4];     // [4-7]   output slot capacities
   uint32_t ibase[3];    // [8-10]  insert slots (IN_LOCAL, IN_W, IN_E): first record
   uint32_t icnt[3];     // [11-13] insert slot record counts
   uint32_t port;        // [14]    tile * PORTS + dir (counters)
   uint32_t nx, ny;      // [15-16] next tile
   uint32_t rl;          // [17]    R + Lk (ps)
   uint32_t tile, dir, cont, nl;   // [18-21] (k_win_bounds, debugging)
   uint32_t oslot[4];    // [22-25] output slot index per field (their exception-tail counts, nexc)
   uint32_t pad0[6];
};
static_assert(sizeof(ChainPort) == 128, "ChainPort is one 128-B line");

// One chain's windows: nW of them, window w = [B[w] << qs, B[w+1] << qs) ps with
// B = wt + wt_off (B[0] = 0, B[nW] = ~0: the last one unbounded; boundaries in units
// of 2^qs ps so that they fit u32), D the longest (reported); its hand-off state
// block and window-bounds block (offsets into ChainArgs::st / bt).  Chains of a phase
// have their own windows, and a chain's windows their own lengths: each window is
// sized from the fill the previous run measured over its time span (engine.hip
// adapt_windows).
struct ChainWin
{
   uint64_t D;
   uint64_t st_off;               // u64 words: state of (port i, window w) at st_off + (i nW + w) SW
   uint64_t bt_off;               // u32 words: bounds of (port i, list j) at bt_off + (i nl + j)(nW + 1)
   uint64_t wt_off;               // u32 words: window boundaries B[0 .. nW] at wt_off (and the fills, ChainArgs::wfill)
   uint32_t nW;
   uint32_t pad;
};
// The window of time t among B[0 .. nW] (B[0] = 0 <= t): the last w with B[w] <= t >> qs.
__device__ __forceinline__ uint32_t win_of(const uint32_t* B, uint32_t nW, uint64_t t, uint32_t qs)
{
   const uint64_t tq64 = t >> qs;
   const uint32_t tq = tq64 < 0xFFFFFFFEull ? (uint32_t) tq64 : 0xFFFFFFFEu;
   uint32_t lo = 0, n = nW;   // B[lo] <= tq; search [lo, lo + n)
   while (n > 1)
   {
      const uint32_t h = n >> 1;
      if (B[lo + h] <= tq) lo += h, n -= h;
      else n = h;
   }
   return lo;
}

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
   const ChainWin* cw;            // [nch] windows per chain
   const uint32_t* tasks;         // [ntasks] c << 16 | w, ordered by the window's start time
   uint32_t cp0;                  // unused (0)
   uint32_t excfix;               // 1: k_exc_merge put the injection level's exception tails in order
   uint64_t etag;                 // epoch << 48
   unsigned* nmax;                // [2 c] the most stream records, [2 c + 1] the most inserts of chain c's steps
   uint64_t* stamps;              // debug (GNOC_STAMPS=1): [(task * len + i) * 16 + k] phase stamps, else null
   uint32_t lookback;             // 1: look-back over earlier windows' AGG / INC; 0: wait for window w-1's INC
   uint32_t fw;                   // this phase's flag word: errflag[4] (X) or errflag[5] (Y)
   uint32_t* nexc;                // exception-tail counts per slot (M/G/1-served turns, mg_emit)
   unsigned long long* port_mg1;  // per-port M/G/1 requests
   unsigned* mgk;                 // [nch] 2 + the last window after which a port of the chain still had no gap
   const uint32_t* mgk_lim;       // k_chain_mix: [nch] windows below it take the M/G/1 path
   // XCD-local task queues (xcd = 1): chains are assigned to the 8 XCDs; a workgroup takes
   // tasks only from the queue of the XCD it runs on (HW_REG_XCC_ID), so a chain's windows
   // hand off through that XCD's L2: granules and spills are stored plain (sc0, kept in the
   // L2) instead of written through, and read with sc1 loads (L1 bypass, L2-served)
   const uint32_t* qoff;          // [NQ + 1] first task of each queue in `tasks`
   unsigned* qctr;                // queue q's dequeue head at qctr[QSTRIDE q]; the exit count at qctr[QSTRIDE NQ]
   uint32_t xcd, qs;              // qs: window boundaries in units of 2^qs ps
   const uint32_t* wt;            // window boundaries (ChainWin::wt_off)
   uint32_t* wfill;               // [wt_off + w] the fullest step of window w: stream records | inserts << 16
};


namespace ch {

// The stream buffer of one wave: the kept list (records continuing from the
// previous port, sorted, rewritten in place by this port) at [0, CAP), this
// port's inserts at [CAP, CAP + ICAP); keys (t - wbase) << 32 | id.
struct Smem
{
   uint64_t key[SBN];
   uint32_t aux[SBN];             // dx | dy << 10 | F << 20
   uint32_t bm[BMW];              // merged positions of the inserts (bitmap)
};

__device__ __forceinline__ uint64_t ld1(const uint64_t* p)
{
   return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st1(uint64_t* p, uint64_t v)
{
   __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// A hand-off store: written through (sc1) for a reader on any XCD, or, with XCD-local
// queues (producer and consumer share the XCD's L2), kept in the L2 (sc0).
__device__ __forceinline__ void sth(uint32_t xcd, uint64_t* p, uint64_t v)
{
   if (CH_XCD_ONLY || xcd) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
   else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr uint32_t NQ = 8;        // XCD-local queues (MI355X: 8 XCDs)
constexpr uint32_t QSTRIDE = 32;  // queue heads 128 B apart
__device__ __forceinline__ uint32_t xcc_id()
{
   return (uint32_t) __builtin_amdgcn_s_getreg(20 | (0 << 6) | ((4 - 1) << 11)) & (NQ - 1);   // hwreg(HW_REG_XCC_ID, 0, 4)
}
// Compiler-only ordering point between LDS phases of the one wave.
__device__ __forceinline__ void wsync() { asm volatile("" ::: "memory"); }

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
// One level of the inclusive max-plus scan of (A, B) pairs, X -> max(X + A, B)
// (cycles relative to the window's base cycle); the identity (0, 0) is what DPP
// leaves in lanes without a source (B >= A >= 0 for every aggregate).
template <int CTRL, int RM>
__device__ __forceinline__ void scan_lvl(uint32_t& A, uint32_t& B)
{
   const uint32_t pa = dpp32<CTRL, RM, 0xF>(A), pb = dpp32<CTRL, RM, 0xF>(B);
   const uint32_t nb = pb + A;
   B = nb > B ? nb : B;
   A += pa;
}
// Inclusive wave scan (GFX9 DPP: row_shr 1, 2, 4, 8; row_bcast 15, 31).
__device__ __forceinline__ void wave_scan(uint32_t& A, uint32_t& B)
{
   scan_lvl<0x111, 0xF>(A, B);
   scan_lvl<0x112, 0xF>(A, B);
   scan_lvl<0x114, 0xF>(A, B);
   scan_lvl<0x118, 0xF>(A, B);
   scan_lvl<0x142, 0xA>(A, B);
   scan_lvl<0x143, 0xC>(A, B);
}
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
// Inclusive wave prefix sum (lane l: lanes 0..l), DPP row_shr / row_bcast.
__device__ __forceinline__ uint32_t wave_sum32_incl(uint32_t v) { return wave_sum32(v); }
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
__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) { return (uint32_t) __builtin_amdgcn_readlane((int) v, l); }
__device__ __forceinline__ uint64_t rdl64(uint64_t v, int l)
{
   return (uint64_t) rdl((uint32_t) v, l) | ((uint64_t) rdl((uint32_t) (v >> 32), l) << 32);
}
// Lanes below this one with their bit set in m.
__device__ __forceinline__ uint32_t mbcnt(uint64_t m)
{
   return __builtin_amdgcn_mbcnt_hi((uint32_t) (m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) m, 0u));
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

__device__ __forceinline__ void flag(const ChainArgs& a, uint32_t f)
{
   atomicOr(a.errflag + a.fw, f);
}
// A window of chain c overflowed LDS: the run retries, halving that chain's windows.
__device__ __forceinline__ void flag_overflow(const ChainArgs& a, uint32_t c, uint32_t why = 0u)
{
   flag(a, F_RETRY | why);
   atomicMax(a.nmax + 2 * c, 0xFFFFFFFFu);
}
__device__ __forceinline__ bool flagged(const ChainArgs& a)
{
   return (__hip_atomic_load(a.errflag + a.fw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & F_ANY) != 0;
}
// The polls' abort check rides along in lane FL (no state word uses it): the flag load
// is issued beside the state reloads, so a poll round costs one memory round trip.
constexpr uint32_t FL = 63;
__device__ __forceinline__ void ld_flag(const ChainArgs& a, uint32_t lane, uint32_t& ef)
{
   if (lane == FL) ef = __hip_atomic_load(a.errflag + a.fw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool aborted(uint32_t ef) { return (rdl(ef, (int) FL) & F_ANY) != 0; }

__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t l)
{
   return (uint32_t) __builtin_amdgcn_ds_bpermute((int) (l << 2), (int) v);
}

// Port descriptor fields (lanes 0-31 of a "pd" register) and the port's insert
// bounds of window w (lanes 32 + j: first record of list j, 32 + nl + j: end).
enum : int { PD_OBASE = 0, PD_OCAP = 4, PD_IBASE = 8, PD_ICNT = 11, PD_PORT = 14, PD_NX = 15, PD_NY = 16, PD_RL = 17,
             PD_OSLOT = 22, PD_LO = 32 };
template <int NL>
__device__ __forceinline__ uint32_t load_pd(const ChainArgs& a, uint32_t cpi, uint64_t bt_off, uint32_t nW, uint32_t i,
                                            uint32_t w)
{
   const uint32_t lane = threadIdx.x;
   if (lane < 32) return reinterpret_cast<const uint32_t*>(a.cp + cpi)[lane];
   const uint32_t l = lane - 32;
   if (l >= 2u * NL) return 0u;
   const uint32_t j = l < (uint32_t) NL ? l : l - NL;
   return a.bt[bt_off + ((uint64_t) i * NL + j) * (nW + 1) + w + (l < (uint32_t) NL ? 0u : 1u)];
}

// A port's insert lists of this window: [lo_j, hi_j) of list j, clamped to the
// slot (bounds come from sorted slots; nothing can load out of range).
template <int NL>
struct Ins
{
   uint32_t off[NL + 1];
   uint32_t base[NL];
};
template <int NL>
__device__ __forceinline__ Ins<NL> ins_lists(uint32_t pd)
{
   Ins<NL> L;
   L.off[0] = 0;
#pragma unroll
   for (int j = 0; j < NL; j++)
   {
      const uint32_t cnt = rdl(pd, PD_ICNT + j);
      const uint32_t lo = min(rdl(pd, PD_LO + j), cnt);
      const uint32_t hi = min(max(rdl(pd, PD_LO + NL + j), lo), cnt);
      L.off[j + 1] = L.off[j] + (hi - lo);
      L.base[j] = rdl(pd, PD_IBASE + j) + lo;
   }
   return L;
}
// Issue the loads of a port's inserts of this window (registers); returns their count.
template <int NL>
__device__ __forceinline__ uint32_t fetch_inserts(const ChainArgs& a, uint32_t pd, Rec (&iv)[IROWS])
{
   const uint32_t lane = threadIdx.x;
   const Ins<NL> L = ins_lists<NL>(pd);
   const uint32_t itot = L.off[NL];
#pragma unroll
   for (int q = 0; q < IROWS; q++)
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
            if (g >= L.off[l]) j = (uint32_t) l;
         iv[q] = a.recs[(uint64_t) L.base[j] + (g - L.off[j])];
      }
   }
   return itot;
}

// Fetched inserts (itot <= ICAP) into the insert region as keys relative to
// wbase.  Y ports' three lists land concatenated and are then merged in place:
// an insert's merged position is the number of inserts whose key is below its own
// (keys (t, id) are unique at a port).  The region is small (~30 keys a step), and
// every lane reads the same key in each iteration of the count (an LDS broadcast),
// so the reads pipeline -- a binary search into each other list was a chain of
// dependent LDS reads (6.4 K cycles a Y step against 1.3 K for an X step's landing,
// profiles/r3_chain_stamps_occupancy.txt).  True if a time offset leaves the
// window's 32-bit range.
template <int NL>
__device__ __forceinline__ bool land_inserts(Smem& sm, const Rec (&iv)[IROWS], uint32_t itot, uint64_t wbase, uint32_t pd)
{
   const uint32_t lane = threadIdx.x;
   bool bad = false;
   uint64_t k[IROWS];
#pragma unroll
   for (int q = 0; q < IROWS; q++)
   {
      const uint32_t g = lane + (uint32_t) q * T;
      const uint64_t dt = iv[q].t - wbase;
      k[q] = (dt << 32) | iv[q].id;
      if (g < itot)
      {
         bad |= dt >= OFF_LIM;
         sm.key[CAP + g] = k[q];
         if (NL == 1) sm.aux[CAP + g] = iv[q].aux;
      }
   }
   if (NL > 1)
   {
      (void) pd;
      wsync();
      uint32_t pos[IROWS] = {};
      static_assert(IROWS == 2, "the count below handles two rows");
      if (itot <= (uint32_t) T)
      {
#pragma unroll 4
         for (uint32_t m = 0; m < itot; m++) pos[0] += sm.key[CAP + m] < k[0] ? 1u : 0u;
      }
      else
      {
#pragma unroll 4
         for (uint32_t m = 0; m < itot; m++)
         {
            const uint64_t x = sm.key[CAP + m];
            pos[0] += x < k[0] ? 1u : 0u;
            pos[1] += x < k[1] ? 1u : 0u;
         }
      }
      // every lane's searches precede every write (one wave: LDS in program order)
      wsync();
#pragma unroll
      for (int q = 0; q < IROWS; q++)
      {
         const uint32_t g = lane + (uint32_t) q * T;
         if (g < itot)
         {
            sm.key[CAP + pos[q]] = k[q];
            sm.aux[CAP + pos[q]] = iv[q].aux;
         }
      }
   }
   wsync();
   return __any(bad);
}

// Cycles of a stream record relative to the window base cycle wb = max(wq - 1, 0):
// Time::toCycles at 1 GHz, ceil((wbase + off) / 1000) - wb, with wbase = 1000 wq + wr
// (32-bit division; off + wr + 999 < 2^32 by the OFF_LIM check on every key).
__device__ __forceinline__ uint32_t rcyc(uint32_t off, uint32_t wr, uint32_t d0)
{
   return (wr + off + 999u) / 1000u + d0;
}

// The merged stream in rows: kept [0, nK), inserts [IB, IB + nI) (both sorted).
// Each insert's merged position is its rank among the kept records + its index;
// those positions form a bitmap, and the record of merged position 64 r + lane
// is insert (inserts before it) or kept record (position - inserts before it).
template <int RW>
__device__ __forceinline__ void load_rows(Smem& sm, uint32_t nK, uint32_t IB, uint32_t nI, uint64_t (&rk)[RW],
                                          uint32_t (&ra)[RW])
{
   const uint32_t lane = threadIdx.x;
   const uint32_t n = nK + nI;
   uint32_t bmv = 0;
   if (nI)
   {
      if (lane < (uint32_t) BMW) sm.bm[lane] = 0u;
      // (at most ICAP inserts, or up to CAP spill-ins on the slow path)
      for (uint32_t m0 = 0; m0 < nI; m0 += T)
      {
         const uint32_t m = m0 + lane;
         if (m < nI)
         {
            const uint32_t P = lb(sm.key, nK, sm.key[IB + m]) + m;
            atomicOr(&sm.bm[P >> 5], 1u << (P & 31));
         }
      }
      wsync();
      if (lane < (uint32_t) BMW) bmv = sm.bm[lane];
   }
   uint32_t ib = 0;
#pragma unroll
   for (int r = 0; r < RW; r++)
   {
      if ((uint32_t) r * T >= n) break;
      const uint64_t M = (uint64_t) rdl(bmv, 2 * r) | ((uint64_t) rdl(bmv, 2 * r + 1) << 32);
      const uint32_t p = (uint32_t) r * T + lane;
      const uint32_t before = ib + mbcnt(M);
      const bool isI = (M >> lane) & 1u;
      uint32_t idx = isI ? IB + before : p - before;
      idx = p < n ? idx : 0u;
      rk[r] = sm.key[idx];
      ra[r] = sm.aux[idx];
      ib += (uint32_t) __popcll(M);
   }
}

// Per-field tables: lane 1 + q holds route field q (SELF, cont, UP, DOWN), the
// lanes of the state words that carry the route counts.
// Lane 1 + q of a row's packed field counts (8 bits per field).
__device__ __forceinline__ uint32_t field_cnt(uint32_t R, uint32_t lane)
{
   return lane - 1u < 4u ? (R >> (8u * (lane - 1u))) & 0xFFu : 0u;
}
// INC granule `lane` (< G_AB) of a port after a window: tail X, the cumulative route
// counts (the field tables, lanes 1..4), "no gap yet".
__device__ __forceinline__ uint64_t inc_word(uint32_t lane, uint64_t Xo, uint32_t cnt_t, uint32_t nogap)
{
   uint64_t v = Xo;
   if (lane - 1u < 4u) v = cnt_t;
   if (lane == G_MODE) v = nogap;
   return v;
}
// Lane l's value of a 64-bit register (ds_bpermute, any lane pattern).
__device__ __forceinline__ uint64_t sh64(uint64_t v, uint32_t l)
{
   return (uint64_t) bperm((uint32_t) v, l & 63u) | ((uint64_t) bperm((uint32_t) (v >> 32), l & 63u) << 32);
}
// Keep a kernel-argument pointer in its own scalar pair (not reloaded as part of
// a wide argument tuple), as a global-memory pointer.
template <typename P>
using gptr = __attribute__((address_space(1))) P*;
template <typename P>
__device__ __forceinline__ gptr<P> sptr(P* p)
{
   asm volatile("" : "+s"(p));
   return (gptr<P>) p;
}
#ifndef CH_PFX
#define CH_PFX 1          // 1: the row scans stage the emit's prefixes and route ranks in LDS (no rescan)
#endif
// A row's emit inputs as the row scan stages them in the kept region of LDS, one u64
// per lane: the exclusive max-plus prefix (exA: flits, < 64 * 2^11; exB: cycles), the
// lane's route rank (< 64) and, for lanes 1 + q, the row's count of field q (<= 64).
constexpr uint32_t PFX_A = (1u << 17) - 1;
static_assert(64u * AUX_F_MAX <= PFX_A, "a row's flit prefix must fit its 17 bits");
__device__ __forceinline__ uint64_t pfx_pack(uint32_t exA, uint32_t rank, uint32_t fc, uint32_t exB)
{
   return (uint64_t) (exA | rank << 17 | fc << 23) | (uint64_t) exB << 32;
}
#ifndef CH_EARLY_PF
#define CH_EARLY_PF 0     // 1: the next ports' inserts / descriptor loaded right after a step's landing
#endif
// A record that leaves the chain at slot position gp.  A turn is read by the next
// launch (the launch's end writes the L2s back): one plain 16-B store.  A spill is
// read in this launch by a later window's task once the producer published a state
// after draining its stores: 8-B stores kept in the XCD's L2 when that task runs on
// the same XCD (XCD-local queues), written through otherwise (MI355X_MICROARCH.md
// "Valid forms").  Every 64th position also writes the slot's key sample.
__device__ __forceinline__ void out_record(gptr<Rec> recs, gptr<uint64_t> samp_t, gptr<uint32_t> samp_id, uint64_t gp,
                                           uint64_t tn, uint32_t id, uint32_t ax, bool spill, uint32_t xcd)
{
   const gptr<uint64_t> q = (gptr<uint64_t>) (recs + gp);
   if (!spill)
   {
      q[0] = tn;
      q[1] = (uint64_t) id | ((uint64_t) ax << 32);
   }
   else if (CH_XCD_ONLY || xcd)
   {
      __hip_atomic_store(q, tn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_store(q + 1, (uint64_t) id | ((uint64_t) ax << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
   }
   else
   {
      __hip_atomic_store(q, tn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(q + 1, (uint64_t) id | ((uint64_t) ax << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
   }
   if ((gp & 63) == 0)
   {
      samp_t[gp >> 6] = tn;
      samp_id[gp >> 6] = id;
   }
}





// ---------------------------------------------------------------------------
// a port whose history tree has had no gap yet: the analytical branch
// ---------------------------------------------------------------------------
// While a queue has never idled its tree holds the one free interval [X, inf): a
// request with X > t + p is served by the M/G/1 formula and leaves X alone
// (queue_model_history_tree.cc:58-64, queue_model_m_g_1.cc:17-46), any other one is
// FIFO, and the first idle cycle makes a gap that ends this for good (:79-86;
// max_list_size >= 3 never prunes it).  A step of such a port first scans FIFO
// (mode_scan): if the branch cannot fire before the first gap, the row-parallel
// emit is exact; otherwise the window's records go through serial_step (kernels.hip,
// the level engine's restatement) in order (mg_emit).

// FIFO scan of the window from the carried tail Xr: the first record that finds the
// queue idle (a gap), the first the branch would serve, and sum p^2 (the M/G/1 sums).
template <typename CycF>
__device__ __forceinline__ void mode_scan(const uint64_t (&rk)[ROWS], const uint32_t (&ra)[ROWS], uint32_t n, uint32_t Xr,
                                          CycF cyc, uint32_t& fgap, uint32_t& ffire, uint64_t& sp2)
{
   const uint32_t lane = threadIdx.x;
   uint32_t Xc = Xr;
   uint64_t s2 = 0;
   fgap = ffire = NONE;
#pragma unroll
   for (int r = 0; r < ROWS; r++)
   {
      if ((uint32_t) r * T >= n) break;
      const uint32_t p0 = (uint32_t) r * T;
      const bool valid = p0 + lane < n;
      const uint32_t tc = cyc((uint32_t) (rk[r] >> 32));
      const uint32_t p = aux_F(ra[r]);
      uint32_t A = valid ? p : 0u, B = valid ? tc + p : 0u;
      wave_scan(A, B);
      const uint32_t exA = dpp32<0x138, 0xF, 0xF>(A), exB = dpp32<0x138, 0xF, 0xF>(B);   // wave_shr 1
      const uint32_t xa = Xc + exA;
      const uint32_t Xb = xa > exB ? xa : exB;
      const uint64_t gm = __ballot(valid && tc > Xb), fm = __ballot(valid && Xb > tc + p);
      if (fgap == NONE && gm) fgap = p0 + (uint32_t) __builtin_ctzll(gm);
      if (ffire == NONE && fm) ffire = p0 + (uint32_t) __builtin_ctzll(fm);
      const uint32_t Xm = Xb > tc ? Xb : tc;
      Xc = rdl(Xm + p, (int) min(63u, n - 1 - p0));
      s2 += valid ? (uint64_t) p * p : 0ull;
   }
   sp2 = rdl64(wave_sum64(s2), 63);
}

// A window of a port whose history tree has had no gap yet, when the M/G/1 branch
// fires in it (queue_model_history_tree.cc:58-64; serial_step is the one-request
// restatement).  Row by row, the requests up to the next event are served FIFO in
// parallel exactly as the common emit serves them: the tail before each lane is
// the row's max-plus prefix from the carried tail X, and two ballots find the first
// lane whose request fires the branch (X > t + p) or finds the queue idle (t > X).
// An M/G/1-served request is served alone (every lane computes the same FP64
// delay from the M/G/1 sums, queue_model_m_g_1.cc:17-46); it leaves X as it is and
// may leave FIFO order: kept, it joins the kept list (sorted afterwards), turning,
// it goes to the exception tail of its output slot (nexc; k_exc_merge puts the tails
// in order before the next phase, k_level reads them), spilled, the step fails (it
// would break the spill ranges' order).  The first idle request ends the no-gap
// prefix for good (:79-86): the rest of the window is plain FIFO.  The M/G/1 sums
// (every request updates them, :48-56) are exact integers: n, sum p, sum p^2, and
// the newest departure.  mst: lanes 0-3 the M/G/1 sums in and out.
struct MgOut
{
   uint64_t ssum, X, maxdep;
   uint32_t nkeep, mode, mg1;
   uint32_t bad;    // R_MGB_* reasons
   uint32_t kend;   // records served here (all of the window)
   bool rte, spilled, kept_exc;
};
// (only in the MG instantiation of k_chain: the common kernel should not pay for it)
template <bool F1>
__device__ __forceinline__ MgOut mg_emit(Smem& sm, const ChainArgs& a, const uint64_t (&rk)[ROWS], const uint32_t (&ra)[ROWS],
                                         uint32_t n, uint32_t fpack, uint32_t wr, uint32_t d0, uint64_t wb, uint64_t wbase,
                                         uint32_t wlen, uint32_t Xr, uint64_t& mst, uint32_t pd0, uint32_t P0n, uint32_t& run_t,
                                         uint32_t obf_t, uint32_t ocf_t)
{
   const double fq = a.c.f;
   const gptr<Rec> recs = (gptr<Rec>) a.recs;
   const gptr<uint64_t> samp_t = (gptr<uint64_t>) a.samp_t;
   const gptr<uint32_t> samp_id = (gptr<uint32_t>) a.samp_id;
   auto cyc = [&](uint32_t off) -> uint32_t {
      if (F1) return rcyc(off, wr, d0);
      return (uint32_t) (cyc_of<false>(wbase + off, fq) - wb);
   };
   auto cps = [&](uint64_t cc) -> uint64_t { return F1 ? cc * 1000ull : ps_of<false>(cc, fq); };
   const uint32_t lane = threadIdx.x;
   const uint32_t nx = rdl(pd0, PD_NX), ny = rdl(pd0, PD_NY), rl = rdl(pd0, PD_RL), dir = rdl(pd0, 19);
   const uint32_t ntile = ny * a.c.W + nx, nside = in_side_after(dir);
   uint64_t narr = rdl64(mst, 0), s1 = rdl64(mst, 1), s2 = rdl64(mst, 2), newest = rdl64(mst, 3);
   uint32_t Xc = Xr;    // the tail, relative to wb
   bool nogap = true;
   MgOut o{};
   o.kend = n;
   uint64_t ssum = 0, rte = 0, spm = 0, ssum_mg = 0;
   uint32_t nkeep = 0, s = 0;   // s: the first request not served yet
   bool kept_exc = false;
#pragma unroll
   for (int r = 0; r < ROWS; r++)
   {
      if ((uint32_t) r * T >= n) break;
      const uint32_t p0 = (uint32_t) r * T, rowlen = min((uint32_t) T, n - p0);
      const uint32_t off = (uint32_t) (rk[r] >> 32), id = (uint32_t) rk[r], ax = ra[r];
      const uint32_t tc = cyc(off), p = aux_F(ax), f = (fpack >> (2 * r)) & 3u;
      while (s < p0 + rowlen)
      {
         const uint32_t lo = s - p0;
         const bool inseg = lane >= lo && lane < rowlen;
         uint32_t A = inseg ? p : 0u, B = inseg ? tc + p : 0u;
         wave_scan(A, B);
         const uint32_t exA = dpp32<0x138, 0xF, 0xF>(A), exB = dpp32<0x138, 0xF, 0xF>(B);   // wave_shr 1
         const uint32_t xa = Xc + exA;
         const uint32_t Xb = xa > exB ? xa : exB;   // the tail ahead of this lane, lanes [lo, lane) served FIFO
         uint32_t q = rowlen;
         bool isgap = false;
         if (nogap)
         {
            const uint64_t gm = __ballot(inseg && tc > Xb), fm = __ballot(inseg && Xb > tc + p);
            if (gm | fm)
            {
               q = (uint32_t) __builtin_ctzll(gm | fm);
               isgap = (gm >> q) & 1ull;
            }
         }
         // lanes [lo, q): FIFO-served, as the common emit serves them
         const bool valid = lane >= lo && lane < q;
         const uint32_t Xm = Xb > tc ? Xb : tc;
         const uint32_t cc = valid ? Xm - tc : 0u;
         if (q > lo) Xc = rdl(Xm + p, (int) (q - 1));
         ssum += cc;
         const uint64_t dn = (uint64_t) off + cps(cc) + rl;   // t' - wbase
         const uint32_t one = valid ? 1u << (8 * f) : 0u;
         const uint32_t inc = wave_sum32(one);
         const uint32_t rank = ((inc - one) >> (8 * f)) & 0xFFu;
         const uint32_t rtot = rdl(inc, 63);
         const uint32_t gb = bperm(obf_t + run_t, 1u + f);
         const uint32_t room = bperm(ocf_t - run_t, 1u + f);
         const uint32_t kb = rdl(run_t, 2) - P0n;
         run_t += field_cnt(rtot, lane);
         const bool keep = valid && f == 1 && dn < wlen;
         const bool out = valid && !keep;
         const bool st = out && rank < room;
         nkeep += (uint32_t) __popcll(__ballot(keep));
         rte |= __ballot(out && rank >= room);
         spm |= __ballot(st && f == 1);
         if (keep)
         {
            sm.key[kb + rank] = (dn << 32) | id;
            sm.aux[kb + rank] = ax;
         }
         if (st) out_record(recs, samp_t, samp_id, (uint64_t) gb + rank, wbase + dn, id, ax, f == 1, a.xcd);
         if (nogap && q > lo)
         {
            // the M/G/1 sums of the FIFO-served requests; FIFO departures rise, the last is X
            narr += q - lo;
            s1 += rdl(A, (int) (q - 1));
            s2 += rdl(wave_sum32(valid ? p * p : 0u), 63);
            newest = newest > wb + Xc ? newest : wb + Xc;
         }
         s = p0 + q;
         if (q == rowlen) break;
         if (isgap)
         {
            // request q finds the queue idle: the no-gap prefix ends here, q on are FIFO
            nogap = false;
            continue;
         }
         // request q: M/G/1-served, the tail untouched
         const uint32_t tq = rdl(tc, (int) q), pq = rdl(p, (int) q), oq = rdl(off, (int) q), iq = rdl(id, (int) q);
         const uint32_t aq = rdl(ax, (int) q), fq1 = rdl(f, (int) q);
         SerialState ms;
         ms.X = wb + Xc;
         ms.g = 0;
         ms.mode = 1;
         ms.s1 = (double) s1;
         ms.s2 = (double) s2;
         ms.narr = narr;
         ms.newest = newest;
         ms.mg1 = 0;
         const uint64_t d = mg1_delay(ms);
         o.mg1++;
         narr += 1;
         s1 += pq;
         s2 += (uint64_t) pq * pq;
         const uint64_t dep = wb + tq + d + pq;
         newest = newest > dep ? newest : dep;
         o.maxdep = dep > o.maxdep ? dep : o.maxdep;
         ssum_mg += d;
         const uint64_t dq = (uint64_t) oq + cps(d) + rl;
         if (fq1 == 1 && dq < wlen)
         {
            if (spm) o.bad |= R_MGB_KEPT;   // kept after a spill
            const uint32_t kq = rdl(run_t, 2) - P0n;
            if (lane == 0)
            {
               sm.key[kq] = (dq << 32) | iq;
               sm.aux[kq] = aq;
            }
            run_t += lane == 2 ? 1u : 0u;
            nkeep++;
            kept_exc = true;
         }
         else if (fq1 == 1)
            o.bad |= R_MGB_SPILL;   // an M/G/1-served spill
         else if (lane == 0)
         {
            // M/G/1-served turn: the exception tail of its output slot (level.hip does the same)
            const uint32_t fd = fq1 == 0 ? P_SELF : fq1 == 2 ? P_UP : P_DOWN;
            const uint32_t osl = slot_of(ntile, fd, slot_side(fd, nside));
            const uint32_t ob = rdl(pd0, PD_OBASE + fq1), oc = rdl(pd0, PD_OCAP + fq1);
            const uint32_t x = atomicAdd(a.nexc + osl, 1u);
            atomicOr(a.errflag + 2, 1u);
            if (x >= oc) atomicOr(a.errflag, 1u);
            else
            {
               const gptr<uint64_t> qq = (gptr<uint64_t>) (recs + (uint64_t) ob + oc - 1 - x);
               __hip_atomic_store(qq, wbase + dq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
               __hip_atomic_store(qq + 1, (uint64_t) iq | ((uint64_t) aq << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
         }
         s = p0 + q + 1;
      }
   }
   wsync();
   o.ssum = rdl64(wave_sum64(ssum), 63) + ssum_mg;
   o.X = wb + Xc;
   o.mode = nogap ? 1u : 0u;
   o.nkeep = nkeep;
   o.rte = rte != 0;
   o.spilled = spm != 0;
   o.kept_exc = kept_exc;
   mst = lane == 0 ? narr : lane == 1 ? s1 : lane == 2 ? s2 : lane == 3 ? newest : 0ull;
   if (newest > M48 || s2 > M48 || narr > M48) o.bad |= R_MGB_OVF;
   return o;
}

// The kept list into (t, id) order after M/G/1-served records joined it: nearly
// sorted (insertion sort, lane 0).
__device__ __forceinline__ void kept_sort(Smem& sm, uint32_t nkeep)
{
   if (threadIdx.x == 0)
      for (uint32_t i = 1; i < nkeep; i++)
      {
         const uint64_t k = sm.key[i];
         const uint32_t v = sm.aux[i];
         uint32_t j = i;
         while (j > 0 && sm.key[j - 1] > k)
         {
            sm.key[j] = sm.key[j - 1];
            sm.aux[j] = sm.aux[j - 1];
            j--;
         }
         sm.key[j] = k;
         sm.aux[j] = v;
      }
   wsync();
}

// The M/G/1 sums after a window served FIFO with no gap (every request updates them,
// queue_model_history_tree.cc:118): n requests, sum p, sum p^2; newest = the last
// departure (FIFO: the tail).  mg_emit already did it for its window.
__device__ __forceinline__ uint64_t mg_after(uint64_t mst, bool mg, uint32_t n, uint32_t totA, uint64_t sp2, uint64_t Xo)
{
   if (mg) return mst;
   const uint32_t lane = threadIdx.x;
   if (lane == 0) return mst + n;
   if (lane == 1) return mst + totA;
   if (lane == 2) return mst + sp2;
   if (lane == 3) return mst > Xo ? mst : Xo;
   return mst;
}
// Every output slot filled: per route field, the FIFO records written plus the
// slot's exception tail (M/G/1-served turns) equal its capacity.
__device__ __forceinline__ bool route_filled(const ChainArgs& a, uint32_t pd0, uint32_t run_t, uint32_t ocf_t)
{
   const uint32_t lane = threadIdx.x;
   bool bad = lane - 1u < 4u && run_t != ocf_t;
   if (!__any(bad)) return true;
   // (a turn slot may end in an exception tail; the continuing slot never does)
   const uint32_t sl = bperm(pd0, (uint32_t) PD_OSLOT - 1u + lane);
   if (bad) bad = lane == 2 || run_t + __hip_atomic_load(a.nexc + sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ocf_t;
   return !__any(bad);
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
#elif defined(CH_MARKS)
#define CH_STAMP(k) asm volatile(";;MARK " #k ::: "memory")   // static instruction counts per phase (asm listing)
#else
#define CH_STAMP(k) \
   do             \
   {              \
   } while (0)
#endif

// Wave priority over a step: raised from the step's start until its state is
// published (the part a successor window waits on), default for the outputs.
// configs[1]: 3.11 -> 3.01 ms per run at priority 2 (CH_PRIO=0: off).
#ifndef CH_PRIO
#define CH_PRIO 2
#endif
#if CH_PRIO
#define CH_PRIO_HI() __builtin_amdgcn_s_setprio(CH_PRIO)
#define CH_PRIO_LO() __builtin_amdgcn_s_setprio(0)
#else
#define CH_PRIO_HI() do {} while (0)
#define CH_PRIO_LO() do {} while (0)
#endif

// ---------------------------------------------------------------------------
// one task, serial protocol: every window waits for window w-1's state of the
// port (published as early as possible); the state block holds SW_SER granules
// ---------------------------------------------------------------------------
// Poll the state words [0, nw) of block s until all carry the epoch tag (lane
// q < nw holds word q).  Wave-wide; false on abort.
__device__ bool poll_words(const ChainArgs& a, const uint64_t* s, uint32_t nw, uint32_t lane, uint64_t& v)
{
   const uint64_t t0 = __builtin_amdgcn_s_memtime();
   uint32_t ef = 0;
   for (;;)
   {
      bool ok = true;
      if (lane < nw) ok = (v & ~M48) == a.etag;
      if (__all(ok)) return true;
      if (aborted(ef)) return false;
      if (__builtin_amdgcn_s_memtime() - t0 > SPIN_CYCLES)
      {
         if (lane == 0) flag(a, F_TIMEOUT);
         return false;
      }
      if (lane < nw) v = ld1(s + lane);
      ld_flag(a, lane, ef);
   }
}

// State word `lane` (< SW_SER) of a port after a window: tail X, route counts (the
// field tables), "no gap yet", the port's unconsumed spill range.
__device__ __forceinline__ uint64_t state_word_ser(uint32_t lane, uint64_t Xo, uint32_t cnt_t, uint32_t nogap, uint32_t Kout,
                                               uint32_t Pend)
{
   uint64_t v = Xo;
   if (lane - 1u < 4u) v = cnt_t;
   if (lane == 5) v = nogap;
   if (lane == 6) v = Kout;
   if (lane == 7) v = Pend;
   return v;
}
template <int NL, bool F1, bool MG = false, bool RF = false>
__device__ __forceinline__ void task_ser(Smem& sm, const ChainArgs& a, uint32_t c, uint32_t w, uint32_t tk)
{
   constexpr bool XC = NL == 1;
   const uint32_t lane = threadIdx.x;
   const uint64_t st_off = a.cw[c].st_off, bt_off = a.cw[c].bt_off;
   const uint32_t nW = a.cw[c].nW;
   // (wave-uniform: kept in scalar registers)
   const uint32_t wb0 = (uint32_t) __builtin_amdgcn_readfirstlane((int) a.wt[a.cw[c].wt_off + w]);
   const uint32_t wb1 = (uint32_t) __builtin_amdgcn_readfirstlane((int) a.wt[a.cw[c].wt_off + w + 1]);
   const uint64_t wbase = (uint64_t) wb0 << a.qs;
   const uint32_t wlen = (w + 1 < nW) ? (uint32_t) (((uint64_t) wb1 << a.qs) - wbase)
                                      : (uint32_t) OFF_LIM;   // kept offsets: t' - wbase < wlen
   const bool lastw = w + 1 >= nW;
   const double fq = a.c.f;
   // base cycle wb: every request of the window has tc >= wb (1 GHz: ceil(t / 1000) > wq - 1;
   // any other frequency: Time::toCycles is monotone in t, so tc >= toCycles(wbase) > wb)
   const uint64_t wq = F1 ? wbase / 1000ull : cyc_of<false>(wbase, fq);
   const uint32_t wr = F1 ? (uint32_t) (wbase - wq * 1000ull) : 0u;
   const uint64_t wb = wq ? wq - 1 : 0;
   const uint32_t d0 = (uint32_t) (wq - wb);
   // window-relative cycles of a stream offset (time_types.h:104-109) and the ps of a
   // contention delay (:81-86): integer at 1 GHz, the reference's double expressions otherwise
   auto cyc = [&](uint32_t off) -> uint32_t {
      if (F1) return rcyc(off, wr, d0);
      return (uint32_t) (cyc_of<false>(wbase + off, fq) - wb);
   };
   auto cps = [&](uint32_t cc) -> uint64_t { return F1 ? (uint64_t) cc * 1000ull : ps_of<false>(cc, fq); };
   const uint32_t len = a.len;
   const uint32_t cpb = c * len;
   const uint32_t mode0 = a.c.analytical ? 1u : 0u;
   const gptr<Rec> recs = sptr(a.recs);
#ifdef CH_STAMPS
   if (a.stamps && lane == 0) a.stamps[(uint64_t) tk * len * 16 + 10] = __builtin_amdgcn_s_memrealtime();
#endif

   // ---- prologue: descriptors of ports 0..2 (with their insert bounds), port 0's
   // inserts landed, port 1's in flight
   uint32_t pd0 = load_pd<NL>(a, cpb, bt_off, nW, 0, w);
   uint32_t pd1 = len > 1 ? load_pd<NL>(a, cpb + 1, bt_off, nW, 1, w) : 0u;
   uint32_t pd2 = len > 2 ? load_pd<NL>(a, cpb + 2, bt_off, nW, 2, w) : 0u;
   Rec iv[IROWS];
   uint32_t nI = fetch_inserts<NL>(a, pd0, iv);
   if (nI > (uint32_t) ICAP)
   {
      if (lane == 0) flag_overflow(a, c, R_OVF_INS);
      return;
   }
   if (land_inserts<NL>(sm, iv, nI, wbase, pd0) && lane == 0) flag(a, F_FALLBACK | R_OFFSET);
   uint32_t itot_f = len > 1 ? fetch_inserts<NL>(a, pd1, iv) : 0u;   // port 1's inserts, landed in step 0
   uint32_t pdn_e = 0;           // (CH_EARLY_PF) port i+3's descriptor, loaded after this step's landing

   uint64_t rk[ROWS];
   uint32_t ra[ROWS];
   uint32_t nK = 0;              // this port's kept records
   uint32_t P0cur = 0, nin_prev = 0, ncont_prev = 0;   // this port's chain input: records before / kept / all of this window
   uint32_t ob1p = 0, oc1p = 0;  // the previous port's chain output slot (spill-ins)
   uint32_t nmax = 0, imax = nI; // the fullest stream / insert list of this task (window sizing)

   for (uint32_t i = 0; i < len; i++)
   {
      const bool has_next = i + 1 < len;
      uint64_t* const stw = a.st + st_off + ((uint64_t) i * nW + w) * SW;          // this window's state
      const uint64_t* const stp = w ? stw - SW : nullptr;                           // predecessor's
      CH_STAMP(0);
      CH_PRIO_HI();
      uint64_t pv = 0;
      if (w && lane < (uint32_t) SW_SER) pv = ld1(stp + lane);
      const uint32_t nx = rdl(pd0, PD_NX), ny = rdl(pd0, PD_NY);

      // ---- [B] the merged stream in rows; per-row max-plus scans, route-field totals
      uint32_t n = nK + nI, IB = CAP;
      uint32_t fpack = 0, tc_t = 0;
      uint32_t totA = 0, totB = 0;
      bool first = true, published = false;
      uint32_t Xr = 0, mode = mode0, Kpp = 0, Pep = 0, Kout = 0, Pend = 0;
      uint64_t mst = 0;   // lanes 0-3: the M/G/1 sums while the queue has had no gap (window 0: none yet)
      uint32_t cin_t = 0;
      const uint32_t itot = itot_f;
      for (;;)
      {
         load_rows<ROWS>(sm, nK, IB, nI, rk, ra);
         if (first) CH_STAMP(1);
         totA = totB = 0;
         fpack = 0;
         tc_t = 0;
#pragma unroll
         for (int r = 0; r < ROWS; r++)
         {
            if ((uint32_t) r * T >= n) break;
            const bool valid = (uint32_t) r * T + lane < n;
            const uint32_t p = aux_F(ra[r]);
            const uint32_t tcv = cyc((uint32_t) (rk[r] >> 32)) + p;   // (every lane: no exec branch)
            uint32_t A = valid ? p : 0u;
            uint32_t B = valid ? tcv : 0u;
            wave_scan(A, B);
            const uint32_t rA = rdl(A, 63), rB = rdl(B, 63);
            const uint32_t nb = totB + rA;
            totB = nb > rB ? nb : rB;
            totA += rA;
            const uint32_t f = route_field<XC>(nx, ny, ra[r]);
            fpack |= (valid ? f : 0u) << (2 * r);
            const uint32_t one = valid ? 1u << (8 * f) : 0u;
            const uint32_t inc = wave_sum32(one);
            const uint32_t fc = field_cnt(rdl(inc, 63), lane);
            tc_t += fc;
            if (CH_PFX && !MG)
            {
               // the emit's inputs of this row into the kept region (the stream is in
               // registers now; the emit's kept records of rows <= r' land below row
               // r' + 1's entries, and a rescan after spill-ins stages them again)
               const uint32_t exA = dpp32<0x138, 0xF, 0xF>(A), exB = dpp32<0x138, 0xF, 0xF>(B);   // wave_shr 1
               sm.key[(uint32_t) r * T + lane] = pfx_pack(exA, ((inc - one) >> (8 * f)) & 0x3Fu, fc, exB);
            }
         }
         if (!first) break;
         CH_STAMP(2);
         first = false;
         // the stream is in registers: the insert region takes the next port's inserts
         if (has_next)
         {
            if (itot > (uint32_t) ICAP)
            {
               if (lane == 0) flag_overflow(a, c, R_OVF_INS);
               return;
            }
            // the prefetched inserts are consumed only here: tie them to the scan's result so
            // the compiler cannot hoist their use (and the wait for their loads, which also
            // waits for the previous step's stores) to the top of the step
#pragma unroll
            for (int q = 0; q < IROWS; q++) asm volatile("" : "+v"(iv[q].t), "+v"(iv[q].id), "+v"(iv[q].aux) : "s"(totB));
            if (land_inserts<NL>(sm, iv, itot, wbase, pd1) && lane == 0) flag(a, F_FALLBACK | R_OFFSET);
            if (CH_EARLY_PF)
            {
               // the insert registers are free again: port i+2's inserts and port i+3's
               // descriptor load while this step scans and emits (the ring moves at the end)
               if (i + 2 < len) itot_f = fetch_inserts<NL>(a, pd2, iv);
               pdn_e = i + 3 < len ? load_pd<NL>(a, cpb + i + 3, bt_off, nW, i + 3, w) : 0u;
            }
         }
         CH_STAMP(3);

         // ---- [D] predecessor's state
         bool ok = true;
         uint64_t X_in = 0;
         if (w)
         {
            ok = poll_words(a, stp, SW_SER, lane, pv);
            X_in = rdl64(pv, 0) & M48;
            cin_t = lane - 1u < 4u ? (uint32_t) (pv & M48) : 0u;
            mode = (uint32_t) (rdl64(pv, 5) & 1u);
            Kpp = (uint32_t) (rdl64(pv, 6) & M48);
            Pep = (uint32_t) (rdl64(pv, 7) & M48);
            // no gap yet: the M/G/1 sums after window w-1 (published with its state; only
            // the MG instantiation serves the branch, the other one declines where it fires)
            if (MG && ok && mode)
            {
               uint64_t mv = 0;
               ok = poll_words(a, stp + G_MG, 4, lane, mv);
               mst = lane < 4u ? mv & M48 : 0ull;
            }
         }
         CH_STAMP(4);
         if (!ok) return;
         // window-relative tail: an earlier tail behaves like the base cycle (every tc > wb)
         const uint64_t xr = X_in > wb ? X_in - wb : 0;
         if (xr >= (1ull << 31))
         {
            if (lane == 0) flag(a, F_FALLBACK | R_TAIL);
            return;
         }
         Xr = (uint32_t) xr;
         Kout = nin_prev ? P0cur + nin_prev : Kpp;   // this port's spill range after this window
         Pend = P0cur + ncont_prev;
         // publish before the outputs unless spill-ins change the stream or the history
         // tree has had no gap yet (then the outputs decide)
         published = !mode && Pep == Kpp;
         if (published && lane < (uint32_t) SW_SER)
         {
            const uint32_t x0 = Xr + totA;
            sth(a.xcd, stw + lane, a.etag | state_word_ser(lane, wb + (x0 > totB ? x0 : totB), cin_t + tc_t, 0u, Kout, Pend));
         }
         if (Pep == Kpp) break;
         // ---- slow path: spill-ins (records the previous port spilled in earlier windows,
         // sorted: FIFO departures) with t in this window join the stream as inserts
         // behind the merged stream, then the rows are rebuilt
         const uint32_t spn = Pep - Kpp;
         if (!(i > 0 && (uint64_t) Kpp + spn <= oc1p))
         {
            if (lane == 0) flag(a, F_FALLBACK | R_SPILLIN);
            return;
         }
         uint32_t skip = 0, take = 0;
         for (uint32_t g0 = 0; g0 < spn; g0 += T)
         {
            const uint32_t g = g0 + lane;
            uint64_t t = 0, ia = 0;
            if (g < spn)
            {
               const uint64_t* r = reinterpret_cast<const uint64_t*>(a.recs + (uint64_t) ob1p + Kpp + g);
               t = ld1(r);
               ia = ld1(r + 1);
            }
            const bool early = g < spn && t < wbase;
            const bool in = g < spn && t >= wbase && t - wbase < wlen;
            const uint64_t mt = __ballot(in);
            const uint32_t dst = n + take + mbcnt(mt);
            if (in && dst < (uint32_t) CAP)
            {
               sm.key[dst] = ((t - wbase) << 32) | (uint32_t) ia;
               sm.aux[dst] = (uint32_t) (ia >> 32);
            }
            skip += (uint32_t) __popcll(__ballot(early));
            take += (uint32_t) __popcll(mt);
            if (__ballot(g < spn && !early && !in)) break;   // the rest leave after this window
         }
         // the spill-in loads have all landed (a wait the compiler sees: no load stays
         // pending into the output rows, where a vmcnt(0) would also wait for the stores)
         __builtin_amdgcn_s_waitcnt(0x0F70);
         wsync();
         if (!nin_prev) Kout = Kpp + skip + take;   // the consumed prefix of the old spills
         if (!take) break;                          // nothing merged: the scan stands
         if (n + take > (uint32_t) CAP)
         {
            if (lane == 0) flag_overflow(a, c, R_OVF_STREAM);
            return;
         }
         // the stream back into the kept region (only now: with nothing merged, the row
         // scans' staged prefixes there stand), the spill-ins behind it
#pragma unroll
         for (int r = 0; r < ROWS; r++)
         {
            const uint32_t p = (uint32_t) r * T + lane;
            if ((uint32_t) r * T >= n) break;
            if (p < n)
            {
               sm.key[p] = rk[r];
               sm.aux[p] = ra[r];
            }
         }
         nK = n;
         IB = n;
         nI = take;
         n += take;          // rescan (the stream changed)
      }
      CH_STAMP(5);
      // publish now (unless the history tree still has no gap: after the outputs)
      if (!published && !mode && lane < (uint32_t) SW_SER)
      {
         const uint32_t x0 = Xr + totA;
         sth(a.xcd, stw + lane, a.etag | state_word_ser(lane, wb + (x0 > totB ? x0 : totB), cin_t + tc_t, 0u, Kout, Pend));
      }

      CH_PRIO_LO();
      // ---- [E] recurrence and outputs, row by row: kept records in place into the kept list
      const uint32_t rl = rdl(pd0, PD_RL);
      // field tables (lane 1 + q): output slot base, capacity, records routed so far
      const uint32_t obf_t = bperm(pd0, lane - 1u), ocf_t = bperm(pd0, lane + 3u);
      uint32_t run_t = cin_t;
      const uint32_t P0n = rdl(cin_t, 2);   // chain-direction records before this window
      const gptr<uint64_t> samp_t = sptr(a.samp_t);
      const gptr<uint32_t> samp_id = sptr(a.samp_id);
      uint64_t ssum = 0;
      uint32_t Xc = Xr, nkeep = 0, fgap = NONE, ffire = NONE;
      uint64_t rte = 0, spm = 0;   // lanes (over all rows) that overflowed an output slot / spilled
      // a port with no gap yet: does the analytical branch fire before the first gap?
      uint64_t sp2 = 0;
      bool mg = false;
      if (MG && mode)
      {
         // (the other instantiations find the first gap and firing in the output rows and
         // decline after them: the serial path lives in the MG one, which the host
         // switches a batch to after such a decline)
         mode_scan(rk, ra, n, Xr, cyc, fgap, ffire, sp2);
         mg = ffire != NONE && (fgap == NONE || ffire < fgap);
      }
      MgOut mo{};
      const bool mgr = MG && mg;   // this window went through mg_emit
      if constexpr (MG)
      {
         if (mg)
         {
            mo = mg_emit<F1>(sm, a, rk, ra, n, fpack, wr, d0, wb, wbase, wlen, Xr, mst, pd0, P0n, run_t, obf_t, ocf_t);
            nkeep = mo.nkeep;
            Xc = (uint32_t) (mo.X - wb);   // (the rest of the window, if any, from here)
         }
      }
      // records [k0, n): FIFO, row-parallel (all of them, or those after an M/G/1 prefix)
      const uint32_t k0 = mgr ? mo.kend : 0u;
      if (k0 < n)
#pragma unroll
      for (int r = 0; r < ROWS; r++)
      {
         if ((uint32_t) r * T >= n) break;
         const uint32_t p0 = (uint32_t) r * T;
         if (p0 + T <= k0) continue;
         const bool valid = p0 + lane < n && p0 + lane >= k0;
         const uint32_t off = (uint32_t) (rk[r] >> 32);
         const uint32_t id = (uint32_t) rk[r];
         const uint32_t ax = ra[r];
         const uint32_t tc = cyc(off);
         const uint32_t p = aux_F(ax);
         // the row's exclusive prefix: staged by the row scan, or (MG: the rows after an
         // M/G/1 prefix start at k0) rescanned
         uint32_t exA, exB, prk = 0, pfc = 0;
         if (CH_PFX && !MG)
         {
            const uint64_t pf = sm.key[p0 + lane];
            exA = (uint32_t) pf & PFX_A;
            prk = ((uint32_t) pf >> 17) & 0x3Fu;
            pfc = ((uint32_t) pf >> 23) & 0x7Fu;
            exB = (uint32_t) (pf >> 32);
         }
         else
         {
            uint32_t A = valid ? p : 0u, B = valid ? tc + p : 0u;
            wave_scan(A, B);
            exA = dpp32<0x138, 0xF, 0xF>(A);   // wave_shr 1
            exB = dpp32<0x138, 0xF, 0xF>(B);
         }
         const uint32_t xa = Xc + exA;
         const uint32_t Xb = xa > exB ? xa : exB;
         const uint32_t Xm = Xb > tc ? Xb : tc;
         const uint32_t cc = valid ? Xm - tc : 0u;
         const uint32_t Xa = Xm + p;
         if (!MG && mode)
         {
            // history tree with no gap yet: an idle period makes one (:79-86); the M/G/1
            // branch fires while there is none and the tail lies beyond t + p (:58-64)
            const uint64_t gm = __ballot(valid && tc > Xb), fm = __ballot(valid && Xb > tc + p);
            if (fgap == NONE && gm) fgap = p0 + (uint32_t) __builtin_ctzll(gm);
            if (ffire == NONE && fm) ffire = p0 + (uint32_t) __builtin_ctzll(fm);
         }
         Xc = rdl(Xa, (int) min(63u, n - 1 - p0));
         ssum += cc;
         const uint64_t dn = (uint64_t) off + cps(cc) + rl;   // t' - wbase
         // route ranks: a packed (8 bits per field) prefix count over the row
         const uint32_t f = (fpack >> (2 * r)) & 3u;
         uint32_t rank, fcnt;
         if (CH_PFX && !MG)
         {
            rank = prk;
            fcnt = pfc;
         }
         else
         {
            const uint32_t one = valid ? 1u << (8 * f) : 0u;
            const uint32_t inc = wave_sum32(one);
            rank = ((inc - one) >> (8 * f)) & 0xFFu;
            fcnt = field_cnt(rdl(inc, 63), lane);
         }
         const uint32_t gb = bperm(obf_t + run_t, 1u + f);     // obase[f] + records of f so far
         const uint32_t room = bperm(ocf_t - run_t, 1u + f);   // ocap[f] - records of f so far
         const uint32_t kb = rdl(run_t, 2) - P0n;              // kept records so far
         run_t += fcnt;
         // continuing: kept (a prefix of the window's continuing records) or spilled;
         // everything else leaves through one 16-B write-through store (turns and spills
         // alike: a spill is read in-launch by task (chain, w+1), MI355X_MICROARCH.md
         // "Valid forms"; a turn by the next launch)
         const bool keep = valid && f == 1 && dn < wlen;
         const bool out = valid && !keep;
         const bool st = out && rank < room;
         nkeep += (uint32_t) __popcll(__ballot(keep));
         rte |= __ballot(out && rank >= room);
         spm |= __ballot(st && f == 1);
         if (keep)
         {
            sm.key[kb + rank] = (dn << 32) | id;
            sm.aux[kb + rank] = ax;
         }
         if (st) out_record(recs, samp_t, samp_id, (uint64_t) gb + rank, wbase + dn, id, ax, f == 1, a.xcd);
      }
      CH_STAMP(6);
      const bool spilled = (mgr && mo.spilled) || spm != 0;
      if (((mgr && mo.rte) || rte != 0) && lane == 0) flag(a, F_ROUTE);
      if (mgr && mo.kept_exc) kept_sort(sm, nkeep);
      if (mgr && mo.spilled && nkeep > mo.nkeep) mo.bad |= R_MGB_KEPT;   // (FIFO after a spill cannot keep)
      if (mgr && mo.bad)
      {
         // an M/G/1-served spill (or a kept record after a spill): the level engine takes it
         if (lane == 0) flag(a, F_FALLBACK | R_MG1 | R_MGBAD | mo.bad);
         return;
      }

      if (spilled && lastw && lane == 0) flag(a, F_FALLBACK | R_LASTSPILL);   // the last window keeps everything
      const uint64_t ssw = (mgr ? mo.ssum : 0ull) + rdl64(wave_sum64(ssum), 63);
      if (spilled) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drained before the next publish
      wsync();

      // ---- [F] late publish (no gap yet), port counters, route check
      const uint32_t x0 = Xr + totA;
      const uint64_t Xo = mgr ? (k0 < n ? wb + Xc : mo.X) : wb + (x0 > totB ? x0 : totB);
      if (!published && mode)
      {
         // the state after the window: still no gap -> the M/G/1 sums go along
         // (not the MG instantiation) the M/G/1 branch served a request before the first gap
         if (!MG && lane == 0 && ffire != NONE && (fgap == NONE || ffire < fgap)) flag(a, F_FALLBACK | R_MG1);
         const uint32_t mout = mgr ? mo.mode : (fgap == NONE ? 1u : 0u);
         if (MG && mout) mst = mg_after(mst, mgr, n, totA, sp2, Xo);
         if (lane < (uint32_t) SW_SER) sth(a.xcd, stw + lane, a.etag | state_word_ser(lane, Xo, run_t, mout, Kout, Pend));
         if (MG && mout && lane == 0) atomicMax(a.mgk + c, w + 2u);   // window w + 1 may still serve M/G/1
         if (MG && mout && lane < 4u) sth(a.xcd, stw + G_MG + lane, a.etag | mst);
      }
      // every record of the port has passed at the last window: the route counts (and
      // the exception tails) fill every output slot
      // (only mg_emit writes exception tails of chain outputs: RF, the common windows of
      // a launch whose first windows take the M/G/1 path, count them too)
      if (lastw && (MG || RF ? !route_filled(a, pd0, run_t, ocf_t) : __any(lane - 1u < 4u && run_t != ocf_t)) && lane == 0)
         flag(a, F_ROUTE);
      if (lane == 0 && n)
      {
         const uint32_t port = rdl(pd0, PD_PORT);
         atomicAdd(&a.port_sum[port], (unsigned long long) ssw);
         atomicAdd(&a.port_cnt[port], (unsigned long long) n);
         atomicAdd(&a.port_flit[port], (unsigned long long) totA);
         atomicMax(&a.port_last[port], (unsigned long long) (mgr && mo.maxdep > Xo ? mo.maxdep : Xo));
         if (mgr && mo.mg1) atomicAdd(&a.port_mg1[port], (unsigned long long) mo.mg1);
      }
      nmax = n > nmax ? n : nmax;
      imax = itot > imax ? itot : imax;   // the next port's inserts (checked against ICAP at landing)
      // the next port's chain input: records before this window, kept, all of this window
      P0cur = P0n;
      nin_prev = nkeep;
      ncont_prev = rdl(tc_t, 2);
      ob1p = rdl(pd0, PD_OBASE + 1);
      oc1p = rdl(pd0, PD_OCAP + 1);
      CH_STAMP(7);
#ifdef CH_STAMPS
      if (a.stamps && lane == 0)
         a.stamps[((uint64_t) tk * len + i) * 16 + 9] = __builtin_amdgcn_s_memrealtime(),   // 100 MHz, one clock for all XCDs
         a.stamps[((uint64_t) tk * len + i) * 16 + 8] = (uint64_t) n | ((uint64_t) itot << 16) |
                                                     ((uint64_t) nkeep << 32) | ((uint64_t) (Pep != Kpp) << 63);
#endif
      if (!has_next) break;
      if (nkeep + itot > (uint32_t) CAP)
      {
         if (lane == 0) flag_overflow(a, c, R_OVF_STREAM);
         return;
      }
      nK = nkeep;
      nI = itot;
      // ---- next prefetches: port i+2's inserts (its descriptor landed a step ago), port
      // i+3's descriptor and bounds; the ring moves on
      if (!CH_EARLY_PF && i + 2 < len) itot_f = fetch_inserts<NL>(a, pd2, iv);
      const uint32_t pdn = CH_EARLY_PF ? pdn_e : i + 3 < len ? load_pd<NL>(a, cpb + i + 3, bt_off, nW, i + 3, w) : 0u;
      pd0 = pd1;
      pd1 = pd2;
      pd2 = pdn;
   }
   if (lane == 0)
   {
      atomicMax(a.nmax + 2 * c, nmax);
      atomicMax(a.nmax + 2 * c + 1, imax);
      a.wfill[a.cw[c].wt_off + w] = min(nmax, 0xFFFFu) | min(imax, 0xFFFFu) << 16;
   }
}


// ---------------------------------------------------------------------------
// one task, look-back protocol (AGG / INC / KO / POST granules)
// ---------------------------------------------------------------------------
template <int NL, bool F1, bool MG = false, bool RF = false>
__device__ __forceinline__ void task_lb(Smem& sm, const ChainArgs& a, uint32_t c, uint32_t w, uint32_t tk)
{
   constexpr bool XC = NL == 1;
   const uint32_t lane = threadIdx.x;
   const uint64_t st_off = a.cw[c].st_off, bt_off = a.cw[c].bt_off;
   const uint32_t nW = a.cw[c].nW;
   // (wave-uniform: kept in scalar registers)
   const uint32_t wb0 = (uint32_t) __builtin_amdgcn_readfirstlane((int) a.wt[a.cw[c].wt_off + w]);
   const uint32_t wb1 = (uint32_t) __builtin_amdgcn_readfirstlane((int) a.wt[a.cw[c].wt_off + w + 1]);
   const uint64_t wbase = (uint64_t) wb0 << a.qs;
   const uint32_t wlen = (w + 1 < nW) ? (uint32_t) (((uint64_t) wb1 << a.qs) - wbase)
                                      : (uint32_t) OFF_LIM;   // kept offsets: t' - wbase < wlen
   const bool lastw = w + 1 >= nW;
   const double fq = a.c.f;
   // base cycle wb: every request of the window has tc >= wb (1 GHz: ceil(t / 1000) > wq - 1;
   // any other frequency: Time::toCycles is monotone in t, so tc >= toCycles(wbase) > wb)
   const uint64_t wq = F1 ? wbase / 1000ull : cyc_of<false>(wbase, fq);
   const uint32_t wr = F1 ? (uint32_t) (wbase - wq * 1000ull) : 0u;
   const uint64_t wb = wq ? wq - 1 : 0;
   const uint32_t d0 = (uint32_t) (wq - wb);
   // window-relative cycles of a stream offset (time_types.h:104-109) and the ps of a
   // contention delay (:81-86): integer at 1 GHz, the reference's double expressions otherwise
   auto cyc = [&](uint32_t off) -> uint32_t {
      if (F1) return rcyc(off, wr, d0);
      return (uint32_t) (cyc_of<false>(wbase + off, fq) - wb);
   };
   auto cps = [&](uint32_t cc) -> uint64_t { return F1 ? (uint64_t) cc * 1000ull : ps_of<false>(cc, fq); };
   const uint32_t len = a.len;
   const uint32_t cpb = c * len;
   const uint32_t mode0 = a.c.analytical ? 1u : 0u;
   const gptr<Rec> recs = sptr(a.recs);
#ifdef CH_STAMPS
   if (a.stamps && lane == 0) a.stamps[(uint64_t) tk * len * 16 + 10] = __builtin_amdgcn_s_memrealtime();
#endif

   // ---- prologue: descriptors of ports 0..2 (with their insert bounds), port 0's
   // inserts landed, port 1's in flight
   uint32_t pd0 = load_pd<NL>(a, cpb, bt_off, nW, 0, w);
   uint32_t pd1 = len > 1 ? load_pd<NL>(a, cpb + 1, bt_off, nW, 1, w) : 0u;
   uint32_t pd2 = len > 2 ? load_pd<NL>(a, cpb + 2, bt_off, nW, 2, w) : 0u;
   Rec iv[IROWS];
   uint32_t nI = fetch_inserts<NL>(a, pd0, iv);
   if (nI > (uint32_t) ICAP)
   {
      if (lane == 0) flag_overflow(a, c, R_OVF_INS);
      return;
   }
   if (land_inserts<NL>(sm, iv, nI, wbase, pd0) && lane == 0) flag(a, F_FALLBACK | R_OFFSET);
   uint32_t itot_f = len > 1 ? fetch_inserts<NL>(a, pd1, iv) : 0u;   // port 1's inserts, landed in step 0
   uint32_t pdn_e = 0;           // (CH_EARLY_PF) port i+3's descriptor, loaded after this step's landing

   uint64_t rk[ROWS];
   uint32_t ra[ROWS];
   uint32_t nK = 0;              // this port's kept records
   uint32_t P0cur = 0, nin_prev = 0;   // the previous port's chain outputs before this window / kept of this window
   uint32_t ob1p = 0, oc1p = 0;  // the previous port's chain output slot (spill-ins)
   uint32_t nmax = 0, imax = nI; // the fullest stream / insert list of this task (window sizing)

   for (uint32_t i = 0; i < len; i++)
   {
      const bool has_next = i + 1 < len;
      uint64_t* const stw = a.st + st_off + ((uint64_t) i * nW + w) * SW;          // this window's state
      CH_STAMP(0);
      CH_PRIO_HI();
      // prefetch for the look-back: lanes [0, SW) the state of (w-1, i), [SW, 2 SW) of (w-2, i),
      // lane LB_POST the POST granule of (w-1, i-1) (the kept count that gives this port's spill range)
      uint64_t pv = 0;
      if (lane < 2u * SW && w > lane / SW) pv = ld1(stw - (lane / SW + 1) * SW + lane % SW);
      else if (lane == LB_POST && w && i) pv = ld1(stw - (uint64_t) nW * SW - SW + G_POST);
      const uint32_t nx = rdl(pd0, PD_NX), ny = rdl(pd0, PD_NY);

      // ---- [B] the merged stream in rows; per-row max-plus scans, route-field totals
      uint32_t n = nK + nI, IB = CAP;
      const uint32_t itot = itot_f;
      uint32_t fpack = 0, tc_t = 0, totA = 0, totB = 0;
      bool first = true;
      // spill-ins: records port i-1 spilled in earlier windows (departures after their
      // window's end) that arrive here in this window.  Pending range [Kpp, Pep): Pep = port
      // i-1's chain outputs before this window (this task's own look-back there), Kpp = the
      // prefix consumed after window w-1 (KO of (w-1, i), or from (w-1, i-1)'s POST when it
      // kept any records: kept records follow every earlier record in FIFO order)
      const uint32_t Pep = P0cur;
      uint32_t Kpp = Pep, skip = 0, take = 0;
      for (;;)
      {
         load_rows<ROWS>(sm, nK, IB, nI, rk, ra);
         if (first) CH_STAMP(1);
         fpack = tc_t = totA = totB = 0;
#pragma unroll
         for (int r = 0; r < ROWS; r++)
         {
            if ((uint32_t) r * T >= n) break;
            const bool valid = (uint32_t) r * T + lane < n;
            const uint32_t p = aux_F(ra[r]);
            const uint32_t tcv = cyc((uint32_t) (rk[r] >> 32)) + p;   // (every lane: no exec branch)
            uint32_t A = valid ? p : 0u;
            uint32_t B = valid ? tcv : 0u;
            wave_scan(A, B);
            const uint32_t rA = rdl(A, 63), rB = rdl(B, 63);
            const uint32_t nb = totB + rA;
            totB = nb > rB ? nb : rB;
            totA += rA;
            const uint32_t f = route_field<XC>(nx, ny, ra[r]);
            fpack |= (valid ? f : 0u) << (2 * r);
            const uint32_t one = valid ? 1u << (8 * f) : 0u;
            const uint32_t inc = wave_sum32(one);
            const uint32_t fc = field_cnt(rdl(inc, 63), lane);
            tc_t += fc;
            if (CH_PFX && !MG)
            {
               // the emit's inputs of this row into the kept region (the stream is in
               // registers now; the emit's kept records of rows <= r' land below row
               // r' + 1's entries, and a rescan after spill-ins stages them again)
               const uint32_t exA = dpp32<0x138, 0xF, 0xF>(A), exB = dpp32<0x138, 0xF, 0xF>(B);   // wave_shr 1
               sm.key[(uint32_t) r * T + lane] = pfx_pack(exA, ((inc - one) >> (8 * f)) & 0x3Fu, fc, exB);
            }
         }
         if (!first) break;
         first = false;
         CH_STAMP(2);
         // the stream is in registers: the insert region takes the next port's inserts
         if (has_next)
         {
            if (itot > (uint32_t) ICAP)
            {
               if (lane == 0) flag_overflow(a, c, R_OVF_INS);
               return;
            }
            // the prefetched inserts are consumed only here: tie them to the scan's result so
            // the compiler cannot hoist their use (and the wait for their loads, which also
            // waits for the previous step's stores) to the top of the step
#pragma unroll
            for (int q = 0; q < IROWS; q++) asm volatile("" : "+v"(iv[q].t), "+v"(iv[q].id), "+v"(iv[q].aux) : "s"(totB));
            if (land_inserts<NL>(sm, iv, itot, wbase, pd1) && lane == 0) flag(a, F_FALLBACK | R_OFFSET);
            if (CH_EARLY_PF)
            {
               // the insert registers are free again: port i+2's inserts and port i+3's
               // descriptor load while this step scans and emits (the ring moves at the end)
               if (i + 2 < len) itot_f = fetch_inserts<NL>(a, pd2, iv);
               pdn_e = i + 3 < len ? load_pd<NL>(a, cpb + i + 3, bt_off, nW, i + 3, w) : 0u;
            }
         }
         // ---- [D1] the predecessor window's state: its KO (or POST) for the spill range,
         // and, with the serial protocol, its INC; one poll reloads every prefetched lane
         if (w)
         {
            const bool need_k = i && Pep;
            const uint64_t t0 = __builtin_amdgcn_s_memtime();
            uint32_t ef = 0;
            for (;;)
            {
               const uint64_t mt = __ballot((pv & ~M48) == a.etag);
               bool ok = a.lookback || (mt & INC_MASK) == INC_MASK;
               if (need_k)
               {
                  const uint64_t ko = rdl64(pv, G_KO), po = rdl64(pv, LB_POST);
                  if ((ko & ~M48) == a.etag) Kpp = (uint32_t) (ko & M48);
                  else if ((po & ~M48) == a.etag && (po >> 32 & 0xFFFFu))
                     Kpp = (uint32_t) po + (uint32_t) (po >> 32 & 0xFFFFu);   // P0 + kept of (w-1, i-1)
                  else ok = false;
               }
               if (ok) break;
               if (aborted(ef)) return;
               if (__builtin_amdgcn_s_memtime() - t0 > SPIN_CYCLES)
               {
                  if (lane == 0) flag(a, F_TIMEOUT);
                  return;
               }
               if (lane < 2u * SW && w > lane / SW) pv = ld1(stw - (lane / SW + 1) * SW + lane % SW);
               else if (lane == LB_POST && i) pv = ld1(stw - (uint64_t) nW * SW - SW + G_POST);
               ld_flag(a, lane, ef);
            }
         }
         if (Kpp >= Pep) break;
         // ---- slow path: the pending spills were written by the windows back to the one
         // whose outputs start at or before Kpp: wait for each one's POST (published once its
         // stores drained); those in this window join the stream as inserts behind the merged
         // stream, and the rows are rebuilt
         const uint32_t spn = Pep - Kpp;
         if (!((uint64_t) Kpp + spn <= oc1p))
         {
            if (lane == 0) flag(a, F_FALLBACK | R_SPILLIN);
            return;
         }
         if (a.lookback)   // (the serial protocol's INC of w-1 implies every earlier window's drain)
         {
            const uint64_t t0 = __builtin_amdgcn_s_memtime();
            uint32_t ef = 0;
            for (uint32_t q = w; q-- > 0;)
            {
               uint64_t po = 0;
               for (;;)
               {
                  if (lane == 0) po = ld1(a.st + st_off + ((uint64_t) (i - 1) * nW + q) * SW + G_POST);
                  ld_flag(a, lane, ef);
                  po = rdl64(po, 0);
                  if ((po & ~M48) == a.etag) break;
                  if (aborted(ef)) return;
                  if (__builtin_amdgcn_s_memtime() - t0 > SPIN_CYCLES)
                  {
                     if (lane == 0) flag(a, F_TIMEOUT);
                     return;
                  }
               }
               if ((uint32_t) po <= Kpp) break;
            }
         }
         for (uint32_t g0 = 0; g0 < spn; g0 += T)
         {
            const uint32_t g = g0 + lane;
            uint64_t t = 0, ia = 0;
            if (g < spn)
            {
               const uint64_t* r = reinterpret_cast<const uint64_t*>(a.recs + (uint64_t) ob1p + Kpp + g);
               t = ld1(r);
               ia = ld1(r + 1);
            }
            const bool early = g < spn && t < wbase;
            const bool in = g < spn && t >= wbase && t - wbase < wlen;
            const uint64_t mt = __ballot(in);
            const uint32_t dst = n + take + mbcnt(mt);
            if (in && dst < (uint32_t) CAP)
            {
               sm.key[dst] = ((t - wbase) << 32) | (uint32_t) ia;
               sm.aux[dst] = (uint32_t) (ia >> 32);
            }
            skip += (uint32_t) __popcll(__ballot(early));
            take += (uint32_t) __popcll(mt);
            if (__ballot(g < spn && !early && !in)) break;   // the rest arrive after this window
         }
         // the spill-in loads have all landed (a wait the compiler sees: no load stays
         // pending into the output rows, where a vmcnt(0) would also wait for the stores)
         __builtin_amdgcn_s_waitcnt(0x0F70);
         wsync();
         if (!take) break;                          // nothing merged: the scan stands
         if (n + take > (uint32_t) CAP)
         {
            if (lane == 0) flag_overflow(a, c, R_OVF_STREAM);
            return;
         }
         // the stream back into the kept region (only now: with nothing merged, the row
         // scans' staged prefixes there stand), the spill-ins behind it
#pragma unroll
         for (int r = 0; r < ROWS; r++)
         {
            const uint32_t p = (uint32_t) r * T + lane;
            if ((uint32_t) r * T >= n) break;
            if (p < n)
            {
               sm.key[p] = rk[r];
               sm.aux[p] = ra[r];
            }
         }
         nK = n;
         IB = n;
         nI = take;
         n += take;          // rescan (the stream changed)
      }
      // this port's consumed spill prefix after this window (KO) and its own aggregate
      // (AGG: B in absolute cycles, A, the window's route counts): what the successors'
      // look-back composes without waiting for this task's predecessor
      const uint32_t Kout = nin_prev ? P0cur + nin_prev : Kpp + skip + take;
      if (lane - (uint32_t) G_AB < 4u && (a.lookback || lane == G_KO))
      {
         uint64_t v = wb + totB;
         if (lane == G_AA) v = totA;
         if (lane == G_AC)
            v = (uint64_t) rdl(tc_t, 1) | (uint64_t) rdl(tc_t, 2) << 12 | (uint64_t) rdl(tc_t, 3) << 24 |
                (uint64_t) rdl(tc_t, 4) << 36;
         if (lane == G_KO) v = Kout;
         sth(a.xcd, stw + lane, a.etag | v);
      }
      CH_STAMP(3);

      // ---- [D] look-back over the earlier windows of this port: the nearest INC (inclusive
      // state), composed with the AGGs of the windows after it.  While the history tree may
      // still have had no gap (an INC with the flag set, or window -1 with the analytical
      // model on) the exact state of window w-1 is needed: wait for its INC.
      uint64_t X_in = 0;
      uint32_t cin_t = 0, mode = mode0;
      uint64_t mst = 0;   // lanes 0-3: the M/G/1 sums while the queue has had no gap (window 0: none yet)
      if (w)
      {
         // lanes [0, SW) hold window w - d, [SW, 2 SW) window w - d - 1; (cA, cB, ccnt_t) is the
         // composition of windows w - d + 1 .. w - 1 (AGG form: X -> max(X + cA, cB))
         bool serial = !a.lookback;
         uint32_t d = 1;
         uint32_t cA = 0, ccnt_t = 0;
         uint64_t cB = 0;
         // prepend window AGG block b (0 or SW) to the composition
         auto prepend = [&](uint32_t b) {
            const uint64_t Bq = rdl64(pv, b + G_AB) & M48;
            const uint32_t Aq = (uint32_t) rdl64(pv, b + G_AA);
            const uint64_t Cq = rdl64(pv, b + G_AC) & M48;
            cB = Bq + cA > cB ? Bq + cA : cB;
            cA += Aq;
            ccnt_t += lane - 1u < 4u ? (uint32_t) ((Cq >> (12 * (lane - 1u))) & 0xFFFu) : 0u;
         };
         const uint64_t t0 = __builtin_amdgcn_s_memtime();
         uint32_t ef = 0;
         for (;;)
         {
            const uint64_t mt = __ballot((pv & ~M48) == a.etag);
            const bool inc1 = (mt & INC_MASK) == INC_MASK, agg1 = (mt & AGG_MASK) == AGG_MASK;
            const bool has2 = w >= d + 1;   // window w - d - 1 exists
            const bool inc2 = has2 && ((mt >> SW) & INC_MASK) == INC_MASK;
            const bool agg2 = has2 && ((mt >> SW) & AGG_MASK) == AGG_MASK;
            // the look-back ends at an INC (block src) or at window -1 (src = 2: tail 0, no
            // records, "no gap yet" iff analytical); an exact "no gap yet" state is needed
            // unless the INC found is window w-1's own
            uint32_t src = NONE;
            bool more = false;          // composed further without reaching an end: reload now
            if (inc1 && (d == 1 || !(rdl64(pv, G_MODE) & 1u))) src = 0;
            else if (inc1 || (serial && d == 1)) serial = true;   // exact: window w-1's INC only
            else if (!serial && agg1)
            {
               prepend(0);
               if (w == d) src = 2;                       // window w-d was window 0
               else if (inc2 && !(rdl64(pv, SW + G_MODE) & 1u)) src = SW;
               else if (inc2) serial = true;
               else if (agg2)
               {
                  prepend(SW);
                  if (w == d + 1) src = 2;                // window w-d-1 was window 0
                  else more = true;
                  d += 2;
               }
               else d += 1;   // window w-d-1 not there yet: it moves to lanes [0, SW)
            }
            if (src == 2 && mode0) serial = true;         // the first window may still have no gap
            if (serial && src != 0) src = NONE;
            if (src != NONE)
            {
               uint64_t Xp = 0;
               uint32_t cp_t = 0, mp = 0;
               if (src != 2)
               {
                  Xp = rdl64(pv, src + G_X) & M48;
                  const uint64_t cw_ = sh64(pv, src + lane);   // lanes 1..4: the cumulative counts
                  cp_t = lane - 1u < 4u ? (uint32_t) (cw_ & M48) : 0u;
                  mp = (uint32_t) (rdl64(pv, src + G_MODE) & 1u);
               }
               const uint64_t xa = Xp + cA;
               X_in = xa > cB ? xa : cB;
               cin_t = cp_t + ccnt_t;
               mode = d == 1 && src == 0 ? mp : 0u;
               break;
            }
            if (serial)
            {
               // exact: wait for window w-1's INC, nothing composed
               d = 1;
               cA = 0;
               cB = 0;
               ccnt_t = 0;
               more = false;
            }
            if (!more)
            {
               if (aborted(ef)) return;
               if (__builtin_amdgcn_s_memtime() - t0 > SPIN_CYCLES)
               {
                  if (lane == 0) flag(a, F_TIMEOUT);
                  return;
               }
            }
            pv = 0;
            if (lane < 2u * SW && w >= d + lane / SW) pv = ld1(stw - (lane / SW + d) * SW + lane % SW);
            ld_flag(a, lane, ef);
         }
      }
      if (MG && w && mode)
      {
         // no gap yet after window w-1 (its own INC, d == 1): the M/G/1 sums it published
         uint64_t mv = 0;
         if (!poll_words(a, stw - SW + G_MG, 4, lane, mv)) return;
         mst = lane < 4u ? mv & M48 : 0ull;
      }
      CH_STAMP(4);
      // window-relative tail: an earlier tail behaves like the base cycle (every tc > wb)
      const uint64_t xr = X_in > wb ? X_in - wb : 0;
      if (xr >= (1ull << 31))
      {
         if (lane == 0) flag(a, F_FALLBACK | R_TAIL);
         return;
      }
      const uint32_t Xr = (uint32_t) xr;
      // INC: publish before the outputs unless the history tree has had no gap yet (then
      // the outputs decide)
      if (!mode && lane < (uint32_t) G_AB)
      {
         const uint32_t x0 = Xr + totA;
         sth(a.xcd, stw + lane, a.etag | inc_word(lane, wb + (x0 > totB ? x0 : totB), cin_t + tc_t, 0u));
      }
      CH_STAMP(5);

      CH_PRIO_LO();
      // ---- [E] recurrence and outputs, row by row: kept records in place into the kept list
      const uint32_t rl = rdl(pd0, PD_RL);
      // field tables (lane 1 + q): output slot base, capacity, records routed so far
      const uint32_t obf_t = bperm(pd0, lane - 1u), ocf_t = bperm(pd0, lane + 3u);
      uint32_t run_t = cin_t;
      const uint32_t P0n = rdl(cin_t, 2);   // chain-direction records before this window
      const gptr<uint64_t> samp_t = sptr(a.samp_t);
      const gptr<uint32_t> samp_id = sptr(a.samp_id);
      uint64_t ssum = 0;
      uint32_t Xc = Xr, nkeep = 0, fgap = NONE, ffire = NONE;
      uint64_t rte = 0, spm = 0;   // lanes (over all rows) that overflowed an output slot / spilled
      // a port with no gap yet: does the analytical branch fire before the first gap?
      uint64_t sp2 = 0;
      bool mg = false;
      if (MG && mode)
      {
         // (the other instantiations find the first gap and firing in the output rows and
         // decline after them: the serial path lives in the MG one, which the host
         // switches a batch to after such a decline)
         mode_scan(rk, ra, n, Xr, cyc, fgap, ffire, sp2);
         mg = ffire != NONE && (fgap == NONE || ffire < fgap);
      }
      MgOut mo{};
      const bool mgr = MG && mg;   // this window went through mg_emit
      if constexpr (MG)
      {
         if (mg)
         {
            mo = mg_emit<F1>(sm, a, rk, ra, n, fpack, wr, d0, wb, wbase, wlen, Xr, mst, pd0, P0n, run_t, obf_t, ocf_t);
            nkeep = mo.nkeep;
            Xc = (uint32_t) (mo.X - wb);   // (the rest of the window, if any, from here)
         }
      }
      // records [k0, n): FIFO, row-parallel (all of them, or those after an M/G/1 prefix)
      const uint32_t k0 = mgr ? mo.kend : 0u;
      if (k0 < n)
#pragma unroll
      for (int r = 0; r < ROWS; r++)
      {
         if ((uint32_t) r * T >= n) break;
         const uint32_t p0 = (uint32_t) r * T;
         if (p0 + T <= k0) continue;
         const bool valid = p0 + lane < n && p0 + lane >= k0;
         const uint32_t off = (uint32_t) (rk[r] >> 32);
         const uint32_t id = (uint32_t) rk[r];
         const uint32_t ax = ra[r];
         const uint32_t tc = cyc(off);
         const uint32_t p = aux_F(ax);
         // the row's exclusive prefix: staged by the row scan, or (MG: the rows after an
         // M/G/1 prefix start at k0) rescanned
         uint32_t exA, exB, prk = 0, pfc = 0;
         if (CH_PFX && !MG)
         {
            const uint64_t pf = sm.key[p0 + lane];
            exA = (uint32_t) pf & PFX_A;
            prk = ((uint32_t) pf >> 17) & 0x3Fu;
            pfc = ((uint32_t) pf >> 23) & 0x7Fu;
            exB = (uint32_t) (pf >> 32);
         }
         else
         {
            uint32_t A = valid ? p : 0u, B = valid ? tc + p : 0u;
            wave_scan(A, B);
            exA = dpp32<0x138, 0xF, 0xF>(A);   // wave_shr 1
            exB = dpp32<0x138, 0xF, 0xF>(B);
         }
         const uint32_t xa = Xc + exA;
         const uint32_t Xb = xa > exB ? xa : exB;
         const uint32_t Xm = Xb > tc ? Xb : tc;
         const uint32_t cc = valid ? Xm - tc : 0u;
         const uint32_t Xa = Xm + p;
         if (!MG && mode)
         {
            // history tree with no gap yet: an idle period makes one (:79-86); the M/G/1
            // branch fires while there is none and the tail lies beyond t + p (:58-64)
            const uint64_t gm = __ballot(valid && tc > Xb), fm = __ballot(valid && Xb > tc + p);
            if (fgap == NONE && gm) fgap = p0 + (uint32_t) __builtin_ctzll(gm);
            if (ffire == NONE && fm) ffire = p0 + (uint32_t) __builtin_ctzll(fm);
         }
         Xc = rdl(Xa, (int) min(63u, n - 1 - p0));
         ssum += cc;
         const uint64_t dn = (uint64_t) off + cps(cc) + rl;   // t' - wbase
         // route ranks: a packed (8 bits per field) prefix count over the row
         const uint32_t f = (fpack >> (2 * r)) & 3u;
         uint32_t rank, fcnt;
         if (CH_PFX && !MG)
         {
            rank = prk;
            fcnt = pfc;
         }
         else
         {
            const uint32_t one = valid ? 1u << (8 * f) : 0u;
            const uint32_t inc = wave_sum32(one);
            rank = ((inc - one) >> (8 * f)) & 0xFFu;
            fcnt = field_cnt(rdl(inc, 63), lane);
         }
         const uint32_t gb = bperm(obf_t + run_t, 1u + f);     // obase[f] + records of f so far
         const uint32_t room = bperm(ocf_t - run_t, 1u + f);   // ocap[f] - records of f so far
         const uint32_t kb = rdl(run_t, 2) - P0n;              // kept records so far
         run_t += fcnt;
         // continuing: kept (a prefix of the window's continuing records) or spilled
         const bool keep = valid && f == 1 && dn < wlen;
         const bool out = valid && !keep;
         const bool st = out && rank < room;
         nkeep += (uint32_t) __popcll(__ballot(keep));
         rte |= __ballot(out && rank >= room);
         spm |= __ballot(st && f == 1);
         if (keep)
         {
            sm.key[kb + rank] = (dn << 32) | id;
            sm.aux[kb + rank] = ax;
         }
         if (st) out_record(recs, samp_t, samp_id, (uint64_t) gb + rank, wbase + dn, id, ax, f == 1, a.xcd);
      }
      CH_STAMP(6);
      const bool spilled = (mgr && mo.spilled) || spm != 0;
      if (((mgr && mo.rte) || rte != 0) && lane == 0) flag(a, F_ROUTE);
      if (mgr && mo.kept_exc) kept_sort(sm, nkeep);
      if (mgr && mo.spilled && nkeep > mo.nkeep) mo.bad |= R_MGB_KEPT;   // (FIFO after a spill cannot keep)
      if (mgr && mo.bad)
      {
         // an M/G/1-served spill (or a kept record after a spill): the level engine takes it
         if (lane == 0) flag(a, F_FALLBACK | R_MG1 | R_MGBAD | mo.bad);
         return;
      }

      if (spilled && lastw && lane == 0) flag(a, F_FALLBACK | R_LASTSPILL);   // the last window keeps everything
      const uint64_t ssw = (mgr ? mo.ssum : 0ull) + rdl64(wave_sum64(ssum), 63);
      if (spilled) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drained before the next publish
      wsync();

      // ---- [F] late INC (no gap yet), POST, port counters, route check
      const uint32_t x0 = Xr + totA;
      const uint64_t Xo = mgr ? (k0 < n ? wb + Xc : mo.X) : wb + (x0 > totB ? x0 : totB);
      if (mode)
      {
         // the state after the window: still no gap -> the M/G/1 sums go along
         // (not the MG instantiation) the M/G/1 branch served a request before the first gap
         if (!MG && lane == 0 && ffire != NONE && (fgap == NONE || ffire < fgap)) flag(a, F_FALLBACK | R_MG1);
         const uint32_t mout = mgr ? mo.mode : (fgap == NONE ? 1u : 0u);
         if (MG && mout) mst = mg_after(mst, mgr, n, totA, sp2, Xo);
         if (MG && mout && lane < 4u) sth(a.xcd, stw + G_MG + lane, a.etag | mst);
         if (lane < (uint32_t) G_AB) sth(a.xcd, stw + lane, a.etag | inc_word(lane, Xo, run_t, mout));
         if (MG && mout && lane == 0) atomicMax(a.mgk + c, w + 2u);   // window w + 1 may still serve M/G/1
      }
      // POST: the chain outputs before this window and whether it kept any (the next
      // window's spill range at the next port, without waiting for its KO)
      if (lane == G_POST) sth(a.xcd, stw + G_POST, a.etag | (uint64_t) P0n | (uint64_t) nkeep << 32);
      // every record of the port has passed at the last window: the route counts (and
      // the exception tails) fill every output slot
      // (only mg_emit writes exception tails of chain outputs: RF, the common windows of
      // a launch whose first windows take the M/G/1 path, count them too)
      if (lastw && (MG || RF ? !route_filled(a, pd0, run_t, ocf_t) : __any(lane - 1u < 4u && run_t != ocf_t)) && lane == 0)
         flag(a, F_ROUTE);
      if (lane == 0 && n)
      {
         const uint32_t port = rdl(pd0, PD_PORT);
         atomicAdd(&a.port_sum[port], (unsigned long long) ssw);
         atomicAdd(&a.port_cnt[port], (unsigned long long) n);
         atomicAdd(&a.port_flit[port], (unsigned long long) totA);
         atomicMax(&a.port_last[port], (unsigned long long) (mgr && mo.maxdep > Xo ? mo.maxdep : Xo));
         if (mgr && mo.mg1) atomicAdd(&a.port_mg1[port], (unsigned long long) mo.mg1);
      }
      nmax = n > nmax ? n : nmax;
      imax = itot > imax ? itot : imax;   // the next port's inserts (checked against ICAP at landing)
      // the next port's chain input: records before this window, kept of this window
      P0cur = P0n;
      nin_prev = nkeep;
      ob1p = rdl(pd0, PD_OBASE + 1);
      oc1p = rdl(pd0, PD_OCAP + 1);
      CH_STAMP(7);
#ifdef CH_STAMPS
      if (a.stamps && lane == 0)
         a.stamps[((uint64_t) tk * len + i) * 16 + 9] = __builtin_amdgcn_s_memrealtime(),   // 100 MHz, one clock for all XCDs
         a.stamps[((uint64_t) tk * len + i) * 16 + 8] = (uint64_t) n | ((uint64_t) itot << 16) |
                                                     ((uint64_t) nkeep << 32) | ((uint64_t) (take != 0) << 63);
#endif
      if (!has_next) break;
      if (nkeep + itot > (uint32_t) CAP)
      {
         if (lane == 0) flag_overflow(a, c, R_OVF_STREAM);
         return;
      }
      nK = nkeep;
      nI = itot;
      // ---- next prefetches: port i+2's inserts (its descriptor landed a step ago), port
      // i+3's descriptor and bounds; the ring moves on
      if (!CH_EARLY_PF && i + 2 < len) itot_f = fetch_inserts<NL>(a, pd2, iv);
      const uint32_t pdn = CH_EARLY_PF ? pdn_e : i + 3 < len ? load_pd<NL>(a, cpb + i + 3, bt_off, nW, i + 3, w) : 0u;
      pd0 = pd1;
      pd1 = pd2;
      pd2 = pdn;
   }
   if (lane == 0)
   {
      atomicMax(a.nmax + 2 * c, nmax);
      atomicMax(a.nmax + 2 * c + 1, imax);
      a.wfill[a.cw[c].wt_off + w] = min(nmax, 0xFFFFu) | min(imax, 0xFFFFu) << 16;
   }
}

// Task dequeue: one head per phase, or (xcd) the queue of the XCD this workgroup runs on.
// Within a queue tasks are in window start-time order, strictly in order to running
// workgroups of that XCD: a task's predecessor (same chain, window - 1, same queue) is
// always held by a running workgroup or done.
struct Deq
{
   const uint32_t* tasks;
   uint32_t qb, qn;
   unsigned* head;
};
__device__ __forceinline__ Deq deq_init(const ChainArgs& a)
{
   Deq d;
   d.tasks = a.tasks;
   if (a.xcd)
   {
      const uint32_t q = xcc_id();
      d.qb = a.qoff[q];
      d.qn = a.qoff[q + 1] - d.qb;
      d.head = a.qctr + QSTRIDE * q;
   }
   else
   {
      d.qb = 0;
      d.qn = a.ntasks;
      d.head = a.ctr;
   }
   return d;
}
__device__ __forceinline__ bool deq_next(const ChainArgs& a, const Deq& d, uint32_t& tk)
{
   uint32_t k = 0;
   if (threadIdx.x == 0) k = atomicAdd(d.head, 1u);
   k = rdl(k, 0);
   tk = d.qb + k;
   return k < d.qn && !flagged(a);
}
// XCD-local queues: the last workgroup to leave checks that every queue was served (an
// XCD that got none of the launch's workgroups leaves its chains undone: the run then
// declines, and the host reruns the batch with the one shared queue).
__device__ __forceinline__ void deq_exit(const ChainArgs& a)
{
   if (!a.xcd || threadIdx.x != 0) return;
   const unsigned x = atomicAdd(a.qctr + QSTRIDE * NQ, 1u);
   if (x + 1 != gridDim.x || flagged(a)) return;   // (an aborted run leaves its queues unfinished)
   for (uint32_t q = 0; q < NQ; q++)
   {
      const unsigned h = __hip_atomic_load(a.qctr + QSTRIDE * q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (h < a.qoff[q + 1] - a.qoff[q]) flag(a, F_FALLBACK | R_XCD);
   }
}

template <int NL, bool F1, bool LB, bool MG = false>
__global__ __launch_bounds__(T, CH_MINW) void k_chain(ChainArgs a)
{
   __shared__ Smem sm;
   // an earlier level served a request by M/G/1 (exception tails): the chain's
   // inputs are not in FIFO order -> the level engine reruns the batch
   // the X phase declined: its outputs are incomplete and the batch reruns on levels
   if (a.fw != 4 && (a.errflag[4] & F_ANY)) return;
   if (a.errflag[2] != 0 && (!a.excfix || (a.errflag[2] & 2u)))
   {
      if (threadIdx.x == 0 && blockIdx.x == 0) flag(a, F_FALLBACK | R_EXC);
      return;
   }
   const Deq dq = deq_init(a);
   uint32_t tk;
   while (deq_next(a, dq, tk))
   {
      const uint32_t cw = a.tasks[tk];
      if (LB) task_lb<NL, F1, MG>(sm, a, cw >> 16, cw & 0xFFFFu, tk);
      else task_ser<NL, F1, MG>(sm, a, cw >> 16, cw & 0xFFFFu, tk);
      wsync();
   }
   deq_exit(a);
}

// An MG batch whose M/G/1 windows are known (mgk_lim[c]: chain c's windows below it
// may serve M/G/1 requests): those tasks take the MG path, the others the common one
// (with the route check that counts exception tails) -- in one launch, so the rest of
// the phase does not wait for the M/G/1 windows' tasks to drain first.
template <int NL, bool F1, bool LB>
__global__ __launch_bounds__(T, CH_MINW) void k_chain_mix(ChainArgs a)
{
   __shared__ Smem sm;
   if (a.fw != 4 && (a.errflag[4] & F_ANY)) return;
   if (a.errflag[2] != 0 && (!a.excfix || (a.errflag[2] & 2u)))
   {
      if (threadIdx.x == 0 && blockIdx.x == 0) flag(a, F_FALLBACK | R_EXC);
      return;
   }
   const Deq dq = deq_init(a);
   uint32_t tk;
   while (deq_next(a, dq, tk))
   {
      const uint32_t cw = a.tasks[tk], c = cw >> 16, w = cw & 0xFFFFu;
      if (w < a.mgk_lim[c])
      {
         if (LB) task_lb<NL, F1, true>(sm, a, c, w, tk);
         else task_ser<NL, F1, true>(sm, a, c, w, tk);
      }
      else
      {
         if (LB) task_lb<NL, F1, false, true>(sm, a, c, w, tk);
         else task_ser<NL, F1, false, true>(sm, a, c, w, tk);
      }
      wsync();
   }
   deq_exit(a);
}

// ---------------------------------------------------------------------------
// exception tails into order (before the chains)
// ---------------------------------------------------------------------------
// A request the injection level served by M/G/1 may leave its queue out of FIFO
// order; k_level stores such records at the end of their slot (nexc counts them,
// errflag[2] says some slot has them).  The chains need every insert slot sorted by
// (t, id), the arrival order at the next port: one workgroup per such slot sorts its
// exceptions in LDS and merges them into the FIFO part in place (the FIFO records
// behind the first exception move up, chunk by chunk from the top), rewriting the
// key samples of every position it writes.  A slot with more than XM exceptions
// raises errflag[2] bit 1 and the chains decline the batch as before.
constexpr int XM = 2048;
constexpr int XT = 256;
constexpr uint32_t XS = 32;   // slots a workgroup scans per round (the tails are spread over the grid)
constexpr uint32_t XU = 8;    // records per thread per moved chunk
__device__ __forceinline__ bool key_lt(uint64_t ta, uint32_t ia, uint64_t tb, uint32_t ib)
{
   return ta < tb || (ta == tb && ia < ib);
}
__global__ __launch_bounds__(XT) void k_exc_merge(uint32_t nslots, const uint32_t* __restrict__ cnt,
                                                  const uint64_t* __restrict__ base, uint32_t* __restrict__ nexc,
                                                  Rec* __restrict__ recs, uint64_t* __restrict__ samp_t,
                                                  uint32_t* __restrict__ samp_id, unsigned* __restrict__ errflag)
{
   __shared__ uint64_t et[XM];
   __shared__ uint32_t eid[XM], eax[XM], edst[XM];
   __shared__ uint32_t s_list[XT], s_n;
   if (errflag[2] == 0) return;   // no exception anywhere
   const uint32_t tid = threadIdx.x;
   for (uint32_t s0 = blockIdx.x * XS; s0 < nslots; s0 += gridDim.x * XS)
   {
      if (tid == 0) s_n = 0;
      __syncthreads();
      const uint32_t sl = s0 + tid;
      if (tid < XS && sl < nslots && nexc[sl]) s_list[atomicAdd(&s_n, 1u)] = sl;
      __syncthreads();
      const uint32_t nl = s_n;
      for (uint32_t q = 0; q < nl; q++)
      {
         const uint32_t slot = s_list[q];
         const uint32_t c = cnt[slot], x = nexc[slot];
         const uint64_t b = base[slot];
         if (x > (uint32_t) XM || x > c)
         {
            if (tid == 0) atomicOr(errflag + 2, 2u);
            continue;
         }
         const uint32_t m = c - x;   // FIFO part [0, m), exception k at c - 1 - k
         uint32_t P = 1;
         while (P < x) P <<= 1;
         for (uint32_t k = tid; k < P; k += XT)
         {
            if (k < x)
            {
               const Rec r = recs[b + c - 1 - k];
               et[k] = r.t;
               eid[k] = r.id;
               eax[k] = r.aux;
            }
            else
            {
               et[k] = ~0ull;
               eid[k] = ~0u;
            }
         }
         __syncthreads();
         // bitonic sort of the exceptions by (t, id)
         for (uint32_t kk = 2; kk <= P; kk <<= 1)
            for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1)
            {
               for (uint32_t i = tid; i < P; i += XT)
               {
                  const uint32_t l = i ^ jj;
                  if (l > i)
                  {
                     const bool up = (i & kk) == 0;
                     const bool gt = key_lt(et[l], eid[l], et[i], eid[i]);
                     if (gt == up)
                     {
                        const uint64_t t0 = et[i];
                        et[i] = et[l];
                        et[l] = t0;
                        const uint32_t i0 = eid[i];
                        eid[i] = eid[l];
                        eid[l] = i0;
                        const uint32_t a0 = eax[i];
                        eax[i] = eax[l];
                        eax[l] = a0;
                     }
                  }
               }
               __syncthreads();
            }
         // each exception's merged position: its rank + the FIFO records before it
         for (uint32_t k = tid; k < x; k += XT)
         {
            uint32_t lo = 0, hi = m;
            while (lo < hi)
            {
               const uint32_t mid = (lo + hi) >> 1;
               const Rec r = recs[b + mid];
               if (key_lt(r.t, r.id, et[k], eid[k])) lo = mid + 1;
               else hi = mid;
            }
            edst[k] = k + lo;
         }
         __syncthreads();
         // FIFO records from the first exception's position up move by the exceptions
         // before them: top chunk first (XU records per thread, their loads in flight
         // together), each chunk read completely before it is written
         const uint32_t i0 = x ? edst[0] : m;
         constexpr uint32_t CH = XU * XT;
         for (uint32_t top = m; top > i0;)
         {
            const uint32_t a0 = top > i0 + CH ? top - CH : i0;
            Rec r[XU];
            uint32_t d[XU];
#pragma unroll
            for (uint32_t u = 0; u < XU; u++)
            {
               const uint32_t i = a0 + u * XT + tid;
               if (i < top) r[u] = recs[b + i];
            }
#pragma unroll
            for (uint32_t u = 0; u < XU; u++)
            {
               const uint32_t i = a0 + u * XT + tid;
               uint32_t lo = 0, hi = x;
               if (i < top)
                  while (lo < hi)
                  {
                     const uint32_t mid = (lo + hi) >> 1;
                     if (key_lt(et[mid], eid[mid], r[u].t, r[u].id)) lo = mid + 1;
                     else hi = mid;
                  }
               d[u] = i + lo;
            }
            __syncthreads();
#pragma unroll
            for (uint32_t u = 0; u < XU; u++)
            {
               const uint32_t i = a0 + u * XT + tid;
               if (i < top)
               {
                  const uint64_t g = b + d[u];
                  recs[g] = r[u];
                  if ((g & 63) == 0)
                  {
                     samp_t[g >> 6] = r[u].t;
                     samp_id[g >> 6] = r[u].id;
                  }
               }
            }
            __syncthreads();
            top = a0;
         }
         for (uint32_t k = tid; k < x; k += XT)
         {
            const uint64_t g = b + edst[k];
            Rec r;
            r.t = et[k];
            r.id = eid[k];
            r.aux = eax[k];
            recs[g] = r;
            if ((g & 63) == 0)
            {
               samp_t[g >> 6] = r.t;
               samp_id[g >> 6] = r.id;
            }
         }
         if (tid == 0) nexc[slot] = 0;
         __syncthreads();
      }
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
      p.obase[f] = used ? (uint32_t) slot_base[os] : 0u;
      p.ocap[f] = used ? slot_cnt[os] : 0u;
      p.oslot[f] = os;
   }
   const uint32_t sides[3] = { IN_LOCAL, IN_W, IN_E };
   for (uint32_t j = 0; j < 3; j++)
   {
      const uint32_t s = slot_of(tile, dir, sides[j]);
      p.ibase[j] = j < nl ? (uint32_t) slot_base[s] : 0u;
      p.icnt[j] = j < nl ? slot_cnt[s] : 0u;
   }
   p.port = tile * PORTS + dir;
   p.tile = tile;
   p.dir = dir;
   p.cont = dir;
   p.nx = ntile % W;
   p.ny = ntile / W;
   p.rl = (uint32_t) rl_of(c, tile);
   p.nl = nl;
   for (int q = 0; q < 6; q++) p.pad0[q] = 0;
   out[k] = p;
}

// One workgroup per (chain port, insert list j0 + j, j < nlrun): bt[w] = first record
// of the slot with t at or after window w's start (w < nW), bt[nW] = record count.  The
// window of t: win_of over the chain's boundaries (the last one is unbounded), so
// bt[w] (0 < w < nW) is the first record whose key t >> qs reaches B[w].  Slots of up
// to WB_SMAX samples search: the slot's 1-in-64 key samples (written by its producer)
// in LDS, one thread per boundary, then the 63 records after the sample in HBM; the
// slot's records themselves are not streamed.  Larger slots scan every record.
constexpr uint32_t WB_SMAX = 4096;
__device__ __forceinline__ uint32_t key_of(uint64_t t, uint32_t qs)
{
   const uint64_t tq64 = t >> qs;
   return tq64 < 0xFFFFFFFEull ? (uint32_t) tq64 : 0xFFFFFFFEu;   // (as win_of)
}
__global__ __launch_bounds__(256) void k_win_bounds(const ChainPort* __restrict__ cp, uint32_t nl, uint32_t len,
                                                    const ChainWin* __restrict__ cw, const Rec* __restrict__ recs,
                                                    const uint64_t* __restrict__ samp_t, uint32_t* __restrict__ bt,
                                                    uint32_t nlrun, uint32_t j0, const unsigned* __restrict__ cond,
                                                    const uint32_t* __restrict__ wt, uint32_t qs)
{
   if (cond && *cond == 0) return;   // k_inj_stream wrote these bounds (it did not decline)
   __shared__ uint32_t sB[IJ_NWB];
   __shared__ uint32_t sS[WB_SMAX];
   const uint32_t k = blockIdx.x / nlrun, j = j0 + blockIdx.x % nlrun, c = k / len, i = k % len;
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
   const uint32_t* B = wt + cw[c].wt_off;
   const uint32_t ns = (n + 63) / 64;
   if (ns <= WB_SMAX)
   {
      // (slot bases are 64-record aligned: sample s is record 64 s of the slot)
      const uint64_t* sp = samp_t + (base >> 6);
      for (uint32_t s = threadIdx.x; s < ns; s += blockDim.x) sS[s] = key_of(sp[s], qs);
      __syncthreads();
      const Rec* r = recs + base;
      for (uint32_t v = threadIdx.x; v <= nW; v += blockDim.x)
      {
         uint32_t res = n;
         if (v == 0) res = 0;
         else if (v < nW)
         {
            const uint32_t key = B[v];
            uint32_t lo = 0, hi = ns;   // first sample at or past key
            while (lo < hi)
            {
               const uint32_t m = (lo + hi) >> 1;
               if (sS[m] < key) lo = m + 1;
               else hi = m;
            }
            if (lo == 0) res = 0;
            else
            {
               uint32_t a = 64 * (lo - 1) + 1, e = min(64 * lo, n);   // record 64 (lo - 1) is below key
               while (a < e)
               {
                  const uint32_t m = (a + e) >> 1;
                  if (key_of(r[m].t, qs) < key) a = m + 1;
                  else e = m;
               }
               res = a;
            }
         }
         b[v] = res;
      }
      return;
   }
   // the chain's window boundaries in LDS (at most IJ_NWB - 1 windows: engine.hip keeps
   // chains within it), the window of a record by a binary search; the previous record's
   // window comes from the neighbouring lane
   const bool inl = nW + 1 <= IJ_NWB;
   if (inl)
      for (uint32_t v = threadIdx.x; v <= nW; v += blockDim.x) sB[v] = B[v];
   __syncthreads();
   const uint32_t* Bs = inl ? sB : B;
   auto win = [&](uint64_t t) -> uint64_t { return win_of(Bs, nW, t, qs); };
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

// ---------------------------------------------------------------------------
// The injection level streamed: one workgroup per source tile walks its injection
// slot in blocks of 1,024 records (4 consecutive per thread), the queue's tail X
// carried from block to block -- no chunk plan, no look-back.  A block: each
// thread composes its records' max-plus aggregate, a wave scan and the four waves'
// aggregates (in order, from X) give every record the tail ahead of it; route
// counts per output field (LEFT, RIGHT, DOWN, UP of the same tile) give FIFO
// positions.  Relative cycles (to the block's first cycle) keep the scan in 32
// bits.  The no-gap M/G/1 prefix (queue_model_history_tree.cc:58-64) is not served
// here: a port whose first arrival is at cycle 0 is checked until its first idle
// cycle, and where the branch would fire the kernel declines (errflag[7]; it also
// flags the X chains, so the rest of the run returns at once): the host reruns the
// batch with k_level's injection level.  Unicast batches of the chain path only.
// ---------------------------------------------------------------------------
#ifndef IJ_PER_V
#define IJ_PER_V 4
#endif
#ifndef IJ_PF
#define IJ_PF 1
#endif
constexpr uint32_t IJ_T = 256, IJ_PER = IJ_PER_V, IJ_BLK = IJ_T * IJ_PER;
//
// With cwx (single-mesh chain runs) it also writes k_win_bounds' bounds of the four
// chain ports' IN_LOCAL lists it fills (X ports: list 0 of bt; Y ports: list 0 of
// 3): bt[w] = first record of the slot with t >= w D, bt[nW] = count.  The output
// slots are FIFO-served in order, so their times do not decrease: every record
// lowers its window's entry (LDS atomicMin), then a suffix min fills the empty
// windows.  Those k_win_bounds launches run only when this kernel declined.
template <bool F1>
__global__ __launch_bounds__(IJ_T) void k_inj_stream(DevCfg c, const uint32_t* __restrict__ slot_cnt,
                                                     const uint64_t* __restrict__ slot_base, Rec* __restrict__ recs,
                                                     uint64_t* __restrict__ samp_t, uint32_t* __restrict__ samp_id,
                                                     unsigned long long* __restrict__ port_sum,
                                                     unsigned long long* __restrict__ port_cnt,
                                                     unsigned long long* __restrict__ port_flit,
                                                     unsigned long long* __restrict__ port_last, unsigned* __restrict__ errflag,
                                                     const ChainWin* __restrict__ cwx, uint32_t* __restrict__ btx,
                                                     const ChainWin* __restrict__ cwy, uint32_t* __restrict__ bty,
                                                     uint32_t stop, const uint32_t* __restrict__ wtx,
                                                     const uint32_t* __restrict__ wty, uint32_t qs)
{
   // stop (the chain path, nothing queued behind): a decline also flags the X chains
   // (errflag[4]) so that every later kernel of the run returns at once
   const unsigned dfl = stop ? F_FALLBACK : 0u;
   __shared__ uint32_t wA[4], wB[4], wc01[4], wc23[4];
   __shared__ uint32_t s_xin[4], s_fb[4][4], s_run[4], s_ev[2], s_decl;
   __shared__ uint64_t s_X;
   __shared__ unsigned long long s_sum[4], s_flit[4];
   __shared__ uint32_t s_bt[4][IJ_NWB], s_nW[4];
   __shared__ uint32_t s_B[4][IJ_NWB];   // the field's chain window boundaries
   __shared__ uint32_t* s_bp[4];
   __shared__ const uint32_t* s_bx[4];
   const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
   const uint32_t tile = blockIdx.x;
   const uint32_t sl = slot_of(tile, P_INJ, IN_LOCAL);
   const uint32_t n = slot_cnt[sl];
   const bool bnd = cwx != nullptr;
   if (n == 0 && !bnd) return;
   const uint64_t base = slot_base[sl];
   uint32_t x, y;
   tile_xy(tile, c.W, c.magicW, x, y);
   uint32_t ob[4], oc[4];
#pragma unroll
   for (uint32_t q = 0; q < 4; q++)
   {
      const uint32_t d = P_LEFT + q;   // LEFT, RIGHT, DOWN, UP
      const uint32_t os = slot_of(tile, d, slot_side(d, IN_LOCAL));
      ob[q] = (uint32_t) slot_base[os];
      oc[q] = slot_cnt[os];
   }
   const double f = c.f;
   if (tid < 4) s_run[tid] = 0;
   if (tid == 0)
   {
      s_X = 0;
      s_decl = 0;
   }
   if (bnd)
   {
      if (tid < 4)
      {
         // the chain port (k_chain_plan's numbering, rows / columns from 0) of field tid
         const uint32_t d = P_LEFT + tid;
         const bool xd = d == P_LEFT || d == P_RIGHT;
         const bool ex = d == P_RIGHT ? x + 1 < c.W : d == P_LEFT ? x >= 1 : d == P_UP ? y + 1 < c.H : y >= 1;
         const uint32_t ch = xd ? 2 * y + (d == P_LEFT) : 2 * x + (d == P_DOWN);
         const uint32_t i = d == P_RIGHT ? x : d == P_LEFT ? c.W - 1 - x : d == P_UP ? y : c.H - 1 - y;
         const ChainWin* cw = xd ? cwx : cwy;
         uint32_t nW = 0;
         if (ex && cw)
         {
            nW = cw[ch].nW;
            s_bp[tid] = (xd ? btx : bty) + cw[ch].bt_off + (uint64_t) i * (xd ? 1u : 3u) * (nW + 1);
         }
         s_nW[tid] = nW;
         s_bx[tid] = ex && cw ? (xd ? wtx : wty) + cw[ch].wt_off : nullptr;
      }
      __syncthreads();
      for (uint32_t q = 0; q < 4; q++)
      {
         for (uint32_t v = tid; v < s_nW[q]; v += IJ_T) s_bt[q][v] = 0xFFFFFFFFu;
         if (s_nW[q])   // (a field without a chain port -- the mesh edge -- has no boundaries)
            for (uint32_t v = tid; v <= s_nW[q]; v += IJ_T) s_B[q][v] = s_bx[q][v];
      }
   }
   // the port starts with no gap in its history tree only if its first request is at cycle 0
   bool nogap = n && c.analytical && cyc_of<F1>(recs[base].t, f) == 0;
   uint64_t ssum = 0, flits = 0;
   __syncthreads();
   // the next block's records are loaded while this one is placed (IJ_PF)
   Rec rn[IJ_PER];
   if (IJ_PF)
   {
#pragma unroll
      for (uint32_t k = 0; k < IJ_PER; k++)
      {
         const uint32_t j = tid * IJ_PER + k;
         if (j < n) rn[k] = recs[base + j];
      }
   }
   for (uint32_t b0 = 0; b0 < n; b0 += IJ_BLK)
   {
      const uint64_t bc = cyc_of<F1>(recs[base + b0].t, f);   // the block's first cycle (the slot is sorted)
      Rec r[IJ_PER];
      uint32_t tr[IJ_PER], pr[IJ_PER], fr[IJ_PER];
      bool vr[IJ_PER];
#pragma unroll
      for (uint32_t k = 0; k < IJ_PER; k++)
      {
         const uint32_t j = b0 + tid * IJ_PER + k;
         vr[k] = j < n;
         if (IJ_PF) r[k] = rn[k];
         else if (vr[k]) r[k] = recs[base + j];
      }
      if (IJ_PF)
      {
#pragma unroll
         for (uint32_t k = 0; k < IJ_PER; k++)
         {
            const uint32_t j = b0 + IJ_BLK + tid * IJ_PER + k;
            if (j < n) rn[k] = recs[base + j];
         }
      }
      uint32_t A = 0, B = 0, c01 = 0, c23 = 0;
      bool wide = false;
#pragma unroll
      for (uint32_t k = 0; k < IJ_PER; k++)
      {
         tr[k] = pr[k] = fr[k] = 0;
         if (!vr[k]) continue;
         const uint64_t tc = cyc_of<F1>(r[k].t, f) - bc;
         wide |= tc >= (1ull << 30);
         tr[k] = (uint32_t) tc;
         pr[k] = aux_F(r[k].aux);
         const uint32_t d = xy_dir(x, y, aux_dx(r[k].aux), aux_dy(r[k].aux)) - P_LEFT;   // 0..3 (never SELF)
         fr[k] = d;
         const uint32_t nb = B + pr[k], nt = tr[k] + pr[k];
         B = nb > nt ? nb : nt;
         A += pr[k];
         if (d < 2) c01 += 1u << (16 * d);
         else c23 += 1u << (16 * (d - 2));
      }
      // the waves' inclusive prefixes; lane 63 holds each wave's aggregate
      uint32_t iA = A, iB = B;
      wave_scan(iA, iB);
      const uint32_t i01 = wave_sum32(c01), i23 = wave_sum32(c23);
      if (lane == 63)
      {
         wA[wv] = iA;
         wB[wv] = iB;
         wc01[wv] = i01;
         wc23[wv] = i23;
      }
      if (wide) s_decl = 1;
      __syncthreads();
      if (tid == 0)
      {
         // the block's first request finds the queue idle when the tail lies before its
         // cycle (a gap, queue_model_history_tree.cc:79-86): the relative tail below is
         // clamped to 0 there, so the per-record check (tc > Xt) cannot see it
         const bool gap0 = s_X < bc;
         uint64_t Xr = s_X > bc ? s_X - bc : 0;   // an earlier tail behaves like the block's first cycle
         if (Xr >= (1ull << 30)) s_decl = 1;
         for (uint32_t q = 0; q < 4; q++)
         {
            s_xin[q] = (uint32_t) Xr;
            const uint64_t xa = Xr + wA[q];
            Xr = xa > wB[q] ? xa : wB[q];
            for (uint32_t d = 0; d < 4; d++)
            {
               s_fb[q][d] = s_run[d];
               s_run[d] += d < 2 ? (wc01[q] >> (16 * d)) & 0xFFFFu : (wc23[q] >> (16 * (d - 2))) & 0xFFFFu;
            }
         }
         s_X = bc + Xr;
         s_ev[0] = gap0 ? 0u : 0xFFFFFFFFu;
         s_ev[1] = 0xFFFFFFFFu;
      }
      __syncthreads();
      if (s_decl)
      {
         if (tid == 0)
         {
            atomicOr(errflag + 7, 1u);
            if (dfl) atomicOr(errflag + 4, dfl);
         }
         return;
      }
      // the tail ahead of this thread: its wave's entry composed with the lanes before it
      const uint32_t exA = dpp32<0x138, 0xF, 0xF>(iA), exB = dpp32<0x138, 0xF, 0xF>(iB);   // wave_shr 1
      const uint32_t xa = s_xin[wv] + exA;
      uint32_t Xt = xa > exB ? xa : exB;
      const uint32_t x01 = i01 - c01, x23 = i23 - c23;   // the wave's field counts ahead of this thread
      uint32_t kr[4] = { 0, 0, 0, 0 };
#pragma unroll
      for (uint32_t k = 0; k < IJ_PER; k++)
      {
         if (!vr[k]) continue;
         const uint32_t tc = tr[k], p = pr[k], d = fr[k];
         if (nogap)
         {
            const uint32_t at = tid * IJ_PER + k;
            if (tc > Xt) atomicMin(&s_ev[0], at);            // the first idle cycle
            else if (Xt > tc + p) atomicMin(&s_ev[1], at);   // the M/G/1 branch would serve it
         }
         const uint32_t cc = Xt > tc ? Xt - tc : 0u;
         Xt = (Xt > tc ? Xt : tc) + p;
         ssum += cc;
         flits += p;
         uint32_t kk = 0, ahead = 0;
#pragma unroll
         for (uint32_t q = 0; q < 4; q++)
            if (q == d)
            {
               kk = kr[q]++;
               ahead = q < 2 ? (x01 >> (16 * q)) & 0xFFFFu : (x23 >> (16 * (q - 2))) & 0xFFFFu;
            }
         uint32_t obd = 0, ocd = 0;
#pragma unroll
         for (uint32_t q = 0; q < 4; q++)
            if (q == d)
            {
               obd = ob[q];
               ocd = oc[q];
            }
         const uint32_t pos = s_fb[wv][d] + ahead + kk;
         if (pos >= ocd)
         {
            atomicOr(errflag, 1u);   // route-count invariant broken: never write outside the slot
            continue;
         }
         const uint64_t gp = (uint64_t) obd + pos;
         Rec o;
         o.t = r[k].t + ps_of<F1>(cc, f);
         o.id = r[k].id;
         o.aux = r[k].aux;
         recs[gp] = o;
         if ((gp & 63) == 0)
         {
            samp_t[gp >> 6] = o.t;
            samp_id[gp >> 6] = o.id;
         }
         if (bnd && s_nW[d])
         {
            // window of the record among the chain's boundaries (as k_win_bounds)
            const uint32_t wl = s_nW[d] - 1;
            const uint64_t w = win_of(s_B[d], s_nW[d], o.t, qs);
            atomicMin(&s_bt[d][w < wl ? w : wl], pos);
         }
      }
      __syncthreads();
      if (nogap)
      {
         // the no-gap prefix: an M/G/1 request before the first idle cycle -> decline;
         // an idle cycle ends the prefix for good (queue_model_history_tree.cc:79-86)
         if (s_ev[1] != 0xFFFFFFFFu && s_ev[1] < s_ev[0])
         {
            if (tid == 0)
            {
               atomicOr(errflag + 7, 2u);
               if (dfl) atomicOr(errflag + 4, dfl);
            }
            return;
         }
         nogap = s_ev[0] == 0xFFFFFFFFu;
      }
   }
   if (bnd)
   {
      // wave q: field q's bounds, a suffix min from the last window down (64 windows a step)
      __syncthreads();
      const uint32_t nW = s_nW[wv];
      if (nW)
      {
         uint32_t* bp = s_bp[wv];
         uint32_t carry = oc[wv];
         if (lane == 0) bp[nW] = carry;
         for (int top = (int) nW - 1; top >= 0; top -= 64)
         {
            const int idx = top - (int) lane;
            uint32_t v = idx >= 0 ? s_bt[wv][idx] : 0xFFFFFFFFu;
            for (int off = 1; off < 64; off <<= 1)
            {
               const uint32_t u = (uint32_t) __shfl_up((int) v, off);
               if ((int) lane >= off) v = v < u ? v : u;
            }
            v = v < carry ? v : carry;
            if (idx >= 0) bp[idx] = v;
            carry = (uint32_t) __shfl((int) v, 63);
         }
      }
      if (n == 0) return;
   }
   // the port's counters (router_model.cc:136-144): contention cycles, requests, flits, last departure
   uint64_t a0 = ssum, a1 = flits;
   for (int off = 32; off > 0; off >>= 1)
   {
      a0 += __shfl_down(a0, off);
      a1 += __shfl_down(a1, off);
   }
   if (lane == 0)
   {
      s_sum[wv] = a0;
      s_flit[wv] = a1;
   }
   __syncthreads();
   if (tid == 0)
   {
      const uint32_t port = tile * PORTS + P_INJ;
      atomicAdd(&port_sum[port], s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3]);
      atomicAdd(&port_cnt[port], (unsigned long long) n);
      atomicAdd(&port_flit[port], s_flit[0] + s_flit[1] + s_flit[2] + s_flit[3]);
      atomicMax(&port_last[port], (unsigned long long) s_X);
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

// The SELF slots' exception counts (the MG instantiation's Y chains may leave tails
// there); every other slot keeps its count, k_exc_merge's refused slots included.
__global__ __launch_bounds__(256) void k_zero_self_nexc(uint32_t ntiles, uint32_t* __restrict__ nexc)
{
   const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
   if (i < ntiles * INS) nexc[slot_of(i / INS, P_SELF, i % INS)] = 0;
}

}  // namespace ch
}  // namespace gnoc
