// level.hip -- v3 engine: one persistent launch per dependency level of the
// output-port DAG, workgroups pulling time-chunks of port arrival streams.
//
// With XY routing (network_model_emesh_hop_by_hop.cc:229-240) the output ports
// form a DAG: injection -> X chain of the source row -> Y chain of the
// destination column -> SELF.  With arrivals served in (time, id) order every
// history-tree queue (queue_model_history_tree.cc:43-126) is the FIFO max-plus
// recurrence
//     c_i = max(X - t_i, 0),  X <- max(t_i, X) + F_i
// plus a serial history-tree/M-G-1 prologue while the queue has never idled
// (queue_model_history_tree.cc:58-64, queue_model_m_g_1.cc:17-56).  A level is
// a set of ports whose inputs are complete; each port's arrival stream is the
// (t, id)-merge of its <= 4 input slots, cut into chunks by (t, id) key range.
//
// One workgroup per chunk:
//   1. key range: an exact index split of the port's largest input; the other
//      inputs are searched with a 64-ary wave search over 1-in-64 key samples
//   2. load the ranges (16-B records) into LDS as SoA keys; merge by galloping
//      co-iteration (rank = own index + lower bounds in the other inputs)
//   3. each thread pulls its contiguous merged segment (<= 8 records) into
//      registers; block max-plus scan: element map X -> max(X + F, t + F),
//      composition (a1,b1).(a2,b2) = (a1 + a2, max(b1 + a2, b2)), plus per
//      next-direction record counts (output positions)
//   4. decoupled look-back over the port's earlier chunks in ONE round trip:
//      every state word is an 8-byte self-validating granule (zeroed per run)
//   5. recurrence and stores straight from registers
// Only max_list_size >= 3 takes this path (engine.hip).  engine.hip includes
// this file twice: LV_GEN 0 is the f = 1 GHz kernel (integer ps <-> cycle
// conversions), LV_GEN 1 (namespace lvg) the kernel for any other frequency
// (Time::toCycles / Latency::toPicosec in double, time_types.h:81-109).  Two
// copies rather than a template flag: the flag alone changed the inlining of the
// f = 1 GHz kernel and cost it 3% on 32x32.
#ifndef LV_GEN
#define LV_GEN 0
#endif
#include "common.h"

namespace gnoc {
#if !LV_GEN

constexpr int LV_T = 256;                // threads per workgroup
#ifndef LV_CAP_V
#define LV_CAP_V 1888
#endif
constexpr int LV_CAP = LV_CAP_V;         // records one leaf holds in LDS
constexpr int LV_PER = (LV_CAP + LV_T - 1) / LV_T;   // records per thread (load phase)
constexpr int LV_IN = 4;                 // input slots per port (SELF, UP, DOWN have 4)
constexpr int LV_SEG = LV_IN + 1;        // + the exception segment
constexpr int LV_MAXLEAF = 32;           // leaves per chunk (bursts); beyond -> errflag, v1 rerun
#ifndef LV_CTGT_V
#define LV_CTGT_V 1700   // configs[1] INJ + SELF levels: 1600 -> 0.412 ms, 1700 -> 0.387 (sweep unchanged)
#endif
constexpr uint32_t LV_CTGT = LV_CTGT_V;  // target records per chunk (the chain path's INJ + SELF levels)
#ifndef LV_CTGT_FULL_V
#define LV_CTGT_FULL_V 1600   // every level on k_level (broadcast passes, declined batches, sweeps): configs[1] 1300 / 1500 / 1600 / 1700 -> 6.14 / 5.93 / 5.85 / 7.05 ms
#endif
constexpr uint32_t LV_CTGT_FULL = LV_CTGT_FULL_V;
constexpr uint64_t LV_SPIN_CYCLES = 1ull << 31;   // give up a wait after ~1 s (errflag -> exact v1 rerun)
constexpr uint64_t LV_TAG = 1ull << 63;
#ifndef LV_QUEUES_V
#define LV_QUEUES_V 1
#endif
#ifndef LV_LATE_ROUNDS
#define LV_LATE_ROUNDS 4   // levels with more chunks than this many rounds of the grid fetch the next chunk late
#endif
#ifndef LV_PORT_QUEUES
#define LV_PORT_QUEUES 1   // 1: port-aligned queue ranges (+ stealing); 0: chunk-interleaved queues
#endif
constexpr uint32_t LV_QUEUES = LV_QUEUES_V;   // chunk dequeue heads per level (power of two)
constexpr uint32_t LV_QB = LV_QUEUES + 2;     // per-level plan words: queue bases, then the late-fetch flag
constexpr int LV_STATE_WORDS = 16;       // u64 per chunk state

// Per-port descriptor, built on device by k_plan_ports from the slot layout.
struct __attribute__((aligned(16))) PortIO3
{
   uint64_t base[LV_IN];     // input slot bases (records)
   uint64_t obase[5];        // output slot base per next direction
   uint32_t slot[LV_IN];     // input slot ids
   uint32_t cnt[LV_IN];      // input slot record counts (main + exceptions)
   uint32_t ocnt[5];         // output slot capacities
   uint32_t oslot[5];        // output slot ids
   uint32_t port, dir, nin, sb;
   uint32_t nx, ny, gbase, nc;
   uint32_t prod[LV_IN];     // plan index of each input's producer port (LV_NO_PROD: the trace)
   uint32_t prod_nc[LV_IN];  // that producer's chunk count: complete when done[prod] == prod_nc
   uint32_t pk, rl, pad1, pad2;    // plan index of the port itself; R + Lk of its tile (ps)
};
static_assert(sizeof(PortIO3) % 16 == 0, "PortIO3 copy granularity");
constexpr uint32_t LV_NO_PROD = 0xFFFFFFFFu;
#endif

#if LV_GEN
namespace lvg {   // (argument-dependent lookup must not see the other copy: each lives in a namespace of its own)
#define LV_CYC(ps) cyc_of<false>((ps), sm.fq)
#define LV_PS(cy) ps_of<false>((cy), sm.fq)
#else
namespace lvx {
#define LV_CYC(ps) cyc1(ps)
#define LV_PS(cy) ((cy) * 1000ull)
#endif

// Carried queue state (exclusive prefix of a chunk / leaf).
struct Carry3
{
   uint64_t X;
   uint32_t mode, g;
   double s1, s2;
   uint64_t narr, newest;
   uint32_t cnt[5];
};

struct LvSmem
{
   uint64_t kt[LV_CAP];      // arrival time (ps)
   uint32_t ki[LV_CAP];      // packet id
   uint32_t ka[LV_CAP];      // aux: dx | dy << 10 | F << 20
   uint16_t perm[LV_CAP];    // merged position -> record slot
   uint16_t tmp[LV_CAP];     // intermediate merge lists
   PortIO3 io;
   Carry3 cy;
   uint64_t wA[LV_T / 64], wB[LV_T / 64], wC[LV_T / 64];
   uint64_t st_sum;
   uint64_t st_flit, st_last;   // sum of F, latest departure (QueueModel utilization, queue_model.cc:49-53)
   uint64_t lk_t[LV_MAXLEAF + 1];
   uint32_t lk_i[LV_MAXLEAF + 1];
   uint32_t lr_lo[LV_MAXLEAF][LV_IN];
   uint32_t nmain[LV_IN], nxe[LV_IN];
   uint32_t lo[LV_IN], hi[LV_IN];
   uint32_t off[LV_SEG], len[LV_SEG];
   uint32_t search[2 * LV_IN];
   uint32_t g, j, E, s0;
   uint32_t nexc_leaf, published, nleaf, st_cnt;
   uint32_t st_mg1, pad0, pad1, pad2;
   uint64_t tm[4];           // debug phase stamps inside a leaf (GNOC_STAMPS)
#if LV_GEN
   double fq;                // network frequency (GHz)
#endif
   // current chunk's key range
   uint64_t klo_t, khi_t;
   uint32_t klo_i, khi_i, has_lo, has_hi, empty, nc;
   uint32_t pk, pad3, pad4, pad5;
   // next chunk, prefetched by waves 1-3 while wave 0 looks back
   struct
   {
      PortIO3 io;
      uint64_t klo_t, khi_t;
      uint32_t klo_i, khi_i;
      uint32_t g, valid, has_lo, has_hi, empty, ready;
      uint32_t pk, deferred, ilo, ihi;
      uint32_t nmain[LV_IN], nxe[LV_IN];
      uint32_t search[2 * LV_IN];
   } nx;
   // this level's dequeue heads: queue q owns chunks [qb[q], qb[q+1]) (level-relative,
   // port-aligned, so a chunk's look-back predecessor is always in its own queue)
   uint32_t qb[LV_QB];        // [LV_QUEUES + 1]: fetch the next chunk after the look-back (long ports)
   uint32_t qdone;            // bit q: queue q handed out its last chunk
};

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
// Workgroup barrier for LDS only.  __syncthreads() is a workgroup fence and
// drains every outstanding global store first (s_waitcnt vmcnt(0)); no thread
// of a chunk reads global data another thread of it wrote, so the chunk
// kernel's barriers only need the LDS counter.
__device__ __forceinline__ void lv_bar()
{
   asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ uint64_t lv_ld(const uint64_t* p)
{
   return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lv_st(uint64_t* p, uint64_t v)
{
   __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Hop-record stores are plain stores: a wave's 16-B records for one next port
// land on nearby lines and combine in L2 before they reach HBM (write-through
// sc1 stores measured 37% slower on 32x32, nontemporal stores 2x slower).
__device__ __forceinline__ void lv_store_rec(Rec* p, uint64_t t, uint32_t id, uint32_t aux)
{
   Rec o;
   o.t = t;
   o.id = id;
   o.aux = aux;
   *p = o;
}

// A record at slot position gp, plus its key sample when gp is a multiple of 64.
__device__ __forceinline__ void lv_put(Rec* __restrict__ recs, uint64_t* __restrict__ samp_t,
                                       uint32_t* __restrict__ samp_id, uint64_t gp, uint64_t tn, uint32_t id, uint32_t ax)
{
   lv_store_rec(recs + gp, tn, id, ax);
   if ((gp & 63) == 0)
   {
      samp_t[gp >> 6] = tn;
      samp_id[gp >> 6] = id;
   }
}

__device__ __forceinline__ bool rlt(const Rec& a, uint64_t t, uint32_t id)
{
   return a.t < t || (a.t == t && a.id < id);
}
__device__ __forceinline__ bool klt(const LvSmem& sm, uint32_t k, uint64_t t, uint32_t id)
{
   const uint64_t kt = sm.kt[k];
   return kt < t || (kt == t && sm.ki[k] < id);
}

__device__ __forceinline__ uint64_t cyc1(uint64_t ps) { return (ps + 999ull) / 1000ull; }

__device__ __forceinline__ void mp_comp(uint64_t& A, uint64_t& B, uint64_t a2, uint64_t b2)
{
   const uint64_t nb = B + a2;
   B = nb > b2 ? nb : b2;
   A += a2;
}

// next direction after leaving through `dir` into tile (nx, ny) (SELF: none)
__device__ __forceinline__ uint32_t next_dir(uint32_t ax, uint32_t dir, uint32_t nx, uint32_t ny)
{
   return dir == P_SELF ? 0u : xy_dir(nx, ny, aux_dx(ax), aux_dy(ax));
}

__device__ __forceinline__ uint32_t cfield(uint64_t c, uint32_t d) { return (uint32_t) ((c >> (12 * d)) & 0xFFFu); }

// lower bound of (t,id) in LDS keys [lo, hi)
__device__ __forceinline__ uint32_t lds_lb(const LvSmem& sm, uint32_t lo, uint32_t hi, uint64_t t, uint32_t id)
{
   while (lo < hi)
   {
      const uint32_t mid = (lo + hi) >> 1;
      if (klt(sm, mid, t, id)) lo = mid + 1;
      else hi = mid;
   }
   return lo;
}

// lower bound of (t,id) in [lo, end), knowing every key before lo is smaller
__device__ __forceinline__ uint32_t lds_gallop(const LvSmem& sm, uint32_t lo, uint32_t end, uint64_t t, uint32_t id)
{
   uint32_t step = 1, hi;
   for (;;)
   {
      const uint32_t pr = lo + step - 1;
      if (pr >= end) { hi = end; break; }
      if (!klt(sm, pr, t, id)) { hi = pr; break; }
      lo = pr + 1;
      step <<= 1;
   }
   return lds_lb(sm, lo, hi, t, id);
}

// 64-ary lower_bound of key (kt,ki) in the sorted main part [0,n) of a slot,
// using its 1-in-64 key samples.  Whole wave calls; result uniform.
__device__ uint32_t wave_lb(const Rec* __restrict__ r, const uint64_t* __restrict__ sp_t,
                            const uint32_t* __restrict__ sp_i, uint32_t n, uint64_t kt, uint32_t ki, uint32_t lane)
{
   if (n == 0) return 0;
   uint32_t lo = 0, hi = (n + 63) / 64;
   while (lo < hi)
   {
      const uint32_t step = (hi - lo + 63) / 64;
      const uint32_t i = lo + lane * step;
      bool t = false;
      if (i < hi) t = sp_t[i] < kt || (sp_t[i] == kt && sp_i[i] < ki);
      const uint32_t c = (uint32_t) __popcll(__ballot(t));
      if (c == 0) hi = lo;
      else
      {
         const uint32_t nh = min(lo + c * step, hi);
         lo = lo + (c - 1) * step + 1;
         hi = nh;
      }
   }
   if (lo == 0) return 0;
   const uint32_t base = (lo - 1) * 64;
   const uint32_t k = base + lane;
   bool t = false;
   if (k < n) t = rlt(r[k], kt, ki);
   return base + (uint32_t) __popcll(__ballot(t));
}

// wave_lb with the key itself read from memory (a sample of the split input):
// the key load and the first level of sample reads are independent, so they
// share one round trip.
__device__ uint32_t wave_lb2(const Rec* __restrict__ r, const uint64_t* __restrict__ sp_t,
                             const uint32_t* __restrict__ sp_i, uint32_t n, const uint64_t* __restrict__ key_t,
                             const uint32_t* __restrict__ key_i, uint32_t lane)
{
   if (n == 0) return 0;
   uint32_t lo = 0, hi = (n + 63) / 64;
   const uint32_t step0 = (hi + 63) / 64;
   const uint32_t i0 = lane * step0;
   uint64_t s0t = 0;
   uint32_t s0i = 0;
   if (i0 < hi) { s0t = sp_t[i0]; s0i = sp_i[i0]; }
   const uint64_t kt = *key_t;
   const uint32_t ki = *key_i;
   {
      const bool t = i0 < hi && (s0t < kt || (s0t == kt && s0i < ki));
      const uint32_t c = (uint32_t) __popcll(__ballot(t));
      if (c == 0) hi = lo;
      else
      {
         const uint32_t nh = min(lo + c * step0, hi);
         lo = lo + (c - 1) * step0 + 1;
         hi = nh;
      }
   }
   while (lo < hi)
   {
      const uint32_t step = (hi - lo + 63) / 64;
      const uint32_t i = lo + lane * step;
      bool t = false;
      if (i < hi) t = sp_t[i] < kt || (sp_t[i] == kt && sp_i[i] < ki);
      const uint32_t c = (uint32_t) __popcll(__ballot(t));
      if (c == 0) hi = lo;
      else
      {
         const uint32_t nh = min(lo + c * step, hi);
         lo = lo + (c - 1) * step + 1;
         hi = nh;
      }
   }
   if (lo == 0) return 0;
   const uint32_t base = (lo - 1) * 64;
   const uint32_t k = base + lane;
   bool t = false;
   if (k < n) t = rlt(r[k], kt, ki);
   return base + (uint32_t) __popcll(__ballot(t));
}

// Exceptions of the port's inputs whose key lies in [klo, khi): exact count
// (block-wide; the exception tails are short).
__device__ uint32_t lv_count_exc(LvSmem& sm, const Rec* __restrict__ recs, uint64_t klo_t, uint32_t klo_i,
                                 uint64_t khi_t, uint32_t khi_i, bool has_lo, bool has_hi)
{
   const uint32_t tid = threadIdx.x;
   lv_bar();
   if (tid == 0) sm.nexc_leaf = 0;
   lv_bar();
   uint32_t mine = 0;
   for (uint32_t s = 0; s < sm.io.nin; s++)
   {
      const Rec* r = recs + sm.io.base[s];
      for (uint32_t i = sm.nmain[s] + tid; i < sm.io.cnt[s]; i += LV_T)
      {
         const Rec v = r[i];
         const bool ge = !has_lo || !rlt(v, klo_t, klo_i);
         const bool lt = !has_hi || rlt(v, khi_t, khi_i);
         mine += (ge && lt) ? 1u : 0u;
      }
   }
   if (mine) atomicAdd(&sm.nexc_leaf, mine);
   lv_bar();
   const uint32_t n = sm.nexc_leaf;
   lv_bar();
   return n;
}

// ---------------------------------------------------------------------------
// merge-path merging of sorted segments in LDS
// A list is a sorted run of record slots: the identity range [off, off+n) of
// the loaded records (idx == nullptr) or idx[off .. off+n).
// ---------------------------------------------------------------------------
struct MList
{
   const uint16_t* idx;
   uint32_t off, n;
};

__device__ __forceinline__ uint32_t ml_at(const MList& l, uint32_t i) { return l.idx ? l.idx[l.off + i] : l.off + i; }

// Output positions [d0, d1) of merge(A, B) -> out[d] (d relative to the job).
// One diagonal binary search, then a sequential merge with the two head keys in
// registers: one dependent LDS read per output.
__device__ void mp_merge_part(const LvSmem& sm, const MList& A, const MList& B, uint16_t* out, uint32_t d0, uint32_t d1)
{
   if (d0 >= d1) return;
   uint32_t lo = d0 > B.n ? d0 - B.n : 0, hi = min(d0, A.n);
   while (lo < hi)
   {
      const uint32_t m = (lo + hi) >> 1;
      const uint32_t sa = ml_at(A, m), sb = ml_at(B, d0 - 1 - m);
      const uint64_t ta = sm.kt[sa], tb = sm.kt[sb];
      if (ta < tb || (ta == tb && sm.ki[sa] < sm.ki[sb])) lo = m + 1;
      else hi = m;
   }
   uint32_t i = lo, j = d0 - lo;
   uint32_t sa = 0, sb = 0;
   uint64_t ta = ~0ull, tb = ~0ull;
   uint32_t ia = ~0u, ib = ~0u;
   if (i < A.n) { sa = ml_at(A, i); ta = sm.kt[sa]; ia = sm.ki[sa]; }
   if (j < B.n) { sb = ml_at(B, j); tb = sm.kt[sb]; ib = sm.ki[sb]; }
   for (uint32_t d = d0; d < d1; d++)
   {
      if (ta < tb || (ta == tb && ia < ib))
      {
         out[d] = (uint16_t) sa;
         if (++i < A.n) { sa = ml_at(A, i); ta = sm.kt[sa]; ia = sm.ki[sa]; }
         else { ta = ~0ull; ia = ~0u; }
      }
      else
      {
         out[d] = (uint16_t) sb;
         if (++j < B.n) { sb = ml_at(B, j); tb = sm.kt[sb]; ib = sm.ki[sb]; }
         else { tb = ~0ull; ib = ~0u; }
      }
   }
}

// One merge round: job 1 = merge(A1, B1) -> out1[0, n1), job 2 (optional) =
// merge(A2, B2) -> out2[0, n2); threads split the n1 + n2 outputs evenly.
__device__ void mp_round(const LvSmem& sm, const MList& A1, const MList& B1, uint16_t* out1, const MList& A2,
                         const MList& B2, uint16_t* out2)
{
   const uint32_t n1 = A1.n + B1.n, n2 = A2.n + B2.n, n = n1 + n2;
   const uint32_t per = (n + LV_T - 1) / LV_T;
   const uint32_t d0 = min(threadIdx.x * per, n), d1 = min(d0 + per, n);
   mp_merge_part(sm, A1, B1, out1, min(d0, n1), min(d1, n1));
   if (n2) mp_merge_part(sm, A2, B2, out2, max(d0, n1) - n1, max(d1, n1) - n1);
}

// Merge the non-empty segments sm.off/len (<= 4 inputs + exceptions) into sm.perm.
__device__ void lv_merge(LvSmem& sm)
{
   const uint32_t tid = threadIdx.x;
   MList S[LV_SEG];
   uint32_t ns = 0, E = 0;
#pragma unroll
   for (int q = 0; q < LV_SEG; q++)
   {
      const uint32_t len = sm.len[q];
      E += len;
      MList l;
      l.idx = nullptr;
      l.off = sm.off[q];
      l.n = len;
      // compact non-empty segments to the front (unrolled selects, no scratch)
#pragma unroll
      for (int r = 0; r < LV_SEG; r++)
         if (len && (uint32_t) r == ns) S[r] = l;
      ns += len ? 1u : 0u;
   }
   const MList none = { nullptr, 0, 0 };
   if (ns <= 1)
   {
      const uint32_t base = ns ? S[0].off : 0;
      for (uint32_t d = tid; d < E; d += LV_T) sm.perm[d] = (uint16_t) (base + d);
   }
   else if (ns == 2)
   {
      mp_round(sm, S[0], S[1], sm.perm, none, none, nullptr);
   }
   else if (ns == 3)
   {
      mp_round(sm, S[0], S[1], sm.tmp, none, none, nullptr);
      lv_bar();
      const MList T01 = { sm.tmp, 0, S[0].n + S[1].n };
      mp_round(sm, T01, S[2], sm.perm, none, none, nullptr);
   }
   else
   {
      const uint32_t n01 = S[0].n + S[1].n, n23 = S[2].n + S[3].n;
      mp_round(sm, S[0], S[1], sm.tmp, S[2], S[3], sm.tmp + n01);
      lv_bar();
      const MList T01 = { sm.tmp, 0, n01 }, T23 = { sm.tmp, n01, n23 };
      mp_round(sm, T01, T23, sm.perm, none, none, nullptr);
      if (ns == 5)
      {
         lv_bar();
         const MList P4 = { sm.perm, 0, n01 + n23 };
         mp_round(sm, P4, S[4], sm.tmp, none, none, nullptr);
         lv_bar();
         for (uint32_t d = tid; d < E; d += LV_T) sm.perm[d] = sm.tmp[d];
      }
   }
   if (tid == 0) sm.E = E;
   lv_bar();
}

// ---------------------------------------------------------------------------
// load + merge one leaf: main ranges sm.lo/hi of every input plus the
// exceptions whose key lies in [klo, khi)
// ---------------------------------------------------------------------------
__device__ void lv_load_merge(LvSmem& sm, const Rec* __restrict__ recs, uint64_t klo_t, uint32_t klo_i, uint64_t khi_t,
                              uint32_t khi_i, bool has_lo, bool has_hi, bool take_exc)
{
   const uint32_t tid = threadIdx.x;
   const uint32_t nin = sm.io.nin;
   if (tid == 0)
   {
      uint32_t o = 0;
      for (uint32_t s = 0; s < (uint32_t) LV_IN; s++)
      {
         sm.off[s] = o;
         sm.len[s] = s < nin ? sm.hi[s] - sm.lo[s] : 0;
         o += sm.len[s];
      }
      sm.off[LV_IN] = o;
      sm.len[LV_IN] = 0;
      sm.nexc_leaf = 0;
   }
   lv_bar();
   {
      // all of this thread's (<= LV_PER) records in flight at once, then to LDS
      const uint32_t tot = sm.off[LV_IN];
      uint32_t o1 = sm.off[1], o2 = sm.off[2], o3 = sm.off[3];
      const Rec* r0 = recs + sm.io.base[0] + sm.lo[0];
      const Rec* r1 = recs + sm.io.base[1] + sm.lo[1] - o1;
      const Rec* r2 = recs + sm.io.base[2] + sm.lo[2] - o2;
      const Rec* r3 = recs + sm.io.base[3] + sm.lo[3] - o3;
      Rec v[LV_PER];
#pragma unroll
      for (int k = 0; k < LV_PER; k++)
      {
         const uint32_t idx = tid + (uint32_t) k * LV_T;
         if (idx < tot)
         {
            const Rec* r = idx >= o3 ? r3 : idx >= o2 ? r2 : idx >= o1 ? r1 : r0;
            v[k] = r[idx];
         }
      }
#pragma unroll
      for (int k = 0; k < LV_PER; k++)
      {
         const uint32_t idx = tid + (uint32_t) k * LV_T;
         if (idx < tot)
         {
            sm.kt[idx] = v[k].t;
            sm.ki[idx] = v[k].id;
            sm.ka[idx] = v[k].aux;
         }
      }
   }
   lv_bar();
   if (tid == 0) sm.tm[0] = __builtin_amdgcn_s_memtime();
   bool anyexc = false;
   for (uint32_t s = 0; s < nin; s++) anyexc |= sm.nxe[s] > 0;
   if (anyexc && take_exc)
   {
      const uint32_t o = sm.off[LV_IN];
      for (uint32_t s = 0; s < nin; s++)
      {
         const Rec* r = recs + sm.io.base[s];
         for (uint32_t i = sm.nmain[s] + tid; i < sm.io.cnt[s]; i += LV_T)
         {
            const Rec v = r[i];
            const bool ge = !has_lo || !rlt(v, klo_t, klo_i);
            const bool lt = !has_hi || rlt(v, khi_t, khi_i);
            if (ge && lt)
            {
               const uint32_t k = atomicAdd(&sm.nexc_leaf, 1u);
               if (o + k < (uint32_t) LV_CAP)
               {
                  sm.kt[o + k] = v.t;
                  sm.ki[o + k] = v.id;
                  sm.ka[o + k] = v.aux;
               }
            }
         }
      }
      lv_bar();
      const uint32_t ne = min(sm.nexc_leaf, (uint32_t) LV_CAP - o);
      // odd-even transposition sort of the (few) exceptions
      for (uint32_t ph = 0; ph < ne; ph++)
      {
         for (uint32_t i = 2 * tid + (ph & 1); i + 1 < ne; i += 2 * LV_T)
         {
            const uint32_t a = o + i, b = o + i + 1;
            if (klt(sm, b, sm.kt[a], sm.ki[a]))
            {
               const uint64_t t = sm.kt[a]; sm.kt[a] = sm.kt[b]; sm.kt[b] = t;
               uint32_t x = sm.ki[a]; sm.ki[a] = sm.ki[b]; sm.ki[b] = x;
               x = sm.ka[a]; sm.ka[a] = sm.ka[b]; sm.ka[b] = x;
            }
         }
         lv_bar();
      }
      if (tid == 0) sm.len[LV_IN] = ne;
   }
   lv_bar();
   if (tid == 0) sm.tm[1] = __builtin_amdgcn_s_memtime();
   lv_merge(sm);
}

// ---------------------------------------------------------------------------
// per-thread merged segment in registers + block scan
// ---------------------------------------------------------------------------
// This thread's contiguous merged segment [a, a+n) of positions [s0, E);
// its records are read from LDS where used (not held across the look-back).
struct Seg
{
   uint32_t a, n;
};

struct Scan3
{
   uint64_t eA, eB, eC;   // exclusive prefix of this thread
   uint64_t tA, tB, tC;   // block totals
};

__device__ __forceinline__ void lv_load_seg(const LvSmem& sm, uint32_t s0, uint32_t E, Seg& sg)
{
   const uint32_t cnt = E - s0;
   const uint32_t per = (cnt + LV_T - 1) / LV_T;   // <= LV_PER since E <= LV_CAP
   const uint32_t a = s0 + min(threadIdx.x * per, cnt);
   const uint32_t b = s0 + min((threadIdx.x + 1) * per, cnt);
   sg.a = a;
   sg.n = b - a;
}

template <bool BC>
__device__ Scan3 lv_scan(LvSmem& sm, const Seg& sg)
{
   const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
   const uint32_t dir = sm.io.dir, nx = sm.io.nx, ny = sm.io.ny;
   uint64_t A = 0, B = 0, C = 0;
   for (uint32_t i = 0; i < sg.n; i++)
   {
      const uint32_t k = sm.perm[sg.a + i];
      const uint32_t ax = sm.ka[k];
      const uint64_t p = aux_F(ax);
      mp_comp(A, B, p, LV_CYC(sm.kt[k]) + p);
      if (!BC || !(ax & AUX_BC)) C += 1ull << (12 * next_dir(ax, dir, nx, ny));   // broadcast children: tails
   }
   uint64_t iA = A, iB = B, iC = C;
   for (int off = 1; off < 64; off <<= 1)
   {
      const uint64_t pA = __shfl_up(iA, off), pB = __shfl_up(iB, off), pC = __shfl_up(iC, off);
      if ((int) lane >= off)
      {
         uint64_t x = pA, y = pB;
         mp_comp(x, y, iA, iB);
         iA = x;
         iB = y;
         iC += pC;
      }
   }
   lv_bar();
   if (lane == 63) { sm.wA[wv] = iA; sm.wB[wv] = iB; sm.wC[wv] = iC; }
   lv_bar();
   Scan3 o;
   uint64_t PA = 0, PB = 0, PC = 0;
   for (uint32_t w = 0; w < wv; w++)
   {
      mp_comp(PA, PB, sm.wA[w], sm.wB[w]);
      PC += sm.wC[w];
   }
   uint64_t xA = __shfl_up(iA, 1), xB = __shfl_up(iB, 1), xC = __shfl_up(iC, 1);
   if (lane == 0) { xA = 0; xB = 0; xC = 0; }
   mp_comp(PA, PB, xA, xB);
   o.eA = PA;
   o.eB = PB;
   o.eC = PC + xC;
   uint64_t TA = 0, TB = 0, TC = 0;
   for (uint32_t w = 0; w < LV_T / 64; w++)
   {
      mp_comp(TA, TB, sm.wA[w], sm.wB[w]);
      TC += sm.wC[w];
   }
   o.tA = TA;
   o.tB = TB;
   o.tC = TC;
   return o;
}

// A broadcast record served with queue delay cc at this port (tc = its arrival
// cycle): the delay its router visit charges -- the max over the visit's ports (bc_visit) -- then its receipt (SELF) or one record into the exception tail of
// each tree port at the next router (bc_mask).  Returns the charged delay.
__device__ uint64_t lv_bcast(const LvSmem& sm, const DevCfg& c, uint64_t t, uint32_t id, uint32_t ax, uint64_t cc,
                             const BcWin& w, uint64_t rl, Rec* __restrict__ recs, uint32_t* __restrict__ nexc,
                             unsigned* __restrict__ errflag)
{
   const uint32_t dir = sm.io.dir;
   uint64_t ch = cc;
   uint64_t v = 0;
   if (dir != P_INJ)
   {
      // all later directions (a port the visit did not select has an empty record;
      // computing this router's tree ports here measured slower)
      v = (uint64_t) c.bc_idx[id] * c.N + sm.io.port / PORTS;
      ch = bc_visit(c, v, dir, 0x1Fu, LV_CYC(t), cc, w);
   }
   const uint64_t tn = t + LV_PS(ch) + rl;
   if (dir == P_SELF)
   {
      c.bc_fin[v] = tn + LV_PS(aux_F(ax));
      return ch;
   }
   const uint32_t m = bc_mask(aux_dx(ax), aux_dy(ax), sm.io.nx, sm.io.ny, c.W, c.H);
   for (uint32_t nd = 0; nd < 5; nd++)
   {
      if (!((m >> nd) & 1u)) continue;
      const uint32_t x = atomicAdd(&nexc[sm.io.oslot[nd]], 1u);
      if (x >= sm.io.ocnt[nd]) { atomicOr(errflag, 1u); continue; }
      lv_store_rec(recs + sm.io.obase[nd] + sm.io.ocnt[nd] - 1 - x, tn, id, ax);
   }
   return ch;
}

// The queue neighbourhood (BcWin) of the broadcast record at merged position j
// (arrival tc, busy-until xb ahead of it), from the chunk's merged records in
// LDS.  Ahead of the previous record the queue was busy until xb - F_prev when
// that exceeds its arrival; otherwise it was idle there (0).
__device__ __noinline__ BcWin lv_bcwin(const LvSmem& sm, uint32_t j, uint64_t tc, uint64_t xb)
{
   BcWin w;
   w.ap = tc;
   w.bp = 0;
   w.b = xb;
   w.an = ~0ull;
   w.bn = xb;
   if (j > 0)
   {
      const uint32_t kp = sm.perm[j - 1];
      const uint64_t ap = LV_CYC(sm.kt[kp]), fp = aux_F(sm.ka[kp]);
      w.ap = ap;
      w.bp = xb > ap + fp ? xb - fp : 0;
   }
   if (j + 1 < sm.E)
   {
      const uint32_t kn = sm.perm[j + 1];
      w.an = LV_CYC(sm.kt[kn]);
      w.bn = (xb > w.an ? xb : w.an) + aux_F(sm.ka[kn]);
   }
   return w;
}

// Serial prefix while the queue has never idled (history tree + M/G/1), one
// thread, from merged position 0; outputs written directly.  -> sm.s0
template <bool BC>
__device__ void lv_serial(LvSmem& sm, const DevCfg& c, Rec* __restrict__ recs, uint64_t* __restrict__ samp_t,
                          uint32_t* __restrict__ samp_id, uint32_t* __restrict__ nexc, uint64_t* __restrict__ final_ps,
                          unsigned* __restrict__ errflag)
{
   if (threadIdx.x == 0)
   {
      const uint32_t E = sm.E;
      const uint32_t dir = sm.io.dir, nx = sm.io.nx, ny = sm.io.ny;
      const uint64_t rl = dir == P_INJ ? 0ull : (uint64_t) sm.io.rl;
      SerialState s;
      s.X = sm.cy.X; s.g = (int) sm.cy.g; s.mode = 1; s.s1 = sm.cy.s1; s.s2 = sm.cy.s2;
      s.narr = sm.cy.narr; s.newest = sm.cy.newest; s.mg1 = 0;
      uint32_t e = 0;
      uint64_t ssum = 0, sflit = 0, slast = 0;
      for (; e < E && s.mode; e++)
      {
         const uint32_t k = sm.perm[e];
         const uint64_t t = sm.kt[k];
         const uint32_t id = sm.ki[k], ax = sm.ka[k];
         const uint64_t mg_before = s.mg1;
         const uint64_t cc = serial_step(s, LV_CYC(t), aux_F(ax), c.max_list, c.analytical);
         if (s.g >= 1) s.mode = 0;
         sflit += aux_F(ax);
         const uint64_t dep = LV_CYC(t) + cc + aux_F(ax);
         slast = slast > dep ? slast : dep;
         if (BC && (ax & AUX_BC))
         {
            ssum += lv_bcast(sm, c, t, id, ax, cc, bc_win_wait(LV_CYC(t), cc), rl, recs, nexc, errflag);
            continue;
         }
         ssum += cc;
         const uint64_t tn = t + LV_PS(cc) + rl;
         if (dir == P_SELF)
         {
            if (id < c.npk) final_ps[id] = tn + LV_PS(aux_F(ax));
            else atomicOr(errflag, 1u);
            continue;
         }
         const uint32_t nd = next_dir(ax, dir, nx, ny);
         Rec o;
         o.t = tn;
         o.id = id;
         o.aux = ax;
         if (s.mg1 != mg_before)
         {
            // M/G/1-served: may leave FIFO order -> exception tail of the slot
            const uint32_t x = atomicAdd(&nexc[sm.io.oslot[nd]], 1u);
            atomicOr(errflag + 2, 1u);   // "some slot has exceptions": later levels read nexc
            if (x >= sm.io.ocnt[nd]) { atomicOr(errflag, 1u); continue; }
            lv_store_rec(recs + sm.io.obase[nd] + sm.io.ocnt[nd] - 1 - x, o.t, o.id, o.aux);
         }
         else
         {
            const uint32_t pos = sm.cy.cnt[nd]++;
            if (pos >= sm.io.ocnt[nd]) { atomicOr(errflag, 1u); continue; }
            lv_put(recs, samp_t, samp_id, sm.io.obase[nd] + pos, tn, id, ax);
         }
      }
      sm.s0 = e;
      sm.cy.X = s.X; sm.cy.g = (uint32_t) s.g; sm.cy.mode = s.mode; sm.cy.s1 = s.s1; sm.cy.s2 = s.s2;
      sm.cy.narr = s.narr; sm.cy.newest = s.newest;
      sm.st_sum += ssum;
      sm.st_flit += sflit;
      sm.st_last = sm.st_last > slast ? sm.st_last : slast;
      sm.st_cnt += e;
      sm.st_mg1 += (uint32_t) s.mg1;
   }
   lv_bar();
}

// Recurrence + stores of this thread's segment from carry sm.cy; then the
// carry advances by the block totals.
template <bool BC>
__device__ void lv_emit(LvSmem& sm, const DevCfg& c, const Seg& sg, const Scan3& so, Rec* __restrict__ recs,
                        uint64_t* __restrict__ samp_t, uint32_t* __restrict__ samp_id, uint64_t* __restrict__ final_ps,
                        uint32_t* __restrict__ nexc, unsigned* __restrict__ errflag)
{
   const uint32_t lane = threadIdx.x & 63;
   const uint32_t dir = sm.io.dir, nx = sm.io.nx, ny = sm.io.ny;
   const uint64_t rl = dir == P_INJ ? 0ull : (uint64_t) sm.io.rl;
   const uint64_t X0 = sm.cy.X;
   uint64_t X = X0 + so.eA;
   X = X > so.eB ? X : so.eB;
   uint64_t ssum = 0;
   uint32_t run[5];
#pragma unroll
   for (int d = 0; d < 5; d++) run[d] = sm.cy.cnt[d] + cfield(so.eC, d);
   for (uint32_t i = 0; i < sg.n; i++)
   {
      {
         const uint32_t k = sm.perm[sg.a + i];
         const uint64_t t = sm.kt[k];
         const uint32_t id = sm.ki[k];
         const uint32_t ax = sm.ka[k];
         const uint64_t tc = LV_CYC(t);
         const uint64_t cc = X > tc ? X - tc : 0;
         const uint64_t xb = X;
         X = (X > tc ? X : tc) + aux_F(ax);
         if (BC && (ax & AUX_BC))
         {
            ssum += lv_bcast(sm, c, t, id, ax, cc, lv_bcwin(sm, sg.a + i, tc, xb), rl, recs, nexc, errflag);
            continue;
         }
         ssum += cc;
         const uint64_t tn = t + LV_PS(cc) + rl;
         if (dir == P_SELF)
         {
            // NetworkModel::processReceivedPacket: + serialization (network_model.cc:142-150)
            if (id < c.npk) final_ps[id] = tn + LV_PS(aux_F(ax));
            else atomicOr(errflag, 1u);
            continue;
         }
         const uint32_t nd = next_dir(ax, dir, nx, ny);
         uint32_t pos = 0;
#pragma unroll
         for (int d = 0; d < 5; d++)
            if (nd == (uint32_t) d) pos = run[d]++;
         if (pos >= sm.io.ocnt[nd])
         {
            atomicOr(errflag, 1u);   // route-count invariant broken: never write outside the slot
            continue;
         }
         const uint64_t gp = sm.io.obase[nd] + pos;
         lv_put(recs, samp_t, samp_id, gp, tn, id, ax);
      }
   }
   for (int off = 32; off > 0; off >>= 1) ssum += __shfl_down(ssum, off);
   if (lane == 0 && ssum) atomicAdd((unsigned long long*) &sm.st_sum, (unsigned long long) ssum);
   lv_bar();
   if (threadIdx.x == 0)
   {
      sm.st_cnt += sm.E - sm.s0;
      const uint64_t nx0 = X0 + so.tA;
      sm.cy.X = nx0 > so.tB ? nx0 : so.tB;
      if (sm.E > sm.s0)
      {
         // FIFO-served: departures increase, the last one is the new queue tail X
         sm.st_flit += so.tA;
         sm.st_last = sm.st_last > sm.cy.X ? sm.st_last : sm.cy.X;
      }
      for (uint32_t d = 0; d < 5; d++) sm.cy.cnt[d] += cfield(so.tC, d);
   }
   lv_bar();
}

// A whole merged leaf from carry sm.cy (serial prefix if needed).
template <bool BC>
__device__ void lv_leaf(LvSmem& sm, const DevCfg& c, Rec* __restrict__ recs, uint64_t* __restrict__ samp_t,
                        uint32_t* __restrict__ samp_id, uint32_t* __restrict__ nexc, uint64_t* __restrict__ final_ps,
                        unsigned* __restrict__ errflag)
{
   if (threadIdx.x == 0) sm.s0 = 0;
   lv_bar();
   if (sm.cy.mode) lv_serial<BC>(sm, c, recs, samp_t, samp_id, nexc, final_ps, errflag);
   Seg sg;
   lv_load_seg(sm, sm.s0, sm.E, sg);
   const Scan3 so = lv_scan<BC>(sm, sg);
   lv_emit<BC>(sm, c, sg, so, recs, samp_t, samp_id, final_ps, nexc, errflag);
}

// ---------------------------------------------------------------------------
// decoupled look-back (wave 0).  Chunk state: 16 x u64, zeroed before the run;
// every word validates itself (8-byte sc1 granules), so one load round trip
// returns flags and data together.
//   [0] A+1  [1] B+1  [2] counts(5 x 12 bit) | TAG                 aggregate
//   [3] X+1  [4] c0 | c1<<31 | TAG  [5] c2 | c3<<31 | TAG
//   [6] c4 | mode<<31 | g<<32 | TAG                                  inclusive
//   [7] s1 [8] s2 [9] narr [10] newest  (serial M/G/1 state, stored before
//   [3..6] and drained, read only when mode == 1)
// ---------------------------------------------------------------------------
__device__ void lv_publish_agg(uint64_t* __restrict__ st, uint32_t g, const Scan3& so)
{
   uint64_t* w = st + (uint64_t) g * LV_STATE_WORDS;
   lv_st(w + 0, so.tA + 1);
   lv_st(w + 1, so.tB + 1);
   lv_st(w + 2, so.tC | LV_TAG);
}

__device__ void lv_publish_inc(uint64_t* __restrict__ st, uint32_t g, const Carry3& cy)
{
   uint64_t* w = st + (uint64_t) g * LV_STATE_WORDS;
   if (cy.mode)
   {
      lv_st(w + 7, (uint64_t) __double_as_longlong(cy.s1));
      lv_st(w + 8, (uint64_t) __double_as_longlong(cy.s2));
      lv_st(w + 9, cy.narr);
      lv_st(w + 10, cy.newest);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
   }
   lv_st(w + 3, cy.X + 1);
   lv_st(w + 4, LV_TAG | (uint64_t) cy.cnt[0] | ((uint64_t) cy.cnt[1] << 31));
   lv_st(w + 5, LV_TAG | (uint64_t) cy.cnt[2] | ((uint64_t) cy.cnt[3] << 31));
   lv_st(w + 6, LV_TAG | (uint64_t) cy.cnt[4] | ((uint64_t) (cy.mode & 1u) << 31) | ((uint64_t) cy.g << 32));
}

__device__ __forceinline__ void lv_take_inc(LvSmem& sm, const uint64_t* __restrict__ w, uint64_t X1, uint64_t c01,
                                            uint64_t c23, uint64_t c4m, uint64_t accA, uint64_t accB,
                                            const uint32_t* accC)
{
   const uint64_t X = X1 - 1;
   const uint64_t nx = X + accA;
   sm.cy.X = nx > accB ? nx : accB;
   sm.cy.mode = (uint32_t) ((c4m >> 31) & 1u);
   sm.cy.g = (uint32_t) ((c4m >> 32) & 0x7FFFFFFFu);
   sm.cy.cnt[0] = (uint32_t) (c01 & 0x7FFFFFFFu) + accC[0];
   sm.cy.cnt[1] = (uint32_t) ((c01 >> 31) & 0x7FFFFFFFu) + accC[1];
   sm.cy.cnt[2] = (uint32_t) (c23 & 0x7FFFFFFFu) + accC[2];
   sm.cy.cnt[3] = (uint32_t) ((c23 >> 31) & 0x7FFFFFFFu) + accC[3];
   sm.cy.cnt[4] = (uint32_t) (c4m & 0x7FFFFFFFu) + accC[4];
   if (sm.cy.mode)
   {
      sm.cy.s1 = __longlong_as_double((long long) lv_ld(w + 7));
      sm.cy.s2 = __longlong_as_double((long long) lv_ld(w + 8));
      sm.cy.narr = lv_ld(w + 9);
      sm.cy.newest = lv_ld(w + 10);
   }
}

__device__ bool lv_lookback(LvSmem& sm, uint32_t gbase, uint32_t j, const uint64_t* __restrict__ st,
                            unsigned* __restrict__ errflag)
{
   const uint32_t lane = threadIdx.x & 63;
   uint64_t accA = 0, accB = 0;
   uint32_t accC[5] = { 0, 0, 0, 0, 0 };
   int32_t look = (int32_t) j - 1;
   uint32_t spins = 0;
   const uint64_t t_start = __builtin_amdgcn_s_memtime();
   for (;;)
   {
      const int32_t ck = look - (int32_t) lane;
      uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0, w4 = 0, w5 = 0, w6 = 0;
      if (ck >= 0)
      {
         const uint64_t* w = st + (uint64_t) (gbase + ck) * LV_STATE_WORDS;
         w0 = lv_ld(w + 0); w1 = lv_ld(w + 1); w2 = lv_ld(w + 2);
         w3 = lv_ld(w + 3); w4 = lv_ld(w + 4); w5 = lv_ld(w + 5); w6 = lv_ld(w + 6);
      }
      const bool aggv = w0 && w1 && (w2 & LV_TAG);
      const bool incv = w3 && (w4 & LV_TAG) && (w5 & LV_TAG) && (w6 & LV_TAG);
      const uint64_t inc = __ballot(ck >= 0 && incv);
      const uint64_t bad = __ballot(ck >= 0 && !incv && !aggv);
      const uint64_t stop = inc | __ballot(ck < 0);
      const int L = stop ? __ffsll((long long) stop) - 1 : 64;
      const uint64_t need = L >= 64 ? ~0ull : ((1ull << L) - 1);
      if (bad & need)
      {
         ++spins;
         if (__builtin_amdgcn_s_memtime() - t_start > LV_SPIN_CYCLES) { if (lane == 0) atomicOr(errflag, 2u); return false; }
         if (__hip_atomic_load(errflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 6u) return false;   // another chunk gave up
         __builtin_amdgcn_s_sleep(1);
         continue;
      }
      // compose aggregates in chunk order: earliest (lane L-1) first ... lane 0 last, then the tail so far
      const uint64_t a = (int) lane < L ? w0 - 1 : 0, b = (int) lane < L ? w1 - 1 : 0;
      uint64_t wa = 0, wb = 0;
      for (int l = L - 1; l >= 0; l--) mp_comp(wa, wb, __shfl(a, l), __shfl(b, l));
      mp_comp(wa, wb, accA, accB);
      accA = wa;
      accB = wb;
#pragma unroll
      for (uint32_t d = 0; d < 5; d++)
      {
         uint32_t v = (int) lane < L ? cfield(w2, d) : 0u;
         for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
         accC[d] += v;
      }
      if (L < 64)
      {
         if (lane == 0) { sm.tm[2] = __builtin_amdgcn_s_memtime(); sm.tm[3] = spins | ((uint64_t) (j - (look - L)) << 32); }
         const int32_t sc = look - L;   // chunk holding an inclusive state (chunk 0 always publishes one)
         const uint64_t X1 = __shfl(w3, L), c01 = __shfl(w4, L), c23 = __shfl(w5, L), c4m = __shfl(w6, L);
         const uint32_t mode = (uint32_t) ((c4m >> 31) & 1u);
         if (mode && sc != (int32_t) j - 1)
         {
            // the queue was still in its serial prefix: FIFO aggregates after it are invalid;
            // wait for the immediate predecessor's inclusive state instead.
            const uint64_t* w = st + (uint64_t) (gbase + j - 1) * LV_STATE_WORDS;
            uint64_t p3, p4, p5, p6;
            for (;;)
            {
               p3 = lv_ld(w + 3); p4 = lv_ld(w + 4); p5 = lv_ld(w + 5); p6 = lv_ld(w + 6);
               if (p3 && (p4 & LV_TAG) && (p5 & LV_TAG) && (p6 & LV_TAG)) break;
               if (__builtin_amdgcn_s_memtime() - t_start > LV_SPIN_CYCLES) { if (lane == 0) atomicOr(errflag, 2u); return false; }
               if (__hip_atomic_load(errflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 6u) return false;
               __builtin_amdgcn_s_sleep(1);
            }
            const uint32_t zero[5] = { 0, 0, 0, 0, 0 };
            if (lane == 0) lv_take_inc(sm, w, p3, p4, p5, p6, 0, 0, zero);
         }
         else if (lane == 0)
         {
            lv_take_inc(sm, st + (uint64_t) (gbase + sc) * LV_STATE_WORDS, X1, c01, c23, c4m, accA, accB, accC);
         }
         return true;
      }
      look -= 64;
   }
}

// ---------------------------------------------------------------------------
// the level kernel: a persistent grid pulls the level's chunks in order
// ---------------------------------------------------------------------------
// Next-chunk prefetch, by waves 1..3 of the workgroup (results in sm.nx).
// lv_fetch_keys: input exception counts, split keys (wave 1), then the sample
// searches of the other inputs (all three waves).  In the cross-level launch
// (XL) it first needs every producer port of the chunk complete: blocking, it
// waits; otherwise it returns false and leaves the work to the take.
template <bool XL>
__device__ __noinline__ bool lv_fetch_keys(LvSmem& sm, bool block, bool anyexc, const Rec* __restrict__ recs,
                                           const uint64_t* __restrict__ samp_t, const uint32_t* __restrict__ samp_id,
                                           const uint32_t* __restrict__ nexc, const uint32_t* __restrict__ done,
                                           unsigned* __restrict__ errflag)
{
   const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
   auto& d = sm.nx;
   if (wv == 1)
   {
      const uint32_t nin = d.io.nin;
      bool go = true;
      if (XL)
      {
         // producer ports complete?  (release: end of every producer chunk)
         const uint64_t t_start = __builtin_amdgcn_s_memtime();
         for (;;)
         {
            bool ok = true;
            if (lane < nin && d.io.prod[lane] != LV_NO_PROD)
               ok = __hip_atomic_load(&done[d.io.prod[lane]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                    d.io.prod_nc[lane];
            if (__all(ok)) break;
            if (!block) { go = false; break; }
            if (__builtin_amdgcn_s_memtime() - t_start > LV_SPIN_CYCLES) { if (lane == 0) atomicOr(errflag, 2u); break; }
            if (__hip_atomic_load(errflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 6u) break;
            __builtin_amdgcn_s_sleep(2);
         }
         if (go)
         {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // this CU's L1 may hold stale lines
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
         }
      }
      if (go)
      {
         if (lane < nin)
         {
            // exception counts only if some earlier level wrote exceptions (rare)
            const uint32_t x = anyexc ? nexc[d.io.slot[lane]] : 0u;
            d.nxe[lane] = x;
            d.nmain[lane] = d.io.cnt[lane] - x;
         }
         asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
         const uint32_t j = d.g - d.io.gbase, nc = d.io.nc, sb = d.io.sb;
         const uint32_t nb = d.nmain[sb];
         uint32_t has_lo = j > 0, has_hi = j + 1 < nc, empty = 0;
         if (nb == 0) { empty = j > 0; has_lo = has_hi = 0; }   // only exceptions: chunk 0 takes all
         // split indices on 64-record boundaries: the split key is a sample
         const uint32_t ilo = (uint32_t) (((uint64_t) j * nb) / nc) & ~63u;
         const uint32_t ihi = (uint32_t) (((uint64_t) (j + 1) * nb) / nc) & ~63u;
         if (lane == 2)
         {
            d.has_lo = has_lo; d.has_hi = has_hi; d.empty = empty;
            d.ilo = ilo; d.ihi = ihi;
            for (uint32_t q = 0; q < 2 * (uint32_t) LV_IN; q++) d.search[q] = 0;
            if (!empty)
            {
               d.search[2 * sb] = has_lo ? ilo : 0;
               d.search[2 * sb + 1] = has_hi ? ihi : nb;
               for (uint32_t s = 0; s < nin; s++)
                  if (s != sb)
                  {
                     if (!has_lo) d.search[2 * s] = 0;
                     if (!has_hi) d.search[2 * s + 1] = d.nmain[s];
                  }
            }
         }
      }
      if (lane == 3) d.deferred = go ? 0u : 1u;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(&d.ready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
   }
   else
   {
      while (__hip_atomic_load(&d.ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
         __builtin_amdgcn_s_sleep(1);
   }
   if (d.deferred) return false;
   const uint32_t sb = d.io.sb;
   const uint64_t kb = d.io.base[sb] >> 6;   // sample index of the split input's first record
   if (wv == 1)
   {
      // the chunk's own key range (exception filter, leaf splits)
      if (lane == 0)
      {
         d.klo_t = 0; d.klo_i = 0;
         if (!d.empty && d.has_lo) { d.klo_t = samp_t[kb + d.ilo / 64]; d.klo_i = samp_id[kb + d.ilo / 64]; }
      }
      if (lane == 1)
      {
         d.khi_t = ~0ull; d.khi_i = ~0u;
         if (!d.empty && d.has_hi) { d.khi_t = samp_t[kb + d.ihi / 64]; d.khi_i = samp_id[kb + d.ihi / 64]; }
      }
   }
   if (d.empty) return true;
   const uint32_t nin = d.io.nin;
   for (uint32_t q = wv - 1; q < 2 * (uint32_t) LV_IN; q += 3)
   {
      const uint32_t s = q >> 1, which = q & 1;
      if (s >= nin || s == sb) continue;
      if ((which == 0 && !d.has_lo) || (which == 1 && !d.has_hi)) continue;
      const uint64_t sbase = d.io.base[s] >> 6;
      const uint64_t ks = kb + (which ? d.ihi : d.ilo) / 64;
      const uint32_t v = wave_lb2(recs + d.io.base[s], samp_t + sbase, samp_id + sbase, d.nmain[s], samp_t + ks,
                                  samp_id + ks, lane);
      if (lane == 0) d.search[q] = v;
   }
   return true;
}

// lv_fetch: dynamic chunk id and its port descriptor (wave 1), then the keys
// if they can be had without blocking.  Waves 1..3 call it.
template <bool XL>
__device__ __noinline__ void lv_fetch(LvSmem& sm, bool first, bool anyexc, uint32_t cb0, uint32_t nch, unsigned* __restrict__ ctr,
                                      const PortIO3* __restrict__ cdesc,
                                      const Rec* __restrict__ recs, const uint64_t* __restrict__ samp_t,
                                      const uint32_t* __restrict__ samp_id, const uint32_t* __restrict__ nexc,
                                      const uint32_t* __restrict__ done, unsigned* __restrict__ errflag)
{
   const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
   auto& d = sm.nx;
   if (wv == 1)
   {
      // 8 dequeue heads (one word saturates near 90 dequeues/us): group q = blockIdx % 8
      // takes chunks q, q+8, q+16, ... in order, so every predecessor of a chunk
      // is held by a running workgroup or done.  The first chunk of each
      // workgroup is static (blockIdx / 8), so a level starts without the atomic.
      uint32_t idx = 0xFFFFFFFFu;
#ifdef LV_QSPREAD
      const uint32_t q0 = (blockIdx.x / 8) & (LV_QUEUES - 1);   // a queue's workgroups on every XCD
#else
      const uint32_t q0 = blockIdx.x & (LV_QUEUES - 1);
#endif
      if (XL || !LV_PORT_QUEUES)
      {
         uint32_t cid = blockIdx.x / LV_QUEUES;
         if (!first)
         {
            if (lane == 0) cid = atomicAdd(ctr + q0, 1u) + (gridDim.x - q0 + LV_QUEUES - 1) / LV_QUEUES;
            cid = __shfl(cid, 0);
         }
         idx = q0 + LV_QUEUES * cid;
      }
      else
      {
         // Port-aligned queues: every chunk of a port sits in one queue and is
         // handed out in order, so its predecessor is already held by a running
         // workgroup (or done).  Group q starts with chunk blockIdx/8 of queue q
         // (static), then takes from its queue's head; a drained queue sends its
         // workgroups on to the next queues (still in-order within each queue).
         if (first)
         {
#ifdef LV_QSPREAD
            const uint32_t k = (blockIdx.x & 7) + 8 * (blockIdx.x / (8 * LV_QUEUES));
#else
            const uint32_t k = blockIdx.x / LV_QUEUES;
#endif
            if (k < sm.qb[q0 + 1] - sm.qb[q0]) idx = sm.qb[q0] + k;
         }
         for (uint32_t t = 0; t < LV_QUEUES && idx == 0xFFFFFFFFu; t++)
         {
            const uint32_t q = (q0 + t) & (LV_QUEUES - 1);
            if ((sm.qdone >> q) & 1u) continue;
            const uint32_t size = sm.qb[q + 1] - sm.qb[q];
            const uint32_t nst = (gridDim.x - q + LV_QUEUES - 1) / LV_QUEUES;   // taken statically
            uint32_t cid = 0xFFFFFFFFu;
            if (size > nst)
            {
               if (lane == 0) cid = atomicAdd(ctr + q, 1u) + nst;
               cid = __shfl(cid, 0);
            }
            if (cid < size) idx = sm.qb[q] + cid;
            else if (lane == 0) sm.qdone |= 1u << q;
         }
      }
      const uint32_t valid = idx < nch ? 1u : 0u;
      const uint32_t g = cb0 + idx;
      if (valid)
      {
         // the chunk's own copy of its port descriptor (k_plan_fill): one load
         const uint32_t* srcw = reinterpret_cast<const uint32_t*>(cdesc + g);
         uint32_t* dstw = reinterpret_cast<uint32_t*>(&d.io);
         constexpr uint32_t PKW = offsetof(PortIO3, pk) / 4;
         if (lane < (uint32_t) (sizeof(PortIO3) / 4))
         {
            const uint32_t v = srcw[lane];
            dstw[lane] = v;
            if (lane == PKW) d.pk = v;
         }
      }
      if (lane == 3) { d.g = g; d.valid = valid; }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
   }
   // waves 2, 3 wait inside lv_fetch_keys for wave 1's ready flag
   if (wv == 1 && !d.valid)
   {
      if (lane == 0)
      {
         d.deferred = 0;
         d.empty = 1;
         __hip_atomic_store(&d.ready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      return;
   }
   lv_fetch_keys<XL>(sm, false, anyexc, recs, samp_t, samp_id, nexc, done, errflag);
}

#define LV_STAMP(k)                                                                                          \
   do                                                                                                       \
   {                                                                                                        \
      if (STAMPS && stamps && tid == 0) stamps[(uint64_t) g * 16 + (k)] = __builtin_amdgcn_s_memtime();     \
   } while (0)

#ifndef LV_MIN_WAVES
#define LV_MIN_WAVES 4   // waves per SIMD the register allocation must leave room for
#endif

template <bool STAMPS, bool XL, bool BC>
__global__ __launch_bounds__(LV_T, LV_MIN_WAVES) void k_level(DevCfg c, uint32_t level, const uint32_t* __restrict__ lvl_cbase,
                                                const uint32_t* __restrict__ lvl_qb,
                                                unsigned* __restrict__ ctr, const PortIO3* __restrict__ cdesc,
                                                Rec* __restrict__ recs,
                                                uint64_t* __restrict__ samp_t, uint32_t* __restrict__ samp_id,
                                                uint32_t* __restrict__ nexc, uint64_t* __restrict__ st,
                                                uint64_t* __restrict__ final_ps,
                                                unsigned long long* __restrict__ port_sum,
                                                unsigned long long* __restrict__ port_cnt,
                                                unsigned long long* __restrict__ port_mg1,
                                                unsigned long long* __restrict__ port_flit,
                                                unsigned long long* __restrict__ port_last, unsigned* __restrict__ errflag,
                                                uint32_t* __restrict__ done, uint64_t* __restrict__ stamps)
{
   __shared__ LvSmem sm;
   const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
   // bit 31 / 30: the level runs only if the streamed injection / SELF level declined
   // (chain.hip k_inj_stream, errflag[7]; k_self_stream, errflag[8])
   if ((level >> 31) && errflag[7] == 0) return;
   if (((level >> 30) & 1u) && errflag[8] == 0) return;
   level &= 0x3FFFFFFFu;
   // per-level launch: chunks of `level`; cross-level launch (XL, level = number of levels): all chunks
   const uint32_t cb0 = XL ? 0u : lvl_cbase[level];
   const uint32_t nch = XL ? lvl_cbase[level] : lvl_cbase[level + 1] - cb0;
   unsigned* const cctr = XL ? ctr : ctr + level * LV_QUEUES;
   // exception tails exist only if an earlier level's M/G/1 path wrote one (flag set
   // before this launch); the cross-level launch always reads the counts
   const bool anyexc = XL || errflag[2] != 0;
   // the chain engine (chain.hip) declined this batch: its outputs are incomplete,
   // the host reruns the batch on the level engine
   if (errflag[4] != 0 || errflag[5] != 0) return;
   if (tid == 0) { sm.nx.ready = 0; sm.qdone = 0; }
#if LV_GEN
   if (tid == 0) sm.fq = c.f;
#endif
   if (!XL && tid < LV_QB) sm.qb[tid] = lvl_qb[level * LV_QB + tid];
   if (XL && tid == 0) sm.qb[LV_QUEUES + 1] = 0;
   lv_bar();
   if (wv >= 1) lv_fetch<XL>(sm, true, anyexc, cb0, nch, cctr, cdesc, recs, samp_t, samp_id, nexc, done, errflag);
   lv_bar();
   for (;;)
   {
      // ---- take the prefetched chunk (its keys first, if they had to wait for producers)
      if (!sm.nx.valid)
      {
         return;
      }
      if (__hip_atomic_load(errflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 6u) return;   // rerun on v1 follows
      if (sm.nx.deferred)
      {
         if (tid == 0) sm.nx.ready = 0;
         lv_bar();
         if (wv >= 1) lv_fetch_keys<XL>(sm, true, anyexc, recs, samp_t, samp_id, nexc, done, errflag);
         lv_bar();
      }
      const uint32_t g = sm.nx.g;
      LV_STAMP(0);
      if (STAMPS && stamps && tid == 0) stamps[(uint64_t) g * 16 + 1] = __builtin_amdgcn_s_memrealtime();
      {
         const uint32_t* srcw = reinterpret_cast<const uint32_t*>(&sm.nx.io);
         uint32_t* dstw = reinterpret_cast<uint32_t*>(&sm.io);
         for (uint32_t k = tid; k < (uint32_t) (sizeof(PortIO3) / 4); k += LV_T) dstw[k] = srcw[k];
         if (tid < (uint32_t) LV_IN)
         {
            sm.nmain[tid] = sm.nx.nmain[tid];
            sm.nxe[tid] = sm.nx.nxe[tid];
         }
         if (tid < 2 * (uint32_t) LV_IN) sm.search[tid] = sm.nx.search[tid];
         if (tid == 0)
         {
            sm.klo_t = sm.nx.klo_t; sm.klo_i = sm.nx.klo_i; sm.khi_t = sm.nx.khi_t; sm.khi_i = sm.nx.khi_i;
            sm.has_lo = sm.nx.has_lo; sm.has_hi = sm.nx.has_hi; sm.empty = sm.nx.empty;
            sm.g = g;
            sm.pk = sm.nx.pk;
            sm.st_sum = 0;
            sm.st_flit = 0;
            sm.st_last = 0;
            sm.st_cnt = 0;
            sm.st_mg1 = 0;
            sm.published = 0;
            sm.cy.X = 0; sm.cy.mode = 0; sm.cy.g = 0; sm.cy.s1 = 0; sm.cy.s2 = 0; sm.cy.narr = 0; sm.cy.newest = 0;
            for (int k = 0; k < 5; k++) sm.cy.cnt[k] = 0;
         }
      }
      lv_bar();
      if (tid == 0) sm.nx.ready = 0;
      bool fetched = false;
      const uint32_t j = g - sm.io.gbase;
      const uint32_t nin = sm.io.nin;
      const bool has_lo = sm.has_lo, has_hi = sm.has_hi, empty = sm.empty;
      const uint64_t klo_t = sm.klo_t, khi_t = sm.khi_t;
      const uint32_t klo_i = sm.klo_i, khi_i = sm.khi_i;
      LV_STAMP(2);
      uint32_t total = 0, totexc = 0;
#pragma unroll
      for (uint32_t s = 0; s < (uint32_t) LV_IN; s++)
      {
         if (s < nin)
         {
            total += sm.search[2 * s + 1] - sm.search[2 * s];
            totexc += sm.nxe[s];
         }
      }
      LV_STAMP(3);
      if (empty) totexc = 0;
      if (totexc) totexc = lv_count_exc(sm, recs, klo_t, klo_i, khi_t, khi_i, has_lo, has_hi);

      if (total + totexc <= (uint32_t) LV_CAP)
      {
         // ---------------- single leaf
         if (tid < (uint32_t) LV_IN)
         {
            sm.lo[tid] = tid < nin ? sm.search[2 * tid] : 0;
            sm.hi[tid] = tid < nin ? sm.search[2 * tid + 1] : 0;
         }
         lv_bar();
         lv_load_merge(sm, recs, klo_t, klo_i, khi_t, khi_i, has_lo, has_hi, !empty);
         LV_STAMP(4);
         if (j == 0)
         {
            // The port starts in the history tree's serial state (no gap yet); its first
            // arrival keeps it there only at cycle 0 (queue_model_history_tree.cc:58-99).
            // An empty chunk 0 (every early record is an exception tail of another
            // chunk's range) hands the untouched serial state on to its successor.
            if (tid == 0 && c.analytical && (sm.E == 0 || LV_CYC(sm.kt[sm.perm[0]]) == 0)) sm.cy.mode = 1;
            if (tid == 0) sm.s0 = 0;
            lv_bar();
         }
         if (j > 0 || !sm.cy.mode)
         {
            if (tid == 0) sm.s0 = 0;
            Seg sg;
            lv_load_seg(sm, 0, sm.E, sg);
            const Scan3 so = lv_scan<BC>(sm, sg);
            LV_STAMP(5);
            if (j > 0)
            {
               if (tid == 0) lv_publish_agg(st, g, so);
               if (STAMPS && stamps && tid == 0) stamps[(uint64_t) g * 16 + 15] = __builtin_amdgcn_s_memrealtime();
               // Long ports: a chunk prefetched here waits for this chunk's look-back and
               // emit, and its successors wait on it in turn (a convoy along the port);
               // those levels fetch after the emit instead.
               const bool late = sm.qb[LV_QUEUES + 1] != 0;
               if (wv == 0) lv_lookback(sm, sm.io.gbase, j, st, errflag);
               else if (!late) lv_fetch<XL>(sm, false, anyexc, cb0, nch, cctr, cdesc, recs, samp_t, samp_id, nexc, done, errflag);
               fetched = !late;
               lv_bar();
            }
            LV_STAMP(6);
            if (!sm.cy.mode)
            {
               // FIFO: the inclusive state is (carry) x (aggregate); publish before the outputs
               if (tid == 0)
               {
                  Carry3 inc = sm.cy;
                  const uint64_t nx0 = inc.X + so.tA;
                  inc.X = nx0 > so.tB ? nx0 : so.tB;
                  for (uint32_t d = 0; d < 5; d++) inc.cnt[d] += cfield(so.tC, d);
                  lv_publish_inc(st, g, inc);
                  sm.published = 1;
               }
               lv_emit<BC>(sm, c, sg, so, recs, samp_t, samp_id, final_ps, nexc, errflag);
            }
            else
            {
               lv_leaf<BC>(sm, c, recs, samp_t, samp_id, nexc, final_ps, errflag);   // serial prefix continues
            }
         }
         else
         {
            lv_leaf<BC>(sm, c, recs, samp_t, samp_id, nexc, final_ps, errflag);
         }
         LV_STAMP(7);
      }
      else
      {
         // ---------------- burst: split the key range into leaves that fit LDS
         if (j > 0 && wv == 0) lv_lookback(sm, sm.io.gbase, j, st, errflag);
         if (tid == 0)
         {
            sm.nleaf = 1;
            sm.lk_t[0] = klo_t; sm.lk_i[0] = klo_i;
            sm.lk_t[1] = khi_t; sm.lk_i[1] = khi_i;
            for (uint32_t s = 0; s < (uint32_t) LV_IN; s++) sm.lr_lo[0][s] = s < nin ? sm.search[2 * s] : 0;
            for (uint32_t s = 0; s < (uint32_t) LV_IN; s++) sm.hi[s] = s < nin ? sm.search[2 * s + 1] : 0;
         }
         lv_bar();
         bool ok = true;
         for (uint32_t iter = 0; iter < 4 * (uint32_t) LV_MAXLEAF && ok; iter++)
         {
            int32_t bad = -1;
            uint32_t bs = 0, bestn = 0;
            for (uint32_t L = 0; L < sm.nleaf && bad < 0; L++)
            {
               uint32_t sz = 0, bn = 0, best = 0;
               for (uint32_t s = 0; s < nin; s++)
               {
                  const uint32_t h = (L + 1 < sm.nleaf) ? sm.lr_lo[L + 1][s] : sm.hi[s];
                  const uint32_t n = h - sm.lr_lo[L][s];
                  sz += n;
                  if (n > bn) { bn = n; best = s; }
               }
               if (totexc && sz <= (uint32_t) LV_CAP)
               {
                  const bool hl = has_lo || L > 0, hh = has_hi || L + 1 < sm.nleaf;
                  sz += lv_count_exc(sm, recs, sm.lk_t[L], sm.lk_i[L], sm.lk_t[L + 1], sm.lk_i[L + 1], hl, hh);
               }
               if (sz > (uint32_t) LV_CAP) { bad = (int32_t) L; bs = best; bestn = bn; }
            }
            if (bad < 0) break;
            // no progress possible (the leaf is exceptions, or one key) -> exact v1 rerun
            if (sm.nleaf >= (uint32_t) LV_MAXLEAF || bestn < 2) { ok = false; break; }
            const uint32_t L = (uint32_t) bad;
            const uint32_t hL = (L + 1 < sm.nleaf) ? sm.lr_lo[L + 1][bs] : sm.hi[bs];
            const uint32_t mid = (sm.lr_lo[L][bs] + hL) / 2;
            const Rec mr = recs[sm.io.base[bs] + mid];
            for (uint32_t q = wv; q < (uint32_t) LV_IN; q += LV_T / 64)
            {
               if (q >= nin) continue;
               uint32_t v = mid;
               if (q != bs)
               {
                  const uint64_t sbase = sm.io.base[q] >> 6;
                  v = wave_lb(recs + sm.io.base[q], samp_t + sbase, samp_id + sbase, sm.nmain[q], mr.t, mr.id, lane);
               }
               if (lane == 0) sm.search[q] = v;
            }
            lv_bar();
            if (tid == 0)
            {
               for (uint32_t M = sm.nleaf; M > L + 1; M--)
                  for (uint32_t s = 0; s < (uint32_t) LV_IN; s++) sm.lr_lo[M][s] = sm.lr_lo[M - 1][s];
               for (uint32_t M = sm.nleaf + 1; M > L + 1; M--) { sm.lk_t[M] = sm.lk_t[M - 1]; sm.lk_i[M] = sm.lk_i[M - 1]; }
               sm.lk_t[L + 1] = mr.t;
               sm.lk_i[L + 1] = mr.id;
               for (uint32_t s = 0; s < (uint32_t) LV_IN; s++) sm.lr_lo[L + 1][s] = s < nin ? sm.search[s] : 0;
               sm.nleaf++;
            }
            lv_bar();
         }
         if (!ok)
         {
            if (tid == 0) atomicOr(errflag, 4u);
         }
         else
         {
            const uint32_t nleaf = sm.nleaf;
            uint32_t rhi[LV_IN];
#pragma unroll
            for (uint32_t s = 0; s < (uint32_t) LV_IN; s++) rhi[s] = sm.hi[s];
            for (uint32_t L = 0; L < nleaf; L++)
            {
               lv_bar();
#pragma unroll
               for (uint32_t s = 0; s < (uint32_t) LV_IN; s++)
                  if (tid == s)
                  {
                     sm.lo[s] = sm.lr_lo[L][s];
                     sm.hi[s] = (L + 1 < nleaf) ? sm.lr_lo[L + 1][s] : rhi[s];
                  }
               lv_bar();
               const bool hl = has_lo || L > 0, hh = has_hi || L + 1 < nleaf;
               lv_load_merge(sm, recs, sm.lk_t[L], sm.lk_i[L], sm.lk_t[L + 1], sm.lk_i[L + 1], hl, hh, true);
               if (j == 0 && L == 0)
               {
                  if (tid == 0 && c.analytical && (sm.E == 0 || LV_CYC(sm.kt[sm.perm[0]]) == 0)) sm.cy.mode = 1;
                  lv_bar();
               }
               lv_leaf<BC>(sm, c, recs, samp_t, samp_id, nexc, final_ps, errflag);
            }
         }
      }

      // ---- next chunk (if not prefetched), inclusive state (if not yet), per-port counters
      lv_bar();
      if (!fetched)
      {
         if (wv >= 1) lv_fetch<XL>(sm, false, anyexc, cb0, nch, cctr, cdesc, recs, samp_t, samp_id, nexc, done, errflag);
      }
      if (tid == 0)
      {
         if (!sm.published) lv_publish_inc(st, g, sm.cy);
         if (STAMPS && stamps)
         {
            stamps[(uint64_t) g * 16 + 8] = __builtin_amdgcn_s_memtime();
            stamps[(uint64_t) g * 16 + 9] = (uint64_t) j | ((uint64_t) sm.io.dir << 32) | ((uint64_t) level << 40);
            stamps[(uint64_t) g * 16 + 11] = __builtin_amdgcn_s_memrealtime();
            stamps[(uint64_t) g * 16 + 10] = sm.st_cnt;
            stamps[(uint64_t) g * 16 + 12] = sm.tm[1];
            stamps[(uint64_t) g * 16 + 13] = sm.tm[2];
            stamps[(uint64_t) g * 16 + 14] = sm.tm[3];
         }
         atomicAdd(&port_sum[sm.io.port], (unsigned long long) sm.st_sum);
         atomicAdd(&port_cnt[sm.io.port], (unsigned long long) sm.st_cnt);
         if (sm.st_mg1) atomicAdd(&port_mg1[sm.io.port], (unsigned long long) sm.st_mg1);
         if (sm.st_flit)
         {
            atomicAdd(&port_flit[sm.io.port], (unsigned long long) sm.st_flit);
            atomicMax(&port_last[sm.io.port], (unsigned long long) sm.st_last);
         }
      }
      if (XL)
      {
         // this chunk's records, samples and exception counts, released to the
         // consumer ports (MI355X_MICROARCH.md, inter-workgroup visibility):
         // every wave drains its stores, one lane releases at agent scope, then counts
         asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
         lv_bar();
         if (tid == 0)
         {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(&done[sm.pk], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
         }
      }
      lv_bar();
   }
}

#undef LV_CYC
#undef LV_PS
#if LV_GEN
}  // namespace lvg
#else
}  // namespace lvx
using namespace lvx;
// ---------------------------------------------------------------------------
// device-side plan
// ---------------------------------------------------------------------------
// One thread per port (level order): input slots, output slots, chunk count.
__global__ __launch_bounds__(256) void k_plan_ports(DevCfg c, uint32_t P, const uint32_t* __restrict__ lvl_ports,
                                                    const uint32_t* __restrict__ port_k,
                                                    const uint32_t* __restrict__ slot_cnt,
                                                    const uint64_t* __restrict__ slot_base, PortIO3* __restrict__ pio,
                                                    uint32_t* __restrict__ pnc, uint32_t ctgt, uint32_t klo0,
                                                    uint32_t khi0, uint32_t klo1, uint32_t khi1)
{
   const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
   if (k >= P) return;
   // ports outside [klo0, khi0) and [klo1, khi1) get no chunks (the chain engine runs
   // only the injection and SELF levels on k_level)
   const bool planned = (k >= klo0 && k < khi0) || (k >= klo1 && k < khi1);
   const uint32_t port = lvl_ports[k];
   PortIO3 io;
   const uint32_t tile = port / PORTS, dir = port % PORTS;
   io.port = port;
   io.dir = dir;
   io.nin = 0;
   io.sb = 0;
   uint32_t tot = 0, best = 0;
   for (uint32_t s = 0; s < (uint32_t) LV_IN; s++)
   {
      io.base[s] = 0; io.slot[s] = 0; io.cnt[s] = 0; io.prod[s] = LV_NO_PROD; io.prod_nc[s] = 0;
   }
   for (uint32_t in = 0; in < INS; in++)
   {
      const uint32_t sl = port * INS + in;
      const uint32_t n = slot_cnt[sl];
      if (n && io.nin < (uint32_t) LV_IN)
      {
         io.slot[io.nin] = sl;
         io.base[io.nin] = slot_base[sl];
         io.cnt[io.nin] = n;
         // the port that writes this slot (XY routing, emesh_hop_by_hop.cc:229-240)
         uint32_t pp = LV_NO_PROD;
         if (in == IN_LOCAL) pp = dir == P_INJ ? LV_NO_PROD : tile * PORTS + P_INJ;
         else if (in == IN_W) pp = (tile - 1) * PORTS + P_RIGHT;
         else if (in == IN_E) pp = (tile + 1) * PORTS + P_LEFT;
         else if (in == IN_S) pp = (tile - c.W) * PORTS + P_UP;
         else if (in == IN_N) pp = (tile + c.W) * PORTS + P_DOWN;
         // (a broadcast sender's own SELF record sits in the S slot of a row-0 tile:
         // no neighbour below, and the INJ port produced it -- XL is off for broadcasts)
         io.prod[io.nin] = (pp == LV_NO_PROD || pp >= c.N * PORTS) ? LV_NO_PROD : port_k[pp];
         io.prod_nc[io.nin] = 0;   // k_plan_expand: the producer's chunk count
         if (n > best) { best = n; io.sb = io.nin; }
         io.nin++;
         tot += n;
      }
   }
   uint32_t ntile = tile, nside = IN_LOCAL;
   if (dir == P_RIGHT) { ntile = tile + 1; nside = IN_W; }
   else if (dir == P_LEFT) { ntile = tile - 1; nside = IN_E; }
   else if (dir == P_UP) { ntile = tile + c.W; nside = IN_S; }
   else if (dir == P_DOWN) { ntile = tile - c.W; nside = IN_N; }
   io.nx = ntile % c.W;
   io.ny = ntile / c.W;
   for (uint32_t d = 0; d < 5; d++)
   {
      const uint32_t os = slot_of(ntile, d, slot_side(d, nside));
      io.oslot[d] = os;
      io.obase[d] = dir == P_SELF ? 0 : slot_base[os];
      io.ocnt[d] = dir == P_SELF ? 0 : slot_cnt[os];
   }
   io.gbase = 0;
   io.nc = 0;     // k_plan_scan decides, k_plan_expand writes
   io.pk = k;
   io.rl = (uint32_t) rl_of(c, tile);
   io.pad1 = io.pad2 = 0;
   pio[k] = io;
   pnc[k] = planned ? tot : 0u;  // records of the port (k_plan_scan turns it into a chunk count)
}

// One block per level.  Records -> chunk counts.  A level runs in rounds of the
// persistent grid and ends with its slowest round, so the chunk size is chosen
// per level to make the chunk count just fit a whole number of rounds:
// rounds = round(records / (ctgt * grid)) (at least 1), then the smallest size c
// with sum over ports of ceil(records_p / c) <= rounds * grid, kept within
// [LV_CMIN, LV_CMAX] (LDS holds LV_CAP records per leaf).
#ifndef LV_CMAX
#define LV_CMAX 1700
#endif
#ifndef LV_CMIN
#define LV_CMIN 384
#endif
#ifndef LV_ROUNDS_FIT
#define LV_ROUNDS_FIT 1   // 1: fit levels of at most LV_FIT_MAX grid rounds (at ctgt); 2: every level; 0: off
#endif
#ifndef LV_FIT_MAX
#define LV_FIT_MAX 5      // in halves of a grid round: 5 = levels of up to 2.5 rounds
#endif
__global__ __launch_bounds__(1024) void k_plan_guided(const uint32_t* __restrict__ lvl_off, uint32_t* __restrict__ pnc,
                                                      uint32_t ctgt, uint64_t grid)
{
   __shared__ uint64_t part[1024];
   __shared__ uint32_t pcnt[1024];
   __shared__ uint32_t csel;
   const uint32_t l = blockIdx.x;
   const uint32_t a = lvl_off[l], b = lvl_off[l + 1], np = b - a;
   const uint32_t per = (np + 1023) / 1024;
   const uint32_t lo = a + min(threadIdx.x * per, np), hi = a + min((threadIdx.x + 1) * per, np);
   uint64_t s = 0;
   uint32_t nz = 0;
   for (uint32_t i = lo; i < hi; i++) { s += pnc[i]; nz += pnc[i] != 0; }
   part[threadIdx.x] = s;
   pcnt[threadIdx.x] = nz;
   __syncthreads();
   for (uint32_t off = 512; off > 0; off >>= 1)
   {
      if (threadIdx.x < off)
      {
         part[threadIdx.x] += part[threadIdx.x + off];
         pcnt[threadIdx.x] += pcnt[threadIdx.x + off];
      }
      __syncthreads();
   }
   if (threadIdx.x == 0)
   {
      const uint64_t R = part[0], P = pcnt[0];
      uint32_t c = ctgt;
      // Fitting every level costs 32x32 (2-3 rounds per level) 7%; levels of about
      // one round (a mesh sharded over 4-8 ranks) gain 7-14%: a second round of a
      // few chunks costs a whole chunk latency.
      const uint64_t nat = R / ctgt + P;   // chunks at the target size (about)
      if (LV_ROUNDS_FIT && R > 0 && (LV_ROUNDS_FIT > 1 || 2 * nat <= (uint64_t) LV_FIT_MAX * grid))
      {
         uint64_t rounds = (R + ctgt * grid / 2) / (ctgt * grid);
         if (rounds < 1) rounds = 1;
         for (;; rounds++)
         {
            const uint64_t slots = rounds * grid;
            if (slots <= P) continue;
            const uint64_t cc = (R + slots - P - 1) / (slots - P);
            if (cc <= LV_CMAX) { c = (uint32_t) (cc < LV_CMIN ? LV_CMIN : cc); break; }
         }
      }
      csel = c;
   }
   __syncthreads();
   const uint32_t c = csel;
   for (uint32_t i = lo; i < hi; i++)
   {
      const uint32_t tot = pnc[i];
      pnc[i] = tot ? (tot + c - 1) / c : 0;
   }
}

// Single block: global exclusive scan of chunk counts (ports are in level
// order), per-level chunk bases.
__global__ __launch_bounds__(1024) void k_plan_scan(uint32_t P, uint32_t L, const uint32_t* __restrict__ lvl_off,
                                                    const uint32_t* __restrict__ pnc, uint32_t* __restrict__ pgb,
                                                    uint32_t* __restrict__ lvl_cbase)
{
   __shared__ uint64_t part[1024];
   const uint32_t per = (P + 1023) / 1024;
   const uint32_t lo = threadIdx.x * per, hi = min(lo + per, P);
   uint64_t s = 0;
   for (uint32_t i = lo; i < hi; i++) s += pnc[i];
   part[threadIdx.x] = s;
   __syncthreads();
   for (uint32_t off = 1; off < 1024; off <<= 1)
   {
      const uint64_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
   }
   uint32_t run = (uint32_t) (part[threadIdx.x] - s);
   for (uint32_t i = lo; i < hi; i++) { pgb[i] = run; run += pnc[i]; }
   __syncthreads();
   for (uint32_t l = threadIdx.x; l <= L; l += 1024) lvl_cbase[l] = l < L ? pgb[lvl_off[l]] : (uint32_t) part[1023];
}

// Look-back state of the chunks this run uses (the count is known on device only).
__global__ __launch_bounds__(256) void k_zero_state(const uint32_t* __restrict__ lvl_cbase, uint32_t L,
                                                    uint64_t* __restrict__ st)
{
   const uint64_t n = (uint64_t) lvl_cbase[L] * LV_STATE_WORDS;
   for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x)
      st[i] = 0;
}

// One wave per level: split the level's chunks into LV_QUEUES port-aligned
// ranges of about equal size (a port's chunks never straddle two queues).
__global__ __launch_bounds__(64) void k_plan_queues(const uint32_t* __restrict__ lvl_off,
                                                    const uint32_t* __restrict__ pgb,
                                                    const uint32_t* __restrict__ lvl_cbase, uint32_t* __restrict__ lvl_qb,
                                                    uint32_t grid)
{
   const uint32_t l = blockIdx.x, q = threadIdx.x;
   const uint32_t a = lvl_off[l], b = lvl_off[l + 1];
   const uint32_t cb = lvl_cbase[l], T = lvl_cbase[l + 1] - cb;
   if (q == LV_QUEUES + 1)
   {
      // measured (32x32 vs 64x64): prefetching during the look-back pays while a level
      // is a few grid rounds; over many rounds the held chunks build a convoy
      lvl_qb[l * LV_QB + q] = T > (uint64_t) LV_LATE_ROUNDS * grid ? 1u : 0u;
      return;
   }
   if (q > LV_QUEUES) return;
   const uint32_t target = (uint32_t) (((uint64_t) q * T) / LV_QUEUES);
   // first port k of the level with pgb[k] - cb >= target
   uint32_t lo = a, hi = b;
   while (lo < hi)
   {
      const uint32_t m = (lo + hi) / 2;
      if (pgb[m] - cb >= target) hi = m;
      else lo = m + 1;
   }
   lvl_qb[l * LV_QB + q] = q == LV_QUEUES || lo == b ? T : pgb[lo] - cb;
}

__global__ __launch_bounds__(256) void k_plan_expand(uint32_t P, PortIO3* __restrict__ pio, const uint32_t* __restrict__ pnc,
                                                     const uint32_t* __restrict__ pgb)
{
   const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
   if (k >= P) return;
   pio[k].gbase = pgb[k];
   pio[k].nc = pnc[k];
   for (uint32_t s = 0; s < (uint32_t) LV_IN; s++)
      if (pio[k].prod[s] != LV_NO_PROD) pio[k].prod_nc[s] = pnc[pio[k].prod[s]];
}

// One wave per port: every chunk gets its own copy of the port descriptor, so
// a dequeue is one dependent load (chunk id -> descriptor) instead of two.
__global__ __launch_bounds__(64) void k_plan_fill(const PortIO3* __restrict__ pio, PortIO3* __restrict__ cdesc)
{
   const uint32_t k = blockIdx.x, lane = threadIdx.x;
   constexpr uint32_t WORDS = sizeof(PortIO3) / 4;
   const uint32_t* src = reinterpret_cast<const uint32_t*>(pio + k);
   const uint32_t v = lane < WORDS ? src[lane] : 0u;
   const uint32_t gb = pio[k].gbase, nc = pio[k].nc;
   for (uint32_t j = 0; j < nc; j++)
      if (lane < WORDS) reinterpret_cast<uint32_t*>(cdesc + gb + j)[lane] = v;
}

#endif
}  // namespace gnoc
#undef LV_GEN
