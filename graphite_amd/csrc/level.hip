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
//   2. load the ranges (16-B records) into LDS; merge by galloping
//      co-iteration (rank = own index + lower bounds in the other inputs)
//   3. block max-plus scan of the chunk: element map X -> max(X + F, t + F),
//      composition (a1,b1).(a2,b2) = (a1 + a2, max(b1 + a2, b2)), plus per
//      next-direction record counts (output positions)
//   4. decoupled look-back over the port's earlier chunks for the carried queue
//      state (aggregate published first, inclusive state right after)
//   5. recurrence per thread segment, departure times written back into LDS
//   6. output pass, lanes over consecutive merged positions, so each wave's
//      records for one next direction land at consecutive HBM addresses
// Only f == 1 GHz and max_list_size >= 3 take this path (engine.hip).
#include "common.h"

namespace gnoc {

constexpr int LV_T = 256;          // threads per workgroup
constexpr int LV_CAP = 2048;       // records one leaf holds in LDS
constexpr int LV_IN = 4;           // input slots per port (SELF, UP, DOWN have 4)
constexpr int LV_SEG = LV_IN + 1;  // + the exception segment
constexpr int LV_MAXLEAF = 32;     // leaves per chunk (bursts); beyond -> errflag, v1 rerun
constexpr uint32_t LV_CTGT = 1200; // target records per chunk
constexpr uint32_t LV_SPIN_LIMIT = 1u << 24;

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
};
static_assert(sizeof(PortIO3) % 16 == 0, "PortIO3 copy granularity");

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
   Rec r[LV_CAP];
   uint16_t perm[LV_CAP];
   PortIO3 io;
   Carry3 cy;
   uint64_t wA[LV_T / 64], wB[LV_T / 64], wC[LV_T / 64];
   uint64_t st_sum;
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
};

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lv_ld_flag(const uint32_t* p)
{
   return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lv_ld(const uint64_t* p)
{
   return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lv_st(uint64_t* p, uint64_t v)
{
   __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool rlt(const Rec& a, uint64_t t, uint32_t id)
{
   return a.t < t || (a.t == t && a.id < id);
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

// lower bound of (t,id) in LDS records [lo, hi)
__device__ __forceinline__ uint32_t lds_lb(const Rec* __restrict__ r, uint32_t lo, uint32_t hi, uint64_t t, uint32_t id)
{
   while (lo < hi)
   {
      const uint32_t mid = (lo + hi) >> 1;
      if (rlt(r[mid], t, id)) lo = mid + 1;
      else hi = mid;
   }
   return lo;
}

// lower bound of (t,id) in [lo, end), knowing every record before lo is smaller
__device__ __forceinline__ uint32_t lds_gallop(const Rec* __restrict__ r, uint32_t lo, uint32_t end, uint64_t t,
                                               uint32_t id)
{
   uint32_t step = 1, hi;
   for (;;)
   {
      const uint32_t pr = lo + step - 1;
      if (pr >= end) { hi = end; break; }
      if (!rlt(r[pr], t, id)) { hi = pr; break; }
      lo = pr + 1;
      step <<= 1;
   }
   return lds_lb(r, lo, hi, t, id);
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

// Exceptions of the port's inputs whose key lies in [klo, khi): exact count
// (block-wide; the exception tails are short).
__device__ uint32_t lv_count_exc(LvSmem& sm, const Rec* __restrict__ recs, uint64_t klo_t, uint32_t klo_i,
                                 uint64_t khi_t, uint32_t khi_i, bool has_lo, bool has_hi)
{
   const uint32_t tid = threadIdx.x;
   __syncthreads();
   if (tid == 0) sm.nexc_leaf = 0;
   __syncthreads();
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
   __syncthreads();
   const uint32_t n = sm.nexc_leaf;
   __syncthreads();
   return n;
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
   __syncthreads();
   for (uint32_t s = 0; s < nin; s++)
   {
      const Rec* r = recs + sm.io.base[s] + sm.lo[s];
      const uint32_t L = sm.len[s], o = sm.off[s];
      for (uint32_t i = tid; i < L; i += LV_T) sm.r[o + i] = r[i];
   }
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
               if (o + k < (uint32_t) LV_CAP) sm.r[o + k] = v;
            }
         }
      }
      __syncthreads();
      const uint32_t ne = min(sm.nexc_leaf, (uint32_t) LV_CAP - o);
      // odd-even transposition sort of the (few) exceptions
      for (uint32_t ph = 0; ph < ne; ph++)
      {
         for (uint32_t i = 2 * tid + (ph & 1); i + 1 < ne; i += 2 * LV_T)
         {
            const Rec a = sm.r[o + i], b = sm.r[o + i + 1];
            if (rlt(b, a.t, a.id)) { sm.r[o + i] = b; sm.r[o + i + 1] = a; }
         }
         __syncthreads();
      }
      if (tid == 0) sm.len[LV_IN] = ne;
   }
   __syncthreads();
   // merge: rank = own index + lower bounds in every other segment
   uint32_t off[LV_SEG], end[LV_SEG], p[LV_SEG];
#pragma unroll
   for (int s = 0; s < LV_SEG; s++)
   {
      off[s] = sm.off[s];
      end[s] = off[s] + sm.len[s];
      p[s] = off[s];
   }
   const uint32_t E = end[LV_SEG - 1];
   const uint32_t per = (E + LV_T - 1) / LV_T;
   const uint32_t k0 = min(tid * per, E), k1 = min(k0 + per, E);
   int cur = -1;
   for (uint32_t k = k0; k < k1; k++)
   {
      int s = 0;
#pragma unroll
      for (int q = 0; q < LV_SEG - 1; q++) s += (k >= end[q]) ? 1 : 0;
      const Rec me = sm.r[k];
      uint32_t own = k;
#pragma unroll
      for (int q = 0; q < LV_SEG; q++) own -= (q == s) ? off[q] : 0u;
      uint32_t rank = own;
#pragma unroll
      for (int o = 0; o < LV_SEG; o++)
      {
         if (o == s || off[o] == end[o]) continue;
         const uint32_t q = (s != cur) ? lds_lb(sm.r, off[o], end[o], me.t, me.id)
                                       : lds_gallop(sm.r, p[o], end[o], me.t, me.id);
         p[o] = q;
         rank += q - off[o];
      }
      cur = s;
      sm.perm[rank] = (uint16_t) k;
   }
   if (tid == 0) sm.E = E;
   __syncthreads();
}

// ---------------------------------------------------------------------------
// block scan of merged positions [s0, E): per-thread contiguous segments
// ---------------------------------------------------------------------------
struct Scan3
{
   uint64_t eA, eB, eC;   // exclusive prefix of this thread
   uint64_t tA, tB, tC;   // block totals
};

__device__ __forceinline__ void lv_seg(uint32_t s0, uint32_t E, uint32_t& a, uint32_t& b)
{
   const uint32_t cnt = E - s0;
   const uint32_t per = (cnt + LV_T - 1) / LV_T;
   a = s0 + min(threadIdx.x * per, cnt);
   b = s0 + min((threadIdx.x + 1) * per, cnt);
}

__device__ Scan3 lv_scan(LvSmem& sm, uint32_t s0, uint32_t E)
{
   const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
   const uint32_t dir = sm.io.dir, nx = sm.io.nx, ny = sm.io.ny;
   uint32_t a, b;
   lv_seg(s0, E, a, b);
   uint64_t A = 0, B = 0, C = 0;
   for (uint32_t e = a; e < b; e++)
   {
      const Rec rc = sm.r[sm.perm[e]];
      const uint64_t p = aux_F(rc.aux);
      mp_comp(A, B, p, cyc1(rc.t) + p);
      C += 1ull << (12 * next_dir(rc.aux, dir, nx, ny));
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
   __syncthreads();
   if (lane == 63) { sm.wA[wv] = iA; sm.wB[wv] = iB; sm.wC[wv] = iC; }
   __syncthreads();
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

// ---------------------------------------------------------------------------
// process a merged leaf from carry sm.cy; write outputs; advance sm.cy
// ---------------------------------------------------------------------------
__device__ void lv_process(LvSmem& sm, const DevCfg& c, bool have_scan, Scan3 so, Rec* __restrict__ recs,
                           uint64_t* __restrict__ samp_t, uint32_t* __restrict__ samp_id, uint32_t* __restrict__ nexc,
                           uint64_t* __restrict__ final_ps, unsigned* __restrict__ errflag)
{
   const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
   const uint32_t E = sm.E;
   const uint32_t dir = sm.io.dir, nx = sm.io.nx, ny = sm.io.ny;
   const uint64_t rl = dir == P_INJ ? 0ull : c.rl_ps;
   // ---- serial prefix while the queue has never idled (history tree + M/G/1)
   if (sm.cy.mode)
   {
      if (tid == 0)
      {
         SerialState s;
         s.X = sm.cy.X; s.g = (int) sm.cy.g; s.mode = 1; s.s1 = sm.cy.s1; s.s2 = sm.cy.s2;
         s.narr = sm.cy.narr; s.newest = sm.cy.newest; s.mg1 = 0;
         uint32_t e = 0;
         uint64_t ssum = 0;
         for (; e < E && s.mode; e++)
         {
            const Rec rc = sm.r[sm.perm[e]];
            const uint64_t mg_before = s.mg1;
            const uint64_t cc = serial_step(s, cyc1(rc.t), aux_F(rc.aux), c.max_list, c.analytical);
            if (s.g >= 1) s.mode = 0;
            ssum += cc;
            const uint64_t tn = rc.t + cc * 1000ull + rl;
            if (dir == P_SELF) { final_ps[rc.id] = tn + 1000ull * aux_F(rc.aux); continue; }
            const uint32_t nd = next_dir(rc.aux, dir, nx, ny);
            Rec o;
            o.t = tn;
            o.id = rc.id;
            o.aux = rc.aux;
            if (s.mg1 != mg_before)
            {
               // M/G/1-served: may leave FIFO order -> exception tail of the slot
               const uint32_t x = atomicAdd(&nexc[sm.io.oslot[nd]], 1u);
               if (x >= sm.io.ocnt[nd]) { atomicOr(errflag, 1u); continue; }
               recs[sm.io.obase[nd] + sm.io.ocnt[nd] - 1 - x] = o;
            }
            else
            {
               const uint32_t pos = sm.cy.cnt[nd]++;
               if (pos >= sm.io.ocnt[nd]) { atomicOr(errflag, 1u); continue; }
               recs[sm.io.obase[nd] + pos] = o;
               if ((pos & 63) == 0)
               {
                  samp_t[(sm.io.obase[nd] + pos) >> 6] = tn;
                  samp_id[(sm.io.obase[nd] + pos) >> 6] = rc.id;
               }
            }
         }
         sm.s0 = e;
         sm.cy.X = s.X; sm.cy.g = (uint32_t) s.g; sm.cy.mode = s.mode; sm.cy.s1 = s.s1; sm.cy.s2 = s.s2;
         sm.cy.narr = s.narr; sm.cy.newest = s.newest;
         sm.st_sum += ssum;
         sm.st_cnt += e;
         sm.st_mg1 += (uint32_t) s.mg1;
      }
      __syncthreads();
      have_scan = false;
   }
   else if (tid == 0)
   {
      sm.s0 = 0;
   }
   __syncthreads();
   const uint32_t s0 = sm.s0;
   if (!have_scan) so = lv_scan(sm, s0, E);
   const uint64_t X0 = sm.cy.X;
   // ---- recurrence per thread segment; departure time back into LDS
   uint32_t a, b;
   lv_seg(s0, E, a, b);
   {
      uint64_t X = X0 + so.eA;
      X = X > so.eB ? X : so.eB;
      uint64_t ssum = 0;
      for (uint32_t e = a; e < b; e++)
      {
         const uint32_t k = sm.perm[e];
         const uint64_t t = sm.r[k].t;
         const uint64_t tc = cyc1(t);
         const uint64_t cc = X > tc ? X - tc : 0;
         X = (X > tc ? X : tc) + aux_F(sm.r[k].aux);
         ssum += cc;
         sm.r[k].t = t + cc * 1000ull + rl;
      }
      for (int off = 32; off > 0; off >>= 1) ssum += __shfl_down(ssum, off);
      if (lane == 0 && ssum) atomicAdd((unsigned long long*) &sm.st_sum, (unsigned long long) ssum);
   }
   __syncthreads();
   // ---- output pass: wave w owns the merged range of its 64 threads' segments
   {
      const uint32_t cnt = E - s0;
      const uint32_t per = (cnt + LV_T - 1) / LV_T;
      const uint32_t wa = s0 + min(wv * 64 * per, cnt), wb = s0 + min((wv + 1) * 64 * per, cnt);
      const uint64_t wpre = __shfl(so.eC, 0);   // counts before this wave's range
      const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
      uint32_t run[5] = { 0, 0, 0, 0, 0 };
      for (uint32_t e0 = wa; e0 < wb; e0 += 64)
      {
         const uint32_t e = e0 + lane;
         const bool valid = e < wb;
         Rec rc;
         rc.t = 0; rc.id = 0; rc.aux = 0;
         if (valid) rc = sm.r[sm.perm[e]];
         if (dir == P_SELF)
         {
            // NetworkModel::processReceivedPacket: + serialization (network_model.cc:142-150)
            if (valid) final_ps[rc.id] = rc.t + 1000ull * aux_F(rc.aux);
            continue;
         }
         const uint32_t nd = next_dir(rc.aux, dir, nx, ny);
         uint32_t pos = 0;
#pragma unroll
         for (uint32_t d = 0; d < 5; d++)
         {
            const uint64_t m = __ballot(valid && nd == d);
            if (nd == d) pos = sm.cy.cnt[d] + cfield(wpre, d) + run[d] + (uint32_t) __popcll(m & lt);
            run[d] += (uint32_t) __popcll(m);
         }
         if (valid && pos >= sm.io.ocnt[nd])
         {
            atomicOr(errflag, 1u);   // route-count invariant broken: never write outside the slot
         }
         else if (valid)
         {
            const uint64_t gp = sm.io.obase[nd] + pos;
            recs[gp] = rc;
            if ((gp & 63) == 0)
            {
               samp_t[gp >> 6] = rc.t;
               samp_id[gp >> 6] = rc.id;
            }
         }
      }
   }
   __syncthreads();
   if (tid == 0)
   {
      sm.st_cnt += E - s0;
      const uint64_t nx0 = X0 + so.tA;
      sm.cy.X = nx0 > so.tB ? nx0 : so.tB;
      for (uint32_t d = 0; d < 5; d++) sm.cy.cnt[d] += cfield(so.tC, d);
   }
   __syncthreads();
}

// ---------------------------------------------------------------------------
// decoupled look-back (wave 0): state layout per chunk (16 x u64)
//   [0] A  [1] B  [2] aggregate counts (5 x 12 bit)
//   [3] cnt0|cnt1<<32  [4] cnt2|cnt3<<32  [5] cnt4  [6] X  [7] mode|g<<32
//   [8] s1  [9] s2  [10] narr  [11] newest
// flags: 1 = aggregate published, 2 = inclusive state published
// ---------------------------------------------------------------------------
__device__ void lv_publish_agg(uint64_t* __restrict__ st, uint32_t* __restrict__ flags, uint32_t g, const Scan3& so)
{
   uint64_t* w = st + (uint64_t) g * 16;
   lv_st(w + 0, so.tA);
   lv_st(w + 1, so.tB);
   lv_st(w + 2, so.tC);
   asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
   __hip_atomic_store(&flags[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void lv_publish_inc(uint64_t* __restrict__ st, uint32_t* __restrict__ flags, uint32_t g, const Carry3& cy)
{
   uint64_t* w = st + (uint64_t) g * 16;
   lv_st(w + 3, (uint64_t) cy.cnt[0] | ((uint64_t) cy.cnt[1] << 32));
   lv_st(w + 4, (uint64_t) cy.cnt[2] | ((uint64_t) cy.cnt[3] << 32));
   lv_st(w + 5, (uint64_t) cy.cnt[4]);
   lv_st(w + 6, cy.X);
   lv_st(w + 7, (uint64_t) cy.mode | ((uint64_t) cy.g << 32));
   lv_st(w + 8, (uint64_t) __double_as_longlong(cy.s1));
   lv_st(w + 9, (uint64_t) __double_as_longlong(cy.s2));
   lv_st(w + 10, cy.narr);
   lv_st(w + 11, cy.newest);
   asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
   __hip_atomic_store(&flags[g], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ bool lv_lookback(LvSmem& sm, uint32_t gbase, uint32_t j, const uint32_t* __restrict__ flags,
                            const uint64_t* __restrict__ st, unsigned* __restrict__ errflag)
{
   const uint32_t lane = threadIdx.x & 63;
   uint64_t accA = 0, accB = 0;
   uint32_t accC[5] = { 0, 0, 0, 0, 0 };
   int32_t look = (int32_t) j - 1;
   uint32_t spins = 0;
   for (;;)
   {
      const int32_t ck = look - (int32_t) lane;
      uint32_t f = 2;
      if (ck >= 0) f = lv_ld_flag(&flags[gbase + ck]);
      const uint64_t inc = __ballot(ck >= 0 && f == 2);
      const uint64_t zero = __ballot(ck >= 0 && f == 0);
      const uint64_t stop = inc | __ballot(ck < 0);
      const int L = stop ? __ffsll((long long) stop) - 1 : 64;
      const uint64_t need = L >= 64 ? ~0ull : ((1ull << L) - 1);
      if (zero & need)
      {
         if (++spins > LV_SPIN_LIMIT) { if (lane == 0) atomicOr(errflag, 2u); return false; }
         __builtin_amdgcn_s_sleep(1);
         continue;
      }
      uint64_t a = 0, b = 0, q = 0;
      if ((int) lane < L)
      {
         const uint64_t* w = st + (uint64_t) (gbase + ck) * 16;
         a = lv_ld(w + 0);
         b = lv_ld(w + 1);
         q = lv_ld(w + 2);
      }
      // compose in chunk order: earliest (lane L-1) first ... lane 0 last, then the tail so far
      uint64_t wa = 0, wb = 0;
      for (int l = L - 1; l >= 0; l--) mp_comp(wa, wb, __shfl(a, l), __shfl(b, l));
      mp_comp(wa, wb, accA, accB);
      accA = wa;
      accB = wb;
#pragma unroll
      for (uint32_t d = 0; d < 5; d++)
      {
         uint32_t v = (int) lane < L ? cfield(q, d) : 0u;
         for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
         accC[d] += v;
      }
      if (L < 64)
      {
         const int32_t sc = look - L;   // chunk holding an inclusive state (chunk 0 always publishes one)
         const uint64_t* w = st + (uint64_t) (gbase + sc) * 16;
         const uint32_t mode = (uint32_t) (lv_ld(w + 7) & 0xFFFFFFFFull);
         if (mode && sc != (int32_t) j - 1)
         {
            // the queue was still in its serial prefix: FIFO aggregates after it are invalid;
            // wait for the immediate predecessor's inclusive state instead.
            const uint32_t pj = gbase + j - 1;
            while (lv_ld_flag(&flags[pj]) != 2)
            {
               if (++spins > LV_SPIN_LIMIT) { if (lane == 0) atomicOr(errflag, 2u); return false; }
               __builtin_amdgcn_s_sleep(1);
            }
            w = st + (uint64_t) pj * 16;
            accA = 0;
            accB = 0;
            for (int d = 0; d < 5; d++) accC[d] = 0;
         }
         if (lane == 0)
         {
            const uint64_t X = lv_ld(w + 6);
            const uint64_t mg = lv_ld(w + 7);
            const uint64_t c01 = lv_ld(w + 3), c23 = lv_ld(w + 4), c4 = lv_ld(w + 5);
            const uint64_t nx = X + accA;
            sm.cy.X = nx > accB ? nx : accB;
            sm.cy.mode = (uint32_t) (mg & 0xFFFFFFFFull);
            sm.cy.g = (uint32_t) (mg >> 32);
            sm.cy.s1 = __longlong_as_double((long long) lv_ld(w + 8));
            sm.cy.s2 = __longlong_as_double((long long) lv_ld(w + 9));
            sm.cy.narr = lv_ld(w + 10);
            sm.cy.newest = lv_ld(w + 11);
            sm.cy.cnt[0] = (uint32_t) (c01 & 0xFFFFFFFFull) + accC[0];
            sm.cy.cnt[1] = (uint32_t) (c01 >> 32) + accC[1];
            sm.cy.cnt[2] = (uint32_t) (c23 & 0xFFFFFFFFull) + accC[2];
            sm.cy.cnt[3] = (uint32_t) (c23 >> 32) + accC[3];
            sm.cy.cnt[4] = (uint32_t) c4 + accC[4];
         }
         return true;
      }
      look -= 64;
   }
}

// ---------------------------------------------------------------------------
// the level kernel: a persistent grid pulls the level's chunks in order
// ---------------------------------------------------------------------------
#define LV_STAMP(k)                                                                                          \
   do                                                                                                       \
   {                                                                                                        \
      if (STAMPS && stamps && tid == 0) stamps[(uint64_t) g * 16 + (k)] = __builtin_amdgcn_s_memtime();     \
   } while (0)

template <bool STAMPS>
__global__ __launch_bounds__(LV_T) void k_level(DevCfg c, uint32_t level, const uint32_t* __restrict__ lvl_cbase,
                                                unsigned* __restrict__ ctr, const uint32_t* __restrict__ chunk_port,
                                                const PortIO3* __restrict__ pio, Rec* __restrict__ recs,
                                                uint64_t* __restrict__ samp_t, uint32_t* __restrict__ samp_id,
                                                uint32_t* __restrict__ nexc, uint32_t* __restrict__ flags,
                                                uint64_t* __restrict__ st, uint64_t* __restrict__ final_ps,
                                                unsigned long long* __restrict__ port_sum,
                                                unsigned long long* __restrict__ port_cnt,
                                                unsigned long long* __restrict__ port_mg1, unsigned* __restrict__ errflag,
                                                uint64_t* __restrict__ stamps)
{
   __shared__ LvSmem sm;
   const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
   const uint32_t cb0 = lvl_cbase[level];
   const uint32_t nch = lvl_cbase[level + 1] - cb0;
   for (;;)
   {
      __syncthreads();
      if (tid == 0)
      {
         const uint32_t cid = atomicAdd(&ctr[level], 1u);   // in order: every predecessor chunk is running
         sm.g = cb0 + cid;
         sm.j = cid < nch ? 1u : 0u;   // temporarily: "valid"
         sm.st_sum = 0;
         sm.st_cnt = 0;
         sm.st_mg1 = 0;
         sm.published = 0;
      }
      __syncthreads();
      if (!sm.j) return;
      const uint32_t g = sm.g;
      LV_STAMP(0);
      const uint32_t pk = chunk_port[g];
      {
         const uint32_t* srcw = reinterpret_cast<const uint32_t*>(pio + pk);
         uint32_t* dstw = reinterpret_cast<uint32_t*>(&sm.io);
         for (uint32_t k = tid; k < (uint32_t) (sizeof(PortIO3) / 4); k += LV_T) dstw[k] = srcw[k];
      }
      __syncthreads();
      const uint32_t j = g - sm.io.gbase, nc = sm.io.nc;
      const uint32_t nin = sm.io.nin;
      if (tid < nin)
      {
         const uint32_t x = nexc[sm.io.slot[tid]];
         sm.nxe[tid] = x;
         sm.nmain[tid] = sm.io.cnt[tid] - x;
      }
      if (tid == 0)
      {
         sm.j = j;
         sm.cy.X = 0; sm.cy.mode = 0; sm.cy.g = 0; sm.cy.s1 = 0; sm.cy.s2 = 0; sm.cy.narr = 0; sm.cy.newest = 0;
         for (int k = 0; k < 5; k++) sm.cy.cnt[k] = 0;
      }
      __syncthreads();
      LV_STAMP(1);

      // ---- chunk key range: exact index split of the largest input
      const uint32_t sb = sm.io.sb;
      const uint32_t nb = sm.nmain[sb];
      bool has_lo = j > 0, has_hi = j + 1 < nc, empty = false;
      if (nb == 0) { empty = j > 0; has_lo = has_hi = false; }   // only exceptions: chunk 0 takes all
      const uint32_t ilo = (uint32_t) (((uint64_t) j * nb) / nc);
      const uint32_t ihi = (uint32_t) (((uint64_t) (j + 1) * nb) / nc);
      uint64_t klo_t = 0, khi_t = ~0ull;
      uint32_t klo_i = 0, khi_i = ~0u;
      if (has_lo) { const Rec r = recs[sm.io.base[sb] + ilo]; klo_t = r.t; klo_i = r.id; }
      if (has_hi) { const Rec r = recs[sm.io.base[sb] + ihi]; khi_t = r.t; khi_i = r.id; }

      LV_STAMP(2);
      // ---- main ranges of the other inputs (waves search in parallel)
      for (uint32_t q = wv; q < 2 * (uint32_t) LV_IN; q += LV_T / 64)
      {
         const uint32_t s = q >> 1, which = q & 1;
         if (s >= nin) continue;
         uint32_t v;
         if (empty) v = 0;
         else if (s == sb) v = which ? (has_hi ? ihi : nb) : (has_lo ? ilo : 0);
         else if (which == 0 && !has_lo) v = 0;
         else if (which == 1 && !has_hi) v = sm.nmain[s];
         else
         {
            const uint64_t sbase = sm.io.base[s] >> 6;
            v = wave_lb(recs + sm.io.base[s], samp_t + sbase, samp_id + sbase, sm.nmain[s], which ? khi_t : klo_t,
                        which ? khi_i : klo_i, lane);
         }
         if (lane == 0) sm.search[q] = v;
      }
      __syncthreads();
      uint32_t total = 0, totexc = 0;
      uint32_t rlo[LV_IN], rhi[LV_IN];
#pragma unroll
      for (uint32_t s = 0; s < (uint32_t) LV_IN; s++)
      {
         rlo[s] = s < nin ? sm.search[2 * s] : 0;
         rhi[s] = s < nin ? sm.search[2 * s + 1] : 0;
         total += rhi[s] - rlo[s];
         totexc += s < nin ? sm.nxe[s] : 0;
      }
      LV_STAMP(3);
      if (empty) totexc = 0;
      if (totexc) totexc = lv_count_exc(sm, recs, klo_t, klo_i, khi_t, khi_i, has_lo, has_hi);

      if (total + totexc <= (uint32_t) LV_CAP)
      {
         // ---------------- single leaf
         if (tid < (uint32_t) LV_IN) { sm.lo[tid] = rlo[tid]; sm.hi[tid] = rhi[tid]; }
         __syncthreads();
         lv_load_merge(sm, recs, klo_t, klo_i, khi_t, khi_i, has_lo, has_hi, !empty);
         LV_STAMP(4);
         if (j == 0)
         {
            if (tid == 0 && c.analytical && sm.E > 0 && cyc1(sm.r[sm.perm[0]].t) == 0) sm.cy.mode = 1;
            __syncthreads();
         }
         bool have = false;
         Scan3 so;
         so.eA = so.eB = so.eC = so.tA = so.tB = so.tC = 0;
         if (j > 0 || !sm.cy.mode)
         {
            so = lv_scan(sm, 0, sm.E);
            have = true;
            LV_STAMP(5);
            if (j > 0)
            {
               if (tid == 0) lv_publish_agg(st, flags, g, so);
               if (wv == 0) lv_lookback(sm, sm.io.gbase, j, flags, st, errflag);
               __syncthreads();
            }
            LV_STAMP(6);
            // FIFO: the inclusive state is (carry) x (aggregate); publish before the outputs
            if (tid == 0 && !sm.cy.mode)
            {
               Carry3 inc = sm.cy;
               const uint64_t nx0 = inc.X + so.tA;
               inc.X = nx0 > so.tB ? nx0 : so.tB;
               for (uint32_t d = 0; d < 5; d++) inc.cnt[d] += cfield(so.tC, d);
               lv_publish_inc(st, flags, g, inc);
               sm.published = 1;
            }
            __syncthreads();
         }
         lv_process(sm, c, have, so, recs, samp_t, samp_id, nexc, final_ps, errflag);
         LV_STAMP(7);
      }
      else
      {
         // ---------------- burst: split the key range into leaves that fit LDS
         if (j > 0 && wv == 0) lv_lookback(sm, sm.io.gbase, j, flags, st, errflag);
         if (tid == 0)
         {
            sm.nleaf = 1;
            sm.lk_t[0] = klo_t; sm.lk_i[0] = klo_i;
            sm.lk_t[1] = khi_t; sm.lk_i[1] = khi_i;
            for (uint32_t s = 0; s < (uint32_t) LV_IN; s++) sm.lr_lo[0][s] = rlo[s];
         }
         __syncthreads();
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
                  const uint32_t h = (L + 1 < sm.nleaf) ? sm.lr_lo[L + 1][s] : rhi[s];
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
            const uint32_t hL = (L + 1 < sm.nleaf) ? sm.lr_lo[L + 1][bs] : rhi[bs];
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
            __syncthreads();
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
            __syncthreads();
         }
         if (!ok)
         {
            if (tid == 0) atomicOr(errflag, 4u);
         }
         else
         {
            const uint32_t nleaf = sm.nleaf;
            for (uint32_t L = 0; L < nleaf; L++)
            {
               if (tid < (uint32_t) LV_IN)
               {
                  sm.lo[tid] = sm.lr_lo[L][tid];
                  sm.hi[tid] = (L + 1 < nleaf) ? sm.lr_lo[L + 1][tid] : rhi[tid];
               }
               __syncthreads();
               const bool hl = has_lo || L > 0, hh = has_hi || L + 1 < nleaf;
               lv_load_merge(sm, recs, sm.lk_t[L], sm.lk_i[L], sm.lk_t[L + 1], sm.lk_i[L + 1], hl, hh, true);
               if (j == 0 && L == 0)
               {
                  if (tid == 0 && c.analytical && sm.E > 0 && cyc1(sm.r[sm.perm[0]].t) == 0) sm.cy.mode = 1;
                  __syncthreads();
               }
               Scan3 so;
               so.eA = so.eB = so.eC = so.tA = so.tB = so.tC = 0;
               lv_process(sm, c, false, so, recs, samp_t, samp_id, nexc, final_ps, errflag);
            }
         }
      }

      // ---- inclusive state (if not yet), per-port counters
      __syncthreads();
      if (tid == 0)
      {
         if (!sm.published) lv_publish_inc(st, flags, g, sm.cy);
         if (STAMPS && stamps)
         {
            stamps[(uint64_t) g * 16 + 8] = __builtin_amdgcn_s_memtime();
            stamps[(uint64_t) g * 16 + 9] = (uint64_t) j | ((uint64_t) sm.io.dir << 32);
            stamps[(uint64_t) g * 16 + 10] = sm.st_cnt;
         }
         atomicAdd(&port_sum[sm.io.port], (unsigned long long) sm.st_sum);
         atomicAdd(&port_cnt[sm.io.port], (unsigned long long) sm.st_cnt);
         if (sm.st_mg1) atomicAdd(&port_mg1[sm.io.port], (unsigned long long) sm.st_mg1);
      }
   }
}

// ---------------------------------------------------------------------------
// device-side plan
// ---------------------------------------------------------------------------
// One thread per port (level order): input slots, output slots, chunk count.
__global__ __launch_bounds__(256) void k_plan_ports(DevCfg c, uint32_t P, const uint32_t* __restrict__ lvl_ports,
                                                    const uint32_t* __restrict__ slot_cnt,
                                                    const uint64_t* __restrict__ slot_base, PortIO3* __restrict__ pio,
                                                    uint32_t* __restrict__ pnc, uint32_t ctgt)
{
   const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
   if (k >= P) return;
   const uint32_t port = lvl_ports[k];
   PortIO3 io;
   const uint32_t tile = port / PORTS, dir = port % PORTS;
   io.port = port;
   io.dir = dir;
   io.nin = 0;
   io.sb = 0;
   uint32_t tot = 0, best = 0;
   for (uint32_t s = 0; s < (uint32_t) LV_IN; s++) { io.base[s] = 0; io.slot[s] = 0; io.cnt[s] = 0; }
   for (uint32_t in = 0; in < INS; in++)
   {
      const uint32_t sl = port * INS + in;
      const uint32_t n = slot_cnt[sl];
      if (n && io.nin < (uint32_t) LV_IN)
      {
         io.slot[io.nin] = sl;
         io.base[io.nin] = slot_base[sl];
         io.cnt[io.nin] = n;
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
      const uint32_t os = slot_of(ntile, d, nside);
      io.oslot[d] = os;
      io.obase[d] = dir == P_SELF ? 0 : slot_base[os];
      io.ocnt[d] = dir == P_SELF ? 0 : slot_cnt[os];
   }
   const uint32_t nc = tot ? (tot + ctgt - 1) / ctgt : 0;
   io.gbase = 0;
   io.nc = nc;
   pio[k] = io;
   pnc[k] = nc;
}

// Single block: global exclusive scan of chunk counts (ports are in level order),
// per-level chunk bases.
__global__ __launch_bounds__(1024) void k_plan_scan(uint32_t P, uint32_t L, const uint32_t* __restrict__ lvl_off,
                                                    const uint32_t* __restrict__ pnc, uint32_t* __restrict__ pgb,
                                                    uint32_t* __restrict__ lvl_cbase)
{
   __shared__ uint32_t part[1024];
   const uint32_t per = (P + 1023) / 1024;
   const uint32_t lo = threadIdx.x * per, hi = min(lo + per, P);
   uint32_t s = 0;
   for (uint32_t i = lo; i < hi; i++) s += pnc[i];
   part[threadIdx.x] = s;
   __syncthreads();
   for (uint32_t off = 1; off < 1024; off <<= 1)
   {
      const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
   }
   uint32_t run = part[threadIdx.x] - s;
   for (uint32_t i = lo; i < hi; i++) { pgb[i] = run; run += pnc[i]; }
   __syncthreads();
   for (uint32_t l = threadIdx.x; l <= L; l += 1024) lvl_cbase[l] = l < L ? pgb[lvl_off[l]] : part[1023];
   // pgb of an empty trailing level equals the total: lvl_off[L] == P handled by the total above
}

__global__ __launch_bounds__(256) void k_plan_expand(uint32_t P, PortIO3* __restrict__ pio, const uint32_t* __restrict__ pnc,
                                                     const uint32_t* __restrict__ pgb, uint32_t* __restrict__ chunk_port)
{
   const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
   if (k >= P) return;
   const uint32_t gb = pgb[k], nc = pnc[k];
   pio[k].gbase = gb;
   for (uint32_t j = 0; j < nc; j++) chunk_port[gb + j] = k;
}

}  // namespace gnoc
