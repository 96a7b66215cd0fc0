// kernels_v2.hip -- chunk-parallel port streams (fast path: f == 1 GHz and
// max_list_size >= 3, i.e. every queue is FIFO once it has idled once).
//
// Each port's whole-trace arrival stream is cut into chunks of ~C2_TARGET
// records by (t, id) key ranges taken from its largest input slot.  One
// workgroup per chunk: it finds its range in every input slot (64-ary wave
// search over 1-in-64 key samples), merges the ranges in LDS, and runs the
// queue recurrence with the carry obtained by decoupled look-back over the
// port's earlier chunks.  The carried state is the max-plus map
//     X -> max(X + A, B)        (A = sum of F, B = max_i (t_i + F-suffix))
// plus per-next-direction record counts (output positions), or, while a
// queue has never idled, the full serial history-tree/M-G-1 state.
//
// Records served by the M/G/1 fallback can leave FIFO order; they are written
// to the END of their destination slot ("exceptions", counted in nexc[]) and
// every consumer chunk merges the exceptions that fall in its key range, so
// the main part of every slot stays sorted.
#include "common.h"

namespace gnoc {

constexpr int C2_CAP = 2048;      // records one chunk leaf holds in LDS
constexpr int C2_T = 256;         // threads per workgroup
constexpr int C2_IN = 4;          // main input slots per port
constexpr int C2_MAXLEAF = 64;    // leaves per chunk (bursts); beyond -> errflag
constexpr uint32_t C2_TARGET = 1024;
constexpr uint32_t SPIN_LIMIT = 1u << 24;

struct ChunkDesc
{
   uint32_t port, j, nc, gbase;   // PortIO index, chunk index in port, chunks of port, state index of chunk 0
};

// carried queue state (exclusive prefix of a chunk / leaf)
struct Carry
{
   uint64_t X;
   uint32_t mode, g;
   double s1, s2;
   uint64_t narr, newest;
   uint32_t cnt[5];
};

// Per-port static description (host-built from the route-static slot layout),
// copied into LDS by every chunk; nmain/nx_exc are refreshed from nexc[].
struct __attribute__((aligned(16))) PortIO
{
   uint32_t tile, dir, port, nin;
   uint64_t base[C2_IN];
   uint32_t slot[C2_IN];
   uint32_t cnt[C2_IN];
   uint32_t nmain[C2_IN];
   uint32_t nx_exc[C2_IN];
   uint64_t obase[5];
   uint32_t oslot[5];
   uint32_t ocnt[5];
   uint32_t ntile, nside, nx, ny;
   uint32_t sb, pad0;
};
static_assert(sizeof(PortIO) % 4 == 0, "PortIO copy granularity");

struct C2Smem
{
   uint64_t kt[C2_CAP];
   uint32_t ki[C2_CAP];
   uint32_t ka[C2_CAP];
   uint16_t perm[C2_CAP];
   // leaf description
   uint32_t lo[C2_IN], hi[C2_IN];      // main ranges per input
   uint32_t off[C2_IN + 1], len[C2_IN + 1];
   uint32_t nexc_leaf;                 // exceptions loaded (input C2_IN)
   uint32_t E;
   // leaf stack (key ranges)
   uint64_t lk_t[C2_MAXLEAF + 1];
   uint32_t lk_i[C2_MAXLEAF + 1];
   uint32_t nleaf;
   uint32_t lr_lo[C2_MAXLEAF][C2_IN];
   // scan scratch
   uint64_t wA[C2_T / 64], wB[C2_T / 64], wC0[C2_T / 64], wC1[C2_T / 64];
   uint32_t s0;
   uint32_t cid;
   uint32_t search[8];
   Carry cy;
   uint64_t st_sum, st_cnt, st_mg1;
   uint32_t published;
   PortIO io;
};

__device__ __forceinline__ uint32_t ld_flag(const uint32_t* p)
{
   return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_st(const uint64_t* p)
{
   return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_st(uint64_t* p, uint64_t v)
{
   __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 64-ary lower_bound of key (kt,ki) in the sorted main part [0,n) of a slot,
// using the slot's 1-in-64 key samples.  Whole wave calls; result uniform.
__device__ uint32_t wave_lower_bound(const Rec* __restrict__ r, const uint64_t* __restrict__ sp_t,
                                     const uint32_t* __restrict__ sp_i, uint32_t n, uint64_t kt, uint32_t ki,
                                     uint32_t lane)
{
   if (n == 0) return 0;
   uint32_t lo = 0, hi = (n + 63) / 64;
   while (lo < hi)
   {
      const uint32_t step = (hi - lo + 63) / 64;
      const uint32_t i = lo + lane * step;
      bool t = false;
      if (i < hi) t = key_lt(sp_t[i], sp_i[i], kt, ki);
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
   if (k < n) t = key_lt(r[k].t, r[k].id, kt, ki);
   return base + (uint32_t) __popcll(__ballot(t));
}

__device__ __forceinline__ void mp_compose(uint64_t& A, uint64_t& B, uint64_t a2, uint64_t b2)
{
   // (A,B) then (a2,b2)
   const uint64_t nb = B + a2;
   B = nb > b2 ? nb : b2;
   A += a2;
}

// Block-wide: per-thread contiguous segment [lo,hi) over merged positions.
// Computes the exclusive (A,B) prefix of this thread and block totals; same for
// packed destination counts (dirs 0-2 in c0 at 21-bit fields, 3-4 in c1).
struct ScanOut
{
   uint64_t eA, eB, tA, tB;
   uint64_t ec0, ec1, tc0, tc1;
};

__device__ __forceinline__ uint32_t route_dir(uint32_t ax, uint32_t dir, uint32_t nx, uint32_t ny, const DevCfg& c)
{
   if (dir == P_SELF) return 0;
   uint32_t dx, dy;
   tile_xy(aux_dst(ax), c.W, c.magicW, dx, dy);
   return xy_dir(nx, ny, dx, dy);
}

__device__ __forceinline__ void add_dir(uint64_t& c0, uint64_t& c1, uint32_t d)
{
   if (d < 3) c0 += 1ull << (21 * d);
   else c1 += 1ull << (21 * (d - 3));
}
__device__ __forceinline__ uint32_t get_dir(uint64_t c0, uint64_t c1, uint32_t d)
{
   return d < 3 ? (uint32_t) ((c0 >> (21 * d)) & 0x1FFFFF) : (uint32_t) ((c1 >> (21 * (d - 3))) & 0x1FFFFF);
}

__device__ ScanOut block_scan_seg(C2Smem& sm, uint32_t lo, uint32_t hi, uint32_t dir, uint32_t nx, uint32_t ny,
                                  const DevCfg& c)
{
   const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
   uint64_t A = 0, B = 0, c0 = 0, c1 = 0;
   for (uint32_t e = lo; e < hi; e++)
   {
      const uint32_t k = sm.perm[e];
      const uint64_t tc = cyc_of<true>(sm.kt[k], c.f);
      const uint64_t p = aux_F(sm.ka[k]);
      mp_compose(A, B, p, tc + p);
      add_dir(c0, c1, route_dir(sm.ka[k], dir, nx, ny, c));
   }
   uint64_t iA = A, iB = B, i0 = c0, i1 = c1;
   for (int off = 1; off < 64; off <<= 1)
   {
      const uint64_t pA = __shfl_up(iA, off), pB = __shfl_up(iB, off);
      const uint64_t p0 = __shfl_up(i0, off), p1 = __shfl_up(i1, off);
      if ((int) lane >= off)
      {
         uint64_t a = pA, b = pB;
         mp_compose(a, b, iA, iB);
         iA = a;
         iB = b;
         i0 += p0;
         i1 += p1;
      }
   }
   __syncthreads();   // protect wA.. from a previous use
   if (lane == 63) { sm.wA[wv] = iA; sm.wB[wv] = iB; sm.wC0[wv] = i0; sm.wC1[wv] = i1; }
   __syncthreads();
   ScanOut o;
   uint64_t PA = 0, PB = 0, P0 = 0, P1 = 0;
   for (uint32_t w = 0; w < wv; w++)
   {
      mp_compose(PA, PB, sm.wA[w], sm.wB[w]);
      P0 += sm.wC0[w];
      P1 += sm.wC1[w];
   }
   uint64_t eA = __shfl_up(iA, 1), eB = __shfl_up(iB, 1), e0 = __shfl_up(i0, 1), e1 = __shfl_up(i1, 1);
   if (lane == 0) { eA = 0; eB = 0; e0 = 0; e1 = 0; }
   mp_compose(PA, PB, eA, eB);
   o.eA = PA;
   o.eB = PB;
   o.ec0 = P0 + e0;
   o.ec1 = P1 + e1;
   uint64_t TA = 0, TB = 0, T0 = 0, T1 = 0;
   for (uint32_t w = 0; w < C2_T / 64; w++)
   {
      mp_compose(TA, TB, sm.wA[w], sm.wB[w]);
      T0 += sm.wC0[w];
      T1 += sm.wC1[w];
   }
   o.tA = TA;
   o.tB = TB;
   o.tc0 = T0;
   o.tc1 = T1;
   return o;
}

// Load one leaf (main ranges sm.lo/hi + exceptions with key in [klo,khi)) into LDS and merge.
__device__ void load_merge(C2Smem& sm, const PortIO& io, const Rec* __restrict__ recs, uint64_t klo_t, uint32_t klo_i,
                           uint64_t khi_t, uint32_t khi_i, bool has_lo, bool has_hi)
{
   const uint32_t tid = threadIdx.x;
   if (tid == 0)
   {
      uint32_t o = 0;
      for (uint32_t s = 0; s < C2_IN; s++)
      {
         sm.off[s] = o;
         sm.len[s] = s < io.nin ? sm.hi[s] - sm.lo[s] : 0;
         o += sm.len[s];
      }
      sm.off[C2_IN] = o;
      sm.len[C2_IN] = 0;
      sm.nexc_leaf = 0;
   }
   __syncthreads();
   for (uint32_t s = 0; s < io.nin; s++)
   {
      const Rec* r = recs + io.base[s] + sm.lo[s];
      const uint32_t L = sm.len[s], o = sm.off[s];
      for (uint32_t i = tid; i < L; i += C2_T)
      {
         const Rec v = r[i];
         sm.kt[o + i] = v.t;
         sm.ki[o + i] = v.id;
         sm.ka[o + i] = v.aux;
      }
   }
   // exceptions (rare): tail [nmain, cnt) of each input
   bool anyexc = false;
   for (uint32_t s = 0; s < io.nin; s++) anyexc |= io.nx_exc[s] > 0;
   if (anyexc)
   {
      const uint32_t o = sm.off[C2_IN];
      for (uint32_t s = 0; s < io.nin; s++)
      {
         const Rec* r = recs + io.base[s];
         for (uint32_t i = io.nmain[s] + tid; i < io.cnt[s]; i += C2_T)
         {
            const Rec v = r[i];
            const bool ge = !has_lo || !key_lt(v.t, v.id, klo_t, klo_i);
            const bool lt = !has_hi || key_lt(v.t, v.id, khi_t, khi_i);
            if (ge && lt)
            {
               const uint32_t k = atomicAdd(&sm.nexc_leaf, 1u);
               if (o + k < (uint32_t) C2_CAP)
               {
                  sm.kt[o + k] = v.t;
                  sm.ki[o + k] = v.id;
                  sm.ka[o + k] = v.aux;
               }
            }
         }
      }
      __syncthreads();
      const uint32_t ne = min(sm.nexc_leaf, (uint32_t) C2_CAP - o);
      // odd-even transposition sort of the (few) exceptions by key
      for (uint32_t ph = 0; ph < ne; ph++)
      {
         for (uint32_t i = 2 * tid + (ph & 1); i + 1 < ne; i += 2 * C2_T)
         {
            const uint32_t a = o + i, b = o + i + 1;
            if (key_lt(sm.kt[b], sm.ki[b], sm.kt[a], sm.ki[a]))
            {
               uint64_t t = sm.kt[a]; sm.kt[a] = sm.kt[b]; sm.kt[b] = t;
               uint32_t x = sm.ki[a]; sm.ki[a] = sm.ki[b]; sm.ki[b] = x;
               x = sm.ka[a]; sm.ka[a] = sm.ka[b]; sm.ka[b] = x;
            }
         }
         __syncthreads();
      }
      if (tid == 0) sm.len[C2_IN] = ne;
   }
   __syncthreads();
   const uint32_t E = sm.off[C2_IN] + sm.len[C2_IN];
   // merge: rank = own index + #smaller keys in every other input (binary search in LDS)
   for (uint32_t k = tid; k < E; k += C2_T)
   {
      uint32_t s = 0;
      while (s < C2_IN && k >= sm.off[s] + sm.len[s]) s++;
      const uint64_t t = sm.kt[k];
      const uint32_t id = sm.ki[k];
      uint32_t rank = k - sm.off[s];
      for (uint32_t o = 0; o <= (uint32_t) C2_IN; o++)
      {
         if (o == s || sm.len[o] == 0) continue;
         uint32_t lo = sm.off[o], hi = sm.off[o] + sm.len[o];
         while (lo < hi)
         {
            const uint32_t mid = (lo + hi) >> 1;
            if (key_lt(sm.kt[mid], sm.ki[mid], t, id)) lo = mid + 1; else hi = mid;
         }
         rank += lo - sm.off[o];
      }
      sm.perm[rank] = (uint16_t) k;
   }
   if (tid == 0) sm.E = E;
   __syncthreads();
}

// Process the merged leaf in LDS starting from carry sm.cy; write outputs; advance sm.cy.
__device__ void process_leaf(C2Smem& sm, const PortIO& io, const DevCfg& c, Rec* __restrict__ recs,
                             uint64_t* __restrict__ samp_t, uint32_t* __restrict__ samp_id,
                             uint32_t* __restrict__ nexc, const uint32_t* __restrict__ slot_cnt,
                             const uint64_t* __restrict__ slot_base, uint64_t* __restrict__ final_ps)
{
   const uint32_t tid = threadIdx.x;
   const uint32_t E = sm.E;
   const uint32_t dir = io.dir;
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
            const uint32_t k = sm.perm[e];
            const uint64_t t = sm.kt[k];
            const uint32_t ax = sm.ka[k], id = sm.ki[k];
            const uint64_t mg_before = s.mg1;
            const uint64_t cc = serial_step(s, cyc_of<true>(t, c.f), aux_F(ax), c.max_list, c.analytical);
            if (s.g >= 1) s.mode = 0;
            ssum += cc;
            const uint64_t tn = t + ps_of<true>(cc, c.f) + (dir == P_INJ ? 0ull : c.rl_ps);
            if (dir == P_SELF) { final_ps[id] = tn + ps_of<true>(aux_F(ax), c.f); continue; }
            const uint32_t nd = route_dir(ax, dir, io.nx, io.ny, c);
            const uint32_t os = io.oslot[nd];
            Rec o;
            o.t = tn;
            o.id = id;
            o.aux = ax;
            if (s.mg1 != mg_before)
            {
               // M/G/1-served: may leave FIFO order -> exception tail of the slot
               const uint32_t x = atomicAdd(&nexc[os], 1u);
               recs[io.obase[nd] + io.ocnt[nd] - 1 - x] = o;
            }
            else
            {
               const uint32_t pos = sm.cy.cnt[nd]++;
               recs[io.obase[nd] + pos] = o;
               if ((pos & 63) == 0)
               {
                  samp_t[io.obase[nd] / 64 + pos / 64] = tn;
                  samp_id[io.obase[nd] / 64 + pos / 64] = id;
               }
            }
         }
         sm.s0 = e;
         sm.cy.X = s.X; sm.cy.g = (uint32_t) s.g; sm.cy.mode = s.mode; sm.cy.s1 = s.s1; sm.cy.s2 = s.s2;
         sm.cy.narr = s.narr; sm.cy.newest = s.newest;
         sm.st_sum += ssum;
         sm.st_cnt += e;
         sm.st_mg1 += s.mg1;
      }
   }
   else if (tid == 0)
   {
      sm.s0 = 0;
   }
   __syncthreads();
   const uint32_t s0 = sm.s0;
   const uint32_t cnt = E - s0;
   const uint32_t per = (cnt + C2_T - 1) / C2_T;
   const uint32_t lo = s0 + min(tid * per, cnt), hi = s0 + min((tid + 1) * per, cnt);
   const ScanOut so = block_scan_seg(sm, lo, hi, dir, io.nx, io.ny, c);
   const uint64_t X0 = sm.cy.X;
   uint64_t X = X0 + so.eA;
   X = X > so.eB ? X : so.eB;
   uint64_t c0 = so.ec0, c1 = so.ec1;
   uint64_t ssum = 0;
   for (uint32_t e = lo; e < hi; e++)
   {
      const uint32_t k = sm.perm[e];
      const uint64_t t = sm.kt[k];
      const uint32_t ax = sm.ka[k], id = sm.ki[k];
      const uint64_t tc = cyc_of<true>(t, c.f);
      const uint64_t cc = X > tc ? X - tc : 0;
      X = (X > tc ? X : tc) + aux_F(ax);
      ssum += cc;
      const uint64_t tn = t + ps_of<true>(cc, c.f) + (dir == P_INJ ? 0ull : c.rl_ps);
      if (dir == P_SELF)
      {
         final_ps[id] = tn + ps_of<true>(aux_F(ax), c.f);
         continue;
      }
      const uint32_t nd = route_dir(ax, dir, io.nx, io.ny, c);
      const uint32_t pos = sm.cy.cnt[nd] + get_dir(c0, c1, nd);
      add_dir(c0, c1, nd);
      const uint64_t gb = io.obase[nd];
      Rec o;
      o.t = tn;
      o.id = id;
      o.aux = ax;
      recs[gb + pos] = o;
      if ((pos & 63) == 0)
      {
         samp_t[gb / 64 + pos / 64] = tn;
         samp_id[gb / 64 + pos / 64] = id;
      }
   }
   // stats
   for (int off = 32; off > 0; off >>= 1) ssum += __shfl_down(ssum, off);
   __syncthreads();
   if ((tid & 63) == 0) atomicAdd((unsigned long long*) &sm.st_sum, (unsigned long long) ssum);
   __syncthreads();
   if (tid == 0)
   {
      sm.st_cnt += cnt;
      uint64_t nx0 = X0 + so.tA;
      sm.cy.X = nx0 > so.tB ? nx0 : so.tB;
      for (uint32_t d = 0; d < 5; d++) sm.cy.cnt[d] += get_dir(so.tc0, so.tc1, d);
   }
   __syncthreads();
}

// Decoupled look-back (wave 0): exclusive carry of chunk j from chunks [0, j).
__device__ bool lookback(C2Smem& sm, uint32_t gbase, uint32_t j, const uint32_t* __restrict__ flags,
                         const uint64_t* __restrict__ st, unsigned* __restrict__ errflag)
{
   const uint32_t lane = threadIdx.x & 63;
   uint64_t accA = 0, accB = 0;       // composed map of chunks (stop, j)
   uint64_t accC[5] = { 0, 0, 0, 0, 0 };
   int32_t look = (int32_t) j - 1;
   uint32_t spins = 0;
   for (;;)
   {
      const int32_t ck = look - (int32_t) lane;
      uint32_t f = 2;
      if (ck >= 0) f = ld_flag(&flags[gbase + ck]);
      const uint64_t inc = __ballot(ck >= 0 && f == 2);
      const uint64_t zero = __ballot(ck >= 0 && f == 0);
      const uint64_t stop = inc | __ballot(ck < 0);
      const int L = stop ? __ffsll((long long) stop) - 1 : 64;
      const uint64_t need = L >= 64 ? ~0ull : ((1ull << L) - 1);
      if (zero & need)
      {
         if (++spins > SPIN_LIMIT) { if (lane == 0) atomicOr(errflag, 2u); return false; }
         __builtin_amdgcn_s_sleep(1);
         continue;
      }
      // aggregates of lanes [0, L): chunk look-l; lane L-1 is the earliest
      uint64_t a = 0, b = 0, q0 = 0, q1 = 0, q2 = 0;
      if ((int) lane < L)
      {
         const uint64_t* w = st + (uint64_t) (gbase + ck) * 16;
         a = ld_st(w + 0);
         b = ld_st(w + 1);
         q0 = ld_st(w + 2);
         q1 = ld_st(w + 3);
         q2 = ld_st(w + 4);
      }
      // compose in chunk order: earliest (lane L-1) first ... lane 0 last, then the accumulated tail
      uint64_t wa = 0, wb = 0;
      for (int l = L - 1; l >= 0; l--)
      {
         const uint64_t la = __shfl(a, l), lb = __shfl(b, l);
         mp_compose(wa, wb, la, lb);
      }
      mp_compose(wa, wb, accA, accB);
      accA = wa;
      accB = wb;
      for (int l = 0; l < L; l++)
      {
         const uint64_t x0 = __shfl(q0, l), x1 = __shfl(q1, l), x2 = __shfl(q2, l);
         accC[0] += x0 & 0xFFFFFFFFull; accC[1] += x0 >> 32;
         accC[2] += x1 & 0xFFFFFFFFull; accC[3] += x1 >> 32;
         accC[4] += x2;
      }
      if (L < 64)
      {
         const int32_t sc = look - L;   // chunk holding an inclusive state (chunk 0 always publishes one)
         const uint64_t* w = st + (uint64_t) (gbase + sc) * 16;
         const uint64_t modeg = ld_st(w + 9);
         const uint32_t mode = (uint32_t) (modeg & 0xFFFFFFFFull);
         if (mode && sc != (int32_t) j - 1)
         {
            // the queue was still in its serial prefix: FIFO aggregates after it are invalid;
            // wait for the immediate predecessor's inclusive state instead.
            const uint32_t pj = gbase + j - 1;
            while (ld_flag(&flags[pj]) != 2)
            {
               if (++spins > SPIN_LIMIT) { if (lane == 0) atomicOr(errflag, 2u); return false; }
               __builtin_amdgcn_s_sleep(1);
            }
            w = st + (uint64_t) pj * 16;
            accA = 0; accB = 0;
            for (int d = 0; d < 5; d++) accC[d] = 0;
         }
         if (lane == 0)
         {
            const uint64_t X = ld_st(w + 8);
            const uint64_t mg = ld_st(w + 9);
            const uint64_t c01 = ld_st(w + 14), c23 = ld_st(w + 15), c4 = ld_st(w + 7);
            uint64_t nx = X + accA;
            sm.cy.X = nx > accB ? nx : accB;
            sm.cy.mode = (uint32_t) (mg & 0xFFFFFFFFull);
            sm.cy.g = (uint32_t) (mg >> 32);
            sm.cy.s1 = __longlong_as_double((long long) ld_st(w + 10));
            sm.cy.s2 = __longlong_as_double((long long) ld_st(w + 11));
            sm.cy.narr = ld_st(w + 12);
            sm.cy.newest = ld_st(w + 13);
            sm.cy.cnt[0] = (uint32_t) ((c01 & 0xFFFFFFFFull) + accC[0]);
            sm.cy.cnt[1] = (uint32_t) ((c01 >> 32) + accC[1]);
            sm.cy.cnt[2] = (uint32_t) ((c23 & 0xFFFFFFFFull) + accC[2]);
            sm.cy.cnt[3] = (uint32_t) ((c23 >> 32) + accC[3]);
            sm.cy.cnt[4] = (uint32_t) (c4 + accC[4]);
         }
         return true;
      }
      look -= 64;
   }
}

__device__ void publish_agg(uint64_t* __restrict__ st, uint32_t* __restrict__ flags, uint32_t cidx, uint64_t A,
                            uint64_t B, uint64_t tc0, uint64_t tc1)
{
   uint64_t* w = st + (uint64_t) cidx * 16;
   st_st(w + 0, A);
   st_st(w + 1, B);
   st_st(w + 2, (uint64_t) get_dir(tc0, tc1, 0) | ((uint64_t) get_dir(tc0, tc1, 1) << 32));
   st_st(w + 3, (uint64_t) get_dir(tc0, tc1, 2) | ((uint64_t) get_dir(tc0, tc1, 3) << 32));
   st_st(w + 4, (uint64_t) get_dir(tc0, tc1, 4));
   asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
   __hip_atomic_store(&flags[cidx], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void publish_inc(uint64_t* __restrict__ st, uint32_t* __restrict__ flags, uint32_t cidx, const Carry& cy)
{
   uint64_t* w = st + (uint64_t) cidx * 16;
   st_st(w + 7, (uint64_t) cy.cnt[4]);
   st_st(w + 8, cy.X);
   st_st(w + 9, (uint64_t) cy.mode | ((uint64_t) cy.g << 32));
   st_st(w + 10, (uint64_t) __double_as_longlong(cy.s1));
   st_st(w + 11, (uint64_t) __double_as_longlong(cy.s2));
   st_st(w + 12, cy.narr);
   st_st(w + 13, cy.newest);
   st_st(w + 14, (uint64_t) cy.cnt[0] | ((uint64_t) cy.cnt[1] << 32));
   st_st(w + 15, (uint64_t) cy.cnt[2] | ((uint64_t) cy.cnt[3] << 32));
   asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
   __hip_atomic_store(&flags[cidx], 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#define STAMP(k)                                                                                         \
   do                                                                                                   \
   {                                                                                                    \
      if (STAMPS && stamps && tid == 0) stamps[(uint64_t) sm.cid * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
   } while (0)

template <bool STAMPS>
__global__ __launch_bounds__(C2_T) void k_chunk(DevCfg c, const ChunkDesc* __restrict__ chunks, const PortIO* __restrict__ ports,
                                                unsigned* __restrict__ ctr,
                                                const uint32_t* __restrict__ slot_cnt, const uint64_t* __restrict__ slot_base,
                                                Rec* __restrict__ recs, uint64_t* __restrict__ samp_t,
                                                uint32_t* __restrict__ samp_id, uint32_t* __restrict__ nexc,
                                                uint32_t* __restrict__ flags, uint64_t* __restrict__ st,
                                                uint64_t* __restrict__ final_ps, unsigned long long* __restrict__ port_sum,
                                                unsigned long long* __restrict__ port_cnt,
                                                unsigned long long* __restrict__ port_mg1, unsigned* __restrict__ errflag,
                                                uint64_t* __restrict__ stamps)
{
   __shared__ C2Smem sm;
   const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
   if (tid == 0)
   {
      sm.cid = atomicAdd(ctr, 1u);   // dynamic order: every predecessor chunk is already running
      sm.st_sum = 0;
      sm.st_cnt = 0;
      sm.st_mg1 = 0;
      sm.published = 0;
   }
   __syncthreads();
   STAMP(0);
   const ChunkDesc d = chunks[sm.cid];
   const uint32_t cidx = d.gbase + d.j;

   // ---- port description -> LDS (one coalesced copy), refresh exception counts
   {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(ports + d.port);
      uint32_t* dstw = reinterpret_cast<uint32_t*>(&sm.io);
      for (uint32_t k = tid; k < (uint32_t) (sizeof(PortIO) / 4); k += C2_T) dstw[k] = src[k];
      __syncthreads();
      if (tid < sm.io.nin)
      {
         const uint32_t x = nexc[sm.io.slot[tid]];
         sm.io.nx_exc[tid] = x;
         sm.io.nmain[tid] = sm.io.cnt[tid] - x;
      }
      __syncthreads();
   }
   const PortIO& io = sm.io;

   // ---- chunk key range from the largest input (exact index split, no search)
   const uint32_t sb = io.sb;
   const uint32_t nb = io.nmain[sb];
   const uint32_t ilo = (uint32_t) (((uint64_t) d.j * nb) / d.nc);
   const uint32_t ihi = (uint32_t) (((uint64_t) (d.j + 1) * nb) / d.nc);
   const bool has_lo = d.j > 0, has_hi = d.j + 1 < d.nc;
   uint64_t klo_t = 0, khi_t = ~0ull;
   uint32_t klo_i = 0, khi_i = ~0u;
   if (has_lo) { const Rec r = recs[io.base[sb] + ilo]; klo_t = r.t; klo_i = r.id; }
   if (has_hi) { const Rec r = recs[io.base[sb] + ihi]; khi_t = r.t; khi_i = r.id; }

   STAMP(1);
   // ---- main ranges of the other inputs (waves search in parallel)
   for (uint32_t q = wv; q < 2 * C2_IN; q += C2_T / 64)
   {
      const uint32_t s = q >> 1, which = q & 1;
      if (s >= io.nin) continue;
      uint32_t v;
      if (s == sb) v = which ? (has_hi ? ihi : nb) : (has_lo ? ilo : 0);
      else if (which == 0 && !has_lo) v = 0;
      else if (which == 1 && !has_hi) v = io.nmain[s];
      else
      {
         const uint64_t sbase = io.base[s] / 64;
         v = wave_lower_bound(recs + io.base[s], samp_t + sbase, samp_id + sbase, io.nmain[s], which ? khi_t : klo_t,
                              which ? khi_i : klo_i, lane);
      }
      if (lane == 0) sm.search[q] = v;
   }
   __syncthreads();
   STAMP(2);
   uint32_t total = 0;
   uint32_t rlo[C2_IN], rhi[C2_IN];
   for (uint32_t s = 0; s < C2_IN; s++)
   {
      rlo[s] = s < io.nin ? sm.search[2 * s] : 0;
      rhi[s] = s < io.nin ? sm.search[2 * s + 1] : 0;
      total += rhi[s] - rlo[s];
   }
   uint32_t totexc = 0;
   for (uint32_t s = 0; s < io.nin; s++) totexc += io.nx_exc[s];

   if (tid == 0)
   {
      sm.cy.X = 0; sm.cy.mode = 0; sm.cy.g = 0; sm.cy.s1 = 0; sm.cy.s2 = 0; sm.cy.narr = 0; sm.cy.newest = 0;
      for (int k = 0; k < 5; k++) sm.cy.cnt[k] = 0;
   }

   if (total + totexc <= (uint32_t) C2_CAP)
   {
      // ---------------- single leaf
      if (tid < C2_IN) { sm.lo[tid] = rlo[tid]; sm.hi[tid] = rhi[tid]; }
      __syncthreads();
      load_merge(sm, io, recs, klo_t, klo_i, khi_t, khi_i, has_lo, has_hi);
      STAMP(3);
      if (d.j == 0)
      {
         if (tid == 0 && c.analytical && sm.E > 0 && cyc_of<true>(sm.kt[sm.perm[0]], c.f) == 0) sm.cy.mode = 1;
         __syncthreads();
      }
      const bool early = d.j > 0 || !sm.cy.mode;
      if (early)
      {
         // FIFO aggregate of this chunk, published before looking back
         const uint32_t E = sm.E;
         const uint32_t per = (E + C2_T - 1) / C2_T;
         const uint32_t lo = min(tid * per, E), hi = min((tid + 1) * per, E);
         const ScanOut so = block_scan_seg(sm, lo, hi, io.dir, io.nx, io.ny, c);
         STAMP(4);
         if (d.j > 0)
         {
            if (tid == 0) publish_agg(st, flags, cidx, so.tA, so.tB, so.tc0, so.tc1);
            STAMP(5);
            if (wv == 0) lookback(sm, d.gbase, d.j, flags, st, errflag);
            __syncthreads();
         }
         STAMP(6);
         // In FIFO mode the inclusive state is exclusive (x) aggregate: publish it now,
         // before writing outputs, so successors stop waiting as early as possible.
         if (tid == 0 && !sm.cy.mode)
         {
            Carry inc = sm.cy;
            const uint64_t nx0 = inc.X + so.tA;
            inc.X = nx0 > so.tB ? nx0 : so.tB;
            for (uint32_t k = 0; k < 5; k++) inc.cnt[k] += get_dir(so.tc0, so.tc1, k);
            publish_inc(st, flags, cidx, inc);
            sm.published = 1;
         }
      }
      process_leaf(sm, io, c, recs, samp_t, samp_id, nexc, slot_cnt, slot_base, final_ps);
      STAMP(7);
   }
   else
   {
      // ---------------- burst: split the key range into leaves that fit LDS
      if (d.j > 0)
      {
         if (wv == 0) lookback(sm, d.gbase, d.j, flags, st, errflag);
      }
      if (tid == 0)
      {
         sm.nleaf = 1;
         sm.lk_t[0] = klo_t; sm.lk_i[0] = klo_i;
         sm.lk_t[1] = khi_t; sm.lk_i[1] = khi_i;
         for (uint32_t s = 0; s < C2_IN; s++) sm.lr_lo[0][s] = rlo[s];
      }
      __syncthreads();
      // Leaves are kept as a sorted boundary list; split the first over-full leaf until all fit.
      // (range of leaf L = [lk[L], lk[L+1]); main index lower bounds per input in lr_lo[L])
      bool ok = true;
      for (uint32_t iter = 0; iter < 4 * C2_MAXLEAF && ok; iter++)
      {
         // find first leaf whose size exceeds the LDS budget (exceptions counted conservatively)
         int32_t bad = -1;
         uint32_t bs = 0;
         for (uint32_t L = 0; L < sm.nleaf && bad < 0; L++)
         {
            uint32_t sz = totexc;
            uint32_t best = 0, bestn = 0;
            for (uint32_t s = 0; s < io.nin; s++)
            {
               const uint32_t h = (L + 1 < sm.nleaf) ? sm.lr_lo[L + 1][s] : rhi[s];
               const uint32_t n = h - sm.lr_lo[L][s];
               sz += n;
               if (n > bestn) { bestn = n; best = s; }
            }
            if (sz > (uint32_t) C2_CAP) { bad = (int32_t) L; bs = best; }
         }
         if (bad < 0) break;
         if (sm.nleaf >= (uint32_t) C2_MAXLEAF) { ok = false; break; }
         // split leaf `bad` at the median of its largest input
         const uint32_t L = (uint32_t) bad;
         const uint32_t hL = (L + 1 < sm.nleaf) ? sm.lr_lo[L + 1][bs] : rhi[bs];
         const uint32_t mid = (sm.lr_lo[L][bs] + hL) / 2;
         const Rec mr = recs[io.base[bs] + mid];
         for (uint32_t q = wv; q < C2_IN; q += C2_T / 64)
         {
            if (q >= io.nin) continue;
            uint32_t v = mid;
            if (q != bs)
            {
               const uint64_t sbase = io.base[q] / 64;
               v = wave_lower_bound(recs + io.base[q], samp_t + sbase, samp_id + sbase, io.nmain[q], mr.t, mr.id, lane);
            }
            if (lane == 0) sm.search[q] = v;
         }
         __syncthreads();
         if (tid == 0)
         {
            for (uint32_t M = sm.nleaf; M > L + 1; M--)
            {
               for (uint32_t s = 0; s < C2_IN; s++) sm.lr_lo[M][s] = sm.lr_lo[M - 1][s];
            }
            for (uint32_t M = sm.nleaf + 1; M > L + 1; M--) { sm.lk_t[M] = sm.lk_t[M - 1]; sm.lk_i[M] = sm.lk_i[M - 1]; }
            sm.lk_t[L + 1] = mr.t;
            sm.lk_i[L + 1] = mr.id;
            for (uint32_t s = 0; s < C2_IN; s++) sm.lr_lo[L + 1][s] = s < io.nin ? sm.search[s] : 0;
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
         for (uint32_t L = 0; L < sm.nleaf; L++)
         {
            if (tid < C2_IN)
            {
               sm.lo[tid] = sm.lr_lo[L][tid];
               sm.hi[tid] = (L + 1 < sm.nleaf) ? sm.lr_lo[L + 1][tid] : rhi[tid];
            }
            __syncthreads();
            const bool hl = has_lo || L > 0, hh = has_hi || L + 1 < sm.nleaf;
            load_merge(sm, io, recs, sm.lk_t[L], sm.lk_i[L], sm.lk_t[L + 1], sm.lk_i[L + 1], hl, hh);
            if (d.j == 0 && L == 0)
            {
               if (tid == 0 && c.analytical && sm.E > 0 && cyc_of<true>(sm.kt[sm.perm[0]], c.f) == 0) sm.cy.mode = 1;
               __syncthreads();
            }
            process_leaf(sm, io, c, recs, samp_t, samp_id, nexc, slot_cnt, slot_base, final_ps);
         }
      }
   }

   // ---- publish inclusive state, per-port counters
   if (tid == 0)
   {
      if (!sm.published) publish_inc(st, flags, cidx, sm.cy);
      if (STAMPS && stamps) stamps[(uint64_t) sm.cid * 16 + 8] = __builtin_amdgcn_s_memtime();
      if (STAMPS && stamps) stamps[(uint64_t) sm.cid * 16 + 9] = (uint64_t) d.j | ((uint64_t) io.dir << 32);
      atomicAdd(&port_sum[io.port], (unsigned long long) sm.st_sum);
      atomicAdd(&port_cnt[io.port], (unsigned long long) sm.st_cnt);
      if (sm.st_mg1) atomicAdd(&port_mg1[io.port], (unsigned long long) sm.st_mg1);
   }
}

// Samples of the (trace-grouped) injection slots: key of every 64th record.
__global__ __launch_bounds__(256) void k_inj_samples(uint32_t N, const uint32_t* __restrict__ slot_cnt,
                                                     const uint64_t* __restrict__ slot_base, const Rec* __restrict__ recs,
                                                     uint64_t* __restrict__ samp_t, uint32_t* __restrict__ samp_id)
{
   const uint32_t tile = blockIdx.x;
   const uint32_t sl = slot_of(tile, P_INJ, IN_LOCAL);
   const uint32_t n = slot_cnt[sl];
   const uint64_t b = slot_base[sl];
   for (uint32_t i = threadIdx.x * 64; i < n; i += 256 * 64)
   {
      samp_t[b / 64 + i / 64] = recs[b + i].t;
      samp_id[b / 64 + i / 64] = recs[b + i].id;
   }
}

}  // namespace gnoc
