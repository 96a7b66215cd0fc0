// kernels.hip -- CDNA4 (gfx950) kernels of the emesh_hop_by_hop timing engine.
//
// The reference walks each packet hop by hop through per-port history-tree
// queues (network_model_emesh_hop_by_hop.cc:146-264, router_model.cc:70-108,
// queue_model_history_tree.cc:43-126).  With XY routing the output-port graph
// is acyclic (injection -> X chain of the source row -> Y chain of the
// destination column -> SELF), and with arrivals served in (time, id) order
// every history-tree queue is the FIFO max-plus recurrence
//     c_i = max(X - t_i, 0),  X <- max(t_i, X) + F_i
// plus an M/G/1 prologue while the queue has never been idle.
// So the engine processes ports level by level along that DAG; each port's
// whole-trace arrival stream is the (t, id)-merge of its input streams, which
// are sorted because each producer emits in FIFO order.
#include "common.h"

namespace gnoc {

// ----------------------------------------------------------------------------
// Port stream kernel: one workgroup owns one output-port queue and streams its
// whole arrival history.  Per round: load up to T records of each input
// stream into LDS, merge the prefix that is provably complete ((t,id) <= the
// smallest last-loaded key of any stream with more data), run the queue
// recurrence (serial M/G/1 prologue while the queue has never idled, then a
// block-wide max-plus scan), and route every record to its next port's input
// slot (or write the packet's final time at SELF).
// ----------------------------------------------------------------------------
constexpr int ST = 256;          // records per input per round
constexpr int STHREADS = 256;
// Broadcast batches (BC): a port's broadcast records (the tails of its input
// slots, written in any order) are sorted in LDS and merged as one more stream.
constexpr int BC_CAP = 4096;

struct SerialState
{
   uint64_t X;        // start of the tail free interval [X, inf)
   int g;             // number of gap intervals in the history tree
   int mode;          // 1 while the serial (tree + M/G/1) path is required
   double s1, s2;     // QueueModelMG1 sums
   uint64_t narr, newest;
   uint64_t mg1;
};

// NS input streams: the <= 4 non-empty input slots of a unicast port, or the 5
// slots' unicast parts plus the broadcast stream.
template <int NS>
struct PortSmem
{
   uint64_t in_t[NS][ST];
   uint32_t in_id[NS][ST];
   uint32_t in_aux[NS][ST];
   uint64_t m_t[NS * ST];
   uint32_t m_id[NS * ST];
   uint32_t m_aux[NS * ST];
   uint64_t m_c[NS * ST];
   uint64_t wA[STHREADS / 64], wB[STHREADS / 64], wC[STHREADS / 64];
   uint32_t e_cnt[NS];
   uint32_t s0;
   SerialState ss;
};

struct BcSmem
{
   uint64_t t[BC_CAP];
   uint32_t i[BC_CAP];
   uint32_t a[BC_CAP];
};

__device__ __forceinline__ bool key_le(uint64_t t1, uint32_t i1, uint64_t t2, uint32_t i2)
{
   return t1 < t2 || (t1 == t2 && i1 <= i2);
}
__device__ __forceinline__ bool key_lt(uint64_t t1, uint32_t i1, uint64_t t2, uint32_t i2)
{
   return t1 < t2 || (t1 == t2 && i1 < i2);
}

// QueueModelMG1::computeQueueDelay (queue_model_m_g_1.cc:17-46); same operation
// order; this translation unit is compiled with -ffp-contract=off.
__device__ uint64_t mg1_delay(const SerialState& s)
{
   if (s.narr == 0) return 0;
   double variance = ((s.s2 / (double) s.narr) - ((s.s1 / (double) s.narr) * (s.s1 / (double) s.narr)));
   double service_rate = 1.0 / (s.s1 / (double) s.narr);
   double arrival_rate = ((double) s.narr) / (double) s.newest;
   if (arrival_rate >= service_rate) arrival_rate = 0.999 * service_rate;
   return (uint64_t) ceil(0.5 * service_rate * arrival_rate * ((1 / (service_rate * service_rate)) + variance) /
                          (service_rate - arrival_rate));
}

// One history-tree request with arrivals in non-decreasing time
// (queue_model_history_tree.cc:43-126 specialised; DESIGN.md "queue").
__device__ uint64_t serial_step(SerialState& s, uint64_t t, uint64_t p, int L, int analytical)
{
   if (s.g + 1 >= L) s.g--;   // :50-56 prune the oldest free interval
   uint64_t d;
   if (analytical && s.g == 0 && s.X > t + p)
   {
      d = mg1_delay(s);        // :58-64 M/G/1 fallback, tree untouched
      s.mg1++;
   }
   else if (t >= s.X)
   {
      d = 0;
      if (t - s.X >= 1) s.g++;   // :79-86 idle period becomes a gap
      s.X = t + p;
   }
   else
   {
      d = s.X - t;               // :101-112 wait for the tail interval
      s.X = s.X + p;
   }
   // QueueModelMG1::updateQueue, queue_model_m_g_1.cc:48-56
   s.s2 += ((double) p * (double) p);
   s.s1 += (double) p;
   s.narr++;
   const uint64_t nw = t + d + p;
   s.newest = s.newest > nw ? s.newest : nw;
   return d;
}

// ----------------------------------------------------------------------------
// Fixup: restore (t, id) order of an input slot whose producer emitted out of
// FIFO order (rare: M/G/1 requests, or f != 1 GHz ties).  Run by the consuming
// port's workgroup before it streams the slot.
// ----------------------------------------------------------------------------
constexpr int FIX_LDS = 2048;

struct FixSmem
{
   uint64_t kt[FIX_LDS];
   uint32_t ki[FIX_LDS];
   uint32_t ka[FIX_LDS];
};

// Block-wide bitonic sort by (t, id) of P (a power of two) LDS entries.
__device__ void bitonic_lds(uint64_t* kt, uint32_t* ki, uint32_t* ka, uint32_t P)
{
   const uint32_t tid = threadIdx.x;
   for (uint32_t k = 2; k <= P; k <<= 1)
   {
      for (uint32_t j = k >> 1; j > 0; j >>= 1)
      {
         for (uint32_t i = tid; i < P; i += blockDim.x)
         {
            const uint32_t l = i ^ j;
            if (l > i)
            {
               const bool up = (i & k) == 0;
               const bool gt = key_lt(kt[l], ki[l], kt[i], ki[i]);
               if (gt == up)
               {
                  uint64_t tt = kt[i]; kt[i] = kt[l]; kt[l] = tt;
                  uint32_t ti = ki[i]; ki[i] = ki[l]; ki[l] = ti;
                  uint32_t ta = ka[i]; ka[i] = ka[l]; ka[l] = ta;
               }
            }
         }
         __syncthreads();
      }
   }
}

__device__ void fixup_slot(FixSmem& fx, Rec* __restrict__ r, uint32_t n)
{
   const uint32_t tid = threadIdx.x;
   if (n <= 1) return;
   if (n <= (uint32_t) FIX_LDS)
   {
      uint32_t P = 1;
      while (P < n) P <<= 1;
      for (uint32_t i = tid; i < P; i += blockDim.x)
      {
         if (i < n) { fx.kt[i] = r[i].t; fx.ki[i] = r[i].id; fx.ka[i] = r[i].aux; }
         else { fx.kt[i] = ~0ull; fx.ki[i] = ~0u; fx.ka[i] = 0; }
      }
      __syncthreads();
      bitonic_lds(fx.kt, fx.ki, fx.ka, P);
      for (uint32_t i = tid; i < n; i += blockDim.x)
      {
         Rec o;
         o.t = fx.kt[i];
         o.id = fx.ki[i];
         o.aux = fx.ka[i];
         r[i] = o;
      }
   }
   else if (tid == 0)
   {
      // nearly sorted: insertion sort, O(n + inversions)
      for (uint32_t i = 1; i < n; i++)
      {
         const Rec v = r[i];
         uint32_t j = i;
         while (j > 0 && key_lt(v.t, v.id, r[j - 1].t, r[j - 1].id)) { r[j] = r[j - 1]; j--; }
         r[j] = v;
      }
   }
   __syncthreads();
}

// BC (batches with broadcasts): each input slot is [unicast part | broadcast
// tail]; the tail holds slot_cnt - bcnt.. slot_cnt, filled through btail in
// any order.  Broadcast children are charged the max departure over their
// router visit's ports (router_model.cc:86-101): this pass's value so far
// so far this pass or predicted from the previous pass (bc_visit).
template <bool F1, bool BC>
__global__ __launch_bounds__(STHREADS) void k_port_stream(DevCfg c, const uint32_t* __restrict__ ports,
                                                          const uint32_t* __restrict__ slot_cnt,
                                                          const uint64_t* __restrict__ slot_base,
                                                          Rec* __restrict__ recs, uint64_t* __restrict__ final_ps,
                                                          uint64_t* __restrict__ port_sum, uint64_t* __restrict__ port_cnt,
                                                          uint64_t* __restrict__ port_mg1, uint64_t* __restrict__ port_flit,
                                                          uint64_t* __restrict__ port_last, uint32_t* __restrict__ dirty,
                                                          unsigned int* __restrict__ errflag,
                                                          const uint32_t* __restrict__ bcnt, uint32_t* __restrict__ btail)
{
   constexpr int SMAXIN = BC ? INS + 1 : 4;   // unicast ports have <= 4 non-empty input sides
   constexpr int SMAXE = ST * SMAXIN;
   using Smem = PortSmem<SMAXIN>;
   __shared__ __attribute__((aligned(16))) char smraw[sizeof(Smem) > sizeof(FixSmem) ? sizeof(Smem) : sizeof(FixSmem)];
   __shared__ __attribute__((aligned(16))) char bcraw[BC ? sizeof(BcSmem) : 16];
   Smem& sm = *reinterpret_cast<Smem*>(smraw);
   FixSmem& fx = *reinterpret_cast<FixSmem*>(smraw);
   BcSmem& bs = *reinterpret_cast<BcSmem*>(bcraw);
   const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
   const uint32_t port = ports[blockIdx.x];
   const uint32_t tile = port / PORTS, dir = port % PORTS;
   auto tail_of = [&](uint32_t sl) -> uint32_t { return BC ? bcnt[sl] : 0u; };

   // restore order of input slots a producer flagged (M/G/1 or f != 1 ties)
   for (uint32_t in = 0; in < INS; in++)
   {
      const uint32_t sl = slot_of(tile, dir, in);
      if (dirty[sl])
      {
         fixup_slot(fx, recs + slot_base[sl], slot_cnt[sl] - tail_of(sl));
         if (tid == 0) dirty[sl] = 0;
      }
   }
   __syncthreads();

   // broadcast tails: sorted in LDS as one stream, or (more than BC_CAP) sorted
   // into their slots, which are then streamed whole
   uint32_t ntail = 0;
   bool tails_lds = false;
   if constexpr (BC)
   {
      for (uint32_t in = 0; in < INS; in++) ntail += bcnt[slot_of(tile, dir, in)];
      tails_lds = ntail <= (uint32_t) BC_CAP;
      if (ntail && tails_lds)
      {
         uint32_t P = 1;
         while (P < ntail) P <<= 1;
         uint32_t o = 0;
         for (uint32_t in = 0; in < INS; in++)
         {
            const uint32_t sl = slot_of(tile, dir, in), k = bcnt[sl];
            const Rec* r = recs + slot_base[sl] + (slot_cnt[sl] - k);
            for (uint32_t i = tid; i < k; i += STHREADS) { bs.t[o + i] = r[i].t; bs.i[o + i] = r[i].id; bs.a[o + i] = r[i].aux; }
            o += k;
         }
         for (uint32_t i = ntail + tid; i < P; i += STHREADS) { bs.t[i] = ~0ull; bs.i[i] = ~0u; bs.a[i] = 0; }
         __syncthreads();
         bitonic_lds(bs.t, bs.i, bs.a, P);
      }
      else if (ntail)
      {
         for (uint32_t in = 0; in < INS; in++)
         {
            const uint32_t sl = slot_of(tile, dir, in);
            if (bcnt[sl]) fixup_slot(fx, recs + slot_base[sl], slot_cnt[sl]);
         }
      }
      __syncthreads();
   }

   // input streams (non-empty slots of this port), block-uniform
   uint64_t ib[SMAXIN];
   uint32_t icnt[SMAXIN];
   uint32_t nin = 0;
   for (uint32_t in = 0; in < INS; in++)
   {
      const uint32_t sl = slot_of(tile, dir, in);
      const uint32_t k = slot_cnt[sl] - (tails_lds ? tail_of(sl) : 0u);
      if (k && nin < (uint32_t) SMAXIN) { ib[nin] = slot_base[sl]; icnt[nin] = k; nin++; }
   }
   const int lds_stream = (BC && tails_lds && ntail) ? (int) nin : -1;
   if (lds_stream >= 0) { ib[nin] = 0; icnt[nin] = ntail; nin++; }
   for (uint32_t k = nin; k < (uint32_t) SMAXIN; k++) { ib[k] = 0; icnt[k] = 0; }

   // output: next tile and input side (same for every record of this port)
   uint32_t tx, ty;
   tile_xy(tile, c.W, c.magicW, tx, ty);
   uint32_t ntile = tile, nin_side = IN_LOCAL;
   if (dir == P_RIGHT) { ntile = tile + 1; nin_side = IN_W; }
   else if (dir == P_LEFT) { ntile = tile - 1; nin_side = IN_E; }
   else if (dir == P_UP) { ntile = tile + c.W; nin_side = IN_S; }
   else if (dir == P_DOWN) { ntile = tile - c.W; nin_side = IN_N; }
   uint32_t nx, ny;
   tile_xy(ntile, c.W, c.magicW, nx, ny);
   uint64_t obase[5];
   uint32_t ocap[5], obc[5];   // unicast capacity, broadcast tail of each next slot
   for (uint32_t d = 0; d < 5; d++)
   {
      const uint32_t sl = slot_of(ntile, d, slot_side(d, nin_side));
      obase[d] = slot_base[sl];
      obc[d] = tail_of(sl);
      ocap[d] = slot_cnt[sl] - obc[d];
   }
   uint32_t ocur[5] = { 0, 0, 0, 0, 0 };   // records written per next-direction

   uint32_t cur[SMAXIN] = {};
   uint64_t X0 = 0;                         // carried queue state (cycles)
   uint64_t st_sum = 0, st_cnt = 0, st_flit = 0, st_last = 0;
   bool first_round = true;

   if (tid == 0)
   {
      sm.ss.X = 0; sm.ss.g = 0; sm.ss.mode = 0; sm.ss.s1 = 0; sm.ss.s2 = 0;
      sm.ss.narr = 0; sm.ss.newest = 0; sm.ss.mg1 = 0;
   }

   for (;;)
   {
      uint32_t nl[SMAXIN];
      uint32_t remtot = 0;
      for (uint32_t k = 0; k < SMAXIN; k++)
      {
         const uint32_t rem = icnt[k] - cur[k];
         nl[k] = rem < (uint32_t) ST ? rem : (uint32_t) ST;
         remtot += rem;
      }
      if (remtot == 0) break;

      // ---- load
      for (uint32_t j = tid; j < (uint32_t) SMAXE; j += STHREADS)
      {
         const uint32_t k = j / ST, i = j % ST;
         if (i < nl[k])
         {
            if (BC && (int) k == lds_stream)
            {
               sm.in_t[k][i] = bs.t[cur[k] + i];
               sm.in_id[k][i] = bs.i[cur[k] + i];
               sm.in_aux[k][i] = bs.a[cur[k] + i];
            }
            else
            {
               const Rec r = recs[ib[k] + cur[k] + i];
               sm.in_t[k][i] = r.t;
               sm.in_id[k][i] = r.id;
               sm.in_aux[k][i] = r.aux;
            }
         }
      }
      __syncthreads();

      // ---- bound = min last-loaded key over streams that continue past this round
      uint64_t bt = ~0ull;
      uint32_t bi = ~0u;
      for (uint32_t k = 0; k < SMAXIN; k++)
      {
         if (icnt[k] - cur[k] > nl[k])
         {
            const uint64_t t = sm.in_t[k][nl[k] - 1];
            const uint32_t id = sm.in_id[k][nl[k] - 1];
            if (key_lt(t, id, bt, bi)) { bt = t; bi = id; }
         }
      }

      // ---- merge: rank = own index + #smaller keys in the other streams
      for (uint32_t j = tid; j < (uint32_t) SMAXE; j += STHREADS)
      {
         const uint32_t k = j / ST, i = j % ST;
         if (i >= nl[k]) continue;
         const uint64_t t = sm.in_t[k][i];
         const uint32_t id = sm.in_id[k][i];
         if (!key_le(t, id, bt, bi)) continue;
         uint32_t rank = i;
         for (uint32_t o = 0; o < SMAXIN; o++)
         {
            if (o == k || nl[o] == 0) continue;
            uint32_t lo = 0, hi = nl[o];
            while (lo < hi)
            {
               const uint32_t mid = (lo + hi) >> 1;
               if (key_lt(sm.in_t[o][mid], sm.in_id[o][mid], t, id)) lo = mid + 1; else hi = mid;
            }
            rank += lo;
         }
         sm.m_t[rank] = t;
         sm.m_id[rank] = id;
         sm.m_aux[rank] = sm.in_aux[k][i];
      }
      if (tid < SMAXIN)
      {
         // emitted count of stream tid: upper_bound of the bound key
         uint32_t lo = 0, hi = nl[tid];
         while (lo < hi)
         {
            const uint32_t mid = (lo + hi) >> 1;
            if (key_le(sm.in_t[tid][mid], sm.in_id[tid][mid], bt, bi)) lo = mid + 1; else hi = mid;
         }
         sm.e_cnt[tid] = lo;
      }
      __syncthreads();
      uint32_t E = 0;
      for (uint32_t k = 0; k < SMAXIN; k++) E += sm.e_cnt[k];

      // ---- queue recurrence
      if (first_round)
      {
         first_round = false;
         if (tid == 0 && c.analytical && E > 0 &&
             (c.max_list <= 2 || cyc_of<F1>(sm.m_t[0], c.f) == 0))
         {
            sm.ss.mode = 1;
         }
         __syncthreads();
      }
      if (sm.ss.mode)
      {
         if (tid == 0)
         {
            SerialState s = sm.ss;
            s.X = X0;
            uint32_t e = 0;
            for (; e < E && s.mode; e++)
            {
               const uint64_t tc = cyc_of<F1>(sm.m_t[e], c.f);
               const uint64_t p = aux_F(sm.m_aux[e]);
               sm.m_c[e] = serial_step(s, tc, p, c.max_list, c.analytical);
               if (c.max_list > 2 && s.g >= 1) s.mode = 0;
            }
            sm.s0 = e;
            sm.ss = s;
         }
         __syncthreads();
         X0 = sm.ss.X;
      }
      else if (tid == 0)
      {
         sm.s0 = 0;
      }
      __syncthreads();
      const uint32_t s0 = sm.s0;

      // block max-plus scan over [s0, E): element map X -> max(X + p, tc + p)
      {
         const uint32_t cnt = E - s0;
         const uint32_t per = (cnt + STHREADS - 1) / STHREADS;
         const uint32_t lo = s0 + min(tid * per, cnt), hi = s0 + min((tid + 1) * per, cnt);
         uint64_t A = 0, B = 0;
         for (uint32_t e = lo; e < hi; e++)
         {
            const uint64_t tc = cyc_of<F1>(sm.m_t[e], c.f);
            const uint64_t p = aux_F(sm.m_aux[e]);
            A += p;
            const uint64_t b1 = B + p, b2 = tc + p;
            B = b1 > b2 ? b1 : b2;
         }
         // inclusive wave scan of (A,B) with op (a1,b1).(a2,b2) = (a1+a2, max(b1+a2, b2))
         uint64_t iA = A, iB = B;
         for (int off = 1; off < 64; off <<= 1)
         {
            const uint64_t pA = __shfl_up(iA, off), pB = __shfl_up(iB, off);
            if ((int) lane >= off)
            {
               const uint64_t nb = pB + iA;
               iB = nb > iB ? nb : iB;
               iA = pA + iA;
            }
         }
         if (lane == 63) { sm.wA[wv] = iA; sm.wB[wv] = iB; }
         __syncthreads();
         // prefix of whole waves before this one
         uint64_t PA = 0, PB = 0;
         for (uint32_t w = 0; w < wv; w++)
         {
            const uint64_t nb = PB + sm.wA[w];
            PB = nb > sm.wB[w] ? nb : sm.wB[w];
            PA += sm.wA[w];
         }
         // exclusive within wave
         uint64_t eA = __shfl_up(iA, 1), eB = __shfl_up(iB, 1);
         if (lane == 0) { eA = 0; eB = 0; }
         // combine: prefix(waves) then exclusive(lanes)
         const uint64_t nb = PB + eA;
         const uint64_t CB = nb > eB ? nb : eB;
         const uint64_t CA = PA + eA;
         uint64_t X = X0 + CA;
         X = X > CB ? X : CB;
         for (uint32_t e = lo; e < hi; e++)
         {
            const uint64_t tc = cyc_of<F1>(sm.m_t[e], c.f);
            const uint64_t p = aux_F(sm.m_aux[e]);
            sm.m_c[e] = X > tc ? X - tc : 0;
            X = (X > tc ? X : tc) + p;
         }
         // new carry = X0 composed with the whole block
         uint64_t TA = 0, TB = 0;
         for (uint32_t w = 0; w < STHREADS / 64; w++)
         {
            const uint64_t b = TB + sm.wA[w];
            TB = b > sm.wB[w] ? b : sm.wB[w];
            TA += sm.wA[w];
         }
         const uint64_t nx0 = X0 + TA;
         X0 = nx0 > TB ? nx0 : TB;
      }
      __syncthreads();

      // ---- outputs: route each record; positions by block prefix count per next direction
      {
         const uint32_t per = (E + STHREADS - 1) / STHREADS;
         const uint32_t lo = min(tid * per, E), hi = min((tid + 1) * per, E);
         uint64_t packed = 0;   // 5 x 12-bit counters (unicast children; broadcast ones go to tails)
         for (uint32_t e = lo; e < hi; e++)
         {
            uint32_t ndir = 0;
            if (dir != P_SELF)
            {
               ndir = xy_dir(nx, ny, aux_dx(sm.m_aux[e]), aux_dy(sm.m_aux[e]));
            }
            if (!(BC && (sm.m_aux[e] & AUX_BC))) packed += 1ull << (12 * ndir);
         }
         uint64_t inc = packed;
         for (int off = 1; off < 64; off <<= 1)
         {
            const uint64_t v = __shfl_up(inc, off);
            if ((int) lane >= off) inc += v;
         }
         if (lane == 63) sm.wC[wv] = inc;
         __syncthreads();
         uint64_t pre = inc - packed;
         for (uint32_t w = 0; w < wv; w++) pre += sm.wC[w];
         uint64_t tot = 0;
         for (uint32_t w = 0; w < STHREADS / 64; w++) tot += sm.wC[w];
         for (uint32_t e = lo; e < hi; e++)
         {
            const uint64_t t = sm.m_t[e];
            const uint32_t id = sm.m_id[e], ax = sm.m_aux[e];
            const uint64_t cc = sm.m_c[e];
            // the delay charged: this queue's, or for a broadcast's router visit the
            // max over the visit's ports (bc_visit).
            uint64_t ch = cc;
            const bool bcr = BC && (ax & AUX_BC);
            uint64_t v = 0;
            if (bcr && dir != P_INJ)
            {
               v = (uint64_t) c.bc_idx[id] * c.N + tile;
               const uint64_t tc = cyc_of<F1>(t, c.f);
               ch = bc_visit(c, v, dir, 0x1Fu, tc, cc, bc_win_wait(tc, cc));
            }
            st_sum += ch;
            st_cnt++;
            {
               // QueueModel utilization (queue_model.cc:49-53): F and departure, in cycles
               const uint64_t p = aux_F(ax), dep = cyc_of<F1>(t, c.f) + cc + p;
               st_flit += p;
               st_last = st_last > dep ? st_last : dep;
            }
            const uint64_t tn = t + ps_of<F1>(ch, c.f) + (dir == P_INJ ? 0ull : rl_of(c, tile));
            if (dir == P_SELF)
            {
               const uint64_t fin = tn + ps_of<F1>(aux_F(ax), c.f);
               if (bcr) c.bc_fin[v] = fin;
               else if (id < c.npk) final_ps[id] = fin;   // (a record's id indexes the batch: bounded as k_level's)
               continue;
            }
            Rec o;
            o.t = tn;
            o.id = id;
            o.aux = ax;
            if (bcr)
            {
               // the tree ports at the next router (bc_mask): one record into the
               // broadcast tail of each
               const uint32_t m = bc_mask(aux_dx(ax), aux_dy(ax), nx, ny, c.W, c.H);
               for (uint32_t nd = 0; nd < 5; nd++)
               {
                  if (!((m >> nd) & 1u)) continue;
                  const uint32_t q = atomicAdd(&btail[slot_of(ntile, nd, slot_side(nd, nin_side))], 1u);
                  if (q >= obc[nd]) { atomicOr(errflag, 1u); continue; }
                  recs[obase[nd] + ocap[nd] + q] = o;
               }
               continue;
            }
            const uint32_t ndir = xy_dir(nx, ny, aux_dx(ax), aux_dy(ax));
            const uint32_t r = (uint32_t) ((pre >> (12 * ndir)) & 0xFFF);
            pre += 1ull << (12 * ndir);
            if (ocur[ndir] + r >= ocap[ndir])
            {
               atomicOr(errflag, 1u);   // route-count invariant broken: never write out of the slot
               continue;
            }
            recs[obase[ndir] + ocur[ndir] + r] = o;
         }
         for (uint32_t d = 0; d < 5; d++) ocur[d] += (uint32_t) ((tot >> (12 * d)) & 0xFFF);
      }

      for (uint32_t k = 0; k < SMAXIN; k++) cur[k] += sm.e_cnt[k];
      __syncthreads();
   }

   // ---- per-port counters (RouterModel::updateContentionCounters, router_model.cc:136-144)
   for (int off = 32; off > 0; off >>= 1)
   {
      st_sum += __shfl_down(st_sum, off);
      st_cnt += __shfl_down(st_cnt, off);
   }
   if (lane == 0) { sm.wA[wv] = st_sum; sm.wB[wv] = st_cnt; }
   __syncthreads();
   uint64_t a = 0, b = 0;
   if (tid == 0)
      for (uint32_t w = 0; w < STHREADS / 64; w++) { a += sm.wA[w]; b += sm.wB[w]; }
   __syncthreads();
   for (int off = 32; off > 0; off >>= 1)
   {
      st_flit += __shfl_down(st_flit, off);
      const uint64_t o = __shfl_down(st_last, off);
      st_last = st_last > o ? st_last : o;
   }
   if (lane == 0) { sm.wA[wv] = st_flit; sm.wB[wv] = st_last; }
   __syncthreads();
   if (tid == 0)
   {
      uint64_t fl = 0, la = 0;
      for (uint32_t w = 0; w < STHREADS / 64; w++) { fl += sm.wA[w]; la = la > sm.wB[w] ? la : sm.wB[w]; }
      port_flit[port] = fl;
      port_last[port] = la;
      port_sum[port] = a;
      port_cnt[port] = b;
      port_mg1[port] = sm.ss.mg1;
      // Unicast outputs can leave FIFO order only through M/G/1 requests or, for
      // f != 1, equal-time pairs; mark this port's output slots for the fixup sort.
      if (dir != P_SELF && (sm.ss.mg1 > 0 || !F1))
         for (uint32_t d = 0; d < 5; d++) dirty[slot_of(ntile, d, slot_side(d, nin_side))] = 1;
   }
}

// ----------------------------------------------------------------------------
// Finalize: zero-load and contention per packet (NetPacket fields).
// ----------------------------------------------------------------------------
template <bool F1>
__global__ __launch_bounds__(256) void k_finalize(DevCfg c, uint64_t n, const uint64_t* __restrict__ inj,
                                                  const uint32_t* __restrict__ src, const uint32_t* __restrict__ aux,
                                                  const uint8_t* __restrict__ routed, uint64_t* __restrict__ final_ps,
                                                  uint64_t* __restrict__ zl, uint64_t* __restrict__ cont, int closed_form,
                                                  uint32_t cx0, uint32_t cx1, uint32_t* __restrict__ lat32,
                                                  unsigned* __restrict__ lat_ovf, const uint32_t* __restrict__ gid,
                                                  const uint64_t* __restrict__ fin_glob)
{
   // lat32 (gnoc_fetch_latency): final_ps - inject_ps as u32; one that does not fit
   // sets *lat_ovf.  Undelivered (other rank) and broadcast packets are not written.
   // gid (a partitioned sharded rank): its delivery level wrote the final times by
   // global id into fin_glob; a routed packet's comes from there.
   for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint32_t dx = aux_dx(aux[i]), dy = aux_dy(aux[i]);
      // a sharded engine delivers the packets of its column band (shard.hip); the
      // others are zeroed when results are read (k_mask_unowned), not here
      if (dx < cx0 || dx >= cx1) continue;
      if (aux[i] & AUX_BC) continue;   // k_bcast_final
      if (!(routed[i] & 1))
      {
         zl[i] = 0;
         cont[i] = 0;
         if (lat32)
         {
            const uint64_t l = final_ps[i] - inj[i];
            lat32[i] = (uint32_t) l;
            if (l >> 32) atomicOr(lat_ovf, 1u);
         }
         continue;
      }
      uint32_t sx, sy;
      tile_xy(src[i], c.W, c.magicW, sx, sy);
      const uint64_t hops = (uint64_t) ((sx > dx ? sx - dx : dx - sx) + (sy > dy ? sy - dy : dy - sy) + 1);
      // Hop::Hop accumulates Latency(0) at injection, Latency(R+Lk) per mesh router,
      // Latency(F) at receive (network_model.cc:142-150, 556-563).
      const uint64_t z = c.hop_counter ? ps_of<F1>((hops - 1) * (c.R + c.Lk), c.f) + ps_of<F1>(aux_F(aux[i]), c.f)
                                       : ps_of<F1>(0, c.f) + hops * rl_of(c, src[i]) + ps_of<F1>(aux_F(aux[i]), c.f);
      zl[i] = z;
      uint64_t fin;
      if (closed_form) fin = inj[i] + z;
      else fin = gid ? fin_glob[gid[i]] : final_ps[i];
      if (closed_form || gid) final_ps[i] = fin;
      const uint64_t l = fin - inj[i];
      cont[i] = l - z;
      if (lat32)
      {
         lat32[i] = (uint32_t) l;
         if (l >> 32) atomicOr(lat_ovf, 1u);
      }
   }
}

// Broadcast receipts, one block per broadcast: per receiving tile the
// zero-load delay (H+1 routers of the tree path, then serialization) and the
// contention; the packet's own entries are those of its latest receipt (lowest
// tile on ties).  Closed form (queue models off): receipt = inject + zero-load.
template <bool F1>
__global__ __launch_bounds__(256) void k_bcast_final(DevCfg c, const uint32_t* __restrict__ bid,
                                                     const uint64_t* __restrict__ inj, const uint32_t* __restrict__ src,
                                                     const uint32_t* __restrict__ aux, const uint8_t* __restrict__ routed,
                                                     uint64_t* __restrict__ bfin, uint64_t* __restrict__ bzl,
                                                     uint64_t* __restrict__ bct, uint64_t* __restrict__ final_ps,
                                                     uint64_t* __restrict__ zl, uint64_t* __restrict__ cont, int closed_form)
{
   __shared__ uint64_t bf[256];
   __shared__ uint32_t bt[256];
   const uint32_t b = blockIdx.x, id = bid[b], N = c.N;
   const uint64_t t0 = inj[id];
   const bool mesh = (routed[id] & 1) != 0;
   uint32_t sx, sy;
   tile_xy(src[id], c.W, c.magicW, sx, sy);
   const uint64_t fps = ps_of<F1>(aux_F(aux[id]), c.f);
   uint64_t best = 0;
   uint32_t btile = 0xFFFFFFFFu;
   for (uint32_t tile = threadIdx.x; tile < N; tile += blockDim.x)
   {
      const uint64_t k = (uint64_t) b * N + tile;
      uint64_t f = t0, z = 0;
      if (mesh)
      {
         uint32_t x, y;
         tile_xy(tile, c.W, c.magicW, x, y);
         const uint64_t hops = (uint64_t) ((x > sx ? x - sx : sx - x) + (y > sy ? y - sy : sy - y) + 1);
         z = ps_of<F1>(0, c.f) + hops * c.rl_ps + fps;
         f = closed_form ? t0 + z : bfin[k];
      }
      bfin[k] = f;
      bzl[k] = z;
      bct[k] = f - t0 - z;
      if (btile == 0xFFFFFFFFu || f > best) { best = f; btile = tile; }
   }
   bf[threadIdx.x] = best;
   bt[threadIdx.x] = btile;
   __syncthreads();
   if (threadIdx.x == 0)
   {
      uint64_t f = 0;
      uint32_t tb = 0xFFFFFFFFu;
      for (uint32_t k = 0; k < blockDim.x; k++)
         if (bt[k] != 0xFFFFFFFFu && (tb == 0xFFFFFFFFu || bf[k] > f || (bf[k] == f && bt[k] < tb))) { f = bf[k]; tb = bt[k]; }
      final_ps[id] = f;
      zl[id] = bzl[(uint64_t) b * N + tb];
      cont[id] = bct[(uint64_t) b * N + tb];
   }
}

// Pass check: a visit whose children were not all charged its final max
// departure (min u or max u != max) sets *changed.  Visits no port reached
// (record untouched) are skipped.
__global__ __launch_bounds__(256) void k_bcast_agree(uint64_t nv, const uint64_t* __restrict__ cur,
                                                     unsigned* __restrict__ changed)
{
   bool ch = false;
   unsigned nch = 0;
   uint64_t tmin = ~0ull;
   for (uint64_t k = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; k < nv; k += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint64_t* r = cur + k * BCS;
      const uint64_t m = r[BC_M], lo = ~r[BC_UMIN], hi = r[BC_UMAX];
      if ((m || hi) && (lo != m || hi != m))
      {
         ch = true;
         nch++;
         tmin = m < tmin ? m : tmin;
      }
   }
   if (__ballot(ch) && (threadIdx.x & 63) == 0) atomicOr(changed, 1u);
   if (nch)
   {
      atomicAdd(changed + 1, nch);
      atomicMin((unsigned long long*) (changed + 2), (unsigned long long) tmin);
   }
}

// Results of packets another rank delivers read 0 (gnoc_get_packet_results).
__global__ __launch_bounds__(256) void k_mask_unowned(uint64_t n, const uint32_t* __restrict__ aux, uint32_t cx0,
                                                      uint32_t cx1, uint64_t* __restrict__ final_ps,
                                                      uint64_t* __restrict__ zl, uint64_t* __restrict__ cont)
{
   for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint32_t dx = aux_dx(aux[i]);
      if (dx >= cx0 && dx < cx1) continue;
      final_ps[i] = 0;
      zl[i] = 0;
      cont[i] = 0;
   }
}

// explicit instantiations
#define GNOC_PORT_STREAM_INST(F1V, BCV)                                                                              \
   template __global__ void k_port_stream<F1V, BCV>(DevCfg, const uint32_t*, const uint32_t*, const uint64_t*, Rec*, \
                                                    uint64_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*, \
                                                    uint32_t*, unsigned int*, const uint32_t*, uint32_t*);
GNOC_PORT_STREAM_INST(true, false)
GNOC_PORT_STREAM_INST(false, false)
GNOC_PORT_STREAM_INST(true, true)
GNOC_PORT_STREAM_INST(false, true)
#undef GNOC_PORT_STREAM_INST
template __global__ void k_bcast_final<true>(DevCfg, const uint32_t*, const uint64_t*, const uint32_t*, const uint32_t*,
                                             const uint8_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*,
                                             uint64_t*, int);
template __global__ void k_bcast_final<false>(DevCfg, const uint32_t*, const uint64_t*, const uint32_t*, const uint32_t*,
                                              const uint8_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*,
                                              uint64_t*, int);
template __global__ void k_finalize<true>(DevCfg, uint64_t, const uint64_t*, const uint32_t*, const uint32_t*,
                                          const uint8_t*, uint64_t*, uint64_t*, uint64_t*, int, uint32_t, uint32_t,
                                          uint32_t*, unsigned*, const uint32_t*, const uint64_t*);
template __global__ void k_finalize<false>(DevCfg, uint64_t, const uint64_t*, const uint32_t*, const uint32_t*,
                                           const uint8_t*, uint64_t*, uint64_t*, uint64_t*, int, uint32_t, uint32_t,
                                           uint32_t*, unsigned*, const uint32_t*, const uint64_t*);

}  // namespace gnoc
