// pipe.hip -- v6 engine: the X and Y phases of the port DAG as port PIPELINES.
//
// Under XY routing (network_model_emesh_hop_by_hop.cc:229-240) the RIGHT ports of a
// row form a chain RIGHT(0,y) -> RIGHT(1,y) -> ...; LEFT, UP and DOWN ports form
// chains the same way (chain.hip).  A port's arrival stream is the (t, id)-merge of
// the chain's own stream and its insert slots (the injection level's output for an X
// port; IN_LOCAL, IN_W, IN_E turns for a Y port), and every queue is the FIFO
// max-plus recurrence of queue_model_history_tree.cc:66-113.
//
// The chain engine (chain.hip) cuts time into windows and walks a chain's ports once
// per window, handing each port's queue state from window to window through HBM.
// Here ONE WAVE OWNS ONE PORT for the whole batch: its queue state never leaves
// registers, and records stream from port to port in arrival order.
//   * A workgroup holds a SEGMENT of S consecutive ports of one chain (wave w < S is
//     port s S + w) plus one SERVICE wave (w = S).  Port i's continuing records go to
//     port i + 1 through an LDS ring (a write count and a read count in LDS; the
//     producer waits only while the ring is full).
//   * The service wave does every HBM load of the segment: it stages each port's
//     insert lists into LDS rings (converted to the internal form), and, for a segment
//     after the first, pulls the previous segment's continuing records into ring 0.
//     Port waves touch HBM only with fire-and-forget stores, so no port ever waits
//     for memory.
//   * The last port of a segment writes its continuing records into the chain slot
//     (HBM), every 16-B record tagged with the run's epoch (write-through stores;
//     the service wave of the next segment polls them with sc1 loads:
//     MI355X_MICROARCH.md "Valid forms", R2 granules).
//   * Turning records go to the next ports' slots in FIFO order (the level engine's
//     layout, with key samples), read by the next launch.
// A port takes rows of up to 64 records: available chain records merged with its
// inserts.  A record is taken only when nothing that may still arrive on the other
// stream can precede it (the other stream has a later record already, or is
// complete: slot counts are known in advance).  A row is one DPP max-plus scan with
// the tail X as carry-in; ballots rank the outputs per route field.
//
// Internal record (K lo, K hi, id, aux), K = tc << 10 | (1023 - rho): tc is the
// arrival cycle ceil(t / 1000) and rho = 1000 tc - t, constant along a packet's route
// at 1 GHz (t' = t + 1000 (c + R + Lk), network_model.cc:556-563).  K orders as t,
// so (K, id) is the reference's (time, packet id) event order.
//
// Exactness guards (the host reruns the batch on the chain engine when one is
// raised): the history tree's M/G/1 branch would serve a request before the port's
// first idle cycle (queue_model_history_tree.cc:58-64); a time beyond 2^31 cycles;
// unmerged exception tails of the injection level.  A guard never stops a wave:
// every port still writes its whole stream, so no consumer waits forever.
#include "common.h"

namespace gnoc {
namespace pp {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
constexpr int T = 64;
constexpr uint32_t SMAX = 15;          // ports per segment (+1 service wave <= 16 waves)
constexpr uint32_t NLD = 8;            // insert chunks the service wave loads per round
constexpr uint32_t NLK = 8;            // link chunks the service wave loads per round
constexpr uint32_t TC_LIM = 1u << 31;  // arrival cycles stay below (32-bit scan with headroom)
// LDS counter words
constexpr uint32_t C_WC = 0;           // [w] ring w written (by port w-1, or the service wave for w = 0)
constexpr uint32_t C_RC = 16;          // [w] ring w consumed (by port w)
constexpr uint32_t C_SW = 32;          // [3 w + j] insert list j of port w staged (service wave)
constexpr uint32_t C_SR = 80;          // [3 w + j] staged records consumed (port w)
#ifndef PIPE_K
#define PIPE_K 4   // records per lane per block (K = 8: 4.37 ms vs 3.86 ms on configs[1] uniform)
#endif
constexpr uint32_t C_SCR = 128;        // [SCR_W w ..] port w's scratch (the block's insert bitmap)
constexpr uint32_t SCR_W = 16;         // (>= BLK / 32 bitmap words)
constexpr uint32_t C_N = C_SCR + SCR_W * 16;
constexpr uint32_t K = PIPE_K;         // records per lane in a block
constexpr uint32_t KB = K;
constexpr uint32_t BLK = K * 64;       // records per block
static_assert(BLK / 32 <= SCR_W && (BLK / 32) % 4 == 0, "bitmap words in the scratch");
constexpr uint32_t RPAD = 16;          // entries after each ring: a trash entry for branch-free writes
constexpr uint32_t OOB = 0xFFFFFFF0u;  // a buffer offset beyond every descriptor: the store is dropped

struct PipeArgs
{
   const ChainPort* cp;        // this phase's ports [nch * len] (chain.hip k_chain_plan)
   Rec* recs;
   uint64_t* samp_t;
   uint32_t* samp_id;
   unsigned long long* port_sum;
   unsigned long long* port_cnt;
   unsigned long long* port_flit;
   unsigned long long* port_last;
   unsigned* errflag;          // [0] route invariant, [2] exception tails exist, [4] X flags, [5] Y flags
   unsigned* ctr;              // role ticket
   uint32_t nch, len;          // chains of the phase, ports per chain
   uint32_t S;                 // ports per segment
   uint32_t fw;                // this phase's flag word (4: X, 5: Y)
   uint32_t rcap;              // chain ring capacity (records, power of 2, >= 2 NLK * 64)
   uint32_t scap;              // staging ring capacity per insert list (power of 2, >= 128)
   uint32_t mcap;              // merged insert ring per Y port (power of 2, >= 128)
   uint32_t tag;               // link-record epoch tag (1 .. 65535)
   uint32_t excfix;            // k_exc_merge put the injection level's exception tails in order
   uint32_t analytical;        // history tree with the M/G/1 fallback
   uint32_t nsamp;             // key-sample entries
   uint32_t spin_shift;        // a wait longer than 2^spin_shift cycles gives up (F_TIMEOUT)
   uint32_t* dbg;              // (GNOC_PIPE_DEBUG) per port / service wave: its state when it gave up or ended
};
constexpr uint32_t DBG_W = 32;   // words per debug record (16 state, 16 timing); ports at [k], service waves at [nch len + role]
#ifdef PIPE_TIMING
constexpr bool TIMING = true;    // (a -DPIPE_TIMING build) cycles per activity in the debug records
#else
constexpr bool TIMING = false;
#endif

struct __attribute__((aligned(16))) R4   // (16-B aligned: one ds_read_b128 / ds_write_b128 per record)
{
   uint32_t klo, khi, id, aux;
};

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t) __builtin_amdgcn_readfirstlane((int) v); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) { return (uint32_t) __builtin_amdgcn_readlane((int) v, (int) l); }
__device__ __forceinline__ uint64_t key64(const R4& r) { return (uint64_t) r.klo | ((uint64_t) r.khi << 32); }
// (K, id) order: the reference's (time, packet id)
__device__ __forceinline__ bool lt(uint64_t ka, uint32_t ia, uint64_t kb, uint32_t ib)
{
   return ka < kb || (ka == kb && ia < ib);
}
__device__ __forceinline__ R4 r4_inf()
{
   R4 r;
   r.klo = 0xFFFFFFFFu;
   r.khi = 0xFFFFFFFFu;
   r.id = 0xFFFFFFFFu;
   r.aux = 0;
   return r;
}
// An HBM record {t ps, id, aux} in the internal form (Time::toCycles at 1 GHz,
// time_types.h:104-109: tc = ceil(t / 1000)).
__device__ __forceinline__ R4 from_rec(const v4u v, bool& bad)
{
   const uint64_t t = (uint64_t) v.x | ((uint64_t) v.y << 32);
   const uint64_t q = t / 1000ull;
   const uint32_t r = (uint32_t) (t - q * 1000ull);
   const uint64_t tc = q + (r ? 1u : 0u);
   const uint32_t rho = r ? 1000u - r : 0u;
   bad |= tc >= (uint64_t) TC_LIM;
   const uint64_t K = (tc << 10) | (uint64_t) (1023u - rho);
   R4 o;
   o.klo = (uint32_t) K;
   o.khi = (uint32_t) (K >> 32);
   o.id = v.z;
   o.aux = v.w;
   return o;
}

__device__ __forceinline__ void flag(const PipeArgs& a, uint32_t f) { atomicOr(a.errflag + a.fw, f); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, uint32_t bytes)
{
   return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short) 0, (int) bytes, 0x00020000);
}
// slot [base, base + cnt) of the record buffer: range-checked, nothing outside it is read or written
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slot_rsrc(const PipeArgs& a, uint32_t base, uint32_t cnt)
{
   return rsrc_of(a.recs + base, cnt * 16u);
}
constexpr int AUX_SC1 = 16;   // buffer-op cache bits: sc1 (write-through stores, L2-coherent loads)

// LDS counters.  A wave's LDS operations execute in program order, so a count written
// after the ring entries it covers is never seen before them.
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p)
{
   return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v)
{
   __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void csync() { asm volatile("" ::: "memory"); }

// The LDS layout of a segment workgroup.
struct Lay
{
   uint32_t* cnt;
   R4* rings;     // [S][rcap]
   R4* stage;     // [S][NL][scap]
   R4* mbuf;      // [S][mcap] (Y ports: the merged insert stream)
   R4* raw;       // [NLK + NLD][64] the service wave's LDS-DMA landing area (HBM record form)
};
template <int NL>
__device__ __forceinline__ Lay lay_of(const PipeArgs& a, uint4* lds)
{
   Lay L;
   L.cnt = reinterpret_cast<uint32_t*>(lds);
   L.rings = reinterpret_cast<R4*>(lds + C_N / 4);
   L.stage = L.rings + (size_t) a.S * (a.rcap + RPAD);
   L.mbuf = L.stage + (size_t) a.S * NL * a.scap;
   L.raw = L.mbuf + (NL > 1 ? (size_t) a.S * a.mcap : 0);
   return L;
}
template <int NL>
__host__ __device__ inline size_t lds_bytes(uint32_t S, uint32_t rcap, uint32_t scap, uint32_t mcap)
{
   return C_N * 4 + (size_t) S * 16 * (rcap + RPAD + (size_t) NL * scap + (NL > 1 ? mcap : 0)) + (size_t) (NLK + NLD) * 64 * 16;
}

// Entries of the window w[0, av) (a ring from base, mask m; av <= 64) below x: binary
// lifting over positions 0 .. 64 (positions >= av count as +inf), 7 steps so that a
// full window whose 64 entries are all below x gives 64.
__device__ __forceinline__ uint32_t lbw(const R4* s, uint32_t base, uint32_t m, uint32_t av, uint64_t xk, uint32_t xi)
{
   uint32_t pos = 0;
#pragma unroll
   for (uint32_t step = 64; step; step >>= 1)
   {
      const uint32_t idx = pos + step - 1;
      const R4 e = s[(base + idx) & m];
      pos = idx < av && lt(key64(e), e.id, xk, xi) ? pos + step : pos;
   }
   return pos;
}

// ---------------------------------------------------------------------------
// the service wave: every HBM load of the segment
// ---------------------------------------------------------------------------
// Loads land in LDS by LDS-DMA (no registers held across the round trip, rolled
// loops: the port waves' loop stays in the instruction cache), then each chunk is
// checked / converted into its ring.
typedef __attribute__((address_space(3))) void* lptr;
template <int AUX>
__device__ __forceinline__ void dma64(const __amdgpu_buffer_rsrc_t& r, R4* dst, uint32_t voff)
{
   __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lptr) dst, 16, voff, 0, 0, AUX);
}

template <int NL>
__device__ void run_service(const PipeArgs& a, const Lay& L, uint32_t c, uint32_t s, uint32_t np)
{
   const uint32_t lane = threadIdx.x & 63u;
   const uint32_t k0 = c * a.len + s * a.S;
   const uint32_t smask = a.scap - 1u, rmask = a.rcap - 1u;
   // port p's insert lists in lane p: first record and count per list
   uint32_t ib0 = 0, ib1 = 0, ib2 = 0, ic0 = 0, ic1 = 0, ic2 = 0;
   if (lane < np)
   {
      const ChainPort& P = a.cp[k0 + lane];
      ib0 = P.ibase[0];
      ic0 = P.icnt[0];
      if (NL > 1)
      {
         ib1 = P.ibase[1];
         ic1 = P.icnt[1];
         ib2 = P.ibase[2];
         ic2 = P.icnt[2];
      }
   }
   // the previous segment's continuing records (chain slot of port s S - 1)
   const bool link = s > 0;
   const uint32_t nin = link ? a.cp[k0 - 1].ocap[1] : 0u;
   const __amdgpu_buffer_rsrc_t r_link = slot_rsrc(a, link ? a.cp[k0 - 1].obase[1] : 0u, nin);
   uint32_t lf = 0;                      // link records pulled into ring 0
   uint32_t sw0 = 0, sw1 = 0, sw2 = 0;   // lane p: list j records staged
   uint32_t rot = 0;
   bool bad = false;
   const uint64_t t0 = __builtin_amdgcn_s_memtime();
   const uint64_t spin = 1ull << a.spin_shift;
   uint32_t why = 0, rounds = 0, idle = 0, nload = 0, nlink = 0;
   for (;;)
   {
      if (__builtin_amdgcn_s_memtime() - t0 > spin)
      {
         why = 1;
         break;
      }
      // ---- which loads this round: link chunks (as ring 0 has room), insert chunks
      // (as staging rings have room), at most NLD, in a rotating order over (port, list)
      uint32_t nlk = 0;
      if (link && lf < nin)
      {
         const uint32_t room = a.rcap - (lf - rfl(lds_ld(L.cnt + C_RC)));
         nlk = min(min(NLK, room / (uint32_t) T), (nin - lf + T - 1) / (uint32_t) T);
      }
      const uint32_t nb = np * NL;
      uint64_t needm = 0;
#pragma unroll
      for (int j = 0; j < NL; j++)
      {
         const uint32_t swj = j == 0 ? sw0 : j == 1 ? sw1 : sw2, icj = j == 0 ? ic0 : j == 1 ? ic1 : ic2;
         const uint32_t sr = lane < np ? lds_ld(L.cnt + C_SR + 3 * lane + j) : 0u;
         const uint64_t nd = __ballot(lane < np && swj < icj && a.scap - (swj - sr) >= (uint32_t) T);
         // bit p NL + j
         for (uint64_t q = nd; q; q &= q - 1) needm |= 1ull << ((uint32_t) __builtin_ctzll(q) * NL + j);
      }
      const uint64_t full = nb >= 64 ? ~0ull : (1ull << nb) - 1ull;
      const uint32_t rs = rot % nb;
      uint64_t sel = rs ? ((needm >> rs) | (needm << (nb - rs))) & full : needm;
      uint32_t nil = (uint32_t) __popcll(sel);
      while (nil > NLD)
      {
         sel &= ~(1ull << (63 - __builtin_clzll(sel)));
         nil--;
      }
      rot++;
      rounds++;
      if (!nlk && !nil)
      {
         // nothing to load: done, or waiting for room / the previous segment
         const bool more = (link && lf < nin) || __any(lane < np && (sw0 < ic0 || sw1 < ic1 || sw2 < ic2));
         if (!more) break;
         idle++;
         __builtin_amdgcn_s_sleep(2);
         continue;
      }
      nload += nil;
      nlink += nlk;
      // ---- every load of the round into the landing area, then one wait
#pragma unroll 1
      for (uint32_t m = 0; m < nlk; m++) dma64<AUX_SC1>(r_link, L.raw + m * T, (lf + m * T + lane) * 16u);
      {
         uint64_t sq = sel;
#pragma unroll 1
         for (uint32_t m = 0; m < nil; m++)
         {
            const uint32_t v = ((uint32_t) __builtin_ctzll(sq) + rs) % nb, p = v / NL, j = v % NL;
            sq &= sq - 1;
            const uint32_t base = rdl(j == 0 ? ib0 : j == 1 ? ib1 : ib2, p);
            const uint32_t cnt = rdl(j == 0 ? ic0 : j == 1 ? ic1 : ic2, p);
            const uint32_t h = rdl(j == 0 ? sw0 : j == 1 ? sw1 : sw2, p);
            dma64<0>(slot_rsrc(a, base, cnt), L.raw + (NLK + m) * T, (h + lane) * 16u);
         }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // ---- link: the tagged prefix into ring 0
      if (nlk)
      {
         uint32_t got = 0;
#pragma unroll 1
         for (uint32_t m = 0; m < nlk; m++)
         {
            const R4 v = L.raw[m * T + lane];
            const uint32_t g = lf + m * T + lane;
            const bool ok = g < nin && (v.khi >> 16) == a.tag;
            const uint64_t mk = __ballot(ok);
            const uint32_t run = mk == ~0ull ? (uint32_t) T : (uint32_t) __builtin_ctzll(~mk);
            if (lane < run)
            {
               R4 r = v;
               r.khi &= 0xFFFFu;
               L.rings[(lf + m * T + lane) & rmask] = r;
            }
            got += run;
            if (run < (uint32_t) T) break;
         }
         if (got)
         {
            lf += got;
            csync();
            if (lane == 0) lds_st(L.cnt + C_WC, lf);
         }
      }
      // ---- inserts: converted into the staging rings (the same pairs, in the same order)
      uint64_t sq = sel;
#pragma unroll 1
      for (uint32_t m = 0; m < nil; m++)
      {
         const uint32_t v = ((uint32_t) __builtin_ctzll(sq) + rs) % nb, p = v / NL, j = v % NL;
         sq &= sq - 1;
         const uint32_t cnt = rdl(j == 0 ? ic0 : j == 1 ? ic1 : ic2, p);
         const uint32_t h = rdl(j == 0 ? sw0 : j == 1 ? sw1 : sw2, p);
         const uint32_t tk = min((uint32_t) T, cnt - h);
         const R4 rw = L.raw[(NLK + m) * T + lane];
         v4u vv;
         vv.x = rw.klo;
         vv.y = rw.khi;
         vv.z = rw.id;
         vv.w = rw.aux;
         bool b = false;
         const R4 r = from_rec(vv, b);
         bad |= b && lane < tk;
         R4* const st = L.stage + ((size_t) p * NL + j) * a.scap;
         if (lane < tk) st[(h + lane) & smask] = r;
         csync();
         if (lane == 0) lds_st(L.cnt + C_SW + 3 * p + j, h + tk);
         if (lane == p)
         {
            if (j == 0) sw0 += tk;
            else if (j == 1) sw1 += tk;
            else sw2 += tk;
         }
      }
   }
   if (why && lane == 0) flag(a, ch::F_TIMEOUT);
   if (__any(bad) && lane == 0) flag(a, ch::F_FALLBACK | ch::R_TAIL);
   if (a.dbg && lane == 0)
   {
      uint32_t* d = a.dbg + ((size_t) a.nch * a.len + s * a.nch + c) * DBG_W;
      d[0] = 0xC0DE0000u | why;
      d[1] = c;
      d[2] = s;
      d[3] = lf;
      d[4] = nin;
      d[5] = lds_ld(L.cnt + C_RC);
      d[6] = np;
      d[16] = (uint32_t) ((__builtin_amdgcn_s_memtime() - t0) >> 8);
      d[17] = rounds;
      d[18] = idle;
      d[19] = nload;
      d[20] = nlink;
   }
}

// ---------------------------------------------------------------------------
// one port (one wave)
// ---------------------------------------------------------------------------
template <int NL>
__device__ void run_port(const PipeArgs& a, const Lay& L, uint32_t c, uint32_t i, uint32_t w)
{
   constexpr bool XC = NL == 1;
   const uint32_t lane = threadIdx.x & 63u;
   const uint32_t S = a.S, len = a.len, rmask = a.rcap - 1u, smask = a.scap - 1u, mmask = a.mcap - 1u;
   const uint32_t k = c * len + i;
   uint32_t* const cnt = L.cnt;
   R4* const ring_in = L.rings + (size_t) w * (a.rcap + RPAD);
   R4* const ring_out = ring_in + a.rcap + RPAD;
   R4* const trash = ring_out + a.rcap;                 // (writes of lanes with nothing to write)
   R4* const stg = L.stage + (size_t) w * NL * a.scap;
   R4* const mb = L.mbuf + (size_t) w * a.mcap;

   const ChainPort& P = a.cp[k];
   const uint32_t nin = i ? a.cp[k - 1].ocap[1] : 0u;   // the chain stream into this port
   const bool has_next = i + 1 < len;
   const bool out_lds = has_next && w + 1 < S;
   const bool out_hbm = has_next && w + 1 == S;
   const uint32_t nx = P.nx, ny = P.ny;
   const uint32_t rlc = P.rl / 1000u;                   // R + Lk in cycles (1 GHz)
   const uint32_t ic0 = P.icnt[0], ic1 = NL > 1 ? P.icnt[1] : 0u, ic2 = NL > 2 ? P.icnt[2] : 0u;
   const uint32_t nins = ic0 + ic1 + ic2;
   const uint32_t ob0 = P.obase[0], ob1 = P.obase[1], ob2 = XC ? P.obase[2] : 0u, ob3 = XC ? P.obase[3] : 0u;
   const uint32_t oc0 = P.ocap[0], oc1 = P.ocap[1], oc2 = XC ? P.ocap[2] : 0u, oc3 = XC ? P.ocap[3] : 0u;
   // the turn slots of the next tile (SELF, UP, DOWN) as one record range [tlo, thi)
   uint32_t tlo = 0xFFFFFFFFu, thi = 0;
   if (oc0) tlo = ob0, thi = ob0 + oc0;
   if (oc2) tlo = min(tlo, ob2), thi = max(thi, ob2 + oc2);
   if (oc3) tlo = min(tlo, ob3), thi = max(thi, ob3 + oc3);
   if (thi == 0) tlo = 0;

   uint32_t rh = 0;                       // chain records consumed
   uint32_t ih = 0;                       // inserts consumed
   uint32_t mw = 0;                       // (Y) merged inserts written into mb
   uint32_t mh0 = 0, mh1 = 0, mh2 = 0;    // (Y) staged records of each list merged
   uint32_t cnt0 = 0, cnt1 = 0, cnt2 = 0, cnt3 = 0;   // outputs per route field (SELF, cont, UP, DOWN)
   uint32_t X = 0;                        // the queue's tail (cycles)
   bool mode = a.analytical != 0;         // the history tree has had no gap yet
   uint64_t ssum = 0;                     // contention cycles (per lane)
   uint32_t n = 0;
   uint64_t flits = 0;
   bool bad = false;                      // a time beyond the 32-bit cycle range
   bool fired = false;                    // the M/G/1 branch would have served a request
   uint32_t why = 0, rows = 0;
   const uint64_t t0 = __builtin_amdgcn_s_memtime();
   const uint64_t spin = 1ull << a.spin_shift;
   // (-DPIPE_TIMING) cycles by activity: waiting for input, for ring room, merging the Y
   // inserts, rows; rows shorter than 64
   uint64_t tw_in = 0, tw_room = 0, t_merge = 0, t_row = 0;
   uint64_t t_a = 0, t_b = 0, t_c = 0, t_d = 0;   // row parts: counts + candidates + merge loop, row read, scan, outputs
   uint32_t short_rows = 0;

   for (;;)
   {
      uint64_t tm0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
      // ---- (Y) the three staged insert lists merged into one stream, 64 at a time:
      // a record's merged position is its index plus its rank in the other two
      // windows; it is taken when that position is < 64 and no record that is not
      // staged yet can precede it (a list still loading bounds the others by its
      // last staged record)
      if (NL == 3 && mw < nins && a.mcap - (mw - ih) >= (uint32_t) T)
      {
         const uint32_t s0 = rfl(lds_ld(cnt + C_SW + 3 * w)), s1 = rfl(lds_ld(cnt + C_SW + 3 * w + 1)),
                        s2 = rfl(lds_ld(cnt + C_SW + 3 * w + 2));
         csync();
         const uint32_t a0 = min(s0 - mh0, (uint32_t) T), a1 = min(s1 - mh1, (uint32_t) T), a2 = min(s2 - mh2, (uint32_t) T);
         const R4* const q0 = stg;
         const R4* const q1 = stg + a.scap;
         const R4* const q2 = stg + 2 * a.scap;
         const R4 c0 = lane < a0 ? q0[(mh0 + lane) & smask] : r4_inf();
         const R4 c1 = lane < a1 ? q1[(mh1 + lane) & smask] : r4_inf();
         const R4 c2 = lane < a2 ? q2[(mh2 + lane) & smask] : r4_inf();
         const uint64_t k0 = key64(c0), k1 = key64(c1), k2 = key64(c2);
         // bound: the last staged record of each list that is still loading (no bound
         // when it has a full window staged: later records have positions >= 64)
         uint64_t bk = ~0ull;
         uint32_t bi = 0xFFFFFFFFu;
         bool none = false;
         auto bound = [&](uint32_t sv, uint32_t icn, uint32_t av, const R4& cv) {
            if (sv >= icn || av >= (uint32_t) T) return;
            if (!av)
            {
               none = true;
               return;
            }
            const uint64_t lk = (uint64_t) rdl(cv.klo, av - 1) | ((uint64_t) rdl(cv.khi, av - 1) << 32);
            const uint32_t li = rdl(cv.id, av - 1);
            if (lt(lk, li, bk, bi))
            {
               bk = lk;
               bi = li;
            }
         };
         bound(s0, ic0, a0, c0);
         bound(s1, ic1, a1, c1);
         bound(s2, ic2, a2, c2);
         if (!none && (a0 | a1 | a2))
         {
            const uint32_t p0 = lane + lbw(q1, mh1, smask, a1, k0, c0.id) + lbw(q2, mh2, smask, a2, k0, c0.id);
            const uint32_t p1 = lane + lbw(q0, mh0, smask, a0, k1, c1.id) + lbw(q2, mh2, smask, a2, k1, c1.id);
            const uint32_t p2 = lane + lbw(q0, mh0, smask, a0, k2, c2.id) + lbw(q1, mh1, smask, a1, k2, c2.id);
            const bool t0k = lane < a0 && p0 < (uint32_t) T && !lt(bk, bi, k0, c0.id);
            const bool t1k = lane < a1 && p1 < (uint32_t) T && !lt(bk, bi, k1, c1.id);
            const bool t2k = lane < a2 && p2 < (uint32_t) T && !lt(bk, bi, k2, c2.id);
            if (t0k) mb[(mw + p0) & mmask] = c0;
            if (t1k) mb[(mw + p1) & mmask] = c1;
            if (t2k) mb[(mw + p2) & mmask] = c2;
            const uint32_t n0 = (uint32_t) __popcll(__ballot(t0k)), n1 = (uint32_t) __popcll(__ballot(t1k)),
                           n2 = (uint32_t) __popcll(__ballot(t2k));
            mh0 += n0;
            mh1 += n1;
            mh2 += n2;
            mw += n0 + n1 + n2;
            csync();
            if (lane == 0)
            {
               lds_st(cnt + C_SR + 3 * w, mh0);
               lds_st(cnt + C_SR + 3 * w + 1, mh1);
               lds_st(cnt + C_SR + 3 * w + 2, mh2);
            }
         }
         if (TIMING)
         {
            const uint64_t tm1 = __builtin_amdgcn_s_memtime();
            t_merge += tm1 - tm0;
            tm0 = tm1;
         }
      }
      // ---- the two streams: chain records in ring_in, inserts (staged list 0 / merged)
      const uint32_t iw = NL == 1 ? rfl(lds_ld(cnt + C_SW + 3 * w)) : mw;
      const uint32_t iav = iw - ih;
      const bool idone = iw >= nins;
      uint32_t rav = 0;
      bool rdone = true;
      if (i)
      {
         rav = rfl(lds_ld(cnt + C_WC + w)) - rh;
         rdone = rh + rav >= nin;
      }
      csync();   // (the entries are read after the counts)
      const R4* const ib = NL == 1 ? stg : mb;
      const uint32_t imask = NL == 1 ? smask : mmask;
      const uint32_t na = min(rav, BLK), ni = min(iav, (uint32_t) T);

      // ---- the block: up to BLK records in merged order.  Each window insert's rank
      // among the chain candidates (binary search over the ring), its merged position
      // = index + rank; an insert is in the block when that is < BLK and no chain
      // record not written yet may precede it (monotone: a prefix of the window)
      uint32_t nblk = 0, qv = 0;
      if (rav | iav)
      {
         uint32_t rank = 0;
         if (ni)
         {
            // rank = chain candidates below the insert: three levels of a k-ary search
            // (strides 64, 8, 1; the pivots of a level are read together, so the search
            // costs three LDS round trips)
            const R4 I = ib[(ih + lane) & imask];   // (lanes >= ni: not used)
            const uint64_t ik = key64(I);
#pragma unroll
            for (uint32_t step = BLK; step; step >>= 1)
            {
               const uint32_t idx = rank + step - 1;
               const R4 e = ring_in[(rh + idx) & rmask];
               rank = idx < na && lt(key64(e), e.id, ik, I.id) ? rank + step : rank;
            }
         }
         const uint32_t P0 = lane + rank;
         const uint64_t vm = __ballot(lane < ni && (rdone || rank < rav) && P0 < BLK);
         qv = vm == ~0ull ? (uint32_t) T : (uint32_t) __builtin_ctzll(~vm);
         nblk = min(BLK, na + qv);
         if (qv == ni && (ni < iav || !idone))
         {
            // every window insert is in the block and another insert (not loaded, or
            // not staged yet) may come next: chain records after the last one wait
            nblk = ni ? min(nblk, rdl(P0, ni - 1) + 1) : 0u;
         }
         // the inserts' merged positions as a bitmap (LDS, BLK bits)
         if (nblk)
         {
            uint32_t* const bm = cnt + C_SCR + SCR_W * w;
            if (lane < BLK / 32) bm[lane] = 0u;
            csync();
            if (lane < qv) atomicOr(bm + (P0 >> 5), 1u << (P0 & 31u));
            csync();
         }
      }
      if (!nblk)
      {
         if (rdone && idone && !rav && !iav) break;   // the port's whole stream has passed
         if (__builtin_amdgcn_s_memtime() - t0 > spin)
         {
            why = 1;
            break;
         }
         if (TIMING) tw_in += __builtin_amdgcn_s_memtime() - tm0;
         __builtin_amdgcn_s_sleep(1);
         continue;
      }
      rows++;
      uint64_t tp = 0;
      if (TIMING)
      {
         short_rows += nblk < BLK ? 1u : 0u;
         tp = __builtin_amdgcn_s_memtime();
         t_a += tp - tm0;
      }
      // ---- lane L takes merged positions K L .. K L + K - 1: inserts before them from
      // the bitmap's word prefix counts, then each record from its ring
      R4 x[KB];
      {
         // the 8 bitmap words in every lane (two broadcast reads), lane L's word (L / 8)
         // and the inserts in the words before it
         constexpr uint32_t NW = BLK / 32;                   // bitmap words
         const uint4* const bm4 = reinterpret_cast<const uint4*>(cnt + C_SCR + SCR_W * w);
         uint32_t bw[NW];
#pragma unroll
         for (uint32_t d = 0; d < NW / 4; d++)
         {
            const uint4 v = bm4[d];
            bw[4 * d] = v.x;
            bw[4 * d + 1] = v.y;
            bw[4 * d + 2] = v.z;
            bw[4 * d + 3] = v.w;
         }
         const uint32_t pb = K * lane;                       // first position of this lane
         const uint32_t wi = pb >> 5, bo = pb & 31u;
         uint32_t mwd = 0, pc = 0, run = 0;
#pragma unroll
         for (uint32_t d = 0; d < NW; d++)
         {
            mwd = wi == d ? bw[d] : mwd;
            pc = wi == d ? run : pc;
            run += __builtin_popcount(bw[d]);
         }
         uint32_t before = pc + __builtin_popcount(mwd & ((1u << bo) - 1u));
#pragma unroll
         for (uint32_t j = 0; j < KB; j++)
         {
            const uint32_t pos = pb + j;
            const bool isI = (mwd >> (bo + j)) & 1u;
            x[j] = r4_inf();
            if (pos < nblk) x[j] = isI ? ib[(ih + before) & imask] : ring_in[(rh + pos - before) & rmask];
            before += isI ? 1u : 0u;
         }
      }
      rh += nblk - qv;
      ih += qv;
      csync();
      if (lane == 0)
      {
         if (i) lds_st(cnt + C_RC + w, rh);               // ring room back to its producer
         if (NL == 1) lds_st(cnt + C_SR + 3 * w, ih);     // staging room back to the service wave
      }
      if (TIMING)
      {
         __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the block has landed
         const uint64_t tq = __builtin_amdgcn_s_memtime();
         t_b += tq - tp;
         tp = tq;
      }

      // ---- FIFO max-plus recurrence: lane-serial composition of its K records, one
      // wave scan of the lane aggregates, then the lane replays its records from its
      // carry-in
      uint32_t tc[KB], F[KB];
      bool vd[KB];
      uint32_t A = 0, B = 0;
#pragma unroll
      for (uint32_t j = 0; j < KB; j++)
      {
         vd[j] = K * lane + j < nblk;
         tc[j] = __builtin_amdgcn_alignbit(x[j].khi, x[j].klo, 10);   // K >> 10
         F[j] = vd[j] ? aux_F(x[j].aux) : 0u;
         const uint32_t bj = vd[j] ? tc[j] + F[j] : 0u;
         const uint32_t nb = B + F[j];
         B = nb > bj ? nb : bj;
         A += F[j];
      }
      ch::wave_scan(A, B);
      const uint32_t exA = ch::dpp32<0x138, 0xF, 0xF>(A), exB = ch::dpp32<0x138, 0xF, 0xF>(B);   // wave_shr 1
      const uint32_t Atot = ch::rdl(A, 63), Btot = ch::rdl(B, 63);
      uint32_t Xl;
      {
         const uint32_t xa = X + exA;
         Xl = xa > exB ? xa : exB;                       // the tail ahead of this lane's first record
      }
      uint32_t tcn[KB];
      uint32_t fg = 0xFFFFu, ff = 0xFFFFu;              // (no gap yet) first gap / firing, by block position
      uint32_t csum = 0;
#pragma unroll
      for (uint32_t j = 0; j < KB; j++)
      {
         const uint32_t Xm = Xl > tc[j] ? Xl : tc[j];
         if (mode)
         {
            // no idle cycle yet: the first request that finds the queue idle makes a gap
            // for good (:79-86); the M/G/1 branch serves one with X > t + p before it (:58-64)
            const uint64_t gm = __ballot(vd[j] && tc[j] > Xl), fm = __ballot(vd[j] && Xl > tc[j] + F[j]);
            if (gm) fg = min(fg, K * (uint32_t) __builtin_ctzll(gm) + j);
            if (fm) ff = min(ff, K * (uint32_t) __builtin_ctzll(fm) + j);
         }
         csum += vd[j] ? Xm - tc[j] : 0u;                // contention (cycles)
         tcn[j] = Xm + rlc;                              // arrival cycle at the next port
         bad |= vd[j] && tcn[j] >= TC_LIM;
         Xl = Xm + F[j];
      }
      if (mode)
      {
         if (ff < fg) fired = true;
         if (fg != 0xFFFFu) mode = false;
      }
      {
         const uint32_t xo = X + Atot;
         X = xo > Btot ? xo : Btot;
      }
      flits += Atot;
      n += nblk;
      ssum += csum;
      if (TIMING)
      {
         const uint64_t tq = __builtin_amdgcn_s_memtime() + (tcn[0] & 0);   // (after the scan's result)
         t_c += tq - tp;
         tp = tq;
      }

      // ---- outputs: per route field, a record's rank = the block's records of its field
      // before it (packed 16-bit counts: fields 0 | 1 and 2 | 3, exclusive wave prefix)
      uint32_t fd[KB];
      uint32_t c01 = 0, c23 = 0;
#pragma unroll
      for (uint32_t j = 0; j < KB; j++)
      {
         const uint32_t dx = x[j].aux & AUX_C_MASK, dy = (x[j].aux >> AUX_C_BITS) & AUX_C_MASK;
         fd[j] = XC ? (dx != nx ? 1u : dy > ny ? 2u : dy < ny ? 3u : 0u) : (dy != ny ? 1u : 0u);
         if (vd[j])
         {
            if (fd[j] < 2u) c01 += 1u << (16u * fd[j]);
            else c23 += 1u << (16u * (fd[j] - 2u));
         }
      }
      uint32_t p01 = ch::wave_sum32_incl(c01), p23 = XC ? ch::wave_sum32_incl(c23) : 0u;
      const uint32_t t01 = ch::rdl(p01, 63), t23 = XC ? ch::rdl(p23, 63) : 0u;
      p01 -= c01;
      p23 -= c23;
      const uint32_t nc = t01 >> 16;                      // continuing records of the block
      if (nc && out_lds)
      {
         // room in the next port's ring
         const uint64_t tr0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
         while (cnt1 + nc - rfl(lds_ld(cnt + C_RC + w + 1)) > a.rcap)
         {
            if (__builtin_amdgcn_s_memtime() - t0 > spin)
            {
               why = 2;
               break;
            }
            __builtin_amdgcn_s_sleep(1);
         }
         if (why) break;
         if (TIMING) tw_room += __builtin_amdgcn_s_memtime() - tr0;
      }
      const __amdgpu_buffer_rsrc_t r1 = slot_rsrc(a, ob1, out_hbm ? oc1 : 0u);
      const __amdgpu_buffer_rsrc_t rT = slot_rsrc(a, tlo, thi - tlo);   // the turn slots (one range)
      // each turn field's next position, relative to tlo
      const uint32_t rb0 = ob0 - tlo + cnt0, rb2 = ob2 - tlo + cnt2, rb3 = ob3 - tlo + cnt3;
      // branch-free per record: a lane with nothing to write for a target writes the
      // trash entry (LDS) or an out-of-range offset (buffer stores drop it)
#pragma unroll
      for (uint32_t j = 0; j < KB; j++)
      {
         const uint32_t f = fd[j];
         const bool lo = f < 2u;
         const uint32_t sh = (f & 1u) * 16u;
         const uint32_t pos = ((lo ? p01 : p23) >> sh) & 0xFFFFu;
         const uint32_t inc = vd[j] ? 1u << sh : 0u;
         p01 += lo ? inc : 0u;
         p23 += lo ? 0u : inc;
         const bool isc = vd[j] && f == 1u, ist = vd[j] && f != 1u;
         // continuing: the next port's ring (or the next segment's link slot)
         R4 o;
         o.klo = (tcn[j] << 10) | (x[j].klo & 1023u);
         o.khi = tcn[j] >> 22;
         o.id = x[j].id;
         o.aux = x[j].aux;
         if (out_lds) *(isc ? ring_out + ((cnt1 + pos) & rmask) : trash) = o;
         else if (out_hbm)
         {
            v4u l;
            l.x = o.klo;
            l.y = o.khi | (a.tag << 16);
            l.z = o.id;
            l.w = o.aux;
            __builtin_amdgcn_raw_buffer_store_b128(l, r1, isc ? (cnt1 + pos) * 16u : OOB, 0, AUX_SC1);
         }
         // turning: the next ports' slots, HBM records {t', id, aux} (t' = 1000 tc' - rho)
         const uint64_t tn = (uint64_t) tcn[j] * 1000ull + (uint64_t) (x[j].klo & 1023u) - 1023ull;
         v4u hv;
         hv.x = (uint32_t) tn;
         hv.y = (uint32_t) (tn >> 32);
         hv.z = x[j].id;
         hv.w = x[j].aux;
         const uint32_t gp = (f == 0u ? rb0 : f == 2u ? rb2 : rb3) + pos;   // relative to tlo
         __builtin_amdgcn_raw_buffer_store_b128(hv, rT, ist ? gp * 16u : OOB, 0, 0);
      }
      if (nc && out_lds)
      {
         csync();
         if (lane == 0) lds_st(cnt + C_WC + w + 1, cnt1 + nc);
      }
      cnt0 += t01 & 0xFFFFu;
      cnt1 += nc;
      cnt2 += t23 & 0xFFFFu;
      cnt3 += t23 >> 16;
      if (TIMING)
      {
         const uint64_t tq = __builtin_amdgcn_s_memtime();
         t_row += tq - tm0;
         t_d += tq - tp;
      }
   }

   // ---- the port's counters (RouterModel::_total_contention_delay / _total_packets,
   // router_model.cc:136-144) and the route-count invariant
   const uint64_t stot = ch::rdl64(ch::wave_sum64(ssum), 63);
   if (lane == 0)
   {
      if (n)
      {
         a.port_sum[P.port] = stot;
         a.port_cnt[P.port] = n;
         a.port_flit[P.port] = flits;
         a.port_last[P.port] = X;
      }
      if (why) flag(a, ch::F_TIMEOUT);
      else if (cnt0 != oc0 || cnt1 != oc1 || cnt2 != oc2 || cnt3 != oc3) flag(a, ch::F_ROUTE);
      if (fired) flag(a, ch::F_FALLBACK | ch::R_MG1);
   }
   if (__any(bad) && lane == 0) flag(a, ch::F_FALLBACK | ch::R_TAIL);
   if (a.dbg && lane == 0)
   {
      uint32_t* d = a.dbg + (size_t) k * DBG_W;
      d[0] = 0xB0DE0000u | why;
      d[1] = i;
      d[2] = w;
      d[3] = rh;
      d[4] = nin;
      d[5] = ih;
      d[6] = nins;
      d[7] = NL == 1 ? lds_ld(cnt + C_SW + 3 * w) : mw;
      d[8] = i ? lds_ld(cnt + C_WC + w) : 0u;
      d[9] = cnt1;
      d[10] = oc1;
      d[11] = mw;
      d[12] = mh0;
      d[13] = mh1;
      d[14] = mh2;
      d[15] = rows;
      d[16] = (uint32_t) ((__builtin_amdgcn_s_memtime() - t0) >> 8);
      d[17] = (uint32_t) (tw_in >> 8);
      d[18] = (uint32_t) (tw_room >> 8);
      d[19] = (uint32_t) (t_merge >> 8);
      d[20] = (uint32_t) (t_row >> 8);
      d[21] = short_rows;
      d[22] = n;
      d[23] = (uint32_t) (t_a >> 8);
      d[24] = (uint32_t) (t_b >> 8);
      d[25] = (uint32_t) (t_c >> 8);
      d[26] = (uint32_t) (t_d >> 8);
   }
}

// The key samples (every 64th record's key, level.hip) of the SELF slots, which the
// SELF level after the pipelines searches; the pipelines' own streams need none.
// One workgroup per (tile, input side) slot.
__global__ __launch_bounds__(256) void k_pipe_samples(uint32_t N, const uint32_t* __restrict__ slot_cnt,
                                                      const uint64_t* __restrict__ slot_base, const Rec* __restrict__ recs,
                                                      uint64_t* __restrict__ samp_t, uint32_t* __restrict__ samp_id)
{
   const uint32_t tile = blockIdx.x / INS, side = blockIdx.x % INS;
   if (tile >= N) return;
   const uint32_t sl = slot_of(tile, P_SELF, side);
   const uint64_t b = slot_base[sl];
   const uint32_t n = slot_cnt[sl];
   for (uint32_t q = threadIdx.x; q * 64u < n; q += blockDim.x)
   {
      const uint64_t r = b + (uint64_t) q * 64u;   // (slots start 64-record aligned)
      samp_t[r >> 6] = recs[r].t;
      samp_id[r >> 6] = recs[r].id;
   }
}

// One workgroup = one segment of one chain: S port waves and the service wave.  The
// role comes from a ticket, so a segment's producer (the same chain's previous
// segment, a smaller ticket) is always running or done.
template <int NL>
__global__ __launch_bounds__(1024) void k_pipe(PipeArgs a)
{
   extern __shared__ uint4 lds[];
   __shared__ uint32_t role_s;
   // the X phase declined (its outputs are incomplete), or the injection level left
   // exception tails the engine has not merged: the batch reruns on the chain engine
   if (a.fw != 4 && (a.errflag[4] & ch::F_ANY)) return;
   if (a.errflag[2] != 0 && (!a.excfix || (a.errflag[2] & 2u)))
   {
      if (threadIdx.x == 0 && blockIdx.x == 0) flag(a, ch::F_FALLBACK | ch::R_EXC);
      return;
   }
   if (threadIdx.x == 0) role_s = atomicAdd(a.ctr, 1u);
   for (uint32_t q = threadIdx.x; q < C_N; q += blockDim.x) reinterpret_cast<uint32_t*>(lds)[q] = 0u;
   __syncthreads();
   const uint32_t role = rfl(role_s);
   const uint32_t w = rfl(threadIdx.x >> 6);
   const uint32_t c = role % a.nch, s = role / a.nch;
   const uint32_t i0 = s * a.S;
   if (i0 >= a.len) return;
   const uint32_t np = min(a.S, a.len - i0);
   const Lay L = lay_of<NL>(a, lds);
   if (w == a.S) run_service<NL>(a, L, c, s, np);
   else if (w < np) run_port<NL>(a, L, c, i0 + w, w);
}

}  // namespace pp
}  // namespace gnoc
