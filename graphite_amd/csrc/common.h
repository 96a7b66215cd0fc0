// common.h -- shared device/host definitions of the emesh timing engine.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace gnoc {

// Output ports per tile (network_model_emesh_hop_by_hop.h:43-50) + injection router port.
enum : uint32_t { P_SELF = 0, P_LEFT = 1, P_RIGHT = 2, P_DOWN = 3, P_UP = 4, P_INJ = 5, PORTS = 6 };

// Input sides of a mesh router output port: where the packet came from.
// IN_LOCAL = from this tile's injection router (emesh_hop_by_hop.cc:151-159),
// IN_W/IN_E/IN_S/IN_N = from the neighbour's RIGHT/LEFT/UP/DOWN output.
enum : uint32_t { IN_LOCAL = 0, IN_W = 1, IN_E = 2, IN_S = 3, IN_N = 4, INS = 5 };

// One hop record in HBM: the arrival of packet `id` at an output-port queue at
// time `t` (picoseconds).  aux packs the destination's mesh coordinates and the
// packet's flit count F, so routing needs no division and no gather downstream:
//   aux = dx | dy << 10 | F << 20 | BC << 31   (W, H <= 1024, F <= 2047; checked at submit)
// A broadcast (BC = 1, emesh_hop_by_hop.cc:163-221) carries the SENDER's
// coordinates in (dx, dy): its tree is a function of the sender.
struct __attribute__((aligned(16))) Rec
{
   uint64_t t;
   uint32_t id;
   uint32_t aux;
};
static_assert(sizeof(Rec) == 16, "Rec must be 16 bytes");

constexpr uint32_t AUX_C_BITS = 10;
constexpr uint32_t AUX_C_MASK = (1u << AUX_C_BITS) - 1;
constexpr uint32_t AUX_F_SHIFT = 2 * AUX_C_BITS;
constexpr uint32_t AUX_F_MAX = (1u << (31 - AUX_F_SHIFT)) - 1;
constexpr uint32_t AUX_BC = 1u << 31;
constexpr uint32_t MESH_DIM_MAX = 1u << AUX_C_BITS;

__host__ __device__ inline uint32_t aux_pack(uint32_t dx, uint32_t dy, uint32_t F)
{
   return dx | (dy << AUX_C_BITS) | (F << AUX_F_SHIFT);
}
__host__ __device__ inline uint32_t aux_dx(uint32_t a) { return a & AUX_C_MASK; }
__host__ __device__ inline uint32_t aux_dy(uint32_t a) { return (a >> AUX_C_BITS) & AUX_C_MASK; }
__host__ __device__ inline uint32_t aux_F(uint32_t a) { return (a >> AUX_F_SHIFT) & AUX_F_MAX; }

__host__ __device__ inline uint32_t slot_of(uint32_t tile, uint32_t dir, uint32_t in)
{
   return (tile * PORTS + dir) * INS + in;
}

// Which input side a packet arrives on after leaving through `dir`.
__host__ __device__ inline uint32_t in_side_after(uint32_t dir)
{
   return dir == P_RIGHT ? IN_W : dir == P_LEFT ? IN_E : dir == P_UP ? IN_S : dir == P_DOWN ? IN_N : IN_LOCAL;
}

struct DevCfg
{
   uint32_t W, H, N;
   uint32_t flit_width;
   uint64_t R, Lk;
   double f;
   uint64_t rl_ps;       // Latency(R + Lk, f).toPicosec()
   int contention;
   int analytical;
   int max_list;
   uint32_t magicW;      // ceil(2^32 / W) style reciprocal for tile -> (x, y)
   // Design-space sweep (gnoc_create_sweep): the mesh is a BX-wide grid of
   // independent BW x BH blocks, one per sweep point, each with its own R + Lk
   // and flit width.  A single mesh is one block (pt_rl == nullptr).
   uint32_t BW, BH, BX;
   // NetworkModelEMeshHopCounter (network_model_emesh_hop_counter.cc:143-157):
   // no routers or queues, latency Latency(H * (R + Lk)) in one conversion
   int hop_counter;
   const uint64_t* pt_rl;   // per point Latency(R + Lk).toPicosec()
   const uint32_t* pt_fw;   // per point flit width
   // Broadcast tree (emesh_hop_by_hop.cc:163-221), nullptr without broadcasts.
   // A router visit v = b * N + tile of broadcast b charges the MAX queue delay
   // over its selected ports (router_model.cc:86-101), i.e. its children leave
   // at the latest departure tc + c over those ports.  A pass keeps per visit
   // (one BCS-word record, bc_cur) that max, the min and max departure u its
   // ports' children were charged, and each port's queue neighbourhood
   // (BcWin); u = max(the port's own departure, the max so far, predictions
   // for the visit's ports the level order serves after this one from the
   // previous pass's record, bc_prev).  The pass is exact when every visit's
   // children got u == its final max (bc_visit, engine.hip gnoc_run).
   const uint32_t* bc_idx;  // packet id -> broadcast index
   const uint64_t* bc_prev; // [v * BCS + ...] previous pass
   uint64_t* bc_cur;        // [v * BCS + ...] this pass (zeroed before it)
   uint64_t* bc_fin;        // [b * N + tile] receipt time (ps)
   // packets of the batch: a SELF port never writes final times beyond it.  A sharded
   // rank's partitioned trace (gnoc_submit): records carry global packet ids (their
   // ties order every rank alike), npk is the whole trace's count, and the delivery
   // level writes by global id into an array of that size (k_finalize reads it back
   // through the rank's gid map)
   uint64_t npk;
};

// A broadcast record's neighbourhood in its port's queue (cycles): the
// arrivals of the records just before and after it (a_prev, a_next), the
// busy-until time ahead of it (B), ahead of it were it behind the next record
// (B_next = max(B, a_next) + F_next) and ahead of the previous record (B_pp).
// The next pass predicts the wait of the visit at its new arrival tc' from the
// slot tc' falls in: exact while at most one record is crossed and the
// queue's other records did not move.  Unknown fields: a_prev = tc (nothing
// earlier predicted), a_next = ~0, B_pp = 0.
enum : uint32_t { BCW_AP = 0, BCW_AN = 1, BCW_B = 2, BCW_BN = 3, BCW_BP = 4, BCW = 5 };
// a visit's record: ~min u, max u, max departure, then BcWin of each direction
enum : uint32_t { BC_UMIN = 0, BC_UMAX = 1, BC_M = 2, BC_WIN = 3, BCS = BC_WIN + 5 * BCW };
struct BcWin
{
   uint64_t ap, an, b, bn, bp;
};
__device__ __forceinline__ uint64_t bc_predict(const uint64_t* __restrict__ prev, uint32_t d, uint64_t tc)
{
   // (loading all five fields up front measured slower: register pressure)
   const uint64_t* w = prev + BC_WIN + d * BCW;
   const uint64_t ap = w[BCW_AP], an = w[BCW_AN];
   const uint64_t b = tc < ap ? w[BCW_BP] : tc > an ? w[BCW_BN] : w[BCW_B];
   return b > tc ? b : 0;
}

// One port (direction dir) of broadcast router visit v (selected ports sel):
// arrival cycle tc, own queue delay cc, its queue neighbourhood w.  Returns the delay the visit
// charges this port's child (router_model.cc:86-101).  The level order serves
// X ports, then Y ports, then SELF: a port predicts the ports served after it
// (bc_predict); the ports served before it are in the max so far.
__device__ __forceinline__ uint64_t bc_visit(const DevCfg& c, uint64_t v, uint32_t dir, uint32_t sel, uint64_t tc,
                                             uint64_t cc, const BcWin& w)
{
   uint64_t* r = c.bc_cur + v * BCS;
   const uint64_t* q = c.bc_prev + v * BCS;
   const uint64_t dep = tc + cc;
   const uint64_t so_far = atomicMax((unsigned long long*) (r + BC_M), (unsigned long long) dep);
   uint64_t u = dep > so_far ? dep : so_far;
   if (dir != P_SELF)
   {
      // the visit's selected ports (sel, bc_mask) served after this one
      const uint32_t later = sel & ~(1u << dir) & ~(dir == P_UP || dir == P_DOWN ? (1u << P_LEFT) | (1u << P_RIGHT) : 0u);
      for (uint32_t d = 0; d < 5; d++)
         if ((later >> d) & 1u)
         {
            const uint64_t p = bc_predict(q, d, tc);
            u = u > p ? u : p;
         }
   }
   atomicMax((unsigned long long*) (r + BC_UMIN), (unsigned long long) ~u);
   atomicMax((unsigned long long*) (r + BC_UMAX), (unsigned long long) u);
   uint64_t* o = r + BC_WIN + dir * BCW;
   o[BCW_AP] = w.ap;
   o[BCW_AN] = w.an;
   o[BCW_B] = w.b;
   o[BCW_BN] = w.bn;
   o[BCW_BP] = w.bp;
   return u - tc;
}

// A neighbourhood that only knows the wait itself (serial history-tree mode,
// whole-port streams): predicts busy-until tc + cc when the queue waited.
__device__ __forceinline__ BcWin bc_win_wait(uint64_t tc, uint64_t cc)
{
   BcWin w;
   w.ap = 0;
   w.an = ~0ull;
   w.b = cc ? tc + cc : 0;
   w.bn = w.b;
   w.bp = w.b;
   return w;
}

// Latency::toPicosec, common/misc/time_types.h:81-86.  F1: f == 1.0 exactly,
// where the double expression equals 1000*c for every c < 2^43.
template <bool F1>
__host__ __device__ __forceinline__ uint64_t ps_of(uint64_t c, double f)
{
   if (F1) return c * 1000ull;
   return (uint64_t) ceil(((double) 1000 * (double) c) / f);
}

// Time::toCycles, common/misc/time_types.h:104-109.  F1 fast path is exact for
// ps < 2^42 * 1000 (validated at submit).
template <bool F1>
__host__ __device__ __forceinline__ uint64_t cyc_of(uint64_t ps, double f)
{
   if (F1) return (ps + 999ull) / 1000ull;
   return (uint64_t) ceil(((double) ps * f) / (double) 1.0e3);
}

// tile -> (x, y) with W <= 65535, tile < 2^20: exact via 32x32->64 multiply.
__host__ __device__ __forceinline__ void tile_xy(uint32_t tile, uint32_t W, uint32_t magicW, uint32_t& x, uint32_t& y)
{
   uint32_t q = (uint32_t) (((uint64_t) tile * magicW) >> 32);
   if ((q + 1) * W <= tile) q++;
   if (q * W > tile) q--;
   y = q;
   x = tile - q * W;
}

// Sweep point of a tile, and the per-point delay / flit width (single mesh: the config's).
__host__ __device__ __forceinline__ uint32_t point_of(const DevCfg& c, uint32_t tile)
{
   const uint32_t x = tile % c.W, y = tile / c.W;
   return (y / c.BH) * c.BX + x / c.BW;
}
__host__ __device__ __forceinline__ uint64_t rl_of(const DevCfg& c, uint32_t tile)
{
   return c.pt_rl ? c.pt_rl[point_of(c, tile)] : c.rl_ps;
}
__host__ __device__ __forceinline__ uint32_t fw_of(const DevCfg& c, uint32_t tile)
{
   return c.pt_fw ? c.pt_fw[point_of(c, tile)] : c.flit_width;
}

// Output ports a broadcast from (sx, sy) requests at router (cx, cy),
// network_model_emesh_hop_by_hop.cc:170-204: UP if cy >= sy, DOWN if cy <= sy,
// along the sender's row RIGHT if cx >= sx and LEFT if cx <= sx, and SELF;
// ports towards an off-mesh tile are dropped (computeTileID, :274-280).
__host__ __device__ __forceinline__ uint32_t bc_mask(uint32_t sx, uint32_t sy, uint32_t cx, uint32_t cy, uint32_t W,
                                                     uint32_t H)
{
   uint32_t m = 1u << P_SELF;
   if (cy >= sy && cy + 1 < H) m |= 1u << P_UP;
   if (cy <= sy && cy >= 1) m |= 1u << P_DOWN;
   if (cy == sy)
   {
      if (cx >= sx && cx + 1 < W) m |= 1u << P_RIGHT;
      if (cx <= sx && cx >= 1) m |= 1u << P_LEFT;
   }
   return m;
}

// Input side of a broadcast's record at router (cx, cy): where its tree edge comes from.
__host__ __device__ __forceinline__ uint32_t bc_in_side(uint32_t sx, uint32_t sy, uint32_t cx, uint32_t cy)
{
   return cy > sy ? IN_S : cy < sy ? IN_N : cx > sx ? IN_W : cx < sx ? IN_E : IN_LOCAL;
}

// Input slot side of a record entering port d of a router from side `side`.
// Only a broadcast sender's own SELF request enters SELF from LOCAL (unicast
// self-sends bypass the mesh); it is kept in the S slot, whose records are
// merged with the others anyway, so every port has <= 4 input slots.
__host__ __device__ __forceinline__ uint32_t slot_side(uint32_t d, uint32_t side)
{
   return d == P_SELF && side == IN_LOCAL ? IN_S : side;
}

// Dimension-ordered XY route step, network_model_emesh_hop_by_hop.cc:229-240.
__host__ __device__ __forceinline__ uint32_t xy_dir(uint32_t cx, uint32_t cy, uint32_t dx, uint32_t dy)
{
   return cx > dx ? P_LEFT : cx < dx ? P_RIGHT : cy > dy ? P_DOWN : cy < dy ? P_UP : P_SELF;
}

}  // namespace gnoc
