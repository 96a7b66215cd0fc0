// shard.hip -- one mesh over several GPUs: the XY turn exchange (gfx950).
//
// XY routing (network_model_emesh_hop_by_hop.cc:229-240) takes a packet along
// the X chain of its SOURCE row, then along the Y chain of its DESTINATION
// column.  So the port DAG splits into two phases with one hand-off between
// them:
//   X phase  injection + LEFT/RIGHT ports, owned by ROW band r = rows [r*H/n, (r+1)*H/n)
//   Y phase  UP/DOWN + SELF ports,          owned by COLUMN band c = cols [c*W/n, (c+1)*W/n)
// Every routed packet has exactly one "turn" record: its arrival at the first
// Y-direction port (UP, DOWN or SELF) of tile (dx, sy).  Those records sit in
// the turn slots (tile, dir in {SELF, DOWN, UP}, in-side in {LOCAL, W, E}),
// written by the row-band owner of sy and read by the column-band owner of dx.
// After the X phase each rank packs, per peer d, the turn slots of the tiles in
// (its rows) x (d's columns); one all-to-all moves them (RCCL over xGMI via
// torch.distributed, or any transport the caller owns); the receiver unpacks
// them into the same slot positions, rebuilds the 1-in-64 key samples and the
// exception counts, and runs the Y phase.  Results are bit-identical to the
// single-GPU run because every port still sees exactly the same arrival
// stream.
//
// Buffer layout per (r -> d) pair, in 16-byte units:
//   [ status ][ nexc of the pair's turn slots, u32 each, padded to 16 B ][ records, slot order ]
// Pair slot order: tiles row-major over (rows(r) x cols(d)), 9 slots per tile.
// The status unit carries the sender's X-phase outcome: nonzero when its X phase
// did not complete (a chain decline, a level the chunked path could not finish, a
// route-count error, or a host-side failure that left the buffer unpacked).  The
// receiver then raises its own X flag word, so its Y chains and levels return at
// once instead of reading the peer's incomplete turn slots; the step's status
// all-reduce makes every rank rerun it (engine.hip gnoc_run_sharded).
#include "common.h"

namespace gnoc {

constexpr uint32_t XS_PER_TILE = 9;

struct XPair
{
   uint32_t x0, nx, y0, ny;   // the pair's tile rectangle
   uint64_t hdr_unit;         // header position in the buffer (16-B units)
   uint64_t rec_unit;         // first record's position in the buffer
   uint64_t expect;           // records the pair must carry (host count at submit)
   uint32_t slot0, nslots;    // this pair's range in the flattened slot list
};

__device__ __forceinline__ uint32_t xs_slot(const XPair& p, uint32_t k, uint32_t W)
{
   const uint32_t tl = k / XS_PER_TILE, j = k - tl * XS_PER_TILE;
   const uint32_t dj = j / 3, in = j - dj * 3;
   const uint32_t dir = dj == 0 ? P_SELF : dj == 1 ? P_DOWN : P_UP;   // in-side: IN_LOCAL, IN_W, IN_E
   const uint32_t ty = tl / p.nx, tx = tl - ty * p.nx;
   return slot_of((p.y0 + ty) * W + p.x0 + tx, dir, in);
}

constexpr uint32_t XR_PEER = 1u << 16;   // errflag[4] reason bit: a peer's X phase did not complete

// One block per pair: exclusive scan of the pair's slot counts -> each slot's
// first record position in the buffer.  Checks the pair total against the
// host's count (route invariant, errflag bit 0).  Send side (buf = the send
// buffer): the pair's status unit from this rank's X-phase flags.  Receive side
// (buf = the received buffer): a peer's nonzero status raises the X flag word.
__global__ __launch_bounds__(1024) void k_x_layout(uint32_t W, const XPair* __restrict__ pairs,
                                                   const uint32_t* __restrict__ slot_cnt,
                                                   uint64_t* __restrict__ xoff, unsigned* __restrict__ errflag,
                                                   uint4* __restrict__ buf, int recv_side)
{
   __shared__ uint64_t part[1024];
   const XPair p = pairs[blockIdx.x];
   if (recv_side && threadIdx.x == 0)
   {
      const uint4 st = buf[p.hdr_unit];
      if (st.x | st.y | st.z | st.w) atomicOr(errflag + 4, 2u | XR_PEER);   // ch::F_FALLBACK | XR_PEER
   }
   uint64_t carry = 0;
   for (uint32_t k0 = 0; k0 < p.nslots; k0 += 1024)
   {
      const uint32_t k = k0 + threadIdx.x;
      const uint64_t v = k < p.nslots ? slot_cnt[xs_slot(p, k, W)] : 0;
      part[threadIdx.x] = v;
      __syncthreads();
      for (uint32_t off = 1; off < 1024; off <<= 1)
      {
         const uint64_t a = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
         __syncthreads();
         part[threadIdx.x] += a;
         __syncthreads();
      }
      if (k < p.nslots) xoff[p.slot0 + k] = p.rec_unit + carry + part[threadIdx.x] - v;
      carry += part[1023];
      __syncthreads();
   }
   if (threadIdx.x == 0 && carry != p.expect) atomicOr(errflag, 1u);
   if (!recv_side && threadIdx.x == 0)
   {
      // this rank's X phase: level errors (route, look-back timeout, unsplittable
      // leaf) and chain flags; written after this pair's own count check
      const unsigned e0 = __hip_atomic_load(errflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned e4 = __hip_atomic_load(errflag + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      buf[p.hdr_unit] = make_uint4((e0 & 7u) | (carry != p.expect ? 1u : 0u), e4 & 0xFu, 0u, 0u);
   }
}

__device__ __forceinline__ uint32_t xs_pair_of(const XPair* __restrict__ pairs, uint32_t np, uint32_t w)
{
   uint32_t q = 0;
   while (q + 1 < np && w >= pairs[q + 1].slot0) q++;
   return q;
}

// One wave per turn slot: its records into the send buffer, its exception count
// into the pair header.
__global__ __launch_bounds__(256) void k_x_pack(uint32_t W, const XPair* __restrict__ pairs, uint32_t np,
                                                uint32_t total_slots, const uint64_t* __restrict__ xoff,
                                                const uint32_t* __restrict__ slot_cnt,
                                                const uint64_t* __restrict__ slot_base, const uint32_t* __restrict__ nexc,
                                                const Rec* __restrict__ recs, uint4* __restrict__ buf)
{
   const uint32_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64, lane = threadIdx.x & 63;
   if (w >= total_slots) return;
   const uint32_t q = xs_pair_of(pairs, np, w);
   const XPair p = pairs[q];
   const uint32_t k = w - p.slot0;
   const uint32_t s = xs_slot(p, k, W);
   const uint32_t n = slot_cnt[s];
   const uint4* src = reinterpret_cast<const uint4*>(recs + slot_base[s]);
   uint4* dst = buf + xoff[w];
   for (uint32_t i = lane; i < n; i += 64) dst[i] = src[i];
   if (lane == 0) reinterpret_cast<uint32_t*>(buf + p.hdr_unit + 1)[k] = nexc[s];
}

// One wave per turn slot: records back into the slot, key samples of the FIFO
// part (the producer writes them in lv_put), exception count; a received
// exception turns on the exception-aware loads of later levels (errflag[2]).
__global__ __launch_bounds__(256) void k_x_unpack(uint32_t W, const XPair* __restrict__ pairs, uint32_t np,
                                                  uint32_t total_slots, const uint64_t* __restrict__ xoff,
                                                  const uint32_t* __restrict__ slot_cnt,
                                                  const uint64_t* __restrict__ slot_base, uint32_t* __restrict__ nexc,
                                                  Rec* __restrict__ recs, uint64_t* __restrict__ samp_t,
                                                  uint32_t* __restrict__ samp_id, const uint4* __restrict__ buf,
                                                  unsigned* __restrict__ errflag)
{
   const uint32_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64, lane = threadIdx.x & 63;
   if (w >= total_slots) return;
   const uint32_t q = xs_pair_of(pairs, np, w);
   const XPair p = pairs[q];
   const uint32_t k = w - p.slot0;
   const uint32_t s = xs_slot(p, k, W);
   const uint32_t n = slot_cnt[s];
   const uint32_t ne = reinterpret_cast<const uint32_t*>(buf + p.hdr_unit + 1)[k];
   const uint64_t base = slot_base[s];
   const uint4* src = buf + xoff[w];
   uint4* dst = reinterpret_cast<uint4*>(recs + base);
   const uint32_t nmain = ne <= n ? n - ne : 0;
   for (uint32_t i = lane; i < n; i += 64)
   {
      const uint4 v = src[i];
      dst[i] = v;
      if (i < nmain && ((base + i) & 63) == 0)
      {
         samp_t[(base + i) >> 6] = (uint64_t) v.x | ((uint64_t) v.y << 32);
         samp_id[(base + i) >> 6] = v.z;
      }
   }
   if (lane == 0)
   {
      nexc[s] = ne;
      if (ne) atomicOr(errflag + 2, 1u);
      if (ne > n) atomicOr(errflag, 1u);
   }
}

// The step's status on the stream path (engine.hip gnoc_run_sharded), as four
// words every rank max-reduces: [0] a host-side failure on this rank, [1] the step
// must rerun on the synchronous protocol (this rank's X phase or a peer's did not
// complete, or a chunked level hit a burst it could not split), [2] a route-count
// invariant broke (internal error), [3] this rank's Y chains declined (it reruns
// its Y levels locally; every rank then agrees on the outcome).
__global__ void k_shard_status(const unsigned* __restrict__ errflag, int host_err, int* __restrict__ st)
{
   if (threadIdx.x != 0) return;
   const unsigned e0 = errflag[0], e4 = errflag[4], e5 = errflag[5];
   st[0] = host_err ? 1 : 0;
   st[1] = ((e4 & 0xFu) || (e0 & 6u)) ? 1 : 0;       // ch::F_ANY on the X word; level errors
   st[2] = ((e0 & 1u) || ((e4 | e5) & 4u)) ? 1 : 0;   // ch::F_ROUTE
   st[3] = (e5 & 0xFu) ? 1 : 0;
}

}  // namespace gnoc
