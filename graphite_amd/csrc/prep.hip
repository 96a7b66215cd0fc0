// prep.hip -- per-run preprocessing of the packet batch (gfx950).
//
// 1. k_classify:   per packet F = computeNumFlits (network_model.cc:202-212),
//                  the corner cases of processCornerCases / isModelEnabled
//                  (network_model.cc:171-183, 413-468: self-sends and unmodeled
//                  packets bypass the mesh), aux = (dx, dy, F), and a per-chunk
//                  histogram of source tiles in LDS (no global atomics).
// 2. k_src_tot / k_inj_base / k_src_offs: injection-slot layout.  The trace is
//                  (t, id)-ordered; grouping it stably by source tile gives every
//                  injection queue (emesh_hop_by_hop.cc:109-112, 151-159) its
//                  arrivals in service order.
// 3. k_scatter4:   the stable group-by-source into the injection slots, ranks from
//                  ballot match masks.
// 4. k_row_hist:   per (source row, group of sources) LDS histograms of the
//                  grouped records: per source (dx, y-class) and per destination.
// 5. k_prow / k_slot_counts: every output-port input slot's record count, in
//                  closed form from those histograms (XY routing is static:
//                  emesh_hop_by_hop.cc:229-240).  Deterministic, atomic-free.
// 6. k_scan_slots: slot bases (64-record aligned, so a slot's 1-in-64 key
//                  samples index as base/64).
// 7. k_plan_*:     per-port descriptors and the chunk -> port map of every level,
//                  on device, so a run needs no host round trip.
#include "common.h"

namespace gnoc {

// ---------------------------------------------------------------------------
// 1. classify
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_classify(DevCfg c, uint64_t n, uint32_t pch, const uint64_t* __restrict__ inj,
                                                  const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                                                  const uint32_t* __restrict__ bits, const uint32_t* __restrict__ flags,
                                                  uint32_t* __restrict__ aux, uint8_t* __restrict__ routed,
                                                  uint64_t* __restrict__ final_ps, uint32_t* __restrict__ hist,
                                                  unsigned long long* __restrict__ counters, uint32_t ry0, uint32_t ry1,
                                                  uint32_t cx0, uint32_t cx1, uint32_t* __restrict__ pcol,
                                                  uint32_t* __restrict__ slot_cnt)
{
   extern __shared__ uint32_t h[];   // N source counters
   const uint32_t N = c.N;
   for (uint32_t s = threadIdx.x; s < N; s += blockDim.x) h[s] = 0;
   __syncthreads();
   const uint64_t lo = (uint64_t) blockIdx.x * pch;
   const uint64_t hi = min(lo + pch, n);
   uint64_t hops = 0, nrouted = 0;
   for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
   {
      const uint32_t s = src[i], d = dst[i];
      const uint32_t fl = flags ? flags[i] : 0u;
      const uint32_t b = bits[i];
      const uint32_t fw = fw_of(c, s);
      const uint32_t F = (b % fw) ? b / fw + 1 : b / fw;
      // a broadcast (flag 2; receiver BROADCAST) is never a self-send (network_model.cc:419)
      const bool bc = (fl & 2u) != 0;
      const bool bypass = (!bc && s == d) || (fl & 1u);
      uint32_t sx, sy, dx, dy;
      tile_xy(s, c.W, c.magicW, sx, sy);
      if (bc) { dx = sx; dy = sy; }
      else tile_xy(d, c.W, c.magicW, dx, dy);
      aux[i] = aux_pack(dx, dy, F) | (bc ? AUX_BC : 0u);
      // bit 0: routed through the mesh; bit 1: and injected in this rank's row band
      const bool mine = sy >= ry0 && sy < ry1;
      routed[i] = bypass ? 0 : mine ? 3 : 1;
      if (bypass)
      {
         final_ps[i] = inj[i];
         continue;
      }
      if (mine) atomicAdd(&h[s], 1u);
      if (pcol && dx >= cx0 && dx < cx1)
      {
         // sharded run, destination in this rank's column band: the Y-leg counts
         // per (column, source row, destination row, side the packet turns from);
         // k_slot_counts_y derives the Y slots and the turn slots from them
         const uint32_t in = sx < dx ? IN_W : sx > dx ? IN_E : IN_LOCAL;
         atomicAdd(&pcol[(((dx - cx0) * c.H + sy) * c.H + dy) * 3 + in], 1u);
      }
      nrouted++;
      // a broadcast visits every router once (N switch-allocator requests)
      hops += bc ? (uint64_t) N : (uint64_t) ((sx > dx ? sx - dx : dx - sx) + (sy > dy ? sy - dy : dy - sy) + 1);
      // and materialises 2N records: injection + N SELF + (N - 1) tree edges
      if (bc) atomicAdd(&counters[2], (unsigned long long) (N - 1));
   }
   __syncthreads();
   uint32_t* hrow = hist + (uint64_t) blockIdx.x * N;
   for (uint32_t s = threadIdx.x; s < N; s += blockDim.x) hrow[s] = h[s];
   __shared__ unsigned long long red[2][4];
   for (int off = 32; off > 0; off >>= 1)
   {
      hops += __shfl_down(hops, off);
      nrouted += __shfl_down(nrouted, off);
   }
   const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
   if (l == 0) { red[0][w] = hops; red[1][w] = nrouted; }
   __syncthreads();
   if (threadIdx.x == 0)
   {
      unsigned long long a = 0, r = 0;
      for (int k = 0; k < (int) (blockDim.x >> 6); k++) { a += red[0][k]; r += red[1][k]; }
      atomicAdd(&counters[0], a);
      atomicAdd(&counters[1], r);
   }
}

// ---------------------------------------------------------------------------
// 0. submit-time checks and statistics (gnoc_submit / gnoc_submit_device)
// ---------------------------------------------------------------------------
// The trace contract of include/gnoc.h on the device: per check the first
// offending packet (atomicMin; the host reports the lowest index, ties in check
// order), the hop records this engine materialises, broadcasts, and for the
// chain engine's window sizing the records per X / Y port over the batch
// (difference arrays along each row / column) and the inserts per port.  A
// sharded engine also counts its turn exchange per (row band, column band).
enum : uint32_t
{
   VB_TILE = 0,      // src or dst out of range
   VB_BC_TREE,       // broadcast, but the model has no broadcast tree
   VB_BC_SHARD,      // broadcast on a sharded or sweep engine
   VB_ORDER,         // inject_ps decreasing
   VB_SWEEP,         // sweep packet crosses sweep points
   VB_ZERO_F,        // routed packet of zero flits
   VB_F_MAX,         // more than AUX_F_MAX flits
   VB_T_MAX,         // inject time >= 2^50 ps
   VB_PACKED,        // delta wire format: the escapes do not match the absolute times given
   VB_KINDS
};
struct ValOut
{
   unsigned long long bad[VB_KINDS];
   unsigned long long records, nbc, pmax, imax, tlast;
};

__device__ __forceinline__ uint32_t band_of(uint32_t y, uint32_t nr, uint32_t D)
{
   return (uint32_t) (((uint64_t) (y + 1) * nr - 1) / D);   // inverse of band_lo(b) = b D / nr
}

// The statistics table (ints, in this order): dxr, dxl [H (W + 1)] (X difference
// arrays), dyu, dyd [W (H + 1)] (Y), insx, insy [2 N] (inserts per X / Y port).
// LH: the block counts into a private copy in LDS (dynamic shared memory: the
// table, then nr^2 turn counts) and stores it to part[block] for k_validate_sum
// -- the per-packet atomics then never meet in L2 (10 M packets on 32x32: 3.5 ms
// of L2 atomics -> LDS).  Otherwise the atomics go to the global table.
template <bool LH>
__global__ __launch_bounds__(256) void k_validate(DevCfg c, uint64_t n, const uint64_t* __restrict__ inj,
                                                  const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                                                  const uint32_t* __restrict__ bits, const uint32_t* __restrict__ flags,
                                                  int tree, uint32_t sweep, uint32_t nr, uint32_t rank, uint32_t xself,
                                                  ValOut* __restrict__ vo,
                                                  int* __restrict__ gtab, uint32_t ntab, int* __restrict__ part,
                                                  unsigned long long* __restrict__ xcnt)
{
   extern __shared__ int lds_tab[];
   const uint32_t N = c.N, W = c.W, H = c.H;
   const bool band_prep = W <= 64 && H <= 64;
   const uint32_t nx2 = nr * nr;
   int* const tab = LH ? lds_tab : gtab;
   uint32_t* const lx = reinterpret_cast<uint32_t*>(lds_tab + ntab);
   if (LH)
   {
      for (uint32_t k = threadIdx.x; k < ntab + nx2; k += blockDim.x) lds_tab[k] = 0;
      __syncthreads();
   }
   int* const dxr = tab;
   int* const dxl = dxr + (size_t) H * (W + 1);
   int* const dyu = dxl + (size_t) H * (W + 1);
   int* const dyd = dyu + (size_t) W * (H + 1);
   int* const insx = dyd + (size_t) W * (H + 1);
   int* const insy = insx + 2 * (size_t) N;
   unsigned long long rec = 0, nbc = 0;
   for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x)
   {
      const uint32_t s = src[i], fl = flags ? flags[i] : 0u;
      const bool bc = (fl & 2u) != 0;
      const uint32_t d = bc ? s : dst[i];   // a broadcast's receiver field is ignored
      const uint64_t t = inj[i];
      if (i == n - 1) vo->tlast = t;
      uint32_t kind = VB_KINDS;
      uint32_t F = 0;
      bool bypass = true;
      if (s >= N || d >= N) kind = VB_TILE;
      else if (bc && !tree) kind = VB_BC_TREE;
      else if (bc && (nr > 1 || sweep)) kind = VB_BC_SHARD;
      else if (i && t < inj[i - 1]) kind = VB_ORDER;
      else if (sweep && point_of(c, s) != point_of(c, d)) kind = VB_SWEEP;
      else
      {
         const uint32_t fw = fw_of(c, s), b = bits[i];
         F = (b % fw) ? b / fw + 1 : b / fw;
         bypass = (!bc && s == d) || (fl & 1u);
         if (F == 0 && !bypass) kind = VB_ZERO_F;
         else if (F > AUX_F_MAX) kind = VB_F_MAX;
         else if (t >= (1ull << 50)) kind = VB_T_MAX;
      }
      if (kind != VB_KINDS)
      {
         atomicMin(&vo->bad[kind], (unsigned long long) i);
         continue;
      }
      nbc += bc ? 1u : 0u;
      if (bypass) continue;
      if (bc)
      {
         rec += 2ull * N;   // injection + N SELF + N - 1 tree edges
         continue;
      }
      uint32_t sx, sy, dx, dy;
      tile_xy(s, W, c.magicW, sx, sy);
      tile_xy(d, W, c.magicW, dx, dy);
      const uint32_t ax = sx > dx ? sx - dx : dx - sx, ay = sy > dy ? sy - dy : dy - sy;
      if (dx > sx)
      {
         atomicAdd(&dxr[sy * (W + 1) + sx], 1);
         atomicAdd(&dxr[sy * (W + 1) + dx], -1);
         atomicAdd(&insx[s * 2], 1);
      }
      else if (dx < sx)
      {
         atomicAdd(&dxl[sy * (W + 1) + dx + 1], 1);
         atomicAdd(&dxl[sy * (W + 1) + sx + 1], -1);
         atomicAdd(&insx[s * 2 + 1], 1);
      }
      if (dy > sy)
      {
         atomicAdd(&dyu[dx * (H + 1) + sy], 1);
         atomicAdd(&dyu[dx * (H + 1) + dy], -1);
         atomicAdd(&insy[(sy * W + dx) * 2], 1);
      }
      else if (dy < sy)
      {
         atomicAdd(&dyd[dx * (H + 1) + dy + 1], 1);
         atomicAdd(&dyd[dx * (H + 1) + sy + 1], -1);
         atomicAdd(&insy[(sy * W + dx) * 2 + 1], 1);
      }
      if (nr <= 1)
      {
         rec += 2 + ax + ay;
         if (xself && c.contention)   // the self-exchange test knob: one turn record per routed packet
         {
            if (LH) atomicAdd(&lx[0], 1u);
            else atomicAdd(&xcnt[0], 1ull);
         }
      }
      else
      {
         // records this rank materialises: injection + X leg in its row band (all
         // injections when prep is not band-local), the turn record on either side,
         // the Y leg in its column band
         const uint32_t rb = band_of(sy, nr, H), cb = band_of(dx, nr, W);
         const bool r_own = rb == rank, c_own = cb == rank;
         rec += (r_own ? 1 + ax : 0) + (!r_own && !band_prep ? 1 : 0) + (r_own || c_own ? 1 : 0) + (c_own ? ay : 0);
         if (c.contention)
         {
            if (LH) atomicAdd(&lx[rb * nr + cb], 1u);
            else atomicAdd(&xcnt[rb * nr + cb], 1ull);
         }
      }
   }
   // wave sums, one atomic per wave
   for (int off = 32; off > 0; off >>= 1)
   {
      rec += __shfl_down(rec, off);
      nbc += __shfl_down(nbc, off);
   }
   if ((threadIdx.x & 63) == 0)
   {
      if (rec) atomicAdd(&vo->records, rec);
      if (nbc) atomicAdd(&vo->nbc, nbc);
   }
   if (LH)
   {
      __syncthreads();
      int* const out = part + (size_t) blockIdx.x * ntab;
      for (uint32_t k = threadIdx.x; k < ntab; k += blockDim.x) out[k] = lds_tab[k];
      for (uint32_t k = threadIdx.x; k < nx2; k += blockDim.x)
         if (lx[k]) atomicAdd(&xcnt[k], (unsigned long long) lx[k]);
   }
}

// The blocks' private tables summed into the global one (a column per thread).
__global__ __launch_bounds__(256) void k_validate_sum(uint32_t ntab, uint32_t nblk, const int* __restrict__ part,
                                                      int* __restrict__ gtab)
{
   const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
   if (k >= ntab) return;
   int acc = 0;
#pragma unroll 8
   for (uint32_t b = 0; b < nblk; b++) acc += part[(size_t) b * ntab + k];
   gtab[k] = acc;
}

// The busiest X / Y port over the batch (prefix sums of the difference arrays)
// and the most inserts of any port.  One workgroup.
__global__ __launch_bounds__(1024) void k_validate_max(uint32_t W, uint32_t H, const int* __restrict__ dxr,
                                                       const int* __restrict__ dxl, const int* __restrict__ dyu,
                                                       const int* __restrict__ dyd, const uint32_t* __restrict__ insx,
                                                       const uint32_t* __restrict__ insy, ValOut* __restrict__ vo)
{
   unsigned long long pm = 0, im = 0;
   for (uint32_t r = threadIdx.x; r < H; r += blockDim.x)
   {
      long long a = 0, b = 0;
      for (uint32_t x = 0; x <= W; x++)
      {
         a += dxr[r * (W + 1) + x];
         b += dxl[r * (W + 1) + x];
         pm = max(pm, (unsigned long long) max(a, b));
      }
   }
   for (uint32_t x = threadIdx.x; x < W; x += blockDim.x)
   {
      long long a = 0, b = 0;
      for (uint32_t y = 0; y <= H; y++)
      {
         a += dyu[x * (H + 1) + y];
         b += dyd[x * (H + 1) + y];
         pm = max(pm, (unsigned long long) max(a, b));
      }
   }
   for (uint32_t k = threadIdx.x; k < 2 * W * H; k += blockDim.x) im = max(im, (unsigned long long) max(insx[k], insy[k]));
   atomicMax(&vo->pmax, pm);
   atomicMax(&vo->imax, im);
}

// ---------------------------------------------------------------------------
// 2. injection-slot layout
// ---------------------------------------------------------------------------
// Sources outside [s0, s1) (another rank's row band) have no injection records here.
// The chunk axis is cut into SRC_SEGS segments (grid y) so a source's sums and
// prefix run in parallel: seg[g][s] = chunks of segment g, then tot[s] = sum over g.
constexpr uint32_t SRC_SEGS = 64;
__device__ __forceinline__ uint32_t seg_ch(uint32_t g, uint32_t nch, uint32_t ns) { return (uint32_t) ((uint64_t) g * nch / ns); }

__global__ __launch_bounds__(256) void k_src_seg(uint32_t N, uint32_t nch, uint32_t ns, const uint32_t* __restrict__ hist,
                                                 uint32_t* __restrict__ seg, uint32_t s0, uint32_t s1)
{
   const uint32_t s = s0 + blockIdx.x * blockDim.x + threadIdx.x, g = blockIdx.y;
   if (s >= s1) return;
   uint32_t t = 0;
   const uint32_t c1 = seg_ch(g + 1, nch, ns);
#pragma unroll 16
   for (uint32_t ch = seg_ch(g, nch, ns); ch < c1; ch++) t += hist[(uint64_t) ch * N + s];
   seg[(uint64_t) g * N + s] = t;
}

__global__ __launch_bounds__(256) void k_src_tot(uint32_t N, uint32_t ns, const uint32_t* __restrict__ seg,
                                                 uint32_t* __restrict__ tot, uint32_t s0, uint32_t s1)
{
   const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
   if (s >= N) return;
   if (s < s0 || s >= s1) { tot[s] = 0; return; }
   uint32_t t = 0;
#pragma unroll 16
   for (uint32_t g = 0; g < ns; g++) t += seg[(uint64_t) g * N + s];
   tot[s] = t;
}

// Single block: injection slot bases (64-aligned) in front of every other slot.
__global__ __launch_bounds__(1024) void k_inj_base(uint32_t N, const uint32_t* __restrict__ tot,
                                                   uint32_t* __restrict__ slot_cnt, uint64_t* __restrict__ slot_base,
                                                   uint64_t* __restrict__ inj_total)
{
   __shared__ uint64_t part[1024];
   const uint32_t per = (N + 1023) / 1024;
   const uint32_t lo = threadIdx.x * per, hi = min(lo + per, N);
   uint64_t s = 0;
   for (uint32_t i = lo; i < hi; i++) s += (tot[i] + 63) & ~63u;
   part[threadIdx.x] = s;
   __syncthreads();
   for (uint32_t off = 1; off < 1024; off <<= 1)
   {
      const uint64_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
   }
   uint64_t run = part[threadIdx.x] - s;
   for (uint32_t i = lo; i < hi; i++)
   {
      const uint32_t sl = slot_of(i, P_INJ, IN_LOCAL);
      slot_base[sl] = run;
      slot_cnt[sl] = tot[i];
      run += (tot[i] + 63) & ~63u;
   }
   if (threadIdx.x == 1023) *inj_total = part[1023];
}

// hist[ch][s] (counts) -> absolute record offsets of chunk ch's first record of source s.
// Grid y = chunk segment g: the running offset starts after segments 0 .. g-1.
__global__ __launch_bounds__(256) void k_src_offs(uint32_t N, uint32_t nch, uint32_t ns, uint32_t* __restrict__ hist,
                                                  const uint32_t* __restrict__ seg,
                                                  const uint64_t* __restrict__ slot_base, uint32_t s0, uint32_t s1)
{
   const uint32_t s = s0 + blockIdx.x * blockDim.x + threadIdx.x, g = blockIdx.y;
   if (s >= s1) return;
   uint32_t run = (uint32_t) slot_base[slot_of(s, P_INJ, IN_LOCAL)];   // < 2^32 records (checked at submit)
   for (uint32_t q = 0; q < g; q++) run += seg[(uint64_t) q * N + s];
   const uint32_t c1 = seg_ch(g + 1, nch, ns);
#pragma unroll 16
   for (uint32_t ch = seg_ch(g, nch, ns); ch < c1; ch++)
   {
      const uint64_t k = (uint64_t) ch * N + s;
      const uint32_t v = hist[k];
      hist[k] = run;
      run += v;
   }
}

// ---------------------------------------------------------------------------
// 3. stable scatter into the injection slots (one wave per chunk)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t match_mask(uint32_t key, bool valid, int nbits)
{
   uint64_t m = __ballot(valid);
   for (int b = 0; b < nbits; b++)
   {
      const bool bit = (key >> b) & 1u;
      const uint64_t bb = __ballot(bit && valid);
      m &= bit ? bb : ~bb;
   }
   return m;
}

// The stable scatter with NW waves per chunk: each wave owns a contiguous 1/NW of
// the chunk; per-wave source counts in LDS (NW * N words) give each wave its
// starting rank, then every wave ranks its part in order, with the next 64
// packets' loads in flight while the current ones are placed.  NW = 8 for
// N <= 2048, 4 for N <= 4096 (64 KiB of counters).  Larger meshes (sweeps) use
// k_scatter: a 2-wave variant needs 65536-packet chunks there and was slower.
constexpr uint32_t SC4_MAXN = 4096;
__host__ __device__ inline int scatter_waves(uint32_t N) { return N <= 2048 ? 8 : 4; }

//
// SPARSE (a sharded rank: only its row band's sources, ~1/nranks of the trace):
// each wave compacts the valid packets of 512 at a time into an LDS buffer, in
// order, and ranks them 64 at a time, so the ballots run per placed packet
// rather than per trace packet.  The buffer follows the NW * N counters.
template <int NW, bool SPARSE>
__global__ __launch_bounds__(512) void k_scatter4(uint64_t n, uint32_t pch, uint32_t N, uint32_t s0, uint32_t S, int nbits,
                                                  const uint32_t* __restrict__ src, const uint8_t* __restrict__ routed,
                                                  const uint64_t* __restrict__ inj, const uint32_t* __restrict__ aux,
                                                  const uint32_t* __restrict__ offs, Rec* __restrict__ recs,
                                                  uint64_t* __restrict__ samp_t, uint32_t* __restrict__ samp_id,
                                                  const uint32_t* __restrict__ gid)
{
   // gid: a sharded rank's partitioned trace -- records carry global packet ids
   extern __shared__ uint32_t h4[];   // [NW][S] per-wave counts of sources s0 .. s0+S-1 -> running ranks
   const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
   for (uint32_t k = threadIdx.x; k < NW * S; k += 64 * NW) h4[k] = 0;
   __syncthreads();
   const uint64_t c0 = (uint64_t) blockIdx.x * pch;
   const uint64_t c1 = min(c0 + pch, n);
   const uint64_t q = (c1 - c0 + NW - 1) / NW;
   const uint64_t lo = min(c0 + w * q, c1), hi = min(lo + q, c1);
   uint32_t* hw = h4 + w * S;
#pragma unroll 8
   for (uint64_t i = lo + lane; i < hi; i += 64)
      if (routed[i] & 2) atomicAdd(&hw[src[i] - s0], 1u);
   __syncthreads();
   // exclusive prefix over waves, plus the chunk's offset for the source
   const uint32_t* orow = offs + (uint64_t) blockIdx.x * N + s0;
   for (uint32_t s2 = threadIdx.x; s2 < S; s2 += 64 * NW)
   {
      uint32_t run = orow[s2];
      for (uint32_t ww = 0; ww < (uint32_t) NW; ww++)
      {
         const uint32_t v = h4[ww * S + s2];
         h4[ww * S + s2] = run;
         run += v;
      }
   }
   __syncthreads();
   const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
   if (SPARSE)
   {
      uint32_t* buf = h4 + NW * S + w * 512;
      for (uint64_t k0 = lo; k0 < hi; k0 += 512)
      {
         bool v[8];
#pragma unroll
         for (int q = 0; q < 8; q++)
         {
            const uint64_t i = k0 + (uint64_t) (q * 64) + lane;
            v[q] = i < hi && (routed[i] & 2) != 0;
         }
         uint32_t tot = 0;
#pragma unroll
         for (int q = 0; q < 8; q++)
         {
            const uint64_t b = __ballot(v[q]);
            if (v[q]) buf[tot + (uint32_t) __popcll(b & lt)] = (uint32_t) (q * 64) + lane;
            tot += (uint32_t) __popcll(b);
         }
         asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
         __builtin_amdgcn_wave_barrier();
         for (uint32_t q = 0; q < tot; q += 64)
         {
            const bool valid = q + lane < tot;
            uint64_t i = 0;
            uint32_t sidx = 0;
            if (valid)
            {
               i = k0 + buf[q + lane];
               sidx = src[i] - s0;
            }
            const uint64_t m = match_mask(sidx, valid, nbits);
            const uint32_t old = valid ? hw[sidx] : 0u;
            __builtin_amdgcn_wave_barrier();
            if (valid)
            {
               const uint32_t rank = old + (uint32_t) __popcll(m & lt);
               if ((63 - __clzll(m)) == (int) lane) hw[sidx] = old + (uint32_t) __popcll(m);
               const uint64_t pos = rank;
               Rec r;
               r.t = inj[i];
               r.id = gid ? gid[i] : (uint32_t) i;
               r.aux = aux[i];
               recs[pos] = r;
               if ((pos & 63) == 0)
               {
                  samp_t[pos >> 6] = r.t;
                  samp_id[pos >> 6] = r.id;
               }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
         }
      }
      return;
   }
   // software pipeline SC_D groups of 64 packets deep: group g + SC_D's loads are
   // issued (all four fields, none waiting on another) before group g is placed,
   // so a wave keeps several KB of loads in flight instead of waiting on each group
   constexpr int SC_D = 4;
   uint32_t pr[SC_D], ps[SC_D], pa[SC_D];
   uint64_t pt[SC_D];
#pragma unroll
   for (int d = 0; d < SC_D; d++)
   {
      const uint64_t i = lo + (uint64_t) d * 64 + lane;
      pr[d] = 0; ps[d] = 0; pa[d] = 0; pt[d] = 0;
      if (i < hi) { pr[d] = routed[i]; ps[d] = src[i]; pt[d] = inj[i]; pa[d] = aux[i]; }
   }
   for (uint64_t k0 = lo; k0 < hi; k0 += 64 * SC_D)
#pragma unroll
   for (int d = 0; d < SC_D; d++)
   {
      const uint64_t k = k0 + (uint64_t) d * 64;
      if (k >= hi) break;
      const bool valid = (pr[d] & 2) != 0;   // a sharded rank places only its row band's packets
      const uint32_t sidx = valid ? ps[d] - s0 : 0u;
      const uint64_t t = pt[d];
      const uint32_t a = pa[d];
      const uint64_t id = k + lane;
      const uint64_t i2 = k + 64 * SC_D + lane;
      pr[d] = 0; ps[d] = 0; pa[d] = 0; pt[d] = 0;
      if (i2 < hi) { pr[d] = routed[i2]; ps[d] = src[i2]; pt[d] = inj[i2]; pa[d] = aux[i2]; }
      const uint64_t m = match_mask(sidx, valid, nbits);
      const uint32_t old = valid ? hw[sidx] : 0u;
      __builtin_amdgcn_wave_barrier();
      if (valid)
      {
         const uint32_t rank = old + (uint32_t) __popcll(m & lt);
         if ((63 - __clzll(m)) == (int) lane) hw[sidx] = old + (uint32_t) __popcll(m);
         const uint64_t pos = rank;
         Rec r;
         r.t = t;
         r.id = gid ? gid[id] : (uint32_t) id;
         r.aux = a;
         recs[pos] = r;
         if ((pos & 63) == 0)
         {
            samp_t[pos >> 6] = r.t;
            samp_id[pos >> 6] = r.id;
         }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
   }
}

// ---------------------------------------------------------------------------
// 4. per-row histograms of the grouped injection records
//    Hs[s][dx][c]   c = 0 (dy < sy), 1 (dy == sy), 2 (dy > sy)      N x W x 3
//    Pp[y][g][dst]  destinations of row y, source group g            H x G x N
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_row_hist(DevCfg c, uint32_t G, const Rec* __restrict__ recs,
                                                  const uint32_t* __restrict__ slot_cnt,
                                                  const uint64_t* __restrict__ slot_base, uint32_t* __restrict__ Hs,
                                                  uint32_t* __restrict__ Pp, int pp_lds, uint32_t ry0)
{
   extern __shared__ uint32_t sm[];
   const uint32_t W = c.W, N = c.N;
   const uint32_t y = ry0 + blockIdx.y, g = blockIdx.x;
   const uint32_t x0 = (uint32_t) (((uint64_t) g * W) / G), x1 = (uint32_t) (((uint64_t) (g + 1) * W) / G);
   const uint32_t nhs = (x1 - x0) * W * 3;
   uint32_t* hs = sm;
   uint32_t* ph = sm + nhs;
   uint32_t* pg = Pp + ((uint64_t) y * G + g) * N;
   for (uint32_t k = threadIdx.x; k < nhs; k += blockDim.x) hs[k] = 0;
   if (pp_lds)
      for (uint32_t k = threadIdx.x; k < N; k += blockDim.x) ph[k] = 0;
   __syncthreads();
   for (uint32_t x = x0; x < x1; x++)
   {
      const uint32_t s = y * W + x;
      const uint32_t sl = slot_of(s, P_INJ, IN_LOCAL);
      const uint32_t cnt = slot_cnt[sl];
      const Rec* r = recs + slot_base[sl];
      uint32_t* hrow = hs + (x - x0) * W * 3;
      for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x)
      {
         const uint32_t a = r[i].aux;
         const uint32_t dx = aux_dx(a), dy = aux_dy(a);
         const uint32_t cl = dy < y ? 0u : dy == y ? 1u : 2u;
         atomicAdd(&hrow[dx * 3 + cl], 1u);
         if (pp_lds) atomicAdd(&ph[dy * W + dx], 1u);
         else atomicAdd(&pg[dy * W + dx], 1u);
      }
   }
   __syncthreads();
   for (uint32_t k = threadIdx.x; k < nhs; k += blockDim.x) Hs[(uint64_t) (y * W + x0) * W * 3 + k] = hs[k];
   if (pp_lds)
      for (uint32_t k = threadIdx.x; k < N; k += blockDim.x) pg[k] = ph[k];
}

// Prow[y][dst] = sum over groups.
__global__ __launch_bounds__(256) void k_prow(uint32_t N, uint32_t H, uint32_t G, const uint32_t* __restrict__ Pp,
                                              uint32_t* __restrict__ Prow)
{
   const uint64_t k = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
   if (k >= (uint64_t) H * N) return;
   const uint64_t y = k / N, d = k % N;
   uint32_t s = 0;
   for (uint32_t g = 0; g < G; g++) s += Pp[(y * G + g) * N + d];
   Prow[k] = s;
}

// One thread per (tile, dir) computes the 5 input-side counts of that output port.
// Packets follow XY routing: X leg in the source row, Y leg in the destination column.
__global__ __launch_bounds__(256) void k_slot_counts(DevCfg c, const uint32_t* __restrict__ Hs,
                                                     const uint32_t* __restrict__ Prow, uint32_t* __restrict__ slot_cnt)
{
   const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
   const uint32_t W = c.W, N = c.N;
   if (k >= N * 5) return;
   const uint32_t tile = k / 5, dir = k % 5;
   const uint32_t x = tile % W, y = tile / W;
   // a sweep mesh's packets stay inside their BW x BH block
   const uint32_t bx0 = x / c.BW * c.BW, bx1 = bx0 + c.BW, by0 = y / c.BH * c.BH, by1 = by0 + c.BH;
   auto hs = [&](uint32_t sx, uint32_t sy, uint32_t dx, uint32_t cl) -> uint32_t {
      return Hs[((uint64_t) (sy * W + sx) * W + dx) * 3 + cl];
   };
   auto prow = [&](uint32_t sy, uint32_t dx, uint32_t dy) -> uint32_t { return Prow[(uint64_t) sy * N + dy * W + dx]; };
   uint32_t cl = 0, cw = 0, ce = 0, cs = 0, cn = 0;
   // IN_LOCAL: packets injected here whose first hop leaves through `dir`
   if (dir == P_RIGHT) { for (uint32_t dx = x + 1; dx < bx1; dx++) cl += hs(x, y, dx, 0) + hs(x, y, dx, 1) + hs(x, y, dx, 2); }
   else if (dir == P_LEFT) { for (uint32_t dx = bx0; dx < x; dx++) cl += hs(x, y, dx, 0) + hs(x, y, dx, 1) + hs(x, y, dx, 2); }
   else if (dir == P_UP) cl = hs(x, y, x, 2);
   else if (dir == P_DOWN) cl = hs(x, y, x, 0);
   // IN_W: X leg moving right through x (sx < x <= dx) in row y
   if (dir == P_RIGHT)
   {
      for (uint32_t sx = bx0; sx < x; sx++)
         for (uint32_t dx = x + 1; dx < bx1; dx++) cw += hs(sx, y, dx, 0) + hs(sx, y, dx, 1) + hs(sx, y, dx, 2);
   }
   else if (dir != P_LEFT)
   {
      const uint32_t want = dir == P_UP ? 2u : dir == P_DOWN ? 0u : 1u;
      for (uint32_t sx = bx0; sx < x; sx++) cw += hs(sx, y, x, want);
   }
   // IN_E: X leg moving left (dx <= x < sx)
   if (dir == P_LEFT)
   {
      for (uint32_t sx = x + 1; sx < bx1; sx++)
         for (uint32_t dx = bx0; dx < x; dx++) ce += hs(sx, y, dx, 0) + hs(sx, y, dx, 1) + hs(sx, y, dx, 2);
   }
   else if (dir != P_RIGHT)
   {
      const uint32_t want = dir == P_UP ? 2u : dir == P_DOWN ? 0u : 1u;
      for (uint32_t sx = x + 1; sx < bx1; sx++) ce += hs(sx, y, x, want);
   }
   // IN_S: Y leg moving up in column x (sy < y <= dy)
   if (dir == P_UP)
   {
      for (uint32_t sy = by0; sy < y; sy++)
         for (uint32_t dy = y + 1; dy < by1; dy++) cs += prow(sy, x, dy);
   }
   else if (dir == P_SELF)
   {
      for (uint32_t sy = by0; sy < y; sy++) cs += prow(sy, x, y);
   }
   // IN_N: Y leg moving down (dy <= y < sy)
   if (dir == P_DOWN)
   {
      for (uint32_t sy = y + 1; sy < by1; sy++)
         for (uint32_t dy = by0; dy < y; dy++) cn += prow(sy, x, dy);
   }
   else if (dir == P_SELF)
   {
      for (uint32_t sy = y + 1; sy < by1; sy++) cn += prow(sy, x, y);
   }
   slot_cnt[slot_of(tile, dir, IN_LOCAL)] = cl;
   slot_cnt[slot_of(tile, dir, IN_W)] = cw;
   slot_cnt[slot_of(tile, dir, IN_E)] = ce;
   slot_cnt[slot_of(tile, dir, IN_S)] = cs;
   slot_cnt[slot_of(tile, dir, IN_N)] = cn;
}

// The same counts, split by leg with the histograms cached in LDS: one block
// per row for the X-leg inputs (LOCAL, W, E), one per column for the Y-leg
// inputs (S, N).  Used when W*W*3 and H*H words fit (W, H <= 64).
__global__ __launch_bounds__(256) void k_slot_counts_x(DevCfg c, const uint32_t* __restrict__ Hs,
                                                       uint32_t* __restrict__ slot_cnt, uint32_t ry0)
{
   extern __shared__ uint32_t hr[];   // Hs rows of this mesh row: [sx][dx][cl], then pt[W][W]
   const uint32_t W = c.W, y = ry0 + blockIdx.x;
   const uint32_t nw = W * W * 3;
   uint32_t* pt = hr + nw;
   for (uint32_t k = threadIdx.x; k < nw; k += blockDim.x) hr[k] = Hs[(uint64_t) y * W * W * 3 + k];
   __syncthreads();
   auto hs = [&](uint32_t sx, uint32_t dx, uint32_t cl) -> uint32_t { return hr[(sx * W + dx) * 3 + cl]; };
   // 2-D prefix of T(sx, dx) = all classes: pt[(a-1)W + b-1] = sum over sx < a, dx < b
   if (threadIdx.x < W)
   {
      uint32_t run = 0;
      for (uint32_t dx = 0; dx < W; dx++)
      {
         run += hs(threadIdx.x, dx, 0) + hs(threadIdx.x, dx, 1) + hs(threadIdx.x, dx, 2);
         pt[threadIdx.x * W + dx] = run;
      }
   }
   __syncthreads();
   if (threadIdx.x < W)
   {
      uint32_t run = 0;
      for (uint32_t sx = 0; sx < W; sx++)
      {
         run += pt[sx * W + threadIdx.x];
         pt[sx * W + threadIdx.x] = run;
      }
   }
   __syncthreads();
   auto P = [&](uint32_t a, uint32_t b) -> uint32_t { return (a && b) ? pt[(a - 1) * W + (b - 1)] : 0u; };
   // sum of T over sx in [a0, a1), dx in [b0, b1)
   auto rect = [&](uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1) -> uint32_t {
      return (a0 >= a1 || b0 >= b1) ? 0u : P(a1, b1) - P(a0, b1) - P(a1, b0) + P(a0, b0);
   };
   for (uint32_t q = threadIdx.x; q < W * 5; q += blockDim.x)
   {
      const uint32_t x = q / 5, dir = q % 5, tile = y * W + x;
      const uint32_t bx0 = x / c.BW * c.BW, bx1 = bx0 + c.BW;
      uint32_t cl = 0, cw = 0, ce = 0;
      if (dir == P_RIGHT) cl = rect(x, x + 1, x + 1, bx1);
      else if (dir == P_LEFT) cl = rect(x, x + 1, bx0, x);
      else if (dir == P_UP) cl = hs(x, x, 2);
      else if (dir == P_DOWN) cl = hs(x, x, 0);
      if (dir == P_RIGHT) cw = rect(bx0, x, x + 1, bx1);
      else if (dir != P_LEFT)
      {
         const uint32_t want = dir == P_UP ? 2u : dir == P_DOWN ? 0u : 1u;
         for (uint32_t sx = bx0; sx < x; sx++) cw += hs(sx, x, want);
      }
      if (dir == P_LEFT) ce = rect(x + 1, bx1, bx0, x);
      else if (dir != P_RIGHT)
      {
         const uint32_t want = dir == P_UP ? 2u : dir == P_DOWN ? 0u : 1u;
         for (uint32_t sx = x + 1; sx < bx1; sx++) ce += hs(sx, x, want);
      }
      slot_cnt[slot_of(tile, dir, IN_LOCAL)] = cl;
      slot_cnt[slot_of(tile, dir, IN_W)] = cw;
      slot_cnt[slot_of(tile, dir, IN_E)] = ce;
   }
}

// Column x = cx0 + blockIdx.x.  pcol == nullptr: read column x of Prow[sy][dst];
// else pcol[x - cx0][sy][dy][side] (sharded runs, counted in k_classify), which
// also gives this column's turn slots (tile (x, sy), dir by dy, side IN_LOCAL/W/E).
__global__ __launch_bounds__(256) void k_slot_counts_y(DevCfg c, const uint32_t* __restrict__ Prow,
                                                       uint32_t* __restrict__ slot_cnt, uint32_t cx0,
                                                       const uint32_t* __restrict__ pcol)
{
   extern __shared__ uint32_t pc[];   // column x: [sy][dy], then its 2-D prefix pt[H][H]
   const uint32_t W = c.W, H = c.H, N = c.N, x = cx0 + blockIdx.x;
   for (uint32_t k = threadIdx.x; k < H * H; k += blockDim.x)
   {
      const uint32_t sy = k / H, dy = k % H;
      const uint32_t* p3 = pcol ? pcol + ((uint64_t) blockIdx.x * H * H + k) * 3 : nullptr;
      pc[k] = pcol ? p3[0] + p3[1] + p3[2] : Prow[(uint64_t) sy * N + dy * W + x];
   }
   if (pcol)
   {
      for (uint32_t q = threadIdx.x; q < H * 9; q += blockDim.x)
      {
         const uint32_t sy = q / 9, dir3 = (q % 9) / 3, in = q % 3;
         const uint32_t dir = dir3 == 0 ? P_SELF : dir3 == 1 ? P_DOWN : P_UP;
         const uint32_t d0 = dir == P_UP ? sy + 1 : dir == P_DOWN ? 0u : sy;
         const uint32_t d1 = dir == P_UP ? H : dir == P_DOWN ? sy : sy + 1;
         const uint32_t* p3 = pcol + ((uint64_t) blockIdx.x * H + sy) * H * 3 + in;
         uint32_t cnt = 0;
         for (uint32_t dy = d0; dy < d1; dy++) cnt += p3[dy * 3];
         slot_cnt[slot_of(sy * W + x, dir, in)] = cnt;
      }
   }
   __syncthreads();
   uint32_t* pt = pc + H * H;   // pt[(a-1)H + b-1] = sum over sy < a, dy < b
   if (threadIdx.x < H)
   {
      uint32_t run = 0;
      for (uint32_t dy = 0; dy < H; dy++)
      {
         run += pc[threadIdx.x * H + dy];
         pt[threadIdx.x * H + dy] = run;
      }
   }
   __syncthreads();
   if (threadIdx.x < H)
   {
      uint32_t run = 0;
      for (uint32_t sy = 0; sy < H; sy++)
      {
         run += pt[sy * H + threadIdx.x];
         pt[sy * H + threadIdx.x] = run;
      }
   }
   __syncthreads();
   auto P = [&](uint32_t a, uint32_t b) -> uint32_t { return (a && b) ? pt[(a - 1) * H + (b - 1)] : 0u; };
   auto rect = [&](uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1) -> uint32_t {
      return (a0 >= a1 || b0 >= b1) ? 0u : P(a1, b1) - P(a0, b1) - P(a1, b0) + P(a0, b0);
   };
   for (uint32_t q = threadIdx.x; q < H * 5; q += blockDim.x)
   {
      const uint32_t y = q / 5, dir = q % 5, tile = y * W + x;
      const uint32_t by0 = y / c.BH * c.BH, by1 = by0 + c.BH;
      uint32_t cs = 0, cn = 0;
      if (dir == P_UP) cs = rect(by0, y, y + 1, by1);
      else if (dir == P_SELF)
      {
         for (uint32_t sy = by0; sy < y; sy++) cs += pc[sy * H + y];
      }
      if (dir == P_DOWN) cn = rect(y + 1, by1, by0, y);
      else if (dir == P_SELF)
      {
         for (uint32_t sy = y + 1; sy < by1; sy++) cn += pc[sy * H + y];
      }
      slot_cnt[slot_of(tile, dir, IN_S)] = cs;
      slot_cnt[slot_of(tile, dir, IN_N)] = cn;
   }
}

// Broadcast-tree records per input slot, added to the unicast counts: one
// thread per (broadcast, router).  The tree visits router (cx, cy) once, from
// side bc_in_side, and requests the ports of bc_mask there.
__global__ __launch_bounds__(256) void k_bcast_slots(DevCfg c, uint32_t nb, const uint32_t* __restrict__ bid,
                                                     const uint32_t* __restrict__ src,
                                                     const uint8_t* __restrict__ routed, uint32_t* __restrict__ slot_cnt,
                                                     uint32_t* __restrict__ bcnt)
{
   const uint64_t k = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
   if (k >= (uint64_t) nb * c.N) return;
   const uint32_t b = (uint32_t) (k / c.N), tile = (uint32_t) (k % c.N);
   const uint32_t id = bid[b];
   if (!(routed[id] & 1)) return;
   uint32_t sx, sy, cx, cy;
   tile_xy(src[id], c.W, c.magicW, sx, sy);
   tile_xy(tile, c.W, c.magicW, cx, cy);
   const uint32_t m = bc_mask(sx, sy, cx, cy, c.W, c.H), in = bc_in_side(sx, sy, cx, cy);
   for (uint32_t d = 0; d < 5; d++)
      if ((m >> d) & 1u)
      {
         const uint32_t sl = slot_of(tile, d, slot_side(d, in));
         atomicAdd(&slot_cnt[sl], 1u);
         atomicAdd(&bcnt[sl], 1u);   // the slot's broadcast tail (kernels.hip, level.hip)
      }
}

// ---------------------------------------------------------------------------
// 6. bases of the non-injection slots, after the injection region (single block)
// ---------------------------------------------------------------------------
// A layout past the record buffer (bound: sized on the host from the trace checks)
// cannot come from a consistent batch; should it happen, the mesh slots are emptied
// (count and base 0) so no later kernel writes outside the buffer, and the host
// refuses the run (gtot[1] > rec_bound).
__global__ __launch_bounds__(1024) void k_scan_slots(uint32_t N, uint32_t* __restrict__ cnt,
                                                     uint64_t* __restrict__ base, const uint64_t* __restrict__ inj_total,
                                                     uint64_t* __restrict__ total, uint64_t bound)
{
   __shared__ uint64_t part[1024];
   // enumerate the 5 mesh directions x 5 inputs of every tile: q -> slot (tile*6 + dir)*5 + in, dir < 5
   const uint32_t nq = N * 25;
   const uint32_t per = (nq + 1023) / 1024;
   const uint32_t lo = threadIdx.x * per, hi = min(lo + per, nq);
   auto slot = [](uint32_t q) { return (q / 25) * (PORTS * INS) + (q % 25); };
   uint64_t s = 0;
   for (uint32_t q = lo; q < hi; q++) s += (cnt[slot(q)] + 63) & ~63u;
   part[threadIdx.x] = s;
   __syncthreads();
   for (uint32_t off = 1; off < 1024; off <<= 1)
   {
      const uint64_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
   }
   uint64_t run = *inj_total + part[threadIdx.x] - s;
   const bool over = *inj_total + part[1023] > bound;
   for (uint32_t q = lo; q < hi; q++)
   {
      const uint32_t c = cnt[slot(q)];
      base[slot(q)] = over ? 0ull : run;
      if (over) cnt[slot(q)] = 0;
      run += (c + 63) & ~63u;
   }
   if (threadIdx.x == 1023) *total = *inj_total + part[1023];
}

template __global__ void k_scatter4<4, false>(uint64_t, uint32_t, uint32_t, uint32_t, uint32_t, int, const uint32_t*, const uint8_t*,
                                       const uint64_t*, const uint32_t*, const uint32_t*, Rec*, uint64_t*, uint32_t*,
                                       const uint32_t*);
template __global__ void k_scatter4<8, false>(uint64_t, uint32_t, uint32_t, uint32_t, uint32_t, int, const uint32_t*, const uint8_t*,
                                       const uint64_t*, const uint32_t*, const uint32_t*, Rec*, uint64_t*, uint32_t*,
                                       const uint32_t*);
template __global__ void k_scatter4<4, true>(uint64_t, uint32_t, uint32_t, uint32_t, uint32_t, int, const uint32_t*, const uint8_t*,
                                       const uint64_t*, const uint32_t*, const uint32_t*, Rec*, uint64_t*, uint32_t*,
                                       const uint32_t*);
template __global__ void k_scatter4<8, true>(uint64_t, uint32_t, uint32_t, uint32_t, uint32_t, int, const uint32_t*, const uint8_t*,
                                       const uint64_t*, const uint32_t*, const uint32_t*, Rec*, uint64_t*, uint32_t*,
                                       const uint32_t*);
template __global__ void k_scatter4<2, true>(uint64_t, uint32_t, uint32_t, uint32_t, uint32_t, int, const uint32_t*, const uint8_t*,
                                       const uint64_t*, const uint32_t*, const uint32_t*, Rec*, uint64_t*, uint32_t*,
                                       const uint32_t*);

// Multi-block variant for large meshes (sweeps): the same slot order, in
// SCAN_SPAN-entry spans.  Pass 1: span sums; pass 2 (one block): span offsets;
// pass 3: bases within each span.
constexpr uint32_t SCAN_SPAN = 4096;

__device__ __forceinline__ uint32_t scan_slot_of(uint32_t q) { return (q / 25) * (PORTS * INS) + (q % 25); }

__global__ __launch_bounds__(256) void k_scan_span_sums(uint32_t nq, const uint32_t* __restrict__ cnt,
                                                        uint64_t* __restrict__ span_sum)
{
   __shared__ uint64_t red[256];
   const uint32_t q0 = blockIdx.x * SCAN_SPAN, q1 = min(q0 + SCAN_SPAN, nq);
   uint64_t a = 0;
   for (uint32_t q = q0 + threadIdx.x; q < q1; q += 256) a += (cnt[scan_slot_of(q)] + 63) & ~63u;
   red[threadIdx.x] = a;
   __syncthreads();
   for (uint32_t off = 128; off > 0; off >>= 1)
   {
      if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
      __syncthreads();
   }
   if (threadIdx.x == 0) span_sum[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(1024) void k_scan_span_offsets(uint32_t nspan, uint64_t* __restrict__ span_sum,
                                                            const uint64_t* __restrict__ inj_total,
                                                            uint64_t* __restrict__ total)
{
   __shared__ uint64_t part[1024];
   const uint32_t per = (nspan + 1023) / 1024;
   const uint32_t lo = min(threadIdx.x * per, nspan), hi = min(lo + per, nspan);
   uint64_t s = 0;
   for (uint32_t i = lo; i < hi; i++) s += span_sum[i];
   part[threadIdx.x] = s;
   __syncthreads();
   for (uint32_t off = 1; off < 1024; off <<= 1)
   {
      const uint64_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
   }
   uint64_t run = *inj_total + part[threadIdx.x] - s;
   for (uint32_t i = lo; i < hi; i++)
   {
      const uint64_t v = span_sum[i];
      span_sum[i] = run;
      run += v;
   }
   if (threadIdx.x == 1023) *total = *inj_total + part[1023];
}

__global__ __launch_bounds__(256) void k_scan_span_bases(uint32_t nq, uint32_t* __restrict__ cnt,
                                                         const uint64_t* __restrict__ span_off, uint64_t* __restrict__ base,
                                                         const uint64_t* __restrict__ total, uint64_t bound)
{
   __shared__ uint64_t part[256];
   const uint32_t q0 = blockIdx.x * SCAN_SPAN, q1 = min(q0 + SCAN_SPAN, nq);
   const uint32_t per = SCAN_SPAN / 256;
   const uint32_t lo = min(q0 + threadIdx.x * per, q1), hi = min(lo + per, q1);
   uint64_t s = 0;
   for (uint32_t q = lo; q < hi; q++) s += (cnt[scan_slot_of(q)] + 63) & ~63u;
   part[threadIdx.x] = s;
   __syncthreads();
   for (uint32_t off = 1; off < 256; off <<= 1)
   {
      const uint64_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
   }
   uint64_t run = span_off[blockIdx.x] + part[threadIdx.x] - s;
   const bool over = *total > bound;   // (k_scan_slots: the same guard)
   for (uint32_t q = lo; q < hi; q++)
   {
      const uint32_t c = cnt[scan_slot_of(q)];
      base[scan_slot_of(q)] = over ? 0ull : run;
      if (over) cnt[scan_slot_of(q)] = 0;
      run += (c + 63) & ~63u;
   }
}

}  // namespace gnoc
