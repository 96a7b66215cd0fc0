// engine.hip -- host orchestration + C ABI (include/gnoc.h) of the MI355X
// emesh_hop_by_hop timing engine.  Single translation unit with the kernels.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "gnoc.h"
#include "kernels.hip"
#include "kernels_v2.hip"

using namespace gnoc;

namespace {

struct DevBuf
{
   void* p = nullptr;
   size_t bytes = 0;
   ~DevBuf() { release(); }
   void release()
   {
      if (p) (void) hipFree(p);
      p = nullptr;
      bytes = 0;
   }
   hipError_t ensure(size_t want)
   {
      if (want <= bytes && p) return hipSuccess;
      release();
      size_t b = want ? want : 16;
      hipError_t e = hipMalloc(&p, b);
      if (e == hipSuccess) bytes = b;
      return e;
   }
   template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

struct LevelPlan
{
   std::vector<uint32_t> ports;        // all levels concatenated
   std::vector<uint32_t> off;          // level -> [off[l], off[l+1])
};

}  // namespace

struct gnoc_engine
{
   gnoc_config cfg{};
   DevCfg dc{};
   bool f1 = true;
   hipStream_t stream = nullptr;
   hipEvent_t ev0 = nullptr, ev1 = nullptr;
   std::string err;

   // trace
   size_t n = 0;
   bool submitted = false, ran = false;
   const uint64_t* d_inj = nullptr;
   const uint32_t *d_src = nullptr, *d_dst = nullptr, *d_bits = nullptr, *d_flags = nullptr;
   DevBuf t_inj, t_src, t_dst, t_bits, t_flags;

   // work
   DevBuf aux, routed, final_ps, zl, cont;
   DevBuf slot_cnt, slot_base, diff, counters;
   DevBuf dirty, recs, port_sum, port_cnt, port_mg1;
   DevBuf hist, offs, plan_ports;
   DevBuf samp_t, samp_id, nexc, cflags, cstate, lctr, chunks, stamps, portio;
   int force_v1 = 0;          // GNOC_ENGINE=v1, or set after a v2 overflow
   int used_v2 = 0;
   uint64_t h_chunks = 0;
   std::vector<uint32_t> h_slot_cnt;
   uint64_t h_counters[2] = { 0, 0 };
   uint64_t h_records = 0;
   uint32_t h_levels = 0;
   double last_ms = 0.0;
   uint64_t* h_pinned = nullptr;

   // kernel profiling (gnoc_set_profiling)
   bool prof = false;
   std::vector<hipEvent_t> evpool;
   std::vector<int> evkid;     // kernel class per recorded launch
   size_t evused = 0;
   double kms[16] = {};
   uint32_t klaunch[16] = {};
};

enum KernelClass { KC_CLASSIFY, KC_CHAIN, KC_SCAN, KC_INJ_COUNT, KC_INJ_OFFS, KC_INJ_SCATTER, KC_PORT, KC_FINALIZE, KC_INJ_SAMPLES, KC_CHUNK, KC_N };
static const char* const kKernelNames[KC_N] = { "k_classify", "k_chain_prefix", "k_scan_slots", "k_inj_group<count>",
                                                "k_inj_offsets", "k_inj_group<scatter>", "k_port_stream", "k_finalize",
                                                "k_inj_samples", "k_chunk" };

static hipError_t prof_mark(gnoc_engine* e, int kid)
{
   if (!e->prof) return hipSuccess;
   while (e->evpool.size() < e->evused + 2)
   {
      hipEvent_t ev;
      hipError_t r = hipEventCreate(&ev);
      if (r != hipSuccess) return r;
      e->evpool.push_back(ev);
   }
   e->evkid.push_back(kid);
   return hipEventRecord(e->evpool[e->evused++], e->stream);
}
static hipError_t prof_end(gnoc_engine* e)
{
   if (!e->prof) return hipSuccess;
   return hipEventRecord(e->evpool[e->evused++], e->stream);
}

// Launch with optional start/end events (kernel class kid).
#define GNOC_LAUNCH(eng, kid, ...)                                     \
   do                                                                  \
   {                                                                   \
      GNOC_HIP(eng, prof_mark(eng, kid));                              \
      hipLaunchKernelGGL(__VA_ARGS__);                                 \
      GNOC_HIP(eng, hipGetLastError());                                \
      GNOC_HIP(eng, prof_end(eng));                                    \
   } while (0)

#define GNOC_HIP(eng, call)                                                                           \
   do                                                                                                 \
   {                                                                                                  \
      hipError_t e_ = (call);                                                                         \
      if (e_ != hipSuccess)                                                                           \
      {                                                                                               \
         (eng)->err = std::string(#call) + ": " + hipGetErrorString(e_);                              \
         return GNOC_EHIP;                                                                            \
      }                                                                                               \
   } while (0)

static hipError_t prof_collect(gnoc_engine* e)
{
   for (int k = 0; k < KC_N; k++) { e->kms[k] = 0; e->klaunch[k] = 0; }
   if (!e->prof) return hipSuccess;
   for (size_t i = 0; i < e->evkid.size(); i++)
   {
      float ms = 0;
      hipError_t r = hipEventElapsedTime(&ms, e->evpool[2 * i], e->evpool[2 * i + 1]);
      if (r != hipSuccess) return r;
      e->kms[e->evkid[i]] += ms;
      e->klaunch[e->evkid[i]]++;
   }
   return hipSuccess;
}

static int fail(gnoc_engine* e, int code, const std::string& msg)
{
   if (e) e->err = msg;
   return code;
}

extern "C" {

int gnoc_abi_version(void) { return GNOC_ABI_VERSION; }

void gnoc_config_default(gnoc_config* cfg, int32_t num_tiles)
{
   std::memset(cfg, 0, sizeof(*cfg));
   cfg->num_tiles = num_tiles;
   cfg->mesh_width = 0;
   cfg->mesh_height = 0;
   cfg->flit_width = 64;            // carbon_sim.cfg:302
   cfg->router_delay = 1;           // :306
   cfg->link_delay = 1;             // :309
   cfg->frequency_ghz = 1.0;        // dvfs/domains default
   cfg->tile_width_mm = 1.0;        // general/tile_width
   cfg->contention_enabled = 1;     // :312
   cfg->queue_type = GNOC_QUEUE_HISTORY_TREE;   // :313
   cfg->analytical_enabled = 1;     // :392
   cfg->max_list_size = 100;        // :391
   cfg->broadcast_tree_enabled = 1; // :303
   cfg->device = 0;
}

int gnoc_create(const gnoc_config* cfg, gnoc_engine** out)
{
   if (!cfg || !out) return GNOC_EINVAL;
   *out = nullptr;
   gnoc_config c = *cfg;
   // NetworkModelEMeshHopByHop::initializeEMeshTopologyParams, emesh_hop_by_hop.cc:47-70
   if (c.num_tiles <= 0 && (c.mesh_width <= 0 || c.mesh_height <= 0)) return GNOC_EINVAL;
   if (c.mesh_width <= 0 || c.mesh_height <= 0)
   {
      c.mesh_width = (int32_t) std::floor(std::sqrt((double) c.num_tiles));
      c.mesh_height = (int32_t) std::ceil(1.0 * c.num_tiles / c.mesh_width);
   }
   if (c.num_tiles <= 0) c.num_tiles = c.mesh_width * c.mesh_height;
   if (c.num_tiles != c.mesh_width * c.mesh_height) return GNOC_EINVAL;   // :56-58
   if (c.num_tiles > (1 << 15)) return GNOC_EUNSUPPORTED;
   if (c.flit_width <= 0) return GNOC_EINVAL;                             // computeNumFlits(-1) = 0 flits
   if (!(c.frequency_ghz > 0.0)) return GNOC_EINVAL;
   // ElectricalLinkModel delay, electrical_link_model.cc:13-16, asserted at emesh_hop_by_hop.cc:126
   const uint64_t link = (uint64_t) std::ceil(c.frequency_ghz * 0.01 * c.tile_width_mm);
   if (link != c.link_delay) return GNOC_EINVAL;
   if (c.router_delay + c.link_delay == 0) return GNOC_EINVAL;
   if (c.queue_type != GNOC_QUEUE_HISTORY_TREE) return GNOC_EUNSUPPORTED;  // basic/history_list: DESIGN.md "next"
   if (c.contention_enabled && c.max_list_size < 2) return GNOC_EINVAL;    // size-1 tree prunes its only node

   gnoc_engine* e = new (std::nothrow) gnoc_engine;
   if (!e) return GNOC_ENOMEM;
   e->cfg = c;
   e->f1 = (c.frequency_ghz == 1.0);
   DevCfg& d = e->dc;
   d.W = (uint32_t) c.mesh_width;
   d.H = (uint32_t) c.mesh_height;
   d.N = (uint32_t) c.num_tiles;
   d.flit_width = (uint32_t) c.flit_width;
   d.R = c.router_delay;
   d.Lk = c.link_delay;
   d.f = c.frequency_ghz;
   d.rl_ps = e->f1 ? ps_of<true>(c.router_delay + c.link_delay, 1.0) : ps_of<false>(c.router_delay + c.link_delay, c.frequency_ghz);
   d.contention = c.contention_enabled;
   d.analytical = c.analytical_enabled;
   d.max_list = c.max_list_size;
   d.magicW = d.W == 1 ? 0xFFFFFFFFu : (uint32_t) ((1ull << 32) / d.W);

   hipError_t he = hipSetDevice(c.device);
   if (he == hipSuccess) he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
   if (he == hipSuccess) he = hipEventCreate(&e->ev0);
   if (he == hipSuccess) he = hipEventCreate(&e->ev1);
   if (he == hipSuccess) he = hipHostMalloc((void**) &e->h_pinned, 64, hipHostMallocDefault);
   if (he != hipSuccess)
   {
      std::string msg = std::string("HIP init failed: ") + hipGetErrorString(he);
      gnoc_destroy(e);
      (void) msg;
      return GNOC_EHIP;
   }
   *out = e;
   return GNOC_OK;
}

void gnoc_destroy(gnoc_engine* e)
{
   if (!e) return;
   (void) hipSetDevice(e->cfg.device);
   if (e->stream) (void) hipStreamSynchronize(e->stream);
   if (e->ev0) (void) hipEventDestroy(e->ev0);
   if (e->ev1) (void) hipEventDestroy(e->ev1);
   if (e->h_pinned) (void) hipHostFree(e->h_pinned);
   for (hipEvent_t ev : e->evpool) (void) hipEventDestroy(ev);
   if (e->stream) (void) hipStreamDestroy(e->stream);
   delete e;
}

const char* gnoc_last_error(const gnoc_engine* e) { return e ? e->err.c_str() : "null engine"; }

static int validate_host_trace(gnoc_engine* e, const gnoc_packets* pk, size_t n)
{
   const uint32_t N = e->dc.N;
   for (size_t i = 0; i < n; i++)
   {
      if (pk->src[i] >= N || pk->dst[i] >= N) return fail(e, GNOC_ETRACE, "tile id out of range at packet " + std::to_string(i));
      if (i && pk->inject_ps[i] < pk->inject_ps[i - 1]) return fail(e, GNOC_ETRACE, "trace not ordered by inject_ps at packet " + std::to_string(i));
      const uint32_t F = (pk->bits[i] + (uint32_t) e->cfg.flit_width - 1) / (uint32_t) e->cfg.flit_width;
      if (F == 0 && pk->src[i] != pk->dst[i]) return fail(e, GNOC_ETRACE, "zero-flit packet " + std::to_string(i));
      if (F > AUX_F_MAX) return fail(e, GNOC_EUNSUPPORTED, "packet longer than 4095 flits");
   }
   if (n && pk->inject_ps[n - 1] >= (1ull << 50)) return fail(e, GNOC_EUNSUPPORTED, "inject time beyond 2^50 ps");
   return GNOC_OK;
}

int gnoc_submit(gnoc_engine* e, const gnoc_packets* pk, size_t n)
{
   if (!e || !pk) return GNOC_EINVAL;
   if (n && (!pk->inject_ps || !pk->src || !pk->dst || !pk->bits)) return fail(e, GNOC_EINVAL, "null trace array");
   if (n >= (1ull << 32) - 1) return fail(e, GNOC_EUNSUPPORTED, "more than 2^32-2 packets");
   int rc = validate_host_trace(e, pk, n);
   if (rc) return rc;
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   GNOC_HIP(e, e->t_inj.ensure(n * 8));
   GNOC_HIP(e, e->t_src.ensure(n * 4));
   GNOC_HIP(e, e->t_dst.ensure(n * 4));
   GNOC_HIP(e, e->t_bits.ensure(n * 4));
   GNOC_HIP(e, e->t_flags.ensure(n * 4));
   if (n)
   {
      GNOC_HIP(e, hipMemcpyAsync(e->t_inj.p, pk->inject_ps, n * 8, hipMemcpyHostToDevice, e->stream));
      GNOC_HIP(e, hipMemcpyAsync(e->t_src.p, pk->src, n * 4, hipMemcpyHostToDevice, e->stream));
      GNOC_HIP(e, hipMemcpyAsync(e->t_dst.p, pk->dst, n * 4, hipMemcpyHostToDevice, e->stream));
      GNOC_HIP(e, hipMemcpyAsync(e->t_bits.p, pk->bits, n * 4, hipMemcpyHostToDevice, e->stream));
      if (pk->flags)
         GNOC_HIP(e, hipMemcpyAsync(e->t_flags.p, pk->flags, n * 4, hipMemcpyHostToDevice, e->stream));
      else
         GNOC_HIP(e, hipMemsetAsync(e->t_flags.p, 0, n * 4, e->stream));
      GNOC_HIP(e, hipStreamSynchronize(e->stream));
   }
   e->d_inj = e->t_inj.as<uint64_t>();
   e->d_src = e->t_src.as<uint32_t>();
   e->d_dst = e->t_dst.as<uint32_t>();
   e->d_bits = e->t_bits.as<uint32_t>();
   e->d_flags = e->t_flags.as<uint32_t>();
   e->n = n;
   e->submitted = true;
   e->ran = false;
   return GNOC_OK;
}

int gnoc_submit_device(gnoc_engine* e, const gnoc_packets* pk, size_t n)
{
   if (!e || !pk) return GNOC_EINVAL;
   if (n && (!pk->inject_ps || !pk->src || !pk->dst || !pk->bits)) return fail(e, GNOC_EINVAL, "null trace array");
   if (n >= (1ull << 32) - 1) return fail(e, GNOC_EUNSUPPORTED, "more than 2^32-2 packets");
   e->d_inj = pk->inject_ps;
   e->d_src = pk->src;
   e->d_dst = pk->dst;
   e->d_bits = pk->bits;
   e->d_flags = pk->flags;
   e->n = n;
   e->submitted = true;
   e->ran = false;
   return GNOC_OK;
}

static void build_plan(const gnoc_engine* e, LevelPlan& lp)
{
   const uint32_t W = e->dc.W, H = e->dc.H, N = e->dc.N;
   const std::vector<uint32_t>& cnt = e->h_slot_cnt;
   auto nonempty = [&](uint32_t port) {
      for (uint32_t in = 0; in < INS; in++)
         if (cnt[port * INS + in]) return true;
      return false;
   };
   lp.ports.clear();
   lp.off.clear();
   auto push_level = [&](const std::vector<uint32_t>& v) {
      lp.off.push_back((uint32_t) lp.ports.size());
      for (uint32_t p : v)
         if (nonempty(p)) lp.ports.push_back(p);
   };
   std::vector<uint32_t> v;
   // level 0: injection ports
   v.clear();
   for (uint32_t t = 0; t < N; t++) v.push_back(t * PORTS + P_INJ);
   push_level(v);
   // X levels 1..W-1: RIGHT at x = l-1, LEFT at x = W-l (all rows)
   for (uint32_t l = 1; l < W; l++)
   {
      v.clear();
      for (uint32_t y = 0; y < H; y++)
      {
         v.push_back((y * W + (l - 1)) * PORTS + P_RIGHT);
         v.push_back((y * W + (W - l)) * PORTS + P_LEFT);
      }
      push_level(v);
   }
   // Y levels: UP at y = k, DOWN at y = H-1-k
   for (uint32_t k = 0; k + 1 < H; k++)
   {
      v.clear();
      for (uint32_t x = 0; x < W; x++)
      {
         v.push_back((k * W + x) * PORTS + P_UP);
         v.push_back(((H - 1 - k) * W + x) * PORTS + P_DOWN);
      }
      push_level(v);
   }
   // SELF level
   v.clear();
   for (uint32_t t = 0; t < N; t++) v.push_back(t * PORTS + P_SELF);
   push_level(v);
   lp.off.push_back((uint32_t) lp.ports.size());
}


constexpr int GNOC_V2_RETRY = 1000;

static int run_levels_v1(gnoc_engine* e)
{
   const DevCfg& c = e->dc;
   hipStream_t s = e->stream;
   LevelPlan lp;
   build_plan(e, lp);
   GNOC_HIP(e, e->plan_ports.ensure(std::max<size_t>(1, lp.ports.size()) * 4));
   if (!lp.ports.empty())
      GNOC_HIP(e, hipMemcpyAsync(e->plan_ports.p, lp.ports.data(), lp.ports.size() * 4, hipMemcpyHostToDevice, s));
   e->h_levels = (uint32_t) (lp.off.size() - 1);
   for (size_t l = 0; l + 1 < lp.off.size(); l++)
   {
      const uint32_t cnt = lp.off[l + 1] - lp.off[l];
      if (!cnt) continue;
      const uint32_t* ports = e->plan_ports.as<uint32_t>() + lp.off[l];
      if (e->f1)
         GNOC_LAUNCH(e, KC_PORT, k_port_stream<true>, dim3(cnt), dim3(STHREADS), 0, s, c, ports, e->slot_cnt.as<uint32_t>(),
                            e->slot_base.as<uint64_t>(), e->recs.as<Rec>(), e->final_ps.as<uint64_t>(),
                            e->port_sum.as<uint64_t>(), e->port_cnt.as<uint64_t>(), e->port_mg1.as<uint64_t>(),
                            e->dirty.as<uint32_t>(), e->counters.as<unsigned int>() + 8);
      else
         GNOC_LAUNCH(e, KC_PORT, k_port_stream<false>, dim3(cnt), dim3(STHREADS), 0, s, c, ports, e->slot_cnt.as<uint32_t>(),
                            e->slot_base.as<uint64_t>(), e->recs.as<Rec>(), e->final_ps.as<uint64_t>(),
                            e->port_sum.as<uint64_t>(), e->port_cnt.as<uint64_t>(), e->port_mg1.as<uint64_t>(),
                            e->dirty.as<uint32_t>(), e->counters.as<unsigned int>() + 8);
   }
   return GNOC_OK;
}

static int run_levels_v2(gnoc_engine* e)
{
   const DevCfg& c = e->dc;
   hipStream_t s = e->stream;
   const uint32_t N = c.N;
   const uint32_t nslots = N * PORTS * INS;
   LevelPlan lp;
   build_plan(e, lp);
   const size_t nlev = lp.off.size() - 1;
   e->h_levels = (uint32_t) nlev;
   // slot bases exactly as k_scan_slots lays them out (64-record aligned)
   std::vector<uint64_t> hbase((size_t) nslots + 1);
   {
      uint64_t run = 0;
      for (uint32_t i = 0; i < nslots; i++) { hbase[i] = run; run += (e->h_slot_cnt[i] + 63) & ~63u; }
      hbase[nslots] = run;
   }
   // port descriptions + chunk plan: ~C2_TARGET records per chunk, cut on the port's largest input
   std::vector<PortIO> pio;
   std::vector<ChunkDesc> ch;
   std::vector<uint32_t> choff(nlev + 1, 0);
   uint32_t g = 0;
   for (size_t l = 0; l < nlev; l++)
   {
      choff[l] = (uint32_t) ch.size();
      for (uint32_t k = lp.off[l]; k < lp.off[l + 1]; k++)
      {
         const uint32_t port = lp.ports[k];
         PortIO io;
         std::memset(&io, 0, sizeof(io));
         io.port = port;
         io.tile = port / PORTS;
         io.dir = port % PORTS;
         uint64_t tot = 0;
         for (uint32_t in = 0; in < INS; in++)
         {
            const uint32_t sl = port * INS + in;
            const uint32_t n = e->h_slot_cnt[sl];
            tot += n;
            if (n && io.nin < C2_IN)
            {
               io.slot[io.nin] = sl;
               io.base[io.nin] = hbase[sl];
               io.cnt[io.nin] = n;
               io.nmain[io.nin] = n;
               if (n > io.cnt[io.sb]) io.sb = io.nin;
               io.nin++;
            }
         }
         io.ntile = io.tile;
         io.nside = IN_LOCAL;
         if (io.dir == P_RIGHT) { io.ntile = io.tile + 1; io.nside = IN_W; }
         else if (io.dir == P_LEFT) { io.ntile = io.tile - 1; io.nside = IN_E; }
         else if (io.dir == P_UP) { io.ntile = io.tile + c.W; io.nside = IN_S; }
         else if (io.dir == P_DOWN) { io.ntile = io.tile - c.W; io.nside = IN_N; }
         io.nx = io.ntile % c.W;
         io.ny = io.ntile / c.W;
         for (uint32_t d = 0; d < 5; d++)
         {
            const uint32_t os = slot_of(io.ntile, d, io.nside);
            io.oslot[d] = os;
            io.obase[d] = io.dir == P_SELF ? 0 : hbase[os];
            io.ocnt[d] = io.dir == P_SELF ? 0 : e->h_slot_cnt[os];
         }
         const uint32_t pidx = (uint32_t) pio.size();
         pio.push_back(io);
         const uint32_t nc = (uint32_t) std::max<uint64_t>(1, (tot + C2_TARGET - 1) / C2_TARGET);
         for (uint32_t j = 0; j < nc; j++) ch.push_back(ChunkDesc{ pidx, j, nc, g });
         g += nc;
      }
   }
   choff[nlev] = (uint32_t) ch.size();
   e->h_chunks = ch.size();
   GNOC_HIP(e, e->portio.ensure(std::max<size_t>(1, pio.size()) * sizeof(PortIO)));
   if (!pio.empty())
      GNOC_HIP(e, hipMemcpyAsync(e->portio.p, pio.data(), pio.size() * sizeof(PortIO), hipMemcpyHostToDevice, s));
   const uint64_t total = e->h_records;
   GNOC_HIP(e, e->samp_t.ensure((total / 64 + 1) * 8));
   GNOC_HIP(e, e->samp_id.ensure((total / 64 + 1) * 4));
   GNOC_HIP(e, e->nexc.ensure((size_t) nslots * 4));
   GNOC_HIP(e, e->cflags.ensure(std::max<size_t>(1, ch.size()) * 4));
   GNOC_HIP(e, e->cstate.ensure(std::max<size_t>(1, ch.size()) * 16 * 8));
   GNOC_HIP(e, e->lctr.ensure(std::max<size_t>(1, nlev) * 4));
   GNOC_HIP(e, e->chunks.ensure(std::max<size_t>(1, ch.size()) * sizeof(ChunkDesc)));
   GNOC_HIP(e, hipMemsetAsync(e->nexc.p, 0, (size_t) nslots * 4, s));
   GNOC_HIP(e, hipMemsetAsync(e->cflags.p, 0, std::max<size_t>(1, ch.size()) * 4, s));
   GNOC_HIP(e, hipMemsetAsync(e->lctr.p, 0, std::max<size_t>(1, nlev) * 4, s));
   if (!ch.empty())
      GNOC_HIP(e, hipMemcpyAsync(e->chunks.p, ch.data(), ch.size() * sizeof(ChunkDesc), hipMemcpyHostToDevice, s));
   if (e->n)
      GNOC_LAUNCH(e, KC_INJ_SAMPLES, k_inj_samples, dim3(N), dim3(256), 0, s, N, e->slot_cnt.as<uint32_t>(),
                  e->slot_base.as<uint64_t>(), e->recs.as<Rec>(), e->samp_t.as<uint64_t>(), e->samp_id.as<uint32_t>());
   const char* stv = std::getenv("GNOC_STAMPS");
   const bool stamps = stv && *stv == '1';
   if (stamps)
   {
      GNOC_HIP(e, e->stamps.ensure(std::max<size_t>(1, ch.size()) * 16 * 8));
      GNOC_HIP(e, hipMemsetAsync(e->stamps.p, 0, std::max<size_t>(1, ch.size()) * 16 * 8, s));
   }
   for (size_t l = 0; l < nlev; l++)
   {
      const uint32_t cnt = choff[l + 1] - choff[l];
      if (!cnt) continue;
      uint64_t* sp = stamps ? e->stamps.as<uint64_t>() + (uint64_t) choff[l] * 16 : nullptr;
      if (stamps)
      GNOC_LAUNCH(e, KC_CHUNK, k_chunk<true>, dim3(cnt), dim3(C2_T), 0, s, c, e->chunks.as<ChunkDesc>() + choff[l], e->portio.as<PortIO>(),
                  e->lctr.as<unsigned>() + l, e->slot_cnt.as<uint32_t>(), e->slot_base.as<uint64_t>(), e->recs.as<Rec>(),
                  e->samp_t.as<uint64_t>(), e->samp_id.as<uint32_t>(), e->nexc.as<uint32_t>(), e->cflags.as<uint32_t>(),
                  e->cstate.as<uint64_t>(), e->final_ps.as<uint64_t>(), e->port_sum.as<unsigned long long>(),
                  e->port_cnt.as<unsigned long long>(), e->port_mg1.as<unsigned long long>(),
                  e->counters.as<unsigned>() + 8, sp);
      else
      GNOC_LAUNCH(e, KC_CHUNK, k_chunk<false>, dim3(cnt), dim3(C2_T), 0, s, c, e->chunks.as<ChunkDesc>() + choff[l], e->portio.as<PortIO>(),
                  e->lctr.as<unsigned>() + l, e->slot_cnt.as<uint32_t>(), e->slot_base.as<uint64_t>(), e->recs.as<Rec>(),
                  e->samp_t.as<uint64_t>(), e->samp_id.as<uint32_t>(), e->nexc.as<uint32_t>(), e->cflags.as<uint32_t>(),
                  e->cstate.as<uint64_t>(), e->final_ps.as<uint64_t>(), e->port_sum.as<unsigned long long>(),
                  e->port_cnt.as<unsigned long long>(), e->port_mg1.as<unsigned long long>(),
                  e->counters.as<unsigned>() + 8, (uint64_t*) nullptr);
   }
   return GNOC_OK;
}

static int run_once(gnoc_engine* e)
{
   if (!e) return GNOC_EINVAL;
   if (!e->submitted) return fail(e, GNOC_ESTATE, "gnoc_run before gnoc_submit");
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   const DevCfg& c = e->dc;
   const size_t n = e->n;
   const uint32_t N = c.N;
   const uint32_t nslots = N * PORTS * INS;
   const size_t nports = (size_t) N * PORTS;
   hipStream_t s = e->stream;

   GNOC_HIP(e, e->aux.ensure(n * 4));
   GNOC_HIP(e, e->routed.ensure(n));
   GNOC_HIP(e, e->final_ps.ensure(n * 8));
   GNOC_HIP(e, e->zl.ensure(n * 8));
   GNOC_HIP(e, e->cont.ensure(n * 8));
   GNOC_HIP(e, e->slot_cnt.ensure((size_t) nslots * 4));
   GNOC_HIP(e, e->slot_base.ensure(((size_t) nslots + 1) * 8));
   const size_t ndiff = 2 * (size_t) c.H * (c.W + 1) + 2 * (size_t) c.W * (c.H + 1);
   GNOC_HIP(e, e->diff.ensure(ndiff * 4));
   GNOC_HIP(e, e->counters.ensure(64));
   GNOC_HIP(e, e->dirty.ensure((size_t) nslots * 4));
   GNOC_HIP(e, e->port_sum.ensure(nports * 8));
   GNOC_HIP(e, e->port_cnt.ensure(nports * 8));
   GNOC_HIP(e, e->port_mg1.ensure(nports * 8));

   e->evused = 0;
   e->evkid.clear();
   GNOC_HIP(e, hipEventRecord(e->ev0, s));
   GNOC_HIP(e, hipMemsetAsync(e->slot_cnt.p, 0, (size_t) nslots * 4, s));
   GNOC_HIP(e, hipMemsetAsync(e->diff.p, 0, ndiff * 4, s));
   GNOC_HIP(e, hipMemsetAsync(e->counters.p, 0, 64, s));
   GNOC_HIP(e, hipMemsetAsync(e->dirty.p, 0, (size_t) nslots * 4, s));
   GNOC_HIP(e, hipMemsetAsync(e->port_sum.p, 0, nports * 8, s));
   GNOC_HIP(e, hipMemsetAsync(e->port_cnt.p, 0, nports * 8, s));
   GNOC_HIP(e, hipMemsetAsync(e->port_mg1.p, 0, nports * 8, s));

   const uint32_t cls_grid = (uint32_t) std::max<size_t>(1, std::min<size_t>((n + 255) / 256, 8192));
   if (n)
      GNOC_LAUNCH(e, KC_CLASSIFY, k_classify, dim3(cls_grid), dim3(256), 0, s, c, (uint64_t) n, e->d_inj, e->d_src, e->d_dst,
                         e->d_bits, e->d_flags, e->aux.as<uint32_t>(), e->routed.as<uint8_t>(), e->final_ps.as<uint64_t>(),
                         e->slot_cnt.as<uint32_t>(), e->diff.as<int32_t>(), e->counters.as<unsigned long long>());
   GNOC_HIP(e, hipGetLastError());

   if (!c.contention)
   {
      // Queue models disabled (router_model.cc:86): latency is zero-load; no contention counters.
      if (n)
      {
         if (e->f1)
            GNOC_LAUNCH(e, KC_FINALIZE, k_finalize<true>, dim3(cls_grid), dim3(256), 0, s, c, (uint64_t) n, e->d_inj, e->d_src,
                               e->aux.as<uint32_t>(), e->routed.as<uint8_t>(), e->final_ps.as<uint64_t>(),
                               e->zl.as<uint64_t>(), e->cont.as<uint64_t>(), 1);
         else
            GNOC_LAUNCH(e, KC_FINALIZE, k_finalize<false>, dim3(cls_grid), dim3(256), 0, s, c, (uint64_t) n, e->d_inj, e->d_src,
                               e->aux.as<uint32_t>(), e->routed.as<uint8_t>(), e->final_ps.as<uint64_t>(),
                               e->zl.as<uint64_t>(), e->cont.as<uint64_t>(), 1);
      }
      GNOC_HIP(e, hipGetLastError());
      GNOC_HIP(e, hipMemcpyAsync(e->h_pinned, e->counters.p, 16, hipMemcpyDeviceToHost, s));
      GNOC_HIP(e, hipEventRecord(e->ev1, s));
      GNOC_HIP(e, hipStreamSynchronize(s));
      e->h_counters[0] = e->h_pinned[0];
      e->h_counters[1] = e->h_pinned[1];
      e->h_records = 0;
      e->h_levels = 0;
      float ms = 0;
      GNOC_HIP(e, hipEventElapsedTime(&ms, e->ev0, e->ev1));
      e->last_ms = ms;
      e->ran = true;
      return GNOC_OK;
   }

   GNOC_LAUNCH(e, KC_CHAIN, k_chain_prefix, dim3((c.W + c.H + 255) / 256), dim3(256), 0, s, c, e->diff.as<int32_t>(),
                      e->slot_cnt.as<uint32_t>());
   GNOC_LAUNCH(e, KC_SCAN, k_scan_slots, dim3(1), dim3(1024), 0, s, nslots, e->slot_cnt.as<uint32_t>(), e->slot_base.as<uint64_t>());
   GNOC_HIP(e, hipGetLastError());

   // read back slot counts (route-static layout) and the record total
   e->h_slot_cnt.resize(nslots);
   GNOC_HIP(e, hipMemcpyAsync(e->h_pinned, e->slot_base.as<uint64_t>() + nslots, 8, hipMemcpyDeviceToHost, s));
   GNOC_HIP(e, hipMemcpyAsync(e->h_pinned + 1, e->counters.p, 16, hipMemcpyDeviceToHost, s));
   GNOC_HIP(e, hipMemcpyAsync(e->h_slot_cnt.data(), e->slot_cnt.p, (size_t) nslots * 4, hipMemcpyDeviceToHost, s));
   GNOC_HIP(e, hipStreamSynchronize(s));
   const uint64_t total = e->h_pinned[0];
   e->h_counters[0] = e->h_pinned[1];
   e->h_counters[1] = e->h_pinned[2];
   e->h_records = total;
   GNOC_HIP(e, e->recs.ensure(total * sizeof(Rec)));

   // injection grouping
   if (n)
   {
      uint32_t chunk = 4096;
      while ((n + chunk - 1) / chunk * (uint64_t) N > (64ull << 20)) chunk *= 2;
      const uint32_t nchunks = (uint32_t) ((n + chunk - 1) / chunk);
      int nbits = 0;
      while ((1u << nbits) < N) nbits++;
      GNOC_HIP(e, e->hist.ensure((size_t) nchunks * N * 4));
      GNOC_HIP(e, e->offs.ensure((size_t) nchunks * N * 8));
      GNOC_LAUNCH(e, KC_INJ_COUNT, k_inj_group<false>, dim3(nchunks), dim3(64), N * 4, s, (uint64_t) n, chunk, N, nbits, e->d_src,
                         e->routed.as<uint8_t>(), e->d_inj, e->aux.as<uint32_t>(), e->hist.as<uint32_t>(),
                         (const uint64_t*) nullptr, (Rec*) nullptr, nchunks);
      GNOC_LAUNCH(e, KC_INJ_OFFS, k_inj_offsets, dim3(N), dim3(256), 0, s, nchunks, e->hist.as<uint32_t>(),
                         e->slot_base.as<uint64_t>(), e->offs.as<uint64_t>());
      GNOC_LAUNCH(e, KC_INJ_SCATTER, k_inj_group<true>, dim3(nchunks), dim3(64), N * 4, s, (uint64_t) n, chunk, N, nbits, e->d_src,
                         e->routed.as<uint8_t>(), e->d_inj, e->aux.as<uint32_t>(), e->hist.as<uint32_t>(),
                         e->offs.as<uint64_t>(), e->recs.as<Rec>(), nchunks);
      GNOC_HIP(e, hipGetLastError());
   }

   const bool v2 = e->f1 && c.max_list >= 3 && !e->force_v1;
   e->used_v2 = v2;
   if (v2)
   {
      int rc = run_levels_v2(e);
      if (rc) return rc;
   }
   else
   {
      int rc = run_levels_v1(e);
      if (rc) return rc;
   }

   if (n)
   {
      if (e->f1)
         GNOC_LAUNCH(e, KC_FINALIZE, k_finalize<true>, dim3(cls_grid), dim3(256), 0, s, c, (uint64_t) n, e->d_inj, e->d_src,
                            e->aux.as<uint32_t>(), e->routed.as<uint8_t>(), e->final_ps.as<uint64_t>(), e->zl.as<uint64_t>(),
                            e->cont.as<uint64_t>(), 0);
      else
         GNOC_LAUNCH(e, KC_FINALIZE, k_finalize<false>, dim3(cls_grid), dim3(256), 0, s, c, (uint64_t) n, e->d_inj, e->d_src,
                            e->aux.as<uint32_t>(), e->routed.as<uint8_t>(), e->final_ps.as<uint64_t>(), e->zl.as<uint64_t>(),
                            e->cont.as<uint64_t>(), 0);
   }
   GNOC_HIP(e, hipGetLastError());
   GNOC_HIP(e, hipEventRecord(e->ev1, s));
   GNOC_HIP(e, hipMemcpyAsync(e->h_pinned + 4, e->counters.as<unsigned int>() + 8, 4, hipMemcpyDeviceToHost, s));
   GNOC_HIP(e, hipStreamSynchronize(s));
   float ms = 0;
   GNOC_HIP(e, hipEventElapsedTime(&ms, e->ev0, e->ev1));
   e->last_ms = ms;
   GNOC_HIP(e, prof_collect(e));
   const unsigned errf = *(unsigned int*) (e->h_pinned + 4);
   if (errf & 1u) return fail(e, GNOC_EHIP, "internal: route-count invariant violated");
   if (errf & 6u) return GNOC_V2_RETRY;   // burst beyond the chunk splitter / look-back timeout
   e->ran = true;
   return GNOC_OK;
}

int gnoc_run(gnoc_engine* e)
{
   if (!e) return GNOC_EINVAL;
   const char* env = std::getenv("GNOC_ENGINE");
   const int forced = env && std::strcmp(env, "v1") == 0;
   e->force_v1 = forced;
   int rc = run_once(e);
   if (rc == GNOC_V2_RETRY)
   {
      e->force_v1 = 1;   // exact but slower whole-port streams
      rc = run_once(e);
      e->force_v1 = forced;
      if (rc == GNOC_V2_RETRY) rc = fail(e, GNOC_EHIP, "internal: v1 path reported overflow");
   }
   return rc;
}

int gnoc_get_packet_results(gnoc_engine* e, uint64_t* final_ps, uint64_t* zero_load_ps, uint64_t* contention_ps, size_t n)
{
   if (!e) return GNOC_EINVAL;
   if (!e->ran) return fail(e, GNOC_ESTATE, "no results: call gnoc_run first");
   if (n != e->n) return fail(e, GNOC_EINVAL, "result array length != submitted packet count");
   if (!n) return GNOC_OK;
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   if (final_ps) GNOC_HIP(e, hipMemcpyAsync(final_ps, e->final_ps.p, n * 8, hipMemcpyDeviceToHost, e->stream));
   if (zero_load_ps) GNOC_HIP(e, hipMemcpyAsync(zero_load_ps, e->zl.p, n * 8, hipMemcpyDeviceToHost, e->stream));
   if (contention_ps) GNOC_HIP(e, hipMemcpyAsync(contention_ps, e->cont.p, n * 8, hipMemcpyDeviceToHost, e->stream));
   GNOC_HIP(e, hipStreamSynchronize(e->stream));
   return GNOC_OK;
}

int gnoc_get_port_stats(gnoc_engine* e, uint64_t* sum_delay, uint64_t* count, uint64_t* mg1_uses, size_t nports)
{
   if (!e) return GNOC_EINVAL;
   if (!e->ran) return fail(e, GNOC_ESTATE, "no results: call gnoc_run first");
   const size_t np = (size_t) e->dc.N * PORTS;
   if (nports != np) return fail(e, GNOC_EINVAL, "nports != num_tiles*6");
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   if (!e->dc.contention)
   {
      if (sum_delay) std::memset(sum_delay, 0, np * 8);
      if (count) std::memset(count, 0, np * 8);
      if (mg1_uses) std::memset(mg1_uses, 0, np * 8);
      return GNOC_OK;
   }
   if (sum_delay) GNOC_HIP(e, hipMemcpyAsync(sum_delay, e->port_sum.p, np * 8, hipMemcpyDeviceToHost, e->stream));
   if (count) GNOC_HIP(e, hipMemcpyAsync(count, e->port_cnt.p, np * 8, hipMemcpyDeviceToHost, e->stream));
   if (mg1_uses) GNOC_HIP(e, hipMemcpyAsync(mg1_uses, e->port_mg1.p, np * 8, hipMemcpyDeviceToHost, e->stream));
   GNOC_HIP(e, hipStreamSynchronize(e->stream));
   return GNOC_OK;
}

int gnoc_get_summary(gnoc_engine* e, gnoc_summary* out)
{
   if (!e || !out) return GNOC_EINVAL;
   std::memset(out, 0, sizeof(*out));
   out->packets = e->n;
   out->mesh_hops = e->h_counters[0];
   out->routed_packets = e->h_counters[1];
   out->records = e->h_records;
   out->levels = e->h_levels;
   out->last_run_ms = e->last_ms;
   out->engine_path = e->dc.contention ? (uint32_t) e->used_v2 : 2u;
   if (e->ran && e->dc.contention)
   {
      std::vector<uint64_t> m((size_t) e->dc.N * PORTS);
      GNOC_HIP(e, hipSetDevice(e->cfg.device));
      GNOC_HIP(e, hipMemcpy(m.data(), e->port_mg1.p, m.size() * 8, hipMemcpyDeviceToHost));
      for (uint64_t v : m) out->mg1_uses += v;
   }
   return GNOC_OK;
}

int gnoc_set_profiling(gnoc_engine* e, int enable)
{
   if (!e) return GNOC_EINVAL;
   e->prof = enable != 0;
   return GNOC_OK;
}

int gnoc_get_kernel_stats(gnoc_engine* e, const char** names, double* total_ms, uint32_t* launches, size_t cap,
                          size_t* count)
{
   if (!e || !count) return GNOC_EINVAL;
   *count = KC_N;
   for (size_t k = 0; k < (size_t) KC_N && k < cap; k++)
   {
      if (names) names[k] = kKernelNames[k];
      if (total_ms) total_ms[k] = e->kms[k];
      if (launches) launches[k] = e->klaunch[k];
   }
   return GNOC_OK;
}

extern "C" __attribute__((visibility("default"))) int gnoc_debug_stamps(gnoc_engine* e, uint64_t* out, size_t cap,
                                                                     size_t* nchunks)
{
   if (!e || !nchunks) return GNOC_EINVAL;
   *nchunks = e->h_chunks;
   if (!out || !e->stamps.p) return GNOC_OK;
   const size_t n = std::min(cap, (size_t) e->h_chunks * 16);
   GNOC_HIP(e, hipMemcpy(out, e->stamps.p, n * 8, hipMemcpyDeviceToHost));
   return GNOC_OK;
}

int gnoc_device_final_ps(gnoc_engine* e, void** dptr)
{
   if (!e || !dptr) return GNOC_EINVAL;
   if (!e->ran) return fail(e, GNOC_ESTATE, "no results: call gnoc_run first");
   *dptr = e->final_ps.p;
   return GNOC_OK;
}

}  // extern "C"
