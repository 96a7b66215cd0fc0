// engine.hip -- host orchestration + C ABI (include/gnoc.h) of the MI355X
// emesh_hop_by_hop timing engine.  Single translation unit with the kernels.
//
// A run is one fixed sequence of launches on the engine's stream:
//   prep (prep.hip)   classify -> injection-slot layout -> stable scatter ->
//                     row histograms -> slot counts -> slot bases
//   plan (level.hip)  per-port descriptors and chunk -> port maps, on device
//   levels            one persistent k_level launch per level of the port DAG
//   finalize          zero-load / contention per packet
// The v3 path never waits for the host between launches.  Configurations the
// chunked path does not cover (f != 1 GHz, max_list_size <= 2) and the rare
// overflow retry use the whole-port stream kernel of kernels.hip (v1), whose
// plan is built on the host from the read-back slot counts.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "gnoc.h"
#include "kernels.hip"
#include "level.hip"
#define LV_GEN 1
#include "level.hip"   // lvg::k_level: any network frequency
#include "prep.hip"
#include "shard.hip"
#include "serial.hip"
#include "chain.hip"


namespace gnoc {
// Packets per prep chunk (k_classify / k_scatter blocks): each chunk keeps an
// N-entry source histogram (hist = 4 B per packet at most), and more, smaller
// chunks keep enough waves in flight for the per-packet latency chains of the
// scatter (16,384-tile sweeps: 65,536 -> 16,384 packets per chunk).
// Trace packets per prep workgroup (k_classify histograms, k_scatter4 ranks).
// configs[1] (GNOC_PREP_CHUNK): 16384 -> 4.025 ms per step, 8192 -> 3.965
// (k_scatter4 0.26 -> 0.23 ms), 4096 -> 3.977 (k_classify's per-chunk
// histograms grow), 2048 -> 4.002.
static inline uint32_t prep_chunk(uint32_t N)
{
   const char* v = std::getenv("GNOC_PREP_CHUNK");
   const uint32_t base = v && std::atoi(v) >= 1024 ? (uint32_t) std::atoi(v) : 8192u;
   return std::max<uint32_t>(base, (N + 63u) & ~63u);
}
}  // namespace gnoc

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
   void swap(DevBuf& o)
   {
      std::swap(p, o.p);
      std::swap(bytes, o.bytes);
   }
};

}  // namespace

enum KernelClass
{
   KC_CLASSIFY, KC_SRC_TOT, KC_INJ_BASE, KC_SRC_OFFS, KC_SCATTER, KC_ROW_HIST, KC_PROW, KC_SLOT_COUNTS, KC_SCAN,
   KC_PLAN, KC_LEVEL, KC_PORT, KC_FINALIZE, KC_BCAST, KC_CHAIN, KC_BOUNDS, KC_INJ, KC_N
};
static const char* const kKernelNames[KC_N] = { "k_classify", "k_src_tot", "k_inj_base", "k_src_offs", "k_scatter",
                                                "k_row_hist", "k_prow", "k_slot_counts", "k_scan_slots", "k_plan",
                                                "k_level", "k_port_stream", "k_finalize", "k_bcast",
                                                "k_chain", "k_win_bounds", "k_inj_stream" };

struct gnoc_engine
{
   gnoc_config cfg{};
   DevCfg dc{};
   bool f1 = true;
   hipStream_t stream = nullptr;
   hipEvent_t ev0 = nullptr, ev1 = nullptr;
   std::string err;
   int level_grid = 0;

   // static level plan of the port DAG (host + device copies)
   std::vector<uint32_t> lvl_ports, lvl_off, port_k;
   DevBuf d_lvl_ports, d_lvl_off, d_port_k;

   // trace
   size_t n = 0;
   uint64_t rec_bound = 0;    // records incl. slot padding (from the trace at submit)
   uint32_t runs = 0, tot_retry = 0, tot_fallback = 0;   // since the last submit (gnoc_summary)
   bool submitted = false, ran = false;
   int inj_bnd = 0;   // this run's k_inj_stream wrote the IN_LOCAL window bounds (unless it declined)
   int inj_host = 0;       // this run's k_inj_stream has no k_level behind it: a decline reruns the batch
   int inj_declined = 0;   // this batch's injection queues fire M/G/1 (or span wide blocks): k_level's level
   const uint64_t* d_inj = nullptr;
   const uint32_t *d_src = nullptr, *d_dst = nullptr, *d_bits = nullptr, *d_flags = nullptr;
   DevBuf t_inj, t_src, t_dst, t_bits, t_flags;
   DevBuf vbuf;                             // submit-time checks and statistics (k_validate)
   // pipelined batches (gnoc_submit_async / gnoc_submit_commit / gnoc_fetch_final_ps):
   // the next batch's trace lands in a second buffer set on a copy stream while a
   // run computes; a run's final_ps is read back on another copy stream while the
   // next run writes a second final_ps buffer (ev_fin / ev_alt: the last read-back
   // of each buffer)
   hipStream_t s_h2d = nullptr, s_d2h = nullptr;
   hipEvent_t ev_h2d = nullptr, ev_done = nullptr, ev_fin = nullptr, ev_alt = nullptr;
   DevBuf t2_inj, t2_src, t2_dst, t2_bits, t2_flags, final_alt;
   // gnoc_fetch_latency: k_finalize also writes final_ps - inject_ps as u32 (double
   // buffered with final_ps) once a caller has asked for it; lat_ovf: one did not fit
   DevBuf lat32, lat32_alt;
   bool want_lat32 = false, lat_ovf = false, lat_written = false;
   DevBuf nw_stage, nw_stage2;               // narrow wire format (gnoc_packets_narrow) before widening
   bool staged_narrow = false;
   bool staged = false, fetched = false;
   gnoc_packets staged_pk{};
   size_t staged_n = 0;
   // gnoc_run_sharded: the engine's own exchange buffers and transport
   DevBuf xsend, xrecv, xflag;
   gnoc_transport tp{};
   void* nccl = nullptr;                    // ncclComm_t (gnoc_shard_set_comm)

   // work
   DevBuf aux, routed, final_ps, zl, cont;
   DevBuf hist, tot, slot_cnt, slot_base, counters, gtot;
   DevBuf recs, samp_t, samp_id, Hs, Pp, Prow, pcol, nexc, dirty, span, srcseg;
   DevBuf pio, pnc, pgb, lvl_cbase, lvl_qb, cdesc, flags, st, lvl_ctr;
   DevBuf port_sum, port_cnt, port_mg1, port_flit, port_last, plan_ports, stamps, done;
   uint64_t h_chunk_bound = 0;
   int force_v1 = 0;
   int used_v3 = 0;
   std::vector<uint32_t> h_slot_cnt;
   uint64_t h_counters[2] = { 0, 0 };
   uint64_t h_records = 0;
   uint32_t h_levels = 0;
   double last_ms = 0.0;
   uint64_t* h_pinned = nullptr;
   uint64_t* h_val = nullptr;               // (pinned, 128 B) a staged batch's ValOut
   DevBuf vbuf2;                            // a staged batch's validation scratch (upload stream)
   bool staged_val = false;                 // the staged batch was validated on the upload stream
   // a delta-format batch (stage_packed): its decoded escape count on the device and
   // the absolute times the caller gave, checked by the validation that follows
   uint64_t layout_bound = 0;   // records the slot layout may span (run_prep)
   const uint64_t* val_esc = nullptr;
   uint64_t val_nabs = 0;

   // a sharded rank's partitioned trace (gnoc_submit): only the packets of its
   // row band (sources) or column band (destinations), in trace order; gid maps
   // them to their global index.  Its delivery level writes final times by global
   // id into fin_glob (a plain scattered store), and k_finalize reads the rank's
   // delivered packets' back by gid.
   bool part = false;
   int xself = 0;                           // test knob GNOC_SHARD_SELF_EXCHANGE: own turn records through the transport
   int declined_once = 0;                   // test knob GNOC_DECLINE_ONCE_RANK: fired
   bool fin_closed = false;                 // finish_enqueue: the closed form finished in run_begin
   size_t n_glob = 0;
   uint64_t h_glob_hops = 0, h_glob_routed = 0;
   std::vector<uint32_t> h_gid;
   DevBuf d_gid, fin_glob;

   // one mesh over several GPUs (gnoc_shard): this rank's row band (X phase)
   // and column band (Y phase), the turn-record exchange layout per peer
   int rank = 0, nranks = 1;
   uint32_t ry0 = 0, ry1 = 0, cx0 = 0, cx1 = 0;
   uint32_t lvl_y0 = 0;                     // index of the first Y level
   std::vector<uint64_t> x_cnt;             // [r * n + d]: turn records row band r -> column band d
   std::vector<XPair> xs_pairs, xr_pairs;   // send / receive layouts (peers in rank order)
   uint32_t xs_slots = 0, xr_slots = 0;
   std::vector<uint64_t> xs_units, xr_units;
   DevBuf d_xs_pairs, d_xr_pairs, xs_off, xr_off;
   bool begun = false;

   // broadcast tree (emesh_hop_by_hop.cc:163-221): packet id -> broadcast index,
   // broadcast -> packet id, per-visit max delays (two passes), receipts
   uint32_t nb = 0;
   uint32_t bc_passes = 0;
   std::vector<uint32_t> h_bid;
   DevBuf d_bidx, d_bid, d_bv[2], d_bfin, d_bzl, d_bct, d_bflag, d_bcnt, d_btail;

   // design-space sweep (gnoc_create_sweep): per-point tables
   int32_t npoints = 1;
   std::vector<uint64_t> h_pt_rl;
   std::vector<uint32_t> h_pt_fw;
   DevBuf d_pt_rl, d_pt_fw;

   // QueueModelBasic with a moving average (gnoc_set_basic_moving_average, serial.hip)
   int ma_type = 0;
   uint32_t ma_window = 1;
   DevBuf ma_t, ma_key, ma_val, ma_key2, ma_val2, ma_lo, ma_hi, ma_d, ma_ref, ma_agg, ma_m, ma_bcnt, ma_hist;
   DevBuf sc_key, sc_rec, sc_hist;          // injection slots of large meshes (radix sort by source)

   // v4 chain engine (chain.hip): per phase (X, Y), per chain, windows of chD ps
   // (sized at submit, then from the fill each run measured per chain)
   bool ch_on = false;
   uint64_t ch_key[4] = { 0, 0, 0, 0 };      // the shape of the batch the windows were sized for
   uint64_t h_tlast = 0;                     // last injection time of the batch (k_validate)
   std::vector<uint64_t> chD[2], chCap[2];   // window length; a length that overflowed LDS (0: none)
   std::vector<uint64_t> chD_run[2];         // the attempt in flight
   std::vector<uint64_t> chD_up[2];          // the window keys the device tables hold (win_key)
   // variable windows (adapt_windows): per chain its boundaries in ps (nW + 1 of them,
   // the last ~0), empty while the chain has uniform windows of chD; chB_D the chD
   // they belong to (a halving changes chD_run and the chain runs uniform windows again)
   std::vector<std::vector<uint64_t>> chB[2];
   std::vector<uint64_t> chB_D[2];
   uint32_t ch_qs = 0;                      // device boundaries in units of 2^qs ps (u32)
   int ch_adapt_left = 0;                   // variable-window adaptations left for this batch shape
   std::vector<uint32_t> h_wt;              // both phases' boundaries as the device holds them
   uint32_t* h_wfill = nullptr;             // (pinned) the last chain run's per-window fills
   size_t h_wfill_cap = 0;
   DevBuf ch_wt, ch_wfill;
   int ch_wfill_read = 0;                   // this run's fills were read back (run_post_enqueue)
   std::vector<ChainWin> h_cw[2];
   std::vector<uint32_t> h_tasks[2];
   // XCD-local task queues (chain.hip deq_init): per phase the first task of each of the
   // ch::NQ queues in h_tasks (chains assigned by their windows), the mode the tables
   // were built for, and whether a run found an XCD without workgroups (then off)
   std::vector<uint32_t> h_qoff[2];
   int ch_xcd_tab = -1, ch_xcd_off = 0;
   uint64_t ch_st_words[2] = { 0, 0 }, ch_bt_words[2] = { 0, 0 };
   unsigned* h_nmax = nullptr;               // pinned: per chain fill maxima of the last run
   DevBuf ch_cw, ch_tasks, ch_nmax;
   uint32_t ch_epoch = 0;
   int ch_grid = 0;
   int ncu = 256;                           // compute units of the device
   int force_levels = 0;
   int ch_declined = 0;                     // this batch fell back from the chain engine: later runs skip it
   int ch_ydeclined = 0;                    // only its Y phase did: later runs take X chains + Y levels (path 5)
   unsigned ch_yflags = 0;                  // the Y phase's chain flags of the last run that declined
   int exc_fix = 0;                         // this batch's injection level leaves exception tails: k_exc_merge
   int ch_mg = 0;                           // this batch's chains meet the no-gap M/G/1 branch: k_chain's MG instantiation
   // MG batches: per phase and chain, the windows that may serve M/G/1 requests (from
   // the last MG run on these windows); those run on the MG instantiation, the rest of
   // the phase on the common one (chain_phase)
   std::vector<uint32_t> h_mgk[2], up_mgk[2], h_tasks2[2];
   std::vector<uint64_t> mgk_D[2];          // the windows h_mgk was measured on
   void* up_p[2] = { nullptr, nullptr };
   int mgk_ok = 0, ch_split = 0;
   int ch_ylocal = 0;   // this run's Y IN_LOCAL window bounds were made beside the X phase's
   DevBuf ch_tasks2;
   std::vector<std::pair<void*, uint64_t>> zq;   // buffers to zero before the first level launch (one k_zero_segs)
   int ch_resized = 0;                      // the windows were already changed during this (sharded) run
   int used_chain = 0;
   uint32_t ncpx = 0, ncpy = 0;
   DevBuf ch_cp, ch_bt, ch_st, ch_ctr, ch_stamps0, ch_stamps1;
   uint32_t n_retry = 0, n_fallback = 0;    // reruns of the last gnoc_run (chain -> smaller windows / levels, v3 -> v1)
   // per phase, the hand-off protocol of k_chain (0: each window waits for window w-1's
   // inclusive state; 1: look-back over earlier windows' aggregates): both are exact, and
   // each is timed once on the settled windows, then the faster one runs
   uint32_t ch_lb_run[2] = { 0, 0 };
   float ch_lb_ms[2][2] = { { -1.f, -1.f }, { -1.f, -1.f } };
   std::vector<uint64_t> ch_lb_D[2];        // the windows those times belong to
   std::vector<uint64_t> ch_prevD[2];       // the windows of the previous attempt
   int ch_lb_dec[2] = { -1, -1 };           // the decision per phase (-1: none yet: serial)
   int ch_trial = 0;                        // this run times a protocol (phases as separate launches)
   hipEvent_t ch_ev[2][2] = { { nullptr, nullptr }, { nullptr, nullptr } };

   // kernel profiling (gnoc_set_profiling)
   bool prof = false;
   std::vector<hipEvent_t> evpool;
   std::vector<int> evkid;
   size_t evused = 0;
   double kms[KC_N] = {};
   uint32_t klaunch[KC_N] = {};
};

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

// Launch with optional start/end events (kernel class kid).
#define GNOC_LAUNCH(eng, kid, ...)                                     \
   do                                                                  \
   {                                                                   \
      GNOC_HIP(eng, prof_mark(eng, kid));                              \
      hipLaunchKernelGGL(__VA_ARGS__);                                 \
      GNOC_HIP(eng, hipGetLastError());                                \
      GNOC_HIP(eng, prof_end(eng));                                    \
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

// Levels of the output-port DAG under XY routing: injection ports; X levels
// (RIGHT at x = l-1, LEFT at x = W-l, every row); Y levels (UP at y = k, DOWN at
// y = H-1-k, every column); SELF ports.  Every port's producers sit in earlier levels.
// A sharded engine keeps the injection and X ports of its row band and the Y and
// SELF ports of its column band (shard.hip); the level sequence stays the same.
static uint32_t band_lo(uint32_t b, uint32_t n, uint32_t D) { return (uint32_t) ((uint64_t) b * D / n); }

static void build_static_levels(gnoc_engine* e)
{
   const uint32_t W = e->dc.W, H = e->dc.H, N = e->dc.N;
   const uint32_t n = (uint32_t) e->nranks, r = (uint32_t) e->rank;
   e->ry0 = band_lo(r, n, H);
   e->ry1 = band_lo(r + 1, n, H);
   e->cx0 = band_lo(r, n, W);
   e->cx1 = band_lo(r + 1, n, W);
   auto& P = e->lvl_ports;
   auto& O = e->lvl_off;
   P.clear();
   O.clear();
   O.push_back(0);
   for (uint32_t y = e->ry0; y < e->ry1; y++)
      for (uint32_t x = 0; x < W; x++) P.push_back((y * W + x) * PORTS + P_INJ);
   O.push_back((uint32_t) P.size());
   // a sweep mesh is a grid of independent BW x BH blocks: levels by in-block coordinate
   const uint32_t BW = e->dc.BW, BH = e->dc.BH;
   for (uint32_t l = 1; l < BW; l++)
   {
      for (uint32_t y = e->ry0; y < e->ry1; y++)
         for (uint32_t b0 = 0; b0 < W; b0 += BW)
         {
            P.push_back((y * W + b0 + (l - 1)) * PORTS + P_RIGHT);
            P.push_back((y * W + b0 + (BW - l)) * PORTS + P_LEFT);
         }
      O.push_back((uint32_t) P.size());
   }
   e->lvl_y0 = (uint32_t) O.size() - 1;
   for (uint32_t k = 0; k + 1 < BH; k++)
   {
      for (uint32_t b0 = 0; b0 < H; b0 += BH)
         for (uint32_t x = e->cx0; x < e->cx1; x++)
         {
            P.push_back(((b0 + k) * W + x) * PORTS + P_UP);
            P.push_back(((b0 + BH - 1 - k) * W + x) * PORTS + P_DOWN);
         }
      O.push_back((uint32_t) P.size());
   }
   for (uint32_t y = 0; y < H; y++)
      for (uint32_t x = e->cx0; x < e->cx1; x++) P.push_back((y * W + x) * PORTS + P_SELF);
   O.push_back((uint32_t) P.size());
   e->port_k.assign((size_t) N * PORTS, 0xFFFFFFFFu);   // port id -> plan index (none: another rank's port)
   for (uint32_t k = 0; k < (uint32_t) P.size(); k++) e->port_k[P[k]] = k;
}

static hipError_t upload_levels(gnoc_engine* e)
{
   hipError_t he = e->d_lvl_ports.ensure(std::max<size_t>(1, e->lvl_ports.size()) * 4);
   if (he == hipSuccess) he = e->d_lvl_off.ensure(e->lvl_off.size() * 4);
   if (he == hipSuccess) he = e->d_port_k.ensure(e->port_k.size() * 4);
   if (he == hipSuccess) he = hipMemcpy(e->d_port_k.p, e->port_k.data(), e->port_k.size() * 4, hipMemcpyHostToDevice);
   if (he == hipSuccess && !e->lvl_ports.empty())
      he = hipMemcpy(e->d_lvl_ports.p, e->lvl_ports.data(), e->lvl_ports.size() * 4, hipMemcpyHostToDevice);
   if (he == hipSuccess) he = hipMemcpy(e->d_lvl_off.p, e->lvl_off.data(), e->lvl_off.size() * 4, hipMemcpyHostToDevice);
   return he;
}

extern "C" {

int gnoc_abi_version(void) { return GNOC_ABI_VERSION; }
#ifndef GNOC_BUILD_ID
#define GNOC_BUILD_ID "unknown"
#endif
const char* gnoc_build_id(void) { return GNOC_BUILD_ID; }

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
   if (c.num_tiles > (1 << 14)) return GNOC_EUNSUPPORTED;
   if (c.mesh_width > (int32_t) MESH_DIM_MAX || c.mesh_height > (int32_t) MESH_DIM_MAX) return GNOC_EUNSUPPORTED;
   if (c.flit_width <= 0) return GNOC_EINVAL;                             // computeNumFlits(-1) = 0 flits
   if (!(c.frequency_ghz > 0.0)) return GNOC_EINVAL;
   // ElectricalLinkModel delay, electrical_link_model.cc:13-16, asserted at emesh_hop_by_hop.cc:126
   const uint64_t link = (uint64_t) std::ceil(c.frequency_ghz * 0.01 * c.tile_width_mm);
   if (link != c.link_delay) return GNOC_EINVAL;
   if (c.router_delay + c.link_delay == 0) return GNOC_EINVAL;
   if (c.queue_type != GNOC_QUEUE_HISTORY_TREE && c.queue_type != GNOC_QUEUE_BASIC &&
       c.queue_type != GNOC_QUEUE_HISTORY_LIST)
      return GNOC_EINVAL;                                                   // queue_model.cc:33-36
   if (c.contention_enabled && c.queue_type != GNOC_QUEUE_BASIC && c.max_list_size < 2)
      return GNOC_EINVAL;                                                   // size-1 tree prunes its only node

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
   if (c.queue_type == GNOC_QUEUE_BASIC)
   {
      // QueueModelBasic without moving average: FIFO, no analytical model, no pruning
      d.analytical = 0;
      d.max_list = 1 << 30;
   }
   else if (c.queue_type == GNOC_QUEUE_HISTORY_LIST && d.max_list < 3)
   {
      // the list prunes after inserting (size > max, history_list.cc:138-141): at
      // max_list_size 2 a gap, once made, is never the last one removed -- the
      // tree's behaviour at max_list_size >= 3
      d.max_list = 3;
   }
   d.magicW = d.W == 1 ? 0xFFFFFFFFu : (uint32_t) ((1ull << 32) / d.W);
   d.BW = d.W;
   d.BH = d.H;
   d.BX = 1;
   d.hop_counter = 0;
   d.pt_rl = nullptr;
   d.pt_fw = nullptr;
   build_static_levels(e);

   hipError_t he = hipSetDevice(c.device);
   if (he == hipSuccess) he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
   if (he == hipSuccess) he = hipEventCreate(&e->ev0);
   if (he == hipSuccess) he = hipEventCreate(&e->ev1);
   if (he == hipSuccess) he = hipHostMalloc((void**) &e->h_pinned, 256, hipHostMallocDefault);
   if (he == hipSuccess) he = hipHostMalloc((void**) &e->h_val, 128, hipHostMallocDefault);
   // per chain fill maxima: 2 u32 for each of the <= 2 (W + H) chains
   if (he == hipSuccess)
      he = hipHostMalloc((void**) &e->h_nmax, 32 * ((size_t) e->dc.W + e->dc.H) + 64, hipHostMallocDefault);
   if (he == hipSuccess) he = upload_levels(e);
   if (he == hipSuccess)
   {
      int per_cu = 0, cus = 0;
      he = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_level<false, true, false>, LV_T, 0);
      if (he == hipSuccess) he = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.device);
      e->level_grid = std::max(1, per_cu) * std::max(1, cus);
      // the chain kernels' residency (a grid beyond it only queues: tasks are handed out in order)
      int c1 = 0, c3 = 0;
      if (he == hipSuccess) he = hipOccupancyMaxActiveBlocksPerMultiprocessor(&c1, ch::k_chain<1, true, false>, ch::T, 0);
      if (he == hipSuccess) he = hipOccupancyMaxActiveBlocksPerMultiprocessor(&c3, ch::k_chain<3, true, true>, ch::T, 0);
      e->ch_grid = std::max(1, std::min(c1, c3)) * std::max(1, cus);
      e->ncu = std::max(1, cus);
   }
   if (he != hipSuccess)
   {
      gnoc_destroy(e);
      return GNOC_EHIP;
   }
   *out = e;
   return GNOC_OK;
}

int gnoc_create_sweep(const gnoc_config* base, const gnoc_point* points, int32_t npoints, gnoc_engine** out)
{
   if (!base || !points || !out || npoints < 1) return GNOC_EINVAL;
   *out = nullptr;
   gnoc_config b = *base;
   if (b.mesh_width <= 0 || b.mesh_height <= 0)
   {
      if (b.num_tiles <= 0) return GNOC_EINVAL;
      b.mesh_width = (int32_t) std::floor(std::sqrt((double) b.num_tiles));
      b.mesh_height = (int32_t) std::ceil(1.0 * b.num_tiles / b.mesh_width);
   }
   if (b.num_tiles <= 0) b.num_tiles = b.mesh_width * b.mesh_height;
   if (b.num_tiles != b.mesh_width * b.mesh_height) return GNOC_EINVAL;
   if (b.frequency_ghz != 1.0 || b.max_list_size < 3) return GNOC_EUNSUPPORTED;   // the chunked path
   std::vector<uint64_t> rl((size_t) npoints);
   std::vector<uint32_t> fw((size_t) npoints);
   for (int32_t p = 0; p < npoints; p++)
   {
      const gnoc_point& q = points[p];
      if (q.flit_width <= 0) return GNOC_EINVAL;
      // each point's own link delay identity (emesh_hop_by_hop.cc:126, electrical_link_model.cc:13-16)
      if ((uint64_t) std::ceil(b.frequency_ghz * 0.01 * q.tile_width_mm) != q.link_delay) return GNOC_EINVAL;
      if (q.router_delay + q.link_delay == 0) return GNOC_EINVAL;
      rl[p] = ps_of<true>(q.router_delay + q.link_delay, 1.0);
      fw[p] = (uint32_t) q.flit_width;
   }
   // blocks laid out BX wide, BY high (unused trailing blocks carry no packets)
   int32_t BX = (int32_t) std::ceil(std::sqrt((double) npoints));
   const int32_t BY = (npoints + BX - 1) / BX;
   for (int32_t p = npoints; p < BX * BY; p++) { rl.push_back(rl[0]); fw.push_back(fw[0]); }
   gnoc_config u = b;
   u.mesh_width = BX * b.mesh_width;
   u.mesh_height = BY * b.mesh_height;
   u.num_tiles = u.mesh_width * u.mesh_height;
   u.flit_width = points[0].flit_width;
   u.router_delay = points[0].router_delay;
   u.link_delay = points[0].link_delay;
   u.tile_width_mm = points[0].tile_width_mm;
   gnoc_engine* e = nullptr;
   int rc = gnoc_create(&u, &e);
   if (rc) return rc;
   e->npoints = npoints;
   e->h_pt_rl = rl;
   e->h_pt_fw = fw;
   e->dc.BW = (uint32_t) b.mesh_width;
   e->dc.BH = (uint32_t) b.mesh_height;
   e->dc.BX = (uint32_t) BX;
   hipError_t he = e->d_pt_rl.ensure(rl.size() * 8);
   if (he == hipSuccess) he = e->d_pt_fw.ensure(fw.size() * 4);
   if (he == hipSuccess) he = hipMemcpy(e->d_pt_rl.p, rl.data(), rl.size() * 8, hipMemcpyHostToDevice);
   if (he == hipSuccess) he = hipMemcpy(e->d_pt_fw.p, fw.data(), fw.size() * 4, hipMemcpyHostToDevice);
   if (he != hipSuccess)
   {
      gnoc_destroy(e);
      return GNOC_EHIP;
   }
   e->dc.pt_rl = e->d_pt_rl.as<uint64_t>();
   e->dc.pt_fw = e->d_pt_fw.as<uint32_t>();
   build_static_levels(e);
   he = upload_levels(e);
   if (he != hipSuccess)
   {
      gnoc_destroy(e);
      return GNOC_EHIP;
   }
   *out = e;
   return GNOC_OK;
}

int gnoc_create_hop_counter(const gnoc_config* cfg, gnoc_engine** out)
{
   if (!cfg || !out) return GNOC_EINVAL;
   *out = nullptr;
   gnoc_config c = *cfg;
   // NetworkModelEMeshHopCounter ctor (network_model_emesh_hop_counter.cc:11-41, 50-94)
   if (c.num_tiles <= 0) return GNOC_EINVAL;
   if (c.link_delay != 1) return GNOC_EINVAL;   // :77 LOG_ASSERT_ERROR(link_delay == 1)
   const int32_t w = (int32_t) std::floor(std::sqrt((double) c.num_tiles));
   const int32_t h = (int32_t) std::ceil(1.0 * c.num_tiles / w);
   // the engine's arrays cover the whole w x h grid; tiles >= num_tiles carry no packets
   c.mesh_width = w;
   c.mesh_height = h;
   const int32_t app = c.num_tiles;
   c.num_tiles = w * h;
   c.tile_width_mm = 1.0 / c.frequency_ghz;   // the link identity gnoc_create checks; the hop counter has none
   c.link_delay = (uint64_t) std::ceil(c.frequency_ghz * 0.01 * c.tile_width_mm);
   c.contention_enabled = 0;                   // no queues (:61 "contention is not modeled")
   gnoc_engine* e = nullptr;
   int rc = gnoc_create(&c, &e);
   if (rc) return rc;
   e->dc.Lk = 1;
   e->dc.hop_counter = 1;
   e->cfg.num_tiles = app;
   e->cfg.link_delay = 1;
   *out = e;
   return GNOC_OK;
}

int gnoc_sweep_layout(const gnoc_engine* e, int32_t* blocks_x, int32_t* blocks_y)
{
   if (!e) return GNOC_EINVAL;
   if (blocks_x) *blocks_x = (int32_t) e->dc.BX;
   if (blocks_y) *blocks_y = (int32_t) (e->dc.H / e->dc.BH);
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
   if (e->h_wfill) (void) hipHostFree(e->h_wfill);
   if (e->h_val) (void) hipHostFree(e->h_val);
   if (e->h_nmax) (void) hipHostFree(e->h_nmax);
   for (hipEvent_t ev : e->evpool) (void) hipEventDestroy(ev);
   for (hipStream_t q : { e->s_h2d, e->s_d2h })
      if (q)
      {
         (void) hipStreamSynchronize(q);
         (void) hipStreamDestroy(q);
      }
   for (hipEvent_t ev : { e->ev_h2d, e->ev_done, e->ev_fin, e->ev_alt, e->ch_ev[0][0], e->ch_ev[0][1], e->ch_ev[1][0],
                          e->ch_ev[1][1] })
      if (ev) (void) hipEventDestroy(ev);
   if (e->stream) (void) hipStreamDestroy(e->stream);
   delete e;
}

const char* gnoc_last_error(const gnoc_engine* e) { return e ? e->err.c_str() : "null engine"; }

// Records the batch materialises: one per injection + one per mesh router
// traversal, plus per-slot 64-record alignment.  Route-static, so known at submit.
static uint64_t record_bound(const gnoc_engine* e, uint64_t records)
{
   return records + 64ull * ((uint64_t) e->dc.N * PORTS * INS) + 64;
}


// Chain-engine windows (chain.hip), per phase: D ps with the busiest port's
// expected records per window near CH_FILL of the LDS stream capacity (and its
// inserts within the insert buffer), assuming a steady rate over [0, t_last].
// nW = t_last / D + 1 windows, the last one unbounded.  D = 0: chain off.  After
// each run adapt_windows resizes D from the fullest step the run measured.
static constexpr double CH_FILL = 0.45;     // first run: the steady-rate estimate (bursts reach ~1.7x on the Y phase)
static constexpr double CH_TARGET = 0.95;    // adapted windows: the fullest step at 0.95 of capacity (0.9: 3.94 ms, 0.95: 3.81, 0.98: 3.89 on configs[1]; 1.0 declines the chains)
static constexpr double CH_GROW = 1.6;       // most a chain's window grows per run
static constexpr uint32_t CH_NW_MAX = 4096;
static constexpr float CH_LB_MARGIN = 0.05f;  // look-back replaces the serial hand-off only when > 5% faster
static constexpr uint64_t CH_D_MIN = 1024, CH_D_MAX = 1ull << 31;   // 32-bit time offsets in a window
static constexpr double CH_TARGET_V = 0.85;  // variable windows: each window's predicted fullest step
static constexpr int CH_ADAPT_RUNS = 8;        // variable-window adaptations per batch shape (hotspot: 3 -> 3.21 ms, 8 -> 3.06)
static uint32_t windows_of(uint64_t D, uint64_t t_last) { return (uint32_t) (t_last / D + 1); }
static uint32_t chain_count(const gnoc_engine* e, int p)
{
   return p == 0 ? (e->dc.W > 1 ? 2 * (e->ry1 - e->ry0) : 0u) : (e->dc.H > 1 ? 2 * (e->cx1 - e->cx0) : 0u);
}
// A window length from a target: clamped to the 32-bit time offsets and to at
// most CH_NW_MAX windows; 0 when it cannot fit (chain engine off).
static uint64_t clamp_window(const gnoc_engine* e, double d)
{
   const uint64_t t_last = e->h_tlast;
   uint64_t D = d >= (double) CH_D_MAX ? CH_D_MAX : (uint64_t) d;
   if (D < CH_D_MIN) D = CH_D_MIN;
   if (windows_of(D, t_last) > CH_NW_MAX) D = t_last / (CH_NW_MAX - 1) + 1;
   // a multiple of the boundaries' unit (2^qs ps)
   const uint64_t u = 1ull << e->ch_qs;
   D = std::max(u, (D + u - 1) / u * u);
   return D > CH_D_MAX ? 0 : D;
}
// The windows a chain runs in this attempt: its variable boundaries when they belong to
// the attempt's length, else uniform windows of that length (ps, nW + 1, the last ~0).
static std::vector<uint64_t> chain_bounds(const gnoc_engine* e, int p, size_t c)
{
   if (c < e->chB[p].size() && !e->chB[p][c].empty() && e->chB_D[p][c] == e->chD_run[p][c]) return e->chB[p][c];
   const uint64_t D = e->chD_run[p][c];
   const uint32_t nW = windows_of(D, e->h_tlast);
   std::vector<uint64_t> b(nW + 1);
   for (uint32_t w = 0; w < nW; w++) b[w] = (uint64_t) w * D;
   b[nW] = ~0ull;
   return b;
}
// The identity of the attempt's windows per chain (the device tables, the protocol
// trials and the M/G/1 window limits belong to one): D, or a hash of the boundaries.
static std::vector<uint64_t> win_key(const gnoc_engine* e, int p)
{
   std::vector<uint64_t> k(e->chD_run[p]);
   for (size_t c = 0; c < k.size(); c++)
      if (c < e->chB[p].size() && !e->chB[p][c].empty() && e->chB_D[p][c] == e->chD_run[p][c])
      {
         uint64_t h = 1469598103934665603ull;
         for (uint64_t v : e->chB[p][c]) h = (h ^ v) * 1099511628211ull;
         k[c] = h | (1ull << 63);
      }
   return k;
}
static void choose_windows(gnoc_engine* e, uint64_t port_max, uint64_t ins_max, uint64_t t_last)
{
   // A batch with the same shape as the last one (packets, busiest port, inserts,
   // last injection) keeps the windows the runs of the last one settled on: the
   // windows change only the schedule, never a result.
   const uint64_t key[4] = { (uint64_t) e->n, port_max, ins_max, t_last };
   const bool same = std::equal(key, key + 4, e->ch_key) && e->ch_on && !std::getenv("GNOC_WINDOW_SHIFT") &&
                     !std::getenv("GNOC_WINDOW_PS") && !std::getenv("GNOC_WINDOW_PS_X") && !std::getenv("GNOC_WINDOW_PS_Y");
   std::copy(key, key + 4, e->ch_key);
   if (!same) e->ch_lb_dec[0] = e->ch_lb_dec[1] = -1;
   e->ch_declined = 0;
   e->ch_ydeclined = 0;
   e->exc_fix = 0;
   e->ch_mg = 0;
   e->mgk_ok = 0;
   e->inj_declined = 0;
   if (same) return;
   const char* fv = std::getenv("GNOC_WINDOW_SHIFT");   // test knob: force the window size (2^shift ps)
   const char* pv = std::getenv("GNOC_WINDOW_PS");      // test knob: force the window size (ps)
   const uint64_t span = t_last + 1;
   double d = 1e300;
   if (port_max) d = std::min(d, CH_FILL * ch::CAP * (double) span / (double) port_max);
   if (ins_max) d = std::min(d, CH_FILL * ch::ICAP * (double) span / (double) ins_max);
   if (fv && std::atoi(fv) > 0) d = (double) (1ull << std::atoi(fv));
   if (pv && std::atoll(pv) > 0) d = (double) std::atoll(pv);
   e->h_tlast = t_last;
   e->ch_qs = 0;
   while ((t_last >> e->ch_qs) >= (1ull << 31)) e->ch_qs++;
   {
      const char* v = std::getenv("GNOC_CH_ADAPT_RUNS");
      e->ch_adapt_left = v && *v ? std::max(0, std::atoi(v)) : CH_ADAPT_RUNS;
   }
   const char* px = std::getenv("GNOC_WINDOW_PS_X");    // experiment knobs: one phase's window size
   const char* py = std::getenv("GNOC_WINDOW_PS_Y");
   e->ch_on = true;
   for (int p = 0; p < 2; p++)
   {
      const char* k = p ? py : px;
      const uint64_t D = clamp_window(e, k && std::atoll(k) > 0 ? (double) std::atoll(k) : d);
      if (!D) e->ch_on = false;
      e->chD[p].assign(chain_count(e, p), D);
      e->chCap[p].assign(chain_count(e, p), 0);
      e->chB[p].assign(chain_count(e, p), std::vector<uint64_t>());
      e->chB_D[p].assign(chain_count(e, p), 0);
   }
   e->ch_declined = 0;
}
// After a chain run without retries: per chain, scale D so that its fullest step
// (stream records, inserts) lands near CH_TARGET of the LDS capacity.  Results do
// not depend on D; a window that overflows later retries with that chain's
// windows halved, and the overflowing length caps the chain.
// Variable windows from the run just measured (its per-window fills, k_chain wfill):
// each window's fullest step (stream records, inserts) over its time span gives a
// density; new boundaries are placed so that every window's predicted fullest step
// is CH_TARGET_V of the LDS capacity.  Adopted when a window of the run came close to
// the capacity, or when the new windows are fewer by more than 5%.  True when the
// chain was handled here (its windows were measured).
static bool adapt_chain_variable(gnoc_engine* e, int p, size_t c)
{
   if (!e->h_wfill || c >= e->h_cw[p].size()) return false;
   const ChainWin& cw = e->h_cw[p][c];
   const uint32_t nW = cw.nW;
   if (!nW || cw.wt_off + nW >= e->h_wt.size()) return false;
   const uint32_t qs = e->ch_qs;
   const uint64_t tl = e->h_tlast + 1;
   std::vector<uint64_t> b(nW + 1);
   for (uint32_t w = 0; w < nW; w++) b[w] = (uint64_t) e->h_wt[cw.wt_off + w] << qs;
   b[nW] = std::max(tl, b[nW - 1] + 1);   // (the last window's span: up to the last injection)
   std::vector<double> rn(nW), ri(nW);
   uint32_t mx = 0;
   for (uint32_t w = 0; w < nW; w++)
   {
      const uint32_t f = e->h_wfill[cw.wt_off + w];
      const uint32_t n = f & 0xFFFFu, ni = f >> 16;
      mx = std::max(mx, n);
      const double len = (double) std::max<uint64_t>(b[w + 1] - b[w], 1);
      rn[w] = (double) std::max(n, 1u) / len;
      ri[w] = (double) ni / len;
   }
   static const double tv = [] {
      const char* v = std::getenv("GNOC_CH_TARGET_V");
      const double x = v && *v ? std::atof(v) : CH_TARGET_V;
      return x > 0.5 && x < 1.0 ? x : CH_TARGET_V;
   }();
   const double tn = tv * ch::CAP, ti = tv * ch::ICAP;
   const uint64_t u = 1ull << qs;
   const uint64_t dmin = std::max(u, (CH_D_MIN + u - 1) / u * u), dmax = CH_D_MAX / u * u;
   std::vector<uint64_t> nb{ 0 };
   uint64_t s0 = 0, dlong = 0;
   uint32_t w = 0;
   for (;;)
   {
      // extend the window from s0 through the old windows' densities
      double an = 0, ai = 0;
      uint64_t t = s0, e1 = ~0ull;
      while (w < nW && b[w + 1] <= t) w++;
      for (uint32_t k = w; k < nW; k++)
      {
         const uint64_t lo = std::max(t, b[k]), hi = b[k + 1];
         double room = rn[k] > 0 ? (tn - an) / rn[k] : 1e300;
         if (ri[k] > 0) room = std::min(room, (ti - ai) / ri[k]);
         if ((double) lo + room < (double) hi)
         {
            e1 = lo + (uint64_t) std::max(room, 0.0);
            break;
         }
         an += rn[k] * (double) (hi - lo);
         ai += ri[k] * (double) (hi - lo);
      }
      // (at most CH_GROW times the run's window there: bursts it did not see)
      const uint64_t grow = (uint64_t) (CH_GROW * (double) (b[std::min(w, nW - 1) + 1] - b[std::min(w, nW - 1)]));
      if (e1 > s0 + grow) e1 = s0 + grow;   // (also where the target is not reached before the end)
      if (e1 == ~0ull || e1 >= tl) break;   // the rest is the last window
      uint64_t len = e1 > s0 ? (e1 - s0) / u * u : 0;
      len = std::min(std::max(len, dmin), dmax);
      s0 += len;
      if (s0 >= tl) break;
      nb.push_back(s0);
      dlong = std::max(dlong, len);
      if (nb.size() > std::min<size_t>(CH_NW_MAX, ch::IJ_NWB - 1)) return true;   // too many: keep the run's windows
   }
   nb.push_back(~0ull);
   const uint32_t nWn = (uint32_t) nb.size() - 1;
   const bool hot = mx > 0.97 * ch::CAP;
   if (std::getenv("GNOC_CHAIN_DEBUG") && nW <= 40)
   {
      std::fprintf(stderr, "gnoc: adapt phase %d chain %zu: %u windows ->", p, c, nW);
      for (uint32_t k = 0; k < nW; k++)
         std::fprintf(stderr, " [%llu %u/%u]", (unsigned long long) b[k], e->h_wfill[cw.wt_off + k] & 0xFFFFu,
                      e->h_wfill[cw.wt_off + k] >> 16);
      std::fprintf(stderr, "\n   new %u:", nWn);
      for (uint32_t k = 0; k < nWn; k++) std::fprintf(stderr, " %llu", (unsigned long long) nb[k]);
      std::fprintf(stderr, "\n");
   }
   if (!hot && nWn * 100 > nW * 95) return true;   // close enough: no churn
   e->chB[p][c] = nb;
   e->chD[p][c] = std::max(dlong, dmin);
   e->chB_D[p][c] = e->chD[p][c];
   return true;
}
static void adapt_windows(gnoc_engine* e)
{
   if (std::getenv("GNOC_WINDOW_SHIFT") || std::getenv("GNOC_WINDOW_PS") || std::getenv("GNOC_WINDOW_PS_X") ||
       std::getenv("GNOC_WINDOW_PS_Y"))
      return;
   const char* vv = std::getenv("GNOC_CH_VARWIN");   // 0: uniform windows per chain only
   const bool var = e->ch_adapt_left > 0 && e->ch_wfill_read && !(vv && *vv && std::atoi(vv) == 0);
   if (e->ch_adapt_left > 0) e->ch_adapt_left--;
   const unsigned* nm = e->h_nmax;
   for (int p = 0; p < 2; p++)
   {
      for (size_t c = 0; c < e->chD[p].size(); c++)
      {
         if (var && adapt_chain_variable(e, p, c)) continue;
         // (a chain on variable windows keeps them once they settled)
         if (c < e->chB[p].size() && !e->chB[p][c].empty() && e->chB_D[p][c] == e->chD[p][c]) continue;
         const unsigned n = nm[2 * c], ni = nm[2 * c + 1];
         if (!n || n == 0xFFFFFFFFu) continue;
         double r = CH_TARGET * ch::CAP / (double) n;
         if (ni) r = std::min(r, 0.95 * ch::ICAP / (double) ni);   // inserts are few: only keep them in the buffer
         if (r > 0.92 && r < 1.08) continue;                        // close enough: no churn
         r = std::min(r, CH_GROW);                                   // bursts the last run did not see: grow in steps
         double d = (double) e->chD[p][c] * r;
         if (e->chCap[p][c]) d = std::min(d, 0.95 * (double) e->chCap[p][c]);   // stay below a size that overflowed
         const uint64_t D = clamp_window(e, d);
         if (D) e->chD[p][c] = D;
      }
      nm += 2 * e->chD[p].size();
   }
}
// After a run that overflowed LDS: halve the windows (in D) of the chains the
// kernel marked (all chains when none is marked) and cap them at the length that
// overflowed.  False when a halved window would leave the allowed range.
static bool halve_overflowed(gnoc_engine* e, std::vector<uint64_t>* D)
{
   bool any = false, ok = true;
   const unsigned* nm = e->h_nmax;
   for (int p = 0; p < 2; p++)
   {
      for (size_t c = 0; c < D[p].size(); c++) any |= nm[2 * c] == 0xFFFFFFFFu;
      nm += 2 * D[p].size();
   }
   nm = e->h_nmax;
   for (int p = 0; p < 2; p++)
   {
      for (size_t c = 0; c < D[p].size(); c++)
      {
         if (any && nm[2 * c] != 0xFFFFFFFFu) continue;
         uint64_t& d = D[p][c];
         if (c < e->chB[p].size() && !e->chB[p][c].empty() && e->chB_D[p][c] == d)
         {
            // variable windows: each one split in two (the chain keeps its shape)
            const std::vector<uint64_t>& b = e->chB[p][c];
            const uint64_t u = 1ull << e->ch_qs;
            std::vector<uint64_t> nb;
            for (size_t w = 0; w + 1 < b.size(); w++)
            {
               nb.push_back(b[w]);
               const uint64_t hi = w + 2 < b.size() ? b[w + 1] : std::max<uint64_t>(b[w] + 2 * u, e->h_tlast + 1);
               const uint64_t mid = b[w] + (hi - b[w]) / 2 / u * u;
               if (mid > b[w] && mid < hi && (w + 2 < b.size() || mid <= e->h_tlast)) nb.push_back(mid);
            }
            nb.push_back(~0ull);
            if (nb.size() - 1 > std::min<size_t>(CH_NW_MAX, ch::IJ_NWB - 1) || d < 2 * CH_D_MIN) ok = false;
            else
            {
               e->chB[p][c] = nb;
               d /= 2;
               e->chB_D[p][c] = d;
            }
            continue;
         }
         if (!e->chCap[p][c] || d < e->chCap[p][c]) e->chCap[p][c] = d;
         if (d < 2 * CH_D_MIN || 2ull * windows_of(d, e->h_tlast) > CH_NW_MAX) ok = false;
         else d /= 2;
      }
      nm += 2 * D[p].size();
   }
   return ok;
}

// The device tables of the attempt's windows (chD_run): per chain its windows,
// state and bounds blocks; the tasks of each phase in window start-time order
// (so a task's predecessor, same chain and window - 1, is always handed out
// first).  Rebuilt only when the lengths change.
// XCD-local queues (chain.hip deq_init): on by default for a grid that covers every XCD
// many times over; GNOC_CH_XCD=0 keeps the one shared queue per phase.
static bool chain_xcd(const gnoc_engine* e)
{
   const char* v = std::getenv("GNOC_CH_XCD");
   if (v && *v && std::atoi(v) == 0) return false;
   return !e->ch_xcd_off && e->ch_grid >= 64 * (int) ch::NQ;
}
static int chain_tables(gnoc_engine* e)
{
   const int xcd = chain_xcd(e) ? 1 : 0;
   const std::vector<uint64_t> key[2] = { win_key(e, 0), win_key(e, 1) };
   if (e->chD_up[0] == key[0] && e->chD_up[1] == key[1] && e->ch_cw.p && e->ch_xcd_tab == xcd) return GNOC_OK;
   e->ch_xcd_tab = xcd;
   const uint32_t lens[2] = { e->dc.W - 1, e->dc.H - 1 }, nls[2] = { 1u, 3u };
   std::vector<std::pair<uint64_t, uint32_t>> order;
   e->h_wt.clear();
   for (int p = 0; p < 2; p++)
   {
      auto& cw = e->h_cw[p];
      cw.assign(e->chD_run[p].size(), ChainWin{});
      uint64_t st = 0, bt = 0;
      order.clear();
      for (size_t c = 0; c < cw.size(); c++)
      {
         // the chain's windows, [b[w], b[w + 1]), the last one unbounded
         const std::vector<uint64_t> b = chain_bounds(e, p, c);
         const uint32_t nW = (uint32_t) b.size() - 1;
         uint64_t dlong = e->chD_run[p][c];
         for (uint32_t w = 0; w + 1 < nW; w++) dlong = std::max(dlong, b[w + 1] - b[w]);
         cw[c].D = dlong;
         cw[c].nW = nW;
         cw[c].st_off = st;
         cw[c].bt_off = bt;
         cw[c].wt_off = e->h_wt.size();
         cw[c].pad = 0;
         for (uint32_t w = 0; w < nW; w++) e->h_wt.push_back((uint32_t) (b[w] >> e->ch_qs));
         e->h_wt.push_back(0xFFFFFFFFu);
         st += (uint64_t) lens[p] * nW * ch::SW;
         bt += (uint64_t) lens[p] * nls[p] * (nW + 1);
         for (uint32_t w = 0; w < nW; w++) order.push_back({ b[w], (uint32_t) (c << 16) | w });
      }
      std::stable_sort(order.begin(), order.end(),
                       [](const std::pair<uint64_t, uint32_t>& x, const std::pair<uint64_t, uint32_t>& y) { return x.first < y.first; });
      // the chains over the queues: longest processing time first by window count (a
      // window costs about the same on every chain: each is sized to the same fill)
      std::vector<uint32_t> qof(cw.size(), 0);
      const uint32_t nq = xcd ? ch::NQ : 1u;
      {
         std::vector<uint32_t> byw(cw.size());
         for (size_t c = 0; c < cw.size(); c++) byw[c] = (uint32_t) c;
         std::stable_sort(byw.begin(), byw.end(), [&](uint32_t x, uint32_t y) { return cw[x].nW > cw[y].nW; });
         std::vector<uint64_t> load(nq, 0);
         for (uint32_t c : byw)
         {
            const uint32_t q = (uint32_t) (std::min_element(load.begin(), load.end()) - load.begin());
            qof[c] = q;
            load[q] += cw[c].nW;
         }
      }
      e->h_tasks[p].clear();
      e->h_tasks[p].reserve(order.size());
      e->h_qoff[p].assign(ch::NQ + 1, 0);
      for (uint32_t q = 0; q < nq; q++)
      {
         e->h_qoff[p][q] = (uint32_t) e->h_tasks[p].size();
         for (const auto& o : order)
            if (qof[o.second >> 16] == q) e->h_tasks[p].push_back(o.second);
      }
      for (uint32_t q = nq; q <= ch::NQ; q++) e->h_qoff[p][q] = (uint32_t) e->h_tasks[p].size();
      e->ch_st_words[p] = st;
      e->ch_bt_words[p] = bt;
   }
   const size_t ncw = e->h_cw[0].size() + e->h_cw[1].size(), nt = e->h_tasks[0].size() + e->h_tasks[1].size();
   GNOC_HIP(e, e->ch_cw.ensure(std::max<size_t>(ncw, 1) * sizeof(ChainWin)));
   GNOC_HIP(e, e->ch_tasks.ensure((std::max<size_t>(nt, 1) + 2 * (ch::NQ + 1)) * 4));
   GNOC_HIP(e, hipMemcpy(e->ch_cw.p, e->h_cw[0].data(), e->h_cw[0].size() * sizeof(ChainWin), hipMemcpyHostToDevice));
   GNOC_HIP(e, hipMemcpy(e->ch_cw.as<ChainWin>() + e->h_cw[0].size(), e->h_cw[1].data(), e->h_cw[1].size() * sizeof(ChainWin),
                         hipMemcpyHostToDevice));
   GNOC_HIP(e, hipMemcpy(e->ch_tasks.p, e->h_tasks[0].data(), e->h_tasks[0].size() * 4, hipMemcpyHostToDevice));
   GNOC_HIP(e, hipMemcpy(e->ch_tasks.as<uint32_t>() + e->h_tasks[0].size(), e->h_tasks[1].data(), e->h_tasks[1].size() * 4,
                         hipMemcpyHostToDevice));
   for (int p = 0; p < 2; p++)
      GNOC_HIP(e, hipMemcpy(e->ch_tasks.as<uint32_t>() + nt + p * (ch::NQ + 1), e->h_qoff[p].data(), (ch::NQ + 1) * 4,
                            hipMemcpyHostToDevice));
   // window boundaries, and the per-window fills the runs report (read back while the
   // windows still adapt)
   GNOC_HIP(e, e->ch_wt.ensure(std::max<size_t>(e->h_wt.size(), 1) * 4));
   GNOC_HIP(e, e->ch_wfill.ensure(std::max<size_t>(e->h_wt.size(), 1) * 4));
   GNOC_HIP(e, hipMemcpy(e->ch_wt.p, e->h_wt.data(), e->h_wt.size() * 4, hipMemcpyHostToDevice));
   if (e->h_wfill_cap < e->h_wt.size())
   {
      if (e->h_wfill) (void) hipHostFree(e->h_wfill);
      e->h_wfill = nullptr;
      e->h_wfill_cap = 0;
      GNOC_HIP(e, hipHostMalloc((void**) &e->h_wfill, e->h_wt.size() * 4, hipHostMallocDefault));
      e->h_wfill_cap = e->h_wt.size();
   }
   e->chD_up[0] = key[0];
   e->chD_up[1] = key[1];
   return GNOC_OK;
}

// The submitted trace's contract checks and statistics, on the device
// (prep.hip k_validate over e->d_*): the first offending packet of any check,
// the hop records this engine materialises, the turn exchange counts of a
// sharded engine, and the chain engine's window size from the busiest port.
__global__ void k_pk_check(const uint64_t* __restrict__ esc, uint64_t n_abs, unsigned long long* __restrict__ bad);
// The trace arrays a validation reads (the current batch's, or a staged one's).
struct ValTrace
{
   const uint64_t* inj;
   const uint32_t *src, *dst, *bits, *flags;
};
static int validate_finish(gnoc_engine* e, const void* h_out, uint64_t* records, uint64_t* nbc);
// The device-side checks and statistics of a batch, enqueued on stream s into the
// scratch vb; the ValOut summary lands in the pinned h_out (validate_finish reads it
// once the stream got there).  xcnt (the exchange counts) stays in vb.
static int validate_launch(gnoc_engine* e, size_t n, ValTrace t, hipStream_t s, DevBuf& vb, void* h_out,
                           unsigned long long** xcnt_out)
{
   const uint32_t N = e->dc.N, W = e->dc.W, H = e->dc.H, nr = (uint32_t) e->nranks;
   const size_t nd = (size_t) 2 * H * (W + 1) + (size_t) 2 * W * (H + 1);   // difference arrays (int)
   const size_t ni = (size_t) 4 * N;                                       // inserts per X / Y port
   const size_t off_x = (sizeof(ValOut) + (nd + ni) * 4 + 7) / 8 * 8;
   // block-private statistics in LDS when the table (+ the turn counts) fits a
   // CU's LDS: nblk partial tables behind the turn counts, summed by k_validate_sum
   const uint32_t ntab = (uint32_t) (nd + ni);
   const size_t lds = ((size_t) ntab + (size_t) nr * nr) * 4;
   const bool lh = n && lds <= 150 * 1024;
   const uint32_t nblk = lh ? (uint32_t) std::min<uint64_t>((n + 4095) / 4096, lds <= 64 * 1024 ? 512 : 256) : 0;
   const size_t off_p = (off_x + (size_t) nr * nr * 8 + 255) / 256 * 256;
   const size_t bytes = off_p + (size_t) nblk * ntab * 4;
   static_assert(sizeof(ValOut) <= 128, "ValOut lands in the 128-B pinned staging");
   GNOC_HIP(e, vb.ensure(bytes));
   GNOC_HIP(e, hipMemsetAsync(vb.p, 0, off_p, s));
   GNOC_HIP(e, hipMemsetAsync(vb.p, 0xFF, sizeof(unsigned long long) * VB_KINDS, s));
   char* base = static_cast<char*>(vb.p);
   ValOut* vo = reinterpret_cast<ValOut*>(base);
   int* dxr = reinterpret_cast<int*>(base + sizeof(ValOut));
   int* dxl = dxr + (size_t) H * (W + 1);
   int* dyu = dxl + (size_t) H * (W + 1);
   int* dyd = dyu + (size_t) W * (H + 1);
   uint32_t* insx = reinterpret_cast<uint32_t*>(dyd + (size_t) W * (H + 1));
   uint32_t* insy = insx + 2 * (size_t) N;
   unsigned long long* xcnt = reinterpret_cast<unsigned long long*>(base + off_x);
   int* part = reinterpret_cast<int*>(base + off_p);
   if (n)
   {
      const int tree = e->cfg.broadcast_tree_enabled && !e->dc.hop_counter;
      const uint32_t sweep = e->npoints > 1 ? 1u : 0u;
      if (lh)
      {
         if (lds > 64 * 1024)
            GNOC_HIP(e, hipFuncSetAttribute(reinterpret_cast<const void*>(&k_validate<true>),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds));
         hipLaunchKernelGGL(k_validate<true>, dim3(nblk), dim3(256), lds, s, e->dc, (uint64_t) n, t.inj, t.src,
                            t.dst, t.bits, t.flags, tree, sweep, nr, (uint32_t) e->rank, (uint32_t) e->xself, vo, dxr, ntab, part, xcnt);
         GNOC_HIP(e, hipGetLastError());
         hipLaunchKernelGGL(k_validate_sum, dim3((ntab + 255) / 256), dim3(256), 0, s, ntab, nblk, part, dxr);
      }
      else
      {
         const uint32_t grid = (uint32_t) std::min<uint64_t>((n + 255) / 256, 4096);
         hipLaunchKernelGGL(k_validate<false>, dim3(grid), dim3(256), 0, s, e->dc, (uint64_t) n, t.inj, t.src,
                            t.dst, t.bits, t.flags, tree, sweep, nr, (uint32_t) e->rank, (uint32_t) e->xself, vo, dxr, ntab, part, xcnt);
      }
      GNOC_HIP(e, hipGetLastError());
      hipLaunchKernelGGL(k_validate_max, dim3(1), dim3(1024), 0, s, W, H, dxr, dxl, dyu, dyd, insx, insy, vo);
      GNOC_HIP(e, hipGetLastError());
   }
   if (e->val_esc)
   {
      hipLaunchKernelGGL(k_pk_check, dim3(1), dim3(1), 0, s, e->val_esc, e->val_nabs, &vo->bad[VB_PACKED]);
      GNOC_HIP(e, hipGetLastError());
      e->val_esc = nullptr;
   }
   GNOC_HIP(e, hipMemcpyAsync(h_out, vo, sizeof(ValOut), hipMemcpyDeviceToHost, s));
   if (xcnt_out) *xcnt_out = xcnt;
   return GNOC_OK;
}
static int device_validate(gnoc_engine* e, size_t n, uint64_t* records, uint64_t* nbc)
{
   const uint32_t nr = (uint32_t) e->nranks;
   hipStream_t s = e->stream;
   unsigned long long* xcnt = nullptr;
   int rc = validate_launch(e, n, ValTrace{ e->d_inj, e->d_src, e->d_dst, e->d_bits, e->d_flags }, s, e->vbuf, e->h_pinned, &xcnt);
   if (rc) return rc;
   e->x_cnt.assign((size_t) nr * nr, 0);
   if (nr > 1 || e->xself) GNOC_HIP(e, hipMemcpyAsync(e->x_cnt.data(), xcnt, (size_t) nr * nr * 8, hipMemcpyDeviceToHost, s));
   GNOC_HIP(e, hipStreamSynchronize(s));
   return validate_finish(e, e->h_pinned, records, nbc);
}
// The host side of a validation: the first offending packet, or the batch's window
// sizing and record bound.
static int validate_finish(gnoc_engine* e, const void* h_out, uint64_t* records, uint64_t* nbc)
{
   ValOut v;
   std::memcpy(&v, h_out, sizeof v);
   // the first offending packet (one check per packet: the first that fails)
   uint32_t k = VB_KINDS;
   for (uint32_t q = 0; q < VB_KINDS; q++)
      if (v.bad[q] != ~0ull && (k == VB_KINDS || v.bad[q] < v.bad[k])) k = q;
   if (k != VB_KINDS)
   {
      const std::string at = std::to_string(e->part && v.bad[k] < e->h_gid.size() ? (uint64_t) e->h_gid[v.bad[k]] : v.bad[k]);
      switch (k)
      {
         case VB_TILE: return fail(e, GNOC_ETRACE, "tile id out of range at packet " + at);
         case VB_BC_TREE:
            // Network::netSend sends one packet per tile when the model has no broadcast
            // capability (network.cc:186-195): the caller expands those.
            return fail(e, GNOC_EINVAL, "broadcast packet " + at +
                                            " but the model has no broadcast tree (the caller expands it, network.cc:186-195)");
         case VB_BC_SHARD: return fail(e, GNOC_EUNSUPPORTED, "broadcast packets on a sharded or sweep engine");
         case VB_ORDER: return fail(e, GNOC_ETRACE, "trace not ordered by inject_ps at packet " + at);
         case VB_SWEEP: return fail(e, GNOC_ETRACE, "sweep packet crosses sweep points at packet " + at);
         case VB_ZERO_F: return fail(e, GNOC_ETRACE, "zero-flit packet " + at);
         case VB_F_MAX: return fail(e, GNOC_EUNSUPPORTED, "packet longer than 2047 flits (packet " + at + ")");
         case VB_PACKED: return fail(e, GNOC_ETRACE, "packed trace: the dt escapes (0xFFFF) do not match n_abs");
         default: return fail(e, GNOC_EUNSUPPORTED, "inject time beyond 2^50 ps at packet " + at);
      }
   }
   choose_windows(e, v.pmax, v.imax, v.tlast);   // (an empty batch: all zero)
   *records = v.records;
   *nbc = v.nbc;
   return GNOC_OK;
}

// Send / receive layouts of the turn exchange (shard.hip), from x_cnt.
static int build_exchange(gnoc_engine* e)
{
   const uint32_t nr = (uint32_t) e->nranks, me = (uint32_t) e->rank, W = e->dc.W, H = e->dc.H;
   e->xs_pairs.clear();
   e->xr_pairs.clear();
   e->xs_units.assign(nr, 0);
   e->xr_units.assign(nr, 0);
   e->xs_slots = e->xr_slots = 0;
   if ((nr <= 1 && !e->xself) || !e->dc.contention) return GNOC_OK;
   uint64_t su = 0, ru = 0;
   for (uint32_t q = 0; q < nr; q++)
   {
      // a rank's own turn records stay in place, except under the self-exchange test
      // knob, which sends them to itself (through the transport) and back into the slots
      if (q == me && !e->xself) continue;
      for (int side = 0; side < 2; side++)
      {
         // side 0: my rows -> q's columns (send); side 1: q's rows -> my columns (receive)
         const uint32_t rr = side ? q : me, cc = side ? me : q;
         XPair p{};
         p.x0 = band_lo(cc, nr, W);
         p.nx = band_lo(cc + 1, nr, W) - p.x0;
         p.y0 = band_lo(rr, nr, H);
         p.ny = band_lo(rr + 1, nr, H) - p.y0;
         p.nslots = p.nx * p.ny * XS_PER_TILE;
         p.expect = e->x_cnt[(size_t) rr * nr + cc];
         const uint64_t hdr = 1 + (p.nslots + 3) / 4;   // status unit + exception counts (shard.hip)
         uint64_t& u = side ? ru : su;
         p.hdr_unit = u;
         p.rec_unit = u + hdr;
         u += hdr + p.expect;
         (side ? e->xr_units : e->xs_units)[q] = hdr + p.expect;
         p.slot0 = side ? e->xr_slots : e->xs_slots;
         (side ? e->xr_slots : e->xs_slots) += p.nslots;
         (side ? e->xr_pairs : e->xs_pairs).push_back(p);
      }
   }
   GNOC_HIP(e, e->d_xs_pairs.ensure(e->xs_pairs.size() * sizeof(XPair)));
   GNOC_HIP(e, e->d_xr_pairs.ensure(e->xr_pairs.size() * sizeof(XPair)));
   GNOC_HIP(e, hipMemcpy(e->d_xs_pairs.p, e->xs_pairs.data(), e->xs_pairs.size() * sizeof(XPair), hipMemcpyHostToDevice));
   GNOC_HIP(e, hipMemcpy(e->d_xr_pairs.p, e->xr_pairs.data(), e->xr_pairs.size() * sizeof(XPair), hipMemcpyHostToDevice));
   GNOC_HIP(e, e->xs_off.ensure((size_t) e->xs_slots * 8));
   GNOC_HIP(e, e->xr_off.ensure((size_t) e->xr_slots * 8));
   return GNOC_OK;
}

// Broadcast tables of the submitted trace (h_bid from validate_host_trace).
static int upload_broadcasts(gnoc_engine* e)
{
   e->nb = (uint32_t) e->h_bid.size();
   e->dc.bc_idx = nullptr;
   e->dc.bc_prev = nullptr;
   e->dc.bc_cur = nullptr;
   e->dc.bc_fin = nullptr;
   if (!e->nb) return GNOC_OK;
   const size_t nv = (size_t) e->nb * e->dc.N;
   std::vector<uint32_t> bidx(e->n, 0xFFFFFFFFu);
   for (uint32_t b = 0; b < e->nb; b++) bidx[e->h_bid[b]] = b;
   GNOC_HIP(e, e->d_bidx.ensure(e->n * 4));
   GNOC_HIP(e, e->d_bid.ensure((size_t) e->nb * 4));
   GNOC_HIP(e, e->d_bv[0].ensure(nv * 8 * BCS));
   GNOC_HIP(e, e->d_bv[1].ensure(nv * 8 * BCS));
   GNOC_HIP(e, e->d_bfin.ensure(nv * 8));
   GNOC_HIP(e, e->d_bzl.ensure(nv * 8));
   GNOC_HIP(e, e->d_bct.ensure(nv * 8));
   GNOC_HIP(e, e->d_bflag.ensure(16));
   GNOC_HIP(e, hipMemcpy(e->d_bidx.p, bidx.data(), e->n * 4, hipMemcpyHostToDevice));
   GNOC_HIP(e, hipMemcpy(e->d_bid.p, e->h_bid.data(), (size_t) e->nb * 4, hipMemcpyHostToDevice));
   e->dc.bc_idx = e->d_bidx.as<uint32_t>();
   e->dc.bc_prev = e->d_bv[0].as<uint64_t>();
   e->dc.bc_cur = e->d_bv[1].as<uint64_t>();
   e->dc.bc_fin = e->d_bfin.as<uint64_t>();
   return GNOC_OK;
}

// The per-run zeroing of counters, slot counts, exception counts and port counters
// in one launch (segment = blockIdx.y) instead of one fill per buffer.  Segment 0
// is the counter block: with broadcasts its word 10 (errflag[2], "slots have
// tails") starts at 1.
constexpr int ZSEG = 10;
struct ZeroSegs
{
   uint32_t* p[ZSEG];
   uint64_t nw[ZSEG];
};
__global__ __launch_bounds__(256) void k_zero_segs(ZeroSegs z, uint32_t w10)
{
   uint32_t* const p = z.p[blockIdx.y];
   const uint64_t n = z.nw[blockIdx.y];
   for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x)
      p[i] = (blockIdx.y == 0 && i == 10) ? w10 : 0u;
}



// A sharded rank keeps only the packets it touches: sources in its row band
// (injection, X phase, turn) or destinations in its column band (Y phase, SELF,
// the results it delivers).  The contract checks a rank could miss on its subset
// (tile range, order) run here over the whole trace; the totals the summary
// reports are the whole mesh's.  Row / column band prep (W, H <= 64) only.
static int partition_trace(gnoc_engine* e, const gnoc_packets* pk, size_t n, gnoc_packets* sub,
                           std::vector<uint64_t>& inj, std::vector<uint32_t>& src, std::vector<uint32_t>& dst,
                           std::vector<uint32_t>& bits, std::vector<uint32_t>& flags)
{
   const uint32_t N = e->dc.N, W = e->dc.W;
   uint64_t hops = 0, routed = 0;
   e->h_gid.clear();
   for (size_t i = 0; i < n; i++)
   {
      const uint32_t s = pk->src[i], d = pk->dst[i], fl = pk->flags ? pk->flags[i] : 0u;
      if (fl & GNOC_PKT_BROADCAST) return fail(e, GNOC_EUNSUPPORTED, "broadcast packets on a sharded or sweep engine");
      if (s >= N || d >= N) return fail(e, GNOC_ETRACE, "tile id out of range at packet " + std::to_string(i));
      if (i && pk->inject_ps[i] < pk->inject_ps[i - 1])
         return fail(e, GNOC_ETRACE, "trace not ordered by inject_ps at packet " + std::to_string(i));
      // the rest of k_validate's per-packet contract, in its order: every rank checks
      // the whole trace, so a bad packet fails gnoc_submit on every rank alike (a rank
      // would otherwise see only the packets it keeps)
      const uint32_t fw = e->dc.flit_width, b = pk->bits[i];
      const uint32_t F = (b % fw) ? b / fw + 1 : b / fw;
      const bool bypass = s == d || (fl & GNOC_PKT_UNMODELED);
      if (F == 0 && !bypass) return fail(e, GNOC_ETRACE, "zero-flit packet " + std::to_string(i));
      if (F > AUX_F_MAX) return fail(e, GNOC_EUNSUPPORTED, "packet longer than 2047 flits (packet " + std::to_string(i) + ")");
      if (pk->inject_ps[i] >= (1ull << 50))
         return fail(e, GNOC_EUNSUPPORTED, "inject time beyond 2^50 ps at packet " + std::to_string(i));
      const uint32_t sx = s % W, sy = s / W, dx = d % W, dy = d / W;
      if (s != d && !(fl & GNOC_PKT_UNMODELED))
      {
         routed++;
         hops += (sx > dx ? sx - dx : dx - sx) + (sy > dy ? sy - dy : dy - sy) + 1;
      }
      if ((sy >= e->ry0 && sy < e->ry1) || (dx >= e->cx0 && dx < e->cx1)) e->h_gid.push_back((uint32_t) i);
   }
   const size_t m = e->h_gid.size();
   inj.resize(m);
   src.resize(m);
   dst.resize(m);
   bits.resize(m);
   flags.resize(m);
   for (size_t k = 0; k < m; k++)
   {
      const size_t i = e->h_gid[k];
      inj[k] = pk->inject_ps[i];
      src[k] = pk->src[i];
      dst[k] = pk->dst[i];
      bits[k] = pk->bits[i];
      flags[k] = pk->flags ? pk->flags[i] : 0u;
   }
   sub->inject_ps = inj.data();
   sub->src = src.data();
   sub->dst = dst.data();
   sub->bits = bits.data();
   sub->flags = flags.data();
   e->h_glob_hops = hops;
   e->h_glob_routed = routed;
   return GNOC_OK;
}

static int submit_tail(gnoc_engine* e, const gnoc_packets* pk, size_t n, bool prevalidated = false);

// Narrow wire format -> the engine's u32 trace arrays (one pass, coalesced).
__global__ __launch_bounds__(256) void k_widen(uint64_t n, const uint16_t* __restrict__ src, const uint16_t* __restrict__ dst,
                                               const uint16_t* __restrict__ bits, const uint8_t* __restrict__ flags,
                                               uint32_t* __restrict__ osrc, uint32_t* __restrict__ odst,
                                               uint32_t* __restrict__ obits, uint32_t* __restrict__ oflags)
{
   for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x)
   {
      osrc[i] = src[i];
      odst[i] = dst[i];
      obits[i] = bits[i];
      oflags[i] = flags ? flags[i] : 0u;
   }
}

// Delta wire format (gnoc_packets_packed) -> the engine's trace arrays.  Blocks of
// PK_B packets, PK_PT consecutive ones per thread.  k_dt_block: each block's escapes
// (dt == 0xFFFF) and its difference sum after the last one; k_dt_carry (one
// workgroup): the escapes before each block and the inject time before its first
// packet, by a segmented scan of the block aggregates (an escape restarts the sum
// at its absolute time); k_dt_unpack: the same inside each block, writing inject_ps
// and widening the other fields.
constexpr uint32_t PK_T = 256, PK_PT = 8, PK_B = PK_T * PK_PT;
constexpr uint16_t PK_ESC = 0xFFFF;
struct PkAgg
{
   uint64_t tail;    // the differences after the last escape (all of them without one)
   uint32_t nesc;
   uint32_t pad;
};
// Segmented inclusive scan over a workgroup of (restart, value) pairs in LDS.
__device__ __forceinline__ void seg_scan(uint32_t* fl, uint64_t* va, uint32_t tid, uint32_t nt)
{
   for (uint32_t d = 1; d < nt; d <<= 1)
   {
      uint32_t f = 0;
      uint64_t v = 0;
      const bool take = tid >= d;
      if (take)
      {
         f = fl[tid - d];
         v = va[tid - d];
      }
      __syncthreads();
      if (take && !fl[tid])
      {
         fl[tid] = f;
         va[tid] += v;
      }
      __syncthreads();
   }
}
__global__ __launch_bounds__(PK_T) void k_dt_block(uint64_t n, const uint16_t* __restrict__ dt, PkAgg* __restrict__ agg)
{
   __shared__ uint32_t fl[PK_T], ne[PK_T];
   __shared__ uint64_t va[PK_T];
   __shared__ uint16_t sd[PK_B];
   const uint32_t tid = threadIdx.x;
   const uint64_t b0 = (uint64_t) blockIdx.x * PK_B;
   // the block's differences through LDS (coalesced), then each thread's PK_PT
   // consecutive ones
#pragma unroll
   for (uint32_t k = 0; k < PK_PT; k++)
   {
      const uint64_t i = b0 + k * PK_T + tid;
      sd[k * PK_T + tid] = i < n ? dt[i] : (uint16_t) 0;
   }
   __syncthreads();
   const uint64_t i0 = b0 + (uint64_t) tid * PK_PT;
   uint32_t f = 0, c = 0;
   uint64_t v = 0;
   for (uint32_t k = 0; k < PK_PT; k++)
   {
      if (i0 + k >= n) break;
      const uint16_t d = sd[tid * PK_PT + k];
      if (d == PK_ESC)
      {
         f = 1;
         v = 0;
         c++;
      }
      else v += d;
   }
   fl[tid] = f;
   va[tid] = v;
   ne[tid] = c;
   __syncthreads();
   seg_scan(fl, va, tid, PK_T);
   if (tid == 0)
   {
      uint32_t t = 0;
      for (uint32_t q = 0; q < PK_T; q++) t += ne[q];
      agg[blockIdx.x] = PkAgg{ va[PK_T - 1], t, fl[PK_T - 1] };
   }
}
// An escape ordinal past the caller's n_abs absolute times reads 0 (never past the
// array); k_pk_check reports the mismatch of escape count and n_abs as a bad batch.
__device__ __forceinline__ uint64_t pk_abs(const uint64_t* __restrict__ abs_ps, uint64_t n_abs, uint64_t i)
{
   return i < n_abs ? abs_ps[i] : 0ull;
}
__global__ __launch_bounds__(1024) void k_dt_carry(uint32_t nblk, uint64_t t0, const uint64_t* __restrict__ abs_ps,
                                                   uint64_t n_abs, const PkAgg* __restrict__ agg, uint64_t* __restrict__ carry,
                                                   uint64_t* __restrict__ escbase)
{
   __shared__ uint32_t fl[1024];
   __shared__ uint64_t va[1024], eb[1024];
   __shared__ uint64_t s_t, s_e;
   const uint32_t tid = threadIdx.x;
   if (tid == 0) { s_t = t0; s_e = 0; }
   __syncthreads();
   for (uint32_t b0 = 0; b0 < nblk; b0 += 1024)
   {
      const uint32_t b = b0 + tid;
      const PkAgg g = b < nblk ? agg[b] : PkAgg{ 0, 0, 0 };
      eb[tid] = g.nesc;
      __syncthreads();
      for (uint32_t d = 1; d < 1024; d <<= 1)   // inclusive prefix of the escape counts
      {
         const uint64_t x = tid >= d ? eb[tid - d] : 0;
         __syncthreads();
         eb[tid] += x;
         __syncthreads();
      }
      const uint64_t ebase = s_e + eb[tid] - g.nesc;   // escapes before block b
      fl[tid] = g.pad;                                  // the block has an escape
      va[tid] = g.pad ? pk_abs(abs_ps, n_abs, ebase + g.nesc - 1) + g.tail : g.tail;
      __syncthreads();
      seg_scan(fl, va, tid, 1024);
      // the time before block b: the previous inclusive value (or the carried one)
      const uint64_t prev = tid == 0 ? s_t : (fl[tid - 1] ? va[tid - 1] : s_t + va[tid - 1]);
      if (b < nblk)
      {
         carry[b] = prev;
         escbase[b] = ebase;
      }
      __syncthreads();
      if (tid == 1023)
      {
         s_t = fl[1023] ? va[1023] : s_t + va[1023];
         s_e += eb[1023];
      }
      __syncthreads();
   }
   if (tid == 0) escbase[nblk] = s_e;   // the batch's escapes (checked against n_abs)
}
// The validation's verdict on a delta-format batch: its escapes must be exactly the
// absolute times the caller gave (else the decode read past them).
__global__ void k_pk_check(const uint64_t* __restrict__ esc, uint64_t n_abs, unsigned long long* __restrict__ bad)
{
   if (*esc != n_abs) *bad = 0ull;
}
__global__ __launch_bounds__(PK_T) void k_dt_unpack(uint64_t n, const uint16_t* __restrict__ dt,
                                                    const uint64_t* __restrict__ abs_ps, uint64_t n_abs,
                                                    const uint64_t* __restrict__ carry,
                                                    const uint64_t* __restrict__ escbase, const uint16_t* __restrict__ src,
                                                    const uint16_t* __restrict__ dst, const uint16_t* __restrict__ bits,
                                                    uint32_t bits_all, const uint8_t* __restrict__ flags,
                                                    uint64_t* __restrict__ oinj, uint32_t* __restrict__ osrc,
                                                    uint32_t* __restrict__ odst, uint32_t* __restrict__ obits,
                                                    uint32_t* __restrict__ oflags)
{
   __shared__ uint32_t fl[PK_T], ne[PK_T];
   __shared__ uint64_t va[PK_T];
   __shared__ uint16_t sd[PK_B];
   __shared__ uint64_t st[PK_B];
   const uint32_t tid = threadIdx.x;
   const uint64_t b0 = (uint64_t) blockIdx.x * PK_B;
   // the other fields widen lane-strided (coalesced); the differences go through
   // LDS to each thread's PK_PT consecutive ones, and the inject times back
#pragma unroll
   for (uint32_t k = 0; k < PK_PT; k++)
   {
      const uint64_t i = b0 + k * PK_T + tid;
      sd[k * PK_T + tid] = i < n ? dt[i] : (uint16_t) 0;
      if (i < n)
      {
         osrc[i] = src[i];
         odst[i] = dst[i];
         obits[i] = bits ? (uint32_t) bits[i] : bits_all;
         oflags[i] = flags ? (uint32_t) flags[i] : 0u;
      }
   }
   __syncthreads();
   const uint64_t i0 = b0 + (uint64_t) tid * PK_PT;
   uint16_t d[PK_PT];
   uint32_t c = 0, f = 0;
   uint64_t tail = 0;
#pragma unroll
   for (uint32_t k = 0; k < PK_PT; k++)
   {
      d[k] = sd[tid * PK_PT + k];
      if (i0 + k < n && d[k] == PK_ESC)
      {
         f = 1;
         tail = 0;
         c++;
      }
      else tail += d[k];
   }
   ne[tid] = c;
   __syncthreads();
   for (uint32_t s = 1; s < PK_T; s <<= 1)   // inclusive prefix of the escape counts
   {
      const uint32_t x = tid >= s ? ne[tid - s] : 0u;
      __syncthreads();
      ne[tid] += x;
      __syncthreads();
   }
   uint64_t eo = escbase[blockIdx.x] + ne[tid] - c;   // this thread's first escape ordinal
   fl[tid] = f;
   va[tid] = f ? pk_abs(abs_ps, n_abs, eo + c - 1) + tail : tail;
   __syncthreads();
   seg_scan(fl, va, tid, PK_T);
   const uint64_t cin = carry[blockIdx.x];
   uint64_t T = tid == 0 ? cin : (fl[tid - 1] ? va[tid - 1] : cin + va[tid - 1]);
#pragma unroll
   for (uint32_t k = 0; k < PK_PT; k++)
   {
      if (i0 + k >= n) break;
      T = d[k] == PK_ESC ? pk_abs(abs_ps, n_abs, eo++) : T + d[k];
      st[tid * PK_PT + k] = T;
   }
   __syncthreads();
#pragma unroll
   for (uint32_t k = 0; k < PK_PT; k++)
   {
      const uint64_t i = b0 + k * PK_T + tid;
      if (i < n) oinj[i] = st[k * PK_T + tid];
   }
}

// Copy a packed trace (host) into the stage buffer and decode it into (inj, src, dst,
// bits, flags) on stream q.
static int stage_packed(gnoc_engine* e, const gnoc_packets_packed* pk, size_t n, DevBuf& stage, DevBuf& inj, DevBuf& src,
                        DevBuf& dst, DevBuf& bits, DevBuf& flags, hipStream_t q)
{
   if (n && (!pk->dt || !pk->src || !pk->dst)) return fail(e, GNOC_EINVAL, "null trace array");
   if (pk->n_abs && !pk->abs_ps) return fail(e, GNOC_EINVAL, "null abs_ps with n_abs > 0");
   if (pk->n_abs > n) return fail(e, GNOC_EINVAL, "more absolute inject times than packets");
   if (n >= (1ull << 32) - 1) return fail(e, GNOC_EUNSUPPORTED, "more than 2^32-2 packets");
   if (e->nranks > 1) return fail(e, GNOC_EUNSUPPORTED, "a sharded engine takes gnoc_submit");
   if (e->dc.N > 65536) return fail(e, GNOC_EUNSUPPORTED, "the packed wire format needs at most 65,536 tiles");
   GNOC_HIP(e, inj.ensure(n * 8));
   GNOC_HIP(e, src.ensure(n * 4));
   GNOC_HIP(e, dst.ensure(n * 4));
   GNOC_HIP(e, bits.ensure(n * 4));
   GNOC_HIP(e, flags.ensure(n * 4));
   const uint32_t nblk = (uint32_t) ((n + PK_B - 1) / PK_B);
   // dt, src, dst, bits (u16) | flags (u8) | abs_ps | block aggregates, carries, escape bases (8-B aligned)
   const size_t o_f8 = n * 8, o_abs = (o_f8 + n + 15) / 16 * 16, o_agg = o_abs + (size_t) pk->n_abs * 8;
   const size_t o_car = o_agg + (size_t) nblk * sizeof(PkAgg), o_eb = o_car + (size_t) nblk * 8;
   GNOC_HIP(e, stage.ensure(o_eb + ((size_t) nblk + 1) * 8 + 16));   // (+ the escape total)
   e->val_esc = nullptr;
   e->val_nabs = pk->n_abs;
   if (!n)
   {
      if (pk->n_abs) return fail(e, GNOC_ETRACE, "packed trace: absolute times given for an empty batch");
      return GNOC_OK;
   }
   char* sb = static_cast<char*>(stage.p);
   uint16_t* s16 = reinterpret_cast<uint16_t*>(sb);
   uint8_t* f8 = reinterpret_cast<uint8_t*>(sb + o_f8);
   uint64_t* ab = reinterpret_cast<uint64_t*>(sb + o_abs);
   PkAgg* agg = reinterpret_cast<PkAgg*>(sb + o_agg);
   uint64_t* car = reinterpret_cast<uint64_t*>(sb + o_car);
   uint64_t* ebs = reinterpret_cast<uint64_t*>(sb + o_eb);
   GNOC_HIP(e, hipMemcpyAsync(s16, pk->dt, n * 2, hipMemcpyHostToDevice, q));
   GNOC_HIP(e, hipMemcpyAsync(s16 + n, pk->src, n * 2, hipMemcpyHostToDevice, q));
   GNOC_HIP(e, hipMemcpyAsync(s16 + 2 * n, pk->dst, n * 2, hipMemcpyHostToDevice, q));
   if (pk->bits) GNOC_HIP(e, hipMemcpyAsync(s16 + 3 * n, pk->bits, n * 2, hipMemcpyHostToDevice, q));
   if (pk->flags) GNOC_HIP(e, hipMemcpyAsync(f8, pk->flags, n, hipMemcpyHostToDevice, q));
   if (pk->n_abs) GNOC_HIP(e, hipMemcpyAsync(ab, pk->abs_ps, (size_t) pk->n_abs * 8, hipMemcpyHostToDevice, q));
   hipLaunchKernelGGL(k_dt_block, dim3(nblk), dim3(PK_T), 0, q, (uint64_t) n, (const uint16_t*) s16, agg);
   hipLaunchKernelGGL(k_dt_carry, dim3(1), dim3(1024), 0, q, nblk, pk->t0, (const uint64_t*) ab, (uint64_t) pk->n_abs,
                      (const PkAgg*) agg, car, ebs);
   e->val_esc = ebs + nblk;
   hipLaunchKernelGGL(k_dt_unpack, dim3(nblk), dim3(PK_T), 0, q, (uint64_t) n, (const uint16_t*) s16, (const uint64_t*) ab,
                      (uint64_t) pk->n_abs, (const uint64_t*) car, (const uint64_t*) ebs, (const uint16_t*) (s16 + n), (const uint16_t*) (s16 + 2 * n),
                      pk->bits ? (const uint16_t*) (s16 + 3 * n) : nullptr, pk->bits_all,
                      pk->flags ? (const uint8_t*) f8 : nullptr, inj.as<uint64_t>(), src.as<uint32_t>(), dst.as<uint32_t>(),
                      bits.as<uint32_t>(), flags.as<uint32_t>());
   GNOC_HIP(e, hipGetLastError());
   return GNOC_OK;
}

// Copy a narrow trace (host) into the stage buffer and widen it into (inj, src, dst,
// bits, flags) on stream q.
static int stage_narrow(gnoc_engine* e, const gnoc_packets_narrow* pk, size_t n, DevBuf& stage, DevBuf& inj, DevBuf& src,
                        DevBuf& dst, DevBuf& bits, DevBuf& flags, hipStream_t q)
{
   if (n && (!pk->inject_ps || !pk->src || !pk->dst || !pk->bits)) return fail(e, GNOC_EINVAL, "null trace array");
   if (n >= (1ull << 32) - 1) return fail(e, GNOC_EUNSUPPORTED, "more than 2^32-2 packets");
   if (e->nranks > 1) return fail(e, GNOC_EUNSUPPORTED, "a sharded engine takes gnoc_submit");
   if (e->dc.N > 65536) return fail(e, GNOC_EUNSUPPORTED, "the narrow wire format needs at most 65,536 tiles");
   GNOC_HIP(e, inj.ensure(n * 8));
   GNOC_HIP(e, src.ensure(n * 4));
   GNOC_HIP(e, dst.ensure(n * 4));
   GNOC_HIP(e, bits.ensure(n * 4));
   GNOC_HIP(e, flags.ensure(n * 4));
   GNOC_HIP(e, stage.ensure(n * 7 + 16));
   if (!n) return GNOC_OK;
   uint16_t* s16 = stage.as<uint16_t>();
   uint8_t* f8 = reinterpret_cast<uint8_t*>(s16 + 3 * n);
   GNOC_HIP(e, hipMemcpyAsync(inj.p, pk->inject_ps, n * 8, hipMemcpyHostToDevice, q));
   GNOC_HIP(e, hipMemcpyAsync(s16, pk->src, n * 2, hipMemcpyHostToDevice, q));
   GNOC_HIP(e, hipMemcpyAsync(s16 + n, pk->dst, n * 2, hipMemcpyHostToDevice, q));
   GNOC_HIP(e, hipMemcpyAsync(s16 + 2 * n, pk->bits, n * 2, hipMemcpyHostToDevice, q));
   if (pk->flags) GNOC_HIP(e, hipMemcpyAsync(f8, pk->flags, n, hipMemcpyHostToDevice, q));
   const uint32_t grid = (uint32_t) std::min<size_t>((n + 255) / 256, 4096);
   hipLaunchKernelGGL(k_widen, dim3(grid), dim3(256), 0, q, (uint64_t) n, (const uint16_t*) s16, (const uint16_t*) (s16 + n),
                      (const uint16_t*) (s16 + 2 * n), pk->flags ? (const uint8_t*) f8 : nullptr, src.as<uint32_t>(),
                      dst.as<uint32_t>(), bits.as<uint32_t>(), flags.as<uint32_t>());
   GNOC_HIP(e, hipGetLastError());
   return GNOC_OK;
}

int gnoc_submit_narrow(gnoc_engine* e, const gnoc_packets_narrow* pk, size_t n)
{
   if (!e || !pk) return GNOC_EINVAL;
   e->submitted = false;
   e->val_esc = nullptr;   // no packed decode behind this batch
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   int rc = stage_narrow(e, pk, n, e->nw_stage, e->t_inj, e->t_src, e->t_dst, e->t_bits, e->t_flags, e->stream);
   if (rc) return rc;
   e->part = false;
   e->n_glob = n;
   e->d_inj = e->t_inj.as<uint64_t>();
   e->d_src = e->t_src.as<uint32_t>();
   e->d_dst = e->t_dst.as<uint32_t>();
   e->d_bits = e->t_bits.as<uint32_t>();
   e->d_flags = e->t_flags.as<uint32_t>();
   e->n = n;
   e->dc.npk = n;
   return submit_tail(e, nullptr, n);
}

int gnoc_submit_packed(gnoc_engine* e, const gnoc_packets_packed* pk, size_t n)
{
   if (!e || !pk) return GNOC_EINVAL;
   e->submitted = false;
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   int rc = stage_packed(e, pk, n, e->nw_stage, e->t_inj, e->t_src, e->t_dst, e->t_bits, e->t_flags, e->stream);
   if (rc) return rc;
   e->part = false;
   e->n_glob = n;
   e->d_inj = e->t_inj.as<uint64_t>();
   e->d_src = e->t_src.as<uint32_t>();
   e->d_dst = e->t_dst.as<uint32_t>();
   e->d_bits = e->t_bits.as<uint32_t>();
   e->d_flags = e->t_flags.as<uint32_t>();
   e->n = n;
   e->dc.npk = n;
   return submit_tail(e, nullptr, n);
}

int gnoc_submit(gnoc_engine* e, const gnoc_packets* pk_in, size_t n)
{
   if (!e || !pk_in) return GNOC_EINVAL;
   if (n && (!pk_in->inject_ps || !pk_in->src || !pk_in->dst || !pk_in->bits)) return fail(e, GNOC_EINVAL, "null trace array");
   if (n >= (1ull << 32) - 1) return fail(e, GNOC_EUNSUPPORTED, "more than 2^32-2 packets");
   e->submitted = false;
   e->val_esc = nullptr;   // no packed decode behind this batch
   const gnoc_packets* pk = pk_in;
   gnoc_packets sub{};
   std::vector<uint64_t> l_inj;
   std::vector<uint32_t> l_src, l_dst, l_bits, l_flags;
   e->part = e->nranks > 1 && e->dc.W <= 64 && e->dc.H <= 64 && e->npoints == 1 && !e->dc.hop_counter && e->dc.contention &&
             !std::getenv("GNOC_NO_PARTITION");
   e->n_glob = n;
   if (e->part)
   {
      const int prc = partition_trace(e, pk_in, n, &sub, l_inj, l_src, l_dst, l_bits, l_flags);
      if (prc) return prc;
      pk = &sub;
      n = e->h_gid.size();
   }
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
   }
   e->d_inj = e->t_inj.as<uint64_t>();
   e->d_src = e->t_src.as<uint32_t>();
   e->d_dst = e->t_dst.as<uint32_t>();
   e->d_bits = e->t_bits.as<uint32_t>();
   e->d_flags = e->t_flags.as<uint32_t>();
   e->n = n;
   e->dc.npk = e->part ? e->n_glob : n;
   if (e->part)
   {
      GNOC_HIP(e, e->d_gid.ensure(n * 4 + 4));
      GNOC_HIP(e, e->fin_glob.ensure(e->n_glob * 8 + 8));
      if (n) GNOC_HIP(e, hipMemcpyAsync(e->d_gid.p, e->h_gid.data(), n * 4, hipMemcpyHostToDevice, e->stream));
   }
   return submit_tail(e, pk, n);
}

// The rest of a host-trace submit, once the trace is in the engine's buffers
// (d_inj .. d_flags, n): the device-side contract checks and statistics, the
// record bound, broadcast tables (from the host flags), the exchange layout.
static int submit_tail(gnoc_engine* e, const gnoc_packets* pk, size_t n, bool prevalidated)
{
   uint64_t records = 0, nbc = 0;
   // (device_validate's sync also ends the copies; a staged batch was checked on the
   // upload stream beside the previous run, its summary is in h_val)
   int rc = prevalidated ? validate_finish(e, e->h_val, &records, &nbc) : device_validate(e, n, &records, &nbc);
   if (rc) return rc;
   if (record_bound(e, records) >= (1ull << 31)) return fail(e, GNOC_EUNSUPPORTED, "more than 2^31 hop records");
   e->rec_bound = record_bound(e, records);
   e->h_bid.clear();
   if (nbc && !pk) return fail(e, GNOC_EUNSUPPORTED, "broadcast packets need gnoc_submit");
   if (nbc)
      for (size_t i = 0; i < n; i++)
         if (pk->flags[i] & GNOC_PKT_BROADCAST) e->h_bid.push_back((uint32_t) i);
   rc = upload_broadcasts(e);
   if (rc) return rc;
   rc = build_exchange(e);
   if (rc) return rc;
   e->runs = e->tot_retry = e->tot_fallback = 0;
   e->submitted = true;
   e->ran = false;
   e->begun = false;
   return GNOC_OK;
}

// ---------------------------------------------------------------------------
// pipelined batches: upload of batch k+1 and read-back of batch k-1 beside run k
// ---------------------------------------------------------------------------
static hipError_t pipe_streams(gnoc_engine* e)
{
   hipError_t he = hipSuccess;
   if (!e->s_h2d) he = hipStreamCreateWithFlags(&e->s_h2d, hipStreamNonBlocking);
   if (he == hipSuccess && !e->s_d2h) he = hipStreamCreateWithFlags(&e->s_d2h, hipStreamNonBlocking);
   for (hipEvent_t* ev : { &e->ev_h2d, &e->ev_done, &e->ev_fin, &e->ev_alt })
      if (he == hipSuccess && !*ev) he = hipEventCreateWithFlags(ev, hipEventDisableTiming);
   return he;
}

// A staged batch's device checks on the upload stream, right behind its copies: they
// run beside the current batch's run instead of after it (gnoc_submit_commit then only
// reads the summary).  Not for the exchange-count statistics of the self-exchange knob.
static int stage_validate(gnoc_engine* e, size_t n)
{
   e->staged_val = false;
   if (e->nranks > 1 || e->xself) return GNOC_OK;
   const int rc = validate_launch(e, n, ValTrace{ e->t2_inj.as<uint64_t>(), e->t2_src.as<uint32_t>(), e->t2_dst.as<uint32_t>(),
                                                  e->t2_bits.as<uint32_t>(), e->t2_flags.as<uint32_t>() },
                                  e->s_h2d, e->vbuf2, e->h_val, nullptr);
   if (!rc) e->staged_val = true;
   return rc;
}

int gnoc_submit_async(gnoc_engine* e, const gnoc_packets* pk, size_t n)
{
   if (!e || !pk) return GNOC_EINVAL;
   if (n && (!pk->inject_ps || !pk->src || !pk->dst || !pk->bits)) return fail(e, GNOC_EINVAL, "null trace array");
   if (n >= (1ull << 32) - 1) return fail(e, GNOC_EUNSUPPORTED, "more than 2^32-2 packets");
   if (e->nranks > 1) return fail(e, GNOC_EUNSUPPORTED, "a sharded engine takes gnoc_submit");
   if (e->staged) return fail(e, GNOC_ESTATE, "a staged batch is waiting for gnoc_submit_commit");
   e->val_esc = nullptr;   // no packed decode behind this batch
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   GNOC_HIP(e, pipe_streams(e));
   GNOC_HIP(e, e->t2_inj.ensure(n * 8));
   GNOC_HIP(e, e->t2_src.ensure(n * 4));
   GNOC_HIP(e, e->t2_dst.ensure(n * 4));
   GNOC_HIP(e, e->t2_bits.ensure(n * 4));
   GNOC_HIP(e, e->t2_flags.ensure(n * 4));
   if (n)
   {
      hipStream_t q = e->s_h2d;
      GNOC_HIP(e, hipMemcpyAsync(e->t2_inj.p, pk->inject_ps, n * 8, hipMemcpyHostToDevice, q));
      GNOC_HIP(e, hipMemcpyAsync(e->t2_src.p, pk->src, n * 4, hipMemcpyHostToDevice, q));
      GNOC_HIP(e, hipMemcpyAsync(e->t2_dst.p, pk->dst, n * 4, hipMemcpyHostToDevice, q));
      GNOC_HIP(e, hipMemcpyAsync(e->t2_bits.p, pk->bits, n * 4, hipMemcpyHostToDevice, q));
      if (pk->flags) GNOC_HIP(e, hipMemcpyAsync(e->t2_flags.p, pk->flags, n * 4, hipMemcpyHostToDevice, q));
      else GNOC_HIP(e, hipMemsetAsync(e->t2_flags.p, 0, n * 4, q));
   }
   int rc = stage_validate(e, n);
   if (rc) return rc;
   GNOC_HIP(e, hipEventRecord(e->ev_h2d, e->s_h2d));
   e->staged = true;
   e->staged_narrow = false;
   e->staged_pk = *pk;
   e->staged_n = n;
   return GNOC_OK;
}

int gnoc_submit_async_narrow(gnoc_engine* e, const gnoc_packets_narrow* pk, size_t n)
{
   if (!e || !pk) return GNOC_EINVAL;
   if (e->staged) return fail(e, GNOC_ESTATE, "a staged batch is waiting for gnoc_submit_commit");
   e->val_esc = nullptr;   // no packed decode behind this batch
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   GNOC_HIP(e, pipe_streams(e));
   int rc = stage_narrow(e, pk, n, e->nw_stage2, e->t2_inj, e->t2_src, e->t2_dst, e->t2_bits, e->t2_flags, e->s_h2d);
   if (!rc) rc = stage_validate(e, n);
   if (rc) return rc;
   GNOC_HIP(e, hipEventRecord(e->ev_h2d, e->s_h2d));
   e->staged = true;
   e->staged_narrow = true;
   e->staged_pk = gnoc_packets{};
   e->staged_n = n;
   return GNOC_OK;
}

int gnoc_submit_async_packed(gnoc_engine* e, const gnoc_packets_packed* pk, size_t n)
{
   if (!e || !pk) return GNOC_EINVAL;
   if (e->staged) return fail(e, GNOC_ESTATE, "a staged batch is waiting for gnoc_submit_commit");
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   GNOC_HIP(e, pipe_streams(e));
   int rc = stage_packed(e, pk, n, e->nw_stage2, e->t2_inj, e->t2_src, e->t2_dst, e->t2_bits, e->t2_flags, e->s_h2d);
   if (!rc) rc = stage_validate(e, n);
   if (rc) return rc;
   GNOC_HIP(e, hipEventRecord(e->ev_h2d, e->s_h2d));
   e->staged = true;
   e->staged_narrow = true;   // (no host arrays kept: unicast batches only, as narrow)
   e->staged_pk = gnoc_packets{};
   e->staged_n = n;
   return GNOC_OK;
}

int gnoc_submit_commit(gnoc_engine* e)
{
   if (!e) return GNOC_EINVAL;
   if (!e->staged) return fail(e, GNOC_ESTATE, "gnoc_submit_commit without gnoc_submit_async");
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   e->staged = false;
   e->submitted = false;
   // the compute stream takes the staged buffers once their upload is done
   GNOC_HIP(e, hipStreamWaitEvent(e->stream, e->ev_h2d, 0));
   e->t_inj.swap(e->t2_inj);
   e->t_src.swap(e->t2_src);
   e->t_dst.swap(e->t2_dst);
   e->t_bits.swap(e->t2_bits);
   e->t_flags.swap(e->t2_flags);
   const size_t n = e->staged_n;
   e->part = false;
   e->n_glob = n;
   e->d_inj = e->t_inj.as<uint64_t>();
   e->d_src = e->t_src.as<uint32_t>();
   e->d_dst = e->t_dst.as<uint32_t>();
   e->d_bits = e->t_bits.as<uint32_t>();
   e->d_flags = e->t_flags.as<uint32_t>();
   e->n = n;
   e->dc.npk = n;
   gnoc_packets pk = e->staged_pk;
   const bool narrow = e->staged_narrow;
   e->staged_narrow = false;
   const bool pre = e->staged_val;
   e->staged_val = false;
   if (pre) GNOC_HIP(e, hipEventSynchronize(e->ev_h2d));   // (the checks' summary is in h_val)
   return submit_tail(e, narrow ? nullptr : &pk, n, pre);
}

int gnoc_fetch_final_ps(gnoc_engine* e, uint64_t* host_out, size_t n)
{
   if (!e || !host_out) return GNOC_EINVAL;
   if (!e->ran) return fail(e, GNOC_ESTATE, "no results: call gnoc_run first");
   if (e->part || e->nranks > 1) return fail(e, GNOC_EUNSUPPORTED, "a sharded rank's results: gnoc_get_packet_results");
   if (n != e->n) return fail(e, GNOC_EINVAL, "n differs from the submitted batch");
   if (e->nb) return fail(e, GNOC_EUNSUPPORTED, "broadcast batches: gnoc_get_packet_results");
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   GNOC_HIP(e, pipe_streams(e));
   GNOC_HIP(e, hipEventRecord(e->ev_done, e->stream));
   GNOC_HIP(e, hipStreamWaitEvent(e->s_d2h, e->ev_done, 0));
   if (n) GNOC_HIP(e, hipMemcpyAsync(host_out, e->final_ps.p, n * 8, hipMemcpyDeviceToHost, e->s_d2h));
   GNOC_HIP(e, hipEventRecord(e->ev_fin, e->s_d2h));
   e->fetched = true;   // the next run writes the other buffer
   return GNOC_OK;
}

int gnoc_fetch_latency(gnoc_engine* e, uint32_t* host_out, size_t n)
{
   if (!e || !host_out) return GNOC_EINVAL;
   if (!e->ran) return fail(e, GNOC_ESTATE, "no results: call gnoc_run first");
   if (e->part || e->nranks > 1) return fail(e, GNOC_EUNSUPPORTED, "a sharded rank's results: gnoc_get_packet_results");
   if (n != e->n) return fail(e, GNOC_EINVAL, "n differs from the submitted batch");
   if (e->nb) return fail(e, GNOC_EUNSUPPORTED, "broadcast batches: gnoc_get_packet_results");
   if (e->ma_type && e->dc.contention) return fail(e, GNOC_EUNSUPPORTED, "moving-average queues: gnoc_fetch_final_ps");
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   if (!e->lat_written)
   {
      // the first call: the u32 array of the last run now (k_finalize again: the same
      // zero-load and contention values), and every later run writes it in k_finalize
      e->want_lat32 = true;
      hipStream_t s = e->stream;
      GNOC_HIP(e, e->lat32.ensure(n * 4 + 4));
      unsigned* lovf = e->counters.as<unsigned>() + 8 + 6;
      const uint32_t fin_grid = (uint32_t) std::max<size_t>(1, std::min<size_t>((n + 255) / 256, 8192));
      const int cf = e->dc.contention ? 0 : 1;
      if (n && e->f1)
         hipLaunchKernelGGL(k_finalize<true>, dim3(fin_grid), dim3(256), 0, s, e->dc, (uint64_t) n, e->d_inj, e->d_src,
                            e->aux.as<uint32_t>(), e->routed.as<uint8_t>(), e->final_ps.as<uint64_t>(), e->zl.as<uint64_t>(),
                            e->cont.as<uint64_t>(), cf, e->cx0, e->cx1, e->lat32.as<uint32_t>(), lovf, nullptr, nullptr);
      else if (n)
         hipLaunchKernelGGL(k_finalize<false>, dim3(fin_grid), dim3(256), 0, s, e->dc, (uint64_t) n, e->d_inj, e->d_src,
                            e->aux.as<uint32_t>(), e->routed.as<uint8_t>(), e->final_ps.as<uint64_t>(), e->zl.as<uint64_t>(),
                            e->cont.as<uint64_t>(), cf, e->cx0, e->cx1, e->lat32.as<uint32_t>(), lovf, nullptr, nullptr);
      GNOC_HIP(e, hipGetLastError());
      GNOC_HIP(e, hipMemcpyAsync(e->h_pinned + 8, e->counters.as<unsigned int>() + 8, 32, hipMemcpyDeviceToHost, s));
      GNOC_HIP(e, hipStreamSynchronize(s));
      e->lat_ovf = (((const unsigned*) (e->h_pinned + 8))[6] & 1u) != 0;
      e->lat_written = true;
   }
   if (e->lat_ovf) return fail(e, GNOC_EUNSUPPORTED, "a packet latency of 2^32 ps or more: use gnoc_fetch_final_ps");
   GNOC_HIP(e, pipe_streams(e));
   GNOC_HIP(e, hipEventRecord(e->ev_done, e->stream));
   GNOC_HIP(e, hipStreamWaitEvent(e->s_d2h, e->ev_done, 0));
   if (n) GNOC_HIP(e, hipMemcpyAsync(host_out, e->lat32.p, n * 4, hipMemcpyDeviceToHost, e->s_d2h));
   GNOC_HIP(e, hipEventRecord(e->ev_fin, e->s_d2h));
   e->fetched = true;   // the next run writes the other buffers
   return GNOC_OK;
}

int gnoc_fetch_wait(gnoc_engine* e)
{
   if (!e) return GNOC_EINVAL;
   if (e->s_d2h) GNOC_HIP(e, hipStreamSynchronize(e->s_d2h));
   return GNOC_OK;
}

int gnoc_submit_device(gnoc_engine* e, const gnoc_packets* pk, size_t n)
{
   if (!e || !pk) return GNOC_EINVAL;
   e->val_esc = nullptr;   // no packed decode behind this batch
   e->part = false;        // a device trace is used as is (every rank reads all of it)
   e->n_glob = n;
   if (n && (!pk->inject_ps || !pk->src || !pk->dst || !pk->bits)) return fail(e, GNOC_EINVAL, "null trace array");
   if (n >= (1ull << 32) - 1) return fail(e, GNOC_EUNSUPPORTED, "more than 2^32-2 packets");
   if (e->nranks > 1) return fail(e, GNOC_EUNSUPPORTED, "a sharded engine takes host traces (gnoc_submit)");
   e->submitted = false;
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   e->d_inj = pk->inject_ps;
   e->d_src = pk->src;
   e->d_dst = pk->dst;
   e->d_bits = pk->bits;
   e->d_flags = pk->flags;
   e->n = n;
   e->dc.npk = n;
   // the same contract as gnoc_submit, checked on the device
   uint64_t records = 0, nbc = 0;
   int rc = device_validate(e, n, &records, &nbc);
   if (rc) return rc;
   if (nbc) return fail(e, GNOC_EUNSUPPORTED, "broadcast packets need a host trace (gnoc_submit)");
   if (record_bound(e, records) >= (1ull << 31)) return fail(e, GNOC_EUNSUPPORTED, "more than 2^31 hop records");
   e->rec_bound = record_bound(e, records);
   e->h_bid.clear();
   rc = upload_broadcasts(e);
   if (rc) return rc;
   e->runs = e->tot_retry = e->tot_fallback = 0;
   e->submitted = true;
   e->ran = false;
   e->begun = false;
   return GNOC_OK;
}

// ---------------------------------------------------------------------------
// v1: whole-port streams, host-built plan (f != 1 GHz, max_list_size <= 2, retries)
// ---------------------------------------------------------------------------
// Where the delivery level writes final times: the local array, or (a partitioned
// rank) the global-id array that k_finalize reads back by gid.
static uint64_t* fin_out(gnoc_engine* e)
{
   return e->part ? e->fin_glob.as<uint64_t>() : e->final_ps.as<uint64_t>();
}

static int run_levels_v1(gnoc_engine* e)
{
   const DevCfg& c = e->dc;
   hipStream_t s = e->stream;
   const uint32_t nslots = c.N * PORTS * INS;
   e->h_slot_cnt.resize(nslots);
   GNOC_HIP(e, hipMemcpyAsync(e->h_slot_cnt.data(), e->slot_cnt.p, (size_t) nslots * 4, hipMemcpyDeviceToHost, s));
   GNOC_HIP(e, hipStreamSynchronize(s));
   std::vector<uint32_t> ports, off;
   for (size_t l = 0; l + 1 < e->lvl_off.size(); l++)
   {
      off.push_back((uint32_t) ports.size());
      for (uint32_t k = e->lvl_off[l]; k < e->lvl_off[l + 1]; k++)
      {
         const uint32_t p = e->lvl_ports[k];
         bool any = false;
         for (uint32_t in = 0; in < INS; in++) any |= e->h_slot_cnt[p * INS + in] != 0;
         if (any) ports.push_back(p);
      }
   }
   off.push_back((uint32_t) ports.size());
   GNOC_HIP(e, e->plan_ports.ensure(std::max<size_t>(1, ports.size()) * 4));
   if (!ports.empty())
      GNOC_HIP(e, hipMemcpyAsync(e->plan_ports.p, ports.data(), ports.size() * 4, hipMemcpyHostToDevice, s));
   GNOC_HIP(e, e->dirty.ensure((size_t) nslots * 4));
   GNOC_HIP(e, hipMemsetAsync(e->dirty.p, 0, (size_t) nslots * 4, s));
   if (e->nb)
   {
      GNOC_HIP(e, e->d_btail.ensure((size_t) nslots * 4));
      GNOC_HIP(e, hipMemsetAsync(e->d_btail.p, 0, (size_t) nslots * 4, s));
   }
   e->h_levels = (uint32_t) (off.size() - 1);
   for (size_t l = 0; l + 1 < off.size(); l++)
   {
      const uint32_t cnt = off[l + 1] - off[l];
      if (!cnt) continue;
      const uint32_t* pp = e->plan_ports.as<uint32_t>() + off[l];
#define GNOC_PORT(F1V, BCV)                                                                                         \
   GNOC_LAUNCH(e, KC_PORT, (k_port_stream<F1V, BCV>), dim3(cnt), dim3(STHREADS), 0, s, c, pp, e->slot_cnt.as<uint32_t>(), \
               e->slot_base.as<uint64_t>(), e->recs.as<Rec>(), fin_out(e), e->port_sum.as<uint64_t>(),                   \
               e->port_cnt.as<uint64_t>(), e->port_mg1.as<uint64_t>(), e->port_flit.as<uint64_t>(),                     \
               e->port_last.as<uint64_t>(), e->dirty.as<uint32_t>(), e->counters.as<unsigned int>() + 8,                \
               (const uint32_t*) e->d_bcnt.as<uint32_t>(), e->d_btail.as<uint32_t>())
      if (e->nb)
      {
         if (e->f1) GNOC_PORT(true, true);
         else GNOC_PORT(false, true);
      }
      else
      {
         if (e->f1) GNOC_PORT(true, false);
         else GNOC_PORT(false, false);
      }
#undef GNOC_PORT
   }
   return GNOC_OK;
}

// ---------------------------------------------------------------------------
// v3: device-planned chunked levels
// ---------------------------------------------------------------------------
// Records per chunk: LV_CTGT for the chain path's injection and SELF levels,
// LV_CTGT_FULL when every level runs on k_level (levels of X / Y ports, with more
// chunks per level in flight), or GNOC_CHUNK (test knob: small chunks put serial
// M/G/1 prefixes and exception tails across many chunk boundaries).
static uint32_t chunk_target(bool full = true)
{
   const char* v = std::getenv("GNOC_CHUNK");
   const long t = v ? std::atol(v) : 0;
   return t > 0 ? (uint32_t) std::min<long>(std::max<long>(t, 64), LV_CMAX) : full ? LV_CTGT_FULL : LV_CTGT;
}
static uint64_t chunk_bound_of(const gnoc_engine* e, uint32_t P)
{
   const uint32_t tgt = std::min(chunk_target(true), chunk_target(false));   // (the more chunks)
   const uint32_t cmin = LV_ROUNDS_FIT ? std::min<uint32_t>(LV_CMIN, tgt) : tgt;   // smallest chunk a level can get
   return e->rec_bound / cmin + P + 1;
}

static int zq_flush(gnoc_engine* e, hipStream_t s);
// ends_only: chunks for the injection and SELF levels only (the chain engine runs the
// X and Y levels; a decline that reruns them on k_level plans again in full).
static int run_plan_v3(gnoc_engine* e, bool ends_only = false)
{
   const DevCfg& c = e->dc;
   hipStream_t s = e->stream;
   const uint32_t P = (uint32_t) e->lvl_ports.size();
   const uint32_t L = (uint32_t) e->lvl_off.size() - 1;
   uint32_t klo0 = 0, khi0 = P, klo1 = 0, khi1 = 0;
   if (ends_only && L >= 2)
   {
      khi0 = e->lvl_off[1];
      klo1 = e->lvl_off[L - 1];
      khi1 = e->lvl_off[L];
   }
   const uint64_t chunk_bound = chunk_bound_of(e, P);
   const uint32_t ctgt = chunk_target(!ends_only);
   GNOC_HIP(e, e->pio.ensure((size_t) P * sizeof(PortIO3)));
   GNOC_HIP(e, e->pnc.ensure((size_t) P * 4));
   GNOC_HIP(e, e->pgb.ensure((size_t) P * 4));
   GNOC_HIP(e, e->lvl_cbase.ensure((size_t) (L + 1) * 4));
   GNOC_HIP(e, e->cdesc.ensure(chunk_bound * sizeof(PortIO3)));
   GNOC_HIP(e, e->st.ensure(chunk_bound * LV_STATE_WORDS * 8));
   GNOC_HIP(e, e->lvl_ctr.ensure((size_t) L * LV_QUEUES * 4));
   GNOC_HIP(e, e->lvl_qb.ensure((size_t) L * LV_QB * 4));
   e->zq.push_back({ e->lvl_ctr.p, (uint64_t) L * LV_QUEUES * 4 });   // zeroed before the first level (zq_flush)
   const uint32_t pg = (P + 255) / 256;
   GNOC_LAUNCH(e, KC_PLAN, k_plan_ports, dim3(pg), dim3(256), 0, s, c, P, e->d_lvl_ports.as<uint32_t>(),
               e->d_port_k.as<uint32_t>(), e->slot_cnt.as<uint32_t>(), e->slot_base.as<uint64_t>(), e->pio.as<PortIO3>(), e->pnc.as<uint32_t>(),
               ctgt, klo0, khi0, klo1, khi1);
   GNOC_LAUNCH(e, KC_PLAN, k_plan_guided, dim3(L), dim3(1024), 0, s, e->d_lvl_off.as<uint32_t>(), e->pnc.as<uint32_t>(),
               ctgt, (uint64_t) e->level_grid);
   GNOC_LAUNCH(e, KC_PLAN, k_plan_scan, dim3(1), dim3(1024), 0, s, P, L, e->d_lvl_off.as<uint32_t>(),
               e->pnc.as<uint32_t>(), e->pgb.as<uint32_t>(), e->lvl_cbase.as<uint32_t>());
   GNOC_LAUNCH(e, KC_PLAN, k_zero_state, dim3(1024), dim3(256), 0, s, e->lvl_cbase.as<uint32_t>(), L,
               e->st.as<uint64_t>());   // look-back granules
   GNOC_LAUNCH(e, KC_PLAN, k_plan_queues, dim3(L), dim3(64), 0, s, e->d_lvl_off.as<uint32_t>(), e->pgb.as<uint32_t>(),
               e->lvl_cbase.as<uint32_t>(), e->lvl_qb.as<uint32_t>(), (uint32_t) e->level_grid);
   GNOC_LAUNCH(e, KC_PLAN, k_plan_expand, dim3(pg), dim3(256), 0, s, P, e->pio.as<PortIO3>(), e->pnc.as<uint32_t>(),
               e->pgb.as<uint32_t>());
   GNOC_LAUNCH(e, KC_PLAN, k_plan_fill, dim3(P), dim3(64), 0, s, e->pio.as<PortIO3>(), e->cdesc.as<PortIO3>());
   e->h_levels = L;
   return GNOC_OK;
}

// Levels [l0, l1) of the plan built by run_plan_v3 (cond: each launch runs only if the
// streamed level declined, 1: injection, errflag[7]; 2: SELF, errflag[8]).
static int run_levels_v3(gnoc_engine* e, uint32_t l0, uint32_t l1, int cond = 0)
{
   const DevCfg& c = e->dc;
   hipStream_t s = e->stream;
   const uint32_t P = (uint32_t) e->lvl_ports.size();
   const uint32_t L = (uint32_t) e->lvl_off.size() - 1;
   const uint64_t chunk_bound = chunk_bound_of(e, P);
   const char* stv = std::getenv("GNOC_STAMPS");
   const bool stamps = stv && *stv == '1';
   e->h_chunk_bound = chunk_bound;
   if (stamps && l0 == 0)
   {
      GNOC_HIP(e, e->stamps.ensure(chunk_bound * 16 * 8));
      GNOC_HIP(e, hipMemsetAsync(e->stamps.p, 0, chunk_bound * 16 * 8, s));
   }
   if (l0 == 0)
   {
      GNOC_HIP(e, e->done.ensure((size_t) std::max<uint32_t>(P, 1) * 4));
      e->zq.push_back({ e->done.p, (uint64_t) std::max<uint32_t>(P, 1) * 4 });
   }
   {
      const int zr = zq_flush(e, s);
      if (zr) return zr;
   }
   // one launch per level (the launch boundary is the level barrier; a persistent
   // cross-level launch with port-level hand-offs was exact but 2.8x slower on 32x32)
   uint64_t* stp = stamps ? e->stamps.as<uint64_t>() : nullptr;
#define GNOC_LEVEL_ARGS(lvl)                                                                                         \
   c, (lvl) | (cond == 1 ? 0x80000000u : cond == 2 ? 0x40000000u : 0u), e->lvl_cbase.as<uint32_t>(), e->lvl_qb.as<uint32_t>(), e->lvl_ctr.as<unsigned>(), e->cdesc.as<PortIO3>(), \
      e->recs.as<Rec>(), e->samp_t.as<uint64_t>(), e->samp_id.as<uint32_t>(), e->nexc.as<uint32_t>(),                 \
      e->st.as<uint64_t>(), fin_out(e), e->port_sum.as<unsigned long long>(),                                          \
      e->port_cnt.as<unsigned long long>(), e->port_mg1.as<unsigned long long>(),                                     \
      e->port_flit.as<unsigned long long>(), e->port_last.as<unsigned long long>(), e->counters.as<unsigned>() + 8,   \
      e->done.as<uint32_t>(), stp
   {
      for (uint32_t l = l0; l < l1 && l < L; l++)
      {
         // f != 1 GHz: the double-conversion copy (no stamps); broadcast batches
         // take the variant with the broadcast branches (lv_bcast)
         if (!e->f1)
         {
            if (e->nb) GNOC_LAUNCH(e, KC_LEVEL, (lvg::k_level<false, false, true>), dim3(e->level_grid), dim3(LV_T), 0, s, GNOC_LEVEL_ARGS(l));
            else GNOC_LAUNCH(e, KC_LEVEL, (lvg::k_level<false, false, false>), dim3(e->level_grid), dim3(LV_T), 0, s, GNOC_LEVEL_ARGS(l));
         }
         else if (e->nb)
         {
            if (stamps) GNOC_LAUNCH(e, KC_LEVEL, (k_level<true, false, true>), dim3(e->level_grid), dim3(LV_T), 0, s, GNOC_LEVEL_ARGS(l));
            else GNOC_LAUNCH(e, KC_LEVEL, (k_level<false, false, true>), dim3(e->level_grid), dim3(LV_T), 0, s, GNOC_LEVEL_ARGS(l));
         }
         else if (stamps) GNOC_LAUNCH(e, KC_LEVEL, (k_level<true, false, false>), dim3(e->level_grid), dim3(LV_T), 0, s, GNOC_LEVEL_ARGS(l));
         else GNOC_LAUNCH(e, KC_LEVEL, (k_level<false, false, false>), dim3(e->level_grid), dim3(LV_T), 0, s, GNOC_LEVEL_ARGS(l));
      }
   }
#undef GNOC_LEVEL_ARGS
   return GNOC_OK;
}

// The injection level of a one-engine unicast chain run: k_inj_stream.  The stream
// also writes the chain ports' IN_LOCAL window bounds, and nothing is queued behind
// it -- a decline flags the X chains (errflag[4], so every later kernel of the run
// returns at once) and the host reruns the batch with the injection level on k_level
// (inj_declined).
static ChainArgs chain_args(gnoc_engine* e, int phase);
static int inj_level(gnoc_engine* e)
{
   const bool chain_bounds = true;
   const char* v = std::getenv("GNOC_INJ_STREAM");
   if ((v && *v && std::atoi(v) == 0) || e->nb || e->nranks > 1 || e->inj_declined)
      return run_levels_v3(e, 0, 1);
   {
      const int zr = zq_flush(e, e->stream);
      if (zr) return zr;
   }
   hipStream_t s = e->stream;
   const uint32_t N = e->dc.N;
   // the chain ports' IN_LOCAL window bounds in the same pass (chain_phase's X launch
   // then bounds only what a decline left), when every chain fits its LDS table
   const ChainWin *cwx = nullptr, *cwy = nullptr;
   uint32_t *btx = nullptr, *bty = nullptr;
   e->inj_bnd = 0;
   const char* bv = std::getenv("GNOC_INJ_BOUNDS");
   if (chain_bounds && !(bv && *bv && std::atoi(bv) == 0) && e->ncpx && e->ry0 == 0 && e->cx0 == 0)
   {
      bool fit = true;
      for (int p = 0; p < 2; p++)
         for (const ChainWin& w : e->h_cw[p]) fit = fit && w.nW + 1 <= ch::IJ_NWB;
      if (fit)
      {
         const ChainArgs ax = chain_args(e, 0);
         cwx = ax.cw;
         btx = const_cast<uint32_t*>(ax.bt);
         if (e->ncpy)
         {
            const ChainArgs ay = chain_args(e, 1);
            cwy = ay.cw;
            bty = const_cast<uint32_t*>(ay.bt);
         }
         e->inj_bnd = 1;
      }
   }
#define GNOC_INJS(F1V)                                                                                               \
   GNOC_LAUNCH(e, KC_INJ, ch::k_inj_stream<F1V>, dim3(N), dim3(ch::IJ_T), 0, s, e->dc, e->slot_cnt.as<uint32_t>(),  \
               e->slot_base.as<uint64_t>(), e->recs.as<Rec>(), e->samp_t.as<uint64_t>(), e->samp_id.as<uint32_t>(),  \
               e->port_sum.as<unsigned long long>(), e->port_cnt.as<unsigned long long>(),                          \
               e->port_flit.as<unsigned long long>(), e->port_last.as<unsigned long long>(),                        \
               e->counters.as<unsigned>() + 8, cwx, btx, cwy, bty, (uint32_t) chain_bounds,                         \
               (const uint32_t*) e->ch_wt.as<uint32_t>(), (const uint32_t*) e->ch_wt.as<uint32_t>(), e->ch_qs)
   if (e->f1) GNOC_INJS(true);
   else GNOC_INJS(false);
#undef GNOC_INJS
   e->inj_host = 1;
   return GNOC_OK;
}

// The SELF level, on k_level's chunks.
static int self_level(gnoc_engine* e)
{
   const uint32_t L = (uint32_t) e->lvl_off.size() - 1;
   return run_levels_v3(e, L - 1, L);
}

constexpr int GNOC_V3_RETRY = 1000;
constexpr int GNOC_CH_RETRY = 1001;      // a chain window overflowed LDS: smaller windows
constexpr int GNOC_CH_FALLBACK = 1002;   // the chain engine cannot take this batch: level engine
constexpr int GNOC_CH_EXC = 1003;        // only the injection level's exception tails: merge them, rerun
constexpr int GNOC_CH_YFALL = 1004;      // only the Y chains declined: Y and SELF levels on k_level
constexpr int GNOC_INJ_DECLINE = 1007;   // the streamed injection level declined: rerun with it on k_level
constexpr int GNOC_CH_MG = 1005;         // the chains met the M/G/1 branch: rerun on the MG instantiation
constexpr int GNOC_CH_XCDOFF = 1008;     // an XCD got none of a chain launch's workgroups: rerun on one shared queue
constexpr size_t CH_CTR_BYTES = 4096;

// ---------------------------------------------------------------------------
// v4: chain engine for the X and Y phases (chain.hip); INJ and SELF levels on k_level
// ---------------------------------------------------------------------------
static bool chain_usable(const gnoc_engine* e)
{
   const char* env = std::getenv("GNOC_ENGINE");
   if (env && (std::strcmp(env, "levels") == 0 || std::strcmp(env, "v1") == 0)) return false;
   return e->ch_on && !e->nb && !e->force_levels && !e->ch_declined && !e->force_v1 && !e->dc.hop_counter &&
          e->dc.max_list >= 3 && (e->dc.W > 1 || e->dc.H > 1) && e->rec_bound < (1ull << 32);   // u32 record indices
}

// Chain descriptors, state buffers, epoch.  After run_plan_v3 (slot layout known).
static int chain_setup(gnoc_engine* e)
{
   const DevCfg& c = e->dc;
   hipStream_t s = e->stream;
   const uint32_t W = c.W, H = c.H;
   e->ncpx = W > 1 ? 2 * (e->ry1 - e->ry0) * (W - 1) : 0;
   e->ncpy = H > 1 ? 2 * (e->cx1 - e->cx0) * (H - 1) : 0;
   const uint32_t ncp = e->ncpx + e->ncpy;
   GNOC_HIP(e, e->ch_cp.ensure((size_t) std::max<uint32_t>(ncp, 1) * sizeof(ChainPort)));
   int rc = chain_tables(e);
   if (rc) return rc;
   // window bounds and hand-off state: the X phase's, then the Y phase's
   GNOC_HIP(e, e->ch_bt.ensure((e->ch_bt_words[0] + e->ch_bt_words[1] + 1) * 4));
   // [0, 1] dequeue heads; XCD-local queues' heads and exit counts from word 64 (X) / 512 (Y)
   GNOC_HIP(e, e->ch_ctr.ensure(CH_CTR_BYTES));
   // per chain fill maxima, away from the flag word every hand-off poll reads (task-end
   // atomics next to it slowed the polls by half)
   // (then per chain the M/G/1 window bound, k_chain mgk)
   const size_t nmx = 3 * (e->h_cw[0].size() + e->h_cw[1].size());
   GNOC_HIP(e, e->ch_nmax.ensure(std::max<size_t>(nmx, 1) * 4));
   e->zq.push_back({ e->ch_nmax.p, (uint64_t) std::max<size_t>(nmx, 1) * 4 });   // (zq_flush: before the INJ level)
   const size_t stb = (e->ch_st_words[0] + e->ch_st_words[1] + ch::SW) * 8;
   const bool fresh = e->ch_st.bytes < stb;
   GNOC_HIP(e, e->ch_st.ensure(stb));
   // hand-off granules carry a 16-bit epoch: a new epoch per attempt, the buffer
   // zeroed when it is new or the epoch wraps
   e->ch_epoch = (e->ch_epoch + 1) & 0xFFFFu;
   if (fresh || e->ch_epoch == 0)
   {
      GNOC_HIP(e, hipMemsetAsync(e->ch_st.p, 0, e->ch_st.bytes, s));
      if (e->ch_epoch == 0) e->ch_epoch = 1;
   }
   e->zq.push_back({ e->ch_ctr.p, CH_CTR_BYTES });
   // The hand-off protocol per phase.  GNOC_CHAIN_LOOKBACK=0/1 forces one.  Otherwise,
   // once the windows have settled (this attempt's windows are the previous attempt's),
   // each protocol is timed once on them, the phases as separate launches (the trial
   // runs), and the decision is kept for the batch until its windows change again:
   // serial unless look-back is faster by more than CH_LB_MARGIN, so near-equal times
   // (configs[1]'s uniform X phase) keep the serial protocol in every process.  Until a
   // decision exists, serial.
   const char* lbv = std::getenv("GNOC_CHAIN_LOOKBACK");
   const std::vector<uint64_t> wkey[2] = { win_key(e, 0), win_key(e, 1) };
   const bool settled = wkey[0] == e->ch_prevD[0] && wkey[1] == e->ch_prevD[1];
   e->ch_prevD[0] = wkey[0];
   e->ch_prevD[1] = wkey[1];
   e->ch_trial = 0;
   for (int p = 0; p < 2; p++)
   {
      if (!e->ch_ev[p][0]) GNOC_HIP(e, hipEventCreate(&e->ch_ev[p][0]));
      if (!e->ch_ev[p][1]) GNOC_HIP(e, hipEventCreate(&e->ch_ev[p][1]));
      if (e->ch_lb_D[p] != wkey[p])
      {
         e->ch_lb_D[p] = wkey[p];
         e->ch_lb_ms[p][0] = e->ch_lb_ms[p][1] = -1.f;
      }
      const float* m = e->ch_lb_ms[p];
      if (m[0] >= 0 && m[1] >= 0) e->ch_lb_dec[p] = m[1] < (1.f - CH_LB_MARGIN) * m[0] ? 1 : 0;
      const bool trial = settled && (m[0] < 0 || m[1] < 0);
      e->ch_trial |= trial;
      e->ch_lb_run[p] = lbv && *lbv ? (uint32_t) (std::atoi(lbv) != 0)
                                    : trial ? (m[0] < 0 ? 0u : 1u) : (e->ch_lb_dec[p] > 0 ? 1u : 0u);
   }
   if (lbv && *lbv) e->ch_trial = 0;
   if (ncp)
      GNOC_LAUNCH(e, KC_PLAN, ch::k_chain_plan, dim3((ncp + 255) / 256), dim3(256), 0, s, c, e->ncpx, e->ncpy, e->ry0,
                  e->cx0, e->slot_cnt.as<uint32_t>(), e->slot_base.as<uint64_t>(), e->ch_cp.as<ChainPort>());
   return GNOC_OK;
}

// The kernel arguments of one phase: 0 = X (rows of this rank), 1 = Y (columns of
// this rank).
static ChainArgs chain_args(gnoc_engine* e, int phase)
{
   const DevCfg& c = e->dc;
   const uint32_t ncp = phase ? e->ncpy : e->ncpx;
   const uint32_t len = phase ? c.H - 1 : c.W - 1;
   ChainArgs a{};
   a.c = c;
   a.cp = e->ch_cp.as<ChainPort>() + (phase ? e->ncpx : 0);
   a.bt = e->ch_bt.as<uint32_t>() + (phase ? e->ch_bt_words[0] : 0);
   a.recs = e->recs.as<Rec>();
   a.samp_t = e->samp_t.as<uint64_t>();
   a.samp_id = e->samp_id.as<uint32_t>();
   a.st = e->ch_st.as<uint64_t>() + (phase ? e->ch_st_words[0] : 0);
   a.port_sum = e->port_sum.as<unsigned long long>();
   a.port_cnt = e->port_cnt.as<unsigned long long>();
   a.port_flit = e->port_flit.as<unsigned long long>();
   a.port_last = e->port_last.as<unsigned long long>();
   a.errflag = e->counters.as<unsigned>() + 8;
   a.ctr = e->ch_ctr.as<unsigned>() + phase;
   a.nch = len ? ncp / len : 0;
   a.len = len;
   a.ntasks = (uint32_t) e->h_tasks[phase].size();
   a.pad2 = 0;
   a.cw = e->ch_cw.as<ChainWin>() + (phase ? e->h_cw[0].size() : 0);
   a.tasks = e->ch_tasks.as<uint32_t>() + (phase ? e->h_tasks[0].size() : 0);
   a.cp0 = 0;
   a.nmax = e->ch_nmax.as<unsigned>() + (phase ? 2 * e->h_cw[0].size() : 0);
   a.mgk = e->ch_nmax.as<unsigned>() + 2 * (e->h_cw[0].size() + e->h_cw[1].size()) + (phase ? e->h_cw[0].size() : 0);
   a.excfix = (uint32_t) e->exc_fix;
   a.etag = (uint64_t) e->ch_epoch << 48;
   a.stamps = nullptr;
   a.lookback = e->ch_lb_run[phase];
   a.fw = phase ? 5u : 4u;
   a.nexc = e->nexc.as<uint32_t>();
   a.port_mg1 = e->port_mg1.as<unsigned long long>();
   a.xcd = (uint32_t) e->ch_xcd_tab;
   a.qoff = e->ch_tasks.as<uint32_t>() + e->h_tasks[0].size() + e->h_tasks[1].size() + phase * (ch::NQ + 1);
   a.qctr = e->ch_ctr.as<unsigned>() + (phase ? 512 : 64);
   a.qs = e->ch_qs;
   a.wt = e->ch_wt.as<uint32_t>();
   a.wfill = e->ch_wfill.as<uint32_t>();
   // the Y phase runs after k_exc_merge put the X phase's exception tails (M/G/1-served
   // turns, chain.hip mg_emit) in order
   if (phase && e->dc.analytical) a.excfix = 1;
   return a;
}

// One phase as its own launch.
static int chain_phase(gnoc_engine* e, int phase)
{
   {
      const int zr = zq_flush(e, e->stream);
      if (zr) return zr;
   }
   hipStream_t s = e->stream;
   const uint32_t ncp = phase ? e->ncpy : e->ncpx;
   if (!ncp) return GNOC_OK;
   ChainArgs a = chain_args(e, phase);
   const uint32_t nl = phase ? 3u : 1u;
   // The Y ports' IN_LOCAL lists are injection outputs, complete with the X phase's
   // inserts: one-engine runs bound them beside the X lists, the Y launch then only
   // its IN_W / IN_E lists (the X phase's turns)
   const bool ylocal = e->nranks <= 1 && e->ncpy;
   // (the IN_LOCAL lists' bounds: already written by k_inj_stream, whose decline
   // stops the run)
   const bool ibnd = e->inj_bnd && e->inj_host;
   const unsigned* icond = nullptr;
   if ((phase == 0 && !ibnd) || (phase == 1 && !e->ch_ylocal))
      GNOC_LAUNCH(e, KC_BOUNDS, ch::k_win_bounds, dim3(ncp * nl), dim3(256), 0, s, a.cp, nl, a.len, a.cw, e->recs.as<Rec>(),
                  e->samp_t.as<uint64_t>(), const_cast<uint32_t*>(a.bt), nl, 0u, phase == 0 ? icond : nullptr, a.wt, a.qs);
   else if (phase == 1)
      GNOC_LAUNCH(e, KC_BOUNDS, ch::k_win_bounds, dim3(ncp * 2), dim3(256), 0, s, a.cp, nl, a.len, a.cw, e->recs.as<Rec>(),
                  e->samp_t.as<uint64_t>(), const_cast<uint32_t*>(a.bt), 2u, 1u, (const unsigned*) nullptr, a.wt, a.qs);
   if (phase == 0)
   {
      if (ylocal)
      {
         const ChainArgs ay = chain_args(e, 1);
         if (!ibnd)
            GNOC_LAUNCH(e, KC_BOUNDS, ch::k_win_bounds, dim3(e->ncpy), dim3(256), 0, s, ay.cp, 3u, ay.len, ay.cw,
                        e->recs.as<Rec>(), e->samp_t.as<uint64_t>(), const_cast<uint32_t*>(ay.bt), 1u, 0u, icond, ay.wt, ay.qs);
         e->ch_ylocal = 1;
      }
   }
   const char* stv = std::getenv("GNOC_STAMPS");
   if (stv && *stv == '1')
   {
      const size_t nst = (size_t) a.ntasks * a.len * 16;
      DevBuf& sb = phase ? e->ch_stamps1 : e->ch_stamps0;
      GNOC_HIP(e, sb.ensure(nst * 8));
      GNOC_HIP(e, hipMemsetAsync(sb.p, 0, nst * 8, s));
      a.stamps = sb.as<uint64_t>();
   }
   const uint32_t grid = (uint32_t) std::min<uint64_t>((uint64_t) e->ch_grid, (uint64_t) a.ntasks);
   GNOC_HIP(e, hipEventRecord(e->ch_ev[phase][0], s));
   // an MG batch whose M/G/1 windows are known for these windows: only those tasks take
   // the MG path (each chain's first windows), the rest of the phase the common one, in
   // one launch (k_chain_mix)
   const std::vector<uint32_t>& mk = e->h_mgk[phase];
   const bool split = e->ch_mg && e->mgk_ok && e->mgk_D[phase] == win_key(e, phase) && !a.stamps && e->nranks <= 1 &&
                      mk.size() == (size_t) a.nch && !std::getenv("GNOC_MG_SPLIT_OFF");
   if (split)
   {
      std::vector<uint32_t>& lim = e->h_tasks2[phase];   // (kept: the source of an async copy)
      lim.assign(mk.begin(), mk.end());
      for (uint32_t& v : lim) v = std::max(1u, v);
      const size_t off = phase ? e->h_cw[0].size() : 0;
      GNOC_HIP(e, e->ch_tasks2.ensure((e->h_cw[0].size() + e->h_cw[1].size()) * 4 + 4));
      if (e->up_mgk[phase] != lim || e->up_p[phase] != e->ch_tasks2.p)
      {
         GNOC_HIP(e, hipMemcpyAsync(e->ch_tasks2.as<uint32_t>() + off, lim.data(), lim.size() * 4, hipMemcpyHostToDevice, s));
         e->up_mgk[phase] = lim;
         e->up_p[phase] = e->ch_tasks2.p;
      }
      a.mgk_lim = e->ch_tasks2.as<uint32_t>() + off;
#define GNOC_CHAIN_MIX(NLV, F1V)                                                                                  \
   do                                                                                                             \
   {                                                                                                              \
      if (a.lookback) GNOC_LAUNCH(e, KC_CHAIN, (ch::k_chain_mix<NLV, F1V, true>), dim3(grid), dim3(ch::T), 0, s, a); \
      else GNOC_LAUNCH(e, KC_CHAIN, (ch::k_chain_mix<NLV, F1V, false>), dim3(grid), dim3(ch::T), 0, s, a);        \
   } while (0)
      if (phase && e->f1) GNOC_CHAIN_MIX(3, true);
      else if (phase) GNOC_CHAIN_MIX(3, false);
      else if (e->f1) GNOC_CHAIN_MIX(1, true);
      else GNOC_CHAIN_MIX(1, false);
#undef GNOC_CHAIN_MIX
      e->ch_split |= 1 << phase;
      GNOC_HIP(e, hipEventRecord(e->ch_ev[phase][1], s));
      return GNOC_OK;
   }
   // f != 1 GHz: the copy with the reference's double ps <-> cycle conversions
   // (ch_mg: the batch's chains met the no-gap M/G/1 branch; the instantiation with
   // the serial path, whose register allocation the common one does not pay for)
#define GNOC_CHAIN(NLV, F1V)                                                                                         \
   do                                                                                                                 \
   {                                                                                                                  \
      if (e->ch_mg && a.lookback) GNOC_LAUNCH(e, KC_CHAIN, (ch::k_chain<NLV, F1V, true, true>), dim3(grid), dim3(ch::T), 0, s, a); \
      else if (e->ch_mg) GNOC_LAUNCH(e, KC_CHAIN, (ch::k_chain<NLV, F1V, false, true>), dim3(grid), dim3(ch::T), 0, s, a); \
      else if (a.lookback) GNOC_LAUNCH(e, KC_CHAIN, (ch::k_chain<NLV, F1V, true>), dim3(grid), dim3(ch::T), 0, s, a); \
      else GNOC_LAUNCH(e, KC_CHAIN, (ch::k_chain<NLV, F1V, false>), dim3(grid), dim3(ch::T), 0, s, a);                \
   } while (0)
   if (phase && e->f1) GNOC_CHAIN(3, true);
   else if (phase) GNOC_CHAIN(3, false);
   else if (e->f1) GNOC_CHAIN(1, true);
   else GNOC_CHAIN(1, false);
#undef GNOC_CHAIN
   GNOC_HIP(e, hipEventRecord(e->ch_ev[phase][1], s));
   return GNOC_OK;
}

static int run_post(gnoc_engine* e, bool closed_form);
static int run_post_enqueue(gnoc_engine* e, bool closed_form);
static int run_post_check(gnoc_engine* e, bool closed_form);

// Zero the queued buffers (e->zq) in one launch.
static int zq_flush(gnoc_engine* e, hipStream_t s)
{
   while (!e->zq.empty())
   {
      ZeroSegs z{};
      uint32_t ns = 0;
      uint64_t mx = 0;
      while (!e->zq.empty() && ns < (uint32_t) ZSEG)
      {
         z.p[ns] = (uint32_t*) e->zq.back().first;
         z.nw[ns] = e->zq.back().second / 4;
         mx = std::max(mx, z.nw[ns]);
         ns++;
         e->zq.pop_back();
      }
      const uint32_t gx = (uint32_t) std::max<uint64_t>(1, std::min<uint64_t>((mx + 255) / 256, 512));
      GNOC_LAUNCH(e, KC_PLAN, k_zero_segs, dim3(gx, ns), dim3(256), 0, s, z, 0u);
   }
   return GNOC_OK;
}

// The injection level's exception tails into (t, id) order (chain.hip k_exc_merge)
static int exc_merge(gnoc_engine* e)
{
   const uint32_t nslots = e->dc.N * PORTS * INS;
   const uint32_t wins = (nslots + ch::XS - 1) / ch::XS;
   GNOC_LAUNCH(e, KC_BOUNDS, ch::k_exc_merge, dim3(std::max(1u, std::min(wins, 2048u))), dim3(ch::XT), 0, e->stream, nslots,
               e->slot_cnt.as<uint32_t>(), e->slot_base.as<uint64_t>(), e->nexc.as<uint32_t>(), e->recs.as<Rec>(),
               e->samp_t.as<uint64_t>(), e->samp_id.as<uint32_t>(), e->counters.as<unsigned>() + 8);
   return GNOC_OK;
}

// Phase 1 of a run: per-run buffers, classification, injection-slot layout,
// stable scatter, closed-form slot counts and bases.  Queue models disabled
// (router_model.cc:86): the closed form finishes the run here (*done = true).
static int run_prep(gnoc_engine* e, bool* done)
{
   *done = false;
   e->inj_bnd = 0;
   e->inj_host = 0;
   if (!e->submitted) return fail(e, GNOC_ESTATE, "gnoc_run before gnoc_submit");
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   const DevCfg& c = e->dc;
   const size_t n = e->n;
   const uint32_t N = c.N, W = c.W, H = c.H;
   const uint32_t nslots = N * PORTS * INS;
   const size_t nports = (size_t) N * PORTS;
   hipStream_t s = e->stream;
   const uint32_t pch = prep_chunk(N);
   const uint32_t nch = (uint32_t) std::max<uint64_t>(1, (n + pch - 1) / pch);
   int nbits = 0;
   while ((1u << nbits) < N) nbits++;
   // Sharded runs prepare only this rank's share: the injection slots and X-leg
   // counts of its row band [pr0, pr1), and (counted in k_classify) the Y-leg and
   // turn-slot counts of its column band.  Meshes over 64 on a side prepare everything.
   const bool band_prep = e->nranks > 1 && W <= 64 && H <= 64;
   const uint32_t pr0 = band_prep ? e->ry0 : 0u, pr1 = band_prep ? e->ry1 : H, nR = pr1 - pr0;
   const uint32_t nC = e->cx1 - e->cx0;
   // row-histogram grouping: ~512 workgroups, LDS per group <= 32 KiB of source bins
   uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>(W, 512 / nR));
   while (G < W && (W / G + 1) * W * 3 > 8192) G++;
   const int pp_lds = N <= 8192;
   size_t rh_lds = (size_t) ((W + G - 1) / G) * W * 3 * 4 + (pp_lds ? (size_t) N * 4 : 0);

   GNOC_HIP(e, e->aux.ensure(n * 4 + 4));
   GNOC_HIP(e, e->routed.ensure(n + 4));
   GNOC_HIP(e, e->final_ps.ensure(n * 8 + 8));
   GNOC_HIP(e, e->zl.ensure(n * 8 + 8));
   GNOC_HIP(e, e->cont.ensure(n * 8 + 8));
   GNOC_HIP(e, e->hist.ensure((size_t) nch * N * 4));
   GNOC_HIP(e, e->tot.ensure((size_t) N * 4));
   GNOC_HIP(e, e->slot_cnt.ensure((size_t) nslots * 4));
   GNOC_HIP(e, e->slot_base.ensure(((size_t) nslots + 1) * 8));
   GNOC_HIP(e, e->counters.ensure(128));
   GNOC_HIP(e, e->gtot.ensure(16));
   GNOC_HIP(e, e->recs.ensure(e->rec_bound * sizeof(Rec)));
   // the slot layout's bound (k_scan_slots empties the mesh slots past it);
   // GNOC_TEST_LAYOUT_BOUND lowers it to exercise that guard
   e->layout_bound = e->rec_bound;
   if (const char* lb = std::getenv("GNOC_TEST_LAYOUT_BOUND"))
      if (*lb) e->layout_bound = std::min<uint64_t>(e->rec_bound, std::strtoull(lb, nullptr, 10));
   GNOC_HIP(e, e->samp_t.ensure((e->rec_bound / 64 + 1) * 8));
   GNOC_HIP(e, e->samp_id.ensure((e->rec_bound / 64 + 1) * 4));
   GNOC_HIP(e, e->Hs.ensure((size_t) N * W * 3 * 4));
   GNOC_HIP(e, e->Pp.ensure((size_t) H * G * N * 4));
   GNOC_HIP(e, e->Prow.ensure((size_t) H * N * 4));
   GNOC_HIP(e, e->nexc.ensure((size_t) nslots * 4));
   GNOC_HIP(e, e->port_sum.ensure(nports * 8));
   GNOC_HIP(e, e->port_cnt.ensure(nports * 8));
   GNOC_HIP(e, e->port_mg1.ensure(nports * 8));
   GNOC_HIP(e, e->port_flit.ensure(nports * 8));
   GNOC_HIP(e, e->port_last.ensure(nports * 8));
   if (band_prep) GNOC_HIP(e, e->pcol.ensure((size_t) nC * H * H * 3 * 4));

   e->evused = 0;
   e->evkid.clear();
   e->zq.clear();
   GNOC_HIP(e, hipEventRecord(e->ev0, s));
   {
      // counters; slot and exception counts; port counters (and the prefix tables the
      // prep kernels accumulate into): one launch.  Broadcast children live in the
      // exception tails of their slots (level.hip lv_bcast): with broadcasts every
      // level reads the tail counts (errflag word 2 = counter word 10 starts at 1)
      ZeroSegs z{};
      uint32_t ns = 0;
      uint64_t mx = 0;
      bool zover = false;   // ZeroSegs holds ZSEG segments: one more per-run buffer belongs in zq
      auto seg = [&](void* p, uint64_t bytes) {
         if (ns >= (uint32_t) ZSEG)
         {
            zover = true;
            return;
         }
         z.p[ns] = (uint32_t*) p;
         z.nw[ns] = bytes / 4;
         mx = std::max(mx, bytes / 4);
         ns++;
      };
      seg(e->counters.p, 128);
      seg(e->slot_cnt.p, (uint64_t) nslots * 4);
      seg(e->nexc.p, (uint64_t) nslots * 4);
      seg(e->port_sum.p, nports * 8);
      seg(e->port_cnt.p, nports * 8);
      seg(e->port_mg1.p, nports * 8);
      seg(e->port_flit.p, nports * 8);
      seg(e->port_last.p, nports * 8);
      if (!pp_lds) seg(e->Pp.p, (uint64_t) H * G * N * 4);
      if (band_prep) seg(e->pcol.p, (uint64_t) nC * H * H * 3 * 4);
      if (zover) return fail(e, GNOC_EHIP, "internal: more per-run zero segments than ZeroSegs holds");
      const uint32_t gx = (uint32_t) std::max<uint64_t>(1, std::min<uint64_t>((mx + 255) / 256, 512));
      GNOC_LAUNCH(e, KC_CLASSIFY, k_zero_segs, dim3(gx, ns), dim3(256), 0, s, z, e->nb ? 1u : 0u);
   }

   // always launched: for an empty batch it writes the all-zero source histogram
   GNOC_LAUNCH(e, KC_CLASSIFY, k_classify, dim3(nch), dim3(256), N * 4, s, c, (uint64_t) n, pch, e->d_inj, e->d_src,
                  e->d_dst, e->d_bits, e->d_flags, e->aux.as<uint32_t>(), e->routed.as<uint8_t>(),
                  e->final_ps.as<uint64_t>(), e->hist.as<uint32_t>(), e->counters.as<unsigned long long>(), pr0, pr1,
                  e->cx0, e->cx1, band_prep ? e->pcol.as<uint32_t>() : nullptr, e->slot_cnt.as<uint32_t>());

   if (!c.contention)
   {
      // Queue models disabled (router_model.cc:86): latency is zero-load; no contention counters.
      int rc = run_post(e, true);
      if (rc) return rc;
      e->h_records = 0;
      e->h_levels = 0;
      e->used_v3 = 0;
      *done = true;
      return GNOC_OK;
   }

   const uint32_t ng = (N + 255) / 256;
   // per-source sums and prefixes over the chunk axis, in SRC_SEGS segments
   const uint32_t nseg = std::min<uint32_t>(SRC_SEGS, nch);
   const uint32_t ngb = (nR * W + 255) / 256;   // this rank's sources [pr0 * W, pr1 * W)
   GNOC_HIP(e, e->srcseg.ensure((size_t) nseg * N * 4));
   if (ngb)
      GNOC_LAUNCH(e, KC_SRC_TOT, k_src_seg, dim3(ngb, nseg), dim3(256), 0, s, N, nch, nseg, e->hist.as<uint32_t>(),
                  e->srcseg.as<uint32_t>(), pr0 * W, pr1 * W);
   GNOC_LAUNCH(e, KC_SRC_TOT, k_src_tot, dim3(ng), dim3(256), 0, s, N, nseg, e->srcseg.as<uint32_t>(),
               e->tot.as<uint32_t>(), pr0 * W, pr1 * W);
   GNOC_LAUNCH(e, KC_INJ_BASE, k_inj_base, dim3(1), dim3(1024), 0, s, N, e->tot.as<uint32_t>(), e->slot_cnt.as<uint32_t>(),
               e->slot_base.as<uint64_t>(), e->gtot.as<uint64_t>());
   if (ngb && N <= SC4_MAXN)   // per-chunk offsets for the scatter kernels (the sort path needs none)
      GNOC_LAUNCH(e, KC_SRC_OFFS, k_src_offs, dim3(ngb, nseg), dim3(256), 0, s, N, nch, nseg, e->hist.as<uint32_t>(),
                  e->srcseg.as<uint32_t>(), e->slot_base.as<uint64_t>(), pr0 * W, pr1 * W);
   if (n && N <= SC4_MAXN)
   {
      const int nw = scatter_waves(N);
      // a sharded rank places only its row band's packets (sources s0 .. s0+S-1):
      // the compacting variant with counters over those sources only
      const uint32_t s0 = band_prep ? pr0 * W : 0u, S = band_prep ? nR * W : N;
      int sbits = 0;
      while ((1u << sbits) < S) sbits++;
#define GNOC_SCATTER(NWV, SP)                                                                                               \
   GNOC_LAUNCH(e, KC_SCATTER, (k_scatter4<NWV, SP>), dim3(nch), dim3(64 * NWV), (size_t) NWV * S * 4 + (SP ? NWV * 2048 : 0), \
               s, (uint64_t) n, pch, N, s0, S, sbits, e->d_src, e->routed.as<uint8_t>(), e->d_inj,                          \
               e->aux.as<uint32_t>(), e->hist.as<uint32_t>(), e->recs.as<Rec>(), e->samp_t.as<uint64_t>(),                  \
               e->samp_id.as<uint32_t>(), e->part ? (const uint32_t*) e->d_gid.as<uint32_t>() : nullptr)
      if (band_prep && S <= 1024) GNOC_SCATTER(8, true);
      else if (band_prep && S <= 2048) GNOC_SCATTER(4, true);
      else if (band_prep) GNOC_SCATTER(2, true);
      else if (nw == 8) GNOC_SCATTER(8, false);
      else GNOC_SCATTER(4, false);
#undef GNOC_SCATTER
   }
   else if (n)
   {
      // large meshes (sweeps): the stable group-by-source as a radix sort of
      // (source, record) pairs, then a coalesced copy into the slots (serial.hip)
      const uint32_t nbk = (uint32_t) ((n + RS_CH - 1) / RS_CH);
      GNOC_HIP(e, e->sc_key.ensure(2 * n * 4 + 8));
      GNOC_HIP(e, e->sc_rec.ensure(2 * n * sizeof(Rec) + 16));
      GNOC_HIP(e, e->sc_hist.ensure(((size_t) RS_BINS * nbk + RS_BINS + N + 8) * 4));
      uint32_t* kA = e->sc_key.as<uint32_t>();
      uint32_t* kB = kA + n;
      Rec* rA = e->sc_rec.as<Rec>();
      Rec* rB = rA + n;
      uint32_t* hist = e->sc_hist.as<uint32_t>();
      uint32_t* dtot = hist + (size_t) RS_BINS * nbk;
      uint32_t* first = dtot + RS_BINS;
      uint32_t* mcnt = first + N;
      const uint32_t grid = (uint32_t) std::min<size_t>((n + 255) / 256, 8192);
      GNOC_LAUNCH(e, KC_SCATTER, k_set_u32, dim3(1), dim3(1), 0, s, mcnt, (uint32_t) n);
      GNOC_LAUNCH(e, KC_SCATTER, k_src_keys, dim3(grid), dim3(256), 0, s, (uint64_t) n, N, e->d_src, e->routed.as<uint8_t>(),
                  e->d_inj, e->aux.as<uint32_t>(), e->part ? (const uint32_t*) e->d_gid.as<uint32_t>() : nullptr, kA, rA);
      for (uint32_t sh = 0; (N >> sh) != 0; sh += 8)   // keys 0 .. N
      {
         GNOC_LAUNCH(e, KC_SCATTER, k_rs_hist<uint32_t>, dim3(nbk), dim3(RS_T), 0, s, (const uint32_t*) mcnt, sh, nbk,
                     (const uint32_t*) kA, hist);
         GNOC_LAUNCH(e, KC_SCATTER, k_rs_offsets, dim3(RS_BINS), dim3(RS_T), 0, s, (const uint32_t*) mcnt, nbk, hist, dtot);
         GNOC_LAUNCH(e, KC_SCATTER, (k_rs_scatter<uint32_t, Rec>), dim3(nbk), dim3(RS_T), 0, s, (const uint32_t*) mcnt, sh,
                     nbk, (const uint32_t*) kA, (const Rec*) rA, (const uint32_t*) hist, (const uint32_t*) dtot, kB, rB);
         std::swap(kA, kB);
         std::swap(rA, rB);
      }
      GNOC_LAUNCH(e, KC_SCATTER, k_src_first, dim3(grid), dim3(256), 0, s, (uint64_t) n, N, (const uint32_t*) kA, first);
      GNOC_LAUNCH(e, KC_SCATTER, k_src_place, dim3(grid), dim3(256), 0, s, (uint64_t) n, N, (const uint32_t*) kA,
                  (const Rec*) rA, (const uint32_t*) first, (const uint64_t*) e->slot_base.as<uint64_t>(), e->recs.as<Rec>(),
                  e->samp_t.as<uint64_t>(), e->samp_id.as<uint32_t>());
   }
   GNOC_LAUNCH(e, KC_ROW_HIST, k_row_hist, dim3(G, nR), dim3(256), rh_lds, s, c, G, e->recs.as<Rec>(),
               e->slot_cnt.as<uint32_t>(), e->slot_base.as<uint64_t>(), e->Hs.as<uint32_t>(), e->Pp.as<uint32_t>(), pp_lds,
               pr0);
   if (!band_prep)
      GNOC_LAUNCH(e, KC_PROW, k_prow, dim3((uint32_t) (((uint64_t) H * N + 255) / 256)), dim3(256), 0, s, N, H, G,
                  e->Pp.as<uint32_t>(), e->Prow.as<uint32_t>());
   if (W <= 64 && H <= 64)
   {
      GNOC_LAUNCH(e, KC_SLOT_COUNTS, k_slot_counts_x, dim3(nR), dim3(256), (size_t) W * W * 4 * 4, s, c,
                  e->Hs.as<uint32_t>(), e->slot_cnt.as<uint32_t>(), pr0);
      if (band_prep)
         GNOC_LAUNCH(e, KC_SLOT_COUNTS, k_slot_counts_y, dim3(nC), dim3(256), (size_t) H * H * 2 * 4, s, c,
                     e->Prow.as<uint32_t>(), e->slot_cnt.as<uint32_t>(), e->cx0, (const uint32_t*) e->pcol.as<uint32_t>());
      else
         GNOC_LAUNCH(e, KC_SLOT_COUNTS, k_slot_counts_y, dim3(W), dim3(256), (size_t) H * H * 2 * 4, s, c,
                     e->Prow.as<uint32_t>(), e->slot_cnt.as<uint32_t>(), 0u, (const uint32_t*) nullptr);
   }
   else
      GNOC_LAUNCH(e, KC_SLOT_COUNTS, k_slot_counts, dim3((N * 5 + 255) / 256), dim3(256), 0, s, c, e->Hs.as<uint32_t>(),
                  e->Prow.as<uint32_t>(), e->slot_cnt.as<uint32_t>());
   if (e->nb)
   {
      GNOC_HIP(e, e->d_bcnt.ensure((size_t) nslots * 4));
      GNOC_HIP(e, hipMemsetAsync(e->d_bcnt.p, 0, (size_t) nslots * 4, s));
      GNOC_LAUNCH(e, KC_BCAST, k_bcast_slots, dim3((uint32_t) (((uint64_t) e->nb * N + 255) / 256)), dim3(256), 0, s, c,
                  e->nb, e->d_bid.as<uint32_t>(), e->d_src, e->routed.as<uint8_t>(), e->slot_cnt.as<uint32_t>(),
                  e->d_bcnt.as<uint32_t>());
   }
   if (N * 25 <= 4 * SCAN_SPAN)
      GNOC_LAUNCH(e, KC_SCAN, k_scan_slots, dim3(1), dim3(1024), 0, s, N, e->slot_cnt.as<uint32_t>(),
                  e->slot_base.as<uint64_t>(), e->gtot.as<uint64_t>(), e->gtot.as<uint64_t>() + 1, (uint64_t) e->layout_bound);
   else
   {
      const uint32_t nq = N * 25, nspan = (nq + SCAN_SPAN - 1) / SCAN_SPAN;
      GNOC_HIP(e, e->span.ensure((size_t) nspan * 8));
      GNOC_LAUNCH(e, KC_SCAN, k_scan_span_sums, dim3(nspan), dim3(256), 0, s, nq, e->slot_cnt.as<uint32_t>(),
                  e->span.as<uint64_t>());
      GNOC_LAUNCH(e, KC_SCAN, k_scan_span_offsets, dim3(1), dim3(1024), 0, s, nspan, e->span.as<uint64_t>(),
                  e->gtot.as<uint64_t>(), e->gtot.as<uint64_t>() + 1);
      GNOC_LAUNCH(e, KC_SCAN, k_scan_span_bases, dim3(nspan), dim3(256), 0, s, nq, e->slot_cnt.as<uint32_t>(),
                  e->span.as<uint64_t>(), e->slot_base.as<uint64_t>(), (const uint64_t*) (e->gtot.as<uint64_t>() + 1),
                  (uint64_t) e->layout_bound);
   }
   return GNOC_OK;
}

// Last phase: per-packet zero-load / contention (packets this rank delivers:
// destination in its column band), end event, counters and flags to the host.
static int run_post_enqueue(gnoc_engine* e, bool closed_form)
{
   const DevCfg& c = e->dc;
   const size_t n = e->n;
   hipStream_t s = e->stream;
   const uint32_t fin_grid = (uint32_t) std::max<size_t>(1, std::min<size_t>((n + 255) / 256, 8192));
   uint32_t* lat = nullptr;
   if (e->want_lat32 && n && !e->nb)
   {
      GNOC_HIP(e, e->lat32.ensure(n * 4));
      lat = e->lat32.as<uint32_t>();
   }
   if (n)
   {
      unsigned* lovf = e->counters.as<unsigned>() + 8 + 6;   // errflag[6]
      const uint32_t* gid_f = e->part ? e->d_gid.as<uint32_t>() : nullptr;   // (final times by global id)
      if (e->f1)
         GNOC_LAUNCH(e, KC_FINALIZE, k_finalize<true>, dim3(fin_grid), dim3(256), 0, s, c, (uint64_t) n, e->d_inj, e->d_src,
                     e->aux.as<uint32_t>(), e->routed.as<uint8_t>(), e->final_ps.as<uint64_t>(), e->zl.as<uint64_t>(),
                     e->cont.as<uint64_t>(), (int) closed_form, e->cx0, e->cx1, lat, lovf, gid_f, e->fin_glob.as<uint64_t>());
      else
         GNOC_LAUNCH(e, KC_FINALIZE, k_finalize<false>, dim3(fin_grid), dim3(256), 0, s, c, (uint64_t) n, e->d_inj,
                     e->d_src, e->aux.as<uint32_t>(), e->routed.as<uint8_t>(), e->final_ps.as<uint64_t>(),
                     e->zl.as<uint64_t>(), e->cont.as<uint64_t>(), (int) closed_form, e->cx0, e->cx1, lat, lovf, gid_f,
                     e->fin_glob.as<uint64_t>());
   }
   e->lat_written = lat != nullptr;
   if (e->nb)
   {
#define GNOC_BFIN(F1V)                                                                                                \
   GNOC_LAUNCH(e, KC_BCAST, k_bcast_final<F1V>, dim3(e->nb), dim3(256), 0, s, c, e->d_bid.as<uint32_t>(), e->d_inj, \
               e->d_src, e->aux.as<uint32_t>(), e->routed.as<uint8_t>(), e->d_bfin.as<uint64_t>(),                  \
               e->d_bzl.as<uint64_t>(), e->d_bct.as<uint64_t>(), e->final_ps.as<uint64_t>(), e->zl.as<uint64_t>(),  \
               e->cont.as<uint64_t>(), (int) closed_form)
      if (e->f1) GNOC_BFIN(true);
      else GNOC_BFIN(false);
#undef GNOC_BFIN
   }
   GNOC_HIP(e, hipEventRecord(e->ev1, s));
   GNOC_HIP(e, hipMemcpyAsync(e->h_pinned, e->counters.p, 24, hipMemcpyDeviceToHost, s));
   GNOC_HIP(e, hipMemcpyAsync(e->h_pinned + 8, e->counters.as<unsigned int>() + 8, 32, hipMemcpyDeviceToHost, s));
   if (!closed_form)
   {
      GNOC_HIP(e, hipMemcpyAsync(e->h_pinned + 3, e->gtot.as<uint64_t>() + 1, 8, hipMemcpyDeviceToHost, s));
      if (e->used_chain)
         GNOC_HIP(e, hipMemcpyAsync(e->h_nmax, e->ch_nmax.p, 12 * (e->h_cw[0].size() + e->h_cw[1].size()),
                                    hipMemcpyDeviceToHost, s));
      // the per-window fills, while the windows adapt (adapt_windows)
      e->ch_wfill_read = 0;
      if (e->used_chain && e->ch_adapt_left > 0 && e->h_wfill && e->h_wt.size() <= e->h_wfill_cap)
      {
         GNOC_HIP(e, hipMemcpyAsync(e->h_wfill, e->ch_wfill.p, e->h_wt.size() * 4, hipMemcpyDeviceToHost, s));
         e->ch_wfill_read = 1;
      }
   }
   return GNOC_OK;
}
// The run's one host sync, then its counters and flags.
static int run_post_check(gnoc_engine* e, bool closed_form)
{
   GNOC_HIP(e, hipStreamSynchronize(e->stream));
   e->h_counters[0] = e->h_pinned[0];
   e->h_counters[1] = e->h_pinned[1];
   float ms = 0;
   GNOC_HIP(e, hipEventElapsedTime(&ms, e->ev0, e->ev1));
   e->last_ms = ms;
   GNOC_HIP(e, prof_collect(e));
   e->lat_ovf = (((const unsigned*) (e->h_pinned + 8))[6] & 1u) != 0;
   if (closed_form)
   {
      e->ran = true;
      return GNOC_OK;
   }
   e->h_records = e->h_counters[0] + e->h_counters[1] + e->h_pinned[2];
   if (e->h_pinned[3] > e->layout_bound) return fail(e, GNOC_EHIP, "internal: slot layout exceeds the record bound");
   const unsigned* ef = (const unsigned*) (e->h_pinned + 8);
   // the streamed injection level declined and stopped the run (inj_level)
   if (e->inj_host && ef[7]) return GNOC_INJ_DECLINE;
   const unsigned errf = ef[0];
   const unsigned cf = ef[4] | ef[5];   // the X phase's and the Y phase's chain flags
   if (e->used_chain && e->ch_trial && !(cf & ch::F_ANY))
   {
      // this run's time of each phase's protocol (chain_setup keeps the faster one)
      for (int p = 0; p < 2; p++)
      {
         float ms = 0;
         if ((p ? e->ncpy && !e->ch_ydeclined : e->ncpx) &&
             hipEventElapsedTime(&ms, e->ch_ev[p][0], e->ch_ev[p][1]) == hipSuccess)
            e->ch_lb_ms[p][e->ch_lb_run[p]] = ms;
      }
      if (std::getenv("GNOC_CHAIN_DEBUG"))
         std::fprintf(stderr, "gnoc: chain protocol X %u (%.3f / %.3f ms)  Y %u (%.3f / %.3f ms)\n", e->ch_lb_run[0],
                      e->ch_lb_ms[0][0], e->ch_lb_ms[0][1], e->ch_lb_run[1], e->ch_lb_ms[1][0], e->ch_lb_ms[1][1]);
   }
   if (e->used_chain && (cf & ch::F_ANY))
   {
      if (std::getenv("GNOC_CHAIN_DEBUG"))
         std::fprintf(stderr, "gnoc: chain engine declined, flags X 0x%x Y 0x%x\n", ef[4], ef[5]);
      if (cf & ch::F_ROUTE)
      {
         char m[96];
         std::snprintf(m, sizeof m, "internal: chain route-count invariant violated (flags 0x%x 0x%x)", ef[4], ef[5]);
         return fail(e, GNOC_EHIP, m);
      }
      e->ch_yflags = ef[5];
      // an XCD-local queue was not served (an XCD without workgroups of the launch): the
      // one shared queue from now on
      if (cf & ch::R_XCD)
      {
         e->ch_xcd_off = 1;
         return GNOC_CH_XCDOFF;
      }
      // Reruns that change how the chains run, each at most once per batch (a rerun
      // meets whatever else declined again, so the other reasons wait for it):
      // the injection level left exception tails -> merge them first ...
      if (!e->exc_fix && e->nranks <= 1 && (ef[4] & ch::R_EXC) && !(ef[2] & 2u)) return GNOC_CH_EXC;
      // ... the no-gap M/G/1 branch -> the instantiation with the serial path (a split
      // run whose common launch met it: the MG instantiation for every window again)
      if (e->ch_split && (cf & ch::R_MG1) && !(cf & ch::F_TIMEOUT) && !(cf & ch::R_MGBAD))
      {
         e->mgk_ok = 0;
         return GNOC_CH_MG;
      }
      if (!e->ch_mg && e->nranks <= 1 && (cf & ch::R_MG1) && !(cf & ch::F_TIMEOUT)) return GNOC_CH_MG;
      // only the Y chains declined, for a reason the level engine takes (the M/G/1
      // branch, a spill range, a hand-off timeout): the X phase's outputs stand
      if (!(ef[4] & ch::F_ANY) && (ef[5] & (ch::F_FALLBACK | ch::F_TIMEOUT)) && !(ef[5] & ch::F_RETRY) && e->nranks <= 1)
         return GNOC_CH_YFALL;
      return (cf & (ch::F_FALLBACK | ch::F_TIMEOUT)) ? GNOC_CH_FALLBACK : GNOC_CH_RETRY;
   }
   // a leaf the splitter could not cut (or a look-back timeout) leaves garbage
   // downstream, so it takes precedence: rerun exactly on the v1 path
   if (errf & 6u)
   {
      if (e->nranks > 1) return fail(e, GNOC_EUNSUPPORTED, "sharded run hit a burst the chunked path cannot split");
      return GNOC_V3_RETRY;
   }
   if (errf & 1u) return fail(e, GNOC_EHIP, "internal: route-count invariant violated");
   if (e->used_chain && e->ch_mg)
   {
      // the windows of each chain that may serve M/G/1 requests (k_chain mgk): the next
      // run of the batch on these windows gives the MG instantiation only those
      const size_t n0 = e->h_cw[0].size(), n1 = e->h_cw[1].size();
      const unsigned* mk = e->h_nmax + 2 * (n0 + n1);
      e->h_mgk[0].assign(mk, mk + n0);
      e->h_mgk[1].assign(mk + n0, mk + n0 + n1);
      e->mgk_D[0] = win_key(e, 0);
      e->mgk_D[1] = win_key(e, 1);
      e->mgk_ok = 1;
   }
   e->ran = true;
   return GNOC_OK;
}
static int run_post(gnoc_engine* e, bool closed_form)
{
   const int rc = run_post_enqueue(e, closed_form);
   return rc ? rc : run_post_check(e, closed_form);
}

static int run_once(gnoc_engine* e)
{
   if (!e) return GNOC_EINVAL;
   bool done = false;
   int rc = run_prep(e, &done);
   if (rc || done) return rc;
   const bool v3 = e->dc.max_list >= 3 && !e->force_v1;
   e->used_v3 = v3;
   e->used_chain = 0;
   if (v3 && chain_usable(e))
   {
      // v4: INJ level, X chains, Y chains, SELF level
      const uint32_t L = (uint32_t) e->lvl_off.size() - 1;
      e->used_chain = 1;
      e->used_v3 = 4;
      e->ch_split = 0;
      e->ch_ylocal = 0;
      rc = run_plan_v3(e, !e->ch_ydeclined);   // (Y on k_level: its levels too)
      if (!rc) rc = chain_setup(e);
      if (!rc) rc = inj_level(e);
      if (!rc && e->exc_fix) rc = exc_merge(e);
      if (!rc) rc = chain_phase(e, 0);
      // turns the X chains served by M/G/1 wait in exception tails: into order first
      // (only the MG instantiation, mg_emit, writes exception tails)
      if (!rc && !e->ch_ydeclined && e->dc.analytical && e->ch_mg) rc = exc_merge(e);
      if (!rc && !e->ch_ydeclined) rc = chain_phase(e, 1);
      const char* xv = std::getenv("GNOC_CHAIN_EXPERIMENT");
      if (!rc && xv && std::atoi(xv))
      {
         // timing experiment (results invalid): stop after the chains
         GNOC_HIP(e, hipEventRecord(e->ev1, e->stream));
         GNOC_HIP(e, hipStreamSynchronize(e->stream));
         float ms = 0;
         GNOC_HIP(e, hipEventElapsedTime(&ms, e->ev0, e->ev1));
         e->last_ms = ms;
         GNOC_HIP(e, prof_collect(e));
         e->ran = true;
         return GNOC_OK;
      }
      // Y phase on the chains, or (this batch's Y chains declined before) on levels
      if (!rc) rc = e->ch_ydeclined ? run_levels_v3(e, e->lvl_y0, L) : self_level(e);
      if (e->ch_ydeclined) e->used_v3 = 5;
   }
   else if (v3)
   {
      rc = run_plan_v3(e);
      if (!rc) rc = run_levels_v3(e, 0, (uint32_t) e->lvl_off.size() - 1);
   }
   else
      rc = run_levels_v1(e);
   if (rc) return rc;
   return run_post(e, false);
}

// After the Y chains declined (GNOC_CH_YFALL): the X phase's outputs and counters
// stand; the Y phase's flags and its ports' counters are cleared, and the Y and
// SELF levels run on k_level (their look-back state is untouched: k_level returned
// at its first check while a chain flag was set).
static int y_levels_rerun(gnoc_engine* e)
{
   hipStream_t s = e->stream;
   GNOC_HIP(e, hipMemsetAsync(e->counters.as<unsigned int>() + 8 + 5, 0, 4, s));
   // the MG instantiation's Y chains may have left exception tails in the SELF slots;
   // every other slot's tails were merged (k_exc_merge) before the Y phase
   if (e->ch_mg)
      GNOC_LAUNCH(e, KC_CHAIN, ch::k_zero_self_nexc, dim3((e->dc.N * INS + 255) / 256), dim3(256), 0, s, e->dc.N,
                  e->nexc.as<uint32_t>());
   const uint32_t np = e->dc.N * PORTS;
   GNOC_LAUNCH(e, KC_CHAIN, ch::k_zero_ports, dim3((np + 255) / 256), dim3(256), 0, s, np,
               (1u << P_UP) | (1u << P_DOWN) | (1u << P_SELF), e->port_sum.as<unsigned long long>(),
               e->port_cnt.as<unsigned long long>(), e->port_mg1.as<unsigned long long>(),
               e->port_flit.as<unsigned long long>(), e->port_last.as<unsigned long long>());
   e->used_chain = 0;
   e->used_v3 = 5;
   int rc = run_plan_v3(e);   // the Y levels' chunks (the chains' plan covered INJ and SELF only)
   if (!rc) rc = run_levels_v3(e, e->lvl_y0, (uint32_t) e->lvl_off.size() - 1);
   if (!rc) rc = run_post(e, false);
   return rc;
}

// ---------------------------------------------------------------------------
// engine path 3: basic queues with a moving average (serial.hip)
// ---------------------------------------------------------------------------
static int run_ma_tb(gnoc_engine* e, uint32_t tb, bool* wider)
{
   *wider = false;
   const DevCfg& c = e->dc;
   const size_t n = e->n;
   const size_t nports = (size_t) c.N * PORTS;
   hipStream_t s = e->stream;
   const uint32_t nlvl = (uint32_t) e->lvl_off.size() - 1;
   uint32_t maxloc = 1;
   for (uint32_t l = 0; l < nlvl; l++) maxloc = std::max(maxloc, e->lvl_off[l + 1] - e->lvl_off[l]);
   const uint32_t nbk = (uint32_t) std::max<size_t>(1, (n + RS_CH - 1) / RS_CH);   // compaction / radix blocks
   GNOC_HIP(e, e->final_ps.ensure(n * 8 + 8));
   GNOC_HIP(e, e->zl.ensure(n * 8 + 8));
   GNOC_HIP(e, e->cont.ensure(n * 8 + 8));
   GNOC_HIP(e, e->ma_t.ensure(n * 8 + 8));
   GNOC_HIP(e, e->ma_key.ensure(n * 8 + 8));
   GNOC_HIP(e, e->ma_key2.ensure(n * 8 + 8));
   GNOC_HIP(e, e->ma_val.ensure(n * 4 + 4));
   GNOC_HIP(e, e->ma_val2.ensure(n * 4 + 4));
   GNOC_HIP(e, e->ma_lo.ensure((size_t) maxloc * 4));
   GNOC_HIP(e, e->ma_hi.ensure((size_t) maxloc * 4));
   GNOC_HIP(e, e->ma_d.ensure(n * 8 + 8));
   GNOC_HIP(e, e->ma_ref.ensure(n * 8 + 8));
   const size_t nsb = (n + MS_CH - 1) / MS_CH + 1;   // scan blocks
   GNOC_HIP(e, e->ma_agg.ensure(nsb * 28 + 64));
   GNOC_HIP(e, e->ma_m.ensure(64));
   GNOC_HIP(e, e->ma_bcnt.ensure(((size_t) nbk + 1) * 4));
   GNOC_HIP(e, e->ma_hist.ensure(((size_t) RS_BINS * nbk + RS_BINS) * 4));
   GNOC_HIP(e, e->counters.ensure(128));
   for (DevBuf* b : { &e->port_sum, &e->port_cnt, &e->port_mg1, &e->port_flit, &e->port_last })
   {
      GNOC_HIP(e, b->ensure(nports * 8));
      GNOC_HIP(e, hipMemsetAsync(b->p, 0, nports * 8, s));
   }
   GNOC_HIP(e, hipMemsetAsync(e->counters.p, 0, 128, s));
   GNOC_HIP(e, hipEventRecord(e->ev0, s));
   const uint32_t grid = (uint32_t) std::max<size_t>(1, std::min<size_t>((n + 255) / 256, 8192));
   unsigned* err = e->counters.as<unsigned>() + 8;
   uint32_t* mcnt = e->ma_m.as<uint32_t>();
   uint32_t* hist = e->ma_hist.as<uint32_t>();
   uint32_t* dtot = hist + (size_t) RS_BINS * nbk;
   if (n)
   {
      hipLaunchKernelGGL(k_ma_init, dim3(grid), dim3(256), 0, s, (uint64_t) n, c.W, e->d_inj, e->d_src, e->d_dst,
                         e->d_flags, e->ma_t.as<uint64_t>(), e->final_ps.as<uint64_t>(), e->zl.as<uint64_t>(),
                         e->cont.as<uint64_t>(), e->counters.as<unsigned long long>());
      GNOC_HIP(e, hipGetLastError());
      for (uint32_t l = 0; l < nlvl; l++)
      {
         const uint32_t k0 = e->lvl_off[l], nloc = e->lvl_off[l + 1] - k0;
         if (!nloc) continue;
         int lb = 0;
         while ((1u << lb) < nloc) lb++;   // port indices < 2^lb
         const uint32_t end_bit = tb + (uint32_t) lb;
         // the level's requests, compacted in packet order, then sorted by (port, t)
         hipLaunchKernelGGL(k_ma_count, dim3(nbk), dim3(RS_T), 0, s, (uint64_t) n, c.W, l, nlvl, e->d_src, e->d_dst,
                            e->d_flags, e->ma_bcnt.as<uint32_t>());
         hipLaunchKernelGGL(k_ma_scan_counts, dim3(1), dim3(1024), 0, s, nbk, e->ma_bcnt.as<uint32_t>(), mcnt);
         hipLaunchKernelGGL(k_ma_keys, dim3(nbk), dim3(RS_T), 0, s, (uint64_t) n, c.W, l, nlvl, k0, tb, e->d_src,
                            e->d_dst, e->d_flags, e->d_port_k.as<uint32_t>(), (const uint64_t*) e->ma_t.as<uint64_t>(),
                            (const uint32_t*) e->ma_bcnt.as<uint32_t>(), e->ma_key.as<uint64_t>(), e->ma_val.as<uint32_t>(),
                            err);
         GNOC_HIP(e, hipGetLastError());
         uint64_t* kA = e->ma_key.as<uint64_t>();
         uint64_t* kB = e->ma_key2.as<uint64_t>();
         uint32_t* vA = e->ma_val.as<uint32_t>();
         uint32_t* vB = e->ma_val2.as<uint32_t>();
         for (uint32_t sh = 0; sh < end_bit; sh += 8)
         {
            hipLaunchKernelGGL(k_rs_hist<uint64_t>, dim3(nbk), dim3(RS_T), 0, s, (const uint32_t*) mcnt, sh, nbk,
                               (const uint64_t*) kA, hist);
            hipLaunchKernelGGL(k_rs_offsets, dim3(RS_BINS), dim3(RS_T), 0, s, (const uint32_t*) mcnt, nbk, hist, dtot);
            hipLaunchKernelGGL((k_rs_scatter<uint64_t, uint32_t>), dim3(nbk), dim3(RS_T), 0, s, (const uint32_t*) mcnt, sh, nbk,
                               (const uint64_t*) kA, (const uint32_t*) vA, (const uint32_t*) hist, (const uint32_t*) dtot,
                               kB, vB);
            std::swap(kA, kB);
            std::swap(vA, vB);
         }
         GNOC_HIP(e, hipGetLastError());
         // sorted requests in (kA, vA); the other pair holds cycles and flits
         GNOC_HIP(e, hipMemsetAsync(e->ma_lo.p, 0, (size_t) nloc * 4, s));
         GNOC_HIP(e, hipMemsetAsync(e->ma_hi.p, 0, (size_t) nloc * 4, s));
         hipLaunchKernelGGL(k_ma_bounds, dim3(grid), dim3(256), 0, s, (const uint32_t*) mcnt, tb, (const uint64_t*) kA,
                            e->ma_lo.as<uint32_t>(), e->ma_hi.as<uint32_t>());
         GNOC_HIP(e, hipGetLastError());
         const uint64_t* skey = kA;
         const uint32_t* sval = vA;
         const uint32_t* lo = e->ma_lo.as<uint32_t>();
         const uint32_t* hi = e->ma_hi.as<uint32_t>();
         const uint32_t* ports = e->d_lvl_ports.as<uint32_t>() + k0;
         uint64_t* tcs = kB;
         uint32_t* Fs = vB;
         uint64_t* ref = e->ma_ref.as<uint64_t>();
#define GNOC_MA_GATHER(MT)                                                                                          \
   hipLaunchKernelGGL(k_ma_gather<MT>, dim3(grid), dim3(256), 0, s, (const uint32_t*) mcnt, tb, c.flit_width, c.f,   \
                      e->ma_window, skey, sval, e->d_bits, lo, tcs, Fs, e->ma_d.as<double>(), ref)
#define GNOC_MA_CHAIN(MT)                                                                                           \
   hipLaunchKernelGGL(k_ma_chain<MT>, dim3(nloc), dim3(64), 0, s, nloc, e->ma_window,                               \
                      (const uint64_t*) tcs, lo, hi, (const double*) e->ma_d.as<double>(), e->ma_ref.as<double>())
         if (e->ma_type == MA_MEDIAN) GNOC_MA_GATHER(MA_MEDIAN);
         else if (e->ma_type == MA_GEOMETRIC) GNOC_MA_GATHER(MA_GEOMETRIC);
         else GNOC_MA_GATHER(MA_ARITHMETIC);
         GNOC_HIP(e, hipGetLastError());
         if (e->ma_type == MA_GEOMETRIC) GNOC_MA_CHAIN(MA_GEOMETRIC);
         else if (e->ma_type == MA_ARITHMETIC) GNOC_MA_CHAIN(MA_ARITHMETIC);
         GNOC_HIP(e, hipGetLastError());
#undef GNOC_MA_GATHER
#undef GNOC_MA_CHAIN
         // the queue: segmented max-plus scan (delays into ma_d, free once the chain ran)
         uint64_t* bA = e->ma_agg.as<uint64_t>();
         uint64_t* bB = bA + nsb;
         uint64_t* qin = bB + nsb;
         uint32_t* bR = reinterpret_cast<uint32_t*>(qin + nsb);
         const uint32_t sgrid = (uint32_t) ((n + MS_CH - 1) / MS_CH);
         uint64_t* dout = e->ma_d.as<uint64_t>();
#define GNOC_MA_SCAN(MT)                                                                                            \
   do                                                                                                               \
   {                                                                                                                \
      hipLaunchKernelGGL(k_ma_scan1<MT>, dim3(sgrid), dim3(MS_T), 0, s, (const uint32_t*) mcnt, tb, skey, lo,       \
                         (const uint64_t*) ref, (const uint32_t*) Fs, bA, bB, bR);                                  \
      hipLaunchKernelGGL(k_ma_scan2, dim3(1), dim3(64), 0, s, (const uint32_t*) mcnt, (const uint64_t*) bA,         \
                         (const uint64_t*) bB, (const uint32_t*) bR, qin);                                          \
      hipLaunchKernelGGL(k_ma_scan3<MT>, dim3(sgrid), dim3(MS_T), 0, s, (const uint32_t*) mcnt, tb, skey, lo, hi,   \
                         ports, (const uint64_t*) ref, (const uint32_t*) Fs, (const uint64_t*) qin, dout,           \
                         e->port_last.as<uint64_t>());                                                              \
   } while (0)
         if (e->ma_type == MA_MEDIAN) GNOC_MA_SCAN(MA_MEDIAN);
         else GNOC_MA_SCAN(MA_ARITHMETIC);   // arithmetic and geometric: ref = (T) mean, the same conversion
#undef GNOC_MA_SCAN
         GNOC_HIP(e, hipGetLastError());
         hipLaunchKernelGGL(k_ma_ports, dim3(nloc, 16), dim3(256), 0, s, ports, lo, hi, (const uint64_t*) dout,
                            (const uint32_t*) Fs, e->port_sum.as<unsigned long long>(),
                            e->port_cnt.as<unsigned long long>(), e->port_flit.as<unsigned long long>());
         GNOC_HIP(e, hipGetLastError());
         hipLaunchKernelGGL(k_ma_apply, dim3(grid), dim3(256), 0, s, (const uint32_t*) mcnt, tb, ports, c.f, c.rl_ps, skey,
                            sval, (const uint32_t*) Fs, (const uint64_t*) dout, e->ma_t.as<uint64_t>(),
                            e->final_ps.as<uint64_t>());
         GNOC_HIP(e, hipGetLastError());
      }
   }
   if (n)
   {
      hipLaunchKernelGGL(k_ma_final, dim3(grid), dim3(256), 0, s, (uint64_t) n, c.W, c.flit_width, c.f, c.rl_ps, e->d_inj,
                         e->d_src, e->d_dst, e->d_bits, e->d_flags, (const uint64_t*) e->final_ps.as<uint64_t>(),
                         e->zl.as<uint64_t>(), e->cont.as<uint64_t>());
      GNOC_HIP(e, hipGetLastError());
   }
   GNOC_HIP(e, hipEventRecord(e->ev1, s));
   GNOC_HIP(e, hipMemcpyAsync(e->h_pinned, e->counters.p, 40, hipMemcpyDeviceToHost, s));
   GNOC_HIP(e, hipStreamSynchronize(s));
   if (*(const unsigned*) (e->h_pinned + 4))
   {
      if (tb < MA_T_BITS)
      {
         *wider = true;
         return GNOC_OK;
      }
      return fail(e, GNOC_EUNSUPPORTED, "packet time beyond 2^49 ps");
   }
   e->h_counters[0] = e->h_pinned[0];
   e->h_counters[1] = e->h_pinned[1];
   e->h_records = e->h_counters[0] + e->h_counters[1];
   e->h_levels = nlvl;
   e->used_v3 = 3;
   float ms = 0;
   GNOC_HIP(e, hipEventElapsedTime(&ms, e->ev0, e->ev1));
   e->last_ms = ms;
   e->ran = true;
   return GNOC_OK;
}

static int run_ma(gnoc_engine* e)
{
   if (!e->submitted) return fail(e, GNOC_ESTATE, "gnoc_run before gnoc_submit");
   if (e->nb) return fail(e, GNOC_EUNSUPPORTED, "broadcast packets with moving-average basic queues");
   // request indices are 32-bit (self-sends and unmodeled packets count too)
   if (e->n > (size_t) INT32_MAX) return fail(e, GNOC_EUNSUPPORTED, "more than 2^31-1 packets on the moving-average path");
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   // 32-bit request times while the batch leaves 2^31 ps of headroom for delays;
   // a request beyond 2^32 ps reruns the batch with 49-bit times
   bool wider = false;
   if (e->h_tlast < (1ull << 31))
   {
      const int rc = run_ma_tb(e, 32, &wider);
      if (rc || !wider) return rc;
   }
   return run_ma_tb(e, MA_T_BITS, &wider);
}

int gnoc_set_basic_moving_average(gnoc_engine* e, int32_t type, uint32_t window_size)
{
   if (!e) return GNOC_EINVAL;
   if (type < GNOC_MOVING_AVG_NONE || type > GNOC_MOVING_AVG_MEDIAN) return fail(e, GNOC_EINVAL, "unknown moving average type");
   if (type != GNOC_MOVING_AVG_NONE && e->cfg.queue_type != GNOC_QUEUE_BASIC)
      return fail(e, GNOC_EINVAL, "moving averages belong to the basic queue model");
   if (type != GNOC_MOVING_AVG_NONE && (window_size < 1 || window_size > (1u << 16)))
      return fail(e, GNOC_EINVAL, "moving_avg_window_size must be in [1, 65536]");
   if (type != GNOC_MOVING_AVG_NONE && (e->nranks > 1 || e->npoints > 1 || e->dc.hop_counter))
      return fail(e, GNOC_EUNSUPPORTED, "moving-average queues run on one unsharded mesh engine");
   // MovingGeometricMean::compute is a chain of pow() calls (moving_average.h:119-135):
   // the engine runs glibc's own pow algorithm and tables (glibc_pow.h), bit-exact.
   e->ma_type = type;
   e->ma_window = type ? window_size : 1;
   e->ran = false;
   return GNOC_OK;
}

static int run_impl(gnoc_engine* e);
int gnoc_run(gnoc_engine* e)
{
   if (!e) return GNOC_EINVAL;
   e->n_retry = e->n_fallback = 0;
   const int rc = run_impl(e);
   e->runs++;
   e->tot_retry += e->n_retry;
   e->tot_fallback += e->n_fallback;
   return rc;
}
static int run_impl(gnoc_engine* e)
{
   if (e->fetched)
   {
      // gnoc_fetch_final_ps is reading the last run's final_ps: this run writes the
      // other buffer, once that buffer's own read-back (two runs ago) has ended
      GNOC_HIP(e, hipSetDevice(e->cfg.device));
      e->final_ps.swap(e->final_alt);
      e->lat32.swap(e->lat32_alt);
      std::swap(e->ev_fin, e->ev_alt);
      GNOC_HIP(e, hipStreamWaitEvent(e->stream, e->ev_fin, 0));
      e->fetched = false;
   }
   if (e->ma_type && e->dc.contention) return run_ma(e);
   if (e->nranks > 1) return fail(e, GNOC_ESTATE, "sharded engine: use gnoc_run_begin / exchange / gnoc_run_finish");
   const char* env = std::getenv("GNOC_ENGINE");
   const int forced = env && std::strcmp(env, "v1") == 0;
   // Broadcast batches run in passes: a router visit of a broadcast charges the
   // max queue delay over the ports it selects (router_model.cc:86-101), and
   // those ports sit on different levels of the port DAG, so a pass charges a
   // visit's ports not yet served this pass their busy-until times of the
   // previous pass.  The event times are the unique causal solution exactly when
   // every visit charged all its children its final max.
   const char* pv = std::getenv("GNOC_BCAST_PASSES");
   const uint32_t max_passes = pv && std::atol(pv) > 0 ? (uint32_t) std::atol(pv) : 256u;
   const size_t nv = (size_t) e->nb * e->dc.N;
   e->bc_passes = 0;
   if (e->nb && e->submitted)
   {
      GNOC_HIP(e, hipSetDevice(e->cfg.device));
      GNOC_HIP(e, hipMemsetAsync(e->d_bv[0].p, 0, nv * 8 * BCS, e->stream));
      e->dc.bc_prev = e->d_bv[0].as<uint64_t>();
      e->dc.bc_cur = e->d_bv[1].as<uint64_t>();
   }
   double ms = 0.0;
   for (;;)
   {
      if (e->nb && e->submitted)
      {
         GNOC_HIP(e, hipMemsetAsync(e->dc.bc_cur, 0, nv * 8 * BCS, e->stream));
      }
      e->force_v1 = forced;
      e->force_levels = 0;
      e->chD_run[0] = e->chD[0];
      e->chD_run[1] = e->chD[1];
      // chain engine: a run that declined only for the injection level's exception tails
      // reruns once with them merged (later runs of the batch merge up front); a window
      // that overflowed LDS reruns with windows half as long (twice as many), up to 3
      // halvings.  Both count as reruns (gnoc_summary.retries); only halvings use up
      // the halving budget.
      int rc = GNOC_OK;
      uint32_t halvings = 0;
      for (;;)
      {
         rc = run_once(e);
         if (rc == GNOC_CH_EXC && !e->exc_fix)
         {
            e->exc_fix = 1;
            e->n_retry++;
            continue;
         }
         if (rc == GNOC_CH_EXC) rc = GNOC_CH_FALLBACK;
         if (rc == GNOC_CH_MG)
         {
            e->ch_mg = 1;
            e->n_retry++;
            continue;
         }
         if (rc == GNOC_INJ_DECLINE)
         {
            e->inj_declined = 1;
            e->n_retry++;
            continue;
         }
         if (rc == GNOC_CH_XCDOFF)
         {
            e->n_retry++;
            continue;
         }
         // halve the windows of the chains that overflowed (all, when none is marked)
         if (rc == GNOC_CH_RETRY && halvings < 3 && halve_overflowed(e, e->chD_run))
         {
            halvings++;
            e->n_retry++;
            continue;
         }
         break;
      }
      if (rc == GNOC_CH_YFALL)
      {
         // only the Y chains declined: the batch's Y and SELF levels run on k_level now.
         // For an M/G/1 request or a spill range (properties of the batch) later runs go
         // there straight after the X chains; a hand-off timeout (a scheduling event)
         // moves this run only.
         e->n_fallback++;
         if (e->ch_yflags & ch::F_FALLBACK) e->ch_ydeclined = 1;
         rc = y_levels_rerun(e);
      }
      if (rc == GNOC_CH_RETRY || rc == GNOC_CH_FALLBACK)
      {
         // the same batch would decline again (deterministic): later runs of it go
         // straight to the level engine (a new submit clears this)
         e->n_fallback++;
         e->force_levels = 1;
         e->ch_declined = 1;
         rc = run_once(e);
      }
      else if (!rc && e->used_chain && halvings)
      {
         // the window sizes that fit: later runs of this batch start with them
         e->chD[0] = e->chD_run[0];
         e->chD[1] = e->chD_run[1];
      }
      else if (!rc && e->used_chain)
         adapt_windows(e);   // the fill this run measured
      if (rc == GNOC_V3_RETRY)
      {
         e->n_fallback++;
         e->force_v1 = 1;   // exact but slower whole-port streams
         rc = run_once(e);
         if (rc == GNOC_V3_RETRY) rc = fail(e, GNOC_EHIP, "internal: v1 path reported overflow");
      }
      e->force_v1 = forced;
      e->force_levels = 0;
      if (rc) return rc;
      ms += e->last_ms;
      e->bc_passes++;
      if (!e->nb || !e->dc.contention) break;
      GNOC_HIP(e, hipMemsetAsync(e->d_bflag.p, 0, 8, e->stream));
      GNOC_HIP(e, hipMemsetAsync(e->d_bflag.as<char>() + 8, 0xFF, 8, e->stream));
      hipLaunchKernelGGL(k_bcast_agree, dim3((uint32_t) std::min<size_t>((nv + 255) / 256, 4096)), dim3(256), 0,
                         e->stream, (uint64_t) nv, (const uint64_t*) e->dc.bc_cur,
                         e->d_bflag.as<unsigned>());
      GNOC_HIP(e, hipGetLastError());
      GNOC_HIP(e, hipMemcpyAsync(e->h_pinned + 6, e->d_bflag.p, 4, hipMemcpyDeviceToHost, e->stream));
      GNOC_HIP(e, hipStreamSynchronize(e->stream));
      if (std::getenv("GNOC_BCAST_DEBUG"))
      {
         unsigned hb[4];
         GNOC_HIP(e, hipMemcpy(hb, e->d_bflag.p, 16, hipMemcpyDeviceToHost));
         std::fprintf(stderr, "bcast pass %u: %.3f ms changed %u min_cycle %llu\n", e->bc_passes, e->last_ms, hb[1],
                      (unsigned long long) (hb[2] | (uint64_t) hb[3] << 32));
         if (const char* dp = std::getenv("GNOC_BCAST_DUMP"))
         {
            // wrong visits of this pass: b, tile, final max, min u, max u, Xb by direction
            std::vector<uint64_t> hu(nv * BCS);
            GNOC_HIP(e, hipMemcpy(hu.data(), e->dc.bc_cur, nv * 8 * BCS, hipMemcpyDeviceToHost));
            FILE* f = std::fopen(dp, e->bc_passes == 1 ? "w" : "a");
            for (size_t k = 0; f && k < nv; k++)
            {
               const uint64_t* r = &hu[k * BCS];
               const uint64_t m = r[BC_M], lo = ~r[BC_UMIN], hi = r[BC_UMAX];
               if (!((m || hi) && (lo != m || hi != m))) continue;
               std::fprintf(f, "%u %zu %zu %llu %llu %llu", e->bc_passes, k / e->dc.N, k % e->dc.N, (unsigned long long) m,
                            (unsigned long long) lo, (unsigned long long) hi);
               for (int d = 0; d < 5; d++) std::fprintf(f, " %llu", (unsigned long long) r[BC_WIN + d * BCW + BCW_B]);
               std::fprintf(f, "\n");
            }
            if (f) std::fclose(f);
         }
      }
      if (!*(unsigned*) (e->h_pinned + 6)) break;
      if (e->bc_passes >= max_passes)
      {
         e->ran = false;
         return fail(e, GNOC_EUNSUPPORTED, "broadcast passes did not converge within " + std::to_string(max_passes) +
                                               " (GNOC_BCAST_PASSES)");
      }
      // this pass's visit records predict the next pass
      uint64_t* const was = const_cast<uint64_t*>(e->dc.bc_prev);
      e->dc.bc_prev = e->dc.bc_cur;
      e->dc.bc_cur = was;
   }
   e->last_ms = ms;
   return GNOC_OK;
}

int gnoc_get_broadcast_results(gnoc_engine* e, uint64_t* final_ps, uint64_t* zero_load_ps, uint64_t* contention_ps,
                               size_t n_entries)
{
   if (!e) return GNOC_EINVAL;
   if (!e->ran) return fail(e, GNOC_ESTATE, "no results: call gnoc_run first");
   const size_t nv = (size_t) e->nb * e->dc.N;
   if (n_entries != nv) return fail(e, GNOC_EINVAL, "broadcast result length != broadcasts x num_tiles");
   if (!nv) return GNOC_OK;
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   if (final_ps) GNOC_HIP(e, hipMemcpyAsync(final_ps, e->d_bfin.p, nv * 8, hipMemcpyDeviceToHost, e->stream));
   if (zero_load_ps) GNOC_HIP(e, hipMemcpyAsync(zero_load_ps, e->d_bzl.p, nv * 8, hipMemcpyDeviceToHost, e->stream));
   if (contention_ps) GNOC_HIP(e, hipMemcpyAsync(contention_ps, e->d_bct.p, nv * 8, hipMemcpyDeviceToHost, e->stream));
   GNOC_HIP(e, hipStreamSynchronize(e->stream));
   return GNOC_OK;
}

int gnoc_get_broadcast_info(const gnoc_engine* e, uint64_t* nbcast, uint32_t* passes)
{
   if (!e) return GNOC_EINVAL;
   if (nbcast) *nbcast = e->nb;
   if (passes) *passes = e->bc_passes;
   return GNOC_OK;
}

// ---------------------------------------------------------------------------
// one mesh over several GPUs (shard.hip)
// ---------------------------------------------------------------------------
int gnoc_shard(gnoc_engine* e, int32_t rank, int32_t nranks)
{
   if (!e) return GNOC_EINVAL;
   if (nranks < 1 || rank < 0 || rank >= nranks) return fail(e, GNOC_EINVAL, "bad rank / nranks");
   if ((uint32_t) nranks > std::min(e->dc.W, e->dc.H)) return fail(e, GNOC_EINVAL, "more ranks than mesh rows or columns");
   if (nranks > 1 && e->npoints > 1) return fail(e, GNOC_EUNSUPPORTED, "a sweep shards by points (one engine per rank)");
   if (nranks > 1 && e->ma_type) return fail(e, GNOC_EUNSUPPORTED, "moving-average queues run on one unsharded mesh engine");
   if (nranks > 1 && e->dc.contention && e->dc.max_list < 3)
      return fail(e, GNOC_EUNSUPPORTED, "sharding needs the chunked path (max_list_size >= 3)");
   e->rank = rank;
   e->nranks = nranks;
   {
      const char* xv = std::getenv("GNOC_SHARD_SELF_EXCHANGE");
      e->xself = xv && *xv && std::atoi(xv) != 0;
   }
   build_static_levels(e);
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   GNOC_HIP(e, upload_levels(e));
   e->submitted = false;
   e->ran = false;
   e->begun = false;
   return GNOC_OK;
}

int gnoc_exchange_counts(gnoc_engine* e, uint64_t* send_units, uint64_t* recv_units, size_t nranks)
{
   if (!e) return GNOC_EINVAL;
   if (!e->submitted) return fail(e, GNOC_ESTATE, "exchange layout is known after gnoc_submit");
   if (nranks != (size_t) e->nranks) return fail(e, GNOC_EINVAL, "nranks != the engine's shard count");
   for (size_t q = 0; q < nranks; q++)
   {
      if (send_units) send_units[q] = q < e->xs_units.size() ? e->xs_units[q] : 0;
      if (recv_units) recv_units[q] = q < e->xr_units.size() ? e->xr_units[q] : 0;
   }
   return GNOC_OK;
}

// ---------------------------------------------------------------------------
// gnoc_run_sharded: begin -> all-to-all (RCCL or the caller's transport) -> finish
// ---------------------------------------------------------------------------
static int rccl_exchange(gnoc_engine* e, const void* send, const uint64_t* su, void* recv, const uint64_t* ru)
{
   ncclComm_t comm = static_cast<ncclComm_t>(e->nccl);
   const int nr = e->nranks;
   // grouped point-to-point: every peer pair is one xGMI transfer (no ring relay)
   if (ncclGroupStart() != ncclSuccess) return fail(e, GNOC_EHIP, "ncclGroupStart");
   uint64_t so = 0, ro = 0;
   const char* bad = nullptr;   // the group is always closed, so the status all-reduce after it runs
   for (int q = 0; q < nr && !bad; q++)
   {
      if (su[q] && ncclSend(static_cast<const char*>(send) + so * 16, su[q] * 16, ncclChar, q, comm, e->stream) != ncclSuccess)
         bad = "ncclSend";
      else if (ru[q] && ncclRecv(static_cast<char*>(recv) + ro * 16, ru[q] * 16, ncclChar, q, comm, e->stream) != ncclSuccess)
         bad = "ncclRecv";
      so += su[q];
      ro += ru[q];
   }
   if (ncclGroupEnd() != ncclSuccess && !bad) bad = "ncclGroupEnd";
   if (bad) return fail(e, GNOC_EHIP, bad);
   return GNOC_OK;   // on the stream: the Y phase that reads the buffer follows in order
}

static int rccl_agree(gnoc_engine* e, int32_t status, int32_t* out)
{
   ncclComm_t comm = static_cast<ncclComm_t>(e->nccl);
   GNOC_HIP(e, e->xflag.ensure(16));
   int32_t* h = reinterpret_cast<int32_t*>(e->h_pinned + 15);
   *h = status;
   GNOC_HIP(e, hipMemcpyAsync(e->xflag.p, h, 4, hipMemcpyHostToDevice, e->stream));
   if (ncclAllReduce(e->xflag.p, e->xflag.p, 1, ncclInt32, ncclMax, comm, e->stream) != ncclSuccess)
      return fail(e, GNOC_EHIP, "ncclAllReduce (status)");
   GNOC_HIP(e, hipMemcpyAsync(h, e->xflag.p, 4, hipMemcpyDeviceToHost, e->stream));
   GNOC_HIP(e, hipStreamSynchronize(e->stream));
   *out = *h;
   return GNOC_OK;
}

// An RCCL communicator for gnoc_shard_set_comm from the library libgnoc itself
// links (so the ncclComm_t handed back is one its ncclSend / ncclRecv accept):
// rank 0 makes the 128-byte unique id, the caller broadcasts it (any channel),
// every rank joins on its device.
int gnoc_rccl_unique_id(void* id128)
{
   if (!id128) return GNOC_EINVAL;
   ncclUniqueId id;
   static_assert(sizeof(ncclUniqueId) == GNOC_RCCL_ID_BYTES, "ncclUniqueId size");
   if (ncclGetUniqueId(&id) != ncclSuccess) return GNOC_EHIP;
   std::memcpy(id128, &id, sizeof id);
   return GNOC_OK;
}

int gnoc_rccl_comm_init(int32_t nranks, int32_t rank, int32_t device, const void* id128, void** comm)
{
   if (!id128 || !comm || nranks < 1 || rank < 0 || rank >= nranks) return GNOC_EINVAL;
   if (hipSetDevice(device) != hipSuccess) return GNOC_EHIP;
   ncclUniqueId id;
   std::memcpy(&id, id128, sizeof id);
   ncclComm_t c = nullptr;
   if (ncclCommInitRank(&c, nranks, id, rank) != ncclSuccess) return GNOC_EHIP;
   *comm = c;
   return GNOC_OK;
}

int gnoc_rccl_comm_destroy(void* comm)
{
   if (!comm) return GNOC_EINVAL;
   return ncclCommDestroy(static_cast<ncclComm_t>(comm)) == ncclSuccess ? GNOC_OK : GNOC_EHIP;
}

int gnoc_shard_set_comm(gnoc_engine* e, void* nccl_comm)
{
   if (!e) return GNOC_EINVAL;
   if (!nccl_comm) return fail(e, GNOC_EINVAL, "null ncclComm_t");
   int nr = 0, rk = 0, dev = -1;
   if (ncclCommCount(static_cast<ncclComm_t>(nccl_comm), &nr) != ncclSuccess ||
       ncclCommUserRank(static_cast<ncclComm_t>(nccl_comm), &rk) != ncclSuccess ||
       ncclCommCuDevice(static_cast<ncclComm_t>(nccl_comm), &dev) != ncclSuccess)
      return fail(e, GNOC_EINVAL, "not a valid ncclComm_t");
   if (nr != e->nranks || rk != e->rank)
      return fail(e, GNOC_EINVAL, "communicator rank / size differ from gnoc_shard's");
   if (dev != e->cfg.device) return fail(e, GNOC_EINVAL, "communicator on another device than the engine's");
   e->nccl = nccl_comm;
   e->tp = gnoc_transport{};
   return GNOC_OK;
}

int gnoc_shard_set_transport(gnoc_engine* e, const gnoc_transport* tp)
{
   if (!e || !tp) return GNOC_EINVAL;
   if (!tp->exchange || !tp->agree) return fail(e, GNOC_EINVAL, "transport needs exchange and agree");
   e->tp = *tp;
   e->nccl = nullptr;
   return GNOC_OK;
}

static int shard_agree(gnoc_engine* e, int rc, const char* what)
{
   int32_t any = 0;
   const int32_t mine = rc ? 1 : 0;
   int trc = e->nccl ? rccl_agree(e, mine, &any) : (e->tp.agree(e->tp.ctx, mine, &any) ? GNOC_EHIP : GNOC_OK);
   if (trc) return rc ? rc : (e->nccl ? trc : fail(e, GNOC_EHIP, std::string("transport agree failed after ") + what));
   if (rc) return rc;
   if (any) return fail(e, GNOC_EHIP, std::string(what) + " failed on another rank");
   return GNOC_OK;
}

static int begin_x(gnoc_engine* e, void* send_buf, bool sync);
static int finish_enqueue(gnoc_engine* e, const void* recv_buf);
static int finish_check(gnoc_engine* e);

// The synchronous protocol: every phase brackets its outcome with a status
// agreement (a failed rank fails every rank; none waits in a collective a peer
// never joins).  Used by the caller-transport path, and by the RCCL path to rerun a
// step whose stream-path status said a rank's X phase did not complete.
static int run_sharded_sync(gnoc_engine* e, const uint64_t* su, const uint64_t* ru)
{
   int rc = shard_agree(e, begin_x(e, e->xsend.p, true), "gnoc_run_begin");
   if (rc) return rc;
   if (e->nccl)
   {
      rc = rccl_exchange(e, e->xsend.p, su, e->xrecv.p, ru);
      if (!rc) GNOC_HIP(e, hipStreamSynchronize(e->stream));
   }
   else if (e->tp.exchange(e->tp.ctx, e->xsend.p, su, e->xrecv.p, ru, e->stream))
      rc = fail(e, GNOC_EHIP, "transport exchange failed");
   rc = shard_agree(e, rc, "the turn exchange");
   if (rc) return rc;
   return shard_agree(e, gnoc_run_finish(e, e->xrecv.p), "gnoc_run_finish");
}

// The stream path over RCCL: X phase, pack, grouped send / receive, Y phase, the
// status all-reduce and the read-back all go onto the engine's stream, then ONE
// host sync.  Every rank issues the same two collectives whatever happens locally:
// a rank that cannot complete its X phase marks its send buffer's pair status units
// (its peers' Y phases then skip), and the reduced status sends every rank to the
// synchronous protocol for this step.
static int run_sharded_stream(gnoc_engine* e, const uint64_t* su, const uint64_t* ru, uint64_t ns, bool* accounted)
{
   hipStream_t s = e->stream;
   ncclComm_t comm = static_cast<ncclComm_t>(e->nccl);
   int lrc = begin_x(e, e->xsend.p, false);
   if (lrc)
   {
      // the buffer may be unpacked: every pair's status unit reads "failed"
      (void) hipMemsetAsync(e->xsend.p, 0xFF, std::max<uint64_t>(ns, 1) * 16, s);
      e->begun = false;
   }
   const int xrc = rccl_exchange(e, e->xsend.p, su, e->xrecv.p, ru);
   if (!lrc && xrc) lrc = xrc;
   if (!lrc)
   {
      lrc = finish_enqueue(e, e->xrecv.p);
      if (lrc) e->begun = false;
   }
   hipError_t he = e->xflag.ensure(16);
   int32_t* hst = reinterpret_cast<int32_t*>(e->h_pinned + 16);
   if (he == hipSuccess)
   {
      hipLaunchKernelGGL(k_shard_status, dim3(1), dim3(64), 0, s, e->counters.as<unsigned>() + 8, lrc ? 1 : 0,
                         e->xflag.as<int>());
      he = hipGetLastError();
   }
   const bool red = he == hipSuccess && ncclAllReduce(e->xflag.p, e->xflag.p, 4, ncclInt32, ncclMax, comm, s) == ncclSuccess;
   if (red) he = hipMemcpyAsync(hst, e->xflag.p, 16, hipMemcpyDeviceToHost, s);
   if (he == hipSuccess) he = hipStreamSynchronize(s);
   if (!red || he != hipSuccess) return fail(e, GNOC_EHIP, "sharded step status all-reduce failed");
   const int32_t st[4] = { hst[0], hst[1], hst[2], hst[3] };
   if (st[0]) return lrc ? lrc : fail(e, GNOC_EHIP, "gnoc_run_sharded failed on another rank");
   if (st[1])
   {
      // a rank's X phase did not complete (a chain decline, an unsplittable burst, an
      // injected decline): the step reruns on the synchronous protocol everywhere.
      // gnoc_run_finish accounts the rerun (one run, its reruns); the stream attempt
      // adds one fallback.
      *accounted = true;
      e->fin_closed = false;
      const int rc = run_sharded_sync(e, su, ru);
      e->n_fallback++;
      e->tot_fallback++;
      return rc;
   }
   if (st[2]) return fail(e, GNOC_EHIP, "internal: route-count invariant violated (sharded step)");
   int rc = finish_check(e);
   if (st[3]) rc = shard_agree(e, rc, "gnoc_run_finish");   // some rank reran its Y levels
   return rc;
}

int gnoc_run_sharded(gnoc_engine* e)
{
   if (!e) return GNOC_EINVAL;
   // one rank without a communicator: the plain run; with one, the full protocol
   // (the exchange group, empty unless GNOC_SHARD_SELF_EXCHANGE, and the status
   // all-reduce), as every rank of a larger communicator runs it
   if (e->nranks <= 1 && !e->nccl && !e->tp.exchange) return gnoc_run(e);
   if (!e->nccl && !e->tp.exchange) return fail(e, GNOC_ESTATE, "gnoc_run_sharded needs gnoc_shard_set_comm or a transport");
   // from here every failure goes through the status agreement, so no peer waits
   // in a collective this rank never joins
   if (!e->submitted)
      return shard_agree(e, fail(e, GNOC_ESTATE, "gnoc_run_sharded before gnoc_submit"), "gnoc_run_begin");
   uint64_t ns = 0, nrv = 0;
   for (uint64_t u : e->xs_units) ns += u;
   for (uint64_t u : e->xr_units) nrv += u;
   hipError_t he = hipSetDevice(e->cfg.device);
   if (he == hipSuccess) he = e->xsend.ensure(std::max<uint64_t>(ns, 1) * 16);
   if (he == hipSuccess) he = e->xrecv.ensure(std::max<uint64_t>(nrv, 1) * 16);
   if (he != hipSuccess)
      return shard_agree(e, fail(e, GNOC_EHIP, std::string("exchange buffers: ") + hipGetErrorString(he)), "gnoc_run_begin");
   std::vector<uint64_t> su((size_t) e->nranks, 0), ru((size_t) e->nranks, 0);
   for (size_t q = 0; q < su.size(); q++)
   {
      su[q] = q < e->xs_units.size() ? e->xs_units[q] : 0;
      ru[q] = q < e->xr_units.size() ? e->xr_units[q] : 0;
   }
   if (!e->nccl) return run_sharded_sync(e, su.data(), ru.data());
   e->n_retry = e->n_fallback = 0;
   bool accounted = false;
   const int rc = run_sharded_stream(e, su.data(), ru.data(), ns, &accounted);
   if (!accounted)
   {
      e->runs++;
      e->tot_retry += e->n_retry;
      e->tot_fallback += e->n_fallback;
   }
   return rc;
}

// The X phase of a sharded run and the pack of the turn records.  sync: the
// transport is the caller's (or the exchange must not start before the buffer is
// complete): a declined X chain reruns on levels here, and the send buffer is
// complete on return.  !sync (gnoc_run_sharded over RCCL): everything stays on the
// stream; a declined X phase is carried by the pairs' status units instead
// (shard.hip), and the step's status all-reduce sends every rank to the rerun.
static int begin_x(gnoc_engine* e, void* send_buf, bool sync)
{
   e->ran = false;
   e->begun = false;
   bool done = false;
   int rc = run_prep(e, &done);
   if (rc) return rc;
   if (done)
   {
      e->begun = true;
      return GNOC_OK;
   }
   e->used_v3 = 1;
   e->used_chain = 0;
   e->n_retry = 0;
   e->n_fallback = 0;
   e->chD_run[0] = e->chD[0];
   e->chD_run[1] = e->chD[1];
   hipStream_t s = e->stream;
   rc = run_plan_v3(e);
   if (!rc && chain_usable(e))
   {
      // v4 X phase; a rank whose chains decline the batch reruns its X levels on
      // k_level before packing (the exchange layout does not depend on the path)
      e->used_chain = 1;
      e->used_v3 = 4;
      rc = chain_setup(e);
      if (!rc) rc = run_levels_v3(e, 0, 1);
      if (!rc) rc = chain_phase(e, 0);
      if (rc) return rc;
      if (!sync) goto pack;
      GNOC_HIP(e, hipMemcpyAsync(e->h_pinned + 8, e->counters.as<unsigned int>() + 8, 32, hipMemcpyDeviceToHost, s));
      GNOC_HIP(e, hipStreamSynchronize(s));
      const unsigned f4 = ((const unsigned*) (e->h_pinned + 8))[4];
      if (f4 & ch::F_ROUTE) return fail(e, GNOC_EHIP, "internal: chain route-count invariant violated");
      if (f4 & ch::F_ANY)
      {
         // an M/G/1 request or exception tails: a property of the batch, so its later
         // runs take the level engine straight away (a new submit clears this)
         // (the M/G/1 branch alone: later runs take k_chain's MG instantiation)
         if ((f4 & ch::F_FALLBACK) && !(f4 & ch::F_TIMEOUT))
         {
            if ((f4 & ch::R_MG1) && !e->ch_mg && !(f4 & ch::F_RETRY)) e->ch_mg = 1;
            else e->ch_declined = 1;
         }
         if (f4 & ch::F_RETRY)
         {
            // windows of this rank's X chains overflowed: shorter ones at the next run
            GNOC_HIP(e, hipMemcpy(e->h_nmax, e->ch_nmax.p, 8 * (e->h_cw[0].size() + e->h_cw[1].size()),
                                  hipMemcpyDeviceToHost));
            (void) halve_overflowed(e, e->chD);
            e->ch_resized = 1;
         }
         e->n_fallback++;
         GNOC_HIP(e, hipMemsetAsync(e->counters.as<unsigned int>() + 8 + 4, 0, 8, s));
         const uint32_t np = e->dc.N * PORTS;
         hipLaunchKernelGGL(ch::k_zero_ports, dim3((np + 255) / 256), dim3(256), 0, s, np,
                            (1u << P_LEFT) | (1u << P_RIGHT), e->port_sum.as<unsigned long long>(),
                            e->port_cnt.as<unsigned long long>(), e->port_mg1.as<unsigned long long>(),
                            e->port_flit.as<unsigned long long>(), e->port_last.as<unsigned long long>());
         GNOC_HIP(e, hipGetLastError());
         rc = run_levels_v3(e, 1, e->lvl_y0);
         if (rc) return rc;
      }
   }
   else if (!rc)
      rc = run_levels_v3(e, 0, e->lvl_y0);
   if (rc) return rc;
   if (sync)
   {
      // a look-back timeout or a leaf the splitter could not cut leaves garbage in
      // the turn slots: fail here, before anything is packed for the peers
      GNOC_HIP(e, hipMemcpyAsync(e->h_pinned + 8, e->counters.as<unsigned int>() + 8, 32, hipMemcpyDeviceToHost, s));
      GNOC_HIP(e, hipStreamSynchronize(s));
      if (((const unsigned*) (e->h_pinned + 8))[0] & 6u)
         return fail(e, GNOC_EUNSUPPORTED, "sharded run hit a burst the chunked path cannot split (X phase)");
   }
pack:
   {
      // test knobs: this rank reports an X-phase failure (the peers must all abort too);
      // this rank's X phase "declines" once on the stream path (its peers' Y phases
      // skip, and every rank reruns the step)
      const char* frv = std::getenv("GNOC_FAIL_RANK");
      if (frv && *frv && std::atoi(frv) == e->rank) return fail(e, GNOC_EHIP, "injected X-phase failure (GNOC_FAIL_RANK)");
      const char* prv = std::getenv("GNOC_DECLINE_ONCE_RANK");
      if (!sync && prv && *prv && std::atoi(prv) == e->rank && !e->declined_once)
      {
         e->declined_once = 1;
         GNOC_HIP(e, hipMemsetAsync(e->counters.as<unsigned int>() + 8 + 4, ch::F_TIMEOUT, 1, s));
      }
   }
   if (e->xs_slots)
   {
      if (!send_buf) return fail(e, GNOC_EINVAL, "null send buffer");
      const uint32_t np = (uint32_t) e->xs_pairs.size();
      hipLaunchKernelGGL(k_x_layout, dim3(np), dim3(1024), 0, s, e->dc.W, e->d_xs_pairs.as<XPair>(),
                         e->slot_cnt.as<uint32_t>(), e->xs_off.as<uint64_t>(), e->counters.as<unsigned>() + 8,
                         reinterpret_cast<uint4*>(send_buf), 0);
      GNOC_HIP(e, hipGetLastError());
      hipLaunchKernelGGL(k_x_pack, dim3((e->xs_slots + 3) / 4), dim3(256), 0, s, e->dc.W, e->d_xs_pairs.as<XPair>(), np,
                         e->xs_slots, e->xs_off.as<uint64_t>(), e->slot_cnt.as<uint32_t>(), e->slot_base.as<uint64_t>(),
                         e->nexc.as<uint32_t>(), e->recs.as<Rec>(), reinterpret_cast<uint4*>(send_buf));
      GNOC_HIP(e, hipGetLastError());
   }
   if (sync) GNOC_HIP(e, hipStreamSynchronize(s));   // the send buffer is complete when this returns
   e->begun = true;
   return GNOC_OK;
}

int gnoc_run_begin(gnoc_engine* e, void* send_buf)
{
   if (!e) return GNOC_EINVAL;
   return begin_x(e, send_buf, true);
}


int gnoc_run_finish(gnoc_engine* e, const void* recv_buf)
{
   if (!e) return GNOC_EINVAL;
   int rc = finish_enqueue(e, recv_buf);
   if (!rc) rc = finish_check(e);
   e->runs++;
   e->tot_retry += e->n_retry;
   e->tot_fallback += e->n_fallback;
   return rc;
}
// The Y phase of a sharded run: the received turn records back into their slots,
// the Y chains (or levels) and the SELF level, the per-packet finish, and the
// read-back of the flags -- all on the stream, no host sync (finish_check syncs).
static int finish_enqueue(gnoc_engine* e, const void* recv_buf)
{
   if (!e->begun) return fail(e, GNOC_ESTATE, "gnoc_run_finish without gnoc_run_begin");
   e->begun = false;
   e->fin_closed = !e->dc.contention;
   if (!e->dc.contention) return GNOC_OK;   // closed form finished in gnoc_run_begin
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   hipStream_t s = e->stream;
   if (e->xr_slots)
   {
      if (!recv_buf) return fail(e, GNOC_EINVAL, "null receive buffer");
      const uint32_t np = (uint32_t) e->xr_pairs.size();
      hipLaunchKernelGGL(k_x_layout, dim3(np), dim3(1024), 0, s, e->dc.W, e->d_xr_pairs.as<XPair>(),
                         e->slot_cnt.as<uint32_t>(), e->xr_off.as<uint64_t>(), e->counters.as<unsigned>() + 8,
                         reinterpret_cast<uint4*>(const_cast<void*>(recv_buf)), 1);
      GNOC_HIP(e, hipGetLastError());
      hipLaunchKernelGGL(k_x_unpack, dim3((e->xr_slots + 3) / 4), dim3(256), 0, s, e->dc.W, e->d_xr_pairs.as<XPair>(), np,
                         e->xr_slots, e->xr_off.as<uint64_t>(), e->slot_cnt.as<uint32_t>(), e->slot_base.as<uint64_t>(),
                         e->nexc.as<uint32_t>(), e->recs.as<Rec>(), e->samp_t.as<uint64_t>(), e->samp_id.as<uint32_t>(),
                         reinterpret_cast<const uint4*>(recv_buf), e->counters.as<unsigned>() + 8);
      GNOC_HIP(e, hipGetLastError());
   }
   const uint32_t L = (uint32_t) e->lvl_off.size() - 1;
   int rc = GNOC_OK;
   if (e->used_chain && !e->ch_ydeclined)
   {
      // exception tails (M/G/1-served turns, here or at a peer) into order for the Y chains
      if (e->dc.analytical) rc = exc_merge(e);
      if (!rc) rc = chain_phase(e, 1);
      if (!rc) rc = run_levels_v3(e, L - 1, L);
   }
   else
   {
      if (e->used_chain) e->used_v3 = 5;   // X chains, Y levels (this batch's Y chains declined)
      rc = run_levels_v3(e, e->lvl_y0, L);
   }
   if (!rc) rc = run_post_enqueue(e, false);
   return rc;
}
// After finish_enqueue: the one host sync, then the checks; a rank whose Y chains
// declined reruns its Y and SELF levels here (local: the exchange is done).
static int finish_check(gnoc_engine* e)
{
   if (e->fin_closed) return GNOC_OK;
   hipStream_t s = e->stream;
   int rc = run_post_check(e, false);
   if (rc == GNOC_V3_RETRY) return fail(e, GNOC_EUNSUPPORTED, "sharded run hit a burst the chunked path cannot split");
   if (!e->used_chain) return rc;
   // (the sharded path's own Y fallback below; its chains run the common instantiation,
   // which declines where the M/G/1 branch fires and leaves no exception tails)
   if (rc == GNOC_CH_EXC || rc == GNOC_CH_YFALL || rc == GNOC_CH_MG || rc == GNOC_CH_XCDOFF) rc = GNOC_CH_FALLBACK;
   // the MG instantiation's Y chains may have left exception tails in the SELF slots
   const bool mg_ran = e->ch_mg != 0;
   // a decline for a property of the batch (not a hand-off timeout): the M/G/1 branch
   // sends later runs to the MG instantiation once, anything else (or the MG
   // instantiation declining too) to the Y levels straight after the exchange
   if (rc == GNOC_CH_FALLBACK && (e->ch_yflags & ch::F_FALLBACK) && !(e->ch_yflags & (ch::F_TIMEOUT | ch::R_XCD)))
   {
      if ((e->ch_yflags & ch::R_MG1) && !mg_ran) e->ch_mg = 1;
      else e->ch_ydeclined = 1;
   }
   // the windows of the next run: from this run's measured fill, or shorter
   // for the chains that overflowed (results never depend on them)
   if (!rc && !e->ch_resized) adapt_windows(e);
   if (rc == GNOC_CH_RETRY) (void) halve_overflowed(e, e->chD);
   e->ch_resized = 0;
   if (rc != GNOC_CH_RETRY && rc != GNOC_CH_FALLBACK) return rc;
   // the Y chains declined: Y and SELF levels on k_level (fresh look-back state)
   e->n_fallback++;
   e->used_chain = 0;
   GNOC_HIP(e, hipMemsetAsync(e->counters.as<unsigned int>() + 8 + 4, 0, 8, s));
   if (mg_ran)
   {
      hipLaunchKernelGGL(ch::k_zero_self_nexc, dim3((e->dc.N * INS + 255) / 256), dim3(256), 0, s, e->dc.N,
                         e->nexc.as<uint32_t>());
      GNOC_HIP(e, hipGetLastError());
   }
   const uint32_t np = e->dc.N * PORTS;
   hipLaunchKernelGGL(ch::k_zero_ports, dim3((np + 255) / 256), dim3(256), 0, s, np,
                      (1u << P_UP) | (1u << P_DOWN) | (1u << P_SELF), e->port_sum.as<unsigned long long>(),
                      e->port_cnt.as<unsigned long long>(), e->port_mg1.as<unsigned long long>(),
                      e->port_flit.as<unsigned long long>(), e->port_last.as<unsigned long long>());
   GNOC_HIP(e, hipGetLastError());
   rc = run_plan_v3(e);
   if (!rc) rc = run_levels_v3(e, e->lvl_y0, (uint32_t) e->lvl_off.size() - 1);
   if (!rc) rc = run_post(e, false);
   return rc;
}

int gnoc_get_packet_results(gnoc_engine* e, uint64_t* final_ps, uint64_t* zero_load_ps, uint64_t* contention_ps, size_t n)
{
   if (!e) return GNOC_EINVAL;
   if (!e->ran) return fail(e, GNOC_ESTATE, "no results: call gnoc_run first");
   if (n != (e->part ? e->n_glob : e->n)) return fail(e, GNOC_EINVAL, "result array length != submitted packet count");
   if (!n) return GNOC_OK;
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   if (e->nranks > 1 && e->n)
   {
      hipLaunchKernelGGL(k_mask_unowned, dim3((uint32_t) std::min<size_t>((e->n + 255) / 256, 8192)), dim3(256), 0,
                         e->stream, (uint64_t) e->n, e->aux.as<uint32_t>(), e->cx0, e->cx1, e->final_ps.as<uint64_t>(),
                         e->zl.as<uint64_t>(), e->cont.as<uint64_t>());
      GNOC_HIP(e, hipGetLastError());
   }
   if (e->part)
   {
      // this rank's packets back to their places in the whole trace; 0 elsewhere
      const size_t m = e->n;
      std::vector<uint64_t> tmp(m);
      uint64_t* outs[3] = { final_ps, zero_load_ps, contention_ps };
      const DevBuf* srcs[3] = { &e->final_ps, &e->zl, &e->cont };
      for (int k = 0; k < 3; k++)
      {
         if (!outs[k]) continue;
         std::memset(outs[k], 0, n * 8);
         if (!m) continue;
         GNOC_HIP(e, hipMemcpyAsync(tmp.data(), srcs[k]->p, m * 8, hipMemcpyDeviceToHost, e->stream));
         GNOC_HIP(e, hipStreamSynchronize(e->stream));
         for (size_t i = 0; i < m; i++) outs[k][e->h_gid[i]] = tmp[i];
      }
      return GNOC_OK;
   }
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

int gnoc_get_port_utilization(gnoc_engine* e, uint64_t* flits, uint64_t* last_cycle, size_t nports)
{
   if (!e) return GNOC_EINVAL;
   if (!e->ran) return fail(e, GNOC_ESTATE, "no results: call gnoc_run first");
   const size_t np = (size_t) e->dc.N * PORTS;
   if (nports != np) return fail(e, GNOC_EINVAL, "nports != num_tiles*6");
   GNOC_HIP(e, hipSetDevice(e->cfg.device));
   if (!e->dc.contention)
   {
      if (flits) std::memset(flits, 0, np * 8);
      if (last_cycle) std::memset(last_cycle, 0, np * 8);
      return GNOC_OK;
   }
   if (flits) GNOC_HIP(e, hipMemcpyAsync(flits, e->port_flit.p, np * 8, hipMemcpyDeviceToHost, e->stream));
   if (last_cycle) GNOC_HIP(e, hipMemcpyAsync(last_cycle, e->port_last.p, np * 8, hipMemcpyDeviceToHost, e->stream));
   GNOC_HIP(e, hipStreamSynchronize(e->stream));
   return GNOC_OK;
}

int gnoc_get_summary(gnoc_engine* e, gnoc_summary* out)
{
   if (!e || !out) return GNOC_EINVAL;
   std::memset(out, 0, sizeof(*out));
   out->packets = e->part ? e->n_glob : e->n;
   // a partitioned rank reports the whole mesh's totals (as an unpartitioned one does)
   out->mesh_hops = e->part ? e->h_glob_hops : e->h_counters[0];
   out->routed_packets = e->part ? e->h_glob_routed : e->h_counters[1];
   out->records = e->h_records;
   out->levels = e->h_levels;
   out->last_run_ms = e->last_ms;
   out->engine_path = e->dc.contention ? (uint32_t) e->used_v3 : 2u;
   out->retries = e->n_retry;
   out->fallbacks = e->n_fallback;
   // per phase: the most windows and the longest window of any chain
   uint32_t nwm[2] = { 0, 0 };
   uint64_t dm[2] = { 0, 0 };
   for (int p = 0; p < 2 && e->used_chain; p++)
      for (const ChainWin& w : e->h_cw[p])
      {
         nwm[p] = std::max(nwm[p], w.nW);
         dm[p] = std::max(dm[p], w.D);
      }
   out->windows = nwm[0];
   uint32_t sh = 0;
   while (sh < 63 && (2ull << sh) <= dm[0]) sh++;
   out->window_shift = e->used_chain ? sh : 0u;
   out->windows_y = nwm[1];
   out->chain_protocol = e->used_chain ? 0x100u | e->ch_lb_run[0] | (e->ch_lb_run[1] << 1) | (e->ch_mg ? 0x400u : 0u) |
                                         (e->ch_split ? 0x800u : 0u) : 0u;
   out->window_ps_x = dm[0];
   out->window_ps_y = dm[1];
   out->runs = e->runs;
   out->retries_total = e->tot_retry;
   out->fallbacks_total = e->tot_fallback;
   out->abi_pad2 = 0;
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

// Debug (tools/stamps.py, GNOC_STAMPS=1): per-chunk phase stamps of the last run.
__attribute__((visibility("default"))) int gnoc_debug_stamps(gnoc_engine* e, uint64_t* out, size_t cap, size_t* nchunks)
{
   if (!e || !nchunks) return GNOC_EINVAL;
   *nchunks = e->h_chunk_bound;
   if (!out || !e->stamps.p) return GNOC_OK;
   const size_t n = std::min(cap, (size_t) e->h_chunk_bound * 16);
   GNOC_HIP(e, hipMemcpy(out, e->stamps.p, n * 8, hipMemcpyDeviceToHost));
   return GNOC_OK;
}

// Debug (tools/chain_stamps.py, GNOC_STAMPS=1): per-step stamps of the last chain run, phase 0 (X) or 1 (Y).
__attribute__((visibility("default"))) int gnoc_debug_chain_stamps(gnoc_engine* e, int phase, uint64_t* out, size_t cap,
                                                                   size_t* count, uint32_t* geom)
{
   if (!e || !count) return GNOC_EINVAL;
   if (phase < 0 || phase > 1) return GNOC_EINVAL;
   const DevBuf& sb = phase == 1 ? e->ch_stamps1 : e->ch_stamps0;
   const uint32_t len = phase ? e->dc.H - 1 : e->dc.W - 1;
   const size_t nt = e->h_tasks[phase].size();
   *count = nt * len * 16;
   if (geom)
   {
      geom[0] = 1;
      geom[1] = (uint32_t) nt;
      geom[2] = len;
      geom[3] = 0u;
   }
   if (!out || !sb.p) return GNOC_OK;
   GNOC_HIP(e, hipMemcpy(out, sb.p, std::min(cap, *count) * 8, hipMemcpyDeviceToHost));
   return GNOC_OK;
}

// Debug (tools/chain_stamps.py): the task table of the last chain run, phase 0 (X) or 1
// (Y): chain << 16 | window per task in dequeue order; out2 (optional) the windows'
// length D per chain.
__attribute__((visibility("default"))) int gnoc_debug_chain_tasks(gnoc_engine* e, int phase, uint32_t* out, size_t cap,
                                                                  size_t* count, uint64_t* dlen, size_t dcap)
{
   if (!e || !count || phase < 0 || phase > 1) return GNOC_EINVAL;
   const std::vector<uint32_t>& t = e->h_tasks[phase];
   *count = t.size();
   if (out) std::copy(t.begin(), t.begin() + std::min(cap, t.size()), out);
   if (dlen)
      for (size_t c = 0; c < std::min(dcap, e->h_cw[phase].size()); c++) dlen[c] = e->h_cw[phase][c].D;
   return GNOC_OK;
}

int gnoc_device_final_ps(gnoc_engine* e, void** dptr)
{
   if (!e || !dptr) return GNOC_EINVAL;
   if (!e->ran) return fail(e, GNOC_ESTATE, "no results: call gnoc_run first");
   if (e->part) return fail(e, GNOC_EUNSUPPORTED, "a sharded rank holds only its own packets' results (gnoc_get_packet_results)");
   *dptr = e->final_ps.p;
   return GNOC_OK;
}

}  // extern "C"
