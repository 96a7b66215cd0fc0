// gnoc_replay -- replay an on-disk packet trace (include/gnoc.h,
// gnoc_trace_header) through the C++ host model on the GPU.
//
//   gnoc_replay TRACE [--results FILE] [--summary TILE|all] [--device D] [--repeat K]
//               [--moving-avg arithmetic_mean|median:WINDOW]
//               [--shards N]                 N ranks in this process (threads), one GPU
//               [--rccl IDFILE:RANK:NRANKS]  this process is RANK of a multi-process RCCL run
//
// --results writes final/zero-load/contention picoseconds (u64[n] each) then the
// per-port contention sum, packet count and analytical-request count
// (u64[num_tiles*6] each).  Prints one JSON line with the run's totals.
// Sharded runs (gnoc_run_sharded, include/gnoc.h) go through the C ABI alone:
// --shards sums the ranks' shares into one results file; under --rccl each
// process writes its own share (FILE.RANK; the element-wise sum is the mesh's).
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "network_model_emesh_hop_by_hop_hip.h"
#include "shard_local.h"

using graphite_amd::NetworkModelEMeshHopByHopHIP;

namespace {

struct Share
{
   std::vector<uint64_t> v;   // fin, zl, ct (n each), port sum, count, mg1 (np each)
   int rc = 0;
   std::string err;
};

// One rank: create, shard, submit, (transport or communicator), run, collect.
void run_rank(const gnoc_config& cfg, const gnoc_trace_queue& q, const gnoc_packets& pk, size_t n, int rank, int nr,
              const gnoc_transport* tp, void* comm, Share& out)
{
   const size_t np = (size_t) cfg.num_tiles * GNOC_PORTS_PER_TILE;
   gnoc_engine* e = nullptr;
   int rc = gnoc_create(&cfg, &e);
   if (!rc && q.ma_type != GNOC_MOVING_AVG_NONE) rc = gnoc_set_basic_moving_average(e, q.ma_type, q.ma_window);
   if (!rc) rc = gnoc_shard(e, rank, nr);
   if (!rc) rc = gnoc_submit(e, &pk, n);
   if (!rc) rc = tp ? gnoc_shard_set_transport(e, tp) : gnoc_shard_set_comm(e, comm);
   const int rr = gnoc_run_sharded(e);   // collective: every rank enters it
   rc = rc ? rc : rr;
   out.v.assign(3 * n + 3 * np, 0);
   uint64_t* v = out.v.data();
   if (!rc) rc = gnoc_get_packet_results(e, v, v + n, v + 2 * n, n);
   if (!rc) rc = gnoc_get_port_stats(e, v + 3 * n, v + 3 * n + np, v + 3 * n + 2 * np, np);
   out.rc = rc;
   if (rc && e) out.err = gnoc_last_error(e);
   gnoc_destroy(e);
}

bool write_results(const std::string& path, const std::vector<uint64_t>& v)
{
   FILE* f = std::fopen(path.c_str(), "wb");
   if (!f) return false;
   bool ok = std::fwrite(v.data(), 8, v.size(), f) == v.size();
   return (std::fclose(f) == 0) && ok;
}

int sharded(const std::string& trace, const std::string& results, int shards, const std::string& rccl, int device)
{
   gnoc_config cfg;
   gnoc_trace_queue q;
   size_t n = 0;
   if (gnoc_trace_file_read_q(trace.c_str(), &cfg, &q, nullptr, nullptr, nullptr, nullptr, nullptr, 0, &n))
   {
      std::fprintf(stderr, "gnoc_replay: cannot read %s\n", trace.c_str());
      return 1;
   }
   cfg.device = device;
   std::vector<uint64_t> inj(n);
   std::vector<uint32_t> src(n), dst(n), bits(n), flags(n);
   if (gnoc_trace_file_read(trace.c_str(), nullptr, inj.data(), src.data(), dst.data(), bits.data(), flags.data(), n, &n))
      return 1;
   const gnoc_packets pk{inj.data(), src.data(), dst.data(), bits.data(), flags.data()};
   const auto t0 = std::chrono::steady_clock::now();
   std::vector<uint64_t> sum;
   int rank = 0, nr = shards;
   if (!rccl.empty())
   {
      // IDFILE:RANK:NRANKS -- rank 0 writes the unique id, the others wait for it
      const size_t a = rccl.find(':'), b = rccl.rfind(':');
      const std::string idf = rccl.substr(0, a);
      rank = std::atoi(rccl.c_str() + a + 1);
      nr = std::atoi(rccl.c_str() + b + 1);
      ncclUniqueId id;
      if (rank == 0)
      {
         ncclGetUniqueId(&id);
         std::ofstream(idf + ".tmp", std::ios::binary).write(reinterpret_cast<const char*>(&id), sizeof id);
         std::rename((idf + ".tmp").c_str(), idf.c_str());
      }
      else
      {
         for (;;)
         {
            std::ifstream f(idf, std::ios::binary);
            if (f.read(reinterpret_cast<char*>(&id), sizeof id)) break;
            std::this_thread::sleep_for(std::chrono::milliseconds(20));
         }
      }
      if (hipSetDevice(device) != hipSuccess) return 1;
      ncclComm_t comm;
      if (ncclCommInitRank(&comm, nr, id, rank) != ncclSuccess)
      {
         std::fprintf(stderr, "gnoc_replay: ncclCommInitRank failed\n");
         return 1;
      }
      Share sh;
      run_rank(cfg, q, pk, n, rank, nr, nullptr, comm, sh);
      ncclCommDestroy(comm);
      if (sh.rc)
      {
         std::fprintf(stderr, "gnoc_replay: rank %d: %s (status %d)\n", rank, sh.err.c_str(), sh.rc);
         return 1;
      }
      sum = sh.v;
      if (!results.empty() && !write_results(results + "." + std::to_string(rank), sum)) return 1;
   }
   else
   {
      graphite_amd::LocalShardTransport tp(nr);
      std::vector<Share> sh(nr);
      std::vector<gnoc_transport> tps;
      for (int r = 0; r < nr; r++) tps.push_back(tp.transport(r));
      std::vector<std::thread> th;
      for (int r = 0; r < nr; r++)
         th.emplace_back([&, r] { run_rank(cfg, q, pk, n, r, nr, &tps[r], nullptr, sh[r]); });
      for (auto& t : th) t.join();
      for (int r = 0; r < nr; r++)
         if (sh[r].rc)
         {
            std::fprintf(stderr, "gnoc_replay: rank %d: %s (status %d)\n", r, sh[r].err.c_str(), sh[r].rc);
            return 1;
         }
      sum.assign(sh[0].v.size(), 0);
      for (int r = 0; r < nr; r++)
         for (size_t i = 0; i < sum.size(); i++) sum[i] += sh[r].v[i];   // each entry non-zero on one rank
      if (!results.empty() && !write_results(results, sum)) return 1;
   }
   const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
   std::printf("{\"packets\": %zu, \"ranks\": %d, \"rank\": %d, \"host_ms\": %.4f}\n", n, nr, rank, ms);
   return 0;
}

}  // namespace

int main(int argc, char** argv)
{
   if (argc < 2)
   {
      std::fprintf(stderr, "usage: %s TRACE [--results FILE] [--summary TILE|all] [--device D] [--repeat K] "
                           "[--moving-avg TYPE:WINDOW]\n", argv[0]);
      return 2;
   }
   std::string results, summary, mavg, rccl;
   int device = 0, repeat = 1, shards = 0;
   for (int i = 2; i + 1 < argc; i += 2)
   {
      if (!std::strcmp(argv[i], "--results")) results = argv[i + 1];
      else if (!std::strcmp(argv[i], "--summary")) summary = argv[i + 1];
      else if (!std::strcmp(argv[i], "--device")) device = std::atoi(argv[i + 1]);
      else if (!std::strcmp(argv[i], "--repeat")) repeat = std::atoi(argv[i + 1]);
      else if (!std::strcmp(argv[i], "--moving-avg")) mavg = argv[i + 1];
      else if (!std::strcmp(argv[i], "--shards")) shards = std::atoi(argv[i + 1]);
      else if (!std::strcmp(argv[i], "--rccl")) rccl = argv[i + 1];
      else
      {
         std::fprintf(stderr, "unknown option %s\n", argv[i]);
         return 2;
      }
   }
   if (shards > 1 || !rccl.empty()) return sharded(argv[1], results, shards, rccl, device);
   try
   {
      std::unique_ptr<NetworkModelEMeshHopByHopHIP> m(NetworkModelEMeshHopByHopHIP::fromTraceFile(argv[1], device));
      if (!mavg.empty())
      {
         // queue_model/basic/moving_avg_type:moving_avg_window_size (overrides the trace header's)
         const size_t c = mavg.find(':');
         const std::string t = mavg.substr(0, c);
         const int32_t type = t == "arithmetic_mean" ? GNOC_MOVING_AVG_ARITHMETIC_MEAN
                            : t == "geometric_mean"  ? GNOC_MOVING_AVG_GEOMETRIC_MEAN
                            : t == "median"          ? GNOC_MOVING_AVG_MEDIAN : -1;
         m->setBasicMovingAverage(type, c == std::string::npos ? 64u : (uint32_t) std::atoi(mavg.c_str() + c + 1));
      }
      double best_ms = 1e30;
      for (int r = 0; r < repeat; r++)
      {
         const auto t0 = std::chrono::steady_clock::now();
         m->run();
         const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
         best_ms = ms < best_ms ? ms : best_ms;
      }
      if (!results.empty())
      {
         FILE* f = std::fopen(results.c_str(), "wb");
         if (!f) throw graphite_amd::NetworkModelError(GNOC_EINVAL, "cannot write " + results);
         const size_t n = m->numPackets(), np = m->portPackets().size();
         bool ok = true;
         ok &= std::fwrite(m->packetTime().data(), 8, n, f) == n;
         ok &= std::fwrite(m->packetZeroLoadDelay().data(), 8, n, f) == n;
         ok &= std::fwrite(m->packetContentionDelay().data(), 8, n, f) == n;
         ok &= std::fwrite(m->portContentionDelay().data(), 8, np, f) == np;
         ok &= std::fwrite(m->portPackets().data(), 8, np, f) == np;
         ok &= std::fwrite(m->portAnalyticalRequests().data(), 8, np, f) == np;
         ok &= std::fclose(f) == 0;
         if (!ok) throw graphite_amd::NetworkModelError(GNOC_EINVAL, "short write to " + results);
      }
      if (!summary.empty())
      {
         const int lo = summary == "all" ? 0 : std::atoi(summary.c_str());
         const int hi = summary == "all" ? m->numTiles() : lo + 1;
         for (int t = lo; t < hi; t++)
         {
            std::cout << "Tile " << t << ":\n  Network (emesh_hop_by_hop_hip):\n";
            m->outputSummary(std::cout, t);
         }
      }
      const gnoc_summary s = m->summary();
      std::printf("{\"packets\": %llu, \"routed_packets\": %llu, \"mesh_hops\": %llu, \"mg1_uses\": %llu, "
                  "\"device_ms\": %.4f, \"host_ms\": %.4f}\n",
                  (unsigned long long) s.packets, (unsigned long long) s.routed_packets,
                  (unsigned long long) s.mesh_hops, (unsigned long long) s.mg1_uses, s.last_run_ms, best_ms);
   }
   catch (const graphite_amd::NetworkModelError& e)
   {
      std::fprintf(stderr, "gnoc_replay: %s (status %d)\n", e.what(), e.status);
      return 1;
   }
   return 0;
}
