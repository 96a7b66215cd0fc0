// gnoc_replay -- replay an on-disk packet trace (include/gnoc.h,
// gnoc_trace_header) through the C++ host model on the GPU.
//
//   gnoc_replay TRACE [--results FILE] [--summary TILE|all] [--device D] [--repeat K]
//               [--moving-avg arithmetic_mean|median:WINDOW]
//
// --results writes final/zero-load/contention picoseconds (u64[n] each) then the
// per-port contention sum, packet count and analytical-request count
// (u64[num_tiles*6] each).  Prints one JSON line with the run's totals.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <memory>
#include <string>

#include "network_model_emesh_hop_by_hop_hip.h"

using graphite_amd::NetworkModelEMeshHopByHopHIP;

int main(int argc, char** argv)
{
   if (argc < 2)
   {
      std::fprintf(stderr, "usage: %s TRACE [--results FILE] [--summary TILE|all] [--device D] [--repeat K] "
                           "[--moving-avg TYPE:WINDOW]\n", argv[0]);
      return 2;
   }
   std::string results, summary, mavg;
   int device = 0, repeat = 1;
   for (int i = 2; i + 1 < argc; i += 2)
   {
      if (!std::strcmp(argv[i], "--results")) results = argv[i + 1];
      else if (!std::strcmp(argv[i], "--summary")) summary = argv[i + 1];
      else if (!std::strcmp(argv[i], "--device")) device = std::atoi(argv[i + 1]);
      else if (!std::strcmp(argv[i], "--repeat")) repeat = std::atoi(argv[i + 1]);
      else if (!std::strcmp(argv[i], "--moving-avg")) mavg = argv[i + 1];
      else
      {
         std::fprintf(stderr, "unknown option %s\n", argv[i]);
         return 2;
      }
   }
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
