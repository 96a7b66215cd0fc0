// Known-answer tests of the C++ host model, in the style of the reference's
// unit tests (tests/unit/history_tree/history_tree.cc): build the model the way
// Graphite would (carbon_sim.cfg keys), route packets, check exact cycles,
// exit 0 on success.  Needs the GPU (runs from tests/test_host_cpp.py).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "network_model_emesh_hop_by_hop_hip.h"

using namespace graphite_amd;

static int failures = 0;
#define EXPECT_EQ(a, b)                                                                                   \
   do                                                                                                     \
   {                                                                                                      \
      const unsigned long long a_ = (unsigned long long) (a), b_ = (unsigned long long) (b);              \
      if (a_ != b_)                                                                                       \
      {                                                                                                   \
         std::fprintf(stderr, "%s:%d: %s == %llu, expected %llu\n", __FILE__, __LINE__, #a, a_, b_);      \
         failures++;                                                                                      \
      }                                                                                                   \
   } while (0)

static NetPacket pkt(uint64_t cycle, int s, int d, uint32_t bits = 576)
{
   NetPacket p;
   p.time = cycle * 1000;
   p.sender = s;
   p.receiver = d;
   p.modeled_bits = bits;
   return p;
}

int main()
{
   CfgView cfg;   // carbon_sim.cfg defaults: 64-bit flits, router 1, link 1, history_tree
   cfg.set("general/total_cores", "16");
   cfg.set("network/emesh_hop_by_hop/flit_width", "64");

   // 1. zero load: latency = (H+1)(R+Lk) + F   (SURVEY.md 8a closed form)
   {
      NetworkModelEMeshHopByHopHIP m(cfg);
      m.routePacket(pkt(0, 0, 15));      // H = 6, F = 9
      m.routePacket(pkt(1000, 5, 6));    // H = 1
      m.run();
      EXPECT_EQ(m.packetTime()[0], (7 * 2 + 9) * 1000);
      EXPECT_EQ(m.packetZeroLoadDelay()[0], (7 * 2 + 9) * 1000);
      EXPECT_EQ(m.packetContentionDelay()[0], 0);
      EXPECT_EQ(m.packetTime()[1] - 1000 * 1000, (2 * 2 + 9) * 1000);
   }
   // 2. two packets injected by one tile in the same cycle: the second waits
   //    F = 9 cycles at the injection queue (FIFO X <- max(t, X) + F), then
   //    rides behind the first with no further contention.
   {
      NetworkModelEMeshHopByHopHIP m(cfg);
      m.routePacket(pkt(10, 0, 3));
      m.routePacket(pkt(10, 0, 3));
      m.run();
      EXPECT_EQ(m.packetContentionDelay()[0], 0);
      EXPECT_EQ(m.packetContentionDelay()[1], 9 * 1000);
      EXPECT_EQ(m.packetTime()[1] - m.packetTime()[0], 9 * 1000);
      EXPECT_EQ(m.portContentionDelay()[0 * GNOC_PORTS_PER_TILE + GNOC_PORT_INJ], 9);
      EXPECT_EQ(m.portPackets()[0 * GNOC_PORTS_PER_TILE + GNOC_PORT_INJ], 2);
   }
   // 3. self-sends and unmodeled packets keep their send time (processCornerCases,
   //    isModelEnabled: network_model.cc:171-183, 413-468)
   {
      NetworkModelEMeshHopByHopHIP m(cfg);
      m.routePacket(pkt(5, 3, 3));
      NetPacket u = pkt(6, 0, 15);
      u.modeled = false;
      m.routePacket(u);
      m.run();
      EXPECT_EQ(m.packetTime()[0], 5000);
      EXPECT_EQ(m.packetTime()[1], 6000);
   }
   // 4. configuration errors are reported, not aborted on
   {
      CfgView bad = cfg;
      bad.set("general/total_cores", "14");   // not W x H (emesh_hop_by_hop.cc:309-320)
      bool threw = false;
      try { NetworkModelEMeshHopByHopHIP m(bad); } catch (const NetworkModelError& e) { threw = e.status == GNOC_EINVAL; }
      EXPECT_EQ(threw, 1);
      EXPECT_EQ(NetworkModelEMeshHopByHopHIP::isTileCountPermissible(14), 0);
      EXPECT_EQ(NetworkModelEMeshHopByHopHIP::isTileCountPermissible(1024), 1);
      std::vector<int> mc = NetworkModelEMeshHopByHopHIP::computeMemoryControllerPositions(4, 16);
      EXPECT_EQ(mc.size(), 4);
      EXPECT_EQ(mc[0], 1 + 1 * 4);
   }
   // 5. broadcast tree (emesh_hop_by_hop.cc:163-221) from tile 5 = (1, 1) of 4x4:
   //    every tile receives at (H+1)(R+Lk) + F; the sender's router selects all
   //    5 ports (crossbar[5]), a row router 4 (UP, DOWN, onward, SELF).
   {
      NetworkModelEMeshHopByHopHIP m(cfg);
      m.routePacket(pkt(0, 5, NetPacket::BROADCAST));
      m.run();
      EXPECT_EQ(m.broadcastReceiptTime(0, 5), (1 * 2 + 9) * 1000);
      EXPECT_EQ(m.broadcastReceiptTime(0, 15), (5 * 2 + 9) * 1000);   // H = 4
      EXPECT_EQ(m.broadcastReceiptContentionDelay(0, 15), 0);
      EXPECT_EQ(m.packetTime()[0], (5 * 2 + 9) * 1000);                 // latest receipt
      EXPECT_EQ(m.routerCrossbarTraversals(5, 5), 9);
      EXPECT_EQ(m.routerCrossbarTraversals(6, 4), 9);
      EXPECT_EQ(m.routerLinkTraversals(6), 4 * 9);
      EXPECT_EQ(m.routerPackets(0), 1);
      CfgView nt = cfg;
      nt.set("network/emesh_hop_by_hop/broadcast_tree_enabled", "false");
      NetworkModelEMeshHopByHopHIP m2(nt);
      bool threw = false;
      try { m2.routePacket(pkt(0, 5, NetPacket::BROADCAST)); } catch (const NetworkModelError& e) { threw = e.status == GNOC_EINVAL; }
      EXPECT_EQ(threw, 1);
   }
   // 6. queue_model/basic moving average: the reference's code defaults when the
   //    section is absent (queue_model_basic.cc:17-19: disabled, window 1, "none")
   {
      CfgView empty;
      int32_t type = -7;
      uint32_t window = 0;
      empty.basicMovingAverage(&type, &window);
      EXPECT_EQ(type, GNOC_MOVING_AVG_NONE);
      EXPECT_EQ(window, 1);
      CfgView on = cfg;
      on.set("queue_model/basic/moving_avg_enabled", "true");
      on.basicMovingAverage(&type, &window);
      EXPECT_EQ(type, GNOC_MOVING_AVG_NONE);   // enabled, type "none": createAvgType gives NULL
      on.set("queue_model/basic/moving_avg_type", "arithmetic_mean");
      on.set("queue_model/basic/moving_avg_window_size", "8");
      on.basicMovingAverage(&type, &window);
      EXPECT_EQ(type, GNOC_MOVING_AVG_ARITHMETIC_MEAN);
      EXPECT_EQ(window, 8);
   }
   if (failures)
   {
      std::fprintf(stderr, "%d failure(s)\n", failures);
      return 1;
   }
   std::printf("test_emesh_hop_by_hop_hip: all checks passed\n");
   return 0;
}
