// network_model_emesh_hop_by_hop_hip.h -- C++ host side of the MI355X
// emesh_hop_by_hop timing engine, shaped like the reference's network-model
// plug-in so a Graphite maintainer can register it next to the CPU model.
//
// Reference interface it mirrors (INTEGRATION.md shows the registration):
//   NetworkModel                          common/network/network_model.h:39-207
//     createModel / parseNetworkType       network_model.cc:50-71, 318-335
//     __routePacket (SEND_TILE)            network_model.cc:87-116
//     processReceivedPacket                network_model.cc:142-150
//     outputSummary                        network_model.cc:274-316
//     isTileCountPermissible, computeMemoryControllerPositions
//                                          network_model.cc:337-411
//   NetworkModelEMeshHopByHop             common/network/models/network_model_emesh_hop_by_hop.{h,cc}
//     ctor config reads                    :16-38  (network/emesh_hop_by_hop/...)
//     routePacket                          :146-264
//     outputContentionModelsSummary        :471-493
//   RouterModel contention counters       common/network/components/router/router_model.cc:136-215
//
// Trace mode: the reference routes one packet per call and returns its hops;
// the engine times a whole batch at once.  routePacket() records a packet
// (what Network::netSend hands the model at SEND_TILE), run() times every hop
// of every recorded packet on the GPU through the C ABI (include/gnoc.h), and
// the results carry the three NetPacket fields the reference updates
// (time, zero_load_delay, contention_delay; network.h:27-55).
//
// Errors: the reference aborts through LOG_PRINT_ERROR (common/misc/log.cc:
// 360-362); this layer throws NetworkModelError carrying the C ABI's status
// and message (uncaught, that terminates the process like the reference).
#pragma once

#include <cstdint>
#include <map>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "gnoc.h"

namespace graphite_amd {

class NetworkModelError : public std::runtime_error
{
public:
   NetworkModelError(int status, const std::string& msg) : std::runtime_error(msg), status(status) {}
   int status;
};

// The Sim()->getCfg() view of carbon_sim.cfg keys the path reads (SURVEY.md
// section 5), with the reference's defaults (carbon_sim.cfg:276-313, 375-392).
class CfgView
{
public:
   void set(const std::string& key, const std::string& value) { _kv[key] = value; }
   int getInt(const std::string& key, int dflt) const;
   bool getBool(const std::string& key, bool dflt) const;
   double getFloat(const std::string& key, double dflt) const;
   std::string getString(const std::string& key, const std::string& dflt) const;
   // gnoc_config for general/total_cores tiles, as NetworkModelEMeshHopByHop's ctor reads it
   gnoc_config toEngineConfig() const;
   // queue_model/basic/moving_avg_* -> GNOC_MOVING_AVG_* and window size
   void basicMovingAverage(int32_t* type, uint32_t* window) const;

private:
   std::map<std::string, std::string> _kv;
};

// Trace-mode NetPacket: the fields this path reads (network.h:27-55).
struct NetPacket
{
   static constexpr int32_t BROADCAST = (int32_t) 0xDEADBABE;   // network.h:54
   uint64_t time = 0;          // NetPacket::time at netSend, picoseconds
   int32_t sender = 0;         // TILE_ID(pkt.sender)
   int32_t receiver = 0;       // TILE_ID(pkt.receiver)
   uint32_t modeled_bits = 0;  // NetworkModel::getModeledLength(pkt)
   bool modeled = true;        // NetworkModel::isModelEnabled(pkt)
   // outputs, filled by run(): NetPacket fields after processReceivedPacket
   uint64_t zero_load_delay = 0;
   uint64_t contention_delay = 0;
};

class NetworkModelEMeshHopByHopHIP
{
public:
   static constexpr const char* kTypeName = "emesh_hop_by_hop_hip";

   explicit NetworkModelEMeshHopByHopHIP(const CfgView& cfg, int device = 0);
   explicit NetworkModelEMeshHopByHopHIP(const gnoc_config& cfg);
   ~NetworkModelEMeshHopByHopHIP();
   NetworkModelEMeshHopByHopHIP(const NetworkModelEMeshHopByHopHIP&) = delete;
   NetworkModelEMeshHopByHopHIP& operator=(const NetworkModelEMeshHopByHopHIP&) = delete;

   // NetworkModel::__routePacket at SEND_TILE, trace mode: record one packet.
   // Packets must arrive in (time, id) order, as the reference's event loop
   // hands them to the model.  Returns the packet id (its index).
   uint32_t routePacket(const NetPacket& pkt);
   void reserve(size_t n);

   // Time every hop of every recorded packet (one gnoc_submit + gnoc_run).
   // queue_model/basic/moving_avg_* on this model's basic queues (GNOC_MOVING_AVG_*;
   // queue_model_basic.cc:7-30).  Written into captured traces (header v2) and
   // applied by fromTraceFile; a version-1 trace replays with NONE unless set here.
   void setBasicMovingAverage(int32_t type, uint32_t window);
   void run();

   // Results of the last run(), indexed by packet id: NetPacket::time,
   // zero_load_delay, contention_delay after processReceivedPacket.
   const std::vector<uint64_t>& packetTime() const { return _final; }
   const std::vector<uint64_t>& packetZeroLoadDelay() const { return _zl; }
   const std::vector<uint64_t>& packetContentionDelay() const { return _ct; }
   // A broadcast's receipt at `tile` (processReceivedPacket of the copy the
   // tree delivers there); the packetTime() entry is its latest receipt.
   uint64_t broadcastReceiptTime(uint32_t id, int tile) const;
   uint64_t broadcastReceiptZeroLoadDelay(uint32_t id, int tile) const;
   uint64_t broadcastReceiptContentionDelay(uint32_t id, int tile) const;

   // RouterModel::_total_contention_delay / _total_packets per output port
   // (index tile*6 + GNOC_PORT_*; GNOC_PORT_INJ = the injection router) and
   // QueueModelHistoryTree::getTotalRequestsUsingAnalyticalModel.
   const std::vector<uint64_t>& portContentionDelay() const { return _psum; }
   const std::vector<uint64_t>& portPackets() const { return _pcnt; }
   const std::vector<uint64_t>& portAnalyticalRequests() const { return _pmg1; }
   // QueueModel utilization operands per output port (queue_model.cc:49-53):
   // _total_utilized_cycles (flits) and _last_request_time (cycles).
   const std::vector<uint64_t>& portUtilizedCycles() const { return _pflit; }
   const std::vector<uint64_t>& portLastRequestTime() const { return _plast; }

   // Mesh-router event counters of a tile (RouterModel::updateEventCounters,
   // router_model.cc:119-127; ElectricalLinkModel::processPacket,
   // electrical_link_model.cc:29-45): flits through the router (= buffer
   // writes = buffer reads), packets through it (= switch allocator
   // requests), crossbar traversals by number of output ports (1..5; a
   // broadcast visit uses several) and flits over its links.  Route-static.
   uint64_t routerFlits(int tile) const;
   uint64_t routerPackets(int tile) const;
   uint64_t routerCrossbarTraversals(int tile, int ports) const;
   uint64_t routerLinkTraversals(int tile) const;

   // The per-tile sim.out network section of NetworkModelEMeshHopByHop::outputSummary
   // (network_model_emesh_hop_by_hop.cc:299-306): NetworkModel::outputSummary
   // (network_model.cc:274-316), the event counters (:436-468) and, when the
   // queue models are enabled, the contention counters (:471-493,
   // router_model.cc:146-215).  Power modelling is off (no power section).
   void outputSummary(std::ostream& out, int tile) const;

   gnoc_summary summary() const;
   int numTiles() const { return _cfg.num_tiles; }
   int meshWidth() const { return _cfg.mesh_width; }
   int meshHeight() const { return _cfg.mesh_height; }
   size_t numPackets() const { return _inj.size(); }

   // Static capability hooks (network_model_emesh_hop_by_hop.cc:309-364).
   static bool isTileCountPermissible(int tile_count);
   static std::vector<int> computeMemoryControllerPositions(int num_memory_controllers, int tile_count);

   // On-disk traces (include/gnoc.h, gnoc_trace_header).
   void writeTrace(const std::string& path) const;
   static NetworkModelEMeshHopByHopHIP* fromTraceFile(const std::string& path, int device = 0);

private:
   void check(int status, const char* what) const;

   gnoc_config _cfg;
   gnoc_trace_queue _queue{GNOC_MOVING_AVG_NONE, 1};   // basic queues' moving average
   gnoc_engine* _eng = nullptr;
   std::vector<uint64_t> _inj;
   std::vector<uint32_t> _src, _dst, _bits, _flags;
   std::vector<uint64_t> _final, _zl, _ct, _psum, _pcnt, _pmg1, _pflit, _plast;
   std::vector<uint32_t> _bidx;                    // packet id -> broadcast index (broadcasts only)
   std::vector<uint64_t> _bfin, _bzl, _bct;        // broadcast receipts [b * N + tile]
   mutable std::vector<uint64_t> _rflit, _rpkt, _rxbar, _rlink;   // event counters, built on first use
   size_t receipt(uint32_t id, int tile) const;
   void buildEventCounters() const;
   bool _ran = false;
};

}  // namespace graphite_amd
