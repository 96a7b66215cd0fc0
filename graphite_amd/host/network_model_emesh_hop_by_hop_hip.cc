// network_model_emesh_hop_by_hop_hip.cc -- see the header for the reference
// interface each member mirrors.  Host C++ only; all timing runs behind the
// C ABI in libgnoc.so (include/gnoc.h).
#include "network_model_emesh_hop_by_hop_hip.h"

#include <cmath>
#include <cstdlib>
#include <cstring>

namespace graphite_amd {

// ---------------------------------------------------------------------------
// CfgView: Sim()->getCfg()->get{Int,Bool,Float,String}(key, default)
// ---------------------------------------------------------------------------
int CfgView::getInt(const std::string& key, int dflt) const
{
   auto it = _kv.find(key);
   return it == _kv.end() ? dflt : (int) std::strtol(it->second.c_str(), nullptr, 0);
}

bool CfgView::getBool(const std::string& key, bool dflt) const
{
   auto it = _kv.find(key);
   if (it == _kv.end()) return dflt;
   const std::string& v = it->second;
   return v == "true" || v == "1" || v == "yes";
}

double CfgView::getFloat(const std::string& key, double dflt) const
{
   auto it = _kv.find(key);
   return it == _kv.end() ? dflt : std::strtod(it->second.c_str(), nullptr);
}

std::string CfgView::getString(const std::string& key, const std::string& dflt) const
{
   auto it = _kv.find(key);
   return it == _kv.end() ? dflt : it->second;
}

gnoc_config CfgView::toEngineConfig() const
{
   gnoc_config c;
   const int tiles = getInt("general/total_cores", 64);                         // carbon_sim.cfg:34
   gnoc_config_default(&c, tiles);
   c.flit_width = getInt("network/emesh_hop_by_hop/flit_width", 64);             // emesh_hop_by_hop.cc:22
   c.broadcast_tree_enabled = getBool("network/emesh_hop_by_hop/broadcast_tree_enabled", true);   // :25
   c.router_delay = (uint64_t) getInt("network/emesh_hop_by_hop/router/delay", 1);                // :95
   c.link_delay = (uint64_t) getInt("network/emesh_hop_by_hop/link/delay", 1);                    // :96
   c.contention_enabled = getBool("network/emesh_hop_by_hop/queue_model/enabled", true);          // :97
   const std::string qt = getString("network/emesh_hop_by_hop/queue_model/type", "history_tree"); // :98
   // QueueModel::create (queue_model.cc:18-38) and each model's keys (carbon_sim.cfg:376-392)
   c.queue_type = qt == "history_tree" ? GNOC_QUEUE_HISTORY_TREE
                : qt == "basic" ? GNOC_QUEUE_BASIC
                : qt == "history_list" ? GNOC_QUEUE_HISTORY_LIST : -1;
   const std::string qk = qt == "history_list" ? "queue_model/history_list/" : "queue_model/history_tree/";
   c.analytical_enabled = getBool(qk + "analytical_model_enabled", true);
   c.max_list_size = getInt(qk + "max_list_size", 100);
   c.tile_width_mm = getFloat("general/tile_width", 1.0);                                        // carbon_sim.cfg:64
   c.frequency_ghz = getFloat("network/frequency", 1.0);   // the network's DVFS domain (dvfs_manager.cc:243-250)
   return c;
}

// ---------------------------------------------------------------------------
// NetworkModelEMeshHopByHopHIP
// ---------------------------------------------------------------------------
NetworkModelEMeshHopByHopHIP::NetworkModelEMeshHopByHopHIP(const CfgView& cfg, int device)
   : NetworkModelEMeshHopByHopHIP([&] {
        gnoc_config c = cfg.toEngineConfig();
        c.device = device;
        return c;
     }())
{
   int32_t type = GNOC_MOVING_AVG_NONE;
   uint32_t window = 1;
   cfg.basicMovingAverage(&type, &window);
   if (_cfg.queue_type == GNOC_QUEUE_BASIC && type != GNOC_MOVING_AVG_NONE) setBasicMovingAverage(type, window);
}

// QueueModelBasic::QueueModelBasic (queue_model_basic.cc:7-30) with its code
// defaults: moving_avg_enabled false, window 1, type "none" (:17-19); a
// carbon_sim.cfg supplies its own values when present.  An unknown type string
// leaves the queue without a moving average, as createAvgType's NULL does
// (moving_average.h:184-188).
void CfgView::basicMovingAverage(int32_t* type, uint32_t* window) const
{
   *type = GNOC_MOVING_AVG_NONE;
   *window = 1;
   if (!getBool("queue_model/basic/moving_avg_enabled", false)) return;
   const std::string t = getString("queue_model/basic/moving_avg_type", "none");
   *type = t == "arithmetic_mean" ? GNOC_MOVING_AVG_ARITHMETIC_MEAN
         : t == "geometric_mean"  ? GNOC_MOVING_AVG_GEOMETRIC_MEAN
         : t == "median"          ? GNOC_MOVING_AVG_MEDIAN : GNOC_MOVING_AVG_NONE;
   *window = (uint32_t) getInt("queue_model/basic/moving_avg_window_size", 1);
}

NetworkModelEMeshHopByHopHIP::NetworkModelEMeshHopByHopHIP(const gnoc_config& cfg) : _cfg(cfg)
{
   if (_cfg.queue_type < 0)
      throw NetworkModelError(GNOC_EINVAL, "queue_model/type: unrecognized queue model");   // queue_model.cc:33-36
   const int rc = gnoc_create(&_cfg, &_eng);
   if (rc)
      throw NetworkModelError(rc, "gnoc_create rejected the emesh_hop_by_hop configuration (status " +
                                      std::to_string(rc) + ")");
   // derived topology (initializeEMeshTopologyParams, emesh_hop_by_hop.cc:47-70)
   if (_cfg.mesh_width <= 0 || _cfg.mesh_height <= 0)
   {
      _cfg.mesh_width = (int32_t) std::floor(std::sqrt((double) _cfg.num_tiles));
      _cfg.mesh_height = (int32_t) std::ceil(1.0 * _cfg.num_tiles / _cfg.mesh_width);
   }
}

NetworkModelEMeshHopByHopHIP::~NetworkModelEMeshHopByHopHIP() { gnoc_destroy(_eng); }

void NetworkModelEMeshHopByHopHIP::setBasicMovingAverage(int32_t type, uint32_t window)
{
   check(gnoc_set_basic_moving_average(_eng, type, window), "queue_model/basic moving average");
   _queue.ma_type = type;
   _queue.ma_window = window;
}

void NetworkModelEMeshHopByHopHIP::check(int status, const char* what) const
{
   if (status) throw NetworkModelError(status, std::string(what) + ": " + gnoc_last_error(_eng));
}

void NetworkModelEMeshHopByHopHIP::reserve(size_t n)
{
   _inj.reserve(n);
   _src.reserve(n);
   _dst.reserve(n);
   _bits.reserve(n);
   _flags.reserve(n);
}

uint32_t NetworkModelEMeshHopByHopHIP::routePacket(const NetPacket& pkt)
{
   // NetworkModel::__routePacket asserts (network_model.cc:109-113), here as errors
   const bool bc = pkt.receiver == NetPacket::BROADCAST;
   if (pkt.sender < 0 || pkt.sender >= _cfg.num_tiles || (!bc && (pkt.receiver < 0 || pkt.receiver >= _cfg.num_tiles)))
      throw NetworkModelError(GNOC_ETRACE, "pkt_sender/pkt_receiver outside the application tiles");
   // hasBroadcastCapability() is broadcast_tree_enabled (emesh_hop_by_hop.cc:25); without
   // it Network::netSend hands the model one unicast per tile (network.cc:186-195)
   if (bc && !_cfg.broadcast_tree_enabled)
      throw NetworkModelError(GNOC_EINVAL, "broadcast without broadcast_tree_enabled: Network::netSend expands it");
   if (!_inj.empty() && pkt.time < _inj.back())
      throw NetworkModelError(GNOC_ETRACE, "packets must be routed in time order");
   _inj.push_back(pkt.time);
   _src.push_back((uint32_t) pkt.sender);
   _dst.push_back(bc ? (uint32_t) pkt.sender : (uint32_t) pkt.receiver);
   _bits.push_back(pkt.modeled_bits);
   _flags.push_back((pkt.modeled ? 0u : GNOC_PKT_UNMODELED) | (bc ? GNOC_PKT_BROADCAST : 0u));
   _ran = false;
   return (uint32_t) (_inj.size() - 1);
}

void NetworkModelEMeshHopByHopHIP::run()
{
   gnoc_packets pk;
   pk.inject_ps = _inj.data();
   pk.src = _src.data();
   pk.dst = _dst.data();
   pk.bits = _bits.data();
   pk.flags = _flags.data();
   const size_t n = _inj.size();
   check(gnoc_submit(_eng, &pk, n), "gnoc_submit");
   check(gnoc_run(_eng), "gnoc_run");
   _final.resize(n);
   _zl.resize(n);
   _ct.resize(n);
   check(gnoc_get_packet_results(_eng, _final.data(), _zl.data(), _ct.data(), n), "gnoc_get_packet_results");
   const size_t np = (size_t) _cfg.num_tiles * GNOC_PORTS_PER_TILE;
   _psum.resize(np);
   _pcnt.resize(np);
   _pmg1.resize(np);
   check(gnoc_get_port_stats(_eng, _psum.data(), _pcnt.data(), _pmg1.data(), np), "gnoc_get_port_stats");
   _pflit.resize(np);
   _plast.resize(np);
   check(gnoc_get_port_utilization(_eng, _pflit.data(), _plast.data(), np), "gnoc_get_port_utilization");
   _bidx.assign(n, 0xFFFFFFFFu);
   uint32_t nb = 0;
   for (size_t i = 0; i < n; i++)
      if (_flags[i] & GNOC_PKT_BROADCAST) _bidx[i] = nb++;
   const size_t nv = (size_t) nb * _cfg.num_tiles;
   _bfin.resize(nv);
   _bzl.resize(nv);
   _bct.resize(nv);
   check(gnoc_get_broadcast_results(_eng, _bfin.data(), _bzl.data(), _bct.data(), nv), "gnoc_get_broadcast_results");
   _rflit.clear();
   _rpkt.clear();
   _ran = true;
}

size_t NetworkModelEMeshHopByHopHIP::receipt(uint32_t id, int tile) const
{
   if (!_ran) throw NetworkModelError(GNOC_ESTATE, "no results before run()");
   if (id >= _bidx.size() || _bidx[id] == 0xFFFFFFFFu) throw NetworkModelError(GNOC_EINVAL, "not a broadcast packet");
   if (tile < 0 || tile >= _cfg.num_tiles) throw NetworkModelError(GNOC_EINVAL, "tile outside the mesh");
   return (size_t) _bidx[id] * _cfg.num_tiles + (size_t) tile;
}
uint64_t NetworkModelEMeshHopByHopHIP::broadcastReceiptTime(uint32_t id, int tile) const { return _bfin[receipt(id, tile)]; }
uint64_t NetworkModelEMeshHopByHopHIP::broadcastReceiptZeroLoadDelay(uint32_t id, int tile) const
{
   return _bzl[receipt(id, tile)];
}
uint64_t NetworkModelEMeshHopByHopHIP::broadcastReceiptContentionDelay(uint32_t id, int tile) const
{
   return _bct[receipt(id, tile)];
}

gnoc_summary NetworkModelEMeshHopByHopHIP::summary() const
{
   gnoc_summary s;
   check(gnoc_get_summary(_eng, &s), "gnoc_get_summary");
   return s;
}

// Time::toCycles / toNanosec (common/misc/time_types.h:99-109)
static uint64_t ps_to_cycles(uint64_t ps, double f) { return (uint64_t) std::ceil(((double) ps * f) / 1.0e3); }
static uint64_t ps_to_ns(uint64_t ps) { return (uint64_t) std::ceil(((double) ps) / 1.0e3); }

// Every routed packet traverses the mesh routers of its source row from sx to
// dx, then of column dx up to dy (XY routing, emesh_hop_by_hop.cc:229-240):
// segment sums with difference arrays, O(packets + tiles).
void NetworkModelEMeshHopByHopHIP::buildEventCounters() const
{
   const int W = _cfg.mesh_width, H = _cfg.mesh_height;
   const uint32_t fw = (uint32_t) _cfg.flit_width;
   std::vector<int64_t> rf((size_t) (W + 1) * H, 0), rp((size_t) (W + 1) * H, 0);
   std::vector<int64_t> cf((size_t) (H + 1) * W, 0), cp((size_t) (H + 1) * W, 0);
   _rxbar.assign((size_t) W * H * 5, 0);
   _rlink.assign((size_t) W * H, 0);
   std::vector<uint64_t> bflit((size_t) W * H, 0), bpkt((size_t) W * H, 0);
   for (size_t i = 0; i < _inj.size(); i++)
   {
      if (_flags[i] & GNOC_PKT_UNMODELED) continue;
      const int64_t F = (_bits[i] % fw) ? _bits[i] / fw + 1 : _bits[i] / fw;
      if (_flags[i] & GNOC_PKT_BROADCAST)
      {
         // the tree visits every router once, selecting UP/DOWN/RIGHT/LEFT/SELF
         // (emesh_hop_by_hop.cc:170-204): crossbar[#ports], one link per port
         const int sx = (int) _src[i] % W, sy = (int) _src[i] / W;
         for (int t = 0; t < W * H; t++)
         {
            const int cx = t % W, cy = t / W;
            int np = 1;
            np += (cy >= sy && cy + 1 < H);
            np += (cy <= sy && cy >= 1);
            if (cy == sy) np += (cx >= sx && cx + 1 < W) + (cx <= sx && cx >= 1);
            bflit[t] += (uint64_t) F;
            bpkt[t] += 1;
            _rxbar[(size_t) t * 5 + np - 1] += (uint64_t) F;
            _rlink[t] += (uint64_t) (F * np);
         }
         continue;
      }
      if (_src[i] == _dst[i]) continue;
      const int sx = (int) _src[i] % W, sy = (int) _src[i] / W, dx = (int) _dst[i] % W, dy = (int) _dst[i] / W;
      const int x0 = sx < dx ? sx : dx, x1 = sx < dx ? dx : sx;
      rf[(size_t) sy * (W + 1) + x0] += F;
      rf[(size_t) sy * (W + 1) + x1 + 1] -= F;
      rp[(size_t) sy * (W + 1) + x0] += 1;
      rp[(size_t) sy * (W + 1) + x1 + 1] -= 1;
      if (dy != sy)
      {
         const int y0 = dy > sy ? sy + 1 : dy, y1 = dy > sy ? dy : sy - 1;
         cf[(size_t) dx * (H + 1) + y0] += F;
         cf[(size_t) dx * (H + 1) + y1 + 1] -= F;
         cp[(size_t) dx * (H + 1) + y0] += 1;
         cp[(size_t) dx * (H + 1) + y1 + 1] -= 1;
      }
   }
   _rflit.assign((size_t) W * H, 0);
   _rpkt.assign((size_t) W * H, 0);
   for (int y = 0; y < H; y++)
   {
      int64_t a = 0, b = 0;
      for (int x = 0; x < W; x++)
      {
         a += rf[(size_t) y * (W + 1) + x];
         b += rp[(size_t) y * (W + 1) + x];
         _rflit[(size_t) y * W + x] += (uint64_t) a;
         _rpkt[(size_t) y * W + x] += (uint64_t) b;
      }
   }
   for (int x = 0; x < W; x++)
   {
      int64_t a = 0, b = 0;
      for (int y = 0; y < H; y++)
      {
         a += cf[(size_t) x * (H + 1) + y];
         b += cp[(size_t) x * (H + 1) + y];
         _rflit[(size_t) y * W + x] += (uint64_t) a;
         _rpkt[(size_t) y * W + x] += (uint64_t) b;
      }
   }
   // a unicast hop crosses the crossbar to one port and one link
   for (size_t t = 0; t < (size_t) W * H; t++)
   {
      _rxbar[t * 5] += _rflit[t];
      _rlink[t] += _rflit[t];
      _rflit[t] += bflit[t];
      _rpkt[t] += bpkt[t];
   }
}

uint64_t NetworkModelEMeshHopByHopHIP::routerCrossbarTraversals(int tile, int ports) const
{
   if (_rpkt.empty()) buildEventCounters();
   if (ports < 1 || ports > 5) throw NetworkModelError(GNOC_EINVAL, "crossbar port count outside 1..5");
   return _rxbar.at((size_t) tile * 5 + ports - 1);
}

uint64_t NetworkModelEMeshHopByHopHIP::routerLinkTraversals(int tile) const
{
   if (_rpkt.empty()) buildEventCounters();
   return _rlink.at((size_t) tile);
}

uint64_t NetworkModelEMeshHopByHopHIP::routerFlits(int tile) const
{
   if (_rflit.empty()) buildEventCounters();
   return _rflit.at((size_t) tile);
}

uint64_t NetworkModelEMeshHopByHopHIP::routerPackets(int tile) const
{
   if (_rpkt.empty()) buildEventCounters();
   return _rpkt.at((size_t) tile);
}

void NetworkModelEMeshHopByHopHIP::outputSummary(std::ostream& out, int tile) const
{
   if (!_ran) throw NetworkModelError(GNOC_ESTATE, "outputSummary before run()");
   if (tile < 0 || tile >= _cfg.num_tiles) throw NetworkModelError(GNOC_EINVAL, "tile outside the mesh");
   const uint32_t fw = (uint32_t) _cfg.flit_width;
   auto flits = [&](uint32_t bits) -> uint64_t { return (bits % fw) ? bits / fw + 1 : bits / fw; };
   // updateSendCounters / updateReceiveCounters (network_model.cc:229-272): modeled,
   // non-self packets; a broadcast counts as sent and broadcasted at its sender
   // and as received, with that receipt's delays, at every tile.
   uint64_t ps = 0, fs = 0, bs = 0, pb = 0, fb = 0, bb = 0, pr = 0, fr = 0, br = 0, lat = 0, cont = 0;
   for (size_t i = 0; i < _inj.size(); i++)
   {
      if (_flags[i] & GNOC_PKT_UNMODELED) continue;
      if (_flags[i] & GNOC_PKT_BROADCAST)
      {
         if ((int) _src[i] == tile)
         {
            ps++; fs += flits(_bits[i]); bs += _bits[i];
            pb++; fb += flits(_bits[i]); bb += _bits[i];
         }
         const size_t k = receipt((uint32_t) i, tile);
         pr++;
         fr += flits(_bits[i]);
         br += _bits[i];
         lat += _bzl[k] + _bct[k];
         cont += _bct[k];
         continue;
      }
      if (_src[i] == _dst[i]) continue;
      if ((int) _src[i] == tile) { ps++; fs += flits(_bits[i]); bs += _bits[i]; }
      if ((int) _dst[i] == tile)
      {
         pr++;
         fr += flits(_bits[i]);
         br += _bits[i];
         lat += _zl[i] + _ct[i];
         cont += _ct[i];
      }
   }
   const double f = _cfg.frequency_ghz;
   out << "    Total Packets Sent: " << ps << "\n";
   out << "    Total Flits Sent: " << fs << "\n";
   out << "    Total Bits Sent: " << bs << "\n";
   out << "    Total Packets Broadcasted: " << pb << "\n";
   out << "    Total Flits Broadcasted: " << fb << "\n";
   out << "    Total Bits Broadcasted: " << bb << "\n";
   out << "    Total Packets Received: " << pr << "\n";
   out << "    Total Flits Received: " << fr << "\n";
   out << "    Total Bits Received: " << br << "\n";
   if (pr > 0)
   {
      out << "    Average Packet Latency (in clock cycles): " << ((float) ps_to_cycles(lat, f)) / pr << "\n";
      out << "    Average Packet Latency (in nanoseconds): " << ((float) ps_to_ns(lat)) / pr << "\n";
      out << "    Average Contention Delay (in clock cycles): " << ((float) ps_to_cycles(cont, f)) / pr << "\n";
      out << "    Average Contention Delay (in nanoseconds): " << ((float) ps_to_ns(cont)) / pr << "\n";
   }
   else
   {
      out << "    Average Packet Latency (in clock cycles): 0\n";
      out << "    Average Packet Latency (in nanoseconds): 0\n";
      out << "    Average Contention Delay (in clock cycles): 0\n";
      out << "    Average Contention Delay (in nanoseconds): 0\n";
   }
   // outputEventCountSummary (:436-468)
   const uint64_t rfl = routerFlits(tile);
   out << "    Event Counters:\n";
   out << "      Buffer Writes: " << rfl << "\n";
   out << "      Buffer Reads: " << rfl << "\n";
   out << "      Switch Allocator Requests: " << routerPackets(tile) << "\n";
   for (int i = 1; i <= 5; i++) out << "      Crossbar[" << i << "] Traversals: " << routerCrossbarTraversals(tile, i) << "\n";
   out << "      Link Traversals: " << routerLinkTraversals(tile) << "\n";
   if (!_cfg.contention_enabled) return;   // emesh_hop_by_hop.cc:304-305
   // outputContentionModelsSummary: the mesh router's 5 output ports
   uint64_t sd = 0, sp = 0, sa = 0;
   float lu = 0.0f;
   for (int p = 0; p < 5; p++)
   {
      const size_t k = (size_t) tile * GNOC_PORTS_PER_TILE + p;
      sd += _psum[k];
      sp += _pcnt[k];
      sa += _pmg1[k];
      // QueueModel::getQueueUtilization (queue_model.cc:56-62)
      lu += (_plast[k] > 0) ? (((float) _pflit[k]) / _plast[k]) : 0.0f;
   }
   lu = lu / 5;   // RouterModel::getAverageLinkUtilization (router_model.cc:167-183)
   out << "    Contention Counters:\n";
   out << "      Average EMesh Router Contention Delay: " << (sp > 0 ? ((float) sd) / sp : 0.0f) << "\n";
   out << "      Average EMesh Router Link Utilization: " << lu << "\n";
   out << "      Analytical Models Used (%): " << (sp > 0 ? ((float) sa * 100) / sp : 0.0f) << "\n";
}

bool NetworkModelEMeshHopByHopHIP::isTileCountPermissible(int tile_count)
{
   const int w = (int) std::floor(std::sqrt((double) tile_count));
   const int h = (int) std::ceil(1.0 * tile_count / w);
   return tile_count == w * h;
}

std::vector<int> NetworkModelEMeshHopByHopHIP::computeMemoryControllerPositions(int num, int tile_count)
{
   const int W = (int) std::floor(std::sqrt((double) tile_count));
   const int H = (int) std::ceil(1.0 * tile_count / W);
   const int mw = (int) std::floor(std::sqrt((double) num));
   const int mh = (int) std::ceil(1.0 * num / mw);
   std::vector<int> out;
   for (int j = 0; j < mh && (int) out.size() < num; j++)
      for (int i = 0; i < mw && (int) out.size() < num; i++)
      {
         int sx = W / mw, sy = H / mh;
         const int bx = i * sx, by = j * sy;
         if (i == mw - 1) sx = W - (mw - 1) * sx;
         if (j == mh - 1) sy = H - (mh - 1) * sy;
         out.push_back((bx + sx / 2) + (by + sy / 2) * W);
      }
   return out;
}

void NetworkModelEMeshHopByHopHIP::writeTrace(const std::string& path) const
{
   gnoc_packets pk;
   pk.inject_ps = _inj.data();
   pk.src = _src.data();
   pk.dst = _dst.data();
   pk.bits = _bits.data();
   pk.flags = _flags.data();
   const int rc = gnoc_trace_file_write_q(path.c_str(), &_cfg, &_queue, &pk, _inj.size());
   if (rc) throw NetworkModelError(rc, "cannot write trace " + path);
}

NetworkModelEMeshHopByHopHIP* NetworkModelEMeshHopByHopHIP::fromTraceFile(const std::string& path, int device)
{
   gnoc_config cfg;
   gnoc_trace_queue q;
   size_t n = 0;
   int rc = gnoc_trace_file_read_q(path.c_str(), &cfg, &q, nullptr, nullptr, nullptr, nullptr, nullptr, 0, &n);
   if (rc) throw NetworkModelError(rc, "cannot read trace " + path);
   cfg.device = device;
   auto* m = new NetworkModelEMeshHopByHopHIP(cfg);
   if (cfg.queue_type == GNOC_QUEUE_BASIC && q.ma_type != GNOC_MOVING_AVG_NONE)
   {
      try
      {
         m->setBasicMovingAverage(q.ma_type, q.ma_window);   // the settings the trace was captured under
      }
      catch (...)
      {
         delete m;
         throw;
      }
   }
   m->_inj.resize(n);
   m->_src.resize(n);
   m->_dst.resize(n);
   m->_bits.resize(n);
   m->_flags.resize(n);
   rc = gnoc_trace_file_read(path.c_str(), nullptr, m->_inj.data(), m->_src.data(), m->_dst.data(), m->_bits.data(),
                             m->_flags.data(), n, &n);
   if (rc)
   {
      delete m;
      throw NetworkModelError(rc, "corrupt trace " + path);
   }
   return m;
}

}  // namespace graphite_amd
