"""Expected sim.out network section of one tile, restated from the reference
from per-packet and per-port results (test helper; the oracle supplies the
results).  Float arithmetic in float32 and C++ ostream formatting (%g, 6
significant digits), as the reference prints them.

  NetworkModel::outputSummary                     network_model.cc:274-316
    send / receive counters                       network_model.cc:229-272, 95-140
  NetworkModelEMeshHopByHop::outputEventCountSummary      network_model_emesh_hop_by_hop.cc:436-468
    RouterModel::updateEventCounters              router_model.cc:119-127
    ElectricalLinkModel::processPacket            electrical_link_model.cc:29-45
  NetworkModelEMeshHopByHop::outputContentionModelsSummary  network_model_emesh_hop_by_hop.cc:471-493
    RouterModel::getAverage*                      router_model.cc:146-215
    QueueModel::getQueueUtilization               queue_model.cc:56-62
"""
import math

import numpy as np

f32 = np.float32


def cfmt(v) -> str:
    """std::ostream << float (default precision 6)."""
    return "%g" % float(f32(v))


def _ceil_div_1000(ps: int) -> int:
    return int(math.ceil(float(ps) / 1.0e3))


def expected_summary(cfg, tr, res, tile: int) -> str:
    W, H = cfg.width, cfg.height
    fw = cfg.flit_width
    src, dst, bits = tr.src.astype(np.int64), tr.dst.astype(np.int64), tr.bits.astype(np.int64)
    flags = tr.flags if tr.flags is not None else np.zeros(len(src), np.uint32)
    F = (bits + fw - 1) // fw
    bcast = (flags & 2) != 0
    modeled = (flags & 1) == 0
    live = (src != dst) & modeled & ~bcast
    bc = bcast & modeled                      # routed on the broadcast tree
    brow = np.cumsum(bcast) - 1               # row of each broadcast in res.bcast_*
    s = (live | bc) & (src == tile)
    sb = bc & (src == tile)
    r = live & (dst == tile)
    lat = int((res.zero_load_ps[r].astype(np.int64) + res.contention_ps[r].astype(np.int64)).sum())
    cont = int(res.contention_ps[r].astype(np.int64).sum())
    pr = int(r.sum())
    fr, br = int(F[r].sum()), int(bits[r].sum())
    inj = tr.inject_ps.astype(np.int64)
    for i in np.nonzero(bc)[0]:
        # every tile receives a broadcast once (NetworkModel::updateReceiveCounters per receipt)
        zl = int(res.bcast_zero_load_ps[brow[i], tile])
        ct = int(res.bcast_final_ps[brow[i], tile]) - int(inj[i]) - zl
        lat += zl + ct
        cont += ct
        pr += 1
        fr += int(F[i])
        br += int(bits[i])
    out = []
    out.append(f"    Total Packets Sent: {int(s.sum())}")
    out.append(f"    Total Flits Sent: {int(F[s].sum())}")
    out.append(f"    Total Bits Sent: {int(bits[s].sum())}")
    out.append(f"    Total Packets Broadcasted: {int(sb.sum())}")
    out.append(f"    Total Flits Broadcasted: {int(F[sb].sum())}")
    out.append(f"    Total Bits Broadcasted: {int(bits[sb].sum())}")
    out.append(f"    Total Packets Received: {pr}")
    out.append(f"    Total Flits Received: {fr}")
    out.append(f"    Total Bits Received: {br}")
    if pr > 0:
        f = cfg.frequency_ghz
        cyc = lambda ps: int(math.ceil((float(ps) * f) / 1.0e3))
        out.append("    Average Packet Latency (in clock cycles): " + cfmt(f32(cyc(lat)) / f32(pr)))
        out.append("    Average Packet Latency (in nanoseconds): " + cfmt(f32(_ceil_div_1000(lat)) / f32(pr)))
        out.append("    Average Contention Delay (in clock cycles): " + cfmt(f32(cyc(cont)) / f32(pr)))
        out.append("    Average Contention Delay (in nanoseconds): " + cfmt(f32(_ceil_div_1000(cont)) / f32(pr)))
    else:
        out += ["    Average Packet Latency (in clock cycles): 0", "    Average Packet Latency (in nanoseconds): 0",
                "    Average Contention Delay (in clock cycles): 0", "    Average Contention Delay (in nanoseconds): 0"]
    # event counters: every routed packet crosses the mesh routers of its XY route
    tx, ty = tile % W, tile // W
    sx, sy, dx, dy = src % W, src // W, dst % W, dst // W
    on_row = live & (sy == ty) & (np.minimum(sx, dx) <= tx) & (tx <= np.maximum(sx, dx))
    on_col = live & (dx == tx) & (dy != sy) & (((dy > sy) & (sy < ty) & (ty <= dy)) | ((dy < sy) & (dy <= ty) & (ty < sy)))
    through = on_row | on_col
    fl = int(F[through].sum())
    xbar = [fl, 0, 0, 0, 0]
    link = fl
    sar = int(through.sum())
    # broadcasts: the tree visits this router once, with UP/DOWN/RIGHT/LEFT/SELF
    # selected as in emesh_hop_by_hop.cc:170-204 (crossbar[#ports], a link per port)
    for i in np.nonzero(bc)[0]:
        bx, by = int(sx[i]), int(sy[i])
        npt = 1 + int(ty >= by and ty + 1 < H) + int(ty <= by and ty >= 1)
        if ty == by:
            npt += int(tx >= bx and tx + 1 < W) + int(tx <= bx and tx >= 1)
        fl += int(F[i])
        sar += 1
        xbar[npt - 1] += int(F[i])
        link += int(F[i]) * npt
    out.append("    Event Counters:")
    out.append(f"      Buffer Writes: {fl}")
    out.append(f"      Buffer Reads: {fl}")
    out.append(f"      Switch Allocator Requests: {sar}")
    for i in range(1, 6):
        out.append(f"      Crossbar[{i}] Traversals: {xbar[i - 1]}")
    out.append(f"      Link Traversals: {link}")
    if cfg.contention_enabled:
        k = tile * 6 + np.arange(5)
        sd, sp, sa = (int(a[k].sum()) for a in (res.port_sum_delay, res.port_count, res.port_mg1))
        lu = f32(0.0)
        for q in k:
            last = int(res.port_last[q])
            lu = f32(lu + (f32(int(res.port_flit[q])) / f32(last) if last > 0 else f32(0.0)))
        lu = f32(lu / f32(5))
        out.append("    Contention Counters:")
        out.append("      Average EMesh Router Contention Delay: " + (cfmt(f32(sd) / f32(sp)) if sp else "0"))
        out.append("      Average EMesh Router Link Utilization: " + cfmt(lu))
        out.append("      Analytical Models Used (%): " + (cfmt(f32(f32(sa) * f32(100)) / f32(sp)) if sp else "0"))
    return "\n".join(out) + "\n"
