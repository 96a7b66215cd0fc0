#!/usr/bin/env python3
"""Benchmark: packet-hops simulated per second for Graphite's emesh_hop_by_hop
network model on MI355X (BASELINE.json metric), plus HBM-roofline fraction.

One step = one complete gnoc_run over a resident synthetic trace: every hop of
every packet through the per-port history-tree/M-G-1 queues, bit-exact with the
reference model (tests/test_gpu_parity.py).  Default workload = BASELINE.json
configs[1]: 32x32 (1024 tiles), uniform_random traffic, offered load 0.005
pkt/tile/cycle, 10,000 packets per tile (10.24 M packets, ~229 M mesh hops).

Multi-GPU (torchrun, one rank per GPU; default workload for N > 1 =
BASELINE.json configs[2]): ONE 64x64 mesh (4096 tiles, offered load 0.002,
10,000 packets per tile: 40.96 M packets, ~1.79 G mesh hops) sharded over the N
ranks (gnoc_shard, shard.hip): rank r runs the injection + X-direction ports of
its row band, one RCCL all-to-all over xGMI moves every packet's turn record to
the owner of its destination column band, and rank r runs the Y-direction and
SELF ports of its column band.  Total work is fixed, so scaling is "strong".
`--workload replicas` instead runs an independent 32x32 batch per rank (weak).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# torch first: libgnoc.so then binds to the same HIP runtime (SONAME libamdhip64.so.7)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
BYTES_PER_HOP = 32.0    # 16-B hop record written once + read once
BYTES_PER_PKT = 24.0    # trace read + final_ps write


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mesh", type=int, default=0, help="mesh side (default: 32, or 64 when sharded)")
    ap.add_argument("--load", type=float, default=0.0, help="offered load (default: 0.005 at 32x32, 0.002 at 64x64)")
    ap.add_argument("--ppt", type=int, default=10000, help="packets per tile")
    ap.add_argument("--mix", choices=("uniform", "hotspot"), default="uniform")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-sample-ppt", type=int, default=1000)
    ap.add_argument("--verify", type=int, default=0, help="also check the GPU result vs the oracle (slow)")
    ap.add_argument("--hotspot", type=int, default=1, help="also time the hotspot half of configs[1] (N=1 mesh)")
    ap.add_argument("--e2e", type=int, default=1, help="also time end to end (host trace -> host results)")
    ap.add_argument("--workload", choices=("auto", "mesh", "sharded", "replicas", "sweep"), default="auto",
                    help="auto: one 32x32 mesh at N=1, one 64x64 mesh sharded over N ranks at N>1")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (a one-GPU box): every rank on device 0, exchange over gloo
    if os.environ.get("GNOC_BENCH_ONE_GPU"):
        local = 0
    backend = os.environ.get("GNOC_BENCH_BACKEND", "nccl")   # nccl = RCCL over xGMI
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)

    from graphite_amd import gnoc
    import numpy as np

    wl = a.workload if a.workload != "auto" else ("mesh" if world == 1 else "sharded")
    if wl == "mesh" and world > 1:
        wl = "replicas"
    if wl == "sweep":
        return sweep_bench(a, world, rank, local)
    sharded = wl == "sharded"
    # BASELINE.json configs[1] (32x32, load 0.005) / configs[2] (64x64, load 0.002)
    W = H = a.mesh or (64 if sharded else 32)
    load = a.load or (0.002 if W == 64 else 0.005)
    hot = 0.2 if a.mix == "hotspot" else 0.0
    t0 = time.time()
    seed = a.seed + (rank if wl == "replicas" else 0)      # a sharded mesh: the same trace on every rank
    tr = gnoc.synthetic_trace(W, H, load, a.ppt, seed=seed, hotspot_fraction=hot, num_hotspots=16)
    gen_s = time.time() - t0
    cfg = gnoc.EngineConfig(num_tiles=W * H, device=local)
    # N > 1 over RCCL: the exchange inside libgnoc (gnoc_run_sharded on an RCCL
    # communicator of libgnoc's own, grouped ncclSend / ncclRecv on the engine's
    # stream); GNOC_BENCH_NATIVE=0 (or the gloo rehearsal) drives it from torch instead
    native = sharded and backend == "nccl" and os.environ.get("GNOC_BENCH_NATIVE", "1") != "0"
    comm = None
    if native:
        # the native path or nothing: a failure on any rank (gnoc_run_sharded max-reduces
        # its status, so a failing rank fails every rank instead of leaving one inside the
        # exchange) ends the bench with exit code 4 -- no silent switch to another exchange
        # (GNOC_BENCH_NATIVE=0 selects the torch-driven one explicitly)
        try:
            comm = gnoc.RcclComm(world, rank, local)
            eng = gnoc.NativeShardedEngine(cfg, rank, world, comm)
        except Exception as ex:   # noqa: BLE001 -- reported, then exit
            print(f"bench: rank {rank}: native RCCL path failed: {ex}", file=sys.stderr, flush=True)
            sys.exit(4)
    if not native:
        eng = gnoc.ShardedEngine(cfg, rank, world) if sharded else gnoc.Engine(cfg)
    eng.submit(tr)          # trace now resident in HBM; steps start from there

    def barrier_sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    m = measure(eng, a, barrier_sync, settle_fixed=sharded)
    elapsed, summ, kst, reruns = m["elapsed"], m["summary"], m["kst"], m["reruns"]

    # end to end (SURVEY.md 8(d) "trace resident in host memory -> results in host
    # memory"): submit from pinned host arrays (host-side trace validation + H2D),
    # run, final_ps back into a pinned host array; reported beside the HBM-resident value
    e2e_ms = e2e_serial_ms = e2e_wide_ms = e2e_fin_ms = e2e_narrow_ms = None
    wire = None
    if not sharded and a.e2e:
        ptr = pinned_trace(tr)
        fins = [torch.empty(len(tr), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64) for _ in range(2)]
        lats = [pinned_array(len(tr), np.uint32) for _ in range(2)]
        K = max(2, a.steps)   # batches per pipelined stream (the fill and the drain inside the clock)
        # the delta wire format (gnoc_packets_packed: u16 inject-time differences and
        # tile ids, lengths / flags only where they vary: 6 B per packet here) and the
        # narrow one (15 B) where the batch fits them, else the 24-B one
        pin = lambda shape, dt: pinned_array(shape[0], dt)   # noqa: E731
        try:
            ntr15 = gnoc.NarrowTrace.of(tr, alloc=pin)
            ktr = gnoc.PackedTrace.of(tr, alloc=pin)
            sub, sub_async, ntr, wire = eng.submit_packed, eng.submit_async_packed, ktr, ktr.wire_bytes() / len(tr)
        except ValueError:
            ntr15 = None
            ntr, sub, sub_async, wire = ptr, eng.submit, eng.submit_async, 24

        def pipelined(submit, submit_async, x, latency=False):
            # batch k+1's upload and batch k's read-back run on copy streams beside run k;
            # the read-back is final_ps (u64) or, narrow, the per-packet latency (u32)
            barrier_sync()
            t_e = time.perf_counter()
            submit(x)
            outs = lats if latency else fins
            for k in range(K):
                if k + 1 < K:
                    submit_async(x)
                eng.run()
                (eng.fetch_latency if latency else eng.fetch_final_ps)(outs[k % 2])
                if k + 1 < K:
                    eng.submit_commit()
            eng.fetch_wait()
            ms = (time.perf_counter() - t_e) / K * 1e3
            want = eng.results().final_ps
            if latency:
                want = (want - tr.inject_ps).astype(np.uint32)
            assert all(np.array_equal(f, want) for f in outs), "pipelined read-back differs from the run's results"
            return ms
        # untimed: the second trace buffers, copy streams, staging areas and latency
        # arrays get allocated
        for sa, x in ((sub_async, ntr), (eng.submit_async, ptr)) + (((eng.submit_async_narrow, ntr15),) if ntr15 else ()):
            sa(x)
            eng.submit_commit()
            eng.run()
            eng.fetch_final_ps(fins[0])
            eng.fetch_wait()
            eng.run()
            eng.fetch_latency(lats[0])
            eng.fetch_wait()
        # one batch at a time: submit (H2D + device checks), run, final_ps read-back
        barrier_sync()
        t_e = time.perf_counter()
        for _ in range(K):
            sub(ntr)
            eng.run()
            eng.final_ps_into(fins[0])
        e2e_serial_ms = (time.perf_counter() - t_e) / K * 1e3
        e2e_ms = pipelined(sub, sub_async, ntr, latency=True)
        e2e_fin_ms = pipelined(sub, sub_async, ntr)
        if ntr15 is not None:
            e2e_narrow_ms = pipelined(eng.submit_narrow, eng.submit_async_narrow, ntr15, latency=True)
        e2e_wide_ms = pipelined(eng.submit, eng.submit_async, ptr) if wire != 24 else e2e_fin_ms

    # this rank's share: mesh hops through the ports it owns, packets it delivers
    res = eng.results()
    pc = res.port_count.reshape(-1, 6)
    my_pkts = int(pc[:, 0].sum())
    hops = int(summ["mesh_hops"])
    pkts = int(summ["routed_packets"])
    t = torch.tensor([elapsed, float(hops), float(pkts)], dtype=torch.float64, device="cuda")
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax[0:1], op=dist.ReduceOp.MAX)
        if not sharded:   # replicas: every rank simulated its own batch
            dist.all_reduce(t[1:3], op=dist.ReduceOp.SUM)
        t[0] = tmax[0]
    elapsed_max, hops_all, pkts_all = float(t[0]), float(t[1]), float(t[2])

    if a.verify:
        from oracle import oracle
        got = eng.gathered_results() if sharded else res
        if rank == 0:
            ref = oracle.run(cfg, tr)
            assert np.array_equal(got.final_ps, ref.final_ps), "GPU result differs from oracle"

    # the other half of BASELINE configs[1] ("uniform-random + hotspot"): the same
    # mesh and load with 20 % of the packets sent to 16 hotspot tiles, one GPU
    hot_line = None
    if wl == "mesh" and world == 1 and a.mix == "uniform" and a.hotspot:
        eng.close()
        trh = gnoc.synthetic_trace(W, H, load, a.ppt, seed=seed, hotspot_fraction=0.2, num_hotspots=16)
        eng = gnoc.Engine(cfg)
        eng.submit(trh)
        mh = measure(eng, a, barrier_sync)
        rh = eng.results()
        pch = rh.port_count.reshape(-1, 6)
        hh = int(mh["summary"]["mesh_hops"])
        rfh = roofline(mh["kst"], pch, mh["summary"], int(pch[:, 0].sum()))
        hot_line = {"workload": f"emesh_hop_by_hop {W}x{H} hotspot(0.2, 16 tiles) load={load} pkts/tile={a.ppt}",
                    "value": hh * a.steps / mh["elapsed"], "ms_per_step": mh["elapsed"] / a.steps * 1e3,
                    "mesh_hops": hh, "engine_path": int(mh["summary"].get("engine_path", -1)),
                    "chain_protocol": chain_protocol(mh["summary"]),
                    "reruns": mh["reruns"], "roofline_frac": rfh["frac"], "kernel": rfh["kernel"],
                    "kernel_avg_us": rfh["kernel_avg_us"], "kernel_ms": {k: round(v[0], 4) for k, v in mh["kst"].items()}}

    if rank == 0:
        value = hops_all * a.steps / elapsed_max
        ms_step = elapsed_max / a.steps * 1e3
        rf = roofline(kst, pc, summ, my_pkts)
        whole_job_gbs = value * (BYTES_PER_HOP + BYTES_PER_PKT * pkts / max(hops, 1)) / 1e9 / world
        workload = f"emesh_hop_by_hop {W}x{H} {a.mix} load={load} pkts/tile={a.ppt}"
        bid = build_id()
        line = {
            "metric": "packet-hops simulated/sec (node) + % HBM roofline, 1024-tile emesh",
            "value": value,
            "unit": "packet-hops/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (synthetic_network.cc uniform_random restated, fixed seeds)",
            "config": {
                "workload": workload,
                "tiles": W * H, "packets": len(tr) * (world if wl == "replicas" else 1), "mesh_hops": int(hops_all),
                "flit_width": 64, "router_delay": 1, "link_delay": 1, "queue": "history_tree+mg1",
                "parallelism": (f"rowband/colband{world} + RCCL grouped send/recv in libgnoc" if native else
                                f"rowband/colband{world} + torch all-to-all ({backend})" if sharded and world > 1 else
                                f"replicas{world}" if world > 1 else "single"),
                "engine_path": int(summ.get("engine_path", -1)),
                "windows": [int(summ.get("windows", 0)), int(summ.get("windows_y", 0))],
                "window_ps": [int(summ.get("window_ps_x", 0)), int(summ.get("window_ps_y", 0))],
                "chain_protocol": chain_protocol(summ),
            },
            # every rerun is exact but slow: counted over the timed steps (gnoc_summary's
            # totals since submit), and the bench refuses a configs[1] number that needed one
            "reruns": reruns,
            "settle_runs": m["settle_runs"],
            "build_id": bid,
            "e2e_ms_per_step": e2e_ms,
            "e2e_serial_ms_per_step": e2e_serial_ms,
            "e2e_final_ps_ms_per_step": e2e_fin_ms,
            "e2e_15B_ms_per_step": e2e_narrow_ms,
            "e2e_24B_ms_per_step": e2e_wide_ms,
            "e2e_wire_bytes_per_packet": wire,
            "e2e_note": "host trace (pinned) -> host results per batch: submit (H2D + device-side decode and trace "
                        "checks) + run + read-back; e2e_ms_per_step pipelined (batch k+1's upload, decode and checks "
                        "on the upload stream and batch k's read-back on a copy stream, beside the runs; a stream of "
                        "--steps batches, its first upload and last read-back inside the clock) in the delta wire format (gnoc_packets_packed)"
                        " with the per-packet latency read back as u32 (gnoc_fetch_latency); "
                        "e2e_final_ps_ms_per_step the same with final_ps (u64); e2e_15B_ms_per_step the narrow wire "
                        "format with the latency; e2e_serial_ms_per_step one batch at a time (delta upload, final_ps);"
                        " e2e_24B_ms_per_step pipelined with the 24-B upload and final_ps",
            "roofline": {
                "bound": "hbm",
                "achieved": rf["achieved"],
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": rf["frac"],
                "traffic": pmc_traffic(workload, rf["kernel"], bid) if world == 1 else None,
                "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/" + PMC_FILE +
                                ", same build_id only)",
                "algorithmic_bytes_per_launch": rf["alg_bytes_per_launch"],
                "kernel": rf["kernel"],
                "kernel_launches": rf["launches"],
                "kernel_avg_us": rf["kernel_avg_us"],
                "whole_job_frac_per_gpu": whole_job_gbs / HBM_PEAK_GBS,
                "scope": "rank 0's launches and its share of the hops",
            },
            "kernel_ms": {k: round(v[0], 4) for k, v in kst.items()},
            "trace_gen_s": round(gen_s, 2),
        }
        if hot_line is not None:
            line["hotspot"] = hot_line
        if a.cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(a, W, H, load, hot)
        print(json.dumps(line), flush=True)
        bad = [ln for ln in [line] + ([hot_line] if hot_line else [])
               if ln["reruns"]["retries"] or ln["reruns"]["fallbacks"] or
               int(ln.get("engine_path", ln.get("config", {}).get("engine_path", -1))) != 4]
        if wl == "mesh" and bad:
            print(f"bench: a timed step needed reruns {[b['reruns'] for b in bad]} or left the chain engine", file=sys.stderr)
            sys.exit(3)

    eng.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


SETTLE_MIN = 12   # > the variable windows' 8 adaptations + the protocol trial runs


def measure(eng, a, barrier_sync, settle_fixed=False):
    """Settle the chain windows, W warmup runs, then EXACTLY K timed runs between
    barrier + synchronize; then one profiled run for per-kernel device times (HIP
    events on the engine's stream).  Reruns are counted over the timed runs from
    gnoc_summary's totals since submit."""
    settle = 0
    # window adaptation (engine.hip adapt_windows): the first runs of a batch shape size
    # the chain windows from the fill they measure (variable boundaries: up to
    # CH_ADAPT_RUNS = 8 adaptations), then time each hand-off protocol once on the
    # settled windows; at least SETTLE_MIN runs, then until one needed no rerun and used
    # the windows of the run before (a sharded engine runs a fixed count: every rank
    # must call the same collectives)
    prev = None
    for settle in range(1, 2 * SETTLE_MIN + 1):
        eng.run()
        sm = eng.summary()
        cur = (sm["windows"], sm["windows_y"], sm["window_ps_x"], sm["window_ps_y"])
        if settle_fixed and settle >= SETTLE_MIN:
            break
        if not settle_fixed and settle >= SETTLE_MIN and sm["retries"] == 0 and sm["fallbacks"] == 0 and cur == prev:
            break
        prev = cur
    for _ in range(a.warmup):
        eng.run()
    s0 = eng.summary()
    barrier_sync()
    t_start = time.perf_counter()
    for _ in range(a.steps):
        eng.run()
    barrier_sync()
    elapsed = time.perf_counter() - t_start
    s1 = eng.summary()
    reruns = {"retries": int(s1["retries_total"] - s0["retries_total"]),
              "fallbacks": int(s1["fallbacks_total"] - s0["fallbacks_total"]),
              "timed_runs": int(s1["runs"] - s0["runs"])}
    eng.set_profiling(True)
    eng.run()
    kst = eng.kernel_stats()
    eng.set_profiling(False)
    return {"elapsed": elapsed, "summary": s1, "kst": kst, "reruns": reruns, "settle_runs": settle}


def chain_protocol(summ):
    """The hand-off protocol each chain phase ran (gnoc_summary.chain_protocol): the
    engine keeps the serial one unless look-back measured > 5 % faster."""
    v = int(summ.get("chain_protocol", 0))
    if not v & 0x100:
        return None
    return {"x": "lookback" if v & 1 else "serial", "y": "lookback" if v & 2 else "serial",
            "mg1_serial": bool(v & 0x400),
            "mg1_split": bool(v & 0x800)}


def roofline(kst, pc, summ, my_pkts):
    """Dominant kernel (most device time on this rank): k_chain (v4: the X and Y port
    chains), k_level (the chunked levels; on v4 the injection and SELF levels only) or
    k_port_stream (v1).  Algorithmic bytes of ITS launches: 32 B per
    hop record it moves -- k_chain: the mesh hops at RIGHT/LEFT/UP/DOWN ports; the
    level kernels: every hop record + 24 B per delivered packet."""
    dom = max(("k_chain", "k_level", "k_port_stream"), key=lambda k: kst.get(k, (0.0, 0))[0])
    port_ms, launches = kst.get(dom, (0.0, 0))
    my_hops = int(pc[:, :5].sum())
    if dom == "k_chain":
        alg = int(pc[:, 1:5].sum()) * BYTES_PER_HOP
    elif int(summ.get("engine_path", 0)) == 4:   # v4 but k_level dominant: injection + SELF levels
        alg = (int(pc[:, 0].sum()) + int(pc[:, 5].sum())) * BYTES_PER_HOP + my_pkts * BYTES_PER_PKT
    else:
        alg = my_hops * BYTES_PER_HOP + my_pkts * BYTES_PER_PKT
    achieved = alg / (port_ms * 1e-3) / 1e9 if port_ms > 0 else 0.0
    return {"kernel": dom, "achieved": achieved, "frac": achieved / HBM_PEAK_GBS, "launches": launches,
            "kernel_avg_us": port_ms * 1e3 / max(launches, 1), "alg_bytes_per_launch": alg / max(launches, 1)}


def build_id():
    from graphite_amd import gnoc
    lib = gnoc.load()
    return lib.gnoc_build_id().decode() if hasattr(lib, "gnoc_build_id") else None


def sweep_points():
    """BASELINE.json configs[4] / SURVEY.md 8(d) config 5: flit width x router delay
    x tile width (-> link delay 1..4 at 1 GHz) x offered load = 256 8x8 points."""
    import itertools
    from graphite_amd import gnoc
    out = []
    for fw, r, tw, load in itertools.product((16, 32, 64, 128), (0, 1, 2, 3), (1.0, 150.0, 250.0, 350.0),
                                             (0.005, 0.01, 0.015, 0.02)):
        out.append((gnoc.SweepPoint(fw, r, int(-(-tw // 100)), tw), load))
    return out


def sweep_bench(a, world, rank, local):
    """Independent sweep points sharded across ranks (no collective on the data
    path: weak in points); each rank times its slice as ONE batch (gnoc_create_sweep)."""
    from graphite_amd import gnoc
    ppt = a.ppt if a.ppt != 10000 else 2000
    pts = sweep_points()
    mine = pts[rank::world]
    base = gnoc.EngineConfig(num_tiles=64, device=local)
    t0 = time.time()
    trs = [gnoc.synthetic_trace(8, 8, load, ppt, seed=a.seed + 7919 * i) for i, (_, load) in
           enumerate(pts) if i % world == rank]
    gen_s = time.time() - t0
    eng = gnoc.SweepEngine(base, [q for q, _ in mine])
    eng.submit(trs)
    for _ in range(a.warmup):
        eng.run()
    summ = eng.summary()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_start = time.perf_counter()
    for _ in range(a.steps):
        eng.run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    eng.set_profiling(True)
    eng.run()
    kst = eng.kernel_stats()
    hops, pkts = int(summ["mesh_hops"]), int(summ["routed_packets"])
    t = torch.tensor([elapsed, float(hops), float(pkts)], dtype=torch.float64, device="cuda")
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax[0:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:3], op=dist.ReduceOp.SUM)
        t[0] = tmax[0]
    if rank == 0:
        elapsed_max, hops_all = float(t[0]), float(t[1])
        lv_ms, lv_n = kst.get("k_level", (0.0, 0))
        alg = hops * BYTES_PER_HOP + pkts * BYTES_PER_PKT
        ach = alg / (lv_ms * 1e-3) / 1e9 if lv_ms > 0 else 0.0
        print(json.dumps({
            "metric": "packet-hops simulated/sec (node) + % HBM roofline, 1024-tile emesh",
            "value": hops_all * a.steps / elapsed_max, "unit": "packet-hops/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed_max / a.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (synthetic_network.cc uniform_random restated, fixed seeds)",
            "config": {"workload": f"sweep: {len(pts)} 8x8 points (flit 16-128 x R 0-3 x Lk 1-4 x load "
                                   f"0.005-0.02), pkts/tile={ppt}", "points_per_rank": len(mine),
                       "parallelism": f"points/{world}", "mesh_hops": int(hops_all)},
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "traffic": None, "kernel": "k_level",
                         "kernel_launches": lv_n, "kernel_avg_us": lv_ms * 1e3 / max(lv_n, 1),
                         "algorithmic_bytes_per_launch": alg / max(lv_n, 1)},
            "kernel_ms": {k: round(v[0], 4) for k, v in kst.items()},
            "engine_path": int(summ.get("engine_path", -1)),
            "reruns": {"retries": int(summ.get("retries", 0)), "fallbacks": int(summ.get("fallbacks", 0))},
            "trace_gen_s": round(gen_s, 2),
            **({"cpu_baseline": sweep_cpu_baseline(a, pts, ppt)} if a.cpu_baseline and world == 1 else {}),
        }), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def _sweep_point_oracle(args):
    """One sweep point through the CPU oracle (a worker process)."""
    import sys as _s
    _s.path.insert(0, ROOT)
    from graphite_amd import gnoc
    from oracle import oracle
    (fw, r, lk, tw), load, ppt, seed = args
    cfg = gnoc.SweepPoint(fw, r, lk, tw).config(gnoc.EngineConfig(num_tiles=64))
    tr = gnoc.synthetic_trace(8, 8, load, ppt, seed=seed)
    t0 = time.perf_counter()
    res = oracle.run(cfg, tr)
    return int(res.port_count.reshape(-1, 6)[:, :5].sum()), time.perf_counter() - t0


def sweep_cpu_baseline(a, pts, ppt, npts=64, workers=None):
    """independent single-threaded oracle processes over the
    host cores this process may run on (sched_getaffinity; nproc and the
    affinity are stated in the record, and at most 16 are used: the GPU box's
    CPU share), on the first `npts` points of the same sweep; aggregate hops /
    oracle time."""
    import multiprocessing as mp
    avail = len(os.sched_getaffinity(0))
    if workers is None:
        workers = max(1, min(avail, 16))
    jobs = [((q.flit_width, q.router_delay, q.link_delay, q.tile_width_mm), load, ppt, a.seed + 7919 * i)
            for i, (q, load) in enumerate(pts[:npts])]
    with mp.get_context("spawn").Pool(workers) as pool:
        out = pool.map(_sweep_point_oracle, jobs)
    hops = sum(h for h, _ in out)
    busy = sum(t for _, t in out) / workers   # oracle time only: worker start-up and trace generation excluded
    return {"value": hops / busy, "unit": "packet-hops/s", "cores": workers, "kind": "port",
            "nproc": os.cpu_count(), "affinity_cpus": avail,
            "sample": f"{npts} of the {len(pts)} sweep points, pkts/tile={ppt}: {hops} mesh hops, "
                      f"{busy:.2f} s of oracle time per worker ({workers} single-threaded oracle processes)"}


def pinned_array(n, dt):
    """A page-locked numpy array (a view of a pinned torch tensor's bytes)."""
    nbytes = int(n) * np.dtype(dt).itemsize
    t = torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=True)
    return t.numpy()[:nbytes].view(dt)


def pinned_trace(tr):
    """The trace in page-locked host memory (numpy views of pinned torch tensors)."""
    from graphite_amd import gnoc

    def pin(x):
        t = torch.empty(x.shape[0], dtype={8: torch.int64, 4: torch.int32}[x.dtype.itemsize], pin_memory=True)
        v = t.numpy().view(x.dtype)
        v[:] = x
        return v
    return gnoc.Trace(pin(tr.inject_ps), pin(tr.src), pin(tr.dst), pin(tr.bits),
                      pin(tr.flags if tr.flags is not None else np.zeros(len(tr), np.uint32)))


PMC_FILE = "r6_pmc.json"


def pmc_traffic(workload, kernel, bid):
    """HBM bytes per launch of the dominant kernel, from the committed PMC passes
    (tools/gpu_round.sh -> tools/prof_summary.py) of this same workload AND this same
    build (gnoc_build_id); None if no such profile is committed."""
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", PMC_FILE)
    try:
        with open(p) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    if d.get("workload") != workload or d.get("kernel") != kernel or not bid or d.get("build_id") != bid:
        return None
    return d.get("traffic_bytes_per_launch")


def cpu_baseline(a, W, H, load, hot):
    """The reference path on one host core over a bounded sample of the same workload:
    the oracle's event loop (oracle/gnoc_oracle.c, the reference's per-hop walk
    restated) with every history-tree queue being the reference's OWN IntervalTree +
    QueueModelMG1 objects, compiled from its sources into oracle/_ref (ref_driver.cc
    restates only computeQueueDelay's 80 lines over them).  Where oracle/_ref is not
    built, the all-restated oracle (sorted-array free list) instead, and the record
    says so.  The restated oracle's rate on the same sample is reported beside it."""
    from graphite_amd import gnoc
    from oracle import oracle
    tr = gnoc.synthetic_trace(W, H, load, a.cpu_sample_ppt, seed=a.seed, hotspot_fraction=hot, num_hotspots=16)
    cfg = gnoc.EngineConfig(num_tiles=W * H)
    t0 = time.perf_counter()
    r = oracle.run(cfg, tr)
    dt_port = time.perf_counter() - t0
    hops = int(r.port_count.reshape(-1, 6)[:, :5].sum())
    ref_q = oracle.ref_lib() is not None
    dt = dt_port
    if ref_q:
        t0 = time.perf_counter()
        rq = oracle.run(cfg, tr, ref_queues=True)
        dt = time.perf_counter() - t0
        assert np.array_equal(rq.final_ps, r.final_ps), "reference queue objects disagree with the oracle"
    return {"value": hops / dt, "unit": "packet-hops/s", "cores": 1, "kind": "port",
            "what": ("the reference's per-hop event walk restated (oracle/gnoc_oracle.c) with the reference's own "
                     "IntervalTree + QueueModelMG1 objects compiled from its sources (oracle/_ref) as every "
                     "history-tree queue, 1 core" if ref_q else
                     "oracle restatement of the reference path (oracle/gnoc_oracle.c), 1 core, sorted-array free "
                     "list instead of the reference's AVL tree (oracle/_ref not built)"),
            "restated_queues_value": hops / dt_port,
            "sample": f"{W}x{H} {a.mix} load={load} pkts/tile={a.cpu_sample_ppt}: {len(tr)} packets, "
                      f"{hops} mesh hops in {dt:.2f} s",
            # the reference itself (compiled from its sources, survey probe): context only,
            # measured in the build container, not on the GPU box
            "reference_probe": {"value": 0.58e6, "unit": "packet-hops/s", "cores": 1,
                                "config": "32x32 emesh_hop_by_hop, 300 pkts/tile at 0.01", "host": "Xeon, survey probe"}}


if __name__ == "__main__":
    main()
