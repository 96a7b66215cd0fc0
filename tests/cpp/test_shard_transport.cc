// A sharded mesh through the C ABI alone (no Python, no torch): gnoc_run_sharded
// over an in-process transport (graphite_amd/host/shard_local.h), one thread per
// rank on one GPU.  The element-wise sum of the ranks' results equals the
// unsharded engine's, bit for bit; a failure on one rank (GNOC_FAIL_RANK) fails
// every rank's gnoc_run_sharded instead of leaving the others waiting.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "gnoc.h"
#include "shard_local.h"

using graphite_amd::LocalShardTransport;

struct Out
{
   std::vector<uint64_t> fin, zl, ct, ps, pc, pm, pf, pl;
   int rc = 0;
};

static int collect(gnoc_engine* e, size_t n, size_t np, Out& o)
{
   o.fin.assign(n, 0);
   o.zl.assign(n, 0);
   o.ct.assign(n, 0);
   o.ps.assign(np, 0);
   o.pc.assign(np, 0);
   o.pm.assign(np, 0);
   o.pf.assign(np, 0);
   o.pl.assign(np, 0);
   int rc = gnoc_get_packet_results(e, o.fin.data(), o.zl.data(), o.ct.data(), n);
   if (!rc) rc = gnoc_get_port_stats(e, o.ps.data(), o.pc.data(), o.pm.data(), np);
   if (!rc) rc = gnoc_get_port_utilization(e, o.pf.data(), o.pl.data(), np);
   return rc;
}

static int run_shards(const gnoc_config& cfg, const gnoc_packets& pk, size_t n, int nr, std::vector<Out>& outs)
{
   LocalShardTransport tp(nr);
   outs.assign(nr, Out());
   const size_t np = (size_t) cfg.num_tiles * GNOC_PORTS_PER_TILE;
   std::vector<std::thread> th;
   for (int r = 0; r < nr; r++)
      th.emplace_back([&, r] {
         gnoc_engine* e = nullptr;
         int rc = gnoc_create(&cfg, &e);
         if (!rc) rc = gnoc_shard(e, r, nr);
         if (!rc) rc = gnoc_submit(e, &pk, n);
         gnoc_transport t = tp.transport(r);
         if (!rc) rc = gnoc_shard_set_transport(e, &t);
         // every rank enters gnoc_run_sharded: its exchange and status agreement are collective
         const int rr = gnoc_run_sharded(e);
         rc = rc ? rc : rr;
         if (!rc) rc = collect(e, n, np, outs[r]);
         if (rc && e) std::fprintf(stderr, "rank %d: %s\n", r, gnoc_last_error(e));
         outs[r].rc = rc;
         gnoc_destroy(e);
      });
   for (auto& t : th) t.join();
   return 0;
}

int main()
{
   const int W = 8, H = 8;
   size_t n = 0;
   gnoc_trace_synthetic(W, H, 1.0, 0.05, 300, 8, 11, 0.0, 16, nullptr, nullptr, nullptr, nullptr, 0, &n);
   std::vector<uint64_t> inj(n);
   std::vector<uint32_t> src(n), dst(n), bits(n), flags(n, 0);
   if (gnoc_trace_synthetic(W, H, 1.0, 0.05, 300, 8, 11, 0.0, 16, inj.data(), src.data(), dst.data(), bits.data(), n, &n))
      return 2;
   gnoc_packets pk{inj.data(), src.data(), dst.data(), bits.data(), flags.data()};
   gnoc_config cfg;
   gnoc_config_default(&cfg, W * H);
   cfg.mesh_width = W;
   cfg.mesh_height = H;
   const size_t np = (size_t) cfg.num_tiles * GNOC_PORTS_PER_TILE;

   gnoc_engine* ref = nullptr;
   Out want;
   if (gnoc_create(&cfg, &ref) || gnoc_submit(ref, &pk, n) || gnoc_run(ref) || collect(ref, n, np, want)) return 3;
   gnoc_destroy(ref);

   int failures = 0;
   for (int nr : {2, 3, 5})
   {
      std::vector<Out> outs;
      run_shards(cfg, pk, n, nr, outs);
      Out sum;
      sum.fin.assign(n, 0), sum.zl.assign(n, 0), sum.ct.assign(n, 0);
      sum.ps.assign(np, 0), sum.pc.assign(np, 0), sum.pm.assign(np, 0), sum.pf.assign(np, 0), sum.pl.assign(np, 0);
      bool ok = true;
      for (auto& o : outs)
      {
         ok &= o.rc == 0;
         if (!ok) break;
         for (size_t i = 0; i < n; i++) sum.fin[i] += o.fin[i], sum.zl[i] += o.zl[i], sum.ct[i] += o.ct[i];
         for (size_t p = 0; p < np; p++)
            sum.ps[p] += o.ps[p], sum.pc[p] += o.pc[p], sum.pm[p] += o.pm[p], sum.pf[p] += o.pf[p], sum.pl[p] += o.pl[p];
      }
      ok = ok && sum.fin == want.fin && sum.zl == want.zl && sum.ct == want.ct && sum.ps == want.ps &&
           sum.pc == want.pc && sum.pm == want.pm && sum.pf == want.pf && sum.pl == want.pl;
      std::printf("%d ranks through the C transport: %s\n", nr, ok ? "identical to unsharded" : "MISMATCH");
      failures += !ok;
   }
   // one rank fails its X phase: every rank's gnoc_run_sharded fails
   setenv("GNOC_FAIL_RANK", "1", 1);
   {
      std::vector<Out> outs;
      run_shards(cfg, pk, n, 3, outs);
      bool all = true;
      for (auto& o : outs) all &= o.rc != 0;
      std::printf("failure on rank 1: %s\n", all ? "every rank failed" : "SOME RANK SUCCEEDED");
      failures += !all;
   }
   unsetenv("GNOC_FAIL_RANK");
   if (failures) return 1;
   std::printf("test_shard_transport: all checks passed\n");
   return 0;
}
