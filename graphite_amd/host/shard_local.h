// shard_local.h -- every rank of a sharded mesh as a thread of ONE process, the
// turn-record exchange as device-to-device copies between the ranks' buffers
// (a gnoc_transport, include/gnoc.h).  The C-ABI counterpart of the Python
// LocalShardSet: gnoc_replay --shards N and the C++ test drive gnoc_run_sharded
// through it on one GPU; on a multi-GPU node the engines take an ncclComm_t
// (gnoc_shard_set_comm) instead.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <vector>

#include "gnoc.h"

namespace graphite_amd {

class LocalShardTransport
{
public:
   explicit LocalShardTransport(int nranks)
      : _n(nranks), _send(nranks, nullptr), _su(nranks), _status(nranks, 0) {}

   // The gnoc_transport of rank r (valid while this object lives).
   gnoc_transport transport(int r)
   {
      _ctx.resize(_n);
      for (int q = 0; q < _n; q++) _ctx[q] = Ctx{this, q};
      gnoc_transport t;
      t.exchange = &LocalShardTransport::exchange;
      t.agree = &LocalShardTransport::agree;
      t.ctx = &_ctx[r];
      return t;
   }

private:
   struct Ctx
   {
      LocalShardTransport* self;
      int rank;
   };

   void barrier()
   {
      std::unique_lock<std::mutex> lk(_m);
      const uint64_t gen = _gen;
      if (++_arrived == _n)
      {
         _arrived = 0;
         _gen++;
         _cv.notify_all();
      }
      else
         _cv.wait(lk, [&] { return _gen != gen; });
   }

   static int exchange(void* ctx, const void* send, const uint64_t* su, void* recv, const uint64_t* ru, void* stream)
   {
      Ctx* c = static_cast<Ctx*>(ctx);
      LocalShardTransport* s = c->self;
      const int me = c->rank, n = s->_n;
      s->_send[me] = static_cast<const char*>(send);
      s->_su[me].assign(su, su + n);
      hipStream_t st = static_cast<hipStream_t>(stream);
      int bad = hipStreamSynchronize(st) != hipSuccess;   // my send buffer is complete
      s->barrier();                                        // ... and every peer's
      uint64_t ro = 0;
      for (int q = 0; q < n; q++)
      {
         // q's block for me starts after q's blocks for the ranks below me
         uint64_t so = 0;
         for (int p = 0; p < me; p++) so += s->_su[q][p];
         if (s->_su[q][me] != ru[q]) bad = 1;
         else if (ru[q])
            bad |= hipMemcpyAsync(static_cast<char*>(recv) + ro * 16, s->_send[q] + so * 16, ru[q] * 16,
                                  hipMemcpyDeviceToDevice, st) != hipSuccess;
         ro += ru[q];
      }
      bad |= hipStreamSynchronize(st) != hipSuccess;
      s->barrier();   // every copy out of every send buffer is done
      return bad;
   }

   static int agree(void* ctx, int32_t status, int32_t* out)
   {
      Ctx* c = static_cast<Ctx*>(ctx);
      LocalShardTransport* s = c->self;
      s->_status[c->rank] = status;
      s->barrier();
      *out = *std::max_element(s->_status.begin(), s->_status.end());
      s->barrier();   // nobody overwrites a status before everyone read the max
      return 0;
   }

   int _n;
   std::vector<const char*> _send;
   std::vector<std::vector<uint64_t>> _su;
   std::vector<int32_t> _status;
   std::vector<Ctx> _ctx;
   std::mutex _m;
   std::condition_variable _cv;
   int _arrived = 0;
   uint64_t _gen = 0;
};

}  // namespace graphite_amd
