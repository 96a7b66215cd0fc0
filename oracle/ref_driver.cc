// ref_driver.cc -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/libgnoc_ref.so).
//
// Links the reference's own, unmodified sources, compiled in place from
// /root/reference by oracle/Makefile:
//   common/misc/interval_tree.cc                          (the AVL free-interval tree)
//   common/shared_models/queue_models/queue_model_m_g_1.cc (the FP64 M/G/1 model)
//   common/misc/time_types.h                              (ps <-> cycle conversions)
//   common/misc/moving_average.h + modulo_num.cc          (QueueModelBasic's moving averages)
// Those three compile with the reference's real headers and -DNDEBUG; nothing
// is stubbed.  queue_model_history_tree.cc itself cannot be compiled here (its
// includes reach common/config/section.hpp -> boost/shared_ptr.hpp, absent), so
// its 80-line computeQueueDelay body (queue_model_history_tree.cc:43-126) is
// restated below on top of the REAL IntervalTree and QueueModelMG1 objects.
//
// Used only by tests/test_oracle.py to pin the C oracle's sorted-array
// restatement of the interval tree and its M/G/1 arithmetic.
#include <stdint.h>
#include <utility>

#include <string>

#include "interval_tree.h"
#include "moving_average.h"
#include "queue_model_m_g_1.h"
#include "time_types.h"

namespace {

struct RefQueue
{
   IntervalTree* tree;
   QueueModelMG1* mg1;
   bool analytical;
   UInt64 min_proc;
   int max_size;
   UInt64 mg1_uses;
};

std::pair<UInt64, UInt64> P(UInt64 a, UInt64 b) { return std::make_pair(a, b); }

IntervalTree::Node* newNode(UInt64 a, UInt64 b)
{
   IntervalTree::Node* n = new IntervalTree::Node();
   n->initialize(P(a, b));
   return n;
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) void* ref_queue_create(int max_list_size, int analytical, uint64_t min_proc)
{
   RefQueue* q = new RefQueue;
   q->tree = new IntervalTree(newNode(0, UINT64_MAX));   // queue_model_history_tree.cc:29-30
   q->mg1 = new QueueModelMG1();
   q->analytical = analytical != 0;
   q->min_proc = min_proc;
   q->max_size = max_list_size;
   q->mg1_uses = 0;
   return q;
}

// Restatement of queue_model_history_tree.cc:43-126 over the real tree/M/G/1.
// Released nodes are leaked on purpose (the reference recycles them through a
// free list; reuse does not affect results).
__attribute__((visibility("default"))) uint64_t ref_queue_compute(void* vq, uint64_t pkt_time, uint64_t processing_time)
{
   RefQueue* q = (RefQueue*) vq;
   UInt64 queue_delay = UINT64_MAX;
   IntervalTree::Node* min_node = q->tree->search(P(0, 1));
   if (q->tree->size() >= (UInt32) q->max_size)
      q->tree->remove(min_node);
   min_node = q->tree->search(P(0, 1));
   if (q->analytical && (min_node->interval.first > (pkt_time + processing_time)))
   {
      q->mg1_uses++;
      queue_delay = q->mg1->computeQueueDelay(pkt_time, processing_time);
   }
   else
   {
      IntervalTree::Node* node = q->tree->search(P(pkt_time, pkt_time + processing_time));
      if (!node) return UINT64_MAX;
      if (pkt_time >= node->interval.first)
      {
         queue_delay = 0;
         if ((pkt_time - node->interval.first) >= q->min_proc)
         {
            if ((node->interval.second - (pkt_time + processing_time)) >= q->min_proc)
               q->tree->insert(newNode(pkt_time + processing_time, node->interval.second));
            node->interval.second = pkt_time;
         }
         else
         {
            if ((node->interval.second - (pkt_time + processing_time)) >= q->min_proc)
            {
               node->interval.first = pkt_time + processing_time;
               node->key = node->interval.first;
            }
            else
               q->tree->remove(node);
         }
      }
      else
      {
         queue_delay = node->interval.first - pkt_time;
         if ((node->interval.second - (node->interval.first + processing_time)) >= q->min_proc)
         {
            node->interval.first = node->interval.first + processing_time;
            node->key = node->interval.first;
         }
         else
            q->tree->remove(node);
      }
   }
   q->mg1->updateQueue(pkt_time, processing_time, queue_delay);
   return queue_delay;
}

__attribute__((visibility("default"))) uint64_t ref_queue_mg1_uses(void* vq) { return ((RefQueue*) vq)->mg1_uses; }
__attribute__((visibility("default"))) uint32_t ref_queue_size(void* vq) { return ((RefQueue*) vq)->tree->size(); }

__attribute__((visibility("default"))) void ref_queue_destroy(void* vq)
{
   RefQueue* q = (RefQueue*) vq;
   delete q->mg1;
   delete q->tree;
   delete q;
}

// The real MovingAverage<UInt64>::createAvgType / compute (moving_average.h),
// as QueueModelBasic builds it (queue_model_basic.cc:27-30, :38-46).
// type: 1 arithmetic_mean, 2 geometric_mean, 3 median (include/gnoc.h).
__attribute__((visibility("default"))) void* ref_ma_create(int type, uint32_t window)
{
   static const char* const names[] = { "", "arithmetic_mean", "geometric_mean", "median" };
   if (type < 1 || type > 3) return 0;
   return MovingAverage<UInt64>::createAvgType(std::string(names[type]), window);
}

__attribute__((visibility("default"))) uint64_t ref_ma_compute(void* m, uint64_t x)
{
   return ((MovingAverage<UInt64>*) m)->compute(x);
}

__attribute__((visibility("default"))) void ref_ma_destroy(void* m) { delete (MovingAverage<UInt64>*) m; }

// Real Latency::toPicosec / Time::toCycles (time_types.h:81-109).
__attribute__((visibility("default"))) uint64_t ref_lat_to_ps(uint64_t cycles, double f)
{
   return Latency(cycles, f).toPicosec();
}

__attribute__((visibility("default"))) uint64_t ref_time_to_cycles(uint64_t ps, double f)
{
   return Time(ps).toCycles(f);
}

}  // extern "C"
