/*
 * gnoc_oracle.c -- CPU ORACLE for the emesh_hop_by_hop timing path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker the HIP engine is
 * compared against; it is never linked into, loaded by, or called from the
 * product library (graphite_amd/_build/libgnoc.so).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 *
 * It is a plain-C restatement of the reference algorithm, function by
 * function, with file:line citations into /root/reference (Graphite):
 *
 *   - QueueModelHistoryTree::computeQueueDelay
 *       common/shared_models/queue_models/queue_model_history_tree.cc:43-126
 *     The AVL interval tree (common/misc/interval_tree.cc:265-394) is
 *     restated as a sorted array of disjoint free intervals with first-fit
 *     search; DESIGN.md and tests/test_oracle.py pin this equivalence
 *     against the real IntervalTree compiled from the reference
 *     (oracle/_ref, see oracle/Makefile).
 *   - QueueModelHistoryList::computeQueueDelay / computeUsingHistoryList
 *       common/shared_models/queue_models/queue_model_history_list.cc:39-146
 *   - QueueModelBasic::computeQueueDelay (moving average disabled)
 *       common/shared_models/queue_models/queue_model_basic.cc:35-61
 *   - QueueModelMG1::computeQueueDelay / updateQueue
 *       common/shared_models/queue_models/queue_model_m_g_1.cc:17-56
 *   - Latency::toPicosec / Time::toCycles   common/misc/time_types.h:81-109
 *   - RouterModel::processPacket            common/network/components/router/router_model.cc:70-108
 *   - ElectricalLinkModel                   common/network/components/link/electrical_link_model.cc:13-45
 *   - NetworkModelEMeshHopByHop::routePacket
 *       common/network/models/network_model_emesh_hop_by_hop.cc:146-264
 *   - NetworkModel::__routePacket / processCornerCases / __processReceivedPacket /
 *     processReceivedPacket / Hop::Hop      common/network/network_model.cc:87-150, 413-468, 556-563
 *   - Network::forwardPacket hop loop       common/network/network.cc:215-262
 *
 * Parity contract: a single-threaded event loop whose
 * priority queue is keyed (time_ps, packet_id); one event per packet at a
 * time; the Hop -> packet field copy of network.cc:234-237.
 *
 * Pinned by: the reference's own known-answer test
 * tests/unit/history_tree/history_tree.cc:9-20 (10 packets, incl. out-of-order
 * arrivals) and by differential tests against oracle/_ref (real
 * IntervalTree + QueueModelMG1 + time_types.h compiled from the reference).
 *
 * Compiled with -ffp-contract=off so the FP64 M/G/1 expression keeps the
 * reference's operation order (no fused multiply-add).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* time_types.h:81-86 and :104-109                                          */
/* ------------------------------------------------------------------------ */
static uint64_t lat_to_ps(uint64_t cycles, double f)
{
   /* (UInt64) ceil( ((double) 1000*_cycles) / ((double) _frequency) ) */
   return (uint64_t) ceil(((double) 1000 * (double) cycles) / ((double) f));
}

static uint64_t time_to_cycles(uint64_t ps, double f)
{
   /* (UInt64) ceil(((double) (_picosec) * ((double) frequency)) / double(1.0e3)) */
   return (uint64_t) ceil(((double) ps * (double) f) / (double) 1.0e3);
}

ORC_EXPORT uint64_t orc_lat_to_ps(uint64_t c, double f) { return lat_to_ps(c, f); }
ORC_EXPORT uint64_t orc_time_to_cycles(uint64_t p, double f) { return time_to_cycles(p, f); }

/* ------------------------------------------------------------------------ */
/* QueueModelHistoryTree (+ QueueModelMG1)                                  */
/* ------------------------------------------------------------------------ */
typedef struct { uint64_t first, second; } orc_interval;

enum { ORC_Q_HISTORY_TREE = 0, ORC_Q_BASIC = 1, ORC_Q_HISTORY_LIST = 2 };   /* include/gnoc.h GNOC_QUEUE_* */

typedef struct
{
   int type;              /* QueueModel::Type, queue_model.cc:18-38        */
   int interleaving;      /* queue_model/history_list/interleaving_enabled */
   uint64_t queue_time;   /* QueueModelBasic::_queue_time                  */
   orc_interval *iv;      /* free intervals, sorted by .first, disjoint    */
   int n;                 /* IntervalTree::_size                           */
   int max_list_size;     /* queue_model/history_tree/max_list_size        */
   int analytical;        /* queue_model/history_tree/analytical_model_enabled */
   uint64_t min_proc;     /* _min_processing_time (RouterModel passes 1)   */
   /* QueueModelMG1 state, queue_model_m_g_1.cc:8-12 */
   double s2, s1;
   uint64_t narr, newest;
   /* MovingAverage<UInt64> of QueueModelBasic (moving_average.h), ma_type 0 = none */
   int ma_type;           /* ORC_MA_*                                      */
   uint32_t ma_max;       /* _max_window_size                              */
   uint64_t *ma_list;     /* _num_list, _max_window_size + 1 entries       */
   uint32_t ma_front, ma_back; /* ModuloNum(_max_window_size + 1) values    */
   double ma_mean;        /* _arithmetic_mean (0.0) / _geometric_mean (1.0) */
   /* counters */
   uint64_t mg1_uses;     /* _total_requests_using_analytical_model        */
   uint64_t total_requests, util_cycles, last_request_time; /* queue_model.cc:40-53 */
   void *ext;             /* history_tree through orc_set_queue_hooks: the hook's queue */
} orc_queue;

/* Optional history-tree queues from outside (bench.py's CPU baseline: the reference's
 * own IntervalTree + QueueModelMG1, oracle/ref_driver.cc over oracle/_ref); NULL: the
 * sorted-array restatement below. */
static void *(*hk_create)(int, int, uint64_t);
static uint64_t (*hk_compute)(void *, uint64_t, uint64_t);
static uint64_t (*hk_mg1_uses)(void *);
static void (*hk_destroy)(void *);

ORC_EXPORT void orc_set_queue_hooks(void *(*create)(int, int, uint64_t), uint64_t (*compute)(void *, uint64_t, uint64_t),
                                    uint64_t (*mg1_uses)(void *), void (*destroy)(void *))
{
   hk_create = create;
   hk_compute = compute;
   hk_mg1_uses = mg1_uses;
   hk_destroy = destroy;
}

/* QueueModel::create(type, min_processing_time), queue_model.cc:18-38.
 * basic: moving average disabled (queue_model_basic.cc:7-30 with
 * moving_avg_enabled = false); history_list: queue_model_history_list.cc:10-32. */
ORC_EXPORT orc_queue *orc_queue_create_type(int type, int max_list_size, int analytical, int interleaving,
                                            uint64_t min_proc)
{
   if (type != ORC_Q_BASIC && (max_list_size < 2 || min_proc < 1))
      return NULL; /* reference aborts / corrupts its tree for these */
   if (type < 0 || type > 2) return NULL;
   if (type == ORC_Q_BASIC) max_list_size = 1;
   orc_queue *q = (orc_queue *) calloc(1, sizeof(orc_queue));
   q->type = type;
   q->interleaving = interleaving;
   q->iv = (orc_interval *) calloc((size_t) max_list_size + 2, sizeof(orc_interval));
   q->max_list_size = max_list_size;
   q->analytical = analytical;
   q->min_proc = min_proc;
   /* queue_model_history_tree.cc:29-30: start node [0, UINT64_MAX) */
   q->iv[0].first = 0;
   q->iv[0].second = UINT64_MAX;
   q->n = 1;
   if (type == ORC_Q_HISTORY_TREE && hk_create) q->ext = hk_create(max_list_size, analytical, min_proc);
   return q;
}

/* MovingAverage<T>::createAvgType, moving_average.h:175-189 (include/gnoc.h GNOC_MOVING_AVG_*) */
enum { ORC_MA_NONE = 0, ORC_MA_ARITHMETIC_MEAN = 1, ORC_MA_GEOMETRIC_MEAN = 2, ORC_MA_MEDIAN = 3 };

/* QueueModelBasic with queue_model/basic/moving_avg_enabled (queue_model_basic.cc:7-30):
 * attach a moving average of type ma_type over max_window_size numbers. */
ORC_EXPORT int orc_queue_set_moving_avg(orc_queue *q, int ma_type, uint32_t max_window_size)
{
   if (!q || q->type != ORC_Q_BASIC || ma_type < ORC_MA_NONE || ma_type > ORC_MA_MEDIAN) return -1;
   if (ma_type != ORC_MA_NONE && max_window_size < 1) return -1;   /* window 0 divides by zero */
   free(q->ma_list);
   q->ma_list = NULL;
   q->ma_type = ma_type;
   if (ma_type == ORC_MA_NONE) return 0;
   q->ma_max = max_window_size;
   q->ma_list = (uint64_t *) calloc((size_t) max_window_size + 1, sizeof(uint64_t));   /* :44-50 */
   q->ma_front = q->ma_back = 0;
   q->ma_mean = (ma_type == ORC_MA_GEOMETRIC_MEAN) ? 1.0 : 0.0;   /* :88, :122 */
   return 0;
}

/* MovingAverage<T>::addToWindow, moving_average.h:57-66 (ModuloNum arithmetic, modulo_num.cc) */
static void ma_add(orc_queue *q, uint64_t x)
{
   const uint32_t M = q->ma_max + 1;
   q->ma_list[q->ma_back] = x;
   q->ma_back = (q->ma_back + 1) % M;
   if (q->ma_back == q->ma_front) q->ma_front = (q->ma_front + 1) % M;
}

/* MovingArithmeticMean / MovingGeometricMean / MovingMedian ::compute,
 * moving_average.h:90-110, 124-145, 153-162 */
ORC_EXPORT uint64_t orc_ma_compute(orc_queue *q, uint64_t x)
{
   const uint32_t M = q->ma_max + 1;
   const uint32_t cw = (q->ma_back >= q->ma_front) ? q->ma_back - q->ma_front : q->ma_back + M - q->ma_front;
   if (q->ma_type == ORC_MA_MEDIAN)
   {
      ma_add(q, x);
      const uint32_t w = (q->ma_back >= q->ma_front) ? q->ma_back - q->ma_front : q->ma_back + M - q->ma_front;
      return q->ma_list[(q->ma_front + (w / 2) % M) % M];
   }
   if (q->ma_type == ORC_MA_ARITHMETIC_MEAN)
   {
      if (cw == q->ma_max)
      {
         const uint64_t old = q->ma_list[q->ma_front];
         q->ma_mean += (((double) x / (double) cw) - ((double) old / (double) cw));
      }
      else
         q->ma_mean = (q->ma_mean * (double) cw + (double) x) / (double) (cw + 1);
   }
   else
   {
      if (cw == q->ma_max)
      {
         const uint64_t old = q->ma_list[q->ma_front];
         q->ma_mean *= (pow((double) x, (1.0 / (double) cw)) / pow((double) old, (1.0 / (double) cw)));
      }
      else
         q->ma_mean = pow(pow(q->ma_mean, (double) cw) * (double) x, (1.0 / (double) (cw + 1)));
   }
   ma_add(q, x);
   return (uint64_t) q->ma_mean;
}

ORC_EXPORT orc_queue *orc_queue_create(int max_list_size, int analytical, uint64_t min_proc)
{
   return orc_queue_create_type(ORC_Q_HISTORY_TREE, max_list_size, analytical, 0, min_proc);
}

ORC_EXPORT void orc_queue_destroy(orc_queue *q)
{
   if (!q) return;
   if (q->ext && hk_destroy) hk_destroy(q->ext);
   free(q->ma_list);
   free(q->iv);
   free(q);
}

ORC_EXPORT uint64_t orc_queue_mg1_uses(const orc_queue *q) { return q->ext ? hk_mg1_uses(q->ext) : q->mg1_uses; }
ORC_EXPORT int orc_queue_size(const orc_queue *q) { return q->n; }

static void iv_remove(orc_queue *q, int i)
{
   memmove(&q->iv[i], &q->iv[i + 1], (size_t) (q->n - i - 1) * sizeof(orc_interval));
   q->n--;
}

static void iv_insert(orc_queue *q, orc_interval v)
{
   int i = q->n;
   while (i > 0 && q->iv[i - 1].first > v.first) { q->iv[i] = q->iv[i - 1]; i--; }
   q->iv[i] = v;
   q->n++;
}

/* IntervalTree::searchTree (interval_tree.cc:365-394) restated.  For the
 * disjoint, non-adjacent, non-empty intervals the history tree maintains, the
 * BST descent returns the FIRST interval in key order that either contains
 * [a, b) or starts after a and is at least (b - a) long. */
static int iv_search(const orc_queue *q, uint64_t a, uint64_t b)
{
   for (int i = 0; i < q->n; i++)
   {
      const orc_interval *v = &q->iv[i];
      if (a >= v->first && b <= v->second) return i;
      if (a < v->first && (v->second - v->first) >= (b - a)) return i;
   }
   return -1;
}

/* QueueModelMG1::computeQueueDelay, queue_model_m_g_1.cc:17-46 */
static uint64_t mg1_delay(const orc_queue *q)
{
   if (q->narr == 0) return 0;
   double variance = ((q->s2 / (double) q->narr) -
                      ((q->s1 / (double) q->narr) * (q->s1 / (double) q->narr)));
   double service_rate = 1.0 / (q->s1 / (double) q->narr);
   double arrival_rate = ((double) q->narr) / (double) q->newest;
   if (arrival_rate >= service_rate)
      arrival_rate = 0.999 * service_rate;
   return (uint64_t) ceil(0.5 * service_rate * arrival_rate *
                          ((1 / (service_rate * service_rate)) + variance) /
                          (service_rate - arrival_rate));
}

/* QueueModelMG1::updateQueue, queue_model_m_g_1.cc:48-56 */
static void mg1_update(orc_queue *q, uint64_t t, uint64_t p, uint64_t d)
{
   q->s2 += ((double) p * (double) p);
   q->s1 += (double) p;
   q->narr++;
   uint64_t nw = t + d + p;
   q->newest = (q->newest > nw) ? q->newest : nw;
}

static void util_update(orc_queue *q, uint64_t t, uint64_t p, uint64_t d)
{
   /* queue_model.cc:48-53 updateQueueUtilizationCounters */
   q->util_cycles += p;
   uint64_t lr = t + d + p;
   q->last_request_time = (q->last_request_time > lr) ? q->last_request_time : lr;
   q->total_requests++;
}

static void iv_insert_at(orc_queue *q, int i, orc_interval v)
{
   memmove(&q->iv[i + 1], &q->iv[i], (size_t) (q->n - i) * sizeof(orc_interval));
   q->iv[i] = v;
   q->n++;
}

/* QueueModelHistoryList::computeUsingHistoryList, queue_model_history_list.cc:70-146.
 * The std::list walk is restated over the sorted array with an index; after an
 * erase the reference's iterator steps back (curr_it--), and stepping back
 * from begin() lands on the list's end sentinel, whose successor is begin(). */
static uint64_t hl_compute(orc_queue *q, uint64_t pkt_time, uint64_t processing_time)
{
   const uint64_t m = q->min_proc;
   uint64_t queue_delay = 0;
   for (int i = 0; i < q->n; i++)
   {
      const orc_interval iv = q->iv[i];
      if ((pkt_time >= iv.first) && ((pkt_time + processing_time) <= iv.second))
      {
         /* :82-96 no additional delay */
         iv_remove(q, i);
         int at = i;
         if ((pkt_time - iv.first) >= m) { orc_interval a = { iv.first, pkt_time }; iv_insert_at(q, at++, a); }
         if ((iv.second - (pkt_time + processing_time)) >= m)
         {
            orc_interval b = { pkt_time + processing_time, iv.second };
            iv_insert_at(q, at, b);
         }
         break;
      }
      else if ((pkt_time < iv.first) && ((iv.first + processing_time) <= iv.second))
      {
         /* :97-108 wait for the interval */
         queue_delay += (iv.first - pkt_time);
         iv_remove(q, i);
         if ((iv.second - (iv.first + processing_time)) >= m)
         {
            orc_interval b = { iv.first + processing_time, iv.second };
            iv_insert_at(q, i, b);
         }
         break;
      }
      else if (q->interleaving)
      {
         if ((pkt_time >= iv.first) && (pkt_time < iv.second))
         {
            /* :111-123 (processing_time -= 0: pkt_time is reassigned first) */
            iv_remove(q, i);
            if ((pkt_time - iv.first) >= m)
            {
               orc_interval a = { iv.first, pkt_time };
               iv_insert_at(q, i, a);
               /* curr_it-- from the element after the insert: the inserted one */
            }
            else
               i--;
            pkt_time = iv.second;
            processing_time -= (iv.second - pkt_time);
         }
         else if (pkt_time < iv.first)
         {
            /* :124-134 */
            iv_remove(q, i);
            i--;
            queue_delay += (iv.first - pkt_time);
            pkt_time = iv.second;
            processing_time -= (iv.second - iv.first);
         }
      }
   }
   if (q->n > q->max_list_size) iv_remove(q, 0);   /* :138-141 */
   return queue_delay;
}

/* QueueModelHistoryList::computeQueueDelay, queue_model_history_list.cc:39-68 */
static uint64_t hl_queue_delay(orc_queue *q, uint64_t t, uint64_t p)
{
   uint64_t d;
   if (q->analytical && ((t + p) < q->iv[0].first))
   {
      q->mg1_uses++;
      d = mg1_delay(q);
   }
   else
      d = hl_compute(q, t, p);
   mg1_update(q, t, p, d);
   util_update(q, t, p, d);
   return d;
}

/* QueueModelBasic::computeQueueDelay, queue_model_basic.cc:35-61: the reference
 * time is the packet time, or the moving average's value with it added (:38-46) */
static uint64_t basic_queue_delay(orc_queue *q, uint64_t t, uint64_t p)
{
   const uint64_t ref_time = q->ma_type ? orc_ma_compute(q, t) : t;
   const uint64_t d = (q->queue_time > ref_time) ? (q->queue_time - ref_time) : 0;
   q->queue_time = ((q->queue_time > ref_time) ? q->queue_time : ref_time) + p;
   util_update(q, ref_time, p, d);
   return d;
}

/* QueueModelHistoryTree::computeQueueDelay, queue_model_history_tree.cc:43-126 */
ORC_EXPORT uint64_t orc_queue_compute(orc_queue *q, uint64_t t, uint64_t p)
{
   if (q->type == ORC_Q_BASIC) return basic_queue_delay(q, t, p);
   if (q->type == ORC_Q_HISTORY_LIST) return hl_queue_delay(q, t, p);
   if (q->ext)
   {
      const uint64_t dh = hk_compute(q->ext, t, p);
      util_update(q, t, p, dh);
      return dh;
   }
   uint64_t d = UINT64_MAX;
   const uint64_t m = q->min_proc;

   /* :49-56  prune the minimum node when the tree is full */
   if (q->n >= q->max_list_size)
      iv_remove(q, 0);

   /* :58-64  analytical fallback when the earliest free interval starts after the packet */
   if (q->analytical && q->iv[0].first > (t + p))
   {
      q->mg1_uses++;
      d = mg1_delay(q);
   }
   else
   {
      int i = iv_search(q, t, t + p);
      if (i < 0) abort(); /* :69-73 LOG_PRINT_ERROR("node = (NULL)") */
      orc_interval *nd = &q->iv[i];
      if (t >= nd->first)
      {
         d = 0;
         if ((t - nd->first) >= m)
         {
            uint64_t second = nd->second;
            nd->second = t;
            if ((second - (t + p)) >= m)
            {
               orc_interval nx = { t + p, second };
               iv_insert(q, nx);
            }
         }
         else
         {
            if ((nd->second - (t + p)) >= m)
               nd->first = t + p;
            else
               iv_remove(q, i);
         }
      }
      else
      {
         d = nd->first - t;
         if ((nd->second - (nd->first + p)) >= m)
            nd->first = nd->first + p;
         else
            iv_remove(q, i);
      }
   }

   /* :118  M/G/1 statistics are updated on every request */
   mg1_update(q, t, p, d);

   util_update(q, t, p, d);
   return d;
}

/* ------------------------------------------------------------------------ */
/* Event-driven network harness                                            */
/* ------------------------------------------------------------------------ */
enum { NODE_SEND = 0, NODE_RECEIVE = 1, NODE_EMESH = 2 };   /* network_model.h:116-117, emesh .h:38-41 */
enum { PORT_SELF = 0, PORT_LEFT, PORT_RIGHT, PORT_DOWN, PORT_UP, PORT_INJ };  /* emesh .h:43-50 + injection */
#define PORTS_PER_TILE 6
#define ORC_FLAG_UNMODELED 1u
#define ORC_FLAG_BROADCAST 2u   /* pkt.receiver == NetPacket::BROADCAST, broadcast tree enabled */

/* One pending Hop.  A unicast packet has one Hop in flight and keeps its state
 * in the per-packet arrays; a broadcast has one per tree edge, so its EMESH
 * events carry the tile and the accumulated zero-load delay themselves.  Events
 * of one packet at one time are at different routers (the tree visits every
 * router once), so their relative order never reaches a queue. */
typedef struct { uint64_t t; uint32_t id; uint32_t tile; uint64_t zl; } heap_ent;

typedef struct { heap_ent *a; size_t n, cap; } heap_t;

static int he_less(heap_ent x, heap_ent y)
{
   return x.t < y.t || (x.t == y.t && (x.id < y.id || (x.id == y.id && x.tile < y.tile)));
}

static void heap_push(heap_t *h, heap_ent e)
{
   if (h->n == h->cap)
   {
      h->cap = h->cap ? h->cap * 2 : 1024;
      h->a = (heap_ent *) realloc(h->a, h->cap * sizeof(heap_ent));
   }
   size_t i = h->n++;
   while (i > 0)
   {
      size_t p = (i - 1) / 2;
      if (!he_less(e, h->a[p])) break;
      h->a[i] = h->a[p];
      i = p;
   }
   h->a[i] = e;
}

static heap_ent heap_pop(heap_t *h)
{
   heap_ent top = h->a[0];
   heap_ent last = h->a[--h->n];
   size_t i = 0;
   for (;;)
   {
      size_t l = 2 * i + 1, r = l + 1, s = i;
      heap_ent best = last;
      if (l < h->n && he_less(h->a[l], best)) { s = l; best = h->a[l]; }
      if (r < h->n && he_less(h->a[r], best)) { s = r; }
      if (s == i) break;
      h->a[i] = h->a[s];
      i = s;
   }
   if (h->n) h->a[i] = last;
   return top;
}

/* Returns 0 on success, <0 on invalid configuration / trace.
 * Outputs are arrays of n (per packet) or 6*W*H (per port, index tile*6+port,
 * port 0..4 = SELF,LEFT,RIGHT,DOWN,UP of the mesh router, 5 = injection router).
 * port_flits / port_last (may be NULL): _total_utilized_cycles and
 * _last_request_time of each port's queue (queue_model.cc:49-53).
 * Broadcast packets (flags & ORC_FLAG_BROADCAST; dst ignored) take the tree
 * branch; bcast_final / bcast_zero_load (may be NULL without broadcasts) get
 * one row of W*H receipts per broadcast, in trace order, column = receiving
 * tile.  A broadcast's per-packet entries are those of its latest receipt
 * (lowest tile on ties). */
/* queue_model/basic/moving_avg_{enabled,type,window_size} for the next orc_run
 * calls (ORC_MA_NONE = moving_avg_enabled false) */
static int g_ma_type = ORC_MA_NONE;
static uint32_t g_ma_window = 1;
ORC_EXPORT int orc_set_basic_moving_avg(int ma_type, uint32_t max_window_size)
{
   if (ma_type < ORC_MA_NONE || ma_type > ORC_MA_MEDIAN || (ma_type && max_window_size < 1)) return -1;
   g_ma_type = ma_type;
   g_ma_window = max_window_size;
   return 0;
}

ORC_EXPORT int orc_run(int mesh_width, int mesh_height, int flit_width,
                       uint64_t router_delay, uint64_t link_delay, double frequency,
                       int contention_enabled, int queue_type, int interleaving, int analytical_enabled,
                       int max_list_size,
                       size_t n, const uint64_t *inject_ps, const uint32_t *src,
                       const uint32_t *dst, const uint32_t *bits, const uint32_t *flags,
                       uint64_t *final_ps, uint64_t *zero_load_ps, uint64_t *contention_ps,
                       uint64_t *port_sum_delay, uint64_t *port_count, uint64_t *port_mg1,
                       uint64_t *port_flits, uint64_t *port_last,
                       uint64_t *bcast_final, uint64_t *bcast_zero_load)
{
   const int W = mesh_width, H = mesh_height;
   if (W <= 0 || H <= 0 || flit_width <= 0 || frequency <= 0.0) return -1;
   if (contention_enabled && queue_type != ORC_Q_BASIC && max_list_size < 2) return -1;
   const uint32_t N = (uint32_t) (W * H);
   const size_t nports = (size_t) N * PORTS_PER_TILE;

   size_t nb = 0;
   for (size_t i = 0; i < n; i++)
   {
      const int bc = (flags[i] & ORC_FLAG_BROADCAST) != 0;
      if (src[i] >= N || (!bc && dst[i] >= N)) return -2;
      if (i > 0 && inject_ps[i] < inject_ps[i - 1]) return -3; /* must be time ordered */
      nb += (size_t) bc;
   }
   if (nb && (!bcast_final || !bcast_zero_load)) return -1;
   uint32_t *bidx = (uint32_t *) malloc((n ? n : 1) * sizeof(uint32_t));
   {
      uint32_t b = 0;
      for (size_t i = 0; i < n; i++) bidx[i] = (flags[i] & ORC_FLAG_BROADCAST) ? b++ : 0xFFFFFFFFu;
   }

   orc_queue **q = NULL;
   if (contention_enabled)
   {
      q = (orc_queue **) calloc(nports, sizeof(orc_queue *));
      for (size_t p = 0; p < nports; p++)
      {
         q[p] = orc_queue_create_type(queue_type, max_list_size, analytical_enabled, interleaving, 1);
         if (!q[p]) return -1;
         if (queue_type == ORC_Q_BASIC && orc_queue_set_moving_avg(q[p], g_ma_type, g_ma_window)) return -1;
      }
   }
   memset(port_sum_delay, 0, nports * sizeof(uint64_t));
   memset(port_count, 0, nports * sizeof(uint64_t));
   memset(port_mg1, 0, nports * sizeof(uint64_t));
   if (port_flits) memset(port_flits, 0, nports * sizeof(uint64_t));
   if (port_last) memset(port_last, 0, nports * sizeof(uint64_t));

   /* per-packet running state (NetPacket fields, network.h:27-55) */
   uint64_t *ptime = (uint64_t *) malloc(n * sizeof(uint64_t));
   uint32_t *ptile = (uint32_t *) malloc(n * sizeof(uint32_t));
   uint8_t *pnode = (uint8_t *) malloc(n ? n : 1);
   heap_t h = { 0, 0, 0 };

   for (size_t i = 0; i < n; i++)
   {
      ptime[i] = inject_ps[i];
      ptile[i] = src[i];
      pnode[i] = NODE_SEND;
      zero_load_ps[i] = 0;
      contention_ps[i] = 0;
      heap_ent e = { inject_ps[i], (uint32_t) i, src[i], 0 };
      heap_push(&h, e);
   }

   const uint64_t rl_ps = lat_to_ps(router_delay + link_delay, frequency);

   while (h.n)
   {
      heap_ent e = heap_pop(&h);
      const uint32_t id = e.id;
      const uint64_t t = e.t;   /* == ptime[id] for a unicast packet */
      const uint32_t F = (bits[id] % (uint32_t) flit_width) ? bits[id] / (uint32_t) flit_width + 1
                                                           : bits[id] / (uint32_t) flit_width; /* network_model.cc:202-212 */
      const int modeled = !(flags[id] & ORC_FLAG_UNMODELED); /* network_model.cc:171-183 */

      const int bc = (flags[id] & ORC_FLAG_BROADCAST) != 0;
      if (pnode[id] == NODE_SEND)
      {
         /* network_model.cc:413-468 processCornerCases: self-send -> RECEIVE, no delay;
          * network_model.cc:129-133 __processReceivedPacket returns early for it.
          * A broadcast is never a self-send (receiver is BROADCAST); its hops to the
          * system tiles (:453-459) are direct and touch no queue. */
         if ((!bc && src[id] == dst[id]) || !modeled)
         {
            /* unmodeled packets traverse with zero router/link delay and no
             * queue interaction (router_model.cc:74-75, electrical_link_model.cc:32-33),
             * and __processReceivedPacket skips serialization. */
            final_ps[id] = t;
            if (bc)
               for (uint32_t c = 0; c < N; c++)
               {
                  bcast_final[(size_t) bidx[id] * N + c] = t;
                  bcast_zero_load[(size_t) bidx[id] * N + c] = 0;
               }
            continue;
         }
         /* emesh routePacket SEND_TILE branch, :151-159: injection router (delay 0) */
         uint64_t c0 = 0;
         if (contention_enabled)
         {
            const size_t port = (size_t) src[id] * PORTS_PER_TILE + PORT_INJ;
            c0 = orc_queue_compute(q[port], time_to_cycles(t, frequency), F);
            port_sum_delay[port] += c0;
            port_count[port]++;
         }
         /* Hop(pkt, tile, EMESH, Latency(0,f), Latency(c0,f)); network_model.cc:556-563 */
         const uint64_t c0ps = lat_to_ps(c0, frequency), zl = lat_to_ps(0, frequency);
         ptime[id] = t + c0ps + zl;
         zero_load_ps[id] += zl;
         contention_ps[id] += c0ps;
         pnode[id] = NODE_EMESH;
         heap_ent ne = { ptime[id], id, src[id], zero_load_ps[id] };
         heap_push(&h, ne);
         continue;
      }

      if (bc)
      {
         /* EMESH broadcast branch, emesh_hop_by_hop.cc:163-221: the tree from the
          * sender -- UP if cy >= sy, DOWN if cy <= sy, along the sender's row
          * RIGHT if cx >= sx and LEFT if cx <= sx, then SELF; off-mesh tiles
          * (computeTileID -> INVALID_TILE_ID, :274-280) are dropped. */
         const int cur = (int) e.tile;
         const int cx = cur % W, cy = cur / W;
         const int sx = (int) (src[id] % (uint32_t) W), sy = (int) (src[id] / (uint32_t) W);
         int ports[5], nexts[5], np = 0;
         if (cy >= sy && cy + 1 < H) { ports[np] = PORT_UP; nexts[np++] = cur + W; }
         if (cy <= sy && cy - 1 >= 0) { ports[np] = PORT_DOWN; nexts[np++] = cur - W; }
         if (cy == sy)
         {
            if (cx >= sx && cx + 1 < W) { ports[np] = PORT_RIGHT; nexts[np++] = cur + 1; }
            if (cx <= sx && cx - 1 >= 0) { ports[np] = PORT_LEFT; nexts[np++] = cur - 1; }
         }
         ports[np] = PORT_SELF;
         nexts[np++] = cur;
         /* every selected link adds link_delay: zero_load += max = Lk; the router
          * adds R (router_model.cc:83) and charges the MAX queue delay over the
          * selected ports to the packet and to every one of them (:86-101, 136-144) */
         uint64_t m = 0;
         if (contention_enabled)
         {
            const uint64_t tc = time_to_cycles(t, frequency);
            for (int k = 0; k < np; k++)
            {
               const uint64_t d = orc_queue_compute(q[(size_t) cur * PORTS_PER_TILE + (size_t) ports[k]], tc, F);
               m = d > m ? d : m;
            }
            for (int k = 0; k < np; k++)
            {
               port_sum_delay[(size_t) cur * PORTS_PER_TILE + (size_t) ports[k]] += m;
               port_count[(size_t) cur * PORTS_PER_TILE + (size_t) ports[k]]++;
            }
         }
         const uint64_t tn = t + lat_to_ps(m, frequency) + rl_ps;
         const uint64_t zn = e.zl + rl_ps;
         for (int k = 0; k < np; k++)
         {
            if (ports[k] == PORT_SELF)
            {
               /* RECEIVE_TILE at this tile: + serialization (network_model.cc:142-150) */
               const uint64_t fps = lat_to_ps(F, frequency);
               bcast_final[(size_t) bidx[id] * N + (size_t) cur] = tn + fps;
               bcast_zero_load[(size_t) bidx[id] * N + (size_t) cur] = zn + fps;
               continue;
            }
            heap_ent ne = { tn, id, (uint32_t) nexts[k], zn };
            heap_push(&h, ne);
         }
         continue;
      }

      /* EMESH unicast branch, :223-256 */
      const int cur = (int) ptile[id];
      const int cx = cur % W, cy = cur / W;
      const int dx = (int) (dst[id] % (uint32_t) W), dy = (int) (dst[id] / (uint32_t) W);
      int port, next;
      if (cx > dx)      { port = PORT_LEFT;  next = cur - 1; }
      else if (cx < dx) { port = PORT_RIGHT; next = cur + 1; }
      else if (cy > dy) { port = PORT_DOWN;  next = cur - W; }
      else if (cy < dy) { port = PORT_UP;    next = cur + W; }
      else              { port = PORT_SELF;  next = cur;     }

      /* RouterModel::processPacket (router_model.cc:70-108) + link (electrical_link_model.cc:29-45) */
      uint64_t c = 0;
      if (contention_enabled)
      {
         const size_t qp = (size_t) cur * PORTS_PER_TILE + (size_t) port;
         c = orc_queue_compute(q[qp], time_to_cycles(t, frequency), F);
         port_sum_delay[qp] += c;
         port_count[qp]++;
      }
      const uint64_t cps = lat_to_ps(c, frequency);
      ptime[id] = t + cps + rl_ps;
      zero_load_ps[id] += rl_ps;
      contention_ps[id] += cps;

      if (port == PORT_SELF)
      {
         /* RECEIVE_TILE: network_model.cc:142-150 serialization, once */
         const uint64_t fps = lat_to_ps(F, frequency);
         ptime[id] += fps;
         zero_load_ps[id] += fps;
         final_ps[id] = ptime[id];
         continue;
      }
      ptile[id] = (uint32_t) next;
      heap_ent ne = { ptime[id], id, (uint32_t) next, 0 };
      heap_push(&h, ne);
   }

   /* a broadcast's per-packet entries: its latest receipt */
   for (size_t i = 0; i < n; i++)
   {
      if (bidx[i] == 0xFFFFFFFFu || !(pnode[i] == NODE_EMESH)) continue;
      const uint64_t *bf = bcast_final + (size_t) bidx[i] * N, *bz = bcast_zero_load + (size_t) bidx[i] * N;
      uint32_t best = 0;
      for (uint32_t c = 1; c < N; c++)
         if (bf[c] > bf[best]) best = c;
      final_ps[i] = bf[best];
      zero_load_ps[i] = bz[best];
      contention_ps[i] = bf[best] - inject_ps[i] - bz[best];
   }
   free(bidx);

   if (contention_enabled)
   {
      for (size_t p = 0; p < nports; p++)
      {
         port_mg1[p] = orc_queue_mg1_uses(q[p]);
         /* QueueModel::getQueueUtilization's operands, queue_model.cc:49-62 */
         if (port_flits) port_flits[p] = q[p]->util_cycles;
         if (port_last) port_last[p] = q[p]->last_request_time;
         orc_queue_destroy(q[p]);
      }
      free(q);
   }
   free(h.a);
   free(ptime);
   free(ptile);
   free(pnode);
   return 0;
}

/* ------------------------------------------------------------------------ */
/* NetworkModelEMeshHopCounter::routePacket, network_model_emesh_hop_counter.cc:143-157,
 * with NetworkModel::__routePacket / __processReceivedPacket (network_model.cc:87-150):
 * one hop SEND_TILE -> RECEIVE_TILE of Latency(H * (R + Lk)), then + Latency(F). */
ORC_EXPORT int orc_run_hop_counter(int num_tiles, int flit_width, uint64_t router_delay, uint64_t link_delay,
                                   double frequency, size_t n, const uint64_t *inject_ps, const uint32_t *src,
                                   const uint32_t *dst, const uint32_t *bits, const uint32_t *flags,
                                   uint64_t *final_ps, uint64_t *zero_load_ps, uint64_t *contention_ps)
{
   if (num_tiles <= 0 || flit_width <= 0 || link_delay != 1) return -1;
   const int W = (int) floor(sqrt((double) num_tiles));
   for (size_t i = 0; i < n; i++)
   {
      if (src[i] >= (uint32_t) num_tiles || dst[i] >= (uint32_t) num_tiles) return -2;
      contention_ps[i] = 0;
      zero_load_ps[i] = 0;
      final_ps[i] = inject_ps[i];
      if (src[i] == dst[i] || (flags[i] & ORC_FLAG_UNMODELED)) continue;   /* corner cases / model disabled */
      const int sx = (int) src[i] % W, sy = (int) src[i] / W, dx = (int) dst[i] % W, dy = (int) dst[i] / W;
      const uint64_t hops = (uint64_t) (abs(sx - dx) + abs(sy - dy));
      const uint32_t F = (bits[i] % (uint32_t) flit_width) ? bits[i] / (uint32_t) flit_width + 1
                                                           : bits[i] / (uint32_t) flit_width;
      const uint64_t lat = lat_to_ps(hops * (router_delay + link_delay), frequency);
      const uint64_t ser = lat_to_ps(F, frequency);
      zero_load_ps[i] = lat + ser;
      final_ps[i] = inject_ps[i] + lat + ser;
   }
   return 0;
}
