/*
 * gnoc.h -- C ABI of the MI355X emesh_hop_by_hop timing engine (libgnoc.so).
 *
 * Drop-in boundary for Graphite's on-chip network timing path.  In Graphite a
 * packet walks
 *   Network::forwardPacket            common/network/network.cc:215-262
 *   NetworkModel::__routePacket       common/network/network_model.cc:87-116
 *   NetworkModelEMeshHopByHop::routePacket
 *                                     common/network/models/network_model_emesh_hop_by_hop.cc:146-264
 *   RouterModel::processPacket        common/network/components/router/router_model.cc:70-108
 *   QueueModelHistoryTree::computeQueueDelay
 *                                     common/shared_models/queue_models/queue_model_history_tree.cc:43-126
 *   NetworkModel::processReceivedPacket
 *                                     common/network/network_model.cc:142-150
 * once per hop, one packet at a time.  This library replaces that whole walk
 * for a batch of packets: the caller submits a (inject_ps, packet_id)-ordered
 * trace, calls gnoc_run, and reads back per-packet final time / zero-load /
 * contention (the three NetPacket fields the reference updates,
 * network.h:27-55) and per-output-port contention counters
 * (RouterModel::_total_contention_delay / _total_packets, router_model.h:84-85,
 * QueueModelHistoryTree::_total_requests_using_analytical_model,
 * queue_model_history_tree.h:38).
 *
 * Plain C types only; no HIP/torch types cross this boundary.  All functions
 * return 0 on success or a negative GNOC_E* code, and never abort (the
 * reference aborts through LOG_PRINT_ERROR, common/misc/log.cc:360-362).
 * Calls on one engine are not thread-safe; distinct engines are independent.
 * The caller owns every array it passes; nothing is retained after a call.
 */
#ifndef GNOC_H
#define GNOC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNOC_ABI_VERSION 4   /* 4: gnoc_submit_packed, gnoc_submit_async_packed, gnoc_fetch_latency */

/* error codes */
#define GNOC_OK             0
#define GNOC_EINVAL        -1   /* bad argument / configuration                    */
#define GNOC_ETRACE        -2   /* trace violates the submit contract              */
#define GNOC_EHIP          -3   /* HIP runtime error (message in gnoc_last_error)  */
#define GNOC_ESTATE        -4   /* call out of order (e.g. run before submit)      */
#define GNOC_EUNSUPPORTED  -5   /* valid for the reference, not implemented here   */
#define GNOC_ENOMEM        -6

/* queue model types, QueueModel::create (common/shared_models/queue_model.cc:18-38).
 * Every queue on this path sees its requests in non-decreasing time order (the
 * reference's event loop is keyed (time, packet id)), so:
 *   history_tree  the FIFO recurrence plus the serial M/G/1 prefix
 *   basic         queue_model_basic.cc:35-61 with moving_avg_enabled = false:
 *                 the plain FIFO recurrence, no analytical model
 *   history_list  queue_model_history_list.cc:39-146: the same behaviour as the
 *                 tree for max_list_size >= 2, with or without interleaving (an
 *                 in-order request never fits an earlier gap); max_list_size and
 *                 analytical_model_enabled are read from queue_model/history_list
 * basic with a moving average (carbon_sim.cfg:376-379, the cfg's default for
 * basic) is set with gnoc_set_basic_moving_average and runs on engine path 3:
 * its reference time is a running FP64 window mean, one serial walk per queue. */
#define GNOC_QUEUE_HISTORY_TREE 0
#define GNOC_QUEUE_BASIC        1
#define GNOC_QUEUE_HISTORY_LIST 2

/* queue_model/basic/moving_avg_type, MovingAverage<T>::createAvgType
 * (common/misc/moving_average.h:175-189); NONE = moving_avg_enabled false */
#define GNOC_MOVING_AVG_NONE            0
#define GNOC_MOVING_AVG_ARITHMETIC_MEAN 1
#define GNOC_MOVING_AVG_GEOMETRIC_MEAN  2
#define GNOC_MOVING_AVG_MEDIAN          3

/* per-packet flags */
#define GNOC_PKT_UNMODELED  0x1u   /* NetworkModel::isModelEnabled() == false
                                      (network_model.cc:171-183): zero delay, no queue update */
#define GNOC_PKT_BROADCAST  0x2u   /* pkt.receiver == NetPacket::BROADCAST with
                                      broadcast_tree_enabled: routed on the broadcast tree
                                      (emesh_hop_by_hop.cc:163-221); dst is ignored.  With the
                                      tree disabled the caller sends one unicast per tile, as
                                      Network::netSend does (network.cc:186-195) */

/* output ports per tile: mesh router ports SELF,LEFT,RIGHT,DOWN,UP
 * (network_model_emesh_hop_by_hop.h:43-50) then the injection router's port */
#define GNOC_PORT_SELF   0
#define GNOC_PORT_LEFT   1
#define GNOC_PORT_RIGHT  2
#define GNOC_PORT_DOWN   3
#define GNOC_PORT_UP     4
#define GNOC_PORT_INJ    5
#define GNOC_PORTS_PER_TILE 6

/* Configuration: exactly the carbon_sim.cfg keys the path reads. */
typedef struct gnoc_config
{
   int32_t  mesh_width;            /* floor(sqrt(N)), emesh_hop_by_hop.cc:54 (0 = derive from num_tiles) */
   int32_t  mesh_height;           /* ceil(N / width), emesh_hop_by_hop.cc:55                            */
   int32_t  num_tiles;             /* general/total_cores (application tiles)                            */
   int32_t  flit_width;            /* network/emesh_hop_by_hop/flit_width (bits)                        */
   uint64_t router_delay;          /* network/emesh_hop_by_hop/router/delay (cycles)                    */
   uint64_t link_delay;            /* network/emesh_hop_by_hop/link/delay (cycles); must equal
                                      ceil(f * 0.01 * tile_width), emesh_hop_by_hop.cc:126              */
   double   frequency_ghz;         /* network DVFS-domain frequency (dvfs/domains), default 1.0        */
   double   tile_width_mm;         /* general/tile_width                                                */
   int32_t  contention_enabled;    /* network/emesh_hop_by_hop/queue_model/enabled                      */
   int32_t  queue_type;            /* network/emesh_hop_by_hop/queue_model/type (GNOC_QUEUE_*)          */
   int32_t  analytical_enabled;    /* queue_model/<type>/analytical_model_enabled (tree, list)          */
   int32_t  max_list_size;         /* queue_model/<type>/max_list_size (>= 2; unused by basic)          */
   int32_t  broadcast_tree_enabled;/* network/emesh_hop_by_hop/broadcast_tree_enabled (GNOC_PKT_BROADCAST) */
   int32_t  device;                /* HIP device ordinal                                                */
} gnoc_config;

/* Fill with carbon_sim.cfg defaults for an N-tile mesh (carbon_sim.cfg:300-313, 388-392). */
void gnoc_config_default(gnoc_config *cfg, int32_t num_tiles);

/* Packet trace, struct-of-arrays.  Packet id = array index.  The trace must
 * be ordered by (inject_ps, id), i.e. inject_ps non-decreasing. */
typedef struct gnoc_packets
{
   const uint64_t *inject_ps;   /* NetPacket::time at Network::netSend                 */
   const uint32_t *src;         /* TILE_ID(pkt.sender)                                  */
   const uint32_t *dst;         /* TILE_ID(pkt.receiver); ignored for GNOC_PKT_BROADCAST */
   const uint32_t *bits;        /* NetworkModel::getModeledLength(pkt), bits            */
   const uint32_t *flags;       /* GNOC_PKT_* (may be NULL = all zero)                  */
} gnoc_packets;

/* The same trace in a narrow wire format, 15 bytes per packet instead of 24: for
 * meshes of at most 65,536 tiles and modeled lengths below 65,536 bits (checked).
 * gnoc_submit_narrow / gnoc_submit_async_narrow copy these over PCIe and widen
 * them on the device (SURVEY.md 8d end-to-end: the host link, not the engine,
 * bounds a host-to-host batch). */
typedef struct gnoc_packets_narrow
{
   const uint64_t *inject_ps;
   const uint16_t *src;
   const uint16_t *dst;
   const uint16_t *bits;
   const uint8_t *flags;        /* may be NULL = all zero */
} gnoc_packets_narrow;

/* The trace in a delta wire format for streamed batches, 6 bytes per packet when
 * the packets share one modeled length and carry no flags (8 / 9 bytes with the
 * optional arrays): the inject times as u16 differences, dt[i] = inject_ps[i] -
 * inject_ps[i-1] with inject_ps[-1] = t0, or 0xFFFF when the difference does not
 * fit below it -- that packet's inject_ps is then the next entry of abs_ps (in
 * packet order, n_abs entries in all).  Tile ids and lengths as in
 * gnoc_packets_narrow.  Decoded on the device by one scan. */
typedef struct gnoc_packets_packed
{
   uint64_t t0;
   const uint16_t *dt;
   const uint64_t *abs_ps;      /* may be NULL when n_abs == 0 */
   uint64_t n_abs;
   const uint16_t *src;
   const uint16_t *dst;
   const uint16_t *bits;        /* may be NULL: every packet has bits_all */
   uint32_t bits_all;
   uint32_t pad;
   const uint8_t *flags;        /* may be NULL = all zero */
} gnoc_packets_packed;

typedef struct gnoc_engine gnoc_engine;

typedef struct gnoc_summary
{
   uint64_t packets;            /* packets submitted                                    */
   uint64_t routed_packets;     /* packets that entered the mesh (not self/unmodeled)   */
   uint64_t mesh_hops;          /* mesh-router traversals = sum over routed of (H+1);
                                   the reference's "Switch Allocator Requests"         */
   uint64_t records;            /* hop records materialised (injection + mesh)          */
   uint64_t mg1_uses;           /* requests served by the M/G/1 fallback                */
   uint32_t levels;             /* dependency levels executed                           */
   uint32_t engine_path;        /* 0 whole-port streams, 1 chunked look-back, 2 closed form,
                                   3 serial moving-average queues, 4 port chains in time windows,
                                   5 port chains for the X phase, chunked look-back for the Y phase
                                   (the batch's Y chains declined, e.g. an M/G/1 request there) */
   double   last_run_ms;        /* device time of the last gnoc_run (HIP events)        */
   /* How the last gnoc_run got there.  Every rerun is exact; these count the
      cost.  retries: chain-engine reruns with windows half as long (a window
      overflowed LDS); fallbacks: reruns on a slower path (chain -> chunked
      levels when a request would take the M/G/1 branch or an earlier level
      wrote exception tails; chunked -> whole-port streams on a look-back
      timeout or an unsplittable burst). */
   uint32_t retries;
   uint32_t fallbacks;
   uint32_t windows;            /* chain-engine time windows of the last attempt, X phase (0 = not used) */
   uint32_t window_shift;       /* floor(log2) of the X phase's window length in ps     */
   uint32_t windows_y;          /* Y phase's windows                                     */
   uint32_t chain_protocol;     /* hand-off protocol of the last chain run: bit 8 set when the chain
                                   engine ran; bit 0 / bit 1 set when the X / Y phase used the
                                   look-back protocol (else serial; look-back is kept only when it
                                   measured > 5% faster than serial on the batch's windows); bit 10 set when
                                   the chains served the no-gap M/G/1 prefix (the batch meets the
                                   history tree's analytical branch in mesh ports); bit 11 set
                                   when only the windows that can serve M/G/1 requests ran on
                                   that instantiation (the rest on the common one) */
   uint64_t window_ps_x;        /* window length (ps) of the X phase                     */
   uint64_t window_ps_y;        /* ... of the Y phase                                    */
   /* since the last gnoc_submit: runs, and the retries / fallbacks of all of them
      (a caller timing several runs checks these, not the last run's) */
   uint32_t runs;
   uint32_t retries_total;
   uint32_t fallbacks_total;
   uint32_t abi_pad2;
} gnoc_summary;   /* ABI 3-4 layout: a client checks gnoc_abi_version() == GNOC_ABI_VERSION first */

/* Replaces NetworkModel::createModel(..., NETWORK_EMESH_HOP_BY_HOP)
 * (network_model.cc:50-71) + the RouterModel/QueueModel::create calls of
 * NetworkModelEMeshHopByHop::createRouterAndLinkModels (emesh_hop_by_hop.cc:73-128).
 * Validates what the reference asserts: N == W*H (:56-58, :309-320), the link
 * delay identity (:126), queue type (queue_model.cc:33-36). */
int gnoc_create(const gnoc_config *cfg, gnoc_engine **out);

/* The library's build identity: a SHA-256 prefix of the device sources and the
 * compile flags it was built from (profiles record it; the bench reports a
 * profile's HBM traffic only for the build that was profiled). */
const char *gnoc_build_id(void);

/* Replaces the moving-average part of QueueModelBasic's constructor
 * (queue_model_basic.cc:7-30: queue_model/basic/moving_avg_enabled, _type,
 * _window_size).  Every basic queue of the engine then computes its reference
 * time as MovingAverage::compute(packet time) (queue_model_basic.cc:38-46).
 * Requires queue_type GNOC_QUEUE_BASIC; window_size in [1, 65536] (the
 * reference divides by zero at 0).  All three averages are bit-exact; the
 * geometric mean runs glibc's own pow (graphite_amd/csrc/glibc_pow.h), so its
 * exactness holds against a reference built on x86-64 glibc 2.35 whose ifunc
 * picks __pow_fma (FMA + AVX2); another libm's pow may differ in the last bit.  Single unsharded mesh engines only
 * (GNOC_EUNSUPPORTED for sharded, sweep and hop-counter engines and, at
 * gnoc_run, for broadcast packets).  Takes effect at the next gnoc_run. */
int gnoc_set_basic_moving_average(gnoc_engine *eng, int32_t type, uint32_t window_size);

/* Replaces the stream of Network::netSend/forwardPacket calls
 * (network.cc:174-262): hands the engine one batch.  Host pointers; copied. */
int gnoc_submit(gnoc_engine *eng, const gnoc_packets *pk, size_t n);

/* Same, but the arrays already live in device memory (HBM) on cfg->device;
 * they must stay valid until gnoc_run returns. */
int gnoc_submit_device(gnoc_engine *eng, const gnoc_packets *pk, size_t n);
int gnoc_submit_narrow(gnoc_engine *eng, const gnoc_packets_narrow *pk, size_t n);
int gnoc_submit_packed(gnoc_engine *eng, const gnoc_packets_packed *pk, size_t n);

/* The host side of the delta wire format: encode a trace as gnoc_submit would take it
 * (the capture hook's layout) into the caller's arrays, one pass over the trace on
 * the host's cores.  dt, src, dst: n entries; bits, flags: n entries each, or NULL
 * (then every packet must have one length / no flags); abs_ps: room for abs_cap
 * escapes.  info: t0, the escapes the trace needs (n_abs; GNOC_EINVAL, arrays
 * unspecified, when above abs_cap: call again with room for n_abs), the length
 * every packet has (bits_all; 0xFFFFFFFF when they differ: pass bits) and the OR
 * of all flags.  GNOC_EINVAL when a tile id, length or flag does not fit the
 * narrow fields; GNOC_ENOMEM when the host is out of memory (the call never
 * throws; threads the host refuses only cost parallelism).  No engine, no device. */
typedef struct gnoc_pack_info
{
   uint64_t t0;
   uint64_t n_abs;
   uint32_t bits_all;
   uint32_t flags_any;
} gnoc_pack_info;
int gnoc_pack_trace(const gnoc_packets *pk, size_t n, uint16_t *dt, uint16_t *src, uint16_t *dst, uint16_t *bits,
                    uint8_t *flags, uint64_t *abs_ps, size_t abs_cap, gnoc_pack_info *info);

/* Runs the whole batch (all hops of all packets) on the GPU.  Blocking. */
int gnoc_run(gnoc_engine *eng);

/* Per-packet results (each pointer may be NULL).  NetPacket::time after
 * NetworkModel::processReceivedPacket, and NetPacket::zero_load_delay /
 * contention_delay, all in picoseconds. */
int gnoc_get_packet_results(gnoc_engine *eng, uint64_t *final_ps, uint64_t *zero_load_ps,
                            uint64_t *contention_ps, size_t n);

/* Per-output-port counters, arrays of num_tiles*6, index tile*6 + GNOC_PORT_*.
 * sum_delay/count = RouterModel::_total_contention_delay/_total_packets
 * (router_model.cc:136-144; injection router for GNOC_PORT_INJ); mg1_uses =
 * QueueModelHistoryTree::getTotalRequestsUsingAnalyticalModel. */
int gnoc_get_port_stats(gnoc_engine *eng, uint64_t *sum_delay, uint64_t *count,
                        uint64_t *mg1_uses, size_t nports);

/* Per-output-port utilization counters, arrays of num_tiles*6 like
 * gnoc_get_port_stats: flits = QueueModel::_total_utilized_cycles (sum of the
 * requests' flit counts) and last_cycle = _last_request_time (latest
 * arrival + queue delay + flits), queue_model.cc:49-53.  The reference's
 * link utilization is flits / last_cycle (QueueModel::getQueueUtilization,
 * queue_model.cc:56-62), averaged over the router's ports
 * (RouterModel::getAverageLinkUtilization, router_model.cc:167-183). */
int gnoc_get_port_utilization(gnoc_engine *eng, uint64_t *flits, uint64_t *last_cycle, size_t nports);

int gnoc_get_summary(gnoc_engine *eng, gnoc_summary *out);

/* Device pointer to the final_ps array (uint64_t[n]) of the last run, for
 * callers that keep results in HBM (e.g. multi-GPU gathers). */
int gnoc_device_final_ps(gnoc_engine *eng, void **dptr);

/* Kernel timing (HIP events on the engine's stream around every launch of
 * gnoc_run).  Off by default; costs one event record per launch when on. */
int gnoc_set_profiling(gnoc_engine *eng, int enable);

/* Per kernel class: name, summed device ms over the last gnoc_run, launches.
 * Fills up to cap entries; *count = number of classes. */
int gnoc_get_kernel_stats(gnoc_engine *eng, const char **names, double *total_ms,
                          uint32_t *launches, size_t cap, size_t *count);

/* ---- broadcast tree (emesh_hop_by_hop.cc:163-221) ----
 * A GNOC_PKT_BROADCAST packet leaves the sender's injection port, then at every
 * router requests UP (cy >= sy), DOWN (cy <= sy), RIGHT (cy == sy, cx >= sx),
 * LEFT (cy == sy, cx <= sx) and SELF, ports off the mesh dropped; the router
 * charges the MAX of those queues' delays to the packet and to each port's
 * contention counters (router_model.cc:86-101, 136-144), and every tile
 * receives it once.  Results per receipt: row b = the b-th broadcast of the
 * trace, column = receiving tile (n_entries = broadcasts x num_tiles).  The
 * packet's own gnoc_get_packet_results entries are those of its latest receipt
 * (lowest tile on ties).  Batches with broadcasts run in passes until the
 * visits' max delays repeat (gnoc_get_broadcast_info: count, passes); not on
 * sharded or sweep engines, and not from device traces. */
int gnoc_get_broadcast_results(gnoc_engine *eng, uint64_t *final_ps, uint64_t *zero_load_ps,
                               uint64_t *contention_ps, size_t n_entries);
int gnoc_get_broadcast_info(const gnoc_engine *eng, uint64_t *nbcast, uint32_t *passes);

/* ---- emesh_hop_counter (network_model_emesh_hop_counter.cc) ---------------
 * The contention-free mesh model: a packet's latency is
 * Latency(H * (router_delay + link_delay)), H = Manhattan distance (:143-157),
 * plus the receive serialization of NetworkModel::processReceivedPacket; no
 * per-port counters.  link_delay must be 1 (:77); mesh_width/height and
 * tile_width are ignored (floor(sqrt(N)) x ceil(N / W), :18-19). */
int gnoc_create_hop_counter(const gnoc_config *cfg, gnoc_engine **out);

/* ---- design-space sweep --------------------------
 * npoints independent simulations of the same mesh size, each with its own
 * flit width, router delay and link delay (the carbon_sim.cfg keys a sweep
 * varies), timed in ONE batch: point p is block p of a grid of blocks_x x
 * blocks_y meshes laid side by side (gnoc_sweep_layout), and XY routing never
 * leaves a packet's block.  A packet of point p, local tiles s -> d, is
 * submitted with global tiles G(p, s) -> G(p, d), where for a W x H point
 *   G(p, t) = ((p / blocks_x) * H + t / W) * (blocks_x * W) + (p % blocks_x) * W + t % W,
 * and the trace is the (inject_ps, point, id)-ordered merge of the points'
 * traces.  Results are per packet and per global port, exactly as each point
 * alone would give.  Needs f = 1 GHz and max_list_size >= 3 (the base config's
 * frequency / queue keys apply to every point). */
typedef struct gnoc_point
{
   int32_t  flit_width;      /* network/emesh_hop_by_hop/flit_width                           */
   uint64_t router_delay;    /* network/emesh_hop_by_hop/router/delay                         */
   uint64_t link_delay;      /* network/emesh_hop_by_hop/link/delay = ceil(f*0.01*tile_width) */
   double   tile_width_mm;   /* general/tile_width                                            */
} gnoc_point;

int gnoc_create_sweep(const gnoc_config *base, const gnoc_point *points, int32_t npoints, gnoc_engine **out);
int gnoc_sweep_layout(const gnoc_engine *eng, int32_t *blocks_x, int32_t *blocks_y);

/* ---- one mesh over several GPUs ---------------------------
 * XY routing (emesh_hop_by_hop.cc:229-240) sends a packet along its source
 * row, then along its destination column.  Rank r of n owns the injection and
 * LEFT/RIGHT ports of mesh rows [r*H/n, (r+1)*H/n) (its row band: the X phase)
 * and the UP/DOWN/SELF ports of columns [r*W/n, (r+1)*W/n) (its column band:
 * the Y phase).  Between the phases every routed packet's one "turn" record
 * moves from the row-band owner of its source to the column-band owner of its
 * destination: one all-to-all, done by the caller (RCCL all_to_all over xGMI,
 * or any transport) on buffers of 16-byte units:
 *   gnoc_shard(eng, rank, n)            before gnoc_submit (same trace on every rank)
 *   gnoc_submit(eng, ...)               host trace; fixes the exchange sizes
 *   gnoc_exchange_counts(eng, s, r, n)  units to send to / receive from each peer
 *   gnoc_run_begin(eng, send_dev)       prep + X phase + pack; the send buffer is
 *                                       complete when it returns
 *   (caller) all_to_all(send_dev -> recv_dev, split sizes s / r)
 *   gnoc_run_finish(eng, recv_dev)      unpack + Y phase + per-packet results
 * Results are bit-identical to an unsharded run.  A rank reports the packets it
 * delivers (destination column in its band) and the ports it owns; every other
 * entry reads 0, so an element-wise sum over ranks is the whole mesh's result.
 * gnoc_run is refused on an engine with n > 1.  Needs max_list_size >= 3
 * when contention is enabled. */
int gnoc_shard(gnoc_engine *eng, int32_t rank, int32_t nranks);
int gnoc_exchange_counts(gnoc_engine *eng, uint64_t *send_units, uint64_t *recv_units, size_t nranks);
int gnoc_run_begin(gnoc_engine *eng, void *send_dev);
int gnoc_run_finish(gnoc_engine *eng, const void *recv_dev);

/* The same run without a caller-side harness (SURVEY.md 8b:
 * gnoc_create_sharded(cfg, rank, nranks, ncclComm_t)): the engine keeps the
 * send / receive buffers and does the all-to-all itself, either over RCCL
 * (gnoc_shard_set_comm: an ncclComm_t of the shard count, this engine's rank,
 * on this engine's device; grouped ncclSend / ncclRecv over xGMI) or through a
 * caller transport (gnoc_shard_set_transport; in-process tests, other fabrics).
 * Around the exchange every rank's status is max-reduced, so a failure on one
 * rank fails every rank's gnoc_run_sharded (none waits on a failed peer). */
typedef struct gnoc_transport
{
   /* Move send_units[q] 16-byte units to rank q and receive recv_units[q] from it
    * (rank q's block starts at the sum of the units of ranks < q; own entry 0).
    * Device buffers; `stream` (a hipStream_t) holds the producing work.
    * Return 0 when the receive buffer is complete. */
   int (*exchange)(void *ctx, const void *send_dev, const uint64_t *send_units, void *recv_dev,
                   const uint64_t *recv_units, void *stream);
   /* *out = max over ranks of `status` (0 = ok); return 0 on success. */
   int (*agree)(void *ctx, int32_t status, int32_t *out);
   void *ctx;
} gnoc_transport;
int gnoc_shard_set_comm(gnoc_engine *eng, void *nccl_comm);
int gnoc_shard_set_transport(gnoc_engine *eng, const gnoc_transport *tp);
int gnoc_run_sharded(gnoc_engine *eng);
/* An ncclComm_t for gnoc_shard_set_comm, made by the RCCL library libgnoc links
 * (callers without their own RCCL binding, e.g. Python over ctypes): rank 0
 * calls gnoc_rccl_unique_id, the caller broadcasts the GNOC_RCCL_ID_BYTES bytes
 * to every rank by any channel, and each rank calls gnoc_rccl_comm_init on its
 * engine's device (collective: every rank must call it).  gnoc_run_sharded with
 * a communicator set runs the whole protocol even at one rank. */
#define GNOC_RCCL_ID_BYTES 128
int gnoc_rccl_unique_id(void *id_out);
int gnoc_rccl_comm_init(int32_t nranks, int32_t rank, int32_t device, const void *id, void **comm_out);
int gnoc_rccl_comm_destroy(void *comm);

/* Pipelined batches (host trace -> host results, SURVEY.md 8d end to end): the
 * upload of batch k+1 and the read-back of batch k overlap the runs beside them.
 *   gnoc_submit_async(eng, pk, n)   starts copying a host trace (page-locked for
 *                                   the copy to overlap) into the engine's second
 *                                   trace buffer on its own stream and returns; the
 *                                   arrays stay valid until gnoc_submit_commit
 *   gnoc_submit_commit(eng)         waits for that copy, checks the batch as
 *                                   gnoc_submit does and makes it the current one
 *   gnoc_fetch_final_ps(eng, out, n) starts copying the last run's final_ps into
 *                                   `out` (page-locked) on a third stream; the next
 *                                   gnoc_run writes a second buffer meanwhile
 *   gnoc_fetch_wait(eng)            waits for the started read-backs
 * e.g. submit(0); loop k: submit_async(k+1); run(k); fetch_final_ps(k);
 * submit_commit(k+1).  Unsharded engines, unicast batches. */
int gnoc_submit_async(gnoc_engine *eng, const gnoc_packets *pk, size_t n);
int gnoc_submit_async_narrow(gnoc_engine *eng, const gnoc_packets_narrow *pk, size_t n);
int gnoc_submit_async_packed(gnoc_engine *eng, const gnoc_packets_packed *pk, size_t n);
int gnoc_submit_commit(gnoc_engine *eng);
int gnoc_fetch_final_ps(gnoc_engine *eng, uint64_t *final_ps_out, size_t n);
/* The narrow read-back: per packet latency_ps = final_ps - inject_ps (NetPacket::time
 * minus its send time, network.cc:215-262) as u32, half the bytes of final_ps.
 * Pipelined like gnoc_fetch_final_ps (same double buffering, gnoc_fetch_wait).
 * GNOC_EUNSUPPORTED if a latency of the last run is 2^32 ps or more (then read
 * final_ps).  The run writes the u32 array only once a caller has asked for it
 * (the first call reads it after the next run). */
int gnoc_fetch_latency(gnoc_engine *eng, uint32_t *latency_ps_out, size_t n);
int gnoc_fetch_wait(gnoc_engine *eng);

const char *gnoc_last_error(const gnoc_engine *eng);
void gnoc_destroy(gnoc_engine *eng);

/* ---- trace helpers (not on the timed path) ---------------------------- */

/* Synthetic traffic of tests/benchmarks/synthetic_network/synthetic_network.cc:
 * per tile, per cycle, Bernoulli(offered_load) with drand48_r seeded
 * (seed + tile) (the reference seeds with time(NULL), common/misc/random.h:15-18);
 * destinations from the reference's uniform_random LCG schedule (:247-301).
 * hotspot_fraction > 0 redirects that fraction of packets (own drand48 stream,
 * seed + 0x5bd1e995 + tile) uniformly to the memory-controller tiles of
 * computeMemoryControllerPositions(num_hotspots, N) (emesh_hop_by_hop.cc:323-364).
 * Packets are 8-byte USER messages -> (sizeof(NetPacket)=64 + payload)*8 bits
 * (network.cc:705-708).  Output is (inject_ps, src)-ordered; ids are ranks.
 * Call with NULL arrays to get the count in *n_out. */
int gnoc_trace_synthetic(int32_t mesh_width, int32_t mesh_height, double frequency_ghz,
                         double offered_load, uint64_t packets_per_tile, uint32_t payload_bytes,
                         uint64_t seed, double hotspot_fraction, int32_t num_hotspots,
                         uint64_t *inject_ps, uint32_t *src, uint32_t *dst, uint32_t *bits,
                         size_t capacity, size_t *n_out);

/* The reference generator's other traffic patterns (NetworkTrafficType,
 * synthetic_network.cc:16-24, 288-341), same timing model as above: every
 * packet of a tile goes to one destination.  BIT_COMPLEMENT and SHUFFLE need a
 * power-of-two tile count; TRANSPOSE a destination inside the mesh (GNOC_EINVAL
 * otherwise, where the reference asserts). */
#define GNOC_TRAFFIC_UNIFORM_RANDOM    0
#define GNOC_TRAFFIC_BIT_COMPLEMENT    1
#define GNOC_TRAFFIC_SHUFFLE           2
#define GNOC_TRAFFIC_TRANSPOSE         3
#define GNOC_TRAFFIC_TORNADO           4
#define GNOC_TRAFFIC_NEAREST_NEIGHBOR  5
int gnoc_trace_synthetic_pattern(int32_t pattern, int32_t mesh_width, int32_t mesh_height, double frequency_ghz,
                                 double offered_load, uint64_t packets_per_tile, uint32_t payload_bytes,
                                 uint64_t seed, double hotspot_fraction, int32_t num_hotspots,
                                 uint64_t *inject_ps, uint32_t *src, uint32_t *dst, uint32_t *bits,
                                 size_t capacity, size_t *n_out);

/* ---- on-disk trace format ----------------------------
 * A batch captured at Network::netSend / NetworkModel::__routePacket(SEND_TILE)
 * (network.cc:174-215, network_model.cc:95-107), with the configuration it was
 * captured under:  gnoc_trace_header (128 bytes, little endian), then the SoA
 * arrays inject_ps[n] (u64), src[n], dst[n], bits[n], flags[n] (u32 each).   */
#define GNOC_TRACE_MAGIC "GNOCTRC1"
typedef struct gnoc_trace_header
{
   char     magic[8];            /* GNOC_TRACE_MAGIC                                  */
   uint32_t version;             /* 2 (version-1 files read with ma_type = NONE)      */
   uint32_t header_bytes;        /* 128                                                */
   uint64_t num_packets;
   gnoc_config cfg;              /* the configuration the trace was captured under     */
   int32_t  ma_type;             /* v2: queue_model/basic moving average (GNOC_MOVING_AVG_*) */
   uint32_t ma_window;           /* v2: its window size                               */
   uint8_t  reserved[128 - 32 - sizeof(gnoc_config)];
} gnoc_trace_header;

/* Queue settings outside gnoc_config that a trace carries (header v2): the basic
 * queue's moving average, gnoc_set_basic_moving_average (queue_model_basic.cc:7-30). */
typedef struct gnoc_trace_queue
{
   int32_t  ma_type;             /* GNOC_MOVING_AVG_NONE = moving_avg_enabled false */
   uint32_t ma_window;
} gnoc_trace_queue;

/* Write a (inject_ps, id)-ordered batch and its configuration to `path`
 * (moving average NONE). */
int gnoc_trace_file_write(const char *path, const gnoc_config *cfg, const gnoc_packets *pk, size_t n);
/* The same with the queue settings (q may be NULL: NONE). */
int gnoc_trace_file_write_q(const char *path, const gnoc_config *cfg, const gnoc_trace_queue *q,
                            const gnoc_packets *pk, size_t n);

/* Read `path`: with NULL arrays, fills *cfg_out and *n_out only; then call
 * again with arrays of capacity >= *n_out. */
int gnoc_trace_file_read(const char *path, gnoc_config *cfg_out, uint64_t *inject_ps, uint32_t *src, uint32_t *dst,
                         uint32_t *bits, uint32_t *flags, size_t capacity, size_t *n_out);
/* The same, also filling *q_out (NONE for a version-1 file) when not NULL. */
int gnoc_trace_file_read_q(const char *path, gnoc_config *cfg_out, gnoc_trace_queue *q_out, uint64_t *inject_ps,
                           uint32_t *src, uint32_t *dst, uint32_t *bits, uint32_t *flags, size_t capacity,
                           size_t *n_out);

int gnoc_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* GNOC_H */
