/*
 * siddhi_gfx.h — C ABI of the MI355X (gfx950) execution path for Siddhi pattern / sequence
 * matching over windowed streams.
 *
 * Plain C types only (no HIP / torch types).  One handle = one SiddhiAppRuntime restricted to
 * the hot-path queries.  Every entry point returns 0 on success or a negative SG_E_* code;
 * sg_last_error() gives the thread-local message.  A descriptor feature the GPU path does not
 * implement yields SG_E_UNSUPPORTED at create time — the Java shim then keeps the stock
 * StateStreamRuntime for that query (never a silently different result).
 *
 * Reference interfaces each entry point replaces (CORE = modules/siddhi-core/src/main/java/io/siddhi/core/):
 *   sg_app_create        SiddhiManager.createSiddhiAppRuntime(String)            CORE/SiddhiManager.java:94-97
 *                        + StateInputStreamParser.parseInputStream              CORE/util/parser/StateInputStreamParser.java:76-146
 *   sg_app_destroy       SiddhiAppRuntime.shutdown()                              CORE/SiddhiAppRuntime.java:116-167
 *   sg_stream_index      SiddhiAppRuntime.getInputHandler(String)                 CORE/SiddhiAppRuntime.java:116-167
 *   sg_add_query_callback / sg_add_stream_callback
 *                        SiddhiAppRuntime.addCallback(query|stream, callback)     CORE/SiddhiAppRuntime.java:116-167
 *   sg_start             SiddhiAppRuntime.start()                                 CORE/SiddhiAppRuntimeImpl.java:449-513
 *   sg_push              InputHandler.send(long,Object[]) / send(Event[])          CORE/stream/input/InputHandler.java:59-94
 *                        -> StreamJunction.Receiver.receive(...)                  CORE/stream/StreamJunction.java:468-480
 *   sg_push_device       same, columns already resident in HBM (zero-copy ingest)
 *   sg_advance_time      TimestampGeneratorImpl.setCurrentTimestamp / wall clock CORE/util/timestamp/TimestampGeneratorImpl.java:105-122
 *   sg_flush + sg_out_*  QueryCallback.receive(ts, in[], removed[]) / StreamCallback.receive(Event[])
 *                        CORE/query/output/callback/QueryCallback.java:61-91, CORE/stream/output/StreamCallback.java:93-104
 *   sg_intern / sg_string  the String <-> dictionary-id mapping the JNI shim keeps for STRING columns
 */
#ifndef SIDDHI_GFX_H
#define SIDDHI_GFX_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_OK 0
#define SG_E_INVALID (-1)      /* bad argument / malformed descriptor */
#define SG_E_UNSUPPORTED (-2)  /* descriptor or batch feature not implemented on the GPU path */
#define SG_E_DEVICE (-3)       /* HIP runtime error */
#define SG_E_CAPACITY (-4)     /* a fixed device pool overflowed (never silently truncated) */
#define SG_E_STATE (-5)        /* call not valid in the current runtime state */

typedef struct sg_app sg_app;

/* Attribute encoding of a column (matches io.siddhi.query.api.definition.Attribute.Type). */
#define SG_T_STRING 0 /* int32 dictionary id */
#define SG_T_INT 1    /* int32 */
#define SG_T_LONG 2   /* int64 */
#define SG_T_FLOAT 3  /* float32 */
#define SG_T_DOUBLE 4 /* float64 */
#define SG_T_BOOL 5   /* uint8 */

typedef struct sg_options {
  int device;          /* HIP device ordinal (default 0) */
  int64_t capacity;    /* expected events per flush (pre-sizes device buffers; 0 = grow) */
} sg_options;

/* Descriptor: the app's streams and queries as JSON, schema include/siddhi_gfx_descriptor.schema.json
 * (version SG_DESCRIPTOR_VERSION; INTEGRATION.md §3 shows the Java side emitting it from the parsed
 * SiddhiApp / StateInputStreamParser graph, siddhi_amd/ql.py emits it from QL text for the tests).
 * Creation lowers every query and needs no GPU: the device is bound at the first sg_start / sg_push.
 * A query no device path lowers does not fail the app: sg_query_path returns SG_E_UNSUPPORTED for it and
 * sg_query_unsupported_reason says why (the shim keeps the stock Java runtime for that query). */
#define SG_DESCRIPTOR_VERSION 1
int sg_app_create(const char* descriptor_json, const sg_options* opts, sg_app** out);
void sg_app_destroy(sg_app* app);
const char* sg_last_error(void);

int sg_stream_index(sg_app* app, const char* stream_name);
int sg_query_index(sg_app* app, const char* query_name);
int sg_stream_arity(sg_app* app, int stream);
int sg_stream_attr_type(sg_app* app, int stream, int attr);
/* Which execution path a query was lowered to (diagnostic): see SG_PATH_*. */
#define SG_PATH_FOLLOWED_BY 1  /* every e1=S[f1] -> e2=S'[f2(e1,e2)] within W : start-parallel scan kernel */
#define SG_PATH_NFA 2          /* general per-partition NFA interpreter kernel */
#define SG_PATH_WINDOW_AGG 3   /* filter + length window + group-by aggregators */
#define SG_PATH_KEYED_FOLLOWED_BY 4  /* partition with (k of S) + every e1 -> e2 within W: key-sorted scan */
#define SG_PATH_WINDOW 5       /* any single-stream query: filter + window + full selector, partitions, expired output */
int sg_query_path(sg_app* app, int query);   /* SG_PATH_* or SG_E_UNSUPPORTED */
/* NULL when the query is lowered, else the reasons every path gave (valid until sg_app_destroy). */
const char* sg_query_unsupported_reason(sg_app* app, int query);
int sg_query_count(sg_app* app);
int sg_stream_count(sg_app* app);

int sg_intern(sg_app* app, const char* s);
const char* sg_string(sg_app* app, int id);

int sg_add_query_callback(sg_app* app, int query);
int sg_add_stream_callback(sg_app* app, int stream);
int sg_start(sg_app* app);
/* Drop every partial match and buffered event but keep device allocations (a restarted runtime). */
int sg_reset(sg_app* app);

/* A columnar batch in host memory.  cols[k] points at n values of the attribute's encoding;
 * nulls (optional) is n*arity bytes, row-major.  batch != 0 means one InputHandler.send(Event[])
 * chunk; batch == 0 means n successive send(ts, data) calls. */
typedef struct sg_batch {
  int64_t n;
  const int64_t* ts;
  const void* const* cols;
  const uint8_t* nulls;
  int batch;
  /* optional: the global arrival sequence number of each event (multi-GPU: events routed to the rank
   * owning their partition key carry their position in the unrouted stream, so every callback's
   * sg_out_callback_seq orders the ranks' outputs back into single-runtime order); NULL = consecutive */
  const int64_t* seq;
} sg_batch;

int sg_push(sg_app* app, int stream, const sg_batch* b);
/* Same, but ts/cols are device pointers (HBM-resident input, adopted without a copy); hip_stream is a
 * hipStream_t or NULL.  Timestamps must be non-decreasing, as sg_push enforces for host batches: the
 * flush checks them while it stages the events (or in one pass) and fails with SG_E_INVALID.  On the followed-by paths (unkeyed and keyed) a column the query never
 * references may be NULL (it is never read), so a multi-GPU router need not move it. */
int sg_push_device(sg_app* app, int stream, int64_t n, const int64_t* d_ts, const void* const* d_cols,
                   int batch, void* hip_stream);
/* sg_push_device with the events' global arrival sequence numbers (int64, device-resident): the input a
 * multi-GPU rank pushes after routing events to their key owners (see sg_batch.seq).  Keyed followed-by
 * path only (SG_E_UNSUPPORTED elsewhere). */
int sg_push_device_seq(sg_app* app, int stream, int64_t n, const int64_t* d_ts, const void* const* d_cols,
                       const int64_t* d_seq, int batch, void* hip_stream);
/* Multi-GPU key sharding of apps whose state follows the clock (playback apps with absent
 * states or time windows): this rank's share of ONE global send.  The global send holds n_global events
 * with timestamps global_ts[k] and arrival seqs seq0 + k (b->batch != 0: one send(Event[]); else n_global
 * successive send(ts, data) calls); b holds the events of it this rank owns, b->seq their global seqs
 * (increasing).  The playback clock advances over every global event as InputHandler.send ->
 * TimestampGeneratorImpl.setCurrentTimestamp does (InputHandler.java:59-70, TimestampGeneratorImpl.java:
 * 105-122), so Scheduler ticks fire on every rank where the single runtime fires them and carry its seq;
 * local events are processed at the clock of their own send.  No reference interface: the split is new. */
int sg_push_shard(sg_app* app, int stream, const sg_batch* b, int64_t n_global, const int64_t* global_ts,
                  int64_t seq0);
/* Multi-GPU split of an unkeyed `every e1 -> e2 within W` query: rank g owns a contiguous
 * time range and also receives the next range's events within W of its end.  Declares that the last
 * n_halo events pushed to `stream` (so far, since sg_reset) are such halo events: at the next flush they
 * complete this range's partials but start none, so the ranks' outputs merged by trigger are the
 * single-GPU output.  No reference interface: the split itself is new (StreamPreStateProcessor.java:
 * 363-403 is the per-partial rule it preserves).  SG_E_UNSUPPORTED on other query paths. */
int sg_set_halo(sg_app* app, int stream, int64_t n_halo);
/* Wall-clock emulation (non-playback apps): System.currentTimeMillis() becomes now_ms. */
int sg_advance_time(sg_app* app, int64_t now_ms);
/* Run the device kernels over everything pushed so far and materialise callbacks. */
int sg_flush(sg_app* app);
/* Like sg_flush, but leave the match records in HBM (no device->host copy): bench path. */
int sg_flush_device(sg_app* app, void* hip_stream);

/* Materialised outputs, in the order the reference fires its callbacks. */
/* Persistence (SiddhiAppRuntime.snapshot() -> byte[] / restore(byte[]), CORE/SiddhiAppRuntimeImpl.java;
 * the per-processor state maps of StreamPreStateProcessor.StreamPreState.snapshot,
 * CORE/query/input/stream/state/StreamPreStateProcessor.java:450-469, the window processors' queues and
 * the aggregators' state maps).  sg_snapshot flushes first (its callbacks stay queued), then writes the
 * state of every query into a malloc'ed buffer released with sg_free_buffer.  sg_restore loads it into an
 * app created from the same descriptor (same queries, same paths) and discards queued callbacks; sends
 * after it continue exactly where the snapshotted runtime stood.  Paths without snapshot support
 * (SG_PATH_FOLLOWED_BY, SG_PATH_KEYED_FOLLOWED_BY, SG_PATH_WINDOW_AGG) make sg_snapshot return
 * SG_E_UNSUPPORTED naming the query; the buffer format is tied to this library build. */
int sg_snapshot(sg_app* app, uint8_t** out, int64_t* len);
int sg_restore(sg_app* app, const uint8_t* buf, int64_t len);
void sg_free_buffer(void* p);

int64_t sg_out_ncallbacks(sg_app* app);
/* kind: 0 = QueryCallback, 1 = StreamCallback; target = query / stream index */
int sg_out_callbacks(sg_app* app, int32_t* kind, int32_t* target, int64_t* ts, int32_t* n_in, int32_t* n_rm);
int64_t sg_out_nrows(sg_app* app);
/* rows: in-events then removed-events per callback; width slots of 8 bytes (int32 sign-extended,
 * float32 bits zero-extended, float64 bits, bool 0/1, string id). */
int sg_out_rows(sg_app* app, int width, int64_t* ts, int64_t* raw, uint8_t* nulls);
/* Arrival sequence number of the send that fired each callback (the merge key of multi-GPU outputs:
 * PartitionStreamReceiver delivers each key's callbacks in global arrival order, a send belongs to one
 * key, hence to one rank). */
int sg_out_callback_seq(sg_app* app, int64_t* seq);
/* For callbacks a Scheduler tick fired (absent states, Scheduler.java:74-104), the scheduler (absent
 * processor) index and the deadline it fired under; -1 / 0 for callbacks of a send itself.  At one seq the
 * single runtime fires the tick's callbacks first (InputHandler.send -> setCurrentTimestamp before the
 * event is dispatched), in (scheduler, deadline) order across partition keys: the multi-GPU merge key after
 * the seq. */
int sg_out_callback_tick(sg_app* app, int32_t* sched, int64_t* deadline);
int sg_out_clear(sg_app* app);

/* Device-resident match statistics of the last flush (bench): number of matches per query. */
int64_t sg_last_match_count(sg_app* app, int query);
/* Average duration (ms) of the dominant kernel over the last flush, measured with HIP events. */
double sg_last_kernel_ms(sg_app* app, const char* kernel);
/* Events the query still holds after its last flush (its buffers are compacted to the open partials /
 * the current window), or -1 where the path does not track it.  Operational metric for long runs. */
int64_t sg_query_buffered(sg_app* app, int query);

/* Run-time compiled kernel of a query on the general NFA path (SG_PATH_NFA).  The library generates HIP source
 * specialised to the query's lowered state graph -- the processor table as compile-time constants (the
 * StreamPre/Post, CountPre/Post, LogicalPre/Post and AbsentPre processors StateInputStreamParser.java:148-408
 * builds), every filter and projection as a straight-line typed function -- and compiles it with hipRTC for
 * gfx950; large flushes then run it instead of the bytecode interpreter (SG_NFA_RTC=0 / 1 / unset: never /
 * always / runs of >= SG_NFA_RTC_MIN events, default 65,536).  Code objects are cached per process and on disk
 * (SG_RTC_CACHE, default <library dir>/rtc_cache).  No reference interface: the JVM runs the processor objects.
 *   sg_query_kernel_source: the generated source; returns its length and copies up to cap - 1 bytes + NUL.
 *   sg_query_compile: compile it into the cache now (no GPU needed; callable from several threads for different
 *   apps); *compile_ms = hipRTC time (0 when cached), *from_cache = 1 when the disk cache held it.
 * Both return SG_E_UNSUPPORTED for a query on another path. */
int64_t sg_query_kernel_source(sg_app* app, int query, char* buf, int64_t cap);
int sg_query_compile(sg_app* app, int query, double* compile_ms, int* from_cache);

/* Cross-rank Scheduler collisions of a partitioned query with absent states (config 5 sharded by key).
 * Scheduler.notifyAt keeps one SchedulerState per deadline in its TreeMultimap (SchedulerState.compareTo
 * == 0, Scheduler.java:77-97, 120-147): when instances of two keys wait on one deadline only the first in
 * the key -> state HashMap's iteration order fires at that tick.  Keys on different ranks never see each
 * other, so a rank in shard mode does not resolve collisions itself: every flush re-runs its instances
 * from the start with the deferrals it was given, logs its firings (and, in mode 2, every notifyAt), and
 * the driver (siddhi_amd/shard.py: resolve_collisions) replays the global map order over all ranks' logs,
 * picks each collision's winner and defers the losers on their owner ranks, until no tick collides.
 * No reference interface: the reference runs one Scheduler per query in one JVM. */
typedef struct sg_sched_fire {
  int64_t key;          /* partition key value (string id / int) */
  int64_t head;         /* the deadline the state was collected under */
  int64_t seq;          /* global arrival seq of the send the tick precedes */
  int32_t tick;         /* Scheduler tick index (identical on every rank: global clock, sg_push_shard) */
  int8_t sched;         /* absent-state Scheduler (order of the absent states in the query) */
  int8_t empty_after;   /* the state's deadline queue is empty after firing: it leaves the map */
  int16_t pad;
} sg_sched_fire;
typedef struct sg_sched_op {  /* one Scheduler.notifyAt */
  int64_t seq;          /* global arrival seq of the send it belongs to (a tick: the send it precedes) */
  int64_t head;         /* firing head deadline (tick phase) */
  int64_t key;          /* partition key value */
  int32_t tick;         /* tick index (tick phase), else -1 */
  int32_t sub;          /* order inside one firing / event */
  int32_t pos;          /* event phase: the event's arrival rank on this rank (orders events of one send) */
  int8_t phase;         /* 0 = inside a tick's onTimeChange, 1 = event processing */
  int8_t kfire;         /* firing Scheduler (tick phase) */
  int8_t ktarget;       /* Scheduler notified */
  int8_t pad;
} sg_sched_op;
/* mode 0: resolve collisions locally (single runtime); 1: shard mode, log firings; 2: also log notifyAt.
 * In shard mode every flush re-runs the rank's instances from the start and reports that whole run's
 * callbacks (a rank with no new events or deferrals since its last run reports the same run again). */
int sg_query_shard_mode(sg_app* app, int query, int mode);
/* The last flush's firing / notifyAt logs (shard mode): returns the count, copies min(count, cap). */
int64_t sg_query_sched_fires(sg_app* app, int query, sg_sched_fire* out, int64_t cap);
int64_t sg_query_sched_ops(sg_app* app, int query, sg_sched_op* out, int64_t cap);
/* Defer the firing of key's instance at (tick, sched): it lost the deadline to another instance. */
int sg_query_sched_defer(sg_app* app, int query, int64_t key, int32_t tick, int32_t sched);
/* The Scheduler ticks' clocks (TimestampGeneratorImpl.currentTime at each onTimeChange, Scheduler.java:74-104;
 * identical on every rank in shard mode) and the shortest absent-state wait (`for` T,
 * AbsentStreamPreStateProcessor.java:35-343): what the driver needs to resolve every collision one round's
 * logs still describe, not only the first.  Returns the tick count, copies min(count, cap) clocks. */
int64_t sg_query_sched_clock(sg_app* app, int query, int64_t* now, int64_t cap, int64_t* min_wait);
/* Streaming shard mode (mode 3): the rank runs like a single runtime -- each flush from its settled base, the
 * exact windowed sweep after a collision (checkpointed pools, only deferred instances re-run, the base moving to
 * the sweep's end) -- and asks `resolve` wherever the single runtime would read its own Scheduler maps, so the
 * driver can answer from every rank's logs:
 *   kind 0 (after a flush's run): the run's firings; returns the first colliding (tick << 8 | sched) across all
 *          ranks, or -1 when none;
 *   kind 1 (one window of the sweep): the window's firings and notifyAt ops; returns 1 with this rank's losers in
 *          `defer` as (key, tick, sched) triples (*ndefer of them, at most cap), or 0 when the window has no
 *          collision left (the driver then advances its maps over the window);
 *   a negative return aborts the flush (SG_E_INVALID).
 * Every rank calls it the same number of times with the same kinds (the window bounds are global ticks), so a
 * driver that all-gathers the logs at each call keeps the ranks in step (siddhi_amd/shard.py StreamingResolver). */
typedef int64_t (*sg_shard_resolver_fn)(void* user, int32_t kind, const sg_sched_fire* fires, int64_t nfires,
                                        const sg_sched_op* ops, int64_t nops, int64_t* defer, int64_t cap,
                                        int64_t* ndefer);
int sg_query_shard_resolver(sg_app* app, int query, sg_shard_resolver_fn resolve, void* user);

/* The pattern state of a pattern / sequence query after the last flush, in the shape of the reference's
 * StreamPreStateProcessor.StreamPreState.snapshot (StreamPreStateProcessor.java:450-469) per partition instance
 * (creation order) and pre-state processor (the parser's preStateProcessors order): JSON
 *   {"instances":[{"key":K|null,"processors":[{"initialized":b,"pending":[SE..],"new_and_every":[SE..]
 *                                               [,"last_scheduled":t]}..]}..]}
 * with SE = {"ts":t,"type":y,"slots":[[[ts, raw attribute slots (null: null)..] per chain event] per slot]}.
 * Copies min(length, cap) bytes (no terminator) and returns the length; SG_E_UNSUPPORTED for other paths. */
int64_t sg_query_state_json(sg_app* app, int query, char* buf, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* SIDDHI_GFX_H */
