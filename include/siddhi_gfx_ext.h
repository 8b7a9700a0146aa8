/* siddhi_gfx_ext.h — the window / aggregator extension surface of libsiddhi_gfx.so.
 *
 * The query-level ABI (siddhi_gfx.h) lowers whole queries.  These entry points back the reference's
 * extension classes one by one, so `SiddhiManager.setExtension("length", GpuLengthWindowProcessor.class)`
 * (CORE/SiddhiManager.java:223-229; WindowProcessorExtensionHolder.java:33-47 caches the map by size, so
 * register before the first app) swaps a built-in for the library's restatement while the rest of the
 * query stays on the stock runtime.  java/src/main/java/io/siddhi/gpu/ext/ holds those classes.
 *
 *   window processors  LengthWindowProcessor.process (:106-141), TimeWindowProcessor.process (:133-169),
 *                      LengthBatchWindowProcessor.process (:154-351); the same restatement the query
 *                      path runs (siddhi_amd/csrc/window_proc.hpp)
 *   aggregators        AttributeAggregatorExecutor.execute (:59-67) with the Sum/Avg/Count/Min/Max
 *                      executors' processAdd / processRemove / reset / canDestroy
 *                      (SumAttributeAggregatorExecutor.java:69-355, ... MaxAttributeAggregatorExecutor.java:69-475)
 *
 * Events stay on the Java side: a window sees ids (the shim's handle of each StreamEvent clone it holds)
 * and timestamps, and answers with the ids it passes on, their types and timestamps, chunk by chunk.
 * Values cross as 8-byte slots: INT/LONG/STRING/BOOL as integers, FLOAT as its IEEE bits in the low 32
 * bits, DOUBLE as its IEEE bits.  Return codes are siddhi_gfx.h's SG_OK / SG_E_*; sg_last_error() says why.
 */
#ifndef SIDDHI_GFX_EXT_H
#define SIDDHI_GFX_EXT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_WIN_LENGTH 1        /* #window.length(L) */
#define SG_WIN_TIME 2          /* #window.time(T ms) */
#define SG_WIN_LENGTH_BATCH 3  /* #window.lengthBatch(L[, streamCurrentEvents]) */

#define SG_EV_CURRENT 0        /* ComplexEvent.Type */
#define SG_EV_EXPIRED 1
#define SG_EV_RESET 3

#define SG_AGG_SUM 0
#define SG_AGG_AVG 1
#define SG_AGG_COUNT 2
#define SG_AGG_MIN 3
#define SG_AGG_MAX 4

typedef struct sg_window sg_window;
typedef struct sg_aggregator sg_aggregator;

/* WindowProcessor.init (AbstractStreamProcessor.initProcessor :66-98): `expired_on` is the query's
 * outputExpectsExpiredEvents (lengthBatch keeps the expired batch only then). */
int sg_window_create(int kind, int64_t param, int stream_current, int expired_on, sg_window** out);
void sg_window_destroy(sg_window* w);

/* processEventChunk of one chunk of n CURRENT events (ids[k], ts[k]) at app clock `now`.  The output
 * chunks are queued in the handle (sg_window_out_*). */
int sg_window_process(sg_window* w, int64_t n, const int64_t* ids, const int64_t* ts, int64_t now);

/* the Scheduler's TIMER chunk(s) at `now` (time windows): every deadline <= now fires one chunk */
int sg_window_on_time(sg_window* w, int64_t now);

/* the earliest Scheduler deadline the window asked for (Scheduler.notifyAt), or INT64_MIN if none */
int64_t sg_window_next_deadline(const sg_window* w);

/* Scheduler.notifyAt deadlines the window queued since the last call (TimeWindowProcessor.java:158-160
 * notifies once per new timestamp): the shim forwards every one to its Scheduler.  out == NULL returns
 * the count without taking them; otherwise cap must hold them all.  Returns the count or SG_E_*. */
int64_t sg_window_take_deadlines(sg_window* w, int64_t* out, int64_t cap);

/* queued output: n_items entries in n_chunks chunks; copy them out (clears the queue).  chunk_end[c] is
 * the index after chunk c's last entry; types are SG_EV_*. */
int sg_window_out_sizes(const sg_window* w, int64_t* n_items, int64_t* n_chunks);
int sg_window_out_copy(sg_window* w, int64_t* ids, int32_t* types, int64_t* ts, int64_t* chunk_end);

/* State.snapshot() / restore(): the held ids and counters (buffer from malloc; sg_free_buffer) */
int sg_window_snapshot(sg_window* w, uint8_t** buf, int64_t* len);
int sg_window_restore(sg_window* w, const uint8_t* buf, int64_t len);

/* AttributeAggregatorExecutor.init: `in_type` is SG_T_* of the argument (count(): any); `track` is
 * min/max trackFutureStates (a sliding window, or expired output: MinAttributeAggregatorExecutor.java:95-98) */
int sg_agg_create(int kind, int in_type, int track, sg_aggregator** out);
void sg_agg_destroy(sg_aggregator* a);
int sg_agg_out_type(const sg_aggregator* a);   /* SG_T_*: sum -> LONG / DOUBLE, avg -> DOUBLE, count -> LONG */

/* execute() for n events in order: types[k] SG_EV_*, in[k] / in_null[k] the argument; out[k] /
 * out_null[k] the aggregate after event k */
int sg_agg_process(sg_aggregator* a, int64_t n, const int32_t* types, const int64_t* in, const uint8_t* in_null,
                   int64_t* out, uint8_t* out_null);

/* canDestroy(): the state is back to its initial value (the state holder may drop it) */
int sg_agg_can_destroy(const sg_aggregator* a);

/* State.snapshot() / restore() of one aggregator state (buffer from malloc; sg_free_buffer).  restore
 * validates the whole buffer before it replaces the state. */
int sg_agg_snapshot(sg_aggregator* a, uint8_t** buf, int64_t* len);
int sg_agg_restore(sg_aggregator* a, const uint8_t* buf, int64_t len);

/* Diagnostic: chunks / batches this process ran on the device (k_ext_len, k_ext_agg_*) rather than on the host
 * restatement (chunks shorter than SG_EXT_DEVICE_MIN, min / max, or sums that could round). */
int64_t sg_ext_device_chunks(void);

#ifdef __cplusplus
}
#endif

#endif
