package io.siddhi.gpu;

import io.siddhi.core.config.SiddhiQueryContext;
import io.siddhi.core.query.ExternalQueryRuntimeProvider;
import io.siddhi.core.stream.StreamJunction;
import io.siddhi.query.api.SiddhiApp;
import io.siddhi.query.api.execution.query.Query;

import java.util.Map;

/**
 * The device's ExternalQueryRuntimeProvider.  siddhi-core consults every provider on the class path before its
 * stock query parser runs, for top-level queries (SiddhiAppParser) and for the queries of a partition block
 * (PartitionParser): java/patches/siddhi-core-external-query-runtime.patch adds that lookup (the stock dispatch
 * is CORE/util/parser/InputStreamParser.java:88-94).  A provider that returns a runtime takes the whole query --
 * input, selector and output -- onto the device; {@code null} keeps the stock StateStreamRuntime /
 * SingleStreamRuntime, so results are never silently different.
 */
public interface PatternRuntimeProvider extends ExternalQueryRuntimeProvider {

    /**
     * @param app            the parsed app (the device runtime lowers all of its queries at once)
     * @param query          the query being parsed
     * @param junctions      the app's stream junctions, by stream id (input subscription, output publish)
     * @param context        the query's context (name, app context: playback, timestamp generator)
     * @return the device runtime of this query, or null when it is not lowered
     */
    @Override
    GpuQueryRuntime lower(SiddhiApp app, Query query, Map<String, StreamJunction> junctions,
                          SiddhiQueryContext context);
}
