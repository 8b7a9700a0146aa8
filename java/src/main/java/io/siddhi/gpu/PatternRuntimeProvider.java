package io.siddhi.gpu;

import io.siddhi.core.config.SiddhiQueryContext;
import io.siddhi.core.stream.StreamJunction;
import io.siddhi.query.api.SiddhiApp;
import io.siddhi.query.api.execution.query.Query;

import java.util.Map;

/**
 * Service-provider hook consulted by the query parser before the stock input-stream parsers run
 * (CORE/util/parser/InputStreamParser.java:88-94; the maintainer's patch adds a
 * {@code ServiceLoader.load(PatternRuntimeProvider.class)} lookup there).  A provider that returns a
 * runtime takes the whole query -- input, selector and output -- onto the device; {@code null} keeps the
 * stock StateStreamRuntime / SingleStreamRuntime, so results are never silently different.
 */
public interface PatternRuntimeProvider {

    /**
     * @param app            the parsed app (the device runtime lowers all of its queries at once)
     * @param query          the query being parsed
     * @param junctions      the app's stream junctions, by stream id (input subscription, output publish)
     * @param context        the query's context (name, app context: playback, timestamp generator)
     * @return the device runtime of this query, or null when it is not lowered
     */
    GpuQueryRuntime lower(SiddhiApp app, Query query, Map<String, StreamJunction> junctions,
                          SiddhiQueryContext context);
}
