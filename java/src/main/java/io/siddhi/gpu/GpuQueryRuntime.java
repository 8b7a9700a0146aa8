package io.siddhi.gpu;

import io.siddhi.core.query.ExternalQueryRuntime;
import io.siddhi.core.query.output.callback.QueryCallback;
import io.siddhi.core.stream.StreamJunction;
import io.siddhi.query.api.definition.Attribute;
import io.siddhi.query.api.definition.StreamDefinition;
import io.siddhi.query.api.execution.query.Query;

import java.util.List;

/**
 * One device-lowered query.  It is the ExternalQueryRuntime the siddhi-core hook registers
 * (java/patches/siddhi-core-external-query-runtime.patch): SiddhiAppRuntime.addCallback reaches it by name, the
 * builder registers its `insert into` stream and junction (SiddhiAppRuntimeBuilder.addQuery's
 * InsertIntoStreamCallback branch) and hands the junction back through {@link #publishTo}, and the app starts and
 * stops it.  Its state travels with the app's snapshot through the GpuApp's StateHolder.
 */
public final class GpuQueryRuntime implements ExternalQueryRuntime {
    private final GpuApp app;
    final int query;
    private final String name;
    private final Query definition;
    private final String outStream;
    private final List<Attribute> outAttrs;

    GpuQueryRuntime(GpuApp app, int query, String name, Query definition, String outStream, List<Attribute> outAttrs) {
        this.app = app;
        this.query = query;
        this.name = name;
        this.definition = definition;
        this.outStream = outStream;
        this.outAttrs = outAttrs;
    }

    @Override
    public String getQueryId() {
        return name;
    }

    @Override
    public Query getQuery() {
        return definition;
    }

    @Override
    public void addCallback(QueryCallback callback) {
        app.addQueryCallback(query, callback);
    }

    @Override
    public StreamDefinition getOutputStreamDefinition() {
        if (outStream == null) {
            return null;
        }
        StreamDefinition d = StreamDefinition.id(outStream);
        for (Attribute a : outAttrs) {
            d.attribute(a.getName(), a.getType());
        }
        return d;
    }

    @Override
    public void publishTo(StreamJunction junction) {
        app.publishStream(junction.getStreamDefinition().getId());
    }

    @Override
    public void start() {
        app.start();
    }

    @Override
    public void stop() {
        app.shutdown();
    }

    /** SG_PATH_* of this query (diagnostic). */
    public int path() {
        return Native.queryPath(app.handle, query);
    }
}
