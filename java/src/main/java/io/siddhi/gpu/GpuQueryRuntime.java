package io.siddhi.gpu;

import io.siddhi.core.query.ExternalQueryRuntime;
import io.siddhi.core.query.output.callback.QueryCallback;
import io.siddhi.query.api.execution.query.Query;

/**
 * One device-lowered query.  It is the ExternalQueryRuntime the siddhi-core hook registers
 * (java/patches/siddhi-core-external-query-runtime.patch): SiddhiAppRuntime.addCallback reaches it by name.
 */
public final class GpuQueryRuntime implements ExternalQueryRuntime {
    private final GpuApp app;
    final int query;
    private final String name;
    private final Query definition;

    GpuQueryRuntime(GpuApp app, int query, String name, Query definition) {
        this.app = app;
        this.query = query;
        this.name = name;
        this.definition = definition;
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

    /** SG_PATH_* of this query (diagnostic). */
    public int path() {
        return Native.queryPath(app.handle, query);
    }
}
