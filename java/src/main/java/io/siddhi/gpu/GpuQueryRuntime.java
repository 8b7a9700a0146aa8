package io.siddhi.gpu;

import io.siddhi.core.query.output.callback.QueryCallback;

/** One device-lowered query: callbacks attach here (QueryRuntime.addCallback). */
public final class GpuQueryRuntime {
    private final GpuApp app;
    final int query;

    GpuQueryRuntime(GpuApp app, int query) {
        this.app = app;
        this.query = query;
    }

    public void addCallback(QueryCallback callback) {
        app.addQueryCallback(query, callback);
    }

    /** SG_PATH_* of this query (diagnostic). */
    public int path() {
        return Native.queryPath(app.handle, query);
    }
}
