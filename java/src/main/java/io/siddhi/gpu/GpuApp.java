package io.siddhi.gpu;

import io.siddhi.core.config.SiddhiAppContext;
import io.siddhi.core.event.ComplexEvent;
import io.siddhi.core.event.Event;
import io.siddhi.core.query.output.callback.QueryCallback;
import io.siddhi.core.stream.StreamJunction;
import io.siddhi.core.util.snapshot.state.State;
import io.siddhi.core.util.snapshot.state.StateFactory;
import io.siddhi.core.util.snapshot.state.StateHolder;
import io.siddhi.query.api.definition.Attribute;

import io.siddhi.query.api.execution.query.Query;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.IntBuffer;
import java.nio.LongBuffer;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.List;
import java.util.Map;

/**
 * The device runtime of one SiddhiApp: input receivers that pack events into direct SoA buffers and push
 * them (sg_push), the output dispatcher that turns the callback queue (sg_out_callbacks / sg_out_rows)
 * back into QueryCallback.receive / junction publishes, and persistence (sg_snapshot / sg_restore).
 *
 * Threading as in the reference: a junction delivers to a receiver under the receiver's monitor
 * (MultiProcessStreamReceiver.java:97); every native call on the handle happens under {@code this}.
 */
final class GpuApp {
    final long handle;
    private final Map<String, StreamJunction> junctions;
    private final SiddhiAppContext appContext;
    private final Map<String, Receiver> receivers = new HashMap<>();
    private final Map<Integer, List<QueryCallback>> queryCallbacks = new HashMap<>();
    private final Map<Integer, String> streamPublish = new HashMap<>();   // device stream -> junction id
    private final Map<String, Integer> dict = new HashMap<>();            // STRING -> dictionary id
    private boolean started;
    private boolean destroyed;

    GpuApp(long handle, Map<String, StreamJunction> junctions, SiddhiAppContext appContext) {
        this.handle = handle;
        this.junctions = junctions;
        this.appContext = appContext;
    }

    synchronized GpuQueryRuntime queryRuntime(String queryName, Query definition, String outStream,
                                              List<Attribute> outAttrs) {
        if (!lowered(queryName)) {
            return null;                                   // stock runtime (reason: Native.unsupportedReason)
        }
        return new GpuQueryRuntime(this, Native.queryIndex(handle, queryName), queryName, definition, outStream,
                outAttrs);
    }

    /** The query runs on the device (every query's path is fixed when the app is created). */
    synchronized boolean lowered(String queryName) {
        int q = Native.queryIndex(handle, queryName);
        return q >= 0 && Native.queryPath(handle, q) != Native.UNSUPPORTED;
    }

    /**
     * SiddhiAppRuntime.snapshot() / persist() / restore(): the device state travels as one State of the app
     * (SiddhiAppContext.generateStateHolder, collected by SnapshotService.fullSnapshot like every stock state).
     */
    void registerState() {
        StateHolder holder = appContext.generateStateHolder("siddhi-gfx", new StateFactory<DeviceState>() {
            @Override
            public DeviceState createNewState() {
                return new DeviceState();
            }
        });
        holder.getState();
        holder.returnState(holder.getState());
    }

    private final class DeviceState extends State {
        @Override
        public boolean canDestroy() {
            return false;
        }

        @Override
        public Map<String, Object> snapshot() {
            Map<String, Object> m = new HashMap<>();
            m.put("siddhi_gfx", GpuApp.this.snapshot());
            return m;
        }

        @Override
        public void restore(Map<String, Object> state) {
            Object b = state.get("siddhi_gfx");
            if (b instanceof byte[]) {
                GpuApp.this.restore((byte[]) b);
            }
        }
    }

    synchronized void addQueryCallback(int query, QueryCallback cb) {
        live("addCallback");
        queryCallbacks.computeIfAbsent(query, k -> new ArrayList<>()).add(cb);
        Native.addQueryCallback(handle, query);
    }

    /** A stock consumer reads the device query's output stream: publish its chunks to the junction. */
    synchronized void publishStream(String streamId) {
        int s = Native.streamIndex(handle, streamId);
        streamPublish.put(s, streamId);
        Native.addStreamCallback(handle, s);
    }

    /** Subscribes one receiver per input stream of the device queries (SiddhiAppRuntimeBuilder.addQuery). */
    synchronized void subscribe(String streamId, List<Attribute> attrs) {
        if (receivers.containsKey(streamId)) {
            return;
        }
        Receiver r = new Receiver(streamId, Native.streamIndex(handle, streamId), attrs);
        receivers.put(streamId, r);
        junctions.get(streamId).subscribe(r);
    }

    synchronized void start() {
        live("start");
        if (!started) {
            Native.start(handle);
            started = true;
        }
    }

    synchronized byte[] snapshot() {
        if (destroyed) {                                   // a shut-down app has no device state to persist
            return null;
        }
        drain();
        return Native.snapshot(handle);
    }

    synchronized void restore(byte[] state) {
        live("restore");
        Native.restore(handle, state);
    }

    synchronized void shutdown() {
        if (destroyed) {                                   // (every device query of the app stops it)
            return;
        }
        drain();
        Native.destroy(handle);
        destroyed = true;
    }

    /** Every native call needs the handle: after shutdown() (Native.destroy) it is gone. */
    private void live(String what) {
        if (destroyed) {
            throw new IllegalStateException(what + " on a device app that was shut down");
        }
    }

    private int intern(String s) {
        Integer id = dict.get(s);
        if (id == null) {
            id = Native.intern(handle, s);
            dict.put(s, id);
        }
        return id;
    }

    // ---- input ---------------------------------------------------------------------------------

    /** StreamJunction.Receiver of one input stream (StreamJunction.java:468-480). */
    private final class Receiver implements StreamJunction.Receiver {
        private final String streamId;
        private final int stream;
        private final List<Attribute> attrs;
        private LongBuffer ts = direct(1024 * 8).asLongBuffer();
        private ByteBuffer[] cols;
        private ByteBuffer nulls;
        private int n;
        private boolean anyNull;

        Receiver(String streamId, int stream, List<Attribute> attrs) {
            this.streamId = streamId;
            this.stream = stream;
            this.attrs = attrs;
            this.cols = new ByteBuffer[attrs.size()];
            grow(1024);
        }

        private void grow(int cap) {
            LongBuffer t = direct(cap * 8).asLongBuffer();
            ts.flip();
            t.put(ts);
            ts = t;
            for (int k = 0; k < cols.length; k++) {
                int w = width(attrs.get(k).getType());
                ByteBuffer c = direct(cap * w);
                if (cols[k] != null) {
                    cols[k].flip();
                    c.put(cols[k]);
                }
                cols[k] = c;
            }
            ByteBuffer nb = direct(cap * cols.length);
            if (nulls != null) {
                nulls.flip();
                nb.put(nulls);
            }
            nulls = nb;
        }

        private void add(long timestamp, Object[] data) {
            if (n == ts.capacity()) {
                grow(2 * n);
            }
            ts.put(timestamp);
            for (int k = 0; k < cols.length; k++) {
                Object v = data[k];
                nulls.put((byte) (v == null ? 1 : 0));
                anyNull |= v == null;
                ByteBuffer c = cols[k];
                switch (attrs.get(k).getType()) {
                    case STRING: c.putInt(v == null ? 0 : intern((String) v)); break;
                    case INT: c.putInt(v == null ? 0 : (Integer) v); break;
                    case LONG: c.putLong(v == null ? 0L : (Long) v); break;
                    case FLOAT: c.putFloat(v == null ? 0f : (Float) v); break;
                    case DOUBLE: c.putDouble(v == null ? 0d : (Double) v); break;
                    case BOOL: c.put((byte) (v != null && (Boolean) v ? 1 : 0)); break;
                    default: throw new UnsupportedOnGpuException("OBJECT attributes are not lowered");
                }
            }
            n++;
        }

        private void push(boolean batch) {
            if (n == 0) {
                return;
            }
            synchronized (GpuApp.this) {
                if (!destroyed) {                          // (a late event after shutdown is dropped, as the
                    Native.push(handle, stream, n, ts, cols, anyNull ? nulls : null, batch);   // stopped
                }                                          // junctions of the stock runtime drop it)
                ts.clear();
                for (ByteBuffer c : cols) {
                    c.clear();
                }
                nulls.clear();
                n = 0;
                anyNull = false;
                if (!destroyed) {
                    drain();
                }
            }
        }

        @Override
        public String getStreamId() {
            return streamId;
        }

        /** The junction is delivering a chunk this app's device output published (see drain()). */
        private boolean echo() {
            return SELF_PUBLISH.get().contains(streamId);
        }

        @Override
        public synchronized void receive(ComplexEvent complexEvent) {    // a junction-internal chunk: one batch
            if (echo()) {
                return;
            }
            for (ComplexEvent e = complexEvent; e != null; e = e.getNext()) {
                add(e.getTimestamp(), e.getOutputData());
            }
            push(true);
        }

        @Override
        public synchronized void receive(Event event) {
            if (echo()) {
                return;
            }
            add(event.getTimestamp(), event.getData());
            push(false);
        }

        @Override
        public synchronized void receive(List<Event> events) {
            if (echo()) {
                return;
            }
            for (Event e : events) {
                add(e.getTimestamp(), e.getData());
            }
            push(true);
        }

        @Override
        public synchronized void receive(long timestamp, Object[] data) {
            if (echo()) {
                return;
            }
            add(timestamp, data);
            push(false);
        }

        @Override
        public synchronized void receive(Event[] events) {             // InputHandler.send(Event[]): one chunk
            if (echo()) {
                return;
            }
            for (Event e : events) {
                add(e.getTimestamp(), e.getData());
            }
            push(true);
        }
    }

    // ---- output --------------------------------------------------------------------------------

    private int width = 1;
    // streams this thread is publishing from drain() (their synchronous echo is dropped).  A stack, not one slot: a
    // stock consumer of a published stream can insert into a stream a device query reads, whose push re-enters
    // drain() on the same thread; the nested publish must not clear the outer one's marker.
    private final ThreadLocal<java.util.ArrayDeque<String>> SELF_PUBLISH =
            ThreadLocal.withInitial(java.util.ArrayDeque::new);

    /** sg_flush, then every queued callback in reference order (one per holder / selector chunk). */
    private void drain() {
        if (destroyed) {
            return;
        }
        Native.flush(handle);
        int ncb = (int) Native.outNCallbacks(handle);
        int nrows = (int) Native.outNRows(handle);
        if (ncb == 0) {
            return;
        }
        IntBuffer kind = buf(0, ncb * 4L).asIntBuffer();
        IntBuffer target = buf(1, ncb * 4L).asIntBuffer();
        LongBuffer cts = buf(2, ncb * 8L).asLongBuffer();
        IntBuffer nIn = buf(3, ncb * 4L).asIntBuffer();
        IntBuffer nRm = buf(4, ncb * 4L).asIntBuffer();
        LongBuffer rts = buf(5, Math.max(nrows, 1) * 8L).asLongBuffer();
        LongBuffer raw = buf(6, Math.max(nrows, 1) * (long) width * 8L).asLongBuffer();
        ByteBuffer nul = buf(7, Math.max(nrows, 1) * (long) width);
        Native.drain(handle, kind, target, cts, nIn, nRm, rts, raw, nul, width);
        // decode the whole drain before any callback runs: a callback may re-enter drain() on this thread (a chained
        // stock query feeding a device query), which refills the shared drain buffers
        int[] kinds = new int[ncb];
        int[] targets = new int[ncb];
        long[] times = new long[ncb];
        Event[][] ins = new Event[ncb][];
        Event[][] rms = new Event[ncb][];
        int r = 0;
        for (int i = 0; i < ncb; i++) {
            kinds[i] = kind.get(i);
            targets[i] = target.get(i);
            times[i] = cts.get(i);
            ins[i] = new Event[nIn.get(i)];
            rms[i] = new Event[nRm.get(i)];
            for (Event[] part : new Event[][]{ins[i], rms[i]}) {
                for (int k = 0; k < part.length; k++, r++) {
                    part[k] = new Event(rts.get(r), decodeRow(kinds[i], targets[i], raw, nul, r));
                }
            }
        }
        for (int i = 0; i < ncb; i++) {
            Event[] in = ins[i];
            Event[] rm = rms[i];
            if (kinds[i] == 0) {
                for (QueryCallback cb : queryCallbacks.getOrDefault(targets[i], List.of())) {
                    cb.receive(times[i], in.length > 0 ? in : null, rm.length > 0 ? rm : null);
                }
            } else {
                String id = streamPublish.get(targets[i]);
                if (id != null) {
                    // InsertIntoStreamCallback.send; this app's own receiver of the stream (if a device query reads
                    // it) drops the synchronous echo: those events already reached it inside the device
                    java.util.ArrayDeque<String> self = SELF_PUBLISH.get();
                    self.push(id);
                    try {
                        junctions.get(id).sendEvent(in);
                    } finally {
                        self.pop();
                    }
                }
            }
        }
    }

    /** Rebuilds one row's Object[] from its 8-byte slots (the output attribute / stream types). */
    private Object[] decodeRow(int kind, int target, LongBuffer raw, ByteBuffer nul, int row) {
        Attribute.Type[] types = kind == 0 ? outputTypes(target) : streamTypes(target);
        Object[] o = new Object[types.length];
        for (int k = 0; k < types.length; k++) {
            if (nul.get(row * width + k) != 0) {
                continue;
            }
            long v = raw.get(row * width + k);
            switch (types[k]) {
                case STRING: o[k] = Native.string(handle, (int) v); break;
                case INT: o[k] = (int) v; break;
                case LONG: o[k] = v; break;
                case FLOAT: o[k] = Float.intBitsToFloat((int) v); break;
                case DOUBLE: o[k] = Double.longBitsToDouble(v); break;
                case BOOL: o[k] = v != 0; break;
                default: o[k] = null;
            }
        }
        return o;
    }

    private final Map<Integer, Attribute.Type[]> outTypes = new HashMap<>();
    private final Map<Integer, Attribute.Type[]> inTypes = new HashMap<>();

    /** Registered by the provider from the descriptor's out_attrs (query) and streams (stream callbacks). */
    void setOutputTypes(int query, Attribute.Type[] types) {
        outTypes.put(query, types);
        width = Math.max(width, types.length);
    }

    void setStreamTypes(int stream, Attribute.Type[] types) {
        inTypes.put(stream, types);
        width = Math.max(width, types.length);
    }

    private Attribute.Type[] outputTypes(int q) {
        return outTypes.get(q);
    }

    private Attribute.Type[] streamTypes(int s) {
        return inTypes.get(s);
    }

    private static int width(Attribute.Type t) {
        return t == Attribute.Type.LONG || t == Attribute.Type.DOUBLE ? 8 : t == Attribute.Type.BOOL ? 1 : 4;
    }

    private final ByteBuffer[] drainBufs = new ByteBuffer[8];

    /** Drain column `i`: a direct buffer of at least `bytes`, kept across drains and grown by doubling (the
     *  native side fills it; a fresh allocateDirect per drain would zero and page in every column each time). */
    private ByteBuffer buf(int i, long bytes) {
        ByteBuffer b = drainBufs[i];
        if (b == null || b.capacity() < bytes) {
            long cap = Math.max(bytes, b == null ? 8L : 2L * b.capacity());
            if (cap > Integer.MAX_VALUE) {
                cap = bytes;
            }
            if (cap > Integer.MAX_VALUE) {
                throw new IllegalStateException("one drain's output column exceeds 2 GB; flush more often");
            }
            b = drainBufs[i] = direct((int) cap);
        }
        b.clear();
        return b;
    }

    private static ByteBuffer direct(int bytes) {
        return ByteBuffer.allocateDirect(Math.max(bytes, 8)).order(ByteOrder.nativeOrder());
    }
}
