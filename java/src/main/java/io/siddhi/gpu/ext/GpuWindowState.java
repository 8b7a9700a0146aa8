package io.siddhi.gpu.ext;

import io.siddhi.core.event.ComplexEvent;
import io.siddhi.core.event.ComplexEventChunk;
import io.siddhi.core.event.stream.StreamEvent;
import io.siddhi.core.event.stream.StreamEventCloner;
import io.siddhi.core.util.snapshot.state.State;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.IntBuffer;
import java.nio.LongBuffer;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;

/**
 * One window instance backed by a native sg_window (include/siddhi_gfx_ext.h).  The native side decides
 * what the window passes on; this class keeps the StreamEvent clones it retains (by id, in window order)
 * and rebuilds the reference's output chunks from the ids it gets back.
 */
final class GpuWindowState extends State {
    final long handle;
    // written after every native call on `handle`: the write keeps this state reachable until the call has
    // returned (Java 8 has no Reference.reachabilityFence), so the phantom-reference release in NativeHandles
    // can never free the handle under a running call
    private volatile int reach;
    private final boolean batch;
    private final boolean expiredOn;
    private long nextId = 0;
    private StreamEvent lastEvent;   // RESET events only reset aggregators: any clone serves as their body
    /** Clones the window retains (ExpiredEventQueue of the reference processors), by id. */
    final LinkedHashMap<Long, StreamEvent> held = new LinkedHashMap<>();

    GpuWindowState(int kind, long param, boolean streamCurrent, boolean expiredOn) {
        handle = NativeExt.windowCreate(kind, param, streamCurrent, expiredOn);
        // released once the state holder drops this state (@purge, canDestroy, app shutdown)
        NativeHandles.track(this, handle, NativeExt::windowDestroy);
        this.batch = kind == NativeExt.WIN_LENGTH_BATCH;
        this.expiredOn = expiredOn;
    }

    private static LongBuffer longs(int n) {
        return ByteBuffer.allocateDirect(Math.max(n, 1) * 8).order(ByteOrder.nativeOrder()).asLongBuffer();
    }

    /**
     * processEventChunk: the CURRENT events of `chunk` enter the native window at app time `now`; returns
     * the output chunks in the reference's order (the processor hands each to nextProcessor).
     */
    List<ComplexEventChunk<StreamEvent>> process(ComplexEventChunk<StreamEvent> chunk, StreamEventCloner cloner,
                                                 long now) {
        List<StreamEvent> cur = new ArrayList<>();
        chunk.reset();
        while (chunk.hasNext()) {
            StreamEvent e = chunk.next();
            if (e.getType() == ComplexEvent.Type.CURRENT) {
                cur.add(e);
            }
        }
        Map<Long, StreamEvent> fresh = new HashMap<>();
        LongBuffer ids = longs(cur.size());
        LongBuffer ts = longs(cur.size());
        for (StreamEvent e : cur) {
            long id = nextId++;
            fresh.put(id, e);
            StreamEvent clone = cloner.copyStreamEvent(e);   // what the window would hold
            clone.setType(ComplexEvent.Type.EXPIRED);
            held.put(id, clone);
            ids.put(id);
            ts.put(e.getTimestamp());
            lastEvent = e;
        }
        NativeExt.windowProcess(handle, cur.size(), ids, ts, now);
        reach = 1;
        return drain(fresh, cloner);
    }

    /** The Scheduler's TIMER event at `now`: expiry chunks of a time window. */
    List<ComplexEventChunk<StreamEvent>> onTime(long now, StreamEventCloner cloner) {
        NativeExt.windowOnTime(handle, now);
        reach = 1;
        return drain(new HashMap<>(), cloner);
    }

    private List<ComplexEventChunk<StreamEvent>> drain(Map<Long, StreamEvent> fresh, StreamEventCloner cloner) {
        long[] sz = NativeExt.windowOutSizes(handle);
        int n = (int) sz[0];
        int nc = (int) sz[1];
        LongBuffer ids = longs(n);
        IntBuffer types = ByteBuffer.allocateDirect(Math.max(n, 1) * 4).order(ByteOrder.nativeOrder()).asIntBuffer();
        LongBuffer ts = longs(n);
        LongBuffer end = longs(nc);
        NativeExt.windowOutCopy(handle, ids, types, ts, end);
        reach = 1;
        List<ComplexEventChunk<StreamEvent>> out = new ArrayList<>(nc);
        int b = 0;
        for (int c = 0; c < nc; c++) {
            ComplexEventChunk<StreamEvent> chunk = new ComplexEventChunk<>();
            int e = (int) end.get(c);
            for (int k = b; k < e; k++) {
                long id = ids.get(k);
                StreamEvent ev;
                switch (types.get(k)) {
                    case NativeExt.EV_CURRENT:
                        if (fresh.containsKey(id)) {
                            ev = fresh.get(id);
                        } else {                                    // a lengthBatch flush of held events
                            ev = cloner.copyStreamEvent(held.get(id));
                            ev.setType(ComplexEvent.Type.CURRENT);
                        }
                        if (batch && !expiredOn) {
                            held.remove(id);                        // never emitted again
                        }
                        break;
                    case NativeExt.EV_EXPIRED:
                        ev = held.remove(id);                       // leaves the window
                        if (ev == null) {                           // length(0): expires at once
                            ev = cloner.copyStreamEvent(fresh.get(id));
                            ev.setType(ComplexEvent.Type.EXPIRED);
                        }
                        break;
                    default:
                        StreamEvent src = fresh.containsKey(id) ? fresh.get(id)
                                : held.containsKey(id) ? held.get(id) : lastEvent;
                        ev = cloner.copyStreamEvent(src);
                        ev.setType(ComplexEvent.Type.RESET);
                        break;
                }
                ev.setTimestamp(ts.get(k));
                chunk.add(ev);
            }
            out.add(chunk);
            b = e;
        }
        return out;
    }

    long nextDeadline() {
        long d = NativeExt.windowNextDeadline(handle);
        reach = 1;
        return d;
    }

    /** The deadlines the native window queued since the last call (Scheduler.notifyAt, in order). */
    long[] takeDeadlines() {
        long[] d = NativeExt.windowTakeDeadlines(handle);
        reach = 1;
        return d;
    }

    @Override
    public boolean canDestroy() {
        return held.isEmpty();
    }

    @Override
    public Map<String, Object> snapshot() {
        Map<String, Object> s = new HashMap<>();
        s.put("Native", NativeExt.windowSnapshot(handle));
        reach = 1;
        s.put("Held", new LinkedHashMap<>(held));
        s.put("NextId", nextId);
        return s;
    }

    @Override
    @SuppressWarnings("unchecked")
    public void restore(Map<String, Object> state) {
        NativeExt.windowRestore(handle, (byte[]) state.get("Native"));
        NativeExt.windowTakeDeadlines(handle);   // the restored Scheduler state re-notifies its own queue
        reach = 1;
        held.clear();
        held.putAll((Map<Long, StreamEvent>) state.get("Held"));
        nextId = (Long) state.get("NextId");
    }
}
