package io.siddhi.gpu.ext;

import java.lang.ref.PhantomReference;
import java.lang.ref.Reference;
import java.lang.ref.ReferenceQueue;
import java.util.Set;
import java.util.concurrent.ConcurrentHashMap;
import java.util.function.LongConsumer;

/**
 * Releases the native sg_window / sg_aggregator behind a per-partition or per-group State once Siddhi's
 * state holder has dropped it (canDestroy, @purge cleanGroupByStates, app shutdown): a phantom reference
 * per State, drained whenever a new handle is tracked (Java 8 has no java.lang.ref.Cleaner).
 */
final class NativeHandles {
    private static final ReferenceQueue<Object> QUEUE = new ReferenceQueue<>();
    private static final Set<Handle> LIVE = ConcurrentHashMap.newKeySet();

    private NativeHandles() {
    }

    private static final class Handle extends PhantomReference<Object> {
        final long ptr;
        final LongConsumer destroy;

        Handle(Object owner, long ptr, LongConsumer destroy) {
            super(owner, QUEUE);
            this.ptr = ptr;
            this.destroy = destroy;
        }
    }

    static void track(Object owner, long ptr, LongConsumer destroy) {
        drain();
        LIVE.add(new Handle(owner, ptr, destroy));
    }

    static void drain() {
        Reference<?> r;
        while ((r = QUEUE.poll()) != null) {
            Handle h = (Handle) r;
            if (LIVE.remove(h)) {
                h.destroy.accept(h.ptr);
            }
        }
    }
}
