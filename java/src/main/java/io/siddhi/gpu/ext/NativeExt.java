package io.siddhi.gpu.ext;

import java.nio.ByteBuffer;
import java.nio.IntBuffer;
import java.nio.LongBuffer;

/**
 * JNI entry points of the extension surface (java/jni/siddhi_gfx_ext_jni.c -> include/siddhi_gfx_ext.h).
 * Handles are the sg_window / sg_aggregator pointers; buffers are direct.
 */
final class NativeExt {
    static {
        System.loadLibrary("siddhi_gfx_jni");
    }

    private NativeExt() {
    }

    static final int WIN_LENGTH = 1;
    static final int WIN_TIME = 2;
    static final int WIN_LENGTH_BATCH = 3;
    static final int EV_CURRENT = 0;
    static final int EV_EXPIRED = 1;
    static final int EV_RESET = 3;
    static final int AGG_SUM = 0;
    static final int AGG_AVG = 1;
    static final int AGG_COUNT = 2;
    static final int AGG_MIN = 3;
    static final int AGG_MAX = 4;

    static native long windowCreate(int kind, long param, boolean streamCurrent, boolean expiredOn);

    static native void windowDestroy(long w);

    static native void windowProcess(long w, int n, LongBuffer ids, LongBuffer ts, long now);

    static native void windowOnTime(long w, long now);

    static native long windowNextDeadline(long w);

    /** The Scheduler.notifyAt deadlines queued since the last call (one per new timestamp), taken. */
    static native long[] windowTakeDeadlines(long w);

    /** [items, chunks] queued by the last process / onTime calls. */
    static native long[] windowOutSizes(long w);

    static native void windowOutCopy(long w, LongBuffer ids, IntBuffer types, LongBuffer ts, LongBuffer chunkEnd);

    static native byte[] windowSnapshot(long w);

    static native void windowRestore(long w, byte[] state);

    static native long aggCreate(int kind, int inType, boolean track);

    static native void aggDestroy(long a);

    static native int aggOutType(long a);

    /** One event: returns the aggregate as an 8-byte slot; nullOut[0] = 1 for null. */
    static native long aggProcess1(long a, int type, long in, boolean inNull, byte[] nullOut);

    static native void aggProcess(long a, int n, IntBuffer types, LongBuffer in, ByteBuffer inNull, LongBuffer out,
                                  ByteBuffer outNull);

    static native boolean aggCanDestroy(long a);

    static native byte[] aggSnapshot(long a);

    static native void aggRestore(long a, byte[] state);
}
