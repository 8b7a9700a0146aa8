package io.siddhi.gpu;

import java.nio.ByteBuffer;
import java.nio.IntBuffer;
import java.nio.LongBuffer;

/**
 * JNI entry points of libsiddhi_gfx_jni.so (java/jni/siddhi_gfx_jni.c), one per C-ABI function of
 * include/siddhi_gfx.h.  All buffers are direct; handles are the sg_app pointer.
 */
final class Native {
    static {
        System.loadLibrary("siddhi_gfx_jni");   // links libsiddhi_gfx.so
    }

    private Native() {
    }

    /** Path ids returned by queryPath (SG_PATH_*); UNSUPPORTED keeps the stock runtime. */
    static final int UNSUPPORTED = -2;
    static final int PATH_FOLLOWED_BY = 1;
    static final int PATH_NFA = 2;
    static final int PATH_WINDOW_AGG = 3;
    static final int PATH_KEYED_FOLLOWED_BY = 4;
    static final int PATH_WINDOW = 5;

    static native long create(String descriptorJson, int device, long capacity);

    static native void destroy(long h);

    static native void start(long h);

    static native void reset(long h);

    static native int queryIndex(long h, String query);

    static native int streamIndex(long h, String stream);

    static native int queryPath(long h, int query);

    static native String unsupportedReason(long h, int query);

    /** Events a device query still holds after its last flush (a gauge for long-running apps; -1: untracked). */
    static native long queryBuffered(long h, int query);

    static native int intern(long h, String s);

    static native String string(long h, int id);

    static native void addQueryCallback(long h, int query);

    static native void addStreamCallback(long h, int stream);

    static native void push(long h, int stream, long n, LongBuffer ts, ByteBuffer[] cols, ByteBuffer nulls,
                            boolean batch);

    static native void advanceTime(long h, long nowMillis);

    static native void flush(long h);

    static native long outNCallbacks(long h);

    static native long outNRows(long h);

    static native void drain(long h, IntBuffer kind, IntBuffer target, LongBuffer ts, IntBuffer nIn, IntBuffer nRm,
                             LongBuffer rowTs, LongBuffer raw, ByteBuffer nulls, int width);

    static native byte[] snapshot(long h);

    static native void restore(long h, byte[] state);
}
