/* siddhi_gfx_jni.c — JNI glue between io.siddhi.gpu.Native (java/src/main/java/io/siddhi/gpu/Native.java)
 * and the C ABI of libsiddhi_gfx.so (include/siddhi_gfx.h).
 *
 *   cc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *      java/jni/siddhi_gfx_jni.c -Lsiddhi_amd/_build -lsiddhi_gfx -o libsiddhi_gfx_jni.so
 *
 * No JDK is installed in the build image of this repository, so this file is not compiled here; every
 * sg_* call it makes is exercised through the same ABI by siddhi_amd/runtime.py (ctypes) in tests/.
 *
 * Buffers: input columns and output arrays are direct java.nio buffers (no copies through the JVM heap);
 * the caller sizes output buffers from outNCallbacks / outNRows.  Errors become Java exceptions:
 * SG_E_UNSUPPORTED -> io.siddhi.gpu.UnsupportedOnGpuException (the provider then keeps the stock
 * runtime for that query), anything else -> io.siddhi.core.exception.SiddhiAppRuntimeException. */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "siddhi_gfx.h"

#define SG_JNI_MAXCOLS 64

static void throw_sg(JNIEnv* env, int rc) {
  const char* cls = rc == SG_E_UNSUPPORTED ? "io/siddhi/gpu/UnsupportedOnGpuException"
                                           : "io/siddhi/core/exception/SiddhiAppRuntimeException";
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, sg_last_error());
}

static sg_app* H(jlong h) { return (sg_app*)(intptr_t)h; }

static void* addr(JNIEnv* env, jobject buf) { return buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL; }

/* ---- lifecycle (SiddhiManager.createSiddhiAppRuntime / SiddhiAppRuntime.start / shutdown) ---- */

JNIEXPORT jlong JNICALL Java_io_siddhi_gpu_Native_create(JNIEnv* env, jclass k, jstring desc, jint device,
                                                         jlong capacity) {
  (void)k;
  const char* d = (*env)->GetStringUTFChars(env, desc, NULL);
  sg_options o;
  o.device = device;
  o.capacity = capacity;
  sg_app* app = NULL;
  const int rc = sg_app_create(d, &o, &app);
  (*env)->ReleaseStringUTFChars(env, desc, d);
  if (rc) { throw_sg(env, rc); return 0; }
  return (jlong)(intptr_t)app;
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_Native_destroy(JNIEnv* env, jclass k, jlong h) {
  (void)env; (void)k;
  sg_app_destroy(H(h));
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_Native_start(JNIEnv* env, jclass k, jlong h) {
  (void)k;
  const int rc = sg_start(H(h));
  if (rc) throw_sg(env, rc);
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_Native_reset(JNIEnv* env, jclass k, jlong h) {
  (void)k;
  const int rc = sg_reset(H(h));
  if (rc) throw_sg(env, rc);
}

/* ---- names, paths, dictionary ---- */

static jint index_of(JNIEnv* env, jlong h, jstring name, int query) {
  const char* s = (*env)->GetStringUTFChars(env, name, NULL);
  const int i = query ? sg_query_index(H(h), s) : sg_stream_index(H(h), s);
  (*env)->ReleaseStringUTFChars(env, name, s);
  return i;
}

JNIEXPORT jint JNICALL Java_io_siddhi_gpu_Native_queryIndex(JNIEnv* env, jclass k, jlong h, jstring name) {
  (void)k;
  return index_of(env, h, name, 1);
}

JNIEXPORT jint JNICALL Java_io_siddhi_gpu_Native_streamIndex(JNIEnv* env, jclass k, jlong h, jstring name) {
  (void)k;
  return index_of(env, h, name, 0);
}

JNIEXPORT jint JNICALL Java_io_siddhi_gpu_Native_queryPath(JNIEnv* env, jclass k, jlong h, jint q) {
  (void)env; (void)k;
  return sg_query_path(H(h), q);
}

JNIEXPORT jlong JNICALL Java_io_siddhi_gpu_Native_queryBuffered(JNIEnv* env, jclass k, jlong h, jint q) {
  (void)env; (void)k;
  return (jlong)sg_query_buffered(H(h), q);
}

JNIEXPORT jstring JNICALL Java_io_siddhi_gpu_Native_unsupportedReason(JNIEnv* env, jclass k, jlong h, jint q) {
  (void)k;
  const char* r = sg_query_unsupported_reason(H(h), q);
  return (*env)->NewStringUTF(env, r ? r : "");
}

JNIEXPORT jint JNICALL Java_io_siddhi_gpu_Native_intern(JNIEnv* env, jclass k, jlong h, jstring s) {
  (void)k;
  const char* c = (*env)->GetStringUTFChars(env, s, NULL);
  const int id = sg_intern(H(h), c);
  (*env)->ReleaseStringUTFChars(env, s, c);
  return id;
}

JNIEXPORT jstring JNICALL Java_io_siddhi_gpu_Native_string(JNIEnv* env, jclass k, jlong h, jint id) {
  (void)k;
  const char* s = sg_string(H(h), id);
  return s ? (*env)->NewStringUTF(env, s) : NULL;
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_Native_addQueryCallback(JNIEnv* env, jclass k, jlong h, jint q) {
  (void)k;
  const int rc = sg_add_query_callback(H(h), q);
  if (rc) throw_sg(env, rc);
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_Native_addStreamCallback(JNIEnv* env, jclass k, jlong h, jint s) {
  (void)k;
  const int rc = sg_add_stream_callback(H(h), s);
  if (rc) throw_sg(env, rc);
}

/* ---- input (InputHandler.send / StreamJunction.Receiver.receive) ----
 * ts: direct LongBuffer of n timestamps; cols: one direct buffer per attribute in SG_T_* encoding;
 * nulls: optional direct ByteBuffer of n*arity flags (row-major); batch: one send(Event[]) chunk. */
JNIEXPORT void JNICALL Java_io_siddhi_gpu_Native_push(JNIEnv* env, jclass k, jlong h, jint stream, jlong n,
                                                      jobject ts, jobjectArray cols, jobject nulls, jboolean batch) {
  (void)k;
  const void* ptrs[SG_JNI_MAXCOLS];
  const jsize m = (*env)->GetArrayLength(env, cols);
  if (m > SG_JNI_MAXCOLS) { throw_sg(env, SG_E_INVALID); return; }
  for (jsize i = 0; i < m; i++) {
    jobject c = (*env)->GetObjectArrayElement(env, cols, i);
    ptrs[i] = addr(env, c);
    (*env)->DeleteLocalRef(env, c);
  }
  sg_batch b;
  b.n = n;
  b.ts = (const int64_t*)addr(env, ts);
  b.cols = ptrs;
  b.nulls = (const uint8_t*)addr(env, nulls);
  b.batch = batch ? 1 : 0;
  b.seq = NULL;
  const int rc = sg_push(H(h), stream, &b);
  if (rc) throw_sg(env, rc);
}

/* TimestampGenerator / Scheduler: the wall clock moved (non-playback apps) */
JNIEXPORT void JNICALL Java_io_siddhi_gpu_Native_advanceTime(JNIEnv* env, jclass k, jlong h, jlong now) {
  (void)k;
  const int rc = sg_advance_time(H(h), now);
  if (rc) throw_sg(env, rc);
}

/* ---- output (QueryCallback.receive / StreamCallback.receive, in sg_out_callbacks order) ---- */

JNIEXPORT void JNICALL Java_io_siddhi_gpu_Native_flush(JNIEnv* env, jclass k, jlong h) {
  (void)k;
  const int rc = sg_flush(H(h));
  if (rc) throw_sg(env, rc);
}

JNIEXPORT jlong JNICALL Java_io_siddhi_gpu_Native_outNCallbacks(JNIEnv* env, jclass k, jlong h) {
  (void)env; (void)k;
  return (jlong)sg_out_ncallbacks(H(h));
}

JNIEXPORT jlong JNICALL Java_io_siddhi_gpu_Native_outNRows(JNIEnv* env, jclass k, jlong h) {
  (void)env; (void)k;
  return (jlong)sg_out_nrows(H(h));
}

/* kind/target/nIn/nRm: IntBuffers, cts: LongBuffer (ncallbacks each); rts: LongBuffer (nrows);
 * raw: LongBuffer (nrows*width 8-byte slots); nulls: ByteBuffer (nrows*width).  Clears the queue. */
JNIEXPORT void JNICALL Java_io_siddhi_gpu_Native_drain(JNIEnv* env, jclass k, jlong h, jobject kind, jobject target,
                                                       jobject cts, jobject nin, jobject nrm, jobject rts,
                                                       jobject raw, jobject nulls, jint width) {
  (void)k;
  sg_app* a = H(h);
  int rc = sg_out_callbacks(a, (int32_t*)addr(env, kind), (int32_t*)addr(env, target), (int64_t*)addr(env, cts),
                            (int32_t*)addr(env, nin), (int32_t*)addr(env, nrm));
  if (!rc) rc = sg_out_rows(a, width, (int64_t*)addr(env, rts), (int64_t*)addr(env, raw), (uint8_t*)addr(env, nulls));
  if (!rc) rc = sg_out_clear(a);
  if (rc) throw_sg(env, rc);
}

/* ---- persistence (SiddhiAppRuntime.snapshot() / restore(byte[])) ---- */

JNIEXPORT jbyteArray JNICALL Java_io_siddhi_gpu_Native_snapshot(JNIEnv* env, jclass k, jlong h) {
  (void)k;
  uint8_t* buf = NULL;
  int64_t len = 0;
  const int rc = sg_snapshot(H(h), &buf, &len);
  if (rc) { throw_sg(env, rc); return NULL; }
  if (len > INT32_MAX) {
    /* an NFA snapshot carries its event store: past 2 GiB it does not fit one byte[] (SG_E_CAPACITY) */
    sg_free_buffer(buf);
    jclass c = (*env)->FindClass(env, "io/siddhi/core/exception/SiddhiAppRuntimeException");
    if (c) (*env)->ThrowNew(env, c, "snapshot larger than 2 GiB does not fit a Java byte[] (SG_E_CAPACITY)");
    return NULL;
  }
  jbyteArray out = (*env)->NewByteArray(env, (jsize)len);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, (jsize)len, (const jbyte*)buf);
  sg_free_buffer(buf);
  return out;
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_Native_restore(JNIEnv* env, jclass k, jlong h, jbyteArray state) {
  (void)k;
  const jsize len = (*env)->GetArrayLength(env, state);
  jbyte* p = (*env)->GetByteArrayElements(env, state, NULL);
  const int rc = sg_restore(H(h), (const uint8_t*)p, (int64_t)len);
  (*env)->ReleaseByteArrayElements(env, state, p, JNI_ABORT);
  if (rc) throw_sg(env, rc);
}
