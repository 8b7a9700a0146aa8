/* siddhi_gfx_ext_jni.c — JNI glue between io.siddhi.gpu.ext.NativeExt and the extension surface of
 * libsiddhi_gfx.so (include/siddhi_gfx_ext.h).  Built into libsiddhi_gfx_jni.so with siddhi_gfx_jni.c:
 *
 *   cc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *      java/jni/siddhi_gfx_jni.c java/jni/siddhi_gfx_ext_jni.c -Lsiddhi_amd/_build -lsiddhi_gfx \
 *      -o libsiddhi_gfx_jni.so
 *
 * Not compiled here (no JDK in this image); tests/test_ext_cpu.py drives the same sg_window_* / sg_agg_*
 * calls through ctypes. */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "siddhi_gfx.h"
#include "siddhi_gfx_ext.h"

static void throw_rt(JNIEnv* env) {
  jclass c = (*env)->FindClass(env, "io/siddhi/core/exception/SiddhiAppRuntimeException");
  if (c) (*env)->ThrowNew(env, c, sg_last_error());
}

static void throw_capacity(JNIEnv* env, const char* what) {
  jclass c = (*env)->FindClass(env, "io/siddhi/core/exception/SiddhiAppRuntimeException");
  if (c) (*env)->ThrowNew(env, c, what);
}

static void* addr(JNIEnv* env, jobject buf) { return buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL; }
static sg_window* W(jlong h) { return (sg_window*)(intptr_t)h; }
static sg_aggregator* A(jlong h) { return (sg_aggregator*)(intptr_t)h; }

/* ---- windows (WindowProcessor.init / processEventChunk / Scheduler TIMER / State.snapshot) ---- */

JNIEXPORT jlong JNICALL Java_io_siddhi_gpu_ext_NativeExt_windowCreate(JNIEnv* env, jclass k, jint kind, jlong param,
                                                                      jboolean sc, jboolean expiredOn) {
  (void)k;
  sg_window* w = NULL;
  if (sg_window_create(kind, param, sc, expiredOn, &w)) { throw_rt(env); return 0; }
  return (jlong)(intptr_t)w;
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_ext_NativeExt_windowDestroy(JNIEnv* env, jclass k, jlong w) {
  (void)env; (void)k;
  sg_window_destroy(W(w));
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_ext_NativeExt_windowProcess(JNIEnv* env, jclass k, jlong w, jint n,
                                                                      jobject ids, jobject ts, jlong now) {
  (void)k;
  if (sg_window_process(W(w), n, (const int64_t*)addr(env, ids), (const int64_t*)addr(env, ts), now)) throw_rt(env);
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_ext_NativeExt_windowOnTime(JNIEnv* env, jclass k, jlong w, jlong now) {
  (void)k;
  if (sg_window_on_time(W(w), now)) throw_rt(env);
}

JNIEXPORT jlong JNICALL Java_io_siddhi_gpu_ext_NativeExt_windowNextDeadline(JNIEnv* env, jclass k, jlong w) {
  (void)env; (void)k;
  return sg_window_next_deadline(W(w));
}

JNIEXPORT jlongArray JNICALL Java_io_siddhi_gpu_ext_NativeExt_windowTakeDeadlines(JNIEnv* env, jclass k, jlong w) {
  (void)k;
  const int64_t n = sg_window_take_deadlines(W(w), NULL, 0);
  if (n < 0) { throw_rt(env); return NULL; }
  int64_t* d = (int64_t*)malloc((size_t)(n > 0 ? n : 1) * 8);
  if (!d) return NULL;
  if (sg_window_take_deadlines(W(w), d, n) < 0) { free(d); throw_rt(env); return NULL; }
  jlongArray r = (*env)->NewLongArray(env, (jsize)n);
  if (r) (*env)->SetLongArrayRegion(env, r, 0, (jsize)n, (const jlong*)d);
  free(d);
  return r;
}

JNIEXPORT jlongArray JNICALL Java_io_siddhi_gpu_ext_NativeExt_windowOutSizes(JNIEnv* env, jclass k, jlong w) {
  (void)k;
  int64_t n = 0, c = 0;
  if (sg_window_out_sizes(W(w), &n, &c)) { throw_rt(env); return NULL; }
  jlongArray r = (*env)->NewLongArray(env, 2);
  jlong v[2] = {n, c};
  (*env)->SetLongArrayRegion(env, r, 0, 2, v);
  return r;
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_ext_NativeExt_windowOutCopy(JNIEnv* env, jclass k, jlong w, jobject ids,
                                                                      jobject types, jobject ts, jobject chunkEnd) {
  (void)k;
  if (sg_window_out_copy(W(w), (int64_t*)addr(env, ids), (int32_t*)addr(env, types), (int64_t*)addr(env, ts),
                         (int64_t*)addr(env, chunkEnd)))
    throw_rt(env);
}

JNIEXPORT jbyteArray JNICALL Java_io_siddhi_gpu_ext_NativeExt_windowSnapshot(JNIEnv* env, jclass k, jlong w) {
  (void)k;
  uint8_t* buf = NULL;
  int64_t len = 0;
  if (sg_window_snapshot(W(w), &buf, &len)) { throw_rt(env); return NULL; }
  if (len > INT32_MAX) { sg_free_buffer(buf); throw_capacity(env, "window snapshot exceeds a Java byte[]"); return NULL; }
  jbyteArray r = (*env)->NewByteArray(env, (jsize)len);
  (*env)->SetByteArrayRegion(env, r, 0, (jsize)len, (const jbyte*)buf);
  sg_free_buffer(buf);
  return r;
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_ext_NativeExt_windowRestore(JNIEnv* env, jclass k, jlong w, jbyteArray st) {
  (void)k;
  const jsize len = (*env)->GetArrayLength(env, st);
  jbyte* b = (*env)->GetByteArrayElements(env, st, NULL);
  const int rc = sg_window_restore(W(w), (const uint8_t*)b, len);
  (*env)->ReleaseByteArrayElements(env, st, b, JNI_ABORT);
  if (rc) throw_rt(env);
}

/* ---- aggregators (AttributeAggregatorExecutor.init / processAdd / processRemove / reset / canDestroy) ---- */

JNIEXPORT jlong JNICALL Java_io_siddhi_gpu_ext_NativeExt_aggCreate(JNIEnv* env, jclass k, jint kind, jint inType,
                                                                   jboolean track) {
  (void)k;
  sg_aggregator* a = NULL;
  if (sg_agg_create(kind, inType, track, &a)) { throw_rt(env); return 0; }
  return (jlong)(intptr_t)a;
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_ext_NativeExt_aggDestroy(JNIEnv* env, jclass k, jlong a) {
  (void)env; (void)k;
  sg_agg_destroy(A(a));
}

JNIEXPORT jint JNICALL Java_io_siddhi_gpu_ext_NativeExt_aggOutType(JNIEnv* env, jclass k, jlong a) {
  (void)env; (void)k;
  return sg_agg_out_type(A(a));
}

JNIEXPORT jlong JNICALL Java_io_siddhi_gpu_ext_NativeExt_aggProcess1(JNIEnv* env, jclass k, jlong a, jint type,
                                                                     jlong in, jboolean inNull, jbyteArray nullOut) {
  (void)k;
  const int32_t t = type;
  const int64_t v = in;
  const uint8_t nn = inNull ? 1 : 0;
  int64_t out = 0;
  uint8_t on = 0;
  if (sg_agg_process(A(a), 1, &t, &v, &nn, &out, &on)) { throw_rt(env); return 0; }
  const jbyte b = (jbyte)on;
  (*env)->SetByteArrayRegion(env, nullOut, 0, 1, &b);
  return out;
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_ext_NativeExt_aggProcess(JNIEnv* env, jclass k, jlong a, jint n, jobject types,
                                                                   jobject in, jobject inNull, jobject out,
                                                                   jobject outNull) {
  (void)k;
  if (sg_agg_process(A(a), n, (const int32_t*)addr(env, types), (const int64_t*)addr(env, in),
                     (const uint8_t*)addr(env, inNull), (int64_t*)addr(env, out), (uint8_t*)addr(env, outNull)))
    throw_rt(env);
}

JNIEXPORT jboolean JNICALL Java_io_siddhi_gpu_ext_NativeExt_aggCanDestroy(JNIEnv* env, jclass k, jlong a) {
  (void)env; (void)k;
  return sg_agg_can_destroy(A(a)) == 1 ? JNI_TRUE : JNI_FALSE;
}

JNIEXPORT jbyteArray JNICALL Java_io_siddhi_gpu_ext_NativeExt_aggSnapshot(JNIEnv* env, jclass k, jlong a) {
  (void)k;
  uint8_t* buf = NULL;
  int64_t len = 0;
  if (sg_agg_snapshot(A(a), &buf, &len)) { throw_rt(env); return NULL; }
  if (len > INT32_MAX) { sg_free_buffer(buf); throw_capacity(env, "aggregator snapshot exceeds a Java byte[]"); return NULL; }
  jbyteArray r = (*env)->NewByteArray(env, (jsize)len);
  if (r) (*env)->SetByteArrayRegion(env, r, 0, (jsize)len, (const jbyte*)buf);
  sg_free_buffer(buf);
  return r;
}

JNIEXPORT void JNICALL Java_io_siddhi_gpu_ext_NativeExt_aggRestore(JNIEnv* env, jclass k, jlong a, jbyteArray st) {
  (void)k;
  const jsize len = (*env)->GetArrayLength(env, st);
  jbyte* b = (*env)->GetByteArrayElements(env, st, NULL);
  const int rc = sg_agg_restore(A(a), (const uint8_t*)b, len);
  (*env)->ReleaseByteArrayElements(env, st, b, JNI_ABORT);
  if (rc) throw_rt(env);
}
