/* jni/gpu_jni.c -- JNI shim for tech.bsdb.gpu.GpuBuild (jni/GpuBuild.java)
 * over the C ABI of include/bsdb_mi355x.h (libbsdb_mi355x.so).
 *
 * Mirrors the reference's JNI conventions (src/main/c/native.c:15-68): jlong
 * handles, GetByteArrayElements + Release(JNI_ABORT) (native.c:63-66),
 * negative codes turned into java.io.IOException.  Unlike native.c, every
 * handle has a free/close, strings are released on every path (native.c:54)
 * and the Java return types match the C ones (Native.java:156 vs native.c:61).
 *
 * Build (needs a JDK's jni.h; none exists in this image or on the GPU box):
 *   gcc -O3 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       jni/gpu_jni.c -Lbsdb_amd -lbsdb_mi355x -o libbsdbgpujni.so
 * tests/test_jni_shim.py checks every native against the header (arity and
 * called symbol) and compiles it against a minimal test-only jni.h.
 */
#include <jni.h>
#include <stdint.h>
#include "bsdb_mi355x.h"

#define P(x) ((void *)(intptr_t)(x))
static void fail(JNIEnv *env, int rc) {
    jclass ex = (*env)->FindClass(env, "java/io/IOException");
    (*env)->ThrowNew(env, ex, bsdb_strerror(rc));
}
#define CHECK(call) do { int rc_ = (call); if (rc_) fail(env, rc_); } while (0)
#define JF(name) JNICALL Java_tech_bsdb_gpu_GpuBuild_##name
/* Strings may be null where the C ABI allows it (index_a_path in exact mode,
 * index paths of the MPHF-only forms): every jstring goes through these. */
static const char *utf(JNIEnv *env, jstring s) { return s ? (*env)->GetStringUTFChars(env, s, NULL) : NULL; }
static void unutf(JNIEnv *env, jstring s, const char *p) { if (s) (*env)->ReleaseStringUTFChars(env, s, p); }

JNIEXPORT jlong JF(open)(JNIEnv *env, jclass c, jint dev) {
    bsdb_ctx *ctx = NULL; CHECK(bsdb_open(dev, &ctx)); return (jlong)(intptr_t)ctx;
}
JNIEXPORT void JF(close)(JNIEnv *env, jclass c, jlong ctx) { CHECK(bsdb_close(P(ctx))); }   /* freed, unlike native.c:50-59 */
JNIEXPORT jlong JF(numBuckets)(JNIEnv *env, jclass c, jlong n) { return (jlong)bsdb_num_buckets((uint64_t)n); }
JNIEXPORT jlong JF(valuesWords)(JNIEnv *env, jclass c, jlong n) { return (jlong)bsdb_values_words((uint64_t)n); }
JNIEXPORT void JF(releaseWorkspace)(JNIEnv *env, jclass c, jlong ctx) { CHECK(bsdb_release_workspace(P(ctx))); }
JNIEXPORT void JF(setVerify)(JNIEnv *env, jclass c, jlong ctx, jboolean on) { CHECK(bsdb_set_verify(P(ctx), on)); }

JNIEXPORT void JF(histogramFixed)(JNIEnv *env, jclass c, jlong ctx, jlong keys, jint L, jlong n, jlong seed, jlong m, jlong counts) {
    CHECK(bsdb_histogram_fixed(P(ctx), P(keys), (uint32_t)L, (uint64_t)n, (uint64_t)seed, (uint64_t)m, P(counts)));
}
JNIEXPORT void JF(histogramVar)(JNIEnv *env, jclass c, jlong ctx, jlong blob, jlong offs, jlong n, jlong seed, jlong m, jlong counts) {
    CHECK(bsdb_histogram_var(P(ctx), P(blob), P(offs), (uint64_t)n, (uint64_t)seed, (uint64_t)m, P(counts)));
}
JNIEXPORT void JF(hashFixed)(JNIEnv *env, jclass c, jlong ctx, jlong keys, jint L, jlong n, jlong seed, jlong sig) {
    CHECK(bsdb_hash_fixed(P(ctx), P(keys), (uint32_t)L, (uint64_t)n, (uint64_t)seed, P(sig)));
}
JNIEXPORT void JF(hashVar)(JNIEnv *env, jclass c, jlong ctx, jlong blob, jlong offs, jlong n, jlong seed, jlong sig) {
    CHECK(bsdb_hash_var(P(ctx), P(blob), P(offs), (uint64_t)n, (uint64_t)seed, P(sig)));
}

JNIEXPORT jbyteArray JF(commUniqueId)(JNIEnv *env, jclass c) {
    uint8_t id[BSDB_COMM_ID_BYTES]; int rc = bsdb_comm_unique_id(id);
    if (rc) { fail(env, rc); return NULL; }
    jbyteArray a = (*env)->NewByteArray(env, BSDB_COMM_ID_BYTES);
    (*env)->SetByteArrayRegion(env, a, 0, BSDB_COMM_ID_BYTES, (const jbyte *)id);
    return a;
}
JNIEXPORT void JF(commInit)(JNIEnv *env, jclass c, jlong ctx, jint nranks, jint rank, jbyteArray id) {
    jbyte *b = (*env)->GetByteArrayElements(env, id, NULL);
    int rc = bsdb_comm_init(P(ctx), nranks, rank, (const uint8_t *)b);
    (*env)->ReleaseByteArrayElements(env, id, b, JNI_ABORT);   /* as native.c:63-66 */
    if (rc) fail(env, rc);
}

JNIEXPORT jlong JF(multiOpen)(JNIEnv *env, jclass c, jintArray devs) {
    jsize k = (*env)->GetArrayLength(env, devs);
    jint *d = (*env)->GetIntArrayElements(env, devs, NULL);
    bsdb_multi *mc = NULL; int rc = bsdb_multi_open((int)k, (const int *)d, &mc);
    (*env)->ReleaseIntArrayElements(env, devs, d, JNI_ABORT);
    if (rc) { fail(env, rc); return 0; }
    return (jlong)(intptr_t)mc;
}
JNIEXPORT void JF(multiClose)(JNIEnv *env, jclass c, jlong mc) { CHECK(bsdb_multi_close(P(mc))); }
JNIEXPORT void JF(multiHistogramFixed)(JNIEnv *env, jclass c, jlong mc, jlong keys, jint L, jlong n, jlong seed, jlong E) {
    CHECK(bsdb_multi_histogram_fixed(P(mc), P(keys), (uint32_t)L, (uint64_t)n, (uint64_t)seed, P(E)));
}
JNIEXPORT void JF(multiHistogramVar)(JNIEnv *env, jclass c, jlong mc, jlong blob, jlong offs, jlong n, jlong seed, jlong E) {
    CHECK(bsdb_multi_histogram_var(P(mc), P(blob), P(offs), (uint64_t)n, (uint64_t)seed, P(E)));
}
JNIEXPORT void JF(multiMphBuildIndexVar)(JNIEnv *env, jclass c, jlong mc, jlong blob, jlong offs, jlong n, jint w,
                                         jlong addr, jlong v8, jlong vl, jboolean approx, jstring ip, jstring ap,
                                         jlong E, jlong values, jlong sig) {
    const char *i = utf(env, ip), *a = utf(env, ap);
    int rc = bsdb_multi_mph_build_index_var(P(mc), P(blob), P(offs), (uint64_t)n, (uint32_t)w, P(addr), P(v8), P(vl),
                                            approx, i, a, P(E), P(values), P(sig));
    unutf(env, ip, i); unutf(env, ap, a);
    if (rc) fail(env, rc);
}
JNIEXPORT void JF(multiMphBuildIndexFixed)(JNIEnv *env, jclass c, jlong mc, jlong keys, jint L, jlong n, jint w,
                                           jlong addr, jlong v8, jlong vl, jboolean approx, jstring ip, jstring ap,
                                           jlong E, jlong values, jlong sig) {
    const char *i = utf(env, ip), *a = utf(env, ap);
    int rc = bsdb_multi_mph_build_index_fixed(P(mc), P(keys), (uint32_t)L, (uint64_t)n, (uint32_t)w, P(addr), P(v8),
                                              P(vl), approx, i, a, P(E), P(values), P(sig));
    unutf(env, ip, i); unutf(env, ap, a);
    if (rc) fail(env, rc);
}

JNIEXPORT jlong JF(mphBuildFixed)(JNIEnv *env, jclass c, jlong ctx, jlong keys, jint L, jlong n, jint w) {
    bsdb_mph *m = NULL; CHECK(bsdb_mph_build_fixed(P(ctx), P(keys), (uint32_t)L, (uint64_t)n, (uint32_t)w, &m));
    return (jlong)(intptr_t)m;
}
JNIEXPORT jlong JF(mphBuildVar)(JNIEnv *env, jclass c, jlong ctx, jlong blob, jlong offs, jlong n, jint w) {
    bsdb_mph *m = NULL; CHECK(bsdb_mph_build_var(P(ctx), P(blob), P(offs), (uint64_t)n, (uint32_t)w, &m));
    return (jlong)(intptr_t)m;
}
JNIEXPORT jlong JF(mphBuildIndexVar)(JNIEnv *env, jclass c, jlong ctx, jlong blob, jlong offs, jlong n, jint w,
                                     jlong addr, jlong v8, jlong vl, jboolean approx, jstring ip, jstring ap) {
    const char *i = utf(env, ip), *a = utf(env, ap);
    bsdb_mph *m = NULL;
    int rc = bsdb_mph_build_index_var(P(ctx), P(blob), P(offs), (uint64_t)n, (uint32_t)w, P(addr), P(v8), P(vl),
                                      approx, i, a, &m);
    unutf(env, ip, i); unutf(env, ap, a);
    if (rc) { fail(env, rc); return 0; }
    return (jlong)(intptr_t)m;
}
JNIEXPORT jlong JF(mphBuildIndexFixed)(JNIEnv *env, jclass c, jlong ctx, jlong keys, jint L, jlong n, jint w,
                                       jlong addr, jlong v8, jlong vl, jboolean approx, jstring ip, jstring ap) {
    const char *i = utf(env, ip), *a = utf(env, ap);
    bsdb_mph *m = NULL;
    int rc = bsdb_mph_build_index_fixed(P(ctx), P(keys), (uint32_t)L, (uint64_t)n, (uint32_t)w, P(addr), P(v8), P(vl),
                                        approx, i, a, &m);
    unutf(env, ip, i); unutf(env, ap, a);
    if (rc) { fail(env, rc); return 0; }
    return (jlong)(intptr_t)m;
}
/* F2 in bounded device memory (README-size sets on one GPU); passesOut[0] = passes used */
JNIEXPORT jlong JF(mphBuildIndexPassesFixed)(JNIEnv *env, jclass c, jlong ctx, jlong keys, jint L, jlong n, jint w,
                                             jlong addr, jlong addrBase, jlong addrStride, jlong v8, jlong vl,
                                             jboolean approx, jint passes, jstring ip, jstring ap, jlongArray passesOut) {
    const char *i = utf(env, ip), *a = utf(env, ap);
    bsdb_mph *m = NULL; uint32_t used = 0;
    int rc = bsdb_mph_build_index_passes_fixed(P(ctx), P(keys), (uint32_t)L, (uint64_t)n, (uint32_t)w, P(addr),
                                               (uint64_t)addrBase, (uint64_t)addrStride, P(v8), P(vl), approx,
                                               (uint32_t)passes, i, a, &m, &used);
    unutf(env, ip, i); unutf(env, ap, a);
    if (rc) { fail(env, rc); return 0; }
    if (passesOut) { jlong u = (jlong)used; (*env)->SetLongArrayRegion(env, passesOut, 0, 1, &u); }
    return (jlong)(intptr_t)m;
}
JNIEXPORT jlong JF(mphBuildIndexPassesVar)(JNIEnv *env, jclass c, jlong ctx, jlong blob, jlong offs, jlong n, jint w,
                                           jlong addr, jlong addrBase, jlong addrStride, jlong v8, jlong vl,
                                           jboolean approx, jint passes, jstring ip, jstring ap, jlongArray passesOut) {
    const char *i = utf(env, ip), *a = utf(env, ap);
    bsdb_mph *m = NULL; uint32_t used = 0;
    int rc = bsdb_mph_build_index_passes_var(P(ctx), P(blob), P(offs), (uint64_t)n, (uint32_t)w, P(addr),
                                             (uint64_t)addrBase, (uint64_t)addrStride, P(v8), P(vl), approx,
                                             (uint32_t)passes, i, a, &m, &used);
    unutf(env, ip, i); unutf(env, ap, a);
    if (rc) { fail(env, rc); return 0; }
    if (passesOut) { jlong u = (jlong)used; (*env)->SetLongArrayRegion(env, passesOut, 0, 1, &u); }
    return (jlong)(intptr_t)m;
}
/* the streaming builder: put() batches straight into HBM, then one build */
JNIEXPORT jlong JF(builderOpen)(JNIEnv *env, jclass c, jlong ctx, jint L, jlong keyCap, jlong blobCap, jboolean approx,
                                jlong addrBase, jlong addrStride) {
    bsdb_builder *b = NULL;
    CHECK(bsdb_builder_open(P(ctx), (uint32_t)L, (uint64_t)keyCap, (uint64_t)blobCap, approx, (uint64_t)addrBase,
                            (uint64_t)addrStride, &b));
    return (jlong)(intptr_t)b;
}
JNIEXPORT void JF(builderAddFixed)(JNIEnv *env, jclass c, jlong b, jlong keys, jint L, jlong cnt, jlong addr, jlong v8,
                                   jlong vl) {
    CHECK(bsdb_builder_add_fixed(P(b), P(keys), (uint32_t)L, (uint64_t)cnt, P(addr), P(v8), P(vl)));
}
JNIEXPORT void JF(builderAddVar)(JNIEnv *env, jclass c, jlong b, jlong blob, jlong offs, jlong cnt, jlong addr, jlong v8,
                                 jlong vl) {
    CHECK(bsdb_builder_add_var(P(b), P(blob), P(offs), (uint64_t)cnt, P(addr), P(v8), P(vl)));
}
JNIEXPORT jlong JF(builderCount)(JNIEnv *env, jclass c, jlong b) {
    uint64_t n = 0; CHECK(bsdb_builder_count(P(b), &n)); return (jlong)n;
}
JNIEXPORT jlong JF(builderFinish)(JNIEnv *env, jclass c, jlong b, jint w, jint passes, jstring ip, jstring ap) {
    const char *i = utf(env, ip), *a = utf(env, ap);
    bsdb_mph *m = NULL;
    int rc = bsdb_builder_finish(P(b), (uint32_t)w, (uint32_t)passes, i, a, &m, NULL);
    unutf(env, ip, i); unutf(env, ap, a);
    if (rc) { fail(env, rc); return 0; }
    return (jlong)(intptr_t)m;
}
JNIEXPORT void JF(builderFree)(JNIEnv *env, jclass c, jlong b) { CHECK(bsdb_builder_free(P(b))); }
JNIEXPORT jlongArray JF(mphInfo)(JNIEnv *env, jclass c, jlong mph) {
    uint64_t n, m, vw, sw; uint32_t w;
    int rc = bsdb_mph_info(P(mph), &n, &m, &w, &vw, &sw);
    if (rc) { fail(env, rc); return NULL; }
    jlong v[5] = {(jlong)n, (jlong)m, (jlong)w, (jlong)vw, (jlong)sw};
    jlongArray a = (*env)->NewLongArray(env, 5);
    if (!a) return NULL;  /* OutOfMemoryError pending */
    (*env)->SetLongArrayRegion(env, a, 0, 5, v);
    return a;
}
JNIEXPORT void JF(mphExport)(JNIEnv *env, jclass c, jlong mph, jlong E, jlong values, jlong sig) {
    CHECK(bsdb_mph_export(P(mph), P(E), P(values), P(sig)));
}
/* {numBuckets, valuesWords, valueBits, sigWords} of an MPHF on n keys (no handle) */
JNIEXPORT jlongArray JF(mphSizes)(JNIEnv *env, jclass c, jlong n, jint w) {
    uint64_t m, vw, vb, sw;
    int rc = bsdb_mph_sizes((uint64_t)n, (uint32_t)w, &m, &vw, &vb, &sw);
    if (rc) { fail(env, rc); return NULL; }
    jlong v[4] = {(jlong)m, (jlong)vw, (jlong)vb, (jlong)sw};
    jlongArray a = (*env)->NewLongArray(env, 4);
    if (!a) return NULL;  /* OutOfMemoryError pending */
    (*env)->SetLongArrayRegion(env, a, 0, 4, v);
    return a;
}
/* the export straight into Java long[] arrays (GovAssembler): each array is
 * held for the copy (GetPrimitiveArrayCritical: no second copy of a multi-GB
 * array) and released with mode 0 (written back); sig may be null (width 0);
 * every array must hold the mphInfo sizes (checked) */
JNIEXPORT void JF(mphExportArrays)(JNIEnv *env, jclass c, jlong mph, jlongArray E, jlongArray values, jlongArray sig) {
    uint64_t n, m, vw, sw; uint32_t w;
    int rc = bsdb_mph_info(P(mph), &n, &m, &w, &vw, &sw);
    if (!rc && (!E || !values || (w && !sig) || (uint64_t)(*env)->GetArrayLength(env, E) < m + 1 ||
                (uint64_t)(*env)->GetArrayLength(env, values) < vw ||
                (w && (uint64_t)(*env)->GetArrayLength(env, sig) < sw)))
        rc = BSDB_EINVAL;
    if (rc) { fail(env, rc); return; }
    void *pe = (*env)->GetPrimitiveArrayCritical(env, E, NULL);
    void *pv = (*env)->GetPrimitiveArrayCritical(env, values, NULL);
    void *ps = w ? (*env)->GetPrimitiveArrayCritical(env, sig, NULL) : NULL;
    rc = (!pe || !pv || (w && !ps)) ? BSDB_ENOMEM : bsdb_mph_export(P(mph), pe, pv, ps);
    if (ps) (*env)->ReleasePrimitiveArrayCritical(env, sig, ps, 0);
    if (pv) (*env)->ReleasePrimitiveArrayCritical(env, values, pv, 0);
    if (pe) (*env)->ReleasePrimitiveArrayCritical(env, E, pe, 0);
    if (rc) fail(env, rc);
}
JNIEXPORT jlong JF(mphImport)(JNIEnv *env, jclass c, jlong ctx, jlong n, jint w, jlong E, jlong values, jlong sig) {
    bsdb_mph *m = NULL; CHECK(bsdb_mph_import(P(ctx), (uint64_t)n, (uint32_t)w, P(E), P(values), P(sig), &m));
    return (jlong)(intptr_t)m;
}
JNIEXPORT void JF(mphDump)(JNIEnv *env, jclass c, jlong mph, jstring path) {
    const char *p = utf(env, path);
    int rc = bsdb_mph_dump(P(mph), p);                          /* (null path: BSDB_EINVAL) */
    unutf(env, path, p);                                        /* released on every path, unlike native.c:54 */
    if (rc) fail(env, rc);
}
JNIEXPORT jlong JF(mphLoad)(JNIEnv *env, jclass c, jlong ctx, jstring path) {
    const char *p = utf(env, path);
    bsdb_mph *m = NULL; int rc = bsdb_mph_load(P(ctx), p, &m);
    unutf(env, path, p);
    if (rc) { fail(env, rc); return 0; }
    return (jlong)(intptr_t)m;
}
JNIEXPORT void JF(mphLookupFixed)(JNIEnv *env, jclass c, jlong mph, jlong keys, jint L, jlong n, jboolean chk, jlong out) {
    CHECK(bsdb_mph_lookup_fixed(P(mph), P(keys), (uint32_t)L, (uint64_t)n, chk, P(out)));
}
JNIEXPORT void JF(mphLookupVar)(JNIEnv *env, jclass c, jlong mph, jlong blob, jlong offs, jlong n, jboolean chk, jlong out) {
    CHECK(bsdb_mph_lookup_var(P(mph), P(blob), P(offs), (uint64_t)n, chk, P(out)));
}
JNIEXPORT void JF(mphFree)(JNIEnv *env, jclass c, jlong mph) { CHECK(bsdb_mph_free(P(mph))); }

JNIEXPORT jlong JF(indexOpen)(JNIEnv *env, jclass c, jlong mph, jboolean approx, jlong ps, jstring ip, jstring ap,
                              jlongArray passesOut) {
    const char *i = utf(env, ip), *a = utf(env, ap);
    bsdb_index *ix = NULL; uint64_t passes = 0;
    int rc = bsdb_index_open(P(mph), approx, (uint64_t)ps, i, a, &ix, &passes);
    unutf(env, ip, i); unutf(env, ap, a);
    if (rc) { fail(env, rc); return 0; }
    jlong p = (jlong)passes; (*env)->SetLongArrayRegion(env, passesOut, 0, 1, &p);
    return (jlong)(intptr_t)ix;
}
JNIEXPORT void JF(indexBeginPass)(JNIEnv *env, jclass c, jlong ix, jlong pass) { CHECK(bsdb_index_begin_pass(P(ix), (uint64_t)pass)); }
JNIEXPORT void JF(indexPutVar)(JNIEnv *env, jclass c, jlong ix, jlong blob, jlong offs, jlong cnt, jlong addr, jlong v8, jlong vl) {
    CHECK(bsdb_index_put_var(P(ix), P(blob), P(offs), (uint64_t)cnt, P(addr), P(v8), P(vl)));
}
JNIEXPORT void JF(indexPutFixed)(JNIEnv *env, jclass c, jlong ix, jlong keys, jint L, jlong cnt, jlong addr, jlong v8, jlong vl) {
    CHECK(bsdb_index_put_fixed(P(ix), P(keys), (uint32_t)L, (uint64_t)cnt, P(addr), P(v8), P(vl)));
}
JNIEXPORT void JF(indexEndPass)(JNIEnv *env, jclass c, jlong ix) { CHECK(bsdb_index_end_pass(P(ix))); }
JNIEXPORT void JF(indexClose)(JNIEnv *env, jclass c, jlong ix) { CHECK(bsdb_index_close(P(ix))); }
JNIEXPORT jlong JF(kvBuildIndex)(JNIEnv *env, jclass c, jlong ctx, jstring kv, jint parts, jint fmt, jint bs,
                                 jint threads, jint w, jboolean approx, jstring ip, jstring ap) {
    const char *k = utf(env, kv), *i = utf(env, ip), *a = utf(env, ap);
    bsdb_mph *m = NULL;
    int rc = bsdb_kv_build_index(P(ctx), k, parts, fmt, (uint32_t)bs, threads, (uint32_t)w, approx, i, a, &m);
    unutf(env, kv, k); unutf(env, ip, i); unutf(env, ap, a);
    if (rc) { fail(env, rc); return 0; }
    return (jlong)(intptr_t)m;
}
