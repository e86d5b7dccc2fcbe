/*
 * redisson_sketch_jni.c -- JNI shim: org.redisson.gpu.SketchNative -> C ABI.
 * Built only where a JDK's jni.h exists (make -C jni JAVA_HOME=...); the
 * GPU build image has none.  Arrays are pinned with GetPrimitiveArrayCritical
 * for the duration of one C-ABI call (the library copies into its own
 * staging, include/redisson_sketch.h "Ownership").
 */
#include <jni.h>
#include <stdint.h>
#include <string.h>

#include "../include/redisson_sketch.h"

#define CTX(h) ((sk_ctx *)(intptr_t)(h))
#define PIN(arr) ((arr) ? (*env)->GetPrimitiveArrayCritical(env, (arr), NULL) : NULL)
#define UNPIN(arr, p, mode) \
    do { if (arr) (*env)->ReleasePrimitiveArrayCritical(env, (arr), (p), (mode)); } while (0)
#define LEN(arr) ((arr) ? (*env)->GetArrayLength(env, (arr)) : 0)

JNIEXPORT jlong JNICALL Java_org_redisson_gpu_SketchNative_open(JNIEnv *env, jclass cls, jint device, jint major,
                                                                jlong maxBit, jlong hllCap, jlong maxBatch) {
    (void)env; (void)cls;
    sk_config cfg = {device, major, (uint64_t)maxBit, (uint64_t)hllCap, (uint64_t)maxBatch};
    sk_ctx *c = NULL;
    return sk_open(&cfg, &c) == SK_OK ? (jlong)(intptr_t)c : 0;
}

JNIEXPORT void JNICALL Java_org_redisson_gpu_SketchNative_close(JNIEnv *env, jclass cls, jlong ctx) {
    (void)env; (void)cls;
    sk_close(CTX(ctx));
}

JNIEXPORT jstring JNICALL Java_org_redisson_gpu_SketchNative_lastError(JNIEnv *env, jclass cls, jlong ctx) {
    (void)cls;
    return (*env)->NewStringUTF(env, sk_last_error(CTX(ctx)));
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_calcSlot(JNIEnv *env, jclass cls, jbyteArray key) {
    (void)cls;
    jsize n = LEN(key);
    void *k = PIN(key);
    jint r = sk_calc_slot((const uint8_t *)k, (uint64_t)n);
    UNPIN(key, k, JNI_ABORT);
    return r;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_del(JNIEnv *env, jclass cls, jlong ctx, jlongArray off,
                                                              jbyteArray keys, jlongArray out) {
    (void)cls;
    jsize n = LEN(off) - 1;
    void *o = PIN(off), *k = PIN(keys), *r = PIN(out);
    jint st = sk_del(CTX(ctx), (uint32_t)n, (const uint64_t *)o, (const uint8_t *)k, (uint64_t *)r);
    UNPIN(out, r, 0); UNPIN(keys, k, JNI_ABORT); UNPIN(off, o, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_pfadd(JNIEnv *env, jclass cls, jlong ctx, jlongArray koff,
                                                                jbyteArray keys, jintArray counts, jlongArray eoff,
                                                                jbyteArray elems, jbyteArray out) {
    (void)cls;
    jsize n = LEN(counts);
    void *ko = PIN(koff), *k = PIN(keys), *c = PIN(counts), *eo = PIN(eoff), *e = PIN(elems), *r = PIN(out);
    jint st = sk_pfadd(CTX(ctx), (uint32_t)n, (const uint64_t *)ko, (const uint8_t *)k, (const uint32_t *)c,
                       (const uint64_t *)eo, (const uint8_t *)e, (uint8_t *)r);
    UNPIN(out, r, 0); UNPIN(elems, e, JNI_ABORT); UNPIN(eoff, eo, JNI_ABORT);
    UNPIN(counts, c, JNI_ABORT); UNPIN(keys, k, JNI_ABORT); UNPIN(koff, ko, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_hllResolve(JNIEnv *env, jclass cls, jlong ctx,
                                                                     jlongArray koff, jbyteArray keys,
                                                                     jintArray out_ids, jbyteArray out_created) {
    (void)cls;
    jsize n = LEN(out_ids);
    void *ko = PIN(koff), *k = PIN(keys), *i = PIN(out_ids), *cr = PIN(out_created);
    jint st = sk_hll_resolve(CTX(ctx), (uint32_t)n, (const uint64_t *)ko, (const uint8_t *)k, (uint32_t *)i,
                             (uint8_t *)cr);
    UNPIN(out_created, cr, 0); UNPIN(out_ids, i, 0); UNPIN(keys, k, JNI_ABORT); UNPIN(koff, ko, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_hllLookup(JNIEnv *env, jclass cls, jlong ctx,
                                                                    jlongArray koff, jbyteArray keys,
                                                                    jintArray out_ids) {
    (void)cls;
    jsize n = LEN(out_ids);
    void *ko = PIN(koff), *k = PIN(keys), *i = PIN(out_ids);
    jint st = sk_hll_lookup(CTX(ctx), (uint32_t)n, (const uint64_t *)ko, (const uint8_t *)k, (uint32_t *)i);
    UNPIN(out_ids, i, 0); UNPIN(keys, k, JNI_ABORT); UNPIN(koff, ko, JNI_ABORT);
    return st;
}

/* sk_type_many: the group-commit coalescer types every key it holds no cached slab id for in one call */
JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_typeMany(JNIEnv *env, jclass cls, jlong ctx, jlongArray koff,
                                                                   jbyteArray keys, jintArray out) {
    (void)cls;
    jsize n = LEN(out);
    void *ko = PIN(koff), *k = PIN(keys), *r = PIN(out);
    jint st = sk_type_many(CTX(ctx), (uint32_t)n, (const uint64_t *)ko, (const uint8_t *)k, (int32_t *)r);
    UNPIN(out, r, 0); UNPIN(keys, k, JNI_ABORT); UNPIN(koff, ko, JNI_ABORT);
    return st;
}

/* sk_pfadd_ids: keys resolved once per tenant (SketchNative.hllResolve) and cached on the Java side */
JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_pfaddIds(JNIEnv *env, jclass cls, jlong ctx, jintArray ids,
                                                                   jintArray counts, jlongArray eoff,
                                                                   jbyteArray elems, jbyteArray out) {
    (void)cls;
    jsize n = LEN(counts);
    void *i = PIN(ids), *c = PIN(counts), *eo = PIN(eoff), *e = PIN(elems), *r = PIN(out);
    jint st = sk_pfadd_ids(CTX(ctx), (uint32_t)n, (const uint32_t *)i, (const uint32_t *)c, (const uint64_t *)eo,
                           (const uint8_t *)e, (uint8_t *)r);
    UNPIN(out, r, 0); UNPIN(elems, e, JNI_ABORT); UNPIN(eoff, eo, JNI_ABORT);
    UNPIN(counts, c, JNI_ABORT); UNPIN(ids, i, JNI_ABORT);
    return st;
}

/* group commit in prefix form: elements = prefix + suffixes (sk_pfadd_ids_prefix) */
JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_pfaddIdsPrefix(JNIEnv *env, jclass cls, jlong ctx,
                                                                         jintArray ids, jbyteArray prefix,
                                                                         jintArray soff, jbyteArray sbytes,
                                                                         jbyteArray out) {
    (void)cls;
    jsize n = LEN(ids), pl = LEN(prefix);
    void *i = PIN(ids), *p = PIN(prefix), *so = PIN(soff), *sb = PIN(sbytes), *r = PIN(out);
    jint st = sk_pfadd_ids_prefix(CTX(ctx), (uint32_t)n, (const uint32_t *)i, (const uint8_t *)p, (uint32_t)pl,
                                  (const uint32_t *)so, (const uint8_t *)sb, (uint8_t *)r);
    UNPIN(out, r, 0); UNPIN(sbytes, sb, JNI_ABORT); UNPIN(soff, so, JNI_ABORT);
    UNPIN(prefix, p, JNI_ABORT); UNPIN(ids, i, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_pfcountIds(JNIEnv *env, jclass cls, jlong ctx,
                                                                     jintArray ids, jlongArray out) {
    (void)cls;
    jsize n = LEN(ids);
    void *i = PIN(ids), *r = PIN(out);
    jint st = sk_pfcount_ids(CTX(ctx), (uint64_t)n, (const uint32_t *)i, (int64_t *)r);
    UNPIN(out, r, 0); UNPIN(ids, i, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_pfcount(JNIEnv *env, jclass cls, jlong ctx, jintArray nk,
                                                                  jlongArray koff, jbyteArray keys, jlongArray out) {
    (void)cls;
    jsize n = LEN(nk);
    void *a = PIN(nk), *ko = PIN(koff), *k = PIN(keys), *r = PIN(out);
    jint st = sk_pfcount(CTX(ctx), (uint32_t)n, (const uint32_t *)a, (const uint64_t *)ko, (const uint8_t *)k,
                         (int64_t *)r);
    UNPIN(out, r, 0); UNPIN(keys, k, JNI_ABORT); UNPIN(koff, ko, JNI_ABORT); UNPIN(nk, a, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_pfmerge(JNIEnv *env, jclass cls, jlong ctx, jbyteArray dest,
                                                                  jlongArray soff, jbyteArray srcs) {
    (void)cls;
    jsize dn = LEN(dest), n = LEN(soff) - 1;
    void *d = PIN(dest), *so = PIN(soff), *s = PIN(srcs);
    jint st = sk_pfmerge(CTX(ctx), (const uint8_t *)d, (uint64_t)dn, (uint32_t)n, (const uint64_t *)so,
                         (const uint8_t *)s);
    UNPIN(srcs, s, JNI_ABORT); UNPIN(soff, so, JNI_ABORT); UNPIN(dest, d, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_setbit(JNIEnv *env, jclass cls, jlong ctx, jlongArray koff,
                                                                 jbyteArray keys, jlongArray offs, jbyteArray vals,
                                                                 jbyteArray out) {
    (void)cls;
    jsize n = LEN(offs);
    void *ko = PIN(koff), *k = PIN(keys), *o = PIN(offs), *v = PIN(vals), *r = PIN(out);
    jint st = sk_setbit(CTX(ctx), (uint32_t)n, (const uint64_t *)ko, (const uint8_t *)k, (const uint64_t *)o,
                        (const uint8_t *)v, (uint8_t *)r);
    UNPIN(out, r, 0); UNPIN(vals, v, JNI_ABORT); UNPIN(offs, o, JNI_ABORT);
    UNPIN(keys, k, JNI_ABORT); UNPIN(koff, ko, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_getbit(JNIEnv *env, jclass cls, jlong ctx, jlongArray koff,
                                                                 jbyteArray keys, jlongArray offs, jbyteArray out) {
    (void)cls;
    jsize n = LEN(offs);
    void *ko = PIN(koff), *k = PIN(keys), *o = PIN(offs), *r = PIN(out);
    jint st = sk_getbit(CTX(ctx), (uint32_t)n, (const uint64_t *)ko, (const uint8_t *)k, (const uint64_t *)o,
                        (uint8_t *)r);
    UNPIN(out, r, 0); UNPIN(offs, o, JNI_ABORT); UNPIN(keys, k, JNI_ABORT); UNPIN(koff, ko, JNI_ABORT);
    return st;
}

#define KEY_U64_OUT(name, fn)                                                                                 \
    JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_##name(JNIEnv *env, jclass cls, jlong ctx,      \
                                                                     jbyteArray key, jlongArray out) {        \
        (void)cls;                                                                                            \
        jsize n = LEN(key);                                                                                   \
        void *k = PIN(key), *r = PIN(out);                                                                    \
        jint st = fn(CTX(ctx), (const uint8_t *)k, (uint64_t)n, r);                                           \
        UNPIN(out, r, 0); UNPIN(key, k, JNI_ABORT);                                                           \
        return st;                                                                                            \
    }
KEY_U64_OUT(bitcount, sk_bitcount)
KEY_U64_OUT(strlen, sk_strlen)
KEY_U64_OUT(bitsetLength, sk_bitset_length)

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_bitop(JNIEnv *env, jclass cls, jlong ctx, jint op,
                                                                jbyteArray dest, jlongArray soff, jbyteArray srcs,
                                                                jlongArray out) {
    (void)cls;
    jsize dn = LEN(dest), n = LEN(soff) - 1;
    void *d = PIN(dest), *so = PIN(soff), *s = PIN(srcs), *r = PIN(out);
    jint st = sk_bitop(CTX(ctx), op, (const uint8_t *)d, (uint64_t)dn, (uint32_t)n, (const uint64_t *)so,
                       (const uint8_t *)s, (uint64_t *)r);
    UNPIN(out, r, 0); UNPIN(srcs, s, JNI_ABORT); UNPIN(soff, so, JNI_ABORT); UNPIN(dest, d, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_type(JNIEnv *env, jclass cls, jlong ctx, jbyteArray key,
                                                               jintArray out) {
    (void)cls;
    jsize n = LEN(key);
    void *k = PIN(key), *r = PIN(out);
    jint st = sk_type(CTX(ctx), (const uint8_t *)k, (uint64_t)n, (int *)r);
    UNPIN(out, r, 0); UNPIN(key, k, JNI_ABORT);
    return st;
}

JNIEXPORT jbyteArray JNICALL Java_org_redisson_gpu_SketchNative_get(JNIEnv *env, jclass cls, jlong ctx,
                                                                   jbyteArray key) {
    (void)cls;
    jsize n = LEN(key);
    jbyte *k = (*env)->GetByteArrayElements(env, key, NULL);
    int64_t len = -1;
    jbyteArray res = NULL;
    if (sk_get(CTX(ctx), (const uint8_t *)k, (uint64_t)n, NULL, 0, &len) == SK_OK && len >= 0) {
        res = (*env)->NewByteArray(env, (jsize)len);
        jbyte *b = (*env)->GetByteArrayElements(env, res, NULL);
        sk_get(CTX(ctx), (const uint8_t *)k, (uint64_t)n, (uint8_t *)b, (uint64_t)len, &len);
        (*env)->ReleaseByteArrayElements(env, res, b, 0);
    }
    (*env)->ReleaseByteArrayElements(env, key, k, JNI_ABORT);
    return res;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_set(JNIEnv *env, jclass cls, jlong ctx, jbyteArray key,
                                                              jbyteArray val) {
    (void)cls;
    jsize n = LEN(key), vn = LEN(val);
    void *k = PIN(key), *v = PIN(val);
    jint st = sk_set(CTX(ctx), (const uint8_t *)k, (uint64_t)n, (const uint8_t *)v, (uint64_t)vn);
    UNPIN(val, v, JNI_ABORT); UNPIN(key, k, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_bloomTryInit(JNIEnv *env, jclass cls, jlong ctx,
                                                                       jbyteArray name, jlong expected, jdouble fpp,
                                                                       jintArray ok) {
    (void)cls;
    jsize n = LEN(name);
    void *nm = PIN(name), *r = PIN(ok);
    jint st = sk_bloom_try_init(CTX(ctx), (const uint8_t *)nm, (uint64_t)n, expected, fpp, (int *)r);
    UNPIN(ok, r, 0); UNPIN(name, nm, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_bloomConfig(JNIEnv *env, jclass cls, jlong ctx,
                                                                      jbyteArray name, jlongArray sizeExp,
                                                                      jintArray k, jdoubleArray fpp) {
    (void)cls;
    jsize n = LEN(name);
    void *nm = PIN(name), *se = PIN(sizeExp), *kk = PIN(k), *f = PIN(fpp);
    int64_t *sev = (int64_t *)se;
    jint st = sk_bloom_config(CTX(ctx), (const uint8_t *)nm, (uint64_t)n, sev, (int32_t *)kk, sev + 1,
                              (double *)f);
    UNPIN(fpp, f, 0); UNPIN(k, kk, 0); UNPIN(sizeExp, se, 0); UNPIN(name, nm, JNI_ABORT);
    return st;
}

#define BLOOM_OP(name, fn)                                                                                   \
    JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_##name(                                        \
        JNIEnv *env, jclass cls, jlong ctx, jbyteArray nmArr, jlong size, jint k, jlongArray eoff,           \
        jbyteArray elems, jbyteArray out) {                                                                  \
        (void)cls;                                                                                           \
        jsize nn = LEN(nmArr), n = LEN(eoff) - 1;                                                            \
        void *nm = PIN(nmArr), *eo = PIN(eoff), *e = PIN(elems), *r = PIN(out);                              \
        jint st = fn(CTX(ctx), (const uint8_t *)nm, (uint64_t)nn, size, k, (uint32_t)n, (const uint64_t *)eo,\
                     (const uint8_t *)e, (uint8_t *)r);                                                      \
        UNPIN(out, r, 0); UNPIN(elems, e, JNI_ABORT); UNPIN(eoff, eo, JNI_ABORT); UNPIN(nmArr, nm, JNI_ABORT);\
        return st;                                                                                           \
    }
BLOOM_OP(bloomAdd, sk_bloom_add)
BLOOM_OP(bloomContains, sk_bloom_contains)

#define BLOOM_PREFIX_OP(name, fn)                                                                            \
    JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_##name(                                        \
        JNIEnv *env, jclass cls, jlong ctx, jbyteArray nmArr, jlong size, jint k, jbyteArray prefix,         \
        jintArray soff, jbyteArray sbytes, jbyteArray out) {                                                 \
        (void)cls;                                                                                           \
        jsize nn = LEN(nmArr), n = LEN(soff) - 1, pl = LEN(prefix);                                          \
        void *nm = PIN(nmArr), *p = PIN(prefix), *so = PIN(soff), *sb = PIN(sbytes), *r = PIN(out);          \
        jint st = fn(CTX(ctx), (const uint8_t *)nm, (uint64_t)nn, size, k, (uint32_t)n, (const uint8_t *)p,  \
                     (uint32_t)pl, (const uint32_t *)so, (const uint8_t *)sb, (uint8_t *)r);                 \
        UNPIN(out, r, 0); UNPIN(sbytes, sb, JNI_ABORT); UNPIN(soff, so, JNI_ABORT);                          \
        UNPIN(prefix, p, JNI_ABORT); UNPIN(nmArr, nm, JNI_ABORT);                                            \
        return st;                                                                                           \
    }
BLOOM_PREFIX_OP(bloomAddPrefix, sk_bloom_add_prefix)
BLOOM_PREFIX_OP(bloomContainsPrefix, sk_bloom_contains_prefix)

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_bloomCount(JNIEnv *env, jclass cls, jlong ctx,
                                                                     jbyteArray name, jintArray out) {
    (void)cls;
    jsize n = LEN(name);
    void *nm = PIN(name), *r = PIN(out);
    jint st = sk_bloom_count(CTX(ctx), (const uint8_t *)nm, (uint64_t)n, (int32_t *)r);
    UNPIN(out, r, 0); UNPIN(name, nm, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_setBitRange(JNIEnv *env, jclass cls, jlong ctx,
                                                                      jbyteArray key, jlong from, jlong to,
                                                                      jboolean value) {
    (void)cls;
    jsize n = LEN(key);
    void *k = PIN(key);
    jint st = sk_set_bit_range(CTX(ctx), (const uint8_t *)k, (uint64_t)n, from, to, value ? 1 : 0);
    UNPIN(key, k, JNI_ABORT);
    return st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_flushall(JNIEnv *env, jclass cls, jlong ctx) {
    (void)env; (void)cls;
    return sk_flushall(CTX(ctx));
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_setAsync(JNIEnv *env, jclass cls, jlong ctx, jboolean on) {
    (void)env; (void)cls;
    return sk_set_async(CTX(ctx), on ? 1 : 0);
}

/* completion tickets: the completion thread polls / waits, event loops never block */
JNIEXPORT jlong JNICALL Java_org_redisson_gpu_SketchNative_ticket(JNIEnv *env, jclass cls, jlong ctx) {
    (void)env; (void)cls;
    uint64_t t = 0;
    return sk_ticket(CTX(ctx), &t) == SK_OK ? (jlong)t : -1;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_poll(JNIEnv *env, jclass cls, jlong ctx, jlong ticket) {
    (void)env; (void)cls;
    int done = 0;
    jint st = sk_poll(CTX(ctx), (uint64_t)ticket, &done);
    return st == SK_OK ? done : st;
}

JNIEXPORT jint JNICALL Java_org_redisson_gpu_SketchNative_await(JNIEnv *env, jclass cls, jlong ctx, jlong ticket) {
    (void)env; (void)cls;
    return sk_wait(CTX(ctx), (uint64_t)ticket);
}
