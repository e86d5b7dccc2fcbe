/*
 * jni_drive.c -- runs the JNI shim (redisson_sketch_jni.c, compiled into this program) through a fake JNIEnv
 * against the real libredisson_sketch.so, so the shim's argument packing (array lengths, offsets, pinned
 * buffers, out arrays, status codes) executes once end to end without a JVM (Java seam item).
 * Java arrays are modelled as {length, element size, data}; the JNIEnv table implements the seven functions the
 * shim calls (jni/stub/jni.h).  Every result is printed as "name v1 v2 ..." for tests/test_jni_drive.py, which
 * replays the same commands through the Python binding and the oracle.  Exit 77 (after the host-only checks)
 * when no GPU can be opened.
 * Build: make -C jni drive   (gcc; no JDK needed)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "redisson_sketch_jni.c"

typedef struct {
    jsize len;
    int esz;
    unsigned char data[];
} FakeArr;

static FakeArr *arr_new(jsize len, int esz) {
    FakeArr *a = (FakeArr *)calloc(1, sizeof(FakeArr) + (size_t)len * (size_t)esz + 16);
    a->len = len;
    a->esz = esz;
    return a;
}
#define A(p) ((jarray)(void *)(p))

static jsize f_len(JNIEnv *e, jarray a) { (void)e; return ((FakeArr *)(void *)a)->len; }
static void *f_pin(JNIEnv *e, jarray a, jboolean *c) { (void)e; (void)c; return ((FakeArr *)(void *)a)->data; }
static void f_unpin(JNIEnv *e, jarray a, void *p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static jbyte *f_bytes(JNIEnv *e, jbyteArray a, jboolean *c) { (void)e; (void)c; return (jbyte *)((FakeArr *)(void *)a)->data; }
static void f_unbytes(JNIEnv *e, jbyteArray a, jbyte *p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static jbyteArray f_newbytes(JNIEnv *e, jsize n) { (void)e; return A(arr_new(n, 1)); }
static jstring f_newstr(JNIEnv *e, const char *s) { (void)e; return (jstring)(void *)strdup(s); }

static const struct JNINativeInterface_ FNS = {f_len, f_pin, f_unpin, f_bytes, f_unbytes, f_newbytes, f_newstr};
static JNIEnv ENV = &FNS;
static JNIEnv *env = &ENV;

/* byte[] of a C string / (long[] off, byte[] bytes) of n strings, as SketchDispatch.Packed builds them */
static jbyteArray jbytes(const char *s) {
    FakeArr *a = arr_new((jsize)strlen(s), 1);
    memcpy(a->data, s, strlen(s));
    return A(a);
}
static void packed(int n, const char **items, jlongArray *off, jbyteArray *bytes) {
    FakeArr *o = arr_new(n + 1, 8);
    size_t tot = 0;
    for (int i = 0; i < n; i++) tot += strlen(items[i]);
    FakeArr *b = arr_new((jsize)(tot + 16), 1);
    int64_t *ov = (int64_t *)o->data;
    size_t p = 0;
    for (int i = 0; i < n; i++) {
        ov[i] = (int64_t)p;
        memcpy(b->data + p, items[i], strlen(items[i]));
        p += strlen(items[i]);
    }
    ov[n] = (int64_t)p;
    *off = A(o);
    *bytes = A(b);
}
static jintArray jints(int n, const int *v) {
    FakeArr *a = arr_new(n, 4);
    if (v) memcpy(a->data, v, (size_t)n * 4);
    return A(a);
}
static jlongArray jlongs(int n, const int64_t *v) {
    FakeArr *a = arr_new(n, 8);
    if (v) memcpy(a->data, v, (size_t)n * 8);
    return A(a);
}
static unsigned char *D(jarray a) { return ((FakeArr *)(void *)a)->data; }

static void pr_u8(const char *name, jint st, jarray a) {
    printf("%s %d", name, st);
    for (jsize i = 0; i < f_len(env, a); i++) printf(" %d", (int)D(a)[i]);
    printf("\n");
}
static void pr_i32(const char *name, jint st, jarray a) {
    printf("%s %d", name, st);
    for (jsize i = 0; i < f_len(env, a); i++) printf(" %d", ((int32_t *)(void *)D(a))[i]);
    printf("\n");
}
static void pr_i64(const char *name, jint st, jarray a) {
    printf("%s %d", name, st);
    for (jsize i = 0; i < f_len(env, a); i++) printf(" %lld", (long long)((int64_t *)(void *)D(a))[i]);
    printf("\n");
}

int main(void) {
    jclass cls = NULL;
    /* host-only entry points first (no device needed) */
    printf("calcSlot %d %d %d\n", Java_org_redisson_gpu_SketchNative_calcSlot(env, cls, jbytes("somekey")),
           Java_org_redisson_gpu_SketchNative_calcSlot(env, cls, jbytes("foo{hash_tag}")),
           Java_org_redisson_gpu_SketchNative_calcSlot(env, cls, jbytes("{bf}__config")));
    fflush(stdout);
    jlong ctx = Java_org_redisson_gpu_SketchNative_open(env, cls, 0, 3, 0, 1024, 1 << 22);
    if (!ctx) {
        printf("NODEVICE\n");
        return 77;
    }
    jlongArray ko, eo;
    jbyteArray kb, eb;
    /* PFADD jd:a x y / PFADD jd:b z / PFADD jd:a x  (RBatch of three commands) */
    const char *pk[] = {"jd:a", "jd:b", "jd:a"}, *pe[] = {"x", "y", "z", "x"};
    int pc[] = {2, 1, 1};
    packed(3, pk, &ko, &kb);
    packed(4, pe, &eo, &eb);
    jbyteArray out3 = f_newbytes(env, 3);
    pr_u8("pfadd", Java_org_redisson_gpu_SketchNative_pfadd(env, cls, ctx, ko, kb, jints(3, pc), eo, eb, out3), out3);
    /* resolve / lookup / pfaddIds / pfcount / pfcountIds */
    const char *rk[] = {"jd:a", "jd:b"};
    packed(2, rk, &ko, &kb);
    jintArray ids = jints(2, NULL);
    jbyteArray cr = f_newbytes(env, 2);
    jint st = Java_org_redisson_gpu_SketchNative_hllResolve(env, cls, ctx, ko, kb, ids, cr);
    pr_u8("resolve_created", st, cr);
    const char *lk[] = {"jd:a", "jd:missing"};
    jlongArray lko;
    jbyteArray lkb;
    packed(2, lk, &lko, &lkb);
    jintArray lids = jints(2, NULL);
    st = Java_org_redisson_gpu_SketchNative_hllLookup(env, cls, ctx, lko, lkb, lids);
    printf("lookup %d %d %d\n", st, ((int32_t *)(void *)D(lids))[0] == ((int32_t *)(void *)D(ids))[0],
           ((int32_t *)(void *)D(lids))[1]);
    const char *qe[] = {"q", "r"};
    int one[] = {1, 1};
    packed(2, qe, &eo, &eb);
    jbyteArray out2 = f_newbytes(env, 2);
    pr_u8("pfaddIds", Java_org_redisson_gpu_SketchNative_pfaddIds(env, cls, ctx, ids, jints(2, one), eo, eb, out2),
          out2);
    /* the same handles in prefix form: elements "pre" + "q2" / "pre" + "r2" */
    {
        FakeArr *so = arr_new(3, 4);
        int32_t *sov = (int32_t *)(void *)so->data;
        sov[0] = 0, sov[1] = 2, sov[2] = 4;
        FakeArr *sb = arr_new(4 + 16, 1);
        memcpy(sb->data, "q2r2", 4);
        pr_u8("pfaddIdsPrefix", Java_org_redisson_gpu_SketchNative_pfaddIdsPrefix(env, cls, ctx, ids, jbytes("pre"),
                                                                                   A(so), A(sb), out2), out2);
    }
    const char *ck[] = {"jd:a", "jd:b", "jd:a", "jd:b", "jd:missing"};
    int nk[] = {1, 1, 3};
    packed(5, ck, &ko, &kb);
    jlongArray cnt = jlongs(3, NULL);
    pr_i64("pfcount", Java_org_redisson_gpu_SketchNative_pfcount(env, cls, ctx, jints(3, nk), ko, kb, cnt), cnt);
    jlongArray cnt2 = jlongs(2, NULL);
    pr_i64("pfcountIds", Java_org_redisson_gpu_SketchNative_pfcountIds(env, cls, ctx, ids, cnt2), cnt2);
    /* PFMERGE jd:m jd:a jd:b */
    packed(2, rk, &ko, &kb);
    st = Java_org_redisson_gpu_SketchNative_pfmerge(env, cls, ctx, jbytes("jd:m"), ko, kb);
    const char *mk[] = {"jd:m"};
    packed(1, mk, &ko, &kb);
    jlongArray cnt1 = jlongs(1, NULL);
    int nk1[] = {1};
    Java_org_redisson_gpu_SketchNative_pfcount(env, cls, ctx, jints(1, nk1), ko, kb, cnt1);
    pr_i64("pfmerge_count", st, cnt1);
    /* SETBIT / GETBIT / BITCOUNT / STRLEN / BITOP / GET / SET / TYPE */
    const char *sk[] = {"jd:s", "jd:s", "jd:s", "jd:t"};
    int64_t so[] = {5, 100, 5, 7};
    packed(4, sk, &ko, &kb);
    jbyteArray sv = f_newbytes(env, 4);
    D(sv)[0] = 1, D(sv)[1] = 1, D(sv)[2] = 0, D(sv)[3] = 1;
    jbyteArray old = f_newbytes(env, 4);
    pr_u8("setbit", Java_org_redisson_gpu_SketchNative_setbit(env, cls, ctx, ko, kb, jlongs(4, so), sv, old), old);
    int64_t go[] = {5, 100, 7, 1 << 20};
    jbyteArray gb = f_newbytes(env, 4);
    const char *gk[] = {"jd:s", "jd:s", "jd:t", "jd:s"};
    packed(4, gk, &ko, &kb);
    pr_u8("getbit", Java_org_redisson_gpu_SketchNative_getbit(env, cls, ctx, ko, kb, jlongs(4, go), gb), gb);
    /* SETBIT_VOID as the Java executors send it: no reply array */
    const char *wk[] = {"jd:w", "jd:w", "jd:w"};
    int64_t wo[] = {3, 3, 9};
    packed(3, wk, &ko, &kb);
    jbyteArray wv = f_newbytes(env, 3);
    D(wv)[0] = 1, D(wv)[1] = 1, D(wv)[2] = 1;
    jint wst = Java_org_redisson_gpu_SketchNative_setbit(env, cls, ctx, ko, kb, jlongs(3, wo), wv, NULL);
    int64_t wg[] = {3, 9, 4};
    jbyteArray wb = f_newbytes(env, 3);
    jint wgs = Java_org_redisson_gpu_SketchNative_getbit(env, cls, ctx, ko, kb, jlongs(3, wg), wb);
    pr_u8("void_getbit", wst ? wst : wgs, wb);
    jlongArray o1 = jlongs(1, NULL);
    pr_i64("bitcount", Java_org_redisson_gpu_SketchNative_bitcount(env, cls, ctx, jbytes("jd:s"), o1), o1);
    pr_i64("strlen", Java_org_redisson_gpu_SketchNative_strlen(env, cls, ctx, jbytes("jd:s"), o1), o1);
    const char *bk[] = {"jd:s", "jd:t"};
    packed(2, bk, &ko, &kb);
    pr_i64("bitop_or", Java_org_redisson_gpu_SketchNative_bitop(env, cls, ctx, 1, jbytes("jd:o"), ko, kb, o1), o1);
    jbyteArray g = Java_org_redisson_gpu_SketchNative_get(env, cls, ctx, jbytes("jd:o"));
    pr_u8("get", g ? 0 : -1, g);
    printf("get_missing %d\n", Java_org_redisson_gpu_SketchNative_get(env, cls, ctx, jbytes("jd:none")) == NULL);
    st = Java_org_redisson_gpu_SketchNative_set(env, cls, ctx, jbytes("jd:v"), jbytes("\x81\x01"));
    jbyteArray gb2 = f_newbytes(env, 2);
    const char *vk[] = {"jd:v", "jd:v"};
    int64_t vo[] = {0, 15};
    packed(2, vk, &ko, &kb);
    Java_org_redisson_gpu_SketchNative_getbit(env, cls, ctx, ko, kb, jlongs(2, vo), gb2);
    pr_u8("set_getbit", st, gb2);
    jintArray ty = jints(1, NULL);
    st = Java_org_redisson_gpu_SketchNative_type(env, cls, ctx, jbytes("jd:a"), ty);
    pr_i32("type_hll", st, ty);
    {   /* typeMany: an HLL, a bit string, a missing key */
        const char *tk[] = {"jd:a", "jd:s", "jd:none"};
        jlongArray tko;
        jbyteArray tkb;
        packed(3, tk, &tko, &tkb);
        jintArray tt = jints(3, NULL);
        st = Java_org_redisson_gpu_SketchNative_typeMany(env, cls, ctx, tko, tkb, tt);
        pr_i32("typeMany", st, tt);
    }
    pr_i64("bitsetLength", Java_org_redisson_gpu_SketchNative_bitsetLength(env, cls, ctx, jbytes("jd:s"), o1), o1);
    /* Bloom: tryInit(100, 0.03) -> 729 bits, k 5 (T:RedissonBloomFilterTest.java:12-16) */
    jintArray ok = jints(1, NULL);
    pr_i32("bloomTryInit", Java_org_redisson_gpu_SketchNative_bloomTryInit(env, cls, ctx, jbytes("jd:bf"), 100, 0.03, ok),
           ok);
    jlongArray se = jlongs(2, NULL);
    jintArray kk = jints(1, NULL);
    FakeArr *fp = arr_new(1, 8);
    st = Java_org_redisson_gpu_SketchNative_bloomConfig(env, cls, ctx, jbytes("jd:bf"), se, kk, A(fp));
    printf("bloomConfig %d %lld %lld %d %.4f\n", st, (long long)((int64_t *)(void *)D(se))[0],
           (long long)((int64_t *)(void *)D(se))[1], ((int32_t *)(void *)D(kk))[0], ((double *)(void *)fp->data)[0]);
    const char *be[] = {"\"e1\"", "\"e2\"", "\"e1\""};
    packed(3, be, &eo, &eb);
    jbyteArray bo = f_newbytes(env, 3);
    pr_u8("bloomAdd", Java_org_redisson_gpu_SketchNative_bloomAdd(env, cls, ctx, jbytes("jd:bf"), 729, 5, eo, eb, bo), bo);
    const char *bc[] = {"\"e1\"", "\"e3\""};
    packed(2, bc, &eo, &eb);
    jbyteArray bco = f_newbytes(env, 2);
    pr_u8("bloomContains",
          Java_org_redisson_gpu_SketchNative_bloomContains(env, cls, ctx, jbytes("jd:bf"), 729, 5, eo, eb, bco), bco);
    printf("bloomContains_changed %d\n",
           Java_org_redisson_gpu_SketchNative_bloomContains(env, cls, ctx, jbytes("jd:bf"), 730, 5, eo, eb, bco));
    {   /* contains of "\"e1\"" and "\"e3\"" in prefix form: prefix "\"e", suffixes 1", 3" */
        FakeArr *so = arr_new(3, 4);
        int32_t *sov = (int32_t *)(void *)so->data;
        sov[0] = 0, sov[1] = 2, sov[2] = 4;
        FakeArr *sb = arr_new(4 + 16, 1);
        memcpy(sb->data, "1\"3\"", 4);
        jbyteArray pco = f_newbytes(env, 2);
        pr_u8("bloomContainsPrefix", Java_org_redisson_gpu_SketchNative_bloomContainsPrefix(
                                         env, cls, ctx, jbytes("jd:bf"), 729, 5, jbytes("\"e"), A(so), A(sb), pco), pco);
        FakeArr *sb2 = arr_new(4 + 16, 1);
        memcpy(sb2->data, "4\"5\"", 4);
        jbyteArray pao = f_newbytes(env, 2);
        pr_u8("bloomAddPrefix", Java_org_redisson_gpu_SketchNative_bloomAddPrefix(
                                    env, cls, ctx, jbytes("jd:bf"), 729, 5, jbytes("\"e"), A(so), A(sb2), pao), pao);
    }
    jintArray bn = jints(1, NULL);
    pr_i32("bloomCount", Java_org_redisson_gpu_SketchNative_bloomCount(env, cls, ctx, jbytes("jd:bf"), bn), bn);
    /* range set, async tickets */
    st = Java_org_redisson_gpu_SketchNative_setBitRange(env, cls, ctx, jbytes("jd:r"), 3, 21, 1);
    pr_i64("setBitRange_bitcount", st == 0 ? Java_org_redisson_gpu_SketchNative_bitcount(env, cls, ctx, jbytes("jd:r"), o1)
                                           : st, o1);
    jlong t = Java_org_redisson_gpu_SketchNative_ticket(env, cls, ctx);
    printf("ticket %d %d\n", t > 0, Java_org_redisson_gpu_SketchNative_await(env, cls, ctx, t));
    /* DEL jd:a (+ a missing key) -> the cached handle of jd:a is stale */
    const char *dk[] = {"jd:a", "jd:zz"};
    packed(2, dk, &ko, &kb);
    jlongArray rm = jlongs(1, NULL);
    pr_i64("del", Java_org_redisson_gpu_SketchNative_del(env, cls, ctx, ko, kb, rm), rm);
    packed(2, qe, &eo, &eb);
    printf("pfaddIds_stale %d\n", Java_org_redisson_gpu_SketchNative_pfaddIds(env, cls, ctx, ids, jints(2, one), eo, eb,
                                                                              out2));
    jstring err = Java_org_redisson_gpu_SketchNative_lastError(env, cls, ctx);
    printf("lastError %s\n", (const char *)(void *)err);
    printf("flushall %d\n", Java_org_redisson_gpu_SketchNative_flushall(env, cls, ctx));
    Java_org_redisson_gpu_SketchNative_close(env, cls, ctx);
    printf("done\n");
    return 0;
}
