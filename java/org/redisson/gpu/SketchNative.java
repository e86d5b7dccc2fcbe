/*
 * JNI binding of libredisson_sketch.so (include/redisson_sketch.h).
 * Source only in this repository (no JDK in the build image); see INTEGRATION.md.
 * Every array argument follows the C ABI: variable-length byte strings are
 * (long[] off (n+1), byte[] bytes); replies are written into caller arrays.
 */
package org.redisson.gpu;

public final class SketchNative {
    static {
        System.loadLibrary("redisson_sketch_jni"); // links libredisson_sketch.so
    }

    private SketchNative() {
    }

    public static final int SK_OK = 0, SK_EWRONGTYPE = -1, SK_ERANGE = -2, SK_ECONFIG = -3, SK_ENOTINIT = -4,
            SK_EDEVICE = -5, SK_EINVAL = -6, SK_ENOMEM = -7, SK_ESYNTAX = -8, SK_ETOOBIG = -9, SK_ECORRUPT = -10,
            SK_ESTALE = -11;

    public static native long open(int device, int redisMajor, long maxBitOffset, long hllCapacity, long maxBatch);
    public static native void close(long ctx);
    public static native String lastError(long ctx);
    public static native int calcSlot(byte[] key);

    public static native int del(long ctx, long[] keyOff, byte[] keys, long[] outRemoved);
    public static native int pfadd(long ctx, long[] keyOff, byte[] keys, int[] elemCounts, long[] elemOff,
                                   byte[] elems, byte[] outChanged);
    /** sk_hll_resolve: name -> slab id, creating empty HLLs (outCreated[i] = 1 if this call created key i). */
    public static native int hllResolve(long ctx, long[] keyOff, byte[] keys, int[] outIds, byte[] outCreated);
    /** sk_hll_lookup: name -> slab handle of EXISTING HLLs (-1 = missing), creating nothing. */
    public static native int hllLookup(long ctx, long[] keyOff, byte[] keys, int[] outIds);
    /** sk_pfadd_ids: slab handles from a cached sk_hll_resolve; SK_ESTALE once the key was deleted / replaced. */
    public static native int pfaddIds(long ctx, int[] keyIds, int[] elemCounts, long[] elemOff, byte[] elems,
                                      byte[] outChanged);
    /* sk_pfadd_ids_prefix: one-element PFADDs whose elements are prefix + suffixes[suffixOff[i] .. suffixOff[i+1]) */
    public static native int pfaddIdsPrefix(long ctx, int[] keyIds, byte[] prefix, int[] suffixOff, byte[] suffixes,
                                            byte[] outChanged);
    public static native int pfcount(long ctx, int[] nkeys, long[] keyOff, byte[] keys, long[] outCounts);
    /** sk_pfcount_ids: RHyperLogLog.count of many keys by cached slab id. */
    public static native int pfcountIds(long ctx, int[] keyIds, long[] outCounts);
    public static native int pfmerge(long ctx, byte[] dest, long[] srcOff, byte[] srcs);
    public static native int setbit(long ctx, long[] keyOff, byte[] keys, long[] offsets, byte[] values,
                                    byte[] outOld);
    public static native int getbit(long ctx, long[] keyOff, byte[] keys, long[] offsets, byte[] outBits);
    public static native int bitcount(long ctx, byte[] key, long[] out);
    public static native int strlen(long ctx, byte[] key, long[] out);
    public static native int bitop(long ctx, int op, byte[] dest, long[] srcOff, byte[] srcs, long[] outLen);
    public static final int SK_TYPE_NONE = 0, SK_TYPE_HLL = 1, SK_TYPE_STRING = 2;
    public static native int type(long ctx, byte[] key, int[] outType);
    /** sk_type_many: types of many keys in one call (outTypes[i] = SK_TYPE_*; 3 = a Bloom filter's name). */
    public static native int typeMany(long ctx, long[] keyOff, byte[] keys, int[] outTypes);
    public static native byte[] get(long ctx, byte[] key); // null when the key does not exist
    public static native int set(long ctx, byte[] key, byte[] value);
    public static native int bitsetLength(long ctx, byte[] key, long[] out);

    public static native int bloomTryInit(long ctx, byte[] name, long expected, double fpp, int[] outOk);
    public static native int bloomConfig(long ctx, byte[] name, long[] sizeExpected, int[] k, double[] fpp);
    public static native int bloomAdd(long ctx, byte[] name, long size, int k, long[] elemOff, byte[] elems,
                                      byte[] out);
    public static native int bloomContains(long ctx, byte[] name, long size, int k, long[] elemOff, byte[] elems,
                                           byte[] out);
    public static native int bloomAddPrefix(long ctx, byte[] name, long size, int k, byte[] prefix, int[] suffixOff,
                                            byte[] suffixes, byte[] out);
    public static native int bloomContainsPrefix(long ctx, byte[] name, long size, int k, byte[] prefix,
                                                 int[] suffixOff, byte[] suffixes, byte[] out);
    public static native int bloomCount(long ctx, byte[] name, int[] out);

    // RBitSet.set(from, to) / clear(from, to) as one device fill (M:RedissonBitSet.java:194-228)
    public static native int setBitRange(long ctx, byte[] key, long from, long to, boolean value);
    public static native int flushall(long ctx);

    // asynchronous submission: _dev / batch calls return once enqueued; a ticket
    // covers everything enqueued so far.  poll: 1 done (ticket released), 0 not
    // yet, < 0 status; await blocks a completion thread, never an event loop.
    public static native int setAsync(long ctx, boolean on);
    public static native long ticket(long ctx);
    public static native int poll(long ctx, long ticket);
    public static native int await(long ctx, long ticket);
}
