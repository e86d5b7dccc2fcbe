/*
 * SketchDispatch -- turns (RedisCommand, params) into C-ABI calls, one command
 * at a time (GpuSketchCommandService) or as same-kind runs of an RBatch
 * (GpuSketchBatchService).  Replies are the raw redis replies (Long / byte[] /
 * "OK"), so the command's own convertor produces what Redisson returns.
 * Source only here; see INTEGRATION.md.
 */
package org.redisson.gpu;

import java.io.ByteArrayOutputStream;
import java.nio.charset.Charset;
import java.util.ArrayList;
import java.util.List;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.ExecutorService;
import java.util.concurrent.Executors;
import java.util.concurrent.ThreadFactory;

import org.redisson.client.RedisException;
import org.redisson.client.codec.Codec;
import org.redisson.client.protocol.RedisCommand;
import org.redisson.client.protocol.RedisCommands;

public final class SketchDispatch {
    private SketchDispatch() {
    }

    public static final class Packed {
        public final long[] off;
        public final byte[] bytes;

        public Packed(List<byte[]> items) {
            off = new long[items.size() + 1];
            ByteArrayOutputStream out = new ByteArrayOutputStream();
            for (int i = 0; i < items.size(); i++) {
                off[i] = out.size();
                out.write(items.get(i), 0, items.get(i).length);
            }
            off[items.size()] = out.size();
            out.write(new byte[16], 0, 16); // device padding contract
            bytes = out.toByteArray();
        }
    }

    /* Elements in prefix form (sk_pfadd_ids_prefix / sk_bloom_*_prefix): the longest prefix every element shares
     * (<= 255 bytes; a codec's type header such as ["java.lang.Long",) and the suffixes with u32 offsets.  Only the
     * suffixes cross the host link; the engine rebuilds the elements on the device. */
    public static final class PrefixPacked {
        public final byte[] prefix;
        public final int[] off;
        public final byte[] suffixes;

        PrefixPacked(List<byte[]> items, int plen) {
            prefix = java.util.Arrays.copyOf(items.get(0), plen);
            off = new int[items.size() + 1];
            int tot = 0;
            for (byte[] x : items) {
                tot += x.length - plen;
            }
            suffixes = new byte[tot + 16]; // device padding contract
            int p = 0;
            for (int i = 0; i < items.size(); i++) {
                byte[] x = items.get(i);
                off[i] = p;
                System.arraycopy(x, plen, suffixes, p, x.length - plen);
                p += x.length - plen;
            }
            off[items.size()] = p;
        }

        /** The prefix form when the items share at least minPrefix bytes, else null. */
        public static PrefixPacked of(List<byte[]> items, int minPrefix) {
            if (items.isEmpty()) {
                return null;
            }
            byte[] first = items.get(0);
            int plen = Math.min(first.length, 255);
            for (int i = 1; i < items.size() && plen >= minPrefix; i++) {
                byte[] x = items.get(i);
                int m = Math.min(plen, x.length), j = 0;
                while (j < m && x[j] == first[j]) {
                    j++;
                }
                plen = j;
            }
            return plen >= minPrefix ? new PrefixPacked(items, plen) : null;
        }
    }

    static final Charset ISO = Charset.forName("ISO-8859-1"); // bytes <-> String one to one

    /* One FIFO worker thread per engine context (SURVEY 8b: no event-loop thread waits on the device).  Single
     * commands and RBatch sketch runs of one context are executed there in submission order. */
    static final ConcurrentHashMap<Long, ExecutorService> WORKERS = new ConcurrentHashMap<Long, ExecutorService>();

    public static ExecutorService worker(final long ctx) {
        ExecutorService w = WORKERS.get(ctx);
        if (w == null) {
            ExecutorService fresh = Executors.newSingleThreadExecutor(new ThreadFactory() {
                @Override
                public Thread newThread(Runnable r) {
                    Thread t = new Thread(r, "sk-engine-" + Long.toHexString(ctx));
                    t.setDaemon(true);
                    return t;
                }
            });
            w = WORKERS.putIfAbsent(ctx, fresh);
            if (w == null) {
                w = fresh;
            } else {
                fresh.shutdown();
            }
        }
        return w;
    }

    /** Before sk_close(ctx): queued work finishes (this waits for it), later submissions are refused. */
    public static void shutdownWorker(long ctx) throws InterruptedException {
        ExecutorService w = WORKERS.remove(ctx);
        if (w != null) {
            w.shutdown();
            while (!w.awaitTermination(1, java.util.concurrent.TimeUnit.SECONDS)) {
                // engine calls in flight: a device batch may take seconds; keep waiting
            }
        }
    }

    /** Drop every per-context table (slab-handle cache) once the context is closed: a later context opened at the
     * same address starts from nothing (ADVICE r3). */
    static void forget(long ctx) {
        SLAB_IDS.remove(ctx);
    }

    /* Per-context HLL name -> slab handle cache (INTEGRATION.md "Caching slab ids").  Filled after a run's
     * name-path PFADD from sk_hll_lookup (which creates nothing).  Every command that can free or replace a key
     * drops the key's entry (DEL, SET, BITOP / PFMERGE destinations, FLUSHALL); a handle cached across a race
     * anyway is refused by the engine (SK_ESTALE: the slab's generation changed) and the run is redone by name,
     * so a stale id can never write into a slab another key owns. */
    static final ConcurrentHashMap<Long, ConcurrentHashMap<String, Integer>> SLAB_IDS =
            new ConcurrentHashMap<Long, ConcurrentHashMap<String, Integer>>();

    static ConcurrentHashMap<String, Integer> slabIds(long ctx) {
        ConcurrentHashMap<String, Integer> m = SLAB_IDS.get(ctx);
        if (m == null) {
            ConcurrentHashMap<String, Integer> fresh = new ConcurrentHashMap<String, Integer>();
            m = SLAB_IDS.putIfAbsent(ctx, fresh);
            if (m == null) {
                m = fresh;
            }
        }
        return m;
    }

    static void invalidate(long ctx, byte[] key) {
        slabIds(ctx).remove(new String(key, ISO));
    }

    static void invalidateAll(long ctx) {
        slabIds(ctx).clear();
    }

    /* A run of PFADD commands: sk_pfadd_ids when every key has a cached slab handle, else sk_pfadd by name, then
     * the run's keys are looked up (they exist now; nothing is created) and cached. */
    static void pfaddRun(long ctx, List<byte[]> keys, Packed k, int[] counts, Packed e, byte[] out) {
        ConcurrentHashMap<String, Integer> cache = slabIds(ctx);
        int n = keys.size();
        int[] ids = new int[n];
        boolean cached = true;
        for (int c = 0; c < n && cached; c++) {
            Integer id = cache.get(new String(keys.get(c), ISO));
            if (id == null) {
                cached = false;
            } else {
                ids[c] = id.intValue();
            }
        }
        if (cached) {
            int st = SketchNative.pfaddIds(ctx, ids, counts, e.off, e.bytes, out);
            if (st != SketchNative.SK_ESTALE) {
                check(ctx, st);
                return;
            }
            for (byte[] key : keys) { // a key of the run was freed since it was cached: redo the run by name
                cache.remove(new String(key, ISO));
            }
        }
        check(ctx, SketchNative.pfadd(ctx, k.off, k.bytes, counts, e.off, e.bytes, out));
        if (SketchNative.hllLookup(ctx, k.off, k.bytes, ids) == SketchNative.SK_OK) {
            for (int c = 0; c < n; c++) {
                if (ids[c] != -1) {
                    cache.put(new String(keys.get(c), ISO), Integer.valueOf(ids[c]));
                }
            }
        }
    }

    public static void check(long ctx, int st) {
        if (st == SketchNative.SK_OK) {
            return;
        }
        if (st == SketchNative.SK_ENOTINIT) {
            throw new IllegalStateException(SketchNative.lastError(ctx));
        }
        if (st == SketchNative.SK_ETOOBIG) {
            throw new IllegalArgumentException(SketchNative.lastError(ctx));
        }
        throw new RedisException(SketchNative.lastError(ctx));
    }

    static byte[] keyBytes(Object key) {
        return key instanceof byte[] ? (byte[]) key : key.toString().getBytes(GpuSketchCommandService.UTF8);
    }

    static boolean engineHolds(long ctx, Object key) {
        int[] t = new int[1];
        return SketchNative.type(ctx, keyBytes(key), t) == SketchNative.SK_OK && t[0] != SketchNative.SK_TYPE_NONE;
    }

    /* DEL k1..kn splits by holder (ADVICE r1): the keys the engine holds are removed there, the rest (the Bloom
     * filter's "{name}__config" hash when redis-server keeps it, RBucket keys, ...) go to redis-server, and the
     * reply is the sum.  out[0] = engine-held keys, out[1] = the others. */
    static List<Object>[] splitDel(long ctx, Object[] params, java.util.Set<String> alsoEngine) {
        @SuppressWarnings("unchecked")
        List<Object>[] out = new List[] {new ArrayList<Object>(), new ArrayList<Object>()};
        for (Object p : params) {
            boolean eng = engineHolds(ctx, p) || (alsoEngine != null && alsoEngine.contains(p.toString()));
            out[eng ? 0 : 1].add(p);
        }
        return out;
    }

    /* GET / SET / DEL on a key the engine holds (engineHolds of the first key).  GET decodes the raw bytes with
     * the command's codec (ByteArrayCodec for RBitSet: the bytes as they are); SET writes the encoded value;
     * DEL removes the given keys from the engine and replies their number. */
    static Object keyCommand(long ctx, Codec codec, RedisCommand<?> command, Object[] params) {
        try {
            String name = command.getName();
            if ("DEL".equals(name)) {
                ArrayList<byte[]> keys = new ArrayList<byte[]>();
                for (int i = 0; i < params.length; i++) {
                    keys.add(GpuSketchCommandService.encodeParam(codec, command, params[i], i + 1));
                }
                Packed k = new Packed(keys);
                long[] removed = new long[1];
                for (byte[] kb : keys) {
                    invalidate(ctx, kb); // the slab may be handed to another key
                }
                check(ctx, SketchNative.del(ctx, k.off, k.bytes, removed));
                return Long.valueOf(removed[0]);
            }
            byte[] key = GpuSketchCommandService.encodeParam(codec, command, params[0], 1);
            if ("GET".equals(name)) {
                byte[] v = SketchNative.get(ctx, key);
                if (v == null) {
                    return null;
                }
                return codec.getValueDecoder().decode(io.netty.buffer.Unpooled.wrappedBuffer(v), null);
            }
            byte[] v = GpuSketchCommandService.encodeParam(codec, command, params[1], 2);
            invalidate(ctx, key); // SET replaces whatever the key held (an HLL's slab is freed)
            check(ctx, SketchNative.set(ctx, key, v));
            return "OK";
        } catch (RedisException e) {
            throw e;
        } catch (Exception e) {
            throw new RedisException(e.getMessage(), e);
        }
    }

    /* One PFCOUNT per command, all of a run's commands in one sk_pfcount (single keys share one histogram
     * launch; multi-key commands are unions). */
    static long[] pfcountRun(long ctx, Codec codec, List<RedisCommand<?>> commands, List<Object[]> paramsList)
            throws Exception {
        int n = paramsList.size();
        int[] nk = new int[n];
        ArrayList<byte[]> keys = new ArrayList<byte[]>();
        for (int c = 0; c < n; c++) {
            Object[] params = paramsList.get(c);
            nk[c] = params.length;
            for (int i = 0; i < params.length; i++) {
                keys.add(GpuSketchCommandService.encodeParam(codec, commands.get(c), params[i], i + 1));
            }
        }
        Packed k = new Packed(keys);
        long[] out = new long[n];
        check(ctx, SketchNative.pfcount(ctx, nk, k.off, k.bytes, out));
        return out;
    }

    static Object single(long ctx, Codec codec, RedisCommand<?> command, Object[] params) {
        try {
            String name = command.getName();
            byte[] key = GpuSketchCommandService.encodeParam(codec, command, params[0], 1);
            if ("PFADD".equals(name)) {
                ArrayList<byte[]> elems = new ArrayList<byte[]>();
                for (int i = 1; i < params.length; i++) {
                    elems.add(GpuSketchCommandService.encodeParam(codec, command, params[i], i + 1));
                }
                Packed k = new Packed(java.util.Collections.singletonList(key));
                Packed e = new Packed(elems);
                byte[] out = new byte[1];
                check(ctx, SketchNative.pfadd(ctx, k.off, k.bytes, new int[] {elems.size()}, e.off, e.bytes, out));
                return Long.valueOf(out[0]);
            }
            if ("PFCOUNT".equals(name)) {
                return Long.valueOf(pfcountRun(ctx, codec, java.util.Collections.<RedisCommand<?>>singletonList(command),
                        java.util.Collections.singletonList(params))[0]);
            }
            if ("GETBIT".equals(name) || "SETBIT".equals(name)) {
                Packed k = new Packed(java.util.Collections.singletonList(key));
                long[] offs = {Long.parseLong(params[1].toString())};
                byte[] out = new byte[1];
                if ("GETBIT".equals(name)) {
                    check(ctx, SketchNative.getbit(ctx, k.off, k.bytes, offs, out));
                } else {
                    byte[] vals = {(byte) Integer.parseInt(params[2].toString())};
                    check(ctx, SketchNative.setbit(ctx, k.off, k.bytes, offs, vals,
                            command == RedisCommands.SETBIT_VOID ? null : out));
                }
                return Long.valueOf(out[0]);
            }
            if ("BITCOUNT".equals(name) || "STRLEN".equals(name)) {
                long[] out = new long[1];
                check(ctx, "BITCOUNT".equals(name) ? SketchNative.bitcount(ctx, key, out)
                        : SketchNative.strlen(ctx, key, out));
                return Long.valueOf(out[0]);
            }
            // PFMERGE dest srcs... / BITOP op dest srcs...
            boolean bitop = "BITOP".equals(name);
            int first = bitop ? 2 : 1;
            ArrayList<byte[]> srcs = new ArrayList<byte[]>();
            for (int i = first; i < params.length; i++) {
                srcs.add(GpuSketchCommandService.encodeParam(codec, command, params[i], i + 1));
            }
            Packed s = new Packed(srcs);
            if (bitop) {
                int op = java.util.Arrays.asList("AND", "OR", "XOR", "NOT").indexOf(params[0].toString());
                byte[] dest = GpuSketchCommandService.encodeParam(codec, command, params[1], 2);
                invalidate(ctx, dest); // BITOP replaces its destination (an HLL there is freed)
                long[] len = new long[1];
                check(ctx, SketchNative.bitop(ctx, op, dest, s.off, s.bytes, len));
                return Long.valueOf(len[0]);
            }
            invalidate(ctx, key); // PFMERGE destination (a string there is adopted or refused, never reused)
            check(ctx, SketchNative.pfmerge(ctx, key, s.off, s.bytes));
            return "OK";
        } catch (RedisException e) {
            throw e;
        } catch (Exception e) {
            throw new RedisException(e.getMessage(), e);
        }
    }
}
