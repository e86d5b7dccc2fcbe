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
import java.util.List;
import java.util.concurrent.ConcurrentHashMap;

import org.redisson.client.RedisException;
import org.redisson.client.codec.Codec;
import org.redisson.client.protocol.RedisCommand;

final class SketchDispatch {
    private SketchDispatch() {
    }

    static final class Packed {
        final long[] off;
        final byte[] bytes;

        Packed(List<byte[]> items) {
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

    static final Charset ISO = Charset.forName("ISO-8859-1"); // bytes <-> String one to one

    /* Per-context HLL name -> slab id cache (INTEGRATION.md "Caching slab ids").  Filled after a key's first
     * name-path PFADD; keyCommand's DEL drops the deleted keys' entries. */
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

    /* A run of PFADD commands: sk_pfadd_ids when every key has a cached slab id, else sk_pfadd by name,
     * then the run's keys are resolved (they exist now; nothing is created) and cached. */
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
            check(ctx, SketchNative.pfaddIds(ctx, ids, counts, e.off, e.bytes, out));
            return;
        }
        check(ctx, SketchNative.pfadd(ctx, k.off, k.bytes, counts, e.off, e.bytes, out));
        byte[] created = new byte[n];
        if (SketchNative.hllResolve(ctx, k.off, k.bytes, ids, created) == SketchNative.SK_OK) {
            for (int c = 0; c < n; c++) {
                cache.put(new String(keys.get(c), ISO), Integer.valueOf(ids[c]));
            }
        }
    }

    static void check(long ctx, int st) {
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

    static boolean engineHolds(long ctx, Object key) {
        int[] t = new int[1];
        byte[] k = key instanceof byte[] ? (byte[]) key : key.toString().getBytes(GpuSketchCommandService.UTF8);
        return SketchNative.type(ctx, k, t) == SketchNative.SK_OK && t[0] != SketchNative.SK_TYPE_NONE;
    }

    /* GET / SET / DEL on a key the engine holds (engineHolds of the first key).  GET decodes the raw bytes with
     * the command's codec (ByteArrayCodec for RBitSet: the bytes as they are); SET writes the encoded value;
     * DEL removes the keys the engine holds and replies their number. */
    static Object keyCommand(long ctx, Codec codec, RedisCommand<?> command, Object[] params) {
        try {
            String name = command.getName();
            if ("DEL".equals(name)) {
                java.util.ArrayList<byte[]> keys = new java.util.ArrayList<byte[]>();
                for (Object p : params) {
                    keys.add(p.toString().getBytes(GpuSketchCommandService.UTF8));
                }
                Packed k = new Packed(keys);
                long[] removed = new long[1];
                ConcurrentHashMap<String, Integer> cache = slabIds(ctx);
                for (byte[] kb : keys) {
                    cache.remove(new String(kb, ISO)); // the slab id may be handed to another key
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
            check(ctx, SketchNative.set(ctx, key, v));
            return "OK";
        } catch (RedisException e) {
            throw e;
        } catch (Exception e) {
            throw new RedisException(e.getMessage(), e);
        }
    }

    static Object single(long ctx, Codec codec, RedisCommand<?> command, Object[] params) {
        try {
            String name = command.getName();
            byte[] key = GpuSketchCommandService.encodeParam(codec, command, params[0], 1);
            if ("PFADD".equals(name)) {
                java.util.ArrayList<byte[]> elems = new java.util.ArrayList<byte[]>();
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
                java.util.ArrayList<byte[]> keys = new java.util.ArrayList<byte[]>();
                for (Object p : params) {
                    keys.add(p.toString().getBytes(GpuSketchCommandService.UTF8));
                }
                Packed k = new Packed(keys);
                long[] out = new long[1];
                check(ctx, SketchNative.pfcount(ctx, new int[] {keys.size()}, k.off, k.bytes, out));
                return Long.valueOf(out[0]);
            }
            if ("GETBIT".equals(name) || "SETBIT".equals(name)) {
                Packed k = new Packed(java.util.Collections.singletonList(key));
                long[] offs = {Long.parseLong(params[1].toString())};
                byte[] out = new byte[1];
                if ("GETBIT".equals(name)) {
                    check(ctx, SketchNative.getbit(ctx, k.off, k.bytes, offs, out));
                } else {
                    byte[] vals = {(byte) Integer.parseInt(params[2].toString())};
                    check(ctx, SketchNative.setbit(ctx, k.off, k.bytes, offs, vals, out));
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
            java.util.ArrayList<byte[]> srcs = new java.util.ArrayList<byte[]>();
            for (int i = first; i < params.length; i++) {
                srcs.add(params[i].toString().getBytes(GpuSketchCommandService.UTF8));
            }
            Packed s = new Packed(srcs);
            if (bitop) {
                int op = java.util.Arrays.asList("AND", "OR", "XOR", "NOT").indexOf(params[0].toString());
                long[] len = new long[1];
                check(ctx, SketchNative.bitop(ctx, op, params[1].toString().getBytes(GpuSketchCommandService.UTF8),
                        s.off, s.bytes, len));
                return Long.valueOf(len[0]);
            }
            check(ctx, SketchNative.pfmerge(ctx, key, s.off, s.bytes));
            return "OK";
        } catch (RedisException e) {
            throw e;
        } catch (Exception e) {
            throw new RedisException(e.getMessage(), e);
        }
    }
}
