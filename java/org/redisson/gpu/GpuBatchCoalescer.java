/*
 * GpuBatchCoalescer -- group commit of concurrently executed RBatches of PFADD commands (the C2 ingestion shape;
 * the Python mirror and its tests are redisson_amd/coalesce.py BatchCoalescer, tests/test_batch_coalesce.py).
 *
 * The reference sends every RBatch as its own pipeline (M:command/CommandBatchService.java:184-293) and
 * redis-server applies the batches one after another.  Here GpuSketchBatchService hands a batch whose commands are
 * all PFADDs on engine-held keys to this coalescer instead of running it alone.  The context's FIFO worker runs
 * each maximal sequence of such batches queued together (up to maxCmds commands) as ONE sk_pfadd_ids call over
 * slab handles cached per tenant (names are typed and resolved only on a cache miss, SK_ESTALE drops the cache);
 * at >= 4 M commands (and >= 160 per HLL key held) the engine applies it with the line schedule (register lines
 * streamed once per call instead of once per element).  The concatenation keeps FIFO order and PFADD replies depend only
 * on order, so every batch gets exactly the replies it would get run alone in that order.  A PFADD on a key of
 * another type fails that command alone inside the engine (pipeline semantics); its batch fails with the
 * engine's error and every other batch of the call completes normally.  Groups run as tasks of the context's FIFO
 * worker, so batches keep the order of their executeAsync calls.  Source only here; see INTEGRATION.md.
 */
package org.redisson.gpu;

import java.util.ArrayList;
import java.util.HashSet;
import java.util.List;
import java.util.Set;

import org.redisson.client.RedisException;

import io.netty.util.concurrent.Promise;

public final class GpuBatchCoalescer {

    /** One RBatch: command c = PFADD keys[c] elems[c] (encoded as CommandEncoder would); one reply per command. */
    static final class Req {
        final List<byte[]> keys;
        final List<byte[][]> elems;
        final Promise<boolean[]> promise;

        Req(List<byte[]> keys, List<byte[][]> elems, Promise<boolean[]> promise) {
            this.keys = keys;
            this.elems = elems;
            this.promise = promise;
        }
    }

    /* A group is one task on the context's FIFO worker (SketchDispatch.worker): PFADD-only batches join the open
     * group until the worker starts it or another batch is queued behind it, so groups are exactly the maximal
     * sequences of PFADD-only batches between other batches, and the worker's FIFO order is kept. */
    final class Group implements Runnable {
        final List<Req> reqs = new ArrayList<Req>();
        int n;
        boolean started;

        @Override
        public void run() {
            synchronized (GpuBatchCoalescer.this) {
                started = true;
                if (open == this) {
                    open = null;
                }
            }
            try {
                execute(reqs);
            } catch (RuntimeException e) {
                for (Req r : reqs) {
                    r.promise.tryFailure(e);
                }
            }
        }
    }

    private static final java.util.concurrent.ConcurrentHashMap<Long, GpuBatchCoalescer> BY_CTX =
            new java.util.concurrent.ConcurrentHashMap<Long, GpuBatchCoalescer>();

    private final long ctx;
    private final int maxCmds;
    private Group open; // guarded by this
    volatile long calls;    // sk_pfadd calls made (one per group)
    volatile long batches;  // batches completed

    private GpuBatchCoalescer(long ctx, int maxCmds) {
        this.ctx = ctx;
        this.maxCmds = maxCmds;
    }

    /** Turn group commit on for a context (GpuSketchBatchService then routes PFADD-only batches here). */
    public static GpuBatchCoalescer enable(long ctx, int maxCmds) {
        GpuBatchCoalescer c = new GpuBatchCoalescer(ctx, maxCmds);
        GpuBatchCoalescer old = BY_CTX.putIfAbsent(ctx, c);
        return old != null ? old : c;
    }

    /** The context's coalescer, or null when group commit is off. */
    public static GpuBatchCoalescer of(long ctx) {
        return BY_CTX.get(ctx);
    }

    public static void disable(long ctx) {
        BY_CTX.remove(ctx);
    }

    /** Enqueue a PFADD-only batch; never blocks on the device. */
    public synchronized void submit(List<byte[]> keys, List<byte[][]> elems, Promise<boolean[]> promise) {
        if (open == null || open.started || open.n + keys.size() > maxCmds) {
            open = new Group();
            SketchDispatch.worker(ctx).execute(open);
        }
        open.reqs.add(new Req(keys, elems, promise));
        open.n += keys.size();
    }

    /** Queue another batch's task behind every group opened so far; later PFADD-only batches open a new group. */
    public synchronized void executeAfter(Runnable task) {
        open = null;
        SketchDispatch.worker(ctx).execute(task);
    }

    /* key -> slab handle (sk_hll_resolve), touched only by the context's worker thread (groups run there); valid
     * until the key is deleted or replaced, which the engine reports as SK_ESTALE without writing anything */
    private final java.util.HashMap<String, Integer> ids = new java.util.HashMap<String, Integer>();

    /* The group's keys without a cached handle: typed in ONE sk_type_many call, the non-string ones resolved
     * (created) in one sk_hll_resolve call; a key holding a plain string is resolved on its own (adopted when it
     * holds a valid HLL string), else its commands fail.  Returns key -> error text of the failing keys; created
     * collects the keys this resolution created (their first PFADD replies 1). */
    private java.util.Map<String, String> resolve(List<byte[]> keys, Set<String> created) {
        java.util.LinkedHashMap<String, byte[]> miss = new java.util.LinkedHashMap<String, byte[]>();
        for (byte[] k : keys) {
            String s = new String(k, SketchDispatch.ISO);
            if (!ids.containsKey(s)) {
                miss.put(s, k);
            }
        }
        java.util.Map<String, String> bad = new java.util.HashMap<String, String>();
        if (miss.isEmpty()) {
            return bad;
        }
        List<byte[]> mk = new ArrayList<byte[]>(miss.values());
        SketchDispatch.Packed pk = new SketchDispatch.Packed(mk);
        int[] types = new int[mk.size()];
        check(SketchNative.typeMany(ctx, pk.off, pk.bytes, types));
        List<byte[]> plain = new ArrayList<byte[]>();
        List<byte[]> strings = new ArrayList<byte[]>();
        for (int i = 0; i < types.length; i++) {
            (types[i] == SketchNative.SK_TYPE_NONE || types[i] == SketchNative.SK_TYPE_HLL ? plain : strings)
                    .add(mk.get(i));
        }
        if (!plain.isEmpty()) {
            SketchDispatch.Packed pp = new SketchDispatch.Packed(plain);
            int[] h = new int[plain.size()];
            byte[] cr = new byte[plain.size()];
            check(SketchNative.hllResolve(ctx, pp.off, pp.bytes, h, cr));
            for (int i = 0; i < h.length; i++) {
                String s = new String(plain.get(i), SketchDispatch.ISO);
                ids.put(s, h[i]);
                if (cr[i] != 0) {
                    created.add(s);
                }
            }
        }
        for (byte[] k : strings) {
            List<byte[]> one = new ArrayList<byte[]>();
            one.add(k);
            SketchDispatch.Packed p1 = new SketchDispatch.Packed(one);
            int[] h = new int[1];
            String s = new String(k, SketchDispatch.ISO);
            if (SketchNative.hllResolve(ctx, p1.off, p1.bytes, h, null) == SketchNative.SK_OK) {
                ids.put(s, h[0]);
            } else {
                bad.put(s, SketchNative.lastError(ctx));
            }
        }
        return bad;
    }

    private void check(int st) {
        if (st != SketchNative.SK_OK) {
            throw new RedisException(SketchNative.lastError(ctx));
        }
    }

    /* The group as ONE sk_pfadd_ids (or sk_pfadd_ids_prefix) call over cached slab handles: no name resolution on
     * the hot path and the library's liveness check on host threads over the ids.  Pageable inputs take HIP's own
     * pageable copy (the library's pinned staging ring is opt-in, SK_STAGE=1, and measured no faster; with the
     * prefix form, Java arrays reach 1.1 G PFADD/s per call, the same as sk_host_alloc memory: profiles/r04k_host).
     * A stale cache is dropped and the group resolved again once. */
    private void execute(List<Req> group) {
        List<byte[]> keys = new ArrayList<byte[]>();
        for (Req r : group) {
            keys.addAll(r.keys);
        }
        int st = SketchNative.SK_OK;
        String err = null;
        byte[] out = new byte[keys.size()];
        java.util.Map<String, String> bad = null;
        Set<String> created = new HashSet<String>();
        for (int attempt = 0; attempt < 2; attempt++) {
            created.clear();
            bad = resolve(keys, created);
            List<Integer> okIds = new ArrayList<Integer>();
            List<byte[]> flat = new ArrayList<byte[]>();
            List<Integer> counts = new ArrayList<Integer>();
            int c = 0;
            for (Req r : group) {
                for (int j = 0; j < r.keys.size(); j++, c++) {
                    String s = new String(r.keys.get(j), SketchDispatch.ISO);
                    if (bad.containsKey(s)) {
                        continue;
                    }
                    okIds.add(ids.get(s));
                    byte[][] es = r.elems.get(j);
                    counts.add(es.length);
                    for (byte[] x : es) {
                        flat.add(x);
                    }
                }
            }
            int[] idv = new int[okIds.size()];
            int[] cnt = new int[okIds.size()];
            for (int i = 0; i < idv.length; i++) {
                idv[i] = okIds.get(i);
                cnt[i] = counts.get(i);
            }
            byte[] sub = new byte[idv.length];
            // one-element commands sharing a codec prefix (every Jackson Long): the prefix form ships only the
            // suffixes and u32 offsets over the host link (sk_pfadd_ids_prefix); anything else the full form
            SketchDispatch.PrefixPacked pp = flat.size() == idv.length ? SketchDispatch.PrefixPacked.of(flat, 8) : null;
            if (idv.length == 0) {
                st = SketchNative.SK_OK;
            } else if (pp != null) {
                st = SketchNative.pfaddIdsPrefix(ctx, idv, pp.prefix, pp.off, pp.suffixes, sub);
            } else {
                SketchDispatch.Packed e = new SketchDispatch.Packed(flat);
                st = SketchNative.pfaddIds(ctx, idv, cnt, e.off, e.bytes, sub);
            }
            if (st == SketchNative.SK_ESTALE && attempt == 0) {
                ids.clear();
                continue;
            }
            err = st == SketchNative.SK_OK ? null : SketchNative.lastError(ctx);
            // scatter the sub-batch's replies back; the command that created its key replies 1
            Set<String> seen = new HashSet<String>();
            int p = 0;
            c = 0;
            for (Req r : group) {
                for (int j = 0; j < r.keys.size(); j++, c++) {
                    String s = new String(r.keys.get(j), SketchDispatch.ISO);
                    if (bad.containsKey(s)) {
                        continue;
                    }
                    out[c] = sub[p++];
                    if (created.contains(s) && seen.add(s)) {
                        out[c] = 1;
                    }
                    seen.add(s);
                }
            }
            break;
        }
        // a device / capacity error fails every batch of the call; a key of another type fails its batches only
        boolean all = st != SketchNative.SK_OK;
        String badMsg = bad.isEmpty() ? null : bad.values().iterator().next();
        int p = 0;
        for (Req r : group) {
            boolean failed = all;
            boolean[] rep = new boolean[r.keys.size()];
            for (int c = 0; c < rep.length; c++, p++) {
                rep[c] = out[p] != 0;
                if (!failed && bad.containsKey(new String(r.keys.get(c), SketchDispatch.ISO))) {
                    failed = true;
                }
            }
            if (failed) {
                r.promise.tryFailure(new RedisException(all ? err : badMsg));
            } else {
                r.promise.trySuccess(rep);
            }
        }
        calls++;
        batches += group.size();
    }
}
