/*
 * GpuSketch -- lifecycle of one engine context in a JVM, and the executor factories the reference's call sites use.
 *
 * open()   sk_open through JNI (one context per GPU; keys are routed by sk_owner = calcSlot % nGPU).
 * install  makes a context the one newBatchService() hands to the reference's internal batches.
 * close()  ends everything keyed by the context, in order, before sk_close: the PFADD group-commit coalescer
 *          (GpuBatchCoalescer.disable), the Bloom coalescers opened on it, the FIFO worker (queued work finishes
 *          first) and the slab-handle caches.  Per-context tables are keyed by the raw ctx pointer, so a context
 *          opened later at the same address must not find the old ones: a cached (slab, generation) handle of the
 *          old context could validate against the new one's fresh generations (ADVICE r3).
 *
 * The reference builds plain CommandBatchService objects for its own internal batches: RBitSet range set/clear
 * (M:RedissonBitSet.java:204,223), RBatch (M:RedissonBatch.java:61), RBatchReactive
 * (M:reactive/RedissonBatchReactive.java:51) and RedissonBloomFilter's pipelines (:94,147,190,231).  Each of those
 * `new CommandBatchService(cm)` becomes `GpuSketch.newBatchService(cm)` (INTEGRATION.md).  Source only here.
 */
package org.redisson.gpu;

import java.util.List;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.CopyOnWriteArrayList;

import org.redisson.command.CommandBatchService;
import org.redisson.connection.ConnectionManager;

public final class GpuSketch {
    private GpuSketch() {
    }

    private static volatile long installed; // 0: no engine, the factories return the reference's classes
    private static final ConcurrentHashMap<Long, List<GpuBloomCoalescer>> BLOOM =
            new ConcurrentHashMap<Long, List<GpuBloomCoalescer>>();

    /** sk_open; throws when the device or the library is unavailable (there is no CPU fallback). */
    public static long open(int device, int redisMajor, long maxBitOffset, long hllCapacity, long maxBatch) {
        long ctx = SketchNative.open(device, redisMajor, maxBitOffset, hllCapacity, maxBatch);
        if (ctx == 0) {
            throw new IllegalStateException("sketch engine: sk_open failed on device " + device);
        }
        return ctx;
    }

    public static void install(long ctx) {
        installed = ctx;
    }

    public static long installed() {
        return installed;
    }

    /** The batch executor for the reference's internal batches: the engine's when a context is installed. */
    public static CommandBatchService newBatchService(ConnectionManager connectionManager) {
        long ctx = installed;
        return ctx != 0 ? new GpuSketchBatchService(connectionManager, ctx)
                : new CommandBatchService(connectionManager);
    }

    static void track(long ctx, GpuBloomCoalescer c) {
        List<GpuBloomCoalescer> l = BLOOM.get(ctx);
        if (l == null) {
            List<GpuBloomCoalescer> fresh = new CopyOnWriteArrayList<GpuBloomCoalescer>();
            l = BLOOM.putIfAbsent(ctx, fresh);
            if (l == null) {
                l = fresh;
            }
        }
        l.add(c);
    }

    /** Close a context and everything keyed by it (see the header); the context must not be used afterwards. */
    public static void close(long ctx) throws InterruptedException {
        if (installed == ctx) {
            installed = 0;
        }
        GpuBatchCoalescer.disable(ctx);          // later PFADD-only batches run alone, on the worker
        List<GpuBloomCoalescer> bl = BLOOM.remove(ctx);
        if (bl != null) {
            for (GpuBloomCoalescer c : bl) {
                c.close();                       // drains its queue, then its thread ends
            }
        }
        SketchDispatch.shutdownWorker(ctx);      // queued commands, batches and groups finish first
        SketchDispatch.forget(ctx);
        SketchNative.close(ctx);
    }
}
