/*
 * GpuBloomCoalescer -- group commit of concurrent RBloomFilter.add / contains calls on the engine (SURVEY 8f
 * rank 2; the Python mirror and its tests are redisson_amd/coalesce.py, tests/test_coalesce.py).
 *
 * The reference pays one pipeline round trip per element (M:RedissonBloomFilter.java:94-100,147-153) and RBatch
 * has no Bloom filter.  Here callers -- user threads and Netty event-loop threads alike -- only enqueue a request
 * and receive a Netty promise; ONE completion thread per engine context drains the queue in FIFO order, merges
 * each maximal run of requests for the same (filter, operation, size, k) into ONE sk_bloom_add /
 * sk_bloom_contains call, splits the replies and completes the promises.  A run never crosses a request of
 * another kind or filter, so every caller sees the linearizable result of the FIFO order; inside a merged add run
 * the engine's replies are the exact sequential replies of the requests in FIFO order.  No event-loop thread
 * ever waits on the device.  A run whose (size, k) no longer match the stored config fails with the engine's
 * "Bloom filter config has been changed" text, which GpuBloomFilter's retry loop handles as the reference does.
 * Source only here; see INTEGRATION.md.
 */
package org.redisson.gpu;

import java.util.ArrayDeque;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.List;

import org.redisson.client.RedisException;

import io.netty.util.concurrent.Promise;

public final class GpuBloomCoalescer implements Runnable {

    /** Any other engine call of a filter (tryInit, the config read, count, delete), run in its FIFO place. */
    public interface Task<T> {
        T call(long ctx);
    }

    static final class Req {
        final byte[] name;
        final boolean add;
        final long size;
        final int k;
        final byte[][] elems;
        final Promise<boolean[]> promise;
        final Task<Object> task;
        final Promise<Object> taskPromise;

        Req(byte[] name, boolean add, long size, int k, byte[][] elems, Promise<boolean[]> promise) {
            this.name = name;
            this.add = add;
            this.size = size;
            this.k = k;
            this.elems = elems;
            this.promise = promise;
            this.task = null;
            this.taskPromise = null;
        }

        Req(Task<Object> task, Promise<Object> taskPromise) {
            this.name = null;
            this.add = false;
            this.size = 0;
            this.k = 0;
            this.elems = new byte[0][];
            this.promise = null;
            this.task = task;
            this.taskPromise = taskPromise;
        }

        boolean sameRun(Req o) {
            // a task is a run of its own: it never merges, and nothing merges across it
            return task == null && o.task == null && add == o.add && size == o.size && k == o.k
                    && Arrays.equals(name, o.name);
        }
    }

    private final long ctx;
    private final int maxBatch;
    private final ArrayDeque<Req> queue = new ArrayDeque<Req>();
    private final Thread thread;
    private boolean stop;
    volatile long calls;     // engine calls made (one per merged run)
    volatile long requests;  // requests completed

    public GpuBloomCoalescer(long ctx, int maxBatch) {
        this.ctx = ctx;
        this.maxBatch = maxBatch;
        this.thread = new Thread(this, "sk-bloom-coalescer");
        this.thread.setDaemon(true);
        this.thread.start();
        GpuSketch.track(ctx, this); // closed by GpuSketch.close(ctx) before the context itself
    }

    /** Enqueue; never blocks on the device.  The promise gets one reply per element.  size = 0: the filter's
     *  config is read on the completion thread right before the engine call (the non-blocking callers' form). */
    public void submit(byte[] name, boolean add, long size, int k, byte[][] elems, Promise<boolean[]> promise) {
        enqueue(new Req(name, add, size, k, elems, promise), promise);
    }

    /** Enqueue any other engine call of a filter: it runs on the completion thread after every request queued
     *  before it, so it neither blocks the caller's (event-loop) thread on the device nor overtakes a queued
     *  add / contains.  The promise completes from that thread. */
    @SuppressWarnings("unchecked")
    public <T> void submitTask(Task<T> task, Promise<T> promise) {
        enqueue(new Req((Task<Object>) (Task<?>) task, (Promise<Object>) (Promise<?>) promise), promise);
    }

    private void enqueue(Req r, Promise<?> promise) {
        synchronized (queue) {
            if (stop) {
                promise.tryFailure(new IllegalStateException("coalescer closed"));
                return;
            }
            queue.addLast(r);
            queue.notify();
        }
    }

    public void close() throws InterruptedException {
        synchronized (queue) {
            stop = true;
            queue.notify();
        }
        thread.join();
    }

    @Override
    public void run() {
        while (true) {
            List<Req> run = new ArrayList<Req>();
            synchronized (queue) {
                while (queue.isEmpty() && !stop) {
                    try {
                        queue.wait();
                    } catch (InterruptedException e) {
                        Thread.currentThread().interrupt();
                        return;
                    }
                }
                if (queue.isEmpty()) {
                    return; // stopped and drained
                }
                Req head = queue.pollFirst();
                run.add(head);
                int n = head.elems.length;
                while (!queue.isEmpty() && queue.peekFirst().sameRun(head)
                        && n + queue.peekFirst().elems.length <= maxBatch) {
                    Req r = queue.pollFirst();
                    n += r.elems.length;
                    run.add(r);
                }
            }
            execute(run);
        }
    }

    private void execute(List<Req> run) {
        Req head = run.get(0);
        if (head.task != null) {
            try {
                head.taskPromise.trySuccess(head.task.call(ctx));
            } catch (RuntimeException e) {
                head.taskPromise.tryFailure(e);
            }
            calls++;
            requests++;
            return;
        }
        long size = head.size;
        int k = head.k;
        if (size == 0) { // config read here, in FIFO order
            long[] se = new long[2];
            int[] kk = new int[1];
            int cs = SketchNative.bloomConfig(ctx, head.name, se, kk, new double[1]);
            if (cs != SketchNative.SK_OK) {
                RuntimeException ex = cs == SketchNative.SK_ENOTINIT
                        ? new IllegalStateException(SketchNative.lastError(ctx))
                        : new RedisException(SketchNative.lastError(ctx));
                for (Req r : run) {
                    r.promise.tryFailure(ex);
                }
                calls++;
                requests += run.size();
                return;
            }
            size = se[0];
            k = kk[0];
        }
        List<byte[]> all = new ArrayList<byte[]>();
        for (Req r : run) {
            all.addAll(Arrays.asList(r.elems));
        }
        byte[] out = new byte[all.size()];
        // elements sharing a codec prefix go in prefix form (only the suffixes cross the host link)
        SketchDispatch.PrefixPacked pp = SketchDispatch.PrefixPacked.of(all, 8);
        int st;
        if (pp != null) {
            st = head.add ? SketchNative.bloomAddPrefix(ctx, head.name, size, k, pp.prefix, pp.off, pp.suffixes, out)
                    : SketchNative.bloomContainsPrefix(ctx, head.name, size, k, pp.prefix, pp.off, pp.suffixes, out);
        } else {
            SketchDispatch.Packed e = new SketchDispatch.Packed(all);
            st = head.add ? SketchNative.bloomAdd(ctx, head.name, size, k, e.off, e.bytes, out)
                    : SketchNative.bloomContains(ctx, head.name, size, k, e.off, e.bytes, out);
        }
        if (st != SketchNative.SK_OK) {
            RuntimeException ex = st == SketchNative.SK_ENOTINIT ? new IllegalStateException(SketchNative.lastError(ctx))
                    : new RedisException(SketchNative.lastError(ctx));
            for (Req r : run) {
                r.promise.tryFailure(ex);
            }
        } else {
            int p = 0;
            for (Req r : run) {
                boolean[] rep = new boolean[r.elems.length];
                for (int i = 0; i < rep.length; i++) {
                    rep[i] = out[p++] != 0;
                }
                r.promise.trySuccess(rep);
            }
        }
        calls++;
        requests += run.size();
    }
}
