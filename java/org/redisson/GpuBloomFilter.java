/*
 * GpuBloomFilter -- RBloomFilter (M:core/RBloomFilter.java:27-60) on the engine's Bloom entry points, the
 * executor path SURVEY 8f rank 2 asks for.  Same behaviour as RedissonBloomFilter (M:RedissonBloomFilter.java):
 *   tryInit      -> sk_bloom_try_init (sizing :69-78,223-252; the config is stored with the filter, Q6 kept)
 *   readConfig   -> sk_bloom_config ("Bloom filter is not initialized!" IllegalStateException, :206-221)
 *   add/contains -> sk_bloom_add / sk_bloom_contains through GpuBloomCoalescer: xx_r39 + farmUo and the k
 *                   probes run on the GPU (Q2: only probes 0..k-2 decide the reply), concurrent calls merge
 *                   into one launch, and the "Bloom filter config has been changed" retry loop of :108-111 /
 *                   :162-166 is kept verbatim (the engine checks size / k as the EVAL of addConfigCheck did)
 *   count        -> sk_bloom_count (:188-199)
 *   delete       -> DEL name {name}__config, both on the engine (:201-203)
 * Every engine call runs on the coalescer's FIFO completion thread: add / contains as merged runs, and tryInit,
 * the config read, count, the getters and delete as tasks in their FIFO place (submitTask), so no caller thread
 * makes a JNI call and a delete never overtakes a queued add / contains (tests/test_coalesce.py, Python twin).
 * It lives in org.redisson next to RedissonBloomFilter (RedissonExpirable's constructors are package-private);
 * Redisson.getBloomFilter returns it when the engine is configured (INTEGRATION.md).  Source only here.
 */
package org.redisson;

import java.nio.charset.Charset;
import java.util.concurrent.ExecutionException;

import org.redisson.client.RedisException;
import org.redisson.client.codec.Codec;
import org.redisson.command.CommandAsyncExecutor;
import org.redisson.core.RBloomFilter;
import org.redisson.gpu.GpuBloomCoalescer;
import org.redisson.gpu.SketchDispatch;
import org.redisson.gpu.SketchNative;

import io.netty.util.concurrent.Future;
import io.netty.util.concurrent.Promise;

public class GpuBloomFilter<T> extends RedissonExpirable implements RBloomFilter<T> {

    private static final Charset UTF8 = Charset.forName("UTF-8");

    private volatile long size;
    private volatile int hashIterations;
    private final long ctx;
    private final GpuBloomCoalescer coalescer;
    private final CommandAsyncExecutor executor;

    public GpuBloomFilter(Codec codec, CommandAsyncExecutor executor, String name, long ctx,
                          GpuBloomCoalescer coalescer) {
        super(codec, executor, name);
        this.executor = executor;
        this.ctx = ctx;
        this.coalescer = coalescer;
    }

    private byte[] nameBytes() {
        return getName().getBytes(UTF8);
    }

    private byte[] encode(T object) {
        try {
            return codec.getValueEncoder().encode(object); // :170-178
        } catch (Exception e) {
            throw new IllegalArgumentException(e);
        }
    }

    /** add / contains: the reference's loop (:80-114, :133-168) with the GPU call in place of the pipeline. */
    private boolean call(boolean add, T object) {
        byte[][] state = {encode(object)};
        while (true) {
            if (size == 0) {
                readConfig();
            }
            Promise<boolean[]> p = executor.getConnectionManager().newPromise();
            coalescer.submit(nameBytes(), add, size, hashIterations, state, p);
            try {
                return p.get()[0];
            } catch (ExecutionException e) {
                Throwable c = e.getCause();
                if (c instanceof RedisException && c.getMessage() != null
                        && c.getMessage().contains("Bloom filter config has been changed")) {
                    readConfig();
                    continue;
                }
                if (c instanceof RuntimeException) {
                    throw (RuntimeException) c;
                }
                throw new RedisException(c.getMessage(), c);
            } catch (InterruptedException e) {
                Thread.currentThread().interrupt();
                throw new RedisException("interrupted", e);
            }
        }
    }

    /** Non-blocking form for event-loop callers: completes from the coalescer's thread.  With no config read yet
     *  the request carries size 0 and the coalescer reads the config in FIFO order (never on the caller's thread). */
    public Future<boolean[]> containsAllAsync(byte[][] encoded) {
        Promise<boolean[]> p = executor.getConnectionManager().newPromise();
        coalescer.submit(nameBytes(), false, size, size == 0 ? 0 : hashIterations, encoded, p);
        return p;
    }

    @Override
    public boolean add(T object) {
        return call(true, object);
    }

    @Override
    public boolean contains(T object) {
        return call(false, object);
    }

    /** Every other engine call of the filter goes through the coalescer's FIFO thread too (VERDICT r4 item 8):
     *  it runs after every add / contains queued before it, and no caller thread makes a JNI call. */
    private <R> Future<R> onWorker(GpuBloomCoalescer.Task<R> task) {
        Promise<R> p = executor.getConnectionManager().newPromise();
        coalescer.submitTask(task, p);
        return p;
    }

    /** The sync API's blocking wait (RedissonObject.get): user threads only, as in the reference. */
    private <R> R await(Future<R> f) {
        try {
            return f.get();
        } catch (ExecutionException e) {
            Throwable c = e.getCause();
            if (c instanceof RuntimeException) {
                throw (RuntimeException) c;
            }
            throw new RedisException(c.getMessage(), c);
        } catch (InterruptedException e) {
            Thread.currentThread().interrupt();
            throw new RedisException("interrupted", e);
        }
    }

    @Override
    public boolean tryInit(final long expectedInsertions, final double falseProbability) {
        final byte[] name = nameBytes();
        boolean ok = await(onWorker(new GpuBloomCoalescer.Task<Boolean>() {
            public Boolean call(long c) {
                int[] out = new int[1];
                SketchDispatch.check(c, SketchNative.bloomTryInit(c, name, expectedInsertions, falseProbability, out));
                return out[0] == 1;
            }
        }));
        readConfig();
        return ok;
    }

    /** {size, expectedInsertions} with k and fpp, read on the worker. */
    private static final class Cfg {
        long size;
        long expected;
        int k;
        double fpp;
    }

    private Cfg config() {
        final byte[] name = nameBytes();
        return await(onWorker(new GpuBloomCoalescer.Task<Cfg>() {
            public Cfg call(long c) {
                long[] se = new long[2];
                int[] k = new int[1];
                double[] fpp = new double[1];
                SketchDispatch.check(c, SketchNative.bloomConfig(c, name, se, k, fpp));
                Cfg r = new Cfg();
                r.size = se[0];
                r.expected = se[1];
                r.k = k[0];
                r.fpp = fpp[0];
                return r;
            }
        }));
    }

    private void readConfig() {
        Cfg c = config();
        size = c.size;
        hashIterations = c.k;
    }

    @Override
    public long getExpectedInsertions() {
        return config().expected;
    }

    @Override
    public double getFalseProbability() {
        return config().fpp;
    }

    @Override
    public long getSize() {
        return config().size;
    }

    @Override
    public int getHashIterations() {
        return config().k;
    }

    @Override
    public int count() {
        final byte[] name = nameBytes();
        return await(onWorker(new GpuBloomCoalescer.Task<Integer>() {
            public Integer call(long c) {
                int[] out = new int[1];
                SketchDispatch.check(c, SketchNative.bloomCount(c, name, out));
                return out[0];
            }
        }));
    }

    /** DEL name {name}__config (:201-203), completed by the coalescer's thread after every request queued before it
     *  (a delete issued after a containsAllAsync on the same thread never overtakes it). */
    @Override
    public Future<Boolean> deleteAsync() {
        final SketchDispatch.Packed k = new SketchDispatch.Packed(java.util.Arrays.asList(nameBytes(),
                ("{" + getName() + "}__config").getBytes(UTF8)));
        return onWorker(new GpuBloomCoalescer.Task<Boolean>() {
            public Boolean call(long c) {
                long[] removed = new long[1];
                SketchDispatch.check(c, SketchNative.del(c, k.off, k.bytes, removed));
                return removed[0] > 0;
            }
        });
    }
}
